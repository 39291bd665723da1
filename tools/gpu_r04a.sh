#!/bin/bash
# Round-4 GPU pass A: the -m gpu suite, the full-size config checks, long-window kernel
# timings, the ts_corr / feature A/B (reciprocal-table divides vs IEEE) at C5's shape on 252
# dates, and the three benches with per-stage times.
cd "$GRAFT_REPO_ROOT"
C5="--dates 252 --assets 10000 --factors 500"
tools/gpu_run.sh \
 "tests:420:python -u -m pytest tests -m 'gpu and not fullsize' -q --maxfail=30 --timeout 200 --timeout-method thread" \
 "full:600:python -u -m pytest tests -m fullsize -q -x --timeout 900 --timeout-method thread" \
 "kb_long:200:python tools/kbench.py --factors 40 --ops ts_decay,ts_rank,ts_mean,ts_decay80,ts_decay150,ts_decay350,ts_rank60,ts_rank200,ts_mean175,ts_mean20_rg,ts_std175_rg,ts_decay150_rg,ts_rank10_rg" \
 "kb_corr_fast:200:python tools/kbench.py --ops ts_corr60,cvf60 $C5" \
 "kb_corr_v1:200:FMX_TS_CORR_V1=1 python tools/kbench.py --ops ts_corr60,cvf60 $C5" \
 "bench_c2:300:python bench.py --steps 10 --warmup 2 --stages --no-cpu-baseline" \
 "bench_c5:300:python bench.py --workload c5 --steps 3 --warmup 1 --stages" \
 "bench_c4:400:python bench.py --workload c4 --steps 3 --warmup 1 --stages"
