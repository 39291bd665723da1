#!/bin/bash
# One GPU measurement cycle: parity tests, bench (stages), rocprof kernel stats (csv),
# and the two PMC passes (FETCH_SIZE, WRITE_SIZE) restricted to libfmx kernels.
# usage: tools/gpu_cycle.sh TAG [bench args...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}; shift
BARGS="$@"
tools/gpu_run.sh \
 "tests_$TAG:500:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "bench_$TAG:300:python bench.py --steps 3 --warmup 1 --stages --no-cpu-baseline $BARGS" \
 "prof_$TAG:300:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline $BARGS" \
 "pmcf_$TAG:240:rocprofv3 --pmc FETCH_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcf_$TAG -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline $BARGS" \
 "pmcw_$TAG:240:rocprofv3 --pmc WRITE_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcw_$TAG -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline $BARGS"
