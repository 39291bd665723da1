#!/bin/bash
# Round 6, call E: ts_set workgroup width A/B (256 / 512 / 1024 adjacent columns), and the
# C5 line with the corr -> feature pass as one launch over all factors.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
KT="python tools/kbench.py --ops ts_set --reps 5 --dates 504"
tools/gpu_run.sh \
  "abE_256:100:$KT" \
  "abE_512:100:FMX_TS_SET_NT=512 $KT" \
  "abE_1024:100:FMX_TS_SET_NT=1024 $KT" \
  "abE_256b:100:$KT" \
  "abE_512b:100:FMX_TS_SET_NT=512 $KT" \
  "abE_1024b:100:FMX_TS_SET_NT=1024 $KT" \
  "bench_c5:300:python -u bench.py --workload c5 --steps 3 --warmup 1 --stages --no-cpu-baseline" \
  "c5full:400:python -u -m pytest tests/test_gpu_fullsize.py -k c5 -x -q --timeout 380 --timeout-method thread -p no:cacheprovider"
