#!/bin/bash
# Round 6, call N: the product library with the IC table sentinels and the two-rows-per-CU
# C5 ranks-only default vs the previous library (base6); the whole GPU suite (not full
# size); the C5 and default bench lines.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
L=$PWD/factormodeling_amd
KI="python tools/kbench.py --ops ic_ranked --reps 5 --dates 252"
K5="python tools/kbench.py --ops rank2,ic_ranked --reps 5 --dates 126 --assets 10000 --factors 500"
tools/gpu_run.sh \
  "abN_base6:150:FMX_LIB=$L/libfmx_var_base6.so $KI && FMX_LIB=$L/libfmx_var_base6.so $K5" \
  "abN_cur:150:$KI && $K5" \
  "abN_base6b:150:FMX_LIB=$L/libfmx_var_base6.so $KI && FMX_LIB=$L/libfmx_var_base6.so $K5" \
  "abN_curb:150:$KI && $K5" \
  "gputests_n:700:python -u -m pytest tests -m 'gpu and not fullsize' -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "bench_c5_n:300:python -u bench.py --workload c5 --steps 3 --warmup 1 --stages" \
  "bench_c2_n:300:python -u bench.py --stages"
