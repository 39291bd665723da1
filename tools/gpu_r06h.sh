#!/bin/bash
# Round 6, call H: winsor order-statistic publish behind a wave-uniform test (cur) vs p6.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
KF="python tools/kbench.py --ops cs_rwzn_rk,cs_rw_rk --reps 10 --dates 252"
L=$PWD/factormodeling_amd
tools/gpu_run.sh \
  "abH_p6:100:FMX_LIB=$L/libfmx_var_p6.so $KF" \
  "abH_cur:100:$KF" \
  "abH_p6b:100:FMX_LIB=$L/libfmx_var_p6.so $KF" \
  "abH_curb:100:$KF" \
  "rank_tests:300:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_rank_stress.py tests/test_gpu_long_rows.py -x -q --timeout 280 --timeout-method thread -p no:cacheprovider"
