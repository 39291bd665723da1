#!/bin/bash
# Round 6, call I: ts_decay's dot as 4 interleaved fma chains (cur) vs one chain (dec1), in
# the fused rolling set and the single-op kernel; decay parity tests.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
KT="python tools/kbench.py --ops ts_set,ts_decay --reps 5 --dates 504"
L=$PWD/factormodeling_amd
tools/gpu_run.sh \
  "abI_dec1:100:FMX_LIB=$L/libfmx_var_dec1.so $KT" \
  "abI_cur:100:$KT" \
  "abI_dec1b:100:FMX_LIB=$L/libfmx_var_dec1.so $KT" \
  "abI_curb:100:$KT" \
  "decay_tests:400:python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_longwin.py tests/test_gpu_configs.py -x -q --timeout 380 --timeout-method thread -p no:cacheprovider"
