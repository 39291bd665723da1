#!/bin/bash
# Round 6, call O: the wave IC's x-side sums formed once for both lags (xshare; xshare8 at
# 8 waves per SIMD) vs the product library; IC tests on xshare.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
L=$PWD/factormodeling_amd
KI="python tools/kbench.py --ops ic_ranked --reps 5 --dates 252"
K5="python tools/kbench.py --ops ic_ranked --reps 5 --dates 126 --assets 10000 --factors 500"
T="python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_configs.py tests/test_gpu_long_rows.py tests/test_gpu_big_grid.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
tools/gpu_run.sh \
  "abO_cur:150:$KI && $K5" \
  "abO_xs:150:FMX_LIB=$L/libfmx_var_xshare.so $KI && FMX_LIB=$L/libfmx_var_xshare.so $K5" \
  "abO_xs8:150:FMX_LIB=$L/libfmx_var_xshare8.so $KI && FMX_LIB=$L/libfmx_var_xshare8.so $K5" \
  "abO_cur2:150:$KI && $K5" \
  "abO_xs2:150:FMX_LIB=$L/libfmx_var_xshare.so $KI && FMX_LIB=$L/libfmx_var_xshare.so $K5" \
  "abO_xs82:150:FMX_LIB=$L/libfmx_var_xshare8.so $KI && FMX_LIB=$L/libfmx_var_xshare8.so $K5" \
  "xshare_tests:500:FMX_LIB=$L/libfmx_var_xshare.so $T"
