#!/bin/bash
# Round 6, call S: the wave IC with two chunks of loads in flight (icpf2: 64 VGPRs, no
# spills) vs one (product); IC tests on icpf2.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
L=$PWD/factormodeling_amd
KI="python tools/kbench.py --ops ic_ranked --reps 5 --dates 252"
K5="python tools/kbench.py --ops ic_ranked --reps 5 --dates 126 --assets 10000 --factors 500"
T="python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_configs.py tests/test_gpu_long_rows.py tests/test_gpu_big_grid.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
tools/gpu_run.sh \
  "abS_cur:150:$KI && $K5" \
  "abS_pf2:150:FMX_LIB=$L/libfmx_var_icpf2.so $KI && FMX_LIB=$L/libfmx_var_icpf2.so $K5" \
  "abS_cur2:150:$KI && $K5" \
  "abS_pf22:150:FMX_LIB=$L/libfmx_var_icpf2.so $KI && FMX_LIB=$L/libfmx_var_icpf2.so $K5" \
  "icpf2_tests:500:FMX_LIB=$L/libfmx_var_icpf2.so $T"
