#!/bin/bash
# Round 6, call D: C5 corr -> feature A/B: r5 kernel (c6a) vs software-pipelined loads
# without (pfns) and with (cur) the sign-only path; parity tests of the corr paths.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
KB="python tools/kbench.py --ops corr_feat60 --reps 5 --dates 252 --assets 10000 --factors 100"
L=$PWD/factormodeling_amd
tools/gpu_run.sh \
  "abD_c6a:120:FMX_LIB=$L/libfmx_var_c6a.so $KB" \
  "abD_pfns:120:FMX_LIB=$L/libfmx_var_pfns.so $KB" \
  "abD_cur:120:$KB" \
  "abD_c6a2:120:FMX_LIB=$L/libfmx_var_c6a.so $KB" \
  "abD_pfns2:120:FMX_LIB=$L/libfmx_var_pfns.so $KB" \
  "abD_cur2:120:$KB" \
  "corrfeat:200:python -u -m pytest tests/test_gpu_corr_feature.py tests/test_gpu_parity.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider"
