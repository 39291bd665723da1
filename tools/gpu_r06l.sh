#!/bin/bash
# Round 6, call L: the splitter table padded against bank conflicts (splpad) and, on top,
# the interval table as 8-byte inverses with the lower bound from the sample below the key
# (splinv) vs the product library: C2 fused pass and C5 ranks-only pass; rank parity tests
# on splinv.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
L=$PWD/factormodeling_amd
K2="python tools/kbench.py --ops cs_rwzn_rk --reps 5 --dates 252"
K5="python tools/kbench.py --ops rank2 --reps 5 --dates 126 --assets 10000 --factors 500"
T="python -u -m pytest tests/test_gpu_rank_stress.py tests/test_gpu_fused.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
tools/gpu_run.sh \
  "abL_base:120:$K2 && $K5" \
  "abL_splpad:120:FMX_LIB=$L/libfmx_var_splpad.so $K2 && FMX_LIB=$L/libfmx_var_splpad.so $K5" \
  "abL_splinv:120:FMX_LIB=$L/libfmx_var_splinv.so $K2 && FMX_LIB=$L/libfmx_var_splinv.so $K5" \
  "abL_base2:120:$K2 && $K5" \
  "abL_splpad2:120:FMX_LIB=$L/libfmx_var_splpad.so $K2 && FMX_LIB=$L/libfmx_var_splpad.so $K5" \
  "abL_splinv2:120:FMX_LIB=$L/libfmx_var_splinv.so $K2 && FMX_LIB=$L/libfmx_var_splinv.so $K5" \
  "splinv_tests:400:FMX_LIB=$L/libfmx_var_splinv.so $T"
