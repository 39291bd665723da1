#!/bin/bash
# Round 6, call R: the C2 Gram's waves on 2 x 3 block tiles (gtile: 5 fragment reads per
# k-step for 6 blocks) vs the product library; Gram / shard tests on gtile.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
L=$PWD/factormodeling_amd
KG="python tools/kbench.py --ops gram_exact_z --reps 5 --dates 252"
T="python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
tools/gpu_run.sh \
  "abR_cur:120:$KG" \
  "abR_gt:120:FMX_LIB=$L/libfmx_var_gtile.so $KG" \
  "abR_cur2:120:$KG" \
  "abR_gt2:120:FMX_LIB=$L/libfmx_var_gtile.so $KG" \
  "gtile_tests:600:FMX_LIB=$L/libfmx_var_gtile.so $T"
