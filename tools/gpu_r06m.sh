#!/bin/bash
# Round 6, call M: (1) the wave IC's block table with 0xffff for absent entries (icsent: no
# per-element count tests) vs the product library, and its IC tests; (2) C5 ranks-only pass,
# persistent 1-row-per-CU kernel vs the 2-rows-per-CU k_cs_rank_fa (FMX_RANK2_PF=0);
# (3) the full-size GPU tests at head.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
L=$PWD/factormodeling_amd
KI="python tools/kbench.py --ops ic_ranked --reps 5 --dates 252"
K5="python tools/kbench.py --ops rank2 --reps 5 --dates 126 --assets 10000 --factors 500"
T="python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_configs.py tests/test_gpu_long_rows.py tests/test_gpu_big_grid.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
tools/gpu_run.sh \
  "abM_icbase:120:$KI" \
  "abM_icsent:120:FMX_LIB=$L/libfmx_var_icsent.so $KI" \
  "abM_icbase2:120:$KI" \
  "abM_icsent2:120:FMX_LIB=$L/libfmx_var_icsent.so $KI" \
  "icsent_tests:500:FMX_LIB=$L/libfmx_var_icsent.so $T" \
  "abM_pf:120:$K5" \
  "abM_fa:120:FMX_RANK2_PF=0 $K5" \
  "abM_pf2:120:$K5" \
  "abM_fa2:120:FMX_RANK2_PF=0 $K5" \
  "fullsize_m:900:python -u -m pytest tests -m fullsize -x -v --timeout 600 --timeout-method thread -p no:cacheprovider"
