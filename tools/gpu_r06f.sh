#!/bin/bash
# Round 6, call F: fused-pass A/B -- c6e (before) vs this tree (64-leaf shuffle combine +
# counting sample sort), FMX_ZN_T64=1 (counting sort only) and nocs (shuffle combine only);
# the ranks-only pass at C5 / C4 widths (counting sort); then the -m gpu suite minus full size.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
KF="python tools/kbench.py --ops cs_rwzn_rk --reps 10 --dates 252"
KR5="python tools/kbench.py --ops rank2 --reps 5 --dates 126 --assets 10000 --factors 100"
KR4="python tools/kbench.py --ops rank2 --reps 5 --dates 126 --assets 3000 --factors 400"
L=$PWD/factormodeling_amd
tools/gpu_run.sh \
  "abF_c6e:100:FMX_LIB=$L/libfmx_var_c6e.so $KF" \
  "abF_cur:100:$KF" \
  "abF_cs:100:FMX_ZN_T64=1 $KF" \
  "abF_nocs:100:FMX_LIB=$L/libfmx_var_nocs.so $KF" \
  "abF_c6e2:100:FMX_LIB=$L/libfmx_var_c6e.so $KF" \
  "abF_cur2:100:$KF" \
  "abF_cs2:100:FMX_ZN_T64=1 $KF" \
  "abF_nocs2:100:FMX_LIB=$L/libfmx_var_nocs.so $KF" \
  "abR5_c6e:100:FMX_LIB=$L/libfmx_var_c6e.so $KR5" \
  "abR5_cur:100:$KR5" \
  "abR4_c6e:100:FMX_LIB=$L/libfmx_var_c6e.so $KR4" \
  "abR4_cur:100:$KR4" \
  "gputests:600:python -u -m pytest tests -m 'gpu and not fullsize' -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
