#!/bin/bash
# Round 6, call V: C5's corr -> feature pass forced to 5 waves per SIMD (96 VGPRs, 52
# spilled) vs 4 (114 VGPRs).
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
L=$PWD/factormodeling_amd
K="python tools/kbench.py --ops corr_feat60 --reps 5 --dates 252 --assets 10000 --factors 100"
tools/gpu_run.sh \
  "abV_cur:120:$K" \
  "abV_w5:120:FMX_LIB=$L/libfmx_var_cfw5.so $K" \
  "abV_cur2:120:$K" \
  "abV_w52:120:FMX_LIB=$L/libfmx_var_cfw5.so $K"
