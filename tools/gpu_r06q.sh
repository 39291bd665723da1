#!/bin/bash
# Round 6, call Q: C5 ranks-only rows as 512-thread workgroups of 20 keys per lane (128 VGPRs,
# no spills, two rows per CU) vs the default 1024 x 10 (64 VGPRs, 16 spilled).
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
K5="python tools/kbench.py --ops rank2 --reps 5 --dates 126 --assets 10000 --factors 500"
tools/gpu_run.sh \
  "abQ_1024:120:$K5" \
  "abQ_512:120:FMX_FA_NT=512 $K5" \
  "abQ_1024b:120:$K5" \
  "abQ_512b:120:FMX_FA_NT=512 $K5"
