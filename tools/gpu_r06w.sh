#!/bin/bash
# Round 6, call W: the A/B switches against the defaults at the final head, one box --
# C2: the IC fused into the rank pass (FMX_FUSED_IC=1), the Gram without the MFMA / staging
# interleave (FMX_GRAM_OPT=0), pair counts by AND + popcount (FMX_GRAM_CNT=0);
# C4: the 8-wave tile kernel (FMX_GRAM_GLDS=8), the register-staged tile kernel (=0).
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
B2="python -u bench.py --steps 5 --warmup 1 --stages --no-cpu-baseline"
B4="python -u bench.py --workload c4 --steps 2 --warmup 1 --stages --no-cpu-baseline"
tools/gpu_run.sh \
  "abW_c2:200:$B2" \
  "abW_c2_fic:200:FMX_FUSED_IC=1 $B2" \
  "abW_c2_gopt0:200:FMX_GRAM_OPT=0 $B2" \
  "abW_c2_cnt0:200:FMX_GRAM_CNT=0 $B2" \
  "abW_c2b:200:$B2" \
  "abW_c4:300:$B4" \
  "abW_c4_g8:300:FMX_GRAM_GLDS=8 $B4" \
  "abW_c4_g0:300:FMX_GRAM_GLDS=0 $B4"
