#!/bin/bash
# Round 6, call G2: sequential step vs the rolling set on a side stream enqueued first
# (overlap) or behind the cross-sectional pass (overlap late), alternating on one box.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
B="python -u bench.py --steps 10 --warmup 2 --stages --no-cpu-baseline"
tools/gpu_run.sh \
  "seq_a:200:$B" \
  "ovl_a:200:FMX_STEP_OVERLAP=1 $B" \
  "ovlL_a:200:FMX_STEP_OVERLAP=1 FMX_OVERLAP_LATE=1 $B" \
  "seq_b:200:$B" \
  "ovl_b:200:FMX_STEP_OVERLAP=1 $B" \
  "ovlL_b:200:FMX_STEP_OVERLAP=1 FMX_OVERLAP_LATE=1 $B"
