#!/bin/bash
# Round 6, call U: records at the final head -- sequential vs overlapped step (alternating),
# and the drop-in API timings (C1, C2 slice).
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
B="python -u bench.py --steps 10 --warmup 2 --stages --no-cpu-baseline"
tools/gpu_run.sh \
  "final_seq_a:200:$B" \
  "final_ovl_a:200:FMX_STEP_OVERLAP=1 $B" \
  "final_seq_b:200:$B" \
  "final_ovl_b:200:FMX_STEP_OVERLAP=1 $B" \
  "dropin_c1_u:150:python -u bench.py --workload c1-dropin --steps 3" \
  "dropin_c2s_u:200:python -u bench.py --workload c2-dropin-slice --steps 2"
