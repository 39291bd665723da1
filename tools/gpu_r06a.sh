#!/bin/bash
# Round 6, call A: fused-pass A/B (r5 library vs this tree), the br fallback of the sharded
# fused pass, the drop-in API timings (C1 and a C2 slice), and the new full-size oracle pins
# of the pruning order (which also check the rdiv z-scores bit for bit at full size).
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
KB="python tools/kbench.py --ops cs_rwzn_rk,cs_zn --reps 5 --dates 252"
tools/gpu_run.sh \
  "ab_base5:100:FMX_LIB=$PWD/factormodeling_amd/libfmx_var_base5.so $KB" \
  "ab_new:100:$KB" \
  "br_shard:150:python -u -m pytest -x -v --timeout 140 --timeout-method thread tests/test_gpu_shard.py -k br_rank_impl -p no:cacheprovider" \
  "dropin_c1:120:python -u bench.py --workload c1-dropin --steps 3" \
  "dropin_c2s:140:python -u bench.py --workload c2-dropin-slice --steps 2" \
  "fs_prune:600:python -u -m pytest -x -v --timeout 590 --timeout-method thread tests/test_gpu_fullsize.py -k 'c2_full_step or zoo or c4_full' -p no:cacheprovider"
