#!/bin/bash
# Round 6, call B: A/B of the fused pass and the wave IC (r5 library vs this tree, base
# measured twice to bracket drift), the -m gpu suite without the full-size configs, and the
# drop-in API timings after the boundary changes.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
KB="python tools/kbench.py --ops cs_rwzn_rk,ic_ranked --reps 10 --dates 252"
B5="FMX_LIB=$PWD/factormodeling_amd/libfmx_var_base5.so"
tools/gpu_run.sh \
  "abB_base5:100:$B5 $KB" \
  "abB_cur:100:$KB" \
  "abB_base5b:100:$B5 $KB" \
  "abB_curb:100:$KB" \
  "gputests:700:python -u -m pytest tests -m 'gpu and not fullsize' -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "dropin_c1:120:python -u bench.py --workload c1-dropin --steps 3" \
  "dropin_c2s:160:python -u bench.py --workload c2-dropin-slice --steps 2"
