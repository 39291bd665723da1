#!/bin/bash
# Round 6, call C: VALU class rates (isa_rates), the C5 corr -> feature A/B (sign-only fast
# path), the fused-pass A/B (ballot count in the moments), the corr parity tests, the
# default C2 bench line + the C5 line with stages, and a PC-sampling try of the fused pass.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
KB="python tools/kbench.py --ops corr_feat60 --reps 5 --dates 252 --assets 10000 --factors 100"
KF="python tools/kbench.py --ops cs_rwzn_rk --reps 10 --dates 252"
L=$PWD/factormodeling_amd
tools/gpu_run.sh \
  "isa_rates:60:tools/isa_rates" \
  "abC_c6a:120:FMX_LIB=$L/libfmx_var_c6a.so $KB" \
  "abC_cur:120:$KB" \
  "abC_c6a2:120:FMX_LIB=$L/libfmx_var_c6a.so $KB" \
  "abC_cur2:120:$KB" \
  "abF_c6b:100:FMX_LIB=$L/libfmx_var_c6b.so $KF" \
  "abF_cur:100:$KF" \
  "abF_c6b2:100:FMX_LIB=$L/libfmx_var_c6b.so $KF" \
  "abF_cur2:100:$KF" \
  "corrfeat:200:python -u -m pytest tests/test_gpu_corr_feature.py tests/test_gpu_fused.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider" \
  "bench_c2:240:python -u bench.py --steps 10 --warmup 2 --stages" \
  "bench_c5:300:python -u bench.py --workload c5 --steps 3 --warmup 1 --stages" \
  "pcs:90:cd /tmp && rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d $GRAFT_REPO_ROOT/gpurun_out/pcs -o pcs --output-format csv -- python $GRAFT_REPO_ROOT/tools/kbench.py --ops cs_rwzn_rk --reps 3 --dates 64"
