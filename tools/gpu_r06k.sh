#!/bin/bash
# Round 6, call K: what bounds C5's corr -> feature pass.  Diagnostic arms (wrong results):
# no reciprocal-table LDS reads (cfrt), no leaving-row loads (cfold), both; PF=2 ring.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
L=$PWD/factormodeling_amd
K="python tools/kbench.py --ops corr_feat60 --reps 5 --dates 252 --assets 10000 --factors 100"
tools/gpu_run.sh \
  "abK_base:150:$K" \
  "abK_cfrt:150:FMX_ALLOW_DIAG=1 FMX_LIB=$L/libfmx_var_cfrt.so $K" \
  "abK_cfold:150:FMX_ALLOW_DIAG=1 FMX_LIB=$L/libfmx_var_cfold.so $K" \
  "abK_cfboth:150:FMX_ALLOW_DIAG=1 FMX_LIB=$L/libfmx_var_cfboth.so $K" \
  "abK_pf2:150:FMX_CORR_FEAT_PF=2 $K" \
  "abK_base2:150:$K" \
  "abK_cfrt2:150:FMX_ALLOW_DIAG=1 FMX_LIB=$L/libfmx_var_cfrt.so $K"
