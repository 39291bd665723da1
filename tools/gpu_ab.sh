#!/bin/bash
# A/B timing of libfmx variants with tools/kbench.py, all in one GPU call.
# usage: tools/gpu_ab.sh "OPS" "KBENCH_ARGS" lib1 lib2 ...   (lib = variant name or "base")
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OPS=$1; shift; KA=$1; shift
specs=()
for v in "$@"; do
  if [ "$v" = base ]; then lib=factormodeling_amd/libfmx.so; else lib=factormodeling_amd/libfmx_var_$v.so; fi
  specs+=("ab_$v:240:FMX_ALLOW_DIAG=1 FMX_LIB=$GRAFT_REPO_ROOT/$lib python tools/kbench.py --ops $OPS --reps 5 $KA")
done
tools/gpu_run.sh "${specs[@]}"
