#!/bin/bash
# GPU: IC parity tests, then the chunked IC kernel's timing over factors-per-workgroup.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ic or metric or select" > gpurun_out/ic_t.log 2>&1 || { tail -30 gpurun_out/ic_t.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/ic_t.log)"
for fc in ${FCS:-8 4 16}; do
  echo "FC=$fc: $(FMX_IC_FC=$fc timeout -k 10 120 python tools/kbench.py --ops ic 2>&1 | grep -v amdgpu | head -1)"
done
