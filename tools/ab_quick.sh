#!/bin/bash
# GPU: rank/IC parity tests + per-kernel timing (fine vs br); KB_OPS selects kernels.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OPS=${KB_OPS:-cs_rank,ic}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PT_ARGS} > gpurun_out/q_tests.log 2>&1
rc=$?; tail -3 gpurun_out/q_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/q_tests.log | head -30; exit $rc; }
timeout -k 10 200 python tools/kbench.py --ops $OPS ${KB_ARGS} 2>&1 | grep -v amdgpu.ids
