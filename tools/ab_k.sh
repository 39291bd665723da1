#!/bin/bash
# GPU: parity tests selected by -k "$1", then kbench timing of ops "$2".
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$1" > gpurun_out/k_tests.log 2>&1
rc=$?; tail -3 gpurun_out/k_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/k_tests.log | head -30; exit $rc; }
timeout -k 10 200 python tools/kbench.py --ops $2 ${KB_ARGS} 2>&1 | grep -v amdgpu.ids
