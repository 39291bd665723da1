#!/bin/bash
# GPU: parity tests, then per-kernel timing of the fine-bucket vs splitter-bucket rank kernels.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -5 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/ab_tests.log | head -30; exit $rc; }
timeout -k 10 200 python tools/kbench.py --ops cs_rank,ic ${KB_ARGS} > gpurun_out/ab_fine.log 2>&1 || exit $?
FMX_RANK_IMPL=br timeout -k 10 200 python tools/kbench.py --ops cs_rank,ic ${KB_ARGS} > gpurun_out/ab_br.log 2>&1 || exit $?
echo "--- fine"; grep -v amdgpu.ids gpurun_out/ab_fine.log; echo "--- br"; grep -v amdgpu.ids gpurun_out/ab_br.log
