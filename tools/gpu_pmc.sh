#!/bin/bash
# SQ counter passes over the per-kernel harness (tools/kbench.py) at a reduced size.
# usage: tools/gpu_pmc.sh TAG "kbench args"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; KARGS=$2
mkdir -p gpurun_out
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
P2="SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-include-regex fmx -f csv -d gpurun_out/sq1_$TAG -o run -- python tools/kbench.py $KARGS > gpurun_out/sq1_$TAG.log 2>&1 || { echo "pass1 rc=$?"; tail -5 gpurun_out/sq1_$TAG.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-include-regex fmx -f csv -d gpurun_out/sq2_$TAG -o run -- python tools/kbench.py $KARGS > gpurun_out/sq2_$TAG.log 2>&1 || { echo "pass2 rc=$?"; tail -5 gpurun_out/sq2_$TAG.log; exit 1; }
echo pmc done
