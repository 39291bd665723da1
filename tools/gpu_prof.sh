#!/bin/bash
# Profile set: kernel stats of the default bench (C2) and the C4 bench, FETCH /
# WRITE passes over the C2 kernels (kbench; ts_mean calibrates FETCH_SIZE), and an MFMA
# pass over the wide Gram (kbench, C4 factors/assets on 252 dates).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-prof}
KOPS="ts_mean,ts_set,cs_zn,cs_rw_rk,ic_ranked,gram"
trap 'find gpurun_out -name "*kernel_trace.csv" -size +2M -delete; find gpurun_out -name "*agent_info.csv" -delete' EXIT
tools/gpu_run.sh \
 "prof_c2_$T:300:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_c2_$T -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline" \
 "prof_c4_$T:400:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_c4_$T -o run -- python bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline" \
 "pmcf_$T:240:timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcf_$T -o run -- python tools/kbench.py --ops $KOPS --reps 1" \
 "pmcw_$T:240:timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcw_$T -o run -- python tools/kbench.py --ops $KOPS --reps 1" \
 "mfma_$T:240:timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU --kernel-include-regex gram -f csv -d gpurun_out/mfma_$T -o run -- python tools/kbench.py --ops gram --reps 1 --dates 252 --assets 3000 --factors 2000" \
 "mfmac2_$T:240:timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU --kernel-include-regex gram -f csv -d gpurun_out/mfmac2_$T -o run -- python tools/kbench.py --ops gram --reps 1"
