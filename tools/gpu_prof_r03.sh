#!/bin/bash
# Round-3 profile set: kernel stats of the three benches, FETCH / WRITE passes over the
# C2 kernels (kbench at the C2 shape; ts_mean calibrates FETCH_SIZE), over the C5 rank /
# IC / ts kernels (kbench at C5's 10,000 assets x 500 factors on 252 dates) and over the
# direct C4 Gram (2000 factors x 3000 assets on 252 dates), and MFMA passes over both Gram
# kernels.  Each rocprofv3 pass is its own step with its own time limit.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r03}
C2OPS="ts_mean,ts_set,cs_zn,gram_exact_z,cs_rw_rk,ic_ranked"
C5OPS="ts_mean,ts_corr60,cvf60,rank2,ic_ranked"
C4="--dates 252 --assets 3000 --factors 2000"
C5="--dates 252 --assets 10000 --factors 500"
trap 'find gpurun_out -name "*kernel_trace.csv" -size +2M -delete; find gpurun_out -name "*agent_info.csv" -delete' EXIT
tools/gpu_run.sh \
 "pmcf_c2_$T:240:timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcf_c2_$T -o run -- python tools/kbench.py --ops $C2OPS --reps 1" \
 "pmcw_c2_$T:240:timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcw_c2_$T -o run -- python tools/kbench.py --ops $C2OPS --reps 1" \
 "pmcf_c5_$T:240:timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcf_c5_$T -o run -- python tools/kbench.py --ops $C5OPS --reps 1 $C5" \
 "pmcw_c5_$T:240:timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcw_c5_$T -o run -- python tools/kbench.py --ops $C5OPS --reps 1 $C5" \
 "pmcf_c4_$T:240:timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcf_c4_$T -o run -- python tools/kbench.py --ops ts_mean,gram_direct --reps 1 $C4" \
 "pmcw_c4_$T:240:timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcw_c4_$T -o run -- python tools/kbench.py --ops ts_mean,gram_direct --reps 1 $C4" \
 "mfma_c4_$T:240:timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU --kernel-include-regex gram -f csv -d gpurun_out/mfma_c4_$T -o run -- python tools/kbench.py --ops gram_direct --reps 1 $C4" \
 "mfma_c2_$T:240:timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU --kernel-include-regex gram -f csv -d gpurun_out/mfma_c2_$T -o run -- python tools/kbench.py --ops cs_zn,gram_exact_z --reps 1"
