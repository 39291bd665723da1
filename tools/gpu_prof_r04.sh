#!/bin/bash
# Round-4 profile set: kernel-trace stats of the three benches; FETCH / WRITE passes
# (traffic per launch) over the C2 kernels, the C5 kernels (252 of the 2520 dates) and the
# C4 exact Gram; VALU / wave-cycle passes over C5's ts_corr, feature and rank kernels and C2's
# rank + winsor; the MFMA pass over the C4 exact Gram.  Each rocprofv3 run is its own step
# with its own time limit; PMC passes never combine with trace domains.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r04}
C2OPS="ts_mean,ts_set,cs_rwzn_rk,cs_zn,gram_exact_z,cs_rw_rk,ic_ranked"
C5OPS="ts_mean,corr_feat60,ts_corr60,cvf60,rank2,ic_ranked"
C4="--dates 252 --assets 3000 --factors 2000"
C5="--dates 252 --assets 10000 --factors 500"
VALU="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD"
trap 'find gpurun_out -name "*kernel_trace.csv" -size +2M -delete; find gpurun_out -name "*agent_info.csv" -delete' EXIT
tools/gpu_run.sh \
 "prof_c2_$T:300:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_c2_$T -o run -- python bench.py --workload c2 --steps 2 --warmup 1 --no-cpu-baseline --stages" \
 "prof_c5_$T:300:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_c5_$T -o run -- python bench.py --workload c5 --steps 2 --warmup 1 --stages" \
 "prof_c4_$T:300:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_c4_$T -o run -- python bench.py --workload c4 --steps 2 --warmup 1 --stages" \
 "pmcf_c2_$T:240:timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcf_c2_$T -o run -- python tools/kbench.py --ops $C2OPS --reps 1" \
 "pmcw_c2_$T:240:timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcw_c2_$T -o run -- python tools/kbench.py --ops $C2OPS --reps 1" \
 "pmcf_c5_$T:240:timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcf_c5_$T -o run -- python tools/kbench.py --ops $C5OPS --reps 1 $C5" \
 "pmcw_c5_$T:240:timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcw_c5_$T -o run -- python tools/kbench.py --ops $C5OPS --reps 1 $C5" \
 "pmcf_c4_$T:240:timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcf_c4_$T -o run -- python tools/kbench.py --ops ts_mean,gram_direct_exact --reps 1 $C4" \
 "pmcw_c4_$T:240:timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcw_c4_$T -o run -- python tools/kbench.py --ops ts_mean,gram_direct_exact --reps 1 $C4" \
 "valu_c5_$T:240:timeout -s KILL 200 rocprofv3 --pmc $VALU --kernel-include-regex fmx -f csv -d gpurun_out/valu_c5_$T -o run -- python tools/kbench.py --ops corr_feat60,ts_corr60,rank2 --reps 1 $C5" \
 "valu_c2_$T:240:timeout -s KILL 200 rocprofv3 --pmc $VALU --kernel-include-regex fmx -f csv -d gpurun_out/valu_c2_$T -o run -- python tools/kbench.py --ops ts_set,cs_rwzn_rk,cs_rw_rk,cs_zn,ic_ranked --reps 1" \
 "mfma_c4_$T:240:timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU --kernel-include-regex gram -f csv -d gpurun_out/mfma_c4_$T -o run -- python tools/kbench.py --ops gram_direct_exact --reps 1 $C4"
