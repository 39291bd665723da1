#!/bin/bash
# Round-4 profile set (d): the C4 exact Gram after the z pass + LDS-DMA tile kernel and the
# i8 pair counts -- kernel stats of the C4 bench, FETCH / WRITE passes (traffic per launch,
# 252 of the 2520 dates), the MFMA / clock pass; the C2 bench stages.  Each rocprofv3 run
# is its own step with its own time limit; PMC passes never combine with trace domains.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-d}
C4="--dates 252 --assets 3000 --factors 2000"
trap 'find gpurun_out -name "*kernel_trace.csv" -size +2M -delete; find gpurun_out -name "*agent_info.csv" -delete' EXIT
tools/gpu_run.sh \
 "prof_c4_$T:300:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_c4_$T -o run -- python bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --stages" \
 "pmcf_c4_$T:240:timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcf_c4_$T -o run -- python tools/kbench.py --ops ts_mean,gram_direct_exact --reps 1 $C4" \
 "pmcw_c4_$T:240:timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcw_c4_$T -o run -- python tools/kbench.py --ops ts_mean,gram_direct_exact --reps 1 $C4" \
 "mfma_c4_$T:240:timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-include-regex gram -f csv -d gpurun_out/mfma_c4_$T -o run -- python tools/kbench.py --ops gram_direct_exact --reps 1 $C4" \
 "bench_c2_$T:300:python bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline --stages"
