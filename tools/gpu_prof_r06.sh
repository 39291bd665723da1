#!/bin/bash
# Round-6 profile set: kernel-trace stats of the default bench command and of the C5 / C4
# benches; FETCH / WRITE passes (traffic per launch) over the C2 kernels, the C5 kernels and
# the C4 Gram (252 of the 2520 dates); instruction / wait / LDS counters of the hot kernels.
# Each rocprofv3 run is its own step with its own time limit; PMC passes never combine with
# trace domains.   usage: tools/gpu_prof_r05.sh TAG [steps...]  (steps: stats pmc counters)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06}; shift
WHAT=${@:-stats pmc counters}
C2OPS="ts_mean,ts_set,cs_rwzn_rk,gram_exact_z,ic_ranked"
C5OPS="ts_mean,corr_feat60,rank2,ic_ranked"
C4="--dates 252 --assets 3000 --factors 2000"
C5="--dates 252 --assets 10000 --factors 500"
CNT="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"
LDS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
trap 'find gpurun_out -name "*kernel_trace.csv" -size +2M -delete; find gpurun_out -name "*agent_info.csv" -delete' EXIT
specs=()
for w in $WHAT; do
  case $w in
  stats) specs+=(
   "prof_default_$T:300:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_default_$T -o run -- python bench.py"
   "prof_c5_$T:300:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_c5_$T -o run -- python bench.py --workload c5 --steps 2 --warmup 1 --stages"
   "prof_c4_$T:300:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_c4_$T -o run -- python bench.py --workload c4 --steps 2 --warmup 1 --stages") ;;
  pmc) specs+=(
   "pmcf_c2_$T:240:timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcf_c2_$T -o run -- python tools/kbench.py --ops $C2OPS --reps 1"
   "pmcw_c2_$T:240:timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcw_c2_$T -o run -- python tools/kbench.py --ops $C2OPS --reps 1"
   "pmcf_c5_$T:240:timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcf_c5_$T -o run -- python tools/kbench.py --ops $C5OPS --reps 1 $C5"
   "pmcw_c5_$T:240:timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcw_c5_$T -o run -- python tools/kbench.py --ops $C5OPS --reps 1 $C5"
   "pmcf_c4_$T:240:timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcf_c4_$T -o run -- python tools/kbench.py --ops ts_mean,gram_direct_exact --reps 1 $C4"
   "pmcw_c4_$T:240:timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcw_c4_$T -o run -- python tools/kbench.py --ops ts_mean,gram_direct_exact --reps 1 $C4") ;;
  counters) specs+=(
   "cnt_c2_$T:240:timeout -s KILL 200 rocprofv3 --pmc $CNT --kernel-include-regex fmx -f csv -d gpurun_out/cnt_c2_$T -o run -- python tools/kbench.py --ops ts_set,cs_rwzn_rk,gram_exact_z,ic_ranked --reps 1 --dates 252"
   "lds_c2_$T:240:timeout -s KILL 200 rocprofv3 --pmc $LDS --kernel-include-regex fmx -f csv -d gpurun_out/lds_c2_$T -o run -- python tools/kbench.py --ops cs_rwzn_rk,ic_ranked --reps 1 --dates 252"
   "cnt_c5_$T:240:timeout -s KILL 200 rocprofv3 --pmc $CNT --kernel-include-regex fmx -f csv -d gpurun_out/cnt_c5_$T -o run -- python tools/kbench.py --ops corr_feat60,rank2,ic_ranked --reps 1 $C5"
   "mfma_c2_$T:240:timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS --kernel-include-regex gram -f csv -d gpurun_out/mfma_c2_$T -o run -- python tools/kbench.py --ops gram_exact_z --reps 1 --dates 252") ;;
  esac
done
tools/gpu_run.sh "${specs[@]}"
