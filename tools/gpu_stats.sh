#!/bin/bash
# Kernel-trace statistics of the C2 / C5 / C4 benches (rocprofv3 --kernel-trace --stats),
# one step each after a warm-up.  usage: tools/gpu_stats.sh TAG [c2 c5 c4]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-stats}; shift
W=${@:-c2 c5 c4}
trap 'find gpurun_out -name "*kernel_trace.csv" -size +2M -delete; find gpurun_out -name "*agent_info.csv" -delete' EXIT
specs=()
for w in $W; do
  specs+=("prof_${w}_$T:400:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_${w}_$T -o run -- python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --stages")
done
tools/gpu_run.sh "${specs[@]}"
