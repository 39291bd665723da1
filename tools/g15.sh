cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-v15}
OPS=ts_mean,ts_std,ts_zscore,ts_rank,ts_decay,cs_rank,cs_zscore,market_neutralize,winsor,ic,gram
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --stages > gpurun_out/bench_$T.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_$T -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$T.log 2>&1 && \
rm -f gpurun_out/prof_$T/run_kernel_trace.csv && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcf_$T -o run -- python tools/kbench.py --reps 1 --ops $OPS > gpurun_out/pmcf_$T.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcw_$T -o run -- python tools/kbench.py --reps 1 --ops $OPS > gpurun_out/pmcw_$T.log 2>&1 && echo all ok
tail -3 gpurun_out/bench_$T.log
