cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OPS=ts_mean,ts_std,ts_zscore,ts_rank,ts_decay,cs_rank,cs_zscore,market_neutralize,winsor,ic,gram
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_v13 -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_v13.log 2>&1 && \
rm -f gpurun_out/prof_v13/run_kernel_trace.csv && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcf_v13 -o run -- python tools/kbench.py --reps 1 --ops $OPS > gpurun_out/pmcf_v13.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcw_v13 -o run -- python tools/kbench.py --reps 1 --ops $OPS > gpurun_out/pmcw_v13.log 2>&1 && echo pmc ok
du -sh gpurun_out/*
