cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_run.sh \
 "tests:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "bench:300:python bench.py --steps 3 --warmup 1 --stages" \
 "prof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline" \
 "pmc_fetch:200:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline" \
 "pmc_write:200:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline"
