cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_run.sh \
 "tests_v12:500:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "bench_v12:400:python bench.py --steps 3 --warmup 1 --stages" \
 "prof_v12:300:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_v12 -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline" \
 "smoke_v12:200:python -c 'import __graft_entry__ as g; g.smoke()'"
