cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_run.sh \
 "tests_v14:500:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "bench_v14:300:python bench.py --steps 3 --warmup 1 --stages --no-cpu-baseline"
