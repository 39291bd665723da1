cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-v18}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$T.log 2>&1 && \
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_$T.log 2>&1 && \
timeout -k 10 300 python tools/csv_bench.py --dates 252 --assets 2000 --factors 20 --threads 16 --dir gpurun_out > gpurun_out/csv_bench_$T.log 2>&1
rc=$?
tail -3 gpurun_out/tests_$T.log; tail -2 gpurun_out/csv_bench_$T.log
exit $rc
