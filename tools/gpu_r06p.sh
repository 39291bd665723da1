#!/bin/bash
# Round 6, call P: final validation at head -- full-size tests, smoke(), the default bench
# line (with cpu_baseline) and the C4 / C5 lines.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
tools/gpu_run.sh \
  "fullsize_p:900:python -u -m pytest tests -m fullsize -x -v --timeout 600 --timeout-method thread -p no:cacheprovider" \
  "smoke_p:200:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "bench_c2_p:300:python -u bench.py" \
  "bench_c5_p:300:python -u bench.py --workload c5 --steps 3 --warmup 1" \
  "bench_c4_p:300:python -u bench.py --workload c4 --steps 3 --warmup 1"
