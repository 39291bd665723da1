#!/bin/bash
# Round 6, call J: validation at head -- the GPU suite (not full size), smoke(), the default
# bench line twice (with its cpu_baseline), and the C4 / C5 lines.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
tools/gpu_run.sh \
  "gputests_j:600:python -u -m pytest tests -m 'gpu and not fullsize' -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "smoke_j:200:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "bench_c2_j1:300:python -u bench.py" \
  "bench_c2_j2:200:python -u bench.py --no-cpu-baseline --stages" \
  "bench_c5_j:300:python -u bench.py --workload c5 --steps 3 --warmup 1" \
  "bench_c4_j:300:python -u bench.py --workload c4 --steps 3 --warmup 1"
