#!/bin/bash
# Round 6, call T: the driver's round-end sequence on the final tree -- the whole -m gpu
# suite (full size included), smoke(), the default bench line.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
tools/gpu_run.sh \
  "gputests_t:1100:python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider" \
  "smoke_t:200:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "bench_c2_t:300:python -u bench.py --steps 20 --warmup 2"
