#!/bin/bash
# Parameterised GPU recipe (replaces the one-off g*.sh scripts): runs the named steps in
# order via tools/gpu_run.sh, each under its own time limit, stopping at a timeout/abort/
# fault.  usage: tools/gpu_steps.sh TAG step [step ...]
#   steps: tests (all -m gpu), t:<pytest -k expr>, smoke, bench[:extra args], stages,
#          prof (rocprofv3 kernel stats of the default bench), pmcf / pmcw (FETCH/WRITE_SIZE),
#          kb:<kbench args>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
specs=()
for s in "$@"; do
  case "$s" in
    tests) specs+=("tests_$TAG:500:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread") ;;
    t:*) specs+=("t_$TAG:400:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k '${s#t:}'") ;;
    smoke) specs+=("smoke_$TAG:200:python -c 'import __graft_entry__ as g; g.smoke()'") ;;
    bench) specs+=("bench_$TAG:300:python bench.py --steps 20 --warmup 5") ;;
    bench:*) specs+=("bench_$TAG:400:python bench.py ${s#bench:}") ;;
    stages) specs+=("stages_$TAG:300:python bench.py --steps 5 --warmup 2 --stages --no-cpu-baseline") ;;
    prof) specs+=("prof_$TAG:300:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline") ;;
    pmcf) specs+=("pmcf_$TAG:240:rocprofv3 --pmc FETCH_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcf_$TAG -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline") ;;
    pmcw) specs+=("pmcw_$TAG:240:rocprofv3 --pmc WRITE_SIZE --kernel-include-regex fmx -f csv -d gpurun_out/pmcw_$TAG -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline") ;;
    kb:*) specs+=("kb_$TAG:240:python tools/kbench.py ${s#kb:}") ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exec_rc=0
tools/gpu_run.sh "${specs[@]}" || exec_rc=$?
exit $exec_rc
