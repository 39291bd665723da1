#!/bin/bash
# Run GPU steps in order; each step has its own time limit.  Stop at the first step that
# times out (124/137), aborts (134) or faults (139); a plain non-zero exit (e.g. a failing
# test) is recorded and the next step still runs.
# usage: tools/gpu_run.sh "<name>:<seconds>:<command>" ...
mkdir -p gpurun_out
rc_all=0
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc after $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  case $rc in
    0) ;;
    124|137|134|139|-6|-11) echo "=== stopping: step $name ended with $rc"; exit $rc ;;
    *) rc_all=$rc ;;
  esac
done
exit $rc_all
