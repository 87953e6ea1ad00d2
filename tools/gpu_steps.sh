#!/bin/bash
# Run GPU steps in order on the gpurun box; each step has its own time limit.
# A step that fails normally (exit 1: a failed assertion) does not stop the
# sequence; a fault, abort, segfault or time limit (124, 134, 137, 139, or any
# code >= 128) ends it: nothing more touches the GPU in this call.
# usage: tools/gpu_steps.sh "NAME|SECONDS|COMMAND" ...
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $name (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "=== stopping: $name ended with $rc"
    exit $rc
  fi
done
exit 0
