#!/bin/bash
# Run GPU steps in order; continue past ordinary test failures (rc 1) but stop
# at faults / aborts / timeouts (rc >= 2) so nothing else touches a sick GPU.
# usage: gpurun_step.sh "<name>:<timeout>:<cmd>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; to="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] $cmd (timeout ${to}s)"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc"; tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ge 2 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
