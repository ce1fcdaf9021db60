#!/bin/bash
# One GPU session: steps run in order under their own time limits; a crash
# (abort/segfault/timeout) ends the session, a plain test failure does not.
# usage: tools/gpu_run.sh "<name>:<timeout_s>:<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; tmo="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (timeout ${tmo}s): $cmd"
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  case $rc in
    0|1|2) ;;   # ok / test failures / usage
    *) echo "=== stopping: $name ended with rc=$rc"; exit $rc ;;
  esac
done
