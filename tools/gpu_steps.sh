#!/usr/bin/env bash
# Run GPU steps in order, each under its own time limit; stop at the first
# step that timed out, was killed, aborted or segfaulted (124/137/134/139, or
# any signal).  Ordinary failures (exit 1/2: test failures) do not stop the
# sequence.  Usage: tools/gpu_steps.sh "name|seconds|command" ...
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rc_all=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"
  secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (${secs}s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then rc_all=$rc; fi
  case $rc in
    0|1|2|3|4|5) ;;
    *) echo "=== fatal rc=$rc: stopping" | tee -a gpurun_out/steps.log; exit $rc ;;
  esac
done
exit $rc_all
