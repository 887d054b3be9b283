#!/bin/bash
# GPU-box step runner (via gpurun, from the repo root):
#   bash tools/gpu_run.sh <tag> '<name>|<seconds>|<command>' ...
# Each step runs under its own time limit with output in gpurun_out/<tag>/<name>.log.  A step that
# ends with 0 (pass) or 1 (test failures) lets the next one run; anything else (a fault, an abort,
# a time limit) ends the call there.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
TAG=$1; shift
mkdir -p "gpurun_out/$TAG"
worst=0
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$TAG/$name.log" 2>&1
  rc=$?
  echo "step $name rc=$rc"
  tail -3 "gpurun_out/$TAG/$name.log"
  [ $rc -gt $worst ] && worst=$rc
  if [ $rc -gt 1 ]; then echo "stopping after $name"; exit $rc; fi
done
exit $worst
