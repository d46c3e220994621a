#!/bin/bash
# Run a sequence of GPU steps on the gpurun box. Each step has its own time
# limit; the sequence stops at the first fault/abort/timeout (any rc other than
# 0 or 1), so nothing else touches the GPU after trouble.
#   usage: scripts/gpu_session.sh "name|timeout|command" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; to="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${to}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 15 "gpurun_out/$name.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "=== stopping: step $name ended with rc=$rc"
    exit "$rc"
  fi
done
