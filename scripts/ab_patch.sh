#!/bin/bash
# Same-box A/B of a kernel patch: run the given commands on the current build (A), apply the
# patch, rebuild in place, run them again (B). Any failing step ends the script.
#   scripts/ab_patch.sh PATCH "cmd1" "cmd2" ...
set -eu
patch="$1"; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in "$@"; do echo "=== A: $c"; timeout -k 10 300 bash -c "$c"; done
git apply "$patch" 2>/dev/null || patch -p1 < "$patch"
timeout -k 10 600 python -m ml_trainer_amd.build -j 16 > gpurun_out/ab_build.log 2>&1
for c in "$@"; do echo "=== B: $c"; timeout -k 10 300 bash -c "$c"; done
