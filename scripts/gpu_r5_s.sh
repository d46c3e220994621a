# host-side anatomy of the LeNet timed region (scripts/debug/timed_region_probe.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5s
timeout -k 10 120 python3 -u scripts/debug/timed_region_probe.py > gpurun_out/r5s/probe.log 2>&1; rc=$?
grep -v "^W2026\|amdgpu.ids" gpurun_out/r5s/probe.log
exit $rc
