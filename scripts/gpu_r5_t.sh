# warm-graph probe on the device-step-limit build (ab/pkg_steplimit)
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5t
PYTHONPATH=ab/pkg_steplimit timeout -k 10 200 python3 -u scripts/debug/warm_graph_probe.py > gpurun_out/r5t/probe.log 2>&1; rc=$?
grep -v "^W2026\|amdgpu.ids" gpurun_out/r5t/probe.log
exit $rc
