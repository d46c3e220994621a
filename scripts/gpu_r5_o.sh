# cold vs warm replays of freshly captured + uploaded multi-step LeNet graphs
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5o
timeout -k 10 120 python3 -u scripts/debug/replay_cold.py > gpurun_out/r5o/replay_cold.log 2>&1; rc=$?
cat gpurun_out/r5o/replay_cold.log | grep -v "^W2026"
exit $rc
