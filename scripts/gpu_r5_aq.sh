# last check on the final build: full GPU suite, smoke, default bench (driver protocol)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/aq
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/aq/gputests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/aq/smoke.log 2>&1 &&
timeout -k 10 120 python -u bench.py > gpurun_out/aq/bench.log 2>&1
rc=$?
tail -1 gpurun_out/aq/gputests.log; tail -1 gpurun_out/aq/smoke.log; grep '^{' gpurun_out/aq/bench.log | cut -c1-160
exit $rc
