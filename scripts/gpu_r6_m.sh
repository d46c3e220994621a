# Driver-protocol LeNet step (--steps 20 --warmup 5): host sync spin (default now) vs ROCm's
# default yield, and steps per graph 5 (default: the warmup replays the timed graph) vs 20 (one
# cold graph) vs a warm 20-step graph (--warmup 20).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6m
O=gpurun_out/r6m
: > $O/spg.jsonl
for rep in 1 2 3; do
  for cfg in "MLT_SYNC_SPIN=0|--steps 20 --warmup 5" "MLT_SYNC_SPIN=1|--steps 20 --warmup 5" "MLT_SYNC_SPIN=1|--steps 20 --warmup 5 --steps-per-graph 20" "MLT_SYNC_SPIN=1|--steps 20 --warmup 20" "MLT_SYNC_SPIN=0|--steps 20 --warmup 20"; do
    e=${cfg%%|*}; a=${cfg#*|}
    env $e timeout -k 10 120 python3 -u bench.py $a --no-fp32-companion > $O/last.log 2>&1 || { tail -5 $O/last.log; exit 1; }
    echo "{\"env\": \"$e\", \"cfg\": \"$a\", \"r\": $(grep '^{' $O/last.log)}" >> $O/spg.jsonl
  done
done
timeout -k 10 200 python3 -u bench.py --steps 1000 --warmup 100 > $O/steady.log 2>&1
echo ok
