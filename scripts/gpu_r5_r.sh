# LeNet driver protocol at K=20: warmup length vs graph length vs the limited-replay warmup, alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5r
mkdir -p $O
: > $O/ab.jsonl
for rep in 1 2 3; do
  for v in "--warmup 5 --steps-per-graph 5" "--warmup 5" "--warmup 20 --steps-per-graph 5" "--warmup 20 --steps-per-graph 20" "--warmup 200 --steps-per-graph 20"; do
    timeout -k 10 120 python3 -u bench.py --steps 20 $v --no-fp32-companion > $O/last.log 2>&1 || { tail -5 $O/last.log; exit 1; }
    echo "{\"rep\": $rep, \"v\": \"$v\", \"line\": $(grep '^{' $O/last.log)}" >> $O/ab.jsonl
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r5r/ab.jsonl"):
    d = json.loads(l)
    print(d["rep"], d["v"], round(d["line"]["ms_per_step"] * 1e3, 3), d["line"]["config"]["hipgraph_steps"])
PY
