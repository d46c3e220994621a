# Decompose the driver-protocol timed region of the LeNet bf16 step: total time T(K) = K steps
# for K = 5 .. 320 at 5 steps per graph (and 1 / 20 per graph at K = 20), fitted as a + b K on the
# host (a = fixed launch / synchronize latency per region, b = device time per step).
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5n
mkdir -p $O
: > $O/region.jsonl
for rep in 1 2; do
  for k in 5 10 20 40 80 160 320; do
    timeout -k 10 120 python3 -u bench.py --steps $k --warmup 5 --steps-per-graph 5 --no-fp32-companion > $O/last.log 2>&1 || { tail -5 $O/last.log; exit 1; }
    echo "{\"rep\": $rep, \"K\": $k, \"spg\": 5, \"line\": $(grep '^{' $O/last.log)}" >> $O/region.jsonl
  done
  for spg in 1 20; do
    timeout -k 10 120 python3 -u bench.py --steps 20 --warmup 20 --steps-per-graph $spg --no-fp32-companion > $O/last.log 2>&1 || { tail -5 $O/last.log; exit 1; }
    echo "{\"rep\": $rep, \"K\": 20, \"spg\": $spg, \"line\": $(grep '^{' $O/last.log)}" >> $O/region.jsonl
  done
done
python3 - <<'PY'
import json
import numpy as np
rows = [json.loads(l) for l in open("gpurun_out/r5n/region.jsonl")]
pts = [(r["K"], r["line"]["ms_per_step"] * r["K"] * 1e3) for r in rows if r["spg"] == 5]
K = np.array([p[0] for p in pts], float); T = np.array([p[1] for p in pts])
b, a = np.polyfit(K, T, 1)
print(f"fit T(K) = {a:.1f} us + {b:.3f} us * K")
for r in rows:
    print(r["rep"], r["K"], r["spg"], round(r["line"]["ms_per_step"] * 1e3, 3), "us/step")
PY
