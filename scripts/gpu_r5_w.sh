# same-box A/B: the build with the two-phase fused exchange (in-tree) vs the one before it (ab/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5w
bash scripts/ab_so.sh "python bench.py --batch 4 --transport xgmi-loopback --no-fp32-companion" \
  "python bench.py --transport xgmi-loopback --no-fp32-companion" || exit 1
cp gpurun_out/ab.jsonl gpurun_out/r5w/ab.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/r5w/ab.jsonl"):
    d = json.loads(l); o = json.loads(d["out"])
    print(d["variant"], d["cmd"][13:60], o["value"], o["ms_per_step"])
PY
