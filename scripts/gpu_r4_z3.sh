#!/bin/bash
# Round 4: round-start build (ab/a_old.so, commit 7782c6c) vs the packed-GELU build (ab/c_pk_q8.so),
# driver protocol, same box: fp8 `large` and BERT-base.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4z3
mkdir -p $O
bash scripts/ab_multi_so.sh "python bench.py --model large --steps 20 --warmup 5" "python bench.py --model bert-base --steps 20 --warmup 5" || exit 1
cp gpurun_out/ab_multi.jsonl $O/ab_multi.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/r4z3/ab_multi.jsonl"):
    d = json.loads(l); o = json.loads(d["out"])
    print(d["variant"], o["config"]["model"][:20], o.get("value"))
PY
