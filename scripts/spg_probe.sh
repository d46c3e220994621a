#!/bin/bash
# LeNet driver-protocol runs (--steps 20 --warmup 5) at several steps-per-graph values,
# interleaved, 3 rounds; one JSON line per run in gpurun_out/spg_probe.jsonl
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/spg_probe.jsonl
for r in 1 2 3; do
  for spg in 0 5 10 4; do
    out=$(timeout -k 5 60 python3 bench.py --steps 20 --warmup 5 --steps-per-graph $spg 2>/dev/null | grep '^{') || exit 3
    echo "{\"round\": $r, \"spg\": $spg, \"res\": $out}" >> gpurun_out/spg_probe.jsonl
    echo "r$r spg=$spg $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
  done
done
