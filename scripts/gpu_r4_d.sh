#!/bin/bash
# Round 4: the fused data-parallel step with the granule exchange ({value, tag} 8-byte granules, no
# flags / barriers): loopback tests + timing against the local step, then the multi-process rehearsals.
set -o pipefail
O=gpurun_out/r4d
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_lenet_bf16.py -k "fused_dp" \
  > $O/t_fdp.log 2>&1 || { tail -30 $O/t_fdp.log; exit 1; }
tail -2 $O/t_fdp.log
: > $O/loop.jsonl
for b in 4 32; do
  for tr in auto xgmi-loopback; do
    timeout -k 10 120 python -u bench.py --steps 3000 --warmup 300 --batch $b --no-fp32-companion \
      --transport $tr --json-out $O/_last.json > /dev/null 2>$O/b.err || { tail $O/b.err; exit 1; }
    cat $O/_last.json >> $O/loop.jsonl; echo >> $O/loop.jsonl
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r4d/loop.jsonl"):
    if not l.strip(): continue
    d = json.loads(l); c = d["config"]
    print(c["per_gpu_batch"], c["dp_transport"], d["ms_per_step"], c["device_ms_per_step"])
PY
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_multiproc_gpu.py -k "fused_dp or three_four_eight" tests/test_trainer_parallel_gpu.py > $O/t_mp.log 2>&1 || { tail -40 $O/t_mp.log; exit 1; }
tail -15 $O/t_mp.log
