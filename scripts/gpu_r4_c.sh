#!/bin/bash
# Round 4: the fused data-parallel step's exchange protocol on one GPU (xGMI loopback): proto 0 =
# sc0 sc1 payload / flags without fences + device error word (default), 1 = release / acquire fences,
# 2 = host-mapped error word, 3 = both (the first version). Then the multi-process rehearsals.
set -o pipefail
O=gpurun_out/r4c
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_lenet_bf16.py -k "fused_dp" \
  > $O/t_fdp.log 2>&1 || { tail -30 $O/t_fdp.log; exit 1; }
tail -2 $O/t_fdp.log
: > $O/loop.jsonl
for b in 4 32; do
  timeout -k 10 120 python -u bench.py --steps 3000 --warmup 300 --batch $b --no-fp32-companion >> $O/loop.jsonl 2>$O/b.err || exit 1
  for pr in 0 1 2 3; do
    MLT_XGMI_PROTO=$pr timeout -k 10 120 python -u bench.py --steps 3000 --warmup 300 --batch $b --no-fp32-companion \
      --transport xgmi-loopback --json-out $O/_last.json > /dev/null 2>$O/b.err || exit 1
    python3 -c "import json; d=json.load(open('$O/_last.json')); d['proto']=$pr; print(json.dumps(d))" >> $O/loop.jsonl
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r4c/loop.jsonl"):
    d = json.loads(l); c = d["config"]
    print(c["per_gpu_batch"], c["dp_transport"], d.get("proto"), d["ms_per_step"], c["device_ms_per_step"])
PY
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_multiproc_gpu.py -k "fused_dp or three_four_eight" tests/test_trainer_parallel_gpu.py > $O/t_mp.log 2>&1 || { tail -40 $O/t_mp.log; exit 1; }
tail -15 $O/t_mp.log
