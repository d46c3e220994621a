# two-phase exchange as kernels of its own (lenet_mwx<D, W | kXchTwo>), X last in the argument list:
# the DP GPU tests, then the loopback A/B against the build before the two-phase form (ab/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5x
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_multiproc_gpu.py tests/test_lenet_bf16.py tests/test_trainer_parallel_gpu.py tests/test_comm_gpu.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/ab_so.sh "python bench.py --batch 4 --transport xgmi-loopback --no-fp32-companion" \
  "python bench.py --transport xgmi-loopback --no-fp32-companion" "python bench.py --no-fp32-companion" || exit 1
cp gpurun_out/ab.jsonl $O/ab.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/r5x/ab.jsonl"):
    d = json.loads(l); o = json.loads(d["out"])
    print(d["variant"], d["cmd"][13:60], o["value"], o["ms_per_step"])
PY
