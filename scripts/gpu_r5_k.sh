# fp8 quantising (q8) FFN epilogues with the exact GELU / GELU' tables (in-tree = ab/a_q8tab.so) vs the
# A&S erf polynomial (ab/b_q8erf.so): GEMM / fp8 GPU tests on the in-tree build, then a same-box
# A/B of the fused FFN bench at the large config's shapes and the fp8 `large` bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5k
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gemm_gpu.py tests/test_fp8_gpu.py tests/test_fp8_fused_gpu.py tests/test_transformer_gpu.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/ab_multi_so.sh "FFN_BENCH_TOKENS=131072,262144 python benchmarks/fp8_fused_ffn_bench.py" \
  "python bench.py --model large --steps 6 --warmup 2" || exit 1
cp gpurun_out/ab_multi.jsonl $O/ab_multi.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/r5k/ab_multi.jsonl"):
    d = json.loads(l)
    try:
        o = json.loads(d["out"])
    except Exception:
        print(d["variant"], d["out"][:300]); continue
    print(d["variant"], o.get("value") or o)
PY
