# (1) cfg 7 GELU / dGELU epilogues from exact bf16-point tables (in-tree = ab/a_tab.so) vs the A&S
#     erf polynomial (ab/b_erf.so); (2) attention backward with explicit packed-f32 softmax-gradient
#     math (ab/c_attnpk.so, table build otherwise). GEMM / transformer / fp8 GPU tests on the in-tree
#     build, attention tests on the packed build, then a same-box A/B of all three builds and the
#     VALU/MFMA PMC pass of the attention kernels for a_tab vs c_attnpk.
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5j
mkdir -p $O
SO=$(ls ml_trainer_amd/_C*.so)
cp "$SO" /tmp/j_intree.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gemm_gpu.py tests/test_transformer_gpu.py tests/test_fp8_gpu.py tests/test_fp8_fused_gpu.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cp ab/c_attnpk.so "$SO"
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -m gpu -x -q -k "attn or attention" --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/attn_tests_pk.log 2>&1
rc=$?
cp /tmp/j_intree.so "$SO"
[ $rc -eq 0 ] || { echo "packed attention build failed its tests"; tail -20 $O/attn_tests_pk.log; exit 1; }
tail -1 $O/attn_tests_pk.log
bash scripts/ab_multi_so.sh "GEMM_BENCH_TOKENS=262144 python benchmarks/gemm_epi_bench.py" \
  "ATTN_B=512 python3 -u benchmarks/attn_bench.py" "python bench.py --model bert-base --steps 20 --warmup 5" || exit 1
cp gpurun_out/ab_multi.jsonl $O/ab_multi.jsonl
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
for v in a_tab c_attnpk; do
  cp ab/$v.so "$SO"
  i=0
  for grp in "$P1" "$P2"; do
    i=$((i + 1))
    ATTN_B=512 timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/${v}_p$i -o run -- \
      python3 -u benchmarks/attn_bench.py > $O/${v}_p$i.log 2>&1 || { cp /tmp/j_intree.so "$SO"; echo "pmc $v p$i failed"; exit 1; }
  done
  cp /tmp/j_intree.so "$SO"
  python3 scripts/pmc_summary.py $O/${v}_p1 $O/${v}_p2 --match attn --jsonl $O/pmc_$v.jsonl > $O/pmc_$v.txt
done
rm -rf $O/a_tab_p* $O/c_attnpk_p*
python3 - <<'PY'
import json
for l in open("gpurun_out/r5j/ab_multi.jsonl"):
    d = json.loads(l)
    try:
        o = json.loads(d["out"])
    except Exception:
        print(d["variant"], d["out"][:200]); continue
    print(d["variant"], o.get("value") or {k: v for k, v in o.items() if k.endswith("tflops") or k.startswith("native")})
PY
