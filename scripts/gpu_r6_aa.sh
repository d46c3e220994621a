# q8 attention epilogue: row-major e5m2 bytes also staged in LDS and stored as 16-byte pieces (q8v3)
# vs the direct dword stores (q8v1): the bitwise tests on q8v3, then the fp8 `large` A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6aa
O=gpurun_out/r6aa
timeout -k 10 300 python -u -m pytest tests/test_fp8_fused_gpu.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -k "attn" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
bash scripts/ab_multi_so.sh "python -u bench.py --model large --steps 20 --warmup 5" &&
cp gpurun_out/ab_multi.jsonl $O/ab.jsonl
echo "rc=$?"
