# raster group width of the 4-wave quantising fp8 FFN GEMMs (MLT_GEMM_W4Q8_GROUP_M 2 / 4 / 8 / 16)
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ao
mkdir -p $O
: > $O/gm.jsonl
for g in 4 2 8 16 4 2 8 16; do
  MLT_GEMM_W4Q8_GROUP_M=$g timeout -k 10 120 python3 -u benchmarks/fp8_q8_decompose.py > $O/d.log 2>&1 || { tail -5 $O/d.log; exit 1; }
  echo "{\"group_m\": $g, \"r\": $(tail -1 $O/d.log)}" >> $O/gm.jsonl
  echo "group_m=$g $(tail -1 $O/d.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["q8_gelu_ms"], d["q8_dgelu_ms"])')"
done
