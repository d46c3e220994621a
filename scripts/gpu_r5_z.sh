# attention backward launch tunables at B512 (ring depth / key-query groups), and BERT-base per-GPU
# batch 1024 vs 1536 under the driver protocol
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5z
mkdir -p $O
: > $O/attn.jsonl
for ring in 4 3; do
  for kv in 2 1; do
    for q in 2 1; do
      MLT_ATTN_RING=$ring MLT_ATTN_DKDV_GROUPS=$kv MLT_ATTN_DQ_GROUPS=$q ATTN_B=512 timeout -k 10 120 python3 -u benchmarks/attn_bench.py \
        > $O/last.log 2>&1 || { tail -5 $O/last.log; exit 1; }
      echo "{\"ring\": $ring, \"kv\": $kv, \"q\": $q, \"r\": $(tail -1 $O/last.log)}" >> $O/attn.jsonl
    done
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r5z/attn.jsonl"):
    d = json.loads(l); r = d["r"]
    print(d["ring"], d["kv"], d["q"], r["native_bwd"], r["native_fwd"])
PY
for b in 1024 1536 1024 1536; do
  timeout -k 10 300 python3 -u bench.py --model bert-base --batch $b --steps 10 --warmup 3 > $O/bert_$b.log 2>&1 || { tail -5 $O/bert_$b.log; exit 1; }
  echo "bert batch $b: $(grep '^{' $O/bert_$b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["peak_hbm_gib"])')"
done
