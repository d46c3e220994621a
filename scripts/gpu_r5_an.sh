# fp8 / bf16 ratio at batch 256 (verdict item): bf16 bert-large vs fp8 large, alternated on one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5an
mkdir -p $O
: > $O/ratio.jsonl
for m in bert-large large bert-large large; do
  timeout -k 10 300 python3 -u bench.py --model $m --batch 256 --steps 10 --warmup 3 > $O/r.log 2>&1 || { tail -5 $O/r.log; exit 1; }
  echo "{\"model\": \"$m\", \"r\": $(grep '^{' $O/r.log)}" >> $O/ratio.jsonl
  echo "$m b256: $(grep '^{' $O/r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["dtype"])')"
done
