# Same-box A/B over several builds of the extension: ab/<name>.so, cycled twice in separate
# processes. Usage: bash scripts/ab_multi_so.sh <cmd...>; lines -> gpurun_out/ab_multi.jsonl
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && rm -f gpurun_out/ab_multi.jsonl
SO=$(ls ml_trainer_amd/_C*.so)
cp "$SO" /tmp/ab_intree.so
for rep in 1 2; do
  for v in ab/*.so; do
    cp "$v" "$SO"
    for c in "$@"; do
      timeout -k 10 240 bash -c "$c" > gpurun_out/ab_last.log 2>&1 || { echo "FAILED ($v): $c"; tail -5 gpurun_out/ab_last.log; cp /tmp/ab_intree.so "$SO"; exit 1; }
      echo "{\"variant\": \"$(basename $v .so)\", \"cmd\": \"$c\", \"out\": $(tail -1 gpurun_out/ab_last.log | python3 -c 'import json,sys; print(json.dumps(sys.stdin.read().strip()))')}" >> gpurun_out/ab_multi.jsonl
    done
  done
done
cp /tmp/ab_intree.so "$SO"
