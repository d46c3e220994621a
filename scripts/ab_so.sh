# Same-box A/B of two builds of the extension: the in-tree build ("new") against ab/_C*.so
# ("old"), alternated new/old/new/old in separate processes. Usage: bash scripts/ab_so.sh <cmd...>
# (each command's last output line is kept, tagged with the variant).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
SO=$(ls ml_trainer_amd/_C*.so)
cp "$SO" /tmp/ab_new.so
for v in new old new old; do
  if [ "$v" = new ]; then cp /tmp/ab_new.so "$SO"; else cp ab/_C*.so "$SO"; fi
  for c in "$@"; do
    timeout -k 10 240 bash -c "$c" > gpurun_out/ab_last.log 2>&1 || { echo "FAILED ($v): $c"; tail -5 gpurun_out/ab_last.log; cp /tmp/ab_new.so "$SO"; exit 1; }
    echo "{\"variant\": \"$v\", \"cmd\": \"$c\", \"out\": $(tail -1 gpurun_out/ab_last.log | python3 -c 'import json,sys; print(json.dumps(sys.stdin.read().strip()))')}" >> gpurun_out/ab.jsonl
  done
done
cp /tmp/ab_new.so "$SO"
