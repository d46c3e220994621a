# host wait mode A/B: MLT_SYNC_SPIN=1 (hipDeviceScheduleSpin) vs 0, LeNet driver protocol, alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && : > gpurun_out/ab_spin.jsonl
for rep in 1 2 3; do
  for sp in 1 0; do
    for b in 32 4; do
      MLT_SYNC_SPIN=$sp timeout -k 10 120 python3 -u bench.py --batch $b --steps 20 --warmup 5 > gpurun_out/ab.log 2>&1 || exit 1
      echo "{\"spin\": $sp, \"batch\": $b, \"rep\": $rep, \"line\": $(grep '^{' gpurun_out/ab.log)}" >> gpurun_out/ab_spin.jsonl
    done
  done
done
MLT_SYNC_SPIN=1 timeout -k 10 120 python3 -u bench.py > gpurun_out/ab.log 2>&1 && echo "{\"spin\": 1, \"batch\": 32, \"rep\": 0, \"line\": $(grep '^{' gpurun_out/ab.log)}" >> gpurun_out/ab_spin.jsonl
