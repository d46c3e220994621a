# (1) the N=2 LeNet bench rehearsal through the xGMI paths on one GPU (scripts/gpu_r6_u.sh);
# (2) streaming stores for the per-sample slabs and the update's outputs (v20) vs plain (v18).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6v
O=gpurun_out/r6v
bash scripts/gpu_r6_u.sh > $O/u.log 2>&1 || { tail -20 $O/u.log; exit 1; }
bash scripts/ab_multi_so.sh "python -u bench.py --steps 20 --warmup 5 --no-fp32-companion" "python -u bench.py --no-fp32-companion" "python -u bench.py --batch 4 --transport xgmi-loopback --no-fp32-companion" &&
cp gpurun_out/ab_multi.jsonl $O/ab.jsonl
echo "rc=$?"
