# one-GPU rehearsal of the N=8 profiling recipe (scripts/scale_curve.sh): the launcher outside the
# profiler, one rocprofv3 per rank (scripts/prof_rank.sh) with bench.py right after its `--`;
# 2 ranks on the box's one GPU -> two per-rank trace directories
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5y
rm -rf $O && mkdir -p $O
export MLT_BENCH_SAME_DEVICE=1 MLT_BENCH_BACKEND=gloo MLT_XGMI_ALLOW_GLOO=1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29561 --no-python scripts/prof_rank.sh $O -- python3 -u bench.py --gpus 2 --steps 100 --warmup 10 \
  --no-fp32-companion > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-300
for r in 0 1; do
  f=$(ls $O/r$r/*kernel_stats.csv 2>/dev/null | head -1)
  echo "== rank $r: $f"; [ -n "$f" ] && head -4 "$f" | cut -c1-160
done
find $O -name "*kernel_trace.csv" -delete
