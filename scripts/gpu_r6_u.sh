# One-GPU rehearsal of the N=2 LeNet bench through the xGMI paths (both ranks on GPU 0, gloo group,
# MLT_XGMI_ALLOW_GLOO): transport bring-up + vote, the graph pre-launch with restore, weak and
# reference batch semantics. Times measure two processes sharing one GPU, not a node.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6u
O=gpurun_out/r6u
export MLT_BENCH_SAME_DEVICE=1 MLT_BENCH_BACKEND=gloo MLT_XGMI_ALLOW_GLOO=1 MLT_XGMI_TIMEOUT_MS=20000
: > $O/rehearse_n2.jsonl
for a in "--scaling weak" "--scaling reference" "--scaling weak --no-prewarm"; do
  timeout -k 10 300 python3 -u bench.py --gpus 2 --steps 20 --warmup 5 --no-fp32-companion $a > $O/last.log 2>&1 || { tail -20 $O/last.log; exit 1; }
  echo "{\"args\": \"$a\", \"r\": $(grep '^{' $O/last.log)}" >> $O/rehearse_n2.jsonl
done
echo ok
