# One-GPU rehearsal of the node recipe (scripts/scale_curve.sh, MLT_SCALE_REHEARSE=1): every line of
# BASELINE configs 2-5 at N in {1, 2}, both ranks on GPU 0 over gloo, small batches.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
MLT_SCALE_REHEARSE=1 timeout -k 10 1000 bash scripts/scale_curve.sh > gpurun_out/rehearse_scale.log 2>&1
rc=$?
cp gpurun_out/scale_curve.jsonl gpurun_out/rehearse_scale_curve.jsonl 2>/dev/null
echo "rc=$rc"
exit $rc
