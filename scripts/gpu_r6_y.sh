# BERT-base (bf16) same-box A/B of the attention kernels before / after the fp8 q8 epilogue
# (a uniform branch + 2-4 VGPRs on the bf16 path), then kernel statistics of the fp8 `large` step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6y
O=gpurun_out/r6y
bash scripts/ab_multi_so.sh "python -u bench.py --model bert-base --steps 20 --warmup 5" &&
cp gpurun_out/ab_multi.jsonl $O/ab.jsonl &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o large -- python3 -u bench.py --model large --steps 3 --warmup 2 > $O/p.log 2>&1
echo "rc=$?"
