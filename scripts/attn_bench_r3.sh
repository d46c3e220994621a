set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for b in 32 128 512; do ATTN_B=$b timeout -k 10 120 python3 -u benchmarks/attn_bench.py >> gpurun_out/attn_bench_r3.jsonl 2>gpurun_out/attn_bench.err || exit 1; done
bash scripts/attn_prof.sh r3 128 > gpurun_out/attn_prof_r3.log 2>&1
