# one-wave-ring GEMM main-loop probe (benchmarks/gemm_w4_probe.hip, built on the CPU side):
# 8192^3 and the BERT-base GEMM shapes at 64K tokens, several K values for a main-loop fit
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 120 ./benchmarks/bin/gemm_w4_probe 8192 8192 8192 65536 3072 768 65536 2304 768 65536 768 768 65536 768 3072 16384 3072 768 16384 3072 1536 16384 3072 3072 > gpurun_out/gemm_probe.jsonl 2> gpurun_out/gemm_probe.err
