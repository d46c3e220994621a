# fp8 quantising FFN1 GEMM: epilogue cost decomposition (benchmarks/fp8_q8_decompose.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5aa
timeout -k 10 200 python3 -u benchmarks/fp8_q8_decompose.py > gpurun_out/r5aa/q8.log 2>&1; rc=$?
grep -v "^W2026\|amdgpu.ids" gpurun_out/r5aa/q8.log | tail -5
exit $rc
