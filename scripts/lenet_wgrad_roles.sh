#!/bin/bash
# Time the LeNet weight-gradient kernel with each role dropped (MLT_LENET_WGRAD_SKIP; needs a
# debug build: python -m ml_trainer_amd.build --debug), to find
# which role sets its critical path. rocprofv3 kernel stats per mask under gpurun_out/wgrad_roles/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/wgrad_roles
for m in 0 1 2 4 3 5 6; do
  MLT_LENET_WGRAD_SKIP=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/wgrad_roles/m$m -o k -- python bench.py --steps 400 --warmup 50 > gpurun_out/wgrad_roles/m$m.log 2>&1 || exit 1
done
