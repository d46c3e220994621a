#!/bin/bash
# Round 4, part B: multi-process rehearsals of the data-parallel paths on one GPU (gloo rendezvous):
# fused vs four-launch bf16 step at W = 2 / 8, the xGMI kernels bit-exact at W = 3 / 4 / 8, the
# Trainer(is_parallel) path incl. TransportError -> resume.
set -o pipefail
O=gpurun_out/r4b
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_multiproc_gpu.py -k "fused_dp or three_four_eight" tests/test_trainer_parallel_gpu.py > $O/t_mp.log 2>&1 || { tail -40 $O/t_mp.log; exit 1; }
tail -15 $O/t_mp.log
