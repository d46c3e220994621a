#!/bin/bash
# Per-rank profiler wrapper for multi-rank runs. The launcher starts one of these per rank:
#   python3 -m torch.distributed.run --no-python --nproc-per-node N ... \
#       scripts/prof_rank.sh OUTDIR -- python3 -u bench.py --gpus N ...
# This shell touches no GPU; it execs rocprofv3 with the rank's program DIRECTLY after `--`, so
# nothing between the profiler (whose preloaded library initialises the GPU) and the program
# spawns or re-execs. WORLD_SIZE / RANK / LOCAL_RANK come from the launcher, so bench.py does not
# self-launch. Each rank writes its own trace under OUTDIR/r<LOCAL_RANK>.
set -eu
out="$1"
shift
if [ "${1:-}" = "--" ]; then shift; fi
: "${LOCAL_RANK:?prof_rank.sh must be started by torch.distributed.run (LOCAL_RANK unset)}"
: "${WORLD_SIZE:?prof_rank.sh must be started by torch.distributed.run (WORLD_SIZE unset)}"
mkdir -p "$out/r$LOCAL_RANK"
exec rocprofv3 --kernel-trace --stats --output-format csv -d "$out/r$LOCAL_RANK" -o "rank$LOCAL_RANK" -- "$@"
