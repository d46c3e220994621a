#!/bin/bash
# Round 4: BERT-base at the new bench default (batch 1024) and at 512, driver protocol.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4y
mkdir -p $O
timeout -k 10 400 python -u bench.py --model bert-base --steps 20 --warmup 5 > $O/bert1024.json 2>$O/b.err || { tail $O/b.err; exit 1; }
tail -1 $O/bert1024.json | cut -c1-200
timeout -k 10 400 python -u bench.py --model bert-base --steps 20 --warmup 5 --batch 512 > $O/bert512.json 2>$O/b.err || { tail $O/b.err; exit 1; }
tail -1 $O/bert512.json | cut -c1-200
