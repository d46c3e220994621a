#!/bin/bash
# Round 4 validation on one box: the whole GPU suite, smoke(), the headline bench under the driver
# protocol (+ batch 4 and the default steady-state run), BERT-base and fp8 large.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4val
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $O/lenet20.json 2>$O/b.err || { tail $O/b.err; exit 1; }
tail -1 $O/lenet20.json | cut -c1-400
timeout -k 10 180 python -u bench.py > $O/lenet_default.json 2>$O/b.err || { tail $O/b.err; exit 1; }
tail -1 $O/lenet_default.json | cut -c1-200
timeout -k 10 180 python -u bench.py --batch 4 --no-fp32-companion > $O/lenet_b4.json 2>$O/b.err || { tail $O/b.err; exit 1; }
tail -1 $O/lenet_b4.json | cut -c1-200
timeout -k 10 300 python -u bench.py --model bert-base --steps 20 --warmup 5 > $O/bert.json 2>$O/b.err || { tail $O/b.err; exit 1; }
tail -1 $O/bert.json | cut -c1-200
timeout -k 10 400 python -u bench.py --model large --steps 20 --warmup 5 > $O/large.json 2>$O/b.err || { tail $O/b.err; exit 1; }
tail -1 $O/large.json | cut -c1-200
timeout -k 10 400 python -u bench.py --model large --steps 6 --warmup 2 --batch 256 > $O/large256.json 2>$O/b.err || { tail $O/b.err; exit 1; }
tail -1 $O/large256.json | cut -c1-200
timeout -k 10 400 python -u bench.py --model bert-large --steps 6 --warmup 2 --batch 256 > $O/bertlarge256.json 2>$O/b.err || { tail $O/b.err; exit 1; }
tail -1 $O/bertlarge256.json | cut -c1-200
