# Final build re-validation after the attention changes: GPU suite, smoke, LeNet / BERT / fp8 benches,
# BERT-base kernel stats. Outputs under gpurun_out/final_b/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/final_b && O=gpurun_out/final_b
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > $O/gputests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/lenet20.log 2>&1 &&
timeout -k 10 200 python -u bench.py --model bert-base --steps 20 --warmup 5 > $O/bert.log 2>&1 &&
timeout -k 10 240 python -u bench.py --model large --steps 6 --warmup 2 > $O/large.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bert -o bert -- python3 -u bench.py --model bert-base --steps 5 --warmup 2 > $O/prof_bert.log 2>&1
