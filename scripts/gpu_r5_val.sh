# Round-5 validation on one MI355X: full GPU suite, smoke, LeNet benches (driver protocol / steady
# state / batch 4 / xGMI loopback), BERT-base and fp8 large under the driver protocol.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/val
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/val/gputests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/val/smoke.log 2>&1 &&
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > gpurun_out/val/lenet20.log 2>&1 &&
timeout -k 10 120 python -u bench.py > gpurun_out/val/lenet.log 2>&1 &&
timeout -k 10 120 python -u bench.py --batch 4 > gpurun_out/val/lenet_b4.log 2>&1 &&
timeout -k 10 120 python -u bench.py --batch 4 --transport xgmi-loopback > gpurun_out/val/lenet_b4_lb.log 2>&1 &&
timeout -k 10 240 python -u bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/val/bert.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model large --steps 6 --warmup 2 > gpurun_out/val/large.log 2>&1
