"""Timeline of the one-launch bf16 LeNet step (lenet_ms<D, 0>, LENET_TRACE): per update block the
start, its wave 0's task issue end / drain, and the arrival; per sample block the start, the moment
it saw all arrivals (weights handed over), and the end; block 0's phase stamps. 100 MHz wall clock.
Usage: python benchmarks/lenet_onelaunch_trace.py [batch] [--jsonl F]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.models.lenet import MLModel  # noqa: E402
from ml_trainer_amd.models.lenet_engine import LeNetStepEngine  # noqa: E402
from ml_trainer_amd.ops.optim import build_optimizer  # noqa: E402
from ml_trainer_amd.utils.flat import FlatParams  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
B = int(args[0]) if args else 32
out = sys.argv[sys.argv.index("--jsonl") + 1] if "--jsonl" in sys.argv else None
dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = MLModel().to(dev)
flat = FlatParams(m.parameters())
opt = build_optimizer("sgd", m.parameters(), lr=1e-3, momentum=0.9, flat=flat)
eng = LeNetStepEngine(m, flat, max_batch=B, optimizer=opt, precision="bf16")
trace = torch.zeros(4096, dtype=torch.float32, device=dev)  # (one-launch stamps up to slot 1299)
eng.bufs["trace"] = trace
eng.eng = eng.C.LeNetEngine(m.cfg_id, B, eng.bufs)  # rebuild with the trace buffer bound
eng.eng.set_ctrl(eng.ctrl)
eng.eng.set_precision(1)
eng.set_optimizer(opt)
N = 4096
data = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8)
targets = torch.randint(0, 10, (N,))
eng.set_dataset(data, targets, batch_size=B)
eng.start_epoch(torch.randperm(N))
eng.train_steps(B, 20, use_graph=False)
C = eng.C
mode = C.LENET_FWD | C.LENET_CE | C.LENET_BWD | C.LENET_OPT | C.LENET_TRACE
U = C.lenet_mfma_kw_blocks(m.cfg_id)  # update blocks = the lenet_mw grid
recs = []
for rep in range(9):
    trace.zero_()
    eng.eng.run(mode, B)  # one launch: this step + the previous step's update
    torch.cuda.synchronize()
    tr = trace.view(torch.int64).cpu().tolist()
    ks = [(tr[600 + 2 * i], tr[1100 + i], tr[601 + 2 * i]) for i in range(min(B, 200))]
    up = [(tr[64 + 5 * u], tr[66 + 5 * u], tr[67 + 5 * u], tr[65 + 5 * u]) for u in range(min(U, 100))]
    t0 = min([a for a, _, _ in ks] + [a for a, _, _, _ in up])
    ns = lambda v: (v - t0) * 10  # noqa: E731
    recs.append({
        "upd_start_ns": [ns(a) for a, _, _, _ in up], "upd_issued_ns": [ns(b) for _, b, _, _ in up],
        "upd_drained_ns": [ns(c) for _, _, c, _ in up], "upd_arrive_ns": [ns(d) for _, _, _, d in up],
        "smp_start_ns": [ns(a) for a, _, _ in ks], "smp_go_ns": [ns(g) for _, g, _ in ks],
        "smp_end_ns": [ns(e) for _, _, e in ks]})
eng.flush()
r = recs[len(recs) // 2]
summ = {k: (min(v), max(v)) for k, v in r.items()}
for k, (lo, hi) in summ.items():
    print(f"  {k:16s} {lo:7d} .. {hi:7d} ns")
rec = {"batch": B, "median_rep": r, "ranges": summ}
if out:
    with open(out, "a") as f:
        f.write(json.dumps(rec) + "\n")
