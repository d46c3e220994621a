"""Per-phase timing of the fused per-sample LeNet kernel (LENET_TRACE): block 0 stores clock64()
stamps at every phase boundary; printed as cycles and microseconds (calibrated against the
100 MHz wall clock). Usage: python benchmarks/lenet_phase_trace.py [batch]"""
import os
import sys

os.environ.setdefault("MLT_LENET_VARIANT", "1")  # LENET_TRACE stamps exist only in the fused kernel
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.models.lenet import MLModel  # noqa: E402
from ml_trainer_amd.models.lenet_engine import LeNetStepEngine  # noqa: E402
from ml_trainer_amd.ops.optim import build_optimizer  # noqa: E402
from ml_trainer_amd.utils.flat import FlatParams  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = MLModel().to(dev)
flat = FlatParams(m.parameters())
opt = build_optimizer("sgd", m.parameters(), lr=1e-3, momentum=0.9, flat=flat)
eng = LeNetStepEngine(m, flat, max_batch=B, optimizer=opt)
N = 4096
data = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8)
targets = torch.randint(0, 10, (N,))
eng.set_dataset(data, targets, batch_size=B)
eng.start_epoch(torch.randperm(N))
eng.train_steps(B, 20, use_graph=False)
C = eng.C
names = ["load+chain", "augment", "conv1", "conv2", "fc+CE+fc-dgrad", "unpool2", "conv2-dgrad"]
rows = []
for rep in range(5):
    eng.eng.run(C.LENET_FWD | C.LENET_CE | C.LENET_BWD | C.LENET_TRACE, B)
    torch.cuda.synchronize()
    st = eng.bufs["slab1"][:20].view(torch.int64).cpu().tolist()
    rows.append(st)
st = rows[-1]
cyc = st[7] - st[0]
us = (st[9] - st[8]) / 100.0
ghz = cyc / (us * 1e3) if us > 0 else float("nan")
print(f"block 0 total: {cyc} cycles = {us:.2f} us ({ghz:.2f} GHz)")
for k, n in enumerate(names):
    d = [r[k + 1] - r[k] for r in rows]
    dm = sorted(d)[len(d) // 2]
    print(f"  {n:18s} {dm:8d} cycles  {dm / ghz / 1e3:7.2f} us")
