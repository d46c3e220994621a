"""Pinned-host prefetcher under a slow consumer, for `rocprofv3 --kernel-trace --memory-copy-trace`:
12 batches of 64 MB through a 3-deep ring (copy stream), each consumed by a chain of 2048^2 GEMMs on
the compute stream. `--summarize DIR` reads the trace CSVs and reports how much of every H2D copy
ran under a kernel (tests/test_lenet_native.py::test_pinned_prefetcher_overlaps_copy_and_compute
checks the wall-time side of the same pipeline)."""
import csv
import glob
import os
import sys


def summarize(d):
    kern = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            kern.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    copies = []
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "HOST_TO_DEVICE" in (r.get("Direction") or r.get("Operation") or ""):
                copies.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    kern.sort()
    copies.sort()
    lines = [f"kernels: {len(kern)}, host-to-device copies: {len(copies)}"]
    tot = ov = 0
    for a, b in copies:
        o = 0
        for s, e in kern:
            if e <= a or s >= b:
                continue
            o += min(b, e) - max(a, s)
        o = min(o, b - a)
        tot += b - a
        ov += o
        lines.append(f"copy {(b - a) / 1e3:9.1f} us, {100.0 * o / max(1, b - a):5.1f} % under kernels")
    lines.append(f"total: {tot / 1e3:.1f} us of copies, {100.0 * ov / max(1, tot):.1f} % overlapped by kernels")
    return "\n".join(lines)


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[1] == "--summarize":
    print(summarize(sys.argv[2]))
    sys.exit(0)

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
nbytes, d, n, reps = 64 << 20, 3, 12, 12
pf = C.PinnedPrefetcher(nbytes, d, 0)
bufs = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(d)]
for i in range(d):
    pf.slot(i).fill_(i + 1)
a = torch.randn(2048, 2048, device=dev)
sink = torch.zeros((), device=dev)


def compute(buf):
    sink.add_(buf[:1 << 20].float().sum())
    x = a
    for _ in range(reps):
        x = torch.mm(x, a).mul_(1e-3)
    sink.add_(x[0, 0])


def pipeline():
    for k in range(d - 1):
        pf.copy_to_device(k, bufs[k], nbytes)
    for k in range(n):
        j = k + d - 1
        if j < n:
            pf.wait(j % d)
            pf.copy_to_device(j % d, bufs[j % d], nbytes)
        pf.acquire(k % d)
        compute(bufs[k % d])
        pf.release(k % d)


for _ in range(2):
    pipeline()
torch.cuda.synchronize()
print("done", float(sink))
