"""Per-phase timing of the bf16 per-sample LeNet kernel (lenet_mfma.hip, LENET_TRACE): block 0
stores s_memtime stamps at every phase boundary (each stamp adds a barrier, so the sum runs a
little over the untraced kernel). Needs a trace build (-DMLT_LENET_TRACE_BUILD=1: the stamps are
compiled out of the shipped kernel). Usage: python benchmarks/lenet_bf16_phases.py [batch] [--jsonl F]"""
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
from ml_trainer_amd.ops._ext import require_native  # noqa: E402
if not require_native().lenet_mfma_trace_build():
    sys.exit("lenet_bf16_phases.py needs a trace build of the extension: python -c \"from ml_trainer_amd.build "
             "import build; build(extra_flags={'lenet_mfma.hip': ['-DMLT_LENET_TRACE_BUILD=1']})\"")
torch.manual_seed(0)
m = MLModel().to(dev)
flat = FlatParams(m.parameters())
opt = build_optimizer("sgd", m.parameters(), lr=1e-3, momentum=0.9, flat=flat)
eng = LeNetStepEngine(m, flat, max_batch=B, optimizer=opt, precision="bf16")
trace = torch.zeros(4096, dtype=torch.float32, device=dev)  # (slots 1024+: per-wave stamps)
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
# stamp slots in kernel order (lenet_mfma.hip stamp(k)); a name per interval
idx = [0, 16, 17, 1, 2, 3, 18, 19, 4, 20, 21, 22, 5, 6, 7, 23, 24, 13]
names = ["P0 loads issued (+ctrl/meta scalar wait)", "P1 zero fill + raw image to LDS", "P1 augment -> xh/xc",
         "P2 conv1", "P3 conv2", "P4 fc1 fwd", "P4 fc2 fwd", "P4 fc3 fwd + softmax-CE", "P6 fc3 dgrad",
         "P7 fc2 dgrad", "-", "P8 fc1 dgrad + unpool", "P10 w2d + dflat/dh1 stores", "P11 conv2 dgrad/wgrad",
         "P13 conv1 wgrad MFMAs",
         "P13 partial sums + slab stores", "end of kernel"]
rows = []
for rep in range(9):
    trace.zero_()  # a stamp the kernel skips this step (e.g. 17: no augmentation on a prep hit) stays 0
    eng.eng.run(C.LENET_FWD | C.LENET_CE | C.LENET_BWD | C.LENET_TRACE, B)
    torch.cuda.synchronize()
    rows.append(trace.view(torch.int64).cpu().tolist())
# drop the stamps that did not run in every rep: their interval merges into the one before it
# (round 5 subtracted an unset stamp here and committed overflowed rows)
keep = [k for k, slot in enumerate(idx) if all(r[slot] != 0 for r in rows)]
assert keep and keep[0] == 0 and keep[-1] == len(idx) - 1, "phase trace: start / end stamps missing"
merged = []
for a, b in zip(keep, keep[1:]):
    merged.append((idx[a], idx[b], " + ".join(names[a:b]) + (" (stamp skipped)" if b - a > 1 else "")))
idx = [idx[k] for k in keep]
names = [n for _, _, n in merged]
st = rows[-1]
cyc = st[13] - st[0]
us = (st[15] - st[14]) / 100.0
ghz = cyc / (us * 1e3) if us > 0 else float("nan")
print(f"block 0 total: {cyc} cycles = {us:.2f} us ({ghz:.2f} GHz), batch {B}")
rec = {"batch": B, "total_cycles": cyc, "total_us": us, "ghz": round(ghz, 3), "phases_us": {}}
for k, n in enumerate(names):
    d = sorted(r[idx[k + 1]] - r[idx[k]] for r in rows)
    dm = d[len(d) // 2]
    rec["phases_us"][n] = round(dm / ghz / 1e3, 3)
    assert dm >= 0, (n, d)
    print(f"  {n:28s} {dm:8d} cycles  {dm / ghz / 1e3:7.2f} us")
# per-wave work-done stamps (slots 1024 + 16 k + w): cycles after the phase's opening stamp, median over reps
wph = [("P2 conv1", 1, 0), ("P3 conv2 / fc3-fc2 dgrad fetch", 2, 1), ("P8 fc1 dgrad + unpool", 22, 2),
       ("P11 conv2 dgrad/wgrad", 6, 3), ("P11 conv2 dgrad MFMAs (waves 0-6)", 6, 5), ("P13 conv1 wgrad", 7, 4)]
rec["wave_done_cycles"] = {}
for name, open_slot, k in wph:
    per = []
    for wv in range(16):
        d = sorted(r[1024 + 16 * k + wv] - r[open_slot] for r in rows if r[1024 + 16 * k + wv] and r[open_slot])
        per.append(d[len(d) // 2] if d else None)
    rec["wave_done_cycles"][name] = per
    print(f"  {name:32s} wave done (cycles after phase start): {per}")
# per-block wall clock (100 MHz): KS blocks (slots 600 + 2b), KW blocks (1200 + 5 blk: start, 4 wave ends;
# the B prep blocks follow the reduction blocks)
tr = rows[-1]
ks = [(tr[600 + 2 * i], tr[601 + 2 * i]) for i in range(min(B, 200))]
C = eng.C
nkw = C.lenet_mfma_kw_blocks(m.cfg_id)
kw = [(tr[1200 + 5 * i], max(tr[1201 + 5 * i:1205 + 5 * i])) for i in range(min(nkw, 160))]
kwp = [(tr[1200 + 5 * i], max(tr[1201 + 5 * i:1205 + 5 * i])) for i in range(nkw, min(nkw + B, 160))]
t0 = min(a for a, _ in ks)
ks_end = max(e for _, e in ks)
print(f"KS blocks: start spread {(max(a for a, _ in ks) - t0) * 10} ns, block time "
      f"{min(e - a for a, e in ks) * 10}..{max(e - a for a, e in ks) * 10} ns, last end at {(ks_end - t0) * 10} ns")
rec["ks_block_ns"] = [[(a - t0) * 10, (e - t0) * 10] for a, e in ks]
if kw:
    k0 = min(a for a, _ in kw)
    print(f"KW blocks ({nkw}): first start {(k0 - ks_end) * 10} ns after the last KS end; start spread "
          f"{(max(a for a, _ in kw) - k0) * 10} ns; last end {(max(e for _, e in kw) - k0) * 10} ns after its first start")
    slow = sorted(range(len(kw)), key=lambda i: kw[i][1])[-5:]
    print("  latest-ending KW blocks:", [(i, (kw[i][0] - k0) * 10, (kw[i][1] - k0) * 10) for i in slow])
    rec["kw_block_ns"] = [[(a - k0) * 10, (e - k0) * 10] for a, e in kw]
    if kwp and all(a and e for a, e in kwp):
        print(f"  prep blocks ({len(kwp)}): start {(min(a for a, _ in kwp) - k0) * 10}..{(max(a for a, _ in kwp) - k0) * 10} ns, "
              f"end {(min(e for _, e in kwp) - k0) * 10}..{(max(e for _, e in kwp) - k0) * 10} ns after the first KW start")
        rec["kw_prep_block_ns"] = [[(a - k0) * 10, (e - k0) * 10] for a, e in kwp]
if out:
    with open(out, "a") as f:
        f.write(json.dumps(rec) + "\n")
