"""Debug: BERT-tiny DDP gradients after ONE backward with the native size-1 communicator vs no
communication, per bucket; then the same with a device synchronise after every bucket launch."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ml_trainer_amd.models.bert import BertClassifier, bert_config  # noqa: E402
from ml_trainer_amd.ops._ext import require_native  # noqa: E402
from ml_trainer_amd.parallel.ddp import DistributedDataParallel  # noqa: E402

dev = torch.device("cuda", 0)
C = require_native()
g = torch.Generator().manual_seed(3)
ids = torch.randint(5, 1000, (2, 128), generator=g).to(dev)
y = torch.randint(0, 2, (2,), generator=g).to(dev)


def run(native, sync=False):
    torch.manual_seed(0)
    m = BertClassifier(bert_config("bert-tiny")).to(dev)
    comm = C.Communicator(C.Communicator.unique_id(), 1, 0, dev.index) if native else False
    ddp = DistributedDataParallel(m, bucket_cap_mb=1.0, first_bucket_mb=0.5, comm=comm)
    if sync:
        orig = ddp._reduce_bucket

        def wrapped(bi, async_op=True):
            torch.cuda.synchronize()
            r = orig(bi, async_op)
            torch.cuda.synchronize()
            return r
        ddp._reduce_bucket = wrapped
    ddp.flat.grad.zero_()
    F.cross_entropy(ddp(ids), y).backward()
    torch.cuda.synchronize()
    return ddp, ddp.flat.grad.clone()


d0, g0 = run(False)
for native, sync in ((True, False), (True, True)):
    d1, g1 = run(native, sync)
    print(f"native={native} sync={sync}: equal={torch.equal(g0, g1)} max|diff|={(g0 - g1).abs().max().item():.3e}")
    for bi, (s, e) in enumerate(d1._buckets):
        dd = (g0[s:e] - g1[s:e]).abs().max().item()
        if dd > 0:
            names = [n for n, p in d1.module.named_parameters()
                     if s <= d1.flat.segment(p)[0] < e]
            print(f"  bucket {bi} [{s},{e}) max|diff| {dd:.3e} params {names[:6]}")
