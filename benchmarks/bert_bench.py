"""BERT classifier training-step benchmark (BASELINE.json configs 4/5: BERT-base
seq 512 bf16; "large" fp8) on one GPU, native kernels vs a PyTorch-eager bf16
baseline of the same model (torch.autocast + SDPA + hipBLASLt) for comparison.

    python benchmarks/bert_bench.py --model bert-base --batch 16 --seq 512 --steps 10
    python benchmarks/bert_bench.py --impl torch      # eager PyTorch baseline

Prints one JSON line per run (samples/s, tokens/s, ms/step, model TFLOP/s).
Synthetic token ids, random-init weights (no network).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def run(args):
    from ml_trainer_amd.models.bert import BertClassifier, bert_config
    from ml_trainer_amd.ops.optim import FusedAdamW
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = bert_config(args.model, **({"layers": args.layers} if args.layers else {}))
    m = BertClassifier(cfg).to(dev)
    if args.impl == "native":
        opt = FusedAdamW(m.parameters(), lr=1e-4, weight_decay=0.01)
        fwd = m
    else:
        opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=0.01, fused=True)
        fwd = m.forward_torch_bf16
    ids = torch.randint(5, cfg.vocab_size, (args.batch, args.seq), device=dev)
    y = torch.randint(0, cfg.num_labels, (args.batch,), device=dev)

    def step():
        opt.zero_grad(set_to_none=False)
        loss = F.cross_entropy(fwd(ids), y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    tokens = args.batch * args.seq
    flops = m.flops_per_token(args.seq) * tokens
    rec = {"bench": "bert_train_step", "impl": args.impl, "model": args.model, "layers": cfg.layers,
           "batch": args.batch, "seq": args.seq, "ms_per_step": dt * 1e3, "samples_per_s": args.batch / dt,
           "tokens_per_s": tokens / dt, "model_tflops": flops / dt / 1e12, "loss": float(loss.detach()),
           "peak_mem_gb": torch.cuda.max_memory_allocated() / 2 ** 30}
    print(json.dumps(rec), flush=True)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert-base")
    ap.add_argument("--layers", type=int, default=0)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--impl", choices=["native", "torch", "both"], default="both")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    recs = []
    for impl in (["native", "torch"] if args.impl == "both" else [args.impl]):
        args.impl = impl
        recs.append(run(args))
    if args.out:
        with open(args.out, "a") as f:
            for r in recs:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
