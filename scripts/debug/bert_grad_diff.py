"""Per-parameter gradient comparison: native BERT-tiny vs fp32 reference."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch, torch.nn.functional as F
from ml_trainer_amd.models.bert import BertClassifier, bert_config
dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = BertClassifier(bert_config("bert-tiny")).to(dev)
ids = torch.randint(5, 1000, (2, 128), device=dev)
for use_mask in (False, True):
    mask = torch.ones(2, 128, dtype=torch.long, device=dev)
    if use_mask:
        mask[1, 100:] = 0
    y = torch.tensor([0, 1], device=dev)
    m.zero_grad()
    out = m(ids, mask)
    F.cross_entropy(out, y).backward()
    gn = {n: p.grad.clone() for n, p in m.named_parameters()}
    m.zero_grad()
    ref = m.forward_reference(ids, mask)
    F.cross_entropy(ref, y).backward()
    print("mask", use_mask, "logits", out.tolist(), ref.tolist())
    for n, p in m.named_parameters():
        r = p.grad
        rel = ((gn[n] - r).norm() / (r.norm() + 1e-12)).item()
        print(f"  {n:45s} rel_l2 {rel:.4f} max_err {(gn[n]-r).abs().max().item():.3e} ref_max {r.abs().max().item():.3e}")
    gp = gn["position_embeddings.weight"][:128]; rp = m.position_embeddings.weight.grad[:128]
    e = (gp - rp).abs().amax(1)
    print("  pos err by position (top 8):", [(int(i), round(float(e[i]), 5), round(float(rp[i].abs().max()), 5)) for i in e.topk(8).indices])
