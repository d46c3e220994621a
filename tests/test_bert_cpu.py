"""BERT classifier plumbing on CPU (the fp32 torch path that is also the GPU numerics oracle)."""
import torch
import torch.nn.functional as F

from ml_trainer_amd.data.text import SyntheticTextClassification
from ml_trainer_amd.models import build_model
from ml_trainer_amd.models.bert import BertClassifier, bert_config


def test_configs():
    base = bert_config("bert-base")
    assert (base.hidden, base.layers, base.heads, base.intermediate) == (768, 12, 12, 3072)
    large = bert_config("large")
    assert (large.hidden, large.layers, large.heads, large.fp8) == (1024, 24, 16, True)
    m = BertClassifier(bert_config("bert-base", layers=1))
    # embeddings + 1 layer + pooler + classifier
    h = 768
    expect = (30522 + 512 + 2) * h + 2 * h + (4 * h * h + 4 * h + 2 * h * 3072 + 3072 + h + 4 * h) + h * h + h + 2 * h + 2
    assert m.num_parameters() == expect


def test_forward_backward_and_mask():
    torch.manual_seed(0)
    m = build_model("bert-tiny")
    ids = torch.randint(5, 1000, (2, 64))
    out = m(ids)
    assert out.shape == (2, 2)
    # padding keys must not change the valid positions' result
    mask = torch.ones(2, 64, dtype=torch.long)
    mask[:, 40:] = 0
    a = m(ids, mask)
    ids2 = ids.clone()
    ids2[:, 40:] = 1
    b = m(ids2, mask)
    torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)
    F.cross_entropy(a, torch.tensor([0, 1])).backward()
    assert all(p.grad is not None for p in m.parameters())


def test_tuple_input_and_dataset():
    ds = SyntheticTextClassification(16, seq_len=32, vocab_size=1000, learnable=True, seed=1)
    x, y = ds[3]
    assert x.shape == (32,) and x.dtype == torch.int64 and y in (0, 1)
    pos = ds.targets == 1
    assert (ds.ids[pos] == 3).any(1).all()
    m = build_model("bert-tiny")
    ids = ds.ids[:4]
    torch.testing.assert_close(m((ids, torch.ones_like(ids))), m(ids))


def test_bert_trains_cpu():
    torch.manual_seed(0)
    m = BertClassifier(bert_config("bert-tiny", layers=1, hidden=128, heads=2, intermediate=256))
    ds = SyntheticTextClassification(16, seq_len=16, vocab_size=1000, learnable=True, seed=2)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    first = None
    for _ in range(40):
        opt.zero_grad()
        loss = F.cross_entropy(m(ds.ids), ds.targets)
        loss.backward()
        opt.step()
        first = first or loss.item()
    assert loss.item() < 0.5 * first
