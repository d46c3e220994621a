"""BERT encoder classifier -- BASELINE.json config 4 ("BERT-base classifier via
src/model.py, seq_len=512 bf16 DDP=8") and config 5 ("large config fp8").

Not part of the reference (its only model is the LeNet of src/model.py); the
model-config decision is recorded in SURVEY.md §7.1 and the README:

* ``bert-base``  12 layers, hidden 768, 12 heads, FFN 3072, vocab 30522, 512 positions
* ``large``      24 layers, hidden 1024, 16 heads, FFN 4096 (fp8 GEMMs, ops/fp8.py)
* ``bert-tiny``  2 layers, hidden 256, 4 heads, FFN 1024 (tests / CPU plumbing)

Post-LN BERT: embeddings(word+pos+type) -> LN -> N x [attention block -> LN -> FFN
block -> LN] -> pooler tanh(W h_CLS) -> classifier. On the GPU every heavy op runs
on the native kernels (ops/transformer.py: MFMA GEMMs with fused epilogues,
flash attention, LayerNorm, embedding gather/scatter, and the classifier head: pooler
GEMM with a tanh epilogue + the num_labels-wide classifier layer of head.hip) with fp32
master weights and bf16 activations. On CPU the
same math runs in plain torch (and serves as the numerics oracle in tests).
Dropout is 0 (deterministic training; the benchmark measures the compute path).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, replace
from typing import Optional

import torch
import torch.nn.functional as F
from torch import nn


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_position: int = 512
    type_vocab: int = 2
    num_labels: int = 2
    ln_eps: float = 1e-12
    init_std: float = 0.02
    fp8: bool = False
    pad_id: Optional[int] = None  # when set, key lengths are derived from trailing pad tokens


_PRESETS = {
    "bert-base": BertConfig(),
    "bert": BertConfig(),
    "bert_base": BertConfig(),
    "large": BertConfig(hidden=1024, layers=24, heads=16, intermediate=4096, fp8=True),
    "bert-large": BertConfig(hidden=1024, layers=24, heads=16, intermediate=4096),
    "bert-tiny": BertConfig(vocab_size=1000, hidden=256, layers=2, heads=4, intermediate=1024, max_position=128),
}


def bert_config(name: str = "bert-base", **overrides) -> BertConfig:
    cfg = _PRESETS[name.lower()]
    return replace(cfg, **overrides) if overrides else cfg


class BertLayer(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        h = c.hidden
        self.c = c
        self.qkv = nn.Linear(h, 3 * h)
        self.out = nn.Linear(h, h)
        self.ln1 = nn.LayerNorm(h, eps=c.ln_eps)
        self.ffn1 = nn.Linear(h, c.intermediate)
        self.ffn2 = nn.Linear(c.intermediate, h)
        self.ln2 = nn.LayerNorm(h, eps=c.ln_eps)

    def forward_native(self, x, lens, B, S):
        from ml_trainer_amd.ops import transformer as T
        if self.c.fp8:
            from ml_trainer_amd.ops.fp8 import FP8 as impl
        else:
            impl = T.BF16
        x = T.attention_ln_block(x, self.qkv.weight, self.qkv.bias, self.out.weight, self.out.bias, self.ln1.weight,
                                 self.ln1.bias, lens, B, S, self.c.heads, self.c.ln_eps, impl)
        return T.ffn_ln_block(x, self.ffn1.weight, self.ffn1.bias, self.ffn2.weight, self.ffn2.bias, self.ln2.weight,
                              self.ln2.bias, self.c.ln_eps, impl)

    def forward_reference(self, x, mask, B, S):
        """fp32 torch reference. x [B*S, h]; mask [B, S] bool (True = valid key)."""
        c = self.c
        H, dh = c.heads, c.hidden // c.heads
        qkv = self.qkv(x).view(B, S, 3, H, dh).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0], qkv[1], qkv[2]
        s = (q @ k.transpose(-1, -2)) / math.sqrt(dh)
        if mask is not None:
            s = s.masked_fill(~mask[:, None, None, :], float("-inf"))
        ctx = (s.softmax(-1) @ v).permute(0, 2, 1, 3).reshape(B * S, c.hidden)
        x = self.ln1(self.out(ctx) + x)
        f = self.ffn2(F.gelu(self.ffn1(x)))
        return self.ln2(f + x)


class BertClassifier(nn.Module):
    def __init__(self, c: Optional[BertConfig] = None):
        super().__init__()
        c = c or BertConfig()
        if c.hidden % c.heads or c.hidden // c.heads != 64:
            raise ValueError("the native attention kernel needs head dim 64")
        self.config = c
        self.word_embeddings = nn.Embedding(c.vocab_size, c.hidden)
        self.position_embeddings = nn.Embedding(c.max_position, c.hidden)
        self.token_type_embeddings = nn.Embedding(c.type_vocab, c.hidden)
        self.emb_ln = nn.LayerNorm(c.hidden, eps=c.ln_eps)
        self.layers = nn.ModuleList([BertLayer(c) for _ in range(c.layers)])
        self.pooler = nn.Linear(c.hidden, c.hidden)
        self.classifier = nn.Linear(c.hidden, c.num_labels)
        self.apply(self._init)

    def _init(self, m):
        std = self.config.init_std
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, std=std)
            nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, std=std)
        elif isinstance(m, nn.LayerNorm):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)

    def _lengths(self, input_ids, attention_mask):
        B, S = input_ids.shape
        if attention_mask is not None:
            return attention_mask.to(torch.int32).sum(1).clamp(min=1).to(torch.int32)
        if self.config.pad_id is not None:
            return (input_ids != self.config.pad_id).to(torch.int32).sum(1).clamp(min=1).to(torch.int32)
        return None

    def forward(self, input_ids, attention_mask=None, token_type_ids=None):
        if isinstance(input_ids, (tuple, list)):
            input_ids, attention_mask = input_ids[0], input_ids[1] if len(input_ids) > 1 else None
        B, S = input_ids.shape
        lens = self._lengths(input_ids, attention_mask)
        if input_ids.is_cuda:
            from ml_trainer_amd.ops import transformer as T
            if self.config.fp8 and torch.is_grad_enabled():
                from ml_trainer_amd.ops.fp8 import context
                context(input_ids.device).update()  # delayed scaling: fold last step's amaxes
            x = T.embeddings(input_ids, token_type_ids, self.word_embeddings.weight, self.position_embeddings.weight,
                             self.token_type_embeddings.weight, S)
            x = T.layer_norm(x, self.emb_ln.weight, self.emb_ln.bias, self.config.ln_eps)
            for layer in self.layers:
                x = layer.forward_native(x, lens, B, S)
            cls = x.view(B, S, -1)[:, 0]  # strided row view: the pooler GEMM reads it in place
            if cls.shape[1] % 8 == 0 and self.pooler.weight.shape[0] % 8 == 0:
                return T.classifier_head(cls, self.pooler.weight, self.pooler.bias, self.classifier.weight,
                                         self.classifier.bias)
            cls = cls.float()
        else:
            cls = self.forward_reference_hidden(input_ids, lens, token_type_ids)
        pooled = torch.tanh(self.pooler(cls))
        return self.classifier(pooled)

    def forward_reference_hidden(self, input_ids, lens=None, token_type_ids=None):
        B, S = input_ids.shape
        pos = torch.arange(S, device=input_ids.device)
        tt = token_type_ids if token_type_ids is not None else torch.zeros_like(input_ids)
        x = self.word_embeddings(input_ids) + self.position_embeddings(pos)[None] + self.token_type_embeddings(tt)
        x = self.emb_ln(x).view(B * S, -1)
        mask = None
        if lens is not None:
            mask = torch.arange(S, device=input_ids.device)[None, :] < lens.to(input_ids.device)[:, None]
        for layer in self.layers:
            x = layer.forward_reference(x, mask, B, S)
        return x.view(B, S, -1)[:, 0]

    def forward_reference(self, input_ids, attention_mask=None, token_type_ids=None):
        lens = self._lengths(input_ids, attention_mask)
        cls = self.forward_reference_hidden(input_ids, lens, token_type_ids)
        return self.classifier(torch.tanh(self.pooler(cls)))

    def forward_torch_bf16(self, input_ids, attention_mask=None, token_type_ids=None):
        """PyTorch-eager bf16 path on the same weights (torch.autocast + SDPA + hipBLASLt): the
        baseline the native kernels are benchmarked and error-budgeted against."""
        c = self.config
        B, S = input_ids.shape
        lens = self._lengths(input_ids, attention_mask)
        mask = None
        if lens is not None:
            mask = (torch.arange(S, device=input_ids.device)[None, :] < lens[:, None])[:, None, None, :]
        with torch.autocast(input_ids.device.type, dtype=torch.bfloat16):
            pos = torch.arange(S, device=input_ids.device)
            tt = token_type_ids if token_type_ids is not None else torch.zeros_like(input_ids)
            x = self.word_embeddings(input_ids) + self.position_embeddings(pos)[None] + self.token_type_embeddings(tt)
            x = self.emb_ln(x)
            for L in self.layers:
                qkv = L.qkv(x).view(B, S, 3, c.heads, 64).permute(2, 0, 3, 1, 4)
                ctx = F.scaled_dot_product_attention(qkv[0], qkv[1], qkv[2], attn_mask=mask)
                x = L.ln1(L.out(ctx.transpose(1, 2).reshape(B, S, -1)) + x)
                x = L.ln2(L.ffn2(F.gelu(L.ffn1(x))) + x)
            return self.classifier(torch.tanh(self.pooler(x[:, 0].float())))

    def num_parameters(self) -> int:
        return sum(p.numel() for p in self.parameters())

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs per token (fwd + bwd = 3x fwd) of the encoder stack."""
        c = self.config
        h, f = c.hidden, c.intermediate
        per_layer = 2 * (3 * h * h + h * h + 2 * h * f) + 2 * 2 * seq_len * h  # linears + QK^T / PV
        return 3.0 * c.layers * per_layer
