"""Model registry.

BASELINE.json configs (the reference itself has no config system; decision
recorded in SURVEY.md §7.1 and README):

* ``tiny``      -- LeNet at reduced width (CPU / gloo plumbing config)
* ``default``   -- the reference LeNet-5 (``src/model.py``), headline benchmark
* ``bert-base`` -- 12-layer, d=768, 12-head encoder classifier (seq 512, bf16)
* ``large``     -- 24-layer, d=1024, 16-head encoder classifier with fp8 GEMMs
"""
from __future__ import annotations

from ml_trainer_amd.models.lenet import MLModel


def build_model(name: str = "default", **kw):
    name = name.lower()
    if name in ("default", "tiny", "lenet"):
        return MLModel("default" if name == "lenet" else name)
    if name in ("bert-base", "bert_base", "bert", "large", "bert-large", "bert-tiny"):
        from ml_trainer_amd.models.bert import BertClassifier, bert_config
        return BertClassifier(bert_config(name, **kw))
    raise ValueError(f"unknown model {name!r}")


__all__ = ["MLModel", "build_model"]
