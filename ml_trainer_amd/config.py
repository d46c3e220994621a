"""Trainer configuration.

Two layers, mirroring the reference:

* the reference's ``**config`` whitelist (``src/trainer.py:26-41``) --
  :data:`ALLOWED_KWARGS` / :data:`CONFIG_DEFAULTS` -- unknown keys raise
  ``TypeError("Keyword argument not understood:", key)`` exactly like the
  reference's ``validate_kwargs``;
* :class:`TrainerOptions` -- MI355X-specific knobs that the reference does not
  have (fused engine, hipGraph, bucket sizes, precision, checkpoint/resume,
  watchdog). They are passed as ``Trainer(..., options=TrainerOptions(...))``
  (or a dict), so the reference's kwarg contract stays byte-for-byte intact.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Any, Dict, Optional

ALLOWED_KWARGS = frozenset({"seed", "scheduler", "optimizer", "momentum", "weight_decay", "lr", "criterion",
                            "metric", "pred_function", "model_dir", "backend"})

# defaults apply only when the key is ABSENT (an explicit None is kept: metric=None disables metrics)
CONFIG_DEFAULTS: Dict[str, Any] = {
    "scheduler": None,
    "optimizer": "sgd",
    "momentum": 0.9,
    "weight_decay": 0.0,
    "lr": 0.001,
    "criterion": "cross_entropy",
    "metric": "accuracy",
    "pred_function": "softmax",
    "model_dir": "model_output",
    "backend": "smddp",
    "seed": 32,
}

SCHEDULERS = ("CosineAnnealingWarmRestarts", "ReduceLROnPlateau", "StepLR")


@dataclass
class TrainerOptions:
    # --- execution -----------------------------------------------------------------
    use_engine: Optional[bool] = None     # fused native step engine (None = auto when eligible)
    use_graph: bool = True                # capture the engine step into hipGraphs
    steps_per_graph: int = 16             # engine steps per captured graph
    device_data: Optional[bool] = None    # upload uint8 datasets to HBM + GPU augmentation (auto)
    per_device_batch: bool = False        # True: batch_size is per GPU (weak scaling); reference divides by W
    amp: Optional[str] = None             # None | "bf16": autocast compute dtype for generic models
    precision: str = "fp32"               # fused LeNet engine: "fp32" (reference dtype) | "bf16" (MFMA step,
                                          # fp32 masters; BASELINE.json configs 2/3)
    grad_clip: Optional[float] = None     # clip-by-global-norm (fused kernel)
    grad_accum_steps: int = 1             # micro-batches per optimizer step (DDP no_sync between)
    # --- distributed ----------------------------------------------------------------
    bucket_cap_mb: float = 32.0
    first_bucket_mb: float = 4.0
    ddp_mode: str = "overlap"             # "overlap" | "manual" (reference _average_gradients semantics)
    zero_stage: int = 0                   # 1: ZeRO-1 (reduce-scatter grads, sharded optimizer state, all-gather)
    global_metrics: bool = False          # all-reduce epoch loss/metric across ranks (reference: rank-local)
    dist_timeout_s: float = 1800.0
    # --- data -------------------------------------------------------------------------
    num_workers: int = 0
    pin_memory: bool = True
    prefetch_depth: int = 2
    # --- fault tolerance / checkpoints ---------------------------------------------------
    resume: bool = False                  # reload model.pth + trainer_state.pt from model_dir
    save_trainer_state: bool = True       # write trainer_state.pt (optimizer/scheduler/epoch/RNG) per epoch
    async_checkpoint: bool = False        # model.pth from a pinned-host snapshot, written by a background
                                          # thread (utils/checkpoint.AsyncCheckpointer); fit() waits at the end
    watchdog_s: Optional[float] = None    # >0: abort if no step progress this long / a collective fails
                                          # (None: 600 s for multi-rank jobs, off otherwise; 0: off)
    fault_inject_step: int = -1           # testing: raise at this global step on rank fault_inject_rank
    fault_inject_rank: int = 0
    # --- observability -------------------------------------------------------------------
    progress: bool = True                 # tqdm bars
    log_interval: int = 0                 # >0: log running loss every N steps (one host sync each)
    metrics_jsonl: Optional[str] = None   # append per-epoch metrics/throughput records here
    profile_ranges: bool = False          # roctx ranges around phases (rocprofv3 --marker-trace)
    determinism_check: bool = False       # cross-rank parameter hash after every epoch

    @classmethod
    def from_any(cls, x) -> "TrainerOptions":
        if x is None:
            return cls()
        if isinstance(x, cls):
            return x
        if isinstance(x, dict):
            names = {f.name for f in dataclasses.fields(cls)}
            bad = set(x) - names
            if bad:
                raise TypeError("Unknown trainer option(s):", sorted(bad))
            return cls(**x)
        raise TypeError(f"options must be TrainerOptions or dict, not {type(x)}")
