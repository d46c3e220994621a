"""Train the reference LeNet for a few Trainer epochs on a fixed synthetic set and save the
weights (run once per kernel path: MLT_LENET_FUSED=0/1, engine on/off), then diff the saves:
  python scripts/debug/engine_drift.py run <tag> <use_engine 0|1>
  python scripts/debug/engine_drift.py diff <tag> <tag> ..."""
import os, sys; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "gpurun_out")

if sys.argv[1] == "run":
    import tempfile
    from ml_trainer_amd.data.cifar10 import SyntheticCIFAR10
    from ml_trainer_amd.models.lenet import MLModel
    from ml_trainer_amd.trainer import Trainer
    from ml_trainer_amd.utils.functions import custom_pre_process_function
    tf = custom_pre_process_function()
    tr = SyntheticCIFAR10(640, train=True, transform=tf, seed=0, learnable=True)
    va = SyntheticCIFAR10(200, train=False, transform=tf, seed=0, learnable=True)
    torch.manual_seed(0)
    m = MLModel()
    t = Trainer(m, datasets=(tr, va), epochs=1, batch_size=64, model_dir=tempfile.mkdtemp(), lr=0.01,
                optimizer="sgd", options={"progress": False, "use_engine": sys.argv[3] == "1"})
    t._train_one_epoch(1)
    torch.cuda.synchronize()
    w_train = [p.detach().clone() for p in t.model.parameters()]
    torch.save({k: v.detach().float().cpu() for k, v in t.model.state_dict().items()},
               os.path.join(OUT, f"drift_{sys.argv[2]}.pt"))
    t._validate_one_epoch()
    torch.cuda.synchronize()
    dv = max((a - p.detach()).abs().max().item() for a, p in zip(w_train, t.model.parameters()))
    print(sys.argv[2], "train", t.train_losses, t.train_metrics, "val", t.val_losses, t.val_metrics,
          "weights moved by validation:", dv)
else:
    tags = sys.argv[2:]
    sd = {g: torch.load(os.path.join(OUT, f"drift_{g}.pt"), weights_only=True) for g in tags}
    for i, a in enumerate(tags):
        for b in tags[i + 1:]:
            d = max((sd[a][k] - sd[b][k]).abs().max().item() for k in sd[a])
            print(f"{a:12s} vs {b:12s} max|dW| {d:.3e}")
