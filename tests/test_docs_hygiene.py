"""Docs that describe the shipped step must match it (VERDICT r5 'What's weak' #6 / #9)."""
import glob
import os
import re

import ml_trainer_amd.models.lenet_engine as le
import ml_trainer_amd.trainer as tr

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_lenet_docstrings_say_two_launches():
    for mod in (tr, le):
        doc = mod.__doc__
        assert re.search(r"\btwo kernels per step\b", doc, re.I), mod.__name__
        assert not re.search(r"\bone kernel per step\b", doc, re.I), mod.__name__


def test_no_one_launch_step_left():
    """The one-launch step (measured slower, r5) is gone: no translation units, no engine switch."""
    kdir = os.path.join(REPO, "ml_trainer_amd", "csrc", "kernels")
    assert not glob.glob(os.path.join(kdir, "lenet_mfma_1l_*.hip"))
    src = open(os.path.join(REPO, "ml_trainer_amd", "csrc", "bindings.cpp")).read()
    assert "onelaunch" not in src and "MLT_LENET_ONELAUNCH" not in src
    assert not hasattr(le.LeNetStepEngine, "flush") and not hasattr(le.LeNetStepEngine, "sync_error")
