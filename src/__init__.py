"""Reference-compatible import surface (``src.trainer``, ``src.model``,
``src.dataloader``, ``src.utils.utils``, ``src.utils.functions``), used by the
reference's notebooks and main.py. The implementation lives in
the ``ml_trainer_amd`` package."""
