"""ml_trainer_amd/build.py incremental-build rules (CPU): an object is rebuilt when it is missing,
older than its source or a header, or was compiled with a different command line."""
import os
import time

from ml_trainer_amd import build


def _touch(path, t):
    with open(path, "a"):
        pass
    os.utime(path, (t, t))


def test_newer_rules(tmp_path):
    src, obj, hdr = tmp_path / "k.hip", tmp_path / "k.hip.o", tmp_path / "h.h"
    now = time.time()
    _touch(src, now - 100)
    _touch(hdr, now - 100)
    cmd = ["hipcc", "-c", str(src), "-o", str(obj), "-O3"]
    assert build._newer(str(src), str(obj), [str(hdr)], cmd)  # no object yet
    _touch(obj, now - 50)
    assert build._newer(str(src), str(obj), [str(hdr)], cmd)  # no command stamp yet
    (tmp_path / "k.hip.o.cmd").write_text(" ".join(cmd))
    assert not build._newer(str(src), str(obj), [str(hdr)], cmd)  # up to date
    assert build._newer(str(src), str(obj), [str(hdr)], cmd + ["-fno-slp-vectorize"])  # flags changed
    _touch(hdr, now)
    assert build._newer(str(src), str(obj), [str(hdr)], cmd)  # header newer than the object
    _touch(hdr, now - 100)
    _touch(src, now)
    assert build._newer(str(src), str(obj), [str(hdr)], cmd)  # source newer than the object


def test_file_flags_cover_the_measured_files():
    # the per-file flags measured in profiles/ab_*_r3.jsonl: no SLP packing beside MFMAs
    assert "-fno-slp-vectorize" in build.FILE_FLAGS["attention.hip"]
    assert "-fno-slp-vectorize" in build.FILE_FLAGS["lenet_mfma.hip"]
    assert "-amdgpu-sched-strategy=max-memory-clause" in build.FILE_FLAGS["lenet_mfma.hip"]
    assert "gemm_tile.hip" not in build.FILE_FLAGS  # measured slower there
