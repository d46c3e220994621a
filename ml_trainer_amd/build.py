"""In-tree build of the native extension ``ml_trainer_amd._C`` for gfx950.

Why a hand-rolled build instead of ``torch.utils.cpp_extension``: the torch
extension builder runs hipify over ``.hip``/``.cu`` sources; this framework is
written for CDNA4 directly, so there is nothing to translate. The build is:

* every ``csrc/kernels/*.hip`` file -> ``hipcc -c --offload-arch=gfx950 -O3``
  (pure HIP, no torch headers: these recompile in seconds);
* ``csrc/bindings.cpp`` and ``csrc/runtime/*.cpp`` (torch/pybind11 glue, the
  graph executor, the pinned-host prefetcher, the RCCL communicator) ->
  ``hipcc -c`` host-only objects with the torch include paths;
* link with ``g++ -shared`` against *torch's own* ``libamdhip64``/``librccl``
  (so exactly one HIP runtime is loaded per process) into
  ``ml_trainer_amd/_C<ext_suffix>.so`` - in-tree, so it ships with the repo
  snapshot to the GPU box and is visible to the round-end loaded-.so audit.

Objects are cached under ``build/`` and rebuilt only when a source or any
header under ``csrc/include`` is newer.

Usage: ``python -m ml_trainer_amd.build [-j N] [--force] [--debug]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig
import time

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD_DIR = os.path.join(REPO_DIR, "build", "mlt")
ARCH = os.environ.get("MLT_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG_DIR, "_C" + suffix)


def _torch_paths():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(tdir, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _deps(src: str, seen=None):
    """The in-tree files ``src`` includes, transitively (``#include "..."`` resolved against its own
    directory and csrc/include): a kernel file rebuilds only when something it includes changed."""
    import re
    seen = set() if seen is None else seen
    try:
        text = open(src).read()
    except OSError:
        return seen
    for name in re.findall(r'^\s*#\s*include\s+"([^"]+)"', text, re.M):
        for d in (os.path.dirname(src), os.path.join(CSRC, "include")):
            f = os.path.join(d, name)
            if os.path.exists(f):
                if f not in seen:
                    seen.add(f)
                    _deps(f, seen)
                break
    return seen


def _newer(src: str, obj: str, deps, cmd=None) -> bool:
    """Rebuild when the object is missing, older than its source or a header, or was compiled with
    a different command line (``<obj>.cmd`` records the last one: a flag change rebuilds)."""
    if not os.path.exists(obj):
        return True
    if cmd is not None:
        try:
            with open(obj + ".cmd") as f:
                if f.read() != " ".join(cmd):
                    return True
        except OSError:
            return True
    t = os.path.getmtime(obj)
    if os.path.getmtime(src) > t:
        return True
    return any(os.path.getmtime(h) > t for h in deps)


def _run(cmd):
    t0 = time.time()
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if p.returncode != 0:
        raise RuntimeError("build step failed:\n" + " ".join(cmd) + "\n" + p.stdout)
    return time.time() - t0, p.stdout


# per-file code-generation flags. attention.hip: MFMA accumulators in arch VGPRs (gfx950's
# register file is unified). By default hipcc puts them in AGPRs and copies every S^T tile to
# VGPRs for the softmax VALU work and every O tile back and forth for the rescale (~80
# v_accvgpr_read/write per 64-key block of the forward); the VGPR form removes those copies.
# -fno-slp-vectorize: hipcc's SLP pass packs adjacent f32 adds / muls of the softmax VALU work
# into v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32, which cost more than two scalar ops when they
# sit between MFMAs (MI355X_MICROARCH.md, "price of one filler beside MFMAs").
# lenet_mfma.hip: the max-memory-clause machine scheduler (loads grouped into clauses issued ahead
# of their uses) measured 1-2 % faster on the latency-chain per-sample step than the default,
# max-ilp and iterative-ilp strategies (profiles/ab_lenet_sched_r3.jsonl).
# lenet_mfma.hip also preloads the leading scalar kernel arguments into SGPRs (the per-sample
# kernel's first-load pointers: no s_load round trip of the kernarg segment before its first loads).
FILE_FLAGS = {"attention.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form", "-fno-slp-vectorize"],
              "lenet_mfma.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-sched-strategy=max-memory-clause",
                                 "-mllvm", "-amdgpu-kernarg-preload-count=12"]}
# translation units split off a kernel file for parallel compilation share its flags ({prefix: file})
FILE_ALIASES = {"lenet_mfma_dp": "lenet_mfma.hip"}  # (lenet_mfma_dp.hip, lenet_mfma_dpw<W>.hip)


def _flag_key(name: str) -> str:
    for prefix, key in FILE_ALIASES.items():
        if name.startswith(prefix):
            return key
    return name


# kernels whose accumulators live in AGPRs owned by inline asm (gemm_w4.hip): the build also emits
# their device asm and fails on any compiler-generated v_accvgpr_write (scripts/check_w4_agpr.py)
AGPR_GUARDED = {"gemm_w4.hip"}


def build(jobs: int = 8, force: bool = False, debug: bool = False, verbose: bool = True, extra_flags=None,
          out_path=None) -> str:
    """extra_flags: {kernel file name: [flags]} on top of FILE_FLAGS; out_path: link elsewhere (A/B
    variants of one kernel file; the objects are rebuilt for the in-tree flags on the next plain build)."""
    import pybind11
    os.makedirs(BUILD_DIR, exist_ok=True)
    tinc, tlib, abi = _torch_paths()
    pyinc = sysconfig.get_paths()["include"]
    common = ["-std=c++17", "-fPIC", f"-I{os.path.join(CSRC, 'include')}", "-D__HIP_PLATFORM_AMD__=1",
              f"-D_GLIBCXX_USE_CXX11_ABI={abi}"]
    opt = ["-O0", "-g"] if debug else ["-O3"]
    if debug:
        common.append("-DMLT_DEBUG=1")

    kernel_srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    host_srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")) +
                       glob.glob(os.path.join(CSRC, "comm", "*.cpp")) +
                       [os.path.join(CSRC, "bindings.cpp")])
    jobs_list = []
    objs = []
    asm_checks = []
    for s in kernel_srcs:
        o = os.path.join(BUILD_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        cmd = [HIPCC, "-c", s, "-o", o, f"--offload-arch={ARCH}", *opt, *common, "-munsafe-fp-atomics",
               "-Wno-unused-result", *FILE_FLAGS.get(_flag_key(os.path.basename(s)), []),
               *(extra_flags or {}).get(_flag_key(os.path.basename(s)), [])]
        if force or _newer(s, o, _deps(s), cmd):
            jobs_list.append(cmd)
            if os.path.basename(s) in AGPR_GUARDED:  # + its device asm for the AGPR-spill guard
                asm_checks.append(os.path.join(BUILD_DIR, os.path.basename(s) + ".s"))
                jobs_list.append([HIPCC, "-S", s, "--cuda-device-only", "-o", asm_checks[-1], f"--offload-arch={ARCH}",
                                  *opt, *common, *FILE_FLAGS.get(os.path.basename(s), []),
                                  *(extra_flags or {}).get(os.path.basename(s), [])])
    for s in host_srcs:
        o = os.path.join(BUILD_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        cmd = [HIPCC, "-c", s, "-o", o, *opt, *common, "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
               f"-I{pyinc}", f"-I{pybind11.get_include()}", *[f"-isystem{i}" for i in tinc], "-I/opt/rocm/include",
               "-Wno-deprecated-declarations", "-Wno-unused-result"]
        if force or _newer(s, o, _deps(s), cmd):
            jobs_list.append(cmd)
    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            futs = {ex.submit(_run, c): c for c in jobs_list}
            for f in cf.as_completed(futs):
                dt, _ = f.result()
                c = futs[f]
                with open(c[c.index("-o") + 1] + ".cmd", "w") as fh:  # the command that built it
                    fh.write(" ".join(c))
                if verbose:
                    src = futs[f][2]
                    print(f"[mlt-build] {os.path.relpath(src, REPO_DIR)}  {dt:.1f}s", flush=True)
    for a in asm_checks:  # asm-owned accumulators: no compiler spill may land in an AGPR
        sys.path.insert(0, os.path.join(REPO_DIR, "scripts"))
        from check_w4_agpr import check
        counts, bad = check(open(a).read())
        if bad:
            raise RuntimeError(f"compiler AGPR writes in asm-owned-accumulator kernels ({a}): {bad}")
        if verbose:
            print(f"[mlt-build] {os.path.basename(a)}: {len(counts)} kernels, no compiler AGPR writes", flush=True)
    out = out_path or ext_path()
    if force or jobs_list or not os.path.exists(out):
        link = ["g++", "-shared", "-o", out, *objs, f"-L{tlib}", f"-Wl,-rpath,{tlib}",
                "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
                "-lamdhip64", "-lrccl", "-Wl,--no-as-needed"]
        roctx = os.path.join(tlib, "libroctx64.so")
        if os.path.exists(roctx):
            link += ["-lroctx64"]
        _run(link)
        if verbose:
            print(f"[mlt-build] linked {os.path.relpath(out, REPO_DIR)}", flush=True)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=int(os.environ.get("MAX_JOBS", "8")))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    a = ap.parse_args(argv)
    build(jobs=min(a.jobs, 16), force=a.force, debug=a.debug)


if __name__ == "__main__":
    main()
