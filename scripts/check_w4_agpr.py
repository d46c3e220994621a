"""Build-time guard for the 4-wave GEMM (gemm_w4.hip): its accumulators live in AGPRs owned by the
inline asm, which the compiler does not know about between the main-loop asm and the epilogue's
reads. A compiler-generated v_accvgpr_write (a VGPR spill into an AGPR) in such a kernel could
overwrite an accumulator, so every gemm_w4 kernel must contain none.
Usage: python scripts/check_w4_agpr.py [asm.s]   (default: compiles gemm_w4.hip to a temp .s)"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def asm_text(path=None):
    if path:
        return open(path).read()
    src = os.path.join(ROOT, "ml_trainer_amd", "csrc", "kernels", "gemm_w4.hip")
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "w4.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-I" + os.path.join(ROOT, "ml_trainer_amd", "csrc", "include"),
                        "-I" + os.path.join(ROOT, "ml_trainer_amd", "csrc", "kernels"),
                        "--cuda-device-only", "-S", src, "-o", out], check=True)
        return open(out).read()


def check(text):
    bad, cur, counts = [], None, {}
    for line in text.split("\n"):
        m = re.match(r"^(_ZN3mlt\d+gemm_w4\w*):", line)
        if m:
            cur = m.group(1)
            counts[cur] = 0
            continue
        if line.startswith(".Lfunc_end"):
            cur = None
        elif cur and "v_accvgpr_write" in line:
            counts[cur] += 1
    for k, n in counts.items():
        if n:
            bad.append((k, n))
    return counts, bad


if __name__ == "__main__":
    counts, bad = check(asm_text(sys.argv[1] if len(sys.argv) > 1 else None))
    for k, n in bad:
        print(f"AGPR spill in {k}: {n} v_accvgpr_write")
    print(f"{len(counts)} gemm_w4 kernels checked, {len(bad)} with compiler AGPR writes")
    sys.exit(1 if bad else 0)
