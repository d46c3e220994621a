"""Generate the main loop of the 4-wave 256x256x64 bf16 GEMM (csrc/kernels/gemm_w4_loop.inc).

Why generated asm: the loop keeps 256 fp32 accumulators per lane in AGPRs (one wave per SIMD, a
128x128 wave tile -- 64 FLOP per LDS byte instead of the ping-pong's 43), and its throughput
depends on WHERE each LDS read, LDS-DMA (glds) and barrier sits between the 128 MFMAs of a K-tile.
hipcc splits such accumulators between VGPRs and AGPRs and re-orders the loads
(profiles/README.md, gemm_ring_probe_r3), so the loop is one asm block with fixed registers:

  a[0:255]   accumulators, acc(i, j) = a[4(8i + j) : 4(8i + j) + 3]  (i: A 16-row block, j: B block)
  v[0:63]    F0 = the kh0 fragments (A0 i -> v[4i:4i+3], B0 j -> v[32+4j : 32+4j+3])
  v[64:127]  F1 = the kh1 fragments (same layout + 64)

Per K-tile t (LDS stage s = t & 1; each stage = A [256 rows][128 B] + B [256 rows][128 B], 16-B
chunks XOR-swizzled by (row >> 1) & 7, conflict-free for the 16-lane groups of ds_read_b128):
  X: 64 MFMAs on F0 (k 0..31 of the tile); 16 ds_read_b128 of the tile's kh1 fragments -> F1
  s_waitcnt vmcnt(0) lgkmcnt(0); s_barrier   (tile t+1 landed everywhere; stage s fully read)
  Y: 64 MFMAs on F1; 16 glds of tile t+2 -> stage s, 16 ds_read_b128 of tile t+1's kh0 -> F0
  s_waitcnt lgkmcnt(0)
One barrier per K-tile (2,048 MFMA cycles per SIMD), reads / DMAs in the first half of each phase
so the second half covers their latency. MFMA operands are swapped (D = B_tile . A_tile^T) so a
lane's accumulator holds 4 consecutive output columns (8-byte bf16 stores in the epilogue).

Usage: python scripts/gen_gemm_w4.py  (rewrites the .inc; the kernel source includes it)
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "ml_trainer_amd", "csrc", "kernels", "gemm_w4_loop.inc")

STAGE = 65536
B_OFF = 32768


def acc(i, j):
    f = 8 * i + j
    return f"a[{4 * f}:{4 * f + 3}]"


def frag(fset, ab, idx):
    base = 64 * fset + (32 if ab == "B" else 0) + 4 * idx
    return f"v[{base}:{base + 3}]"


def mfma(fset, k, zero_c=False):
    i, j = k // 8, k % 8
    c = "0" if zero_c else acc(i, j)  # the first K-tile starts from C = 0 (no accumulator zeroing)
    return f"v_mfma_f32_16x16x32_bf16 {acc(i, j)}, {frag(fset, 'B', j)}, {frag(fset, 'A', i)}, {c}"


def read(fset, idx, stage, kh, bn=False, an=False):
    """idx 0..7: A fragment idx, 8..15: B fragment idx - 8 (kh fragments of `stage`). With bn (B
    stored [k][n], n-contiguous: the dgrad layout) a B fragment is two ds_read_b64_tr_b16 (k rows
    kh*32 + 8g + q and + 4) from the per-fragment lane address v[192 + 8 stage + j]; with an (A stored
    [k][m]: the weight-gradient layout) the same for A from v[208 + 8 stage + i]."""
    ab = "A" if idx < 8 else "B"
    n = idx % 8
    if (ab == "B" and bn) or (ab == "A" and an):
        base = 64 * fset + (32 if ab == "B" else 0) + 4 * n
        off = (B_OFF if ab == "B" else 0) + kh * 16384
        areg = (192 if ab == "B" else 208) + 8 * stage + n
        return [f"ds_read_b64_tr_b16 v[{base}:{base + 1}], v{areg} offset:{off}",
                f"ds_read_b64_tr_b16 v[{base + 2}:{base + 3}], v{areg} offset:{off + 2048}"]
    reg = f"%[r{ab.lower()}{stage}{kh}]"
    return [f"ds_read_b128 {frag(fset, ab, n)}, {reg} offset:{n * 2048}"]


def reads(fset, stage, kh, bn, an=False):
    return [r for idx in range(16) for r in read(fset, idx, stage, kh, bn, an)]


def glds(p, stage):
    """p 0..7: A rows (p*4 + w)*8.., p 8..15: B."""
    ab = "a" if p < 8 else "b"
    q = p % 8
    imm = stage * STAGE + (B_OFF if ab == "b" else 0) + q * 4096
    sp = "s[88:89]" if ab == "a" else "s[90:91]"
    return [f"s_add_u32 m0, %[lw], {imm}", f"global_load_lds_dwordx4 %[g{ab}{q}], {sp}"]


def adv(bn, an=False):
    """advance the DMA sources by one K-tile: 128 B of a k-contiguous row; 64 rows of an mn-contiguous one"""
    a = "%[astep]" if an else "128"
    b = "%[bstep]" if bn else "128"
    return [f"s_add_u32 s88, s88, {a}", "s_addc_u32 s89, s89, 0", f"s_add_u32 s90, s90, {b}", "s_addc_u32 s91, s91, 0"]


def phase_x(stage, out, bn, zero_c=False, an=False):
    """64 MFMAs on F0; the tile's kh1 fragments -> F1, one read per MFMA gap from the start (16
    ds_read_b128, 8 + 16 with transposed B, 32 with both transposed)."""
    rd = reads(1, stage, 1, bn, an)
    for k in range(64):
        out.append(mfma(0, k, zero_c))
        if bn or an:
            if k < len(rd):
                out.append(rd[k])
        elif k % 2 == 0 and k < 32:
            out.append(rd[k // 2])


def sync(out):
    out.append("s_waitcnt vmcnt(0) lgkmcnt(0)")
    out.append("s_barrier")


def phase_y(stage, do_glds, do_reads, out, bn, an=False):
    """DMAs one per 4 MFMAs over the whole phase (each costs ~60 issue cycles beside the MFMAs, so
    bunching them in the first half stalled the MFMA stream: 1,494 vs 1,570 TF at 8192^3), reads
    of the next tile's kh0 fragments one per odd MFMA gap (with both operands transposed, 32 reads:
    the odd gaps below 48 and the gaps 2 mod 4 below 32, so the last lands well before the wait)."""
    rd = reads(0, stage ^ 1, 0, bn, an) if do_reads else []
    if an:
        slots = sorted([k for k in range(1, 48, 2)] + [k for k in range(2, 32, 4)])
    else:
        slots = [k for k in range(1, 64, 2)]
    at = {k: i for i, k in enumerate(slots)}
    for k in range(64):
        out.append(mfma(1, k))
        if do_glds and k % 4 == 0:
            out.extend(glds(k // 4, stage))
        if k in at and at[k] < len(rd):
            out.append(rd[at[k]])
    if do_glds:
        out += adv(bn, an)
    if do_reads:
        out.append("s_waitcnt lgkmcnt(0)")


def build(bn=False, an=False):
    out = ["s_mov_b64 s[88:89], %[sa]", "s_mov_b64 s[90:91], %[sb]"]
    if bn:  # per-fragment transposed-read lane addresses: v[192 + j] = (32 j ^ X) + R, stage 1 + 64 KB
        for j in range(8):
            out.append(f"v_xor_b32 v{192 + j}, {32 * j}, %[rbx]")
            out.append(f"v_add_u32 v{192 + j}, v{192 + j}, %[rbr]")
            out.append(f"v_add_u32 v{200 + j}, 0x10000, v{192 + j}")
    if an:  # the same for A (its own row / column base, the same XOR term)
        for j in range(8):
            out.append(f"v_xor_b32 v{208 + j}, {32 * j}, %[rbx]")
            out.append(f"v_add_u32 v{208 + j}, v{208 + j}, %[rar]")
            out.append(f"v_add_u32 v{216 + j}, 0x10000, v{208 + j}")
    # prologue: DMA tiles 0 / 1 into stages 0 / 1, F0 <- tile 0 kh0
    for t in range(2):
        for p in range(16):
            out.extend(glds(p, t))
        out += adv(bn, an)
    out.append("s_waitcnt vmcnt(16)")
    out.append("s_barrier")
    out += reads(0, 0, 0, bn, an)
    out.append("s_waitcnt lgkmcnt(0)")
    # first pair peeled (tile 0 starts from C = 0); np = nk / 2 - 2 more full pairs, then the last
    phase_x(0, out, bn, zero_c=True, an=an)
    sync(out)
    phase_y(0, True, True, out, bn, an)
    phase_x(1, out, bn, an=an)
    sync(out)
    phase_y(1, True, True, out, bn, an)
    out += ["s_cmp_eq_u32 %[np], 0", "s_cbranch_scc1 L_w4_last_%="]
    out.append("L_w4_loop_%=:")
    for s in range(2):
        phase_x(s, out, bn, an=an)
        sync(out)
        phase_y(s, True, True, out, bn, an)
    out += ["s_sub_u32 %[np], %[np], 1", "s_cmp_lg_u32 %[np], 0", "s_cbranch_scc1 L_w4_loop_%="]
    out.append("L_w4_last_%=:")
    # last pair: no DMAs, no reads past the last tile
    phase_x(0, out, bn, an=an)
    sync(out)
    phase_y(0, False, True, out, bn, an)
    phase_x(1, out, bn, an=an)
    sync(out)
    phase_y(1, False, False, out, bn, an)
    # MFMA -> v_accvgpr_read hazard before the epilogue's reads
    out += ["s_nop 15", "s_nop 15", "s_nop 7"]
    return out


# ---- fp8 (block-scaled v_mfma_scale_f32_16x16x128_f8f6f4, scales fixed at 1.0) ------------------
# A K-tile is 128 fp8 = the same 128-byte LDS rows. Fragment = 32 bytes per lane (8 VGPRs, two
# ds_read_b128 of chunks 2g and 2g + 1). Registers: A double-buffered v[0:63] / v[64:127], B
# single-buffered v[128:191] and refilled column by column: 64 MFMAs per K-tile in column-major
# order (j outer), so B_j is free 8 MFMAs after its first use; its next-tile copy is read 2 MFMAs
# after its last use (no WAR on an MFMA source still in flight). The tile's barrier sits after the
# refill of B_7 (read at MFMA 1 of the tile from the tile's own stage): from there the stage is
# read out, so the DMAs of tile t + 2 go into it, and tile t + 1 (landed: vmcnt(0)) is readable.
# 32 cycles per MFMA on one SIMD -> 2,048 cycles per K-tile of 128: twice the bf16 FLOP rate.
def f8_frag(buf, idx):
    base = {"A0": 0, "A1": 64, "B": 128}[buf] + 8 * idx
    return base


def f8_read(buf, idx, stage):
    ab = "b" if buf == "B" else "a"
    b = f8_frag(buf, idx)
    return [f"ds_read_b128 v[{b}:{b + 3}], %[r{ab}L{stage}] offset:{idx * 2048}",
            f"ds_read_b128 v[{b + 4}:{b + 7}], %[r{ab}H{stage}] offset:{idx * 2048}"]


def f8_mfma(k, acur, zero_c):
    j, i = k // 8, k % 8
    c = "0" if zero_c else acc(i, j)
    a, b = f8_frag(acur, i), f8_frag("B", j)
    return (f"v_mfma_scale_f32_16x16x128_f8f6f4 {acc(i, j)}, v[{b}:{b + 7}], v[{a}:{a + 7}], {c}, v192, v192 "
            "op_sel_hi:[0,0,0] cbsz:%[fb] blgp:%[fa]")


def f8_tile(stage, acur, anext, out, zero_c=False, refill_b7=True, do_glds=True, do_reads=True):
    ra = [r for idx in range(8) for r in f8_read(anext, idx, stage ^ 1)] if do_reads else []
    for k in range(64):
        out.append(f8_mfma(k, acur, zero_c))
        if k == 1 and refill_b7:
            out += f8_read("B", 7, stage)
        if k == 2:
            out += ["s_waitcnt vmcnt(0) lgkmcnt(0)", "s_barrier"]
        if do_glds and k >= 3 and (k - 3) % 4 == 0:
            out.extend(glds((k - 3) // 4, stage))
        if do_reads:
            if k >= 9 and (k - 9) % 8 == 0 and (k - 9) // 8 < 7:  # B_j of the next tile, j = 0..6
                out += f8_read("B", (k - 9) // 8, stage ^ 1)
            if 4 <= k <= 34 and k % 2 == 0:
                out.append(ra[(k - 4) // 2])
    if do_glds:
        out += adv(False)
    if do_reads:
        out.append("s_waitcnt lgkmcnt(2)")  # all but B_6's two reads: the next tile's first MFMAs' operands


def build_f8():
    out = ["s_mov_b64 s[88:89], %[sa]", "s_mov_b64 s[90:91], %[sb]", "v_mov_b32 v192, 0x7f"]
    for t in range(2):
        for p in range(16):
            out.extend(glds(p, t))
        out += adv(False)
    out += ["s_waitcnt vmcnt(16)", "s_barrier"]
    for idx in range(8):
        out += f8_read("A0", idx, 0)
    for idx in range(8):
        out += f8_read("B", idx, 0)
    out.append("s_waitcnt lgkmcnt(0)")
    f8_tile(0, "A0", "A1", out, zero_c=True, refill_b7=False)
    f8_tile(1, "A1", "A0", out)
    out += ["s_cmp_eq_u32 %[np], 0", "s_cbranch_scc1 L_w4f8_last_%="]
    out.append("L_w4f8_loop_%=:")
    f8_tile(0, "A0", "A1", out)
    f8_tile(1, "A1", "A0", out)
    out += ["s_sub_u32 %[np], %[np], 1", "s_cmp_lg_u32 %[np], 0", "s_cbranch_scc1 L_w4f8_loop_%="]
    out.append("L_w4f8_last_%=:")
    f8_tile(0, "A0", "A1", out, do_glds=False)
    f8_tile(1, "A1", "A0", out, do_glds=False, do_reads=False)
    out += ["s_nop 15", "s_nop 15", "s_nop 15", "s_nop 7"]
    return out


def emit(f, name, lines):
    f.write(f"// {name}: {len(lines)} instructions\n#define {name} \\\n")
    for ln in lines:
        f.write(f'  "{ln}\\n" \\\n')
    f.write('  ""\n')


def main():
    clob = ", ".join(f'"v{r}"' for r in range(128)) + ", " + ", ".join(f'"a{r}"' for r in range(256))
    clob += ', "s88", "s89", "s90", "s91", "m0", "scc"'
    with open(OUT, "w") as f:
        f.write("// GENERATED by scripts/gen_gemm_w4.py -- do not edit. Main loop of gemm_w4_kernel\n")
        f.write("// (see the generator's docstring for the schedule).\n")
        emit(f, "MLT_W4_LOOP_ASM", build())
        emit(f, "MLT_W4_LOOP_ASM_BN", build(bn=True))
        f.write(f"#define MLT_W4_CLOBBERS {clob}\n")
        clob_bn = clob + ", " + ", ".join(f'"v{r}"' for r in range(192, 208))
        f.write(f"#define MLT_W4_CLOBBERS_BN {clob_bn}\n")
        emit(f, "MLT_W4_LOOP_ASM_ANBN", build(bn=True, an=True))
        clob_anbn = clob + ", " + ", ".join(f'"v{r}"' for r in range(192, 224))
        f.write(f"#define MLT_W4_CLOBBERS_ANBN {clob_anbn}\n")
        emit(f, "MLT_W4F8_LOOP_ASM", build_f8())
        clob_f8 = ", ".join(f'"v{r}"' for r in range(193)) + ", " + ", ".join(f'"a{r}"' for r in range(256))
        clob_f8 += ', "s88", "s89", "s90", "s91", "m0", "scc"'
        f.write(f"#define MLT_W4F8_CLOBBERS {clob_f8}\n")
        # the epilogue's LDS image straight from the accumulators (ds_write takes AGPR data on gfx950:
        # no v_accvgpr_read per element): half h = fragments 8 (4h + i) + j, lane-relative row 16 i,
        # column 16 j of the 132-float-pitch image -> immediate offsets from one address register.
        # Half 0 opens with 3 x s_nop 7 (24 wait states): the MFMA -> LDS-read-of-its-result hazard
        # against the main loop's last MFMAs is not interlocked.
        for h in range(2):
            lines = ["s_nop 7", "s_nop 7", "s_nop 7"] if h == 0 else []
            for i in range(4):
                for j in range(8):
                    fr = 8 * (4 * h + i) + j
                    lines.append(f"ds_write_b128 %[va], a[{4 * fr}:{4 * fr + 3}] offset:{i * 16 * 132 * 4 + j * 64}")
            emit(f, f"MLT_W4_IMG_H{h}", lines)
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
