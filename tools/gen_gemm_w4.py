"""Generate cram_amd/csrc/gemm_w4_loop.inc: the hand-placed main loop of gemm_w4_kernel (cram_gemm.hip).

One workgroup = 4 waves (one per SIMD) computing a 256 (activation rows m) x 256 (weight rows n) output tile; wave w
owns n rows 128 (w & 1) .. +127 and m rows 128 (w >> 1) .. +127, i.e. 8 x 8 tiles of v_mfma_f32_16x16x32_bf16 whose
accumulators live in a[0:255] (tile (a, b) = weight fragment a, activation fragment b -> a[4 (8 a + b) .. +3]).
K advances in 64-deep tiles through a two-stage LDS ring (stage s: weight image at 64 KiB * s, activation image at
+32 KiB; 256 rows of 128 B, 16-byte chunk c of row r at slot c ^ ((r >> 1) & 7): conflict-free fragment reads).

Per K-tile t (stage s = t & 1 holds tile t, stage s ^ 1 holds tile t + 1, possibly still landing), 128 MFMAs:
  k-step 0 (MFMAs 0-63, fragment set F0 read during the previous tile):
    the 8 activation fragments of k-step 1 (F1) read from LDS              -> lgkmcnt(0), barrier B1
    the 8 activation LDS-DMA pieces of tile t + 2 into stage s (every wave has read stage s's activations)
    the 8 weight fragments of k-step 1 read                                 -> lgkmcnt(0), barrier B2
  k-step 1 (MFMAs 64-127, F1):
    the 8 weight LDS-DMA pieces of tile t + 2 into stage s
    vmcnt(16): this wave's pieces of tile t + 1 (issued one tile ago) landed -> barrier B3 (every wave's)
    the 16 fragments of tile t + 1's k-step 0 (F0) read from stage s ^ 1    -> lgkmcnt(0) before the last MFMA
Every other instruction sits in a gap between two MFMAs, one or two per gap: the stream of the vendor's 256 x 256 x 64
kernel, which keeps the matrix pipe fed from a single wave per SIMD.  The last two tiles run without DMA (and the very
last without the next tile's reads and B3).

Run:  python tools/gen_gemm_w4.py  (writes the .inc; the build does not run this)
"""
import os

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cram_amd", "csrc",
                   "gemm_w4_loop.inc")

# hard-coded fragment registers (clobbered): F0 = X0 v[128:159], Y0 v[160:191]; F1 = X1 v[192:223], Y1 v[224:255]
X = {0: 128, 1: 192}
Y = {0: 160, 1: 224}

# asm operands (named): %[rx0] %[rx1] %[ry0] %[ry1] LDS read bases (k-step 0 / 1, stage folded in, toggled per tile);
# %[vx0..7] %[vy0..7] per-lane DMA source offsets (row and swizzled chunk; a row past M is out of the descriptor's
# range and reads zeros); %[sx] %[sy] buffer descriptors; %[so] the K offset of the next tile to stage (soffset,
# +128 B per tile: outside the range check, which covers the rows); %[mx] %[my] LDS destination of the wave's first
# piece in the stage written next (toggled per tile); %[n] loop count


def mfma(a, b, ks):
    acc = 4 * (8 * a + b)
    return (f'v_mfma_f32_16x16x32_" TY " a[{acc}:{acc + 3}], v[{X[ks] + 4 * a}:{X[ks] + 4 * a + 3}], '
            f"v[{Y[ks] + 4 * b}:{Y[ks] + 4 * b + 3}], a[{acc}:{acc + 3}]")


def read(kind, ks, f):
    base = X[ks] if kind == "x" else Y[ks]
    return f"ds_read_b128 v[{base + 4 * f}:{base + 4 * f + 3}], %[r{kind}{ks}] offset:{2048 * f}"


def dma(kind, i):
    return f"buffer_load_dwordx4 %[v{kind}{i}], %[s{kind}], %[so] offen lds"


def dma_group(kind, step_apart=True):
    """8 pieces of one operand: m0 set in an earlier gap, stepped 4 KiB (32 image rows) after every piece (the wave's
    pieces are every fourth 8-row block, so the 4 waves' i-th pieces land side by side); then the destination toggles
    to the other stage, and after the weight group (the second of a tile) the K offset moves to the next tile,
    wrapping at the end of the K range (%[kend] = the range's bytes per row).  Returned as a list of (slot offset,
    instructions): with step_apart the m0 step of a piece goes one MFMA after the piece (as the vendor stream places
    it: an m0 write right behind the LDS-DMA that reads m0 waits for that piece to issue), never in the same gap."""
    out = [(0, [f"s_mov_b32 m0, %[m{kind}]"])]
    for i in range(8):
        out.append((0, [dma(kind, i)]))
        if i < 7:
            out.append((1 if step_apart else 0, ["s_add_u32 m0, m0, 4096"]))
    tail = [f"s_xor_b32 %[m{kind}], %[m{kind}], 0x10000"]
    if kind == "x":
        tail += ["s_add_u32 %[so], %[so], 128", "s_cmp_eq_u32 %[so], %[kend]", "s_cselect_b32 %[so], 0, %[so]"]
    out.append((0, tail))
    return out


def place_dma(gaps, slots, kind):
    """Put dma_group(kind) at its slots: slots = [m0 setup, piece 0..7, tail]; each m0 step one gap after its piece."""
    grp = dma_group(kind)
    it = iter(slots)
    last = None
    for off, ins in grp:
        if off == 0:
            last = next(it)
            gaps[last].extend(ins)
        else:
            gaps[last + off].extend(ins)


# Gap slots of one K-tile (instructions issued after MFMA i), placed as the vendor kernel places them: a counter
# wait always one MFMA before its barrier (the matrix pipe has work while the wave waits at the barrier), the pieces of
# each operand spread over two intervals, the next tile's fragments read from B3 on.
VENDOR = dict(
    Y1=[0, 2, 4, 6, 8, 10, 12, 14],                            # k-step 1 activation fragments
    B1=(20, 21),                                               # lgkmcnt(0) | s_barrier
    YDMA=[15, 22, 25, 28, 31, 34, 52, 55, 58, 59],             # m0 setup, 8 pieces, stage toggle
    X1=[24, 27, 30, 33, 36, 38, 40, 42],                       # k-step 1 weight fragments
    B2=(50, 51),
    XDMA=[60, 61, 64, 85, 87, 89, 96, 100, 124, 125],          # m0 setup, 8 pieces, toggle + K offset
    LATE=3,                                                    # weight pieces issued after B3
    TOGGLE=[83, 84],                                           # read bases to the next stage (2 per gap)
    B3=(91, 92),                                               # vmcnt | s_barrier
    NEXT_Y0=[93, 94, 95, 97, 98, 102, 103, 104],               # next tile's k-step 0 fragments
    NEXT_X0=[105, 106, 109, 112, 114, 117, 120, 123],
    LGKM_END=126)
# (variant B: every piece of tile t + 2 before B3 -- measured 0.95-0.97x of A, r04; dropped)
# Round 5 probes (same-process A/B on the sweep's five GEMMs, tools/ab_gemm_builds.py, profiles/r05/ab_loop/; every
# output bit-equal): C 0.92-0.96x, D 0.99-1.00x, E 0.92-0.97x of A -- the vendor placement stays.
# variant C (r05 probe): one rendezvous for both operands' k-step 1 fragments (B12) instead of B1 + B2 -- every wave
# has read all of stage s once its 16 k-step 1 fragments have landed, so both DMA groups of tile t + 2 may follow
TWO_BARRIER = dict(
    Y1=[0, 2, 4, 6, 8, 10, 12, 14],
    X1=[16, 18, 20, 22, 24, 26, 28, 30],
    B12=(40, 41),
    YDMA=[42, 43, 46, 49, 52, 55, 58, 61, 64, 66],
    XDMA=[67, 68, 71, 74, 77, 80, 96, 100, 124, 125],
    LATE=3,
    TOGGLE=[83, 84],
    B3=(91, 92),
    NEXT_Y0=[93, 94, 95, 97, 98, 102, 103, 104],
    NEXT_X0=[105, 106, 109, 112, 114, 117, 120, 123],
    LGKM_END=126)
# variants D / E (r05 probe): the wait closing a tile counts (lgkmcnt(3)): the next tile's last three weight fragments
# (first used by MFMA 40) may still be landing while its first MFMAs issue; the k-step 1 rendezvous (<= gap 39) or,
# without DMA, an extra wait at gap 20 drains them
VAR_D = dict(VENDOR, LGKM_END_N=3, CARRY_WAIT=20)
VAR_E = dict(TWO_BARRIER, B12=(38, 39), LGKM_END_N=3, CARRY_WAIT=20)
VARIANTS = {"A": VENDOR}           # (+ "C": TWO_BARRIER, "D": VAR_D, "E": VAR_E to rebuild the probes)


# Diagnostic stamps (variant "S", -DCRAM_W4_STAMPS builds only): s_memtime brackets around each rendezvous, the
# cycles accumulated per wave in s[80:87] (B1, B2, B3, whole tiles); an SMEM result needs lgkmcnt(0), so the stamps
# sit only where no LDS read is outstanding (before B1 / B2 the wait is the rendezvous' own lgkmcnt(0)).
def stamp_open():
    return ["s_memtime s[88:89]"]


def stamp_close(acc):
    return ["s_memtime s[90:91]", "s_waitcnt lgkmcnt(0)", "s_sub_u32 s90, s90, s88", f"s_add_u32 s{acc}, s{acc}, s90"]


def body(dma_on: bool, next_on: bool, c=VENDOR, stamps=False):
    """Instruction list of one K-tile: 128 MFMAs with the other instructions placed in their gaps (slot table c)."""
    gaps = {i: [] for i in range(128)}          # instructions issued after MFMA i

    def place(slots, groups):
        assert len(slots) == len(groups)
        for s, g in zip(slots, groups):
            gaps[s].extend(g)

    place(c["Y1"], [[read("y", 1, f)] for f in range(8)])
    place(c["X1"], [[read("x", 1, f)] for f in range(8)])
    if dma_on and "B12" in c:
        gaps[c["B12"][0]] += (stamp_open() if stamps else []) + ["s_waitcnt lgkmcnt(0)"]
        gaps[c["B12"][1]] += ["s_barrier"] + (stamp_close(80) if stamps else [])
        place_dma(gaps, c["YDMA"], "y")
        place_dma(gaps, c["XDMA"], "x")
    elif dma_on:
        gaps[c["B1"][0]] += (stamp_open() if stamps else []) + ["s_waitcnt lgkmcnt(0)"]
        gaps[c["B1"][1]] += ["s_barrier"] + (stamp_close(80) if stamps else [])
        place_dma(gaps, c["YDMA"], "y")
        gaps[c["B2"][0]] += (stamp_open() if stamps else []) + ["s_waitcnt lgkmcnt(0)"]
        gaps[c["B2"][1]] += ["s_barrier"] + (stamp_close(81) if stamps else [])
        place_dma(gaps, c["XDMA"], "x")
    else:                                                   # k-step 1's fragments land before its MFMAs
        if c.get("CARRY_WAIT") is not None:
            gaps[c["CARRY_WAIT"]].append("s_waitcnt lgkmcnt(0)")
        gaps[(c["B12"] if "B12" in c else c["B2"])[0]].append("s_waitcnt lgkmcnt(0)")
    if next_on:
        toggle = ["v_xor_b32 %[rx0], 0x10000, %[rx0]", "v_xor_b32 %[ry0], 0x10000, %[ry0]",
                  "v_xor_b32 %[rx1], 0x10000, %[rx1]", "v_xor_b32 %[ry1], 0x10000, %[ry1]"]
        place(c["TOGGLE"], [toggle[:2], toggle[2:]])
        # this wave's pieces of tile t + 1 (all but the 3 issued after B3 of the previous tile's iteration... i.e.
        # every piece older than this tile's 13 pre-B3 pieces) have landed
        gaps[c["B3"][0]] += (stamp_open() if stamps else []) + [
            f"s_waitcnt vmcnt({16 - c['LATE']})" if dma_on else "s_waitcnt vmcnt(0)"]
        gaps[c["B3"][1]] += ["s_barrier"] + (stamp_close(82) if stamps else [])
        place(c["NEXT_Y0"], [[read("y", 0, f)] for f in range(8)])
        place(c["NEXT_X0"], [[read("x", 0, f)] for f in range(8)])
        gaps[c["LGKM_END"]].append(f"s_waitcnt lgkmcnt({c.get('LGKM_END_N', 0)})")
    lines = []
    if stamps and dma_on:                        # whole-tile time: the bracket closes after the last MFMA
        lines += ["s_memtime s[92:93]"]
    for i in range(128):
        a, b = divmod(i % 64, 8)
        lines.append(mfma(a, b, i // 64))
        lines.extend(gaps[i])
    if stamps and dma_on:
        lines += ["s_memtime s[94:95]", "s_waitcnt lgkmcnt(0)", "s_sub_u32 s94, s94, s92", "s_add_u32 s83, s83, s94",
                  "s_add_u32 s84, s84, 1"]
    return lines


def prologue():
    """Tiles 0 and 1 into stages 0 and 1 (16 pieces each), wait for tile 0, read its k-step 0 fragments."""
    lines = ["s_nop 4"]                            # descriptors may come straight from a VALU SGPR write
    for _tile in range(2):
        for kind in ("y", "x"):                    # the loop's order: activations, then weights (+ K offset)
            for _, g in dma_group(kind, step_apart=False):
                for ln in g:
                    lines.append(ln)
                    if ln.startswith(("s_mov_b32 m0", "s_add_u32 m0")):
                        lines.append("s_nop 0")    # one wait state between an m0 write and the piece reading it
    lines += ["s_waitcnt vmcnt(16)", "s_barrier"]           # tile 0 landed (tile 1's 16 pieces may be in flight)
    for f in range(8):
        lines += [read("x", 0, f), read("y", 0, f)]
    lines.append("s_waitcnt lgkmcnt(0)")
    return lines


def emit():
    out = ["// GENERATED by tools/gen_gemm_w4.py -- do not edit.  The main loop of gemm_w4_kernel (cram_gemm.hip).",
           "// Operands: see the generator's docstring.  Requires K-tiles per range >= 2.  TY: bf16 or f16 (a string literal)."]

    def put(lines):
        for ln in lines:
            out.append(f'  "{ln}\\n\\t" \\')

    for name, c, st in [(k, v, False) for k, v in VARIANTS.items()] + [("S", VENDOR, True)]:
        full, nodma, last = body(True, True, c, st), body(False, True, c, st), body(False, False, c, st)
        out.append(f"// variant {name}")
        out.append(f"#define CRAM_GEMM_W4_LOOP_{name}(TY) \\")
        put((["s_mov_b32 s80, 0", "s_mov_b32 s81, 0", "s_mov_b32 s82, 0", "s_mov_b32 s83, 0", "s_mov_b32 s84, 0"]
             if st else []) + prologue())
        put(["s_cmp_eq_u32 %[n], 0", "s_cbranch_scc1 2f", "1:"])   # (the wrap's s_cmp sits before this one)
        put(full)
        put(["s_sub_u32 %[n], %[n], 1", "s_cmp_eq_u32 %[n], 0", "s_cbranch_scc0 1b", "2:"])
        put(nodma)
        put(last)
        out.append('  ""')
        n_mfma = sum(1 for ln in full if ln.startswith("v_mfma"))
        print(f"variant {name}: {len(full)} instructions per K-tile ({n_mfma} MFMAs)")
    with open(OUT, "w") as f:
        f.write("\n".join(out) + "\n")
    print(f"wrote {OUT}")


if __name__ == "__main__":
    emit()
