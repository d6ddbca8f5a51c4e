"""Layout model of the four-wave GEMMs (csrc/kernels/gemm_nt4.hip, gemm_wg4.hip), on CPU.

The kernels' index arithmetic, restated in Python, checked for what the GPU tests can only
see indirectly:
  * every LDS-DMA piece lands lane-linearly and the pieces of a K-tile cover each
    (image row, 16-B chunk) exactly once, with the source row / chunk the swizzle and the
    B-column permutation ask for;
  * the fragment reads are bank-conflict free in the lane groups of MI355X_MICROARCH.md
    §LDS (ds_read_b128: 4 groups of 16 lanes; ds_read_b64_tr_b16: 2 halves of 32);
  * the NT epilogue's stores cover the wave's 128 x 128 outputs exactly once, 16
    consecutive bytes per lane, one 256-B row segment per 16 lanes;
  * the weight-grad epilogue's LDS re-shaping is conflict free too.
"""

import itertools

B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
               list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
               list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64))]
HALVES = [list(range(32)), list(range(32, 64))]
W128_GROUPS = [list(range(8 * g, 8 * g + 8)) for g in range(8)]


def worst_degree(addrs, groups, width, nbanks=64):
    """max over lane groups of the number of distinct addresses sharing a bank"""
    worst = 1
    for grp in groups:
        banks = {}
        for lane in grp:
            a = addrs[lane]
            for w in range(width // 4):
                banks.setdefault((a // 4 + w) % nbanks, set()).add(a)
        worst = max(worst, max(len(v) for v in banks.values()))
    return worst


# ------------------------------------------------------------------- NT kernel (nt4)
def nt4_s(row):  # 16-B chunk swizzle of a [256][64] bf16 image (128-B rows)
    return (row >> 1) & 7


def nt4_pi(q):  # B image row q holds tile column pi(q) (128 h + 16 j + r -> 128 h + 8 r + j)
    h, j, r = q >> 7, (q >> 4) & 7, q & 15
    return 128 * h + 8 * r + j


def test_nt4_dma_pieces_cover_images():
    for operand in ("A", "B"):
        seen = {}
        for wave, p, lane in itertools.product(range(4), range(8), range(64)):
            li, lc = lane >> 3, lane & 7
            P = 8 * wave + p
            lds = P * 1024 + 16 * lane            # lane-linear DMA destination
            q, phys = lds // 128, (lds % 128) // 16
            assert q == 8 * P + li and phys == lc
            logical = lc ^ ((4 * (p & 1) + (li >> 1)) & 7)  # the kernel's per-lane source chunk
            assert logical == phys ^ nt4_s(q)
            if operand == "A":
                src_row = 64 * wave + 8 * p + li
            else:  # soB row base + 8 li (voB)
                src_row = 128 * (wave >> 1) + 64 * (p & 1) + 4 * (wave & 1) + (p >> 1) + 8 * li
                assert src_row == nt4_pi(q)
            key = (src_row, logical)
            assert key not in seen
            seen[key] = q
        assert len(seen) == 256 * 8


def test_nt4_fragment_reads_conflict_free():
    for wm, wn, kk, f in itertools.product(range(2), range(2), range(2), range(8)):
        a_addrs, b_addrs = [], []
        for lane in range(64):
            ch = ((4 * kk + (lane >> 4)) ^ (((lane & 15) >> 1) & 7))
            a_row = wm * 128 + 16 * f + (lane & 15)
            b_row = wn * 128 + 16 * f + (lane & 15)
            a_addrs.append(a_row * 128 + ch * 16)
            b_addrs.append(32768 + b_row * 128 + ch * 16)
            # the logical chunk read is what the MFMA lane needs: k = 8 (4 kk + lane >> 4) ..
            assert ch ^ nt4_s(a_row) == 4 * kk + (lane >> 4)
        assert worst_degree(a_addrs, B128_GROUPS, 16) == 1
        assert worst_degree(b_addrs, B128_GROUPS, 16) == 1


def test_nt4_epilogue_stores_cover_tile():
    for wm, wn in itertools.product(range(2), range(2)):
        seen = set()
        for i, e in itertools.product(range(8), range(4)):
            segs = {}
            for lane in range(64):
                r, q = lane & 15, lane >> 4
                row = wm * 128 + 16 * i + 4 * q + e
                col0 = wn * 128 + 8 * r
                # the lane's 8 values are acc[i][j][e], j = 0..7: output column = pi(B image row)
                cols = [nt4_pi(wn * 128 + 16 * j + r) for j in range(8)]
                assert cols == list(range(col0, col0 + 8))
                # MFMA D layout (A operand first): element e of lane l is row 4 (l >> 4) + e
                for c in cols:
                    assert (row, c) not in seen
                    seen.add((row, c))
                segs.setdefault(row, []).append(col0)
            for row, c0s in segs.items():  # 16 lanes x 16 B = one 256-B row segment
                assert sorted(c0s) == list(range(min(c0s), min(c0s) + 128, 8))
        assert len(seen) == 128 * 128


# ----------------------------------------------------------- weight-grad kernel (wgrad4)
def wg_g(r):
    return (r & 3) | (((r >> 3) & 1) << 2)


def test_wg4_dma_pieces_cover_images():
    seen = {}
    for wave, p, lane in itertools.product(range(4), range(8), range(64)):
        h, lc = lane >> 5, lane & 31
        P = 8 * wave + p
        lds = P * 1024 + 16 * lane
        row, phys = lds // 512, (lds % 512) // 16
        assert row == 16 * wave + 2 * p + h and phys == lc
        pp = (p & 1) | ((p >> 2) << 1)
        rep = (pp & 1) | ((pp >> 1) << 2)           # the class representative the kernel uses
        logical = lc ^ (2 * wg_g(2 * rep + h))
        assert logical == phys ^ (2 * wg_g(row))      # same swizzle as the piece's own row
        key = (row, logical)
        assert key not in seen
        seen[key] = True
    assert len(seen) == 64 * 32


def test_wg4_transposed_reads_conflict_free():
    for wm, kk, hf, f in itertools.product(range(2), range(2), range(2), range(8)):
        addrs = []
        for lane in range(64):
            ig = lane & 15
            fq, fp = ig >> 2, ig & 3
            krow = 8 * (lane >> 4) + fq + 32 * kk + 4 * hf
            fa = wm * 8 + f
            chunk = (2 * fa + (fp >> 1)) ^ (2 * wg_g(krow))
            addrs.append(krow * 512 + chunk * 16 + (fp & 1) * 8)
            # logical columns 16 fa + 4 fp .. +3 of token row krow
            assert (chunk ^ (2 * wg_g(krow))) * 8 + (fp & 1) * 4 == 16 * fa + 4 * fp
        assert worst_degree(addrs, HALVES, 8) == 1


def test_wg4_epilogue_reshape_conflict_free():
    # writes: lane l, fragment row ii, column block j -> [16 ii + (l & 15)][16 j + 4 (l >> 4)]
    for ii, j in itertools.product(range(4), range(8)):
        addrs = []
        for lane in range(64):
            row = 16 * ii + (lane & 15)
            u = 4 * j + (lane >> 4)
            addrs.append(row * 512 + ((u ^ (row & 7)) << 4))
        assert worst_degree(addrs, W128_GROUPS, 16, nbanks=32) == 1
    # reads: row rr, column c = 64 c2 + lane (one fp32 per lane)
    for rr, c2 in itertools.product(range(64), range(2)):
        addrs = []
        for lane in range(64):
            c = 64 * c2 + lane
            addrs.append(rr * 512 + (((c >> 2) ^ (rr & 7)) << 4) + (c & 3) * 4)
        assert worst_degree(addrs, HALVES, 4, nbanks=32) == 1


# -------------------------------------------------------- persistent tile walk (nt4)
def nt4_tile_coords(seq, tiles_m, tiles_n, gm):
    """q_tile_coords: groups of gm row blocks x every column, column-major inside a group."""
    per = gm * tiles_n
    grp = seq // per
    first = grp * gm
    g = min(gm, tiles_m - first)
    inn = seq - grp * per
    return first + inn % g, inn // g


def test_nt4_tile_walk_is_a_bijection():
    # the default group sizes (4 for N <= 1024, 1 up to 4096, 8 beyond) and partial last groups
    for tiles_m, tiles_n in ((480, 3), (480, 9), (480, 12), (480, 197), (7, 3), (13, 5), (1, 1), (9, 197)):
        for gm in (1, 2, 4, 8, 16):
            seen = {nt4_tile_coords(s, tiles_m, tiles_n, gm) for s in range(tiles_m * tiles_n)}
            assert seen == {(m, n) for m in range(tiles_m) for n in range(tiles_n)}, (tiles_m, tiles_n, gm)
