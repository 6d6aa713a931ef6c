"""LDS bank-conflict model of the f32 GEMM fast path's stage image (hvae_gemm.hip FImg / fast_lstore / compute).

Image: [8 k-chunks][CS rows][4 k] floats. A [k][r]-ordered operand (the fast path's A^T and B) is stored with
ds_write_b32 (2 lane groups of 32, bank (dword) mod 32); the MFMA fragments are read with ds_read_b128 (4 lane
groups of 16, {0-3,12-15,20-27}, {4-11,16-19,28-31} and +32, bank (dword) mod 64), per MI355X_MICROARCH.md's
LDS table. `layout` 0 is the first image (CS = R + 4), 1 the kernel's (FAST_LAYOUT): CS = R and row r in slot
r ^ ((r >> 3) & 3) of its chunk.
"""
G128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
        list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
G128 = G128 + [[lane + 32 for lane in g] for g in G128]
G32 = [list(range(32)), list(range(32, 64))]


def _worst(groups, addr_of, nbytes, nbanks):
    worst = 1
    for g in groups:
        banks = {}
        for lane in g:
            a = addr_of(lane)
            for b in range(a // 4, (a + nbytes) // 4):
                banks.setdefault(b % nbanks, set()).add(a)
        worst = max(worst, max(len(v) for v in banks.values()))
    return worst


def cs(R, layout):
    return R + 4 if layout == 0 else R


def slot(layout, r):
    return r if layout == 0 else r ^ ((r >> 3) & 3)


def store_addr(R, layout, f, s):
    """Byte address of the s-th ds_write_b32 of float4 f (thread t + 256 i) of a [k][r] operand."""
    k, r4 = f // (R // 4), f % (R // 4)
    return 4 * ((k >> 2) * cs(R, layout) * 4 + 4 * slot(layout, 4 * r4 + s) + (k & 3))


def read_addr(R, layout, half, j, i, lane):
    """Byte address of the fragment read a_[(4 j + q) * CS + 16 i] + wm + c16 of wave row half `half`."""
    q, c16 = lane >> 4, lane & 15
    return 16 * ((4 * j + q) * cs(R, layout) + slot(layout, half * (R // 2) + c16 + 16 * i))


def worst_conflicts(R, layout):
    """(ds_write_b32 worst, ds_read_b128 worst) over one stage of one operand."""
    w_st = 1
    for i in range(R * 32 // 4 // 256):
        for wave in range(4):
            for s in range(4):
                w_st = max(w_st, _worst(G32, lambda l: store_addr(R, layout, 64 * wave + l + 256 * i, s), 4, 32))
    w_rd = max(_worst(G128, lambda l: read_addr(R, layout, half, j, i, l), 16, 64)
               for half in range(2) for j in range(2) for i in range(R // 32))
    return w_st, w_rd


def covers(R, layout):
    """Every (k, row) slot of the stage is written exactly once."""
    seen = set()
    for f in range(8 * R):
        for s in range(4):
            seen.add(store_addr(R, layout, f, s))
    return len(seen) == 32 * R


if __name__ == "__main__":
    for R in (32, 64):
        for layout in (0, 1):
            print(R, layout, worst_conflicts(R, layout), covers(R, layout))
