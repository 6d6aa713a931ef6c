"""CPU checks of the fp8 decoder's tile image layout (hvae_decoder.hip f8_off / f8_sw / f8_item_of)."""
import sys
from pathlib import Path

import pytest

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "scripts"))
import check_fp8_banks as fb  # noqa: E402


@pytest.mark.parametrize("D", [128, 256, 384, 768])
def test_fp8_image_reads_conflict_free(D):
    """Both operand reads of the sweep (row ds_read_b128, transposed ds_read_b64_tr_b8) hit distinct banks."""
    assert fb.worst_conflicts(D) == (1, 1)


@pytest.mark.parametrize("D", [128, 256, 384, 768])
def test_fp8_swizzle_is_a_permutation_within_rows(D):
    for it in range(64):
        chunks = sorted((fb.f8_off(D, it, ch) - it * D) // 16 for ch in range(D // 16))
        assert chunks == list(range(D // 16))


def test_gemm2_item_map_covers_the_tile():
    """Element j of lane half h of the GEMM2 operand covers each of the 64 items of a tile exactly once."""
    items = sorted(fb.f8_item_of(h, j) for h in range(2) for j in range(32))
    assert items == list(range(64))


def test_dec4_bf16_reads_conflict_free():
    """bf16 version-4 sweep (k_dec4_bf16, d = 768): with DEC4_ROWMAP's row map GEMM1's ds_read_b128, GEMM2's
    ds_read_b64_tr_b16 and the P reads all hit distinct banks; the natural row order was 2-way on GEMM1
    (SQ_LDS_BANK_CONFLICT 8.3e8 -> 6.4e7 per launch on MI355X, profiles/r02s3_pmc_dec4_lds.txt)."""
    import check_dec4_banks as db
    assert db.worst_conflicts(0x1320) == (1, 1, 1)
    assert db.worst_conflicts(0x3210)[0] == 2


def test_dec4_row_map_is_a_permutation():
    """Each wave half's 16 MFMA rows read 16 distinct own items, and lane block g's S^T rows are the items the
    kernel's P positions and tail mask assume (4 dec4_rowblk(g) + r)."""
    import check_dec4_banks as db
    for dh in range(2):
        rows, held = db.gemm1_rows(0x1320, dh)
        assert sorted(rows) == list(range(16 * dh, 16 * dh + 16))
        assert sorted(i for g in range(4) for i in held[g]) == list(range(16 * dh, 16 * dh + 16))
        for g in range(4):  # MFMA output row 4 g + r is A row 4 g + r
            assert held[g] == rows[4 * g: 4 * g + 4]


@pytest.mark.parametrize("R", [32, 64])
def test_gemm_fast_image(R):
    """f32 GEMM fast path (hvae_gemm.hip FImg, FAST_LAYOUT 1): every (k, row) slot of a stage is stored once,
    the fragment reads are conflict-free and the transposing stores at most 2-way (the first image: 2-way reads,
    4- and 8-way stores)."""
    import check_gemm_banks as gb
    assert gb.covers(R, 1)
    st, rd = gb.worst_conflicts(R, 1)
    assert rd == 1 and st <= 2
    assert gb.worst_conflicts(R, 0) == ((4, 2) if R == 32 else (8, 2))


def test_dec6_bf16_reads_conflict_free():
    """bf16 version-6 sweep (k_dec6_bf16, d = 768): with the image's chunk XOR 2 ((row >> 2) & 1) the GEMM1 row
    reads (ds_read_b128, 16x16x32 A operand) and the GEMM2 transposed reads (ds_read_b64_tr_b16, E^T, the k slots
    of a lane group 4 consecutive rows) hit distinct banks in natural row order; version 2's XOR
    ((row >> 2) & 3) would be 2-way on both."""
    import check_dec6_banks as d6
    assert d6.worst_conflicts(d6.KERNEL_BASES, d6.KERNEL_SWZ) == (1, 1)
    assert d6.worst_conflicts((0, 4, 8, 12), 0x84) == (2, 2)


def test_dec6_dma_pieces_cover_the_tile():
    """Wave w's 12 LDS-DMA pieces of a tile (rows 8 w .. + 7, piece i = 2 seg + half) write every byte of the
    48-KiB image once, each lane's 16 B the image position of the source chunk it loads."""
    import check_dec6_banks as d6
    seen = {}
    for w in range(4):
        for i in range(12):
            lds_base = w * 2048 + (i >> 1) * 8192 + (i & 1) * 1024
            for lane in range(64):
                row = 8 * w + ((lane >> 2) & 7)
                src = 128 * i + 64 * (lane >> 5) + 16 * ((lane & 3) ^ (2 * ((lane >> 4) & 1)))  # bytes in the row
                d = src // 2  # first dim of the 16-B chunk
                dst = lds_base + 16 * lane
                assert dst == d6.image_off(row, d, d6.swz_of(d6.KERNEL_SWZ))
                seen[dst] = seen.get(dst, 0) + 1
    assert sorted(seen) == list(range(0, 48 * 1024, 16)) and set(seen.values()) == {1}
