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
