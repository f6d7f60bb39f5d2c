"""CPU checks of layout rules the kernels rely on (restated from the device code).

* chunk_of_block (two-pass-lanczos_amd/csrc/tpl_kcommon.h): the XCD-affine order of the
  chunk part of an SpMV grid is a bijection onto the chunks (padding blocks map to -1),
  whatever the number of bin blocks in front of it — correctness never depends on the
  placement it aims for.
* the placement it aims for: with block b on XCD b % 8, chunk c lands on XCD
  (c // cpe) % 8, the XCD of element-wise block c // cpe (cpe = kElemRows / kChunkRows
  chunks per element-wise block; 4 in the shipped build, 2 and 1 checked as well).
"""
import pytest

from conftest import CHUNK_ROWS, ELEM_ROWS

CPE = ELEM_ROWS // CHUNK_ROWS


def chunk_of_block(i, n_slice_blocks, n_chunks, cpe=CPE):
    x = ((i & 7) + n_slice_blocks) & 7
    c = (i // (8 * cpe)) * (8 * cpe) + cpe * x + ((i >> 3) % cpe)
    return c if c < n_chunks else -1


def spmv_grid(n_slice_blocks, n_chunks, cpe=CPE):
    g = 8 * cpe
    return n_slice_blocks + (n_chunks + g - 1) // g * g


@pytest.mark.parametrize("cpe", [1, 2, CPE])
@pytest.mark.parametrize("nsb", [0, 1, 2, 5, 8, 13, 571, 578])
@pytest.mark.parametrize("n_chunks", [1, 2, 7, 15, 16, 17, 31, 33, 977])
def test_chunk_order_is_a_bijection(cpe, nsb, n_chunks):
    g = spmv_grid(nsb, n_chunks, cpe)
    got = [chunk_of_block(b - nsb, nsb, n_chunks, cpe) for b in range(nsb, g)]
    real = sorted(c for c in got if c >= 0)
    assert real == list(range(n_chunks))
    assert len(got) - len(real) < 8 * cpe  # padding stays below one group


@pytest.mark.parametrize("cpe", [1, 2, CPE])
@pytest.mark.parametrize("nsb", [0, 3, 571])
def test_chunk_order_is_xcd_affine(cpe, nsb):
    n_chunks = 977
    for b in range(nsb, spmv_grid(nsb, n_chunks, cpe)):
        c = chunk_of_block(b - nsb, nsb, n_chunks, cpe)
        if c >= 0:
            assert b % 8 == (c // cpe) % 8
