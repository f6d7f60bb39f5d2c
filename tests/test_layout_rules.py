"""CPU checks of layout rules the kernels rely on (restated from the device code).

* chunk_of_block (two-pass-lanczos_amd/csrc/tpl_kcommon.h): the XCD-affine order of the
  chunk part of an SpMV grid is a bijection onto the chunks (padding blocks map to -1),
  whatever the number of bin blocks in front of it — correctness never depends on the
  placement it aims for.
* the placement it aims for: with block b on XCD b % 8, chunk c lands on XCD (c // 2) % 8,
  the XCD of element-wise block c // 2 (E = 1024 rows = two 512-row chunks).
"""
import pytest


def chunk_of_block(i, n_slice_blocks, n_chunks):
    x = ((i & 7) + n_slice_blocks) & 7
    c = (i >> 4) * 16 + 2 * x + ((i >> 3) & 1)
    return c if c < n_chunks else -1


def spmv_grid(n_slice_blocks, n_chunks):
    return n_slice_blocks + (n_chunks + 15) // 16 * 16


@pytest.mark.parametrize("nsb", [0, 1, 2, 5, 8, 13, 571, 578])
@pytest.mark.parametrize("n_chunks", [1, 2, 7, 15, 16, 17, 31, 977])
def test_chunk_order_is_a_bijection(nsb, n_chunks):
    g = spmv_grid(nsb, n_chunks)
    got = [chunk_of_block(b - nsb, nsb, n_chunks) for b in range(nsb, g)]
    real = sorted(c for c in got if c >= 0)
    assert real == list(range(n_chunks))
    assert len(got) - len(real) < 16  # padding stays below one 16-block group


@pytest.mark.parametrize("nsb", [0, 3, 571])
def test_chunk_order_is_xcd_affine(nsb):
    n_chunks = 977
    for b in range(nsb, spmv_grid(nsb, n_chunks)):
        c = chunk_of_block(b - nsb, nsb, n_chunks)
        if c >= 0:
            assert b % 8 == (c // 2) % 8
