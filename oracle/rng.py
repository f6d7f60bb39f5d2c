"""Restatement of the reference's random vectors — TEST INFRASTRUCTURE (oracle).

The reference draws b with ``StdRng::seed_from_u64(42)`` and
``Mat::from_fn(n, 1, |_, _| rng.random())`` (tests/correctness.rs:109-110,
src/bin/stability.rs:257-258, src/algorithms/mod.rs:439-440). Pinned crates
(Cargo.lock): rand 0.9.2, rand_core 0.9.3, rand_chacha 0.9.0 — not vendored, so
this follows their published algorithms:

* ``SeedableRng::seed_from_u64`` (rand_core 0.9): 8 rounds of PCG32
  (state = state * 6364136223846793005 + 11634580027462260723; xorshifted =
  ((state >> 18) ^ state) >> 27; rotate right by state >> 59), little-endian
  words -> the 32-byte ChaCha key.
* ``StdRng`` = ChaCha12 (rand_chacha): constants "expand 32-byte k", 64-bit block
  counter in words 12-13 starting at 0, stream words 14-15 = 0, 6 double rounds,
  feed-forward add; keystream words consumed in order.
* ``next_u64`` = (w[2i+1] << 32) | w[2i]; ``random::<f64>()`` = (u64 >> 11) * 2^-53.

Pinned by tests/test_oracle_golden.py against the published results/accuracy_*.csv
(which depend on every entry of b) — b[0..4] = 0.52655741, 0.54272521, 0.6364651,
0.40590176.
"""
from __future__ import annotations

import numpy as np

_M64 = (1 << 64) - 1
_M32 = 0xFFFFFFFF


def _seed_words(state: int) -> list[int]:
    out = []
    for _ in range(8):
        state = (state * 6364136223846793005 + 11634580027462260723) & _M64
        xs = (((state >> 18) ^ state) >> 27) & _M32
        rot = state >> 59
        out.append(((xs >> rot) | (xs << ((32 - rot) & 31))) & _M32)
    return out


def _rotl(x, r):
    return (x << np.uint32(r)) | (x >> np.uint32(32 - r))


def _chacha12_blocks(key: list[int], first_block: int, nblocks: int) -> np.ndarray:
    """Keystream words of blocks [first_block, first_block + nblocks), shape (nblocks*16,)."""
    ctr = np.arange(first_block, first_block + nblocks, dtype=np.uint64)
    init = np.zeros((16, nblocks), dtype=np.uint32)
    init[0:4] = np.array([0x61707865, 0x3320646E, 0x79622D32, 0x6B206574], dtype=np.uint32)[:, None]
    init[4:12] = np.array(key, dtype=np.uint32)[:, None]
    init[12] = (ctr & np.uint64(_M32)).astype(np.uint32)
    init[13] = (ctr >> np.uint64(32)).astype(np.uint32)
    x = [init[i].copy() for i in range(16)]

    def qr(a, b, c, d):
        x[a] += x[b]; x[d] ^= x[a]; x[d] = _rotl(x[d], 16)
        x[c] += x[d]; x[b] ^= x[c]; x[b] = _rotl(x[b], 12)
        x[a] += x[b]; x[d] ^= x[a]; x[d] = _rotl(x[d], 8)
        x[c] += x[d]; x[b] ^= x[c]; x[b] = _rotl(x[b], 7)

    with np.errstate(over="ignore"):
        for _ in range(6):
            qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
            qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
        out = np.stack(x) + init
    return out.T.reshape(-1)  # block-major: block0 words 0..15, block1, ...


class StdRng:
    """rand 0.9 StdRng (ChaCha12) restated for f64 draws."""

    def __init__(self, seed: int):
        self.key = _seed_words(seed & _M64)
        self.word = 0  # next keystream word index

    def random_f64(self, n: int) -> np.ndarray:
        if self.word % 2:
            raise NotImplementedError("odd word offset (mixed u32/u64 draws) not needed here")
        nwords = 2 * n
        first_block = self.word // 16
        off = self.word % 16
        nblocks = (off + nwords + 15) // 16
        w = _chacha12_blocks(self.key, first_block, nblocks)[off:off + nwords].astype(np.uint64)
        self.word += nwords
        u = w[0::2] | (w[1::2] << np.uint64(32))
        return (u >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def std_rng_vector(n: int, seed: int = 42) -> np.ndarray:
    """``Mat::from_fn(n, 1, |_, _| rng.random())`` with ``StdRng::seed_from_u64(seed)``."""
    return StdRng(seed).random_f64(n)
