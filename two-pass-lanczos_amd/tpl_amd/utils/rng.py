"""``StdRng::seed_from_u64(seed)`` + ``rng.random::<f64>()`` of rand 0.9 (ChaCha12),
used by the experiment harness to draw the same b as the reference's binaries
(src/bin/stability.rs:257-258, src/bin/orthogonality.rs:163-164).

Pinned crates (Cargo.lock): rand 0.9.2, rand_core 0.9.3, rand_chacha 0.9.0.
seed_from_u64: 8 PCG32 outputs -> the 32-byte key; ChaCha12 with a 64-bit block
counter (words 12-13) and zero stream; next_u64 = (w[2i+1] << 32) | w[2i];
f64 = (u64 >> 11) * 2^-53. b[0..4] = 0.52655741, 0.54272521, 0.6364651, 0.40590176.
"""
from __future__ import annotations

import numpy as np

_M64 = (1 << 64) - 1
_M32 = 0xFFFFFFFF
_SIGMA = np.array([0x61707865, 0x3320646E, 0x79622D32, 0x6B206574], dtype=np.uint32)


def _key(seed: int) -> np.ndarray:
    words, st = [], seed & _M64
    for _ in range(8):
        st = (st * 6364136223846793005 + 11634580027462260723) & _M64
        xs = (((st >> 18) ^ st) >> 27) & _M32
        r = st >> 59
        words.append(((xs >> r) | (xs << ((32 - r) & 31))) & _M32)
    return np.array(words, dtype=np.uint32)


def _blocks(key: np.ndarray, nblocks: int) -> np.ndarray:
    """ChaCha12 keystream of blocks 0 .. nblocks-1, flattened block by block."""
    s = np.zeros((16, nblocks), dtype=np.uint32)
    s[0:4] = _SIGMA[:, None]
    s[4:12] = key[:, None]
    ctr = np.arange(nblocks, dtype=np.uint64)
    s[12] = (ctr & np.uint64(_M32)).astype(np.uint32)
    s[13] = (ctr >> np.uint64(32)).astype(np.uint32)
    x = s.copy()

    def rotl(v, r):
        return (v << np.uint32(r)) | (v >> np.uint32(32 - r))

    def quarter(a, b, c, d):
        x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 16)
        x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 12)
        x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 8)
        x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 7)

    with np.errstate(over="ignore"):
        for _ in range(6):  # 12 rounds = 6 double rounds
            for q in ((0, 4, 8, 12), (1, 5, 9, 13), (2, 6, 10, 14), (3, 7, 11, 15),
                      (0, 5, 10, 15), (1, 6, 11, 12), (2, 7, 8, 13), (3, 4, 9, 14)):
                quarter(*q)
        x += s
    return x.T.reshape(-1)


def std_rng_f64(n: int, seed: int = 42) -> np.ndarray:
    """``Mat::from_fn(n, 1, |_, _| rng.random())`` after ``StdRng::seed_from_u64(seed)``."""
    w = _blocks(_key(seed), (2 * n + 15) // 16)[:2 * n].astype(np.uint64)
    u = w[0::2] | (w[1::2] << np.uint64(32))
    return (u >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
