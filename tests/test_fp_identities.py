"""CPU: the floating-point identities the kernels rely on to move work off dependent chains
without changing a bit (tpl_kcommon.h).

* x + (-0.0) == x bit for bit for every double x (signed zeros, subnormals, infinities;
  a NaN stays a NaN): the bins' piece sums and the chunks' row sums add -0.0 for entries
  past a piece's end / padding instead of selecting after the add.
* x + y == y + x bit for bit (IEEE addition is commutative): the DPP butterflies add a
  lane's value and its partner's in either order on the two lanes of a pair.
"""
import numpy as np


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.int64)


def _samples(rng, n):
    specials = np.array([0.0, -0.0, 5e-324, -5e-324, 2.2250738585072014e-308, 1e-310,
                         -1e-310, 1.0, -1.0, 1.7976931348623157e308, -1.7976931348623157e308,
                         np.inf, -np.inf])
    x = rng.standard_normal(n) * 10.0 ** rng.integers(-320, 300, n)
    return np.concatenate([specials, x])


def test_adding_negative_zero_is_the_identity():
    x = _samples(np.random.default_rng(11), 200000)
    y = x + (-0.0)
    assert np.array_equal(_bits(y), _bits(x))
    nan = np.array([np.nan])
    assert np.isnan(nan + (-0.0))[0]


def test_addition_commutes_bitwise():
    rng = np.random.default_rng(12)
    x, y = _samples(rng, 100000), _samples(rng, 100000)
    with np.errstate(invalid="ignore", over="ignore"):
        a, b = x + y, y + x
    ok = ~np.isnan(a)
    assert np.array_equal(np.isnan(a), np.isnan(b))
    assert np.array_equal(_bits(a[ok]), _bits(b[ok]))
