"""CPU: the device exp(T_k) e_1 algorithm (tpl_kernels.hip k_ftk_exp), restated in numpy
(oracle/ftk_ref.py exp_chebyshev), against LAPACK's EVD (the reference's method,
src/bin/stability.rs:175-193). Tolerance stated in tests/test_gpu_device_exp.py: for every
case the algorithm keeps (it hands ||y|| < 1e-3 exp(lambda_max) back to the host),
||y - y_evd|| <= 1e-11 ||y|| and <= 1e-12 exp(lambda_max)."""
import numpy as np
import pytest
from scipy.linalg import eigvalsh_tridiagonal

from conftest import harness_b, load_kkt

import oracle
from oracle import ftk_ref


def check(al, be):
    y = ftk_ref.exp_chebyshev(al, be)
    if y is None:
        return False
    yr = ftk_ref.exp(al, be)
    lm = float(eigvalsh_tridiagonal(al, be[:len(al) - 1])[-1]) if len(al) > 1 else float(al[0])
    err = np.linalg.norm(y - yr)
    assert err <= 1e-11 * np.linalg.norm(yr), (err, np.linalg.norm(yr))
    assert err <= 1e-12 * np.exp(lm)
    return True


@pytest.mark.parametrize("k", [1, 2, 3, 10, 60, 200])
def test_restatement_vs_evd(k):
    rng = np.random.default_rng(k)
    kept = 0
    for al, be in ((np.zeros(k), rng.uniform(0.5, 20.0, k - 1)),
                   (rng.standard_normal(k) * 5.0, rng.uniform(0.01, 3.0, k - 1)),
                   (rng.uniform(-1000.0, -0.1, k), rng.uniform(0.0, 50.0, k - 1)),
                   (rng.uniform(-10.0, -0.1, k), rng.uniform(0.0, 1.0, k - 1))):
        kept += check(al, be)
    assert kept >= 1  # random T: e_1 is often far from the top of the spectrum


def test_restatement_hands_back():
    assert ftk_ref.exp_chebyshev(np.array([0.0, np.nan]), np.array([1.0])) is None
    assert ftk_ref.exp_chebyshev(np.array([-1e6, 1e6]), np.array([1.0])) is None


def test_restatement_on_config2_tk(kkt50k):
    """configs[1]'s own T_k (50k arcs, k = 200, the harness b, reference-order pass one):
    kept on the device, within 1e-14 of LAPACK (a 35-digit evaluation puts the expansion
    at 6e-16 and LAPACK at 4e-15 of the truth)."""
    a = kkt50k.a
    al, be, s, bn, _ = oracle.Operator(a).pass_one(harness_b(a), 200)
    y = ftk_ref.exp_chebyshev(al, be)
    assert y is not None
    yr = ftk_ref.exp(al, be)
    assert np.linalg.norm(y - yr) <= 1e-14 * np.linalg.norm(yr)
