"""CPU checks of oracle_train_fwd_bwd_masked (the f64 yardstick of
tests/test_parity_masks_gpu.py)."""
import numpy as np

import srcnn_oracle as orc
from hip_util import make_batch, make_params

CFG = (64, 32, 9, 1, 5)


def _case(batch=3, size=21, seed=1):
    rng = np.random.default_rng(seed)
    X, T = make_batch(rng, batch, size, size)
    params = make_params(rng, CFG, sd=0.05)
    return X, T, params


def _masks(acts, batch, size):
    n1, n2, f1, f2, f3 = CFG
    w1 = size - f1 + 1
    w2 = w1 - f2 + 1
    w3 = w2 - f3 + 1
    s1, s2, s3 = batch * w1 * w1 * n1, batch * w2 * w2 * n2, batch * w3 * w3
    return acts[:s1] > 0, acts[s1:s1 + s2] > 0, acts[s1 + s2:s1 + s2 + s3] > 0, s1, s2


def test_own_masks_reproduce_the_plain_step_bit_for_bit():
    X, T, params = _case()
    for O in (orc.ORACLE, orc.f64):
        g0 = np.linspace(-1e-3, 1e-3, params.size)
        g, acts = O.train_fwd_bwd(CFG, X, T, 21, 21, 3, params, g0, want_acts=True)
        m1, m2, m3, _, _ = _masks(acts, 3, 21)
        gm, acts_m = O.train_fwd_bwd_masked(CFG, X, T, 21, 21, 3, params, g0, m1, m2, m3, want_acts=True)
        np.testing.assert_array_equal(gm, g)
        np.testing.assert_array_equal(acts_m, acts)


def test_all_off_layer1_decisions():
    """m1 = 0 everywhere: A1 = 0 and delta1 = 0, so gW1 = gB1 = gW2 = 0, and
    every layer-2 unit the mask keeps on outputs exactly its bias B2."""
    X, T, params = _case(batch=2)
    n1, n2 = CFG[0], CFG[1]
    g, acts = orc.f64.train_fwd_bwd(CFG, X, T, 21, 21, 2, params, np.zeros(params.size), want_acts=True)
    m1, m2, m3, s1, s2 = _masks(acts, 2, 21)
    gm, am = orc.f64.train_fwd_bwd_masked(CFG, X, T, 21, 21, 2, params, np.zeros(params.size),
                                          np.zeros_like(m1), np.ones_like(m2), m3, want_acts=True)
    nw1, nw2 = 81 * n1, n1 * n2
    assert not gm[:nw1 + n1 + nw2].any()
    assert not am[:s1].any() and not am[-s1:].any()
    B2 = params[nw1 + n1 + nw2:nw1 + n1 + nw2 + n2]
    np.testing.assert_array_equal(am[s1:s1 + s2].reshape(-1, n2), np.broadcast_to(B2, (s2 // n2, n2)))


def test_last_layer_mask_switches_the_quirk():
    """m3 = 1 everywhere turns the relu' quirk of last_layer_delta.cl:45 off:
    delta3 = A3 - T on every pixel (the plain squared-error gradient)."""
    X, T, params = _case(batch=1)
    g, acts = orc.f64.train_fwd_bwd(CFG, X, T, 21, 21, 1, params, np.zeros(params.size), want_acts=True)
    m1, m2, m3, s1, s2 = _masks(acts, 1, 21)
    _, am = orc.f64.train_fwd_bwd_masked(CFG, X, T, 21, 21, 1, params, np.zeros(params.size), m1, m2,
                                         np.ones_like(m3), want_acts=True)
    s3 = m3.size
    A3, D3 = am[s1 + s2:s1 + s2 + s3], am[s1 + s2 + s3:s1 + s2 + 2 * s3]
    pad = (21 - 9) // 2
    Tc = T.reshape(21, 21)[pad:21 - pad, pad:21 - pad].ravel()
    np.testing.assert_array_equal(D3, A3 - Tc.astype(np.float64))
