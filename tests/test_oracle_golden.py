"""Pin the CPU oracle against the reference's own golden vectors.

Every fixture comes from the reference test suite (tests/golden/make_golden.py
lists the source file:line of each).  Tolerances follow the precision the
reference printed its expected values with (3 or 4 decimals), NOT the
reference's one-sided compare (test/TestCase.cpp:48-62): every check here
is two-sided.
"""
import json
import os

import numpy as np
import pytest

import srcnn_oracle as orc

from conftest import GOLDEN


def load(name):
    with open(os.path.join(GOLDEN, name)) as fh:
        return json.load(fh)


@pytest.mark.parametrize("case", sorted(load("layer_test_cases.json").keys()))
def test_layer_forward_test_cases(case):
    """test/specs/LayerTest.cpp:97-130 on test/data/test_cases.json (ReLU on)."""
    d = load("layer_test_cases.json")[case]
    out = orc.conv_fwd(d["input"], d["weights"], d["bias"], d["input_w"], d["input_h"],
                       d["n_prev_filter_cnt"], d["current_filter_count"], d["f_spatial_size"],
                       True, 1)
    np.testing.assert_allclose(out, np.array(d["output"], np.float32), rtol=0, atol=5e-4)


def test_layer_deltas_spec():
    """test/specs/LayerDeltasTest.cpp:141-193: prev output = relu(input_x)."""
    d = load("layer_deltas.json")
    y = np.maximum(np.array(d["input_x"], np.float32), 0)
    out = orc.conv_delta(d["deltas"], y, d["weights"], d["f_next"], d["n_prev_layer"], d["n_next"],
                         d["curr_w"], d["curr_h"], 1)
    np.testing.assert_allclose(out, np.array(d["expected"], np.float32), rtol=0, atol=2e-6)


def test_backpropagation_spec():
    """test/specs/BackpropagationTest.cpp:135-159: grad_w init 1.5, grad_b init 0."""
    d = load("backprop.json")
    gW0 = np.full(54, d["grad_w_init"], np.float32)
    gB0 = np.zeros(3, np.float32)
    out_w = d["in_w"] - d["f"] + 1
    gW, gB = orc.conv_grad_acc(d["input"], d["deltas"], gW0, gB0, d["n_prev"], d["n_cur"], d["f"],
                               out_w, out_w, 1)
    np.testing.assert_allclose(gW, np.array(d["expected_grad_w"], np.float32), rtol=0, atol=6e-5)
    np.testing.assert_allclose(gB, np.array(d["expected_grad_b"], np.float32), rtol=0, atol=6e-4)


def test_update_parameters_spec():
    """test/specs/UpdateParametersTest.cpp:65-105 (fixed seed instead of the clock)."""
    rng = np.random.default_rng(1234)
    n_prev, n_cur, f, batch = 2, 400, 5, 2
    momentum, lr = np.float32(0.8), np.float32(0.001)
    for size in (f * f * n_prev * n_cur, n_cur):
        cur = (rng.integers(0, 2560, size) / 10.0).astype(np.float32)
        grad = (rng.integers(0, 2560, size) / 100.0).astype(np.float32)
        prev = (rng.integers(0, 2560, size) / 10.0).astype(np.float32)
        deltas = momentum * prev + lr * grad                       # :35
        expected = cur - deltas / np.float32(batch)                 # :36
        W, B, dW, dB = orc.sgd_update(cur, cur[:1], grad, grad[:1], prev, prev[:1], 0.8, 0.0, 0.001, batch)
        np.testing.assert_allclose(W, expected, rtol=1e-6, atol=1e-4)
        np.testing.assert_allclose(dW, deltas, rtol=1e-6, atol=1e-4)


def test_last_layer_delta_spec():
    """test/specs/LastLayerDeltaTest.cpp:34-83: 6x6 algo result, padding 4."""
    rng = np.random.default_rng(7)
    algo_w = algo_h = 6
    pad = 4
    gw, gh = algo_w + 2 * pad, algo_h + 2 * pad
    gt = np.full(gw * gh, 99999.0, np.float32)
    algo = np.zeros(algo_w * algo_h, np.float32)
    exp = np.zeros_like(algo)
    for i in range(algo_w * algo_h):
        r, c = divmod(i, algo_w)
        t = np.float32(rng.integers(0, 256) / 100.0)
        x = np.float32(rng.integers(0, 2560) / 1000.0) - np.float32(1.28)   # both ReLU branches
        y = max(x, np.float32(0))
        exp[i] = (y - t) * (1.0 if x > 0 else 0.0)                          # :64
        gt[(r + pad) * gw + pad + c] = t
        algo[i] = y
    out = orc.last_delta(gt, algo, gw, gh, algo_w, algo_h, 1)
    np.testing.assert_array_equal(out, exp)


def test_squared_error_spec():
    """test/specs/SquaredErrorTest.cpp:31-82: 1000x2000, padding 4."""
    rng = np.random.default_rng(3)
    aw, ah, pad = 1000, 2000, 4
    gw, gh = aw + 2 * pad, ah + 2 * pad
    gt = np.full((gh, gw), 99999.0, np.float32)
    gt[pad:pad + ah, pad:pad + aw] = rng.integers(0, 256, (ah, aw))
    algo = (rng.integers(0, 2560, (ah, aw)) / 10.0).astype(np.float32)
    d = gt[pad:pad + ah, pad:pad + aw].astype(np.float64) - algo
    expected = float(np.sum(d * d))
    got = orc.sq_err(gt.ravel(), algo.ravel(), gw, gh, aw, ah, 1)
    assert abs(got - expected) <= 1e-6 * expected


@pytest.mark.parametrize("squared", [False, True])
def test_sum_spec(squared):
    """test/specs/SumTest.cpp:27-58: 0..899, margin 20 (:47; the float result
    cannot hold 242595150 exactly)."""
    data = np.arange(900, dtype=np.float32)
    expected = sum(i * i if squared else i for i in range(900))
    assert orc.buf_sum(data, squared) == pytest.approx(expected, abs=20)


def test_subtract_from_all_spec():
    """test/specs/SubtractFromAllTest.cpp:27-50."""
    data = np.arange(900, dtype=np.float32)
    np.testing.assert_array_equal(orc.sub_from_all(data, 450.0), data - 450.0)


@pytest.mark.parametrize("normalize", [True, False])
def test_extract_luma_spec(normalize):
    """test/specs/ExtractLumaTest.cpp:50-74 on test/data/color_grid.png.
    The spec's expected values are hand-typed to 3 decimals and one of them is
    3.8e-3 off; the tolerance is the spec's own margin 0.005 (TestCase.cpp:51)."""
    d = load("extract_luma.json")
    exp = np.array(d["expected_normalized"], np.float32)
    if not normalize:
        exp = exp * 255
    out = orc.extract_luma(np.array(d["rgba"], np.uint8), d["w"], d["h"], normalize)
    np.testing.assert_allclose(out, exp, rtol=0, atol=5e-3 if normalize else 5e-3 * 255)


def test_swap_luma_spec():
    """test/specs/SwapLumaTest.cpp:39-90.  The reference decodes the input
    JPEG with stb_image, the fixture with PIL: 55 of 3072 channels differ by
    1 LSB outside the luma area (pure decoder difference) and 5 by 2 LSB
    inside it, so parity is bounded by 2 LSB on <=2.5% of the channels."""
    d = load("swap_luma.json")
    w, h, pad = d["w"], d["h"], d["padding"]
    lw, lh = w - 2 * pad, h - 2 * pad
    n = lw * lw                                              # :48 (luma_w * luma_w)
    new_luma = (np.arange(n, dtype=np.float32) * np.float32(1.0)) / np.float32(n)
    out = orc.swap_luma(np.array(d["rgba"], np.uint8), new_luma, w, h, lw, lh).astype(int)
    exp = np.array(d["expected_rgba"], np.uint8).reshape(-1, 4)[:, :3].reshape(-1).astype(int)
    diff = np.abs(out - exp)
    assert diff.max() <= 2
    assert np.count_nonzero(diff) <= 0.025 * diff.size


def test_train_step_matches_op_composition():
    """ConfigBasedDataPipeline.cpp:200-361: the orchestrated step equals the
    ops composed by hand, and one update moves params as update_parameters.cl."""
    cfg = (8, 4, 5, 1, 3)
    w = h = 13
    batch = 3
    rng = np.random.default_rng(0)
    P = orc.param_count(*cfg)
    params = (rng.standard_normal(P) * 0.1).astype(np.float32)
    X = rng.random(batch * w * h).astype(np.float32) - 0.5
    T = rng.random(batch * w * h).astype(np.float32)
    g, acts = orc.train_fwd_bwd(cfg, X, T, w, h, batch, params, np.zeros(P, np.float32), want_acts=True)
    # compose by hand
    n1, n2, f1, f2, f3 = cfg
    o = [0, f1 * f1 * n1]
    o += [o[1] + n1, o[1] + n1 + f2 * f2 * n1 * n2]
    o += [o[3] + n2, o[3] + n2 + f3 * f3 * n2]
    W1, B1 = params[o[0]:o[1]], params[o[1]:o[2]]
    W2, B2 = params[o[2]:o[3]], params[o[3]:o[4]]
    W3, B3 = params[o[4]:o[5]], params[o[5]:]
    w1, w2, w3 = w - f1 + 1, w - f1 - f2 + 2, w - f1 - f2 - f3 + 3
    A1 = orc.conv_fwd(X, W1, B1, w, h, 1, n1, f1, True, batch)
    A2 = orc.conv_fwd(A1, W2, B2, w1, w1, n1, n2, f2, True, batch)
    A3 = orc.conv_fwd(A2, W3, B3, w2, w2, n2, 1, f3, False, batch)
    np.testing.assert_array_equal(acts[:A1.size], A1)
    out = orc.forward(cfg, X, w, h, batch, params)
    np.testing.assert_array_equal(out, A3)
    D3 = orc.last_delta(T, A3, w, h, w3, w3, batch)
    D2 = orc.conv_delta(D3, A2, W3, f3, n2, 1, w2, w2, batch)
    D1 = orc.conv_delta(D2, A1, W2, f2, n1, n2, w1, w1, batch)
    gW1, gB1 = orc.conv_grad_acc(X, D1, np.zeros_like(W1), np.zeros_like(B1), 1, n1, f1, w1, w1, batch)
    np.testing.assert_array_equal(g[o[0]:o[1]], gW1)
    np.testing.assert_array_equal(g[o[1]:o[2]], gB1)
    mom = np.zeros(P, np.float32)
    p2, g2, m2 = orc.update_all(cfg, params, g, mom, 0.9, 1e-3, [1e-4, 1e-4, 1e-5], batch)
    assert not g2.any()
    lr = np.concatenate([np.full(o[2], 1e-4), np.full(o[4] - o[2], 1e-4), np.full(P - o[4], 1e-5)]).astype(np.float32)
    wd = np.zeros(P, np.float32)
    wd[o[0]:o[1]] = wd[o[2]:o[3]] = wd[o[4]:o[5]] = np.float32(1e-3)
    dw = lr * g + wd * params
    np.testing.assert_allclose(m2, dw, rtol=1e-6, atol=1e-12)
    np.testing.assert_allclose(p2, params - dw / np.float32(batch), rtol=1e-6, atol=1e-9)
