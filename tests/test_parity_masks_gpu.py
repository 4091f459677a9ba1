"""ReLU-decision parity: the gradients of the HIP path against the exact
gradients of the ReLU decisions the HIP path itself made.

A ReLU whose pre-activation lies within fp32 rounding of zero can go either
way in any fp32 summation order, and that element's whole delta then enters
(or leaves) the weight gradients (src/kernel/layer_deltas.cl:72-77, :112;
backpropagate.cl:89-106).  The other parity tests excuse such flips with an
absolute floor (hip_util.FLIP_FLOOR).  Here no floor is used: the HIP path's
own A1 / A2 / A3 (srcnn_train_activations) give the masks, the double-precision
oracle recomputes the step under those masks
(oracle_train_fwd_bwd_masked), and every gradient element must match that
exact result within max(1e-4, 4 x the fp32 oracle's own error under the same
masks) -- the elementwise bound of hip_util.assert_close with abs_floor = 0.
Elements that cancel (the sum of their terms' magnitudes far above the
result) may instead lie within 0.25 x Higham's probabilistic rounding
estimate of an fp32 sum of their terms (hip_util.K_ROUND; an estimate, not a
bound), and at most a handful per array may pass by that clause alone
(hip_util.MAX_ROUND_ONLY), so an accumulation regression cannot hide there.

Each flip is also checked to be a genuine rounding case: its exact
pre-activation lies within AMBIG x (sum of the absolute values of its terms)
of zero.  The last layer's ReLU' (the quirk of last_layer_delta.cl:45) is taken from
the HIP path's A3 the same way.

For the wide batch of 64 distinct tiles x 64 copies the yardstick of the
reference algorithm's own error is the reference's sequential fp32 sum of
4096 per-sample partial gradients (backpropagate.cl:110's order, the oracle's
order), formed from the exact per-sample partials rounded to fp32 -- not the
oracle's 64-tile sum times 64, whose error is that of 64 terms.
"""
import numpy as np
import pytest

import srcnn_oracle as orc
from hip_util import RTOL, assert_close, log_record, make_batch, make_params

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

NETS = {"default": (64, 32, 9, 1, 5), "example": (32, 16, 9, 1, 5), "wide": (128, 64, 9, 5, 5)}
# a decision is ambiguous when |exact pre-activation| <= AMBIG x sum |terms|:
# far above fp32's unit roundoff times the term count of any layer here
# (<= 3201 terms x 6e-8 = 2e-4 worst case, ~1e-6 typical), far below the
# activations' own spread
AMBIG = 1e-5


@pytest.fixture(scope="module")
def S():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import srcnn_amd
    return srcnn_amd


def D(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()


def H(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def dims(cfg, w, h):
    n1, n2, f1, f2, f3 = cfg
    w1, h1 = w - f1 + 1, h - f1 + 1
    w2, h2 = w1 - f2 + 1, h1 - f2 + 1
    return w1, h1, w2, h2, w2 - f3 + 1, h2 - f3 + 1


def hip_step(S, cfg, X, T, w, h, batch, params, g0):
    """srcnn_train_fwd_bwd, then the activations it left in the workspace."""
    net = S.Net(*cfg)
    w1, h1, w2, h2, _, _ = dims(cfg, w, h)
    nbytes = S.train_workspace_bytes(net, w, h, batch)
    ws = torch.empty(nbytes // 4 + 64, dtype=torch.float32, device="cuda")
    g = D(g0)
    S.train_fwd_bwd(net, D(X), D(T), w, h, batch, D(params), g, None, ws, nbytes)
    path = S.last_path()
    w3, h3 = dims(cfg, w, h)[4:]
    A1 = torch.empty(batch * w1 * h1 * cfg[0], dtype=torch.float32, device="cuda")
    A2 = torch.empty(batch * w2 * h2 * cfg[1], dtype=torch.float32, device="cuda")
    A3 = torch.empty(batch * w3 * h3, dtype=torch.float32, device="cuda")
    S.train_activations(net, w, h, batch, ws, nbytes, A1, A2, A3)
    return H(g), H(A1), H(A2), H(A3), path


def split(cfg, params):
    n1, n2, f1, f2, f3 = cfg
    sizes = [f1 * f1 * n1, n1, f2 * f2 * n1 * n2, n2, f3 * f3 * n2, 1]
    out, o = [], 0
    for s in sizes:
        out.append(params[o:o + s])
        o += s
    return out


def decisions(cfg, X, w, h, batch, params, A1m):
    """Exact (f64) pre-activations of layers 1 and 2 and the sums of the
    absolute values of their terms; layer 2 is fed the masked exact A1."""
    n1, n2, f1, f2, f3 = cfg
    W1, B1, W2, B2, W3, B3 = split(cfg, np.asarray(params, np.float64))
    w1, h1, w2, h2, _, _ = dims(cfg, w, h)
    F = orc.f64
    pre1 = F.conv_fwd(X, W1, B1, w, h, 1, n1, f1, 0, batch)
    mag1 = F.conv_fwd(np.abs(X), np.abs(W1), np.abs(B1), w, h, 1, n1, f1, 0, batch)
    pre2 = F.conv_fwd(A1m, W2, B2, w1, h1, n1, n2, f2, 0, batch)
    mag2 = F.conv_fwd(np.abs(A1m), np.abs(W2), np.abs(B2), w1, h1, n1, n2, f2, 0, batch)
    return pre1, mag1, pre2, mag2


def check_flips(what, mask, pre, mag):
    """Every HIP decision that differs from the exact one is a rounding case."""
    exact = pre > 0
    flips = mask != exact
    amb = np.abs(pre) <= AMBIG * mag
    n_flip, n_amb = int(flips.sum()), int(amb.sum())
    bad = int((flips & ~amb).sum())
    assert bad == 0, "%s: %d ReLU decisions differ from the exact sign outside the rounding band" % (what, bad)
    return n_flip, n_amb


def sample_partials(cfg, X, w, h, batch, acts):
    """Exact (f64) per-sample partial gradients [batch][P] from the masked
    oracle's activations (A1|A2|A3|D3|D2|D1): backpropagate.cl:89-106 per
    sample, before the cross-sample sum of :110."""
    from numpy.lib.stride_tricks import sliding_window_view as win
    n1, n2, f1, f2, f3 = cfg
    w1, h1, w2, h2, w3, h3 = dims(cfg, w, h)
    s1, s2, s3 = w1 * h1 * n1, w2 * h2 * n2, w3 * h3
    o = np.cumsum([0, s1 * batch, s2 * batch, s3 * batch, s3 * batch, s2 * batch, s1 * batch])
    A1 = acts[o[0]:o[1]].reshape(batch, h1, w1, n1)
    A2 = acts[o[1]:o[2]].reshape(batch, h2, w2, n2)
    D3 = acts[o[3]:o[4]].reshape(batch, h3, w3, 1)
    D2 = acts[o[4]:o[5]].reshape(batch, h2, w2, n2)
    D1 = acts[o[5]:o[6]].reshape(batch, h1, w1, n1)
    Xs = np.asarray(X, np.float64).reshape(batch, h, w, 1)

    def grad(inp, d, f):  # [batch][f][f][n_prev][n_cur], [batch][n_cur]
        oh, ow = d.shape[1], d.shape[2]
        v = win(inp, (oh, ow), axis=(1, 2))  # [b][f][f][n_prev][oh][ow]
        gw = np.einsum("bijkyx,byxn->bijkn", v, d, optimize=True)
        return gw.reshape(batch, -1), d.sum(axis=(1, 2))
    parts = []
    for inp, d, f in ((Xs, D1, f1), (A1, D2, f2), (A2, D3, f3)):
        gw, gb = grad(inp, d, f)
        parts += [gw, gb]
    return np.concatenate(parts, axis=1)


def sequential_f32_sum(partials, rep, g0):
    """fp32 g0 + p_0 + p_1 + ... over rep copies of the batch, in sample order."""
    p32 = partials.astype(np.float32)
    acc = np.asarray(g0, np.float32).copy()
    for _ in range(rep):
        for row in p32:
            acc += row
    return acc


def masked_parity(S, cfg, name, X, T, w, h, batch, params, g0, rep=1):
    """The HIP step on `rep` copies of the batch against the masked oracles on
    one copy (the copies must make identical decisions)."""
    n1, n2, f1, f2, f3 = cfg
    w1, h1, w2, h2, w3, h3 = dims(cfg, w, h)
    Xb, Tb = (np.tile(X, rep), np.tile(T, rep)) if rep > 1 else (X, T)
    got, A1, A2, A3h, path = hip_step(S, cfg, Xb, Tb, w, h, batch * rep, params, g0)
    m1, m2, m3 = A1 > 0, A2 > 0, A3h > 0
    if rep > 1:
        ms = [m.reshape(rep, -1) for m in (m1, m2, m3)]
        assert all((m == m[0]).all() for m in ms), "copies made different decisions"
        m1, m2, m3 = (m[0] for m in ms)
    zero = np.zeros_like(g0, dtype=np.float64)
    # exact gradients of the HIP path's decisions
    xg_m, xacts = orc.f64.train_fwd_bwd_masked(cfg, X, T, w, h, batch, params, zero, m1, m2, m3,
                                               want_acts=True)
    assert np.abs(xg_m).max() > 0, "degenerate case: every gradient is zero"
    xg_m = rep * xg_m + g0
    # every differing decision lies in the rounding band of its exact value
    s1, s2, s3 = batch * w1 * h1 * n1, batch * w2 * h2 * n2, batch * w3 * h3
    pre1, mag1, pre2, mag2 = decisions(cfg, X, w, h, batch, params, xacts[:s1])
    W1, B1, W2, B2, W3, B3 = split(cfg, np.asarray(params, np.float64))
    pre3 = xacts[s1 + s2:s1 + s2 + s3]
    mag3 = orc.f64.conv_fwd(np.abs(xacts[s1:s1 + s2]), np.abs(W3), np.abs(B3), w2, h2, n2, 1, f3, 0, batch)
    flips = [check_flips("%s A%d" % (name, k + 1), m, p, mg)
             for k, (m, p, mg) in enumerate(((m1, pre1, mag1), (m2, pre2, mag2), (m3, pre3, mag3)))]
    rec = {"what": "relu decisions %s b%d x%d" % (name, batch, rep), "path": path}
    for k, (nf, na) in enumerate(flips):
        rec["flips_A%d" % (k + 1)] = nf * rep
        rec["ambiguous_A%d" % (k + 1)] = na * rep
    log_record(rec)
    # the reference algorithm's own fp32 result under the same decisions
    if rep == 1:
        ref32, _ = orc.train_fwd_bwd_masked(cfg, X, T, w, h, batch, params, g0, m1, m2, m3)
    else:
        ref32 = sequential_f32_sum(sample_partials(cfg, X, w, h, batch, xacts), rep, g0)
    mag, nterms = term_magnitudes(cfg, X, w, h, batch, xacts, rep, g0)
    off = np.cumsum([0] + [p.size for p in split(cfg, params)])
    for i, nm in enumerate(["W1", "B1", "W2", "B2", "W3", "B3"]):
        sl = slice(off[i], off[i + 1])
        assert_close(got[sl], ref32[sl], RTOL, "%s masked grad %s (%s, b%d x%d)" % (name, nm, path, batch, rep),
                     xg_m[sl], abs_floor=0.0, mag=mag[sl], nterms=nterms[i // 2])
    return flips


def term_magnitudes(cfg, X, w, h, batch, xacts, rep, g0):
    """Per gradient element, the sum of the absolute values of its terms
    (backpropagate.cl:104 / :94 over pixels and the rep x batch samples, plus
    the accumulated g0) and, per layer, the number of those terms."""
    n1, n2, f1, f2, f3 = cfg
    w1, h1, w2, h2, w3, h3 = dims(cfg, w, h)
    s1, s2, s3 = batch * w1 * h1 * n1, batch * w2 * h2 * n2, batch * w3 * h3
    o = np.cumsum([0, s1, s2, s3, s3, s2, s1])
    A1, A2 = np.abs(xacts[o[0]:o[1]]), np.abs(xacts[o[1]:o[2]])
    D3, D2, D1 = np.abs(xacts[o[3]:o[4]]), np.abs(xacts[o[4]:o[5]]), np.abs(xacts[o[5]:o[6]])
    F = orc.f64
    parts = []
    for inp, d, npv, ncu, f, ow, oh in ((np.abs(np.asarray(X, np.float64)), D1, 1, n1, f1, w1, h1),
                                        (A1, D2, n1, n2, f2, w2, h2), (A2, D3, n2, 1, f3, w3, h3)):
        gw, gb = F.conv_grad_acc(inp, d, np.zeros(f * f * npv * ncu), np.zeros(ncu), npv, ncu, f, ow, oh, batch)
        parts += [gw, gb]
    mag = rep * np.concatenate(parts) + np.abs(np.asarray(g0, np.float64))
    nterms = [rep * batch * w1 * h1 + 1, rep * batch * w2 * h2 + 1, rep * batch * w3 * h3 + 1]
    return mag, nterms


@pytest.mark.parametrize("path", [0, 1], ids=["auto", "generic"])
@pytest.mark.parametrize("name,batch,size", [("default", 513, 33), ("default", 600, 33),
                                             ("example", 257, 33), ("default", 65, 36)])
def test_gradients_under_hip_relu_decisions(S, path, name, batch, size):
    """test_train_step_vs_oracle's inputs (seed 42, weights N(0, 0.05), an
    accumulated g0) without FLIP_FLOOR."""
    cfg = NETS[name]
    rng = np.random.default_rng(42)
    X, T = make_batch(rng, batch, size, size)
    params = make_params(rng, cfg, sd=0.05)
    g0 = (1e-3 * rng.standard_normal(params.size)).astype(np.float32)
    S.set_path(path)
    try:
        masked_parity(S, cfg, name, X, T, size, size, batch, params, g0)
    finally:
        S.set_path(0)


def test_full_batch_gradients_under_hip_relu_decisions(S):
    """BASELINE.json configs[1] at its own size: 4096 tiles, no floor."""
    cfg = NETS["default"]
    rng = np.random.default_rng(2024)
    X, T = make_batch(rng, 4096, 33, 33)
    params = make_params(rng, cfg, sd=0.05)
    masked_parity(S, cfg, "default", X, T, 33, 33, 4096, params, np.zeros(params.size, np.float32))


def test_wide_gradients_under_hip_relu_decisions(S):
    cfg = NETS["wide"]
    rng = np.random.default_rng(11)
    X, T = make_batch(rng, 300, 33, 33)
    params = make_params(rng, cfg, sd=0.05)
    g0 = (1e-3 * rng.standard_normal(params.size)).astype(np.float32)
    masked_parity(S, cfg, "wide", X, T, 33, 33, 300, params, g0)


def test_wide_batch_4096_gradients_under_hip_relu_decisions(S):
    """BASELINE.json configs[3] at its own size: 64 distinct tiles x 64 copies
    (test_wide_gpu.test_wide_full_batch_4096_vs_oracle's inputs), no floor."""
    cfg = NETS["wide"]
    rng = np.random.default_rng(4096)
    X, T = make_batch(rng, 64, 33, 33)
    params = make_params(rng, cfg, sd=0.05)
    masked_parity(S, cfg, "wide", X, T, 33, 33, 64, params, np.zeros(params.size, np.float32), rep=64)
