"""Helpers shared by the GPU tests: device buffers (torch, plumbing only),
tolerance checks, synthetic SRCNN inputs."""
import json
import os

import numpy as np

# fp32 tolerance of BASELINE.json's north_star ("outputs within 1e-4 rel of
# the reference"), checked two ways by assert_close:
#   normwise     every element within RTOL x (|ref| + max|ref|) of the fp32
#                oracle (the reference's loop nests and accumulation order)
#   elementwise  on every SIGNIFICANT element (|exact| >= SIG x max|exact|),
#                the relative error against the exact result -- the oracle's
#                double-precision build (oracle/srcnn_oracle_f64.c) -- must be
#                <= max(RTOL, K_REF x E), where E is the fp32 oracle's WORST
#                relative error over the significant elements of the same
#                array (one bound per array, not per element)
# The K_REF x E clause is for sums that cancel: a gradient element made of a
# few thousand terms can come out 1000x smaller than its terms, and there any
# two fp32 summation orders (the reference's sample-serial loop, the HIP
# path's blocked sums) differ by far more than 1e-4 of the element.  It is one
# bound per array on purpose: which cancelling element a given order happens
# to get right is luck, so the error one order makes at an element does not
# bound what another order makes there; the worst error of the reference's
# order over the array is the scale of the cancellation error it accepts.
# Gradients add an absolute floor of FLIP_FLOOR x max|exact|: a ReLU decision
# whose pre-activation lies within fp32 rounding of zero can go either way in
# any fp32 order, and the whole delta of that element then enters (or leaves)
# the weight gradients.  tests/test_parity_masks_gpu.py pins this floor: it
# recomputes the exact gradients under the HIP path's own ReLU decisions
# (oracle_train_fwd_bwd_masked) and checks them with no floor at all, and
# checks that every flipped decision lies inside the rounding band.
# A third, order-independent clause applies where the caller supplies the sum
# of the absolute values of each element's terms (mag) and their count n: an
# element is also within tolerance if its error is at most K_ROUND x U_ROUND x
# sqrt(n) x mag.  U_ROUND x sqrt(n) x mag is Higham's PROBABILISTIC estimate of
# the rounding error of an fp32 summation of those terms ("Accuracy and
# Stability of Numerical Algorithms", 2nd ed., 3.5 / 4.2: errors of random
# sign grow like sqrt(n)); it is not a bound -- the deterministic worst case
# is about (n - 1) x U_ROUND x mag.  K_ROUND = 0.25 keeps it well inside that
# estimate (the worst ratio measured in round 3 was 0.044 of the unscaled
# estimate).  It only matters where a sum cancels (mag >> |exact|), and a real
# accumulation regression must not hide behind it: at most MAX_ROUND_ONLY
# elements (or ROUND_ONLY_FRAC of the significant ones, if more) of an array
# may pass by this clause alone.
# Measured, not assumed: tests report every error (SRCNN_PARITY_LOG).
U_ROUND = 2.0 ** -24
K_ROUND = 0.25
MAX_ROUND_ONLY = 4
ROUND_ONLY_FRAC = 1e-4
RTOL = 1e-4
SIG = 1e-3
K_REF = 4.0
FLIP_FLOOR = 2e-5
# SRCNN_PARITY_LOG=<file>: append one JSON line per check with the achieved
# normwise and elementwise errors (the GPU sessions collect them)
PARITY_LOG = os.environ.get("SRCNN_PARITY_LOG")


def log_record(rec):
    """Append one JSON line to the parity log (SRCNN_PARITY_LOG), if set."""
    if PARITY_LOG:
        with open(PARITY_LOG, "a") as fh:
            fh.write(json.dumps(rec) + "\n")


def dev(a, torch):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t, torch):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def max_rel_err(got, ref):
    got = np.asarray(got, np.float64).ravel()
    ref = np.asarray(ref, np.float64).ravel()
    scale = np.abs(ref).max() if ref.size else 0.0
    if scale == 0:
        return float(np.abs(got - ref).max()) if ref.size else 0.0
    return float((np.abs(got - ref) / (np.abs(ref) + scale)).max())


def max_elem_rel_err(got, exact, sig=SIG):
    """(max |g - x| / |x| over elements with |x| >= sig * max|x|, count)."""
    got = np.asarray(got, np.float64).ravel()
    exact = np.asarray(exact, np.float64).ravel()
    if exact.size == 0:
        return 0.0, 0
    a = np.abs(exact)
    if a.max() == 0:
        return 0.0, 0
    m = a >= sig * a.max()
    return float((np.abs(got[m] - exact[m]) / a[m]).max()), int(m.sum())


def assert_close(got, ref, rtol=RTOL, what="", ref64=None, abs_floor=0.0, mag=None, nterms=None):
    """Normwise check against the fp32 oracle `ref`; with `ref64` (the same
    computation by the double-precision oracle) also the elementwise check
    described at RTOL, each element allowed abs_floor x max|ref64| on top
    (FLIP_FLOOR for gradients), and with `mag` / `nterms` the rounding-bound
    clause described at U_ROUND.  Returns the normwise error."""
    got = np.asarray(got)
    ref = np.asarray(ref)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    assert np.all(np.isfinite(got)), what + ": non-finite values"
    err = max_rel_err(got, ref)
    rec = {"what": what, "n": int(ref.size), "normwise": err, "rtol": rtol}
    el = el_ref = None
    if ref64 is not None:
        ref64 = np.asarray(ref64)
        assert ref64.shape == ref.shape, (what, ref64.shape, ref.shape)
        el, n_sig = max_elem_rel_err(got, ref64)
        el_ref, _ = max_elem_rel_err(ref, ref64)
        bound = max(rtol, K_REF * el_ref)
        x = np.abs(np.asarray(ref64, np.float64).ravel())
        sig = x >= SIG * x.max() if x.size and x.max() > 0 else np.zeros(x.size, bool)
        dev_ = np.abs(np.asarray(got, np.float64).ravel() - np.asarray(ref64, np.float64).ravel())
        over = dev_ - bound * x - abs_floor * (x.max() if x.size else 0.0)
        if mag is not None:
            rb = K_ROUND * U_ROUND * np.sqrt(np.asarray(nterms, np.float64)) * \
                np.abs(np.asarray(mag, np.float64)).ravel()
            rb = np.broadcast_to(rb, dev_.shape)
            with np.errstate(divide="ignore", invalid="ignore"):
                ratio = np.where(rb > 0, dev_ / rb, 0.0)
            rec["rounding_ratio_max"] = float(ratio[sig].max()) if sig.any() else 0.0
            n_over_rtol = int((over[sig] > 0).sum())
            rec["n_over_rtol"] = n_over_rtol
            over = np.minimum(over, dev_ - rb)
            n_round_only = n_over_rtol - int((over[sig] > 0).sum())
            rec["n_round_only"] = n_round_only
            allowed = max(MAX_ROUND_ONLY, int(ROUND_ONLY_FRAC * int(sig.sum())))
            assert n_round_only <= allowed, (
                "%s: %d significant elements pass only by the rounding-estimate clause (> %d allowed): "
                "an accumulation regression, not cancellation" % (what, n_round_only, allowed))
        n_over = int((over[sig] > 0).sum())
        rec.update(elementwise=el, elementwise_fp32_oracle=el_ref, significant=n_sig,
                   abs_floor=abs_floor, n_over=n_over)
    log_record(rec)
    assert err <= rtol, "%s: max normwise rel err %.3e > %.1e" % (what, err, rtol)
    if el is not None:
        assert n_over == 0, ("%s: %d of %d significant elements off the exact result by more than "
                             "%.2e rel + %.1e x max (max rel err %.3e; fp32 oracle's own %.3e)"
                             % (what, n_over, n_sig, bound, abs_floor, el, el_ref))
    return err


def smooth_patches(rng, batch, w, h, up=4):
    """clip(smooth random field) as in SURVEY.md 8(d): uniform grid upsampled."""
    gh, gw = h // up + 2, w // up + 2
    g = rng.random((batch, gh, gw)).astype(np.float32)
    ys = np.linspace(0, gh - 1.001, h)
    xs = np.linspace(0, gw - 1.001, w)
    y0, x0 = ys.astype(int), xs.astype(int)
    fy, fx = (ys - y0)[None, :, None], (xs - x0)[None, None, :]
    a = g[:, y0][:, :, x0]
    b = g[:, y0][:, :, x0 + 1]
    c = g[:, y0 + 1][:, :, x0]
    d = g[:, y0 + 1][:, :, x0 + 1]
    img = (a * (1 - fx) + b * fx) * (1 - fy) + (c * (1 - fx) + d * fx) * fy
    return np.clip(img, 0, 1).astype(np.float32)


def make_batch(rng, batch, w, h):
    """(X = patch - its mean, T = patch + N(0, 0.02)) like Main_cl.cpp:135-141."""
    P = smooth_patches(rng, batch, w, h)
    X = P - P.reshape(batch, -1).mean(axis=1)[:, None, None]
    T = P + rng.normal(0, 0.02, P.shape).astype(np.float32)
    return X.astype(np.float32).ravel(), T.astype(np.float32).ravel()


def make_params(rng, net_tuple, sd=1e-3, mean=0.0):
    import srcnn_oracle as orc
    P = orc.param_count(*net_tuple)
    return (mean + sd * rng.standard_normal(P)).astype(np.float32)
