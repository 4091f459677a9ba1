"""Helpers shared by the GPU tests: device buffers (torch, plumbing only),
tolerance checks, synthetic SRCNN inputs."""
import numpy as np

# Normwise fp32 tolerance of BASELINE.json's north_star ("outputs within 1e-4
# rel of the reference"): every element within 1e-4 x (|ref| + max|ref|).
RTOL = 1e-4


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


def assert_close(got, ref, rtol=RTOL, what=""):
    got = np.asarray(got)
    ref = np.asarray(ref)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    assert np.all(np.isfinite(got)), what + ": non-finite values"
    err = max_rel_err(got, ref)
    assert err <= rtol, "%s: max normwise rel err %.3e > %.1e" % (what, err, rtol)
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
