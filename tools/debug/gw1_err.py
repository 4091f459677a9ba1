"""Debug: where do the HIP W1 gradients of the 600-tile default step differ
from the exact (f64 oracle) result?"""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "cnn-super-resolution_amd")):
    sys.path.insert(0, p)
import numpy as np, torch
import srcnn_amd as S, srcnn_oracle as orc
from hip_util import make_batch, make_params
cfg = (64, 32, 9, 1, 5)
for batch, zero_g0 in ((600, False), (600, True), (257, False)):
    net = S.Net(*cfg)
    rng = np.random.default_rng(42)
    X, T = make_batch(rng, batch, 33, 33)
    params = make_params(rng, cfg, sd=0.05)
    P = params.size
    g0 = (1e-3 * rng.standard_normal(P)).astype(np.float32)
    if zero_g0:
        g0[:] = 0
    rg, _ = orc.train_fwd_bwd(cfg, X, T, 33, 33, batch, params, g0)
    xg, acts64 = orc.f64.train_fwd_bwd(cfg, X, T, 33, 33, batch, params, g0, want_acts=True)
    nb = S.train_workspace_bytes(net, 33, 33, batch)
    res = {}
    for path in (0, 1):
        S.set_path(path)
        ws = torch.empty(nb // 4 + 64, device="cuda")
        g = torch.from_numpy(g0.copy()).cuda()
        S.train_fwd_bwd(net, torch.from_numpy(X).cuda(), torch.from_numpy(T).cuda(), 33, 33, batch,
                        torch.from_numpy(params).cuda(), g, None, ws, nb)
        torch.cuda.synchronize()
        res[path] = g.cpu().numpy()[:5184]
    S.set_path(0)
    x = xg[:5184]; r = rg[:5184]
    a = np.abs(x); m = a >= 1e-3 * a.max()
    for name, v in (("fp32 oracle", r), ("auto", res[0]), ("generic", res[1])):
        e = np.abs(v - x) / np.maximum(a, 1e-30)
        e[~m] = 0
        i = int(e.argmax())
        print(batch, "g0=0" if zero_g0 else "g0", name, "max elem err %.3e at %d (tap %d ch %d) x=%.6e v=%.6e max|x|=%.3e  abs err / max = %.2e"
              % (e[i], i, i // 64, i % 64, x[i], v[i], a.max(), np.abs(v - x).max() / a.max()))
    d = np.abs(res[0] - x) / a.max()
    per_tap = d.reshape(81, 64).max(axis=1)
    print("   worst taps (auto):", np.argsort(-per_tap)[:8], per_tap[np.argsort(-per_tap)[:8]])
    print("   auto vs generic max abs/max: %.2e" % (np.abs(res[0] - res[1]).max() / a.max()))
