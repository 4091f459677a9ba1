"""Debug: the op-level chain (forward, last delta, deltas, grads) of one
training chunk through the C ABI vs the oracle, tensor by tensor."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "cnn-super-resolution_amd")):
    sys.path.insert(0, p)
import numpy as np, torch
import srcnn_amd as S, srcnn_oracle as orc
from hip_util import make_batch, make_params, max_rel_err
for cfg, w, B in (((128, 64, 9, 5, 5), 25, 5), ((128, 64, 9, 5, 5), 33, 3), ((64, 32, 9, 1, 5), 33, 5)):
    n1, n2, f1, f2, f3 = cfg
    rng = np.random.default_rng(3)
    X, T = make_batch(rng, B, w, w)
    prm = make_params(rng, cfg, sd=0.05)
    P = prm.size
    _, acts = orc.train_fwd_bwd(cfg, X, T, w, w, B, prm, np.zeros(P, np.float32), want_acts=True)
    rg, _ = orc.train_fwd_bwd(cfg, X, T, w, w, B, prm, np.zeros(P, np.float32))
    w1 = w - f1 + 1; w2 = w1 - f2 + 1; w3 = w2 - f3 + 1
    s1, s2, s3 = B * w1 * w1 * n1, B * w2 * w2 * n2, B * w3 * w3
    rA1, rA2, rA3 = acts[:s1], acts[s1:s1 + s2], acts[s1 + s2:s1 + s2 + s3]
    rD3 = acts[s1 + s2 + s3:s1 + s2 + 2 * s3]; rD2 = acts[s1 + s2 + 2 * s3:s1 + 2 * s2 + 2 * s3]; rD1 = acts[s1 + 2 * s2 + 2 * s3:]
    dev = torch.device("cuda", 0)
    D = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)
    H = lambda t: (torch.cuda.synchronize(), t.cpu().numpy())[1]
    net = S.Net(*cfg)
    off = S.net_offsets(net) + [P]
    Wt = [D(prm[off[2 * i]:off[2 * i + 1]]) for i in range(3)]
    Bt = [D(prm[off[2 * i + 1]:off[2 * i + 2]]) for i in range(3)]
    A1, A2, A3 = torch.zeros(s1, device=dev), torch.zeros(s2, device=dev), torch.zeros(s3, device=dev)
    D3, D2, D1 = torch.zeros(s3, device=dev), torch.zeros(s2, device=dev), torch.zeros(s1, device=dev)
    Xd, Td = D(X), D(T)
    S.conv_fwd(Xd, A1, Wt[0], Bt[0], w, w, 1, n1, f1, 1, B); p1 = S.last_path()
    S.conv_fwd(D(rA1), A2, Wt[1], Bt[1], w1, w1, n1, n2, f2, 1, B); p2 = S.last_path()
    S.conv_fwd(D(rA2), A3, Wt[2], Bt[2], w2, w2, n2, 1, f3, 0, B); p3 = S.last_path()
    S.last_delta(Td, D(rA3), D3, w, w, w3, w3, B)
    S.conv_delta(D(rD3), D(rA2), D2, Wt[2], f3, n2, 1, w2, w2, B); p4 = S.last_path()
    S.conv_delta(D(rD2), D(rA1), D1, Wt[1], f2, n1, n2, w1, w1, B); p5 = S.last_path()
    print(cfg, w, B, "paths", p1, p2, p3, p4, p5)
    for nm, g, r in (("A1", A1, rA1), ("A2", A2, rA2), ("A3", A3, rA3), ("D3", D3, rD3), ("D2", D2, rD2), ("D1", D1, rD1)):
        print("  %s %.2e" % (nm, max_rel_err(H(g), r)))
    gws = torch.zeros(64 << 20, device=dev)
    for li, (inp, dl, npv, ncu, f, ow) in enumerate(((X, rD1, 1, n1, f1, w1), (rA1, rD2, n1, n2, f2, w2), (rA2, rD3, n2, 1, f3, w3))):
        gW, gB = torch.zeros(off[2 * li + 1] - off[2 * li], device=dev), torch.zeros(off[2 * li + 2] - off[2 * li + 1], device=dev)
        nb = S.conv_grad_workspace_bytes(npv, ncu, f, ow, ow, B)
        S.conv_grad_acc(D(inp), D(dl), gW, gB, npv, ncu, f, ow, ow, B, gws, nb)
        print("  gW%d %.2e gB%d %.2e (%s)" % (li + 1, max_rel_err(H(gW), rg[off[2 * li]:off[2 * li + 1]]), li + 1,
              max_rel_err(H(gB), rg[off[2 * li + 1]:off[2 * li + 2]]), S.last_path()))
