"""Debug: the CBDP caller-owned-pools flow (op-level calls, mini-batch chunks)
for the wide net vs the oracle."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "cnn-super-resolution_amd")):
    sys.path.insert(0, p)
import numpy as np, torch
import srcnn_amd as S, srcnn_oracle as orc
from hip_util import make_batch, make_params, max_rel_err
cfg = (128, 64, 9, 5, 5); n1, n2, f1, f2, f3 = cfg
w, N, mini, lr = 25, 5, 3, [1e-3, 1e-3, 1e-4]
rng = np.random.default_rng(9)
X, T = make_batch(rng, N, w, w)
p0 = make_params(rng, cfg, sd=0.05)
P = p0.size
net = S.Net(*cfg)
off = S.net_offsets(net) + [P]
w1 = w - f1 + 1; w2 = w1 - f2 + 1; w3 = w2 - f3 + 1
dev = torch.device("cuda", 0)
D = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)
prm = D(p0); grads = torch.zeros(P, device=dev); mom = torch.zeros(P, device=dev)
Wt = [prm[off[2 * i]:off[2 * i + 1]] for i in range(3)]; Bt = [prm[off[2 * i + 1]:off[2 * i + 2]] for i in range(3)]
gW = [grads[off[2 * i]:off[2 * i + 1]] for i in range(3)]; gB = [grads[off[2 * i + 1]:off[2 * i + 2]] for i in range(3)]
mW = [mom[off[2 * i]:off[2 * i + 1]] for i in range(3)]; mB = [mom[off[2 * i + 1]:off[2 * i + 2]] for i in range(3)]
A1 = torch.zeros(mini * w1 * w1 * n1, device=dev); A2 = torch.zeros(mini * w2 * w2 * n2, device=dev)
A3 = torch.zeros(mini * w3 * w3, device=dev); D3 = torch.zeros_like(A3); D2 = torch.zeros_like(A2); D1 = torch.zeros_like(A1)
ws = torch.zeros(64 << 20, device=dev)
Xd, Td = D(X), D(T)
po, go, mo = p0.copy(), np.zeros(P, np.float32), np.zeros(P, np.float32)
t = w * w
for epoch in range(3):
    for c0 in range(0, N, mini):
        n = min(mini, N - c0)
        x, tt = Xd[c0 * t:(c0 + n) * t], Td[c0 * t:(c0 + n) * t]
        S.conv_fwd(x, A1, Wt[0], Bt[0], w, w, 1, n1, f1, 1, n)
        S.conv_fwd(A1, A2, Wt[1], Bt[1], w1, w1, n1, n2, f2, 1, n)
        S.conv_fwd(A2, A3, Wt[2], Bt[2], w2, w2, n2, 1, f3, 0, n)
        S.last_delta(tt, A3, D3, w, w, w3, w3, n)
        S.conv_delta(D3, A2, D2, Wt[2], f3, n2, 1, w2, w2, n)
        S.conv_delta(D2, A1, D1, Wt[1], f2, n1, n2, w1, w1, n)
        for (inp, dl, npv, ncu, f, ow, li) in ((A2, D3, n2, 1, f3, w3, 2), (A1, D2, n1, n2, f2, w2, 1), (x, D1, 1, n1, f1, w1, 0)):
            nb = S.conv_grad_workspace_bytes(npv, ncu, f, ow, ow, n)
            S.conv_grad_acc(inp, dl, gW[li], gB[li], npv, ncu, f, ow, ow, n, ws, nb)
        go, _ = orc.train_fwd_bwd(cfg, X[c0 * t:(c0 + n) * t], T[c0 * t:(c0 + n) * t], w, w, n, po, go)
    torch.cuda.synchronize()
    print("epoch", epoch, "grads vs oracle %.3e" % max_rel_err(grads.cpu().numpy(), go))
    for li in (2, 1, 0):
        S.sgd_update(Wt[li], Bt[li], gW[li], gB[li], mW[li], mB[li], 0.9, 1e-3, lr[li], N, Wt[li].numel(), Bt[li].numel())
    grads.zero_()
    po, go, mo = orc.update_all(cfg, po, go, mo, 0.9, 1e-3, lr, N)
    torch.cuda.synchronize()
    print("   params vs oracle %.3e" % max_rel_err(prm.cpu().numpy(), po))

# ---- the net-level (fused wide) flow on the same data ----
prm2 = D(p0); g2 = torch.zeros(P, device=dev); m2 = torch.zeros(P, device=dev)
nbw = S.train_workspace_bytes(net, w, w, mini)
wsw = torch.zeros(nbw // 4 + 64, device=dev)
for epoch in range(3):
    for c0 in range(0, N, mini):
        n = min(mini, N - c0)
        S.train_fwd_bwd(net, Xd[c0 * t:(c0 + n) * t], Td[c0 * t:(c0 + n) * t], w, w, n, prm2, g2, None, wsw, nbw)
    print("net-level path", S.last_path())
    S.update_all(net, prm2, g2, m2, 0.9, 1e-3, lr, N)
torch.cuda.synchronize()
print("net-level params vs oracle %.3e" % max_rel_err(prm2.cpu().numpy(), po))
# validation error of both parameter sets (forward + sq err), vs the oracle's
for name, pp in (("op-level", prm), ("net-level", prm2)):
    out = torch.zeros(N * w3 * w3, device=dev)
    nbf = S.forward_workspace_bytes(net, w, w, N)
    wsf = torch.zeros(nbf // 4 + 64, device=dev)
    S.forward(net, Xd, w, w, N, pp, out, wsf, nbf)
    torch.cuda.synchronize()
    e = orc.sq_err(T, out.cpu().numpy(), w, w, w3, w3, N)
    print(name, "validation err", e)
print("oracle validation err", orc.sq_err(T, orc.forward(cfg, X, w, w, N, po), w, w, w3, w3, N))
