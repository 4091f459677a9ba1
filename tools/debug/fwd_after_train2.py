import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "cnn-super-resolution_amd")):
    sys.path.insert(0, p)
import numpy as np, torch
import srcnn_amd as S, srcnn_oracle as orc
from hip_util import make_batch, make_params, max_rel_err
cfg = (128, 64, 9, 5, 5); w, N, mini = 25, 5, 3
rng = np.random.default_rng(5)
X, T = make_batch(rng, N, w, w)
prm = make_params(rng, cfg, sd=0.05)
net = S.Net(*cfg)
nbt = S.train_workspace_bytes(net, w, w, mini)
ws = torch.zeros(nbt // 4 + 64, device="cuda")
st = S.stream_create()
g = torch.zeros(prm.size, device="cuda")
pd = torch.from_numpy(prm).cuda()
Xb = torch.zeros(mini * w * w, device="cuda"); Tb = torch.zeros(mini * w * w, device="cuda")
Xd, Td = torch.from_numpy(X).cuda(), torch.from_numpy(T).cuda()
t = w * w
out = torch.zeros(mini * 81, device="cuda")
for rep in range(2):
    for c0 in range(0, N, mini):
        n = min(mini, N - c0)
        Xb[:n * t].copy_(Xd[c0 * t:(c0 + n) * t]); Tb[:n * t].copy_(Td[c0 * t:(c0 + n) * t])
        torch.cuda.synchronize()
        S.train_fwd_bwd(net, Xb, Tb, w, w, n, pd, g, None, ws, S.train_workspace_bytes(net, w, w, n), st)
        S.stream_sync(st)
    for c0 in range(0, N, mini):
        n = min(mini, N - c0)
        Xb[:n * t].copy_(Xd[c0 * t:(c0 + n) * t])
        torch.cuda.synchronize()
        nbf = S.forward_workspace_bytes(net, w, w, n)
        S.forward(net, Xb, w, w, n, pd, out, ws, nbf, st)
        S.stream_sync(st)
        ref = orc.forward(cfg, X[c0 * t:(c0 + n) * t], w, w, n, prm)
        o = out.cpu().numpy()[:n * 81]
        print(rep, c0, n, "%.3e" % max_rel_err(o, ref), "bad", int((np.abs(o - ref) > 1e-3 * np.abs(ref).max()).sum()))
