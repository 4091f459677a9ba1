import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "cnn-super-resolution_amd")):
    sys.path.insert(0, p)
import numpy as np, torch
import srcnn_amd as S, srcnn_oracle as orc
from hip_util import make_batch, make_params, max_rel_err
cfg = (128, 64, 9, 5, 5); w, B = 25, 3
rng = np.random.default_rng(5)
X, T = make_batch(rng, B, w, w)
prm = make_params(rng, cfg, sd=0.05)
ref = orc.forward(cfg, X, w, w, B, prm)
net = S.Net(*cfg)
nbt = S.train_workspace_bytes(net, w, w, B)
ws = torch.zeros(nbt // 4 + 64, device="cuda")
st = S.stream_create()
g = torch.zeros(prm.size, device="cuda")
Xd, Td, pd = torch.from_numpy(X).cuda(), torch.from_numpy(T).cuda(), torch.from_numpy(prm).cuda()
torch.cuda.synchronize()
S.train_fwd_bwd(net, Xd, Td, w, w, B, pd, g, None, ws, nbt, st)
S.stream_sync(st)
nbf = S.forward_workspace_bytes(net, w, w, B)
for trial in range(3):
    out = torch.zeros(ref.size, device="cuda")
    torch.cuda.synchronize()
    S.forward(net, Xd, w, w, B, pd, out, ws, nbf, st)
    S.stream_sync(st)
    o = out.cpu().numpy()
    print(trial, "%.3e" % max_rel_err(o, ref), "bad outputs:", int((np.abs(o - ref) > 1e-3 * np.abs(ref).max()).sum()), "of", o.size)
# per-layer intermediates of a fresh forward after another train step
S.train_fwd_bwd(net, Xd, Td, w, w, B, pd, g, None, ws, nbt, st)
S.stream_sync(st)
n1, n2, f1, f2, f3 = cfg
w1, w2 = w - 8, w - 12
s1 = B * w1 * w1 * n1
A1 = ws[:s1]
off = S.net_offsets(net)
S.conv_fwd(Xd, A1, pd[off[0]:off[1]], pd[off[1]:off[2]], w, w, 1, n1, f1, 1, B, st)
S.stream_sync(st)
_, acts = orc.train_fwd_bwd(cfg, X, T, w, w, B, prm, np.zeros(prm.size, np.float32), want_acts=True)
a1 = A1.cpu().numpy()
bad = np.nonzero(np.abs(a1 - acts[:s1]) > 1e-3 * np.abs(acts[:s1]).max())[0]
print("A1 after train: bad", bad.size, bad[:10], "pixels", np.unique(bad // n1 % (w1 * w1))[:20])
