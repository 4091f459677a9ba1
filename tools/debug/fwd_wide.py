import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "cnn-super-resolution_amd")):
    sys.path.insert(0, p)
import numpy as np, torch
import srcnn_amd as S, srcnn_oracle as orc
from hip_util import make_batch, make_params, max_rel_err
cfg = (128, 64, 9, 5, 5)
for w, B in ((25, 3), (25, 2), (33, 3)):
    rng = np.random.default_rng(5)
    X, T = make_batch(rng, B, w, w)
    prm = make_params(rng, cfg, sd=0.05)
    ref = orc.forward(cfg, X, w, w, B, prm)
    net = S.Net(*cfg)
    nb = S.forward_workspace_bytes(net, w, w, B)
    for trial in range(2):
        ws = torch.full((nb // 4 + 64,), float("nan"), device="cuda")
        out = torch.full((ref.size,), float("nan"), device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        S.forward(net, torch.from_numpy(X).cuda(), w, w, B, torch.from_numpy(prm).cuda(), out, ws, nb, s)
        torch.cuda.synchronize()
        print(w, B, trial, S.last_path(), "%.3e" % max_rel_err(out.cpu().numpy(), ref), np.isnan(out.cpu().numpy()).sum())
    # same, on a non-blocking stream of our own
    st = S.stream_create()
    ws = torch.zeros(nb // 4 + 64, device="cuda")
    out = torch.zeros(ref.size, device="cuda")
    torch.cuda.synchronize()
    S.forward(net, torch.from_numpy(X).cuda(), w, w, B, torch.from_numpy(prm).cuda(), out, ws, nb, st)
    S.stream_sync(st)
    print(w, B, "own stream", "%.3e" % max_rel_err(out.cpu().numpy(), ref))
