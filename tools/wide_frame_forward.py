#!/usr/bin/env python3
"""Wide net (128, 64, 9, 5, 5) forward of one 1920x1080 frame through
srcnn_forward: the op-level gfx950 kernels on image windows (auto path)
against the generic kernels (SRCNN generic path), ms per frame and the
largest difference relative to max|output|.

    python tools/wide_frame_forward.py
"""
import sys, time, json
sys.path.insert(0, "cnn-super-resolution_amd")
import numpy as np, torch
import srcnn_amd as S
net_t = (128, 64, 9, 5, 5)
net = S.Net(*net_t)
w, h = 1920, 1080
dev = torch.device("cuda", 0)
x = torch.rand(w * h, device=dev) - 0.5
prm = (torch.randn(S.net_param_count(net), device=dev) * 1e-3)
out = torch.empty((w - 16) * (h - 16), device=dev)
nb = S.forward_workspace_bytes(net, w, h, 1)
ws = torch.empty(nb // 4 + 64, device=dev)
res = {}
for p in (0, 1):
    S.set_path(p)
    S.forward(net, x, w, h, 1, prm, out, ws, nb)
    torch.cuda.synchronize()
    n = 3 if p == 0 else 1
    t0 = time.perf_counter()
    for _ in range(n):
        S.forward(net, x, w, h, 1, prm, out, ws, nb)
    torch.cuda.synchronize()
    res["auto" if p == 0 else "generic"] = {"ms": round((time.perf_counter() - t0) / n * 1e3, 2), "path": S.last_path()}
    if p == 0:
        ref = out.clone()
S.set_path(0)
res["max_rel_diff_vs_generic"] = float((out - ref).abs().max() / ref.abs().max())
res["frame"] = "%dx%d" % (w, h)
print(json.dumps(res))
