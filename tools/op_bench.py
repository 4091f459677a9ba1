#!/usr/bin/env python3
"""Per-operator timing of the op-level C ABI (the reference-side DataPipeline
binding) on the training-tile shapes: one
ConfigBasedDataPipeline::execute_batch + update_parameters composed of
srcnn_conv_fwd / srcnn_last_delta / srcnn_conv_delta / srcnn_conv_grad_acc /
srcnn_sgd_update calls, as src/ConfigBasedDataPipeline.cpp:200-361 issues
them.  Prints one JSON object: ms per op (HIP events on the stream), the path
that served each op (srcnn_last_path) and the whole op-level step next to the
fused net-level step (srcnn_train_fwd_bwd + srcnn_update_all).

    python tools/op_bench.py [--net 64,32,9,1,5] [--batch 4096] [--tile 33] [--path auto|generic]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cnn-super-resolution_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--net", default="64,32,9,1,5")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--tile", type=int, default=33)
    ap.add_argument("--path", choices=["auto", "generic"], default="auto")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import srcnn_amd as S
    from hip_util import make_batch

    n1, n2, f1, f2, f3 = (int(v) for v in a.net.split(","))
    net = S.Net(n1, n2, f1, f2, f3)
    B, w = a.batch, a.tile
    w1 = w - f1 + 1
    w2 = w1 - f2 + 1
    w3 = w2 - f3 + 1
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    X, T = make_batch(rng, B, w, w)
    Xd, Td = torch.from_numpy(X).to(dev), torch.from_numpy(T).to(dev)
    P = S.net_param_count(net)
    off = S.net_offsets(net) + [P]
    prm = torch.from_numpy((0.05 * rng.standard_normal(P)).astype(np.float32)).to(dev)
    grads = torch.zeros(P, device=dev)
    mom = torch.zeros(P, device=dev)
    A1 = torch.empty(B * w1 * w1 * n1, device=dev)
    A2 = torch.empty(B * w2 * w2 * n2, device=dev)
    A3 = torch.empty(B * w3 * w3, device=dev)
    D3, D2, D1 = torch.empty_like(A3), torch.empty_like(A2), torch.empty_like(A1)
    gws_b = max(S.conv_grad_workspace_bytes(1, n1, f1, w1, w1, B),
                S.conv_grad_workspace_bytes(n1, n2, f2, w2, w2, B),
                S.conv_grad_workspace_bytes(n2, 1, f3, w3, w3, B))
    gws = torch.empty(gws_b // 4 + 64, device=dev)
    W = [prm[off[2 * i]:off[2 * i + 1]] for i in range(3)]
    Bs = [prm[off[2 * i + 1]:off[2 * i + 2]] for i in range(3)]
    gW = [grads[off[2 * i]:off[2 * i + 1]] for i in range(3)]
    gB = [grads[off[2 * i + 1]:off[2 * i + 2]] for i in range(3)]
    mW = [mom[off[2 * i]:off[2 * i + 1]] for i in range(3)]
    mB = [mom[off[2 * i + 1]:off[2 * i + 2]] for i in range(3)]
    S.set_path(0 if a.path == "auto" else 1)
    ops = [
        ("fwd_l1", lambda: S.conv_fwd(Xd, A1, W[0], Bs[0], w, w, 1, n1, f1, 1, B)),
        ("fwd_l2", lambda: S.conv_fwd(A1, A2, W[1], Bs[1], w1, w1, n1, n2, f2, 1, B)),
        ("fwd_l3", lambda: S.conv_fwd(A2, A3, W[2], Bs[2], w2, w2, n2, 1, f3, 0, B)),
        ("last_delta", lambda: S.last_delta(Td, A3, D3, w, w, w3, w3, B)),
        ("delta2", lambda: S.conv_delta(D3, A2, D2, W[2], f3, n2, 1, w2, w2, B)),
        ("delta1", lambda: S.conv_delta(D2, A1, D1, W[1], f2, n1, n2, w1, w1, B)),
        ("grad3", lambda: S.conv_grad_acc(A2, D3, gW[2], gB[2], n2, 1, f3, w3, w3, B, gws, gws_b)),
        ("grad2", lambda: S.conv_grad_acc(A1, D2, gW[1], gB[1], n1, n2, f2, w2, w2, B, gws, gws_b)),
        ("grad1", lambda: S.conv_grad_acc(Xd, D1, gW[0], gB[0], 1, n1, f1, w1, w1, B, gws, gws_b)),
        ("update", lambda: [S.sgd_update(W[i], Bs[i], gW[i], gB[i], mW[i], mB[i], 0.9, 1e-3, 1e-4, B,
                                         W[i].numel(), Bs[i].numel()) for i in (2, 1, 0)]),
    ]
    res, paths = {}, {}
    for name, fn in ops:  # warm
        fn()
        paths[name] = S.last_path()
    torch.cuda.synchronize()
    for name, fn in ops:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) / a.reps, 4)
    op_step = sum(res.values())
    # the fused net-level step on the same data
    nb = S.train_workspace_bytes(net, w, w, B)
    ws = torch.empty(nb // 4 + 64, device=dev)

    def fused():
        S.train_fwd_bwd(net, Xd, Td, w, w, B, prm, grads, None, ws, nb)
        S.update_all(net, prm, grads, mom, 0.9, 1e-3, [1e-4, 1e-4, 1e-5], B)
    for _ in range(3):
        fused()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        fused()
    e1.record()
    torch.cuda.synchronize()
    fused_ms = e0.elapsed_time(e1) / a.reps
    print(json.dumps({"net": a.net, "batch": B, "tile": w, "path": a.path, "ms": res, "served_by": paths,
                      "op_level_step_ms": round(op_step, 4), "net_level_step_ms": round(fused_ms, 4),
                      "net_level_path": S.last_path(), "ratio": round(op_step / fused_ms, 3)}))


if __name__ == "__main__":
    main()
