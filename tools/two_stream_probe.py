"""Probe: does splitting the 4096-tile step into two half-batch calls on two
HIP streams (so one half's l3 / d1c can overlap the other half's l12 and the
kernel tails fill each other's idle CUs) beat one call on the whole batch?
Times srcnn_train_fwd_bwd only (no update), steady state, same process."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cnn-super-resolution_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import srcnn_amd as S  # noqa: E402
from hip_util import make_batch  # noqa: E402

dev = torch.device("cuda", 0)
net = S.Net(64, 32, 9, 1, 5)
B, W = 4096, 33
X, T = make_batch(np.random.default_rng(0), B, W, W)
Xd, Td = torch.from_numpy(X).to(dev), torch.from_numpy(T).to(dev)
P = S.net_param_count(net)
p = torch.randn(P, device=dev) * 1e-3
s0, s1 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
nb_full = S.train_workspace_bytes(net, W, W, B)
nb_half = S.train_workspace_bytes(net, W, W, B // 2)
ws_full = torch.empty(nb_full // 4 + 64, device=dev)
ws_h = [torch.empty(nb_half // 4 + 64, device=dev) for _ in range(2)]
g_full = torch.zeros(P, device=dev)
g_h = [torch.zeros(P, device=dev) for _ in range(2)]
half = B // 2 * W * W


def one():
    S.train_fwd_bwd(net, Xd, Td, W, W, B, p, g_full, None, ws_full, nb_full, s0.cuda_stream)


def two(streams):
    for i in range(2):
        S.train_fwd_bwd(net, Xd[i * half:(i + 1) * half], Td[i * half:(i + 1) * half], W, W, B // 2, p,
                        g_h[i], None, ws_h[i], nb_half, streams[i].cuda_stream)


def timeit(fn, n=60, warm=30):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


for rep in range(2):
    print("rep %d: one call %.4f ms | two halves, one stream %.4f ms | two halves, two streams %.4f ms"
          % (rep, timeit(one), timeit(lambda: two([s0, s0])), timeit(lambda: two([s0, s1]))), flush=True)
