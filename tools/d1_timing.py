"""Section timing of the d1_grad12 kernel, wave 0 of each block (diagnostics
build: tools/build_variant.sh d1t -DSRCNN_D1_TIMING): one training step, then per-phase cycles averaged
over blocks."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SRCNN_HIP_LIB", os.path.join(ROOT, "cnn-super-resolution_amd/lib/variants/libsrcnn_hip_d1t.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cnn-super-resolution_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import srcnn_amd as S  # noqa: E402
from hip_util import make_batch  # noqa: E402

dev = torch.device("cuda", 0)
net = S.Net(64, 32, 9, 1, 5)
B = 4096
X, T = make_batch(np.random.default_rng(0), B, 33, 33)
Xd, Td = torch.from_numpy(X).to(dev), torch.from_numpy(T).to(dev)
P = S.net_param_count(net)
p = (torch.randn(P, device=dev) * 1e-3)
g = torch.zeros(P, device=dev)
nb = S.train_workspace_bytes(net, 33, 33, B)
ws = torch.empty(nb // 4 + 64, device=dev)
for _ in range(3):
    S.train_fwd_bwd(net, Xd, Td, 33, 33, B, p, g, None, ws, nb)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (1024 * 4 * 8))()
assert S.lib().srcnn_debug_d1_timing(buf) == 0
t8 = np.array(buf, dtype=np.float64).reshape(1024, 4, 8)
t8 = t8[t8[:, :, :6].sum(axis=(1, 2)) > 0]
clk = t8[:, :, 6] / np.maximum(t8[:, :, 7], 1) * 0.1  # GHz (s_memrealtime ticks at 100 MHz)
print("held shader clock over the kernel: median %.3f GHz (min %.3f, max %.3f); block span %.1f us"
      % (np.median(clk), clk.min(), clk.max(), np.median(t8[:, :, 7]) / 100.0))
t = t8[:, :, :6]
nb = len(t)
chunks = (B / nb) * 20 / 4  # chunks per wave (20 per 33x33 sample)
# NOTE: the compiler does not order s_memtime against MFMAs: the section
# split is approximate (e.g. "other" absorbs gW1 MFMAs issued after its tick)
names = ["wait DMA (+xbt)", "delta1", "gW2", "sample top (vmcnt+barrier)", "gW1", "other"]
for w in range(4):
    tot = t[:, w].sum(axis=1).mean()
    print("wave %d: total %.0f cycles/block = %.1f us at 2.2 GHz" % (w, tot, tot / 2.2e3))
    for i, n in enumerate(names):
        print("   %-28s %10.0f cycles/block  %5.1f%%  (%.0f per chunk)" % (n, t[:, w, i].mean(), 100 * t[:, w, i].mean() / tot, t[:, w, i].mean() / chunks))
print("product probe (srcnn_profile_clock, blocks 0-7): %.3f GHz" % S.profile_clock("delta1_grad12_fused"))
