"""Phase timing of the l3_delta kernel (diagnostics build, tools/build_variant.sh
l3t -DSRCNN_L3_TIMING): one training step, then per-phase cycles averaged
over blocks."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SRCNN_HIP_LIB", os.path.join(ROOT, "cnn-super-resolution_amd/lib/variants/libsrcnn_hip_l3t.so"))
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
buf = (ctypes.c_ulonglong * (1024 * 4))()
assert S.lib().srcnn_debug_l3_timing(buf) == 0
t = np.array(buf, dtype=np.float64).reshape(1024, 4)
t = t[t.sum(axis=1) > 0]
spb = B / len(t)  # samples per block
names = ["Q mfma", "L3 gather+delta3", "delta2+gW3 (wave 0)", "top wait (DMA+barrier)"]
tot = t.sum(axis=1).mean()
for i, n in enumerate(names):
    print("%-18s %10.0f cycles/block  %5.1f%%  (%.0f per sample)" % (n, t[:, i].mean(), 100 * t[:, i].mean() / tot, t[:, i].mean() / spb))
print("%d blocks, total %.0f cycles/block = %.1f us at 2.2 GHz" % (len(t), tot, tot / 2.2e3))
