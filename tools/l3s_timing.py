"""Per-wave step-loop timing of the unit-stream l3s kernel (diagnostics build,
tools/build_variant.sh l3st -DSRCNN_L3_TIMING): one training step at batch
4096, then per wave the share of its loop cycles spent in the top-of-step
vmcnt wait + barrier (s_memtime)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SRCNN_L3"] = "stream"
os.environ.setdefault("SRCNN_HIP_LIB", os.path.join(ROOT, "cnn-super-resolution_amd/lib/variants/libsrcnn_hip_l3st.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cnn-super-resolution_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import srcnn_amd as S  # noqa: E402
from hip_util import make_batch  # noqa: E402

dev = torch.device("cuda", 0)
net = S.Net(64, 32, 9, 1, 5)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
X, T = make_batch(np.random.default_rng(0), B, 33, 33)
Xd, Td = torch.from_numpy(X).to(dev), torch.from_numpy(T).to(dev)
P = S.net_param_count(net)
p = (torch.randn(P, device=dev) * 1e-3)
g = torch.zeros(P, device=dev)
nb = S.train_workspace_bytes(net, 33, 33, B)
ws = torch.empty(nb // 4 + 64, device=dev)
for _ in range(5):
    S.train_fwd_bwd(net, Xd, Td, 33, 33, B, p, g, None, ws, nb)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (768 * 8))()
assert S.lib().srcnn_debug_l3s_timing(buf) == 0
t = np.array(buf, dtype=np.float64).reshape(768, 4, 2)
t = t[t[:, :, 1].sum(axis=1) > 0]
steps = (B / len(t)) * 40 + 9
for w in range(4):
    wait, tot = t[:, w, 0].mean(), t[:, w, 1].mean()
    print("wave %d: loop %8.0f cycles (%.0f per step), top wait + barrier %5.1f%%" % (w, tot, tot / steps, 100 * wait / tot))
print("%d blocks, %.1f steps per block" % (len(t), steps))
