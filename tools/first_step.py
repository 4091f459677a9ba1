"""Where does the first default-net step after another workload wait?
Wall time of each call of the first steps with a device sync after it."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
import srcnn_amd as S  # noqa: E402


def timed(label, fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("%-28s enqueue %7.2f ms  total %7.2f ms" % (label, (t1 - t) * 1e3, (t2 - t) * 1e3), flush=True)


net_t = bench.DEFAULT_NET
net = S.Net(*net_t)
dev = torch.device("cuda", 0)
B, w = 4096, 33
P = S.net_param_count(net)
X, T = bench.synthetic_batch(np.random.default_rng(1), B, w, w)
Xd, Td = torch.from_numpy(X).to(dev), torch.from_numpy(T).to(dev)
params = torch.from_numpy(bench.init_params(net_t, P)).to(dev)
grads = torch.zeros(P, device=dev)
mom = torch.zeros(P, device=dev)
nb = S.train_workspace_bytes(net, w, w, B)
ws = torch.empty(nb // 4 + 64, device=dev)
s = torch.cuda.current_stream().cuda_stream
mode = sys.argv[1] if len(sys.argv) > 1 else "wide"
print("== mode", mode)
if mode == "wide":
    print(bench.wide_training(S)["ms_per_step"])
elif mode == "wide_sleep":
    print(bench.wide_training(S)["ms_per_step"])
    time.sleep(0.2)
elif mode == "fwd":
    print(bench.forward_4k(S, net_t)["ms_per_frame"])
elif mode == "wide_noprof":
    S.profile_enable = lambda on: None
    print(bench.wide_training(S)["ms_per_step"])
elif mode == "wide_raw":
    # the wide net's step without bench.py's wrapper, tensors kept alive
    wn = S.Net(*bench.WIDE_NET)
    WP = S.net_param_count(wn)
    wp = torch.from_numpy(bench.init_params(bench.WIDE_NET, WP)).to(dev)
    wg, wm = torch.zeros(WP, device=dev), torch.zeros(WP, device=dev)
    wnb = S.train_workspace_bytes(wn, w, w, B)
    wws = torch.empty(wnb // 4 + 64, device=dev)
    for i in range(3):
        timed("wide step %d" % i, lambda: S.train_fwd_bwd(wn, Xd, Td, w, w, B, wp, wg, None, wws, wnb, s))
for i in range(4):
    timed("step %d train_fwd_bwd" % i,
          lambda: S.train_fwd_bwd(net, Xd, Td, w, w, B, params, grads, None, ws, nb, s))
    timed("step %d update_all" % i,
          lambda: S.update_all(net, params, grads, mom, 0.9, 1e-3, [1e-4, 1e-4, 1e-5], B, s))
