"""One rank's strong-scaling step on one GPU (BASELINE.json configs[2]: the
4096-tile global batch sharded 512 per GPU at N = 8), as bench.py --gpus N
runs it, with a ONE-rank RCCL communicator standing in for the 8-rank one
(so the all-reduce costs its launch, not its xGMI latency):

  lazy      srcnn_train_fwd_bwd_lazy (previous update inside l12) + allreduce
  separate  srcnn_train_fwd_bwd + allreduce + srcnn_update_all
  step      srcnn_train_step (one device, no all-reduce: the N = 1 headline)

usage: python tools/strong_shard.py [--batch 512] [--steps 300] [--warmup 50]
Prints one JSON line per mode: ms/step (host clock over the timed steps,
synced) and the per-kernel split (srcnn_profile_* on every 5th step)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
import srcnn_amd as S  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=512)
ap.add_argument("--steps", type=int, default=300)
ap.add_argument("--warmup", type=int, default=50)
ap.add_argument("--modes", default="lazy,separate,step")
ap.add_argument("--global-batch", type=int, default=4096)
args = ap.parse_args()

torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
net_t = bench.DEFAULT_NET
net = S.Net(*net_t)
P = S.net_param_count(net)
B, w = args.batch, bench.TILE
X, T = bench.synthetic_batch(np.random.default_rng(1234), B, w, w)
Xd, Td = torch.from_numpy(X).to(dev), torch.from_numpy(T).to(dev)
p0 = bench.init_params(net_t, P)
nb = S.train_workspace_bytes(net, w, w, B)
ws = torch.empty(nb // 4 + 64, device=dev)
hs = torch.cuda.Stream(device=dev)
s = hs.cuda_stream
lr, mu, wd = [1e-4, 1e-4, 1e-5], 0.9, 1e-3
comm = S.comm_init_rank(1, S.comm_id(), 0)
S.preload(net)


def run(mode):
    pb = [torch.from_numpy(p0.copy()).to(dev), torch.empty(P, device=dev)]
    mb = [torch.zeros(P, device=dev), torch.empty(P, device=dev)]
    g = torch.zeros(P, device=dev)
    st = {"cur": 0, "pending": 0}

    def lazy():
        c = st["cur"]
        S.train_fwd_bwd_lazy(net, Xd, Td, w, w, B, pb[c], pb[1 - c], mb[c], mb[1 - c], g, mu, wd, lr,
                             st["pending"], None, ws, nb, s)
        if st["pending"]:
            st["cur"] = 1 - c
        S.allreduce_grads(comm, g, P, s)
        st["pending"] = args.global_batch

    def separate():
        S.train_fwd_bwd(net, Xd, Td, w, w, B, pb[0], g, None, ws, nb, s)
        S.allreduce_grads(comm, g, P, s)
        S.update_all(net, pb[0], g, mb[0], mu, wd, lr, args.global_batch, s)

    def step():
        S.train_step(net, Xd, Td, w, w, B, pb[0], g, mb[0], mu, wd, lr, args.global_batch, None, ws, nb, s)

    fn = {"lazy": lazy, "separate": separate, "step": step}[mode]
    sync = torch.cuda.synchronize
    n_settle = bench.settle(fn, 50.0, sync, 1, "gloo", dev)
    el, n_prof, _ = bench.timed_region(fn, args.steps, args.warmup, 1, 5, s, S, False, "gloo", dev, sync)
    stats = S.profile_stats()
    return {"mode": mode, "batch": B, "ms_per_step": round(el / args.steps * 1e3, 5),
            "settle_steps": n_settle, "steps": args.steps,
            "kernels_us": {k: round(t / n_prof * 1e3, 2) for k, (c, t) in stats.items()}}


for m in args.modes.split(","):
    print(json.dumps(run(m)), flush=True)
S.comm_destroy(comm)
