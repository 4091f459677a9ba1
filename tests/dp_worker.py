"""One rank of the data-parallel GPU test (tests/test_dp_gpu.py); not a test.

Runs STEPS data-parallel SRCNN training steps of the HIP path
(srcnn_train_fwd_bwd on this rank's shard -> all-reduce of the flat gradient
buffer -> srcnn_update_all with batch = global tile count) under
srcnn_amd.parallel.DataParallelStep, then writes its parameters and the kernel
path that served the step.

Both ranks sit on device 0 of the one-GPU box.  RCCL refuses two ranks on
one device, so the collective here is the process group's gloo all_reduce on
a host copy of the gradient buffer (injected as DataParallelStep's
`allreduce`); the RCCL stage itself is covered by test_dp_gpu.py's
single-rank communicator tests and by bench.py on the 8-GPU node.

usage: RANK=r WORLD_SIZE=n MASTER_ADDR=127.0.0.1 MASTER_PORT=p \
       python dp_worker.py OUT_DIR NET GLOBAL_BATCH STEPS TILE
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for _p in (HERE, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "cnn-super-resolution_amd")):
    sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

LR = [1e-4, 1e-4, 1e-5]


def main():
    out_dir, net_s, gb, steps, tile = sys.argv[1:6]
    net_t = tuple(int(v) for v in net_s.split(","))
    gb, steps, tile = int(gb), int(steps), int(tile)
    import srcnn_amd as S
    from srcnn_amd import parallel
    from hip_util import make_batch, make_params

    rank, world, _ = parallel.env_world()
    torch.cuda.set_device(0)
    parallel.init("gloo")
    rng = np.random.default_rng(2024)
    X, T = make_batch(rng, gb, tile, tile)
    p0 = make_params(rng, net_t, sd=0.05)
    start, count = parallel.shard(gb, rank, world)
    n = tile * tile
    dev = torch.device("cuda", 0)
    Xd = torch.from_numpy(X[start * n:(start + count) * n].copy()).to(dev)
    Td = torch.from_numpy(T[start * n:(start + count) * n].copy()).to(dev)
    net = S.Net(*net_t)
    P = S.net_param_count(net)
    params = torch.from_numpy(p0).to(dev)
    grads = torch.zeros(P, dtype=torch.float32, device=dev)
    mom = torch.zeros(P, dtype=torch.float32, device=dev)
    nbytes = S.train_workspace_bytes(net, tile, tile, max(count, 1))
    ws = torch.empty(nbytes // 4 + 64, dtype=torch.float32, device=dev)
    paths = []

    def fwd_bwd(g):
        S.train_fwd_bwd(net, Xd, Td, tile, tile, count, params, g, None, ws, nbytes)
        paths.append(S.last_path())

    def update(nb):
        S.update_all(net, params, grads, mom, 0.9, 1e-3, LR, nb)

    def allreduce(g):  # gloo on a host copy (both ranks share device 0)
        torch.cuda.synchronize()
        h = g.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM)
        g.copy_(h.to(dev))

    if os.environ.get("SRCNN_DP_LAZY"):
        # bench.py's N > 1 step: srcnn_train_fwd_bwd_lazy (ping-ponged
        # parameters, the previous update inside the first kernel) + all-reduce
        def fwd_bwd_lazy(pi, po, mi, mo, g, pending):
            S.train_fwd_bwd_lazy(net, Xd, Td, tile, tile, count, pi, po, mi, mo, g, 0.9, 1e-3, LR,
                                 pending, None, ws, nbytes)
            paths.append(S.last_path())

        def update_lazy(p, m, g, nb):
            S.update_all(net, p, g, m, 0.9, 1e-3, LR, nb)

        step = parallel.LazyDataParallelStep(params, torch.empty_like(params), mom, torch.empty_like(mom),
                                             grads, fwd_bwd_lazy, update_lazy, gb, allreduce=allreduce)
    else:
        step = parallel.DataParallelStep(grads, fwd_bwd, update, gb, allreduce=allreduce)
    for _ in range(steps):
        step()
    if os.environ.get("SRCNN_DP_LAZY"):
        params, mom = step.finish()
    torch.cuda.synchronize()
    np.save(os.path.join(out_dir, "params_%d.npy" % rank), params.cpu().numpy())
    with open(os.path.join(out_dir, "path_%d.txt" % rank), "w") as fh:
        fh.write(",".join(paths))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
