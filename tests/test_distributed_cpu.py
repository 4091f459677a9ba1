"""Data-parallel step (srcnn_amd/parallel.py) with world_size 2 and 3 over gloo.

Each rank accumulates the gradients of its contiguous shard of the global
tile batch, one all-reduce sums them, every rank applies the same update
with batch = global tile count.  The compute is injected:
here the oracle on CPU tensors (the GPU run injects the HIP calls), so this
checks the sharding, the collective and the update contract, against one
process training on the union batch.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT  # noqa: F401  (sys.path set-up)

NET = (64, 32, 9, 1, 5)
W = H = 21
LR = [1e-4, 1e-4, 1e-5]
STEPS = 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data(global_batch):
    from hip_util import make_batch, make_params
    rng = np.random.default_rng(77)
    X, T = make_batch(rng, global_batch, W, H)
    return X, T, make_params(rng, NET)


def _train(rank, world, global_batch, port, out_dir):
    """One rank: returns (writes) the parameters after STEPS steps."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import srcnn_oracle as orc
    from srcnn_amd import parallel
    orc.set_threads(1)
    parallel.init("gloo")
    X, T, p0 = _data(global_batch)
    start, count = parallel.shard(global_batch, rank, world)
    tile = W * H
    Xs, Ts = X[start * tile:(start + count) * tile], T[start * tile:(start + count) * tile]
    state = {"params": p0.copy(), "mom": np.zeros_like(p0)}
    grads = torch.zeros(p0.size, dtype=torch.float32)

    def fwd_bwd(g):
        if count:
            new, _ = orc.train_fwd_bwd(NET, Xs, Ts, W, H, count, state["params"], g.numpy().copy())
            g.copy_(torch.from_numpy(new))

    def update(nb):
        p, gz, m = orc.update_all(NET, state["params"], grads.numpy().copy(), state["mom"],
                                  0.9, 1e-3, LR, nb)
        state["params"], state["mom"] = p, m
        grads.copy_(torch.from_numpy(gz))

    step = parallel.DataParallelStep(grads, fwd_bwd, update, global_batch)
    for _ in range(STEPS):
        step()
    np.save(os.path.join(out_dir, "params_%d.npy" % rank), state["params"])
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


def _train_lazy(rank, world, global_batch, port, out_dir):
    """The same training with parallel.LazyDataParallelStep: each step's
    update applied out of place by the next step (srcnn_train_fwd_bwd_lazy's
    contract, here on the oracle), finish() applying the last one."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import srcnn_oracle as orc
    from srcnn_amd import parallel
    orc.set_threads(1)
    parallel.init("gloo")
    X, T, p0 = _data(global_batch)
    start, count = parallel.shard(global_batch, rank, world)
    tile = W * H
    Xs, Ts = X[start * tile:(start + count) * tile], T[start * tile:(start + count) * tile]
    P = p0.size
    bufs = [torch.from_numpy(p0.copy()), torch.full((P,), float("nan")),
            torch.zeros(P), torch.full((P,), float("nan"))]
    grads = torch.full((P,), float("nan"))  # overwritten by every step

    def fwd_bwd_lazy(pi, po, mi, mo, g, pending):
        cur = pi
        if pending:
            p, _, m = orc.update_all(NET, pi.numpy().copy(), g.numpy().copy(), mi.numpy().copy(),
                                     0.9, 1e-3, LR, pending)
            po.copy_(torch.from_numpy(p))
            mo.copy_(torch.from_numpy(m))
            cur = po
        new = np.zeros(P, np.float32)
        if count:
            new, _ = orc.train_fwd_bwd(NET, Xs, Ts, W, H, count, cur.numpy().copy(), new)
        g.copy_(torch.from_numpy(new))

    def update(p, m, g, nb):
        pn, gz, mn = orc.update_all(NET, p.numpy().copy(), g.numpy().copy(), m.numpy().copy(),
                                    0.9, 1e-3, LR, nb)
        p.copy_(torch.from_numpy(pn))
        m.copy_(torch.from_numpy(mn))
        g.copy_(torch.from_numpy(gz))

    step = parallel.LazyDataParallelStep(bufs[0], bufs[1], bufs[2], bufs[3], grads, fwd_bwd_lazy, update,
                                         global_batch)
    for _ in range(STEPS):
        step()
    p, _ = step.finish()
    np.save(os.path.join(out_dir, "lazy_%d.npy" % rank), p.numpy())
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world,global_batch", [(2, 6), (3, 7)])
def test_lazy_step_bit_identical_to_separate_update(tmp_path, world, global_batch):
    """LazyDataParallelStep (the N > 1 bench step) against DataParallelStep:
    the same parameters bit for bit after STEPS steps, on every rank."""
    for fn in (_train, _train_lazy):
        mp.start_processes(fn, args=(world, global_batch, _free_port(), str(tmp_path)),
                           nprocs=world, join=True, start_method="spawn")
    for r in range(world):
        a = np.load(tmp_path / ("params_%d.npy" % r))
        b = np.load(tmp_path / ("lazy_%d.npy" % r))
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def _single(global_batch):
    import srcnn_oracle as orc
    X, T, p = _data(global_batch)
    mom, g = np.zeros_like(p), np.zeros_like(p)
    for _ in range(STEPS):
        g, _ = orc.train_fwd_bwd(NET, X, T, W, H, global_batch, p, g)
        p, g, mom = orc.update_all(NET, p, g, mom, 0.9, 1e-3, LR, global_batch)
    return p


@pytest.mark.parametrize("world,global_batch", [(2, 6), (3, 7), (2, 1)])
def test_data_parallel_matches_union_batch(tmp_path, world, global_batch):
    mp.start_processes(_train, args=(world, global_batch, _free_port(), str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    ref = _single(global_batch)
    outs = [np.load(tmp_path / ("params_%d.npy" % r)) for r in range(world)]
    for r in range(1, world):  # replicas bit-identical
        assert np.array_equal(outs[0], outs[r])
    # same math, different summation order of the per-shard gradient sums
    err = np.abs(outs[0] - ref).max() / (np.abs(ref).max() + 1e-30)
    assert err < 1e-6, err
    assert not np.array_equal(outs[0], _data(global_batch)[2])  # it trained


def test_shard_partition():
    from srcnn_amd import parallel
    for gb in (0, 1, 7, 4096, 4097):
        for world in (1, 2, 3, 8):
            got = [parallel.shard(gb, r, world) for r in range(world)]
            assert sum(c for _, c in got) == gb
            pos = 0
            for s, c in got:
                assert s == pos
                pos += c
            assert max(c for _, c in got) - min(c for _, c in got) <= 1
    with pytest.raises(ValueError):
        parallel.shard(4, 2, 2)


if __name__ == "__main__":
    sys.exit(pytest.main([__file__, "-q"]))
