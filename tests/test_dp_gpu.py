"""Data-parallel training of the HIP path on the GPU.

- world_size 2: two rank processes on device 0 run the HIP training step
  under srcnn_amd.parallel.DataParallelStep on their shards of one global
  batch.  The replicas must be bit-identical, and equal (1e-4 rel) to one
  process training the union batch, both on the HIP path and in the oracle.
- the RCCL stage of the C ABI (srcnn_comm_*, srcnn_allreduce_grads) on a
  one-rank communicator: ncclCommInitAll and ncclCommInitRank, the in-place
  sum on the compute stream (the 8-GPU all-reduce is bench.py's, run by the
  driver on a whole node).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import srcnn_oracle as orc
from conftest import ROOT
from hip_util import FLIP_FLOOR, assert_close, make_batch, make_params

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

LR = [1e-4, 1e-4, 1e-5]


@pytest.fixture(scope="module")
def S():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import srcnn_amd
    return srcnn_amd


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _union_hip(S, net_t, gb, steps, tile):
    rng = np.random.default_rng(2024)
    X, T = make_batch(rng, gb, tile, tile)
    p0 = make_params(rng, net_t, sd=0.05)
    net = S.Net(*net_t)
    P = S.net_param_count(net)
    dev = torch.device("cuda", 0)
    Xd, Td = torch.from_numpy(X).to(dev), torch.from_numpy(T).to(dev)
    params = torch.from_numpy(p0.copy()).to(dev)
    grads = torch.zeros(P, device=dev)
    mom = torch.zeros(P, device=dev)
    nbytes = S.train_workspace_bytes(net, tile, tile, gb)
    ws = torch.empty(nbytes // 4 + 64, device=dev)
    for _ in range(steps):
        S.train_fwd_bwd(net, Xd, Td, tile, tile, gb, params, grads, None, ws, nbytes)
        S.update_all(net, params, grads, mom, 0.9, 1e-3, LR, gb)
    torch.cuda.synchronize()
    return p0, params.cpu().numpy(), X, T


def _union_oracle(net_t, X, T, p0, gb, steps, tile, o=orc.ORACLE):
    p, g, m = o.f(p0).copy(), o.zeros(p0.size), o.zeros(p0.size)
    for _ in range(steps):
        g, _ = o.train_fwd_bwd(net_t, X, T, tile, tile, gb, p, g)
        p, g, m = o.update_all(net_t, p, g, m, 0.9, 1e-3, LR, gb)
    return p


def _run_two_ranks(tmp_path, net_t, gb, steps, tile, lazy=False):
    world = 2
    port = _free_port()
    worker = os.path.join(ROOT, "tests", "dp_worker.py")
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.pop("SRCNN_DP_LAZY", None)
        if lazy:
            env["SRCNN_DP_LAZY"] = "1"
        procs.append(subprocess.Popen(
            [sys.executable, worker, str(tmp_path), ",".join(map(str, net_t)), str(gb), str(steps),
             str(tile)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    for p in procs:
        out, _ = p.communicate(timeout=240)
        assert p.returncode == 0, out.decode()[-3000:]
    return [np.load(tmp_path / ("params_%d.npy" % r)) for r in range(world)]


@pytest.mark.parametrize("net_t,gb,tile,want", [
    ((64, 32, 9, 1, 5), 96, 33, "fused"),     # default net, fused kernels
    ((64, 32, 9, 1, 5), 7, 21, "fused"),      # odd batch: ranks get 4 and 3 tiles
    ((16, 8, 5, 3, 3), 10, 19, "generic"),   # spatial middle layer, op-level path
], ids=["default", "ragged", "spatial"])
def test_two_ranks_match_union_batch(S, tmp_path, net_t, gb, tile, want):
    steps, world = 2, 2
    reps = _run_two_ranks(tmp_path, net_t, gb, steps, tile)
    assert np.array_equal(reps[0], reps[1]), "replicas diverged"
    for r in range(world):
        paths = (tmp_path / ("path_%d.txt" % r)).read_text().split(",")
        assert set(paths) == {want}, paths
    p0, hip_union, X, T = _union_hip(S, net_t, gb, steps, tile)
    ref = _union_oracle(net_t, X, T, p0, gb, steps, tile)
    ref64 = _union_oracle(net_t, X, T, p0, gb, steps, tile, orc.f64)
    # the update moves the parameters by ~lr*g/batch: compare the movement
    # (the f64 movement from the same fp32 start)
    assert not np.array_equal(reps[0], p0)
    mv64 = ref64 - p0.astype(np.float64)
    assert_close(reps[0] - p0, ref - p0, what="2-rank step vs oracle union batch", ref64=mv64,
                 abs_floor=FLIP_FLOOR)
    assert_close(hip_union - p0, ref - p0, what="HIP union batch vs oracle union batch", ref64=mv64,
                 abs_floor=FLIP_FLOOR)


def _check_identity_allreduce(S, comm):
    dev = torch.device("cuda", 0)
    v = torch.arange(8129, dtype=torch.float32, device=dev) * 0.5 - 7.0
    want = v.cpu().numpy()
    stream = torch.cuda.current_stream().cuda_stream
    S.allreduce_grads(comm, v, v.numel(), stream)
    torch.cuda.synchronize()
    assert np.array_equal(v.cpu().numpy(), want)  # one rank: the sum is the buffer itself


def test_rccl_comm_init_all_one_device(S):
    comms = S.comm_init_all([0])
    try:
        assert S.comm_rank(comms[0]) == (0, 1)
        _check_identity_allreduce(S, comms[0])
    finally:
        S.comm_destroy(comms[0])


def test_rccl_comm_init_rank_one_rank(S):
    uid = S.comm_id()
    assert len(uid) == S.COMM_ID_BYTES
    c = S.comm_init_rank(1, uid, 0)
    try:
        assert S.comm_rank(c) == (0, 1)
        _check_identity_allreduce(S, c)
    finally:
        S.comm_destroy(c)


def test_rccl_invalid_arguments(S):
    with pytest.raises(S.SrcnnError):
        S.comm_init_rank(2, S.comm_id(), 5)
    with pytest.raises(S.SrcnnError):
        S.comm_init_all([S.device_count()])
    with pytest.raises(S.SrcnnError):
        S.allreduce_grads(None, 0, 4)


@pytest.mark.parametrize("net_t,gb,tile", [
    ((64, 32, 9, 1, 5), 96, 33),
    ((16, 8, 5, 3, 3), 10, 19),
], ids=["default", "spatial"])
def test_two_ranks_lazy_step_equals_separate_update(S, tmp_path, net_t, gb, tile):
    """bench.py's N > 1 step (LazyDataParallelStep over
    srcnn_train_fwd_bwd_lazy) on two ranks: bit-identical to the
    fwd_bwd -> all-reduce -> update_all sequence on every rank."""
    (tmp_path / "sep").mkdir()
    (tmp_path / "lazy").mkdir()
    sep = _run_two_ranks(tmp_path / "sep", net_t, gb, 3, tile)
    lazy = _run_two_ranks(tmp_path / "lazy", net_t, gb, 3, tile, lazy=True)
    for r in range(2):
        assert np.array_equal(sep[r].view(np.uint32), lazy[r].view(np.uint32)), r


LAZY_CASES = [
    # net, tile, batch, kernel family expected
    ((64, 32, 9, 1, 5), 33, 512, "fused"),    # the strong-scaling shard: l12 grid 512, l3r two samples / block
    ((64, 32, 9, 1, 5), 33, 4096, "fused"),   # the weak-scaling batch
    ((64, 32, 9, 1, 5), 33, 1, "fused"),      # one l12 block writes every updated parameter
    ((64, 32, 9, 1, 5), 33, 37, "fused"),     # ragged grid: parameter slices of uneven blocks
    ((32, 16, 9, 1, 5), 33, 40, "fused"),     # n2 = 16: l3_delta, d1_grad12
    ((64, 32, 9, 1, 3), 27, 24, "fused"),     # f3 = 3
    ((64, 32, 9, 1, 5), 39, 12, "fused"),     # layer 3 on the op-level kernels (tile > 640 A2 px)
    ((128, 64, 9, 5, 5), 33, 16, "wide"),     # the lazy_update launch, then the wide step
    ((16, 8, 5, 3, 3), 19, 10, "generic"),    # op-level / generic kernels
]


@pytest.mark.parametrize("net_t,tile,batch,want", LAZY_CASES,
                         ids=["b512", "b4096", "b1", "b37", "n16", "f3", "t39", "wide", "spatial"])
def test_lazy_sequence_bit_identical(S, net_t, tile, batch, want):
    """srcnn_train_fwd_bwd_lazy over 3 steps (RCCL all-reduce on a one-rank
    communicator after each) + the final srcnn_update_all is bit-identical to
    srcnn_train_fwd_bwd + srcnn_allreduce_grads + srcnn_update_all per step:
    parameters, momentum and the (zeroed) gradients."""
    steps, gb = 3, batch * 3  # the update divides by the global batch
    rng = np.random.default_rng(91)
    X, T = make_batch(rng, batch, tile, tile)
    p0 = make_params(rng, net_t, sd=0.05)
    net = S.Net(*net_t)
    P = S.net_param_count(net)
    dev = torch.device("cuda", 0)
    Xd, Td = torch.from_numpy(X).to(dev), torch.from_numpy(T).to(dev)
    nbytes = S.train_workspace_bytes(net, tile, tile, batch)
    ws = torch.empty(nbytes // 4 + 64, device=dev)
    uid = S.comm_id()
    comm = S.comm_init_rank(1, uid, 0)
    stream = torch.cuda.current_stream().cuda_stream
    try:
        # reference sequence
        p = torch.from_numpy(p0.copy()).to(dev)
        g = torch.zeros(P, device=dev)
        m = torch.zeros(P, device=dev)
        for _ in range(steps):
            S.train_fwd_bwd(net, Xd, Td, tile, tile, batch, p, g, None, ws, nbytes, stream)
            S.allreduce_grads(comm, g, P, stream)
            S.update_all(net, p, g, m, 0.9, 1e-3, LR, gb, stream)
        # lazy sequence (grads start as garbage: every step overwrites them)
        pb = [torch.from_numpy(p0.copy()).to(dev), torch.full((P,), float("nan"), device=dev)]
        mb = [torch.zeros(P, device=dev), torch.full((P,), float("nan"), device=dev)]
        gl = torch.full((P,), float("nan"), device=dev)
        cur, pending, paths = 0, 0, []
        for _ in range(steps):
            S.train_fwd_bwd_lazy(net, Xd, Td, tile, tile, batch, pb[cur], pb[1 - cur], mb[cur], mb[1 - cur],
                                 gl, 0.9, 1e-3, LR, pending, None, ws, nbytes, stream)
            paths.append(S.last_path())
            if pending:
                cur = 1 - cur
            S.allreduce_grads(comm, gl, P, stream)
            pending = gb
        S.update_all(net, pb[cur], gl, mb[cur], 0.9, 1e-3, LR, pending, stream)
        torch.cuda.synchronize()
    finally:
        S.comm_destroy(comm)
    assert set(paths) == {want}, paths
    bits = lambda t: t.cpu().numpy().view(np.uint32)  # noqa: E731
    assert not np.array_equal(bits(p), p0.view(np.uint32))
    assert np.array_equal(bits(pb[cur]), bits(p)), "parameters"
    assert np.array_equal(bits(mb[cur]), bits(m)), "momentum"
    assert not gl.cpu().numpy().any() and not g.cpu().numpy().any()


def test_lazy_rejects_overlap_and_applies_update_without_tiles(S):
    net = S.Net(64, 32, 9, 1, 5)
    P = S.net_param_count(net)
    dev = torch.device("cuda", 0)
    buf = torch.zeros(4 * P, device=dev)
    g = torch.zeros(P, device=dev)
    X = torch.zeros(33 * 33, device=dev)
    nbytes = S.train_workspace_bytes(net, 33, 33, 1)
    ws = torch.empty(nbytes // 4 + 64, device=dev)
    with pytest.raises(S.SrcnnError):  # params_out overlaps params_in
        S.train_fwd_bwd_lazy(net, X, X, 33, 33, 1, buf, buf[P // 2:], buf[2 * P:3 * P], buf[3 * P:], g,
                             0.9, 1e-3, LR, 4, None, ws, nbytes)
    # batch 0: the pending update alone, gradients zeroed (the reference's
    # update_parameters over an empty chunk)
    rng = np.random.default_rng(3)
    p0 = rng.standard_normal(P).astype(np.float32)
    g0 = rng.standard_normal(P).astype(np.float32)
    pi, po = torch.from_numpy(p0).to(dev), torch.zeros(P, device=dev)
    mi, mo = torch.zeros(P, device=dev), torch.zeros(P, device=dev)
    gd = torch.from_numpy(g0).to(dev)
    S.train_fwd_bwd_lazy(net, X, X, 33, 33, 0, pi, po, mi, mo, gd, 0.9, 1e-3, LR, 8, None, ws, nbytes)
    pr, gr, mr = pi.clone(), torch.from_numpy(g0).to(dev), mi.clone()
    S.update_all(net, pr, gr, mr, 0.9, 1e-3, LR, 8)
    torch.cuda.synchronize()
    assert np.array_equal(po.cpu().numpy(), pr.cpu().numpy())
    assert np.array_equal(mo.cpu().numpy(), mr.cpu().numpy())
    assert not gd.cpu().numpy().any()
