"""bench.py's multi-rank path end to end on CPU, with a stand-in library.

The first run of `bench.py --gpus N --comm srcnn` with N > 1 ranks on real
GPUs is the driver's 8-GPU node (RCCL refuses two ranks on one device, so the
one-GPU box cannot run it).  Here two gloo ranks run `bench.main` itself up
to and through the library calls, with `S` replaced by StubS: a recording
stand-in for srcnn_amd (no kernels; its all-reduce is a real gloo collective
on CPU tensors) and a CPU device object in place of CudaDevice.  Checked:
  - the RCCL id made on rank 0 reaches every rank's srcnn_comm_init_rank;
  - a communicator reporting another rank count ends every rank non-zero
    before any step, with no JSON line;
  - every rank issues the same collectives, one per step, in the weak and the
    strong sub-records, settle() steps included (their count agreed over the
    ranks), and the lazy step's update flags follow the ping-pong contract;
  - an exception on one rank ends every rank non-zero well inside the group
    timeout (no peer left blocked in a collective);
  - the HIP-graph branch is agreed before any replay (advisor r04).
Reference loop being sharded: src/Main_cl.cpp:161-195,
src/ConfigBasedDataPipeline.cpp:325-361.
"""
import contextlib
import json
import multiprocessing as mp
import os
import socket
import sys
import time

import torch

from conftest import ROOT

P_DEFAULT = 8129  # default net's flat parameter count


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class CpuDevice:
    """CudaDevice stand-in: CPU tensors, no stream, nothing to sync."""
    dev = torch.device("cpu")
    stream = None

    def sync(self):
        pass

    def on_stream(self):
        return contextlib.nullcontext()


class StubError(RuntimeError):
    pass


class StubS:
    """Recording stand-in for the srcnn_amd binding (the calls bench.py
    makes).  Every call is appended to self.log; allreduce_grads is a real
    gloo all-reduce so mismatched collective counts would hang / fail."""
    SrcnnError = StubError

    class Net:
        def __init__(self, n1, n2, f1, f2, f3):
            self.n1, self.n2, self.f1, self.f2, self.f3 = n1, n2, f1, f2, f3

    def __init__(self, rank, log_path, comm_ranks=None, fail_at=None, step_sleep=0.0):
        self.rank = rank
        self.log = []
        self.log_path = log_path
        self.comm_ranks = comm_ranks
        self.fail_at = fail_at
        self.step_sleep = step_sleep
        self.steps = 0

    def _rec(self, *ev):
        self.log.append(list(ev))
        with open(self.log_path, "w") as fh:
            json.dump(self.log, fh)

    # runtime / profiling
    def set_path(self, p):
        self._rec("set_path", p)

    def preload(self, net):
        self._rec("preload")

    def net_param_count(self, net):
        return P_DEFAULT

    def train_workspace_bytes(self, net, w, h, batch):
        return 256

    def profile_reset(self):
        self._rec("profile_reset")

    def profile_enable(self, on):
        pass

    def profile_stats(self):
        return {}

    def profile_clock(self, name):
        return None

    def last_path(self):
        return "stub"

    # training
    def _step(self, kind, batch):
        self.steps += 1
        if self.fail_at is not None and self.steps == self.fail_at:
            self._rec("raise", kind, batch)
            raise StubError("injected failure on rank %d at call %d" % (self.rank, self.steps))
        if self.step_sleep:
            time.sleep(self.step_sleep)

    def train_fwd_bwd_lazy(self, net, X, T, w, h, batch, pin, pout, min_, mout, grads, mu, wd, lr,
                           pending, sq, ws, wsb, stream):
        self._rec("lazy", batch, pending, pin.data_ptr() != pout.data_ptr())
        self._step("lazy", batch)
        if pending:  # out of place, as the library (values irrelevant here)
            pout.copy_(pin - 1e-3 * grads / pending)
            mout.copy_(min_)
        grads.fill_(float(self.rank + 1))

    def train_fwd_bwd(self, net, X, T, w, h, batch, params, grads, sq, ws, wsb, stream):
        self._rec("fwd_bwd", batch)
        self._step("fwd_bwd", batch)
        grads.add_(float(self.rank + 1))

    def update_all(self, net, params, grads, mom, mu, wd, lr, batch, stream):
        self._rec("update", batch)
        params.sub_(1e-3 * grads / batch)
        grads.zero_()

    def train_step(self, *a):
        self._rec("train_step")
        self._step("train_step", a[5])

    # RCCL stage
    def comm_id(self):
        uid = bytes((self.rank * 7 + i * 13) % 256 for i in range(128))
        self._rec("comm_id", uid.hex())
        return uid

    def comm_init_rank(self, n, uid, rank):
        self._rec("comm_init_rank", uid.hex(), n, rank)
        return 0xC0FFEE

    def comm_rank(self, c):
        world = int(os.environ["WORLD_SIZE"])
        return self.rank, self.comm_ranks if self.comm_ranks is not None else world

    def allreduce_grads(self, c, buf, count, s):
        import torch.distributed as dist
        self._rec("allreduce", int(count))
        dist.all_reduce(buf, op=dist.ReduceOp.SUM)

    def comm_destroy(self, c):
        self._rec("comm_destroy")

    class Graph:  # replaced per instance when a test needs capture
        def __init__(self, fn, stream):
            raise StubError("no graphs in the stand-in")


def _rank_main(rank, world, port, argv, out_dir, stub_kw):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SRCNN_DIST_TIMEOUT_S="60")
    for k in ("TORCHELASTIC_RUN_ID",):
        os.environ.pop(k, None)
    out = open(os.path.join(out_dir, "out_%d.txt" % rank), "w")
    err = open(os.path.join(out_dir, "err_%d.txt" % rank), "w")
    os.dup2(out.fileno(), 1)
    os.dup2(err.fileno(), 2)
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "cnn-super-resolution_amd"))
    import bench
    kw = dict(stub_kw.get("all", {}))
    kw.update(stub_kw.get(rank, {}))
    S = StubS(rank, os.path.join(out_dir, "log_%d.json" % rank), **kw)
    bench.main(argv, S=S, device=CpuDevice())


def _run_ranks(tmp_path, argv, world=2, stub_kw=None, timeout=150):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, argv, str(tmp_path), stub_kw or {}))
             for r in range(world)]
    t0 = time.time()
    for p in procs:
        p.start()
    for p in procs:
        p.join(max(1.0, timeout - (time.time() - t0)))
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
        p.join()
    assert not alive, "rank(s) still running after %ds: a peer is blocked" % timeout
    logs = []
    for r in range(world):
        path = tmp_path / ("log_%d.json" % r)
        logs.append(json.loads(path.read_text()) if path.exists() else [])
    outs = [(tmp_path / ("out_%d.txt" % r)).read_text() for r in range(world)]
    errs = [(tmp_path / ("err_%d.txt" % r)).read_text() for r in range(world)]
    return [p.exitcode for p in procs], logs, outs, errs, time.time() - t0


BASE = ["--gpus", "2", "--no-wide", "--no-forward", "--no-cpu-baseline", "--batch", "8"]


def _collectives(log):
    return [e for e in log if e[0] in ("allreduce", "lazy", "fwd_bwd", "update")]


def _phases(log):
    """split a rank's lazy steps by batch: weak (8 tiles) and strong (2048)"""
    out = {}
    for e in log:
        if e[0] == "lazy":
            out.setdefault(e[1], []).append(e)
    return out


def test_two_ranks_same_collectives_per_step(tmp_path):
    steps, warmup = 3, 2
    codes, logs, outs, errs, _ = _run_ranks(
        tmp_path, BASE + ["--steps", str(steps), "--warmup", str(warmup), "--settle-ms", "0"])
    assert codes == [0, 0], errs
    # the RCCL id: made once, on rank 0, and the same bytes reach both ranks
    ids = [e for e in logs[0] if e[0] == "comm_id"]
    assert len(ids) == 1 and not [e for e in logs[1] if e[0] == "comm_id"]
    inits = [[e for e in lg if e[0] == "comm_init_rank"] for lg in logs]
    assert [i[0][1] for i in inits] == [ids[0][1]] * 2
    assert [i[0][2:] for i in inits] == [[2, 0], [2, 1]]
    # identical collective sequences on both ranks
    assert _collectives(logs[0]) == [e for e in _collectives(logs[1])]
    per = _phases(logs[0])
    n = steps + warmup + 3 * 0  # settle off
    assert sorted(per) == [8, 2048]  # weak (--batch 8) and strong (4096 / 2) sub-records
    for batch, evs in per.items():
        assert len(evs) == n
        # the first step of a region owes nothing; every later one applies the
        # previous step's update (global batch), out of place
        assert evs[0][2] == 0 and all(e[2] == (16 if batch == 8 else 4096) for e in evs[1:])
        assert all(e[3] for e in evs)
    ar = [e for e in logs[0] if e[0] == "allreduce"]
    assert len(ar) == 2 * n and all(e[1] == P_DEFAULT for e in ar)
    # each region's owed update is applied once after its timed steps
    assert [e[1] for e in logs[0] if e[0] == "update"] == [16, 4096]
    # one JSON line on rank 0, none on rank 1
    line = json.loads(outs[0].strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["config"]["rccl_ranks"] == 2
    assert line["config"]["grad_allreduce"] == "srcnn_allreduce_grads (RCCL)"
    assert "lazy" in line["config"]["step_call"]
    assert line["strong"]["batch_per_gpu"] == 2048 and line["strong"]["steps"] == steps
    assert outs[1].strip() == ""


def test_settle_steps_agreed_over_ranks(tmp_path):
    """settle(): the ranks measure different step times (rank 1 sleeps 4x
    longer) but must run the same number of settle steps (MAX)."""
    codes, logs, outs, errs, _ = _run_ranks(
        tmp_path, BASE + ["--steps", "2", "--warmup", "1", "--settle-ms", "20", "--no-strong"],
        stub_kw={0: {"step_sleep": 0.001}, 1: {"step_sleep": 0.004}})
    assert codes == [0, 0], errs
    n0 = len([e for e in logs[0] if e[0] == "allreduce"])
    n1 = len([e for e in logs[1] if e[0] == "allreduce"])
    assert n0 == n1 > 2 + 1 + 3
    line = json.loads(outs[0].strip().splitlines()[-1])
    assert line["config"]["settle_steps"] == n0 - 3


def test_separate_update_step(tmp_path):
    codes, logs, outs, errs, _ = _run_ranks(
        tmp_path, BASE + ["--steps", "2", "--warmup", "1", "--settle-ms", "0", "--no-strong",
                          "--dp-step", "separate"])
    assert codes == [0, 0], errs
    seq = [e[0] for e in logs[0] if e[0] in ("fwd_bwd", "allreduce", "update")]
    assert seq == ["fwd_bwd", "allreduce", "update"] * 3
    assert _collectives(logs[0]) == _collectives(logs[1])


def test_rccl_rank_count_mismatch_exits_every_rank(tmp_path):
    codes, logs, outs, errs, _ = _run_ranks(
        tmp_path, BASE + ["--steps", "2", "--warmup", "1", "--settle-ms", "0"],
        stub_kw={"all": {"comm_ranks": 3}})
    assert all(c != 0 for c in codes), codes
    assert all("RCCL communicator has rank" in e for e in errs)
    assert not any(e[0] in ("lazy", "allreduce") for lg in logs for e in lg)
    assert outs[0].strip() == ""


def test_failure_on_one_rank_ends_every_rank(tmp_path):
    """rank 1 raises inside its 3rd step while rank 0 proceeds to that step's
    all-reduce: both must exit non-zero, long before the 60 s group timeout."""
    codes, logs, outs, errs, took = _run_ranks(
        tmp_path, BASE + ["--steps", "3", "--warmup", "2", "--settle-ms", "0"],
        stub_kw={1: {"fail_at": 3}})
    assert codes[1] != 0 and codes[0] != 0, codes
    assert "injected failure on rank 1" in errs[1]
    assert took < 45, took
    assert outs[0].strip() == ""


def _graph_rank(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "cnn-super-resolution_amd"))
    import bench
    import torch.distributed as dist
    from srcnn_amd import parallel
    parallel.init("gloo", timeout_s=60)
    S = StubS(rank, os.path.join(out_dir, "log_%d.json" % rank))
    calls = {"direct": 0, "replay": 0}
    t = torch.zeros(4)

    class Graph:  # rank 0 captures, rank 1 fails
        def __init__(self, fn, stream):
            if rank == 1:
                raise StubError("capture failed")

        def launch(self):
            calls["replay"] += 1
            dist.all_reduce(t)

        def close(self):
            pass

    S.Graph = Graph

    def step():
        calls["direct"] += 1
        dist.all_reduce(t)

    bench.timed_region(step, 3, 1, world, 1, None, S, True, "gloo", torch.device("cpu"), lambda: None)
    with open(os.path.join(out_dir, "calls_%d.json" % rank), "w") as fh:
        json.dump(calls, fh)
    dist.destroy_process_group()


def test_graph_agreed_before_any_replay(tmp_path):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_graph_rank, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert [p.exitcode for p in procs] == [0, 0]
    calls = [json.loads((tmp_path / ("calls_%d.json" % r)).read_text()) for r in range(2)]
    # nobody replayed (rank 1 could not capture), both ran the same direct steps
    assert calls[0] == calls[1] == {"direct": 1 + 3, "replay": 0}
