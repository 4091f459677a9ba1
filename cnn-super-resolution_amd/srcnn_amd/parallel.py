"""Data-parallel training step: one process per GPU, one gradient all-reduce.

SURVEY.md 8(e): tiles are independent, so a step shards the tile batch over
ranks (contiguous slices, rank r takes [r*B/N, (r+1)*B/N)), each rank
accumulates the gradients of its slice into the flat buffer
[gW1|gB1|gW2|gB2|gW3|gB3], ONE all-reduce(SUM) combines them (RCCL over xGMI
with the "nccl" backend; gloo in the CPU tests), and every rank applies the
same update with batch = global tile count, so the parameter replicas stay
identical.  This replaces the reference's single-queue
`execute_batch -> update_parameters` sequence
(src/ConfigBasedDataPipeline.cpp:128-195, :325-361; src/Main_cl.cpp:157-195)
for N devices.

Compute is injected (`fwd_bwd(grads)`, `update(batch)`): on a GPU these are
`srcnn_amd.train_fwd_bwd` / `srcnn_amd.update_all` on the HIP stream the
collective runs on; nothing here computes anything itself.

The collective is injected too.  Two implementations:
  SrcnnComm      the library's own RCCL stage (srcnn_comm_init_rank +
                 srcnn_allreduce_grads, include/srcnn.h) on the compute stream;
                 torch.distributed only ships the 128-byte RCCL id and runs
                 the barriers (the default of bench.py)
  torch          dist.all_reduce on the process group (RCCL with backend
                 "nccl"; gloo in the CPU tests and the one-GPU rehearsal)
"""
import contextlib
import datetime
import os
import sys

import torch
import torch.distributed as dist


def env_world():
    """(rank, world_size, local_rank) from the torch.distributed.run env."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


@contextlib.contextmanager
def _stdout_to_stderr():
    """fd-level redirect: gloo prints its "[Gloo] Rank r is connected ..."
    lines to stdout, where the bench's one JSON line must stand alone."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def init(backend, device=None, timeout_s=None):
    """init_process_group from the env (MASTER_ADDR defaults to 127.0.0.1).
    Collectives of the group time out after `timeout_s` (default
    SRCNN_DIST_TIMEOUT_S or 600 s) instead of torch's 30 minutes, so a rank
    left waiting on a peer that died fails instead of hanging."""
    rank, world, _ = env_world()
    if world <= 1:
        return rank, world
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if timeout_s is None:
        timeout_s = float(os.environ.get("SRCNN_DIST_TIMEOUT_S", "600"))
    kw = {"device_id": device} if device is not None and backend == "nccl" else {}
    kw["timeout"] = datetime.timedelta(seconds=timeout_s)
    with _stdout_to_stderr():
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
        dist.barrier()  # gloo connects its mesh lazily on some versions
    return rank, world


def shard(global_batch, rank, world):
    """Contiguous slice [start, start+count) of the global tile batch for `rank`
    (the remainder goes to the lowest ranks, one tile each)."""
    if global_batch < 0 or world < 1 or not 0 <= rank < world:
        raise ValueError("bad shard request")
    base, rem = divmod(global_batch, world)
    start = rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


def frame_band(w, h, net_dims, rank, world):
    """Row band of one frame for `rank` (inference shards by
    spatial tile with a halo and needs no collective).  The output rows of the
    valid convolution [0, h - ctx), ctx = f1 + f2 + f3 - 3 (the 12-row halo of
    the default net), are split contiguously as `shard` splits tiles; the
    band's input rows are its output rows plus ctx rows of context below.
    Rows are contiguous in the row-major frame, so a band is a plain slice of
    the input and output buffers: (in_row0, in_rows, out_row0, out_rows)."""
    f1, f2, f3 = net_dims
    ctx = f1 + f2 + f3 - 3
    if w <= ctx or h <= ctx:
        raise ValueError("frame smaller than the network's receptive field")
    o0, n = shard(h - ctx, rank, world)
    return o0, (n + ctx) if n else 0, o0, n


def forward_band(S, net, X, w, h, params, out, ws, ws_bytes, stream, rank, world):
    """srcnn_forward of this rank's row band of one w x h frame: X and out are
    the whole frame's (flat, row-major) input and output tensors; only the
    band's slices are read and written.  Returns the band's output row range."""
    i0, ni, o0, no = frame_band(w, h, (net.f1, net.f2, net.f3), rank, world)
    if no:
        ctx = net.f1 + net.f2 + net.f3 - 3
        ow = w - ctx
        S.forward(net, X[i0 * w:(i0 + ni) * w], w, ni, 1, params, out[o0 * ow:(o0 + no) * ow], ws,
                  ws_bytes, stream)
    return o0, no


class SrcnnComm:
    """RCCL communicator of libsrcnn_hip.so for this rank (one process per
    GPU): rank 0 makes the unique id (srcnn_comm_id), the process group
    broadcasts it, every rank calls srcnn_comm_init_rank on its current
    device.  `allreduce(buf, count)` = srcnn_allreduce_grads on `stream`."""

    def __init__(self, S, stream=None, group=None):
        self.S = S
        self.stream = stream
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        box = [S.comm_id() if self.rank == 0 else None]
        dist.broadcast_object_list(box, src=0, group=group)
        self.comm = S.comm_init_rank(self.world, box[0], self.rank)

    def __call__(self, grads):
        self.S.allreduce_grads(self.comm, grads, grads.numel(), self.stream)

    def close(self):
        if self.comm:
            self.S.comm_destroy(self.comm)
            self.comm = None


class DataParallelStep:
    """fwd_bwd(grads) accumulates this rank's gradients; update(global_batch)
    applies the SGD step and zeroes the gradients (srcnn_update_all).
    `allreduce(grads)` sums the flat gradient buffer over ranks in place
    (default: dist.all_reduce on `group`; SrcnnComm for the C-ABI stage)."""

    def __init__(self, grads, fwd_bwd, update, global_batch, group=None, allreduce=None):
        if not isinstance(grads, torch.Tensor) or grads.dtype != torch.float32:
            raise TypeError("grads must be a float32 tensor (the flat gradient buffer)")
        self.grads = grads
        self.fwd_bwd = fwd_bwd
        self.update = update
        self.global_batch = int(global_batch)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self._allreduce = allreduce

    def allreduce(self):
        """Sum the flat gradient buffer over ranks (one collective per step)."""
        if self.world <= 1:
            return
        if self._allreduce is not None:
            self._allreduce(self.grads)
        else:
            dist.all_reduce(self.grads, op=dist.ReduceOp.SUM, group=self.group)

    def __call__(self):
        self.fwd_bwd(self.grads)
        self.allreduce()
        self.update(self.global_batch)


class LazyDataParallelStep:
    """The same data-parallel training, one launch shorter per step: step t's
    SGD update is applied by step t + 1's first kernel
    (srcnn_train_fwd_bwd_lazy), so a step is
        fwd_bwd_lazy(p_in, p_out, m_in, m_out, grads, pending) -> allreduce(grads)
    with the parameter and momentum buffers ping-ponged (the update is out of
    place: every block of the first kernel reads the old values).  `pending`
    is the global batch of the update still owed (0 before the first step);
    `finish()` applies it (srcnn_update_all on the current buffers) and
    returns them.  Bit-identical to DataParallelStep's fwd_bwd -> allreduce ->
    update sequence.

    fwd_bwd_lazy(p_in, p_out, m_in, m_out, grads, pending) and
    update(params, mom, grads, batch) are injected as in DataParallelStep."""

    def __init__(self, params, params2, mom, mom2, grads, fwd_bwd_lazy, update, global_batch,
                 group=None, allreduce=None):
        for t in (params, params2, mom, mom2, grads):
            if not isinstance(t, torch.Tensor) or t.dtype != torch.float32:
                raise TypeError("parameter, momentum and gradient buffers must be float32 tensors")
        self.P = [params, params2]
        self.M = [mom, mom2]
        self.grads = grads
        self.fwd_bwd_lazy = fwd_bwd_lazy
        self.update = update
        self.global_batch = int(global_batch)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self._allreduce = allreduce
        self.cur = 0        # index of the buffers holding the current parameters
        self.pending = 0    # batch of the update not yet applied (0: none)

    def allreduce(self):
        if self.world <= 1:
            return
        if self._allreduce is not None:
            self._allreduce(self.grads)
        else:
            dist.all_reduce(self.grads, op=dist.ReduceOp.SUM, group=self.group)

    def __call__(self):
        i, o = self.cur, 1 - self.cur
        self.fwd_bwd_lazy(self.P[i], self.P[o], self.M[i], self.M[o], self.grads, self.pending)
        if self.pending:
            self.cur = o
        self.allreduce()
        self.pending = self.global_batch

    def finish(self):
        """Apply the owed update; returns (params, momentum) now current."""
        if self.pending:
            self.update(self.P[self.cur], self.M[self.cur], self.grads, self.pending)
            self.pending = 0
        return self.P[self.cur], self.M[self.cur]
