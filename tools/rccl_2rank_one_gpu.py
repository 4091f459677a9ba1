"""Probe: can the library's RCCL stage (srcnn_comm_init_rank +
srcnn_allreduce_grads) form a 2-rank communicator with both ranks on device 0
of a one-GPU box?  Not a test (RCCL normally takes one rank per device); it
records what RCCL does.  Each rank all-reduces a gradient-sized buffer
(8,129 floats, the default net) holding rank + 1 and checks the sum.

  timeout -k 10 90 python tools/rccl_2rank_one_gpu.py
"""
import multiprocessing as mp
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cnn-super-resolution_amd"))

P = 8129


def rank_main(rank, nranks, q_id, q_out):
    try:
        import torch
        import srcnn_amd as S
        torch.cuda.set_device(0)
        if rank == 0:
            uid = S.comm_id()
            for _ in range(nranks - 1):
                q_id.put(uid)
        else:
            uid = q_id.get(timeout=30)
        comm = S.comm_init_rank(nranks, uid, rank)
        r, n = S.comm_rank(comm)
        buf = torch.full((P,), float(rank + 1), device="cuda:0")
        for _ in range(3):
            buf.fill_(float(rank + 1))
            S.allreduce_grads(comm, buf, P, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        want = nranks * (nranks + 1) / 2
        ok = bool((buf == want).all().item())
        S.comm_destroy(comm)
        q_out.put((rank, "ok" if ok else "wrong sum %r" % buf[:4].tolist(), r, n, S.comm_version()))
    except Exception as e:  # report, do not hang the parent
        q_out.put((rank, "error: %s" % e, None, None, traceback.format_exc()[-400:]))


def main():
    ctx = mp.get_context("spawn")
    q_id, q_out = ctx.Queue(), ctx.Queue()
    nranks = 2
    ps = [ctx.Process(target=rank_main, args=(r, nranks, q_id, q_out)) for r in range(nranks)]
    for p in ps:
        p.start()
    res = []
    for _ in ps:
        try:
            res.append(q_out.get(timeout=75))
        except Exception:
            res.append(("?", "no answer within 75 s", None, None, None))
    for p in ps:
        p.join(timeout=5)
        if p.is_alive():
            p.kill()
    for r in sorted(res, key=lambda t: str(t[0])):
        print("rank", r[0], r[1], "comm rank/size", r[2], r[3], r[4])
    return 0 if all(r[1] == "ok" for r in res) else 1


if __name__ == "__main__":
    sys.exit(main())
