"""srcnn_amd -- Python binding of libsrcnn_hip.so over its C ABI (include/srcnn.h).

This is a thin ctypes layer: every call goes straight to an extern "C" entry
point of the HIP library; there is no Python or CPU implementation of any
operator behind it.  If the library is missing, importing this module fails
loudly (build it with `make -C cnn-super-resolution_amd`).

Device memory is passed as integer addresses, so torch tensors work
(`tensor.data_ptr()`), as do buffers from `malloc()` below.  torch is imported
first when available so that this library and torch share one HIP runtime.
"""
import ctypes
import os

try:  # share torch's HIP runtime (same SONAME) when torch is present
    import torch  # noqa: F401
except Exception:  # pragma: no cover - CLI-only environments
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
LIB_PATH = os.environ.get("SRCNN_HIP_LIB", os.path.join(PKG, "lib", "libsrcnn_hip.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError("libsrcnn_hip.so not built at %s (run `make -C %s`)" % (LIB_PATH, PKG))

_lib = ctypes.CDLL(LIB_PATH)

_P = ctypes.c_void_p
_U = ctypes.c_uint32
_I = ctypes.c_int
_F = ctypes.c_float
_S = ctypes.c_size_t


class Net(ctypes.Structure):
    """srcnn_net: Config n1, n2, f1, f2, f3 (reference src/Config.hpp:27-28)."""
    _fields_ = [("n1", _U), ("n2", _U), ("f1", _U), ("f2", _U), ("f3", _U)]

    def __repr__(self):
        return "Net(n1=%d, n2=%d, f1=%d, f2=%d, f3=%d)" % (self.n1, self.n2, self.f1, self.f2, self.f3)


_NP = ctypes.POINTER(Net)

# name -> (restype, argtypes); int restype = status code checked by _call
SIGNATURES = {
    "srcnn_abi_version": (_I, []),
    "srcnn_last_error": (ctypes.c_char_p, []),
    "srcnn_device_count": (_I, [ctypes.POINTER(_I)]),
    "srcnn_set_device": (_I, [_I]),
    "srcnn_device_name": (_I, [ctypes.c_char_p, _S]),
    "srcnn_malloc": (_I, [ctypes.POINTER(_P), _S]),
    "srcnn_free": (_I, [_P]),
    "srcnn_memcpy_h2d": (_I, [_P, _P, _S, _P]),
    "srcnn_memcpy_d2h": (_I, [_P, _P, _S, _P]),
    "srcnn_memcpy_d2d": (_I, [_P, _P, _S, _P]),
    "srcnn_fill_f32": (_I, [_P, _F, _S, _P]),
    "srcnn_stream_create": (_I, [ctypes.POINTER(_P)]),
    "srcnn_stream_destroy": (_I, [_P]),
    "srcnn_stream_sync": (_I, [_P]),
    "srcnn_device_sync": (_I, []),
    "srcnn_event_create": (_I, [ctypes.POINTER(_P)]),
    "srcnn_event_destroy": (_I, [_P]),
    "srcnn_event_record": (_I, [_P, _P]),
    "srcnn_event_sync": (_I, [_P]),
    "srcnn_event_elapsed_ms": (_I, [_P, _P, ctypes.POINTER(_F)]),
    "srcnn_graph_begin": (_I, [_P]),
    "srcnn_graph_end": (_I, [_P, ctypes.POINTER(_P)]),
    "srcnn_graph_launch": (_I, [_P, _P]),
    "srcnn_graph_destroy": (_I, [_P]),
    "srcnn_conv_fwd": (_I, [_P, _P, _P, _P, _U, _U, _U, _U, _U, _I, _U, _P]),
    "srcnn_last_delta": (_I, [_P, _P, _P, _U, _U, _U, _U, _U, _P]),
    "srcnn_conv_delta": (_I, [_P, _P, _P, _P, _U, _U, _U, _U, _U, _U, _P]),
    "srcnn_conv_grad_workspace_bytes": (_S, [_U, _U, _U, _U, _U, _U]),
    "srcnn_conv_grad_acc": (_I, [_P, _P, _P, _P, _U, _U, _U, _U, _U, _U, _P, _S, _P]),
    "srcnn_sgd_update": (_I, [_P, _P, _P, _P, _P, _P, _F, _F, _F, _U, _U, _U, _P]),
    "srcnn_reduce_workspace_bytes": (_S, [_S]),
    "srcnn_sq_err": (_I, [_P, _P, _P, _U, _U, _U, _U, _U, _P, _S, _P]),
    "srcnn_sum": (_I, [_P, _S, _I, _P, _P, _S, _P]),
    "srcnn_sub_scalar": (_I, [_P, _F, _S, _P]),
    "srcnn_sub_mean": (_I, [_P, _S, _P, _P, _S, _P]),
    "srcnn_extract_luma": (_I, [_P, _P, _U, _U, _I, _P]),
    "srcnn_swap_luma": (_I, [_P, _P, _P, _U, _U, _U, _U, _P]),
    "srcnn_net_offsets": (_I, [_NP, ctypes.POINTER(_S)]),
    "srcnn_net_param_count": (_S, [_NP]),
    "srcnn_train_workspace_bytes": (_S, [_NP, _U, _U, _U]),
    "srcnn_train_fwd_bwd": (_I, [_NP, _P, _P, _U, _U, _U, _P, _P, _P, _P, _S, _P]),
    "srcnn_update_all": (_I, [_NP, _P, _P, _P, _F, _F, ctypes.POINTER(_F), _U, _P]),
    "srcnn_train_step": (_I, [_NP, _P, _P, _U, _U, _U, _P, _P, _P, _F, _F, ctypes.POINTER(_F), _U,
                              _P, _P, _S, _P]),
    "srcnn_train_fwd_bwd_lazy": (_I, [_NP, _P, _P, _U, _U, _U, _P, _P, _P, _P, _P, _F, _F,
                                      ctypes.POINTER(_F), _U, _P, _P, _S, _P]),
    "srcnn_train_activations":(_I, [_NP, _U, _U, _U, _P, _S, _P, _P, _P, _P]),
    "srcnn_preload": (_I, [_NP]),
    "srcnn_forward_workspace_bytes": (_S, [_NP, _U, _U, _U]),
    "srcnn_forward": (_I, [_NP, _P, _U, _U, _U, _P, _P, _P, _S, _P]),
    "srcnn_profile_enable": (_I, [_I]),
    "srcnn_profile_reset": (_I, []),
    "srcnn_profile_count": (_I, [ctypes.POINTER(_I)]),
    "srcnn_profile_get": (_I, [_I, ctypes.c_char_p, _S, ctypes.POINTER(ctypes.c_uint64),
                               ctypes.POINTER(ctypes.c_double)]),
    "srcnn_profile_print": (_I, []),
    "srcnn_profile_clock": (_I, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double)]),
    "srcnn_set_path": (_I, [_I]),
    "srcnn_set_arith": (_I, [_I]),
    "srcnn_get_arith": (_I, []),
    "srcnn_get_path": (_I, []),
    "srcnn_last_path": (ctypes.c_char_p, []),
    "srcnn_last_kernels": (ctypes.c_char_p, []),
    "srcnn_comm_id": (_I, [ctypes.c_char_p]),
    "srcnn_comm_init_rank": (_I, [ctypes.POINTER(_P), _I, ctypes.c_char_p, _I]),
    "srcnn_comm_init_all": (_I, [ctypes.POINTER(_P), _I, ctypes.POINTER(_I)]),
    "srcnn_comm_destroy": (_I, [_P]),
    "srcnn_comm_rank": (_I, [_P, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "srcnn_comm_group_start": (_I, []),
    "srcnn_comm_group_end": (_I, []),
    "srcnn_allreduce_grads": (_I, [_P, _P, _S, _P]),
    "srcnn_comm_version": (_I, [ctypes.POINTER(_I), ctypes.c_char_p, _S]),
}

for _name, (_res, _args) in SIGNATURES.items():
    _fn = getattr(_lib, _name)
    _fn.restype = _res
    _fn.argtypes = _args


class SrcnnError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("srcnn error %d: %s" % (code, msg))
        self.code = code


OK, ERR_INVALID, ERR_HIP, ERR_WORKSPACE, ERR_ALLOC, ERR_COMM = 0, -1, -2, -3, -4, -5
COMM_ID_BYTES = 128


def _call(name, *args):
    rc = getattr(_lib, name)(*args)
    if rc != 0:
        raise SrcnnError(rc, _lib.srcnn_last_error().decode())
    return rc


def lib():
    return _lib


def last_error():
    return _lib.srcnn_last_error().decode()


def abi_version():
    return _lib.srcnn_abi_version()


def exported_symbols():
    return list(SIGNATURES)


def ptr(t):
    """Device address of a torch tensor / int / None."""
    if t is None:
        return None
    if isinstance(t, int):
        return t
    return t.data_ptr()


def cur_stream():
    """hipStream_t of torch's current stream (0 = default)."""
    if torch is None:
        return None
    return torch.cuda.current_stream().cuda_stream


# ---- runtime ----
def device_count():
    c = _I()
    _call("srcnn_device_count", ctypes.byref(c))
    return c.value


def set_device(d):
    _call("srcnn_set_device", d)


def device_name():
    buf = ctypes.create_string_buffer(256)
    _call("srcnn_device_name", buf, 256)
    return buf.value.decode()


def malloc(nbytes):
    p = _P()
    _call("srcnn_malloc", ctypes.byref(p), nbytes)
    return p.value or 0


def free(p):
    _call("srcnn_free", p)


def stream_create():
    s = _P()
    _call("srcnn_stream_create", ctypes.byref(s))
    return s.value


def stream_sync(s=None):
    _call("srcnn_stream_sync", s)


def event_create():
    e = _P()
    _call("srcnn_event_create", ctypes.byref(e))
    return e.value


def event_record(e, s=None):
    _call("srcnn_event_record", e, s)


def event_sync(e):
    _call("srcnn_event_sync", e)


def event_elapsed_ms(a, b):
    ms = _F()
    _call("srcnn_event_elapsed_ms", a, b, ctypes.byref(ms))
    return ms.value


def event_destroy(e):
    _call("srcnn_event_destroy", e)


def memcpy_h2d(dst, src_addr, nbytes, s=None):
    _call("srcnn_memcpy_h2d", dst, src_addr, nbytes, s)


def memcpy_d2h(dst_addr, src, nbytes, s=None):
    _call("srcnn_memcpy_d2h", dst_addr, src, nbytes, s)


def fill_f32(dst, value, count, s=None):
    _call("srcnn_fill_f32", ptr(dst), value, count, s)


# ---- operators (argument order = include/srcnn.h) ----
def conv_fwd(inp, out, W, B, in_w, in_h, n_prev, n_cur, f, relu, batch, s=None):
    _call("srcnn_conv_fwd", ptr(inp), ptr(out), ptr(W), ptr(B), in_w, in_h, n_prev, n_cur, f,
          int(relu), batch, s)


def last_delta(gt, y, d, gt_w, gt_h, out_w, out_h, batch, s=None):
    _call("srcnn_last_delta", ptr(gt), ptr(y), ptr(d), gt_w, gt_h, out_w, out_h, batch, s)


def conv_delta(d_next, y_curr, d_curr, W_next, f_next, n_curr, n_next, curr_w, curr_h, batch, s=None):
    _call("srcnn_conv_delta", ptr(d_next), ptr(y_curr), ptr(d_curr), ptr(W_next), f_next, n_curr,
          n_next, curr_w, curr_h, batch, s)


def conv_grad_workspace_bytes(n_prev, n_cur, f, out_w, out_h, batch):
    return _lib.srcnn_conv_grad_workspace_bytes(n_prev, n_cur, f, out_w, out_h, batch)


def conv_grad_acc(inp, delta, gW, gB, n_prev, n_cur, f, out_w, out_h, batch, ws, ws_bytes, s=None):
    _call("srcnn_conv_grad_acc", ptr(inp), ptr(delta), ptr(gW), ptr(gB), n_prev, n_cur, f, out_w,
          out_h, batch, ptr(ws), ws_bytes, s)


def sgd_update(W, B, gW, gB, dW, dB, momentum, wd, lr, batch, nW, nB, s=None):
    _call("srcnn_sgd_update", ptr(W), ptr(B), ptr(gW), ptr(gB), ptr(dW), ptr(dB), momentum, wd, lr,
          batch, nW, nB, s)


def reduce_workspace_bytes(n):
    return _lib.srcnn_reduce_workspace_bytes(n)


def sq_err(gt, y, result, gt_w, gt_h, out_w, out_h, batch, ws, ws_bytes, s=None):
    _call("srcnn_sq_err", ptr(gt), ptr(y), ptr(result), gt_w, gt_h, out_w, out_h, batch, ptr(ws),
          ws_bytes, s)


def buf_sum(data, n, squared, result, ws, ws_bytes, s=None):
    _call("srcnn_sum", ptr(data), n, int(squared), ptr(result), ptr(ws), ws_bytes, s)


def sub_scalar(data, value, n, s=None):
    _call("srcnn_sub_scalar", ptr(data), value, n, s)


def sub_mean(data, n, mean, ws, ws_bytes, s=None):
    _call("srcnn_sub_mean", ptr(data), n, ptr(mean), ptr(ws), ws_bytes, s)


def extract_luma(rgba, luma, w, h, normalize, s=None):
    _call("srcnn_extract_luma", ptr(rgba), ptr(luma), w, h, int(normalize), s)


def swap_luma(rgba, new_luma, rgb, w, h, luma_w, luma_h, s=None):
    _call("srcnn_swap_luma", ptr(rgba), ptr(new_luma), ptr(rgb), w, h, luma_w, luma_h, s)


# ---- network level ----
def net_offsets(net):
    arr = (_S * 6)()
    _call("srcnn_net_offsets", ctypes.byref(net), arr)
    return list(arr)


def net_param_count(net):
    return _lib.srcnn_net_param_count(ctypes.byref(net))


def train_workspace_bytes(net, w, h, batch):
    return _lib.srcnn_train_workspace_bytes(ctypes.byref(net), w, h, batch)


def train_fwd_bwd(net, X, T, w, h, batch, params, grads, sq_err_dev, ws, ws_bytes, s=None):
    _call("srcnn_train_fwd_bwd", ctypes.byref(net), ptr(X), ptr(T), w, h, batch, ptr(params),
          ptr(grads), ptr(sq_err_dev), ptr(ws), ws_bytes, s)


def update_all(net, params, grads, mom, momentum, wd, lr, batch, s=None):
    lr_arr = (_F * 3)(*lr)
    _call("srcnn_update_all", ctypes.byref(net), ptr(params), ptr(grads), ptr(mom), momentum, wd,
          lr_arr, batch, s)


def train_step(net, X, T, w, h, batch, params, grads, mom, momentum, wd, lr, update_batch,
               sq_err_dev, ws, ws_bytes, s=None):
    """srcnn_train_step: train_fwd_bwd + update_all on one device (the update
    fused into the gradient reduction on the fused path)."""
    lr_arr = (_F * 3)(*lr)
    _call("srcnn_train_step", ctypes.byref(net), ptr(X), ptr(T), w, h, batch, ptr(params),
          ptr(grads), ptr(mom), momentum, wd, lr_arr, update_batch, ptr(sq_err_dev), ptr(ws),
          ws_bytes, s)


def train_fwd_bwd_lazy(net, X, T, w, h, batch, params_in, params_out, mom_in, mom_out, grads,
                       momentum, wd, lr, update_batch, sq_err_dev, ws, ws_bytes, s=None):
    """srcnn_train_fwd_bwd_lazy: the pending update of `grads` (update_batch
    > 0) out of place into params_out / mom_out, then this step's gradients
    over the batch on the updated parameters, written to `grads`."""
    lr_arr = (_F * 3)(*lr)
    _call("srcnn_train_fwd_bwd_lazy", ctypes.byref(net), ptr(X), ptr(T), w, h, batch, ptr(params_in),
          ptr(params_out), ptr(mom_in), ptr(mom_out), ptr(grads), momentum, wd, lr_arr, update_batch,
          ptr(sq_err_dev), ptr(ws), ws_bytes, s)


class Graph:
    """A replayable HIP graph of the library calls `fn()` enqueues on `stream`
    (srcnn_graph_begin / _end); `launch()` replays it on the same stream."""

    def __init__(self, fn, stream):
        if not stream:
            raise ValueError("graph capture needs a created stream (not the NULL stream)")
        self.stream = stream
        self.handle = _P()
        _call("srcnn_graph_begin", stream)
        try:
            fn()
        finally:
            _call("srcnn_graph_end", stream, ctypes.byref(self.handle))

    def launch(self):
        _call("srcnn_graph_launch", self.handle, self.stream)

    def close(self):
        if self.handle:
            _call("srcnn_graph_destroy", self.handle)
            self.handle = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def train_activations(net, w, h, batch, ws, ws_bytes, A1, A2, A3, s=None):
    """srcnn_train_activations: the last training call's activations of the
    three layers in `ws`, copied out in the reference HWC layout."""
    _call("srcnn_train_activations", ctypes.byref(net), w, h, batch, ptr(ws), ws_bytes, ptr(A1),
          ptr(A2), ptr(A3), s)


def forward_workspace_bytes(net, w, h, batch):
    return _lib.srcnn_forward_workspace_bytes(ctypes.byref(net), w, h, batch)


def forward(net, X, w, h, batch, params, out, ws, ws_bytes, s=None):
    _call("srcnn_forward", ctypes.byref(net), ptr(X), w, h, batch, ptr(params), ptr(out), ptr(ws),
          ws_bytes, s)


def set_path(p):
    _call("srcnn_set_path", p)


def set_arith(a):
    """0: split-bf16 matrix-core products (default), 1: fp32 MFMA only."""
    _call("srcnn_set_arith", a)


def get_arith():
    return _lib.srcnn_get_arith()


def get_path():
    return _lib.srcnn_get_path()


def preload(net):
    """Resolve the net's gfx950 kernels on the current device (srcnn_preload):
    the runtime's lazy kernel setup happens here, not in the first step."""
    _call("srcnn_preload", ctypes.byref(net))


def last_kernels():
    """Kernel variants of this thread's most recent training call, as a list
    (srcnn_last_kernels), e.g. ["l12_fwd", "l3r_delta", "d1c_grad12", ...]."""
    v = _lib.srcnn_last_kernels().decode()
    return v.split(",") if v else []


def last_path():
    """Kernel family of this thread's most recent conv / network call:
    "fused", "wide", "fast", "generic" or "" (srcnn_last_path)."""
    return _lib.srcnn_last_path().decode()


# ---- multi-GPU: RCCL gradient reduction (srcnn_comm_*, srcnn_allreduce_grads) ----
def comm_id():
    """128-byte RCCL unique id (ncclGetUniqueId), made on ONE rank."""
    buf = ctypes.create_string_buffer(COMM_ID_BYTES)
    _call("srcnn_comm_id", buf)
    return buf.raw


def comm_init_rank(nranks, uid, rank):
    """Communicator of `rank` on the current device (one process per GPU)."""
    if len(uid) != COMM_ID_BYTES:
        raise ValueError("comm id must be %d bytes" % COMM_ID_BYTES)
    c = _P()
    _call("srcnn_comm_init_rank", ctypes.byref(c), nranks, uid, rank)
    return c.value


def comm_init_all(devices):
    """One communicator per device of one process (ncclCommInitAll)."""
    n = len(devices)
    comms = (_P * n)()
    devs = (_I * n)(*devices)
    _call("srcnn_comm_init_all", comms, n, devs)
    return list(comms)


def comm_destroy(c):
    _call("srcnn_comm_destroy", c)


def comm_rank(c):
    r, n = _I(), _I()
    _call("srcnn_comm_rank", c, ctypes.byref(r), ctypes.byref(n))
    return r.value, n.value


def comm_version():
    """(RCCL version code, path of the librccl the library is bound to)."""
    v = _I()
    buf = ctypes.create_string_buffer(4096)
    _call("srcnn_comm_version", ctypes.byref(v), buf, len(buf))
    return v.value, buf.value.decode()


def allreduce_grads(c, buf, count, s=None):
    """In-place sum of `count` floats over all ranks, on stream `s`."""
    _call("srcnn_allreduce_grads", c, ptr(buf), count, s)


# ---- profiling (reference `profile` mode) ----
def profile_enable(on=True):
    _call("srcnn_profile_enable", int(bool(on)))


def profile_reset():
    _call("srcnn_profile_reset")


def profile_stats():
    """{kernel name: (launches, total_ms)}; waits for recorded events."""
    n = _I()
    _call("srcnn_profile_count", ctypes.byref(n))
    out = {}
    buf = ctypes.create_string_buffer(256)
    for i in range(n.value):
        cnt, ms = ctypes.c_uint64(), ctypes.c_double()
        _call("srcnn_profile_get", i, buf, 256, ctypes.byref(cnt), ctypes.byref(ms))
        out[buf.value.decode()] = (cnt.value, ms.value)
    return out


def profile_clock(kernel):
    """Shader clock (GHz) held during the last launch of a fused kernel, or None."""
    ghz = ctypes.c_double()
    _call("srcnn_profile_clock", kernel.encode(), ctypes.byref(ghz))
    return ghz.value if ghz.value > 0 else None


def profile_print():
    _call("srcnn_profile_print")
