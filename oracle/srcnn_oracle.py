"""ctypes/numpy front-end of the CPU oracle (oracle/srcnn_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product path.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libsrcnn_oracle.so")

_f32p = ctypes.POINTER(ctypes.c_float)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        i, f, sz, u = ctypes.c_int, ctypes.c_float, ctypes.c_size_t, ctypes.c_uint
        sig = {
            "oracle_set_threads": [i],
            "oracle_conv_fwd": [_f32p, _f32p, _f32p, _f32p, i, i, i, i, i, i, i],
            "oracle_last_delta": [_f32p, _f32p, _f32p, i, i, i, i, i],
            "oracle_conv_delta": [_f32p, _f32p, _f32p, _f32p, i, i, i, i, i, i],
            "oracle_conv_grad_acc": [_f32p, _f32p, _f32p, _f32p, i, i, i, i, i, i],
            "oracle_sgd_update": [_f32p, _f32p, _f32p, _f32p, _f32p, _f32p, f, f, f, u, i, i],
            "oracle_sq_err": [_f32p, _f32p, i, i, i, i, i],
            "oracle_sum": [_f32p, sz, i],
            "oracle_sub_from_all": [_f32p, f, sz],
            "oracle_extract_luma": [_u8p, _f32p, i, i, i],
            "oracle_swap_luma": [_u8p, _f32p, _u8p, i, i, i, i],
            "oracle_param_count": [i, i, i, i, i],
            "oracle_train_acts_floats": [i, i, i, i, i, i, i, i],
            "oracle_train_fwd_bwd": [i, i, i, i, i, _f32p, _f32p, i, i, i, _f32p, _f32p, _f32p],
            "oracle_update_all": [i, i, i, i, i, _f32p, _f32p, _f32p, f, f, _f32p, u],
            "oracle_forward": [i, i, i, i, i, _f32p, i, i, i, _f32p, _f32p],
        }
        for name, argt in sig.items():
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = None
        L.oracle_set_threads.restype = ctypes.c_int
        L.oracle_sq_err.restype = ctypes.c_float
        L.oracle_sum.restype = ctypes.c_float
        L.oracle_param_count.restype = ctypes.c_size_t
        L.oracle_train_acts_floats.restype = ctypes.c_size_t
        _lib = L
    return _lib


def set_threads(n):
    """Set the OpenMP team size; returns the number of threads in use."""
    return lib().oracle_set_threads(int(n))


def _p(a):
    assert a.flags["C_CONTIGUOUS"]
    if a.dtype == np.float32:
        return a.ctypes.data_as(_f32p)
    if a.dtype == np.uint8:
        return a.ctypes.data_as(_u8p)
    raise TypeError(a.dtype)


def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def conv_fwd(x, W, B, in_w, in_h, n_prev, n_cur, f, relu, batch):
    x, W, B = f32(x), f32(W), f32(B)
    out = np.zeros(batch * (in_w - f + 1) * (in_h - f + 1) * n_cur, np.float32)
    lib().oracle_conv_fwd(_p(x), _p(out), _p(W), _p(B), in_w, in_h, n_prev, n_cur, f, int(relu), batch)
    return out


def last_delta(gt, y, gt_w, gt_h, out_w, out_h, batch):
    gt, y = f32(gt), f32(y)
    d = np.zeros(batch * out_w * out_h, np.float32)
    lib().oracle_last_delta(_p(gt), _p(y), _p(d), gt_w, gt_h, out_w, out_h, batch)
    return d


def conv_delta(d_next, y_curr, W_next, f_next, n_curr, n_next, curr_w, curr_h, batch):
    d_next, y_curr, W_next = f32(d_next), f32(y_curr), f32(W_next)
    d = np.zeros(batch * curr_w * curr_h * n_curr, np.float32)
    lib().oracle_conv_delta(_p(d_next), _p(y_curr), _p(d), _p(W_next), f_next, n_curr, n_next,
                            curr_w, curr_h, batch)
    return d


def conv_grad_acc(inp, delta, gW, gB, n_prev, n_cur, f, out_w, out_h, batch):
    """Accumulates into copies of gW/gB and returns them."""
    inp, delta = f32(inp), f32(delta)
    gW, gB = f32(gW).copy(), f32(gB).copy()
    lib().oracle_conv_grad_acc(_p(inp), _p(delta), _p(gW), _p(gB), n_prev, n_cur, f, out_w, out_h, batch)
    return gW, gB


def sgd_update(W, B, gW, gB, dW, dB, momentum, wd, lr, batch):
    W, B, dW, dB = f32(W).copy(), f32(B).copy(), f32(dW).copy(), f32(dB).copy()
    gW, gB = f32(gW), f32(gB)
    lib().oracle_sgd_update(_p(W), _p(B), _p(gW), _p(gB), _p(dW), _p(dB), momentum, wd, lr, batch,
                            W.size, B.size)
    return W, B, dW, dB


def sq_err(gt, y, gt_w, gt_h, out_w, out_h, batch):
    return lib().oracle_sq_err(_p(f32(gt)), _p(f32(y)), gt_w, gt_h, out_w, out_h, batch)


def buf_sum(data, squared=False):
    d = f32(data)
    return lib().oracle_sum(_p(d), d.size, int(squared))


def sub_from_all(data, value):
    d = f32(data).copy()
    lib().oracle_sub_from_all(_p(d), value, d.size)
    return d


def extract_luma(rgba, w, h, normalize):
    rgba = np.ascontiguousarray(rgba, dtype=np.uint8)
    out = np.zeros(w * h, np.float32)
    lib().oracle_extract_luma(_p(rgba), _p(out), w, h, int(normalize))
    return out


def swap_luma(rgba, new_luma, w, h, luma_w, luma_h):
    rgba = np.ascontiguousarray(rgba, dtype=np.uint8)
    out = np.zeros(w * h * 3, np.uint8)
    lib().oracle_swap_luma(_p(rgba), _p(f32(new_luma)), _p(out), w, h, luma_w, luma_h)
    return out


def param_count(n1, n2, f1, f2, f3):
    return lib().oracle_param_count(n1, n2, f1, f2, f3)


def train_fwd_bwd(cfg, X, T, w, h, batch, params, grads, want_acts=False):
    n1, n2, f1, f2, f3 = cfg
    X, T, params = f32(X), f32(T), f32(params)
    grads = f32(grads).copy()
    acts = None
    if want_acts:
        acts = np.zeros(lib().oracle_train_acts_floats(n1, n2, f1, f2, f3, w, h, batch), np.float32)
    lib().oracle_train_fwd_bwd(n1, n2, f1, f2, f3, _p(X), _p(T), w, h, batch, _p(params), _p(grads),
                               _p(acts) if acts is not None else None)
    return grads, acts


def update_all(cfg, params, grads, mom, momentum, wd, lr, batch):
    n1, n2, f1, f2, f3 = cfg
    params, grads, mom = f32(params).copy(), f32(grads).copy(), f32(mom).copy()
    lr = f32(lr)
    lib().oracle_update_all(n1, n2, f1, f2, f3, _p(params), _p(grads), _p(mom), momentum, wd, _p(lr), batch)
    return params, grads, mom


def forward(cfg, X, w, h, batch, params):
    n1, n2, f1, f2, f3 = cfg
    pad = f1 + f2 + f3 - 3
    out = np.zeros(batch * (w - pad) * (h - pad), np.float32)
    lib().oracle_forward(n1, n2, f1, f2, f3, _p(f32(X)), w, h, batch, _p(f32(params)), _p(out))
    return out
