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
LIB64_PATH = os.path.join(HERE, "build", "libsrcnn_oracle_f64.so")

_u8p = ctypes.POINTER(ctypes.c_uint8)


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


class Oracle:
    """The restatement at one arithmetic precision: np.float32 (the oracle
    proper, libsrcnn_oracle.so) or np.float64 (the same loop nests in double,
    libsrcnn_oracle_f64.so, the exact-arithmetic yardstick)."""

    def __init__(self, path, dtype):
        self.path, self.dtype, self._lib = path, np.dtype(dtype), None
        self._rp = ctypes.POINTER(ctypes.c_float if self.dtype == np.float32 else ctypes.c_double)

    def lib(self):
        if self._lib is None:
            if not os.path.exists(self.path):
                build()
            L = ctypes.CDLL(self.path)
            i, sz, u = ctypes.c_int, ctypes.c_size_t, ctypes.c_uint
            r = ctypes.c_float if self.dtype == np.float32 else ctypes.c_double
            fp = self._rp
            sig = {
                "oracle_set_threads": [i],
                "oracle_conv_fwd": [fp, fp, fp, fp, i, i, i, i, i, i, i],
                "oracle_last_delta": [fp, fp, fp, i, i, i, i, i],
                "oracle_conv_delta": [fp, fp, fp, fp, i, i, i, i, i, i],
                "oracle_conv_grad_acc": [fp, fp, fp, fp, i, i, i, i, i, i],
                "oracle_sgd_update": [fp, fp, fp, fp, fp, fp, r, r, r, u, i, i],
                "oracle_sq_err": [fp, fp, i, i, i, i, i],
                "oracle_sum": [fp, sz, i],
                "oracle_sub_from_all": [fp, r, sz],
                "oracle_extract_luma": [_u8p, fp, i, i, i],
                "oracle_swap_luma": [_u8p, fp, _u8p, i, i, i, i],
                "oracle_param_count": [i, i, i, i, i],
                "oracle_train_acts_floats": [i, i, i, i, i, i, i, i],
                "oracle_train_fwd_bwd": [i, i, i, i, i, fp, fp, i, i, i, fp, fp, fp],
                "oracle_train_fwd_bwd_masked": [i, i, i, i, i, fp, fp, i, i, i, fp, fp, fp, _u8p, _u8p, _u8p],
                "oracle_update_all": [i, i, i, i, i, fp, fp, fp, r, r, fp, u],
                "oracle_forward": [i, i, i, i, i, fp, i, i, i, fp, fp],
            }
            for name, argt in sig.items():
                fn = getattr(L, name)
                fn.argtypes = argt
                fn.restype = None
            L.oracle_set_threads.restype = ctypes.c_int
            L.oracle_sq_err.restype = r
            L.oracle_sum.restype = r
            L.oracle_param_count.restype = ctypes.c_size_t
            L.oracle_train_acts_floats.restype = ctypes.c_size_t
            self._lib = L
        return self._lib

    def set_threads(self, n):
        """Set the OpenMP team size; returns the number of threads in use."""
        return self.lib().oracle_set_threads(int(n))

    def _p(self, a):
        assert a.flags["C_CONTIGUOUS"]
        if a.dtype == self.dtype:
            return a.ctypes.data_as(self._rp)
        if a.dtype == np.uint8:
            return a.ctypes.data_as(_u8p)
        raise TypeError(a.dtype)

    def f(self, a):
        return np.ascontiguousarray(a, dtype=self.dtype)

    def zeros(self, n):
        return np.zeros(n, self.dtype)

    def conv_fwd(self, x, W, B, in_w, in_h, n_prev, n_cur, f, relu, batch):
        x, W, B = self.f(x), self.f(W), self.f(B)
        out = self.zeros(batch * (in_w - f + 1) * (in_h - f + 1) * n_cur)
        self.lib().oracle_conv_fwd(self._p(x), self._p(out), self._p(W), self._p(B), in_w, in_h, n_prev, n_cur, f, int(relu), batch)
        return out

    def last_delta(self, gt, y, gt_w, gt_h, out_w, out_h, batch):
        gt, y = self.f(gt), self.f(y)
        d = self.zeros(batch * out_w * out_h)
        self.lib().oracle_last_delta(self._p(gt), self._p(y), self._p(d), gt_w, gt_h, out_w, out_h, batch)
        return d

    def conv_delta(self, d_next, y_curr, W_next, f_next, n_curr, n_next, curr_w, curr_h, batch):
        d_next, y_curr, W_next = self.f(d_next), self.f(y_curr), self.f(W_next)
        d = self.zeros(batch * curr_w * curr_h * n_curr)
        self.lib().oracle_conv_delta(self._p(d_next), self._p(y_curr), self._p(d), self._p(W_next), f_next, n_curr, n_next,
                                curr_w, curr_h, batch)
        return d

    def conv_grad_acc(self, inp, delta, gW, gB, n_prev, n_cur, f, out_w, out_h, batch):
        """Accumulates into copies of gW/gB and returns them."""
        inp, delta = self.f(inp), self.f(delta)
        gW, gB = self.f(gW).copy(), self.f(gB).copy()
        self.lib().oracle_conv_grad_acc(self._p(inp), self._p(delta), self._p(gW), self._p(gB), n_prev, n_cur, f, out_w, out_h, batch)
        return gW, gB

    def sgd_update(self, W, B, gW, gB, dW, dB, momentum, wd, lr, batch):
        W, B, dW, dB = self.f(W).copy(), self.f(B).copy(), self.f(dW).copy(), self.f(dB).copy()
        gW, gB = self.f(gW), self.f(gB)
        self.lib().oracle_sgd_update(self._p(W), self._p(B), self._p(gW), self._p(gB), self._p(dW), self._p(dB), momentum, wd, lr, batch,
                                W.size, B.size)
        return W, B, dW, dB

    def sq_err(self, gt, y, gt_w, gt_h, out_w, out_h, batch):
        return self.lib().oracle_sq_err(self._p(self.f(gt)), self._p(self.f(y)), gt_w, gt_h, out_w, out_h, batch)

    def buf_sum(self, data, squared=False):
        d = self.f(data)
        return self.lib().oracle_sum(self._p(d), d.size, int(squared))

    def sub_from_all(self, data, value):
        d = self.f(data).copy()
        self.lib().oracle_sub_from_all(self._p(d), value, d.size)
        return d

    def extract_luma(self, rgba, w, h, normalize):
        rgba = np.ascontiguousarray(rgba, dtype=np.uint8)
        out = self.zeros(w * h)
        self.lib().oracle_extract_luma(self._p(rgba), self._p(out), w, h, int(normalize))
        return out

    def swap_luma(self, rgba, new_luma, w, h, luma_w, luma_h):
        rgba = np.ascontiguousarray(rgba, dtype=np.uint8)
        out = np.zeros(w * h * 3, np.uint8)
        self.lib().oracle_swap_luma(self._p(rgba), self._p(self.f(new_luma)), self._p(out), w, h, luma_w, luma_h)
        return out

    def param_count(self, n1, n2, f1, f2, f3):
        return self.lib().oracle_param_count(n1, n2, f1, f2, f3)

    def train_fwd_bwd(self, cfg, X, T, w, h, batch, params, grads, want_acts=False):
        n1, n2, f1, f2, f3 = cfg
        X, T, params = self.f(X), self.f(T), self.f(params)
        grads = self.f(grads).copy()
        acts = None
        if want_acts:
            acts = self.zeros(self.lib().oracle_train_acts_floats(n1, n2, f1, f2, f3, w, h, batch))
        self.lib().oracle_train_fwd_bwd(n1, n2, f1, f2, f3, self._p(X), self._p(T), w, h, batch, self._p(params), self._p(grads),
                                   self._p(acts) if acts is not None else None)
        return grads, acts

    def train_fwd_bwd_masked(self, cfg, X, T, w, h, batch, params, grads, m1, m2, m3, want_acts=False):
        """train_fwd_bwd with the ReLU decisions of the three layers given as
        boolean arrays in A1's / A2's / A3's layout (e.g. the HIP path's A > 0)."""
        n1, n2, f1, f2, f3 = cfg
        X, T, params = self.f(X), self.f(T), self.f(params)
        grads = self.f(grads).copy()
        m1 = np.ascontiguousarray(m1, dtype=np.uint8).ravel()
        m2 = np.ascontiguousarray(m2, dtype=np.uint8).ravel()
        w1, h1 = w - f1 + 1, h - f1 + 1
        w2, h2 = w1 - f2 + 1, h1 - f2 + 1
        m3 = np.ascontiguousarray(m3, dtype=np.uint8).ravel()
        assert m1.size == batch * w1 * h1 * n1 and m2.size == batch * w2 * h2 * n2
        assert m3.size == batch * (w2 - f3 + 1) * (h2 - f3 + 1)
        acts = None
        if want_acts:
            acts = self.zeros(self.lib().oracle_train_acts_floats(n1, n2, f1, f2, f3, w, h, batch))
        self.lib().oracle_train_fwd_bwd_masked(n1, n2, f1, f2, f3, self._p(X), self._p(T), w, h, batch,
                                               self._p(params), self._p(grads),
                                               self._p(acts) if acts is not None else None,
                                               self._p(m1), self._p(m2), self._p(m3))
        return grads, acts

    def update_all(self, cfg, params, grads, mom, momentum, wd, lr, batch):
        n1, n2, f1, f2, f3 = cfg
        params, grads, mom = self.f(params).copy(), self.f(grads).copy(), self.f(mom).copy()
        lr = self.f(lr)
        self.lib().oracle_update_all(n1, n2, f1, f2, f3, self._p(params), self._p(grads), self._p(mom), momentum, wd, self._p(lr), batch)
        return params, grads, mom

    def forward(self, cfg, X, w, h, batch, params):
        n1, n2, f1, f2, f3 = cfg
        pad = f1 + f2 + f3 - 3
        out = self.zeros(batch * (w - pad) * (h - pad))
        self.lib().oracle_forward(n1, n2, f1, f2, f3, self._p(self.f(X)), w, h, batch, self._p(self.f(params)), self._p(out))
        return out


ORACLE = Oracle(LIB_PATH, np.float32)
f64 = Oracle(LIB64_PATH, np.float64)


def lib():
    return ORACLE.lib()


def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


for _name in ("set_threads", "conv_fwd", "last_delta", "conv_delta", "conv_grad_acc", "sgd_update",
              "sq_err", "buf_sum", "sub_from_all", "extract_luma", "swap_luma", "param_count",
              "train_fwd_bwd", "train_fwd_bwd_masked", "update_all", "forward"):
    globals()[_name] = getattr(ORACLE, _name)
