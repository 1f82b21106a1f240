"""ctypes wrapper of oracle/build/libfa_oracle.so (the C tiled restatement). TEST INFRASTRUCTURE ONLY."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "libfa_oracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            subprocess.run(["make", "-C", _HERE], check=True, capture_output=True)
        L = ctypes.CDLL(_SO)
        fp = ctypes.POINTER(ctypes.c_float)
        ip = ctypes.POINTER(ctypes.c_int32)
        L.fa_oracle_fwd.argtypes = [fp, fp, fp, ip, ip, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_float, ctypes.c_float, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                    ctypes.c_int, fp, fp]
        L.fa_oracle_fwd.restype = None
        L.fa_oracle_rnd16.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_int]
        L.fa_oracle_rnd16.restype = ctypes.c_uint32
        L.fa_oracle_philox.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32), ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_uint32)]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def fwd(q, k, v, cu_q, cu_k, softmax_scale, p_dropout=0.0, seed=0, offset=0, causal=False, round_p=0):
    """q (total_q,H,D), k/v (total_k,H,D) float32 numpy; cu int32. round_p: 0 none, 1 bf16, 2 fp16.
    Returns (out (total_q,H,D) f32, lse (B,H,max_q) f32)."""
    q, k, v = [np.ascontiguousarray(x, dtype=np.float32) for x in (q, k, v)]
    cu_q = np.ascontiguousarray(cu_q, dtype=np.int32)
    cu_k = np.ascontiguousarray(cu_k, dtype=np.int32)
    B = len(cu_q) - 1
    H, D = q.shape[1], q.shape[2]
    max_q = int(np.max(np.diff(cu_q))) if B else 0
    lse_stride = max(max_q, 1)
    out = np.zeros_like(q)
    lse = np.full((B, H, lse_stride), np.nan, dtype=np.float32)
    f = ctypes.c_float
    lib().fa_oracle_fwd(_p(q, f), _p(k, f), _p(v, f), _p(cu_q, ctypes.c_int32), _p(cu_k, ctypes.c_int32), B, H, D,
                        lse_stride, softmax_scale, p_dropout, seed, offset, 1 if causal else 0, round_p,
                        _p(out, f), _p(lse, f))
    return out, lse


def philox(ctr, key, rounds):
    c = (ctypes.c_uint32 * 4)(*ctr)
    kk = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib().fa_oracle_philox(c, kk, rounds, o)
    return list(o)


def rnd16(seed, offset, bh, row, col):
    return lib().fa_oracle_rnd16(seed, offset, bh, row, col)
