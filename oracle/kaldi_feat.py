"""ORACLE — test infrastructure only (see oracle/__init__.py).

ctypes wrapper of oracle/kaldi_feat.c, the plain-C restatement of Kaldi's apply-cmvn
(transform/cmvn.cc ApplyCmvn) and add-deltas (feat/feature-functions.cc DeltaFeatures) that every
shipped cfg pipes its features through (data_io.py:18).  Parity UNPINNED against Kaldi itself
(third-party, absent here, no output fixture in the reference).
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libkaldi_feat.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE, "_build/libkaldi_feat.so"], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(
                os.path.join(_HERE, "kaldi_feat.c")):
            build()
        L = C.CDLL(_SO)
        vp, i64 = C.c_void_p, C.c_int64
        L.kf_cmvn_norm.argtypes = [vp, C.c_int, C.c_int, C.c_int, vp, vp]
        L.kf_cmvn_norm.restype = C.c_int
        L.kf_apply_cmvn.argtypes = [vp, i64, C.c_int, vp, vp, C.c_int]
        L.kf_apply_cmvn.restype = None
        L.kf_delta_scales.argtypes = [C.c_int, C.c_int, vp]
        L.kf_delta_scales.restype = None
        L.kf_add_deltas.argtypes = [vp, i64, C.c_int, C.c_int, C.c_int, vp]
        L.kf_add_deltas.restype = None
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def cmvn_norm(stats, norm_vars):
    stats = np.ascontiguousarray(stats, dtype=np.float64)
    rows, dim = stats.shape[0], stats.shape[1] - 1
    off = np.empty(dim, np.float32)
    sc = np.empty(dim, np.float32)
    rc = lib().kf_cmvn_norm(_p(stats), rows, dim, int(norm_vars), _p(off), _p(sc))
    if rc != 0:
        raise ValueError("kf_cmvn_norm: %d" % rc)
    return off, sc


def delta_scales(order, window):
    maxoff = order * window
    out = np.empty((order + 1, 2 * maxoff + 1), np.float32)
    lib().kf_delta_scales(order, window, _p(out))
    return out


def apply_cmvn(feats, stats, norm_vars=False):
    x = np.array(feats, dtype=np.float32, copy=True, order="C")
    off, sc = cmvn_norm(stats, norm_vars)
    lib().kf_apply_cmvn(_p(x), x.shape[0], x.shape[1], _p(off), _p(sc), int(norm_vars))
    return x


def add_deltas(feats, order=2, window=2):
    x = np.ascontiguousarray(feats, dtype=np.float32)
    out = np.empty((x.shape[0], x.shape[1] * (order + 1)), np.float32)
    lib().kf_add_deltas(_p(x), x.shape[0], x.shape[1], order, window, _p(out))
    return out


def pipeline(fea, stats, utt2spk=None, norm_means=True, norm_vars=False, order=None, window=2):
    """copy-feats | apply-cmvn [--utt2spk] | add-deltas on a {utt: (T, D)} dict.  Utterances
    without statistics are dropped (apply-cmvn writes nothing for them)."""
    out = {}
    for k, m in fea.items():
        x = np.asarray(m, np.float32)
        if stats is not None and norm_means:
            sk = utt2spk.get(k) if utt2spk is not None else k
            if sk is None or sk not in stats:
                continue
            x = apply_cmvn(x, stats[sk], norm_vars)
        if order is not None:
            x = add_deltas(x, order, window)
        out[k] = x
    return out
