"""ctypes binding of libpkc.so (the C ABI declared in include/pkc.h).

The product path has no CPU fallback: if libpkc.so is missing or does not load, every entry point
raises.  Build it with ``python -c "import __graft_entry__ as g; g.build()"`` (or pkc/_build.py).
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PKC_LIB", os.path.join(_HERE, "libpkc.so"))

ABI_VERSION = 9         # include/pkc.h PKC_ABI_VERSION
PKC_OK, PKC_ERR_ARG, PKC_ERR_HIP, PKC_ERR_IO, PKC_ERR_UNSUPPORTED = 0, -1, -2, -3, -4
PREC_FP32, PREC_BF16, PREC_BF16IN, PREC_BF16X3 = 0, 1, 2, 3
ACT = {"linear": 0, "relu": 1, "tanh": 2, "sigmoid": 3, "htanh": 4, "leaky_relu": 5, "elu": 6}
NORM_NONE, NORM_BN_TRAIN, NORM_BN_EVAL = 0, 1, 2
OPT = {"sgd": 0, "rmsprop": 1, "adam": 2}

p_f = C.POINTER(C.c_float)
vp = C.c_void_p
i64 = C.c_int64


class DenseFwdArgs(C.Structure):
    _fields_ = [("M", C.c_int), ("N", C.c_int), ("nslab", C.c_int),
                ("zslab", vp), ("slab_stride", i64), ("bias", vp),
                ("norm", C.c_int), ("gamma", vp), ("beta", vp),
                ("running_mean", vp), ("running_var", vp), ("momentum", C.c_float), ("eps", C.c_float),
                ("save_mean", vp), ("save_invstd", vp),
                ("act", C.c_int), ("drop_p", C.c_float), ("seed", C.c_uint64), ("step_ctr", vp),
                ("stream_id", i64), ("keep_in", vp), ("keep_out", vp), ("xhat", vp), ("out", vp),
                ("count_n", i64), ("out_bf16", vp)]


class DenseBwdArgs(C.Structure):
    _fields_ = [("M", C.c_int), ("N", C.c_int), ("nslab", C.c_int),
                ("gslab", vp), ("slab_stride", i64), ("norm", C.c_int), ("act", C.c_int),
                ("gamma", vp), ("beta", vp), ("save_invstd", vp), ("xhat", vp), ("keep", vp),
                ("drop_p", C.c_float), ("dz", vp), ("dgamma", vp), ("dbeta", vp), ("dbias", vp),
                ("dz_bf16", vp), ("dz_scratch", C.c_int)]


class NllArgs(C.Structure):
    _fields_ = [("M", C.c_int), ("N", C.c_int), ("nslab", C.c_int), ("zslab", vp),
                ("slab_stride", i64), ("bias", vp), ("labels", vp), ("label_stride", i64),
                ("weight", C.c_float), ("logp", vp), ("log_prior", vp), ("dlogits", vp),
                ("row_loss", vp), ("row_err", vp), ("dlogits_bf16", vp)]


class OptTensor(C.Structure):
    _fields_ = [("p", vp), ("g", vp), ("s1", vp), ("s2", vp), ("s3", vp), ("mask", vp), ("n", i64),
                ("kind", C.c_int), ("lr", C.c_float), ("wd", C.c_float), ("momentum", C.c_float),
                ("dampening", C.c_float), ("alpha", C.c_float), ("eps", C.c_float),
                ("beta1", C.c_float), ("beta2", C.c_float), ("clampv", C.c_float),
                ("nesterov", C.c_int), ("centered", C.c_int), ("amsgrad", C.c_int), ("step", C.c_int),
                ("qout", vp), ("qbits", C.c_int), ("bout", vp)]


class OptSeg(C.Structure):
    _fields_ = [("tensor", C.c_int), ("chunk0", C.c_int), ("nchunks", C.c_int), ("reserved", C.c_int),
                ("p", vp), ("g", vp), ("s1", vp), ("s2", vp), ("s3", vp), ("mask", vp), ("qout", vp),
                ("bout", vp), ("n", i64)]


OPT_SEGS_MAX = 8        # include/pkc.h PKC_OPT_SEGS_MAX


CELL_LIGRU, CELL_LSTM, CELL_GRU, CELL_MINGRU, CELL_RNN = 0, 1, 2, 3, 4


class RnnArgs(C.Structure):
    _fields_ = [("cell", C.c_int), ("T", C.c_int), ("B", C.c_int), ("H", C.c_int), ("bidir", C.c_int),
                ("act", C.c_int), ("train", C.c_int), ("wpre", vp), ("U", vp * 4),
                ("drop_p", C.c_float), ("seed", C.c_uint64), ("step_ctr", vp), ("stream_id", i64),
                ("drop_mask_in", vp), ("drop_mask", vp), ("hs", vp), ("cs", vp), ("gates", vp),
                ("y", vp), ("dy", vp), ("dy_nslab", C.c_int), ("dy_slab_stride", i64),
                ("dgates", vp), ("work", vp), ("qbits", C.c_int), ("hq", vp), ("rh", vp), ("ut", vp),
                ("ln_gamma", vp), ("ln_beta", vp), ("ln_eps", C.c_float), ("ln_xhat", vp),
                ("ln_stat", vp), ("ln_g", vp), ("ln_dgamma", vp), ("ln_dbeta", vp),
                ("kmap_fwd", vp), ("kmap_bwd", vp), ("kmap_s_fwd", C.c_int), ("kmap_s_bwd", C.c_int),
                ("step_bf16", C.c_int), ("hs_h", vp), ("U_h", vp * 4), ("ut_h", vp), ("dgates_h", vp),
                ("persist_fwd", vp), ("persist_bwd", vp), ("persist_kb", C.c_int),
                ("qh_exact", C.c_int)]


class GemmProblem(C.Structure):
    _fields_ = [("a_kcontig", C.c_int), ("b_kcontig", C.c_int), ("M", C.c_int), ("N", C.c_int),
                ("K", C.c_int), ("splits", C.c_int), ("A", vp), ("lda", i64), ("B", vp),
                ("ldb", i64), ("C", vp), ("ldc", i64), ("slab_stride", i64), ("kind", C.c_int),
                ("X1", vp), ("X2", vp), ("X3", vp), ("ktiles", vp), ("kmax", C.c_int)]


OP_GEMM, OP_COLSUM, OP_LOSS, OP_OPTIM, OP_SLABSUM, OP_GATHER = 0, 1, 2, 3, 4, 5


class BnBwdEpi(C.Structure):
    _fields_ = [("xhat", vp), ("keep", vp), ("gamma", vp), ("beta", vp), ("part", vp),
                ("act", C.c_int), ("drop_p", C.c_float)]

REG_L1, REG_L2 = 1, 2


class RegItem(C.Structure):
    _fields_ = [("p", vp), ("g", vp), ("ld", i64), ("r0", C.c_int), ("r1", C.c_int),
                ("c0", C.c_int), ("c1", C.c_int), ("block", C.c_int), ("assign", C.c_int)]


_SIGS = {
    "pkc_reg_partial": (C.c_int, [C.c_int, vp, C.c_int, vp, vp]),
    "pkc_reg_finalize": (C.c_int, [C.c_int, vp, C.c_int, vp, C.c_float, vp, vp, C.c_int, vp]),
    "pkc_reg_grad": (C.c_int, [C.c_int, vp, C.c_int, vp, vp]),
    "pkc_ark_cm_size": (i64, [vp, i64]),
    "pkc_ark_decode_cm": (C.c_int, [vp, i64, vp]),
    "pkc_prune_work_size": (i64, []),
    "pkc_prune": (C.c_int, [vp, i64, C.c_double, vp, vp, vp]),
    "pkc_layernorm_fwd": (C.c_int, [C.c_int, C.c_int, C.c_int, vp, i64, vp, vp, vp, C.c_float, vp, vp,
                                    vp, vp]),
    "pkc_layernorm_bwd": (C.c_int, [C.c_int, C.c_int, C.c_int, vp, i64, vp, vp, vp, vp, vp, vp, vp,
                                    vp]),
    "pkc_gemm_grouped": (C.c_int, [C.c_int, vp, C.c_int, vp]),
    "pkc_fakequant_weight": (C.c_int, [vp, vp, i64, C.c_int, vp]),
    "pkc_fakequant_input": (C.c_int, [vp, vp, i64, C.c_int, C.c_int, vp, vp]),
    "pkc_pattern_mask": (C.c_int, [vp, C.c_int, C.c_int, vp, C.c_int, C.c_int, C.c_int, vp, vp]),
    "pkc_rnn_fwd": (C.c_int, [C.POINTER(RnnArgs), vp]),
    "pkc_rnn_persist_form": (C.c_int, [C.POINTER(RnnArgs), C.c_int]),
    "pkc_rnn_bwd": (C.c_int, [C.POINTER(RnnArgs), vp, vp]),
    "pkc_seq_gather": (C.c_int, [vp, i64, C.c_int, vp, C.c_int, vp, vp, vp, C.c_int, C.c_int, vp, vp,
                                 vp]),
    "pkc_abi_version": (C.c_int, []),
    "pkc_last_error": (C.c_char_p, []),
    "pkc_gemm": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, i64, vp, i64,
                           vp, i64, C.c_int, i64, vp]),
    "pkc_gemm_pick_splits": (C.c_int, [C.c_int, C.c_int, C.c_int]),
    "pkc_dense_fwd": (C.c_int, [C.POINTER(DenseFwdArgs), vp, vp]),
    "pkc_dense_fwd_pre": (C.c_int, [C.POINTER(DenseFwdArgs), vp, C.c_int, vp]),
    "pkc_gemm_colstats_ok": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, i64,
                                       vp, i64]),
    "pkc_gemm_colstats": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, i64, vp,
                                    i64, vp, i64, vp, vp, vp]),
    "pkc_dense_bwd": (C.c_int, [C.POINTER(DenseBwdArgs), vp, vp]),
    "pkc_dense_bwd_pre": (C.c_int, [C.POINTER(DenseBwdArgs), vp, C.c_int, vp]),
    "pkc_gemm_grouped_tile": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp,
                                        i64, vp, i64]),
    "pkc_rnn_persist_geometry": (C.c_int, [C.POINTER(C.c_int)] * 5),
    "pkc_gemm_bnbwd_ok": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, i64,
                                    vp, i64]),
    "pkc_dense_work_size": (i64, [C.c_int, C.c_int]),
    "pkc_dense_fwd_stats": (C.c_int, [C.POINTER(DenseFwdArgs), vp, vp, vp]),
    "pkc_dense_fwd_sync_apply": (C.c_int, [C.POINTER(DenseFwdArgs), vp, vp, C.c_int, vp]),
    "pkc_dense_bwd_stats": (C.c_int, [C.POINTER(DenseBwdArgs), vp, vp, vp]),
    "pkc_dense_bwd_sync_apply": (C.c_int, [C.POINTER(DenseBwdArgs), vp, vp, C.c_int, vp]),
    "pkc_nll_fused": (C.c_int, [C.POINTER(NllArgs), vp]),
    "pkc_loss_finalize": (C.c_int, [C.c_int, vp, vp, C.c_int, vp, vp, vp, vp, vp]),
    "pkc_nll_fused_multi": (C.c_int, [vp, C.c_int, vp]),
    "pkc_logsoftmax_bwd": (C.c_int, [C.c_int, C.c_int, vp, vp, vp, vp]),
    "pkc_colsum": (C.c_int, [C.c_int, C.c_int, C.c_int, vp, i64, vp, C.c_int, vp]),
    "pkc_optim_step": (C.c_int, [vp, C.c_int, vp, C.c_int, vp]),
    "pkc_optim_chunks": (C.c_int, [C.POINTER(i64), C.c_int, C.POINTER(C.c_int32), C.c_int]),
    "pkc_apply_mask": (C.c_int, [vp, vp, i64, C.c_float, vp]),
    "pkc_batch_gather": (C.c_int, [vp, i64, C.c_int, vp, C.c_int, C.c_int, i64, vp, vp, vp, C.c_int,
                                   vp, vp]),
    "pkc_cast_bf16": (C.c_int, [vp, vp, i64, vp]),
    "pkc_cw_stats": (C.c_int, [vp, i64, C.c_int, C.c_int, C.c_int, vp, vp, vp, vp]),
    "pkc_cw_stats_work_size": (i64, [i64, C.c_int, C.c_int, C.c_int]),
    "pkc_dense_gemm_fwd_ok": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, vp, i64, vp, i64]),
    "pkc_dense_gemm_fwd": (C.c_int, [C.c_int, vp, i64, vp, i64, C.c_int, C.POINTER(DenseFwdArgs),
                                     vp]),
    "pkc_cw_apply": (C.c_int, [vp, i64, C.c_int, C.c_int, C.c_int, vp, vp, vp, vp, i64, vp]),
    "pkc_cw_apply_rows": (C.c_int, [vp, i64, C.c_int, C.c_int, C.c_int, vp, vp, vp, i64, i64, vp,
                                    i64, vp]),
    "pkc_feat_frontend": (C.c_int, [vp, C.c_int, i64, vp, vp, vp, vp, vp, vp, C.c_int, vp, C.c_int,
                                    C.c_int, vp, vp]),
    "pkc_ark_write_mat": (C.c_int, [C.c_char_p, C.c_int, C.c_char_p, i64, i64, vp]),
    "pkc_ark_index": (i64, [C.c_char_p, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64), i64,
                            C.c_char_p, i64]),
    "pkc_ark_read_rows": (C.c_int, [C.c_char_p, i64, i64, i64, vp]),
}

_lib = None


class PkcError(RuntimeError):
    pass


def tree_digest():
    """The source digest of the tree this package runs from (None when csrc/ is absent, e.g. an
    installed library used through PKC_LIB without sources)."""
    from ._build import CSRC, INCLUDE, src_digest
    if not (os.path.isdir(CSRC) and os.path.isdir(INCLUDE)):
        return None
    return src_digest()


def check_provenance(L):
    """Refuse a libpkc.so built from other sources than the tree's csrc/ + include/."""
    L.pkc_src_digest.restype = C.c_char_p
    L.pkc_src_digest.argtypes = []
    built = L.pkc_src_digest().decode()
    want = tree_digest()
    if want is not None and built != want:
        raise PkcError("libpkc.so was built from other sources (digest %s..., tree %s...): "
                       "rebuild it (__graft_entry__.build())" % (built[:12], want[:12]))
    return built


def lib():
    """Load libpkc.so once; raise (never fall back) if it is not there."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PkcError("libpkc.so not found at %s: build it first (__graft_entry__.build())"
                           % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.pkc_abi_version() != ABI_VERSION:
            raise PkcError("libpkc ABI mismatch")
        check_provenance(L)
        _lib = L
    return _lib


def check(status, what=""):
    if status != PKC_OK:
        raise PkcError("%s failed (%d): %s" % (what, status, lib().pkc_last_error().decode()))
    return status


def call(name, *args):
    return check(getattr(lib(), name)(*args), name)


def ptr(t):
    """Device/host pointer of a tensor (None -> NULL)."""
    return None if t is None else C.c_void_p(t.data_ptr())
