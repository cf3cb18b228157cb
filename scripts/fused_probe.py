"""Per-launch device time of the fused B = 128 layer kernels (pkc_dense_gemm_fwd, ...) against the
split-K matmul + BatchNorm launch pair they replace, over contraction depths and column counts
(graph replays of back-to-back launches, scripts/kbench.timed).  Usage:
python scripts/fused_probe.py"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pytorch-kaldi-cgs_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch  # noqa: E402

from kbench import stream, timed  # noqa: E402
from pkc import _lib as L  # noqa: E402
from pkc._lib import call, ptr  # noqa: E402

DEV = "cuda"


def args(M, N, bufs, p=0.15):
    return L.DenseFwdArgs(M=M, N=N, nslab=bufs["S"], zslab=bufs["slab"].data_ptr(),
                          slab_stride=M * N, bias=bufs["b"].data_ptr(), norm=L.NORM_BN_TRAIN,
                          gamma=bufs["g"].data_ptr(), beta=bufs["be"].data_ptr(),
                          running_mean=bufs["rm"].data_ptr(), running_var=bufs["rv"].data_ptr(),
                          momentum=0.05, eps=1e-5, save_mean=bufs["sm"].data_ptr(),
                          save_invstd=bufs["si"].data_ptr(), act=L.ACT["relu"], drop_p=p, seed=1,
                          step_ctr=bufs["ctr"].data_ptr(), stream_id=0, keep_in=None,
                          keep_out=bufs["keep"].data_ptr(), xhat=bufs["xh"].data_ptr(),
                          out=None, out_bf16=bufs["oh"].data_ptr())


def main():
    M = 128
    for N, K in ((1024, 1024), (1024, 440), (1024, 256), (1024, 64), (256, 1024), (2048, 1024)):
        X = torch.randn(M, K, device=DEV).bfloat16()
        W = torch.randn(N, K, device=DEV).bfloat16()
        S = L.lib().pkc_gemm_pick_splits(M, N, K)
        bufs = dict(S=S, slab=torch.zeros(S, M, N, device=DEV), b=torch.zeros(N, device=DEV),
                    g=torch.ones(N, device=DEV), be=torch.zeros(N, device=DEV),
                    rm=torch.zeros(N, device=DEV), rv=torch.ones(N, device=DEV),
                    sm=torch.zeros(N, device=DEV), si=torch.zeros(N, device=DEV),
                    ctr=torch.zeros(2, dtype=torch.int64, device=DEV),
                    keep=torch.zeros(M, N, dtype=torch.uint8, device=DEV),
                    xh=torch.zeros(M, N, device=DEV),
                    oh=torch.zeros(M, N, dtype=torch.bfloat16, device=DEV))
        a = args(M, N, bufs)
        work = torch.zeros(L.lib().pkc_dense_work_size(M, N), device=DEV)

        def fused():
            call("pkc_dense_gemm_fwd", L.PREC_BF16IN, ptr(X), K, ptr(W), K, K, C.byref(a), stream())

        def gemm():
            call("pkc_gemm", L.PREC_BF16IN, 1, 1, M, N, K, ptr(X), K, ptr(W), K, ptr(bufs["slab"]),
                 N, S, M * N, stream())

        def dense():
            call("pkc_dense_fwd", C.byref(a), ptr(work), stream())

        def pair():
            gemm()
            dense()

        t = {k: timed(f) for k, f in (("fused", fused), ("gemm", gemm), ("dense", dense),
                                      ("pair", pair))}
        print("M=%d N=%d K=%d splits=%d: fused %.2f us | split-K gemm %.2f + BN %.2f = pair %.2f us"
              % (M, N, K, S, t["fused"], t["gemm"], t["dense"], t["pair"]), flush=True)


if __name__ == "__main__":
    main()
