"""Kernel micro-benchmarks at the C2 shapes (B = 128 frames): per-launch device time of each libpkc
entry point, measured as hipGraph replays of 50 back-to-back launches (so the number includes the
dependent-kernel boundary a real step pays).  Usage: python scripts/kbench.py [filter]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pytorch-kaldi-cgs_amd"))

import torch  # noqa: E402

from pkc import _lib as L  # noqa: E402
from pkc._lib import call, ptr  # noqa: E402

DEV = "cuda"
REPS = 50


def timed(fn, reps=REPS):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1000.0 / reps)
    return best


def stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def f32(*shape):
    return torch.randn(*shape, device=DEV, dtype=torch.float32)


def bench_gemm(rows):
    M = 128
    shapes = [("fwd", 1, 1, M, 1024, 1024), ("fwd", 1, 1, M, 1024, 440), ("fwd", 1, 1, M, 1928, 1024),
              ("dX", 1, 0, M, 1024, 1024), ("dX", 1, 0, M, 1024, 1928),
              ("dW", 0, 0, 1024, 1024, M), ("dW", 0, 0, 1928, 1024, M), ("dW", 0, 0, 1024, 440, M)]
    for prec in (L.PREC_BF16IN, L.PREC_BF16, L.PREC_FP32):
        for name, akc, bkc, m, n, k in shapes:
            A = f32(m * k)
            B = f32(n * k)
            if prec == L.PREC_BF16IN:
                A, B = A.bfloat16(), B.bfloat16()
            lda = k if akc else m
            ldb = k if bkc else n
            for sp in sorted({1, 2, 4, 8, L.lib().pkc_gemm_pick_splits(m, n, k)}):
                if sp > 1 and (k // sp) < 32:
                    continue
                Cb = f32(sp * m * n)

                def fn():
                    call("pkc_gemm", prec, akc, bkc, m, n, k, ptr(A), lda, ptr(B), ldb, ptr(Cb), n,
                         sp, m * n, stream())
                us = timed(fn)
                rows.append(("gemm_%s_%s %dx%dx%d s%d" % (name, ["fp32", "bf16", "bf16in"][prec], m, n,
                                                           k, sp), us))


def bench_biggemm(rows):
    """The sequence configs' non-recurrent matmuls (C4: T*B = 5440 rows, 4 gates x 1024, bidir
    input 2048), fp32 exact MFMA: achieved TFLOP/s."""
    R, N, K = 5440, 1024, 2048
    for name, akc, bkc, m, n, k in (("fwd", 1, 1, R, N, K), ("dX", 1, 0, R, K, N),
                                    ("dW", 0, 0, N, K, R), ("dU", 0, 0, N, N, R)):
        A = f32(m * k)
        B = f32(n * k)
        Cb = f32(m * n)
        lda = k if akc else m
        ldb = k if bkc else n
        for prec in (L.PREC_FP32, L.PREC_BF16):
            def fn():
                call("pkc_gemm", prec, akc, bkc, m, n, k, ptr(A), lda, ptr(B), ldb, ptr(Cb), n, 1,
                     m * n, stream())
            us = timed(fn, reps=5)
            rows.append(("big_%s_%s %dx%dx%d (%.0f TF/s)" % (name, ["fp32", "bf16"][prec], m, n, k,
                                                             2.0 * m * n * k / us / 1e6), us))


def bench_dense(rows):
    M = 128
    for N, ns in ((1024, 1), (1024, 4), (1024, 8)):
        z = f32(ns * M * N)
        bias, gamma, beta = f32(N), f32(N), f32(N)
        rm, rv = torch.zeros(N, device=DEV), torch.ones(N, device=DEV)
        sm, si = f32(N), f32(N)
        xhat, out = f32(M * N), f32(M * N)
        keep = torch.zeros(M * N, dtype=torch.uint8, device=DEV)
        ctr = torch.zeros(2, dtype=torch.int64, device=DEV)
        work = f32(L.lib().pkc_dense_work_size(M, N))
        a = L.DenseFwdArgs(M=M, N=N, nslab=ns, zslab=z.data_ptr(), slab_stride=M * N,
                           bias=bias.data_ptr(), norm=L.NORM_BN_TRAIN, gamma=gamma.data_ptr(),
                           beta=beta.data_ptr(), running_mean=rm.data_ptr(), running_var=rv.data_ptr(),
                           momentum=0.05, eps=1e-5, save_mean=sm.data_ptr(), save_invstd=si.data_ptr(),
                           act=L.ACT["relu"], drop_p=0.15, seed=1, step_ctr=ctr.data_ptr(), stream_id=3,
                           keep_in=None, keep_out=keep.data_ptr(), xhat=xhat.data_ptr(),
                           out=out.data_ptr(), count_n=0)
        rows.append(("dense_fwd N=%d s%d" % (N, ns),
                     timed(lambda: call("pkc_dense_fwd", C.byref(a), ptr(work), stream()))))
        dz = f32(M * N)
        dg, db, dbi = f32(N), f32(N), f32(N)
        b = L.DenseBwdArgs(M=M, N=N, nslab=ns, gslab=z.data_ptr(), slab_stride=M * N,
                           norm=L.NORM_BN_TRAIN, act=L.ACT["relu"], gamma=gamma.data_ptr(),
                           beta=beta.data_ptr(), save_invstd=si.data_ptr(), xhat=xhat.data_ptr(),
                           keep=keep.data_ptr(), drop_p=0.15, dz=dz.data_ptr(), dgamma=dg.data_ptr(),
                           dbeta=db.data_ptr(), dbias=dbi.data_ptr())
        rows.append(("dense_bwd N=%d s%d" % (N, ns),
                     timed(lambda: call("pkc_dense_bwd", C.byref(b), ptr(work), stream()))))


def bench_heads(rows):
    M = 128
    for N, ns in ((1928, 1), (1928, 4), (48, 1)):
        z = f32(ns * M * N)
        bias = f32(N)
        labels = torch.randint(0, N, (M,), dtype=torch.int32, device=DEV)
        logp, dl = f32(M * N), f32(M * N)
        rl, re = f32(M), f32(M)
        a = L.NllArgs(M=M, N=N, nslab=ns, zslab=z.data_ptr(), slab_stride=M * N, bias=bias.data_ptr(),
                      labels=labels.data_ptr(), label_stride=1, weight=1.0, logp=logp.data_ptr(),
                      log_prior=None, dlogits=dl.data_ptr(), row_loss=rl.data_ptr(),
                      row_err=re.data_ptr())
        rows.append(("nll N=%d s%d" % (N, ns), timed(lambda: call("pkc_nll_fused", C.byref(a), stream()))))
        out = f32(N)
        rows.append(("colsum N=%d" % N, timed(lambda: call("pkc_colsum", M, N, 1, ptr(dl), 0, ptr(out), 0,
                                                             stream()))))


def bench_optim(rows):
    sizes = [1024 * 440, 1024] * 1 + [1024 * 1024, 1024] * 4 + [1024 * 3] * 0
    head = [1928 * 1024, 1928, 48 * 1024, 48]
    ts = []
    for i, n in enumerate(sizes + head):
        p, g, s1 = f32(n), f32(n) * 1e-3, torch.zeros(n, device=DEV)
        ts.append((p, g, s1, 0 if i < len(sizes) else 1))
    arr = (L.OptTensor * len(ts))()
    for i, (p, g, s1, kind) in enumerate(ts):
        t = arr[i]
        t.p, t.g, t.s1, t.n, t.kind = p.data_ptr(), g.data_ptr(), s1.data_ptr(), p.numel(), kind
        t.lr, t.alpha, t.eps, t.step = 1e-3, 0.95, 1e-8, 1
    desc = torch.frombuffer(bytearray(C.string_at(arr, C.sizeof(arr))), dtype=torch.uint8).to(DEV)
    sz = (C.c_int64 * len(ts))(*[t[0].numel() for t in ts])
    nch = L.lib().pkc_optim_chunks(sz, len(ts), None, 0)
    cm = (C.c_int32 * (2 * nch))()
    L.lib().pkc_optim_chunks(sz, len(ts), cm, nch)
    import numpy as np
    cmap = torch.from_numpy(np.frombuffer(cm, dtype=np.int32).copy()).to(DEV)
    nparam = sum(t[0].numel() for t in ts)
    us = timed(lambda: call("pkc_optim_step", ptr(desc), len(ts), ptr(cmap), nch, stream()), reps=20)
    rows.append(("optim %.2fM params" % (nparam / 1e6), us))


def bench_floor(rows):
    x = torch.zeros(64, device=DEV)
    rows.append(("torch add_ 64 floats (floor)", timed(lambda: x.add_(1.0))))
    y = torch.zeros(1 << 20, device=DEV)
    rows.append(("torch add_ 4 MB", timed(lambda: y.add_(1.0))))


def main():
    flt = sys.argv[1] if len(sys.argv) > 1 else ""
    rows = []
    bench_floor(rows)
    for name, fn in (("gemm", bench_gemm), ("biggemm", bench_biggemm), ("dense", bench_dense),
                     ("heads", bench_heads), ("optim", bench_optim)):
        if flt and flt not in name:
            continue
        fn(rows)
    for k, us in rows:
        print("%-40s %8.2f us" % (k, us))


if __name__ == "__main__":
    main()
