"""GPU parity of the individual HIP kernels (through the C ABI) against PyTorch-CPU references of
the same ops (fp32 / fp64)."""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _s():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


@pytest.fixture(scope="module")
def L():
    from pkc import _lib
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    _lib.lib()
    return _lib


GEMM_SHAPES = [(128, 1024, 1024), (128, 1928, 1024), (128, 48, 1024), (128, 1024, 440),
               (37, 70, 45), (16, 96, 32), (64, 64, 32), (1, 5, 3), (200, 130, 260)]


def _tol(prec, K):
    """Absolute tolerance of a K-deep product of N(0,1) operands: exact fp32 (0), bf16-rounded
    operands vs their own rounded values (1, 2), compensated bf16 vs the UNROUNDED fp32 operands
    (3: the dropped lo*lo term and the tails' own rounding, ~2^-16 relative per product)."""
    return {0: 2e-5, 1: 1e-3, 2: 1e-3, 3: 6e-5}[prec] * K ** 0.5


@pytest.mark.parametrize("prec", [0, 1, 2, 3])
@pytest.mark.parametrize("M,N,K", GEMM_SHAPES)
@pytest.mark.parametrize("orient", ["nt", "nn", "tn"])
def test_gemm(L, prec, M, N, K, orient):
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    # logical C[M,N] = sum_k A(m,k) B(n,k)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g)
    akc, bkc = {"nt": (1, 1), "nn": (1, 0), "tn": (0, 0)}[orient]
    Ast = A if akc else A.t().contiguous()      # stored (M,K) or (K,M)
    Bst = B if bkc else B.t().contiguous()
    if prec in (1, 2):
        A = A.bfloat16().float()
        B = B.bfloat16().float()
    ref = (A.double() @ B.double().t()).float()
    splits = L.lib().pkc_gemm_pick_splits(M, N, K)
    Ad, Bd = Ast.to(DEV), Bst.to(DEV)
    if prec == 2:                                  # operands stored as bf16 in HBM
        Ad, Bd = Ad.bfloat16().contiguous(), Bd.bfloat16().contiguous()
    Cd = torch.full((splits, M, N), float("nan"), device=DEV)
    L.call("pkc_gemm", prec, akc, bkc, M, N, K, L.ptr(Ad), Ast.shape[1], L.ptr(Bd), Bst.shape[1],
           L.ptr(Cd), N, splits, M * N, _s())
    out = Cd.sum(0).cpu()
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=_tol(prec, K))
    if prec == 3 and K >= 256:    # and it is fp32-class: well inside plain bf16's error
        exact = A.double() @ B.double().t()
        e3 = (out.double() - exact).abs().max().item()
        eb = ((A.bfloat16().double() @ B.bfloat16().double().t()) - exact).abs().max().item()
        assert e3 < 0.05 * eb, (e3, eb)


@pytest.mark.parametrize("orient", ["nt", "nn", "tn"])
@pytest.mark.parametrize("M,N,K,grouped,splits", [(2048, 1280, 1024, False, 1),
                                                  (2048, 1280, 2048, False, 2),
                                                  (1000, 700, 1100, True, 1),
                                                  (4096, 1024, 1024, True, 1)])
def test_gemm_bf16x3_big_body(L, orient, M, N, K, grouped, splits):
    """Compensated bf16 (PKC_PREC_BF16X3) on the 128x128 tile body (head and tail bf16 images in
    LDS, 3 MFMAs per product: lo*hi, hi*lo, hi*hi): standalone (>= 160 tiles) and grouped (>= 32
    tiles, K >= 1024) launches, every operand orientation (row-major, m-contiguous PAIR staging),
    ragged edges, split-K slabs.  Against the fp64 product of the unrounded operands at ~2^-16
    relative per product, and well inside plain bf16's error."""
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g)
    akc, bkc = {"nt": (1, 1), "nn": (1, 0), "tn": (0, 0)}[orient]
    Ast = A if akc else A.t().contiguous()
    Bst = B if bkc else B.t().contiguous()
    Ad, Bd = Ast.to(DEV), Bst.to(DEV)
    assert L.lib().pkc_gemm_grouped_tile(3, akc, bkc, M, N, K, L.ptr(Ad), Ast.shape[1], L.ptr(Bd),
                                         Bst.shape[1]) == 128
    Cd = torch.full((splits, M, N), float("nan"), device=DEV)
    if grouped:
        pr = L.GemmProblem(a_kcontig=akc, b_kcontig=bkc, M=M, N=N, K=K, splits=splits,
                           A=Ad.data_ptr(), lda=Ast.shape[1], B=Bd.data_ptr(), ldb=Bst.shape[1],
                           C=Cd.data_ptr(), ldc=N, slab_stride=M * N)
        L.call("pkc_gemm_grouped", 3, C.byref(pr), 1, _s())
    else:
        L.call("pkc_gemm", 3, akc, bkc, M, N, K, L.ptr(Ad), Ast.shape[1], L.ptr(Bd), Bst.shape[1],
               L.ptr(Cd), N, splits, M * N, _s())
    out = Cd.sum(0).cpu().double()
    exact = A.double() @ B.double().t()
    e3 = (out - exact).abs().max().item()
    assert e3 <= _tol(3, K), (e3, _tol(3, K))
    # plain bf16's error on a row block (the full fp64 bf16 product is slow on the CPU)
    eb = ((A[:256].bfloat16().double() @ B.bfloat16().double().t()) - exact[:256]).abs().max().item()
    assert e3 < 0.05 * eb, (e3, eb)


@pytest.mark.parametrize("prec", [0, 2, 3])
def test_gemm_grouped(L, prec):
    """Several matmuls of different orientation / shape / split count in one launch."""
    g = torch.Generator().manual_seed(11)
    specs = [("nt", 128, 1928, 1024, 5), ("nt", 128, 48, 1024, 8), ("tn", 1024, 440, 128, 1),
             ("nn", 128, 1024, 1024, 8), ("nn", 37, 70, 45, 1), ("tn", 16, 96, 32, 1)]
    probs, keep, refs = [], [], []
    for orient, M, N, K, sp in specs:
        A = torch.randn(M, K, generator=g)
        B = torch.randn(N, K, generator=g)
        akc, bkc = {"nt": (1, 1), "nn": (1, 0), "tn": (0, 0)}[orient]
        Ast = A if akc else A.t().contiguous()
        Bst = B if bkc else B.t().contiguous()
        if prec in (1, 2):
            A, B = A.bfloat16().float(), B.bfloat16().float()
        refs.append((A.double() @ B.double().t()).float())
        Ad, Bd = Ast.to(DEV), Bst.to(DEV)
        if prec == 2:
            Ad, Bd = Ad.bfloat16().contiguous(), Bd.bfloat16().contiguous()
        Cd = torch.full((sp, M, N), float("nan"), device=DEV)
        keep += [Ad, Bd, Cd]
        probs.append(L.GemmProblem(a_kcontig=akc, b_kcontig=bkc, M=M, N=N, K=K, splits=sp,
                                   A=Ad.data_ptr(), lda=Ast.shape[1], B=Bd.data_ptr(),
                                   ldb=Bst.shape[1], C=Cd.data_ptr(), ldc=N, slab_stride=M * N))
    arr = (L.GemmProblem * len(probs))(*probs)
    L.call("pkc_gemm_grouped", prec, arr, len(probs), _s())
    torch.cuda.synchronize()
    for (orient, M, N, K, sp), ref, Cd in zip(specs, refs, keep[2::3]):
        torch.testing.assert_close(Cd.sum(0).cpu(), ref, rtol=1e-4, atol=_tol(prec, K))


@pytest.mark.parametrize("prec", [0, 3])
def test_gemm_grouped_c2_backward(L, prec):
    """The C2 step's backward launch shapes, every problem on the 16-byte path (the vec-only
    grouped instance held to 4 waves per SIMD): dW (K = 128 batch rows) and split-K dX."""
    g = torch.Generator().manual_seed(13)
    specs = [("nn", 128, 1024, 1024, 4), ("tn", 1024, 1024, 128, 1), ("nn", 128, 1024, 1928, 7),
             ("tn", 1928, 1024, 128, 1), ("tn", 1024, 440, 128, 1)]
    probs, keep, refs = [], [], []
    for orient, M, N, K, sp in specs:
        A = torch.randn(M, K, generator=g) * 1e-3
        B = torch.randn(N, K, generator=g)
        akc, bkc = {"nt": (1, 1), "nn": (1, 0), "tn": (0, 0)}[orient]
        Ast = A if akc else A.t().contiguous()
        Bst = B if bkc else B.t().contiguous()
        refs.append((A.double() @ B.double().t()))
        Ad, Bd = Ast.to(DEV), Bst.to(DEV)
        Cd = torch.full((sp, M, N), float("nan"), device=DEV)
        keep += [Ad, Bd, Cd]
        probs.append(L.GemmProblem(a_kcontig=akc, b_kcontig=bkc, M=M, N=N, K=K, splits=sp,
                                   A=Ad.data_ptr(), lda=Ast.shape[1], B=Bd.data_ptr(),
                                   ldb=Bst.shape[1], C=Cd.data_ptr(), ldc=N, slab_stride=M * N))
    arr = (L.GemmProblem * len(probs))(*probs)
    L.call("pkc_gemm_grouped", prec, arr, len(probs), _s())
    torch.cuda.synchronize()
    for (orient, M, N, K, sp), ref, Cd in zip(specs, refs, keep[2::3]):
        got = Cd.sum(0).cpu().double()
        rel = ((got - ref).norm() / ref.norm()).item()
        assert rel < (1e-6 if prec == 0 else 3e-5), (orient, M, N, K, rel)


@pytest.mark.parametrize("prec,M,p", [(2, 4096, 0.15), (2, 1000, 0.0), (1, 2048, 0.15)])
def test_gemm_bnbwd_epilogue(L, prec, M, p):
    """pkc_bn_bwd_epi: the dX matmul (M x 1024 x 1024, the 128x128 body in a grouped launch) stores
    dy = g keep / (1 - p) relu'(gamma xhat + beta) and per-128-row-block column sums of dy and
    dy * xhat; pkc_dense_bwd_pre on them = pkc_dense_bwd (statistics pass) on g.  (Exact fp32
    takes the 128x128 body only from 1024 tiles on: at these shapes it has no epilogue form.)"""
    N, K = 1024, 1024
    g = torch.Generator().manual_seed(M + int(100 * p))
    A = torch.randn(M, K, generator=g)
    W = torch.randn(K, N, generator=g) * K ** -0.5        # dX = A W (b stored as (K, N): m-contig)
    xhat = torch.randn(M, N, generator=g)
    keep = (torch.rand(M, N, generator=g) > p).to(torch.uint8)
    gamma, beta = torch.rand(N, generator=g) + 0.5, torch.randn(N, generator=g) * 0.1
    dt = torch.bfloat16 if prec == 2 else torch.float32
    Ad, Wd = A.to(DEV).to(dt).contiguous(), W.to(DEV).to(dt).contiguous()
    if prec:
        A, W = A.bfloat16().float(), W.bfloat16().float()
    assert L.lib().pkc_gemm_bnbwd_ok(prec, 1, 0, M, N, K, L.ptr(Ad), K, L.ptr(Wd), N) == 128
    assert L.lib().pkc_gemm_bnbwd_ok(0, 1, 0, M, N, K, L.ptr(Ad), K, L.ptr(Wd), N) == 0
    dev = {k: v.to(DEV).contiguous() for k, v in dict(xhat=xhat, keep=keep, gamma=gamma, beta=beta).items()}
    work = torch.zeros(L.lib().pkc_dense_work_size(M, N), device=DEV)
    dz = torch.full((M, N), float("nan"), device=DEV)
    epi = L.BnBwdEpi(xhat=dev["xhat"].data_ptr(), keep=dev["keep"].data_ptr() if p > 0 else None,
                     gamma=dev["gamma"].data_ptr(), beta=dev["beta"].data_ptr(),
                     part=work.data_ptr(), act=L.ACT["relu"], drop_p=p)
    pr = L.GemmProblem(a_kcontig=1, b_kcontig=0, M=M, N=N, K=K, splits=1, A=Ad.data_ptr(), lda=K,
                       B=Wd.data_ptr(), ldb=N, C=dz.data_ptr(), ldc=N, slab_stride=0,
                       X1=C.addressof(epi))
    L.call("pkc_gemm_grouped", prec, C.byref(pr), 1, _s())
    torch.cuda.synchronize()
    gref = A.double() @ W.double()
    y = xhat.double() * gamma.double() + beta.double()
    dyr = gref * (keep.double() / (1 - p) if p > 0 else 1.0) * (y > 0).double()
    tol = (2e-5 if prec == 0 else 1e-3) * K ** 0.5 * K ** -0.5 * 4
    torch.testing.assert_close(dz.cpu().double(), dyr, rtol=1e-3, atol=tol)
    nb = -(-M // 128)
    part = work[:2 * N * nb].view(nb, 2, N).cpu().double()
    got = dz.cpu().double()
    for b in range(nb):
        blk, xb = got[128 * b:128 * (b + 1)], xhat.double()[128 * b:128 * (b + 1)]
        torch.testing.assert_close(part[b, 0], blk.sum(0), rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(part[b, 1], (blk * xb).sum(0), rtol=1e-4, atol=1e-4)
    # the rest of the backward from the partials vs the statistics-pass form on the same g
    gd = torch.from_numpy(gref.float().numpy()).to(DEV) if prec == 0 else None
    if gd is None:      # the same g the epilogue saw: recompute the product without it
        gd = torch.full((M, N), float("nan"), device=DEV)
        L.call("pkc_gemm", prec, 1, 0, M, N, K, L.ptr(Ad), K, L.ptr(Wd), N, L.ptr(gd), N, 1, 0, _s())
    invstd = (torch.rand(N, generator=g) + 0.5).to(DEV)
    outs = []
    for fn in ("pkc_dense_bwd", "pkc_dense_bwd_pre"):
        dzo = dz.clone() if fn == "pkc_dense_bwd_pre" else torch.zeros(M, N, device=DEV)
        dg, db, dbias = (torch.zeros(N, device=DEV) for _ in range(3))
        a = L.DenseBwdArgs(M=M, N=N, nslab=1, gslab=gd.data_ptr(), slab_stride=M * N,
                           norm=L.NORM_BN_TRAIN, act=L.ACT["relu"], gamma=dev["gamma"].data_ptr(),
                           beta=dev["beta"].data_ptr(), save_invstd=invstd.data_ptr(),
                           xhat=dev["xhat"].data_ptr(), keep=dev["keep"].data_ptr() if p > 0 else None,
                           drop_p=p, dz=dzo.data_ptr(), dgamma=dg.data_ptr(), dbeta=db.data_ptr(),
                           dbias=dbias.data_ptr())
        if fn == "pkc_dense_bwd":
            w2 = torch.zeros_like(work)
            L.call(fn, C.byref(a), L.ptr(w2), _s())
        else:
            L.call(fn, C.byref(a), L.ptr(work), 128, _s())
        outs.append((dzo.cpu(), dg.cpu(), db.cpu()))
    (z0, g0, b0), (z1, g1, b1) = outs
    torch.testing.assert_close(g1, g0, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(b1, b0, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(z1, z0, rtol=1e-4, atol=1e-5)


def test_gemm_unaligned_lda(L):
    """First layer reading straight out of a (N, 442) chunk matrix: scalar-load path."""
    M, N, K = 33, 64, 440
    X = torch.randn(M, 442)
    W = torch.randn(N, K)
    ref = X[:, :K].double() @ W.double().t()
    Xd, Wd = X.to(DEV), W.to(DEV)
    Cd = torch.zeros(M, N, device=DEV)
    L.call("pkc_gemm", 0, 1, 1, M, N, K, L.ptr(Xd), 442, L.ptr(Wd), K, L.ptr(Cd), N, 1, 0, _s())
    torch.testing.assert_close(Cd.cpu().double(), ref, rtol=1e-5, atol=1e-4)


def _bn_ref(z, gamma, beta, act, keep, p):
    zz = z.clone().requires_grad_(True)
    gg = gamma.clone().requires_grad_(True)
    bb = beta.clone().requires_grad_(True)
    y = torch.nn.functional.batch_norm(zz, None, None, gg, bb, training=True, momentum=0.05, eps=1e-5)
    a = {"relu": torch.relu, "tanh": torch.tanh, "sigmoid": torch.sigmoid, "linear": lambda t: t}[act](y)
    if p > 0:
        a = a * keep / (1 - p)
    return zz, gg, bb, a


@pytest.mark.parametrize("act", ["relu", "tanh", "sigmoid", "linear"])
@pytest.mark.parametrize("p", [0.0, 0.15])
@pytest.mark.parametrize("M,N,S", [(128, 1024, 4), (16, 48, 1), (50, 70, 3), (100, 1028, 7), (300, 64, 2),
                                   (2000, 256, 1), (1700, 100, 3), (200, 24, 2), (256, 64, 1),
                                   (129, 40, 8), (4096, 1024, 1), (4112, 1280, 2)])
def test_dense_bn_fwd_bwd(L, act, p, M, N, S):
    g = torch.Generator().manual_seed(M + N + S)
    slabs = torch.randn(S, M, N, generator=g)
    bias = torch.randn(N, generator=g) * 0.1
    gamma = torch.rand(N, generator=g) + 0.5
    beta = torch.randn(N, generator=g) * 0.1
    keep = (torch.rand(M, N, generator=g) > p).to(torch.uint8)
    z = slabs.sum(0) + bias
    zz, gg, bb, a = _bn_ref(z, gamma, beta, act, keep.float(), p)
    gout = torch.randn(2, M, N, generator=g)
    a.backward(gout.sum(0))
    d = {k: v.to(DEV) for k, v in dict(slabs=slabs, bias=bias, gamma=gamma, beta=beta,
                                        keep=keep, gout=gout).items()}
    rm, rv = torch.zeros(N, device=DEV), torch.ones(N, device=DEV)
    sm, si = torch.zeros(N, device=DEV), torch.zeros(N, device=DEV)
    xhat, out = torch.zeros(M, N, device=DEV), torch.zeros(M, N, device=DEV)
    a_ = L.DenseFwdArgs(M=M, N=N, nslab=S, zslab=d["slabs"].data_ptr(), slab_stride=M * N,
                        bias=d["bias"].data_ptr(), norm=L.NORM_BN_TRAIN, gamma=d["gamma"].data_ptr(),
                        beta=d["beta"].data_ptr(), running_mean=rm.data_ptr(),
                        running_var=rv.data_ptr(), momentum=0.05, eps=1e-5, save_mean=sm.data_ptr(),
                        save_invstd=si.data_ptr(), act=L.ACT[act], drop_p=p, seed=1, step_ctr=None,
                        stream_id=0, keep_in=d["keep"].data_ptr() if p > 0 else None,
                        keep_out=None, xhat=xhat.data_ptr(), out=out.data_ptr())
    work = torch.zeros(L.lib().pkc_dense_work_size(M, N), device=DEV)
    L.call("pkc_dense_fwd", C.byref(a_), L.ptr(work), _s())
    torch.testing.assert_close(out.cpu(), a.detach(), rtol=1e-4, atol=1e-5)
    mu = z.mean(0)
    var = z.var(0, unbiased=True)
    torch.testing.assert_close(rm.cpu(), 0.05 * mu, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(rv.cpu(), 0.95 + 0.05 * var, rtol=1e-4, atol=1e-6)
    dz = torch.zeros(M, N, device=DEV)
    dgam, dbet, dbias = (torch.zeros(N, device=DEV) for _ in range(3))
    b_ = L.DenseBwdArgs(M=M, N=N, nslab=2, gslab=d["gout"].data_ptr(), slab_stride=M * N,
                        norm=L.NORM_BN_TRAIN, act=L.ACT[act], gamma=d["gamma"].data_ptr(),
                        beta=d["beta"].data_ptr(), save_invstd=si.data_ptr(), xhat=xhat.data_ptr(),
                        keep=d["keep"].data_ptr() if p > 0 else None, drop_p=p, dz=dz.data_ptr(),
                        dgamma=dgam.data_ptr(), dbeta=dbet.data_ptr(), dbias=dbias.data_ptr())
    L.call("pkc_dense_bwd", C.byref(b_), L.ptr(work), _s())
    # a pre-activation within rounding of a kink (ReLU at 0) may take the other branch on the GPU;
    # through the BN mean terms that changes its whole column: compare the other columns
    y = torch.nn.functional.batch_norm(z, None, None, gamma, beta, training=True, eps=1e-5)
    # (fp32 differences here are ~1e-6 of y's scale; at M = 2000 rows a 1e-4 margin would drop
    # a fifth of the columns)
    cols = (y.abs() > 1e-5).all(0) if act == "relu" else torch.ones(N, dtype=torch.bool)
    assert cols.float().mean() > 0.95
    torch.testing.assert_close(dz.cpu()[:, cols], zz.grad[:, cols], rtol=1e-3, atol=1e-5)
    torch.testing.assert_close(dgam.cpu()[cols], gg.grad[cols], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dbet.cpu()[cols], bb.grad[cols], rtol=1e-4, atol=1e-4)
    assert (dbias.cpu() == 0).all()          # bias before BN: exact zero gradient
    # ... which autograd reproduces up to the rounding of an M-term fp32 sum
    assert zz.grad.sum(0).abs().max() < 1e-4 * max(1.0, M / 256)


@pytest.mark.parametrize("act", ["relu", "tanh"])
@pytest.mark.parametrize("p", [0.0, 0.15])
@pytest.mark.parametrize("M,N,K", [(128, 1024, 1024), (128, 1024, 440), (100, 64, 96), (1, 16, 8),
                                   (128, 48, 1032)])
def test_dense_gemm_fwd_fused(L, act, p, M, N, K):
    """pkc_dense_gemm_fwd (matmul + BatchNorm / activation / dropout in one launch, every row of a
    16-column strip per workgroup) against torch on the bf16-rounded operands: out, xhat, the
    batch statistics, running statistics, keep mask; the fp32-staged form (PKC_PREC_BF16) equal
    bit for bit to the bf16-stored one (BF16IN), and both equal to the split-K matmul + pkc_dense_fwd
    path up to the fp32 summation order of the K-deep products."""
    g = torch.Generator().manual_seed(M * 3 + N + K)
    X = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / K ** 0.5
    bias = torch.randn(N, generator=g) * 0.1
    gamma = torch.rand(N, generator=g) + 0.5
    beta = torch.randn(N, generator=g) * 0.1
    keep = (torch.rand(M, N, generator=g) > p).to(torch.uint8)
    z = (X.bfloat16().double() @ W.bfloat16().double().t()).float() + bias
    _, _, _, ref = _bn_ref(z, gamma, beta, act, keep.float(), p) if M > 1 else (None,) * 4
    d = {k: v.to(DEV) for k, v in dict(X=X, W=W, bias=bias, gamma=gamma, beta=beta,
                                        keep=keep).items()}
    outs = {}
    for prec in (1, 2):                          # PKC_PREC_BF16 (fp32 staged), PKC_PREC_BF16IN
        Xd, Wd = (d["X"], d["W"]) if prec == 1 else (d["X"].bfloat16(), d["W"].bfloat16())
        rm, rv = torch.zeros(N, device=DEV), torch.ones(N, device=DEV)
        sm, si = torch.zeros(N, device=DEV), torch.zeros(N, device=DEV)
        xhat, out = torch.zeros(M, N, device=DEV), torch.zeros(M, N, device=DEV)
        outh = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
        kout = torch.zeros(M, N, dtype=torch.uint8, device=DEV)
        a_ = L.DenseFwdArgs(M=M, N=N, nslab=1, zslab=None, slab_stride=0, bias=d["bias"].data_ptr(),
                            norm=L.NORM_BN_TRAIN, gamma=d["gamma"].data_ptr(),
                            beta=d["beta"].data_ptr(), running_mean=rm.data_ptr(),
                            running_var=rv.data_ptr(), momentum=0.05, eps=1e-5,
                            save_mean=sm.data_ptr(), save_invstd=si.data_ptr(), act=L.ACT[act],
                            drop_p=p, seed=1, step_ctr=None, stream_id=0,
                            keep_in=d["keep"].data_ptr() if p > 0 else None,
                            keep_out=kout.data_ptr() if p > 0 else None, xhat=xhat.data_ptr(),
                            out=out.data_ptr(), out_bf16=outh.data_ptr())
        assert L.lib().pkc_dense_gemm_fwd_ok(prec, M, N, K, C.c_void_p(Xd.data_ptr()), K,
                                             C.c_void_p(Wd.data_ptr()), K)
        L.call("pkc_dense_gemm_fwd", prec, L.ptr(Xd), K, L.ptr(Wd), K, K, C.byref(a_), _s())
        torch.cuda.synchronize()
        outs[prec] = [t.cpu() for t in (out, xhat, sm, si, rm, rv, outh.float(), kout)]
    for a, b in zip(outs[1], outs[2]):
        assert torch.equal(a, b), "fp32-staged and bf16-stored operands differ"
    out, xhat, sm, si, rm, rv, outh, kout = outs[2]
    assert torch.equal(outh, out.bfloat16().float())
    if p > 0:
        assert torch.equal(kout, keep)
    if M == 1:                                   # one row: BatchNorm gives beta, xhat 0
        assert torch.equal(xhat, torch.zeros_like(xhat))
        return
    mu, var = z.double().mean(0), z.double().var(0, unbiased=False)
    torch.testing.assert_close(sm, mu.float(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(si, (1 / (var + 1e-5).sqrt()).float(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rm, 0.05 * mu.float(), rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(rv, 0.95 + 0.05 * z.var(0, unbiased=True), rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(xhat, ((z.double() - mu) / (var + 1e-5).sqrt()).float(), rtol=1e-4,
                               atol=2e-5)
    torch.testing.assert_close(out, ref.detach(), rtol=1e-4, atol=2e-5)
    # the unfused path (split-K slabs + pkc_dense_fwd) on the same rounded operands
    splits = L.lib().pkc_gemm_pick_splits(M, N, K)
    Cd = torch.zeros(splits, M, N, device=DEV)
    Xb, Wb = d["X"].bfloat16(), d["W"].bfloat16()
    L.call("pkc_gemm", 2, 1, 1, M, N, K, L.ptr(Xb), K, L.ptr(Wb), K, L.ptr(Cd), N, splits, M * N,
           _s())
    rm2, rv2 = torch.zeros(N, device=DEV), torch.ones(N, device=DEV)
    sm2, si2 = torch.zeros(N, device=DEV), torch.zeros(N, device=DEV)
    xhat2, out2 = torch.zeros(M, N, device=DEV), torch.zeros(M, N, device=DEV)
    a2 = L.DenseFwdArgs(M=M, N=N, nslab=splits, zslab=Cd.data_ptr(), slab_stride=M * N,
                        bias=d["bias"].data_ptr(), norm=L.NORM_BN_TRAIN, gamma=d["gamma"].data_ptr(),
                        beta=d["beta"].data_ptr(), running_mean=rm2.data_ptr(),
                        running_var=rv2.data_ptr(), momentum=0.05, eps=1e-5, save_mean=sm2.data_ptr(),
                        save_invstd=si2.data_ptr(), act=L.ACT[act], drop_p=p, seed=1, step_ctr=None,
                        stream_id=0, keep_in=d["keep"].data_ptr() if p > 0 else None, keep_out=None,
                        xhat=xhat2.data_ptr(), out=out2.data_ptr())
    work = torch.zeros(L.lib().pkc_dense_work_size(M, N), device=DEV)
    L.call("pkc_dense_fwd", C.byref(a2), L.ptr(work), _s())
    torch.testing.assert_close(out, out2.cpu(), rtol=1e-4, atol=2e-5)
    torch.testing.assert_close(xhat, xhat2.cpu(), rtol=1e-4, atol=2e-5)


def test_dense_dropout_rate_and_determinism(L):
    M, N, p = 256, 512, 0.15
    z = torch.randn(1, M, N, device=DEV)
    ctr = torch.tensor([3, 0], dtype=torch.int64, device=DEV)
    outs, keeps = [], []
    for _ in range(2):
        keep = torch.zeros(M, N, dtype=torch.uint8, device=DEV)
        out = torch.zeros(M, N, device=DEV)
        a_ = L.DenseFwdArgs(M=M, N=N, nslab=1, zslab=z.data_ptr(), slab_stride=M * N, bias=None,
                            norm=L.NORM_NONE, act=L.ACT["linear"], drop_p=p, seed=7,
                            step_ctr=ctr.data_ptr(), stream_id=5, keep_out=keep.data_ptr(),
                            out=out.data_ptr())
        L.call("pkc_dense_fwd", C.byref(a_), None, _s())
        outs.append(out.cpu())
        keeps.append(keep.cpu())
    assert torch.equal(keeps[0], keeps[1])
    rate = 1 - keeps[0].float().mean().item()
    assert abs(rate - p) < 0.01
    k = keeps[0].bool()
    torch.testing.assert_close(outs[0][k], z[0].cpu()[k] / (1 - p))
    assert (outs[0][~k] == 0).all()


def test_nll_fused_multi_equals_single(L):
    """Both heads' LogSoftmax/NLL in one launch == one launch per head."""
    M = 128
    outs = []
    heads = [(1928, 5), (48, 8)]
    g = torch.Generator().manual_seed(3)
    data = [(torch.randn(S, M, N, generator=g).to(DEV), torch.randn(N, generator=g).to(DEV),
             torch.randint(0, N, (M,), generator=g, dtype=torch.int32).to(DEV)) for N, S in heads]
    for multi in (False, True):
        args = (L.NllArgs * 2)()
        bufs = []
        for i, ((N, S), (z, b, lab)) in enumerate(zip(heads, data)):
            lp, dl, rl, re_ = (torch.zeros(M, N, device=DEV), torch.zeros(M, N, device=DEV),
                               torch.zeros(M, device=DEV), torch.zeros(M, device=DEV))
            bufs.append((lp, dl, rl, re_))
            args[i] = L.NllArgs(M=M, N=N, nslab=S, zslab=z.data_ptr(), slab_stride=M * N,
                                bias=b.data_ptr(), labels=lab.data_ptr(), label_stride=1, weight=0.5,
                                logp=lp.data_ptr(), dlogits=dl.data_ptr(), row_loss=rl.data_ptr(),
                                row_err=re_.data_ptr())
        if multi:
            L.call("pkc_nll_fused_multi", args, 2, _s())
        else:
            for i in range(2):
                L.call("pkc_nll_fused", C.byref(args[i]), _s())
        torch.cuda.synchronize()
        outs.append([[t.cpu() for t in bb] for bb in bufs])
    for a, b in zip(outs[0], outs[1]):
        for x, y in zip(a, b):
            assert torch.equal(x, y)


@pytest.mark.parametrize("M,N,S", [(128, 1928, 4), (128, 48, 2), (7, 100, 1)])
def test_nll_fused(L, M, N, S):
    g = torch.Generator().manual_seed(N)
    slabs = torch.randn(S, M, N, generator=g) * 3
    bias = torch.randn(N, generator=g)
    lab = torch.randint(0, N, (M, 2), generator=g, dtype=torch.int32)
    z = (slabs.sum(0) + bias).requires_grad_(True)
    lp = torch.log_softmax(z, 1)
    loss = torch.nn.functional.nll_loss(lp, lab[:, 1].long())
    (0.7 * loss).backward()
    err = (lp.argmax(1) != lab[:, 1].long()).float().mean()
    d = [t.to(DEV) for t in (slabs, bias, lab)]
    logp, dl = torch.zeros(M, N, device=DEV), torch.zeros(M, N, device=DEV)
    rl, re_ = torch.zeros(M, device=DEV), torch.zeros(M, device=DEV)
    a = L.NllArgs(M=M, N=N, nslab=S, zslab=d[0].data_ptr(), slab_stride=M * N, bias=d[1].data_ptr(),
                  labels=d[2].data_ptr() + 4, label_stride=2, weight=0.7, logp=logp.data_ptr(),
                  log_prior=None, dlogits=dl.data_ptr(), row_loss=rl.data_ptr(), row_err=re_.data_ptr())
    L.call("pkc_nll_fused", C.byref(a), _s())
    torch.testing.assert_close(logp.cpu(), lp.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(dl.cpu(), z.grad, rtol=1e-4, atol=1e-7)
    torch.testing.assert_close(rl.mean().cpu(), loss.detach(), rtol=1e-5, atol=1e-6)
    assert abs(re_.mean().item() - err.item()) < 1e-6
    out, acc = torch.zeros(3, device=DEV), torch.zeros(2, device=DEV)
    ptrs = torch.tensor([rl.data_ptr()], dtype=torch.int64, device=DEV)
    w = torch.tensor([0.7], device=DEV)
    ctr = torch.zeros(1, dtype=torch.int64, device=DEV)
    L.call("pkc_loss_finalize", 1, L.ptr(ptrs), L.ptr(w), M, L.ptr(re_), L.ptr(out), L.ptr(acc),
           L.ptr(ctr), _s())
    torch.testing.assert_close(out[0].cpu(), 0.7 * loss.detach(), rtol=1e-5, atol=1e-6)
    assert int(ctr.item()) == 1
    # the same reduction as an operation of a grouped launch, beside a column sum
    out2, acc2 = torch.zeros_like(out), torch.zeros_like(acc)
    cs = torch.zeros(N, device=DEV)
    ops = (L.GemmProblem * 2)(
        L.GemmProblem(kind=L.OP_LOSS, M=1, N=M, A=ptrs.data_ptr(), B=w.data_ptr(),
                      C=out2.data_ptr(), X1=re_.data_ptr(), X2=acc2.data_ptr(), X3=ctr.data_ptr()),
        L.GemmProblem(kind=L.OP_COLSUM, M=M, N=N, A=dl.data_ptr(), C=cs.data_ptr()))
    L.call("pkc_gemm_grouped", 0, ops, 2, _s())
    torch.testing.assert_close(out2.cpu(), out.cpu())
    torch.testing.assert_close(cs.cpu(), dl.sum(0).cpu(), rtol=1e-5, atol=1e-6)
    assert int(ctr.item()) == 2


@pytest.mark.parametrize("kind", ["sgd", "rmsprop", "adam", "sgd_mom"])
def test_optimizer_step_matches_torch(L, kind):
    g = torch.Generator().manual_seed(3)
    sizes = [1000, 5000, 3]
    ps = [torch.randn(n, generator=g) for n in sizes]
    masks = [None, (torch.rand(5000, generator=g) > 0.5).float(), None]
    grads = [[torch.randn(n, generator=g) for n in sizes] for _ in range(3)]
    ref = [p.clone().requires_grad_(True) for p in ps]
    if kind == "sgd":
        opt = torch.optim.SGD(ref, lr=0.08)
    elif kind == "sgd_mom":
        opt = torch.optim.SGD(ref, lr=0.05, momentum=0.9, nesterov=True, weight_decay=1e-3)
    elif kind == "rmsprop":
        opt = torch.optim.RMSprop(ref, lr=4e-4, alpha=0.95, eps=1e-8)
    else:
        opt = torch.optim.Adam(ref, lr=1e-3, betas=(0.9, 0.98), eps=1e-8)
    dps = [p.to(DEV) for p in ps]
    for i, m in enumerate(masks):
        if m is not None:
            dps[i].mul_(m.to(DEV))
            with torch.no_grad():
                ref[i].mul_(m)
    dgs = [torch.zeros(n, device=DEV) for n in sizes]
    st = [[torch.zeros(n, device=DEV) for n in sizes] for _ in range(3)]
    dmask = [m.to(DEV) if m is not None else None for m in masks]
    n = len(sizes)
    szs = (C.c_int64 * n)(*sizes)
    nch = L.lib().pkc_optim_chunks(szs, n, None, 0)
    cmap = (C.c_int32 * (2 * nch))()
    L.lib().pkc_optim_chunks(szs, n, cmap, nch)
    dmap = torch.from_numpy(np.frombuffer(cmap, dtype=np.int32).copy()).to(DEV)
    for step in range(3):
        arr = (L.OptTensor * n)()
        for i in range(n):
            t = arr[i]
            t.p, t.g, t.s1, t.s2, t.s3 = (dps[i].data_ptr(), dgs[i].data_ptr(), st[0][i].data_ptr(),
                                          st[1][i].data_ptr(), st[2][i].data_ptr())
            t.mask = dmask[i].data_ptr() if dmask[i] is not None else None
            t.n = sizes[i]
            t.step = step + 1
            if kind == "sgd":
                t.kind, t.lr = 0, 0.08
            elif kind == "sgd_mom":
                t.kind, t.lr, t.momentum, t.nesterov, t.wd = 0, 0.05, 0.9, 1, 1e-3
            elif kind == "rmsprop":
                t.kind, t.lr, t.alpha, t.eps = 1, 4e-4, 0.95, 1e-8
            else:
                t.kind, t.lr, t.beta1, t.beta2, t.eps = 2, 1e-3, 0.9, 0.98, 1e-8
        desc = torch.frombuffer(bytearray(C.string_at(arr, C.sizeof(arr))), dtype=torch.uint8).to(DEV)
        for i in range(n):
            dgs[i].copy_(grads[step][i].to(DEV))
            ref[i].grad = grads[step][i].clone()
        L.call("pkc_optim_step", L.ptr(desc), n, L.ptr(dmap), nch, _s())
        opt.step()
        with torch.no_grad():
            for i, m in enumerate(masks):
                if m is not None:
                    ref[i].mul_(m)
    for i in range(n):
        torch.testing.assert_close(dps[i].cpu(), ref[i].detach(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("L_,R_", [(5, 5), (2, 1), (0, 0), (1, 3)])
def test_context_window_chunk_prep(L, L_, R_):
    """pkc_cw_stats/pkc_cw_apply vs the oracle's numpy float64 load_chunk (+ shuffle)."""
    from oracle import loader as OL
    from pkc import data_io
    rs = np.random.RandomState(L_ * 10 + R_)
    fea = {"u%02d" % i: (rs.randn(rs.randint(20, 90), 40) + rs.randn(1, 40)).astype(np.float32)
           for i in range(9)}
    cd = {k: rs.randint(2, 1928, size=len(v)).astype(np.int32) for k, v in fea.items()}
    mono = {k: rs.randint(1, 49, size=len(v)).astype(np.int32) for k, v in fea.items()}
    names, end, fcols, lcols, ref = OL.read_lab_fea([("fmllr", fea, L_, R_)],
                                                    [("lab_cd", cd), ("lab_mono", mono)], False,
                                                    rng=np.random.RandomState(2234))
    ch = data_io.prepare_chunk(fea, [cd, mono], ["lab_cd", "lab_mono"], L_, R_, 1000,
                               shuffle_rng=np.random.RandomState(2234), fea_name="fmllr")
    assert ch.names == names
    np.testing.assert_array_equal(ch.end_index, end)
    C_ = 40 * (L_ + R_ + 1)
    np.testing.assert_allclose(ch.feats.cpu().numpy(), ref[:, :C_].astype(np.float32), rtol=1e-6,
                               atol=1e-6)
    np.testing.assert_array_equal(ch.labels.cpu().numpy(), ref[:, C_:].astype(np.int32))


@pytest.mark.parametrize("shape,perc,zeros", [((1024, 440), 70.0, 0.0), ((64, 64), 50.0, 0.5),
                                              ((33, 17), 12.5, 0.0), ((128, 96), 99.9, 0.3),
                                              ((40, 40), 0.0, 0.0), ((40, 40), 100.0, 0.0)])
def test_prune_matches_numpy_percentile(L, shape, perc, zeros):
    """pkc_prune == quantized_modules.prune (np.percentile 'linear' + strict >) bit for bit,
    including matrices that are partly zero (HCGS-masked) and the 0 / 100 edges."""
    from oracle.masks import prune_mask
    g = torch.Generator().manual_seed(int(perc * 10) + shape[0])
    w = torch.randn(*shape, generator=g)
    if zeros:
        w = w * (torch.rand(*shape, generator=g) > zeros).float()
    ref_mask = prune_mask(w, perc)
    wd = w.to(DEV).contiguous()
    mask = torch.full(shape, 7.0, device=DEV)
    work = torch.zeros(L.lib().pkc_prune_work_size(), dtype=torch.uint8, device=DEV)
    L.call("pkc_prune", L.ptr(wd), w.numel(), C.c_double(perc), L.ptr(mask), L.ptr(work), _s())
    torch.cuda.synchronize()
    assert torch.equal(mask.cpu(), ref_mask)
    assert torch.equal(wd.cpu(), w * ref_mask)


# shapes that take the 128x128 body (pkc_gemm_big.h: >= 160 output tiles of 128x128, 16-byte
# operand paths): ragged M / N tails, K tails off the 32/64 k-tile, split-K slabs
BIG_SHAPES = [(4096, 4096, 256, 1), (2048, 1280, 440, 1), (2056, 1288, 1000, 1), (4096, 1024, 1024, 2), (5280, 1024, 2048, 1),
              (1032, 2600, 136, 3),
              # <= 256 tiles, K % 64 == 0: the LDS-DMA ring body for bf16-stored operands (prec 2),
              # ragged M / N tails, 3 to 32 k-tiles per workgroup
              (4096, 1024, 1024, 1), (2056, 1288, 1024, 1), (2048, 1280, 2048, 1), (1280, 2048, 192, 1)]


@pytest.mark.parametrize("prec", [0, 1, 2])
@pytest.mark.parametrize("M,N,K,splits", BIG_SHAPES)
@pytest.mark.parametrize("orient", ["nt", "nn", "tn", "tt"])
def test_gemm_big_tile(L, prec, M, N, K, splits, orient):
    """The large-M matmuls of the sequence models and big-batch MLPs (the 128x128 tile body) vs
    fp64 products of the same (bf16-rounded for prec 1/2) operands, in every orientation."""
    g = torch.Generator().manual_seed(M + 3 * N + 7 * K)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g)
    akc, bkc = {"nt": (1, 1), "nn": (1, 0), "tn": (0, 0), "tt": (0, 1)}[orient]
    Ast = A if akc else A.t().contiguous()
    Bst = B if bkc else B.t().contiguous()
    if prec >= 1:
        A = A.bfloat16().float()
        B = B.bfloat16().float()
    ref = (A.double() @ B.double().t()).float()
    Ad, Bd = Ast.to(DEV), Bst.to(DEV)
    if prec == 2:
        Ad, Bd = Ad.bfloat16().contiguous(), Bd.bfloat16().contiguous()
    Cd = torch.full((splits, M, N), float("nan"), device=DEV)
    L.call("pkc_gemm", prec, akc, bkc, M, N, K, L.ptr(Ad), Ast.shape[1], L.ptr(Bd), Bst.shape[1],
           L.ptr(Cd), N, splits, M * N, _s())
    out = Cd.sum(0).cpu()
    tol = 2e-5 * K ** 0.5 if prec == 0 else 1e-3 * K ** 0.5
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=tol)
    if prec == 0 and splits == 1:
        # exact fp32 MFMA chains: the same sums as the 64x64 tile up to fp32 summation order
        assert torch.isfinite(out).all()


@pytest.mark.parametrize("prec", [0, 2])
def test_gemm_grouped_big(L, prec):
    """A grouped launch mixing 128x128-tile problems (the B = 4096 MLP backward's dX and dW) with
    64x64 ones and split-K slabs."""
    g = torch.Generator().manual_seed(5)
    specs = [("nn", 4096, 1024, 1024, 1), ("tn", 1024, 1024, 4096, 2), ("nt", 128, 48, 1024, 4),
             ("nn", 37, 70, 45, 1)]
    probs, keep, refs = [], [], []
    for orient, M, N, K, sp in specs:
        A = torch.randn(M, K, generator=g)
        B = torch.randn(N, K, generator=g)
        akc, bkc = {"nt": (1, 1), "nn": (1, 0), "tn": (0, 0)}[orient]
        Ast = A if akc else A.t().contiguous()
        Bst = B if bkc else B.t().contiguous()
        if prec in (1, 2):
            A, B = A.bfloat16().float(), B.bfloat16().float()
        refs.append((A.double() @ B.double().t()).float())
        Ad, Bd = Ast.to(DEV), Bst.to(DEV)
        if prec == 2:
            Ad, Bd = Ad.bfloat16().contiguous(), Bd.bfloat16().contiguous()
        Cd = torch.full((sp, M, N), float("nan"), device=DEV)
        keep += [Ad, Bd, Cd]
        probs.append(L.GemmProblem(a_kcontig=akc, b_kcontig=bkc, M=M, N=N, K=K, splits=sp,
                                   A=Ad.data_ptr(), lda=Ast.shape[1], B=Bd.data_ptr(),
                                   ldb=Bst.shape[1], C=Cd.data_ptr(), ldc=N, slab_stride=M * N))
    arr = (L.GemmProblem * len(probs))(*probs)
    L.call("pkc_gemm_grouped", prec, arr, len(probs), _s())
    for (orient, M, N, K, sp), ref, Cd in zip(specs, refs, keep[2::3]):
        torch.testing.assert_close(Cd.sum(0).cpu(), ref, rtol=1e-4, atol=_tol(prec, K))


@pytest.mark.parametrize("prec", [0, 2])
@pytest.mark.parametrize("M", [128, 2400])
def test_gemm_block_sparse_matches_dense(L, prec, M):
    """Block-sparse W (k-tile lists from a static mask, pkc.engine.ktile_table): forward
    Z = X (W*mask)^T and dX = dZ (W*mask) skip the all-zero 64x32 weight tiles and give exactly
    the dense matmul's result (the skipped products are zero weights)."""
    from pkc.engine import ktile_table
    g = torch.Generator().manual_seed(M)
    N_out, K_in = 550, 440
    blk = (torch.rand(-(-N_out // 32), -(-K_in // 32), generator=g) < 0.25).float()
    mask = blk.repeat_interleave(32, 0).repeat_interleave(32, 1)[:N_out, :K_in]
    mask = mask * (torch.rand(N_out, K_in, generator=g) < 0.5).float()   # level-2 zeros inside
    W = torch.randn(N_out, K_in, generator=g) * mask
    X = torch.randn(M, K_in, generator=g)
    dZ = torch.randn(M, N_out, generator=g)
    dt = torch.bfloat16 if prec == 2 else torch.float32
    Wd, Xd, dZd = W.to(DEV, dt), X.to(DEV, dt), dZ.to(DEV, dt)
    for transpose in (False, True):
        kt = ktile_table(mask.to(DEV), transpose, DEV)
        assert kt is not None and kt[2] < 0.6
        if not transpose:   # Z[M, N_out] = X W^T
            shape = dict(a_kcontig=1, b_kcontig=1, M=M, N=N_out, K=K_in, A=Xd.data_ptr(), lda=K_in,
                         B=Wd.data_ptr(), ldb=K_in)
            Mo, No = M, N_out
        else:               # dX[M, K_in] = dZ W
            shape = dict(a_kcontig=1, b_kcontig=0, M=M, N=K_in, K=N_out, A=dZd.data_ptr(), lda=N_out,
                         B=Wd.data_ptr(), ldb=K_in)
            Mo, No = M, K_in
        outs = []
        for sparse in (False, True):
            Cd = torch.full((Mo, No), float("nan"), device=DEV)
            extra = dict(ktiles=kt[0].data_ptr(), kmax=kt[1]) if sparse else {}
            pr = L.GemmProblem(splits=1, C=Cd.data_ptr(), ldc=No, slab_stride=Mo * No, **shape, **extra)
            L.call("pkc_gemm_grouped", prec, C.byref(pr), 1, _s())
            outs.append(Cd.cpu())
        torch.testing.assert_close(outs[1], outs[0], rtol=0, atol=0)
        ref = (X.double() @ W.double().t()) if not transpose else (dZ.double() @ W.double())
        if prec == 0:
            torch.testing.assert_close(outs[1], ref.float(), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("prec", [0, 2])
def test_gemm_grouped_sparse_big_slabsum(L, prec):
    """One grouped launch mixing a block-sparse problem, a dense one the 128x128 body would take on
    its own (it must run the 64x64 body in a sparse launch), and a slab-sum operation (a split-K
    dW's partial slabs into one gradient, summed in slab order)."""
    from pkc.engine import ktile_table
    g = torch.Generator().manual_seed(11)
    dt = torch.bfloat16 if prec == 2 else torch.float32
    N_out, K_in, M = 550, 440, 2400
    blk = (torch.rand(-(-N_out // 32), -(-K_in // 32), generator=g) < 0.25).float()
    mask = blk.repeat_interleave(32, 0).repeat_interleave(32, 1)[:N_out, :K_in]
    W = torch.randn(N_out, K_in, generator=g) * mask
    X = torch.randn(M, K_in, generator=g)
    kt = ktile_table(mask.to(DEV), False, DEV)
    A2, B2 = torch.randn(4096, 1024, generator=g), torch.randn(1024, 1024, generator=g)
    slabs = torch.randn(3, 1000, generator=g)
    Wd, Xd, A2d, B2d = W.to(DEV, dt), X.to(DEV, dt), A2.to(DEV, dt), B2.to(DEV, dt)
    C1 = torch.full((M, N_out), float("nan"), device=DEV)
    C2 = torch.full((4096, 1024), float("nan"), device=DEV)
    sd, Cs = slabs.to(DEV), torch.full((1000,), float("nan"), device=DEV)
    probs = [L.GemmProblem(a_kcontig=1, b_kcontig=1, M=M, N=N_out, K=K_in, splits=1, A=Xd.data_ptr(),
                           lda=K_in, B=Wd.data_ptr(), ldb=K_in, C=C1.data_ptr(), ldc=N_out,
                           slab_stride=M * N_out, ktiles=kt[0].data_ptr(), kmax=kt[1]),
             L.GemmProblem(a_kcontig=1, b_kcontig=1, M=4096, N=1024, K=1024, splits=1,
                           A=A2d.data_ptr(), lda=1024, B=B2d.data_ptr(), ldb=1024, C=C2.data_ptr(),
                           ldc=1024, slab_stride=0),
             L.GemmProblem(kind=L.OP_SLABSUM, M=3, N=1000, A=sd.data_ptr(), C=Cs.data_ptr(),
                           slab_stride=1000)]
    arr = (L.GemmProblem * 3)(*probs)
    L.call("pkc_gemm_grouped", prec, arr, 3, _s())
    torch.cuda.synchronize()
    if prec == 2:
        W, X, A2, B2 = (t.bfloat16().float() for t in (W, X, A2, B2))
    tol = 2e-5 if prec == 0 else 1e-3
    torch.testing.assert_close(C1.cpu(), (X.double() @ W.double().t()).float(), rtol=1e-4,
                               atol=tol * K_in ** 0.5)
    torch.testing.assert_close(C2.cpu(), (A2.double() @ B2.double().t()).float(), rtol=1e-4,
                               atol=tol * 1024 ** 0.5)
    assert torch.equal(Cs.cpu(), (slabs[0] + slabs[1]) + slabs[2])


# the large-batch forward with the BatchNorm column statistics in the matmul epilogue: shapes that
# take the 128x128 body (LDS-DMA ring: bf16-stored operands, K % 64 == 0; register body otherwise),
# ragged row / column tails, the first layer's K = 440
COLSTATS_SHAPES = [(4096, 1024, 1024, 2), (4096, 1024, 440, 2), (2056, 1288, 1024, 2),
                   (2056, 1288, 1000, 1), (4096, 4096, 256, 0),
                   # fewer than 160 128x128 tiles: the 64x64 body's 64-row partials (B = 1024)
                   (1024, 1024, 1024, 2), (1000, 1032, 440, 2), (1032, 520, 1000, 1), (264, 200, 96, 0),
                   # compensated bf16: the 64x64 body at every size (no 128x128 form)
                   (1024, 1024, 1024, 3), (4096, 1024, 440, 3)]


@pytest.mark.parametrize("M,N,K,prec", COLSTATS_SHAPES)
def test_gemm_colstats_dense_fwd_pre(L, M, N, K, prec):
    """pkc_gemm_colstats: the one-slab product and per-block column (mean + bias, M2) vs fp64 of
    the same operands (128-row blocks from the 128x128 body, 64-row ones from the 64x64 body);
    pkc_dense_fwd_pre on those partials vs pkc_dense_fwd (the stats-pass form) on the same slab —
    the same BatchNorm up to fp32 summation order."""
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) * K ** -0.5
    bias = torch.randn(N, generator=g) * 0.1
    dt = torch.bfloat16 if prec == 2 else torch.float32
    Ad, Wd, bd = A.to(DEV).to(dt).contiguous(), W.to(DEV).to(dt).contiguous(), bias.to(DEV)
    if prec in (1, 2):
        A, W = A.bfloat16().float(), W.bfloat16().float()
    rows = L.lib().pkc_gemm_colstats_ok(prec, 1, 1, M, N, K, L.ptr(Ad), K, L.ptr(Wd), K)
    tiles = -(-M // 128) * -(-N // 128)
    assert rows == (128 if tiles >= (1024 if prec == 0 else 160) else 64), rows
    Cd = torch.full((M, N), float("nan"), device=DEV)
    work = torch.zeros(L.lib().pkc_dense_work_size(M, N), device=DEV)
    L.call("pkc_gemm_colstats", prec, 1, 1, M, N, K, L.ptr(Ad), K, L.ptr(Wd), K, L.ptr(Cd), N,
           L.ptr(bd), L.ptr(work), _s())
    ref = A.double() @ W.double().t()
    torch.testing.assert_close(Cd.cpu().double(), ref, rtol=1e-4, atol=_tol(prec, K))
    nb = -(-M // rows)
    part = work[:2 * N * nb].view(nb, 2, N).cpu().double()
    z = Cd.cpu().double() + bias.double()
    for b in range(nb):
        blk = z[rows * b:rows * (b + 1)]
        mu = blk.mean(0)
        torch.testing.assert_close(part[b, 0], mu, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(part[b, 1], ((blk - mu) ** 2).sum(0), rtol=1e-4, atol=1e-4)
    # the apply from the partials vs the stats-pass form on the same slab
    gamma = (torch.rand(N, generator=g) + 0.5).to(DEV)
    beta = (torch.randn(N, generator=g) * 0.1).to(DEV)
    outs = []
    for fn in ("pkc_dense_fwd", "pkc_dense_fwd_pre"):
        rm, rv = torch.zeros(N, device=DEV), torch.ones(N, device=DEV)
        sm, si = torch.zeros(N, device=DEV), torch.zeros(N, device=DEV)
        xhat, out = torch.zeros(M, N, device=DEV), torch.zeros(M, N, device=DEV)
        keep = torch.zeros(M, N, dtype=torch.uint8, device=DEV)
        a_ = L.DenseFwdArgs(M=M, N=N, nslab=1, zslab=Cd.data_ptr(), slab_stride=M * N,
                            bias=bd.data_ptr(), norm=L.NORM_BN_TRAIN, gamma=gamma.data_ptr(),
                            beta=beta.data_ptr(), running_mean=rm.data_ptr(),
                            running_var=rv.data_ptr(), momentum=0.05, eps=1e-5,
                            save_mean=sm.data_ptr(), save_invstd=si.data_ptr(), act=L.ACT["relu"],
                            drop_p=0.15, seed=5, step_ctr=None, stream_id=3, keep_in=None,
                            keep_out=keep.data_ptr(), xhat=xhat.data_ptr(), out=out.data_ptr())
        if fn == "pkc_dense_fwd":
            w2 = torch.zeros_like(work)
            L.call(fn, C.byref(a_), L.ptr(w2), _s())
        else:
            L.call(fn, C.byref(a_), L.ptr(work), rows, _s())
        outs.append((out.cpu(), xhat.cpu(), keep.cpu(), rm.cpu(), rv.cpu(), sm.cpu(), si.cpu()))
    (o0, x0, k0, rm0, rv0, sm0, si0), (o1, x1, k1, rm1, rv1, sm1, si1) = outs
    assert torch.equal(k0, k1)                   # same dropout bits
    torch.testing.assert_close(x1, x0, rtol=1e-4, atol=2e-5)
    torch.testing.assert_close(o1, o0, rtol=1e-4, atol=2e-5)
    for u, v in ((rm1, rm0), (rv1, rv0), (sm1, sm0), (si1, si0)):
        torch.testing.assert_close(u, v, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("R,Cc,P,ph,pw", [(2048, 512, 16, 8, 8), (512, 440, 20, 8, 8),
                                          (64, 48, 32, 8, 8), (96, 64, 12, 4, 4)])
def test_pattern_mask_matches_oracle(L, R, Cc, P, ph, pw):
    """pkc_pattern_mask (sparsity.py:1112-1146; the 8 x 8 register form and the generic kernel)
    against oracle.masks.apply_patterns, exactly: random tiles, tiles of equal values (every pattern
    of the same nnz ties: the mask sums the tied patterns) and all-zero tiles (every pattern ties)."""
    from oracle.masks import apply_patterns
    from pkc._lib import call, ptr
    g = torch.Generator().manual_seed(R + Cc + P)
    W = torch.randn(R, Cc, generator=g)
    W[:ph, :4 * pw] = 0.5                        # equal-valued tiles
    W[ph:2 * ph, :2 * pw] = 0.0                  # zero tiles
    pat = (torch.rand(P, ph, pw, generator=g) < 0.25).float()
    pat[:, 0, 0] = 1.0                           # every pattern nonempty
    pat[1] = pat[0]                              # two identical patterns: always tied
    Wd, pd = W.to(DEV), pat.to(DEV)
    out = torch.full((R, Cc), -1.0, device=DEV)
    call("pkc_pattern_mask", ptr(Wd), R, Cc, ptr(pd), P, ph, pw, ptr(out), _s())
    torch.cuda.synchronize()
    ref = apply_patterns(W.numpy(), pat.numpy())
    got = out.cpu().numpy()
    assert np.array_equal(got, ref), "%d of %d mask values differ" % (int((got != ref).sum()), got.size)
    assert got.max() >= 2.0                      # ties present
