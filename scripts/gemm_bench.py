"""Large-M matmul throughput (TFLOP/s) of pkc_gemm at the sequence models' projection shapes and
the B = 4096 MLP, in every orientation the engine uses.  Run twice (PKC_GEMM_BIG=0 / 1) for the
64x64 vs 128x128 tile A/B.  Usage: python scripts/gemm_bench.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pytorch-kaldi-cgs_amd"))

import torch  # noqa: E402

from pkc import _lib as L  # noqa: E402

SHAPES = [  # (label, prec, akc, bkc, M, N, K)
    ("c4 fwd W 5280x1024x2048 fp32", 0, 1, 1, 5280, 1024, 2048),
    ("c4 dX 5280x2048x1024 fp32", 0, 1, 0, 5280, 2048, 1024),
    ("c4 dW 1024x2048x5280 fp32", 0, 0, 0, 1024, 2048, 5280),
    ("c4 fwd W0 5280x1024x440 fp32", 0, 1, 1, 5280, 1024, 440),
    ("mlp B4096 fwd 4096x1024x1024 bf16", 2, 1, 1, 4096, 1024, 1024),
    ("mlp B4096 dX 4096x1024x1024 bf16", 2, 1, 0, 4096, 1024, 1024),
    ("mlp B4096 dW 1024x1024x4096 bf16", 2, 0, 0, 1024, 1024, 4096),
    ("mlp B4096 head 4096x1928x1024 bf16", 2, 1, 1, 4096, 1928, 1024),
    ("square 8192 bf16", 2, 1, 1, 8192, 8192, 8192),
    ("square 4096 fp32", 0, 1, 1, 4096, 4096, 4096),
]


def main():
    s = torch.cuda.current_stream()
    out = {"PKC_GEMM_BIG": os.environ.get("PKC_GEMM_BIG", "1")}
    for lab, prec, akc, bkc, M, N, K in SHAPES:
        dt = torch.bfloat16 if prec == 2 else torch.float32
        A = torch.randn(M, K, device="cuda").to(dt) if akc else torch.randn(K, M, device="cuda").to(dt)
        B = torch.randn(N, K, device="cuda").to(dt) if bkc else torch.randn(K, N, device="cuda").to(dt)
        splits = L.lib().pkc_gemm_pick_splits(M, N, K)
        C = torch.empty(splits, M, N, device="cuda")
        args = (prec, akc, bkc, M, N, K, L.ptr(A), A.shape[1], L.ptr(B), B.shape[1], L.ptr(C), N,
                splits, M * N, L.C.c_void_p(s.cuda_stream))
        for _ in range(3):
            L.call("pkc_gemm", *args)
        torch.cuda.synchronize()
        reps = max(3, int(2e12 / (2.0 * M * N * K)))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            L.call("pkc_gemm", *args)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000.0 / reps
        out[lab] = {"us": round(us, 2), "tflops": round(2.0 * M * N * K / us / 1e6, 1), "splits": splits}
        print(lab, out[lab], flush=True)
        if "mlp" not in lab:
            continue
        # the same matmul as a one-problem grouped launch (the engine's form at large batches:
        # 128x128 tiles from 32 tiles up), split-K 1 / 2 / 4
        for sp in (1, 2, 4):
            Cg = torch.empty(sp, M, N, device="cuda")
            pr = L.GemmProblem(a_kcontig=akc, b_kcontig=bkc, M=M, N=N, K=K, splits=sp, A=L.ptr(A),
                               lda=A.shape[1], B=L.ptr(B), ldb=B.shape[1], C=L.ptr(Cg), ldc=N,
                               slab_stride=M * N)
            arr = (L.GemmProblem * 1)(pr)
            for _ in range(3):
                L.call("pkc_gemm_grouped", prec, arr, 1, L.C.c_void_p(s.cuda_stream))
            e0.record()
            for _ in range(reps):
                L.call("pkc_gemm_grouped", prec, arr, 1, L.C.c_void_p(s.cuda_stream))
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1000.0 / reps
            key = lab + " grouped s%d" % sp
            out[key] = {"us": round(us, 2), "tflops": round(2.0 * M * N * K / us / 1e6, 1)}
            print(key, out[key], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
