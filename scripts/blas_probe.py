"""Probe: the vendor library's (hipBLASLt through torch.matmul) bf16 GEMM time at the B = 4096 MLP
shapes, graph-replayed (20 matmuls per graph) so host dispatch does not count — a yardstick for
the hand-written 128x128 / LDS-DMA bodies (pkc_gemm).  Usage: python scripts/blas_probe.py"""
import torch


def t(f, n=20, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            f()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            f()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / (reps * n)


for (M, N, K, lab) in [(4096, 1024, 1024, "fwd"), (4096, 1024, 440, "fwd440"),
                       (4096, 1976, 1024, "heads fwd"), (1024, 1024, 4096, "dW"),
                       (4096, 1024, 1976, "heads dX"), (1976, 1024, 4096, "heads dW"),
                       (128, 1024, 1024, "b128 fwd"), (8192, 8192, 8192, "sq8k")]:
    A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    B = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    n = 2 if M == 8192 else 20
    us = t(lambda: torch.matmul(A, B.t(), out=C), n=n)
    print("%-10s %5dx%5dx%5d  %8.2f us %7.1f TF/s" % (lab, M, N, K, us, 2 * M * N * K / us / 1e6),
          flush=True)
