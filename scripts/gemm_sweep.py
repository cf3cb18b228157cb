"""Per-launch time of the bf16 forward matmul X W^T (N = K = 1024) over M around one 128x128 tile
per CU (256 tiles at M = 4096): where the time steps shows how many tiles run at once.
Usage: python scripts/gemm_sweep.py   (SWEEP_M=4096: that shape only)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pytorch-kaldi-cgs_amd"))

import torch  # noqa: E402

from pkc import _lib as L  # noqa: E402


def main():
    N = K = 1024
    print("CUs", torch.cuda.get_device_properties(0).multi_processor_count, flush=True)
    ms = (1024, 2048, 3072, 3584, 3840, 3968, 4096, 4224, 4352, 4608, 5120, 6144, 8192)
    if os.environ.get("SWEEP_M"):      # one shape (PMC passes)
        ms = (int(os.environ["SWEEP_M"]),)
    for M in ms:
        A = torch.randn(M, K, device="cuda").bfloat16()
        B = torch.randn(N, K, device="cuda").bfloat16()
        C = torch.empty(M, N, device="cuda")
        def args():   # on the stream current at the call (the capture stream inside the graph)
            return (L.PREC_BF16IN, 1, 1, M, N, K, L.ptr(A), K, L.ptr(B), K, L.ptr(C), N, 1, M * N,
                    L.C.c_void_p(torch.cuda.current_stream().cuda_stream))
        for _ in range(3):
            L.call("pkc_gemm", *args())
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(20):
                L.call("pkc_gemm", *args())
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(5):
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e3 / 20)
        tiles = -(-M // 128) * (N // 128)
        print("M %5d tiles %4d  %.2f us  %.1f TF/s" % (M, tiles, best, 2.0 * M * N * K / best / 1e6),
              flush=True)


if __name__ == "__main__":
    main()
