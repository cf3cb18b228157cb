"""Phase breakdown of the fused B = 128 layer kernel pkc_dense_gemm_fwd (measurement only).

Runs the kernel at the C2 layer shape on the phase-trace build (pkc/libpkc_trace.so, built with
`python pytorch-kaldi-cgs_amd/pkc/_build.py --trace`; pkc_fused.hip PKC_FTR stamps the shader clock
at its phase boundaries after draining the workgroup's memory counters) and prints the median
duration of every phase over the workgroups of the last launch.  Usage:
PKC_LIB=pytorch-kaldi-cgs_amd/pkc/libpkc_trace.so python scripts/trace_fused.py [K]"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
sys.path.insert(0, os.path.join(ROOT, "pytorch-kaldi-cgs_amd"))

PHASES = ["strip product (operand DMA + MFMA)", "partial-strip reduction (LDS)",
          "BatchNorm column statistics", "epilogue + stores"]


def main():
    assert "libpkc_trace" in os.environ.get("PKC_LIB", ""), "set PKC_LIB to the trace build"
    import torch
    import fused_probe as FP
    from pkc import _lib as L
    from pkc._lib import call, ptr
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    M, N = 128, 1024
    X = torch.randn(M, K, device="cuda").bfloat16()
    W = torch.randn(N, K, device="cuda").bfloat16()
    bufs = dict(S=1, slab=torch.zeros(1, M, N, device="cuda"), b=torch.zeros(N, device="cuda"),
                g=torch.ones(N, device="cuda"), be=torch.zeros(N, device="cuda"),
                rm=torch.zeros(N, device="cuda"), rv=torch.ones(N, device="cuda"),
                sm=torch.zeros(N, device="cuda"), si=torch.zeros(N, device="cuda"),
                ctr=torch.zeros(2, dtype=torch.int64, device="cuda"),
                keep=torch.zeros(M, N, dtype=torch.uint8, device="cuda"),
                xh=torch.zeros(M, N, device="cuda"),
                oh=torch.zeros(M, N, dtype=torch.bfloat16, device="cuda"))
    a = FP.args(M, N, bufs)
    for _ in range(20):
        call("pkc_dense_gemm_fwd", L.PREC_BF16IN, ptr(X), K, ptr(W), K, K, C.byref(a),
             C.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    n = 4096 * 8
    buf = (C.c_ulonglong * n)()
    assert L.lib().pkc_trace_read_fused(buf, n) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8).astype(np.int64)[:N // 16]
    cyc = np.diff(t[:, 1:6], axis=1)
    real_ns = (t[:, 7] - t[:, 0]) * 10.0
    clk = float(np.median((t[:, 5] - t[:, 1]) / np.maximum(real_ns, 1)))
    out = {"M": M, "N": N, "K": K, "workgroups": int(len(t)), "clock_ghz_median": round(clk, 3),
           "launch_span_ns": float((t[:, 7].max() - t[:, 0].min()) * 10.0),
           "workgroup_ns_median": float(np.median(real_ns)),
           "start_skew_ns": float((t[:, 0].max() - t[:, 0].min()) * 10.0),
           "entry_to_parameters_ns_median": None,
           "phases": {PHASES[i]: {"ns_median": round(float(np.median(cyc[:, i])) / clk, 1),
                                  "ns_max": round(float(cyc[:, i].max()) / clk, 1)}
                      for i in range(4)}}
    # entry (real-time) -> parameters loaded: from the real-time span minus the shader-clock phases
    out["entry_to_parameters_ns_median"] = round(float(np.median(
        real_ns - (t[:, 5] - t[:, 1]) / clk)), 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
