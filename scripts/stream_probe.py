"""Do two independent kernel chains captured on two streams of one hipGraph run concurrently on
MI355X?  (Decides whether the backward's dW / optimizer launches can be moved off the critical
dX -> BatchNorm-backward chain.)  Usage: python scripts/stream_probe.py"""
import torch


def chain(x, n):
    for _ in range(n):
        x.mul_(1.0001).add_(1e-7)


def main():
    dev = "cuda"
    a = torch.zeros(1 << 22, device=dev)      # 16 MB: ~5 us per kernel
    b = torch.zeros(1 << 22, device=dev)
    n = 20
    s0 = torch.cuda.Stream()
    s1 = torch.cuda.Stream()
    res = {}
    for mode in ("serial", "forked"):
        g = torch.cuda.CUDAGraph()
        s0.wait_stream(torch.cuda.current_stream())
        with torch.cuda.graph(g, stream=s0):
            if mode == "serial":
                chain(a, n)
                chain(b, n)
            else:
                s1.wait_stream(s0)
                chain(a, n)
                with torch.cuda.stream(s1):
                    chain(b, n)
                s0.wait_stream(s1)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(5):
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e3)
        res[mode] = best
    # single chain for reference
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s0):
        chain(a, n)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    res["one_chain"] = e0.elapsed_time(e1) * 1e3
    print({k: round(v, 1) for k, v in res.items()}, "us for", 2 * n, "kernels per chain")


if __name__ == "__main__":
    main()
