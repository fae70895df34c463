#!/usr/bin/env python
"""Per-kernel cost floor of a graph-replayed chain of dependent tiny kernels on this GPU (what a
launch costs when its work is negligible), and of two such chains on two forked streams."""
import torch


def chain(n, x):
    for _ in range(n):
        x.add_(1.0)


def main():
    dev = "cuda"
    x = torch.zeros(64, device=dev)
    y = torch.zeros(64, device=dev)
    s = torch.cuda.Stream()
    s2 = torch.cuda.Stream()
    n = 1000
    with torch.cuda.stream(s):
        chain(10, x)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        chain(n, x)
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2, stream=s):
        ev = torch.cuda.Event()
        ev.record(s)
        s2.wait_event(ev)
        chain(n, x)
        with torch.cuda.stream(s2):
            chain(n, y)
        ev2 = torch.cuda.Event()
        ev2.record(s2)
        s.wait_event(ev2)
    for name, gr, k in (("1 stream", g, n), ("2 streams", g2, 2 * n)):
        for _ in range(3):
            gr.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f"{name}: {k} kernels in {ms:.3f} ms per replay -> {ms * 1000 / n:.2f} us per kernel of one chain",
              flush=True)


if __name__ == "__main__":
    main()
