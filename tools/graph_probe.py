"""Probe HIP-graph replay costs on this runtime (design input, not a test).

1. per-node cost of a captured chain of tiny kernels;
2. whether two captured branches (fork/join over a side stream) overlap,
   using spin kernels of known length.
"""
import time

import torch


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def capture(body):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        body()
    return g


def main():
    dev = torch.device("cuda", 0)
    x = torch.zeros(64, device=dev)
    side = torch.cuda.Stream()

    for n in (50, 200):
        def chain():
            for _ in range(n):
                x.add_(1.0)
        g = capture(chain)
        print(f"chain of {n} tiny kernels: graph {timed(g.replay) / n:.2f} us/node, "
              f"eager {timed(chain) / n:.2f} us/launch")

    cyc = 200_000  # spin length
    def one():
        torch.cuda._sleep(cyc)
    g1 = capture(one)
    t_one = timed(g1.replay)
    print(f"one spin kernel: {t_one:.1f} us")

    def serial():
        for _ in range(20):
            torch.cuda._sleep(cyc)
    def forked():
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        with torch.cuda.stream(side):
            for _ in range(10):
                torch.cuda._sleep(cyc)
        for _ in range(10):
            torch.cuda._sleep(cyc)
        main.wait_stream(side)
    gs, gf = capture(serial), capture(forked)
    print(f"20 spins serial: graph {timed(gs.replay):.0f} us, eager {timed(serial):.0f} us")
    print(f"2 x 10 spins forked: graph {timed(gf.replay):.0f} us, eager {timed(forked):.0f} us")

    def forked_interleaved():
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        for _ in range(10):
            with torch.cuda.stream(side):
                torch.cuda._sleep(cyc)
            torch.cuda._sleep(cyc)
        main.wait_stream(side)
    gi = capture(forked_interleaved)
    print(f"2 x 10 spins forked, interleaved issue: graph {timed(gi.replay):.0f} us, "
          f"eager {timed(forked_interleaved):.0f} us")


if __name__ == "__main__":
    main()
