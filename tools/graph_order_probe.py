"""When does a replayed HIP graph's second stream start, launched from idle?

Captures graphs of 1-thread stamp launches (scgib_stamp: the device wall
clock into a slot) on the capture stream ("main") and one forked stream
("side"), in several shapes, and prints, for a replay from idle (after a
synchronize) and for a steady replay (host ahead), when each chain's first
and last stamp ran.  The bench's first timed step showed the side stream's
forward chain starting ~170 us late (bench.py SCGIB_STAMPS_FIRST=1).

    python tools/graph_order_probe.py
"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("s-cgib_amd")
ops, _lib = pkg.ops, pkg._lib


def build(shape, buf, n_main, n_side, side_first, tail_main):
    """shape: labels list filled with (slot, label); returns the graph."""
    main = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    labels = []

    def st(label):
        labels.append(label)
        _lib.call("scgib_stamp", ops._p(buf), len(labels) - 1, ops._stream())

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        st("root[main]")
        side.wait_stream(torch.cuda.current_stream())

        def side_chain():
            with torch.cuda.stream(side):
                for i in range(n_side):
                    st(f"side.{i}")

        def main_chain():
            for i in range(n_main):
                st(f"main.{i}")

        if side_first:
            side_chain()
            main_chain()
        else:
            main_chain()
            side_chain()
        torch.cuda.current_stream().wait_stream(side)
        for i in range(tail_main):
            st(f"tail.{i}")
    shape[:] = labels
    return g


def report(tag, buf, labels):
    t = buf[:len(labels)].cpu().tolist()
    t0 = min(t)
    us = {lab: (v - t0) / 100.0 for lab, v in zip(labels, t)}

    def span(prefix):
        v = [u for lab, u in us.items() if lab.startswith(prefix)]
        return (min(v), max(v)) if v else (float("nan"), float("nan"))
    m, s, tl = span("main."), span("side."), span("tail.")
    print(f"  {tag:6s} main {m[0]:7.1f}..{m[1]:7.1f}  side {s[0]:7.1f}..{s[1]:7.1f}  "
          f"tail {tl[0]:7.1f}..{tl[1]:7.1f} us")


def main():
    torch.cuda.init()
    dev = torch.device("cuda", 0)
    buf = torch.zeros(1024, dtype=torch.int64, device=dev)
    shapes = [  # (n_main, n_side, side_first, tail_main)
        (60, 20, True, 0), (60, 20, False, 0), (20, 60, True, 0), (20, 60, False, 0),
        (20, 20, True, 60), (20, 20, False, 60), (40, 40, True, 0),
    ]
    for n_main, n_side, side_first, tail in shapes:
        labels = []
        g = build(labels, buf, n_main, n_side, side_first, tail)
        print(f"main {n_main} side {n_side} side captured first {side_first} main tail {tail}:")
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        buf.zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        report("idle", buf, labels)
        for _ in range(8):
            g.replay()
        torch.cuda.synchronize()
        report("steady", buf, labels)
        del g
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
