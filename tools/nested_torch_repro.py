"""Narrow the nested-fork capture crash to the torch layer that causes it.

tools/nested_capture_repro.hip shows plain HIP capture handles a nested fork
(origin -> side -> aux -> side -> origin), global capture mode, events
destroyed mid-capture included.  tools/capture_probe.py shows torch.cuda.graph
crashing in capture_end for every nested case.  These variants run the same
nested fork with plain torch streams (no autograd), each in its own process:

  plain          y = x * 3 allocated on the nested stream during capture
  prealloc       the same op into a tensor allocated before the capture
  flat_alloc     allocation on a one-level fork (control)
  events_kept    nested, explicit Events kept alive until after capture_end
  nested_noop    nested fork/join with no work and no allocation on aux

python tools/nested_torch_repro.py  ->  one line per variant (rc, last output)
"""
import subprocess
import sys

import torch

VARIANTS = ["plain", "prealloc", "flat_alloc", "events_kept", "nested_noop"]


def run(name):
    import faulthandler
    faulthandler.enable()
    dev = torch.device("cuda", 0)
    side, aux = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    x = torch.randn(4096, device=dev)
    pre = torch.empty_like(x)
    keep = []

    def wait(dst, src):
        if name == "events_kept":
            e = torch.cuda.Event()
            e.record(src)
            dst.wait_event(e)
            keep.append(e)
        else:
            dst.wait_stream(src)

    def body():
        cur = torch.cuda.current_stream()
        a = x * 2.0
        wait(side, cur)
        with torch.cuda.stream(side):
            if name == "flat_alloc":
                y = a * 3.0
            else:
                wait(aux, side)
                with torch.cuda.stream(aux):
                    if name == "prealloc":
                        torch.mul(a, 3.0, out=pre)
                        y = pre
                    elif name == "nested_noop":
                        y = a
                    else:
                        y = a * 3.0
                wait(side, aux)
        wait(cur, side)
        return y + 1.0

    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = body()
    print("captured", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print(name, "ok", float(out.sum()), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
    else:
        for v in VARIANTS:
            r = subprocess.run([sys.executable, __file__, v], capture_output=True, text=True,
                               timeout=120)
            out = " | ".join(r.stdout.strip().splitlines()[-2:])
            err = " | ".join(ln.strip() for ln in r.stderr.strip().splitlines()[-6:])
            print(f"{v}: rc={r.returncode} {out} {err[:600] if r.returncode else ''}", flush=True)
