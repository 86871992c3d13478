"""Probe which stream fork/join patterns survive HIP-graph capture of a
backward pass.  Each case runs in its own subprocess (a failed capture can
segfault):  python tools/capture_probe.py  ->  one line per case."""
import subprocess
import sys

import torch

CASES = ["bwd_fork_join", "bwd_fork_join_2streams", "bwd_fork_join_nested", "fwd_fork_join",
         "fwd_nested", "bwd_flat2", "bwd_seq2", "bwd_nested_nokernel", "bwd_nested_clone",
         "bwd_nested_record", "bwd_nested_status", "bwd_flat_ret_side"]


def run_case(name):
    import faulthandler
    faulthandler.enable()  # a segfault prints the Python frame it happened in
    dev = torch.device("cuda", 0)
    aux = torch.cuda.Stream(dev)
    side = torch.cuda.Stream(dev)

    def fork_join(x):
        cur = torch.cuda.current_stream()
        aux.wait_stream(cur)
        with torch.cuda.stream(aux):
            y = x * 2.0
        cur.wait_stream(aux)
        return y

    class F(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            if name == "fwd_fork_join":
                return fork_join(x)
            if name == "fwd_nested":
                cur = torch.cuda.current_stream()
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    a = fork_join(x)
                cur.wait_stream(side)
                return a
            return x * 3.0

        @staticmethod
        def backward(ctx, g):
            if name == "bwd_fork_join":
                return fork_join(g)
            if name == "bwd_fork_join_2streams":
                cur = torch.cuda.current_stream()
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    a = fork_join(g)
                b = fork_join(g)
                cur.wait_stream(side)
                return a + b
            if name == "bwd_fork_join_nested":
                cur = torch.cuda.current_stream()
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    a = fork_join(g)
                cur.wait_stream(side)
                return a
            if name == "bwd_flat2":
                cur = torch.cuda.current_stream()
                side.wait_stream(cur)
                aux.wait_stream(cur)
                with torch.cuda.stream(side):
                    a = g * 2.0
                with torch.cuda.stream(aux):
                    b = g * 5.0
                cur.wait_stream(side)
                cur.wait_stream(aux)
                return a + b
            if name == "bwd_seq2":
                cur = torch.cuda.current_stream()
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    a = g * 2.0
                cur.wait_stream(side)
                return fork_join(a)
            if name in ("bwd_nested_clone", "bwd_nested_record", "bwd_nested_status"):
                # the nested case with the returned gradient re-homed on the
                # current stream (clone) or its side-stream block recorded on it,
                # and a probe of the capture status seen inside the nested fork
                cur = torch.cuda.current_stream()
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    aux.wait_stream(side)
                    with torch.cuda.stream(aux):
                        if name == "bwd_nested_status":
                            print("capturing on nested aux:",
                                  torch.cuda.is_current_stream_capturing(), flush=True)
                        y = g * 2.0
                    side.wait_stream(aux)
                cur.wait_stream(side)
                if name == "bwd_nested_record":
                    y.record_stream(cur)
                    return y
                return y.clone()
            if name == "bwd_flat_ret_side":  # flat fork, side-allocated result returned
                cur = torch.cuda.current_stream()
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    a = g * 2.0
                cur.wait_stream(side)
                return a
            if name == "bwd_nested_nokernel":
                cur = torch.cuda.current_stream()
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    aux.wait_stream(side)
                    with torch.cuda.stream(aux):
                        b = g * 5.0
                    side.wait_stream(aux)
                cur.wait_stream(side)
                return b
            return g * 3.0

    w = torch.randn(1024, device=dev, requires_grad=True)

    def body():
        loss = F.apply(w).sum()
        loss.backward()
        return loss

    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    w.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    print("captured", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print(name, "ok", float(w.grad.sum()))


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run_case(sys.argv[1])
    else:
        for c in CASES:
            r = subprocess.run([sys.executable, __file__, c], capture_output=True, text=True,
                               timeout=120)
            out = " | ".join(r.stdout.strip().splitlines()[-3:])
            err = " | ".join(ln.strip() for ln in r.stderr.strip().splitlines()[-8:])
            print(f"{c}: rc={r.returncode} {out} {err[:900] if r.returncode else ''}", flush=True)
