"""Time the GIN-layer GEMM shapes under hipBLASLt vs rocBLAS (torch backends)."""
import torch

dev = torch.device("cuda", 0)


def bench(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for lib in ("cublaslt", "cublas"):
    torch.backends.cuda.preferred_blas_library(lib)
    for n in (9216, 27904):
        for din in (32, 64, 128):
            x = torch.randn(n, din, device=dev)
            dy = torch.randn(n, 64, device=dev)
            w = torch.randn(64, din, device=dev)
            t_fwd = bench(lambda: torch.nn.functional.linear(x, w))
            t_dw = bench(lambda: dy.t().mm(x))
            t_dx = bench(lambda: dy.mm(w))
            print(f"{lib:9s} n={n:6d} din={din:3d}  fwd {t_fwd:7.2f}us  dW {t_dw:7.2f}us  dX {t_dx:7.2f}us",
                  flush=True)
