"""Diagnostics for the two-lane replay (ops.SplitGraph): the bench's pretrain
step built twice from the same state — whole / split, whole / whole or
split / split (argv[1]) — replayed in lock-step with the same explicit noise;
after every replay the losses, parameters, Adam state, BN buffers and the
static batch / ego buffers are compared and the first differences printed.
Usage: python tools/split_diag.py whole|split|whole-split|whole-whole|split-split [B] [K]
(SPLIT_DIAG_OUT=dir: the first model's states saved there for a cross-process compare)."""
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def state(model, opt, static):
    out = {n: p.detach().clone() for n, p in model.named_parameters()}
    out.update({"buf." + n: b.detach().clone() for n, b in model.named_buffers()})
    for n, p in model.named_parameters():
        for k, v in (opt.state.get(p) or {}).items():
            if torch.is_tensor(v):
                out[f"opt.{n}.{k}"] = v.detach().clone()
    for k, v in vars(static).items():
        if torch.is_tensor(v):
            out["static." + k] = v.detach().clone()
    return out


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "whole-split"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    pkg = importlib.import_module("s-cgib_amd")
    import bench
    from test_gpu_trajectory import _pretrain_model
    dev = torch.device("cuda", 0)
    k, POOL = 1, 3
    F_in = pkg.synth.WORKLOADS["qm9"][2]
    hosts = [pkg.graph.collate_pyg(pkg.synth.molecules(B, "qm9", seed=30 + i))[0]
             for i in range(POOL)]
    n_cap = pkg.graph.StaticBatch.capacities(hosts, k, slack=1.02)[0]
    gen = torch.Generator().manual_seed(77)
    noise = [(torch.rand(n_cap, generator=gen), torch.rand(n_cap, 64, generator=gen))
             for _ in range(K)]
    runs = []
    for split in [m == "split" for m in mode.split("-")]:
        model = _pretrain_model(pkg, F_in, k, B, dev)
        opt = pkg.optim.Adam(model.parameters(), lr=1e-4, weight_decay=5e-5)
        s_ug = torch.zeros(n_cap, device=dev)
        s_uf = torch.zeros(n_cap, 64, device=dev)
        rs = bench.build_replay_step(model, opt, hosts, k, B, dev, prefetch=True,
                                     noise=(s_ug, s_uf), split=split)
        print(mode, "split" if rs.split is not None else "whole",
              rs.split.info if rs.split is not None else rs.graph_nodes, flush=True)
        runs.append((model, opt, rs, s_ug, s_uf))
    out_dir = os.environ.get("SPLIT_DIAG_OUT")
    if out_dir:  # the first model's state after the build and after every replay
        os.makedirs(out_dir, exist_ok=True)
        torch.cuda.synchronize()
        torch.save({k: v.cpu() for k, v in state(runs[0][0], runs[0][1], runs[0][2].static).items()},
                   os.path.join(out_dir, f"{mode}_built.pt"))
    if len(runs) == 2:
        torch.cuda.synchronize()
        sa = state(runs[0][0], runs[0][1], runs[0][2].static)
        sb = state(runs[1][0], runs[1][1], runs[1][2].static)
        bad = [n for n in sa if not torch.equal(sa[n], sb[n])]
        print(f"after build: {len(bad)} differing tensors: {bad[:12]}", flush=True)
    for j in range(K):
        st = []
        for model, opt, rs, s_ug, s_uf in runs:
            if os.environ.get("SPLIT_DIAG_PAD0"):  # noise on the batch's rows only, pad rows 0
                n = hosts[(int(rs.pool["cursor"][0])) % POOL].num_nodes()
                s_ug.zero_()
                s_uf.zero_()
                s_ug[:n].copy_(noise[j][0][:n])
                s_uf[:n].copy_(noise[j][1][:n])
            else:
                s_ug.copy_(noise[j][0])
                s_uf.copy_(noise[j][1])
            torch.cuda.synchronize()
            words = {k: pkg.ops._xq_words(dev, k).tolist() for k in ("pair_fwd", "pair_bwd")}
            kl, rec, con = rs.step(j)
            torch.cuda.synchronize()
            print(f"  replay {j} {'split' if rs.split is not None else 'whole'}: xq words before "
                  f"{words} after {[pkg.ops._xq_words(dev, k).tolist() for k in ('pair_fwd', 'pair_bwd')]}",
                  flush=True)
            st.append((torch.stack([kl, rec, con]).clone(), state(model, opt, rs.static)))
        if out_dir:
            torch.save({k: v.cpu() for k, v in st[0][1].items()},
                       os.path.join(out_dir, f"{mode}_r{j}.pt"))
        if len(st) < 2:
            print(f"replay {j}: losses {st[0][0].tolist()}", flush=True)
            continue
        (la, sa), (lb, sb) = st
        bad = [n for n in sa if not torch.equal(sa[n], sb[n])]
        worst = sorted(((float((sa[n].double() - sb[n].double()).abs().max()) /
                         max(float(sb[n].double().abs().max()), 1e-30), n) for n in bad
                        if sa[n].is_floating_point()), reverse=True)[:5]
        print(f"replay {j}: losses equal {torch.equal(la, lb)} {la.tolist()} {lb.tolist()}; "
              f"{len(bad)} differing tensors: {bad[:8]}; worst rel {worst}", flush=True)
    print("timeouts", pkg.ops.xq_timeouts(dev))


if __name__ == "__main__":
    main()
