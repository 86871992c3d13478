"""BASELINE.json configs[4] on the device: the ogbg-molhiv fine-tune step from
pre_training_v1_GIN_64_5_1.pt (bench.py --finetune molhiv).

One step = the batch load + on-device ego-nets (the reference extracts them
in its data loader, exp_molhiv.py) + Mainmodel_finetuning.forward in train
mode (models.py:501-520: transfer_d, the pretrained Mainmodel_continue's
extract_features with the reference's freezing quirk, MLP, Set2Set, predict,
sigmoid) + BCE loss (models.py:522-523) + backward + Adam(lr 1e-3, weight
decay 1e-5) over the model's parameters (exp_molhiv.py:160,
train_molhiv.py:107-152), captured as ONE HIP graph in capacity mode and
replayed over a pool of resident synthetic molhiv-shaped batches of B = 32
(the reference's default batch size for this driver; --batch to change).

The pretrained weights are the shipped checkpoint's 544 tensors as read
weights-only by s-cgib_amd/refckpt.py into tests/golden/ (no pickle is loaded
here); the fine-tune head's own weights are seeded random; targets are seeded
random {0, 1} labels per batch.  The CPU baseline is the oracle's fine-tune
step (oracle/scgib_ref.py finetune_forward + backward + Adam, ego-nets
pre-extracted as the reference's loader does) on a bounded sample.
"""
from __future__ import annotations

import json
import os
import statistics
import time
from types import SimpleNamespace

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.abspath(__file__))
CKPT = os.path.join(ROOT, "tests", "golden", "ckpt_pre_training_v1_GIN_64_5_1.npz")


def load_pretrained(pkg, args):
    """The shipped checkpoint's module chain (4 levels, 544 tensors) from the
    committed weights-only fixture."""
    with np.load(CKPT, allow_pickle=False) as d:
        levels = [(s.split(":")[0], int(s.split(":")[1])) for s in d["levels"].tolist()]
        cfg = {k[4:]: (d[k].item() if d[k].dtype.kind in "iuf" else str(d[k]))
               for k in d.files if k.startswith("cfg_")}
        sd = {k[3:]: torch.tensor(d[k]) for k in d.files if k.startswith("sd/")}
    return pkg.models.model_from_state(levels, cfg, sd, args), levels, cfg


def make_finetune_model(pkg, F_in, B, dev, seed=0, dataset="ogbg-molhiv", num_classes=1):
    """Mainmodel_finetuning around the shipped checkpoint's chain: molhiv's
    BCE head (exp_molhiv.py, num_classes 1) by default; Mutagenicity's CE
    head with dataset="Mutagenicity", num_classes=2 (exp_tudataset.py)."""
    args = SimpleNamespace(recons_type="adj", useAtt=1, readout_f="sum", d_transfer=32,
                           batch_size=B, gin_layers=5, task="graph_classification",
                           dataset=dataset, device=dev)
    torch.manual_seed(seed)
    pre, levels, cfg = load_pretrained(pkg, args)
    k = int(cfg["k_transition"])
    ft = pkg.models.Mainmodel_finetuning(args, F_in, 64, 4, 4, k, num_classes, pre, "GIN")
    return ft.to(dev).train(), k


def oracle_params(pkg, ft):
    """fp32 CPU leaves of the fine-tune model for the oracle: only the
    parameters the step trains require grad (the freezing quirk)."""
    from oracle import scgib_ref as R
    trainable = {n for n, p in ft.named_parameters() if p.requires_grad}
    p = R.make_params({k: v.detach().cpu().numpy() for k, v in ft.state_dict().items()},
                      requires_grad=False)
    for k, v in p.items():
        if k in trainable:
            v.requires_grad_(True)
    return p


def cpu_baseline(bench, ft, host_batches, targets, seconds):
    """The oracle's fine-tune step on this host's cores (torch's default
    thread count = the CPU share), bounded sample."""
    from oracle import egonet
    from oracle import scgib_ref as R
    p = oracle_params(bench.pkg, ft)
    opt = torch.optim.Adam([v for v in p.values() if v.requires_grad], lr=1e-3, weight_decay=1e-5)
    buffers = {k: v for k, v in p.items() if "running" in k or "num_batches" in k}
    k = int(ft.k_transition)
    times = []
    t_end = time.perf_counter() + seconds
    i = 0
    # BASELINE.md §2's protocol: 3 warm-up steps, then the median of >= 10
    while time.perf_counter() < t_end or i < bench.CPU_WARMUP + bench.CPU_MIN_STEPS:
        gh = host_batches[i % len(host_batches)]
        t0 = time.perf_counter()
        sizes, ecount, nodes, esrc, edst = egonet.egonets(gh.rowptr.numpy(), gh.col.numpy(), k)
        off = np.repeat(np.concatenate([[0], np.cumsum(sizes)[:-1]]), ecount)
        src, dst = gh.edges()
        batch = {"src": src, "dst": dst, "counts": torch.from_numpy(gh.batch_num_nodes_host())}
        ego = {"src": torch.from_numpy(esrc + off), "dst": torch.from_numpy(edst + off),
               "counts": torch.from_numpy(sizes)}
        x = F.normalize(gh.ndata["x"].float())
        n = x.shape[0]
        opt.zero_grad(set_to_none=True)
        scores = R.finetune_forward(p, batch, ego, x, x[torch.from_numpy(nodes)],
                                    torch.rand(n), torch.rand(n, 64), "ogbg-molhiv", buffers)
        loss = F.binary_cross_entropy(scores, targets[i % len(targets)].cpu())
        loss.backward()
        opt.step()
        if i >= bench.CPU_WARMUP:
            times.append(time.perf_counter() - t0)
        i += 1
    B = host_batches[0].batch_size
    ms = statistics.median(times) * 1e3
    return {"value": round(B / (ms * 1e-3), 1), "unit": "graphs/s", "ms_per_step": round(ms, 3),
            "steps": len(times), "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"median of {len(times)} oracle fine-tune steps (finetune_forward + BCE + "
                      f"backward + Adam, fp32, per-graph loops; ego-nets by oracle/egonet.py in "
                      f"the step) of B={B} molhiv-like molecules after {bench.CPU_WARMUP} "
                      f"warm-up, ~{seconds:.0f} s"}


def build_finetune_step(pkg, ft, opt, host, targets, k, B, dev, prefetch=True, noise=None,
                        warm=3, split=True, noise_prefetch=False):
    """The fine-tune step (train_molhiv.py:107-152: forward, BCE, backward,
    Adam) as ONE captured HIP graph in capacity mode over a resident pool of
    the host batches ``host`` and their ``targets`` ([B, 1] each): the pool's
    next batch, its target rows and the ego-nets the previous step built for
    it loaded inside the graph.  ``warm`` eager steps on a side stream first
    (allocator, Adam state).  ``noise`` = (u_gate [n_cap], u_feat [n_cap, 64])
    static device buffers the step reads instead of its own device draws
    (tests/test_gpu_trajectory.py).  ``split``: replay as two linear lanes
    (ops.SplitGraph) where the hand-off rule allows.  ``noise_prefetch``
    (noise None): the device noise one step ahead, as the pretrain bench
    (ops.NoisePrefetch) — off by default here: with the lower GIN layers
    frozen the fine-tune's backward core chain is the longer one, and the
    draw at its end measured 0.2876-0.2890 vs 0.2854-0.2855 ms per step
    (profiles/r06_noise/finetune_ab.txt).  Returns replay() (one step), the captured graph,
    the static scores and loss, the static batch, the device pool and its
    prefetches."""
    n_cap, e_cap, mgn, caps = pkg.graph.StaticBatch.capacities(host, k, slack=1.02)
    F_in = host[0].ndata["x"].shape[1]
    static = pkg.graph.StaticBatch(B, n_cap, e_cap, F_in, mgn, caps, dev, k=k)
    padded = []
    for gh in host:
        gx = pkg.graph.GraphBatch.from_edges(*[t.numpy() for t in gh.edges()], gh.num_nodes(), True,
                                             gh.batch_num_nodes_host())
        dict.__setitem__(gx.ndata, "x", F.normalize(gh.ndata["x"].float()))
        padded.append(static.pad(gx))
    pool = static.pool(padded)
    # the ego-nets one batch ahead, as the pretrain bench (graph.EgoPrefetch):
    # each step builds the next batch's on the encoder pair's idle queue during
    # the loss section, and the next batch load moves them in with the batch
    pf = None
    if prefetch:
        pf = pkg.graph.EgoPrefetch(static, pool)
        pf.prime()
    nf = None
    if noise is None and noise_prefetch:
        nf = pkg.ops.NoisePrefetch(static.graph, dev)
        nf.prime()
    # the targets walk their own resident pool in step with the batches: one
    # pool-copy launch per step (its own cursor, advanced like the batch's)
    tdev = [t.to(dev).contiguous() for t in targets]
    ttable = torch.tensor([t.data_ptr() for t in tdev], dtype=torch.int64, device=dev)
    tcursor = torch.zeros(2, dtype=torch.int32, device=dev)
    tg = torch.empty(B, 1, dtype=torch.float32, device=dev)
    one = torch.ones((), dtype=torch.float32, device=dev)  # d loss / d loss, resident (no fill per step)

    def body():
        static.load_next(pool, pf)
        pkg._lib.call("scgib_pool_copy", pkg.ops._p(ttable), len(tdev), pkg.ops._p(tcursor),
                      pkg.ops._p(tg), tg.numel() * 4, pkg.ops._stream())
        scores, *_ = ft(static.graph, static.x, None, None, 1, None, 2, dev, B, noise=noise)
        loss = ft.loss(scores, tg)
        torch.autograd.backward(loss, one)
        if pf is not None:
            pf.join()  # (no-op: the encoder pair's backward joined it)
        return scores.detach(), loss.detach()

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm-up: allocator, Adam state
        for _ in range(warm):
            opt.zero_grad(set_to_none=True)
            body()
            opt.step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    opt.zero_grad(set_to_none=True)
    if os.environ.get("SCGIB_STAMPS"):  # diagnostics: wall-clock stamps in the captured step
        pkg.ops.stamps_enable(dev, int(os.environ["SCGIB_STAMPS"]))
    graph = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(graph):
        scores, loss = body()
        opt.step()
    try:
        nodes = pkg.ops.graph_node_counts(graph)
    except Exception:  # noqa: BLE001 (diagnostic field only)
        nodes = None
    lanes = None
    if split and pkg.ops.xq_enabled():
        try:
            lanes = pkg.ops.SplitGraph(graph, dev)
        except pkg.ops.SplitUnsupported:
            lanes = None
    if lanes is None:
        graph.instantiate()
    if nodes is not None:
        nodes = dict(nodes, replay=(
            {k: lanes.info[k] for k in ("lane0_nodes", "lane1_nodes", "handoffs")}
            if lanes is not None else "whole graph"))
    # (`one` held for the captured backward, as bench.build_replay_step does)
    return SimpleNamespace(replay=lanes.replay if lanes is not None else graph.replay,
                           graph=graph, split=lanes, scores=scores, loss=loss, static=static,
                           pool=pool, padded=padded, prefetch=pf, noise_prefetch=nf,
                           targets=(tdev, ttable, tcursor, tg), graph_nodes=nodes, one=one)


FT_STAMPS_FILE = os.environ.get("SCGIB_FT_STAMPS_FILE",
                                os.path.join(ROOT, "profiles", "ft_stamps_current.json"))
# the main stream's stamps of one replayed fine-tune step (ops.stamp, level 1)
# in order: the phases between consecutive ones partition the step's
# critical path (the ego chain runs beside the first and fourth)
CRITICAL_PHASES = (("fwd.fork[main]", "fwd.joined[main]", "encoders_fwd (core chain + join)"),
                   ("fwd.joined[main]", "interaction_end", "interaction"),
                   ("interaction_end", "bwd.start[main]",
                    "head: MLP, Set2Set, predict, BCE and their backward"),
                   ("bwd.start[main]", "bwd.joined[main]", "encoders_bwd (both chains + join)"),
                   ("bwd.joined[main]", "adam_end", "adam"))


def critical_path(bench, ms_per_step):
    """finetune.critical_path_us: the replayed step's critical path by phase
    from the device wall-clock stamps of a stamped run of this same command
    (tools/gpu_round.sh, SCGIB_STAMPS=1 SCGIB_STAMPS_JSON=...); the stamps
    add launches, so the stamped run's own ms/step is reported beside it.
    None when the file is of another configuration."""
    st = bench._load_json(FT_STAMPS_FILE)
    if st.get("_config") != bench.RUN_CONFIG or not st.get("stamps"):
        return None
    t = {lab: us for lab, us in st["stamps"]}
    phases = {name: round(t[b] - t[a], 2) for a, b, name in CRITICAL_PHASES if a in t and b in t}
    first = t.get(CRITICAL_PHASES[0][0])
    last = t.get(CRITICAL_PHASES[-1][1])
    span = None if first is None or last is None else round(last - first, 2)
    return {"phases_us": phases, "stamped_span_us": span,
            "stamped_ms_per_step": st.get("ms_per_step"),
            "outside_span_us": (None if span is None else
                                round(ms_per_step * 1e3 - span, 2)),
            "stamps_file": os.path.relpath(FT_STAMPS_FILE, ROOT),
            "note": "device wall-clock stamps of the main stream in one replayed step of a "
                    "stamped run (level 1); outside_span = this run's ms/step minus the stamped "
                    "span: the batch load, the replay's head and the gap between replays"}


def run(bench, a, dev):
    """bench.py --finetune molhiv: returns the JSON line (dict)."""
    pkg = bench.pkg
    workload = "molhiv"
    F_in = pkg.synth.WORKLOADS[workload][2]
    B = a.batch if a.batch != 512 else 32  # (bench's pretrain default 512 -> the fine-tune's 32)
    ft, k = make_finetune_model(pkg, F_in, B, dev)
    gen = torch.Generator().manual_seed(7)
    host, padded_src = [], []
    for i in range(a.pool):
        gh, _ = pkg.graph.collate_pyg(pkg.synth.molecules(B, workload, seed=500 + i))
        host.append(gh)
    targets = [torch.randint(0, 2, (B, 1), generator=gen).float() for _ in range(a.pool)]
    bench.RUN_CONFIG = {"workload": "molhiv-finetune", "batch": B, "k": k}
    opt = pkg.optim.Adam(ft.parameters(), lr=1e-3, weight_decay=1e-5)
    fs = build_finetune_step(pkg, ft, opt, host, targets, k, B, dev,
                             prefetch=not a.no_ego_prefetch, split=not a.no_split)
    replay, static_loss, prefetch = fs.replay, fs.loss, fs.prefetch
    for _ in range(a.warmup):
        replay()
    bench.progress(f"fine-tune warm-up done; timing {a.steps} steps")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        replay()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if pkg.ops.xq_timeouts(dev) or pkg.ops.handoff_fault(dev):
        raise SystemExit("bench: a cross-queue hand-off wait timed out (ops.XQ_FLAGS)")
    pkg.ops.check_handoff(dev)
    if os.environ.get("SCGIB_STAMPS"):
        stamps = pkg.ops.stamps_read()
        for lab, us in stamps:
            bench.progress(f"stamp {us:9.2f} us  {lab}")
        if os.environ.get("SCGIB_STAMPS_JSON"):  # tools/gpu_round.sh: the critical-path file
            with open(os.environ["SCGIB_STAMPS_JSON"], "w") as fh:
                json.dump({"_config": bench.RUN_CONFIG, "level": int(os.environ["SCGIB_STAMPS"]),
                           "ms_per_step": round(elapsed / a.steps * 1e3, 4),
                           "stamps": [[lab, round(us, 2)] for lab, us in stamps]}, fh, indent=1)
        pkg.ops.stamps_enable(dev, 0)
        pkg.ops._STAMPS["buf"] = None
    final_loss = float(static_loss.item())
    # kernel timer: eager fine-tune steps on one stream, HIP events per launch
    kernels = {}
    if not a.no_kernel_timer:
        entries = [e for spec in bench.KERNELS.values() for e in spec["entries"]]
        steps_t = min(a.steps, 10)
        pkg.models.FORK_ENCODERS = False
        try:
            with bench.KernelTimer(*entries) as timer:
                for i in range(steps_t):
                    gh = host[i % len(host)]
                    g = gh.to(dev)
                    x = F.normalize(g.ndata["x"].float())
                    ft.zero_grad(set_to_none=True)
                    scores, *_ = ft(g, x, None, None, 1, None, 2, dev, B)
                    ft.loss(scores, targets[i % len(targets)].to(dev)).backward()
        finally:
            pkg.models.FORK_ENCODERS = True
        for name, spec in bench.KERNELS.items():
            r = timer.kernel_summary(spec, steps_t)
            if r is not None:
                kernels[name] = bench.roofline_entry(name, spec["desc"], r, spec["pmc"])
    dominant = max(kernels, key=lambda kk: kernels[kk]["per_step_us"]) if kernels else None
    cpu = None if a.no_cpu_baseline else cpu_baseline(bench, ft, host, targets, a.cpu_seconds / 2)
    n_nodes = statistics.mean(g.num_nodes() for g in host)
    return {
        "metric": "graphs/sec (ogbg-molhiv fine-tune step from pre_training_v1_GIN_64_5_1, "
                  "GIN-64x5) on 1 MI355X",
        "value": round(B * a.steps / elapsed, 1), "unit": "graphs/s", "n_gpus": 1,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (seeded molhiv-like molecules, F=9 OGB features, random {0,1} "
                "targets); pretrained weights: the shipped checkpoint's tensors (weights-only "
                "fixture), head weights seeded random",
        "config": {"workload": f"molhiv fine-tune step, batch {B}, k={k} (BASELINE.json "
                               "configs[4]), Mainmodel_finetuning + BCE + Adam(1e-3, wd 1e-5)",
                   "launch": "hip-graph replay (capacity mode)",
                   "ego_build": ("in the step, for the batch the next step loads "
                                 "(graph.EgoPrefetch)" if prefetch is not None
                                 else "at the head of the step (device k-hop builder)"),
                   "trainable": sum(p.numel() for p in ft.parameters() if p.requires_grad),
                   "nodes_per_batch": round(n_nodes, 1), "parallelism": "dp1",
                   "graph_nodes": fs.graph_nodes,
                   "host_enqueue_ms": round(t_enq / a.steps * 1e3, 4),
                   "final_loss": round(final_loss, 4)},
        "roofline": kernels.get(dominant),
        "roofline_kernels": kernels or None,
        "critical_path_us": critical_path(bench, elapsed / a.steps * 1e3),
        "cpu_baseline": cpu,
    }


def main_line(bench, a, dev):
    line = run(bench, a, dev)
    print(json.dumps(line), flush=True)
