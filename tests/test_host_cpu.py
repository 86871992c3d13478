"""CPU-only tests: C-ABI exports, ego-net oracle vs goldens, host ingest/collate.

No compute call touches the GPU here."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT, load_golden
from oracle import dgl_semantics as D
from oracle import egonet


# ---------------------------------------------------------------------------
def header_symbols():
    src = open(os.path.join(ROOT, "include", "scgib.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|int64_t|const char \*)\s*(scgib_\w+)\(", src,
                                 re.M)))


def test_library_exports_every_header_symbol(pkg):
    lib_mod = pkg._lib
    lib = ctypes.CDLL(lib_mod.LIB_PATH)  # loads without a GPU: nothing is launched
    syms = header_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(lib_mod.SIGNATURES), "ctypes signature table out of sync"
    loaded = lib_mod.load()
    assert loaded.scgib_abi_version() == lib_mod.ABI_VERSION
    assert loaded.scgib_strerror(-1).decode().startswith("invalid")


def test_argument_errors_do_not_launch(pkg):
    lib = pkg._lib.load()
    # negative / invalid sizes and null pointers are rejected before any launch
    assert lib.scgib_gin_aggregate(None, None, None, -1, 64, 1.0, None, None, None) == -1
    assert lib.scgib_gin_aggregate(None, None, None, 10, 63, 1.0, None, None, None) == -1
    assert lib.scgib_gin_aggregate(None, None, None, 0, 64, 1.0, None, None, None) == 0
    assert lib.scgib_segment_sum(None, None, 5, 64, None, None, None) == -1
    assert lib.scgib_egonet_count(None, None, None, 1, 10, 1, 1000, None, None, None, None,
                                  None, None) == -1
    assert lib.scgib_recon_fwd(None, None, None, 0, 0, None, None, None, None, None) == -1
    assert lib.scgib_gin_layer_fwd(None, 48, None, None, None, 10, 1.0, None, None, None, None,
                                   None, None, None, None, None, None) == -1
    assert lib.scgib_egonet_workspace_bytes(1000) >= 8
    assert lib.scgib_recon_partials_floats(9000) > 36 * 4096


# ---------------------------------------------------------------------------
def test_egonet_oracle_matches_reference_goldens():
    d = load_golden("ingest_egonet")
    checked = 0
    for i in range(int(d["num_mols"])):
        if not d[f"m{i}_kept"]:
            continue
        g = D.Graph(d[f"m{i}_src"], d[f"m{i}_dst"], int(d[f"m{i}_n"]))
        rp, col = D.csr_from_graph(g)
        for k in (1, 2, 3):
            s, e, nodes, es, ed = egonet.egonets(rp, col, k)
            np.testing.assert_array_equal(s, d[f"m{i}_k{k}_sizes"])
            np.testing.assert_array_equal(nodes, d[f"m{i}_k{k}_nodes"])
            np.testing.assert_array_equal(e, d[f"m{i}_k{k}_ecount"])
            np.testing.assert_array_equal(es, d[f"m{i}_k{k}_esrc"])
            np.testing.assert_array_equal(ed, d[f"m{i}_k{k}_edst"])
            checked += 1
    assert checked >= 30


def test_egonet_oracle_k1_size_identity(pkg):
    # k = 1 on a simple graph: |ball(v)| = 1 + deg(v)  =>  N_s = N + E
    mols = pkg.synth.molecules(64, "qm9", seed=5)
    g, _ = pkg.graph.collate_pyg(mols)
    s, e, *_ = egonet.egonets(g.rowptr.numpy(), g.col.numpy(), 1)
    assert s.sum() == g.num_nodes() + g.num_edges()


# ---------------------------------------------------------------------------
def test_ingest_matches_reference_load_dgl_fromPyG(pkg):
    """A1: graph + to_bidirected + the skip rule, against util.load_dgl_fromPyG."""
    d = load_golden("ingest_egonet")
    for i in range(int(d["num_mols"])):
        ei, x = d[f"m{i}_edge_index"], d[f"m{i}_x"]
        if not d[f"m{i}_kept"]:
            with pytest.raises(pkg.graph.GraphIngestError):
                pkg.graph.from_pyg(ei, x)
            continue
        g = pkg.graph.from_pyg(ei, x)
        assert g.num_nodes() == int(d[f"m{i}_n"])
        s, t = g.edges()
        np.testing.assert_array_equal(s.numpy(), d[f"m{i}_src"])
        np.testing.assert_array_equal(t.numpy(), d[f"m{i}_dst"])


def test_collate_equals_batch_of_singles(pkg):
    mols = pkg.synth.molecules(40, "pcqm4mv2", seed=3)
    bad = (np.array([[0, 1], [1, 0]]), np.zeros((3, 9), np.float32))  # trailing isolated atom
    mols.insert(7, bad)
    g, kept = pkg.graph.collate_pyg(mols)
    assert 7 not in kept and len(kept) == 40
    singles = [pkg.graph.from_pyg(*mols[i]) for i in kept]
    gb = pkg.graph.batch(singles)
    np.testing.assert_array_equal(g.rowptr.numpy(), gb.rowptr.numpy())
    np.testing.assert_array_equal(g.col.numpy(), gb.col.numpy())
    np.testing.assert_array_equal(g.graph_ptr.numpy(), gb.graph_ptr.numpy())
    np.testing.assert_array_equal(g.batch_num_nodes().numpy(), gb.batch_num_nodes().numpy())
    np.testing.assert_array_equal(g.batch_num_edges().numpy(), gb.batch_num_edges().numpy())
    assert torch.equal(g.ndata["x"], gb.ndata["x"])
    # DGL edge order of the batch: (src, dst) sorted
    s, t = g.edges()
    key = s.numpy() * g.num_nodes() + t.numpy()
    assert (np.diff(key) > 0).all()


def test_adj_to_dense_and_symmetry(pkg):
    g, _ = pkg.graph.collate_pyg(pkg.synth.molecules(5, "qm9", seed=1))
    a = g.adj().to_dense()
    assert torch.equal(a, a.t())
    assert int(a.sum()) == g.num_edges()


def test_ndata_rowcount_checked(pkg):
    g, _ = pkg.graph.collate_pyg(pkg.synth.molecules(3, "qm9", seed=1))
    with pytest.raises(pkg.graph.GraphIngestError):
        g.ndata["h"] = torch.zeros(g.num_nodes() + 1, 4)


def test_product_ops_refuse_cpu_tensors(pkg):
    g, _ = pkg.graph.collate_pyg(pkg.synth.molecules(3, "qm9", seed=1))
    with pytest.raises(pkg._lib.ScgibError):
        pkg.ops.gin_aggregate(torch.zeros(g.num_nodes(), 64), g)
    with pytest.raises(pkg._lib.ScgibError):
        pkg.graph.egonet_batch(g, 1)


@pytest.mark.parametrize("workload", ["qm9", "molpcba", "pcqm4mv2", "mutagenicity"])
def test_synthetic_shapes(pkg, workload):
    mols = pkg.synth.molecules(256, workload, seed=0)
    g, kept = pkg.graph.collate_pyg(mols)
    assert len(kept) == 256  # the generator never emits molecules the reference would skip
    mu = pkg.synth.WORKLOADS[workload][0]
    assert abs(g.num_nodes() / 256 - mu) < 0.15 * mu
    deg = np.diff(g.rowptr.numpy())
    assert deg.min() >= 1


def test_dgl_dropin_khop_and_ingest(pkg):
    """s-cgib_amd/dgl.py (the drop-in DGL surface) against the reference goldens:
    graph -> to_bidirected -> ndata['x'] (util.py:317-321) and khop_in_subgraph
    per node (exp_pretraining.py:269-272)."""
    dgl = pkg.dgl
    d = load_golden("ingest_egonet")
    for i in range(int(d["num_mols"])):
        ei, x = d[f"m{i}_edge_index"], d[f"m{i}_x"]
        try:
            g = dgl.to_bidirected(dgl.graph((torch.from_numpy(ei[0]), torch.from_numpy(ei[1]))))
            g.ndata["x"] = torch.from_numpy(x)
            kept = True
        except (pkg.graph.GraphIngestError, ValueError):
            kept = False
        assert kept == bool(d[f"m{i}_kept"]), i
        if not kept:
            continue
        s, t = g.edges()
        np.testing.assert_array_equal(s.numpy(), d[f"m{i}_src"])
        np.testing.assert_array_equal(t.numpy(), d[f"m{i}_dst"])
        for k in (1, 2):
            nodes, es, ed, sizes = [], [], [], []
            for v in range(g.num_nodes()):
                sg, _ = dgl.khop_in_subgraph(g, v, k)
                nodes.append(sg.ndata["_ID"].numpy())
                a, b = sg.edges()
                es.append(a.numpy())
                ed.append(b.numpy())
                sizes.append(sg.num_nodes())
                assert torch.equal(sg.ndata["x"], g.ndata["x"][sg.ndata["_ID"]])
            np.testing.assert_array_equal(np.array(sizes), d[f"m{i}_k{k}_sizes"])
            np.testing.assert_array_equal(np.concatenate(nodes), d[f"m{i}_k{k}_nodes"])
            np.testing.assert_array_equal(np.concatenate(es), d[f"m{i}_k{k}_esrc"])
            np.testing.assert_array_equal(np.concatenate(ed), d[f"m{i}_k{k}_edst"])


def _header_prototypes():
    """{name: [param kind]} from include/scgib.h; kind in P (pointer), I64, I32, F, D."""
    src = open(os.path.join(ROOT, "include", "scgib.h")).read()
    src = re.sub(r"/\*.*?\*/|//[^\n]*", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"(?:int|int32_t|int64_t|const char \*)\s*(scgib_\w+)\(([^)]*)\)\s*;", src):
        params = [p.strip() for p in m.group(2).split(",") if p.strip() not in ("", "void")]
        kinds = []
        for p in params:
            if "*" in p or p.startswith("scgib_stream_t"):
                kinds.append("P")
            elif p.startswith("int64_t"):
                kinds.append("I64")
            elif p.startswith("int32_t") or p.startswith("int "):
                kinds.append("I32")
            elif p.startswith("float"):
                kinds.append("F")
            elif p.startswith("double"):
                kinds.append("D")
            else:
                raise AssertionError(f"unparsed parameter {p!r} of {m.group(1)}")
        out[m.group(1)] = kinds
    return out


def test_ctypes_table_matches_header_prototypes(pkg):
    L = pkg._lib
    kind = {L._P: "P", L._I64: "I64", L._I32: "I32", L._F: "F", L._D: "D"}
    protos = _header_prototypes()
    assert set(protos) == set(L.SIGNATURES)
    for name, (_, argtypes) in L.SIGNATURES.items():
        assert [kind[t] for t in argtypes] == protos[name], name


def test_checkpoint_roundtrip_continue(pkg, tmp_path):
    """save_checkpoint / load_checkpoint of a nested Mainmodel_continue (weights
    only, nothing unpickled) and the fine-tune freezing quirk on top of it."""
    from types import SimpleNamespace
    args = SimpleNamespace(recons_type="adj", useAtt=1, readout_f="sum", d_transfer=32,
                           batch_size=8, gin_layers=4, task="graph_classification",
                           dataset="Mutagenicity")
    inner = pkg.models.Mainmodel(args, 14, 64, 4, 4, 1, "GIN")
    pre = pkg.models.Mainmodel_continue(args, 14, 64, 4, 4, 1, 2, inner, "GIN")
    path = str(tmp_path / "pre.pt")
    pkg.models.save_checkpoint(pre, path, args, in_dim=14, num_classes=2)
    back = pkg.models.load_checkpoint(path, args)
    a, b = pre.state_dict(), back.state_dict()
    assert set(a) == set(b) and all(torch.equal(a[k], b[k]) for k in a)
    ft = pkg.models.Mainmodel_finetuning(args, 14, 64, 4, 4, 1, 2, path, "GIN")
    frozen = {n for n, p in ft.named_parameters() if not p.requires_grad}
    assert frozen and all(n.startswith("model.") and "layers.2" not in n for n in frozen)
    assert all(p.requires_grad for n, p in ft.named_parameters()
               if n.startswith("model.") and "layers.2" in n)


def test_adam_rejects_cpu_parameters(pkg):
    """The device optimizer fails loudly on CPU tensors (no CPU fallback)."""
    p = torch.zeros(4, requires_grad=True)
    p.grad = torch.ones(4)
    opt = pkg.optim.Adam([p], lr=1e-3)
    with pytest.raises(pkg._lib.ScgibError):
        opt.step()
    with pytest.raises(NotImplementedError):
        pkg.optim.Adam([p], amsgrad=True)


def test_checkpoint_roundtrip_domainadapt(pkg, tmp_path):
    """A domain-adapted model (wrapping a Mainmodel_continue wrapping a
    Mainmodel) saves and loads weights-only, nesting rebuilt from the config."""
    from types import SimpleNamespace
    args = SimpleNamespace(recons_type="adj", useAtt=1, readout_f="sum", d_transfer=32,
                           batch_size=8, gin_layers=4, task="graph_classification",
                           dataset="ogbg-molhiv")
    inner = pkg.models.Mainmodel(args, 9, 64, 4, 4, 1, "GIN")
    pre = pkg.models.Mainmodel_continue(args, 9, 64, 4, 4, 1, 1, inner, "GIN")
    da = pkg.models.Mainmodel_domainadapt(args, 9, 64, 4, 4, 1, 1, pre, "GIN")
    assert all(p.requires_grad for p in da.parameters())
    path = str(tmp_path / "da.pt")
    pkg.models.save_checkpoint(da, path, args, in_dim=9, num_classes=1)
    back = pkg.models.load_checkpoint(path, args)
    assert type(back).__name__ == "Mainmodel_domainadapt"
    assert type(back.model).__name__ == "Mainmodel_continue"
    a, b = da.state_dict(), back.state_dict()
    assert set(a) == set(b) and all(torch.equal(a[k], b[k]) for k in a)
    ft = pkg.models.Mainmodel_finetuning(args, 9, 64, 4, 4, 1, 1, path, "GIN")
    assert type(ft.model).__name__ == "Mainmodel_domainadapt"


# ---------------------------------------------------------------------------
# §8(f) #2: on-disk CSR cache
# ---------------------------------------------------------------------------
def _records(pkg, n, seed, bad_at=()):
    mols = pkg.synth.molecules(n, "qm9", seed=seed)
    rng = np.random.default_rng(seed)
    recs = [(ei, x, rng.integers(0, 2, size=(1, 3)).astype(np.float32)) for ei, x in mols]
    for i in bad_at:  # trailing isolated atom: x has a row the edges never reach
        ei, x, y = recs[i]
        recs[i] = (ei, np.concatenate([x, x[:1]]), y)
    return recs


def test_csr_cache_roundtrip_matches_collate(pkg, tmp_path):
    recs = _records(pkg, 60, 3, bad_at=(7, 31))
    c = pkg.cache.write(recs, str(tmp_path), "QM9", cap=None, logm_k=(1, 2))
    assert len(c) == 58 and c.meta["missing"] == 2 and c.meta["records_read"] == 60
    kept = [i for i in range(60) if i not in (7, 31)]
    np.testing.assert_array_equal(np.asarray(c.kept), kept)
    c = pkg.cache.open_cache(str(tmp_path), "QM9")  # memory-mapped
    order = np.random.default_rng(0).permutation(len(c))[:23]
    g, y, logms = c.collate(order, k_logm=2)
    ref, _ = pkg.graph.collate_pyg([recs[kept[i]][:2] for i in order])
    for a in ("rowptr", "col", "graph_ptr"):
        assert torch.equal(getattr(g, a), getattr(ref, a)), a
    assert torch.equal(g.ndata["x"], ref.ndata["x"])
    np.testing.assert_array_equal(g.batch_num_edges().numpy(), ref.batch_num_edges().numpy())
    assert torch.equal(y, torch.from_numpy(np.stack([recs[kept[i]][2] for i in order])))
    for j, i in enumerate(order):
        gi = pkg.graph.from_pyg(*recs[kept[i]][:2])
        np.testing.assert_array_equal(logms[j].numpy(), pkg.graph.trans_logM(gi, 2).numpy())
    seen = np.concatenate([b[1].numpy()[:, 0, 0] * 0 + np.arange(len(b[1]))
                           for b in c.batches(16, seed=1)])
    assert len(seen) == len(c)


def test_csr_cache_cap_and_name_alias(pkg, tmp_path):
    """Records at index >= cap are never read; skipped records count towards
    the cap (exp_molpcba.py:333); 'mol-PCBA' resolves to the cache the
    molpcba preprocessor names 'ogbg-molpcba' (exp_molpcba.py:373 vs
    exp_pretraining.py:218)."""
    recs = _records(pkg, 30, 4, bad_at=(3,))

    def gen():
        for i, r in enumerate(recs):
            if i >= 10:
                raise AssertionError("record past the cap was read")
            yield r
    c = pkg.cache.write(gen(), str(tmp_path), "ogbg-molpcba", cap=10)
    assert len(c) == 9 and c.meta["missing"] == 1
    c2 = pkg.cache.open_cache(str(tmp_path), "mol-PCBA")
    assert c2.path == c.path and len(c2) == 9
    with pytest.raises(FileNotFoundError):
        pkg.cache.open_cache(str(tmp_path), "QM9")


def test_csr_cache_reference_ingest_goldens(pkg, tmp_path):
    """The cache applies load_dgl_fromPyG + the skip rule exactly as the
    reference did on its own inputs (golden ingest_egonet)."""
    d = load_golden("ingest_egonet")
    nm = int(d["num_mols"])
    recs = [(d[f"m{i}_edge_index"], d[f"m{i}_x"]) for i in range(nm)]
    c = pkg.cache.write(recs, str(tmp_path), "golden", cap=None)
    kept = [i for i in range(nm) if d[f"m{i}_kept"]]
    np.testing.assert_array_equal(np.asarray(c.kept), kept)
    for j, i in enumerate(kept):
        s, t = c.graph(j).edges()
        np.testing.assert_array_equal(s.numpy(), d[f"m{i}_src"])
        np.testing.assert_array_equal(t.numpy(), d[f"m{i}_dst"])


def test_ego_bounds_match_oracle_sizes(pkg):
    """graph.ego_bounds (capacity sizing for k-hop ego-nets) equals the oracle's
    ego-net sizes for the node count and bounds the edge count."""
    from oracle import egonet
    mols = pkg.synth.molecules(40, "pcqm4mv2", seed=3)
    g, _ = pkg.graph.collate_pyg(mols)
    for k in (1, 2, 3):
        ns, es, dmax = pkg.graph.ego_bounds(g, k)
        sizes, ecount, _, _, _ = egonet.egonets(g.rowptr.numpy(), g.col.numpy(), k)
        assert ns == int(sizes.sum())
        assert es >= int(ecount.sum())
        assert dmax == int(np.diff(g.rowptr.numpy()).max())


def test_slab_scope_rules(pkg, monkeypatch):
    """ops.SlabScope (host logic, no launch): usable only while open, with
    every parameter a contiguous fp32 leaf whose .grad is None, and with no
    other scope awaiting its backward; take() closes it and hands over the
    jobs."""
    ops = pkg.ops
    monkeypatch.setattr(ops.SlabScope, "_device_ok", staticmethod(lambda p: True))
    w = torch.zeros(4, requires_grad=True)
    # parameters autograd would cast or copy the returned gradient for: inline
    assert not ops.SlabScope().usable((torch.zeros(4, dtype=torch.float64, requires_grad=True),))
    assert not ops.SlabScope().usable((torch.zeros(4, 2, requires_grad=True).t(),))
    a = ops.SlabScope()
    assert a.usable((w, None))
    slab, out = torch.zeros(8), torch.zeros(4)
    a.add(slab, out, 4, 2)
    w.grad = torch.zeros(4)
    assert not a.usable((w,))
    w.grad = None
    b = ops.SlabScope()  # a second forward before a's backward: neither defers
    assert not a.usable((w,)) and not b.usable((w,))
    jobs, keep = a.take()
    assert len(jobs) == 1 and jobs[0].n_slabs == 2 and jobs[0].width == 4
    assert keep[0] is slab and keep[1] is out
    assert not a.usable((w,))
    del b
    c = ops.SlabScope()  # a closed scope does not poison a new one
    assert c.usable((w,))
    h = w.register_hook(lambda g: g)  # a gradient hook reads the tensor early: inline
    assert not c.usable((w,))
    h.remove()
    assert c.usable((w,))


REF_CKPT = "/root/reference/outputs/pre_training_v1_GIN_64_5_1.pt"


def _ckpt_fixture():
    d = load_golden("ckpt_pre_training_v1_GIN_64_5_1")
    levels = [(s.split(":")[0], int(s.split(":")[1])) for s in d["levels"].tolist()]
    cfg = {k[4:]: (v.item() if v.dtype.kind in "iuf" else str(v)) for k, v in d.items()
           if k.startswith("cfg_")}
    sd = {k[3:]: torch.tensor(v) for k, v in d.items() if k.startswith("sd/")}
    return levels, cfg, sd


@pytest.mark.skipif(not os.path.exists(REF_CKPT), reason="the reference tree is not here")
def test_reference_checkpoint_reads_weights_only(pkg):
    """refckpt.read on the shipped whole-module pickle (models.py:421):
    weights-only through inert stand-ins, the same 544 tensors as the
    committed fixture, and models.load_checkpoint rebuilds the 4-level
    wrapper chain with them (strict)."""
    levels, cfg, sd = pkg.refckpt.read(REF_CKPT)
    f_levels, f_cfg, f_sd = _ckpt_fixture()
    assert levels == f_levels and set(sd) == set(f_sd) and len(sd) == 544
    for k, v in sd.items():
        assert torch.equal(v, f_sd[k]), k
    assert cfg["gin_layers"] == 5 and cfg["k_transition"] == 1 and cfg["in_dim"] == 9
    args = type("A", (), {"task": "graph_classification"})()
    m = pkg.models.load_checkpoint(REF_CKPT, args)
    assert type(m).__name__ == "Mainmodel_continue"
    assert type(m.model.model.model).__name__ == "Mainmodel"
    got = m.state_dict()
    assert all(torch.equal(got[k], v) for k, v in sd.items())


def test_checkpoint_levels_roundtrip(pkg, tmp_path):
    """The fixture's 4-level chain (each level its own transfer_d width)
    through save_checkpoint / load_checkpoint (weights only), and a file
    naming a class outside the known set is refused before loading."""
    levels, cfg, sd = _ckpt_fixture()
    m = pkg.models.model_from_state(levels, cfg, sd)
    path = str(tmp_path / "ckpt.pt")
    args = type("A", (), {"recons_type": "adj", "useAtt": 1, "readout_f": "sum",
                          "d_transfer": 32, "gin_layers": 5, "task": "graph_classification",
                          "batch_size": 16})()
    pkg.models.save_checkpoint(m, path, args, in_dim=levels[0][1])
    m2 = pkg.models.load_checkpoint(path, args)
    s2 = m2.state_dict()
    assert set(s2) == set(sd) and all(torch.equal(s2[k], v) for k, v in sd.items())
    bad = str(tmp_path / "bad.pt")
    torch.save({"x": torch.zeros(1)}, bad)
    assert not pkg.refckpt.is_reference_module_checkpoint(bad)
    with pytest.raises(pkg.refckpt.RefCheckpointError):
        pkg.refckpt.read(bad)


def test_pickle_globals_resolves_memo_references(pkg, tmp_path):
    """STACK_GLOBAL operands fetched from the memo (protocol 4 memoizes the
    module string and BINGETs it for the next class of the same module) are
    resolved, not taken from the last two literals; an operand that is not a
    string is refused.  The pickle bytes are built by hand (disassembled only)."""
    import pickletools
    import zipfile

    def zipped(name, payload):
        p = str(tmp_path / name)
        with zipfile.ZipFile(p, "w") as z:
            z.writestr("archive/data.pkl", payload)
        return p

    # [models.Mainmodel, models.GIN] with 'models' memoized once and fetched
    u = lambda s: b"\x8c" + bytes([len(s)]) + s.encode()  # SHORT_BINUNICODE
    payload = (b"\x80\x04]\x94(" + u("models") + b"\x94" + u("Mainmodel") + b"\x94\x93\x94"
               + b"h\x01" + u("GIN") + b"\x94\x93\x94e.")
    pickletools.dis(payload, out=open(os.devnull, "w"))  # well-formed
    assert pkg.refckpt.pickle_globals(zipped("memo.pt", payload)) == {"models.Mainmodel",
                                                                       "models.GIN"}
    bad = b"\x80\x04]\x94(" + u("models") + b"\x94K\x05\x93\x94e."  # name = BININT1 5
    with pytest.raises(pkg.refckpt.RefCheckpointError):
        pkg.refckpt.pickle_globals(zipped("bad_sg.pt", bad))


def test_bench_kernel_table_evaluates(pkg):
    """bench.py imports on a CPU host and every KERNELS entry's bytes / flops
    evaluate on a per-layer launch meta."""
    import importlib
    import sys
    sys.path.insert(0, ROOT)
    bench = importlib.import_module("bench")
    layer = {"n": 1000, "e": 2000, "d_in": 64}
    for name, spec in bench.KERNELS.items():
        b = bench._call_meta(spec["bytes"], layer)
        f = bench._call_meta(spec["flops"], layer)
        assert b > 0 and f >= 0, name


def test_xq_handoffs_off_under_serialised_dispatch(pkg, monkeypatch):
    """ops.XQ_FLAGS's default: the signal / wait hand-offs need concurrent
    queues, so they are off under PMC counter collection, kernel tracing or
    serialised / blocking launches (a replayed graph could order a wait before
    its signal on one queue)."""
    for k in ("ROCPROF_COUNTER_COLLECTION", "ROCPROF_KERNEL_TRACE", "AMD_SERIALIZE_KERNEL",
              "HIP_LAUNCH_BLOCKING", "CUDA_LAUNCH_BLOCKING"):
        monkeypatch.delenv(k, raising=False)
    assert not pkg.ops._dispatch_serialised()
    monkeypatch.setenv("AMD_SERIALIZE_KERNEL", "0")
    assert not pkg.ops._dispatch_serialised()
    for k in ("ROCPROF_COUNTER_COLLECTION", "ROCPROF_KERNEL_TRACE", "AMD_SERIALIZE_KERNEL",
              "HIP_LAUNCH_BLOCKING"):
        monkeypatch.setenv(k, "1")
        assert pkg.ops._dispatch_serialised()
        monkeypatch.delenv(k)


def test_handoff_rule(pkg):
    """ops.handoff_rule — the signal / wait hand-offs only
    where the step's two chains can be on hardware queues the device runs
    concurrently: not under serialised dispatch, not with one hardware queue
    per process or one graph-execution stream, not with more local ranks than
    devices (LOCAL_WORLD_SIZE, not the global world: a multi-node job with one
    rank per GPU keeps them)."""
    rule = pkg.ops.handoff_rule
    assert rule(1, {})[0]
    assert rule(8, {"LOCAL_WORLD_SIZE": "8", "WORLD_SIZE": "16"})[0]   # 2 nodes x 8 GPUs
    assert rule(None, {"LOCAL_WORLD_SIZE": "2"})[0]                    # device count unknown
    assert rule(1, {"GPU_MAX_HW_QUEUES": "4", "DEBUG_HIP_FORCE_GRAPH_QUEUES": "4"})[0]
    for env, dc in (({"LOCAL_WORLD_SIZE": "2"}, 1), ({"LOCAL_WORLD_SIZE": "9"}, 8),
                    ({"GPU_MAX_HW_QUEUES": "1"}, 1), ({"DEBUG_HIP_FORCE_GRAPH_QUEUES": "1"}, 1),
                    ({"AMD_SERIALIZE_KERNEL": "3"}, 1), ({"ROCPROF_KERNEL_TRACE": "1"}, 8)):
        ok, why = rule(dc, env)
        assert not ok and why, env
    # the module default follows the process environment and the local device
    # count, resolved on first use (every entry point gets it)
    import torch
    keep = pkg.ops.XQ_FLAGS, pkg.ops.XQ_REASON
    try:
        pkg.ops.XQ_FLAGS = None
        assert pkg.ops.xq_enabled() == rule(torch.cuda.device_count())[0]
        assert pkg.ops.XQ_FLAGS is not None and pkg.ops.XQ_REASON
    finally:
        pkg.ops.XQ_FLAGS, pkg.ops.XQ_REASON = keep


def test_check_handoff_raises_on_host_fault_word(pkg):
    """The host half of the hand-off fault: a set pinned word makes
    ops.check_handoff (run by every model forward and optimizer step) raise a
    ScgibError that names the hand-off; clean words pass."""
    import torch
    ops = pkg.ops
    key = 977  # a device index no real device uses
    ops._HOST_FAULT[key] = torch.zeros(1, dtype=torch.int32)
    try:
        ops.check_handoff()
        ops._HOST_FAULT[key][0] = 1
        with pytest.raises(pkg._lib.ScgibError, match="hand-off"):
            ops.check_handoff()
        with pytest.raises(pkg._lib.ScgibError, match="hand-off"):
            ops.aside_guard(lambda: None)()
    finally:
        ops._HOST_FAULT.pop(key, None)


def test_slab_scope_defers_launches_once(pkg):
    """ops.SlabScope.defer (the Set2Set LSTM weight gradients): a deferred
    launch runs exactly once — taken by the encoder pair's backward
    (take_later), or by the scope's end-of-backward flush when no pair
    backward takes it — and its tensors stay referenced until then."""
    import torch
    ops = pkg.ops
    calls = []
    sc = ops.SlabScope()
    t = torch.zeros(3)
    sc.defer(lambda: calls.append("a"), t)
    sc.defer(lambda: calls.append("b"), t)
    assert len(sc.later) == 2 and sc.later[0][1][0] is t
    later = sc.take_later()
    assert [f() for f, _ in later] and calls == ["a", "b"] and not sc.later
    sc._flush()  # nothing left: no launch twice
    assert calls == ["a", "b"]
    sc2 = ops.SlabScope()
    sc2.defer(lambda: calls.append("c"), t)
    sc2._flush()  # no pair backward took it: the flush runs it
    assert calls == ["a", "b", "c"] and not sc2.later and not sc2.open
    sc2._flush()
    assert calls == ["a", "b", "c"]


def test_scan_arena_carves_disjoint_zeroed_ranges(pkg):
    """ops._scan_carve (the scan-state arena): disjoint, 256-B aligned, zeroed
    ranges from one arena; a request past its end opens a new arena (the old
    ranges stay valid)."""
    import torch
    ops = pkg.ops
    key = 977  # a device index no real device uses
    try:
        a = ops._scan_carve(key, "cpu", 1024)
        b = ops._scan_carve(key, "cpu", 100)
        c = ops._scan_carve(key, "cpu", 1024)
        assert a.data_ptr() + 1024 * 4 == b.data_ptr()
        assert c.data_ptr() == b.data_ptr() + 128 * 4  # 100 words rounded to 64-word ranges
        assert int(a.abs().sum() + b.abs().sum() + c.abs().sum()) == 0
        big = ops._scan_carve(key, "cpu", ops._SCAN_ARENA_WORDS)
        assert len(ops._SCAN_ARENAS[key]) == 2 and big.numel() == ops._SCAN_ARENA_WORDS
        assert int(big.abs().sum()) == 0
    finally:
        ops._SCAN_ARENAS.pop(key, None)
        ops._SCAN_NEXT.pop(key, None)


def test_set2set_rejects_widths_past_the_device_readout(pkg):
    """the device Set2Set holds a graph's features 64 lanes wide;
    a wider one (domain adaptation over raw features wider than 64) is refused
    when the model is built, with a message, not at its first step."""
    pkg.models.Set2Set(64, 2, 1)
    pkg.models.Set2Set(9, 2, 1)
    with pytest.raises(NotImplementedError, match="width 65"):
        pkg.models.Set2Set(65, 2, 1)
