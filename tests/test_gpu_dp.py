"""The data-parallel step on the HIP kernels (replica mode),
VERDICT r03 item 4: two gloo ranks on one GPU run the product step
(tests/dp_worker.py: capacity mode, captured forward + backward + bucket pack,
the all-reduce between replays, captured unpack + Adam) on the two shards of
one molecule set, each with its own explicit noise.  Checked here:

  * both replicas hold bitwise the same parameters and BatchNorm statistics
    after the step;
  * they equal ONE process applying scgib Adam to the mean of the two shards'
    HIP gradients (and the mean of their BN statistics) — bitwise: the bucket
    is (g0 + g1) * 0.5 either way;
  * the mean of the shards' HIP gradients matches the fp64 oracle's mean of
    the shards' gradients (oracle/scgib_ref.py, exp_pretraining.py:321-323)
    within the config-parity bars (tests/test_gpu_config_parity.py: per-tensor
    rel-L2 2e-3 on every tensor), the mean BN statistics within 1e-4, and each
    shard's losses within 1e-4.
"""
import copy
import importlib
import os
import socket
import subprocess
import sys

import pytest
import torch

from conftest import ROOT, check_grads_model, rel_err

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(ROOT, "tests"))
import dp_worker as W  # noqa: E402
from test_gpu_config_parity import EACH_TOL, LOSS_TOL, _oracle  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def ranks(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    out = tmp_path_factory.mktemp("dp")
    env = dict(os.environ, SCGIB_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "dp_worker.py"), str(out)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return [torch.load(os.path.join(out, f"rank{i}.pt"), weights_only=True) for i in (0, 1)]


def test_replicas_identical_after_step(ranks):
    a, b = ranks[0]["after"], ranks[1]["after"]
    assert a["xq_timeouts"] == 0 and b["xq_timeouts"] == 0
    for k, v in a["params"].items():
        assert torch.equal(v, b["params"][k]), k
    for k, v in a["buffers"].items():
        assert torch.equal(v, b["buffers"][k]), k
    # and the step changed something (the all-reduced update was applied)
    init = ranks[0]["init"]
    assert any(not torch.equal(v, init[k]) for k, v in a["params"].items())


def test_step_equals_adam_on_mean_gradient(pkg, ranks):
    dev = torch.device("cuda", 0)
    F_in = pkg.synth.WORKLOADS[W.WORKLOAD][2]
    model = W.make_model(pkg, F_in, W.B_TOTAL // 2).to(dev).train()
    model.load_state_dict(ranks[0]["init"])
    g0, g1 = ranks[0]["raw"]["grads"], ranks[1]["raw"]["grads"]
    params = dict(model.named_parameters())
    for k, p in params.items():
        p.grad = ((g0[k] + g1[k]) * 0.5).to(dev) if k in g0 else None
    bufs = dict(model.named_buffers())
    b0, b1 = ranks[0]["raw"]["buffers"], ranks[1]["raw"]["buffers"]
    with torch.no_grad():
        for k, v in bufs.items():
            if k.endswith(("running_mean", "running_var")):
                v.copy_((b0[k] + b1[k]) * 0.5)
            else:
                assert torch.equal(b0[k], b1[k]), k  # num_batches_tracked: one step each
                v.copy_(b0[k])
    opt = pkg.optim.Adam(model.parameters(), lr=1e-3, weight_decay=5e-5)
    opt.step()
    torch.cuda.synchronize()
    after = ranks[0]["after"]
    for k, p in params.items():
        assert torch.equal(p.detach().cpu(), after["params"][k]), k
    for k, v in bufs.items():
        assert torch.equal(v.cpu(), after["buffers"][k]), k


def test_mean_gradient_matches_oracle(pkg, ranks):
    F_in = pkg.synth.WORKLOADS[W.WORKLOAD][2]
    B = W.B_TOTAL // 2
    init = ranks[0]["init"]
    refs = []
    for r in (0, 1):
        gh, u_gate, u_feat = W.shard_and_noise(pkg, r, 2)
        model = W.make_model(pkg, F_in, B).train()
        model.load_state_dict(init)
        ref = _oracle(pkg, copy.deepcopy(model), gh, W.K, u_gate, u_feat, B)
        for name, a, b in zip(("kl", "contrastive", "recon"), ranks[r]["raw"]["losses"].tolist(),
                              ref["losses"]):
            assert rel_err(a, b) < LOSS_TOL, (r, name, a, b)
        refs.append(ref)
    mean_ref = {k: 0.5 * (refs[0]["grads"][k] + refs[1]["grads"][k]) for k in refs[0]["grads"]}
    g0, g1 = ranks[0]["raw"]["grads"], ranks[1]["raw"]["grads"]
    errs = check_grads_model(mean_ref, lambda n: (g0[n] + g1[n]) * 0.5, each_tol=EACH_TOL)
    worst = max(errs.items(), key=lambda kv: kv[1])
    print(f"dp mean gradient: worst per-tensor rel-L2 {worst[0]} {worst[1]:.2e}")
    after = ranks[0]["after"]["buffers"]
    for k in refs[0]["buffers"]:
        if k.endswith(("running_mean", "running_var")):
            want = 0.5 * (refs[0]["buffers"][k].double() + refs[1]["buffers"][k].double())
            assert rel_err(after[k], want) < 1e-4, k
