"""The two-lane replay's plan (csrc/graph_split.hip, scgib_graph_split_plan),
checked on the host: no device is needed to plan, only to replay.

The plan turns a captured DAG into two in-order lanes joined by signal / wait
hand-offs (DESIGN.md §3 "Host enqueue").  Its claim: whatever order the two
queues run in, the lanes finish (no deadlock) and every edge of the DAG — and
every in-graph hand-off the graph does not show as an edge — is honoured.
Here that is checked by executing the plan's lanes in a simulator under
adversarial and random schedules, on the step's own shape and on random
captures of two and three streams with forks, joins and in-graph hand-offs.
"""
import ctypes
import random

import numpy as np
import pytest

EUNSUPPORTED = -2


def _plan(pkg, n, edges, hidden=()):
    lib = pkg._lib.load()
    i32 = np.int32
    frm = np.array([e[0] for e in edges] or [0], i32)
    to = np.array([e[1] for e in edges] or [0], i32)
    hs = np.array([h[0] for h in hidden] or [0], i32)
    hw = np.array([h[1] for h in hidden] or [0], i32)
    lane, pos, ws, ss = (np.full(n, -7, i32) for _ in range(4))
    info = np.zeros(4, i32)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rc = lib.scgib_graph_split_plan(n, len(edges), p(frm), p(to), len(hidden), p(hs), p(hw),
                                    p(lane), p(pos), p(ws), p(ss), p(info))
    return rc, dict(lane=lane, pos=pos, wait=ws, signal=ss, slots=int(info[0]),
                    start=int(info[1]), end=int(info[2]), loose=int(info[3]))


def _lanes(n, pl):
    """The two lanes as item lists: ("node", v) / ("wait", slot) / ("signal", slot)."""
    seq = [[], []]
    for v in sorted(range(n), key=lambda v: (pl["lane"][v], pl["pos"][v])):
        seq[pl["lane"][v]].append(v)
    items = [[], []]
    if pl["start"] >= 0:
        items[0].append(("signal", pl["start"]))
        items[1].append(("wait", pl["start"]))
    for l in (0, 1):
        for v in seq[l]:
            if pl["wait"][v] >= 0:
                items[l].append(("wait", int(pl["wait"][v])))
            items[l].append(("node", v))
            if pl["signal"][v] >= 0:
                items[l].append(("signal", int(pl["signal"][v])))
    if pl["end"] >= 0:
        items[1].append(("signal", pl["end"]))
        items[0].append(("wait", pl["end"]))
    return items


def _execute(n, edges, hidden, pl, pick):
    """Run the lanes; pick(runnable lanes) chooses which advances.  Returns the
    global execution index of every node, or raises on a deadlock."""
    items = _lanes(n, pl)
    head = [0, 0]
    posted = {}  # slot -> signals posted - waits passed
    done = {}
    hidden_sig = {w: s for s, w in hidden}
    step = 0

    def runnable(l):
        if head[l] >= len(items[l]):
            return False
        kind, x = items[l][head[l]]
        if kind == "wait":
            return posted.get(x, 0) > 0
        if kind == "node" and x in hidden_sig:  # an in-graph wait kernel
            return hidden_sig[x] in done
        return True

    while head[0] < len(items[0]) or head[1] < len(items[1]):
        ready = [l for l in (0, 1) if runnable(l)]
        assert ready, f"deadlock at heads {head}: {[items[l][head[l]:head[l] + 1] for l in (0, 1)]}"
        l = pick(ready)
        kind, x = items[l][head[l]]
        if kind == "wait":
            posted[x] -= 1
        elif kind == "signal":
            posted[x] = posted.get(x, 0) + 1
        else:
            done[x] = step
            step += 1
        head[l] += 1
    assert sorted(done) == list(range(n))
    return done


def _check(n, edges, hidden, pl, seed=0):
    rng = random.Random(seed)
    schedules = [lambda r: r[0], lambda r: r[-1]] + [lambda r: rng.choice(r)] * 20
    for pick in schedules:
        at = _execute(n, edges, hidden, pl, pick)
        for u, v in edges:
            assert at[u] < at[v], (u, v)
        for s, w in hidden:
            assert at[s] < at[w], (s, w)


def _capture(rng, streams, ops, handoffs=True):
    """A random stream capture: kernels on `streams` streams, forks / joins as
    edges from another stream's last node, and in-graph hand-offs as a signal
    node on one stream and a wait node on another (hidden pairs).  Stream 0
    is the origin: the others fork from it first and join it last."""
    edges, hidden, last = [], [], [None] * streams
    n = 0

    def node(s, extra=()):
        nonlocal n
        v = n
        n += 1
        if last[s] is not None:
            edges.append((last[s], v))
        for u in extra:
            if u is not None and u != last[s]:
                edges.append((u, v))
        last[s] = v
        return v

    node(0)
    forked = [True] + [False] * (streams - 1)
    pending = []  # (signal node, target stream)
    for _ in range(ops):
        s = rng.randrange(streams)
        if not forked[s]:
            node(s, (last[0],))  # fork from the origin
            forked[s] = True
            continue
        r = rng.random()
        if r < 0.15 and streams > 1:  # a stream dependency on another stream's work so far
            t = rng.choice([x for x in range(streams) if x != s and forked[x]] or [s])
            node(s, (last[t],))
        elif r < 0.25 and handoffs and streams > 1:  # an in-graph signal, waited later elsewhere
            sig = node(s)
            t = rng.choice([x for x in range(streams) if x != s])
            pending.append((sig, t))
        elif r < 0.35 and pending:
            sig, t = pending.pop(0)
            if forked[t]:
                hidden.append((sig, node(t)))
        else:
            node(s)
    for s in range(1, streams):  # join everything back into the origin
        if forked[s]:
            node(0, (last[s],))
    return n, edges, hidden


def test_plan_of_the_step_shape(pkg):
    """The pretraining step: batch load, fork, ego / core forward chains, the
    forward hand-off (ego -> interaction), loss section, the backward hand-off
    (loss section -> core chain), the backward chains, join, reduce + Adam."""
    edges, hidden = [], []
    load = 0
    ego_f = list(range(1, 7))      # side stream
    core_f = list(range(7, 13))    # origin
    sig_f, wait_f = 13, 14         # side signal, origin wait
    loss = [15, 16, 17]            # origin
    sig_b, wait_b = 18, 19         # origin signal, side wait
    ego_b = [20, 21, 22, 23]       # origin
    core_b = [24, 25, 26]          # side
    join, adam = 27, 28
    chain = lambda c: edges.extend(zip(c, c[1:]))  # noqa: E731
    chain([load] + core_f + [wait_f] + loss + [sig_b] + ego_b + [join, adam])
    chain([load] + ego_f + [sig_f, wait_b] + core_b)
    edges.append((core_b[-1], join))
    hidden = [(sig_f, wait_f), (sig_b, wait_b)]
    n = 29
    rc, pl = _plan(pkg, n, edges, hidden)
    assert rc == 0
    assert pl["loose"] == 0 and pl["slots"] == 2, pl  # the fork and the join
    assert len(set(pl["lane"][core_f])) == 1 and len(set(pl["lane"][ego_f])) == 1
    assert pl["lane"][sig_f] != pl["lane"][wait_f] and pl["lane"][sig_b] != pl["lane"][wait_b]
    _check(n, edges, hidden, pl)


@pytest.mark.parametrize("streams", [1, 2, 3])
def test_plan_random_captures_execute_in_order(pkg, streams):
    rng = random.Random(1000 + streams)
    checked = refused = 0
    for trial in range(150):
        n, edges, hidden = _capture(rng, streams, rng.randrange(5, 60))
        rc, pl = _plan(pkg, n, edges, hidden)
        if rc == EUNSUPPORTED:  # an in-graph hand-off the two lanes cannot keep in order
            refused += 1
            assert streams == 3 or hidden, "only hand-offs or a third chain can be refused"
            continue
        assert rc == 0
        if streams < 3:
            assert pl["loose"] == 0
        _check(n, edges, hidden, pl, seed=trial)
        checked += 1
    assert checked >= 100, (checked, refused)


def test_plan_refuses_a_handoff_against_the_order(pkg):
    # a wait node that precedes its own signal on one chain
    edges = [(0, 1), (1, 2)]
    rc, _ = _plan(pkg, 3, edges, [(2, 1)])
    assert rc == EUNSUPPORTED


def test_plan_rejects_bad_arguments(pkg):
    assert _plan(pkg, 2, [(0, 5)])[0] == -1
