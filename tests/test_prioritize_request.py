"""Prioritize of one extender request in request order:
pas_tas_prioritize_request against the oracle's or_ordered_list_request, which is pinned to
the reference's OrderedList vectors (operator_test.go:60-61) and to a pure-Python
restatement of prioritizeNodesForRule (telemetryscheduler.go:128-149) with a stable sort.
The CPU tests check the oracle; the gpu tests check libpas.so against it."""
import numpy as np
import pytest

import pas_amd
from helpers import OPS, NamedSnapshot, golden, pack_bits
from oracle import RULE_DTYPE

G = golden()
_gen = [50_000]


def rule(metric, op, target=0):
    r = np.zeros(1, RULE_DTYPE)
    r[0]["metric"], r[0]["op"], r[0]["target"] = metric, op, target
    return r[0]


def python_request_order(v_milli, present_bool, prio, req):
    """filteredNodeData over args.Nodes.Items (one entry per name, first occurrence) then
    OrderedList with a stable sort: the A.3 order, as request positions."""
    m, op = int(prio["metric"]), int(prio["op"])
    n_nodes = v_milli.shape[1]
    if m < 0 or m >= v_milli.shape[0] or not present_bool[m].any():
        return []
    seen, items = set(), []
    for j, n in enumerate(req):
        if n < 0 or n >= n_nodes or n in seen:
            continue
        seen.add(n)
        if present_bool[m, n]:
            items.append((int(v_milli[m, n]), j))
    if op == 1:
        items.sort(key=lambda t: -t[0])
    elif op == 0:
        items.sort(key=lambda t: t[0])
    return [j for _, j in items]


def random_request(rng, n_nodes, n_req, unknown=0.05, dup=0.1):
    req = rng.integers(0, max(n_nodes, 1), n_req).astype(np.int32)
    if n_req and n_nodes:
        # a permutation prefix so most nodes appear once, then duplicates / unknowns
        base = rng.permutation(n_nodes)[: n_req].astype(np.int32)
        req[: len(base)] = base
        req[rng.random(n_req) < dup] = rng.integers(0, n_nodes, 1)[0]
    req[rng.random(n_req) < unknown] = -1
    return req


def random_snapshot(rng, n, m, n_vals=5, absent=0.2):
    v = rng.integers(0, n_vals, (m, n)).astype(np.int64) * 1000
    v[:, ::7] = rng.integers(-2**62, 2**62, (m, len(range(0, n, 7))))
    pres_b = rng.random((m, n)) >= absent
    return v, pres_b, pack_bits(pres_b)


# ------------------------------------------------------------------- oracle (CPU)

def test_oracle_g2_ordered_list(oracle):
    g = G["G2_ordered_list"]
    snap = NamedSnapshot({"m": dict(zip(g["nodes"], g["values"]))})
    req = np.array([snap.node_index[n] for n in g["nodes"]], np.int32)
    for c in g["cases"]:
        pos = oracle.prioritize_request(snap.v_milli, snap.present,
                                        rule(0, OPS[c["operator"]]), req)
        assert [g["nodes"][j] for j in pos] == c["want"]


def test_oracle_g5_prioritize(oracle):
    g = G["G5_prioritize"]
    snap = NamedSnapshot(g["metrics"], g["nodes"])
    req = np.array([snap.node_index[n] for n in g["nodes"]], np.int32)
    pos = oracle.prioritize_request(snap.v_milli, snap.present, rule(0, OPS["GreaterThan"]),
                                    req)
    assert [[g["nodes"][j], 10 - i] for i, j in enumerate(pos)] == g["want"]


@pytest.mark.parametrize("seed", range(8))
def test_oracle_matches_python_restatement(oracle, seed):
    rng = np.random.default_rng(seed)
    n, m = int(rng.integers(1, 300)), 3
    v, pres_b, pres = random_snapshot(rng, n, m)
    for op in (0, 1, 2, 7):
        for n_req in (0, 1, n, 2 * n):
            req = random_request(rng, n, n_req)
            want = python_request_order(v, pres_b, rule(op % 3, op), req)
            got = oracle.prioritize_request(v, pres, rule(op % 3, op), req)
            assert list(got) == want


def test_oracle_ties_follow_request_not_node_index(oracle):
    # three nodes with one value: the request lists them in reverse
    v = np.full((1, 3), 5000, np.int64)
    pres_b = np.ones((1, 3), bool)
    req = np.array([2, 0, 1], np.int32)
    for op in (0, 1, 2):
        assert list(oracle.prioritize_request(v, pack_bits(pres_b), rule(0, op), req)) == [0, 1, 2]


# ------------------------------------------------------------------- libpas.so (GPU)

def upload(ctx, v, pres):
    _gen[0] += 1
    ctx.tas_snapshot_set(_gen[0], v, pres)
    return _gen[0]


@pytest.mark.gpu
def test_gpu_golden_g2_g5(ctx):
    g = G["G2_ordered_list"]
    snap = NamedSnapshot({"m": dict(zip(g["nodes"], g["values"]))})
    gen = upload(ctx, snap.v_milli, snap.present)
    req = np.array([snap.node_index[n] for n in g["nodes"]], np.int32)
    for c in g["cases"]:
        pos = ctx.tas_prioritize_request(gen, rule(0, OPS[c["operator"]]), req)
        assert [g["nodes"][j] for j in pos] == c["want"]
    g = G["G5_prioritize"]
    snap = NamedSnapshot(g["metrics"], g["nodes"])
    gen = upload(ctx, snap.v_milli, snap.present)
    req = np.array([snap.node_index[n] for n in g["nodes"]], np.int32)
    pos = ctx.tas_prioritize_request(gen, rule(0, OPS["GreaterThan"]), req)
    assert [[g["nodes"][j], 10 - i] for i, j in enumerate(pos)] == g["want"]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 1000, 4097, 65537])
def test_gpu_random_parity(ctx, oracle, n):
    rng = np.random.default_rng(n)
    m = 3
    v, pres_b, pres = random_snapshot(rng, n, m, n_vals=1 + n // 50)
    gen = upload(ctx, v, pres)
    for op in (0, 1, 2, 5):
        for n_req in sorted({0, 1, n // 2, n, n + n // 3}):
            req = random_request(rng, n, n_req)
            pr = rule(int(rng.integers(0, m)), op)
            want = oracle.prioritize_request(v, pres, pr, req)
            got = ctx.tas_prioritize_request(gen, pr, req)
            np.testing.assert_array_equal(got, want, err_msg=f"op {op} n_req {n_req}")


@pytest.mark.gpu
def test_gpu_reversed_request_ties(ctx, oracle):
    # every value tied, request in reverse node order: the list is the request order
    n = 5000
    v = np.zeros((1, n), np.int64)
    pres_b = np.ones((1, n), bool)
    gen = upload(ctx, v, pack_bits(pres_b))
    req = np.arange(n - 1, -1, -1, dtype=np.int32)
    for op in (0, 1, 2):
        got = ctx.tas_prioritize_request(gen, rule(0, op), req)
        np.testing.assert_array_equal(got, np.arange(n))


@pytest.mark.gpu
def test_gpu_extremes_and_out_of_range(ctx, oracle):
    # INT64 extremes sort correctly; indices past n_nodes count as unknown nodes
    v = np.array([[np.iinfo(np.int64).min, np.iinfo(np.int64).max, 0, -1, 1]], np.int64)
    pres_b = np.array([[True, True, True, False, True]])
    pres = pack_bits(pres_b)
    gen = upload(ctx, v, pres)
    req = np.array([4, 99, 3, 1, -7, 0, 2, 1], np.int32)
    for op in (0, 1, 2):
        want = python_request_order(v, pres_b, rule(0, op), req)
        assert list(ctx.tas_prioritize_request(gen, rule(0, op), req)) == want


@pytest.mark.gpu
def test_gpu_no_rule_empty_and_errors(ctx):
    v = np.arange(10, dtype=np.int64)[None, :] * 1000
    gen = upload(ctx, v, pack_bits(np.ones((1, 10), bool)))
    req = np.arange(10, dtype=np.int32)
    assert len(ctx.tas_prioritize_request(gen, rule(-1, 1), req)) == 0
    assert len(ctx.tas_prioritize_request(gen, rule(0, 1), req[:0])) == 0
    with pytest.raises(pas_amd.PasError):
        ctx.tas_prioritize_request(gen, rule(1, 1), req)  # metric past n_metrics
    with pytest.raises(pas_amd.PasError):
        ctx.tas_prioritize_request(gen + 1, rule(0, 1), req)  # stale generation


@pytest.mark.gpu
def test_gpu_device_entry_matches_host(ctx, oracle):
    import torch
    rng = np.random.default_rng(7)
    n = 20000
    v, pres_b, pres = random_snapshot(rng, n, 2, n_vals=40)
    gen = upload(ctx, v, pres)
    req = random_request(rng, n, n)
    pr = rule(1, 0)
    want = oracle.prioritize_request(v, pres, pr, req)
    req_t = torch.from_numpy(req).cuda()
    pos_t = torch.empty(n, dtype=torch.int32, device="cuda")
    len_t = torch.empty(1, dtype=torch.int32, device="cuda")
    ctx.tas_prioritize_request_device(gen, pr, n, req_t, pos_t, len_t,
                                      stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    k = int(len_t.item())
    np.testing.assert_array_equal(pos_t[:k].cpu().numpy(), want)
    assert (pos_t[k:] == -1).all()


@pytest.mark.gpu
def test_gpu_empty_snapshot_empty_request(ctx):
    # N = 0 and n_req = 0: every workspace part is 0 bytes; the call is an empty list, not a
    # sizing failure
    gen = upload(ctx, np.zeros((1, 0), np.int64), np.zeros((1, 0), np.uint64))
    assert len(ctx.tas_prioritize_request(gen, rule(0, 1), np.zeros(0, np.int32))) == 0
    # unknown nodes only (req -1): nothing listed
    assert len(ctx.tas_prioritize_request(gen, rule(0, 0), np.full(3, -1, np.int32))) == 0
