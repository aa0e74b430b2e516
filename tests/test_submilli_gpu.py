"""Sub-milli metric values on the device.

The reference compares resource.Quantity values exactly: CmpInt64 against the integer rule
target and Cmp between values (telemetry-aware-scheduling/pkg/strategies/core/
operator.go:16-22, 37-39).  ParseQuantity keeps at most 9 fractional digits, so a column at
decimal scale k = its values' most decimal places holds every value exactly as an int64
(pas_tas_snapshot_set_scale); targets compare as target * 10^k.  Here the device columns come
from the product's Quantity conversion (pas_amd.snapshot), and the oracle gets each value as
its own exact decimal (u, s) from Python's decimal module (or_*_dec: values aligned to 1e-9
in 128-bit integers) -- two independent paths, bit-exact on filter, prioritize (with ties
inside one milli bucket), the deschedule sweep and label plan, one request's prioritize and
the C5 top-k records."""
from decimal import Decimal

import numpy as np
import pytest
import torch

import pas_amd
from pas_amd import snapshot as sn
from pas_amd import workload as wl
from helpers import RULE_DTYPE, pack_bits, unpack_bits
from test_labels import _fused_and_separate
from test_quantity_scaled import go_value, want_decimals

pytestmark = pytest.mark.gpu


def exact_decimal(lit):
    """(u, s) with value = u * 10^-s exactly, s = the value's decimal places."""
    v = go_value(lit)
    s = want_decimals(v)
    return int(v.scaleb(s)), s


def oracle_arrays(metrics, nodes, metric_names):
    """Per-value (u [M][N], s [M][N]) and presence, from the literals through Decimal."""
    M, N = len(metric_names), len(nodes)
    u = np.zeros((M, N), np.int64)
    s = np.zeros((M, N), np.int8)
    pres = np.zeros((M, N), bool)
    idx = {n: i for i, n in enumerate(nodes)}
    for m, name in enumerate(metric_names):
        for node, lit in metrics[name].items():
            u[m, idx[node]], s[m, idx[node]] = exact_decimal(lit)
            pres[m, idx[node]] = True
    return u, s, pack_bits(pres)


LITERAL_COLUMNS = {
    # ties inside one milli bucket (0.0005 / 0.0007 / 0.0005), 1e-7, 1500u = 0.0015
    "ratio": ["0.0005", "0.0007", "1500u", "1e-7", "0.0015", "0.001", "2m", "0.0005", "0",
              "-0.0003", "999999n", "1", "0.9999999", "1.0000001", "-1e-9", "0.5"],
    "load": ["1.5", "1.25", "1.125", "1.0625", "2", "1.5", "0.75", "3", "1.03125", "2.5",
             "1", "0", "-0.5", "1.5", "4", "1.0000005"],
    "temp": ["70", "71", "69", "70", "72", "68", "70", "75", "60", "80", "70", "71", "69",
             "70", "72", "68"],
}


def literal_case():
    nodes = [f"node-{i}" for i in range(16)]
    metrics = {name: {nodes[i]: lit for i, lit in enumerate(col) if not (name == "load" and
                                                                          i == 7)}
               for name, col in LITERAL_COLUMNS.items()}
    return nodes, metrics, list(LITERAL_COLUMNS)


def rule_batch(rng, M, P, R, targets):
    """targets: a list for every operator, or {op: list} (keeps pass sets large)."""
    rules, off = [], [0]
    prio = np.zeros(P, RULE_DTYPE)
    for p in range(P):
        for _ in range(R):
            op = int(rng.integers(0, 3))
            t = targets[op] if isinstance(targets, dict) else targets
            rules.append((int(rng.integers(0, M)), op, int(rng.choice(t))))
        off.append(len(rules))
        prio[p] = (int(rng.integers(0, M)), int(rng.integers(0, 3)), 0)
    return np.array(rules, RULE_DTYPE), np.array(off, np.int32), prio


def test_literal_snapshot_all_paths(ctx, oracle):
    nodes, metrics, names = literal_case()
    v, pres, scale = sn.tas_snapshot_from_metrics(metrics, nodes, names)
    assert scale.tolist() == [9, 7, 3]
    u, s, opres = oracle_arrays(metrics, nodes, names)
    np.testing.assert_array_equal(pres, opres)
    gen = 9100
    ctx.tas_snapshot_set(gen, v, pres, scale)
    rng = np.random.default_rng(0x5B1)
    rules, off, prio = rule_batch(rng, len(names), 60, 2, [-1, 0, 1, 2, 70, 71])
    gp, go, gl = ctx.tas_eval(gen, rules, off, prio)
    op_, oo, ol = oracle.tas_eval(u, opres, rules, off, prio, v_scale=s)
    np.testing.assert_array_equal(gp, op_)
    np.testing.assert_array_equal(gl, ol)
    for p in range(len(gl)):
        np.testing.assert_array_equal(go[p, : gl[p]], oo[p, : ol[p]], err_msg=f"pod {p}")
    # the sub-milli order itself: ratio ascending puts 1e-7 below 0.0005 (== 0.0005) < 0.0007
    lt = np.zeros(1, RULE_DTYPE)
    lt[0] = (0, 0, 0)
    _, o1, l1 = ctx.tas_eval(gen, np.zeros(0, RULE_DTYPE), np.zeros(2, np.int32), lt)
    order = [nodes[i] for i in o1[0, : l1[0]]]
    assert order.index("node-3") < order.index("node-0") < order.index("node-7") < \
        order.index("node-1") < order.index("node-5") < order.index("node-2")
    # deschedule sweep + label plan, unfused and fused
    dr, doff, _ = rule_batch(rng, len(names), 6, 2, [0, 1, 70])
    want_v = oracle.tas_violations(u, opres, dr, doff, v_scale=s)
    np.testing.assert_array_equal(ctx.tas_violations(gen, dr, doff), want_v)
    labels = wl.pack_bits(rng.random((6, len(nodes))) < 0.5)
    f, sep = _fused_and_separate(ctx, gen, len(nodes), 6, dr, doff, labels)
    want = oracle.label_plan(want_v, labels, len(nodes))
    np.testing.assert_array_equal(f[0], want_v)
    for i in (1, 2):
        np.testing.assert_array_equal(f[i], want[i - 1])
        np.testing.assert_array_equal(sep[i], want[i - 1])
    # one request's prioritize, in request order
    req = rng.permutation(len(nodes)).astype(np.int32)
    for p in range(10):
        np.testing.assert_array_equal(
            ctx.tas_prioritize_request(gen, prio[p], req),
            oracle.prioritize_request(u, opres, prio[p], req, v_scale=s))


def scaled_snapshot(rng, N, scales):
    """Columns at the given decimal scales: values on a 1e-4 grid in [-1000, 1000] (many
    ties inside one milli bucket) for scales >= 4, integers / milli otherwise; the oracle's
    copy spells each value with its own fewest decimal places."""
    M = len(scales)
    v = np.zeros((M, N), np.int64)
    for m, k in enumerate(scales):
        step = 10**max(k - 4, 0) if k >= 4 else 1
        v[m] = rng.integers(-10**7, 10**7, N) * step if k >= 4 else \
            rng.integers(-10**(3 + k), 10**(3 + k), N)
        v[m, rng.random(N) < 0.05] = 0
        v[m, rng.random(N) < 0.05] = 10**k * rng.integers(-3, 4)  # integer values: Equals hits
    pres_b = rng.random((M, N)) < 0.99
    u = v.copy()
    s = np.repeat(np.array(scales, np.int8)[:, None], N, 1)
    for _ in range(9):  # fewest places per value (trailing zeros stripped)
        z = (u % 10 == 0) & (s > 0)
        u = np.where(z, u // 10, u)
        s = np.where(z, s - 1, s).astype(np.int8)
    return v, pack_bits(pres_b), u, s


# values in [-1000, 1000]: LessThan / GreaterThan rules near the ends hit few nodes, Equals
# rules hit the integer values
RANDOM_TARGETS = {0: [-999, -998, -1000, -990], 1: [999, 998, 1000, 990], 2: list(range(-3, 4))}


@pytest.mark.parametrize("N", [4097, 70_001])
def test_random_scaled_columns(ctx, oracle, N):
    rng = np.random.default_rng(N)
    scales = [0, 3, 4, 5, 6, 7, 8, 9]
    v, pres, u, s = scaled_snapshot(rng, N, scales)
    gen = 9200 + N % 97
    ctx.tas_snapshot_set(gen, v, pres, scales)
    rules, off, prio = rule_batch(rng, len(scales), 64, 15, RANDOM_TARGETS)
    cand = wl.pack_bits(rng.random((64, N)) < 0.9)
    gp, go, gl = ctx.tas_eval(gen, rules, off, prio, cand)
    op_, oo, ol = oracle.tas_eval(u, pres, rules, off, prio, cand, v_scale=s)
    np.testing.assert_array_equal(gp, op_)
    np.testing.assert_array_equal(gl, ol)
    for p in range(len(gl)):
        np.testing.assert_array_equal(go[p, : gl[p]], oo[p, : ol[p]], err_msg=f"pod {p}")
    # deschedule, fused and unfused
    dr, doff, _ = rule_batch(rng, len(scales), 16, 4, RANDOM_TARGETS)
    want_v = oracle.tas_violations(u, pres, dr, doff, v_scale=s)
    labels = wl.pack_bits(rng.random((16, N)) < 0.3)
    f, sep = _fused_and_separate(ctx, gen, N, 16, dr, doff, labels)
    np.testing.assert_array_equal(f[0], want_v)
    np.testing.assert_array_equal(sep[0], want_v)
    want = oracle.label_plan(want_v, labels, N)
    for i in (1, 2):
        np.testing.assert_array_equal(f[i], want[i - 1])
    assert f[3] == sep[3] == want[2]
    # C5 records on one shard: the first k of each pod's list
    k = 16
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    key = torch.empty((64, k), dtype=torch.int64, device="cuda")
    node = torch.empty((64, k), dtype=torch.int32, device="cuda")
    ln = torch.empty(64, dtype=torch.int32, device="cuda")
    ctx.tas_topk_device(gen, 64, len(rules), dev(rules.view(np.uint8)), dev(off),
                        dev(prio.view(np.uint8)), dev(cand.view(np.int64)), k, 0, key, node, ln)
    ctx.synchronize()
    got_n, got_l = node.cpu().numpy(), ln.cpu().numpy()
    for p in range(64):
        m = min(k, int(ol[p]))
        assert got_l[p] == m
        np.testing.assert_array_equal(got_n[p, :m], oo[p, :m])


def test_scale_errors(ctx):
    v = np.zeros((2, 10), np.int64)
    pres = pack_bits(np.ones((2, 10), bool))
    ctx.tas_snapshot_set(9300, v, pres)
    for bad in ([3], [3, 10], [-1, 3]):
        with pytest.raises(pas_amd.PasError) as e:
            ctx.tas_snapshot_set_scale(9300, bad)
        assert e.value.code == pas_amd._lib.PAS_EINVAL
    with pytest.raises(pas_amd.PasError) as e:
        ctx.tas_snapshot_set_scale(9301, [3, 3])
    assert e.value.code == pas_amd._lib.PAS_ESTALE


def test_deschedule_1m_scaled(ctx, oracle):
    """C4 shape (1M nodes x 16 strategies x 4 rules) over sub-milli columns."""
    rng = np.random.default_rng(0xC4D)
    N = 1_000_000
    scales = [4, 9, 6, 3, 7, 5, 8, 0]
    v, pres, u, s = scaled_snapshot(rng, N, scales)
    ctx.tas_snapshot_set(9400, v, pres, scales)
    dr, doff, _ = rule_batch(rng, len(scales), 16, 4, RANDOM_TARGETS)
    want_v = oracle.tas_violations(u, pres, dr, doff, v_scale=s)
    f, sep = _fused_and_separate(ctx, 9400, N, 16, dr, doff, None)
    np.testing.assert_array_equal(f[0], want_v)
    want = oracle.label_plan(want_v, None, N)
    np.testing.assert_array_equal(f[1], want[0])
    assert f[3] == sep[3] == want[2]
