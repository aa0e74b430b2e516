"""TAS filter / prioritize / deschedule through libpas.so's HIP kernels, checked bit-exact
against the CPU oracle and the reference's golden vectors.  Marked gpu."""
import numpy as np
import pytest

import pas_amd
from pas_amd import workload as wl
from helpers import NamedSnapshot, golden, unpack_bits

pytestmark = pytest.mark.gpu
G = golden()
_gen = [1000]


def upload(ctx, v_milli, present):
    _gen[0] += 1
    ctx.tas_snapshot_set(_gen[0], v_milli, present)
    return _gen[0]


def assert_same(ctx, oracle, v, pres, rules, off, prio, cand, flags):
    gen = upload(ctx, v, pres)
    gp, go, gl = ctx.tas_eval(gen, rules, off, prio, cand, flags)
    op_, oo, ol = oracle.tas_eval(v, pres, rules, off, prio, cand, flags)
    if flags & 1:
        np.testing.assert_array_equal(gp, op_)
    if flags & 2:
        np.testing.assert_array_equal(gl, ol)
        for p in range(len(gl)):
            np.testing.assert_array_equal(go[p, : gl[p]], oo[p, : ol[p]], err_msg=f"pod {p}")


# ---------------------------------------------------------------- golden vectors

def _gpu_filter(ctx, snap, named_rules, nodes):
    gen = upload(ctx, snap.v_milli, snap.present)
    rules = snap.rules(named_rules)
    off = np.array([0, len(rules)], np.int32)
    pass_out, _, _ = ctx.tas_eval(gen, rules, off, snap.rules([["", "LessThan", 0]]),
                                  snap.cand(nodes), pas_amd.PAS_TAS_FILTER)
    passed = unpack_bits(pass_out, len(snap.nodes))[0]
    return [n for n in nodes if passed[snap.node_index[n]]]


def _gpu_prioritize(ctx, snap, named_rule, nodes):
    gen = upload(ctx, snap.v_milli, snap.present)
    _, order, lens = ctx.tas_eval(gen, snap.rules([]), np.zeros(2, np.int32),
                                  snap.rules([named_rule]), snap.cand(nodes),
                                  pas_amd.PAS_TAS_PRIORITIZE)
    return snap.names(order[0, : lens[0]])


def _gpu_violated(ctx, snap, named_rules):
    gen = upload(ctx, snap.v_milli, snap.present)
    rules = snap.rules(named_rules)
    viol = ctx.tas_violations(gen, rules, np.array([0, len(rules)], np.int32))
    return sorted(snap.names(np.nonzero(unpack_bits(viol, len(snap.nodes))[0])[0]))


def test_golden_g2_ordered_list(ctx):
    g = G["G2_ordered_list"]
    snap = NamedSnapshot({"m": dict(zip(g["nodes"], g["values"]))})
    for c in g["cases"]:
        assert _gpu_prioritize(ctx, snap, ["m", c["operator"], 0], g["nodes"]) == c["want"]


def test_golden_g3_g4_violated(ctx):
    for key in ("G3_violated", "G4_deschedule_enforce"):
        g = G[key]
        snap = NamedSnapshot(g["metrics"], g.get("nodes", ()))
        for c in g["cases"]:
            assert _gpu_violated(ctx, snap, c["rules"]) == sorted(c["want"]), c["name"]
            # the same rules as a dontschedule filter over every node
            passed = _gpu_filter(ctx, snap, c["rules"], snap.nodes)
            assert sorted(set(snap.nodes) - set(passed)) == sorted(c["want"]), c["name"]


def test_golden_g5_g6_prioritize(ctx):
    g = G["G5_prioritize"]
    snap = NamedSnapshot(g["metrics"], g["nodes"])
    order = _gpu_prioritize(ctx, snap, g["policy"]["scheduleonmetric"][0], g["nodes"])
    assert [[h, 10 - i] for i, h in enumerate(order)] == g["want"]
    for c in G["G6_prioritize_errors"]["cases"]:
        if c.get("decode_error") or not c["policy_cached"]:
            continue
        snap = NamedSnapshot(c["metrics"], c["nodes"])
        order = _gpu_prioritize(ctx, snap, ["dummyMetric1", "GreaterThan", 0], c["nodes"])
        assert [[h, 10 - i] for i, h in enumerate(order)] == c["want"]
    # metric not in the cache -> empty list (telemetryscheduler.go:130-133, 92-96)
    assert _gpu_prioritize(ctx, snap, ["nope", "GreaterThan", 0], snap.nodes) == []


def test_golden_g7_filter(ctx):
    g = G["G7_filter"]
    for c in g["cases"]:
        snap = NamedSnapshot(c["metrics"], g["nodes"])
        passed = _gpu_filter(ctx, snap, g["policy"]["dontschedule"], g["nodes"])
        assert [n for n in g["nodes"] if n not in passed] == c["want_failed"]
        assert passed == c["want_passed"]


def test_golden_g8_e2e(ctx):
    g = G["G8_e2e"]
    snap = NamedSnapshot(g["metrics"], g["nodes"])
    for c in g["filter_cases"]:
        assert _gpu_filter(ctx, snap, c["dontschedule"], g["nodes"]) == c["want_pass"]
    for c in g["prioritize_cases"]:
        feasible = _gpu_filter(ctx, snap, c["dontschedule"], g["nodes"])
        order = _gpu_prioritize(ctx, snap, c["scheduleonmetric"][0], feasible)
        assert [[h, 10 - i] for i, h in enumerate(order)] == c["want_derived"]
        # fused filter + prioritize in one call gives the same list
        gen = upload(ctx, snap.v_milli, snap.present)
        rules = snap.rules(c["dontschedule"])
        _, o2, l2 = ctx.tas_eval(gen, rules, np.array([0, len(rules)], np.int32),
                                 snap.rules(c["scheduleonmetric"][:1]), snap.cand(g["nodes"]))
        assert snap.names(o2[0, : l2[0]]) == order
    for c in g["deschedule_cases"]:
        assert _gpu_violated(ctx, snap, c["rules"]) == c["want"]


# ---------------------------------------------------------------- random parity

def random_case(rng, n, m, p, r_max, absent=0.1, tie_vals=None, cand_frac=None):
    if tie_vals is None:
        v = rng.integers(-5_000_000, 5_000_000, size=(m, n), dtype=np.int64)
    else:
        v = rng.choice(np.array(tie_vals, np.int64), size=(m, n))
    pres_b = rng.random((m, n)) >= absent
    if m > 1:
        pres_b[m - 1] = False  # one metric "not in the cache"
    pres = wl.pack_bits(pres_b)
    n_r = rng.integers(0, r_max + 1, size=p)
    off = np.zeros(p + 1, np.int32)
    off[1:] = np.cumsum(n_r)
    nr = int(off[-1])
    rules = np.zeros(nr, pas_amd.RULE_DTYPE)
    rules["metric"] = rng.integers(-1, m + 1, size=nr)  # includes missing metrics
    rules["op"] = rng.integers(0, 3, size=nr)
    # targets around the values (milli/1000), plus saturating extremes
    t = rng.integers(-5_000, 5_000, size=nr)
    ext = rng.random(nr)
    t = np.where(ext < 0.03, np.int64(2**62), t)
    t = np.where((ext >= 0.03) & (ext < 0.06), np.int64(-2**62), t)
    if tie_vals is not None:
        t = np.where(ext > 0.5, rng.choice(np.array(tie_vals) // 1000, size=nr), t)
    rules["target"] = t
    prio = np.zeros(p, pas_amd.RULE_DTYPE)
    prio["metric"] = rng.integers(-1, m + 1, size=p)
    prio["op"] = rng.integers(0, 4, size=p)  # 3 = another operator string: unsorted branch
    cand = None
    if cand_frac is not None:
        cand = wl.pack_bits(rng.random((p, n)) < cand_frac)
    return v, pres, rules, off, prio, cand


@pytest.mark.parametrize("n", [1, 31, 32, 33, 63, 64, 65, 127, 1000, 4097])
@pytest.mark.parametrize("flags", [1, 2, 3])
def test_random_parity_shapes(ctx, oracle, n, flags):
    rng = np.random.default_rng(n * 10 + flags)
    for cand_frac in (None, 0.7):
        v, pres, rules, off, prio, cand = random_case(rng, n, 4, 9, 5, cand_frac=cand_frac)
        assert_same(ctx, oracle, v, pres, rules, off, prio, cand, flags)


@pytest.mark.parametrize("seed", range(6))
def test_random_parity_ties_and_dense_violations(ctx, oracle, seed):
    rng = np.random.default_rng(100 + seed)
    # few distinct values -> large tie groups and rules violated by most nodes
    v, pres, rules, off, prio, cand = random_case(
        rng, 3000, 5, 24, 70, tie_vals=[0, 1000, 2000, 2500, 7000, -1000],
        cand_frac=0.9 if seed % 2 else None)
    assert_same(ctx, oracle, v, pres, rules, off, prio, cand, 3)


@pytest.mark.parametrize("p", [1024, 1101])
def test_random_parity_large_batches(ctx, oracle, p):
    """Batches of ~1k pods over few metrics: large buckets (hundreds of pods per order
    column, so many 16-pod emit rounds per segment), with and without candidate masks."""
    rng = np.random.default_rng(p)
    for cand_frac in (None, 0.8):
        v, pres, rules, off, prio, cand = random_case(
            rng, 2000, 3, p, 6, tie_vals=[0, 1000, 2000, 3000, -4000] if cand_frac else None,
            cand_frac=cand_frac)
        assert_same(ctx, oracle, v, pres, rules, off, prio, cand, 3)
        assert_same(ctx, oracle, v, pres, rules, off, prio, cand, 2)


@pytest.mark.parametrize("seed", [0, 1])
def test_random_parity_flags_candidates_ties(ctx, oracle, seed):
    """Filter only, prioritize only (candidates = cand) and both, with candidate masks and
    tie-heavy columns."""
    rng = np.random.default_rng(500 + seed)
    for n, cand_frac, ties in ((777, None, None), (2048, 0.8, None),
                               (3001, 0.9, [0, 1000, 2000, -3000])):
        v, pres, rules, off, prio, cand = random_case(rng, n, 5, 40, 12, tie_vals=ties,
                                                      cand_frac=cand_frac)
        for flags in (1, 2, 3):
            assert_same(ctx, oracle, v, pres, rules, off, prio, cand, flags)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1023, 1024, 1025, 2047, 2048, 4096, 4097])
def test_segment_boundaries(ctx, oracle, n):
    """Node counts around the 64-node words and the 1024-position order segments (the
    padded order rows end in a sentinel segment)."""
    rng = np.random.default_rng(n)
    v, pres, rules, off, prio, cand = random_case(rng, n, 4, 24, 6, cand_frac=0.9)
    for flags in (2, 3):
        assert_same(ctx, oracle, v, pres, rules, off, prio, cand, flags)
    v, pres, rules, off, prio, _ = random_case(rng, n, 4, 24, 6)
    assert_same(ctx, oracle, v, pres, rules, off, prio, None, 3)


def test_many_rules_per_pod_chunked(ctx, oracle):
    # more than the kernel's 64-rule LDS chunk
    rng = np.random.default_rng(7)
    v, pres, rules, off, prio, cand = random_case(rng, 5000, 6, 4, 200)
    off = np.array([0, 150, 151, 151, len(rules)], np.int32)
    assert_same(ctx, oracle, v, pres, rules, off, prio, cand, 3)


def test_all_absent_and_empty(ctx, oracle):
    n, m = 700, 3
    v = np.zeros((m, n), np.int64)
    pres = wl.pack_bits(np.zeros((m, n), bool))
    rules = pas_amd.make_rules([0, 1, 2], [0, 1, 2], [1, 1, 1])
    off = np.array([0, 3, 3], np.int32)
    prio = pas_amd.make_rules([0, 1], [1, 0], [0, 0])
    assert_same(ctx, oracle, v, pres, rules, off, prio, None, 3)
    gen = upload(ctx, v, pres)
    p, o, l = ctx.tas_eval(gen, rules, off, prio)
    assert (l == 0).all()
    assert (unpack_bits(p, n) == True).all()  # noqa: E712 - nothing violates


def test_c1_config(ctx, oracle):
    # BASELINE.json configs[0]: 1 pod x 1k nodes x 3 rules (2 dontschedule + 1 scheduleonmetric)
    snap = wl.make_tas_snapshot(1000, 3, seed=0xC1)
    batch = wl.make_tas_batch(snap, 1, 2, seed=0xC1)
    assert_same(ctx, oracle, snap.v_milli, snap.present, batch.rules, batch.rule_off, batch.prio,
                None, 3)


@pytest.mark.slow
def test_c2_shape_pod_sample(ctx, oracle):
    # configs[1] node/metric/rule shape (100k nodes, 64 metrics, 15 + 1 rules) on 48 pods
    snap = wl.make_tas_snapshot(100_000, 64, seed=0xC2)
    batch = wl.make_tas_batch(snap, 48, 15, seed=0xC2)
    assert_same(ctx, oracle, snap.v_milli, snap.present, batch.rules, batch.rule_off, batch.prio,
                None, 3)
    cb = wl.make_tas_batch(snap, 16, 15, seed=0xC2 + 1, cand_frac=0.8)
    assert_same(ctx, oracle, snap.v_milli, snap.present, cb.rules, cb.rule_off, cb.prio, cb.cand,
                3)


def _oracle_compare_threaded(oracle, snap, batch, passed, lens, order, threads=16, chunk=16):
    """Every pod of the batch through the oracle (C restatement), pods split over host
    threads in chunks (the ctypes calls release the GIL), each chunk compared bit-exact with
    the GPU's pass rows, list lengths and ordered lists.  Returns the mismatching pods."""
    from concurrent.futures import ThreadPoolExecutor
    p = len(batch.prio)

    def run(lo):
        hi = min(p, lo + chunk)
        r0, r1 = int(batch.rule_off[lo]), int(batch.rule_off[hi])
        off = (batch.rule_off[lo: hi + 1] - r0).astype(np.int32)
        op_, oo, ol = oracle.tas_eval(snap.v_milli, snap.present, batch.rules[r0:r1], off,
                                      batch.prio[lo:hi], None, 3)
        bad = []
        for i in range(hi - lo):
            q = lo + i
            if (lens[q] != ol[i] or not np.array_equal(passed[q], op_[i])
                    or not np.array_equal(order[q, : lens[q]], oo[i, : ol[i]])):
                bad.append(q)
        return bad

    with ThreadPoolExecutor(threads) as ex:
        return [q for bad in ex.map(run, range(0, p, chunk)) for q in bad]


@pytest.mark.slow
def test_c2_full_size_properties(ctx, oracle):
    """configs[1] at full size (4096 pods x 100k nodes x 16 rules), device-resident: every
    pod's pass row, list length and whole ordered list bit-exact against the oracle (16 host
    threads, ~3 s), plus the documented order checked on the device for a pod sample."""
    import time
    import torch
    snap = wl.make_tas_snapshot(100_000, 64, seed=0xC2)
    batch = wl.make_tas_batch(snap, 4096, 15, seed=0xC2)
    n, p = 100_000, 4096
    dev = torch.device("cuda:0")
    gen = upload(ctx, snap.v_milli, snap.present)
    rules_t = torch.from_numpy(batch.rules.view(np.uint8).copy()).to(dev)
    off_t = torch.from_numpy(batch.rule_off).to(dev)
    prio_t = torch.from_numpy(batch.prio.view(np.uint8).copy()).to(dev)
    pass_t = torch.empty((p, pas_amd.w64(n)), dtype=torch.int64, device=dev)
    order_t = torch.empty((p, n), dtype=torch.int32, device=dev)
    len_t = torch.empty(p, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    ctx.tas_eval_device(gen, p, len(batch.rules), rules_t, off_t, prio_t, None, 3, pass_t,
                        order_t, len_t, s)
    torch.cuda.synchronize()
    lens = len_t.cpu().numpy()
    passed = pass_t.cpu().numpy().view(np.uint64)
    order = order_t.cpu().numpy()  # 1.6 GB
    t0 = time.perf_counter()
    bad = _oracle_compare_threaded(oracle, snap, batch, passed, lens, order)
    print(f"C2 full batch vs oracle: {p} pods in {time.perf_counter() - t0:.1f} s, "
          f"sum of list lengths {int(lens.sum())}")
    assert not bad, f"{len(bad)} of {p} pods differ from the oracle (first {bad[:8]})"
    del order
    # the documented order on the device, independent of the oracle
    vals = torch.from_numpy(snap.v_milli).to(dev)
    pres_b = torch.from_numpy(snap.present_bool).to(dev)
    pass_b = torch.from_numpy(unpack_bits(passed, n)).to(dev)
    m0 = torch.from_numpy(batch.prio["metric"].astype(np.int64)).to(dev)
    ops = batch.prio["op"]
    expect_len = (pass_b & pres_b[m0]).sum(dim=1).cpu().numpy()
    np.testing.assert_array_equal(lens, expect_len)
    for q in range(0, p, 16):
        L = int(lens[q])
        idx = order_t[q, :L].long()
        v = vals[m0[q]][idx]
        assert bool(pass_b[q][idx].all()) and bool(pres_b[m0[q]][idx].all())
        if ops[q] == 1:
            ok = (v[1:] < v[:-1]) | ((v[1:] == v[:-1]) & (idx[1:] > idx[:-1]))
        elif ops[q] == 0:
            ok = (v[1:] > v[:-1]) | ((v[1:] == v[:-1]) & (idx[1:] > idx[:-1]))
        else:
            ok = idx[1:] > idx[:-1]
        assert bool(ok.all()), f"pod {q} not in documented order"


@pytest.mark.parametrize("flags", [1, 2, 3])
def test_global_pass_bitmap_path(ctx, oracle, monkeypatch, flags):
    # the path for clusters past the LDS pass bitmap, forced at small sizes: the same
    # results with the bitmaps in global scratch (PAS_EVAL_GLOBAL_PASS)
    monkeypatch.setenv("PAS_EVAL_GLOBAL_PASS", "1")
    rng = np.random.default_rng(70 + flags)
    for n in (1, 65, 1025, 5000):
        for cand_frac in (None, 0.6):
            v, pres, rules, off, prio, cand = random_case(rng, n, 4, 7, 5, cand_frac=cand_frac)
            assert_same(ctx, oracle, v, pres, rules, off, prio, cand, flags)


@pytest.mark.slow
def test_cluster_past_lds_bitmap(ctx, oracle):
    # 1.3M nodes: the pass bitmap no longer fits a workgroup's LDS (~1.1M nodes), so the
    # kernel keeps it in global scratch; full ordered lists, filter rows and lengths vs the
    # oracle
    rng = np.random.default_rng(13)
    v, pres, rules, off, prio, cand = random_case(rng, 1_300_000, 3, 6, 4, cand_frac=0.5)
    assert_same(ctx, oracle, v, pres, rules, off, prio, cand, 3)


def test_deschedule_parity(ctx, oracle):
    rng = np.random.default_rng(4)
    for n in (1, 64, 65, 5000):
        v, pres, rules, off, _, _ = random_case(rng, n, 5, 7, 6)
        gen = upload(ctx, v, pres)
        np.testing.assert_array_equal(ctx.tas_violations(gen, rules, off),
                                      oracle.tas_violations(v, pres, rules, off))


def test_deschedule_empty_strategies_and_skipped_rules(ctx, oracle):
    # strategies without rules (first, middle, last), rules on metrics not in the cache
    # (skipped, strategy.go:37-40), more rules than one batch of the sweep's loads
    rng = np.random.default_rng(11)
    n, m = 3000, 6
    v, pres, _, _, _, _ = random_case(rng, n, m, 1, 1)
    counts = [0, 3, 0, 0, 21, 1, 15, 0]
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    rules = np.zeros(int(off[-1]), pas_amd.RULE_DTYPE)
    rules["metric"] = rng.integers(0, m, size=len(rules))
    rules["op"] = rng.integers(0, 3, size=len(rules))
    rules["target"] = rng.integers(-5_000, 5_000, size=len(rules))
    rules["metric"][::5] = -1
    rules["metric"][2::7] = m + 3
    gen = upload(ctx, v, pres)
    got = ctx.tas_violations(gen, rules, off)
    np.testing.assert_array_equal(got, oracle.tas_violations(v, pres, rules, off))
    assert not got[[0, 2, 3, 7]].any()


@pytest.mark.slow
def test_c4_deschedule_sweep_1m(ctx, oracle):
    # configs[3] per-GPU work at full node count: 1M nodes x 64 metrics, 16 strategies x 4 rules
    snap = wl.make_tas_snapshot(1_000_000, 64, seed=0xC4)
    rules, off = wl.make_deschedule_rules(snap, 16, 4, seed=0xC4)
    gen = upload(ctx, snap.v_milli, snap.present)
    got = ctx.tas_violations(gen, rules, off)
    np.testing.assert_array_equal(got, oracle.tas_violations(snap.v_milli, snap.present, rules,
                                                             off))
    frac = unpack_bits(got, 1_000_000).mean()
    assert 0.005 < frac < 0.05  # ~4 rules x 0.5 % per strategy


# ---------------------------------------------------------------- error paths

def test_errors(ctx):
    n, m = 100, 2
    v = np.zeros((m, n), np.int64)
    pres = wl.pack_bits(np.ones((m, n), bool))
    gen = upload(ctx, v, pres)
    prio = pas_amd.make_rules([0], [1], [0])
    with pytest.raises(pas_amd.PasError) as e:
        ctx.tas_eval(gen + 1, pas_amd.make_rules([0], [0], [1]), np.array([0, 1], np.int32), prio)
    assert e.value.code == -2  # PAS_ESTALE
    # unknown operator on a cached metric: the reference panics (operator.go:25) -> EINVAL
    with pytest.raises(pas_amd.PasError) as e:
        ctx.tas_eval(gen, pas_amd.make_rules([0], [9], [1]), np.array([0, 1], np.int32), prio)
    assert e.value.code == -1
    # ... but on a metric missing from the cache the rule is skipped first (strategy.go:28-32)
    p, _, _ = ctx.tas_eval(gen, pas_amd.make_rules([-1], [9], [1]), np.array([0, 1], np.int32),
                           prio)
    assert unpack_bits(p, n).all()
    with pytest.raises(pas_amd.PasError) as e:
        ctx.tas_eval(gen, pas_amd.make_rules([0], [0], [1]), np.array([1, 1], np.int32), prio)
    assert e.value.code == -1


def test_unknown_operator_on_empty_metric_map(ctx, oracle):
    """A cached metric with no node entries: Violated ranges over an empty map, so
    EvaluateRule (and its panic on an unknown operator, operator.go:25) never runs."""
    n = 300
    v = np.arange(2 * n, dtype=np.int64).reshape(2, n) * 1000
    present = np.ones((2, n), bool)
    present[1] = False
    pres = wl.pack_bits(present)
    gen = upload(ctx, v, pres)
    rules = pas_amd.make_rules([1, 0], [9, 1], [0, 100])
    off = np.array([0, 2], np.int32)
    prio = pas_amd.make_rules([0], [0], [0])
    got = ctx.tas_eval(gen, rules, off, prio)
    want = oracle.tas_eval(v, pres, rules, off, prio, None, 3)
    np.testing.assert_array_equal(got[0], want[0])
    np.testing.assert_array_equal(got[2], want[2])
    np.testing.assert_array_equal(got[1][0, :got[2][0]], want[1][0, :want[2][0]])


def test_evals_pipelined_on_streams(oracle):
    """Batches issued on three streams in turn without host synchronisation (bench.py
    --pipeline): each stream's calls take their own scratch slot, so consecutive batches
    overlap; every batch's pass rows, lengths and ordered lists equal the oracle's."""
    import torch
    snap = wl.make_tas_snapshot(3000, 8, seed=0x71)
    batches = [wl.make_tas_batch(snap, p, 6, seed=0x71 + i, cand_frac=0.8)
               for i, p in enumerate((300, 77, 513, 300))]
    c = pas_amd.Context(0)
    try:
        s0 = torch.cuda.current_stream()
        c.tas_snapshot_set_device(5, 3000, 8, torch.from_numpy(snap.v_milli).cuda(),
                                  torch.from_numpy(snap.present.view(np.int64)).cuda(), s0)
        streams = [torch.cuda.Stream() for _ in range(3)]
        for st in streams:
            st.wait_stream(s0)
        flags = pas_amd.PAS_TAS_FILTER | pas_amd.PAS_TAS_PRIORITIZE
        outs = []
        for rep in range(2):
            for i, b in enumerate(batches):
                st = streams[(rep * len(batches) + i) % 3]
                with torch.cuda.stream(st):
                    t = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in
                         (b.rules.view(np.uint8), b.rule_off, b.prio.view(np.uint8),
                          b.cand.view(np.int64))]
                    P = len(b.prio)
                    pt = torch.empty((P, pas_amd.w64(3000)), dtype=torch.int64, device="cuda")
                    ot = torch.empty((P, 3000), dtype=torch.int32, device="cuda")
                    lt = torch.empty(P, dtype=torch.int32, device="cuda")
                c.tas_eval_device(5, P, len(b.rules), t[0], t[1], t[2], t[3], flags, pt, ot, lt,
                                  st)
                outs.append((i, t, pt, ot, lt))
        torch.cuda.synchronize()
        for i, _, pt, ot, lt in outs:
            b = batches[i]
            wp, wo, wl_ = oracle.tas_eval(snap.v_milli, snap.present, b.rules, b.rule_off, b.prio,
                                          b.cand, 3)
            np.testing.assert_array_equal(pt.cpu().numpy().view(np.uint64), wp)
            gl = lt.cpu().numpy()
            np.testing.assert_array_equal(gl, wl_)
            go = ot.cpu().numpy()
            for p in range(len(gl)):
                np.testing.assert_array_equal(go[p, :gl[p]], wo[p, :gl[p]])
    finally:
        c.close()
