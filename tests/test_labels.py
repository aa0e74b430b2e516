"""Deschedule label plan and patch body (Deschedule.updateNodeLabels / patchNode,
deschedule/enforce.go:74-151).  The JSON encoder is host code in libpas.so and runs on CPU;
the plan kernel is checked on the GPU, bit-exact against the oracle, end to end from the
sweep (pas_tas_violations) through the plan to the patched labels."""
import json

import numpy as np
import pytest

import pas_amd
from pas_amd import workload as wl
from helpers import golden, unpack_bits
from test_oracle_golden import apply_label_patch

G = golden()


def random_names(rng, s):
    alphabet = list("abcdefghij-.") + ["<", ">", "&", '"', "\\", "\n", "\t", "\x01", "/"]
    return ["p%d-" % i + "".join(rng.choice(alphabet, size=rng.integers(0, 12))) for i in range(s)]


# ---------------------------------------------------------------- host JSON (CPU)

def test_patch_json_matches_oracle(oracle):
    rng = np.random.default_rng(11)
    for s in (0, 1, 2, 7, 63, 64):
        names = random_names(rng, s)
        live = (1 << s) - 1
        for _ in range(20):
            add = int(rng.integers(0, 1 << 62, dtype=np.int64)) & live
            rem = int(rng.integers(0, 1 << 62, dtype=np.int64)) & live & ~add
            got = pas_amd.label_patch_json(names, add, rem)
            assert got == oracle.label_patch_json(names, add, rem)
            ops = json.loads(got)  # valid JSON whose strings decode to the names
            n_add = bin(add).count("1")
            assert len(ops) == n_add + 2 * bin(rem).count("1")
            want = [("add", names[i], "violating") for i in range(s) if add >> i & 1]
            for i in range(s):
                if rem >> i & 1:
                    want += [("remove", names[i], ""), ("add", names[i], "null")]
            assert [(o["op"], o["path"][len("/metadata/labels/"):], o["value"]) for o in ops] \
                == want


def test_patch_json_go_encoding():
    # encoding/json escapes <, >, & and control bytes as \u00XX (HTML-safe by default)
    got = pas_amd.label_patch_json(["a<b>&c\x1f"], 1, 0)
    assert got == (b'[{"op":"add","path":"/metadata/labels/a\\u003cb\\u003e\\u0026c\\u001f",'
                   b'"value":"violating"}]')
    assert pas_amd.label_patch_json(["x"], 0, 0) == b"[]"  # payload := []patchValue{}


def test_patch_json_capacity_and_errors():
    lib = pas_amd.LIB
    import ctypes
    names = (ctypes.c_char_p * 2)(b"alpha", b"beta")
    n = ctypes.c_int64()
    buf = ctypes.create_string_buffer(8)
    assert lib.pas_label_patch_json(2, names, 3, 0, buf, 8, ctypes.byref(n)) == \
        pas_amd._lib.PAS_ECAPACITY
    full = n.value
    buf = ctypes.create_string_buffer(full)
    assert lib.pas_label_patch_json(2, names, 3, 0, buf, full, ctypes.byref(n)) == 0
    assert n.value == full and json.loads(buf.raw)[1]["path"] == "/metadata/labels/beta"
    # mask bits past n_strategies, n_strategies > 64
    assert lib.pas_label_patch_json(2, names, 4, 0, buf, full, ctypes.byref(n)) == \
        pas_amd._lib.PAS_EINVAL
    assert lib.pas_label_patch_json(65, names, 0, 0, buf, full, ctypes.byref(n)) == \
        pas_amd._lib.PAS_EINVAL


# ---------------------------------------------------------------- plan kernel (GPU)

def _plan_case(rng, n, s, density=0.3):
    w = (n + 63) // 64
    if n == 0 or s == 0:
        return np.zeros((s, w), np.uint64), np.zeros((s, w), np.uint64)
    viol = wl.pack_bits(rng.random((s, n)) < density)
    labels = wl.pack_bits(rng.random((s, n)) < 0.5)
    assert viol.shape == (s, w)
    return viol, labels


@pytest.mark.gpu
def test_label_plan_parity(ctx, oracle):
    rng = np.random.default_rng(12)
    for n in (0, 1, 63, 64, 65, 1000, 4097):
        for s in (0, 1, 5, 64):
            viol, labels = _plan_case(rng, n, s)
            for lab in (labels, None):
                got = ctx.tas_label_plan(n, viol, lab)
                want = oracle.label_plan(viol, lab, n)
                np.testing.assert_array_equal(got[0], want[0], err_msg=f"add n={n} s={s}")
                np.testing.assert_array_equal(got[1], want[1], err_msg=f"rem n={n} s={s}")
                assert got[2] == want[2], (n, s)


@pytest.mark.gpu
def test_label_plan_golden_g4(ctx, oracle):
    # the reference's own Enforce test (enforce_test.go:38-52): sweep on the GPU, plan on
    # the GPU, patch body from libpas.so, applied to node-1's labels
    from helpers import NamedSnapshot
    g = G["G4_deschedule_enforce"]
    snap = NamedSnapshot(g["metrics"], g["nodes"])
    policy = g["policy"]
    for gen, c in enumerate(g["cases"], start=7000):
        ctx.tas_snapshot_set(gen, snap.v_milli, snap.present)
        rules = snap.rules(c["rules"])
        viol = ctx.tas_violations(gen, rules, np.array([0, len(rules)], np.int32))
        labels = np.zeros_like(viol)
        if policy in c["labels"]:
            labels[0, 0] = 1
        add, rem, total = ctx.tas_label_plan(len(g["nodes"]), viol, labels)
        assert total == c["derived"]["total"], c["name"]
        body = pas_amd.label_patch_json([policy], int(add[0]), int(rem[0]))
        assert body.decode() == c["derived"]["patch"], c["name"]
        after = apply_label_patch(c["labels"], body)
        assert [n for n in g["nodes"] if after.get(policy) == "violating"] == c["want"]


@pytest.mark.gpu
def test_label_plan_device_after_sweep(ctx, oracle):
    # device chain at configs[3] shape (1M nodes x 16 strategies): sweep -> plan, resident
    import torch
    n, s = 1_000_000, 16
    snap = wl.make_tas_snapshot(n, 64, seed=0xC4)
    rules, off = wl.make_deschedule_rules(snap, s, 4, seed=0xC4)
    gen = 7100
    ctx.tas_snapshot_set(gen, snap.v_milli, snap.present)
    dev = torch.device("cuda", 0)
    rules_t = torch.from_numpy(rules.view(np.uint8).copy()).to(dev)
    off_t = torch.from_numpy(off).to(dev)
    w = (n + 63) // 64
    viol_t = torch.empty((s, w), dtype=torch.int64, device=dev)
    ctx.tas_violations_device(gen, s, len(rules), rules_t, off_t, viol_t)
    rng = np.random.default_rng(13)
    labels = wl.pack_bits(rng.random((s, n)) < 0.1)
    labels_t = torch.from_numpy(labels.view(np.int64)).to(dev)
    add_t = torch.empty(n, dtype=torch.int64, device=dev)
    rem_t = torch.empty(n, dtype=torch.int64, device=dev)
    total_t = torch.empty(1, dtype=torch.int64, device=dev)
    ctx.tas_label_plan_device(n, s, viol_t, labels_t, add_t, rem_t, total_t)
    torch.cuda.synchronize()
    viol = viol_t.cpu().numpy().view(np.uint64)
    want = oracle.label_plan(viol, labels, n)
    np.testing.assert_array_equal(add_t.cpu().numpy().view(np.uint64), want[0])
    np.testing.assert_array_equal(rem_t.cpu().numpy().view(np.uint64), want[1])
    assert int(total_t.item()) == want[2]
    # size-independent properties: add is the column of the sweep; add & remove disjoint;
    # total = n * s - violated pairs
    a = add_t.cpu().numpy().view(np.uint64)
    assert not np.any(a & rem_t.cpu().numpy().view(np.uint64))
    assert want[2] == n * s - int(unpack_bits(viol, n).sum())
    # the fused sweep + plan at the same shape: the same bitmaps, masks and count
    f_viol_t = torch.empty_like(viol_t)
    f_add_t, f_rem_t, f_total_t = (torch.empty_like(add_t), torch.empty_like(rem_t),
                                   torch.empty_like(total_t))
    ctx.tas_deschedule_device(gen, s, len(rules), rules_t, off_t, f_viol_t, labels_t, f_add_t,
                              f_rem_t, f_total_t)
    torch.cuda.synchronize()
    assert torch.equal(f_viol_t, viol_t) and torch.equal(f_add_t, add_t)
    assert torch.equal(f_rem_t, rem_t) and torch.equal(f_total_t, total_t)


def _fused_and_separate(ctx, gen, n, s, rules, off, labels, names=None):
    """pas_tas_deschedule_device and the sweep + plan pair on the same resident inputs."""
    import torch
    dev = torch.device("cuda", 0)
    w = (n + 63) // 64
    rules_t = torch.from_numpy(rules.view(np.uint8).copy()).to(dev)
    off_t = torch.from_numpy(off).to(dev)
    labels_t = None if labels is None else torch.from_numpy(labels.view(np.int64).copy()).to(dev)
    out = {}
    for name in ("fused", "separate"):
        viol_t = torch.full((max(s, 1), max(w, 1)), -1, dtype=torch.int64, device=dev)
        add_t = torch.full((max(n, 1),), -1, dtype=torch.int64, device=dev)
        rem_t = torch.full((max(n, 1),), -1, dtype=torch.int64, device=dev)
        total_t = torch.full((1,), -7, dtype=torch.int64, device=dev)
        if name == "fused":
            ctx.tas_deschedule_device(gen, s, len(rules), rules_t, off_t, viol_t, labels_t, add_t,
                                      rem_t, total_t, names=names)
        else:
            ctx.tas_violations_device(gen, s, len(rules), rules_t, off_t, viol_t)
            ctx.tas_label_plan_device(n, s, viol_t, labels_t, add_t, rem_t, total_t, names=names)
        torch.cuda.synchronize()
        out[name] = (viol_t.cpu().numpy().view(np.uint64)[:s, :w],
                     add_t.cpu().numpy().view(np.uint64)[:n],
                     rem_t.cpu().numpy().view(np.uint64)[:n], int(total_t.item()))
    return out["fused"], out["separate"]


@pytest.mark.gpu
def test_deschedule_fused_parity(ctx, oracle):
    # the sweep with its label plan in one pass equals the two calls and the oracle, for node
    # counts off the 64-node words and the waves' 8-word runs, 1..64 strategies, with and
    # without carried labels, and strategies without rules
    rng = np.random.default_rng(14)
    gen = 7200
    for n in (1, 63, 64, 65, 511, 513, 4097, 70_001):
        snap = wl.make_tas_snapshot(n, 8, seed=n)
        ctx.tas_snapshot_set(gen, snap.v_milli, snap.present)
        for s in (1, 5, 16, 64):
            rules, off = wl.make_deschedule_rules(snap, s, 2, seed=n + s)
            if s >= 5:  # strategies 1 and 3 without rules
                cnt = np.diff(off).copy()
                cnt[1] = cnt[3] = 0
                keep = np.concatenate([np.arange(off[i], off[i] + cnt[i]) for i in range(s)])
                rules = rules[keep]
                off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int32)
            want_v = oracle.tas_violations(snap.v_milli, snap.present, rules, off)
            labels = wl.pack_bits(rng.random((s, n)) < 0.4)
            for lab in (labels, None):
                f, sep = _fused_and_separate(ctx, gen, n, s, rules, off, lab)
                np.testing.assert_array_equal(f[0], want_v, err_msg=f"viol n={n} s={s}")
                want = oracle.label_plan(want_v, lab, n)
                for i, what in ((1, "add"), (2, "rem")):
                    np.testing.assert_array_equal(f[i], want[i - 1], err_msg=f"{what} n={n} s={s}")
                    np.testing.assert_array_equal(f[i], sep[i], err_msg=f"{what} n={n} s={s}")
                assert f[3] == want[2] == sep[3], (n, s)
        gen += 1


@pytest.mark.gpu
def test_deschedule_fused_no_strategies_and_errors(ctx):
    import torch
    n = 1000
    snap = wl.make_tas_snapshot(n, 4, seed=3)
    ctx.tas_snapshot_set(7300, snap.v_milli, snap.present)
    dev = torch.device("cuda", 0)
    add_t = torch.full((n,), -1, dtype=torch.int64, device=dev)
    rem_t = torch.full((n,), -1, dtype=torch.int64, device=dev)
    total_t = torch.full((1,), -7, dtype=torch.int64, device=dev)
    off_t = torch.zeros(1, dtype=torch.int32, device=dev)
    viol_t = torch.zeros(1, dtype=torch.int64, device=dev)
    ctx.tas_deschedule_device(7300, 0, 0, None, off_t, viol_t, None, add_t, rem_t, total_t)
    torch.cuda.synchronize()
    assert not add_t.any() and not rem_t.any() and int(total_t.item()) == 0
    with pytest.raises(pas_amd.PasError) as e:  # more than 64 strategies
        ctx.tas_deschedule_device(7300, 65, 0, None, off_t, viol_t, None, add_t, rem_t, total_t)
    assert e.value.code == pas_amd._lib.PAS_EINVAL
    with pytest.raises(pas_amd.PasError) as e:  # stale generation
        ctx.tas_deschedule_device(7299, 1, 0, None, off_t, viol_t, None, add_t, rem_t, total_t)


@pytest.mark.gpu
def test_label_plan_errors(ctx):
    with pytest.raises(pas_amd.PasError) as e:
        ctx.tas_label_plan(10, np.zeros((65, 1), np.uint64))
    assert e.value.code == pas_amd._lib.PAS_EINVAL


# ---------------------------------------------------------------- shared policy names (GPU)
# updateNodeLabels keys its non-violated set by policy NAME (enforce.go:89-134): a name is
# removed / counted once, and only when none of its strategies is violated.

def random_shared_names(rng, s, pool):
    """s policy names drawn from `pool` distinct ones (repeats likely)."""
    return [f"pol-{int(i)}" for i in rng.integers(0, pool, size=s)]


def name_labels(rng, names, n, density=0.5):
    """Labels rows [S][W64] that agree within a name (the label is the node's)."""
    uniq = sorted(set(names))
    rows = {u: wl.pack_bits(rng.random((1, n)) < density)[0] for u in uniq}
    return np.stack([rows[x] for x in names]) if names else np.zeros((0, (n + 63) // 64),
                                                                      np.uint64)


@pytest.mark.gpu
def test_label_plan_golden_g4n(ctx, oracle):
    """The derived G4n cases through the GPU sweep and both plan paths (two calls, fused)."""
    from helpers import NamedSnapshot
    from test_oracle_golden import g4n_inputs
    g = G["G4n_shared_policy_name"]
    snap = NamedSnapshot(g["metrics"], g["nodes"])
    for gen, c in enumerate(g["cases"], start=7400):
        ctx.tas_snapshot_set(gen, snap.v_milli, snap.present)
        names, rules, off, viol_o, labels = g4n_inputs(oracle, c, snap, g["nodes"])
        viol = ctx.tas_violations(gen, rules, off)
        np.testing.assert_array_equal(viol, viol_o)
        add, rem, total = ctx.tas_label_plan(1, viol, labels, names)
        bits = lambda m: [j for j in range(len(names)) if int(m) >> j & 1]  # noqa: E731
        assert bits(add[0]) == c["add"] and bits(rem[0]) == c["remove"], c["name"]
        assert total == c["total"], c["name"]
        assert pas_amd.label_patch_json(names, int(add[0]), int(rem[0])).decode() == c["patch"]
        f, sep = _fused_and_separate(ctx, gen, 1, len(names), rules, off, labels, names)
        assert (int(f[1][0]), int(f[2][0]), f[3]) == (int(add[0]), int(rem[0]), total), c["name"]
        assert (int(sep[1][0]), int(sep[2][0]), sep[3]) == (int(add[0]), int(rem[0]), total)


@pytest.mark.gpu
def test_label_plan_shared_names_parity(ctx, oracle):
    """Random plans with repeated names (and rows of non-first strategies that disagree with
    their name's first row: only the first is read) equal the oracle's name-keyed plan."""
    rng = np.random.default_rng(15)
    for n in (1, 63, 64, 65, 1000, 4097):
        for s in (2, 5, 16, 33, 64):
            for pool in (1, 3, max(s // 2, 1)):
                names = random_shared_names(rng, s, pool)
                viol, _ = _plan_case(rng, n, s, density=0.05)
                labels = name_labels(rng, names, n)
                noisy = labels.copy()
                noisy[1:] ^= wl.pack_bits(rng.random((s - 1, n)) < 0.3)
                for lab in (labels, noisy, None):
                    got = ctx.tas_label_plan(n, viol, lab, names)
                    want = oracle.label_plan(viol, lab, n, names)
                    np.testing.assert_array_equal(got[0], want[0], err_msg=f"add {n} {s} {pool}")
                    np.testing.assert_array_equal(got[1], want[1], err_msg=f"rem {n} {s} {pool}")
                    assert got[2] == want[2], (n, s, pool)
                # distinct names given explicitly = names omitted
                uniq = [f"u{j}" for j in range(s)]
                a = ctx.tas_label_plan(n, viol, labels, uniq)
                b = ctx.tas_label_plan(n, viol, labels)
                assert all(np.array_equal(x, y) for x, y in zip(a[:2], b[:2])) and a[2] == b[2]


@pytest.mark.gpu
def test_deschedule_fused_shared_names_parity(ctx, oracle):
    rng = np.random.default_rng(16)
    gen = 7500
    for n in (65, 513, 70_001):
        snap = wl.make_tas_snapshot(n, 8, seed=n + 1)
        ctx.tas_snapshot_set(gen, snap.v_milli, snap.present)
        for s, pool in ((2, 1), (16, 4), (64, 9)):
            rules, off = wl.make_deschedule_rules(snap, s, 2, seed=n + s + 1)
            names = random_shared_names(rng, s, pool)
            want_v = oracle.tas_violations(snap.v_milli, snap.present, rules, off)
            labels = name_labels(rng, names, n, 0.4)
            for lab in (labels, None):
                f, sep = _fused_and_separate(ctx, gen, n, s, rules, off, lab, names)
                want = oracle.label_plan(want_v, lab, n, names)
                np.testing.assert_array_equal(f[0], want_v)
                for i, what in ((1, "add"), (2, "rem")):
                    np.testing.assert_array_equal(f[i], want[i - 1], err_msg=f"{what} {n} {s}")
                    np.testing.assert_array_equal(sep[i], want[i - 1], err_msg=f"{what} {n} {s}")
                assert f[3] == want[2] == sep[3], (n, s)
        gen += 1


@pytest.mark.gpu
def test_deschedule_shared_names_1m(ctx, oracle):
    """C4 shape (1M nodes x 16 strategies x 4 rules) with the 16 strategies under 5 policy
    names: fused and two-call plans equal the oracle; totals obey the per-name identity."""
    n, s = 1_000_000, 16
    snap = wl.make_tas_snapshot(n, 64, seed=0xC4)
    rules, off = wl.make_deschedule_rules(snap, s, 4, seed=0xC4)
    gen = 7600
    ctx.tas_snapshot_set(gen, snap.v_milli, snap.present)
    rng = np.random.default_rng(17)
    names = [f"pol-{j % 5}" for j in range(s)]
    labels = name_labels(rng, names, n, 0.1)
    f, sep = _fused_and_separate(ctx, gen, n, s, rules, off, labels, names)
    want_v = oracle.tas_violations(snap.v_milli, snap.present, rules, off)
    np.testing.assert_array_equal(f[0], want_v)
    want = oracle.label_plan(want_v, labels, n, names)
    for i in (1, 2):
        np.testing.assert_array_equal(f[i], want[i - 1])
        np.testing.assert_array_equal(sep[i], want[i - 1])
    assert f[3] == sep[3] == want[2]
    # size-independent: total = sum over names of nodes where no strategy of the name violates
    bits = unpack_bits(want_v, n)
    expect = sum(int((~bits[[j for j in range(s) if names[j] == u]].any(axis=0)).sum())
                 for u in set(names))
    assert want[2] == expect
