"""Column refresh of the resident TAS snapshot (pas_tas_snapshot_update; the reference's
AutoUpdatingCache.updateMetric replaces one metric's node map, cache/autoupdating.go:45-73).
After any sequence of column updates, filter / prioritize / deschedule must equal the oracle
on the updated matrix, i.e. a full rebuild.  Marked gpu."""
import numpy as np
import pytest

import pas_amd
from pas_amd import workload as wl
from test_tas_gpu import assert_same, random_case

pytestmark = pytest.mark.gpu


def _new_columns(rng, k, n, tie=False, absent=0.1):
    if tie:
        v = rng.choice(np.array([0, 1000, 2000, -1000], np.int64), size=(k, n))
    else:
        v = rng.integers(-5_000_000, 5_000_000, size=(k, n), dtype=np.int64)
    pres_b = rng.random((k, n)) >= absent
    if k > 1:
        pres_b[0] = rng.random(n) < 0.5 if n > 1 else pres_b[0]
    return v, wl.pack_bits(pres_b) if n else np.zeros((k, 0), np.uint64)


@pytest.mark.parametrize("n", [1, 63, 1000, 1025, 5000])
def test_update_matches_full_rebuild(ctx, oracle, n):
    rng = np.random.default_rng(100 + n)
    m = 7
    v, pres, rules, off, prio, cand = random_case(rng, n, m, 24, 6, cand_frac=0.8)
    gen = 5000 + n * 10
    ctx.tas_snapshot_set(gen, v, pres)
    for rnd in range(4):
        k = int(rng.integers(1, m + 1))
        cols = rng.choice(m, size=k, replace=False).astype(np.int32)
        nv, npres = _new_columns(rng, k, n, tie=rnd % 2 == 1)
        ctx.tas_snapshot_update(gen, gen + 1, cols, nv, npres)
        gen += 1
        v[cols] = nv
        pres[cols] = npres
        # the evaluation through the updated snapshot == the oracle on the new matrix
        gp, go, gl = ctx.tas_eval(gen, rules, off, prio, cand)
        op_, oo, ol = oracle.tas_eval(v, pres, rules, off, prio, cand)
        np.testing.assert_array_equal(gp, op_)
        np.testing.assert_array_equal(gl, ol)
        for p in range(len(gl)):
            np.testing.assert_array_equal(go[p, : gl[p]], oo[p, : ol[p]], err_msg=f"pod {p}")
        np.testing.assert_array_equal(ctx.tas_violations(gen, rules, off[:5]),
                                      oracle.tas_violations(v, pres, rules, off[:5]))
    assert ctx.tas_snapshot_info()[0] == gen


def test_update_all_columns_and_empty(ctx, oracle):
    rng = np.random.default_rng(7)
    n, m = 3000, 5
    v, pres, rules, off, prio, _ = random_case(rng, n, m, 16, 5)
    ctx.tas_snapshot_set(6000, v, pres)
    # every column, one of them emptied (metric dropped from the cache)
    nv, npres = _new_columns(rng, m, n)
    npres[2] = 0
    cols = np.array([4, 3, 2, 1, 0], np.int32)  # any order
    ctx.tas_snapshot_update(6000, 6001, cols, nv, npres)
    v[cols] = nv
    pres[cols] = npres
    assert_same(ctx, oracle, v, pres, rules, off, prio, None, 3)
    # no columns: only the generation moves
    gen = ctx.tas_snapshot_info()[0]
    ctx.tas_snapshot_update(gen, gen + 1, [], np.zeros((0, n), np.int64),
                            np.zeros((0, (n + 63) // 64), np.uint64))
    assert ctx.tas_snapshot_info()[0] == gen + 1


def test_update_device_form(ctx, oracle):
    import torch
    rng = np.random.default_rng(8)
    n, m = 20_000, 6
    v, pres, rules, off, prio, cand = random_case(rng, n, m, 32, 8, cand_frac=0.9)
    ctx.tas_snapshot_set(6100, v, pres)
    cols = np.array([1, 4], np.int32)
    nv, npres = _new_columns(rng, 2, n)
    dev = torch.device("cuda", 0)
    v_t = torch.from_numpy(nv).to(dev)
    p_t = torch.from_numpy(npres.view(np.int64)).to(dev)
    ctx.tas_snapshot_update_device(6100, 6101, cols, v_t, p_t)
    torch.cuda.synchronize()
    v[cols] = nv
    pres[cols] = npres
    gp, go, gl = ctx.tas_eval(6101, rules, off, prio, cand)
    op_, oo, ol = oracle.tas_eval(v, pres, rules, off, prio, cand)
    np.testing.assert_array_equal(gp, op_)
    np.testing.assert_array_equal(gl, ol)
    for p in range(len(gl)):
        np.testing.assert_array_equal(go[p, : gl[p]], oo[p, : ol[p]])


def test_update_errors(ctx):
    n, m = 100, 3
    v = np.zeros((m, n), np.int64)
    pres = wl.pack_bits(np.ones((m, n), bool))
    ctx.tas_snapshot_set(6200, v, pres)
    one_v, one_p = v[:1].copy(), pres[:1].copy()
    cases = [
        (6199, [0], pas_amd._lib.PAS_ESTALE),    # wrong base generation
        (6200, [3], pas_amd._lib.PAS_EINVAL),    # column out of range
        (6200, [-1], pas_amd._lib.PAS_EINVAL),
    ]
    for gen_from, cols, code in cases:
        with pytest.raises(pas_amd.PasError) as e:
            ctx.tas_snapshot_update(gen_from, 6300, cols, one_v, one_p)
        assert e.value.code == code, cols
    with pytest.raises(pas_amd.PasError) as e:  # duplicate columns
        ctx.tas_snapshot_update(6200, 6300, [1, 1], np.zeros((2, n), np.int64),
                                np.zeros((2, 2), np.uint64))
    assert e.value.code == pas_amd._lib.PAS_EINVAL
    assert ctx.tas_snapshot_info()[0] == 6200  # a refused update leaves the snapshot


@pytest.mark.slow
def test_update_c4_scale(ctx, oracle):
    # 1M nodes x 64 metrics resident; refresh 8 columns; the deschedule sweep must equal the
    # oracle on the refreshed matrix
    snap = wl.make_tas_snapshot(1_000_000, 64, seed=0xC4)
    rules, off = wl.make_deschedule_rules(snap, 16, 4, seed=0xC4)
    ctx.tas_snapshot_set(6400, snap.v_milli, snap.present)
    rng = np.random.default_rng(9)
    cols = rng.choice(64, size=8, replace=False).astype(np.int32)
    fresh = wl.make_tas_snapshot(1_000_000, 8, seed=0xC4 + 1)
    ctx.tas_snapshot_update(6400, 6401, cols, fresh.v_milli, fresh.present)
    v = snap.v_milli.copy()
    p = snap.present.copy()
    v[cols] = fresh.v_milli
    p[cols] = fresh.present
    np.testing.assert_array_equal(ctx.tas_violations(6401, rules, off),
                                  oracle.tas_violations(v, p, rules, off))
