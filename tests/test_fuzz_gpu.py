"""Seeded random shapes through the HIP path, bit-exact against the oracle: a bounded slice of
the sweeps in scripts/diag/{tas,gas,c5}_fuzz.py (whose full runs are in
profiles/r06_fuzz_summary.txt).  Marked gpu."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "scripts", "diag"))
import c5_fuzz  # noqa: E402
import gas_fuzz  # noqa: E402
import tas_fuzz  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed0", [70_001, 70_101])
def test_tas_fuzz_slice(ctx, oracle, seed0):
    for seed in range(seed0, seed0 + 40):
        rng = np.random.default_rng(seed)
        meta, v, pres, scales, rules, off, prio, cand, flags = tas_fuzz.case(rng)
        u, s = tas_fuzz.oracle_scale(v, scales)
        ctx.tas_snapshot_set(seed, v, pres, [int(k) for k in scales])
        gp, go, gl = ctx.tas_eval(seed, rules, off, prio, cand, flags)
        op_, oo, ol = oracle.tas_eval(u, pres, rules, off, prio, cand, flags, v_scale=s)
        if flags & 1:
            np.testing.assert_array_equal(gp, op_, err_msg=str(meta))
        if flags & 2:
            np.testing.assert_array_equal(gl, ol, err_msg=str(meta))
            for q in range(len(gl)):
                np.testing.assert_array_equal(go[q, : gl[q]], oo[q, : ol[q]], err_msg=str(meta))
        np.testing.assert_array_equal(ctx.tas_violations(seed, rules, off),
                                      oracle.tas_violations(u, pres, rules, off, v_scale=s),
                                      err_msg=str(meta))


@pytest.mark.parametrize("seed0", [80_001, 80_201])
def test_gas_fuzz_slice(ctx, oracle, seed0):
    for seed in range(seed0, seed0 + 150):
        meta, args = gas_fuzz.case(np.random.default_rng(seed))
        ctx.gas_snapshot_set(seed, *args[:3])
        got = ctx.gas_fit(seed, *args[3:], meta["i915"])
        np.testing.assert_array_equal(got, oracle.gas_fit(*args, meta["i915"]), err_msg=str(meta))


def test_c5_fuzz_slice(ctx, oracle):
    for seed in range(90_001, 90_041):
        rng = np.random.default_rng(seed)
        meta, v, pres, scales, rules, off, prio, cand, _ = tas_fuzz.case(rng)
        n, P = v.shape[1], len(prio)
        gmeta, (n_cards, cap, used, req, mask, ncont) = gas_fuzz.case(rng, n=n, p=P)
        mask = mask | np.where(rng.random(mask.shape) < 0.05, 0x80000000, 0).astype(np.uint32)
        k = int(rng.choice([1, 5, 16, 70, 300]))
        base = int(rng.choice([0, 1234]))
        u, s = tas_fuzz.oracle_scale(v, scales)
        ctx.tas_snapshot_set(2 * seed, v, pres, [int(x) for x in scales])
        ctx.gas_snapshot_set(2 * seed + 1, n_cards, cap, used)
        dev = c5_fuzz.dev
        key = torch.empty((P, k), dtype=torch.int64, device="cuda")
        node = torch.empty((P, k), dtype=torch.int32, device="cuda")
        ln = torch.empty(P, dtype=torch.int32, device="cuda")
        ctx.tas_gas_topk_device(2 * seed, 2 * seed + 1, P, len(rules),
                                dev(rules.view(np.uint8)) if rules.size else None, dev(off),
                                dev(prio.view(np.uint8)),
                                None if cand is None else dev(cand.view(np.int64)),
                                req.shape[1], gmeta["i915"], dev(req), dev(mask.view(np.int32)),
                                dev(ncont), k, base, key, node, ln)
        ctx.synchronize()
        want = c5_fuzz.expected(v, u, s, pres, rules, off, prio, cand,
                                (n_cards, cap, used, req, mask, ncont), gmeta["i915"], k, base)
        for g, w in zip((key, node, ln), want):
            np.testing.assert_array_equal(g.cpu().numpy(), w, err_msg=f"{meta} {gmeta} k {k}")
