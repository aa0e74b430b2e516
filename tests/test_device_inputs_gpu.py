"""Malformed device inputs the host cannot check (the _device entry points take HBM arrays):
a rule_off that is not a CSR over [0, n_rules] (negative, past n_rules, decreasing) and
n_containers outside [0, max_containers].  The kernels clamp them where they read them
(rule_span in tas_eval.hip, tas_gas_topk.hip; n_containers as gas_prep_kernel), so no access
leaves the arrays; these tests pin the clamped reading against the oracle and check that the
context stays exact afterwards.  Marked gpu."""
import os
import sys

import numpy as np
import pytest
import torch

import pas_amd
from pas_amd import workload as wl
from test_tas_gpu import random_case

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "scripts", "diag"))


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def per_pod_clamp(off, n_rules):
    """The eval / C5 reading: pod p owns [a, b) with a = clamp(off[p], 0, n), b = clamp(off[p+1],
    a, n); returned as (rules index list per pod)."""
    spans = []
    for p in range(len(off) - 1):
        a = min(max(int(off[p]), 0), n_rules)
        b = min(max(int(off[p + 1]), a), n_rules)
        spans.append((a, b))
    return spans


def csr_from_spans(rules, spans):
    idx = [i for a, b in spans for i in range(a, b)]
    off = np.zeros(len(spans) + 1, np.int32)
    off[1:] = np.cumsum([b - a for a, b in spans])
    return rules[np.array(idx, np.int64)] if idx else rules[:0], off


def sweep_clamp(off, n_rules):
    """The deschedule sweep's reading: offsets walked in order, clamped into [r_begin, r_end]
    and non-decreasing."""
    S = len(off) - 1
    rb = min(max(int(off[0]), 0), n_rules)
    re_ = min(max(int(off[S]), rb), n_rules)
    e = [rb]
    for k in range(1, S):
        e.append(min(max(int(off[k]), e[-1]), re_))
    e.append(re_ if S > 0 else rb)
    return [(e[s], e[s + 1]) for s in range(S)]


def bad_offsets(rng, n_pods, n_rules):
    off = np.sort(rng.integers(0, n_rules + 1, size=n_pods + 1)).astype(np.int32)
    off[0] = 0
    off[-1] = n_rules
    k = rng.choice(n_pods + 1, size=max(3, n_pods // 4), replace=False)
    off[k] = rng.choice([-7, -1, n_rules + 1, n_rules + 1000, 2**31 - 1, -2**31], size=len(k))
    # and a decreasing stretch
    i = int(rng.integers(1, n_pods))
    off[i], off[i - 1] = min(int(off[i - 1]), int(off[i])) - 3, max(int(off[i - 1]), 5)
    return off


def test_eval_device_malformed_rule_off(ctx, oracle):
    rng = np.random.default_rng(0xBAD0)
    v, pres, rules, off, prio, cand = random_case(rng, 3000, 5, 40, 12, cand_frac=0.9)
    n = v.shape[1]
    ctx.tas_snapshot_set(77, v, pres)
    nr = len(rules)
    boff = bad_offsets(rng, 40, nr)
    P = 40
    W = (n + 63) // 64
    pass_t = torch.zeros((P, W), dtype=torch.int64, device="cuda")
    order_t = torch.zeros((P, n), dtype=torch.int32, device="cuda")
    len_t = torch.zeros(P, dtype=torch.int32, device="cuda")
    ctx.tas_eval_device(77, P, nr, dev(rules.view(np.uint8)), dev(boff),
                        dev(prio.view(np.uint8)), dev(cand.view(np.int64)), 3, pass_t, order_t,
                        len_t)
    ctx.synchronize()
    crules, coff = csr_from_spans(rules, per_pod_clamp(boff, nr))
    wp, wo, wl_ = oracle.tas_eval(v, pres, crules, coff, prio, cand, 3)
    np.testing.assert_array_equal(pass_t.cpu().numpy().view(np.uint64), wp)
    gl = len_t.cpu().numpy()
    np.testing.assert_array_equal(gl, wl_)
    go = order_t.cpu().numpy()
    for p in range(P):
        np.testing.assert_array_equal(go[p, : gl[p]], wo[p, : wl_[p]])
    # the context is still exact for a well-formed batch
    gp, go2, gl2 = ctx.tas_eval(77, rules, off, prio, cand, 3)
    op_, oo, ol = oracle.tas_eval(v, pres, rules, off, prio, cand, 3)
    np.testing.assert_array_equal(gp, op_)
    np.testing.assert_array_equal(gl2, ol)


@pytest.mark.parametrize("fused", [False, True])
def test_sweep_device_malformed_rule_off(ctx, oracle, fused):
    rng = np.random.default_rng(0xBAD1 + fused)
    v, pres, rules, off, _, _ = random_case(rng, 5000, 6, 12, 6)
    n = v.shape[1]
    ctx.tas_snapshot_set(78, v, pres)
    nr = len(rules)
    S = 12
    boff = bad_offsets(rng, S, nr)
    W = (n + 63) // 64
    viol_t = torch.zeros((S, W), dtype=torch.int64, device="cuda")
    if fused:
        add_t = torch.zeros(n, dtype=torch.int64, device="cuda")
        rem_t = torch.zeros(n, dtype=torch.int64, device="cuda")
        tot_t = torch.zeros(1, dtype=torch.int64, device="cuda")
        ctx.tas_deschedule_device(78, S, nr, dev(rules.view(np.uint8)), dev(boff), viol_t, None,
                                  add_t, rem_t, tot_t)
    else:
        ctx.tas_violations_device(78, S, nr, dev(rules.view(np.uint8)), dev(boff), viol_t)
    ctx.synchronize()
    crules, coff = csr_from_spans(rules, sweep_clamp(boff, nr))
    want = oracle.tas_violations(v, pres, crules, coff)
    np.testing.assert_array_equal(viol_t.cpu().numpy().view(np.uint64), want)
    np.testing.assert_array_equal(ctx.tas_violations(78, rules, off),
                                  oracle.tas_violations(v, pres, rules, off))


def test_gas_fit_device_n_containers_out_of_range(ctx, oracle):
    from test_gas_gpu import random_gas
    rng = np.random.default_rng(0xBAD2)
    n_cards, cap, used, req, mask, ncont = random_gas(rng, 900, 8, 3, 200, 4, i915=0)
    ctx.gas_snapshot_set(79, n_cards, cap, used)
    bad = ncont.copy()
    bad[::7] = -5
    bad[3::11] = 4 + 9  # past max_containers (4)
    bad[5::13] = 2**31 - 1
    P, N, C = req.shape[0], len(n_cards), req.shape[1]
    res_t = torch.zeros((P, N), dtype=torch.int32, device="cuda")
    ctx.gas_fit_device(79, P, C, 0, dev(req), dev(mask.view(np.int32)), dev(bad), res_t)
    ctx.synchronize()
    want = oracle.gas_fit(n_cards, cap, used, req, mask, np.clip(bad, 0, C).astype(np.int32), 0)
    np.testing.assert_array_equal(res_t.cpu().numpy().view(np.uint32), want)
    np.testing.assert_array_equal(ctx.gas_fit(79, req, mask, ncont, 0),
                                  oracle.gas_fit(n_cards, cap, used, req, mask, ncont, 0))


def test_c5_device_malformed_inputs(ctx, oracle):
    import c5_fuzz
    from test_gas_gpu import random_gas
    rng = np.random.default_rng(0xBAD3)
    v, pres, rules, off, prio, cand = random_case(rng, 2000, 4, 30, 8, cand_frac=0.9)
    n, P = v.shape[1], 30
    n_cards, cap, used, req, mask, ncont = random_gas(rng, n, 8, 3, P, 4, i915=0)
    cap *= 4
    nr = len(rules)
    boff = bad_offsets(rng, P, nr)
    bad_nc = ncont.copy()
    bad_nc[::5] = 99
    bad_nc[1::7] = -2
    ctx.tas_snapshot_set(80, v, pres)
    ctx.gas_snapshot_set(81, n_cards, cap, used)
    k = 16
    key = torch.empty((P, k), dtype=torch.int64, device="cuda")
    node = torch.empty((P, k), dtype=torch.int32, device="cuda")
    ln = torch.empty(P, dtype=torch.int32, device="cuda")
    ctx.tas_gas_topk_device(80, 81, P, nr, dev(rules.view(np.uint8)), dev(boff),
                            dev(prio.view(np.uint8)), dev(cand.view(np.int64)), req.shape[1], 0,
                            dev(req), dev(mask.view(np.int32)), dev(bad_nc), k, 0, key, node, ln)
    ctx.synchronize()
    crules, coff = csr_from_spans(rules, per_pod_clamp(boff, nr))
    gas = (n_cards, cap, used, req, mask, np.clip(bad_nc, 0, req.shape[1]).astype(np.int32))
    want = c5_fuzz.expected(v, v, np.zeros_like(v, dtype=np.int8) + 3, pres, crules, coff, prio,
                            cand, gas, 0, k, 0)
    for g, w in zip((key, node, ln), want):
        np.testing.assert_array_equal(g.cpu().numpy(), w)


def test_gas_snapshot_device_card_count_past_max(ctx, oracle):
    """A device n_cards past max_cards is stored as max_cards (the host form's PAS_EINVAL case):
    every node's word is the oracle's on the clamped count."""
    from test_gas_gpu import random_gas
    rng = np.random.default_rng(0xBAD4)
    for k in (3, 8, 12):
        n_cards, cap, used, req, mask, ncont = random_gas(rng, 700, k, 3, 60, 4, i915=0)
        bad = n_cards.copy()
        bad[::9] = k + 5
        bad[4::17] = 2**31 - 1
        ctx.gas_snapshot_set_device(82 + k, len(bad), k, 3, dev(bad), dev(cap), dev(used))
        ctx.synchronize()
        got = ctx.gas_fit(82 + k, req, mask, ncont, 0)
        want = oracle.gas_fit(np.minimum(bad, k).astype(np.int32), cap, used, req, mask, ncont, 0)
        np.testing.assert_array_equal(got, want)
