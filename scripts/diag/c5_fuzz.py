"""Seeded fuzz sweep of C5's combined top-k (pas_tas_gas_topk_device) against the oracle.

Expected records of pod p, from the oracle alone: the GAS fit of p on every node
(oracle.gas_fit, bit 31), ANDed with p's candidate mask, as the candidates of the TAS eval
(oracle.tas_eval: dontschedule rules, then the prioritize order); the first k entries of that
list as (key, node_base + node) with key ~v (GreaterThan), v (LessThan) or 0 (pas.h), INT64_MAX
/ INT32_MAX past the list's end, and the list length min(k, L).  TAS shapes as tas_fuzz.py
(random column scales, ties, saturating targets, unknown operators), GAS as gas_fuzz.py on the
same nodes and pods (unknown-kind containers at 5 %).  One line per case.

  python scripts/diag/c5_fuzz.py --cases 300 [--seed0 1]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gas_fuzz  # noqa: E402
import tas_fuzz  # noqa: E402
from tas_fuzz import oracle, pas_amd, wl  # noqa: E402

GT, LT = 1, 0
I64, I32 = np.iinfo(np.int64).max, np.iinfo(np.int32).max


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def expected(v, u, s, pres, rules, off, prio, cand, gas_args, i915, k, node_base):
    n = v.shape[1]
    P = len(prio)
    fit = (oracle.gas_fit(*gas_args, i915) >> 31).astype(bool)
    c = fit if cand is None else fit & wl.unpack_bits(cand, n)
    _, order, lens = oracle.tas_eval(u, pres, rules, off, prio, wl.pack_bits(c), 3, v_scale=s)
    keys = np.full((P, k), I64, np.int64)
    nodes = np.full((P, k), I32, np.int32)
    ln = np.minimum(lens, k).astype(np.int32)
    for p in range(P):
        m = int(ln[p])
        if m == 0:
            continue
        loc = order[p, :m]
        nodes[p, :m] = loc + node_base
        op = int(prio["op"][p])
        if op == GT:
            keys[p, :m] = np.invert(v[prio["metric"][p], loc])
        elif op == LT:
            keys[p, :m] = v[prio["metric"][p], loc]
        else:
            keys[p, :m] = 0
    return keys, nodes, ln


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=300)
    ap.add_argument("--seed0", type=int, default=1)
    a = ap.parse_args()
    oracle.load()
    ctx = pas_amd.Context(0)
    t0 = time.time()
    for i in range(a.cases):
        seed = a.seed0 + i
        rng = np.random.default_rng(seed)
        meta, v, pres, scales, rules, off, prio, cand, _ = tas_fuzz.case(rng)
        n, P = v.shape[1], len(prio)
        gmeta, gas_args = gas_fuzz.case(rng, n=n, p=P)
        i915 = gmeta["i915"]
        n_cards, cap, used, req, mask, ncont = gas_args
        mask = mask | np.where(rng.random(mask.shape) < 0.05, 0x80000000, 0).astype(np.uint32)
        gas_args = (n_cards, cap, used, req, mask, ncont)
        k = int(rng.choice([1, 5, 16, 70, 300]))
        node_base = int(rng.choice([0, 1234, 1 << 20]))
        u, s = tas_fuzz.oracle_scale(v, scales)
        gen_t, gen_g = 2 * seed, 2 * seed + 1
        ctx.tas_snapshot_set(gen_t, v, pres, [int(x) for x in scales])
        ctx.gas_snapshot_set(gen_g, n_cards, cap, used)
        rules_t = dev(rules.view(np.uint8)) if rules.size else None
        off_t, prio_t = dev(off), dev(prio.view(np.uint8))
        cand_t = None if cand is None else dev(cand.view(np.int64))
        key = torch.empty((P, k), dtype=torch.int64, device="cuda")
        node = torch.empty((P, k), dtype=torch.int32, device="cuda")
        ln = torch.empty(P, dtype=torch.int32, device="cuda")
        ctx.tas_gas_topk_device(gen_t, gen_g, P, len(rules), rules_t, off_t, prio_t, cand_t,
                                req.shape[1], i915, dev(req), dev(mask.view(np.int32)),
                                dev(ncont), k, node_base, key, node, ln)
        ctx.synchronize()
        wk, wn, wl_ = expected(v, u, s, pres, rules, off, prio, cand, gas_args, i915, k,
                               node_base)
        got = (key.cpu().numpy(), node.cpu().numpy(), ln.cpu().numpy())
        bad = [nm for nm, g, w in zip(("keys", "nodes", "lens"), got, (wk, wn, wl_))
               if not np.array_equal(g, w)]
        kept = float((wl_ > 0).mean()) if P else 0.0
        print(f"case {i} seed {seed} k {k} {meta} gas {gmeta} "
              f"{'MISMATCH ' + ','.join(bad) if bad else 'ok'} nonempty {kept:.2f} "
              f"{time.time() - t0:.0f}s", flush=True)
        if bad:
            ctx.close()
            sys.exit(1)
    ctx.close()
    print(f"c5_fuzz: {a.cases} cases bit-exact")


if __name__ == "__main__":
    main()
