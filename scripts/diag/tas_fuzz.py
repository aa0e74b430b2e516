"""Seeded fuzz sweep of the TAS path (pas_tas_eval, pas_tas_violations, pas_tas_label_plan
through libpas.so) against the oracle.

Beyond tests/test_tas_gpu.py's fixed cases: random node counts around the 64-node word and
1024-position segment edges, 1-8 metrics at random decimal scales (0-9: sub-milli values, ties
inside one milli bucket), tie-heavy or wide columns, absent values, missing metrics, saturating
and exact-hit targets, every operator plus an unknown prioritize operator, candidate masks,
filter-only / prioritize-only / both, and shared deschedule policy names.  One line per case;
the first mismatch stops the sweep.

  python scripts/diag/tas_fuzz.py --cases 300 [--seed0 1]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "platform-aware-scheduling_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import oracle  # noqa: E402  (test infrastructure: the checker)
import pas_amd  # noqa: E402
from pas_amd import workload as wl  # noqa: E402


def case(rng):
    n = int(rng.choice([1, 63, 64, 65, 1023, 1024, 1025, 2047, 3000, 5000, 20_000]))
    n = max(1, n + int(rng.integers(-2, 3)))
    m = int(rng.integers(1, 9))
    p = int(rng.choice([1, 7, 64, 200]))
    r_max = int(rng.choice([0, 3, 15, 70]))
    scales = rng.integers(0, 10, size=m)
    ties = bool(rng.random() < 0.5)
    v = np.zeros((m, n), np.int64)
    for j, k in enumerate(scales):
        one = 10 ** int(k)
        if ties:  # few distinct values: whole units and a few fractions of one
            pool = np.array([0, 1, 2, -3, 7], np.int64) * one
            if k >= 1:
                pool = np.concatenate([pool, pool + one // 10])
            v[j] = rng.choice(pool, size=n)
        else:
            v[j] = rng.integers(-10**6, 10**6, size=n) * max(one // 1000, 1)
    pres_b = rng.random((m, n)) >= rng.choice([0.0, 0.1, 0.5])
    if m > 1 and rng.random() < 0.3:
        pres_b[m - 1] = False  # a metric no node reports
    pres = wl.pack_bits(pres_b)
    n_r = rng.integers(0, r_max + 1, size=p)
    off = np.zeros(p + 1, np.int32)
    off[1:] = np.cumsum(n_r)
    nr = int(off[-1])
    rules = np.zeros(nr, pas_amd.RULE_DTYPE)
    rules["metric"] = rng.integers(-1, m + 1, size=nr)
    rules["op"] = rng.integers(0, 3, size=nr)
    # targets in whole units: near the values, exact hits, saturating extremes
    t = rng.integers(-1000, 1000, size=nr)
    sel = rng.random(nr)
    t = np.where(sel < 0.3, rng.choice([0, 1, 2, -3, 7], size=nr), t)
    t = np.where((sel >= 0.3) & (sel < 0.33), np.int64(2**62), t)
    t = np.where((sel >= 0.33) & (sel < 0.36), np.int64(-2**62), t)
    t = np.where((sel >= 0.36) & (sel < 0.38), np.int64(2**63 - 1), t)
    rules["target"] = t
    prio = np.zeros(p, pas_amd.RULE_DTYPE)
    prio["metric"] = rng.integers(-1, m + 1, size=p)
    prio["op"] = rng.integers(0, 4, size=p)  # 3: another operator string
    cand = wl.pack_bits(rng.random((p, n)) < rng.choice([0.5, 0.9, 1.0])) \
        if rng.random() < 0.5 else None
    flags = int(rng.choice([1, 2, 3]))
    meta = dict(n=n, m=m, p=p, r_max=r_max, ties=ties, flags=flags, cand=cand is not None,
                scales="".join(str(int(k)) for k in scales))
    return meta, v, pres, scales, rules, off, prio, cand, flags


def oracle_scale(v, scales):
    """The oracle's per-value spelling: value = u * 10^-s with the fewest places."""
    u = v.copy()
    s = np.repeat(np.array(scales, np.int8)[:, None], v.shape[1], 1)
    for _ in range(9):
        z = (u % 10 == 0) & (s > 0)
        u = np.where(z, u // 10, u)
        s = np.where(z, s - 1, s).astype(np.int8)
    return u, s


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
        meta, v, pres, scales, rules, off, prio, cand, flags = case(rng)
        u, s = oracle_scale(v, scales)
        ctx.tas_snapshot_set(seed, v, pres, [int(k) for k in scales])
        gp, go, gl = ctx.tas_eval(seed, rules, off, prio, cand, flags)
        op_, oo, ol = oracle.tas_eval(u, pres, rules, off, prio, cand, flags, v_scale=s)
        bad = None
        if flags & 1 and not np.array_equal(gp, op_):
            bad = "pass"
        if flags & 2 and not bad:
            if not np.array_equal(gl, ol):
                bad = "len"
            else:
                for q in range(len(gl)):
                    if not np.array_equal(go[q, : gl[q]], oo[q, : ol[q]]):
                        bad = f"order pod {q}"
                        break
        # the same rules as deschedule strategies (a pod's rules = one strategy), then the
        # label plan with some strategies sharing a policy name
        if not bad:
            gv = ctx.tas_violations(seed, rules, off)
            wv = oracle.tas_violations(u, pres, rules, off, v_scale=s)
            if not np.array_equal(gv, wv):
                bad = "violations"
            else:
                S = min(64, len(off) - 1)  # a label plan takes at most 64 strategies
                labels = wl.pack_bits(rng.random((S, v.shape[1])) < 0.3)
                names = [f"pol{int(x)}" for x in rng.integers(0, S // 2 + 1, size=S)]
                g = ctx.tas_label_plan(v.shape[1], gv[:S], labels, names)
                w = oracle.label_plan(wv[:S], labels, v.shape[1], names)
                if not all(np.array_equal(np.asarray(x), np.asarray(y)) for x, y in zip(g, w)):
                    bad = "label plan"
        print(f"case {i} seed {seed} {meta} {bad or 'ok'} {time.time() - t0:.0f}s", flush=True)
        if bad:
            ctx.close()
            sys.exit(1)
    ctx.close()
    print(f"tas_fuzz: {a.cases} cases bit-exact")


if __name__ == "__main__":
    main()
