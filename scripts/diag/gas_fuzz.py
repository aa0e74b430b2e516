"""Seeded fuzz sweep of the GAS fit (pas_gas_fit through libpas.so) against the oracle.

Beyond tests/test_gas_gpu.py's fixed cases: many pods per list (several rank groups of <= 127
thresholds each, and group boundaries inside runs of equal thresholds), tie-heavy and wide
value ranges, every container count and kind mask, i915 anywhere or absent, extreme int64
values.  Each case prints one line (the GPU box's hang detector needs output); the first
mismatch stops the sweep with the case's parameters.

  python scripts/diag/gas_fuzz.py --cases 200 [--seed0 1] [--bind]
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


def case(rng, n=None, p=None):
    q = int(rng.integers(1, 5))
    k = int(rng.choice([1, 2, 3, 4, 5, 7, 8]))
    n = int(rng.integers(1, 1500)) if n is None else n
    p = int(rng.choice([1, 50, 127, 128, 200, 400, 1000, 2500])) if p is None else p
    c = int(rng.integers(1, 5))
    i915 = int(rng.integers(-1, q))
    col = max(i915, 0)
    style = rng.choice(["ties", "wide", "extreme"])
    hi = {"ties": 8, "wide": 1 << 40, "extreme": 1 << 40}[style]
    n_cards = rng.integers(-1, k + 1, size=n).astype(np.int32)
    cap = rng.integers(0, hi * 2 + 1, size=(n, q)).astype(np.int64)
    cap[rng.random((n, q)) < 0.05] = 0
    used = rng.integers(0, hi + 1, size=(n, k, q)).astype(np.int64)
    req = rng.integers(0, hi + 1, size=(p, c, q)).astype(np.int64)
    if i915 >= 0:
        req[:, :, col] = rng.choice([0, 1, 1, 1, 2, 3], size=(p, c))
    mask = rng.integers(0, 1 << q, size=(p, c)).astype(np.uint32)
    ncont = rng.integers(0, c + 1, size=p).astype(np.int32)
    if style == "extreme":
        big = np.int64(2**63 - 1)
        used[rng.random((n, k, q)) < 0.05] = -5
        used[rng.random((n, k, q)) < 0.05] = big - 3
        cap[rng.random((n, q)) < 0.05] = big
        req[rng.random((p, c, q)) < 0.05] = -2
        req[rng.random((p, c, q)) < 0.03] = big
    if i915 >= 0:  # at most 8 selections per pod (the packed word's budget)
        sel = np.where((mask >> col & 1).astype(bool) & (req[:, :, col] > 0),
                       np.minimum(req[:, :, col], 9), 0)  # clamped: no int64 overflow
        live = np.arange(c)[None, :] < ncont[:, None]
        for pi in np.nonzero((sel * live).sum(1) > 8)[0]:
            while int((sel[pi] * live[pi]).sum()) > 8:
                j = int(rng.integers(0, c))
                req[pi, j, col] = 0
                sel[pi, j] = 0
    return dict(q=q, k=k, n=n, p=p, c=c, i915=i915, style=str(style)), \
        (n_cards, cap, used, req, mask, ncont)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=200)
    ap.add_argument("--seed0", type=int, default=1)
    ap.add_argument("--bind", action="store_true", help="also bind, then fit the committed usage")
    a = ap.parse_args()
    oracle.load()
    ctx = pas_amd.Context(0)
    t0 = time.time()
    for i in range(a.cases):
        seed = a.seed0 + i
        meta, args = case(np.random.default_rng(seed))
        i915 = meta["i915"]
        ctx.gas_snapshot_set(seed, *args[:3])
        got = ctx.gas_fit(seed, *args[3:], i915)
        want = oracle.gas_fit(*args, i915)
        ok = np.array_equal(got, want)
        print(f"case {i} seed {seed} {meta} {'ok' if ok else 'MISMATCH'} "
              f"fit {float((want >> 31).mean()) if want.size else 0:.2f} {time.time() - t0:.0f}s",
              flush=True)
        if ok and a.bind and meta["p"] > 0 and meta["n"] > 0:
            # binds of random pods to random nodes, committed (bindNode), then a fit on the
            # committed usage: statuses, words and usage against the oracle's in-order binds
            rng = np.random.default_rng(seed + 10**6)
            B = int(rng.integers(1, 300))
            pods = rng.integers(0, meta["p"], size=B).astype(np.int32)
            nodes = rng.integers(0, meta["n"], size=B).astype(np.int32)
            res, st = ctx.gas_bind(seed, seed + 10**7, pods, nodes, *args[3:], i915)
            w_used, w_res, w_st = oracle.gas_bind(*args, i915, pods, nodes)
            _, after = ctx.gas_snapshot_get()
            got2 = ctx.gas_fit(seed + 10**7, *args[3:], i915)
            want2 = oracle.gas_fit(args[0], args[1], w_used, *args[3:], i915)
            ok = (np.array_equal(res, w_res) and np.array_equal(st, w_st)
                  and np.array_equal(after, w_used) and np.array_equal(got2, want2))
            if not ok:
                print(f"bind mismatch: res {np.array_equal(res, w_res)} st "
                      f"{np.array_equal(st, w_st)} used {np.array_equal(after, w_used)} fit "
                      f"{np.array_equal(got2, want2)}")
                got, want = got2, want2
        if not ok:
            bad = np.argwhere(got != want)
            print("first mismatches (pod, node, got, want):",
                  [(int(x), int(y), hex(int(got[x, y])), hex(int(want[x, y]))) for x, y in bad[:8]])
            ctx.close()
            sys.exit(1)
    ctx.close()
    print(f"gas_fuzz: {a.cases} cases bit-exact")


if __name__ == "__main__":
    main()
