"""Diagnostic: lazy combined top-k vs the composed path vs the oracle composition, one case."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("platform-aware-scheduling_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import torch  # noqa: E402

import oracle  # noqa: E402
import pas_amd  # noqa: E402
from pas_amd import workload as wl  # noqa: E402
from test_shard import _lazy_vs_composed, make_case  # noqa: E402

k, n, cards, cand_frac = [int(x) if i < 3 else float(x) for i, x in enumerate(sys.argv[1:5])]
snap, batch = make_case(0x60 + k + cards, n, 6, 96, 7, cand_frac=cand_frac)
rng = np.random.default_rng(k * 7 + n)
gsnap = wl.make_gas_snapshot(n, seed=0x61 + k)
gbatch = wl.make_gas_batch(96, seed=0x61 + k)
flag = rng.random(gbatch.req_mask.shape) < float(sys.argv[5])
gbatch.req_mask = gbatch.req_mask | np.where(flag, 0x80000000, 0).astype(np.uint32)
batch.prio["metric"][::17] = 99
ctx = pas_amd.Context(0)
base = int(sys.argv[6]) if len(sys.argv) > 6 else 0
(kc, nc, lc), (kl, nl, ll) = _lazy_vs_composed(ctx, snap.v_milli, snap.present, batch, gsnap,
                                               gbatch, batch.cand, k, base, wl.I915)
print("keys equal", np.array_equal(kc, kl), "nodes equal", np.array_equal(nc, nl),
      "lens equal", np.array_equal(lc, ll))
for p in range(len(batch.prio)):
    if not np.array_equal(kc[p], kl[p]):
        j = int(np.nonzero(kc[p] != kl[p])[0][0])
        print("pod", p, "op", batch.prio["op"][p], "len", lc[p], ll[p], "first diff", j,
              "keys", kc[p, j:j + 3], kl[p, j:j + 3], "nodes", nc[p, j:j + 3], nl[p, j:j + 3])
        break
nc = np.where(nc == np.iinfo(np.int32).max, nc, nc - base)
nl = np.where(nl == np.iinfo(np.int32).max, nl, nl - base)
words = oracle.gas_fit(gsnap.n_cards, gsnap.cap, gsnap.used, gbatch.req, gbatch.req_mask,
                       gbatch.n_containers, wl.I915)
fitb = wl.pack_bits((words >> 31).astype(bool))
cand = fitb & batch.cand
_, order, lens = oracle.tas_eval(snap.v_milli, snap.present, batch.rules, batch.rule_off,
                                 batch.prio, cand, 3)
bad_c = bad_l = 0
for p in range(len(batch.prio)):
    m = min(k, int(lens[p]))
    want = order[p, :m]
    okc = lc[p] == m and np.array_equal(nc[p, :m], want)
    okl = ll[p] == m and np.array_equal(nl[p, :m], want)
    bad_c += not okc
    bad_l += not okl
    if not okl and bad_l <= 3:
        print("pod", p, "op", batch.prio["op"][p], "m", m, "lazy len", ll[p], "comp len", lc[p])
        print(" want", want[:20])
        print(" lazy", nl[p, :20])
print("composed bad", bad_c, "lazy bad", bad_l, "of", len(batch.prio))
ctx.close()
