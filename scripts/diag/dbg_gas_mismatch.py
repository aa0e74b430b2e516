"""Diagnostic: first mismatches of the GAS fit vs the oracle on test_random_parity's inputs."""
import os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(R, "platform-aware-scheduling_amd"), os.path.join(R, "oracle"), os.path.join(R, "tests")):
    sys.path.insert(0, p)
import oracle, pas_amd
from test_gas_gpu import random_gas, gpu_fit
q, k = int(sys.argv[1]), int(sys.argv[2])
ctx = pas_amd.Context(0)
rng = np.random.default_rng(q * 100 + k)
for extreme in (False, True):
    i915 = -1 if (extreme and q == 2) else (q - 1 if k == 3 else 0)
    args = random_gas(rng, 777, k, q, 23, 4, extreme, i915)
    got = gpu_fit(ctx, *args, i915)
    want = oracle.gas_fit(*args, i915)
    bad = np.argwhere(got != want)
    print("extreme", extreme, "mismatches", len(bad))
    n_cards, cap, used, req, mask, ncont = args
    cols = sorted(set(int(b[1]) for b in bad))
    print("bad nodes", cols[:40], "of", len(cols))
    print("bad pods", sorted(set(int(b[0]) for b in bad)))
    for p_, n_ in bad[:12]:
        print(p_, n_, hex(int(got[p_, n_])), hex(int(want[p_, n_])), "nc", n_cards[n_], "cap", cap[n_], "used", used[n_].tolist(),
              "req", req[p_, :ncont[p_]].tolist(), "mask", mask[p_, :ncont[p_]].tolist())
