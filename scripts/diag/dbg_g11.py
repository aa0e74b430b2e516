import sys, os
sys.path[:0] = ["tests", "platform-aware-scheduling_amd", "oracle"]
import numpy as np, pas_amd, oracle
from helpers import golden, decode_gas_word
from test_oracle_golden import commit_pod, gas_readme_case
G = golden()
ctx = pas_amd.Context(0)
gen = [100]
for name in ("memory_example", "millicores_example"):
    ex = G["G11_gas_readme"][name]
    kinds, cards, n_cards, cap, used, req, mask = gas_readme_case(ex)
    for want in ex["want"]:
        gen[0] += 1
        ctx.gas_snapshot_set(gen[0], n_cards, cap, used)
        got = ctx.gas_fit(gen[0], req, mask, np.array([1], np.int32), 0)
        w = oracle.gas_fit(n_cards, cap, used, req, mask, np.array([1], np.int32), 0)
        print(name, "cap", cap.tolist(), "used", used.tolist(), "req", req.tolist(), "mask", mask.tolist(), "gpu", hex(int(got[0,0])), "oracle", hex(int(w[0,0])), "want", want)
        fits, sel = decode_gas_word(w[0, 0])
        if fits: commit_pod(used[0], req[0], mask[0], [sel])
