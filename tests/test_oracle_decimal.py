"""The oracle's exact decimal values: or_evaluate_rule_dec / or_cmp_dec
restate Quantity.CmpInt64 / Quantity.Cmp (telemetry-aware-scheduling/pkg/strategies/core/
operator.go:16-22, 37-39) on u * 10^-s, checked here against Python's decimal module, and the
batched filter / prioritize against a pure-Python loop over Decimal values."""
from decimal import Decimal

import numpy as np

from helpers import RULE_DTYPE, pack_bits, unpack_bits

OPS = {0: lambda c: c < 0, 1: lambda c: c > 0, 2: lambda c: c == 0}


def dec(u, s):
    return Decimal(int(u)).scaleb(-int(s))


def test_cmp_and_evaluate_rule_against_decimal(oracle):
    rng = np.random.default_rng(0xDEC)
    for _ in range(20000):
        s1, s2 = (int(x) for x in rng.integers(0, 10, 2))
        lim = 2**62
        u1 = int(rng.integers(-lim, lim)) if rng.random() < 0.5 else int(rng.integers(-5000, 5000))
        u2 = u1 * 10**(s2 - s1) if (rng.random() < 0.2 and s2 >= s1) else int(rng.integers(-5000, 5000))
        if not -2**63 <= u2 < 2**63:
            u2 = 7
        a, b = dec(u1, s1), dec(u2, s2)
        assert oracle.cmp_dec(u1, s1, u2, s2) == (a > b) - (a < b)
        t = int(rng.integers(-10**6, 10**6)) if rng.random() < 0.8 else int(rng.integers(-lim, lim))
        for op in (0, 1, 2):
            c = (a > t) - (a < t)
            assert oracle.evaluate_rule_dec(u1, s1, op, t) == int(OPS[op](c)), (u1, s1, op, t)
    assert oracle.evaluate_rule_dec(1, 0, 7, 0) == -1  # unknown operator: the reference panics


def test_tas_eval_dec_against_python_loop(oracle):
    """Sub-milli values, several scales per column (the same value spelled at different
    scales), ties within one milli bucket: filter bits and ordered lists equal a literal
    Python restatement of Violated / filterNodes / OrderedList over Decimal values."""
    rng = np.random.default_rng(0xDE2)
    M, N, P = 4, 300, 40
    base = rng.integers(-2000, 2000, size=(M, N))  # in units of 1e-4: 0.0005-step ties
    u = np.zeros((M, N), np.int64)
    sc = np.zeros((M, N), np.int8)
    for m in range(M):
        for n in range(N):
            s = int(rng.integers(4, 10))  # the value base * 1e-4 written with s places
            u[m, n] = int(base[m, n]) * 10**(s - 4)
            sc[m, n] = s
    pres_b = rng.random((M, N)) < 0.95
    present = pack_bits(pres_b)
    vals = [[dec(u[m, n], sc[m, n]) for n in range(N)] for m in range(M)]
    rules, off, prio = [], [0], np.zeros(P, RULE_DTYPE)
    for p in range(P):
        for _ in range(3):
            rules.append((int(rng.integers(0, M)), int(rng.integers(0, 3)),
                          int(rng.integers(-1, 2))))
        off.append(len(rules))
        prio[p] = (int(rng.integers(0, M)), int(rng.integers(0, 3)), 0)
    rules = np.array(rules, RULE_DTYPE)
    off = np.array(off, np.int32)
    pass_o, order_o, len_o = oracle.tas_eval(u, present, rules, off, prio, v_scale=sc)
    for p in range(P):
        viol = set()
        for r in rules[off[p]:off[p + 1]]:
            m, op, t = int(r["metric"]), int(r["op"]), int(r["target"])
            for n in range(N):
                if pres_b[m, n] and OPS[op]((vals[m][n] > t) - (vals[m][n] < t)):
                    viol.add(n)
        passing = [n for n in range(N) if n not in viol]
        assert unpack_bits(pass_o[p], N).nonzero()[0].tolist() == passing
        m, op = int(prio[p]["metric"]), int(prio[p]["op"])
        items = [n for n in passing if pres_b[m, n]]
        if op == 1:
            items.sort(key=lambda n: -vals[m][n])  # stable: ties keep node order
        elif op == 0:
            items.sort(key=lambda n: vals[m][n])
        assert order_o[p, : len_o[p]].tolist() == items, p
