"""The oracle with pods of more than 64 card selections (CPU).

  * or_gas_fit / or_gas_bind loop `gpuNum < numI915` without a bound, as
    gpu-aware-scheduling/pkg/gpuscheduler/scheduler.go:213-247 does: checked against a
    pure-Python transcription of that loop on small cases (numI915 up to a few hundred, the
    GPU plugin's shared-dev-num regime);
  * the card-runs restatement the kernels use past 64 selections per container
    (csrc/gas_runs.h) is modelled here in Python and checked against the oracle's literal
    loop, including int64-extreme requests and usages;
  * or_gas_release_counts equals or_gas_release on the same annotation written as a list.
"""
import numpy as np
import pytest

INT64_MAX = 2**63 - 1


def kind_fits(need, cap, used):
    # checkResourceCapacity for one kind (scheduler.go:341-383), Go int64 wrap on the sum
    if need < 0 or cap <= 0 or used < 0:
        return False
    s = used + need
    if s > INT64_MAX:
        return False
    return cap >= s


def go_div(a, b):
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def per_gpu(req_row, mask, q_n, num):
    r = [int(req_row[q]) for q in range(q_n)]
    if num > 1:
        r = [go_div(v, num) for v in r]
    return r


def literal_fit(n_cards, cap, used, req, mask, ncont, p, n, i915=0):
    """runSchedulingLogic as written: returns (fits, list of (container, card))."""
    q_n = cap.shape[1]
    if n_cards[n] <= 0:
        return False, []
    k_n = min(int(n_cards[n]), used.shape[1])
    w = [[int(used[n, k, q]) for q in range(q_n)] for k in range(k_n)]
    sel = []
    for c in range(int(ncont[p])):
        m = int(mask[p, c])
        if m == 0:
            continue
        num = int(req[p, c, i915]) if (m >> i915) & 1 and req[p, c, i915] > 0 else 0
        r = per_gpu(req[p, c], m, q_n, num)
        for _ in range(num):
            chosen = -1
            for k in range(k_n):
                ok = not (m & 0x80000000)
                for q in range(q_n):
                    if (m >> q) & 1:
                        ok = ok and kind_fits(r[q], int(cap[n, q]), w[k][q])
                if ok:
                    chosen = k
                    break
            if chosen < 0:
                return False, []
            for q in range(q_n):
                if (m >> q) & 1:
                    w[chosen][q] += r[q]
            sel.append((c, chosen))
    return True, sel


def runs_fit(n_cards, cap, used, req, mask, ncont, p, n, i915=0):
    """The card-runs restatement (csrc/gas_runs.h) for every container."""
    q_n = cap.shape[1]
    if n_cards[n] <= 0:
        return False, []
    k_n = min(int(n_cards[n]), used.shape[1])
    w = [[int(used[n, k, q]) for q in range(q_n)] for k in range(k_n)]
    sel = []
    for c in range(int(ncont[p])):
        m = int(mask[p, c])
        if m == 0:
            continue
        num = int(req[p, c, i915]) if (m >> i915) & 1 and req[p, c, i915] > 0 else 0
        if num == 0:
            continue
        r = per_gpu(req[p, c], m, q_n, num)
        rem = num
        for k in range(k_n):
            if rem == 0:
                break
            t = INT64_MAX
            if m & 0x80000000:
                t = 0
            for q in range(q_n):
                if not (m >> q) & 1:
                    continue
                capq = int(cap[n, q])
                if r[q] < 0 or capq <= 0 or w[k][q] < 0 or w[k][q] > capq:
                    t = 0
                elif r[q] > 0:
                    t = min(t, (capq - w[k][q]) // r[q])
            t = min(t, rem)
            if t <= 0:
                continue
            for q in range(q_n):
                if (m >> q) & 1:
                    w[k][q] += t * r[q]
            rem -= t
            sel += [(c, k)] * t
        if rem:
            return False, []
    return True, sel


def case(rng, n, k, q, p, c, extreme=False):
    n_cards = rng.integers(-1, k + 1, size=n).astype(np.int32)
    cap = rng.integers(500, 20_000, size=(n, q)).astype(np.int64)
    cap[:, 0] = rng.integers(1, 120, size=n)
    cap[rng.random((n, q)) < 0.05] = 0
    used = rng.integers(0, 300, size=(n, k, q)).astype(np.int64)
    used[:, :, 0] = rng.integers(0, 30, size=(n, k))
    req = np.zeros((p, c, q), np.int64)
    mask = rng.integers(0, 1 << q, size=(p, c)).astype(np.uint32)
    ncont = rng.integers(1, c + 1, size=p).astype(np.int32)
    for pi in range(p):
        for ci in range(ncont[pi]):
            num = int(rng.integers(0, 160))
            if num:
                mask[pi, ci] |= 1
            req[pi, ci, 0] = num
            req[pi, ci, 1:] = rng.integers(0, 60, size=q - 1) * max(num, 1)
    if extreme:
        used[rng.random((n, k, q)) < 0.05] = -3
        used[rng.random((n, k, q)) < 0.05] = INT64_MAX - 7
        cap[:, 1:][rng.random((n, q - 1)) < 0.05] = INT64_MAX  # (i915 capacity stays small:
        # numI915 = INT64_MAX selections on it would never end, here or in the reference)
        req[rng.random((p, c, q)) < 0.05] = -2
        big = rng.random((p, c)) < 0.05
        req[:, :, 0][big] = INT64_MAX
        mask[rng.random((p, c)) < 0.05] |= 0x80000000
    return n_cards, cap, used, req, mask, ncont


@pytest.mark.parametrize("extreme", [False, True])
@pytest.mark.parametrize("k,q", [(4, 2), (8, 3)])
def test_oracle_literal_and_runs(oracle, k, q, extreme):
    rng = np.random.default_rng(k * 31 + q + extreme)
    args = case(rng, 24, k, q, 10, 3, extreme)
    want, sel, nsel = oracle.gas_fit(*args, 0, selections=True)
    n_limit = 0
    for p in range(10):
        for n in range(24):
            fits, lit = literal_fit(*args, p, n)
            fits_r, run = runs_fit(*args, p, n)
            assert (fits, lit) == (fits_r, run), (p, n)
            assert bool(want[p, n] >> 31) == fits
            if fits and len(lit) > 64:
                n_limit += 1
                assert want[p, n] == 0x80000000 | (14 << 24) and nsel[p, n] == -1
            elif fits:
                assert nsel[p, n] == len(lit)
                assert [int(x) for x in sel[p, n, :len(lit)]] == [kk for _, kk in lit]
    assert n_limit > 5


def test_bind_counts_equal_selection(oracle):
    rng = np.random.default_rng(3)
    n_cards, cap, used, req, mask, ncont = case(rng, 12, 8, 2, 20, 3)
    pods = rng.integers(0, 20, size=40).astype(np.int32)
    nodes = rng.integers(0, 12, size=40).astype(np.int32)
    after, res, st, cnt = oracle.gas_bind(n_cards, cap, used, req, mask, ncont, 0, pods, nodes,
                                          counts=True)
    # replay: each bind's counts are the literal selection on the usage before it
    u = used.copy()
    for b, (p, n) in enumerate(zip(pods, nodes)):
        fits, lit = literal_fit(n_cards, cap, u, req, mask, ncont, p, n)
        want = np.zeros(cnt.shape[1:], np.int64)
        if fits:
            for c, kk in lit:
                want[c, kk] += 1
            assert st[b] == 0
            # commit: request / numCards per selection
            for c in range(int(ncont[p])):
                kc = int(want[c].sum())
                if kc == 0:
                    continue
                r = per_gpu(req[p, c], int(mask[p, c]), cap.shape[1], kc)
                for kk in range(cnt.shape[2]):
                    for qq in range(cap.shape[1]):
                        if (int(mask[p, c]) >> qq) & 1:
                            u[n, kk, qq] += r[qq] * int(want[c, kk])
        else:
            assert st[b] == 1
        np.testing.assert_array_equal(cnt[b], want)
    np.testing.assert_array_equal(after, u)
    assert (cnt.sum(axis=(1, 2)) > 64).any()


def test_release_counts_equals_list(oracle):
    rng = np.random.default_rng(11)
    n_cards, cap, used, req, mask, ncont = case(rng, 10, 8, 3, 12, 3)
    pods = np.arange(12, dtype=np.int32)
    nodes = rng.integers(0, 10, size=12).astype(np.int32)
    counts = rng.integers(0, 4, size=(12, 3, 8)).astype(np.int64)
    counts[:, :, 6:] = 0
    cpc = counts.sum(axis=2).astype(np.int32)
    assert cpc.sum(axis=1).max() <= 64
    cards = np.full((12, 64), -1, np.int32)
    for r in range(12):
        lst = [k for c in range(3) for k in range(8) for _ in range(int(counts[r, c, k]))]
        cards[r, :len(lst)] = lst
    a_used, a_st = oracle.gas_release(n_cards, used, req, mask, ncont, pods, nodes, cpc, cards)
    b_used, b_st = oracle.gas_release_counts(n_cards, used, req, mask, ncont, pods, nodes, counts)
    np.testing.assert_array_equal(a_st, b_st)
    np.testing.assert_array_equal(a_used, b_used)
