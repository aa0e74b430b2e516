"""GAS per-card first fit through libpas.so's HIP kernel, bit-exact against the oracle
(card selections included) and the reference's golden vectors.  Marked gpu."""
import numpy as np
import pytest

import pas_amd
from pas_amd import workload as wl
from helpers import decode_gas_word, golden
from test_oracle_golden import commit_pod, gas_readme_case

pytestmark = pytest.mark.gpu
G = golden()
_gen = [5000]


def gpu_fit(ctx, n_cards, cap, used, req, mask, ncont, i915):
    _gen[0] += 1
    ctx.gas_snapshot_set(_gen[0], n_cards, cap, used)
    return ctx.gas_fit(_gen[0], req, mask, ncont, i915)


def test_golden_g10_no_label(ctx):
    res = gpu_fit(ctx, np.array([0, -1], np.int32), np.zeros((2, 1), np.int64),
                  np.zeros((2, 1, 1), np.int64), np.zeros((1, 1, 1), np.int64),
                  np.zeros((1, 1), np.uint32), np.array([1], np.int32), 0)
    assert not decode_gas_word(res[0, 0])[0] and not decode_gas_word(res[0, 1])[0]
    # checkResourceCapacity(need {foo:1}, capacity {}, used {}) == false (scheduler_test.go:122-131)
    res = gpu_fit(ctx, np.array([1], np.int32), np.zeros((1, 1), np.int64),
                  np.zeros((1, 1, 1), np.int64), np.ones((1, 1, 1), np.int64),
                  np.array([[1]], np.uint32), np.array([1], np.int32), 0)
    assert not decode_gas_word(res[0, 0])[0]


def test_golden_g11_readme(ctx):
    g = G["G11_gas_readme"]
    for ex in (g["memory_example"], g["millicores_example"]):
        kinds, cards, n_cards, cap, used, req, mask = gas_readme_case(ex)
        for want in ex["want"]:
            res = gpu_fit(ctx, n_cards, cap, used, req, mask, np.array([1], np.int32), 0)
            fits, sel = decode_gas_word(res[0, 0])
            assert fits == want["fits"]
            if fits:
                assert ",".join(cards[k] for k in sel) == want["annotation"]
                commit_pod(used[0], req[0], mask[0], [sel])


def random_gas(rng, n, k, q, p, c, extreme=False, i915=0):
    n_cards = rng.integers(-1, k + 1, size=n).astype(np.int32)
    cap = rng.integers(0, 1000, size=(n, q)).astype(np.int64)
    cap[rng.random((n, q)) < 0.05] = 0
    used = rng.integers(0, 1000, size=(n, k, q)).astype(np.int64)
    req = rng.integers(0, 600, size=(p, c, q)).astype(np.int64)
    col = max(i915, 0)
    req[:, :, col] = rng.integers(0, 4, size=(p, c))
    mask = rng.integers(0, 1 << q, size=(p, c)).astype(np.uint32)
    ncont = rng.integers(0, c + 1, size=p).astype(np.int32)
    if extreme:
        big = np.int64(2**63 - 1)
        used[rng.random((n, k, q)) < 0.05] = -5
        used[rng.random((n, k, q)) < 0.05] = big - 3
        cap[rng.random((n, q)) < 0.05] = big
        req[rng.random((p, c, q)) < 0.05] = -2
        req[rng.random((p, c, q)) < 0.03] = big
    # keep within the packed 8-selection budget per pod
    for pi in range(p):
        while i915 >= 0 and sum(int(req[pi, ci, col]) for ci in range(ncont[pi])
                                if (mask[pi, ci] >> col & 1) and req[pi, ci, col] > 0) > 8:
            req[pi, rng.integers(0, c), col] = 0
    return n_cards, cap, used, req, mask, ncont


@pytest.mark.parametrize("q", [1, 2, 3, 4])
@pytest.mark.parametrize("k", [1, 3, 8])
def test_random_parity(ctx, oracle, q, k):
    rng = np.random.default_rng(q * 100 + k)
    for extreme in (False, True):
        i915 = -1 if (extreme and q == 2) else (q - 1 if k == 3 else 0)
        args = random_gas(rng, 777, k, q, 23, 4, extreme, i915)
        got = gpu_fit(ctx, *args, i915)
        want = oracle.gas_fit(*args, i915)
        np.testing.assert_array_equal(got, want)


def test_c3_shape_pod_sample(ctx, oracle):
    # configs[2] node shape: 50k nodes x 8 cards x 3 kinds, on 64 pods (full oracle check)
    snap = wl.make_gas_snapshot(50_000, seed=0xC3)
    batch = wl.make_gas_batch(64, seed=0xC3)
    got = gpu_fit(ctx, snap.n_cards, snap.cap, snap.used, batch.req, batch.req_mask,
                  batch.n_containers, wl.I915)
    want = oracle.gas_fit(snap.n_cards, snap.cap, snap.used, batch.req, batch.req_mask,
                          batch.n_containers, wl.I915)
    np.testing.assert_array_equal(got, want)
    fit_frac = (got >> 31).mean()
    assert 0.3 < fit_frac < 0.99


def test_selections_past_64_evaluated(ctx, oracle):
    # 65 selections on 8 cards of per-GPU i915 capacity 100: fits (card 0 takes all), the word
    # is bit 31 | PAS_GAS_SEL_LIMIT (tests/test_gas_many_selections.py has the full parity)
    req = np.zeros((1, 2, 1), np.int64)
    req[0, :, 0] = [40, 25]
    args = (np.array([8], np.int32), np.full((1, 1), 100, np.int64),
            np.zeros((1, 8, 1), np.int64), req, np.ones((1, 2), np.uint32),
            np.array([2], np.int32), 0)
    got = gpu_fit(ctx, *args)
    np.testing.assert_array_equal(got, oracle.gas_fit(*args))
    assert int(got[0, 0]) == 0x80000000 | (14 << 24)


def test_same_card_reuse_and_container_accumulation(ctx, oracle):
    # per-GPU i915 capacity 300 (shared-dev-num), so one card can take every selection;
    # a second container sees the first one's usage (scheduler.go:317-319)
    n_cards = np.array([2], np.int32)
    cap = np.array([[300, 1000]], np.int64)
    used = np.zeros((1, 2, 2), np.int64)
    req = np.array([[[2, 800], [1, 300]]], np.int64)  # per GPU: [1, 400] x2, then [1, 300]
    mask = np.array([[3, 3]], np.uint32)
    got = gpu_fit(ctx, n_cards, cap, used, req, mask, np.array([2], np.int32), 0)
    assert decode_gas_word(got[0, 0]) == (True, [0, 0, 1])
    np.testing.assert_array_equal(got, oracle.gas_fit(n_cards, cap, used, req, mask,
                                                      np.array([2], np.int32), 0))


def test_two_selection_take_overflow(ctx, oracle):
    # two containers, one card each; the first takes INT64_MAX of a kind on card 0, so the
    # second's check on card 0 overflows (used + need < 0 -> false, scheduler.go:367-371) and
    # it must go to card 1
    big = np.int64(2**63 - 1)
    n_cards = np.array([2], np.int32)
    cap = np.array([[10, big]], np.int64)
    used = np.zeros((1, 2, 2), np.int64)
    req = np.array([[[1, big], [1, 5]]], np.int64)
    mask = np.array([[3, 3]], np.uint32)
    ncont = np.array([2], np.int32)
    want = oracle.gas_fit(n_cards, cap, used, req, mask, ncont, 0)
    assert decode_gas_word(want[0, 0]) == (True, [0, 1])
    got = gpu_fit(ctx, n_cards, cap, used, req, mask, ncont, 0)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_extreme_multi_selection_fuzz(ctx, oracle, seed):
    # near-int64 capacities, usages and requests across several selections per pod: every
    # overflow branch of checkResourceCapacity / addRM (scheduler.go:341-383,
    # resource_map.go:77-98) through the single, two-selection and multi-selection paths
    rng = np.random.default_rng(seed)
    big = 2**63 - 1
    n, k, q, p, c = 300, 3, 2, 64, 4
    n_cards = rng.integers(0, k + 1, size=n).astype(np.int32)
    cap = rng.choice(np.array([big, big - 1, 2**62, 2**61, 10], np.int64), size=(n, q))
    used = rng.choice(np.array([0, 1, 2**62, 2**61, big - 5], np.int64), size=(n, k, q))
    req = rng.choice(np.array([1, 2, 2**60, 2**61, 2**62, big - 1, big], np.int64),
                     size=(p, c, q))
    req[:, :, 0] = rng.integers(1, 3, size=(p, c))  # i915 selections per container
    mask = np.full((p, c), 3, np.uint32)
    ncont = rng.integers(1, c + 1, size=p).astype(np.int32)
    for pi in range(p):  # at most 8 selections per pod
        while int(req[pi, :ncont[pi], 0].sum()) > 8:
            ncont[pi] -= 1
    want = oracle.gas_fit(n_cards, cap, used, req, mask, ncont, 0)
    got = gpu_fit(ctx, n_cards, cap, used, req, mask, ncont, 0)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("q", [2, 3, 4])
def test_kind_skip_lists(ctx, oracle, q):
    # a roomy cluster: every real card has >= 500 free of kinds 1.., so pods whose needs (plus
    # their earlier takes) stay within that minimum are filed under a kind-skipping list; the
    # boundary (== and == + 1 of the minimum), pods requesting a single kind (which must keep
    # failing on missing cards), nodes with fewer cards than K and nodes without the label
    rng = np.random.default_rng(40 + q)
    n, k, p, c = 500, 4, 96, 3
    n_cards = rng.integers(-1, k + 1, size=n).astype(np.int32)
    cap = np.full((n, q), 2000, np.int64)
    cap[:, 0] = 4
    used = rng.integers(0, 1500, size=(n, k, q)).astype(np.int64)
    used[:, :, 0] = rng.integers(0, 5, size=(n, k))
    used[n_cards <= 0] = 1999  # unlabelled nodes do not lower the minimum
    real = np.arange(k)[None, :] < np.maximum(n_cards, 0)[:, None]
    gmin = [(cap[:, None, j] - used[:, :, j])[real].min() for j in range(q)]
    req = rng.integers(0, 40, size=(p, c, q)).astype(np.int64)
    req[:, :, 0] = rng.integers(0, 3, size=(p, c))
    for pi in range(0, p, 4):  # exactly at / one beyond the minimum of kind 1 (one selection)
        req[pi, 0, 1] = gmin[1] + (pi // 4) % 2
    mask = rng.integers(0, 1 << q, size=(p, c)).astype(np.uint32) | 1
    mask[::5] = 1  # only i915: nothing to skip but the last common kind
    mask[1::7] = 3
    ncont = rng.integers(1, c + 1, size=p).astype(np.int32)
    ncont[::4] = 1
    want = oracle.gas_fit(n_cards, cap, used, req, mask, ncont, 0)
    got = gpu_fit(ctx, n_cards, cap, used, req, mask, ncont, 0)
    np.testing.assert_array_equal(got, want)
    assert 0.1 < (want >> 31).mean() < 0.95


SPLITS = {4: [(4,), (2, 2), (1, 1, 1, 1), (2, 1, 1), (1, 2, 1), (1, 1, 2), (3, 1), (1, 3)],
          3: [(3,), (2, 1), (1, 2), (1, 1, 1)]}
PATTERNS = {4: {(4,), (1, 3), (2, 2), (1, 1, 2), (1, 1, 1, 1)}, 3: {(3,), (1, 2), (1, 1, 1)}}


@pytest.mark.parametrize("sel", [3, 4])
@pytest.mark.parametrize("q", [2, 3, 4])
@pytest.mark.parametrize("k", [4, 8])
def test_closed_form_64bit_rows(ctx, oracle, sel, q, k):
    """Pods of exactly 3 or 4 selections in a kind-skip list (every real card keeps >= 5 of
    kind 0 free): the closed forms (4: gas_rfit_seq_kernel on 64-bit one-card rows, GasFour /
    rfour; 3: gas_rfit_closed_kernel on ranks).  Every container split (identical selections: the reused masks), small frees
    so that selections share cards in every occupancy pattern, needs of 2^62 on nodes with
    int64-max capacity (rows whose sums overflow int64), nodes with fewer cards than K or no
    label, a kind-1 request that one pod in 7 drops; words and node bitmaps against the
    oracle."""
    import torch
    rng = np.random.default_rng(700 + 100 * sel + 10 * q + k)
    n, p, c = 700, 192, 4
    big = 2**63 - 1
    n_cards = rng.integers(-1, k + 1, size=n).astype(np.int32)
    cap = np.zeros((n, q), np.int64)
    cap[:, 0] = 10
    cap[:, 1:] = rng.choice(np.array([12, 20, 40, big], np.int64), size=(n, q - 1))
    used = rng.integers(0, 8, size=(n, k, q)).astype(np.int64)
    used[:, :, 0] = rng.integers(0, 6, size=(n, k))
    req = np.zeros((p, c, q), np.int64)
    mask = np.zeros((p, c), np.uint32)
    ncont = np.zeros(p, np.int32)
    for pi in range(p):
        split = SPLITS[sel][pi % len(SPLITS[sel])]
        ncont[pi] = len(split)
        huge = pi % 11 == 3 and all(s == 1 for s in split)
        for ci, ni in enumerate(split):
            req[pi, ci, 0] = ni
            per = rng.integers(1, 9, size=q - 1)
            req[pi, ci, 1:] = per * ni
            if huge:
                req[pi, ci, 1] = 2**62
            mask[pi, ci] = (1 << q) - 1
            if q > 2 and pi % 7 == 5:
                mask[pi, ci] &= ~np.uint32(2)  # kind 1 not requested (kinds 2.. are)
    want = oracle.gas_fit(n_cards, cap, used, req, mask, ncont, 0)
    got = gpu_fit(ctx, n_cards, cap, used, req, mask, ncont, 0)
    np.testing.assert_array_equal(got, want)
    fits = (want >> 31).astype(bool)
    assert 0.05 < fits.mean() < 0.95
    # every occupancy pattern of the 4 selections occurs among the fitting words
    cards = [decode_gas_word(w)[1] for w in want[fits][:20000]]
    patterns = {tuple(sorted(np.unique(cs, return_counts=True)[1])) for cs in cards}
    assert PATTERNS[sel] <= patterns
    # the node bitmaps of the same fit
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    bm = torch.zeros((p, (n + 63) // 64), dtype=torch.int64, device="cuda")
    ctx.gas_fit_bitmap_device(_gen[0], p, c, 0, dev(req), dev(mask.view(np.int32)), dev(ncont),
                              bm)
    ctx.synchronize()
    np.testing.assert_array_equal(wl.unpack_bits(bm.cpu().numpy().view(np.uint64), n), fits)


@pytest.mark.parametrize("cap_max", [2**31 - 2, 2**31 - 1])
def test_narrow_kind_boundary(ctx, oracle, cap_max):
    # kinds whose cap stays <= INT32_MAX - 1 on every node compare in 32 bits (needs clamped):
    # needs around INT32_MAX and beyond, over-committed cards (used > cap: free < -1), negative
    # usage, and the first value that keeps the kind 64-bit; one and several selections
    rng = np.random.default_rng(cap_max & 0xFF)
    n, k, q, p, c = 300, 4, 3, 64, 3
    n_cards = rng.integers(0, k + 1, size=n).astype(np.int32)
    cap = rng.choice(np.array([1, 1000, cap_max - 5, cap_max], np.int64), size=(n, q))
    cap[:, 2] = 2**40  # one kind always 64-bit
    used = rng.choice(np.array([0, 1, 999, cap_max - 6, cap_max, 2**31 + 7, 2**40, -3], np.int64),
                      size=(n, k, q))
    req = rng.choice(np.array([0, 1, 5, cap_max - 6, cap_max - 1, 2**31 - 1, 2**31, 2**33],
                              np.int64), size=(p, c, q))
    req[:, :, 0] = rng.integers(1, 3, size=(p, c))  # i915 selections per container
    mask = rng.integers(0, 1 << q, size=(p, c)).astype(np.uint32) | 1
    ncont = rng.integers(1, c + 1, size=p).astype(np.int32)
    want = oracle.gas_fit(n_cards, cap, used, req, mask, ncont, 0)
    got = gpu_fit(ctx, n_cards, cap, used, req, mask, ncont, 0)
    np.testing.assert_array_equal(got, want)
    assert 0.02 < (want >> 31).mean() < 0.98


@pytest.mark.parametrize("k", [3, 8, 12])
def test_unknown_kind_flag_parity(ctx, oracle, k):
    # containers flagged PAS_REQ_UNKNOWN_KIND (they also request a gpu.intel.com/ kind the
    # snapshot lacks): a pod with such a container and numI915 > 0 fits no node; with
    # numI915 == 0 the flag changes nothing (scheduler.go:206-215, 349-354).  Single,
    # multi-selection and (k = 12: nodes past 8 cards) generic kernels.
    rng = np.random.default_rng(900 + k)
    n_cards, cap, used, req, mask, ncont = random_gas(rng, 500, k, 3, 80, 4, i915=0)
    flag = rng.random(mask.shape) < 0.15
    mask = mask | np.where(flag, pas_amd._lib.PAS_REQ_UNKNOWN_KIND, 0).astype(np.uint32)
    want = oracle.gas_fit(n_cards, cap, used, req, mask, ncont, 0)
    got = gpu_fit(ctx, n_cards, cap, used, req, mask, ncont, 0)
    np.testing.assert_array_equal(got, want)
    # pods whose flagged container selects a card never fit; flagged containers with no
    # selection leave the pod's result as without the flag
    sel = (req[:, :, 0] > 0) & ((mask & 1) == 1)
    live = np.arange(mask.shape[1])[None, :] < ncont[:, None]
    blocked = (flag & sel & live).any(axis=1)
    assert blocked.any() and not (want[blocked] >> 31).any()
    clean = oracle.gas_fit(n_cards, cap, used, req, mask & 0x7FFFFFFF, ncont, 0)
    np.testing.assert_array_equal(want[~blocked], clean[~blocked])


def test_fits_alternating_streams(oracle):
    """Back-to-back fits on different streams without host synchronisation: each
    fit starts from list counts the previous fit's prep kernel zeroed on ITS stream, and the
    context's scratch is shared, so a fit on another stream waits for the previous fit
    (gas_fit_launch).  Fresh context, batches of different shapes, every result checked."""
    import torch
    gs = wl.make_gas_snapshot(6000, seed=0x5A)
    batches = [wl.make_gas_batch(p, seed=0x5A + i) for i, p in enumerate((900, 300, 1500, 40))]
    c = pas_amd.Context(0)
    try:
        s0 = torch.cuda.current_stream()
        c.gas_snapshot_set_device(9, 6000, gs.used.shape[1], gs.used.shape[2],
                                  torch.from_numpy(gs.n_cards).cuda(),
                                  torch.from_numpy(gs.cap).cuda(),
                                  torch.from_numpy(gs.used).cuda(), s0)
        streams = [torch.cuda.Stream(), torch.cuda.Stream(), None]
        outs = []
        for rep in range(3):
            for i, b in enumerate(batches):
                s = streams[(rep + i) % 3]
                st = s if s is not None else s0
                st.wait_stream(s0)
                with torch.cuda.stream(st):
                    req = torch.from_numpy(b.req).cuda()
                    mask = torch.from_numpy(b.req_mask.view(np.int32)).cuda()
                    nc = torch.from_numpy(b.n_containers).cuda()
                    res = torch.empty((len(b.n_containers), 6000), dtype=torch.int32,
                                      device="cuda")
                c.gas_fit_device(9, len(b.n_containers), b.req.shape[1], wl.I915, req, mask, nc,
                                 res, stream=st)
                outs.append((i, res, st))
        torch.cuda.synchronize()
        want = [oracle.gas_fit(gs.n_cards, gs.cap, gs.used, b.req, b.req_mask, b.n_containers,
                               wl.I915) for b in batches]
        for i, res, _ in outs:
            np.testing.assert_array_equal(res.cpu().numpy().view(np.uint32), want[i])
    finally:
        c.close()
