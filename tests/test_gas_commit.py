"""GAS bind-time commit (GASExtender.bindNode, scheduler.go:385-445, and
Cache.adjustPodResources, node_resource_cache.go:187-287) patched into the resident snapshot.
The oracle's bind/release are pinned by the README worked example (G11: pods bound in turn)
and by the resourceMap vectors (G9); the GPU path is checked against the oracle, bit-exact
in the usage it leaves, the words it returns and the statuses."""
import numpy as np
import pytest

import pas_amd
from pas_amd import workload as wl
from helpers import decode_gas_word, golden
from test_gas_gpu import random_gas
from test_oracle_golden import commit_pod, gas_readme_case

G = golden()


def annotation_cards(word, req, mask, ncont, i915):
    """cards_per_container / cards of a bind result word (the gas-container-cards
    annotation: container c takes its numI915 selections, in order)."""
    c_max = req.shape[0]
    cpc = np.zeros(c_max, np.int32)
    cards = np.full(8, -1, np.int32)
    _, sel = decode_gas_word(word)
    j = 0
    for c in range(ncont):
        n = 0
        if mask[c] and i915 >= 0 and (mask[c] >> i915) & 1 and req[c, i915] > 0:
            n = int(req[c, i915])
        cpc[c] = n
        cards[j:j + n] = sel[j:j + n]
        j += n
    return cpc, cards


# ------------------------------------------------------------------ oracle (CPU)

def test_oracle_bind_readme_in_turn(oracle):
    # README.md:15-21: three 5 GB pods bound in turn on a 2-GPU 16 GB node -> card0, card1,
    # then no fit; the usage after the binds is the README's accounting
    ex = G["G11_gas_readme"]["memory_example"]
    kinds, cards, n_cards, cap, used, req, mask = gas_readme_case(ex)
    req3 = np.repeat(req, 3, axis=0)
    mask3 = np.repeat(mask, 3, axis=0)
    after, res, st = oracle.gas_bind(n_cards, cap, used, req3, mask3, np.ones(3, np.int32), 0,
                                     [0, 1, 2], [0, 0, 0])
    got = []
    for w in res:
        fits, sel = decode_gas_word(w)
        got.append({"fits": True, "annotation": ",".join(cards[k] for k in sel)} if fits
                   else {"fits": False})
    assert got == ex["want"]
    assert list(st) == [0, 0, 1]
    want = used.copy()
    commit_pod(want[0], req[0], mask[0], [[0]])
    commit_pod(want[0], req[0], mask[0], [[1]])
    np.testing.assert_array_equal(after, want)


def test_oracle_bind_then_release_restores(oracle):
    rng = np.random.default_rng(21)
    n_cards, cap, used, req, mask, ncont = random_gas(rng, 40, 4, 3, 30, 3, i915=0)
    pods = np.arange(30, dtype=np.int32)
    nodes = rng.integers(0, 40, size=30).astype(np.int32)
    after, res, st = oracle.gas_bind(n_cards, cap, used, req, mask, ncont, 0, pods, nodes)
    ok = np.nonzero(st == 0)[0]
    assert len(ok) > 0
    cpc = np.zeros((len(ok), req.shape[1]), np.int32)
    cards = np.zeros((len(ok), 8), np.int32)
    for i, b in enumerate(ok):
        cpc[i], cards[i] = annotation_cards(res[b], req[b], mask[b], ncont[b], 0)
    back, st2 = oracle.gas_release(n_cards, after, req, mask, ncont, pods[ok], nodes[ok], cpc,
                                   cards)
    assert (st2 == 0).all()
    # add then subtract of the same shares restores every kind that did not clamp
    np.testing.assert_array_equal(back, used)


def test_oracle_release_errors(oracle):
    # subtractRM: negative amount -> errInput; a card the node does not have -> errInput;
    # results below zero clamp (resource_map.go:103-127)
    n_cards = np.array([2], np.int32)
    used = np.array([[[5, 10], [0, 0]]], np.int64)
    req = np.array([[[4, 30]], [[-1, 0]], [[1, 1]]], np.int64)
    mask = np.array([[3], [3], [3]], np.uint32)
    ncont = np.ones(3, np.int32)
    cpc = np.ones((3, 1), np.int32)
    cards = np.array([[0] + [0] * 7, [0] + [0] * 7, [5] + [0] * 7], np.int32)
    after, st = oracle.gas_release(n_cards, used, req, mask, ncont, [0, 1, 2], [0, 0, 0], cpc,
                                   cards)
    assert list(st) == [0, 2, 2]
    np.testing.assert_array_equal(after[0, 0], [1, 0])  # 10 - 30 clamps to 0


# ------------------------------------------------------------------ device (GPU)

_gen = [9000]


def _upload(ctx, n_cards, cap, used):
    _gen[0] += 1
    ctx.gas_snapshot_set(_gen[0], n_cards, cap, used)
    return _gen[0]


@pytest.mark.gpu
def test_bind_readme_in_turn(ctx, oracle):
    ex = G["G11_gas_readme"]["memory_example"]
    kinds, cards, n_cards, cap, used, req, mask = gas_readme_case(ex)
    gen = _upload(ctx, n_cards, cap, used)
    req3, mask3 = np.repeat(req, 3, axis=0), np.repeat(mask, 3, axis=0)
    res, st = ctx.gas_bind(gen, gen + 1, [0, 1, 2], [0, 0, 0], req3, mask3,
                           np.ones(3, np.int32), 0)
    assert list(st) == [pas_amd._lib.PAS_GAS_OK, pas_amd._lib.PAS_GAS_OK,
                        pas_amd._lib.PAS_GAS_WONT_FIT]
    assert [",".join(cards[k] for k in decode_gas_word(w)[1]) for w in res[:2]] == \
        ["card0", "card1"]
    g, after = ctx.gas_snapshot_get()
    assert g == gen + 1
    want, _, _ = oracle.gas_bind(n_cards, cap, used, req3, mask3, np.ones(3, np.int32), 0,
                                 [0, 1, 2], [0, 0, 0])
    np.testing.assert_array_equal(after, want)


@pytest.mark.gpu
@pytest.mark.parametrize("q,k", [(1, 1), (3, 8), (4, 3), (2, 8)])
def test_bind_release_parity(ctx, oracle, q, k):
    rng = np.random.default_rng(31 * q + k)
    for extreme in (False, True):
        i915 = 0
        n_cards, cap, used, req, mask, ncont = random_gas(rng, 60, k, q, 80, 4, extreme, i915)
        gen = _upload(ctx, n_cards, cap, used)
        pods = rng.integers(0, 80, size=200).astype(np.int32)
        nodes = rng.integers(0, 12, size=200).astype(np.int32)  # many binds per node
        res, st = ctx.gas_bind(gen, gen + 1, pods, nodes, req, mask, ncont, i915)
        w_used, w_res, w_st = oracle.gas_bind(n_cards, cap, used, req, mask, ncont, i915, pods,
                                              nodes)
        np.testing.assert_array_equal(res, w_res)
        np.testing.assert_array_equal(st, w_st)
        _, after = ctx.gas_snapshot_get()
        np.testing.assert_array_equal(after, w_used)
        # a fit batch after the binds == the oracle's fit on the committed usage
        got = ctx.gas_fit(gen + 1, req, mask, ncont, i915)
        np.testing.assert_array_equal(got, oracle.gas_fit(n_cards, cap, w_used, req, mask, ncont,
                                                          i915))
        # release the bound pods (their annotations) plus invalid cards / negative requests
        ok = np.nonzero(st == 0)[0][:60]
        cpc = np.zeros((len(ok), req.shape[1]), np.int32)
        cards = np.zeros((len(ok), 8), np.int32)
        for i, b in enumerate(ok):
            cpc[i], cards[i] = annotation_cards(res[b], req[pods[b]], mask[pods[b]],
                                                ncont[pods[b]], i915)
        if len(ok) > 2:
            cards[0, 0] = 7 if k < 8 else -1  # beyond the node's cards
        st2 = ctx.gas_release(gen + 1, gen + 2, pods[ok], nodes[ok], req, mask, ncont, cpc,
                              cards)
        w_back, w_st2 = oracle.gas_release(n_cards, w_used, req, mask, ncont, pods[ok], nodes[ok],
                                           cpc, cards)
        np.testing.assert_array_equal(st2, w_st2)
        _, back = ctx.gas_snapshot_get()
        np.testing.assert_array_equal(back, w_back)


@pytest.mark.gpu
def test_bind_c3_scale(ctx, oracle):
    # C3 snapshot (50k nodes x 8 cards): 4096 binds spread over the cluster
    snap = wl.make_gas_snapshot(50_000, seed=0xC3)
    batch = wl.make_gas_batch(4096, seed=0xC3)
    gen = _upload(ctx, snap.n_cards, snap.cap, snap.used)
    rng = np.random.default_rng(5)
    pods = np.arange(4096, dtype=np.int32)
    nodes = rng.integers(0, 50_000, size=4096).astype(np.int32)
    res, st = ctx.gas_bind(gen, gen + 1, pods, nodes, batch.req, batch.req_mask,
                           batch.n_containers, wl.I915)
    w_used, w_res, w_st = oracle.gas_bind(snap.n_cards, snap.cap, snap.used, batch.req,
                                          batch.req_mask, batch.n_containers, wl.I915, pods,
                                          nodes)
    np.testing.assert_array_equal(res, w_res)
    np.testing.assert_array_equal(st, w_st)
    _, after = ctx.gas_snapshot_get()
    np.testing.assert_array_equal(after, w_used)


@pytest.mark.gpu
def test_bind_errors(ctx):
    n_cards = np.array([2, 2], np.int32)
    cap = np.full((2, 1), 10, np.int64)
    used = np.zeros((2, 2, 1), np.int64)
    gen = _upload(ctx, n_cards, cap, used)
    req = np.array([[[9]]], np.int64)
    mask = np.array([[1]], np.uint32)
    one = np.ones(1, np.int32)
    for kw, code in [(dict(gen_from=gen - 1, nodes=[0]), pas_amd._lib.PAS_ESTALE),
                     (dict(gen_from=gen, nodes=[2]), pas_amd._lib.PAS_EINVAL)]:
        with pytest.raises(pas_amd.PasError) as e:
            ctx.gas_bind(kw["gen_from"], gen + 1, [0], kw["nodes"], req, mask, one, 0)
        assert e.value.code == code
    # more than 64 selections are evaluated: 65 do not fit 2 cards of capacity 10
    res, st = ctx.gas_bind(gen, gen + 1, [0], [0], np.array([[[65]]], np.int64), mask, one, 0)
    assert st[0] == pas_amd._lib.PAS_GAS_WONT_FIT and res[0] == 0
    assert ctx.gas_snapshot_get()[0] == gen + 1


@pytest.mark.gpu
def test_fit_bind_fit_refreshes_kind_minima(ctx, oracle):
    # The fit caches each kind's minimum free over the snapshot per epoch (kind skipping,
    # gas_fit.hip).  Fit, then binds that exhaust card0's i915 on node 0 (the minimum drops
    # from 2 to 0), then fit again on the same context: a stale minimum would skip the i915
    # compare and pick card0; the reference picks card1.  Release restores it.
    n_cards = np.full(4, 2, np.int32)
    cap = np.tile(np.array([[2, 1000]], np.int64), (4, 1))
    used = np.zeros((4, 2, 2), np.int64)
    req = np.array([[[1, 10]]], np.int64)
    mask = np.array([[3]], np.uint32)
    ncont = np.ones(1, np.int32)
    gen = _upload(ctx, n_cards, cap, used)
    before = ctx.gas_fit(gen, req, mask, ncont, 0)
    assert decode_gas_word(before[0, 0]) == (True, [0])
    res, st = ctx.gas_bind(gen, gen + 1, [0, 0], [0, 0], req, mask, ncont, 0)
    assert list(st) == [0, 0]
    w_used, _, _ = oracle.gas_bind(n_cards, cap, used, req, mask, ncont, 0, [0, 0], [0, 0])
    after = ctx.gas_fit(gen + 1, req, mask, ncont, 0)
    want = oracle.gas_fit(n_cards, cap, w_used, req, mask, ncont, 0)
    assert decode_gas_word(want[0, 0]) == (True, [1])
    np.testing.assert_array_equal(after, want)
    cpc = np.ones((2, 1), np.int32)
    cards = np.zeros((2, 8), np.int32)
    st2 = ctx.gas_release(gen + 1, gen + 2, [0, 0], [0, 0], req, mask, ncont, cpc, cards)
    assert list(st2) == [0, 0]
    again = ctx.gas_fit(gen + 2, req, mask, ncont, 0)
    np.testing.assert_array_equal(again, before)


@pytest.mark.gpu
def test_unknown_kind_bind_release(ctx, oracle):
    # a container flagged PAS_REQ_UNKNOWN_KIND (a gpu.intel.com/ kind the snapshot lacks):
    # with numI915 > 0 the bind does not fit; with numI915 == 0 it binds with no cards; a
    # release naming cards for such a container is errInput (subtractRM of a missing key)
    unk = pas_amd._lib.PAS_REQ_UNKNOWN_KIND
    n_cards = np.full(3, 2, np.int32)
    cap = np.tile(np.array([[4, 1000]], np.int64), (3, 1))
    used = np.zeros((3, 2, 2), np.int64)
    req = np.array([[[1, 10], [0, 0]], [[0, 5], [1, 10]], [[1, 10], [1, 5]]], np.int64)
    mask = np.array([[3 | unk, 0], [2 | unk, 3], [3, 3]], np.uint32)
    ncont = np.array([1, 2, 2], np.int32)
    gen = _upload(ctx, n_cards, cap, used)
    pods, nodes = [0, 1, 2], [0, 1, 2]
    res, st = ctx.gas_bind(gen, gen + 1, pods, nodes, req, mask, ncont, 0)
    w_used, w_res, w_st = oracle.gas_bind(n_cards, cap, used, req, mask, ncont, 0, pods, nodes)
    assert list(w_st) == [pas_amd._lib.PAS_GAS_WONT_FIT, 0, 0]
    np.testing.assert_array_equal(res, w_res)
    np.testing.assert_array_equal(st, w_st)
    _, after = ctx.gas_snapshot_get()
    np.testing.assert_array_equal(after, w_used)
    rel_mask = mask.copy()
    rel_mask[2, 0] |= unk  # the annotation names a card for a flagged container
    cpc = np.array([[0, 1], [1, 1]], np.int32)
    cards = np.zeros((2, 8), np.int32)
    st2 = ctx.gas_release(gen + 1, gen + 2, [1, 2], [1, 2], req, rel_mask, ncont, cpc, cards)
    w_back, w_st2 = oracle.gas_release(n_cards, w_used, req, rel_mask, ncont, [1, 2], [1, 2], cpc,
                                       cards)
    assert list(w_st2) == [0, pas_amd._lib.PAS_GAS_ERR_INPUT]
    np.testing.assert_array_equal(st2, w_st2)
    _, back = ctx.gas_snapshot_get()
    np.testing.assert_array_equal(back, w_back)
