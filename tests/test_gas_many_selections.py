"""GAS pods of more than PAS_GAS_MAX_SELECTIONS card selections, bit-exact against the oracle.

The reference loops `gpuNum < numI915` with no bound (gpu-aware-scheduling/pkg/gpuscheduler/
scheduler.go:213-247); with the GPU plugin's shared-dev-num (docs/gpu_plugin/overlays/
fractional_resources/add-args.yaml:11: 300 per card) one card takes hundreds of selections.
The kernels evaluate a container of more than 64 selections as card runs (csrc/gas_runs.h);
the oracle keeps the literal per-selection loop, so these tests check the two against each
other: fit words (bit 31 | PAS_GAS_SEL_LIMIT), bitmaps, the lazy C5 top-k, bind with the
selection as counts per container and card (pas_gas_bind_counts), release from counts
(pas_gas_release_counts) and the extender's annotation.  Marked gpu."""
import numpy as np
import pytest
import torch

import pas_amd
from pas_amd import _lib

pytestmark = pytest.mark.gpu
_gen = [40000]


def _upload(ctx, n_cards, cap, used):
    _gen[0] += 1
    ctx.gas_snapshot_set(_gen[0], n_cards, cap, used)
    return _gen[0]


def shared_case(rng, n, k, q, p, c, share=300, big_frac=0.5, max_sel=700):
    """Nodes whose cards take up to `share` i915 selections each (shared-dev-num), pods of
    which about big_frac request more than 64 selections in all (containers of up to max_sel),
    the rest 0-8.  Per-GPU amounts of the other kinds are small against the capacities, so the
    i915 count and the other kinds both bind."""
    n_cards = rng.integers(-1, k + 1, size=n).astype(np.int32)
    n_cards[rng.random(n) < 0.6] = k
    cap = rng.integers(2_000, 200_000, size=(n, q)).astype(np.int64)
    cap[:, 0] = rng.integers(1, share + 1, size=n)
    cap[rng.random((n, q)) < 0.03] = 0
    used = rng.integers(0, 2_000, size=(n, k, q)).astype(np.int64)
    used[:, :, 0] = rng.integers(0, share // 2 + 1, size=(n, k))
    req = np.zeros((p, c, q), np.int64)
    mask = rng.integers(0, 1 << q, size=(p, c)).astype(np.uint32)
    ncont = rng.integers(1, c + 1, size=p).astype(np.int32)
    for pi in range(p):
        big = rng.random() < big_frac
        for ci in range(ncont[pi]):
            num = int(rng.integers(0, max_sel + 1)) if big else int(rng.integers(0, 4))
            if num:
                mask[pi, ci] |= 1
            req[pi, ci, 0] = num
            # per-GPU amounts of 0-400 (after the divide by numI915)
            req[pi, ci, 1:] = rng.integers(0, 400, size=q - 1) * max(num, 1)
        if big and sum(int(req[pi, ci, 0]) for ci in range(ncont[pi])) <= 64:
            req[pi, 0, 0], mask[pi, 0] = 65 + int(rng.integers(0, 200)), mask[pi, 0] | 1
    return n_cards, cap, used, req, mask, ncont


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


@pytest.mark.parametrize("k,q", [(8, 3), (16, 2), (64, 2), (4, 4)])
def test_fit_parity(ctx, oracle, k, q):
    rng = np.random.default_rng(k * 10 + q)
    n_cards, cap, used, req, mask, ncont = shared_case(rng, 600, k, q, 48, 3)
    want = oracle.gas_fit(n_cards, cap, used, req, mask, ncont, 0)
    gen = _upload(ctx, n_cards, cap, used)
    got = ctx.gas_fit(gen, req, mask, ncont, 0)
    np.testing.assert_array_equal(got, want)
    limit = (want >> 24) & 15 == _lib.PAS_GAS_SEL_LIMIT
    assert limit.sum() > 100 and ((want[limit] >> 31) == 1).all()
    sel = np.array([sum(int(req[p, c, 0]) for c in range(ncont[p]) if mask[p, c] & 1)
                    for p in range(len(ncont))])
    assert ctx.gas_limit_count() == int((sel > 64).sum())
    # some big pods fit nowhere, some fit most nodes
    big = sel > 64
    assert 0.05 < (want[big] >> 31).mean() < 0.95
    # bitmaps
    p, c, _ = req.shape
    n = len(n_cards)
    fit_t = torch.zeros((p, (n + 63) // 64), dtype=torch.int64, device="cuda")
    ctx.gas_fit_bitmap_device(gen, p, c, 0, _dev(req), _dev(mask.view(np.int32)), _dev(ncont),
                              fit_t)
    ctx.synchronize()
    bits = np.unpackbits(fit_t.cpu().numpy().view(np.uint8), axis=1, bitorder="little")[:, :n]
    np.testing.assert_array_equal(bits, (want >> 31).astype(np.uint8))


def test_fit_extremes(ctx, oracle):
    # numI915 up to INT64_MAX per container, per-GPU needs of 0 (one card takes everything),
    # usage past capacity, zero capacities, unknown kinds on big containers
    rng = np.random.default_rng(99)
    n_cards, cap, used, req, mask, ncont = shared_case(rng, 300, 8, 3, 40, 3, max_sel=400)
    big = np.int64(2**63 - 1)
    req[0, 0, 0], req[0, 0, 1:], mask[0, 0] = big, 0, 1        # never fits (capacity runs out)
    req[1, :, :] = 0
    req[1, 0, 0], mask[1, 0], ncont[1] = 150, 1, 1             # needs 0 of every other kind
    req[2, 0, 0], mask[2, 0] = 2**40, 3                        # per-GPU need of kind 1 == 0
    req[3, 1, 0], mask[3, 1], ncont[3] = 100, 1 | 0x80000000, 2  # unknown kind: fits nowhere
    used[::7, :, 1] = cap[::7, None, 1] + 5                    # usage past capacity
    used[::11, 2, 2] = -1                                      # negative usage
    want = oracle.gas_fit(n_cards, cap, used, req, mask, ncont, 0)
    gen = _upload(ctx, n_cards, cap, used)
    np.testing.assert_array_equal(ctx.gas_fit(gen, req, mask, ncont, 0), want)
    assert (want[0] == 0).all() and (want[3] == 0).all()
    assert (want[1] >> 31).any()


@pytest.mark.parametrize("k", [8, 16, 64])
def test_bind_counts_and_release_counts_parity(ctx, oracle, k):
    rng = np.random.default_rng(500 + k)
    n_cards, cap, used, req, mask, ncont = shared_case(rng, 30, k, 3, 50, 3, max_sel=300)
    gen = _upload(ctx, n_cards, cap, used)
    pods = rng.integers(0, 50, size=120).astype(np.int32)
    nodes = rng.integers(0, 30, size=120).astype(np.int32)
    res, st, cnt = ctx.gas_bind(gen, gen + 1, pods, nodes, req, mask, ncont, 0, counts=True)
    w_used, w_res, w_st, w_cnt = oracle.gas_bind(n_cards, cap, used, req, mask, ncont, 0, pods,
                                                 nodes, counts=True)
    np.testing.assert_array_equal(res, w_res)
    np.testing.assert_array_equal(st, w_st)
    np.testing.assert_array_equal(cnt, w_cnt)
    _, after = ctx.gas_snapshot_get()
    np.testing.assert_array_equal(after, w_used)
    ok = st == _lib.PAS_GAS_OK
    assert ((res[ok] >> 24) & 15 == _lib.PAS_GAS_SEL_LIMIT).sum() >= 5
    assert cnt[ok].sum(axis=(1, 2)).max() > 64
    # the counts are the selections: per container, numI915 of them
    for b in np.nonzero(ok)[0]:
        for ci in range(ncont[pods[b]]):
            want_n = int(req[pods[b], ci, 0]) if mask[pods[b], ci] & 1 else 0
            assert cnt[b, ci].sum() == max(want_n, 0)
    # release the committed binds from their counts (one with a card past the node's cards)
    rel = np.nonzero(ok)[0][:60]
    rcnt = cnt[rel].copy()
    bad = None
    for i, b in enumerate(rel):
        nc = int(n_cards[nodes[b]])
        if 0 < nc < k and rcnt[i, 0].sum() > 0:
            rcnt[i, 0, nc] += 1  # a card the label does not list -> input error
            bad = i
            break
    st2 = ctx.gas_release_counts(gen + 1, gen + 2, pods[rel], nodes[rel], req, mask, ncont, rcnt)
    w_back, w_st2 = oracle.gas_release_counts(n_cards, w_used, req, mask, ncont, pods[rel],
                                              nodes[rel], rcnt)
    np.testing.assert_array_equal(st2, w_st2)
    if bad is not None:
        assert st2[bad] == _lib.PAS_GAS_ERR_INPUT
    _, back = ctx.gas_snapshot_get()
    np.testing.assert_array_equal(back, w_back)


def test_bind_ex_reports_counts_only_past_64(ctx, oracle):
    rng = np.random.default_rng(77)
    n_cards, cap, used, req, mask, ncont = shared_case(rng, 20, 8, 2, 30, 2, max_sel=200)
    gen = _upload(ctx, n_cards, cap, used)
    pods = np.arange(30, dtype=np.int32)
    nodes = rng.integers(0, 20, size=30).astype(np.int32)
    res, st, cards, nsel = ctx.gas_bind(gen, gen + 1, pods, nodes, req, mask, ncont, 0,
                                        selections=True)
    _, w_res, w_st, w_cards, w_nsel = oracle.gas_bind(n_cards, cap, used, req, mask, ncont, 0,
                                                      pods, nodes, selections=True)
    np.testing.assert_array_equal(res, w_res)
    np.testing.assert_array_equal(st, w_st)
    np.testing.assert_array_equal(nsel, w_nsel)
    np.testing.assert_array_equal(cards, w_cards)
    assert (nsel == -1).any() and (cards[nsel == -1] == 0).all()


def test_release_counts_errors(ctx):
    n_cards = np.array([2], np.int32)
    gen = _upload(ctx, n_cards, np.full((1, 1), 10, np.int64), np.zeros((1, 2, 1), np.int64))
    req = np.full((1, 1, 1), 4, np.int64)
    mask = np.ones((1, 1), np.uint32)
    one = np.ones(1, np.int32)
    for counts in (np.array([[[-1, 2]]]), np.array([[[2**62, 2**62]]])):
        with pytest.raises(pas_amd.PasError) as e:
            ctx.gas_release_counts(gen, gen + 1, [0], [0], req, mask, one, counts)
        assert e.value.code == _lib.PAS_EINVAL
    assert ctx.gas_snapshot_get()[0] == gen


def test_lazy_topk_with_many_selections(ctx):
    """pas_tas_gas_topk_device (card runs in lane_fit) equals fit bitmaps -> TAS top-k on a
    batch where half the pods make more than 64 selections."""
    from pas_amd import workload as wl
    from test_shard import _lazy_vs_composed, make_case
    n = 3000
    snap, batch = make_case(0x91, n, 6, 64, 7, cand_frac=0.8)
    rng = np.random.default_rng(0x91)
    nc, cap, used, req, mask, ncont = shared_case(rng, n, 8, 3, 64, 3, max_sel=400)
    gsnap, gbatch = wl.GasSnapshotData(nc, cap, used), wl.GasBatch(req, mask, ncont)
    composed, lazy = _lazy_vs_composed(ctx, snap.v_milli, snap.present, batch, gsnap, gbatch,
                                       None, 16, 0, 0)
    for a, b in zip(composed, lazy):
        np.testing.assert_array_equal(a, b)
    big = np.array([sum(int(req[p, c, 0]) for c in range(ncont[p]) if mask[p, c] & 1) > 64
                    for p in range(64)])
    assert (lazy[2][big] > 0).sum() >= 5


def test_extender_annotation_many_selections(ctx):
    """The GAS extender's bind annotates a 130-selection pod with every card, in container
    order (scheduler.go:317-335)."""
    import json
    from pas_amd import extender as ext
    from pas_amd import snapshot as sn
    kinds = ["gpu.intel.com/i915", "gpu.intel.com/millicores"]
    nodes = [{"labels": {"gpu.intel.com/cards": "card0.card1.card2"},
              "allocatable": {"gpu.intel.com/i915": "300", "gpu.intel.com/millicores": "3000"}}]
    n_cards, cap, used, card_names = sn.gas_snapshot_from_nodes(nodes, kinds)
    gen = _upload(ctx, n_cards, cap, used)
    pod = {"metadata": {"name": "p", "namespace": "default"},
           "spec": {"containers": [
               {"name": "a", "resources": {"requests": {"gpu.intel.com/i915": "130",
                                                        "gpu.intel.com/millicores": "1300"}}},
               {"name": "b", "resources": {"requests": {"gpu.intel.com/i915": "5",
                                                        "gpu.intel.com/millicores": "50"}}}]}}
    g = ext.GASExtender(ctx, gen, ["n0"], card_names, kinds, {("default", "p"): pod})
    code, _ = g.bind(json.dumps({"PodName": "p", "PodNamespace": "default", "PodUID": "",
                                 "Node": "n0"}).encode())
    assert code == 200
    first, second = pod["metadata"]["annotations"]["gas-container-cards"].split("|")
    # per-GPU capacity 100 i915 / 1000 millicores: card0 takes 100 selections of 10 m, card1
    # the other 30; the second container continues on card1
    assert first.split(",") == ["card0"] * 100 + ["card1"] * 30
    assert second.split(",") == ["card1"] * 5
