"""GAS beyond the packed word: pods with 9..64 card selections and nodes with 9..64 cards
(gas_fit_generic_kernel), bit-exact against the oracle's full selections (words, side records
of PAS_GAS_SEL_EXTENDED words, bitmaps), the PAS_GAS_SEL_LIMIT words past 64 selections,
and bind / release of wide annotations (pas_gas_bind_ex / pas_gas_release_ex).

The reference has no such limits (scheduler.go:200-257 loops over every gpuNum and card); the
GPU plugin's shared-dev-num makes one card take many selections, which is what the per-GPU
i915 capacities > 1 below model.  Marked gpu."""
import numpy as np
import pytest
import torch

import pas_amd
from pas_amd import _lib

pytestmark = pytest.mark.gpu
_gen = [20000]


def _upload(ctx, n_cards, cap, used):
    _gen[0] += 1
    ctx.gas_snapshot_set(_gen[0], n_cards, cap, used)
    return _gen[0]


def random_wide(rng, n, k, q, p, c, sel_max, share=4):
    """Nodes of up to k cards, pods of up to sel_max selections (i915 column 0, per-GPU i915
    capacity 1..share so that cards are shared), usages leaving a good share of fits."""
    n_cards = rng.integers(-1, k + 1, size=n).astype(np.int32)
    n_cards[rng.random(n) < 0.5] = k  # many full-width nodes
    cap = rng.integers(500, 2000, size=(n, q)).astype(np.int64)
    cap[:, 0] = rng.integers(1, share + 1, size=n)
    used = rng.integers(0, 400, size=(n, k, q)).astype(np.int64)
    used[:, :, 0] = rng.integers(0, 2, size=(n, k))
    req = rng.integers(0, 300, size=(p, c, q)).astype(np.int64)
    mask = rng.integers(0, 1 << q, size=(p, c)).astype(np.uint32) | 1
    ncont = rng.integers(1, c + 1, size=p).astype(np.int32)
    for pi in range(p):
        total = int(rng.integers(0, sel_max + 1))
        split = np.sort(rng.integers(0, total + 1, size=ncont[pi] - 1))
        counts = np.diff(np.concatenate([[0], split, [total]]))
        req[pi, :ncont[pi], 0] = counts
        req[pi, :ncont[pi], 1:] *= np.maximum(counts, 1)[:, None]  # per-GPU amounts stay sane
    return n_cards, cap, used, req, mask, ncont


def check_fit_ex(ctx, oracle, n_cards, cap, used, req, mask, ncont, i915=0):
    gen = _upload(ctx, n_cards, cap, used)
    want, w_sel, w_nsel = oracle.gas_fit(n_cards, cap, used, req, mask, ncont, i915,
                                         selections=True)
    got, side = ctx.gas_fit_ex(gen, req, mask, ncont, i915, side_cap=16)
    np.testing.assert_array_equal(got, want)
    ext = np.argwhere((want >> 24) & 15 == oracle.SEL_EXTENDED)
    assert len(side) == len(ext)
    if len(ext):
        np.testing.assert_array_equal(side["pod"], ext[:, 0])
        np.testing.assert_array_equal(side["node"], ext[:, 1])
        np.testing.assert_array_equal(side["n_sel"], w_nsel[ext[:, 0], ext[:, 1]])
        np.testing.assert_array_equal(side["card"], w_sel[ext[:, 0], ext[:, 1]])
    # the plain host call gives the same words
    np.testing.assert_array_equal(ctx.gas_fit(gen, req, mask, ncont, i915), want)
    return gen, want, ext


@pytest.mark.parametrize("sel_max", [12, 16])
def test_wide_selections_parity(ctx, oracle, sel_max):
    # pods of 9..16 selections on 8-card nodes: the fast kernels leave them to the generic
    # path, which writes PAS_GAS_SEL_EXTENDED words and side records
    rng = np.random.default_rng(sel_max)
    args = random_wide(rng, 700, 8, 3, 40, 4, sel_max)
    _, want, ext = check_fit_ex(ctx, oracle, *args)
    assert len(ext) > 50
    assert 0.1 < (want >> 31).mean() < 0.95


@pytest.mark.parametrize("k", [9, 12, 16, 64])
def test_wide_cards_parity(ctx, oracle, k):
    # nodes of 9..64 cards next to narrow ones, pods of 0..12 selections: selections that land
    # on card ranks >= 8 do not pack either
    rng = np.random.default_rng(100 + k)
    args = random_wide(rng, 500, k, 2, 48, 3, 12, share=2)
    _, want, ext = check_fit_ex(ctx, oracle, *args)
    assert len(ext) > 20
    assert 0.1 < (want >> 31).mean() < 0.95


def test_wide_device_paths(ctx, oracle):
    # the _device calls: ex words + side records + count on the device, bitmaps with the wide
    # pairs or-ed in, and pods past 64 selections (PAS_GAS_SEL_LIMIT words) counted
    rng = np.random.default_rng(7)
    n_cards, cap, used, req, mask, ncont = random_wide(rng, 300, 12, 2, 30, 3, 16)
    req[5, :, 0] = 0
    req[5, 0, 0] = 40
    req[5, 1, 0] = 25  # 65 selections
    mask[5, :2] |= 1
    ncont[5] = max(ncont[5], 2)
    req[9, 0, 0] = 2**62  # a wrapping sum of i915 requests saturates, not wraps
    req[9, 1, 0] = 2**62
    mask[9, :2] |= 1
    ncont[9] = max(ncont[9], 2)
    cap[:60, 0] = 40  # shared-dev-num: some nodes take pod 5's 65 selections
    want, w_sel, w_nsel = oracle.gas_fit(n_cards, cap, used, req, mask, ncont, 0,
                                         selections=True)
    fits5 = want[5] >> 31 == 1
    assert fits5.any() and ((want[5][fits5] >> 24) & 15 == oracle.SEL_LIMIT).all()
    assert (want[9] == 0).all()  # 2^63 selections: capacity runs out
    gen = _upload(ctx, n_cards, cap, used)
    np.testing.assert_array_equal(ctx.gas_fit(gen, req, mask, ncont, 0), want)
    dev = torch.device("cuda", 0)
    p, c, q = req.shape
    n = len(n_cards)
    req_t = torch.from_numpy(req).to(dev)
    mask_t = torch.from_numpy(mask.view(np.int32)).to(dev)
    ncont_t = torch.from_numpy(ncont).to(dev)
    res_t = torch.empty((p, n), dtype=torch.int32, device=dev)
    cap_side = 4096
    side_t = torch.zeros((cap_side, _lib.GAS_SELECTION_DTYPE.itemsize), dtype=torch.uint8,
                         device=dev)
    count_t = torch.zeros(1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream()
    ctx.gas_fit_ex_device(gen, p, c, 0, req_t, mask_t, ncont_t, res_t, side_t, cap_side,
                          count_t, stream)
    torch.cuda.synchronize()
    got = res_t.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got, want)
    assert ctx.gas_limit_count() == 2
    ext = np.argwhere((want >> 24) & 15 == oracle.SEL_EXTENDED)
    count = int(count_t.item())
    assert count == len(ext) and 0 < count <= cap_side
    side = side_t[:count].cpu().numpy().view(_lib.GAS_SELECTION_DTYPE).reshape(-1)
    side = side[np.lexsort((side["node"], side["pod"]))]
    np.testing.assert_array_equal(side["pod"], ext[:, 0])
    np.testing.assert_array_equal(side["node"], ext[:, 1])
    np.testing.assert_array_equal(side["card"], w_sel[ext[:, 0], ext[:, 1]])
    # a too-small side buffer: the count still reports every record
    ctx.gas_fit_ex_device(gen, p, c, 0, req_t, mask_t, ncont_t, res_t, side_t, 3, count_t,
                          stream)
    torch.cuda.synchronize()
    assert int(count_t.item()) == count
    # bitmaps
    w = (n + 63) // 64
    fit_t = torch.zeros((p, w), dtype=torch.int64, device=dev)
    ctx.gas_fit_bitmap_device(gen, p, c, 0, req_t, mask_t, ncont_t, fit_t, stream)
    torch.cuda.synchronize()
    bits = np.unpackbits(fit_t.cpu().numpy().view(np.uint8), axis=1,
                         bitorder="little")[:, :n]
    np.testing.assert_array_equal(bits, (want >> 31).astype(np.uint8))
    assert ctx.gas_limit_count() == 2
    # a batch without such pods resets the count
    ncont2 = ncont.copy()
    ncont2[[5, 9]] = 0
    ctx.gas_fit_device(gen, p, c, 0, req_t, mask_t, torch.from_numpy(ncont2).to(dev), res_t,
                       stream)
    assert ctx.gas_limit_count() == 0


@pytest.mark.parametrize("k,sel_max", [(8, 14), (16, 10), (64, 16)])
def test_wide_bind_release_parity(ctx, oracle, k, sel_max):
    # bind_ex returns the full selection; release_ex takes 64-card annotations back out
    rng = np.random.default_rng(k * 3 + sel_max)
    n_cards, cap, used, req, mask, ncont = random_wide(rng, 40, k, 2, 60, 3, sel_max)
    gen = _upload(ctx, n_cards, cap, used)
    pods = rng.integers(0, 60, size=150).astype(np.int32)
    nodes = rng.integers(0, 30, size=150).astype(np.int32)
    res, st, cards, nsel = ctx.gas_bind(gen, gen + 1, pods, nodes, req, mask, ncont, 0,
                                        selections=True)
    w_used, w_res, w_st, w_cards, w_nsel = oracle.gas_bind(n_cards, cap, used, req, mask, ncont,
                                                           0, pods, nodes, selections=True)
    np.testing.assert_array_equal(res, w_res)
    np.testing.assert_array_equal(st, w_st)
    np.testing.assert_array_equal(nsel, w_nsel)
    np.testing.assert_array_equal(cards, w_cards)
    assert ((res >> 24) & 15 == oracle.SEL_EXTENDED).sum() >= 3
    _, after = ctx.gas_snapshot_get()
    np.testing.assert_array_equal(after, w_used)
    ok = np.nonzero(st == 0)[0][:80]
    c = req.shape[1]
    cpc = np.zeros((len(ok), c), np.int32)
    rel = np.full((len(ok), 64), -1, np.int32)
    for i, b in enumerate(ok):
        p = pods[b]
        for ci in range(ncont[p]):
            cpc[i, ci] = max(int(req[p, ci, 0]), 0) if mask[p, ci] & 1 else 0
        rel[i, :nsel[b]] = cards[b, :nsel[b]]
    if len(ok) > 3:
        rel[1, 0] = k + 1  # a card the node does not have -> input error
    st2 = ctx.gas_release(gen + 1, gen + 2, pods[ok], nodes[ok], req, mask, ncont, cpc, rel)
    w_back, w_st2 = oracle.gas_release(n_cards, w_used, req, mask, ncont, pods[ok], nodes[ok],
                                       cpc, rel)
    np.testing.assert_array_equal(st2, w_st2)
    _, back = ctx.gas_snapshot_get()
    np.testing.assert_array_equal(back, w_back)


def test_selection_sum_past_int64(ctx, oracle):
    # two containers requesting 2^62 i915 each: evaluated (no wrap), no fit
    n_cards = np.array([2], np.int32)
    cap, used = np.full((1, 1), 10, np.int64), np.zeros((1, 2, 1), np.int64)
    gen = _upload(ctx, n_cards, cap, used)
    req = np.full((1, 2, 1), 2**62, np.int64)
    mask = np.ones((1, 2), np.uint32)
    two = np.array([2], np.int32)
    want = oracle.gas_fit(n_cards, cap, used, req, mask, two, 0)
    assert want[0, 0] == 0
    np.testing.assert_array_equal(ctx.gas_fit(gen, req, mask, two, 0), want)
    res, st = ctx.gas_bind(gen, gen + 1, [0], [0], req, mask, two, 0)
    assert res[0] == 0 and st[0] == _lib.PAS_GAS_WONT_FIT


@pytest.mark.parametrize("extra", [0, 7, 48])
def test_result_row_pitch(ctx, oracle, extra):
    # pas_gas_fit_ld_device: rows at a pitch ld >= N (here N + extra, and N rounded up to 32
    # words) hold the dense words; the padding is not written.  Wide nodes (generic kernel),
    # pods past 8 selections (generic) and the ranked fast kernels all honour the pitch.
    rng = np.random.default_rng(11 + extra)
    n_cards, cap, used, req, mask, ncont = random_wide(rng, 1000, 12, 3, 200, 3, 12)
    want, w_sel, _ = oracle.gas_fit(n_cards, cap, used, req, mask, ncont, 0, selections=True)
    gen = _upload(ctx, n_cards, cap, used)
    dev = torch.device("cuda", 0)
    p, c, q = req.shape
    n = len(n_cards)
    ld = n + extra if extra else (n + 31) // 32 * 32 + 32
    req_t = torch.from_numpy(req).to(dev)
    mask_t = torch.from_numpy(mask.view(np.int32)).to(dev)
    ncont_t = torch.from_numpy(ncont).to(dev)
    res_t = torch.full((p, ld), -0x21524111, dtype=torch.int32, device=dev)  # 0xDEADBEEF
    cap_side = 1 << 16
    side_t = torch.zeros((cap_side, _lib.GAS_SELECTION_DTYPE.itemsize), dtype=torch.uint8,
                         device=dev)
    count_t = torch.zeros(1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream()
    ctx.gas_fit_ld_device(gen, p, c, 0, req_t, mask_t, ncont_t, res_t, ld, side_t, cap_side,
                          count_t, stream)
    torch.cuda.synchronize()
    got = res_t.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got[:, :n], want)
    assert (got[:, n:] == 0xDEADBEEF).all()
    ext = np.argwhere((want >> 24) & 15 == oracle.SEL_EXTENDED)
    count = int(count_t.item())
    assert count == len(ext)
    side = side_t[:count].cpu().numpy().view(_lib.GAS_SELECTION_DTYPE).reshape(-1)
    side = side[np.lexsort((side["node"], side["pod"]))]
    np.testing.assert_array_equal(side["card"], w_sel[ext[:, 0], ext[:, 1]])
    # no side buffer
    res_t.fill_(-0x21524111)
    ctx.gas_fit_ld_device(gen, p, c, 0, req_t, mask_t, ncont_t, res_t, ld, stream=stream)
    torch.cuda.synchronize()
    got = res_t.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got[:, :n], want)
    assert (got[:, n:] == 0xDEADBEEF).all()
    with pytest.raises(pas_amd.PasError):
        ctx.gas_fit_ld_device(gen, p, c, 0, req_t, mask_t, ncont_t, res_t, n - 1, stream=stream)


@pytest.mark.parametrize("past", [False, True])
def test_result_batches_either_side_of_2gib(ctx, oracle, past):
    """Word results of < 2^31 bytes are stored through one buffer descriptor with the row
    offset as the store's scalar offset (gas_fit.hip, ResSoff); a batch of >= 2^31 bytes (here
    through a pitch of ~2.7M words) takes the per-row descriptors.  Same words either way, the
    padding untouched (its last column included)."""
    rng = np.random.default_rng(77)
    n_cards, cap, used, req, mask, ncont = random_wide(rng, 1000, 8, 3, 200, 3, 8)
    want = oracle.gas_fit(n_cards, cap, used, req, mask, ncont, 0)
    gen = _upload(ctx, n_cards, cap, used)
    dev = torch.device("cuda", 0)
    p, c, _ = req.shape
    n = len(n_cards)
    ld = (1 << 31) // (4 * p) + 64 if past else n + 96
    assert (p * ld * 4 >= 1 << 31) == past
    res_t = torch.full((p, ld), -0x21524111, dtype=torch.int32, device=dev)  # 0xDEADBEEF
    stream = torch.cuda.current_stream()
    ctx.gas_fit_ld_device(gen, p, c, 0, torch.from_numpy(req).to(dev),
                          torch.from_numpy(mask.view(np.int32)).to(dev),
                          torch.from_numpy(ncont).to(dev), res_t, ld, stream=stream)
    torch.cuda.synchronize()
    got = res_t[:, : n + 64].cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got[:, :n], want)
    assert (got[:, n:] == 0xDEADBEEF).all()
    assert (res_t[:, -1].cpu().numpy().view(np.uint32) == 0xDEADBEEF).all()
    del res_t
    torch.cuda.empty_cache()
