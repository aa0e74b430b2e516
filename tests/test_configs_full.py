"""BASELINE configs at their full bench sizes, checked against the oracle (marked gpu, slow).

* C3 (configs[2]): the whole 10k-pod x 50k-node GAS batch the bench times, every
  (pod, node) word bit-exact against oracle.gas_fit (scheduler.go:280-383), and the fit
  bitmaps of pas_gas_fit_bitmap_device equal to bit 31 of the words.
* C5 (configs[4]): 64k pods x 1M nodes, TAS + GAS combined: each node range keeps its
  pods' first k HostPriorityList entries over the nodes that pass TAS and fit GAS, and the
  ranges are merged (pas_topk_merge_device).  Two ways to a range's records: the GAS fit
  bitmaps as TAS candidates of pas_tas_topk_device (every (pod, node) evaluated), and
  pas_tas_gas_topk_device (bench.py's step: evaluated along each pod's order until k are
  kept).  Checked
    - for a 128-pod sample, bit-exact against the oracle composition oracle.gas_fit ->
      candidate bitmap -> oracle.tas_eval (telemetryscheduler.go:128-149,184-225) -> first k;
    - for all 65,536 pods: the 8-range merge equals the whole-cluster (one range) lists, the
      lazy path equals the composed one (1 and 8 ranges), and
      len = min(k, |fit AND pass AND present|), entries unique, every entry fits / passes /
      has the metric, order ascending in (key, node) (the documented tie rule, pas.h).
The collectives of the multi-rank path are covered over gloo in test_shard.py; here the
ranges are simulated as separate contexts on one GPU.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

import pas_amd
from pas_amd import workload as wl
from pas_amd.shard import node_range
from helpers import unpack_bits

pytestmark = [pytest.mark.gpu, pytest.mark.slow]
THREADS = max(1, min(16, os.cpu_count() or 1))


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _chunks(n, per):
    return [(lo, min(n, lo + per)) for lo in range(0, n, per)]


def popcount64(x):
    """Per-element popcount of an int64 tensor (SWAR on the device)."""
    x = x - ((x >> 1) & 0x5555555555555555)
    x = (x & 0x3333333333333333) + ((x >> 2) & 0x3333333333333333)
    x = (x + (x >> 4)) & 0x0F0F0F0F0F0F0F0F
    return (x * 0x0101010101010101) >> 56 & 0x7F


def test_popcount64_helper():
    v = np.array([0, 1, -1, 2**62, 0x5555555555555555, -(2**63)], np.int64)
    got = popcount64(torch.from_numpy(v)).numpy()
    assert list(got) == [bin(int(x) & (2**64 - 1)).count("1") for x in v]


def test_c3_full_batch(ctx, oracle):
    snap = wl.make_gas_snapshot(50_000, seed=0xC3)
    batch = wl.make_gas_batch(10_000, seed=0xC3)
    P, N = 10_000, 50_000
    K, Q = snap.used.shape[1], snap.used.shape[2]
    C = batch.req.shape[1]
    s = torch.cuda.current_stream()
    ctx.gas_snapshot_set_device(71, N, K, Q, _dev(snap.n_cards), _dev(snap.cap), _dev(snap.used),
                                s)
    req_t, mask_t = _dev(batch.req), _dev(batch.req_mask.view(np.int32))
    nc_t = _dev(batch.n_containers)
    res_t = torch.empty((P, N), dtype=torch.int32, device="cuda")
    ctx.gas_fit_device(71, P, C, wl.I915, req_t, mask_t, nc_t, res_t, s)
    fit_t = torch.empty((P, pas_amd.w64(N)), dtype=torch.int64, device="cuda")
    ctx.gas_fit_bitmap_device(71, P, C, wl.I915, req_t, mask_t, nc_t, fit_t, s)
    torch.cuda.synchronize()
    # fit bitmaps = bit 31 of the words, for the whole batch (on the device)
    bits = ((res_t >> 31) & 1).to(torch.uint8)
    pad = pas_amd.w64(N) * 64 - N
    bits = torch.nn.functional.pad(bits, (0, pad)).view(P, -1, 64).to(torch.int64)
    words = (bits << torch.arange(64, device="cuda")).sum(dim=2)
    assert torch.equal(words, fit_t)
    got = res_t.cpu().numpy().view(np.uint32)
    del res_t, fit_t, bits, words

    def check(lo, hi):
        want = oracle.gas_fit(snap.n_cards, snap.cap, snap.used, batch.req[lo:hi],
                              batch.req_mask[lo:hi], batch.n_containers[lo:hi], wl.I915)
        return lo if np.array_equal(got[lo:hi], want) else -1 - lo

    with ThreadPoolExecutor(THREADS) as ex:
        bad = [r for r in ex.map(lambda b: check(*b), _chunks(P, 100)) if r < 0]
    assert not bad, f"pods from {[-1 - b for b in bad][:5]} differ from the oracle"
    frac = float((got >> 31).mean())
    assert 0.3 < frac < 0.99, frac


class _C5:
    """The C5 workload as bench.py builds it (same generators and seeds)."""

    def __init__(self, P=65_536, N=1_000_000, M=64, R=15, k=16):
        self.P, self.N, self.M, self.k = P, N, M, k
        self.tsnap = wl.make_tas_snapshot(N, M, seed=0xC5)
        self.tbatch = wl.make_tas_batch(self.tsnap, P, R, seed=0xC5)
        self.gsnap = wl.make_gas_snapshot(N, seed=0xC5)
        self.gbatch = wl.make_gas_batch(P, seed=0xC5)

    def run_ranges(self, world, lazy=False):
        """(nodes [P][k], lens [P], fit bitmaps of the whole cluster [P][W64] or None) over
        `world` node ranges, each in its own context, merged on the device.  lazy: the
        combined top-k along each pod's order (pas_tas_gas_topk_device, bench.py's C5 step)
        instead of fit bitmaps -> pas_tas_topk_device."""
        P, N, k = self.P, self.N, self.k
        t, g = self.tsnap, self.gsnap
        rules_t, off_t = _dev(self.tbatch.rules.view(np.uint8)), _dev(self.tbatch.rule_off)
        prio_t = _dev(self.tbatch.prio.view(np.uint8))
        req_t, mask_t = _dev(self.gbatch.req), _dev(self.gbatch.req_mask.view(np.int32))
        nc_t = _dev(self.gbatch.n_containers)
        C = self.gbatch.req.shape[1]
        keys, nodes, fits = [], [], []
        for r in range(world):
            n0, n1 = node_range(N, world, r)
            nl = n1 - n0
            with pas_amd.Context(0) as c:
                s = torch.cuda.current_stream()
                c.tas_snapshot_set_device(1, nl, self.M, _dev(t.v_milli[:, n0:n1]),
                                          _dev(t.present[:, n0 // 64:(n1 + 63) // 64]
                                               .view(np.int64)), s)
                c.gas_snapshot_set_device(2, nl, g.used.shape[1], g.used.shape[2],
                                          _dev(g.n_cards[n0:n1]), _dev(g.cap[n0:n1]),
                                          _dev(g.used[n0:n1]), s)
                key = torch.empty((P, k), dtype=torch.int64, device="cuda")
                node = torch.empty((P, k), dtype=torch.int32, device="cuda")
                ln = torch.empty(P, dtype=torch.int32, device="cuda")
                if lazy:
                    c.tas_gas_topk_device(1, 2, P, len(self.tbatch.rules), rules_t, off_t, prio_t,
                                          None, C, wl.I915, req_t, mask_t, nc_t, k, n0, key, node,
                                          ln, s)
                    torch.cuda.synchronize()
                    keys.append(key)
                    nodes.append(node)
                    continue
                fit_t = torch.empty((P, pas_amd.w64(nl)), dtype=torch.int64, device="cuda")
                c.gas_fit_bitmap_device(2, P, C, wl.I915, req_t, mask_t, nc_t, fit_t, s)
                c.tas_topk_device(1, P, len(self.tbatch.rules), rules_t, off_t, prio_t, fit_t, k,
                                  n0, key, node, ln, s)
                if world == 1:  # pass bitmaps of the whole cluster for the property checks
                    pass_t = torch.empty_like(fit_t)
                    c.tas_eval_device(1, P, len(self.tbatch.rules), rules_t, off_t, prio_t,
                                      fit_t, pas_amd.PAS_TAS_FILTER, pass_t, None, None, s)
                    fits.append((fit_t, pass_t))
                torch.cuda.synchronize()
                keys.append(key)
                nodes.append(node)
        out_node = torch.empty((P, k), dtype=torch.int32, device="cuda")
        out_len = torch.empty(P, dtype=torch.int32, device="cuda")
        with pas_amd.Context(0) as c:
            c.topk_merge_device(P, k, world, torch.stack(keys), torch.stack(nodes), out_node,
                                out_len, torch.cuda.current_stream())
            torch.cuda.synchronize()
        return out_node, out_len, (fits[0] if fits else None)


    def run_grid(self, node_shards, pod_groups):
        """The GridTopK split simulated on one GPU: pod group gi's pods (pod_slice) over each of
        the node_shards ranges (pod_batch_slice of the batch, rules rebased), the lazy combined
        top-k per (group, shard) in a context of its own, merged within the group; the groups'
        lists concatenated ([P][k], [P])."""
        from pas_amd.shard import pod_batch_slice, pod_slice
        P, N, k = self.P, self.N, self.k
        t, g = self.tsnap, self.gsnap
        out_nodes, out_lens = [], []
        for gi in range(pod_groups):
            p0, p1 = pod_slice(P, pod_groups, gi)
            rules, off, prio, req, mask, nc = pod_batch_slice(
                p0, p1, self.tbatch.rules, self.tbatch.rule_off, self.tbatch.prio,
                self.gbatch.req, self.gbatch.req_mask, self.gbatch.n_containers)
            n = p1 - p0
            rules_t, off_t, prio_t = _dev(rules.view(np.uint8)), _dev(off), _dev(prio.view(np.uint8))
            req_t, mask_t, nc_t = _dev(req), _dev(mask.view(np.int32)), _dev(nc)
            keys, nodes = [], []
            for si in range(node_shards):
                n0, n1 = node_range(N, node_shards, si)
                with pas_amd.Context(0) as c:
                    st = torch.cuda.current_stream()
                    c.tas_snapshot_set_device(1, n1 - n0, self.M, _dev(t.v_milli[:, n0:n1]),
                                              _dev(t.present[:, n0 // 64:(n1 + 63) // 64]
                                                   .view(np.int64)), st)
                    c.gas_snapshot_set_device(2, n1 - n0, g.used.shape[1], g.used.shape[2],
                                              _dev(g.n_cards[n0:n1]), _dev(g.cap[n0:n1]),
                                              _dev(g.used[n0:n1]), st)
                    key = torch.empty((n, k), dtype=torch.int64, device="cuda")
                    node = torch.empty((n, k), dtype=torch.int32, device="cuda")
                    ln = torch.empty(n, dtype=torch.int32, device="cuda")
                    c.tas_gas_topk_device(1, 2, n, len(rules), rules_t, off_t, prio_t, None,
                                          req.shape[1], wl.I915, req_t, mask_t, nc_t, k, n0, key,
                                          node, ln, st)
                    torch.cuda.synchronize()
                    keys.append(key)
                    nodes.append(node)
            out_node = torch.empty((n, k), dtype=torch.int32, device="cuda")
            out_len = torch.empty(n, dtype=torch.int32, device="cuda")
            with pas_amd.Context(0) as c:
                c.topk_merge_device(n, k, node_shards, torch.stack(keys), torch.stack(nodes),
                                    out_node, out_len, torch.cuda.current_stream())
                torch.cuda.synchronize()
            out_nodes.append(out_node)
            out_lens.append(out_len)
        return torch.cat(out_nodes), torch.cat(out_lens)


@pytest.fixture(scope="module")
def c5():
    return _C5()


def c5_oracle_sample(c5, per_cell=24, total=1024):
    """Pods of the C5 batch to check against the oracle: up to `per_cell` of every cell of
    (prioritize op) x (selection class: 0 / 1 / 2 / 3 / 4-8 card selections, the GAS kernels'
    lists) x (same-metric rule: none / on the prioritize metric / on it with the prioritize
    op, i.e. excluding the head of the pod's order: the lazy kernel's range jump,
    tas_gas_topk.hip), then evenly spaced pods up to `total`.  Returns (pods, cells)."""
    tb, gb = c5.tbatch, c5.gbatch
    P = c5.P
    live = np.arange(gb.req.shape[1])[None, :] < gb.n_containers[:, None]
    sel = np.where(live & ((gb.req_mask & 1) != 0), gb.req[:, :, wl.I915], 0).sum(axis=1)
    cls = np.minimum(sel, 4)
    pm, po = tb.prio["metric"], tb.prio["op"]
    rm = tb.rules["metric"].reshape(P, -1)
    ro = tb.rules["op"].reshape(P, -1)
    same = rm == pm[:, None]
    head = same & (ro == po[:, None]) & (po[:, None] != 2)
    jump = np.where(head.any(axis=1), 2, np.where(same.any(axis=1), 1, 0))
    rng = np.random.default_rng(0x5A)
    picked, cells = [], {}
    for op in range(3):
        for c in range(5):
            for j in range(3):
                ids = np.flatnonzero((po == op) & (cls == c) & (jump == j))
                cells[(op, c, j)] = len(ids)
                if len(ids):
                    picked.append(rng.choice(ids, size=min(per_cell, len(ids)), replace=False))
    picked = np.unique(np.concatenate(picked))
    rest = np.setdiff1d(np.linspace(0, P - 1, total, dtype=np.int64), picked)
    pods = np.unique(np.concatenate([picked, rest[: max(0, total - len(picked))]]))
    return pods, cells


def test_c5_sample_vs_oracle_composition(c5, oracle):
    """>= 1,024 pods of the C5 batch, chosen to cover every (prioritize op x selection class x
    same-metric rule) cell (c5_oracle_sample): GPU merged lists (8 ranges, the lazy combined
    top-k bench.py times) == oracle composition.  ~0.33 s of oracle work per pod (GAS fit and
    TAS eval over 1M nodes), ~25 s on 16 threads."""
    nodes8, lens8, _ = c5.run_ranges(8, lazy=True)
    nodes8, lens8 = nodes8.cpu().numpy(), lens8.cpu().numpy()
    sample, cells = c5_oracle_sample(c5)
    assert len(sample) >= 1024
    # every op x class x jump cell the batch has is in the sample
    assert sum(1 for v in cells.values() if v) >= 40, cells
    t, g, tb, gb = c5.tsnap, c5.gsnap, c5.tbatch, c5.gbatch

    def compose(i):
        p = int(sample[i])
        words = oracle.gas_fit(g.n_cards, g.cap, g.used, gb.req[p:p + 1], gb.req_mask[p:p + 1],
                               gb.n_containers[p:p + 1], wl.I915)
        cand = wl.pack_bits((words >> 31).astype(bool))
        rules = tb.rules[tb.rule_off[p]:tb.rule_off[p + 1]]
        off = np.array([0, len(rules)], np.int32)
        _, order, lens = oracle.tas_eval(t.v_milli, t.present, rules, off, tb.prio[p:p + 1],
                                         cand, 3)
        m = min(c5.k, int(lens[0]))
        return p, order[0, :m].copy(), int((words >> 31).sum())

    with ThreadPoolExecutor(THREADS) as ex:
        results = list(ex.map(compose, range(len(sample))))
    nonempty = 0
    for p, want, n_fit in results:
        assert lens8[p] == len(want), p
        np.testing.assert_array_equal(nodes8[p, :len(want)], want)
        assert (nodes8[p, len(want):] == -1).all()
        nonempty += len(want) > 0
    assert nonempty > len(sample) // 2  # the sample exercises real lists


def test_c5_full_batch_properties(c5):
    """All 65,536 pods: 8-range merge == whole cluster, and the size-independent properties."""
    P, N, k = c5.P, c5.N, c5.k
    nodes1, lens1, (fit_t, pass_t) = c5.run_ranges(1)
    nodes8, lens8, _ = c5.run_ranges(8)
    assert torch.equal(lens1, lens8)
    assert torch.equal(nodes1, nodes8)
    # the lazy combined top-k (bench.py's C5 step), whole cluster and 8 ranges: every pod
    for world in (1, 8):
        lz_nodes, lz_lens, _ = c5.run_ranges(world, lazy=True)
        assert torch.equal(lz_lens, lens1), world
        assert torch.equal(lz_nodes, nodes1), world
    # the 2-D split (GridTopK): 2 node shards x 4 pod groups, and 1 x 8 (pure pod sharding)
    for shards, groups in ((2, 4), (1, 8)):
        g_nodes, g_lens = c5.run_grid(shards, groups)
        assert torch.equal(g_lens, lens1), (shards, groups)
        assert torch.equal(g_nodes, nodes1), (shards, groups)
    # every pass bit is also a fit bit (pass = cand AND NOT violated)
    assert not bool(((pass_t & ~fit_t) != 0).any())
    vals = _dev(c5.tsnap.v_milli)
    pres = _dev(c5.tsnap.present.view(np.int64))
    m0 = _dev(c5.tbatch.prio["metric"].astype(np.int64))
    ops = _dev(c5.tbatch.prio["op"].astype(np.int64))
    for lo, hi in _chunks(P, 8192):
        cnt = popcount64(pass_t[lo:hi] & pres[m0[lo:hi]]).sum(dim=1)
        assert torch.equal(lens1[lo:hi].long(), torch.clamp(cnt, max=k)), lo
    ln = lens1.long()
    j = torch.arange(k, device="cuda")[None, :]
    live = j < ln[:, None]
    assert bool((nodes1[~live] == -1).all())
    idx = torch.where(live, nodes1.long(), torch.zeros_like(nodes1, dtype=torch.long))
    word, bit = idx >> 6, idx & 63
    rows = torch.arange(P, device="cuda")[:, None]
    assert bool((((pass_t[rows, word] >> bit) & 1)[live] == 1).all())
    assert bool((((pres[m0[:, None], word] >> bit) & 1)[live] == 1).all())
    v = vals[m0[:, None], idx]
    key = torch.where(ops[:, None] == 1, ~v, torch.where(ops[:, None] == 0, v, torch.zeros_like(v)))
    both = live[:, 1:] & live[:, :-1]
    asc = (key[:, 1:] > key[:, :-1]) | ((key[:, 1:] == key[:, :-1]) & (idx[:, 1:] > idx[:, :-1]))
    assert bool(asc[both].all()), "lists not ascending in (key, node): duplicates or misorder"
    assert float((ln > 0).float().mean()) > 0.5
