"""Node-sharded evaluation (pas_amd/shard.py).

A rank holds a contiguous node range of the cluster; per pod it keeps the first k entries
of its shard's HostPriorityList as (key, global node) records, the records are
all-gathered and merged.  Parity: the merged lists equal the first k entries of the
oracle's list over the whole cluster (telemetryscheduler.go:128-149 / operator.go:30-42),
and gathered shard violation bitmaps equal the cluster sweep (deschedule/strategy.go:31-50).
CPU tests run the collectives over gloo with the oracle as the per-shard evaluator; GPU
tests run the HIP top-k and merge kernels.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from helpers import pack_bits, unpack_bits

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GT, LT = 1, 0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def shard_snapshot(v, pres, n0, n1):
    n = v.shape[1]
    pb = unpack_bits(pres, n)[:, n0:n1]
    return np.ascontiguousarray(v[:, n0:n1]), pack_bits(pb)


def shard_cand(cand, n, n0, n1):
    if cand is None:
        return None
    return pack_bits(unpack_bits(cand, n)[:, n0:n1])


def order_keys(v, prio, nodes, p):
    """Merge keys of global node ids under pod p's prioritize operator (pas.h)."""
    op = int(prio["op"][p])
    if op == GT:
        return np.invert(v[prio["metric"][p], nodes])
    if op == LT:
        return v[prio["metric"][p], nodes]
    return np.zeros(len(nodes), np.int64)


def records(oracle, v, pres, rules, off, prio, cand, n0, n1, k):
    """Per-shard records (keys [P][k], nodes [P][k]) from the oracle's shard lists."""
    n = v.shape[1]
    sv, sp = shard_snapshot(v, pres, n0, n1)
    _, order, lens = oracle.tas_eval(sv, sp, rules, off, prio, shard_cand(cand, n, n0, n1), 3)
    P = len(prio)
    keys = np.full((P, k), np.iinfo(np.int64).max, np.int64)
    nodes = np.full((P, k), np.iinfo(np.int32).max, np.int32)
    for p in range(P):
        m = min(k, int(lens[p]))
        g = order[p, :m].astype(np.int64) + n0
        nodes[p, :m] = g
        keys[p, :m] = order_keys(v, prio, g, p)
    return keys, nodes


def merge_records(keys_all, nodes_all, k):
    """Reference merge: the k smallest (key, node) records per pod."""
    S, P, _ = keys_all.shape
    out = []
    for p in range(P):
        recs = [(int(keys_all[s, p, j]), int(nodes_all[s, p, j])) for s in range(S)
                for j in range(k) if nodes_all[s, p, j] != np.iinfo(np.int32).max]
        out.append([nd for _, nd in sorted(recs)[:k]])
    return out


def make_case(seed, n, m, p, r, cand_frac=None):
    sys.path.insert(0, os.path.join(ROOT, "platform-aware-scheduling_amd"))
    from pas_amd import workload as wl
    snap = wl.make_tas_snapshot(n, m, seed=seed)
    batch = wl.make_tas_batch(snap, p, r, seed=seed, cand_frac=cand_frac)
    rng = np.random.default_rng(seed)
    # ties and the unsorted branch: some integer-valued entries, some Equals pods
    batch.prio["op"][rng.random(p) < 0.15] = 2
    return snap, batch


# ------------------------------------------------------------------------------ CPU


def test_node_range_partitions():
    from pas_amd.shard import node_range
    for n in (0, 1, 63, 64, 65, 1000, 100_003):
        for world in (1, 2, 3, 8):
            rs = [node_range(n, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            for (a0, a1), (b0, b1) in zip(rs, rs[1:]):
                assert a1 == b0 and (a0 % 64 == 0 or a0 == n)
            assert all(a0 <= a1 for a0, a1 in rs)


def test_merge_of_shard_lists_is_global_list(oracle):
    """Union-merge of shard top-k equals the global top-k (single process, oracle)."""
    from pas_amd.shard import node_range
    snap, batch = make_case(0xC5, 3000, 6, 40, 4, cand_frac=0.85)
    v, pres = snap.v_milli, snap.present
    _, order, lens = oracle.tas_eval(v, pres, batch.rules, batch.rule_off, batch.prio,
                                     batch.cand, 3)
    for world in (2, 3, 5):
        for k in (1, 7, 16):
            recs = [records(oracle, v, pres, batch.rules, batch.rule_off, batch.prio, batch.cand,
                            *node_range(v.shape[1], world, r), k) for r in range(world)]
            merged = merge_records(np.stack([a for a, _ in recs]),
                                   np.stack([b for _, b in recs]), k)
            for p in range(len(batch.prio)):
                want = list(order[p, :min(k, int(lens[p]))])
                assert merged[p] == want, (world, k, p)


def _gloo_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    for p in (os.path.join(ROOT, "platform-aware-scheduling_amd"), os.path.join(ROOT, "oracle"),
              os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import oracle
    from pas_amd import distrib
    from pas_amd.shard import _all_gather, gather_violations, node_range
    from pas_amd import workload as wl

    distrib.setup("gloo")
    snap, batch = make_case(0xC4, 2500, 5, 12, 3, cand_frac=0.9)
    v, pres = snap.v_milli, snap.present
    n = v.shape[1]
    n0, n1 = node_range(n, world, rank)
    k = 8
    keys, nodes = records(oracle, v, pres, batch.rules, batch.rule_off, batch.prio, batch.cand,
                          n0, n1, k)
    P = len(batch.prio)
    keys_all = _all_gather(torch.from_numpy(keys), world).numpy().reshape(world, P, k)
    nodes_all = _all_gather(torch.from_numpy(nodes), world).numpy().reshape(world, P, k)
    merged = merge_records(keys_all, nodes_all, k)
    # deschedule: shard sweeps gathered into the cluster bitmap
    drules, doff = wl.make_deschedule_rules(snap, 4, 3, seed=0xC4)
    sv, sp = shard_snapshot(v, pres, n0, n1)
    viol = oracle.tas_violations(sv, sp, drules, doff)
    full = gather_violations(torch.from_numpy(viol.view(np.int64)), world, n).numpy()
    padded = np.full((P, k), -1, np.int64)
    for p, lst in enumerate(merged):
        padded[p, :len(lst)] = lst
    np.save(os.path.join(out_dir, f"merged{rank}.npy"), padded)
    np.save(os.path.join(out_dir, f"viol{rank}.npy"), full[:, :(n + 63) // 64])
    distrib.teardown(world)


def test_sharded_records_over_gloo(tmp_path, oracle):
    world = 2
    mp.spawn(_gloo_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    snap, batch = make_case(0xC4, 2500, 5, 12, 3, cand_frac=0.9)
    v, pres = snap.v_milli, snap.present
    _, order, lens = oracle.tas_eval(v, pres, batch.rules, batch.rule_off, batch.prio,
                                     batch.cand, 3)
    sys.path.insert(0, os.path.join(ROOT, "platform-aware-scheduling_amd"))
    from pas_amd import workload as wl
    drules, doff = wl.make_deschedule_rules(snap, 4, 3, seed=0xC4)
    want_viol = oracle.tas_violations(v, pres, drules, doff)
    for r in range(world):
        merged = np.load(tmp_path / f"merged{r}.npy")
        for p in range(len(batch.prio)):
            m = min(8, int(lens[p]))
            np.testing.assert_array_equal(merged[p, :m], order[p, :m])
            assert (merged[p, m:] == -1).all()
        viol = np.load(tmp_path / f"viol{r}.npy")
        np.testing.assert_array_equal(viol.view(np.uint64), want_viol)


# ------------------------------------------------------------------------------ GPU


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _rule_tensors(batch, cand):
    rules_t = _dev(batch.rules.view(np.uint8))
    off_t = _dev(batch.rule_off)
    prio_t = _dev(batch.prio.view(np.uint8))
    cand_t = None if cand is None else _dev(cand.view(np.int64))
    return rules_t, off_t, prio_t, cand_t


def _shard_records_gpu(v, pres, batch, cand, n0, n1, k, gen):
    import pas_amd
    n = v.shape[1]
    sv, sp = shard_snapshot(v, pres, n0, n1)
    with pas_amd.Context(0) as c:
        c.tas_snapshot_set(gen, sv, sp)
        rules_t, off_t, prio_t, cand_t = _rule_tensors(batch, shard_cand(cand, n, n0, n1))
        P = len(batch.prio)
        key = torch.empty((P, k), dtype=torch.int64, device="cuda")
        node = torch.empty((P, k), dtype=torch.int32, device="cuda")
        ln = torch.empty(P, dtype=torch.int32, device="cuda")
        c.tas_topk_device(gen, P, len(batch.rules), rules_t, off_t, prio_t, cand_t, k, n0, key,
                          node, ln)
        c.synchronize()
        return key, node, ln


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 5, 16, 300])
def test_topk_records_match_oracle(oracle, k):
    from pas_amd.shard import node_range
    snap, batch = make_case(0x51, 4100, 6, 48, 5, cand_frac=0.9)
    v, pres = snap.v_milli, snap.present
    for world, r in ((1, 0), (3, 1), (3, 2)):
        n0, n1 = node_range(v.shape[1], world, r)
        key, node, ln = _shard_records_gpu(v, pres, batch, batch.cand, n0, n1, k, 7)
        want_k, want_n = records(oracle, v, pres, batch.rules, batch.rule_off, batch.prio,
                                 batch.cand, n0, n1, k)
        np.testing.assert_array_equal(node.cpu().numpy(), want_n)
        np.testing.assert_array_equal(key.cpu().numpy(), want_k)
        np.testing.assert_array_equal(ln.cpu().numpy(),
                                      (want_n != np.iinfo(np.int32).max).sum(1))


@pytest.mark.gpu
@pytest.mark.parametrize("world,k", [(2, 16), (3, 7), (8, 16), (4, 1)])
def test_sharded_merge_equals_global_list(ctx, oracle, world, k):
    """Device records of every shard, merged on device, equal the oracle's global lists."""
    from pas_amd.shard import node_range
    snap, batch = make_case(0x52 + world, 5000, 8, 64, 6, cand_frac=0.8)
    v, pres = snap.v_milli, snap.present
    recs = [_shard_records_gpu(v, pres, batch, batch.cand, *node_range(v.shape[1], world, r), k,
                               9) for r in range(world)]
    keys_all = torch.stack([a for a, _, _ in recs])
    nodes_all = torch.stack([b for _, b, _ in recs])
    P = len(batch.prio)
    out_node = torch.empty((P, k), dtype=torch.int32, device="cuda")
    out_len = torch.empty(P, dtype=torch.int32, device="cuda")
    ctx.topk_merge_device(P, k, world, keys_all, nodes_all, out_node, out_len)
    ctx.synchronize()
    _, order, lens = oracle.tas_eval(v, pres, batch.rules, batch.rule_off, batch.prio,
                                     batch.cand, 3)
    got_n, got_l = out_node.cpu().numpy(), out_len.cpu().numpy()
    for p in range(P):
        m = min(k, int(lens[p]))
        assert got_l[p] == m
        np.testing.assert_array_equal(got_n[p, :m], order[p, :m])
        assert (got_n[p, m:] == -1).all()


@pytest.mark.gpu
def test_gas_fit_bitmap_matches_words(ctx):
    from pas_amd import workload as wl
    gs = wl.make_gas_snapshot(3000, seed=0xC3)
    gb = wl.make_gas_batch(70, seed=0xC3)
    ctx.gas_snapshot_set(31, gs.n_cards, gs.cap, gs.used)
    words = ctx.gas_fit(31, gb.req, gb.req_mask, gb.n_containers, wl.I915)
    P, N = words.shape
    fit_t = torch.full((P, (N + 63) // 64), -1, dtype=torch.int64, device="cuda")
    ctx.gas_fit_bitmap_device(31, P, gb.req.shape[1], wl.I915, _dev(gb.req),
                              _dev(gb.req_mask.view(np.int32)), _dev(gb.n_containers), fit_t)
    ctx.synchronize()
    got = unpack_bits(fit_t.cpu().numpy().view(np.uint64), N)
    np.testing.assert_array_equal(got, (words >> 31).astype(bool))


def _gpu_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK="0")
    for p in (os.path.join(ROOT, "platform-aware-scheduling_amd"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import pas_amd
    from pas_amd import distrib
    from pas_amd.shard import ShardedTopK, node_range

    distrib.setup("gloo")  # ranks share the box's one GPU: collectives through host memory
    torch.cuda.set_device(0)
    snap, batch = make_case(0x53, 6000, 6, 50, 5, cand_frac=0.85)
    v, pres = snap.v_milli, snap.present
    n0, n1 = node_range(v.shape[1], world, rank)
    sv, sp = shard_snapshot(v, pres, n0, n1)
    with pas_amd.Context(0) as c:
        c.tas_snapshot_set(3, sv, sp)
        rules_t, off_t, prio_t, cand_t = _rule_tensors(batch, shard_cand(batch.cand, v.shape[1],
                                                                         n0, n1))
        st = ShardedTopK(c, 12, world, rank, n0)
        # rank 0: the kernels on a stream of their own (ordered against the collectives with
        # wait_stream); rank 1: torch's current stream (stream=None)
        s = torch.cuda.Stream() if rank == 0 else None
        out_node, out_len = st.run(3, len(batch.prio), len(batch.rules), rules_t, off_t, prio_t,
                                   cand_t, stream=s)
        torch.cuda.synchronize()
        np.save(os.path.join(out_dir, f"nodes{rank}.npy"), out_node.cpu().numpy())
        np.save(os.path.join(out_dir, f"lens{rank}.npy"), out_len.cpu().numpy())
    distrib.teardown(world)


@pytest.mark.gpu
def test_sharded_topk_two_ranks_one_gpu(tmp_path, oracle):
    """ShardedTopK end to end in two processes (gloo between them, one GPU)."""
    world = 2
    mp.spawn(_gpu_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    snap, batch = make_case(0x53, 6000, 6, 50, 5, cand_frac=0.85)
    _, order, lens = oracle.tas_eval(snap.v_milli, snap.present, batch.rules, batch.rule_off,
                                     batch.prio, batch.cand, 3)
    for r in range(world):
        nodes = np.load(tmp_path / f"nodes{r}.npy")
        ln = np.load(tmp_path / f"lens{r}.npy")
        for p in range(len(batch.prio)):
            m = min(12, int(lens[p]))
            assert ln[p] == m
            np.testing.assert_array_equal(nodes[p, :m], order[p, :m])


def _lazy_vs_composed(ctx, v, pres, batch, gsnap, gbatch, cand, k, node_base, i915):
    """pas_tas_gas_topk_device vs pas_gas_fit_bitmap_device -> pas_tas_topk_device on one
    context (both device paths), records and lengths."""
    P = len(batch.prio)
    n = v.shape[1]
    gen_t, gen_g = 4101, 4102
    ctx.tas_snapshot_set(gen_t, v, pres)
    ctx.gas_snapshot_set(gen_g, gsnap.n_cards, gsnap.cap, gsnap.used)
    rules_t, off_t, prio_t, cand_t = _rule_tensors(batch, cand)
    req_t, mask_t = _dev(gbatch.req), _dev(gbatch.req_mask.view(np.int32))
    nc_t = _dev(gbatch.n_containers)
    C = gbatch.req.shape[1]
    fit_t = torch.empty((P, (n + 63) // 64), dtype=torch.int64, device="cuda")
    ctx.gas_fit_bitmap_device(gen_g, P, C, i915, req_t, mask_t, nc_t, fit_t)
    ctx.synchronize()  # (the context's stream) before torch's stream reads fit_t
    if cand_t is not None:
        fit_t &= cand_t
        torch.cuda.synchronize()
    out = []
    for lazy in (False, True):
        key = torch.empty((P, k), dtype=torch.int64, device="cuda")
        node = torch.empty((P, k), dtype=torch.int32, device="cuda")
        ln = torch.empty(P, dtype=torch.int32, device="cuda")
        if lazy:
            ctx.tas_gas_topk_device(gen_t, gen_g, P, len(batch.rules), rules_t, off_t, prio_t,
                                    cand_t, C, i915, req_t, mask_t, nc_t, k, node_base, key,
                                    node, ln)
        else:
            ctx.tas_topk_device(gen_t, P, len(batch.rules), rules_t, off_t, prio_t, fit_t, k,
                                node_base, key, node, ln)
        ctx.synchronize()
        out.append((key.cpu().numpy(), node.cpu().numpy(), ln.cpu().numpy()))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("k,n,cards,cand_frac", [(16, 5000, 8, None), (1, 3000, 8, 0.7),
                                                 (70, 4200, 8, 0.9), (300, 2000, 3, None),
                                                 (16, 3000, 12, 0.8)])
def test_tas_gas_topk_equals_composition(ctx, k, n, cards, cand_frac):
    """The lazy combined top-k equals GAS fit bitmaps -> TAS top-k (the composed C5 path):
    records (key, global node) and lengths, with candidate masks, ties and Equals pods,
    unknown-kind containers, pods with no fitting node and nodes of 9-16 cards."""
    from pas_amd import workload as wl
    from test_gas_gpu import random_gas
    snap, batch = make_case(0x60 + k + cards, n, 6, 96, 7, cand_frac=cand_frac)
    rng = np.random.default_rng(k * 7 + n)
    if cards == 8:
        gsnap = wl.make_gas_snapshot(n, seed=0x61 + k)
        gbatch = wl.make_gas_batch(96, seed=0x61 + k)
        i915 = wl.I915
    else:
        nc, cap, used, req, mask, ncont = random_gas(rng, n, cards, 3, 96, 4, i915=0)
        cap *= 4  # roomy enough that most pods fit somewhere
        req[0, 0, 0], mask[0, 0], ncont[0] = 70, 1, max(ncont[0], 1)  # past 64 selections
        gsnap, gbatch = wl.GasSnapshotData(nc, cap, used), wl.GasBatch(req, mask, ncont)
        i915 = 0
    flag = rng.random(gbatch.req_mask.shape) < 0.05
    gbatch.req_mask = gbatch.req_mask | np.where(flag, 0x80000000, 0).astype(np.uint32)
    batch.prio["metric"][::17] = 99  # no scheduling rule: empty list
    composed, lazy = _lazy_vs_composed(ctx, snap.v_milli, snap.present, batch, gsnap, gbatch,
                                       batch.cand, k, 1234, i915)
    for a, b in zip(composed, lazy):
        np.testing.assert_array_equal(b, a)
    assert (composed[2] > 0).mean() > 0.4


# ------------------------------------------------------------------- full lists over shards


def test_pod_slice_partitions():
    from pas_amd.shard import pod_slice
    for n in (0, 1, 5, 64, 1001):
        for world in (1, 2, 3, 8):
            rs = [pod_slice(n, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            for (a0, a1), (b0, b1) in zip(rs, rs[1:]):
                assert a1 == b0 and a0 <= a1


def merge_full(keys_in, nodes_in):
    """Reference merge of [S][P][w] shard runs: each pod's real records in (key, node) order."""
    S, P, w = keys_in.shape
    out = []
    for p in range(P):
        recs = [(int(keys_in[s, p, j]), int(nodes_in[s, p, j])) for s in range(S)
                for j in range(w) if nodes_in[s, p, j] != np.iinfo(np.int32).max]
        out.append([nd for _, nd in sorted(recs)])
    return out


def _gloo_full_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    for p in (os.path.join(ROOT, "platform-aware-scheduling_amd"), os.path.join(ROOT, "oracle"),
              os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import oracle
    from pas_amd import distrib
    from pas_amd.shard import _all_to_all, node_range, pod_slice

    distrib.setup("gloo")
    snap, batch = make_case(0xF1, 1300, 5, 11, 3, cand_frac=0.9)
    v, pres = snap.v_milli, snap.present
    n = v.shape[1]
    n0, n1 = node_range(n, world, rank)
    a0, a1 = node_range(n, world, 0)
    w = a1 - a0  # the widest shard
    P = len(batch.prio)
    per = (P + world - 1) // world
    keys = np.full((world * per, w), np.iinfo(np.int64).max, np.int64)
    nodes = np.full((world * per, w), np.iinfo(np.int32).max, np.int32)
    k, nd = records(oracle, v, pres, batch.rules, batch.rule_off, batch.prio, batch.cand, n0, n1,
                    w)
    keys[:P], nodes[:P] = k, nd
    keys_in = _all_to_all(torch.from_numpy(keys).view(world, per, w), world).numpy()
    nodes_in = _all_to_all(torch.from_numpy(nodes).view(world, per, w), world).numpy()
    p0, p1 = pod_slice(P, world, rank)
    merged = merge_full(keys_in, nodes_in)[:p1 - p0]
    padded = np.full((max(p1 - p0, 0), n), -1, np.int64)
    for i, lst in enumerate(merged):
        padded[i, :len(lst)] = lst
    np.save(os.path.join(out_dir, f"full{rank}.npy"), padded)
    distrib.teardown(world)


@pytest.mark.parametrize("world", [2, 3])
def test_full_lists_over_gloo(tmp_path, oracle, world):
    """The all-to-all of whole-shard records to the pods' owners, merged, gives the oracle's
    cluster HostPriorityList for every pod (CPU, gloo; the oracle as the shard evaluator)."""
    from pas_amd.shard import pod_slice
    mp.spawn(_gloo_full_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
             join=True)
    snap, batch = make_case(0xF1, 1300, 5, 11, 3, cand_frac=0.9)
    _, order, lens = oracle.tas_eval(snap.v_milli, snap.present, batch.rules, batch.rule_off,
                                     batch.prio, batch.cand, 3)
    P = len(batch.prio)
    for r in range(world):
        p0, p1 = pod_slice(P, world, r)
        got = np.load(tmp_path / f"full{r}.npy")
        for i, p in enumerate(range(p0, p1)):
            m = int(lens[p])
            np.testing.assert_array_equal(got[i, :m], order[p, :m])
            assert (got[i, m:] == -1).all()


@pytest.mark.gpu
@pytest.mark.parametrize("S,w", [(1, 5), (2, 1), (2, 1500), (3, 700), (5, 300), (8, 1024),
                                 (8, 1025), (4, 3000)])
def test_list_merge_kernel(ctx, S, w):
    """pas_list_merge_device vs a sort of the union: random sorted runs with tied keys, keys
    at INT64_MAX, empty and full runs, tile boundaries (1024 outputs per workgroup)."""
    rng = np.random.default_rng(S * 1000 + w)
    P = 6
    keys = np.full((S, P, w), np.iinfo(np.int64).max, np.int64)
    nodes = np.full((S, P, w), np.iinfo(np.int32).max, np.int32)
    perm = rng.permutation(S * w * 4).astype(np.int32)
    for p in range(P):
        ids = perm[p * 0: S * w * 4].reshape(-1)[: S * w].reshape(S, w)
        for s in range(S):
            ln = [0, w, int(rng.integers(0, w + 1))][(p + s) % 3]
            k = rng.integers(-5, 5, size=ln).astype(np.int64) * (2**61)  # many ties
            k[rng.random(ln) < 0.05] = np.iinfo(np.int64).max  # real records at the max key
            order = np.lexsort((ids[s, :ln], k))
            keys[s, p, :ln] = k[order]
            nodes[s, p, :ln] = ids[s, :ln][order]
    want = merge_full(keys, nodes)
    ld = S * w + 3
    out = torch.full((P, ld), -7, dtype=torch.int32, device="cuda")
    ln = torch.empty(P, dtype=torch.int32, device="cuda")
    ctx.list_merge_device(P, S, w, _dev(keys), _dev(nodes), out, ln, out_ld=ld)
    ctx.synchronize()
    got, got_l = out.cpu().numpy(), ln.cpu().numpy()
    for p in range(P):
        m = len(want[p])
        assert got_l[p] == m
        np.testing.assert_array_equal(got[p, :m], want[p])
        assert (got[p, m:S * w] == -1).all() and (got[p, S * w:] == -7).all()


@pytest.mark.gpu
@pytest.mark.parametrize("w", [5000, 70000])
def test_list_merge_single_shard_fresh_context(w):
    """One shard (no merge round) on a context whose merge scratch was never grown: the run is
    copied with sentinels as -1, nothing written past the list's row (the single-run
    case once sized its cut buffer for width/1024 tiles but launched 2·width/1024)."""
    import pas_amd
    rng = np.random.default_rng(w)
    P = 5
    keys = np.full((1, P, w), np.iinfo(np.int64).max, np.int64)
    nodes = np.full((1, P, w), np.iinfo(np.int32).max, np.int32)
    for p in range(P):
        ln = [0, w, int(rng.integers(0, w + 1)), 1, w - 1][p]
        k = np.sort(rng.integers(-3, 3, size=ln).astype(np.int64))
        keys[0, p, :ln] = k
        nodes[0, p, :ln] = rng.permutation(w)[:ln].astype(np.int32)
        o = np.lexsort((nodes[0, p, :ln], k))
        nodes[0, p, :ln] = nodes[0, p, :ln][o]
    want = merge_full(keys, nodes)
    ld = w + 9
    c = pas_amd.Context(0)
    try:
        out = torch.full((P + 1, ld), -7, dtype=torch.int32, device="cuda")
        ln = torch.empty(P, dtype=torch.int32, device="cuda")
        c.list_merge_device(P, 1, w, _dev(keys), _dev(nodes), out, ln, out_ld=ld)
        c.synchronize()
    finally:
        c.close()
    got, got_l = out.cpu().numpy(), ln.cpu().numpy()
    for p in range(P):
        m = len(want[p])
        assert got_l[p] == m
        np.testing.assert_array_equal(got[p, :m], want[p])
        assert (got[p, m:w] == -1).all() and (got[p, w:] == -7).all()
    assert (got[P] == -7).all()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_full_list_over_shards_equals_global(ctx, oracle, world):
    """Whole-shard device records of every shard, merged on device, equal the oracle's
    full HostPriorityList over the cluster for every pod."""
    from pas_amd.shard import node_range
    snap, batch = make_case(0xF2 + world, 4100, 6, 40, 5, cand_frac=0.85)
    v, pres = snap.v_milli, snap.present
    n = v.shape[1]
    a0, a1 = node_range(n, world, 0)
    w = a1 - a0
    recs = [_shard_records_gpu(v, pres, batch, batch.cand, *node_range(n, world, r), w, 11)
            for r in range(world)]
    keys_all = torch.stack([a for a, _, _ in recs])
    nodes_all = torch.stack([b for _, b, _ in recs])
    P = len(batch.prio)
    out = torch.empty((P, world * w), dtype=torch.int32, device="cuda")
    ln = torch.empty(P, dtype=torch.int32, device="cuda")
    ctx.list_merge_device(P, world, w, keys_all, nodes_all, out, ln)
    ctx.synchronize()
    _, order, lens = oracle.tas_eval(v, pres, batch.rules, batch.rule_off, batch.prio,
                                     batch.cand, 3)
    got, got_l = out.cpu().numpy(), ln.cpu().numpy()
    np.testing.assert_array_equal(got_l, lens)
    for p in range(P):
        m = int(lens[p])
        np.testing.assert_array_equal(got[p, :m], order[p, :m])
        assert (got[p, m:] == -1).all()


def _gpu_full_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK="0")
    for p in (os.path.join(ROOT, "platform-aware-scheduling_amd"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import pas_amd
    from pas_amd import distrib
    from pas_amd.shard import ShardedFullList, node_range

    distrib.setup("gloo")  # ranks share the box's one GPU: collectives through host memory
    torch.cuda.set_device(0)
    snap, batch = make_case(0xF3, 5000, 6, 21, 5, cand_frac=0.85)
    v, pres = snap.v_milli, snap.present
    n = v.shape[1]
    n0, n1 = node_range(n, world, rank)
    a0, a1 = node_range(n, world, 0)
    sv, sp = shard_snapshot(v, pres, n0, n1)
    with pas_amd.Context(0) as c:
        c.tas_snapshot_set(3, sv, sp)
        rules_t, off_t, prio_t, cand_t = _rule_tensors(batch, shard_cand(batch.cand, n, n0, n1))
        fl = ShardedFullList(c, a1 - a0, world, rank, n0)
        s = torch.cuda.Stream() if rank == 0 else None
        p0, p1, out, ln = fl.run(3, len(batch.prio), len(batch.rules), rules_t, off_t, prio_t,
                                 cand_t, stream=s)
        torch.cuda.synchronize()
        np.save(os.path.join(out_dir, f"fl{rank}.npy"), out.cpu().numpy())
        np.save(os.path.join(out_dir, f"fll{rank}.npy"), ln.cpu().numpy())
        np.save(os.path.join(out_dir, f"flp{rank}.npy"), np.array([p0, p1]))
    distrib.teardown(world)


@pytest.mark.gpu
def test_sharded_full_list_two_ranks_one_gpu(tmp_path, oracle):
    """ShardedFullList end to end in two processes (gloo between them, one GPU): each rank
    returns the cluster's full lists of its pod slice."""
    world = 2
    mp.spawn(_gpu_full_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
             join=True)
    snap, batch = make_case(0xF3, 5000, 6, 21, 5, cand_frac=0.85)
    _, order, lens = oracle.tas_eval(snap.v_milli, snap.present, batch.rules, batch.rule_off,
                                     batch.prio, batch.cand, 3)
    seen = 0
    for r in range(world):
        out, ln = np.load(tmp_path / f"fl{r}.npy"), np.load(tmp_path / f"fll{r}.npy")
        p0, p1 = np.load(tmp_path / f"flp{r}.npy")
        for i, p in enumerate(range(p0, p1)):
            m = int(lens[p])
            assert ln[i] == m
            np.testing.assert_array_equal(out[i, :m], order[p, :m])
            assert (out[i, m:] == -1).all()
            seen += 1
    assert seen == len(batch.prio)
