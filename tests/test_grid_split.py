"""The 2-D multi-GPU split of the C5 top-k (pas_amd.shard.GridTopK):
node_shards x pod groups.  CPU part: world-4 gloo runs of the split's own code (process
groups, pod slices, per-group all-gather and merge) with the device kernels replaced by the
oracle composition (GAS fit -> TAS eval, first k of each list), for 2 x 2, 1 x 4 and 4 x 1,
against the whole-cluster lists.  GPU part: test_configs_full.py runs the kernels over a
simulated 2 x 4 split of the full C5 batch."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(ROOT, "platform-aware-scheduling_amd"), os.path.join(ROOT, "oracle"),
           os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from test_shard import merge_records, order_keys  # noqa: E402

P, N, M, R, K = 24, 1500, 5, 4, 6
I32_MAX = np.iinfo(np.int32).max
I64_MAX = np.iinfo(np.int64).max


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def case():
    from pas_amd import workload as wl
    tsnap = wl.make_tas_snapshot(N, M, seed=0x6D)
    tbatch = wl.make_tas_batch(tsnap, P, R, seed=0x6D)
    gsnap = wl.make_gas_snapshot(N, seed=0x6D)
    gbatch = wl.make_gas_batch(P, seed=0x6D)
    return tsnap, tbatch, gsnap, gbatch


def composed_lists(oracle, tsnap, gsnap, rules, off, prio, req, mask, ncont, n0, n1):
    """Per pod the first K of the shard's list over nodes that fit and pass (oracle)."""
    from pas_amd import workload as wl
    words = oracle.gas_fit(gsnap.n_cards[n0:n1], gsnap.cap[n0:n1], gsnap.used[n0:n1], req,
                           mask, ncont, wl.I915)
    cand = wl.pack_bits((words >> 31).astype(bool))
    from test_shard import shard_snapshot
    sv, sp = shard_snapshot(tsnap.v_milli, tsnap.present, n0, n1)
    _, order, lens = oracle.tas_eval(sv, sp, rules, off, prio, cand, 3)
    return order, lens


class OracleCtx:
    """The two device entry points GridTopK calls, restated with the oracle on CPU tensors."""

    def __init__(self, oracle, tsnap, gsnap, n0, n1):
        self.o, self.t, self.g, self.n0, self.n1 = oracle, tsnap, gsnap, n0, n1

    def tas_gas_topk_device(self, tas_gen, gas_gen, n_pods, n_rules, rules_t, off_t, prio_t,
                            cand_t, C, i915, req_t, mask_t, ncont_t, k, node_base, key, node,
                            ln, stream=None):
        from helpers import RULE_DTYPE
        rules = rules_t.numpy().view(RULE_DTYPE)
        prio = prio_t.numpy().view(RULE_DTYPE)
        order, lens = composed_lists(self.o, self.t, self.g, rules, off_t.numpy(), prio,
                                     req_t.numpy(), mask_t.numpy().view(np.uint32),
                                     ncont_t.numpy(), self.n0, self.n1)
        key.fill_(I64_MAX)
        node.fill_(I32_MAX)
        for p in range(n_pods):
            m = min(k, int(lens[p]))
            g = order[p, :m].astype(np.int64) + node_base
            node[p, :m] = torch.from_numpy(g.astype(np.int32))
            key[p, :m] = torch.from_numpy(order_keys(self.t.v_milli, prio, g, p))
            ln[p] = m

    def topk_merge_device(self, n_pods, k, n_shards, keys_all, nodes_all, out_node, out_len,
                          stream=None):
        merged = merge_records(keys_all.view(n_shards, n_pods, k).numpy(),
                               nodes_all.view(n_shards, n_pods, k).numpy(), k)
        out_node.fill_(-1)
        for p, lst in enumerate(merged):
            out_node[p, :len(lst)] = torch.tensor(lst, dtype=torch.int32)
            out_len[p] = len(lst)


def _worker(rank, world, s, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    for p in (os.path.join(ROOT, "platform-aware-scheduling_amd"), os.path.join(ROOT, "oracle"),
              os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import oracle
    from pas_amd import distrib
    from pas_amd.shard import GridTopK, grid_position, node_range
    distrib.setup("gloo")
    tsnap, tbatch, gsnap, gbatch = case()
    _, shard_id = grid_position(world, s, rank)
    n0, n1 = node_range(N, s, shard_id)
    grid = GridTopK(OracleCtx(oracle, tsnap, gsnap, n0, n1), K, world, rank, s, P, N,
                    tbatch.rules, tbatch.rule_off, tbatch.prio, gbatch.req, gbatch.req_mask,
                    gbatch.n_containers, device="cpu")
    nodes, lens = grid.run(1, 2, 0)
    np.save(os.path.join(out_dir, f"group{rank}.npy"), nodes.numpy())
    np.save(os.path.join(out_dir, f"glen{rank}.npy"), lens.numpy())
    all_nodes, all_lens = grid.gather()
    np.save(os.path.join(out_dir, f"all{rank}.npy"), all_nodes.numpy())
    np.save(os.path.join(out_dir, f"alen{rank}.npy"), all_lens.numpy())
    distrib.teardown(world)


@pytest.mark.parametrize("s", [2, 1, 4])
def test_grid_world4_equals_whole_cluster(tmp_path, oracle, s):
    world = 4
    mp.spawn(_worker, args=(world, s, _free_port(), str(tmp_path)), nprocs=world, join=True)
    from pas_amd.shard import pod_slice
    tsnap, tbatch, gsnap, gbatch = case()
    order, lens = composed_lists(oracle, tsnap, gsnap, tbatch.rules, tbatch.rule_off,
                                 tbatch.prio, gbatch.req, gbatch.req_mask, gbatch.n_containers,
                                 0, N)
    want = np.full((P, K), -1, np.int32)
    for p in range(P):
        m = min(K, int(lens[p]))
        want[p, :m] = order[p, :m]
    g = world // s
    for r in range(world):
        p0, p1 = pod_slice(P, g, r // s)
        np.testing.assert_array_equal(np.load(tmp_path / f"group{r}.npy"), want[p0:p1])
        np.testing.assert_array_equal(np.load(tmp_path / f"glen{r}.npy"),
                                      (want[p0:p1] >= 0).sum(1))
        np.testing.assert_array_equal(np.load(tmp_path / f"all{r}.npy"), want)
        np.testing.assert_array_equal(np.load(tmp_path / f"alen{r}.npy"), (want >= 0).sum(1))


def test_grid_position_and_memory_model():
    from pas_amd.shard import grid_position, min_node_shards, snapshot_bytes_per_node
    assert [grid_position(8, 2, r) for r in range(4)] == [(0, 0), (0, 1), (1, 0), (1, 1)]
    with pytest.raises(ValueError):
        grid_position(8, 3, 0)
    # 1M nodes x 64 metrics is ~5 GB: one shard at every world size; a cluster past the
    # budget takes the fewest shards that divide the world
    assert snapshot_bytes_per_node(64) * 1_000_000 < 6e9
    for world in (1, 2, 4, 8):
        assert min_node_shards(world, 1_000_000, 64, budget_bytes=144e9) == 1
    assert min_node_shards(8, 100_000_000, 64, budget_bytes=144e9) == 4
    assert min_node_shards(8, 100_000_000, 64, budget_bytes=1e9) == 8
