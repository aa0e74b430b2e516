"""The N>1 bench path on CPU: world_size-2 gloo process groups.

bench.py shards by pod (independent pending pods, replicated snapshot)
and its only cross-rank traffic is the timing protocol in pas_amd/distrib.py.  These tests
run that protocol over gloo and check that pod sharding is exact: the union of the ranks'
results on their pod shards equals one evaluation of the whole batch (oracle as checker).
"""
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _slice_batch(batch, pods):
    """Rules CSR, prio and cand restricted to the listed pods (in that order)."""
    rules, off = [], [0]
    for p in pods:
        a, b = batch.rule_off[p], batch.rule_off[p + 1]
        rules.append(batch.rules[a:b])
        off.append(off[-1] + (b - a))
    rules = np.concatenate(rules) if rules else batch.rules[:0]
    cand = None if batch.cand is None else batch.cand[pods]
    return rules, np.asarray(off, dtype=np.int32), batch.prio[pods], cand


def _worker(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(WORLD),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    sys.path.insert(0, os.path.join(ROOT, "platform-aware-scheduling_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pas_amd import distrib
    from pas_amd import workload as wl
    import oracle

    world, r, _ = distrib.setup("gloo")
    assert (world, r) == (WORLD, rank)

    # timing protocol: the slower rank's time wins on every rank
    naps = [0.002, 0.006]
    elapsed = distrib.timed_steps(lambda: time.sleep(naps[rank]), 5, 1, world, sync=lambda: None)

    # pod sharding: every rank evaluates a contiguous shard of one global batch
    snap = wl.make_tas_snapshot(2000, 4, seed=0xC2)
    batch = wl.make_tas_batch(snap, 10, 3, seed=0xC2, cand_frac=0.9)
    P = len(batch.prio)
    lo, hi = rank * P // world, (rank + 1) * P // world
    rules, off, prio, cand = _slice_batch(batch, list(range(lo, hi)))
    pass_out, order, lens = oracle.tas_eval(snap.v_milli, snap.present, rules, off, prio, cand, 3)
    shards = distrib.gather_objects((lo, hi, pass_out, order, lens), world)
    seeds = distrib.gather_objects(distrib.batch_seed(0xC2, rank), world)
    arrays = {"elapsed": np.float64(elapsed), "seeds": np.asarray(seeds)}
    for i, (slo, shi, sp, so, sl) in enumerate(shards):
        arrays.update({f"b{i}": np.asarray([slo, shi]), f"p{i}": sp, f"o{i}": so, f"l{i}": sl})
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **arrays)
    distrib.teardown(world)


@pytest.fixture(scope="module")
def gloo_run(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("gloo"))
    mp.start_processes(_worker, args=(_free_port(), out), nprocs=WORLD, join=True,
                       start_method="spawn")
    runs = []
    for r in range(WORLD):
        z = np.load(os.path.join(out, f"rank{r}.npz"))
        shards = [(int(z[f"b{i}"][0]), int(z[f"b{i}"][1]), z[f"p{i}"], z[f"o{i}"], z[f"l{i}"])
                  for i in range(WORLD)]
        runs.append({"elapsed": float(z["elapsed"]), "seeds": list(z["seeds"]),
                     "shards": shards})
    return runs


def test_timing_is_max_over_ranks(gloo_run):
    e = [r["elapsed"] for r in gloo_run]
    assert e[0] == e[1]                    # every rank reports the same (max) time
    assert e[0] >= 5 * 0.006               # at least the slower rank's 5 timed steps


def test_rank_batches_are_independent(gloo_run):
    seeds = gloo_run[0]["seeds"]
    assert len(set(seeds)) == WORLD


def test_pod_shards_reassemble_to_the_whole_batch(gloo_run):
    sys.path.insert(0, os.path.join(ROOT, "platform-aware-scheduling_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pas_amd import workload as wl
    import oracle
    snap = wl.make_tas_snapshot(2000, 4, seed=0xC2)
    batch = wl.make_tas_batch(snap, 10, 3, seed=0xC2, cand_frac=0.9)
    want_pass, want_order, want_len = oracle.tas_eval(
        snap.v_milli, snap.present, batch.rules, batch.rule_off, batch.prio, batch.cand, 3)
    for lo, hi, pass_out, order, lens in gloo_run[0]["shards"]:
        np.testing.assert_array_equal(pass_out, want_pass[lo:hi])
        np.testing.assert_array_equal(lens, want_len[lo:hi])
        for i in range(hi - lo):
            np.testing.assert_array_equal(order[i, :lens[i]], want_order[lo + i, :lens[i]])


def test_whole_job_rate():
    sys.path.insert(0, os.path.join(ROOT, "platform-aware-scheduling_amd"))
    from pas_amd import distrib
    assert distrib.whole_job_rate(4096 * 100_000, 8, 10, 2.0) == 4096 * 100_000 * 8 * 10 / 2.0


def _settle_worker(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(WORLD),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    sys.path.insert(0, os.path.join(ROOT, "platform-aware-scheduling_amd"))
    import torch
    import torch.distributed as dist
    from pas_amd import distrib
    world, _, _ = distrib.setup("gloo")
    # a step holding a collective, slower on rank 1: settle must stop both ranks at the same
    # step count, or the faster one would wait in an all-reduce nobody joins
    naps = [0.001, 0.004]

    def step():
        time.sleep(naps[rank])
        t = torch.ones(1)
        dist.all_reduce(t)
    n = distrib.settle(step, 0.15, sync=lambda: None, world=world)
    elapsed = distrib.timed_steps(step, 3, 1, world, sync=lambda: None)
    np.save(os.path.join(out_dir, f"settle{rank}.npy"), np.array([n, elapsed]))
    distrib.teardown(world)


def test_settle_agrees_across_ranks(tmp_path):
    mp.spawn(_settle_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    a, b = (np.load(tmp_path / f"settle{r}.npy") for r in range(WORLD))
    assert a[0] == b[0] and a[0] >= 4 and a[0] % 4 == 0
