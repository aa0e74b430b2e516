"""The RCCL branches of pas_amd.shard / pas_amd.distrib on the one-GPU box (marked gpu).

Multi-rank tests here use gloo (the box has one GPU, RCCL needs one device per rank), and
every collective short-cuts at world size 1.  A world-1 "nccl" process group is legal on one
GPU, so this test creates one through distrib.setup (with device_id, as bench.py's ranks do)
and forces the collectives through torch.distributed (distrib.force_collectives): the exact
all_gather_into_tensor, all_to_all_single, all_reduce, barrier and all_gather_object calls of
a multi-GPU job run over RCCL, and their results must equal the short-cut (world-1) path's.
"""
import json
import os
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from test_shard import (ROOT, _free_port, _rule_tensors, make_case, shard_cand,
                        shard_snapshot)

pytestmark = pytest.mark.gpu


def _rccl_worker(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="1",
                      RANK="0", LOCAL_RANK="0")
    for p in (os.path.join(ROOT, "platform-aware-scheduling_amd"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import pas_amd
    from pas_amd import distrib, shard
    from pas_amd import workload as wl

    world, _, _ = distrib.setup("nccl", force_group=True)
    assert world == 1 and dist.get_backend() == "nccl"
    res = {}
    try:
        g = torch.Generator(device="cpu").manual_seed(7)
        x = torch.randint(-2**62, 2**62, (37, 5), generator=g, dtype=torch.int64).cuda()
        snap, batch = make_case(0x54, 3000, 6, 40, 5, cand_frac=0.85)
        v, pres = snap.v_milli, snap.present
        gs = wl.make_gas_snapshot(3000, seed=0x54)
        gb = wl.make_gas_batch(40, seed=0x54)
        outs = {}
        with pas_amd.Context(0) as c:
            sv, sp = shard_snapshot(v, pres, 0, v.shape[1])
            c.tas_snapshot_set(3, sv, sp)
            c.gas_snapshot_set(4, gs.n_cards, gs.cap, gs.used)
            rules_t, off_t, prio_t, cand_t = _rule_tensors(batch, shard_cand(batch.cand,
                                                                             v.shape[1], 0,
                                                                             v.shape[1]))
            req_t = torch.from_numpy(gb.req).cuda()
            mask_t = torch.from_numpy(gb.req_mask.view(np.int32)).cuda()
            nc_t = torch.from_numpy(gb.n_containers).cuda()
            viol = torch.randint(-2**62, 2**62, (5, 47), generator=g, dtype=torch.int64).cuda()
            for forced in (False, True):
                distrib.CALLS.clear()
                ctxm = distrib.force_collectives() if forced else _nullcontext()
                with ctxm:
                    o = {}
                    o["gather"] = shard._all_gather(x, 1).cpu()
                    o["a2a"] = shard._all_to_all(x.view(1, 37, 5), 1).cpu()
                    o["viol"] = shard.gather_violations(viol, 1, 47 * 64 - 5).cpu()
                    st = shard.ShardedTopK(c, 9, 1, 0, 0)
                    n1, l1 = st.run(3, len(batch.prio), len(batch.rules), rules_t, off_t, prio_t,
                                    cand_t, stream=torch.cuda.Stream())
                    o["topk"] = (n1.cpu().clone(), l1.cpu().clone())
                    n2, l2 = st.run_tas_gas(3, 4, len(batch.prio), len(batch.rules), rules_t,
                                            off_t, prio_t, gb.req.shape[1], wl.I915, req_t,
                                            mask_t, nc_t, cand_t)
                    o["tas_gas"] = (n2.cpu().clone(), l2.cpu().clone())
                    fl = shard.ShardedFullList(c, v.shape[1], 1, 0, 0)
                    _, _, n3, l3 = fl.run(3, len(batch.prio), len(batch.rules), rules_t, off_t,
                                          prio_t, cand_t)
                    o["full"] = (n3.cpu().clone(), l3.cpu().clone())
                    o["max"] = distrib.max_over_ranks(1.25, 1)
                    distrib.barrier(1)
                    o["objs"] = distrib.gather_objects("r0", 1)
                    torch.cuda.synchronize()
                outs[forced] = o
                if forced:
                    res["calls"] = dict(distrib.CALLS)
                else:
                    assert not distrib.CALLS, dict(distrib.CALLS)
        same = {}
        for name in outs[False]:
            a, b = outs[False][name], outs[True][name]
            if isinstance(a, tuple):
                same[name] = all(torch.equal(p, q) for p, q in zip(a, b))
            elif isinstance(a, torch.Tensor):
                same[name] = torch.equal(a, b)
            else:
                same[name] = a == b
        res["same"] = same
        res["backend"] = dist.get_backend()
    finally:
        distrib.teardown(1, force_group=True)
    with open(os.path.join(out_dir, "rccl.json"), "w") as f:
        json.dump(res, f)


class _nullcontext:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def test_rccl_world1_collectives_equal_shortcut(tmp_path):
    """A world-1 RCCL group runs every collective of the node-sharded paths (ShardedTopK,
    ShardedFullList, gather_violations, the timing all-reduce, barrier, object gather) and
    gives the short-cut path's results bit for bit."""
    mp.spawn(_rccl_worker, args=(_free_port(), str(tmp_path)), nprocs=1, join=True)
    res = json.loads((tmp_path / "rccl.json").read_text())
    assert res["backend"] == "nccl"
    assert all(res["same"].values()), res["same"]
    calls = res["calls"]
    for name in ("all_gather_into_tensor", "all_to_all_single", "all_reduce", "barrier",
                 "all_gather_object"):
        assert calls.get(name, 0) > 0, calls
    assert "all_gather" not in calls  # the gloo staging path did not run
