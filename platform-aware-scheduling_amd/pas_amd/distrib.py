"""Process-per-GPU plumbing for bench.py: rendezvous, barriers, max-over-ranks timing.

The TAS/GAS batches shard by pod (every pending pod is scheduled independently against
the same snapshot, telemetryscheduler.go:184-225 and gpuscheduler/scheduler.go:449-482 take
one pod per request), so N ranks run N independent batches with no data-path collective.
The only cross-rank traffic is the timing protocol below: a barrier on both sides of the
timed region and an all-reduce(MAX) of the elapsed time.  The same code runs over RCCL
("nccl") on GPUs and over gloo on CPU in the tests.
"""
import contextlib
import os
import time
from collections import Counter

import torch

# torch.distributed calls made by this package, by name (the RCCL evidence of
# tests/test_rccl.py; a counter add per collective)
CALLS: Counter = Counter()
_FORCE = [False]


@contextlib.contextmanager
def force_collectives():
    """Run every collective of this package through torch.distributed even at world size 1
    (which otherwise short-cuts them): a world-1 RCCL group then executes the same
    all_gather_into_tensor / all_to_all_single / all_reduce calls a multi-GPU job makes."""
    old = _FORCE[0]
    _FORCE[0] = True
    try:
        yield
    finally:
        _FORCE[0] = old


def collective(world):
    """True when a collective over `world` ranks must go through torch.distributed."""
    return world > 1 or _FORCE[0]


def setup(backend=None, force_group=False):
    """Read RANK/LOCAL_RANK/WORLD_SIZE (torchrun) and join the process group when N > 1 (or
    always, with force_group: a world-1 group for tests/test_rccl.py).

    backend None picks "nccl" (RCCL) when HIP devices are visible, else "gloo"."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = backend != "gloo" and torch.cuda.is_available()
    if gpu:
        torch.cuda.set_device(local if world > 1 else 0)
    if world > 1 or force_group:
        import torch.distributed as dist
        if backend is None:
            backend = "nccl" if gpu else "gloo"
        kw = {"device_id": torch.device("cuda", local)} if backend == "nccl" else {}
        dist.init_process_group(backend=backend, **kw)
    return world, rank, local


def teardown(world, force_group=False):
    if world > 1 or force_group:
        import torch.distributed as dist
        dist.destroy_process_group()


def _device():
    import torch.distributed as dist
    return "cuda" if dist.get_backend() == "nccl" else "cpu"


def barrier(world):
    if collective(world):
        import torch.distributed as dist
        CALLS["barrier"] += 1
        dist.barrier()


def max_over_ranks(x, world):
    if not collective(world):
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=_device())
    CALLS["all_reduce"] += 1
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_objects(obj, world):
    """All ranks' `obj`, in rank order (tests and result checks only)."""
    if not collective(world):
        return [obj]
    import torch.distributed as dist
    out = [None] * max(world, dist.get_world_size())
    CALLS["all_gather_object"] += 1
    dist.all_gather_object(out, obj)
    return out


def settle(step, seconds, sync=None, world=1):
    """Untimed steps for `seconds` of wall time before the warmup: the first ~20 steps of a
    fresh process run a few % slower (clocks, page tables), which a handful of warmup steps
    does not cover.  Returns the number of steps run.  With world > 1 every rank runs the
    same number of steps (the ranks agree after each round of 4), since a step may hold a
    collective: ranks stopping at different counts would leave one waiting forever."""
    if sync is None:
        sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
    n, t0 = 0, time.perf_counter()
    while True:
        go = time.perf_counter() - t0 < seconds
        if world > 1:
            go = max_over_ranks(0.0 if go else 1.0, world) == 0.0  # all ranks still in time
        if not go:
            return n
        for _ in range(4):
            step()
        n += 4
        sync()


def timed_steps(step, steps, warmup, world, sync=None, gpu=None, fork=None, join=None):
    """Run `warmup` untimed steps, then time exactly `steps` steps bracketed by
    sync + barrier on both sides; returns the MAX elapsed seconds over ranks.
    gpu: a dict that receives "ms_per_step", the GPU time of the timed steps measured by two
    HIP events on the current stream around them (no events between the steps).
    fork / join: called right after the start event and right before the end event (steps
    launched on streams of their own: those wait for the start and the end waits for them)."""
    if sync is None:
        sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
    for _ in range(warmup):
        step()
    sync()
    barrier(world)
    sync()
    ev = None
    if gpu is not None:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    t0 = time.perf_counter()
    if ev:
        ev[0].record()
    if fork:
        fork()
    for _ in range(steps):
        step()
    if join:
        join()
    if ev:
        ev[1].record()
    sync()
    barrier(world)
    t1 = time.perf_counter()
    if ev:
        gpu["ms_per_step"] = ev[0].elapsed_time(ev[1]) / max(steps, 1)
    return max_over_ranks(t1 - t0, world)


def whole_job_rate(units_per_rank_per_step, world, steps, elapsed_s):
    """bench.py's `value`: units ALL ranks processed / the max-over-ranks wall time."""
    return units_per_rank_per_step * world * steps / elapsed_s


def batch_seed(base, rank):
    """Seed of rank `rank`'s independent pod batch (weak scaling: same size per rank)."""
    return base + 7919 * rank


def launch_local_ranks(n, argv, master_port=None):
    """Start `argv` as n local ranks (RANK = LOCAL_RANK = r, WORLD_SIZE = n, rendezvous on
    127.0.0.1) the way torchrun would, wait for all of them and return the first non-zero
    exit status (0 if every rank succeeded).  The caller must not have initialised HIP:
    the children are fresh processes (no fork of a GPU context, no exec of this one)."""
    import signal
    import socket
    import subprocess
    if master_port is None:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            master_port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(master_port))
        procs.append(subprocess.Popen(argv, env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:  # one rank failed: the others would block in a collective
                    q.send_signal(signal.SIGTERM)
        if pending:
            time.sleep(0.05)
    return rc if rc >= 0 else 128 - rc
