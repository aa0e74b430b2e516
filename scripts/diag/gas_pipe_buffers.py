"""Diagnostic: C3 GAS fits per batch on 1 / 2 streams with 1 / 2 result buffers, to separate
the cross-stream ordering from the result working set (round 6).
Prints ms per batch for each variant (GPU events around 20 batches after 3 warmup)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "platform-aware-scheduling_amd"))
import pas_amd  # noqa: E402
from pas_amd import workload as wl  # noqa: E402

P, N, STEPS = 10000, 50000, 20
ctx = pas_amd.Context(0)
main = torch.cuda.current_stream()
ctx.set_stream(main)
snap = wl.make_gas_snapshot(N, seed=0xC3)
batch = wl.make_gas_batch(P, seed=0xC3)
dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
K, Q = snap.used.shape[1], snap.used.shape[2]
C = batch.req.shape[1]
ctx.gas_snapshot_set_device(1, N, K, Q, dev(snap.n_cards), dev(snap.cap), dev(snap.used), main)
req_t, mask_t, nc_t = dev(batch.req), dev(batch.req_mask.view(np.int32)), dev(batch.n_containers)
ld = (N + 31) // 32 * 32
bufs = [torch.empty((P, ld), dtype=torch.int32, device="cuda") for _ in range(2)]
lanes = [torch.cuda.Stream() for _ in range(2)]


def run(n_streams, n_bufs):
    streams = [main] if n_streams == 1 else lanes[:n_streams]

    def step(i):
        s = streams[i % n_streams]
        ctx.gas_fit_ld_device(1, P, C, wl.I915, req_t, mask_t, nc_t, bufs[i % n_bufs], ld,
                              stream=s)

    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(main)
    for s in lanes:
        s.wait_stream(main)
    for i in range(STEPS):
        step(i)
    for s in lanes:
        main.wait_stream(s)
    b.record(main)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / STEPS


if len(sys.argv) > 1:  # one variant (kernel-trace timelines): gas_pipe_buffers.py STREAMS
    STEPS = 8
    print(f"streams={sys.argv[1]} ms/batch={run(int(sys.argv[1]), 2):.4f}", flush=True)
else:
    for rnd in range(2):
        for ns, nb in ((1, 1), (1, 2), (2, 1), (2, 2)):
            print(f"streams={ns} buffers={nb} ms/batch={run(ns, nb):.4f}", flush=True)
ctx.synchronize()
