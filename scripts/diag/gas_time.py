"""Diagnostic: C3 fit time only (no result checks), for A/B builds whose results are not
exact (e.g. PAS_GAS_DIAG_NORANK).  usage: python gas_time.py [reps]  (run from a tree)."""
import os
import sys

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(R, "platform-aware-scheduling_amd"))
import pas_amd  # noqa: E402
from pas_amd import workload as wl  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
P, N = 10_000, 50_000
ctx = pas_amd.Context(0)
s = torch.cuda.current_stream()
ctx.set_stream(s)
snap = wl.make_gas_snapshot(N, seed=0xC3)
batch = wl.make_gas_batch(P, seed=0xC3)
K, Q = snap.used.shape[1], snap.used.shape[2]
dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
ctx.gas_snapshot_set_device(1, N, K, Q, dev(snap.n_cards), dev(snap.cap), dev(snap.used), s)
req_t, mask_t, nc_t = dev(batch.req), dev(batch.req_mask.view(np.int32)), dev(batch.n_containers)
ld = (N + 31) // 32 * 32
res = torch.empty((P, ld), dtype=torch.int32, device="cuda")
C = batch.req.shape[1]
for _ in range(200):
    ctx.gas_fit_ld_device(1, P, C, wl.I915, req_t, mask_t, nc_t, res, ld, stream=s)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record(s)
for _ in range(reps):
    ctx.gas_fit_ld_device(1, P, C, wl.I915, req_t, mask_t, nc_t, res, ld, stream=s)
b.record(s)
torch.cuda.synchronize()
print(f"{os.path.basename(R)} C3 ms {a.elapsed_time(b) / reps:.4f}")
