"""Diagnostic: store rate of the TAS ordered-list pattern, one block per
row (the eval kernel) against several blocks per row with a decoupled look-back
(scripts/diag/tas_store.hip).  C2 shape: 4096 rows of 100 000 positions, ~92 % kept per
1024-position segment (1.5 GB of list entries).
Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC scripts/diag/tas_store.hip -o scripts/diag/tas_store.so"""
import ctypes
import os

import numpy as np
import torch

here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "tas_store.so"))
P, N, SEG = 4096, 100_000, 1024
n_seg = (N + SEG - 1) // SEG
rng = np.random.default_rng(0x57)
seg_len = np.full(n_seg, SEG)
seg_len[-1] = N - SEG * (n_seg - 1)
cnt = rng.binomial(np.broadcast_to(seg_len, (P, n_seg)), 0.92).astype(np.int32)
total = int(cnt.sum())
out = torch.empty((P, N), dtype=torch.int32, device="cuda")
cnt_t = torch.from_numpy(cnt).cuda()
ms = ctypes.c_float()
print(f"entries {total} ({total * 4 / 1e9:.3f} GB), {n_seg} segments per row")
for rnd in range(2):
    cases = ((0, 4), (1, 16), (2, 2), (2, 4), (2, 8), (2, 16), (3, 4), (4, 2), (4, 4), (4, 8))
    if rnd == 0:
        cases = cases + ((1, 2), (1, 4), (1, 8))
    for m, per in cases:
        G = (n_seg + per - 1) // per
        flags = torch.zeros(P * G, dtype=torch.int64, device="cuda")
        grp = np.add.reduceat(cnt, np.arange(0, n_seg, per), axis=1)
        pre = np.concatenate([np.zeros((P, 1), np.int64), np.cumsum(grp, axis=1)[:, :-1]], 1)
        pre_t = torch.from_numpy(np.ascontiguousarray(pre)).cuda()
        rc = lib.run(ctypes.c_void_p(out.data_ptr()), ctypes.c_int64(N),
                     ctypes.c_void_p(cnt_t.data_ptr()), P, n_seg, m, per,
                     ctypes.c_void_p(flags.data_ptr()), ctypes.c_void_p(pre_t.data_ptr()), 10,
                     ctypes.byref(ms))
        assert rc == 0, rc
        us = ms.value * 1e3
        print(f"map={m} segs/block={per:2d} blocks/row={G if m in (1, 2, 4) else 1:3d}: {us:7.1f} us "
              f"{total * 4 / (us * 1e-6) / 1e12:5.2f} TB/s", flush=True)
# a plain fill of the same buffer for reference
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(10):
    out.view(-1)[: total].fill_(7)
b.record()
b.synchronize()
us = a.elapsed_time(b) / 10 * 1e3
print(f"torch fill_ of the same bytes: {us:7.1f} us {total * 4 / (us * 1e-6) / 1e12:5.2f} TB/s")
