"""Diagnostic: HBM write rate of GAS result-word store patterns (scripts/diag/gas_store.hip).
Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC scripts/diag/gas_store.hip -o scripts/diag/gas_store.so
usage: python3 scripts/diag/gas_store.py [P]"""
import ctypes
import os
import sys

import torch

here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "gas_store.so"))
P = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
N = 50_000
x = torch.empty((P, 65_536), dtype=torch.int32, device="cuda")
ms = ctypes.c_float()
import os as _os
only = _os.environ.get("GAS_STORE_MAPS")
cases = [(m, 50_016, 1, 256, b, a) for m in (0, 1) for b in (8192, 16384) for a in (1, 0)]
cases += [(1, 50_016, 4, 256, 8192, 1), (1, 50_000, 1, 256, 8192, 1)]
cases += [(2, 50_000, 4, 256, b, a) for b in (2048, 8192) for a in (1, 0)]
cases += [(3, 50_000, u, t, 0, a) for u in (1, 4, 16) for t in (256, 1024) for a in (1, 0)]
if only:
    cases = [c for c in cases if str(c[0]) in only.split(",")]
if os.environ.get("GAS_STORE_ONESHOT"):  # one-shot row pieces vs the looped tiles
    cases = [(m, 50_016, 4, 256, 0, 1) for m in (4, 5)]
    cases += [(m, 50_016, npl, 256, b, 1) for m in (0, 1, 6) for npl in (1, 4)
              for b in (2048, 8192, 32768)]
if os.environ.get("GAS_STORE_STREAMS"):  # whole-row streams (TAS lists): concurrency sweep
    cases = [(4, 50_016, 4, 256, 0, 1)]
    cases += [(7, 50_016, 4, t, g, a) for t in (256, 1024) for g in (128, 256, 512, 1024, 2048, 4096)
              for a in (1, 0)]
if os.environ.get("GAS_STORE_PITCHES"):  # pitch sweep of the fit kernels' mapping (map 0)
    cases = [(0, 50_016 + 32 * i, 1, 256, 8192, 1) for i in range(40)]
    cases += [(0, p, 1, 256, 8192, 1) for p in (51_200, 52_224, 53_248, 57_344, 65_536)]
for m, pitch, npl, tpb, blocks, aux in cases:
    lib.run(ctypes.c_void_p(x.data_ptr()), P, N, pitch, npl, tpb, blocks, aux, m, 10,
            ctypes.byref(ms))
    gb = P * N * 4 / 1e9
    print(f"map={m} pitch={pitch} npl={npl} tpb={tpb:4d} blocks={blocks:5d} "
          f"{'nt   ' if aux else 'plain'}: {ms.value * 1e3:7.1f} us "
          f"{gb / ms.value:6.0f} GB/s", flush=True)
if os.environ.get("GAS_STORE_PITCHES") or os.environ.get("GAS_STORE_ONESHOT") or \
        os.environ.get("GAS_STORE_STREAMS"):
    sys.exit(0)
t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
y = x[:, :N]
for _ in range(3): x.fill_(7)
t0.record()
for _ in range(10): x.fill_(7)
t1.record(); torch.cuda.synchronize()
print(f"torch fill_ of the {P} x 50048 buffer: {t0.elapsed_time(t1) / 10 * 1e3:7.1f} us "
      f"{P * 50_048 * 4 / 1e9 / (t0.elapsed_time(t1) / 10):6.0f} GB/s", flush=True)
