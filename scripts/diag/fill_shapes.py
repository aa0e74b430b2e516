"""Diagnostic: HBM store rate of a linear fill by issue shape (not product code)."""
import ctypes, os, torch
here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "write_pattern.so"))
x = torch.empty((4096, 100000), dtype=torch.int32, device="cuda")
n = x.numel()
ms = ctypes.c_float()
for _ in range(3):
    x.zero_()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    x.zero_()
e1.record(); torch.cuda.synchronize()
t = e0.elapsed_time(e1) / 20
print(f"torch zero_: {t:.3f} ms {n*4/t/1e6:.0f} GB/s")
for tpb in (256, 1024):
    for U in (1, 2, 4, 8):
        for nt in (0, 1):
            for wg in (2048, 8192, 32768):
                lib.run5(ctypes.c_void_p(x.data_ptr()), ctypes.c_int64(n), U, nt, wg, tpb, 20,
                         ctypes.byref(ms))
                print(f"tpb={tpb} U={U} nt={nt} wg={wg}: {ms.value:.3f} ms {n*4/ms.value/1e6:.0f} GB/s")
