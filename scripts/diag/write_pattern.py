import ctypes, os, subprocess, torch
here = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(here, "write_pattern.so")
lib = ctypes.CDLL(so)
x = torch.empty((4096, 100000), dtype=torch.int32, device="cuda")
ms = ctypes.c_float()
for piece in (928, 1024):
    for mode, name in ((0, "row-major"), (1, "segment-major")):
        lib.run(ctypes.c_void_p(x.data_ptr()), 4096, 98, mode, piece, 20, ctypes.byref(ms))
        gb = 4096 * 98 * piece * 4 / 1e9
        print(f"piece {piece*4} B {name}: {ms.value:.3f} ms  {gb/ms.value*1e3:.0f} GB/s")
