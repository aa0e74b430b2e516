import ctypes, os, torch
here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "write_pattern.so"))
x = torch.empty((4096, 100000), dtype=torch.int32, device="cuda")
ms = ctypes.c_float()
piece = 928
gb = 4096 * 98 * piece * 4 / 1e9
for mode, wg, name in ((0, 0, "1 wave/piece row-major"), (1, 0, "1 wave/piece seg-major"),
                       (2, 1024, "persistent interleaved wg=1024"),
                       (2, 2048, "persistent interleaved wg=2048"),
                       (2, 4096, "persistent interleaved wg=4096"),
                       (3, 1024, "persistent contiguous wg=1024"),
                       (3, 2048, "persistent contiguous wg=2048")):
    lib.run(ctypes.c_void_p(x.data_ptr()), 4096, 98, mode, piece, 20, wg, ctypes.byref(ms))
    print(f"{name}: {ms.value:.3f} ms  {gb/ms.value*1e3:.0f} GB/s")
n = x.numel()
for kind, wg, name, nbytes in ((0, 1024, "linear fill wg=1024", n * 4), (0, 4096, "linear fill wg=4096", n * 4),
                               (0, 16384, "linear fill wg=16384", n * 4),
                               (1, 4096, "linear fill NT wg=4096", n * 4),
                               (2, 1024, "pieces NT wg=1024", gb * 1e9), (2, 4096, "pieces NT wg=4096", gb * 1e9)):
    lib.run2(ctypes.c_void_p(x.data_ptr()), ctypes.c_int64(n), kind, wg, 20, ctypes.byref(ms))
    print(f"{name}: {ms.value:.3f} ms  {nbytes/ms.value/1e6:.0f} GB/s")
for wg in (1024, 4096):
    lib.run3(ctypes.c_void_p(x.data_ptr()), wg, 20, ctypes.byref(ms))
    print(f"pieces NT dword wg={wg}: {ms.value:.3f} ms  {gb/ms.value*1e3:.0f} GB/s")
for R in (1, 2, 4, 8, 98):
    for wg in (2048, 8192):
        lib.run4(ctypes.c_void_p(x.data_ptr()), wg, R, 20, ctypes.byref(ms))
        print(f"runs of {R} pieces NT wg={wg}: {ms.value:.3f} ms  {gb/ms.value*1e3:.0f} GB/s")
