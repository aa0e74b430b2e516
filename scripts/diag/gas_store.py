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
x = torch.empty((P, 50_048), dtype=torch.int32, device="cuda")
ms = ctypes.c_float()
for pitch in (50_000, 50_048):
    for npl in (1, 2, 4):
        for tpb in (256, 64):
            for blocks in (8192, 16384):
                for aux in (1, 0):
                    lib.run(ctypes.c_void_p(x.data_ptr()), P, N, pitch, npl, tpb, blocks, aux, 10,
                            ctypes.byref(ms))
                    gb = P * N * 4 / 1e9
                    print(f"pitch={pitch} npl={npl} tpb={tpb:4d} blocks={blocks:5d} "
                          f"{'nt   ' if aux else 'plain'}: {ms.value * 1e3:7.1f} us "
                          f"{gb / ms.value:6.0f} GB/s", flush=True)
