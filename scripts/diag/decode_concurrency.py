"""Diagnostic: one-thread pas_decode_args of the 100k-node body run by 1..16 host threads at
once (ctypes releases the GIL): does per-thread decode throughput hold up on this machine?"""
import ctypes
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "platform-aware-scheduling_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from pas_amd import _lib, wire  # noqa: E402

names = [f"node-{i:06d}" for i in range(100_000)]
body = bench.synthetic_args_body(names)
table = wire.NameTable(names)
lib = _lib.load()
lib.pas_decode_set_threads(1)
n = len(names)
vp = ctypes.c_void_p


def run(times):
    info = _lib.PasArgsInfo()
    req = np.zeros(n, np.int32)
    cand = np.zeros((n + 63) // 64, np.uint64)
    for _ in range(3):
        t0 = time.perf_counter()
        lib.pas_decode_args(table._h, body, len(body), 0, req.ctypes.data_as(vp), n, None,
                            cand.ctypes.data_as(vp), ctypes.byref(info))
        times.append(time.perf_counter() - t0)


for nt in (1, 2, 4, 8, 16):
    times = []
    th = [threading.Thread(target=run, args=(times,)) for _ in range(nt)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    print(f"{nt:2d} concurrent one-thread decodes: median {np.median(times) * 1e3:.1f} ms per call",
          flush=True)
