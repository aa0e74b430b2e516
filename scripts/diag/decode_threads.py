"""Diagnostic: pas_decode_args time of the bench's 100k-node body per host thread count."""
import ctypes
import os
import sys
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
info = _lib.PasArgsInfo()
n = len(names)
req = np.zeros(n, np.int32)
spans = np.zeros((n, 2), np.int64)
cand = np.zeros((n + 63) // 64, np.uint64)
vp = ctypes.c_void_p
for th in [int(x) for x in (sys.argv[1:] or ["1", "2", "4", "8", "12", "16"])]:
    lib.pas_decode_set_threads(th)
    ts = []
    for _ in range(7):
        t0 = time.perf_counter()
        rc = lib.pas_decode_args(table._h, body, len(body), _lib.PAS_ARGS_NODES,
                                 req.ctypes.data_as(vp), n, spans.ctypes.data_as(vp),
                                 cand.ctypes.data_as(vp), ctypes.byref(info))
        ts.append(time.perf_counter() - t0)
        assert rc == 0 and info.n_req == n
    t = float(np.median(ts))
    print(f"threads {th:2d}: {t * 1e3:6.2f} ms  {len(body) / t / 1e9:5.2f} GB/s", flush=True)
print("os.cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
