"""Diagnostic: pas_encode_tas_filter_result time for the bench's 100k-node request (node JSON
spliced from the request body, 92 % of the nodes passing) per host thread count."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "platform-aware-scheduling_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from pas_amd import _lib, wire  # noqa: E402

n = 100_000
names = [f"node-{i:06d}" for i in range(n)]
body = bench.synthetic_args_body(names)
table = wire.NameTable(names)
name_arr = wire.NodeTable(names).names
lib = _lib.load()
info = _lib.PasArgsInfo()
req = np.zeros(n, np.int32)
spans = np.zeros((n, 2), np.int64)
cand = np.zeros((n + 63) // 64, np.uint64)
vp = ctypes.c_void_p
body_buf = ctypes.c_char_p(body)
base = ctypes.cast(body_buf, ctypes.c_void_p).value
rc = lib.pas_decode_args(table._h, body_buf, len(body), _lib.PAS_ARGS_NODES, req.ctypes.data_as(vp),
                         n, spans.ctypes.data_as(vp), cand.ctypes.data_as(vp), ctypes.byref(info))
assert rc == 0
addr = np.zeros(n, np.uint64)
lens = np.zeros(n, np.int64)
addr[req] = base + spans[:, 0].astype(np.uint64)
lens[req] = spans[:, 1]
passed = np.random.default_rng(1).random(n) < 0.92
row = np.packbits(passed, bitorder="little")
row = np.pad(row, (0, (-len(row)) % 8)).view(np.uint64)
cap = 1 << 28
out = ctypes.create_string_buffer(cap)
out_len = ctypes.c_int64()
ref = None
for th in [int(x) for x in (sys.argv[1:] or ["1", "2", "4", "8", "16"])]:
    lib.pas_decode_set_threads(th)
    ts = []
    for _ in range(9):
        t0 = time.perf_counter()
        rc = lib.pas_encode_tas_filter_result(
            n, req.ctypes.data_as(vp), row.ctypes.data_as(vp), name_arr,
            addr.ctypes.data_as(ctypes.POINTER(ctypes.c_char_p)), lens.ctypes.data_as(vp), out, cap,
            ctypes.byref(out_len))
        ts.append(time.perf_counter() - t0)
        assert rc == 0
    got = out.raw[:out_len.value]
    ref = ref or got
    assert got == ref
    t = float(np.median(ts))
    print(f"threads {th:2d}: {t * 1e3:6.2f} ms  {out_len.value / t / 1e9:5.2f} GB/s", flush=True)
