"""pas_encode_tas_filter_result over host threads (the node objects of the items array copied
in parallel, csrc/wire_json.cpp) gives exactly the one-thread body, and the capacity contract
holds across the copy (bytes past cap counted, not stored).  The body is the reference's
json.NewEncoder(w).Encode(FilterResult) (telemetryscheduler.go:184-225, 238-244)."""
import ctypes
import json

import numpy as np
import pytest

from pas_amd import _lib, wire


@pytest.fixture(scope="module")
def table():
    rng = np.random.default_rng(8)
    n = 40000
    names = [f"node-{i:06d}" for i in range(n)]
    objs = [json.dumps({"metadata": {"name": names[i], "labels": {"l": "x" * int(rng.integers(0, 300))}},
                        "status": {"allocatable": {"cpu": str(i % 97)}}},
                       separators=(",", ":")).encode() for i in range(n)]
    return wire.NodeTable(names, objs), names, objs


def encode(table, req, pass_row, threads, cap=None):
    lib = _lib.load()
    assert lib.pas_decode_set_threads(threads) == 0
    try:
        if cap is None:
            return wire.tas_filter_result(req, pass_row, table)
        req = np.ascontiguousarray(req, np.int32)
        pass_row = np.ascontiguousarray(pass_row, np.uint64)
        buf = ctypes.create_string_buffer(max(cap, 1))
        n = ctypes.c_int64()
        rc = lib.pas_encode_tas_filter_result(
            len(req), req.ctypes.data_as(ctypes.c_void_p), pass_row.ctypes.data_as(ctypes.c_void_p),
            table.names, table.node_json, table.node_json_len.ctypes.data_as(ctypes.c_void_p), buf,
            cap, ctypes.byref(n))
        return rc, n.value, buf.raw[:cap]
    finally:
        lib.pas_decode_set_threads(0)


def expected(names, objs, req, passed):
    items = [objs[n] for n in req if passed[n]]
    ok = [names[n] for n in req if passed[n]]
    bad = sorted({names[n] for n in req if not passed[n]})
    body = (b'{"Nodes":{"metadata":{},"items":' +
            ((b"[" + b",".join(items) + b"]") if items else b"null") +
            b'},"NodeNames":[' + b"".join(json.dumps(x).encode() + b"," for x in ok) + b'""],' +
            b'"FailedNodes":{' + b",".join(json.dumps(x).encode() + b':"Node violates"'
                                          for x in bad) + b'},"Error":""}\n')
    return body


@pytest.mark.parametrize("frac", [0.0, 0.01, 0.5, 0.97, 1.0])
def test_threads_equal_one_thread_and_reference(table, frac):
    t, names, objs = table
    rng = np.random.default_rng(int(frac * 100))
    n = len(names)
    req = rng.permutation(n)[: n - 123].astype(np.int32)
    passed = rng.random(n) < frac
    row = np.packbits(passed, bitorder="little")
    row = np.pad(row, (0, (-len(row)) % 8)).view(np.uint64)
    one = encode(t, req, row, 1)
    assert one == expected(names, objs, req, passed)
    for threads in (2, 5, 16):
        assert encode(t, req, row, threads) == one


@pytest.mark.parametrize("cut", [0, 1, 37, 1000, 3_000_000, -2, -1])
def test_capacity_past_the_parallel_copy(table, cut):
    t, names, objs = table
    rng = np.random.default_rng(3)
    n = len(names)
    req = np.arange(n, dtype=np.int32)
    passed = rng.random(n) < 0.9
    row = np.packbits(passed, bitorder="little")
    row = np.pad(row, (0, (-len(row)) % 8)).view(np.uint64)
    full = encode(t, req, row, 1)
    cap = cut if cut >= 0 else len(full) + cut + 1
    for threads in (1, 8):
        rc, out_len, got = encode(t, req, row, threads, cap=cap)
        assert out_len == len(full)
        assert rc == (_lib.PAS_OK if cap >= len(full) else _lib.PAS_ECAPACITY)
        assert got[:cap] == full[:cap]


def _with_threads(threads, fn):
    lib = _lib.load()
    assert lib.pas_decode_set_threads(threads) == 0
    try:
        return fn()
    finally:
        lib.pas_decode_set_threads(0)


def test_host_priority_list_threads():
    # HostPriorityList of 60k entries ({"Host":..,"Score":10-i}, Score past -59 990), names
    # with escapes and multi-byte code points
    rng = np.random.default_rng(4)
    names = [f"né-{i}" + ("<&>" if i % 7 == 0 else "") + ('"' if i % 11 == 0 else "")
             for i in range(70000)]
    table = wire.NodeTable(names)
    order = rng.permutation(70000)[:60000].astype(np.int32)
    one = _with_threads(1, lambda: wire.host_priority_list(order, table))
    want = (json.dumps([{"Host": names[o], "Score": 10 - i} for i, o in enumerate(order)],
                       separators=(",", ":"), ensure_ascii=False)
            .replace("<", "\\u003c").replace(">", "\\u003e").replace("&", "\\u0026")
            .encode() + b"\n")
    assert one == want
    for threads in (3, 16):
        assert _with_threads(threads, lambda: wire.host_priority_list(order, table)) == one


def test_node_names_with_spaces_threads(table):
    # NodeNames is strings.Split of "name name ... " on " ": names with spaces split
    t, names, objs = table
    spaced = [n.replace("-0", " 0") if i % 5 == 0 else n for i, n in enumerate(names)]
    t2 = wire.NodeTable(spaced, objs)
    n = len(names)
    req = np.arange(n, dtype=np.int32)
    passed = np.random.default_rng(9).random(n) < 0.8
    row = np.packbits(passed, bitorder="little")
    row = np.pad(row, (0, (-len(row)) % 8)).view(np.uint64)
    one = encode(t2, req, row, 1)
    got = json.loads(one)
    want_names = " ".join(spaced[i] for i in range(n) if passed[i]) + " "
    assert got["NodeNames"] == want_names.split(" ")
    for threads in (2, 16):
        assert encode(t2, req, row, threads) == one


def test_host_priority_list_threads_past_the_estimate():
    # names far longer than the per-item estimate (40 B) and full of escapes (6 output bytes
    # per input byte): every thread's range outgrows its first buffer and is encoded again
    names = [("<" * 40) + f"-{i}-" + ("\u2028" * 8) for i in range(9000)]
    table = wire.NodeTable(names)
    order = np.random.default_rng(9).permutation(9000).astype(np.int32)
    one = _with_threads(1, lambda: wire.host_priority_list(order, table))
    want = (json.dumps([{"Host": names[o], "Score": 10 - i} for i, o in enumerate(order)],
                       separators=(",", ":"), ensure_ascii=False)
            .replace("<", "\\u003c").replace("\u2028", "\\u2028").encode() + b"\n")
    assert one == want
    for threads in (2, 8, 16):
        assert _with_threads(threads, lambda: wire.host_priority_list(order, table)) == one
