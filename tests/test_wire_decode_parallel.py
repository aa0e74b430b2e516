"""pas_decode_args over host threads (structural index + items decoded in parallel,
csrc/wire_decode.cpp) gives exactly the one-thread decode: request node ids, candidate
bitmap, item spans, args info and every error — on large bodies whose chunk boundaries fall
inside strings, escapes, backslash runs, nested containers and unknown fields (SURVEY.md §8
f2; telemetryscheduler.go:63-78)."""
import ctypes
import json

import numpy as np
import pytest

from pas_amd import _lib, wire


def decode(table, body, threads):
    lib = _lib.load()
    assert lib.pas_decode_set_threads(threads) == 0
    try:
        n = table.size + 64
        info = _lib.PasArgsInfo()
        req = np.full(n, -7, np.int32)
        spans = np.zeros((n, 2), np.int64)
        cand = np.zeros((table.size + 63) // 64, np.uint64)
        vp = ctypes.c_void_p
        rc = lib.pas_decode_args(table._h, body, len(body), _lib.PAS_ARGS_NODES,
                                 req.ctypes.data_as(vp), n, spans.ctypes.data_as(vp),
                                 cand.ctypes.data_as(vp), ctypes.byref(info))
        k = info.n_req if rc == 0 else 0
        return (rc, info.has_nodes, info.has_node_names, info.n_req, info.n_unknown,
                info.pod_off, info.pod_len, req[:k].tobytes(), spans[:k].tobytes(),
                cand.tobytes() if rc == 0 else b"")
    finally:
        lib.pas_decode_set_threads(0)


def node_json(name, i, rng):
    # labels with structural characters, escapes and backslash runs inside strings, nested
    # arrays / objects, numbers, true/false/null: everything the index must see through
    tricky = ['a,b', '}]', '[{', '\\"quoted\\"', 'back\\\\\\\\slash', 'x\\\\', '\\u00e9\\u2028',
              '{\\"k\\":[1,2]}', '\\\\', 'end\\\\\\\\\\\\']
    t = tricky[i % len(tricky)]
    extra = "".join(',"f%d":[%d,{"x":"%s"},[[],{}],true,null,-1.5e3]' % (j, j, t)
                    for j in range(int(rng.integers(0, 4))))
    return ('{"metadata":{"name":"%s","labels":{"l":"%s","n":"%d"}},"spec":{"taints":[]},'
            '"status":{"images":[{"names":["r/%s@sha"],"sizeBytes":%d}]%s}}'
            % (name, t, i, t, i * 7, extra))


def body_of(items, pod='{"metadata":{"name":"p","labels":{"telemetry-policy":"x"}}}',
            tail=',"NodeNames":null'):
    return ('{"Pod":%s,"Nodes":{"metadata":{},"items":[%s]}%s}' % (pod, ",".join(items), tail)
            ).encode()


@pytest.fixture(scope="module")
def case():
    rng = np.random.default_rng(5)
    names = [f"node-{i:06d}" for i in range(30000)]
    table = wire.NameTable(names)
    order = rng.permutation(len(names))
    items = [node_json(names[j] if i % 97 else f"unknown-{i}", i, rng)
             for i, j in enumerate(order)]
    return table, items


@pytest.mark.parametrize("threads", [2, 3, 8, 16])
def test_parallel_equals_sequential(case, threads):
    table, items = case
    body = body_of(items)
    assert len(body) > 4 << 20
    want = decode(table, body, 1)
    assert want[0] == 0 and want[3] == len(items) and want[4] > 0
    assert decode(table, body, threads) == want


@pytest.mark.parametrize("shift", [0, 1, 2, 63, 64, 65, 1000])
def test_chunk_boundaries_everywhere(case, shift):
    # leading whitespace moves every chunk boundary against the content
    table, items = case
    body = b" " * shift + body_of(items[:9000]) + b"\n"
    assert decode(table, body, 7) == decode(table, body, 1)


@pytest.mark.parametrize("mutate", [
    "unterminated", "bad_escape", "missing_comma", "extra_comma", "trailing_comma",
    "leading_comma", "type_error", "bad_close", "control_char", "deep"])
def test_errors_same_as_sequential(case, mutate):
    table, items = case
    items = list(items[:8000])
    k = 4321
    if mutate == "unterminated":
        items[k] = items[k][:40]
    elif mutate == "bad_escape":
        items[k] = items[k].replace('"l":"', '"l":"\\q', 1)
    elif mutate == "missing_comma":
        items[k] = items[k] + items[k + 1]
        del items[k + 1]
    elif mutate == "extra_comma":
        items.insert(k, "")
    elif mutate == "trailing_comma":
        items.append("")
    elif mutate == "leading_comma":
        items.insert(0, "")
    elif mutate == "type_error":
        items[k] = items[k].replace('"name":"', '"name":5,"x":"', 1)
    elif mutate == "bad_close":
        items[k] = items[k][:-1] + "]"
    elif mutate == "control_char":
        items[k] = items[k].replace('"l":"', '"l":"\x01', 1)
    elif mutate == "deep":
        # under an unknown key (skipped, still depth-checked by the scanner): an array under
        # "spec" would be a type error of its own (NodeSpec is a struct)
        items[k] = '{"x":' + "[" * 9997 + "]" * 9997 + "}"  # past encoding/json's 10000
    body = body_of(items)
    seq = decode(table, body, 1)
    assert seq[0] != 0 or mutate == "deep"
    assert decode(table, body, 8) == seq


def test_depth_just_inside_limit(case):
    table, items = case
    items = list(items[:6000])
    items[100] = '{"x":' + "[" * 9995 + "]" * 9995 + "}"  # depth 4 + 9995 < 10001
    body = body_of(items)
    seq = decode(table, body, 1)
    assert seq[0] == 0
    assert decode(table, body, 8) == seq


def test_shapes_the_index_declines(case):
    table, items = case
    big = list(items[:6000])
    bodies = [
        body_of([]) + b" " * (6 << 20),                           # empty items, large body
        body_of(big, tail=',"Nodes":{"items":[%s]}' % ",".join(big[:10])),   # Nodes twice
        body_of(big).replace(b'"items":[', b'"items":[],"Items":[', 1),      # items twice
        body_of(big, pod='{"spec":{"containers":[%s]}}' % ",".join(['{"name":"c"}'] * 90000)),
        ('{"Nodes":{"items":[%s]},"Pod":null}' % ",".join(big)).encode(),
        ('[%s]' % ",".join(big)).encode(),                         # not an object
        ('{"Nodes":[%s]}' % ",".join(big)).encode(),               # NodeList not an object
        ('{"Pod":{"x":[%s]},"Nodes":{"items":[]}}' % ",".join(big)).encode(),
    ]
    for b in bodies:
        assert decode(table, b, 8) == decode(table, b, 1)


def test_invalid_utf8_and_unicode_names(case):
    table, items = case
    items = list(items[:6000])
    items[10] = items[10].replace('"l":"', '"l":"\xff\xfe', 1)
    items[11] = '{"metadata":{"name":"n\\u00f8de-\\ud83d\\ude00"}}'
    items[12] = '{"metadata":{"name":"node-000012\\u0000"}}'
    body = body_of(items).replace(b"\xc3\xbf\xc3\xbe", b"\xff\xfe")
    assert decode(table, body, 8) == decode(table, body, 1)


def test_thread_count_api():
    lib = _lib.load()
    assert lib.pas_decode_set_threads(-1) == _lib.PAS_EINVAL
    assert lib.pas_decode_threads(100) == 1  # under 1 MB per thread: one thread
    assert lib.pas_decode_set_threads(4) == 0
    assert lib.pas_decode_threads(90 << 20) == 4
    assert lib.pas_decode_threads(3 << 20) == 3
    assert lib.pas_decode_set_threads(0) == 0
    assert 1 <= lib.pas_decode_threads(90 << 20) <= 16
