"""Wire encoders: the extender response bodies, byte-exact with what the
reference's handlers write through json.NewEncoder(w).Encode (Go 1.16 encoding/json).
Host code in libpas.so, so these run on CPU.  The expected bytes come from an independent
Python restatement of encoding/json's rules (struct fields in declaration order, map keys
sorted, HTML-safe string escaping, nil slices as null, trailing newline) and from the
reference's own test expectations (G5 HostPriorityList, G7 FailedNodes)."""
import json

import numpy as np
import pytest

from helpers import golden
from pas_amd import wire

G = golden()


def go_string(b: bytes) -> bytes:
    """encodeState.string (encoding/json/encode.go, Go 1.16) with escapeHTML = true."""
    out = bytearray(b'"')
    i = 0
    while i < len(b):
        c = b[i]
        if c < 0x80:
            if c in (0x22, 0x5C):
                out += b"\\" + bytes([c])
            elif c == 0x0A:
                out += b"\\n"
            elif c == 0x0D:
                out += b"\\r"
            elif c == 0x09:
                out += b"\\t"
            elif c < 0x20 or c in (0x3C, 0x3E, 0x26):
                out += b"\\u00%02x" % c
            else:
                out.append(c)
            i += 1
            continue
        # decode one rune as utf8.DecodeRune does; invalid -> one byte of U+FFFD
        for n in (2, 3, 4):
            try:
                ch = b[i:i + n].decode("utf-8")
            except UnicodeDecodeError:
                continue
            if len(ch) == 1:
                break
        else:
            out += b"\\ufffd"
            i += 1
            continue
        if ch in ("\u2028", "\u2029"):
            out += b"\\u%04x" % ord(ch)
        else:
            out += ch.encode("utf-8")
        i += n
    out += b'"'
    return bytes(out)


def go_priority_list(hosts):
    items = [b'{"Host":' + go_string(h) + b',"Score":' + str(10 - i).encode() + b"}"
             for i, h in enumerate(hosts)]
    return b"[" + b",".join(items) + b"]\n"


def go_failed(names, reason):
    keys = sorted(set(names))
    return b"{" + b",".join(go_string(k) + b":" + go_string(reason) for k in keys) + b"}"


def table(names, json_blobs=None):
    t = wire.NodeTable([""] * len(names), json_blobs)
    # keep raw bytes names (invalid UTF-8 included)
    t._names = [n if isinstance(n, bytes) else n.encode() for n in names]
    t.names = (wire.c_char_p * max(len(t._names), 1))(*t._names)
    return t


def random_names(rng, n):
    pool = [b"a", b"-", b".", b"7", b"<", b">", b"&", b'"', b"\\", b"\n", b"\x01", b"\x7f",
            "é".encode(), "\u2028".encode(), "\u2029".encode(), "😀".encode(), b"\xff",
            b"\xc3", b"\xe2\x80", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b" "]
    return [b"node-%d-" % i + b"".join(pool[j] for j in rng.integers(0, len(pool), size=6))
            for i in range(n)]


def test_go_string_restatement_matches_json_dumps_on_valid_text():
    # sanity of the Python restatement itself: for valid UTF-8 without the HTML / line-separator
    # cases it must agree with a plain compact JSON encoder
    for s in ["node A", "kind-worker2", "é ü 😀", "tab\there", 'q"uote', "back\\slash"]:
        assert go_string(s.encode()) == json.dumps(s, ensure_ascii=False).encode()


def test_priority_list_golden_g5():
    g = G["G5_prioritize"]
    t = table(g["nodes"])
    order = [g["nodes"].index(h) for h, _ in g["want"]]
    got = wire.host_priority_list(order, t)
    assert json.loads(got) == [{"Host": h, "Score": s} for h, s in g["want"]]
    assert got == b'[{"Host":"node A","Score":10},{"Host":"node B","Score":9}]\n'


def test_priority_list_random_and_negative_scores():
    rng = np.random.default_rng(1)
    names = random_names(rng, 40)
    t = table(names)
    for ln in (0, 1, 11, 12, 40):
        order = rng.permutation(40)[:ln]
        assert wire.host_priority_list(order, t) == go_priority_list([names[i] for i in order])
    assert wire.host_priority_list([], t) == b"[]\n"  # &extender.HostPriorityList{}


def test_tas_filter_result_golden_g7():
    g = G["G7_filter"]
    blobs = [b'{"metadata":{"name":"%s"},"spec":{},"status":{}}' % n.encode()
             for n in g["nodes"]]
    t = table(g["nodes"], blobs)
    t.node_json = (wire.c_char_p * len(blobs))(*blobs)
    for c in g["cases"]:
        passed = np.array([n in c["want_passed"] for n in g["nodes"]])
        row = np.zeros(1, np.uint64)
        for i, p in enumerate(passed):
            if p:
                row[0] |= np.uint64(1 << i)
        got = wire.tas_filter_result(np.arange(len(g["nodes"])), row, t)
        res = json.loads(got)
        # the reference test's assertion: FailedNodes keys (scheduler_test.go:321-337)
        assert sorted(res["FailedNodes"]) == sorted(c["want_failed"])
        assert res["NodeNames"] == c["want_node_names"]
        items = [blobs[i] for i in range(len(g["nodes"])) if passed[i]]
        want = (b'{"Nodes":{"metadata":{},"items":' +
                (b"[" + b",".join(items) + b"]" if items else b"null") +
                b'},"NodeNames":[' +
                b"".join(go_string(x.encode()) + b"," for x in c["want_node_names"][:-1]) +
                b'""],"FailedNodes":' + go_failed([n.encode() for n in c["want_failed"]],
                                                  b"Node violates") + b',"Error":""}\n')
        assert got == want


def test_tas_filter_result_random():
    rng = np.random.default_rng(2)
    n = 300
    names = random_names(rng, n)
    blobs = [b'{"metadata":{"name":%s}}' % go_string(x) for x in names]
    t = table(names, blobs)
    t.node_json = (wire.c_char_p * n)(*blobs)
    for frac in (0.0, 0.5, 1.0):
        req = rng.choice(n, size=120, replace=True)  # duplicates: FailedNodes dedups
        bits = rng.random(n) < frac
        row = np.zeros((n + 63) // 64, np.uint64)
        for i in np.nonzero(bits)[0]:
            row[i >> 6] |= np.uint64(1 << (i & 63))
        got = wire.tas_filter_result(req, row, t)
        kept = [i for i in req if bits[i]]
        node_names = b"".join(names[i] + b" " for i in kept).split(b" ")
        want = (b'{"Nodes":{"metadata":{},"items":' +
                (b"[" + b",".join(blobs[i] for i in kept) + b"]" if kept else b"null") +
                b'},"NodeNames":[' + b",".join(go_string(x) for x in node_names) +
                b'],"FailedNodes":' + go_failed([names[i] for i in req if not bits[i]],
                                                b"Node violates") + b',"Error":""}\n')
        assert got == want


def test_gas_filter_result():
    rng = np.random.default_rng(3)
    n = 200
    names = random_names(rng, n)
    t = table(names)
    reason = b"Not enough GPU-resources for deployment"
    for frac in (0.0, 0.3, 1.0):
        req = rng.choice(n, size=90, replace=False)
        bits = rng.random(n) < frac
        row = np.zeros((n + 63) // 64, np.uint64)
        for i in np.nonzero(bits)[0]:
            row[i >> 6] |= np.uint64(1 << (i & 63))
        got = wire.gas_filter_result(req, row, t)
        kept = [names[i] for i in req if bits[i]]
        want = (b'{"Nodes":null,"NodeNames":' +
                (b"[" + b",".join(go_string(x) for x in kept) + b"]" if kept else b"null") +
                b',"FailedNodes":' + go_failed([names[i] for i in req if not bits[i]], reason) +
                b',"Error":""}\n')
        assert got == want
    # empty NodeNames: the misconfiguration error (scheduler.go:455-461)
    err = json.loads(wire.gas_filter_result([], np.zeros(4, np.uint64), t))
    assert err == {"Nodes": None, "NodeNames": None, "FailedNodes": None,
                   "Error": "No nodes to compare. This should not happen, perhaps the extender "
                            "is misconfigured with NodeCacheCapable == false."}


def test_encoder_errors_and_capacity():
    import ctypes
    from pas_amd import _lib
    lib = _lib.load()
    t = table(["a", "b"])
    order = np.array([0, 1], np.int32)
    n = ctypes.c_int64()
    buf = ctypes.create_string_buffer(4)
    rc = lib.pas_encode_host_priority_list(2, order.ctypes.data_as(ctypes.c_void_p), t.names, buf,
                                           4, ctypes.byref(n))
    assert rc == _lib.PAS_ECAPACITY and n.value == len(go_priority_list([b"a", b"b"]))
    bad = np.array([-1], np.int32)
    assert lib.pas_encode_host_priority_list(1, bad.ctypes.data_as(ctypes.c_void_p), t.names, buf,
                                             4, ctypes.byref(n)) == _lib.PAS_EINVAL
