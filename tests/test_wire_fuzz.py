"""Seeded mutation fuzz of the host request decoders in libpas.so (pas_decode_args,
pas_decode_request_names, pas_decode_pod_policy, pas_decode_pod_requests): the bodies an
extender receives come off the network, so every mutation of a valid body (bit flips, cut,
repeated and spliced ranges, inserted JSON punctuation, truncation) must either decode or fail
with PAS_EDECODE, never crash or read past the body.  Under scripts/sanitize.sh the same run
goes through the ASan + UBSan build.  Where Python's json module accepts a mutated nodes body
with plain ASCII keys and unique, string-valued names, the decoded node ids must be those names'
table ids.  Host code: runs without a GPU."""
import json
import os

import numpy as np
import pytest

from pas_amd import _lib, wire

NAMES = ["node-0", "node-1", "node-2", "gpu-a", "gpu-b", "é-node", "n\\\"q"]
KINDS = ["gpu.intel.com/i915", "gpu.intel.com/memory.max", "gpu.intel.com/millicores"]
PUNCT = [b"{", b"}", b"[", b"]", b",", b":", b'"', b"\\", b"null", b"-", b"1e9", b"\\u00e9",
         b"\\ud800", b"\xff", b"\x00", b" "]


def bodies():
    items = ",".join('{"metadata":{"name":%s,"labels":{"a":"b"}},"status":{"x":[1,2.5,null]}}'
                     % json.dumps(n) for n in NAMES + ["zz"])
    pod = ('{"metadata":{"namespace":"ns","labels":{"telemetry-policy":"p"}},'
           '"spec":{"containers":[{"name":"c0","resources":{"requests":{'
           '"gpu.intel.com/i915":"1","gpu.intel.com/memory.max":"5G"}}},'
           '{"name":"c1","resources":{"requests":{"gpu.intel.com/millicores":500,'
           '"cpu":"2"},"limits":{"gpu.intel.com/i915":"1"}}}]}}')
    return [
        ('{"Pod":%s,"Nodes":{"metadata":{},"items":[%s]}}' % (pod, items)).encode(),
        ('{"Pod":%s,"NodeNames":%s}' % (pod, json.dumps(NAMES + ["zz"]))).encode(),
        pod.encode(),
    ]


def mutate(rng, b):
    b = bytearray(b)
    for _ in range(int(rng.integers(1, 4))):
        n = len(b)
        op = int(rng.integers(0, 6))
        i = int(rng.integers(0, n + 1))
        j = min(n, i + int(rng.integers(0, 24)))
        if op == 0 and n:  # bit flip
            k = int(rng.integers(0, n))
            b[k] ^= 1 << int(rng.integers(0, 8))
        elif op == 1:  # cut a range
            del b[i:j]
        elif op == 2:  # repeat a range
            b[i:i] = b[i:j]
        elif op == 3:  # splice a range elsewhere
            k = int(rng.integers(0, n + 1))
            b[k:k] = b[i:j]
        elif op == 4:  # inserted punctuation
            b[i:i] = PUNCT[int(rng.integers(0, len(PUNCT)))]
        else:  # truncation
            del b[i:]
    return bytes(b)


def python_names(body):
    """The request's node names when Python's json accepts the body unambiguously (ASCII keys,
    no repeated keys, names all strings, no NaN / Infinity, no lone surrogates), else None."""
    def no_dupes(pairs):
        keys = [k for k, _ in pairs]
        if len(set(k.lower() for k in keys)) != len(keys) or not all(k.isascii() for k in keys):
            raise ValueError
        return dict(pairs)
    def no_constant(_):  # NaN / Infinity: Python extensions Go rejects
        raise ValueError
    try:
        d = json.loads(body, object_pairs_hook=no_dupes, parse_constant=no_constant)
    except (ValueError, RecursionError):
        return None
    if not isinstance(d, dict) or "Nodes" not in d or not isinstance(d["Nodes"], dict):
        return None
    items = d["Nodes"].get("items")
    if not isinstance(items, list):
        return None
    names = []
    for it in items:
        md = it.get("metadata") if isinstance(it, dict) else None
        if not isinstance(md, dict) or not isinstance(md.get("name"), str):
            return None
        try:  # lone surrogate escapes: Go substitutes U+FFFD, Python keeps them
            md["name"].encode("utf-8")
        except UnicodeEncodeError:
            return None
        names.append(md["name"])
    return names


@pytest.mark.parametrize("seed", range(8))
def test_mutated_bodies_decode_or_fail_cleanly(seed):
    rng = np.random.default_rng(seed)
    table = wire.NameTable(NAMES)
    checked = 0
    for base in bodies():
        for _ in range(int(os.environ.get("PAS_WIRE_FUZZ_N", "1000"))):
            body = mutate(rng, base)
            for which in (_lib.PAS_ARGS_NODES, _lib.PAS_ARGS_NODE_NAMES):
                try:
                    info, idx, _, spans = wire.decode_args(table, body, which,
                                                           which == _lib.PAS_ARGS_NODES)
                except _lib.PasError as e:
                    assert e.code == _lib.PAS_EDECODE, (body, e)
                    continue
                assert all(-1 <= int(x) < len(NAMES) for x in idx), body
                for o, n in (spans if spans is not None else []):
                    assert 0 <= o and o + n <= len(body), body
                if which == _lib.PAS_ARGS_NODES:
                    want = python_names(body)
                    if want is not None:
                        ids = [table.lookup(n) for n in want]
                        assert list(idx) == ids, body
                        checked += 1
                try:
                    wire.decode_request_names(body, which)
                except _lib.PasError as e:
                    assert e.code == _lib.PAS_EDECODE, (body, e)
            for fn in (lambda b: wire.decode_pod_policy(b, "telemetry-policy"),
                       lambda b: wire.decode_pod_requests(b, KINDS)):
                try:
                    fn(body)
                except _lib.PasError as e:
                    assert e.code == _lib.PAS_EDECODE, (body, e)
    table.close()
    assert checked > 20  # some mutations stay valid JSON and are cross-checked
