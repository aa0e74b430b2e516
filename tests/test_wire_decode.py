"""Request decoding in libpas.so (pas_decode_args / pas_decode_request_names /
pas_decode_pod_policy / pas_decode_pod_requests) against the encoding/json
(Go 1.16) behaviour the reference's handlers get from json.NewDecoder(r.Body).Decode(&args)
(telemetryscheduler.go:63-78, gpuscheduler/scheduler.go:486-505) and
resource.Quantity.UnmarshalJSON (apimachinery v0.22.2).  The expected values restate the
documented encoding/json rules (there is no Go toolchain here to run them): parity unpinned
beyond those rules.  Host code: runs without a GPU."""
import json

import numpy as np
import pytest

from pas_amd import _lib, wire

NAMES = ["node-0", "node-1", "node-2", "gpu-a", "gpu-b"]
T = None


def table():
    global T
    if T is None:
        T = wire.NameTable(NAMES)
    return T


def nodes_body(names, key="Nodes", pod=None, extra=""):
    items = ",".join('{"metadata":{"name":%s},"status":{"x":[1,2]}}' % json.dumps(n)
                     for n in names)
    pod = pod if pod is not None else '{"metadata":{"labels":{"telemetry-policy":"p"}}}'
    return ('{"Pod":%s,"%s":{"metadata":{},"items":[%s]}%s}' % (pod, key, items, extra)).encode()


def decode(body, which=_lib.PAS_ARGS_NODES, spans=False):
    return wire.decode_args(table(), body, which, spans)


def edecode(body, which=_lib.PAS_ARGS_NODES):
    with pytest.raises(_lib.PasError) as e:
        decode(body, which)
    assert e.value.code == _lib.PAS_EDECODE


def test_name_table():
    t = wire.NameTable(["a", "b", "a", ""])
    assert [t.lookup(x) for x in ["a", "b", "", "c"]] == [0, 1, 3, -1]  # repeated: first id


def test_nodes_items_ids_cand_spans():
    body = nodes_body(["node-2", "zz", "node-0", "node-2"])
    info, idx, cand, spans = decode(body, spans=True)
    assert info.has_nodes == 1 and info.has_node_names == 0
    assert list(idx) == [2, -1, 0, 2] and info.n_unknown == 1
    assert int(cand[0]) == 0b101
    items = json.loads(body)["Nodes"]["items"]
    for (o, n), item in zip(spans, items):
        assert json.loads(body[o:o + n]) == item
    pod = body[info.pod_off:info.pod_off + info.pod_len]
    assert json.loads(pod) == json.loads(body)["Pod"]
    assert wire.decode_request_names(body, _lib.PAS_ARGS_NODES) == ["node-2", "zz", "node-0",
                                                                    "node-2"]


def test_node_names_list():
    body = b'{"Pod":{},"NodeNames":["gpu-b","gpu-a","nope"]}'
    info, idx, cand, _ = decode(body, _lib.PAS_ARGS_NODE_NAMES)
    assert info.has_node_names == 1 and info.has_nodes == 0
    assert list(idx) == [4, 3, -1]
    info, idx, _, _ = decode(body, _lib.PAS_ARGS_NODES)  # the other list: absent
    assert info.n_req == 0 and info.has_nodes == 0


@pytest.mark.parametrize("key", ["nodes", "NODES", "nOdEs", "Node\\u017f", "NODE\\u017f"])
def test_case_insensitive_keys(key):
    # Args has no json tags: "Nodes" matches by equalFoldRight (an 's' in the name also
    # accepts U+017F LATIN SMALL LETTER LONG S)
    info, idx, _, _ = decode(nodes_body(["node-1"], key=key))
    assert info.has_nodes == 1 and list(idx) == [1]


@pytest.mark.parametrize("key", ["Node", "Nodess", "N0des", "Nodes\\u0000"])
def test_non_matching_keys_are_skipped(key):
    info, _, _, _ = decode(nodes_body(["node-1"], key=key))
    assert info.has_nodes == 0


def test_fold_in_nested_fields():
    body = (b'{"nodes":{"ITEM\\u017f":[{"METADATA":{"NAME":"node-1"}},'
            b'{"metadata":{"Name":"node-2"}}]}}')
    assert list(decode(body)[1]) == [1, 2]
    # K in "kind" folds with U+212A KELVIN SIGN; its value must be a string
    edecode(b'{"Nodes":{"\\u212aind":5,"items":[]}}')
    assert decode(b'{"Nodes":{"\\u212aind":"NodeList","items":[]}}')[0].has_nodes == 1


def test_nulls():
    assert decode(b'{"Nodes":null}')[0].has_nodes == 0
    info = decode(b'{"Nodes":{"items":null}}')[0]
    assert info.has_nodes == 1 and info.n_req == 0
    # null name: the string keeps its zero value
    info, idx, _, _ = decode(b'{"Nodes":{"items":[{"metadata":{"name":null}},null,{}]}}')
    assert info.n_req == 3 and info.n_unknown == 3
    assert wire.decode_request_names(b'{"Nodes":{"items":[{"metadata":null}]}}',
                                     _lib.PAS_ARGS_NODES) == [""]
    assert decode(b'null')[0].has_nodes == 0  # the zero Args
    info = decode(b'{"NodeNames":[null,"node-0"]}', _lib.PAS_ARGS_NODE_NAMES)[0]
    assert info.n_req == 2 and info.n_unknown == 1


@pytest.mark.parametrize("body", [
    b'', b'   ', b'{', b'{"Nodes":{"items":[}', b'{"Nodes":}', b'{"Nodes":{"items":[{"a":1,}]}}',
    b'{"Nodes":{"items":[]}', b'[1,2', b'{"a":01}', b'{"a":"\x01"}', b'{"a":"\\x"}',
    b'{"a":tru}', b'{"a":-}', b'{"a":1.}', b'{"a":1e}', b'\xef\xbb\xbf{}',
])
def test_syntax_errors(body):
    edecode(body)


@pytest.mark.parametrize("body", [
    b'[]', b'"x"', b'5', b'true',
    b'{"Nodes":[]}', b'{"Nodes":"x"}', b'{"Nodes":{"items":{}}}', b'{"Nodes":{"items":[5]}}',
    b'{"Nodes":{"items":[{"metadata":[]}]}}', b'{"Nodes":{"items":[{"metadata":{"name":5}}]}}',
    b'{"Nodes":{"metadata":5,"items":[]}}', b'{"NodeNames":{}}', b'{"NodeNames":[1]}',
    b'{"Pod":[]}', b'{"Pod":5}',
])
def test_type_errors(body):
    # an UnmarshalTypeError fails Decode (after the value), whichever list is wanted
    edecode(body)
    edecode(body, _lib.PAS_ARGS_NODE_NAMES)


def test_trailing_bytes_ignored():
    # Decoder.Decode reads one value
    assert list(decode(nodes_body(["node-0"]) + b' garbage {')[1]) == [0]


def test_unknown_keys_and_values_skipped():
    body = (b'{"x":{"y":[1,2.5e-3,-0,true,false,null,"s\\u00e9\\n"]},"Nodes":{"items":'
            b'[{"spec":{"taints":[{"k":"v"}]},"metadata":{"labels":{"a":"b"},"name":"node-2",'
            b'"uid":"u"}}]},"z":-12.5E+4}')
    assert list(decode(body)[1]) == [2]


def test_string_escapes_and_invalid_utf8():
    t = wire.NameTable(["node-1", "a�b", "\U0001F600", "x�"])
    def ids(names_json):
        info, idx, _, _ = wire.decode_args(t, b'{"NodeNames":' + names_json + b'}',
                                           _lib.PAS_ARGS_NODE_NAMES)
        return list(idx)
    assert ids(b'["no\\u0064e-\\u0031"]') == [0]
    assert ids(b'["a\xffb"]') == [1]                 # invalid byte -> U+FFFD
    assert ids(b'["a\\ud800b"]') == [1]              # unpaired surrogate -> U+FFFD
    assert ids(b'["\\ud83d\\ude00"]') == [2]         # surrogate pair
    assert ids(b'["\xf0\x9f\x98\x80"]') == [2]       # raw UTF-8
    assert ids(b'["x\xed\xa0\x80"]') == [-1]         # encoded surrogate: 3 x U+FFFD
    assert ids(b'["x\xc0"]') == [3]


def test_depth_limit():
    ok = b'{"x":' + b'[' * 9999 + b']' * 9999 + b',"NodeNames":["node-1"]}'
    assert list(decode(ok, _lib.PAS_ARGS_NODE_NAMES)[1]) == [1]
    edecode(b'{"x":' + b'[' * 10000 + b']' * 10000 + b'}')


def test_repeated_keys():
    # a repeated slice decodes element-wise into the old one (encoding/json array()): a null
    # element keeps the earlier value, the length is the new one
    body = b'{"NodeNames":["node-0","node-1","node-2"],"nodenames":[null,"gpu-a"]}'
    assert list(decode(body, _lib.PAS_ARGS_NODE_NAMES)[1]) == [0, 3]
    body = b'{"NodeNames":["node-0"],"NodeNames":null,"NodeNames":[null]}'
    assert list(decode(body, _lib.PAS_ARGS_NODE_NAMES)[1]) == [-1]
    # Nodes is a pointer: a second object decodes into the same NodeList
    body = (b'{"Nodes":{"items":[{"metadata":{"name":"node-1"}},{"metadata":{"name":"node-2"}}]},'
            b'"nodes":{"kind":"NodeList"}}')
    assert list(decode(body)[1]) == [1, 2]
    body = (b'{"Nodes":{"items":[{"metadata":{"name":"node-1"}},{"metadata":{"name":"node-2"}}]},'
            b'"Nodes":{"items":[{"status":{}}]}}')
    assert list(decode(body)[1]) == [1]


def test_large_request_grows_buffers():
    names = [f"n{i}" for i in range(5000)]
    t = wire.NameTable(names)
    body = json.dumps({"Pod": {}, "NodeNames": names[::-1]}).encode()
    info, idx, cand, _ = wire.decode_args(t, body, _lib.PAS_ARGS_NODE_NAMES)
    assert list(idx) == list(range(4999, -1, -1))
    assert np.unpackbits(cand.view(np.uint8)).sum() == 5000
    assert wire.decode_request_names(body, _lib.PAS_ARGS_NODE_NAMES) == names[::-1]


# ---------------------------------------------------------------------------- pod fields

def test_pod_policy():
    pod = b'{"metadata":{"namespace":"default","labels":{"app":"x","telemetry-policy":"p1"}}}'
    assert wire.decode_pod_policy(pod, "telemetry-policy") == ("default", "p1")
    assert wire.decode_pod_policy(pod, "Telemetry-Policy") == ("default", None)  # map: exact
    assert wire.decode_pod_policy(b'{"METADATA":{"NameSpace":"ns"}}', "l") == ("ns", None)
    # null value in a map[string]string: the key is present with ""
    assert wire.decode_pod_policy(b'{"metadata":{"labels":{"l":null}}}', "l") == ("", "")
    assert wire.decode_pod_policy(b'{"metadata":{"labels":{"l":"a"},"labels":null}}',
                                  "l") == ("", None)
    # a repeated labels object decodes into the same map
    assert wire.decode_pod_policy(b'{"metadata":{"labels":{"l":"a"},"labels":{"m":"b"}}}',
                                  "l") == ("", "a")
    assert wire.decode_pod_policy(b'', "l") == ("", None)
    assert wire.decode_pod_policy(b'null', "l") == ("", None)
    for bad in (b'{"metadata":{"labels":{"l":5}}}', b'{"metadata":{"namespace":1}}',
                b'{"metadata":[]}', b'[]'):
        with pytest.raises(_lib.PasError) as e:
            wire.decode_pod_policy(bad, "l")
        assert e.value.code == _lib.PAS_EDECODE


KINDS = ["gpu.intel.com/i915", "gpu.intel.com/memory.max", "gpu.intel.com/millicores"]


def pod_with(*containers):
    return json.dumps({"spec": {"containers": [
        {"name": f"c{i}", "resources": {"requests": r}} for i, r in enumerate(containers)]}})


def test_pod_requests():
    pod = pod_with({"gpu.intel.com/i915": "1", "gpu.intel.com/memory.max": "5G", "cpu": "2"},
                   {},
                   {"gpu.intel.com/millicores": 500, "gpu.intel.com/i915": "2"}).encode()
    req, mask, nc, unknown = wire.decode_pod_requests(pod, KINDS)
    assert nc[0] == 3 and unknown == 0
    assert list(mask[0]) == [0b011, 0, 0b101]
    assert req[0, 0, 0] == 1 and req[0, 0, 1] == 5_000_000_000
    assert req[0, 2, 2] == 500 and req[0, 2, 0] == 2


@pytest.mark.parametrize("q,want", [
    ('"1000m"', 0),         # int64Amount with negative scale: AsInt64 -> (0, false)
    ('"1.5Ki"', 0),         # inf.Dec-backed: (0, false)
    ('"9223372036854775807"', 0),
    ('"16Gi"', 16 * 2**30), ('" 7 "', 7), ('" 7"', 7), ('null', 0), ('3', 3), ('1e3', 1000),
])
def test_pod_request_quantities(q, want):
    pod = ('{"spec":{"containers":[{"resources":{"requests":{"gpu.intel.com/i915":%s}}}]}}'
           % q).encode()
    req, mask, nc, _ = wire.decode_pod_requests(pod, KINDS)
    assert int(req[0, 0, 0]) == want and mask[0, 0] == 1  # the key exists either way


@pytest.mark.parametrize("q", ['"abc"', '"5\\u0047"', 'true', '{}', '[]', '"1 G"'])
def test_pod_request_quantity_errors(q):
    # Quantity.UnmarshalJSON -> ParseQuantity error -> the whole decode fails, also for a
    # resource outside gpu.intel.com and also on the TAS path (which reads no requests)
    for name in ("gpu.intel.com/i915", "cpu"):
        pod = ('{"spec":{"containers":[{"resources":{"requests":{"%s":%s}}}]}}'
               % (name, q)).encode()
        for kinds in (KINDS, []):
            with pytest.raises(_lib.PasError) as e:
                wire.decode_pod_requests(pod, kinds)
            assert e.value.code == _lib.PAS_EDECODE


def test_pod_requests_unknown_and_repeated():
    pod = (b'{"spec":{"containers":[{"resources":{"requests":{"gpu.intel.com/i915":"1",'
           b'"gpu.intel.com/tiles":"2","gpu.intel.com/i915":"3"}}}]}}')
    req, mask, nc, unknown = wire.decode_pod_requests(pod, KINDS)
    assert unknown == 1 and req[0, 0, 0] == 3
    assert mask[0, 0] == 1 | _lib.PAS_REQ_UNKNOWN_KIND  # flagged: no node has that key
    # containers is a slice: a repeated key decodes element-wise into the old containers
    pod = (b'{"spec":{"containers":[{"resources":{"requests":{"gpu.intel.com/i915":"1"}}},{}],'
           b'"containers":[null]}}')
    req, mask, nc, _ = wire.decode_pod_requests(pod, KINDS)
    assert nc[0] == 1 and req[0, 0, 0] == 1 and mask[0, 0] == 1
    req, mask, nc, _ = wire.decode_pod_requests(b'{"spec":{"containers":null}}', KINDS)
    assert nc[0] == 0
    many = pod_with(*[{"gpu.intel.com/i915": "1"}] * 40).encode()  # grows past 16 containers
    req, mask, nc, _ = wire.decode_pod_requests(many, KINDS)
    assert nc[0] == 40 and (req[0, :, 0] == 1).all()


def test_pod_requests_unknown_kind_flag_per_container():
    # only the container that names a kind outside the list is flagged; a non-gpu.intel.com
    # resource is not a GAS key at all (resourcePrefix, utils.go:9-12)
    pod = pod_with({"gpu.intel.com/i915": "1"},
                   {"gpu.intel.com/tiles": "1", "cpu": "1"},
                   {"gpu.intel.com/tiles": "0", "gpu.intel.com/i915": "0"},
                   {"memory": "1Gi"}).encode()
    req, mask, nc, unknown = wire.decode_pod_requests(pod, KINDS)
    assert nc[0] == 4 and unknown == 2
    u = _lib.PAS_REQ_UNKNOWN_KIND
    assert list(mask[0]) == [1, u, 1 | u, 0]


@pytest.mark.parametrize("meta", [
    b'{"labels":{"app":5}}', b'{"labels":{"telemetry-policy":"p","x":true}}',
    b'{"annotations":{"a":{}}}', b'{"labels":[]}', b'{"annotations":7}'])
def test_pod_metadata_maps_type_checked(meta):
    # ObjectMeta labels / annotations are map[string]string: a non-string value anywhere
    # fails json.Decode (TAS: empty body; GAS: 404), not only under the policy label
    pod = b'{"metadata":' + meta + b',"spec":{"containers":[]}}'
    with pytest.raises(_lib.PasError) as e:
        wire.decode_pod_policy(pod, "telemetry-policy")
    assert e.value.code == _lib.PAS_EDECODE
    with pytest.raises(_lib.PasError) as e:
        wire.decode_pod_requests(pod, KINDS)
    assert e.value.code == _lib.PAS_EDECODE


def test_pod_metadata_maps_null_values_ok():
    pod = (b'{"metadata":{"namespace":"ns","labels":{"a":null,"telemetry-policy":"p"},'
           b'"annotations":null},"spec":{"containers":[]}}')
    assert wire.decode_pod_policy(pod, "telemetry-policy") == ("ns", "p")
    assert wire.decode_pod_requests(pod, KINDS)[2][0] == 0


@pytest.mark.parametrize("limits,ok", [
    (b'{"cpu":"2","gpu.intel.com/i915":"1"}', True), (b'null', True),
    (b'{"cpu":"abc"}', False), (b'{"memory":true}', False), (b'[]', False)])
def test_container_limits_validated(limits, ok):
    # ResourceRequirements.limits is a ResourceList too: every Quantity is parsed on decode
    pod = (b'{"spec":{"containers":[{"resources":{"limits":' + limits +
           b',"requests":{"gpu.intel.com/i915":"1"}}}]}}')
    if ok:
        req, mask, nc, _ = wire.decode_pod_requests(pod, KINDS)
        assert nc[0] == 1 and mask[0, 0] == 1 and req[0, 0, 0] == 1
    else:
        with pytest.raises(_lib.PasError) as e:
            wire.decode_pod_requests(pod, KINDS)
        assert e.value.code == _lib.PAS_EDECODE
