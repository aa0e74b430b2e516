"""Extender response bodies from index outputs (include/pas.h "Wire encoders").

Thin wrappers over the host encoders in libpas.so: byte-exact json.NewEncoder(w).Encode
output of the reference's handlers (telemetryscheduler.go:152-158, 238-244;
gpuscheduler/scheduler.go:508-513).
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_char_p, c_int64
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import PasError


class NodeTable:
    """Names (and optionally the JSON text of each v1.Node) indexed by snapshot node id,
    converted once per snapshot."""

    def __init__(self, names: Sequence[str], node_json: Optional[Sequence[bytes]] = None):
        self._names = [n.encode() for n in names]
        self.names = (c_char_p * max(len(self._names), 1))(*self._names)
        self.node_json = None
        self.node_json_len = None
        if node_json is not None:
            self._json = [bytes(j) for j in node_json]
            self.node_json = (c_char_p * max(len(self._json), 1))(*self._json)
            self.node_json_len = np.array([len(j) for j in self._json], np.int64)

    def __len__(self):
        return len(self._names)


def _call(fn, *args) -> bytes:
    n = c_int64()
    cap = 4096
    while True:
        buf = ctypes.create_string_buffer(cap)
        rc = fn(*args, buf, cap, byref(n))
        if rc == _lib.PAS_OK:
            return buf.raw[:n.value]
        if rc != _lib.PAS_ECAPACITY:
            raise PasError(rc, fn.__name__)
        cap = n.value


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a.size else None


def host_priority_list(order, table: NodeTable) -> bytes:
    """[{"Host":..,"Score":10-i},...]\\n of one pod's ordered list (order_out[p, :len[p]])."""
    order = _i32(order)
    return _call(_lib.load().pas_encode_host_priority_list, len(order), _ptr(order), table.names)


def tas_filter_result(req_nodes, pass_row, table: NodeTable) -> bytes:
    """TAS FilterResult of one pod: request node ids in order, its pass_out row."""
    req_nodes = _i32(req_nodes)
    pass_row = np.ascontiguousarray(pass_row, dtype=np.uint64)
    assert table.node_json is not None, "the TAS FilterResult carries the node objects"
    return _call(_lib.load().pas_encode_tas_filter_result, len(req_nodes), _ptr(req_nodes),
                 _ptr(pass_row), table.names, table.node_json,
                 table.node_json_len.ctypes.data_as(ctypes.c_void_p))


def gas_filter_result(req_nodes, fit_row, table: NodeTable) -> bytes:
    """GAS FilterResult of one pod: request node ids in order, its fit bitmap row."""
    req_nodes = _i32(req_nodes)
    fit_row = np.ascontiguousarray(fit_row, dtype=np.uint64)
    return _call(_lib.load().pas_encode_gas_filter_result, len(req_nodes), _ptr(req_nodes),
                 _ptr(fit_row), table.names)


def binding_result(error: str = "") -> bytes:
    """BindingResult {"Error": ...} of a GAS bind."""
    return _call(_lib.load().pas_encode_binding_result, error.encode())


# ---------------------------------------------------------------------------- request decoding

class NameTable:
    """pas_name_table: snapshot node names -> node ids, built once per snapshot."""

    def __init__(self, names: Sequence[str]):
        self._l = _lib.load()
        self.size = len(names)
        enc = [n.encode() for n in names]
        arr = (c_char_p * max(len(enc), 1))(*enc)
        h = ctypes.c_void_p()
        rc = self._l.pas_name_table_create(len(enc), arr, byref(h))
        if rc != _lib.PAS_OK:
            raise PasError(rc, "pas_name_table_create")
        self._h = h

    def lookup(self, name: str) -> int:
        b = name.encode()
        return self._l.pas_name_table_lookup(self._h, b, len(b))

    def close(self):
        if getattr(self, "_h", None):
            self._l.pas_name_table_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - best effort
        self.close()


def decode_args(table: NameTable, body: bytes, which: int, spans: bool = False):
    """pas_decode_args: (info, req_node int32 [n_req], cand uint64 [W64(table)], item spans
    int64 [n_req][2] or None).  Raises PasError(PAS_EDECODE) where the reference's decode
    fails."""
    l = _lib.load()
    info = _lib.PasArgsInfo()
    cap = max(table.size, 1024)  # a request rarely lists more nodes than the snapshot holds
    w = max((table.size + 63) // 64, 1)
    while True:
        req = np.zeros(max(cap, 1), np.int32)
        cand = np.zeros(w, np.uint64)
        sp = np.zeros((max(cap, 1), 2), np.int64) if spans else None
        rc = l.pas_decode_args(table._h, body, len(body), which, _ptr(req), cap,
                               _ptr(sp) if spans else None, _ptr(cand), byref(info))
        if rc == _lib.PAS_OK:
            n = info.n_req
            return info, req[:n], cand, (sp[:n] if spans else None)
        if rc != _lib.PAS_ECAPACITY:
            raise PasError(rc, "pas_decode_args")
        cap = info.n_req


def decode_request_names(body: bytes, which: int):
    """pas_decode_request_names: the request's node names (unescaped, request order)."""
    l = _lib.load()
    total, n = c_int64(), ctypes.c_int32()
    cap, ocap = 4096, 1024
    while True:
        buf = ctypes.create_string_buffer(max(cap, 1))
        offs = np.zeros(max(ocap, 1), np.int64)
        rc = l.pas_decode_request_names(body, len(body), which, buf, cap, _ptr(offs), ocap,
                                        byref(total), byref(n))
        if rc == _lib.PAS_OK:
            raw = buf.raw
            return [raw[offs[i]:offs[i + 1]].decode("utf-8", "surrogateescape")
                    for i in range(n.value)]
        if rc != _lib.PAS_ECAPACITY:
            raise PasError(rc, "pas_decode_request_names")
        cap, ocap = total.value, n.value + 1


def decode_pod_policy(pod: bytes, label: str):
    """pas_decode_pod_policy: (namespace, labels[label] or None)."""
    l = _lib.load()
    ns_len, lab_len = c_int64(), c_int64()
    cap = 256
    while True:
        ns = ctypes.create_string_buffer(cap)
        lab = ctypes.create_string_buffer(cap)
        rc = l.pas_decode_pod_policy(pod, len(pod), label.encode(), ns, cap, byref(ns_len), lab,
                                     cap, byref(lab_len))
        if rc == _lib.PAS_OK:
            value = None if lab_len.value < 0 else lab.raw[:lab_len.value].decode(
                "utf-8", "surrogateescape")
            return ns.raw[:ns_len.value].decode("utf-8", "surrogateescape"), value
        if rc != _lib.PAS_ECAPACITY:
            raise PasError(rc, "pas_decode_pod_policy")
        cap = max(ns_len.value, lab_len.value, 1)


def decode_pod_requests(pod: bytes, kinds: Sequence[str], max_containers: int = 16):
    """pas_decode_pod_requests: (req [1][C][Q] int64, req_mask [1][C] uint32, n_containers [1]
    int32, n_unknown) with C = max(1, containers)."""
    l = _lib.load()
    enc = [k.encode() for k in kinds]
    karr = (c_char_p * max(len(enc), 1))(*enc)
    nc, nu = ctypes.c_int32(), ctypes.c_int32()
    cap = max_containers
    while True:
        c = max(cap, 1)
        req = np.zeros((1, c, len(kinds)), np.int64)
        mask = np.zeros((1, c), np.uint32)
        rc = l.pas_decode_pod_requests(pod, len(pod), len(enc), karr, cap, _ptr(req), _ptr(mask),
                                       byref(nc), byref(nu))
        if rc == _lib.PAS_OK:
            c = max(nc.value, 1)
            return req[:, :c], mask[:, :c], np.array([nc.value], np.int32), nu.value
        if rc != _lib.PAS_ECAPACITY:
            raise PasError(rc, "pas_decode_pod_requests")
        cap = nc.value
