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
