"""ctypes binding of lib/libpas.so (the C-ABI declared in include/pas.h).

The library is the product: HIP kernels for gfx950 behind a plain C ABI.  This module
only loads it and declares the signatures.  There is no fallback: if the shared
object is missing the import fails loudly.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_int64, c_uint32, c_uint64, c_void_p

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_PKG_DIR), "lib", "libpas.so")
# the same library built with the GAS fault-injection knob (test tooling only)
FAULT_LIB_PATH = os.path.join(os.path.dirname(_PKG_DIR), "lib", "libpas_fault.so")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_PKG_DIR)), "include", "pas.h")

PAS_OK = 0
PAS_EINVAL = -1
PAS_ESTALE = -2
PAS_ENOTEXACT = -3
PAS_EDEVICE = -4
PAS_ENOMEM = -5
PAS_ENOSNAP = -6
PAS_ECAPACITY = -7
PAS_EDECODE = -8

STATUS_NAMES = {
    PAS_OK: "PAS_OK",
    PAS_EINVAL: "PAS_EINVAL",
    PAS_ESTALE: "PAS_ESTALE",
    PAS_ENOTEXACT: "PAS_ENOTEXACT",
    PAS_EDEVICE: "PAS_EDEVICE",
    PAS_ENOMEM: "PAS_ENOMEM",
    PAS_ENOSNAP: "PAS_ENOSNAP",
    PAS_ECAPACITY: "PAS_ECAPACITY",
    PAS_EDECODE: "PAS_EDECODE",
}

PAS_OP_LESS_THAN = 0
PAS_OP_GREATER_THAN = 1
PAS_OP_EQUALS = 2

PAS_TAS_FILTER = 1
PAS_TAS_PRIORITIZE = 2

PAS_GAS_MAX_CARDS = 64
PAS_GAS_MAX_RES = 4
PAS_GAS_MAX_SELECTIONS = 64
PAS_GAS_PACKED = 8
PAS_REQ_UNKNOWN_KIND = 0x80000000
PAS_GAS_SEL_EXTENDED = 15
PAS_GAS_SEL_LIMIT = 14

PAS_GAS_OK = 0
PAS_GAS_WONT_FIT = 1
PAS_GAS_ERR_INPUT = 2
PAS_GAS_ERR_OVERFLOW = 3

PAS_K_TAS_EVAL = 1
PAS_K_TAS_VIOLATIONS = 2
PAS_K_GAS_PREP = 3
PAS_K_GAS_FIT = 4
PAS_K_TAS_PREP = 5
PAS_K_TAS_LABELS = 6
PAS_K_TAS_SPAN = 7
PAS_K_PRIO_REQUEST = 8
PAS_K_TAS_GAS_TOPK = 9
KERNEL_NAMES = {
    PAS_K_TAS_LABELS: "label_plan_kernel",
    PAS_K_TAS_EVAL: "tas_eval_kernel",
    PAS_K_TAS_VIOLATIONS: "tas_violations_kernel",
    PAS_K_GAS_PREP: "gas_prep_kernel",
    PAS_K_GAS_FIT: "gas_fit_kernel",
    PAS_K_TAS_PREP: "tas_prep_kernel",
    PAS_K_TAS_SPAN: "tas_eval_span",
    PAS_K_PRIO_REQUEST: "prio_request_span",
    PAS_K_TAS_GAS_TOPK: "tas_gas_topk_kernel",
}


class PasError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"{STATUS_NAMES.get(code, code)}: {message}")
        self.code = code


PAS_ARGS_NODES = 0
PAS_ARGS_NODE_NAMES = 1


class PasArgsInfo(ctypes.Structure):
    _fields_ = [("has_nodes", c_int32), ("has_node_names", c_int32), ("n_req", c_int32),
                ("n_unknown", c_int32), ("pod_off", c_int64), ("pod_len", c_int64)]


class PasConfig(ctypes.Structure):
    _fields_ = [("device", c_int32), ("reserved", c_int32)]


# pas_gas_selection (include/pas.h) as a numpy record: the side buffer of pas_gas_fit_ex.
GAS_SELECTION_DTYPE = np.dtype([("pod", np.int32), ("node", np.int32), ("n_sel", np.int32),
                                ("reserved", np.int32), ("card", np.uint8, (PAS_GAS_MAX_SELECTIONS,))])
assert GAS_SELECTION_DTYPE.itemsize == 16 + PAS_GAS_MAX_SELECTIONS


# Every exported symbol with (restype, argtypes); tests check this list against pas.h.
_P = c_void_p
SIGNATURES = {
    "pas_abi_version": (c_int, []),
    "pas_create": (c_int, [POINTER(PasConfig), POINTER(c_void_p)]),
    "pas_destroy": (None, [_P]),
    "pas_last_error": (c_char_p, [_P]),
    "pas_set_stream": (c_int, [_P, _P]),
    "pas_synchronize": (c_int, [_P]),
    "pas_parse_operator": (c_int, [c_char_p]),
    "pas_quantity_to_milli": (c_int, [c_char_p, POINTER(c_int64)]),
    "pas_quantity_as_int64": (c_int, [c_char_p, POINTER(c_int64)]),
    "pas_quantity_to_scaled": (c_int, [c_char_p, c_int32, POINTER(c_int64)]),
    "pas_quantity_decimals": (c_int, [c_char_p, POINTER(c_int32)]),
    "pas_tas_snapshot_set": (c_int, [_P, c_uint64, c_int32, c_int32, _P, _P]),
    "pas_tas_snapshot_set_device": (c_int, [_P, c_uint64, c_int32, c_int32, _P, _P, _P]),
    "pas_tas_snapshot_update": (c_int, [_P, c_uint64, c_uint64, c_int32, _P, _P, _P]),
    "pas_tas_snapshot_update_device": (
        c_int, [_P, c_uint64, c_uint64, c_int32, _P, _P, _P, _P]),
    "pas_tas_snapshot_info":(c_int, [_P, POINTER(c_uint64), POINTER(c_int32), POINTER(c_int32)]),
    "pas_tas_snapshot_set_scale": (c_int, [_P, c_uint64, c_int32, _P, _P]),
    "pas_tas_eval": (c_int, [_P, c_uint64, c_int32, _P, _P, _P, _P, c_uint32, _P, _P, _P]),
    "pas_tas_prioritize_request": (c_int, [_P, c_uint64, _P, c_int32, _P, _P, _P]),
    "pas_tas_prioritize_request_device": (c_int, [_P, c_uint64, _P, c_int32, _P, _P, _P, _P]),
    "pas_tas_eval_device": (
        c_int,
        [_P, c_uint64, c_int32, c_int32, _P, _P, _P, _P, c_uint32, _P, _P, _P, _P],
    ),
    "pas_tas_violations": (c_int, [_P, c_uint64, c_int32, _P, _P, _P]),
    "pas_tas_violations_device": (c_int, [_P, c_uint64, c_int32, c_int32, _P, _P, _P, _P]),
    "pas_tas_label_plan": (c_int, [_P, c_int32, c_int32, _P, _P, _P, _P, _P, _P]),
    "pas_tas_label_plan_device": (c_int, [_P, c_int32, c_int32, _P, _P, _P, _P, _P, _P, _P]),
    "pas_tas_deschedule_device": (c_int, [_P, c_uint64, c_int32, c_int32, _P, _P, _P, _P, _P, _P,
                                          _P, _P, _P]),
    "pas_label_patch_json": (
        c_int,
        [c_int32, POINTER(c_char_p), c_uint64, c_uint64, c_char_p, c_int64, POINTER(c_int64)],
    ),
    "pas_gas_snapshot_set": (c_int, [_P, c_uint64, c_int32, c_int32, c_int32, _P, _P, _P]),
    "pas_gas_snapshot_set_device": (
        c_int,
        [_P, c_uint64, c_int32, c_int32, c_int32, _P, _P, _P, _P],
    ),
    "pas_gas_fit": (c_int, [_P, c_uint64, c_int32, c_int32, c_int32, _P, _P, _P, _P]),
    "pas_gas_fit_device": (
        c_int,
        [_P, c_uint64, c_int32, c_int32, c_int32, _P, _P, _P, _P, _P],
    ),
    "pas_gas_fit_ex": (
        c_int,
        [_P, c_uint64, c_int32, c_int32, c_int32, _P, _P, _P, _P, _P, c_int64, POINTER(c_int64)],
    ),
    "pas_gas_fit_ex_device": (
        c_int,
        [_P, c_uint64, c_int32, c_int32, c_int32, _P, _P, _P, _P, _P, c_int64, _P, _P],
    ),
    "pas_gas_fit_ld_device": (
        c_int,
        [_P, c_uint64, c_int32, c_int32, c_int32, _P, _P, _P, _P, c_int64, _P, c_int64, _P, _P],
    ),
    "pas_gas_limit_count": (c_int, [_P, POINTER(c_int64)]),
    "pas_gas_fit_bitmap_device": (
        c_int,
        [_P, c_uint64, c_int32, c_int32, c_int32, _P, _P, _P, _P, _P],
    ),
    "pas_gas_bind": (
        c_int,
        [_P, c_uint64, c_uint64, c_int32, _P, _P, c_int32, c_int32, c_int32, _P, _P, _P, _P, _P],
    ),
    "pas_gas_bind_ex": (
        c_int,
        [_P, c_uint64, c_uint64, c_int32, _P, _P, c_int32, c_int32, c_int32, _P, _P, _P, _P, _P,
         _P, _P],
    ),
    "pas_gas_bind_counts": (
        c_int,
        [_P, c_uint64, c_uint64, c_int32, _P, _P, c_int32, c_int32, c_int32, _P, _P, _P, _P, _P,
         _P],
    ),
    "pas_gas_release": (
        c_int,
        [_P, c_uint64, c_uint64, c_int32, _P, _P, c_int32, c_int32, _P, _P, _P, _P, _P, _P],
    ),
    "pas_gas_release_counts": (
        c_int,
        [_P, c_uint64, c_uint64, c_int32, _P, _P, c_int32, c_int32, _P, _P, _P, _P, _P],
    ),
    "pas_gas_release_ex": (
        c_int,
        [_P, c_uint64, c_uint64, c_int32, _P, _P, c_int32, c_int32, _P, _P, _P, _P, _P, _P],
    ),
    "pas_gas_snapshot_get": (c_int, [_P, POINTER(c_uint64), _P]),
    "pas_tas_topk_device": (
        c_int,
        [_P, c_uint64, c_int32, c_int32, _P, _P, _P, _P, c_int32, c_int32, _P, _P, _P, _P],
    ),
    "pas_tas_gas_topk_device": (
        c_int,
        [_P, c_uint64, c_uint64, c_int32, c_int32, _P, _P, _P, _P, c_int32, c_int32, _P, _P, _P,
         c_int32, c_int32, _P, _P, _P, _P],
    ),
    "pas_topk_merge_device": (c_int, [_P, c_int32, c_int32, c_int32, _P, _P, _P, _P, _P]),
    "pas_list_merge_device": (c_int, [_P, c_int32, c_int32, c_int32, _P, _P, _P, c_int64, _P,
                                      _P]),
    "pas_encode_host_priority_list": (
        c_int, [c_int32, _P, POINTER(c_char_p), c_char_p, c_int64, POINTER(c_int64)]),
    "pas_encode_tas_filter_result": (
        c_int, [c_int32, _P, _P, POINTER(c_char_p), POINTER(c_char_p), _P, c_char_p, c_int64,
                POINTER(c_int64)]),
    "pas_encode_gas_filter_result": (
        c_int, [c_int32, _P, _P, POINTER(c_char_p), c_char_p, c_int64, POINTER(c_int64)]),
    "pas_encode_binding_result": (c_int, [c_char_p, c_char_p, c_int64, POINTER(c_int64)]),
    "pas_name_table_create": (c_int, [c_int32, POINTER(c_char_p), POINTER(c_void_p)]),
    "pas_name_table_destroy": (None, [_P]),
    "pas_name_table_lookup": (c_int32, [_P, c_char_p, c_int64]),
    "pas_decode_args": (
        c_int, [_P, c_char_p, c_int64, c_int32, _P, c_int64, _P, _P, POINTER(PasArgsInfo)]),
    "pas_decode_request_names": (
        c_int, [c_char_p, c_int64, c_int32, _P, c_int64, _P, c_int64, POINTER(c_int64),
                POINTER(c_int32)]),
    "pas_decode_pod_policy": (
        c_int, [c_char_p, c_int64, c_char_p, _P, c_int64, POINTER(c_int64), _P, c_int64,
                POINTER(c_int64)]),
    "pas_decode_pod_requests": (
        c_int, [c_char_p, c_int64, c_int32, POINTER(c_char_p), c_int32, _P, _P,
                POINTER(c_int32), POINTER(c_int32)]),
    "pas_decode_set_threads": (c_int, [c_int32]),
    "pas_decode_threads": (c_int32, [c_int64]),
    "pas_set_timing": (c_int, [_P, c_int]),
    "pas_kernel_time": (c_int, [_P, c_int32, POINTER(c_double), POINTER(c_int64)]),
    "pas_reset_timing": (c_int, [_P]),
}

_lib = None


def _load_host_only(path: str) -> ctypes.CDLL:
    """A host-only build of the C++ translation units (wire encoders, request decode,
    Quantity parsing) under a sanitizer, `make -C platform-aware-scheduling_amd sanitize`
    (scripts/sanitize.sh).  It has no HIP code: only the symbols it exports are bound, and a
    test that reaches a device entry point fails on the missing attribute."""
    lib = ctypes.CDLL(path)
    for name, (restype, argtypes) in SIGNATURES.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            continue
        fn.restype = restype
        fn.argtypes = argtypes
    return lib


def load() -> ctypes.CDLL:
    """Load libpas.so once; raises if it has not been built.  PAS_HOST_LIB=<path> loads a
    sanitizer build of the host-only translation units instead (test tooling only)."""
    global _lib
    if _lib is not None:
        return _lib
    host = os.environ.get("PAS_HOST_LIB")
    if host:
        _lib = _load_host_only(host)
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not found: build it with `make -C platform-aware-scheduling_amd` "
            "(or __graft_entry__.build()); there is no CPU fallback"
        )
    # One HIP runtime per process: torch's wheel ships its own libamdhip64.so with the
    # same soname (libamdhip64.so.7).  Loading torch first makes libpas.so bind to that
    # instance, so device pointers from torch allocations and torch streams are valid in
    # both; loading libpas.so first would leave torch a second runtime that cannot
    # initialise the device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    for name, (restype, argtypes) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = restype
        fn.argtypes = argtypes
    _lib = lib
    return lib


_fault = None


def load_fault() -> ctypes.CDLL:
    """lib/libpas_fault.so: libpas.so compiled with PAS_GAS_FAULT_INJECTION=1, whose GAS fits
    read PAS_GAS_FORCE_TIMEOUT=n (the next n fits' side-stream waits give up at once).  Test
    tooling for the fail-loud path of the fork / join; the product library has no such knob."""
    global _fault
    if _fault is not None:
        return _fault
    load()  # torch's HIP runtime first (see load)
    if not os.path.exists(FAULT_LIB_PATH):
        raise ImportError(f"{FAULT_LIB_PATH} not found: build it with "
                          "`make -C platform-aware-scheduling_amd`")
    lib = ctypes.CDLL(FAULT_LIB_PATH)
    for name, (restype, argtypes) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = restype
        fn.argtypes = argtypes
    _fault = lib
    return lib
