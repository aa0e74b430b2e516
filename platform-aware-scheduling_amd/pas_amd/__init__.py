"""pas_amd — Python handle on the MI355X-native Platform Aware Scheduling evaluator.

The evaluator itself is lib/libpas.so (HIP kernels for gfx950 + the C-ABI of
include/pas.h); this package loads it with ctypes and adds synthetic workloads.
Importing it loads the library and fails loudly when it has not been built.
"""
from . import _lib
from ._lib import (PAS_OP_EQUALS, PAS_OP_GREATER_THAN, PAS_OP_LESS_THAN, PAS_TAS_FILTER,
                   PAS_TAS_PRIORITIZE, PasError)
from .context import (RULE_DTYPE, Context, label_patch_json, make_rules, parse_operator,
                      quantity_as_int64, quantity_decimals, quantity_to_milli,
                      quantity_to_scaled, w64)

LIB = _lib.load()

__all__ = [
    "Context", "PasError", "RULE_DTYPE", "make_rules", "parse_operator", "quantity_to_milli",
    "quantity_to_scaled", "quantity_decimals",
    "quantity_as_int64", "w64", "label_patch_json", "PAS_OP_LESS_THAN", "PAS_OP_GREATER_THAN", "PAS_OP_EQUALS",
    "PAS_TAS_FILTER", "PAS_TAS_PRIORITIZE", "LIB",
]
