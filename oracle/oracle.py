"""ctypes wrapper of oracle/build/liboracle.so — the CPU restatement of the reference.

TEST INFRASTRUCTURE ONLY.  Used by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker / baseline; never by the product package.
Parity status: pinned against the reference's own test vectors and e2e fixtures
(tests/golden/); the Go reference cannot be built in this image.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_int, c_int32, c_int64, c_uint32, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# PAS_ORACLE_LIB=<path>: a sanitizer build of the same restatement (make -C oracle sanitize)
LIB_PATH = os.environ.get("PAS_ORACLE_LIB") or os.path.join(HERE, "build", "liboracle.so")

RULE_DTYPE = np.dtype([("metric", "<i4"), ("op", "<i4"), ("target", "<i8")], align=True)
RM_MAX_KEYS = 8


class OrRm(ctypes.Structure):
    _fields_ = [("has", ctypes.c_uint8 * RM_MAX_KEYS), ("val", c_int64 * RM_MAX_KEYS)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = ctypes.CDLL(LIB_PATH)
    P = c_void_p
    sigs = {
        "or_evaluate_rule": (c_int, [c_int64, c_int32, c_int64]),
        "or_violated": (c_int, [c_int32, c_int32, P, P, P, c_int32, P]),
        "or_ordered_list": (c_int32, [c_int32, c_int32, P, P, P, P, P]),
        "or_ordered_list_request": (c_int32, [c_int32, c_int32, P, P, P, c_int32, P, P]),
        "or_tas_eval": (c_int, [c_int32, c_int32, P, P, c_int32, P, P, P, P, c_uint32, P, P, P]),
        "or_tas_violations": (c_int, [c_int32, c_int32, P, P, c_int32, P, P, P]),
        "or_evaluate_rule_dec": (c_int, [c_int64, c_int32, c_int32, c_int64]),
        "or_cmp_dec": (c_int, [c_int64, c_int32, c_int64, c_int32]),
        "or_tas_eval_dec": (c_int, [c_int32, c_int32, P, P, P, c_int32, P, P, P, P, c_uint32,
                                    P, P, P]),
        "or_ordered_list_request_dec": (c_int32, [c_int32, c_int32, P, P, P, P, c_int32, P, P]),
        "or_tas_violations_dec": (c_int, [c_int32, c_int32, P, P, P, c_int32, P, P, P]),
        "or_rm_add": (c_int, [POINTER(OrRm), c_int32, c_int64]),
        "or_rm_subtract": (c_int, [POINTER(OrRm), c_int32, c_int64]),
        "or_rm_add_rm": (c_int, [POINTER(OrRm), POINTER(OrRm)]),
        "or_rm_subtract_rm": (c_int, [POINTER(OrRm), POINTER(OrRm)]),
        "or_rm_divide": (c_int, [POINTER(OrRm), c_int64]),
        "or_check_resource_capacity": (c_int, [POINTER(OrRm), POINTER(OrRm), POINTER(OrRm)]),
        "or_gas_fit_ex": (c_int, [c_int32, c_int32, c_int32, P, P, P, c_int32, c_int32, c_int32,
                                  P, P, P, P, P, P]),
        "or_gas_fit": (c_int, [c_int32, c_int32, c_int32, P, P, P, c_int32, c_int32, c_int32,
                               P, P, P, P]),
        "or_gas_bind": (c_int, [c_int32, c_int32, c_int32, P, P, P, c_int32, P, P, c_int32,
                                c_int32, P, P, P, P, P, P, P, P]),
        "or_gas_release_counts": (c_int, [c_int32, c_int32, c_int32, P, P, c_int32, P, P,
                                          c_int32, P, P, P, P, P]),
        "or_gas_release": (c_int, [c_int32, c_int32, c_int32, P, P, c_int32, P, P, c_int32,
                                   P, P, P, P, P, c_int32, P]),
        "or_label_plan": (c_int, [c_int32, c_int32, P, P, P, P, P, P]),
        "or_label_patch_json": (c_int64, [c_int32, P, ctypes.c_uint64, ctypes.c_uint64,
                                          ctypes.c_char_p, c_int64]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _p(a):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(c_void_p)


def w64(n):
    return (n + 63) // 64


def evaluate_rule(v_milli: int, op: int, target: int) -> int:
    return load().or_evaluate_rule(v_milli, op, target)


def _scale(v_scale, shape):
    """Per-value decimal places [M][N] (int8; value = v * 10^-scale) or None (milli)."""
    if v_scale is None:
        return None
    sc = np.ascontiguousarray(v_scale, np.int8)
    assert sc.shape == shape and sc.min(initial=0) >= 0 and sc.max(initial=0) <= 9
    return sc


def evaluate_rule_dec(u: int, s: int, op: int, target: int) -> int:
    return load().or_evaluate_rule_dec(u, s, op, target)


def cmp_dec(u1: int, s1: int, u2: int, s2: int) -> int:
    return load().or_cmp_dec(u1, s1, u2, s2)


def tas_eval(v_milli, present, rules, rule_off, prio, cand=None, flags=3, v_scale=None):
    """v_scale: per-value decimal places (value = v * 10^-v_scale), None = milli."""
    v = np.ascontiguousarray(v_milli, np.int64)
    m, n = v.shape
    p = np.ascontiguousarray(present, np.uint64)
    rules = np.ascontiguousarray(rules, RULE_DTYPE)
    rule_off = np.ascontiguousarray(rule_off, np.int32)
    prio = np.ascontiguousarray(prio, RULE_DTYPE)
    n_pods = rule_off.shape[0] - 1
    if cand is not None:
        cand = np.ascontiguousarray(cand, np.uint64)
    pass_out = np.zeros((n_pods, w64(n)), np.uint64) if flags & 1 else None
    order = np.zeros((n_pods, max(n, 1)), np.int32) if flags & 2 else None
    lens = np.zeros(n_pods, np.int32) if flags & 2 else None
    sc = _scale(v_scale, v.shape)
    rc = load().or_tas_eval_dec(n, m, _p(v), _p(sc), _p(p), n_pods,
                                _p(rules) if rules.size else None, _p(rule_off), _p(prio),
                                _p(cand), flags, _p(pass_out), _p(order), _p(lens))
    if rc != 0:
        raise ValueError("oracle: invalid operator (the reference panics)")
    return pass_out, order, lens


def prioritize_request(v_milli, present, prio, req_node, v_scale=None):
    """Request positions best-first for one request (SURVEY.md A.3 tie order)."""
    v = np.ascontiguousarray(v_milli, np.int64)
    m, n = v.shape
    p = np.ascontiguousarray(present, np.uint64)
    rule = np.ascontiguousarray(np.asarray(prio, RULE_DTYPE).reshape(1))
    req = np.ascontiguousarray(req_node, np.int32)
    out = np.zeros(max(len(req), 1), np.int32)
    sc = _scale(v_scale, v.shape)
    k = load().or_ordered_list_request_dec(n, m, _p(v), _p(sc), _p(p), _p(rule), len(req),
                                           _p(req), _p(out))
    return out[:k]


def tas_violations(v_milli, present, rules, rule_off, v_scale=None):
    v = np.ascontiguousarray(v_milli, np.int64)
    m, n = v.shape
    p = np.ascontiguousarray(present, np.uint64)
    rules = np.ascontiguousarray(rules, RULE_DTYPE)
    rule_off = np.ascontiguousarray(rule_off, np.int32)
    s = rule_off.shape[0] - 1
    out = np.zeros((s, w64(n)), np.uint64)
    sc = _scale(v_scale, v.shape)
    rc = load().or_tas_violations_dec(n, m, _p(v), _p(sc), _p(p), s,
                                      _p(rules) if rules.size else None, _p(rule_off), _p(out))
    if rc != 0:
        raise ValueError("oracle: invalid operator (the reference panics)")
    return out


MAX_SEL = 64  # OR_GAS_MAX_SEL
SEL_EXTENDED = 15
SEL_LIMIT = 14


def gas_fit(n_cards, cap, used, req, req_mask, n_containers, i915_index, selections=False):
    """Result words [P][N]; with selections=True also (sel [P][N][64] uint8, nsel [P][N];
    nsel -1 and sel zero for a fitting pod of more than 64 selections)."""
    n_cards = np.ascontiguousarray(n_cards, np.int32)
    cap = np.ascontiguousarray(cap, np.int64)
    used = np.ascontiguousarray(used, np.int64)
    req = np.ascontiguousarray(req, np.int64)
    req_mask = np.ascontiguousarray(req_mask, np.uint32)
    n_containers = np.ascontiguousarray(n_containers, np.int32)
    n, k, q = used.shape
    p, c, _ = req.shape
    out = np.zeros((p, n), np.uint32)
    sel = np.zeros((p, n, MAX_SEL), np.uint8) if selections else None
    nsel = np.zeros((p, n), np.int32) if selections else None
    rc = load().or_gas_fit_ex(n, k, q, _p(n_cards), _p(cap), _p(used), p, c, i915_index,
                              _p(req), _p(req_mask), _p(n_containers), _p(out), _p(sel),
                              _p(nsel))
    if rc != 0:
        raise ValueError(f"oracle gas_fit failed: {rc}")
    return (out, sel, nsel) if selections else out


def gas_bind(n_cards, cap, used, req, req_mask, n_containers, i915_index, pods, nodes,
             selections=False, counts=False):
    """Binds in order (bindNode: runSchedulingLogic + adjustPodResources(add)).
    Returns (used after, result words, statuses) [+ (cards [B][64], nsel [B])]
    [+ (counts [B][C][K] selections per container and card,)]."""
    n_cards = np.ascontiguousarray(n_cards, np.int32)
    cap = np.ascontiguousarray(cap, np.int64)
    used = np.array(used, np.int64, copy=True, order="C")
    req = np.ascontiguousarray(req, np.int64)
    req_mask = np.ascontiguousarray(req_mask, np.uint32)
    n_containers = np.ascontiguousarray(n_containers, np.int32)
    pods = np.ascontiguousarray(pods, np.int32)
    nodes = np.ascontiguousarray(nodes, np.int32)
    n, k, q = used.shape
    c = req.shape[1]
    b = len(pods)
    res = np.zeros(b, np.uint32)
    st = np.zeros(b, np.int32)
    cards = np.zeros((b, MAX_SEL), np.uint8)
    nsel = np.zeros(b, np.int32)
    cnt = np.zeros((b, c, k), np.int64)
    rc = load().or_gas_bind(n, k, q, _p(n_cards), _p(cap), _p(used), b, _p(pods), _p(nodes), c,
                            i915_index, _p(req), _p(req_mask), _p(n_containers), _p(res),
                            _p(st), _p(cards), _p(nsel), _p(cnt))
    if rc != 0:
        raise ValueError(f"oracle gas_bind failed: {rc}")
    out = (used, res, st) + ((cards, nsel) if selections else ())
    return out + (cnt,) if counts else out


def gas_release(n_cards, used, req, req_mask, n_containers, pods, nodes, cards_per_container,
                cards):
    """Pods leaving nodes (adjustPodResources(remove)).  cards [R][8] or [R][64].
    Returns (used after, statuses)."""
    n_cards = np.ascontiguousarray(n_cards, np.int32)
    used = np.array(used, np.int64, copy=True, order="C")
    req = np.ascontiguousarray(req, np.int64)
    req_mask = np.ascontiguousarray(req_mask, np.uint32)
    n_containers = np.ascontiguousarray(n_containers, np.int32)
    pods = np.ascontiguousarray(pods, np.int32)
    nodes = np.ascontiguousarray(nodes, np.int32)
    cpc = np.ascontiguousarray(cards_per_container, np.int32)
    r = len(pods)
    cards = np.ascontiguousarray(cards, np.int32).reshape(r, -1)
    n, k, q = used.shape
    c = req.shape[1]
    st = np.zeros(r, np.int32)
    rc = load().or_gas_release(n, k, q, _p(n_cards), _p(used), r, _p(pods), _p(nodes), c,
                               _p(req), _p(req_mask), _p(n_containers), _p(cpc), _p(cards),
                               cards.shape[1] if r else 8, _p(st))
    if rc != 0:
        raise ValueError(f"oracle gas_release failed: {rc}")
    return used, st


def gas_release_counts(n_cards, used, req, req_mask, n_containers, pods, nodes, counts):
    """gas_release with each annotation as counts [R][C][K] (cards per container and card).
    Returns (used after, statuses)."""
    n_cards = np.ascontiguousarray(n_cards, np.int32)
    used = np.array(used, np.int64, copy=True, order="C")
    req = np.ascontiguousarray(req, np.int64)
    req_mask = np.ascontiguousarray(req_mask, np.uint32)
    n_containers = np.ascontiguousarray(n_containers, np.int32)
    pods = np.ascontiguousarray(pods, np.int32)
    nodes = np.ascontiguousarray(nodes, np.int32)
    counts = np.ascontiguousarray(counts, np.int64)
    r = len(pods)
    n, k, q = used.shape
    c = req.shape[1]
    assert counts.shape == (r, c, k)
    st = np.zeros(r, np.int32)
    rc = load().or_gas_release_counts(n, k, q, _p(n_cards), _p(used), r, _p(pods), _p(nodes), c,
                                      _p(req), _p(req_mask), _p(n_containers), _p(counts),
                                      _p(st))
    if rc != 0:
        raise ValueError(f"oracle gas_release_counts failed: {rc}")
    return used, st


def label_plan(viol, labels, n_nodes, names=None):
    """updateNodeLabels per node: (add masks, remove masks, totalViolations).  names[s] =
    policy name of strategy s (None: all distinct); a name's remove bit and labels row are
    those of its first strategy."""
    viol = np.ascontiguousarray(viol, np.uint64)
    s = viol.shape[0]
    labels = None if labels is None else np.ascontiguousarray(labels, np.uint64)
    arr = None
    if names is not None:
        assert len(names) == s
        arr = (ctypes.c_char_p * max(s, 1))(*[n.encode() for n in names])
    add = np.zeros(n_nodes, np.uint64)
    rem = np.zeros(n_nodes, np.uint64)
    total = c_int64(0)
    rc = load().or_label_plan(n_nodes, s, None if arr is None else ctypes.cast(arr, c_void_p),
                              _p(viol), _p(labels), _p(add), _p(rem), ctypes.byref(total))
    if rc != 0:
        raise ValueError("oracle label_plan: more than 64 strategies")
    return add, rem, total.value


def label_patch_json(names, add, rem) -> bytes:
    arr = (ctypes.c_char_p * len(names))(*[n.encode() for n in names])
    buf = ctypes.create_string_buffer(1 << 16)
    n = load().or_label_patch_json(len(names), ctypes.cast(arr, c_void_p), int(add), int(rem),
                                   buf, len(buf))
    if n < 0:
        raise ValueError("oracle label_patch_json: buffer too small")
    return buf.raw[:n]


def rm(d: dict, keys: list) -> OrRm:
    """Build an or_rm from {name: value} with key ids from `keys`."""
    r = OrRm()
    for name, v in d.items():
        i = keys.index(name)
        r.has[i] = 1
        r.val[i] = v
    return r


def rm_dict(r: OrRm, keys: list) -> dict:
    return {keys[i]: r.val[i] for i in range(len(keys)) if r.has[i]}
