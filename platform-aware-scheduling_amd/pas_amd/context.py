"""Thin Python handle over a pas_ctx (include/pas.h).

Host entry points take/return numpy arrays; *_device entry points take objects with a
``data_ptr()`` (torch tensors on the GPU) and a HIP stream handle, so benchmarks can run
with every input already resident in HBM.
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_double, c_int32, c_int64, c_uint64, c_void_p
from typing import Optional, Tuple

import numpy as np

from . import _lib
from ._lib import PasError

# pas_rule {int32 metric; int32 op; int64 target}
RULE_DTYPE = np.dtype([("metric", "<i4"), ("op", "<i4"), ("target", "<i8")], align=True)
assert RULE_DTYPE.itemsize == 16


def w64(n: int) -> int:
    return (n + 63) // 64


def make_rules(metric, op, target) -> np.ndarray:
    metric = np.asarray(metric, dtype=np.int32)
    r = np.zeros(metric.shape[0], dtype=RULE_DTYPE)
    r["metric"] = metric
    r["op"] = np.asarray(op, dtype=np.int32)
    r["target"] = np.asarray(target, dtype=np.int64)
    return r


def _ptr(a: Optional[np.ndarray]):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays passed to libpas must be C-contiguous"
    return a.ctypes.data_as(c_void_p)


def _dptr(t):
    if t is None:
        return None
    return c_void_p(t.data_ptr())


PAS_STREAM_NULL = 1  # include/pas.h: the HIP null stream (NULL names the context's stream)


def _stream(s):
    """A hip_stream argument: None = the context's current stream; a torch.cuda.Stream or a raw
    handle otherwise, torch's default (null) stream as PAS_STREAM_NULL."""
    if s is None:
        return None
    h = s if isinstance(s, int) else s.cuda_stream
    return c_void_p(h if h != 0 else PAS_STREAM_NULL)


def parse_operator(op: str) -> int:
    """core.EvaluateRule's operator lookup (operator.go:14-25) via the C-ABI."""
    return _lib.load().pas_parse_operator(op.encode())


def quantity_to_milli(q: str) -> int:
    """Exact value*1000 of a resource.Quantity string; PasError(PAS_ENOTEXACT) otherwise."""
    out = c_int64()
    rc = _lib.load().pas_quantity_to_milli(q.encode(), byref(out))
    if rc != _lib.PAS_OK:
        raise PasError(rc, f"quantity {q!r}")
    return out.value


def quantity_to_scaled(q: str, places: int) -> int:
    """Exact value * 10^places (0..9) of a resource.Quantity string; PasError(PAS_ENOTEXACT)
    when that is not an integer or is outside int64."""
    out = c_int64()
    rc = _lib.load().pas_quantity_to_scaled(q.encode(), places, byref(out))
    if rc != _lib.PAS_OK:
        raise PasError(rc, f"quantity {q!r} at 10^-{places}")
    return out.value


def quantity_decimals(q: str) -> int:
    """The fewest decimal places (0..9) that hold the parsed quantity exactly."""
    out = ctypes.c_int32()
    rc = _lib.load().pas_quantity_decimals(q.encode(), byref(out))
    if rc != _lib.PAS_OK:
        raise PasError(rc, f"quantity {q!r}")
    return out.value


def quantity_as_int64(q: str) -> int:
    """resource.Quantity.AsInt64 with `ok` ignored (gpuscheduler/utils.go:23)."""
    out = c_int64()
    rc = _lib.load().pas_quantity_as_int64(q.encode(), byref(out))
    if rc != _lib.PAS_OK:
        raise PasError(rc, f"quantity {q!r}")
    return out.value


def label_patch_json(names, add_mask: int, remove_mask: int) -> bytes:
    """JSON PATCH body of one node's label update (deschedule/enforce.go:74-86, 104-135)."""
    l = _lib.load()
    arr = (ctypes.c_char_p * max(len(names), 1))(*[n.encode() for n in names])
    n = c_int64()
    cap = 256
    while True:
        buf = ctypes.create_string_buffer(cap)
        rc = l.pas_label_patch_json(len(names), arr, add_mask, remove_mask, buf, cap, byref(n))
        if rc == _lib.PAS_OK:
            return buf.raw[:n.value]
        if rc != _lib.PAS_ECAPACITY:
            raise PasError(rc, "pas_label_patch_json")
        cap = n.value


class Context:
    """One pas_ctx bound to a HIP device."""

    def __init__(self, device: int = -1, lib=None):
        self._l = lib if lib is not None else _lib.load()
        h = c_void_p()
        cfg = _lib.PasConfig(device, 0)
        rc = self._l.pas_create(byref(cfg), byref(h))
        if rc != _lib.PAS_OK:
            raise PasError(rc, "pas_create failed (no usable HIP device?)")
        self._h = h
        self.n_nodes = 0
        self.n_metrics = 0
        self.gas_shape = (0, 0, 0)

    # ------------------------------------------------------------------ plumbing
    def close(self):
        if getattr(self, "_h", None):
            self._l.pas_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc: int, what: str):
        if rc != _lib.PAS_OK:
            msg = self._l.pas_last_error(self._h)
            raise PasError(rc, f"{what}: {msg.decode() if msg else ''}")

    def last_error(self) -> str:
        return self._l.pas_last_error(self._h).decode()

    def set_stream(self, stream):
        self._check(self._l.pas_set_stream(self._h, _stream(stream)), "pas_set_stream")

    def synchronize(self):
        self._check(self._l.pas_synchronize(self._h), "pas_synchronize")

    # ------------------------------------------------------------------ timing
    def set_timing(self, level):
        """0/False = off, 1 = whole paths (PAS_TIMING_SPAN), 2/True = every launch."""
        level = 2 if level is True else int(level)
        self._check(self._l.pas_set_timing(self._h, level), "pas_set_timing")

    def kernel_time(self, kernel_id: int) -> Tuple[float, int]:
        ms = c_double()
        n = c_int64()
        self._check(self._l.pas_kernel_time(self._h, kernel_id, byref(ms), byref(n)),
                    "pas_kernel_time")
        return ms.value, n.value

    def reset_timing(self):
        self._check(self._l.pas_reset_timing(self._h), "pas_reset_timing")

    # ------------------------------------------------------------------ TAS
    def tas_snapshot_set(self, gen: int, v_milli: np.ndarray, present: np.ndarray,
                         scale=None):
        """Columns of value * 1000, or of value * 10^scale[m] (pas_tas_snapshot_set_scale)."""
        v = np.ascontiguousarray(v_milli, dtype=np.int64)
        m, n = v.shape
        p = np.ascontiguousarray(present, dtype=np.uint64)
        assert p.shape == (m, w64(n)), (p.shape, (m, w64(n)))
        self._check(self._l.pas_tas_snapshot_set(self._h, gen, n, m, _ptr(v), _ptr(p)),
                    "pas_tas_snapshot_set")
        self.n_nodes, self.n_metrics = n, m
        if scale is not None:
            self.tas_snapshot_set_scale(gen, scale)

    def tas_snapshot_set_scale(self, gen: int, scale, stream=None):
        """Decimal scale per column (0..9): column m holds value * 10^scale[m]."""
        sc = np.ascontiguousarray(scale, dtype=np.int32)
        self._check(self._l.pas_tas_snapshot_set_scale(self._h, gen, len(sc),
                                                       _ptr(sc) if sc.size else None,
                                                       _stream(stream)),
                    "pas_tas_snapshot_set_scale")

    def tas_snapshot_set_device(self, gen: int, n_nodes: int, n_metrics: int, v_t, p_t,
                                stream=None):
        self._check(self._l.pas_tas_snapshot_set_device(self._h, gen, n_nodes, n_metrics,
                                                        _dptr(v_t), _dptr(p_t),
                                                        _stream(stream)),
                    "pas_tas_snapshot_set_device")
        self.n_nodes, self.n_metrics = n_nodes, n_metrics

    def tas_snapshot_update(self, gen_from: int, gen_to: int, cols, v_milli: np.ndarray,
                            present: np.ndarray):
        """Replace metric columns `cols` (AutoUpdatingCache.updateMetric) and re-sort them."""
        cols = np.ascontiguousarray(cols, dtype=np.int32)
        v = np.ascontiguousarray(v_milli, dtype=np.int64).reshape(len(cols), self.n_nodes)
        p = np.ascontiguousarray(present, dtype=np.uint64).reshape(len(cols), w64(self.n_nodes))
        self._check(self._l.pas_tas_snapshot_update(
            self._h, gen_from, gen_to, len(cols), _ptr(cols) if cols.size else None,
            _ptr(v) if v.size else None, _ptr(p) if p.size else None), "pas_tas_snapshot_update")

    def tas_snapshot_update_device(self, gen_from: int, gen_to: int, cols, v_t, p_t,
                                   stream=None):
        cols = np.ascontiguousarray(cols, dtype=np.int32)
        self._check(self._l.pas_tas_snapshot_update_device(
            self._h, gen_from, gen_to, len(cols), _ptr(cols) if cols.size else None, _dptr(v_t),
            _dptr(p_t), _stream(stream)), "pas_tas_snapshot_update_device")

    def tas_snapshot_info(self):
        g = c_uint64()
        n = c_int32()
        m = c_int32()
        self._check(self._l.pas_tas_snapshot_info(self._h, byref(g), byref(n), byref(m)),
                    "pas_tas_snapshot_info")
        return g.value, n.value, m.value

    def tas_eval(self, gen: int, rules: np.ndarray, rule_off: np.ndarray, prio: np.ndarray,
                 cand: Optional[np.ndarray] = None,
                 flags: int = _lib.PAS_TAS_FILTER | _lib.PAS_TAS_PRIORITIZE):
        """Returns (pass[P, W64] uint64 or None, order[P, N] int32 or None, len[P] or None)."""
        rule_off = np.ascontiguousarray(rule_off, dtype=np.int32)
        n_pods = rule_off.shape[0] - 1
        rules = np.ascontiguousarray(rules, dtype=RULE_DTYPE)
        prio = np.ascontiguousarray(prio, dtype=RULE_DTYPE)
        assert prio.shape[0] == n_pods
        n = self.n_nodes
        if cand is not None:
            cand = np.ascontiguousarray(cand, dtype=np.uint64)
            assert cand.shape == (n_pods, w64(n))
        pass_out = np.zeros((n_pods, w64(n)), np.uint64) if flags & _lib.PAS_TAS_FILTER else None
        order = np.zeros((n_pods, n), np.int32) if flags & _lib.PAS_TAS_PRIORITIZE else None
        lens = np.zeros(n_pods, np.int32) if flags & _lib.PAS_TAS_PRIORITIZE else None
        rc = self._l.pas_tas_eval(self._h, gen, n_pods, _ptr(rules) if rules.size else None,
                                  _ptr(rule_off), _ptr(prio), _ptr(cand), flags, _ptr(pass_out),
                                  _ptr(order), _ptr(lens))
        self._check(rc, "pas_tas_eval")
        return pass_out, order, lens

    def tas_eval_device(self, gen: int, n_pods: int, n_rules: int, rules_t, rule_off_t, prio_t,
                        cand_t, flags: int, pass_t, order_t, len_t, stream=None):
        rc = self._l.pas_tas_eval_device(self._h, gen, n_pods, n_rules, _dptr(rules_t),
                                         _dptr(rule_off_t), _dptr(prio_t), _dptr(cand_t), flags,
                                         _dptr(pass_t), _dptr(order_t), _dptr(len_t),
                                         _stream(stream))
        self._check(rc, "pas_tas_eval_device")

    def tas_prioritize_request(self, gen: int, prio, req_node) -> np.ndarray:
        """Request positions best-first for one extender request (pas_tas_prioritize_request,
        SURVEY.md A.3 tie order); req_node[j] = snapshot node of Items[j] or -1."""
        rule = np.ascontiguousarray(np.asarray(prio, dtype=RULE_DTYPE).reshape(1))
        req = np.ascontiguousarray(req_node, dtype=np.int32)
        pos = np.zeros(max(len(req), 1), np.int32)
        n = ctypes.c_int32(0)
        rc = self._l.pas_tas_prioritize_request(self._h, gen, _ptr(rule), len(req), _ptr(req),
                                                _ptr(pos), ctypes.byref(n))
        self._check(rc, "pas_tas_prioritize_request")
        return pos[: n.value]

    def tas_prioritize_request_device(self, gen: int, prio, n_req: int, req_t, pos_t, len_t,
                                      stream=None):
        rule = np.ascontiguousarray(np.asarray(prio, dtype=RULE_DTYPE).reshape(1))
        rc = self._l.pas_tas_prioritize_request_device(self._h, gen, _ptr(rule), n_req,
                                                       _dptr(req_t), _dptr(pos_t), _dptr(len_t),
                                                       _stream(stream))
        self._check(rc, "pas_tas_prioritize_request_device")

    def tas_violations(self, gen: int, rules: np.ndarray, rule_off: np.ndarray) -> np.ndarray:
        rule_off = np.ascontiguousarray(rule_off, dtype=np.int32)
        s = rule_off.shape[0] - 1
        rules = np.ascontiguousarray(rules, dtype=RULE_DTYPE)
        out = np.zeros((s, w64(self.n_nodes)), np.uint64)
        rc = self._l.pas_tas_violations(self._h, gen, s, _ptr(rules) if rules.size else None,
                                        _ptr(rule_off), _ptr(out))
        self._check(rc, "pas_tas_violations")
        return out

    def tas_violations_device(self, gen: int, n_strat: int, n_rules: int, rules_t, rule_off_t,
                              viol_t, stream=None):
        rc = self._l.pas_tas_violations_device(self._h, gen, n_strat, n_rules, _dptr(rules_t),
                                               _dptr(rule_off_t), _dptr(viol_t),
                                               _stream(stream))
        self._check(rc, "pas_tas_violations_device")

    @staticmethod
    def _name_ids(names, n_strat: int):
        """int32 name ids of policy names (None: all distinct) as pas_tas_label_plan takes
        them: equal names, equal ids."""
        if names is None:
            return None
        assert len(names) == n_strat, "one policy name per strategy"
        ids = {}
        return np.array([ids.setdefault(n, len(ids)) for n in names], np.int32)

    def tas_label_plan(self, n_nodes: int, viol: np.ndarray, labels: Optional[np.ndarray] = None,
                       names=None):
        """(add [n_nodes] u64, remove [n_nodes] u64, total) of updateNodeLabels
        (deschedule/enforce.go:99-151) from viol[S][W64] and labels[S][W64] (or None);
        names[s] = policy name of strategy s (None: all distinct)."""
        viol = np.ascontiguousarray(viol, dtype=np.uint64)
        s = viol.shape[0]
        if labels is not None:
            labels = np.ascontiguousarray(labels, dtype=np.uint64)
            assert labels.shape == viol.shape, "labels must have the shape of viol"
        ids = self._name_ids(names, s)
        add = np.zeros(n_nodes, np.uint64)
        rem = np.zeros(n_nodes, np.uint64)
        total = c_int64()
        rc = self._l.pas_tas_label_plan(self._h, n_nodes, s, _ptr(viol) if viol.size else None,
                                        _ptr(ids), _ptr(labels) if labels is not None and
                                        labels.size else None, _ptr(add), _ptr(rem),
                                        byref(total))
        self._check(rc, "pas_tas_label_plan")
        return add, rem, total.value

    def tas_label_plan_device(self, n_nodes: int, n_strat: int, viol_t, labels_t, add_t, rem_t,
                              total_t, stream=None, names=None):
        ids = self._name_ids(names, n_strat)
        rc = self._l.pas_tas_label_plan_device(self._h, n_nodes, n_strat, _dptr(viol_t),
                                               _ptr(ids), _dptr(labels_t), _dptr(add_t),
                                               _dptr(rem_t), _dptr(total_t), _stream(stream))
        self._check(rc, "pas_tas_label_plan_device")

    def tas_deschedule_device(self, gen: int, n_strat: int, n_rules: int, rules_t, rule_off_t,
                              viol_t, labels_t, add_t, rem_t, total_t, stream=None, names=None):
        """The sweep and its label plan in one pass (pas_tas_deschedule_device): viol_t as
        tas_violations_device, add_t / rem_t / total_t as tas_label_plan_device on it."""
        ids = self._name_ids(names, n_strat)
        rc = self._l.pas_tas_deschedule_device(self._h, gen, n_strat, n_rules, _dptr(rules_t),
                                               _dptr(rule_off_t), _dptr(viol_t), _ptr(ids),
                                               _dptr(labels_t), _dptr(add_t), _dptr(rem_t),
                                               _dptr(total_t), _stream(stream))
        self._check(rc, "pas_tas_deschedule_device")

    # ------------------------------------------------------------------ GAS
    def gas_snapshot_set(self, gen: int, n_cards: np.ndarray, cap_per_gpu: np.ndarray,
                         used: np.ndarray):
        n_cards = np.ascontiguousarray(n_cards, dtype=np.int32)
        cap = np.ascontiguousarray(cap_per_gpu, dtype=np.int64)
        used = np.ascontiguousarray(used, dtype=np.int64)
        n, k, q = used.shape
        assert cap.shape == (n, q) and n_cards.shape == (n,)
        self._check(self._l.pas_gas_snapshot_set(self._h, gen, n, k, q, _ptr(n_cards),
                                                 _ptr(cap), _ptr(used)),
                    "pas_gas_snapshot_set")
        self.gas_shape = (n, k, q)

    def gas_snapshot_set_device(self, gen: int, n_nodes: int, max_cards: int, n_res: int,
                                n_cards_t, cap_t, used_t, stream=None):
        self._check(self._l.pas_gas_snapshot_set_device(self._h, gen, n_nodes, max_cards, n_res,
                                                        _dptr(n_cards_t), _dptr(cap_t),
                                                        _dptr(used_t), _stream(stream)),
                    "pas_gas_snapshot_set_device")
        self.gas_shape = (n_nodes, max_cards, n_res)

    def gas_fit(self, gen: int, req: np.ndarray, req_mask: np.ndarray, n_containers: np.ndarray,
                i915_index: int) -> np.ndarray:
        req = np.ascontiguousarray(req, dtype=np.int64)
        p, c, q = req.shape
        req_mask = np.ascontiguousarray(req_mask, dtype=np.uint32)
        n_containers = np.ascontiguousarray(n_containers, dtype=np.int32)
        assert req_mask.shape == (p, c) and n_containers.shape == (p,)
        out = np.zeros((p, self.gas_shape[0]), np.uint32)
        rc = self._l.pas_gas_fit(self._h, gen, p, c, i915_index, _ptr(req), _ptr(req_mask),
                                 _ptr(n_containers), _ptr(out))
        self._check(rc, "pas_gas_fit")
        return out

    def gas_fit_ex(self, gen: int, req: np.ndarray, req_mask: np.ndarray,
                   n_containers: np.ndarray, i915_index: int, side_cap: int = 1024):
        """pas_gas_fit_ex: (words [P][N], side records) — one GAS_SELECTION_DTYPE record per
        PAS_GAS_SEL_EXTENDED word (sorted by pod, node).  A side buffer that was too small is
        grown to the reported count and the call repeated."""
        req = np.ascontiguousarray(req, dtype=np.int64)
        p, c, q = req.shape
        req_mask = np.ascontiguousarray(req_mask, dtype=np.uint32)
        n_containers = np.ascontiguousarray(n_containers, dtype=np.int32)
        assert req_mask.shape == (p, c) and n_containers.shape == (p,)
        out = np.zeros((p, self.gas_shape[0]), np.uint32)
        while True:
            side = np.zeros(max(side_cap, 1), _lib.GAS_SELECTION_DTYPE)
            count = c_int64(0)
            rc = self._l.pas_gas_fit_ex(self._h, gen, p, c, i915_index, _ptr(req), _ptr(req_mask),
                                        _ptr(n_containers), _ptr(out), _ptr(side), side_cap,
                                        byref(count))
            self._check(rc, "pas_gas_fit_ex")
            if count.value <= side_cap:
                break
            side_cap = count.value
        side = side[:count.value]
        return out, side[np.lexsort((side["node"], side["pod"]))]

    def gas_fit_ex_device(self, gen: int, n_pods: int, max_containers: int, i915_index: int,
                          req_t, mask_t, ncont_t, res_t, side_t, side_cap: int, count_t,
                          stream=None):
        rc = self._l.pas_gas_fit_ex_device(self._h, gen, n_pods, max_containers, i915_index,
                                           _dptr(req_t), _dptr(mask_t), _dptr(ncont_t),
                                           _dptr(res_t), _dptr(side_t), side_cap, _dptr(count_t),
                                           _stream(stream))
        self._check(rc, "pas_gas_fit_ex_device")

    def gas_limit_count(self) -> int:
        """Pods of the last GAS fit beyond PAS_GAS_MAX_SELECTIONS (pas_gas_limit_count)."""
        v = c_int64(0)
        self._check(self._l.pas_gas_limit_count(self._h, byref(v)), "pas_gas_limit_count")
        return v.value

    def gas_bind(self, gen_from: int, gen_to: int, pods, nodes, req: np.ndarray,
                 req_mask: np.ndarray, n_containers: np.ndarray, i915_index: int,
                 selections: bool = False, counts: bool = False):
        """GASExtender.bindNode for binds (pods[b] -> nodes[b]) in order, committed into the
        resident usage.  Returns (result words, statuses), plus (cards [B][64], n_sel [B]) with
        selections=True (pas_gas_bind_ex), or plus counts [B][C][K] (selections per container
        and card, any number) with counts=True (pas_gas_bind_counts)."""
        req = np.ascontiguousarray(req, dtype=np.int64)
        p, c, q = req.shape
        req_mask = np.ascontiguousarray(req_mask, dtype=np.uint32)
        n_containers = np.ascontiguousarray(n_containers, dtype=np.int32)
        pods = np.ascontiguousarray(pods, dtype=np.int32)
        nodes = np.ascontiguousarray(nodes, dtype=np.int32)
        res = np.zeros(len(pods), np.uint32)
        st = np.zeros(len(pods), np.int32)
        if counts:
            cnt = np.zeros((len(pods), c, self.gas_shape[1]), np.int64)
            rc = self._l.pas_gas_bind_counts(self._h, gen_from, gen_to, len(pods), _ptr(pods),
                                             _ptr(nodes), p, c, i915_index, _ptr(req),
                                             _ptr(req_mask), _ptr(n_containers), _ptr(res),
                                             _ptr(st), _ptr(cnt))
            self._check(rc, "pas_gas_bind_counts")
            return res, st, cnt
        if not selections:
            rc = self._l.pas_gas_bind(self._h, gen_from, gen_to, len(pods), _ptr(pods),
                                      _ptr(nodes), p, c, i915_index, _ptr(req), _ptr(req_mask),
                                      _ptr(n_containers), _ptr(res), _ptr(st))
            self._check(rc, "pas_gas_bind")
            return res, st
        cards = np.zeros((len(pods), _lib.PAS_GAS_MAX_SELECTIONS), np.uint8)
        nsel = np.zeros(len(pods), np.int32)
        rc = self._l.pas_gas_bind_ex(self._h, gen_from, gen_to, len(pods), _ptr(pods),
                                     _ptr(nodes), p, c, i915_index, _ptr(req), _ptr(req_mask),
                                     _ptr(n_containers), _ptr(res), _ptr(st), _ptr(cards),
                                     _ptr(nsel))
        self._check(rc, "pas_gas_bind_ex")
        return res, st, cards, nsel

    def gas_release(self, gen_from: int, gen_to: int, pods, nodes, req: np.ndarray,
                    req_mask: np.ndarray, n_containers: np.ndarray, cards_per_container,
                    cards) -> np.ndarray:
        """adjustPodResources(remove) for pods leaving nodes; returns statuses.  cards is
        [R][8] (pas_gas_release) or [R][64] (pas_gas_release_ex)."""
        req = np.ascontiguousarray(req, dtype=np.int64)
        p, c, q = req.shape
        req_mask = np.ascontiguousarray(req_mask, dtype=np.uint32)
        n_containers = np.ascontiguousarray(n_containers, dtype=np.int32)
        pods = np.ascontiguousarray(pods, dtype=np.int32)
        nodes = np.ascontiguousarray(nodes, dtype=np.int32)
        cpc = np.ascontiguousarray(cards_per_container, dtype=np.int32).reshape(len(pods), c)
        cards = np.ascontiguousarray(cards, dtype=np.int32)
        ex = cards.size == len(pods) * _lib.PAS_GAS_MAX_SELECTIONS and cards.size > 0
        cards = cards.reshape(len(pods), _lib.PAS_GAS_MAX_SELECTIONS if ex else _lib.PAS_GAS_PACKED)
        st = np.zeros(len(pods), np.int32)
        fn = self._l.pas_gas_release_ex if ex else self._l.pas_gas_release
        rc = fn(self._h, gen_from, gen_to, len(pods), _ptr(pods), _ptr(nodes), p, c, _ptr(req),
                _ptr(req_mask), _ptr(n_containers), _ptr(cpc), _ptr(cards), _ptr(st))
        self._check(rc, "pas_gas_release_ex" if ex else "pas_gas_release")
        return st

    def gas_release_counts(self, gen_from: int, gen_to: int, pods, nodes, req: np.ndarray,
                           req_mask: np.ndarray, n_containers: np.ndarray,
                           counts) -> np.ndarray:
        """adjustPodResources(remove) with each annotation as counts [R][C][K] (container c
        lists card k that many times; pas_gas_release_counts); returns statuses."""
        req = np.ascontiguousarray(req, dtype=np.int64)
        p, c, q = req.shape
        req_mask = np.ascontiguousarray(req_mask, dtype=np.uint32)
        n_containers = np.ascontiguousarray(n_containers, dtype=np.int32)
        pods = np.ascontiguousarray(pods, dtype=np.int32)
        nodes = np.ascontiguousarray(nodes, dtype=np.int32)
        counts = np.ascontiguousarray(counts, dtype=np.int64).reshape(
            len(pods), c, self.gas_shape[1])
        st = np.zeros(len(pods), np.int32)
        rc = self._l.pas_gas_release_counts(self._h, gen_from, gen_to, len(pods), _ptr(pods),
                                            _ptr(nodes), p, c, _ptr(req), _ptr(req_mask),
                                            _ptr(n_containers), _ptr(counts), _ptr(st))
        self._check(rc, "pas_gas_release_counts")
        return st

    def gas_snapshot_get(self):
        """(generation, used [N][K][Q]) of the resident GAS snapshot."""
        n, k, q = self.gas_shape
        used = np.zeros((n, k, q), np.int64)
        g = c_uint64()
        self._check(self._l.pas_gas_snapshot_get(self._h, byref(g), _ptr(used)),
                    "pas_gas_snapshot_get")
        return g.value, used

    def gas_fit_device(self, gen: int, n_pods: int, max_containers: int, i915_index: int, req_t,
                       mask_t, ncont_t, res_t, stream=None):
        rc = self._l.pas_gas_fit_device(self._h, gen, n_pods, max_containers, i915_index,
                                        _dptr(req_t), _dptr(mask_t), _dptr(ncont_t),
                                        _dptr(res_t), _stream(stream))
        self._check(rc, "pas_gas_fit_device")

    def gas_fit_ld_device(self, gen: int, n_pods: int, max_containers: int, i915_index: int,
                          req_t, mask_t, ncont_t, res_t, ld_res: int, side_t=None,
                          side_cap: int = 0, count_t=None, stream=None):
        """pas_gas_fit_ld_device: words of (pod p, node n) at res_t.view(-1)[p * ld_res + n]."""
        rc = self._l.pas_gas_fit_ld_device(self._h, gen, n_pods, max_containers, i915_index,
                                           _dptr(req_t), _dptr(mask_t), _dptr(ncont_t),
                                           _dptr(res_t), ld_res,
                                           _dptr(side_t) if side_t is not None else None,
                                           side_cap,
                                           _dptr(count_t) if count_t is not None else None,
                                           _stream(stream))
        self._check(rc, "pas_gas_fit_ld_device")

    def gas_fit_bitmap_device(self, gen: int, n_pods: int, max_containers: int, i915_index: int,
                              req_t, mask_t, ncont_t, fit_t, stream=None):
        """GAS fit verdicts as node bitmaps fit_t[n_pods][W64] (pas_gas_fit_bitmap_device)."""
        rc = self._l.pas_gas_fit_bitmap_device(self._h, gen, n_pods, max_containers, i915_index,
                                               _dptr(req_t), _dptr(mask_t), _dptr(ncont_t),
                                               _dptr(fit_t), _stream(stream))
        self._check(rc, "pas_gas_fit_bitmap_device")

    # ------------------------------------------------------------------ node shards
    def tas_topk_device(self, gen: int, n_pods: int, n_rules: int, rules_t, rule_off_t, prio_t,
                        cand_t, k: int, node_base: int, key_t, node_t, len_t, stream=None):
        """First k HostPriorityList entries of this node shard as merge records
        (pas_tas_topk_device): key_t int64 [P][k], node_t int32 [P][k], len_t int32 [P]."""
        rc = self._l.pas_tas_topk_device(self._h, gen, n_pods, n_rules, _dptr(rules_t),
                                         _dptr(rule_off_t), _dptr(prio_t), _dptr(cand_t), k,
                                         node_base, _dptr(key_t), _dptr(node_t), _dptr(len_t),
                                         _stream(stream))
        self._check(rc, "pas_tas_topk_device")

    def tas_gas_topk_device(self, tas_gen: int, gas_gen: int, n_pods: int, n_rules: int, rules_t,
                            rule_off_t, prio_t, cand_t, max_containers: int, i915_index: int,
                            req_t, mask_t, ncont_t, k: int, node_base: int, key_t, node_t, len_t,
                            stream=None):
        """The same records over the nodes that pass TAS and fit the pod's GPU request
        (pas_tas_gas_topk_device: evaluated along each pod's order until k are kept)."""
        rc = self._l.pas_tas_gas_topk_device(
            self._h, tas_gen, gas_gen, n_pods, n_rules, _dptr(rules_t), _dptr(rule_off_t),
            _dptr(prio_t), _dptr(cand_t), max_containers, i915_index, _dptr(req_t),
            _dptr(mask_t), _dptr(ncont_t), k, node_base, _dptr(key_t), _dptr(node_t),
            _dptr(len_t), _stream(stream))
        self._check(rc, "pas_tas_gas_topk_device")

    def topk_merge_device(self, n_pods: int, k: int, n_shards: int, keys_t, nodes_t, out_node_t,
                          out_len_t, stream=None):
        """Merge of [n_shards][P][k] records into the global first-k lists."""
        rc = self._l.pas_topk_merge_device(self._h, n_pods, k, n_shards, _dptr(keys_t),
                                           _dptr(nodes_t), _dptr(out_node_t), _dptr(out_len_t),
                                           _stream(stream))
        self._check(rc, "pas_topk_merge_device")

    def list_merge_device(self, n_pods: int, n_shards: int, width: int, keys_t, nodes_t,
                          out_node_t, out_len_t, out_ld: int = 0, stream=None):
        """Merge of [n_shards][P][width] whole-shard records (pas_tas_topk_device with
        k = width) into the cluster's full lists out_node [P][>= n_shards * width]."""
        out_ld = out_ld or n_shards * width
        rc = self._l.pas_list_merge_device(self._h, n_pods, n_shards, width, _dptr(keys_t),
                                           _dptr(nodes_t), _dptr(out_node_t), out_ld,
                                           _dptr(out_len_t), _stream(stream))
        self._check(rc, "pas_list_merge_device")
