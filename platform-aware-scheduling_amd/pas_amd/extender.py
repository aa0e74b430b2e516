"""The reference's extender handlers over the C-ABI (BASELINE north_star: "drops in behind
the existing scheduler/filter and scheduler/prioritize HTTP verbs").

MetricsExtender mirrors telemetry-aware-scheduling/pkg/telemetryscheduler/telemetryscheduler.go
and GASExtender mirrors gpu-aware-scheduling/pkg/gpuscheduler/scheduler.go: same verbs, same
request decoding (extender.Args, BindingArgs), same status codes and bodies, same early
returns.  The evaluation goes through libpas.so (pas_tas_eval, pas_gas_fit, pas_gas_bind) and
the bodies through its wire encoders.  A verb takes the request body and returns
(HTTP status, response body), as an http.ResponseWriter would have received them.

The Go shim is the production host; this module is its restatement for the
tests, with the same names and error behaviour.
"""
from __future__ import annotations

import json
from typing import Dict, List, Mapping, Optional, Sequence, Tuple

import numpy as np

from . import _lib, wire
from .context import Context, make_rules, parse_operator, quantity_as_int64, w64

TAS_POLICY_LABEL = "telemetry-policy"  # telemetryscheduler.go: tasPolicy
I915 = "gpu.intel.com/i915"


def _field(obj, name):
    """encoding/json field lookup for BindingArgs (extender.Args goes through
    pas_decode_args): exact key first, then case-insensitive."""
    if not isinstance(obj, dict):
        return None
    if name in obj:
        return obj[name]
    low = name.lower()
    for k, v in obj.items():
        if k.lower() == low:
            return v
    return None


def _decode(body: bytes):
    if not body:
        raise ValueError("request body empty")
    return json.loads(body)


def _compact(item: bytes) -> bytes:
    """Compact re-encoding of one node item the library's decoder accepted.  Invalid UTF-8
    becomes U+FFFD, as Go's decoder maps it; nesting past Python's recursion limit (Go allows
    10000 levels) keeps the item's own bytes."""
    try:
        return json.dumps(json.loads(item.decode("utf-8", "replace")), separators=(",", ":"),
                          ensure_ascii=False).encode()
    except RecursionError:
        return item


class HandlerPanic(RuntimeError):
    """The reference handler panicked: core.EvaluateRule indexed its operator map with an
    unknown operator and called the nil function (operator.go:13-26).  net/http recovers a
    handler's panic and closes the connection, so no status line and no body reach the
    scheduler; in the deschedule controller's goroutine the panic ends the process."""


def _raise_if_panic(e: "_lib.PasError"):
    """PAS_EINVAL from a host entry's rule validation is the reference's panic."""
    if e.code == _lib.PAS_EINVAL and "unknown operator" in str(e):
        raise HandlerPanic(str(e)) from e
    raise e


def _op_code(op: str) -> int:
    """pas_op of a TASPolicyRule operator; an unknown one is passed on as an invalid code: the
    library skips it where its rule is never evaluated (metric not cached or cached with no
    node, strategy.go:27-36) and returns PAS_EINVAL where EvaluateRule would run."""
    code = parse_operator(op)
    return code if code >= 0 else 3


class MetricsExtender:
    """TAS extender: Filter / Prioritize / Bind (telemetryscheduler.go:36-244).

    policies: {(namespace, name): {"dontschedule": [(metric, op, target)],
                                   "scheduleonmetric": [(metric, op, target)]}}
    The context holds the TAS snapshot of generation `gen` over `node_names` x `metric_names`.
    """

    def __init__(self, ctx: Context, gen: int, node_names: Sequence[str],
                 metric_names: Sequence[str], policies: Mapping[Tuple[str, str], dict]):
        self.ctx, self.gen = ctx, gen
        self.node_names = list(node_names)
        self.node_index = {n: i for i, n in enumerate(node_names)}
        self.metric_index = {m: i for i, m in enumerate(metric_names)}
        self.policies = policies
        self.table = wire.NodeTable(node_names)
        self.name_table = wire.NameTable(node_names)

    # -- helpers ------------------------------------------------------------------
    def _decode(self, body: bytes):
        """DecodeExtenderRequest (:63-78) through pas_decode_args: (info, request node ids,
        candidate bitmap, item spans, (namespace, policy label)).  The pod's quantities are
        part of the reference's decode, so they are validated too.  Raises ValueError on a
        decode error or "no nodes in list"."""
        try:
            info, idx, cand, spans = wire.decode_args(self.name_table, body, _lib.PAS_ARGS_NODES,
                                                      spans=True)
            pod = body[info.pod_off: info.pod_off + info.pod_len]
            policy_ref = wire.decode_pod_policy(pod, TAS_POLICY_LABEL)
            wire.decode_pod_requests(pod, [])
        except _lib.PasError as e:
            if e.code != _lib.PAS_EDECODE:
                raise
            raise ValueError("error decoding request") from e
        if not info.has_nodes:
            raise ValueError("no nodes in list")
        return info, idx, cand, spans, policy_ref

    def _policy(self, policy_ref) -> Optional[dict]:
        """getPolicyFromPod (:103-112) on the decoded (namespace, label value)."""
        ns, name = policy_ref
        if name is None:
            return None
        return self.policies.get((ns, name))

    def _names(self, body, info, idx):
        """Request node names in order: snapshot names, or the decoded ones when the request
        names nodes the snapshot does not hold."""
        if info.n_unknown:
            return wire.decode_request_names(body, _lib.PAS_ARGS_NODES)
        return [self.node_names[i] for i in idx]

    def _rules(self, triples):
        metric, op, target = [], [], []
        for m, o, t in triples:
            metric.append(self.metric_index.get(m, -1))  # not cached: skipped (strategy.go:28-32)
            op.append(_op_code(o))
            target.append(int(t))
        return make_rules(metric, op, target)

    # -- verbs --------------------------------------------------------------------
    def filter(self, body: bytes) -> Tuple[int, bytes]:
        """Filter + filterNodes + WriteFilterResponse (:162-244)."""
        try:
            info, idx, cand, spans, policy_ref = self._decode(body)
        except ValueError:
            return 200, b""  # decode error: nothing written (:164-168)
        policy = self._policy(policy_ref)
        rules = (policy or {}).get("dontschedule") or []
        if policy is None or not rules:
            return 404, b"null\n"  # nil FilterResult (:189-198)
        # Violated runs before the empty-list check (:199-203), so an unknown operator on a
        # cached metric panics even for an empty node list
        r = self._rules(rules)
        try:
            pass_out, _, _ = self.ctx.tas_eval(self.gen, r, np.array([0, len(r)], np.int32),
                                               make_rules([-1], [0], [0]), cand[None, :],
                                               _lib.PAS_TAS_FILTER)
        except _lib.PasError as e:
            _raise_if_panic(e)
        if info.n_req == 0:
            return 404, b"null\n"  # nil FilterResult (:200-203)
        # the shim's json.Marshal of each v1.Node (here: the compact re-encoding of the item)
        blobs = [_compact(body[o:o + n]) for o, n in spans]
        table = wire.NodeTable(self._names(body, info, idx), blobs)
        order = np.arange(info.n_req, dtype=np.int32)
        # the pass row re-indexed to the request's own order (duplicates keep their verdict);
        # a node without metrics in the snapshot is in no violating set, so it passes
        # (dontschedule/strategy.go:25-44 only ranges over the metric cache's nodes)
        row = np.zeros(w64(info.n_req), np.uint64)
        for j, i in enumerate(idx):
            if i < 0 or (int(pass_out[0, i >> 6]) >> (int(i) & 63)) & 1:
                row[j >> 6] |= np.uint64(1 << (j & 63))
        return 200, wire.tas_filter_result(order, row, table)

    def prioritize(self, body: bytes) -> Tuple[int, bytes]:
        """Prioritize + prioritizeNodes + WritePrioritizeResponse (:36-158)."""
        try:
            info, idx, cand, _, policy_ref = self._decode(body)
        except ValueError:
            return 200, b""
        if info.n_req == 0:
            return 200, b""  # no nodes: nothing written (:46-49)
        status = 200
        if policy_ref[1] is None:
            status = 400  # (:50-53), then the (empty) list is still written
        policy = self._policy(policy_ref)
        prio = (policy or {}).get("scheduleonmetric") or []
        # getSchedulingRule (:115-124): first rule with a metric name; errors -> []
        if policy is None or not prio or not prio[0][0]:
            return status, b"[]\n"
        if prio[0][0] not in self.metric_index:  # ReadMetric error -> [] (:130-133)
            return status, b"[]\n"
        # nodes without metrics in the snapshot are left out, as filteredNodeData keeps only
        # nodes with a metric (telemetryscheduler.go:128-149); ties keep request order
        # (SURVEY.md A.3): pas_tas_prioritize_request lists request positions
        code = parse_operator(prio[0][1])
        p = make_rules([self.metric_index[prio[0][0]]], [code if code >= 0 else 3],
                       [int(prio[0][2])])
        pos = self.ctx.tas_prioritize_request(self.gen, p[0], idx)
        table = wire.NodeTable(self._names(body, info, idx))
        return status, wire.host_priority_list(pos, table)

    def bind(self, body: bytes) -> Tuple[int, bytes]:
        return 404, b""  # not implemented by TAS (:178-181)


class GASExtender:
    """GAS extender: Filter / Bind / Prioritize (gpuscheduler/scheduler.go:385-573).

    The context holds the GAS snapshot (generation `gen`) built by
    pas_amd.snapshot.gas_snapshot_from_nodes over `node_names` with `card_names` and `kinds`;
    `pods` resolves BindingArgs to pods ({(namespace, name): v1.Pod JSON object})."""

    def __init__(self, ctx: Context, gen: int, node_names: Sequence[str],
                 card_names: Sequence[Sequence[str]], kinds: Sequence[str],
                 pods: Optional[Dict[Tuple[str, str], dict]] = None):
        self.ctx, self.gen = ctx, gen
        self.node_names = list(node_names)
        self.node_index = {n: i for i, n in enumerate(node_names)}
        self.name_table = wire.NameTable(node_names)
        self.card_names = card_names
        self.kinds = list(kinds)
        self.pods = pods if pods is not None else {}
        self.i915 = self.kinds.index(I915) if I915 in self.kinds else -1

    def _requests(self, pod_json: bytes):
        """containerRequests (utils.go:14-32) through pas_decode_pod_requests: gpu.intel.com/
        requests as AsInt64 (ok ignored) in the pas_gas_fit layout, plus each container's
        numI915 (its annotation segment length)."""
        # a container requesting a gpu.intel.com/ kind no node has carries
        # PAS_REQ_UNKNOWN_KIND in its mask: with numI915 > 0 it fits no node (capacity lacks
        # the key, :349-354), with numI915 == 0 it makes no selection (:206-215)
        req, mask, ncont, _ = wire.decode_pod_requests(pod_json, self.kinds)
        per_container = []
        for ci in range(int(ncont[0])):
            on = self.i915 >= 0 and (int(mask[0, ci]) >> self.i915) & 1
            per_container.append(max(int(req[0, ci, self.i915]), 0) if on else 0)
        return req, mask, ncont, per_container

    def filter(self, body: bytes) -> Tuple[int, bytes]:
        """Filter + filterNodes (:449-482, 523-543), the body decoded by pas_decode_args."""
        try:
            info, idx, cand, _ = wire.decode_args(self.name_table, body,
                                                  _lib.PAS_ARGS_NODE_NAMES)
            req, mask, ncont, _ = self._requests(body[info.pod_off: info.pod_off + info.pod_len])
        except _lib.PasError as e:
            if e.code != _lib.PAS_EDECODE:
                raise
            return 404, b""  # errDecode (:499-501, 528-533)
        if info.n_req == 0:
            return 404, wire.gas_filter_result([], np.zeros(1, np.uint64), wire.NodeTable([]))
        names = (wire.decode_request_names(body, _lib.PAS_ARGS_NODE_NAMES) if info.n_unknown
                 else [self.node_names[i] for i in idx])
        res = self.ctx.gas_fit(self.gen, req, mask, ncont, self.i915)
        fit = np.zeros(w64(info.n_req), np.uint64)
        for j, i in enumerate(idx):
            if i >= 0 and int(res[0, i]) >> 31:  # unknown node: FetchNode error
                fit[j >> 6] |= np.uint64(1 << (j & 63))
        return 200, wire.gas_filter_result(np.arange(info.n_req, dtype=np.int32), fit,
                                           wire.NodeTable(names))

    def bind(self, body: bytes) -> Tuple[int, bytes]:
        """Bind + bindNode (:385-445, 546-566): fit on the current usage, commit, annotate."""
        try:
            args = _decode(body)
        except ValueError:
            return 404, b""
        key = (_field(args, "PodNamespace") or "", _field(args, "PodName") or "")
        pod = self.pods.get(key)
        if pod is None:  # fetchPod: the lister's NotFound error (node_resource_cache.go:460-471)
            return 404, self._error(f'pod "{key[1]}" not found')
        node_name = _field(args, "Node") or ""
        node = self.node_index.get(node_name)
        req, mask, ncont, per_container = self._requests(json.dumps(pod).encode())
        if node is None:  # runSchedulingLogic -> FetchNode error (:282-288)
            return 404, self._error(f'node "{node_name}" not found')
        # the selection as counts per container and card: any number of selections
        res, st, cnt = self.ctx.gas_bind(self.gen, self.gen + 1, [0], [node], req, mask, ncont,
                                         self.i915, counts=True)
        self.gen += 1
        if st[0] != _lib.PAS_GAS_OK:
            return 404, self._error("will not fit")  # errWontFit (:49)
        from .snapshot import annotation_counts
        names = self.card_names[node]
        pod.setdefault("metadata", {}).setdefault("annotations", {})[
            "gas-container-cards"] = annotation_counts(cnt[0, :, : len(names)], int(ncont[0]),
                                                       names)
        return 200, wire.binding_result("")

    def prioritize(self, body: bytes) -> Tuple[int, bytes]:
        return 404, b""  # not implemented by GAS (:517-519)

    @staticmethod
    def _error(msg: str) -> bytes:
        """BindingResult{Error: msg} through json.NewEncoder (:508-513)."""
        return wire.binding_result(msg)


def _strategy_equals(a: Tuple[str, list], b: Tuple[str, list]) -> bool:
    """deschedule.Strategy.Equals (deschedule/strategy.go:60-78): same policy name and the
    same non-empty rule list (metric, target, operator per position)."""
    (na, ra), (nb, rb) = a, b
    if na != nb or not ra or len(ra) != len(rb):
        return False
    return all(x[0] == y[0] and int(x[2]) == int(y[2]) and x[1] == y[1] for x, y in zip(ra, rb))


class DescheduleEnforcer:
    """deschedule.Strategy.Enforce over the registered deschedule strategies
    (telemetry-aware-scheduling/pkg/strategies/deschedule/enforce.go:57-164):
    nodeStatusForStrategy (pas_tas_violations), updateNodeLabels (pas_tas_label_plan) and
    the PATCH bodies (pas_label_patch_json).

    strategies: [(policy name, [(metric, op, target), ...])] in registration order.  As
    MetricEnforcer.AddStrategy (core/enforcer.go:84-103) a strategy Equals to one already
    registered is dropped; strategies that only share a policy name stay, and the label plan
    keys removes and totalViolations by name (enforce.go:89-134).  More than 64 strategies
    are planned in groups of <= 64 that keep each name's strategies together."""

    MAX_PLAN = 64  # strategies per pas_tas_label_plan call

    def __init__(self, ctx: Context, gen: int, node_names: Sequence[str],
                 metric_names: Sequence[str], strategies: Sequence[Tuple[str, list]]):
        self.ctx, self.gen = ctx, gen
        self.node_names = list(node_names)
        self.metric_index = {m: i for i, m in enumerate(metric_names)}
        registered: List[Tuple[str, list]] = []
        for st in strategies:
            if not any(_strategy_equals(r, st) for r in registered):
                registered.append(st)
        self.names = [s[0] for s in registered]
        metric, op, target, off = [], [], [], [0]
        for _, rules in registered:
            for m, o, t in rules:
                metric.append(self.metric_index.get(m, -1))
                op.append(_op_code(o))  # unknown: skipped or the panic, as in filter
                target.append(int(t))
            off.append(len(metric))
        self.rules = make_rules(metric, op, target)
        self.rule_off = np.array(off, np.int32)
        # plan groups: whole names, first-registration order, <= 64 strategies per group
        by_name: Dict[str, List[int]] = {}
        for i, n in enumerate(self.names):
            by_name.setdefault(n, []).append(i)
        self.groups: List[List[int]] = [[]]
        for members in by_name.values():
            if len(members) > self.MAX_PLAN:
                raise ValueError(f"policy name {self.names[members[0]]!r}: more than "
                                 f"{self.MAX_PLAN} registered deschedule strategies")
            if len(self.groups[-1]) + len(members) > self.MAX_PLAN:
                self.groups.append([])
            self.groups[-1].extend(members)

    def enforce(self, node_labels: Sequence[Mapping[str, str]]):
        """(totalViolations, {node name: PATCH body}) for the listed nodes' current labels;
        every node gets a body, "[]" when nothing changes (enforce.go:104-135)."""
        n, s = len(self.node_names), len(self.names)
        try:
            viol = self.ctx.tas_violations(self.gen, self.rules, self.rule_off)
        except _lib.PasError as e:
            _raise_if_panic(e)
        labels = np.zeros((s, w64(n)), np.uint64)
        for i, lab in enumerate(node_labels):
            for j, name in enumerate(self.names):
                if name in lab:
                    labels[j, i >> 6] |= np.uint64(1 << (i & 63))
        from .context import label_patch_json
        total = 0
        adds: List[List[bytes]] = [[] for _ in range(n)]
        rems: List[List[bytes]] = [[] for _ in range(n)]
        for g in self.groups:
            if not g:
                continue
            names = [self.names[j] for j in g]
            add, rem, t = self.ctx.tas_label_plan(n, viol[g], labels[g], names)
            total += t
            for i in range(n):
                a, r = int(add[i]), int(rem[i])
                if a:
                    adds[i].append(label_patch_json(names, a, 0)[1:-1])
                if r:
                    rems[i].append(label_patch_json(names, 0, r)[1:-1])
        bodies = {self.node_names[i]: b"[" + b",".join(adds[i] + rems[i]) + b"]"
                  for i in range(n)}
        return total, bodies
