"""The extender verbs end to end, as the reference's handler tests drive them
(telemetryscheduler/scheduler_test.go: JSON requests built from twoNodeArgument / noPolicyPod,
responses decoded and compared), through pas_amd.extender over libpas.so.  Marked gpu."""
import json

import numpy as np
import pytest

import pas_amd
from pas_amd import extender as ext
from pas_amd import snapshot as sn
from helpers import golden

pytestmark = pytest.mark.gpu
G = golden()

# scheduler_test.go:28-62
TEST_POLICY1 = {("default", "test-policy"): {
    "scheduleonmetric": [("dummyMetric1", "GreaterThan", 0)],
    "dontschedule": [("dummyMetric1", "GreaterThan", 40)]}}
TEST_POLICY2 = {("default", "other-policy"): TEST_POLICY1[("default", "test-policy")]}


def node(name):
    return {"metadata": {"name": name}, "spec": {}, "status": {}}


def args(pod_labels, names, key_case=str):
    a = {"Pod": {"metadata": {"name": "big pod", "labels": pod_labels, "namespace": "default"}},
         "Nodes": {"metadata": {}, "items": [node(n) for n in names]},
         "NodeNames": list(names)}
    return json.dumps({key_case(k): v for k, v in a.items()}).encode()


TWO_NODES = dict(pod_labels={"telemetry-policy": "test-policy"}, names=["node A", "node B"])


def tas(ctx, metric_values, policies, gen):
    names = ["node A", "node B"]
    v, pres, scale = sn.tas_snapshot_from_metrics(
        {"dummyMetric1": {k: str(x) for k, x in metric_values.items()}}, names)
    ctx.tas_snapshot_set(gen, v, pres, scale)
    return ext.MetricsExtender(ctx, gen, names, ["dummyMetric1"], policies)


def test_prioritize_golden_g5(ctx):
    g = G["G5_prioritize"]
    m = tas(ctx, g["metrics"]["dummyMetric1"], TEST_POLICY1, 8100)
    for case in (str, str.lower):  # the kube-scheduler sends lower-case keys
        status, body = m.prioritize(args(**TWO_NODES, key_case=case))
        assert status == 200
        assert [[h["Host"], h["Score"]] for h in json.loads(body)] == g["want"]
        assert body.endswith(b"\n")


def test_prioritize_ties_keep_request_order(ctx):
    # equal values: the HostPriorityList follows args.Nodes.Items, whatever
    # the snapshot's node numbering; a repeated name is listed once
    m = tas(ctx, {"node A": 50, "node B": 50}, TEST_POLICY1, 8103)
    for names in (["node B", "node A"], ["node A", "node B"], ["node B", "node B", "node A"]):
        status, body = m.prioritize(args(TWO_NODES["pod_labels"], names))
        assert status == 200
        want = list(dict.fromkeys(names))
        assert [[h["Host"], h["Score"]] for h in json.loads(body)] == [
            [n, 10 - i] for i, n in enumerate(want)]


def test_prioritize_errors_g6(ctx):
    # policy not found -> [] (scheduler_test.go:175-183)
    m = tas(ctx, {"node A": 90, "node B": 100}, TEST_POLICY2, 8101)
    assert m.prioritize(args(**TWO_NODES)) == (200, b"[]\n")
    # unlabelled pod -> 400 and [] (scheduler_test.go:104-112; telemetryscheduler.go:50-53)
    m = tas(ctx, {"node A": 100, "node B": 90}, TEST_POLICY1, 8102)
    status, body = m.prioritize(args({"useless-label": "test-policy"}, ["node A"]))
    assert status == 400 and body == b"[]\n"
    # malformed arguments: extender.Args{} has Nodes == nil -> decode error, nothing written
    assert m.prioritize(b"{}") == (200, b"")
    assert m.prioritize(b"") == (200, b"")


def test_filter_golden_g7(ctx):
    g = G["G7_filter"]
    for gen, c in enumerate(g["cases"], start=8110):
        m = tas(ctx, c["metrics"]["dummyMetric1"], TEST_POLICY1, gen)
        status, body = m.filter(args(**TWO_NODES))
        assert status == 200
        res = json.loads(body)
        # the reference test's assertion (scheduler_test.go:321-337)
        assert sorted(res["FailedNodes"]) == sorted(c["want_failed"])
        assert res["NodeNames"] == c["want_node_names"]
        assert [it["metadata"]["name"] for it in res["Nodes"]["items"] or []] == c["want_passed"]


def test_filter_nil_results(ctx):
    m = tas(ctx, {"node A": 10, "node B": 30}, TEST_POLICY1, 8120)
    # no policy label, policy not cached, no nodes: nil FilterResult -> 404 + null
    assert m.filter(args({"useless-label": "x"}, ["node A"])) == (404, b"null\n")
    m2 = tas(ctx, {"node A": 10, "node B": 30}, TEST_POLICY2, 8121)
    assert m2.filter(args(**TWO_NODES)) == (404, b"null\n")
    # an empty node list: Violated still runs first (telemetryscheduler.go:199-203), on the
    # resident snapshot (m2 replaced m's)
    m4 = tas(ctx, {"node A": 10, "node B": 30}, TEST_POLICY1, 8123)
    assert m4.filter(args({"telemetry-policy": "test-policy"}, [])) == (404, b"null\n")
    # no dontschedule strategy
    m3 = tas(ctx, {"node A": 10}, {("default", "test-policy"): {
        "scheduleonmetric": [("dummyMetric1", "GreaterThan", 0)]}}, 8122)
    assert m3.filter(args(**TWO_NODES)) == (404, b"null\n")
    assert m.bind(b"{}") == (404, b"")


def gas_cluster():
    nodes = [{"labels": {"gpu.intel.com/cards": "card0.card1"},
              "allocatable": {"gpu.intel.com/i915": "2", "gpu.intel.com/memory.max": "16G"}},
             {"labels": {}, "allocatable": {}}]
    return ["node-1", "node-2"], nodes


def gas_pod(name, mem="5G", i915="1"):
    return {"metadata": {"name": name, "namespace": "default"},
            "spec": {"containers": [{"resources": {"requests": {
                "gpu.intel.com/i915": i915, "gpu.intel.com/memory.max": mem}}}]}}


def test_gas_filter_and_bind_readme(ctx):
    # README.md:15-21 worked example through the GAS verbs: three 5 GB pods bound in turn
    names, nodes = gas_cluster()
    kinds = ["gpu.intel.com/i915", "gpu.intel.com/memory.max"]
    n_cards, cap, used, card_names = sn.gas_snapshot_from_nodes(nodes, kinds)
    ctx.gas_snapshot_set(8200, n_cards, cap, used)
    pods = {("default", f"p{i}"): gas_pod(f"p{i}") for i in range(3)}
    g = ext.GASExtender(ctx, 8200, names, card_names, kinds, pods)
    body = json.dumps({"Pod": pods[("default", "p0")], "NodeNames": names}).encode()
    status, out = g.filter(body)
    res = json.loads(out)
    assert status == 200 and res["NodeNames"] == ["node-1"]
    assert res["FailedNodes"] == {"node-2": "Not enough GPU-resources for deployment"}
    want = G["G11_gas_readme"]["memory_example"]["want"]
    for i, w in enumerate(want):
        status, out = g.bind(json.dumps({"PodName": f"p{i}", "PodNamespace": "default",
                                         "PodUID": "", "Node": "node-1"}).encode())
        if w["fits"]:
            assert (status, out) == (200, b'{"Error":""}\n')
            ann = pods[("default", f"p{i}")]["metadata"]["annotations"]["gas-container-cards"]
            assert ann == w["annotation"]
        else:
            assert (status, out) == (404, b'{"Error":"will not fit"}\n')
    # after the binds the node is full for a fourth pod: filter sees the committed usage
    status, out = g.filter(body)
    assert json.loads(out)["NodeNames"] is None
    # errors
    assert g.filter(json.dumps({"Pod": pods[("default", "p0")], "NodeNames": []}).encode())[0] == 404
    assert g.bind(json.dumps({"PodName": "nope", "PodNamespace": "default"}).encode()) == \
        (404, b'{"Error":"pod \\"nope\\" not found"}\n')
    assert g.prioritize(b"{}") == (404, b"")


def test_deschedule_enforce_g4(ctx):
    # deschedule/enforce_test.go:38-52 through the Enforce mirror
    from test_oracle_golden import apply_label_patch
    g = G["G4_deschedule_enforce"]
    for gen, c in enumerate(g["cases"], start=8300):
        v, pres, scale = sn.tas_snapshot_from_metrics(
            {m: {k: str(x) for k, x in vals.items()} for m, vals in g["metrics"].items()},
            g["nodes"], ["memory", "cpu"])
        ctx.tas_snapshot_set(gen, v, pres, scale)
        e = ext.DescheduleEnforcer(ctx, gen, g["nodes"], ["memory", "cpu"],
                                   [(g["policy"], [tuple(r) for r in c["rules"]])])
        total, bodies = e.enforce([c["labels"]])
        assert total == c["derived"]["total"]
        assert bodies["node-1"].decode() == c["derived"]["patch"]
        after = apply_label_patch(c["labels"], bodies["node-1"])
        assert [n for n in g["nodes"] if after.get(g["policy"]) == "violating"] == c["want"]


def test_deschedule_enforce_shared_names(ctx):
    """G4n (derived): registered strategies that share a policy name, through the Enforce
    mirror: one remove / count per name (enforce.go:89-134)."""
    from test_oracle_golden import apply_label_patch
    g = G["G4n_shared_policy_name"]
    v, pres, scale = sn.tas_snapshot_from_metrics(
        {m: {k: str(x) for k, x in vals.items()} for m, vals in g["metrics"].items()},
        g["nodes"], ["memory"])
    ctx.tas_snapshot_set(8310, v, pres, scale)
    for c in g["cases"]:
        e = ext.DescheduleEnforcer(ctx, 8310, g["nodes"], ["memory"],
                                   [(nm, [tuple(r) for r in rules])
                                    for nm, rules in c["strategies"]])
        total, bodies = e.enforce([c["labels"]])
        assert total == c["total"], c["name"]
        assert bodies["node-1"].decode() == c["patch"], c["name"]
        after = apply_label_patch(c["labels"], bodies["node-1"])
        assert (after.get("p") == "violating") == bool(c["add"])


def test_deschedule_enforce_registry_dedupe(ctx):
    """AddStrategy (core/enforcer.go:84-103) drops a strategy Equals to a registered one
    (deschedule/strategy.go:60-78: same name, same non-empty rules); same name with other
    rules, or empty rules, stays."""
    names = ["node A", "node B"]
    v, pres, scale = sn.tas_snapshot_from_metrics({"m": {"node A": "50", "node B": "30"}}, names,
                                              ["m"])
    ctx.tas_snapshot_set(8320, v, pres, scale)
    r1 = [("m", "GreaterThan", 40)]
    e = ext.DescheduleEnforcer(ctx, 8320, names, ["m"],
                               [("p", r1), ("p", list(r1)), ("p", [("m", "GreaterThan", 41)]),
                                ("q", []), ("q", [])])
    assert e.names == ["p", "p", "q", "q"]
    total, bodies = e.enforce([{}, {"p": "violating"}])
    # node A: p violated (twice: r1 and GreaterThan 41), q not -> 1; node B: p, q not -> 2
    assert total == 3
    assert json.loads(bodies["node A"]) == [
        {"op": "add", "path": "/metadata/labels/p", "value": "violating"}] * 2
    assert json.loads(bodies["node B"]) == [
        {"op": "remove", "path": "/metadata/labels/p", "value": ""},
        {"op": "add", "path": "/metadata/labels/p", "value": "null"}]


def _update_node_labels(names, viol_bits, node_labels):
    """updateNodeLabels (enforce.go:99-151) literally: per node, allPolicies by name, delete
    per violating strategy, remove + null / count per remaining name.  Returns (total,
    [sorted ops per node])."""
    total, out = 0, []
    for i, lab in enumerate(node_labels):
        non_violated = dict.fromkeys(names)
        ops = []
        for j, nm in enumerate(names):
            if viol_bits[j, i]:
                non_violated.pop(nm, None)
                ops.append(("add", nm, "violating"))
        for nm in non_violated:
            if nm in lab:
                ops += [("remove", nm, ""), ("add", nm, "null")]
            total += 1
        out.append(sorted(ops))
    return total, out


def test_deschedule_enforce_more_than_64_strategies(ctx, oracle):
    """150 strategies under 40 policy names: planned in groups of <= 64 whole names; the
    total and every node's set of operations equal the literal restatement."""
    from helpers import unpack_bits
    rng = np.random.default_rng(21)
    n_nodes, metrics = 300, ["m0", "m1", "m2"]
    nodes = [f"node-{i}" for i in range(n_nodes)]
    vals = {m: {nd: str(int(rng.integers(0, 100))) for nd in nodes if rng.random() > 0.05}
            for m in metrics}
    v, pres, scale = sn.tas_snapshot_from_metrics(vals, nodes, metrics)
    ctx.tas_snapshot_set(8330, v, pres, scale)
    strategies = []
    for j in range(150):
        rules = [(metrics[int(rng.integers(0, 3))], ["LessThan", "GreaterThan", "Equals"][
            int(rng.integers(0, 3))], int(rng.integers(0, 100))) for _ in range(2)]
        strategies.append((f"pol-{int(rng.integers(0, 40))}", rules))
    e = ext.DescheduleEnforcer(ctx, 8330, nodes, metrics, strategies)
    assert len(e.groups) >= 3 and all(len(g) <= 64 for g in e.groups)
    for g in e.groups:  # whole names per group
        assert not ({e.names[j] for j in g} & {e.names[j] for h in e.groups if h is not g
                                                 for j in h})
    node_labels = [{nm: "violating" for nm in set(e.names) if rng.random() < 0.3}
                   for _ in nodes]
    total, bodies = e.enforce(node_labels)
    viol = oracle.tas_violations(v, pres, e.rules, e.rule_off)
    want_total, want_ops = _update_node_labels(e.names, unpack_bits(viol, n_nodes), node_labels)
    assert total == want_total
    for i, nd in enumerate(nodes):
        got = sorted((o["op"], o["path"][len("/metadata/labels/"):], o["value"])
                     for o in json.loads(bodies[nd]))
        assert got == want_ops[i], nd


def test_gas_filter_unknown_kind(ctx):
    # a request for a gpu.intel.com/ kind no node has (scheduler.go:206-215, 349-354): with
    # an i915 in the same container every node fails; without one it fits with no cards
    names, nodes = gas_cluster()
    kinds = ["gpu.intel.com/i915", "gpu.intel.com/memory.max"]
    n_cards, cap, used, card_names = sn.gas_snapshot_from_nodes(nodes, kinds)
    ctx.gas_snapshot_set(8400, n_cards, cap, used)
    g = ext.GASExtender(ctx, 8400, names, card_names, kinds)

    def filt(requests):
        pod = {"metadata": {"name": "u", "namespace": "default"},
               "spec": {"containers": [{"resources": {"requests": r}} for r in requests]}}
        status, out = g.filter(json.dumps({"Pod": pod, "NodeNames": names}).encode())
        assert status == 200
        return json.loads(out)["NodeNames"]

    assert filt([{"gpu.intel.com/i915": "1", "gpu.intel.com/tiles": "1"}]) is None
    assert filt([{"gpu.intel.com/tiles": "1"}, {"gpu.intel.com/i915": "1"}]) == ["node-1"]
    assert filt([{"gpu.intel.com/i915": "1", "gpu.intel.com/memory.max": "1G"},
                 {"gpu.intel.com/i915": "1", "gpu.intel.com/foo": "0"}]) is None


def _tas2(ctx, metrics, policies, gen):
    """Two cached metrics: dummyMetric1 on both nodes, emptyMetric cached with no node."""
    names = ["node A", "node B"]
    v, pres, scale = sn.tas_snapshot_from_metrics(
        {"dummyMetric1": {k: str(x) for k, x in metrics.items()}, "emptyMetric": {}}, names,
        ["dummyMetric1", "emptyMetric"])
    ctx.tas_snapshot_set(gen, v, pres, scale)
    return ext.MetricsExtender(ctx, gen, names, ["dummyMetric1", "emptyMetric"], policies)


def test_filter_unknown_operator(ctx):
    """An unknown operator is never evaluated on an uncached metric or a metric cached with no
    node (dontschedule/strategy.go:27-36: ReadMetric error -> continue; an empty node map ->
    no EvaluateRule call), so the filter result is the other rules' one.  On a cached metric
    with nodes core.EvaluateRule calls a nil function (operator.go:13-26): the handler panics,
    net/http drops the connection — HandlerPanic, nothing written."""
    vals = {"node A": 50, "node B": 30}  # node A violates GreaterThan 40
    # NodeNames: strings.Split(availableNodeNames, " ") of "node B " (telemetryscheduler.go:213)
    want_failed, want_names = ["node A"], ["node", "B", ""]
    for gen, bad in enumerate([("absentMetric", "Foo", 1), ("emptyMetric", "greaterthan", 1)],
                              start=8500):
        pol = {("default", "test-policy"): {
            "scheduleonmetric": [("dummyMetric1", "GreaterThan", 0)],
            "dontschedule": [bad, ("dummyMetric1", "GreaterThan", 40)]}}
        m = _tas2(ctx, vals, pol, gen)
        status, body = m.filter(args(**TWO_NODES))
        assert status == 200
        res = json.loads(body)
        assert sorted(res["FailedNodes"]) == want_failed and res["NodeNames"] == want_names
        # prioritize never evaluates dontschedule rules
        assert m.prioritize(args(**TWO_NODES))[0] == 200
    pol = {("default", "test-policy"): {
        "scheduleonmetric": [("dummyMetric1", "GreaterThan", 0)],
        "dontschedule": [("dummyMetric1", "GreaterThan", 40), ("dummyMetric1", "Foo", 1)]}}
    m = _tas2(ctx, vals, pol, 8510)
    with pytest.raises(ext.HandlerPanic):
        m.filter(args(**TWO_NODES))
    # Violated runs before the empty-node-list check (telemetryscheduler.go:199-203)
    with pytest.raises(ext.HandlerPanic):
        m.filter(args({"telemetry-policy": "test-policy"}, []))
    # a scheduleonmetric rule with an unknown operator is not a panic: OrderedList leaves the
    # list unsorted (operator.go:30-42), request order here
    pol2 = {("default", "test-policy"): {"scheduleonmetric": [("dummyMetric1", "Foo", 0)]}}
    m2 = _tas2(ctx, vals, pol2, 8511)
    status, body = m2.prioritize(args(**TWO_NODES))
    assert status == 200
    assert [[h["Host"], h["Score"]] for h in json.loads(body)] == [["node A", 10], ["node B", 9]]


def test_deschedule_unknown_operator(ctx):
    """deschedule.Violated (deschedule/strategy.go:31-50) skips the same rules, and panics in
    the controller goroutine on a cached, non-empty metric."""
    names = ["node A", "node B"]
    v, pres, scale = sn.tas_snapshot_from_metrics(
        {"dummyMetric1": {"node A": "50", "node B": "30"}, "emptyMetric": {}}, names,
        ["dummyMetric1", "emptyMetric"])
    ctx.tas_snapshot_set(8520, v, pres, scale)
    strategies = [("pol-a", [("absentMetric", "Foo", 1), ("dummyMetric1", "GreaterThan", 40)]),
                  ("pol-b", [("emptyMetric", "Bar", 1)])]
    e = ext.DescheduleEnforcer(ctx, 8520, names, ["dummyMetric1", "emptyMetric"], strategies)
    total, bodies = e.enforce([{}, {}])
    # pol-a: node A violates; pol-b: nobody.  totalViolations counts the non-violated pairs
    assert total == 3
    assert json.loads(bodies["node A"]) == [
        {"op": "add", "path": "/metadata/labels/pol-a", "value": "violating"}]
    assert json.loads(bodies["node B"]) == []
    e2 = ext.DescheduleEnforcer(ctx, 8520, names, ["dummyMetric1", "emptyMetric"],
                                [("pol-c", [("dummyMetric1", "LessThen", 40)])])
    with pytest.raises(ext.HandlerPanic):
        e2.enforce([{}, {}])
