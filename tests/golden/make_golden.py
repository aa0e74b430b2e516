#!/usr/bin/env python3
"""Writes tests/golden/reference_vectors.json: the reference's own test vectors and e2e
fixtures for the filter/prioritize/deschedule/GAS-fit path, transcribed as data.

The Go reference (Go 1.16 + k8s.io/apimachinery v0.22.2) cannot be built or run in
this image (no Go toolchain, no module cache), so parity is pinned on these vectors
(SURVEY.md Appendix B).  Each entry cites the reference file:line it was read from
(paths relative to the reference root).  Entries marked "derived" are outcomes the
reference test sets up but does not assert (it only checks wantErr); their expected
value is what the cited reference code returns for that input.
"""
import json
import os

V = {}

# G1 core.EvaluateRule (telemetry-aware-scheduling/pkg/strategies/core/operator_test.go:33-38)
V["G1_evaluate_rule"] = {
    "source": "telemetry-aware-scheduling/pkg/strategies/core/operator_test.go:33-38",
    "cases": [
        {"name": "LessThan true", "value": 100, "operator": "LessThan", "target": 1000, "want": True},
        {"name": "GreaterThan true", "value": 100000, "operator": "GreaterThan", "target": 1, "want": True},
        {"name": "Equals true", "value": 1, "operator": "Equals", "target": 1, "want": True},
        {"name": "LessThan false", "value": 10000, "operator": "LessThan", "target": 10, "want": False},
        {"name": "GreaterThan false", "value": 1, "operator": "GreaterThan", "target": 10000, "want": False},
        {"name": "Equals false", "value": 1, "operator": "Equals", "target": 100, "want": False},
    ],
}

# G2 core.OrderedList (operator_test.go:60-61)
V["G2_ordered_list"] = {
    "source": "telemetry-aware-scheduling/pkg/strategies/core/operator_test.go:60-61",
    "nodes": ["node A", "node B", "node C"],
    "values": [100, 200, 10],
    "cases": [
        {"operator": "LessThan", "want": ["node C", "node A", "node B"]},
        {"operator": "GreaterThan", "want": ["node B", "node A", "node C"]},
    ],
}

# G3 Violated (dontschedule/strategy_test.go:27-29, deschedule/strategy_test.go:100-102);
# cache: "memory" = {node-1: 10} (strategy_test.go:33 / :106)
V["G3_violated"] = {
    "source": ["telemetry-aware-scheduling/pkg/strategies/dontschedule/strategy_test.go:27-33",
               "telemetry-aware-scheduling/pkg/strategies/deschedule/strategy_test.go:100-106"],
    "metrics": {"memory": {"node-1": 10}},
    "cases": [
        {"name": "One node violating", "rules": [["memory", "GreaterThan", 9]], "want": ["node-1"]},
        {"name": "No nodes violating", "rules": [["memory", "GreaterThan", 11]], "want": []},
        {"name": "No metric found", "rules": [["mem", "GreaterThan", 9]], "want": []},
    ],
}

# G4 deschedule Enforce (deschedule/enforce_test.go:38-52)
V["G4_deschedule_enforce"] = {
    "source": "telemetry-aware-scheduling/pkg/strategies/deschedule/enforce_test.go:38-52",
    "metrics": {"memory": {"node-1": 100}},
    "nodes": ["node-1"],
    "policy": "deschedule-test",
    # "labels": node-1's labels before Enforce (enforce_test.go:40, :46); "want" = nodes
    # listed by deschedule-test=violating afterwards (:68-84).  The label plan and patch body
    # are derived (the test does not inspect them): updateNodeLabels (enforce.go:99-151) and
    # json.Marshal of patchValue (enforce.go:21-25, 74-86).
    "cases": [
        {"name": "node label test", "labels": {"deschedule-test": ""},
         "rules": [["memory", "GreaterThan", 1], ["cpu", "LessThan", 10]], "want": ["node-1"],
         "derived": {"add": ["deschedule-test"], "remove": [], "total": 0,
                     "patch": '[{"op":"add","path":"/metadata/labels/deschedule-test",'
                              '"value":"violating"}]'}},
        {"name": "node unlabel test", "labels": {"deschedule-test": "violating"},
         "rules": [["memory", "GreaterThan", 1000], ["cpu", "LessThan", 10]], "want": [],
         "derived": {"add": [], "remove": ["deschedule-test"], "total": 1,
                     "patch": '[{"op":"remove","path":"/metadata/labels/deschedule-test",'
                              '"value":""},{"op":"add","path":"/metadata/labels/'
                              'deschedule-test","value":"null"}]'}},
    ],
}

# G4n deschedule strategies that share a policy name (derived; no reference test covers it).
# SetPolicyName takes ObjectMeta.Name without the namespace (controller/controller.go:80), and
# AddStrategy drops only Equals duplicates: same name AND the same non-empty rules
# (core/enforcer.go:84-103, deschedule/strategy.go:60-78).  So policies "p" in two namespaces
# with different rules are two registered strategies named "p".  updateNodeLabels keys the
# non-violated set by NAME (allPolicies, enforce.go:89-95; delete(nonViolatedPolicies, name)
# per violating strategy, :108-109): a name is removed / counted once, and only when none of
# its strategies is violated (:118-134); each violating strategy appends its own "add" (:110-115).
# "strategies" lists (name, rules) in registration order; outcomes read off enforce.go:99-151.
_ADD_P = '{"op":"add","path":"/metadata/labels/p","value":"violating"}'
_REM_P = ('{"op":"remove","path":"/metadata/labels/p","value":""},'
          '{"op":"add","path":"/metadata/labels/p","value":"null"}')
V["G4n_shared_policy_name"] = {
    "source": ["telemetry-aware-scheduling/pkg/strategies/deschedule/enforce.go:89-134",
               "telemetry-aware-scheduling/pkg/strategies/core/enforcer.go:84-103",
               "telemetry-aware-scheduling/pkg/controller/controller.go:80"],
    "derived": True,
    "metrics": {"memory": {"node-1": 100}},
    "nodes": ["node-1"],
    "cases": [
        {"name": "one of two same-name strategies violating, node labelled",
         "strategies": [["p", [["memory", "GreaterThan", 1]]],
                        ["p", [["memory", "GreaterThan", 1000]]]],
         "labels": {"p": "violating"},
         "add": [0], "remove": [], "total": 0, "patch": "[" + _ADD_P + "]"},
        {"name": "violating strategy registered second",
         "strategies": [["p", [["memory", "GreaterThan", 1000]]],
                        ["p", [["memory", "GreaterThan", 1]]]],
         "labels": {"p": "null"},
         "add": [1], "remove": [], "total": 0, "patch": "[" + _ADD_P + "]"},
        {"name": "both same-name strategies violating: one add each",
         "strategies": [["p", [["memory", "GreaterThan", 1]]],
                        ["p", [["memory", "LessThan", 1000]]]],
         "labels": {},
         "add": [0, 1], "remove": [], "total": 0, "patch": "[" + _ADD_P + "," + _ADD_P + "]"},
        {"name": "neither violating: one remove pair, counted once",
         "strategies": [["p", [["memory", "GreaterThan", 1000]]],
                        ["p", [["memory", "LessThan", 1]]]],
         "labels": {"p": "violating"},
         "add": [], "remove": [0], "total": 1, "patch": "[" + _REM_P + "]"},
        {"name": "a second name, not violated and not carried, is counted",
         "strategies": [["p", [["memory", "GreaterThan", 1]]],
                        ["p", [["memory", "GreaterThan", 1000]]],
                        ["q", [["memory", "Equals", 7]]]],
         "labels": {"p": "violating"},
         "add": [0], "remove": [], "total": 1, "patch": "[" + _ADD_P + "]"},
    ],
}

# testPolicy1 (telemetryscheduler/scheduler_test.go:44-62)
TEST_POLICY1 = {
    "name": "test-policy", "namespace": "default",
    "scheduleonmetric": [["dummyMetric1", "GreaterThan", 0]],
    "dontschedule": [["dummyMetric1", "GreaterThan", 40]],
}

# G5/G6 Prioritize (telemetryscheduler/scheduler_test.go:166-200)
V["G5_prioritize"] = {
    "source": "telemetry-aware-scheduling/pkg/telemetryscheduler/scheduler_test.go:166-173",
    "policy": TEST_POLICY1,
    "metrics": {"dummyMetric1": {"node A": 100, "node B": 90}},
    "nodes": ["node A", "node B"],
    "want": [["node A", 10], ["node B", 9]],
}
V["G6_prioritize_errors"] = {
    "source": "telemetry-aware-scheduling/pkg/telemetryscheduler/scheduler_test.go:175-200",
    "cases": [
        {"name": "policy not found", "note": "pod label test-policy, only other-policy cached "
         "(scheduler_test.go:63-81) -> getPolicyFromPod error -> empty list "
         "(telemetryscheduler.go:82-86)", "policy_cached": False,
         "metrics": {"dummyMetric1": {"node A": 90, "node B": 100}},
         "nodes": ["node A", "node B"], "want": []},
        {"name": "cache returns error if empty (derived)", "note": "the test only checks "
         "wantErr; prioritizeNodesForRule over nodes [node A] with dummyMetric1 = {node A: 100} "
         "returns [{node A 10}] (telemetryscheduler.go:128-149)", "policy_cached": True,
         "metrics": {"dummyMetric1": {"node A": 100}}, "nodes": ["node A"],
         "want": [["node A", 10]]},
        {"name": "malformed arguments return error", "note": "extender.Args{} -> Nodes == nil "
         "-> decode error (telemetryscheduler.go:74-76) -> no body", "decode_error": True},
    ],
}

# G7 Filter (telemetryscheduler/scheduler_test.go:277-292); request nodes = twoNodeArgument
V["G7_filter"] = {
    "source": "telemetry-aware-scheduling/pkg/telemetryscheduler/scheduler_test.go:277-292",
    "policy": TEST_POLICY1,
    "nodes": ["node A", "node B"],
    # The test asserts FailedNodes only (:321-337).  Derived: the nodes kept, and NodeNames =
    # strings.Split(availableNodeNames, " ") (telemetryscheduler.go:209-212), which splits the
    # test's space-containing names.
    "cases": [
        {"name": "get and return node test", "metrics": {"dummyMetric1": {"node A": 10, "node B": 30}},
         "want_failed": [], "want_passed": ["node A", "node B"],
         "want_node_names": ["node", "A", "node", "B", ""]},
        {"name": "filter out one node", "metrics": {"dummyMetric1": {"node A": 50, "node B": 30}},
         "want_failed": ["node A"], "want_passed": ["node B"], "want_node_names": ["node", "B", ""]},
    ],
}

# G8 e2e fixtures: .github/scripts/policies/node{1,2,3} mounted on kind-worker, -2, -3
# (.github/scripts/e2e_setup_cluster.sh:54-68); policies .github/e2e/e2e_test.go:82-85,290-317
V["G8_e2e"] = {
    "source": [".github/scripts/policies/node1", ".github/scripts/policies/node2",
               ".github/scripts/policies/node3", ".github/e2e/e2e_test.go:82-85,95-96,132,167,290-317"],
    "nodes": ["kind-worker", "kind-worker2", "kind-worker3"],
    "metrics": {
        "filter1_metric": {"kind-worker": 10, "kind-worker2": 20, "kind-worker3": 10},
        "filter2_metric": {"kind-worker": 0, "kind-worker2": 0, "kind-worker3": 0},
        "prioritize1_metric": {"kind-worker": 1000, "kind-worker2": 9999, "kind-worker3": 0},
        "deschedule1_metric": {"kind-worker2": 9},
    },
    "filter_cases": [
        {"name": "Filter all but one node", "dontschedule": [["filter1_metric", "LessThan", 20]],
         "want_pass": ["kind-worker2"]},
        {"name": "Filter all nodes", "dontschedule": [["filter2_metric", "Equals", 0]],
         "want_pass": []},
    ],
    "prioritize_cases": [
        {"name": "Prioritize to highest score node",
         "scheduleonmetric": [["prioritize1_metric", "GreaterThan", 0]],
         "dontschedule": [["filter1_metric", "Equals", 2000000]],
         "want_first": "kind-worker2",
         "want_derived": [["kind-worker2", 10], ["kind-worker", 9], ["kind-worker3", 8]]},
    ],
    "deschedule_cases": [
        {"name": "Label node for deschedule", "rules": [["deschedule1_metric", "GreaterThan", 8]],
         "want": ["kind-worker2"]},
    ],
}

# G9 resourceMap arithmetic (gpu-aware-scheduling/pkg/gpuscheduler/resource_map_test.go:16-119).
# Each case is a sequence of operations on one map, as the goconvey blocks run in order.
INT64_MAX = 9223372036854775807
V["G9_resource_map"] = {
    "source": "gpu-aware-scheduling/pkg/gpuscheduler/resource_map_test.go:16-119",
    "cases": [
        {"name": "TestDivision", "start": {"foo": 2}, "ops": [
            {"op": "divide", "arg": -1, "want_err": True, "want": {"foo": 2}},
            {"op": "divide", "arg": 1, "want_err": False, "want": {"foo": 2}},
            {"op": "divide", "arg": 2, "want_err": False, "want": {"foo": 1}}]},
        {"name": "TestAdd", "start": {"foo": 2}, "ops": [
            {"op": "add", "key": "foo", "arg": INT64_MAX - 2, "want_err": False, "want": {"foo": INT64_MAX}},
            {"op": "add", "key": "foo", "arg": 1, "want_err": "overflow", "want": {"foo": INT64_MAX}}]},
        {"name": "TestSubtract", "start": {"foo": 2}, "ops": [
            {"op": "subtract", "key": "bar", "arg": 2, "want_err": True, "want": {"foo": 2}},
            {"op": "subtract", "key": "foo", "arg": 1, "want_err": False, "want": {"foo": 1}},
            {"op": "subtract", "key": "foo", "arg": 2, "want_err": False, "want": {"foo": 0}}]},
        {"name": "TestAddRM overflow", "start": {"foo": 4, "foo2": 5, "foo3": INT64_MAX}, "ops": [
            {"op": "addRM", "src": {"foo": 2, "foo2": 3, "foo3": INT64_MAX}, "want_err": "overflow",
             "want": {"foo": 4, "foo2": 5, "foo3": INT64_MAX}}]},
        {"name": "TestAddRM fits", "start": {"foo": 2, "foo2": 3}, "ops": [
            {"op": "addRM", "src": {"foo": 4, "foo2": 5, "foo3": INT64_MAX}, "want_err": False,
             "want": {"foo": 6, "foo2": 8, "foo3": INT64_MAX}}]},
        {"name": "TestSubtractRM", "start": {"foo": 4, "foo2": 5, "foo3": INT64_MAX}, "ops": [
            {"op": "subtractRM", "src": {"unknown": 2, "foo2": 3}, "want_err": True,
             "want": {"foo": 4, "foo2": 5, "foo3": INT64_MAX}},
            {"op": "subtractRM", "src": {"foo": 2, "foo2": 3, "foo3": INT64_MAX}, "want_err": False,
             "want": {"foo": 2, "foo2": 2, "foo3": 0}}]},
    ],
}

# G10 checkResourceCapacity with empty capacity (scheduler_test.go:122-131) and nodes
# without the cards label (scheduler_test.go:225-236 -> getNodeGPUList nil -> errWontFit,
# scheduler.go:290-298)
V["G10_gas_checks"] = {
    "source": ["gpu-aware-scheduling/pkg/gpuscheduler/scheduler_test.go:122-131",
               "gpu-aware-scheduling/pkg/gpuscheduler/scheduler_test.go:225-236"],
    "check_capacity": [{"need": {"foo": 1}, "capacity": {}, "used": {}, "want": False}],
    "no_label_node_fits": False,
}

# G11 GAS README worked examples (gpu-aware-scheduling/README.md:15-21)
V["G11_gas_readme"] = {
    "source": "gpu-aware-scheduling/README.md:15-21",
    "memory_example": {
        "note": "2 GPUs, 16 GB advertised -> 8 GB per GPU; three pods of 5 GB bound in turn",
        "cards": ["card0", "card1"],
        "allocatable": {"gpu.intel.com/i915": 2, "gpu.intel.com/memory.max": 16000000000},
        "pod_request": {"gpu.intel.com/i915": 1, "gpu.intel.com/memory.max": 5000000000},
        "want": [{"fits": True, "annotation": "card0"}, {"fits": True, "annotation": "card1"},
                 {"fits": False}],
    },
    "millicores_example": {
        "note": "i915 = 2, millicores = 2000, per-GPU capacity 1000 -> 1000 on each of two GPUs",
        "cards": ["card0", "card1"],
        "allocatable": {"gpu.intel.com/i915": 2, "gpu.intel.com/millicores": 2000},
        "pod_request": {"gpu.intel.com/i915": 2, "gpu.intel.com/millicores": 2000},
        "want": [{"fits": True, "annotation": "card0,card1"}],
    },
}

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_vectors.json")
    with open(out, "w") as f:
        json.dump(V, f, indent=1, sort_keys=True)
        f.write("\n")
    print("wrote", out)
