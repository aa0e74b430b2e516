"""Pins the CPU oracle (oracle/pas_oracle.c) to the reference's own test vectors and
e2e fixtures (tests/golden/reference_vectors.json).  CPU only."""
import numpy as np
import pytest

from helpers import OPS, NamedSnapshot, decode_gas_word, golden, unpack_bits

G = golden()


def test_g1_evaluate_rule(oracle):
    # telemetry-aware-scheduling/pkg/strategies/core/operator_test.go:33-38
    for c in G["G1_evaluate_rule"]["cases"]:
        got = oracle.evaluate_rule(c["value"] * 1000, OPS[c["operator"]], c["target"])
        assert got == int(c["want"]), c["name"]


def test_g1_unknown_operator_is_error(oracle):
    # operator.go:25 — a nil map entry; the reference panics
    assert oracle.evaluate_rule(1000, 7, 1) == -1


def test_evaluate_rule_exact_milli_and_saturation(oracle):
    # value 10.001 vs target 10: GreaterThan true, Equals false (CmpInt64 is exact)
    assert oracle.evaluate_rule(10001, OPS["GreaterThan"], 10) == 1
    assert oracle.evaluate_rule(10001, OPS["Equals"], 10) == 0
    assert oracle.evaluate_rule(9999, OPS["LessThan"], 10) == 1
    big = 2**63 - 1
    # targets whose *1000 exceeds int64: every value is LessThan, none GreaterThan/Equals
    assert oracle.evaluate_rule(big, OPS["LessThan"], big) == 1
    assert oracle.evaluate_rule(big, OPS["GreaterThan"], big) == 0
    assert oracle.evaluate_rule(-big - 1, OPS["GreaterThan"], -big - 1) == 1


def _prioritize(oracle, snap, named_rule, cand_names):
    prio = snap.rules([named_rule])
    rules = snap.rules([])
    rule_off = np.zeros(2, np.int32)
    _, order, lens = oracle.tas_eval(snap.v_milli, snap.present, rules, rule_off, prio,
                                     cand=snap.cand(cand_names), flags=2)
    return snap.names(order[0, : lens[0]])


def test_g2_ordered_list(oracle):
    g = G["G2_ordered_list"]
    snap = NamedSnapshot({"m": dict(zip(g["nodes"], g["values"]))})
    for c in g["cases"]:
        assert _prioritize(oracle, snap, ["m", c["operator"], 0], g["nodes"]) == c["want"]


def _violated(oracle, snap, named_rules):
    rules = snap.rules(named_rules)
    off = np.array([0, len(rules)], np.int32)
    viol = oracle.tas_violations(snap.v_milli, snap.present, rules, off)
    return sorted(snap.names(np.nonzero(unpack_bits(viol, len(snap.nodes))[0])[0]))


def test_g3_violated(oracle):
    g = G["G3_violated"]
    snap = NamedSnapshot(g["metrics"])
    for c in g["cases"]:
        assert _violated(oracle, snap, c["rules"]) == sorted(c["want"]), c["name"]


def apply_label_patch(labels: dict, body: bytes) -> dict:
    """JSON PATCH (RFC 6902) add/remove on /metadata/labels/<key>, as the API server applies
    the body of Deschedule.patchNode (enforce.go:74-86)."""
    import json
    out = dict(labels)
    for op in json.loads(body):
        prefix = "/metadata/labels/"
        assert op["path"].startswith(prefix)
        key = op["path"][len(prefix):]
        if op["op"] == "remove":
            assert key in out, "remove of a missing label fails the whole patch"
            del out[key]
        else:
            assert op["op"] == "add"
            out[key] = op["value"]
    return out


def test_g4_deschedule_enforce(oracle):
    g = G["G4_deschedule_enforce"]
    snap = NamedSnapshot(g["metrics"], g["nodes"])
    policy = g["policy"]
    for c in g["cases"]:
        assert _violated(oracle, snap, c["rules"]) == sorted(c["want"]), c["name"]
        rules = snap.rules(c["rules"])
        viol = oracle.tas_violations(snap.v_milli, snap.present, rules,
                                     np.array([0, len(rules)], np.int32))
        labels = np.zeros_like(viol)
        for i, node in enumerate(g["nodes"]):
            if policy in c["labels"]:  # every node of this fixture carries c["labels"]
                labels[0, i >> 6] |= np.uint64(1 << (i & 63))
        add, rem, total = oracle.label_plan(viol, labels, len(g["nodes"]))
        d = c["derived"]
        assert [policy] * int(add[0]) == d["add"] and [policy] * int(rem[0]) == d["remove"]
        assert total == d["total"], c["name"]
        body = oracle.label_patch_json([policy], add[0], rem[0])
        assert body.decode() == d["patch"], c["name"]
        # the reference's assertion: nodes listed by <policy>=violating after the patch
        after = apply_label_patch(c["labels"], body)
        got = [n for n in g["nodes"] if after.get(policy) == "violating"]
        assert got == c["want"], c["name"]


def g4n_inputs(oracle, case, snap, nodes):
    """(names, viol [S][W64], labels [S][W64]) of one G4n case: every strategy's labels row
    says whether the node carries the label of the strategy's policy name."""
    names = [s[0] for s in case["strategies"]]
    rules, off = [], [0]
    for _, named in case["strategies"]:
        rules.extend(snap.rules(named).tolist())
        off.append(len(rules))
    rules = np.array(rules, dtype=snap.rules([]).dtype)
    off = np.array(off, np.int32)
    viol = oracle.tas_violations(snap.v_milli, snap.present, rules, off)
    labels = np.zeros_like(viol)
    for j, name in enumerate(names):
        for i in range(len(nodes)):
            if name in case["labels"]:
                labels[j, i >> 6] |= np.uint64(1 << (i & 63))
    return names, rules, off, viol, labels


def test_g4n_shared_policy_name(oracle):
    """Strategies that share a policy name: remove / null and totalViolations per distinct
    name (enforce.go:89-134), one add per violating strategy (:108-117)."""
    g = G["G4n_shared_policy_name"]
    snap = NamedSnapshot(g["metrics"], g["nodes"])
    for c in g["cases"]:
        names, _, _, viol, labels = g4n_inputs(oracle, c, snap, g["nodes"])
        add, rem, total = oracle.label_plan(viol, labels, len(g["nodes"]), names)
        bits = lambda m: [s for s in range(len(names)) if int(m) >> s & 1]  # noqa: E731
        assert bits(add[0]) == c["add"] and bits(rem[0]) == c["remove"], c["name"]
        assert total == c["total"], c["name"]
        assert oracle.label_patch_json(names, add[0], rem[0]).decode() == c["patch"], c["name"]
        # the label ends "violating" exactly when some strategy of the name is violated
        after = apply_label_patch(c["labels"], oracle.label_patch_json(names, add[0], rem[0]))
        assert (after.get("p") == "violating") == bool(c["add"]), c["name"]


def _filter(oracle, snap, named_rules, nodes):
    rules = snap.rules(named_rules)
    off = np.array([0, len(rules)], np.int32)
    prio = snap.rules([["", "LessThan", 0]])
    pass_out, _, _ = oracle.tas_eval(snap.v_milli, snap.present, rules, off, prio,
                                     cand=snap.cand(nodes), flags=1)
    passed = unpack_bits(pass_out, len(snap.nodes))[0]
    return [n for n in nodes if passed[snap.node_index[n]]]


def test_g5_prioritize(oracle):
    g = G["G5_prioritize"]
    snap = NamedSnapshot(g["metrics"], g["nodes"])
    order = _prioritize(oracle, snap, g["policy"]["scheduleonmetric"][0], g["nodes"])
    assert [[h, 10 - i] for i, h in enumerate(order)] == g["want"]


def test_g6_prioritize_errors(oracle):
    for c in G["G6_prioritize_errors"]["cases"]:
        if c.get("decode_error") or not c["policy_cached"]:
            continue  # resolved before any metric is read (host shim)
        snap = NamedSnapshot(c["metrics"], c["nodes"])
        order = _prioritize(oracle, snap, ["dummyMetric1", "GreaterThan", 0], c["nodes"])
        assert [[h, 10 - i] for i, h in enumerate(order)] == c["want"], c["name"]


def test_g7_filter(oracle):
    g = G["G7_filter"]
    for c in g["cases"]:
        snap = NamedSnapshot(c["metrics"], g["nodes"])
        passed = _filter(oracle, snap, g["policy"]["dontschedule"], g["nodes"])
        failed = [n for n in g["nodes"] if n not in passed]
        assert failed == c["want_failed"], c["name"]
        assert passed == c["want_passed"], c["name"]
        # NodeNames = strings.Split("<passed names, each + ' '>", " ") (:209-212)
        assert "".join(n + " " for n in passed).split(" ") == c["want_node_names"], c["name"]


def test_g8_e2e(oracle):
    g = G["G8_e2e"]
    snap = NamedSnapshot(g["metrics"], g["nodes"])
    for c in g["filter_cases"]:
        assert _filter(oracle, snap, c["dontschedule"], g["nodes"]) == c["want_pass"], c["name"]
    for c in g["prioritize_cases"]:
        feasible = _filter(oracle, snap, c["dontschedule"], g["nodes"])
        order = _prioritize(oracle, snap, c["scheduleonmetric"][0], feasible)
        assert order[0] == c["want_first"]
        assert [[h, 10 - i] for i, h in enumerate(order)] == c["want_derived"]
    for c in g["deschedule_cases"]:
        assert _violated(oracle, snap, c["rules"]) == c["want"], c["name"]


def test_g9_resource_map(oracle):
    for c in G["G9_resource_map"]["cases"]:
        keys = sorted(set(c["start"]) | {k for op in c["ops"] for k in
                                         list(op.get("src", {})) + [op.get("key", "foo")]})
        m = oracle.rm(c["start"], keys)
        for op in c["ops"]:
            if op["op"] == "divide":
                err = oracle.load().or_rm_divide(m, op["arg"])
            elif op["op"] == "add":
                err = oracle.load().or_rm_add(m, keys.index(op["key"]), op["arg"])
            elif op["op"] == "subtract":
                err = oracle.load().or_rm_subtract(m, keys.index(op["key"]), op["arg"])
            elif op["op"] == "addRM":
                err = oracle.load().or_rm_add_rm(m, oracle.rm(op["src"], keys))
            else:
                err = oracle.load().or_rm_subtract_rm(m, oracle.rm(op["src"], keys))
            if op["want_err"] == "overflow":
                assert err == 2, (c["name"], op)
            else:
                assert bool(err) == op["want_err"], (c["name"], op)
            assert oracle.rm_dict(m, keys) == op["want"], (c["name"], op)


def test_g10_check_capacity_and_no_label(oracle):
    g = G["G10_gas_checks"]
    for c in g["check_capacity"]:
        keys = ["foo"]
        got = oracle.load().or_check_resource_capacity(
            oracle.rm(c["need"], keys), oracle.rm(c["capacity"], keys), oracle.rm(c["used"], keys))
        assert bool(got) == c["want"]
    # a node without the cards label never fits, even for a pod with no GPU request
    res = oracle.gas_fit(np.array([0], np.int32), np.zeros((1, 1), np.int64),
                         np.zeros((1, 1, 1), np.int64), np.zeros((1, 1, 1), np.int64),
                         np.zeros((1, 1), np.uint32), np.array([1], np.int32), 0)
    assert decode_gas_word(res[0, 0])[0] is g["no_label_node_fits"]


def gas_readme_case(example):
    """(n_cards, cap, used, req, mask) for a README example: one node, kinds in order."""
    kinds = list(example["allocatable"])
    cards = example["cards"]
    cap = np.array([[example["allocatable"][k] // len(cards) for k in kinds]], np.int64)
    used = np.zeros((1, len(cards), len(kinds)), np.int64)
    req = np.array([[[example["pod_request"].get(k, 0) for k in kinds]]], np.int64)
    mask = np.array([[sum(1 << i for i, k in enumerate(kinds) if k in example["pod_request"])]],
                    np.uint32)
    return kinds, cards, np.array([len(cards)], np.int32), cap, used, req, mask


def commit_pod(used_node, req_c, mask_c, cards_per_container):
    """Bind-time usage commit, as adjustPodResources (node_resource_cache.go:236-287):
    each container's request divided by its number of cards is added to every card."""
    for req, mask, cards in zip(req_c, mask_c, cards_per_container):
        if not cards:
            continue
        share = np.where([(mask >> q) & 1 for q in range(req.shape[0])], req // len(cards), 0)
        for k in cards:
            used_node[k] += share


def test_g11_gas_readme(oracle):
    g = G["G11_gas_readme"]
    for ex in (g["memory_example"], g["millicores_example"]):
        kinds, cards, n_cards, cap, used, req, mask = gas_readme_case(ex)
        for want in ex["want"]:
            res = oracle.gas_fit(n_cards, cap, used, req, mask, np.array([1], np.int32), 0)
            fits, sel = decode_gas_word(res[0, 0])
            assert fits == want["fits"]
            if fits:
                assert ",".join(cards[k] for k in sel) == want["annotation"]
                commit_pod(used[0], req[0], mask[0], [sel])


def test_unknown_kind_semantics(oracle):
    # runSchedulingLogic with a gpu.intel.com/ key no capacity map has (scheduler.go:206-215,
    # 341-383): numI915 > 0 -> checkResourceCapacity fails on every card -> errWontFit;
    # numI915 == 0 -> no selection, the pod fits with an empty annotation segment
    unk = 0x80000000
    n_cards = np.array([2], np.int32)
    cap = np.array([[4, 1000]], np.int64)
    used = np.zeros((1, 2, 2), np.int64)
    req = np.array([[[1, 10]], [[0, 10]], [[1, 10]]], np.int64)
    mask = np.array([[3 | unk], [2 | unk], [3]], np.uint32)
    got = oracle.gas_fit(n_cards, cap, used, req, mask, np.ones(3, np.int32), 0)
    assert [int(w) >> 31 for w in got[:, 0]] == [0, 1, 1]
    assert int(got[1, 0]) == 0x80000000  # fits, no cards
