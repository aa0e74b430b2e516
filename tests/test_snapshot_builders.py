"""Host snapshot builders (pas_amd/snapshot.py) checked against a literal
map-based restatement of the reference's GAS scheduling logic (gpuscheduler/scheduler.go:
132-338: label split, sort.Strings card order, vanished cards, per-GPU capacity, first fit with
accumulation) and against the README worked examples (G11).  The builder and the restatement
run on CPU; the GPU test runs the device fit on the built snapshot."""
import numpy as np
import pytest

import pas_amd
from pas_amd import snapshot as sn
from helpers import golden

G = golden()
I915 = "gpu.intel.com/i915"
MC = "gpu.intel.com/millicores"
MEM = "gpu.intel.com/memory.max"
KINDS = [I915, MC, MEM]


def go_div(v, d):
    q = abs(v) // d
    return -q if v < 0 else q


def check_capacity(need, capacity, used):
    """checkResourceCapacity (scheduler.go:341-383) over maps."""
    for res, n in need.items():
        if n < 0:
            return False
        c = capacity.get(res, 0)
        if c <= 0:
            return False
        u = used.get(res, 0)
        if u < 0:
            return False
        s = u + n
        if s > 2**63 - 1:
            return False
        if c < s:
            return False
    return True


def run_scheduling_logic(node, pod):
    """runSchedulingLogic (scheduler.go:280-338) on maps; returns the annotation or None."""
    if node is None:
        return None
    labels = node.get("labels") or {}
    if "gpu.intel.com/cards" not in labels:
        return None
    gpus = labels["gpu.intel.com/cards"].split(".")
    cap = {r: go_div(pas_amd.quantity_as_int64(q), len(gpus))
           for r, q in (node.get("allocatable") or {}).items() if r.startswith("gpu.intel.com/")}
    used = {c: dict(m) for c, m in (node.get("usage") or {}).items()}
    for g in gpus:
        used.setdefault(g, {})
    gpu_map = set(gpus)
    parts = []
    for req in pod:
        cards = []
        if req:
            per = dict(req)
            num = req.get(I915, 0) if req.get(I915, 0) > 0 else 0
            if num > 1:
                per = {r: go_div(v, num) for r, v in per.items()}
            for _ in range(num):
                fitted = False
                for name in sorted(used, key=lambda s: s.encode()):
                    if name not in gpu_map:
                        continue
                    if check_capacity(per, cap, used[name]):
                        for r, v in per.items():
                            used[name][r] = used[name].get(r, 0) + v
                        fitted = True
                        cards.append(name)
                        break
                if not fitted:
                    return None
        parts.append(",".join(cards))
    return "|".join(parts)


def random_cluster(rng, n):
    nodes = []
    for i in range(n):
        r = rng.random()
        if r < 0.05:
            nodes.append(None)  # not in the lister
            continue
        node = {"labels": {}, "allocatable": {}, "usage": {}}
        if r > 0.1:
            k = int(rng.integers(1, 6))
            names = ["card%d" % int(x) for x in rng.choice(12, size=k, replace=False)]
            if rng.random() < 0.2:
                names.append(names[0])  # duplicate in the label: counts in gpuCount
            node["labels"]["gpu.intel.com/cards"] = ".".join(names)
            node["allocatable"] = {I915: str(int(rng.integers(0, 4)) * len(names)),
                                   MC: str(1000 * len(names)),
                                   MEM: "%dGi" % (16 * len(names))}
            for c in set(names) | {"card99"}:  # card99: stale usage, not in the label
                node["usage"][c] = {I915: int(rng.integers(0, 3)),
                                    MC: int(rng.integers(0, 900)),
                                    MEM: int(rng.integers(0, 8 << 30))}
        nodes.append(node)
    return nodes


def random_pods(rng, p):
    pods = []
    for _ in range(p):
        pod = []
        for _ in range(int(rng.integers(1, 4))):
            if rng.random() < 0.1:
                pod.append({})  # a container without GPU resources
                continue
            pod.append({I915: int(rng.integers(0, 3)), MC: int(rng.integers(10, 700)),
                        MEM: int(rng.integers(1 << 28, 9 << 30))})
        pods.append(pod)
    return pods


def pack_pods(pods, c_max):
    p = len(pods)
    req = np.zeros((p, c_max, len(KINDS)), np.int64)
    mask = np.zeros((p, c_max), np.uint32)
    ncont = np.zeros(p, np.int32)
    for i, pod in enumerate(pods):
        ncont[i] = len(pod)
        for c, r in enumerate(pod):
            for j, kname in enumerate(KINDS):
                if kname in r:
                    req[i, c, j] = r[kname]
                    mask[i, c] |= 1 << j
    return req, mask, ncont


def container_i915(pod):
    return [r.get(I915, 0) if r.get(I915, 0) > 0 else 0 for r in pod]


def test_card_order_and_capacity_quirks():
    nodes = [{"labels": {"gpu.intel.com/cards": "card2.card10.card1"},
              "allocatable": {I915: "3", MC: "3000"},
              "usage": {"card10": {MC: 5}, "card7": {MC: 9}}},
             {"labels": {"gpu.intel.com/cards": "card0.card0"}, "allocatable": {MC: "1001"}},
             {"labels": {}}, None]
    n_cards, cap, used, names = sn.gas_snapshot_from_nodes(nodes, KINDS)
    assert names[0] == ["card1", "card10", "card2"]  # sort.Strings: "card10" < "card2"
    assert list(n_cards) == [3, 1, 0, -1]
    assert cap[0].tolist() == [1, 1000, 0]
    assert cap[1].tolist() == [0, 500, 0]  # "card0.card0": gpuCount 2, one distinct card
    assert used[0, 1].tolist() == [0, 5, 0]  # card10's usage; stale card7 is not a card


def test_builder_matches_map_restatement(oracle):
    rng = np.random.default_rng(5)
    nodes = random_cluster(rng, 120)
    pods = random_pods(rng, 40)
    n_cards, cap, used, names = sn.gas_snapshot_from_nodes(nodes, KINDS)
    req, mask, ncont = pack_pods(pods, 3)
    res = oracle.gas_fit(n_cards, cap, used, req, mask, ncont, 0)
    for p, pod in enumerate(pods):
        for n, node in enumerate(nodes):
            want = run_scheduling_logic(node, pod)
            word = int(res[p, n])
            if want is None:
                assert not (word >> 31), (p, n)
            else:
                assert word >> 31, (p, n)
                assert sn.annotation(word, container_i915(pod), names[n]) == want, (p, n)


def test_tas_builder_exactness():
    metrics = {"m1": {"a": "1.5", "b": "2", "zz": "7"}, "m2": {"b": "1m", "a": "0.0001"},
               "m4": {"a": "1e-7", "b": "1500u"}, "m5": {"a": "9e15"}}
    v, pres, scale = sn.tas_snapshot_from_metrics(metrics, ["a", "b"],
                                                  ["m1", "m2", "m3", "m4", "m5"])
    # milli unless a value needs more places: every value kept, exactly
    assert scale.tolist() == [3, 4, 3, 7, 3]
    assert v[0].tolist() == [1500, 2000] and v[1].tolist() == [1, 10]
    assert v[3].tolist() == [1, 15000] and v[4, 0] == 9 * 10**18
    assert int(pres[0, 0]) == 0b11 and int(pres[1, 0]) == 0b11 and int(pres[2, 0]) == 0
    # a column that needs both 7 places and 1e12: outside int64 at 10^-7 -> named error
    with pytest.raises(pas_amd.PasError) as e:
        sn.tas_snapshot_from_metrics({"big": {"a": "1e-7", "b": "1e12"}}, ["a", "b"])
    assert e.value.code == pas_amd._lib.PAS_ENOTEXACT and "big" in str(e.value)


@pytest.mark.gpu
def test_device_fit_on_built_snapshot(ctx):
    rng = np.random.default_rng(6)
    nodes = random_cluster(rng, 300)
    pods = random_pods(rng, 64)
    n_cards, cap, used, names = sn.gas_snapshot_from_nodes(nodes, KINDS)
    req, mask, ncont = pack_pods(pods, 3)
    ctx.gas_snapshot_set(9900, n_cards, cap, used)
    res = ctx.gas_fit(9900, req, mask, ncont, 0)
    for p, pod in enumerate(pods):
        for n, node in enumerate(nodes):
            want = run_scheduling_logic(node, pod)
            word = int(res[p, n])
            assert bool(word >> 31) == (want is not None), (p, n)
            if want is not None:
                assert sn.annotation(word, container_i915(pod), names[n]) == want, (p, n)
