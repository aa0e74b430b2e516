"""Synthetic clusters for BASELINE.json's configs.

No datasets exist for this path, so every config is generated from a fixed seed:

* TAS (C1, C2, C4, C5): metric values uniform in [0, 100000.000] (milli units),
  5 % of entries drawn from 10 "popular" integer values per metric (ties, and targets
  for Equals rules), 1 % of (node, metric) entries absent.  dontschedule / deschedule
  rules pick a metric uniformly, an operator uniformly from {LessThan, GreaterThan,
  Equals}, and a target at a 0.3-0.7 % quantile (LessThan), 99.3-99.7 % (GreaterThan)
  or a popular value (Equals), so each rule is violated by ~0.5 % of nodes.
  scheduleonmetric: GreaterThan 45 %, LessThan 45 %, Equals 10 % (Equals takes the
  reference's unsorted branch, operator.go:35-40).
* GAS (C3): K = 8 cards card0..card7, Q = 3 kinds {i915, millicores, memory.max},
  per-GPU capacity 300 / 1000 / 16e9, usage uniform in [0, 90 %] of it, 2 % of nodes
  without the cards label; pods with 1-4 containers (70/15/10/5 %), i915 0/1/2
  (10/80/10 %), millicores 10-600, memory.max 1e8-8e9.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from .context import RULE_DTYPE, w64

LT, GT, EQ = 0, 1, 2
POPULAR = 10


@dataclass
class TasSnapshotData:
    v_milli: np.ndarray   # [M, N] int64
    present: np.ndarray   # [M, W64] uint64
    present_bool: np.ndarray  # [M, N] bool
    popular: np.ndarray   # [M, POPULAR] int64, integer units
    sorted_present: list  # per metric: ascending present values (milli)


@dataclass
class TasBatch:
    rules: np.ndarray     # RULE_DTYPE, dontschedule rules of all pods
    rule_off: np.ndarray  # [P+1] int32
    prio: np.ndarray      # [P] RULE_DTYPE, scheduleonmetric rule 0
    cand: Optional[np.ndarray] = None  # [P, W64] uint64 or None


def pack_bits(b: np.ndarray) -> np.ndarray:
    """bool [..., N] -> uint64 [..., W64], node n at bit n & 63 of word n >> 6."""
    b = np.asarray(b, dtype=bool)
    n = b.shape[-1]
    pad = w64(n) * 64 - n
    if pad:
        b = np.concatenate([b, np.zeros(b.shape[:-1] + (pad,), bool)], axis=-1)
    by = np.packbits(b.reshape(b.shape[:-1] + (-1, 8)), axis=-1, bitorder="little")
    return np.ascontiguousarray(by.reshape(b.shape[:-1] + (-1,))).view("<u8").reshape(
        b.shape[:-1] + (w64(n),))


def unpack_bits(words: np.ndarray, n: int) -> np.ndarray:
    words = np.ascontiguousarray(words, dtype="<u8")
    by = words.view(np.uint8).reshape(words.shape[:-1] + (-1,))
    bits = np.unpackbits(by, axis=-1, bitorder="little")
    return bits[..., :n].astype(bool)


def make_tas_snapshot(n_nodes: int, n_metrics: int, seed: int,
                      absent_frac: float = 0.01, popular_frac: float = 0.05) -> TasSnapshotData:
    rng = np.random.default_rng(seed)
    v = rng.integers(0, 100_000_000, size=(n_metrics, n_nodes), dtype=np.int64, endpoint=True)
    popular = rng.integers(0, 100_000, size=(n_metrics, POPULAR), dtype=np.int64, endpoint=True)
    pop_mask = rng.random((n_metrics, n_nodes)) < popular_frac
    pick = rng.integers(0, POPULAR, size=(n_metrics, n_nodes))
    pop_vals = np.take_along_axis(popular, pick, axis=1) * 1000
    v = np.where(pop_mask, pop_vals, v)
    present_bool = rng.random((n_metrics, n_nodes)) >= absent_frac
    # absent entries carry garbage on purpose: the device must never read them
    v = np.where(present_bool, v, np.int64(-7777777))
    sorted_present = [np.sort(v[m][present_bool[m]]) for m in range(n_metrics)]
    return TasSnapshotData(v, pack_bits(present_bool), present_bool, popular, sorted_present)


def _targets(snap: TasSnapshotData, metric: np.ndarray, op: np.ndarray,
             rng: np.random.Generator) -> np.ndarray:
    t = np.zeros(metric.shape[0], np.int64)
    for i, (m, o) in enumerate(zip(metric.tolist(), op.tolist())):
        sv = snap.sorted_present[m]
        if sv.size == 0:
            t[i] = 0
            continue
        if o == LT:
            q = rng.uniform(0.003, 0.007)
            t[i] = sv[int(q * (sv.size - 1))] // 1000
        elif o == GT:
            q = rng.uniform(0.993, 0.997)
            t[i] = sv[int(q * (sv.size - 1))] // 1000
        else:
            t[i] = snap.popular[m][rng.integers(0, POPULAR)]
    return t


def make_tas_batch(snap: TasSnapshotData, n_pods: int, rules_per_pod: int, seed: int,
                   cand_frac: Optional[float] = None) -> TasBatch:
    """Per pod: `rules_per_pod` dontschedule rules + one scheduleonmetric rule."""
    rng = np.random.default_rng(seed)
    m_total = snap.v_milli.shape[0]
    n_nodes = snap.v_milli.shape[1]
    nr = n_pods * rules_per_pod
    metric = rng.integers(0, m_total, size=nr).astype(np.int32)
    op = rng.integers(0, 3, size=nr).astype(np.int32)
    rules = np.zeros(nr, RULE_DTYPE)
    rules["metric"] = metric
    rules["op"] = op
    rules["target"] = _targets(snap, metric, op, rng)
    rule_off = (np.arange(n_pods + 1, dtype=np.int64) * rules_per_pod).astype(np.int32)
    prio = np.zeros(n_pods, RULE_DTYPE)
    prio["metric"] = rng.integers(0, m_total, size=n_pods)
    u = rng.random(n_pods)
    prio["op"] = np.where(u < 0.45, GT, np.where(u < 0.90, LT, EQ))
    prio["target"] = 0
    cand = None
    if cand_frac is not None:
        cand = pack_bits(rng.random((n_pods, n_nodes)) < cand_frac)
    return TasBatch(rules, rule_off, prio, cand)


def make_deschedule_rules(snap: TasSnapshotData, n_strategies: int, rules_per_strategy: int,
                          seed: int):
    rng = np.random.default_rng(seed)
    m_total = snap.v_milli.shape[0]
    nr = n_strategies * rules_per_strategy
    # every column referenced once while there are columns left (C4: 64 rules over the 64
    # metrics, so a sweep reads 8 * M * N bytes of values)
    if nr <= m_total:
        metric = rng.permutation(m_total)[:nr].astype(np.int32)
    else:
        metric = rng.integers(0, m_total, size=nr).astype(np.int32)
    op = rng.integers(0, 3, size=nr).astype(np.int32)
    rules = np.zeros(nr, RULE_DTYPE)
    rules["metric"] = metric
    rules["op"] = op
    rules["target"] = _targets(snap, metric, op, rng)
    rule_off = (np.arange(n_strategies + 1) * rules_per_strategy).astype(np.int32)
    return rules, rule_off


# ---------------------------------------------------------------------------- GAS

GAS_KINDS = ("gpu.intel.com/i915", "gpu.intel.com/millicores", "gpu.intel.com/memory.max")
I915 = 0


@dataclass
class GasSnapshotData:
    n_cards: np.ndarray  # [N] int32
    cap: np.ndarray      # [N, Q] int64
    used: np.ndarray     # [N, K, Q] int64


@dataclass
class GasBatch:
    req: np.ndarray          # [P, C, Q] int64 (container totals, AsInt64 values)
    req_mask: np.ndarray     # [P, C] uint32
    n_containers: np.ndarray  # [P] int32


def make_gas_snapshot(n_nodes: int, seed: int, k: int = 8, no_label_frac: float = 0.02,
                      var_cards: bool = False) -> GasSnapshotData:
    rng = np.random.default_rng(seed)
    per_gpu = np.array([300, 1000, 16_000_000_000], np.int64)
    q = per_gpu.shape[0]
    n_cards = np.full(n_nodes, k, np.int32)
    if var_cards:
        n_cards = rng.integers(1, k + 1, size=n_nodes).astype(np.int32)
    n_cards[rng.random(n_nodes) < no_label_frac] = 0
    cap = np.tile(per_gpu, (n_nodes, 1))
    frac = rng.uniform(0.0, 0.9, size=(n_nodes, k, q))
    used = (frac * per_gpu[None, None, :]).astype(np.int64)
    used[np.arange(k)[None, :] >= n_cards[:, None]] = 0
    return GasSnapshotData(n_cards, cap, used)


def make_gas_batch(n_pods: int, seed: int, max_containers: int = 4) -> GasBatch:
    rng = np.random.default_rng(seed)
    q = len(GAS_KINDS)
    n_cont = rng.choice([1, 2, 3, 4], size=n_pods, p=[0.70, 0.15, 0.10, 0.05]).astype(np.int32)
    n_cont = np.minimum(n_cont, max_containers)
    req = np.zeros((n_pods, max_containers, q), np.int64)
    mask = np.zeros((n_pods, max_containers), np.uint32)
    ni = rng.choice([0, 1, 2], size=(n_pods, max_containers), p=[0.10, 0.80, 0.10])
    req[:, :, 0] = ni
    req[:, :, 1] = rng.integers(10, 600, size=(n_pods, max_containers), endpoint=True)
    req[:, :, 2] = rng.integers(100_000_000, 8_000_000_000, size=(n_pods, max_containers),
                                endpoint=True)
    mask[:] = 0b110 | np.where(ni > 0, 1, 0).astype(np.uint32)
    live = np.arange(max_containers)[None, :] < n_cont[:, None]
    mask[~live] = 0
    req[~live] = 0
    return GasBatch(req, mask, n_cont)
