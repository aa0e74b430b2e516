"""Host-side snapshot builders: the reference's cache contents in the
layouts of pas_tas_snapshot_set / pas_gas_snapshot_set.  This is the work the Go shim does once
per cache refresh; it is restated here so the whole path can be exercised from the
reference's own data shapes (metric maps of Quantity strings, node labels, usage maps).

TAS (cache/autoupdating.go:76-85, metrics/client.go:25-32): one column per metric name, one
row bit per node that has the metric, value * 10^scale exact (pas_quantity_to_scaled) with the
column's scale the most decimal places among its values (at least 3, milli): ParseQuantity
keeps at most 9, so every column is exact unless its range at that scale passes int64
(pas_tas_snapshot_set_scale).

GAS (gpuscheduler/scheduler.go:132-178, 269-275; node_resource_cache.go:474-491):
  cards      strings.Split(label "gpu.intel.com/cards", ".") -- duplicates and empty names
             included -- gives gpuCount; the cards a selection walks are the node's usage map
             keys plus the label cards (addEmptyResourceMaps), in sort.Strings order, minus
             cards not in the label (skipped as "vanished"): the sorted distinct label cards
  capacity   AsInt64 of every allocatable "gpu.intel.com/*" resource, divided by gpuCount
             (truncating); a kind the node does not advertise has capacity 0 (fails as missing)
  used       the usage map of each of those cards (a missing kind is 0)
  n_cards    number of those cards; 0 without the label (errWontFit, :290-298); -1 for a node
             the lister does not know (FetchNode error, :282-288)
"""
from __future__ import annotations

from typing import Dict, List, Mapping, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from .context import quantity_as_int64, quantity_decimals, quantity_to_scaled, w64

GPU_LIST_LABEL = "gpu.intel.com/cards"
RESOURCE_PREFIX = "gpu.intel.com/"


def tas_snapshot_from_metrics(metrics: Mapping[str, Mapping[str, str]],
                              node_names: Sequence[str],
                              metric_names: Optional[Sequence[str]] = None):
    """(v [M][N] int64, present [M][W64] uint64, scale [M] int32) from {metric: {node:
    quantity string}}: column m holds value * 10^scale[m] exactly, scale[m] the most decimal
    places among the column's values (pas_quantity_decimals; 3 for a column of milli-exact
    values or none), for Context.tas_snapshot_set(gen, v, present, scale).  Nodes not in
    node_names are ignored.  A column whose values need more range than int64 at that scale
    raises PasError(PAS_ENOTEXACT) naming the metric: no value is dropped."""
    metric_names = list(metrics) if metric_names is None else list(metric_names)
    index = {n: i for i, n in enumerate(node_names)}
    n, m = len(node_names), len(metric_names)
    v = np.zeros((m, n), np.int64)
    present = np.zeros((m, w64(n)), np.uint64)
    scale = np.full(m, 3, np.int32)
    for j, name in enumerate(metric_names):
        items = [(index[node], q) for node, q in metrics.get(name, {}).items() if node in index]
        k = max([quantity_decimals(q) for _, q in items], default=0)
        scale[j] = max(k, 3)  # milli unless a value needs more places
        for i, q in items:
            try:
                v[j, i] = quantity_to_scaled(q, int(scale[j]))
            except _lib.PasError as e:
                if e.code != _lib.PAS_ENOTEXACT:
                    raise
                raise _lib.PasError(e.code, f"metric {name!r}: {q!r} at 10^-{scale[j]} is "
                                            "outside int64") from None
            present[j, i >> 6] |= np.uint64(1 << (i & 63))
    return v, present, scale


def go_sort_strings(names):
    """sort.Strings: bytewise order of the UTF-8 encodings ("card10" < "card2")."""
    return sorted(names, key=lambda s: s.encode())


def gas_snapshot_from_nodes(nodes: Sequence[Optional[dict]], kinds: Sequence[str],
                            max_cards: int = _lib.PAS_GAS_MAX_CARDS):
    """(n_cards [N] int32, cap_per_gpu [N][Q] int64, used [N][K][Q] int64, card_names) from
    per-node dicts {"labels": {...}, "allocatable": {resource: quantity}, "usage":
    {card: {resource: int}}}, or None for a node the lister does not know.  card_names[n]
    lists the node's cards in rank order (rank = the 3-bit index in a pas_gas_fit word, or the
    byte of a pas_gas_selection record).  K is the largest card count of the nodes (at least
    1); a node with more than max_cards cards is PAS_ECAPACITY."""
    q = len(kinds)
    n = len(nodes)
    n_cards = np.zeros(n, np.int32)
    card_names: List[List[str]] = []
    for i, node in enumerate(nodes):
        labels = (node.get("labels") or {}) if node is not None else {}
        if node is None or GPU_LIST_LABEL not in labels:
            n_cards[i] = -1 if node is None else 0
            card_names.append([])
            continue
        cards = go_sort_strings(set(labels[GPU_LIST_LABEL].split(".")))
        if len(cards) > max_cards:
            raise _lib.PasError(_lib.PAS_ECAPACITY,
                                f"node {i}: {len(cards)} cards > {max_cards} (PAS_GAS_MAX_CARDS)")
        n_cards[i] = len(cards)
        card_names.append(cards)
    k = max([1] + [len(c) for c in card_names])
    cap = np.zeros((n, q), np.int64)
    used = np.zeros((n, k, q), np.int64)
    for i, node in enumerate(nodes):
        if n_cards[i] <= 0:
            continue
        gpu_count = len(node["labels"][GPU_LIST_LABEL].split("."))
        alloc = node.get("allocatable") or {}
        for j, kind in enumerate(kinds):
            if kind in alloc and kind.startswith(RESOURCE_PREFIX):
                # resourceMap.divide: Go integer division truncates toward zero
                value = quantity_as_int64(alloc[kind])
                share = abs(value) // gpu_count
                cap[i, j] = -share if value < 0 else share
        usage: Dict[str, Dict[str, int]] = node.get("usage") or {}
        for r, card in enumerate(card_names[i]):
            for j, kind in enumerate(kinds):
                used[i, r, j] = int(usage.get(card, {}).get(kind, 0))
    return n_cards, cap, used, card_names


def annotation(word: int, container_i915: Sequence[int], card_names: Sequence[str],
               selection=None) -> str:
    """The "gas-container-cards" annotation (scheduler.go:317-335) of a pas_gas_fit word:
    container c takes its next container_i915[c] selections; cards joined by ",", containers
    by "|".  A PAS_GAS_SEL_EXTENDED word needs its selection (the card ranks of its
    pas_gas_selection record, or of pas_gas_bind_ex)."""
    s_field = (int(word) >> 24) & 15
    if selection is not None:
        ranks = [int(r) for r in selection]
    elif s_field == _lib.PAS_GAS_SEL_EXTENDED:
        raise ValueError("PAS_GAS_SEL_EXTENDED word: pass its selection record")
    else:
        ranks = [(int(word) >> (3 * s)) & 7 for s in range(s_field)]
    out, pos = [], 0
    for n in container_i915:
        out.append(",".join(card_names[r] for r in ranks[pos:pos + n]))
        pos += n
    return "|".join(out)


def annotation_counts(counts, n_containers: int, card_names: Sequence[str]) -> str:
    """The "gas-container-cards" annotation from pas_gas_bind_counts' counts [C][K]: container
    c lists card k counts[c][k] times, in card order (its selections' order: first fit with
    one per-GPU request never returns to a card it has passed, scheduler.go:200-257)."""
    out = []
    for c in range(int(n_containers)):
        out.append(",".join(card_names[k] for k in range(len(card_names))
                            for _ in range(int(counts[c][k]))))
    return "|".join(out)
