"""Shared test helpers: named (reference-style) fixtures -> packed C-ABI inputs."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
RULE_DTYPE = np.dtype([("metric", "<i4"), ("op", "<i4"), ("target", "<i8")], align=True)
OPS = {"LessThan": 0, "GreaterThan": 1, "Equals": 2}


def golden():
    with open(os.path.join(HERE, "golden", "reference_vectors.json")) as f:
        return json.load(f)


def w64(n):
    return (n + 63) // 64


def pack_bits(b):
    b = np.asarray(b, dtype=bool)
    n = b.shape[-1]
    out = np.zeros(b.shape[:-1] + (w64(n),), np.uint64)
    idx = np.nonzero(b)
    for pos in zip(*idx):
        *lead, nn = pos
        out[tuple(lead) + (nn >> 6,)] |= np.uint64(1) << np.uint64(nn & 63)
    return out


def unpack_bits(words, n):
    words = np.ascontiguousarray(words, dtype="<u8")
    by = words.view(np.uint8).reshape(words.shape[:-1] + (-1,))
    return np.unpackbits(by, axis=-1, bitorder="little")[..., :n].astype(bool)


class NamedSnapshot:
    """metrics {name: {node: integer value}} over a node list -> SoA int64 milli columns."""

    def __init__(self, metrics, nodes=()):
        self.nodes = list(nodes)
        for per_node in metrics.values():
            for node in per_node:
                if node not in self.nodes:
                    self.nodes.append(node)
        self.metric_names = list(metrics)
        self.metric_index = {m: i for i, m in enumerate(self.metric_names)}
        self.node_index = {n: i for i, n in enumerate(self.nodes)}
        m_cnt, n_cnt = max(len(self.metric_names), 1), len(self.nodes)
        self.v_milli = np.zeros((m_cnt, n_cnt), np.int64)
        pres = np.zeros((m_cnt, n_cnt), bool)
        for name, per_node in metrics.items():
            mi = self.metric_index[name]
            for node, v in per_node.items():
                self.v_milli[mi, self.node_index[node]] = int(v) * 1000
                pres[mi, self.node_index[node]] = True
        self.present_bool = pres
        self.present = pack_bits(pres)

    def rules(self, named_rules):
        r = np.zeros(len(named_rules), RULE_DTYPE)
        for i, (metric, op, target) in enumerate(named_rules):
            r[i]["metric"] = self.metric_index.get(metric, -1)
            r[i]["op"] = OPS.get(op, 99)
            r[i]["target"] = target
        return r

    def cand(self, names):
        b = np.zeros(len(self.nodes), bool)
        for n in names:
            b[self.node_index[n]] = True
        return pack_bits(b[None, :])

    def names(self, idx):
        return [self.nodes[i] for i in idx]


def decode_gas_word(word):
    """(fits, [card ranks]) from a pas_gas_fit result word."""
    word = int(word)
    fits = bool(word >> 31)
    nsel = (word >> 24) & 0xF
    return fits, [(word >> (3 * j)) & 7 for j in range(nsel)] if fits else []
