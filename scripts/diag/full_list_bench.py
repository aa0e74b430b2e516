#!/usr/bin/env python3
"""Diagnostic: full-list prioritize over S node shards on one GPU (C2 shape by default).

S contexts each hold one node shard of the C2 snapshot (node_range); per step every shard
writes its whole-shard records (pas_tas_topk_device with k = the widest shard) and one
context merges the S runs into the cluster lists (pas_list_merge_device) — the work one
rank does for all pods when the all-to-all is left out.  Prints per-phase GPU ms (HIP events
on the launch stream), the merge's algorithmic bytes per second, and checks a sample of pods
against the single-context full list (pas_tas_eval_device over the whole snapshot).

usage: full_list_bench.py [--pods 4096] [--nodes 100000] [--shards 8] [--steps 10]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "platform-aware-scheduling_amd"))

import pas_amd  # noqa: E402
from pas_amd import workload as wl  # noqa: E402
from pas_amd.shard import node_range  # noqa: E402


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=4096)
    ap.add_argument("--nodes", type=int, default=100_000)
    ap.add_argument("--metrics", type=int, default=64)
    ap.add_argument("--rules", type=int, default=16)
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    P, N, M, S = a.pods, a.nodes, a.metrics, a.shards
    snap = wl.make_tas_snapshot(N, M, seed=0xC2)
    batch = wl.make_tas_batch(snap, P, a.rules - 1, seed=0xC2)
    stream = torch.cuda.current_stream()
    rules_t = dev(batch.rules.view(np.uint8))
    off_t = dev(batch.rule_off)
    prio_t = dev(batch.prio.view(np.uint8))
    n_rules = len(batch.rules)
    a0, a1 = node_range(N, S, 0)
    w = a1 - a0
    ctxs = []
    for r in range(S):
        n0, n1 = node_range(N, S, r)
        c = pas_amd.Context(0)
        c.set_stream(stream)
        pres = np.unpackbits(snap.present.view(np.uint8), axis=1, bitorder="little")[:, n0:n1]
        sp = np.packbits(pres, axis=1, bitorder="little")
        sp = np.pad(sp, ((0, 0), (0, (-sp.shape[1]) % 8))).view(np.uint64)
        c.tas_snapshot_set(1, np.ascontiguousarray(snap.v_milli[:, n0:n1]), sp)
        ctxs.append((c, n0))
    keys = torch.empty((S, P, w), dtype=torch.int64, device="cuda")
    nodes = torch.empty((S, P, w), dtype=torch.int32, device="cuda")
    lens = torch.empty((S, P), dtype=torch.int32, device="cuda")
    out = torch.empty((P, S * w), dtype=torch.int32, device="cuda")
    out_len = torch.empty(P, dtype=torch.int32, device="cuda")

    def records():
        for r, (c, n0) in enumerate(ctxs):
            c.tas_topk_device(1, P, n_rules, rules_t, off_t, prio_t, None, w, n0, keys[r],
                              nodes[r], lens[r], stream)

    def merge():
        ctxs[0][0].list_merge_device(P, S, w, keys, nodes, out, out_len, stream=stream)

    for _ in range(2):
        records()
        merge()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    t_rec = t_merge = 0.0
    for _ in range(a.steps):
        ev[0].record(stream)
        records()
        ev[1].record(stream)
        merge()
        ev[2].record(stream)
        torch.cuda.synchronize()
        t_rec += ev[0].elapsed_time(ev[1])
        t_merge += ev[1].elapsed_time(ev[2])
    t_rec /= a.steps
    t_merge /= a.steps
    total = int(out_len.sum().item())
    # merge traffic: round 0 reads the S real runs, each later round reads what the one before
    # wrote (12 B per record of the padded rows); the last round writes 4-B node ids
    rounds = max(1, (S - 1).bit_length())
    rows = P * (1 << (S - 1).bit_length()) * w
    merge_bytes = 12 * P * S * w + 24 * rows * (rounds - 1) + 4 * P * S * w
    # single-context reference lists for a sample of pods
    ref = pas_amd.Context(0)
    ref.tas_snapshot_set(2, snap.v_milli, snap.present)
    order = torch.empty((P, N), dtype=torch.int32, device="cuda")
    ln = torch.empty(P, dtype=torch.int32, device="cuda")
    pass_t = torch.empty((P, (N + 63) // 64), dtype=torch.int64, device="cuda")
    ref.tas_eval_device(2, P, n_rules, rules_t, off_t, prio_t, None, 3, pass_t, order, ln)
    ref.synchronize()
    ok = bool(torch.equal(ln, out_len))
    for p in range(0, P, max(1, P // 64)):
        m = int(ln[p])
        ok = ok and bool(torch.equal(order[p, :m], out[p, :m]))
    print(json.dumps({"pods": P, "nodes": N, "shards": S, "width": w, "records_ms": t_rec,
                      "merge_ms": t_merge, "list_entries": total,
                      "merge_GBps": merge_bytes / (t_merge / 1e3) / 1e9, "sample_equal": ok}))
    for c, _ in ctxs:
        c.close()
    ref.close()


if __name__ == "__main__":
    main()
