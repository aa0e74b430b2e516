"""Diagnostic: GAS fit span time per selection count S on the C3 snapshot (50k nodes x 8
cards).  For each S a batch of P pods that all have S selections, in two shapes:
  split: one container asking i915 = S (S identical per-GPU selections)
  cont:  S containers asking i915 = 1 each (distinct needs)
prints us per 1000 pods.  usage: python3 scripts/diag/gas_mix.py [P]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# PAS_DIAG_PKG: a copy of the package whose lib/libpas.so is an A/B build
sys.path.insert(0, os.environ.get("PAS_DIAG_PKG", os.path.join(ROOT, "platform-aware-scheduling_amd")))
import pas_amd  # noqa: E402
from pas_amd import _lib, workload as wl  # noqa: E402


def batch(P, S, shape, rng, C=8):
    req = np.zeros((P, C, 3), np.int64)
    mask = np.zeros((P, C), np.uint32)
    nc = np.zeros(P, np.int32)
    if shape == "split":
        nc[:] = 1
        req[:, 0, 0] = S
        req[:, 0, 1] = rng.integers(10, 600, P) * max(S, 1)
        req[:, 0, 2] = rng.integers(100_000_000, 8_000_000_000, P) * max(S, 1)
        mask[:, 0] = 0b111 if S > 0 else 0b110
    else:
        nc[:] = max(S, 1)
        for c in range(max(S, 1)):
            req[:, c, 0] = 1 if S > 0 else 0
            req[:, c, 1] = rng.integers(10, 600, P)
            req[:, c, 2] = rng.integers(100_000_000, 8_000_000_000, P)
            mask[:, c] = 0b111 if S > 0 else 0b110
    return req, mask, nc


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    N = 50_000
    dev = torch.device("cuda", 0)
    ctx = pas_amd.Context(0)
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream)
    snap = wl.make_gas_snapshot(N, seed=0xC3)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    ctx.gas_snapshot_set_device(1, N, 8, 3, t(snap.n_cards), t(snap.cap), t(snap.used), stream)
    rng = np.random.default_rng(5)
    res = torch.empty((P, N), dtype=torch.int32, device=dev)
    smax = int(os.environ.get("PAS_DIAG_SMAX", "8"))
    cases = [("real", None)] + [(sh, s) for s in range(1, smax + 1) for sh in ("split", "cont")]
    only = os.environ.get("PAS_DIAG_ONLY")  # e.g. "split:2"
    if only:
        sh, sv = only.split(":")
        cases = [(sh, int(sv) if sv != "None" else None)]
    for shape, S in cases:
        if shape == "real":
            b = wl.make_gas_batch(P, seed=3, max_containers=8)
            req, mask, nc = b.req, b.req_mask, b.n_containers
        else:
            req, mask, nc = batch(P, S, shape, rng)
        rt, mt, nt = t(req), t(mask.view(np.int32)), t(nc)
        for _ in range(2):
            ctx.gas_fit_device(1, P, req.shape[1], wl.I915, rt, mt, nt, res, stream)
        torch.cuda.synchronize()
        ctx.reset_timing()
        ctx.set_timing(1)
        for _ in range(5):
            ctx.gas_fit_device(1, P, req.shape[1], wl.I915, rt, mt, nt, res, stream)
        torch.cuda.synchronize()
        ctx.set_timing(0)
        ms, n = ctx.kernel_time(_lib.PAS_K_GAS_FIT)
        fit = float((res.cpu().numpy().view(np.uint32) >> 31).mean())
        print(f"{shape:5s} S={S}  fit span {ms / n * 1e3:8.1f} us  "
              f"{ms / n * 1e3 / P * 1000:8.1f} us/1000 pods  fit={fit:.3f}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
