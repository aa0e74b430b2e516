"""Diagnostic: C2 wall time per step with timing events off / span / per-kernel, and with
more steps (fixed per-run costs).  usage: python3 scripts/diag/tas_wall.py"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "platform-aware-scheduling_amd"))
import pas_amd  # noqa: E402
from pas_amd import _lib, workload as wl  # noqa: E402


def main():
    P, N, M, R = 4096, 100_000, 64, 15
    ctx = pas_amd.Context(0)
    if os.environ.get("PAS_DIAG_STREAM") == "torch":  # bench.py's setup: a torch stream
        torch.cuda.set_stream(torch.cuda.Stream())
    stream = torch.cuda.current_stream()
    print("stream handle", stream.cuda_stream, flush=True)
    ctx.set_stream(stream)
    snap = wl.make_tas_snapshot(N, M, seed=0xC2)
    batch = wl.make_tas_batch(snap, P, R, seed=0xC2)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    ctx.tas_snapshot_set_device(1, N, M, d(snap.v_milli), d(snap.present.view(np.int64)), stream)
    rules_t, off_t, prio_t = d(batch.rules.view(np.uint8)), d(batch.rule_off), d(batch.prio.view(np.uint8))
    pass_t = torch.empty((P, pas_amd.w64(N)), dtype=torch.int64, device="cuda")
    order_t = torch.empty((P, N), dtype=torch.int32, device="cuda")
    len_t = torch.empty(P, dtype=torch.int32, device="cuda")
    flags = pas_amd.PAS_TAS_FILTER | pas_amd.PAS_TAS_PRIORITIZE

    def step():
        ctx.tas_eval_device(1, P, len(batch.rules), rules_t, off_t, prio_t, None, flags, pass_t,
                            order_t, len_t, stream)

    for _ in range(5):
        step()
    for rep in range(2):
        for timing in (0, 1):
            for steps in (20, 100):
                ctx.reset_timing()
                ctx.set_timing(timing)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps):
                    step()
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / steps * 1e3
                ctx.set_timing(0)
                span, n = ctx.kernel_time(_lib.PAS_K_TAS_SPAN)
                print(f"rep {rep} timing {timing} steps {steps:3d}: wall {ms:.4f} ms/step"
                      + (f"  span {span / max(n, 1):.4f}" if n else ""), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
