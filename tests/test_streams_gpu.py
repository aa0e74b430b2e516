"""One context, more streams than scratch slots (include/pas.h at PAS_STREAM_NULL; csrc
pas_api.hip aux_acquire): TAS evals and GAS fits issued round-robin on six streams without
host synchronisation, with growing batch sizes so that slots taken over from another stream
are also re-allocated.  A call on a stream whose slot another stream last used must wait for
that stream's queued work (an event) before reusing the slot's scratch; every result is
checked against the oracle."""
import numpy as np
import pytest

import pas_amd
from pas_amd import workload as wl

pytestmark = pytest.mark.gpu


def test_six_streams_tas_and_gas_on_one_context(oracle):
    import torch
    N = 4000
    tsnap = wl.make_tas_snapshot(N, 8, seed=0x61)
    gsnap = wl.make_gas_snapshot(N, seed=0x62)
    tb = [wl.make_tas_batch(tsnap, p, 6, seed=0x63 + i, cand_frac=0.9)
          for i, p in enumerate((64, 257, 700, 1300))]
    gb = [wl.make_gas_batch(p, seed=0x64 + i) for i, p in enumerate((50, 400, 1200, 2500))]
    c = pas_amd.Context(0)
    try:
        s0 = torch.cuda.current_stream()
        c.tas_snapshot_set_device(3, N, 8, torch.from_numpy(tsnap.v_milli).cuda(),
                                  torch.from_numpy(tsnap.present.view(np.int64)).cuda(), s0)
        c.gas_snapshot_set_device(4, N, gsnap.used.shape[1], gsnap.used.shape[2],
                                  torch.from_numpy(gsnap.n_cards).cuda(),
                                  torch.from_numpy(gsnap.cap).cuda(),
                                  torch.from_numpy(gsnap.used).cuda(), s0)
        streams = [torch.cuda.Stream() for _ in range(6)]
        for st in streams:
            st.wait_stream(s0)
        flags = pas_amd.PAS_TAS_FILTER | pas_amd.PAS_TAS_PRIORITIZE
        tas_out, gas_out = [], []
        k = 0
        for rep in range(3):
            for i in range(4):  # sizes grow within a rep: slots are re-allocated as they move
                st = streams[k % 6]
                k += 1
                b = tb[i]
                with torch.cuda.stream(st):
                    t = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in
                         (b.rules.view(np.uint8), b.rule_off, b.prio.view(np.uint8),
                          b.cand.view(np.int64))]
                    P = len(b.prio)
                    pt = torch.empty((P, pas_amd.w64(N)), dtype=torch.int64, device="cuda")
                    ot = torch.empty((P, N), dtype=torch.int32, device="cuda")
                    lt = torch.empty(P, dtype=torch.int32, device="cuda")
                c.tas_eval_device(3, P, len(b.rules), t[0], t[1], t[2], t[3], flags, pt, ot, lt,
                                  st)
                tas_out.append((i, t, pt, ot, lt))
                st = streams[k % 6]
                k += 1
                g = gb[i]
                with torch.cuda.stream(st):
                    req = torch.from_numpy(g.req).cuda()
                    mask = torch.from_numpy(g.req_mask.view(np.int32)).cuda()
                    nc = torch.from_numpy(g.n_containers).cuda()
                    res = torch.empty((len(g.n_containers), N), dtype=torch.int32,
                                      device="cuda")
                c.gas_fit_device(4, len(g.n_containers), g.req.shape[1], wl.I915, req, mask, nc,
                                 res, stream=st)
                gas_out.append((i, (req, mask, nc), res))
        torch.cuda.synchronize()
        want_t = [oracle.tas_eval(tsnap.v_milli, tsnap.present, b.rules, b.rule_off, b.prio,
                                  b.cand, 3) for b in tb]
        for i, _, pt, ot, lt in tas_out:
            wp, wo, wlen = want_t[i]
            np.testing.assert_array_equal(pt.cpu().numpy().view(np.uint64), wp)
            gl = lt.cpu().numpy()
            np.testing.assert_array_equal(gl, wlen)
            go = ot.cpu().numpy()
            for p in range(len(gl)):
                np.testing.assert_array_equal(go[p, :gl[p]], wo[p, :gl[p]])
        want_g = [oracle.gas_fit(gsnap.n_cards, gsnap.cap, gsnap.used, g.req, g.req_mask,
                                 g.n_containers, wl.I915) for g in gb]
        for i, _, res in gas_out:
            np.testing.assert_array_equal(res.cpu().numpy().view(np.uint32), want_g[i])
    finally:
        c.close()
