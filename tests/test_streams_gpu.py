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


@pytest.mark.parametrize("global_pass", [0, 1])
def test_six_streams_tas_and_gas_on_one_context(oracle, monkeypatch, global_pass):
    """global_pass = 1: the evals keep their pass bitmaps in global memory (the layout of
    clusters past ~1.1M nodes, PAS_EVAL_GLOBAL_PASS), one buffer per stream slot."""
    import torch
    monkeypatch.setenv("PAS_EVAL_GLOBAL_PASS", str(global_pass))
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


def test_request_prioritize_and_label_plan_on_four_streams(oracle):
    """pas_tas_prioritize_request_device and pas_tas_label_plan_device issued round-robin on
    four streams without host synchronisation (their workspaces are per-stream slot
    buffers, pas_internal.h SlotBuf), growing sizes so that buffers are re-allocated while
    other streams' calls are queued; every result against the oracle."""
    import torch
    N = 6000
    snap = wl.make_tas_snapshot(N, 8, seed=0x71)
    batch = wl.make_tas_batch(snap, 8, 4, seed=0x72)
    c = pas_amd.Context(0)
    try:
        s0 = torch.cuda.current_stream()
        c.tas_snapshot_set_device(5, N, 8, torch.from_numpy(snap.v_milli).cuda(),
                                  torch.from_numpy(snap.present.view(np.int64)).cuda(), s0)
        streams = [torch.cuda.Stream() for _ in range(4)]
        for st in streams:
            st.wait_stream(s0)
        rng = np.random.default_rng(0x73)
        prio_out, plan_out = [], []
        k = 0
        for rep in range(3):
            for n_req in (100, 900, 2500, N):
                st = streams[k % 4]
                k += 1
                req = rng.permutation(N).astype(np.int32)[:n_req]
                req[rng.random(n_req) < 0.05] = -1  # names the snapshot does not know
                prio = batch.prio[k % len(batch.prio)]
                with torch.cuda.stream(st):
                    req_t = torch.from_numpy(req).cuda()
                    pos_t = torch.empty(n_req, dtype=torch.int32, device="cuda")
                    len_t = torch.empty(1, dtype=torch.int32, device="cuda")
                c.tas_prioritize_request_device(5, prio, n_req, req_t, pos_t, len_t, stream=st)
                prio_out.append((prio, req, req_t, pos_t, len_t))
                st = streams[k % 4]
                k += 1
                n = n_req * 7 + 13
                s = 3 + rep * 5
                viol = wl.pack_bits(rng.random((s, n)) < 0.3)
                labels = wl.pack_bits(rng.random((s, n)) < 0.5)
                with torch.cuda.stream(st):
                    viol_t = torch.from_numpy(viol.view(np.int64)).cuda()
                    lab_t = torch.from_numpy(labels.view(np.int64)).cuda()
                    add_t = torch.empty(n, dtype=torch.int64, device="cuda")
                    rem_t = torch.empty(n, dtype=torch.int64, device="cuda")
                    tot_t = torch.empty(1, dtype=torch.int64, device="cuda")
                c.tas_label_plan_device(n, s, viol_t, lab_t, add_t, rem_t, tot_t, stream=st)
                plan_out.append((n, viol, labels, viol_t, lab_t, add_t, rem_t, tot_t))
        torch.cuda.synchronize()
        for prio, req, _, pos_t, len_t in prio_out:
            want = oracle.prioritize_request(snap.v_milli, snap.present, prio, req)
            L = int(len_t.item())
            np.testing.assert_array_equal(pos_t.cpu().numpy()[:L], want)
        for n, viol, labels, _, _, add_t, rem_t, tot_t in plan_out:
            want = oracle.label_plan(viol, labels, n)
            np.testing.assert_array_equal(add_t.cpu().numpy().view(np.uint64), want[0])
            np.testing.assert_array_equal(rem_t.cpu().numpy().view(np.uint64), want[1])
            assert int(tot_t.item()) == want[2]
    finally:
        c.close()
