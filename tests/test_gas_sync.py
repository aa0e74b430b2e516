"""The GAS fit's internal fork / join (gas_fit.hip): a fit is complete or an error, as the
reference's filter answer is (gpu-aware-scheduling/pkg/gpuscheduler/scheduler.go:449-482).

With device flags a side-stream wait that gives up aborts its fit (the fit kernels return at
entry) and the call's synchronization reports PAS_EDEVICE: the host forms themselves, the
_device forms through pas_synchronize.  The fault-injection build lib/libpas_fault.so reads
PAS_GAS_FORCE_TIMEOUT=n when a context resolves its sync mode: the next n flag-mode fits'
waits give up at once (the product library has no such knob).  A fit behind more
than a second of the caller's own work on its stream still completes (the waits start
timing when the fit's prep starts)."""
import os

import numpy as np
import pytest

import pas_amd
from pas_amd import workload as wl

pytestmark = pytest.mark.gpu


def _new_ctx(monkeypatch, force=None):
    """A flag-mode context: of the product library, or (force=n) of the fault-injection
    build with its next n fits' waits forced to give up."""
    monkeypatch.setenv("PAS_GAS_SYNC", "flags")
    if force is None:
        monkeypatch.delenv("PAS_GAS_FORCE_TIMEOUT", raising=False)
        return pas_amd.Context(0)
    monkeypatch.setenv("PAS_GAS_FORCE_TIMEOUT", str(force))
    return pas_amd.Context(0, lib=pas_amd._lib.load_fault())


def _case(oracle, n=3000, p=64, seed=0xC3):
    gs = wl.make_gas_snapshot(n, seed=seed)
    gb = wl.make_gas_batch(p, seed=seed)
    want = oracle.gas_fit(gs.n_cards, gs.cap, gs.used, gb.req, gb.req_mask, gb.n_containers,
                          wl.I915)
    return gs, gb, want


def _device_inputs(gb, n):
    import torch
    dev = torch.device("cuda", 0)
    req_t = torch.from_numpy(np.ascontiguousarray(gb.req)).to(dev)
    mask_t = torch.from_numpy(np.ascontiguousarray(gb.req_mask).view(np.int32)).to(dev)
    nc_t = torch.from_numpy(np.ascontiguousarray(gb.n_containers)).to(dev)
    res_t = torch.full((len(gb.n_containers), n), -1, dtype=torch.int32, device=dev)
    return req_t, mask_t, nc_t, res_t


def test_forced_timeout_host_form_fails_then_recovers(oracle, monkeypatch):
    gs, gb, want = _case(oracle)
    ctx = _new_ctx(monkeypatch, force=1)
    try:
        ctx.gas_snapshot_set(1, gs.n_cards, gs.cap, gs.used)
        with pytest.raises(pas_amd.PasError) as e:
            ctx.gas_fit(1, gb.req, gb.req_mask, gb.n_containers, wl.I915)
        assert e.value.code == pas_amd._lib.PAS_EDEVICE
        assert "timed out" in ctx.last_error()
        # the report is cleared: the next call runs and is exact
        got = ctx.gas_fit(1, gb.req, gb.req_mask, gb.n_containers, wl.I915)
        np.testing.assert_array_equal(got, want)
        ctx.synchronize()  # nothing left to report
    finally:
        ctx.close()


def test_forced_timeout_device_form_reported_by_synchronize(oracle, monkeypatch):
    import torch
    gs, gb, want = _case(oracle, seed=0xC31)
    ctx = _new_ctx(monkeypatch, force=1)
    try:
        ctx.gas_snapshot_set(2, gs.n_cards, gs.cap, gs.used)
        req_t, mask_t, nc_t, res_t = _device_inputs(gb, len(gs.n_cards))
        p, c = gb.req_mask.shape
        ctx.gas_fit_device(2, p, c, wl.I915, req_t, mask_t, nc_t, res_t)  # enqueues: PAS_OK
        with pytest.raises(pas_amd.PasError) as e:
            ctx.synchronize()
        assert e.value.code == pas_amd._lib.PAS_EDEVICE
        # the aborted fit's side-stream kernels returned at entry: its words are not all
        # written (the untouched -1 fill shows through), so they must not be used
        assert (res_t == -1).any()
        res_t.fill_(-1)
        ctx.gas_fit_device(2, p, c, wl.I915, req_t, mask_t, nc_t, res_t)
        ctx.synchronize()
        np.testing.assert_array_equal(res_t.cpu().numpy().view(np.uint32), want)
    finally:
        ctx.close()
    torch.cuda.synchronize()


def test_forced_timeout_reported_by_next_fit(oracle, monkeypatch):
    """A _device caller that never calls pas_synchronize learns of it from its next fit."""
    gs, gb, want = _case(oracle, seed=0xC32)
    ctx = _new_ctx(monkeypatch, force=1)
    try:
        ctx.gas_snapshot_set(3, gs.n_cards, gs.cap, gs.used)
        req_t, mask_t, nc_t, res_t = _device_inputs(gb, len(gs.n_cards))
        p, c = gb.req_mask.shape
        ctx.gas_fit_device(3, p, c, wl.I915, req_t, mask_t, nc_t, res_t)
        import torch
        torch.cuda.synchronize()
        with pytest.raises(pas_amd.PasError) as e:
            ctx.gas_fit_device(3, p, c, wl.I915, req_t, mask_t, nc_t, res_t)
        assert e.value.code == pas_amd._lib.PAS_EDEVICE
        got = ctx.gas_fit(3, gb.req, gb.req_mask, gb.n_containers, wl.I915)
        np.testing.assert_array_equal(got, want)
    finally:
        ctx.close()


def _sleep_cycles_for(seconds):
    """torch.cuda._sleep cycles that spin about `seconds` on this device (calibrated)."""
    import torch
    s = torch.cuda.Stream()
    cycles = 50_000_000
    with torch.cuda.stream(s):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        torch.cuda._sleep(cycles)
        b.record()
    b.synchronize()
    ms = max(a.elapsed_time(b), 1e-3)
    return int(cycles * seconds * 1e3 / ms)


def test_fit_behind_long_work_on_its_stream(oracle, monkeypatch):
    """More than the old 1 s wait limit of the caller's own work queued on the fit's stream
    ahead of it: the fit still completes exactly, with no fault."""
    import torch
    gs, gb, want = _case(oracle, seed=0xC33)
    ctx = _new_ctx(monkeypatch)
    try:
        ctx.gas_snapshot_set(4, gs.n_cards, gs.cap, gs.used)
        req_t, mask_t, nc_t, res_t = _device_inputs(gb, len(gs.n_cards))
        p, c = gb.req_mask.shape
        cycles = _sleep_cycles_for(1.5)
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            torch.cuda._sleep(cycles)
            ctx.gas_fit_device(4, p, c, wl.I915, req_t, mask_t, nc_t, res_t, stream=st)
            b.record()
        st.synchronize()
        ctx.synchronize()
        assert a.elapsed_time(b) > 1100, "the queued work should outlast the old 1 s limit"
        np.testing.assert_array_equal(res_t.cpu().numpy().view(np.uint32), want)
    finally:
        ctx.close()


def test_fits_on_four_streams_stay_exact(oracle, monkeypatch):
    """Fits on four streams of one flag-mode context, issued without host waits: a fit that
    finds another stream's fit in flight is ordered after it; every result is exact."""
    import torch
    gs, gb, want = _case(oracle, n=20000, p=256, seed=0xC34)
    ctx = _new_ctx(monkeypatch)
    try:
        ctx.gas_snapshot_set(5, gs.n_cards, gs.cap, gs.used)
        streams = [torch.cuda.Stream() for _ in range(4)]
        bufs = [_device_inputs(gb, len(gs.n_cards)) for _ in streams]
        p, c = gb.req_mask.shape
        for rnd in range(3):
            for st, (req_t, mask_t, nc_t, res_t) in zip(streams, bufs):
                with torch.cuda.stream(st):
                    res_t.fill_(-1)
                    ctx.gas_fit_device(5, p, c, wl.I915, req_t, mask_t, nc_t, res_t, stream=st)
        ctx.synchronize()
        torch.cuda.synchronize()
        for _, _, _, res_t in bufs:
            np.testing.assert_array_equal(res_t.cpu().numpy().view(np.uint32), want)
    finally:
        ctx.close()
