#!/usr/bin/env python3
"""Benchmark: BASELINE.json's metric on its 1-GPU config.

Default workload (configs[1]): one step = one batched TAS filter + prioritize pass of
4096 pending pods x 100k nodes x 16 rules (15 dontschedule + 1 scheduleonmetric) over
a 64-metric node snapshot, every input resident in HBM.  value = pod-node evaluations
per second over the whole job.  With N GPUs every rank evaluates its own 4096-pod
batch against the same (replicated) snapshot — pending pods are independent, so the
path shards by pod with no data-path collective ("scaling": "weak").

Also: --workload gas (configs[2], 10k pods x 50k nodes x 8 cards), --workload deschedule
(configs[3]: 1M nodes x 64 rules, node-sharded over the ranks, violations all-gathered) and
--workload c5 (configs[4]: 64k pods x 1M nodes TAS+GAS, node-sharded, per-pod top-k merge).

Prints ONE JSON line on rank 0.  See DESIGN.md §Measurement for the byte model.
"""
import argparse
import json
import os
import sys
import time

T_START = time.perf_counter()

import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "platform-aware-scheduling_amd"))


def _load_distrib():
    """pas_amd/distrib.py by path: importing the package would load libpas.so, and the parent
    that launches one child per GPU must not touch HIP at all."""
    import importlib.util
    path = os.path.join(ROOT, "platform-aware-scheduling_amd", "pas_amd", "distrib.py")
    spec = importlib.util.spec_from_file_location("pas_amd_distrib_bench", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


distrib = _load_distrib()
timed_steps, whole_job_rate = distrib.timed_steps, distrib.whole_job_rate

# libpas.so and the modules that load it are imported in main(), after the decision to
# launch one child process per GPU: the launching parent must not initialise HIP.
pas_amd = _lib = shard = wl = None


def _load_package():
    global pas_amd, _lib, shard, wl
    import pas_amd as _p
    from pas_amd import _lib as _l, shard as _s, workload as _w
    pas_amd, _lib, shard, wl = _p, _l, _s, _w

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "pod-node evals/sec (filter+prioritize), 4k pods×100k nodes; % of HBM peak"


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


# streams of the pipelined run reported beside the headline (same-box sweeps, DESIGN.md §5:
# TAS best at 2, deeper pipelines thrash the list stores; GAS, issue-bound, gains to 4)
PIPE_TAS, PIPE_GAS = 2, 4


def pipelined_record(depth, elapsed, gpu_ms, units, world, steps, alg_bytes):
    """The same steps on `depth` streams in turn: whole-job rate and the path's HBM fraction
    over the GPU time per step (consecutive launches overlap, so a launch's own duration is
    longer than the time per step: rocprofv3 averages do not apply to this record)."""
    return {"pipeline_streams": depth, "value": units * world * steps / elapsed,
            "ms_per_step": elapsed / steps * 1e3, "gpu_ms_per_step": gpu_ms,
            "achieved_gbs": alg_bytes / (gpu_ms / 1e3) / 1e9,
            "frac": alg_bytes / (gpu_ms / 1e3) / 1e9 / HBM_PEAK_GBS}


def load_traffic(name):
    """Per-launch HBM bytes for `name` from the committed rocprofv3 PMC summary, if any."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(name)
    except (OSError, ValueError):
        return None


# ------------------------------------------------------------------------------- TAS

def snapshot_refresh_ms(ctx, N, M, v_t, p_t, stream, gen=1):
    """Wall time of a full re-upload of the resident snapshot (buffers already allocated)
    and of one- and eight-column refreshes (AutoUpdatingCache.updateMetric).  The contents
    are re-uploaded unchanged and the snapshot ends at generation `gen`."""
    out = {}
    eight = list(range(0, M, max(M // 8, 1)))[:8]
    cases = [("full", None, None, None), ("1_column", [0], v_t[:1], p_t[:1]),
             ("8_columns", eight, v_t[eight].contiguous(), p_t[eight].contiguous())]
    for name, cols, cv, cp in cases:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if cols is None:
            ctx.tas_snapshot_set_device(gen + 1, N, M, v_t, p_t, stream)
        else:
            ctx.tas_snapshot_update_device(gen, gen + 1, cols, cv, cp, stream)
        torch.cuda.synchronize()
        out[name] = (time.perf_counter() - t0) * 1e3
        ctx.tas_snapshot_update_device(gen + 1, gen, [], None, None, stream)
    torch.cuda.synchronize()
    return out


class StreamPipeline:
    """Consecutive steps on `depth` streams of their own, in turn (depth 1: every step on the
    launch stream).  launch(k, stream) issues step k's work into output set k % depth, so batch
    i + 1's prep and first blocks run under batch i's last ones (the context keeps one scratch
    slot per stream).  fork / join order the streams after the timed region's start event and
    the end event after them (distrib.timed_steps)."""

    def __init__(self, stream, depth, launch):
        self.stream, self.depth, self.launch = stream, max(1, depth), launch
        self.lanes = [stream] if self.depth == 1 else [torch.cuda.Stream()
                                                      for _ in range(self.depth)]
        self.turn = 0

    def step(self):
        k = self.turn % self.depth
        self.turn += 1
        self.launch(k, self.lanes[k])

    def fork(self):
        for ln in self.lanes:
            if ln is not self.stream:
                ln.wait_stream(self.stream)

    def join(self):
        for ln in self.lanes:
            if ln is not self.stream:
                self.stream.wait_stream(ln)

    def sync(self):
        self.join()
        torch.cuda.synchronize()

    def timed(self, steps, warmup, world, settle=0.0):
        """(wall seconds max over ranks, GPU ms per step) of `steps` timed steps, after
        `settle` seconds of untimed steps and `warmup` more."""
        if settle > 0:
            distrib.settle(self.step, settle, sync=self.sync, world=world)
        for _ in range(warmup):
            self.step()
        gpu = {}
        el = timed_steps(self.step, steps, 0, world, gpu=gpu, fork=self.fork, join=self.join)
        torch.cuda.synchronize()
        return el, gpu["ms_per_step"]


def bench_tas(args, world, rank):
    P, N, M, R = args.pods, args.nodes, args.metrics, args.rules - 1
    ctx = pas_amd.Context(torch.cuda.current_device())
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream)
    snap = wl.make_tas_snapshot(N, M, seed=0xC2)
    batch = wl.make_tas_batch(snap, P, R, seed=distrib.batch_seed(0xC2, rank))
    v_t, p_t = dev(snap.v_milli), dev(snap.present.view(np.int64))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.tas_snapshot_set_device(1, N, M, v_t, p_t, stream)
    torch.cuda.synchronize()
    snapshot_ms = (time.perf_counter() - t0) * 1e3
    refresh = snapshot_refresh_ms(ctx, N, M, v_t, p_t, stream)
    rules_t = dev(batch.rules.view(np.uint8))
    off_t = dev(batch.rule_off)
    prio_t = dev(batch.prio.view(np.uint8))
    n_rules = len(batch.rules)
    flags = pas_amd.PAS_TAS_FILTER | pas_amd.PAS_TAS_PRIORITIZE
    # --pipeline D: consecutive batches on D streams of their own (outputs per stream), so
    # batch i + 1's prep and first blocks run under batch i's eval; D = 1 (default): every
    # step on the launch stream.  A pipelined run (PIPE_TAS streams) is reported beside it.
    D = max(1, args.pipeline)
    depth = max(D, PIPE_TAS)
    outs = [(torch.empty((P, pas_amd.w64(N)), dtype=torch.int64, device="cuda"),
             torch.empty((P, N), dtype=torch.int32, device="cuda"),
             torch.empty(P, dtype=torch.int32, device="cuda")) for _ in range(depth)]
    pass_t, order_t, len_t = outs[0]

    def launch(k, s):
        pt, ot, lt = outs[k]
        ctx.tas_eval_device(1, P, n_rules, rules_t, off_t, prio_t, None, flags, pt, ot, lt, s)

    pipe = StreamPipeline(stream, D, launch)
    step = pipe.step
    settle_steps = distrib.settle(step, args.settle, sync=pipe.sync, world=world)
    # timed steps: two HIP events on the launch stream around all of them (events between
    # the steps would add ~10 us each to the wall)
    elapsed, span_ms = pipe.timed(args.steps, args.warmup, world)
    # per-kernel breakdown from extra, untimed steps (events around every launch)
    ctx.reset_timing()
    ctx.set_timing(2)
    n_detail = min(args.steps, 5)
    for _ in range(n_detail):
        step()
    pipe.sync()
    ctx.set_timing(0)
    kern, launches = {}, {}
    for kid in (_lib.PAS_K_TAS_PREP, _lib.PAS_K_TAS_EVAL):
        ms, n = ctx.kernel_time(kid)
        kern[_lib.KERNEL_NAMES[kid]] = ms / n_detail
        launches[_lib.KERNEL_NAMES[kid]] = n // n_detail
    sum_len = int(len_t.sum().item())
    # algorithmic bytes per step: columns + presence + pass bitmaps +
    # ordered lists + lengths, plus the rule tables; divided by the span of the path
    w = pas_amd.w64(N)
    alg_bytes = 8 * M * N + 8 * M * w + 8 * P * w + 4 * sum_len + 4 * P + 16 * (n_rules + P)
    kernel_s = span_ms / 1e3
    achieved = alg_bytes / kernel_s / 1e9
    value = whole_job_rate(P * N, world, args.steps, elapsed)
    traffic = load_traffic("tas_path")
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "pod-node evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (seeded cluster snapshot + pod batch, SURVEY.md §8(d) distributions)",
        "config": {"settle_steps": settle_steps, 
            "workload": "tas_filter_prioritize (BASELINE configs[1])",
            "pods_per_gpu": P, "nodes": N, "metrics": M, "rules_per_pod": R + 1,
            "parallelism": f"pod-sharded x{world} (independent batches, replicated snapshot)",
            "pipeline_streams": D,
            "prioritize_entries_per_step": sum_len * world,
            "snapshot_build_ms": snapshot_ms, "snapshot_refresh_ms": refresh,
            "kernel_ms_per_step": kern,
            "launches_per_step": launches,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "tas path: tas_prep (rule ranges + pod grouping) and tas_eval "
                      "(filter + ordered lists) on one stream (two HIP events on the launch "
                      "stream around the timed steps)",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "algorithmic_bytes": alg_bytes,
            "kernel_ms": kernel_s * 1e3,
        },
    }
    if D == 1 and PIPE_TAS > 1 and not args.no_pipelined:
        el2, ms2 = StreamPipeline(stream, PIPE_TAS, launch).timed(args.steps, args.warmup, world,
                                                                  args.settle)
        out["pipelined"] = pipelined_record(PIPE_TAS, el2, ms2, P * N, world, args.steps,
                                            alg_bytes)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_tas(snap, batch, args.cpu_seconds)
    if rank == 0 and not args.no_request_latency:
        out["request_latency"] = request_latency(ctx, batch, N)
    ctx.close()
    return out


def synthetic_args_body(names, seed=7):
    """An extender.Args body as the kube-scheduler posts it with NodeCacheCapable false
    (extender/types.go:36-46): the pod plus every candidate as a full v1.Node (~1 KB each:
    labels, allocatable / capacity, conditions, a few images).  Synthetic, seeded."""
    rng = np.random.default_rng(seed)
    parts = []
    for i, n in enumerate(names):
        img = ",".join('{"names":["registry.local/app-%d@sha256:%064x"],"sizeBytes":%d}'
                       % (j, int(rng.integers(1 << 62)), int(rng.integers(1 << 30)))
                       for j in range(3))
        parts.append(
            '{"metadata":{"name":"%s","uid":"%08x-0000-4000-8000-%012x","resourceVersion":"%d",'
            '"labels":{"kubernetes.io/hostname":"%s","kubernetes.io/os":"linux",'
            '"telemetry.aware.scheduling.policy":"violating"}},'
            '"spec":{"podCIDR":"10.%d.%d.0/24"},'
            '"status":{"capacity":{"cpu":"64","memory":"527988604Ki","pods":"110"},'
            '"allocatable":{"cpu":"63500m","memory":"527374204Ki","pods":"110"},'
            '"conditions":[{"type":"Ready","status":"True","reason":"KubeletReady"}],'
            '"images":[%s]}}' % (n, i, i, i, n, (i >> 8) & 255, i & 255, img))
    pod = ('{"metadata":{"name":"p0","namespace":"default","labels":{"telemetry-policy":'
           '"bench"}},"spec":{"containers":[{"name":"c","resources":{"requests":{"cpu":"1"}}}]}}')
    return ('{"Pod":%s,"Nodes":{"metadata":{},"items":[%s]},"NodeNames":null}'
            % (pod, ",".join(parts))).encode()


def request_latency(ctx, batch, n_nodes, reps=5):
    """End-to-end latency of one TAS filter request and one prioritize request over the
    resident n_nodes snapshot: pas_decode_args of a full-NodeList body
    (every node a candidate) -> pas_tas_eval (filter: candidate bitmap up, pass row down) /
    pas_tas_prioritize_request (request node ids up, ordered request positions down) ->
    pas_encode_tas_filter_result / pas_encode_host_priority_list.  The
    name table and the snapshot-name array are per snapshot (built once, untimed); node JSON
    for the FilterResult points into the request body.  Median of reps."""
    import ctypes
    from pas_amd import wire
    names = [f"node-{i:06d}" for i in range(n_nodes)]
    body = synthetic_args_body(names)
    table = wire.NameTable(names)
    lib = _lib.load()
    name_arr = wire.NodeTable(names).names
    r0, r1 = int(batch.rule_off[0]), int(batch.rule_off[1])
    rules = batch.rules[r0:r1]
    prio = batch.prio[:1]
    info = _lib.PasArgsInfo()
    req = np.zeros(n_nodes, np.int32)
    spans = np.zeros((n_nodes, 2), np.int64)
    cand = np.zeros((1, pas_amd.w64(n_nodes)), np.uint64)
    body_buf = ctypes.c_char_p(body)  # keeps the address above valid
    base = ctypes.cast(body_buf, ctypes.c_void_p).value
    addr = np.zeros(n_nodes, np.uint64)
    lens = np.zeros(n_nodes, np.int64)
    out_len = ctypes.c_int64()
    cap = 1 << 28
    out = ctypes.create_string_buffer(cap)
    vp = ctypes.c_void_p
    t = {"decode_ms": [], "eval_filter_ms": [], "encode_filter_ms": [], "eval_prioritize_ms": [],
         "encode_prioritize_ms": []}
    for _ in range(reps):
        t0 = time.perf_counter()
        rc = lib.pas_decode_args(table._h, body_buf, len(body), _lib.PAS_ARGS_NODES,
                                 req.ctypes.data_as(vp), n_nodes, spans.ctypes.data_as(vp),
                                 cand.ctypes.data_as(vp), ctypes.byref(info))
        assert rc == 0 and info.n_req == n_nodes and info.n_unknown == 0
        t1 = time.perf_counter()
        pass_out, _, _ = ctx.tas_eval(1, rules, np.array([0, r1 - r0], np.int32), prio, cand,
                                      _lib.PAS_TAS_FILTER)
        t2 = time.perf_counter()
        addr[req] = base + spans[:, 0].astype(np.uint64)
        lens[req] = spans[:, 1]
        rc = lib.pas_encode_tas_filter_result(
            n_nodes, req.ctypes.data_as(vp), pass_out.ctypes.data_as(vp), name_arr,
            addr.ctypes.data_as(ctypes.POINTER(ctypes.c_char_p)), lens.ctypes.data_as(vp), out,
            cap, ctypes.byref(out_len))
        assert rc == 0
        filter_bytes = out_len.value
        t3 = time.perf_counter()
        pos = ctx.tas_prioritize_request(1, prio[0], req)
        t4 = time.perf_counter()
        # request positions index the request's own names; this body lists the snapshot's
        # nodes in snapshot order, so those are name_arr
        rc = lib.pas_encode_host_priority_list(len(pos), pos.ctypes.data_as(vp), name_arr,
                                               out, cap, ctypes.byref(out_len))
        assert rc == 0
        t5 = time.perf_counter()
        for k, v in zip(t, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4)):
            t[k].append(v * 1e3)
    res = {k: float(np.median(v)) for k, v in t.items()}
    res["filter_total_ms"] = res["decode_ms"] + res["eval_filter_ms"] + res["encode_filter_ms"]
    res["prioritize_total_ms"] = (res["decode_ms"] + res["eval_prioritize_ms"]
                                  + res["encode_prioritize_ms"])
    res.update(nodes=n_nodes, body_bytes=len(body), filter_response_bytes=filter_bytes,
               decode_gb_per_s=len(body) / res["decode_ms"] / 1e6,
               decode_threads=int(lib.pas_decode_threads(len(body))),
               note="host API calls (PCIe transfers of the candidate bitmap, pass row and "
                    "ordered list included); median of %d" % reps)
    table.close()
    return res


def cpu_threads():
    """Host threads for the CPU baseline: the box's CPU share for one GPU (16), at most."""
    return max(1, min(16, os.cpu_count() or 1))


def threaded_rate(run_range, n_items, per_item_s, budget_s, threads):
    """Items/s of run_range(lo, hi) over a bounded sample split across `threads` Python
    threads (the oracle's ctypes calls release the GIL).  Returns (rate, items, seconds)."""
    from concurrent.futures import ThreadPoolExecutor
    items = int(max(threads, min(n_items, budget_s * threads / max(per_item_s, 1e-6))))
    # small chunks handed out dynamically (pods differ in cost)
    chunk = max(1, items // (threads * 8))
    bounds = [(lo, min(items, lo + chunk)) for lo in range(0, items, chunk)]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda b: run_range(*b), bounds))
    t = time.perf_counter() - t0
    return items / t, items, t


def cpu_baseline_tas(snap, batch, budget_s):
    """The C restatement of the reference (oracle/) on a bounded pod sample: one thread, and
    pods partitioned over the host threads (SURVEY.md §8(d) Plan B)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    N = snap.v_milli.shape[1]

    def run_range(lo, hi):
        if hi <= lo:
            return
        off = batch.rule_off[lo: hi + 1] - batch.rule_off[lo]
        oracle.tas_eval(snap.v_milli, snap.present,
                        batch.rules[batch.rule_off[lo]: batch.rule_off[hi]], off,
                        batch.prio[lo:hi], None, 3)

    t0 = time.perf_counter()
    run_range(0, 1)
    one = time.perf_counter() - t0
    single, pods1, t1 = threaded_rate(run_range, len(batch.prio), one, budget_s / 2, 1)
    threads = cpu_threads()
    multi, pods_t, tt = threaded_rate(run_range, len(batch.prio), one, budget_s / 2, threads)
    return {"value": multi * N, "unit": "pod-node evals/s", "cores": threads, "kind": "port",
            "single_thread_value": single * N,
            "sample": f"{pods_t} pods x {N} nodes x 16 rules over {threads} threads in "
                      f"{tt:.1f} s (1 thread: {pods1} pods in {t1:.1f} s); first pods of the "
                      "rank-0 batch; oracle/pas_oracle.c, C restatement of the reference"}


# ------------------------------------------------------------------------------- GAS

def bench_gas(args, world, rank):
    P, N = args.pods, args.nodes
    ctx = pas_amd.Context(torch.cuda.current_device())
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream)
    snap = wl.make_gas_snapshot(N, seed=0xC3)
    batch = wl.make_gas_batch(P, seed=distrib.batch_seed(0xC3, rank))
    K, Q = snap.used.shape[1], snap.used.shape[2]
    C = batch.req.shape[1]
    ctx.gas_snapshot_set_device(1, N, K, Q, dev(snap.n_cards), dev(snap.cap), dev(snap.used),
                                stream)
    req_t, mask_t = dev(batch.req), dev(batch.req_mask.view(np.int32))
    nc_t = dev(batch.n_containers)
    # result rows at a pitch of N rounded up to 32 words (pas_gas_fit_ld_device): every row
    # starts on a 128-B line; --gas-pitch dense writes [P][N] rows
    ld = N if args.gas_pitch == "dense" else (N + 31) // 32 * 32
    # --pipeline D: consecutive batches on D streams of their own (results per stream): batch
    # i + 1's prep kernels run under batch i's fit kernels (one scratch slot per stream); a
    # pipelined run (PIPE_GAS streams) is reported beside the D = 1 line
    D = max(1, args.pipeline)
    depth = max(D, PIPE_GAS)
    results = [torch.empty((P, ld), dtype=torch.int32, device="cuda") for _ in range(depth)]
    res_t = results[0]

    def launch(k, s):
        ctx.gas_fit_ld_device(1, P, C, wl.I915, req_t, mask_t, nc_t, results[k], ld, stream=s)

    pipe = StreamPipeline(stream, D, launch)
    step = pipe.step
    settle_steps = distrib.settle(step, args.settle, sync=pipe.sync, world=world)
    elapsed, gpu_ms = pipe.timed(args.steps, args.warmup, world)
    gpu = {"ms_per_step": gpu_ms}
    # the fit launches alone, from extra, untimed steps (span events around them)
    ctx.reset_timing()
    ctx.set_timing(1)
    for _ in range(min(args.steps, 5)):
        step()
    pipe.sync()
    ctx.set_timing(0)
    pipelined = None
    if D == 1 and PIPE_GAS > 1 and not args.no_pipelined:
        pipelined = StreamPipeline(stream, PIPE_GAS, launch).timed(args.steps, args.warmup,
                                                                   world, args.settle)
    written = max(D, PIPE_GAS if pipelined else 1)  # result sets some step wrote
    assert all(torch.equal(r, res_t) for r in results[1:written]), "pipeline results differ"
    k_ms, k_n = ctx.kernel_time(_lib.PAS_K_GAS_FIT)
    # the same batch into dense [P][N] rows (pas_gas_fit_device), untimed extra steps
    dense_ms = None
    if ld != N:
        dres_t = torch.empty((P, N), dtype=torch.int32, device="cuda")
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            ctx.gas_fit_device(1, P, C, wl.I915, req_t, mask_t, nc_t, dres_t, stream)
        a.record(stream)
        for _ in range(args.steps):
            ctx.gas_fit_device(1, P, C, wl.I915, req_t, mask_t, nc_t, dres_t, stream)
        b.record(stream)
        b.synchronize()
        dense_ms = a.elapsed_time(b) / args.steps
        # (PAS_BENCH_ABLATED: timing runs of diagnostic builds whose outputs are wrong on purpose)
        assert os.environ.get("PAS_BENCH_ABLATED") or torch.equal(dres_t, res_t[:, :N]), \
            "dense and pitched results differ"
        del dres_t
    alg_bytes = N * (8 * Q + 8 * K * Q + 4) + P * (8 * C * Q + 4 * C + 4) + 4 * P * N
    kernel_s = gpu["ms_per_step"] / 1e3
    achieved = alg_bytes / kernel_s / 1e9
    out = {
        "metric": "GAS per-card fit evals/sec (pod-node fits), 10k pods×50k nodes×8 cards",
        "value": whole_job_rate(P * N, world, args.steps, elapsed), "unit": "pod-node fits/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int64", "data": "synthetic (SURVEY.md §8(d) C3)",
        "config": {"settle_steps": settle_steps, "workload": "gas_fit (BASELINE configs[2])", "pods_per_gpu": P, "nodes": N,
                   "cards": K, "resources": Q, "result_row_pitch": ld, "pipeline_streams": D,
                   "dense_pitch_gpu_ms_per_step": dense_ms,
                   "fit_fraction": float((res_t[:, :N].cpu().numpy().view(np.uint32) >> 31)
                                         .mean())},
        "roofline": {"bound": "hbm",
                     "kernel": "gas fit path: gas_prep_kernel, gas_rank_prep_kernel, "
                               "gas_rfit_single_kernel, gas_rfit_closed_kernel, "
                               "gas_rfit_seq_kernel and gas_fit_generic_kernel (two HIP "
                               "events on the launch stream "
                               "around the timed steps)",
                     "fit_launches_ms": k_ms / max(k_n, 1),
                     "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": load_traffic("gas_fit_kernel"), "algorithmic_bytes": alg_bytes,
                     "kernel_ms": kernel_s * 1e3},
    }
    if pipelined:
        out["pipelined"] = pipelined_record(PIPE_GAS, pipelined[0], pipelined[1], P * N, world,
                                            args.steps, alg_bytes)
    # The fit kernels are bound by VALU issue, not by HBM: their VALU
    # wave-instructions per step (SQ_INSTS_VALU, committed PMC pass) over the same GPU time,
    # against the chip's issue rate at 4 cycles per wave64 VALU instruction: 1024 SIMDs x
    # 2.4 GHz / 4 (scripts/diag/issue_rates.hip measures 4.3 for this mix; valu_rate.hip has
    # the per-form costs: 2.4-2.7 for plain VOP2 ops, 4.0-4.8 for the VOP3 and 64-bit forms
    # the fit loops are made of, so this is the mix's rate, not an absolute ceiling).
    valu = load_traffic("gas_fit_valu_per_step")
    if valu:
        peak = 1024 * 2.4e9 / 4
        out["issue_roofline"] = {
            "bound": "valu_issue", "unit": "wave-instructions/s", "achieved": valu / kernel_s,
            "peak": peak, "frac": valu / kernel_s / peak, "valu_per_step": valu,
            "salu_per_step": load_traffic("gas_fit_salu_per_step"),
            "source": "profiles/traffic.json (rocprofv3 --pmc SQ_INSTS_VALU, fit kernels)"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle

        def run_range(lo, hi):
            if hi > lo:
                oracle.gas_fit(snap.n_cards, snap.cap, snap.used, batch.req[lo:hi],
                               batch.req_mask[lo:hi], batch.n_containers[lo:hi], wl.I915)

        t0 = time.perf_counter()
        run_range(0, 1)
        one = time.perf_counter() - t0
        single, pods1, t1 = threaded_rate(run_range, P, one, args.cpu_seconds / 2, 1)
        threads = cpu_threads()
        multi, pods_t, tt = threaded_rate(run_range, P, one, args.cpu_seconds / 2, threads)
        out["cpu_baseline"] = {"value": multi * N, "unit": "pod-node fits/s", "cores": threads,
                               "kind": "port", "single_thread_value": single * N,
                               "sample": f"{pods_t} pods x {N} nodes over {threads} threads in "
                                         f"{tt:.1f} s (1 thread: {pods1} pods in {t1:.1f} s)"}
    ctx.close()
    return out


# ------------------------------------------------------------------------ deschedule

def shard_tas(snap, n0, n1):
    """Columns of nodes [n0, n1) (n0 a multiple of 64, as pas_amd.shard.node_range gives)."""
    v = np.ascontiguousarray(snap.v_milli[:, n0:n1])
    pres = np.ascontiguousarray(snap.present[:, n0 // 64:(n1 + 63) // 64])
    return v, pres


def bench_deschedule(args, world, rank):
    """configs[3]: the sweep over N nodes, node-sharded over the ranks (strong scaling);
    every rank ends the step with the cluster violation bitmaps (all-gather)."""
    N, M, S = args.nodes, args.metrics, 16
    ctx = pas_amd.Context(torch.cuda.current_device())
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream)
    snap = wl.make_tas_snapshot(N, M, seed=0xC4)
    n0, n1 = shard.node_range(N, world, rank)
    v, pres = shard_tas(snap, n0, n1)
    n_local = n1 - n0
    rules, off = wl.make_deschedule_rules(snap, S, 4, seed=0xC4)
    v_t, p_t = dev(v), dev(pres.view(np.int64))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.tas_snapshot_set_device(1, n_local, M, v_t, p_t, stream)
    torch.cuda.synchronize()
    snapshot_ms = (time.perf_counter() - t0) * 1e3
    refresh = snapshot_refresh_ms(ctx, n_local, M, v_t, p_t, stream)
    del v_t, p_t
    rules_t, off_t = dev(rules.view(np.uint8)), dev(off)
    viol_t = torch.empty((S, pas_amd.w64(n_local)), dtype=torch.int64, device="cuda")
    # labels the nodes carry before Enforce (10 % of (node, strategy) pairs), and the per-node
    # add / remove masks of updateNodeLabels (enforce.go:99-151) for the rank's shard
    lab = wl.pack_bits(np.random.default_rng(0xC4 + rank).random((S, n_local)) < 0.1)
    labels_t = dev(lab.view(np.int64))
    add_t = torch.empty(n_local, dtype=torch.int64, device="cuda")
    rem_t = torch.empty(n_local, dtype=torch.int64, device="cuda")
    total_t = torch.empty(1, dtype=torch.int64, device="cuda")
    gathered = {}

    fused = not getattr(args, "deschedule_separate", False)

    def step():
        if fused:  # the sweep with its label plan in one pass
            ctx.tas_deschedule_device(1, S, len(rules), rules_t, off_t, viol_t, labels_t, add_t,
                                      rem_t, total_t, stream)
        else:
            ctx.tas_violations_device(1, S, len(rules), rules_t, off_t, viol_t, stream)
            ctx.tas_label_plan_device(n_local, S, viol_t, labels_t, add_t, rem_t, total_t,
                                      stream)
        gathered["v"] = shard.gather_violations(viol_t, world, N)

    settle_steps = distrib.settle(step, args.settle, world=world)
    for _ in range(args.warmup):
        step()
    ctx.reset_timing()
    ctx.set_timing(1)
    elapsed = timed_steps(step, args.steps, 0, world)
    ctx.set_timing(0)
    k_ms, k_n = ctx.kernel_time(_lib.PAS_K_TAS_VIOLATIONS)
    l_ms, l_n = ctx.kernel_time(_lib.PAS_K_TAS_LABELS)
    w = pas_amd.w64(n_local)
    alg_bytes = 8 * M * n_local + 8 * M * w + 8 * S * w
    if fused:  # the plan's label words read and add / remove masks written by the same kernel
        alg_bytes += 8 * S * w + 16 * n_local
    kernel_s = (k_ms / max(k_n, 1)) / 1e3
    achieved = alg_bytes / kernel_s / 1e9
    out = {
        "metric": "TAS deschedule sweep node-rule evals/sec, 1M nodes×64 rules",
        "value": N * len(rules) * args.steps / elapsed,
        "unit": "node-rule evals/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (SURVEY.md §8(d) C4)",
        "config": {"settle_steps": settle_steps, "workload": "tas_deschedule_sweep (BASELINE configs[3])", "nodes": N,
                   "nodes_per_gpu": n_local, "metrics": M, "strategies": S, "rules": len(rules),
                   "step": ("sweep with its label plan fused (add/remove masks per node)"
                            if fused else "sweep, then label plan (add/remove masks per node)")
                           + " + all-gather",
                   "snapshot_build_ms": snapshot_ms, "snapshot_refresh_ms": refresh,
                   "parallelism": f"node-sharded x{world}, violation bitmaps all-gathered"},
        "label_plan_ms": None if fused else l_ms / max(l_n, 1),
        "roofline": {"bound": "hbm", "kernel": "tas_violations_run_kernel", "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": load_traffic("tas_violations_kernel"),
                     "algorithmic_bytes": alg_bytes, "kernel_ms": kernel_s * 1e3},
    }
    ctx.close()
    return out


# ------------------------------------------------------------------------------- C5

def c5_setup(args, world, rank, node_shards=None, host=None):
    """The C5 workload on this rank: its node range of the cluster -- node shard rank % s of
    s = node_shards (default world: one shard per rank; 1: every node) -- as resident TAS and
    GAS snapshots (generations 1 and 2), the pod batch on the device.  host: a dict that
    receives the host batches (tbatch, gbatch)."""
    P, N, M, R = args.pods, args.nodes, args.metrics, args.rules - 1
    ctx = pas_amd.Context(torch.cuda.current_device())
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream)
    s = world if node_shards is None else node_shards
    n0, n1 = shard.node_range(N, s, rank % s)
    tsnap = wl.make_tas_snapshot(N, M, seed=0xC5)
    v, pres = shard_tas(tsnap, n0, n1)
    ctx.tas_snapshot_set_device(1, n1 - n0, M, dev(v), dev(pres.view(np.int64)), stream)
    tbatch = wl.make_tas_batch(tsnap, P, R, seed=0xC5)
    del tsnap, v, pres
    gsnap = wl.make_gas_snapshot(N, seed=0xC5)
    ctx.gas_snapshot_set_device(2, n1 - n0, gsnap.used.shape[1], gsnap.used.shape[2],
                                dev(gsnap.n_cards[n0:n1]), dev(gsnap.cap[n0:n1]),
                                dev(gsnap.used[n0:n1]), stream)
    gbatch = wl.make_gas_batch(P, seed=0xC5)
    del gsnap
    t = {"rules": dev(tbatch.rules.view(np.uint8)), "off": dev(tbatch.rule_off),
         "prio": dev(tbatch.prio.view(np.uint8)), "req": dev(gbatch.req),
         "mask": dev(gbatch.req_mask.view(np.int32)), "ncont": dev(gbatch.n_containers),
         "n_rules": len(tbatch.rules), "C": gbatch.req.shape[1]}
    if host is not None:
        host["tbatch"], host["gbatch"] = tbatch, gbatch
    return ctx, stream, n0, n1, t


def c5_step_fn(ctx, stream, topk, P, t):
    """One C5 step: the rank's combined TAS + GAS records along each pod's order
    (pas_tas_gas_topk_device), all-gathered and merged into every pod's global first k."""
    result = {}

    def step():
        result["nodes"], result["len"] = topk.run_tas_gas(
            1, 2, P, t["n_rules"], t["rules"], t["off"], t["prio"], t["C"], wl.I915, t["req"],
            t["mask"], t["ncont"], stream=stream)
    return step, result


def bench_c5(args, world, rank):
    """configs[4]: TAS+GAS over a node-sharded cluster: per rank, each pod's first k nodes of
    the shard that pass its dontschedule filter and fit its GPU request, evaluated along the
    pod's prioritize order until k are kept (pas_tas_gas_topk_device); the records of all
    ranks are all-gathered (RCCL) and merged into the cluster's first k per pod (strong
    scaling: the cluster is fixed).  value = pods whose top-k list is produced per second;
    the (pod, node) pairs actually evaluated are reported beside it, never counted as the
    P x N evaluations the composed path would perform."""
    P, N, M, R, K = args.pods, args.nodes, args.metrics, args.rules - 1, args.topk
    ctx, stream, n0, n1, t = c5_setup(args, world, rank)
    topk = shard.ShardedTopK(ctx, K, world, rank, n0)
    step, result = c5_step_fn(ctx, stream, topk, P, t)
    settle_steps = distrib.settle(step, args.settle, world=world)
    for _ in range(args.warmup):
        step()
    gpu = {}
    elapsed = timed_steps(step, args.steps, 0, world, gpu=gpu)
    # the combined kernel alone, from extra untimed steps (events around the launch)
    ctx.reset_timing()
    ctx.set_timing(2)
    n_detail = min(args.steps, 5)
    for _ in range(n_detail):
        step()
    ctx.set_timing(0)
    k_ms, k_n = ctx.kernel_time(_lib.PAS_K_TAS_GAS_TOPK)
    out = {
        "metric": "combined TAS+GAS per-pod top-k lists/sec, 64k pods x 1M nodes, node-sharded",
        "value": P * args.steps / elapsed,
        "unit": "pods/s (top-k HostPriorityLists)",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (SURVEY.md §8(d) C5)",
        "config": {"settle_steps": settle_steps,
                   "workload": "tas_gas_topk_node_sharded (BASELINE configs[4])", "pods": P,
                   "nodes": N, "nodes_per_gpu": n1 - n0, "metrics": M, "rules_per_pod": R + 1,
                   "topk": K, "parallelism": f"node-sharded x{world}, top-k records "
                                             "all-gathered and merged",
                   "step": "pas_tas_gas_topk_device (filter + fit along each pod's order until "
                           "k kept) + all-gather + pas_topk_merge_device",
                   "topk_kernel_ms": k_ms / max(k_n, 1),
                   "gpu_ms_per_step": gpu["ms_per_step"],
                   "mean_list_len": float(result["len"].float().mean().item())},
    }
    ctx.close()
    return out


def grid_c5_record(a, world, rank, node_shards):
    """The C5 step over a node_shards x (world / node_shards) grid (shard.GridTopK), timed with
    the barrier / max-over-ranks protocol; returns (record, every pod's lists gathered)."""
    host = {}
    ctx, stream, n0, n1, t = c5_setup(a, world, rank, node_shards, host=host)
    del t
    tb, gb = host["tbatch"], host["gbatch"]
    grid = shard.GridTopK(ctx, a.topk, world, rank, node_shards, a.pods, a.nodes, tb.rules,
                          tb.rule_off, tb.prio, gb.req, gb.req_mask, gb.n_containers)
    for _ in range(a.warmup):
        grid.run(1, 2, wl.I915, stream)
    el = timed_steps(lambda: grid.run(1, 2, wl.I915, stream), a.steps, 0, world)
    # the combined kernel alone (extra untimed steps, events around the launch)
    ctx.reset_timing()
    ctx.set_timing(2)
    for _ in range(3):
        grid.run(1, 2, wl.I915, stream)
    ctx.set_timing(0)
    k_ms, k_n = ctx.kernel_time(_lib.PAS_K_TAS_GAS_TOPK)
    lists = grid.gather()
    g = world // node_shards
    rec = {"split": f"{node_shards} node shard(s) x {g} pod group(s)",
           "node_shards": node_shards, "pod_groups": g, "pods_per_gpu": grid.p1 - grid.p0,
           "nodes_per_gpu": n1 - n0, "topk": a.topk,
           "step_collective": ("all-gather of records within each pod group + merge"
                               if node_shards > 1 else "none (lists gathered once at the end)"),
           "ms_per_step": el / a.steps * 1e3, "pods_per_s": a.pods * a.steps / el,
           "topk_kernel_ms": k_ms / max(k_n, 1), "scaling": "strong"}
    ctx.close()
    del grid
    torch.cuda.empty_cache()
    return rec, (lists[0].cpu(), lists[1].cpu())


def node_sharded_record(args, world, rank):
    """The north_star's 1M-node scaling point, run inside a multi-GPU bench.py call: the C5
    step (64k pods x 1M nodes) over the 2-D split of shard.GridTopK -- s node shards x
    world / s pod groups -- at s = the fewest shards the snapshot memory needs
    (shard.min_node_shards: 1 at 1M nodes, pure pod sharding), at s = world (pure node
    sharding, the path for clusters past one GPU's memory) and, from 4 ranks, at s = 2; plus
    the C4 deschedule sweep (1M nodes x 64 rules + all-gather of the violation bitmaps).  Each
    is timed with the same barrier / max-over-ranks protocol, and every split's lists are
    checked equal.  The driver's 1/2/4/8 runs of bench.py then carry the curves without a
    --workload flag (DESIGN.md §6 cost model: per-rank kernel work (P / g) x (N / s))."""
    import argparse as _ap
    import torch.distributed as dist
    rec = {"nodes": 1_000_000, "world_size": world,
           "backend": dist.get_backend() if world > 1 else None}
    a = _ap.Namespace(**vars(args))
    a.pods, a.nodes, a.steps, a.warmup, a.settle = args.ns_pods, args.ns_nodes, 10, 2, 0.1
    rec["nodes"] = a.nodes
    s_mem = shard.min_node_shards(world, a.nodes, a.metrics)
    splits = [("c5_topk", s_mem), ("c5_topk_node_sharded", world)]
    if world >= 4 and world % 2 == 0:
        splits.append(("c5_topk_grid_2", 2))
    lists = {}
    for name, s in splits:
        if any(s == s2 for s2 in lists):
            continue
        rec[name], lists[s] = grid_c5_record(a, world, rank, s)
    ref = lists[s_mem]
    same = all(torch.equal(v[0], ref[0]) and torch.equal(v[1], ref[1]) for v in lists.values())
    rec["splits_agree"] = all(distrib.gather_objects(same, world))
    rec["c5_topk"]["entries"] = int(ref[1].to(torch.int64).sum().item())
    d = bench_deschedule(a, world, rank)
    rec["c4_deschedule"] = {"nodes_per_gpu": d["config"]["nodes_per_gpu"],
                            "ms_per_step": d["ms_per_step"],
                            "node_rule_evals_per_s": d["value"],
                            "sweep_kernel_ms": d["roofline"]["kernel_ms"], "scaling": "strong"}
    return rec


def bench_launch_check(args, world, rank):
    """Self-launch check (tests/test_bench_launch.py): the ranks bench.py started join a
    gloo group and time empty steps with the same barrier / max-over-ranks protocol."""
    elapsed = timed_steps(lambda: None, args.steps, args.warmup, world,
                          sync=lambda: None)
    import torch.distributed as dist
    return {"metric": "launch check", "value": float(world), "unit": "ranks", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / max(args.steps, 1) * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "none",
            "data": "none", "config": {"workload": "launch_check", "world_size":
                                       dist.get_world_size() if world > 1 else 1,
                                       "backend": dist.get_backend() if world > 1 else None,
                                       "rank0_pid": os.getpid()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gas-pitch", choices=["aligned", "dense"], default="aligned",
                    help="GAS result rows: N rounded up to 32 words (default) or dense N")
    ap.add_argument("--workload", choices=["tas", "gas", "deschedule", "c5", "launch_check"],
                    default="tas")
    ap.add_argument("--pods", type=int, default=None)
    ap.add_argument("--nodes", type=int, default=None)
    ap.add_argument("--metrics", type=int, default=64)
    ap.add_argument("--rules", type=int, default=16)
    ap.add_argument("--topk", type=int, default=16)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--settle", type=float, default=0.3,
                    help="seconds of untimed steps before the warmup steps (clocks settle)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-node-sharded", action="store_true",
                    help="with --gpus N > 1: skip the node-sharded 1M-node sub-record")
    ap.add_argument("--ns-pods", type=int, default=65_536,
                    help="pods of the node-sharded sub-record's C5 step")
    ap.add_argument("--ns-nodes", type=int, default=1_000_000,
                    help="cluster nodes of the node-sharded sub-record")
    ap.add_argument("--backend", choices=["auto", "nccl", "gloo"], default="auto",
                    help="collective backend of a multi-rank run (auto: RCCL on GPUs); gloo "
                         "lets several ranks share one GPU (tests)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="TAS/GAS: consecutive batches on this many streams of their own (1: "
                         "the launch stream only)")
    ap.add_argument("--no-pipelined", action="store_true",
                    help="skip the pipelined sub-record (kernel profiles of the D = 1 line)")
    ap.add_argument("--deschedule-separate", action="store_true",
                    help="deschedule: the sweep and the label plan as two calls (default: "
                         "pas_tas_deschedule_device, one pass)")
    ap.add_argument("--no-request-latency", action="store_true",
                    help="skip the f2 request-latency leg of the TAS workload")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # no launcher: start one child per GPU (fresh processes, nothing initialised here)
        sys.exit(distrib.launch_local_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)]
                                            + sys.argv[1:]))
    if env_world is not None and int(env_world) != args.gpus:
        ap.error(f"--gpus {args.gpus} disagrees with WORLD_SIZE={env_world} from the launcher")
    defaults = {"tas": (4096, 100_000), "gas": (10_000, 50_000), "deschedule": (0, 1_000_000),
                "c5": (65_536, 1_000_000), "launch_check": (0, 0)}
    dp, dn = defaults[args.workload]
    args.pods = args.pods or dp
    args.nodes = args.nodes or dn
    if args.workload == "launch_check":
        world, rank, _ = distrib.setup("gloo")
        out = bench_launch_check(args, world, rank)
    else:
        _load_package()
        world, rank, _ = distrib.setup(None if args.backend == "auto" else args.backend)
        if args.backend == "gloo" and torch.cuda.is_available():
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0"))
                                  % torch.cuda.device_count())
        # a stream of our own (not the null stream): libpas launches on it, and the timing
        # events of distrib.timed_steps are recorded on it
        torch.cuda.set_stream(torch.cuda.Stream())
        fn = {"tas": bench_tas, "gas": bench_gas, "deschedule": bench_deschedule,
              "c5": bench_c5}[args.workload]
        out = fn(args, world, rank)
        if world > 1:
            import torch.distributed as dist
            out["config"]["world_size"] = dist.get_world_size()
            out["config"]["backend"] = dist.get_backend()
            if args.workload == "tas" and not args.no_node_sharded:
                # the north_star's node-sharded curve at 1M nodes rides on every multi-GPU
                # run of the headline workload (the N = 1 line is unchanged)
                out["node_sharded"] = node_sharded_record(args, world, rank)
            # orchestration cost of the multi-rank run: each rank's wall time
            # since its start and its peak host RSS
            import resource
            mine = (round(time.perf_counter() - T_START, 1),
                    resource.getrusage(resource.RUSAGE_SELF).ru_maxrss // 1024)
            per = distrib.gather_objects(mine, world)
            out["config"]["rank_wall_s"] = [p[0] for p in per]
            out["config"]["rank_host_rss_peak_mb"] = [p[1] for p in per]
    if rank == 0:
        print(json.dumps(out), flush=True)
    distrib.teardown(world)


if __name__ == "__main__":
    main()
