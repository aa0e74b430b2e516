"""Node-sharded evaluation across the GPUs of one node (BASELINE configs[3-4]).

Every reference computation on the path is per node given the snapshot: the filter verdict
(dontschedule.Violated, telemetryscheduler.go:184-225), the deschedule violations
(deschedule/strategy.go:31-50) and the GAS fit (gpuscheduler/scheduler.go:280-338).  Only
the prioritize order (core.OrderedList, operator.go:30-42) is global.  So each rank holds a
contiguous node range of the cluster as its resident snapshot and:

  * top-k prioritize: evaluates every pod (of its pod group, GridTopK) against its shard, keeps the first k entries of
    the shard's HostPriorityList as (key, global node) records (pas_tas_topk_device, or
    pas_tas_gas_topk_device for TAS + GAS), the records of all ranks are all-gathered over
    RCCL, and every rank merges them into the exact global first k (pas_topk_merge_device);
  * deschedule sweep: sweeps its shard's nodes and all-gathers the violation bitmaps
    (S x W64 words per shard; shard ranges are multiples of 64 nodes so the words of all
    ranks concatenate into the cluster bitmap).

  * full-list prioritize (C2 semantics over node shards): every rank lists each pod's whole
    shard HostPriorityList as records (pas_tas_topk_device with k = the widest shard), an
    all-to-all sends each pod's records to the rank that owns the pod (pods in contiguous
    slices), and the owner merges the shards' runs into the cluster list
    (pas_list_merge_device).  The lists stay pod-sharded: [P][N] int32 over the whole batch
    need not fit one GPU.

Collectives are torch.distributed all-gathers / all-to-alls: RCCL ("nccl") over xGMI between
GPUs; with the gloo backend (CPU tests, or several ranks sharing one GPU) the device buffers
are staged through host memory.
"""
from typing import Tuple

import torch

from .distrib import CALLS, collective


def node_range(n_total: int, world: int, rank: int, align: int = 64) -> Tuple[int, int]:
    """Contiguous node range [n0, n1) of `rank`: shards are multiples of `align` nodes (the
    bitmap word), the last takes the remainder."""
    units = (n_total + align - 1) // align
    per = (units + world - 1) // world
    n0 = min(n_total, rank * per * align)
    n1 = min(n_total, (rank + 1) * per * align)
    return n0, n1


def _all_gather(t: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """[world * t.numel()] concatenation of every rank's `t` (same shape on all ranks) over
    `group` (a torch.distributed process group of `world` ranks; None = the default group)."""
    if not collective(world):
        return t.reshape(-1)
    import torch.distributed as dist
    flat = t.contiguous().reshape(-1)
    if dist.get_backend(group) == "nccl":
        out = torch.empty(world * flat.numel(), dtype=flat.dtype, device=flat.device)
        CALLS["all_gather_into_tensor"] += 1
        dist.all_gather_into_tensor(out, flat, group=group)
        return out
    host = flat.cpu()
    parts = [torch.empty_like(host) for _ in range(world)]
    CALLS["all_gather"] += 1
    dist.all_gather(parts, host, group=group)
    return torch.cat(parts).to(flat.device)


def _all_to_all(t: torch.Tensor, world: int) -> torch.Tensor:
    """t [world, ...]: chunk t[q] goes to rank q; returns [world, ...] with out[s] = the chunk
    rank s sent to this rank."""
    if not collective(world):
        return t
    import torch.distributed as dist
    flat = t.contiguous()
    if dist.get_backend() == "nccl":
        out = torch.empty_like(flat)
        CALLS["all_to_all_single"] += 1
        dist.all_to_all_single(out, flat)
        return out
    host = flat.cpu()
    parts = [torch.empty_like(host) for _ in range(world)]
    CALLS["all_gather"] += 1
    dist.all_gather(parts, host)
    r = dist.get_rank()
    return torch.stack([part[r] for part in parts]).to(flat.device)


def pod_slice(n_pods: int, world: int, rank: int) -> Tuple[int, int]:
    """Pods [p0, p1) whose full lists `rank` owns: contiguous slices of ceil(P / world)."""
    per = (n_pods + world - 1) // world
    return min(n_pods, rank * per), min(n_pods, (rank + 1) * per)


class ShardedFullList:
    """Per-pod full HostPriorityList over a node-sharded TAS snapshot (one instance per rank).

    The rank's Context holds nodes [node_base, node_base + n_local); `width` >= every rank's
    n_local (node_range's first shard).  `run` returns (p0, p1, nodes [p1 - p0][world * width]
    int32 global node ids, -1 past len, lens [p1 - p0] int32) for the pods this rank owns
    (pod_slice)."""

    def __init__(self, ctx, width: int, world: int, rank: int, node_base: int, device="cuda"):
        self.ctx, self.width, self.world, self.rank = ctx, width, world, rank
        self.node_base = node_base
        self.device = device
        self._bufs = {}

    def _buf(self, name, shape, dtype):
        return _cached(self._bufs, name, shape, dtype, self.device)

    def run(self, gen: int, n_pods: int, n_rules: int, rules_t, rule_off_t, prio_t, cand_t=None,
            stream=None):
        w, world = self.width, self.world
        per = (n_pods + world - 1) // world
        on_gpu = torch.cuda.is_available() and str(self.device).startswith("cuda")
        cur = torch.cuda.current_stream() if on_gpu else None
        if stream is None:
            stream = cur
        # records of every pod over this shard, pods past n_pods (slice padding) all sentinels
        key = self._buf("key", (world * per, w), torch.int64)
        node = self._buf("node", (world * per, w), torch.int32)
        ln = self._buf("len", (world * per,), torch.int32)
        key[n_pods:].fill_(2**63 - 1)
        node[n_pods:].fill_(2**31 - 1)
        if on_gpu and stream != cur:
            stream.wait_stream(cur)
        self.ctx.tas_topk_device(gen, n_pods, n_rules, rules_t, rule_off_t, prio_t, cand_t, w,
                                 self.node_base, key, node, ln, stream)
        if on_gpu and stream != cur:
            cur.wait_stream(stream)
        # [owner rank][its pods][w] -> [shard][my pods][w]
        keys_in = _all_to_all(key.view(world, per, w), world)
        nodes_in = _all_to_all(node.view(world, per, w), world)
        if on_gpu and stream != cur:
            stream.wait_stream(cur)
        p0, p1 = pod_slice(n_pods, world, self.rank)
        out_node = self._buf("out_node", (per, world * w), torch.int32)
        out_len = self._buf("out_len", (per,), torch.int32)
        if per:
            self.ctx.list_merge_device(per, world, w, keys_in, nodes_in, out_node, out_len,
                                       stream=stream)
        if on_gpu and stream != cur:
            cur.wait_stream(stream)
        return p0, p1, out_node[:p1 - p0], out_len[:p1 - p0]


def _cached(bufs, name, shape, dtype, device):
    b = bufs.get(name)
    if b is None or tuple(b.shape) != tuple(shape):
        b = torch.empty(shape, dtype=dtype, device=device)
        bufs[name] = b
    return b


class ShardedTopK:
    """Per-pod global top-k over a node-sharded TAS snapshot (one instance per rank).

    The rank's Context holds the snapshot of nodes [node_base, node_base + n_local);
    `run` returns (nodes [P][k] int32 global node ids, -1 past len; lens [P] int32), the
    same on every rank of `group` (a process group of `world` ranks, the node shards of the
    cluster; None = the default group)."""

    def __init__(self, ctx, k: int, world: int, rank: int, node_base: int, device="cuda",
                 group=None):
        self.ctx, self.k, self.world, self.rank = ctx, k, world, rank
        self.node_base = node_base
        self.device = device
        self.group = group
        self._bufs = {}

    def _buf(self, name, shape, dtype):
        return _cached(self._bufs, name, shape, dtype, self.device)

    def run(self, gen: int, n_pods: int, n_rules: int, rules_t, rule_off_t, prio_t, cand_t=None,
            stream=None):
        """`stream`: the torch.cuda.Stream the kernels run on (None = torch's current stream).
        The collectives run on torch's current stream, so the two are ordered with
        wait_stream in both directions when they differ."""
        def records(key, node, ln, s):
            self.ctx.tas_topk_device(gen, n_pods, n_rules, rules_t, rule_off_t, prio_t, cand_t,
                                     self.k, self.node_base, key, node, ln, s)
        return self._run(n_pods, records, stream)

    def run_tas_gas(self, tas_gen: int, gas_gen: int, n_pods: int, n_rules: int, rules_t,
                    rule_off_t, prio_t, max_containers: int, i915_index: int, req_t, mask_t,
                    ncont_t, cand_t=None, stream=None):
        """The combined TAS + GAS top-k (BASELINE configs[4]): the shard's records over the
        nodes that pass the pod's dontschedule filter and fit its GPU request
        (pas_tas_gas_topk_device on the rank's resident TAS and GAS snapshots), merged."""
        def records(key, node, ln, s):
            self.ctx.tas_gas_topk_device(tas_gen, gas_gen, n_pods, n_rules, rules_t, rule_off_t,
                                         prio_t, cand_t, max_containers, i915_index, req_t,
                                         mask_t, ncont_t, self.k, self.node_base, key, node, ln,
                                         s)
        return self._run(n_pods, records, stream)

    def _run(self, n_pods, records, stream):
        k = self.k
        on_gpu = torch.cuda.is_available() and str(self.device).startswith("cuda")
        cur = torch.cuda.current_stream() if on_gpu else None
        if stream is None:
            stream = cur
        key = self._buf("key", (n_pods, k), torch.int64)
        node = self._buf("node", (n_pods, k), torch.int32)
        ln = self._buf("len", (n_pods,), torch.int32)
        if on_gpu and stream != cur:
            stream.wait_stream(cur)  # the caller's inputs (rules, candidates) are written
        records(key, node, ln, stream)
        if on_gpu and stream != cur:
            cur.wait_stream(stream)  # records written before the all-gather reads them
        keys_all = _all_gather(key, self.world, self.group)
        nodes_all = _all_gather(node, self.world, self.group)
        if on_gpu and stream != cur:
            stream.wait_stream(cur)  # gathered records complete before the merge reads them
        out_node = self._buf("out_node", (n_pods, k), torch.int32)
        out_len = self._buf("out_len", (n_pods,), torch.int32)
        self.ctx.topk_merge_device(n_pods, k, self.world, keys_all, nodes_all, out_node, out_len,
                                   stream)
        if on_gpu and stream != cur:
            cur.wait_stream(stream)  # the caller reads the merged lists on its stream
        return out_node, out_len


def grid_position(world: int, node_shards: int, rank: int) -> Tuple[int, int]:
    """(pod group, node shard) of `rank` in a node_shards x (world / node_shards) grid: the
    node shards of one pod group are consecutive ranks."""
    if node_shards < 1 or world % node_shards:
        raise ValueError(f"node_shards={node_shards} must divide world={world}")
    return rank // node_shards, rank % node_shards


def snapshot_bytes_per_node(n_metrics: int, cards: int = 8, kinds: int = 3) -> int:
    """Device bytes per node of the resident state a C5 rank holds (tas_snapshot.hip /
    gas_fit.hip): TAS columns 8 M + presence M / 8, the sorted values 8 M, three orders 12 M,
    the build's sort keys and ids 40 M, the lazy top-k's node-major copies 8 M + M / 8; GAS
    capacity 8 Q, usage and the card-major free table 16 K Q, card count 4."""
    return 76 * n_metrics + (n_metrics + 31) // 32 * 8 + 8 * kinds + 16 * cards * kinds + 4


def min_node_shards(world: int, n_nodes: int, n_metrics: int, cards: int = 8, kinds: int = 3,
                    budget_bytes: float = None) -> int:
    """The fewest node shards s (a divisor of world) whose per-rank snapshot fits
    `budget_bytes` (default: half of the device's memory, else 144 GB = half of an MI355X's
    288 GB): 1 for every BASELINE config (1M nodes x 64 metrics is ~5 GB)."""
    if budget_bytes is None:
        total = 288e9
        if torch.cuda.is_available():
            total = torch.cuda.get_device_properties(0).total_memory
        budget_bytes = total / 2
    per_node = snapshot_bytes_per_node(n_metrics, cards, kinds)
    for s in range(1, world + 1):
        if world % s == 0:
            n0, n1 = node_range(n_nodes, s, 0)
            if (n1 - n0) * per_node <= budget_bytes:
                return s
    return world


def pod_batch_slice(p0: int, p1: int, rules, rule_off, prio, req, mask, ncont):
    """Host arrays of pods [p0, p1) of a TAS + GAS batch, rule offsets rebased to 0."""
    r0, r1 = int(rule_off[p0]), int(rule_off[p1])
    return (rules[r0:r1], (rule_off[p0:p1 + 1] - r0).astype(rule_off.dtype), prio[p0:p1],
            req[p0:p1], mask[p0:p1], ncont[p0:p1])


class GridTopK:
    """The combined TAS + GAS top-k (BASELINE configs[4]) over a 2-D split: node_shards = s
    node shards x g = world / s pod groups.  Rank r is node shard r % s
    of pod group r // s: its Context holds nodes node_range(N, s, r % s) of the cluster as the
    resident TAS and GAS snapshots, and it evaluates the pods of pod_slice(P, g, r // s) only.
    Each step the group's s ranks all-gather their records over the group's process group and
    merge them into the group's pods' final lists (identical on those s ranks); groups never
    talk during a step (a pod is one scheduling request, telemetryscheduler.go:184-225,
    gpuscheduler/scheduler.go:449-482).  Per-rank kernel work is (P / g) pods x (N / s) nodes.
    s = 1 is pure pod sharding (no step collective; the snapshot replicated), s = world pure
    node sharding (ShardedTopK); min_node_shards picks the fewest shards the memory needs.
    `gather` assembles every group's lists once, at the end.

    rules / rule_off / prio / req / mask / ncont: host arrays of the WHOLE batch; the rank's
    pod slice is cut out here, once.  Every rank constructs every group's process group (a
    collective call), in the same order."""

    def __init__(self, ctx, k: int, world: int, rank: int, node_shards: int, n_pods: int,
                 n_nodes: int, rules, rule_off, prio, req, mask, ncont, device="cuda"):
        import numpy as np
        self.ctx, self.k, self.world, self.rank = ctx, k, world, rank
        self.s = node_shards
        self.g = world // node_shards
        self.group_id, self.shard_id = grid_position(world, node_shards, rank)
        self.n0, self.n1 = node_range(n_nodes, self.s, self.shard_id)
        self.n_pods = n_pods
        self.p0, self.p1 = pod_slice(n_pods, self.g, self.group_id)
        self.per = (n_pods + self.g - 1) // self.g
        pg = None
        if collective(world) and 1 < self.s < world:
            import torch.distributed as dist
            for gi in range(self.g):  # every rank creates every group, in order
                grp = dist.new_group(list(range(gi * self.s, (gi + 1) * self.s)))
                if gi == self.group_id:
                    pg = grp
        self.topk = ShardedTopK(ctx, k, self.s, self.shard_id, self.n0, device, group=pg)

        def dev(a):
            return torch.from_numpy(np.ascontiguousarray(a)).to(device)
        r, off, pr, rq, mk, nc = pod_batch_slice(self.p0, self.p1, rules, rule_off, prio, req,
                                                 mask, ncont)
        self.n_rules = len(r)
        self.rules, self.off, self.prio = dev(r.view(np.uint8)), dev(off), dev(pr.view(np.uint8))
        self.req, self.mask, self.ncont = dev(rq), dev(mk.view(np.int32)), dev(nc)
        self.C = req.shape[1]
        # the group's lists padded to `per` rows for the final gather
        self.out_node = torch.full((self.per, k), -1, dtype=torch.int32, device=device)
        self.out_len = torch.zeros((self.per,), dtype=torch.int32, device=device)

    def run(self, tas_gen: int, gas_gen: int, i915_index: int, stream=None):
        """One step: the group's pods' first k (final lists: node ids, -1 past len)."""
        n = self.p1 - self.p0
        if n:
            nodes, lens = self.topk.run_tas_gas(tas_gen, gas_gen, n, self.n_rules, self.rules,
                                                self.off, self.prio, self.C, i915_index,
                                                self.req, self.mask, self.ncont, None, stream)
            self.out_node[:n], self.out_len[:n] = nodes, lens
        return self.out_node[:n], self.out_len[:n]

    def gather(self):
        """Every pod's list on every rank ([P][k], [P]): one all-gather of the groups' lists
        (shard 0 of each group), at the end of the job, not per step."""
        nodes = _all_gather(self.out_node, self.world).view(self.world, self.per, self.k)
        lens = _all_gather(self.out_len, self.world).view(self.world, self.per)
        first = torch.arange(0, self.world, self.s, device=nodes.device)
        return (nodes[first].reshape(-1, self.k)[:self.n_pods],
                lens[first].reshape(-1)[:self.n_pods])


_PAD = {}  # gather_violations' padded rows of a narrower last shard, by shape and device


def gather_violations(viol_local: torch.Tensor, world: int, n_total: int) -> torch.Tensor:
    """Cluster violation bitmaps [S][W64(n_total)] from every rank's [S][W64_shard] sweep.

    Shard widths are static (node_range over n_total): every shard but the last has the
    same word count wmax, the last is copied into a zero-padded buffer of that width (kept
    across calls: its extra words stay zero) for the collective, and the concatenation is
    trimmed to W64(n_total).  No size exchange and no allocation run per step."""
    s, w = viol_local.shape
    if not collective(world):
        return viol_local
    n0, n1 = node_range(n_total, world, 0)
    wmax = (n1 - n0 + 63) // 64
    if w > wmax:
        raise ValueError(f"shard has {w} words, node_range gives at most {wmax}")
    padded = viol_local
    if w < wmax:
        key = (s, wmax, viol_local.dtype, str(viol_local.device))
        padded = _PAD.get(key)
        if padded is None:
            padded = _PAD[key] = torch.zeros((s, wmax), dtype=viol_local.dtype,
                                             device=viol_local.device)
        padded[:, :w] = viol_local
    parts = _all_gather(padded, world).reshape(world, s, wmax)
    return parts.permute(1, 0, 2).reshape(s, world * wmax)[:, :(n_total + 63) // 64]
