"""bench.py's self-launch: `python bench.py --gpus N` without a launcher starts N ranks itself.

The driver's scaling runs may call bench.py either through torchrun (WORLD_SIZE set) or
directly; both must end with one JSON line from rank 0 whose n_gpus is the real world size.
The `launch_check` workload runs the same launcher, rendezvous and timing protocol over
gloo without touching a GPU.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=120):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e,
                          capture_output=True, text=True, timeout=timeout)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_self_launch_two_ranks():
    r = _run(["--gpus", "2", "--workload", "launch_check", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = lines[0]
    assert out["n_gpus"] == 2 and out["config"]["world_size"] == 2
    assert out["config"]["backend"] == "gloo"
    assert out["steps"] == 3 and out["warmup"] == 1


def test_single_rank_needs_no_launcher():
    r = _run(["--workload", "launch_check", "--steps", "2"])
    assert r.returncode == 0, r.stderr
    assert _json_lines(r.stdout)[0]["n_gpus"] == 1


def test_gpus_must_match_launcher_world():
    r = _run(["--gpus", "2", "--workload", "launch_check"], env={"WORLD_SIZE": "3"})
    assert r.returncode != 0
    assert "disagrees with WORLD_SIZE" in r.stderr


def test_failing_rank_fails_the_launch():
    sys.path.insert(0, os.path.join(ROOT, "platform-aware-scheduling_amd"))
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "distrib_t", os.path.join(ROOT, "platform-aware-scheduling_amd", "pas_amd", "distrib.py"))
    d = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(d)
    code = "import os, sys, time; r = int(os.environ['RANK']); time.sleep(0.2); sys.exit(3 if r == 1 else 0)"
    assert d.launch_local_ranks(2, [sys.executable, "-c", code]) == 3
    assert d.launch_local_ranks(3, [sys.executable, "-c", "import os; assert os.environ['WORLD_SIZE'] == '3'"]) == 0


import pytest  # noqa: E402


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_multi_rank_bench_carries_node_sharded_record():
    """`bench.py --gpus 2` of the headline workload: rank 0's line carries the node-sharded
    sub-record (C5 top-k + C4 sweep over a node-sharded cluster, all-gathers across the
    ranks).  Two ranks share the box's one GPU, so the collectives run over gloo here; the
    driver's 8-GPU node runs the same code over RCCL."""
    r = _run(["--gpus", "2", "--backend", "gloo", "--pods", "256", "--nodes", "20000",
              "--ns-pods", "1024", "--ns-nodes", "60000", "--steps", "3", "--warmup", "1",
              "--settle", "0.2", "--no-cpu-baseline", "--no-request-latency"], timeout=840)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    out = lines[0]
    assert out["n_gpus"] == 2 and out["config"]["world_size"] == 2
    ns = out["node_sharded"]
    assert ns["world_size"] == 2 and ns["backend"] == "gloo" and ns["nodes"] == 60000
    # the 2-D split (shard.GridTopK) at the memory-minimal shard count: 1 node shard x 2 pod
    # groups (pure pod sharding), and at 2 x 1 (pure node sharding); the same lists
    c5 = ns["c5_topk"]
    assert c5["node_shards"] == 1 and c5["pod_groups"] == 2
    assert c5["pods_per_gpu"] == 512 and c5["nodes_per_gpu"] == 60000
    assert c5["ms_per_step"] > 0 and 0 < c5["entries"] <= 1024 * 16
    nsh = ns["c5_topk_node_sharded"]
    assert nsh["node_shards"] == 2 and nsh["pods_per_gpu"] == 1024
    assert nsh["nodes_per_gpu"] == 30016 and nsh["ms_per_step"] > 0
    assert ns["splits_agree"] is True
    c4 = ns["c4_deschedule"]
    assert c4["nodes_per_gpu"] == 30016 and c4["ms_per_step"] > 0
