#!/usr/bin/env python3
"""Writes tests/golden/quantity_literals.json: every resource.Quantity literal the reference
itself holds (deployment YAML, docs, e2e fixtures, Go tests), with the two values the path
derives from it:

  * milli: Quantity value x 1000 — what a TAS metric of that value compares as
    (core.EvaluateRule: value.CmpInt64(target), operator.go:13-26; the build's int64-milli
    column);
  * as_int64: Quantity.AsInt64() with `ok` ignored — what GAS reads from a request or an
    allocatable entry (gpuscheduler/utils.go:23, scheduler.go:155).  apimachinery v0.22.2
    returns (0, false) for a value held with a negative scale (a milli suffix) and for the
    inf.Dec representation; otherwise the integer.

The expected values are written out by hand from the literal's decimal / binary SI suffix
(k = 1e3, M = 1e6, G = 1e9; Ki = 2^10, Mi = 2^20; m = 1e-3), not computed by the build's
own parser.  The reference does not vendor apimachinery, so these literals are the whole of
what pins the Quantity restatement (csrc/quantity.cpp) to the reference; every other input
is "parity unpinned" (DESIGN.md §4).  Paths are relative to the reference root.
"""
import json
import os

MI = 2 ** 20
LITERALS = [
    # GAS container requests
    {"literal": "1", "source": "gpu-aware-scheduling/docs/example/bb_example.yaml:21",
     "field": "requests gpu.intel.com/i915", "milli": 1000, "as_int64": 1},
    {"literal": "100", "source": "gpu-aware-scheduling/docs/example/bb_example.yaml:22",
     "field": "requests gpu.intel.com/millicores", "milli": 100_000, "as_int64": 100},
    {"literal": "1G", "source": "gpu-aware-scheduling/docs/example/bb_example.yaml:23",
     "field": "requests gpu.intel.com/memory.max", "milli": 10 ** 12, "as_int64": 10 ** 9},
    {"literal": "10", "source": "gpu-aware-scheduling/docs/usage.md:62",
     "field": "requests gpu.intel.com/millicores", "milli": 10_000, "as_int64": 10},
    {"literal": "10M", "source": "gpu-aware-scheduling/docs/usage.md:63",
     "field": "requests gpu.intel.com/memory.max", "milli": 10 ** 10, "as_int64": 10 ** 7},
    {"literal": "1", "source": "gpu-aware-scheduling/pkg/gpuscheduler/node_resource_cache_test.go:129",
     "field": "MustParse gpu.intel.com/i915", "milli": 1000, "as_int64": 1},
    # deployment resources (container requests / limits of the extenders themselves)
    {"literal": "500Mi", "source": "telemetry-aware-scheduling/deploy/tas-deployment.yaml:37",
     "field": "limits memory", "milli": 500 * MI * 1000, "as_int64": 500 * MI},
    {"literal": "500m", "source": "telemetry-aware-scheduling/deploy/tas-deployment.yaml:38",
     "field": "limits cpu", "milli": 500, "as_int64": 0},
    {"literal": "100Mi", "source": "telemetry-aware-scheduling/deploy/tas-deployment.yaml:40",
     "field": "requests memory", "milli": 100 * MI * 1000, "as_int64": 100 * MI},
    {"literal": "100m", "source": "telemetry-aware-scheduling/deploy/tas-deployment.yaml:41",
     "field": "requests cpu", "milli": 100, "as_int64": 0},
    {"literal": "150m", "source": "telemetry-aware-scheduling/docs/power/collectd/daemonset.yaml:27",
     "field": "limits cpu", "milli": 150, "as_int64": 0},
    {"literal": "100Mi", "source": "telemetry-aware-scheduling/docs/power/collectd/daemonset.yaml:28",
     "field": "limits memory", "milli": 100 * MI * 1000, "as_int64": 100 * MI},
    {"literal": "100m", "source": "telemetry-aware-scheduling/docs/power/collectd/daemonset.yaml:30",
     "field": "requests cpu", "milli": 100, "as_int64": 0},
    {"literal": "50Mi", "source": "telemetry-aware-scheduling/docs/power/collectd/daemonset.yaml:31",
     "field": "requests memory", "milli": 50 * MI * 1000, "as_int64": 50 * MI},
    # TAS metric values (custom metrics API MetricValue.Value, metrics/client.go:64-78), as
    # the e2e node-exporter files and the Go tests give them
    {"literal": "10", "source": ".github/scripts/policies/node1 (node_filter1_metric)",
     "field": "metric value", "milli": 10_000, "as_int64": 10},
    {"literal": "0", "source": ".github/scripts/policies/node1 (node_filter2_metric)",
     "field": "metric value", "milli": 0, "as_int64": 0},
    {"literal": "1000", "source": ".github/scripts/policies/node1 (node_prioritize1_metric)",
     "field": "metric value", "milli": 1_000_000, "as_int64": 1000},
    {"literal": "50", "source": "telemetry-aware-scheduling/pkg/metrics/client_test.go:104",
     "field": "NewQuantity(50, DecimalSI)", "milli": 50_000, "as_int64": 50},
    {"literal": "90", "source": "telemetry-aware-scheduling/pkg/telemetryscheduler/scheduler_test.go:170",
     "field": "NewQuantity(90, DecimalSI)", "milli": 90_000, "as_int64": 90},
]

# The example pod of docs/example/bb_example.yaml:15-23 as the scheduler receives its v1.Pod:
# the manifest sets limits only; the API server defaults the requests of extended resources
# to their limits, so containerRequests (utils.go:14-32) reads the same three values.
BB_POD = {
    "source": "gpu-aware-scheduling/docs/example/bb_example.yaml:15-23 (requests defaulted "
              "from limits)",
    "pod": {"metadata": {"name": "bb-example", "namespace": "default"},
            "spec": {"containers": [{"name": "gpu-resource-request", "resources": {
                "limits": {"gpu.intel.com/i915": "1", "gpu.intel.com/millicores": "100",
                           "gpu.intel.com/memory.max": "1G"},
                "requests": {"gpu.intel.com/i915": "1", "gpu.intel.com/millicores": "100",
                             "gpu.intel.com/memory.max": "1G"}}}]}},
    "kinds": ["gpu.intel.com/i915", "gpu.intel.com/millicores", "gpu.intel.com/memory.max"],
    "want_requests": [[1, 100, 10 ** 9]],
}


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "quantity_literals.json"), "w") as f:
        json.dump({"literals": LITERALS, "bb_example_pod": BB_POD}, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
