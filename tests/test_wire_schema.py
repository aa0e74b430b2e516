"""Type checks of every v1.Pod / v1.Node field in request decoding (csrc/k8s_schema.h,
wire_decode.cpp check_value): json.NewDecoder(r.Body).Decode(&args) in the reference's
handlers (telemetryscheduler.go:63-78, gpuscheduler/scheduler.go:486-505) fails the request
on a value of the wrong JSON type anywhere in extender.Args, and on a Quantity / metav1.Time /
IntOrString its UnmarshalJSON rejects.  The expectations restate Go 1.16 encoding/json and
time.Parse(RFC3339) and k8s.io/api v0.22.2's field types (no Go toolchain here: parity
unpinned beyond those published rules).  Host code: runs without a GPU."""
import copy
import json

import pytest

from pas_amd import _lib, wire

NAMES = ["node-0", "node-1"]
KINDS = ["gpu.intel.com/i915", "gpu.intel.com/millicores", "gpu.intel.com/memory.max"]

NODE = {
    "kind": "Node", "apiVersion": "v1",
    "metadata": {
        "name": "node-0", "uid": "7b5d0a3c-0000-4000-8000-000000000001",
        "resourceVersion": "123", "generation": 3,
        "creationTimestamp": "2021-06-01T10:00:00Z",
        "labels": {"kubernetes.io/hostname": "node-0"},
        "annotations": {"node.alpha.kubernetes.io/ttl": "0"},
        "ownerReferences": [{"apiVersion": "v1", "kind": "X", "name": "o", "uid": "u",
                             "controller": True, "blockOwnerDeletion": False}],
        "finalizers": ["f"],
        "managedFields": [{"manager": "kubelet", "operation": "Update", "apiVersion": "v1",
                           "time": "2021-06-01T10:00:00Z", "fieldsType": "FieldsV1",
                           "fieldsV1": {"f:status": {"f:allocatable": {".": {}}}}}],
    },
    "spec": {"podCIDR": "10.0.0.0/24", "podCIDRs": ["10.0.0.0/24"], "providerID": "p",
             "unschedulable": False,
             "taints": [{"key": "k", "value": "v", "effect": "NoSchedule",
                         "timeAdded": "2021-06-01T10:00:00+02:00"}],
             "configSource": {"configMap": {"namespace": "n", "name": "c",
                                            "kubeletConfigKey": "k"}}},
    "status": {
        "capacity": {"cpu": "64", "memory": "527988604Ki", "gpu.intel.com/i915": 2},
        "allocatable": {"cpu": "63500m", "memory": " 1Gi ", "pods": "110"},
        "phase": "Running",
        "conditions": [{"type": "Ready", "status": "True",
                        "lastHeartbeatTime": "2021-06-01T10:00:00.123456789Z",
                        "lastTransitionTime": "2020-02-29T23:59:59-07:00",
                        "reason": "KubeletReady", "message": "ok"}],
        "addresses": [{"type": "InternalIP", "address": "10.0.0.1"}],
        "daemonEndpoints": {"kubeletEndpoint": {"Port": 10250}},
        "nodeInfo": {"machineID": "m", "kubeletVersion": "v1.22.2", "architecture": "amd64"},
        "images": [{"names": ["registry/app@sha256:00"], "sizeBytes": 123456789}],
        "volumesInUse": ["v"], "volumesAttached": [{"name": "v", "devicePath": "/dev/x"}],
        "config": {"active": {"configMap": {"name": "c"}}, "error": ""},
    },
}

CONTAINER = {
    "name": "c", "image": "img", "command": ["sh"], "args": ["-c", "true"], "workingDir": "/",
    "ports": [{"name": "http", "containerPort": 8080, "hostPort": 0, "protocol": "TCP"}],
    "envFrom": [{"prefix": "P_", "configMapRef": {"name": "cm", "optional": True}}],
    "env": [{"name": "A", "value": "1"},
            {"name": "B", "valueFrom": {"resourceFieldRef": {"resource": "limits.cpu",
                                                             "divisor": "1m"}}},
            {"name": "C", "valueFrom": {"fieldRef": {"fieldPath": "metadata.name"}}}],
    "resources": {"requests": {"gpu.intel.com/i915": "1", "cpu": "500m"},
                  "limits": {"gpu.intel.com/i915": 1}},
    "volumeMounts": [{"name": "v", "mountPath": "/v", "readOnly": True}],
    "livenessProbe": {"httpGet": {"path": "/h", "port": 8080, "scheme": "HTTP",
                                  "httpHeaders": [{"name": "a", "value": "b"}]},
                      "initialDelaySeconds": 3, "periodSeconds": 10},
    "readinessProbe": {"tcpSocket": {"port": "http"}, "timeoutSeconds": 1},
    "lifecycle": {"preStop": {"exec": {"command": ["sleep", "1"]}}},
    "securityContext": {"capabilities": {"add": ["NET_ADMIN"]}, "runAsUser": 1000,
                        "privileged": False, "seccompProfile": {"type": "RuntimeDefault"}},
    "terminationMessagePolicy": "File", "imagePullPolicy": "IfNotPresent",
    "stdin": False, "tty": False,
}

POD = {
    "kind": "Pod", "apiVersion": "v1",
    "metadata": {"name": "p", "namespace": "default",
                 "labels": {"telemetry-policy": "p"},
                 "creationTimestamp": "2021-06-01T10:00:00Z",
                 "deletionGracePeriodSeconds": 30},
    "spec": {
        "volumes": [{"name": "v", "emptyDir": {"sizeLimit": "1Gi"}},
                    {"name": "s", "secret": {"secretName": "s", "defaultMode": 420,
                                             "items": [{"key": "k", "path": "p"}]}},
                    {"name": "pr", "projected": {"sources": [
                        {"serviceAccountToken": {"expirationSeconds": 3607, "path": "t"}},
                        {"downwardAPI": {"items": [{"path": "l", "fieldRef": {
                            "fieldPath": "metadata.labels"}}]}}]}},
                    {"name": "e", "ephemeral": {"volumeClaimTemplate": {"spec": {
                        "accessModes": ["ReadWriteOnce"],
                        "resources": {"requests": {"storage": "1Gi"}}}}}}],
        "initContainers": [{"name": "init", "image": "i"}],
        "containers": [CONTAINER],
        "restartPolicy": "Always", "terminationGracePeriodSeconds": 30,
        "dnsPolicy": "ClusterFirst", "nodeSelector": {"a": "b"},
        "serviceAccountName": "sa", "automountServiceAccountToken": True,
        "hostNetwork": False, "securityContext": {"fsGroup": 2000,
                                                  "supplementalGroups": [1, 2],
                                                  "sysctls": [{"name": "n", "value": "v"}]},
        "imagePullSecrets": [{"name": "r"}], "schedulerName": "default-scheduler",
        "affinity": {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
            "nodeSelectorTerms": [{"matchExpressions": [
                {"key": "k", "operator": "In", "values": ["v"]}]}]},
            "preferredDuringSchedulingIgnoredDuringExecution": [
                {"weight": 1, "preference": {"matchFields": []}}]},
            "podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
                {"weight": 100, "podAffinityTerm": {"topologyKey": "t",
                                                    "labelSelector": {"matchLabels": {}}}}]}},
        "tolerations": [{"key": "k", "operator": "Exists", "effect": "NoExecute",
                         "tolerationSeconds": 300}],
        "priority": 0, "enableServiceLinks": True, "preemptionPolicy": "PreemptLowerPriority",
        "overhead": {"cpu": "10m"},
        "topologySpreadConstraints": [{"maxSkew": 1, "topologyKey": "z",
                                       "whenUnsatisfiable": "DoNotSchedule"}],
    },
    "status": {"phase": "Pending", "qosClass": "Burstable",
               "conditions": [{"type": "PodScheduled", "status": "False",
                               "lastProbeTime": None,
                               "lastTransitionTime": "2021-06-01T10:00:00Z"}],
               "startTime": "2021-06-01T10:00:00Z",
               "containerStatuses": [{"name": "c", "ready": False, "restartCount": 0,
                                      "state": {"waiting": {"reason": "Pending"}},
                                      "lastState": {"terminated": {
                                          "exitCode": 137, "signal": 9,
                                          "finishedAt": "2021-06-01T10:00:00Z"}}}]},
}


def body(pod=POD, nodes=(NODE,)):
    return json.dumps({"Pod": pod, "Nodes": {"metadata": {"resourceVersion": "1"},
                                             "items": list(nodes)}}).encode()


def ok(b):
    info, idx, _, _ = wire.decode_args(wire.NameTable(NAMES), b, _lib.PAS_ARGS_NODES)
    return list(idx)


def fails(b):
    with pytest.raises(_lib.PasError) as e:
        wire.decode_args(wire.NameTable(NAMES), b, _lib.PAS_ARGS_NODES)
    assert e.value.code == _lib.PAS_EDECODE


def with_path(obj, path, value):
    o = copy.deepcopy(obj)
    cur = o
    for k in path[:-1]:
        cur = cur[k]
    cur[path[-1]] = value
    return o


def test_full_pod_and_node_decode():
    assert ok(body()) == [0]
    p = json.dumps(POD).encode()
    assert wire.decode_pod_policy(p, "telemetry-policy")[1] == "p"
    req, mask, nc, _ = wire.decode_pod_requests(p, KINDS)
    assert int(nc[0]) == 1 and int(req[0, 0, 0]) == 1 and int(mask[0, 0]) == 1


NODE_BAD = [
    (("status",), 5),
    (("status", "capacity", "cpu"), "abc"),            # ParseQuantity
    (("status", "capacity", "cpu"), True),
    (("status", "capacity", "cpu"), {"a": 1}),
    (("status", "capacity", "cpu"), "\\u0036"),          # raw bytes go to ParseQuantity
    (("metadata", "generation"), 1.5),
    (("metadata", "generation"), "1"),
    (("metadata", "generation"), 9223372036854775808),
    (("metadata", "generation"), -9223372036854775809),
    (("metadata", "generation"), 1e3),
    (("metadata", "labels"), {"a": 1}),
    (("metadata", "finalizers"), "f"),
    (("metadata", "ownerReferences", 0, "controller"), "true"),
    (("metadata", "creationTimestamp"), 1622541600),
    (("metadata", "creationTimestamp"), "2021-13-01T10:00:00Z"),
    (("metadata", "creationTimestamp"), "2021-02-29T10:00:00Z"),   # not a leap year
    (("metadata", "creationTimestamp"), "2021-04-31T10:00:00Z"),
    (("metadata", "creationTimestamp"), "2021-06-01t10:00:00Z"),
    (("metadata", "creationTimestamp"), "2021-06-01T10:00:00"),
    (("metadata", "creationTimestamp"), "2021-06-01T10:00:00Zx"),
    (("metadata", "creationTimestamp"), "2021-06-01T24:00:00Z"),
    (("metadata", "creationTimestamp"), "2021-06-01T10:60:00Z"),
    (("metadata", "creationTimestamp"), "2021-06-01T10:00:60Z"),
    (("metadata", "creationTimestamp"), "2021-6-01T10:00:00Z"),
    (("metadata", "creationTimestamp"), "21-06-01T10:00:00Z"),
    (("metadata", "creationTimestamp"), "2021-06-01T10:00:00.1234567890Z"),
    (("metadata", "creationTimestamp"), "2021-06-01T10:00:00+0100"),
    (("metadata", "creationTimestamp"), "2021-06-01T10:00:00*01:00"),
    (("metadata", "creationTimestamp"), "2021-06-01T10:00:00.Z"),
    (("spec", "taints"), {"key": "k"}),
    (("spec", "unschedulable"), 0),
    (("spec", "podCIDRs"), [1]),
    (("status", "daemonEndpoints", "kubeletEndpoint", "Port"), 2147483648),
    (("status", "daemonEndpoints", "kubeletEndpoint", "Port"), "10250"),
    (("status", "images", 0, "sizeBytes"), "1"),
    (("status", "conditions", 0, "lastHeartbeatTime"), ""),
    (("status", "nodeInfo"), []),
]


@pytest.mark.parametrize("path,value", NODE_BAD)
def test_mistyped_node_field_fails(path, value):
    b = body(nodes=(NODE, with_path(NODE, path, value)))
    if path == ("status", "capacity", "cpu") and value == "\\u0036":
        b = body(nodes=(NODE, with_path(NODE, path, "X"))).replace(b'"X"', b'"\\u0036"')
    fails(b)


NODE_GOOD = [
    (("metadata", "generation"), -9223372036854775808),
    (("metadata", "generation"), 9223372036854775807),
    (("metadata", "generation"), -0),
    (("metadata", "generation"), None),
    (("metadata", "creationTimestamp"), None),
    (("metadata", "creationTimestamp"), "2021-06-01T7:00:00Z"),        # "15": 1 or 2 digits
    (("metadata", "creationTimestamp"), "2020-02-29T00:00:00Z"),
    (("metadata", "creationTimestamp"), "2000-02-29T00:00:00Z"),
    (("metadata", "creationTimestamp"), "2021-06-01T10:00:00.0000000001Z"),  # < 1e9
    (("metadata", "creationTimestamp"), "2021-06-01T10:00:00+99:99"),  # no range check
    (("metadata", "managedFields", 0, "fieldsV1"), [1, "x", None]),    # raw JSON
    (("status", "capacity"), None),
    (("status", "capacity", "cpu"), 12),
    (("status", "capacity", "cpu"), "  5 "),
    (("status", "capacity", "cpu"), None),
    (("status", "x-unknown"), {"any": [1, 2.5, True]}),
    (("spec", "taints"), None),
    (("status", "daemonEndpoints", "kubeletEndpoint", "Port"), -2147483648),
    (("status", "daemonEndpoints", "kubeletEndpoint", "port"), 1),     # case folding
]


@pytest.mark.parametrize("path,value", NODE_GOOD)
def test_well_typed_node_field_decodes(path, value):
    assert ok(body(nodes=(NODE, with_path(NODE, path, value)))) == [0, 0]


def test_folded_keys_are_checked():
    n = copy.deepcopy(NODE)
    n["STATUS"] = n.pop("status")
    assert ok(body(nodes=(n,))) == [0]
    n["STATUS"]["Capacity"] = {"cpu": "bad"}
    fails(body(nodes=(n,)))


POD_BAD = [
    (("spec", "containers", 0, "ports", 0, "containerPort"), "8080"),
    (("spec", "containers", 0, "ports", 0, "containerPort"), 2147483648),
    (("spec", "containers", 0, "livenessProbe", "httpGet", "port"), 1.5),
    (("spec", "containers", 0, "livenessProbe", "httpGet", "port"), True),
    (("spec", "containers", 0, "livenessProbe", "httpGet", "port"), {"a": 1}),
    (("spec", "containers", 0, "readinessProbe", "tcpSocket", "port"), 2147483648),
    (("spec", "containers", 0, "env", 1, "valueFrom", "resourceFieldRef", "divisor"), "1x"),
    (("spec", "containers", 0, "stdin"), "false"),
    (("spec", "containers", 0, "command"), "sh"),
    (("spec", "volumes", 0, "emptyDir", "sizeLimit"), "big"),
    (("spec", "volumes", 1, "secret", "defaultMode"), "0644"),
    (("spec", "affinity", "nodeAffinity", "preferredDuringSchedulingIgnoredDuringExecution",
      0, "weight"), 1.0),
    (("spec", "tolerations", 0, "tolerationSeconds"), "300"),
    (("spec", "overhead", "cpu"), "?"),
    (("spec", "priority"), 2147483648),
    (("spec", "securityContext", "supplementalGroups"), [1, "2"]),
    (("status", "startTime"), "yesterday"),
    (("status", "containerStatuses", 0, "lastState", "terminated", "exitCode"), "137"),
    (("metadata", "deletionGracePeriodSeconds"), 1.5),
]


@pytest.mark.parametrize("path,value", POD_BAD)
def test_mistyped_pod_field_fails(path, value):
    bad = with_path(POD, path, value)
    fails(body(pod=bad))
    p = json.dumps(bad).encode()
    with pytest.raises(_lib.PasError):
        wire.decode_pod_policy(p, "telemetry-policy")
    with pytest.raises(_lib.PasError):
        wire.decode_pod_requests(p, KINDS)


POD_GOOD = [
    (("spec", "containers", 0, "livenessProbe", "httpGet", "port"), "8080"),
    (("spec", "containers", 0, "livenessProbe", "httpGet", "port"), -2147483648),
    (("spec", "containers", 0, "livenessProbe", "httpGet", "port"), None),
    (("spec", "volumes", 0, "emptyDir", "sizeLimit"), 1024),
    (("spec", "containers", 0, "x-extra"), [{"deep": [[[]]]}]),
    (("status",), None),
]


@pytest.mark.parametrize("path,value", POD_GOOD)
def test_well_typed_pod_field_decodes(path, value):
    assert ok(body(pod=with_path(POD, path, value))) == [0]


def test_list_metadata_typed():
    b = json.loads(body())
    b["Nodes"]["metadata"] = {"remainingItemCount": "3"}
    fails(json.dumps(b).encode())
    b["Nodes"]["metadata"] = {"remainingItemCount": 3, "continue": "c"}
    assert ok(json.dumps(b).encode()) == [0]


def test_threaded_decode_checks_types():
    # a body large enough for the threaded item decode (several MB): one bad item among many
    nodes = [with_path(NODE, ("metadata", "name"), "node-%d" % (i % 2)) for i in range(6000)]
    good = body(nodes=nodes)
    assert len(good) > 4 << 20
    assert ok(good)[:4] == [0, 1, 0, 1]
    nodes[4321] = with_path(nodes[4321], ("status", "images", 0, "sizeBytes"), 1.5)
    fails(body(nodes=nodes))
