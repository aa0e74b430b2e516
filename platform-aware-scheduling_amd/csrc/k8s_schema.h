// k8s_schema.h — the Go types extender.Args decodes into, as JSON type descriptors (host only,
// included by wire_decode.cpp).
//
// The reference decodes every request with json.NewDecoder(r.Body).Decode(&args) into
// extender.Args {Pod *v1.Pod; Nodes *v1.NodeList; NodeNames *[]string}
// (telemetryscheduler.go:63-78, gpuscheduler/scheduler.go:486-505), so a value of the wrong
// JSON type anywhere inside the pod or a node fails the request, not only in the fields the
// extenders read.  These tables restate k8s.io/api v0.22.2 core/v1 (and the apimachinery
// v0.22.2 metav1 / resource / intstr types they embed) field by field: the JSON name of every
// field (`json:"..."` tags; embedded `json:",inline"` structs flattened into their parent) and
// the Go type it decodes into.  Neither module is vendored in the reference (go.mod pins
// them); this is a restatement of their published types, parity unpinned by the reference's
// own tests (no test of the reference sends a mistyped field).
//
// Kinds (what json.Unmarshal accepts for each, Go 1.16 encoding/json):
//   kString       JSON string (numbers, bools, objects, arrays: UnmarshalTypeError)
//   kBool         true / false
//   kInt32/kInt64 a number strconv.ParseInt accepts (no fraction or exponent) in range
//   kQuantity     resource.Quantity.UnmarshalJSON: the literal bytes, quotes stripped and
//                 spaces trimmed, must ParseQuantity
//   kTime         metav1.Time.UnmarshalJSON: a JSON string that time.Parse(RFC3339) accepts
//   kIntOrString  intstr.IntOrString: a string, or a number that is an int32
//   kRaw          metav1.FieldsV1 (raw JSON, any value)
//   kMap          map[string]elem (keys are any strings)
//   kSlice        []elem
//   kStruct       fields matched as encoding/json does (exact name, else case folding)
// null is accepted for every kind (a pointer / map / slice becomes nil, anything else keeps
// its value; the UnmarshalJSON methods above accept "null").
#pragma once

#include <cstdint>

namespace pas_schema {

enum class GoKind : uint8_t {
  kString, kBool, kInt32, kInt64, kQuantity, kTime, kIntOrString, kRaw, kMap, kSlice, kStruct
};
struct GoField;
struct GoType {
  GoKind kind;
  const GoType* elem;     // kMap / kSlice
  const GoField* fields;  // kStruct, declaration order
  int32_t n_fields;
};
constexpr int32_t name_len(const char* s) { return *s ? 1 + name_len(s + 1) : 0; }
struct GoField {
  constexpr GoField(const char* n, const GoType* t) : name(n), len(name_len(n)), type(t) {}
  const char* name;
  int32_t len;
  const GoType* type;
};

#define PAS_GO_STRUCT(T, ...)                                                     \
  const GoField T##_fields[] = {__VA_ARGS__};                                     \
  const GoType T{GoKind::kStruct, nullptr, T##_fields,                            \
                 (int32_t)(sizeof(T##_fields) / sizeof(GoField))}
#define PAS_GO_SLICE(T, E) const GoType T{GoKind::kSlice, &E, nullptr, 0}
#define PAS_GO_MAP(T, E) const GoType T{GoKind::kMap, &E, nullptr, 0}

const GoType String{GoKind::kString, nullptr, nullptr, 0};
const GoType Bool{GoKind::kBool, nullptr, nullptr, 0};
const GoType Int32{GoKind::kInt32, nullptr, nullptr, 0};
const GoType Int64{GoKind::kInt64, nullptr, nullptr, 0};
const GoType Quantity{GoKind::kQuantity, nullptr, nullptr, 0};
const GoType Time{GoKind::kTime, nullptr, nullptr, 0};
const GoType IntOrString{GoKind::kIntOrString, nullptr, nullptr, 0};
const GoType FieldsV1{GoKind::kRaw, nullptr, nullptr, 0};

PAS_GO_SLICE(StringSlice, String);
PAS_GO_SLICE(Int64Slice, Int64);
PAS_GO_MAP(StringMap, String);
PAS_GO_MAP(ResourceList, Quantity);  // map[ResourceName]resource.Quantity

// ---------------------------------------------------------------- apimachinery meta/v1
PAS_GO_STRUCT(OwnerReference, {"apiVersion", &String}, {"kind", &String}, {"name", &String},
              {"uid", &String}, {"controller", &Bool}, {"blockOwnerDeletion", &Bool});
PAS_GO_SLICE(OwnerReferenceSlice, OwnerReference);
PAS_GO_STRUCT(ManagedFieldsEntry, {"manager", &String}, {"operation", &String},
              {"apiVersion", &String}, {"time", &Time}, {"fieldsType", &String},
              {"fieldsV1", &FieldsV1}, {"subresource", &String});
PAS_GO_SLICE(ManagedFieldsEntrySlice, ManagedFieldsEntry);
// ObjectMeta (types.go): field order as declared
PAS_GO_STRUCT(ObjectMeta, {"name", &String}, {"generateName", &String}, {"namespace", &String},
              {"selfLink", &String}, {"uid", &String}, {"resourceVersion", &String},
              {"generation", &Int64}, {"creationTimestamp", &Time},
              {"deletionTimestamp", &Time}, {"deletionGracePeriodSeconds", &Int64},
              {"labels", &StringMap}, {"annotations", &StringMap},
              {"ownerReferences", &OwnerReferenceSlice}, {"finalizers", &StringSlice},
              {"clusterName", &String}, {"managedFields", &ManagedFieldsEntrySlice});
PAS_GO_STRUCT(ListMeta, {"selfLink", &String}, {"resourceVersion", &String},
              {"continue", &String}, {"remainingItemCount", &Int64});
PAS_GO_STRUCT(LabelSelectorRequirement, {"key", &String}, {"operator", &String},
              {"values", &StringSlice});
PAS_GO_SLICE(LabelSelectorRequirementSlice, LabelSelectorRequirement);
PAS_GO_STRUCT(LabelSelector, {"matchLabels", &StringMap},
              {"matchExpressions", &LabelSelectorRequirementSlice});

// ---------------------------------------------------------------- core/v1 shared pieces
PAS_GO_STRUCT(LocalObjectReference, {"name", &String});
PAS_GO_SLICE(LocalObjectReferenceSlice, LocalObjectReference);
PAS_GO_STRUCT(TypedLocalObjectReference, {"apiGroup", &String}, {"kind", &String},
              {"name", &String});
PAS_GO_STRUCT(ObjectFieldSelector, {"apiVersion", &String}, {"fieldPath", &String});
PAS_GO_STRUCT(ResourceFieldSelector, {"containerName", &String}, {"resource", &String},
              {"divisor", &Quantity});
PAS_GO_STRUCT(KeyToPath, {"key", &String}, {"path", &String}, {"mode", &Int32});
PAS_GO_SLICE(KeyToPathSlice, KeyToPath);
PAS_GO_STRUCT(ResourceRequirements, {"limits", &ResourceList}, {"requests", &ResourceList});

// ---------------------------------------------------------------- volumes
PAS_GO_STRUCT(HostPathVolumeSource, {"path", &String}, {"type", &String});
PAS_GO_STRUCT(EmptyDirVolumeSource, {"medium", &String}, {"sizeLimit", &Quantity});
PAS_GO_STRUCT(GCEPersistentDiskVolumeSource, {"pdName", &String}, {"fsType", &String},
              {"partition", &Int32}, {"readOnly", &Bool});
PAS_GO_STRUCT(AWSElasticBlockStoreVolumeSource, {"volumeID", &String}, {"fsType", &String},
              {"partition", &Int32}, {"readOnly", &Bool});
PAS_GO_STRUCT(GitRepoVolumeSource, {"repository", &String}, {"revision", &String},
              {"directory", &String});
PAS_GO_STRUCT(SecretVolumeSource, {"secretName", &String}, {"items", &KeyToPathSlice},
              {"defaultMode", &Int32}, {"optional", &Bool});
PAS_GO_STRUCT(NFSVolumeSource, {"server", &String}, {"path", &String}, {"readOnly", &Bool});
PAS_GO_STRUCT(ISCSIVolumeSource, {"targetPortal", &String}, {"iqn", &String}, {"lun", &Int32},
              {"iscsiInterface", &String}, {"fsType", &String}, {"readOnly", &Bool},
              {"portals", &StringSlice}, {"chapAuthDiscovery", &Bool},
              {"chapAuthSession", &Bool}, {"secretRef", &LocalObjectReference},
              {"initiatorName", &String});
PAS_GO_STRUCT(GlusterfsVolumeSource, {"endpoints", &String}, {"path", &String},
              {"readOnly", &Bool});
PAS_GO_STRUCT(PersistentVolumeClaimVolumeSource, {"claimName", &String}, {"readOnly", &Bool});
PAS_GO_STRUCT(RBDVolumeSource, {"monitors", &StringSlice}, {"image", &String},
              {"fsType", &String}, {"pool", &String}, {"user", &String}, {"keyring", &String},
              {"secretRef", &LocalObjectReference}, {"readOnly", &Bool});
PAS_GO_STRUCT(FlexVolumeSource, {"driver", &String}, {"fsType", &String},
              {"secretRef", &LocalObjectReference}, {"readOnly", &Bool},
              {"options", &StringMap});
PAS_GO_STRUCT(CinderVolumeSource, {"volumeID", &String}, {"fsType", &String},
              {"readOnly", &Bool}, {"secretRef", &LocalObjectReference});
PAS_GO_STRUCT(CephFSVolumeSource, {"monitors", &StringSlice}, {"path", &String},
              {"user", &String}, {"secretFile", &String}, {"secretRef", &LocalObjectReference},
              {"readOnly", &Bool});
PAS_GO_STRUCT(FlockerVolumeSource, {"datasetName", &String}, {"datasetUUID", &String});
PAS_GO_STRUCT(DownwardAPIVolumeFile, {"path", &String}, {"fieldRef", &ObjectFieldSelector},
              {"resourceFieldRef", &ResourceFieldSelector}, {"mode", &Int32});
PAS_GO_SLICE(DownwardAPIVolumeFileSlice, DownwardAPIVolumeFile);
PAS_GO_STRUCT(DownwardAPIVolumeSource, {"items", &DownwardAPIVolumeFileSlice},
              {"defaultMode", &Int32});
PAS_GO_STRUCT(FCVolumeSource, {"targetWWNs", &StringSlice}, {"lun", &Int32},
              {"fsType", &String}, {"readOnly", &Bool}, {"wwids", &StringSlice});
PAS_GO_STRUCT(AzureFileVolumeSource, {"secretName", &String}, {"shareName", &String},
              {"readOnly", &Bool});
PAS_GO_STRUCT(ConfigMapVolumeSource, {"name", &String}, {"items", &KeyToPathSlice},
              {"defaultMode", &Int32}, {"optional", &Bool});
PAS_GO_STRUCT(VsphereVirtualDiskVolumeSource, {"volumePath", &String}, {"fsType", &String},
              {"storagePolicyName", &String}, {"storagePolicyID", &String});
PAS_GO_STRUCT(QuobyteVolumeSource, {"registry", &String}, {"volume", &String},
              {"readOnly", &Bool}, {"user", &String}, {"group", &String}, {"tenant", &String});
PAS_GO_STRUCT(AzureDiskVolumeSource, {"diskName", &String}, {"diskURI", &String},
              {"cachingMode", &String}, {"fsType", &String}, {"readOnly", &Bool},
              {"kind", &String});
PAS_GO_STRUCT(PhotonPersistentDiskVolumeSource, {"pdID", &String}, {"fsType", &String});
PAS_GO_STRUCT(SecretProjection, {"name", &String}, {"items", &KeyToPathSlice},
              {"optional", &Bool});
PAS_GO_STRUCT(DownwardAPIProjection, {"items", &DownwardAPIVolumeFileSlice});
PAS_GO_STRUCT(ConfigMapProjection, {"name", &String}, {"items", &KeyToPathSlice},
              {"optional", &Bool});
PAS_GO_STRUCT(ServiceAccountTokenProjection, {"audience", &String},
              {"expirationSeconds", &Int64}, {"path", &String});
PAS_GO_STRUCT(VolumeProjection, {"secret", &SecretProjection},
              {"downwardAPI", &DownwardAPIProjection}, {"configMap", &ConfigMapProjection},
              {"serviceAccountToken", &ServiceAccountTokenProjection});
PAS_GO_SLICE(VolumeProjectionSlice, VolumeProjection);
PAS_GO_STRUCT(ProjectedVolumeSource, {"sources", &VolumeProjectionSlice},
              {"defaultMode", &Int32});
PAS_GO_STRUCT(PortworxVolumeSource, {"volumeID", &String}, {"fsType", &String},
              {"readOnly", &Bool});
PAS_GO_STRUCT(ScaleIOVolumeSource, {"gateway", &String}, {"system", &String},
              {"secretRef", &LocalObjectReference}, {"sslEnabled", &Bool},
              {"protectionDomain", &String}, {"storagePool", &String},
              {"storageMode", &String}, {"volumeName", &String}, {"fsType", &String},
              {"readOnly", &Bool});
PAS_GO_STRUCT(StorageOSVolumeSource, {"volumeName", &String}, {"volumeNamespace", &String},
              {"fsType", &String}, {"readOnly", &Bool}, {"secretRef", &LocalObjectReference});
PAS_GO_STRUCT(CSIVolumeSource, {"driver", &String}, {"readOnly", &Bool}, {"fsType", &String},
              {"volumeAttributes", &StringMap}, {"nodePublishSecretRef", &LocalObjectReference});
PAS_GO_STRUCT(PersistentVolumeClaimSpec, {"accessModes", &StringSlice},
              {"selector", &LabelSelector}, {"resources", &ResourceRequirements},
              {"volumeName", &String}, {"storageClassName", &String}, {"volumeMode", &String},
              {"dataSource", &TypedLocalObjectReference},
              {"dataSourceRef", &TypedLocalObjectReference});
PAS_GO_STRUCT(PersistentVolumeClaimTemplate, {"metadata", &ObjectMeta},
              {"spec", &PersistentVolumeClaimSpec});
PAS_GO_STRUCT(EphemeralVolumeSource, {"volumeClaimTemplate", &PersistentVolumeClaimTemplate});
// Volume: name + VolumeSource inline
PAS_GO_STRUCT(Volume, {"name", &String}, {"hostPath", &HostPathVolumeSource},
              {"emptyDir", &EmptyDirVolumeSource},
              {"gcePersistentDisk", &GCEPersistentDiskVolumeSource},
              {"awsElasticBlockStore", &AWSElasticBlockStoreVolumeSource},
              {"gitRepo", &GitRepoVolumeSource}, {"secret", &SecretVolumeSource},
              {"nfs", &NFSVolumeSource}, {"iscsi", &ISCSIVolumeSource},
              {"glusterfs", &GlusterfsVolumeSource},
              {"persistentVolumeClaim", &PersistentVolumeClaimVolumeSource},
              {"rbd", &RBDVolumeSource}, {"flexVolume", &FlexVolumeSource},
              {"cinder", &CinderVolumeSource}, {"cephfs", &CephFSVolumeSource},
              {"flocker", &FlockerVolumeSource}, {"downwardAPI", &DownwardAPIVolumeSource},
              {"fc", &FCVolumeSource}, {"azureFile", &AzureFileVolumeSource},
              {"configMap", &ConfigMapVolumeSource},
              {"vsphereVolume", &VsphereVirtualDiskVolumeSource},
              {"quobyte", &QuobyteVolumeSource}, {"azureDisk", &AzureDiskVolumeSource},
              {"photonPersistentDisk", &PhotonPersistentDiskVolumeSource},
              {"projected", &ProjectedVolumeSource}, {"portworxVolume", &PortworxVolumeSource},
              {"scaleIO", &ScaleIOVolumeSource}, {"storageos", &StorageOSVolumeSource},
              {"csi", &CSIVolumeSource}, {"ephemeral", &EphemeralVolumeSource});
PAS_GO_SLICE(VolumeSlice, Volume);

// ---------------------------------------------------------------- containers
PAS_GO_STRUCT(ContainerPort, {"name", &String}, {"hostPort", &Int32},
              {"containerPort", &Int32}, {"protocol", &String}, {"hostIP", &String});
PAS_GO_SLICE(ContainerPortSlice, ContainerPort);
PAS_GO_STRUCT(ConfigMapEnvSource, {"name", &String}, {"optional", &Bool});
PAS_GO_STRUCT(SecretEnvSource, {"name", &String}, {"optional", &Bool});
PAS_GO_STRUCT(EnvFromSource, {"prefix", &String}, {"configMapRef", &ConfigMapEnvSource},
              {"secretRef", &SecretEnvSource});
PAS_GO_SLICE(EnvFromSourceSlice, EnvFromSource);
PAS_GO_STRUCT(ConfigMapKeySelector, {"name", &String}, {"key", &String}, {"optional", &Bool});
PAS_GO_STRUCT(SecretKeySelector, {"name", &String}, {"key", &String}, {"optional", &Bool});
PAS_GO_STRUCT(EnvVarSource, {"fieldRef", &ObjectFieldSelector},
              {"resourceFieldRef", &ResourceFieldSelector},
              {"configMapKeyRef", &ConfigMapKeySelector}, {"secretKeyRef", &SecretKeySelector});
PAS_GO_STRUCT(EnvVar, {"name", &String}, {"value", &String}, {"valueFrom", &EnvVarSource});
PAS_GO_SLICE(EnvVarSlice, EnvVar);
PAS_GO_STRUCT(VolumeMount, {"name", &String}, {"readOnly", &Bool}, {"mountPath", &String},
              {"subPath", &String}, {"mountPropagation", &String}, {"subPathExpr", &String});
PAS_GO_SLICE(VolumeMountSlice, VolumeMount);
PAS_GO_STRUCT(VolumeDevice, {"name", &String}, {"devicePath", &String});
PAS_GO_SLICE(VolumeDeviceSlice, VolumeDevice);
PAS_GO_STRUCT(ExecAction, {"command", &StringSlice});
PAS_GO_STRUCT(HTTPHeader, {"name", &String}, {"value", &String});
PAS_GO_SLICE(HTTPHeaderSlice, HTTPHeader);
PAS_GO_STRUCT(HTTPGetAction, {"path", &String}, {"port", &IntOrString}, {"host", &String},
              {"scheme", &String}, {"httpHeaders", &HTTPHeaderSlice});
PAS_GO_STRUCT(TCPSocketAction, {"port", &IntOrString}, {"host", &String});
PAS_GO_STRUCT(Handler, {"exec", &ExecAction}, {"httpGet", &HTTPGetAction},
              {"tcpSocket", &TCPSocketAction});
// Probe: Handler inline (v0.22 has no gRPC action)
PAS_GO_STRUCT(Probe, {"exec", &ExecAction}, {"httpGet", &HTTPGetAction},
              {"tcpSocket", &TCPSocketAction}, {"initialDelaySeconds", &Int32},
              {"timeoutSeconds", &Int32}, {"periodSeconds", &Int32},
              {"successThreshold", &Int32}, {"failureThreshold", &Int32},
              {"terminationGracePeriodSeconds", &Int64});
PAS_GO_STRUCT(Lifecycle, {"postStart", &Handler}, {"preStop", &Handler});
PAS_GO_STRUCT(Capabilities, {"add", &StringSlice}, {"drop", &StringSlice});
PAS_GO_STRUCT(SELinuxOptions, {"user", &String}, {"role", &String}, {"type", &String},
              {"level", &String});
PAS_GO_STRUCT(WindowsSecurityContextOptions, {"gmsaCredentialSpecName", &String},
              {"gmsaCredentialSpec", &String}, {"runAsUserName", &String},
              {"hostProcess", &Bool});
PAS_GO_STRUCT(SeccompProfile, {"type", &String}, {"localhostProfile", &String});
PAS_GO_STRUCT(SecurityContext, {"capabilities", &Capabilities}, {"privileged", &Bool},
              {"seLinuxOptions", &SELinuxOptions},
              {"windowsOptions", &WindowsSecurityContextOptions}, {"runAsUser", &Int64},
              {"runAsGroup", &Int64}, {"runAsNonRoot", &Bool},
              {"readOnlyRootFilesystem", &Bool}, {"allowPrivilegeEscalation", &Bool},
              {"procMount", &String}, {"seccompProfile", &SeccompProfile});
#define PAS_GO_CONTAINER_FIELDS                                                            \
  {"name", &String}, {"image", &String}, {"command", &StringSlice}, {"args", &StringSlice}, \
      {"workingDir", &String}, {"ports", &ContainerPortSlice},                             \
      {"envFrom", &EnvFromSourceSlice}, {"env", &EnvVarSlice},                             \
      {"resources", &ResourceRequirements}, {"volumeMounts", &VolumeMountSlice},           \
      {"volumeDevices", &VolumeDeviceSlice}, {"livenessProbe", &Probe},                    \
      {"readinessProbe", &Probe}, {"startupProbe", &Probe}, {"lifecycle", &Lifecycle},     \
      {"terminationMessagePath", &String}, {"terminationMessagePolicy", &String},          \
      {"imagePullPolicy", &String}, {"securityContext", &SecurityContext},                 \
      {"stdin", &Bool}, {"stdinOnce", &Bool}, {"tty", &Bool}
PAS_GO_STRUCT(Container, PAS_GO_CONTAINER_FIELDS);
PAS_GO_SLICE(ContainerSlice, Container);
// EphemeralContainer: EphemeralContainerCommon inline (Container's fields) + target
PAS_GO_STRUCT(EphemeralContainer, PAS_GO_CONTAINER_FIELDS, {"targetContainerName", &String});
PAS_GO_SLICE(EphemeralContainerSlice, EphemeralContainer);
#undef PAS_GO_CONTAINER_FIELDS

// ---------------------------------------------------------------- pod spec
PAS_GO_STRUCT(Sysctl, {"name", &String}, {"value", &String});
PAS_GO_SLICE(SysctlSlice, Sysctl);
PAS_GO_STRUCT(PodSecurityContext, {"seLinuxOptions", &SELinuxOptions},
              {"windowsOptions", &WindowsSecurityContextOptions}, {"runAsUser", &Int64},
              {"runAsGroup", &Int64}, {"runAsNonRoot", &Bool},
              {"supplementalGroups", &Int64Slice}, {"fsGroup", &Int64},
              {"sysctls", &SysctlSlice}, {"fsGroupChangePolicy", &String},
              {"seccompProfile", &SeccompProfile});
PAS_GO_STRUCT(NodeSelectorRequirement, {"key", &String}, {"operator", &String},
              {"values", &StringSlice});
PAS_GO_SLICE(NodeSelectorRequirementSlice, NodeSelectorRequirement);
PAS_GO_STRUCT(NodeSelectorTerm, {"matchExpressions", &NodeSelectorRequirementSlice},
              {"matchFields", &NodeSelectorRequirementSlice});
PAS_GO_SLICE(NodeSelectorTermSlice, NodeSelectorTerm);
PAS_GO_STRUCT(NodeSelector, {"nodeSelectorTerms", &NodeSelectorTermSlice});
PAS_GO_STRUCT(PreferredSchedulingTerm, {"weight", &Int32}, {"preference", &NodeSelectorTerm});
PAS_GO_SLICE(PreferredSchedulingTermSlice, PreferredSchedulingTerm);
PAS_GO_STRUCT(NodeAffinity, {"requiredDuringSchedulingIgnoredDuringExecution", &NodeSelector},
              {"preferredDuringSchedulingIgnoredDuringExecution",
               &PreferredSchedulingTermSlice});
PAS_GO_STRUCT(PodAffinityTerm, {"labelSelector", &LabelSelector},
              {"namespaces", &StringSlice}, {"topologyKey", &String},
              {"namespaceSelector", &LabelSelector});
PAS_GO_SLICE(PodAffinityTermSlice, PodAffinityTerm);
PAS_GO_STRUCT(WeightedPodAffinityTerm, {"weight", &Int32},
              {"podAffinityTerm", &PodAffinityTerm});
PAS_GO_SLICE(WeightedPodAffinityTermSlice, WeightedPodAffinityTerm);
PAS_GO_STRUCT(PodAffinity,
              {"requiredDuringSchedulingIgnoredDuringExecution", &PodAffinityTermSlice},
              {"preferredDuringSchedulingIgnoredDuringExecution",
               &WeightedPodAffinityTermSlice});
PAS_GO_STRUCT(PodAntiAffinity,
              {"requiredDuringSchedulingIgnoredDuringExecution", &PodAffinityTermSlice},
              {"preferredDuringSchedulingIgnoredDuringExecution",
               &WeightedPodAffinityTermSlice});
PAS_GO_STRUCT(Affinity, {"nodeAffinity", &NodeAffinity}, {"podAffinity", &PodAffinity},
              {"podAntiAffinity", &PodAntiAffinity});
PAS_GO_STRUCT(Toleration, {"key", &String}, {"operator", &String}, {"value", &String},
              {"effect", &String}, {"tolerationSeconds", &Int64});
PAS_GO_SLICE(TolerationSlice, Toleration);
PAS_GO_STRUCT(HostAlias, {"ip", &String}, {"hostnames", &StringSlice});
PAS_GO_SLICE(HostAliasSlice, HostAlias);
PAS_GO_STRUCT(PodDNSConfigOption, {"name", &String}, {"value", &String});
PAS_GO_SLICE(PodDNSConfigOptionSlice, PodDNSConfigOption);
PAS_GO_STRUCT(PodDNSConfig, {"nameservers", &StringSlice}, {"searches", &StringSlice},
              {"options", &PodDNSConfigOptionSlice});
PAS_GO_STRUCT(PodReadinessGate, {"conditionType", &String});
PAS_GO_SLICE(PodReadinessGateSlice, PodReadinessGate);
PAS_GO_STRUCT(TopologySpreadConstraint, {"maxSkew", &Int32}, {"topologyKey", &String},
              {"whenUnsatisfiable", &String}, {"labelSelector", &LabelSelector});
PAS_GO_SLICE(TopologySpreadConstraintSlice, TopologySpreadConstraint);
PAS_GO_STRUCT(PodSpec, {"volumes", &VolumeSlice}, {"initContainers", &ContainerSlice},
              {"containers", &ContainerSlice},
              {"ephemeralContainers", &EphemeralContainerSlice}, {"restartPolicy", &String},
              {"terminationGracePeriodSeconds", &Int64}, {"activeDeadlineSeconds", &Int64},
              {"dnsPolicy", &String}, {"nodeSelector", &StringMap},
              {"serviceAccountName", &String}, {"serviceAccount", &String},
              {"automountServiceAccountToken", &Bool}, {"nodeName", &String},
              {"hostNetwork", &Bool}, {"hostPID", &Bool}, {"hostIPC", &Bool},
              {"shareProcessNamespace", &Bool}, {"securityContext", &PodSecurityContext},
              {"imagePullSecrets", &LocalObjectReferenceSlice}, {"hostname", &String},
              {"subdomain", &String}, {"affinity", &Affinity}, {"schedulerName", &String},
              {"tolerations", &TolerationSlice}, {"hostAliases", &HostAliasSlice},
              {"priorityClassName", &String}, {"priority", &Int32},
              {"dnsConfig", &PodDNSConfig}, {"readinessGates", &PodReadinessGateSlice},
              {"runtimeClassName", &String}, {"enableServiceLinks", &Bool},
              {"preemptionPolicy", &String}, {"overhead", &ResourceList},
              {"topologySpreadConstraints", &TopologySpreadConstraintSlice},
              {"setHostnameAsFQDN", &Bool});

// ---------------------------------------------------------------- pod status
PAS_GO_STRUCT(PodCondition, {"type", &String}, {"status", &String},
              {"lastProbeTime", &Time}, {"lastTransitionTime", &Time}, {"reason", &String},
              {"message", &String});
PAS_GO_SLICE(PodConditionSlice, PodCondition);
PAS_GO_STRUCT(PodIP, {"ip", &String});
PAS_GO_SLICE(PodIPSlice, PodIP);
PAS_GO_STRUCT(ContainerStateWaiting, {"reason", &String}, {"message", &String});
PAS_GO_STRUCT(ContainerStateRunning, {"startedAt", &Time});
PAS_GO_STRUCT(ContainerStateTerminated, {"exitCode", &Int32}, {"signal", &Int32},
              {"reason", &String}, {"message", &String}, {"startedAt", &Time},
              {"finishedAt", &Time}, {"containerID", &String});
PAS_GO_STRUCT(ContainerState, {"waiting", &ContainerStateWaiting},
              {"running", &ContainerStateRunning}, {"terminated", &ContainerStateTerminated});
PAS_GO_STRUCT(ContainerStatus, {"name", &String}, {"state", &ContainerState},
              {"lastState", &ContainerState}, {"ready", &Bool}, {"restartCount", &Int32},
              {"image", &String}, {"imageID", &String}, {"containerID", &String},
              {"started", &Bool});
PAS_GO_SLICE(ContainerStatusSlice, ContainerStatus);
PAS_GO_STRUCT(PodStatus, {"phase", &String}, {"conditions", &PodConditionSlice},
              {"message", &String}, {"reason", &String}, {"nominatedNodeName", &String},
              {"hostIP", &String}, {"podIP", &String}, {"podIPs", &PodIPSlice},
              {"startTime", &Time}, {"initContainerStatuses", &ContainerStatusSlice},
              {"containerStatuses", &ContainerStatusSlice}, {"qosClass", &String},
              {"ephemeralContainerStatuses", &ContainerStatusSlice});
// Pod: TypeMeta inline (kind, apiVersion)
PAS_GO_STRUCT(Pod, {"kind", &String}, {"apiVersion", &String}, {"metadata", &ObjectMeta},
              {"spec", &PodSpec}, {"status", &PodStatus});

// ---------------------------------------------------------------- node
PAS_GO_STRUCT(Taint, {"key", &String}, {"value", &String}, {"effect", &String},
              {"timeAdded", &Time});
PAS_GO_SLICE(TaintSlice, Taint);
PAS_GO_STRUCT(ConfigMapNodeConfigSource, {"namespace", &String}, {"name", &String},
              {"uid", &String}, {"resourceVersion", &String}, {"kubeletConfigKey", &String});
PAS_GO_STRUCT(NodeConfigSource, {"configMap", &ConfigMapNodeConfigSource});
PAS_GO_STRUCT(NodeSpec, {"podCIDR", &String}, {"podCIDRs", &StringSlice},
              {"providerID", &String}, {"unschedulable", &Bool}, {"taints", &TaintSlice},
              {"configSource", &NodeConfigSource}, {"externalID", &String});
PAS_GO_STRUCT(NodeCondition, {"type", &String}, {"status", &String},
              {"lastHeartbeatTime", &Time}, {"lastTransitionTime", &Time},
              {"reason", &String}, {"message", &String});
PAS_GO_SLICE(NodeConditionSlice, NodeCondition);
PAS_GO_STRUCT(NodeAddress, {"type", &String}, {"address", &String});
PAS_GO_SLICE(NodeAddressSlice, NodeAddress);
PAS_GO_STRUCT(DaemonEndpoint, {"Port", &Int32});  // `json:"Port"`
PAS_GO_STRUCT(NodeDaemonEndpoints, {"kubeletEndpoint", &DaemonEndpoint});
PAS_GO_STRUCT(NodeSystemInfo, {"machineID", &String}, {"systemUUID", &String},
              {"bootID", &String}, {"kernelVersion", &String}, {"osImage", &String},
              {"containerRuntimeVersion", &String}, {"kubeletVersion", &String},
              {"kubeProxyVersion", &String}, {"operatingSystem", &String},
              {"architecture", &String});
PAS_GO_STRUCT(ContainerImage, {"names", &StringSlice}, {"sizeBytes", &Int64});
PAS_GO_SLICE(ContainerImageSlice, ContainerImage);
PAS_GO_STRUCT(AttachedVolume, {"name", &String}, {"devicePath", &String});
PAS_GO_SLICE(AttachedVolumeSlice, AttachedVolume);
PAS_GO_STRUCT(NodeConfigStatus, {"assigned", &NodeConfigSource}, {"active", &NodeConfigSource},
              {"lastKnownGood", &NodeConfigSource}, {"error", &String});
PAS_GO_STRUCT(NodeStatus, {"capacity", &ResourceList}, {"allocatable", &ResourceList},
              {"phase", &String}, {"conditions", &NodeConditionSlice},
              {"addresses", &NodeAddressSlice}, {"daemonEndpoints", &NodeDaemonEndpoints},
              {"nodeInfo", &NodeSystemInfo}, {"images", &ContainerImageSlice},
              {"volumesInUse", &StringSlice}, {"volumesAttached", &AttachedVolumeSlice},
              {"config", &NodeConfigStatus});
// Node: TypeMeta inline
PAS_GO_STRUCT(Node, {"kind", &String}, {"apiVersion", &String}, {"metadata", &ObjectMeta},
              {"spec", &NodeSpec}, {"status", &NodeStatus});

#undef PAS_GO_STRUCT
#undef PAS_GO_SLICE
#undef PAS_GO_MAP

}  // namespace pas_schema
