/*
 * pas.h — C-ABI of the MI355X-native Platform Aware Scheduling evaluator.
 *
 * This is the drop-in boundary beneath the reference's extender.Scheduler
 * HTTP verbs (extender/types.go:11-15; registered at extender/scheduler.go:86-91).
 * The Go handlers keep decoding extender.Args and encoding FilterResult /
 * HostPriorityList; the compute they do per request is replaced by the batched
 * entry points below (cgo binding shown in INTEGRATION.md).
 *
 * Conventions
 *   - Plain C types only; no exceptions or aborts cross this boundary.
 *   - Every function returns a pas_status (0 = OK, negative = error) and leaves a
 *     message retrievable with pas_last_error(ctx).
 *   - Host-pointer entry points copy their inputs in and results out and return
 *     when the results are in host memory.  *_device entry points take device
 *     pointers and a hipStream_t (as void*) and return once the work is enqueued.
 *   - A pas_ctx is NOT thread safe: callers serialise calls per context (the GAS
 *     extender already holds GASExtender.rwmutex around filter/bind,
 *     gpu-aware-scheduling/pkg/gpuscheduler/scheduler.go:463-465).
 *   - Bitmaps are little-endian uint64 words, node n at bit (n & 63) of word n >> 6;
 *     W64(n) = (n + 63) / 64 words per row, bits >= n_nodes are zero.
 *   - Metric values are int64 fixed-point columns: column m holds value * 10^scale[m] of
 *     the reference's resource.Quantity (telemetry-aware-scheduling/pkg/metrics/
 *     client.go:25-29), scale 3 ("milli") unless pas_tas_snapshot_set_scale says otherwise.
 *     ParseQuantity keeps at most 9 fractional digits (it rounds to 1e-9), so a column with
 *     scale = the most decimal places of its values (pas_quantity_decimals, 0..9) is exact;
 *     pas_quantity_to_scaled() converts a Quantity string and reports PAS_ENOTEXACT only
 *     when value * 10^scale is outside int64.
 */
#ifndef PAS_H_
#define PAS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PAS_ABI_VERSION 3

typedef enum pas_status {
  PAS_OK = 0,
  PAS_EINVAL = -1,     /* bad argument (shape, operator, null pointer) */
  PAS_ESTALE = -2,     /* generation mismatch between call and resident snapshot */
  PAS_ENOTEXACT = -3,  /* a value is not representable as exact int64 milli */
  PAS_EDEVICE = -4,    /* HIP runtime error */
  PAS_ENOMEM = -5,     /* device or host allocation failed */
  PAS_ENOSNAP = -6,    /* no snapshot uploaded yet */
  PAS_ECAPACITY = -7,  /* shape exceeds a documented kernel limit / an output buffer */
  PAS_EDECODE = -8     /* request body that json.Decoder.Decode(&args) rejects */
} pas_status;

/* TASPolicyRule.Operator (telemetrypolicy/api/v1alpha1/types.go:31-35), evaluated as
 * in core.EvaluateRule (strategies/core/operator.go:13-26).  Any other string panics
 * in the reference (operator.go:25: nil map entry); here it is PAS_EINVAL. */
typedef enum pas_op {
  PAS_OP_LESS_THAN = 0,
  PAS_OP_GREATER_THAN = 1,
  PAS_OP_EQUALS = 2
} pas_op;

/* One TASPolicyRule with the metric name resolved to a snapshot column.
 * metric < 0 or >= n_metrics means "metric not in the cache": the rule is skipped,
 * as dontschedule.Violated does on a ReadMetric error (dontschedule/strategy.go:28-32). */
typedef struct pas_rule {
  int32_t metric;
  int32_t op;      /* pas_op */
  int64_t target;  /* TASPolicyRule.Target, integer units (NOT milli) */
} pas_rule;

typedef struct pas_config {
  int32_t device;    /* HIP device ordinal; -1 = current device */
  int32_t reserved;  /* must be 0 */
} pas_config;

typedef struct pas_ctx pas_ctx;

int pas_abi_version(void);

/* Context: owns one HIP stream (replaceable with pas_set_stream), the resident
 * snapshots and scratch. */
int pas_create(const pas_config* cfg, pas_ctx** out);
void pas_destroy(pas_ctx* ctx);
const char* pas_last_error(const pas_ctx* ctx);
int pas_set_stream(pas_ctx* ctx, void* hip_stream); /* NULL = the context's own stream */
/* A hip_stream argument (here and in every _device entry point) of NULL names the context's
 * current stream; PAS_STREAM_NULL names the HIP null stream (e.g. torch's default stream).
 * Evaluation calls may be issued on several streams without host synchronisation: the
 * context keeps per-stream scratch (calls on two or more streams in turn overlap), orders a
 * call after the last user of the scratch it takes over, and orders readers of data it
 * derives from a snapshot after that data's build.  A call that CHANGES a resident snapshot
 * (snapshot_set, snapshot_update, gas_bind, gas_release) must be ordered by the caller after
 * the calls on other streams that still read it. */
#define PAS_STREAM_NULL ((void*)1)
/* Waits for the context's stream and for the last calls on every other stream the context
 * ran on (and the GAS fits' internal side streams).  Returns PAS_EDEVICE when a GAS fit
 * enqueued since the last report could not complete: one of its internal stream waits gave
 * up (pas_gas_fit_device: its outputs are not to be used); the report is cleared, so the
 * next call starts clean.  The host-pointer GAS forms report this themselves. */
int pas_synchronize(pas_ctx* ctx);

/* Operator string -> pas_op ("LessThan", "GreaterThan", "Equals"), else PAS_EINVAL.
 * Replaces the map lookup in core.EvaluateRule (operator.go:14-25). */
int pas_parse_operator(const char* op);

/* resource.Quantity string -> the parsed quantity's value * 1000, exactly.  Parsing is
 * resource.ParseQuantity of k8s.io/apimachinery v0.22.2 (sign, digits, optional fraction,
 * suffix n u m k M G T P E Ki Mi Gi Ti Pi Ei or e/E exponent), including its inf.Dec
 * path: values it cannot hold as int64Amount are rounded away from zero to 1e-9 and
 * capped at +-(2^63 - 1) — the value core.EvaluateRule compares (operator.go:16-22).
 * PAS_ENOTEXACT if that value has sub-milli precision or is outside int64 milli range;
 * PAS_EINVAL if ParseQuantity would fail. */
int pas_quantity_to_milli(const char* quantity, int64_t* milli_out);
/* The same at any decimal scale: value * 10^places exactly, 0 <= places <= 9 (EINVAL
 * otherwise); PAS_ENOTEXACT if that is not an integer or is outside int64.
 * pas_quantity_to_milli is places = 3. */
int pas_quantity_to_scaled(const char* quantity, int32_t places, int64_t* out);
/* The fewest decimal places (0..9) that hold the parsed value exactly: "1500u" -> 4,
 * "0.0005" -> 4, "1e-7" -> 7, "2k" -> 0, "1.5" -> 1. */
int pas_quantity_decimals(const char* quantity, int32_t* places);

/* resource.ParseQuantity(quantity).AsInt64() with `ok` ignored, as the reference uses it
 * (gpuscheduler/utils.go:23, scheduler.go:155).  That is 0 — even for integral values —
 * for an inf.Dec-backed quantity (19 or more significant digits, a fraction with a
 * binary suffix, a binary suffix past the int64Amount precision estimate such as "1Pi",
 * scale below nano) and for an int64Amount with negative scale ("1000m", "10.0");
 * value * 10^scale (0 on overflow) otherwise.  Pass the string the informer decoded: the
 * apiserver stores quantities in canonical form ("1000m" arrives as "1").
 * PAS_EINVAL if ParseQuantity would fail. */
int pas_quantity_as_int64(const char* quantity, int64_t* out);

/* ------------------------------------------------------------------------- */
/* Telemetry Aware Scheduling                                                */
/* ------------------------------------------------------------------------- */

/* Upload a node-metric snapshot: the content of AutoUpdatingCache's
 * "metrics/<name>" entries (cache/autoupdating.go:76-85) as SoA columns.
 *   v_milli [n_metrics][n_nodes]      value * 1000 (ignored where not present), or
 *                                     value * 10^scale[m] with pas_tas_snapshot_set_scale
 *   present [n_metrics][W64(n_nodes)] node has this metric (NodeMetricsInfo key set)
 * The device builds per-metric sorted orders once here, so that per-request
 * evaluation never sorts (core.OrderedList, operator.go:30-42, sorts per request).
 * gen is an opaque generation id checked by the eval calls (PAS_ESTALE). */
int pas_tas_snapshot_set(pas_ctx* ctx, uint64_t gen, int32_t n_nodes, int32_t n_metrics,
                         const int64_t* v_milli, const uint64_t* present);
int pas_tas_snapshot_set_device(pas_ctx* ctx, uint64_t gen, int32_t n_nodes, int32_t n_metrics,
                                const int64_t* d_v_milli, const uint64_t* d_present,
                                void* hip_stream);
int pas_tas_snapshot_info(const pas_ctx* ctx, uint64_t* gen, int32_t* n_nodes,
                          int32_t* n_metrics);

/* Decimal scale of each column of the resident snapshot generation gen: column m holds
 * value * 10^col_scale[m] (0 <= col_scale[m] <= 9, host array of n_metrics = the snapshot's
 * metric count).  Every column is 3 (milli) after pas_tas_snapshot_set[_device]; a column
 * refresh keeps the column's scale.  Rule targets are integers (TASPolicyRule.Target,
 * telemetrypolicy/api/v1alpha1/types.go:31-35), so core.EvaluateRule's CmpInt64
 * (operator.go:16-22) is exact against target * 10^scale (saturated past int64), and
 * OrderedList's Cmp (:37,39) is the integer order of one column: sub-milli metric values
 * evaluate on the device exactly.  Order this call after evaluations on
 * other streams that still read the snapshot, as a snapshot change; it is synchronous on
 * hip_stream (NULL: the context's stream). */
int pas_tas_snapshot_set_scale(pas_ctx* ctx, uint64_t gen, int32_t n_metrics,
                               const int32_t* col_scale, void* hip_stream);

/* Column refresh: AutoUpdatingCache.updateMetric replaces one metric's whole node map
 * (cache/autoupdating.go:45-73, WriteMetric :100-112).  Replaces the resident snapshot's
 * columns cols[0 .. n_cols) (distinct metric indices, host array) with
 * v_milli[n_cols][n_nodes] / present[n_cols][W64] and rebuilds only their orders; the
 * snapshot moves from generation gen_from (PAS_ESTALE otherwise) to gen_to.  Node count and
 * metric count are unchanged (a new node or metric column needs pas_tas_snapshot_set).
 * The _device form is asynchronous on hip_stream except for the copy of cols. */
int pas_tas_snapshot_update(pas_ctx* ctx, uint64_t gen_from, uint64_t gen_to, int32_t n_cols,
                            const int32_t* cols, const int64_t* v_milli,
                            const uint64_t* present);
int pas_tas_snapshot_update_device(pas_ctx* ctx, uint64_t gen_from, uint64_t gen_to,
                                   int32_t n_cols, const int32_t* cols, const int64_t* d_v_milli,
                                   const uint64_t* d_present, void* hip_stream);

#define PAS_TAS_FILTER 1u      /* produce pass_out (MetricsExtender.filterNodes) */
#define PAS_TAS_PRIORITIZE 2u  /* produce order_out/order_len (prioritizeNodesForRule) */

/* Batched TAS filter + prioritize for n_pods pending pods against the resident
 * snapshot.  Replaces, per pod:
 *   filter:     dontschedule.Strategy.Violated (dontschedule/strategy.go:25-44) and the
 *               candidate loop of MetricsExtender.filterNodes (telemetryscheduler.go:204-211)
 *   prioritize: prioritizeNodesForRule (telemetryscheduler.go:128-149) with
 *               core.OrderedList (operator.go:30-42).
 * Inputs
 *   rules, rule_off  CSR of each pod's dontschedule rules: pod p owns
 *                    rules[rule_off[p] .. rule_off[p+1])
 *   prio             [n_pods] scheduleonmetric Rules[0] (getSchedulingRule,
 *                    telemetryscheduler.go:115-124); metric < 0 = no rule / missing metric
 *   cand             [n_pods][W64] candidate bitmaps (args.Nodes), or NULL = every node
 * Outputs
 *   pass_out   [n_pods][W64]  cand AND NOT violated            (flag PAS_TAS_FILTER)
 *   order_out  [n_pods][n_nodes], order_len [n_pods]           (flag PAS_TAS_PRIORITIZE)
 *              node indices of prioritize candidates that have the metric, best first;
 *              HostPriority.Score of entry i is 10 - i (telemetryscheduler.go:145).
 *              Candidates are pass_out when PAS_TAS_FILTER is also set (kube-scheduler
 *              prioritizes the filter-feasible nodes), else cand.
 * Order (the reference's is Go-map order + unstable sort.Slice, i.e. unspecified for
 * ties and for operators other than LessThan/GreaterThan): GreaterThan = value
 * descending, LessThan = value ascending, ties by ascending node index; any other
 * operator = ascending node index.  The oracle uses the same rule.
 * The _device form cannot check d_rule_off on the host: each pod's span is read clamped,
 * [a, b) with a = clamp(rule_off[p], 0, n_rules), b = clamp(rule_off[p+1], a, n_rules), so an
 * offset array that is not a CSR never takes a kernel outside the rules. */
int pas_tas_eval(pas_ctx* ctx, uint64_t gen, int32_t n_pods, const pas_rule* rules,
                 const int32_t* rule_off, const pas_rule* prio, const uint64_t* cand,
                 uint32_t flags, uint64_t* pass_out, int32_t* order_out, int32_t* order_len);
int pas_tas_eval_device(pas_ctx* ctx, uint64_t gen, int32_t n_pods, int32_t n_rules,
                        const pas_rule* d_rules, const int32_t* d_rule_off,
                        const pas_rule* d_prio, const uint64_t* d_cand, uint32_t flags,
                        uint64_t* d_pass_out, int32_t* d_order_out, int32_t* d_order_len,
                        void* hip_stream);

/* Prioritize of ONE extender request in the request's own terms.  Replaces
 * prioritizeNodesForRule (telemetryscheduler.go:128-149) + core.OrderedList
 * (operator.go:30-42) for args.Nodes.Items given as
 *   req_node [n_req]  snapshot node index of Items[j] (pas_decode_args' req_node; -1 or any
 *                     index outside [0, n_nodes) = a node the snapshot does not hold)
 *   prio              the pod's scheduleonmetric Rules[0] (host struct); metric < 0 = no
 *                     rule / metric not cached -> empty list
 * Outputs
 *   pos_out  [n_req]  request positions j of the listed nodes, best first (-1 past len);
 *                     HostPriority i is {Items[pos_out[i]].Name, 10 - i}
 *   len_out           entries: the distinct request nodes that have the metric
 * Order: GreaterThan value descending, LessThan ascending, ties by ascending position of
 * the node's first occurrence in the request; any other operator: first occurrences in
 * request order.  (pas_tas_eval breaks ties by snapshot node index instead; the two agree
 * when the request lists nodes in snapshot order.)  A repeated name is listed once
 * (filteredNodeData is a map, :135-139).  The _device form takes device req_node /
 * pos_out / len_out and is asynchronous on hip_stream. */
int pas_tas_prioritize_request(pas_ctx* ctx, uint64_t gen, const pas_rule* prio, int32_t n_req,
                               const int32_t* req_node, int32_t* pos_out, int32_t* len_out);
int pas_tas_prioritize_request_device(pas_ctx* ctx, uint64_t gen, const pas_rule* prio,
                                      int32_t n_req, const int32_t* d_req_node,
                                      int32_t* d_pos_out, int32_t* d_len_out,
                                      void* hip_stream);

/* Deschedule sweep: for each registered deschedule strategy s (rules
 * rules[rule_off[s] .. rule_off[s+1])), the node set of deschedule.Strategy.Violated
 * (deschedule/strategy.go:31-50), as the bitmap viol_out[s][W64].  The per-node
 * policy lists of nodeStatusForStrategy (deschedule/enforce.go:154-164) are the
 * columns of this matrix.  The _device forms (and pas_tas_deschedule_device) read d_rule_off
 * clamped into [0, n_rules] and non-decreasing, in strategy order, so an offset array that is
 * not a CSR never takes the sweep outside the rules or the strategies. */
int pas_tas_violations(pas_ctx* ctx, uint64_t gen, int32_t n_strategies, const pas_rule* rules,
                       const int32_t* rule_off, uint64_t* viol_out);
int pas_tas_violations_device(pas_ctx* ctx, uint64_t gen, int32_t n_strategies,
                              int32_t n_rules, const pas_rule* d_rules,
                              const int32_t* d_rule_off, uint64_t* d_viol_out,
                              void* hip_stream);

/* Deschedule label plan (Deschedule.updateNodeLabels, deschedule/enforce.go:99-151) for
 * n_strategies <= 64 strategies from a sweep's viol[s][W64(n_nodes)] and the nodes' labels.
 * The reference keys its non-violated set by policy NAME (allPolicies, :89-95), and two
 * registered strategies may share a name (SetPolicyName drops the namespace,
 * controller/controller.go:80; AddStrategy drops only Equals duplicates,
 * core/enforcer.go:84-103):
 *   name_id      [s] host array: strategies s and t share a policy name iff
 *                name_id[s] == name_id[t] (any int32 values); NULL = all names distinct.
 *                A name is represented by its first strategy k (lowest index).
 *   labels       [s][W64] bit set = the node carries label <policy name of s> (any value);
 *                only the rows of each name's first strategy are read; NULL = no node
 *                carries any
 *   add_out      [n_nodes] bit s = strategy s violated at the node: add "<name>":
 *                "violating", one entry per violating strategy (:108-117)
 *   remove_out   [n_nodes] bit k = name k (its first strategy) violated by none of its
 *                strategies and carried: remove it, then add it as "null" (:118-132)
 *   total_out    the function's int result: the count of NON-violated (node, name) pairs
 *                (totalViolations++ sits in the non-violated loop, :133)
 * More than 64 strategies: call per group of <= 64 that keeps every name's strategies
 * together, OR the masks' strategy offsets back in and sum the totals (DescheduleEnforcer).
 * pas_label_patch_json renders one node's masks as the PATCH body.  The _device forms take
 * device viol / labels / outputs and a host name_id, and are asynchronous on hip_stream. */
int pas_tas_label_plan(pas_ctx* ctx, int32_t n_nodes, int32_t n_strategies,
                       const uint64_t* viol, const int32_t* name_id, const uint64_t* labels,
                       uint64_t* add_out, uint64_t* remove_out, int64_t* total_out);
int pas_tas_label_plan_device(pas_ctx* ctx, int32_t n_nodes, int32_t n_strategies,
                              const uint64_t* d_viol, const int32_t* name_id,
                              const uint64_t* d_labels, uint64_t* d_add_out,
                              uint64_t* d_remove_out, int64_t* d_total_out, void* hip_stream);

/* The deschedule sweep and its label plan in one pass (Deschedule.Cleanup's violation lists,
 * deschedule/strategy.go:31-50, then updateNodeLabels, enforce.go:99-151): outputs as
 * pas_tas_violations_device (viol_out) followed by pas_tas_label_plan_device on those
 * bitmaps for the snapshot's n_nodes (name_id / labels / add_out / remove_out / total_out),
 * without re-reading the bitmaps.  n_strategies <= 64. */
int pas_tas_deschedule_device(pas_ctx* ctx, uint64_t gen, int32_t n_strategies,
                              int32_t n_rules, const pas_rule* d_rules,
                              const int32_t* d_rule_off, uint64_t* d_viol_out,
                              const int32_t* name_id, const uint64_t* d_labels,
                              uint64_t* d_add_out, uint64_t* d_remove_out, int64_t* d_total_out,
                              void* hip_stream);

/* json.Marshal of the node's []patchValue (enforce.go:21-25, 74-86) for the masks of
 * pas_tas_label_plan: adds in strategy order, then a remove + add "null" pair per removed
 * label in the order of the names' first strategies (the reference emits these in Go-map
 * order).  names[s] = policy name of strategy s.  Writes at most cap bytes (no terminator); *len = full length;
 * PAS_ECAPACITY if it exceeds cap.  Host-only. */
int pas_label_patch_json(int32_t n_strategies, const char* const* names, uint64_t add_mask,
                         uint64_t remove_mask, char* buf, int64_t cap, int64_t* len);

/* ------------------------------------------------------------------------- */
/* GPU Aware Scheduling                                                      */
/* ------------------------------------------------------------------------- */

#define PAS_GAS_MAX_CARDS 64      /* cards per node (label gpu.intel.com/cards entries) */
#define PAS_GAS_MAX_RES 4         /* gpu.intel.com/ resource kinds per batch */
#define PAS_GAS_MAX_SELECTIONS 64 /* card selections per pod reported in cards / side records;
                                     pods with more are evaluated exactly (PAS_GAS_SEL_LIMIT) */
#define PAS_GAS_PACKED 8          /* selections / card ranks the packed result word holds */
#define PAS_REQ_UNKNOWN_KIND 0x80000000u /* req_mask: requests a kind the snapshot lacks */
/* bits 24-27 of a result word besides a count S <= PAS_GAS_PACKED: */
#define PAS_GAS_SEL_EXTENDED 15   /* the pod fits (bit 31 set) but its card selection does not
                                     pack: more than 8 selections or a card rank >= 8; the
                                     selection is in the side buffer of pas_gas_fit_ex */
#define PAS_GAS_SEL_LIMIT 14      /* the pod fits (bit 31 set) with more than
                                     PAS_GAS_MAX_SELECTIONS selections: neither packed nor in
                                     the side buffer; pas_gas_bind_counts reports them per
                                     container and card.  Such pods are counted by
                                     pas_gas_limit_count */

/* Card selection of one (pod, node) that does not fit the packed word (PAS_GAS_SEL_EXTENDED):
 * card[0 .. n_sel) are the ranks of the node's cards, selection by selection (containers in
 * order), i.e. the "gas-container-cards" annotation (:317-335). */
typedef struct pas_gas_selection {
  int32_t pod;
  int32_t node;
  int32_t n_sel;
  int32_t reserved;
  uint8_t card[PAS_GAS_MAX_SELECTIONS];
} pas_gas_selection;

/* Frozen allocation snapshot (Cache.getNodeResourceStatus,
 * gpuscheduler/node_resource_cache.go:474-491) in node-major SoA:
 *   n_cards     [n_nodes]  unique card names of label gpu.intel.com/cards; 0 = label
 *                          missing (getNodeGPUList -> nil, scheduler.go:132-148,
 *                          errWontFit at :294-298); -1 = node not in the lister
 *                          (FetchNode error, :282-288)
 *   cap_per_gpu [n_nodes][n_res]        AsInt64(allocatable) / len(label split),
 *                                       truncating (getPerGPUResourceCapacity :164-178);
 *                                       0 where the node lacks the resource
 *   used        [n_nodes][max_cards][n_res] usage of the node's cards in lexicographic
 *                                       (sort.Strings, :216-224) order of card name;
 *                                       cards in the usage map but not in the label are
 *                                       left out (skipped at :230-234)
 * max_cards <= PAS_GAS_MAX_CARDS (64), n_res <= PAS_GAS_MAX_RES.  The host form rejects
 * n_cards[n] > max_cards (PAS_EINVAL); the _device form stores such a count as max_cards. */
int pas_gas_snapshot_set(pas_ctx* ctx, uint64_t gen, int32_t n_nodes, int32_t max_cards,
                         int32_t n_res, const int32_t* n_cards, const int64_t* cap_per_gpu,
                         const int64_t* used);
int pas_gas_snapshot_set_device(pas_ctx* ctx, uint64_t gen, int32_t n_nodes, int32_t max_cards,
                                int32_t n_res, const int32_t* d_n_cards,
                                const int64_t* d_cap_per_gpu, const int64_t* d_used,
                                void* hip_stream);

/* GAS filter for a batch of pods over every node of the snapshot: one
 * runSchedulingLogic (scheduler.go:280-338) per (pod, node), first-fit over cards
 * with checkResourceCapacity (:341-383).
 *   req       [n_pods][max_containers][n_res] AsInt64 container requests
 *             (containerRequests, utils.go:14-32); res_index i915 identifies
 *             gpu.intel.com/i915 among the n_res kinds (or -1 if absent)
 *   req_mask  [n_pods][max_containers] bit q set = container requests kind q
 *             (the key exists in its resourceMap, even with value 0); bit 31
 *             (PAS_REQ_UNKNOWN_KIND) = the container also requests a gpu.intel.com/ kind
 *             outside the snapshot's n_res kinds.  No node's capacity map has that key, so
 *             every checkResourceCapacity of the container fails (:349-354): with
 *             numI915 > 0 the pod fits no node; with numI915 == 0 it makes no selection
 *             and the flag changes nothing (:206-215)
 *   n_containers [n_pods]
 * Output res_out[n_pods][n_nodes], one word per (pod, node):
 *   bit 31     the pod fits (node passes GASExtender.filterNodes, :467-473)
 *   bits 24-27 number of card selections S (= sum of per-container i915 counts) when
 *              S <= 8 and every selected card rank is < 8; else PAS_GAS_SEL_EXTENDED
 *              (fits, selection in pas_gas_fit_ex's side buffer) or PAS_GAS_SEL_LIMIT
 *   bits 0-23  S 3-bit card ranks (lexicographic index into the node's cards),
 *              selection j at bits 3j..3j+2, containers in order, i.e. the
 *              "gas-container-cards" annotation (:317-335) in packed form; 0 otherwise.
 * The reference has no limit on selections per pod or cards per node (scheduler.go:200-257;
 * the GPU plugin's -shared-dev-num lets one card take many selections); here nodes may have
 * up to PAS_GAS_MAX_CARDS cards, and pods any number of selections (numI915 up to INT64_MAX
 * per container): a container's selections are runs on ascending cards (a card first fit
 * passes over never fits again within the container), evaluated in O(cards).  A fitting pod
 * of more than PAS_GAS_MAX_SELECTIONS selections gets bit 31 | PAS_GAS_SEL_LIMIT << 24.
 * The _device forms read d_n_containers[p] clamped into [0, max_containers] (the host form
 * rejects values outside it with PAS_EINVAL). */
int pas_gas_fit(pas_ctx* ctx, uint64_t gen, int32_t n_pods, int32_t max_containers,
                int32_t i915_index, const int64_t* req, const uint32_t* req_mask,
                const int32_t* n_containers, uint32_t* res_out);
int pas_gas_fit_device(pas_ctx* ctx, uint64_t gen, int32_t n_pods, int32_t max_containers,
                       int32_t i915_index, const int64_t* d_req, const uint32_t* d_req_mask,
                       const int32_t* d_n_containers, uint32_t* d_res_out, void* hip_stream);

/* pas_gas_fit plus the side buffer of the selections that do not pack: side[0 .. cap) gets
 * one record per PAS_GAS_SEL_EXTENDED word (in no particular order); *side_count = the number
 * of such words (records beyond cap are dropped: call again with a larger buffer). */
int pas_gas_fit_ex(pas_ctx* ctx, uint64_t gen, int32_t n_pods, int32_t max_containers,
                   int32_t i915_index, const int64_t* req, const uint32_t* req_mask,
                   const int32_t* n_containers, uint32_t* res_out, pas_gas_selection* side,
                   int64_t side_cap, int64_t* side_count);
/* d_side_count: device int64, zeroed by the call, then the count (read it after the stream). */
int pas_gas_fit_ex_device(pas_ctx* ctx, uint64_t gen, int32_t n_pods, int32_t max_containers,
                          int32_t i915_index, const int64_t* d_req, const uint32_t* d_req_mask,
                          const int32_t* d_n_containers, uint32_t* d_res_out,
                          pas_gas_selection* d_side, int64_t side_cap, int64_t* d_side_count,
                          void* hip_stream);

/* pas_gas_fit_ex_device with a result row pitch: the word of (pod p, node n) goes to
 * d_res_out[p * ld_res + n], ld_res >= n_nodes (words n_nodes .. ld_res - 1 of a row are not
 * written).  A pitch that is a multiple of 32 words starts every row on a 128-byte line: the
 * fit kernels store a wave's 64 node words as one 256-byte piece of a row, and pieces that
 * straddle lines (every other row of an odd-multiple-of-16 dense pitch, e.g. 50 000) are
 * written ~25 % slower.  The selection side buffer is optional (d_side / d_side_count null,
 * side_cap 0).  Same results as pas_gas_fit_ex_device otherwise (scheduler.go:449-482). */
int pas_gas_fit_ld_device(pas_ctx* ctx, uint64_t gen, int32_t n_pods, int32_t max_containers,
                          int32_t i915_index, const int64_t* d_req, const uint32_t* d_req_mask,
                          const int32_t* d_n_containers, uint32_t* d_res_out, int64_t ld_res,
                          pas_gas_selection* d_side, int64_t side_cap, int64_t* d_side_count,
                          void* hip_stream);

/* Pods of the last GAS fit call on this context with more than PAS_GAS_MAX_SELECTIONS
 * selections (their fitting words are PAS_GAS_SEL_LIMIT).  Waits for the call's stream. */
int pas_gas_limit_count(pas_ctx* ctx, int64_t* n_pods_out);

/* GAS filter verdicts only, as node bitmaps fit_out[n_pods][W64(n_nodes)] (bit = bit 31 of
 * the pas_gas_fit word).  Used to intersect GAS with TAS candidates (cand of the TAS calls)
 * without materialising the per-(pod, node) words. */
int pas_gas_fit_bitmap_device(pas_ctx* ctx, uint64_t gen, int32_t n_pods, int32_t max_containers,
                              int32_t i915_index, const int64_t* d_req,
                              const uint32_t* d_req_mask, const int32_t* d_n_containers,
                              uint64_t* d_fit_out, void* hip_stream);

/* Bind-time commit (GASExtender.bindNode, scheduler.go:385-445): for binds b in call order,
 * pod bind_pod[b] (an index into the req / req_mask / n_containers batch, as pas_gas_fit)
 * onto node bind_node[b]: runSchedulingLogic on the node's CURRENT resident usage, then
 * Cache.adjustPodResources(add) with the resulting annotation (node_resource_cache.go:
 * 240-287), applied to the resident used[N][K][Q] in place.  Binds to the same node see
 * each other in call order.  res_out[b] = the pas_gas_fit word for that (pod, node) at bind
 * time, status_out[b] = PAS_GAS_OK or PAS_GAS_WONT_FIT (then nothing changes).  The
 * snapshot moves from generation gen_from (PAS_ESTALE otherwise) to gen_to. */
#define PAS_GAS_OK 0
#define PAS_GAS_WONT_FIT 1
#define PAS_GAS_ERR_INPUT 2    /* resource_map.go errInput: nothing changes */
#define PAS_GAS_ERR_OVERFLOW 3 /* resource_map.go errOverflow: nothing changes */
int pas_gas_bind(pas_ctx* ctx, uint64_t gen_from, uint64_t gen_to, int32_t n_binds,
                 const int32_t* bind_pod, const int32_t* bind_node, int32_t n_pods,
                 int32_t max_containers, int32_t i915_index, const int64_t* req,
                 const uint32_t* req_mask, const int32_t* n_containers, uint32_t* res_out,
                 int32_t* status_out);
/* pas_gas_bind plus every bind's full card selection: cards_out[b][0 .. n_sel_out[b]) (ranks,
 * selection by selection; n_sel_out 0 when it does not fit), for selections that do not
 * pack into the result word.  A bind of more than PAS_GAS_MAX_SELECTIONS selections has
 * n_sel_out -1 and cards_out zero: pas_gas_bind_counts reports it. */
int pas_gas_bind_ex(pas_ctx* ctx, uint64_t gen_from, uint64_t gen_to, int32_t n_binds,
                    const int32_t* bind_pod, const int32_t* bind_node, int32_t n_pods,
                    int32_t max_containers, int32_t i915_index, const int64_t* req,
                    const uint32_t* req_mask, const int32_t* n_containers, uint32_t* res_out,
                    int32_t* status_out, uint8_t* cards_out /*[n_binds][64]*/,
                    int32_t* n_sel_out);

/* pas_gas_bind with every bind's selection as counts, for any number of selections:
 * counts_out[b][c][k] = the selections container c made on card k (int64; all 0 when the
 * bind does not fit).  Within a container the selections are in ascending card order (first
 * fit with one per-GPU request never returns to a card it has passed), so the counts are the
 * "gas-container-cards" annotation: container c lists card k counts_out[b][c][k] times, in
 * card order (scheduler.go:200-257, 317-335). */
int pas_gas_bind_counts(pas_ctx* ctx, uint64_t gen_from, uint64_t gen_to, int32_t n_binds,
                        const int32_t* bind_pod, const int32_t* bind_node, int32_t n_pods,
                        int32_t max_containers, int32_t i915_index, const int64_t* req,
                        const uint32_t* req_mask, const int32_t* n_containers,
                        uint32_t* res_out, int32_t* status_out,
                        int64_t* counts_out /*[n_binds][max_containers][max_cards]*/);

/* Pods leaving nodes: Cache.adjustPodResources(remove) (node_resource_cache.go:240-287) with
 * each pod's annotation, in call order.  Container c of release r has cards_per_container
 * [r][c] cards (its "gas-container-cards" segment), listed in container order in
 * cards[r][8] (at most 8 in all; pas_gas_release_ex: 64) as ranks into the node's cards; request / count is subtracted from each card
 * (subtractRM, resource_map.go:55-73,103-127: clamp at 0; a negative amount, or a card the
 * node's label does not list, is an input error and nothing changes).  The snapshot keeps
 * no "key absent" state: a label card has every kind, so subtracting from a kind that was
 * never added clamps at 0 where the reference reports errInput. */
int pas_gas_release(pas_ctx* ctx, uint64_t gen_from, uint64_t gen_to, int32_t n_releases,
                    const int32_t* rel_pod, const int32_t* rel_node, int32_t n_pods,
                    int32_t max_containers, const int64_t* req, const uint32_t* req_mask,
                    const int32_t* n_containers, const int32_t* cards_per_container,
                    const int32_t* cards, int32_t* status_out);
/* pas_gas_release with cards[r][PAS_GAS_MAX_SELECTIONS] (annotations of up to 64 cards). */
int pas_gas_release_ex(pas_ctx* ctx, uint64_t gen_from, uint64_t gen_to, int32_t n_releases,
                       const int32_t* rel_pod, const int32_t* rel_node, int32_t n_pods,
                       int32_t max_containers, const int64_t* req, const uint32_t* req_mask,
                       const int32_t* n_containers, const int32_t* cards_per_container,
                       const int32_t* cards, int32_t* status_out);

/* pas_gas_release with each annotation as counts[r][c][k] (container c lists card k that many
 * times; numCards = the row's sum), for annotations of any length.  Negative counts or a row
 * sum past INT64_MAX: PAS_EINVAL; a count on a card rank >= the node's n_cards: input error
 * (status PAS_GAS_ERR_INPUT), as a card the label does not list. */
int pas_gas_release_counts(pas_ctx* ctx, uint64_t gen_from, uint64_t gen_to,
                           int32_t n_releases, const int32_t* rel_pod, const int32_t* rel_node,
                           int32_t n_pods, int32_t max_containers, const int64_t* req,
                           const uint32_t* req_mask, const int32_t* n_containers,
                           const int64_t* counts /*[n_releases][max_containers][max_cards]*/,
                           int32_t* status_out);

/* Read back the resident usage used[N][K][Q] and its generation. */
int pas_gas_snapshot_get(pas_ctx* ctx, uint64_t* gen, int64_t* used_out);

/* ------------------------------------------------------------------------- */
/* Node-sharded snapshots                                  */
/* ------------------------------------------------------------------------- */

/* A GPU holding nodes [node_base, node_base + n_nodes) of the cluster as its resident
 * TAS snapshot evaluates every pod's filter + prioritize over that shard and keeps the
 * first k entries of the shard's HostPriorityList (as pas_tas_eval_device with both flags
 * would list them) as merge records:
 *   top_node [n_pods][k]  global node index (node_base + shard index); INT32_MAX past len
 *   top_key  [n_pods][k]  order key: ~value for GreaterThan, value for LessThan, 0 for any
 *                         other operator (value = the node's v_milli of the prioritize
 *                         metric); INT64_MAX past len
 *   top_len  [n_pods]     min(k, entries)
 * Ascending (key, node) is the HostPriorityList order, so the merge of all shards' records
 * (pas_topk_merge_device) is exactly the first k entries over the whole cluster. */
int pas_tas_topk_device(pas_ctx* ctx, uint64_t gen, int32_t n_pods, int32_t n_rules,
                        const pas_rule* d_rules, const int32_t* d_rule_off,
                        const pas_rule* d_prio, const uint64_t* d_cand, int32_t k,
                        int32_t node_base, int64_t* d_top_key, int32_t* d_top_node,
                        int32_t* d_top_len, void* hip_stream);

/* Full-list prioritize over node shards: the cluster's whole
 * HostPriorityList per pod from every shard's whole list.  keys / nodes [n_shards][n_pods]
 * [width] are the shards' records as pas_tas_topk_device writes them with k = width (>= the
 * widest shard; INT64_MAX / INT32_MAX past each list).  out_node[p][0 .. out_len[p]) = the
 * merged list (ascending (key, node): the order prioritizeNodesForRule lists,
 * telemetryscheduler.go:128-149), global node ids, -1 in positions
 * [out_len[p], n_shards * width); row pitch out_ld >= n_shards * width.  Exact: no
 * (key, node) pair repeats across shards. */
int pas_list_merge_device(pas_ctx* ctx, int32_t n_pods, int32_t n_shards, int32_t width,
                          const int64_t* d_keys, const int32_t* d_nodes, int32_t* d_out_node,
                          int64_t out_ld, int32_t* d_out_len, void* hip_stream);

/* The same records for the combined TAS + GAS filter (BASELINE configs[4]): the first k
 * entries of the shard's HostPriorityList over the nodes that pass the pod's dontschedule
 * filter (and d_cand when given) AND fit its GPU request (runSchedulingLogic on the
 * context's resident GAS snapshot of the same nodes, gpuscheduler/scheduler.go:280-338).
 * Equal to pas_gas_fit_bitmap_device over the shard followed by pas_tas_topk_device with
 * the fit bitmaps (intersected with d_cand) as candidates, but evaluated along each pod's
 * order: a node is filtered and fitted only until k nodes are kept, so a pod costs about
 * k / (pass rate) node evaluations instead of the shard's n_nodes.  The GAS arguments are
 * those of pas_gas_fit_device (any number of selections).  The two snapshots must hold the
 * same number of nodes (PAS_EINVAL otherwise). */
int pas_tas_gas_topk_device(pas_ctx* ctx, uint64_t tas_gen, uint64_t gas_gen, int32_t n_pods,
                            int32_t n_rules, const pas_rule* d_rules, const int32_t* d_rule_off,
                            const pas_rule* d_prio, const uint64_t* d_cand,
                            int32_t max_containers, int32_t i915_index, const int64_t* d_req,
                            const uint32_t* d_req_mask, const int32_t* d_n_containers,
                            int32_t k, int32_t node_base, int64_t* d_top_key,
                            int32_t* d_top_node, int32_t* d_top_len, void* hip_stream);

/* Merge of n_shards record sets laid out [n_shards][n_pods][k] (the layout of an
 * all-gather of the per-shard top_key / top_node): out_node[n_pods][k] = the k smallest
 * (key, node) records' nodes in order (-1 past out_len), out_len = min(k, records). */
int pas_topk_merge_device(pas_ctx* ctx, int32_t n_pods, int32_t k, int32_t n_shards,
                          const int64_t* d_keys, const int32_t* d_nodes, int32_t* d_out_node,
                          int32_t* d_out_len, void* hip_stream);

/* ------------------------------------------------------------------------- */
/* Wire encoders, host only                                */
/* ------------------------------------------------------------------------- */

/* Response bodies exactly as the reference's handlers write them with
 * json.NewEncoder(w).Encode (encoding/json of Go 1.16, HTML-safe escaping, trailing "\n").
 * Each writes at most cap bytes (no terminator), sets *out_len to the full length, and
 * returns PAS_ECAPACITY when it exceeds cap.  names[i] / node_json[i] are indexed by
 * snapshot node id.
 *
 * HostPriorityList of one pod (WritePrioritizeResponse, telemetryscheduler.go:152-158):
 * order[0 .. len) from pas_tas_eval's order_out row -> [{"Host":..,"Score":10-i},...]. */
int pas_encode_host_priority_list(int32_t len, const int32_t* order, const char* const* names,
                                  char* buf, int64_t cap, int64_t* out_len);

/* TAS FilterResult of one pod (filterNodes + WriteFilterResponse, telemetryscheduler.go:
 * 184-225, 238-244): the request's nodes req_node[0 .. n_req) in request order, the pod's
 * pass_out row; node_json[i] (node_json_len[i] bytes) = the JSON of node i as the Go shim
 * encodes a v1.Node (spliced into "items").  The nil results (no policy label, policy not
 * cached, no dontschedule rules, no nodes: :189-203) are the body "null\n", written by
 * the shim. */
int pas_encode_tas_filter_result(int32_t n_req, const int32_t* req_node, const uint64_t* pass,
                                 const char* const* names, const char* const* node_json,
                                 const int64_t* node_json_len, char* buf, int64_t cap,
                                 int64_t* out_len);

/* GAS FilterResult of one pod (GASExtender.filterNodes, gpuscheduler/scheduler.go:449-482):
 * request node names in order, fit = the pod's row of pas_gas_fit_bitmap_device (or bit 31
 * of the pas_gas_fit words, packed); n_req == 0 gives the reference's error result. */
int pas_encode_gas_filter_result(int32_t n_req, const int32_t* req_node, const uint64_t* fit,
                                 const char* const* names, char* buf, int64_t cap,
                                 int64_t* out_len);

/* BindingResult of GASExtender.bindNode (scheduler.go:385-445): {"Error":"<error>"}; NULL or
 * "" for success. */
int pas_encode_binding_result(const char* error, char* buf, int64_t cap, int64_t* out_len);

/* ------------------------------------------------------------------------- */
/* Wire decoding, host only                                */
/* ------------------------------------------------------------------------- */

/* Snapshot node names -> node ids (the numbering of the TAS / GAS snapshots), built once per
 * snapshot; a repeated name keeps its first id.  Lookup of len bytes: id or -1. */
typedef struct pas_name_table pas_name_table;
int pas_name_table_create(int32_t n_names, const char* const* names, pas_name_table** out);
void pas_name_table_destroy(pas_name_table* table);
int32_t pas_name_table_lookup(const pas_name_table* table, const char* name, int64_t len);

#define PAS_ARGS_NODES 0      /* args.Nodes.Items[].Name: TAS (NodeCacheCapable false) */
#define PAS_ARGS_NODE_NAMES 1 /* *args.NodeNames: GAS (NodeCacheCapable true) */
typedef struct pas_args_info {
  int32_t has_nodes;      /* args.Nodes != nil (TAS: "no nodes in list" otherwise, :74-76) */
  int32_t has_node_names; /* args.NodeNames != nil */
  int32_t n_req;          /* request nodes of the chosen list, in request order */
  int32_t n_unknown;      /* of them not in the table (req_node -1) */
  int64_t pod_off;        /* byte span of the Pod object in the body; pod_len 0: absent / null */
  int64_t pod_len;
} pas_args_info;

/* extender.Args (extender/types.go:36-46) as json.NewDecoder(body).Decode(&args) fills it
 * (telemetryscheduler.go:63-78; gpuscheduler/scheduler.go:486-505), reduced to what the
 * handlers read: the request's node list `which` resolved through the name table into
 * req_node[0 .. n_req) (request order, -1 for a node not in the table), the candidate bitmap
 * cand[W64(table size)] of the known ones (may be NULL), and for PAS_ARGS_NODES the byte span
 * (offset, length) of each item in item_span[n_req][2] (may be NULL).  PAS_EDECODE for what
 * the reference's decode rejects (empty body, syntax, a wrong JSON type on the fields read);
 * PAS_ECAPACITY (info filled) when n_req > node_cap.  Matching of keys, null handling and
 * repeated keys follow encoding/json of Go 1.16 (csrc/wire_decode.cpp). */
int pas_decode_args(const pas_name_table* table, const char* body, int64_t len, int32_t which,
                    int32_t* req_node, int64_t node_cap, int64_t* item_span, uint64_t* cand,
                    pas_args_info* info);

/* The request node names themselves (unescaped, request order), for nodes the table does not
 * know (their FailedNodes / NodeNames entries): name i is buf[offsets[i] .. offsets[i+1]).
 * PAS_ECAPACITY (*total_len, *n_req set) when buf or offsets[n_req + 1] is too small. */
int pas_decode_request_names(const char* body, int64_t len, int32_t which, char* buf,
                             int64_t cap, int64_t* offsets, int64_t offsets_cap,
                             int64_t* total_len, int32_t* n_req);

/* getPolicyFromPod's reads of a v1.Pod JSON (telemetryscheduler.go:103-112): the namespace
 * (*ns_len bytes) and the value of labels[label] (*label_len bytes, -1 if the key is absent).
 * PAS_ECAPACITY (lengths set) when a buffer is too small; PAS_EDECODE as pas_decode_args. */
int pas_decode_pod_policy(const char* pod, int64_t len, const char* label, char* ns_buf,
                          int64_t ns_cap, int64_t* ns_len, char* label_buf, int64_t label_cap,
                          int64_t* label_len);

/* Host threads pas_decode_args may use for one large body: the structural index and the
 * items of a NodeList are split over them (about one per MB of body; results identical to
 * one thread).  n = 0: automatic (up to 16, the GPU box's CPU share per GPU); process-wide.
 * pas_decode_threads: the count a body of that size gets. */
int pas_decode_set_threads(int32_t n);
int32_t pas_decode_threads(int64_t body_len);

/* containerRequests of a v1.Pod JSON (gpuscheduler/utils.go:14-32): per container, the
 * requests named gpu.intel.com/... as AsInt64 values (ok ignored), in the pas_gas_fit layout
 * req[max_containers][n_kinds] / req_mask[max_containers] for kinds[0 .. n_kinds), and
 * *n_containers = len(spec.containers).  gpu.intel.com requests of other kinds are counted
 * in *n_unknown, and such a container's req_mask carries PAS_REQ_UNKNOWN_KIND (with
 * numI915 > 0 it fits no node: capacity lacks the key, scheduler.go:349-354).  n_kinds <= 31.  A quantity ParseQuantity rejects is PAS_EDECODE
 * (Quantity.UnmarshalJSON); PAS_ECAPACITY when n_containers > max_containers.  With
 * n_kinds 0 (req may be NULL) it only validates the quantities, as the TAS decode does. */
int pas_decode_pod_requests(const char* pod, int64_t len, int32_t n_kinds,
                            const char* const* kinds, int32_t max_containers, int64_t* req,
                            uint32_t* req_mask, int32_t* n_containers, int32_t* n_unknown);

/* ------------------------------------------------------------------------- */
/* Instrumentation                                                           */
/* ------------------------------------------------------------------------- */

/* Kernel timing with HIP events on the stream each kernel is launched on.
 * Kernel ids: */
#define PAS_K_TAS_EVAL 1       /* per pod: pass bitmap + ordered host list (fused) */
#define PAS_K_TAS_VIOLATIONS 2 /* deschedule sweep */
#define PAS_K_GAS_PREP 3       /* per-GPU container requests */
#define PAS_K_GAS_FIT 4        /* per (pod, node) first fit */
#define PAS_K_TAS_PREP 5       /* rule ranges + pods bucketed by prioritize order */
#define PAS_K_TAS_LABELS 6     /* deschedule label plan */
#define PAS_K_TAS_SPAN 7       /* whole pas_tas_eval path: first launch start to last launch end */
#define PAS_K_PRIO_REQUEST 8   /* whole pas_tas_prioritize_request path (keys, sort, positions) */
#define PAS_K_TAS_GAS_TOPK 9   /* combined TAS + GAS top-k along each pod's order */
#define PAS_K_COUNT 10
#define PAS_TIMING_SPAN 1    /* whole paths: PAS_K_TAS_SPAN, PAS_K_PRIO_REQUEST, the GAS fit and
                                deschedule launches */
#define PAS_TIMING_KERNELS 2 /* every launch (events between launches add small gaps) */
int pas_set_timing(pas_ctx* ctx, int level); /* 0 = off */
/* Sum of elapsed ms and number of launches recorded for a kernel since the last reset. */
int pas_kernel_time(pas_ctx* ctx, int32_t kernel_id, double* total_ms, int64_t* launches);
int pas_reset_timing(pas_ctx* ctx);

#ifdef __cplusplus
}
#endif

#endif /* PAS_H_ */
