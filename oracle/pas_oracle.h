/*
 * pas_oracle.h — CPU restatement of the reference's filter/prioritize/deschedule and
 * GAS fit semantics.  TEST INFRASTRUCTURE ONLY: imported by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg, and only as the
 * checker.  The product (platform-aware-scheduling_amd/) never links or calls it.
 *
 * Parity is pinned by the reference's own table-driven test vectors and e2e
 * fixtures, transcribed under tests/golden/ (SURVEY.md Appendix B, G1-G11); the
 * reference itself (Go 1.16 + k8s.io/apimachinery v0.22.2) cannot be built here.
 *
 * Every function names the reference lines it restates.  It deliberately uses the
 * reference's loop structure (rule -> node map -> EvaluateRule; sort per request;
 * per (pod, node) sequential container/card loop) and exact 128-bit arithmetic, not
 * the device's sorted-range / saturating formulation.
 */
#ifndef PAS_ORACLE_H_
#define PAS_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_rule {
  int32_t metric;  /* column, or <0 = metric not in cache */
  int32_t op;      /* 0 LessThan, 1 GreaterThan, 2 Equals, other = invalid */
  int64_t target;  /* integer units */
} or_rule;

/* core.EvaluateRule (telemetry-aware-scheduling/pkg/strategies/core/operator.go:13-26):
 * Quantity.CmpInt64(target) == -1 / 1 / 0, restated on an exact milli value.
 * Returns 1/0, or -1 for an operator the reference would panic on (operator.go:25). */
int or_evaluate_rule(int64_t v_milli, int32_t op, int64_t target);

/* The same on an exact decimal value u * 10^-s, 0 <= s <= 9 (every value resource.ParseQuantity
 * yields: 9 fractional digits at most, |value| <= 2^63 - 1); -2 for s out of range.  Values
 * are aligned to 10^-9 in 128-bit integers, as inf.Dec.Cmp aligns scales. */
int or_evaluate_rule_dec(int64_t u, int32_t s, int32_t op, int64_t target);
/* Quantity.Cmp of two such values: -1 / 0 / 1. */
int or_cmp_dec(int64_t u1, int32_t s1, int64_t u2, int32_t s2);

/* The _dec variants below take every value as v[m][n] * 10^-v_scale[m][n] (v_scale NULL =
 * milli, 3, as the variants without the suffix). */

/* Strategy.Violated for dontschedule (dontschedule/strategy.go:25-44) and deschedule
 * (deschedule/strategy.go:31-50) — identical loops.  violating[n] set to 1 for every
 * node of the union.  Returns 0, or -1 on an invalid operator. */
int or_violated(int32_t n_nodes, int32_t n_metrics, const int64_t* v_milli,
                const uint64_t* present, const or_rule* rules, int32_t n_rules,
                uint8_t* violating);

/* prioritizeNodesForRule (telemetryscheduler/telemetryscheduler.go:128-149) with
 * core.OrderedList (operator.go:30-42): candidates (cand[n] != 0) that have the metric,
 * GreaterThan = descending, LessThan = ascending, other = unsorted; ties and the
 * unsorted case follow the documented rule "ascending node index" (the reference's
 * order there is Go-map order, i.e. unspecified).  Writes node indices best-first to
 * out and returns the count. */
int32_t or_ordered_list(int32_t n_nodes, int32_t n_metrics, const int64_t* v_milli,
                        const uint64_t* present, const or_rule* rule, const uint8_t* cand,
                        int32_t* out);

/* The same for one extender request in the request's own terms:
 * req_node[j] = snapshot node of args.Nodes.Items[j] (-1 / out of range = not in the
 * snapshot).  filteredNodeData (telemetryscheduler.go:135-139) keeps one entry per name;
 * the entries are taken in order of first occurrence and stably sorted by value, so ties
 * (and every entry for other operators) keep ascending first-occurrence position.  Writes
 * request positions best-first to out_pos and returns the count. */
int32_t or_ordered_list_request(int32_t n_nodes, int32_t n_metrics, const int64_t* v_milli,
                                const uint64_t* present, const or_rule* rule, int32_t n_req,
                                const int32_t* req_node, int32_t* out_pos);

/* Batched equivalent of pas_tas_eval (include/pas.h): per pod, filterNodes
 * (telemetryscheduler.go:184-225) and/or prioritizeNodesForRule.  Same argument
 * layout as the C-ABI host entry point.  Returns 0 or -1 (invalid operator). */
int or_tas_eval(int32_t n_nodes, int32_t n_metrics, const int64_t* v_milli,
                const uint64_t* present, int32_t n_pods, const or_rule* rules,
                const int32_t* rule_off, const or_rule* prio, const uint64_t* cand,
                uint32_t flags, uint64_t* pass_out, int32_t* order_out, int32_t* order_len);
int or_tas_eval_dec(int32_t n_nodes, int32_t n_metrics, const int64_t* v_milli,
                    const int8_t* v_scale, const uint64_t* present, int32_t n_pods,
                    const or_rule* rules, const int32_t* rule_off, const or_rule* prio,
                    const uint64_t* cand, uint32_t flags, uint64_t* pass_out,
                    int32_t* order_out, int32_t* order_len);
int32_t or_ordered_list_request_dec(int32_t n_nodes, int32_t n_metrics, const int64_t* v_milli,
                                    const int8_t* v_scale, const uint64_t* present,
                                    const or_rule* rule, int32_t n_req, const int32_t* req_node,
                                    int32_t* out_pos);

/* nodeStatusForStrategy (deschedule/enforce.go:154-164): per strategy, Violated as a
 * bitmap viol_out[s][W64]. */
int or_tas_violations(int32_t n_nodes, int32_t n_metrics, const int64_t* v_milli,
                      const uint64_t* present, int32_t n_strategies, const or_rule* rules,
                      const int32_t* rule_off, uint64_t* viol_out);
int or_tas_violations_dec(int32_t n_nodes, int32_t n_metrics, const int64_t* v_milli,
                          const int8_t* v_scale, const uint64_t* present, int32_t n_strategies,
                          const or_rule* rules, const int32_t* rule_off, uint64_t* viol_out);

/* Deschedule.updateNodeLabels (deschedule/enforce.go:99-151) per node, for S <= 64
 * registered strategies with policy names names[s] (NULL = all distinct).  The reference
 * keys the non-violated set by policy NAME (allPolicies, :89-95; delete per violating
 * strategy, :109), and two registered strategies can share one (AddStrategy drops only
 * Equals duplicates, core/enforcer.go:84-103).  A name is represented by its first
 * strategy k; labels[k] row = the nodes carrying the label <name>.
 *   add[n] bit s = strategy s violated at node n (one "violating" add per strategy, :108-117)
 *   rem[n] bit k = name k violated by none of its strategies and carried (remove + add
 *                  "null", :118-132)
 *   *total_violations = the NON-violated (node, name) pairs (totalViolations++, :133). */
int or_label_plan(int32_t n_nodes, int32_t n_strat, const char* const* names,
                  const uint64_t* viol, const uint64_t* labels, uint64_t* add, uint64_t* rem,
                  int64_t* total_violations);
/* json.Marshal of the node's []patchValue (enforce.go:20-24, 76-83): adds in strategy
 * order, then remove + add-null pairs in strategy order (the reference's order is map
 * iteration).  Returns the length, or -1 if cap is too small. */
int64_t or_label_patch_json(int32_t n_strat, const char* const* names, uint64_t add, uint64_t rem,
                            char* buf, int64_t cap);

/* ---- GAS ---------------------------------------------------------------- */

/* A resourceMap (gpuscheduler/resource_map.go:20) restated over small integer key
 * ids: has[k] says the key exists, val[k] its int64 amount. */
#define OR_RM_MAX_KEYS 8
typedef struct or_rm {
  uint8_t has[OR_RM_MAX_KEYS];
  int64_t val[OR_RM_MAX_KEYS];
} or_rm;

enum { OR_RM_OK = 0, OR_RM_ERR_INPUT = 1, OR_RM_ERR_OVERFLOW = 2 };

int or_rm_add(or_rm* rm, int32_t key, int64_t value);         /* resource_map.go:77-98 */
int or_rm_subtract(or_rm* rm, int32_t key, int64_t value);    /* resource_map.go:103-127 */
int or_rm_add_rm(or_rm* rm, const or_rm* src);                /* resource_map.go:38-53 */
int or_rm_subtract_rm(or_rm* rm, const or_rm* src);           /* resource_map.go:58-73 */
int or_rm_divide(or_rm* rm, int64_t divider);                 /* resource_map.go:129-145 */
/* checkResourceCapacity (gpuscheduler/scheduler.go:341-383). */
int or_check_resource_capacity(const or_rm* need, const or_rm* capacity, const or_rm* used);

#define OR_GAS_MAX_CARDS 64
#define OR_GAS_MAX_SEL 64
#define OR_GAS_SEL_EXTENDED 15
#define OR_GAS_SEL_LIMIT 14
/* req_mask bit 31: the container requests a gpu.intel.com/ kind outside the packed kinds
 * (include/pas.h PAS_REQ_UNKNOWN_KIND); restated as the key OR_UNKNOWN_KEY of its request
 * map, which no capacity or usage map holds (containerRequests keeps every gpu.intel.com/
 * key, utils.go:14-32; checkResourceCapacity then fails on it, scheduler.go:349-354). */
#define OR_REQ_UNKNOWN_KIND 0x80000000u
#define OR_UNKNOWN_KEY (OR_RM_MAX_KEYS - 1)

/* GAS filter over every (pod, node) of a packed snapshot, one runSchedulingLogic
 * (scheduler.go:280-338) each; same layouts and result encoding as pas_gas_fit (words of
 * selections that do not pack: OR_GAS_SEL_EXTENDED; fitting pods with more than 64
 * selections: bit 31 | OR_GAS_SEL_LIMIT << 24).  No bound on numI915 (the loop ends at the
 * first selection no card fits).  or_gas_fit_ex also returns every fitting pair's full
 * selection: sel_out[P][N][64] card ranks, nsel_out[P][N] counts (-1 past 64 selections,
 * sel_out then zero; NULL: not wanted). */
int or_gas_fit_ex(int32_t n_nodes, int32_t max_cards, int32_t n_res, const int32_t* n_cards,
                  const int64_t* cap_per_gpu, const int64_t* used, int32_t n_pods,
                  int32_t max_containers, int32_t i915_index, const int64_t* req,
                  const uint32_t* req_mask, const int32_t* n_containers, uint32_t* res_out,
                  uint8_t* sel_out, int32_t* nsel_out);
int or_gas_fit(int32_t n_nodes, int32_t max_cards, int32_t n_res, const int32_t* n_cards,
               const int64_t* cap_per_gpu, const int64_t* used, int32_t n_pods,
               int32_t max_containers, int32_t i915_index, const int64_t* req,
               const uint32_t* req_mask, const int32_t* n_containers, uint32_t* res_out);

/* GASExtender.bindNode (scheduler.go:385-445) for binds b = 0 .. n_binds-1 in order: pod
 * bind_pod[b] onto node bind_node[b] — runSchedulingLogic on the node's current usage
 * (:280-338), then Cache.adjustPodResources(add) with the resulting annotation
 * (node_resource_cache.go:240-287: per container, request / numCards added to each of its
 * cards, all or nothing).  used is updated in place.  res_out[b] = the packed result word
 * (as or_gas_fit; 0 when it does not fit), status[b] = OR_GAS_* below; cards_out / nsel_out
 * the full selection of each committed bind. */
enum { OR_GAS_OK = 0, OR_GAS_WONT_FIT = 1, OR_GAS_ERR_INPUT = 2, OR_GAS_ERR_OVERFLOW = 3 };
int or_gas_bind(int32_t n_nodes, int32_t max_cards, int32_t n_res, const int32_t* n_cards,
                const int64_t* cap_per_gpu, int64_t* used, int32_t n_binds,
                const int32_t* bind_pod, const int32_t* bind_node, int32_t max_containers,
                int32_t i915_index, const int64_t* req, const uint32_t* req_mask,
                const int32_t* n_containers, uint32_t* res_out, int32_t* status,
                uint8_t* cards_out /*[n_binds][64] or NULL*/, int32_t* nsel_out,
                int64_t* counts_out /*[n_binds][max_containers][max_cards] or NULL*/);
/* cards_out / nsel_out as or_gas_fit_ex's sel_out / nsel_out; counts_out[b][c][k] = the
 * selections of container c on card k (any count). */
/* Cache.adjustPodResources(remove) (node_resource_cache.go:240-287) for pods leaving nodes,
 * in order: container c's cards are cards[r][off .. off + n_cc[r][c]) (off = sum of the
 * earlier containers' counts; ranks into the node's cards); its request / n_cc is
 * subtracted from each (subtractRM: clamp at 0; a negative amount or a key the card does
 * not have -> input error, nothing changes).  A card rank outside the node's cards is a
 * card without usage keys. */
int or_gas_release(int32_t n_nodes, int32_t max_cards, int32_t n_res, const int32_t* n_cards,
                   int64_t* used, int32_t n_rel, const int32_t* rel_pod,
                   const int32_t* rel_node, int32_t max_containers, const int64_t* req,
                   const uint32_t* req_mask, const int32_t* n_containers,
                   const int32_t* cards_per_container, const int32_t* cards,
                   int32_t cards_stride /*8 or 64*/, int32_t* status);
/* or_gas_release with the annotation as counts[r][c][k] (container c lists card k that many
 * times, in card order) — annotations of any length. */
int or_gas_release_counts(int32_t n_nodes, int32_t max_cards, int32_t n_res,
                          const int32_t* n_cards, int64_t* used, int32_t n_rel,
                          const int32_t* rel_pod, const int32_t* rel_node,
                          int32_t max_containers, const int64_t* req, const uint32_t* req_mask,
                          const int32_t* n_containers, const int64_t* counts, int32_t* status);

#ifdef __cplusplus
}
#endif

#endif /* PAS_ORACLE_H_ */
