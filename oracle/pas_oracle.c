/*
 * pas_oracle.c — CPU restatement of the reference semantics (see pas_oracle.h).
 * TEST INFRASTRUCTURE ONLY; never linked into the product library.
 *
 * Reference root: tejasshahintel/platform-aware-scheduling @ 2025-02-20.
 *   TAS: telemetry-aware-scheduling/pkg/{strategies,telemetryscheduler}
 *   GAS: gpu-aware-scheduling/pkg/gpuscheduler
 */
#include "pas_oracle.h"

#include <stdlib.h>
#include <stdio.h>
#include <string.h>

static inline int has_bit(const uint64_t* bits, int64_t i) {
  return (int)((bits[i >> 6] >> (i & 63)) & 1u);
}

static inline int64_t w64(int32_t n) { return ((int64_t)n + 63) / 64; }

/* Metric column m "exists in the cache" when it has at least one node: the cache never
 * stores an empty NodeMetricsInfo (nilPayloadCheck, cache/autoupdating.go:138-145), so
 * ReadMetric errors exactly when the column is empty (autoupdating.go:76-85). */
static int metric_in_cache(int32_t n_nodes, int32_t n_metrics, const uint64_t* present,
                           int32_t m) {
  if (m < 0 || m >= n_metrics) return 0;
  const uint64_t* row = present + (int64_t)m * w64(n_nodes);
  for (int64_t w = 0; w < w64(n_nodes); ++w)
    if (row[w]) return 1;
  return 0;
}

/* A metric value as the exact decimal the reference holds: unscaled u and decimal places s,
 * value = u * 10^-s (inf.Dec's {unscaled, scale}; an int64Amount{value, scale} is the same
 * with s = -scale).  resource.ParseQuantity rounds every value to 9 fractional digits
 * (inf.RoundUp at Nano) and caps it at 2^63 - 1, so 0 <= s <= 9 covers every Quantity a
 * metric can hold.  Comparisons align both operands to 10^-9 (u * 10^(9 - s)) in 128-bit
 * integers, as inf.Dec.Cmp aligns scales before comparing unscaled values: exact, no
 * rounding, no saturation.  vs == NULL: every value is milli (s = 3). */
static const __int128 kPow10[10] = {1, 10, 100, 1000, 10000, 100000, 1000000, 10000000,
                                    100000000, 1000000000};

static inline __int128 nano_of(const int64_t* v, const int8_t* vs, int64_t i) {
  const int s = vs ? vs[i] : 3;
  return (__int128)v[i] * kPow10[9 - s];
}

/* Quantity.CmpInt64(target) on a value in units of 1e-9. */
static int cmp_int64_nano(__int128 v, int64_t target) {
  const __int128 t = (__int128)target * kPow10[9];
  return v < t ? -1 : (v > t ? 1 : 0);
}

/* operator.go:13-26 on an aligned value. */
static int evaluate_rule_nano(__int128 v, int32_t op, int64_t target) {
  const int cmp = cmp_int64_nano(v, target); /* Quantity.CmpInt64 */
  switch (op) {
    case 0: return cmp == -1; /* "LessThan"    operator.go:15-17 */
    case 1: return cmp == 1;  /* "GreaterThan" operator.go:18-20 */
    case 2: return cmp == 0;  /* "Equals"      operator.go:21-23 */
    default: return -1;       /* nil map entry -> panic at operator.go:25 */
  }
}

int or_evaluate_rule(int64_t v_milli, int32_t op, int64_t target) {
  return evaluate_rule_nano((__int128)v_milli * kPow10[6], op, target);
}

int or_evaluate_rule_dec(int64_t u, int32_t s, int32_t op, int64_t target) {
  if (s < 0 || s > 9) return -2;
  return evaluate_rule_nano((__int128)u * kPow10[9 - s], op, target);
}

int or_cmp_dec(int64_t u1, int32_t s1, int64_t u2, int32_t s2) {
  const __int128 a = (__int128)u1 * kPow10[9 - s1], b = (__int128)u2 * kPow10[9 - s2];
  return a < b ? -1 : (a > b ? 1 : 0);
}

/* dontschedule/strategy.go:25-44 (deschedule/strategy.go:31-50 is the same loop). */
static int violated_dec(int32_t n_nodes, int32_t n_metrics, const int64_t* v_milli,
                        const int8_t* v_scale, const uint64_t* present, const or_rule* rules,
                        int32_t n_rules, uint8_t* violating) {
  memset(violating, 0, (size_t)n_nodes);
  for (int32_t r = 0; r < n_rules; ++r) {            /* for _, rule := range d.Rules */
    const or_rule* rule = &rules[r];
    if (!metric_in_cache(n_nodes, n_metrics, present, rule->metric))
      continue;                                      /* ReadMetric err -> continue :28-32 */
    if (rule->op < 0 || rule->op > 2)
      return -1; /* EvaluateRule runs for >= 1 node of the map: panic (operator.go:25) */
    const int64_t base = (int64_t)rule->metric * n_nodes;
    const uint64_t* pres = present + (int64_t)rule->metric * w64(n_nodes);
    for (int32_t n = 0; n < n_nodes; ++n) {          /* for nodeName, nodeMetric := range */
      if (!has_bit(pres, n)) continue;
      if (evaluate_rule_nano(nano_of(v_milli, v_scale, base + n), rule->op, rule->target))
        violating[n] = 1;                            /* violatingNodes[nodeName] = nil */
    }
  }
  return 0;
}

int or_violated(int32_t n_nodes, int32_t n_metrics, const int64_t* v_milli,
                const uint64_t* present, const or_rule* rules, int32_t n_rules,
                uint8_t* violating) {
  return violated_dec(n_nodes, n_metrics, v_milli, NULL, present, rules, n_rules, violating);
}

/* ---- OrderedList ---------------------------------------------------------- */

typedef struct sortable {
  int32_t node;
  __int128 value; /* units of 1e-9: Quantity.Cmp is integer order here */
} sortable;

/* Stable merge sort; `desc` selects the GreaterThan comparator (operator.go:37),
 * otherwise LessThan (operator.go:39).  Stability over input in node-index order is
 * the documented tie-break. */
static void merge_sort(sortable* a, sortable* tmp, int32_t n, int desc) {
  if (n < 2) return;
  if (n <= 16) { /* insertion sort, stable */
    for (int32_t i = 1; i < n; ++i) {
      sortable x = a[i];
      int32_t j = i - 1;
      while (j >= 0 && (desc ? (x.value > a[j].value) : (x.value < a[j].value))) {
        a[j + 1] = a[j];
        --j;
      }
      a[j + 1] = x;
    }
    return;
  }
  const int32_t h = n / 2;
  merge_sort(a, tmp, h, desc);
  merge_sort(a + h, tmp, n - h, desc);
  int32_t i = 0, j = h, k = 0;
  while (i < h && j < n) {
    const int take_right = desc ? (a[j].value > a[i].value) : (a[j].value < a[i].value);
    tmp[k++] = take_right ? a[j++] : a[i++];
  }
  while (i < h) tmp[k++] = a[i++];
  while (j < n) tmp[k++] = a[j++];
  memcpy(a, tmp, (size_t)n * sizeof(sortable));
}

static int32_t ordered_list_dec(int32_t n_nodes, int32_t n_metrics, const int64_t* v_milli,
                                const int8_t* v_scale, const uint64_t* present,
                                const or_rule* rule, const uint8_t* cand, int32_t* out) {
  /* getSchedulingRule (telemetryscheduler.go:115-124) already rejected rules without a
   * metric name; a metric missing from the cache makes prioritizeNodesForRule fail
   * (:130-133) and prioritizeNodes answer with an empty list (:92-96). */
  if (!metric_in_cache(n_nodes, n_metrics, present, rule->metric)) return 0;
  const int64_t base = (int64_t)rule->metric * n_nodes;
  const uint64_t* pres = present + (int64_t)rule->metric * w64(n_nodes);
  sortable* items = (sortable*)malloc(sizeof(sortable) * (size_t)(n_nodes > 0 ? n_nodes : 1));
  sortable* tmp = (sortable*)malloc(sizeof(sortable) * (size_t)(n_nodes > 0 ? n_nodes : 1));
  int32_t cnt = 0;
  /* filteredNodeData: candidates that have the metric (telemetryscheduler.go:135-139) */
  for (int32_t n = 0; n < n_nodes; ++n) {
    if (!cand[n] || !has_bit(pres, n)) continue;
    items[cnt].node = n;
    items[cnt].value = nano_of(v_milli, v_scale, base + n);
    ++cnt;
  }
  if (rule->op == 1) merge_sort(items, tmp, cnt, 1);       /* "GreaterThan" :36-37 */
  else if (rule->op == 0) merge_sort(items, tmp, cnt, 0);  /* "LessThan"    :38-39 */
  /* any other operator: no sort (switch without default, :35-40) */
  for (int32_t i = 0; i < cnt; ++i) out[i] = items[i].node; /* Score: 10 - i, :145 */
  free(items);
  free(tmp);
  return cnt;
}

int32_t or_ordered_list(int32_t n_nodes, int32_t n_metrics, const int64_t* v_milli,
                        const uint64_t* present, const or_rule* rule, const uint8_t* cand,
                        int32_t* out) {
  return ordered_list_dec(n_nodes, n_metrics, v_milli, NULL, present, rule, cand, out);
}

int32_t or_ordered_list_request_dec(int32_t n_nodes, int32_t n_metrics, const int64_t* v_milli,
                                    const int8_t* v_scale, const uint64_t* present,
                                    const or_rule* rule, int32_t n_req, const int32_t* req_node,
                                    int32_t* out_pos) {
  if (rule->metric < 0 || !metric_in_cache(n_nodes, n_metrics, present, rule->metric)) return 0;
  const int64_t base = (int64_t)rule->metric * n_nodes;
  const uint64_t* pres = present + (int64_t)rule->metric * w64(n_nodes);
  const size_t cap = (size_t)(n_req > 0 ? n_req : 1);
  sortable* items = (sortable*)malloc(sizeof(sortable) * cap);
  sortable* tmp = (sortable*)malloc(sizeof(sortable) * cap);
  uint8_t* seen = (uint8_t*)calloc((size_t)(n_nodes > 0 ? n_nodes : 1), 1);
  int32_t cnt = 0;
  for (int32_t j = 0; j < n_req; ++j) {       /* for _, node := range nodes.Items */
    const int32_t n = req_node[j];
    if (n < 0 || n >= n_nodes || seen[n]) continue;  /* not cached / map key already set */
    seen[n] = 1;
    if (!has_bit(pres, n)) continue;          /* if v, ok := nodeData[node.Name]; ok */
    items[cnt].node = j;
    items[cnt].value = nano_of(v_milli, v_scale, base + n);
    ++cnt;
  }
  if (rule->op == 1) merge_sort(items, tmp, cnt, 1);
  else if (rule->op == 0) merge_sort(items, tmp, cnt, 0);
  for (int32_t i = 0; i < cnt; ++i) out_pos[i] = items[i].node;
  free(items);
  free(tmp);
  free(seen);
  return cnt;
}

int32_t or_ordered_list_request(int32_t n_nodes, int32_t n_metrics, const int64_t* v_milli,
                                const uint64_t* present, const or_rule* rule, int32_t n_req,
                                const int32_t* req_node, int32_t* out_pos) {
  return or_ordered_list_request_dec(n_nodes, n_metrics, v_milli, NULL, present, rule, n_req,
                                     req_node, out_pos);
}

int or_tas_eval_dec(int32_t n_nodes, int32_t n_metrics, const int64_t* v_milli,
                    const int8_t* v_scale, const uint64_t* present, int32_t n_pods,
                    const or_rule* rules, const int32_t* rule_off, const or_rule* prio,
                    const uint64_t* cand, uint32_t flags, uint64_t* pass_out,
                    int32_t* order_out, int32_t* order_len) {
  const int64_t W = w64(n_nodes);
  uint8_t* viol = (uint8_t*)malloc((size_t)(n_nodes > 0 ? n_nodes : 1));
  uint8_t* cset = (uint8_t*)malloc((size_t)(n_nodes > 0 ? n_nodes : 1));
  int rc = 0;
  for (int32_t p = 0; p < n_pods && rc == 0; ++p) {
    /* candidate set (args.Nodes.Items) */
    for (int32_t n = 0; n < n_nodes; ++n)
      cset[n] = cand ? (uint8_t)has_bit(cand + (int64_t)p * W, n) : 1;
    if (flags & 1u) {
      /* filterNodes: violatingNodes := dontscheduleStrategy.Violated(m.cache) (:199) */
      if (violated_dec(n_nodes, n_metrics, v_milli, v_scale, present, rules + rule_off[p],
                       rule_off[p + 1] - rule_off[p], viol) != 0) {
        rc = -1;
        break;
      }
      uint64_t* row = pass_out + (int64_t)p * W;
      memset(row, 0, (size_t)W * sizeof(uint64_t));
      for (int32_t n = 0; n < n_nodes; ++n) { /* for _, node := range args.Nodes.Items */
        if (!cset[n]) continue;
        if (viol[n]) {
          cset[n] = 0;                        /* failedNodes[node.Name] = "Node violates" */
        } else {
          row[n >> 6] |= 1ull << (n & 63);    /* filteredNodes = append(...) */
        }
      }
    }
    if (flags & 2u) {
      /* prioritize over the filter-feasible set (kube-scheduler passes only those) */
      const or_rule* r = &prio[p];
      int32_t len = 0;
      if (r->metric >= 0) {
        /* an unknown operator is not an error here: OrderedList's switch has no default
         * (operator.go:35-40), the list is just left unsorted */
        len = ordered_list_dec(n_nodes, n_metrics, v_milli, v_scale, present, r, cset,
                               order_out + (int64_t)p * n_nodes);
      }
      order_len[p] = len;
    }
  }
  free(viol);
  free(cset);
  return rc;
}

int or_tas_eval(int32_t n_nodes, int32_t n_metrics, const int64_t* v_milli,
                const uint64_t* present, int32_t n_pods, const or_rule* rules,
                const int32_t* rule_off, const or_rule* prio, const uint64_t* cand,
                uint32_t flags, uint64_t* pass_out, int32_t* order_out, int32_t* order_len) {
  return or_tas_eval_dec(n_nodes, n_metrics, v_milli, NULL, present, n_pods, rules, rule_off,
                         prio, cand, flags, pass_out, order_out, order_len);
}

int or_tas_violations_dec(int32_t n_nodes, int32_t n_metrics, const int64_t* v_milli,
                          const int8_t* v_scale, const uint64_t* present, int32_t n_strategies,
                          const or_rule* rules, const int32_t* rule_off, uint64_t* viol_out) {
  const int64_t W = w64(n_nodes);
  uint8_t* viol = (uint8_t*)malloc((size_t)(n_nodes > 0 ? n_nodes : 1));
  int rc = 0;
  /* for strat := range enforcer.RegisteredStrategies[StrategyType] (enforce.go:156) */
  for (int32_t s = 0; s < n_strategies; ++s) {
    if (violated_dec(n_nodes, n_metrics, v_milli, v_scale, present, rules + rule_off[s],
                     rule_off[s + 1] - rule_off[s], viol) != 0) {
      rc = -1;
      break;
    }
    uint64_t* row = viol_out + (int64_t)s * W;
    memset(row, 0, (size_t)W * sizeof(uint64_t));
    for (int32_t n = 0; n < n_nodes; ++n) /* violations[node] = append(..., policy) */
      if (viol[n]) row[n >> 6] |= 1ull << (n & 63);
  }
  free(viol);
  return rc;
}

int or_tas_violations(int32_t n_nodes, int32_t n_metrics, const int64_t* v_milli,
                      const uint64_t* present, int32_t n_strategies, const or_rule* rules,
                      const int32_t* rule_off, uint64_t* viol_out) {
  return or_tas_violations_dec(n_nodes, n_metrics, v_milli, NULL, present, n_strategies, rules,
                               rule_off, viol_out);
}

/* ---- deschedule label payloads ------------------------------------------- */

int or_label_plan(int32_t n_nodes, int32_t n_strat, const char* const* names,
                  const uint64_t* viol, const uint64_t* labels, uint64_t* add, uint64_t* rem,
                  int64_t* total_violations) {
  if (n_strat < 0 || n_strat > 64) return -1;
  const int64_t w = w64(n_nodes);
  /* allPolicies (enforce.go:89-95): the registered strategies' policy NAMES as a set.  A
   * name is represented by its first strategy (first[s] = lowest t with names[t] == names[s]);
   * that strategy's labels row says whether a node carries the label <name>. */
  int32_t first[64];
  for (int32_t s = 0; s < n_strat; ++s) {
    first[s] = s;
    if (names)
      for (int32_t t = 0; t < s; ++t)
        if (strcmp(names[t], names[s]) == 0) { first[s] = t; break; }
  }
  int64_t total = 0;
  for (int32_t n = 0; n < n_nodes; ++n) {          /* for _, node := range allNodes.Items */
    uint64_t a = 0, r = 0;
    uint8_t non_violated[64];                      /* nonViolatedPolicies = allPolicies(...) */
    for (int32_t s = 0; s < n_strat; ++s) non_violated[s] = first[s] == s;
    for (int32_t s = 0; s < n_strat; ++s)          /* for _, policyName := range viols[node] */
      if (has_bit(viol + s * w, n)) {
        non_violated[first[s]] = 0;                /* delete(nonViolatedPolicies, name) */
        a |= 1ull << s;                            /* one "add" per violating strategy */
      }
    for (int32_t k = 0; k < n_strat; ++k)          /* for policyName := range nonViolated... */
      if (non_violated[k]) {
        if (labels && has_bit(labels + k * w, n)) r |= 1ull << k;  /* remove + add "null" */
        ++total;                                   /* totalViolations++ per name (:133) */
      }
    add[n] = a;
    rem[n] = r;
  }
  *total_violations = total;
  return 0;
}

/* Go encoding/json string: ", \, control characters, and the HTML-safe <, >, &. */
static int64_t json_str(const char* s, char* buf, int64_t pos, int64_t cap) {
  static const char hex[] = "0123456789abcdef";
  char tmp[8];
  if (pos < cap) buf[pos] = '"';
  ++pos;
  for (const unsigned char* c = (const unsigned char*)s; *c; ++c) {
    int len = 0;
    if (*c == '"' || *c == '\\') { tmp[0] = '\\'; tmp[1] = (char)*c; len = 2; }
    else if (*c == '\n') { tmp[0] = '\\'; tmp[1] = 'n'; len = 2; }
    else if (*c == '\r') { tmp[0] = '\\'; tmp[1] = 'r'; len = 2; }
    else if (*c == '\t') { tmp[0] = '\\'; tmp[1] = 't'; len = 2; }
    else if (*c < 0x20 || *c == '<' || *c == '>' || *c == '&') {
      tmp[0] = '\\'; tmp[1] = 'u'; tmp[2] = '0'; tmp[3] = '0';
      tmp[4] = hex[*c >> 4]; tmp[5] = hex[*c & 15]; len = 6;
    } else { tmp[0] = (char)*c; len = 1; }
    for (int i = 0; i < len; ++i, ++pos)
      if (pos < cap) buf[pos] = tmp[i];
  }
  if (pos < cap) buf[pos] = '"';
  return pos + 1;
}

static int64_t json_lit(const char* s, char* buf, int64_t pos, int64_t cap) {
  for (; *s; ++s, ++pos)
    if (pos < cap) buf[pos] = *s;
  return pos;
}

static int64_t json_patch(const char* op, const char* name, const char* value, char* buf,
                          int64_t pos, int64_t cap, int first) {
  char path[1024];
  snprintf(path, sizeof path, "/metadata/labels/%s", name);
  if (!first) pos = json_lit(",", buf, pos, cap);
  pos = json_lit("{\"op\":", buf, pos, cap);
  pos = json_str(op, buf, pos, cap);
  pos = json_lit(",\"path\":", buf, pos, cap);
  pos = json_str(path, buf, pos, cap);
  pos = json_lit(",\"value\":", buf, pos, cap);
  pos = json_str(value, buf, pos, cap);
  return json_lit("}", buf, pos, cap);
}

int64_t or_label_patch_json(int32_t n_strat, const char* const* names, uint64_t add, uint64_t rem,
                            char* buf, int64_t cap) {
  int64_t pos = json_lit("[", buf, 0, cap);
  int first = 1;
  for (int32_t s = 0; s < n_strat; ++s)
    if (add >> s & 1) {
      pos = json_patch("add", names[s], "violating", buf, pos, cap, first);
      first = 0;
    }
  for (int32_t s = 0; s < n_strat; ++s)
    if (rem >> s & 1) {
      pos = json_patch("remove", names[s], "", buf, pos, cap, first);
      pos = json_patch("add", names[s], "null", buf, pos, cap, 0);
      first = 0;
    }
  pos = json_lit("]", buf, pos, cap);
  return pos <= cap ? pos : -1;
}

/* ---- GAS resourceMap ------------------------------------------------------ */

int or_rm_add(or_rm* rm, int32_t key, int64_t value) {
  if (value < 0) return OR_RM_ERR_INPUT;               /* minAllowedInput, :78-82 */
  if (rm->has[key]) {
    value = (int64_t)((uint64_t)value + (uint64_t)rm->val[key]); /* Go wraps */
    if (value < 0) return OR_RM_ERR_OVERFLOW;          /* :88-92 */
  }
  rm->has[key] = 1;
  rm->val[key] = value;
  return OR_RM_OK;
}

int or_rm_subtract(or_rm* rm, int32_t key, int64_t value) {
  if (value < 0) return OR_RM_ERR_INPUT;               /* :104-108 */
  if (!rm->has[key]) return OR_RM_ERR_INPUT;           /* non-existing key, :120-124 */
  rm->val[key] = (int64_t)((uint64_t)rm->val[key] - (uint64_t)value);
  if (rm->val[key] < 0) rm->val[key] = 0;              /* capped to zero, :114-119 */
  return OR_RM_OK;
}

int or_rm_add_rm(or_rm* rm, const or_rm* src) {
  or_rm copy = *rm;                                    /* mapCopy := rm.newCopy() */
  for (int32_t k = 0; k < OR_RM_MAX_KEYS; ++k) {
    if (!src->has[k]) continue;
    const int err = or_rm_add(&copy, k, src->val[k]);
    if (err) return err;                               /* nothing added on error */
  }
  *rm = copy;                                          /* rm.copyFrom(mapCopy) */
  return OR_RM_OK;
}

int or_rm_subtract_rm(or_rm* rm, const or_rm* src) {
  or_rm copy = *rm;
  for (int32_t k = 0; k < OR_RM_MAX_KEYS; ++k) {
    if (!src->has[k]) continue;
    const int err = or_rm_subtract(&copy, k, src->val[k]);
    if (err) return err;
  }
  *rm = copy;
  return OR_RM_OK;
}

int or_rm_divide(or_rm* rm, int64_t divider) {       /* Go int: 64 bits */
  if (divider < 1) return OR_RM_ERR_INPUT;             /* :130-134 */
  if (divider == 1) return OR_RM_OK;
  for (int32_t k = 0; k < OR_RM_MAX_KEYS; ++k)
    if (rm->has[k]) rm->val[k] = rm->val[k] / divider; /* truncating, :140-142 */
  return OR_RM_OK;
}

int or_check_resource_capacity(const or_rm* need, const or_rm* capacity, const or_rm* used) {
  for (int32_t k = 0; k < OR_RM_MAX_KEYS; ++k) {       /* for resName, resNeed := range */
    if (!need->has[k]) continue;
    const int64_t res_need = need->val[k];
    if (res_need < 0) return 0;                                  /* :343-347 */
    if (!capacity->has[k] || capacity->val[k] <= 0) return 0;    /* :349-354 */
    const int64_t res_cap = capacity->val[k];
    const int64_t res_used = used->has[k] ? used->val[k] : 0;    /* missing = 0, :356 */
    if (res_used < 0) return 0;                                  /* :358-362 */
    const int64_t sum = (int64_t)((uint64_t)res_used + (uint64_t)res_need);
    if (sum < 0) return 0;                                       /* overflow, :367-371 */
    if (res_cap < sum) return 0;                                 /* :373-377 */
  }
  return 1;
}

/* ---- GAS runSchedulingLogic over the packed snapshot ---------------------- */

/* A growable list of card ranks: the pod's selections in order (the annotation). */
typedef struct {
  int32_t* v;
  int64_t n, cap;
} card_list;

/* More selections than this: the literal loop would not finish in a test's time (the
 * reference appends numI915 card names one by one); the oracle reports an error instead. */
#define OR_SEL_LIST_MAX ((int64_t)1 << 26)

static int list_push(card_list* l, int32_t k) {
  if (l->n >= OR_SEL_LIST_MAX) return -1;
  if (l->n == l->cap) {
    const int64_t cap = l->cap ? 2 * l->cap : 256;
    int32_t* v = (int32_t*)realloc(l->v, (size_t)cap * sizeof(int32_t));
    if (!v) return -1;
    l->v = v;
    l->cap = cap;
  }
  l->v[l->n++] = k;
  return 0;
}

/* runSchedulingLogic (:280-338) of pod p on node n over the packed snapshot, as the reference
 * writes it: per container getPerGPUResourceRequest (:180-190), then numI915 times the first
 * card in sort.Strings order passing checkResourceCapacity on the working copy, which then
 * takes the request (addRM, :200-257).  No bound on numI915: the loop ends at the first
 * selection no card fits.  Returns 1 (fits) / 0; the selections go to `sel` and, per
 * container, their count to cont_n[c] (when not NULL).  -1 on allocation failure. */
static int fit_one(int32_t max_cards, int32_t n_res, int32_t nc_node, const int64_t* cap_per_gpu,
                   const int64_t* used, int32_t max_containers, int32_t i915_index,
                   const int64_t* req, const uint32_t* req_mask, int32_t n_containers,
                   card_list* sel, int64_t* cont_n) {
  sel->n = 0;
  for (int32_t c = 0; cont_n && c < max_containers; ++c) cont_n[c] = 0;
  /* iCache.FetchNode error (:282-288) / no cards label -> errWontFit (:290-298) */
  if (nc_node <= 0) return 0;
  const int32_t ncard = nc_node < max_cards ? nc_node : max_cards;
  or_rm capacity, node_used[OR_GAS_MAX_CARDS];
  memset(&capacity, 0, sizeof capacity);
  for (int32_t q = 0; q < n_res; ++q) {                 /* getPerGPUResourceCapacity */
    capacity.has[q] = 1;
    capacity.val[q] = cap_per_gpu[q];
  }
  /* readNodeResources deep copy (node_resource_cache.go:474-491) + addEmptyResourceMaps
   * (:269-275): a fresh copy per (pod, node) */
  for (int32_t k = 0; k < ncard; ++k) {
    memset(&node_used[k], 0, sizeof(or_rm));
    for (int32_t q = 0; q < n_res; ++q) {
      node_used[k].has[q] = 1;
      node_used[k].val[q] = used[(int64_t)k * n_res + q];
    }
  }
  for (int32_t c = 0; c < n_containers; ++c) {         /* for i, containerRequest */
    const uint32_t mask = req_mask[c];
    if (mask == 0) continue;                            /* len(containerRequest) == 0 -> [] :206-208 */
    or_rm per_gpu;                                      /* getPerGPUResourceRequest :180-190 */
    memset(&per_gpu, 0, sizeof per_gpu);
    for (int32_t q = 0; q < n_res; ++q)
      if (mask & (1u << q)) { per_gpu.has[q] = 1; per_gpu.val[q] = req[(int64_t)c * n_res + q]; }
    if (mask & OR_REQ_UNKNOWN_KIND) per_gpu.has[OR_UNKNOWN_KEY] = 1;  /* no capacity key */
    int64_t num_i915 = 0;                               /* getNumI915 :192-198 */
    if (i915_index >= 0 && per_gpu.has[i915_index] && per_gpu.val[i915_index] > 0)
      num_i915 = per_gpu.val[i915_index];
    if (num_i915 > 1) or_rm_divide(&per_gpu, num_i915);
    for (int64_t g = 0; g < num_i915; ++g) {            /* for gpuNum := 0; gpuNum < numI915 */
      int fitted = 0;
      /* cards in sort.Strings order; stale cards are absent from the packed snapshot, which
       * equals skipping them (!gpuMap[gpuName] -> continue, :230-234) */
      for (int32_t k = 0; k < ncard; ++k) {
        if (or_check_resource_capacity(&per_gpu, &capacity, &node_used[k])) {
          if (or_rm_add_rm(&node_used[k], &per_gpu) == OR_RM_OK) {
            fitted = 1;
            if (list_push(sel, k)) return -1;           /* cards = append(cards, gpuName) */
            if (cont_n) ++cont_n[c];
          }
          break;
        }
      }
      if (!fitted) return 0;                            /* errWontFit :249-253 */
    }
  }
  return 1;
}

/* The pas_gas_fit word of a fitting selection list. */
static uint32_t fit_word(const card_list* sel) {
  if (sel->n > OR_GAS_MAX_SEL) return 0x80000000u | ((uint32_t)OR_GAS_SEL_LIMIT << 24);
  int packable = sel->n <= 8;
  for (int64_t j = 0; j < sel->n; ++j) packable = packable && sel->v[j] < 8;
  if (!packable) return 0x80000000u | ((uint32_t)OR_GAS_SEL_EXTENDED << 24);
  uint32_t word = 0x80000000u | ((uint32_t)sel->n << 24);
  for (int64_t j = 0; j < sel->n; ++j) word |= (uint32_t)sel->v[j] << (3 * j);
  return word;
}

/* Builds the reference's maps from the packed layout: capacity has every resource kind
 * with a positive per-GPU value... careful: a kind whose per-GPU capacity is 0 may
 * still be a key of the capacity map, but checkResourceCapacity treats "missing" and
 * "<= 0" identically (:349-354), so has = 1 with the stored value is equivalent. */
int or_gas_fit_ex(int32_t n_nodes, int32_t max_cards, int32_t n_res, const int32_t* n_cards,
                  const int64_t* cap_per_gpu, const int64_t* used, int32_t n_pods,
                  int32_t max_containers, int32_t i915_index, const int64_t* req,
                  const uint32_t* req_mask, const int32_t* n_containers, uint32_t* res_out,
                  uint8_t* sel_out, int32_t* nsel_out) {
  if (max_cards > OR_GAS_MAX_CARDS || n_res > OR_UNKNOWN_KEY) return -1;
  card_list sel = {0};
  int rc = 0;
  for (int32_t p = 0; p < n_pods && !rc; ++p) {
    for (int32_t n = 0; n < n_nodes; ++n) {
      const int64_t pn = (int64_t)p * n_nodes + n;
      const int f = fit_one(max_cards, n_res, n_cards[n], cap_per_gpu + (int64_t)n * n_res,
                            used + (int64_t)n * max_cards * n_res, max_containers, i915_index,
                            req + (int64_t)p * max_containers * n_res,
                            req_mask + (int64_t)p * max_containers, n_containers[p], &sel, NULL);
      if (f < 0) { rc = -3; break; }
      res_out[pn] = f ? fit_word(&sel) : 0u;
      if (nsel_out) nsel_out[pn] = !f ? 0 : sel.n > OR_GAS_MAX_SEL ? -1 : (int32_t)sel.n;
      if (sel_out) {
        memset(sel_out + pn * OR_GAS_MAX_SEL, 0, OR_GAS_MAX_SEL);
        if (f && sel.n <= OR_GAS_MAX_SEL)
          for (int64_t j = 0; j < sel.n; ++j) sel_out[pn * OR_GAS_MAX_SEL + j] = (uint8_t)sel.v[j];
      }
    }
  }
  free(sel.v);
  return rc;
}

int or_gas_fit(int32_t n_nodes, int32_t max_cards, int32_t n_res, const int32_t* n_cards,
               const int64_t* cap_per_gpu, const int64_t* used, int32_t n_pods,
               int32_t max_containers, int32_t i915_index, const int64_t* req,
               const uint32_t* req_mask, const int32_t* n_containers, uint32_t* res_out) {
  return or_gas_fit_ex(n_nodes, max_cards, n_res, n_cards, cap_per_gpu, used, n_pods,
                       max_containers, i915_index, req, req_mask, n_containers, res_out, NULL,
                       NULL);
}

/* ---- GAS bind-time commit ------------------------------------------------- */

/* The node's usage as resourceMaps (every kind of a labelled card is a key). */
static void node_maps(int32_t max_cards, int32_t n_res, int32_t ncard, const int64_t* u,
                      or_rm* out) {
  for (int32_t k = 0; k < max_cards; ++k) {
    memset(&out[k], 0, sizeof(or_rm));
    if (k >= ncard) continue;
    for (int32_t q = 0; q < n_res; ++q) {
      out[k].has[q] = 1;
      out[k].val[q] = u[(int64_t)k * n_res + q];
    }
  }
}

static void container_map(int32_t n_res, const int64_t* req, uint32_t mask, or_rm* out) {
  memset(out, 0, sizeof(or_rm));                    /* containerRequests (utils.go:14-32) */
  for (int32_t q = 0; q < n_res; ++q)
    if (mask & (1u << q)) { out->has[q] = 1; out->val[q] = req[q]; }
  if (mask & OR_REQ_UNKNOWN_KIND) out->has[OR_UNKNOWN_KEY] = 1;  /* a kind no map holds */
}

int or_gas_bind(int32_t n_nodes, int32_t max_cards, int32_t n_res, const int32_t* n_cards,
                const int64_t* cap_per_gpu, int64_t* used, int32_t n_binds,
                const int32_t* bind_pod, const int32_t* bind_node, int32_t max_containers,
                int32_t i915_index, const int64_t* req, const uint32_t* req_mask,
                const int32_t* n_containers, uint32_t* res_out, int32_t* status,
                uint8_t* cards_out, int32_t* nsel_out, int64_t* counts_out) {
  if (max_cards > OR_GAS_MAX_CARDS || n_res > OR_UNKNOWN_KEY) return -1;
  card_list sel = {0};
  int64_t* cont_n = (int64_t*)calloc((size_t)(max_containers > 0 ? max_containers : 1),
                                     sizeof(int64_t));
  if (!cont_n) return -3;
  int rc = 0;
  const int64_t ck = (int64_t)max_containers * max_cards;
  for (int32_t b = 0; b < n_binds; ++b) {
    const int32_t p = bind_pod[b], n = bind_node[b];
    if (n < 0 || n >= n_nodes) { rc = -1; break; }
    int64_t* u = used + (int64_t)n * max_cards * n_res;
    if (cards_out) memset(cards_out + (int64_t)b * OR_GAS_MAX_SEL, 0, OR_GAS_MAX_SEL);
    if (nsel_out) nsel_out[b] = 0;
    if (counts_out)
      for (int64_t j = 0; j < ck; ++j) counts_out[b * ck + j] = 0;
    /* runSchedulingLogic(pod, node) on the current usage */
    const int f = fit_one(max_cards, n_res, n_cards[n], cap_per_gpu + (int64_t)n * n_res, u,
                          max_containers, i915_index, req + (int64_t)p * max_containers * n_res,
                          req_mask + (int64_t)p * max_containers, n_containers[p], &sel, cont_n);
    if (f < 0) { rc = -3; break; }
    res_out[b] = f ? fit_word(&sel) : 0u;
    if (!f) { status[b] = OR_GAS_WONT_FIT; continue; }
    /* adjustPodResources(add): the annotation lists, per container, the cards of its
     * selections (numCards = numI915); checked on a copy, then applied */
    or_rm maps[OR_GAS_MAX_CARDS];
    node_maps(max_cards, n_res, n_cards[n], u, maps);
    int64_t s_i = 0;
    int32_t err = OR_RM_OK;
    for (int32_t c = 0; c < n_containers[p] && !err; ++c) {
      const int64_t base = (int64_t)p * max_containers + c;
      const int64_t k_c = cont_n[c];
      if (k_c <= 0) continue;                       /* empty segment: skipped */
      or_rm r;
      container_map(n_res, req + base * n_res, req_mask[base], &r);
      or_rm_divide(&r, k_c);
      for (int64_t g = 0; g < k_c && !err; ++g, ++s_i)
        err = or_rm_add_rm(&maps[sel.v[s_i]], &r);
    }
    if (err) {                                       /* nothing changes */
      status[b] = err == OR_RM_ERR_OVERFLOW ? OR_GAS_ERR_OVERFLOW : OR_GAS_ERR_INPUT;
      continue;
    }
    for (int32_t k = 0; k < n_cards[n]; ++k)
      for (int32_t q = 0; q < n_res; ++q) u[(int64_t)k * n_res + q] = maps[k].val[q];
    if (cards_out && sel.n <= OR_GAS_MAX_SEL)
      for (int64_t j = 0; j < sel.n; ++j) cards_out[(int64_t)b * OR_GAS_MAX_SEL + j] = (uint8_t)sel.v[j];
    if (nsel_out) nsel_out[b] = sel.n > OR_GAS_MAX_SEL ? -1 : (int32_t)sel.n;
    if (counts_out) {
      int64_t j = 0;
      for (int32_t c = 0; c < n_containers[p]; ++c)
        for (int64_t g = 0; g < cont_n[c]; ++g, ++j) ++counts_out[b * ck + (int64_t)c * max_cards + sel.v[j]];
    }
    status[b] = OR_GAS_OK;
  }
  free(sel.v);
  free(cont_n);
  return rc;
}

/* One pod leaving node n: container c's annotation segment is cards[off .. off + cpc[c]). */
static int32_t release_one(int32_t max_cards, int32_t n_res, int32_t nc_node, int64_t* u,
                           int32_t n_containers, const int64_t* req, const uint32_t* req_mask,
                           const int64_t* cpc, const int32_t* cards, int64_t n_cards_list) {
  const int32_t ncard = nc_node > 0 ? nc_node : 0;
  or_rm maps[OR_GAS_MAX_CARDS], stale;
  node_maps(max_cards, n_res, ncard, u, maps);
  int64_t off = 0;
  int32_t err = OR_RM_OK;
  for (int32_t c = 0; c < n_containers && !err; ++c) {
    const int64_t k_c = cpc[c];
    if (k_c <= 0) continue;                          /* empty segment */
    or_rm q;
    container_map(n_res, req + (int64_t)c * n_res, req_mask[c], &q);
    or_rm_divide(&q, k_c);
    for (int64_t j = 0; j < k_c && !err; ++j) {
      const int32_t k = off + j < n_cards_list ? cards[off + j] : -1;
      if (k >= 0 && k < ncard) {
        err = or_rm_subtract_rm(&maps[k], &q);
      } else {                                       /* new empty map for the card */
        memset(&stale, 0, sizeof stale);
        err = or_rm_subtract_rm(&stale, &q);
      }
    }
    off += k_c;
  }
  if (err) return OR_GAS_ERR_INPUT;
  for (int32_t k = 0; k < ncard; ++k)
    for (int32_t q = 0; q < n_res; ++q) u[(int64_t)k * n_res + q] = maps[k].val[q];
  return OR_GAS_OK;
}

int or_gas_release(int32_t n_nodes, int32_t max_cards, int32_t n_res, const int32_t* n_cards,
                   int64_t* used, int32_t n_rel, const int32_t* rel_pod,
                   const int32_t* rel_node, int32_t max_containers, const int64_t* req,
                   const uint32_t* req_mask, const int32_t* n_containers,
                   const int32_t* cards_per_container, const int32_t* cards, int32_t cards_stride,
                   int32_t* status) {
  if (max_cards > OR_GAS_MAX_CARDS || n_res > OR_UNKNOWN_KEY) return -1;
  int64_t* cpc = (int64_t*)calloc((size_t)(max_containers > 0 ? max_containers : 1),
                                  sizeof(int64_t));
  if (!cpc) return -3;
  int rc = 0;
  for (int32_t r = 0; r < n_rel; ++r) {
    const int32_t p = rel_pod[r], n = rel_node[r];
    if (n < 0 || n >= n_nodes) { rc = -1; break; }
    for (int32_t c = 0; c < max_containers; ++c)
      cpc[c] = cards_per_container[(int64_t)r * max_containers + c];
    status[r] = release_one(max_cards, n_res, n_cards[n], used + (int64_t)n * max_cards * n_res,
                            n_containers[p], req + (int64_t)p * max_containers * n_res,
                            req_mask + (int64_t)p * max_containers, cpc,
                            cards + (int64_t)r * cards_stride, cards_stride);
  }
  free(cpc);
  return rc;
}

int or_gas_release_counts(int32_t n_nodes, int32_t max_cards, int32_t n_res,
                          const int32_t* n_cards, int64_t* used, int32_t n_rel,
                          const int32_t* rel_pod, const int32_t* rel_node,
                          int32_t max_containers, const int64_t* req, const uint32_t* req_mask,
                          const int32_t* n_containers, const int64_t* counts, int32_t* status) {
  if (max_cards > OR_GAS_MAX_CARDS || n_res > OR_UNKNOWN_KEY) return -1;
  int64_t* cpc = (int64_t*)calloc((size_t)(max_containers > 0 ? max_containers : 1),
                                  sizeof(int64_t));
  card_list list = {0};
  int rc = cpc ? 0 : -3;
  const int64_t ck = (int64_t)max_containers * max_cards;
  for (int32_t r = 0; r < n_rel && !rc; ++r) {
    const int32_t p = rel_pod[r], n = rel_node[r];
    if (n < 0 || n >= n_nodes) { rc = -1; break; }
    /* the annotation the counts stand for: per container, card k counts[r][c][k] times, in
     * card order */
    list.n = 0;
    for (int32_t c = 0; c < max_containers && !rc; ++c) {
      cpc[c] = 0;
      for (int32_t k = 0; k < max_cards && !rc; ++k) {
        const int64_t t = counts[r * ck + (int64_t)c * max_cards + k];
        for (int64_t j = 0; j < t && !rc; ++j) rc = list_push(&list, k) ? -3 : 0;
        cpc[c] += t > 0 ? t : 0;
      }
    }
    if (rc) break;
    status[r] = release_one(max_cards, n_res, n_cards[n], used + (int64_t)n * max_cards * n_res,
                            n_containers[p], req + (int64_t)p * max_containers * n_res,
                            req_mask + (int64_t)p * max_containers, cpc, list.v, list.n);
  }
  free(list.v);
  free(cpc);
  return rc;
}
