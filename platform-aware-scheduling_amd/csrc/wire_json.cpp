// wire_json.cpp — extender response bodies from the evaluator's index outputs (SURVEY.md
// §8 f2), byte for byte what the reference's handlers write with
// json.NewEncoder(w).Encode(result) (a trailing newline included):
//
//   HostPriorityList (extender/types.go:25-33), WritePrioritizeResponse
//     (telemetryscheduler.go:152-158):  [{"Host":"<name>","Score":<10-i>},...]
//   TAS FilterResult (types.go:56-66), filterNodes + WriteFilterResponse
//     (telemetryscheduler.go:184-225, 238-244):
//     {"Nodes":{"metadata":{},"items":[<node>,...]},"NodeNames":["a","b",""],
//      "FailedNodes":{"<name>":"Node violates",...},"Error":""}
//     items is null when no node passes (a nil []v1.Node); NodeNames is
//     strings.Split("<name> <name> ... ", " ") (:209-212): a trailing "", and a name with
//     spaces split into pieces; map keys are sorted, as encoding/json does.
//   GAS FilterResult, filterNodes (gpuscheduler/scheduler.go:449-482):
//     {"Nodes":null,"NodeNames":[...] or null,"FailedNodes":{...},"Error":""}
//     and the misconfiguration error result for an empty NodeNames (:455-461).
//
// The struct fields carry no json tags, so keys are the Go field names; v1.NodeList has
// TypeMeta inline (kind / apiVersion omitempty, absent here) and ListMeta under "metadata"
// (all fields omitempty: {}).  Node objects are spliced in as the caller's JSON text of each
// node (the shim keeps json.Marshal(node) per snapshot node: nodes do not change between
// requests).  Names are Kubernetes node names; the string encoder is nevertheless the
// general one (json_out.h).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "host_pool.h"
#include "json_out.h"
#include "pas.h"

namespace {

bool passed(const uint64_t* bits, int32_t n) { return (bits[n >> 6] >> (n & 63)) & 1ull; }

// FailedNodes: distinct names sorted bytewise (Go sorts map keys by their string).
void failed_nodes(pas::JsonOut& o, std::vector<const char*>& names, const char* reason) {
  std::sort(names.begin(), names.end(), [](const char* a, const char* b) {
    return std::strcmp(a, b) < 0;
  });
  names.erase(std::unique(names.begin(), names.end(),
                          [](const char* a, const char* b) { return std::strcmp(a, b) == 0; }),
              names.end());
  o.put('{');
  for (size_t i = 0; i < names.size(); ++i) {
    if (i) o.put(',');
    o.str(names[i]);
    o.put(':');
    o.str(reason);
  }
  o.put('}');
}

// Items [0, n) joined by `sep` (0: none), encode(o, i) writing item i.  Many items are split
// over host threads: each thread encodes a contiguous range into a buffer of its own (a
// counting pass for the size, then the writing pass), and the pieces are appended in order.
template <class F>
void encode_items(pas::JsonOut& o, int64_t n, char sep, int64_t bytes_per_item, F&& encode) {
  // one thread per 256 KiB of output: the items' scattered reads, not the bytes, set the pace
  const int T = n >= 4096 ? (int)std::min<int64_t>(pas::host_threads_for(4 * n * bytes_per_item),
                                                   n / 1024)
                          : 1;
  auto range = [&](pas::JsonOut& w, int64_t i0, int64_t i1) {
    for (int64_t i = i0; i < i1; ++i) {
      if (i && sep) w.put(sep);
      encode(w, i);
    }
  };
  if (T <= 1) {
    range(o, 0, n);
    return;
  }
  // kHostPieces ranges per thread, taken in turn
  const int R = (int)std::min<int64_t>((int64_t)T * pas::kHostPieces, n / 256);
  std::vector<std::string> part((size_t)R);
  auto run = [&](int t) {
    const int64_t i0 = n * t / R, i1 = n * (t + 1) / R;
    // one pass into a buffer of twice the estimate; a range that outgrows it (long names,
    // escapes) is encoded again at its counted length
    std::string& b = part[(size_t)t];
    b.resize((size_t)(2 * bytes_per_item * (i1 - i0) + 4096));
    pas::JsonOut w{&b[0], (int64_t)b.size()};
    range(w, i0, i1);
    if (w.pos > (int64_t)b.size()) {
      b.resize((size_t)w.pos);
      pas::JsonOut again{&b[0], (int64_t)b.size()};
      range(again, i0, i1);
    }
    b.resize((size_t)w.pos);
  };
  if (!pas::host_parallel(R, run, T)) {
    range(o, 0, n);
    return;
  }
  for (const std::string& s : part) o.raw(s.data(), (int64_t)s.size());
}

int finish(pas::JsonOut& o, int64_t* out_len) {
  o.put('\n');  // json.Encoder terminates each value with a newline
  *out_len = o.pos;
  return o.pos <= o.cap ? PAS_OK : PAS_ECAPACITY;
}

bool out_ok(char* buf, int64_t cap, int64_t* out_len) {
  return out_len && cap >= 0 && (cap == 0 || buf);
}

}  // namespace

extern "C" {

int pas_encode_host_priority_list(int32_t len, const int32_t* order, const char* const* names,
                                  char* buf, int64_t cap, int64_t* out_len) {
  if (len < 0 || (len > 0 && (!order || !names)) || !out_ok(buf, cap, out_len))
    return PAS_EINVAL;
  for (int32_t i = 0; i < len; ++i)
    if (order[i] < 0 || !names[order[i]]) return PAS_EINVAL;
  pas::JsonOut o{buf, cap};
  o.put('[');
  encode_items(o, len, ',', 40, [&](pas::JsonOut& w, int64_t i) {
    // the names are read in list order, i.e. scattered over the table: fetch ahead
    if (i + 64 < len) __builtin_prefetch(&names[order[i + 64]]);
    if (i + 24 < len) __builtin_prefetch(names[order[i + 24]]);
    w.lit("{\"Host\":");
    w.str(names[order[i]]);
    w.lit(",\"Score\":");
    w.integer(10 - i);  // Score: 10 - i (telemetryscheduler.go:145-147)
    w.put('}');
  });
  o.put(']');
  return finish(o, out_len);
}

int pas_encode_tas_filter_result(int32_t n_req, const int32_t* req_node, const uint64_t* pass,
                                 const char* const* names, const char* const* node_json,
                                 const int64_t* node_json_len, char* buf, int64_t cap,
                                 int64_t* out_len) {
  if (n_req < 0 || (n_req > 0 && (!req_node || !pass || !names || !node_json || !node_json_len)) ||
      !out_ok(buf, cap, out_len))
    return PAS_EINVAL;
  for (int32_t i = 0; i < n_req; ++i)
    if (req_node[i] < 0 || !names[req_node[i]] || !node_json[req_node[i]] ||
        node_json_len[req_node[i]] < 0)
      return PAS_EINVAL;
  pas::JsonOut o{buf, cap};
  bool any = false;
  for (int32_t i = 0; i < n_req && !any; ++i) any = passed(pass, req_node[i]);
  o.lit("{\"Nodes\":{\"metadata\":{},\"items\":");
  if (!any) {
    o.lit("null");
  } else {
    o.put('[');
    // the passing nodes' JSON, comma-separated: offsets first, then the copies over host
    // threads (chunks of about equal bytes); bytes past cap are counted, not stored
    std::vector<int32_t> item;
    std::vector<int64_t> at;
    int64_t pos = o.pos;
    for (int32_t i = 0; i < n_req; ++i) {
      const int32_t n = req_node[i];
      if (!passed(pass, n)) continue;
      if (!item.empty()) ++pos;  // the comma before it
      item.push_back(n);
      at.push_back(pos);
      pos += node_json_len[n];
    }
    const int64_t begin = o.pos, end = pos;
    const int T = (int)std::min<int64_t>(pas::host_threads_for(end - begin), (int64_t)item.size());
    // kHostPieces byte ranges per thread, taken in turn
    const int R = (int)std::min<int64_t>((int64_t)std::max(T, 1) * pas::kHostPieces,
                                         std::max<int64_t>((int64_t)item.size(), 1));
    auto copy = [&](int t) {
      const int64_t lo = begin + (end - begin) * t / R;
      const int64_t hi = t == R - 1 ? INT64_MAX : begin + (end - begin) * (t + 1) / R;
      size_t j = std::lower_bound(at.begin(), at.end(), lo) - at.begin();
      for (; j < item.size() && at[j] < hi; ++j) {
        const int64_t a = at[j], len = node_json_len[item[j]];
        if (j > 0 && a - 1 < cap) buf[a - 1] = ',';
        if (a < cap) std::memcpy(buf + a, node_json[item[j]], (size_t)std::min(len, cap - a));
      }
    };
    if (T <= 1 || !pas::host_parallel(R, copy, T))
      for (int t = 0; t < R; ++t) copy(t);
    o.pos = end;
    o.put(']');
  }
  o.lit("},\"NodeNames\":[");
  std::vector<const char*> failed;
  std::vector<const char*> ok_names;
  for (int32_t i = 0; i < n_req; ++i) {
    const int32_t n = req_node[i];
    (passed(pass, n) ? ok_names : failed).push_back(names[n]);
  }
  // availableNodeNames += node.Name + " ", later split on " ": a name with spaces becomes
  // several entries; each followed by a comma, then the final "" of the split
  encode_items(o, (int64_t)ok_names.size(), 0, 24, [&](pas::JsonOut& w, int64_t i) {
    const char* p = ok_names[(size_t)i];
    for (;;) {
      const char* sp = std::strchr(p, ' ');
      const int64_t len = sp ? sp - p : (int64_t)std::strlen(p);
      w.str_n(p, len);
      w.put(',');
      if (!sp) break;
      p = sp + 1;
    }
  });
  o.lit("\"\"],\"FailedNodes\":");
  // strings.Join([]string{"Node violates"}, policy.Name) is "Node violates" (:206)
  failed_nodes(o, failed, "Node violates");
  o.lit(",\"Error\":\"\"}");
  return finish(o, out_len);
}

int pas_encode_gas_filter_result(int32_t n_req, const int32_t* req_node, const uint64_t* fit,
                                 const char* const* names, char* buf, int64_t cap,
                                 int64_t* out_len) {
  if (n_req < 0 || (n_req > 0 && (!req_node || !fit || !names)) || !out_ok(buf, cap, out_len))
    return PAS_EINVAL;
  for (int32_t i = 0; i < n_req; ++i)
    if (req_node[i] < 0 || !names[req_node[i]]) return PAS_EINVAL;
  pas::JsonOut o{buf, cap};
  if (n_req == 0) {  // args.NodeNames nil or empty (:455-461)
    o.lit("{\"Nodes\":null,\"NodeNames\":null,\"FailedNodes\":null,\"Error\":");
    o.str("No nodes to compare. This should not happen, perhaps the extender is "
          "misconfigured with NodeCacheCapable == false.");
    o.put('}');
    return finish(o, out_len);
  }
  o.lit("{\"Nodes\":null,\"NodeNames\":");
  bool first = true;
  std::vector<const char*> failed;
  for (int32_t i = 0; i < n_req; ++i) {
    const int32_t n = req_node[i];
    if (!passed(fit, n)) {
      failed.push_back(names[n]);
      continue;
    }
    o.put(first ? '[' : ',');
    first = false;
    o.str(names[n]);
  }
  if (first)
    o.lit("null");  // var nodeNames []string stays nil
  else
    o.put(']');
  o.lit(",\"FailedNodes\":");
  failed_nodes(o, failed, "Not enough GPU-resources for deployment");
  o.lit(",\"Error\":\"\"}");
  return finish(o, out_len);
}

// BindingResult (extender/types.go:79-82) of GASExtender.bindNode (scheduler.go:385-445):
// {"Error":"<err.Error()>"} or {"Error":""} on success.
int pas_encode_binding_result(const char* error, char* buf, int64_t cap, int64_t* out_len) {
  if (!out_ok(buf, cap, out_len)) return PAS_EINVAL;
  pas::JsonOut o{buf, cap};
  o.lit("{\"Error\":");
  o.str(error ? error : "");
  o.put('}');
  return finish(o, out_len);
}

}  // extern "C"
