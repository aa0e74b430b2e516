// wire_decode.cpp — extender request decoding, host only.
//
// The reference decodes every Filter / Prioritize body with
//   json.NewDecoder(r.Body).Decode(&args)          (extender.Args, extender/types.go:36-46)
// in MetricsExtender.DecodeExtenderRequest (telemetryscheduler.go:63-78) and
// GASExtender.decodeRequest (gpuscheduler/scheduler.go:486-505), then walks
// args.Nodes.Items (TAS) or *args.NodeNames (GAS) in request order.  Here one pass over the
// body resolves the request's nodes to snapshot node ids (a name table built once per
// snapshot) and sets the candidate bitmap the TAS / GAS calls take, without materialising
// the v1.NodeList.  The pod's policy label / namespace (getPolicyFromPod,
// telemetryscheduler.go:103-112) and its gpu.intel.com requests (containerRequests,
// gpuscheduler/utils.go:14-32) come from the Pod value's span.
//
// encoding/json (Go 1.16) semantics restated for the fields on this path:
//   - one value is read; bytes after it are not looked at (Decoder.Decode); an empty body is
//     an error (io.EOF); syntax errors and nesting deeper than 10000 are errors;
//   - object keys are unescaped, then matched to struct fields exactly or, failing that, by
//     the field's fold function (foldFunc: equalFoldRight for names with k/s, which also
//     accepts U+212A KELVIN SIGN and U+017F LATIN SMALL LETTER LONG S; ASCII letter folding
//     otherwise); map keys (labels, requests) match exactly; a repeated key is decoded again
//     (the last one wins for the values read here); unknown keys are skipped;
//   - null leaves a string unchanged and sets a pointer / slice / map to nil; a value of the
//     wrong JSON type is an UnmarshalTypeError, reported after the whole value is decoded, so
//     the request fails as a decode error;
//   - strings: \uXXXX escapes with UTF-16 surrogate pairs (an unpaired surrogate becomes
//     U+FFFD), invalid UTF-8 bytes become U+FFFD, raw control characters are syntax errors;
//   - resource.Quantity.UnmarshalJSON (apimachinery v0.22.2 quantity.go): null is the zero
//     quantity; otherwise the literal bytes, with surrounding quotes removed and spaces
//     trimmed, go to ParseQuantity (a failure is a decode error).
// Every field of v1.Pod / v1.NodeList is type-checked against k8s.io/api v0.22.2's Go types
// (k8s_schema.h: a mistyped field anywhere, e.g. a node's "status": 5 or a malformed
// creationTimestamp, fails the request as it fails the reference's decode); unknown keys
// are skipped as syntax.
#include <emmintrin.h>

#ifdef PAS_DECODE_TRACE  // diagnostic builds: phase times of the threaded decode on stderr
#include <chrono>
#include <cstdio>
#define PAS_TRACE_T0(v) const auto v = std::chrono::steady_clock::now()
#define PAS_TRACE_MS(msg, v)                                                       \
  std::fprintf(stderr, "decode %s %.3f ms\n", msg,                                \
               std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - v).count())
#else
#define PAS_TRACE_T0(v)
#define PAS_TRACE_MS(msg, v)
#endif

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include "host_pool.h"
#include "k8s_schema.h"
#include "pas.h"

namespace {

constexpr int kMaxDepth = 10000;  // encoding/json maxNestingDepth

// ---------------------------------------------------------------------------- field folding

bool has_special_fold(const char* f) {  // foldFunc: 'k' / 's' in the name -> equalFoldRight
  for (; *f; ++f) {
    const char b = (char)(*f | 0x20);
    if (b == 'k' || b == 's') return true;
  }
  return false;
}

// bytes.EqualFold-style matches of a key (unescaped) against an ASCII-letter field name.
bool fold_match(const char* field, std::string_view key) {
  const size_t fl = std::strlen(field);
  if (key.size() == fl && std::memcmp(key.data(), field, fl) == 0) return true;
  if (!has_special_fold(field)) {  // simpleLetterEqualFold
    if (key.size() != fl) return false;
    for (size_t i = 0; i < fl; ++i)
      if ((field[i] & ~0x20) != (key[i] & ~0x20)) return false;
    return true;
  }
  // equalFoldRight(field, key)
  size_t t = 0;
  for (size_t i = 0; i < fl; ++i) {
    if (t >= key.size()) return false;
    const unsigned char tb = (unsigned char)key[t];
    const char sb = field[i];
    if (tb < 0x80) {
      if (sb != (char)tb) {
        const char su = (char)(sb & ~0x20);
        if (su < 'A' || su > 'Z' || su != (char)(tb & ~0x20)) return false;
      }
      ++t;
      continue;
    }
    // multi-byte rune in the key: only KELVIN SIGN (E2 84 AA) for k and LONG S (C5 BF) for s
    const char sl = (char)(sb | 0x20);
    if (sl == 's' && t + 1 < key.size() && tb == 0xC5 && (unsigned char)key[t + 1] == 0xBF) {
      t += 2;
    } else if (sl == 'k' && t + 2 < key.size() && tb == 0xE2 &&
               (unsigned char)key[t + 1] == 0x84 && (unsigned char)key[t + 2] == 0xAA) {
      t += 3;
    } else {
      return false;
    }
  }
  return t == key.size();
}

// ---------------------------------------------------------------------------- scanner

void put_utf8(std::string* o, uint32_t r) {
  if (r < 0x80) {
    o->push_back((char)r);
  } else if (r < 0x800) {
    o->push_back((char)(0xC0 | (r >> 6)));
    o->push_back((char)(0x80 | (r & 0x3F)));
  } else if (r < 0x10000) {
    o->push_back((char)(0xE0 | (r >> 12)));
    o->push_back((char)(0x80 | ((r >> 6) & 0x3F)));
    o->push_back((char)(0x80 | (r & 0x3F)));
  } else {
    o->push_back((char)(0xF0 | (r >> 18)));
    o->push_back((char)(0x80 | ((r >> 12) & 0x3F)));
    o->push_back((char)(0x80 | ((r >> 6) & 0x3F)));
    o->push_back((char)(0x80 | (r & 0x3F)));
  }
}

// Length of a valid UTF-8 sequence at s (utf8.DecodeRune), 0 if invalid.
int utf8_valid(const unsigned char* s, const unsigned char* end) {
  const unsigned char c = s[0];
  const ptrdiff_t n = end - s;
  auto cont = [](unsigned char x) { return (x & 0xC0) == 0x80; };
  if (c >= 0xC2 && c <= 0xDF) return n >= 2 && cont(s[1]) ? 2 : 0;
  if (c >= 0xE0 && c <= 0xEF) {
    if (n < 3 || !cont(s[1]) || !cont(s[2])) return 0;
    if (c == 0xE0 && s[1] < 0xA0) return 0;  // overlong
    if (c == 0xED && s[1] >= 0xA0) return 0;  // surrogate
    return 3;
  }
  if (c >= 0xF0 && c <= 0xF4) {
    if (n < 4 || !cont(s[1]) || !cont(s[2]) || !cont(s[3])) return 0;
    if (c == 0xF0 && s[1] < 0x90) return 0;
    if (c == 0xF4 && s[1] >= 0x90) return 0;
    return 4;
  }
  return 0;
}

int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

// First byte at or after p that ends a run of plain string bytes (>= 0x20, < 0x80, not '"'
// or '\\'), 16 bytes per step (SSE2: bytes >= 0x80 compare below 0x20 as signed).
inline const char* scan_plain(const char* p, const char* end) {
  const __m128i quote = _mm_set1_epi8('"'), bslash = _mm_set1_epi8('\\');
  const __m128i space = _mm_set1_epi8(0x20);
  while (end - p >= 16) {
    const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
    const __m128i m = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(v, quote), _mm_cmpeq_epi8(v, bslash)),
                                   _mm_cmplt_epi8(v, space));
    const int mask = _mm_movemask_epi8(m);
    if (mask) return p + __builtin_ctz((unsigned)mask);
    p += 16;
  }
  while (p < end && (unsigned char)*p >= 0x20 && *p != '"' && *p != '\\' &&
         (unsigned char)*p < 0x80)
    ++p;
  return p;
}

struct Scanner {
  const char* p;
  const char* end;
  bool syntax_err = false;  // malformed JSON: nothing is decoded
  bool type_err = false;    // UnmarshalTypeError: reported after the value
  int depth = 0;

  void ws() {
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  bool fail() {
    syntax_err = true;
    return false;
  }
  char peek() {
    ws();
    return p < end ? *p : '\0';
  }
  bool eat(char c) {
    ws();
    if (p < end && *p == c) {
      ++p;
      return true;
    }
    return false;
  }

  // A string token at p (after ws).  out: the unescaped value (Go's unquote), or null to
  // validate only.  *raw_begin / *raw_end: the bytes between the quotes.
  bool string(std::string* out, const char** raw_begin = nullptr, const char** raw_end = nullptr) {
    ws();
    if (p >= end || *p != '"') return fail();
    ++p;
    if (raw_begin) *raw_begin = p;
    if (out) out->clear();
    const char* run = p;  // pending bytes copied verbatim
    auto flush = [&](const char* upto) {
      if (out && upto > run) out->append(run, (size_t)(upto - run));
    };
    while (true) {
      p = scan_plain(p, end);  // fast path: plain ASCII bytes
      if (p >= end) return fail();
      const unsigned char c = (unsigned char)*p;
      if (c == '"') {
        flush(p);
        if (raw_end) *raw_end = p;
        ++p;
        return true;
      }
      if (c < 0x20) return fail();
      if (c == '\\') {
        flush(p);
        if (p + 1 >= end) return fail();
        const char e = p[1];
        p += 2;
        char simple = 0;
        switch (e) {
          case '"': simple = '"'; break;
          case '\\': simple = '\\'; break;
          case '/': simple = '/'; break;
          case 'b': simple = '\b'; break;
          case 'f': simple = '\f'; break;
          case 'n': simple = '\n'; break;
          case 'r': simple = '\r'; break;
          case 't': simple = '\t'; break;
          case 'u': break;
          default: return fail();
        }
        if (simple) {
          if (out) out->push_back(simple);
        } else {
          auto hex4 = [&](const char* q, uint32_t* v) {
            if (end - q < 4) return false;
            uint32_t r = 0;
            for (int i = 0; i < 4; ++i) {
              const int h = hexval(q[i]);
              if (h < 0) return false;
              r = r << 4 | (uint32_t)h;
            }
            *v = r;
            return true;
          };
          uint32_t r;
          if (!hex4(p, &r)) return fail();
          p += 4;
          if (r >= 0xD800 && r < 0xE000) {
            // utf16.DecodeRune with a following \uXXXX; else U+FFFD (the next escape, if any,
            // is decoded on its own)
            uint32_t r2;
            if (r < 0xDC00 && end - p >= 6 && p[0] == '\\' && p[1] == 'u' && hex4(p + 2, &r2) &&
                r2 >= 0xDC00 && r2 < 0xE000) {
              r = 0x10000 + ((r - 0xD800) << 10) + (r2 - 0xDC00);
              p += 6;
            } else {
              r = 0xFFFD;
            }
          }
          if (out) put_utf8(out, r);
        }
        run = p;
        continue;
      }
      // c >= 0x80: a valid sequence is kept, an invalid byte becomes U+FFFD
      const int n = utf8_valid(reinterpret_cast<const unsigned char*>(p),
                               reinterpret_cast<const unsigned char*>(end));
      if (n) {
        p += n;
      } else {
        flush(p);
        if (out) put_utf8(out, 0xFFFD);
        ++p;
        run = p;
      }
    }
  }

  bool number() {
    ws();
    const char* s = p;
    if (p < end && *p == '-') ++p;
    if (p >= end) return fail();
    if (*p == '0') {
      ++p;
    } else if (*p >= '1' && *p <= '9') {
      while (p < end && *p >= '0' && *p <= '9') ++p;
    } else {
      return fail();
    }
    if (p < end && *p == '.') {
      ++p;
      if (p >= end || *p < '0' || *p > '9') return fail();
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    if (p < end && (*p == 'e' || *p == 'E')) {
      ++p;
      if (p < end && (*p == '+' || *p == '-')) ++p;
      if (p >= end || *p < '0' || *p > '9') return fail();
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    return p > s;
  }

  bool literal(const char* lit) {
    ws();
    const size_t n = std::strlen(lit);
    if ((size_t)(end - p) < n || std::memcmp(p, lit, n) != 0) return fail();
    p += n;
    return true;
  }

  bool enter() {
    if (++depth > kMaxDepth) return fail();
    return true;
  }

  // Any value, syntax-checked and skipped.
  bool skip() {
    const char c = peek();
    switch (c) {
      case '"': return string(nullptr);
      case '{': {
        if (!enter()) return false;
        ++p;
        if (eat('}')) { --depth; return true; }
        do {
          if (!string(nullptr) || !eat(':') || !skip()) return fail();
        } while (eat(','));
        if (!eat('}')) return fail();
        --depth;
        return true;
      }
      case '[': {
        if (!enter()) return false;
        ++p;
        if (eat(']')) { --depth; return true; }
        do {
          if (!skip()) return fail();
        } while (eat(','));
        if (!eat(']')) return fail();
        --depth;
        return true;
      }
      case 't': return literal("true");
      case 'f': return literal("false");
      case 'n': return literal("null");
      default: return number();
    }
  }

  // An object key: a view of the raw bytes when they need no unescaping, else of scratch.
  bool key(std::string_view* out, std::string* scratch) {
    ws();
    if (p >= end || *p != '"') return fail();
    const char* b = p + 1;
    const char* q = scan_plain(b, end);
    if (q < end && *q == '"') {
      *out = std::string_view(b, (size_t)(q - b));
      p = q + 1;
      return true;
    }
    if (!string(scratch)) return false;
    *out = std::string_view(*scratch);
    return true;
  }

  // Iterate an object's members: f(key) is called with p at the value and must consume it.
  template <typename F>
  bool object(F&& f) {
    if (!enter()) return false;
    if (!eat('{')) return fail();
    if (eat('}')) { --depth; return true; }
    std::string scratch;
    std::string_view k;
    do {
      if (!key(&k, &scratch) || !eat(':')) return fail();
      if (!f(k)) return false;
    } while (eat(','));
    if (!eat('}')) return fail();
    --depth;
    return true;
  }

  template <typename F>
  bool array(F&& f) {
    if (!enter()) return false;
    if (!eat('[')) return fail();
    if (eat(']')) { --depth; return true; }
    int64_t i = 0;
    do {
      if (!f(i++)) return false;
    } while (eat(','));
    if (!eat(']')) return fail();
    --depth;
    return true;
  }

  // A value of the wrong JSON type for the field: skip it, remember the type error.
  bool mismatch() {
    type_err = true;
    return skip();
  }

  // null?  (consumed)
  bool null_value() {
    if (peek() == 'n') return literal("null");
    return false;
  }
};

// A string field: null leaves *v unchanged; other non-strings are type errors.
bool string_field(Scanner& s, std::string* v) {
  const char c = s.peek();
  if (c == 'n') return s.literal("null");
  if (c != '"') return s.mismatch();
  return s.string(v);
}

// A map[string]string field (ObjectMeta labels / annotations): null is a nil map, every
// value must be a string or null (json.Unmarshal fails on any other value, whichever key it
// sits under).  on_entry(key, value) sees each string entry in order.
template <class F>
bool string_map(Scanner& s, F&& on_entry) {
  const char c = s.peek();
  if (c == 'n') return s.literal("null");
  if (c != '{') return s.mismatch();
  return s.object([&](std::string_view k) {
    std::string v;  // a fresh element: null stores ""
    if (!string_field(s, &v)) return false;
    on_entry(k, v);
    return true;
  });
}

// ---------------------------------------------------------------------------- typed skip
//
// Every value inside the Pod and the nodes is checked against the Go type json.Unmarshal
// decodes it into (k8s_schema.h), so a request the reference fails with an
// UnmarshalTypeError (or a Quantity / Time / IntOrString UnmarshalJSON error) fails here too.

std::string trim_space(const std::string& v);  // strings.TrimSpace, below

// strconv.ParseInt(tok, 10, 64) succeeds and the value fits `bits` (reflect OverflowInt):
// JSON number tokens with a fraction or an exponent fail ParseInt.
bool go_int_ok(const char* b, const char* e, int bits) {
  bool neg = false;
  if (b < e && *b == '-') {
    neg = true;
    ++b;
  }
  if (b == e) return false;
  const uint64_t limit = (bits == 32 ? (1ull << 31) : (1ull << 63)) - (neg ? 0 : 1);
  uint64_t v = 0;
  for (; b < e; ++b) {
    if (*b < '0' || *b > '9') return false;
    const uint64_t d = (uint64_t)(*b - '0');
    if (v > (limit - d) / 10) return false;
    v = v * 10 + d;
  }
  return true;
}

// Resource.Quantity.UnmarshalJSON on a value's literal bytes (apimachinery v0.22.2
// quantity.go): null handled by the caller; one pair of surrounding quotes removed, spaces
// trimmed, then ParseQuantity.
// The common forms first: [sign] digits + a suffix of the suffixer's tables, no fraction or
// exponent, and no byte that trimming could remove (such a string always parses:
// parseQuantityString accepts it and the digits make the inf.Dec path's SetString succeed);
// everything else goes through the full ParseQuantity restatement.
bool quantity_simple(std::string_view q) {
  size_t i = 0;
  if (i < q.size() && (q[i] == '-' || q[i] == '+')) ++i;
  const size_t d0 = i;
  while (i < q.size() && q[i] >= '0' && q[i] <= '9') ++i;
  if (i == d0) return false;
  const std::string_view suf = q.substr(i);
  static const char* const kSuffixes[] = {"",   "n",  "u",  "m",  "k",  "M",  "G",  "T",
                                          "P",  "E",  "Ki", "Mi", "Gi", "Ti", "Pi", "Ei"};
  for (const char* x : kSuffixes)
    if (suf == x) return true;
  return false;
}

bool quantity_literal_ok(const char* b, const char* e) {
  std::string_view lit(b, (size_t)(e - b));
  if (lit.size() >= 2 && lit.front() == '"' && lit.back() == '"') lit = lit.substr(1, lit.size() - 2);
  if (quantity_simple(lit)) return true;
  const std::string q = trim_space(std::string(lit));
  int64_t v;
  return q.find('\0') == std::string::npos && pas_quantity_as_int64(q.c_str(), &v) == PAS_OK;
}

// time.Parse(time.RFC3339, v) of Go 1.16 (format.go), accept / reject only.  Layout chunks:
// "2006" (4 bytes, the first a digit, atoi), "-", "01" (2 digits, 1..12), "-", "02"
// (2 digits), "T", "15" (1 or 2 digits, < 24), ":", "04" (2 digits, < 60), ":", "05"
// (2 digits, < 60, then an optional '.' + digits: parseNanoseconds, < 1e9), "Z07:00" ('Z',
// or sign + atoi(2) + ':' + atoi(2), no range check), nothing after; the day must exist in
// the month (daysIn, leap years).
bool time_atoi(std::string_view s, int64_t* out) {  // the time package's atoi / leadingInt
  bool neg = false;
  if (!s.empty() && (s[0] == '-' || s[0] == '+')) {
    neg = s[0] == '-';
    s.remove_prefix(1);
  }
  uint64_t x = 0;
  size_t i = 0;
  for (; i < s.size() && s[i] >= '0' && s[i] <= '9'; ++i) {
    if (x > (1ull << 63) / 10) return false;
    x = x * 10 + (uint64_t)(s[i] - '0');
    if (x > (1ull << 63)) return false;
  }
  if (i != s.size()) return false;
  const int64_t v = (int64_t)x;  // int(q): 2^63 wraps negative, as in Go
  *out = neg ? -v : v;
  return true;
}

bool rfc3339_ok(std::string_view v) {
  auto digit = [&](size_t i) { return i < v.size() && v[i] >= '0' && v[i] <= '9'; };
  auto getnum = [&](bool fixed, int* out) {
    if (!digit(0)) return false;
    if (!digit(1)) {
      if (fixed) return false;
      *out = v[0] - '0';
      v.remove_prefix(1);
      return true;
    }
    *out = (v[0] - '0') * 10 + (v[1] - '0');
    v.remove_prefix(2);
    return true;
  };
  auto lit = [&](char c) {
    if (v.empty() || v[0] != c) return false;
    v.remove_prefix(1);
    return true;
  };
  if (v.size() < 4 || !digit(0)) return false;
  int64_t year;
  if (!time_atoi(v.substr(0, 4), &year)) return false;
  v.remove_prefix(4);
  int month, day, hour, minute, sec;
  if (!lit('-') || !getnum(true, &month) || month < 1 || month > 12) return false;
  if (!lit('-') || !getnum(true, &day)) return false;
  if (!lit('T') || !getnum(false, &hour) || hour >= 24) return false;
  if (!lit(':') || !getnum(true, &minute) || minute >= 60) return false;
  if (!lit(':') || !getnum(true, &sec) || sec >= 60) return false;
  if (v.size() >= 2 && v[0] == '.' && digit(1)) {  // fractional seconds the layout lacks
    size_t n = 2;
    while (digit(n)) ++n;
    int64_t ns;
    if (!time_atoi(v.substr(1, n - 1), &ns) || ns < 0 || ns >= 1000000000) return false;
    v.remove_prefix(n);
  }
  if (!v.empty() && v[0] == 'Z') {
    v.remove_prefix(1);
  } else {
    if (v.size() < 6 || v[3] != ':') return false;
    int64_t hh, mm;
    if (!time_atoi(v.substr(1, 2), &hh) || !time_atoi(v.substr(4, 2), &mm)) return false;
    if (v[0] != '+' && v[0] != '-') return false;
    v.remove_prefix(6);
  }
  if (!v.empty()) return false;  // extra text
  static const int kDays[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  const bool leap = year % 4 == 0 && (year % 100 != 0 || year % 400 == 0);
  const int dim = kDays[month - 1] + (month == 2 && leap ? 1 : 0);
  return day >= 1 && day <= dim;
}

// The struct field a key decodes into: an exact name match, else the first field (declaration
// order) whose fold function matches (encoding/json object(): nameIndex, then equalFold).
const pas_schema::GoField* go_field(const pas_schema::GoType* t, std::string_view key) {
  for (int32_t i = 0; i < t->n_fields; ++i) {
    const pas_schema::GoField& f = t->fields[i];
    if ((size_t)f.len == key.size() && f.name[0] == key[0] &&
        std::memcmp(f.name, key.data(), key.size()) == 0)
      return &f;
  }
  for (int32_t i = 0; i < t->n_fields; ++i)
    if (fold_match(t->fields[i].name, key)) return &t->fields[i];
  return nullptr;
}

bool check_value(Scanner& s, const pas_schema::GoType* t);

// A struct value; hook(field) returns -1 to check the field's value by its type, else it has
// consumed the value (1: ok, 0: failed).  Unknown keys are skipped (no DisallowUnknownFields).
template <class Hook>
bool check_struct(Scanner& s, const pas_schema::GoType* t, Hook&& hook) {
  const char c = s.peek();
  if (c == 'n') return s.literal("null");
  if (c != '{') return s.mismatch();
  return s.object([&](std::string_view k) {
    const pas_schema::GoField* f = go_field(t, k);
    if (!f) return s.skip();
    const int r = hook(f);
    if (r >= 0) return r != 0;
    return check_value(s, f->type);
  });
}

bool check_value(Scanner& s, const pas_schema::GoType* t) {
  using pas_schema::GoKind;
  const char c = s.peek();
  if (c == 'n') return s.literal("null");  // accepted by every kind
  switch (t->kind) {
    case GoKind::kString:
      if (c != '"') return s.mismatch();
      return s.string(nullptr);
    case GoKind::kBool:
      if (c == 't') return s.literal("true");
      if (c == 'f') return s.literal("false");
      return s.mismatch();
    case GoKind::kIntOrString:
      if (c == '"') return s.string(nullptr);  // intstr.UnmarshalJSON: StrVal
      [[fallthrough]];                         // else IntVal (int32)
    case GoKind::kInt32:
    case GoKind::kInt64: {
      if (c != '-' && (c < '0' || c > '9')) return s.mismatch();
      const char* b = s.p;
      if (!s.number()) return false;
      if (!go_int_ok(b, s.p, t->kind == GoKind::kInt64 ? 64 : 32)) s.type_err = true;
      return true;
    }
    case GoKind::kQuantity: {
      const char* b = s.p;
      if (!s.skip()) return false;
      if (!quantity_literal_ok(b, s.p)) s.type_err = true;
      return true;
    }
    case GoKind::kTime: {
      if (c != '"') return s.mismatch();  // json.Unmarshal(b, &str)
      std::string v;
      if (!s.string(&v)) return false;
      if (!rfc3339_ok(v)) s.type_err = true;
      return true;
    }
    case GoKind::kRaw:
      return s.skip();
    case GoKind::kMap:
      if (c != '{') return s.mismatch();
      return s.object([&](std::string_view) { return check_value(s, t->elem); });
    case GoKind::kSlice:
      if (c != '[') return s.mismatch();
      return s.array([&](int64_t) { return check_value(s, t->elem); });
    case GoKind::kStruct:
      return check_struct(s, t, [](const pas_schema::GoField*) { return -1; });
  }
  return s.skip();
}

// The whole v1.Pod value type-checked (the pod entry points decode a pod on its own; the Args
// decode checks it in place).
bool pod_typed_ok(const char* pod, int64_t len) {
  Scanner s{pod, pod + len};
  return check_value(s, &pas_schema::Pod) && !s.syntax_err && !s.type_err;
}

}  // namespace

// ---------------------------------------------------------------------------- name table

struct pas_name_table {
  std::vector<std::string> names;
  std::vector<int32_t> slots;  // open addressing, -1 empty
  uint64_t mask = 0;

  static uint64_t hash(std::string_view s) {  // FNV-1a, 64-bit
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
    return h ^ (h >> 29);
  }
  int32_t find(std::string_view s) const {
    if (slots.empty()) return -1;
    for (uint64_t i = hash(s) & mask;; i = (i + 1) & mask) {
      const int32_t id = slots[i];
      if (id < 0) return -1;
      if (names[(size_t)id] == s) return id;
    }
  }
};

namespace {

// The request node list being decoded.  A slice decodes element-wise into what it already
// holds (encoding/json array(): elements past the old length start from zero), so a repeated
// key keeps earlier values where the new element leaves them unset.
struct NodeList {
  std::vector<std::string> names;
  std::vector<int64_t> spans;  // [2 * i]: offset, length of item i's latest decode
};

// v1.Node: metadata.name is read (*name keeps its value on null / absence); every other
// field is type-checked (k8s_schema.h).
bool decode_node(Scanner& s, std::string* name) {
  using namespace pas_schema;
  return check_struct(s, &Node, [&](const GoField* f) -> int {
    if (f->type != &ObjectMeta) return -1;
    return check_struct(s, &ObjectMeta, [&](const GoField* mf) -> int {
      if (mf != &ObjectMeta_fields[0]) return -1;  // "name"
      return string_field(s, name) ? 1 : 0;
    }) ? 1 : 0;
  });
}

struct ItemIndex;
bool fast_items(ItemIndex* idx, Scanner& s, NodeList* out);
void item_list_changed(ItemIndex* idx);

// v1.NodeList: items (null sets the slice to nil).  idx (optional): the body's structural
// index; the first decode of a NodeList's items array goes through it in parallel.
bool decode_node_list(Scanner& s, NodeList* out, const char* base, ItemIndex* idx) {
  return s.object([&](std::string_view k) {
    if (fold_match("items", k)) {
      const char c = s.peek();
      if (idx) item_list_changed(idx);
      if (c == 'n') {
        out->names.clear();
        out->spans.clear();
        return s.literal("null");
      }
      if (c != '[') return s.mismatch();
      if (idx && out->names.empty() && fast_items(idx, s, out)) return true;
      size_t n = 0;
      const bool ok = s.array([&](int64_t i) {
        if ((size_t)i >= out->names.size()) {
          out->names.emplace_back();
          out->spans.resize(out->names.size() * 2);
        }
        n = (size_t)i + 1;
        s.ws();
        const char* b = s.p;
        if (!decode_node(s, &out->names[(size_t)i])) return false;
        out->spans[2 * (size_t)i] = (int64_t)(b - base);
        out->spans[2 * (size_t)i + 1] = (int64_t)(s.p - b);
        return true;
      });
      out->names.resize(n);
      out->spans.resize(2 * n);
      return ok;
    }
    if (fold_match("metadata", k)) return check_value(s, &pas_schema::ListMeta);
    if (fold_match("kind", k) || fold_match("apiVersion", k)) {
      std::string ignored;
      return string_field(s, &ignored);
    }
    return s.skip();
  });
}

// ---------------------------------------------------------------------------- parallel items
//
// A 100k-node NodeList body is ~90 MB, nearly all of it the items array.  For a large body
// the decode splits it over host threads without changing what is decoded:
//   1. Structural index, per 64-byte block (SSE2 masks of quotes, backslashes, brackets,
//      commas), per chunk of the body in parallel: a chunk's unescaped-quote parity and its
//      bracket depth change for both possible in-string states at its start (the escape
//      state at its start is the parity of the backslash run before it); a prefix over the
//      chunks gives each chunk's in-string state and depth; a second parallel pass records
//      the commas at depth 3 and the closings of depth-3 containers.
//   2. The sequential decode runs as before until it reaches an items array at depth 2 (the
//      Args object, then the NodeList).  Its end is the first depth-3 closing after it; the
//      depth-3 commas between are the item boundaries.
//   3. The items are decoded in parallel, each by the same decode_node on its own byte range
//      (a Scanner at depth 3), which must consume the range exactly (value + whitespace).
// Every byte outside the items array is decoded sequentially and every byte inside belongs
// to exactly one item range, so a body accepted this way is valid JSON of the same shape and
// decodes to the same values.  Anything else (an item failing, a repeated items key, no
// closing found) returns to the sequential decode of that array, which then reports exactly
// what the sequential path reports.
constexpr int64_t kParBytesPerThread = 1 << 20;
constexpr int kParMaxThreads = 16;  // the GPU box's CPU share per GPU
constexpr int kPieces = pas::kHostPieces;
std::atomic<int32_t> g_decode_threads{0};  // pas_decode_set_threads; 0 = automatic

int decode_threads_for(int64_t len) {
  const int32_t set = g_decode_threads.load(std::memory_order_relaxed);
  const int hw = std::max(1, (int)std::thread::hardware_concurrency());
  const int64_t t = std::min<int64_t>(set > 0 ? set : std::min(hw, kParMaxThreads),
                                      len / kParBytesPerThread);
  return (int)std::max<int64_t>(1, t);
}

// Worker threads kept across calls (a decode runs four parallel steps; starting 15 threads
// per step cost ~0.3 ms each on the GPU box).  One parallel step at a time uses the pool; a
// concurrent call (another goroutine's request) starts threads of its own instead.  After a
// fork the child gets a new pool (the parent's workers do not exist there).
class WorkerPool {
 public:
  static WorkerPool* get() {
    static std::mutex mk;
    static WorkerPool* pool = nullptr;
    std::lock_guard<std::mutex> g(mk);
    if (!pool || pool->pid_ != getpid()) pool = new WorkerPool();  // (never freed: process-wide)
    return pool;
  }
  // Runs f(i) for i in [0, n) on the caller and up to threads - 1 workers (each taking the next
  // i until none is left); false if the pool is busy or cannot grow (nothing run).
  bool run(int n, int threads, const std::function<void(int)>& f) {
    std::unique_lock<std::mutex> busy(busy_, std::try_to_lock);
    if (!busy.owns_lock()) return false;
    threads = std::min(n, threads);
    try {
      while ((int)workers_.size() < threads - 1) workers_.emplace_back([this] { loop(); });
    } catch (...) {
      return false;
    }
    uint32_t ep;
    {
      std::lock_guard<std::mutex> g(m_);
      task_ = &f;
      n_ = n;
      pending_ = n;
      seats_ = threads - 1;  // workers that may join this run
      ep = (uint32_t)++epoch_;
      next_.store((uint64_t)ep << 32);
    }
    cv_.notify_all();
    work(&f, n, ep);
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return pending_ == 0; });
    task_ = nullptr;
    return true;
  }

 private:
  WorkerPool() : pid_(getpid()) {}
  // Items of run `ep` only: next_ holds {epoch, next item}, so a worker still leaving an
  // earlier run (its last item done, the caller already returned and started a new run) takes
  // nothing from the new one; task and n are the copies the worker read under m_.
  void work(const std::function<void(int)>* task, int n, uint32_t ep) {
    for (;;) {
      uint64_t v = next_.load();
      int i;
      do {
        if ((uint32_t)(v >> 32) != ep) return;
        i = (int)(uint32_t)v;
        if (i >= n) return;
      } while (!next_.compare_exchange_weak(v, v + 1));
      (*task)(i);
      std::lock_guard<std::mutex> g(m_);
      if (--pending_ == 0) done_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* task;
      int n;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return epoch_ != seen && task_ != nullptr; });
        seen = epoch_;
        if (seats_ <= 0) continue;  // the run has its threads: wait for the next one
        --seats_;
        task = task_;
        n = n_;
      }
      work(task, n, (uint32_t)seen);
    }
  }
  const pid_t pid_;
  std::mutex busy_, m_;
  std::condition_variable cv_, done_;
  std::vector<std::thread> workers_;
  const std::function<void(int)>* task_ = nullptr;
  int n_ = 0, pending_ = 0, seats_ = 0;
  std::atomic<uint64_t> next_{0};  // {epoch (32 bits), next item (32 bits)}
  uint64_t epoch_ = 0;
};

// f(i) for i in [0, n) on up to `threads` threads (default n), each taking the next i until
// none is left: the pool, or fresh threads when it is busy.  More pieces than threads balance
// threads the host delays.  Returns false (nothing run) when no thread can be started.
template <class F>
bool parallel_for(int n, F&& f, int threads = 0) {
  if (threads <= 0 || threads > n) threads = n;
#ifdef PAS_DECODE_TRACE
  std::vector<double> busy((size_t)n, 0.0);
  PAS_TRACE_T0(t_spawn);
  auto g = [&](int i) {
    PAS_TRACE_T0(t_run);
    f(i);
    busy[(size_t)i] =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_run).count();
  };
#else
  auto& g = f;
#endif
  const std::function<void(int)> fn = [&g](int i) { g(i); };
  bool ran = n <= 1 ? (n == 1 ? g(0) : void(), true) : WorkerPool::get()->run(n, threads, fn);
  if (!ran) {
    std::atomic<int> next{0};
    auto take = [&] {
      for (int i; (i = next.fetch_add(1)) < n;) g(i);
    };
    std::vector<std::thread> th;
    try {
      th.reserve((size_t)std::max(threads - 1, 0));
      for (int i = 1; i < threads; ++i) th.emplace_back(take);
    } catch (...) {
      next.store(n);  // the started threads take nothing more
      for (auto& x : th) x.join();
      return false;
    }
    take();
    for (auto& x : th) x.join();
  }
#ifdef PAS_DECODE_TRACE
  PAS_TRACE_MS("parallel step", t_spawn);
  std::fprintf(stderr, "decode busy max %.3f min %.3f ms (n=%d)\n",
               *std::max_element(busy.begin(), busy.end()),
               *std::min_element(busy.begin(), busy.end()), n);
#endif
  return true;
}

}  // namespace

int pas::host_threads_for(int64_t bytes) { return decode_threads_for(bytes); }

bool pas::host_parallel(int n, const std::function<void(int)>& f, int threads) {
  return parallel_for(n, f, threads);
}

namespace {

struct Masks {
  uint64_t quote, bs, open, close, comma;
};

// 64 bytes at p: '"', '\\', '{' or '[' (c | 0x20 == '{'), '}' or ']', ','.
inline Masks classify64(const char* p) {
  Masks m{0, 0, 0, 0, 0};
  const __m128i q = _mm_set1_epi8('"'), b = _mm_set1_epi8('\\'), o = _mm_set1_epi8('{');
  const __m128i c = _mm_set1_epi8('}'), k = _mm_set1_epi8(','), lc = _mm_set1_epi8(0x20);
  for (int i = 0; i < 4; ++i) {
    const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 16 * i));
    const __m128i vl = _mm_or_si128(v, lc);
    const int sh = 16 * i;
    m.quote |= (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(v, q)) << sh;
    m.bs |= (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(v, b)) << sh;
    m.open |= (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(vl, o)) << sh;
    m.close |= (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(vl, c)) << sh;
    m.comma |= (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(v, k)) << sh;
  }
  return m;
}

// Bytes of the block escaped by a backslash (carry: the block's first byte is).
inline uint64_t escaped_mask(uint64_t bs, bool* carry) {
  if (!bs) {
    const uint64_t e = *carry ? 1ull : 0ull;
    *carry = false;
    return e;
  }
  uint64_t e = 0;
  bool esc = *carry;
  for (int i = 0; i < 64; ++i) {
    if (esc) {
      e |= 1ull << i;
      esc = false;
    } else if ((bs >> i) & 1ull) {
      esc = true;
    }
  }
  *carry = esc;
  return e;
}

inline uint64_t prefix_xor(uint64_t x) {
  x ^= x << 1;
  x ^= x << 2;
  x ^= x << 4;
  x ^= x << 8;
  x ^= x << 16;
  x ^= x << 32;
  return x;
}

struct ItemIndex {
  const char* body = nullptr;
  int64_t len = 0;
  int threads = 1;
  bool built = false;
  std::vector<int64_t> events;  // pos * 2 + 1: closing of a depth-3 container; pos * 2: comma
  // the items' snapshot ids, looked up by the threads that decoded them (table set): valid
  // while no later key changed the list (ids_mods == mods)
  const pas_name_table* table = nullptr;
  std::vector<int32_t> ids;
  uint64_t mods = 0, ids_mods = ~0ull;

  // Walks the 64-byte blocks of [b, e) (the last one padded with spaces): f(block start,
  // masks, escaped bytes), the escape state carried from the backslash run before b.
  template <class F>
  void blocks(int64_t b, int64_t e, F&& f) const {
    int64_t r = b;
    while (r > 0 && body[r - 1] == '\\') --r;
    bool carry = ((b - r) & 1) != 0;
    char pad[64];
    for (int64_t x = b; x < e; x += 64) {
      const char* p = body + x;
      if (e - x < 64) {
        std::memset(pad, ' ', sizeof pad);
        std::memcpy(pad, p, (size_t)(e - x));
        p = pad;
      }
      const Masks m = classify64(p);
      f(x, p, m, escaped_mask(m.bs, &carry));
    }
  }

  void build() {
    // kPieces chunks per thread, taken in turn by the threads (balances a delayed thread)
    const int T = threads * kPieces;
    const int64_t cs = ((len + T - 1) / T + 63) & ~int64_t(63);
    std::vector<int64_t> par(T, 0), d_out(T, 0), d_in(T, 0);
    // pass 1: quote parity and depth change per chunk, for both start states
    if (!parallel_for(T, [&](int t) {
          const int64_t b = std::min(len, t * cs), e = std::min(len, b + cs);
          uint64_t instr = 0, pq = 0;
          int64_t dout = 0, din = 0;
          blocks(b, e, [&](int64_t, const char*, const Masks& m, uint64_t esc) {
            const uint64_t qu = m.quote & ~esc;
            const uint64_t mask = prefix_xor(qu) ^ instr;  // 1: inside (start outside)
            instr = (mask >> 63) ? ~0ull : 0ull;
            pq ^= (uint64_t)__builtin_popcountll(qu) & 1ull;
            dout += __builtin_popcountll(m.open & ~mask) - __builtin_popcountll(m.close & ~mask);
            din += __builtin_popcountll(m.open & mask) - __builtin_popcountll(m.close & mask);
          });
          par[t] = (int64_t)pq;
          d_out[t] = dout;
          d_in[t] = din;
        }, threads))
      return;
    std::vector<char> in0(T, 0);
    std::vector<int64_t> depth0(T, 0);
    for (int t = 1; t < T; ++t) {
      in0[t] = (char)(in0[t - 1] ^ (par[t - 1] & 1));
      depth0[t] = depth0[t - 1] + (in0[t - 1] ? d_in[t - 1] : d_out[t - 1]);
    }
    // pass 2: depth-3 commas and closings, in body order
    std::vector<std::vector<int64_t>> ev(T);
    if (!parallel_for(T, [&](int t) {
          const int64_t b = std::min(len, t * cs), e = std::min(len, b + cs);
          uint64_t instr = in0[t] ? ~0ull : 0ull;
          int64_t depth = depth0[t];
          std::vector<int64_t>& out = ev[t];
          blocks(b, e, [&](int64_t x, const char*, const Masks& m, uint64_t esc) {
            const uint64_t mask = prefix_xor(m.quote & ~esc) ^ instr;
            instr = (mask >> 63) ? ~0ull : 0ull;
            const uint64_t op = m.open & ~mask, cl = m.close & ~mask;
            const int no = __builtin_popcountll(op), nc = __builtin_popcountll(cl);
            // the depth stays within [depth - nc, depth + no] in this block: most blocks lie
            // inside an item (depth >= 4) and hold no depth-3 comma or closing
            if (depth - nc <= 3 && depth + no >= 3) {
              uint64_t ev = (cl | m.comma) & ~mask;
              while (ev) {
                const int i = __builtin_ctzll(ev);
                const uint64_t bit = 1ull << i, below = bit - 1;
                ev &= ev - 1;
                // depth just before byte i
                if (depth + __builtin_popcountll(op & below) - __builtin_popcountll(cl & below) == 3)
                  out.push_back((x + i) * 2 + ((cl & bit) ? 1 : 0));
              }
            }
            depth += no - nc;
          });
        }, threads))
      return;
    size_t total = 0;
    for (const auto& v : ev) total += v.size();
    events.reserve(total);
    for (const auto& v : ev) events.insert(events.end(), v.begin(), v.end());
    built = true;
  }
};

void item_list_changed(ItemIndex* idx) { ++idx->mods; }

// The items array at s.p ('[' of the first items key of a NodeList at depth 2) decoded in
// parallel; false (s untouched) to decode it sequentially instead.
bool fast_items(ItemIndex* idx, Scanner& s, NodeList* out) {
  if (!idx->built || s.depth != 2) return false;
  const int64_t p0 = s.p - idx->body;
  const std::vector<int64_t>& ev = idx->events;
  auto it = std::lower_bound(ev.begin(), ev.end(), p0 * 2 + 2);
  std::vector<int64_t> cut{p0};  // '[' , the commas, ']'
  for (; it != ev.end() && !(*it & 1); ++it) cut.push_back(*it >> 1);
  if (it == ev.end()) return false;
  cut.push_back(*it >> 1);
  const size_t n_items = cut.size() - 1;
  std::vector<std::string> names(n_items);
  std::vector<int64_t> spans(2 * n_items);
  std::vector<int32_t> ids(idx->table ? n_items : 0);
  std::atomic<bool> ok{true};
  bool empty = false;
  if (n_items == 1) {  // "[]" (whitespace only) or one item
    Scanner w{idx->body + cut[0] + 1, idx->body + cut[1]};
    w.ws();
    empty = w.p == w.end;
  }
#ifdef PAS_DECODE_ITEMS_T1  // diagnostic: the items on one thread
  const int T = 1;
#else
  const int T = std::max(1, std::min<int>(idx->threads * kPieces, (int)(n_items / 256)));
#endif
  PAS_TRACE_T0(t_items);
  if (!empty &&
      !parallel_for(T, [&](int t) {
        const size_t lo = n_items * (size_t)t / (size_t)T, hi = n_items * (size_t)(t + 1) / (size_t)T;
        for (size_t i = lo; i < hi && ok.load(std::memory_order_relaxed); ++i) {
          Scanner w{idx->body + cut[i] + 1, idx->body + cut[i + 1]};
          w.depth = 3;
          w.ws();
          const char* b = w.p;
          const bool good = decode_node(w, &names[i]);
          const char* e = w.p;
          w.ws();
          if (!good || w.syntax_err || w.type_err || w.p != w.end || e == b) {
            ok.store(false, std::memory_order_relaxed);
            return;
          }
          spans[2 * i] = (int64_t)(b - idx->body);
          spans[2 * i + 1] = (int64_t)(e - b);
          if (idx->table) ids[i] = idx->table->find(names[i]);
        }
      }, idx->threads))
    return false;
  PAS_TRACE_MS("items", t_items);
  if (!ok.load()) return false;
  if (empty) {
    names.clear();
    spans.clear();
  }
  out->names = std::move(names);
  out->spans = std::move(spans);
  if (idx->table) {
    if (empty) ids.clear();
    idx->ids = std::move(ids);
    idx->ids_mods = idx->mods;
  }
  s.p = idx->body + cut.back() + 1;
  return true;
}

// strings.TrimSpace: ASCII spaces and the Unicode White_Space code points.
std::string trim_space(const std::string& v) {
  auto space_at = [&](size_t i, bool back) -> size_t {  // byte length of a space at i, or 0
    static const char* const kSpaces[] = {" ", "\t", "\n", "\v", "\f", "\r",
                                          "\xc2\x85", "\xc2\xa0", "\xe1\x9a\x80",
                                          "\xe2\x80\x80", "\xe2\x80\x81", "\xe2\x80\x82",
                                          "\xe2\x80\x83", "\xe2\x80\x84", "\xe2\x80\x85",
                                          "\xe2\x80\x86", "\xe2\x80\x87", "\xe2\x80\x88",
                                          "\xe2\x80\x89", "\xe2\x80\x8a", "\xe2\x80\xa8",
                                          "\xe2\x80\xa9", "\xe2\x80\xaf", "\xe2\x81\x9f",
                                          "\xe3\x80\x80"};
    for (const char* sp : kSpaces) {
      const size_t n = std::strlen(sp);
      if (back) {
        if (i >= n && v.compare(i - n, n, sp) == 0) return n;
      } else if (v.compare(i, n, sp) == 0) {
        return n;
      }
    }
    return 0;
  };
  size_t b = 0, e = v.size();
  for (size_t n; b < e && (n = space_at(b, false));) b += n;
  for (size_t n; e > b && (n = space_at(e, true));) e -= n;
  return v.substr(b, e - b);
}

}  // namespace

extern "C" {

int pas_name_table_create(int32_t n_names, const char* const* names, pas_name_table** out) {
  if (!out || n_names < 0 || (n_names > 0 && !names)) return PAS_EINVAL;
  *out = nullptr;
  for (int32_t i = 0; i < n_names; ++i)
    if (!names[i]) return PAS_EINVAL;
  pas_name_table* t = new (std::nothrow) pas_name_table;
  if (!t) return PAS_ENOMEM;
  try {
    t->names.reserve((size_t)n_names);
    for (int32_t i = 0; i < n_names; ++i) t->names.emplace_back(names[i]);
    uint64_t cap = 16;
    while (cap < (uint64_t)n_names * 2) cap <<= 1;
    t->slots.assign(cap, -1);
    t->mask = cap - 1;
    for (int32_t i = 0; i < n_names; ++i) {
      const std::string& s = t->names[(size_t)i];
      for (uint64_t h = pas_name_table::hash(s) & t->mask;; h = (h + 1) & t->mask) {
        const int32_t id = t->slots[h];
        if (id < 0) {
          t->slots[h] = i;
          break;
        }
        if (t->names[(size_t)id] == s) break;  // a repeated name keeps its first id
      }
    }
  } catch (...) {
    delete t;
    return PAS_ENOMEM;
  }
  *out = t;
  return PAS_OK;
}

void pas_name_table_destroy(pas_name_table* t) { delete t; }

int32_t pas_name_table_lookup(const pas_name_table* t, const char* name, int64_t len) {
  if (!t || !name || len < 0) return -1;
  return t->find(std::string_view(name, (size_t)len));
}

}  // extern "C"

namespace {

// Decode of extender.Args shared by pas_decode_args / pas_decode_request_names: the chosen
// list's names (unescaped, request order), the item spans and the Pod span.
// table / ids (optional): the items' snapshot ids, looked up by the decoding threads; *ids
// is left empty when they were not (small body, or the list changed after the fast path).
int decode_args_core(const char* body, int64_t len, int32_t which,
                     std::vector<std::string>* names, std::vector<int64_t>* spans,
                     pas_args_info* info, const pas_name_table* table = nullptr,
                     std::vector<int32_t>* ids = nullptr) {
  std::memset(info, 0, sizeof *info);
  Scanner s{body, body + len};
  ItemIndex index;
  ItemIndex* idx = nullptr;
  if (which == PAS_ARGS_NODES && (index.threads = decode_threads_for(len)) > 1) {
    index.body = body;
    index.len = len;
    index.table = ids ? table : nullptr;
    PAS_TRACE_T0(t_index);
    index.build();
    PAS_TRACE_MS("index", t_index);
    idx = &index;
  }
  NodeList nodes;
  std::vector<std::string> node_names;
  bool has_nodes = false, has_names = false;
  const char* pod_b = nullptr;
  const char* pod_e = nullptr;
  s.ws();
  if (s.p >= s.end) return PAS_EDECODE;  // io.EOF: "request body empty" / errDecode
  const char c0 = *s.p;
  bool ok;
  if (c0 == 'n') {
    ok = s.literal("null");  // decodes to the zero Args
  } else if (c0 != '{') {
    ok = s.skip();
    s.type_err = true;
  } else {
    ok = s.object([&](std::string_view k) {
      if (fold_match("Pod", k)) {
        const char c = s.peek();
        if (c == 'n') return s.literal("null");  // a struct keeps its value
        if (c != '{') return s.mismatch();
        pod_b = s.p;
        if (!check_value(s, &pas_schema::Pod)) return false;  // v1.Pod, type-checked
        pod_e = s.p;
        return true;
      }
      if (fold_match("Nodes", k)) {
        if (idx) item_list_changed(idx);
        const char c = s.peek();
        if (c == 'n') {
          has_nodes = false;
          nodes.names.clear();
          nodes.spans.clear();
          return s.literal("null");
        }
        if (c != '{') return s.mismatch();
        if (!has_nodes) {  // a new NodeList; a repeated key decodes into the same one
          nodes.names.clear();
          nodes.spans.clear();
        }
        has_nodes = true;
        return decode_node_list(s, &nodes, body, idx);
      }
      if (fold_match("NodeNames", k)) {
        const char c = s.peek();
        if (c == 'n') {
          has_names = false;
          node_names.clear();
          return s.literal("null");
        }
        if (c != '[') return s.mismatch();
        if (!has_names) node_names.clear();
        has_names = true;
        size_t n = 0;
        const bool r = s.array([&](int64_t i) {
          if ((size_t)i >= node_names.size()) node_names.emplace_back();
          n = (size_t)i + 1;
          return string_field(s, &node_names[(size_t)i]);
        });
        node_names.resize(n);
        return r;
      }
      return s.skip();
    });
  }
  if (!ok || s.syntax_err || s.type_err) return PAS_EDECODE;
  info->has_nodes = has_nodes ? 1 : 0;
  info->has_node_names = has_names ? 1 : 0;
  if (pod_b) {
    info->pod_off = (int64_t)(pod_b - body);
    info->pod_len = (int64_t)(pod_e - pod_b);
  }
  if (which == PAS_ARGS_NODES) {
    if (ids && idx && idx->table && idx->ids_mods == idx->mods &&
        idx->ids.size() == nodes.names.size())
      *ids = std::move(idx->ids);
    *names = std::move(nodes.names);
    if (spans) *spans = std::move(nodes.spans);
  } else {
    *names = std::move(node_names);
  }
  info->n_req = (int32_t)names->size();
  return PAS_OK;
}

}  // namespace

extern "C" {

int pas_decode_args(const pas_name_table* t, const char* body, int64_t len, int32_t which,
                    int32_t* req_node, int64_t node_cap, int64_t* item_span, uint64_t* cand,
                    pas_args_info* info) {
  if (!t || !info || len < 0 || (len > 0 && !body) || node_cap < 0 ||
      (node_cap > 0 && !req_node) || (which != PAS_ARGS_NODES && which != PAS_ARGS_NODE_NAMES) ||
      (item_span && which != PAS_ARGS_NODES))
    return PAS_EINVAL;
  std::vector<std::string> names;
  std::vector<int64_t> spans;
  std::vector<int32_t> ids;
  const int rc = decode_args_core(body, len, which, &names, item_span ? &spans : nullptr, info,
                                  t, &ids);
  if (rc != PAS_OK) return rc;
  if (cand) std::memset(cand, 0, sizeof(uint64_t) * ((t->names.size() + 63) / 64));
  const bool fits = (int64_t)names.size() <= node_cap;
  if (!ids.empty() || names.empty()) {  // looked up by the threads that decoded the items
    for (size_t i = 0; i < ids.size(); ++i) {
      const int32_t id = ids[i];
      if (id < 0)
        ++info->n_unknown;
      else if (cand)
        cand[id >> 6] |= 1ull << (id & 63);
      if (fits) req_node[i] = id;
    }
    if (!fits) return PAS_ECAPACITY;
    if (item_span && !spans.empty())
      std::memcpy(item_span, spans.data(), sizeof(int64_t) * spans.size());
    return PAS_OK;
  }
  // name lookups, split over host threads for a large request (candidate bits or-ed in)
  const size_t n = names.size();
  const int T = n >= 16384 ? decode_threads_for(len) : 1;
  std::vector<int32_t> unknown((size_t)T, 0);
  auto lookup = [&](int th) {
    const size_t lo = n * (size_t)th / (size_t)T, hi = n * (size_t)(th + 1) / (size_t)T;
    for (size_t i = lo; i < hi; ++i) {
      const int32_t id = t->find(names[i]);
      if (id < 0)
        ++unknown[(size_t)th];
      else if (cand)
        __atomic_fetch_or(&cand[id >> 6], 1ull << (id & 63), __ATOMIC_RELAXED);
      if (fits) req_node[i] = id;
    }
  };
  PAS_TRACE_T0(t_lookup);
  if (T <= 1 || !parallel_for(T, lookup)) {
    std::fill(unknown.begin(), unknown.end(), 0);
    if (cand) std::memset(cand, 0, sizeof(uint64_t) * ((t->names.size() + 63) / 64));
    for (int th = 0; th < T; ++th) lookup(th);
  }
  PAS_TRACE_MS("lookups", t_lookup);
  for (int32_t u : unknown) info->n_unknown += u;
  if (!fits) return PAS_ECAPACITY;
  if (item_span && !spans.empty())
    std::memcpy(item_span, spans.data(), sizeof(int64_t) * spans.size());
  return PAS_OK;
}

int pas_decode_set_threads(int32_t n) {
  if (n < 0) return PAS_EINVAL;
  g_decode_threads.store(n, std::memory_order_relaxed);
  return PAS_OK;
}

int32_t pas_decode_threads(int64_t body_len) {
  return body_len < 0 ? 1 : (int32_t)decode_threads_for(body_len);
}

int pas_decode_request_names(const char* body, int64_t len, int32_t which, char* buf,
                             int64_t cap, int64_t* offsets, int64_t offsets_cap,
                             int64_t* total_len, int32_t* n_req) {
  if (len < 0 || (len > 0 && !body) || cap < 0 || (cap > 0 && !buf) || offsets_cap < 0 ||
      (offsets_cap > 0 && !offsets) || !total_len || !n_req ||
      (which != PAS_ARGS_NODES && which != PAS_ARGS_NODE_NAMES))
    return PAS_EINVAL;
  std::vector<std::string> names;
  pas_args_info info;
  const int rc = decode_args_core(body, len, which, &names, nullptr, &info);
  if (rc != PAS_OK) return rc;
  int64_t total = 0;
  for (const std::string& n : names) total += (int64_t)n.size();
  *total_len = total;
  *n_req = (int32_t)names.size();
  if (total > cap || (int64_t)names.size() + 1 > offsets_cap) return PAS_ECAPACITY;
  int64_t pos = 0;
  for (size_t i = 0; i < names.size(); ++i) {
    offsets[i] = pos;
    if (!names[i].empty()) std::memcpy(buf + pos, names[i].data(), names[i].size());
    pos += (int64_t)names[i].size();
  }
  offsets[names.size()] = pos;
  return PAS_OK;
}

int pas_decode_pod_policy(const char* pod, int64_t len, const char* label, char* ns_buf,
                          int64_t ns_cap, int64_t* ns_len, char* label_buf, int64_t label_cap,
                          int64_t* label_len) {
  if (len < 0 || (len > 0 && !pod) || !label || !ns_len || !label_len || ns_cap < 0 ||
      label_cap < 0 || (ns_cap > 0 && !ns_buf) || (label_cap > 0 && !label_buf))
    return PAS_EINVAL;
  std::string ns, value;
  bool has_label = false;
  const std::string_view want(label);
  if (len > 0) {
    Scanner s{pod, pod + len};
    const char c = s.peek();
    bool ok;
    if (c == 'n') {
      ok = s.literal("null");
    } else if (c != '{') {
      ok = s.skip();
      s.type_err = true;
    } else {
      ok = s.object([&](std::string_view k) {
        if (!fold_match("metadata", k)) return s.skip();
        const char m = s.peek();
        if (m == 'n') return s.literal("null");
        if (m != '{') return s.mismatch();
        return s.object([&](std::string_view mk) {
          if (fold_match("namespace", mk)) return string_field(s, &ns);
          if (fold_match("annotations", mk)) return string_map(s, [](std::string_view, auto&) {});
          if (!fold_match("labels", mk)) return s.skip();
          if (s.peek() == 'n') has_label = false;  // a nil map
          // a map decodes into the existing map (entries accumulate across repeated keys);
          // every entry is type-checked, not only the policy label
          return string_map(s, [&](std::string_view lk, const std::string& v) {
            if (lk != want) return;
            has_label = true;
            value = v;
          });
        });
      });
    }
    if (!ok || s.syntax_err || s.type_err || !pod_typed_ok(pod, len)) return PAS_EDECODE;
  }
  *ns_len = (int64_t)ns.size();
  *label_len = has_label ? (int64_t)value.size() : -1;
  if ((int64_t)ns.size() > ns_cap || (has_label && (int64_t)value.size() > label_cap))
    return PAS_ECAPACITY;
  if (!ns.empty()) std::memcpy(ns_buf, ns.data(), ns.size());
  if (has_label && !value.empty()) std::memcpy(label_buf, value.data(), value.size());
  return PAS_OK;
}

int pas_decode_pod_requests(const char* pod, int64_t len, int32_t n_kinds,
                            const char* const* kinds, int32_t max_containers, int64_t* req,
                            uint32_t* req_mask, int32_t* n_containers, int32_t* n_unknown) {
  if (len < 0 || (len > 0 && !pod) || n_kinds < 0 || n_kinds > 31 || (n_kinds > 0 && !kinds) ||
      max_containers < 0 || (max_containers > 0 && ((n_kinds > 0 && !req) || !req_mask)) ||
      !n_containers ||
      !n_unknown)
    return PAS_EINVAL;
  for (int32_t q = 0; q < n_kinds; ++q)
    if (!kinds[q]) return PAS_EINVAL;
  static const char kPrefix[] = "gpu.intel.com/";  // resourcePrefix (utils.go:9-12)
  struct Container {
    std::vector<std::string> names;  // requests keys in the map (unique, last value wins)
    std::vector<int64_t> values;
  };
  std::vector<Container> cont;
  if (len > 0) {
    Scanner s{pod, pod + len};
    bool ok;
    // ResourceList values: Quantity.UnmarshalJSON on the literal bytes
    auto quantity = [&](int64_t* v) {
      s.ws();
      const char* b = s.p;
      if (!s.skip()) return false;
      std::string lit(b, (size_t)(s.p - b));
      if (lit == "null") {
        *v = 0;
        return true;
      }
      if (lit.size() >= 2 && lit.front() == '"' && lit.back() == '"')
        lit = lit.substr(1, lit.size() - 2);
      const std::string q = trim_space(lit);
      if (q.find('\0') != std::string::npos || pas_quantity_as_int64(q.c_str(), v) != PAS_OK) {
        s.type_err = true;  // ParseQuantity error -> the decode fails
      }
      return true;
    };
    auto container = [&](Container* ct) {
      const char c = s.peek();
      if (c == 'n') return s.literal("null");
      if (c != '{') return s.mismatch();
      return s.object([&](std::string_view k) {
        if (!fold_match("resources", k)) return s.skip();
        const char r = s.peek();
        if (r == 'n') return s.literal("null");
        if (r != '{') return s.mismatch();
        return s.object([&](std::string_view rk) {
          if (fold_match("limits", rk)) {  // a ResourceList too: every value is parsed
            const char m = s.peek();
            if (m == 'n') return s.literal("null");
            if (m != '{') return s.mismatch();
            return s.object([&](std::string_view) {
              int64_t v = 0;
              return quantity(&v);
            });
          }
          if (!fold_match("requests", rk)) return s.skip();
          const char m = s.peek();
          if (m == 'n') {
            ct->names.clear();
            ct->values.clear();
            return s.literal("null");
          }
          if (m != '{') return s.mismatch();
          return s.object([&](std::string_view name) {
            int64_t v = 0;
            if (!quantity(&v)) return false;
            for (size_t i = 0; i < ct->names.size(); ++i)
              if (ct->names[i] == name) {
                ct->values[i] = v;
                return true;
              }
            ct->names.emplace_back(name);
            ct->values.push_back(v);
            return true;
          });
        });
      });
    };
    const char c = s.peek();
    if (c == 'n') {
      ok = s.literal("null");
    } else if (c != '{') {
      ok = s.skip();
      s.type_err = true;
    } else {
      ok = s.object([&](std::string_view k) {
        if (fold_match("metadata", k)) {  // ObjectMeta maps are type-checked as Go decodes them
          const char m = s.peek();
          if (m == 'n') return s.literal("null");
          if (m != '{') return s.mismatch();
          return s.object([&](std::string_view mk) {
            if (fold_match("labels", mk) || fold_match("annotations", mk))
              return string_map(s, [](std::string_view, auto&) {});
            return s.skip();
          });
        }
        if (!fold_match("spec", k)) return s.skip();
        const char sp = s.peek();
        if (sp == 'n') return s.literal("null");
        if (sp != '{') return s.mismatch();
        return s.object([&](std::string_view sk) {
          if (!fold_match("containers", sk)) return s.skip();
          const char a = s.peek();
          if (a == 'n') {
            cont.clear();
            return s.literal("null");
          }
          if (a != '[') return s.mismatch();
          // the slice is reused: elements keep what an earlier "containers" decoded
          size_t n = 0;
          bool r = s.array([&](int64_t i) {
            if ((size_t)i >= cont.size()) cont.emplace_back();
            n = (size_t)i + 1;
            return container(&cont[(size_t)i]);
          });
          cont.resize(n);
          return r;
        });
      });
    }
    if (!ok || s.syntax_err || s.type_err || !pod_typed_ok(pod, len)) return PAS_EDECODE;
  }
  *n_containers = (int32_t)cont.size();
  *n_unknown = 0;
  if ((int64_t)cont.size() > max_containers) return PAS_ECAPACITY;
  for (size_t c = 0; c < cont.size(); ++c) {
    req_mask[c] = 0;
    for (int32_t q = 0; q < n_kinds; ++q) req[(int64_t)c * n_kinds + q] = 0;
    for (size_t i = 0; i < cont[c].names.size(); ++i) {
      const std::string& name = cont[c].names[i];
      if (name.compare(0, sizeof kPrefix - 1, kPrefix) != 0) continue;
      int32_t q = 0;
      while (q < n_kinds && name != kinds[q]) ++q;
      if (q == n_kinds) {  // no node's capacity has the key: every check fails (:349-354)
        ++*n_unknown;
        req_mask[c] |= PAS_REQ_UNKNOWN_KIND;
        continue;
      }
      req[(int64_t)c * n_kinds + q] = cont[c].values[i];
      req_mask[c] |= 1u << q;
    }
  }
  return PAS_OK;
}

}  // extern "C"
