// quantity.cpp — resource.Quantity parsing as k8s.io/apimachinery v0.22.2 does it (host only).
//
// The reference reads quantities in two places on the hot path:
//   * TAS rule compares: Quantity.CmpInt64 / Cmp on metric values
//     (telemetry-aware-scheduling/pkg/strategies/core/operator.go:16-22,37-39) — the exact
//     value of the parsed quantity;
//   * GAS requests / capacities: Quantity.AsInt64 with `ok` ignored
//     (gpu-aware-scheduling/pkg/gpuscheduler/utils.go:23, scheduler.go:155).
// Both see the Quantity that resource.ParseQuantity builds (quantity.go in apimachinery
// v0.22.2; the module is not vendored in the reference, go.sum pins it).  Its published
// behaviour, restated here:
//   1. parseQuantityString splits <sign><digits>[.<digits>]<suffix>, stripping leading zeros
//      of the integer part; "0" is a fast path (value 0).
//   2. The suffix picks base / exponent / format: "" n u m k M G T P E (DecimalSI),
//      Ki Mi Gi Ti Pi Ei (BinarySI, base 2), e<int> / E<int> (DecimalExponent).
//   3. Fast path — an int64Amount{value, scale}:
//        DecimalSI / DecimalExponent: precision = 18 - (len(num) + len(denom));
//        BinarySI with exponent >= 0 and no fraction:
//            precision = 15 - len(num) - int(exponent * 3 / 10) - 1, mantissa = 2^exponent;
//        otherwise precision = -1.
//      With precision >= 0: scale = exponent (decimal) or 0 (binary), minus len(denom); if
//      scale >= -9, value = int(num + denom) * mantissa when that does not overflow.
//   4. Otherwise an inf.Dec: the exact value, rounded AWAY from zero to 9 fractional digits
//      (inf.RoundUp at Nano) unless it is 0, then capped to +-(2^63 - 1).
//   AsInt64: an inf.Dec -> (0, false); an int64Amount with scale 0 -> value, scale < 0 ->
//   (0, false), scale > 0 -> value * 10^scale, (0, false) on overflow.
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "pas.h"

namespace pas {
namespace {

// Non-negative big integer in base 1e9 limbs (little-endian), for the inf.Dec path.
struct Big {
  std::vector<uint32_t> l;  // empty = 0
  static constexpr uint32_t kBase = 1000000000u;
  bool zero() const { return l.empty(); }
  void trim() {
    while (!l.empty() && l.back() == 0) l.pop_back();
  }
  void mul_small(uint32_t m) {
    uint64_t carry = 0;
    for (uint32_t& x : l) {
      const uint64_t v = (uint64_t)x * m + carry;
      x = (uint32_t)(v % kBase);
      carry = v / kBase;
    }
    while (carry) {
      l.push_back((uint32_t)(carry % kBase));
      carry /= kBase;
    }
  }
  void add_small(uint32_t a) {
    uint64_t carry = a;
    for (size_t i = 0; carry && i < l.size(); ++i) {
      const uint64_t v = (uint64_t)l[i] + carry;
      l[i] = (uint32_t)(v % kBase);
      carry = v / kBase;
    }
    if (carry) l.push_back((uint32_t)carry);
  }
  // divides by m, returns the remainder
  uint32_t div_small(uint32_t m) {
    uint64_t rem = 0;
    for (size_t i = l.size(); i-- > 0;) {
      const uint64_t v = rem * kBase + l[i];
      l[i] = (uint32_t)(v / m);
      rem = v % m;
    }
    trim();
    return (uint32_t)rem;
  }
  // value if it fits 127 bits, else false
  bool to_i128(__int128* out) const {
    __int128 v = 0;
    const __int128 lim = (((__int128)1) << 126) / kBase;
    for (size_t i = l.size(); i-- > 0;) {
      if (v > lim) return false;
      v = v * kBase + l[i];
    }
    *out = v;
    return true;
  }
};

struct Parsed {
  bool dec = false;     // inf.Dec-backed (AsInt64 -> 0)
  int64_t value = 0;    // int64Amount.value (signed)
  int32_t scale = 0;    // int64Amount.scale: value * 10^scale
  __int128 nano = 0;    // inf.Dec: the value in units of 1e-9 (rounded, capped)
};

bool is_digit(char c) { return c >= '0' && c <= '9'; }

// parseQuantityString: sign, integer digits (leading zeros stripped), fraction, suffix.
// Returns false on a format error.
bool split(const std::string& s, bool* positive, std::string* num, std::string* denom,
           std::string* suffix) {
  *positive = true;
  size_t pos = 0, end = s.size();
  if (pos < end && (s[0] == '-' || s[0] == '+')) {
    *positive = s[0] != '-';
    ++pos;
  }
  while (pos < end && s[pos] == '0') ++pos;  // leading zeros
  if (pos >= end) {                          // all zeros (or just a sign)
    *num = "0";
    return true;
  }
  size_t i = pos;
  while (i < end && is_digit(s[i])) ++i;
  *num = s.substr(pos, i - pos);
  pos = i;
  if (num->empty()) *num = "0";
  if (pos < end && s[pos] == '.') {
    ++pos;
    i = pos;
    while (i < end && is_digit(s[i])) ++i;
    *denom = s.substr(pos, i - pos);
    pos = i;
  }
  const size_t suffix_start = pos;
  static const char kSuffixChars[] = "eEinumkKMGTP";
  while (pos < end && std::strchr(kSuffixChars, s[pos]) != nullptr) ++pos;
  if (pos < end && (s[pos] == '-' || s[pos] == '+')) ++pos;
  while (pos < end && is_digit(s[pos])) ++pos;
  if (pos < end) return false;  // ErrFormatWrong
  *suffix = s.substr(suffix_start);
  return true;
}

// quantitySuffixer.interpret: base (10 or 2), exponent, binary?, ok.
bool interpret(const std::string& suf, int* base, int32_t* exponent, bool* binary) {
  static const struct {
    const char* s;
    int32_t e;
  } dec[] = {{"n", -9}, {"u", -6}, {"m", -3}, {"", 0},  {"k", 3},
             {"M", 6},  {"G", 9},  {"T", 12}, {"P", 15}, {"E", 18}};
  static const struct {
    const char* s;
    int32_t e;
  } bin[] = {{"Ki", 10}, {"Mi", 20}, {"Gi", 30}, {"Ti", 40}, {"Pi", 50}, {"Ei", 60}};
  *binary = false;
  for (const auto& d : dec)
    if (suf == d.s) {
      *base = 10;
      *exponent = d.e;
      return true;
    }
  for (const auto& b : bin)
    if (suf == b.s) {
      *base = 2;
      *exponent = b.e;
      *binary = true;
      return true;
    }
  if (suf.size() > 1 && (suf[0] == 'e' || suf[0] == 'E')) {
    // strconv.ParseInt(suffix[1:], 10, 64), then int32(parsed)
    size_t i = 1;
    bool neg = false;
    if (suf[i] == '+' || suf[i] == '-') neg = suf[i++] == '-';
    if (i >= suf.size()) return false;
    __int128 v = 0;
    for (; i < suf.size(); ++i) {
      if (!is_digit(suf[i])) return false;
      v = v * 10 + (suf[i] - '0');
      if (v > (__int128)INT64_MAX + 1) return false;  // ParseInt range error
    }
    if (neg) v = -v;
    if (v > INT64_MAX || v < INT64_MIN) return false;
    *base = 10;
    *exponent = (int32_t)(uint32_t)(uint64_t)(int64_t)v;  // int32(parsed) truncates
    return true;
  }
  return false;
}

bool mul64(int64_t a, int64_t b, int64_t* out) {  // int64Multiply
  if (a == 0 || b == 0 || a == 1 || b == 1) {
    *out = (int64_t)((uint64_t)a * (uint64_t)b);
    return true;
  }
  if (a == INT64_MIN || b == INT64_MIN) return false;
  const int64_t c = (int64_t)((uint64_t)a * (uint64_t)b);
  *out = c;
  return c / b == a;
}

constexpr int32_t kNano = -9;
const __int128 kMaxNano = (__int128)INT64_MAX * 1000000000;  // maxAllowed = 2^63 - 1

// resource.ParseQuantity.
int parse_quantity(const char* str, Parsed* q) {
  if (!str) return PAS_EINVAL;
  const std::string s(str);
  if (s.empty()) return PAS_EINVAL;
  *q = Parsed{};
  if (s == "0") return PAS_OK;
  bool positive;
  std::string num, denom, suffix;
  if (!split(s, &positive, &num, &denom, &suffix)) return PAS_EINVAL;
  int base;
  int32_t exponent;
  bool binary;
  if (!interpret(suffix, &base, &exponent, &binary)) return PAS_EINVAL;
  int32_t precision = 0, scale = 0;
  int64_t mantissa = 1;
  if (!binary) {
    scale = exponent;
    precision = 18 - (int32_t)(num.size() + denom.size());
  } else if (exponent >= 0 && denom.empty()) {
    mantissa = (int64_t)((uint64_t)mantissa << (uint64_t)exponent);
    precision = 15 - (int32_t)num.size() - (int32_t)((float)exponent * 3 / 10) - 1;
  } else {
    precision = -1;
  }
  if (precision >= 0) {
    scale -= (int32_t)denom.size();
    if (scale >= kNano) {
      const std::string shifted = num + denom;  // <= 18 digits: ParseInt cannot fail
      int64_t value = 0;
      for (char c : shifted) value = value * 10 + (c - '0');
      int64_t result;
      if (mul64(value, mantissa, &result)) {
        q->dec = false;
        q->value = positive ? result : -result;
        q->scale = scale;
        return PAS_OK;
      }
    }
  }
  // inf.Dec: value = digits(num.denom) * base^exponent (binary: * 2^exponent), exact, then
  // rounded away from zero at 9 fractional digits and capped at 2^63 - 1.
  q->dec = true;
  Big u;
  int32_t frac = (int32_t)denom.size();  // decimal places of the unscaled digits
  for (char c : num + denom) {
    u.mul_small(10);
    u.add_small((uint32_t)(c - '0'));
  }
  u.trim();
  if (base == 10) {
    frac -= exponent;  // SetScale(Scale() - exponent)
  } else {
    for (int32_t i = 0; i < exponent; ++i) u.mul_small(2);  // * 2^exponent (Ki .. Ei)
  }
  // to units of 1e-9: multiply by 10^(9 - frac) or divide (rounding up) by 10^(frac - 9)
  bool inexact = false;
  if (u.zero()) {
    q->nano = 0;
    return PAS_OK;
  }
  if (frac < 9) {
    for (int32_t i = frac; i < 9; ++i) {
      u.mul_small(10);
      if (u.l.size() > 6) break;  // > 1e45: certainly above the cap
    }
  } else {
    for (int32_t i = 9; i < frac; ++i) {
      if (u.div_small(10) != 0) inexact = true;
      if (u.zero()) break;
    }
  }
  __int128 nano = 0;
  if (u.l.size() > 6 || !u.to_i128(&nano) || nano > kMaxNano) {
    nano = kMaxNano;
  } else if (inexact) {
    nano += 1;  // RoundUp: away from zero (the magnitude is rounded before the sign)
    if (nano > kMaxNano) nano = kMaxNano;
  }
  q->nano = positive ? nano : -nano;
  return PAS_OK;
}

}  // namespace
}  // namespace pas

using pas::Parsed;

extern "C" {

int pas_quantity_as_int64(const char* quantity, int64_t* out) {
  if (!out) return PAS_EINVAL;
  Parsed q;
  const int rc = pas::parse_quantity(quantity, &q);
  if (rc != PAS_OK) return rc;
  *out = 0;
  if (q.dec || q.scale < 0) return PAS_OK;  // (0, false); the reference ignores ok
  int64_t v = q.value;
  for (int32_t i = 0; i < q.scale; ++i)  // positiveScaleInt64
    if (!pas::mul64(v, 10, &v)) return PAS_OK;
  *out = v;
  return PAS_OK;
}

int pas_quantity_to_scaled(const char* quantity, int32_t places, int64_t* out) {
  if (!out || places < 0 || places > 9) return PAS_EINVAL;
  Parsed q;
  const int rc = pas::parse_quantity(quantity, &q);
  if (rc != PAS_OK) return rc;
  __int128 v;
  if (q.dec) {  // units of 1e-9 -> units of 10^-places
    __int128 div = 1;
    for (int32_t i = places; i < 9; ++i) div *= 10;
    if (q.nano % div != 0) return PAS_ENOTEXACT;
    v = q.nano / div;
  } else {  // value * 10^(scale + places)
    v = q.value;
    int32_t e = q.scale + places;
    for (; e > 0; --e) {
      v *= 10;
      if (v > INT64_MAX || v < INT64_MIN) return PAS_ENOTEXACT;
    }
    for (; e < 0; ++e) {
      if (v % 10 != 0) return PAS_ENOTEXACT;
      v /= 10;
    }
  }
  if (v > INT64_MAX || v < INT64_MIN) return PAS_ENOTEXACT;
  *out = (int64_t)v;
  return PAS_OK;
}

int pas_quantity_to_milli(const char* quantity, int64_t* milli_out) {
  return pas_quantity_to_scaled(quantity, 3, milli_out);
}

int pas_quantity_decimals(const char* quantity, int32_t* places) {
  if (!places) return PAS_EINVAL;
  Parsed q;
  const int rc = pas::parse_quantity(quantity, &q);
  if (rc != PAS_OK) return rc;
  int32_t k = 0;
  if (q.dec) {  // 9 minus the trailing zero digits of the nano value
    __int128 n = q.nano;
    k = 9;
    while (k > 0 && n % 10 == 0) {
      n /= 10;
      --k;
    }
  } else if (q.scale < 0) {  // -scale minus the trailing zero digits of the value
    int64_t v = q.value;
    k = -q.scale;
    while (k > 0 && v % 10 == 0) {
      v /= 10;
      --k;
    }
  }
  *places = k;
  return PAS_OK;
}

}  // extern "C"
