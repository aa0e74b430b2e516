// json_out.h — byte-exact encoding/json (Go 1.16) output for the wire encoders.
//
// The reference writes every extender response with json.NewEncoder(w).Encode(v)
// (telemetryscheduler.go:152-158, 238-244; gpuscheduler/scheduler.go:508-513) and label
// patches with json.Marshal (deschedule/enforce.go:75).  Strings follow encodeState.string
// with HTML escaping on (the default): '"' and '\\' backslash-escaped, \n \r \t short forms,
// other bytes < 0x20 and '<' '>' '&' as \u00XX, the code points U+2028 / U+2029 as \u2028 /
// \u2029, and each invalid UTF-8 byte as \ufffd.  Writes past `cap` are counted, not stored, so a caller
// learns the full length from one pass.
#pragma once

#include <cstdint>
#include <cstring>

namespace pas {

struct JsonOut {
  char* buf;
  int64_t cap;
  int64_t pos = 0;

  void put(char c) {
    if (pos < cap) buf[pos] = c;
    ++pos;
  }
  void raw(const char* s, int64_t n) {
    if (pos < cap) std::memcpy(buf + pos, s, (size_t)(pos + n <= cap ? n : cap - pos));
    pos += n;
  }
  // inline: for a string literal the compiler folds strlen to a constant
  void lit(const char* s) { raw(s, (int64_t)std::strlen(s)); }
  void integer(int64_t v) {
    char tmp[24];
    int n = 24;
    uint64_t u = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    do {
      tmp[--n] = (char)('0' + u % 10);
      u /= 10;
    } while (u);
    if (v < 0) tmp[--n] = '-';
    raw(tmp + n, 24 - n);
  }

  // UTF-8 sequence length at s (1..4, within the `avail` bytes left) if valid per Go's
  // utf8.DecodeRuneInString, else 0; *rune gets the code point.
  static int utf8_len(const unsigned char* s, int64_t avail, uint32_t* rune) {
    const unsigned char c = s[0];
    if (c < 0x80) { *rune = c; return 1; }
    auto cont = [&](int i) { return i < avail && (s[i] & 0xC0) == 0x80; };
    if (c >= 0xC2 && c <= 0xDF && cont(1)) {
      *rune = ((c & 0x1Fu) << 6) | (s[1] & 0x3Fu);
      return 2;
    }
    if (c >= 0xE0 && c <= 0xEF && cont(1) && cont(2)) {
      const uint32_t r = ((c & 0x0Fu) << 12) | ((s[1] & 0x3Fu) << 6) | (s[2] & 0x3Fu);
      if (r < 0x800 || (r >= 0xD800 && r <= 0xDFFF)) return 0;  // overlong / surrogate
      *rune = r;
      return 3;
    }
    if (c >= 0xF0 && c <= 0xF4 && cont(1) && cont(2) && cont(3)) {
      const uint32_t r = ((c & 0x07u) << 18) | ((s[1] & 0x3Fu) << 12) | ((s[2] & 0x3Fu) << 6) |
                         (s[3] & 0x3Fu);
      if (r < 0x10000 || r > 0x10FFFF) return 0;
      *rune = r;
      return 4;
    }
    return 0;
  }

  // String body (no quotes) of the NUL-terminated s.
  void str_body(const char* s) { str_body_n(s, (int64_t)std::strlen(s)); }

  // ASCII bytes that are copied as they are (no escape): 0x20-0x7F but '"' '\\' '<' '>' '&'.
  struct PlainTable {
    bool v[256];
    constexpr PlainTable() : v() {
      for (int c = 0x20; c < 0x80; ++c)  // DEL (0x7F) is not escaped by Go
        v[c] = c != '"' && c != '\\' && c != '<' && c != '>' && c != '&';
    }
  };
  static bool plain(unsigned char c) {
    static constexpr PlainTable t{};
    return t.v[c];
  }

  // String body (no quotes) of the n bytes at s: runs of plain bytes are copied whole, every
  // other byte takes the escape path below.  When the worst case (6 output bytes per input
  // byte) fits the buffer, the body is written through a local pointer (stores through a
  // char pointer may alias `pos`, which would otherwise be reloaded and stored per byte).
  void str_body_n(const char* s, int64_t n) {
    static const char hex[] = "0123456789abcdef";
    const unsigned char* p = reinterpret_cast<const unsigned char*>(s);
    const unsigned char* end = p + n;
    if (pos <= cap && cap - pos >= 6 * n) {
      char* w = buf + pos;
      while (p < end) {
        const unsigned char c = *p;
        if (plain(c)) {
          *w++ = (char)c;
          ++p;
          continue;
        }
        if (c < 0x80) {
          *w++ = '\\';
          switch (c) {
            case '"': *w++ = '"'; break;
            case '\\': *w++ = '\\'; break;
            case '\n': *w++ = 'n'; break;
            case '\r': *w++ = 'r'; break;
            case '\t': *w++ = 't'; break;
            default:
              std::memcpy(w, "u00", 3);
              w[3] = hex[c >> 4];
              w[4] = hex[c & 15];
              w += 5;
          }
          ++p;
          continue;
        }
        uint32_t r = 0;
        const int len = utf8_len(p, end - p, &r);
        if (len == 0) {
          std::memcpy(w, "\\ufffd", 6);
          w += 6;
          ++p;
        } else if (r == 0x2028 || r == 0x2029) {
          std::memcpy(w, r == 0x2028 ? "\\u2028" : "\\u2029", 6);
          w += 6;
          p += len;
        } else {
          std::memcpy(w, p, (size_t)len);
          w += len;
          p += len;
        }
      }
      pos = w - buf;
      return;
    }
    while (p < end) {
      const unsigned char* run = p;
      while (run < end && plain(*run)) ++run;
      if (run > p) {
        raw(reinterpret_cast<const char*>(p), run - p);
        p = run;
        if (p == end) break;
      }
      const unsigned char c = *p;
      if (c < 0x80) {
        switch (c) {
          case '"': put('\\'); put('"'); break;
          case '\\': put('\\'); put('\\'); break;
          case '\n': put('\\'); put('n'); break;
          case '\r': put('\\'); put('r'); break;
          case '\t': put('\\'); put('t'); break;
          default:
            if (c < 0x20 || c == '<' || c == '>' || c == '&') {
              lit("\\u00");
              put(hex[c >> 4]);
              put(hex[c & 15]);
            } else {
              put((char)c);
            }
        }
        ++p;
        continue;
      }
      uint32_t r = 0;
      const int len = utf8_len(p, end - p, &r);
      if (len == 0) {
        lit("\\ufffd");
        ++p;
      } else if (r == 0x2028 || r == 0x2029) {
        lit(r == 0x2028 ? "\\u2028" : "\\u2029");
        p += len;
      } else {
        raw(reinterpret_cast<const char*>(p), len);
        p += len;
      }
    }
  }
  void str(const char* s) {
    put('"');
    str_body(s);
    put('"');
  }
  void str_n(const char* s, int64_t n) {
    put('"');
    str_body_n(s, n);
    put('"');
  }
};

}  // namespace pas
