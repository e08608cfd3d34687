// jsonl.cpp — collector JSONL -> History. Restates eventsFromReader
// (golang/s2-porcupine/main.go:529-563) with Go encoding/json semantics:
//   * a stream of JSON values (json.Decoder): any whitespace separation, no
//     line-length limit (main_test.go:34-101);
//   * Record{event, client_id, op_id} struct fields match keys
//     case-insensitively (Go's fold, incl. U+212A KELVIN / U+017F LONG S), the
//     last duplicate wins, unknown keys are ignored, null leaves a field as is;
//   * EventWrapper / StartEvent / FinishEvent custom unmarshalers
//     (main.go:32-70, 100-156, 163-188): map keys "Start", "Finish", "Append",
//     "AppendSuccess", ... match exactly; a duplicate "event" key re-runs the
//     wrapper's unmarshaler on the same value (Start/Finish accumulate);
//   * integers decode only from integer literals in range (strconv.ParseUint /
//     ParseInt), strings are UTF-8-sanitised (invalid bytes -> U+FFFD);
//   * len(record_hashes) != num_records is an error (main.go:62-64).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "history.h"
#include "s2lincheck.h"

namespace s2lc {
namespace {

enum JType : uint8_t { J_NULL, J_FALSE, J_TRUE, J_NUM, J_STR, J_ARR, J_OBJ };

struct JNode {
  JType t;
  uint32_t a;  // NUM: offset of literal; STR: string index; ARR/OBJ: first child slot
  uint32_t b;  // NUM: literal length; ARR/OBJ: child count
};

struct Parser {
  const uint8_t* p;
  const uint8_t* end;
  const uint8_t* base;
  std::vector<JNode> nodes;
  std::vector<uint32_t> kids;       // ARR: node ids; OBJ: (key string id, node id) pairs
  std::vector<std::string> strs;
  std::string err;
  int depth = 0;

  void reset() { nodes.clear(); kids.clear(); strs.clear(); }
  bool fail(const char* msg) {
    if (err.empty()) {
      char buf[160];
      snprintf(buf, sizeof buf, "%s at offset %zu", msg, (size_t)(p - base));
      err = buf;
    }
    return false;
  }
  void ws() {
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  static void put_utf8(std::string& s, uint32_t cp) {
    if (cp < 0x80) s.push_back((char)cp);
    else if (cp < 0x800) { s.push_back((char)(0xC0 | (cp >> 6))); s.push_back((char)(0x80 | (cp & 0x3F))); }
    else if (cp < 0x10000) {
      s.push_back((char)(0xE0 | (cp >> 12))); s.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      s.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      s.push_back((char)(0xF0 | (cp >> 18))); s.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      s.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); s.push_back((char)(0x80 | (cp & 0x3F)));
    }
  }
  bool hex4(uint32_t& v) {
    if (end - p < 4) return fail("bad \\u escape");
    v = 0;
    for (int i = 0; i < 4; ++i) {
      uint8_t c = p[i];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else return fail("bad \\u escape");
    }
    p += 4;
    return true;
  }
  // Decode a string literal (p at opening quote) with Go's replacement rules.
  bool str(std::string& out) {
    ++p;
    out.clear();
    while (true) {
      if (p >= end) return fail("unexpected end of input in string");
      uint8_t c = *p;
      if (c == '"') { ++p; return true; }
      if (c < 0x20) return fail("invalid character in string literal");
      if (c == '\\') {
        ++p;
        if (p >= end) return fail("unexpected end of input in string");
        uint8_t e = *p++;
        switch (e) {
          case '"': out.push_back('"'); break;
          case '\\': out.push_back('\\'); break;
          case '/': out.push_back('/'); break;
          case 'b': out.push_back('\b'); break;
          case 'f': out.push_back('\f'); break;
          case 'n': out.push_back('\n'); break;
          case 'r': out.push_back('\r'); break;
          case 't': out.push_back('\t'); break;
          case 'u': {
            uint32_t cp;
            if (!hex4(cp)) return false;
            if (cp >= 0xD800 && cp < 0xDC00) {  // high surrogate: needs a low one
              if (end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
                const uint8_t* save = p;
                p += 2;
                uint32_t lo;
                if (!hex4(lo)) return false;
                if (lo >= 0xDC00 && lo < 0xE000) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                else { cp = 0xFFFD; p = save; }
              } else cp = 0xFFFD;
            } else if (cp >= 0xDC00 && cp < 0xE000) cp = 0xFFFD;
            put_utf8(out, cp);
            break;
          }
          default: return fail("invalid escape in string literal");
        }
        continue;
      }
      if (c < 0x80) { out.push_back((char)c); ++p; continue; }
      // validate one UTF-8 sequence; invalid byte -> U+FFFD (Go decodeState.unquote)
      int n = 0; uint32_t cp = 0, minv = 0;
      if ((c & 0xE0) == 0xC0) { n = 2; cp = c & 0x1F; minv = 0x80; }
      else if ((c & 0xF0) == 0xE0) { n = 3; cp = c & 0x0F; minv = 0x800; }
      else if ((c & 0xF8) == 0xF0) { n = 4; cp = c & 0x07; minv = 0x10000; }
      bool ok = n > 0 && end - p >= n;
      for (int i = 1; ok && i < n; ++i) {
        if ((p[i] & 0xC0) != 0x80) ok = false;
        else cp = (cp << 6) | (p[i] & 0x3F);
      }
      if (ok && (cp < minv || cp > 0x10FFFF || (cp >= 0xD800 && cp < 0xE000))) ok = false;
      if (ok) { out.append((const char*)p, (size_t)n); p += n; }
      else { put_utf8(out, 0xFFFD); ++p; }
    }
  }
  bool number(uint32_t& node) {
    const uint8_t* s = p;
    if (*p == '-') ++p;
    if (p >= end) return fail("unexpected end of input in number");
    if (*p == '0') ++p;
    else if (*p >= '1' && *p <= '9') { while (p < end && *p >= '0' && *p <= '9') ++p; }
    else return fail("invalid character in numeric literal");
    if (p < end && *p == '.') {
      ++p;
      if (p >= end || *p < '0' || *p > '9') return fail("invalid character after decimal point");
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    if (p < end && (*p == 'e' || *p == 'E')) {
      ++p;
      if (p < end && (*p == '+' || *p == '-')) ++p;
      if (p >= end || *p < '0' || *p > '9') return fail("invalid character in exponent");
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    node = (uint32_t)nodes.size();
    nodes.push_back({J_NUM, (uint32_t)(s - base), (uint32_t)(p - s)});
    return true;
  }
  bool lit(const char* w, JType t, uint32_t& node) {
    size_t n = strlen(w);
    if ((size_t)(end - p) < n) { p = end; return fail("unexpected end of input"); }
    if (memcmp(p, w, n) != 0) return fail("invalid literal");
    p += n;
    node = (uint32_t)nodes.size();
    nodes.push_back({t, 0, 0});
    return true;
  }
  bool value(uint32_t& node) {
    ws();
    if (p >= end) return fail("unexpected end of JSON input");
    uint8_t c = *p;
    if (c == '{') {
      if (++depth > 10000) return fail("exceeded max depth");
      ++p;
      std::vector<uint32_t> local;
      ws();
      if (p < end && *p == '}') { ++p; }
      else {
        while (true) {
          ws();
          if (p >= end) return fail("unexpected end of JSON input");
          if (*p != '"') return fail("invalid character looking for beginning of object key string");
          std::string key;
          if (!str(key)) return false;
          ws();
          if (p >= end) return fail("unexpected end of JSON input");
          if (*p != ':') return fail("invalid character after object key");
          ++p;
          uint32_t v;
          if (!value(v)) return false;
          local.push_back((uint32_t)strs.size());
          strs.push_back(std::move(key));
          local.push_back(v);
          ws();
          if (p >= end) return fail("unexpected end of JSON input");
          if (*p == ',') { ++p; continue; }
          if (*p == '}') { ++p; break; }
          return fail("invalid character after object key:value pair");
        }
      }
      --depth;
      node = (uint32_t)nodes.size();
      nodes.push_back({J_OBJ, (uint32_t)kids.size(), (uint32_t)(local.size() / 2)});
      kids.insert(kids.end(), local.begin(), local.end());
      return true;
    }
    if (c == '[') {
      if (++depth > 10000) return fail("exceeded max depth");
      ++p;
      std::vector<uint32_t> local;
      ws();
      if (p < end && *p == ']') { ++p; }
      else {
        while (true) {
          uint32_t v;
          if (!value(v)) return false;
          local.push_back(v);
          ws();
          if (p >= end) return fail("unexpected end of JSON input");
          if (*p == ',') { ++p; continue; }
          if (*p == ']') { ++p; break; }
          return fail("invalid character after array element");
        }
      }
      --depth;
      node = (uint32_t)nodes.size();
      nodes.push_back({J_ARR, (uint32_t)kids.size(), (uint32_t)local.size()});
      kids.insert(kids.end(), local.begin(), local.end());
      return true;
    }
    if (c == '"') {
      std::string s;
      if (!str(s)) return false;
      node = (uint32_t)nodes.size();
      nodes.push_back({J_STR, (uint32_t)strs.size(), 0});
      strs.push_back(std::move(s));
      return true;
    }
    if (c == '-' || (c >= '0' && c <= '9')) return number(node);
    if (c == 't') return lit("true", J_TRUE, node);
    if (c == 'f') return lit("false", J_FALSE, node);
    if (c == 'n') return lit("null", J_NULL, node);
    return fail("invalid character looking for beginning of value");
  }
};

// ---------------------------------------------------------- Go decoding ---
struct Dec {
  Parser& P;
  std::string err;
  explicit Dec(Parser& p) : P(p) {}

  const JNode& n(uint32_t i) const { return P.nodes[i]; }
  const char* type_name(uint32_t i) const {
    switch (n(i).t) {
      case J_NULL: return "null";
      case J_FALSE: case J_TRUE: return "bool";
      case J_NUM: return "number";
      case J_STR: return "string";
      case J_ARR: return "array";
      default: return "object";
    }
  }
  bool type_err(uint32_t i, const char* go_type) {
    if (err.empty()) err = std::string("json: cannot unmarshal ") + type_name(i) + " into Go value of type " + go_type;
    return false;
  }
  // Go struct-field key match: bytes.EqualFold semantics against an ASCII
  // lower-case field name (k and s also match U+212A and U+017F).
  static bool fold_eq(const std::string& key, const char* field) {
    size_t i = 0, j = 0, fl = strlen(field);
    while (i < key.size()) {
      if (j >= fl) return false;
      unsigned char c = (unsigned char)key[i];
      char f = field[j];
      if (c < 0x80) {
        char lc = (c >= 'A' && c <= 'Z') ? (char)(c + 32) : (char)c;
        if (lc != f) return false;
        ++i; ++j;
        continue;
      }
      if (key.compare(i, 3, "\xE2\x84\xAA") == 0 && f == 'k') { i += 3; ++j; continue; }  // KELVIN SIGN
      if (key.compare(i, 2, "\xC5\xBF") == 0 && f == 's') { i += 2; ++j; continue; }      // LONG S
      return false;
    }
    return j == fl;
  }
  // Map lookup (exact key, last duplicate wins).
  int64_t map_get(uint32_t obj, const char* key) const {
    const JNode& o = n(obj);
    int64_t found = -1;
    for (uint32_t k = 0; k < o.b; ++k)
      if (P.strs[P.kids[o.a + 2 * k]] == key) found = P.kids[o.a + 2 * k + 1];
    return found;
  }
  bool u64(uint32_t i, uint64_t& v, const char* go_type = "uint64") {
    const JNode& x = n(i);
    if (x.t == J_NULL) return true;  // null into a non-pointer: no-op
    if (x.t != J_NUM) return type_err(i, go_type);
    const uint8_t* s = P.base + x.a;
    uint64_t r = 0;
    for (uint32_t k = 0; k < x.b; ++k) {
      uint8_t c = s[k];
      if (c < '0' || c > '9') return type_err(i, go_type);  // sign, fraction, exponent
      if (r > (~0ull - (c - '0')) / 10) return type_err(i, go_type);
      r = r * 10 + (c - '0');
    }
    v = r;
    return true;
  }
  bool i64(uint32_t i, int64_t& v) {
    const JNode& x = n(i);
    if (x.t == J_NULL) return true;
    if (x.t != J_NUM) return type_err(i, "int");
    const uint8_t* s = P.base + x.a;
    uint32_t k = 0;
    bool neg = false;
    if (x.b && s[0] == '-') { neg = true; k = 1; }
    uint64_t r = 0;
    for (; k < x.b; ++k) {
      uint8_t c = s[k];
      if (c < '0' || c > '9') return type_err(i, "int");
      if (r > (~0ull - (c - '0')) / 10) return type_err(i, "int");
      r = r * 10 + (c - '0');
    }
    if (!neg && r > (uint64_t)INT64_MAX) return type_err(i, "int");
    if (neg && r > (uint64_t)INT64_MAX + 1) return type_err(i, "int");
    v = neg ? (int64_t)(0 - r) : (int64_t)r;
    return true;
  }
  bool opt_str(uint32_t i, bool& has, std::string& s) {
    const JNode& x = n(i);
    if (x.t == J_NULL) { has = false; return true; }
    if (x.t != J_STR) return type_err(i, "string");
    has = true;
    s = P.strs[x.a];
    return true;
  }
  bool opt_u64(uint32_t i, bool& has, uint64_t& v) {
    if (n(i).t == J_NULL) { has = false; return true; }
    v = 0;
    if (!u64(i, v)) return false;
    has = true;
    return true;
  }

  // AppendArgs (main.go:18-24) decoded into call event e.
  bool append_args(uint32_t i, Event& e, History& h, std::vector<uint64_t>& hashes) {
    const JNode& x = n(i);
    if (x.t == J_NULL) return true;
    if (x.t != J_OBJ) return type_err(i, "main.AppendArgs");
    bool has_set = false, has_tok = false;
    std::string set_s, tok_s;
    for (uint32_t k = 0; k < x.b; ++k) {
      const std::string& key = P.strs[P.kids[x.a + 2 * k]];
      uint32_t v = P.kids[x.a + 2 * k + 1];
      if (fold_eq(key, "num_records")) { if (!u64(v, e.num_records)) return false; }
      else if (fold_eq(key, "record_hashes")) {
        const JNode& a = n(v);
        if (a.t == J_NULL) { hashes.clear(); continue; }
        if (a.t != J_ARR) return type_err(v, "[]uint64");
        hashes.assign(a.b, 0);
        for (uint32_t q = 0; q < a.b; ++q) {
          uint64_t hv = 0;
          if (!u64(P.kids[a.a + q], hv)) return false;
          hashes[q] = hv;
        }
      } else if (fold_eq(key, "set_fencing_token")) { if (!opt_str(v, has_set, set_s)) return false; }
      else if (fold_eq(key, "fencing_token")) { if (!opt_str(v, has_tok, tok_s)) return false; }
      else if (fold_eq(key, "match_seq_num")) {
        bool hm = false; uint64_t mv = 0;
        if (!opt_u64(v, hm, mv)) return false;
        e.has_msn = hm; e.msn = mv;
      }
    }
    e.set_tok = has_set ? h.intern(set_s) : 0;
    e.batch_tok = has_tok ? h.intern(tok_s) : 0;
    return true;
  }

  // StartEvent.UnmarshalJSON, main.go:32-70 + inputFromStart, main.go:428-464
  bool start(uint32_t i, Event& e, History& h, std::vector<uint64_t>& hashes, bool& appended) {
    const JNode& x = n(i);
    if (x.t == J_STR || x.t == J_NULL) {  // json.Unmarshal(data, &str) succeeds
      const std::string s = x.t == J_STR ? P.strs[x.a] : std::string();
      if (s == "CheckTail") { e.input_type = S2LC_INPUT_CHECK_TAIL; return true; }
      if (s == "Read") { e.input_type = S2LC_INPUT_READ; return true; }
      err = "parsing Start: unknown string start event: " + s;
      return false;
    }
    if (x.t != J_OBJ) { type_err(i, "map[string]json.RawMessage"); err = "parsing Start: " + err; return false; }
    int64_t a = map_get(i, "Append");
    if (a < 0) { err = "parsing Start: unknown start event format"; return false; }
    e.input_type = S2LC_INPUT_APPEND;
    e.has_num_records = 1;
    e.num_records = 0;
    hashes.clear();
    if (!append_args((uint32_t)a, e, h, hashes)) { err = "parsing Start: parsing Append args: " + err; return false; }
    if ((uint64_t)hashes.size() != e.num_records) {
      err = "parsing Start: append has " + std::to_string(hashes.size()) + " record_hashes but " +
            std::to_string(e.num_records) + " records";
      return false;
    }
    appended = true;
    return true;
  }

  bool result_obj(uint32_t i, Event& e, bool read, const char* go_type) {
    const JNode& x = n(i);
    e.failure = 0; e.definite = 0; e.has_tail = 1; e.tail = 0;
    e.has_hash = read ? 1 : 0; e.stream_hash = 0;
    if (x.t == J_NULL) return true;
    if (x.t != J_OBJ) return type_err(i, go_type);
    for (uint32_t k = 0; k < x.b; ++k) {
      const std::string& key = P.strs[P.kids[x.a + 2 * k]];
      uint32_t v = P.kids[x.a + 2 * k + 1];
      if (fold_eq(key, "tail")) { if (!u64(v, e.tail)) return false; }
      else if (read && fold_eq(key, "stream_hash")) { if (!u64(v, e.stream_hash)) return false; }
    }
    return true;
  }

  // FinishEvent.UnmarshalJSON, main.go:100-156 + outputFromFinish, main.go:466-523
  bool finish(uint32_t i, Event& e) {
    const JNode& x = n(i);
    if (x.t == J_STR || x.t == J_NULL) {
      const std::string s = x.t == J_STR ? P.strs[x.a] : std::string();
      e.has_tail = 0; e.has_hash = 0;
      if (s == "AppendDefiniteFailure") { e.failure = 1; e.definite = 1; return true; }
      if (s == "AppendIndefiniteFailure") { e.failure = 1; e.definite = 0; return true; }
      if (s == "ReadFailure" || s == "CheckTailFailure") { e.failure = 1; e.definite = 1; return true; }
      err = "parsing Finish: unknown string finish event: " + s;
      return false;
    }
    if (x.t != J_OBJ) { type_err(i, "map[string]json.RawMessage"); err = "parsing Finish: " + err; return false; }
    int64_t v;
    if ((v = map_get(i, "AppendSuccess")) >= 0) {
      if (!result_obj((uint32_t)v, e, false, "main.AppendSuccessResult")) { err = "parsing Finish: parsing AppendSuccess result: " + err; return false; }
      return true;
    }
    if ((v = map_get(i, "ReadSuccess")) >= 0) {
      if (!result_obj((uint32_t)v, e, true, "main.ReadSuccessResult")) { err = "parsing Finish: parsing ReadSuccess result: " + err; return false; }
      return true;
    }
    if ((v = map_get(i, "CheckTailSuccess")) >= 0) {
      if (!result_obj((uint32_t)v, e, false, "main.CheckTailSuccessResult")) { err = "parsing Finish: parsing CheckTailSuccess result: " + err; return false; }
      return true;
    }
    err = "parsing Finish: unknown finish event format";
    return false;
  }
};


// ------------------------------------------------------------ fast path ---
// The collector's own serialisation (serde, history.rs; the simulator writes
// the same bytes): fixed key order, no whitespace inside a record, integers
// as plain digits, token strings without escapes. A record in exactly that
// form is decoded here without building a JSON tree; any byte that deviates
// sends the record to the general parser above (which also owns every error
// message), so the result is the same History either way (tests/test_jsonl.py
// compares both paths).
// eight characters as the little-endian word Fast::word() reads
constexpr uint64_t word8(const char (&w)[9]) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | (uint8_t)w[i];
  return v;
}

struct Fast {
  const uint8_t* p;
  const uint8_t* end;
  const uint8_t* lo;  // the record's first byte (tail8 reads up to 8 bytes before a digit run)
  // the literal w at p (eight bytes per compare; w is a compile-time constant)
  template <size_t N>
  bool lit(const char (&w)[N]) {
    constexpr size_t n = N - 1;
    static_assert(n >= 1, "literal");
    if ((size_t)(end - p) < (n < 8 ? 8 : n)) return lit_short(w);
    // whole 8-byte words, the last one overlapping the one before (n >= 8),
    // or one masked word (n < 8): no byte loop
    if constexpr (n >= 8) {
      for (size_t i = 0; i + 8 <= n; i += 8) {
        uint64_t a, b;
        memcpy(&a, p + i, 8);
        memcpy(&b, w + i, 8);
        if (a != b) return false;
      }
      if constexpr (n % 8 != 0) {
        uint64_t a, b;
        memcpy(&a, p + n - 8, 8);
        memcpy(&b, w + n - 8, 8);
        if (a != b) return false;
      }
    } else {
      uint64_t a, b = 0;
      memcpy(&a, p, 8);
      memcpy(&b, w, n);
      if ((a & (~0ull >> (8 * (8 - n)))) != b) return false;
    }
    p += n;
    return true;
  }
  // (within 8 bytes of the end of the input)
  template <size_t N>
  bool lit_short(const char (&w)[N]) {
    constexpr size_t n = N - 1;
    if ((size_t)(end - p) < n) return false;
    for (size_t i = 0; i < n; ++i)
      if (p[i] != (uint8_t)w[i]) return false;
    p += n;
    return true;
  }
  bool peek(char c) const { return p < end && *p == (uint8_t)c; }
  // the eight bytes at p (0, which no record text matches, within 8 bytes of the end)
  uint64_t word() const {
    uint64_t w = 0;
    if (end - p >= 8) memcpy(&w, p, 8);
    return w;
  }
  // a non-negative integer literal in uint64 range, not followed by a
  // fraction or exponent (those are type errors: the general parser reports them)
  static bool is_digit(uint8_t c) { return c >= '0' && c <= '9'; }
  // eight ASCII digits -> value (little-endian SWAR)
  static uint32_t eight(const uint8_t* q) {
    uint64_t v;
    memcpy(&v, q, 8);
    return eight_v(v);
  }
  static uint32_t eight_v(uint64_t v) {
    v -= 0x3030303030303030ull;
    v = v * 10 + (v >> 8);
    v = (((v & 0x000000FF000000FFull) * 0x000F424000000064ull) +
         (((v >> 16) & 0x000000FF000000FFull) * 0x0000271000000001ull)) >> 32;
    return (uint32_t)v;
  }
  // the k (1..8) digits ending at e: the eight bytes before e with the
  // leading 8 - k replaced by '0'
  static uint32_t tail8(const uint8_t* e, size_t k) {
    uint64_t v;
    memcpy(&v, e - 8, 8);
    const uint64_t keep = ~0ull << (8 * (8 - k));
    return eight_v((v & keep) | (0x3030303030303030ull & ~keep));
  }
  // length of the digit run at s (eight bytes per step: the first byte whose
  // high nibble is not 3, or whose value + 6 leaves the 0x3_ range, ends it)
  size_t digits(const uint8_t* s) const {
    size_t n = 0;
    while (s + n + 8 <= end) {
      uint64_t v;
      memcpy(&v, s + n, 8);
      const uint64_t a = (v & 0xF0F0F0F0F0F0F0F0ull) ^ 0x3030303030303030ull;
      const uint64_t b = ((v + 0x0606060606060606ull) & 0xF0F0F0F0F0F0F0F0ull) ^ 0x3030303030303030ull;
      const uint64_t m = a | b;
      if (m) return n + (size_t)(__builtin_ctzll(m) >> 3);
      n += 8;
    }
    while (s + n < end && is_digit(s[n])) ++n;
    return n;
  }
  bool u64(uint64_t& v) {
    const uint8_t* s = p;
    if (end - s >= 8) {  // fewer than 8 digits: one load, right-aligned by a shift
      uint64_t w;
      memcpy(&w, s, 8);
      const uint64_t a = (w & 0xF0F0F0F0F0F0F0F0ull) ^ 0x3030303030303030ull;
      const uint64_t b = ((w + 0x0606060606060606ull) & 0xF0F0F0F0F0F0F0F0ull) ^ 0x3030303030303030ull;
      const uint64_t m = a | b;
      if (m) {
        const unsigned n = (unsigned)__builtin_ctzll(m) >> 3;  // digits
        if (n == 0 || (n > 1 && s[0] == '0')) return false;
        const unsigned sh = 8 * (8 - n);  // 8..56
        const uint64_t x = (w << sh) | (0x3030303030303030ull >> (64 - sh));
        v = eight_v(x);
        p = s + n;
        const uint8_t c = *p;  // (n < 8: the terminator is inside the loaded word)
        return !(c == '.' || c == 'e' || c == 'E');
      }
    }
    p += digits(s);
    const size_t n = (size_t)(p - s);
    if (n == 0 || n > 20 || (n > 1 && s[0] == '0')) return false;
    uint64_t r = 0;
    if (s - lo >= 8) {  // (always, after a record's key) right-aligned 8-digit groups, no digit loop
      if (n <= 8) {
        r = tail8(p, n);
      } else if (n <= 16) {
        r = (uint64_t)tail8(p - 8, n - 8) * 100000000ull + eight(p - 8);
      } else {
        const uint64_t hi = tail8(p - 16, n - 16);  // the leading 1..4 digits
        const uint64_t rest = (uint64_t)eight(p - 16) * 100000000ull + eight(p - 8);
        if (hi > 1844 || (hi == 1844 && rest > 6744073709551615ull)) return false;  // beyond uint64
        r = hi * 10000000000000000ull + rest;
      }
    } else {
      if (n == 20 && memcmp(s, "18446744073709551615", 20) > 0) return false;  // beyond uint64
      size_t k = 0;
      for (; k + 8 <= n; k += 8) r = r * 100000000ull + eight(s + k);
      for (; k < n; ++k) r = r * 10 + (uint64_t)(s[k] - '0');
    }
    v = r;
    return !(p < end && (*p == '.' || *p == 'e' || *p == 'E'));
  }
  bool i64(int64_t& v) {
    uint64_t u;
    if (!u64(u) || u > (uint64_t)INT64_MAX) return false;
    v = (int64_t)u;
    return true;
  }
  // "..." of printable ASCII without escapes; s/n = the contents
  bool plain_str(const char*& s, size_t& n) {
    if (!peek('"')) return false;
    const uint8_t* q = ++p;
    while (p < end && *p != '"') {
      if (*p < 0x20 || *p >= 0x80 || *p == '\\') return false;
      ++p;
    }
    if (p >= end) return false;
    s = (const char*)q;
    n = (size_t)(p - q);
    ++p;
    return true;
  }
  // null | "token"
  bool opt_tok(bool& has, const char*& s, size_t& n) {
    if (lit("null")) { has = false; return true; }
    has = true;
    return plain_str(s, n);
  }
};

// One record of the collector's form, decoded (its record hashes appended to
// h.pool at hash_off); fields a record does not carry stay 0, as in Event.
struct FastRec {
  int64_t client_id = 0, op_id = 0;
  uint64_t num_records = 0, msn = 0, hash_off = 0, hash_cnt = 0, tail = 0, stream_hash = 0;
  uint32_t set_tok = 0, batch_tok = 0;
  uint8_t kind = 0, input_type = 0, has_num_records = 0, has_msn = 0;
  uint8_t failure = 0, definite = 0, has_tail = 0, has_hash = 0;
};

// One record at base; returns the bytes consumed (0: not in the collector's
// form; h.pool and h.tokens unchanged).
size_t fast_parse(const uint8_t* base, const uint8_t* end, History& h, FastRec& e) {
  Fast F{base, end, base};
  const size_t pool0 = h.pool.size();
  bool set_has = false, tok_has = false;
  const char *set_s = nullptr, *tok_s = nullptr;
  size_t set_n = 0, tok_n = 0;
  auto undo = [&]() {
    h.pool.resize(pool0);
    return (size_t)0;
  };
  if (!F.lit("{\"event\":{\"")) return undo();
  // the record's kind from the next eight bytes, then its fixed text checked
  // whole (one compare per kind instead of trying the literals in turn)
  const uint64_t k = F.word();
  if (k == word8("Start\":\"")) {
    F.p += 8;
    e.kind = 0;
    if (F.lit("Read\"")) e.input_type = S2LC_INPUT_READ;
    else if (F.lit("CheckTail\"")) e.input_type = S2LC_INPUT_CHECK_TAIL;
    else return undo();
  } else if (k == word8("Start\":{")) {
    F.p += 8;
    e.kind = 0;
    if (!F.lit("\"Append\":{\"num_records\":")) return undo();
    e.input_type = S2LC_INPUT_APPEND;
    e.has_num_records = 1;
    if (!F.u64(e.num_records) || !F.lit(",\"record_hashes\":[")) return undo();
    if (!F.peek(']')) {
      for (;;) {
        uint64_t v;
        if (!F.u64(v)) return undo();
        h.pool.push_back(v);
        if (F.peek(',')) { ++F.p; continue; }
        break;
      }
    }
    if (!F.lit("],\"set_fencing_token\":") || !F.opt_tok(set_has, set_s, set_n)) return undo();
    if (!F.lit(",\"fencing_token\":") || !F.opt_tok(tok_has, tok_s, tok_n)) return undo();
    if (!F.lit(",\"match_seq_num\":")) return undo();
    if (!F.lit("null")) {
      if (!F.u64(e.msn)) return undo();
      e.has_msn = 1;
    }
    if (!F.lit("}}")) return undo();
    e.hash_off = pool0;
    e.hash_cnt = h.pool.size() - pool0;
    if (e.hash_cnt != e.num_records) return undo();  // the general parser reports the mismatch
  } else if (k == word8("Finish\":")) {
    F.p += 8;
    e.kind = 1;
    const uint64_t k2 = F.word();
    if (k2 == word8("\"AppendD")) {
      if (!F.lit("\"AppendDefiniteFailure\"")) return undo();
      e.failure = 1; e.definite = 1;
    } else if (k2 == word8("\"AppendI")) {
      if (!F.lit("\"AppendIndefiniteFailure\"")) return undo();
      e.failure = 1; e.definite = 0;
    } else if (k2 == word8("\"ReadFai")) {
      if (!F.lit("\"ReadFailure\"")) return undo();
      e.failure = 1; e.definite = 1;
    } else if (k2 == word8("\"CheckTa")) {
      if (!F.lit("\"CheckTailFailure\"")) return undo();
      e.failure = 1; e.definite = 1;
    } else {
      e.has_tail = 1;
      if (k2 == word8("{\"Append")) {
        if (!F.lit("{\"AppendSuccess\":{\"tail\":") || !F.u64(e.tail)) return undo();
      } else if (k2 == word8("{\"CheckT")) {
        if (!F.lit("{\"CheckTailSuccess\":{\"tail\":") || !F.u64(e.tail)) return undo();
      } else if (k2 == word8("{\"ReadSu")) {
        e.has_hash = 1;
        if (!F.lit("{\"ReadSuccess\":{\"tail\":") || !F.u64(e.tail) || !F.lit(",\"stream_hash\":") ||
            !F.u64(e.stream_hash))
          return undo();
      } else {
        return undo();
      }
      if (!F.lit("}}")) return undo();
    }
  } else {
    return undo();
  }
  if (!F.lit("},\"client_id\":") || !F.i64(e.client_id) || !F.lit(",\"op_id\":") || !F.i64(e.op_id) ||
      !F.lit("}"))
    return undo();
  // the next byte must end the value (whitespace, end of input, or the next record)
  if (F.p < end && !(*F.p == ' ' || *F.p == '\t' || *F.p == '\n' || *F.p == '\r' || *F.p == '{')) return undo();
  if (set_has) e.set_tok = h.intern(std::string(set_s, set_n));
  if (tok_has) e.batch_tok = h.intern(std::string(tok_s, tok_n));
  return (size_t)(F.p - base);
}

// One record at base appended to h.events; returns the bytes consumed (0: not
// in the collector's form, nothing was changed).
size_t fast_record(const uint8_t* base, const uint8_t* end, History& h) {
  FastRec r;
  const size_t used = fast_parse(base, end, h, r);
  if (!used) return 0;
  Event& e = h.events.emplace_back();
  e.op_id = r.op_id;
  e.client_id = r.client_id;
  e.num_records = r.num_records;
  e.msn = r.msn;
  e.hash_off = r.hash_off;
  e.hash_cnt = r.hash_cnt;
  e.tail = r.tail;
  e.stream_hash = r.stream_hash;
  e.set_tok = r.set_tok;
  e.batch_tok = r.batch_tok;
  e.kind = r.kind;
  e.input_type = r.input_type;
  e.has_num_records = r.has_num_records;
  e.has_msn = r.has_msn;
  e.failure = r.failure;
  e.definite = r.definite;
  e.has_tail = r.has_tail;
  e.has_hash = r.has_hash;
  return used;
}

bool json_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

// The direct decode behind load_jsonl_finalized: the records of the
// collector's form straight into the finalized History, in one pass over the
// bytes. Each op's record (OpRec) is filled in op order, its call fields at
// the Start and its return fields at the Finish, and its chain is chosen at
// the Start: finalize's greedy colouring takes, for op d in call order, the
// chain whose last op returned earliest if that return precedes d's call.
// Every op returned by then precedes the call and every op still open returns
// after it, so the choice needs only the returns seen so far. The records are
// then laid out chain-major with their sentinels and P1 suffix bounds, as
// finalize writes them. Returns false (h left for recycle()) on anything
// else: a record not in the collector's form, op ids out of order, a second
// Start or Finish, an op never returned, more than 2^16 - 1 tokens.
struct DirectScratch {  // load_direct's working arrays, per decoder thread
  std::vector<OpRec> orec;  // per dense op (op-major)
  std::vector<uint32_t> chain_of, chain_len, last, fill;
  std::vector<std::pair<uint32_t, uint32_t>> heap;  // (last return, chain), many chains
};
thread_local DirectScratch direct_scratch;

bool load_direct(const uint8_t* buf, size_t len, History& h) {
  DirectScratch& S = direct_scratch;
  constexpr uint32_t OPEN = EV_INF;  // a chain whose last op has not returned
  std::vector<OpRec>& orec = S.orec;
  std::vector<uint32_t>&chain_of = S.chain_of, &chain_len = S.chain_len, &last = S.last;
  auto& heap = S.heap;
  orec.clear(); chain_of.clear(); chain_len.clear(); last.clear(); heap.clear();
  // (sized for the collector's records, ~107 bytes per event and ~21 per
  // record hash; a history past these grows them as usual)
  orec.reserve(len / 128 + 16);
  h.pool.reserve(h.pool.size() + len / 48 + 16);
  h.lazy_client.reserve(len / 64 + 16);
  bool use_heap = false;
  uint32_t returned = 0;
  const uint8_t* p = buf;
  const uint8_t* const end = buf + len;
  auto gt = std::greater<std::pair<uint32_t, uint32_t>>();
  for (;;) {
    while (p < end && json_ws(*p)) ++p;
    if (p >= end) break;
    __builtin_prefetch(p + 768);  // (~7 records ahead: the input streams from DRAM)
    FastRec r;
    const size_t used = fast_parse(p, end, h, r);
    if (!used) return false;
    p += used;
    const size_t ev = h.lazy_client.size();
    if (ev >= (size_t)EV_INF - 1) return false;
    h.lazy_client.push_back(r.client_id);
    if (r.kind == 0) {
      if (r.op_id != (int64_t)orec.size()) return false;  // dense id = op id (renumber's first appearance)
      const uint32_t d = (uint32_t)orec.size();
      OpRec& o = orec.emplace_back();
      o.num_records = r.num_records;
      o.msn = r.msn;
      o.sufmin = REQ_NONE;
      o.call_ev = (uint32_t)ev;
      o.ret_ev = EV_INF;
      o.hash_off = (uint32_t)r.hash_off;
      o.hash_cnt = (uint32_t)r.hash_cnt;
      o.batch_tok = (uint16_t)r.batch_tok;
      o.set_tok = (uint16_t)r.set_tok;
      o.flags = r.input_type | (r.has_msn ? OPF_HAS_MSN : 0u);  // (the return's bits at the Finish)
      if (r.hash_off > 0xFFFFFFFFull || r.batch_tok > 0xFFFF || r.set_tok > 0xFFFF) return false;
      uint32_t c = EV_INF;
      if (!use_heap) {
        uint32_t best = EV_INF;
        const uint32_t nk = (uint32_t)last.size();
        for (uint32_t k = 0; k < nk; ++k) {  // (branch-free: which chain ended first is data)
          const uint32_t x = last[k];
          const bool lt = x < best;
          best = lt ? x : best;
          c = lt ? k : c;
        }
      } else if (!heap.empty()) {
        std::pop_heap(heap.begin(), heap.end(), gt);
        c = heap.back().second;
        heap.pop_back();
      }
      if (c == EV_INF) {
        c = (uint32_t)chain_len.size();
        chain_len.push_back(0);
        last.push_back(OPEN);
      }
      chain_of.push_back(c);
      chain_len[c]++;
      last[c] = OPEN;
      if (!use_heap && last.size() > 32) {  // many chains: a heap of the returned chain ends (same choices)
        use_heap = true;
        for (uint32_t k = 0; k < (uint32_t)last.size(); ++k)
          if (last[k] != OPEN) heap.emplace_back(last[k], k);
        std::make_heap(heap.begin(), heap.end(), gt);
      }
      (void)d;
    } else {
      if (r.op_id < 0 || r.op_id >= (int64_t)orec.size()) return false;
      const uint32_t d = (uint32_t)r.op_id;
      OpRec& o = orec[d];
      if (o.ret_ev != EV_INF) return false;  // a second Finish: the literal search's case
      o.ret_ev = (uint32_t)ev;
      o.out_tail = r.tail;
      o.out_hash = r.stream_hash;
      o.flags = op_flags((uint8_t)(o.flags & OPF_KIND_MASK), o.flags & OPF_HAS_MSN, r.failure, r.definite, r.has_tail,
                         r.has_hash);
      const uint32_t c = chain_of[d];
      last[c] = (uint32_t)ev;  // (d is its chain's last op: ops join only chains whose last op returned)
      if (use_heap) {
        heap.emplace_back((uint32_t)ev, c);
        std::push_heap(heap.begin(), heap.end(), gt);
      }
      returned++;
    }
  }
  const uint32_t m = (uint32_t)orec.size();
  if (returned != m || h.tokens.size() > 0xFFFF || h.pool.size() > 0xFFFFFFFFull) return false;
  // finalize's state (history.cpp), from the op-major records
  h.status = 0;
  h.error.clear();
  h.structural = 0;
  h.literal = false;
  h.lit_id.clear();
  h.lit_match.clear();
  h.n_ops = m;
  h.op_ids.resize(m);
  h.op_call.resize(m);
  h.op_ret.resize(m);
  uint64_t total = 0;
  bool nowrap = true;
  for (uint32_t d = 0; d < m; ++d) {
    const OpRec& o = orec[d];
    h.op_ids[d] = d;
    h.op_call[d] = o.call_ev;
    h.op_ret[d] = o.ret_ev;
    if ((o.flags & OPF_KIND_MASK) != S2LC_INPUT_APPEND) continue;
    if (o.num_records > (1ull << 63) - total) nowrap = false;
    else total += o.num_records;
  }
  // (a zero-record append carrying hashes is not in the collector's form:
  // hash_cnt == num_records there)
  h.hflags = H_P4 | H_IDEFER;
  if (nowrap) h.hflags |= H_NOWRAP | H_P2OK;
  if (nowrap && total <= 0xFFFFFFFCull) h.hflags |= H_TAIL32;
  const uint32_t K = (uint32_t)chain_len.size();
  h.K = K;
  h.chain_start.resize(K + 1);
  h.max_chain_len = 0;
  uint32_t pos = 0;
  for (uint32_t c = 0; c < K; ++c) {
    h.chain_start[c] = pos;
    pos += chain_len[c] + 1;
    h.max_chain_len = std::max<uint32_t>(h.max_chain_len, chain_len[c]);
  }
  h.chain_start[K] = pos;
  h.rec_op.assign(pos, EV_INF);
  h.op_rec.resize(m);
  std::vector<uint32_t>& fill = S.fill;
  fill.assign(h.chain_start.begin(), h.chain_start.end() - 1);
  for (uint32_t d = 0; d < m; ++d) {  // call order within every chain
    const uint32_t q = fill[chain_of[d]]++;
    h.rec_op[q] = d;
    h.op_rec[d] = q;
  }
  // the records in position order, each written once
  h.recs.clear();
  h.recs.reserve(pos);
  uint32_t n_ident = 0;
  for (uint32_t q = 0; q < pos; ++q) {
    const uint32_t d = h.rec_op[q];
    if (d == EV_INF) {
      h.recs.push_back(OpRec{});
      continue;
    }
    h.recs.push_back(orec[d]);
    if (orec[d].flags & OPF_CLS_E) n_ident++;
  }
  h.n_ident = n_ident;
  for (uint32_t c = 0; c < K; ++c) {
    const uint32_t q = h.chain_start[c + 1] - 1;
    OpRec& s = h.recs[q];  // sentinel
    s.call_ev = EV_INF;
    s.ret_ev = EV_INF;
    s.flags = OPF_SENTINEL;
    s.sufmin = REQ_NONE;
    uint64_t run = REQ_NONE;  // suffix minimum of the pre-tail each constraining op requires
    for (uint32_t x = q; x-- > h.chain_start[c];) {
      OpRec& o = h.recs[x];
      if (o.flags & OPF_CONSTRAIN) {
        uint64_t req;
        if ((o.flags & OPF_KIND_MASK) == S2LC_INPUT_APPEND)
          req = o.out_tail >= o.num_records ? o.out_tail - o.num_records : 0;  // 0: unsatisfiable
        else if (!(o.flags & OPF_FAIL))
          req = o.out_tail;
        else
          req = REQ_HASH_ONLY;
        if (req > REQ_HASH_ONLY) req = REQ_HASH_ONLY;
        run = std::min(run, req);
      }
      o.sufmin = run;
    }
  }
  h.events.clear();
  h.lazy_once = std::make_unique<std::once_flag>();
  return true;
}

}  // namespace

int load_jsonl(const uint8_t* buf, size_t len, History& h, std::string& err) {
  Parser P;
  P.base = buf;
  P.p = buf;
  P.end = buf + len;
  std::vector<uint64_t> hashes;
  const bool fast = getenv("S2LC_JSONL_GENERAL") == nullptr;  // tests: the general parser only
  {
    // size the event / hash arrays once (a record per line in the collector's
    // output): growing them record by record re-maps large blocks, which
    // serialises parallel decoders on the process's address-space lock. The
    // bound is the shortest record's length (a Finish without a value, ~60
    // bytes): counting the lines instead cost a quarter of the decode
    // (memchr per ~107-byte record), and untouched capacity is never faulted in.
    h.events.reserve(h.events.size() + len / 56 + 16);
    h.pool.reserve(h.pool.size() + len / 24);
  }
  while (true) {
    P.ws();
    if (P.p >= P.end) return 0;  // io.EOF
    if (fast) {
      __builtin_prefetch(P.p + 768);
      const size_t used = fast_record(P.p, P.end, h);
      if (used) {
        P.p += used;
        continue;
      }
    }
    const size_t rec_off = (size_t)(P.p - buf);
    P.reset();
    uint32_t root;
    if (!P.value(root)) {
      err = "decode record at byte offset " + std::to_string((size_t)(P.p - buf)) + ": " + P.err;
      return S2LC_EDECODE;
    }
    Dec D(P);
    const JNode& r = P.nodes[root];
    // Record{Event EventWrapper; ClientID int; OpID int} (main.go:190-194)
    bool has_start = false, has_finish = false;
    Event se, fe;       // accumulated Start / Finish across duplicate "event" keys
    bool se_append = false;
    std::vector<uint64_t> se_hashes;
    int64_t client = 0, op = 0;
    bool ok = true;
    if (r.t == J_OBJ) {
      for (uint32_t k = 0; k < r.b && ok; ++k) {
        const std::string& key = P.strs[P.kids[r.a + 2 * k]];
        uint32_t v = P.kids[r.a + 2 * k + 1];
        if (Dec::fold_eq(key, "event")) {
          // EventWrapper.UnmarshalJSON (main.go:163-188), called even for null
          const JNode& ev = P.nodes[v];
          if (ev.t != J_OBJ && ev.t != J_NULL) { ok = D.type_err(v, "map[string]json.RawMessage"); break; }
          if (ev.t == J_OBJ) {
            int64_t s = D.map_get(v, "Start");
            if (s >= 0) {
              Event tmp;
              bool app = false;
              std::vector<uint64_t> hs;
              if (!D.start((uint32_t)s, tmp, h, hs, app)) { ok = false; break; }
              se = tmp; se_append = app; se_hashes.swap(hs);
              has_start = true;
            }
            int64_t f = D.map_get(v, "Finish");
            if (f >= 0) {
              Event tmp;
              if (!D.finish((uint32_t)f, tmp)) { ok = false; break; }
              fe = tmp;
              has_finish = true;
            }
          }
          if (has_start == has_finish) {
            D.err = std::string("expected exactly one of Start/Finish, got Start=") + (has_start ? "true" : "false") +
                    " Finish=" + (has_finish ? "true" : "false");
            ok = false;
          }
        } else if (Dec::fold_eq(key, "client_id")) {
          ok = D.i64(v, client);
        } else if (Dec::fold_eq(key, "op_id")) {
          ok = D.i64(v, op);
        }
      }
    } else if (r.t != J_NULL) {
      ok = D.type_err(root, "main.Record");
    }
    if (!ok) {
      err = "decode record at byte offset " + std::to_string((size_t)(P.p - buf)) + ": " + D.err;
      return S2LC_EDECODE;
    }
    Event e;
    if (has_start) {
      e = se;
      e.kind = 0;
      if (se_append) {
        e.hash_off = h.pool.size();
        e.hash_cnt = se_hashes.size();
        h.pool.insert(h.pool.end(), se_hashes.begin(), se_hashes.end());
      }
    } else if (has_finish) {
      e = fe;
      e.kind = 1;
    } else {
      err = "record at byte offset " + std::to_string(rec_off) + " has neither Start nor Finish event";
      return S2LC_EDECODE;
    }
    e.op_id = op;
    e.client_id = client;
    h.events.push_back(e);
  }
}

void load_scratch_trim() { direct_scratch = DirectScratch(); }

int load_jsonl_finalized(const uint8_t* buf, size_t len, History& h, std::string& err) {
  const char* e = getenv("S2LC_JSONL_DIRECT");  // 0: always the event list + finalize (tests compare the two)
  if (!(e && *e == '0') && getenv("S2LC_JSONL_GENERAL") == nullptr) {
    if (load_direct(buf, len, h)) return 0;
    h.recycle();
  }
  int rc = load_jsonl(buf, len, h, err);
  if (rc) return rc;
  rc = h.finalize();
  if (rc) err = h.error;
  return rc;
}

}  // namespace s2lc
