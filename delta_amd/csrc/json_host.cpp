#include "json_host.h"

#include <cstring>

namespace dr {
namespace {

struct P {
  const char* p;
  const char* e;
  std::string err;
  void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n')) ++p; }
  bool fail(const char* m) { if (err.empty()) err = m; return false; }
  static void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) o += char(cp);
    else if (cp < 0x800) { o += char(0xC0 | (cp >> 6)); o += char(0x80 | (cp & 63)); }
    else if (cp < 0x10000) { o += char(0xE0 | (cp >> 12)); o += char(0x80 | ((cp >> 6) & 63)); o += char(0x80 | (cp & 63)); }
    else { o += char(0xF0 | (cp >> 18)); o += char(0x80 | ((cp >> 12) & 63)); o += char(0x80 | ((cp >> 6) & 63)); o += char(0x80 | (cp & 63)); }
  }
  bool hex4(uint32_t* v) {
    if (e - p < 4) return fail("bad \\u escape");
    *v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p++;
      int d = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10 : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : -1;
      if (d < 0) return fail("bad hex digit");
      *v = *v * 16 + uint32_t(d);
    }
    return true;
  }
  bool str(std::string& o) {
    if (p >= e || *p != '"') return fail("expected string");
    ++p;
    while (p < e) {
      char c = *p++;
      if (c == '"') return true;
      if (c != '\\') { o += c; continue; }
      if (p >= e) return fail("bad escape");
      char x = *p++;
      switch (x) {
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          uint32_t cp;
          if (!hex4(&cp)) return false;
          if (cp >= 0xD800 && cp < 0xDC00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            const char* save = p;
            p += 2;
            uint32_t lo;
            if (hex4(&lo) && lo >= 0xDC00 && lo < 0xE000) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            else p = save;
          }
          put_utf8(o, cp);
          break;
        }
        default: o += x; break;
      }
    }
    return fail("unterminated string");
  }
  bool val(JVal& v, int depth) {
    if (depth > 256) return fail("nesting too deep");
    ws();
    if (p >= e) return fail("unexpected end");
    char c = *p;
    if (c == '{') {
      ++p;
      v.t = JVal::OBJ;
      ws();
      if (p < e && *p == '}') { ++p; return true; }
      for (;;) {
        ws();
        std::string k;
        if (!str(k)) return false;
        ws();
        if (p >= e || *p != ':') return fail("expected ':'");
        ++p;
        v.o.emplace_back(std::move(k), JVal());
        if (!val(v.o.back().second, depth + 1)) return false;
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == '}') { ++p; return true; }
        return fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++p;
      v.t = JVal::ARR;
      ws();
      if (p < e && *p == ']') { ++p; return true; }
      for (;;) {
        v.a.emplace_back();
        if (!val(v.a.back(), depth + 1)) return false;
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == ']') { ++p; return true; }
        return fail("expected ',' or ']'");
      }
    }
    if (c == '"') { v.t = JVal::STR; return str(v.s); }
    if (c == 't' && e - p >= 4 && !memcmp(p, "true", 4)) { v.t = JVal::BOOL; v.b = true; p += 4; return true; }
    if (c == 'f' && e - p >= 5 && !memcmp(p, "false", 5)) { v.t = JVal::BOOL; v.b = false; p += 5; return true; }
    if (c == 'n' && e - p >= 4 && !memcmp(p, "null", 4)) { v.t = JVal::NUL; p += 4; return true; }
    const char* b = p;
    while (p < e && (strchr("0123456789+-.eE", *p) != nullptr)) ++p;
    if (p == b) return fail("unexpected character");
    v.t = JVal::NUM;
    v.s.assign(b, p);
    return true;
  }
};

}  // namespace

bool JVal::is_int() const {
  if (t != NUM || s.empty()) return false;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (!(c >= '0' && c <= '9') && !(i == 0 && c == '-')) return false;
  }
  try {  // a long: out of range is not one (the device decoders agree)
    (void)std::stoll(s);
  } catch (...) {
    return false;
  }
  return true;
}

int64_t JVal::as_int() const { return is_int() ? std::stoll(s) : 0; }

bool json_parse(const char* p, size_t n, JVal* out, std::string* err) {
  P ps{p, p + n, {}};
  *out = JVal();
  bool ok = ps.val(*out, 0);
  if (ok) {
    ps.ws();
    if (ps.p != ps.e) ok = ps.fail("trailing characters");
  }
  if (!ok && err) *err = ps.err;
  return ok;
}

std::string json_quote(const std::string& s) {
  std::string o = "\"";
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      case '\b': o += "\\b"; break;
      case '\f': o += "\\f"; break;
      default:
        if (c < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); o += b; }
        else o += char(c);
    }
  }
  return o + "\"";
}

std::string json_dump(const JVal& v) {
  switch (v.t) {
    case JVal::NUL: return "null";
    case JVal::BOOL: return v.b ? "true" : "false";
    case JVal::NUM: return v.s;
    case JVal::STR: return json_quote(v.s);
    case JVal::ARR: {
      std::string o = "[";
      for (size_t i = 0; i < v.a.size(); ++i) { if (i) o += ","; o += json_dump(v.a[i]); }
      return o + "]";
    }
    case JVal::OBJ: {
      std::string o = "{";
      for (size_t i = 0; i < v.o.size(); ++i) {
        if (i) o += ",";
        o += json_quote(v.o[i].first) + ":" + json_dump(v.o[i].second);
      }
      return o + "}";
    }
  }
  return "null";
}

}  // namespace dr
