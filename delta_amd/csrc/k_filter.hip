// K5: partition pruning over the resident live AddFiles -- DeltaLog.filterFileList with the
// filters rewritten by rewritePartitionFilters (D/DeltaLog.scala:500-547): every partition column
// reference becomes Cast(partitionValues[col] AS partitionSchema(col).type), the conjuncts are
// ANDed, and a file is kept where the predicate is TRUE (three-valued logic; NULL drops it).
//
// k_pv_extract (once per state and partition column, cached on the state): one thread per live
// file locates the file's partition values -- in its JSON line (`add.partitionValues` object,
// resident in d_json) or in the checkpoint's decoded `add.partitionValues` map column (entries of
// its row) -- and casts them with Spark 3.1's non-ANSI Cast(string AS type) as restated by the
// oracle (oracle/delta_oracle.py:cast_string) into typed columns.
// k_filter_typed (per dr_filter): one thread per live file runs the postfix predicate program
// (include/deltareplay.h, dr_pred_op) over the typed columns.
#include "dev_common.h"
#include "kernels.h"
#include "../../include/deltareplay.h"
#include <hipcub/device/device_merge_sort.hpp>

namespace dr {
namespace dev {

enum PvState : uint8_t { PV_NULL = 0, PV_RAW = 1, PV_ESCAPED = 2 };

// ---- minimal JSON walking over one line -------------------------------------------------------------
__device__ __forceinline__ bool is_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
__device__ __forceinline__ const uint8_t* skip_ws(const uint8_t* p, const uint8_t* e) {
  while (p < e && is_ws(*p)) ++p;
  return p;
}
// p points after an opening quote; returns the closing quote (or e)
__device__ const uint8_t* str_close(const uint8_t* p, const uint8_t* e, bool* esc) {
  while (p < e) {
    const uint8_t c = *p;
    if (c == '"') return p;
    if (c == '\\') { *esc = true; p += 2; continue; }
    ++p;
  }
  return e;
}
// skips one JSON value starting at p (after whitespace); returns the position after it
__device__ const uint8_t* skip_value(const uint8_t* p, const uint8_t* e) {
  if (p >= e) return e;
  if (*p == '"') {
    bool esc = false;
    const uint8_t* q = str_close(p + 1, e, &esc);
    return q < e ? q + 1 : e;
  }
  if (*p == '{' || *p == '[') {
    int depth = 0;
    while (p < e) {
      const uint8_t c = *p;
      if (c == '"') {
        bool esc = false;
        const uint8_t* q = str_close(p + 1, e, &esc);
        p = q < e ? q + 1 : e;
        continue;
      }
      if (c == '{' || c == '[') ++depth;
      else if (c == '}' || c == ']') {
        if (--depth == 0) return p + 1;
      }
      ++p;
    }
    return e;
  }
  while (p < e && *p != ',' && *p != '}' && *p != ']' && !is_ws(*p)) ++p;
  return p;
}

// JSON string span (raw, maybe escaped) == target bytes
__device__ bool span_eq(const uint8_t* s, uint32_t n, bool esc, const uint8_t* t, uint32_t tn) {
  if (!esc) {
    if (n != tn) return false;
    for (uint32_t k = 0; k < n; ++k)
      if (s[k] != t[k]) return false;
    return true;
  }
  if (n > 128) return false;
  uint8_t buf[160];
  const uint32_t m = json_unescape(s, n, buf);
  if (m != tn) return false;
  for (uint32_t k = 0; k < m; ++k)
    if (buf[k] != t[k]) return false;
  return true;
}

__device__ __forceinline__ bool key_is(const uint8_t* s, uint32_t n, bool esc, const char* lit, uint32_t ln) {
  return span_eq(s, n, esc, reinterpret_cast<const uint8_t*>(lit), ln);
}

// Iterates the members of the object starting at p ('{'); f(key, klen, kesc, value_start) returns
// the position after the value. Returns false on malformed input.
template <typename F>
__device__ __forceinline__ bool each_member(const uint8_t* p, const uint8_t* e, F&& f) {
  if (p >= e || *p != '{') return false;
  ++p;
  while (true) {
    p = skip_ws(p, e);
    if (p >= e) return false;
    if (*p == '}') return true;
    if (*p == ',') { ++p; continue; }
    if (*p != '"') return false;
    bool kesc = false;
    const uint8_t* k0 = p + 1;
    const uint8_t* k1 = str_close(k0, e, &kesc);
    if (k1 >= e) return false;
    p = skip_ws(k1 + 1, e);
    if (p >= e || *p != ':') return false;
    p = skip_ws(p + 1, e);
    p = f(k0, uint32_t(k1 - k0), kesc, p);
    if (p == nullptr) return false;
  }
}

// ---- casts: Cast(string AS type), non-ANSI (failure -> NULL) ----------------------------------------
struct SV {
  int64_t v;
  const uint8_t* s;
  uint32_t n;
  uint8_t null, str;
};

__device__ __forceinline__ bool cast_ws(uint8_t c) {  // UTF8String.trim-like set of the restatement
  return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == 0x0b || c == 0x0c;
}

__device__ bool parse_int(const uint8_t* s, uint32_t n, int type, int64_t* out) {
  uint32_t i = 0;
  while (i < n && cast_ws(s[i])) ++i;
  while (n > i && cast_ws(s[n - 1])) --n;
  if (i >= n) return false;
  bool neg = false;
  if (s[i] == '+' || s[i] == '-') { neg = s[i] == '-'; ++i; }
  if (i >= n) return false;
  uint64_t acc = 0;
  for (; i < n; ++i) {
    const uint8_t c = s[i];
    if (c < '0' || c > '9') return false;
    const uint64_t d = c - '0';
    if (acc > (~0ull - d) / 10) return false;  // beyond 64 bits: out of every range
    acc = acc * 10 + d;
  }
  uint64_t lim_pos, lim_neg;  // |min|, max
  switch (type) {
    case DR_T_BYTE: lim_pos = 127; lim_neg = 128; break;
    case DR_T_SHORT: lim_pos = 32767; lim_neg = 32768; break;
    case DR_T_INT: lim_pos = 2147483647ull; lim_neg = 2147483648ull; break;
    default: lim_pos = 9223372036854775807ull; lim_neg = 9223372036854775808ull; break;
  }
  if (neg ? acc > lim_neg : acc > lim_pos) return false;
  *out = neg ? int64_t(0 - acc) : int64_t(acc);
  return true;
}

__device__ __forceinline__ uint8_t lower(uint8_t c) { return (c >= 'A' && c <= 'Z') ? uint8_t(c + 32) : c; }

__device__ bool parse_bool(const uint8_t* s, uint32_t n, int64_t* out) {
  uint32_t i = 0;
  while (i < n && cast_ws(s[i])) ++i;
  while (n > i && cast_ws(s[n - 1])) --n;
  const uint32_t m = n - i;
  uint8_t b[5] = {0, 0, 0, 0, 0};
  if (m == 0 || m > 5) return false;
  for (uint32_t k = 0; k < m; ++k) b[k] = lower(s[i + k]);
  auto is = [&](const char* w, uint32_t wl) {
    if (wl != m) return false;
    for (uint32_t k = 0; k < wl; ++k)
      if (b[k] != uint8_t(w[k])) return false;
    return true;
  };
  if (is("t", 1) || is("true", 4) || is("y", 1) || is("yes", 3) || is("1", 1)) { *out = 1; return true; }
  if (is("f", 1) || is("false", 5) || is("n", 1) || is("no", 2) || is("0", 1)) { *out = 0; return true; }
  return false;
}

__device__ __forceinline__ int64_t days_from_civil(int64_t y, int64_t m, int64_t d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const int64_t yoe = y - era * 400;
  const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}

// yyyy[-m[m][-d[d]][( |T)...]] after trimming (oracle/delta_oracle.py:cast_string "date")
__device__ bool parse_date(const uint8_t* s, uint32_t n, int64_t* out) {
  uint32_t i = 0;
  while (i < n && cast_ws(s[i])) ++i;
  while (n > i && cast_ws(s[n - 1])) --n;
  auto digit = [&](uint32_t k) { return k < n && s[k] >= '0' && s[k] <= '9'; };
  if (n - i < 4) return false;
  int64_t y = 0;
  for (int k = 0; k < 4; ++k) {
    if (!digit(i)) return false;
    y = y * 10 + (s[i++] - '0');
  }
  int64_t mo = 1, d = 1;
  if (i < n) {
    if (s[i] != '-') return false;
    ++i;
    if (!digit(i)) return false;
    mo = s[i++] - '0';
    if (digit(i)) mo = mo * 10 + (s[i++] - '0');
    if (i < n) {
      if (s[i] != '-') return false;
      ++i;
      if (!digit(i)) return false;
      d = s[i++] - '0';
      if (digit(i)) d = d * 10 + (s[i++] - '0');
      if (i < n && s[i] != ' ' && s[i] != 'T') return false;
    }
  }
  if (mo < 1 || mo > 12 || d < 1) return false;
  const bool leap = (y % 4 == 0 && y % 100 != 0) || y % 400 == 0;
  const int mdays[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  const int64_t dim = mdays[mo - 1] + (mo == 2 && leap ? 1 : 0);
  if (d > dim) return false;
  *out = days_from_civil(y, mo, d);
  return true;
}

// ---- casts of partitionValues_parsed's other types (D/Checkpoints.scala:380-388: Cast(pv AS type)) --
// float / double, decimal(p, s), timestamp and binary partition columns. The K5 predicate program
// does not take them (check_program); the checkpoint writer does.
__device__ __forceinline__ bool jws(uint8_t c) { return c <= ' '; }  // String.trim / UTF8String.trimAll

// Double.parseDouble / Float.parseFloat of the trimmed text (Java's FloatingDecimal grammar: sign,
// NaN, Infinity, digits with one '.', exponent, an f/F/d/D suffix), else Spark's special literals
// (Cast.processFloatingPointSpecialLiterals: inf, +inf, infinity, +infinity, -inf, -infinity, nan,
// any case). Exact here on Clinger's fast path (<= 19 significant digits; double: mantissa <= 2^53,
// |10-exponent| <= 22; float: <= 2^24, <= 10); other well-formed numbers (and hex) come back
// FP_HARD and the host converts them with its correctly rounded strtod / strtof.
enum FpRes : int { FP_NULL = 0, FP_OK = 1, FP_HARD = 2 };
__device__ int parse_fp(const uint8_t* s, uint32_t n, bool is_float, uint64_t* bits) {
  uint32_t i = 0;
  while (i < n && jws(s[i])) ++i;
  while (n > i && jws(s[n - 1])) --n;
  const uint32_t b0 = i;
  bool neg = false;
  auto special = [&]() -> int {
    char t[10];
    const uint32_t m = n - b0;
    if (m == 0 || m > 9) return FP_NULL;
    for (uint32_t k = 0; k < m; ++k) t[k] = char(lower(s[b0 + k]));
    auto is = [&](const char* w) {
      uint32_t k = 0;
      for (; w[k]; ++k)
        if (k >= m || t[k] != w[k]) return false;
      return k == m;
    };
    int sign = 0;
    if (is("inf") || is("+inf") || is("infinity") || is("+infinity")) sign = 1;
    else if (is("-inf") || is("-infinity")) sign = -1;
    else if (is("nan")) {
      *bits = is_float ? 0x7fc00000ull : 0x7ff8000000000000ull;
      return FP_OK;
    } else return FP_NULL;
    *bits = is_float ? (sign > 0 ? 0x7f800000ull : 0xff800000ull) : (sign > 0 ? 0x7ff0000000000000ull : 0xfff0000000000000ull);
    return FP_OK;
  };
  if (i >= n) return FP_NULL;
  if (s[i] == '+' || s[i] == '-') { neg = s[i] == '-'; ++i; }
  auto word = [&](const char* w, uint32_t wl) {
    if (n - i != wl) return false;
    for (uint32_t k = 0; k < wl; ++k)
      if (s[i + k] != uint8_t(w[k])) return false;
    return true;
  };
  if (word("NaN", 3)) { *bits = is_float ? 0x7fc00000ull : 0x7ff8000000000000ull; return FP_OK; }
  if (word("Infinity", 8)) {
    *bits = is_float ? (neg ? 0xff800000ull : 0x7f800000ull) : (neg ? 0xfff0000000000000ull : 0x7ff0000000000000ull);
    return FP_OK;
  }
  if (i + 1 < n && s[i] == '0' && (s[i + 1] | 0x20) == 'x') return FP_HARD;  // hexadecimal significand
  uint64_t w = 0;
  int32_t sig = 0, dexp = 0;
  bool any = false, dot = false, trunc = false;
  for (; i < n; ++i) {
    const uint8_t c = s[i];
    if (c == '.') {
      if (dot) return special();
      dot = true;
      continue;
    }
    if (c < '0' || c > '9') break;
    any = true;
    if (w == 0 && c == '0') {  // leading zero
      if (dot) --dexp;
      continue;
    }
    if (sig < 19) {
      w = w * 10 + (c - '0');
      ++sig;
      if (dot) --dexp;
    } else {
      trunc = trunc || c != '0';
      if (!dot) ++dexp;
    }
  }
  if (!any) return special();
  if (i < n && (s[i] == 'e' || s[i] == 'E')) {
    ++i;
    bool eneg = false;
    if (i < n && (s[i] == '+' || s[i] == '-')) { eneg = s[i] == '-'; ++i; }
    if (i >= n || s[i] < '0' || s[i] > '9') return special();
    int64_t e = 0;
    for (; i < n && s[i] >= '0' && s[i] <= '9'; ++i) e = e < 100000 ? e * 10 + (s[i] - '0') : e;
    dexp += int32_t(eneg ? -e : e);
  }
  if (i < n && (s[i] == 'f' || s[i] == 'F' || s[i] == 'd' || s[i] == 'D')) ++i;
  if (i != n) return special();
  if (w == 0) {  // a signed zero
    *bits = is_float ? (neg ? 0x80000000ull : 0ull) : (neg ? 0x8000000000000000ull : 0ull);
    return FP_OK;
  }
  if (trunc) return FP_HARD;
  const double p10[23] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11,
                          1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  if (is_float) {
    if (w > (1ull << 24) || dexp < -10 || dexp > 10) return FP_HARD;
    const float m = float(w), q = float(p10[dexp < 0 ? -dexp : dexp]);
    float f = dexp < 0 ? __fdiv_rn(m, q) : __fmul_rn(m, q);
    if (neg) f = -f;
    *bits = __float_as_uint(f);
    return FP_OK;
  }
  if (w > (1ull << 53) || dexp < -22 || dexp > 22) return FP_HARD;
  const double m = double(w), q = p10[dexp < 0 ? -dexp : dexp];
  double d = dexp < 0 ? __ddiv_rn(m, q) : __dmul_rn(m, q);
  if (neg) d = -d;
  *bits = uint64_t(__double_as_longlong(d));
  return FP_OK;
}

// Decimal.fromString + changePrecision(p, s) (non-ANSI): java.math.BigDecimal of the trimmed text
// ([sign] digits [. digits] [e|E [sign] digits]), rounded HALF_UP to `scale`; null when the unscaled
// value needs more than `prec` digits. Two's complement unscaled value in lo / hi (128 bits).
__device__ bool parse_decimal(const uint8_t* s, uint32_t n, int prec, int scale, uint64_t* lo, int64_t* hi) {
  uint32_t i = 0;
  while (i < n && jws(s[i])) ++i;
  while (n > i && jws(s[n - 1])) --n;
  if (i >= n) return false;
  bool neg = false;
  if (s[i] == '+' || s[i] == '-') { neg = s[i] == '-'; ++i; }
  const uint32_t d0 = i;
  uint32_t ndig = 0, frac = 0;
  bool dot = false;
  for (; i < n; ++i) {
    if (s[i] == '.') {
      if (dot) return false;
      dot = true;
      continue;
    }
    if (s[i] < '0' || s[i] > '9') break;
    ++ndig;
    if (dot) ++frac;
  }
  if (!ndig) return false;
  const uint32_t d1 = i;  // digits (and the '.') in [d0, d1)
  int64_t e = 0;
  if (i < n && (s[i] == 'e' || s[i] == 'E')) {
    ++i;
    bool eneg = false;
    if (i < n && (s[i] == '+' || s[i] == '-')) { eneg = s[i] == '-'; ++i; }
    if (i >= n || s[i] < '0' || s[i] > '9') return false;
    for (; i < n && s[i] >= '0' && s[i] <= '9'; ++i) {
      e = e * 10 + (s[i] - '0');
      if (e > 4000000000ll) return false;  // beyond BigDecimal's int scale
    }
    if (eneg) e = -e;
  }
  if (i != n) return false;
  // value = digits * 10^(e - frac); unscaled = digits * 10^(e - frac + scale)
  const int64_t shift = e - int64_t(frac) + scale;
  const int64_t keep = int64_t(ndig) + (shift < 0 ? shift : 0);  // digits kept before rounding
  unsigned __int128 v = 0;
  int64_t k = 0;
  uint32_t round_digit = 0;
  bool big = false;
  for (uint32_t j = d0; j < d1; ++j) {
    if (s[j] == '.') continue;
    const uint32_t dg = s[j] - '0';
    if (k < keep) {
      if (v != 0 || dg != 0) {
        if (v > (~(unsigned __int128)0) / 10 - 10) big = true;
        else v = v * 10 + dg;
      }
    } else if (k == keep) {
      round_digit = dg;
    }
    ++k;
  }
  if (big) return false;
  if (shift > 0) {
    for (int64_t t = 0; t < shift; ++t) {
      if (v > (~(unsigned __int128)0) / 10) return false;
      v *= 10;
      if (v == 0) break;
    }
  }
  if (round_digit >= 5) v += 1;  // ROUND_HALF_UP on the magnitude
  unsigned __int128 lim = 1;
  for (int t = 0; t < prec; ++t) lim *= 10;
  if (v >= lim) return false;
  const unsigned __int128 r = neg ? (unsigned __int128)0 - v : v;
  *lo = uint64_t(r);
  *hi = int64_t(uint64_t(r >> 64));
  return true;
}

// DateTimeUtils.stringToTimestamp (Spark 3.1) with the session time zone UTC: [+-]yyyy[y..][-[m]m
// [-[d]d[( |T)[h]h:[m]m[:[s]s[.fraction]][zone]]]], fraction truncated to microseconds, zone Z / UTC /
// UT / GMT with an optional [+-]h[h][[:]mm[[:]ss]] offset, or a bare offset. Time-only strings (today's
// date) and region zone ids (daylight saving rules) read as null here: parity unpinned.
__device__ bool tz_offset(const uint8_t* z, uint32_t n, int64_t* secs) {
  uint32_t i = 0;
  while (i < n && jws(z[i])) ++i;
  while (n > i && jws(z[n - 1])) --n;
  auto pre = [&](const char* w, uint32_t wl) {
    if (n - i < wl) return false;
    for (uint32_t k = 0; k < wl; ++k)
      if (z[i + k] != uint8_t(w[k])) return false;
    return true;
  };
  if (n - i == 1 && z[i] == 'Z') { *secs = 0; return true; }
  if (pre("UTC", 3)) i += 3;
  else if (pre("GMT", 3)) i += 3;
  else if (pre("UT", 2)) i += 2;
  else if (i >= n || (z[i] != '+' && z[i] != '-')) return false;
  if (i == n) { *secs = 0; return true; }
  if (z[i] != '+' && z[i] != '-') return false;
  const bool neg = z[i] == '-';
  ++i;
  int f[3] = {0, 0, 0}, nf = 0;
  while (i < n && nf < 3) {
    int dg = 0, v = 0;
    while (i < n && z[i] >= '0' && z[i] <= '9' && dg < 2) { v = v * 10 + (z[i] - '0'); ++i; ++dg; }
    if (dg == 0) return false;
    f[nf++] = v;
    if (i < n && z[i] == ':') ++i;
  }
  if (i != n || f[0] > 18 || f[1] > 59 || f[2] > 59) return false;
  const int64_t t = int64_t(f[0]) * 3600 + f[1] * 60 + f[2];
  *secs = neg ? -t : t;
  return true;
}

__device__ bool parse_timestamp(const uint8_t* s, uint32_t n, int64_t* micros) {
  uint32_t j = 0;
  while (j < n && jws(s[j])) ++j;
  while (n > j && jws(s[n - 1])) --n;
  if (j >= n) return false;
  int64_t seg[9] = {1, 1, 1, 0, 0, 0, 0, 0, 0};
  int i = 0, digits = 0, milli_digits = 0, sign = 1;
  int64_t cur = 0;
  bool just_time = false;
  int32_t tz0 = -1;
  auto valid = [&](int sg, int d) {
    return sg == 6 || (sg == 0 && d >= 4 && d <= 6) || (sg == 7 && d <= 2) ||
           (sg != 0 && sg != 6 && sg != 7 && d > 0 && d <= 2);
  };
  const uint32_t start = j;
  if (s[j] == '-' || s[j] == '+') { sign = s[j] == '-' ? -1 : 1; ++j; }
  const bool signed_year = j > start;
  for (; j < n; ++j) {
    const uint8_t b = s[j];
    if (b < '0' || b > '9') {
      if (j == start && b == 'T') {
        just_time = true;
        i += 3;
      } else if (i < 2) {
        if (b == '-') {
          if (!valid(i, digits)) return false;
          seg[i++] = cur; cur = 0; digits = 0;
        } else if (i == 0 && b == ':' && !signed_year) {
          just_time = true;
          if (!valid(3, digits)) return false;
          seg[3] = cur; cur = 0; digits = 0;
          i = 4;
        } else return false;
      } else if (i == 2) {
        if (b != ' ' && b != 'T') return false;
        if (!valid(i, digits)) return false;
        seg[i++] = cur; cur = 0; digits = 0;
      } else if (i == 3 || i == 4) {
        if (b != ':') return false;
        if (!valid(i, digits)) return false;
        seg[i++] = cur; cur = 0; digits = 0;
      } else if (i == 5 || i == 6) {
        if (!valid(i, digits)) return false;
        seg[i] = cur; cur = 0; digits = 0;
        if (b == '.' && i == 5) {
          ++i;
        } else {
          ++i;
          tz0 = int32_t(j);
          j = n - 1;
        }
        if (i == 6 && b != '.') ++i;
      } else {
        if (i < 9 && (b == ':' || b == ' ')) {
          if (!valid(i, digits)) return false;
          seg[i++] = cur; cur = 0; digits = 0;
        } else return false;
      }
    } else {
      if (i == 6) ++milli_digits;
      if (i != 6 || digits < 6) cur = cur * 10 + (b - '0');
      if (cur > 100000000000ll) return false;
      ++digits;
    }
  }
  if (!valid(i, digits)) return false;
  if (i > 8) return false;
  seg[i] = cur;
  while (milli_digits < 6) { seg[6] *= 10; ++milli_digits; }
  if (just_time) return false;  // LocalDate.now(zone): not a function of the value
  int64_t off = 0;
  if (tz0 >= 0 && !tz_offset(s + tz0, n - uint32_t(tz0), &off)) return false;
  const int64_t y = seg[0] * sign, mo = seg[1], d = seg[2];
  if (mo < 1 || mo > 12 || d < 1 || seg[3] > 23 || seg[4] > 59 || seg[5] > 59) return false;
  const bool leap = (y % 4 == 0 && y % 100 != 0) || y % 400 == 0;
  const int mdays[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  if (d > mdays[mo - 1] + (mo == 2 && leap ? 1 : 0)) return false;
  const int64_t days = days_from_civil(y, mo, d);
  *micros = (days * 86400 + seg[3] * 3600 + seg[4] * 60 + seg[5] - off) * 1000000ll + seg[6];
  return true;
}

__device__ SV cast_value(const uint8_t* s, uint32_t n, bool present, int type) {
  SV r{0, nullptr, 0, 1, 0};
  if (!present) return r;
  if (type == DR_T_STRING) {
    r.null = 0; r.str = 1; r.s = s; r.n = n;
    return r;
  }
  int64_t v = 0;
  bool ok = false;
  if (type == DR_T_BOOLEAN) ok = parse_bool(s, n, &v);
  else if (type == DR_T_DATE) ok = parse_date(s, n, &v);
  else ok = parse_int(s, n, type, &v);
  if (ok) { r.null = 0; r.v = v; }
  return r;
}

__device__ int cmp_sv(const SV& a, const SV& b) {
  if (a.str && b.str) {
    const uint32_t m = a.n < b.n ? a.n : b.n;
    for (uint32_t k = 0; k < m; ++k)
      if (a.s[k] != b.s[k]) return a.s[k] < b.s[k] ? -1 : 1;
    return a.n == b.n ? 0 : (a.n < b.n ? -1 : 1);
  }
  return a.v == b.v ? 0 : (a.v < b.v ? -1 : 1);
}

constexpr int PV_STACK = 32;

// ---- k_pv_extract --------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_pv_extract(PvExtractArgs a) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= a.n_live) return;
  const uint32_t act = a.live[i];
  const uint8_t* vp[PV_MAXC];
  uint32_t vn[PV_MAXC];
  uint8_t vs[PV_MAXC];
  for (int c = 0; c < a.ncols; ++c) { vp[c] = nullptr; vn[c] = 0; vs[c] = PV_NULL; }
  auto match = [&](const uint8_t* k, uint32_t kn, bool kesc) -> int {
    for (int c = 0; c < a.ncols; ++c)
      if (span_eq(k, kn, kesc, a.col_names + a.col_name_off[c], uint32_t(a.col_name_off[c + 1] - a.col_name_off[c])))
        return c;
    return -1;
  };
  const bool from_json = a.act_flags ? !(a.act_flags[act] & F_FROM_CKPT) : act >= a.ck_rows;
  if (from_json) {
    // JSON line: {"add":{..., "partitionValues":{"c":"v", ...}, ...}}
    const uint8_t* json = a.act_flags ? reinterpret_cast<const uint8_t*>(a.json_bases[a.src_id[act]]) : a.json;
    const uint8_t* b = json + a.src_off[act];
    const uint8_t* e = b + a.src_len[act];
    const uint8_t* p = skip_ws(b, e);
    bool ok = each_member(p, e, [&](const uint8_t* k, uint32_t kn, bool kesc, const uint8_t* v) -> const uint8_t* {
      if (key_is(k, kn, kesc, "add", 3) && v < e && *v == '{') {
        bool ok2 = each_member(v, e, [&](const uint8_t* k2, uint32_t kn2, bool kesc2, const uint8_t* v2) -> const uint8_t* {
          if (key_is(k2, kn2, kesc2, "partitionValues", 15)) {
            if (v2 < e && *v2 == '{') {
              // Jackson map deserialisation: a repeated key keeps the last value
              bool ok3 = each_member(v2, e, [&](const uint8_t* k3, uint32_t kn3, bool kesc3, const uint8_t* v3) -> const uint8_t* {
                const int c = match(k3, kn3, kesc3);
                const uint8_t* end3 = skip_value(v3, e);
                if (c >= 0) {
                  if (v3 < e && *v3 == '"') {
                    bool vesc = false;
                    const uint8_t* q = str_close(v3 + 1, e, &vesc);
                    vp[c] = v3 + 1; vn[c] = uint32_t(q - v3 - 1); vs[c] = vesc ? PV_ESCAPED : PV_RAW;
                  } else if (v3 < e && *v3 == 'n') {
                    vs[c] = PV_NULL;
                  } else {  // non-string token: Spark keeps its JSON text
                    vp[c] = v3; vn[c] = uint32_t(end3 - v3); vs[c] = PV_RAW;
                  }
                }
                return end3;
              });
              if (!ok3) return nullptr;
            }
          }
          return skip_value(v2, e);
        });
        if (!ok2) return nullptr;
      }
      return skip_value(v, e);
    });
    if (!ok) atomicOr(a.error, 1u);
    // escaped values are unescaped into the arena (sized by a counting pass)
    for (int c = 0; c < a.ncols; ++c) {
      if (vs[c] != PV_ESCAPED) continue;
      if (!a.arena) { atomicAdd(a.arena_need, (unsigned long long)vn[c]); vs[c] = PV_NULL; continue; }
      const unsigned long long o = atomicAdd(a.arena_fill, (unsigned long long)vn[c]);
      if (o + vn[c] > a.arena_cap) { atomicOr(a.error, 2u); vs[c] = PV_NULL; continue; }
      uint8_t* dst = a.arena + o;
      vn[c] = json_unescape(vp[c], vn[c], dst);
      vp[c] = dst;
      vs[c] = PV_RAW;
    }
  } else if (a.has_map) {
    const uint64_t r = a.src_off[act];
    for (uint64_t en = a.row_start[r]; en < a.row_start[r + 1]; ++en) {
      if (a.key_def[en] != a.key_max_def) continue;  // null / empty map
      const int c = match(reinterpret_cast<const uint8_t*>(a.key_ptr[en]), a.key_len[en], false);
      if (c < 0) continue;
      if (a.val_def[en] == a.val_max_def) {
        vp[c] = reinterpret_cast<const uint8_t*>(a.val_ptr[en]); vn[c] = a.val_len[en]; vs[c] = PV_RAW;
      } else {
        vs[c] = PV_NULL;
      }
    }
  }
  for (int c = 0; c < a.ncols; ++c) {
    const PvColumn& col = a.cols[c];
    const int base = col.type & 0xff;
    const bool present = vs[c] != PV_NULL;
    if (base == DR_T_FLOAT || base == DR_T_DOUBLE) {
      uint64_t bits = 0;
      const int r = present ? parse_fp(vp[c], vn[c], base == DR_T_FLOAT, &bits) : FP_NULL;
      col.isnull[i] = r != FP_OK;
      if (base == DR_T_FLOAT) col.w32[i] = uint32_t(bits);
      else col.w64[i] = int64_t(bits);
      if (r == FP_HARD) {  // the host converts it (rare: > 19 digits, large exponents, hex)
        const unsigned long long k = atomicAdd(col.nhard, 1ull);
        if (col.hard) {  // null on the counting pass: the host sizes the list and reruns
          col.hard[3 * k] = i;
          col.hard[3 * k + 1] = reinterpret_cast<uint64_t>(vp[c]);
          col.hard[3 * k + 2] = vn[c];
        }
      }
      continue;
    }
    if (base == DR_T_DECIMAL) {
      uint64_t lo = 0;
      int64_t hi = 0;
      const bool ok = present && parse_decimal(vp[c], vn[c], (col.type >> 8) & 0xff, (col.type >> 16) & 0xff, &lo, &hi);
      col.isnull[i] = !ok;
      col.w64[i] = int64_t(lo);
      col.w64hi[i] = hi;
      if (col.w32) col.w32[i] = uint32_t(lo);  // precision <= 9: Parquet INT32
      continue;
    }
    if (base == DR_T_TIMESTAMP) {
      int64_t us = 0;
      const bool ok = present && parse_timestamp(vp[c], vn[c], &us);
      col.isnull[i] = !ok;
      col.w64[i] = us;
      continue;
    }
    const SV v = cast_value(vp[c], vn[c], present, base == DR_T_BINARY ? DR_T_STRING : col.type);
    col.isnull[i] = v.null;
    if (col.type == DR_T_STRING || base == DR_T_BINARY) {
      col.sptr[i] = reinterpret_cast<uint64_t>(v.s);
      col.slen[i] = v.n;
      uint64_t s8 = 0;
      for (uint32_t k = 0; k < 8; ++k) s8 = (s8 << 8) | (k < v.n && !v.null ? v.s[k] : 0u);
      if (col.s8) col.s8[i] = s8;
    } else if (col.type == DR_T_LONG) {
      col.w64[i] = v.v;
    } else {
      col.w32[i] = uint32_t(int32_t(v.v));
    }
  }
}

// ---- k_filter_typed ------------------------------------------------------------------------------
__device__ __forceinline__ SV load_col(const PvColumn& col, uint64_t i) {
  SV r{0, nullptr, 0, col.isnull[i], 0};
  if (r.null) return r;
  if (col.type == DR_T_STRING) {
    r.str = 1;
    r.s = reinterpret_cast<const uint8_t*>(col.sptr[i]);
    r.n = col.slen[i];
  } else if (col.type == DR_T_LONG) {
    r.v = col.w64[i];
  } else {
    r.v = int64_t(int32_t(col.w32[i]));
  }
  return r;
}

__global__ void __launch_bounds__(256) k_filter_typed(FilterTypedArgs a) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= a.n_live) return;
  SV st[PV_STACK];
  int sp = 0;
  bool bad = false;
  for (int k = 0; k < a.nops && !bad; ++k) {
    const int op = a.ops[2 * k], arg = a.ops[2 * k + 1];
    switch (op) {
      case DR_OP_COL: {
        st[sp++] = load_col(a.cols[arg], i);
        break;
      }
      case DR_OP_LIT: {
        SV v{0, nullptr, 0, 1, 0};
        if (!a.lit_null[arg]) {
          v.null = 0;
          if (a.lit_types[arg] == DR_T_STRING) {
            v.str = 1;
            v.s = a.lit_str + a.lit_str_off[arg];
            v.n = uint32_t(a.lit_str_off[arg + 1] - a.lit_str_off[arg]);
          } else {
            v.v = a.lit_i64[arg];
          }
        }
        st[sp++] = v;
        break;
      }
      case DR_OP_EQ: case DR_OP_NE: case DR_OP_LT: case DR_OP_LE: case DR_OP_GT: case DR_OP_GE: {
        const SV y = st[--sp], x = st[--sp];
        SV r{0, nullptr, 0, 1, 0};
        if (!x.null && !y.null) {
          const int c = cmp_sv(x, y);
          r.null = 0;
          r.v = op == DR_OP_EQ ? c == 0 : op == DR_OP_NE ? c != 0 : op == DR_OP_LT ? c < 0
              : op == DR_OP_LE ? c <= 0 : op == DR_OP_GT ? c > 0 : c >= 0;
        }
        st[sp++] = r;
        break;
      }
      case DR_OP_NSEQ: {
        const SV y = st[--sp], x = st[--sp];
        SV r{0, nullptr, 0, 0, 0};
        r.v = (x.null && y.null) || (!x.null && !y.null && cmp_sv(x, y) == 0);
        st[sp++] = r;
        break;
      }
      // In(value, list) (Catalyst In.eval): true if some element equals the value; otherwise null
      // if the value or any element is null; otherwise false. Accumulator: v = found, str = anynull.
      case FILTER_OP_IN_START: {
        st[sp++] = SV{0, nullptr, 0, 0, 0};
        break;
      }
      case FILTER_OP_IN_STEP: {
        const SV y = st[--sp];
        SV& acc = st[sp - 1];
        const SV& x = st[sp - 2];
        if (y.null) acc.str = 1;
        else if (!x.null && cmp_sv(x, y) == 0) acc.v = 1;
        break;
      }
      case FILTER_OP_IN_END: {
        const SV acc = st[--sp];
        const SV x = st[sp - 1];
        SV r{0, nullptr, 0, 1, 0};
        if (!x.null) {
          if (acc.v) { r.null = 0; r.v = 1; }
          else if (!acc.str) { r.null = 0; r.v = 0; }
        }
        st[sp - 1] = r;
        break;
      }
      case DR_OP_ISNULL: case DR_OP_ISNOTNULL: {
        const SV x = st[--sp];
        SV r{0, nullptr, 0, 0, 0};
        r.v = op == DR_OP_ISNULL ? x.null : !x.null;
        st[sp++] = r;
        break;
      }
      case DR_OP_AND: {
        const SV y = st[--sp], x = st[--sp];
        SV r{0, nullptr, 0, 1, 0};
        if ((!x.null && !x.v) || (!y.null && !y.v)) { r.null = 0; r.v = 0; }
        else if (!x.null && !y.null) { r.null = 0; r.v = 1; }
        st[sp++] = r;
        break;
      }
      case DR_OP_OR: {
        const SV y = st[--sp], x = st[--sp];
        SV r{0, nullptr, 0, 1, 0};
        if ((!x.null && x.v) || (!y.null && y.v)) { r.null = 0; r.v = 1; }
        else if (!x.null && !y.null) { r.null = 0; r.v = 0; }
        st[sp++] = r;
        break;
      }
      case DR_OP_NOT: {
        SV& x = st[sp - 1];
        if (!x.null) x.v = !x.v;
        break;
      }
      default: bad = true;
    }
  }
  a.flag[i] = (!bad && sp == 1 && !st[0].null && st[0].v) ? 1u : 0u;
}

// ---- k_filter_leaf ---------------------------------------------------------------------------------
// Tri-states: 0 false, 1 true, 2 null (Catalyst's three-valued logic).
__device__ __forceinline__ int bytes_cmp(const uint8_t* a, uint32_t an, const uint8_t* b, uint32_t bn) {
  const uint32_t m = an < bn ? an : bn;
  for (uint32_t k = 0; k < m; ++k)
    if (a[k] != b[k]) return a[k] < b[k] ? -1 : 1;
  return an == bn ? 0 : (an < bn ? -1 : 1);
}

__device__ __forceinline__ uint32_t eval_leaf(const FilterLeafArgs& a, const FilterLeaf& L, uint64_t i,
                                              const int64_t* lit_i64, const uint64_t* lit_s8) {
  const PvColumn& col = a.cols[L.col];
  const bool vnull = col.isnull[i] != 0;
  if (L.op == DR_OP_ISNULL) return vnull ? 1u : 0u;
  if (L.op == DR_OP_ISNOTNULL) return vnull ? 0u : 1u;
  if (L.op == DR_OP_NSEQ && (vnull || L.lit_null)) return (vnull && L.lit_null) ? 1u : 0u;
  if (L.op != DR_OP_IN && L.lit_null) return 2u;
  if (vnull) return 2u;
  const bool str = col.type == DR_T_STRING;
  uint32_t vn = 0;
  uint64_t v8 = 0;
  int64_t v = 0;
  if (str) {
    vn = col.slen[i];
    v8 = col.s8[i];
  } else {
    v = col.type == DR_T_LONG ? col.w64[i] : int64_t(int32_t(col.w32[i]));
  }
  // strings: the big-endian 8-byte prefixes order like the bytes; equal prefixes of two values of
  // at most 8 bytes leave only the lengths; otherwise the value bytes are gathered
  auto cmp_lit = [&](int32_t k) -> int {
    if (str) {
      const uint64_t o = a.lit_str_off[k];
      const uint32_t ln = uint32_t(a.lit_str_off[k + 1] - o);
      const uint64_t l8 = lit_s8[k];
      if (v8 != l8) return v8 < l8 ? -1 : 1;
      if (vn <= 8 && ln <= 8) return vn == ln ? 0 : (vn < ln ? -1 : 1);
      return bytes_cmp(reinterpret_cast<const uint8_t*>(col.sptr[i]), vn, a.lit_str + o, ln);
    }
    const int64_t x = lit_i64[k];
    return v == x ? 0 : (v < x ? -1 : 1);
  };
  if (L.op == DR_OP_IN && L.pad == 1) {  // an integer set as a bitmap over [min, min + 64 * words)
    const uint64_t d = uint64_t(v) - uint64_t(lit_i64[L.lit]);
    const uint64_t nbits = uint64_t(lit_i64[L.lit + 1]) * 64;
    if (d < nbits && ((uint64_t(lit_i64[L.lit + 2 + (d >> 6)]) >> (d & 63)) & 1u)) return 1u;
    return L.lit_null ? 2u : 0u;
  }
  if (L.op == DR_OP_IN) {  // binary search of the sorted set
    int32_t lo = L.lit, hi = L.lit + L.nlit;
    while (lo < hi) {
      const int32_t mid = (lo + hi) >> 1;
      const int c = cmp_lit(mid);
      if (c == 0) return 1u;
      if (c > 0) lo = mid + 1; else hi = mid;
    }
    return L.lit_null ? 2u : 0u;
  }
  const int c = cmp_lit(L.lit);
  switch (L.op) {
    case DR_OP_EQ: case DR_OP_NSEQ: return c == 0;
    case DR_OP_NE: return c != 0;
    case DR_OP_LT: return c < 0;
    case DR_OP_LE: return c <= 0;
    case DR_OP_GT: return c > 0;
    default: return c >= 0;
  }
}

// Four files per thread, strided by the workgroup (each load instruction of a wave reads 64
// consecutive files): a leaf's column loads for all four are issued before any is compared, so one
// round trip serves four files. The result leaves as bits -- one 64-bit mask per 64 files, in file
// order -- plus the workgroup's count, which k_select_bits turns into the selected ordinals after a
// scan of the counts (no 4-byte flag per file, no scan over files).
#ifndef DR_FL_PER
#define DR_FL_PER 4
#endif
#ifndef DR_FL_GRID
#define DR_FL_GRID 4  // resident workgroups per CU of the persistent grid (0: one workgroup per tile)
#endif
constexpr int FL_T = 256, FL_PER = DR_FL_PER;
constexpr uint32_t FL_FILES = FL_T * FL_PER;  // files per tile (4 FL_PER mask words)

// The leaf result from a column value already in registers (nul, v = integer or big-endian 8-byte
// string prefix, vn = string length); the long-string gather reads the column by file ordinal i.
// The literals are the workgroup's LDS copies (li: integers and IN sets, ls8 / lso: the string
// literals' prefixes and offsets).
__device__ __forceinline__ uint32_t leaf_value(const uint8_t* lit_str, const FilterLeaf& L, const PvColumn& col,
                                               uint64_t i, uint32_t nul, int64_t v, uint32_t vn, const int64_t* li,
                                               const uint64_t* ls8, const uint64_t* lso) {
  const bool str = L.ctype == DR_T_STRING;
  const bool vnull = nul != 0;
  if (L.op == DR_OP_ISNULL) return vnull ? 1u : 0u;
  if (L.op == DR_OP_ISNOTNULL) return vnull ? 0u : 1u;
  if (L.op == DR_OP_NSEQ && (vnull || L.lit_null)) return (vnull && L.lit_null) ? 1u : 0u;
  if (L.op != DR_OP_IN && L.lit_null) return 2u;
  if (vnull) return 2u;
  const uint64_t v8 = uint64_t(v);
  auto cmp_lit = [&](int32_t k) -> int {
    if (str) {
      const uint64_t o = lso[k];
      const uint32_t ln = uint32_t(lso[k + 1] - o);
      const uint64_t l8 = ls8[k];
      if (v8 != l8) return v8 < l8 ? -1 : 1;
      if (vn <= 8 && ln <= 8) return vn == ln ? 0 : (vn < ln ? -1 : 1);
      return bytes_cmp(reinterpret_cast<const uint8_t*>(col.sptr[i]), vn, lit_str + o, ln);
    }
    const int64_t x = li[k];
    return v == x ? 0 : (v < x ? -1 : 1);
  };
  if (L.op == DR_OP_IN && L.pad == 1) {  // an integer set as a bitmap over [min, min + 64 * words)
    const uint64_t d = uint64_t(v) - uint64_t(li[L.lit]);
    const uint64_t nbits = uint64_t(li[L.lit + 1]) * 64;
    return (d < nbits && ((uint64_t(li[L.lit + 2 + uint32_t((nbits ? min(d, nbits - 1) : 0ull) >> 6)]) >> (d & 63)) & 1u)) ? 1u
           : (L.lit_null ? 2u : 0u);
  }
  if (L.op == DR_OP_IN) {  // binary search of the sorted set
    int32_t lo = L.lit, hi = L.lit + L.nlit;
    while (lo < hi) {
      const int32_t mid = (lo + hi) >> 1;
      const int c = cmp_lit(mid);
      if (c == 0) return 1u;
      if (c > 0) lo = mid + 1; else hi = mid;
    }
    return L.lit_null ? 2u : 0u;
  }
  const int c = cmp_lit(L.lit);
  switch (L.op) {
    case DR_OP_EQ: case DR_OP_NSEQ: return c == 0;
    case DR_OP_NE: return c != 0;
    case DR_OP_LT: return c < 0;
    case DR_OP_LE: return c <= 0;
    case DR_OP_GT: return c > 0;
    default: return c >= 0;
  }
}

// One column's values of a thread's FL_PER files (strided by the workgroup: each load instruction
// of a wave reads 64 consecutive files; all loads in flight before any is used). The tile's base is
// folded into uniform column pointers, so every load is a scalar base plus a 32-bit lane offset.
__device__ __forceinline__ void load_col4(const FilterLeafArgs& a, const PvColumn& col, int ctype, uint64_t base,
                                          bool full, uint32_t (&nul)[FL_PER], uint32_t (&vn)[FL_PER],
                                          int64_t (&v)[FL_PER]) {
  const bool str = ctype == DR_T_STRING, lng = ctype == DR_T_LONG;  // uniform
  const uint8_t* pn = col.isnull + base;
#pragma unroll
  for (int j = 0; j < FL_PER; ++j) {
    const uint32_t o = threadIdx.x + uint32_t(j) * FL_T;
    const bool ok = full || base + o < a.n_live;
    nul[j] = ok ? pn[o] : 1u;
    vn[j] = 0;
    v[j] = 0;
    if (str) {
      vn[j] = ok ? col.slen[base + o] : 0u;
      v[j] = ok ? int64_t(col.s8[base + o]) : 0;
    } else if (lng) {
      v[j] = ok ? col.w64[base + o] : 0;
    } else {
      v[j] = ok ? int64_t(int32_t(col.w32[base + o])) : 0;
    }
  }
}

// Persistent workgroups (grid-stride over tiles of FL_FILES files). The program, its leaves and
// every literal are copied to LDS once per workgroup, and the leaf fields are read as wave-uniform
// (scalar) values, so a tile issues no load but its column values: r04's first persistent build read
// the leaf from LDS into vector registers, which turned the column descriptor and every literal into
// per-lane global loads -- three dependent round trips per leaf and tile (2.53 ms for 100M files).
// When the program reads at most FL_UCOLS distinct columns, every value a tile needs is loaded up
// front and each leaf reads its column's slot (fixed by the host: a scalar branch picks it);
// otherwise each leaf loads its own column. A wave adds its selected count to its tile's (zeroed)
// count: no barrier per tile.
constexpr int FL_MAXPROG = 128, FL_MAXLEAF = 64, FL_MAXI64 = 1024, FL_MAXSTR = 256;
__global__ void __launch_bounds__(FL_T) k_filter_leaf(FilterLeafArgs a) {
  __shared__ int32_t sprog[2 * FL_MAXPROG];
  __shared__ FilterLeaf sleaf[FL_MAXLEAF];
  __shared__ int64_t slit[FL_MAXI64];
  __shared__ uint64_t ss8[FL_MAXSTR + 1], ssoff[FL_MAXSTR + 1];
  for (int k = threadIdx.x; k < 2 * a.nprog; k += FL_T) sprog[k] = a.prog[k];
  for (int k = threadIdx.x; k < a.nleaves; k += FL_T) sleaf[k] = a.leaves[k];
  for (int k = threadIdx.x; k < a.n_i64; k += FL_T) slit[k] = a.lit_i64[k];
  for (int k = threadIdx.x; k <= a.n_str; k += FL_T) {
    ss8[k] = a.lit_s8[k];
    ssoff[k] = a.lit_str_off[k];
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t ntiles = (a.n_live + FL_FILES - 1) / FL_FILES;
  const int nu = a.nucol;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t base = tile * FL_FILES;
    const bool full = base + FL_FILES <= a.n_live;  // uniform: no per-file bound check
    // the tile's column values: slot u holds predicate column a.ucol[u]
    uint32_t cn[FL_UCOLS][FL_PER], cl[FL_UCOLS][FL_PER];
    int64_t cv[FL_UCOLS][FL_PER];
#pragma unroll
    for (int u = 0; u < FL_UCOLS; ++u) {
      if (u >= nu) break;  // uniform
      const PvColumn& col = a.cols[a.ucol[u]];
      load_col4(a, col, col.type, base, full, cn[u], cl[u], cv[u]);
    }
    uint64_t stk[FL_PER];  // per file: 2 bits per entry, top at the low end
#pragma unroll
    for (int j = 0; j < FL_PER; ++j) stk[j] = 0;
    for (int k = 0; k < a.nprog; ++k) {
      const int op = __builtin_amdgcn_readfirstlane(sprog[2 * k]);
      if (op == LEAF_OP_LEAF) {
        const int li = __builtin_amdgcn_readfirstlane(sprog[2 * k + 1]);
        FilterLeaf L;
        L.col = __builtin_amdgcn_readfirstlane(sleaf[li].col);
        L.op = __builtin_amdgcn_readfirstlane(sleaf[li].op);
        L.lit = __builtin_amdgcn_readfirstlane(sleaf[li].lit);
        L.nlit = __builtin_amdgcn_readfirstlane(sleaf[li].nlit);
        L.lit_null = __builtin_amdgcn_readfirstlane(sleaf[li].lit_null);
        L.pad = __builtin_amdgcn_readfirstlane(sleaf[li].pad);
        L.slot = __builtin_amdgcn_readfirstlane(sleaf[li].slot);
        L.ctype = __builtin_amdgcn_readfirstlane(sleaf[li].ctype);
        const PvColumn& col = a.cols[L.col];  // read only by the long-string gather
        uint32_t n0[FL_PER], l0[FL_PER];
        int64_t v0[FL_PER];
        if (L.slot >= 0) {  // uniform: the preloaded slot (a select per value, no load)
#pragma unroll
          for (int j = 0; j < FL_PER; ++j) {
            n0[j] = cn[0][j];
            l0[j] = cl[0][j];
            v0[j] = cv[0][j];
#pragma unroll
            for (int u = 1; u < FL_UCOLS; ++u)
              if (u == L.slot) { n0[j] = cn[u][j]; l0[j] = cl[u][j]; v0[j] = cv[u][j]; }
          }
        } else {
          load_col4(a, col, L.ctype, base, full, n0, l0, v0);
        }
#pragma unroll
        for (int j = 0; j < FL_PER; ++j)
          stk[j] = (stk[j] << 2) |
                   leaf_value(a.lit_str, L, col, base + threadIdx.x + uint64_t(j) * FL_T, n0[j], v0[j], l0[j], slit, ss8, ssoff);
      } else if (op == LEAF_OP_NOT) {
#pragma unroll
        for (int j = 0; j < FL_PER; ++j) {
          const uint64_t x = stk[j] & 3u;
          stk[j] = (stk[j] & ~3ull) | (x == 2u ? 2u : (x ^ 1u));
        }
      } else {
#pragma unroll
        for (int j = 0; j < FL_PER; ++j) {
          const uint32_t y = uint32_t(stk[j] & 3u), x = uint32_t((stk[j] >> 2) & 3u);
          uint32_t rr;
          if (op == LEAF_OP_AND) rr = (x == 0u || y == 0u) ? 0u : (x == 1u && y == 1u) ? 1u : 2u;
          else rr = (x == 1u || y == 1u) ? 1u : (x == 0u && y == 0u) ? 0u : 2u;
          stk[j] = ((stk[j] >> 4) << 2) | rr;
        }
      }
    }
    uint32_t cnt = 0;
#pragma unroll
    for (int j = 0; j < FL_PER; ++j) {
      const bool f = (full || base + threadIdx.x + uint64_t(j) * FL_T < a.n_live) && (stk[j] & 3u) == 1u;
      const unsigned long long m = __ballot(f);
      if (lane == 0) a.mask[base / 64 + 4 * j + wv] = m;
      cnt += uint32_t(__popcll(m));
    }
    if (lane == 0 && cnt) atomicAdd(&a.wg_count[tile], cnt);
  }
}

// ---- K5 dictionary path ----------------------------------------------------------------------------
// Partition columns are low-cardinality by construction (one value per directory), so the typed
// cache is dictionary-encoded once per column: every distinct non-NULL value gets a u16 code
// (code 0 is NULL). A leaf is then evaluated once per code (k_dict_leaf: leaf_value on the code's
// representative row, so the three-valued semantics are the typed path's own), and k_filter_dict
// reads 2 bytes per file and column and looks the leaf results up in LDS (r04: the typed pass read
// 28 B per file in nine loads and evaluated every leaf per file: 1.93 ms for 100M files).
// Keys: the integer value itself (exact), or a string's xxh64 (k_dict_verify compares every file's
// bytes with its code's representative, so a hash collision abandons the dictionary).
__device__ __forceinline__ uint64_t dict_mix(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  return k ^ (k >> 33);
}
__device__ __forceinline__ bool dict_key(const PvColumn& c, uint64_t i, uint64_t* key) {
  if (c.isnull[i]) return false;
  const int base = c.type & 0xff;
  if (base == DR_T_STRING || base == DR_T_BINARY) *key = xxh64(reinterpret_cast<const uint8_t*>(c.sptr[i]), c.slen[i]);
  else if (c.w64) *key = uint64_t(c.w64[i]);
  else *key = uint64_t(c.w32[i]);
  return true;
}

// Inserts (key, row) into an open-addressing table (tag 0 empty, ~0 being written, 1 + row taken),
// one probe step per loop iteration for every lane, so a lane that finds a slot being written by
// another lane of its wave retries after that lane's write instead of spinning past it. Returns
// false when the table is full.
template <bool Lds>
__device__ __forceinline__ bool dict_put(uint64_t* keys, uint32_t* tags, uint32_t mask, uint64_t key, uint32_t row) {
  uint32_t h = uint32_t(dict_mix(key) >> 15) & mask;
  uint32_t probes = 0;
  bool done = false, ok = true;
  while (!done) {
    const uint32_t t = atomicCAS(&tags[h], 0u, 0xffffffffu);
    if (t == 0u) {
      keys[h] = key;
      if (!Lds) __threadfence();
      atomicExch(&tags[h], 1u + row);
      done = true;
    } else if (t != 0xffffffffu) {
      const uint64_t k = Lds ? *reinterpret_cast<volatile uint64_t*>(&keys[h])
                             : __hip_atomic_load(&keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (k == key) {
        done = true;
      } else {
        h = (h + 1) & mask;
        if (++probes > mask) { done = true; ok = false; }
      }
    }
  }
  return ok;
}

constexpr uint32_t DICT_T = 256, DICT_PER = 8, DICT_LSLOTS = 1024;
__global__ void __launch_bounds__(DICT_T) k_dict_insert(PvDictArgs a) {
  __shared__ uint64_t lkey[DICT_LSLOTS];
  __shared__ uint32_t ltag[DICT_LSLOTS];
  for (uint32_t k = threadIdx.x; k < DICT_LSLOTS; k += DICT_T) ltag[k] = 0;
  __syncthreads();
  const uint64_t base = uint64_t(blockIdx.x) * DICT_T * DICT_PER;
  // the workgroup's distinct keys first (a handful for a partition column), then those go global
  for (uint32_t j = 0; j < DICT_PER; ++j) {
    const uint64_t i = base + threadIdx.x + uint64_t(j) * DICT_T;
    uint64_t key;
    if (i < a.n && dict_key(a.col, i, &key))
      if (!dict_put<true>(lkey, ltag, DICT_LSLOTS - 1, key, uint32_t(i)))
        if (!dict_put<false>(a.key_tab, a.tag_tab, DICT_SLOTS - 1, key, uint32_t(i))) atomicOr(&a.ctr[1], 1ull);
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < DICT_LSLOTS; k += DICT_T) {
    const uint32_t t = ltag[k];
    if (t && !dict_put<false>(a.key_tab, a.tag_tab, DICT_SLOTS - 1, lkey[k], t - 1u)) atomicOr(&a.ctr[1], 1ull);
  }
}

__global__ void __launch_bounds__(256) k_dict_occupied(PvDictArgs a, uint32_t* occ) {
  const uint32_t h = blockIdx.x * 256 + threadIdx.x;
  if (h < DICT_SLOTS) occ[h] = a.tag_tab[h] != 0u;
}

// code = 1 + rank of the occupied slot; rep[code] = the slot's first row
__global__ void __launch_bounds__(256) k_dict_number(PvDictArgs a, const uint64_t* scan) {
  const uint32_t h = blockIdx.x * 256 + threadIdx.x;
  if (h >= DICT_SLOTS || !a.tag_tab[h]) return;
  const uint64_t c = scan[h] + 1;
  if (c >= DICT_MAX) return;  // too many values: the host abandons the dictionary
  a.slot_code[h] = uint32_t(c);
  a.rep[c] = a.tag_tab[h] - 1u;
}

__global__ void __launch_bounds__(256) k_dict_code(PvDictArgs a) {
  const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= a.n) return;
  uint64_t key;
  uint16_t c = 0;
  if (dict_key(a.col, i, &key)) {
    uint32_t h = uint32_t(dict_mix(key) >> 15) & (DICT_SLOTS - 1);
    for (uint32_t p = 0; p < DICT_SLOTS && a.key_tab[h] != key; ++p) h = (h + 1) & (DICT_SLOTS - 1);
    c = uint16_t(a.slot_code[h]);
    // strings: the code's representative must hold the same bytes (a 64-bit hash collision would
    // merge two values)
    const int base = a.col.type & 0xff;
    if (base == DR_T_STRING || base == DR_T_BINARY) {
      const uint32_t r = a.rep[c];
      const uint32_t n0 = a.col.slen[i];
      bool same = n0 == a.col.slen[r] && a.col.s8[i] == a.col.s8[r];
      if (same && n0 > 8)
        same = bytes_equal(reinterpret_cast<const uint8_t*>(a.col.sptr[i]), reinterpret_cast<const uint8_t*>(a.col.sptr[r]), n0);
      if (!same) atomicOr(&a.ctr[1], 2ull);
    }
  }
  a.code[i] = c;
}

// One thread per (leaf, code): the leaf on the code's representative value (code 0: NULL).
__global__ void __launch_bounds__(256) k_dict_leaf(DictLeafArgs a, uint32_t total) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= total) return;
  int32_t l = 0;
  while (l + 1 < a.nleaves && a.tab_off[l + 1] <= t) ++l;
  const FilterLeaf L = a.leaves[l];
  const uint32_t k = t - a.tab_off[l];
  const PvColumn& col = a.cols[L.col];
  uint32_t nul = 1, vn = 0;
  int64_t v = 0;
  uint64_t row = 0;
  if (k > 0) {
    row = a.rep[L.col][k];
    nul = 0;
    if (L.ctype == DR_T_STRING) {
      vn = col.slen[row];
      v = int64_t(col.s8[row]);
    } else {
      v = L.ctype == DR_T_LONG ? col.w64[row] : int64_t(int32_t(col.w32[row]));
    }
  }
  a.tab[t] = uint8_t(leaf_value(a.lit_str, L, col, row, nul, v, vn, a.lit_i64, a.lit_s8, a.lit_str_off));
}

// The per-file pass over codes: tiles of FL_FILES files, FL_PER per lane; every leaf is one LDS
// byte read per file.
constexpr uint32_t FD_MAXTAB = 32768;
__global__ void __launch_bounds__(FL_T) k_filter_dict(FilterDictArgs a) {
  __shared__ int32_t sprog[2 * FL_MAXPROG];
  __shared__ FilterLeaf sleaf[FL_MAXLEAF];
  __shared__ uint32_t stoff[FL_MAXLEAF + 1];
  __shared__ uint8_t stab[FD_MAXTAB];
  for (int k = threadIdx.x; k < 2 * a.nprog; k += FL_T) sprog[k] = a.prog[k];
  for (int k = threadIdx.x; k < a.nleaves; k += FL_T) sleaf[k] = a.leaves[k];
  for (int k = threadIdx.x; k <= a.nleaves; k += FL_T) stoff[k] = a.tab_off[k];
  for (uint32_t k = threadIdx.x; k < a.tab_bytes; k += FL_T) stab[k] = a.tab[k];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t ntiles = (a.n_live + FL_FILES - 1) / FL_FILES;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t base = tile * FL_FILES;
    const bool full = base + FL_FILES <= a.n_live;
    uint32_t cd[FL_UCOLS][FL_PER];
#pragma unroll
    for (int u = 0; u < FL_UCOLS; ++u) {
      if (u >= a.nslot) break;  // uniform
      const uint16_t* cp = a.code[u] + base;
#pragma unroll
      for (int j = 0; j < FL_PER; ++j) {
        const uint32_t o = threadIdx.x + uint32_t(j) * FL_T;
        cd[u][j] = (full || base + o < a.n_live) ? uint32_t(cp[o]) : 0u;
      }
    }
    uint64_t stk[FL_PER];
#pragma unroll
    for (int j = 0; j < FL_PER; ++j) stk[j] = 0;
    for (int k = 0; k < a.nprog; ++k) {
      const int op = __builtin_amdgcn_readfirstlane(sprog[2 * k]);
      if (op == LEAF_OP_LEAF) {
        const int li = __builtin_amdgcn_readfirstlane(sprog[2 * k + 1]);
        const int slot = __builtin_amdgcn_readfirstlane(sleaf[li].slot);
        const uint32_t off = uint32_t(__builtin_amdgcn_readfirstlane(int(stoff[li])));
#pragma unroll
        for (int j = 0; j < FL_PER; ++j) {
          uint32_t c = cd[0][j];
#pragma unroll
          for (int u = 1; u < FL_UCOLS; ++u)
            if (u == slot) c = cd[u][j];
          stk[j] = (stk[j] << 2) | stab[off + c];
        }
      } else if (op == LEAF_OP_NOT) {
#pragma unroll
        for (int j = 0; j < FL_PER; ++j) {
          const uint64_t x = stk[j] & 3u;
          stk[j] = (stk[j] & ~3ull) | (x == 2u ? 2u : (x ^ 1u));
        }
      } else {
#pragma unroll
        for (int j = 0; j < FL_PER; ++j) {
          const uint32_t y = uint32_t(stk[j] & 3u), x = uint32_t((stk[j] >> 2) & 3u);
          uint32_t rr;
          if (op == LEAF_OP_AND) rr = (x == 0u || y == 0u) ? 0u : (x == 1u && y == 1u) ? 1u : 2u;
          else rr = (x == 1u || y == 1u) ? 1u : (x == 0u && y == 0u) ? 0u : 2u;
          stk[j] = ((stk[j] >> 4) << 2) | rr;
        }
      }
    }
    uint32_t cnt = 0;
#pragma unroll
    for (int j = 0; j < FL_PER; ++j) {
      const bool f = (full || base + threadIdx.x + uint64_t(j) * FL_T < a.n_live) && (stk[j] & 3u) == 1u;
      const unsigned long long m = __ballot(f);
      if (lane == 0) a.mask[base / 64 + 4 * j + wv] = m;
      cnt += uint32_t(__popcll(m));
    }
    if (lane == 0 && cnt) atomicAdd(&a.wg_count[tile], cnt);
  }
}

// The selected ordinals of one k_filter_leaf workgroup's files, in file order: its 16 mask words
// and the exclusive scan of the workgroups' counts give every selected file its output position.
__global__ void __launch_bounds__(FL_T) k_select_bits(const uint64_t* mask, const uint64_t* wg_off, uint64_t n,
                                                    int64_t* out) {
  __shared__ uint64_t w[FL_FILES / 64];
  __shared__ uint32_t before[FL_FILES / 64];
  const uint64_t base = uint64_t(blockIdx.x) * FL_FILES;
  if (threadIdx.x < FL_FILES / 64) w[threadIdx.x] = mask[base / 64 + threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (uint32_t k = 0; k < FL_FILES / 64; ++k) { before[k] = s; s += uint32_t(__popcll(w[k])); }
  }
  __syncthreads();
  const uint64_t o = wg_off[blockIdx.x];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < FL_PER; ++j) {
    const uint32_t k = 4 * j + wv;
    const uint64_t m = w[k];
    if ((m >> lane) & 1ull)
      out[o + before[k] + uint32_t(__popcll(m & ((1ull << lane) - 1ull)))] = int64_t(base + uint64_t(j) * FL_T + threadIdx.x);
  }
}

// checkpoint map column: row_start[k] = index of the k-th entry with repetition level 0
__global__ void k_row_starts(const uint8_t* rep, uint64_t n, const uint64_t* pos, uint64_t* row_start) {
  const uint64_t e = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e < n && rep[e] == 0) row_start[pos[e]] = e;
}
__global__ void k_rep0_flags(const uint8_t* rep, uint64_t n, uint32_t* f) {
  const uint64_t e = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e < n) f[e] = rep[e] == 0;
}
__global__ void k_select(const uint32_t* flag, const uint64_t* pos, uint64_t n, int64_t* out) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n && flag[i]) out[pos[i]] = int64_t(i);
}

// ---- full-record checksum (dr_state_record_sums) ------------------------------------------------
// One lane per exported record: the eight canonical words (oracle/delta_oracle.py:record_hash) from
// the export columns, xxh64 of them, and a wave + workgroup sum added once per workgroup. Integer
// addition mod 2^64 is order-free, so the result does not depend on the survivors' order.
constexpr uint64_t REC_SEED = 0x5EED, REC_GOLD = 0x9E3779B97F4A7C15ull, REC_NULLV = 0x5BD1E9955BD1E995ull;

__device__ inline uint64_t rec_map_hash(uint8_t is_null, uint64_t e0, uint64_t e1, const int64_t* koff,
                                        const uint8_t* kb, const int64_t* voff, const uint8_t* vb,
                                        const uint8_t* vnull, uint64_t ks, uint64_t vs) {
  if (is_null) return 0;
  uint64_t h = 1 + (e1 - e0);
  for (uint64_t e = e0; e < e1; ++e) {
    const uint64_t hk = xxh64(kb + koff[e], uint32_t(koff[e + 1] - koff[e]), ks);
    const uint64_t hv = vnull[e] ? REC_NULLV : xxh64(vb + voff[e], uint32_t(voff[e + 1] - voff[e]), vs);
    h += hk * REC_GOLD + hv;
  }
  return h;
}

// xxh64 of eight little-endian words (64 bytes: two 32-byte stripes, no tail).
__device__ inline uint64_t xxh64_words8(const uint64_t* w, uint64_t seed) {
  uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
  for (int s = 0; s < 8; s += 4) {
    v1 = xx_round(v1, w[s]);
    v2 = xx_round(v2, w[s + 1]);
    v3 = xx_round(v3, w[s + 2]);
    v4 = xx_round(v4, w[s + 3]);
  }
  uint64_t h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
  h = xx_merge(h, v1);
  h = xx_merge(h, v2);
  h = xx_merge(h, v3);
  h = xx_merge(h, v4);
  h += 64;
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

__global__ void __launch_bounds__(256) k_record_hash(RecordHashArgs a) {
  __shared__ unsigned long long part[4];
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  uint64_t r = 0;
  if (i < a.n) {
    uint64_t w[8];
    w[0] = uint64_t(a.side);
    w[1] = xxh64(a.path_bytes + a.path_off[i], uint32_t(a.path_off[i + 1] - a.path_off[i]), 0);
    w[2] = uint64_t(a.size[i]);
    if (a.side == 0) {
      w[3] = uint64_t(a.mtime[i]);
      w[4] = 0;
      w[5] = a.stats_null[i] ? 0
                             : xxh64(a.stats_bytes + a.stats_off[i], uint32_t(a.stats_off[i + 1] - a.stats_off[i]), 1);
    } else {
      const bool has = a.flags[i] & F_HAS_DELTS;
      w[3] = has ? a.delts[i] : 0;
      w[4] = (has ? 1u : 0u) | (a.efm[i] ? 2u : 0u);
      w[5] = 0;
    }
    w[6] = rec_map_hash(a.pv_null[i], a.pv_entry[i], a.pv_entry[i + 1], a.pv_key_off, a.pv_key_bytes, a.pv_val_off,
                        a.pv_val_bytes, a.pv_val_null, 2, 3);
    w[7] = rec_map_hash(a.tags_null[i], a.tags_entry[i], a.tags_entry[i + 1], a.tags_key_off, a.tags_key_bytes,
                        a.tags_val_off, a.tags_val_bytes, a.tags_val_null, 4, 5);
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = (a.field_mask >> k) & 1u ? w[k] : 0ull;
    r = xxh64_words8(w, REC_SEED);
    if (a.out) a.out[i] = r;
  }
  for (int o = 32; o > 0; o >>= 1) r += __shfl_down(r, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = r;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(a.sum, part[0] + part[1] + part[2] + part[3]);
}

}  // namespace dev

static inline unsigned g256(uint64_t n) { return unsigned((n + 255) / 256); }

uint32_t filter_max_cols() { return PV_MAXC; }
uint32_t filter_max_stack() { return dev::PV_STACK; }

void launch_pv_extract(const PvExtractArgs& a, hipStream_t st) {
  if (a.n_live) DR_LAUNCH(dev::k_pv_extract, dim3(g256(a.n_live)), dim3(256), 0, st, a);
}
uint64_t filter_leaf_groups(uint64_t n) { return (n + dev::FL_FILES - 1) / dev::FL_FILES; }
uint32_t filter_leaf_mask_words() { return dev::FL_FILES / 64; }
void launch_filter_leaf(const FilterLeafArgs& a, hipStream_t st) {
  if (a.nprog > dev::FL_MAXPROG || a.nleaves > dev::FL_MAXLEAF)
    throw std::runtime_error("filter program too long for the leaf kernel");
  // persistent: four resident workgroups per CU (119 VGPRs: 4 waves/SIMD), each walking tiles grid-stride
  const unsigned g = unsigned(DR_FL_GRID ? std::min<uint64_t>(filter_leaf_groups(a.n_live), 256 * DR_FL_GRID)
                                          : filter_leaf_groups(a.n_live));
  if (a.n_live) DR_LAUNCH(dev::k_filter_leaf, dim3(g), dim3(dev::FL_T), 0, st, a);
}
uint32_t filter_leaf_max_prog() { return dev::FL_MAXPROG; }
void launch_dict_insert(const PvDictArgs& a, hipStream_t st) {
  const uint64_t per = uint64_t(dev::DICT_T) * dev::DICT_PER;
  if (a.n) DR_LAUNCH(dev::k_dict_insert, dim3(unsigned((a.n + per - 1) / per)), dim3(dev::DICT_T), 0, st, a);
}
void launch_dict_occupied(const PvDictArgs& a, uint32_t* occ, hipStream_t st) {
  DR_LAUNCH(dev::k_dict_occupied, dim3(DICT_SLOTS / 256), dim3(256), 0, st, a, occ);
}
void launch_dict_number(const PvDictArgs& a, const uint64_t* scan, hipStream_t st) {
  DR_LAUNCH(dev::k_dict_number, dim3(DICT_SLOTS / 256), dim3(256), 0, st, a, scan);
}
void launch_dict_code(const PvDictArgs& a, hipStream_t st) {
  if (a.n) DR_LAUNCH(dev::k_dict_code, dim3(g256(a.n)), dim3(256), 0, st, a);
}
void launch_dict_leaf(const DictLeafArgs& a, uint32_t total, hipStream_t st) {
  if (total) DR_LAUNCH(dev::k_dict_leaf, dim3(unsigned((total + 255) / 256)), dim3(256), 0, st, a, total);
}
uint32_t filter_dict_max_tab() { return dev::FD_MAXTAB; }
void launch_filter_dict(const FilterDictArgs& a, hipStream_t st) {
  if (a.nprog > dev::FL_MAXPROG || a.nleaves > dev::FL_MAXLEAF || a.tab_bytes > dev::FD_MAXTAB)
    throw std::runtime_error("filter program too long for the dictionary kernel");
  const unsigned g = unsigned(std::min<uint64_t>(filter_leaf_groups(a.n_live), 256 * 8));
  if (a.n_live) DR_LAUNCH(dev::k_filter_dict, dim3(g), dim3(dev::FL_T), 0, st, a);
}
uint32_t filter_leaf_max_i64() { return dev::FL_MAXI64; }
uint32_t filter_leaf_max_str() { return dev::FL_MAXSTR; }
uint32_t filter_leaf_max_leaves() { return dev::FL_MAXLEAF; }
void launch_select_bits(const uint64_t* mask, const uint64_t* wg_off, uint64_t n, int64_t* out, hipStream_t st) {
  if (n) DR_LAUNCH(dev::k_select_bits, dim3(unsigned(filter_leaf_groups(n))), dim3(dev::FL_T), 0, st, mask, wg_off, n, out);
}
void launch_filter_typed(const FilterTypedArgs& a, hipStream_t st) {
  if (a.n_live) DR_LAUNCH(dev::k_filter_typed, dim3(g256(a.n_live)), dim3(256), 0, st, a);
}
void launch_rep0_flags(const uint8_t* rep, uint64_t n, uint32_t* f, hipStream_t st) {
  if (n) DR_LAUNCH(dev::k_rep0_flags, dim3(g256(n)), dim3(256), 0, st, rep, n, f);
}
void launch_row_starts(const uint8_t* rep, uint64_t n, const uint64_t* pos, uint64_t* row_start, hipStream_t st) {
  if (n) DR_LAUNCH(dev::k_row_starts, dim3(g256(n)), dim3(256), 0, st, rep, n, pos, row_start);
}
void launch_record_hash(const RecordHashArgs& a, hipStream_t st) {
  if (a.n) DR_LAUNCH(dev::k_record_hash, dim3(g256(a.n)), dim3(256), 0, st, a);
}
void launch_select(const uint32_t* flag, const uint64_t* pos, uint64_t n, int64_t* out, hipStream_t st) {
  if (n) DR_LAUNCH(dev::k_select, dim3(g256(n)), dim3(256), 0, st, flag, pos, n, out);
}

// ---- scan-side consumers -------------------------------------------------------------------------
namespace dev {

// Jackson's long from a JSON number token: an integer literal that fits int64 (anything else --
// fraction, exponent, string, overflow -- leaves the primitive's default 0, as the host export does).
__device__ bool json_int64(const uint8_t* p, const uint8_t* e, int64_t* out) {
  bool neg = false;
  if (p < e && *p == '-') { neg = true; ++p; }
  if (p >= e || *p < '0' || *p > '9') return false;
  uint64_t v = 0;
  while (p < e && *p >= '0' && *p <= '9') {
    const uint64_t d = uint64_t(*p - '0');
    if (v > (uint64_t(INT64_MAX) + (neg ? 1 : 0) - d) / 10) return false;
    v = v * 10 + d;
    ++p;
  }
  if (p < e && (*p == '.' || *p == 'e' || *p == 'E')) return false;
  *out = neg ? int64_t(0 - v) : int64_t(v);
  return true;
}

__global__ void __launch_bounds__(256) k_mtime_extract(MtimeArgs a) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= a.n_live) return;
  const uint32_t act = a.live[i];
  int64_t mt = 0;
  const bool from_json = a.act_flags ? !(a.act_flags[act] & F_FROM_CKPT) : act >= a.ck_rows;
  if (from_json) {
    const uint8_t* json = a.act_flags ? reinterpret_cast<const uint8_t*>(a.json_bases[a.src_id[act]]) : a.json;
    const uint8_t* b = json + a.src_off[act];
    const uint8_t* e = b + a.src_len[act];
    const uint8_t* p = skip_ws(b, e);
    const bool ok = each_member(p, e, [&](const uint8_t* k, uint32_t kn, bool kesc, const uint8_t* v) -> const uint8_t* {
      if (key_is(k, kn, kesc, "add", 3) && v < e && *v == '{') {
        const bool ok2 = each_member(v, e, [&](const uint8_t* k2, uint32_t kn2, bool kesc2, const uint8_t* v2) -> const uint8_t* {
          const uint8_t* end2 = skip_value(v2, e);
          if (key_is(k2, kn2, kesc2, "modificationTime", 16)) {
            int64_t x;
            mt = json_int64(v2, end2, &x) ? x : 0;  // a repeated member: the last one wins
          }
          return end2;
        });
        if (!ok2) return nullptr;
      }
      return skip_value(v, e);
    });
    if (!ok) atomicOr(a.error, 1u);
  } else if (a.ck_def) {
    const uint64_t r = a.src_off[act];
    if (a.ck_def[r] == a.ck_max_def) mt = a.ck_val[r];
  }
  a.out[i] = mt;
}

struct ScanOrderLess {
  const int64_t* mt;
  const uint64_t* pp;
  const uint32_t* pl;
  __device__ bool operator()(uint32_t x, uint32_t y) const {
    if (mt[x] != mt[y]) return mt[x] < mt[y];
    const int c = bytes_cmp(reinterpret_cast<const uint8_t*>(pp[x]), pl[x], reinterpret_cast<const uint8_t*>(pp[y]), pl[y]);
    return c != 0 ? c < 0 : x < y;
  }
};

__device__ __forceinline__ int tuple_cmp(const GroupCols& g, uint32_t x, uint32_t y) {
  for (int c = 0; c < g.ncols; ++c) {
    const uint8_t nx = g.isnull[c][x], ny = g.isnull[c][y];
    if (nx != ny) return nx ? -1 : 1;  // nulls first
    if (nx) continue;
    const int r = bytes_cmp(reinterpret_cast<const uint8_t*>(g.sptr[c][x]), g.slen[c][x],
                            reinterpret_cast<const uint8_t*>(g.sptr[c][y]), g.slen[c][y]);
    if (r) return r;
  }
  return 0;
}

struct GroupLess {
  GroupCols g;
  __device__ bool operator()(uint32_t x, uint32_t y) const {
    const int c = tuple_cmp(g, x, y);
    return c != 0 ? c < 0 : x < y;
  }
};

__global__ void __launch_bounds__(256) k_group_flags(const uint32_t* keys, uint64_t n, GroupCols g, uint32_t* flag) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  flag[i] = i == 0 || tuple_cmp(g, keys[i - 1], keys[i]) != 0;
}

}  // namespace dev

void launch_mtime_extract(const MtimeArgs& a, hipStream_t st) {
  if (a.n_live) DR_LAUNCH(dev::k_mtime_extract, dim3(unsigned((a.n_live + 255) / 256)), dim3(256), 0, st, a);
}

void launch_sort_scan_order(void* temp, size_t* temp_bytes, uint32_t* keys, uint64_t n, const int64_t* mtime,
                            const uint64_t* path_ptr, const uint32_t* path_len, hipStream_t st) {
  const dev::ScanOrderLess less{mtime, path_ptr, path_len};
  if (hipcub::DeviceMergeSort::SortKeys(temp, *temp_bytes, keys, n, less, st) != hipSuccess)
    throw std::runtime_error("scan-order merge sort failed");
}

void launch_sort_groups(void* temp, size_t* temp_bytes, uint32_t* keys, uint64_t n, const GroupCols& g,
                        hipStream_t st) {
  const dev::GroupLess less{g};
  if (hipcub::DeviceMergeSort::SortKeys(temp, *temp_bytes, keys, n, less, st) != hipSuccess)
    throw std::runtime_error("partition-group merge sort failed");
}

void launch_group_flags(const uint32_t* keys, uint64_t n, const GroupCols& g, uint32_t* flag, hipStream_t st) {
  if (n) DR_LAUNCH(dev::k_group_flags, dim3(unsigned((n + 255) / 256)), dim3(256), 0, st, keys, n, g, flag);
}

// ---- device export of the survivors' records (dr_state_export) -----------------------------------
// The fields the replay kernels do not keep -- modificationTime, stats, partitionValues, tags,
// extendedFileMetadata, a checkpoint remove's size -- read per survivor from its JSON line (the
// add / remove object, Jackson semantics: a repeated member keeps the last value; a repeated map key
// keeps its first position and last value, as a LinkedHashMap) or from the checkpoint's decoded
// leaves (row-indexed flat columns, map entries by row). Strings are unescaped; a non-string value
// where a string is expected keeps its JSON text without insignificant whitespace.
namespace dev {

// Short copies (map keys and values): eight loads in flight before their stores (a plain byte loop
// waits for each load, and on gfx9 a load's wait also waits for every earlier store).
__device__ __forceinline__ void bytes_copy(uint8_t* d, const uint8_t* s, uint32_t n) {
  for (uint32_t k0 = 0; k0 < n; k0 += 8) {
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      const uint32_t b = k0 + k < n ? uint32_t(s[k0 + k]) : 0u;
      if (k < 4) lo |= b << (8 * k); else hi |= b << (8 * (k - 4));
    }
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k)
      if (k0 + k < n) d[k0 + k] = uint8_t((k < 4 ? lo : hi) >> (8 * (k & 3)));
  }
}

__device__ uint32_t json_unescape_len(const uint8_t* s, uint32_t n) {
  uint32_t o = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (s[i] != '\\' || i + 1 >= n) { ++o; continue; }
    const uint8_t e = s[++i];
    if (e != 'u') { ++o; continue; }
    uint32_t cp = 0;
    for (int k = 0; k < 4 && i + 1 < n; ++k) cp = cp * 16 + uint32_t(hexval(s[++i]) & 15);
    if (cp >= 0xD800 && cp < 0xDC00 && i + 6 < n && s[i + 1] == '\\' && s[i + 2] == 'u') {
      uint32_t lo = 0;
      for (int k = 0; k < 4; ++k) lo = lo * 16 + uint32_t(hexval(s[i + 3 + k]) & 15);
      if (lo >= 0xDC00 && lo < 0xE000) { cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00); i += 6; }
    }
    o += cp < 0x80 ? 1 : cp < 0x800 ? 2 : cp < 0x10000 ? 3 : 4;
  }
  return o;
}

// JSON text of [v, end) without whitespace outside strings (out null: length only)
__device__ uint32_t compact_json(const uint8_t* v, const uint8_t* end, uint8_t* out) {
  uint32_t o = 0;
  bool in_str = false;
  for (const uint8_t* p = v; p < end; ++p) {
    const uint8_t c = *p;
    if (in_str) {
      if (out) out[o] = c;
      ++o;
      if (c == '\\' && p + 1 < end) {
        ++p;
        if (out) out[o] = *p;
        ++o;
      } else if (c == '"') {
        in_str = false;
      }
      continue;
    }
    if (is_ws(c)) continue;
    if (c == '"') in_str = true;
    if (out) out[o] = c;
    ++o;
  }
  return o;
}

// A JSON value where a string is expected: {null?, bytes}. Pass 1 counts, pass 2 writes at out.
__device__ __forceinline__ uint32_t string_value(const uint8_t* v, const uint8_t* end, bool* is_null, uint8_t* out) {
  *is_null = false;
  if (v < end && *v == '"') {
    bool esc = false;
    const uint8_t* q = str_close(v + 1, end, &esc);
    const uint32_t n = uint32_t(q - v - 1);
    if (!esc) {
      if (out) for (uint32_t k = 0; k < n; ++k) out[k] = v[1 + k];
      return n;
    }
    return out ? json_unescape(v + 1, n, out) : json_unescape_len(v + 1, n);
  }
  if (v < end && *v == 'n' && end - v == 4) {  // null
    *is_null = true;
    if (out) { out[0] = 'n'; out[1] = 'u'; out[2] = 'l'; out[3] = 'l'; }  // the host export's json_dump text
    return 4;
  }
  return compact_json(v, end, out);
}

__device__ bool keys_equal(const uint8_t* a, uint32_t an, bool aesc, const uint8_t* b, uint32_t bn, bool besc) {
  if (!aesc && !besc) return an == bn && bytes_equal(a, b, an);
  if (!aesc) return span_eq(b, bn, besc, a, an);
  if (!besc) return span_eq(a, an, aesc, b, bn);
  if (an > 128 || bn > 128) return an == bn && bytes_equal(a, b, an);
  uint8_t buf[160];
  const uint32_t m = json_unescape(b, bn, buf);
  return span_eq(a, an, aesc, buf, m);
}

struct MapSink {
  uint32_t n, kb, vb;                   // entries and bytes so far
  uint64_t* ksrc;                       // pass 2, checkpoint rows: this record's first entry's source slots
  uint64_t* vsrc;
  uint32_t* klen;
  uint32_t* vlen;
  uint8_t* kbytes;                      // pass 2: this record's first key byte
  uint8_t* vbytes;
  int64_t* koff;                        // pass 2: this record's first entry's end-offset slot
  int64_t* voff;
  uint8_t* vnull;
  int64_t kbase, vbase;                 // absolute offsets of kbytes / vbytes
};

__device__ __forceinline__ void sink_entry_json(MapSink& m, bool write, const uint8_t* k, uint32_t kn, bool kesc, const uint8_t* v,
                                const uint8_t* vend) {
  const uint32_t kl = kesc ? (write ? json_unescape(k, kn, m.kbytes + m.kb) : json_unescape_len(k, kn))
                           : (write ? (bytes_copy(m.kbytes + m.kb, k, kn), kn) : kn);
  bool vn;
  const uint32_t vl = string_value(v, vend, &vn, write ? m.vbytes + m.vb : nullptr);
  m.kb += kl;
  m.vb += vl;
  if (write) {
    m.koff[m.n] = m.kbase + m.kb;
    m.voff[m.n] = m.vbase + m.vb;
    m.vnull[m.n] = vn ? 1 : 0;
  }
  ++m.n;
}

// Entries of the JSON object at m0 ('{') into the sink (first position, last value per key).
__device__ __forceinline__ bool json_map(const uint8_t* m0, const uint8_t* e, MapSink& m, bool write) {
  return each_member(m0, e, [&](const uint8_t* k, uint32_t kn, bool kesc, const uint8_t* v) -> const uint8_t* {
    const uint8_t* vend = skip_value(v, e);
    bool first = true, after = false;
    const uint8_t* lv = v;
    const uint8_t* lend = vend;
    each_member(m0, e, [&](const uint8_t* k2, uint32_t kn2, bool kesc2, const uint8_t* v2) -> const uint8_t* {
      const uint8_t* vend2 = skip_value(v2, e);
      if (k2 == k) {
        after = true;
      } else if (keys_equal(k, kn, kesc, k2, kn2, kesc2)) {
        if (!after) first = false;
        else { lv = v2; lend = vend2; }
      }
      return vend2;
    });
    if (first) sink_entry_json(m, write, k, kn, kesc, lv, lend);
    return vend;
  });
}

// A checkpoint row's map entries, CK_BATCH at a time: the batch's levels, lengths and addresses are
// loaded before any is used (r04: one entry's chain of loads per step left pass 1 latency-bound).
// Pass 2 writes the entries' offsets and their sources; the bytes follow in k_gather_bytes.
constexpr uint32_t CK_BATCH = 4;
template <bool Write>
__device__ __forceinline__ void ck_map(const ExpMap& cm, uint64_t r, MapSink& m, uint8_t* is_null) {
  *is_null = 1;
  if (!cm.row_start) return;
  const uint64_t e0 = cm.row_start[r], e1 = cm.row_start[r + 1];
  for (uint64_t b = e0; b < e1; b += CK_BATCH) {
    int kd[CK_BATCH], vd[CK_BATCH];
    uint32_t kl[CK_BATCH], vl[CK_BATCH];
    uint64_t kp[CK_BATCH], vp[CK_BATCH];
#pragma unroll
    for (uint32_t q = 0; q < CK_BATCH; ++q) {
      const uint64_t en = b + q;
      const bool ok = en < e1;
      kd[q] = ok ? int(cm.kdef[en]) : -1;
      kl[q] = ok ? cm.klen[en] : 0u;
      vd[q] = ok ? int(cm.vdef[en]) : 0;
      vl[q] = ok ? cm.vlen[en] : 0u;
      if (Write) {
        kp[q] = ok ? cm.kptr[en] : 0ull;
        vp[q] = ok ? cm.vptr[en] : 0ull;
      }
    }
#pragma unroll
    for (uint32_t q = 0; q < CK_BATCH; ++q) {
      const int d = kd[q];
      if (d >= cm.map_def) *is_null = 0;
      if (d < cm.entry_def) continue;  // also the batch's entries past the row (-1)
      const bool vn = vd[q] != cm.vmax;
      const uint32_t vlen = vn ? 0u : vl[q];
      if (Write) {  // the bytes are copied by k_gather_bytes, several lanes per string
        m.ksrc[m.n] = kp[q];
        m.klen[m.n] = kl[q];
        m.vsrc[m.n] = vp[q];
        m.vlen[m.n] = vlen;
      }
      m.kb += kl[q];
      m.vb += vlen;
      if (Write) {
        m.koff[m.n] = m.kbase + m.kb;
        m.voff[m.n] = m.vbase + m.vb;
        m.vnull[m.n] = vn ? 1 : 0;
      }
      ++m.n;
    }
  }
}

// The walkers above step through a line one dependent byte at a time, so each step costs a load's
// round trip: from L2 a lane spends ~2.5 us per survivor line (r04 probe: 15 + 32 ms for the live
// side's two passes at config 3). k_export therefore stages its wave's lines in LDS first -- each
// lane copies its own line with independent 16-byte loads, EXP_BATCH in flight -- and walks the
// staged copy (generic pointers: a line that does not fit is walked in place). A slot holds the
// line's aligned 16-byte chunks, so the line sits at slot + (start & 15); the buffer keeps 32 bytes of
// padding after the last slot for the walkers' word reads past a line's end.
#ifndef DR_EXP_STAGE
#define DR_EXP_STAGE 24576
#endif
constexpr uint32_t EXP_STAGE = DR_EXP_STAGE;
constexpr uint32_t EXP_BATCH = 8;

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t* total) {
  const int lane = threadIdx.x & 63;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  *total = __shfl(x, 63, 64);
  return x - v;
}

// Pass 2's output streams: the wave's records write each stream to one contiguous range (the
// exclusive scans of pass 1's counts), so the records' bytes and entries are assembled in LDS and
// the wave stores each range with aligned 16-byte stores. Written in place instead, every byte store
// sat in the same counter as the walkers' generic (flat) reads of the staged line, and each such read
// waited for the stores before it.
#ifndef DR_EXP_OUT
#define DR_EXP_OUT 16384
#endif
constexpr uint32_t EXP_OUT = DR_EXP_OUT;  // 0: pass 2 writes in place
enum ExpStream { XS_STATS, XS_PVK, XS_PVV, XS_TGK, XS_TGV, XS_PVKO, XS_PVVO, XS_PVVN, XS_TGKO, XS_TGVO, XS_TGVN, XS_N };

// One record of k_export (pass 1: scalars and counts; pass 2: bytes and entries into the sinks).
__device__ __forceinline__ void export_record(const ExportArgs& a, uint64_t i, uint32_t act, bool json_lane,
                                              const uint8_t* line, uint32_t glen, bool write, MapSink& pv,
                                              MapSink& tg, uint8_t* sbytes) {
  int64_t size = a.act_size[act], mt = 0;
  uint8_t efm = 0, snull = 1, pnull = 1, tnull = 1;
  uint32_t slen = 0;
  if (json_lane) {
    const uint8_t* b = line;
    const uint8_t* e = b + glen;
    const char* side = a.side == 0 ? "add" : "remove";
    const uint32_t sl = a.side == 0 ? 3 : 6;
    // the side's object: the last member of that name (a repeated member keeps its last value)
    const uint8_t* obj = nullptr;
    const bool ok = each_member(skip_ws(b, e), e, [&](const uint8_t* k, uint32_t kn, bool kesc, const uint8_t* v) -> const uint8_t* {
      if (key_is(k, kn, kesc, side, sl)) obj = (v < e && *v == '{') ? v : nullptr;
      return skip_value(v, e);
    });
    if (!ok) atomicOr(a.error, 1u);
    if (obj) {
      // last occurrence of each field
      const uint8_t *st = nullptr, *st_end = nullptr, *pvo = nullptr, *tgo = nullptr;
      bool pv_seen = false, tg_seen = false;
      each_member(obj, e, [&](const uint8_t* k, uint32_t kn, bool kesc, const uint8_t* v) -> const uint8_t* {
        const uint8_t* vend = skip_value(v, e);
        if (key_is(k, kn, kesc, "modificationTime", 16)) {
          int64_t x;
          mt = json_int64(v, vend, &x) ? x : 0;
        } else if (key_is(k, kn, kesc, "extendedFileMetadata", 20)) {
          efm = (vend - v == 4 && v[0] == 't') ? 1 : 0;
        } else if (key_is(k, kn, kesc, "stats", 5)) {
          st = v;
          st_end = vend;
        } else if (key_is(k, kn, kesc, "partitionValues", 15)) {
          pv_seen = true;
          pvo = (v < e && *v == '{') ? v : nullptr;
          pnull = (v < e && *v == 'n') ? 1 : 0;
        } else if (key_is(k, kn, kesc, "tags", 4)) {
          tg_seen = true;
          tgo = (v < e && *v == '{') ? v : nullptr;
          tnull = (v < e && *v == 'n') ? 1 : 0;
        }
        return vend;
      });
      if (st && !(st_end - st == 4 && st[0] == 'n')) {  // a null stats member is absent
        bool sn;
        slen = string_value(st, st_end, &sn, sbytes);
        snull = 0;
      }
      if (!pv_seen) pnull = 1;
      if (!tg_seen) tnull = 1;
      if (pvo) json_map(pvo, e, pv, write);
      if (tgo) json_map(tgo, e, tg, write);
    }
  } else {
    const uint64_t r = a.src_off[act];
    if (a.ck_mtime.def && a.ck_mtime.def[r] == a.ck_mtime.max_def) mt = a.ck_mtime.ival[r];
    if (a.side == 1) {
      size = (a.ck_size.def && a.ck_size.def[r] == a.ck_size.max_def) ? a.ck_size.ival[r] : 0;
    }
    if (a.ck_efm.def && a.ck_efm.def[r] == a.ck_efm.max_def) efm = a.ck_efm.ival[r] != 0;
    if (a.ck_stats.def && a.ck_stats.def[r] == a.ck_stats.max_def) {
      snull = 0;
      slen = a.ck_stats.slen[r];
      if (!write) a.stats_src[i] = a.ck_stats.sptr[r];  // copied by k_gather_bytes after pass 2
    }
    if (write) {
      ck_map<true>(a.ck_pv, r, pv, &pnull);
      ck_map<true>(a.ck_tags, r, tg, &tnull);
    } else {
      ck_map<false>(a.ck_pv, r, pv, &pnull);
      ck_map<false>(a.ck_tags, r, tg, &tnull);
    }
  }
  if (!write) {
    a.size[i] = size;
    a.mtime[i] = mt;
    a.efm[i] = efm;
    a.stats_null[i] = snull;
    a.pv_null[i] = pnull;
    a.tags_null[i] = tnull;
    a.cnt[EXC_STATS][i] = slen;
    a.stats_srclen[i] = json_lane ? 0u : slen;
    a.cnt[EXC_PV_N][i] = pv.n;
    a.cnt[EXC_PV_KB][i] = pv.kb;
    a.cnt[EXC_PV_VB][i] = pv.vb;
    a.cnt[EXC_TAGS_N][i] = tg.n;
    a.cnt[EXC_TAGS_KB][i] = tg.kb;
    a.cnt[EXC_TAGS_VB][i] = tg.vb;
  }
}

// Stage: the launch covers JSON survivors (a replay's export order puts the checkpoint's survivors
// first, launched apart with no line stage, so their blocks keep the occupancy of a small LDS).
template <bool Write, bool Stage>
__global__ void __launch_bounds__(64) k_export(ExportArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t sbuf[Stage ? EXP_STAGE + 32 : 16];
  __shared__ __attribute__((aligned(16))) uint8_t obuf[Write && EXP_OUT ? EXP_OUT : 16];
  const uint64_t k = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const bool live_lane = k < a.npos;
  const uint64_t i = a.pos ? (live_lane ? a.pos[k] : 0ull) : k;
  const uint32_t act = live_lane ? a.idx[i] : 0u;
  const bool json_lane = live_lane && (a.act_flags ? !(a.act_flags[act] & F_FROM_CKPT) : act >= a.ck_rows);
  const uint8_t* gline = nullptr;
  uint32_t glen = 0;
  if (json_lane) {
    const uint8_t* json = a.act_flags && a.src_id ? reinterpret_cast<const uint8_t*>(a.json_bases[a.src_id[act]]) : a.json;
    gline = json + a.src_off[act];
    glen = a.src_len[act];
  }
  const uint32_t head = uint32_t(reinterpret_cast<uintptr_t>(gline) & 15u);
  const uint32_t need = Stage && json_lane && glen <= EXP_STAGE ? (head + glen + 15u) & ~15u : 0u;
  uint32_t tot;
  const uint32_t at = wave_excl_scan(need, &tot);
  const bool staged = need && at + need <= EXP_STAGE;
  if (staged) {
    const uint4* src = reinterpret_cast<const uint4*>(gline - head);
    uint4* dst = reinterpret_cast<uint4*>(sbuf + at);
    const uint32_t nv = need / 16;
    for (uint32_t k0 = 0; k0 < nv; k0 += EXP_BATCH) {
      uint4 v[EXP_BATCH];
#pragma unroll
      for (uint32_t k = 0; k < EXP_BATCH; ++k) v[k] = src[min(k0 + k, nv - 1)];
#pragma unroll
      for (uint32_t k = 0; k < EXP_BATCH; ++k)
        if (k0 + k < nv) dst[k0 + k] = v[k];
    }
  }
  const bool write = Write;
  // pass 2: the block's range of every output stream, placed in obuf when all of them fit
  uint8_t* gdst[XS_N];
  uint32_t esz[XS_N], lofs[XS_N], bytes[XS_N];
  uint64_t lo[XS_N];
  bool ostaged = false;
  if (write) {
    const uint64_t i0 = uint64_t(blockIdx.x) * blockDim.x, i1 = min(i0 + blockDim.x, a.n);  // pass 2: pos is null
    const int cnt_of[XS_N] = {EXC_STATS, EXC_PV_KB, EXC_PV_VB, EXC_TAGS_KB, EXC_TAGS_VB, EXC_PV_N, EXC_PV_N, EXC_PV_N,
                              EXC_TAGS_N, EXC_TAGS_N, EXC_TAGS_N};
    uint8_t* const base[XS_N] = {a.stats_bytes, a.pv_key_bytes, a.pv_val_bytes, a.tags_key_bytes, a.tags_val_bytes,
                                 reinterpret_cast<uint8_t*>(a.pv_key_off + 1), reinterpret_cast<uint8_t*>(a.pv_val_off + 1),
                                 a.pv_val_null, reinterpret_cast<uint8_t*>(a.tags_key_off + 1),
                                 reinterpret_cast<uint8_t*>(a.tags_val_off + 1), a.tags_val_null};
    uint32_t end = 0;
#pragma unroll
    for (int k = 0; k < XS_N; ++k) {
      esz[k] = (k == XS_PVKO || k == XS_PVVO || k == XS_TGKO || k == XS_TGVO) ? 8u : 1u;
      lo[k] = a.off[cnt_of[k]][i0];
      const uint64_t hi = a.off[cnt_of[k]][i1];
      gdst[k] = base[k] + esz[k] * lo[k];
      const uint64_t nb = esz[k] * (hi - lo[k]);
      bytes[k] = uint32_t(min(nb, uint64_t(0xffffffffu)));
      const uint32_t g15 = uint32_t(reinterpret_cast<uintptr_t>(gdst[k]) & 15u);
      lofs[k] = ((end + 15u) & ~15u) + g15;  // the LDS copy shares the destination's 16-byte phase
      end = nb > EXP_OUT ? EXP_OUT + 1 : lofs[k] + bytes[k];
    }
    ostaged = EXP_OUT > 0 && end <= EXP_OUT;
  }
  __syncthreads();
  if (live_lane) {
    const uint8_t* line = staged ? static_cast<const uint8_t*>(sbuf + at + head) : gline;
    MapSink pv{};
    MapSink tg = pv;
    uint8_t* sbytes = nullptr;
    if (write) {
      auto dst = [&](int k, uint64_t first) -> uint8_t* {
        return ostaged ? obuf + lofs[k] + esz[k] * (first - lo[k]) : gdst[k] + esz[k] * (first - lo[k]);
      };
      pv.kbytes = dst(XS_PVK, a.off[EXC_PV_KB][i]);
      pv.vbytes = dst(XS_PVV, a.off[EXC_PV_VB][i]);
      pv.koff = reinterpret_cast<int64_t*>(dst(XS_PVKO, a.off[EXC_PV_N][i]));
      pv.voff = reinterpret_cast<int64_t*>(dst(XS_PVVO, a.off[EXC_PV_N][i]));
      pv.vnull = dst(XS_PVVN, a.off[EXC_PV_N][i]);
      pv.kbase = int64_t(a.off[EXC_PV_KB][i]);
      pv.vbase = int64_t(a.off[EXC_PV_VB][i]);
      tg.kbytes = dst(XS_TGK, a.off[EXC_TAGS_KB][i]);
      tg.vbytes = dst(XS_TGV, a.off[EXC_TAGS_VB][i]);
      tg.koff = reinterpret_cast<int64_t*>(dst(XS_TGKO, a.off[EXC_TAGS_N][i]));
      tg.voff = reinterpret_cast<int64_t*>(dst(XS_TGVO, a.off[EXC_TAGS_N][i]));
      tg.vnull = dst(XS_TGVN, a.off[EXC_TAGS_N][i]);
      tg.kbase = int64_t(a.off[EXC_TAGS_KB][i]);
      tg.vbase = int64_t(a.off[EXC_TAGS_VB][i]);
      sbytes = dst(XS_STATS, a.off[EXC_STATS][i]);
      const uint64_t pe = a.off[EXC_PV_N][i], te = a.off[EXC_TAGS_N][i];
      pv.ksrc = a.pv_ksrc + pe;
      pv.vsrc = a.pv_vsrc + pe;
      pv.klen = a.pv_klen + pe;
      pv.vlen = a.pv_vlen + pe;
      tg.ksrc = a.tags_ksrc + te;
      tg.vsrc = a.tags_vsrc + te;
      tg.klen = a.tags_klen + te;
      tg.vlen = a.tags_vlen + te;
    }
    export_record(a, i, act, json_lane, line, glen, write, pv, tg, sbytes);
  }
  if (!ostaged) return;  // block-uniform
  __syncthreads();
  // store every stream's range: whole aligned 16-byte chunks, bytewise at the two ends
#pragma unroll
  for (int k = 0; k < XS_N; ++k) {
    const uint32_t nb = bytes[k];
    if (!nb) continue;
    const uintptr_t g0 = reinterpret_cast<uintptr_t>(gdst[k]);
    const uintptr_t c0 = g0 & ~uintptr_t(15), c1 = (g0 + nb + 15) & ~uintptr_t(15);
    const uint32_t nch = uint32_t((c1 - c0) / 16);
    for (uint32_t c = threadIdx.x; c < nch; c += blockDim.x) {
      const uintptr_t ca = c0 + 16u * c;
      const int64_t rel = int64_t(ca) - int64_t(g0);  // chunk start relative to the range (may be < 0)
      if (ca >= g0 && ca + 16 <= g0 + nb) {
        *reinterpret_cast<uint4*>(ca) = *reinterpret_cast<const uint4*>(obuf + lofs[k] + rel);
      } else {
        for (uint32_t q = 0; q < 16; ++q) {
          const uintptr_t x = ca + q;
          if (x >= g0 && x < g0 + nb) *reinterpret_cast<uint8_t*>(x) = obuf[lofs[k] + (rel + q)];
        }
      }
    }
  }
}

__global__ void __launch_bounds__(256) k_export_flags(ExportArgs a, uint32_t* json) {
  const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= a.n) return;
  const uint32_t act = a.idx[i];
  json[i] = (a.act_flags ? !(a.act_flags[act] & F_FROM_CKPT) : act >= a.ck_rows) ? 1u : 0u;
}

__global__ void __launch_bounds__(256) k_export_split(const uint32_t* json, const uint64_t* jscan, uint64_t n,
                                                      uint32_t* jpos, uint32_t* cpos) {
  const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const uint64_t j = jscan[i];
  if (json[i]) jpos[j] = uint32_t(i);
  else cpos[i - j] = uint32_t(i);
}

}  // namespace dev

void launch_export(const ExportArgs& a, bool stage, hipStream_t st) {
  const uint64_t m = a.pos ? a.npos : a.n;
  if (!m) return;
  ExportArgs b = a;
  b.npos = m;
  const dim3 g(unsigned((m + 63) / 64));
  if (a.write) DR_LAUNCH((dev::k_export<true, true>), g, dim3(64), 0, st, b);
  else if (stage) DR_LAUNCH((dev::k_export<false, true>), g, dim3(64), 0, st, b);
  else DR_LAUNCH((dev::k_export<false, false>), g, dim3(64), 0, st, b);
}

void launch_export_flags(const ExportArgs& a, uint32_t* json, hipStream_t st) {
  if (a.n) DR_LAUNCH(dev::k_export_flags, dim3(unsigned((a.n + 255) / 256)), dim3(256), 0, st, a, json);
}

void launch_export_split(const uint32_t* json, const uint64_t* jscan, uint64_t n, uint32_t* jpos, uint32_t* cpos,
                         hipStream_t st) {
  if (n) DR_LAUNCH(dev::k_export_split, dim3(unsigned((n + 255) / 256)), dim3(256), 0, st, json, jscan, n, jpos, cpos);
}

}  // namespace dr
