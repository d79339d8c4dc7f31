// K1 line parser: one lane owns one newline-delimited JSON line (one Delta log action) and walks it
// in 16-byte windows. Each window is classified with SWAR byte tests into 16-bit masks (quote,
// backslash, structural, space, control); escapes and string state are resolved on those masks
// with carries from the previous window (the bit-parallel quote/escape method of simdjson, on
// 16-bit lanes), which yields the window's token mask. A table-free DFA then consumes only the
// tokens (brackets, ':', ',', quotes, scalar starts) -- about 45 per add line instead of ~330
// bytes -- validating JSON grammar and extracting the SingleAction envelope (unwrap priority,
// D/actions/actions.scala:523-541) and the add/remove path, size and deletionTimestamp
// (AddFile/RemoveFile field names, D/actions/actions.scala:220-320).
//
// Semantics match Spark's JSON reader over Action.logSchema in PERMISSIVE mode
// (D/DeltaLogFileIndex.scala:67): a line that is not a valid JSON object is a null row (K_ERROR,
// counted, ignored), unknown fields are ignored, a member whose value is null is absent, a repeated
// member keeps its last value (every occurrence is converted when read, as Spark's streaming
// JacksonParser does). The fast instantiation flags the lines it does not decide (a backslash inside
// a key it must match, tab / CR outside strings, nesting deeper than 62) as `hard`; the General
// instantiation of the same walker decides those (k_json_hard re-parses them).
//
// Written for HIP device code and for the host (tests/json_lane_host.cpp builds it with g++ to
// fuzz it against Python's json module).
#pragma once
#include <cstdint>
#include <cstring>

#if defined(__HIPCC__)
#define JL_HD __host__ __device__ __forceinline__
#define JL_UNROLL _Pragma("unroll")
#else
#define JL_HD inline
#define JL_UNROLL
#endif

namespace dr {
namespace jl {

enum : uint8_t { K_NONE = 0, K_ADD = 1, K_REMOVE = 2, K_METADATA = 3, K_TXN = 4, K_PROTOCOL = 5, K_CDC = 6,
                 K_COMMITINFO = 7, K_ERROR = 15 };
enum : uint8_t { F_HAS_DELTS = 1, F_PATH_ESCAPED = 4, F_PATH_NULL = 8 };

struct LineOut {
  uint8_t kind;
  uint8_t flags;
  uint8_t hard;        // undecided: re-parse with the general parser
  uint32_t path_off;   // path content span, relative to the line start
  uint32_t path_len;
  int64_t size;
  int64_t delts;
};

// ---- SWAR byte classes -------------------------------------------------------------------------
// 0x80 in every byte of y that is zero (exact, no cross-byte borrows)
JL_HD uint32_t zbytes(uint32_t y) { return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y | 0x7F7F7F7Fu); }
// 0x80 in every byte of x that is < 0x20
JL_HD uint32_t lt20(uint32_t x) { return ~((x | 0x80808080u) - 0x20202020u) & ~x & 0x80808080u; }
// bits 7, 15, 23, 31 -> bits 0..3
JL_HD uint32_t gather4(uint32_t m) {
  m >>= 7;
  m |= m >> 7;
  m |= m >> 14;
  return m & 0xFu;
}
JL_HD uint32_t prefix_xor16(uint32_t x) {
  x ^= x << 1;
  x ^= x << 2;
  x ^= x << 4;
  x ^= x << 8;
  return x & 0xFFFFu;
}

struct Win {
  uint32_t q, bs, st, sp, ctrl;  // 16-bit masks
};

// Byte classes by two 16-entry nibble tables (class = HI[x >> 4] & LO[x & 15], zero for x >= 0x80),
// looked up four bytes at a time with v_perm_b32: bit 0 '"', bit 1 '\\', bit 2 one of {}[], bit 3
// ' ', bit 4 ':', bit 5 ',', bit 6 a control byte < 0x20. Each class is a product set (high
// nibbles x low nibbles), so the AND of the two lookups has no cross terms.
JL_HD uint32_t perm_b32(uint32_t s0, uint32_t s1, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(s0, s1, sel);
#else
  uint32_t r = 0;
  for (int k = 0; k < 4; ++k) {
    const uint32_t b = (sel >> (8 * k)) & 0xFFu;
    const uint32_t v = b < 4 ? (s1 >> (8 * b)) & 0xFFu : b < 8 ? (s0 >> (8 * (b - 4))) & 0xFFu : b == 0x0C ? 0u : 0xFFu;
    r |= v << (8 * k);
  }
  return r;
#endif
}
constexpr uint32_t CLS_LO0 = 0x40414048u, CLS_LO1 = 0x40404040u, CLS_LO2 = 0x44504040u, CLS_LO3 = 0x40404462u;
constexpr uint32_t CLS_HI0 = 0x10294040u, CLS_HI1 = 0x04000600u;
JL_HD uint32_t class_bytes(uint32_t x) {
  const uint32_t lo = x & 0x0F0F0F0Fu;
  const uint32_t sel = lo & 0x07070707u;
  const uint32_t a = perm_b32(CLS_LO1, CLS_LO0, sel), b = perm_b32(CLS_LO3, CLS_LO2, sel);
  const uint32_t m8 = perm_b32(0u, 0u, ((lo >> 3) & 0x01010101u) | 0x0C0C0C0Cu);  // 0xFF where lo >= 8
  const uint32_t tlo = (m8 & b) | (~m8 & a);
  const uint32_t thi = perm_b32(CLS_HI1, CLS_HI0, (x >> 4) & 0x07070707u);
  const uint32_t neg = perm_b32(0u, 0u, ((x >> 7) & 0x01010101u) | 0x0C0C0C0Cu);  // 0xFF where x >= 0x80
  return tlo & thi & ~neg;
}
JL_HD uint32_t gather_bit(uint32_t r, int c) {  // bit c of each byte -> 4-bit mask
  uint32_t m = (r >> c) & 0x01010101u;
  m |= m >> 7;
  m |= m >> 14;
  return m & 0xFu;
}
// Exchanges the bits at positions p and p + delta wherever `mask` has p (a swap of two bit-index
// bits of the word).
JL_HD uint32_t delta_swap(uint32_t y, uint32_t delta, uint32_t mask) {
  const uint32_t t = (y ^ (y >> delta)) & mask;
  return y ^ t ^ (t << delta);
}

// The window's 16-bit masks from its four class dwords without a per-class bit gather: each byte's
// four tokenizer classes (quote, backslash, structural = {}[]:, , space) as a nibble; two dwords'
// nibbles share a word (byte j: byte j of the first, byte 4 + j of the second in the high nibble),
// so word g holds bit 8j + 4h + c for class c of window byte 8g + 4h + j; exchanging the index
// fields j and c (two delta swaps) makes byte c of word g the class-c mask of bytes 8g..8g+7, and
// two byte permutes assemble the four masks. Control bytes (rare) take the per-class gather.
JL_HD void classify(const uint32_t w[4], Win& m) {
  uint32_t r[4], nib[4];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
  for (int d = 0; d < 4; ++d) {
    r[d] = class_bytes(w[d]);
    nib[d] = (r[d] & 0x0F0F0F0Fu) | (((r[d] >> 2) | (r[d] >> 3)) & 0x04040404u);
  }
  uint32_t y0 = nib[0] | (nib[1] << 4), y1 = nib[2] | (nib[3] << 4);
  y0 = delta_swap(delta_swap(y0, 7, 0x00AA00AAu), 14, 0x0000CCCCu);
  y1 = delta_swap(delta_swap(y1, 7, 0x00AA00AAu), 14, 0x0000CCCCu);
  const uint32_t qb = perm_b32(y1, y0, 0x05010400u), ss = perm_b32(y1, y0, 0x07030602u);
  m.q = qb & 0xFFFFu;
  m.bs = qb >> 16;
  m.st = ss & 0xFFFFu;
  m.sp = ss >> 16;
  m.ctrl = 0;
  if ((r[0] | r[1] | r[2] | r[3]) & 0x40404040u)
    for (int d = 0; d < 4; ++d) m.ctrl |= gather_bit(r[d], 6) << (4 * d);
}

JL_HD uint32_t win_byte(const uint32_t w[4], uint32_t k) {
  const uint32_t d = k >> 2;
  const uint32_t x = d == 0 ? w[0] : d == 1 ? w[1] : d == 2 ? w[2] : w[3];
  return (x >> (8 * (k & 3))) & 0xFFu;
}

JL_HD uint32_t ctz32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return uint32_t(__builtin_ctz(x));
#else
  return uint32_t(__builtin_ctz(x));
#endif
}
JL_HD uint32_t popc32(uint32_t x) { return uint32_t(__builtin_popcount(x)); }

// ---- scalars ----------------------------------------------------------------------------------
enum : uint8_t { SC_BAD = 0, SC_NULL, SC_TRUE, SC_FALSE, SC_INT, SC_NUM };

// ---- keys ----------------------------------------------------------------------------------------
JL_HD bool key_eq(const uint8_t* s, uint32_t n, const char* k, uint32_t kn) {
  if (n != kn) return false;
  for (uint32_t i = 0; i < n; ++i)
    if (s[i] != uint8_t(k[i])) return false;
  return true;
}
// top-level member -> action kind (0: not an action)
JL_HD uint8_t action_key(const uint8_t* s, uint32_t n) {
  switch (n) {
    case 3:
      if (key_eq(s, n, "add", 3)) return K_ADD;
      if (key_eq(s, n, "txn", 3)) return K_TXN;
      if (key_eq(s, n, "cdc", 3)) return K_CDC;
      return 0;
    case 6: return key_eq(s, n, "remove", 6) ? K_REMOVE : 0;
    case 8:
      if (key_eq(s, n, "metaData", 8)) return K_METADATA;
      if (key_eq(s, n, "protocol", 8)) return K_PROTOCOL;
      return 0;
    case 10: return key_eq(s, n, "commitInfo", 10) ? K_COMMITINFO : 0;
    default: return 0;
  }
}
enum : uint8_t { FK_OTHER = 0, FK_PATH, FK_SIZE, FK_DELTS };
JL_HD uint8_t file_key(const uint8_t* s, uint32_t n) {
  if (n == 4) {
    if (key_eq(s, n, "path", 4)) return FK_PATH;
    if (key_eq(s, n, "size", 4)) return FK_SIZE;
    return FK_OTHER;
  }
  if (n == 17 && key_eq(s, n, "deletionTimestamp", 17)) return FK_DELTS;
  return FK_OTHER;
}

// ---- phase 1: tokenizer ----------------------------------------------------------------------------
// A token is one u32: line offset << 16 | aux << 4 | class. Scalars are emitted when their run
// ends, with aux = run length, so phase 2 never scans for a scalar's end.
// T_STRING / T_STRING_ESC: a whole string (offset of its opening quote, body length in aux) -- one
// token instead of an open/close pair when the body is shorter than 4096 bytes.
enum : uint32_t { T_OBJ_OPEN = 0, T_ARR_OPEN, T_OBJ_CLOSE, T_ARR_CLOSE, T_COLON, T_COMMA, T_STR_OPEN,
                  T_STR_CLOSE, T_STR_CLOSE_ESC, T_SCALAR, T_STRING, T_STRING_ESC };
constexpr uint32_t TOK_MAX_LINE = 65535;   // longer lines go to the General walker
constexpr uint32_t TOK_MAX_SCALAR = 4095;

// Up to 20 bytes at s as little-endian words (w[0] holds s[0..3]). Bytes at or past n are
// unspecified: on the device they come from the line buffer (zero-padded past its end), on the
// host they are zero. Three aligned 16-byte loads and funnel shifts, no per-byte loads.
JL_HD void load20(const uint8_t* s, uint32_t n, uint32_t w[5]) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uintptr_t a = reinterpret_cast<uintptr_t>(s);
  const uint4* b = reinterpret_cast<const uint4*>(s - (a & 15u));  // pointer arithmetic keeps an LDS address space
  const uint4 x = b[0], y = b[1], z = b[2];
  const uint32_t v[12] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w, z.x, z.y, z.z, z.w};
  const uint32_t q = uint32_t(a >> 2) & 3u, r = uint32_t(a) & 3u;
  uint32_t u[6];
JL_UNROLL
  for (int i = 0; i < 6; ++i) u[i] = q == 0 ? v[i] : q == 1 ? v[i + 1] : q == 2 ? v[i + 2] : v[i + 3];
JL_UNROLL
  for (int i = 0; i < 5; ++i) w[i] = __builtin_amdgcn_alignbyte(u[i + 1], u[i], r);
#else
  uint8_t t[20] = {0};
  std::memcpy(t, s, n < 20 ? n : 20);
  std::memcpy(w, t, 20);
#endif
}
// 0x80 in each byte of x that is an ASCII digit.
JL_HD uint32_t digit_bytes(uint32_t x) {
  return zbytes((x & 0xF0F0F0F0u) ^ 0x30303030u) & ~(((x & 0x0F0F0F0Fu) + 0x06060606u) << 3) & 0x80808080u;
}
// Value of the 4 ASCII digits of x (first digit in the low byte).
JL_HD uint32_t digits4(uint32_t x) {
  uint32_t d = x - 0x30303030u;
  d = d * 10u + (d >> 8);                          // bytes 0, 2: two-digit values
  return ((d & 0x00FF00FFu) * 0x00640001u) >> 16;  // 100 * hi pair + lo pair
}
JL_HD uint32_t key_mask(uint32_t n) { return n >= 4 ? 0xFFFFFFFFu : (1u << (8 * n)) - 1u; }

// action_key / file_key on word loads (the fast walker's keys are unescaped line bytes).
JL_HD uint8_t action_key_w(const uint8_t* s, uint32_t n) {
  if (n != 3 && n != 6 && n != 8 && n != 10) return 0;
  uint32_t w[5];
  load20(s, n, w);
  const uint32_t a = w[0], b = w[1], c = w[2];
  if (n == 3) {
    const uint32_t t = a & 0xFFFFFFu;
    return t == 0x646461u ? K_ADD : t == 0x6E7874u ? K_TXN : t == 0x636463u ? K_CDC : 0;  // add txn cdc
  }
  if (n == 6) return (a == 0x6F6D6572u && (b & 0xFFFFu) == 0x6576u) ? K_REMOVE : 0;  // remo ve
  if (n == 8) {
    if (a == 0x6174656Du && b == 0x61746144u) return K_METADATA;                    // meta Data
    if (a == 0x746F7270u && b == 0x6C6F636Fu) return K_PROTOCOL;                    // prot ocol
    return 0;
  }
  return (a == 0x6D6D6F63u && b == 0x6E497469u && (c & 0xFFFFu) == 0x6F66u) ? K_COMMITINFO : 0;  // comm itIn fo
}
JL_HD uint8_t file_key_w(const uint8_t* s, uint32_t n) {
  if (n != 4 && n != 17) return FK_OTHER;
  uint32_t w[5];
  load20(s, n, w);
  if (n == 4) return w[0] == 0x68746170u ? FK_PATH : w[0] == 0x657A6973u ? FK_SIZE : FK_OTHER;  // path size
  return (w[0] == 0x656C6564u && w[1] == 0x6E6F6974u && w[2] == 0x656D6954u && w[3] == 0x6D617473u &&
          (w[4] & 0xFFu) == 0x70u) ? FK_DELTS : FK_OTHER;  // dele tion Time stam p
}
// Scalar tokens: null / true / false and plain integers of up to 19 digits decoded from word
// loads; anything else (fractions, exponents, 20+ characters, malformed) takes scalar_class.
JL_HD uint8_t scalar_class(const uint8_t* s, uint32_t L, int64_t* val);
JL_HD uint8_t scalar_fast(const uint8_t* s, uint32_t L, int64_t* val) {
  if (L > 20) return scalar_class(s, L, val);
  uint32_t w[5];
  load20(s, L, w);
  if (L == 4 && w[0] == 0x6C6C756Eu) return SC_NULL;   // null
  if (L == 4 && w[0] == 0x65757274u) return SC_TRUE;   // true
  if (L == 5 && w[0] == 0x736C6166u && (w[1] & 0xFFu) == 0x65u) return SC_FALSE;  // fals e
  const uint32_t neg = (w[0] & 0xFFu) == 0x2Du ? 1u : 0u;
  uint32_t dm = 0;
JL_UNROLL
  for (int d = 0; d < 5; ++d) dm |= gather4(digit_bytes(w[d])) << (4 * d);
  const uint32_t need = ((1u << L) - 1u) & ~neg;
  const uint32_t nd = L - neg;
  if (nd == 0 || nd > 19 || (dm & need) != need) return scalar_class(s, L, val);
  if (neg) {
JL_UNROLL
    for (int i = 0; i < 4; ++i) w[i] = (w[i] >> 8) | (w[i + 1] << 24);
    w[4] >>= 8;
  }
  if (nd > 1 && (w[0] & 0xFFu) == 0x30u) return SC_BAD;  // leading zero
  const uint32_t g = nd >> 2, r = nd & 3u;
  uint64_t v = 0;
JL_UNROLL
  for (uint32_t k = 0; k < 4; ++k)
    if (k < g) v = v * 10000ull + digits4(w[k]);
  if (r) {
    const uint32_t x = g == 0 ? w[0] : g == 1 ? w[1] : g == 2 ? w[2] : g == 3 ? w[3] : w[4];
    const uint32_t sh = 8u * (4u - r);
    v = v * (r == 1 ? 10ull : r == 2 ? 100ull : 1000ull) + digits4((x << sh) | (0x30303030u >> (32u - sh)));
  }
  // LongType: VALUE_NUMBER_INT within [-2^63, 2^63-1] (19 digits fit in 64 bits unsigned)
  if (v > (neg ? 0x8000000000000000ull : 0x7FFFFFFFFFFFFFFFull)) return SC_NUM;
  *val = neg ? int64_t(0ull - v) : int64_t(v);
  return SC_INT;
}

JL_HD uint32_t tok_make(uint32_t off, uint32_t aux, uint32_t cls) { return (off << 16) | (aux << 4) | cls; }
JL_HD uint32_t tok_off(uint32_t t) { return t >> 16; }
JL_HD uint32_t tok_aux(uint32_t t) { return (t >> 4) & 0xFFFu; }
JL_HD uint32_t tok_cls(uint32_t t) { return t & 0xFu; }

enum : uint8_t { ST_OK = 0, ST_BAD = 1, ST_HARD = 2 };

struct Tokenizer {
  uint32_t esc_carry = 0, in_str = 0, sc_carry = 0;
  uint32_t pend_bs = 0;      // a backslash in the string still open
  uint32_t sc_start = 0;     // line offset where the open scalar run began
  uint32_t sc_bytes = 0;     // scalar bytes seen (each must belong to a validated scalar)
  uint32_t str_open = 0;     // line offset of the open string's quote
  uint8_t status = ST_OK;
};

// Loads the aligned 16-byte window at a (a is 16-byte aligned; the buffer is readable there).
JL_HD void load_window(const uint8_t* a, uint32_t w[4]) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint4 v = *reinterpret_cast<const uint4*>(a);
  w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
#else
  std::memcpy(w, a, 16);
#endif
}

// Tokenizes the window whose byte 0 has line offset `lo` (may be negative for the first window).
template <bool General, typename Emit>
JL_HD void tokenize_window(const uint8_t* p, uint32_t n, const uint32_t w[4], int32_t lo, Tokenizer& tz,
                           Emit&& emit) {
  uint32_t valid = 0xFFFFu;
  if (lo < 0) valid &= 0xFFFFu << uint32_t(-lo);
  if (lo + 16 > int32_t(n)) valid &= (1u << uint32_t(int32_t(n) - lo)) - 1u;
  Win m;
#if defined(DR_JL_EXP) && DR_JL_EXP >= 3
  // timing experiment only (scripts/build_variant.sh): the window loads without their classification
  // (every byte a space: no tokens, no state), to split K1's cost into loads and SWAR classes
  {
    uint32_t x = w[0] ^ w[1] ^ w[2] ^ w[3];
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(x));
#endif
    m.q = 0; m.bs = 0; m.st = 0; m.ctrl = 0;
    m.sp = 0xFFFFu | (x & 0u);
  }
#else
  classify(w, m);
#endif
  m.q &= valid; m.bs &= valid; m.st &= valid; m.sp &= valid; m.ctrl &= valid;
  // escaped bytes: those preceded by an odd run of backslashes (carry from the previous window)
  uint32_t escaped = 0;
  if (m.bs | tz.esc_carry) {
    const uint32_t bsn = m.bs & ~tz.esc_carry;
    const uint32_t follows = ((bsn << 1) | tz.esc_carry) & 0xFFFFu;
    const uint32_t odd_starts = bsn & ~0x5555u & ~follows;
    const uint32_t sum = odd_starts + bsn;
    escaped = (0x5555u ^ ((sum << 1) & 0xFFFFu)) & follows;
    tz.esc_carry = (sum >> 16) & 1u;
  }
  const uint32_t quote = m.q & ~escaped;
  const uint32_t instr = prefix_xor16(quote) ^ (tz.in_str ? 0xFFFFu : 0u);
  tz.in_str = (instr >> 15) & 1u;
  if (m.ctrl & instr) { tz.status = ST_BAD; return; }  // control byte inside a string
  uint32_t ws = m.sp;
  if (m.ctrl & ~instr) {
    if (!General) { tz.status = ST_HARD; return; }
    // tab and CR are whitespace between tokens; any other control byte there is malformed
    uint32_t tabcr = 0;
    for (int d = 0; d < 4; ++d)
      tabcr |= gather4(zbytes(w[d] ^ 0x09090909u) | zbytes(w[d] ^ 0x0D0D0D0Du)) << (4 * d);
    if ((m.ctrl & ~instr) & ~tabcr) { tz.status = ST_BAD; return; }
    ws |= m.ctrl & ~instr;
  }
  // escape sequences other than \" and \\ must be one of \/ \b \f \n \r \t \uXXXX
  uint32_t oddesc = escaped & ~(m.q | m.bs) & valid;
  while (oddesc) {
    const uint32_t k = ctz32(oddesc);
    oddesc &= oddesc - 1;
    const uint32_t c = win_byte(w, k);
    if (c == 'u') {
      const uint32_t off = uint32_t(lo + int32_t(k));
      if (off + 4 >= n) { tz.status = ST_BAD; return; }
      for (uint32_t h = 1; h <= 4; ++h) {
        const uint32_t x = p[off + h] | 0x20u;
        if (!((x >= '0' && x <= '9') || (x >= 'a' && x <= 'f'))) { tz.status = ST_BAD; return; }
      }
    } else if (!(c == '/' || c == 'b' || c == 'f' || c == 'n' || c == 'r' || c == 't')) {
      tz.status = ST_BAD;
      return;
    }
  }
  const uint32_t st = m.st & ~instr;
  const uint32_t sc = valid & ~instr & ~quote & ~st & ~ws;
  tz.sc_bytes += popc32(sc);
  // a scalar run that ended at the previous window's last byte
  if (tz.sc_carry && !(sc & 1u)) {
    const uint32_t end = uint32_t(lo);  // one past the run
    const uint32_t len = end - tz.sc_start;
    if (len > TOK_MAX_SCALAR) { tz.status = ST_BAD; return; }
    emit(tok_make(tz.sc_start, len, T_SCALAR));
  }
  const uint32_t sc_begin = sc & ~(((sc << 1) | tz.sc_carry) & 0xFFFFu);
  const uint32_t sc_end = sc & ~(sc >> 1) & 0x7FFFu;  // run ends inside this window
  tz.sc_carry = (sc >> 15) & 1u;
  // Opening quotes take no loop step: a closing quote finds its string's opening quote as the highest
  // opening-quote bit below it (or the one carried from an earlier window), so only closing quotes,
  // structurals and scalar ends are visited (about two thirds of the steps of a writer's add line).
  const uint32_t oq_all = quote & instr;
  uint32_t tok = st | (quote & ~instr) | sc_end;
#if defined(DR_JL_EXP) && DR_JL_EXP >= 2
  tok = 0;  // timing experiment only (scripts/build_variant.sh): masks without token emission
#endif
  uint32_t begins = sc_begin;
  while (tok) {
    const uint32_t k = ctz32(tok);
    tok &= tok - 1;
    const uint32_t off = uint32_t(lo + int32_t(k));
    const uint32_t bit = 1u << k;
    if (quote & bit) {  // a closing quote
      const uint32_t below = bit - 1u;
      const uint32_t oq = oq_all & below;
      uint32_t open_off;
      bool has_bs;
      if (oq) {
        const uint32_t ok = 31u - uint32_t(__builtin_clz(oq));
        open_off = uint32_t(lo + int32_t(ok));
        has_bs = (m.bs & below & ~((2u << ok) - 1u)) != 0;
      } else {
        open_off = tz.str_open;
        has_bs = tz.pend_bs || (m.bs & below) != 0;
      }
      const uint32_t len = off - open_off - 1u;
      if (len < 4096u) {
        emit(tok_make(open_off, len, has_bs ? T_STRING_ESC : T_STRING));
      } else {
        emit(tok_make(open_off, 0, T_STR_OPEN));
        emit(tok_make(off, 0, has_bs ? T_STR_CLOSE_ESC : T_STR_CLOSE));
      }
    } else if (st & bit) {
      const uint32_t c = win_byte(w, k);
      const uint32_t cls = c == ':' ? T_COLON : c == ',' ? T_COMMA
                         : ((c & 2u) ? T_OBJ_OPEN : T_OBJ_CLOSE) + ((c & 0x20u) ? 0u : 1u);
      emit(tok_make(off, 0, cls));
    } else {  // a scalar run ends at k
      // its start is in this window (a begin bit at or below k) or carried from an earlier one
      const uint32_t bb = begins & ((bit << 1) - 1u);
      uint32_t start = tz.sc_start;
      if (bb) {
        const uint32_t kb = 31u - uint32_t(__builtin_clz(bb));
        start = uint32_t(lo + int32_t(kb));
        begins &= ~((bit << 1) - 1u);
      }
      const uint32_t len = off + 1 - start;
      if (len > TOK_MAX_SCALAR) { tz.status = ST_BAD; return; }
      emit(tok_make(start, len, T_SCALAR));
    }
  }
  if (begins) tz.sc_start = uint32_t(lo + int32_t(ctz32(begins)));  // a run that continues
  // a string still open at the window end: where it opened, and whether it holds a backslash yet
  if (tz.in_str) {
    if (oq_all) {
      const uint32_t ok = 31u - uint32_t(__builtin_clz(oq_all));
      tz.str_open = uint32_t(lo + int32_t(ok));
      tz.pend_bs = (m.bs & ~((2u << ok) - 1u)) != 0;
    } else {
      tz.pend_bs = tz.pend_bs || m.bs != 0;
    }
  }
}

// Line end: a scalar running to the last byte.
template <typename Emit>
JL_HD void tokenize_end(uint32_t n, Tokenizer& tz, Emit&& emit) {
  if (tz.status == ST_OK && tz.in_str) emit(tok_make(tz.str_open, 0, T_STR_OPEN));  // never closed
  if (tz.status == ST_OK && tz.sc_carry) {
    const uint32_t len = n - tz.sc_start;
    if (len > TOK_MAX_SCALAR) { tz.status = ST_BAD; return; }
    emit(tok_make(tz.sc_start, len, T_SCALAR));
    tz.sc_carry = 0;
  }
}

// ---- phase 2: grammar + SingleAction extraction ----------------------------------------------------
enum : uint8_t { S_START = 0, S_OBJ_FIRST, S_KEY, S_COLON, S_VALUE, S_ARR_FIRST, S_AFTER, S_DONE, S_STR };

struct FileObj {
  uint32_t path_off, path_len;
  int64_t size, delts;
  uint8_t flags;  // F_HAS_DELTS | F_PATH_ESCAPED | F_PATH_NULL
};

constexpr uint32_t GEN_MAX_DEPTH = 1024;  // General mode: deeper nesting is an error row

template <bool General>
struct Dfa {
  uint8_t state = S_START, key_role = 0, k1 = 0, k2 = 0, status = ST_OK;
  bool in_file = false;
  uint32_t depth = 0;
  uint64_t arr_bits = 0;  // bit d: the container at depth d is an array (d < 64)
  uint64_t deep_bits[General ? GEN_MAX_DEPTH / 64 : 1];  // General mode only
  uint32_t present = 0;   // bit per action kind whose (last) value is non-null
  uint32_t str_start = 0;
  uint32_t sc_checked = 0;
  FileObj cur{0, 0, 0, 0, F_PATH_NULL}, fadd{0, 0, 0, 0, F_PATH_NULL}, frm{0, 0, 0, 0, F_PATH_NULL};

  JL_HD bool is_arr(uint32_t d) const {
    if constexpr (General) {
      if (d >= 64) return ((deep_bits[d >> 6] >> (d & 63)) & 1ull) != 0;
    }
    return ((arr_bits >> (d & 63)) & 1ull) != 0;
  }
  JL_HD void set_arr(uint32_t d, bool a) {
    if constexpr (General) {
      if (d >= 64) {
        uint64_t& word = deep_bits[d >> 6];
        word = a ? (word | (1ull << (d & 63))) : (word & ~(1ull << (d & 63)));
        return;
      }
    }
    const uint64_t bit = 1ull << (d & 63);
    arr_bits = a ? (arr_bits | bit) : (arr_bits & ~bit);
  }
};

// Unescapes a short JSON string body (a member name) into buf; returns its length, or 0xFFFFFFFF if
// it does not fit (no key this walker matches is longer than 17 bytes).
JL_HD uint32_t unescape_key(const uint8_t* s, uint32_t n, uint8_t* buf, uint32_t cap) {
  uint32_t o = 0;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t c = s[i];
    if (c == '\\' && i + 1 < n) {
      const uint32_t e = s[++i];
      if (e == 'u' && i + 4 < n) {
        uint32_t cp = 0;
        for (int h = 0; h < 4; ++h) {
          const uint32_t x = s[++i] | 0x20u;
          cp = cp * 16 + (x <= '9' ? x - '0' : x - 'a' + 10);
        }
        if (cp >= 0x80) return 0xFFFFFFFFu;  // no matched key holds non-ASCII characters
        c = cp;
      } else {
        c = e == 'b' ? 8 : e == 'f' ? 12 : e == 'n' ? 10 : e == 'r' ? 13 : e == 't' ? 9 : e;
      }
    }
    if (o >= cap) return 0xFFFFFFFFu;
    buf[o++] = uint8_t(c);
  }
  return o;
}

// Validates a scalar of known extent (JSON number grammar without leading zeros, or a literal).
JL_HD uint8_t scalar_class(const uint8_t* s, uint32_t L, int64_t* val) {
  if (L == 4 && s[0] == 'n' && s[1] == 'u' && s[2] == 'l' && s[3] == 'l') return SC_NULL;
  if (L == 4 && s[0] == 't' && s[1] == 'r' && s[2] == 'u' && s[3] == 'e') return SC_TRUE;
  if (L == 5 && s[0] == 'f' && s[1] == 'a' && s[2] == 'l' && s[3] == 's' && s[4] == 'e') return SC_FALSE;
  uint32_t i = 0;
  const bool neg = L > 0 && s[0] == '-';
  if (neg) ++i;
  if (i >= L || s[i] < '0' || s[i] > '9') return SC_BAD;
  uint64_t v = 0;
  bool ovf = false;
  if (s[i] == '0') {
    ++i;
  } else {
    while (i < L && s[i] >= '0' && s[i] <= '9') {
      const uint64_t dg = uint64_t(s[i] - '0');
      if (v > (0xFFFFFFFFFFFFFFFFull - dg) / 10ull) ovf = true;
      v = v * 10ull + dg;
      ++i;
    }
  }
  bool integral = true;
  if (i < L && s[i] == '.') {
    integral = false;
    ++i;
    const uint32_t f0 = i;
    while (i < L && s[i] >= '0' && s[i] <= '9') ++i;
    if (i == f0) return SC_BAD;
  }
  if (i < L && (s[i] == 'e' || s[i] == 'E')) {
    integral = false;
    ++i;
    if (i < L && (s[i] == '+' || s[i] == '-')) ++i;
    const uint32_t x0 = i;
    while (i < L && s[i] >= '0' && s[i] <= '9') ++i;
    if (i == x0) return SC_BAD;
  }
  if (i != L) return SC_BAD;
  if (!integral) return SC_NUM;
  // LongType: VALUE_NUMBER_INT within [-2^63, 2^63-1]
  if (ovf || v > (neg ? 0x8000000000000000ull : 0x7FFFFFFFFFFFFFFFull)) return SC_NUM;
  *val = neg ? int64_t(0ull - v) : int64_t(v);
  return SC_INT;
}

// String open / close steps of the DFA (a T_STRING token runs both).
template <bool General>
JL_HD bool dfa_str_open(uint32_t off, Dfa<General>& d) {
  const uint8_t stt = d.state;
  if (stt == S_OBJ_FIRST || stt == S_KEY) d.key_role = 1;
  else if (stt == S_VALUE || stt == S_ARR_FIRST) d.key_role = 0;
  else { d.status = ST_BAD; return false; }
  d.state = S_STR;
  d.str_start = off + 1;
  return true;
}
template <bool General>
JL_HD void dfa_str_close(const uint8_t* p, uint32_t off, bool has_bs, Dfa<General>& d) {
  const uint8_t* s = p + d.str_start;
  const uint32_t sl = off - d.str_start;
  if (d.key_role) {
    if (d.depth == 1 || (d.depth == 2 && d.in_file)) {
      if (has_bs) {
        if constexpr (!General) {
          d.status = ST_HARD;
          return;
        } else {
          uint8_t kb[24];
          const uint32_t kl = unescape_key(s, sl, kb, 24);
          if (d.depth == 1) d.k1 = kl == 0xFFFFFFFFu ? 0 : action_key(kb, kl);
          else d.k2 = kl == 0xFFFFFFFFu ? FK_OTHER : file_key(kb, kl);
        }
      } else {
        if (d.depth == 1) d.k1 = action_key_w(s, sl);
        else d.k2 = file_key_w(s, sl);
      }
    }
    d.state = S_COLON;
  } else {
    if (d.depth == 1) {
      if (d.k1 == K_ADD || d.k1 == K_REMOVE) { d.status = ST_BAD; return; }  // struct from a string
      if (d.k1) d.present |= 1u << d.k1;
    } else if (d.depth == 2 && d.in_file) {
      if (d.k2 == FK_PATH) {
        d.cur.path_off = d.str_start;
        d.cur.path_len = sl;
        d.cur.flags = uint8_t((d.cur.flags & ~(F_PATH_NULL | F_PATH_ESCAPED)) | (has_bs ? F_PATH_ESCAPED : 0));
      } else if (d.k2 == FK_SIZE || d.k2 == FK_DELTS) {
        d.status = ST_BAD;  // LongType from a string token
        return;
      }
    }
    d.state = S_AFTER;
  }
}

// One token through the JSON grammar and the Action.logSchema extraction.
template <bool General>
JL_HD void dfa_token(const uint8_t* p, uint32_t tok, Dfa<General>& d) {
  const uint32_t cls = tok_cls(tok), off = tok_off(tok);
  const uint8_t stt = d.state;
  if (cls >= T_STRING) {
    if (dfa_str_open(off, d)) dfa_str_close(p, off + 1 + tok_aux(tok), cls == T_STRING_ESC, d);
    return;
  }
  if (cls == T_STR_OPEN) {
    dfa_str_open(off, d);
    return;
  }
  if (cls == T_STR_CLOSE || cls == T_STR_CLOSE_ESC) {
    dfa_str_close(p, off, cls == T_STR_CLOSE_ESC, d);
    return;
  }
  if (cls == T_SCALAR) {
    if (!(stt == S_VALUE || stt == S_ARR_FIRST)) { d.status = ST_BAD; return; }
    const uint32_t L = tok_aux(tok);
    int64_t v = 0;
    const uint8_t sc = scalar_fast(p + off, L, &v);
    if (sc == SC_BAD) { d.status = ST_BAD; return; }
    d.sc_checked += L;
    if (d.depth == 1) {
      if (sc == SC_NULL) {
        if (d.k1) d.present &= ~(1u << d.k1);
        if (d.k1 == K_ADD) d.fadd = FileObj{0, 0, 0, 0, F_PATH_NULL};
        if (d.k1 == K_REMOVE) d.frm = FileObj{0, 0, 0, 0, F_PATH_NULL};
      } else {
        if (d.k1 == K_ADD || d.k1 == K_REMOVE) { d.status = ST_BAD; return; }
        if (d.k1) d.present |= 1u << d.k1;
      }
    } else if (d.depth == 2 && d.in_file) {
      if (d.k2 == FK_PATH) {
        if (sc != SC_NULL) { d.status = ST_BAD; return; }
        d.cur.path_off = 0;
        d.cur.path_len = 0;
        d.cur.flags = uint8_t((d.cur.flags & ~F_PATH_ESCAPED) | F_PATH_NULL);
      } else if (d.k2 == FK_SIZE) {
        if (sc == SC_NULL) d.cur.size = 0;
        else if (sc == SC_INT) d.cur.size = v;
        else { d.status = ST_BAD; return; }
      } else if (d.k2 == FK_DELTS) {
        if (sc == SC_NULL) { d.cur.delts = 0; d.cur.flags &= ~F_HAS_DELTS; }
        else if (sc == SC_INT) { d.cur.delts = v; d.cur.flags |= F_HAS_DELTS; }
        else { d.status = ST_BAD; return; }
      }
    }
    d.state = S_AFTER;
    return;
  }
  if (cls == T_COLON) {
    if (stt != S_COLON) { d.status = ST_BAD; return; }
    d.state = S_VALUE;
    return;
  }
  if (cls == T_COMMA) {
    if (stt != S_AFTER || d.depth == 0) { d.status = ST_BAD; return; }
    d.state = d.is_arr(d.depth) ? S_VALUE : S_KEY;
    return;
  }
  if (cls == T_OBJ_OPEN || cls == T_ARR_OPEN) {
    const bool arr = cls == T_ARR_OPEN;
    if (!(stt == S_VALUE || stt == S_ARR_FIRST || (stt == S_START && !arr))) { d.status = ST_BAD; return; }
    if (d.depth == 2 && d.in_file && d.k2 != FK_OTHER) { d.status = ST_BAD; return; }  // path/size/delts container
    if (d.depth == 1 && (d.k1 == K_ADD || d.k1 == K_REMOVE)) {
      if (arr) { d.status = ST_BAD; return; }
      d.in_file = true;
      d.k2 = FK_OTHER;
      d.cur = FileObj{0, 0, 0, 0, F_PATH_NULL};
    }
    if (d.depth >= 62) {
      if (!General) { d.status = ST_HARD; return; }
      if (d.depth + 1 >= GEN_MAX_DEPTH) { d.status = ST_BAD; return; }
    }
    ++d.depth;
    d.set_arr(d.depth, arr);
    d.state = arr ? S_ARR_FIRST : S_OBJ_FIRST;
    return;
  }
  // T_OBJ_CLOSE / T_ARR_CLOSE
  {
    const bool arr = cls == T_ARR_CLOSE;
    if (d.depth == 0) { d.status = ST_BAD; return; }
    const bool top_arr = d.is_arr(d.depth);
    if (arr != top_arr || !(stt == S_AFTER || stt == (arr ? S_ARR_FIRST : S_OBJ_FIRST))) { d.status = ST_BAD; return; }
    if (d.depth == 2) {  // the value of a top-level member closes
      if (d.in_file) {
        // field-wise selects (a struct copy to one of two destinations would go through scratch)
        const bool ad = d.k1 == K_ADD;
        d.fadd.path_off = ad ? d.cur.path_off : d.fadd.path_off;
        d.fadd.path_len = ad ? d.cur.path_len : d.fadd.path_len;
        d.fadd.size = ad ? d.cur.size : d.fadd.size;
        d.fadd.delts = ad ? d.cur.delts : d.fadd.delts;
        d.fadd.flags = ad ? d.cur.flags : d.fadd.flags;
        d.frm.path_off = ad ? d.frm.path_off : d.cur.path_off;
        d.frm.path_len = ad ? d.frm.path_len : d.cur.path_len;
        d.frm.size = ad ? d.frm.size : d.cur.size;
        d.frm.delts = ad ? d.frm.delts : d.cur.delts;
        d.frm.flags = ad ? d.frm.flags : d.cur.flags;
        d.in_file = false;
      }
      if (d.k1) d.present |= 1u << d.k1;
    }
    --d.depth;
    d.state = d.depth == 0 ? S_DONE : S_AFTER;
  }
}

template <bool General>
JL_HD void dfa_finish(const Tokenizer& tz, const Dfa<General>& d, LineOut& out) {
  out.kind = K_NONE;
  out.flags = 0;
  out.hard = 0;
  out.path_off = 0;
  out.path_len = 0;
  out.size = 0;
  out.delts = 0;
  if (tz.status == ST_HARD || d.status == ST_HARD) { out.hard = 1; return; }
  if (tz.status == ST_OK && d.status == ST_OK && d.state == S_START && tz.sc_bytes == 0) return;  // blank
  if (tz.status != ST_OK || d.status != ST_OK || d.state != S_DONE || tz.sc_bytes != d.sc_checked) {
    out.kind = K_ERROR;
    return;
  }
  // unwrap priority add > remove > metaData > txn > protocol > cdc > commitInfo
  const uint32_t pr = d.present;
  out.kind = (pr & (1u << K_ADD)) ? K_ADD : (pr & (1u << K_REMOVE)) ? K_REMOVE
           : (pr & (1u << K_METADATA)) ? K_METADATA : (pr & (1u << K_TXN)) ? K_TXN
           : (pr & (1u << K_PROTOCOL)) ? K_PROTOCOL : (pr & (1u << K_CDC)) ? K_CDC
           : (pr & (1u << K_COMMITINFO)) ? K_COMMITINFO : K_NONE;
  if (out.kind == K_ADD || out.kind == K_REMOVE) {
    const bool ad = out.kind == K_ADD;  // field-wise selects keep both records in registers
    out.flags = ad ? d.fadd.flags : d.frm.flags;
    out.path_off = ad ? d.fadd.path_off : d.frm.path_off;
    out.path_len = ad ? d.fadd.path_len : d.frm.path_len;
    out.size = ad ? d.fadd.size : d.frm.size;
    out.delts = ad ? d.fadd.delts : d.frm.delts;
  }
}

// Whole-line walk (phases interleaved per window): the host reference and the General kernel.
template <bool General>
JL_HD void parse_line_t(const uint8_t* p, uint32_t n, LineOut& out) {
  Tokenizer tz;
  Dfa<General> d;
  if (n > TOK_MAX_LINE) {
    if (!General) { out = LineOut{0, 0, 1, 0, 0, 0, 0}; return; }
  }
  const uintptr_t pa = reinterpret_cast<uintptr_t>(p);
  const uint8_t* base = p - (pa & 15u);
  const uint32_t o0 = uint32_t(pa & 15);
  const uint32_t nwin = (o0 + n + 15) >> 4;
  auto step = [&](uint32_t t) {
    if (d.status == ST_OK) dfa_token<General>(p, t, d);
  };
  for (uint32_t j = 0; j < nwin && tz.status == ST_OK && d.status == ST_OK; ++j) {
    uint32_t w[4];
    load_window(base + 16u * j, w);
    tokenize_window<General>(p, n, w, int32_t(16u * j) - int32_t(o0), tz, step);
  }
  tokenize_end(n, tz, step);
  dfa_finish<General>(tz, d, out);
}

JL_HD void parse_line(const uint8_t* p, uint32_t n, LineOut& out) { parse_line_t<false>(p, n, out); }
JL_HD void parse_line_general(const uint8_t* p, uint32_t n, LineOut& out) { parse_line_t<true>(p, n, out); }

}  // namespace jl
}  // namespace dr
