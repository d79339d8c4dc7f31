// K1: newline-delimited JSON commit files -> action records (replaces Spark's JsonFileFormat +
// Jackson over Action.logSchema, D/DeltaLogFileIndex.scala:67, D/Snapshot.scala:244-263).
//
// Stage 1 (k_json_index / k_json_place): a structural index of the newline bytes, built from
// 16-byte vector loads in one pass; a raw '\n' can never sit inside a JSON string, so every newline is a line
// boundary. Stage 2 (k_json_lines): one lane per line walks the line in 16-byte SWAR windows
// (json_lane.h: bit-parallel quote/escape masks, token DFA), classifies the SingleAction envelope
// with unwrap priority (D/actions/actions.scala:523-541), pulls add/remove path / size /
// deletionTimestamp and hashes the path (K3's xxh64) while its bytes are in cache.
#include <cstdlib>
#include <type_traits>

#include "dev_common.h"
#include "kernels.h"
#include "json_lane.h"
#include "canon.h"
#include "wave.h"
#include "ix_dev.h"

namespace dr {
namespace dev {

// LDS index checks of the tape kernels (build_tape, tape_lines, k_apply_commit, k_json_lines<true>):
// built with -DDR_BOUNDS_CHECK (delta_amd/libdeltareplay_bounds.so, tests/test_gpu_bounds.py) every
// computed stage / tape index is compared with its array's extent before use; a miss counts in
// dr_lds_bounds_hits and prints the site (a ds_read out of the workgroup's allocation reads 0 instead
// of faulting, so an over-read would otherwise only show as a wrong token). Compiled out otherwise.
#ifdef DR_BOUNDS_CHECK
__device__ unsigned int dr_lds_bounds_hits;
#define DR_LDS_CHECK(ok, site, idx, lim)                                                                       \
  do {                                                                                                       \
    if (!(ok) && atomicAdd(&dr_lds_bounds_hits, 1u) < 32u)                                                   \
      printf("LDS-BOUNDS %s: index %llu, extent %llu (block %u thread %u)\n", site, (unsigned long long)(idx), \
             (unsigned long long)(lim), blockIdx.x, threadIdx.x);                                           \
  } while (0)
#else
#define DR_LDS_CHECK(ok, site, idx, lim) \
  do {                                   \
  } while (0)
#endif

constexpr int JSON_THREADS = 256;
constexpr int JSON_BYTES_PER_THREAD = 64;
constexpr int JSON_BYTES_PER_BLOCK = JSON_THREADS * JSON_BYTES_PER_THREAD;

// 0x80 in every byte of w that equals '\n'. Exact per byte: the shorter (x - 0x01..) & ~x test
// also flags a 0x0b byte above a newline (the borrow crosses into it), which split lines at "\n\v"
// (found by the device walker fuzz, tests/test_gpu_edge_cases.py).
__device__ __forceinline__ uint32_t nl_bytes(uint32_t w) {
  const uint32_t y = w ^ 0x0a0a0a0au;
  return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y | 0x7F7F7F7Fu);
}
__device__ __forceinline__ uint32_t count_nl_word(uint32_t w) { return __builtin_popcount(nl_bytes(w)); }

// Stage 1 reads the JSON once: every 16 KiB block finds its newlines (64 bytes per thread, a
// block-wide scan of the per-thread counts ranks them) and stores their block-relative positions
// as u16 in the block's slot of JSON_SLOT entries, plus its count. After the scan of the counts,
// k_json_place expands the slots into the global newline array (12 B per line of traffic instead
// of a second pass over the bytes); a block with more than JSON_SLOT newlines (lines averaging
// under 32 bytes) is re-scanned there.
constexpr int JSON_SLOT = 512;

// Block-wide ranks of this thread's newlines; calls put(rank, block-relative position) for each.
template <typename Put>
__device__ __forceinline__ uint32_t block_newlines(const uint8_t* __restrict__ buf, uint64_t len, uint64_t blk,
                                                   Put put) {
  __shared__ uint32_t wsum[JSON_THREADS / 64];
  const uint32_t rel0 = threadIdx.x * JSON_BYTES_PER_THREAD;
  const uint64_t base = blk * JSON_BYTES_PER_BLOCK + rel0;
  uint32_t words[16];
  uint32_t c = 0;
  const bool full = base + JSON_BYTES_PER_THREAD <= len;
  if (full) {
    const uint4* p = reinterpret_cast<const uint4*>(buf + base);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint4 v = p[i];
      words[4 * i] = v.x; words[4 * i + 1] = v.y; words[4 * i + 2] = v.z; words[4 * i + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) c += count_nl_word(words[i]);
  } else {
    for (uint64_t i = base; i < len; ++i) c += buf[i] == '\n';
  }
  // block-wide exclusive scan of c
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t incl = c;
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  uint32_t woff = 0, total = 0;
  for (int i = 0; i < JSON_THREADS / 64; ++i) {
    woff += i < wv ? wsum[i] : 0u;
    total += wsum[i];
  }
  uint32_t r = woff + incl - c;
  if (full) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      uint32_t t = nl_bytes(words[i]);
      while (t) {
        put(r++, rel0 + 4 * i + (__builtin_ctz(t) >> 3));
        t &= t - 1;
      }
    }
  } else {
    for (uint64_t i = base; i < len; ++i)
      if (buf[i] == '\n') put(r++, uint32_t(i - blk * JSON_BYTES_PER_BLOCK));
  }
  return total;
}

__global__ void __launch_bounds__(JSON_THREADS) k_json_index(const uint8_t* __restrict__ buf, uint64_t len,
                                                            uint32_t* __restrict__ block_counts,
                                                            uint16_t* __restrict__ slots) {
  uint16_t* slot = slots + uint64_t(blockIdx.x) * JSON_SLOT;
  const uint32_t total = block_newlines(buf, len, blockIdx.x, [&](uint32_t r, uint32_t pos) {
    if (r < uint32_t(JSON_SLOT)) slot[r] = uint16_t(pos);
  });
  if (threadIdx.x == 0) block_counts[blockIdx.x] = total;
}

// A segment of one index block (a streamed commit): the newline positions written directly (no
// slots, no scan, no k_json_place), off2 = {0, count}, and the first nzero words of `zero` cleared
// (the parse counters: one launch instead of a fill, an index, three scans and a placement).
__global__ void __launch_bounds__(JSON_THREADS) k_json_index1(const uint8_t* __restrict__ buf, uint64_t len,
                                                             uint64_t* __restrict__ nl, uint64_t* __restrict__ off2,
                                                             uint64_t* __restrict__ zero, uint32_t nzero) {
  if (threadIdx.x < nzero) zero[threadIdx.x] = 0;
  const uint32_t total = block_newlines(buf, len, 0, [&](uint32_t r, uint32_t pos) { nl[r] = pos; });
  if (threadIdx.x == 0) {
    off2[0] = 0;
    off2[1] = total;
  }
}

// Writes the byte position of every newline, in order: nl[block_off[b] + rank] = pos.
__global__ void __launch_bounds__(JSON_THREADS) k_json_place(const uint8_t* __restrict__ buf, uint64_t len,
                                                            const uint32_t* __restrict__ block_counts,
                                                            const uint64_t* __restrict__ block_off,
                                                            const uint16_t* __restrict__ slots,
                                                            uint64_t* __restrict__ nl) {
  const uint32_t cnt = block_counts[blockIdx.x];
  const uint64_t base = uint64_t(blockIdx.x) * JSON_BYTES_PER_BLOCK;
  uint64_t* out = nl + block_off[blockIdx.x];
  if (cnt <= uint32_t(JSON_SLOT)) {
    const uint16_t* slot = slots + uint64_t(blockIdx.x) * JSON_SLOT;
    for (uint32_t k = threadIdx.x; k < cnt; k += JSON_THREADS) out[k] = base + slot[k];
  } else {
    block_newlines(buf, len, blockIdx.x, [&](uint32_t r, uint32_t pos) { out[r] = base + pos; });
  }
}

// ---- per-line parse (json_lane.h walker) --------------------------------------------------------
constexpr int JL_T = 64;             // one wave: one lane per line

// Writes line `line`'s action arrays from the walker's result; `lp` is where its bytes were read
// (`gp`: its global address).
__device__ __forceinline__ void emit_line(const JsonParseArgs& a, uint64_t line, uint64_t b, uint32_t n,
                                          const uint8_t* lp, const uint8_t* gp, const jl::LineOut& o) {
  const uint64_t idx = a.base + line;
  uint8_t flags = 0;
  uint64_t key = 0, path = 0;
  uint32_t plen = 0;
  int64_t size = 0, delts = 0;
  const uint8_t kind = o.kind;
  if (kind == K_ADD || kind == K_REMOVE) {
    flags = o.flags;  // F_HAS_DELTS / F_PATH_ESCAPED / F_PATH_NULL share dev_common.h's values
    path = reinterpret_cast<uint64_t>(gp + o.path_off);
    plen = o.path_len;
    size = o.size;
    delts = o.delts;
    if (!(flags & F_PATH_NULL)) {
      if ((flags & F_PATH_ESCAPED) || path_is_special(lp + o.path_off, plen)) {
        flags |= F_SPECIAL_PATH;
        atomicAdd(reinterpret_cast<unsigned long long*>(a.special_count), 1ull);
        atomicAdd(reinterpret_cast<unsigned long long*>(a.special_bytes), (unsigned long long)(plen + 8));
      } else {
        key = path_key(lp + o.path_off, plen);
      }
    } else {
      path = 0;
      plen = 0;
    }
  } else if (kind == K_METADATA || kind == K_TXN || kind == K_PROTOCOL) {
    // protocol / metaData / txn: reduced on the host (the reference's single `null` partition); the
    // line and its byte offset, so the host reads them back once, after the whole replay is queued
    const unsigned long long slot = atomicAdd(reinterpret_cast<unsigned long long*>(a.nonfile_count), 1ull);
    if (slot < a.nonfile_cap) {
      a.nonfile_idx[2 * slot] = line;
      a.nonfile_idx[2 * slot + 1] = b;
    }
  } else if (kind == K_ERROR) {
    atomicAdd(reinterpret_cast<unsigned long long*>(a.error_count), 1ull);
  }
  a.kind[idx] = kind;
  a.flags[idx] = flags;
  a.key[idx] = key;
  a.path_ptr[idx] = path;
  a.path_len[idx] = plen;
  if (a.path_ref) a.path_ref[idx] = pack_ref(path, plen);
  a.size[idx] = size;
  a.delts[idx] = delts;
  a.src_off[idx] = b;
  a.src_len[idx] = n;
}

// 64 consecutive lines per block, one lane per line, two phases (json_lane.h):
//  1. each lane tokenizes its line window by window (16-byte global loads, SWAR masks) into its
//     column of an LDS token buffer;
//  2. the DFA consumes the buffer BY TOKEN INDEX: lines of one commit share their shape (all adds,
//     or all removes), so the 64 lanes take the same grammar branch at the same step instead of
//     diverging byte by byte.
// The buffer is flushed through phase 2 whenever a lane could overflow it, and at the end.
#ifndef DR_JL_TOKCAP
#define DR_JL_TOKCAP 40  // 10 KiB LDS per wave: 4 waves/SIMD (80: 20 KiB, LDS-bound at 2; sweep r01: 80 -> 40 = 4.02 -> 2.87 ms, 32 flushes too often)
#endif
constexpr int JL_TOKCAP = DR_JL_TOKCAP;
#ifndef DR_JL_FLUSH
#define DR_JL_FLUSH (DR_JL_TOKCAP - 16)  // a window adds at most 16 tokens
#endif
constexpr int JL_FLUSH = DR_JL_FLUSH;

#ifndef DR_JL_BATCH
#define DR_JL_BATCH 2  // windows per load batch; 2 (pairs) sweep r01: 2.86 -> 2.77 ms, 12.14 -> 11.98 ms/step same box
#endif
#ifndef DR_JL_WAVES
#define DR_JL_WAVES 1
#endif
// Small segments (a streamed commit: at most JL_SMALL_LINES lines) take the staged walker: each
// wave copies its lines' byte region into LDS with coalesced 16-byte loads and every lane walks its
// line from LDS, so the walk's dependent reads cost LDS latency instead of a global round trip each
// (one wave of a commit has no other waves to hide them behind); lines the fast walker defers are
// deferred to k_json_hard like the bulk segment's: the General walker's stack arrays would give the
// staged kernel a private segment (r03 inlined it: 272 B of scratch per lane). Every stage read is a
// ds_read: the stage is reached through the LDS array itself, never through a generic pointer that
// could also be global (r03's one-walker build did that and faulted). For the bulk
// segment the stage halves occupancy and loses (r03: 8.2 vs 2.79 ms), so it keeps the global walker.
constexpr uint32_t JL_SMALL_LINES = 256;
constexpr uint32_t JL_STAGE_BYTES = 24u * 1024u;

// One lane's line walk: tokenize window by window into the LDS token buffer, the DFA by token index
// (see below); `p` is the line's first byte wherever it is read from (LDS or global).
template <bool InlineHard = false>
__device__ __forceinline__ void walk_line(const JsonParseArgs& a, uint32_t* tokbuf, uint32_t lane, uint64_t line,
                                          bool live, uint64_t b, uint32_t n, const uint8_t* p) {
  jl::Tokenizer tz;
  jl::Dfa<false> d;
  if (!live) tz.status = jl::ST_BAD;
  else if (n > jl::TOK_MAX_LINE) tz.status = jl::ST_HARD;
  const uint32_t o0 = uint32_t(b & 15);
  const uint8_t* base = p - o0;
  const uint32_t nwin = tz.status == jl::ST_OK ? (o0 + n + 15) >> 4 : 0;
  uint32_t nt = 0;
#if DR_JL_BATCH > 1
  uint4 batch[DR_JL_BATCH];
#endif
  auto push = [&](uint32_t t) {
    tokbuf[nt * JL_T + lane] = t;
    ++nt;
  };
  for (uint32_t j = 0;; ++j) {
    if (j < nwin && tz.status == jl::ST_OK) {
      uint32_t w[4];
#if DR_JL_BATCH > 1
      // windows in batches: DR_JL_BATCH consecutive 16 B requests per lane issued together (the
      // line's cache lines are asked for while still resident, other waves competing for L2)
      if (j % DR_JL_BATCH == 0) {
        const uint4* q = reinterpret_cast<const uint4*>(base + 16u * j);
#pragma unroll
        for (int k = 0; k < DR_JL_BATCH; ++k) batch[k] = j + k < nwin ? q[k] : make_uint4(0, 0, 0, 0);
      }
      uint4 v0 = batch[0];
#pragma unroll
      for (int k = 1; k < DR_JL_BATCH; ++k)
        if (j % DR_JL_BATCH == uint32_t(k)) v0 = batch[k];
      w[0] = v0.x; w[1] = v0.y; w[2] = v0.z; w[3] = v0.w;
#else
      jl::load_window(base + 16u * j, w);
#endif
      jl::tokenize_window<false>(p, n, w, int32_t(16u * j) - int32_t(o0), tz, push);
      if (j + 1 == nwin) jl::tokenize_end(n, tz, push);
    }
    const bool more = j + 1 < nwin && tz.status == jl::ST_OK;
    const bool anymore = __ballot(more) != 0ull;
    if (!anymore || __ballot(nt > uint32_t(JL_FLUSH)) != 0ull) {
      uint32_t mx = nt;
      for (int o = 32; o > 0; o >>= 1) mx = max(mx, uint32_t(__shfl_xor(int(mx), o, 64)));
#if !defined(DR_JL_EXP)  // DR_JL_EXP: timing experiments only (scripts/build_variant.sh), no DFA
      for (uint32_t t = 0; t < mx; ++t)
        if (t < nt && d.status == jl::ST_OK) jl::dfa_token<false>(p, tokbuf[t * JL_T + lane], d);
#endif
      nt = 0;
    }
    if (!anymore) break;
  }
  if (!live) return;
  jl::LineOut o;
  jl::dfa_finish<false>(tz, d, o);
  if (o.hard) {
    if constexpr (InlineHard) {
      const uint8_t* gp = a.buf + b;
      jl::parse_line_general(gp, n, o);
      emit_line(a, line, b, n, gp, gp, o);
    } else {
      const unsigned long long k = atomicAdd(a.hard_count, 1ull);
      a.hard_idx[k] = line;
    }
    return;
  }
  emit_line(a, line, b, n, p, a.buf + b, o);
}

// ---- the wave-cooperative tokenizer of small segments (the tape) ------------------------------------
// A streamed commit is a few lines in one wave; walked one lane per line, every lane's ~20 windows
// are a serial chain with nothing to hide its latency (r03: 96 us of a 6-line commit's apply). Here
// the wave sweeps the staged region 1 KiB per step (lane l: the aligned 16-byte window l of the
// step), classifies each window with the walker's SWAR masks, and resolves the state that crosses
// windows with ballots instead of a serial walk: backslash-run parity (the nearest lower window that
// is not all backslashes decides it), in-string parity (a prefix XOR of the windows' quote
// parities), scalar runs, and for every closing quote the position of its opening quote and whether
// a backslash lies between them. Tokens go in byte order to an LDS tape -- structural bytes, one
// T_STRING per string (at its closing quote, carrying the opening position and the body length), one
// T_SCALAR per scalar run (at its first byte; its length is the distance to the next token), one T_NL
// per newline -- and each lane then runs the walker's DFA over its own line's stretch of the tape
// (r02 built this for the bulk segment, exact on every parity test but slower there: a 64-line wave
// has no idle lanes and its lines' tokens are uneven across windows).
//
// The tape covers the canonical Delta writer's lines: a region with whitespace or a control byte
// outside a string, a newline inside a string, an escape other than \" \\ \/ \b \f \n \r \t, a
// string of 4096 bytes or more, or more tokens than the tape holds sends the whole wave (a
// wave-uniform branch) to the per-lane walker, which decides every line exactly as before.
constexpr uint32_t T_NL = 12;
constexpr uint32_t TAPE_CAP = 4096;  // tokens (16 KiB of LDS)

constexpr uint64_t STRUCT_CLS = (uint64_t(jl::T_COLON) << 40) | (uint64_t(jl::T_OBJ_OPEN) << 44) |
                                (uint64_t(jl::T_COMMA) << 48) | (uint64_t(jl::T_OBJ_CLOSE) << 52);

// Bytes escaped by a backslash run, with the run parity carried in (cin) and out (*cout): the
// per-lane walker's rule (json_lane.h tokenize_window).
__device__ __forceinline__ uint32_t escape16(uint32_t bs, uint32_t cin, uint32_t* cout) {
  const uint32_t bsn = bs & ~cin;
  const uint32_t follows = ((bsn << 1) | cin) & 0xFFFFu;
  const uint32_t odd_starts = bsn & ~0x5555u & ~follows;
  const uint32_t sum = odd_starts + bsn;
  *cout = (sum >> 16) & 1u;
  return (0x5555u ^ ((sum << 1) & 0xFFFFu)) & follows;
}

__device__ __forceinline__ uint64_t lanes_below() { return (1ull << wv::lane_id()) - 1ull; }

// Orders one wave's LDS accesses across its lanes (the staged walkers run each wave on its own:
// a workgroup barrier would wait for waves that never arrive)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Value of `v` in the highest lane below this one whose `has` is set, or `dflt` when there is none
// (an exclusive last-writer scan on DPP).
__device__ __forceinline__ int32_t from_lower(bool has, int32_t v, int32_t dflt) {
  constexpr uint32_t NONE = 0x80000000u;
  uint32_t x = has ? uint32_t(v) : NONE;
  x = wv::scan_incl(x, NONE, [](uint32_t e, uint32_t l) { return l == NONE ? e : l; });
  x = wv::shr1(x, NONE);
  return x == NONE ? dflt : int32_t(x);
}

// The tape of the region [rb, rb + R) of the stage (R includes the last line's newline). Returns
// true when every line of the wave is on it (wave-uniform); false sends the wave to the walker.
// TCap: the tape's tokens, NL: the lines it may hold, SW: the stage's 16-byte words.
template <uint32_t TCap, uint32_t NL, uint32_t SW>
__device__ __forceinline__ bool build_tape(const uint4* stage, uint32_t rb, uint32_t R, uint32_t nlines, uint32_t* tape,
                           uint16_t* nltok, uint8_t* tline, unsigned long long* phase = nullptr) {
  const uint32_t lane = wv::lane_id();
  // the region and the 48 bytes the token reads reach past it (lds20 from a token's start, the
  // stage's tail) must lie in the stage: otherwise the wave goes to the General walker, which reads
  // the line from global memory (a region past the stage would be read as zeros)
  DR_LDS_CHECK(uint64_t(rb) + R + 48 <= uint64_t(SW) * 16, "build_tape region", uint64_t(rb) + R + 48, SW * 16);
  if (uint64_t(rb) + R + 48 > uint64_t(SW) * 16) return false;
  const uint32_t a0 = rb & ~15u;
  const uint32_t skew = rb - a0;
  const uint32_t total = skew + R;
  const uint32_t nsteps = (total + 1023u) >> 10;
  uint32_t esc_c = 0, instr_c = 0, sc_c = 0, tbase = 0, nlc = 0;
  int32_t open_c = -1, bs_c = -1;
  for (uint32_t s = 0; s < nsteps; ++s) {
    const uint64_t ts0 = phase ? __builtin_amdgcn_s_memtime() : 0;
    const uint32_t wpos = (s << 10) + (lane << 4);
    const int32_t lo = int32_t(wpos) - int32_t(skew);  // region offset of the window's byte 0
    // unconditional (clamped) stage read and masks: a guarded read is a branch
    DR_LDS_CHECK(wpos >= total || ((a0 + wpos) >> 4) < SW, "build_tape stage", (a0 + wpos) >> 4, SW);
    const uint4 v = stage[min((a0 + wpos) >> 4, SW - 1)];
    const uint32_t keep = wpos < total ? ~0u : 0u;
    const uint32_t w[4] = {v.x & keep, v.y & keep, v.z & keep, v.w & keep};
    const uint32_t vlo = lo < 0 ? (0xFFFFu << uint32_t(min(-lo, 16))) & 0xFFFFu : 0xFFFFu;
    const int32_t rem = int32_t(R) - lo;  // bytes of the region from the window's byte 0
    const uint32_t vhi = rem >= 16 ? 0xFFFFu : rem <= 0 ? 0u : (1u << uint32_t(rem)) - 1u;
    const uint32_t valid = vlo & vhi;
    jl::Win m;
    jl::classify(w, m);
    m.q &= valid; m.bs &= valid; m.st &= valid; m.sp &= valid; m.ctrl &= valid;
    uint32_t nl = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) nl |= jl::gather4(jl::zbytes(w[d] ^ 0x0a0a0a0au)) << (4 * d);
    nl &= valid;
    // backslash runs: a window that is not all backslashes decides its carry-out by itself
    uint32_t c0;
    escape16(m.bs, 0u, &c0);
    const bool allbs = m.bs == 0xFFFFu;
    const uint32_t cin = uint32_t(from_lower(!allbs, int32_t(c0), int32_t(esc_c)));
    uint32_t cout;
    const uint32_t escaped = escape16(m.bs, cin, &cout);
    esc_c = uint32_t(__builtin_amdgcn_readlane(int(allbs ? cin : cout), 63));
    // string state: prefix XOR of the windows' quote parities
    const uint32_t quote = m.q & ~escaped;
    const unsigned long long par = __ballot(__builtin_popcount(quote) & 1);
    const uint32_t sin = instr_c ^ uint32_t(__popcll(par & lanes_below()) & 1);
    const uint32_t instr = jl::prefix_xor16(quote) ^ (sin ? 0xFFFFu : 0u);
    instr_c ^= uint32_t(__popcll(par) & 1);
    bool bad = (m.ctrl & ~(nl & ~instr)) != 0 || (m.sp & ~instr) != 0;
    uint32_t oddesc = escaped & ~(m.q | m.bs) & valid;
    while (oddesc) {  // escapes other than \" and \\ (rare)
      const uint32_t k = jl::ctz32(oddesc);
      oddesc &= oddesc - 1;
      const uint32_t c = jl::win_byte(w, k);
      bad |= !(c == '/' || c == 'b' || c == 'f' || c == 'n' || c == 'r' || c == 't');
    }
    const uint32_t st = m.st & ~instr;
    const uint32_t sc = valid & ~instr & ~quote & ~st & ~m.sp & ~m.ctrl;
    const uint32_t sc_prev = wv::shr1(sc >> 15, sc_c) & 1u;
    const uint32_t sc_begin = sc & ~(((sc << 1) | sc_prev) & 0xFFFFu);
    sc_c = uint32_t(__builtin_amdgcn_readlane(int(sc >> 15), 63)) & 1u;
    const uint32_t open = quote & instr, close = quote & ~instr;
    const uint32_t bsin = m.bs & instr;
    // latest opening quote / in-string backslash before this window
    const int32_t last_open = open ? lo + 31 - __builtin_clz(open) : -1;
    const int32_t last_bs = bsin ? lo + 31 - __builtin_clz(bsin) : -1;
    const int32_t open_in = from_lower(open != 0, last_open, open_c);
    const int32_t bs_in = from_lower(bsin != 0, last_bs, bs_c);
    open_c = __builtin_amdgcn_readlane(open ? last_open : open_in, 63);
    bs_c = __builtin_amdgcn_readlane(bsin ? last_bs : bs_in, 63);
    const uint32_t tm = st | close | sc_begin | nl;
    // token and newline ranks: one wave scan of both counts (16-bit halves)
    const uint32_t cnt = uint32_t(__builtin_popcount(tm)) | (uint32_t(__builtin_popcount(nl)) << 16);
    const uint32_t incl = wv::scan_incl(cnt, 0u, [](uint32_t e, uint32_t l) { return e + l; });
    const uint32_t tot = uint32_t(__builtin_amdgcn_readlane(int(incl), 63));
    if (__ballot(bad)) return false;
    if (tbase + (tot & 0xFFFFu) > TCap || nlc + (tot >> 16) > NL) return false;
    uint32_t idx = tbase + ((incl - cnt) & 0xFFFFu);
    uint32_t nlr = nlc + ((incl - cnt) >> 16);
    bool longstr = false;
    const uint64_t ts1 = phase ? __builtin_amdgcn_s_memtime() : 0;
    uint32_t t = tm;
    const uint64_t wlo = uint64_t(w[0]) | (uint64_t(w[1]) << 32), whi = uint64_t(w[2]) | (uint64_t(w[3]) << 32);
    while (t) {
      const uint32_t k = jl::ctz32(t);
      t &= t - 1;
      const uint32_t bit = 1u << k, below = bit - 1u;
      const uint32_t pos = uint32_t(lo + int32_t(k));
      const uint32_t ob = open & below, bb = bsin & below;
      const int32_t op = ob ? lo + 31 - __builtin_clz(ob) : open_in;
      const int32_t lb = bb ? lo + 31 - __builtin_clz(bb) : bs_in;
      const uint32_t blen = pos - uint32_t(op) - 1u;
      const uint32_t c = uint32_t(((k & 8u) ? whi : wlo) >> ((k & 7u) * 8u)) & 0xFFu;
      // structural class by the low nibble ({ [ : B, } ] : D, ':' A, ',' C) from a nibble table, + 1
      // for the square brackets (bit 5 clear): a compare chain on c compiles to a branch tree
      const uint32_t lo4 = c & 15u;
      const uint32_t scls = uint32_t((STRUCT_CLS >> (4u * lo4)) & 15u) + (((0x2800u >> lo4) & ~(c >> 5)) & 1u);
      const bool isclose = (close & bit) != 0;
      longstr |= isclose & (blen >= 4096u);
      const uint32_t stok = (uint32_t(op) << 16) | ((blen & 0xFFFu) << 4) | (lb > op ? jl::T_STRING_ESC : jl::T_STRING);
      const uint32_t otok = (pos << 16) | ((st & bit) ? scls : (sc_begin & bit) ? jl::T_SCALAR : T_NL);
      DR_LDS_CHECK(idx < TCap, "build_tape tape", idx, TCap);
      DR_LDS_CHECK(nlr < NL || !(nl & bit), "build_tape nltok", nlr, NL);
      tline[idx] = uint8_t(nlr);
      const bool isnl = (nl & bit) != 0;
      nltok[isnl ? nlr : NL] = uint16_t(idx);  // slot NL: a sink for the other tokens
      nlr += isnl ? 1u : 0u;
      tape[idx++] = isclose ? stok : otok;
    }
    if (phase && lane == 0) {
      atomicAdd(&phase[6], (unsigned long long)(ts1 - ts0));
      atomicAdd(&phase[7], (unsigned long long)(__builtin_amdgcn_s_memtime() - ts1));
    }
    if (__ballot(longstr)) return false;
    tbase += tot & 0xFFFFu;
    nlc += tot >> 16;
  }
  return nlc == nlines;
}

// ---- the tape's grammar and extraction, wave-parallel over tokens -----------------------------------
// A streamed commit has a handful of lines: walking each line's tokens in its own lane (the DFA of
// json_lane.h) is a serial chain of ~40 dependent steps whose every step executes the union of the
// lanes' branches (r04: 95K clocks of a 6-line commit's 115K). Here lane l takes token 64r + l of
// the tape in round r, and everything the DFA derives from its state comes from wave scans instead:
//  * the nesting depth before each token (a segmented prefix sum of +1 / -1, reset at each line's
//    first token);
//  * the kind of container open at that depth (a last-writer-wins scan over levels 1..7: an open at
//    level L writes bit L; the last open at the token's level is the innermost open container,
//    exactly as a stack would have it);
//  * the latest object opened at level 2 (a max scan): a depth-2 member's enclosing top-level member.
// Grammar is checked per token from its class, its two predecessors' classes and that container kind
// (the JSON transitions the DFA encodes: a key follows '{' or an object's ',', ':' follows a key, a
// value follows ':' or an array's '[' / ',', ',' and a close follow a value or their own open).
// Extraction keeps the DFA's last-value-wins rules by keeping, per line, the LAST top-level member of
// each action kind and the LAST path / size / deletionTimestamp member inside add / remove members
// (LDS atomicMax on token index * 2 + non-null); a field index below its kind's last member belongs
// to an earlier member and does not count. Anything the fast DFA would defer (an escaped key at depth
// <= 2, nesting past the scanned levels) or reject (a grammar or typing error) sends the line to the
// General walker (k_json_hard / k_tail_post), which decides every line exactly: the deferral needs no
// K_ERROR logic here, and lines the tape accepts are decided as the DFA decides them.
constexpr uint32_t TW_LEVELS = 7;  // container levels the type scan tracks (deeper: General walker)
template <uint32_t NL>
struct TapeAgg {
  int32_t mem[NL][8];      // per line and action kind: last top-level member's value token * 2 + non-null
  int32_t fld[NL][2][4];   // per line, add / remove: last path / size / deletionTimestamp value token * 2 + non-null
  uint32_t defer[NL];
};

__device__ __forceinline__ uint32_t type_combine(uint32_t early, uint32_t late) {
  const uint32_t lm = late & 0xFFu;
  return ((early | late) & 0xFFu) | (((((early >> 8) & ~lm) | (late >> 8)) & 0xFFu) << 8);
}

// Branch-free token helpers of the tape walk: a wave executes every branch any of its lanes takes,
// so the walk computes the key and scalar classes of every lane with selects from one 20-byte load
// each. A scalar that is not null / true / false or a plain integer of at most 19 digits (a fraction,
// an exponent, 20+ characters) is reported as SC_BAD: its line goes to the General walker, which
// decides it.
// 20 bytes at s (in the LDS stage) as little-endian words: six dword reads from the dword below s
// and byte funnel shifts (a select over the 16-byte phase of s compiles to a branch tree)
__device__ __forceinline__ void lds20(const uint8_t* s, uint32_t w[5]) {
  const uint32_t r = uint32_t(reinterpret_cast<uintptr_t>(s)) & 3u;
  const uint32_t* b = reinterpret_cast<const uint32_t*>(s - r);
  uint32_t u[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) u[k] = b[k];
#pragma unroll
  for (int k = 0; k < 5; ++k) w[k] = __builtin_amdgcn_alignbyte(u[k + 1], u[k], r);
}

// action kind (low nibble) and file-field key (high nibble) of a member name of n bytes
__device__ __forceinline__ uint32_t key_kinds(const uint32_t w[5], uint32_t n) {
  const uint32_t a = w[0], b = w[1], c = w[2], t = a & 0xFFFFFFu;
  const uint32_t k3 = t == 0x646461u ? jl::K_ADD : t == 0x6E7874u ? jl::K_TXN : t == 0x636463u ? jl::K_CDC : 0u;
  const uint32_t k6 = (a == 0x6F6D6572u && (b & 0xFFFFu) == 0x6576u) ? jl::K_REMOVE : 0u;
  const uint32_t k8 = (a == 0x6174656Du && b == 0x61746144u) ? jl::K_METADATA
                    : (a == 0x746F7270u && b == 0x6C6F636Fu) ? jl::K_PROTOCOL : 0u;
  const uint32_t k10 = (a == 0x6D6D6F63u && b == 0x6E497469u && (c & 0xFFFFu) == 0x6F66u) ? jl::K_COMMITINFO : 0u;
  const uint32_t k1 = n == 3 ? k3 : n == 6 ? k6 : n == 8 ? k8 : n == 10 ? k10 : 0u;
  const uint32_t f4 = a == 0x68746170u ? jl::FK_PATH : a == 0x657A6973u ? jl::FK_SIZE : jl::FK_OTHER;
  const uint32_t f17 = (a == 0x656C6564u && b == 0x6E6F6974u && c == 0x656D6954u && w[3] == 0x6D617473u &&
                        (w[4] & 0xFFu) == 0x70u) ? jl::FK_DELTS : jl::FK_OTHER;
  const uint32_t k2 = n == 4 ? f4 : n == 17 ? f17 : jl::FK_OTHER;
  return k1 | (k2 << 4);
}

__device__ __forceinline__ uint8_t scalar_tape(const uint32_t w0[5], uint32_t L, int64_t* val) {
  uint32_t w[5];
  const bool neg = (w0[0] & 0xFFu) == 0x2Du;
#pragma unroll
  for (int d = 0; d < 5; ++d) w[d] = neg ? ((w0[d] >> 8) | (d < 4 ? (w0[d + 1] << 24) : 0u)) : w0[d];
  uint32_t dm = 0;
#pragma unroll
  for (int d = 0; d < 5; ++d) dm |= jl::gather4(jl::digit_bytes(w[d])) << (4 * d);
  const uint32_t nd = L - (neg ? 1u : 0u);
  const uint32_t need = nd >= 20 ? 0xFFFFFu : (1u << nd) - 1u;
  const bool isint = (L <= 20) & (nd >= 1) & (nd <= 19) & ((dm & need) == need) & !((nd > 1) & ((w[0] & 0xFFu) == 0x30u));
  const uint32_t g = nd >> 2, r = nd & 3u;
  uint64_t v = 0;
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    const uint64_t nv = v * 10000ull + jl::digits4(w[k]);
    v = k < g ? nv : v;
  }
  uint32_t x = 0;  // w[g], as masks (a select chain on g compiles to a branch tree)
#pragma unroll
  for (uint32_t k = 0; k < 5; ++k) x |= w[k] & (0u - uint32_t(g == k));
  const uint32_t sh = 8u * (4u - r);
  const uint64_t rv = v * (r == 1 ? 10ull : r == 2 ? 100ull : 1000ull) +
                      jl::digits4((x << (sh & 31u)) | (0x30303030u >> ((32u - sh) & 31u)));
  v = r ? rv : v;
  const bool fits = v <= (neg ? 0x8000000000000000ull : 0x7FFFFFFFFFFFFFFFull);
  *val = neg ? int64_t(0ull - v) : int64_t(v);
  return (L == 4 && w0[0] == 0x6C6C756Eu) ? jl::SC_NULL
       : (L == 4 && w0[0] == 0x65757274u) ? jl::SC_TRUE
       : (L == 5 && w0[0] == 0x736C6166u && (w0[1] & 0xFFu) == 0x65u) ? jl::SC_FALSE
       : (isint && fits) ? jl::SC_INT : jl::SC_BAD;
}

// sp: the region's first byte in the stage, sp_ext: the stage bytes from sp (the checks' extent)
template <uint32_t TCap, uint32_t NL>
__device__ __forceinline__ void tape_lines(const JsonParseArgs& a, uint64_t line0, uint32_t nlines, const uint8_t* sp,
                                           uint32_t sp_ext, uint64_t gb, const uint32_t* tape, const uint16_t* nltok,
                                           const uint8_t* tline, TapeAgg<NL>& g) {
  (void)sp_ext;
  const uint32_t lane = wv::lane_id();
  const uint64_t tw0 = a.phase ? __builtin_amdgcn_s_memtime() : 0;
  if (lane < NL) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      g.mem[lane][k] = -1;
      g.fld[lane][k >> 2][k & 3] = -1;
    }
    g.defer[lane] = 0;
  }
  wave_sync();
  const uint32_t ntok = uint32_t(nltok[nlines - 1]) + 1u;
  int32_t dcarry = 0, ocarry = -1;
  uint32_t tcarry = 0, ptail1 = T_NL, ptail2 = T_NL;  // the previous round's last two tokens
  for (uint32_t r0 = 0; r0 < ntok; r0 += JL_T) {
    const uint32_t i = r0 + lane;
    const bool in = i < ntok;
    // unconditional reads (clamped into the arrays): a guarded LDS read is a branch
    const uint32_t tk = tape[min(i, TCap - 1)], nx = tape[min(i + 1, TCap - 1)];
    const uint32_t tl = tline[min(i, TCap - 1)];
    const uint32_t tok = in ? tk : 15u;
    const uint32_t nxt = i + 1 < ntok ? nx : tok;
    const uint32_t line = in ? tl : 0u;
    const uint32_t ptok = wv::shr1(tok, ptail1), pptok = wv::shr1(ptok, ptail2);
    ptail1 = wv::last_uniform(tok);
    ptail2 = wv::last_uniform(ptok);
    // the token's bytes (a scalar's) and its key's (the string two tokens back), one load each
    uint32_t sw[5], kw[5];
    DR_LDS_CHECK(!in || (tok >> 16) + 24u <= sp_ext, "tape_lines token bytes", (tok >> 16) + 24u, sp_ext);
    DR_LDS_CHECK(!in || (pptok >> 16) + 25u <= sp_ext, "tape_lines key bytes", (pptok >> 16) + 25u, sp_ext);
    DR_LDS_CHECK(!in || line < NL, "tape_lines line", line, NL);
    lds20(sp + (tok >> 16), sw);
    lds20(sp + (pptok >> 16) + 1u, kw);
    const uint32_t cls = tok & 0xFu;
    const uint32_t pc0 = ptok & 0xFu;
    const bool first = pc0 == T_NL;  // the first token of its line
    const uint32_t ppc0 = pptok & 0xFu;
    const int32_t delta = cls <= jl::T_ARR_OPEN ? 1 : (cls == jl::T_OBJ_CLOSE || cls == jl::T_ARR_CLOSE) ? -1 : 0;
    const uint32_t kk = key_kinds(kw, (pptok >> 4) & 0xFFFu);
    const uint32_t k1 = kk & 0xFu, k2 = kk >> 4;
    // depth after the token: segmented inclusive scan (flag in bit 31: a line's first token), lines
    // restart at 0
    uint32_t sg = (first ? 0x80000000u : 0u) | (uint32_t(delta) & 0x7FFFFFFFu);
    sg = wv::scan_incl(sg, 0u, [](uint32_t e, uint32_t l) {
      return (l & 0x80000000u) ? l : ((e & 0x80000000u) | ((e + l) & 0x7FFFFFFFu));
    });
    int32_t v = int32_t(sg << 1) >> 1;
    if (!(sg & 0x80000000u)) v += dcarry;
    dcarry = __builtin_amdgcn_readlane(v, 63);
    const int32_t D = v - delta;  // depth before the token
    // container kinds by level: bit L of the low byte = level L opened, of the high byte = an array
    const bool opens = delta > 0;
    uint32_t x = opens && v <= int32_t(TW_LEVELS) ? ((1u << v) | (uint32_t(cls == jl::T_ARR_OPEN) << (8 + v))) : 0u;
    x = type_combine(tcarry, wv::scan_incl(x, 0u, type_combine));
    tcarry = wv::last_uniform(x);
    // the latest container opened at level 2 (a top-level member's value) with its member's action
    // kind: index * 8 + kind, a max scan
    const bool m2open = opens && v == 2 && pc0 == jl::T_COLON;
    int32_t o2 = int32_t(wv::scan_incl(m2open ? (i << 3) | k1 : 0xFFFFFFFFu, 0xFFFFFFFFu,
                                       [](uint32_t e, uint32_t l) { return uint32_t(max(int32_t(e), int32_t(l))); }));
    o2 = max(o2, ocarry);
    ocarry = __builtin_amdgcn_readlane(o2, 63);
    const bool lvl = D >= 1 && D <= int32_t(TW_LEVELS) && ((x >> D) & 1u);
    const bool ctx_arr = lvl && ((x >> (8 + D)) & 1u), ctx_obj = lvl && !ctx_arr;
    const uint32_t ppc = (first || ppc0 == T_NL) ? 15u : ppc0;  // 15: the line's start
    const bool is_str = cls == jl::T_STRING || cls == jl::T_STRING_ESC;
    const bool is_sc = cls == jl::T_SCALAR;
    const bool pstr = pc0 == jl::T_STRING || pc0 == jl::T_STRING_ESC;
    const bool prev_key = pstr && (ppc == jl::T_OBJ_OPEN || (ppc == jl::T_COMMA && ctx_obj));
    const bool prev_vend = pc0 == jl::T_SCALAR || pc0 == jl::T_OBJ_CLOSE || pc0 == jl::T_ARR_CLOSE || (pstr && !prev_key);
    const bool value_pos = pc0 == jl::T_COLON || (ctx_arr && (pc0 == jl::T_ARR_OPEN || pc0 == jl::T_COMMA));
    const bool cur_key = is_str && (pc0 == jl::T_OBJ_OPEN || (pc0 == jl::T_COMMA && ctx_obj));
    int64_t sv;
    const uint32_t L = (nxt >> 16) - (tok >> 16);
    const uint8_t sc = scalar_tape(sw, L, &sv);
    // the classes are disjoint: one term holds (bitwise, so that nothing compiles to a branch)
    const bool is_nl = cls == T_NL;
    const bool inner = !is_nl & !first & (D >= 1);
    const bool okv = (is_nl & (D == 0)) | (!is_nl & first & (cls == jl::T_OBJ_OPEN)) |
                     (inner & ((opens & value_pos & (v <= int32_t(TW_LEVELS))) |
                               (is_sc & value_pos & (sc != jl::SC_BAD)) |
                               (is_str & ((cur_key & !((cls == jl::T_STRING_ESC) & (D <= 2))) | value_pos)) |
                               ((cls == jl::T_COLON) & prev_key) | ((cls == jl::T_COMMA) & prev_vend) |
                               ((cls == jl::T_OBJ_CLOSE) & ctx_obj & ((pc0 == jl::T_OBJ_OPEN) | prev_vend)) |
                               ((cls == jl::T_ARR_CLOSE) & ctx_arr & ((pc0 == jl::T_ARR_OPEN) | prev_vend))));
    // a member's value (its key is pptok): top-level members by action kind, add / remove fields
    const bool member = in & !first & (pc0 == jl::T_COLON);
    const bool nonnull = !(is_sc & (sc == jl::SC_NULL));
    const int32_t rec = int32_t(2u * i) + (nonnull ? 1 : 0);
    const uint32_t ek1 = uint32_t(o2) & (o2 >= 0 ? 7u : 0u);
    const bool file1 = (k1 == jl::K_ADD) | (k1 == jl::K_REMOVE), efile = (ek1 == jl::K_ADD) | (ek1 == jl::K_REMOVE);
    const bool m1 = member & (D == 1) & (k1 != 0);
    const bool mf = member & (D == 2) & efile & (k2 != jl::FK_OTHER);
    const bool bad1 = m1 & file1 & nonnull & (cls != jl::T_OBJ_OPEN);
    const bool path_ok = is_str | !nonnull, num_ok = is_sc & ((sc == jl::SC_NULL) | (sc == jl::SC_INT));
    const bool badf = mf & !((k2 == jl::FK_PATH) ? path_ok : num_ok);
    if (m1) atomicMax(&g.mem[line][k1], rec);
    if (mf) atomicMax(&g.fld[line][ek1 == jl::K_REMOVE ? 1 : 0][k2], rec);
    if (in & !(okv & !bad1 & !badf)) g.defer[line] = 1u;
    if (a.phase && r0 == 0 && lane == 0) atomicAdd(&a.phase[5], (unsigned long long)(__builtin_amdgcn_s_memtime() - tw0));
  }
  wave_sync();
  if (a.phase && lane == 0) atomicAdd(&a.phase[3], (unsigned long long)(__builtin_amdgcn_s_memtime() - tw0));
  if (lane >= nlines) return;
  const uint64_t line = line0 + lane;
  const uint32_t te = nltok[lane];
  const uint32_t ts = lane ? uint32_t(nltok[lane - 1]) + 1u : 0u;
  DR_LDS_CHECK(te < TCap && ts <= TCap, "tape_lines line tokens", te, TCap);
  const uint32_t ls = lane ? (tape[ts - 1] >> 16) + 1u : 0u;  // line start (region offset)
  const uint32_t n = (tape[te] >> 16) - ls;
  if (g.defer[lane]) {
    const unsigned long long k = atomicAdd(a.hard_count, 1ull);
    a.hard_idx[k] = line;
    return;
  }
  // unwrap priority add > remove > metaData > txn > protocol > cdc > commitInfo (json_lane.h dfa_finish)
  jl::LineOut o{};
  o.kind = jl::K_NONE;
  const uint8_t order[7] = {jl::K_ADD, jl::K_REMOVE, jl::K_METADATA, jl::K_TXN, jl::K_PROTOCOL, jl::K_CDC, jl::K_COMMITINFO};
#pragma unroll
  for (int k = 6; k >= 0; --k)
    if (g.mem[lane][order[k]] >= 0 && (g.mem[lane][order[k]] & 1)) o.kind = order[k];
  if (o.kind == jl::K_ADD || o.kind == jl::K_REMOVE) {
    const int32_t m = g.mem[lane][o.kind] >> 1;
    const int32_t* fl = g.fld[lane][o.kind == jl::K_REMOVE ? 1 : 0];
    o.flags = jl::F_PATH_NULL;
    const int32_t tp = fl[jl::FK_PATH], tz = fl[jl::FK_SIZE], td = fl[jl::FK_DELTS];
    if (tp >= 0 && (tp >> 1) > m && (tp & 1)) {
      DR_LDS_CHECK(uint32_t(tp >> 1) < TCap, "tape_lines path token", tp >> 1, TCap);
      const uint32_t t = tape[tp >> 1];
      o.path_off = (t >> 16) + 1u - ls;
      o.path_len = (t >> 4) & 0xFFFu;
      o.flags = (t & 0xFu) == jl::T_STRING_ESC ? jl::F_PATH_ESCAPED : 0;
    }
    // size / deletionTimestamp: both tokens' words in one pass (an absent field reads token 0)
    const bool hz = tz >= 0 && (tz >> 1) > m && (tz & 1), hd = td >= 0 && (td >> 1) > m && (td & 1);
    const uint32_t iz = hz ? uint32_t(tz >> 1) : 0u, id = hd ? uint32_t(td >> 1) : 0u;
    // a scalar is always followed by its ',' or '}' token, so iz + 1 < ntok <= TCap; clamped anyway
    DR_LDS_CHECK(iz + 1 < TCap && id + 1 < TCap, "tape_lines scalar tokens", max(iz, id) + 1, TCap);
    const uint32_t az = tape[iz], bz = tape[min(iz + 1, TCap - 1)], ad = tape[id], bd = tape[min(id + 1, TCap - 1)];
    DR_LDS_CHECK((az >> 16) + 24u <= sp_ext && (ad >> 16) + 24u <= sp_ext, "tape_lines scalar bytes",
                 max(az >> 16, ad >> 16) + 24u, sp_ext);
    uint32_t wz[5], wd[5];
    lds20(sp + (az >> 16), wz);
    lds20(sp + (ad >> 16), wd);
    int64_t vz, vd;
    (void)scalar_tape(wz, (bz >> 16) - (az >> 16), &vz);
    (void)scalar_tape(wd, (bd >> 16) - (ad >> 16), &vd);
    o.size = hz ? vz : 0;
    o.delts = hd ? vd : 0;
    if (hd) o.flags |= jl::F_HAS_DELTS;
  }
  emit_line(a, line, gb + ls, n, sp + ls, a.buf + gb + ls, o);
}

// 64 consecutive lines per block, one lane per line, two phases (json_lane.h):
//  1. each lane tokenizes its line window by window (16-byte loads, SWAR masks) into its column of
//     an LDS token buffer;
//  2. the DFA consumes the buffer BY TOKEN INDEX: lines of one commit share their shape (all adds,
//     or all removes), so the 64 lanes take the same grammar branch at the same step instead of
//     diverging byte by byte.
// The buffer is flushed through phase 2 whenever a lane could overflow it, and at the end.
template <bool Stage>
__global__ void __launch_bounds__(JL_T, DR_JL_WAVES) k_json_lines(JsonParseArgs a) {
  __shared__ uint32_t tokbuf[Stage ? 1 : JL_TOKCAP * JL_T];
  __shared__ uint4 stage[Stage ? JL_STAGE_BYTES / 16 : 1];
  __shared__ uint32_t tape[Stage ? TAPE_CAP : 1];
  __shared__ uint16_t nltok[Stage ? JL_T + 1 : 1];
  __shared__ uint8_t tline[Stage ? TAPE_CAP : 1];
  __shared__ std::conditional_t<Stage, TapeAgg<JL_T>, uint32_t> agg;
  const uint32_t lane = threadIdx.x;
  const uint64_t line = uint64_t(blockIdx.x) * JL_T + lane;
  const bool live = line < a.nlines;
  if constexpr (Stage) {
    uint64_t tp0 = a.phase ? __builtin_amdgcn_s_memtime() : 0;
    auto phase = [&](int k) {
      if (!a.phase) return;
      const uint64_t t = __builtin_amdgcn_s_memtime();
      if (lane == 0) atomicAdd(&a.phase[k], (unsigned long long)(t - tp0));
      tp0 = t;
    };
    if (a.zero) {  // the whole segment in this wave; its newline index and counter reset here
      if (lane < a.nzero) a.zero[lane] = 0;
      const uint32_t len = uint32_t(a.buf_len);
      const uint4* src = reinterpret_cast<const uint4*>(a.buf);
      const uint32_t nq = ((len + 15u) >> 4) + 3u;
      DR_LDS_CHECK(nq <= JL_STAGE_BYTES / 16, "k_json_lines fused stage", nq, JL_STAGE_BYTES / 16);
      for (uint32_t k = lane; k < min(nq, JL_STAGE_BYTES / 16); k += JL_T) stage[k] = src[k];
      __threadfence();  // the cleared counters reach L2 before any atomic on them
      __syncthreads();
      phase(0);
      const uint32_t nw = uint32_t(a.nlines);
      const bool taped = build_tape<TAPE_CAP, JL_T, JL_STAGE_BYTES / 16>(stage, 0u, len, nw, tape, nltok, tline, a.phase);
      phase(1);
      __syncthreads();
      if (taped) {
        DR_LDS_CHECK(lane >= nw || lane < JL_T, "k_json_lines nltok", lane, JL_T);
        if (lane < nw) a.nl_out[lane] = tape[nltok[lane]] >> 16;  // the newline positions, from the tape
        if (lane == 0) {
          a.off2[0] = 0;
          a.off2[1] = nw;
        }
        tape_lines<TAPE_CAP, JL_T>(a, 0, nw, reinterpret_cast<const uint8_t*>(stage), JL_STAGE_BYTES, 0, tape, nltok, tline,
                                   agg);
        phase(2);
        if (a.phase && lane == 0) atomicAdd(&a.phase[4], 1ull);
        return;
      }
      // off the tape: index the newlines from the stage; every line goes to the General walker
      uint32_t base = 0;
      for (uint32_t s0 = 0; s0 < len; s0 += 16u * JL_T) {
        const uint32_t wpos = s0 + 16u * lane;
        DR_LDS_CHECK(wpos >= len || (wpos >> 4) < JL_STAGE_BYTES / 16, "k_json_lines stage", wpos >> 4,
                     JL_STAGE_BYTES / 16);
        const uint4 v = stage[min(wpos >> 4, JL_STAGE_BYTES / 16 - 1)];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        uint32_t m = 0;
#pragma unroll
        for (int d = 0; d < 4; ++d) m |= jl::gather4(jl::zbytes(w[d] ^ 0x0a0a0a0au)) << (4 * d);
        const int32_t rem = int32_t(len) - int32_t(wpos);
        m &= rem >= 16 ? 0xFFFFu : rem <= 0 ? 0u : (1u << uint32_t(rem)) - 1u;
        const uint32_t c = __builtin_popcount(m);
        const uint32_t incl = wv::scan_incl(c, 0u, [](uint32_t e, uint32_t l) { return e + l; });
        uint32_t r = base + incl - c;
        while (m) {
          a.nl_out[r++] = wpos + jl::ctz32(m);
          m &= m - 1;
        }
        base += wv::last_uniform(incl);
      }
      if (lane == 0) {
        a.off2[0] = 0;
        a.off2[1] = base;
        atomicAdd(a.hard_count, (unsigned long long)nw);
      }
      if (lane < nw) a.hard_idx[lane] = lane;
      return;
    }
    // the wave's region: [its first line's 16-byte block, its last line's end rounded up to 16);
    // the JSON buffer's 64-byte zero pad keeps the rounded end readable
    const uint64_t first = uint64_t(blockIdx.x) * JL_T;
    const uint64_t last = min(first + JL_T, a.nlines) - 1;
    const uint64_t r0 = (first == 0 ? 0 : a.nl[first - 1] + 1) & ~uint64_t(15);
    const uint64_t r1 = (a.nl[last] + 16) & ~uint64_t(15);
    if (r1 - r0 + 48 <= JL_STAGE_BYTES) {  // + the walker's reads past a line end (load20, pairs)
      const uint4* src = reinterpret_cast<const uint4*>(a.buf + r0);
      const uint32_t nq = uint32_t((r1 - r0) >> 4) + 3;
      for (uint32_t k = lane; k < nq; k += JL_T) stage[k] = src[k];
      __syncthreads();
      phase(0);
      const uint32_t nw = uint32_t(last - first + 1);
      const uint64_t rb = first == 0 ? 0 : a.nl[first - 1] + 1;  // the wave's first line
      const bool taped = build_tape<TAPE_CAP, JL_T, JL_STAGE_BYTES / 16>(stage, uint32_t(rb - r0), uint32_t(a.nl[last] + 1 - rb), nw,
                                                                       tape, nltok, tline, a.phase);
      phase(1);
      if (taped) {
        __syncthreads();
        tape_lines<TAPE_CAP, JL_T>(a, first, nw, reinterpret_cast<const uint8_t*>(stage) + (rb - r0),
                                   JL_STAGE_BYTES - uint32_t(rb - r0), rb, tape, nltok, tline, agg);
        phase(2);
        if (a.phase && lane == 0) atomicAdd(&a.phase[4], 1ull);
        return;
      }
    }
    // a region off the tape (non-canonical bytes, or larger than the stage): its lines go to
    // k_json_hard's General walker, which decides any line. Keeping the per-lane walker out of this
    // kernel keeps its code to the tape path: a streamed commit's kernel starts with a cold
    // instruction cache on whichever CU it lands, so its executed code is fetched once per commit.
    if (live) {
      const unsigned long long k = atomicAdd(a.hard_count, 1ull);
      a.hard_idx[k] = line;
    }
    return;
  }
  const uint64_t b = !live ? 0 : line == 0 ? 0 : a.nl[line - 1] + 1;
  const uint32_t n = live ? uint32_t(a.nl[line] - b) : 0;
  walk_line(a, tokbuf, lane, line, live, b, n, a.buf + b);
}

// The General walker over the deferred lines (tab / CR whitespace, escaped member names, deep
// nesting): grid-stride over a device-side count.
__global__ void __launch_bounds__(64) k_json_hard(JsonParseArgs a) {
  const uint64_t cnt = *a.hard_count;
  for (uint64_t k = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < cnt; k += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t line = a.hard_idx[k];
    const uint64_t b = line == 0 ? 0 : a.nl[line - 1] + 1;
    const uint32_t n = uint32_t(a.nl[line] - b);
    const uint8_t* gp = a.buf + b;
    jl::LineOut o;
    jl::parse_line_general(gp, n, o);
    emit_line(a, line, b, n, gp, gp, o);
  }
}

// A small commit-only segment's work after the line walk, in one workgroup: the lines the fast
// walker deferred (General walker), then the special paths' canonicalisation (k_canon's body) --
// one launch instead of two for a streamed commit, whose kernels each cost a launch and a cold
// start rather than their work.
__device__ __forceinline__ void tail_post_body(const JsonParseArgs& a, const CanonArgs& c) {
  // an atomic load: in k_apply_commit the count was raised by this workgroup's atomics (at L2)
  const uint64_t cnt = __hip_atomic_load(a.hard_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // special paths so far (the walk's; the General walker's lines add theirs below)
  const uint64_t nsp0 = __hip_atomic_load(a.special_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (uint64_t k = threadIdx.x; k < cnt; k += blockDim.x) {
    // The deferred line numbers (hard_idx) and the newline index (nl) become addresses here: the r05
    // aperture violation in this kernel (k_tail_post, private_seg_size 272) read them from blocks
    // released before this deferred launch, whose 0xA5 poison sent gp far outside the
    // JSON buffer. The bounds build checks both against their extents and skips a bad line.
    const uint64_t line = a.hard_idx[k];
    DR_LDS_CHECK(line < a.nlines, "tail_post deferred line (global)", line, a.nlines);
#ifdef DR_BOUNDS_CHECK
    if (line >= a.nlines) continue;
#endif
    const uint64_t b = line == 0 ? 0 : a.nl[line - 1] + 1;
    DR_LDS_CHECK(b <= a.nl[line] && a.nl[line] < a.buf_len, "tail_post line bytes (global)", a.nl[line], a.buf_len);
#ifdef DR_BOUNDS_CHECK
    if (!(b <= a.nl[line] && a.nl[line] < a.buf_len)) continue;
#endif
    const uint32_t n = uint32_t(a.nl[line] - b);
    const uint8_t* gp = a.buf + b;
    jl::LineOut o;
    jl::parse_line_general(gp, n, o);
    emit_line(a, line, b, n, gp, gp, o);
  }
  if (!cnt && !nsp0) return;  // nothing to canonicalise (uniform: the loads are the workgroup's)
  __threadfence_block();
  __syncthreads();
  for (uint64_t i = threadIdx.x; i < c.n; i += blockDim.x) canon_one(c, i);
}

__global__ void __launch_bounds__(256) k_tail_post(JsonParseArgs a, CanonArgs c) { tail_post_body(a, c); }

// A streamed commit's whole apply after its line walk, in one workgroup (launch_apply_small): the
// deferred lines and canonicalisation, the append to the chain store (k_append_actions) with the
// index counters' reset, and the index's two passes (k_ix_touch_delta), each step behind a fence
// and a barrier -- one launch where three followed each other, each with its dispatch and cold start.
__device__ __forceinline__ void apply_small_body(const JsonParseArgs& a, const CanonArgs& c, const AppendArgs& p,
                                                 const IndexArgs& x, bool ctr_set) {
  const uint32_t t = threadIdx.x;
  __shared__ unsigned long long sums[6];
  if (t < 6) sums[t] = 0;  // ordered before their use by the next barrier
  if (!ctr_set) {  // (k_apply_commit clears them with the parse counters)
    if (t < p.nctr) p.ctr[t] = t == p.ctr_at ? p.ctr_val : 0ull;
    __threadfence();
    __syncthreads();
  }
  uint64_t tp0 = a.phase ? __builtin_amdgcn_s_memtime() : 0;
  auto phase = [&](int k) {  // DR_JSON_PHASES (k_apply_commit): 8 post-parse, 9 append, 10 touch, 11 delta
    if (!a.phase) return;
    const uint64_t tn = __builtin_amdgcn_s_memtime();
    if (t == 0) atomicAdd(&a.phase[k], (unsigned long long)(tn - tp0));
    tp0 = tn;
  };
  if (a.hard_count) {
    tail_post_body(a, c);
    __threadfence();
    __syncthreads();
  }
  phase(8);
  // the append: each thread its own action, whose fields pass 1 then takes from registers (no
  // barrier: pass 2, which reads other threads' actions, follows the next one)
  const uint64_t i = x.lo + t;
  IxTouch T;
  if (t < p.n) {
    const uint8_t kind = p.src.kind[t], flags = p.src.flags[t];
    const uint64_t key = p.src.key[t], pp = p.src.path_ptr[t];
    const uint32_t pl = p.src.path_len[t];
    const int64_t size = p.src.size[t], delts = p.src.delts[t];
    p.dst.kind[t] = kind;
    p.dst.flags[t] = flags;
    p.dst.key[t] = key;
    p.dst.path_ptr[t] = pp;
    p.dst.path_len[t] = pl;
    p.dst.size[t] = size;
    p.dst.delts[t] = delts;
    p.dst.src_off[t] = p.src.src_off[t];
    p.dst.src_len[t] = p.src.src_len[t];
    p.src_id[t] = p.sid;
    phase(9);
    if (i < x.hi) ix_touch_pre_v(x, i, kind, flags, key, pp, pl, size, delts, T);
  }
  __threadfence();
  __syncthreads();
  phase(10);
  Contrib cc{0, 0, 0, 0, 0};
  unsigned long long files = 0;
  if (i < x.hi) ix_delta_post(x, i, T, cc, files);
  flush_contrib_block(x, cc, files, sums);
  if (a.phase) {
    __syncthreads();
    phase(11);
  }
}

__global__ void __launch_bounds__(IX_T) k_apply_small(JsonParseArgs a, CanonArgs c, AppendArgs p, IndexArgs x) {
  apply_small_body(a, c, p, x, false);
}

// A streamed commit's whole apply in one workgroup of AC_WAVES waves (launch_apply_commit): the
// commit's bytes staged in LDS once, its newline index (wave 0), then each wave builds the token
// tape of its share of the lines and walks it (the small-segment walker of k_json_lines<true>, on
// wave-private tapes), and after a barrier the rest of the apply (apply_small_body). The waves split
// the walk that one wave did serially, and the parse, post-parse, append and index passes are one
// dispatch.
constexpr uint32_t AC_WAVES = 8;  // the walk's waves (the apply after it uses the first IX_T threads)
constexpr uint32_t AC_LINES = (JSON_FUSE_MAX_LINES + AC_WAVES - 1) / AC_WAVES;  // lines per wave
constexpr uint32_t AC_TCAP = 1024;                                            // tape tokens per wave
constexpr uint32_t AC_SW = JSON_BYTES_PER_BLOCK / 16 + 4;                      // one index block + pad
__global__ void __launch_bounds__(AC_WAVES * 64) k_apply_commit(JsonParseArgs a, CanonArgs c, AppendArgs p, IndexArgs x,
                                                                uint64_t exp_n, ReadbackArgs rb) {
  __shared__ uint4 stage[AC_SW];
  __shared__ uint32_t tape[AC_WAVES][AC_TCAP];
  __shared__ uint8_t tline[AC_WAVES][AC_TCAP];
  __shared__ uint16_t nltok[AC_WAVES][AC_LINES + 1];
  __shared__ TapeAgg<AC_LINES> agg[AC_WAVES];
  __shared__ uint32_t nlpos[JSON_FUSE_MAX_LINES];
  const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
  const uint32_t len = uint32_t(a.buf_len), nlines = uint32_t(a.nlines);
  uint64_t tp0 = a.phase ? __builtin_amdgcn_s_memtime() : 0;
  auto phase = [&](int k) {  // DR_JSON_PHASES: 0 stage, 1 newline index, 2 walk, 6 apply, 12 expiry, 13 readback (slot 4: calls)
    if (!a.phase) return;
    const uint64_t tn = __builtin_amdgcn_s_memtime();
    if (t == 0) atomicAdd(&a.phase[k], (unsigned long long)(tn - tp0));
    tp0 = tn;
  };
  if (t < a.nzero) a.zero[t] = 0;
  if (t < p.nctr) p.ctr[t] = t == p.ctr_at ? p.ctr_val : 0ull;  // the index counters (apply_small_body)
  {
    const uint4* src = reinterpret_cast<const uint4*>(a.buf);
    DR_LDS_CHECK(((len + 15u) >> 4) + 3u <= AC_SW, "k_apply_commit stage load", ((len + 15u) >> 4) + 3u, AC_SW);
    const uint32_t nq = min(((len + 15u) >> 4) + 3u, AC_SW);
    for (uint32_t k = t; k < nq; k += AC_WAVES * 64) stage[k] = src[k];
  }
  __threadfence();  // the cleared counters reach L2 before any atomic on them
  __syncthreads();
  phase(0);
  if (w == 0) {  // the newline index: LDS for the waves, nl for the General walker
    uint32_t base = 0;
    for (uint32_t s0 = 0; s0 < len; s0 += 16u * 64u) {
      const uint32_t wpos = s0 + 16u * lane;
      DR_LDS_CHECK(wpos >= len || (wpos >> 4) < AC_SW, "k_apply_commit stage", wpos >> 4, AC_SW);
      const uint4 v = stage[min(wpos >> 4, AC_SW - 1)];
      const uint32_t ww[4] = {v.x, v.y, v.z, v.w};
      uint32_t m = 0;
#pragma unroll
      for (int d = 0; d < 4; ++d) m |= jl::gather4(jl::zbytes(ww[d] ^ 0x0a0a0a0au)) << (4 * d);
      const int32_t rem = int32_t(len) - int32_t(wpos);
      m &= rem >= 16 ? 0xFFFFu : rem <= 0 ? 0u : (1u << uint32_t(rem)) - 1u;
      const uint32_t cnt = __builtin_popcount(m);
      const uint32_t incl = wv::scan_incl(cnt, 0u, [](uint32_t e, uint32_t l) { return e + l; });
      uint32_t r = base + incl - cnt;
      while (m) {
        const uint32_t pos = wpos + jl::ctz32(m);
        if (r < JSON_FUSE_MAX_LINES) nlpos[r] = pos;
        a.nl_out[r++] = pos;
        m &= m - 1;
      }
      base += wv::last_uniform(incl);
    }
    if (lane == 0) {
      a.off2[0] = 0;
      a.off2[1] = base;
    }
    // nlpos[0 .. nlines) must all be written: the host's line count is the staged newline count
    DR_LDS_CHECK(base >= nlines && nlines <= JSON_FUSE_MAX_LINES, "k_apply_commit newlines", base, nlines);
  }
  __syncthreads();
  phase(1);
  const uint32_t per = (nlines + AC_WAVES - 1) / AC_WAVES;  // lines per wave (<= AC_LINES)
  const uint32_t l0 = w * per, l1 = min(l0 + per, nlines);
  if (l0 < l1) {
    const uint32_t nw = l1 - l0;
    const uint32_t rb = l0 ? nlpos[l0 - 1] + 1u : 0u;
    const uint32_t R = nlpos[l1 - 1] + 1u - rb;
    const bool taped = build_tape<AC_TCAP, AC_LINES, AC_SW>(stage, rb, R, nw, tape[w], nltok[w], tline[w]);
    wave_sync();
    if (taped) {
      tape_lines<AC_TCAP, AC_LINES>(a, l0, nw, reinterpret_cast<const uint8_t*>(stage) + rb, AC_SW * 16 - rb, rb,
                                    tape[w], nltok[w], tline[w], agg[w]);
    } else if (lane < nw) {  // off the tape: the General walker (apply_small_body) decides these lines
      const unsigned long long k = atomicAdd(a.hard_count, 1ull);
      a.hard_idx[k] = l0 + lane;
    }
  }
  __threadfence();
  __syncthreads();
  phase(2);
  apply_small_body(a, c, p, x, true);
  phase(6);
  if (a.phase && t == 0) atomicAdd(&a.phase[4], 1ull);
  // r06: the expiry of a short tombstone-candidate list and the readback, which followed as a second
  // launch (k_ix_expire or k_readback), run here behind a fence and a barrier: one launch per commit
  if (exp_n | rb.n[0]) {  // kernel arguments: uniform
    __threadfence();
    __syncthreads();
    if (exp_n) {
      Contrib ce{0, 0, 0, 0, 0};
      // one workgroup walks the whole list: EXP_U entries per thread in flight (most fail the cutoff
      // window on the entry alone, so the list loads are the chain to overlap)
      constexpr uint32_t EXP_U = 8, EXP_STEP = AC_WAVES * 64;
      for (uint64_t j0 = t; j0 < exp_n; j0 += EXP_U * EXP_STEP) {
        ulonglong2 e[EXP_U];
#pragma unroll
        for (uint32_t u = 0; u < EXP_U; ++u) {
          const uint64_t j = j0 + u * EXP_STEP;
          e[u] = j < exp_n ? x.tomb_list[j] : make_ulonglong2(~0ull, 0ull);  // ~0: outside [0, lo)
        }
#pragma unroll
        for (uint32_t u = 0; u < EXP_U; ++u) expire_entry(x, e[u], ce);
      }
      flush_contrib(x, ce, 0);
      __threadfence();
      __syncthreads();
      phase(12);
    }
#pragma unroll
    for (int s = 0; s < READBACK_SPANS; ++s)
      for (uint32_t k = t; k < rb.n[s]; k += AC_WAVES * 64)
        rb.dst[s][k] = __hip_atomic_load(rb.src[s] + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    readback_flag(rb);
    phase(13);
  }
}

}  // namespace dev

// ---- launchers -----------------------------------------------------------------------------------
uint64_t json_num_blocks(uint64_t len) { return (len + dev::JSON_BYTES_PER_BLOCK - 1) / dev::JSON_BYTES_PER_BLOCK; }

uint64_t json_slot_entries(uint64_t len) { return json_num_blocks(len) * dev::JSON_SLOT; }

void launch_json_index(const uint8_t* buf, uint64_t len, uint32_t* block_counts, uint16_t* slots, hipStream_t st) {
  uint64_t nb = json_num_blocks(len);
  if (nb) DR_LAUNCH(dev::k_json_index, dim3(unsigned(nb)), dim3(dev::JSON_THREADS), 0, st, buf, len,
                             block_counts, slots);
}

void launch_json_place(const uint8_t* buf, uint64_t len, const uint32_t* block_counts, const uint64_t* block_off,
                       const uint16_t* slots, uint64_t* nl, hipStream_t st) {
  uint64_t nb = json_num_blocks(len);
  if (nb) DR_LAUNCH(dev::k_json_place, dim3(unsigned(nb)), dim3(dev::JSON_THREADS), 0, st, buf, len,
                             block_counts, block_off, slots, nl);
}

void launch_json_index1(const uint8_t* buf, uint64_t len, uint64_t* nl, uint64_t* off2, uint64_t* zero,
                        uint32_t nzero, hipStream_t st) {
  DR_LAUNCH(dev::k_json_index1, dim3(1), dim3(dev::JSON_THREADS), 0, st, buf, len, nl, off2, zero, nzero);
}

void launch_json_parse(const JsonParseArgs& a, hipStream_t st) {
  if (!a.nlines) return;
  const dim3 grid(unsigned((a.nlines + dev::JL_T - 1) / dev::JL_T));
  // DR_OPT_JSON_STAGED (tests): every segment through the staged kernel, 64 lines per workgroup
  if (a.nlines <= dev::JL_SMALL_LINES || a.force_staged) DR_LAUNCH(dev::k_json_lines<true>, grid, dim3(dev::JL_T), 0, st, a);
  else DR_LAUNCH(dev::k_json_lines<false>, grid, dim3(dev::JL_T), 0, st, a);
}

void launch_tail_post(const JsonParseArgs& a, const CanonArgs& c, hipStream_t st) {
  DR_LAUNCH(dev::k_tail_post, dim3(1), dim3(256), 0, st, a, c);
}

void launch_apply_small(const JsonParseArgs* ja, const CanonArgs& cg, const AppendArgs& ap, const IndexArgs& ix,
                        hipStream_t st) {
  JsonParseArgs none{};
  DR_LAUNCH(dev::k_apply_small, dim3(1), dim3(dev::IX_T), 0, st, ja ? *ja : none, cg, ap, ix);
}

void launch_apply_commit(const JsonParseArgs& ja, const CanonArgs& cg, const AppendArgs& ap, const IndexArgs& ix,
                         hipStream_t st, uint64_t exp_n, const ReadbackArgs* rb) {
  ReadbackArgs none{};
  DR_LAUNCH(dev::k_apply_commit, dim3(1), dim3(dev::AC_WAVES * 64), 0, st, ja, cg, ap, ix, exp_n, rb ? *rb : none);
}

void launch_json_hard(const JsonParseArgs& a, hipStream_t st) {
  if (!a.nlines) return;
  // grid-stride over the device-side count of deferred lines (usually none: the workgroups exit)
  const unsigned g = unsigned(std::min<uint64_t>(256, (a.nlines + 63) / 64));
  DR_LAUNCH(dev::k_json_hard, dim3(g), dim3(64), 0, st, a);
}

}  // namespace dr
