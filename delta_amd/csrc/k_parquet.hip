// K2: Parquet checkpoint decode on the GPU (replaces Spark's ParquetFileFormat / parquet-mr record
// assembly over the checkpoint, D/DeltaLogFileIndex.scala:68, D/Snapshot.scala:244-263).
//
// Pages are planned on the host (footer + page headers); the device inflates SNAPPY pages into an
// arena, decodes dictionary pages into a pool, then decodes v1/v2 data pages of the flat
// file-action columns (add.path, add.size, remove.path, remove.deletionTimestamp): RLE/bit-packed
// definition levels, PLAIN and PLAIN_DICTIONARY/RLE_DICTIONARY values.
#include "dev_common.h"
#include "kernels.h"

namespace dr {
namespace dev {

enum PqErr : uint32_t { PQE_SNAPPY = 1, PQE_LEVELS = 2, PQE_VALUES = 3, PQE_DICT = 4, PQE_ENCODING = 5 };

__device__ __forceinline__ void set_err(uint32_t* e, uint32_t code) { atomicCAS(e, 0u, code); }

// ---- SNAPPY (one lane per page) ------------------------------------------------------------------
__device__ bool snappy_page(const uint8_t* in, uint32_t n, uint8_t* out, uint32_t out_len) {
  uint32_t ip = 0;
  uint64_t total = 0;
  for (int s = 0; ip < n && s < 35; s += 7) {
    uint8_t b = in[ip++];
    total |= uint64_t(b & 0x7f) << s;
    if (!(b & 0x80)) break;
  }
  if (total != out_len) return false;
  uint32_t op = 0;
  while (ip < n) {
    const uint8_t tag = in[ip++];
    const uint32_t t = tag & 3;
    uint32_t len, off = 0;
    if (t == 0) {
      len = tag >> 2;
      if (len >= 60) {
        const uint32_t nb = len - 59;
        if (ip + nb > n) return false;
        len = 0;
        for (uint32_t b = 0; b < nb; ++b) len |= uint32_t(in[ip + b]) << (8 * b);
        ip += nb;
      }
      len += 1;
      if (ip + len > n || op + len > out_len) return false;
      for (uint32_t k = 0; k < len; ++k) out[op + k] = in[ip + k];
      ip += len;
      op += len;
      continue;
    }
    if (t == 1) {
      if (ip + 1 > n) return false;
      len = ((tag >> 2) & 7) + 4;
      off = (uint32_t(tag >> 5) << 8) | in[ip];
      ip += 1;
    } else if (t == 2) {
      if (ip + 2 > n) return false;
      len = (tag >> 2) + 1;
      off = uint32_t(in[ip]) | (uint32_t(in[ip + 1]) << 8);
      ip += 2;
    } else {
      if (ip + 4 > n) return false;
      len = (tag >> 2) + 1;
      off = uint32_t(in[ip]) | (uint32_t(in[ip + 1]) << 8) | (uint32_t(in[ip + 2]) << 16) |
            (uint32_t(in[ip + 3]) << 24);
      ip += 4;
    }
    if (off == 0 || off > op || op + len > out_len) return false;
    for (uint32_t k = 0; k < len; ++k) out[op + k] = out[op - off + k];
    op += len;
  }
  return op == out_len;
}

__global__ void k_pq_inflate(ParquetArgs a) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.npages) return;
  const PageDesc& pg = a.pages[i];
  const uint8_t* src = reinterpret_cast<const uint8_t*>(pg.src);
  uint8_t* dst = reinterpret_cast<uint8_t*>(pg.dst);
  uint32_t lv = pg.kind == PG_DATA_V2 ? uint32_t(pg.v2_def_len + pg.v2_rep_len) : 0u;
  for (uint32_t k = 0; k < lv; ++k) dst[k] = src[k];
  const bool compressed = pg.codec == 1 && !(pg.kind == PG_DATA_V2 && !pg.v2_compressed);
  if (compressed) {
    if (!snappy_page(src + lv, pg.csize - lv, dst + lv, pg.usize - lv)) set_err(a.error, PQE_SNAPPY);
  } else {
    for (uint32_t k = lv; k < pg.usize; ++k) dst[k] = src[k];
  }
}

// ---- RLE / bit-packed hybrid decoder -------------------------------------------------------------
struct Rle {
  const uint8_t* p;
  const uint8_t* end;
  int width;
  uint32_t run_left;   // values left in the current run
  bool packed;
  uint32_t value;      // RLE value
  uint64_t acc;        // bit-packed accumulator
  int have;
  bool bad;

  __device__ void init(const uint8_t* b, const uint8_t* e, int w) {
    p = b; end = e; width = w; run_left = 0; packed = false; value = 0; acc = 0; have = 0; bad = false;
  }
  __device__ bool next_run() {
    uint64_t h = 0;
    int s = 0;
    for (;;) {
      if (p >= end) { bad = true; return false; }
      uint8_t b = *p++;
      h |= uint64_t(b & 0x7f) << s;
      s += 7;
      if (!(b & 0x80)) break;
      if (s > 63) { bad = true; return false; }
    }
    if (h & 1) {
      packed = true;
      run_left = uint32_t(h >> 1) * 8;
      acc = 0;
      have = 0;
    } else {
      packed = false;
      run_left = uint32_t(h >> 1);
      value = 0;
      for (int b = 0; b < (width + 7) / 8; ++b) {
        if (p >= end) { bad = true; return false; }
        value |= uint32_t(*p++) << (8 * b);
      }
    }
    return true;
  }
  __device__ uint32_t get() {
    while (run_left == 0) {
      if (!next_run()) return 0;
    }
    --run_left;
    if (!packed) return value;
    while (have < width) {
      acc |= uint64_t(p < end ? *p : 0) << have;
      ++p;
      have += 8;
    }
    uint32_t v = width ? uint32_t(acc & ((1ull << width) - 1)) : 0;
    acc >>= width;
    have -= width;
    return v;
  }
};

__device__ __forceinline__ int level_width(int max_level) {
  int w = 0;
  while ((1 << w) <= max_level) ++w;
  return max_level == 0 ? 0 : w;
}

__global__ void k_pq_dict(ParquetArgs a) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.npages) return;
  const PageDesc& pg = a.pages[i];
  if (pg.kind != PG_DICT) return;
  const uint8_t* p = reinterpret_cast<const uint8_t*>(pg.dst);
  const uint8_t* end = p + pg.usize;
  for (uint32_t k = 0; k < pg.num_values; ++k) {
    if (pg.phys == 6) {  // BYTE_ARRAY
      if (end - p < 4) { set_err(a.error, PQE_DICT); return; }
      uint32_t l = load_u32(p);
      p += 4;
      if (uint64_t(end - p) < l) { set_err(a.error, PQE_DICT); return; }
      a.dict_ptr[pg.dict_base + k] = reinterpret_cast<uint64_t>(p);
      a.dict_len[pg.dict_base + k] = l;
      p += l;
    } else if (pg.phys == 2) {
      if (end - p < 8) { set_err(a.error, PQE_DICT); return; }
      a.dict_ptr[pg.dict_base + k] = load_u64(p);
      p += 8;
    } else if (pg.phys == 1) {
      if (end - p < 4) { set_err(a.error, PQE_DICT); return; }
      a.dict_ptr[pg.dict_base + k] = uint64_t(int64_t(int32_t(load_u32(p))));
      p += 4;
    } else {
      set_err(a.error, PQE_ENCODING);
      return;
    }
  }
}

__global__ void k_pq_data(ParquetArgs a) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.npages) return;
  const PageDesc& pg = a.pages[i];
  if (pg.kind == PG_DICT) return;
  const FlatColumn& col = a.cols[pg.col];
  const uint8_t* p = reinterpret_cast<const uint8_t*>(pg.dst);
  const uint8_t* end = p + pg.usize;
  const int dw = level_width(pg.max_def);
  Rle defs;
  if (pg.kind == PG_DATA_V2) {
    defs.init(p + pg.v2_rep_len, p + pg.v2_rep_len + pg.v2_def_len, dw);
    p += pg.v2_rep_len + pg.v2_def_len;
  } else if (pg.max_def > 0) {
    if (end - p < 4) { set_err(a.error, PQE_LEVELS); return; }
    uint32_t l = load_u32(p);
    p += 4;
    if (uint64_t(end - p) < l) { set_err(a.error, PQE_LEVELS); return; }
    defs.init(p, p + l, dw);
    p += l;
  }
  const bool dict = pg.encoding == 2 || pg.encoding == 8;
  Rle idx;
  if (dict) {
    if (pg.dict < 0) { set_err(a.error, PQE_DICT); return; }
    int w = p < end ? *p : 0;
    idx.init(p + 1, end, w);
  } else if (pg.encoding != 0) {
    set_err(a.error, PQE_ENCODING);
    return;
  }
  const uint32_t dict_base = dict ? a.pages[pg.dict].dict_base : 0;
  const uint32_t dict_n = dict ? a.pages[pg.dict].num_values : 0;
  uint32_t bool_bit = 0;
  for (uint32_t k = 0; k < pg.num_values; ++k) {
    const uint64_t row = pg.row_base + k;
    int d = pg.max_def > 0 ? int(defs.get()) : 0;
    if (defs.bad && pg.max_def > 0) { set_err(a.error, PQE_LEVELS); return; }
    col.def[row] = uint8_t(d);
    if (d != pg.max_def) continue;
    if (dict) {
      uint32_t j = idx.get();
      if (idx.bad || j >= dict_n) { set_err(a.error, PQE_DICT); return; }
      if (pg.phys == 6) {
        col.sptr[row] = a.dict_ptr[dict_base + j];
        col.slen[row] = a.dict_len[dict_base + j];
      } else {
        col.ival[row] = int64_t(a.dict_ptr[dict_base + j]);
      }
    } else if (pg.phys == 6) {
      if (end - p < 4) { set_err(a.error, PQE_VALUES); return; }
      uint32_t l = load_u32(p);
      p += 4;
      if (uint64_t(end - p) < l) { set_err(a.error, PQE_VALUES); return; }
      col.sptr[row] = reinterpret_cast<uint64_t>(p);
      col.slen[row] = l;
      p += l;
    } else if (pg.phys == 2) {
      if (end - p < 8) { set_err(a.error, PQE_VALUES); return; }
      col.ival[row] = int64_t(load_u64(p));
      p += 8;
    } else if (pg.phys == 1) {
      if (end - p < 4) { set_err(a.error, PQE_VALUES); return; }
      col.ival[row] = int64_t(int32_t(load_u32(p)));
      p += 4;
    } else if (pg.phys == 0) {
      col.ival[row] = (p[bool_bit >> 3] >> (bool_bit & 7)) & 1;
      ++bool_bit;
    } else {
      set_err(a.error, PQE_ENCODING);
      return;
    }
  }
}

// Checkpoint row -> action. unwrap priority add > remove (D/actions/actions.scala:523-541);
// rows holding neither are protocol/metaData/txn rows decoded on the host.
__global__ void k_ckpt_assemble(CkptAssembleArgs a) {
  const uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (r >= a.nrows) return;
  const uint64_t idx = a.row_base + r;
  uint8_t kind = K_NONE, flags = F_FROM_CKPT;
  const uint8_t* path = nullptr;
  uint32_t plen = 0;
  int64_t size = 0, delts = 0;
  const int ad = a.add_path.def[r];
  const int rd = a.has_rm ? int(a.rm_path.def[r]) : 0;
  if (ad >= a.add_def) {
    kind = K_ADD;
    if (ad == a.add_path_max) {
      path = reinterpret_cast<const uint8_t*>(a.add_path.sptr[r]);
      plen = a.add_path.slen[r];
    } else {
      flags |= F_PATH_NULL;
    }
    if (a.add_size.def[r] == a.add_size_max) size = a.add_size.ival[r];
  } else if (a.has_rm && rd >= a.rm_def) {
    kind = K_REMOVE;
    if (rd == a.rm_path_max) {
      path = reinterpret_cast<const uint8_t*>(a.rm_path.sptr[r]);
      plen = a.rm_path.slen[r];
    } else {
      flags |= F_PATH_NULL;
    }
    if (a.rm_delts.def && a.rm_delts.def[r] == a.rm_delts_max) {
      delts = a.rm_delts.ival[r];
      flags |= F_HAS_DELTS;
    }
  }
  uint64_t key = 0;
  if ((kind == K_ADD || kind == K_REMOVE) && !(flags & F_PATH_NULL)) {
    if (path_is_special(path, plen)) {
      flags |= F_SPECIAL_PATH;
      atomicAdd(reinterpret_cast<unsigned long long*>(a.special_count), 1ull);
      atomicAdd(reinterpret_cast<unsigned long long*>(a.special_bytes), (unsigned long long)(plen + 8));
    } else {
      key = path_key(path, plen);
    }
  }
  a.act.kind[idx] = kind;
  a.act.flags[idx] = flags;
  a.act.key[idx] = key;
  a.act.path_ptr[idx] = reinterpret_cast<uint64_t>(path);
  a.act.path_len[idx] = plen;
  a.act.size[idx] = size;
  a.act.delts[idx] = delts;
  a.act.src_off[idx] = r;
  a.act.src_len[idx] = 0;
}

}  // namespace dev

void launch_pq_inflate(const ParquetArgs& a, hipStream_t st) {
  if (a.npages) hipLaunchKernelGGL(dev::k_pq_inflate, dim3((a.npages + 63) / 64), dim3(64), 0, st, a);
}
void launch_pq_dict(const ParquetArgs& a, hipStream_t st) {
  if (a.npages) hipLaunchKernelGGL(dev::k_pq_dict, dim3((a.npages + 63) / 64), dim3(64), 0, st, a);
}
void launch_pq_data(const ParquetArgs& a, hipStream_t st) {
  if (a.npages) hipLaunchKernelGGL(dev::k_pq_data, dim3((a.npages + 63) / 64), dim3(64), 0, st, a);
}
void launch_ckpt_assemble(const CkptAssembleArgs& a, hipStream_t st) {
  if (a.nrows) hipLaunchKernelGGL(dev::k_ckpt_assemble, dim3(unsigned((a.nrows + 255) / 256)), dim3(256), 0, st, a);
}

}  // namespace dr
