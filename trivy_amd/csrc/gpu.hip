// MI355X (gfx950) device path of the secret engine: K1 keyword automaton and K2
// rule-group DFAs over a device-resident batch of file blobs.
//
// Work decomposition: files are packed back to back in one HBM stream; a lane owns a
// chunk of `chunk` bytes (a chunk may hold pieces of several files).  For each file
// piece [a, b) the lane runs the DFA in inject mode (a thread starts at every byte)
// and, if the file continues past b, follows the threads that started inside its
// piece in noinject mode until they have all died (K2), or keeps going for the
// longest-keyword overlap (K1).  Every match start is owned by exactly one lane, so no
// lane needs state from a neighbour and the reported end offsets are exact for the
// DFA's language (dfa.hpp).
//
//   K1   dense over every chunk: keyword bits per file (per-lane LDS accumulator,
//        one atomicOr per word per piece).
//   gate one thread per file: which K2 groups a file's keyword bits switch on; per
//        group gated bytes/files (LDS atomics, one global atomic per block).
//   K2   per rule group: DENSE (every chunk, lanes skip ungated pieces) when the group
//        is gated on a large share of the batch, otherwise LIST: only the (file, chunk)
//        items of gated files, appended by the gate_list pass.  Accepts append
//        {file, rule, end} candidate records with an atomic counter.
// Tables: transitions (u16: next | 0x8000 accept bit), byte classes, and -- when the
// DFA's accepts depend on the state only (no look-ahead assertion) -- the per-state
// accept index and the accept masks all live in LDS, so an accept never waits on L2.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <vector>

#include "internal.hpp"

namespace tsg {

#define HIP_TRY(x)                                                                    \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess)                                                             \
      return fail(TSG_ERR_GPU, std::string(#x) + ": " + hipGetErrorString(e_));       \
  } while (0)

struct DevDFA {
  const uint16_t* tab;        // [ns * nc] next | 0x8000 if the transition accepts
  const uint16_t* acc;        // [ns * nc] accept-mask index (look-ahead DFAs)
  const uint16_t* acc_state;  // [ns] accept-mask index per state (state_acc DFAs)
  const uint16_t* eot;        // [ns] accept-mask index at end of text
  const uint16_t* to_ni;      // [ns] noinject twin
  const uint8_t* dead;        // [ns]
  const uint64_t* masks;      // [nmasks * mw]
  const uint8_t* cls;         // [256]
  const uint32_t* rules;      // K2: group-local id -> global rule
  uint32_t nc, ns, mw, nmasks, state_acc, ext;
  uint32_t start[4];
  // LDS layout (bytes)
  uint32_t o_cls, o_accs, o_masks, o_kwacc, lds_bytes;
};

struct DevCand {
  uint32_t file, rule, end;
};

// ---------------------------------------------------------------- small kernels
__global__ void chunk_file_kernel(const uint64_t* __restrict__ off, uint32_t nfiles, uint32_t chunk,
                                  uint32_t* __restrict__ chunk_file) {
  uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= nfiles) return;
  uint64_t fs = off[f], fe = off[f + 1];
  if (fe == fs) return;
  uint64_t c0 = (fs + chunk - 1) / chunk, c1 = (fe + chunk - 1) / chunk;  // chunks starting in f
  for (uint64_t c = c0; c < c1; c++) chunk_file[c] = f;
}

__device__ __forceinline__ bool group_gated(const uint32_t* __restrict__ kwf, const uint32_t* __restrict__ gm,
                                            uint32_t W, uint32_t always) {
  if (always) return true;
  for (uint32_t w = 0; w < W; w++)
    if (kwf[w] & gm[w]) return true;
  return false;
}

// per group: gated bytes and files (block-local LDS atomics, then one global atomic)
__global__ void gate_count_kernel(const uint64_t* __restrict__ off, uint32_t nfiles,
                                  const uint32_t* __restrict__ kw, uint32_t W,
                                  const uint32_t* __restrict__ gmask, const uint32_t* __restrict__ galways,
                                  uint32_t G, unsigned long long* __restrict__ gbytes,
                                  uint32_t* __restrict__ gfiles) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  unsigned long long* sb = (unsigned long long*)smem;
  uint32_t* sf = (uint32_t*)(sb + G);
  for (uint32_t g = threadIdx.x; g < G; g += blockDim.x) {
    sb[g] = 0;
    sf[g] = 0;
  }
  __syncthreads();
  uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f < nfiles) {
    uint64_t len = off[f + 1] - off[f];
    if (len) {
      const uint32_t* kwf = kw + (size_t)f * W;
      for (uint32_t g = 0; g < G; g++)
        if (group_gated(kwf, gmask + (size_t)g * W, W, galways[g])) {
          atomicAdd(&sb[g], (unsigned long long)len);
          atomicAdd(&sf[g], 1u);
        }
    }
  }
  __syncthreads();
  for (uint32_t g = threadIdx.x; g < G; g += blockDim.x) {
    if (sb[g]) atomicAdd(&gbytes[g], sb[g]);
    if (sf[g]) atomicAdd(&gfiles[g], sf[g]);
  }
}

// LIST-mode groups: append one (file, chunk) item per chunk a gated file touches
__global__ void gate_list_kernel(const uint64_t* __restrict__ off, uint32_t nfiles,
                                 const uint32_t* __restrict__ kw, uint32_t W,
                                 const uint32_t* __restrict__ gmask, const uint32_t* __restrict__ galways,
                                 const uint32_t* __restrict__ list_groups, uint32_t nlist,
                                 const uint64_t* __restrict__ item_base, uint32_t* __restrict__ item_count,
                                 uint2* __restrict__ items, uint32_t chunk) {
  uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= nfiles) return;
  uint64_t fs = off[f], fe = off[f + 1];
  if (fe == fs) return;
  const uint32_t* kwf = kw + (size_t)f * W;
  uint32_t c0 = (uint32_t)(fs / chunk), c1 = (uint32_t)((fe - 1) / chunk);
  for (uint32_t j = 0; j < nlist; j++) {
    uint32_t g = list_groups[j];
    if (!group_gated(kwf, gmask + (size_t)g * W, W, galways[g])) continue;
    uint32_t n = c1 - c0 + 1;
    uint32_t base = atomicAdd(&item_count[j], n);
    uint2* it = items + item_base[j] + base;
    for (uint32_t k = 0; k < n; k++) it[k] = make_uint2(f, c0 + k);
  }
}

// ---------------------------------------------------------------- the scan kernel
__device__ __forceinline__ uint32_t ctx_of(uint8_t c) {
  if (c == '\n') return 1;
  if ((c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_') return 2;
  return 3;
}

// dense items are kStreams consecutive chunks; inside one file they are stepped as
// kStreams interleaved DFA chains (ILP to cover the LDS latency)
constexpr int kStreams = 4;

struct ScanArgsDev {
  const uint8_t* data;
  const uint64_t* off;
  const uint32_t* chunk_file;
  uint64_t total, nitems;
  uint32_t chunk, ext_cap;
  uint32_t* kw;
  uint32_t kw_words;
  const uint32_t* gmask;  // K2 dense: this group's keyword mask [kw_words]
  uint32_t galways;
  const uint2* items;     // K2 list mode
  DevCand* cand;
  uint32_t* cand_count;
  uint32_t cand_cap;
  uint32_t* ovf;
};

template <bool KW>
struct Lane {
  const DevDFA& d;
  const ScanArgsDev& A;
  const uint16_t* s_tab;
  const uint8_t* s_cls;
  const uint16_t* s_accs;
  const uint64_t* s_masks;
  uint32_t* s_kwacc;
  uint32_t file;
  uint64_t fs;

  // rare path (an accept); the unrolled loops below never call it directly: they only OR
  // the accept bits of 16 transitions and replay the word through step() when one is set
  __device__ __forceinline__ void emit(uint32_t mi, uint64_t pos) {
    const uint64_t* m = (d.state_acc && mi < d.nmasks) ? s_masks + (size_t)mi * d.mw : d.masks + (size_t)mi * d.mw;
    if (KW) {
      for (uint32_t w = 0; w < d.mw; w++) {
        uint64_t v = m[w];
        if (2 * w < A.kw_words) s_kwacc[(2 * w) * blockDim.x + threadIdx.x] |= (uint32_t)v;
        if (2 * w + 1 < A.kw_words) s_kwacc[(2 * w + 1) * blockDim.x + threadIdx.x] |= (uint32_t)(v >> 32);
      }
    } else {
      uint64_t v = m[0];
      while (v) {
        uint32_t k = __builtin_ctzll(v);
        v &= v - 1;
        uint32_t idx = atomicAdd(A.cand_count, 1u);
        if (idx < A.cand_cap) {
          A.cand[idx].file = file;
          A.cand[idx].rule = d.rules[k];
          A.cand[idx].end = (uint32_t)(pos - fs);
        } else {
          A.ovf[file] = 1;
        }
      }
    }
  }

  __device__ __forceinline__ uint32_t step(uint32_t s, uint32_t byte, uint64_t pos) {
    const uint32_t ix = s * d.nc + s_cls[byte];
    const uint32_t e = s_tab[ix];
    if (__builtin_expect(e & 0x8000u, 0)) emit(d.state_acc ? s_accs[s] : d.acc[ix], pos);
    return e & 0x7FFFu;
  }

  // transition only; accept bit returned in bit 15
  __device__ __forceinline__ uint32_t fast(uint32_t s, uint32_t byte) const {
    return s_tab[s * d.nc + s_cls[byte]];
  }

  // 16 bytes: tight loop, then a (rare) replay with accept handling
  __device__ __forceinline__ uint32_t step16(uint32_t s, const uint4 v, uint64_t p) {
    const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
    const uint32_t s0 = s;
    uint32_t any = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t e = fast(s, (wv[k >> 2] >> ((k & 3) * 8)) & 0xFF);
      any |= e;
      s = e & 0x7FFFu;
    }
    if (__builtin_expect(any & 0x8000u, 0)) replay16(s0, v, p);
    return s;
  }

  // no dynamically indexed arrays (they would live in scratch): bytes are selected
  __device__ __forceinline__ void replay16(uint32_t s, const uint4 v, uint64_t p) {
#pragma unroll 1
    for (uint32_t k = 0; k < 16; k++) {
      const uint32_t w = k < 8 ? (k < 4 ? v.x : v.y) : (k < 12 ? v.z : v.w);
      s = step(s, (w >> ((k & 3) * 8)) & 0xFF, p + k);
    }
  }

  // tail of a stream that ends at b (< fe): K1 keyword overlap / K2 noinject follow-up
  __device__ __forceinline__ void tail(uint32_t s, uint64_t fe, uint64_t b) {
    const uint8_t* data = A.data;
    if (KW) {
      const uint64_t le = min(fe, b + d.ext);
      uint64_t q = b;
      for (; q < le; q++) s = step(s, data[q], q);
      if (q >= fe) {
        const uint32_t m = d.eot[s];
        if (m) emit(m, fe);
      }
      return;
    }
    if (b >= fe) {
      const uint32_t m = d.eot[s];
      if (m) emit(m, fe);
      return;
    }
    s = d.to_ni[s];
    uint64_t q = b;
    while (q < fe && !d.dead[s]) {
      if (q - b >= A.ext_cap) {
        A.ovf[file] = 1;
        return;
      }
      s = step(s, data[q], q);
      q++;
    }
    if (q == fe && !d.dead[s]) {
      const uint32_t m = d.eot[s];
      if (m) emit(m, fe);
    }
  }

  // NS consecutive chunks [a, a + NS*C) that all lie inside file [fs, fe): NS independent
  // DFA chains interleaved byte by byte, so NS LDS look-ups are in flight per lane
  template <int NS>
  __device__ void streams(uint64_t fe, uint64_t a, uint32_t C) {
    const uint8_t* data = A.data;
    if (KW)
      for (uint32_t w = 0; w < A.kw_words; w++) s_kwacc[w * blockDim.x + threadIdx.x] = 0;
    uint32_t s[NS];
#pragma unroll
    for (int i = 0; i < NS; i++) {
      const uint64_t b0 = a + (uint64_t)i * C;
      s[i] = (b0 == fs) ? d.start[0] : d.start[ctx_of(data[b0 - 1])];
    }
    uint4 cur[NS];
#pragma unroll
    for (int i = 0; i < NS; i++) cur[i] = *(const uint4*)(data + a + (uint64_t)i * C);
    for (uint32_t j = 0; j < C; j += 16) {
      uint4 nxt[NS];
#pragma unroll
      for (int i = 0; i < NS; i++) nxt[i] = *(const uint4*)(data + a + (uint64_t)i * C + j + 16);
      uint32_t wv[NS][4];
#pragma unroll
      for (int i = 0; i < NS; i++) {
        wv[i][0] = cur[i].x;
        wv[i][1] = cur[i].y;
        wv[i][2] = cur[i].z;
        wv[i][3] = cur[i].w;
      }
      uint32_t s0[NS], any[NS];
#pragma unroll
      for (int i = 0; i < NS; i++) {
        s0[i] = s[i];
        any[i] = 0;
      }
#pragma unroll
      for (int k = 0; k < 16; k++)
#pragma unroll
        for (int i = 0; i < NS; i++) {
          const uint32_t e = fast(s[i], (wv[i][k >> 2] >> ((k & 3) * 8)) & 0xFF);
          any[i] |= e;
          s[i] = e & 0x7FFFu;
        }
#pragma unroll
      for (int i = 0; i < NS; i++)
        if (__builtin_expect(any[i] & 0x8000u, 0)) replay16(s0[i], cur[i], a + (uint64_t)i * C + j);
#pragma unroll
      for (int i = 0; i < NS; i++) cur[i] = nxt[i];
    }
#pragma unroll
    for (int i = 0; i < NS; i++) tail(s[i], fe, a + (uint64_t)(i + 1) * C);
    if (KW)
      for (uint32_t w = 0; w < A.kw_words; w++) {
        uint32_t v = s_kwacc[w * blockDim.x + threadIdx.x];
        if (v) atomicOr(&A.kw[(size_t)file * A.kw_words + w], v);
      }
  }

  // one file piece [a, se) of file [fs, fe)
  __device__ void piece(uint64_t fe, uint64_t a, uint64_t se) {
    const uint8_t* data = A.data;
    if (KW)
      for (uint32_t w = 0; w < A.kw_words; w++) s_kwacc[w * blockDim.x + threadIdx.x] = 0;
    uint32_t s = (a == fs) ? d.start[0] : d.start[ctx_of(data[a - 1])];
    uint64_t p = a;
    const uint64_t le = KW ? min(fe, se + d.ext) : se;
    while (p < le && (p & 15)) {
      s = step(s, data[p], p);
      p++;
    }
    if (p + 16 <= le) {
      // one 16-byte word in flight ahead of the one being stepped (the stream is padded
      // by 64 bytes, so the look-ahead load never leaves the allocation)
      uint4 cur = *(const uint4*)(data + p);
      while (p + 16 <= le) {
        const uint4 nxt = *(const uint4*)(data + p + 16);
        s = step16(s, cur, p);
        cur = nxt;
        p += 16;
      }
    }
    while (p < le) {
      s = step(s, data[p], p);
      p++;
    }
    if (le >= fe) {
      const uint32_t m = d.eot[s];
      if (m) emit(m, fe);
    } else if (!KW) {
      // follow the threads that started in [a, se) past the chunk end
      s = d.to_ni[s];
      uint64_t q = se;
      bool over = false;
      while (q < fe && !d.dead[s]) {
        if (q - se >= A.ext_cap) {
          over = true;
          break;
        }
        s = step(s, data[q], q);
        q++;
      }
      if (over) {
        A.ovf[file] = 1;
      } else if (q == fe && !d.dead[s]) {
        const uint32_t m = d.eot[s];
        if (m) emit(m, fe);
      }
    }
    if (KW)
      for (uint32_t w = 0; w < A.kw_words; w++) {
        uint32_t v = s_kwacc[w * blockDim.x + threadIdx.x];
        if (v) atomicOr(&A.kw[(size_t)file * A.kw_words + w], v);
      }
  }
};

template <bool KW, bool LIST>
__global__ void __launch_bounds__(256) dfa_scan_kernel(DevDFA d, ScanArgsDev A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint16_t* s_tab = (uint16_t*)smem;
  uint8_t* s_cls = smem + d.o_cls;
  uint16_t* s_accs = (uint16_t*)(smem + d.o_accs);
  uint64_t* s_masks = (uint64_t*)(smem + d.o_masks);
  const uint32_t tab_entries = d.ns * d.nc;
  {
    const uint32_t* src = (const uint32_t*)d.tab;
    uint32_t* dst = (uint32_t*)s_tab;
    for (uint32_t i = threadIdx.x; i < (tab_entries + 1) / 2; i += blockDim.x) dst[i] = src[i];
  }
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) s_cls[i] = d.cls[i];
  if (d.state_acc) {
    for (uint32_t i = threadIdx.x; i < d.ns; i += blockDim.x) s_accs[i] = d.acc_state[i];
    for (uint32_t i = threadIdx.x; i < d.nmasks * d.mw; i += blockDim.x) s_masks[i] = d.masks[i];
  }
  __syncthreads();

  Lane<KW> L{d, A, s_tab, s_cls, s_accs, s_masks, (uint32_t*)(smem + d.o_kwacc), 0, 0};
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t it = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; it < A.nitems; it += stride) {
    if (LIST) {
      const uint2 item = A.items[it];
      const uint32_t f = item.x;
      const uint64_t fs = A.off[f], fe = A.off[f + 1];
      const uint64_t a = max(fs, (uint64_t)item.y * A.chunk);
      const uint64_t b = min(fe, (uint64_t)(item.y + 1) * A.chunk);
      if (a < b) {
        L.file = f;
        L.fs = fs;
        L.piece(fe, a, b);
      }
    } else {
      // item = kStreams consecutive chunks
      uint64_t a = it * kStreams * A.chunk;
      const uint64_t b = min(a + (uint64_t)kStreams * A.chunk, A.total);
      uint32_t f = A.chunk_file[it * kStreams];
      {
        const uint64_t fs = A.off[f], fe = A.off[f + 1];
        if (b == a + (uint64_t)kStreams * A.chunk && b <= fe) {  // common case: one file
          if (KW || group_gated(A.kw + (size_t)f * A.kw_words, A.gmask, A.kw_words, A.galways)) {
            L.file = f;
            L.fs = fs;
            L.template streams<kStreams>(fe, a, A.chunk);
          }
          continue;
        }
      }
      while (a < b) {
        const uint64_t fs = A.off[f], fe = A.off[f + 1];
        if (fe == fs) {
          f++;
          continue;
        }
        // the lane owns every match start in [item start, b): pieces may span chunks
        const uint64_t se = min(b, fe);
        if (KW || group_gated(A.kw + (size_t)f * A.kw_words, A.gmask, A.kw_words, A.galways)) {
          L.file = f;
          L.fs = fs;
          L.piece(fe, a, se);
        }
        a = se;
        f++;
      }
    }
  }
}

// ---------------------------------------------------------------- host side
struct DeviceDFA {
  DevDFA dev{};
  std::vector<void*> allocs;
};

template <class T>
static int upload_vec(const std::vector<T>& v, const T** dst, std::vector<void*>* allocs) {
  void* p = nullptr;
  size_t bytes = std::max<size_t>(v.size() * sizeof(T), 16);
  HIP_TRY(hipMalloc(&p, bytes));
  if (!v.empty()) HIP_TRY(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  allocs->push_back(p);
  *dst = (const T*)p;
  return TSG_OK;
}

static uint32_t align16(uint32_t x) { return (x + 15) & ~15u; }

static int make_device_dfa(const DFA& d, const std::vector<uint32_t>& rules, uint32_t kw_words,
                           bool kw_mode, DeviceDFA* out) {
  if (d.nstates >= 0x8000) return fail(TSG_ERR_INTERNAL, "DFA too large for u16 tables");
  const size_t nc = d.nclasses;
  std::vector<uint16_t> tab((size_t)d.nstates * nc), acc(tab.size()), accs(d.nstates, 0);
  bool state_acc = true;
  for (int s = 0; s < d.nstates; s++) {
    uint32_t a0 = d.acc[(size_t)s * nc];
    for (size_t c = 0; c < nc; c++) {
      size_t i = (size_t)s * nc + c;
      if (d.acc[i] > 0xFFFF) return fail(TSG_ERR_INTERNAL, "too many accept masks");
      tab[i] = (uint16_t)(d.next[i] | (d.acc[i] ? 0x8000u : 0u));
      acc[i] = (uint16_t)d.acc[i];
      if (d.acc[i] != a0) state_acc = false;
    }
    accs[s] = (uint16_t)a0;
  }
  std::vector<uint16_t> eot(d.nstates), ni(d.nstates);
  for (int s = 0; s < d.nstates; s++) {
    eot[s] = (uint16_t)d.eot_acc[s];
    ni[s] = (uint16_t)d.to_noinject[s];
  }
  std::vector<uint8_t> dead(d.dead.begin(), d.dead.end());
  std::vector<uint64_t> masks;
  for (const auto& m : d.masks) masks.insert(masks.end(), m.begin(), m.end());
  std::vector<uint8_t> cls(d.cls, d.cls + 256);
  DevDFA& v = out->dev;
  int rc;
  if ((rc = upload_vec(tab, &v.tab, &out->allocs))) return rc;
  if ((rc = upload_vec(acc, &v.acc, &out->allocs))) return rc;
  if ((rc = upload_vec(accs, &v.acc_state, &out->allocs))) return rc;
  if ((rc = upload_vec(eot, &v.eot, &out->allocs))) return rc;
  if ((rc = upload_vec(ni, &v.to_ni, &out->allocs))) return rc;
  if ((rc = upload_vec(dead, &v.dead, &out->allocs))) return rc;
  if ((rc = upload_vec(masks, &v.masks, &out->allocs))) return rc;
  if ((rc = upload_vec(cls, &v.cls, &out->allocs))) return rc;
  if ((rc = upload_vec(rules, &v.rules, &out->allocs))) return rc;
  v.nc = (uint32_t)nc;
  v.ns = (uint32_t)d.nstates;
  v.mw = (uint32_t)d.mask_words;
  v.nmasks = (uint32_t)d.masks.size();
  v.ext = d.max_len > 1 ? (uint32_t)(d.max_len - 1) : 0;
  for (int k = 0; k < 4; k++) v.start[k] = d.start[k];
  // LDS layout
  uint32_t o = align16((uint32_t)(tab.size() * 2));
  v.o_cls = o;
  o += 256;
  v.o_accs = o;
  v.o_masks = o;
  v.state_acc = 0;
  const uint32_t acc_bytes = align16(d.nstates * 2) + align16((uint32_t)masks.size() * 8);
  if (state_acc && o + acc_bytes + 16 * 1024 <= 150 * 1024) {
    v.state_acc = 1;
    v.o_masks = o + align16(d.nstates * 2);
    o += acc_bytes;
  }
  v.o_kwacc = o;
  if (kw_mode) o += kw_words * 256 * 4;
  v.lds_bytes = o + 16;
  return TSG_OK;
}

}  // namespace tsg

using namespace tsg;

struct tsg_ctx {
  int device = 0;
  const tsg_ruleset* rs = nullptr;
  tsg_ctx_options opt{};
  hipStream_t stream = nullptr;
  hipEvent_t ev[8];
  DeviceDFA kw;
  std::vector<DeviceDFA> groups;
  uint32_t* d_gmask = nullptr;    // [G * W]
  uint32_t* d_galways = nullptr;  // [G]
  // batch
  const uint8_t* h_data = nullptr;
  const uint64_t* h_off = nullptr;
  const char* h_paths = nullptr;
  const uint64_t* h_poff = nullptr;
  uint32_t nfiles = 0;
  uint64_t total = 0;
  uint8_t* d_data = nullptr;
  size_t d_data_cap = 0;
  uint64_t* d_off = nullptr;
  size_t d_off_cap = 0;
  uint32_t* d_chunk_file = nullptr;
  size_t d_chunk_cap = 0;
  uint32_t* d_kw = nullptr;
  size_t d_kw_cap = 0;
  uint32_t* d_ovf = nullptr;
  size_t d_ovf_cap = 0;
  DevCand* d_cand = nullptr;
  uint32_t* d_count = nullptr;      // [0] candidates
  unsigned long long* d_gbytes = nullptr;  // [G]
  uint32_t* d_gfiles = nullptr;     // [G]
  uint32_t* d_list_groups = nullptr;
  uint64_t* d_item_base = nullptr;
  uint32_t* d_item_count = nullptr;
  uint2* d_items = nullptr;
  size_t d_items_cap = 0;
  // host mirrors
  KernelOutput ko;
  uint32_t* h_count = nullptr;
  std::vector<unsigned long long> h_gbytes;
  std::vector<uint32_t> h_gfiles;
  tsg_stats stats{};
  int grid = 0;
  bool uploaded = false;

  ~tsg_ctx() {
    hipSetDevice(device);
    for (auto* p : kw.allocs) hipFree(p);
    for (auto& g : groups)
      for (auto* p : g.allocs) hipFree(p);
    hipFree(d_gmask);
    hipFree(d_galways);
    hipFree(d_data);
    hipFree(d_off);
    hipFree(d_chunk_file);
    hipFree(d_kw);
    hipFree(d_ovf);
    hipFree(d_cand);
    hipFree(d_count);
    hipFree(d_gbytes);
    hipFree(d_gfiles);
    hipFree(d_list_groups);
    hipFree(d_item_base);
    hipFree(d_item_count);
    hipFree(d_items);
    if (h_count) hipHostFree(h_count);
    for (auto& e : ev)
      if (e) hipEventDestroy(e);
    if (stream) hipStreamDestroy(stream);
  }
};

template <class T>
static int ensure(T** p, size_t* cap, size_t n) {
  if (*cap >= n && *p) return TSG_OK;
  if (*p) HIP_TRY(hipFree(*p));
  *p = nullptr;
  size_t alloc = std::max<size_t>(n, 16);
  HIP_TRY(hipMalloc((void**)p, alloc * sizeof(T)));
  *cap = alloc;
  return TSG_OK;
}

template <bool KW, bool LIST>
static int launch_scan(tsg_ctx* c, const DevDFA& d, ScanArgsDev A) {
  if (A.nitems == 0) return TSG_OK;
  if (d.lds_bytes > 160 * 1024) return fail(TSG_ERR_INTERNAL, "DFA tables exceed LDS");
  auto fn = dfa_scan_kernel<KW, LIST>;
  if (d.lds_bytes > 64 * 1024)
    HIP_TRY(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)d.lds_bytes));
  const int block = 256;
  uint64_t need = (A.nitems + block - 1) / block;
  int grid = (int)std::min<uint64_t>(need, (uint64_t)c->grid);
  hipLaunchKernelGGL(fn, dim3(grid), dim3(block), d.lds_bytes, c->stream, d, A);
  HIP_TRY(hipGetLastError());
  return TSG_OK;
}

extern "C" {

int tsg_ctx_create(int device, const tsg_ruleset* rs, const tsg_ctx_options* opt, tsg_ctx** out) {
  if (!rs || !out) return fail(TSG_ERR_ARG, "bad argument");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(TSG_ERR_GPU, "no such HIP device");
  HIP_TRY(hipSetDevice(device));
  auto c = std::make_unique<tsg_ctx>();
  std::memset(c->ev, 0, sizeof(c->ev));
  c->device = device;
  c->rs = rs;
  if (opt) c->opt = *opt;
  if (c->opt.chunk_bytes == 0) c->opt.chunk_bytes = 256;
  if (c->opt.chunk_bytes % 16) return fail(TSG_ERR_ARG, "chunk_bytes must be a multiple of 16");
  if (c->opt.ext_cap == 0) c->opt.ext_cap = 1u << 16;
  if (c->opt.cand_capacity == 0) c->opt.cand_capacity = 1u << 22;
  HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  for (auto& e : c->ev) HIP_TRY(hipEventCreate(&e));
  const Plan& p = *rs->plan;
  const uint32_t W = (uint32_t)p.kw_words;
  int rc;
  if ((rc = make_device_dfa(*p.kw_dfa, {}, W, true, &c->kw))) return rc;
  std::vector<uint32_t> gmask, galways;
  for (const auto& g : p.groups) {
    DeviceDFA dd;
    if ((rc = make_device_dfa(*g.dfa, g.rules, W, false, &dd))) return rc;
    c->groups.push_back(std::move(dd));
    gmask.insert(gmask.end(), g.kwmask.begin(), g.kwmask.end());
    galways.push_back(g.always ? 1 : 0);
  }
  const size_t G = p.groups.size();
  std::vector<void*> tmp;
  const uint32_t* cg = nullptr;
  if ((rc = upload_vec(gmask, &cg, &tmp))) return rc;
  c->d_gmask = (uint32_t*)cg;
  if ((rc = upload_vec(galways, &cg, &tmp))) return rc;
  c->d_galways = (uint32_t*)cg;
  HIP_TRY(hipMalloc((void**)&c->d_cand, sizeof(DevCand) * c->opt.cand_capacity));
  HIP_TRY(hipMalloc((void**)&c->d_count, sizeof(uint32_t) * 4));
  HIP_TRY(hipMalloc((void**)&c->d_gbytes, sizeof(unsigned long long) * (G + 1)));
  HIP_TRY(hipMalloc((void**)&c->d_gfiles, sizeof(uint32_t) * (G + 1)));
  HIP_TRY(hipMalloc((void**)&c->d_list_groups, sizeof(uint32_t) * (G + 1)));
  HIP_TRY(hipMalloc((void**)&c->d_item_base, sizeof(uint64_t) * (G + 1)));
  HIP_TRY(hipMalloc((void**)&c->d_item_count, sizeof(uint32_t) * (G + 1)));
  HIP_TRY(hipHostMalloc((void**)&c->h_count, sizeof(uint32_t) * 4, hipHostMallocDefault));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  c->grid = prop.multiProcessorCount * 8;
  *out = c.release();
  return TSG_OK;
}

void tsg_ctx_destroy(tsg_ctx* ctx) { delete ctx; }

int tsg_batch_upload(tsg_ctx* c, const uint8_t* data, const uint64_t* offsets, uint32_t nfiles,
                     const char* paths, const uint64_t* path_offsets) {
  if (!c || !offsets || !path_offsets) return fail(TSG_ERR_ARG, "bad argument");
  HIP_TRY(hipSetDevice(c->device));
  const uint64_t total = offsets[nfiles];
  if (offsets[0] != 0) return fail(TSG_ERR_ARG, "offsets[0] must be 0");
  for (uint32_t i = 0; i < nfiles; i++)
    if (offsets[i + 1] < offsets[i]) return fail(TSG_ERR_ARG, "offsets must be non-decreasing");
  const uint32_t chunk = c->opt.chunk_bytes;
  if (total / chunk >= (1ull << 32) - 2) return fail(TSG_ERR_ARG, "batch too large for u32 chunk ids");
  int rc;
  if ((rc = ensure(&c->d_data, &c->d_data_cap, (size_t)total + 64))) return rc;
  if ((rc = ensure(&c->d_off, &c->d_off_cap, (size_t)nfiles + 1))) return rc;
  const uint64_t nchunks = (total + chunk - 1) / chunk;
  if ((rc = ensure(&c->d_chunk_file, &c->d_chunk_cap, (size_t)nchunks + 1))) return rc;
  const int W = c->rs->plan->kw_words;
  if ((rc = ensure(&c->d_kw, &c->d_kw_cap, (size_t)nfiles * W + 1))) return rc;
  if ((rc = ensure(&c->d_ovf, &c->d_ovf_cap, (size_t)nfiles + 1))) return rc;
  if (total) HIP_TRY(hipMemcpyAsync(c->d_data, data, total, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemsetAsync(c->d_data + total, 0, 64, c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_off, offsets, sizeof(uint64_t) * (nfiles + 1), hipMemcpyHostToDevice, c->stream));
  if (nfiles) {
    chunk_file_kernel<<<(nfiles + 255) / 256, 256, 0, c->stream>>>(c->d_off, nfiles, chunk, c->d_chunk_file);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->h_data = data;
  c->h_off = offsets;
  c->h_paths = paths;
  c->h_poff = path_offsets;
  c->nfiles = nfiles;
  c->total = total;
  c->uploaded = true;
  return TSG_OK;
}

int tsg_batch_kernels(tsg_ctx* c) {
  if (!c || !c->uploaded) return fail(TSG_ERR_ARG, "no batch uploaded");
  HIP_TRY(hipSetDevice(c->device));
  const Plan& p = *c->rs->plan;
  const uint32_t W = (uint32_t)p.kw_words;
  const uint32_t chunk = c->opt.chunk_bytes;
  const uint64_t nchunks = (c->total + chunk - 1) / chunk;
  const uint32_t F = c->nfiles;
  const uint32_t G = (uint32_t)c->groups.size();
  hipStream_t st = c->stream;
  HIP_TRY(hipEventRecord(c->ev[0], st));
  if (F) {
    HIP_TRY(hipMemsetAsync(c->d_kw, 0, sizeof(uint32_t) * (size_t)F * W, st));
    HIP_TRY(hipMemsetAsync(c->d_ovf, 0, sizeof(uint32_t) * F, st));
  }
  HIP_TRY(hipMemsetAsync(c->d_count, 0, sizeof(uint32_t) * 4, st));
  HIP_TRY(hipMemsetAsync(c->d_gbytes, 0, sizeof(unsigned long long) * (G + 1), st));
  HIP_TRY(hipMemsetAsync(c->d_gfiles, 0, sizeof(uint32_t) * (G + 1), st));
  HIP_TRY(hipMemsetAsync(c->d_item_count, 0, sizeof(uint32_t) * (G + 1), st));
  HIP_TRY(hipEventRecord(c->ev[1], st));

  ScanArgsDev A{};
  A.data = c->d_data;
  A.off = c->d_off;
  A.chunk_file = c->d_chunk_file;
  A.total = c->total;
  A.chunk = chunk;
  A.ext_cap = c->opt.ext_cap;
  A.kw = c->d_kw;
  A.kw_words = W;
  A.cand = c->d_cand;
  A.cand_count = c->d_count;
  A.cand_cap = c->opt.cand_capacity;
  A.ovf = c->d_ovf;
  int rc;
  // ---- K1
  A.nitems = (nchunks + kStreams - 1) / kStreams;
  if ((rc = launch_scan<true, false>(c, c->kw.dev, A))) return rc;
  HIP_TRY(hipEventRecord(c->ev[2], st));
  // ---- gate: per-group gated bytes / files
  if (F && G) {
    size_t lds = G * (sizeof(unsigned long long) + sizeof(uint32_t)) + 16;
    gate_count_kernel<<<(F + 255) / 256, 256, lds, st>>>(c->d_off, F, c->d_kw, W, c->d_gmask, c->d_galways,
                                                           G, c->d_gbytes, c->d_gfiles);
    HIP_TRY(hipGetLastError());
  }
  c->h_gbytes.assign(G, 0);
  c->h_gfiles.assign(G, 0);
  if (G) {
    HIP_TRY(hipMemcpyAsync(c->h_gbytes.data(), c->d_gbytes, sizeof(unsigned long long) * G, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(c->h_gfiles.data(), c->d_gfiles, sizeof(uint32_t) * G, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  // DENSE when a group is gated on a large share of the batch, LIST otherwise
  std::vector<uint32_t> list_groups, dense_groups;
  std::vector<uint64_t> base;
  uint64_t nitems_total = 0, k2_bytes = 0;
  for (uint32_t g = 0; g < G; g++) {
    k2_bytes += c->h_gbytes[g];
    if (c->h_gbytes[g] == 0) continue;
    if (c->h_gbytes[g] * 4 > c->total) {
      dense_groups.push_back(g);
    } else {
      list_groups.push_back(g);
      base.push_back(nitems_total);
      nitems_total += c->h_gbytes[g] / chunk + 2ull * c->h_gfiles[g];
    }
  }
  if (!list_groups.empty()) {
    if ((rc = ensure(&c->d_items, &c->d_items_cap, (size_t)nitems_total))) return rc;
    HIP_TRY(hipMemcpyAsync(c->d_list_groups, list_groups.data(), sizeof(uint32_t) * list_groups.size(),
                           hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(c->d_item_base, base.data(), sizeof(uint64_t) * base.size(), hipMemcpyHostToDevice, st));
    gate_list_kernel<<<(F + 255) / 256, 256, 0, st>>>(c->d_off, F, c->d_kw, W, c->d_gmask, c->d_galways,
                                                       c->d_list_groups, (uint32_t)list_groups.size(),
                                                       c->d_item_base, c->d_item_count, c->d_items, chunk);
    HIP_TRY(hipGetLastError());
  }
  std::vector<uint32_t> item_count(list_groups.size(), 0);
  if (!list_groups.empty()) {
    HIP_TRY(hipMemcpyAsync(item_count.data(), c->d_item_count, sizeof(uint32_t) * list_groups.size(),
                           hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  HIP_TRY(hipEventRecord(c->ev[3], st));
  // ---- K2
  for (uint32_t g : dense_groups) {
    ScanArgsDev B = A;
    B.nitems = (nchunks + kStreams - 1) / kStreams;
    B.gmask = c->d_gmask + (size_t)g * W;
    B.galways = p.groups[g].always ? 1 : 0;
    if ((rc = launch_scan<false, false>(c, c->groups[g].dev, B))) return rc;
  }
  for (size_t j = 0; j < list_groups.size(); j++) {
    ScanArgsDev B = A;
    B.nitems = item_count[j];
    B.items = c->d_items + base[j];
    if ((rc = launch_scan<false, true>(c, c->groups[list_groups[j]].dev, B))) return rc;
  }
  HIP_TRY(hipEventRecord(c->ev[4], st));
  HIP_TRY(hipMemcpyAsync(c->h_count, c->d_count, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  uint32_t n = std::min(*c->h_count, c->opt.cand_capacity);
  c->ko.cand.resize(n);
  c->ko.kw.resize((size_t)F * W);
  std::vector<uint32_t> ovf(F);
  if (n) HIP_TRY(hipMemcpyAsync(c->ko.cand.data(), c->d_cand, sizeof(DevCand) * n, hipMemcpyDeviceToHost, st));
  if (F) {
    HIP_TRY(hipMemcpyAsync(c->ko.kw.data(), c->d_kw, sizeof(uint32_t) * (size_t)F * W, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(ovf.data(), c->d_ovf, sizeof(uint32_t) * F, hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(hipEventRecord(c->ev[5], st));
  HIP_TRY(hipStreamSynchronize(st));
  c->ko.overflow.assign(F, 0);
  for (uint32_t i = 0; i < F; i++) c->ko.overflow[i] = ovf[i] ? 1 : 0;
  float t[5] = {0, 0, 0, 0, 0};
  for (int k = 0; k < 5; k++) HIP_TRY(hipEventElapsedTime(&t[k], c->ev[k], c->ev[k + 1]));
  c->stats.k1_ms = t[1];
  c->stats.k2_ms = t[3];
  c->stats.aux_ms = t[0] + t[2] + t[4];
  c->stats.bytes = c->total;
  c->stats.k2_bytes = k2_bytes;
  c->stats.candidates = *c->h_count;
  c->stats.overflow = *c->h_count > c->opt.cand_capacity ? 1 : 0;
  c->stats.k2_launches = (uint32_t)(dense_groups.size() + list_groups.size());
  return TSG_OK;
}

int tsg_batch_scan(tsg_ctx* c, tsg_result** out) {
  if (!c || !out) return fail(TSG_ERR_ARG, "bad argument");
  int rc = tsg_batch_kernels(c);
  if (rc) return rc;
  try {
    auto t0 = std::chrono::steady_clock::now();
    BatchView b{c->h_data, c->h_off, c->nfiles, c->h_paths, c->h_poff};
    std::vector<FileResult> res;
    int nt = c->opt.host_threads > 0 ? c->opt.host_threads : 16;
    resolve_batch(c->rs->rs, *c->rs->plan, b, c->ko, nt, &res);
    auto r = std::make_unique<tsg_result>();
    serialize_results(res, &r->buf);
    auto t1 = std::chrono::steady_clock::now();
    c->stats.resolve_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    uint64_t nres = 0;
    for (const auto& fr : res) nres += fr.status == kHasFindings;
    c->stats.files_resolved = nres;
    *out = r.release();
    return TSG_OK;
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& ex) {
    return fail(TSG_ERR_INTERNAL, ex.what());
  }
}

int tsg_scan_batch(tsg_ctx* c, const uint8_t* data, const uint64_t* offsets, uint32_t nfiles,
                   const char* paths, const uint64_t* path_offsets, tsg_result** out) {
  int rc = tsg_batch_upload(c, data, offsets, nfiles, paths, path_offsets);
  if (rc) return rc;
  return tsg_batch_scan(c, out);
}

int tsg_ctx_get_stats(const tsg_ctx* c, tsg_stats* out) {
  if (!c || !out) return fail(TSG_ERR_ARG, "bad argument");
  *out = c->stats;
  return TSG_OK;
}

}  // extern "C"
