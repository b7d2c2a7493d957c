// MI355X (gfx950) device path of the secret engine: K1 keyword automaton and K2
// rule-group DFAs over a device-resident batch of file blobs.
//
// Work decomposition (one lane = one chunk of `chunk` bytes of the concatenated
// batch stream; files are packed back to back, a chunk may hold pieces of several
// files).  For each file piece [a, b) a lane runs the DFA in inject mode (a thread
// starts at every byte) and, if the file continues past b, follows the threads that
// started inside its piece in noinject mode until they are all dead.  Every match
// start is owned by exactly one lane, so no lane needs state from its neighbour and
// the reported end offsets are exact (dfa.hpp).  Accepts are rare events:
//   K1: keyword bits, OR-ed per lane in LDS and flushed with one atomicOr per word
//       per file piece;
//   K2: candidate records {file, rule, end} appended with an atomic counter.
// Tables: the DFA transition table (u16: next state | accept bit) and the byte-class
// map live in LDS; accept masks / EOT / mode tables stay in global memory (L2) since
// they are only read on accept or after a chunk end.
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
  const uint16_t* tab;     // [ns * nc] next | 0x8000 if the transition accepts
  const uint16_t* acc;     // [ns * nc] accept-mask index
  const uint16_t* eot;     // [ns] accept-mask index at end of text
  const uint16_t* to_ni;   // [ns] noinject twin
  const uint8_t* dead;     // [ns]
  const uint64_t* masks;   // [nmasks * mw]
  const uint8_t* cls;      // [256]
  const uint32_t* rules;   // K2: group-local id -> global rule
  const uint32_t* kwmask;  // K2: [kw_words]
  uint32_t nc, ns, mw, always;
  uint32_t ext;  // K1 overlap: longest keyword - 1
  uint32_t start[4];
};

struct DevCand {
  uint32_t file, rule, end;
};

// ---------------------------------------------------------------- kernels
__global__ void chunk_file_kernel(const uint64_t* __restrict__ off, uint32_t nfiles, uint32_t chunk,
                                  uint32_t* __restrict__ chunk_file) {
  uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= nfiles) return;
  uint64_t fs = off[f], fe = off[f + 1];
  if (fe == fs) return;
  // chunks whose first byte lies in [fs, fe)
  uint64_t c0 = (fs + chunk - 1) / chunk, c1 = (fe + chunk - 1) / chunk;
  for (uint64_t c = c0; c < c1; c++) chunk_file[c] = f;
}

__device__ __forceinline__ uint32_t ctx_of(uint8_t c) {
  if (c == '\n') return 1;
  if ((c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_') return 2;
  return 3;
}

template <bool KW>
struct Sink {
  // KW: per-lane keyword accumulator in LDS (kw_words x blockDim), flushed per file piece
  uint32_t* lds_acc;
  uint32_t kw_words;
  uint32_t* kw;
  // K2
  DevCand* cand;
  uint32_t* cand_count;
  uint32_t cand_cap;
  uint32_t* ovf;
  uint32_t file;

  __device__ __forceinline__ void accept(const DevDFA& d, uint32_t mi, uint32_t pos) {
    const uint64_t* m = d.masks + (size_t)mi * d.mw;
    if (KW) {
      for (uint32_t w = 0; w < d.mw; w++) {
        uint64_t v = m[w];
        if (2 * w < kw_words) lds_acc[(2 * w) * blockDim.x + threadIdx.x] |= (uint32_t)v;
        if (2 * w + 1 < kw_words) lds_acc[(2 * w + 1) * blockDim.x + threadIdx.x] |= (uint32_t)(v >> 32);
      }
    } else {
      uint64_t v = m[0];
      while (v) {
        uint32_t k = __builtin_ctzll(v);
        v &= v - 1;
        uint32_t idx = atomicAdd(cand_count, 1u);
        if (idx < cand_cap) {
          cand[idx].file = file;
          cand[idx].rule = d.rules[k];
          cand[idx].end = pos;
        } else {
          ovf[file] = 1;
        }
      }
    }
  }

  __device__ __forceinline__ void begin() {
    if (KW)
      for (uint32_t w = 0; w < kw_words; w++) lds_acc[w * blockDim.x + threadIdx.x] = 0;
  }
  __device__ __forceinline__ void end() {
    if (KW)
      for (uint32_t w = 0; w < kw_words; w++) {
        uint32_t v = lds_acc[w * blockDim.x + threadIdx.x];
        if (v) atomicOr(&kw[(size_t)file * kw_words + w], v);
      }
  }
};

template <bool KW>
__global__ void __launch_bounds__(256) dfa_scan_kernel(
    DevDFA d, const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ chunk_file, uint64_t total, uint64_t nchunks, uint32_t chunk,
    uint32_t ext_cap, uint32_t* __restrict__ kw, uint32_t kw_words, DevCand* __restrict__ cand,
    uint32_t* __restrict__ cand_count, uint32_t cand_cap, uint32_t* __restrict__ ovf) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t tab_entries = d.ns * d.nc;
  uint16_t* s_tab = (uint16_t*)smem;
  uint8_t* s_cls = smem + ((tab_entries * 2 + 15) & ~15u);
  uint32_t* s_acc = (uint32_t*)(s_cls + 256);
  for (uint32_t i = threadIdx.x; i < tab_entries; i += blockDim.x) s_tab[i] = d.tab[i];
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) s_cls[i] = d.cls[i];
  __syncthreads();

  Sink<KW> sink;
  sink.lds_acc = s_acc;
  sink.kw_words = kw_words;
  sink.kw = kw;
  sink.cand = cand;
  sink.cand_count = cand_count;
  sink.cand_cap = cand_cap;
  sink.ovf = ovf;
  const uint32_t nc = d.nc;

  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nchunks;
       c += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t a = c * chunk;
    const uint64_t b = min(a + chunk, total);
    uint32_t f = chunk_file[c];
    while (a < b) {
      const uint64_t fs = off[f], fe = off[f + 1];
      if (fe == fs) {
        f++;
        continue;
      }
      const uint64_t se = min(b, fe);
      bool gated = true;
      if (!KW) {
        gated = d.always != 0;
        for (uint32_t w = 0; w < kw_words && !gated; w++) gated = (kw[(size_t)f * kw_words + w] & d.kwmask[w]) != 0;
      }
      if (gated) {
        sink.file = f;
        sink.begin();
        uint32_t s = (a == fs) ? d.start[0] : d.start[ctx_of(data[a - 1])];
        uint64_t p = a;
#define TSG_STEP(BYTE, POS)                                              \
  {                                                                      \
    const uint32_t cl_ = s_cls[(BYTE)];                                  \
    const uint32_t ix_ = s * nc + cl_;                                   \
    const uint32_t e_ = s_tab[ix_];                                      \
    if (__builtin_expect(e_ & 0x8000u, 0)) sink.accept(d, d.acc[ix_], (uint32_t)((POS) - fs)); \
    s = e_ & 0x7FFFu;                                                    \
  }
        // K1: keywords are bounded -> overlap of ext bytes in inject mode instead of noinject
        const uint64_t le = KW ? min(fe, se + d.ext) : se;
        while (p < le && (p & 15)) {
          TSG_STEP(data[p], p);
          p++;
        }
        while (p + 16 <= le) {
          const uint4 v = *(const uint4*)(data + p);
          const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int k = 0; k < 16; k++) TSG_STEP((wv[k >> 2] >> ((k & 3) * 8)) & 0xFF, p + k);
          p += 16;
        }
        while (p < le) {
          TSG_STEP(data[p], p);
          p++;
        }
        if (le >= fe) {
          const uint32_t m = d.eot[s];
          if (m) sink.accept(d, m, (uint32_t)(fe - fs));
        } else if (!KW) {
          // follow the threads that started in [a, se) past the chunk end
          s = d.to_ni[s];
          uint64_t q = se;
          bool over = false;
          while (q < fe && !d.dead[s]) {
            if (q - se >= ext_cap) {
              over = true;
              break;
            }
            TSG_STEP(data[q], q);
            q++;
          }
          if (over) {
            ovf[f] = 1;
          } else if (q == fe && !d.dead[s]) {
            const uint32_t m = d.eot[s];
            if (m) sink.accept(d, m, (uint32_t)(fe - fs));
          }
        }
#undef TSG_STEP
        sink.end();
      }
      a = se;
      f++;
    }
  }
}

// ---------------------------------------------------------------- host side
struct DeviceDFA {
  DevDFA dev{};
  std::vector<void*> allocs;
  uint32_t lds_table_bytes = 0;
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

static int make_device_dfa(const DFA& d, const std::vector<uint32_t>& rules,
                           const std::vector<uint32_t>& kwmask, bool always, DeviceDFA* out) {
  if (d.nstates >= 0x8000) return fail(TSG_ERR_INTERNAL, "DFA too large for u16 tables");
  std::vector<uint16_t> tab((size_t)d.nstates * d.nclasses), acc(tab.size());
  for (size_t i = 0; i < tab.size(); i++) {
    if (d.acc[i] > 0xFFFF) return fail(TSG_ERR_INTERNAL, "too many accept masks");
    tab[i] = (uint16_t)(d.next[i] | (d.acc[i] ? 0x8000u : 0u));
    acc[i] = (uint16_t)d.acc[i];
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
  if ((rc = upload_vec(eot, &v.eot, &out->allocs))) return rc;
  if ((rc = upload_vec(ni, &v.to_ni, &out->allocs))) return rc;
  if ((rc = upload_vec(dead, &v.dead, &out->allocs))) return rc;
  if ((rc = upload_vec(masks, &v.masks, &out->allocs))) return rc;
  if ((rc = upload_vec(cls, &v.cls, &out->allocs))) return rc;
  if ((rc = upload_vec(rules, &v.rules, &out->allocs))) return rc;
  if ((rc = upload_vec(kwmask, &v.kwmask, &out->allocs))) return rc;
  v.nc = (uint32_t)d.nclasses;
  v.ns = (uint32_t)d.nstates;
  v.mw = (uint32_t)d.mask_words;
  v.always = always ? 1 : 0;
  v.ext = d.max_len > 1 ? (uint32_t)(d.max_len - 1) : 0;
  for (int k = 0; k < 4; k++) v.start[k] = d.start[k];
  out->lds_table_bytes = (uint32_t)(((tab.size() * 2 + 15) & ~(size_t)15) + 256);
  return TSG_OK;
}

}  // namespace tsg

using namespace tsg;

struct tsg_ctx {
  int device = 0;
  const tsg_ruleset* rs = nullptr;
  tsg_ctx_options opt{};
  hipStream_t stream = nullptr;
  hipEvent_t ev[64];
  DeviceDFA kw;
  std::vector<DeviceDFA> groups;
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
  uint32_t* d_count = nullptr;
  // host mirrors
  KernelOutput ko;
  uint32_t* h_count = nullptr;
  tsg_stats stats{};
  int grid = 0;
  bool uploaded = false;

  ~tsg_ctx() {
    hipSetDevice(device);
    for (auto* p : kw.allocs) hipFree(p);
    for (auto& g : groups)
      for (auto* p : g.allocs) hipFree(p);
    hipFree(d_data);
    hipFree(d_off);
    hipFree(d_chunk_file);
    hipFree(d_kw);
    hipFree(d_ovf);
    hipFree(d_cand);
    hipFree(d_count);
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
  int rc;
  if ((rc = make_device_dfa(*p.kw_dfa, {}, {}, true, &c->kw))) return rc;
  for (const auto& g : p.groups) {
    DeviceDFA dd;
    if ((rc = make_device_dfa(*g.dfa, g.rules, g.kwmask, g.always, &dd))) return rc;
    c->groups.push_back(std::move(dd));
  }
  HIP_TRY(hipMalloc((void**)&c->d_cand, sizeof(DevCand) * c->opt.cand_capacity));
  HIP_TRY(hipMalloc((void**)&c->d_count, sizeof(uint32_t) * 4));
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
  if (total >= (1ull << 40)) return fail(TSG_ERR_ARG, "batch too large");
  int rc;
  if ((rc = ensure(&c->d_data, &c->d_data_cap, (size_t)total + 64))) return rc;
  if ((rc = ensure(&c->d_off, &c->d_off_cap, (size_t)nfiles + 1))) return rc;
  const uint32_t chunk = c->opt.chunk_bytes;
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
  hipStream_t st = c->stream;
  HIP_TRY(hipEventRecord(c->ev[0], st));
  if (F) {
    HIP_TRY(hipMemsetAsync(c->d_kw, 0, sizeof(uint32_t) * (size_t)F * W, st));
    HIP_TRY(hipMemsetAsync(c->d_ovf, 0, sizeof(uint32_t) * F, st));
  }
  HIP_TRY(hipMemsetAsync(c->d_count, 0, sizeof(uint32_t) * 4, st));
  HIP_TRY(hipEventRecord(c->ev[1], st));
  const int block = 256;
  uint64_t need_blocks = (nchunks + block - 1) / block;
  int grid = (int)std::min<uint64_t>(need_blocks ? need_blocks : 1, (uint64_t)c->grid);
  if (nchunks) {
    size_t lds = c->kw.lds_table_bytes + (size_t)W * block * 4;
    if (lds > 160 * 1024) return fail(TSG_ERR_INTERNAL, "keyword automaton exceeds LDS");
    HIP_TRY(hipFuncSetAttribute((const void*)dfa_scan_kernel<true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(dfa_scan_kernel<true>, dim3(grid), dim3(block), lds, st, c->kw.dev, c->d_data,
                       c->d_off, c->d_chunk_file, c->total, nchunks, chunk, c->opt.ext_cap, c->d_kw, W,
                       c->d_cand, c->d_count, c->opt.cand_capacity, c->d_ovf);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipEventRecord(c->ev[2], st));
  if (nchunks) {
    for (auto& g : c->groups) {
      size_t lds = g.lds_table_bytes + 16;
      if (lds > 64 * 1024)
        HIP_TRY(hipFuncSetAttribute((const void*)dfa_scan_kernel<false>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      hipLaunchKernelGGL(dfa_scan_kernel<false>, dim3(grid), dim3(block), lds, st, g.dev, c->d_data,
                         c->d_off, c->d_chunk_file, c->total, nchunks, chunk, c->opt.ext_cap, c->d_kw,
                         W, c->d_cand, c->d_count, c->opt.cand_capacity, c->d_ovf);
      HIP_TRY(hipGetLastError());
    }
  }
  HIP_TRY(hipEventRecord(c->ev[3], st));
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
  HIP_TRY(hipEventRecord(c->ev[4], st));
  HIP_TRY(hipStreamSynchronize(st));
  c->ko.overflow.assign(F, 0);
  for (uint32_t i = 0; i < F; i++) c->ko.overflow[i] = ovf[i] ? 1 : 0;
  float k1 = 0, k2 = 0, a0 = 0, a1 = 0;
  HIP_TRY(hipEventElapsedTime(&a0, c->ev[0], c->ev[1]));
  HIP_TRY(hipEventElapsedTime(&k1, c->ev[1], c->ev[2]));
  HIP_TRY(hipEventElapsedTime(&k2, c->ev[2], c->ev[3]));
  HIP_TRY(hipEventElapsedTime(&a1, c->ev[3], c->ev[4]));
  c->stats.k1_ms = k1;
  c->stats.k2_ms = k2;
  c->stats.aux_ms = a0 + a1;
  c->stats.bytes = c->total;
  c->stats.candidates = *c->h_count;
  c->stats.overflow = *c->h_count > c->opt.cand_capacity ? 1 : 0;
  c->stats.k2_launches = (uint32_t)c->groups.size();
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
