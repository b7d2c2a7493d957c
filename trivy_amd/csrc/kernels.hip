// MI355X (gfx950) kernels of the secret engine over a batch of file blobs packed back to
// back in one HBM stream (chunk c = bytes [c*C, (c+1)*C)), and the host code that builds
// their tables and enqueues one batch on a lane (device.hpp).
//
//   K1   one dense pass over every byte: the Aho-Corasick automaton of the rule set's
//        literals (keywords of Rule.MatchKeywords + anchor literals) stepped from LDS,
//        fused with two saturating run counters (class U = token bytes, class D = digits).
//        Outputs per-file keyword bits and per-chunk event bits (plan.hpp kEv*).  The
//        automaton runs over the batch as one byte stream; each chain first replays `warm`
//        bytes before its segment, so every literal / run ending inside it is seen.
//   K1X  (large rule sets only) the literals of >= 4 bytes that do not fit K1's LDS
//        automaton: a hashed 4-gram prefilter over every byte (LDS bitmap) and an exact
//        verification of the hit positions; ORs keyword and event bits into K1's output.
//   gates per file: which K2 groups the keyword bits switch on; per chunk: which of those
//        groups have an event within `back` chunks after it -> (file, chunk) items,
//        counted; a one-block layout kernel turns the counts into item regions and K2's
//        work list on the device (no host round trip); the items are then written.
//   K2   a persistent grid over the work list: each entry is up to 512 items of one rule
//        group (two DFA chains per lane, quad-transposed loads) or a dense range of the
//        batch; the group's DFA stays staged in LDS across consecutive entries.  A lane
//        runs its chunk in inject mode and then follows the threads that started in it
//        until they die (noinject), so every match end is found by the lane that owns its
//        start.  Accepts append {file, rule, end} candidates (wave-aggregated atomics).
// Exactness: K1 keyword bits are exact (files with folding runes are flagged), events
// are a necessary condition of every match of the rule's GPU program (plan.cpp), so the
// candidate set is a superset of the exact match ends; the host resolves exactly.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "device.hpp"
#include "internal.hpp"
#include "k1f.hpp"

namespace tsg {

// how K2 covers a rule group in one batch (layout_kernel)
enum : uint8_t { kGroupNone = 0, kGroupList = 1, kGroupDense = 2, kGroupSkip = 3 };

#define HIP_TRY(x)                                                                    \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess)                                                             \
      return fail(TSG_ERR_GPU, std::string(#x) + ": " + hipGetErrorString(e_));       \
  } while (0)

constexpr int kStreams = 4;  // K2 dense: chunks per lane
#ifndef K1_CHAINS
#define K1_CHAINS 2
#endif
#ifndef K1_UNROLL
#define K1_UNROLL 8  // K1: bytes of a word unrolled (8 of 16: profiles/r04/k1g, 0.394 ms against 0.420 for 16)
#endif
constexpr int kK1Chains = K1_CHAINS;  // K1: chains per lane (independent dependent-LDS chains)
constexpr int kK1Seg = 8;     // K1: consecutive chunks per chain
// legacy K1 layout: static LDS size classes (KiB): 3, 2 or 1 blocks per CU, of 512, 512
// and 1024 threads (16 waves per CU at 4 per SIMD, whose registers bound a lane)
constexpr int kK1Lds[3] = {52, 80, 156};
constexpr int kK1BlocksPerCU[3] = {3, 2, 1};
constexpr __host__ __device__ int k1_threads(int ldsk) { return ldsk == 156 ? 1024 : 512; }
// legacy class words replicated per lane of a 32-lane half ([byte][lane & 31] words: every
// lane reads its own bank) when the automaton leaves room for it; else 256 words
constexpr uint32_t kK1RepBytes = 256 * 32 * 4;
constexpr int kBlock = 256;
constexpr int kCounts = 48;  // per-batch device counters (lane_create); 32..39: kernel clocks
constexpr int kClk = 32;     // u64 clock stamps at counts + kClk (device wall clock, see K1FArgs::clk)
constexpr int kPad = 256;     // zero bytes before and after the batch in HBM (>= K1 warm-up)
#ifndef ITEMS_BPC
#define ITEMS_BPC 8  // item passes: blocks per CU
#endif
constexpr int kMaxBack = 16;  // event windows up to this many chunks; larger -> whole file

// ---------------------------------------------------------------- device tables
// K2 tables name a state by its row (state * nc): next = tab[row + class] needs no
// multiply; the per-state tables are indexed by state_of(row).
struct DevDFA {  // K2 rule group
  const uint16_t* tab;        // [ns * nc] next row | 0x8000 if the transition accepts
  const uint16_t* acc;        // [ns * nc] accept-mask index (look-ahead DFAs)
  const uint16_t* acc_state;  // [ns] accept-mask index per state (state_acc DFAs)
  const uint16_t* eot;        // [ns] accept-mask index at end of text
  const uint16_t* to_ni;      // [ns] row of the noinject twin
  const uint8_t* dead;        // [ns] bit 0 dead, bit 1 immortal (DFA::immortal)
  const uint64_t* masks;      // [nmasks * mw]
  const uint8_t* cls;         // [256]
  const uint32_t* rules;      // group-local id -> global rule
  uint32_t nc, ns, mw, nmasks, state_acc;
  uint32_t nrules;            // rules in the group
  uint32_t inv_nc;            // ceil(2^32 / nc): state_of(row) = umulhi(row, inv_nc), exact below 2^16
  uint32_t start[4];          // start rows per previous-byte context
  uint32_t o_cls, o_dead, o_accs, o_masks, lds_bytes;  // LDS layout (stage_dfa)
};

struct DevK1 {
  // States are renumbered so that the ones whose arrival must be reported (they end a
  // literal) come last, and a state is named by its row: next = tab[row + class] needs no
  // multiply, and "arrival reports" is next >= acc_row.  Packed layout: a row is the byte
  // offset of its first entry in the LDS table, the class entry holds class * 2 + the
  // table's LDS offset; legacy: a row is the entry index (id * stride).
  const uint16_t* tab;    // [ns * stride] row of the next state
  const uint32_t* cls;    // legacy: [256] class * 2 | 0xFF00 if in run class D | 0xFFFF0000 if in U
  const uint32_t* pcls;   // packed: [256 * 2] {class * 2 + kK1PTab, in D | in U << 16}
  const uint16_t* accs;   // [ns] accept-mask index of the literals a state ends
  const uint32_t* masks;  // [nmasks * mw] keyword words (kw_words), then the event word
  uint32_t nc, ns, nmasks, mw, kw_words, start, warm, kU, kD;  // start: row; kD legacy: threshold << 8
  uint32_t acc_row;
  uint32_t row_unit;   // row of state id = id * row_unit
  uint32_t tab_words;  // dwords of the transition table (staged into LDS)
  uint32_t packed;     // layout (see above)
  uint32_t lds_class;  // legacy: index into kK1Lds
  uint32_t rep;        // legacy: class table replicated per lane (K1_REP layout)
  const uint16_t* kw_len;  // [kw_words * 32] byte length of each keyword (rare path)
  uint32_t kw_maxlen;      // longest keyword: an occurrence ending this far into a file fits
};

struct DevCand {
  uint32_t file, rule, end;
};

__device__ __forceinline__ uint32_t ctx_of(uint8_t c) {
  if (c == '\n') return 1;
  if ((c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_') return 2;
  return 3;
}

__device__ __forceinline__ uint32_t byte_of(const uint4 v, uint32_t k) {
  const uint32_t w = k < 8 ? (k < 4 ? v.x : v.y) : (k < 12 ? v.z : v.w);
  return (w >> ((k & 3) * 8)) & 0xFF;
}

// ---------------------------------------------------------------- file map
// The coarse file map: cf[k] = the file holding batch byte k << kCfShift (the last file
// starting at or before it; empty files never hold a byte).  The file holding byte p then
// lies in [cf[k], cf[k + 1]] for k = p >> kCfShift, found by a short binary search over the
// offsets.  Every caller is on a sparse path (K1 accepts, K1X hits, event chunks, dense
// entries), so one entry per 16 KiB replaces a full per-chunk map (17 MB per GiB batch).
constexpr uint32_t kCfShift = 14;

__device__ __forceinline__ uint32_t bsearch_file(const uint64_t* __restrict__ off, uint32_t lo, uint32_t hi,
                                                 uint64_t p) {
  while (hi - lo > 1) {  // invariant: off[lo] <= p, the answer in [lo, hi)
    const uint32_t mid = (lo + hi) >> 1;
    if (off[mid] <= p) lo = mid;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ uint32_t file_of(const uint32_t* __restrict__ cf, const uint64_t* __restrict__ off,
                                            uint32_t nfiles, uint64_t p) {
  const uint64_t k = p >> kCfShift;
  return bsearch_file(off, cf[k], min(nfiles, cf[k + 1] + 1), p);
}

// nbytes of src (16-B aligned, readable to the next multiple of 16: upload_vec pads) into
// LDS at dst (16-B aligned), eight 16-B loads in flight per thread: a block restages a DFA
// of up to 48 KB in two memory round trips.  (One dword per thread and iteration, each load
// waited on before the next, cost ~50 us per restage: most of a K2 list entry's time,
// profiles/r05/k2t1.)
__device__ __forceinline__ void stage16(uint8_t* dst, const void* src, uint32_t nbytes) {
  const uint32_t n = (nbytes + 15) / 16;
  const uint4* s = (const uint4*)src;
  uint4* d = (uint4*)dst;
  for (uint32_t i0 = threadIdx.x; i0 < n; i0 += 8 * blockDim.x) {
    uint4 v[8];
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) {
      const uint32_t i = i0 + k * blockDim.x;
      v[k] = i < n ? s[i] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) {
      const uint32_t i = i0 + k * blockDim.x;
      if (i < n) d[i] = v[k];
    }
  }
}

// ---------------------------------------------------------------- per-batch preparation
// One kernel replaces the per-batch runtime fills: it zeroes the lane's output and counter
// buffers and the zero tail after the batch (K1's chains read past its end), and builds the
// coarse file map.  (Each fill was a runtime kernel of its own, ~7 us each, 16 per batch.)
constexpr int kPrepZeros = 16;
struct PrepArgs {
  const uint64_t* off;
  uint32_t nfiles;
  uint64_t ncf;  // entries of cf
  uint32_t* cf;
  uint8_t* zp[kPrepZeros];  // byte ranges to zero
  uint64_t zn[kPrepZeros];
  uint32_t nz;
};

__device__ __forceinline__ void zero_range(uint8_t* p, uint64_t n, uint64_t tid, uint64_t nth) {
  const uint64_t a = min<uint64_t>(n, (16 - ((uintptr_t)p & 15)) & 15);  // bytes before 16-B alignment
  const uint64_t body = (n - a) / 16;
  for (uint64_t i = tid; i < a; i += nth) p[i] = 0;
  uint4* q = (uint4*)(p + a);
  for (uint64_t i = tid; i < body; i += nth) q[i] = make_uint4(0, 0, 0, 0);
  uint8_t* t = p + a + body * 16;
  for (uint64_t i = tid; i < n - a - body * 16; i += nth) t[i] = 0;
}

__global__ void __launch_bounds__(256) prep_kernel(PrepArgs A) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t k = tid; k < A.ncf; k += nth) A.cf[k] = bsearch_file(A.off, 0, A.nfiles, k << kCfShift);
  for (uint32_t z = 0; z < A.nz; z++) zero_range(A.zp[z], A.zn[z], tid, nth);
}

// ---------------------------------------------------------------- outputs to the host
// One kernel writes a batch's outputs straight into pinned, host-mapped memory: the
// candidate records (their count is only known on the device), per-file flags (bit 0 the
// overflow flag, bit 1 folding runes present: the fallback keywords' bits, bit 2 the
// file's keyword row was written), the keyword rows the host reads -- files with
// candidates (K2's hascand) or a flag, every file when the plan has host-only rules or K2
// skipped a group; each row once -- and the small arrays (counters, skipped groups).  The
// host reads a keyword row only with bit 2 set (plan.cpp resolve_batch checks it).
// It replaces the candidate copy kernel and five runtime D2H copies; the sparse rows cut
// the PCIe writes of a 1 GiB batch from ~1.4 MB to ~0.2 MB.  Every range starts 16-B
// aligned on both sides (host_out_alloc, hipMalloc).
constexpr int kOutCopies = 4;
struct OutArgs {
  const uint32_t* count;  // device counters (0 candidates, 7 groups skipped)
  uint32_t cand_cap;
  const uint8_t* cand;  // DevCand records
  uint8_t* cand_host;
  const uint8_t* src[kOutCopies];
  uint8_t* dst[kOutCopies];
  uint64_t n[kOutCopies];
  uint32_t nc;
  const uint32_t* kw;  // [F * W] device keyword bits
  uint32_t* kw_host;
  const uint8_t* ovf;  // [F] device overflow flags
  const uint8_t* hascand;  // [F] device: the file has a candidate record
  uint8_t* flags_host;
  uint32_t F, W, fb_lo, fb_hi;  // fallback keywords (folding runes): ids [fb_lo, fb_hi)
  uint32_t all_rows;            // every keyword row (host-only rules)
};

__device__ __forceinline__ void copy_range(uint8_t* __restrict__ d, const uint8_t* __restrict__ s, uint64_t n,
                                           uint64_t tid, uint64_t nth) {
  const uint64_t body = n / 16;
  for (uint64_t i = tid; i < body; i += nth) ((uint4*)d)[i] = ((const uint4*)s)[i];
  for (uint64_t i = body * 16 + tid; i < n; i += nth) d[i] = s[i];
}

__global__ void __launch_bounds__(256) outputs_kernel(OutArgs A) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (uint64_t)gridDim.x * blockDim.x;
  const uint32_t ncand = min(A.count[0], A.cand_cap);
  copy_range(A.cand_host, A.cand, (uint64_t)ncand * 12u, tid, nth);
  for (uint32_t c = 0; c < A.nc; c++) copy_range(A.dst[c], A.src[c], A.n[c], tid, nth);
  const bool all = A.all_rows || A.count[7] != 0;
  if (all) copy_range((uint8_t*)A.kw_host, (const uint8_t*)A.kw, (uint64_t)A.F * A.W * 4u, tid, nth);
  for (uint64_t f = tid; f < A.F; f += nth) {
    const uint32_t* row = A.kw + f * A.W;
    uint32_t fold = 0;
    for (uint32_t k = A.fb_lo; k < A.fb_hi; k++) fold |= (row[k / 32] >> (k % 32)) & 1u;
    const uint8_t fl = (A.ovf[f] ? 1 : 0) | (fold ? 2 : 0);
    const bool put = all || fl || A.hascand[f];
    A.flags_host[f] = fl | (put ? 4 : 0);
    if (put && !all)
      for (uint32_t w = 0; w < A.W; w++) A.kw_host[f * A.W + w] = row[w];
  }
}

// ---------------------------------------------------------------- K1
typedef unsigned short us2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));  // 8-byte aligned: one ds_read_b64

// Two LDS layouts of the literal automaton.
//
// Packed (K1P, every rule set whose automaton rows fit 16-bit byte offsets; the builtin
// rules: 515 states x 46 entries): per byte ONE ds_read_b64 of the byte's class entry and
// ONE ds_read_u16 of the transition, and four VALU ops:
//   a   = v_perm(word, lane8, sel)     the entry's address b * 256 + (lane % 32) * 8, built
//                                      from the byte in place (no extract, no shift)
//   e   = class entry {class * 2 + kK1PTab, keep}
//   s   = tab[s + e.x]                 s is the row's byte offset: no scale, no mask
//   cnt = cnt * keep + keep  (v_pk_mad_u16, saturating)   keep = {in D, in U}: the two run
//                                      counters grow by one or drop to zero in one op
//   mx  = max(mx, cnt), top = max(top, s) (every other byte: v_max3)
// against 7.9 for the legacy layout (profiles/r03: bfe + shift + or for the class address,
// a mask and a shift for the transition address, an add, an and and a max for the
// counters, and per-byte dword selects of a half-unrolled loop).  The class entries are
// replicated per lane of a 32-lane half ([byte][lane % 32], 8 B each: 32 lanes read 256
// contiguous bytes, conflict-free), 64 KiB; the transitions follow at kK1PTab.
//
// Legacy (automata too large for 16-bit byte offsets, e.g. a large user rule set): class
// words (class * 2 | 0xFF00 if in D | 0xFFFF0000 if in U), replicated per lane where the
// automaton leaves room (K1_REP), the transition table after them, rows as entry indices.
constexpr uint32_t kK1PTab = 256 * 256;  // packed: class entries below, transitions above
constexpr int kK1PLdsK = 128;            // packed: static LDS image, KiB (1 block of 1024 per CU)


__device__ __forceinline__ uint32_t pk_mad_sat(uint32_t cnt, uint32_t keep) {
  uint32_t r;
  asm("v_pk_mad_u16 %0, %1, %2, %2 clamp" : "=v"(r) : "v"(cnt), "v"(keep));
  return r;
}

// legacy run counters: high half = U run length, low half = D run length << 8 (both
// saturating); m (the byte's class word) keeps the halves of the classes the byte is in
__device__ __forceinline__ uint32_t run_step(uint32_t cnt, uint32_t m) {
  const us2 inc = {(unsigned short)0x0100, (unsigned short)0x0001};
  us2 c = __builtin_elementwise_add_sat(__builtin_bit_cast(us2, cnt), inc);
  return __builtin_bit_cast(uint32_t, c) & m;
}
__device__ __forceinline__ uint32_t run_max(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t,
                            __builtin_elementwise_max(__builtin_bit_cast(us2, a), __builtin_bit_cast(us2, b)));
}

struct K1Args {
  const uint8_t* data;
  const uint64_t* off;
  const uint32_t* cf;  // coarse file map (file_of)
  uint64_t total, nchunks, nitems, item_step;
  uint32_t chunk, nfiles;
  uint32_t* kw;    // [nfiles * kw_words]
  uint32_t* ev;    // [nchunks, padded to whole items]
  uint32_t* hits;  // [ns] arrivals per accepting state (sampling pass) or null
  uint32_t seg;    // consecutive chunks per chain
};

// one chain = one segment of consecutive chunks: automaton row, run counters, the running
// maximum of the counters and the event bits of the current chunk.  Chains do not track
// files: the automaton and the counters run over the batch as one byte stream (a chunk's
// events are then a superset of its files' own, see k1_reference), and the rare accept
// path finds the file of each keyword occurrence and keeps it only if it lies inside it.
// Quad transpose (K1 loads): the 4 lanes of a quad load 64 contiguous bytes of ONE
// stream per instruction (lane q gets its word q), so a wave instruction touches 16
// 64-byte segments instead of 64 scattered 16-byte words.  After loads for the 4 streams
// of the quad, lane q holds word q of every stream; two DPP butterfly stages (across
// lane^1, then lane^2) leave lane q with the 4 words of its own stream.
__device__ __forceinline__ uint32_t dpp_xor1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ uint32_t dpp_xor2(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
}
// a[t] = word q of stream t  ->  a[w] = word w of stream q   (q = lane & 3)
__device__ __forceinline__ void quad_transpose(uint32_t (&a)[4], bool b0, bool b1) {
#pragma unroll
  for (int p = 0; p < 4; p += 2) {
    const uint32_t r = dpp_xor1(b0 ? a[p] : a[p + 1]);
    if (b0) a[p] = r;
    else a[p + 1] = r;
  }
#pragma unroll
  for (int p = 0; p < 2; p++) {
    const uint32_t r = dpp_xor2(b1 ? a[p] : a[p + 2]);
    if (b1) a[p] = r;
    else a[p + 2] = r;
  }
}
__device__ __forceinline__ void quad_transpose4(uint4 (&v)[4], bool b0, bool b1) {
  uint32_t x[4] = {v[0].x, v[1].x, v[2].x, v[3].x}, y[4] = {v[0].y, v[1].y, v[2].y, v[3].y};
  uint32_t z[4] = {v[0].z, v[1].z, v[2].z, v[3].z}, w[4] = {v[0].w, v[1].w, v[2].w, v[3].w};
  quad_transpose(x, b0, b1);
  quad_transpose(y, b0, b1);
  quad_transpose(z, b0, b1);
  quad_transpose(w, b0, b1);
#pragma unroll
  for (int t = 0; t < 4; t++) v[t] = make_uint4(x[t], y[t], z[t], w[t]);
}

struct K1Chain {
  uint32_t s, cnt, mx, evl;
};

__device__ __forceinline__ uint32_t word_of(const uint4 v, int k) {  // (k constant: no select)
  return k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w;
}

// K1 arrival in reporting row r at batch byte q: keyword bits of q's file (each keyword only
// if it starts inside that file), event bits of the chunk (into evl)
__device__ __forceinline__ void k1_accept(const DevK1& d, const K1Args& A, uint32_t& evl, uint32_t r, uint64_t q) {
  const uint32_t id = r / d.row_unit;
  if (A.hits && q < A.total) atomicAdd(&A.hits[id], 1u);
  const uint32_t* m = d.masks + (size_t)d.accs[id] * d.mw;
  evl |= m[d.kw_words];
  if (q >= A.total) return;
  const uint32_t f = file_of(A.cf, A.off, A.nfiles, q);
  const uint64_t avail = q - A.off[f] + 1;  // bytes of f up to and including q
  uint32_t* kwf = A.kw + (size_t)f * d.kw_words;
  for (uint32_t w = 0; w < d.kw_words; w++) {
    uint32_t bits = m[w];
    if (!bits) continue;
    if (avail < d.kw_maxlen) {
      for (uint32_t t = bits; t; t &= t - 1) {
        const uint32_t k = __builtin_ctz(t);
        if (d.kw_len[w * 32 + k] > avail) bits &= ~(1u << k);
      }
      if (!bits) continue;
    }
    atomicOr(&kwf[w], bits);
  }
}

template <int KWW, bool PACKED, bool REP>
struct K1Lane {
  const DevK1& d;
  const K1Args& A;
  const uint8_t* smem;    // the block's LDS image
  const uint8_t* s_tab;   // legacy: the transition table
  const uint32_t* s_cls;  // legacy: this lane's column of the class words (REP) or the table
  uint32_t lane8;         // packed: (lane % 32) * 8

  // byte k (0..3) of dword w: the chain's row s and run counters cnt step once
  __device__ __forceinline__ void step(uint32_t& s, uint32_t& cnt, uint32_t w, int k) const {
    if constexpr (PACKED) {
      const uint32_t a = __builtin_amdgcn_perm(w, lane8, 0x0C0C0000u | ((4u + (uint32_t)k) << 8));
      const u32x2 e = *(const u32x2*)(smem + a);
      s = *(const uint16_t*)(smem + s + e.x);
      cnt = pk_mad_sat(cnt, e.y);
    } else {
      const uint32_t b = (w >> (8 * k)) & 0xFFu;
      const uint32_t m = REP ? s_cls[b << 5] : s_cls[b];
      s = *(const uint16_t*)(s_tab + (s + s + (m & 0xFFu)));
      cnt = run_step(cnt, m);
    }
  }
  __device__ __forceinline__ uint32_t run_bits(uint32_t mx) const {
    return ((mx >> 16) >= d.kU ? kEvRunU : 0u) | ((mx & 0xFFFFu) >= d.kD ? kEvRunD : 0u);
  }
  // NS chains, 16 bytes each, interleaved byte by byte (fully unrolled: constant byte
  // positions); a word in which a chain reached a reporting row is replayed on the rare
  // path.  pos[i]: batch byte of chain i's word.
  template <int NS>
  __device__ __forceinline__ void fast16(K1Chain (&c)[NS], const uint4 (&v)[NS], const uint64_t (&pos)[NS]) {
    uint32_t s0[NS], top[NS];
#pragma unroll
    for (int i = 0; i < NS; i++) {
      s0[i] = c[i].s;
      top[i] = 0;
    }
#pragma unroll K1_UNROLL
    for (int k = 0; k < 16; k++)
#pragma unroll
      for (int i = 0; i < NS; i++) {
        step(c[i].s, c[i].cnt, word_of(v[i], k), k & 3);
        top[i] = max(top[i], c[i].s);
        c[i].mx = run_max(c[i].mx, c[i].cnt);
      }
    // a word in which a chain reached a reporting row is replayed byte by byte (rare: the
    // adaptation keeps arrivals near one per 4 KiB); a ghost word (pos = total) reports nothing
#pragma unroll
    for (int i = 0; i < NS; i++)
      if (__builtin_expect(top[i] >= d.acc_row && pos[i] < A.total, 0)) c[i].evl |= replay(s0[i], pos[i]);
  }
  // the word at batch byte p again, byte by byte from row s: every arrival sets its keyword
  // bits; returns the word's event bits
  __device__ __forceinline__ uint32_t replay(uint32_t s, uint64_t p) const {
    const uint4 v = *(const uint4*)(A.data + p);
    uint32_t evl = 0, cnt = 0;
#pragma unroll 1
    for (uint32_t k = 0; k < 16; k++) {
      step(s, cnt, k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w, (int)(k & 3));
      if (s >= d.acc_row) k1_accept(d, A, evl, s, p + k);
    }
    return evl;
  }

  // An item = NS segments of A.seg consecutive chunks; quad lane t walks item it0 + t of ib
  // bytes (a ghost lane past the last item repeats it0 and stores nothing).  Chain i walks
  // segment i (its state carries from one chunk to the next, so only the segment start
  // needs the warm-up replay of the d.warm bytes before it); loads are quad-transposed.
  template <int NS>
  __device__ __forceinline__ void item_quad(uint64_t it0, uint64_t ib, uint32_t q) {
    const uint8_t* data = A.data;
    const uint32_t C = A.chunk;
    const uint64_t L = (uint64_t)C * A.seg;  // segment bytes
    const bool ghost = it0 + q >= A.nitems;
    const uint64_t a = (ghost ? it0 : it0 + q) * ib;
    const uint64_t c0 = a / C;
    const bool b0 = q & 1, b1 = (q >> 1) & 1;
    K1Chain c[NS];
#pragma unroll
    for (int i = 0; i < NS; i++) {
      c[i].s = d.start;
      c[i].cnt = 0;
      c[i].mx = 0;
      c[i].evl = 0;
    }
    // warm-up: the d.warm bytes before each segment (the front pad before byte 0), with
    // no reporting: afterwards row and counters equal those of the one-stream run
    for (uint32_t j = 0; j < d.warm; j += 16) {
      uint4 v[NS];
#pragma unroll
      for (int i = 0; i < NS; i++) v[i] = *(const uint4*)(data + a + (uint64_t)i * L - d.warm + j);
#pragma unroll
      for (int k = 0; k < 16; k++)
#pragma unroll
        for (int i = 0; i < NS; i++) step(c[i].s, c[i].cnt, word_of(v[i], k), k & 3);
    }
    const uint8_t* src[4];  // word q of quad lane t's item
#pragma unroll
    for (int t = 0; t < 4; t++) src[t] = data + (it0 + t < A.nitems ? it0 + t : it0) * ib + 16u * q;
    uint32_t jc = 0;
    uint64_t ci = c0;
    auto word_end = [&]() __attribute__((always_inline)) {
      jc += 16;
      if (jc == C) {
        if (!ghost)
#pragma unroll
          for (int i = 0; i < NS; i++) A.ev[ci + (uint64_t)i * A.seg] = c[i].evl | run_bits(c[i].mx);
#pragma unroll
        for (int i = 0; i < NS; i++) {
          c[i].evl = 0;
          c[i].mx = 0;
        }
        jc = 0;
        ci++;
      }
    };
    auto word = [&](uint64_t jw, const uint4 (&v)[NS]) __attribute__((always_inline)) {
      uint64_t pos[NS];
#pragma unroll
      for (int i = 0; i < NS; i++) pos[i] = ghost ? A.total : a + (uint64_t)i * L + jw;
      fast16<NS>(c, v, pos);
      word_end();
    };
    // 64 bytes of every chain at j: transpose, then the 4 words in order (each word's
    // registers picked with constant indices so the arrays stay in VGPRs)
    auto block = [&](uint64_t j, uint4 (&r)[NS][4]) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < NS; i++) quad_transpose4(r[i], b0, b1);
      uint4 v0[NS], v1[NS], v2[NS], v3[NS];
#pragma unroll
      for (int i = 0; i < NS; i++) {
        v0[i] = r[i][0];
        v1[i] = r[i][1];
        v2[i] = r[i][2];
        v3[i] = r[i][3];
      }
      word(j, v0);
      word(j + 16, v1);
      word(j + 32, v2);
      word(j + 48, v3);
    };
    auto load = [&](uint4 (&r)[NS][4], uint64_t j) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < NS; i++)
#pragma unroll
        for (int t = 0; t < 4; t++) r[i][t] = *(const uint4*)(src[t] + ((uint64_t)i * L + j));
    };
    // one 64-B block per chain, stepped in place, then reloaded (profiles/r03/k1: 0.400 ->
    // 0.385 ms per GiB against a copy of the block)
    uint4 r0[NS][4];
    load(r0, 0);
    for (uint64_t j = 0; j < L; j += 64) {
      block(j, r0);
      load(r0, j + 64);
    }
  }
};

// The K1 kernel: every block stages the automaton once (a persistent grid), then its quads
// walk 4 consecutive items together (uniform trip count inside a quad).  Accept masks stay
// in global memory (rare path).  LDSK: the static LDS image in KiB.
template <int KWW, bool PACKED, int LDSK, bool REP, int TPB>
__global__ void __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(4, 8))) k1_kernel(DevK1 d, K1Args A) {
  constexpr int NS = kK1Chains;
  __shared__ __attribute__((aligned(16))) uint8_t smem[LDSK * 1024];
  const uint32_t* tsrc = (const uint32_t*)d.tab;
  if constexpr (PACKED) {
    static_assert(LDSK * 1024 >= (int)kK1PTab + 65536, "packed K1 image: 64 KiB of class entries + 64 KiB of rows");
    u32x2* dst = (u32x2*)smem;  // [byte][lane % 32]
    const u32x2* src = (const u32x2*)d.pcls;
    for (uint32_t i = threadIdx.x; i < 256u * 32u; i += blockDim.x) dst[i] = src[i >> 5];
    uint32_t* tdst = (uint32_t*)(smem + kK1PTab);
    for (uint32_t i = threadIdx.x; i < d.tab_words; i += blockDim.x) tdst[i] = tsrc[i];
  } else {
    constexpr uint32_t kTabOff = REP ? kK1RepBytes : 1024;
    static_assert(!REP || LDSK * 1024 > (int)kK1RepBytes, "K1_REP needs room for the automaton");
    uint32_t* s_cls = (uint32_t*)smem;
    uint32_t* tdst = (uint32_t*)(smem + kTabOff);
    for (uint32_t i = threadIdx.x; i < d.tab_words; i += blockDim.x) tdst[i] = tsrc[i];
    for (uint32_t i = threadIdx.x; i < (REP ? 256u * 32u : 256u); i += blockDim.x) s_cls[i] = d.cls[REP ? i >> 5 : i];
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 31;
  K1Lane<KWW, PACKED, REP> L{d, A, smem, smem + (REP ? kK1RepBytes : 1024), (const uint32_t*)smem + (REP ? lane : 0),
                             lane * 8};
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint32_t q = threadIdx.x & 3;
  const uint64_t ib = (uint64_t)A.item_step * NS * A.seg * A.chunk;
  for (uint64_t it0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) & ~3ull; it0 < A.nitems; it0 += stride)
    L.template item_quad<NS>(it0, ib, q);
}

// ---------------------------------------------------------------- K1F
// The filter-and-verify K1 (k1f.hpp): every wave streams a contiguous range of 1 KiB tiles,
// lane l taking the 16-byte word at tile + 16 l (one coalesced 16-B load per lane).  Per
// byte: the address of its entry from the byte in place (v_perm), one ds_read_b128 of the
// entry (replicated per 16 lanes: conflict-free whatever the text), and per window end R(q)
// = and3 + and.  Nothing waits on the previous byte.  The three look-behind bytes of lane l's
// windows come from lane l-1 as partial ANDs (DPP wave_shr), lane 0's from the previous
// tile's lane 63 (readlane); the run flags of words l-1 and l-2 likewise.  A word whose
// windows name a bucket is listed in a per-wave LDS ring (word offset, groups of four window
// ends, bucket union); 64 listed words are verified together, one per lane, against the
// bucket's literal records (window compare, then the whole literal), and a match sets its
// event bits (its last byte's chunk) and keyword bit (the file holding that byte, when the
// literal starts inside it) with atomics.  Run events are ORed per chunk over the lanes of
// the chunk (ballots) and written with one atomic per chunk; prep zeroes the events.  The
// block's part of the coarse file map sits in LDS, so a keyword arrival away from file
// starts sets its bit without a global load, and a literal inside the captured bytes is
// compared without one: the verification of the last words of the range (which nothing
// overlaps) costs LDS latency, not HBM round trips under full streaming load.
#ifndef K1F_QUEUE
#define K1F_QUEUE 128
#endif
#ifndef K1F_SHARES
#define K1F_SHARES 1  // tile ranges by the waves' SIMD slots (0: equal; measurement builds)
#endif
#ifndef K1F_STEAL
#define K1F_STEAL 0  // 1/K1F_STEAL of a block's tiles claimed in chunks by the first waves done
#endif               // (0: none; measured without gain, profiles/r06/o: variants fs*, fc*)
#ifndef K1F_STEAL_CHUNK
#define K1F_STEAL_CHUNK 8  // tiles per claim
#endif
#ifndef K1F_NO_END_ATOMICS
#define K1F_NO_END_ATOMICS 0  // (1: no block-end counters or stamp; a timing probe only)
#endif
#ifndef K1F_WTRACE
#define K1F_WTRACE 0  // per-wave trace (TSG_K1F_TRACE; measurement builds, variant "ftr")
#endif
constexpr uint32_t kFQueue = K1F_QUEUE;                    // ring entries (32 B) per wave
static_assert(kFQueue >= 64 && (kFQueue & (kFQueue - 1)) == 0, "a tile lists up to 64 words");
constexpr uint32_t kFEntBytes = 256 * 256;                 // 256 entries x 16 replicas x 16 B
constexpr uint32_t kFQueueOff = kFEntBytes;
#ifndef K1F_THREADS
#define K1F_THREADS 1024
#endif
constexpr int kFThreads = K1F_THREADS;                     // one block per CU
constexpr uint32_t kFImgOff = kFQueueOff + (kFThreads / 64) * kFQueue * 32;
constexpr uint32_t kFCfOff = kFImgOff + kFImgMax;
constexpr uint32_t kFCfMax = 512;                          // coarse file map entries in LDS
constexpr uint32_t kFStOff = kFCfOff + 4 * kFCfMax;        // block counters (listed, arrivals, reserve claims)
constexpr uint32_t kFBitsOff = kFStOff + 16;               // the block's event-chunk bitmap (event list)
constexpr uint32_t kFBitsWords = 3 * kFThreads;             // 12 KiB: 98,304 chunks of the block's range
constexpr uint32_t kFZoneOff = kFBitsOff + 4 * kFBitsWords;  // zone chunks marked: own [0, 32), next [32, 64) words
constexpr uint32_t kFZoneChunks = 1024;                     // zone chunks per side (launch_k1f checks)
constexpr uint32_t kFLds = kFZoneOff + 2 * kFZoneChunks / 8;  // 158 KiB at 1024 threads
static_assert(kFLds <= 160 * 1024, "K1F's LDS");
#ifndef K1F_DEPTH
#define K1F_DEPTH 4
#endif

constexpr uint32_t kFDepth = K1F_DEPTH;                    // tiles in flight per wave

struct DevK1F {
  const uint4* ent;    // [256] entries d_0..d_3
  const uint8_t* img;  // verification image (k1f.hpp)
  uint32_t img_bytes, kw_words, nlit;
};

struct K1FArgs {
  const uint8_t* data;
  const uint64_t* off;
  const uint32_t* cf;  // coarse file map (file_of)
  uint32_t total, chunk, nfiles, ntiles, ncf;  // ncf: entries of cf
  uint32_t* kw;
  uint32_t* ev;     // zeroed by prep; ORed into
  uint32_t* hits;   // [nlit] verified arrivals per record (sampling pass) or null
  uint32_t* stats;  // [2] listed words, verified arrivals (zeroed by prep)
  // null, or the batch's clock stamps (u64, zeroed by prep; device wall clock): [0] ~first
  // block start (atomicMax of the complement = min), [1] last block end; the gates pass
  // writes [2] ~its first block start, K2 [3] its last block end.  The kernels' own
  // durations, beside the HIP events around their launches (bench.py reports both).
  unsigned long long* clk;
  // the event list (null: none; the gates pass compacts the events instead): every chunk
  // whose event word K1F makes non-zero, once, in no particular order (ItemArgs::evlist).
  // A chunk of a block's range at least `zone` bytes past its start gets events from that
  // block alone (a literal ends at most zone - 1 bytes past its window end): the block marks
  // it in an LDS bitmap and lists its marked chunks at its end.  The chunks of the first
  // zone bytes of a range get events from that block and the blocks before it: each block
  // marks the zone chunks it touches (its own zone and the next range's) in LDS, and at its
  // end claims them in `claim` (a bit per chunk, zeroed by prep); the block whose claim
  // sets a chunk's bit lists it.  (No atomic in the tile loop returns a value: a returning
  // one there made the compiler wait for every tile load in flight.)
  uint32_t* evlist;
  uint32_t* nev;
  uint32_t zone;
  uint32_t evcap;  // entries of evlist (a bound; the list holds each chunk once)
  uint32_t* claim;
  // null, or per wave (measurements, TSG_K1F_TRACE): {start after the staging, end of its
  // tiles, tiles << 32 | listed words, XCC_ID << 32 | HW_ID} (wall clock, 100 MHz)
  unsigned long long* wtrace;
};

// lane i <- lane i - 1, lane 0 <- old (DPP wave_shr:1, out-of-range source keeps old)
__device__ __forceinline__ uint32_t f_shr1(uint32_t v, uint32_t old) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}
// lane i <- lane i - 1, lane 0 <- lane 63 (DPP wave_ror:1; every lane has a source, so no
// "old" operand: one instruction instead of a zeroing move and the DPP move)
__device__ __forceinline__ uint32_t f_ror1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x13C, 0xF, 0xF, true);
}
// lane l <- lane l - 1 of this tile, lane 0 <- lane 63 of the previous tile
__device__ __forceinline__ uint32_t f_prev(uint32_t cur, uint32_t prev) { return f_shr1(cur, f_ror1(prev)); }

__device__ __forceinline__ uint32_t f_load4u(const uint8_t* data, uint32_t a) {  // bytes a..a+3
  const uint32_t* p = (const uint32_t*)(data + (a & ~3u));
  return __builtin_amdgcn_alignbyte(p[1], p[0], a & 3u);
}

// a lane's 16 bytes of a tile, non-temporal (the batch streams through once): K1F 0.255 ->
// 0.251 ms and K2 0.129 -> 0.122 ms per GiB against default-policy loads (profiles/r05/c3;
// K1F_NT=0 builds the default policy for measurement)
#ifndef K1F_NT
#define K1F_NT 1
#endif
typedef uint32_t f_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 f_tile_load(const uint8_t* p) {
#if K1F_NT
  const f_u32x4 v = __builtin_nontemporal_load((const f_u32x4*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
#else
  return *(const uint4*)p;
#endif
}

struct FCarry {  // the previous tile's per-lane window partials and run flags (f_prev)
  uint32_t a, b, c, m, m1;
};

struct K1FLane {
  const DevK1F& d;
  const K1FArgs& A;
  const uint8_t* smem;
  uint32_t lane, lane16;

  // One tile: the lane's 16 bytes v at batch byte pos.  Returns the run events of the word
  // (kEvRunU / kEvRunD) and the OR of its windows by groups of four (g[i]: ends 4i..4i+3).
  __device__ __forceinline__ uint4 entry(uint32_t w, int k) const {  // byte k (0..3) of dword w
    return *(const uint4*)(smem + __builtin_amdgcn_perm(w, lane16, 0x0C0C0000u | ((4u + (uint32_t)k) << 8)));
  }
  // One tile: the lane's 16 bytes v.  Returns the run events of the word (kEvRunU /
  // kEvRunD) and the OR of its windows by groups of four (g[i]: window ends 4i..4i+3).  In
  // three phases (bytes 13-15, 0-7, 8-12) so that at most 8 entries are live: the registers
  // left over hold more tiles in flight (kFDepth).
  __device__ __forceinline__ uint32_t tile(uint4 v, FCarry& cy, uint32_t (&g)[4]) const {
    // bytes 13..15: the partial windows lane l+1 needs
    const uint4 e13 = entry(v.w, 1), e14 = entry(v.w, 2), e15 = entry(v.w, 3);
    const uint32_t ao = k1f_and3(e13.x, e14.y, e15.z), bo = e14.x & e15.y, co = e15.x;
    const uint32_t ai = f_prev(ao, cy.a), bi = f_prev(bo, cy.b), ci = f_prev(co, cy.c);
    cy.a = ao;
    cy.b = bo;
    cy.c = co;
    uint32_t r[16];
    __builtin_amdgcn_sched_barrier(0);
    {  // bytes 0..7
      uint4 e[8];
#pragma unroll
      for (int k = 0; k < 8; k++) e[k] = entry(k < 4 ? v.x : v.y, k & 3);
      r[0] = ai & e[0].w;
      r[1] = k1f_and3(bi, e[0].z, e[1].w);
      r[2] = k1f_and3(ci, e[0].y, e[1].z) & e[2].w;
#pragma unroll
      for (int k = 3; k < 8; k++) r[k] = k1f_and3(e[k - 3].x, e[k - 2].y, e[k - 1].z) & e[k].w;
      // partial windows ending at 8, 9, 10
      r[8] = k1f_and3(e[5].x, e[6].y, e[7].z);
      r[9] = e[6].x & e[7].y;
      r[10] = e[7].x;
    }
    __builtin_amdgcn_sched_barrier(0);
    {  // bytes 8..12 (13..15 from above)
      uint4 e[8];
#pragma unroll
      for (int k = 0; k < 5; k++) e[k] = entry(k < 4 ? v.z : v.w, k & 3);
      e[5] = e13;
      e[6] = e14;
      e[7] = e15;
      r[8] &= e[0].w;
      r[9] = k1f_and3(r[9], e[0].z, e[1].w);
      r[10] = k1f_and3(r[10], e[0].y, e[1].z) & e[2].w;
#pragma unroll
      for (int k = 3; k < 8; k++) r[8 + k] = k1f_and3(e[k - 3].x, e[k - 2].y, e[k - 1].z) & e[k].w;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) g[i] = k1f_or3(r[4 * i], r[4 * i + 1], r[4 * i + 2]) | r[4 * i + 3];
    const uint32_t m = k1f_flags(r[3], r[7], r[11], r[15]);
    const uint32_t m1 = f_prev(m, cy.m), m2 = f_prev(m1, cy.m1);
    cy.m = m;
    cy.m1 = m1;
    return k1f_runs(m, m1, m2);
  }
  // the same with all 16 entries read at once (one LDS round trip per tile, 64 VGPRs of
  // entries; measurement build K1F_ALL16)
  __device__ __forceinline__ uint32_t tile16(uint4 v, FCarry& cy, uint32_t (&g)[4]) const {
    uint4 e[16];
#pragma unroll
    for (int k = 0; k < 16; k++) e[k] = entry(k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w, k & 3);
    const uint32_t ao = k1f_and3(e[13].x, e[14].y, e[15].z), bo = e[14].x & e[15].y, co = e[15].x;
    const uint32_t ai = f_prev(ao, cy.a), bi = f_prev(bo, cy.b), ci = f_prev(co, cy.c);
    cy.a = ao;
    cy.b = bo;
    cy.c = co;
    uint32_t r[16];
    r[0] = ai & e[0].w;
    r[1] = k1f_and3(bi, e[0].z, e[1].w);
    r[2] = k1f_and3(ci, e[0].y, e[1].z) & e[2].w;
#pragma unroll
    for (int k = 3; k < 16; k++) r[k] = k1f_and3(e[k - 3].x, e[k - 2].y, e[k - 1].z) & e[k].w;
#pragma unroll
    for (int i = 0; i < 4; i++) g[i] = k1f_or3(r[4 * i], r[4 * i + 1], r[4 * i + 2]) | r[4 * i + 3];
    const uint32_t m = k1f_flags(r[3], r[7], r[11], r[15]);
    const uint32_t m1 = f_prev(m, cy.m), m2 = f_prev(m1, cy.m1);
    cy.m = m;
    cy.m1 = m1;
    return k1f_runs(m, m1, m2);
  }
};

// Verification of listed words (k1f_kernel drains its ring 64 words at a time):
// the LDS image of the literal records and the byte entries, either replicated per 16 lanes
// (k1f_kernel's table: entry of byte b at b << 8 | lane16) or plain (entry at b << 4).
// bytes o .. o+3 (o <= 19) of the captured bytes w
__device__ __forceinline__ uint32_t f_wat(const uint32_t (&w)[6], uint32_t o) {
  const uint32_t i = o >> 2;
  const uint32_t lo = i == 0 ? w[0] : i == 1 ? w[1] : i == 2 ? w[2] : i == 3 ? w[3] : w[4];
  const uint32_t hi = i == 0 ? w[1] : i == 1 ? w[2] : i == 2 ? w[3] : i == 3 ? w[4] : w[5];
  return __builtin_amdgcn_alignbyte(hi, lo, o & 3u);
}

// event bits `bits` for chunk c (K1FArgs::evlist): c in [c_lo, c_hi) -> the block's bitmap,
// c in [z_lo, c_lo) (its zone) or [c_hi, c_hi + kFZoneChunks) (the next range's) -> the zone
// bitmaps
struct K1FMark {
  const K1FArgs& A;
  uint32_t* lbm;  // LDS bitmap of chunks [c_lo, c_hi)
  uint32_t* lzm;  // LDS bitmaps of chunks [z_lo, z_lo + kFZoneChunks), [c_hi, c_hi + kFZoneChunks)
  uint32_t z_lo, c_lo, c_hi;
  __device__ __forceinline__ void operator()(uint32_t c, uint32_t bits) const {
    atomicOr(&A.ev[c], bits);
    if (!A.evlist) return;
    if (c >= c_lo && c < c_hi) {
      atomicOr(&lbm[(c - c_lo) >> 5], 1u << ((c - c_lo) & 31));
    } else {
      const uint32_t z = c < c_lo ? c - z_lo : kFZoneChunks + (c - c_hi);
      if (z < 2 * kFZoneChunks) atomicOr(&lzm[z >> 5], 1u << (z & 31));
    }
  }
};

struct K1FVerify {
  const DevK1F& d;
  const K1FArgs& A;
  const uint8_t* img;  // the verification image in LDS
  const uint8_t* ent;  // the entries in LDS
  uint32_t eshift, lane16;
  const uint32_t* lcf;  // cf[kc0 .. kc0 + ncl) in LDS
  uint32_t kc0, ncl;
  const K1FMark& mark;

  // a verified occurrence of record i starting at s, ending at e (< total)
  __device__ __forceinline__ void report(const K1FLit& L, uint32_t i, uint32_t s, uint32_t e, uint32_t& narr) const {
    narr++;
    if (A.hits) atomicAdd(&A.hits[i], 1u);
    if (L.ev) mark(e / A.chunk, L.ev);
    if (L.kw >= 0) {
      // the same file holds the first bytes of the coarse blocks of s and past e's: no file
      // starts in (s, e], the literal lies inside the file holding e
      const uint32_t ks = (s >> kCfShift) - kc0, ke = (e >> kCfShift) + 1 - kc0;
      uint32_t f;
      bool in;
      if (ks < ncl && ke < ncl && lcf[ks] == lcf[ke]) {
        f = lcf[ks];
        in = true;
      } else {
        f = file_of(A.cf, A.off, A.nfiles, e);
        in = s >= A.off[f];
      }
      if (in) atomicOr(&A.kw[(size_t)f * d.kw_words + (uint32_t)L.kw / 32], 1u << ((uint32_t)L.kw % 32));
    }
  }

  // The listed word at P with its bytes P-4 .. P+15 as captured at listing (w[0..4]): every
  // window end of the groups in gm, against the buckets in bu.  Only a window that equals a
  // literal's reads the batch again, for the part of the literal outside the captured bytes.
  __device__ void verify(uint32_t P, uint32_t gm, uint32_t bu, const uint32_t (&w)[6], uint32_t& narr) const {
    const uint16_t* bstart = (const uint16_t*)img;
    const K1FLit* recs = (const K1FLit*)(img + kFImgLits);
    for (uint32_t k = 0; k < 16; k++) {
      if (!((gm >> (k >> 2)) & 1)) continue;
      const uint32_t win = f_wat(w, k + 1);  // window bytes P+k-3 .. P+k
      uint32_t bm = bu;
#pragma unroll
      for (int j = 0; j < 4; j++)
        bm &= *(const uint32_t*)(ent + ((((win >> (8 * j)) & 0xFFu) << eshift) | lane16) + 4 * j);
      bm &= 0xFFFFu;
      if (!bm) continue;
      const uint32_t q = P + k, wl = k1f_lower4(win);
      for (; bm; bm &= bm - 1) {
        const uint32_t b = __builtin_ctz(bm);
        for (uint32_t i = bstart[b]; i < bstart[b + 1]; i++) {
          const K1FLit L = recs[i];
          if ((wl & L.wmask) != L.wkey || q < L.wend) continue;
          const uint32_t s = q - L.wend, e = s + L.len - 1;
          if (e >= A.total) continue;
          bool eq = true;
          if (s + 4 >= P && e < P + 16) {  // inside the captured bytes
            const uint32_t os = s + 4 - P;
#pragma unroll
            for (uint32_t tt = 0; tt < 20; tt += 4) {
              if (tt < L.len) {
                const uint32_t dv = k1f_lower4(f_wat(w, os + tt));
                const uint32_t lv = *(const uint32_t*)(img + L.boff + tt);
                const uint32_t mk = L.len - tt >= 4 ? ~0u : (1u << (8 * (L.len - tt))) - 1u;
                eq = eq && ((dv ^ lv) & mk) == 0;
              }
            }
            if (eq) report(L, i, s, e, narr);
            continue;
          }
          // the whole literal, 32 bytes per round from aligned dword loads issued together
          // (one dependent load per dword cost a round trip each: profiles/r05/ab3)
          const uint32_t* dw = (const uint32_t*)(A.data + (s & ~3u));
          const uint32_t sh = s & 3u;
          for (uint32_t t = 0; t < L.len && eq; t += 32) {
            uint32_t dd[9];
#pragma unroll
            for (int u = 0; u < 9; u++) dd[u] = t + 4 * u < L.len + 4 ? dw[t / 4 + u] : 0u;
#pragma unroll
            for (int u = 0; u < 8; u++) {
              const uint32_t tt = t + 4 * u;
              if (tt < L.len) {
                const uint32_t dv = k1f_lower4(__builtin_amdgcn_alignbyte(dd[u + 1], dd[u], sh));
                const uint32_t lv = *(const uint32_t*)(img + L.boff + tt);
                const uint32_t mk = L.len - tt >= 4 ? ~0u : (1u << (8 * (L.len - tt))) - 1u;
                eq = eq && ((dv ^ lv) & mk) == 0;
              }
            }
          }
          if (eq) report(L, i, s, e, narr);
        }
      }
    }
  }
};

__global__ void __launch_bounds__(kFThreads) k1f_kernel(DevK1F d, K1FArgs A) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[kFLds];
  if (A.clk && threadIdx.x == 0 && blockIdx.x < 8)  // (the first blocks dispatched: GATES_STAMPS)
    atomicMax(&A.clk[0], ~(unsigned long long)wall_clock64());
  {  // the entries (replicated) and the image, every load issued before the stores
    constexpr uint32_t kRep = 256u * 16u / kFThreads, kImg = kFImgMax / 16 / kFThreads;
    uint4 e[kRep], m[kImg];
#pragma unroll
    for (uint32_t k = 0; k < kRep; k++) e[k] = d.ent[(threadIdx.x + k * kFThreads) >> 4];
#pragma unroll
    for (uint32_t k = 0; k < kImg; k++) {
      const uint32_t i = threadIdx.x + k * kFThreads;
      m[k] = i < d.img_bytes / 16 ? ((const uint4*)d.img)[i] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (uint32_t k = 0; k < kRep; k++) ((uint4*)smem)[threadIdx.x + k * kFThreads] = e[k];
#pragma unroll
    for (uint32_t k = 0; k < kImg; k++) {
      const uint32_t i = threadIdx.x + k * kFThreads;
      if (i < d.img_bytes / 16) ((uint4*)(smem + kFImgOff))[i] = m[k];
    }
  }
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wpb = blockDim.x >> 6;
  const uint32_t gw = blockIdx.x * wpb + wave, nw = gridDim.x * wpb;
  // the coarse file map around the block's bytes (literals reach 4 KiB either side)
  const uint64_t bb0 = (uint64_t)blockIdx.x * wpb * A.ntiles / nw * kFTile;
  const uint64_t bb1 = (uint64_t)(blockIdx.x + 1) * wpb * A.ntiles / nw * kFTile;
  const uint32_t kc0 = (uint32_t)((bb0 > 4096 ? bb0 - 4096 : 0) >> kCfShift);
  const uint64_t kc1 = min<uint64_t>(A.ncf, ((bb1 + 4096) >> kCfShift) + 2);
  const uint32_t ncl = kc1 > kc0 ? (uint32_t)min<uint64_t>(kc1 - kc0, kFCfMax) : 0u;
  uint32_t* lcf = (uint32_t*)(smem + kFCfOff);
  for (uint32_t i = threadIdx.x; i < ncl; i += blockDim.x) lcf[i] = A.cf[kc0 + i];
  uint32_t* bst = (uint32_t*)(smem + kFStOff);  // listed words, arrivals
  if (threadIdx.x < 3) bst[threadIdx.x] = 0;
  // the event list: the block's non-zone chunks [c_lo, c_hi) in the LDS bitmap, the zone
  // chunks in the zone bitmaps
  uint32_t* lbm = (uint32_t*)(smem + kFBitsOff);
  uint32_t* lzm = (uint32_t*)(smem + kFZoneOff);
  const uint32_t z_lo = (uint32_t)(bb0 / A.chunk);
  const uint32_t c_hi = max(z_lo, (uint32_t)(min<uint64_t>(bb1, A.total + (uint64_t)A.chunk - 1) / A.chunk));
  const uint32_t c_lo = min(c_hi, (uint32_t)((bb0 + A.zone + A.chunk - 1) / A.chunk));
  const uint32_t nbw = A.evlist ? (c_hi - c_lo + 31) / 32 : 0u;  // (<= kFBitsWords: launch_k1f)
  for (uint32_t i = threadIdx.x; i < nbw; i += blockDim.x) lbm[i] = 0;
  if (threadIdx.x < 2 * kFZoneChunks / 32) lzm[threadIdx.x] = 0;
  const K1FMark mark{A, lbm, lzm, z_lo, c_lo, c_hi};
  __syncthreads();
  // The block's tiles [bt0, bt1) split over its waves unequally: the four waves a SIMD holds
  // do not share it evenly -- per wave of one launch, 140 / 166 / 196 / 228 us for the same
  // 256 tiles by the wave's slot on its SIMD, which follows the wave's index in the block
  // (slot = wave / 4: waves are created in order and dealt round-robin to the SIMDs;
  // TSG_K1F_TRACE, tools/k1ftrace.py, profiles/r06/j).  With equal ranges the block waited
  // for its slot-3 waves; ranges in proportion to the slots' measured speeds end closer
  // together.  A slot's speed depends on the shares (the more tiles slot 0 takes, the slower
  // the others' tiles run), so the shares are a fixed point: 1 / (us per tile) of each slot
  // measured with the previous shares, three rounds from equal ranges (k1ftrace.py
  // "shares_next"; 0.248 -> 0.2298 -> 0.2227 -> 0.2196 ms per GiB, profiles/r06/l, m, o).
  // (Any split is correct: each wave scans its own contiguous range after the tile before.)
  // With K1F_STEAL the last 1/K1F_STEAL of the block's tiles is a reserve [bs, bt1) the
  // waves claim in chunks of K1F_STEAL_CHUNK tiles (an LDS counter) once their own range is
  // done.  The shares leave a block's waves 16-32 us apart at the end; the reserve evens
  // them out (every slot's waves 201-203 us) but the launch is no shorter: the blocks' own
  // means differ by as much (189-200 us), and every chunk restarts the load queue
  // (profiles/r06/o: 0.2191-0.2205 ms per GiB for 1/8 and 1/16, 0.227 for 1/4, shares
  // alone 0.2193-0.2199).
  uint32_t t0, t1, bs, bt1;
  {
    const uint64_t bt0 = (uint64_t)blockIdx.x * wpb * A.ntiles / nw;
    bt1 = (uint32_t)((uint64_t)(blockIdx.x + 1) * wpb * A.ntiles / nw);
    bs = K1F_STEAL ? bt1 - (uint32_t)((bt1 - bt0) / K1F_STEAL) : bt1;
#if K1F_SHARES
    constexpr uint32_t kShare[4] = {361, 282, 207, 150};  // per slot: its speed, all four slots busy
    const uint32_t tot = (wpb / 4) * (kShare[0] + kShare[1] + kShare[2] + kShare[3]);
    uint32_t before = 0;
    for (uint32_t w = 0; w < wave; w++) before += kShare[(w * 4 / wpb) & 3];
    const uint32_t mine = kShare[(wave * 4 / wpb) & 3];
    t0 = (uint32_t)(bt0 + (bs - bt0) * before / tot);
    t1 = (uint32_t)(bt0 + (bs - bt0) * (before + mine) / tot);
#else
    t0 = (uint32_t)(bt0 + (bs - bt0) * wave / wpb);
    t1 = (uint32_t)(bt0 + (bs - bt0) * (wave + 1) / wpb);
#endif
  }
#if K1F_WTRACE
  if (A.wtrace && lane == 0) {
    A.wtrace[4 * gw] = wall_clock64();
    A.wtrace[4 * gw + 3] = ((unsigned long long)__builtin_amdgcn_s_getreg(20 | (15 << 11)) << 32) |
                           (uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11));
  }
#endif
  uint32_t ntile = 0;  // (trace: tiles this wave scanned)
  if (t0 < t1 || bs < bt1) {  // (waves without tiles wait at the block barrier below)
  const K1FLane L{d, A, smem, lane, (lane & 15u) << 4};
  uint4* ring = (uint4*)(smem + kFQueueOff) + 2 * wave * kFQueue;  // 2 x uint4 per entry
  uint32_t qh = 0, qn = 0, nlisted = 0, narr = 0;
  // n (<= 64) listed words verified, one per lane, from their captured bytes
  auto drain = [&](uint32_t n) __attribute__((always_inline)) {
    __builtin_amdgcn_wave_barrier();
    if (lane < n) {
      const uint32_t i = (qh + lane) & (kFQueue - 1);
      const uint4 x = ring[2 * i], y = ring[2 * i + 1];
      const uint32_t w[6] = {x.z, x.w, y.x, y.y, y.z, 0u};
      const K1FVerify V{d, A, smem + kFImgOff, smem, 8, (lane & 15u) << 4, lcf, kc0, ncl, mark};
      V.verify(x.x, x.y & 0xFu, x.y >> 16, w, narr);
    }
    __builtin_amdgcn_wave_barrier();
    qh = (qh + n) & (kFQueue - 1);
    qn -= n;
  };
  FCarry cy{0, 0, 0, 0, 0};  // (the warm-up tile's own inputs do not reach its outputs)
  // vw: lane 63's last dword of the previous tile (the captured bytes before lane 0's word),
  // kept in a scalar register: a per-lane copy of the tile's .w held its queue register past
  // the reload and made the loop wait for the loads in flight at its back edge
  uint32_t g[4], vw = 0;
  // A listed word enters the ring with its 20 bytes (the 4 before it from the previous
  // lane), so its verification reads LDS, not the batch; 64 listed words are verified
  // together.  The batch has a zero tail of 8 KiB: no load leaves the batch and its tail.
  const uint8_t* base = A.data + 16u * lane;
  auto body = [&](uint4 v, uint32_t t) __attribute__((always_inline)) {
    const uint32_t pos = t * kFTile + 16u * lane;
#if K1F_ALL16
    const uint32_t rb = L.tile16(v, cy, g);
#else
    const uint32_t rb = L.tile(v, cy, g);
#endif
      // run events: one atomic per chunk (the leader lane of each chunk in the tile)
    const uint64_t bu = __ballot(rb & 1u), bd = __ballot(rb & 2u);
    if (__builtin_expect(bu | bd, 0)) {
      const uint32_t c = pos / A.chunk;
      const bool lead = lane == 0 || pos - c * A.chunk < 16u;
      const uint64_t ld = __ballot(lead);
      if (lead) {
        const uint64_t above = ld & (~0ull << lane << 1);
        const uint64_t gm = (above ? (above & (~above + 1)) - 1 : ~0ull) & (~0ull << lane);
        const uint32_t bits = ((bu & gm) ? kEvRunU : 0u) | ((bd & gm) ? kEvRunD : 0u);
        if (bits) mark(c, bits);
      }
    }
    // listed words
    const uint32_t un = k1f_or3(g[0], g[1], g[2]) | g[3];
    const uint32_t bun = un & 0xFFFFu;
    const uint64_t hb = __ballot(bun != 0);
    if (__builtin_expect(hb != 0, 0)) {
      const uint32_t n = (uint32_t)__popcll(hb);
      if (kFQueue < 128 && qn + n > kFQueue) drain(qn);  // (a small ring: room for the tile's words)
      const uint32_t wprev = f_shr1(v.w, vw);  // bytes pos-4 .. pos-1 (all lanes: DPP)
      if (bun) {
        const uint32_t slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(hb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hb, 0u));
        const uint32_t gm = ((g[0] & 0xFFFFu) ? 1u : 0u) | ((g[1] & 0xFFFFu) ? 2u : 0u) | ((g[2] & 0xFFFFu) ? 4u : 0u) |
                            ((g[3] & 0xFFFFu) ? 8u : 0u);
        const uint32_t i = (qh + qn + slot) & (kFQueue - 1);
        ring[2 * i] = make_uint4(pos, gm | bun << 16, wprev, v.x);
        ring[2 * i + 1] = make_uint4(v.y, v.z, v.w, 0u);
      }
      qn += n;
      nlisted += n;
      if (qn >= 64) drain(64);
    }
    vw = __builtin_amdgcn_readlane(v.w, 63);
  };
  for (;;) {  // the wave's own range, then reserve chunks
  if (t0 < t1) {
  // the range's loads: the tile before t0 (its carries; zero bytes before the batch) first,
  // then the first kFDepth tiles, so the warm-up waits only for its own load.  The batch has
  // a zero tail of 8 KiB: loads past the last tile stay inside it.
  const uint4 vwu = f_tile_load(A.data + (size_t)(t0 > 0 ? t0 - 1 : 0) * kFTile + 16u * lane);
  uint4 p[kFDepth];
#pragma unroll
  for (uint32_t k = 0; k < kFDepth; k++) p[k] = f_tile_load(base + (size_t)(t0 + k) * kFTile);
  {
    const uint4 v = t0 > 0 ? vwu : make_uint4(0, 0, 0, 0);
    (void)L.tile(v, cy, g);
    vw = __builtin_amdgcn_readlane(v.w, 63);
  }
  // the tiles of the range, kFDepth loads in flight (memory latency bounds a wave with fewer:
  // profiles/r05/kv2)
  uint32_t t = t0;
  for (; t + kFDepth <= t1; t += kFDepth) {
    // the words listed so far are verified before the range's last tiles, while their loads
    // are in flight: a verification at the very end (a literal read back, a file lookup)
    // would extend the kernel by its latency (profiles/r05/ab3)
    if (t + 2 * kFDepth > t1 && qn) drain(qn);
    // each tile is consumed before its queue register is reloaded: no register copies at
    // the loop's back edge, whose vmcnt(0) waited for the youngest load every kFDepth tiles
    // (the loop waits vmcnt(kFDepth - 1) before each tile instead)
#pragma unroll
    for (uint32_t k = 0; k < kFDepth; k++) {
      body(p[k], t + k);
      p[k] = f_tile_load(base + (size_t)(t + kFDepth + k) * kFTile);
    }
  }
#pragma unroll
  for (uint32_t k = 0; k < kFDepth - 1; k++)
    if (t + k < t1) body(p[k], t + k);
  ntile += t1 - t0;
  }
  if (bs >= bt1) break;
  uint32_t c = 0;
  if (lane == 0) c = atomicAdd(&bst[2], (uint32_t)K1F_STEAL_CHUNK);
  c = __builtin_amdgcn_readfirstlane(c);
  if (c >= bt1 - bs) break;
  t0 = bs + c;
  t1 = min(t0 + (uint32_t)K1F_STEAL_CHUNK, bt1);
  }
  if (qn) drain(qn);
  // the counters: per wave, per block in LDS, one global atomic per block (a same-address
  // atomic from every lane or wave at the end of the kernel serialised into its tail:
  // 20 us per launch, profiles/r05/ab6)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) narr += __shfl_xor(narr, o);
  if (lane == 0) {
    atomicAdd(&bst[0], nlisted);
    atomicAdd(&bst[1], narr);
  }
#if K1F_WTRACE
  if (A.wtrace && lane == 0) {
    A.wtrace[4 * gw + 1] = wall_clock64();
    A.wtrace[4 * gw + 2] = ((unsigned long long)ntile << 32) | nlisted;
  }
#endif
  }
  __syncthreads();
  if (A.evlist && threadIdx.x < 2 * kFZoneChunks / 32) {  // the zone chunks this block touched
    for (uint32_t b = lzm[threadIdx.x]; b; b &= b - 1) {
      const uint32_t z = 32 * threadIdx.x + __builtin_ctz(b);
      const uint32_t c = z < kFZoneChunks ? z_lo + z : c_hi + (z - kFZoneChunks);
      const uint32_t bit = 1u << (c & 31);
      if (!(atomicOr(&A.claim[c >> 5], bit) & bit)) {
        const uint32_t i = atomicAdd(A.nev, 1u);
        if (i < A.evcap) A.evlist[i] = c;
      }
    }
  }
  if (nbw) {  // the block's marked chunks into the event list: one claim per block
    uint32_t wv[kFBitsWords / kFThreads], n = 0;
#pragma unroll
    for (uint32_t k = 0; k < kFBitsWords / kFThreads; k++) {
      const uint32_t i = threadIdx.x + k * kFThreads;
      wv[k] = i < nbw ? lbm[i] : 0u;
      n += __popc(wv[k]);
    }
    uint32_t inc = n;  // inclusive scan over the wave, then over the block's waves in LDS
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o);
      if (lane >= (uint32_t)o) inc += t;
    }
    uint32_t* s_w = (uint32_t*)(smem + kFQueueOff);  // (the verification rings are drained)
    if (lane == 63) s_w[wave] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t tot = 0;
      for (uint32_t w = 0; w < wpb; w++) tot += s_w[w];
      s_w[kFThreads / 64] = tot ? atomicAdd(A.nev, tot) : 0u;
    }
    __syncthreads();
    uint32_t at = s_w[kFThreads / 64] + inc - n;
    for (uint32_t w = 0; w < wave; w++) at += s_w[w];
#pragma unroll
    for (uint32_t k = 0; k < kFBitsWords / kFThreads; k++)
      for (uint32_t b = wv[k]; b; b &= b - 1, at++)
        if (at < A.evcap) A.evlist[at] = c_lo + 32 * (threadIdx.x + k * kFThreads) + __builtin_ctz(b);
  }
  if (threadIdx.x == 0 && !K1F_NO_END_ATOMICS) {
    if (bst[0]) atomicAdd(&A.stats[0], bst[0]);
    if (bst[1]) atomicAdd(&A.stats[1], bst[1]);
    if (A.clk) atomicMax(&A.clk[1], (unsigned long long)wall_clock64());
  }
}

// ---------------------------------------------------------------- K1X
// Literals K1's automaton has no room for (Plan::x_lits: keywords and anchors of a large
// user rule set).  k1x_kernel samples a 4-byte window every STEP bytes of the batch (STEP =
// Plan::x_step; 4: the word's aligned dwords, no byte shifts), ASCII case folded, and tests
// its hash against a blocked Bloom filter in LDS (x_hash: one of 2^15 dwords, two bits in
// it) holding, for every literal, its 4-grams at offsets j0..j0+STEP-1 (Plan::x_j0, windows
// source text rarely holds) -- every occurrence of a literal covers exactly one sampled
// window.  Each 16-byte word with a hit is listed (one record per lane-word, a
// 16-bit mask of hit window positions).  k1x_verify_kernel then looks every listed window up
// in an open-addressing table (4-gram -> {literal, offset}) and checks each candidate start
// exactly; a match sets its keyword bit (the whole literal inside the file holding its last
// byte, K1's accept rule) and chunk event bits (chunk of the last byte) with atomics.  A lane
// whose record does not fit the list verifies inline.
struct DevK1X {
  const uint32_t* bitmap;  // [kXDwords] blocked Bloom filter
  const uint4* slots;      // [mask + 1] {4-gram, first entry, count, 0}; count 0 = empty
  uint32_t mask, shift;    // open addressing from slot (4-gram * 0x85EBCA6B) >> shift
  const uint32_t* lits;    // the slots' entries back to back: literal | offset of the 4-gram << 24
  const uint8_t* bytes;    // literal bytes, each 4-aligned and zero padded
  const uint32_t* off;     // [n] literal starts in bytes
  const uint32_t* len;     // [n] literal lengths
  const int32_t* kwid;     // [n] keyword id or -1
  const uint32_t* ev;      // [n] event bits
  uint32_t kw_words;
  uint32_t step;           // Plan::x_step: 1, 2 or 4
  // slots, lits, off, len, kwid, ev and bytes are parts of one image (16-B aligned parts), which
  // k1x_verify_kernel stages in LDS when it fits
  const uint8_t* img;
  uint32_t img_bytes;
};
constexpr uint32_t kXImgLds = 128 * 1024;  // verify: largest image staged in LDS


struct K1XArgs {
  const uint8_t* data;
  const uint64_t* off;
  const uint32_t* cf;  // coarse file map (file_of)
  uint64_t total;
  uint32_t chunk, nfiles;
  uint32_t* kw;
  uint32_t* ev;
  uint2* list;      // {word index, hit mask}, one slice per k1x_kernel block
  uint32_t* count;  // [blocks] records in each slice
  uint32_t cap;     // records in all slices
  uint32_t* stats;  // {records listed, words verified inline} (batch counts 14, 15)
};

__device__ __forceinline__ uint32_t x_lower4(uint32_t x) {
  // ASCII 'A'..'Z' -> +0x20, every other byte unchanged (bytes >= 0x80 keep bit 7)
  const uint32_t t = x & 0x7F7F7F7Fu;
  const uint32_t ge_a = t + 0x3F3F3F3Fu;  // bit 7 set: byte >= 0x41
  const uint32_t gt_z = t + 0x25252525u;  // bit 7 set: byte >= 0x5B
  const uint32_t up = (ge_a & ~gt_z) & ~x & 0x80808080u;
  return x | (up >> 2);
}


// x_hash / x_bits of plan.hpp (the host builds the filter with those)
__device__ __forceinline__ uint32_t x_hash_dev(uint32_t w) { return w * 2654435761u; }
__device__ __forceinline__ uint32_t x_bits_dev(uint32_t h) { return 1u << ((h >> 12) & 31) | 1u << ((h >> 7) & 31); }

__device__ __forceinline__ uint32_t x_low_byte(uint8_t c) { return (c >= 'A' && c <= 'Z') ? c + 32u : c; }

// exact check of the literals whose 4-gram at some offset j starts at batch byte p (window
// w = its 4 lowercased bytes): each candidate literal starts at p - j
#ifdef K1X_DIAG  // measurement builds: slot probes, entries examined, literal matches
#define K1X_DIAG_ADD(i, v) atomicAdd(&A.stats[(i)], (v))
#else
#define K1X_DIAG_ADD(i, v) ((void)0)
#endif
__device__ void k1x_verify_at(const DevK1X& x, const K1XArgs& A, uint64_t p, uint32_t w) {
  // (the product's top bits: its low bits see only the window's first bytes)
  uint32_t h = (w * 0x85EBCA6Bu) >> x.shift;
  for (;;) {
    const uint4 sl = x.slots[h];
    K1X_DIAG_ADD(-4, 1u);
    if (sl.z == 0) return;  // no literal with this 4-gram
    if (sl.x == w) {
      K1X_DIAG_ADD(-6, sl.z);
      for (uint32_t e = 0; e < sl.z; e++) {
        const uint32_t ent = x.lits[sl.y + e];
        const uint32_t i = ent & 0xFFFFFFu, j = ent >> 24;
        if (p < j) continue;
        const uint64_t s = p - j;
        const uint32_t a = x.off[i], len = x.len[i];
        if (s + len > A.total) continue;
        // compare 32 bytes per round from aligned dword loads issued together (a byte loop
        // of dependent loads cost 0.19 ms per GiB on configs[3]); the batch has a zero tail
        const uint32_t* lw = (const uint32_t*)(x.bytes + a);  // 4-aligned, zero padded
        const uint32_t* dw = (const uint32_t*)(A.data + (s & ~3ull));
        const uint32_t sh = (uint32_t)(s & 3);
        bool eq = true;
        for (uint32_t k = 0; k < len && eq; k += 32) {
          uint32_t d[9];
#pragma unroll
          for (int u = 0; u < 9; u++) d[u] = k + 4 * u < len + 4 ? dw[k / 4 + u] : 0u;
#pragma unroll
          for (int u = 0; u < 8; u++) {
            const uint32_t kk = k + 4 * u;
            if (kk < len) {
              const uint32_t v = x_lower4(sh ? __builtin_amdgcn_alignbyte(d[u + 1], d[u], sh) : d[u]);
              const uint32_t m = len - kk >= 4 ? ~0u : (1u << (8 * (len - kk))) - 1u;
              eq = eq && ((v ^ lw[kk / 4]) & m) == 0;
            }
          }
        }
        if (!eq) continue;
        K1X_DIAG_ADD(-5, 1u);
        const uint64_t q = s + len - 1;
        if (x.ev[i]) atomicOr(&A.ev[q / A.chunk], x.ev[i]);
        const int32_t k = x.kwid[i];
        if (k >= 0) {
          const uint32_t f = file_of(A.cf, A.off, A.nfiles, q);
          if (s >= A.off[f]) atomicOr(&A.kw[(size_t)f * x.kw_words + k / 32], 1u << (k % 32));
        }
      }
      return;
    }
    h = (h + 1) & x.mask;
  }
}

constexpr int kK1XBlock = 1024;
#ifndef K1X_WORDS
#define K1X_WORDS 4
#endif
constexpr int kXWords = K1X_WORDS;  // words per lane per round (k1x_kernel)

// the window at byte k of a word (d: its dwords and the next word's first)
__device__ __forceinline__ uint32_t k1x_window(const uint32_t (&d)[5], int k) {
  return (k & 3) ? __builtin_amdgcn_alignbyte(d[k / 4 + 1], d[k / 4], k & 3) : d[k / 4];
}

template <int STEP>
__device__ __forceinline__ uint32_t k1x_hits(const uint32_t* s_bm, const uint32_t (&d)[5]) {
  uint32_t hits = 0;
#pragma unroll
  for (int k = 0; k < 16; k += STEP) {
    const uint32_t h = x_hash_dev(k1x_window(d, k)), m = x_bits_dev(h);  // d: folded (x_fold)
    hits |= (uint32_t)((s_bm[h >> (32 - kXDwordBits)] & m) == m) << k;
  }
  return hits;
}

// Each block lists its hit records in its own slice of A.list (an LDS counter, no global
// atomics); a record past the slice is verified inline.  A.count[block] = records kept.
template <int STEP>
__global__ void __launch_bounds__(kK1XBlock) k1x_kernel(DevK1X x, K1XArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_bm[];  // the filter, then the block's record counter
  uint32_t* s_n = s_bm + kXDwords;
  stage16((uint8_t*)s_bm, x.bitmap, kXDwords * 4);
  if (threadIdx.x == 0) *s_n = 0;
  __syncthreads();
  const uint32_t slice = A.cap / gridDim.x;
  uint2* list = A.list + (size_t)blockIdx.x * slice;
  const uint64_t nwords = (A.total + 15) / 16;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  // kXWords words per lane per round (each load coalesced across the wave), the next
  // round's words in flight while this round is hashed: at 2 waves per SIMD (the 128 KiB
  // bitmap) one word ahead left every round waiting for HBM
  constexpr int U = kXWords;
  uint4 v[U];
  uint32_t nx[U];
  auto load = [&](uint64_t w0) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t w = w0 + (uint64_t)u * stride;
      // (the batch is padded with zero bytes past its end)
      v[u] = w < nwords ? *(const uint4*)(A.data + w * 16) : make_uint4(0, 0, 0, 0);
      // (STEP 4 never shifts a window into the next word)
      if constexpr (STEP < 4) nx[u] = w < nwords ? *(const uint32_t*)(A.data + w * 16 + 16) : 0u;
      else nx[u] = 0u;
    }
  };
  uint64_t wi = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  load(wi);
  for (; wi < nwords; wi += (uint64_t)U * stride) {
    uint4 cv[U];
    uint32_t cn[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      cv[u] = v[u];
      cn[u] = nx[u];
    }
    load(wi + (uint64_t)U * stride);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t w = wi + (uint64_t)u * stride;
      if (w >= nwords) break;
      // the filter's keys are case folded by setting bit 5 of every byte (x_fold: exact for
      // ASCII letters, a coarser fold elsewhere -- verification is exact)
      const uint32_t d[5] = {cv[u].x | kXFold, cv[u].y | kXFold, cv[u].z | kXFold, cv[u].w | kXFold,
                             cn[u] | kXFold};
      uint32_t hits = k1x_hits<STEP>(s_bm, d);
      // positions past the batch end never count (their window holds pad bytes)
      const uint64_t p0 = w * 16;
      if (p0 + 16 > A.total) hits &= (1u << (uint32_t)(A.total - p0)) - 1u;
      if (__builtin_expect(hits != 0, 0)) {
        const uint32_t slot = atomicAdd(s_n, 1u);
        if (slot < slice) {
          list[slot] = make_uint2((uint32_t)w, hits);
        } else {
          const uint32_t lw[5] = {x_lower4(cv[u].x), x_lower4(cv[u].y), x_lower4(cv[u].z), x_lower4(cv[u].w),
                                  x_lower4(cn[u])};
          for (uint32_t t = hits; t; t &= t - 1) {
            const int k = __builtin_ctz(t);
            k1x_verify_at(x, A, p0 + k, k1x_window(lw, k));
          }
        }
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t n = *s_n, kept = min(n, slice);
    A.count[blockIdx.x] = kept;
    atomicAdd(&A.stats[0], kept);
    if (n > kept) atomicAdd(&A.stats[1], n - kept);
  }
}

static const void* k1x_fn(uint32_t step) {
  if (step == 4) return (const void*)k1x_kernel<4>;
  if (step == 2) return (const void*)k1x_kernel<2>;
  return (const void*)k1x_kernel<1>;
}

// One block per k1x_kernel block, its slice of the list.  LDS: the table image is staged
// first, so the lookups of a 4-gram that the text holds often (thousands of threads on the
// same slot, entries and literal bytes) are LDS broadcasts instead of one L2 channel's
// queue -- 10x on configs[3] (profiles/r04/xv).
constexpr int kXVerifyBlock = 1024;
template <bool LDS>
__global__ void __launch_bounds__(kXVerifyBlock) k1x_verify_kernel(DevK1X x, K1XArgs A, uint32_t nblocks) {
  extern __shared__ __attribute__((aligned(16))) uint8_t x_img[];
  const uint32_t b = blockIdx.x;
  const uint32_t n = A.count[b];
  if (n == 0) return;
  DevK1X y = x;
  if constexpr (LDS) {
    stage16(x_img, x.img, x.img_bytes / 16 * 16);
    __syncthreads();
    auto rebase = [&](auto* p) { return (decltype(p))(x_img + ((const uint8_t*)p - x.img)); };
    y.slots = rebase(x.slots);
    y.lits = rebase(x.lits);
    y.off = rebase(x.off);
    y.len = rebase(x.len);
    y.kwid = rebase(x.kwid);
    y.ev = rebase(x.ev);
    y.bytes = rebase(x.bytes);
  }
  const uint32_t slice = A.cap / nblocks;
  for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) {
    const uint2 r = A.list[(size_t)b * slice + j];
    const uint64_t p0 = (uint64_t)r.x * 16;
    for (uint32_t t = r.y; t; t &= t - 1) {
      const uint64_t p = p0 + __builtin_ctz(t);
      const uint32_t w = x_low_byte(A.data[p]) | x_low_byte(A.data[p + 1]) << 8 | x_low_byte(A.data[p + 2]) << 16 |
                         x_low_byte(A.data[p + 3]) << 24;
      k1x_verify_at(y, A, p, w);
    }
  }
}

// ---------------------------------------------------------------- gate + items
__device__ __forceinline__ bool group_gated(const uint32_t* __restrict__ kwf, const uint32_t* __restrict__ gm,
                                            uint32_t W, uint32_t always) {
  if (always) return true;
  for (uint32_t w = 0; w < W; w++)
    if (kwf[w] & gm[w]) return true;
  return false;
}

// per file: bit g of ggate[f * GW + g / 64] = group g gated (Rule.MatchKeywords may pass):
// the always-gated groups, ORed with the groups of every keyword bit the file has (a file
// holds few keywords, so the cost is its set bits x GW, not groups x keyword words)
__device__ __forceinline__ void ggate_file(uint32_t f, const uint32_t* __restrict__ kw, uint32_t F, uint32_t W,
                                           const unsigned long long* __restrict__ kwg,
                                           const unsigned long long* __restrict__ galw, uint32_t GW,
                                           unsigned long long* __restrict__ ggate) {
  if (f >= F) return;
  const uint32_t* kwf = kw + (size_t)f * W;
  for (uint32_t w0 = 0; w0 < GW; w0 += 8) {
    const uint32_t n = min(8u, GW - w0);
    unsigned long long acc[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; j++) acc[j] = j < n ? galw[w0 + j] : 0ull;
    for (uint32_t i = 0; i < W; i++)
      for (uint32_t bits = kwf[i]; bits; bits &= bits - 1) {
        const unsigned long long* row = kwg + (size_t)(i * 32 + __builtin_ctz(bits)) * GW + w0;
#pragma unroll
        for (uint32_t j = 0; j < 8; j++)
          if (j < n) acc[j] |= row[j];
      }
#pragma unroll
    for (uint32_t j = 0; j < 8; j++)
      if (j < n) ggate[(size_t)f * GW + w0 + j] = acc[j];
  }
}

struct ItemArgs {
  const uint64_t* off;
  const uint32_t* cf;  // coarse file map (file_of)
  const uint32_t* ev;
  const uint32_t* evlist;           // chunks with event bits (ev_compact_block, or K1F)
  const uint32_t* nev;              // [1] length of evlist
  uint32_t evcap;                   // entries of evlist (a bound on *nev)
  const unsigned long long* ggate;  // [F * GW]
  const unsigned long long* gofbit;  // [32 * GW] groups listening to event bit b; bit 31 = every chunk
  const uint32_t* gevents;          // [G]
  const uint32_t* gback;            // [G] chunks (kMaxBack + 1 = whole file)
  uint64_t nchunks;
  uint32_t F, G, GW, chunk, maxback;
  uint32_t* count;            // [G]
  uint32_t* bcount;           // [gridDim.x * G] each count block's place in each group's items
  uint32_t* cursor;           // [G]
  uint2* items;
  // ggate == null (K1F listed the events, no gates pass ran): a file's group gates from its
  // keyword bits, as ggate_file computes them
  const uint32_t* kw;
  uint32_t W;
  const unsigned long long* kwg;
  const unsigned long long* galw;
  unsigned long long* clk;  // K1FArgs::clk ([2]: the item passes' first block start)
  uint32_t kwg_lds;         // kwg staged in the passes' LDS (its bytes; 0: read from global)
};

// Chunks whose K1 event word is not empty, compacted into `list`.  One pass: each thread tests 32 consecutive chunks (eight 16-B loads in flight), the block
// scans the counts and claims its output range with one atomic per 32 * kBlock chunks.
// (Blocks' ranges land in the list in claim order; its readers do not need it sorted.)
constexpr uint32_t kEvPer = 32;
__device__ __forceinline__ void ev_compact_block(const uint32_t* __restrict__ ev, uint64_t nchunks,
                                                 uint32_t* __restrict__ list, uint32_t* __restrict__ count,
                                                 uint32_t bid, uint32_t nblocks) {
  __shared__ uint32_t s_wave[kBlock / 64];
  __shared__ uint32_t s_base;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr uint64_t kPer = (uint64_t)kEvPer * kBlock;
  for (uint64_t c0 = (uint64_t)bid * kPer; c0 < nchunks; c0 += (uint64_t)nblocks * kPer) {
    const uint64_t c = c0 + (uint64_t)threadIdx.x * kEvPer;
    uint32_t has = 0;
    if (c + kEvPer <= nchunks) {
      uint4 v[kEvPer / 4];
#pragma unroll
      for (uint32_t i = 0; i < kEvPer / 4; i++) v[i] = *(const uint4*)(ev + c + 4 * i);
#pragma unroll
      for (uint32_t i = 0; i < kEvPer / 4; i++)
        has |= ((v[i].x & ~kEvAlways) != 0 ? 1u : 0u) << (4 * i) | ((v[i].y & ~kEvAlways) != 0 ? 2u : 0u) << (4 * i) |
               ((v[i].z & ~kEvAlways) != 0 ? 4u : 0u) << (4 * i) | ((v[i].w & ~kEvAlways) != 0 ? 8u : 0u) << (4 * i);
    } else {
      for (uint32_t i = 0; i < kEvPer && c + i < nchunks; i++) has |= ((ev[c + i] & ~kEvAlways) != 0 ? 1u : 0u) << i;
    }
    const uint32_t n = __popc(has);
    // inclusive scan over the wave
    uint32_t inc = n;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o);
      if (lane >= (uint32_t)o) inc += t;
    }
    if (lane == 63) s_wave[wave] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t tot = 0;
      for (uint32_t w = 0; w < kBlock / 64; w++) tot += s_wave[w];
      s_base = tot ? atomicAdd(count, tot) : 0;
    }
    __syncthreads();
    uint32_t at = s_base + inc - n;
    for (uint32_t w = 0; w < wave; w++) at += s_wave[w];
    for (uint32_t t = has; t; t &= t - 1) list[at++] = (uint32_t)(c + __builtin_ctz(t));
    __syncthreads();  // s_wave / s_base reuse
  }
}

// The two passes that follow K1 and need nothing of each other, in one launch: blocks
// [0, ev_blocks) compact the event chunks, the rest compute the files' group gates.
struct GateArgs {
  const uint32_t* ev;
  uint64_t nchunks;
  uint32_t* evlist;
  uint32_t* nev;
  uint32_t ev_blocks;
  const uint32_t* kw;
  uint32_t F, W, GW;
  const unsigned long long* kwg;
  const unsigned long long* galw;
  unsigned long long* ggate;
  unsigned long long* clk;  // K1FArgs::clk
  uint32_t kwg_lds;         // kwg staged in LDS (its bytes; 0: read from global)
};
// (a file's gate is an OR over its keyword bits of kwg rows: from global memory, one L2
// round trip per bit -- a file of a 1,000-rule set holds a hundred of them -- so the table
// is staged in LDS when it fits)
constexpr uint32_t kKwgLdsMax = 48 * 1024;
#ifndef GATES_STAMPS
#define GATES_STAMPS 8  // blocks that stamp the chain's start (measurement builds: more)
#endif
__global__ void __launch_bounds__(kBlock) gates_kernel(GateArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  // (the chain's start: the first blocks only -- blocks are dispatched in order, and ~850
  // same-address atomics at the start of every block of the launch queue on one line)
  if (threadIdx.x == 0 && blockIdx.x < GATES_STAMPS) atomicMax(&A.clk[2], ~(unsigned long long)wall_clock64());
  if (blockIdx.x < A.ev_blocks) {
    ev_compact_block(A.ev, A.nchunks, A.evlist, A.nev, blockIdx.x, A.ev_blocks);
  } else {
    const unsigned long long* kwg = A.kwg;
    if (A.kwg_lds) {
      stage16(smem, A.kwg, A.kwg_lds);
      __syncthreads();
      kwg = (const unsigned long long*)smem;
    }
    ggate_file((blockIdx.x - A.ev_blocks) * blockDim.x + threadIdx.x, A.kw, A.F, A.W, kwg, A.galw, A.GW, A.ggate);
  }
}

// Items of the K2 list: (file f, chunk c) for group g iff g is gated for f and a chunk in
// [c, c + back_g] of f carries one of g's event bits (groups listening to every chunk:
// all chunks of f).  Work is generated from the sparse event chunks: event chunk e emits
// c in (previous event chunk of g, e] within back_g chunks before e and inside f, so every
// item comes from the first event chunk at or after it, exactly once.  Threads
// [0, nev) take event chunks, [nev, nev + F) take the files of every-chunk groups.
// visit(f, g, c_lo, c_hi): items c_lo..c_hi.
// the group tables gen_items reads per candidate, staged in the item passes' LDS
static inline size_t item_lds_host(uint32_t G, uint32_t GW) { return 256 * (size_t)GW + 8 * (size_t)G; }
constexpr uint32_t kItemKwgLdsMax = 16 * 1024;  // kwg staged in the item passes' LDS up to this
struct ItemLds {
  const unsigned long long* gofbit;  // [32 * GW]
  const uint32_t* gback;             // [G]
  const uint32_t* gevents;           // [G]
  const unsigned long long* kwg;     // [32 * W * GW] (LDS when ItemArgs::kwg_lds, else global)
};
__device__ __forceinline__ uint32_t item_lds_bytes(const ItemArgs& A) { return 256 * A.GW + 8 * A.G + A.kwg_lds; }
// copies the tables to smem (8-aligned); the caller's __syncthreads() publishes them
__device__ __forceinline__ ItemLds item_lds_load(const ItemArgs& A, uint8_t* smem) {
  unsigned long long* gofbit = (unsigned long long*)smem;
  uint32_t* gback = (uint32_t*)(gofbit + 32 * A.GW);
  uint32_t* gevents = gback + A.G;
  for (uint32_t i = threadIdx.x; i < 32 * A.GW; i += blockDim.x) gofbit[i] = A.gofbit[i];
  for (uint32_t i = threadIdx.x; i < A.G; i += blockDim.x) {
    gback[i] = A.gback[i];
    gevents[i] = A.gevents[i];
  }
  const unsigned long long* kwg = A.kwg;
  if (A.kwg_lds) {
    unsigned long long* k = (unsigned long long*)(gevents + A.G);
    for (uint32_t i = threadIdx.x; i < A.kwg_lds / 8; i += blockDim.x) k[i] = A.kwg[i];
    kwg = k;
  }
  return ItemLds{gofbit, gback, gevents, kwg};
}

// word w of file f's group gates (ggate_file's value)
__device__ __forceinline__ unsigned long long file_gate(const ItemArgs& A, const ItemLds& T, uint32_t f, uint32_t w) {
  if (A.ggate) return A.ggate[(size_t)f * A.GW + w];
  const uint32_t* kwf = A.kw + (size_t)f * A.W;
  unsigned long long acc = A.galw[w];
  for (uint32_t i = 0; i < A.W; i++)
    for (uint32_t bits = kwf[i]; bits; bits &= bits - 1) acc |= T.kwg[(size_t)(i * 32 + __builtin_ctz(bits)) * A.GW + w];
  return acc;
}

template <class V>
__device__ __forceinline__ void gen_items(const ItemArgs& A, const ItemLds& T, uint64_t t, V visit) {
  // (the unit's list entry is loaded beside the list's length, not after it: one memory
  // round trip less on the chain every item pass waits for)
  const uint32_t ev_t = t < A.evcap ? A.evlist[t] : 0u;
  const uint32_t nev = min(*A.nev, A.evcap);
  const uint32_t C = A.chunk;
  if (t < nev) {
    const uint64_t e = ev_t;
    const uint32_t evb = A.ev[e] & ~kEvAlways;
    const uint64_t ce = (e + 1) * C;
    // the event words of the kMaxBack chunks before e, loaded together (a dependent load per
    // chunk of the back scan cost a round trip each)
    // (five 16-B loads from the aligned base below e - 16: one wide request per lane each)
    uint32_t pw[kMaxBack];
    if (e >= (uint64_t)kMaxBack) {
      const uint64_t b0 = (e - kMaxBack) & ~3ull;
      const uint32_t sh = (uint32_t)(e - kMaxBack - b0);  // 0..3
      uint32_t x[20];
#pragma unroll
      for (int j = 0; j < 5; j++) {
        const uint4 q = *(const uint4*)(A.ev + b0 + 4 * j);
        x[4 * j] = q.x;
        x[4 * j + 1] = q.y;
        x[4 * j + 2] = q.z;
        x[4 * j + 3] = q.w;
      }
#pragma unroll
      for (int i = 0; i < kMaxBack; i++) {  // ev[e - 1 - i] = x[sh + 15 - i]
        const int k = kMaxBack - 1 - i;
        pw[i] = sh == 0 ? x[k] : sh == 1 ? x[k + 1] : sh == 2 ? x[k + 2] : x[k + 3];
      }
    } else {
#pragma unroll
      for (int i = 0; i < kMaxBack; i++) pw[i] = e > (uint64_t)i ? A.ev[e - 1 - i] : 0u;
    }
    for (uint32_t f = file_of(A.cf, A.off, A.F, e * C); f < A.F && A.off[f] < ce; f++) {
      const uint64_t fs = A.off[f], fe = A.off[f + 1];
      if (fe == fs) continue;
      const uint64_t fc0 = fs / C;
      for (uint32_t w = 0; w < A.GW; w++) {
        unsigned long long cand = 0;
        for (uint32_t bits = evb; bits; bits &= bits - 1) cand |= T.gofbit[__builtin_ctz(bits) * A.GW + w];
        cand &= file_gate(A, T, f, w) & ~T.gofbit[31 * A.GW + w];
        while (cand) {
          const uint32_t g = w * 64 + __builtin_ctzll(cand);
          cand &= cand - 1;
          const uint32_t back = T.gback[g], gev = T.gevents[g];  // back <= kMaxBack here
          const uint64_t lo0 = e > fc0 + back ? e - back : fc0;
          const uint32_t lim = (uint32_t)(e - lo0);  // chunks e-1 .. lo0
          uint32_t m = 0;  // bit i: chunk e-1-i carries one of g's events
#pragma unroll
          for (int i = 0; i < kMaxBack; i++) m |= ((pw[i] & gev) != 0 && (uint32_t)i < lim ? 1u : 0u) << i;
          visit(f, g, m ? e - __builtin_ctz(m) : lo0, e);
        }
      }
    }
  } else if (t < (uint64_t)nev + A.F) {
    const uint32_t f = (uint32_t)(t - nev);
    const uint64_t fs = A.off[f], fe = A.off[f + 1];
    if (fe == fs) return;
    for (uint32_t w = 0; w < A.GW; w++) {
      unsigned long long cand = file_gate(A, T, f, w) & T.gofbit[31 * A.GW + w];
      while (cand) {
        const uint32_t g = w * 64 + __builtin_ctzll(cand);
        cand &= cand - 1;
        visit(f, g, fs / C, (fe - 1) / C);
      }
    }
  }
}

// Both item passes run a fixed grid over the work units t in [0, nev + F) (nev is read on
// the device, so the host never waits for it), each block visiting the same units twice.
// count pass: items per group (block totals in LDS, one global atomic per group and block)
#ifndef ITEMS_BASE_IN_COUNT
#define ITEMS_BASE_IN_COUNT 1  // (0: the emit pass reserves the block's ranges; measurement builds)
#endif
__global__ void __launch_bounds__(kBlock) items_count_kernel(ItemArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  if (!A.ggate && threadIdx.x == 0 && blockIdx.x < GATES_STAMPS)  // (no gates pass)
    atomicMax(&A.clk[2], ~(unsigned long long)wall_clock64());
  const ItemLds T = item_lds_load(A, smem);
  uint32_t* s_count = (uint32_t*)(smem + item_lds_bytes(A));
  for (uint32_t g = threadIdx.x; g < A.G; g += blockDim.x) s_count[g] = 0;
  __syncthreads();
  const uint64_t nt = (uint64_t)min(*A.nev, A.evcap) + A.F, stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += stride)
    gen_items(A, T, t, [&](uint32_t, uint32_t g, uint64_t lo, uint64_t hi) { atomicAdd(&s_count[g], (uint32_t)(hi - lo + 1)); });
  __syncthreads();
  // the block's place in each group's region, reserved here: the emit pass's blocks then
  // start without a returning atomic per group (those queued on the groups' cursors)
  for (uint32_t g = threadIdx.x; g < A.G; g += blockDim.x) {
#if ITEMS_BASE_IN_COUNT
    A.bcount[(size_t)blockIdx.x * A.G + g] = s_count[g] ? atomicAdd(&A.count[g], s_count[g]) : 0u;
#else
    A.bcount[(size_t)blockIdx.x * A.G + g] = s_count[g];
    if (s_count[g]) atomicAdd(&A.count[g], s_count[g]);
#endif
  }
}

// ---------------------------------------------------------------- device-side item layout
// Every block of the emit pass decides, from the item counts, how K2 covers each group (the
// same decision in every block: the counts are final when the pass starts), so neither the
// host nor a one-block launch stands between the two item passes:
//   list   (kGroupList)  its items go to a region of the item array; K2 entries of up to
//                        kEntryItems items
//   dense  (kGroupDense) its items cover more than half the batch: K2 entries of
//                        kEntryChunks consecutive chunks of the whole batch, gated per file
//   skip   (kGroupSkip)  over the item capacity or the dense budget: K2 does not scan it
//                        and the host resolves its rules like rules without a GPU program
// Groups are taken in id order, so the outcome is deterministic.  K2's work list is written
// by all blocks (a list group's entries by block g mod grid, a dense group's sliced over the
// grid), the counters and skip flags by block 0.
struct LayoutArgs {
  const uint32_t* gcount;  // [G]
  uint32_t G;
  uint64_t nchunks, items_cap;
  uint32_t max_dense;
  uint4* entries;     // K2 work list of list groups: {group, first item, n, kGroupList}
  uint32_t* nentries;
  uint4* dentries;    // ... of dense groups: {group, first chunk, n, kGroupDense}
  uint32_t* ndentries;
  uint8_t* gskip;     // [G] (to the host)
  uint32_t* stats;    // [1] items listed, [2] entries, [3] skipped groups
};


// K2's list kernel block (measurement builds vary it).  The stepping is bound by LDS bank
// conflicts of the transition reads (random rows), so a CU's entries take the same time
// however its waves are grouped: 1,024-thread blocks (one DFA staged for 16 waves, 292
// entries of 2,048 items in about one round) ran 0.141 ms against 0.132 for 256 threads
// (972 entries of 512), profiles/r05/c6.
#ifndef K2_LIST_BLOCK
#define K2_LIST_BLOCK 256
#endif
constexpr int kK2Block = K2_LIST_BLOCK;
constexpr uint32_t kEntryItems = 2 * kK2Block;  // two chains per lane
constexpr uint32_t kEntryChunks = kStreams * kBlock;

// exclusive prefix sums of N values at once over the block (one LDS exchange, two barriers
// for all of them); returns the totals in tot.  s_wave: [N * waves]
template <int N>
__device__ void block_exclusive_scan_n(const unsigned long long (&v)[N], unsigned long long (&out)[N],
                                       unsigned long long (&tot)[N], unsigned long long* s_wave) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  unsigned long long x[N];
#pragma unroll
  for (int k = 0; k < N; k++) x[k] = v[k];
  for (int o = 1; o < 64; o <<= 1) {
#pragma unroll
    for (int k = 0; k < N; k++) {
      const unsigned long long y = __shfl_up(x[k], o);
      if (lane >= (uint32_t)o) x[k] += y;
    }
  }
  if (lane == 63)
#pragma unroll
    for (int k = 0; k < N; k++) s_wave[k * nw + wave] = x[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; k++) {
    unsigned long long before = 0, total = 0;
    for (uint32_t w = 0; w < nw; w++) {
      const unsigned long long t = s_wave[k * nw + w];
      before += w < wave ? t : 0;
      total += t;
    }
    out[k] = before + x[k] - v[k];
    tot[k] = total;
  }
  __syncthreads();
}

// the layout into s_kind / s_gbase ([G] in LDS) and K2's work list (see above)
__device__ void layout_block(const LayoutArgs& A, uint8_t* s_kind, uint32_t* s_gbase) {
  __shared__ unsigned long long s_wave64[3 * (kBlock / 64)];
  __shared__ unsigned long long s_carry[5];  // items, entries, dense groups, skipped groups, dense entries
  __shared__ uint2 s_dense[kBlock];  // dense groups of the tile: group, first dense entry
  __shared__ uint32_t s_ndense;
  __shared__ uint4 s_lst[kBlock];    // this block's list groups of the tile: group, first entry, first item, items
  __shared__ uint32_t s_nlst;
  const uint32_t ndent_all = (uint32_t)((A.nchunks + kEntryChunks - 1) / kEntryChunks);
  if (threadIdx.x < 5) s_carry[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t g0 = 0; g0 < A.G; g0 += blockDim.x) {
    if (threadIdx.x == 0) {
      s_ndense = 0;
      s_nlst = 0;
    }
    const uint32_t g = g0 + threadIdx.x;
    const uint64_t cnt = g < A.G ? A.gcount[g] : 0;
    const bool dense_want = cnt * 2 > A.nchunks;
    // dense budget first (in group order), then the item capacity for list groups (the
    // scans of one tile of groups in two rounds of one block exchange each: five separate
    // scans cost ten barriers per tile, a 1,000-rule set has four tiles)
    const bool want_list = cnt && !dense_want;
    unsigned long long p1[2], t1[2];
    block_exclusive_scan_n<2>({dense_want ? 1ull : 0ull, want_list ? cnt : 0ull}, p1, t1, s_wave64);
    const unsigned long long dpre = p1[0], dtot = t1[0], ipre = p1[1], itot = t1[1];
    const bool dense = dense_want && s_carry[2] + dpre < A.max_dense;
    const bool list = want_list && s_carry[0] + ipre + cnt <= A.items_cap;
    // items of groups that fit are placed at their prefix position (a skipped group's
    // range stays unused: the regions keep group order)
    const uint64_t nent = list ? (cnt + kEntryItems - 1) / kEntryItems : 0;
    const uint64_t ndent = dense ? ndent_all : 0;
    const bool skip = cnt && !list && !dense;
    unsigned long long p2[3], t2[3];
    block_exclusive_scan_n<3>({(unsigned long long)nent, (unsigned long long)ndent, skip ? 1ull : 0ull}, p2, t2, s_wave64);
    const unsigned long long epre = p2[0], etot = t2[0], dpre2 = p2[1], dtot2 = t2[1], stot = t2[2];
    // (entries_cap covers every list entry the item capacity allows plus max_dense dense
    // groups, so the work list always fits)
    const uint64_t e0 = s_carry[1] + epre, d0 = s_carry[4] + dpre2;
    const uint8_t k = !cnt ? kGroupNone : list ? kGroupList : dense ? kGroupDense : kGroupSkip;
    if (g < A.G) {
      s_kind[g] = k;
      s_gbase[g] = (uint32_t)(s_carry[0] + ipre);
      if (blockIdx.x == 0) A.gskip[g] = k == kGroupSkip ? 1 : 0;
    }
    if (k == kGroupList && g % gridDim.x == blockIdx.x)
      s_lst[atomicAdd(&s_nlst, 1u)] = make_uint4(g, (uint32_t)e0, (uint32_t)(s_carry[0] + ipre), (uint32_t)cnt);
    if (k == kGroupDense) s_dense[atomicAdd(&s_ndense, 1u)] = make_uint2(g, (uint32_t)d0);
    __syncthreads();
    // a list group's entries (a hundred for a group of 65 k items) by the whole block (one
    // thread writing them in a row held its block ~5 us, profiles/r05/ab/er2)
    for (uint32_t t = 0; t < s_nlst; t++) {
      const uint4 lg = s_lst[t];
      const uint32_t nl = (lg.w + kEntryItems - 1) / kEntryItems;
      for (uint32_t i = threadIdx.x; i < nl; i += blockDim.x) {
        const uint32_t first = i * kEntryItems;
        A.entries[(size_t)lg.y + i] = make_uint4(lg.x, lg.z + first, min(kEntryItems, lg.w - first), kGroupList);
      }
    }
    // a dense group's entries (nchunks / kEntryChunks of them: thousands) over the grid
    for (uint32_t t = 0; t < s_ndense; t++) {
      const uint2 dg = s_dense[t];
      for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < ndent_all; i += gridDim.x * blockDim.x) {
        const uint64_t first = (uint64_t)i * kEntryChunks;
        A.dentries[dg.y + i] = make_uint4(dg.x, (uint32_t)first,
                                          (uint32_t)min<uint64_t>(kEntryChunks, A.nchunks - first), kGroupDense);
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      s_carry[0] += itot;
      s_carry[1] += etot;
      s_carry[2] += dtot;
      s_carry[3] += stot;
      s_carry[4] += dtot2;
    }
    __syncthreads();
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *A.nentries = (uint32_t)s_carry[1];
    *A.ndentries = (uint32_t)s_carry[4];
    A.stats[1] = (uint32_t)min<unsigned long long>(s_carry[0], 0xFFFFFFFFull);
    A.stats[2] = (uint32_t)s_carry[1];
    A.stats[3] = (uint32_t)s_carry[3];
  }
}

// emit pass (same grid as the count pass, so block b generates the items block b counted):
// the layout (above), then the block writes its items into the range of each listed group
// the count pass reserved for it
__global__ void __launch_bounds__(kBlock) items_emit_kernel(ItemArgs A, LayoutArgs LA) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const ItemLds T = item_lds_load(A, smem);  // (published by layout_block's barriers)
  uint32_t* s_count = (uint32_t*)(smem + item_lds_bytes(A));
  uint32_t* s_base = s_count + A.G;
  uint32_t* s_gbase = s_base + A.G;
  uint8_t* s_kind = (uint8_t*)(s_gbase + A.G);
  layout_block(LA, s_kind, s_gbase);
  const uint64_t nt = (uint64_t)min(*A.nev, A.evcap) + A.F, stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (uint32_t g = threadIdx.x; g < A.G; g += blockDim.x) {
#if ITEMS_BASE_IN_COUNT
    s_base[g] = s_kind[g] == kGroupList ? s_gbase[g] + A.bcount[(size_t)blockIdx.x * A.G + g] : 0u;
#else
    const uint32_t n = s_kind[g] == kGroupList ? A.bcount[(size_t)blockIdx.x * A.G + g] : 0;
    s_base[g] = n ? s_gbase[g] + atomicAdd(&A.cursor[g], n) : 0;
#endif
    s_count[g] = 0;
  }
  __syncthreads();
  for (uint64_t t = t0; t < nt; t += stride)
    gen_items(A, T, t, [&](uint32_t f, uint32_t g, uint64_t lo, uint64_t hi) {
      if (s_kind[g] != kGroupList) return;
      const uint32_t n = (uint32_t)(hi - lo + 1);
      uint32_t at = s_base[g] + atomicAdd(&s_count[g], n);
      for (uint64_t c = lo; c <= hi; c++) A.items[at++] = make_uint2(f, (uint32_t)c);
    });
}

// ---------------------------------------------------------------- K2
struct K2Args {
  const uint8_t* data;
  const uint64_t* off;
  const uint32_t* cf;  // coarse file map (file_of)
  uint64_t total, nchunks;
  uint32_t chunk, ext_cap, nfiles;
  const uint32_t* kw;
  uint32_t kw_words;
  const uint32_t* gmask;    // [G * kw_words] keyword gate of each group (dense entries)
  const uint32_t* galways;  // [G]
  const uint2* items;       // list entries: (file, chunk)
  const uint4* entries;     // list entries {group, first item, n, kind} (layout_kernel)
  const uint32_t* nentries;
  const uint4* dentries;    // dense entries {group, first chunk, n, kind}
  const uint32_t* ndentries;
  DevCand* cand;
  uint32_t* cand_count;
  uint32_t cand_cap;
  uint8_t* ovf;
  uint8_t* hascand;  // [nfiles] 1: the file has a candidate record (outputs_kernel's rows)
  uint32_t* diag;  // null, or [4]: tail bytes, longest tail, tails over 4 KiB, word replays
  uint32_t* claim;  // [2] next list / dense entry (zeroed per batch)
  uint32_t word_recs;  // accepting words as one kCandWord record each (groups < 2^14)
  // null, or per entry kTraceW words {start, end (wall clock, 100 MHz), group << 32 | items,
  // XCC_ID << 32 | HW_ID, then (K2_TRACE_CTR builds only) replayed words, candidates,
  // tail bytes, longest tail} written by the block that ran it (TSG_K2_TRACE)
  unsigned long long* etrace;
  unsigned long long* clk;  // K1FArgs::clk
};
constexpr int kTraceW = 8;
#ifdef K2_TRACE_CTR  // measurement builds: per-entry counters of the running entry
__shared__ unsigned long long* s_ectr;
#define K2_CTR(k, op, v) (s_ectr ? (void)op(&s_ectr[k], (unsigned long long)(v)) : (void)0)
#else
#define K2_CTR(k, op, v) ((void)0)
#endif
#ifdef K2_TRACE_PHASE  // measurement builds: wall-clock stamps of thread 0 in words 4..7
__shared__ unsigned long long* s_tph;
#define K2_PHASE(k) (s_tph && threadIdx.x == 0 ? (void)(s_tph[k] = wall_clock64()) : (void)0)
#else
#define K2_PHASE(k) ((void)0)
#endif

// Candidate emission, wave-aggregated: the lanes that reach an accept together reserve
// their records with ONE atomic (ballot, popcount prefix, broadcast of the base).  A record
// past the capacity flags its file for whole-file host resolution instead.
// end == kCandWhole: "resolve this rule over the whole file" (a follow-on tail past
// ext_cap), which the host reads instead of an end offset (plan.hpp kCandWhole)
__device__ __forceinline__ void emit_cand(const K2Args& A, uint32_t file, uint32_t rule, uint64_t end) {
  const unsigned long long m = __ballot(1);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t leader = (uint32_t)__builtin_ctzll(m);
  uint32_t base = 0;
  if (lane == leader) {
    base = atomicAdd(A.cand_count, (uint32_t)__popcll(m));
    K2_CTR(1, atomicAdd, __popcll(m));
  }
  base = __shfl(base, (int)leader);
  const uint32_t idx = base + (uint32_t)__popcll(m & ((1ull << lane) - 1));
  if (idx < A.cand_cap && (end < kCandWhole || end == (uint64_t)kCandWhole)) {
    A.cand[idx] = DevCand{file, rule, (uint32_t)end};
  } else {
    A.ovf[file] = 1;  // (also a file of 4 GiB or more: its 32-bit end offsets would wrap)
    if (idx < A.cand_cap) A.cand[idx] = DevCand{file, rule, 0};
  }
  A.hascand[file] = 1;
}

#ifdef K2_NOINL  // the rare paths out of line (their registers do not add to the hot loop's)
#define K2_NOINLINE __attribute__((noinline))
#else
#define K2_NOINLINE __forceinline__
#endif
#ifdef K2_W
#define K2_WAVES __attribute__((amdgpu_waves_per_eu(K2_W, 8)))
#else
#define K2_WAVES
#endif
struct Lane {
  const DevDFA& d;
  const K2Args& A;
  const uint16_t* s_tab;
  const uint8_t* s_cls;
  const uint16_t* s_accs;
  const uint64_t* s_masks;
  uint32_t file;
  uint64_t fs;
  uint32_t group;

  // accept at end of text (rare): one record per rule of the state's end-of-text mask
  __device__ __forceinline__ void emit(uint32_t mi, uint64_t pos) {
    const uint64_t* m = (d.state_acc && mi < d.nmasks) ? s_masks + (size_t)mi * d.mw : d.masks + (size_t)mi * d.mw;
    for (uint32_t w = 0; w < d.mw; w++)
      for (uint64_t v = m[w]; v; v &= v - 1)
        emit_cand(A, file, d.rules[w * 64 + __builtin_ctzll(v)], pos - fs);
  }

  __device__ __forceinline__ uint32_t state_of(uint32_t row) const { return __umulhi(row, d.inv_nc); }

  // the record of an accepting transition (kCandTrans: the host expands its accept mask)
  __device__ __forceinline__ uint32_t trans(uint32_t ix) const { return kCandTrans | (group << 16) | ix; }
  // An accepting 16-B word as ONE record (kCandWord): the row before byte p, p's offset in
  // the file; the host replays the word from there to the word's end (or the file's) and
  // expands every accepting transition on the way (plan.cpp resolve_batch).  Without it
  // (more groups than 14 bits), replay_emit writes the transitions themselves.
  __device__ __forceinline__ void accept_word(uint32_t s0, const uint4 v, int lo, int hi, uint64_t wb) {
    if (A.word_recs)
      emit_cand(A, file, kCandTrans | kCandWord | (group << 16) | s0, wb + (uint64_t)lo - fs);
    else
      replay_emit(s0, v, lo, hi, wb);
  }
  // one candidate record at idx (see emit_cand)
  __device__ __forceinline__ void put(uint32_t idx, uint32_t rule, uint64_t end) const {
    if (idx < A.cand_cap && end < kCandWhole) {
      A.cand[idx] = DevCand{file, rule, (uint32_t)end};
    } else {
      A.ovf[file] = 1;
      if (idx < A.cand_cap) A.cand[idx] = DevCand{file, rule, 0};
    }
    A.hascand[file] = 1;
  }
  // A word with an accept, again from registers (bytes lo..hi-1 of v, batch position wb):
  // its accepting transitions are counted, reserved with one atomic and written as
  // transition records.  A relaxed unbounded rule accepts at every byte of a long token
  // run; emitting those one by one, each after a dependent global lookup of the accept
  // mask and the rules, made entries of a few dozen items the kernel's long pole
  // (profiles/r03/d2, r03/k2a: 30-80 items, ~600 candidates, 0.4-0.5 ms).
  __device__ K2_NOINLINE void replay_emit(uint32_t s0, const uint4 v, int lo, int hi, uint64_t wb) {
    uint32_t n = 0, r = s0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t e = s_tab[r + s_cls[byte_of(v, k)]];
      const bool in = k >= lo && k < hi;
      n += (in && (e & 0x8000u)) ? 1u : 0u;
      r = in ? (e & 0x7FFFu) : r;
    }
    if (!n) return;
    uint32_t at = atomicAdd(A.cand_count, n);
    K2_CTR(1, atomicAdd, n);
    r = s0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t ix = r + s_cls[byte_of(v, k)];
      const uint32_t e = s_tab[ix];
      const bool in = k >= lo && k < hi;
      if (in && (e & 0x8000u)) put(at++, trans(ix), wb + k - fs);
      r = in ? (e & 0x7FFFu) : r;
    }
  }

  // s is a row throughout
  __device__ __forceinline__ uint32_t step(uint32_t s, uint32_t byte, uint64_t pos) {
    const uint32_t ix = s + s_cls[byte];
    const uint32_t e = s_tab[ix];
    if (__builtin_expect(e & 0x8000u, 0)) emit_cand(A, file, trans(ix), pos - fs);
    return e & 0x7FFFu;
  }

  __device__ __forceinline__ uint32_t fast(uint32_t s, uint32_t byte) const { return s_tab[s + s_cls[byte]]; }

  __device__ __forceinline__ void replay16(uint32_t s, const uint4, uint64_t p) {
#pragma unroll 1
    for (uint32_t k = 0; k < 16; k++) s = step(s, A.data[p + k], p + k);
  }

  __device__ __forceinline__ uint32_t step16(uint32_t s, const uint4 v, uint64_t p) {
    const uint32_t s0 = s;
    uint32_t any = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t e = fast(s, byte_of(v, k));
      any |= e;
      s = e & 0x7FFFu;
    }
    if (__builtin_expect(any & 0x8000u, 0)) replay16(s0, v, p);
    return s;
  }

  // matches that started before b: follow them past b (noinject) until they all die
  __device__ K2_NOINLINE void tail(uint32_t s, uint64_t fe, uint64_t b) {
    if (b >= fe) {
      const uint32_t m = d.eot[state_of(s)];
      if (m) emit(m, fe);
      return;
    }
    tail_ni(d.to_ni[state_of(s)], fe, b);
  }
  // the same from the noinject row already looked up (s = to_ni of the chain's row, b < fe)
  __device__ K2_NOINLINE void tail_ni(uint32_t s, uint64_t fe, uint64_t b) {
    const uint8_t* data = A.data;
    const uint8_t* dead = s_cls + (d.o_dead - d.o_cls);  // (staged: stage_dfa)
    // 16 bytes per load (the next word in flight), liveness checked once per word: a dead
    // noinject state is absorbing and accepts nothing, so stepping on inside the word
    // changes no output.  (The batch is padded, so whole-word loads past fe are safe.)
    // Each word is stepped from registers over its bytes in [q, fe); a word with an accepting
    // transition is recorded by accept_word (one record or atomic for the word: tails of a
    // relaxed unbounded rule accept at every byte of a long token).
    uint64_t q = b;
    uint64_t w = q & ~15ull;
    uint4 cur = *(const uint4*)(data + w);
    while (q < fe && !(dead[state_of(s)] & 1)) {
      // past ext_cap, or in a state whose threads never die (the tail would run to the end
      // of the file): the group's rules over the whole file, on the host
      if (q - b >= A.ext_cap || (dead[state_of(s)] & 2)) {
        for (uint32_t k = 0; k < d.nrules; k++) emit_cand(A, file, d.rules[k], kCandWhole);
        return;
      }
      const uint4 nxt = *(const uint4*)(data + w + 16);
      const uint64_t e = min(fe, w + 16);
      const int lo = (int)(q - w), hi = (int)(e - w);
      const uint32_t s0 = s;
      uint32_t any = 0;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const uint32_t t = s_tab[s + s_cls[byte_of(cur, k)]];
        const bool in = k >= lo && k < hi;
        any |= in ? t : 0u;
        s = in ? (t & 0x7FFFu) : s;
      }
      if (__builtin_expect(any & 0x8000u, 0)) accept_word(s0, cur, lo, hi, w);
      q = e;
      cur = nxt;
      w += 16;
    }
    K2_CTR(2, atomicAdd, q - b);
    K2_CTR(3, atomicMax, q - b);
    if (A.diag) {
      const uint32_t n = (uint32_t)min<uint64_t>(q - b, 0xFFFFFFFFull);
      atomicAdd(&A.diag[0], n);
      atomicMax(&A.diag[1], n);
      if (n > 4096) atomicAdd(&A.diag[2], 1u);
    }
    if (q >= fe && !(dead[state_of(s)] & 1)) {
      const uint32_t m = d.eot[state_of(s)];
      if (m) emit(m, fe);
    }
  }

  // NS consecutive chunks [a, a + NS*C) inside file [fs, fe): NS interleaved chains
  template <int NS>
  __device__ void streams(uint64_t fe, uint64_t a, uint32_t C) {
    const uint8_t* data = A.data;
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
          const uint32_t e = fast(s[i], byte_of(cur[i], k));
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
  }

  // one file piece [a, se) of file [fs, fe)
  __device__ void piece(uint64_t fe, uint64_t a, uint64_t se) {
    const uint8_t* data = A.data;
    uint32_t s = (a == fs) ? d.start[0] : d.start[ctx_of(data[a - 1])];
    uint64_t p = a;
    while (p < se && (p & 15)) {
      s = step(s, data[p], p);
      p++;
    }
    if (p + 16 <= se) {
      uint4 cur = *(const uint4*)(data + p);
      while (p + 16 <= se) {
        const uint4 nxt = *(const uint4*)(data + p + 16);
        s = step16(s, cur, p);
        cur = nxt;
        p += 16;
      }
    }
    while (p < se) {
      s = step(s, data[p], p);
      p++;
    }
    tail(s, fe, se);
  }
};

__device__ __forceinline__ void stage_dfa(const DevDFA& d, uint8_t* smem) {
  stage16(smem, d.tab, (d.ns * d.nc + 1) / 2 * 4);
  stage16(smem + d.o_cls, d.cls, 256);
  stage16(smem + d.o_dead, d.dead, d.ns);
  if (d.state_acc) {
    stage16(smem + d.o_accs, d.acc_state, d.ns * 2);
    stage16(smem + d.o_masks, d.masks, d.nmasks * d.mw * 8);
  }
  __syncthreads();
}

// One list entry: up to kEntryItems (file, chunk) items of group d, in rounds of two per
// lane stepped as two interleaved DFA chains.  Items are whole chunks of the batch stream
// (aligned to the chunk size, a multiple of 64).  Bytes of a chunk outside the item's file
// are stepped as no-ops (the file's first byte starts from the start state of its
// context, its end stops the chain).
// A chain keeps 32-bit fields only (the chunk index, not a 64-bit base; the file start is
// reloaded on the rare accept), so the hot loop fits 128 VGPRs: 4 waves per SIMD.
struct K2Item {
  uint32_t s, file;
  uint32_t lo, hi;  // the chunk's bytes inside its file: [base + lo, base + hi)
  uint32_t chunk;   // base = chunk * C
  uint64_t fe;      // the file's end (the tail's bound)
};

template <bool RICH>
__device__ __forceinline__ void k2_list_pair(const DevDFA& d, const K2Args& A, const uint16_t* s_tab,
                                             const uint8_t* s_cls, const uint16_t* s_accs,
                                             const uint64_t* s_masks, uint32_t g, uint32_t first, uint32_t n);

template <bool RICH>
__device__ __forceinline__ void k2_list_entry(const DevDFA& d, const K2Args& A, const uint16_t* s_tab,
                                              const uint8_t* s_cls, const uint16_t* s_accs,
                                              const uint64_t* s_masks, uint4 en) {
  for (uint32_t r0i = 0; r0i < en.z; r0i += 2 * kK2Block)
    k2_list_pair<RICH>(d, A, s_tab, s_cls, s_accs, s_masks, en.x, en.y + r0i, min(en.z - r0i, (uint32_t)(2 * kK2Block)));
}

// items [first, first + n) of an entry, n <= 2 * kK2Block: two per lane.  RICH (the staged
// table already limits the CU to two blocks, so a wave may hold 256 VGPRs): both chains
// stepped in one loop and the next 64-B blocks loaded while the current ones are stepped.
template <bool RICH>
__device__ __forceinline__ void k2_list_pair(const DevDFA& d, const K2Args& A, const uint16_t* s_tab,
                                             const uint8_t* s_cls, const uint16_t* s_accs,
                                             const uint64_t* s_masks, uint32_t g, uint32_t first, uint32_t n) {
  const uint32_t C = A.chunk;
  K2Item it[2];
  bool live[2];
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const uint32_t k = threadIdx.x + (uint32_t)i * kK2Block;
    live[i] = k < n;
    const uint2 item = A.items[first + (live[i] ? k : 0)];
    it[i].file = item.x;
    it[i].chunk = item.y;
    const uint64_t base = (uint64_t)item.y * C;
    // the byte before the chunk, loaded beside the offsets (it is the context byte unless
    // the file starts inside the chunk, and then the start state needs none)
    const uint8_t before = base ? A.data[base - 1] : 0;
    const uint64_t fs = A.off[item.x], fe = A.off[item.x + 1];
    const uint64_t a = max(fs, base);
    it[i].fe = fe;
    it[i].lo = (uint32_t)(a - base);
    it[i].hi = live[i] ? (uint32_t)(min(fe, base + C) - base) : it[i].lo;  // a ghost steps nothing
    it[i].s = a == fs ? d.start[0] : d.start[ctx_of(before)];
  }
  Lane L{d, A, s_tab, s_cls, s_accs, s_masks, 0, 0, g};
  if (C & 127) {  // chunk sizes that are not whole 128-byte lines (tests): lane by lane
#pragma unroll
    for (int i = 0; i < 2; i++)
      if (live[i]) {
        const uint64_t base = (uint64_t)it[i].chunk * C;
        L.file = it[i].file;
        L.fs = A.off[it[i].file];
        L.piece(A.off[it[i].file + 1], base + it[i].lo, base + it[i].hi);
      }
    return;
  }
  // bytes [base + o, base + o + 16) of chain c, stepped where they lie in [lo, hi)
  auto word = [&](K2Item& c, uint32_t o, const uint4 v) __attribute__((always_inline)) {
    const int32_t lo = min(16, max(0, (int32_t)c.lo - (int32_t)o));
    const int32_t hi = min(16, max(0, (int32_t)c.hi - (int32_t)o));
    const uint32_t mask = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
    uint32_t s = c.s, any = 0;
    const uint32_t s0 = s;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t e = s_tab[s + s_cls[byte_of(v, k)]];
      const bool in = (mask >> k) & 1u;
      any |= in ? e : 0u;
      s = in ? (e & 0x7FFFu) : s;
    }
    if (__builtin_expect(any & 0x8000u, 0)) {  // an accept: replay the word, emitting
      if (A.diag) atomicAdd(&A.diag[3], 1u);
      K2_CTR(0, atomicAdd, 1);
      L.file = c.file;
      L.fs = A.off[c.file];
      L.accept_word(s0, v, lo, hi, (uint64_t)c.chunk * C + o);
    }
    c.s = s;
  };
  // both chains in ONE loop: their transition reads issue back to back (RICH)
  auto word2 = [&](uint32_t o, const uint4 v0, const uint4 v1) __attribute__((always_inline)) {
    K2Item& c0 = it[0];
    K2Item& c1 = it[1];
    const int32_t lo0 = min(16, max(0, (int32_t)c0.lo - (int32_t)o)), hi0 = min(16, max(0, (int32_t)c0.hi - (int32_t)o));
    const int32_t lo1 = min(16, max(0, (int32_t)c1.lo - (int32_t)o)), hi1 = min(16, max(0, (int32_t)c1.hi - (int32_t)o));
    const uint32_t m0 = ((1u << hi0) - 1u) & ~((1u << lo0) - 1u), m1 = ((1u << hi1) - 1u) & ~((1u << lo1) - 1u);
    uint32_t s0 = c0.s, s1 = c1.s, any0 = 0, any1 = 0;
    const uint32_t r0 = s0, r1 = s1;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t e0 = s_tab[s0 + s_cls[byte_of(v0, k)]];
      const uint32_t e1 = s_tab[s1 + s_cls[byte_of(v1, k)]];
      const bool in0 = (m0 >> k) & 1u, in1 = (m1 >> k) & 1u;
      any0 |= in0 ? e0 : 0u;
      any1 |= in1 ? e1 : 0u;
      s0 = in0 ? (e0 & 0x7FFFu) : s0;
      s1 = in1 ? (e1 & 0x7FFFu) : s1;
    }
    if (__builtin_expect((any0 | any1) & 0x8000u, 0)) {  // an accept: one record per word
      if (any0 & 0x8000u) {
        if (A.diag) atomicAdd(&A.diag[3], 1u);
        K2_CTR(0, atomicAdd, 1);
        L.file = c0.file;
        L.fs = A.off[c0.file];
        L.accept_word(r0, v0, lo0, hi0, (uint64_t)c0.chunk * C + o);
      }
      if (any1 & 0x8000u) {
        if (A.diag) atomicAdd(&A.diag[3], 1u);
        K2_CTR(0, atomicAdd, 1);
        L.file = c1.file;
        L.fs = A.off[c1.file];
        L.accept_word(r1, v1, lo1, hi1, (uint64_t)c1.chunk * C + o);
      }
    }
    c0.s = s0;
    c1.s = s1;
  };
  K2_PHASE(1);
  // a wave without items steps nothing (an entry's last round leaves ghost lanes whose LDS
  // reads would load the CU for nothing)
  if (__ballot(live[0]) == 0) return;  // (live[1] implies live[0])
  // Quad-transposed loads: the four lanes of a quad fetch 64 contiguous bytes of one lane's
  // chunk per instruction (one 64-B memory request), two DPP stages give each lane its own
  // chunk's four words.  (Each lane loading its own 16-B words, two words ahead, fetched
  // every 64-B sector up to four times: 24 waves per CU keep ~6 MB of lines open per XCD
  // against 4 MB of L2 -- 3.3x K2's item bytes in the FETCH pass and 0.139 against 0.126 ms
  // in the bench, profiles/r05/bench.)
  const uint32_t lane = threadIdx.x & 63, q = lane & 3;
  const bool b0 = q & 1, b1 = (q >> 1) & 1;
  uint4 x0[4], y0[4];
  const uint8_t* dq = A.data + 16u * q;
#define K2_LOAD_T(X, Y, J, T)                                                                 \
  X[T] = *(const uint4*)(dq + (uint64_t)__shfl(it[0].chunk, (int)((lane & ~3u) + T)) * C + (J)); \
  Y[T] = *(const uint4*)(dq + (uint64_t)__shfl(it[1].chunk, (int)((lane & ~3u) + T)) * C + (J));
#define K2_LOAD(X, Y, J) \
  K2_LOAD_T(X, Y, J, 0)  \
  K2_LOAD_T(X, Y, J, 1)  \
  K2_LOAD_T(X, Y, J, 2)  \
  K2_LOAD_T(X, Y, J, 3)
#define K2_BLOCK(X, Y, J)                                                       \
  quad_transpose4(X, b0, b1);                                                   \
  quad_transpose4(Y, b0, b1);                                                   \
  _Pragma("unroll") for (int w = 0; w < 4; w++) {                              \
    word(it[0], (uint32_t)(J) + 16u * w, X[w]);                                 \
    word(it[1], (uint32_t)(J) + 16u * w, Y[w]);                                 \
  }
  if constexpr (RICH) {
#define K2_BLOCK2(X, Y, J)                                                      \
  quad_transpose4(X, b0, b1);                                                   \
  quad_transpose4(Y, b0, b1);                                                   \
  _Pragma("unroll") for (int w = 0; w < 4; w++) word2((uint32_t)(J) + 16u * w, X[w], Y[w]);
    uint4 x1[4], y1[4];
    K2_LOAD(x0, y0, 0)
    // two 64-B blocks per chain in registers: block j + 64 loads while block j steps
    for (uint32_t j = 0; j < C; j += 128) {
      if (j + 64 < C) {
        K2_LOAD(x1, y1, j + 64)
      }
      K2_BLOCK2(x0, y0, j)
      if (j + 64 >= C) break;
      if (j + 128 < C) {
        K2_LOAD(x0, y0, j + 128)
      }
      K2_BLOCK2(x1, y1, j + 64)
    }
#undef K2_BLOCK2
  } else {
    K2_LOAD(x0, y0, 0)
    // one 64-B block per chain, stepped in place, then reloaded
    for (uint32_t j = 0; j < C; j += 64) {
      K2_BLOCK(x0, y0, j)
      if (j + 64 < C) {
        K2_LOAD(x0, y0, j + 64)
      }
    }
  }
#undef K2_LOAD_T
#undef K2_LOAD
#undef K2_BLOCK
  K2_PHASE(2);
  // matches that started in the chunk and run past it (inside the file): follow them.  The
  // noinject rows of both chains are looked up together, the file ends kept from the setup.
  uint32_t ni[2];
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const uint64_t b = (uint64_t)it[i].chunk * C + it[i].hi;
    ni[i] = live[i] && b < it[i].fe ? d.to_ni[L.state_of(it[i].s)] : 0u;
  }
#pragma unroll
  for (int i = 0; i < 2; i++)
    if (live[i]) {
      const uint64_t b = (uint64_t)it[i].chunk * C + it[i].hi;
      L.file = it[i].file;
      L.fs = A.off[it[i].file];
      if (b < it[i].fe)
        L.tail_ni(ni[i], it[i].fe, b);
      else
        L.tail(it[i].s, it[i].fe, b);
    }
  K2_PHASE(3);
}

// One dense entry: chunks [first, first + n) of the batch, kStreams consecutive chunks per
// lane, every file piece scanned where the group is gated for its file.
__device__ __forceinline__ void k2_dense_entry(const DevDFA& d, const K2Args& A, uint32_t g, const uint16_t* s_tab,
                                               const uint8_t* s_cls, const uint16_t* s_accs,
                                               const uint64_t* s_masks, uint4 en) {
  Lane L{d, A, s_tab, s_cls, s_accs, s_masks, 0, 0, g};
  const uint32_t* gm = A.gmask + (size_t)g * A.kw_words;
  const uint32_t always = A.galways[g];
  const uint64_t c0 = en.y + (uint64_t)threadIdx.x * kStreams;
  if (c0 >= (uint64_t)en.y + en.z) return;
  uint64_t a = c0 * A.chunk;
  const uint64_t b = min((c0 + kStreams) * A.chunk, A.total);
  uint32_t f = file_of(A.cf, A.off, A.nfiles, a);
  {
    const uint64_t fs = A.off[f], fe = A.off[f + 1];
    if (b == a + (uint64_t)kStreams * A.chunk && a >= fs && b <= fe) {  // common case: one file
      if (group_gated(A.kw + (size_t)f * A.kw_words, gm, A.kw_words, always)) {
        L.file = f;
        L.fs = fs;
        L.template streams<kStreams>(fe, a, A.chunk);
      }
      return;
    }
  }
  while (a < b) {
    const uint64_t fs = A.off[f], fe = A.off[f + 1];
    if (fe <= a) {
      f++;
      continue;
    }
    const uint64_t se = min(b, fe);
    if (group_gated(A.kw + (size_t)f * A.kw_words, gm, A.kw_words, always)) {
      L.file = f;
      L.fs = fs;
      L.piece(fe, a, se);
    }
    a = se;
    f++;
  }
}

// K2: persistent grids over the work lists.  Blocks claim entries dynamically (one
// atomic per entry), so blocks that drew light entries take more; a block restages the
// DFA only when its next entry belongs to another group.
template <bool DENSE, bool RICH = false>
__device__ __forceinline__ void k2_run(const DevDFA* __restrict__ dfas, const K2Args& A, const uint4* entries,
                                       uint32_t E, uint32_t* claim, uint8_t* smem) {
  __shared__ uint32_t s_e;
  uint32_t staged = 0xFFFFFFFFu;
  uint32_t prev = 0xFFFFFFFFu;  // the entry this block ran last (trace)
#ifdef K2_TRACE_CTR
  if (threadIdx.x == 0) s_ectr = nullptr;
#endif
#ifdef K2_TRACE_PHASE
  if (threadIdx.x == 0) s_tph = nullptr;
#endif
  // An empty list (the dense pass, usually) ends the block without a claim: 512 blocks'
  // returning atomics on one address took ~10 us of an empty launch.  (A plain load of the
  // claim counter before each atomic, to skip the claims past the list's end, made the
  // list pass 0.110 -> 0.145 ms per GiB: loads and atomics on the counters' line, which
  // also holds the candidate counter, profiles/r06/k2p.)
  if (E == 0) return;
  bool ran = false;  // (the end stamp: only a block that ran an entry)
  for (;;) {
    if (threadIdx.x == 0) s_e = atomicAdd(claim, 1u);
    __syncthreads();
    const uint32_t e = s_e;
    __syncthreads();  // every lane has read s_e (and is done with the previous entry)
    if (!DENSE && A.etrace && threadIdx.x == 0) {  // trace: the previous entry ends, this one starts
      const unsigned long long now = wall_clock64();
      if (prev != 0xFFFFFFFFu) A.etrace[(size_t)prev * kTraceW + 1] = now;
      if (e < E) {
        const uint4 en = entries[e];
        A.etrace[(size_t)e * kTraceW + 0] = now;
        A.etrace[(size_t)e * kTraceW + 2] = ((unsigned long long)en.x << 32) | en.z;
        A.etrace[(size_t)e * kTraceW + 3] = ((unsigned long long)__builtin_amdgcn_s_getreg(20 | (15 << 11)) << 32) |
                                            (uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11));
#ifdef K2_TRACE_CTR
        s_ectr = A.etrace + (size_t)e * kTraceW + 4;
#endif
#ifdef K2_TRACE_PHASE
        s_tph = A.etrace + (size_t)e * kTraceW + 4;
#endif
      }
    }
#if defined(K2_TRACE_CTR) || defined(K2_TRACE_PHASE)
    __syncthreads();
#endif
    prev = e;
    if (e >= E) {
      if (ran && threadIdx.x == 0) atomicMax(&A.clk[3], (unsigned long long)wall_clock64());
      break;
    }
    ran = true;
    const uint4 en = entries[e];
    const uint32_t g = __builtin_amdgcn_readfirstlane(en.x);
    const DevDFA& d = dfas[g];  // (a reference: uniform fields load into SGPRs, no copy)
    if (g != staged) {
      stage_dfa(d, smem);
      staged = g;
    }
    K2_PHASE(0);
    const uint16_t* s_tab = (const uint16_t*)smem;
    if (DENSE)
      k2_dense_entry(d, A, g, s_tab, smem + d.o_cls, (const uint16_t*)(smem + d.o_accs), (const uint64_t*)(smem + d.o_masks), en);
    else
      k2_list_entry<RICH>(d, A, s_tab, smem + d.o_cls, (const uint16_t*)(smem + d.o_accs), (const uint64_t*)(smem + d.o_masks), en);
  }
}

__global__ void __launch_bounds__(kK2Block) K2_WAVES k2_kernel(const DevDFA* __restrict__ dfas, K2Args A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  k2_run<false>(dfas, A, A.entries, *A.nentries, A.claim, smem);
}
// the list pass when the staged table allows two blocks per CU at most (> 53 KiB): eight
// waves per CU, so each may hold 256 VGPRs (k2_list_pair<true>)
__global__ void __launch_bounds__(kK2Block) __attribute__((amdgpu_waves_per_eu(1, 2)))
k2_kernel_rich(const DevDFA* __restrict__ dfas, K2Args A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  k2_run<false, true>(dfas, A, A.entries, *A.nentries, A.claim, smem);
}

__global__ void __launch_bounds__(kBlock) k2_dense_kernel(const DevDFA* __restrict__ dfas, K2Args A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  k2_run<true>(dfas, A, A.dentries, *A.ndentries, A.claim + 1, smem);
}

// ---------------------------------------------------------------- host side
template <class T>
static int upload_vec(const std::vector<T>& v, const T** dst, std::vector<void*>* allocs) {
  void* p = nullptr;
  // whole 16-B units, zero padded: the kernels stage tables with 16-B loads (stage16)
  const size_t bytes = (std::max<size_t>(v.size() * sizeof(T), 16) + 15) & ~(size_t)15;
  HIP_TRY(hipMalloc(&p, bytes));
  HIP_TRY(hipMemset(p, 0, bytes));
  if (!v.empty()) HIP_TRY(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  allocs->push_back(p);
  *dst = (const T*)p;
  return TSG_OK;
}

static uint32_t align16(uint32_t x) { return (x + 15) & ~15u; }

static int make_device_dfa(const DFA& dd, const std::vector<uint32_t>& rules, DevDFA* out,
                           std::vector<void*>* allocs) {
  if (dd.nstates >= 0x8000) return fail(TSG_ERR_INTERNAL, "DFA too large for u16 tables");
  out->nrules = (uint32_t)rules.size();
  // rows of at least 2 entries (state_of's reciprocal needs nc >= 2): a one-class DFA gets a
  // duplicate column no byte maps to
  DFA padded;
  const DFA* dp = &dd;
  if (dd.nclasses < 2) {
    padded = dd;
    padded.nclasses = 2;
    padded.next.clear();
    padded.acc.clear();
    for (int st = 0; st < dd.nstates; st++)
      for (int c = 0; c < 2; c++) {
        padded.next.push_back(dd.next[st]);
        padded.acc.push_back(dd.acc[st]);
      }
    dp = &padded;
  }
  const DFA& d = *dp;
  const size_t nc = d.nclasses;
  std::vector<uint16_t> tab((size_t)d.nstates * nc), acc(tab.size()), accs(d.nstates, 0);
  bool state_acc = true;
  if ((size_t)(d.nstates - 1) * nc >= 0x8000) return fail(TSG_ERR_INTERNAL, "DFA rows do not fit 15 bits");
  for (int s = 0; s < d.nstates; s++) {
    uint32_t a0 = d.acc[(size_t)s * nc];
    for (size_t c = 0; c < nc; c++) {
      size_t i = (size_t)s * nc + c;
      if (d.acc[i] > 0xFFFF) return fail(TSG_ERR_INTERNAL, "too many accept masks");
      tab[i] = (uint16_t)((d.next[i] * nc) | (d.acc[i] ? 0x8000u : 0u));
      acc[i] = (uint16_t)d.acc[i];
      if (d.acc[i] != a0) state_acc = false;
    }
    accs[s] = (uint16_t)a0;
  }
  std::vector<uint16_t> eot(d.nstates), ni(d.nstates);
  for (int s = 0; s < d.nstates; s++) {
    eot[s] = (uint16_t)d.eot_acc[s];
    ni[s] = (uint16_t)(d.to_noinject[s] * nc);
  }
  std::vector<uint8_t> dead(d.nstates);
  for (int s = 0; s < d.nstates; s++)
    dead[s] = (d.dead[s] ? 1 : 0) | ((size_t)s < d.immortal.size() && d.immortal[s] ? 2 : 0);
  std::vector<uint64_t> masks;
  for (const auto& m : d.masks) masks.insert(masks.end(), m.begin(), m.end());
  std::vector<uint8_t> cls(d.cls, d.cls + 256);
  std::vector<uint16_t> tabp = tab;
  if (tabp.size() & 1) tabp.push_back(0);  // the kernels stage whole dwords
  DevDFA& v = *out;
  int rc;
  if ((rc = upload_vec(tabp, &v.tab, allocs))) return rc;
  if ((rc = upload_vec(acc, &v.acc, allocs))) return rc;
  if ((rc = upload_vec(accs, &v.acc_state, allocs))) return rc;
  if ((rc = upload_vec(eot, &v.eot, allocs))) return rc;
  if ((rc = upload_vec(ni, &v.to_ni, allocs))) return rc;
  if ((rc = upload_vec(dead, &v.dead, allocs))) return rc;
  if ((rc = upload_vec(masks, &v.masks, allocs))) return rc;
  if ((rc = upload_vec(cls, &v.cls, allocs))) return rc;
  if ((rc = upload_vec(rules, &v.rules, allocs))) return rc;
  v.nc = (uint32_t)nc;
  v.ns = (uint32_t)d.nstates;
  v.mw = (uint32_t)d.mask_words;
  v.nmasks = (uint32_t)d.masks.size();
  for (int k = 0; k < 4; k++) v.start[k] = d.start[k] * (uint32_t)nc;
  v.inv_nc = (uint32_t)((0x100000000ull + nc - 1) / nc);
  // LDS layout
  uint32_t o = align16((uint32_t)(tab.size() * 2));
  v.o_cls = o;
  o += 256;
  v.o_dead = o;  // the tails' per-word liveness test reads it
  o += align16((uint32_t)d.nstates);
  v.o_accs = o;
  v.o_masks = o;
  v.state_acc = 0;
  const uint32_t acc_bytes = align16(d.nstates * 2) + align16((uint32_t)masks.size() * 8);
  if (state_acc && o + acc_bytes + 16 * 1024 <= 150 * 1024) {
    v.state_acc = 1;
    v.o_masks = o + align16(d.nstates * 2);
    o += acc_bytes;
  }
  v.lds_bytes = o + 16;
  if (v.lds_bytes > 160 * 1024) return fail(TSG_ERR_INTERNAL, "DFA tables exceed LDS");
  return TSG_OK;
}

// perf experiments only (results are not exact): bit 0 strips the K1 accept flags
struct K1Host {  // host copies of the K1 tables (adaptation rebuilds the device table)
  std::vector<uint16_t> tab, accs;
  std::vector<uint32_t> masks;
  std::vector<uint32_t> order;  // device state id -> automaton state
  uint32_t stride = 0;          // row stride of tab (>= the class count)
  uint32_t unit = 1;            // row of state id = id * stride * unit (packed: 2, bytes)
};

// K1 LDS class of a legacy transition table of tab_bytes (2 * the class count for the REP
// layout, preferred; 3 = too large)
static int k1_lds_class(size_t tab_bytes) {
  for (int k = 0; k < 3; k++)
    if (tab_bytes + kK1RepBytes <= (size_t)kK1Lds[k] * 1024) return 2 * k + 1;
  return tab_bytes + 1024 <= (size_t)kK1Lds[2] * 1024 ? 2 * 2 : 2 * 3;
}

// the packed layout holds rows as 16-bit byte offsets: ns * stride u16 entries in 64 KiB
static bool k1_packed_fits(size_t ns, size_t rs) {
#ifdef K1_LEGACY  // measurement builds: the legacy layout for every automaton
  (void)ns;
  (void)rs;
  return false;
#else
  return ns * rs * 2 <= 65536;
#endif
}

// Row stride (u16 entries) of the K1 table: the class count padded to 2 mod 4, so a row is
// an odd number of dwords and equal classes of different rows fall in different LDS banks
// (ds_read_u16 banks are dword mod 32).  Padding is skipped when it would change the
// layout (packed -> legacy, or a larger legacy LDS image) or overflow the 16-bit rows.
static size_t k1_stride(size_t nc, size_t ns) {
  size_t rs = nc;
  while (rs % 4 != 2) rs++;
  auto tab = [&](size_t r) { return (ns * r + (ns * r & 1)) * 2; };
  if (k1_packed_fits(ns, nc)) return k1_packed_fits(ns, rs) ? rs : nc;
  if ((ns - 1) * rs > 0xFFFF || k1_lds_class(tab(rs)) != k1_lds_class(tab(nc))) return nc;
  return rs;
}

// Device numbering of the K1 automaton: states whose arrival is reported (they end a
// literal, and are not `quiet`) last; rows = id * stride * unit.
static int k1_tables(const Plan& p, const std::vector<uint8_t>& quiet, K1Host* h, uint32_t* start_row,
                     uint32_t* acc_row) {
  const DFA& d = *p.kw_dfa;
  const size_t nc = d.nclasses, ns = d.nstates;
  const size_t rs = k1_stride(nc, ns);
  h->stride = (uint32_t)rs;
  h->unit = k1_packed_fits(ns, rs) ? 2 : 1;
  const size_t row = rs * h->unit;
  if ((ns - 1) * row > 0xFFFF) return fail(TSG_ERR_INTERNAL, "keyword automaton too large for 16-bit rows");
  std::vector<uint32_t> newid(ns);
  h->order.clear();
  for (int pass = 0; pass < 2; pass++)
    for (size_t st = 0; st < ns; st++) {
      const bool rep = d.eot_acc[st] && !quiet[st];
      if (rep == (pass == 1)) {
        newid[st] = (uint32_t)h->order.size();
        h->order.push_back((uint32_t)st);
      }
    }
  uint32_t first_rep = (uint32_t)ns;
  for (size_t i = 0; i < ns; i++) {
    const uint32_t st = h->order[i];
    if (d.eot_acc[st] && !quiet[st]) {
      first_rep = (uint32_t)i;
      break;
    }
  }
  h->tab.assign(ns * rs + (ns * rs & 1), 0);  // the kernel stages whole dwords
  h->accs.assign(ns, 0);
  for (size_t i = 0; i < ns; i++) {
    const uint32_t st = h->order[i];
    h->accs[i] = (uint16_t)d.eot_acc[st];
    for (size_t c = 0; c < nc; c++) h->tab[i * rs + c] = (uint16_t)(newid[d.next[st * nc + c]] * row);
  }
  *start_row = newid[d.start[kCtxBOT]] * (uint32_t)row;
  *acc_row = first_rep * (uint32_t)row;
  return TSG_OK;
}

// K1X tables: the 4-gram bitmap, the 4-gram -> {literal, offset} table and the literals
static int make_device_k1x(const Plan& p, DevK1X* out, std::vector<void*>* allocs) {
  *out = DevK1X{};
  out->kw_words = (uint32_t)p.kw_words;
  out->step = (uint32_t)p.x_step;
  if (p.x_lits.empty()) return TSG_OK;
  if (p.x_step != 1 && p.x_step != 2 && p.x_step != 4) return fail(TSG_ERR_INTERNAL, "K1X step not 1, 2 or 4");
  const size_t n = p.x_lits.size();
  std::vector<uint32_t> bitmap(kXDwords, 0);
  std::map<uint32_t, std::vector<uint32_t>> by4;
  std::vector<uint8_t> bytes;
  std::vector<uint32_t> off(n), len(n), ev(n);
  std::vector<int32_t> kwid(n);
  if (n >= (1u << 24) || p.x_j0.size() != n) return fail(TSG_ERR_INTERNAL, "bad K1X literal table");
  for (size_t i = 0; i < n; i++) {
    const std::string& L = p.x_lits[i];
    const uint32_t j0 = p.x_j0[i];
    if (L.size() < j0 + (size_t)p.x_step + 3 || j0 + p.x_step > 256)
      return fail(TSG_ERR_INTERNAL, "K1X literal shorter than its windows");
    for (uint32_t j = j0; j < j0 + (uint32_t)p.x_step; j++) {  // an occurrence at s is sampled at one s + j
      const uint32_t w = x_prefix4((const uint8_t*)L.data() + j);
      const uint32_t h = x_hash(x_fold(w));
      bitmap[x_dword(h)] |= x_bits(h);
      by4[w].push_back((uint32_t)i | j << 24);
    }
    off[i] = (uint32_t)bytes.size();
    len[i] = (uint32_t)L.size();
    bytes.insert(bytes.end(), L.begin(), L.end());
    bytes.resize((bytes.size() + 3) / 4 * 4, 0);
    ev[i] = p.x_event[i];
    kwid[i] = p.x_kw[i];
  }
  uint32_t nslots = 16, lg = 4;
  while (nslots < 2 * by4.size()) {
    nslots *= 2;
    lg++;
  }
  std::vector<uint4> slots(nslots, make_uint4(0, 0, 0, 0));
  std::vector<uint32_t> lits;
  for (const auto& kv : by4) {
    uint32_t h = (kv.first * 0x85EBCA6Bu) >> (32 - lg);
    while (slots[h].z) h = (h + 1) & (nslots - 1);
    slots[h] = make_uint4(kv.first, (uint32_t)lits.size(), (uint32_t)kv.second.size(), 0);
    lits.insert(lits.end(), kv.second.begin(), kv.second.end());
  }
  int rc;
  if ((rc = upload_vec(bitmap, &out->bitmap, allocs))) return rc;
  // the verify tables as one image: slots | lits | off | len | kwid | ev | bytes
  std::vector<uint8_t> img;
  auto part = [&](const void* src, size_t n) {
    const size_t at = img.size();
    img.resize((at + n + 15) / 16 * 16, 0);
    if (n) std::memcpy(img.data() + at, src, n);
    return at;
  };
  const size_t o_slots = part(slots.data(), slots.size() * sizeof(uint4));
  const size_t o_lits = part(lits.data(), lits.size() * 4);
  const size_t o_off = part(off.data(), off.size() * 4);
  const size_t o_len = part(len.data(), len.size() * 4);
  const size_t o_kwid = part(kwid.data(), kwid.size() * 4);
  const size_t o_ev = part(ev.data(), ev.size() * 4);
  const size_t o_bytes = part(bytes.data(), bytes.size());
  if (img.size() > 0xFFFFFFFFu) return fail(TSG_ERR_INTERNAL, "K1X tables too large");
  const uint8_t* dimg = nullptr;
  if ((rc = upload_vec(img, &dimg, allocs))) return rc;
  out->img = dimg;
  out->img_bytes = (uint32_t)img.size();
  out->slots = (const uint4*)(dimg + o_slots);
  out->lits = (const uint32_t*)(dimg + o_lits);
  out->off = (const uint32_t*)(dimg + o_off);
  out->len = (const uint32_t*)(dimg + o_len);
  out->kwid = (const int32_t*)(dimg + o_kwid);
  out->ev = (const uint32_t*)(dimg + o_ev);
  out->bytes = dimg + o_bytes;
  out->mask = nslots - 1;
  out->shift = 32 - lg;
  return TSG_OK;
}

static int make_device_k1(const Plan& p, DevK1* out, std::vector<void*>* allocs, K1Host* host) {
  const DFA& d = *p.kw_dfa;
  const size_t nc = d.nclasses;
  if (nc > 128) return fail(TSG_ERR_INTERNAL, "keyword automaton has too many classes");
  for (int st = 0; st < d.nstates; st++)
    for (size_t c = 0; c < nc; c++)
      if (d.acc[(size_t)st * nc + c] != d.eot_acc[st])
        return fail(TSG_ERR_INTERNAL, "keyword automaton accepts are not state-based");
  DevK1& v = *out;
  int rc;
  if ((rc = k1_tables(p, std::vector<uint8_t>(d.nstates, 0), host, &v.start, &v.acc_row))) return rc;
  v.packed = host->unit == 2 ? 1u : 0u;
  std::vector<uint32_t> cls(256), pcls(512);
  for (int b = 0; b < 256; b++) {
    cls[b] = (uint32_t)d.cls[b] * 2 | ((p.run_cls[b] & 2) ? 0xFF00u : 0u) | ((p.run_cls[b] & 1) ? 0xFFFF0000u : 0u);
    pcls[2 * b] = (uint32_t)d.cls[b] * 2 + kK1PTab;
    pcls[2 * b + 1] = ((p.run_cls[b] & 2) ? 1u : 0u) | ((p.run_cls[b] & 1) ? 1u << 16 : 0u);
  }
  const uint32_t W = (uint32_t)p.kw_words, mw = W + 1;
  std::vector<uint32_t> masks((size_t)d.masks.size() * mw, 0);
  for (size_t m = 0; m < d.masks.size(); m++) {
    for (int k = 0; k < p.n_kw; k++)
      if ((d.masks[m][k / 64] >> (k % 64)) & 1) masks[m * mw + k / 32] |= 1u << (k % 32);
    masks[m * mw + W] = p.kw_mask_events[m];
  }
  if ((rc = upload_vec(host->tab, &v.tab, allocs))) return rc;
  if ((rc = upload_vec(cls, &v.cls, allocs))) return rc;
  if ((rc = upload_vec(pcls, &v.pcls, allocs))) return rc;
  if ((rc = upload_vec(host->accs, &v.accs, allocs))) return rc;
  if ((rc = upload_vec(masks, &v.masks, allocs))) return rc;
  v.nc = host->stride;  // the kernel's row stride
  v.row_unit = host->stride * host->unit;
  v.tab_words = (uint32_t)(host->tab.size() / 2);
  v.ns = (uint32_t)d.nstates;
  v.nmasks = (uint32_t)d.masks.size();
  v.mw = mw;
  v.kw_words = W;
  v.warm = (uint32_t)p.warm;
  v.kU = (uint32_t)p.run_k[0];
  v.kD = v.packed ? (uint32_t)p.run_k[1] : (uint32_t)p.run_k[1] << 8;
  std::vector<uint16_t> kwlen((size_t)W * 32, 0);
  v.kw_maxlen = 1;
  for (int k = 0; k < p.n_kw; k++) {
    kwlen[k] = p.kw_len[k];
    v.kw_maxlen = std::max<uint32_t>(v.kw_maxlen, p.kw_len[k]);
  }
  if ((rc = upload_vec(kwlen, &v.kw_len, allocs))) return rc;
  host->masks = masks;
  const int lc = k1_lds_class(host->tab.size() * 2);
  v.lds_class = (uint32_t)(lc >> 1);
  v.rep = (uint32_t)(lc & 1);
  if (!v.packed && v.lds_class > 2) return fail(TSG_ERR_INTERNAL, "keyword automaton exceeds LDS");
  return TSG_OK;
}

// ---------------------------------------------------------------- rule tables on a device
struct DeviceRules {
  uint32_t all_kw_rows = 0;  // the plan has host-only rules: the host reads every keyword row
  int device = 0;
  const Plan* plan = nullptr;
  uint32_t chunk = 256, ext_cap = 1u << 16, adapt_mib = 0;
  int grid = 0;          // 8 blocks per CU
  int cus = 0;
  int k2_grid = 0, k2_dense_grid = 0;  // resident blocks of the persistent K2 kernels
  bool k2_rich = false;                 // the list pass runs k2_kernel_rich (same residency)
  hipEvent_t kernels_done = nullptr;   // end of the kernels of the last enqueued batch
  bool kernels_done_valid = false;
  std::vector<void*> tables;
  DevK1 k1{};
  K1Host k1h;
  DevK1X k1x{};
  bool has_k1x = false;
  bool use_k1f = false;  // K1 is the filter-and-verify K1F (k1f.hpp), else the automaton
  uint32_t k1f_maxlen = 4;  // longest K1F literal (its event list's zone)
  DevK1F k1f{};
  K1FTables k1ft;        // host copy (the adaptation rebuilds it)
  uint32_t* d_fhits = nullptr;  // [n_lit] K1F sampling counters
  uint32_t* d_hits = nullptr;
  bool adapted = false;
  uint32_t hot_states = 0;
  std::shared_ptr<const std::vector<uint8_t>> kw_unknown;
  std::vector<uint32_t> h_galways, h_gevents;
  std::vector<unsigned long long> h_gofbit;
  std::vector<DevDFA> groups;
  DevDFA* d_groups = nullptr;
  uint32_t* d_gmask = nullptr;
  uint32_t* d_galways = nullptr;
  unsigned long long* d_kwg = nullptr;   // [n_kw * GW] groups each keyword bit gates
  unsigned long long* d_galw = nullptr;  // [GW] always-gated groups (d_galways as bits)
  uint32_t* d_gevents = nullptr;
  uint32_t* d_gback = nullptr;
  unsigned long long* d_gofbit = nullptr;
  std::vector<uint32_t> gback;
  uint32_t GW = 1, maxback = 0, max_lds = 0;
  ~DeviceRules() {
    (void)hipSetDevice(device);
    if (kernels_done) (void)hipEventDestroy(kernels_done);
    for (auto* p : tables) (void)hipFree(p);
    (void)hipFree(d_hits);
    (void)hipFree(d_fhits);
  }
};

// HBM buffers, stream and events of one lane (one batch in flight on the device).
struct LaneState {
  DeviceRules* d = nullptr;
  hipStream_t st = nullptr;
  uint8_t* data_alloc = nullptr;  // kPad | batch | tail
  size_t data_cap = 0;
  uint8_t* meta = nullptr;        // the batch's file offsets (one H2D per batch)
  size_t meta_cap = 0;
  const uint64_t* off = nullptr;  // into meta (last batch)
  uint32_t* cf = nullptr;         // coarse file map (file_of)
  size_t cf_cap = 0;
  uint32_t* ev_bits = nullptr;
  size_t ev_cap = 0;
  uint2* xlist = nullptr;  // K1X hit records
  size_t xlist_cap = 0;
  uint32_t* xcount = nullptr;  // K1X records per block
  size_t xcount_cap = 0;
  uint32_t* evlist = nullptr;
  size_t evlist_cap = 0;
  uint32_t* zclaim = nullptr;  // K1F's zone claims (K1FArgs::claim): a bit per chunk
  size_t zclaim_cap = 0;
  unsigned long long* wtrace = nullptr;  // K1F's per-wave trace (TSG_K1F_TRACE)
  size_t wtrace_cap = 0, wtrace_n = 0;
  uint32_t* kw = nullptr;
  size_t kw_cap = 0;
  unsigned long long* ggate = nullptr;
  size_t ggate_cap = 0;
  uint8_t* ovf = nullptr;
  size_t ovf_cap = 0;
  uint8_t* hascand = nullptr;
  size_t hascand_cap = 0;
  uint2* items = nullptr;
  size_t items_cap = 0;
  uint4* entries = nullptr;
  size_t entries_cap = 0;
  uint4* dentries = nullptr;
  size_t dentries_cap = 0;
  DevCand* cand = nullptr;
  uint32_t cand_cap = 0;
  uint32_t* counts = nullptr;   // [16] 0 candidates, 1 event chunks, 2 K2 entries, ...
  uint32_t* gcount = nullptr;   // [G]
  uint32_t* bcount = nullptr;   // [grid * G] items_count_kernel's per-block counts
  uint32_t* cursor = nullptr;   // [G]
  uint8_t* gskip = nullptr;     // [G]
  unsigned long long* etrace = nullptr;  // [entries_cap * kTraceW] K2 entry trace (TSG_K2_TRACE)
  size_t etrace_cap = 0;
  uint64_t nchunks = 0;         // last batch
  ~LaneState() {
    if (!d) return;
    (void)hipSetDevice(d->device);
    if (st) (void)hipStreamSynchronize(st);
    void* bufs[] = {data_alloc, meta, cf, ev_bits, xlist, xcount, evlist, zclaim, wtrace, kw, ggate, ovf, hascand,
                    items, entries, dentries, cand, counts, gcount, bcount, cursor, gskip, etrace};
    for (void* b : bufs) (void)hipFree(b);
    if (st) (void)hipStreamDestroy(st);
  }
};

template <class T>
static int ensure(T** p, size_t* cap, size_t n) {
  if (*cap >= n && *p) return TSG_OK;
  if (*p) HIP_TRY(hipFree(*p));  // (hipFree waits for the device)
  *p = nullptr;
  const size_t alloc = std::max<size_t>(n + n / 8, 16);
  HIP_TRY(hipMalloc((void**)p, (alloc * sizeof(T) + 15) & ~(size_t)15));
  *cap = alloc;
  return TSG_OK;
}

template <bool PACKED, int LDSK, bool REP, int TPB>
static const void* k1_fn_w(uint32_t kw_words) {
  if (kw_words <= 1) return (const void*)k1_kernel<1, PACKED, LDSK, REP, TPB>;
  if (kw_words <= 2) return (const void*)k1_kernel<2, PACKED, LDSK, REP, TPB>;
  if (kw_words <= 4) return (const void*)k1_kernel<4, PACKED, LDSK, REP, TPB>;
  return (const void*)k1_kernel<8, PACKED, LDSK, REP, TPB>;
}

// the kernel of a layout and its block size / blocks per CU
static const void* k1_fn(const DevK1& k, int* threads, int* per_cu) {
  if (k.packed) {
    *threads = 1024;
    *per_cu = 1;
    return k1_fn_w<true, kK1PLdsK, true, 1024>(k.kw_words);
  }
  const uint32_t lc = std::min<uint32_t>(k.lds_class, 2);
  *threads = k1_threads(kK1Lds[lc]);
  *per_cu = kK1BlocksPerCU[lc];
  switch (lc) {
    case 0: return k1_fn_w<false, kK1Lds[0], true, k1_threads(kK1Lds[0])>(k.kw_words);
    case 1: return k1_fn_w<false, kK1Lds[1], true, k1_threads(kK1Lds[1])>(k.kw_words);
    default:
      return k.rep ? k1_fn_w<false, kK1Lds[2], true, k1_threads(kK1Lds[2])>(k.kw_words)
                   : k1_fn_w<false, kK1Lds[2], false, k1_threads(kK1Lds[2])>(k.kw_words);
  }
}

// a persistent grid of the resident blocks (each block stages the automaton once)
static int launch_k1(DeviceRules* r, const K1Args& A, hipStream_t st) {
  int threads = 0, per_cu = 0;
  const void* fn = k1_fn(r->k1, &threads, &per_cu);
  const uint64_t cap = (uint64_t)r->cus * per_cu;
  const int grid = (int)std::min<uint64_t>((A.nitems + threads - 1) / threads, cap);
  DevK1 d = r->k1;
  K1Args a = A;
  void* args[] = {&d, &a};
  HIP_TRY(hipLaunchKernel(fn, dim3(grid), dim3(threads), args, 0, st));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipGetLastError());
  return TSG_OK;
}

// K1 adaptation (once per device, on the first large batch): a sampling pass counts the
// arrivals in every accepting state; the most frequent states stop raising the accept
// flag until the rest arrive at most once per 4 KiB.  The literals those states end are
// then unknown per file: their keyword gates open (the host checks them exactly), their
// anchor events fire everywhere.  Results are unchanged; K1 stops paying per-occurrence
// accepts for words like "key" that occur in most files anyway.  The device is idle
// while the shared tables change (every lane is synchronized first).
static int apply_unknown(DeviceRules* r, const std::shared_ptr<std::vector<uint8_t>>& kw_unknown, uint32_t ev_hot);
static int adapt_k1(DeviceRules* r, LaneState* l, uint64_t total, uint32_t nfiles, uint64_t nchunks, uint64_t k1_items) {
  const Plan& p = *r->plan;
  HIP_TRY(hipDeviceSynchronize());
  const uint32_t ns = r->k1.ns, W = r->k1.kw_words, mw = r->k1.mw;
  const uint64_t step = std::max<uint64_t>(1, k1_items / 16384);
  const uint64_t nsamp = (k1_items + step - 1) / step;
  HIP_TRY(hipMemsetAsync(r->d_hits, 0, sizeof(uint32_t) * ns, l->st));
  K1Args A{l->data_alloc + kPad, l->off, l->cf, total, nchunks, nsamp, step, r->chunk,
           nfiles, l->kw, l->ev_bits, r->d_hits, (uint32_t)kK1Seg};
  int rc;
  if ((rc = launch_k1(r, A, l->st))) return rc;
  std::vector<uint32_t> hits(ns);
  HIP_TRY(hipMemcpyAsync(hits.data(), r->d_hits, sizeof(uint32_t) * ns, hipMemcpyDeviceToHost, l->st));
  HIP_TRY(hipStreamSynchronize(l->st));
  r->adapted = true;
  const uint64_t sample_bytes = nsamp * kK1Chains * A.seg * r->chunk;
  uint64_t tot = 0;
  std::vector<uint32_t> order;
  for (uint32_t s = 0; s < ns; s++)
    if (hits[s]) {
      tot += hits[s];
      order.push_back(s);
    }
  std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return hits[a] > hits[b]; });
  const uint64_t budget = sample_bytes / 4096;  // reporting budget: one arrival per 4 KiB
  std::vector<uint8_t> hot(p.kw_dfa->nstates, 0);  // automaton states that stop reporting
  auto kw_unknown = std::make_shared<std::vector<uint8_t>>(p.n_kw, 0);
  uint32_t ev_hot = 0, nhot = 0;
  for (uint32_t s : order) {  // s: device state id
    if (tot <= budget) break;
    const uint32_t* m = r->k1h.masks.data() + (size_t)r->k1h.accs[s] * mw;
    bool fallback = false;  // folding-rune literals must stay exact (they force host resolution)
    for (int k = p.fb_kw0; k < p.n_kw; k++) fallback |= (m[k / 32] >> (k % 32)) & 1;
    if (fallback) continue;
    hot[r->k1h.order[s]] = 1;
    nhot++;
    tot -= hits[s];
    for (int k = 0; k < p.n_kw; k++)
      if ((m[k / 32] >> (k % 32)) & 1) (*kw_unknown)[k] = 1;
    ev_hot |= m[W];
  }
  r->hot_states = nhot;
  if (!nhot) return TSG_OK;
  if ((rc = k1_tables(p, hot, &r->k1h, &r->k1.start, &r->k1.acc_row))) return rc;
  HIP_TRY(hipMemcpy((void*)r->k1.tab, r->k1h.tab.data(), r->k1h.tab.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy((void*)r->k1.accs, r->k1h.accs.data(), r->k1h.accs.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
  return apply_unknown(r, kw_unknown, ev_hot);
}

// After an adaptation: the gates of groups with an unknown keyword open, and the events of
// hot anchor literals fire everywhere.
static int apply_unknown(DeviceRules* r, const std::shared_ptr<std::vector<uint8_t>>& kw_unknown, uint32_t ev_hot) {
  const Plan& p = *r->plan;
  const uint32_t G = (uint32_t)r->groups.size();
  std::vector<uint32_t> galways = r->h_galways, gevents = r->h_gevents;
  std::vector<unsigned long long> gofbit = r->h_gofbit;
  for (uint32_t g = 0; g < G; g++) {
    for (uint32_t q : p.groups[g].rules)
      if (p.rule_kw_mode[q] == kKwBits)
        for (uint32_t k : p.rule_kws[q])
          if ((*kw_unknown)[k]) galways[g] = 1;
    if (gevents[g] & ev_hot) {
      gevents[g] |= kEvAlways;
      gofbit[31 * r->GW + g / 64] |= 1ull << (g % 64);
    }
  }
  HIP_TRY(hipMemcpy(r->d_galways, galways.data(), sizeof(uint32_t) * G, hipMemcpyHostToDevice));
  {
    std::vector<unsigned long long> galw(r->GW, 0);
    for (uint32_t g = 0; g < G; g++)
      if (galways[g]) galw[g / 64] |= 1ull << (g % 64);
    HIP_TRY(hipMemcpy(r->d_galw, galw.data(), sizeof(unsigned long long) * galw.size(), hipMemcpyHostToDevice));
  }
  HIP_TRY(hipMemcpy(r->d_gevents, gevents.data(), sizeof(uint32_t) * G, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(r->d_gofbit, gofbit.data(), sizeof(unsigned long long) * gofbit.size(), hipMemcpyHostToDevice));
  r->kw_unknown = kw_unknown;
  return TSG_OK;
}

// K1F's tables (r->k1ft) into their fixed device buffers
static int upload_k1f(DeviceRules* r) {
  const K1FTables& t = r->k1ft;
  if (t.ent.size() != 256 * 4 || t.img.size() > kFImgMax || t.img.size() % 16)
    return fail(TSG_ERR_INTERNAL, "bad K1F tables");
  HIP_TRY(hipMemcpy((void*)r->k1f.ent, t.ent.data(), 256 * 16, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy((void*)r->k1f.img, t.img.data(), t.img.size(), hipMemcpyHostToDevice));
  r->k1f.img_bytes = (uint32_t)t.img.size();
  r->k1f.nlit = t.nlit;
  // the event list's zone (K1FArgs::zone): a literal ends at most len - 2 bytes past the
  // start of a range its window end precedes
  const K1FLit* recs = (const K1FLit*)(t.img.data() + kFImgLits);
  r->k1f_maxlen = 4;
  for (uint32_t i = 0; i < t.nlit; i++) r->k1f_maxlen = std::max<uint32_t>(r->k1f_maxlen, recs[i].len);
  return TSG_OK;
}

// K1F's grid for ntiles tiles: one block per CU
static int k1f_grid(const DeviceRules* r, uint32_t ntiles) {
  const uint32_t wpb = kFThreads / 64;
  uint64_t cap = (uint64_t)r->cus;
  if (const int64_t g = knobs().k1f_grid.load()) cap = std::min<uint64_t>(cap, (uint64_t)g);  // (test knob)
  return (int)std::max<uint64_t>(1, std::min<uint64_t>((ntiles + wpb - 1) / wpb, cap));
}

// K1F builds the event list itself (K1FArgs::evlist) when chunks tile its 1 KiB tiles and a
// block's range of chunks fits the LDS bitmap
static bool k1f_lists(const DeviceRules* r, uint32_t ntiles, uint32_t chunk) {
  if (chunk == 0 || chunk > kFTile || kFTile % chunk) return false;
  if ((r->k1f_maxlen + chunk - 1) / chunk + 1 > kFZoneChunks) return false;
  const uint64_t grid = (uint64_t)k1f_grid(r, ntiles), wpb = kFThreads / 64, nw = grid * wpb;
  const uint64_t block_tiles = (wpb * ntiles + nw - 1) / nw + 1;  // (ranges differ by at most one tile per wave)
  return block_tiles * (kFTile / chunk) <= 32ull * kFBitsWords;
}

// one K1F launch over the first ntiles tiles of the batch
static int launch_k1f(DeviceRules* r, const K1FArgs& A, hipStream_t st) {
  if (A.evlist && !k1f_lists(r, A.ntiles, A.chunk)) return fail(TSG_ERR_INTERNAL, "K1F event list without room");
  k1f_kernel<<<k1f_grid(r, A.ntiles), kFThreads, 0, st>>>(r->k1f, A);
  HIP_TRY(hipGetLastError());
  return TSG_OK;
}

// K1F adaptation (once per device, on the first large batch), the counterpart of adapt_k1:
// a sampling launch over the first 16 MiB counts the verified arrivals of every literal;
// the most frequent leave the filter until the rest arrive at most once per 4 KiB.  Their
// keywords become unknown (the host checks them exactly) and their events fire everywhere,
// so results are unchanged; K1F stops verifying words like "key" that most files hold.
// The filter is then rebuilt for the data: each window and bucket priced by its count in a
// sample of the batch, so few words are listed for verification (profiles/r05/kv1: the
// model-priced buckets listed 1.24 words per KiB and their verification cost 0.2 ms per GiB).
static int adapt_k1f(DeviceRules* r, LaneState* l, const K1FArgs& A0, const uint8_t* host_data) {
  const Plan& p = *r->plan;
  HIP_TRY(hipDeviceSynchronize());
  const uint32_t nrec = r->k1ft.nlit;
  HIP_TRY(hipMemsetAsync(r->d_fhits, 0, sizeof(uint32_t) * std::max<uint32_t>(1, nrec), l->st));
  K1FArgs A = A0;
  A.ntiles = std::min<uint32_t>(A0.ntiles, (16u << 20) / kFTile);
  A.hits = r->d_fhits;
  A.stats = l->counts + 24;  // (the batch's own counters stay those of its real launch)
  A.clk = nullptr;
  A.evlist = nullptr;
  A.nev = nullptr;
  int rc;
  if ((rc = launch_k1f(r, A, l->st))) return rc;
  std::vector<uint32_t> hits(std::max<uint32_t>(1, nrec));
  HIP_TRY(hipMemcpyAsync(hits.data(), r->d_fhits, sizeof(uint32_t) * hits.size(), hipMemcpyDeviceToHost, l->st));
  HIP_TRY(hipStreamSynchronize(l->st));
  r->adapted = true;
  const uint64_t sample_bytes = std::min<uint64_t>((uint64_t)A.ntiles * kFTile, A.total);
  const K1FLit* recs = (const K1FLit*)(r->k1ft.img.data() + kFImgLits);
  std::vector<uint32_t> order;
  uint64_t tot = 0;
  for (uint32_t i = 0; i < nrec; i++)
    if (hits[i]) {
      tot += hits[i];
      order.push_back(i);
    }
  std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return hits[a] > hits[b]; });
  const uint64_t budget = sample_bytes / 4096;  // reporting budget: one arrival per 4 KiB
  std::vector<uint8_t> quiet(p.n_lit, 0);
  auto kw_unknown = std::make_shared<std::vector<uint8_t>>(p.n_kw, 0);
  uint32_t ev_hot = 0, nhot = 0;
  for (uint32_t i : order) {
    if (tot <= budget) break;
    const uint32_t id = recs[i].id;
    if ((int)id >= p.fb_kw0 && (int)id < p.n_kw) continue;  // folding runes stay exact
    quiet[id] = 1;
    nhot++;
    tot -= hits[i];
    if ((int)id < p.n_kw) (*kw_unknown)[id] = 1;
    ev_hot |= p.lit_event[id];
  }
  r->hot_states = nhot;
  // the windows and buckets again, without the hot literals and priced by their counts in a
  // sample of the batch (16 pieces of 128 KiB spread over it: 2 MiB)
  std::vector<uint8_t> sample;
  const uint64_t piece = 128 << 10, npieces = 16;
  for (uint64_t k = 0; k < npieces; k++) {
    const uint64_t at = A.total <= piece * npieces ? k * piece : k * ((A.total - piece) / (npieces - 1));
    if (at >= A.total) break;
    const uint64_t n = std::min<uint64_t>(piece, A.total - at);
    sample.insert(sample.end(), host_data + at, host_data + at + n);
  }
  K1FTables t;
  if (!k1f_build(p, quiet, &t, nullptr, sample.data(), sample.size()))
    return fail(TSG_ERR_INTERNAL, "K1F tables without the hot literals");
  r->k1ft = std::move(t);
  if ((rc = upload_k1f(r))) return rc;
  return nhot ? apply_unknown(r, kw_unknown, ev_hot) : TSG_OK;
}

int device_rules_create(int device, const Plan& p, uint32_t chunk, uint32_t ext_cap, uint32_t adapt_mib,
                        DeviceRules** out) {
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(TSG_ERR_GPU, "no such HIP device");
  HIP_TRY(hipSetDevice(device));
  auto r = std::make_unique<DeviceRules>();
  r->device = device;
  r->plan = &p;
  r->chunk = chunk;
  r->ext_cap = ext_cap;
  r->adapt_mib = adapt_mib;
  if (p.warm > kPad) return fail(TSG_ERR_CONFIG, "a keyword is longer than the K1 warm-up window");
  int rc;
  if ((rc = make_device_k1(p, &r->k1, &r->tables, &r->k1h))) return rc;
  if ((rc = make_device_k1x(p, &r->k1x, &r->tables))) return rc;
  r->has_k1x = !p.x_lits.empty();
  if (!knobs().k1_automaton.load() && k1f_build(p, {}, &r->k1ft, nullptr)) {
    // fixed-size device tables: the adaptation rewrites them in place
    void* ent = nullptr;
    void* img = nullptr;
    HIP_TRY(hipMalloc(&ent, 256 * 16));
    r->tables.push_back(ent);
    HIP_TRY(hipMalloc(&img, kFImgMax));
    r->tables.push_back(img);
    r->k1f.ent = (const uint4*)ent;
    r->k1f.img = (const uint8_t*)img;
    r->k1f.kw_words = (uint32_t)p.kw_words;
    if ((rc = upload_k1f(r.get()))) return rc;
    HIP_TRY(hipMalloc((void**)&r->d_fhits, sizeof(uint32_t) * std::max(1, p.n_lit)));
    r->use_k1f = true;
  }
  for (uint8_t h : p.rule_hostonly) r->all_kw_rows |= h;
  if (r->has_k1x)  // the 128 KiB prefix bitmap is dynamic LDS
    HIP_TRY(hipFuncSetAttribute(k1x_fn(r->k1x.step), hipFuncAttributeMaxDynamicSharedMemorySize,
                                kXDwords * 4 + 16));
  if (r->has_k1x && r->k1x.img_bytes <= kXImgLds)
    HIP_TRY(hipFuncSetAttribute((const void*)k1x_verify_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                r->k1x.img_bytes));
  HIP_TRY(hipMalloc((void**)&r->d_hits, sizeof(uint32_t) * r->k1.ns));
  const uint32_t G = (uint32_t)p.groups.size();
  if (G > 0x7FFF) return fail(TSG_ERR_INTERNAL, "more K2 groups than transition records can name");
  r->GW = std::max<uint32_t>(1, (G + 63) / 64);
  std::vector<uint32_t> gmask, galways, gevents;
  std::vector<unsigned long long> gofbit(32 * r->GW, 0);
  for (uint32_t g = 0; g < G; g++) {
    const auto& gp = p.groups[g];
    DevDFA dd{};
    if ((rc = make_device_dfa(*gp.dfa, gp.rules, &dd, &r->tables))) return rc;
    r->max_lds = std::max(r->max_lds, dd.lds_bytes);
    r->groups.push_back(dd);
    gmask.insert(gmask.end(), gp.kwmask.begin(), gp.kwmask.end());
    galways.push_back(gp.always ? 1 : 0);
    gevents.push_back(gp.events);
    uint32_t back = group_back(gp, chunk);
    if (back > (uint32_t)kMaxBack) back = kMaxBack + 1;
    r->gback.push_back(back);
    if (back <= (uint32_t)kMaxBack) r->maxback = std::max(r->maxback, back);
    for (int b = 0; b < 32; b++)
      if (((gp.events >> b) & 1) || back > (uint32_t)kMaxBack) gofbit[b * r->GW + g / 64] |= 1ull << (g % 64);
  }
  r->max_lds = std::max<uint32_t>(r->max_lds, 16);
  {  // the item passes' LDS: group tables (item_lds_bytes), counts, ranges, bases, kinds
    const size_t emit_lds = item_lds_host(G, r->GW) + kItemKwgLdsMax + 13 * (size_t)G + 16;
    if (emit_lds > 160 * 1024) return fail(TSG_ERR_INTERNAL, "too many rule groups for the item passes");
    if (emit_lds > 64 * 1024) {
      HIP_TRY(hipFuncSetAttribute((const void*)items_emit_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)emit_lds));
      HIP_TRY(hipFuncSetAttribute((const void*)items_count_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)emit_lds));
    }
  }
  if (r->max_lds > 64 * 1024) {
    HIP_TRY(hipFuncSetAttribute((const void*)k2_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)r->max_lds));
    HIP_TRY(hipFuncSetAttribute((const void*)k2_kernel_rich, hipFuncAttributeMaxDynamicSharedMemorySize, (int)r->max_lds));
    HIP_TRY(hipFuncSetAttribute((const void*)k2_dense_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)r->max_lds));
  }
  const uint32_t* cg = nullptr;
  if ((rc = upload_vec(gmask, &cg, &r->tables))) return rc;
  r->d_gmask = (uint32_t*)cg;
  if ((rc = upload_vec(galways, &cg, &r->tables))) return rc;
  r->d_galways = (uint32_t*)cg;
  if ((rc = upload_vec(gevents, &cg, &r->tables))) return rc;
  r->d_gevents = (uint32_t*)cg;
  if ((rc = upload_vec(r->gback, &cg, &r->tables))) return rc;
  r->d_gback = (uint32_t*)cg;
  const unsigned long long* cb = nullptr;
  if ((rc = upload_vec(gofbit, &cb, &r->tables))) return rc;
  {  // the gate kernel's tables: keyword -> groups, always-gated groups as bits
    const uint32_t nkw = (uint32_t)p.kw_words * 32;
    std::vector<unsigned long long> kwg((size_t)nkw * r->GW, 0), galw(r->GW, 0);
    for (uint32_t g = 0; g < G; g++) {
      for (uint32_t k = 0; k < nkw; k++)
        if ((gmask[(size_t)g * p.kw_words + k / 32] >> (k % 32)) & 1) kwg[(size_t)k * r->GW + g / 64] |= 1ull << (g % 64);
      if (galways[g]) galw[g / 64] |= 1ull << (g % 64);
    }
    const unsigned long long* c64 = nullptr;
    if ((rc = upload_vec(kwg, &c64, &r->tables))) return rc;
    r->d_kwg = (unsigned long long*)c64;
    if ((rc = upload_vec(galw, &c64, &r->tables))) return rc;
    r->d_galw = (unsigned long long*)c64;
  }
  r->h_galways = galways;
  r->h_gevents = gevents;
  r->h_gofbit = gofbit;
  r->d_gofbit = (unsigned long long*)cb;
  const DevDFA* cd = nullptr;
  if ((rc = upload_vec(r->groups, &cd, &r->tables))) return rc;
  r->d_groups = (DevDFA*)cd;
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  r->cus = prop.multiProcessorCount;
  r->grid = prop.multiProcessorCount * 8;
  // (orders the next batch's kernels after this one's on the same device: a device-scope
  // release is enough)
  HIP_TRY(hipEventCreateWithFlags(&r->kernels_done, hipEventDisableTiming | hipEventReleaseToDevice));
  int occ = 0;
  HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)k2_kernel, kK2Block, r->max_lds));
  r->k2_grid = r->cus * std::max(occ, 1);
  {  // when the staged table already holds the CU to as many blocks as the rich variant's
     // registers do, that variant runs (builtin rules, 64 KiB groups: 2 blocks per CU)
    int occ_rich = 0;
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_rich, (const void*)k2_kernel_rich, kK2Block, r->max_lds));
    r->k2_rich = occ_rich >= 1 && occ_rich >= occ;
  }
  HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)k2_dense_kernel, kBlock, r->max_lds));
  r->k2_dense_grid = r->cus * std::max(occ, 1);
  *out = r.release();
  return TSG_OK;
}

void device_rules_destroy(DeviceRules* d) { delete d; }

std::shared_ptr<const std::vector<uint8_t>> device_rules_kw_unknown(const DeviceRules* d) { return d->kw_unknown; }
uint32_t device_rules_hot_states(const DeviceRules* d) { return d->hot_states; }
bool device_rules_k1_filter(const DeviceRules* d) { return d->use_k1f; }

int lane_create(DeviceRules* d, LaneState** out) {
  HIP_TRY(hipSetDevice(d->device));
  auto l = std::make_unique<LaneState>();
  l->d = d;
  HIP_TRY(hipStreamCreateWithFlags(&l->st, hipStreamNonBlocking));
  const uint32_t G = std::max<uint32_t>(1, (uint32_t)d->groups.size());
  // per-batch counters: 0 candidates, 1 event chunks, 2 K2 entries, 3 dense entries, 5-7
  // layout (5 items, 6 entries, 7 groups skipped), 8-11 K2 diagnostics,
  // 12-13 K2 claim cursors (list, dense), 14-15 K1X (records listed, inline verified),
  // 16-17 K1F (words listed, literal occurrences verified), 24-25 the same of the
  // adaptation's sampling launch
  HIP_TRY(hipMalloc((void**)&l->counts, sizeof(uint32_t) * kCounts));
  HIP_TRY(hipMalloc((void**)&l->gcount, sizeof(uint32_t) * G));
  HIP_TRY(hipMalloc((void**)&l->bcount, sizeof(uint32_t) * G * (size_t)d->grid));
  HIP_TRY(hipMalloc((void**)&l->cursor, sizeof(uint32_t) * G));
  HIP_TRY(hipMalloc((void**)&l->gskip, G));
  *out = l.release();
  return TSG_OK;
}

void lane_destroy(LaneState* l) { delete l; }
hipStream_t lane_stream(LaneState* l) { return l->st; }

static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

void host_out_free(HostOut* o) {
  void* ps[] = {o->blk, o->cand};
  for (void* p : ps)
    if (p) (void)hipHostFree(p);
  for (auto& e : o->ev)
    if (e) (void)hipEventDestroy(e);
  *o = HostOut{};
}

int host_out_alloc(const DeviceRules* d, uint32_t files_cap, HostOut* o) {
  HIP_TRY(hipSetDevice(d->device));
  HostOut h;
  h.files_cap = std::max<uint32_t>(files_cap, 1);
  h.cand_cap = 1u << 22;
  h.groups = std::max<uint32_t>(1, (uint32_t)d->groups.size());
  h.kw_words = (uint32_t)d->plan->kw_words;
  // one host-mapped block for the small outputs (each part 256-B aligned): counts | gskip |
  // ovf | kw
  const size_t o_gskip = 256, o_ovf = o_gskip + al256(h.groups), o_kw = o_ovf + al256(h.files_cap),
               bytes = o_kw + al256(sizeof(uint32_t) * (size_t)h.files_cap * h.kw_words);
  auto fail_free = [&](hipError_t e, const char* what) {
    host_out_free(&h);
    return fail(TSG_ERR_GPU, std::string(what) + ": " + hipGetErrorString(e));
  };
  hipError_t e;
  if ((e = hipHostMalloc((void**)&h.blk, bytes, hipHostMallocMapped)) != hipSuccess) return fail_free(e, "hipHostMalloc");
  if ((e = hipHostGetDevicePointer((void**)&h.blk_dev, h.blk, 0)) != hipSuccess) return fail_free(e, "hipHostGetDevicePointer");
  h.counts = (uint32_t*)h.blk;
  {
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, d->device) == hipSuccess && khz > 0)
      h.wall_khz = (uint32_t)khz;
  }
  h.gskip = h.blk + o_gskip;
  h.ovf = h.blk + o_ovf;
  h.kw = (uint32_t*)(h.blk + o_kw);
  if ((e = hipHostMalloc((void**)&h.cand, sizeof(Candidate) * (size_t)h.cand_cap, hipHostMallocMapped)) != hipSuccess)
    return fail_free(e, "hipHostMalloc");
  if ((e = hipHostGetDevicePointer((void**)&h.cand_dev, h.cand, 0)) != hipSuccess) return fail_free(e, "hipHostGetDevicePointer");
  // ev[0 .. kEvDone) only time the stages: no system-scope fence when they are recorded (the
  // default event writes back and invalidates the caches, a gap of 6-13 us after each kernel
  // they follow: profiles/r05/final3/bench/timeline.txt); ev[kEvDone] completes the batch for
  // the host and keeps it
  for (int k = 0; k <= kEvDone; k++)
    if ((e = k < kEvDone ? hipEventCreateWithFlags(&h.ev[k], hipEventDisableSystemFence) : hipEventCreate(&h.ev[k])) !=
        hipSuccess)
      return fail_free(e, "hipEventCreate");
  *o = h;
  return TSG_OK;
}

int enqueue_scan(DeviceRules* r, LaneState* l, const ScanInput& in, HostOut* out) {
  const Plan& p = *r->plan;
  HIP_TRY(hipSetDevice(r->device));
  const uint32_t W = (uint32_t)p.kw_words;
  const uint32_t C = r->chunk;
  const uint32_t F = in.nfiles;
  const uint64_t total = in.total;
  const uint32_t G = (uint32_t)r->groups.size();
  hipStream_t st = l->st;
  if (F > out->files_cap) return fail(TSG_ERR_ARG, "batch has more files than its output buffers");
  if (total / C >= (1ull << 32) - 2) return fail(TSG_ERR_ARG, "batch too large for u32 chunk ids");
  const uint64_t nchunks = (total + C - 1) / C;
  l->nchunks = nchunks;
  // K1F addresses the batch with 32-bit offsets (and its tiles past the end)
  const bool k1f = r->use_k1f && total + (1u << 16) < (1ull << 32);
  int rc;
  // ---- buffers (grown on demand; growing waits for the device)
  // (K1F reads whole 1 KiB tiles, kFDepth past its last: at least 8 KiB of zero tail)
  const size_t tail = std::max<size_t>((size_t)kK1Chains * kK1Seg * C + kPad, 8192);
  const size_t meta_bytes = sizeof(uint64_t) * ((size_t)F + 1);
  // one H2D when the slot has room behind the batch: [batch | zero tail | offsets]
  const size_t o_off = ((size_t)total + tail + 15) & ~(size_t)15;
  const bool one_copy = in.room == in.data && in.room_bytes >= o_off + meta_bytes;
  if ((rc = ensure(&l->data_alloc, &l->data_cap, kPad + o_off + meta_bytes))) return rc;
  uint8_t* data = l->data_alloc + kPad;
  if (one_copy) {
    l->off = (const uint64_t*)(data + o_off);
  } else {
    if ((rc = ensure(&l->meta, &l->meta_cap, meta_bytes))) return rc;
    l->off = (const uint64_t*)l->meta;
  }
  const uint64_t k1_item_chunks = (uint64_t)kK1Chains * kK1Seg;
  const uint64_t nchunks_pad = (nchunks + k1_item_chunks - 1) / k1_item_chunks * k1_item_chunks + 1;
  const uint64_t ncf = (total >> kCfShift) + 2;
  if ((rc = ensure(&l->cf, &l->cf_cap, (size_t)ncf))) return rc;
  if ((rc = ensure(&l->ev_bits, &l->ev_cap, (size_t)nchunks_pad + 4))) return rc;
  // K1X hit records: one per 256 bytes (a lane-word with a hit past that verifies inline)
  if (r->has_k1x && (rc = ensure(&l->xlist, &l->xlist_cap, (size_t)(total / 256 + 65536)))) return rc;
  if (r->has_k1x && (rc = ensure(&l->xcount, &l->xcount_cap, (size_t)std::max(r->cus, 1)))) return rc;
  if ((rc = ensure(&l->evlist, &l->evlist_cap, (size_t)nchunks_pad))) return rc;
  const uint64_t zclaim_words = nchunks_pad / 32 + 2;
  if (k1f && (rc = ensure(&l->zclaim, &l->zclaim_cap, (size_t)zclaim_words))) return rc;
  if ((rc = ensure(&l->kw, &l->kw_cap, (size_t)F * W + 1))) return rc;
  if ((rc = ensure(&l->ggate, &l->ggate_cap, (size_t)F * r->GW + 1))) return rc;
  if ((rc = ensure(&l->ovf, &l->ovf_cap, (size_t)F + 1))) return rc;
  if ((rc = ensure(&l->hascand, &l->hascand_cap, (size_t)F + 1))) return rc;
  // item capacity: twice the batch's chunks (the builtin rules list ~11 % of them); over
  // it, groups are skipped (kGroupSkip) and resolved on the host, never dropped
  const uint64_t items_cap = std::max<uint64_t>(2 * nchunks, 1u << 16);
  const uint32_t max_dense = 16;
  const uint64_t entries_cap = items_cap / kEntryItems + G + 1;
  const uint64_t dentries_cap = (uint64_t)max_dense * ((nchunks + kEntryChunks - 1) / kEntryChunks + 1);
  if ((rc = ensure(&l->items, &l->items_cap, (size_t)items_cap))) return rc;
  if ((rc = ensure(&l->entries, &l->entries_cap, (size_t)entries_cap))) return rc;
  if ((rc = ensure(&l->dentries, &l->dentries_cap, (size_t)dentries_cap))) return rc;
  if (!l->cand || l->cand_cap < out->cand_cap) {
    if (l->cand) HIP_TRY(hipFree(l->cand));
    HIP_TRY(hipMalloc((void**)&l->cand, sizeof(DevCand) * (size_t)out->cand_cap));
    l->cand_cap = out->cand_cap;
  }
  // ---- H2D from the pinned slot: the batch, its zero tail and its file offsets in one
  // runtime copy (the paths stay on the host, where Global.AllowPath is settled per file,
  // scanner.go:343-347); a buffer without room behind the batch takes a second copy
  HIP_TRY(hipEventRecord(out->ev[0], st));
  if (one_copy) {
    std::memset(in.room + total, 0, o_off - total);
    std::memcpy(in.room + o_off, in.off, meta_bytes);
    HIP_TRY(hipMemcpyAsync(data, in.room, o_off + meta_bytes, hipMemcpyHostToDevice, st));
    HIP_TRY(hipEventRecord(out->ev[1], st));
  } else {
    if (total) HIP_TRY(hipMemcpyAsync(data, in.data, total, hipMemcpyHostToDevice, st));
    HIP_TRY(hipEventRecord(out->ev[1], st));
    HIP_TRY(hipMemcpyAsync(l->meta, in.off, meta_bytes, hipMemcpyHostToDevice, st));
  }
  HIP_TRY(hipEventRecord(out->ev[2], st));
  // ---- prep: zero fills and the coarse file map, one kernel
  {
    PrepArgs PA{};
    PA.off = l->off;
    PA.nfiles = F;
    PA.ncf = F ? ncf : 0;
    PA.cf = l->cf;
    bool too_many = false;
    auto zero = [&](void* ptr, uint64_t n) {
      if (!n) return;
      if (PA.nz == (uint32_t)kPrepZeros) {
        too_many = true;
        return;
      }
      PA.zp[PA.nz] = (uint8_t*)ptr;
      PA.zn[PA.nz++] = n;
    };
    zero(l->data_alloc, kPad);
    if (!one_copy) zero(data + total, tail);
    zero(l->kw, sizeof(uint32_t) * (uint64_t)F * W);
    zero(l->ovf, F);
    zero(l->hascand, F);
    zero(l->counts, sizeof(uint32_t) * kCounts);
    if (k1f) zero(l->ev_bits, sizeof(uint32_t) * nchunks_pad);  // K1F ORs events in
    if (k1f) zero(l->zclaim, sizeof(uint32_t) * zclaim_words);    // K1F's zone claims
    zero(l->gcount, sizeof(uint32_t) * G);
    zero(l->cursor, sizeof(uint32_t) * G);
    zero(l->gskip, G);
    if (too_many) return fail(TSG_ERR_INTERNAL, "more zero fills than the prep kernel takes");
    const uint64_t work = std::max<uint64_t>({PA.ncf, (uint64_t)F * W / 4, one_copy ? 1 : tail / 16, k1f ? nchunks_pad / 4 : 1, 1});
    const int pgrid = (int)std::min<uint64_t>((work + 255) / 256, (uint64_t)r->grid);
    prep_kernel<<<pgrid, 256, 0, st>>>(PA);
    HIP_TRY(hipGetLastError());
  }
  // the kernels of consecutive batches run one after the other (each has the whole chip;
  // their HIP-event times are the kernels' own), while this lane's H2D and prep above
  // overlapped the previous batch's kernels on the other lane (prep touches this lane's
  // buffers only: off the critical path, 17 us per batch with its event)
  HIP_TRY(hipEventRecord(out->ev[3], st));
  if (r->kernels_done_valid) HIP_TRY(hipStreamWaitEvent(st, r->kernels_done, 0));
  HIP_TRY(hipEventRecord(out->ev[4], st));

  // ---- K1
  const uint64_t k1_items = (nchunks + k1_item_chunks - 1) / k1_item_chunks;
  const uint64_t adapt_bytes = r->adapt_mib == 0xFFFFFFFFu ? ~0ull : (uint64_t)(r->adapt_mib ? r->adapt_mib : 16) << 20;
  const uint32_t k1f_tiles = (uint32_t)((total + kFTile - 1) / kFTile);
  // K1F lists the event chunks itself: no compaction pass, and the item passes gate files
  // from their keyword bits (no gates pass at all)
  // (K1X, when a plan has it, adds events after K1: the gates pass lists them all)
  // (opt-in, knob k1f_list: kernel-only on the configs[1] batch it cost K1F ~3 us and the
  // item passes ~5 us more than the gates pass it replaces, profiles/r06/d)
  const bool k1f_list = k1f && total && !r->has_k1x && knobs().k1f_list.load() && k1f_lists(r, k1f_tiles, C);
  if (k1f) {
    K1FArgs A{data, l->off, l->cf, (uint32_t)total, C, F, k1f_tiles, F ? (uint32_t)ncf : 0u,
              l->kw, l->ev_bits, nullptr, l->counts + 16, (unsigned long long*)(l->counts + kClk),
              nullptr, nullptr, r->k1f_maxlen, 0, nullptr, nullptr};
    if (!r->adapted && total >= adapt_bytes && (rc = adapt_k1f(r, l, A, in.data))) return rc;
    if (k1f_list) {
      A.evlist = l->evlist;
      A.nev = l->counts + 1;
      A.evcap = (uint32_t)std::min<size_t>(l->evlist_cap, 0xFFFFFFFFu);
      A.zone = r->k1f_maxlen;  // (after the adaptation's rebuild)
      A.claim = l->zclaim;
    }
    static const bool wtrace = getenv("TSG_K1F_TRACE") != nullptr;
    if (wtrace && total) {
      const size_t nw = (size_t)k1f_grid(r, k1f_tiles) * (kFThreads / 64);
      if ((rc = ensure(&l->wtrace, &l->wtrace_cap, 4 * nw))) return rc;
      HIP_TRY(hipMemsetAsync(l->wtrace, 0, sizeof(unsigned long long) * 4 * nw, st));
      A.wtrace = l->wtrace;
      l->wtrace_n = 4 * nw;
    }
    if (total && (rc = launch_k1f(r, A, st))) return rc;
  } else if (!r->adapted && k1_items >= 64 && total >= adapt_bytes) {
    if ((rc = adapt_k1(r, l, total, F, nchunks, k1_items))) return rc;
  }
  if (!k1f && k1_items) {
    K1Args A{data, l->off, l->cf, total, nchunks, k1_items, 1, C, F, l->kw, l->ev_bits, nullptr, (uint32_t)kK1Seg};
    if ((rc = launch_k1(r, A, st))) return rc;
  }
  if (r->has_k1x && total) {  // the hashed literals of a large rule set, after K1's stores
    const int xg = (int)std::max<uint64_t>(1, std::min<uint64_t>((total / 16 + kK1XBlock - 1) / kK1XBlock,
                                                                   (uint64_t)r->cus));
    K1XArgs X{data, l->off, l->cf, total, C, F, l->kw, l->ev_bits, l->xlist, l->xcount,
              (uint32_t)std::min<size_t>(l->xlist_cap, 0xFFFFFFFFu), l->counts + 14};
    void* xa[] = {(void*)&r->k1x, (void*)&X};
    HIP_TRY(hipLaunchKernel(k1x_fn(r->k1x.step), dim3(xg), dim3(kK1XBlock), xa, kXDwords * 4 + 16, st));
    if (r->k1x.img_bytes <= kXImgLds)
      k1x_verify_kernel<true><<<xg, kXVerifyBlock, r->k1x.img_bytes, st>>>(r->k1x, X, (uint32_t)xg);
    else
      k1x_verify_kernel<false><<<xg, kXVerifyBlock, 0, st>>>(r->k1x, X, (uint32_t)xg);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipEventRecord(out->ev[5], st));

  // ---- gates, items, device-side layout
  ItemArgs IA{};
  IA.off = l->off;
  IA.cf = l->cf;
  IA.ev = l->ev_bits;
  IA.ggate = l->ggate;
  IA.gofbit = r->d_gofbit;
  IA.gevents = r->d_gevents;
  IA.gback = r->d_gback;
  IA.nchunks = nchunks;
  IA.F = F;
  IA.G = G;
  IA.GW = r->GW;
  IA.chunk = C;
  IA.maxback = r->maxback;
  IA.count = l->gcount;
  IA.bcount = l->bcount;
  IA.cursor = l->cursor;
  IA.evlist = l->evlist;
  IA.nev = l->counts + 1;
  IA.evcap = (uint32_t)std::min<size_t>(l->evlist_cap, 0xFFFFFFFFu);
  IA.items = l->items;
  IA.kw = l->kw;
  IA.W = W;
  IA.kwg = r->d_kwg;
  IA.galw = r->d_galw;
  IA.clk = (unsigned long long*)(l->counts + kClk);
  const bool work = F && G && nchunks;
  if (work && k1f_list) {
    IA.ggate = nullptr;  // (files gated from their keyword bits in the item passes)
  } else if (work) {
    const uint32_t cgrid = (uint32_t)std::min<uint64_t>((nchunks + kEvPer * kBlock - 1) / (kEvPer * kBlock), (uint64_t)r->grid);
    const uint32_t kwg_bytes = (uint32_t)(32ull * W * r->GW * 8);
    GateArgs GA{l->ev_bits, nchunks, l->evlist, l->counts + 1, cgrid, l->kw, F, W, r->GW, r->d_kwg, r->d_galw, l->ggate,
                (unsigned long long*)(l->counts + kClk), kwg_bytes <= kKwgLdsMax ? kwg_bytes : 0u};
    gates_kernel<<<cgrid + (F + kBlock - 1) / kBlock, kBlock, GA.kwg_lds, st>>>(GA);
    HIP_TRY(hipGetLastError());
  }
  if (work) {
    // both items passes (bcount holds grid x G); ITEMS_BPC blocks per CU
    const int igrid = std::min(r->grid, r->cus * ITEMS_BPC);
    const uint32_t kwg_bytes = (uint32_t)(32ull * W * r->GW * 8);
    IA.kwg_lds = !IA.ggate && kwg_bytes <= kItemKwgLdsMax ? kwg_bytes : 0u;
    const size_t ilds = item_lds_host(G, r->GW) + IA.kwg_lds;
    hipLaunchKernelGGL(items_count_kernel, dim3(igrid), dim3(kBlock), ilds + G * sizeof(uint32_t) + 16, st, IA);
    HIP_TRY(hipGetLastError());
    LayoutArgs LA{l->gcount, G, nchunks, items_cap, max_dense, l->entries, l->counts + 2,
                  l->dentries, l->counts + 3, l->gskip, l->counts + 4};
    hipLaunchKernelGGL(items_emit_kernel, dim3(igrid), dim3(kBlock), ilds + 3 * G * sizeof(uint32_t) + G + 16, st, IA, LA);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipEventRecord(out->ev[6], st));

  // ---- K2 over the work list
  if (work) {
    K2Args A{};
    A.data = data;
    A.off = l->off;
    A.cf = l->cf;
    A.total = total;
    A.nchunks = nchunks;
    A.chunk = C;
    A.ext_cap = r->ext_cap;
    A.nfiles = F;
    A.kw = l->kw;
    A.kw_words = W;
    A.gmask = r->d_gmask;
    A.galways = r->d_galways;
    A.items = l->items;
    A.entries = l->entries;
    A.nentries = l->counts + 2;
    A.dentries = l->dentries;
    A.ndentries = l->counts + 3;
    A.cand = l->cand;
    A.cand_count = l->counts;
    A.cand_cap = out->cand_cap;
    A.ovf = l->ovf;
    A.hascand = l->hascand;
    static const bool diag = getenv("TSG_K2_DIAG") != nullptr;
    A.diag = diag ? l->counts + 8 : nullptr;
    A.claim = l->counts + 12;
    A.word_recs = G <= 0x3FFF;
    static const bool trace = getenv("TSG_K2_TRACE") != nullptr;
    if (trace && (rc = ensure(&l->etrace, &l->etrace_cap, (size_t)entries_cap * kTraceW))) return rc;
    if (trace) HIP_TRY(hipMemsetAsync(l->etrace, 0, sizeof(unsigned long long) * entries_cap * kTraceW, st));
    A.etrace = trace ? l->etrace : nullptr;
    A.clk = (unsigned long long*)(l->counts + kClk);
    // one block per resident slot (the grids are persistent)
    if (r->k2_rich)
      hipLaunchKernelGGL(k2_kernel_rich, dim3(r->k2_grid), dim3(kK2Block), r->max_lds, st, (const DevDFA*)r->d_groups, A);
    else
      hipLaunchKernelGGL(k2_kernel, dim3(r->k2_grid), dim3(kK2Block), r->max_lds, st, (const DevDFA*)r->d_groups, A);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k2_dense_kernel, dim3(r->k2_dense_grid), dim3(kBlock), r->max_lds, st,
                       (const DevDFA*)r->d_groups, A);
    HIP_TRY(hipGetLastError());
    // (the dense pass on a second stream beside the list pass: K2 0.125 -> 0.152 ms per
    // batch, the two grids slowed each other; profiles/r04/e)
  }
  HIP_TRY(hipEventRecord(out->ev[7], st));
  HIP_TRY(hipEventRecord(r->kernels_done, st));
  r->kernels_done_valid = true;

  // ---- outputs straight into the pinned, host-mapped block (no runtime copies)
  {
    OutArgs OA{};
    OA.count = l->counts;
    OA.cand_cap = out->cand_cap;
    OA.cand = (const uint8_t*)l->cand;
    OA.cand_host = (uint8_t*)out->cand_dev;
    auto copy = [&](void* host, const void* dev, uint64_t n) {
      if (n) {
        OA.dst[OA.nc] = out->blk_dev + ((uint8_t*)host - out->blk);
        OA.src[OA.nc] = (const uint8_t*)dev;
        OA.n[OA.nc++] = n;
      }
    };
    copy(out->counts, l->counts, sizeof(uint32_t) * kCounts);
    copy(out->gskip, l->gskip, G);
    OA.kw = l->kw;
    OA.kw_host = (uint32_t*)(out->blk_dev + ((uint8_t*)out->kw - out->blk));
    OA.ovf = l->ovf;
    OA.hascand = l->hascand;
    OA.flags_host = out->blk_dev + (out->ovf - out->blk);
    OA.F = F;
    OA.W = W;
    OA.fb_lo = (uint32_t)p.fb_kw0;
    OA.fb_hi = (uint32_t)p.n_kw;
    OA.all_rows = r->all_kw_rows;
    outputs_kernel<<<128, 256, 0, st>>>(OA);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipEventRecord(out->ev[kEvDone], st));
  return TSG_OK;
}

int batch_times(const HostOut* o, ScanTimes* t) {
  float x[kEvDone] = {};
  for (int k = 0; k < kEvDone; k++) HIP_TRY(hipEventElapsedTime(&x[k], o->ev[k], o->ev[k + 1]));
  t->h2d = x[0];
  t->meta = x[1];
  t->prep = x[2];  // (prep runs before the wait on the other lane's kernels)
  t->wait = x[3];
  t->k1 = x[4];
  t->gates = x[5];
  t->k2 = x[6];
  t->out = x[7];
  // the kernels' own spans by the device wall clock (stamps in counts + kClk; 0 if a
  // kernel did not run)
  const unsigned long long* c = (const unsigned long long*)(o->counts + kClk);
  const double per_ms = o->wall_khz ? (double)o->wall_khz : 100000.0;
  const unsigned long long k1s = ~c[0], k1e = c[1], k2e = c[3];
  t->k1_clk = c[0] && k1e > k1s ? (float)((k1e - k1s) / per_ms) : 0.f;
  t->chain_clk = c[0] && k2e > k1s ? (float)((k2e - k1s) / per_ms) : 0.f;
  t->post_k1_clk = c[2] && k2e > ~c[2] ? (float)((k2e - ~c[2]) / per_ms) : 0.f;
  return TSG_OK;
}

int lane_k2_trace(LaneState* l, std::vector<unsigned long long>* out) {
  HIP_TRY(hipSetDevice(l->d->device));
  HIP_TRY(hipStreamSynchronize(l->st));
  out->clear();
  if (!l->etrace) return TSG_OK;
  uint32_t counts[16];
  HIP_TRY(hipMemcpy(counts, l->counts, sizeof(counts), hipMemcpyDeviceToHost));
  const size_t n = std::min<size_t>((size_t)counts[2] * kTraceW, l->etrace_cap);
  out->resize(n);
  if (n) HIP_TRY(hipMemcpy(out->data(), l->etrace, n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return TSG_OK;
}

int lane_k1f_trace(LaneState* l, std::vector<unsigned long long>* out) {
  HIP_TRY(hipSetDevice(l->d->device));
  HIP_TRY(hipStreamSynchronize(l->st));
  out->assign(l->wtrace ? l->wtrace_n : 0, 0);
  if (!out->empty()) HIP_TRY(hipMemcpy(out->data(), l->wtrace, out->size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return TSG_OK;
}

int lane_kw(LaneState* l, uint32_t* kw, size_t n) {
  HIP_TRY(hipSetDevice(l->d->device));
  HIP_TRY(hipStreamSynchronize(l->st));
  if (n) HIP_TRY(hipMemcpy(kw, l->kw, sizeof(uint32_t) * n, hipMemcpyDeviceToHost));
  return TSG_OK;
}

int lane_events(LaneState* l, uint32_t* ev, size_t n) {
  HIP_TRY(hipSetDevice(l->d->device));
  HIP_TRY(hipStreamSynchronize(l->st));
  if (n && l->nchunks)
    HIP_TRY(hipMemcpy(ev, l->ev_bits, sizeof(uint32_t) * std::min<uint64_t>(n, l->nchunks), hipMemcpyDeviceToHost));
  return TSG_OK;
}

}  // namespace tsg
