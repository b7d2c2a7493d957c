// MI355X (gfx950) device path of the secret engine over a device-resident batch of file
// blobs packed back to back in one HBM stream (chunk c = bytes [c*C, (c+1)*C)).
//
//   K1   one dense pass over every byte: the Aho-Corasick automaton of the rule set's
//        literals (keywords of Rule.MatchKeywords + anchor literals) stepped from LDS,
//        fused with two saturating run counters (class U = token bytes, class D = digits).
//        Outputs per-file keyword bits and per-chunk event bits (plan.hpp kEv*).  A lane
//        owns kStreams consecutive chunks of one file and steps them as independent
//        chains; each chain first replays `warm` bytes of the chunk before it, so every
//        literal / run that ends inside the chunk is seen without state from other lanes.
//   gate per file: which K2 groups the keyword bits switch on; per chunk: which of those
//        groups have an event within `back` chunks after it -> (file, chunk) items,
//        counted, then appended into per-group regions.
//   K2   per rule group, its DFA (LDS-resident) over the group's items: one fused launch
//        for all sparse groups (a block per (group, item range)), a dense launch for a
//        group whose items cover a large share of the batch.  A lane runs its chunk in
//        inject mode and then follows the threads that started in it until they die
//        (noinject), so every match end is found by the lane that owns its start.
//        Accepts append {file, rule, end} candidate records.
// Exactness: K1 keyword bits are exact (files with folding runes are flagged), events
// are a necessary condition of every match of the rule's GPU program (plan.cpp), so the
// candidate set is a superset of the exact match ends; the host resolves exactly.
#include <hip/hip_runtime.h>
#include <malloc.h>
#include <mutex>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <future>
#include <vector>

#include "internal.hpp"

namespace tsg {

#define HIP_TRY(x)                                                                    \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess)                                                             \
      return fail(TSG_ERR_GPU, std::string(#x) + ": " + hipGetErrorString(e_));       \
  } while (0)

#ifndef K1_UNROLL
#define K1_UNROLL 16
#endif
#ifdef K1_EXP_COAL  // timing experiment only (wrong results): wave-coalesced loads
#define K1_ADDR(a, i, off) \
  (((a) / ((uint64_t)NS * L * 64) * ((uint64_t)NS * L * 64)) + ((uint64_t)((off) / 16) * NS + (i)) * 1024 + (threadIdx.x & 63) * 16)
#else
#define K1_ADDR(a, i, off) ((a) + (uint64_t)(i) * L + (off))
#endif
constexpr int kStreams = 4;       // K2 dense: chunks per lane
constexpr int kK1MaxStreams = 8;  // K1: chains per lane, the largest variant
constexpr int kK1Seg = 8;         // K1: consecutive chunks per chain
// static LDS size classes of the K1 kernel (KiB): 3, 2 or 1 blocks per CU
constexpr int kK1Lds[3] = {52, 80, 156};
constexpr uint32_t kK1Tab = 1024;  // K1 LDS: 256 class words, then the transition table   // independent DFA chains per lane (dense passes)
constexpr int kBlock = 256;
// K1 block and occupancy target: two blocks of K1_BLOCK threads share a CU's LDS (one
// 80 KiB automaton image each); K1_WAVES waves per SIMD bounds the registers per lane
#ifndef K1_BLOCK
#define K1_BLOCK 256
#endif
#ifndef K1_WAVES
#define K1_WAVES 2
#endif
constexpr int kK1Block = K1_BLOCK;
constexpr int kPad = 256;     // zero bytes before and after the batch in HBM (>= K1 warm-up)
constexpr int kMaxBack = 16;  // event windows up to this many chunks; larger -> whole file

// ---------------------------------------------------------------- device tables
struct DevDFA {  // K2 rule group
  const uint16_t* tab;        // [ns * nc] next | 0x8000 if the transition accepts
  const uint16_t* acc;        // [ns * nc] accept-mask index (look-ahead DFAs)
  const uint16_t* acc_state;  // [ns] accept-mask index per state (state_acc DFAs)
  const uint16_t* eot;        // [ns] accept-mask index at end of text
  const uint16_t* to_ni;      // [ns] noinject twin
  const uint8_t* dead;        // [ns]
  const uint64_t* masks;      // [nmasks * mw]
  const uint8_t* cls;         // [256]
  const uint32_t* rules;      // group-local id -> global rule
  uint32_t nc, ns, mw, nmasks, state_acc;
  uint32_t start[4];
  uint32_t o_cls, o_accs, o_masks, lds_bytes;
};

struct DevK1 {
  // States are renumbered so that the ones whose arrival must be reported (they end a
  // literal) come last, and a state is named by its row (id * nc): next = tab[row + class]
  // needs no multiply, and "arrival reports" is next >= acc_row.
  const uint16_t* tab;    // [ns * nc] row of the next state
  const uint32_t* cls;    // [256] class * 2 | 0xFF00 if in run class D | 0xFFFF0000 if in U
  const uint16_t* accs;   // [ns] accept-mask index of the literals a state ends
  const uint32_t* masks;  // [nmasks * mw] keyword words (kw_words), then the event word
  uint32_t nc, ns, nmasks, mw, kw_words, start, warm, kU, kD;  // start: row; kD = threshold << 8
  uint32_t acc_row;
  uint32_t lds_class;  // index into kK1Lds
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

__global__ void chunk_file_kernel(const uint64_t* __restrict__ off, uint32_t nfiles, uint32_t chunk,
                                  uint32_t* __restrict__ chunk_file) {
  uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= nfiles) return;
  uint64_t fs = off[f], fe = off[f + 1];
  if (fe == fs) return;
  uint64_t c0 = (fs + chunk - 1) / chunk, c1 = (fe + chunk - 1) / chunk;  // chunks starting in f
  for (uint64_t c = c0; c < c1; c++) chunk_file[c] = f;
}

// ---------------------------------------------------------------- Global.AllowPath
// One thread per file runs the allow-path DFA of the rule set over its path (the host's
// path_allowed, plan.cpp): 1 = some global allow-path regexp matches, 0 = none, 2 = the
// path holds a non-ASCII byte (the DFA is exact on ASCII paths only; the host decides).
struct DevPathDFA {
  const uint32_t* next;  // [ns * nc]
  const uint32_t* acc;   // [ns * nc] accept-mask index of the transition (0 = none)
  const uint32_t* eot;   // [ns] accept at end of text
  const uint8_t* cls;    // [256]
  uint32_t nc, start;
};

__global__ void path_allow_kernel(DevPathDFA d, const uint8_t* __restrict__ paths,
                                  const uint64_t* __restrict__ poff, uint32_t nfiles, uint8_t* __restrict__ out) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= nfiles) return;
  const uint64_t a = poff[f], b = poff[f + 1];
  bool ascii = true;
  for (uint64_t p = a; p < b; p++) ascii &= paths[p] < 0x80;
  if (!ascii) {
    out[f] = 2;
    return;
  }
  uint32_t s = d.start;
  for (uint64_t p = a; p < b; p++) {
    const uint32_t e = s * d.nc + d.cls[paths[p]];
    if (d.acc[e]) {
      out[f] = 1;
      return;
    }
    s = d.next[e];
  }
  out[f] = d.eot[s] ? 1 : 0;
}

// ---------------------------------------------------------------- K1
typedef unsigned short us2 __attribute__((ext_vector_type(2)));

// K1 class table in LDS.  The class word of a byte is class * 2 (low byte) | 0xFF00 if the
// byte is in run class D | 0xFFFF0000 if in U.  The table holds it as u16 (class * 2 |
// D << 14 | U << 15): 512 bytes, so the bytes of text hit twice fewer LDS banks per
// dword than with a 1 KiB u32 table, and one v_perm (sign bits of bytes 1 of e and
// e << 1) rebuilds the word.  Built with K1_CLS16; the default u32 table measured faster.
#ifndef K1_CLS16
typedef uint32_t k1cls_t;
__device__ __forceinline__ uint32_t k1_class_word(uint32_t e) { return e; }
#else
typedef uint16_t k1cls_t;
__device__ __forceinline__ uint32_t k1_class_word(uint32_t e) {
  return __builtin_amdgcn_perm(e << 1, e, 0x08080A00u);
}
#endif

// run counters: high half = U run length, low half = D run length << 8 (both saturating);
// m (the byte's class word) keeps the halves of the classes the byte belongs to
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
  const uint32_t* chunk_file;
  uint64_t total, nchunks, nitems, item_step;
  uint32_t chunk, nfiles;
  uint32_t* kw;    // [nfiles * kw_words]
  uint32_t* ev;    // [nchunks, padded to whole items]
  uint32_t* hits;  // [ns] arrivals per accepting state (sampling pass) or null
  uint32_t streams;  // chains per lane
  uint32_t seg;      // consecutive chunks per chain
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

template <int KWW>
struct K1Lane {
  const DevK1& d;
  const K1Args& A;
  const uint16_t* s_tab;
  const k1cls_t* s_cls;
  const uint16_t* s_accs;
  const uint32_t* s_masks;

  // the class word of byte b (see k1cls_t)
  __device__ __forceinline__ uint32_t cls(uint32_t b) const { return k1_class_word(s_cls[b]); }
  // m's low byte is the byte's class * 2: the entry's byte offset is 2 * row + m[7:0]
  __device__ __forceinline__ uint32_t next(uint32_t s, uint32_t m) const {
    return *(const uint16_t*)((const uint8_t*)s_tab + (s + s + (m & 0xFFu)));
  }
  // arrival in reporting row r with batch byte q: keyword bits of q's file (each keyword
  // only if it starts inside that file), event bits of the chain's chunk
  __device__ __forceinline__ void accept(K1Chain& c, uint32_t r, uint64_t q) {
    const uint32_t id = r / d.nc;
    if (A.hits && q < A.total) atomicAdd(&A.hits[id], 1u);
    const uint32_t* m = s_masks + (size_t)s_accs[id] * d.mw;
    c.evl |= m[d.kw_words];
    if (q >= A.total) return;
    uint32_t f = A.chunk_file[q / A.chunk];  // file holding the chunk's first byte
    while (A.off[f + 1] <= q) f++;
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
  __device__ __forceinline__ uint32_t run_bits(uint32_t mx) const {
    return ((mx >> 16) >= d.kU ? kEvRunU : 0u) | ((mx & 0xFFFFu) >= d.kD ? kEvRunD : 0u);
  }
  // the word at batch byte p again, byte by byte from row s, reporting every arrival
  __device__ __forceinline__ void replay16(K1Chain& c, uint32_t s, const uint4 v, uint64_t p) {
#pragma unroll 1
    for (uint32_t k = 0; k < 16; k++) {
      s = next(s, cls(byte_of(v, k)));
      if (s >= d.acc_row) accept(c, s, p + k);
    }
  }
  // NS chains, 16 bytes each, interleaved byte by byte; a word in which a chain reached a
  // reporting row is replayed on the rare path.  pos[i]: batch byte of chain i's word.
  template <int NS>
  __device__ __forceinline__ void fast16(K1Chain (&c)[NS], const uint4 (&v)[NS], const uint64_t (&pos)[NS]) {
    uint32_t s0[NS], top[NS];
#pragma unroll
    for (int i = 0; i < NS; i++) {
      s0[i] = c[i].s;
      top[i] = 0;
    }
#pragma unroll(NS > 4 ? K1_UNROLL / 4 : K1_UNROLL)
    for (int k = 0; k < 16; k++)
#pragma unroll
      for (int i = 0; i < NS; i++) {
#ifdef K1_EXP_NO_CLS  // timing experiments only: wrong results
        const uint32_t m = (byte_of(v[i], k) & 0x3Fu) * 2u;
#else
        const uint32_t m = cls(byte_of(v[i], k));
#endif
#ifdef K1_EXP_NO_TAB
        c[i].s = (c[i].s + m) & 0x3FFFu;
#else
        c[i].s = next(c[i].s, m);
#endif
        top[i] = max(top[i], c[i].s);
#ifndef K1_EXP_NO_RUNS
        c[i].cnt = run_step(c[i].cnt, m);
        c[i].mx = run_max(c[i].mx, c[i].cnt);
#endif
      }
#pragma unroll
    for (int i = 0; i < NS; i++)
      if (__builtin_expect(top[i] >= d.acc_row, 0)) replay16(c[i], s0[i], v[i], pos[i]);
  }

  // item = NS segments of A.seg consecutive chunks from a; chain i walks segment i (its
  // state carries from one chunk to the next, so only the segment start needs the warm-up
  // replay), the NS chains interleaved byte by byte
  template <int NS>
  __device__ void item(uint64_t a) {
    const uint8_t* data = A.data;
    const uint32_t C = A.chunk;
    const uint64_t L = (uint64_t)C * A.seg;  // segment bytes
    const uint64_t c0 = a / C;
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
        for (int i = 0; i < NS; i++) {
          const uint32_t m = cls(byte_of(v[i], k));
          c[i].s = next(c[i].s, m);
          c[i].cnt = run_step(c[i].cnt, m);
        }
    }
    // Four words in flight per chain, each register set consumed in place (the loop body
    // is unrolled four times): a set is refilled right after its word is stepped, so a
    // load has three words of work to land, and no register copy waits on a pending load.
    uint32_t jc = 0;   // offset inside the current chunk
    uint64_t ci = c0;  // chunk index of chain 0
    auto word = [&](uint64_t j, const uint4 (&v)[NS]) {
      uint64_t pos[NS];
#pragma unroll
      for (int i = 0; i < NS; i++) pos[i] = a + (uint64_t)i * L + j;
      fast16<NS>(c, v, pos);
      jc += 16;
      if (jc == C) {  // chunk end (uniform across the lane's chains): its event bits
#pragma unroll
        for (int i = 0; i < NS; i++) {
          A.ev[ci + (uint64_t)i * A.seg] = c[i].evl | run_bits(c[i].mx);
          c[i].evl = 0;
          c[i].mx = 0;
        }
        jc = 0;
        ci++;
      }
    };
    auto load = [&](uint4 (&v)[NS], uint64_t j) {
#pragma unroll
      for (int i = 0; i < NS; i++) v[i] = *(const uint4*)(data + K1_ADDR(a, i, j));
    };
    uint4 b0[NS], b1[NS], b2[NS], b3[NS];
    load(b0, 0);
    load(b1, 16);
    load(b2, 32);
    load(b3, 48);
    for (uint64_t j = 0; j < L; j += 64) {  // L is a multiple of 128
      word(j, b0);
      load(b0, j + 64);
      word(j + 16, b1);
      load(b1, j + 80);
      word(j + 32, b2);
      load(b2, j + 96);
      word(j + 48, b3);
      load(b3, j + 112);
    }
  }

  // The same walk with quad-transposed loads (see quad_transpose): quad lane t walks item
  // it0 + t of ib bytes (a ghost lane past the last item repeats it0 and stores nothing).
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
    for (uint32_t j = 0; j < d.warm; j += 16) {
      uint4 v[NS];
#pragma unroll
      for (int i = 0; i < NS; i++) v[i] = *(const uint4*)(data + a + (uint64_t)i * L - d.warm + j);
#pragma unroll
      for (int k = 0; k < 16; k++)
#pragma unroll
        for (int i = 0; i < NS; i++) {
          const uint32_t m = cls(byte_of(v[i], k));
          c[i].s = next(c[i].s, m);
          c[i].cnt = run_step(c[i].cnt, m);
        }
    }
    const uint8_t* src[4];  // word q of quad lane t's item
#pragma unroll
    for (int t = 0; t < 4; t++) src[t] = data + (it0 + t < A.nitems ? it0 + t : it0) * ib + 16u * q;
    uint32_t jc = 0;
    uint64_t ci = c0;
    auto word = [&](uint64_t jw, const uint4 (&v)[NS]) __attribute__((always_inline)) {
      uint64_t pos[NS];
#pragma unroll
      for (int i = 0; i < NS; i++) pos[i] = ghost ? A.total : a + (uint64_t)i * L + jw;
      fast16<NS>(c, v, pos);
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
    uint4 r0[NS][4], r1[NS][4];
    load(r0, 0);
    load(r1, 64);
    for (uint64_t j = 0; j < L; j += 128) {  // L is a multiple of 128
      block(j, r0);
      load(r0, j + 128);
      block(j + 64, r1);
      load(r1, j + 192);
    }
  }
};

// K1 LDS image (static, so every table address is a constant): the 256 class words at 0
// (a byte's word is at byte * 4), the transitions from 1 KiB.  Accept masks stay in
// global memory (rare path).
template <int KWW, int LDSK, int NS>
__global__ void __launch_bounds__(kK1Block) __attribute__((amdgpu_waves_per_eu(K1_WAVES, 8))) k1_kernel(DevK1 d, K1Args A) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[LDSK * 1024];
  k1cls_t* s_cls = (k1cls_t*)smem;
  uint16_t* s_tab = (uint16_t*)(smem + 1024);
  {
    const uint32_t* src = (const uint32_t*)d.tab;
    uint32_t* dst = (uint32_t*)s_tab;
    for (uint32_t i = threadIdx.x; i < (d.ns * d.nc + 1) / 2; i += blockDim.x) dst[i] = src[i];
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
      const uint32_t w = d.cls[i];
#ifndef K1_CLS16
      s_cls[i] = w;
#else
      s_cls[i] = (k1cls_t)((w & 0xFFu) | ((w >> 31) << 15) | (((w >> 15) & 1u) << 14));
#endif
    }
  }
  __syncthreads();
  K1Lane<KWW> L{d, A, s_tab, s_cls, d.accs, d.masks};
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
#ifdef K1_NO_QUAD
  for (uint64_t it = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; it < A.nitems; it += stride)
    L.template item<NS>(it * A.item_step * NS * A.seg * A.chunk);
#else
  // quads walk 4 consecutive items together (uniform trip count inside a quad)
  const uint32_t q = threadIdx.x & 3;
  const uint64_t ib = (uint64_t)A.item_step * NS * A.seg * A.chunk;
  for (uint64_t it0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) & ~3ull; it0 < A.nitems; it0 += stride)
    L.template item_quad<NS>(it0, ib, q);
#endif
}

// ---------------------------------------------------------------- gate + items
__device__ __forceinline__ bool group_gated(const uint32_t* __restrict__ kwf, const uint32_t* __restrict__ gm,
                                            uint32_t W, uint32_t always) {
  if (always) return true;
  for (uint32_t w = 0; w < W; w++)
    if (kwf[w] & gm[w]) return true;
  return false;
}

// per file: bit g of ggate[f * GW + g / 64] = group g gated (Rule.MatchKeywords may pass)
__global__ void ggate_kernel(const uint32_t* __restrict__ kw, uint32_t F, uint32_t W,
                             const uint32_t* __restrict__ gmask, const uint32_t* __restrict__ galways,
                             uint32_t G, uint32_t GW, unsigned long long* __restrict__ ggate) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  const uint32_t* kwf = kw + (size_t)f * W;
  for (uint32_t w = 0; w < GW; w++) {
    unsigned long long bits = 0;
    for (uint32_t g = w * 64; g < min(G, w * 64 + 64); g++)
      if (group_gated(kwf, gmask + (size_t)g * W, W, galways[g])) bits |= 1ull << (g - w * 64);
    ggate[(size_t)f * GW + w] = bits;
  }
}

struct ItemArgs {
  const uint64_t* off;
  const uint32_t* chunk_file;
  const uint32_t* ev;
  const uint32_t* evlist;           // chunks with event bits (ev_compact_kernel)
  const uint32_t* nev;              // [1] length of evlist
  const unsigned long long* ggate;  // [F * GW]
  const unsigned long long* gofbit;  // [32 * GW] groups listening to event bit b; bit 31 = every chunk
  const uint32_t* gevents;          // [G]
  const uint32_t* gback;            // [G] chunks (kMaxBack + 1 = whole file)
  uint64_t nchunks;
  uint32_t F, G, GW, chunk, maxback;
  uint32_t* count;            // [G]
  const uint64_t* base;       // [G] item region of each group (emit pass), null: count pass
  uint32_t* cursor;           // [G]
  const uint8_t* listed;      // [G] 1 = list group (emit pass)
  uint2* items;
};

// chunks whose K1 event word is not empty, compacted into `list`: each block takes a
// contiguous range, counts it, reserves its output with ONE global atomic, then writes its
// chunks in order (wave ballots + an LDS prefix over the block's waves)
__global__ void __launch_bounds__(kBlock) ev_compact_kernel(const uint32_t* __restrict__ ev, uint64_t nchunks,
                                                            uint32_t* __restrict__ list, uint32_t* __restrict__ count) {
  __shared__ uint32_t s_wave[kBlock / 64];
  __shared__ uint32_t s_base;
  const uint64_t per = (nchunks + gridDim.x - 1) / gridDim.x;
  const uint64_t c0 = (uint64_t)blockIdx.x * per, c1 = min(nchunks, c0 + per);
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t n = 0;
  for (uint64_t c = c0 + threadIdx.x; c < c1; c += blockDim.x) n += (ev[c] & ~kEvAlways) != 0;
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
  if (lane == 0) s_wave[wave] = n;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (uint32_t w = 0; w < kBlock / 64; w++) tot += s_wave[w];
    s_base = tot ? atomicAdd(count, tot) : 0;
  }
  __syncthreads();
  uint32_t at = s_base;
  for (uint64_t cb = c0; cb < c1; cb += blockDim.x) {
    const uint64_t c = cb + threadIdx.x;
    const bool has = c < c1 && (ev[c] & ~kEvAlways) != 0;
    const unsigned long long m = __ballot(has);
    __syncthreads();  // s_wave reuse
    if (lane == 0) s_wave[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0, tot = 0;
    for (uint32_t w = 0; w < kBlock / 64; w++) {
      before += w < wave ? s_wave[w] : 0;
      tot += s_wave[w];
    }
    if (has) list[at + before + __popcll(m & ((1ull << lane) - 1))] = (uint32_t)c;
    at += tot;
  }
}

// Items of the K2 list: (file f, chunk c) for group g iff g is gated for f and a chunk in
// [c, c + back_g] of f carries one of g's event bits (groups listening to every chunk:
// all chunks of f).  Work is generated from the sparse event chunks: event chunk e emits
// c in (previous event chunk of g, e] within back_g chunks before e and inside f, so every
// item comes from the first event chunk at or after it, exactly once.  Threads
// [0, nev) take event chunks, [nev, nev + F) take the files of every-chunk groups.
// visit(f, g, c_lo, c_hi): items c_lo..c_hi.
template <class V>
__device__ __forceinline__ void gen_items(const ItemArgs& A, uint64_t t, V visit) {
  const uint32_t nev = *A.nev;
  const uint32_t C = A.chunk;
  if (t < nev) {
    const uint64_t e = A.evlist[t];
    const uint32_t evb = A.ev[e] & ~kEvAlways;
    const uint64_t ce = (e + 1) * C;
    for (uint32_t f = A.chunk_file[e]; f < A.F && A.off[f] < ce; f++) {
      const uint64_t fs = A.off[f], fe = A.off[f + 1];
      if (fe == fs) continue;
      const uint64_t fc0 = fs / C;
      for (uint32_t w = 0; w < A.GW; w++) {
        unsigned long long cand = 0;
        for (uint32_t bits = evb; bits; bits &= bits - 1) cand |= A.gofbit[__builtin_ctz(bits) * A.GW + w];
        cand &= A.ggate[(size_t)f * A.GW + w] & ~A.gofbit[31 * A.GW + w];
        while (cand) {
          const uint32_t g = w * 64 + __builtin_ctzll(cand);
          cand &= cand - 1;
          const uint32_t back = A.gback[g];
          uint64_t lo = e > fc0 + back ? e - back : fc0;
          for (uint64_t q = e; q > lo;) {
            q--;
            if (A.ev[q] & A.gevents[g]) {
              lo = q + 1;
              break;
            }
          }
          visit(f, g, lo, e);
        }
      }
    }
  } else if (t < (uint64_t)nev + A.F) {
    const uint32_t f = (uint32_t)(t - nev);
    const uint64_t fs = A.off[f], fe = A.off[f + 1];
    if (fe == fs) return;
    for (uint32_t w = 0; w < A.GW; w++) {
      unsigned long long cand = A.ggate[(size_t)f * A.GW + w] & A.gofbit[31 * A.GW + w];
      while (cand) {
        const uint32_t g = w * 64 + __builtin_ctzll(cand);
        cand &= cand - 1;
        visit(f, g, fs / C, (fe - 1) / C);
      }
    }
  }
}

// count pass: items per group (block totals in LDS, one global atomic per group and block)
__global__ void __launch_bounds__(kBlock) items_count_kernel(ItemArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* s_count = (uint32_t*)smem;
  for (uint32_t g = threadIdx.x; g < A.G; g += blockDim.x) s_count[g] = 0;
  __syncthreads();
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  gen_items(A, t, [&](uint32_t, uint32_t g, uint64_t lo, uint64_t hi) { atomicAdd(&s_count[g], (uint32_t)(hi - lo + 1)); });
  __syncthreads();
  for (uint32_t g = threadIdx.x; g < A.G; g += blockDim.x)
    if (s_count[g]) atomicAdd(&A.count[g], s_count[g]);
}

// emit pass: the block counts its items again, reserves one range per group with a single
// global atomic, then writes its items into it
__global__ void __launch_bounds__(kBlock) items_emit_kernel(ItemArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* s_count = (uint32_t*)smem;
  uint32_t* s_base = s_count + A.G;
  for (uint32_t g = threadIdx.x; g < A.G; g += blockDim.x) s_count[g] = 0;
  __syncthreads();
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  gen_items(A, t, [&](uint32_t, uint32_t g, uint64_t lo, uint64_t hi) {
    if (A.listed[g]) atomicAdd(&s_count[g], (uint32_t)(hi - lo + 1));
  });
  __syncthreads();
  for (uint32_t g = threadIdx.x; g < A.G; g += blockDim.x) {
    s_base[g] = s_count[g] ? (uint32_t)A.base[g] + atomicAdd(&A.cursor[g], s_count[g]) : 0;
    s_count[g] = 0;
  }
  __syncthreads();
  gen_items(A, t, [&](uint32_t f, uint32_t g, uint64_t lo, uint64_t hi) {
    if (!A.listed[g]) return;
    const uint32_t n = (uint32_t)(hi - lo + 1);
    uint32_t at = s_base[g] + atomicAdd(&s_count[g], n);
    for (uint64_t c = lo; c <= hi; c++) A.items[at++] = make_uint2(f, (uint32_t)c);
  });
}

// ---------------------------------------------------------------- K2
struct ScanArgsDev {
  const uint8_t* data;
  const uint64_t* off;
  const uint32_t* chunk_file;
  uint64_t total, nitems;
  uint32_t chunk, ext_cap;
  const uint32_t* kw;
  uint32_t kw_words;
  const uint32_t* gmask;  // dense: this group's keyword mask [kw_words]
  uint32_t galways;
  const uint2* items;     // list mode
  DevCand* cand;
  uint32_t* cand_count;
  uint32_t cand_cap;
  uint32_t* ovf;
};

struct Lane {
  const DevDFA& d;
  const ScanArgsDev& A;
  const uint16_t* s_tab;
  const uint8_t* s_cls;
  const uint16_t* s_accs;
  const uint64_t* s_masks;
  uint32_t file;
  uint64_t fs;

  // rare path (an accept); the unrolled loops below never call it directly: they only OR
  // the accept bits of 16 transitions and replay the word through step() when one is set
  __device__ __forceinline__ void emit(uint32_t mi, uint64_t pos) {
    const uint64_t* m = (d.state_acc && mi < d.nmasks) ? s_masks + (size_t)mi * d.mw : d.masks + (size_t)mi * d.mw;
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

  __device__ __forceinline__ uint32_t step(uint32_t s, uint32_t byte, uint64_t pos) {
    const uint32_t ix = s * d.nc + s_cls[byte];
    const uint32_t e = s_tab[ix];
    if (__builtin_expect(e & 0x8000u, 0)) emit(d.state_acc ? s_accs[s] : d.acc[ix], pos);
    return e & 0x7FFFu;
  }

  __device__ __forceinline__ uint32_t fast(uint32_t s, uint32_t byte) const {
    return s_tab[s * d.nc + s_cls[byte]];
  }

  __device__ __forceinline__ void replay16(uint32_t s, const uint4 v, uint64_t p) {
#pragma unroll 1
    for (uint32_t k = 0; k < 16; k++) s = step(s, byte_of(v, k), p + k);
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
  __device__ __forceinline__ void tail(uint32_t s, uint64_t fe, uint64_t b) {
    const uint8_t* data = A.data;
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
  uint16_t* s_tab = (uint16_t*)smem;
  const uint32_t* src = (const uint32_t*)d.tab;
  uint32_t* dst = (uint32_t*)s_tab;
  for (uint32_t i = threadIdx.x; i < (d.ns * d.nc + 1) / 2; i += blockDim.x) dst[i] = src[i];
  uint8_t* s_cls = smem + d.o_cls;
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) s_cls[i] = d.cls[i];
  if (d.state_acc) {
    uint16_t* s_accs = (uint16_t*)(smem + d.o_accs);
    uint64_t* s_masks = (uint64_t*)(smem + d.o_masks);
    for (uint32_t i = threadIdx.x; i < d.ns; i += blockDim.x) s_accs[i] = d.acc_state[i];
    for (uint32_t i = threadIdx.x; i < d.nmasks * d.mw; i += blockDim.x) s_masks[i] = d.masks[i];
  }
  __syncthreads();
}

// dense: every chunk of the batch, lanes skip the pieces of files the group is not gated on
__global__ void __launch_bounds__(kBlock) k2_dense_kernel(DevDFA d, ScanArgsDev A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  stage_dfa(d, smem);
  Lane L{d, A, (const uint16_t*)smem, smem + d.o_cls, (const uint16_t*)(smem + d.o_accs),
         (const uint64_t*)(smem + d.o_masks), 0, 0};
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t it = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; it < A.nitems; it += stride) {
    uint64_t a = it * kStreams * A.chunk;
    const uint64_t b = min(a + (uint64_t)kStreams * A.chunk, A.total);
    uint32_t f = A.chunk_file[it * kStreams];
    {
      const uint64_t fs = A.off[f], fe = A.off[f + 1];
      if (b == a + (uint64_t)kStreams * A.chunk && b <= fe) {  // common case: one file
        if (group_gated(A.kw + (size_t)f * A.kw_words, A.gmask, A.kw_words, A.galways)) {
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
      if (group_gated(A.kw + (size_t)f * A.kw_words, A.gmask, A.kw_words, A.galways)) {
        L.file = f;
        L.fs = fs;
        L.piece(fe, a, se);
      }
      a = se;
      f++;
    }
  }
}

// list: block b scans items [first, first + n) of group g; blkmap[b] = (g, first, n)
__global__ void __launch_bounds__(kBlock) k2_list_kernel(const DevDFA* __restrict__ dfas,
                                                         const uint4* __restrict__ blkmap,
                                                         ScanArgsDev A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint4 bm = blkmap[blockIdx.x];
  const DevDFA d = dfas[__builtin_amdgcn_readfirstlane(bm.x)];
  stage_dfa(d, smem);
  Lane L{d, A, (const uint16_t*)smem, smem + d.o_cls, (const uint16_t*)(smem + d.o_accs),
         (const uint64_t*)(smem + d.o_masks), 0, 0};
  for (uint32_t i = threadIdx.x; i < bm.z; i += blockDim.x) {
    const uint2 item = A.items[bm.y + i];
    const uint32_t f = item.x;
    const uint64_t fs = A.off[f], fe = A.off[f + 1];
    const uint64_t a = max(fs, (uint64_t)item.y * A.chunk);
    const uint64_t b = min(fe, (uint64_t)(item.y + 1) * A.chunk);
    if (a < b) {
      L.file = f;
      L.fs = fs;
      L.piece(fe, a, b);
    }
  }
}

// ---------------------------------------------------------------- host side
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

static int make_device_dfa(const DFA& d, const std::vector<uint32_t>& rules, DevDFA* out,
                           std::vector<void*>* allocs) {
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
  v.lds_bytes = o + 16;
  if (v.lds_bytes > 160 * 1024) return fail(TSG_ERR_INTERNAL, "DFA tables exceed LDS");
  return TSG_OK;
}

// perf experiments only (results are not exact): bit 0 strips the K1 accept flags
static int k1_debug() {
  const char* e = getenv("TSG_K1_DEBUG");
  return e ? atoi(e) : 0;
}

struct K1Host {  // host copies of the K1 tables (adaptation rebuilds the device table)
  std::vector<uint16_t> tab, accs;
  std::vector<uint32_t> masks;
  std::vector<uint32_t> order;  // device state id -> automaton state
  uint32_t stride = 0;          // row stride of tab (>= the class count)
};

// Device numbering of the K1 automaton: states whose arrival is reported (they end a
// literal, and are not `quiet`) last; rows = id * nc.
// Row stride (u16 entries) of the K1 table: the class count padded to 2 mod 4, so a row is
// an odd number of dwords and equal classes of different rows fall in different LDS banks
// (ds_read_u16 banks are dword mod 32).  Padding is skipped when it would need a larger LDS
// image or overflow the 16-bit rows.  TSG_K1_STRIDE=0 turns it off (measurements).
static size_t k1_stride(size_t nc, size_t ns) {
  const char* e = getenv("TSG_K1_STRIDE");
  if (e && atoi(e) == 0) return nc;
  size_t rs = nc;
  while (rs % 4 != 2) rs++;
  auto lds_class = [&](size_t r) {
    for (int k = 0; k < 3; k++)
      if (ns * r * 2 + 2 + 1024 <= (size_t)kK1Lds[k] * 1024) return k;
    return 3;
  };
  if ((ns - 1) * rs > 0xFFFF || lds_class(rs) != lds_class(nc)) return nc;
  return rs;
}

static int k1_tables(const Plan& p, const std::vector<uint8_t>& quiet, K1Host* h, uint32_t* start_row,
                     uint32_t* acc_row) {
  const DFA& d = *p.kw_dfa;
  const size_t nc = d.nclasses, ns = d.nstates;
  const size_t rs = k1_stride(nc, ns);
  h->stride = (uint32_t)rs;
  if ((ns - 1) * rs > 0xFFFF) return fail(TSG_ERR_INTERNAL, "keyword automaton too large for 16-bit rows");
  std::vector<uint32_t> newid(ns);
  h->order.clear();
  for (int pass = 0; pass < 2; pass++)
    for (size_t st = 0; st < ns; st++) {
      const bool rep = d.eot_acc[st] && !quiet[st] && !(k1_debug() & 1);
      if (rep == (pass == 1)) {
        newid[st] = (uint32_t)h->order.size();
        h->order.push_back((uint32_t)st);
      }
    }
  uint32_t first_rep = (uint32_t)ns;
  for (size_t i = 0; i < ns; i++) {
    const uint32_t st = h->order[i];
    if (d.eot_acc[st] && !quiet[st] && !(k1_debug() & 1)) {
      first_rep = (uint32_t)i;
      break;
    }
  }
  h->tab.assign(ns * rs + (ns * rs & 1), 0);  // the kernel stages whole dwords
  h->accs.assign(ns, 0);
  for (size_t i = 0; i < ns; i++) {
    const uint32_t st = h->order[i];
    h->accs[i] = (uint16_t)d.eot_acc[st];
    for (size_t c = 0; c < nc; c++) h->tab[i * rs + c] = (uint16_t)(newid[d.next[st * nc + c]] * rs);
  }
  *start_row = newid[d.start[kCtxBOT]] * (uint32_t)rs;
  *acc_row = first_rep * (uint32_t)rs;
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
  std::vector<uint32_t> cls(256);
  for (int b = 0; b < 256; b++)
    cls[b] = (uint32_t)d.cls[b] * 2 | ((p.run_cls[b] & 2) ? 0xFF00u : 0u) | ((p.run_cls[b] & 1) ? 0xFFFF0000u : 0u);
  const uint32_t W = (uint32_t)p.kw_words, mw = W + 1;
  std::vector<uint32_t> masks((size_t)d.masks.size() * mw, 0);
  for (size_t m = 0; m < d.masks.size(); m++) {
    for (int k = 0; k < p.n_kw; k++)
      if ((d.masks[m][k / 64] >> (k % 64)) & 1) masks[m * mw + k / 32] |= 1u << (k % 32);
    masks[m * mw + W] = p.kw_mask_events[m];
  }
  if ((rc = upload_vec(host->tab, &v.tab, allocs))) return rc;
  if ((rc = upload_vec(cls, &v.cls, allocs))) return rc;
  if ((rc = upload_vec(host->accs, &v.accs, allocs))) return rc;
  if ((rc = upload_vec(masks, &v.masks, allocs))) return rc;
  v.nc = host->stride;  // the kernel's row stride
  v.ns = (uint32_t)d.nstates;
  v.nmasks = (uint32_t)d.masks.size();
  v.mw = mw;
  v.kw_words = W;
  v.warm = (uint32_t)p.warm;
  v.kU = (uint32_t)p.run_k[0];
  v.kD = (uint32_t)p.run_k[1] << 8;
  std::vector<uint16_t> kwlen((size_t)W * 32, 0);
  v.kw_maxlen = 1;
  for (int k = 0; k < p.n_kw; k++) {
    kwlen[k] = p.kw_len[k];
    v.kw_maxlen = std::max<uint32_t>(v.kw_maxlen, p.kw_len[k]);
  }
  if ((rc = upload_vec(kwlen, &v.kw_len, allocs))) return rc;
  host->masks = masks;
  const uint32_t need = (uint32_t)(host->tab.size() * 2) + 1024;
  v.lds_class = 3;
  for (uint32_t k = 0; k < 3; k++)
    if (need <= (uint32_t)kK1Lds[k] * 1024) {
      v.lds_class = k;
      break;
    }
  if (v.lds_class > 2) return fail(TSG_ERR_INTERNAL, "keyword automaton exceeds LDS");
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
  std::vector<void*> tables;        // every rule-table allocation
  DevK1 k1{};
  K1Host k1h;
  uint32_t* d_hits = nullptr;       // [K1 states] (adaptation sample)
  bool adapted = false;
  uint32_t hot_states = 0;
  std::vector<uint8_t> kw_unknown;  // [n_kw] keywords K1 stopped reporting
  std::vector<uint32_t> h_galways, h_gevents;
  std::vector<unsigned long long> h_gofbit;
  std::vector<DevDFA> groups;
  DevDFA* d_groups = nullptr;       // [G] (list kernel)
  DevPathDFA pathdfa{};
  bool has_pathdfa = false;
  uint8_t* d_paths = nullptr;       // the batch's paths
  size_t d_paths_cap = 0;
  uint64_t* d_poff = nullptr;
  size_t d_poff_cap = 0;
  uint8_t* d_pathok = nullptr;      // [F] path_allow_kernel output
  size_t d_pathok_cap = 0;
  uint32_t* d_gmask = nullptr;      // [G * W]
  uint32_t* d_galways = nullptr;    // [G]
  uint32_t* d_gevents = nullptr;    // [G]
  uint32_t* d_gback = nullptr;      // [G]
  unsigned long long* d_gofbit = nullptr;  // [32 * GW]
  std::vector<uint32_t> gback;
  uint32_t GW = 1, maxback = 0;
  // batch
  const uint8_t* h_data = nullptr;
  const uint64_t* h_off = nullptr;
  const char* h_paths = nullptr;
  const uint64_t* h_poff = nullptr;
  uint32_t nfiles = 0;
  uint64_t total = 0;
  uint8_t* d_data_alloc = nullptr;  // kPad | batch | kPad
  uint8_t* d_data = nullptr;
  size_t d_data_cap = 0;
  uint64_t* d_off = nullptr;
  size_t d_off_cap = 0;
  uint32_t* d_chunk_file = nullptr;
  size_t d_chunk_cap = 0;
  uint32_t* d_ev = nullptr;
  size_t d_ev_cap = 0;
  uint32_t* d_evlist = nullptr;  // chunks with events
  size_t d_evlist_cap = 0;
  uint32_t* d_kw = nullptr;
  size_t d_kw_cap = 0;
  unsigned long long* d_ggate = nullptr;
  size_t d_ggate_cap = 0;
  uint32_t* d_ovf = nullptr;
  size_t d_ovf_cap = 0;
  DevCand* d_cand = nullptr;
  uint32_t* d_count = nullptr;      // [0] candidates
  uint32_t* d_gcount = nullptr;     // [G] items per group
  uint32_t* d_cursor = nullptr;     // [G]
  uint64_t* d_base = nullptr;       // [G]
  uint8_t* d_listed = nullptr;      // [G]
  uint4* d_blkmap = nullptr;
  size_t d_blkmap_cap = 0;
  uint2* d_items = nullptr;
  size_t d_items_cap = 0;
  // host mirrors
  KernelOutput ko;
  std::vector<std::shared_ptr<KernelOutput>> ko_pool;  // outputs of submitted batches
  std::vector<uint32_t> h_ovf;
  uint32_t* h_count = nullptr;
  tsg_stats stats{};
  int grid = 0;
  bool uploaded = false;
  // host resolutions of submitted batches, oldest first (tsg_batch_submit / collect)
  struct Pending {
    std::future<std::unique_ptr<tsg_result>> res;
    std::shared_ptr<std::pair<double, uint64_t>> done;  // resolve ms, files with findings
  };
  std::deque<Pending> pending;

  ~tsg_ctx() {
    for (auto& pj : pending)
      if (pj.res.valid()) pj.res.wait();
    (void)hipSetDevice(device);
    for (auto* p : tables) (void)hipFree(p);
    (void)hipFree(d_hits);
    (void)hipFree(d_data_alloc);
    (void)hipFree(d_off);
    (void)hipFree(d_chunk_file);
    (void)hipFree(d_ev);
    (void)hipFree(d_evlist);
    (void)hipFree(d_kw);
    (void)hipFree(d_ggate);
    (void)hipFree(d_ovf);
    (void)hipFree(d_cand);
    (void)hipFree(d_count);
    (void)hipFree(d_gcount);
    (void)hipFree(d_cursor);
    (void)hipFree(d_base);
    (void)hipFree(d_listed);
    (void)hipFree(d_blkmap);
    (void)hipFree(d_items);
    (void)hipFree(d_paths);
    (void)hipFree(d_poff);
    (void)hipFree(d_pathok);
    if (h_count) hipHostFree(h_count);
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
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

template <int LDSK, int NS>
static const void* k1_fn_w(uint32_t kw_words) {
  if (kw_words <= 1) return (const void*)k1_kernel<1, LDSK, NS>;
  if (kw_words <= 2) return (const void*)k1_kernel<2, LDSK, NS>;
  if (kw_words <= 4) return (const void*)k1_kernel<4, LDSK, NS>;
  return (const void*)k1_kernel<8, LDSK, NS>;
}

template <int NS>
static const void* k1_fn_ns(uint32_t kw_words, uint32_t lds_class) {
  switch (lds_class) {
    case 0: return k1_fn_w<kK1Lds[0], NS>(kw_words);
    case 1: return k1_fn_w<kK1Lds[1], NS>(kw_words);
    default: return k1_fn_w<kK1Lds[2], NS>(kw_words);
  }
}

// independent K1 chains per lane: 2 (quad-transposed loads keep two 64-byte blocks per
// chain in registers), or 4 with TSG_K1_NS=4 (measurements)
static uint32_t k1_streams() {
  const char* e = getenv("TSG_K1_NS");
  return (e && atoi(e) == 4) ? 4u : 2u;
}

static const void* k1_fn(uint32_t kw_words, uint32_t lds_class, uint32_t ns) {
  return ns == 2 ? k1_fn_ns<2>(kw_words, lds_class) : k1_fn_ns<4>(kw_words, lds_class);
}

static int launch_k1(tsg_ctx* c, const K1Args& A) {
  static const int gmul = getenv("TSG_K1_GRID") ? atoi(getenv("TSG_K1_GRID")) : 0;
  const uint64_t cap = (uint64_t)c->grid / 8 * (gmul > 0 ? gmul : 8);
  const int grid = (int)std::min<uint64_t>((A.nitems + kK1Block - 1) / kK1Block, cap);
  DevK1 d = c->k1;
  K1Args a = A;
  void* args[] = {&d, &a};
  HIP_TRY(hipLaunchKernel(k1_fn(c->k1.kw_words, c->k1.lds_class, A.streams), dim3(grid), dim3(kK1Block), args, 0,
                          c->stream));
  HIP_TRY(hipGetLastError());
  return TSG_OK;
}

// K1 adaptation (once per context, on the first large batch): a sampling pass counts the
// arrivals in every accepting state; the most frequent states stop raising the accept
// flag until the rest arrive at most once per 4 KiB.  The literals those states end are
// then unknown per file: their keyword gates open (host checks them exactly), their
// anchor events fire everywhere.  Results are unchanged; K1 stops paying per-occurrence
// accepts for words like "key" that occur in most files anyway.
static int adapt_k1(tsg_ctx* c, uint64_t nchunks, uint64_t k1_items) {
  const Plan& p = *c->rs->plan;
  const uint32_t ns = c->k1.ns, W = c->k1.kw_words, mw = c->k1.mw, G = (uint32_t)c->groups.size();
  const uint64_t step = std::max<uint64_t>(1, k1_items / 16384);
  const uint64_t nsamp = (k1_items + step - 1) / step;
  HIP_TRY(hipMemsetAsync(c->d_hits, 0, sizeof(uint32_t) * ns, c->stream));
  K1Args A{c->d_data, c->d_off, c->d_chunk_file, c->total, nchunks, nsamp, step, c->opt.chunk_bytes,
           c->nfiles, c->d_kw, c->d_ev, c->d_hits, k1_streams(), (uint32_t)kK1Seg};
  int rc;
  if ((rc = launch_k1(c, A))) return rc;
  std::vector<uint32_t> hits(ns);
  HIP_TRY(hipMemcpyAsync(hits.data(), c->d_hits, sizeof(uint32_t) * ns, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->adapted = true;
  const uint64_t sample_bytes = nsamp * A.streams * A.seg * c->opt.chunk_bytes;
  uint64_t total = 0;
  std::vector<uint32_t> order;
  for (uint32_t s = 0; s < ns; s++)
    if (hits[s]) {
      total += hits[s];
      order.push_back(s);
    }
  std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return hits[a] > hits[b]; });
  const uint64_t budget = sample_bytes / 4096;
  std::vector<uint8_t> hot(p.kw_dfa->nstates, 0);  // automaton states that stop reporting
  std::vector<uint8_t> kw_unknown(p.n_kw, 0);
  uint32_t ev_hot = 0, nhot = 0;
  for (uint32_t s : order) {  // s: device state id
    if (total <= budget) break;
    const uint32_t* m = c->k1h.masks.data() + (size_t)c->k1h.accs[s] * mw;
    bool fallback = false;  // folding-rune literals must stay exact (they force host resolution)
    for (int k = p.fb_kw0; k < p.n_kw; k++) fallback |= (m[k / 32] >> (k % 32)) & 1;
    if (fallback) continue;
    hot[c->k1h.order[s]] = 1;
    nhot++;
    total -= hits[s];
    for (int k = 0; k < p.n_kw; k++)
      if ((m[k / 32] >> (k % 32)) & 1) kw_unknown[k] = 1;
    ev_hot |= m[W];
  }
  c->hot_states = nhot;
  if (!nhot) return TSG_OK;
  int rc2;
  if ((rc2 = k1_tables(p, hot, &c->k1h, &c->k1.start, &c->k1.acc_row))) return rc2;
  HIP_TRY(hipMemcpy((void*)c->k1.tab, c->k1h.tab.data(), c->k1h.tab.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy((void*)c->k1.accs, c->k1h.accs.data(), c->k1h.accs.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
  // gates of groups with an unknown keyword open; events of hot anchor literals fire everywhere
  std::vector<uint32_t> galways = c->h_galways, gevents = c->h_gevents;
  std::vector<unsigned long long> gofbit = c->h_gofbit;
  for (uint32_t g = 0; g < G; g++) {
    for (uint32_t r : p.groups[g].rules)
      if (p.rule_kw_mode[r] == kKwBits)
        for (uint32_t k : p.rule_kws[r])
          if (kw_unknown[k]) galways[g] = 1;
    if (gevents[g] & ev_hot) {
      gevents[g] |= kEvAlways;
      gofbit[31 * c->GW + g / 64] |= 1ull << (g % 64);
    }
  }
  HIP_TRY(hipMemcpy(c->d_galways, galways.data(), sizeof(uint32_t) * G, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(c->d_gevents, gevents.data(), sizeof(uint32_t) * G, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(c->d_gofbit, gofbit.data(), sizeof(unsigned long long) * gofbit.size(), hipMemcpyHostToDevice));
  c->kw_unknown = kw_unknown;
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
  // The per-batch host buffers (keyword bits, result vectors, serialized results) are
  // tens of MB: keep such blocks on the heap (reused, already faulted in) instead of
  // fresh mmap'ed pages for every batch.
  static std::once_flag heap_once;
  std::call_once(heap_once, [] {
    mallopt(M_MMAP_THRESHOLD, 32 << 20);
    mallopt(M_TRIM_THRESHOLD, 1 << 30);
  });
  for (auto& e : c->ev) HIP_TRY(hipEventCreate(&e));
  const Plan& p = *rs->plan;
  const uint32_t W = (uint32_t)p.kw_words;
  const uint32_t chunk = c->opt.chunk_bytes;
  if (p.warm > kPad) return fail(TSG_ERR_CONFIG, "a keyword is longer than the K1 warm-up window");
  int rc;
  if ((rc = make_device_k1(p, &c->k1, &c->tables, &c->k1h))) return rc;
  HIP_TRY(hipMalloc((void**)&c->d_hits, sizeof(uint32_t) * c->k1.ns));
  if (const DFA* pd = p.allow_path_dfa.get()) {
    const uint32_t* t = nullptr;
    if ((rc = upload_vec(pd->next, &t, &c->tables))) return rc;
    c->pathdfa.next = t;
    if ((rc = upload_vec(pd->acc, &t, &c->tables))) return rc;
    c->pathdfa.acc = t;
    if ((rc = upload_vec(pd->eot_acc, &t, &c->tables))) return rc;
    c->pathdfa.eot = t;
    const uint8_t* cl = nullptr;
    if ((rc = upload_vec(std::vector<uint8_t>(pd->cls, pd->cls + 256), &cl, &c->tables))) return rc;
    c->pathdfa.cls = cl;
    c->pathdfa.nc = (uint32_t)pd->nclasses;
    c->pathdfa.start = pd->start[kCtxBOT];
    c->has_pathdfa = true;
  }
  const uint32_t G = (uint32_t)p.groups.size();
  c->GW = std::max<uint32_t>(1, (G + 63) / 64);
  std::vector<uint32_t> gmask, galways, gevents;
  std::vector<unsigned long long> gofbit(32 * c->GW, 0);
  uint32_t max_lds = 0;
  for (uint32_t g = 0; g < G; g++) {
    const auto& gp = p.groups[g];
    DevDFA dd{};
    if ((rc = make_device_dfa(*gp.dfa, gp.rules, &dd, &c->tables))) return rc;
    max_lds = std::max(max_lds, dd.lds_bytes);
    c->groups.push_back(dd);
    gmask.insert(gmask.end(), gp.kwmask.begin(), gp.kwmask.end());
    galways.push_back(gp.always ? 1 : 0);
    gevents.push_back(gp.events);
    uint32_t back = group_back(gp, chunk);
    if (back > (uint32_t)kMaxBack) back = kMaxBack + 1;
    c->gback.push_back(back);
    if (back <= (uint32_t)kMaxBack) c->maxback = std::max(c->maxback, back);
    for (int b = 0; b < 32; b++)
      if (((gp.events >> b) & 1) || back > (uint32_t)kMaxBack) gofbit[b * c->GW + g / 64] |= 1ull << (g % 64);
  }
  if (max_lds > 64 * 1024) {
    HIP_TRY(hipFuncSetAttribute((const void*)k2_list_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)max_lds));
    HIP_TRY(hipFuncSetAttribute((const void*)k2_dense_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)max_lds));
  }
  const uint32_t* cg = nullptr;
  if ((rc = upload_vec(gmask, &cg, &c->tables))) return rc;
  c->d_gmask = (uint32_t*)cg;
  if ((rc = upload_vec(galways, &cg, &c->tables))) return rc;
  c->d_galways = (uint32_t*)cg;
  if ((rc = upload_vec(gevents, &cg, &c->tables))) return rc;
  c->d_gevents = (uint32_t*)cg;
  if ((rc = upload_vec(c->gback, &cg, &c->tables))) return rc;
  c->d_gback = (uint32_t*)cg;
  const unsigned long long* cb = nullptr;
  if ((rc = upload_vec(gofbit, &cb, &c->tables))) return rc;
  c->h_galways = galways;
  c->h_gevents = gevents;
  c->h_gofbit = gofbit;
  c->d_gofbit = (unsigned long long*)cb;
  const DevDFA* cd = nullptr;
  if ((rc = upload_vec(c->groups, &cd, &c->tables))) return rc;
  c->d_groups = (DevDFA*)cd;
  HIP_TRY(hipMalloc((void**)&c->d_cand, sizeof(DevCand) * c->opt.cand_capacity));
  HIP_TRY(hipMalloc((void**)&c->d_count, sizeof(uint32_t) * 4));
  HIP_TRY(hipMalloc((void**)&c->d_gcount, sizeof(uint32_t) * (G + 1)));
  HIP_TRY(hipMalloc((void**)&c->d_cursor, sizeof(uint32_t) * (G + 1)));
  HIP_TRY(hipMalloc((void**)&c->d_base, sizeof(uint64_t) * (G + 1)));
  HIP_TRY(hipMalloc((void**)&c->d_listed, G + 1));
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
  if (total && !data) return fail(TSG_ERR_ARG, "bad argument");
  const uint32_t chunk = c->opt.chunk_bytes;
  if (total / chunk >= (1ull << 32) - 2) return fail(TSG_ERR_ARG, "batch too large for u32 chunk ids");
  int rc;
  // front pad: K1 warm-up reads before the first chunk; tail: whole K1 items + look-ahead
  const size_t tail = (size_t)kK1MaxStreams * kK1Seg * chunk + kPad;
  if (c->d_data_cap < (size_t)total + kPad + tail || !c->d_data_alloc) {
    if (c->d_data_alloc) HIP_TRY(hipFree(c->d_data_alloc));
    c->d_data_alloc = nullptr;
    HIP_TRY(hipMalloc((void**)&c->d_data_alloc, (size_t)total + kPad + tail));
    c->d_data_cap = (size_t)total + kPad + tail;
  }
  c->d_data = c->d_data_alloc + kPad;
  if ((rc = ensure(&c->d_off, &c->d_off_cap, (size_t)nfiles + 1))) return rc;
  const uint64_t nchunks = (total + chunk - 1) / chunk;
  // K1 items are kStreams chunks: chunk-indexed arrays are padded to whole items
  const uint64_t k1_item_chunks = (uint64_t)kK1MaxStreams * kK1Seg;
  const uint64_t nchunks_pad = (nchunks + k1_item_chunks - 1) / k1_item_chunks * k1_item_chunks + 1;
  if ((rc = ensure(&c->d_chunk_file, &c->d_chunk_cap, (size_t)nchunks_pad))) return rc;
  if ((rc = ensure(&c->d_ev, &c->d_ev_cap, (size_t)nchunks_pad))) return rc;
  if ((rc = ensure(&c->d_evlist, &c->d_evlist_cap, (size_t)nchunks_pad))) return rc;
  const int W = c->rs->plan->kw_words;
  if ((rc = ensure(&c->d_kw, &c->d_kw_cap, (size_t)nfiles * W + 1))) return rc;
  if ((rc = ensure(&c->d_ggate, &c->d_ggate_cap, (size_t)nfiles * c->GW + 1))) return rc;
  if ((rc = ensure(&c->d_ovf, &c->d_ovf_cap, (size_t)nfiles + 1))) return rc;
  HIP_TRY(hipMemsetAsync(c->d_data_alloc, 0, kPad, c->stream));
  if (total) HIP_TRY(hipMemcpyAsync(c->d_data, data, total, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemsetAsync(c->d_data + total, 0, tail, c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_off, offsets, sizeof(uint64_t) * (nfiles + 1), hipMemcpyHostToDevice, c->stream));
  if (c->has_pathdfa && nfiles) {
    const uint64_t pbytes = path_offsets[nfiles];
    if ((rc = ensure(&c->d_paths, &c->d_paths_cap, (size_t)pbytes + 1))) return rc;
    if ((rc = ensure(&c->d_poff, &c->d_poff_cap, (size_t)nfiles + 1))) return rc;
    if ((rc = ensure(&c->d_pathok, &c->d_pathok_cap, (size_t)nfiles))) return rc;
    if (pbytes) HIP_TRY(hipMemcpyAsync(c->d_paths, paths, pbytes, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_poff, path_offsets, sizeof(uint64_t) * (nfiles + 1), hipMemcpyHostToDevice,
                           c->stream));
  }
  HIP_TRY(hipMemsetAsync(c->d_chunk_file, 0, sizeof(uint32_t) * nchunks_pad, c->stream));
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
  HIP_TRY(hipMemsetAsync(c->d_gcount, 0, sizeof(uint32_t) * (G + 1), st));
  HIP_TRY(hipMemsetAsync(c->d_cursor, 0, sizeof(uint32_t) * (G + 1), st));
  HIP_TRY(hipEventRecord(c->ev[1], st));

  // ---- K1
  const uint32_t k1s = k1_streams();
  const uint64_t k1_items = (nchunks + (uint64_t)k1s * kK1Seg - 1) / ((uint64_t)k1s * kK1Seg);
  int rc;
  const uint64_t adapt_bytes = c->opt.adapt_mib == 0xFFFFFFFFu ? ~0ull
                               : (uint64_t)(c->opt.adapt_mib ? c->opt.adapt_mib : 64) << 20;
  if (!c->adapted && k1_items >= 64 && c->total >= adapt_bytes)
    if ((rc = adapt_k1(c, nchunks, k1_items))) return rc;
  if (k1_items) {
    K1Args A{c->d_data, c->d_off, c->d_chunk_file, c->total, nchunks, k1_items, 1, chunk, F, c->d_kw, c->d_ev,
             nullptr, k1s, (uint32_t)kK1Seg};
    if ((rc = launch_k1(c, A))) return rc;
  }
  HIP_TRY(hipEventRecord(c->ev[2], st));

  // ---- gate + item counts
  std::vector<uint32_t> gcount(G, 0);
  ItemArgs IA{};
  IA.off = c->d_off;
  IA.chunk_file = c->d_chunk_file;
  IA.ev = c->d_ev;
  IA.ggate = c->d_ggate;
  IA.gofbit = c->d_gofbit;
  IA.gevents = c->d_gevents;
  IA.gback = c->d_gback;
  IA.nchunks = nchunks;
  IA.F = F;
  IA.G = G;
  IA.GW = c->GW;
  IA.chunk = chunk;
  IA.maxback = c->maxback;
  IA.count = c->d_gcount;
  IA.cursor = c->d_cursor;
  IA.listed = c->d_listed;
  IA.evlist = c->d_evlist;
  IA.nev = c->d_count + 1;
  int igrid = 0;
  if (F && G && nchunks) {
    if (c->has_pathdfa) {
      path_allow_kernel<<<(F + 255) / 256, 256, 0, st>>>(c->pathdfa, c->d_paths, c->d_poff, F, c->d_pathok);
      HIP_TRY(hipGetLastError());
    }
    ggate_kernel<<<(F + 255) / 256, 256, 0, st>>>(c->d_kw, F, W, c->d_gmask, c->d_galways, G, c->GW, c->d_ggate);
    HIP_TRY(hipGetLastError());
    const uint32_t cgrid = (uint32_t)std::min<uint64_t>((nchunks + kBlock - 1) / kBlock, (uint64_t)c->grid);
    ev_compact_kernel<<<cgrid, kBlock, 0, st>>>(c->d_ev, nchunks, c->d_evlist, c->d_count + 1);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(c->h_count + 1, c->d_count + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    igrid = (int)(((uint64_t)c->h_count[1] + F + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(items_count_kernel, dim3(igrid), dim3(kBlock), G * sizeof(uint32_t) + 16, st, IA);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(gcount.data(), c->d_gcount, sizeof(uint32_t) * G, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  // DENSE when a group's items cover a large share of the batch, LIST otherwise
  std::vector<uint32_t> dense;
  std::vector<uint64_t> base(G, 0);
  std::vector<uint8_t> listed(G, 0);
  std::vector<uint4> blkmap;
  uint64_t nitems = 0, k2_bytes = 0;
  uint32_t list_lds = 0;
  const uint32_t per_block = kBlock * 2;
  for (uint32_t g = 0; g < G; g++) {
    if (gcount[g] == 0) continue;
    k2_bytes += (uint64_t)gcount[g] * chunk;
    if ((uint64_t)gcount[g] * 2 > nchunks || nitems + gcount[g] >= (1ull << 31)) {
      dense.push_back(g);
      continue;
    }
    listed[g] = 1;
    base[g] = nitems;
    for (uint32_t first = 0; first < gcount[g]; first += per_block)
      blkmap.push_back(make_uint4(g, (uint32_t)nitems + first, std::min(per_block, gcount[g] - first), 0));
    nitems += gcount[g];
    list_lds = std::max(list_lds, c->groups[g].lds_bytes);
  }
  if (nitems) {
    if ((rc = ensure(&c->d_items, &c->d_items_cap, (size_t)nitems))) return rc;
    if ((rc = ensure(&c->d_blkmap, &c->d_blkmap_cap, blkmap.size()))) return rc;
    HIP_TRY(hipMemcpyAsync(c->d_base, base.data(), sizeof(uint64_t) * G, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(c->d_listed, listed.data(), G, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(c->d_blkmap, blkmap.data(), sizeof(uint4) * blkmap.size(), hipMemcpyHostToDevice, st));
    IA.base = c->d_base;
    IA.items = c->d_items;
    hipLaunchKernelGGL(items_emit_kernel, dim3(igrid), dim3(kBlock), 2 * G * sizeof(uint32_t) + 16, st, IA);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipEventRecord(c->ev[3], st));

  // ---- K2
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
  if (nitems) {
    ScanArgsDev B = A;
    B.items = c->d_items;
    B.nitems = nitems;
    hipLaunchKernelGGL(k2_list_kernel, dim3((uint32_t)blkmap.size()), dim3(kBlock), list_lds, st,
                       (const DevDFA*)c->d_groups, (const uint4*)c->d_blkmap, B);
    HIP_TRY(hipGetLastError());
  }
  for (uint32_t g : dense) {
    ScanArgsDev B = A;
    B.nitems = (nchunks + kStreams - 1) / kStreams;
    B.gmask = c->d_gmask + (size_t)g * W;
    B.galways = p.groups[g].always ? 1 : 0;
    const int grid = (int)std::min<uint64_t>((B.nitems + kBlock - 1) / kBlock, (uint64_t)c->grid);
    hipLaunchKernelGGL(k2_dense_kernel, dim3(grid), dim3(kBlock), c->groups[g].lds_bytes, st, c->groups[g], B);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipEventRecord(c->ev[4], st));
  HIP_TRY(hipMemcpyAsync(c->h_count, c->d_count, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  uint32_t n = std::min(*c->h_count, c->opt.cand_capacity);
  c->ko.cand.resize(n);
  c->ko.kw.resize((size_t)F * W);
  std::vector<uint32_t>& ovf = c->h_ovf;
  ovf.resize(F);
  if (n) HIP_TRY(hipMemcpyAsync(c->ko.cand.data(), c->d_cand, sizeof(DevCand) * n, hipMemcpyDeviceToHost, st));
  if (F) {
    HIP_TRY(hipMemcpyAsync(c->ko.kw.data(), c->d_kw, sizeof(uint32_t) * (size_t)F * W, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(ovf.data(), c->d_ovf, sizeof(uint32_t) * F, hipMemcpyDeviceToHost, st));
  }
  if (!(F && c->has_pathdfa)) c->ko.path_ok.clear();
  if (F && c->has_pathdfa) {
    c->ko.path_ok.resize(F);
    HIP_TRY(hipMemcpyAsync(c->ko.path_ok.data(), c->d_pathok, F, hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(hipEventRecord(c->ev[5], st));
  HIP_TRY(hipStreamSynchronize(st));
  c->ko.kw_unknown = c->kw_unknown;
  c->ko.overflow.resize(F);
  for (uint32_t i = 0; i < F; i++) c->ko.overflow[i] = ovf[i] ? 1 : 0;
  float t[5] = {0, 0, 0, 0, 0};
  for (int k = 0; k < 5; k++) HIP_TRY(hipEventElapsedTime(&t[k], c->ev[k], c->ev[k + 1]));
  c->stats.k1_ms = t[1];
  c->stats.gate_ms = t[2];
  c->stats.k2_ms = t[3];
  c->stats.aux_ms = t[0] + t[4];
  c->stats.bytes = c->total;
  c->stats.k2_bytes = k2_bytes;
  c->stats.k2_items = nitems;
  c->stats.candidates = *c->h_count;
  c->stats.overflow = *c->h_count > c->opt.cand_capacity ? 1 : 0;
  c->stats.k2_launches = (uint32_t)(dense.size() + (nitems ? 1 : 0));
  c->stats.k1_hot_states = c->hot_states;
  return TSG_OK;
}

// Host resolution of one batch's kernel output (exact findings, serialized).
static std::unique_ptr<tsg_result> resolve_job(const tsg_ruleset* rs, BatchView b, const KernelOutput& ko,
                                               int nt, std::pair<double, uint64_t>* done) {
  auto t0 = std::chrono::steady_clock::now();
  BatchResult res;
  resolve_batch(rs->rs, *rs->plan, b, ko, nt, &res);
  auto t1 = std::chrono::steady_clock::now();
  auto r = std::make_unique<tsg_result>();
  serialize_batch(res, &r->buf, nt);
  if (getenv("TSG_PROF"))
    fprintf(stderr, "resolve_job: resolve_batch %.1f ms, serialize %.1f ms\n",
            std::chrono::duration<double, std::milli>(t1 - t0).count(),
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count());
  done->first = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  done->second = 0;
  for (uint8_t st : res.status) done->second += st == kHasFindings;
  return r;
}

int tsg_batch_submit(tsg_ctx* c) {
  if (!c) return fail(TSG_ERR_ARG, "bad argument");
  int rc = tsg_batch_kernels(c);
  if (rc) return rc;
  try {
    tsg_ctx::Pending pj;
    pj.done = std::make_shared<std::pair<double, uint64_t>>(0.0, 0);
    // the batch's output goes to a pooled KernelOutput no pending job holds; c->ko gets
    // that entry's buffers back, so the next batch reuses their pages (no allocation and
    // no page faults for the tens of MB of keyword bits per batch)
    std::shared_ptr<KernelOutput> ko;
    for (auto& e : c->ko_pool)
      if (e.use_count() == 1) {
        ko = e;
        break;
      }
    if (!ko) {
      ko = std::make_shared<KernelOutput>();
      c->ko_pool.push_back(ko);
    }
    std::swap(*ko, c->ko);
    BatchView b{c->h_data, c->h_off, c->nfiles, c->h_paths, c->h_poff};
    const tsg_ruleset* rs = c->rs;
    const int nt = c->opt.host_threads > 0 ? c->opt.host_threads : 16;
    auto done = pj.done;
    pj.res = std::async(std::launch::async, [rs, b, ko, nt, done]() { return resolve_job(rs, b, *ko, nt, done.get()); });
    c->pending.push_back(std::move(pj));
    return TSG_OK;
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& ex) {
    return fail(TSG_ERR_INTERNAL, ex.what());
  }
}

int tsg_batch_collect(tsg_ctx* c, tsg_result** out) {
  if (!c || !out) return fail(TSG_ERR_ARG, "bad argument");
  if (c->pending.empty()) return fail(TSG_ERR_ARG, "no submitted batch");
  tsg_ctx::Pending pj = std::move(c->pending.front());
  c->pending.pop_front();
  try {
    std::unique_ptr<tsg_result> r = pj.res.get();
    c->stats.resolve_ms = pj.done->first;
    c->stats.files_resolved = pj.done->second;
    *out = r.release();
    return TSG_OK;
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& ex) {
    return fail(TSG_ERR_INTERNAL, ex.what());
  }
}

int tsg_batch_pending(const tsg_ctx* c) { return c ? (int)c->pending.size() : TSG_ERR_ARG; }

int tsg_batch_scan(tsg_ctx* c, tsg_result** out) {
  if (!c || !out) return fail(TSG_ERR_ARG, "bad argument");
  if (!c->pending.empty()) return fail(TSG_ERR_ARG, "collect the submitted batches first");
  int rc = tsg_batch_submit(c);
  if (rc) return rc;
  return tsg_batch_collect(c, out);
}

int tsg_scan_batch(tsg_ctx* c, const uint8_t* data, const uint64_t* offsets, uint32_t nfiles,
                   const char* paths, const uint64_t* path_offsets, tsg_result** out) {
  int rc = tsg_batch_upload(c, data, offsets, nfiles, paths, path_offsets);
  if (rc) return rc;
  return tsg_batch_scan(c, out);
}

int tsg_batch_k1_output(tsg_ctx* c, uint32_t* kw, size_t kw_len, uint32_t* ev, size_t ev_len) {
  if (!c || !c->uploaded) return fail(TSG_ERR_ARG, "no batch uploaded");
  HIP_TRY(hipSetDevice(c->device));
  const uint64_t nchunks = (c->total + c->opt.chunk_bytes - 1) / c->opt.chunk_bytes;
  if (kw) std::memcpy(kw, c->ko.kw.data(), sizeof(uint32_t) * std::min(kw_len, c->ko.kw.size()));
  if (ev && nchunks)
    HIP_TRY(hipMemcpy(ev, c->d_ev, sizeof(uint32_t) * std::min<uint64_t>(ev_len, nchunks), hipMemcpyDeviceToHost));
  return TSG_OK;
}

int tsg_ctx_get_stats(const tsg_ctx* c, tsg_stats* out) {
  if (!c || !out) return fail(TSG_ERR_ARG, "bad argument");
  *out = c->stats;
  return TSG_OK;
}

}  // extern "C"
