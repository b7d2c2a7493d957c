// K1F cost bisection (round 6 measurement, not product code).
//
// k1f_kernel (kernels.hip) runs one 1,024-thread block per CU, every wave streaming its own
// range of 1 KiB tiles with four tiles in flight in registers.  Its loop alone (loads, no
// filter) streams 0.976 GB in 0.154 ms (tools/stream_floor.hip, reg4), the whole kernel
// takes 0.25 ms, and without its tile loads (K1F_NOLOAD) it takes the same.  This program
// adds K1F's pieces to that loop one at a time, on a text-like 1 GiB batch with a filter
// table of the product's shape (random bucket bits, the run flags of alnum / digit bytes):
//   V0  loads only (XOR of the words)
//   V1  + the 16 entry reads per tile (ds_read_b128, replicated layout), ANDed together
//   V2  + the window ANDs and the bucket union per word, ballot of listed words
//   V3  + the run flags and run events (k1f_flags / k1f_runs, DPP look-behind), ballots
//   V4  V3 with the 16 entries of a tile read at once
//   V5  V3 without the cross-lane look-behind (the DPP moves)
//   V6  V3 with each tile consumed before its queue register is reloaded (no register
//       copies at the loop's back edge, so no vmcnt(0) there)
//   V7  V6 with two copies of the table in LDS, the waves of SIMDs {0,1} reading one and
//       those of {2,3} the other
//   V8  V6 with three of four waves starting ~8 us late (staggered phases)
// and times each (V3 also at 512 threads per block, one and two blocks per CU); V3 stamps
// the shader clock against the 100 MHz wall clock.  L64_*: the same work with each lane
// holding 64 contiguous bytes (lab64_k), the per-word overheads (look-behind, run flags of
// the neighbours) paid once per 64 B instead of per 16 B.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I trivy_amd/csrc -I include \
//          -o tools/k1f_lab tools/k1f_lab.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "k1f.hpp"

#define CHECK(x)                                              \
  do {                                                        \
    hipError_t e = (x);                                       \
    if (e != hipSuccess) {                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
      exit(1);                                                \
    }                                                         \
  } while (0)

using namespace tsg;
constexpr uint32_t kTile = 1024;
constexpr size_t kBytes = 1ull << 30;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
  const u32x4 v = __builtin_nontemporal_load((const u32x4*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t shr1(uint32_t v, uint32_t old) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t ror1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x13C, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t prev(uint32_t cur, uint32_t p) { return shr1(cur, ror1(p)); }
__device__ __forceinline__ uint32_t prev_none(uint32_t cur, uint32_t p) { return cur ^ p; }

struct Carry {
  uint32_t a, b, c, m, m1;
};

template <int V>
struct Lane {
  __device__ __forceinline__ uint32_t prev(uint32_t cur, uint32_t p) const {
    if constexpr (V == 5) return prev_none(cur, p);  // (V6 keeps the DPP)
    return ::prev(cur, p);
  }
  const uint8_t* smem;
  uint32_t lane16;
  __device__ __forceinline__ uint4 entry(uint32_t w, int k) const {
    return *(const uint4*)(smem + __builtin_amdgcn_perm(w, lane16, 0x0C0C0000u | ((4u + (uint32_t)k) << 8)));
  }
  // V4: V3's logic with all 16 entries read at once (one LDS round trip per tile)
  __device__ __forceinline__ uint32_t tile16(uint4 v, Carry& cy, uint32_t& un) const {
    uint4 e[16];
#pragma unroll
    for (int k = 0; k < 16; k++) e[k] = entry(k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w, k & 3);
    const uint32_t ao = k1f_and3(e[13].x, e[14].y, e[15].z), bo = e[14].x & e[15].y, co = e[15].x;
    const uint32_t ai = prev(ao, cy.a), bi = prev(bo, cy.b), ci = prev(co, cy.c);
    cy.a = ao;
    cy.b = bo;
    cy.c = co;
    uint32_t r[16];
    r[0] = ai & e[0].w;
    r[1] = k1f_and3(bi, e[0].z, e[1].w);
    r[2] = k1f_and3(ci, e[0].y, e[1].z) & e[2].w;
#pragma unroll
    for (int k = 3; k < 16; k++) r[k] = k1f_and3(e[k - 3].x, e[k - 2].y, e[k - 1].z) & e[k].w;
    uint32_t g[4];
#pragma unroll
    for (int i = 0; i < 4; i++) g[i] = k1f_or3(r[4 * i], r[4 * i + 1], r[4 * i + 2]) | r[4 * i + 3];
    un = k1f_or3(g[0], g[1], g[2]) | g[3];
    const uint32_t m = k1f_flags(r[3], r[7], r[11], r[15]);
    const uint32_t m1 = prev(m, cy.m), m2 = prev(m1, cy.m1);
    cy.m = m;
    cy.m1 = m1;
    return k1f_runs(m, m1, m2);
  }
  // one 16-B sub-word of a lane's 64 contiguous bytes (lab64_k): look-behind partials in
  // (ai, bi, ci), its own bytes 13..15's partials out (for the next sub-word), the bucket
  // union and the run flags m (k1f_flags)
  __device__ __forceinline__ void sub(uint4 v, uint32_t& ai, uint32_t& bi, uint32_t& ci, uint32_t& un,
                                      uint32_t& m) const {
    uint32_t r[16];
    {
      uint4 e[8];
#pragma unroll
      for (int k = 0; k < 8; k++) e[k] = entry(k < 4 ? v.x : v.y, k & 3);
      r[0] = ai & e[0].w;
      r[1] = k1f_and3(bi, e[0].z, e[1].w);
      r[2] = k1f_and3(ci, e[0].y, e[1].z) & e[2].w;
#pragma unroll
      for (int k = 3; k < 8; k++) r[k] = k1f_and3(e[k - 3].x, e[k - 2].y, e[k - 1].z) & e[k].w;
      r[8] = k1f_and3(e[5].x, e[6].y, e[7].z);
      r[9] = e[6].x & e[7].y;
      r[10] = e[7].x;
    }
    __builtin_amdgcn_sched_barrier(0);
    {
      uint4 e[8];
#pragma unroll
      for (int k = 0; k < 8; k++) e[k] = entry(k < 4 ? v.z : v.w, k & 3);
      r[8] &= e[0].w;
      r[9] = k1f_and3(r[9], e[0].z, e[1].w);
      r[10] = k1f_and3(r[10], e[0].y, e[1].z) & e[2].w;
#pragma unroll
      for (int k = 3; k < 8; k++) r[8 + k] = k1f_and3(e[k - 3].x, e[k - 2].y, e[k - 1].z) & e[k].w;
      ai = k1f_and3(e[5].x, e[6].y, e[7].z);
      bi = e[6].x & e[7].y;
      ci = e[7].x;
    }
    uint32_t g[4];
#pragma unroll
    for (int i = 0; i < 4; i++) g[i] = k1f_or3(r[4 * i], r[4 * i + 1], r[4 * i + 2]) | r[4 * i + 3];
    un = k1f_or3(g[0], g[1], g[2]) | g[3];
    m = k1f_flags(r[3], r[7], r[11], r[15]);
  }
  // returns run bits (V3) and the bucket union (V>=2) / AND of everything (V1)
  __device__ __forceinline__ uint32_t tile(uint4 v, Carry& cy, uint32_t& un) const {
    if constexpr (V == 1) {
      uint32_t x = ~0u;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const uint4 e = entry(k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w, k & 3);
        x = k1f_and3(x, e.x, e.y) & e.z & e.w;
      }
      un = x;
      return 0;
    } else {
      const uint4 e13 = entry(v.w, 1), e14 = entry(v.w, 2), e15 = entry(v.w, 3);
      const uint32_t ao = k1f_and3(e13.x, e14.y, e15.z), bo = e14.x & e15.y, co = e15.x;
      const uint32_t ai = prev(ao, cy.a), bi = prev(bo, cy.b), ci = prev(co, cy.c);
      cy.a = ao;
      cy.b = bo;
      cy.c = co;
      uint32_t r[16];
      __builtin_amdgcn_sched_barrier(0);
      {
        uint4 e[8];
#pragma unroll
        for (int k = 0; k < 8; k++) e[k] = entry(k < 4 ? v.x : v.y, k & 3);
        r[0] = ai & e[0].w;
        r[1] = k1f_and3(bi, e[0].z, e[1].w);
        r[2] = k1f_and3(ci, e[0].y, e[1].z) & e[2].w;
#pragma unroll
        for (int k = 3; k < 8; k++) r[k] = k1f_and3(e[k - 3].x, e[k - 2].y, e[k - 1].z) & e[k].w;
        r[8] = k1f_and3(e[5].x, e[6].y, e[7].z);
        r[9] = e[6].x & e[7].y;
        r[10] = e[7].x;
      }
      __builtin_amdgcn_sched_barrier(0);
      {
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
      uint32_t g[4];
#pragma unroll
      for (int i = 0; i < 4; i++) g[i] = k1f_or3(r[4 * i], r[4 * i + 1], r[4 * i + 2]) | r[4 * i + 3];
      un = k1f_or3(g[0], g[1], g[2]) | g[3];
      if constexpr (V == 2) return 0;
      const uint32_t m = k1f_flags(r[3], r[7], r[11], r[15]);
      const uint32_t m1 = prev(m, cy.m), m2 = prev(m1, cy.m1);
      cy.m = m;
      cy.m1 = m1;
      return k1f_runs(m, m1, m2);
    }
  }
};

template <int V>
__global__ void __launch_bounds__(1024) lab_k(const uint8_t* data, const uint4* ent, uint32_t ntiles,
                                               uint32_t* out, unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[V == 7 ? 131072 : 65536];
  long long c0 = 0, w0 = 0;
  if (V == 3 && blockIdx.x == 0 && threadIdx.x == 0) {
    c0 = clock64();
    w0 = wall_clock64();
  }
  if (V >= 1) {
    for (uint32_t i = threadIdx.x; i < (V == 7 ? 8192u : 4096u); i += blockDim.x) ((uint4*)smem)[i] = ent[(i & 4095) >> 4];
    __syncthreads();
  }
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wpb = blockDim.x >> 6;
  const uint32_t gw = blockIdx.x * wpb + wave, nw = gridDim.x * wpb;
  const uint32_t t0 = (uint32_t)((uint64_t)gw * ntiles / nw), t1 = (uint32_t)((uint64_t)(gw + 1) * ntiles / nw);
  // V7: the table copy of the wave's SIMD half (HW_ID bits 5:4 = SIMD)
  const uint32_t simd = ((uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11)) >> 4) & 3u;
  const Lane<V> L{smem + (V == 7 ? (simd >> 1) * 65536u : 0u), (lane & 15u) << 4};
  if (V == 8 && (wave & 3)) __builtin_amdgcn_s_sleep(127);  // staggered starts (127 x 64 cycles)
  Carry cy{0, 0, 0, 0, 0};
  uint32_t acc = 0, nl = 0, nr = 0;
  const uint8_t* base = data + 16u * lane;
  auto body = [&](uint4 v) __attribute__((always_inline)) {
    if constexpr (V == 0) {
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    } else {
      uint32_t un;
      const uint32_t rb = V == 4 ? L.tile16(v, cy, un) : L.tile(v, cy, un);  // (V6: V3's tile)
      if constexpr (V == 1) {
        acc ^= un;
      } else {
        const uint64_t hb = __ballot((un & 0xFFFFu) != 0);
        if (__builtin_expect(hb != 0, 0)) nl += (uint32_t)__popcll(hb);
        if constexpr (V >= 3) {
          const uint64_t bu = __ballot(rb & 1u), bd = __ballot(rb & 2u);
          if (__builtin_expect((bu | bd) != 0, 0)) nr += (uint32_t)__popcll(bu | bd);
        }
      }
    }
  };
  constexpr int D = 4;
  uint4 p[D];
#pragma unroll
  for (int k = 0; k < D; k++) p[k] = ld16(base + (size_t)(t0 + k) * kTile);
  uint32_t t = t0;
  for (; t + D <= t1; t += D) {
#pragma unroll
    for (int k = 0; k < D; k++) {
      if constexpr (V >= 6) {  // the tile consumed before its register is reloaded: no copies
        body(p[k]);
        p[k] = ld16(base + (size_t)(t + D + k) * kTile);
      } else {
        const uint4 v = p[k];
        p[k] = ld16(base + (size_t)(t + D + k) * kTile);
        body(v);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < D - 1; k++)
    if (t + k < t1) body(p[k]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc + nl + nr;
  if (V == 3 && blockIdx.x == 0 && threadIdx.x == 0 && blockDim.x == 1024) {
    clk[0] = clock64() - c0;
    clk[1] = wall_clock64() - w0;
  }
}

// lane-contiguous 64 B: 4 KiB tiles, lane l's bytes [64 l, 64 l + 64) by four 16-B loads
// (each load instruction of the wave covers its 4 KiB at a 64-B stride); one tile in flight.
// V0: loads only; V1: the filter and run flags of the four sub-words, the look-behind from
// the previous lane once per 64 B (DPP), the run events of the four sub-words from their
// flags in registers
template <int V>
__global__ void __launch_bounds__(1024) lab64_k(const uint8_t* data, const uint4* ent, uint32_t ntiles,
                                                 uint32_t* out, unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[65536];
  if (V >= 1) {
    for (uint32_t i = threadIdx.x; i < 4096; i += blockDim.x) ((uint4*)smem)[i] = ent[i >> 4];
    __syncthreads();
  }
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wpb = blockDim.x >> 6;
  const uint32_t gw = blockIdx.x * wpb + wave, nw = gridDim.x * wpb;
  const uint32_t nt4 = ntiles / 4;
  const uint32_t t0 = (uint32_t)((uint64_t)gw * nt4 / nw), t1 = (uint32_t)((uint64_t)(gw + 1) * nt4 / nw);
  const Lane<3> L{smem, (lane & 15u) << 4};
  uint32_t ca = 0, cb = 0, cc = 0, cm3 = 0, cm2 = 0;
  uint32_t acc = 0, nl = 0, nr = 0;
  const uint8_t* base = data + 64u * lane;
  auto body = [&](const uint4 (&v)[4]) __attribute__((always_inline)) {
    if constexpr (V == 0) {
#pragma unroll
      for (int k = 0; k < 4; k++) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    } else {
      // the last sub-word's bytes 13..15: the next lane's look-behind
      const uint4 e13 = L.entry(v[3].w, 1), e14 = L.entry(v[3].w, 2), e15 = L.entry(v[3].w, 3);
      const uint32_t ao = k1f_and3(e13.x, e14.y, e15.z), bo = e14.x & e15.y, co = e15.x;
      uint32_t ai = prev(ao, ca), bi = prev(bo, cb), ci = prev(co, cc);
      ca = ao;
      cb = bo;
      cc = co;
      uint32_t un[4], m[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        __builtin_amdgcn_sched_barrier(0);
        L.sub(v[k], ai, bi, ci, un[k], m[k]);
      }
      const uint32_t pm3 = prev(m[3], cm3), pm2 = prev(m[2], cm2);
      cm3 = m[3];
      cm2 = m[2];
      const uint32_t rb = k1f_runs(m[0], pm3, pm2) | k1f_runs(m[1], m[0], pm3) | k1f_runs(m[2], m[1], m[0]) |
                          k1f_runs(m[3], m[2], m[1]);
      const uint32_t u = k1f_or3(un[0], un[1], un[2]) | un[3];
      const uint64_t hb = __ballot((u & 0xFFFFu) != 0);
      if (__builtin_expect(hb != 0, 0)) nl += (uint32_t)__popcll(hb);
      const uint64_t bu = __ballot(rb & 1u), bd = __ballot(rb & 2u);
      if (__builtin_expect((bu | bd) != 0, 0)) nr += (uint32_t)__popcll(bu | bd);
    }
  };
  uint4 p[4];
#pragma unroll
  for (int k = 0; k < 4; k++) p[k] = ld16(base + (size_t)t0 * 4 * kTile + 16 * k);
  for (uint32_t t = t0; t < t1; t++) {
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      v[k] = p[k];
      p[k] = ld16(base + (size_t)(t + 1) * 4 * kTile + 16 * k);
    }
    body(v);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc + nl + nr;
}

template <typename F>
static float run(const char* name, F launch, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  launch();
  CHECK(hipDeviceSynchronize());
  std::vector<float> v;
  for (int r = 0; r < reps; r++) {
    CHECK(hipEventRecord(a));
    launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    v.push_back(ms);
  }
  std::sort(v.begin(), v.end());
  const float med = v[v.size() / 2];
  printf("{\"kernel\": \"%s\", \"ms_median\": %.4f, \"ms_min\": %.4f, \"TBps\": %.3f, \"frac\": %.3f}\n", name, med, v[0],
         kBytes / med / 1e9, kBytes / med / 1e9 / 8.0);
  fflush(stdout);
  return med;
}

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (uint32_t)(rng >> 11);
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 15;
  // text-like bytes: identifiers, numbers, punctuation, spaces, newlines
  std::vector<uint8_t> h(kBytes + (64 << 10));
  {
    static const char punct[] = " ,.;:()[]{}=\"'/+-_*<>#";
    size_t i = 0;
    while (i < kBytes) {
      const uint32_t r = rnd();
      const uint32_t kind = r % 100, len = 1 + (r >> 8) % 12;
      for (uint32_t k = 0; k < len && i < kBytes; k++) {
        const uint32_t s = rnd();
        h[i++] = kind < 60 ? (uint8_t)('a' + s % 26 - ((s >> 8) % 8 == 0 ? 32 : 0))
                 : kind < 70 ? (uint8_t)('0' + s % 10)
                 : kind < 97 ? (uint8_t)punct[s % (sizeof(punct) - 1)]
                             : (uint8_t)'\n';
      }
    }
  }
  uint32_t ent[256 * 4];
  for (int b = 0; b < 256; b++) {
    const bool U = isalnum(b) || b == '_' || b == '-' || b == '+' || b == '/' || b == '=';
    const bool D = b >= '0' && b <= '9';
    for (int j = 0; j < 4; j++) {
      uint32_t lo = 0;
      for (int k = 0; k < 16; k++) lo |= (rnd() % 100 < 5 ? 1u : 0u) << k;
      uint32_t hi = 0xFFu & ~(1u << j) & ~(1u << (4 + j));
      hi |= (U ? 1u : 0u) << j | (D ? 1u : 0u) << (4 + j);
      ent[b * 4 + j] = lo | hi << 16 | 0xFF000000u;
    }
  }
  uint8_t* buf;
  uint4* dent;
  uint32_t* out;
  unsigned long long* clk;
  CHECK(hipMalloc(&buf, h.size()));
  CHECK(hipMalloc(&dent, sizeof(ent)));
  CHECK(hipMalloc(&out, 64 << 20));
  CHECK(hipMalloc(&clk, 64));
  CHECK(hipMemcpy(buf, h.data(), h.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dent, ent, sizeof(ent), hipMemcpyHostToDevice));
  hipDeviceProp_t pr;
  CHECK(hipGetDeviceProperties(&pr, 0));
  const int cus = pr.multiProcessorCount;
  const uint32_t nt = kBytes / kTile;
#define R(name, V) run(name, [&] { lab_k<V><<<cus, 1024>>>(buf, dent, nt, out, clk); }, reps)
  R("V0_loads", 0);
  R("V1_entries", 1);
  R("V2_filter", 2);
  const float ms = R("V3_runs", 3);
  R("V4_all16", 4);
  R("V5_noDPP", 5);
  R("V6_noCopyQ", 6);
  R("V7_tablePerSimdHalf", 7);
  R("V8_stagger", 8);
  run("V3_512thr", [&] { lab_k<3><<<cus, 512>>>(buf, dent, nt, out, clk); }, reps);
  run("V3_2x512", [&] { lab_k<3><<<2 * cus, 512>>>(buf, dent, nt, out, clk); }, reps);
  run("V6_2x512", [&] { lab_k<6><<<2 * cus, 512>>>(buf, dent, nt, out, clk); }, reps);
  run("V6_4x256", [&] { lab_k<6><<<4 * cus, 256>>>(buf, dent, nt, out, clk); }, reps);
  run("V0_512thr", [&] { lab_k<0><<<cus, 512>>>(buf, dent, nt, out, clk); }, reps);
  // (L64: lane-contiguous 64 B streams at 3.8 TB/s -- profiles/r06/c/lab.json -- not pursued)
  unsigned long long c[2];
  CHECK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  printf("{\"block0_cycles\": %llu, \"block0_wall_ticks\": %llu, \"shader_MHz\": %.0f, \"kernel_ms\": %.4f}\n", c[0], c[1],
         c[1] ? c[0] / (c[1] / 100.0) : 0.0, ms);
  return 0;
}
