// Streaming floor of K1F's load structure (round 6 measurement, not product code).
//
// K1F (kernels.hip) runs one 1,024-thread block per CU; each wave streams its own contiguous
// range of 1 KiB tiles (lane l: 16 B at tile + 16 l).  Its load-only build reached 0.229 ms
// per 0.976 GB with four tiles in flight (register queue) and 0.213 with eight.  This program
// times, on the same 0.976 GB, the load structures K1F could use, with a trivial consumer
// (XOR of the words, one store per thread):
//   grid      grid-stride 16-B loads, 2,048 x 256 threads (the plain streaming ceiling)
//   regD      K1F's structure: per-wave ranges, D tiles in flight in registers
//   ldsD      per-wave ranges, D tiles in flight through an LDS ring filled by
//             global_load_lds_dwordx4 (LDS-DMA; the consumer reads its 16 B back with
//             ds_read_b128), an extra LDS reservation standing in for K1F's tables
//   blkD      per-block ranges: step i of the block reads 16 contiguous tiles, wave w the
//             w-th (register queue)
// All kernels: nt loads (K1F's policy) unless the name ends in "_d".
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/stream_floor tools/stream_floor.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                \
  do {                                                          \
    hipError_t e = (x);                                         \
    if (e != hipSuccess) {                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));   \
      exit(1);                                                  \
    }                                                           \
  } while (0)

constexpr uint32_t kTile = 1024;
constexpr size_t kBytes = 976128930ull / kTile * kTile;  // one configs[1] batch
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
  if constexpr (NT) {
    const u32x4 v = __builtin_nontemporal_load((const u32x4*)p);
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *(const uint4*)p;
  }
}

__global__ void __launch_bounds__(256) grid_k(const uint8_t* p, uint32_t ntiles, uint32_t* out) {
  uint32_t acc = 0;
  const size_t n16 = (size_t)ntiles * (kTile / 16);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = ld16<true>(p + 16 * i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// K1F's structure with a register queue of D tiles
template <int D, bool NT, int LDSRES>
__global__ void __launch_bounds__(1024) reg_k(const uint8_t* p, uint32_t ntiles, uint32_t* out) {
  __shared__ uint32_t res[LDSRES / 4 + 1];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wpb = blockDim.x >> 6;
  const uint32_t gw = blockIdx.x * wpb + wave, nw = gridDim.x * wpb;
  const uint32_t t0 = (uint32_t)((uint64_t)gw * ntiles / nw), t1 = (uint32_t)((uint64_t)(gw + 1) * ntiles / nw);
  const uint8_t* base = p + 16u * lane;
  uint32_t acc = 0;
  uint4 q[D];
#pragma unroll
  for (int k = 0; k < D; k++) q[k] = ld16<NT>(base + (size_t)(t0 + k) * kTile);
  uint32_t t = t0;
  for (; t + D <= t1; t += D) {
#pragma unroll
    for (int k = 0; k < D; k++) {
      const uint4 v = q[k];
      q[k] = ld16<NT>(base + (size_t)(t + D + k) * kTile);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
      acc = __builtin_amdgcn_update_dpp(0, (int)acc, 0x13C, 0xF, 0xF, false) ^ acc;  // a little work
    }
  }
#pragma unroll
  for (int k = 0; k < D - 1; k++)
    if (t + k < t1) acc ^= q[k].x ^ q[k].y;
  if (LDSRES) res[threadIdx.x % (LDSRES / 4)] = acc;
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// the same through an LDS ring of D tiles per wave, filled by LDS-DMA
template <int D, bool NT>
__device__ __forceinline__ void glds(const uint8_t* g, uint32_t* lds) {
  // asm, so the compiler inserts no vmcnt(0) of its own for the DMA (it did at the loop head)
  uint32_t keep;
  const uint32_t dst = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  if constexpr (NT)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(__builtin_amdgcn_readfirstlane(dst)) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(__builtin_amdgcn_readfirstlane(dst)) : "memory");
}

template <int D, bool NT, int LDSRES>
__global__ void __launch_bounds__(1024) lds_k(const uint8_t* p, uint32_t ntiles, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint32_t ring[16 * D * kTile / 4];
  __shared__ uint32_t res[LDSRES / 4 + 1];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wpb = blockDim.x >> 6;
  const uint32_t gw = blockIdx.x * wpb + wave, nw = gridDim.x * wpb;
  const uint32_t t0 = (uint32_t)((uint64_t)gw * ntiles / nw), t1 = (uint32_t)((uint64_t)(gw + 1) * ntiles / nw);
  const uint8_t* base = p + 16u * lane;
  uint32_t* wr = ring + wave * D * (kTile / 4);
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < D; k++) glds<D, NT>(base + (size_t)(t0 + k) * kTile, wr + k * (kTile / 4));
  uint32_t t = t0;
  for (; t + D <= t1; t += D) {
#pragma unroll
    for (int k = 0; k < D; k++) {
      // tile t+k landed when at most D-1 younger DMAs are outstanding
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D - 1) : "memory");
      const uint4 v = *(const uint4*)(wr + k * (kTile / 4) + 4 * lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the read is done before the slot refills
      glds<D, NT>(base + (size_t)(t + D + k) * kTile, wr + k * (kTile / 4));
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
      acc = __builtin_amdgcn_update_dpp(0, (int)acc, 0x13C, 0xF, 0xF, false) ^ acc;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (LDSRES) res[threadIdx.x % (LDSRES / 4)] = acc;
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// per-block ranges: the block's 16 waves read 16 contiguous tiles per step
template <int D, bool NT>
__global__ void __launch_bounds__(1024) blk_k(const uint8_t* p, uint32_t ntiles, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wpb = blockDim.x >> 6;
  const uint32_t nsteps = ntiles / wpb;
  const uint32_t s0 = (uint32_t)((uint64_t)blockIdx.x * nsteps / gridDim.x),
                 s1 = (uint32_t)((uint64_t)(blockIdx.x + 1) * nsteps / gridDim.x);
  const uint8_t* base = p + (size_t)wave * kTile + 16u * lane;
  const size_t st = (size_t)wpb * kTile;
  uint32_t acc = 0;
  uint4 q[D];
#pragma unroll
  for (int k = 0; k < D; k++) q[k] = ld16<NT>(base + (s0 + k) * st);
  uint32_t s = s0;
  for (; s + D <= s1; s += D) {
#pragma unroll
    for (int k = 0; k < D; k++) {
      const uint4 v = q[k];
      q[k] = ld16<NT>(base + (s + D + k) * st);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
      acc = __builtin_amdgcn_update_dpp(0, (int)acc, 0x13C, 0xF, 0xF, false) ^ acc;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <typename F>
static void run(const char* name, F launch, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  launch();  // warm
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
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 15;
  uint8_t* buf;
  uint32_t* out;
  CHECK(hipMalloc(&buf, kBytes + (64 << 10)));
  CHECK(hipMalloc(&out, 64 << 20));
  CHECK(hipMemset(buf, 0x5A, kBytes + (64 << 10)));
  hipDeviceProp_t pr;
  CHECK(hipGetDeviceProperties(&pr, 0));
  const int cus = pr.multiProcessorCount;
  const uint32_t nt = kBytes / kTile;
#define R(name, K, G, B) run(name, [&] { K<<<G, B>>>(buf, nt, out); }, reps)
  R("grid", grid_k, 2048, 256);
  R("reg4", (reg_k<4, true, 0>), cus, 1024);
  R("reg4_d", (reg_k<4, false, 0>), cus, 1024);
  R("reg8", (reg_k<8, true, 0>), cus, 1024);
  R("reg12", (reg_k<12, true, 0>), cus, 1024);
  R("blk4", (blk_k<4, true>), cus, 1024);
  R("blk8", (blk_k<8, true>), cus, 1024);
  R("lds2", (lds_k<2, true, 64 * 1024>), cus, 1024);
  R("lds3", (lds_k<3, true, 64 * 1024>), cus, 1024);
  R("lds4", (lds_k<4, true, 64 * 1024>), cus, 1024);
  R("lds4_d", (lds_k<4, false, 64 * 1024>), cus, 1024);
  R("lds5", (lds_k<5, true, 64 * 1024>), cus, 1024);
  R("lds6", (lds_k<6, true, 0>), cus, 1024);
  R("lds8", (lds_k<8, true, 0>), cus, 1024);
  R("reg4_2cu", (reg_k<4, true, 0>), 2 * cus, 1024);
  return 0;
}
