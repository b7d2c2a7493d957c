// FETCH_SIZE calibration for K1's access pattern (MI355X_MICROARCH.md: FETCH_SIZE is exact
// only for what it was calibrated on; "calibrate on a known byte count in your own access
// pattern").  Each kernel reads the same 2 GiB (far beyond the 256 MiB Infinity Cache)
// exactly once and stores one checksum word per thread:
//   stream16  one 16-B load per lane per instruction, consecutive lanes consecutive
//   quad64    K1's pattern: the 4 lanes of a quad load 64 contiguous bytes of one lane's
//             2-KiB segment per instruction; two 64-B blocks per chain in flight
//   quad128   the same, but each quad reads whole 128-B lines (two 64-B loads issued back
//             to back for the same stream)
// Run:  rocprofv3 --pmc FETCH_SIZE -- tools/fetch_calib   (one launch of each kernel)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                         \
  do {                                                                   \
    hipError_t e = (x);                                                  \
    if (e != hipSuccess) {                                               \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));            \
      exit(1);                                                           \
    }                                                                    \
  } while (0)

constexpr size_t kBytes = 2ull << 30;
constexpr int kSeg = 2048;  // one chain's segment (K1: 8 chunks of 256 B)

__global__ void stream16(const uint4* __restrict__ p, size_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// item = 2 segments (2 chains) per lane; a quad walks 4 consecutive items
template <int LINE>
__global__ void quad(const uint8_t* __restrict__ p, size_t nitems, uint32_t* out) {
  const uint32_t q = threadIdx.x & 3;
  const size_t ib = 2 * kSeg;
  uint32_t acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t it0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) & ~3ull; it0 < nitems; it0 += stride) {
    const uint8_t* src[4];
    for (int t = 0; t < 4; t++) src[t] = p + (it0 + t) * ib + 16u * q;
    for (int j = 0; j < kSeg; j += LINE) {
      uint4 r[2][LINE / 16];
#pragma unroll
      for (int i = 0; i < 2; i++)
#pragma unroll
        for (int h = 0; h < LINE / 64; h++)
#pragma unroll
          for (int t = 0; t < 4; t++) r[i][h * 4 + t] = *(const uint4*)(src[t] + i * kSeg + j + h * 64);
#pragma unroll
      for (int i = 0; i < 2; i++)
#pragma unroll
        for (int k = 0; k < LINE / 16; k++) acc ^= r[i][k].x ^ r[i][k].y ^ r[i][k].z ^ r[i][k].w;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  uint8_t* buf;
  uint32_t* out;
  CHECK(hipMalloc(&buf, kBytes));
  CHECK(hipMalloc(&out, 1 << 24));
  CHECK(hipMemset(buf, 0x5A, kBytes));
  const int grid = 2048, block = 256;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  float ms;
  CHECK(hipEventRecord(a));
  stream16<<<grid, block>>>((const uint4*)buf, kBytes / 16, out);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  CHECK(hipEventElapsedTime(&ms, a, b));
  printf("stream16 %zu bytes %.3f ms %.1f GB/s\n", kBytes, ms, kBytes / ms / 1e6);
  const size_t nitems = kBytes / (2 * kSeg);
  CHECK(hipEventRecord(a));
  quad<64><<<grid, block>>>(buf, nitems, out);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  CHECK(hipEventElapsedTime(&ms, a, b));
  printf("quad64 %zu bytes %.3f ms %.1f GB/s\n", kBytes, ms, kBytes / ms / 1e6);
  CHECK(hipEventRecord(a));
  quad<128><<<grid, block>>>(buf, nitems, out);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  CHECK(hipEventElapsedTime(&ms, a, b));
  printf("quad128 %zu bytes %.3f ms %.1f GB/s\n", kBytes, ms, kBytes / ms / 1e6);
  CHECK(hipDeviceSynchronize());
  return 0;
}
