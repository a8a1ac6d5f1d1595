// Micro-benchmark: Philox4x32-10 cost on gfx950 (diagnostic only).
// Variants: MAD (64-bit product -> v_mad_u64_u32) vs HILO (__umulhi + mul),
// chains = independent Philox streams interleaved per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

template <bool MAD>
__device__ __forceinline__ void round1(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                                       uint32_t k0, uint32_t k1) {
  uint32_t hi0, lo0, hi1, lo1;
  if (MAD) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    hi0 = p0 >> 32; lo0 = (uint32_t)p0; hi1 = p1 >> 32; lo1 = (uint32_t)p1;
  } else {
    hi0 = __umulhi(0xD2511F53u, c0); lo0 = 0xD2511F53u * c0;
    hi1 = __umulhi(0xCD9E8D57u, c2); lo1 = 0xCD9E8D57u * c2;
  }
  const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
  c1 = lo1; c3 = lo0; c0 = n0; c2 = n2;
}

template <bool MAD, int CH>
__global__ void kern(uint32_t* out, int iters, uint32_t k0, uint32_t k1) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t c[CH][4];
#pragma unroll
  for (int h = 0; h < CH; ++h) { c[h][0] = i; c[h][1] = h; c[h][2] = 7; c[h][3] = 9; }
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
    uint32_t a = k0, b = k1;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
#pragma unroll
      for (int h = 0; h < CH; ++h) round1<MAD>(c[h][0], c[h][1], c[h][2], c[h][3], a, b);
      a += 0x9E3779B9u; b += 0xBB67AE85u;
    }
#pragma unroll
    for (int h = 0; h < CH; ++h) { acc ^= c[h][0] ^ c[h][3]; c[h][1] += it; }
  }
  out[i] = acc;
}

template <bool MAD, int CH>
void run(int B, int iters) {
  uint32_t* d;
  hipMalloc(&d, (size_t)B * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((kern<MAD, CH>), dim3(B / 256), dim3(256), 0, 0, d, iters, 1u, 2u);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  hipLaunchKernelGGL((kern<MAD, CH>), dim3(B / 256), dim3(256), 0, 0, d, iters, 1u, 2u);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double blocks = (double)B * iters * CH;
  const double waves_per_simd = (double)B / 64 / 1024;
  printf("%s CH=%d B=%8d waves/SIMD=%5.1f: %8.3f ms  %.3f Gblocks/s  cycles/block/wave(@2.4GHz, per SIMD)=%.1f\n",
         MAD ? "MAD " : "HILO", CH, B, waves_per_simd, ms, blocks / ms / 1e6,
         ms * 1e-3 * 2.4e9 / (iters * CH * waves_per_simd));
  hipFree(d);
}

int main() {
  for (int B : {65536, 262144, 1048576}) {
    run<true, 1>(B, 200); run<true, 2>(B, 100); run<true, 4>(B, 50);
    run<false, 1>(B, 200); run<false, 2>(B, 100); run<false, 4>(B, 50);
  }
  return 0;
}
