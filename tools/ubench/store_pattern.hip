// Micro-benchmark (diagnostic only): the trajectory output pattern of the
// paired rollout written by store instructions of different widths, with no
// tick computed -- what the bench step's store stream can reach per form.
//
// Output as orx_rollout writes it: obs int32 [T][14][B], act int8 [T][B][2].
// 32 games per wave, lane = 2 * game + player (the paired form), 256-thread
// workgroups, every wave runs T ticks of its 32 games.
//   dword   : each lane stores its player's 7 fields (7 buffer_store_dword,
//             two 128-B row segments per instruction) + 1 buffer_store_byte
//             -- the committed kernel's pattern
//   x4lds   : each lane writes its 7 fields into a per-wave LDS tile
//             [14][32] (+ the action bytes), reads it back as 16-B pieces and
//             stores 2 buffer_store_dwordx4 (rows 0-7, rows 8-13 + act)
//   x2lds   : the same tile stored as 4 buffer_store_dwordx2
//   flat4   : the same byte count as one contiguous dwordx4 stream (ceiling)
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/bin/store_pattern tools/ubench/store_pattern.hip
//   tools/ubench/bin/store_pattern [games] [ticks] [streams]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

constexpr int kFields = 14;
constexpr int kAuxNt = 2;  // nontemporal, as the kernel's whole-line stores

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, (int32_t)bytes, 0x00020000);
}

// tick values: cheap, lane-dependent, not foldable
__device__ __forceinline__ int32_t val(int t, uint32_t lane, int k) {
  return (int32_t)((uint32_t)t * 2654435761u ^ (lane << 4) ^ (uint32_t)k);
}

__global__ void __launch_bounds__(256) k_dword(int32_t* obs, int8_t* act, uint32_t B, int T) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t i = ((blockIdx.x * 256u + threadIdx.x) >> 6) * 32u + (lane >> 1);
  if (i >= B) return;
  const uint32_t who = lane & 1u;
  uint32_t vo[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const uint32_t row = k < 4 ? (uint32_t)k + 4u * who : k == 4 ? 8u + who : k == 5 ? 10u + 2u * who : 11u + 2u * who;
    vo[k] = (row * B + i) * 4u;
    asm volatile("" : "+v"(vo[k]));
  }
  const uint32_t va = 2u * i + who;
  for (int t = 0; t < T; ++t) {
    const auto ro = rsrc(obs + (size_t)t * kFields * B, kFields * B * 4u);
    const auto ra = rsrc(act + (size_t)t * 2u * B, 2u * B);
#pragma unroll
    for (int k = 0; k < 7; ++k)
      __builtin_amdgcn_raw_buffer_store_b32(val(t, lane, k), ro, (int32_t)vo[k], 0, kAuxNt);
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)val(t, lane, 9), ra, (int32_t)va, 0, kAuxNt);
  }
}

// LDS tile per wave: 14 rows x 32 dwords (1,792 B) + 64 action bytes = 1,856 B
template <int W>
__global__ void __launch_bounds__(256) k_lds(int32_t* obs, int8_t* act, uint32_t B, int T) {
  __shared__ uint32_t tile[4][464];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t g0 = ((blockIdx.x * 256u + threadIdx.x) >> 6) * 32u;
  if (g0 >= B) return;
  const uint32_t who = lane & 1u, g = lane >> 1;
  uint32_t* tl = tile[wv];
  // write side: field k of this lane's player goes to row rows[k], column g
  uint32_t wo[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const uint32_t row = k < 4 ? (uint32_t)k + 4u * who : k == 4 ? 8u + who : k == 5 ? 10u + 2u * who : 11u + 2u * who;
    wo[k] = row * 32u + g;
  }
  for (int t = 0; t < T; ++t) {
    const auto ro = rsrc(obs + (size_t)t * kFields * B, kFields * B * 4u);
    const auto ra = rsrc(act + (size_t)t * 2u * B, 2u * B);
#pragma unroll
    for (int k = 0; k < 7; ++k) tl[wo[k]] = (uint32_t)val(t, lane, k);
    reinterpret_cast<uint8_t*>(tl + 448)[lane] = (uint8_t)val(t, lane, 9);
    __builtin_amdgcn_wave_barrier();
    if constexpr (W == 4) {
      // piece p = 16 B: rows 0-7 by lanes 0-63 (8 pieces per row), rows 8-13
      // by lanes 0-47, act (64 B) by lanes 48-51
      {
        const uint32_t row = lane >> 3, col = (lane & 7u) * 4u;
        const uint4 v = *reinterpret_cast<const uint4*>(tl + row * 32u + col);
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v), ro,
            (int32_t)((row * B + g0 + col) * 4u), 0, kAuxNt);
      }
      if (lane < 52u) {
        const uint32_t row = 8u + (lane >> 3), col = (lane & 7u) * 4u;
        const uint4 v = *reinterpret_cast<const uint4*>(tl + (lane < 48u ? row * 32u + col : 448u + (lane - 48u) * 4u));
        const auto vv = __builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v);
        if (lane < 48u)
          __builtin_amdgcn_raw_buffer_store_b128(vv, ro, (int32_t)((row * B + g0 + col) * 4u), 0, kAuxNt);
        else
          __builtin_amdgcn_raw_buffer_store_b128(vv, ra, (int32_t)(2u * g0 + (lane - 48u) * 16u), 0, kAuxNt);
      }
    } else {
      // 8-B pieces: 16 per row; instructions cover rows 4j..4j+3 (j = 0..3)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t row = 4u * j + (lane >> 4), col = (lane & 15u) * 2u;
        if (j < 3 || lane < 40u) {
          const bool is_act = j == 3 && lane >= 32u;
          const uint2 v = *reinterpret_cast<const uint2*>(tl + (is_act ? 448u + (lane - 32u) * 2u : row * 32u + col));
          const auto vv = __builtin_bit_cast(__attribute__((ext_vector_type(2))) uint32_t, v);
          if (!is_act)
            __builtin_amdgcn_raw_buffer_store_b64(vv, ro, (int32_t)((row * B + g0 + col) * 4u), 0, kAuxNt);
          else
            __builtin_amdgcn_raw_buffer_store_b64(vv, ra, (int32_t)(2u * g0 + (lane - 32u) * 8u), 0, kAuxNt);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// the same bytes per tick as one contiguous region per wave (1,856 B)
__global__ void __launch_bounds__(256) k_flat4(int32_t* obs, int8_t* act, uint32_t B, int T) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t w = (blockIdx.x * 256u + threadIdx.x) >> 6;
  const uint32_t g0 = w * 32u;
  if (g0 >= B) return;
  for (int t = 0; t < T; ++t) {
    const auto ro = rsrc(obs + (size_t)t * kFields * B, kFields * B * 4u);
    const auto ra = rsrc(act + (size_t)t * 2u * B, 2u * B);
    const uint32_t v = (uint32_t)val(t, lane, 0);
    __attribute__((ext_vector_type(4))) uint32_t vv = {v, v + 1u, v + 2u, v + 3u};
    // obs: 14 * 32 * 4 = 1,792 B of this wave's contiguous slice
    __builtin_amdgcn_raw_buffer_store_b128(vv, ro, (int32_t)(g0 * 56u + lane * 16u), 0, kAuxNt);
    if (lane < 48u)
      __builtin_amdgcn_raw_buffer_store_b128(vv, ro, (int32_t)(g0 * 56u + 1024u + lane * 16u), 0, kAuxNt);
    else if (lane < 52u)
      __builtin_amdgcn_raw_buffer_store_b128(vv, ra, (int32_t)(2u * g0 + (lane - 48u) * 16u), 0, kAuxNt);
  }
}

typedef void (*KFn)(int32_t*, int8_t*, uint32_t, int);

int main(int argc, char** argv) {
  const uint32_t games = argc > 1 ? (uint32_t)atoi(argv[1]) : 65536u;
  const int T = argc > 2 ? atoi(argv[2]) : 128;
  const int S = argc > 3 ? atoi(argv[3]) : 2;  // concurrent streams (the bench's shards)
  const uint32_t B = games / S;
  struct { const char* name; KFn fn; } forms[] = {
      {"dword", k_dword}, {"x4lds", k_lds<4>}, {"x2lds", k_lds<2>}, {"flat4", k_flat4}};
  int32_t* obs[4];
  int8_t* act[4];
  hipStream_t st[4];
  for (int s = 0; s < S; ++s) {
    CHECK(hipMalloc(&obs[s], (size_t)T * kFields * B * 4));
    CHECK(hipMalloc(&act[s], (size_t)T * 2 * B));
    CHECK(hipStreamCreateWithFlags(&st[s], hipStreamNonBlocking));
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const uint32_t blocks = (B / 32u * 64u + 255u) / 256u;
  const double bytes = (double)games * T * 58.0;
  for (int rep = 0; rep < 3; ++rep) {
    for (auto& f : forms) {
      const int iters = 20;
      for (int w = 0; w < 3; ++w)
        for (int s = 0; s < S; ++s) f.fn<<<blocks, 256, 0, st[s]>>>(obs[s], act[s], B, T);
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0, 0));
      for (int it = 0; it < iters; ++it) {
        for (int s = 0; s < S; ++s) f.fn<<<blocks, 256, 0, st[s]>>>(obs[s], act[s], B, T);
        CHECK(hipDeviceSynchronize());
      }
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / iters;
      printf("{\"form\": \"%s\", \"games\": %u, \"ticks\": %d, \"streams\": %d, \"us_per_step\": %.2f, "
             "\"TBps\": %.3f}\n", f.name, games, T, S, us, bytes / (us * 1e-6) / 1e12);
    }
  }
  // check: the dword and LDS forms write the same bytes
  return 0;
}
