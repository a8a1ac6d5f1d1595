// Micro-benchmark (diagnostic only): issue cost of the instructions the
// rollout tick is made of, for ONE wave per SIMD (the C3 headline shape) and
// for two.  Each kernel runs `iters` trips of a block of 16 independent
// instances of one instruction (inline asm, distinct registers) and records
// s_memtime around the loop; prints cycles per instruction per wave.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/bin/isa_rate tools/ubench/isa_rate.hip
//   tools/ubench/bin/isa_rate
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>


// v registers v[100..147] are reserved through clobbers; asm operates on them
#define K_BODY(NAME, ASMLINE)                                                                  \
  __global__ void __launch_bounds__(64) NAME(uint64_t* out, int iters) {                      \
    asm volatile("v_mov_b32 v100, %0\n v_mov_b32 v101, 3\n v_mov_b32 v102, 5\n"             \
                 "v_mov_b32 v103, 7\n s_mov_b64 s[40:41], -1\n s_mov_b32 s42, 0x1234\n"      \
                 :: "v"(threadIdx.x) : "v100", "v101", "v102", "v103", "s40", "s41", "s42"); \
    uint64_t t0, t1;                                                                           \
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0));                            \
    for (int it = 0; it < iters; ++it) {                                                       \
      asm volatile(ASMLINE ::: "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107",\
                   "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116",     \
                   "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125",     \
                   "v126", "v127", "v128", "v129", "v130", "v131", "v132", "v133", "v134",     \
                   "v135", "v136", "v137", "v138", "v139", "v140", "v141", "v142", "v143",     \
                   "v144", "v145", "v146", "v147", "s40", "s41", "s42", "s43", "s44", "s45",   \
                   "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55",       \
                   "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65",       \
                   "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73");                     \
    }                                                                                          \
    asm volatile("s_waitcnt vmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1));      \
    if ((threadIdx.x & 63) == 0) out[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;  \
  }

#define L16(F) F(104) F(105) F(106) F(107) F(108) F(109) F(110) F(111) F(112) F(113) F(114) F(115) F(116) F(117) F(118) F(119)
#define L16P(F) F(104,105) F(106,107) F(108,109) F(110,111) F(112,113) F(114,115) F(116,117) F(118,119) \
  F(120,121) F(122,123) F(124,125) F(126,127) F(128,129) F(130,131) F(132,133) F(134,135)
#define L16S(F) F(44,45) F(46,47) F(48,49) F(50,51) F(52,53) F(54,55) F(56,57) F(58,59) \
  F(60,61) F(62,63) F(64,65) F(66,67) F(68,69) F(70,71) F(72,73) F(44,45)

#define A_ADD(r) "v_add_u32 v" #r ", v100, v101\n"
#define A_BITOP3(r) "v_bitop3_b32 v" #r ", v100, v101, v102 bitop3:0x96\n"
#define A_MULHI(r) "v_mul_hi_u32 v" #r ", v100, v101\n"
#define A_MULLO(r) "v_mul_lo_u32 v" #r ", v100, v101\n"
#define A_MAD64(a, b) "v_mad_u64_u32 v[" #a ":" #b "], s[40:41], v100, s42, 0\n"
#define A_LSHL64(a, b) "v_lshlrev_b64 v[" #a ":" #b "], 3, v[100:101]\n"
#define A_CND(r) "v_cndmask_b32_e64 v" #r ", v100, v101, s[40:41]\n"
#define A_CMP(a, b) "v_cmp_eq_u32_e64 s[" #a ":" #b "], v100, v101\n"
#define A_SAND(a, b) "s_and_b64 s[" #a ":" #b "], s[40:41], exec\n"
#define A_PKMIN(r) "v_pk_min_u16 v" #r ", v100, v101\n"
#define A_FFBL(r) "v_ffbl_b32 v" #r ", v100\n"
#define A_BFE(r) "v_bfe_u32 v" #r ", v100, v101, 3\n"
// a dependent chain: each instruction reads the previous result
#define D_ADD(r) "v_add_u32 v100, v100, v101\n"
#define D_MAD64(a, b) "v_mad_u64_u32 v[100:101], s[40:41], v100, s42, 0\n"
#define D_CMPCND(a, b) "v_cmp_eq_u32_e64 s[40:41], v100, v101\n v_cndmask_b32_e64 v100, v102, v101, s[40:41]\n"

K_BODY(k_add, L16(A_ADD))
K_BODY(k_bitop3, L16(A_BITOP3))
K_BODY(k_mulhi, L16(A_MULHI))
K_BODY(k_mullo, L16(A_MULLO))
K_BODY(k_mad64, L16P(A_MAD64))
K_BODY(k_lshl64, L16P(A_LSHL64))
K_BODY(k_cnd, L16(A_CND))
K_BODY(k_cmp, L16S(A_CMP))
K_BODY(k_sand, L16S(A_SAND))
K_BODY(k_pkmin, L16(A_PKMIN))
K_BODY(k_ffbl, L16(A_FFBL))
K_BODY(k_bfe, L16(A_BFE))
K_BODY(k_dep_add, L16(D_ADD))
K_BODY(k_dep_mad64, L16P(D_MAD64))
K_BODY(k_dep_cmpcnd, L16P(D_CMPCND))
// mixed: 8 v_add + 8 s_and (do VALU and SALU of one wave overlap?)
#define MIX(a, b) "v_add_u32 v104, v100, v101\n s_and_b64 s[" #a ":" #b "], s[40:41], exec\n"
#define L8S(F) F(44,45) F(46,47) F(48,49) F(50,51) F(52,53) F(54,55) F(56,57) F(58,59)
K_BODY(k_mix, L8S(MIX))

// 16 buffer_store_dword per trip (nt), distinct rows of a 64 MiB scratch
// buffer whose resource is built in s[60:63]; the loop advances the row
#define A_ST(r) "buffer_store_dword v100, v" #r ", s[60:63], 0 offen nt\n"
__global__ void __launch_bounds__(64) k_store(uint64_t* out, int iters, uint32_t* buf) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t w = blockIdx.x;
  uint64_t t0, t1;
  asm volatile(
      "v_mov_b32 v100, %0\n"
      "v_lshlrev_b32 v104, 2, %0\n v_add_u32 v105, 256, v104\n v_add_u32 v106, 512, v104\n"
      "v_add_u32 v107, 768, v104\n v_add_u32 v108, 1024, v104\n v_add_u32 v109, 1280, v104\n"
      "v_add_u32 v110, 1536, v104\n v_add_u32 v111, 1792, v104\n v_add_u32 v112, 2048, v104\n"
      "v_add_u32 v113, 2304, v104\n v_add_u32 v114, 2560, v104\n v_add_u32 v115, 2816, v104\n"
      "v_add_u32 v116, 3072, v104\n v_add_u32 v117, 3328, v104\n v_add_u32 v118, 3584, v104\n"
      "v_add_u32 v119, 3840, v104\n"
      :: "v"(lane) : "v100", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111",
      "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119");
  // per wave: its own 16 KiB window, advanced by 4 KiB per trip, wrapping at 64 KiB
  uint64_t base = (uint64_t)buf + (uint64_t)w * 65536u;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0));
  for (int it = 0; it < iters; ++it) {
    const uint64_t b = base + (uint64_t)((it & 15) * 4096);
    asm volatile("s_mov_b32 s60, %0\n s_mov_b32 s61, %1\n s_mov_b32 s62, -1\n"
                 "s_mov_b32 s63, 0x00020000\n" L16(A_ST)
                 :: "s"((uint32_t)b), "s"((uint32_t)(b >> 32))
                 : "s60", "s61", "s62", "s63", "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1));
  if (lane == 0) out[w] = t1 - t0;
}

// the same stream as 8 dwordx2 / 4 dwordx4 stores per trip (same bytes)
#define A_ST2(r) "buffer_store_dwordx2 v[100:101], v" #r ", s[60:63], 0 offen nt\n"
#define A_ST4(r) "buffer_store_dwordx4 v[100:103], v" #r ", s[60:63], 0 offen nt\n"
#define L8(F) F(104) F(105) F(106) F(107) F(108) F(109) F(110) F(111)
#define L4(F) F(104) F(105) F(106) F(107)
template <int W>
__global__ void __launch_bounds__(64) k_storew(uint64_t* out, int iters, uint32_t* buf) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t w = blockIdx.x;
  uint64_t t0, t1;
  // row r of the trip at r * 64 * 4 * W bytes: lane offset lane * 4 * W
  asm volatile(
      "v_mov_b32 v100, %0\n v_mov_b32 v101, %0\n v_mov_b32 v102, %0\n v_mov_b32 v103, %0\n"
      "v_lshlrev_b32 v104, %1, %0\n v_add_u32 v105, %2, v104\n v_add_u32 v106, %2, v105\n"
      "v_add_u32 v107, %2, v106\n v_add_u32 v108, %2, v107\n v_add_u32 v109, %2, v108\n"
      "v_add_u32 v110, %2, v109\n v_add_u32 v111, %2, v110\n"
      :: "v"(lane), "s"(W == 2 ? 3 : 4), "s"(256 * W)
      : "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110",
        "v111");
  uint64_t base = (uint64_t)buf + (uint64_t)w * 65536u;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0));
  for (int it = 0; it < iters; ++it) {
    const uint64_t b = base + (uint64_t)((it & 15) * 4096);
    if constexpr (W == 2)
      asm volatile("s_mov_b32 s60, %0\n s_mov_b32 s61, %1\n s_mov_b32 s62, -1\n"
                   "s_mov_b32 s63, 0x00020000\n" L8(A_ST2)
                   :: "s"((uint32_t)b), "s"((uint32_t)(b >> 32)) : "s60", "s61", "s62", "s63", "memory");
    else
      asm volatile("s_mov_b32 s60, %0\n s_mov_b32 s61, %1\n s_mov_b32 s62, -1\n"
                   "s_mov_b32 s63, 0x00020000\n" L4(A_ST4)
                   :: "s"((uint32_t)b), "s"((uint32_t)(b >> 32)) : "s60", "s61", "s62", "s63", "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1));
  if (lane == 0) out[w] = t1 - t0;
}

// HBM streaming stores: each wave writes its own contiguous region (rows
// advance, never wrap: `iters` x 4 KiB per wave), W dwords per lane per store
template <int W>
__global__ void __launch_bounds__(64) k_stream(uint64_t* out, int iters, uint32_t* buf) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t w = blockIdx.x;
  uint64_t t0, t1;
  asm volatile(
      "v_mov_b32 v100, %0\n v_mov_b32 v101, %0\n v_mov_b32 v102, %0\n v_mov_b32 v103, %0\n"
      "v_lshlrev_b32 v104, %1, %0\n v_add_u32 v105, %2, v104\n v_add_u32 v106, %2, v105\n"
      "v_add_u32 v107, %2, v106\n v_add_u32 v108, %2, v107\n v_add_u32 v109, %2, v108\n"
      "v_add_u32 v110, %2, v109\n v_add_u32 v111, %2, v110\n v_add_u32 v112, %2, v111\n"
      "v_add_u32 v113, %2, v112\n v_add_u32 v114, %2, v113\n v_add_u32 v115, %2, v114\n"
      "v_add_u32 v116, %2, v115\n v_add_u32 v117, %2, v116\n v_add_u32 v118, %2, v117\n"
      "v_add_u32 v119, %2, v118\n"
      :: "v"(lane), "s"(W == 1 ? 2 : W == 2 ? 3 : 4), "s"(256 * W)
      : "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110",
        "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119");
  const uint64_t base = (uint64_t)buf + (uint64_t)w * (uint64_t)iters * 4096u;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0));
  for (int it = 0; it < iters; ++it) {
    const uint64_t b = base + (uint64_t)it * 4096u;
    if constexpr (W == 1)
      asm volatile("s_mov_b32 s60, %0\n s_mov_b32 s61, %1\n s_mov_b32 s62, -1\n"
                   "s_mov_b32 s63, 0x00020000\n" L16(A_ST)
                   :: "s"((uint32_t)b), "s"((uint32_t)(b >> 32)) : "s60", "s61", "s62", "s63", "memory");
    else if constexpr (W == 2)
      asm volatile("s_mov_b32 s60, %0\n s_mov_b32 s61, %1\n s_mov_b32 s62, -1\n"
                   "s_mov_b32 s63, 0x00020000\n" L8(A_ST2)
                   :: "s"((uint32_t)b), "s"((uint32_t)(b >> 32)) : "s60", "s61", "s62", "s63", "memory");
    else
      asm volatile("s_mov_b32 s60, %0\n s_mov_b32 s61, %1\n s_mov_b32 s62, -1\n"
                   "s_mov_b32 s63, 0x00020000\n" L4(A_ST4)
                   :: "s"((uint32_t)b), "s"((uint32_t)(b >> 32)) : "s60", "s61", "s62", "s63", "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1));
  if (lane == 0) out[w] = t1 - t0;
}

// a per-lane branch around an empty block (never taken: the mask is empty),
// as the rollout's rare-block test: v_cmp, s_and_saveexec, s_cbranch_execz,
// s_or exec -- 16 per trip, each with its own v_cmp
#define A_BR(r) "v_cmp_eq_u32 vcc, v100, v101\n s_and_saveexec_b64 s[44:45], vcc\n" \
  "s_cbranch_execz 1f\n v_add_u32 v" #r ", v100, v101\n 1:\n s_or_b64 exec, exec, s[44:45]\n"
K_BODY(k_branch, L16(A_BR))
// the same number of v_cmp + SALU without the branch
#define A_NOBR(r) "v_cmp_eq_u32 vcc, v100, v101\n s_and_saveexec_b64 s[44:45], vcc\n" \
  "s_or_b64 exec, exec, s[44:45]\n"
K_BODY(k_nobranch, L16(A_NOBR))

typedef void (*kfn)(uint64_t*, int);

int main() {
  struct K { const char* name; kfn f; int per_iter; };
  std::vector<K> ks = {
      {"v_add_u32", k_add, 16},        {"v_bitop3_b32", k_bitop3, 16},
      {"v_mul_hi_u32", k_mulhi, 16},   {"v_mul_lo_u32", k_mullo, 16},
      {"v_mad_u64_u32", k_mad64, 16},  {"v_lshlrev_b64", k_lshl64, 16},
      {"v_cndmask(sgpr)", k_cnd, 16},  {"v_cmp_e64->sgpr", k_cmp, 16},
      {"s_and_b64", k_sand, 16},       {"v_pk_min_u16", k_pkmin, 16},
      {"v_ffbl_b32", k_ffbl, 16},      {"v_bfe_u32", k_bfe, 16},
      {"dep v_add chain", k_dep_add, 16}, {"dep v_mad_u64 chain", k_dep_mad64, 16},
      {"dep v_cmp->v_cndmask pair", k_dep_cmpcnd, 16}, {"v_add+s_and pair", k_mix, 8},
      {"v_cmp+saveexec+cbranch(not taken)+or", k_branch, 16},
      {"v_cmp+saveexec+or (no branch)", k_nobranch, 16},
  };
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  uint64_t* d;
  const int maxw = 4 * cus * 4;
  hipMalloc(&d, maxw * sizeof(uint64_t));
  const int iters = 4096;
  for (int wps : {1, 2}) {
    const int waves = 4 * cus * wps;
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.f, dim3(waves), dim3(64), 0, 0, d, 16);
      hipDeviceSynchronize();
      hipLaunchKernelGGL(k.f, dim3(waves), dim3(64), 0, 0, d, iters);
      hipDeviceSynchronize();
      std::vector<uint64_t> h(waves);
      hipMemcpy(h.data(), d, waves * sizeof(uint64_t), hipMemcpyDeviceToHost);
      double s = 0;
      for (auto v : h) s += (double)v;
      s /= waves;
      printf("{\"waves_per_simd\": %d, \"instr\": \"%s\", \"cycles_per_instr\": %.2f}\n", wps,
             k.name, s / ((double)iters * k.per_iter));
    }
  }
  uint32_t* buf;
  hipMalloc(&buf, (size_t)maxw * 65536u);
  for (int wps : {1, 2}) {
    const int waves = 4 * cus * wps;
    hipLaunchKernelGGL(k_store, dim3(waves), dim3(64), 0, 0, d, 16, buf);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(k_store, dim3(waves), dim3(64), 0, 0, d, iters, buf);
    hipDeviceSynchronize();
    std::vector<uint64_t> h(waves);
    hipMemcpy(h.data(), d, waves * sizeof(uint64_t), hipMemcpyDeviceToHost);
    double s = 0;
    for (auto v : h) s += (double)v;
    s /= waves;
    printf("{\"waves_per_simd\": %d, \"instr\": \"buffer_store_dword nt (L2-resident rows)\", "
           "\"cycles_per_instr\": %.2f}\n", wps, s / ((double)iters * 16));
  }
  for (int W : {2, 4})
    for (int wps : {1, 2}) {
      const int waves = 4 * cus * wps;
      auto f = W == 2 ? k_storew<2> : k_storew<4>;
      hipLaunchKernelGGL(f, dim3(waves), dim3(64), 0, 0, d, 16, buf);
      hipDeviceSynchronize();
      hipLaunchKernelGGL(f, dim3(waves), dim3(64), 0, 0, d, iters, buf);
      hipDeviceSynchronize();
      std::vector<uint64_t> h(waves);
      hipMemcpy(h.data(), d, waves * sizeof(uint64_t), hipMemcpyDeviceToHost);
      double s = 0;
      for (auto v : h) s += (double)v;
      s /= waves;
      printf("{\"waves_per_simd\": %d, \"instr\": \"buffer_store_dwordx%d nt (L2-resident)\", "
             "\"cycles_per_instr\": %.2f, \"cycles_per_256B\": %.2f}\n", wps, W,
             s / ((double)iters * (16 / W)), s / ((double)iters * 16));
    }
  // HBM stream: 1024 (2048) waves x iters2 x 4 KiB (>= 2 GiB, past the 256 MiB MALL)
  const int iters2 = 512;
  uint32_t* big;
  hipMalloc(&big, (size_t)maxw * iters2 * 4096u);
  for (int W : {1, 2, 4})
    for (int wps : {1, 2, 3}) {
      const int waves = 4 * cus * wps;
      auto f = W == 1 ? k_stream<1> : W == 2 ? k_stream<2> : k_stream<4>;
      hipLaunchKernelGGL(f, dim3(waves), dim3(64), 0, 0, d, iters2, big);
      hipDeviceSynchronize();
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(f, dim3(waves), dim3(64), 0, 0, d, iters2, big);
      hipEventRecord(e1, 0);
      hipDeviceSynchronize();
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      std::vector<uint64_t> h(waves);
      hipMemcpy(h.data(), d, waves * sizeof(uint64_t), hipMemcpyDeviceToHost);
      double s = 0;
      for (auto v : h) s += (double)v;
      s /= waves;
      const double bytes = (double)waves * iters2 * 4096.0;
      printf("{\"waves_per_simd\": %d, \"instr\": \"HBM stream dwordx%d nt\", "
             "\"cycles_per_256B_per_wave\": %.2f, \"TBps\": %.3f}\n", wps, W,
             s / ((double)iters2 * 16), bytes / (ms * 1e-3) / 1e12);
    }
  hipFree(big);
  hipFree(buf);
  hipFree(d);
  return 0;
}
