// orx_engine.hip -- MI355X (gfx950) batched tick engine for Optimax Rogue.
//
// One lane = one game.  All per-game state is struct-of-arrays with the batch
// axis contiguous, so every field load/store of a wavefront is one coalesced
// 256-byte access.  The tick is integer/branch work; there is nothing for the
// matrix cores.  See DESIGN.md for the byte accounting and the roofline.
//
// Reference semantics restated here (paths relative to the reference repo):
//   Updater.update            optimax_rogue/logic/updater.py:76-162
//   Updater.handle_move       optimax_rogue/logic/updater.py:180-243
//   Updater.handle_descend    optimax_rogue/logic/updater.py:259-296
//   Updater.handle_combat     optimax_rogue/logic/updater.py:298-338
//   Updater.should_despawn    optimax_rogue/logic/updater.py:245-257
//   calculate_pos             optimax_rogue/logic/updater.py:340-351
//   Dungeon.is_blocked        optimax_rogue/game/world.py:41-46
//   Dungeon.get_random_unblocked optimax_rogue/game/world.py:57-66
//   EmptyDungeonGenerator.spawn_dungeon optimax_rogue/logic/worldgen.py:33-43
//   Together/SeparatedGameStartGenerator.setup_game worldgen.py:77-87,124-135
//   RandomBot.move            optimax_rogue_bots/randombot.py:20-21
//   StaircaseBot.move         optimax_rogue_bots/staircasebot.py:9-21
//
// Closed forms used instead of the reference's W x H tile arrays (each is
// checked against the oracle's literal tile scan in tests/):
//   * walls: the EmptyDungeonGenerator border, so is_blocked(x, y) is
//     x <= 0 || x >= W-1 || y <= 0 || y >= H-1;
//   * a dungeon is its staircase (sx, sy), regenerated from the Philox key
//     (episode, depth, generation) whenever a player enters it, so no
//     per-depth storage exists however deep the players go;
//   * get_random_unblocked: the c-th Ground tile in x-major order is interior
//     index c (+1 past the staircase) -> x = 1 + ci / (H-2), y = 1 + ci % (H-2);
//   * World.dungeons membership is derived from the players' start and
//     current depths (DESIGN.md "Dungeon presence").
//
// Performance structure (gfx950, one wave per SIMD at the 65,536-game config):
//   * the common tick is straight-line: the per-tick random words (policy and
//     initiative streams, two Philox blocks each) are generated unconditionally
//     and interleaved, accepted words are picked with selects; only lanes that
//     exhaust 8 words take the generic stream loop (rare);
//   * Philox rounds use v_mad_u64_u32 (64-bit product) and SGPR key schedule;
//   * NPC occupancy is a packed 16-bit compare against registers (NCAP slots,
//     a template parameter: 0, 8 or 16), dead slots hold 0xFFFF (no target);
//   * rare events (descend, NPC hits, game start) sit behind branches, each
//     with a single Philox call site.
#include <hip/hip_runtime.h>

#include <atomic>
#include <type_traits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../include/orx.h"

// Split build (optimax_rogue_amd/build.py): this file is compiled ORX_NPARTS
// times in parallel.  Part 0 holds the host side (the C-ABI) and declares
// every kernel instance `extern template`; part k >= 1 explicitly
// instantiates its share of the instances (the lists before the host side).
// Without ORX_NPARTS it is one translation unit (the stamps builds).
#ifdef ORX_NPARTS
#define ORX_HOST_TU (ORX_PART == 0)
#else
#define ORX_HOST_TU 1
#endif

namespace orx_dev {

// ---------------------------------------------------------------------------
// Philox4x32-10 and the reference's bounded-integer transforms
// ---------------------------------------------------------------------------
enum : uint32_t {
  PUR_INIT = 1, PUR_DUNGEON = 2, PUR_SHUFFLE = 3, PUR_SPAWN = 4, PUR_POLICY = 5,
  PUR_RESOLVE = 6,  // ORX_EXT_RANDOM_DOUBLE_DEATH
  PUR_TICK = 7,     // the tick's CPython-random bit reservoir (bots, shuffles)
  PUR_ITEM = 8,     // ORX_EXT_ITEMS: an NPC's drop (c2 = tick, block = NPC slot)
  PUR_NPC = 9       // the enemy AI's random.choice draws (cfg.npc_policy RANDOM; c2 = tick)
};
#define ORX_LIKELY(x) __builtin_expect(!!(x), 1)
#define ORX_UNLIKELY(x) __builtin_expect(!!(x), 0)

constexpr uint32_t kWordCap = 4096;  // per stream; exceeding it stops the game
constexpr int32_t kStartTick = 1;     // GameState.tick of a fresh game (worldgen.py:87,133)
constexpr uint32_t kDeadSlot = 0xFFFFu;

// Diagnostic builds only (-DORX_DIAG=bits; results are wrong): rollout_kernel
// 64: the paired RandomBot form's tick block from a cheap hash (no Philox);
// 16 writes no trajectory; 32 runs no tick (the trajectory stores alone: the
// store ceiling of the launch's own output pattern).  Used by
// tools/ab_rollout.py and tools/ab_bench_step.py to attribute time.
#ifndef ORX_DIAG
#define ORX_DIAG 0
#endif
// -DORX_STAMPS (diagnostic builds): rollout_kernel lane 0 of each wave
// records s_memtime at 8 points into g_stamps; orx_diag_stamps copies them out.
#ifdef ORX_STAMPS
__device__ uint64_t g_stamps[65536 * 16];
#define ORX_STAMP(j)                                                               \
  if ((threadIdx.x & 63) == 0)                                                     \
    g_stamps[(size_t)((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 16 + (j)] =   \
        __builtin_amdgcn_s_memtime()
// per-wave counts of rare-block entries (stamp slots 5..7): the block's first
// active lane counts the entry; the lanes' counts are summed at the end
#define ORX_COUNT(var)                                                                   \
  var += (__lane_id() == (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec())) ? 1u : 0u
// shader-clock cycles a wave spends in a rare-block branch (stamp slots 11..14),
// accumulated by the branch's first active lane
#define ORX_CYC_BEGIN(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define ORX_CYC_END(var, v)                                                            \
  var += (__lane_id() == (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec()))     \
             ? (uint32_t)(__builtin_amdgcn_s_memtime() - (v)) : 0u
// the moving-NPC rollout's sections: the first active lane of a wave adds
// the section's shader-clock cycles to the wave's slot j (a vector atomic;
// orx_diag_stamps_clear zeroes the slots first)
#define ORX_MCYC_BEGIN(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define ORX_MCYC_END(j, v)                                                                \
  if (__lane_id() == (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec()))             \
  atomicAdd((unsigned long long*)&g_stamps[(size_t)((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * \
                                               16 + (j)],                                  \
            (unsigned long long)(__builtin_amdgcn_s_memtime() - (v)))
#else
#define ORX_STAMP(j) ((void)0)
#define ORX_COUNT(var) ((void)0)
#define ORX_CYC_BEGIN(v) ((void)0)
#define ORX_CYC_END(var, v) ((void)0)
#define ORX_MCYC_BEGIN(v) ((void)0)
#define ORX_MCYC_END(j, v) ((void)0)
#endif
#ifndef ORX_ROLLOUT_BLOCK
#define ORX_ROLLOUT_BLOCK 256
#endif
constexpr int kRolloutBlock = ORX_ROLLOUT_BLOCK;  // rollout_kernel workgroup size
// Games per rollout wave ("lanes", a power of two 1..64) is a launch
// argument: below 64 the wave's upper lanes idle so that a small batch still
// puts a wave on every SIMD (orx_rollout picks it from the batch and the CU
// count, rollout_lanes()).

#ifndef ORX_XCD_REMAP
#define ORX_XCD_REMAP 1
#endif
#ifndef ORX_SPLIT_TICK
// pair_rollout_kernel's RandomBot tick blocks (PM 1), one Philox pass per two
// ticks: lane 2j draws tick t's block and lane 2j+1 tick t+1's, the pair
// swaps them, and the next trip uses the held block (a reset redraws).  1:
// the compact-row form only; 2: every PM 1 form; 0 (the product): none --
// measured in round 5 (profiles/r05_v5/ab_forms.jsonl, three rounds on one
// box): compact rows 73.2-74.3 us with it against 73.1-75.1 without, the
// int32 headline step 88.1-89.1 against 85.0-86.5 and C2 49.7-50.0 against
// 47.9-48.5 (as in round 3, profiles/r03_v11).
#define ORX_SPLIT_TICK 0
#endif
#ifndef ORX_LEAN
// pair_rollout_kernel's lean StaircaseBot spans: off (measured slower, DESIGN
// s7.2: the launch is set by its slowest waves, which run few lean ticks and
// pay the span computation on every general tick); -DORX_LEAN=1 builds them
#define ORX_LEAN 0
#endif
// The rollout kernels' workgroup order, XCD-aware: the dispatcher deals
// workgroups round-robin over the chip's 8 XCDs (workgroup b to XCD b % 8),
// so XCD x takes the x-th contiguous run of the grid.  Neighbouring
// workgroups' games -- which share a 128-B trajectory row segment when a
// workgroup holds fewer than 32 games -- then write it through one XCD's L2,
// where the line is merged, instead of two L2s each writing back a partial
// line.
__device__ __forceinline__ uint32_t xcd_block() {
  const uint32_t b = blockIdx.x;
  if (!ORX_XCD_REMAP) return b;
  const uint32_t g = gridDim.x, q = g >> 3, r = g & 7u, x = b & 7u;
  return x * q + (x < r ? x : r) + (b >> 3);
}

struct Key {
  uint32_t k0, k1;
};

struct W4 {
  uint32_t a, b, c, d;
};

__device__ __forceinline__ W4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, Key key) {
  uint32_t k0 = key.k0, k1 = key.k1;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    // three-input xor in one v_bitop3_b32 (the compiler emits two v_xor here)
    const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);
    const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return W4{c0, c1, c2, c3};
}

// Words a and b of a Philox block with the last round's other half deferred:
// words c and d follow from the round-10 inputs (h0, h3) by finish_cd, for the
// rare cases that read them (the paired rollout's common tick needs a and b).
__device__ __forceinline__ W4 philox_ab(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                        Key key, uint32_t& h0, uint32_t& h3) {
  uint32_t k0 = key.k0, k1 = key.k1;
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);
    const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
  h0 = c0;
  h3 = c3;
  return W4{(uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96), (uint32_t)p1, 0u, 0u};
}
__device__ __forceinline__ void finish_cd(W4& w, uint32_t h0, uint32_t h3, Key key) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * h0;
  w.c = (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), h3, key.k1 + 9u * 0xBB67AE85u, 0x96);
  w.d = (uint32_t)p0;
}

__device__ __forceinline__ uint32_t tag(uint32_t purpose, uint32_t gen) {
  return (purpose << 28) | (gen << 24);
}

// A lazily evaluated word stream: counter (game, ep, c2, tag | block).
struct Stream {
  uint32_t c0, c1, c2, c3;
  uint32_t idx;
  W4 w;

  __device__ __forceinline__ void init(uint32_t game, uint32_t ep, uint32_t cc2, uint32_t t,
                                       uint32_t start = 0) {
    c0 = game; c1 = ep; c2 = cc2; c3 = t; idx = start;
  }
  __device__ __forceinline__ uint32_t next(Key key) {
    const uint32_t j = idx & 3u;
    if (j == 0) w = philox(c0, c1, c2, c3 | (idx >> 2), key);
    ++idx;
    return j == 0 ? w.a : j == 1 ? w.b : j == 2 ? w.c : w.d;
  }
};

// numpy legacy RandomState.randint(low, high): rng = high-1-low; rng == 0
// draws nothing; otherwise masked rejection on 32-bit words.
struct NpBound {
  uint32_t rng, mask;
  __device__ __forceinline__ void set(int32_t n) {  // n = high - low
    rng = (uint32_t)(n - 1);
    mask = rng ? 0xFFFFFFFFu >> __clz(rng) : 0u;
  }
};

// ---------------------------------------------------------------------------
// Per-game registers
// ---------------------------------------------------------------------------
struct Player {
  int32_t x, y, d, hp, sx, sy;
  int32_t lay;    // bank layout of the player's depth (dungeon bank only)
  int32_t move;   // validated move for this tick
  int32_t tx, ty; // target cell of `move` from the pre-tick position
  // character mechanics (ORX_EXT_RPG; never touched by the kernels that are
  // compiled with those flags known off)
  int32_t mana, xp, dmg, mhp, nitems;
  int32_t cool;   // ORX_EXT_README_COMBAT: ticks of cooldown left
  int32_t heal;   // this tick's move is ORX_MOVE_HEAL (a Stay)
  int32_t hd;     // damage of this tick's hit on an NPC
};

// Field-wise select: a conditional copy of the whole struct would be lowered
// through scratch memory (two allocas + pointer select).
__device__ __forceinline__ Player pick(bool c, const Player& a, const Player& b) {
  Player r;
  r.x = c ? a.x : b.x;
  r.y = c ? a.y : b.y;
  r.d = c ? a.d : b.d;
  r.hp = c ? a.hp : b.hp;
  r.sx = c ? a.sx : b.sx;
  r.sy = c ? a.sy : b.sy;
  r.lay = c ? a.lay : b.lay;
  r.move = c ? a.move : b.move;
  r.tx = c ? a.tx : b.tx;
  r.ty = c ? a.ty : b.ty;
  r.mana = c ? a.mana : b.mana;
  r.xp = c ? a.xp : b.xp;
  r.dmg = c ? a.dmg : b.dmg;
  r.mhp = c ? a.mhp : b.mhp;
  r.nitems = c ? a.nitems : b.nitems;
  r.cool = c ? a.cool : b.cool;
  r.heal = c ? a.heal : b.heal;
  r.hd = c ? a.hd : b.hd;
  return r;
}

// Depths each player's dstore ring holds (orx_dstore_depths, include/orx.h):
// the smallest power of two >= max(max_ticks, ORX_DSTORE_MIN), capped at
// ORX_DSTORE_MAX; ORX_DSTORE_UNBOUNDED without a tick limit.
__host__ __device__ inline uint32_t dstore_depths(int32_t max_ticks) {
  if (max_ticks <= 0) return ORX_DSTORE_UNBOUNDED;
  uint32_t n = ORX_DSTORE_MIN;
  while (n < (uint32_t)max_ticks && n < ORX_DSTORE_MAX) n <<= 1;
  return n;
}

struct Cfg {  // device copy of orx_cfg_t plus derived constants (all wave-uniform)
  int32_t W, H, despawn, max_ticks, start_mode, d1, d2, K;
  int32_t npc_hp, player_hp, player_dmg_net, autoreset;
  int32_t npc_pol, npc_dmg_net;  // the enemy AI (ORX_NPC_*) and an NPC's damage - armor
  int32_t ext, sep_period;  // ORX_EXT_* build extensions (0 in FAST kernels)
  // character mechanics (ORX_EXT_RPG)
  int32_t player_dmg, player_armor, mana_max, mana_third, mana_regen, mana_pp;
  int32_t xp_kill, xp_level, drop_pct, item_bonus, item_slots, cooldown;
  int32_t ih;        // H - 2 (interior column height)
  uint32_t dstore_n; // stock-seed mode: depths per player's dstore ring (a power of two)
  // ceil(2^32 / d) for d = ih and d = H: n / d == umulhi(n, magic) for every
  // n < 2^16 (error < n / 2^32 <= 1/d), so set only when the dividends
  // (interior / grid cell indices) stay below 2^16; 0 = divide
  uint32_t ih_magic, h_magic;
  // separation damage's ceil(k / sep_period) as a multiply: for every
  // n < 2^31, n / P == (n * sep_m) >> sep_sh with l = ceil(log2 P),
  // sep_m = floor(2^(31+l) / P) + 1 < 2^32, sep_sh = 31 + l (the error term
  // n * (sep_m * P - 2^(31+l)) / (P * 2^(31+l)) stays below 1/P)
  uint32_t sep_m;
  int32_t sep_sh;
  NpBound ground;    // randint(n_ground), n_ground = (W-2)(H-2) - 1
  NpBound stair_x;   // randint(1, W-2)
  NpBound stair_y;   // randint(1, H-2)
  // dungeon bank (n_layouts > 0): layouts as Dungeon.tiles, Ground lists, meta
  int32_t L;
  NpBound layout;    // randint(L)
  const uint8_t* tiles;
  const uint16_t* gground;
  const int32_t* gmeta;
  bool lds_tiles;    // the bank's tiles are staged in orx_lds_tiles (rollout)
};

// The dungeon bank's tiles in LDS (the rollout stages them once per block
// when they fit the device's per-workgroup LDS; every tile test of the tick
// then reads LDS instead of waiting out an L2 round trip -- at one wave per
// SIMD nothing hides that latency).  Above kMaxLdsTiles (the default
// per-workgroup limit) the launch raises the kernel's limit first.
extern __shared__ uint8_t orx_lds_tiles[];
inline constexpr uint32_t kMaxLdsTiles = 64 * 1024;
inline constexpr uint32_t kMaxLdsBlock = 160 * 1024;  // LDS per CU (one workgroup may take it all)

struct Deltas {  // counter / return increments, flushed once per launch
  int32_t combat, descend, dungeon, npc_death, ret, eps;
#ifdef ORX_STAMPS
  uint32_t n_rare = 0, n_ordered = 0, n_hits = 0, n_desc = 0, n_meet = 0,  // rare-block entries
           n_reset = 0;
  uint32_t n_lean = 0;  // lean ticks (pair_rollout_kernel's StaircaseBot spans)
  uint32_t cy_rare = 0, cy_reset = 0, cy_ordered = 0, cy_desc = 0;  // cycles in them
#endif
};

// Update-event sink (orx_step_events): records {type, iden, a, b} in the
// order the reference appends GameStateUpdates (updater.py:133-145).  With
// EV = false every emit compiles away.
template <bool EV>
struct Events {
  int32_t* base;  // this game's [cap][4]
  int32_t n;
  int32_t cap = ORX_MAX_EVENTS;  // records per game (orx_max_events)
  __device__ __forceinline__ void emit(int32_t type, int32_t iden, int32_t a, int32_t b) {
    if constexpr (EV) {
      if (n < cap) {
        base[4 * n] = type; base[4 * n + 1] = iden; base[4 * n + 2] = a; base[4 * n + 3] = b;
      }
      ++n;
    }
  }
};

// NPC slots in registers: packed (x | y << 8) u16 pairs; dead slot = 0xFFFF,
// which no legal target can equal (targets are interior cells, x, y <= 254).
template <int NCAP>
struct Npcs {
  static constexpr int kRegs = NCAP > 0 ? NCAP / 2 : 1;
  // named registers (an array would be demoted to scratch by SROA)
  uint32_t q0, q1, q2, q3, q4, q5, q6, q7;
  uint32_t alive;

  __device__ __forceinline__ uint32_t rd(int r) const {
    switch (r) {
      case 0: return q0; case 1: return q1; case 2: return q2; case 3: return q3;
      case 4: return q4; case 5: return q5; case 6: return q6; default: return q7;
    }
  }
  __device__ __forceinline__ void wr(int r, uint32_t v) {
    switch (r) {
      case 0: q0 = v; break; case 1: q1 = v; break; case 2: q2 = v; break;
      case 3: q3 = v; break; case 4: q4 = v; break; case 5: q5 = v; break;
      case 6: q6 = v; break; default: q7 = v; break;
    }
  }
  __device__ __forceinline__ void clear() {
    q0 = q1 = q2 = q3 = q4 = q5 = q6 = q7 = 0xFFFFFFFFu;
    alive = 0;
  }
  // the alive mask (GameState.entities membership), one bit per slot
  __device__ __forceinline__ void bind(const orx_state_t&, const Cfg&, uint32_t, uint32_t) {}
  __device__ __forceinline__ bool is_alive(int k) const { return (alive >> k) & 1u; }
  __device__ __forceinline__ void mark_alive(int k) { alive |= 1u << k; }
  __device__ __forceinline__ void mark_dead(int k) { alive &= ~(1u << k); }
  __device__ __forceinline__ bool any_alive() const { return alive != 0; }
  __device__ __forceinline__ int count_alive() const { return __popc(alive); }
  __device__ __forceinline__ void store_alive(uint32_t* rows, uint32_t, uint32_t i) const {
    rows[i] = alive;
  }
  __device__ __forceinline__ uint32_t get(int k) const {
    return (rd(k >> 1) >> ((k & 1) * 16)) & 0xFFFFu;
  }
  __device__ __forceinline__ void set(int k, uint32_t v) {
    const int sh = (k & 1) * 16;
    wr(k >> 1, (rd(k >> 1) & ~(0xFFFFu << sh)) | ((v & 0xFFFFu) << sh));
  }
  // The game setup fills slots 0, 1, ... in order with a per-lane count: a
  // runtime slot index would lower to a branch ladder, so each placement is
  // shifted in at the top of the slot chain (v_alignbit per register, kept
  // where `take` is false) and align(n) moves the n placed slots down to 0.
  __device__ __forceinline__ void push_top(uint32_t v, bool take) {
    if constexpr (NCAP > 0) {
#pragma unroll
      for (int r = 0; r < kRegs; ++r) {  // ascending: q[r + 1] is still the old one
        const uint32_t hi = r + 1 < kRegs ? rd(r + 1) : v;
        const uint32_t n = __builtin_amdgcn_alignbit(hi, rd(r), 16);
        wr(r, take ? n : rd(r));
      }
    }
  }
  __device__ __forceinline__ void align(int n) {
    if (n < NCAP) {
#pragma unroll
      for (int k = 0; k < NCAP; ++k) push_top(0xFFFFu, k < NCAP - n);
    }
  }
  // True iff some slot holds `key`: zero-halfword test on (slots ^ key),
  // (v - 0x00010001) & ~v & 0x80008000 is nonzero iff a 16-bit half is zero.
  __device__ __forceinline__ bool any(uint32_t key) const {
    if constexpr (NCAP == 0) {
      return false;
    } else {
      const uint32_t k2 = key | (key << 16);
      uint32_t z = 0;
#pragma unroll
      for (int r = 0; r < kRegs; ++r) {
        const uint32_t x = rd(r) ^ k2;
        z |= (x - 0x00010001u) & ~x & 0x80008000u;
      }
      return z != 0;
    }
  }
  // Slot holding `key` (a live NPC), or -1.
  __device__ __forceinline__ int find(uint32_t key) const {
    if constexpr (NCAP == 0) {
      return -1;
    } else {
      const uint32_t k2 = key | (key << 16);
      uint32_t hitmask = 0;
#pragma unroll
      for (int r = 0; r < kRegs; ++r) {
        const uint32_t x = rd(r) ^ k2;
        // zero-halfword flags as in any(): a low half is flagged iff zero; a
        // high half can be falsely flagged only above a true low-half match,
        // and the lowest flag wins
        const uint32_t z = (x - 0x00010001u) & ~x & 0x80008000u;
        hitmask |= ((z >> 15) | (z >> 30)) << (2 * r);  // bit 2r: low half, 2r+1: high
      }
      return hitmask ? (int)__builtin_ctz(hitmask) : -1;
    }
  }
  // A live NPC holds `key` (with ORX_EXT_ITEMS a slot may hold its dropped
  // item instead; keys of occupied slots are distinct).
  __device__ __forceinline__ bool live(uint32_t key) const {
    const int k = find(key);
    return k >= 0 && is_alive(k);
  }
  // slot k's cell / slot k := v for a runtime k (the moving-NPC tick's
  // initiative order): a select of the 64-bit register pair k >> 2, then
  // shifts -- get(k) / set(k) through rd / wr would demote q0..q7 to scratch
  __device__ __forceinline__ uint32_t get_rt(int k) const {
    if constexpr (NCAP == 0) {
      return 0xFFFFu;
    } else {
      const int j = k >> 2;
      uint64_t p = (uint64_t)q0 | ((uint64_t)q1 << 32);
      if constexpr (NCAP > 4) p = j == 1 ? ((uint64_t)q2 | ((uint64_t)q3 << 32)) : p;
      if constexpr (NCAP > 8) {
        p = j == 2 ? ((uint64_t)q4 | ((uint64_t)q5 << 32)) : p;
        p = j == 3 ? ((uint64_t)q6 | ((uint64_t)q7 << 32)) : p;
      }
      return (uint32_t)(p >> (16 * (k & 3))) & 0xFFFFu;
    }
  }
  __device__ __forceinline__ void set_rt(int k, uint32_t v) {
    if constexpr (NCAP > 0) {
      const int sh = 16 * (k & 3), j = k >> 2;
      const uint64_t m = 0xFFFFull << sh, b = (uint64_t)(v & 0xFFFFu) << sh;
      uint64_t p = (uint64_t)q0 | ((uint64_t)q1 << 32);
      p = j == 0 ? ((p & ~m) | b) : p;
      q0 = (uint32_t)p; q1 = (uint32_t)(p >> 32);
      if constexpr (NCAP > 4) {
        p = (uint64_t)q2 | ((uint64_t)q3 << 32);
        p = j == 1 ? ((p & ~m) | b) : p;
        q2 = (uint32_t)p; q3 = (uint32_t)(p >> 32);
      }
      if constexpr (NCAP > 8) {
        p = (uint64_t)q4 | ((uint64_t)q5 << 32);
        p = j == 2 ? ((p & ~m) | b) : p;
        q4 = (uint32_t)p; q5 = (uint32_t)(p >> 32);
        p = (uint64_t)q6 | ((uint64_t)q7 << 32);
        p = j == 3 ? ((p & ~m) | b) : p;
        q6 = (uint32_t)p; q7 = (uint32_t)(p >> 32);
      }
    }
  }
  // slot k := dead for a runtime k: 64-bit shifts over register pairs (a
  // switch on k lowers to a branch ladder)
  __device__ __forceinline__ void kill(int k) {
    if constexpr (NCAP > 0) {
      const uint64_t m = 0xFFFFull << (16 * (k & 3));
      const int j = k >> 2;
      uint64_t p = (uint64_t)q0 | ((uint64_t)q1 << 32);
      p |= j == 0 ? m : 0ull;
      q0 = (uint32_t)p; q1 = (uint32_t)(p >> 32);
      p = (uint64_t)q2 | ((uint64_t)q3 << 32);
      p |= j == 1 ? m : 0ull;
      q2 = (uint32_t)p; q3 = (uint32_t)(p >> 32);
      if constexpr (NCAP > 8) {
        p = (uint64_t)q4 | ((uint64_t)q5 << 32);
        p |= j == 2 ? m : 0ull;
        q4 = (uint32_t)p; q5 = (uint32_t)(p >> 32);
        p = (uint64_t)q6 | ((uint64_t)q7 << 32);
        p |= j == 3 ? m : 0ull;
        q6 = (uint32_t)p; q7 = (uint32_t)(p >> 32);
      }
    }
  }
};

// Dense NPCs (K > 16, up to 255): the NPCs of a game live in HBM -- an
// occupancy grid of its NPC depth, one byte per cell (slot + 1, 0 = empty;
// st.npc_grid [B][W*H], cell x * H + y, one game's grid contiguous so a reset
// clears it with wide stores), the slot rows npc_pos / npc_health, and the
// alive bits as rows of 32 (npc_alive [ceil(K/32)][B]).  A target test is one
// byte load instead of a register scan; it is the form for NPC counts that
// no register file holds (GameState.entities is unbounded, state.py:25-34).
constexpr int kDense = 256;

// The rollout also stages each game's occupancy as a bitmap in LDS (one bit
// per cell, 512 B per 64x64 game), so the tick's two target tests read LDS:
// at one wave per SIMD an HBM round trip per tick would not be hidden.
template <>
struct Npcs<kDense> {
  uint8_t* grid;   // this game's grid
  uint16_t* pos;   // npc_pos + i (stride B)
  uint32_t* rows;  // npc_alive + i (stride B)
  uint32_t B;
  int32_t H, cells, K;
  bool staged;     // the bitmap copy in LDS (rollout) is kept in step
  uint32_t boff;   // its first word in orx_lds_tiles

  __device__ __forceinline__ void bind(const orx_state_t& st, const Cfg& c, uint32_t B_,
                                       uint32_t i) {
    B = B_; H = c.H; cells = c.W * c.H; K = c.K;
    grid = st.npc_grid + (size_t)i * (size_t)cells;
    pos = st.npc_pos + i;
    rows = st.npc_alive + i;
    staged = false;
    boff = 0;
  }
  __device__ __forceinline__ uint32_t* lds() const {
    return reinterpret_cast<uint32_t*>(orx_lds_tiles);
  }
  __device__ __forceinline__ int cell(uint32_t key) const {
    return (int)(key & 0xFFu) * H + (int)(key >> 8);
  }
  __device__ __forceinline__ void clear_bits() {
    for (int w = 0; w < (cells + 31) >> 5; ++w) lds()[boff + w] = 0u;
  }
  // builds this game's LDS bitmap at word `off` from its live NPCs
  __device__ __forceinline__ void stage(uint32_t off) {
    boff = off;
    staged = true;
    clear_bits();
    // per row of 32 slots: its alive word and all 32 positions in flight at
    // once (one HBM round trip per row, not per NPC)
    for (int r = 0; r < (K + 31) >> 5; ++r) {
      const uint32_t a = rows[(size_t)r * B];
      uint32_t p[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) p[j] = pos[(size_t)min(r * 32 + j, K - 1) * B];
#pragma unroll
      for (int j = 0; j < 32; ++j)
        if ((a >> j) & 1u) {
          const int cl = cell(p[j]);
          lds()[boff + (cl >> 5)] |= 1u << (cl & 31);
        }
    }
  }
  __device__ __forceinline__ void clear() {  // the grid and the alive rows
    // (a game's row starts on a 4-byte boundary only when W * H is a
    // multiple of 4: bytes up to the first boundary, words, the tail bytes)
    const int head = min((int)((4u - ((uint32_t)(uintptr_t)grid & 3u)) & 3u), cells);
    for (int j = 0; j < head; ++j) grid[j] = 0;
    uint32_t* g4 = reinterpret_cast<uint32_t*>(grid + head);
    const int words = (cells - head) >> 2;
    for (int j = 0; j < words; ++j) g4[j] = 0u;
    for (int j = head + 4 * words; j < cells; ++j) grid[j] = 0;
    for (int r = 0; r < (K + 31) >> 5; ++r) rows[(size_t)r * B] = 0u;
    if (staged) clear_bits();
  }
  __device__ __forceinline__ bool is_alive(int k) const {
    return (rows[(size_t)(k >> 5) * B] >> (k & 31)) & 1u;
  }
  __device__ __forceinline__ void mark_alive(int k) { rows[(size_t)(k >> 5) * B] |= 1u << (k & 31); }
  __device__ __forceinline__ void mark_dead(int k) { rows[(size_t)(k >> 5) * B] &= ~(1u << (k & 31)); }
  __device__ __forceinline__ bool any_alive() const { return true; }  // (an optimization only)
  __device__ __forceinline__ int count_alive() const {
    int n = 0;
    for (int r = 0; r < (K + 31) >> 5; ++r) n += __popc(rows[(size_t)r * B]);
    return n;
  }
  __device__ __forceinline__ void store_alive(uint32_t*, uint32_t, uint32_t) const {}  // in place
  __device__ __forceinline__ uint32_t get(int k) const { return pos[(size_t)k * B]; }
  __device__ __forceinline__ uint32_t get_rt(int k) const { return get(k); }
  __device__ __forceinline__ void set_rt(int k, uint32_t key) { set(k, key); }
  __device__ __forceinline__ void set(int k, uint32_t key) {
    const int cl = cell(key);
    grid[cl] = (uint8_t)(k + 1);
    pos[(size_t)k * B] = (uint16_t)key;
    if (staged) lds()[boff + (cl >> 5)] |= 1u << (cl & 31);
  }
  __device__ __forceinline__ bool any(uint32_t key) const {
    const int cl = cell(key);
    if (staged) return (lds()[boff + (cl >> 5)] >> (cl & 31)) & 1u;
    return grid[cl] != 0;
  }
  __device__ __forceinline__ int find(uint32_t key) const { return (int)grid[cell(key)] - 1; }
  __device__ __forceinline__ bool live(uint32_t key) const {
    const int k = find(key);
    return k >= 0 && is_alive(k);
  }
  __device__ __forceinline__ void kill(int k) { kill_at(get(k)); }
  __device__ __forceinline__ void kill_at(uint32_t key) {  // the NPC on cell `key`
    const int cl = cell(key);
    grid[cl] = 0;
    if (staged) lds()[boff + (cl >> 5)] &= ~(1u << (cl & 31));
  }
};

// Both players' NPC occupancy tests in one pass over the slot registers
// (the rollout's common path): with K = k1 | k2 << 16 and its half-swap Ks,
// the packed 16-bit minimum over (slots ^ K) has a zero low half iff some
// low slot holds k1 and a zero high half iff some high slot holds k2; over
// (slots ^ Ks) the same for the other two pairings.
template <int NCAP>
__device__ __forceinline__ void npc_any2(const Npcs<NCAP>& npc, uint32_t k1, uint32_t k2,
                                         bool& h1, bool& h2) {
  if constexpr (NCAP == 0) {
    h1 = h2 = false;
  } else if constexpr (NCAP == kDense) {
    h1 = npc.any(k1);
    h2 = npc.any(k2);
  } else {
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const uint32_t K = k1 | (k2 << 16), Ks = k2 | (k1 << 16);
    u16x2 mx = __builtin_bit_cast(u16x2, npc.rd(0) ^ K);
    u16x2 my = __builtin_bit_cast(u16x2, npc.rd(0) ^ Ks);
#pragma unroll
    for (int r = 1; r < Npcs<NCAP>::kRegs; ++r) {
      mx = __builtin_elementwise_min(mx, __builtin_bit_cast(u16x2, npc.rd(r) ^ K));
      my = __builtin_elementwise_min(my, __builtin_bit_cast(u16x2, npc.rd(r) ^ Ks));
    }
    const u16x2 z = __builtin_elementwise_min(mx, my.yx);
    h1 = z.x == 0;
    h2 = z.y == 0;
  }
}

// One key against every slot (the paired rollout's per-player test): the
// zero-halfword test of npc_any2 on (slots ^ key:key), the two halves of the
// running minimum folded at the end.
// npc_any1 for a register-slot game with the NPC depth folded into the key:
// dk = 0x80008000 when the player is not on the NPCs' depth (a half no slot
// holds: live keys keep bit 15 clear, dead slots are 0xFFFF), 0 when it is
template <int NCAP>
__device__ __forceinline__ bool npc_any1_dk(const Npcs<NCAP>& npc, uint32_t k, uint32_t dk) {
  if constexpr (NCAP == 0 || NCAP == kDense) {
    return false;
  } else {
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const uint32_t KK = ((k << 16) | dk) | k;
    u16x2 m = __builtin_bit_cast(u16x2, npc.rd(0) ^ KK);
#pragma unroll
    for (int r = 1; r < Npcs<NCAP>::kRegs; ++r)
      m = __builtin_elementwise_min(m, __builtin_bit_cast(u16x2, npc.rd(r) ^ KK));
    return __builtin_elementwise_min(m, m.yx).x == 0;
  }
}

template <int NCAP>
__device__ __forceinline__ bool npc_any1(const Npcs<NCAP>& npc, uint32_t k) {
  if constexpr (NCAP == 0) {
    return false;
  } else if constexpr (NCAP == kDense) {
    return npc.any(k);
  } else {
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const uint32_t KK = k | (k << 16);
    u16x2 m = __builtin_bit_cast(u16x2, npc.rd(0) ^ KK);
#pragma unroll
    for (int r = 1; r < Npcs<NCAP>::kRegs; ++r)
      m = __builtin_elementwise_min(m, __builtin_bit_cast(u16x2, npc.rd(r) ^ KK));
    return __builtin_elementwise_min(m, m.yx).x == 0;
  }
}

__device__ __forceinline__ uint32_t pack_xy(int32_t x, int32_t y) {
  return (uint32_t)(x & 0xFF) | ((uint32_t)(y & 0xFF) << 8);
}

// calculate_pos (updater.py:340-351) as two 2-bit lookup tables indexed by the
// move (1..5): entry = delta + 1.  Up (0,-1), Right (+1,0), Down (0,+1),
// Left (-1,0), Stay (0,0).
constexpr uint32_t kDx = (1u << 2) | (2u << 4) | (1u << 6) | (0u << 8) | (1u << 10);
constexpr uint32_t kDy = (0u << 2) | (1u << 4) | (2u << 6) | (1u << 8) | (1u << 10);
__device__ __forceinline__ void calc_pos(int32_t x, int32_t y, int32_t m, int32_t& nx, int32_t& ny) {
  const uint32_t sh = (uint32_t)m << 1;
  nx = x + (int32_t)((kDx >> sh) & 3u) - 1;
  ny = y + (int32_t)((kDy >> sh) & 3u) - 1;
}

// Dungeon.tiles[x, y] of bank layout `lay` (x, y inside the grid).
// (The two reads must stay two: merged, they become one flat load of a
// selected pointer, whose completion waits for every vector memory operation
// in flight -- the trajectory stores of the ticks before -- measured +10% on
// a bank's rollout.  The asm on the global read keeps them apart.)
__device__ __forceinline__ uint32_t bank_tile_at(const Cfg& c, uint32_t idx) {
  if (c.lds_tiles) return orx_lds_tiles[idx];
  uint32_t r = c.tiles[idx];
  asm volatile("" : "+v"(r));
  return r;
}
__device__ __forceinline__ uint32_t bank_tile(const Cfg& c, int32_t lay, int32_t x, int32_t y) {
  return bank_tile_at(c, (uint32_t)lay * (uint32_t)(c.W * c.H) + (uint32_t)(x * c.H + y));
}
// The same from the LDS copy (launches that staged the bank: the paired form)
__device__ __forceinline__ uint32_t bank_tile_lds(const Cfg& c, int32_t lay, int32_t x, int32_t y) {
  return orx_lds_tiles[(uint32_t)lay * (uint32_t)(c.W * c.H) + (uint32_t)(x * c.H + y)];
}

// Dungeon.is_blocked (world.py:41-46).  GRID = dungeon bank: outside the grid
// or a Wall tile; else EmptyDungeonGenerator's border.
template <bool GRID>
__device__ __forceinline__ bool blocked(const Cfg& c, int32_t lay, int32_t x, int32_t y) {
  if constexpr (GRID) {
    if (x < 0 || x >= c.W || y < 0 || y >= c.H) return true;
    return bank_tile(c, lay, x, y) == ORX_TILE_WALL;
  } else {
    return x <= 0 || x >= c.W - 1 || y <= 0 || y >= c.H - 1;
  }
}

// dung.tiles[newx, newy] == Tile.StaircaseDown (updater.py:205-206) for an
// unblocked target: any staircase tile of a bank layout; the one staircase of
// an EmptyDungeonGenerator dungeon.
template <bool GRID>
__device__ __forceinline__ bool stair_tile(const Cfg& c, const Player& p, int32_t x, int32_t y) {
  if constexpr (GRID)
    return bank_tile(c, p.lay, x, y) == ORX_TILE_STAIRCASE_DOWN;
  else
    return x == p.sx && y == p.sy;
}

// randint(n_ground) bound of a dungeon (world.py:62).
template <bool GRID>
__device__ __forceinline__ NpBound ground_bound(const Cfg& c, int32_t lay) {
  if constexpr (!GRID) {
    return c.ground;
  } else {
    NpBound b;
    b.set(c.gmeta[4 * lay]);
    return b;
  }
}

// choice-th Ground tile, x-major order: the bank's Ground list, or the
// closed form for the dungeon with staircase (sx, sy).
template <bool GRID>
__device__ __forceinline__ void ground_cell(const Cfg& c, uint32_t ch, int32_t lay, int32_t sx,
                                            int32_t sy, int32_t& x, int32_t& y) {
  if constexpr (GRID) {
    const uint32_t flat = c.gground[(size_t)lay * (uint32_t)(c.W * c.H) + ch];
    const uint32_t q = c.h_magic ? __umulhi(flat, c.h_magic) : flat / (uint32_t)c.H;
    x = (int32_t)q;
    y = (int32_t)(flat - q * (uint32_t)c.H);
    return;
  }
  const uint32_t s_idx = (uint32_t)((sx - 1) * c.ih + (sy - 1));
  const uint32_t ci = ch + (ch >= s_idx ? 1u : 0u);
  const uint32_t q = c.ih_magic ? __umulhi(ci, c.ih_magic) : ci / (uint32_t)c.ih;
  x = 1 + (int32_t)q;
  y = 1 + (int32_t)(ci - q * (uint32_t)c.ih);
}

// EmptyDungeonGenerator.spawn_dungeon (worldgen.py:33-43) from a word
// stream: randint(1, W-2) then randint(1, H-2); or, with a dungeon bank,
// layout randint(L) and its staircase.  S = Stream (keyed Philox) or
// MtStream (stock-seed numpy state).  One loop, one draw site.
template <bool GRID, class S>
__device__ __forceinline__ void dungeon_draw(const Cfg& c, S& s, Key key, int32_t& sx, int32_t& sy,
                                          int32_t& lay, bool& err) {
  if constexpr (GRID) {
    uint32_t v = 0;
    bool ok = c.layout.rng == 0;
    for (uint32_t t = 0; t < kWordCap && !ok; ++t) {
      v = s.next(key) & c.layout.mask;
      ok = v <= c.layout.rng;
    }
    if (!ok) { err = true; v = 0; }
    lay = (int32_t)v;
    sx = c.gmeta[4 * lay + 1];
    sy = c.gmeta[4 * lay + 2];
    return;
  }
  lay = -1;
  int n = 0;
  int32_t v0 = 0, v1 = 0;
  for (uint32_t t = 0; t < 2 * kWordCap && n < 2; ++t) {
    const NpBound b = n == 0 ? c.stair_x : c.stair_y;
    uint32_t v = 0;
    if (b.rng != 0) {  // rng 0 consumes no word
      v = s.next(key) & b.mask;
      if (v > b.rng) continue;
    }
    if (n == 0) v0 = (int32_t)v; else v1 = (int32_t)v;
    ++n;
  }
  if (n < 2) err = true;
  sx = 1 + v0;
  sy = 1 + v1;
}

// EmptyDungeonGenerator.spawn_dungeon from the first block of its keyed
// stream: randint(1, W-2) takes the first accepted of words a, b, c and
// randint(1, H-2) the first accepted word after it.  False when the block
// holds no such pair (p ~ 1e-5 at 128x128) or a bound consumes no word
// (W or H = 4); the caller then runs dungeon_draw, which reads the same words.
__device__ __forceinline__ bool stair_from_block(const Cfg& c, const W4& w, int32_t& sx,
                                                 int32_t& sy) {
  const NpBound bx = c.stair_x, by = c.stair_y;
  if (bx.rng == 0u || by.rng == 0u) return false;
  const uint32_t x0 = w.a & bx.mask, x1 = w.b & bx.mask, x2 = w.c & bx.mask;
  const uint32_t y1 = w.b & by.mask, y2 = w.c & by.mask, y3 = w.d & by.mask;
  const bool ax0 = x0 <= bx.rng, ax1 = x1 <= bx.rng, ax2 = x2 <= bx.rng;
  const bool ay1 = y1 <= by.rng, ay2 = y2 <= by.rng, ay3 = y3 <= by.rng;
  const uint32_t y_after1 = ay2 ? y2 : y3;               // y after x at word b
  const uint32_t y_after0 = ay1 ? y1 : y_after1;         // y after x at word a
  sx = 1 + (int32_t)(ax0 ? x0 : ax1 ? x1 : x2);
  sy = 1 + (int32_t)(ax0 ? y_after0 : ax1 ? y_after1 : y3);
  return ax0 ? (ay1 | ay2 | ay3) : ax1 ? (ay2 | ay3) : (ax2 & ay3);
}

// The keyed form: words from (episode, depth, generation).
template <bool GRID>
__device__ __forceinline__ void dungeon_stair(const Cfg& c, Key key, uint32_t game, uint32_t ep,
                                           int32_t depth, uint32_t gen, int32_t& sx, int32_t& sy,
                                           int32_t& lay, bool& err) {
  Stream s;
  s.init(game, ep, (uint32_t)depth, tag(PUR_DUNGEON, gen));
  dungeon_draw<GRID>(c, s, key, sx, sy, lay, err);
}

// ---------------------------------------------------------------------------
// Stock-seed mode (cfg.rng = ORX_RNG_MT19937): MT19937 states in HBM
// ---------------------------------------------------------------------------
// One game's MT19937 (CPython random or numpy RandomState), column stride B:
// words [0, 624), index at [624].  Lazy twist: word i of a new round is
// regenerated when it is first drawn -- it needs word i+1 of the old round
// and word i+397 mod 624 (old for i < 227, already new otherwise), exactly
// the in-place order of genrand_uint32's block twist (_randommodule.c), so
// the outputs are identical while a draw touches 3 words instead of 624.
struct MtStream {
  uint32_t* s;
  uint32_t B, idx;
  __device__ __forceinline__ void open(uint32_t* base, uint32_t B_, uint32_t i) {
    s = base + i;
    B = B_;
    idx = s[624 * (size_t)B];
  }
  __device__ __forceinline__ void close() const { s[624 * (size_t)B] = idx; }
  __device__ __forceinline__ uint32_t next(Key) {
    if (idx >= 624u) idx = 0;
    const uint32_t i = idx++;
    const uint32_t i1 = i == 623u ? 0u : i + 1u;
    const uint32_t im = i < 227u ? i + 397u : i - 227u;
    const uint32_t y = (s[(size_t)i * B] & 0x80000000u) | (s[(size_t)i1 * B] & 0x7fffffffu);
    uint32_t v = s[(size_t)im * B] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    s[(size_t)i * B] = v;
    v ^= v >> 11;
    v ^= (v << 7) & 0x9d2c5680u;
    v ^= (v << 15) & 0xefc60000u;
    v ^= v >> 18;
    return v;
  }
};

// CPython Random._randbelow_with_getrandbits(n): k = n.bit_length(),
// getrandbits(k) = word >> (32 - k), redraw while >= n (random.py).
template <class S>
__device__ __forceinline__ uint32_t py_randbelow(S& s, Key key, uint32_t n, bool& err) {
  const uint32_t sh = __clz(n);  // 32 - bit_length(n)
  for (uint32_t t = 0; t < kWordCap; ++t) {
    const uint32_t r = s.next(key) >> sh;
    if (r < n) return r;
  }
  err = true;
  return 0;
}

// Where the world-generation words come from.  PhiloxSrc: keyed streams per
// purpose (dungeons regenerate from their key, nothing stored).  MtSrc: the
// game's numpy RandomState, consumed in the reference's call order; a
// dungeon's staircase cannot be regenerated, so every dungeon a player enters
// is kept in that player's dstore ring (slot (depth - its start depth) mod N,
// N = orx_dstore_depths >= max_ticks) for the other player to find: the only
// present dungeon a player looks up is one the other player entered and has
// since left (Unreachable: other.start <= nd < other.d, updater.py:272-280),
// fewer than max_ticks of its descents ago.
struct PhiloxSrc {
  static constexpr bool kMt = false;
  Key key;
  uint32_t game, ep;
  __device__ __forceinline__ Stream init() const {
    Stream s;
    s.init(game, ep, 0, tag(PUR_INIT, 0));
    return s;
  }
  __device__ __forceinline__ Stream spawn(int32_t tick) const {
    Stream s;
    s.init(game, ep, (uint32_t)tick, tag(PUR_SPAWN, 0));
    return s;
  }
  template <bool GRID>
  __device__ __forceinline__ void dungeon(const Cfg& c, int32_t depth, uint32_t gen, int32_t& sx,
                                          int32_t& sy, int32_t& lay, bool& err) const {
    dungeon_stair<GRID>(c, key, game, ep, depth, gen, sx, sy, lay, err);
  }
  __device__ __forceinline__ bool recall(int32_t, int32_t, int32_t, int32_t&, int32_t&,
                                         int32_t&) const {
    return false;  // present dungeons are regenerated from their key
  }
  __device__ __forceinline__ void remember(int32_t, int32_t, int32_t, int32_t, int32_t,
                                           int32_t) const {}
};

struct MtSrc {
  static constexpr bool kMt = true;
  MtStream py, np;  // CPython random (bots, shuffles), numpy RandomState (world)
  int32_t* ds;      // this game's dstore column, stride B: [2][N][2]
  uint32_t B, dmask;  // dmask = N - 1 (N a power of two)
  __device__ __forceinline__ void open(const orx_state_t& st, const Cfg& c, uint32_t B_,
                                       uint32_t i) {
    py.open(st.mt_py, B_, i);
    np.open(st.mt_np, B_, i);
    ds = st.dstore + i;
    B = B_;
    dmask = c.dstore_n - 1u;
  }
  // row of player `who` (1 or 2) for depth d entered from start depth `start`
  __device__ __forceinline__ size_t row(int32_t who, int32_t start, int32_t d) const {
    const size_t k = (size_t)(who == 1 ? 0u : dmask + 1u) + ((uint32_t)(d - start) & dmask);
    return 2 * k * B;
  }
  __device__ __forceinline__ void close() const { py.close(); np.close(); }
  __device__ __forceinline__ MtStream& init() { return np; }
  __device__ __forceinline__ MtStream& spawn(int32_t) { return np; }
  template <bool GRID>
  __device__ __forceinline__ void dungeon(const Cfg& c, int32_t, uint32_t, int32_t& sx,
                                          int32_t& sy, int32_t& lay, bool& err) {
    dungeon_draw<GRID>(c, np, Key{0, 0}, sx, sy, lay, err);
  }
  // the dungeon at `depth` as player `who` (started at `start`) entered it
  __device__ __forceinline__ bool recall(int32_t who, int32_t start, int32_t depth, int32_t& sx,
                                         int32_t& sy, int32_t& lay) const {
    const size_t slot = row(who, start, depth);
    if (ds[slot] != depth) return false;
    const uint32_t v = (uint32_t)ds[slot + B];
    sx = (int32_t)(v & 0xFFu);
    sy = (int32_t)((v >> 8) & 0xFFu);
    lay = (int32_t)(v >> 16) - 1;
    return true;
  }
  __device__ __forceinline__ void remember(int32_t who, int32_t start, int32_t depth, int32_t sx,
                                           int32_t sy, int32_t lay) const {
    const size_t slot = row(who, start, depth);
    ds[slot] = depth;
    ds[slot + B] = (int32_t)(((uint32_t)sx & 0xFFu) | (((uint32_t)sy & 0xFFu) << 8) |
                             ((uint32_t)(lay + 1) << 16));
  }
};

// An empty asm that "changes" its operands: values derived from them after
// this point are recomputed rather than kept live from before it (and the
// operands are computed before it, not sunk into a later branch).
__device__ __forceinline__ void launder(int32_t& a, int32_t& b, int32_t& c, int32_t& d) {
  asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}
__device__ __forceinline__ void launder_w4(W4& w) {
  asm volatile("" : "+v"(w.a), "+v"(w.b), "+v"(w.c), "+v"(w.d));
}

// ---------------------------------------------------------------------------
// Game start (setup_game + NPC spawner), all placements in one rejection loop
// over the INIT stream (one Philox call site, one division site).
// ---------------------------------------------------------------------------
template <int NCAP, bool GRID, class Src>
__device__ __forceinline__ void setup_game(const Cfg& c, Key key, Src& src, Player& p1,
                                        Player& p2, Npcs<NCAP>& npc, int32_t& tick,
                                        int32_t& status) {
  bool err = false;
  const bool sep = c.start_mode == ORX_START_SEPARATED;
  p1.d = sep ? c.d1 : 0;
  p2.d = sep ? c.d2 : 0;
  // keyed streams: a staircase straight from its stream's first block (the
  // loop in dungeon_draw only when that block holds no accepted pair)
  bool drawn1 = false, drawn2 = false;
  W4 wi = {0u, 0u, 0u, 0u};  // the INIT stream's first block (keyed streams)
  if constexpr (!Src::kMt && !GRID) {
    // the dungeon's and the INIT stream's first blocks are independent: drawn
    // side by side, one Philox dependency chain's latency covers both
    p1.lay = p2.lay = -1;
    W4 wd = philox(src.game, src.ep, (uint32_t)p1.d, tag(PUR_DUNGEON, 0), key);
    wi = philox(src.game, src.ep, 0u, tag(PUR_INIT, 0), key);
    launder_w4(wd);
    launder_w4(wi);
    drawn1 = stair_from_block(c, wd, p1.sx, p1.sy);
    if (sep)
      drawn2 = stair_from_block(c, philox(src.game, src.ep, (uint32_t)p2.d, tag(PUR_DUNGEON, 0),
                                          key), p2.sx, p2.sy);
  }
  if (!drawn1) src.template dungeon<GRID>(c, p1.d, 0, p1.sx, p1.sy, p1.lay, err);
  src.remember(1, p1.d, p1.d, p1.sx, p1.sy, p1.lay);
  if (sep) {
    if (!drawn2) src.template dungeon<GRID>(c, p2.d, 0, p2.sx, p2.sy, p2.lay, err);
  } else {
    p2.sx = p1.sx; p2.sy = p1.sy; p2.lay = p1.lay;
  }
  src.remember(2, p2.d, p2.d, p2.sx, p2.sy, p2.lay);
  npc.clear();
  auto&& s = src.init();
  const int total = 2 + (NCAP ? c.K : 0);
  int placed = 0;
  p1.x = p1.y = p2.x = p2.y = 0;
  const NpBound g1 = ground_bound<GRID>(c, p1.lay), g2 = ground_bound<GRID>(c, p2.lay);
  uint32_t t_start = 0;  // words the loop's cap counts as taken
  if constexpr (!Src::kMt && !GRID) {
    // both players from the INIT stream's first block, as selects over its
    // four words (the loop below takes the same words one at a time); the
    // stream is left after the last word taken, for the NPCs.  A block with
    // fewer than two accepted, distinct cells (~1e-3 at 64x64) falls through
    // to the loop from word 0.
    if (g1.rng != 0u && g2.rng != 0u) {
      const W4 w = wi;  // block 0 of s
      int n = 0;
      uint32_t used = 0;
      int32_t x1 = 0, y1 = 0, x2 = 0, y2 = 0;
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t word = j == 0 ? w.a : j == 1 ? w.b : j == 2 ? w.c : w.d;
        const bool is_p2 = n == 1;
        const NpBound gb = is_p2 ? g2 : g1;
        const uint32_t v = word & gb.mask;
        int32_t x, y;
        ground_cell<GRID>(c, v, -1, is_p2 ? p2.sx : p1.sx, is_p2 ? p2.sy : p1.sy, x, y);
        const bool take = n < 2 && v <= gb.rng && !(is_p2 && !sep && x == x1 && y == y1);
        x1 = (take && n == 0) ? x : x1;
        y1 = (take && n == 0) ? y : y1;
        x2 = (take && is_p2) ? x : x2;
        y2 = (take && is_p2) ? y : y2;
        used = take ? j + 1u : used;
        n += take ? 1 : 0;
      }
      if (n == 2) {
        p1.x = x1; p1.y = y1; p2.x = x2; p2.y = y2;
        s.w = w;
        s.idx = used;
        t_start = used;
        placed = 2;
      }
    }
  }
  if constexpr (!Src::kMt && !GRID && NCAP > 0 && NCAP != kDense) {
    // the register NPCs from the INIT stream's first twelve words as straight
    // selects (the loop below takes the same words one at a time, drawing a
    // block at every fourth behind a branch): blocks 1 and 2 drawn side by
    // side, each word placing the next NPC unless it is rejected or its cell
    // is taken; the loop resumes at word 12 when fewer than K were placed
    // (~4% of games at 64x64).  An episode start (C3's synchronized resets,
    // the character mechanics' deaths) pays a third of the loop's cost.
    if (placed == 2 && placed < total) {
      W4 b1 = philox(src.game, src.ep, 0u, tag(PUR_INIT, 0) | 1u, key);
      W4 b2 = philox(src.game, src.ep, 0u, tag(PUR_INIT, 0) | 2u, key);
      launder_w4(b1);
      launder_w4(b2);
      const W4 w0 = s.w;  // block 0 (the players' words)
      const bool p2_here = p2.d == p1.d;
#pragma unroll
      for (uint32_t j = 0; j < 12; ++j) {
        const W4& b = j < 4 ? w0 : j < 8 ? b1 : b2;
        const uint32_t k = j & 3u;
        const uint32_t word = k == 0 ? b.a : k == 1 ? b.b : k == 2 ? b.c : b.d;
        const uint32_t v = word & g1.mask;
        int32_t x, y;
        ground_cell<false>(c, v, -1, p1.sx, p1.sy, x, y);
        const uint32_t cell = pack_xy(x, y);
        const bool occ = (x == p1.x && y == p1.y) || (p2_here && x == p2.x && y == p2.y) ||
                         npc.any(cell);
        const bool take = j >= t_start && placed < total && v <= g1.rng && !occ;
        npc.push_top(cell, take);
        npc.alive |= take ? 1u << (placed - 2) : 0u;
        placed += take ? 1 : 0;
      }
      s.w = b2;
      s.idx = 12u;
      t_start = 12u;
    }
  }
  for (uint32_t t = t_start; t < kWordCap && placed < total; ++t) {
    // placement 0: player 1, 1: player 2, 2+k: NPC k (all NPCs on p1's depth)
    const bool is_p2 = placed == 1;
    const NpBound gb = is_p2 ? g2 : g1;
    uint32_t v = 0;
    if (gb.rng != 0) {
      v = s.next(key) & gb.mask;
      if (v > gb.rng) continue;
    }
    const int32_t sx = is_p2 ? p2.sx : p1.sx, sy = is_p2 ? p2.sy : p1.sy;
    const int32_t lay = is_p2 ? p2.lay : p1.lay;
    int32_t x, y;
    ground_cell<GRID>(c, v, lay, sx, sy, x, y);
    bool occ = false;
    if (placed >= 1) occ = x == p1.x && y == p1.y && (placed >= 2 || !sep);
    if (placed >= 2) {
      occ = occ || (p2.d == p1.d && x == p2.x && y == p2.y);
      if constexpr (NCAP == kDense) occ = occ || npc.find(pack_xy(x, y)) >= 0;
      else occ = occ || npc.any(pack_xy(x, y));
    }
    if (occ) continue;
    if (placed == 0) { p1.x = x; p1.y = y; }
    else if (placed == 1) { p2.x = x; p2.y = y; }
    else if constexpr (NCAP == kDense) {
      npc.set(placed - 2, pack_xy(x, y));
      npc.mark_alive(placed - 2);
    } else if constexpr (NCAP > 0) {
      npc.push_top(pack_xy(x, y), true);
      npc.mark_alive(placed - 2);
    }
    ++placed;
  }
  if constexpr (NCAP > 0 && NCAP != kDense) npc.align(placed - 2);
  if (placed < total) err = true;
  p1.hp = c.player_hp;
  p2.hp = c.player_hp;
  // character mechanics (ORX_EXT_RPG): a fresh character's attributes
  p1.mana = p2.mana = c.mana_max;
  p1.xp = p2.xp = 0;
  p1.dmg = p2.dmg = c.player_dmg;
  p1.mhp = p2.mhp = c.player_hp;
  p1.nitems = p2.nitems = 0;
  p1.cool = p2.cool = 0;
  tick = kStartTick;
  status = err ? ORX_STATUS_RNG_EXHAUSTED : ORX_IN_PROGRESS;
}

template <int NCAP, bool GRID = false>
__device__ __forceinline__ void setup_game(const Cfg& c, Key key, uint32_t game, uint32_t ep,
                                        Player& p1, Player& p2, Npcs<NCAP>& npc, int32_t& tick,
                                        int32_t& status) {
  PhiloxSrc src{key, game, ep};
  setup_game<NCAP, GRID>(c, key, src, p1, p2, npc, tick, status);
}

// ---------------------------------------------------------------------------
// Descend (rare): dungeon presence, staircase, spawn cell
// ---------------------------------------------------------------------------
// Dungeon presence when `self` enters depth nd (derivation in DESIGN.md):
//   Unreachable: World has nd iff the other player has been on nd
//                (other.start <= nd <= other.d); generation is always 0.
//   Unused:      World == {p1.d, p2.d}, so nd is present iff other.d == nd;
//                a fresh copy is generation 1 iff the other player already
//                passed through nd (other.start <= nd < other.d).
template <int NCAP, bool EV, bool GRID, class Src, class S>
__device__ __forceinline__ void descend(const Cfg& c, Key key, Src& src, Player& self,
                                     const Player& other, int32_t other_start,
                                     const Npcs<NCAP>& npc, S& spawn, Deltas& dl, bool& err,
                                     int32_t self_iden, Events<EV>& ev) {
  const int32_t nd = self.d + 1;
  bool present;
  uint32_t gen = 0;
  if (c.despawn == ORX_DESPAWN_UNREACHABLE) {
    present = other_start <= nd && nd <= other.d;
  } else {
    present = other.d == nd;
    gen = (!present && other_start <= nd && nd < other.d) ? 1u : 0u;
  }
  // keyed streams: the new dungeon's first block and the SPAWN stream's are
  // independent, so they are drawn side by side (one Philox chain's latency
  // for both) even when the dungeon is the other player's
  constexpr bool kFirst = !Src::kMt && !GRID && std::is_same<S, Stream>::value;
  W4 wd = {0u, 0u, 0u, 0u}, ws = {0u, 0u, 0u, 0u};
  if constexpr (kFirst) {
    wd = philox(src.game, src.ep, (uint32_t)nd, tag(PUR_DUNGEON, gen), key);
    ws = philox(spawn.c0, spawn.c1, spawn.c2, spawn.c3, key);
    launder_w4(wd);
    launder_w4(ws);
  }
  int32_t sx, sy, lay;
  if (present && other.d == nd) {
    sx = other.sx; sy = other.sy; lay = other.lay;
  } else if (!(present && src.recall(3 - self_iden, other_start, nd, sx, sy, lay))) {
    // keyed: regenerate (present or not); stock-seed: a present dungeon must
    // be in the other player's ring (orx_dstore_depths: always, up to
    // max_ticks), else draw it
    if (Src::kMt && present) err = true;
    bool drawn = false;
    if constexpr (!Src::kMt && !GRID) {  // straight from the stream's first block
      lay = -1;
      if constexpr (kFirst) drawn = stair_from_block(c, wd, sx, sy);
      else
        drawn = stair_from_block(c, philox(src.game, src.ep, (uint32_t)nd, tag(PUR_DUNGEON, gen),
                                           key), sx, sy);
    }
    if (!drawn) src.template dungeon<GRID>(c, nd, gen, sx, sy, lay, err);
  }
  src.remember(self_iden, self_iden == 1 ? c.d1 : c.d2, nd, sx, sy, lay);
  if (!present) {
    dl.dungeon += 1;
    ev.emit(ORX_EV_DUNGEON, 0, nd, 0);                 // updater.py:278-280
  }
  const bool npc_depth = NCAP > 0 && nd == c.d1 && npc.any_alive();
  int32_t x = 0, y = 0;
  bool done = false;
  const NpBound gb = ground_bound<GRID>(c, lay);
  if constexpr (std::is_same<S, Stream>::value && !GRID) {
    // the common spawn: the first word of a fresh SPAWN stream accepted and
    // the cell free; otherwise the loop below replays the stream from there
    if (spawn.idx == 0u && gb.rng != 0u) {
      const W4 w = ws;  // block 0 of spawn
      const uint32_t v = w.a & gb.mask;
      if (v <= gb.rng) {
        ground_cell<GRID>(c, v, lay, sx, sy, x, y);
        bool occ = other.d == nd && other.x == x && other.y == y;
        if (npc_depth) occ = occ || npc_on(c, npc, pack_xy(x, y));
        done = !occ;
        if (done) {  // the stream now stands after its first word
          spawn.w = w;
          spawn.idx = 1u;
        }
      }
    }
  }
  for (uint32_t t = 0; t < kWordCap && !done; ++t) {
    uint32_t v = 0;
    if (gb.rng != 0) {
      v = spawn.next(key) & gb.mask;
      if (v > gb.rng) continue;
    }
    ground_cell<GRID>(c, v, lay, sx, sy, x, y);
    bool occ = other.d == nd && other.x == x && other.y == y;
    if (npc_depth) occ = occ || npc_on(c, npc, pack_xy(x, y));
    done = !occ;
  }
  if (!done) err = true;
  self.d = nd; self.x = x; self.y = y; self.sx = sx; self.sy = sy; self.lay = lay;
  dl.descend += 1;
  ev.emit(ORX_EV_POSITION, self_iden, nd, (x & 0xFFFF) | (y << 16));  // updater.py:287-290
}

// ---------------------------------------------------------------------------
// Random bits of one tick
// ---------------------------------------------------------------------------
// A tick's CPython-random draws (getrandbits(k), k <= 32) come first from
// reservoir segments of ONE Philox block, the tick block (game, episode,
// tick, TICK), consumed least-significant bits first; a segment with fewer
// than k bits left is skipped, and once none is left a draw takes the top k
// bits of the next word of the purpose's own stream (SHUFFLE / POLICY, from
// word 0).  DESIGN.md §4, make_golden.TickBits.
//  * word a (32 bits): the updater's shuffles.  random.shuffle([p1, p2]) =
//    randbelow(2), k = 2: 16 two-bit fields, accepted iff the high bit is
//    clear; player 1 acts first iff the first accepted field == 1
//    (updater.py:114).  All 16 rejected: 2^-16.
//  * bits 0-29 of word b, then of word c: the bots.  RandomBot.move =
//    Move(1 + randbelow(5)), k = 3: ten three-bit fields per word, rejected
//    iff >= 5 (bit2 & (bit1 | bit0)); p1's draws then p2's.  Fewer than two
//    accepted in word b: ~1e-3; in both words: ~1e-7.
// One block per game-tick (per-purpose whole-word streams needed four).
__device__ __forceinline__ W4 tick_block(Key key, uint32_t game, uint32_t ep, int32_t tick) {
  return philox(game, ep, (uint32_t)tick, tag(PUR_TICK, 0), key);
}

// v_med3_i32: x clamped to [lo, hi]
__device__ __forceinline__ int32_t med3_i32(int32_t x, int32_t lo, int32_t hi) {
  int32_t r;
  asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(lo), "s"(hi));
  return r;
}
// x clamped to [1, hi] (the interior's lower bound as an inline constant)
__device__ __forceinline__ int32_t med3_1(int32_t x, int32_t hi) {
  int32_t r;
  asm("v_med3_i32 %0, %1, 1, %2" : "=v"(r) : "v"(x), "s"(hi));
  return r;
}

// v_ffbl_b32: index of the lowest set bit, 0xFFFFFFFF for 0 (an opaque asm
// so the compiler neither adds a zero guard nor reasons from ctz(0) being UB)
__device__ __forceinline__ uint32_t ffbl(uint32_t x) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// bit 0 of each accepted three-bit field among a word's low ten
__device__ __forceinline__ uint32_t accepted3(uint32_t w) {
  return ~((w >> 2) & (w | (w >> 1))) & 0x09249249u;
}

// RandomBot draws r0, r1 (`need` of them) from the tick block's bot segments.
__device__ __forceinline__ void moves_from_block(const W4& tb, int need, Key key, uint32_t game,
                                                 uint32_t ep, int32_t tick, int32_t& m0,
                                                 int32_t& m1, bool& err) {
  const uint32_t acc = accepted3(tb.b);
  const uint32_t acc2 = acc & (acc - 1u);
  // (| bit 31: a defined shift when the mask is empty; the value is then unused)
  m0 = (int32_t)((tb.b >> __builtin_ctz(acc | 0x80000000u)) & 7u) + 1;
  m1 = (int32_t)((tb.b >> __builtin_ctz(acc2 | 0x80000000u)) & 7u) + 1;
  const int got = acc == 0 ? 0 : acc2 == 0 ? 1 : 2;
  if (ORX_UNLIKELY(got < need)) {  // rare: word c's segment, then the POLICY stream's words
    int g = got;
    uint32_t ac = accepted3(tb.c);
    for (int j = 0; j < 2 && g < need && ac; ++j) {
      const int32_t v = (int32_t)((tb.c >> __builtin_ctz(ac)) & 7u) + 1;
      if (g == 0) m0 = v; else m1 = v;
      ++g;
      ac &= ac - 1u;
    }
    if (g < need) {
      Stream s;
      s.init(game, ep, (uint32_t)tick, tag(PUR_POLICY, 0), 0);
      for (uint32_t i = 0; i < kWordCap && g < need; ++i) {
        const uint32_t r = s.next(key) >> 29;
        if (r >= 5u) continue;
        if (g == 0) m0 = (int32_t)r + 1; else m1 = (int32_t)r + 1;
        ++g;
      }
      if (g < need) err = true;
    }
  }
}

__device__ __forceinline__ bool first_from_packed(uint32_t pk, Key key, uint32_t game, uint32_t ep,
                                                  int32_t tick, bool& err) {
  const uint32_t acc = ~(pk >> 1) & 0x55555555u;
  int res = acc ? (int)((pk >> __builtin_ctz(acc | 0x80000000u)) & 1u) : -1;
  if (ORX_UNLIKELY(res < 0)) {  // rare (2^-16): the SHUFFLE stream's words
    Stream s;
    s.init(game, ep, (uint32_t)tick, tag(PUR_SHUFFLE, 0), 0);
    for (uint32_t i = 0; i < kWordCap && res < 0; ++i) {
      const uint32_t r = s.next(key) >> 30;
      if (r < 2u) res = (int)r;
    }
    if (res < 0) { err = true; res = 0; }
  }
  return res == 1;
}

__device__ __forceinline__ bool p1_first_draw(Key key, uint32_t game, uint32_t ep, int32_t tick,
                                              bool& err) {
  return first_from_packed(tick_block(key, game, ep, tick).a, key, game, ep, tick, err);
}

// RandomBot / StaircaseBot moves for both players (policy codes ORX_POLICY_*)
// given the RandomBot draws r0 (first random player), r1 (second).
__device__ __forceinline__ void assign_moves(int32_t pol1, int32_t pol2, int32_t r0, int32_t r1,
                                             const Player& p1, const Player& p2, int32_t& a1,
                                             int32_t& a2) {
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int32_t pol = p == 0 ? pol1 : pol2;
    const Player& me = p == 0 ? p1 : p2;
    int32_t a = p == 0 ? a1 : a2;
    if (pol == ORX_POLICY_RANDOM) {
      a = (p == 1 && pol1 == ORX_POLICY_RANDOM) ? r1 : r0;
    } else if (pol == ORX_POLICY_STAIRCASE) {
      const int32_t dx = me.sx - me.x, dy = me.sy - me.y;
      const int32_t adx = dx < 0 ? -dx : dx, ady = dy < 0 ? -dy : dy;
      a = adx > ady ? (dx > 0 ? ORX_MOVE_RIGHT : ORX_MOVE_LEFT)
                    : (dy > 0 ? ORX_MOVE_DOWN : ORX_MOVE_UP);
    } else if (pol == ORX_POLICY_STAY) {
      a = ORX_MOVE_STAY;
    }
    if (p == 0) a1 = a; else a2 = a;
  }
}

// tb: this tick's block (its bot segments are ignored when no player is random).
__device__ __forceinline__ void policy_pair(Key key, uint32_t game, uint32_t ep, int32_t tick,
                                            int32_t pol1, int32_t pol2, const W4& tb,
                                            const Player& p1, const Player& p2, int32_t& a1,
                                            int32_t& a2) {
  const int need = (pol1 == ORX_POLICY_RANDOM) + (pol2 == ORX_POLICY_RANDOM);
  int32_t r0 = ORX_MOVE_STAY, r1 = ORX_MOVE_STAY;
  bool err = false;
  if (need) moves_from_block(tb, need, key, game, ep, tick, r0, r1, err);
  assign_moves(pol1, pol2, r0, r1, p1, p2, a1, a2);
}

// ---------------------------------------------------------------------------
// The tick
// ---------------------------------------------------------------------------
// NPC health, two stores with one interface (get: the int8 value sign-extended;
// put: its low byte).  NpcMem: the HBM rows (stride B), read only when a hit
// happens -- the step kernels, where other waves hide that load.  NpcHpRegs:
// one byte per slot in registers, loaded and stored once per launch -- the
// rollout, whose lone wave per SIMD would otherwise stall a full HBM round
// trip on every tick in which one of its 64 games hits an NPC.
struct NpcMem {
  uint16_t* pos;
  int8_t* hp;
  uint32_t B, i;
  __device__ __forceinline__ int get(int k) const { return hp[(size_t)k * B + i]; }
  __device__ __forceinline__ void put(int k, int v) const { hp[(size_t)k * B + i] = (int8_t)v; }
};

template <int NCAP>
struct NpcHpRegs {
  // slot k: byte k & 3 of h[k >> 2], i.e. byte k & 7 of the 64-bit pair
  // (h0, h1) or (h2, h3) by k >> 3 -- a runtime k through 64-bit shifts, no
  // switch (which lowers to a branch ladder)
  uint32_t h0, h1, h2, h3;
  __device__ __forceinline__ int get(int k) const {
    const uint64_t p = (NCAP <= 8 || (k >> 3) == 0) ? ((uint64_t)h0 | ((uint64_t)h1 << 32))
                                                    : ((uint64_t)h2 | ((uint64_t)h3 << 32));
    return (int)(int8_t)(p >> (8 * (k & 7)));
  }
  __device__ __forceinline__ void put(int k, int v) {
    const int sh = 8 * (k & 7);
    const uint64_t m = 0xFFull << sh, b = (uint64_t)((uint32_t)v & 0xFFu) << sh;
    uint64_t p = (uint64_t)h0 | ((uint64_t)h1 << 32);
    p = (k >> 3) == 0 ? ((p & ~m) | b) : p;
    h0 = (uint32_t)p; h1 = (uint32_t)(p >> 32);
    if constexpr (NCAP > 8) {
      p = (uint64_t)h2 | ((uint64_t)h3 << 32);
      p = (k >> 3) == 1 ? ((p & ~m) | b) : p;
      h2 = (uint32_t)p; h3 = (uint32_t)(p >> 32);
    }
  }
  __device__ __forceinline__ void fill(int v) {
    h0 = h1 = h2 = h3 = ((uint32_t)v & 0xFFu) * 0x01010101u;
  }
  // unconditional loads, as load_npcs (slots >= K hold a copy of slot K-1)
  __device__ __forceinline__ void load(const int8_t* hp, int K, uint32_t B, uint32_t i) {
    uint32_t v[NCAP];
#pragma unroll
    for (int k = 0; k < NCAP; ++k) v[k] = (uint8_t)hp[(size_t)min(k, K - 1) * B + i];
    h0 = h1 = h2 = h3 = 0;
#pragma unroll
    for (int k = 0; k < NCAP; ++k) h0 = k < 4 ? (h0 | v[k] << (8 * k)) : h0;
#pragma unroll
    for (int k = 4; k < NCAP; ++k) h1 = k < 8 ? (h1 | v[k] << (8 * (k - 4))) : h1;
#pragma unroll
    for (int k = 8; k < NCAP; ++k) h2 = k < 12 ? (h2 | v[k] << (8 * (k - 8))) : h2;
#pragma unroll
    for (int k = 12; k < NCAP; ++k) h3 = h3 | v[k] << (8 * (k - 12));
  }
  __device__ __forceinline__ void store(int8_t* hp, int K, uint32_t B, uint32_t i) const {
#pragma unroll
    for (int k = 0; k < NCAP; ++k)
      if (k < K) hp[(size_t)k * B + i] = (int8_t)get(k);
  }
};

// ---------------------------------------------------------------------------
// Character mechanics (ORX_EXT_MANA / HEAL / LEVELING / ITEMS; readme.md:44,
// 72, 74 -- no reference code, parameters in orx_cfg_t, include/orx.h)
// ---------------------------------------------------------------------------
// Items on the floor of the NPCs' depth.  The item NPC k dropped lies on its
// cell and inherits its slot register (a slot holds a live NPC, its item or
// nothing), so the one slot scan of a tick tests targets for both: `on` bit k
// = slot k holds an item, `kind` bit k: 1 = max health.
template <int NCAP>
struct Items {
  uint32_t on, kind;
  __device__ __forceinline__ void clear() { on = kind = 0; }
};

// A live NPC stands on `key` (NPC occupancy for moves and spawn cells): with
// items in the slots the slot must be a live NPC's.
template <int NCAP>
__device__ __forceinline__ bool npc_on(const Cfg& c, const Npcs<NCAP>& npc, uint32_t key) {
  return (c.ext & ORX_EXT_ITEMS) ? npc.live(key) : npc.any(key);
}

// Whole points from up to a third of the manabar, at most `cap` of them.
__device__ __forceinline__ int32_t mana_points(const Cfg& c, int32_t mana, int32_t cap) {
  const int32_t p = min(mana, c.mana_third) / c.mana_pp;
  return min(p, cap);
}

// handle_combat's damage for a player attacker (updater.py:313, 331):
// og_dmg = damage - armor; with ORX_EXT_MANA plus the mana spent on it.
__device__ __forceinline__ int32_t rpg_attack(const Cfg& c, Player& self) {
  int32_t d = self.dmg - c.player_armor;
  if (c.ext & ORX_EXT_MANA) {
    const int32_t pts = mana_points(c, self.mana, 0x7FFFFFFF);
    self.mana -= pts * c.mana_pp;
    d += pts;
  }
  return d > 0 ? d : 0;
}

// ORX_EXT_LEVELING: a kill's experience; crossing a level refills a living
// player's health and mana.
__device__ __forceinline__ void gain_xp(const Cfg& c, Player& p) {
  const int32_t before = p.xp / c.xp_level;
  p.xp += c.xp_kill;
  if (p.xp / c.xp_level > before && p.hp > 0) {
    p.hp = p.mhp;
    if (c.ext & ORX_EXT_MANA) p.mana = c.mana_max;
  }
}

// ORX_EXT_ITEMS: NPC k, swept at cell key `cell` in tick `tick`, may drop
// its item (one Philox block of purpose ITEM, block index = slot).
template <int NCAP>
__device__ __forceinline__ void drop_item(const Cfg& c, Key key, uint32_t game, uint32_t ep,
                                          int32_t tick, int k, uint32_t cell, Npcs<NCAP>& npc,
                                          Items<NCAP>& it) {
  const W4 w = philox(game, ep, (uint32_t)tick, tag(PUR_ITEM, 0) | (uint32_t)k, key);
  if ((int32_t)__umulhi(w.a, 100u) < c.drop_pct) {
    npc.set(k, cell);
    it.on |= 1u << k;
    it.kind = (it.kind & ~(1u << k)) | ((w.b & 1u) << k);
  }
}

// ORX_EXT_ITEMS: a player that stepped onto an item's cell takes it when it
// has a free item spot.
template <int NCAP>
__device__ __forceinline__ void pick_up(const Cfg& c, Player& self, Npcs<NCAP>& npc,
                                        Items<NCAP>& it) {
  const int k = npc.find(pack_xy(self.x, self.y));
  if (k >= 0 && ((it.on >> k) & 1u) && self.nitems < c.item_slots) {
    const bool health_item = (it.kind >> k) & 1u;
    it.on &= ~(1u << k);
    npc.kill(k);
    it.kind &= ~(1u << k);
    self.nitems += 1;
    if (health_item) {
      self.mhp += c.item_bonus;
      self.hp += c.item_bonus;
    } else {
      self.dmg += c.item_bonus;
    }
  }
}

// ORX_EXT_README_COMBAT (readme.md:69-70): the players' combat as one
// simultaneous resolution before the moves (include/orx.h has the table); an
// attacker becomes a Stay, damage is applied here; NPC combat is left to
// handle_move.  Called with player 1 then player 2 (event order).
__device__ __forceinline__ void make_stay(Player& p) {
  p.move = ORX_MOVE_STAY;
  p.tx = p.x;
  p.ty = p.y;
}

template <bool EV>
__device__ __forceinline__ void readme_combat(const Cfg& c, Player& a, Player& b, Deltas& dl,
                                              Events<EV>& ev) {
  const bool cda = a.cool > 0, cdb = b.cool > 0;  // this tick's cooldowns
  a.cool = max(a.cool - 1, 0);
  b.cool = max(b.cool - 1, 0);
  if (a.d != b.d) return;
  bool amov = a.move != ORX_MOVE_STAY, bmov = b.move != ORX_MOVE_STAY;
  // on cooldown an attack is measured as a Stay
  if (cda && amov && ((a.tx == b.x && a.ty == b.y) || (bmov && a.tx == b.tx && a.ty == b.ty))) {
    make_stay(a);
    amov = false;
  }
  if (cdb && bmov && ((b.tx == a.x && b.ty == a.y) || (amov && b.tx == a.tx && b.ty == a.ty))) {
    make_stay(b);
    bmov = false;
  }
  const bool a_cur = amov && a.tx == b.x && a.ty == b.y;
  const bool b_cur = bmov && b.tx == a.x && b.ty == a.y;
  const bool same = amov && bmov && a.tx == b.tx && a.ty == b.ty;
  if (a_cur && b_cur) {  // both attack the other's cell: half damage, cooldown
    const int32_t da = rpg_attack(c, a) / 2, db = rpg_attack(c, b) / 2;
    b.hp -= da;
    a.hp -= db;
    a.cool = b.cool = c.cooldown;
    make_stay(a);
    make_stay(b);
    dl.combat += 2;
    ev.emit(ORX_EV_COMBAT, 1, 2, ORX_FLAG_PARRY);
    ev.emit(ORX_EV_COMBAT, 2, 1, ORX_FLAG_PARRY);
    return;
  }
  if (same) {  // both into one cell: full damage
    const int32_t da = rpg_attack(c, a), db = rpg_attack(c, b);
    b.hp -= da;
    a.hp -= db;
    make_stay(a);
    make_stay(b);
    dl.combat += 2;
    ev.emit(ORX_EV_COMBAT, 1, 2, ORX_FLAG_AMBUSH);
    ev.emit(ORX_EV_COMBAT, 2, 1, ORX_FLAG_AMBUSH);
    return;
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) {  // one-sided: the attacker stays
    Player& t = s ? b : a;
    Player& v = s ? a : b;
    if (!(s ? b_cur : a_cur)) continue;
    const bool v_moves = v.move != ORX_MOVE_STAY, v_cd = s ? cda : cdb;
    if (!v_moves && v_cd) {
      v.hp -= rpg_attack(c, t);  // cannot defend: full damage
    } else if (!v_moves) {
      t.cool = max(t.cool, 1);   // negated; the attacker cannot attack or defend next tick
    }
    ev.emit(ORX_EV_COMBAT, s ? 2 : 1, s ? 1 : 2, v_moves ? ORX_FLAG_FLEE : ORX_FLAG_BLOCK);
    dl.combat += 1;
    make_stay(t);
  }
}

// handle_move for `self` (updater.py:180-243), branch-free except for the
// rare descend.  Returns true if the target cell holds an NPC (the slot is
// resolved in npc_hits); combat against the other player is applied here.
template <int NCAP, bool EV, bool GRID, class Src, class S>
__device__ __forceinline__ bool handle_move(const Cfg& c, Key key, Src& src, Player& self,
                                            Player& other, int32_t other_start,
                                            Npcs<NCAP>& npc, Items<NCAP>& items,
                                            S& spawn, Deltas& dl, bool& err, int32_t self_iden,
                                            bool self_first, Events<EV>& ev) {
  if ((c.ext & ORX_EXT_HEAL) && self.heal && self.hp > 0) {  // readme.md:74
    const int32_t pts = mana_points(c, self.mana, max(self.mhp - self.hp, 0));
    self.mana -= pts * c.mana_pp;
    self.hp += pts;
    if (pts > 0) ev.emit(ORX_EV_HEALTH, self_iden, pts, 0);
  }
  const bool moving = self.move != ORX_MOVE_STAY;
  const int32_t tx = self.tx, ty = self.ty;
  const bool occ_other = moving && other.d == self.d && other.x == tx && other.y == ty;
  // bitwise, not short-circuit: no branch around the slot scan
  const bool hit_npc = NCAP > 0 && (moving & !occ_other & (self.d == c.d1) &
                                    npc_on(c, npc, pack_xy(tx, ty)));
  const bool free = moving && !occ_other && !hit_npc;
  const bool stairs = free && stair_tile<GRID>(c, self, tx, ty);
  const bool step = free && !stairs;
  self.x = step ? tx : self.x;
  self.y = step ? ty : self.y;
  // Block / Parry / Ambush / Flee (updater.py:222-243): without a Modifier
  // subclass every flag deals og_dmg = attacker.damage - attacker.armor.
  dl.combat += (occ_other || hit_npc) ? 1 : 0;
  int32_t dmg = c.player_dmg_net > 0 ? c.player_dmg_net : 0;
  if (c.ext & ORX_EXT_RPG) dmg = (occ_other || hit_npc) ? rpg_attack(c, self) : 0;
  other.hp -= occ_other ? dmg : 0;
  self.hd = dmg;  // an NPC hit's damage, applied by npc_hits after both moves
  if (NCAP > 0 && (c.ext & ORX_EXT_ITEMS) && step && self.d == c.d1)
    pick_up(c, self, npc, items);
  if constexpr (EV) {
    if (occ_other) {
      int32_t ox, oy;
      calc_pos(other.x, other.y, other.move, ox, oy);
      const int32_t flag = other.move == ORX_MOVE_STAY        ? ORX_FLAG_BLOCK
                           : (ox == tx && oy == ty)            ? ORX_FLAG_PARRY
                           : !self_first                       ? ORX_FLAG_AMBUSH
                                                               : ORX_FLAG_FLEE;
      ev.emit(ORX_EV_COMBAT, self_iden, 3 - self_iden, flag);
    }
    if (hit_npc) ev.emit(ORX_EV_COMBAT, self_iden, 3 + npc.find(pack_xy(tx, ty)), ORX_FLAG_BLOCK);
    if (step) ev.emit(ORX_EV_POSITION, self_iden, self.d, (tx & 0xFFFF) | (ty << 16));
  }
  if (ORX_UNLIKELY(stairs))
    descend<NCAP, EV, GRID>(c, key, src, self, other, other_start, npc, spawn, dl, err,
                            self_iden, ev);
  return hit_npc;
}

// handle_combat on NPC defenders (hits of d0 then d1 damage, in the attackers'
// order), then the death sweep (updater.py:136-145): only NPCs hit this tick
// can reach health <= 0.  kill0 / kill1: attacker 0's / 1's hit took its NPC
// to health <= 0 (ORX_EXT_LEVELING's kill credit).
template <int NCAP, bool EV, class M>
__device__ __forceinline__ void npc_hits(const Cfg& c, Npcs<NCAP>& npc, M& m, int h0, int h1,
                                         int d0, int d1, Deltas& dl, Events<EV>& ev,
                                         bool& kill0, bool& kill1, uint32_t key0 = 0,
                                         uint32_t key1 = 0) {
  int v0 = m.get(h0 >= 0 ? h0 : h1), v1 = m.get(h1 >= 0 ? h1 : h0);
  if (h0 >= 0) v0 -= d0;
  const int v0a = v0;
  if (h1 >= 0) { v1 = (h1 == h0) ? v0 - d1 : v1 - d1; if (h1 == h0) v0 = v1; }
  kill0 = h0 >= 0 && v0a <= 0;
  kill1 = h1 >= 0 && v1 <= 0 && !(h1 == h0 && v0a <= 0);
  // the int8 rows keep health above -128 (a death is decided on the int)
  if (h0 >= 0) m.put(h0, max(v0, -128));
  if (h1 >= 0 && h1 != h0) m.put(h1, max(v1, -128));
  // the sweep walks GameState.entities backwards: higher slot first
  const bool swap = h1 > h0;
  const int ks[2] = {swap ? h1 : h0, swap ? h0 : h1};
  const int vs[2] = {swap ? v1 : v0, swap ? v0 : v1};
  const uint32_t cs[2] = {swap ? key1 : key0, swap ? key0 : key1};
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int k = ks[j];
    // dense NPCs: a hit slot is a live NPC's (the grid holds nothing else), so
    // only a second hit on the same NPC is not (no HBM re-read of the alive row)
    const bool live = NCAP == kDense ? !(j == 1 && ks[1] == ks[0]) : npc.is_alive(k);
    if (k >= 0 && vs[j] <= 0 && live) {
      npc.mark_dead(k);
      if constexpr (NCAP == kDense) npc.kill_at(cs[j]);  // the cell is known: no slot lookup
      else npc.kill(k);
      dl.npc_death += 1;
      ev.emit(ORX_EV_DEATH, 3 + k, 0, 0);
    }
  }
}

template <bool EV>
__device__ __forceinline__ void end_tick(const Cfg& c, Key key, uint32_t game, uint32_t ep,
                                         Player& p1, Player& p2, int32_t& tick, int32_t& status,
                                         bool err, Deltas& dl, Events<EV>& ev,
                                         int32_t& sep_start);

// One Updater.update for an in-progress game; p1.move/p2.move = raw moves.
template <int NCAP, bool EV, bool GRID, class Src, class M>
__device__ __forceinline__ void tick_game(const Cfg& c, Key key, Src& src, uint32_t game,
                                          uint32_t ep, bool p1_first, Player& p1, Player& p2,
                                          Npcs<NCAP>& npc, Items<NCAP>& items, M& m,
                                          int32_t& tick, int32_t& status, bool& err, Deltas& dl,
                                          Events<EV>& ev, int32_t& sep_start) {
  if (c.ext & ORX_EXT_HEAL) {  // a heal is a Stay that converts mana (readme.md:74)
    p1.heal = p1.move == ORX_MOVE_HEAL;
    p2.heal = p2.move == ORX_MOVE_HEAL;
    p1.move = p1.heal ? ORX_MOVE_STAY : p1.move;
    p2.move = p2.heal ? ORX_MOVE_STAY : p2.move;
  } else {
    p1.heal = p2.heal = 0;
  }
  calc_pos(p1.x, p1.y, p1.move, p1.tx, p1.ty);         // updater.py:89-98
  if (blocked<GRID>(c, p1.lay, p1.tx, p1.ty)) p1.move = ORX_MOVE_STAY;
  calc_pos(p2.x, p2.y, p2.move, p2.tx, p2.ty);
  if (blocked<GRID>(c, p2.lay, p2.tx, p2.ty)) p2.move = ORX_MOVE_STAY;
  if (c.ext & ORX_EXT_README_COMBAT) {  // the readme's combat table, before the moves
    if (p1.move == ORX_MOVE_STAY) make_stay(p1);
    if (p2.move == ORX_MOVE_STAY) make_stay(p2);
    readme_combat(c, p1, p2, dl, ev);
  }

  // p1_first: the player shuffle (updater.py:114).  The NPC shuffle (:127)
  // draws later words of the same per-tick stream and only orders Stay-ing
  // NPCs, so it is unobservable and skipped.
  auto&& spawn = src.spawn(tick);
  Player A = pick(p1_first, p1, p2);
  Player Bp = pick(p1_first, p2, p1);
  const int32_t a_start = p1_first ? c.d1 : c.d2;
  const int32_t b_start = p1_first ? c.d2 : c.d1;
  const int32_t a_iden = p1_first ? 1 : 2;
  const bool hA = handle_move<NCAP, EV, GRID>(c, key, src, A, Bp, b_start, npc, items, spawn,
                                              dl, err, a_iden, true, ev);
  const bool hB = handle_move<NCAP, EV, GRID>(c, key, src, Bp, A, a_start, npc, items, spawn,
                                              dl, err, 3 - a_iden, false, ev);
  if (NCAP > 0 && ORX_UNLIKELY(hA || hB)) {
    // NPCs never move and are swept only after both moves: the slots found at
    // the targets now are the ones that were attacked.
    const int h0 = hA ? npc.find(pack_xy(A.tx, A.ty)) : -1;
    const int h1 = hB ? npc.find(pack_xy(Bp.tx, Bp.ty)) : -1;
    bool kA = false, kB = false;
    npc_hits(c, npc, m, h0, h1, A.hd, Bp.hd, dl, ev, kA, kB, pack_xy(A.tx, A.ty),
             pack_xy(Bp.tx, Bp.ty));
    if (c.ext & (ORX_EXT_LEVELING | ORX_EXT_ITEMS)) {  // readme.md:44
      if ((c.ext & ORX_EXT_LEVELING) && kA) gain_xp(c, A);
      if ((c.ext & ORX_EXT_LEVELING) && kB) gain_xp(c, Bp);
      if ((c.ext & ORX_EXT_ITEMS) && kA)
        drop_item(c, key, game, ep, tick, h0, pack_xy(A.tx, A.ty), npc, items);
      if ((c.ext & ORX_EXT_ITEMS) && kB)
        drop_item(c, key, game, ep, tick, h1, pack_xy(Bp.tx, Bp.ty), npc, items);
    }
  }
  p1 = pick(p1_first, A, Bp);
  p2 = pick(p1_first, Bp, A);
  if (c.ext & ORX_EXT_MANA) {  // the end of the tick: mana regeneration
    p1.mana = min(p1.mana + c.mana_regen, c.mana_max);
    p2.mana = min(p2.mana + c.mana_regen, c.mana_max);
  }

  end_tick<EV>(c, key, game, ep, p1, p2, tick, status, err, dl, ev, sep_start);
}

// The end of Updater.update after the death sweep: the build extensions'
// separation damage and random double-death winner (readme.md:46-48), tick++
// and the result (updater.py:148-162).
template <bool EV>
__device__ __forceinline__ void end_tick(const Cfg& c, Key key, uint32_t game, uint32_t ep,
                                         Player& p1, Player& p2, int32_t& tick, int32_t& status,
                                         bool err, Deltas& dl, Events<EV>& ev,
                                         int32_t& sep_start) {
  if (c.ext & ORX_EXT_SEPARATION_DAMAGE) {  // build extension (readme.md:46-47)
    if (p1.d != p2.d) {
      if (sep_start < 0) sep_start = tick;
      const int32_t k = tick - sep_start + 1;
      const int32_t dmg = (k + c.sep_period - 1) / c.sep_period;
      const bool p1_behind = p1.d < p2.d;
      if (p1_behind) p1.hp -= dmg; else p2.hp -= dmg;
      ev.emit(ORX_EV_HEALTH, p1_behind ? 1 : 2, -dmg, 0);
    } else {
      sep_start = -1;
    }
  }
  bool p2_wins_draw = false;
  if ((c.ext & ORX_EXT_RANDOM_DOUBLE_DEATH) && p1.hp <= 0 && p2.hp <= 0) {  // readme.md:47-48
    Stream r;
    r.init(game, ep, (uint32_t)tick, tag(PUR_RESOLVE, 0));
    p2_wins_draw = (r.next(key) >> 31) != 0;
  }

  tick += 1;                                           // updater.py:148-162
  // as selects, lowest precedence first (a divergent if-chain here costs the
  // lone wave taken branches every tick)
  const bool dead1 = p1.hp <= 0, dead2 = p2.hp <= 0;
  const int32_t both = !(c.ext & ORX_EXT_RANDOM_DOUBLE_DEATH) ? ORX_TIE
                       : p2_wins_draw                         ? ORX_PLAYER2_WIN
                                                              : ORX_PLAYER1_WIN;
  int32_t s = (c.max_ticks && tick >= c.max_ticks) ? ORX_TIE : ORX_IN_PROGRESS;
  s = dead2 ? ORX_PLAYER1_WIN : s;
  s = dead1 ? (dead2 ? both : ORX_PLAYER2_WIN) : s;
  s = err ? ORX_STATUS_RNG_EXHAUSTED : s;
  status = s;
  dl.ret += (s == ORX_PLAYER1_WIN ? 1 : 0) - (s == ORX_PLAYER2_WIN ? 1 : 0);
  dl.eps += (uint32_t)(s - ORX_PLAYER1_WIN) <= (uint32_t)(ORX_TIE - ORX_PLAYER1_WIN) ? 1 : 0;
}

// ---------------------------------------------------------------------------
// Moving NPCs (cfg.npc_policy != ORX_NPC_STAY): the reference's enemy-AI hook
// Updater.decide_npc_move (updater.py:165-178) and its literal resolution of
// every NPC move -- decisions for all NPCs before any move (:116-126), the
// NPC shuffle (:127), handle_move for the players then the NPCs in that order
// (:133-134, 180-243; NPC-vs-player and NPC-vs-NPC Block / Ambush / Flee, an
// NPC stepping onto a staircase dies, :263-270), the death sweep (:136-145).
// One lane per game, the literal sequence (the generic form of every entry
// point; include/orx.h ORX_NPC_* has the policies).
// ---------------------------------------------------------------------------
// getrandbits(k) of the tick's CPython-random draws in keyed mode: the low k
// bits of a reservoir segment (LSB first; a segment with fewer than k left is
// skipped for good), then the top k bits of the next word of stream `s`;
// with `refill` every word of `s` is a 30-bit segment of its own (the NPC
// stream, purpose NPC, c2 = tick).  make_golden.TickBits / NpcBits.
// The stream's first NB 4-word blocks are drawn up front, in the tick's
// uniform control flow: its consumers run in per-lane loops (the AI's
// rejection draws, the Fisher-Yates shuffle), where a Philox call inside the
// loop body costs the whole wave whenever any one lane crosses a block
// boundary.  Words past them come from the lazy Stream at block NB.
template <int NB>
struct AheadStream {
  static_assert(NB == 1 || NB == 2, "one or two blocks ahead");
  Stream s;
  W4 w0, w1;
  uint32_t i;
  __device__ __forceinline__ void init(uint32_t game, uint32_t ep, uint32_t cc2, uint32_t t,
                                       Key key) {
    s.init(game, ep, cc2, t, 4u * NB);
    w0 = philox(game, ep, cc2, t, key);
    if constexpr (NB > 1) w1 = philox(game, ep, cc2, t | 1u, key);
    i = 0;
  }
  __device__ __forceinline__ uint32_t next(Key key) {
    if (i < 4u * NB) {
      const uint32_t j = i & 3u;
      const W4 v = (NB > 1 && i >= 4u) ? w1 : w0;
      ++i;
      return j == 0 ? v.a : j == 1 ? v.b : j == 2 ? v.c : v.d;
    }
    return s.next(key);
  }
};

template <class S>
struct PyBits {
  uint32_t res;
  int32_t nb;
  bool refill;
  S s;
  __device__ __forceinline__ uint32_t bits(int k, Key key) {
    if (nb < k) {
      if (refill) {
        res = s.next(key) & 0x3FFFFFFFu;
        nb = 30;
      } else {
        nb = 0;
      }
    }
    if (nb >= k) {
      const uint32_t r = res & ((1u << k) - 1u);
      res >>= k;
      nb -= k;
      return r;
    }
    return s.next(key) >> (32 - k);
  }
};
// stock-seed mode: the game's CPython random (getrandbits(k) = word >> (32 - k))
struct MtBits {
  MtStream* py;
  __device__ __forceinline__ uint32_t bits(int k, Key key) { return py->next(key) >> (32 - k); }
};
// Random._randbelow_with_getrandbits(n) over a bit source (random.py)
template <class Bits>
__device__ __forceinline__ uint32_t randbelow_bits(Bits& b, Key key, uint32_t n, bool& err) {
  const int k = 32 - __clz(n);
  for (uint32_t t = 0; t < kWordCap; ++t) {
    const uint32_t r = b.bits(k, key);
    if (r < n) return r;
  }
  err = true;
  return 0;
}

// Keyed mode's AI draws of a tick, branch-free: random.choice(list(Move))
// for n NPCs is randbelow(5) n times over the NPC stream's 30-bit segments,
// i.e. NPC j's value is the j-th accepted 3-bit field (value < 5) of the
// field sequence (10 per word, LSB first; kWordCap rejections in a row give
// up with 0 and err, as randbelow_bits).  A word's ten fields are scanned
// unrolled, and the lanes loop over words, not over draws.  Returns the
// values packed 3 bits apiece.
template <class D>
__device__ __forceinline__ D ai_choices(PyBits<AheadStream<1>>& ai, Key key, int n, bool& err) {
  D draws = 0;
  int cnt = 0;
  uint32_t rej = 0;
#pragma unroll 1
  while (cnt < n) {
    const uint32_t seg = ai.s.next(key) & 0x3FFFFFFFu;
#pragma unroll
    for (int f = 0; f < 10; ++f) {
      const uint32_t v = (seg >> (3 * f)) & 7u;
      const bool active = cnt < n, acc = v < 5u;
      const uint32_t rj = acc ? 0u : rej + 1u;
      const bool give = !acc && rj >= kWordCap;
      const bool take = active && (acc || give);
      draws |= take ? (D)(acc ? v : 0u) << (3 * cnt) : (D)0;
      err |= active && give;
      rej = take ? 0u : (active ? rj : rej);
      cnt += take ? 1 : 0;
    }
  }
  return draws;
}

// ai_choices for at most 8 NPCs from the first three words alone, without a
// loop: each segment's ten acceptance bits by bit slicing (a field v = b2 b1
// b0 is rejected iff b2 & (b1 | b0)), then NPC j's value is the field at the
// lowest acceptance bit left.  Returns false (nothing consumed: ai_choices
// then runs from word 0) when the 30 fields hold fewer than n accepted ones
// (p ~ 1e-5 per game-tick at n = 8).
__device__ __forceinline__ bool ai_choices8(const PyBits<AheadStream<1>>& ai, int n,
                                            uint32_t& draws) {
  constexpr uint32_t M = 0x09249249u;  // bit 3f of each of the ten fields
  const uint32_t s0 = ai.s.w0.a & 0x3FFFFFFFu, s1 = ai.s.w0.b & 0x3FFFFFFFu,
                 s2 = ai.s.w0.c & 0x3FFFFFFFu;
  auto acc = [](uint32_t sg) {
    const uint32_t b0 = sg & M, b1 = (sg >> 1) & M, b2 = (sg >> 2) & M;
    return ~(b2 & (b1 | b0)) & M;
  };
  uint32_t m0 = acc(s0), m1 = acc(s1), m2 = acc(s2);
  if (__popc(m0) + __popc(m1) + __popc(m2) < n) return false;
  uint32_t d = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bool h0 = m0 != 0u, h1 = m1 != 0u;
    const uint32_t mm = h0 ? m0 : h1 ? m1 : m2;
    const uint32_t ss = h0 ? s0 : h1 ? s1 : s2;
    const uint32_t v = (ss >> __builtin_ctz(mm | 0x80000000u)) & 7u;
    const bool take = j < n;
    d |= take ? v << (3 * j) : 0u;
    m0 = (take && h0) ? (m0 & (m0 - 1u)) : m0;
    m1 = (take && !h0 && h1) ? (m1 & (m1 - 1u)) : m1;
    m2 = (take && !h0 && !h1) ? (m2 & (m2 - 1u)) : m2;
  }
  draws = d;
  return true;
}

// Keyed mode's Fisher-Yates draws of random.shuffle over n entries:
// randbelow(i + 1) for i = n-1 .. 1 from the shuffle source (the tick
// block's reservoir, then one word per draw), one draw per trip of a single
// per-lane loop, branch-free but for the rare word past the two blocks drawn
// ahead.  Returns draw j of position i at bits 4 i.
template <class J>
__device__ __forceinline__ J shuffle_draws(PyBits<AheadStream<2>>& sh, Key key, int n, bool& err) {
  J js = 0;
  int i = n - 1;
  uint32_t rej = 0, res = sh.res, wi = sh.s.i;
  int32_t nb = sh.nb;
  // the words drawn ahead as a queue: q0 is word wi; a trip that takes a
  // word shifts it (eight selects, no branch)
  uint32_t q0 = sh.s.w0.a, q1 = sh.s.w0.b, q2 = sh.s.w0.c, q3 = sh.s.w0.d;
  uint32_t q4 = sh.s.w1.a, q5 = sh.s.w1.b, q6 = sh.s.w1.c, q7 = sh.s.w1.d;
  for (uint32_t k = 0; k < wi; ++k) {  // (words the initiative draw took: none in practice)
    q0 = q1; q1 = q2; q2 = q3; q3 = q4; q4 = q5; q5 = q6; q6 = q7;
  }
#pragma unroll 1
  while (i >= 1) {
    const uint32_t bound = (uint32_t)i + 1u;
    const int kb = 32 - __clz(bound);
    const bool take_res = nb >= kb;
    uint32_t w = q0;
    if (!take_res && wi >= 8u) w = sh.s.s.next(key);  // past the blocks drawn ahead (rare)
    const uint32_t r = take_res ? (res & ((1u << kb) - 1u)) : (w >> (32 - kb));
    res = take_res ? (res >> kb) : res;
    nb = take_res ? nb - kb : 0;
    wi += take_res ? 0u : 1u;
    q0 = take_res ? q0 : q1; q1 = take_res ? q1 : q2; q2 = take_res ? q2 : q3;
    q3 = take_res ? q3 : q4; q4 = take_res ? q4 : q5; q5 = take_res ? q5 : q6;
    q6 = take_res ? q6 : q7;
    const bool acc = r < bound;
    const uint32_t rj = acc ? 0u : rej + 1u;
    const bool give = !acc && rj >= kWordCap;
    const bool step = acc || give;
    err |= give;
    js |= step ? (J)(acc ? r : 0u) << (4 * i) : (J)0;
    rej = step ? 0u : rj;
    i -= step ? 1 : 0;
  }
  return js;
}

// The tick's NPC updents (updater.py:116-128): each NPC's decided move (by
// slot), the shuffled order (position j -> slot) and which have acted.
// Register NPCs: packed in 64-bit registers (4-bit slots, 3-bit moves, runtime
// indices through shifts); dense NPCs: per-lane arrays.
template <int NCAP>
struct NpcTurns {
  uint64_t ord, mv;
  uint32_t acted;
  __device__ __forceinline__ void clear() { ord = mv = 0ull; acted = 0u; }
  __device__ __forceinline__ int slot(int j) const { return (int)((ord >> (4 * j)) & 15ull); }
  __device__ __forceinline__ void set_slot(int j, int k) {
    ord = (ord & ~(15ull << (4 * j))) | ((uint64_t)k << (4 * j));
  }
  __device__ __forceinline__ int32_t move(int k) const { return (int32_t)((mv >> (3 * k)) & 7ull); }
  __device__ __forceinline__ void set_move(int k, int32_t m) {
    mv = (mv & ~(7ull << (3 * k))) | ((uint64_t)m << (3 * k));
  }
  __device__ __forceinline__ bool has_acted(int k) const { return (acted >> k) & 1u; }
  __device__ __forceinline__ void mark(int k) { acted |= 1u << k; }
};
template <>
struct NpcTurns<kDense> {
  uint8_t ord_[ORX_MAX_NPCS], mv_[ORX_MAX_NPCS];
  uint32_t acted_[(ORX_MAX_NPCS + 31) / 32];
  __device__ __forceinline__ void clear() {
    for (int r = 0; r < (ORX_MAX_NPCS + 31) / 32; ++r) acted_[r] = 0u;
  }
  __device__ __forceinline__ int slot(int j) const { return ord_[j]; }
  __device__ __forceinline__ void set_slot(int j, int k) { ord_[j] = (uint8_t)k; }
  __device__ __forceinline__ int32_t move(int k) const { return mv_[k]; }
  __device__ __forceinline__ void set_move(int k, int32_t m) { mv_[k] = (uint8_t)m; }
  __device__ __forceinline__ bool has_acted(int k) const { return (acted_[k >> 5] >> (k & 31)) & 1u; }
  __device__ __forceinline__ void mark(int k) { acted_[k >> 5] |= 1u << (k & 31); }
};

// Register NPCs (moves decided): true iff no mover's target is a live NPC's
// cell or another mover's target -- then the NPCs' handle_move calls commute
// (updater.py:133-134: a move to a free cell, a hit on a player, or a
// staircase death), whatever order the shuffle gives.  Dead slots hold
// 0xFFFF, which no interior target equals.
template <int NCAP>
__device__ __forceinline__ bool npc_moves_commute(const Cfg& c, const Npcs<NCAP>& npc,
                                                  const NpcTurns<NCAP>& turns) {
  uint32_t t[NCAP > 0 ? NCAP : 1];
  bool clash = false;
#pragma unroll
  for (int k = 0; k < NCAP; ++k) {
    const int32_t mv = turns.move(k);
    const bool mover = k < c.K && npc.is_alive(k) && mv != ORX_MOVE_STAY;
    const uint32_t cell = npc.get(k);
    int32_t tx, ty;
    calc_pos((int32_t)(cell & 0xFFu), (int32_t)(cell >> 8), mv, tx, ty);
    const uint32_t tk = pack_xy(tx, ty);
    t[k] = mover ? tk : 0x10000u + (uint32_t)k;  // (distinct non-cells for the others)
    clash = clash || (mover && npc.any(tk));
  }
#pragma unroll
  for (int k = 1; k < NCAP; ++k)
#pragma unroll
    for (int j = 0; j < k; ++j) clash = clash || t[j] == t[k];
  return !clash;
}

// The dungeon of the NPCs' depth nd (player 1's start depth) at the start of
// the tick: a player's, when one stands on nd; else, under Unreachable with
// player 2 still above nd (player 1 started on nd and has left it), its
// generation-0 staircase from its key (stock-seed mode: player 1's dstore
// ring); absent otherwise -- despawned (updater.py:245-257).
struct NpcDepth {
  bool present;
  int32_t sx, sy, lay;
};

template <bool GRID, class Src>
__device__ __forceinline__ NpcDepth npc_depth(const Cfg& c, Key key, Src& src, uint32_t game,
                                              uint32_t ep, const Player& p1, const Player& p2,
                                              bool& err) {
  NpcDepth d{false, -1, -1, -1};
  const int32_t nd = c.d1;
  if (p1.d == nd) {
    d = NpcDepth{true, p1.sx, p1.sy, p1.lay};
  } else if (p2.d == nd) {
    d = NpcDepth{true, p2.sx, p2.sy, p2.lay};
  } else if (c.despawn == ORX_DESPAWN_UNREACHABLE && p2.d < nd) {
    d.present = true;
    if constexpr (Src::kMt) {
      if (!src.recall(1, c.d1, nd, d.sx, d.sy, d.lay)) err = true;
    } else {
      dungeon_stair<GRID>(c, key, game, ep, nd, 0u, d.sx, d.sy, d.lay, err);
    }
  }
  return d;
}

// dung.tiles[x, y] == StaircaseDown on the NPCs' depth (x, y in the grid)
template <bool GRID>
__device__ __forceinline__ bool npc_stair(const Cfg& c, const NpcDepth& d, int32_t x, int32_t y) {
  if constexpr (GRID) return bank_tile(c, d.lay, x, y) == ORX_TILE_STAIRCASE_DOWN;
  else return x == d.sx && y == d.sy;
}

// A player stands next to a staircase tile of the NPCs' depth: its NPCs stay
// (the AI's guard, include/orx.h ORX_NPC_*)
template <bool GRID>
__device__ __forceinline__ bool next_to_stairs(const Cfg& c, const NpcDepth& d, const Player& p) {
  if constexpr (GRID) {
    bool any = false;
#pragma unroll
    for (int m = ORX_MOVE_UP; m <= ORX_MOVE_LEFT; ++m) {
      int32_t x, y;
      calc_pos(p.x, p.y, m, x, y);
      any = any || (x >= 0 && x < c.W && y >= 0 && y < c.H && npc_stair<true>(c, d, x, y));
    }
    return any;
  } else {
    return abs(p.x - d.sx) + abs(p.y - d.sy) == 1;
  }
}

// The AI's move m for the NPC on cell key `nk`, or Stay where it is blocked
template <bool GRID>
__device__ __forceinline__ int32_t npc_step_or_stay(const Cfg& c, const NpcDepth& d, uint32_t nk,
                                                    int32_t m) {
  int32_t tx, ty;
  calc_pos((int32_t)(nk & 0xFFu), (int32_t)(nk >> 8), m, tx, ty);
  return blocked<GRID>(c, d.lay, tx, ty) ? ORX_MOVE_STAY : m;
}

// decide_npc_move (updater.py:165-178) for the NPC on cell key `nk`
template <bool GRID, class Bits>
__device__ __forceinline__ int32_t decide_npc_move(const Cfg& c, Key key, const NpcDepth& d,
                                                   bool freeze, const Player& p1,
                                                   const Player& p2, uint32_t nk, Bits& ai,
                                                   bool& err) {
  if (!d.present || freeze) return ORX_MOVE_STAY;
  const int32_t x = (int32_t)(nk & 0xFFu), y = (int32_t)(nk >> 8);
  int32_t m;
  if (c.npc_pol == ORX_NPC_RANDOM) {
    m = 1 + (int32_t)randbelow_bits(ai, key, 5u, err);   // random.choice(list(Move))
  } else {                                               // ORX_NPC_CHASE
    const bool h1 = p1.d == c.d1, h2 = p2.d == c.d1;
    if (!h1 && !h2) return ORX_MOVE_STAY;
    const int32_t d1 = abs(p1.x - x) + abs(p1.y - y), d2 = abs(p2.x - x) + abs(p2.y - y);
    const bool to2 = h2 && (!h1 || d2 < d1);
    const int32_t dx = (to2 ? p2.x : p1.x) - x, dy = (to2 ? p2.y : p1.y) - y;
    m = abs(dx) > abs(dy) ? (dx > 0 ? ORX_MOVE_RIGHT : ORX_MOVE_LEFT)
                          : (dy > 0 ? ORX_MOVE_DOWN : ORX_MOVE_UP);
  }
  return npc_step_or_stay<GRID>(c, d, nk, m);
}

// The flag of a move into an occupied cell (updater.py:222-243): the
// occupant (now on the target) Stays -> Block; its own target is the cell ->
// Parry (dead code: an occupant on the cell never targets it); it acted
// before the mover -> Ambush; else Flee.
__device__ __forceinline__ int32_t occupant_flag(int32_t tx, int32_t ty, int32_t occ_move,
                                                 bool occ_acted) {
  int32_t ox, oy;
  calc_pos(tx, ty, occ_move, ox, oy);
  return occ_move == ORX_MOVE_STAY ? ORX_FLAG_BLOCK
         : (ox == tx && oy == ty)  ? ORX_FLAG_PARRY
         : occ_acted               ? ORX_FLAG_AMBUSH
                                   : ORX_FLAG_FLEE;
}

// handle_move for a player in the moving-NPC tick (its occupancy test sees
// the NPCs where they stand now; a hit NPC's flag follows its decided move)
template <int NCAP, bool EV, bool GRID, class Src, class S, class M>
__device__ __forceinline__ void mov_player(const Cfg& c, Key key, Src& src, Player& self,
                                           Player& other, int32_t other_start, bool self_first,
                                           int32_t self_iden, Npcs<NCAP>& npc,
                                           const NpcTurns<NCAP>& turns, M& m, S& spawn,
                                           Deltas& dl, bool& err, Events<EV>& ev) {
  if (self.move == ORX_MOVE_STAY) return;
  const int32_t tx = self.tx, ty = self.ty;
  const int32_t dmg = c.player_dmg_net;
  if (other.d == self.d && other.x == tx && other.y == ty) {
    const int32_t flag = occupant_flag(tx, ty, other.move, !self_first);
    if (dmg > 0) other.hp -= dmg;
    dl.combat += 1;
    ev.emit(ORX_EV_COMBAT, self_iden, 3 - self_iden, flag);
    return;
  }
  const int q = (NCAP > 0 && self.d == c.d1) ? npc.find(pack_xy(tx, ty)) : -1;
  if (q >= 0) {
    const int32_t flag = occupant_flag(tx, ty, turns.move(q), turns.has_acted(q));
    if (dmg > 0) m.put(q, max(m.get(q) - dmg, -128));
    dl.combat += 1;
    ev.emit(ORX_EV_COMBAT, self_iden, 3 + q, flag);
    return;
  }
  if (stair_tile<GRID>(c, self, tx, ty)) {
    descend<NCAP, EV, GRID>(c, key, src, self, other, other_start, npc, spawn, dl, err, self_iden,
                            ev);
    return;
  }
  self.x = tx;
  self.y = ty;
  ev.emit(ORX_EV_POSITION, self_iden, self.d, (tx & 0xFFFF) | (ty << 16));
}

// handle_move for NPC slot k (its decided move mv != Stay) on the NPCs' depth
template <int NCAP, bool EV, bool GRID, class M>
__device__ __forceinline__ void mov_npc(const Cfg& c, int k, int32_t mv, Player& p1, Player& p2,
                                        Npcs<NCAP>& npc, const NpcTurns<NCAP>& turns,
                                        const NpcDepth& d, M& m, Deltas& dl, Events<EV>& ev) {
  const uint32_t k0 = npc.get_rt(k);
  int32_t tx, ty;
  calc_pos((int32_t)(k0 & 0xFFu), (int32_t)(k0 >> 8), mv, tx, ty);
  const uint32_t tk = pack_xy(tx, ty);
  const int32_t nd = c.d1, dmg = c.npc_dmg_net;
  const bool on1 = p1.d == nd && p1.x == tx && p1.y == ty;
  const bool on2 = p2.d == nd && p2.x == tx && p2.y == ty;
  if (on1 || on2) {  // the players acted first: Block or Ambush
    const int32_t flag = occupant_flag(tx, ty, on1 ? p1.move : p2.move, true);
    if (dmg > 0) {
      if (on1) p1.hp -= dmg;
      else p2.hp -= dmg;
    }
    dl.combat += 1;
    ev.emit(ORX_EV_COMBAT, 3 + k, on1 ? 1 : 2, flag);
    return;
  }
  const int q = npc.find(tk);
  if (q >= 0) {
    const int32_t flag = occupant_flag(tx, ty, turns.move(q), turns.has_acted(q));
    if (dmg > 0) m.put(q, max(m.get(q) - dmg, -128));
    dl.combat += 1;
    ev.emit(ORX_EV_COMBAT, 3 + k, 3 + q, flag);
    return;
  }
  if (npc_stair<GRID>(c, d, tx, ty)) {  // handle_descend: an NPC dies (updater.py:263-270)
    ev.emit(ORX_EV_DEATH, 3 + k, 0, 0);
    npc.mark_dead(k);
    npc.kill(k);
    dl.npc_death += 1;
    return;
  }
  if constexpr (NCAP == kDense) npc.kill_at(k0);  // (the old cell of the occupancy grid)
  npc.set_rt(k, tk);
  ev.emit(ORX_EV_POSITION, 3 + k, nd, (tx & 0xFFFF) | (ty << 16));
}

// mov_npc where the tick's NPC moves commute (npc_moves_commute): the
// target holds no NPC, so the move is a hit on a player (Block or Ambush:
// the players acted first), a staircase death or a free step; no event list
template <int NCAP, bool GRID>
__device__ __forceinline__ void mov_npc_free(const Cfg& c, int k, int32_t mv, Player& p1,
                                             Player& p2, Npcs<NCAP>& npc, const NpcDepth& d,
                                             Deltas& dl) {
  const uint32_t k0 = npc.get(k);
  int32_t tx, ty;
  calc_pos((int32_t)(k0 & 0xFFu), (int32_t)(k0 >> 8), mv, tx, ty);
  const int32_t nd = c.d1, dmg = c.npc_dmg_net;
  const bool on1 = p1.d == nd && p1.x == tx && p1.y == ty;
  const bool on2 = p2.d == nd && p2.x == tx && p2.y == ty;
  if (on1 || on2) {
    if (dmg > 0) {
      if (on1) p1.hp -= dmg;
      else p2.hp -= dmg;
    }
    dl.combat += 1;
  } else if (npc_stair<GRID>(c, d, tx, ty)) {  // handle_descend: the NPC dies
    npc.mark_dead(k);
    npc.kill(k);
    dl.npc_death += 1;
  } else {
    npc.set(k, pack_xy(tx, ty));
  }
}

// The death sweep over every NPC (updater.py:136-145: GameState.entities
// backwards, i.e. descending slots), any of which may have been hit
template <int NCAP, bool EV, class M>
__device__ __forceinline__ void npc_sweep(const Cfg& c, Npcs<NCAP>& npc, M& m, Deltas& dl,
                                          Events<EV>& ev) {
  if constexpr (NCAP == kDense) {
    for (int r = (c.K - 1) >> 5; r >= 0; --r) {
      uint32_t a = npc.rows[(size_t)r * npc.B];
      while (a) {
        const int j = 31 - __clz(a);
        a &= ~(1u << j);
        const int k = 32 * r + j;
        if (m.get(k) <= 0) {
          ev.emit(ORX_EV_DEATH, 3 + k, 0, 0);
          npc.mark_dead(k);
          npc.kill(k);
          dl.npc_death += 1;
        }
      }
    }
  } else if constexpr (NCAP > 0) {
#pragma unroll
    for (int k = NCAP - 1; k >= 0; --k) {
      if (k < c.K && npc.is_alive(k) && m.get(k) <= 0) {
        ev.emit(ORX_EV_DEATH, 3 + k, 0, 0);
        npc.mark_dead(k);
        npc.kill(k);
        dl.npc_death += 1;
      }
    }
  }
}

template <int NCAP, bool EV, bool GRID, class Src, class M, class BitsS, class BitsA>
__device__ __forceinline__ void tick_moving_body(const Cfg& c, Key key, Src& src, uint32_t game,
                                                 uint32_t ep, Player& p1, Player& p2,
                                                 Npcs<NCAP>& npc, M& m, int32_t& tick,
                                                 int32_t& status, bool& err, Deltas& dl,
                                                 Events<EV>& ev, int32_t& sep_start, BitsS& sh,
                                                 BitsA& ai) {
  ORX_MCYC_BEGIN(cy0);
  p1.heal = p2.heal = 0;
  calc_pos(p1.x, p1.y, p1.move, p1.tx, p1.ty);          // updater.py:89-98
  if (blocked<GRID>(c, p1.lay, p1.tx, p1.ty)) p1.move = ORX_MOVE_STAY;
  calc_pos(p2.x, p2.y, p2.move, p2.tx, p2.ty);
  if (blocked<GRID>(c, p2.lay, p2.tx, p2.ty)) p2.move = ORX_MOVE_STAY;
  const bool p1_first = randbelow_bits(sh, key, 2u, err) == 1u;   // :114
  NpcTurns<NCAP> turns;
  turns.clear();
  int n = 0;
  bool order_free = false;  // this game's NPC moves commute (keyed mode, no event list)
  NpcDepth d{false, -1, -1, -1};
  if constexpr (NCAP > 0) {
    d = npc_depth<GRID>(c, key, src, game, ep, p1, p2, err);
    const bool freeze = d.present && ((p1.d == c.d1 && next_to_stairs<GRID>(c, d, p1)) ||
                                      (p2.d == c.d1 && next_to_stairs<GRID>(c, d, p2)));
    ORX_MCYC_END(0, cy0);
    ORX_MCYC_BEGIN(cy1);
    // decide_npc_move for every NPC in GameState.entities order (:116-126)
    if constexpr (NCAP == kDense) {
      for (int r = 0; r < (c.K + 31) >> 5; ++r) {
        uint32_t a = npc.rows[(size_t)r * npc.B];
        while (a) {
          const int k = 32 * r + (int)__builtin_ctz(a);
          a &= a - 1u;
          turns.set_move(k, decide_npc_move<GRID>(c, key, d, freeze, p1, p2, npc.get(k), ai, err));
          turns.set_slot(n++, k);
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < NCAP; ++k)
        if (k < c.K && npc.is_alive(k)) turns.set_slot(n++, k);
      if (c.npc_pol == ORX_NPC_RANDOM && d.present && !freeze) {
        // random.choice(list(Move)) per NPC as ONE per-lane loop over all the
        // NPCs' rejection draws (randbelow_bits unrolled by hand: same draws,
        // same give-up rule), so a wave iterates the max over its lanes of
        // the draws' sum -- a loop per NPC would cost the sum over NPCs of
        // the max, ~2x the draws at 64 lanes
        // The loop only collects the accepted draws (3 bits each, in alive
        // order); the moves follow in an unrolled pass over the slots, where
        // slot k's draw is the one at its rank among the alive slots.
        uint64_t draws = 0;
        if constexpr (std::is_same_v<BitsA, PyBits<AheadStream<1>>> && NCAP <= 8) {
          uint32_t d8 = 0;
          if (ai_choices8(ai, n, d8)) draws = d8;
          else draws = ai_choices<uint32_t>(ai, key, n, err);
        } else if constexpr (std::is_same_v<BitsA, PyBits<AheadStream<1>>>) {
          draws = ai_choices<std::conditional_t<(NCAP <= 10), uint32_t, uint64_t>>(ai, key, n, err);
        } else {  // stock-seed mode: a word of the game's CPython random per draw
          int j = 0;
          uint32_t tries = 0;
#pragma unroll 1
          while (j < n) {
            const uint32_t r = ai.bits(3, key);
            const bool acc = r < 5u;
            const bool give_up = !acc && ++tries >= kWordCap;
            if (acc || give_up) {
              err |= give_up;
              draws |= (uint64_t)(acc ? r : 0u) << (3 * j);
              ++j;
              tries = 0;
            }
          }
        }
#pragma unroll
        for (int k = 0; k < NCAP; ++k) {
          if (k < c.K && npc.is_alive(k)) {
            const int rank = __popc(npc.alive & ((1u << k) - 1u));
            const int32_t mv = 1 + (int32_t)((draws >> (3 * rank)) & 7ull);
            turns.set_move(k, npc_step_or_stay<GRID>(c, d, npc.get(k), mv));
          }
        }
      } else {
#pragma unroll 1
        for (int j = 0; j < n; ++j) {
          const int k = turns.slot(j);
          turns.set_move(k, decide_npc_move<GRID>(c, key, d, freeze, p1, p2, npc.get_rt(k), ai,
                                                  err));
        }
      }
    }
    ORX_MCYC_END(1, cy1);
    ORX_MCYC_BEGIN(cy2);
    // random.shuffle(npcs) (:127): Fisher-Yates over the list, its rejection
    // draws as one per-lane loop (as the AI's above)
    if constexpr (NCAP == kDense) {
      int i = n - 1;
      uint32_t tries = 0;
#pragma unroll 1
      while (i >= 1) {
        const uint32_t bound = (uint32_t)i + 1u;
        const uint32_t r = sh.bits(32 - __clz(bound), key);
        const bool acc = r < bound;
        const bool give_up = !acc && ++tries >= kWordCap;
        if (acc || give_up) {
          err |= give_up;
          const int jj = acc ? (int)r : 0;
          const int si = turns.slot(i), sj = turns.slot(jj);
          turns.set_slot(i, sj);
          turns.set_slot(jj, si);
          --i;
          tries = 0;
        }
      }
    } else if constexpr (NCAP > 0) {
      // register NPCs: the loop collects each position's accepted draw (4
      // bits at 4 i), the swaps follow unrolled, in the shuffle's order
      uint64_t js = 0;
      bool shuffled = true;
      if constexpr (std::is_same_v<BitsS, PyBits<AheadStream<2>>>) {
        // keyed mode without an event list: where no mover's target is an
        // NPC's cell or another mover's target, the NPCs' handle_move calls
        // commute (each is a move to a free cell, a hit on a player -- the
        // players moved first -- or a staircase death), so their order is
        // unobservable and its draws are skipped (the SHUFFLE stream is the
        // tick's own: nothing later reads it).  Only games whose NPCs
        // interact run the Fisher-Yates draws.
        shuffled = EV || !npc_moves_commute<NCAP>(c, npc, turns);
        order_free = !shuffled;
        if (shuffled)
          js = shuffle_draws<std::conditional_t<(NCAP <= 8), uint32_t, uint64_t>>(sh, key, n,
                                                                                 err);
      } else {  // stock-seed mode
        int i = n - 1;
        uint32_t tries = 0;
#pragma unroll 1
        while (i >= 1) {
          const uint32_t bound = (uint32_t)i + 1u;
          const uint32_t r = sh.bits(32 - __clz(bound), key);
          const bool acc = r < bound;
          const bool give_up = !acc && ++tries >= kWordCap;
          if (acc || give_up) {
            err |= give_up;
            js |= (uint64_t)(acc ? r : 0u) << (4 * i);
            --i;
            tries = 0;
          }
        }
      }
#pragma unroll
      for (int ii = NCAP - 1; ii >= 1; --ii) {
        if (shuffled && ii < n) {
          const int jj = (int)((js >> (4 * ii)) & 15ull);
          const int si = turns.slot(ii), sj = turns.slot(jj);
          turns.set_slot(ii, sj);
          turns.set_slot(jj, si);
        }
      }
    }
    ORX_MCYC_END(2, cy2);
  }
  ORX_MCYC_BEGIN(cy3);
  // handle_move in initiative order (:133-134): the players, then the NPCs
  auto&& spawn = src.spawn(tick);
  Player A = pick(p1_first, p1, p2);
  Player Bp = pick(p1_first, p2, p1);
  const int32_t a_iden = p1_first ? 1 : 2;
  mov_player<NCAP, EV, GRID>(c, key, src, A, Bp, p1_first ? c.d2 : c.d1, true, a_iden, npc, turns,
                             m, spawn, dl, err, ev);
  mov_player<NCAP, EV, GRID>(c, key, src, Bp, A, p1_first ? c.d1 : c.d2, false, 3 - a_iden, npc,
                             turns, m, spawn, dl, err, ev);
  p1 = pick(p1_first, A, Bp);
  p2 = pick(p1_first, Bp, A);
  ORX_MCYC_END(3, cy3);
  ORX_MCYC_BEGIN(cy4);
  if constexpr (NCAP > 0) {
    // a wave whose every game's NPC moves commute takes them per slot,
    // unrolled (constant slot indices, no occupant scan); otherwise the
    // shuffled order, as the reference
    bool done = false;
    if constexpr (NCAP != kDense && !EV) {
      if (__builtin_amdgcn_ballot_w64(!order_free) == 0ull) {
#pragma unroll
        for (int k = 0; k < NCAP; ++k) {
          const int32_t mv = turns.move(k);
          if (k < c.K && npc.is_alive(k) && mv != ORX_MOVE_STAY)
            mov_npc_free<NCAP, GRID>(c, k, mv, p1, p2, npc, d, dl);
        }
        done = true;
      }
    }
    if (!done) {
#pragma unroll 1
      for (int j = 0; j < n; ++j) {
        const int k = turns.slot(j);
        const int32_t mv = turns.move(k);
        if (mv != ORX_MOVE_STAY) mov_npc<NCAP, EV, GRID>(c, k, mv, p1, p2, npc, turns, d, m, dl, ev);
        turns.mark(k);
      }
    }
    ORX_MCYC_END(4, cy4);
    npc_sweep(c, npc, m, dl, ev);                       // :136-145
  }
  ORX_MCYC_BEGIN(cy5);
  end_tick<EV>(c, key, game, ep, p1, p2, tick, status, err, dl, ev, sep_start);
  ORX_MCYC_END(5, cy5);
}

// One Updater.update with moving NPCs (p1.move / p2.move = the raw moves):
// the tick's CPython-random draws -- the player shuffle, the AI's choices, the
// NPC shuffle -- from the tick block's word a and the SHUFFLE / NPC streams
// (keyed), or from the game's CPython random in the reference's call order
// (stock-seed mode).
template <int NCAP, bool EV, bool GRID, class Src, class M>
__device__ __forceinline__ void tick_moving(const Cfg& c, Key key, Src& src, uint32_t game,
                                            uint32_t ep, Player& p1, Player& p2,
                                            Npcs<NCAP>& npc, M& m, int32_t& tick,
                                            int32_t& status, bool& err, Deltas& dl,
                                            Events<EV>& ev, int32_t& sep_start,
                                            const W4* tb = nullptr) {
  if constexpr (Src::kMt) {
    MtBits b{&src.py};
    tick_moving_body<NCAP, EV, GRID>(c, key, src, game, ep, p1, p2, npc, m, tick, status, err, dl,
                                     ev, sep_start, b, b);
  } else {
    // (blocks ahead: the shuffle of 8 NPCs takes ~5 words past the tick
    // block's word, the AI's choices of 8 ~2)
    PyBits<AheadStream<2>> sh;
    PyBits<AheadStream<1>> ai;
    sh.res = tb ? tb->a : tick_block(key, game, ep, tick).a;  // (the caller's block if drawn)
    sh.nb = 32;
    sh.refill = false;
    sh.s.init(game, ep, (uint32_t)tick, tag(PUR_SHUFFLE, 0), key);
    ai.res = 0u;
    ai.nb = 0;
    ai.refill = true;
    ai.s.init(game, ep, (uint32_t)tick, tag(PUR_NPC, 0), key);
    tick_moving_body<NCAP, EV, GRID>(c, key, src, game, ep, p1, p2, npc, m, tick, status, err, dl,
                                     ev, sep_start, sh, ai);
  }
}

// Event records per game-tick (orx_max_events): 6 + 2 K with moving NPCs
__host__ __device__ inline int32_t max_events_for(int32_t npc_policy, int32_t K) {
  return (npc_policy != ORX_NPC_STAY && 6 + 2 * K > ORX_MAX_EVENTS) ? 6 + 2 * K : ORX_MAX_EVENTS;
}

// After a moving-NPC tick: the register NPCs' cells to HBM (the dense form
// moves them in place)
template <int NCAP>
__device__ __forceinline__ void store_npc_cells(const orx_state_t& st, const Cfg& c, uint32_t B,
                                                uint32_t i, const Npcs<NCAP>& npc) {
  if constexpr (NCAP > 0 && NCAP != kDense) {
#pragma unroll
    for (int k = 0; k < NCAP; ++k)
      if (k < c.K) st.npc_pos[(size_t)k * B + i] = (uint16_t)npc.get(k);
  }
}

template <int NCAP, bool EV, bool GRID = false, class M>
__device__ __forceinline__ void tick_game(const Cfg& c, Key key, uint32_t game, uint32_t ep,
                                          bool p1_first, Player& p1, Player& p2,
                                          Npcs<NCAP>& npc, Items<NCAP>& items, M& m,
                                          int32_t& tick, int32_t& status, bool& err, Deltas& dl,
                                          Events<EV>& ev, int32_t& sep_start) {
  PhiloxSrc src{key, game, ep};
  tick_game<NCAP, EV, GRID>(c, key, src, game, ep, p1_first, p1, p2, npc, items, m, tick, status,
                            err, dl, ev, sep_start);
}

// The character mechanics' state (ORX_EXT_RPG): p_rpg rows and the items.
// Without those flags only the register copies are zeroed (dead code in the
// kernels that know the flags are off).
template <int NCAP>
__device__ __forceinline__ void load_rpg(const orx_state_t& st, const Cfg& c, uint32_t B,
                                         uint32_t i, Player& p1, Player& p2, Npcs<NCAP>& npc,
                                         Items<NCAP>& it) {
  it.clear();
  p1.heal = p2.heal = 0;
  p1.hd = p2.hd = 0;
  if (!(c.ext & ORX_EXT_CHARACTER)) {
    p1.mana = p2.mana = p1.xp = p2.xp = p1.nitems = p2.nitems = p1.cool = p2.cool = 0;
    p1.dmg = p2.dmg = c.player_dmg;
    p1.mhp = p2.mhp = c.player_hp;
    return;
  }
  const int32_t* r = st.p_rpg + i;
  const size_t f = 2 * (size_t)B;
  p1.mana = r[ORX_RPG_MANA * f];           p2.mana = r[ORX_RPG_MANA * f + B];
  p1.xp = r[ORX_RPG_XP * f];               p2.xp = r[ORX_RPG_XP * f + B];
  p1.dmg = r[ORX_RPG_DAMAGE * f];          p2.dmg = r[ORX_RPG_DAMAGE * f + B];
  p1.mhp = r[ORX_RPG_MAX_HEALTH * f];      p2.mhp = r[ORX_RPG_MAX_HEALTH * f + B];
  p1.nitems = r[ORX_RPG_ITEMS * f];        p2.nitems = r[ORX_RPG_ITEMS * f + B];
  p1.cool = r[ORX_RPG_COOLDOWN * f];       p2.cool = r[ORX_RPG_COOLDOWN * f + B];
  if constexpr (NCAP > 0) {
    if (c.ext & ORX_EXT_ITEMS) {  // (after load_npcs) items into their NPCs' slots
      it.on = st.item_mask[i];
      it.kind = st.item_mask[B + i];
      for (int k = 0; k < c.K; ++k)
        if ((it.on >> k) & 1u) npc.set(k, st.item_pos[(size_t)k * B + i]);
    }
  }
}

template <int NCAP>
__device__ __forceinline__ void store_rpg(const orx_state_t& st, const Cfg& c, uint32_t B,
                                          uint32_t i, const Player& p1, const Player& p2,
                                          const Npcs<NCAP>& npc, const Items<NCAP>& it) {
  if (!(c.ext & ORX_EXT_CHARACTER)) return;
  int32_t* r = st.p_rpg + i;
  const size_t f = 2 * (size_t)B;
  r[ORX_RPG_MANA * f] = p1.mana;           r[ORX_RPG_MANA * f + B] = p2.mana;
  r[ORX_RPG_XP * f] = p1.xp;               r[ORX_RPG_XP * f + B] = p2.xp;
  r[ORX_RPG_DAMAGE * f] = p1.dmg;          r[ORX_RPG_DAMAGE * f + B] = p2.dmg;
  r[ORX_RPG_MAX_HEALTH * f] = p1.mhp;      r[ORX_RPG_MAX_HEALTH * f + B] = p2.mhp;
  r[ORX_RPG_ITEMS * f] = p1.nitems;        r[ORX_RPG_ITEMS * f + B] = p2.nitems;
  r[ORX_RPG_COOLDOWN * f] = p1.cool;       r[ORX_RPG_COOLDOWN * f + B] = p2.cool;
  if constexpr (NCAP > 0) {
    if (c.ext & ORX_EXT_ITEMS) {
      st.item_mask[i] = it.on;
      st.item_mask[B + i] = it.kind;
      for (int k = 0; k < c.K; ++k)
        if ((it.on >> k) & 1u) st.item_pos[(size_t)k * B + i] = (uint16_t)npc.get(k);
    }
  }
}

// ---------------------------------------------------------------------------
// SoA load / store helpers (32-bit lane index: B < 2^31)
// ---------------------------------------------------------------------------
template <bool GRID = false>
__device__ __forceinline__ void load_players(const orx_state_t& st, uint32_t B, uint32_t i,
                                             Player& p1, Player& p2) {
  p1.x = st.p_x[i];           p2.x = st.p_x[B + i];
  p1.y = st.p_y[i];           p2.y = st.p_y[B + i];
  p1.d = st.p_depth[i];       p2.d = st.p_depth[B + i];
  p1.hp = st.p_health[i];     p2.hp = st.p_health[B + i];
  p1.sx = st.st_x[i];         p2.sx = st.st_x[B + i];
  p1.sy = st.st_y[i];         p2.sy = st.st_y[B + i];
  p1.lay = GRID ? st.p_layout[i] : -1;
  p2.lay = GRID ? st.p_layout[B + i] : -1;
}

template <bool GRID = false>
__device__ __forceinline__ void store_players(const orx_state_t& st, uint32_t B, uint32_t i,
                                              const Player& p1, const Player& p2, bool stairs) {
  st.p_x[i] = p1.x;           st.p_x[B + i] = p2.x;
  st.p_y[i] = p1.y;           st.p_y[B + i] = p2.y;
  st.p_depth[i] = p1.d;       st.p_depth[B + i] = p2.d;
  st.p_health[i] = p1.hp;     st.p_health[B + i] = p2.hp;
  if (stairs) {
    st.st_x[i] = p1.sx;       st.st_x[B + i] = p2.sx;
    st.st_y[i] = p1.sy;       st.st_y[B + i] = p2.sy;
    if constexpr (GRID) {
      st.p_layout[i] = (int16_t)p1.lay;
      st.p_layout[B + i] = (int16_t)p2.lay;
    }
  }
}

// store_players after a tick of step_kernel: the depth rows (and the
// staircases) only when a player descended, the health rows only when `hp`
// (a combat, under the reference's rules; always with extensions, which
// change health in more ways), so the per-tick step moves 16 B less per game
// on most ticks
template <bool GRID = false>
__device__ __forceinline__ void store_players_tick(const orx_state_t& st, uint32_t B, uint32_t i,
                                                   const Player& p1, const Player& p2,
                                                   bool descended, bool hp) {
  st.p_x[i] = p1.x;           st.p_x[B + i] = p2.x;
  st.p_y[i] = p1.y;           st.p_y[B + i] = p2.y;
  if (hp) {
    st.p_health[i] = p1.hp;   st.p_health[B + i] = p2.hp;
  }
  if (descended) {
    st.p_depth[i] = p1.d;     st.p_depth[B + i] = p2.d;
    st.st_x[i] = p1.sx;       st.st_x[B + i] = p2.sx;
    st.st_y[i] = p1.sy;       st.st_y[B + i] = p2.sy;
    if constexpr (GRID) {
      st.p_layout[i] = (int16_t)p1.lay;
      st.p_layout[B + i] = (int16_t)p2.lay;
    }
  }
}

// Every slot's row is loaded unconditionally (slot k >= K re-reads row K-1
// and is masked off): a `k < K` guard would put each load behind a branch and
// a vmcnt(0) wait, and a lone wave per SIMD then pays one HBM round trip per
// slot (measured: a dozen serialized round trips per rollout launch).
template <int NCAP>
__device__ __forceinline__ void load_npcs(const orx_state_t& st, const Cfg& c, uint32_t B,
                                          uint32_t i, Npcs<NCAP>& npc) {
  if constexpr (NCAP == kDense) {  // the grid stays in HBM
    npc.bind(st, c, B, i);
  } else {
    npc.clear();
    if constexpr (NCAP > 0) {
      uint32_t v[NCAP];
#pragma unroll
      for (int k = 0; k < NCAP; ++k)
        v[k] = st.npc_pos[(size_t)min(k, c.K - 1) * B + i];
      npc.alive = st.npc_alive[i];
#pragma unroll
      for (int k = 0; k < NCAP; ++k)
        npc.set(k, (k < c.K && ((npc.alive >> k) & 1u)) ? v[k] : kDeadSlot);
    }
  }
}

// After a game start: NPC positions and health to HBM.
template <int NCAP>
__device__ __forceinline__ void store_new_npcs(const orx_state_t& st, const Cfg& c, uint32_t B,
                                            uint32_t i, const Npcs<NCAP>& npc,
                                            bool health = true) {
  if constexpr (NCAP > 0) {
    for (int k = 0; k < c.K; ++k) {
      // (dense NPCs: set() wrote the positions)
      if constexpr (NCAP != kDense) st.npc_pos[(size_t)k * B + i] = (uint16_t)npc.get(k);
      if (health) st.npc_health[(size_t)k * B + i] = (int8_t)c.npc_hp;
    }
  }
}

// All reads first, then all writes: interleaved read-modify-writes of
// may-alias int32 rows would serialize into one HBM round trip each.
__device__ __forceinline__ void flush_deltas(const orx_state_t& st, uint32_t B, uint32_t i,
                                             const Deltas& dl) {
  const bool cnt = st.counters && (dl.combat | dl.descend | dl.dungeon | dl.npc_death);
  if (cnt || dl.eps) {
    // without counters the four reads hit ret_sum[i] (valid, unused)
    const int32_t* c = (st.counters ? st.counters : st.ret_sum) + i;
    const size_t cs = st.counters ? B : 0;
    const int32_t c0 = c[0], c1 = c[cs], c2 = c[2 * cs], c3 = c[3 * cs];
    const int32_t r = st.ret_sum[i], e = st.ep_count[i];
    if (cnt) {
      st.counters[i] = c0 + dl.combat;
      st.counters[B + i] = c1 + dl.descend;
      st.counters[2 * (size_t)B + i] = c2 + dl.dungeon;
      st.counters[3 * (size_t)B + i] = c3 + dl.npc_death;
    }
    if (dl.eps) {
      st.ret_sum[i] = r + dl.ret;
      st.ep_count[i] = e + dl.eps;
    }
  }
}

// ceil(k / sep_period) for 1 <= k, k + sep_period - 1 < 2^31 (Cfg::sep_m)
__device__ __forceinline__ int32_t sep_ceil(const Cfg& c, int32_t k) {
  const uint32_t n = (uint32_t)(k + c.sep_period - 1);
  return (int32_t)(((uint64_t)n * c.sep_m) >> c.sep_sh);
}

__device__ __forceinline__ Cfg make_cfg(const orx_cfg_t& h, const orx_state_t& st) {
  Cfg c;
  c.W = h.width; c.H = h.height; c.despawn = h.despawn; c.max_ticks = h.max_ticks;
  c.start_mode = h.start_mode;
  c.d1 = h.start_mode == ORX_START_SEPARATED ? h.p1_depth : 0;
  c.d2 = h.start_mode == ORX_START_SEPARATED ? h.p2_depth : 0;
  c.K = h.n_npcs; c.npc_hp = h.npc_health; c.player_hp = h.player_health;
  c.player_dmg_net = h.player_damage - h.player_armor;
  c.npc_pol = h.npc_policy;
  c.npc_dmg_net = h.npc_damage - h.npc_armor;
  c.autoreset = h.autoreset;
  c.ext = h.flags;
  c.sep_period = h.sep_period > 0 ? h.sep_period : 1;
  c.sep_sh = 31;           // P = 1 (unused without separation damage)
  c.sep_m = 0x80000001u;
  if (h.flags & ORX_EXT_SEPARATION_DAMAGE) {  // (wave-uniform; the division only when used)
    const uint32_t P = (uint32_t)c.sep_period;
    const int32_t l = P > 1u ? 32 - __clz(P - 1u) : 0;
    c.sep_sh = 31 + l;
    c.sep_m = (uint32_t)((1ull << (31 + l)) / P) + 1u;
  }
  c.player_dmg = h.player_damage; c.player_armor = h.player_armor;
  c.mana_max = h.mana_max; c.mana_third = h.mana_max / 3; c.mana_regen = h.mana_regen;
  c.mana_pp = h.mana_per_point > 0 ? h.mana_per_point : 1;
  c.xp_kill = h.xp_per_kill; c.xp_level = h.xp_per_level > 0 ? h.xp_per_level : 1;
  c.drop_pct = h.item_drop_pct; c.item_bonus = h.item_bonus; c.item_slots = h.item_slots;
  c.cooldown = h.combat_cooldown;
  c.ih = h.height - 2;
  c.dstore_n = dstore_depths(h.max_ticks);
  c.ih_magic = (int64_t)(h.width - 2) * (h.height - 2) <= 65536
                   ? (uint32_t)(0xFFFFFFFFu / (uint32_t)c.ih + 1u) : 0u;
  c.h_magic = (int64_t)h.width * h.height <= 65536
                  ? (uint32_t)(0xFFFFFFFFu / (uint32_t)h.height + 1u) : 0u;
  c.ground.set((h.width - 2) * (h.height - 2) - 1);
  c.stair_x.set(h.width - 3);
  c.stair_y.set(h.height - 3);
  c.L = h.n_layouts;
  c.layout.set(h.n_layouts > 0 ? h.n_layouts : 1);
  c.tiles = st.bank_tiles;
  c.gground = st.bank_ground;
  c.gmeta = st.bank_meta;
  c.lds_tiles = false;
  return c;
}

__device__ __forceinline__ bool valid_move(const Cfg& c, int32_t m) {
  return m >= ORX_MOVE_UP && m <= ((c.ext & ORX_EXT_HEAL) ? ORX_MOVE_HEAL : ORX_MOVE_STAY);
}

__device__ __forceinline__ uint16_t pack_actions(int32_t a1, int32_t a2) {
  return (uint16_t)((uint32_t)(uint8_t)a1 | ((uint32_t)(uint8_t)a2 << 8));
}

// ---------------------------------------------------------------------------
// Kernels (NCAP = NPC slot capacity: 0, 8 or 16)
// ---------------------------------------------------------------------------
template <int NCAP, bool GRID>
__global__ void __launch_bounds__(256) reset_kernel(orx_cfg_t hc, orx_state_t st,
                                                    const uint8_t* __restrict__ mask, uint32_t B,
                                                    Key key, uint32_t off) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  if (mask && !mask[i]) return;
  const Cfg c = make_cfg(hc, st);
  Player p1, p2;
  Npcs<NCAP> npc;
  npc.bind(st, c, B, i);
  int32_t tick, status;
  setup_game<NCAP, GRID>(c, key, off + i, (uint32_t)st.episode[i], p1, p2, npc, tick, status);
  store_players<GRID>(st, B, i, p1, p2, true);
  Items<NCAP> items;
  items.clear();
  store_rpg(st, c, B, i, p1, p2, npc, items);
  st.tick[i] = tick;
  st.status[i] = status;
  if (c.ext & ORX_EXT_SEPARATION_DAMAGE) st.sep_start[i] = -1;
  if constexpr (NCAP > 0) {
    npc.store_alive(st.npc_alive, B, i);
    store_new_npcs(st, c, B, i, npc);
  }
}

// EXT = false: the reference's rules only (cfg.flags == 0), the extension
// code compiled out -- fewer registers, so more waves per SIMD hide the
// state loads (the per-tick drop-in's common case)
// One game's Updater.update (or its autoreset): the per-tick step kernels'
// body.  get_action(p1, p2, tick, ep, tb) yields the game's packed action pair
// (player 1 in the low byte).  Without an output callback (NoOut: the step
// kernels) it is called only for a game in progress, with p1 / p2 / tick /
// ep / tb not loaded.  With one (env_step_kernel) every state word is loaded
// up front -- one round trip for the whole launch -- get_action sees the
// pre-tick players and the tick block for every game (one Philox block serves
// player 2's RandomBot and the initiative draw), and out(p1, p2, tick,
// status) receives the post-step state from registers (no re-read of what
// was just stored).
#ifndef ORX_STEP_EAGER
#define ORX_STEP_EAGER 1
#endif
struct NoOut {
  __device__ __forceinline__ void operator()(const Player&, const Player&, int32_t, int32_t) {}
};

template <int NCAP, bool EV, bool GRID, bool EXT, bool MOV, class A, class O = NoOut>
__device__ __forceinline__ void step_game(const orx_cfg_t& hc, const orx_state_t& st, A get_action,
                                          uint32_t B, uint32_t i, Key key, uint32_t off,
                                          int32_t* __restrict__ events,
                                          int32_t* __restrict__ n_events, O out = O{}) {
  constexpr bool kOut = !std::is_same<O, NoOut>::value;
  // every state word and the action pair in one round trip (a finished game
  // discards some) -- the step kernels too: loaded behind the status and
  // action tests, a game in progress waited out three round trips in a row
  constexpr bool kEager = kOut || ORX_STEP_EAGER;
  Cfg c = make_cfg(hc, st);
  if constexpr (!EXT) c.ext = 0;
  const uint32_t game = off + i;
  int32_t status = st.status[i];
  Npcs<NCAP> npc;
  npc.bind(st, c, B, i);
  Player p1, p2;
  int32_t tick = 0;
  uint32_t ep = 0;
  uint16_t a = 0;
  Items<NCAP> items;
  int32_t sep = -1;
  W4 tb0{0, 0, 0, 0};  // (kOut) the tick block: player 2's policy and the initiative draw
  if constexpr (kEager) {
    load_players<GRID>(st, B, i, p1, p2);
    tick = st.tick[i];
    ep = (uint32_t)st.episode[i];
    load_npcs(st, c, B, i, npc);
    load_rpg(st, c, B, i, p1, p2, npc, items);
    if (c.ext & ORX_EXT_SEPARATION_DAMAGE) sep = st.sep_start[i];
    if constexpr (kOut) tb0 = tick_block(key, game, ep, tick);
    a = get_action(p1, p2, tick, ep, tb0);
  }
  if (status != ORX_IN_PROGRESS) {
    if (EV) n_events[i] = 0;
    if (!c.autoreset) {
      out(p1, p2, tick, status);
      return;
    }
    const uint32_t ep1 = (kEager ? ep : (uint32_t)st.episode[i]) + 1u;
    setup_game<NCAP, GRID>(c, key, game, ep1, p1, p2, npc, tick, status);
    store_players<GRID>(st, B, i, p1, p2, true);
    items.clear();
    store_rpg(st, c, B, i, p1, p2, npc, items);
    st.tick[i] = tick;
    st.status[i] = status;
    st.episode[i] = (int32_t)ep1;
    if (c.ext & ORX_EXT_SEPARATION_DAMAGE) st.sep_start[i] = -1;
    if constexpr (NCAP > 0) {
      npc.store_alive(st.npc_alive, B, i);
      store_new_npcs(st, c, B, i, npc);
    }
    out(p1, p2, tick, status);
    return;
  }
  if constexpr (!kEager) a = get_action(p1, p2, tick, ep, tb0);
  p1.move = (int8_t)(a & 0xFF);
  p2.move = (int8_t)(a >> 8);
  if (!valid_move(c, p1.move) || !valid_move(c, p2.move)) {
    st.status[i] = ORX_STATUS_BAD_ACTION;
    if (EV) n_events[i] = 0;
    out(p1, p2, tick, (int32_t)ORX_STATUS_BAD_ACTION);
    return;
  }
  if constexpr (!kEager) {
    ep = (uint32_t)st.episode[i];
    tick = st.tick[i];
    load_players<GRID>(st, B, i, p1, p2);
    load_npcs(st, c, B, i, npc);
    load_rpg(st, c, B, i, p1, p2, npc, items);
    if (c.ext & ORX_EXT_SEPARATION_DAMAGE) sep = st.sep_start[i];
  }
  NpcMem m{st.npc_pos, st.npc_health, B, i};
  Deltas dl = {0, 0, 0, 0, 0, 0};
  const int32_t ev_cap = MOV ? max_events_for(c.npc_pol, c.K) : ORX_MAX_EVENTS;
  Events<EV> ev{EV ? events + (size_t)i * (size_t)ev_cap * 4 : nullptr, 0, ev_cap};
  bool err = false;
  if constexpr (MOV) {  // moving NPCs: the literal ordered tick draws its own shuffles
    PhiloxSrc src{key, game, ep};
    tick_moving<NCAP, EV, GRID>(c, key, src, game, ep, p1, p2, npc, m, tick, status, err, dl, ev,
                                sep);
    store_npc_cells(st, c, B, i, npc);
  } else {
    const bool p1_first = kOut ? first_from_packed(tb0.a, key, game, ep, tick, err)
                               : p1_first_draw(key, game, ep, tick, err);
    tick_game<NCAP, EV, GRID>(c, key, game, ep, p1_first, p1, p2, npc, items, m, tick, status,
                              err, dl, ev, sep);
  }
  if (c.ext & ORX_EXT_SEPARATION_DAMAGE) st.sep_start[i] = sep;
  store_rpg(st, c, B, i, p1, p2, npc, items);
  store_players_tick<GRID>(st, B, i, p1, p2, dl.descend != 0, EXT ? true : dl.combat != 0);
  st.tick[i] = tick;
  if (status != ORX_IN_PROGRESS) st.status[i] = status;  // (it was InProgress)
  if (NCAP > 0 && dl.npc_death) npc.store_alive(st.npc_alive, B, i);
  flush_deltas(st, B, i, dl);
  if (EV) n_events[i] = ev.n;
  out(p1, p2, tick, status);
}

template <int NCAP, bool EV, bool GRID, bool EXT = true, bool MOV = false>
__global__ void __launch_bounds__(256) step_kernel(orx_cfg_t hc, orx_state_t st,
                                                   const int8_t* __restrict__ actions, uint32_t B,
                                                   Key key, uint32_t off,
                                                   int32_t* __restrict__ events,
                                                   int32_t* __restrict__ n_events) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  step_game<NCAP, EV, GRID, EXT, MOV>(
      hc, st,
      [&](const Player&, const Player&, int32_t, uint32_t, const W4&) {
        return reinterpret_cast<const uint16_t*>(actions)[i];
      },
      B, i, key, off, events, n_events);
}

#if ORX_HOST_TU
__global__ void __launch_bounds__(256) policy_kernel(orx_state_t st, int32_t pol1, int32_t pol2,
                                                     int8_t* __restrict__ actions, uint32_t B,
                                                     Key key, uint32_t off) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  Player p1, p2;
  if (pol1 == ORX_POLICY_STAIRCASE || pol2 == ORX_POLICY_STAIRCASE) {
    p1.x = st.p_x[i]; p2.x = st.p_x[B + i];
    p1.y = st.p_y[i]; p2.y = st.p_y[B + i];
    p1.sx = st.st_x[i]; p2.sx = st.st_x[B + i];
    p1.sy = st.st_y[i]; p2.sy = st.st_y[B + i];
  }
  const bool need_rng = pol1 == ORX_POLICY_RANDOM || pol2 == ORX_POLICY_RANDOM;
  const uint32_t ep = need_rng ? (uint32_t)st.episode[i] : 0u;
  const int32_t tick = need_rng ? st.tick[i] : 0;
  uint16_t* out = reinterpret_cast<uint16_t*>(actions);
  int32_t a1 = ORX_MOVE_STAY, a2 = ORX_MOVE_STAY;
  if (pol1 == ORX_POLICY_NONE || pol2 == ORX_POLICY_NONE) {
    const uint16_t prev = out[i];
    a1 = (int8_t)(prev & 0xFF);
    a2 = (int8_t)(prev >> 8);
  }
  const W4 tb = need_rng ? tick_block(key, off + i, ep, tick) : W4{0, 0, 0, 0};
  policy_pair(key, off + i, ep, tick, pol1, pol2, tb, p1, p2, a1, a2);
  out[i] = pack_actions(a1, a2);
}
#endif  // ORX_HOST_TU

// A learner's tick (orx_env_step, VecEnv.step): the learner's actions read at
// their own width (dsize bytes; anything outside 1..max move becomes 0, which
// the step turns into ORX_STATUS_BAD_ACTION, so a wrapped int8 never becomes
// a legal move), player 2's move from policy `pol2` when cols == 1 (the
// pre-tick players), the pair written to act (the engine's actions buffer),
// step_game, and the game's observation row [14], status, reward (player 1's
// view: +1 / -1 on the tick its episode ends in a win / loss) and done (that
// tick; an engine stop code >= 16 is a truncation) -- VecEnv.outcome on
// device, no host sync.  Every state word is loaded once up front and the
// row comes from registers (step_game's output callback): one HBM round trip
// per launch.  The rows [B][14] are written through LDS (lds_rows): each
// thread parks its 14 words, and the workgroup then stores its 256 rows as
// one contiguous 14 KiB run, every store instruction a full 256-byte
// segment -- written directly, a lane's 14 stores land 56 B apart and each
// instruction touches 28 cache lines.  bad_count (may be NULL): += the games
// whose actions were refused this tick (one atomic per wave that has any).
#ifndef ORX_ENV_WAVES
#define ORX_ENV_WAVES 1
#endif
#ifndef ORX_ENV_DIAG  // diagnostic builds: 1 no tick, 2 no observation rows
#define ORX_ENV_DIAG 0
#endif
template <int NCAP, bool GRID, bool EXT, bool MOV = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ORX_ENV_WAVES)))
env_step_kernel(
    orx_cfg_t hc, orx_state_t st, const void* __restrict__ actions, int32_t dsize, int32_t cols,
    int32_t pol2, int8_t* __restrict__ act, int32_t* __restrict__ obs, float* __restrict__ reward,
    uint8_t* __restrict__ done, int32_t* __restrict__ status_out, uint32_t* __restrict__ bad_count,
    uint32_t B, Key key, uint32_t off, int32_t lds_rows, uint32_t lanes) {
  __shared__ __attribute__((aligned(16))) int32_t rows_lds[256 * ORX_OBS_FIELDS];
  // `lanes` games per wave (64, or 32: two half-full waves per SIMD at the
  // config batch, whose state loads then overlap the other wave's tick); a
  // workgroup's games are contiguous, its row in LDS is the game's index in it
  const uint32_t wl = threadIdx.x & 63u;
  const uint32_t gi = (threadIdx.x >> 6) * lanes + wl;   // the game's index in the workgroup
  const uint32_t per_block = (blockDim.x >> 6) * lanes;
  const uint32_t i = blockIdx.x * per_block + gi;
  const bool live = wl < lanes && i < B;
  bool bad = false;
  if (live) {
    const int64_t hi = (EXT && (hc.flags & ORX_EXT_HEAL)) ? ORX_MOVE_HEAL : ORX_MOVE_STAY;
    auto learner = [&](uint32_t k) -> int32_t {
      int64_t v;
      if (dsize == 1) v = reinterpret_cast<const int8_t*>(actions)[k];
      else if (dsize == 2) v = reinterpret_cast<const int16_t*>(actions)[k];
      else if (dsize == 4) v = reinterpret_cast<const int32_t*>(actions)[k];
      else v = reinterpret_cast<const int64_t*>(actions)[k];
      return (v >= ORX_MOVE_UP && v <= hi) ? (int32_t)v : 0;
    };
    // player 1's (and with cols == 2 player 2's) learner action, read before
    // the state so that both loads are in flight together
    const int32_t l1 = learner(cols == 1 ? i : 2u * i);
    const int32_t l2 = cols == 2 ? learner(2u * i + 1u) : (int32_t)ORX_MOVE_STAY;
    uint16_t pair = 0;
    int32_t before = ORX_IN_PROGRESS;
    auto get_action = [&](const Player& p1, const Player& p2, int32_t tick, uint32_t ep,
                          const W4& tb) {
      int32_t a1 = l1, a2 = l2;
      if (cols == 1 && pol2 != ORX_POLICY_STAY) {  // (orx_env_step refuses POLICY_NONE here)
        int32_t keep = a1;
        policy_pair(key, off + i, ep, tick, ORX_POLICY_NONE, pol2, tb, p1, p2, keep, a2);
      }
      pair = pack_actions(a1, a2);
      return pair;
    };
    auto out = [&](const Player& p1, const Player& p2, int32_t tick, int32_t after) {
      const int32_t row[ORX_OBS_FIELDS] = {p1.x, p1.y, p1.d, p1.hp, p2.x, p2.y, p2.d, p2.hp,
                                           tick, after, p1.sx, p1.sy, p2.sx, p2.sy};
      if constexpr ((ORX_ENV_DIAG & 2) != 0) {  // diagnostic: no observation rows
        if (row[0] == -12345) obs[i] = row[1];   // (keeps the row's values live)
      } else if (lds_rows) {  // (uniform) seven 8-byte LDS writes (a row is 56 B)
        int2* r2 = reinterpret_cast<int2*>(rows_lds + gi * ORX_OBS_FIELDS);
#pragma unroll
        for (int f = 0; f < ORX_OBS_FIELDS / 2; ++f) r2[f] = make_int2(row[2 * f], row[2 * f + 1]);
      } else {
#pragma unroll
        for (int f = 0; f < ORX_OBS_FIELDS; ++f) obs[(size_t)i * ORX_OBS_FIELDS + f] = row[f];
      }
      const bool ended = before == ORX_IN_PROGRESS && after >= ORX_PLAYER1_WIN &&
                         (after <= ORX_TIE || after >= ORX_STATUS_BAD_ACTION);
      done[i] = ended ? 1 : 0;
      reward[i] = !ended ? 0.0f : after == ORX_PLAYER1_WIN ? 1.0f
                                : after == ORX_PLAYER2_WIN ? -1.0f : 0.0f;
      if (status_out) status_out[i] = after;
      bad = before == ORX_IN_PROGRESS && after == ORX_STATUS_BAD_ACTION;
    };
    before = st.status[i];
    if constexpr ((ORX_ENV_DIAG & 1) != 0) {  // diagnostic: no tick (the outputs of the loaded state)
      Player p1, p2;
      load_players<GRID>(st, B, i, p1, p2);
      pair = pack_actions(l1, l2);
      out(p1, p2, st.tick[i], before);
    } else {
      step_game<NCAP, false, GRID, EXT, MOV>(hc, st, get_action, B, i, key, off, nullptr,
                                             nullptr, out);
    }
    reinterpret_cast<uint16_t*>(act)[i] = pair;
  }
  if (lds_rows && (ORX_ENV_DIAG & 2) == 0) {  // the workgroup's rows as one run (uniform)
    __syncthreads();
    const uint32_t g0 = blockIdx.x * per_block;
    const uint32_t n = (g0 < B ? min(B - g0, per_block) : 0u) * ORX_OBS_FIELDS;
    int32_t* base = obs + (size_t)g0 * ORX_OBS_FIELDS;
    // 16-byte stores (a full block's run is 896 of them; its base is
    // 14,336 B-aligned), the run's last n % 4 words one by one
    const uint32_t n4 = n >> 2;
    const int4* src4 = reinterpret_cast<const int4*>(rows_lds);
    int4* dst4 = reinterpret_cast<int4*>(base);
#pragma unroll
    for (int k = 0; k < (256 * ORX_OBS_FIELDS / 4 + 255) / 256; ++k) {
      const uint32_t j = (uint32_t)k * blockDim.x + threadIdx.x;
      if (j < n4) dst4[j] = src4[j];
    }
    const uint32_t jt = (n4 << 2) + threadIdx.x;
    if (jt < n) base[jt] = rows_lds[jt];
  }
  if (bad_count) {  // uniform (idle lanes: bad false)
    const uint64_t m = __builtin_amdgcn_ballot_w64(bad);
    if (m != 0ull && __lane_id() == (uint32_t)__builtin_ctzll(m))
      __hip_atomic_fetch_add(bad_count, (uint32_t)__builtin_popcountll(m), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  }
}

// One player descends -- the common case of handle_descend (updater.py:259-296)
// on a keyed empty dungeon -- as straight-line selects: the staircase from
// the first block of the new depth's (episode, depth, generation) stream, or
// the other player's when it stands on that depth; the spawn cell from the
// first word of the tick's SPAWN stream, taken when that word is accepted and
// the cell is neither of the other player's cells (before and after its
// move; then the initiative order cannot matter and no clash is possible)
// and no NPC lives on the new depth.  Both blocks are drawn side by side.
// Writes the descender's depth, cell and staircase and returns true; false
// (nothing written) sends the tick to the general form.  st1: player 1
// descends.  (ox0, oy0) / (ox1, oy1): the other player's cell before / after
// its move this tick.
template <int NCAP>
__device__ __forceinline__ bool fast_descend(const Cfg& c, Key key, uint32_t game, uint32_t ep,
                                             int32_t t0, bool st1, Player& p1, Player& p2,
                                             int32_t ox0, int32_t oy0, int32_t ox1, int32_t oy1,
                                             const Npcs<NCAP>& npc, Deltas& dl) {
  const int32_t sd = st1 ? p1.d : p2.d, od = st1 ? p2.d : p1.d;
  const int32_t o_start = st1 ? c.d2 : c.d1;
  const int32_t nd = sd + 1;
  bool present;
  uint32_t gen = 0;
  if (c.despawn == ORX_DESPAWN_UNREACHABLE) {
    present = o_start <= nd && nd <= od;
  } else {
    present = od == nd;
    gen = (!present && o_start <= nd && nd < od) ? 1u : 0u;
  }
  const bool other_on = od == nd;
  W4 wd = philox(game, ep, (uint32_t)nd, tag(PUR_DUNGEON, gen), key);
  W4 ws = philox(game, ep, (uint32_t)t0, tag(PUR_SPAWN, 0), key);
  launder_w4(wd);
  launder_w4(ws);
  int32_t sx, sy;
  bool ok = stair_from_block(c, wd, sx, sy);
  const bool o_stairs = present & other_on;
  sx = o_stairs ? (st1 ? p2.sx : p1.sx) : sx;
  sy = o_stairs ? (st1 ? p2.sy : p1.sy) : sy;
  ok |= o_stairs;
  const uint32_t v = ws.a & c.ground.mask;
  int32_t x, y;
  ground_cell<false>(c, v, -1, sx, sy, x, y);
  const bool touch = other_on & (((x == ox1) & (y == oy1)) | ((x == ox0) & (y == oy0)));
  const bool npc_depth = NCAP > 0 && nd == c.d1 && npc.any_alive();
  ok = ok & (c.ground.rng != 0u) & (v <= c.ground.rng) & !touch & !npc_depth;
  if (ok) {
    p1.d = st1 ? nd : p1.d;
    p1.x = st1 ? x : p1.x;
    p1.y = st1 ? y : p1.y;
    p1.sx = st1 ? sx : p1.sx;
    p1.sy = st1 ? sy : p1.sy;
    p2.d = st1 ? p2.d : nd;
    p2.x = st1 ? p2.x : x;
    p2.y = st1 ? p2.y : y;
    p2.sx = st1 ? p2.sx : sx;
    p2.sy = st1 ? p2.sy : sy;
    dl.descend += 1;
    dl.dungeon += present ? 0 : 1;
  }
  return ok;
}

// updater.py:150-162 over the max_ticks result the rollout's common path set,
// after a combat or separation damage there (the ordered path has its own
// chain; a double death is a Tie: ORX_EXT_RANDOM_DOUBLE_DEATH is ordered).
__device__ __forceinline__ void deaths_over(const Player& p1, const Player& p2, bool end,
                                            int32_t& status, Deltas& dl) {
  const bool d1 = p1.hp <= 0, d2 = p2.hp <= 0;
  if ((d1 | d2) && status != ORX_STATUS_RNG_EXHAUSTED) {
    const int32_t s = d1 ? (d2 ? ORX_TIE : ORX_PLAYER2_WIN) : ORX_PLAYER1_WIN;
    dl.eps += end ? 0 : 1;
    dl.ret += (s == ORX_PLAYER1_WIN ? 1 : 0) - (s == ORX_PLAYER2_WIN ? 1 : 0);
    status = s;
  }
}

// The rare block of a rollout tick (rollout_tick's comment lists its cases),
// from the pre-tick state: finishes the game's tick in place and returns
// whether it ran the ordered tick (which applies its own extensions).  Also
// the paired rollout's rare path (pair_rollout_kernel), where both lanes of a
// game run it on the same rebuilt pair of players.
template <int NCAP, bool GRID, class M>
__device__ __forceinline__ bool rare_tick(const Cfg& c, const orx_state_t& st, uint32_t B,
                                          uint32_t i, Key key, uint32_t game, uint32_t& ep,
                                          Player& p1, Player& p2, Npcs<NCAP>& npc,
                                          Items<NCAP>& items, M& hp, int32_t& tick,
                                          int32_t& status, Deltas& dl, int32_t& sep,
                                          bool& restarted, const W4& tb, int need, int32_t t1x,
                                          int32_t t1y, int32_t t2x, int32_t t2y,
                                          bool ext_ordered, bool bad_action = false) {
  if (bad_action) {  // a replay's pair outside the Move codes: the game stops (orx_step)
    status = ORX_STATUS_BAD_ACTION;
    return false;
  }
  launder(t1x, t1y, t2x, t2y);
  launder(p1.x, p1.y, p2.x, p2.y);
  launder(p1.d, p2.d, p1.sx, p1.sy);
  launder(p2.sx, p2.sy, status, tick);
  const bool in_progress = status == ORX_IN_PROGRESS;
  const bool meet = ((uint32_t)(p1.d ^ p2.d) |
                     min((uint32_t)(t1x ^ p2.x) | (uint32_t)(t1y ^ p2.y),
                         min((uint32_t)(t2x ^ p1.x) | (uint32_t)(t2y ^ p1.y),
                             (uint32_t)(t1x ^ t2x) | (uint32_t)(t1y ^ t2y)))) == 0u;
  const uint32_t k1 = (uint32_t)t1x | ((uint32_t)t1y << 8);
  const uint32_t k2 = (uint32_t)t2x | ((uint32_t)t2y << 8);
  const bool hit1 = NCAP > 0 && (p1.d == c.d1) && npc_on(c, npc, k1);
  const bool hit2 = NCAP > 0 && (p2.d == c.d1) && npc_on(c, npc, k2);
  const bool st1 = stair_tile<GRID>(c, p1, t1x, t1y), st2 = stair_tile<GRID>(c, p2, t2x, t2y);
  const bool desc_meet = (st1 & (p2.d == p1.d + 1)) | (st2 & (p1.d == p2.d + 1));
  // the character mechanics (ORX_EXT_RPG) keep the common path's rules:
  // each attacker's own mana and damage, NPC hits and the kill credit in the
  // drawn order, steps onto items; a descend-meet (whose clash would undo a
  // step) takes the ordered tick
  const bool rpg_ordered = ((c.ext & ORX_EXT_CHARACTER) && desc_meet) ||
                           ((c.ext & ORX_EXT_README_COMBAT) && meet);
  // an NPC standing on a staircase (left there when an Unused-despawned
  // depth is regenerated with its staircase elsewhere) is attacked, not
  // descended through: handle_move tests pos_lookup before the tile
  // (updater.py:199-207), which the ordered tick follows literally
  const bool npc_stair = (hit1 & st1) | (hit2 & st2);
  const bool full0 =
      (meet & (st1 | st2)) | (st1 & st2) | ext_ordered | rpg_ordered | npc_stair;
  // the games that always use the initiative order: the ordered tick and a
  // meet.  A descend into the other's depth uses it only when its spawn
  // candidate is one of the other player's two cells (before and after its
  // move): the descend branch draws it then (first_from_packed)
  const bool ordered_use = in_progress & (full0 | meet);
  uint32_t pk_shf = tb.a;
  if (need == 0 && ordered_use) pk_shf = tick_block(key, game, ep, tick).a;
  // all sixteen 2-bit shuffle fields rejected (high bits all set): the
  // SHUFFLE stream fallback and its cap, in the ordered tick
  const bool shf_reject = ordered_use & ((pk_shf | 0x55555555u) == 0xFFFFFFFFu);
  const bool full = full0 | shf_reject;
  const bool took_ordered = in_progress & full;
  const int32_t t0 = tick, ft = tick + 1;
  const bool end = c.max_ticks && ft >= c.max_ticks;
  if (!in_progress) {
    if (c.autoreset) {  // the next episode (worldgen.py:77-87, 124-135)
#ifdef ORX_STAMPS
      ORX_COUNT(dl.n_reset);
      ORX_CYC_BEGIN(cy1);
#endif
      ep += 1;
      setup_game<NCAP, GRID>(c, key, game, ep, p1, p2, npc, tick, status);
      items.clear();
      if constexpr (NCAP > 0) {
        if constexpr (NCAP == kDense) {
          store_new_npcs(st, c, B, i, npc, true);  // health rows in HBM
        } else {
          store_new_npcs(st, c, B, i, npc, false);  // health: from hp at the end
          hp.fill(c.npc_hp);
        }
      }
      restarted = true;
      sep = -1;
#ifdef ORX_STAMPS
      ORX_CYC_END(dl.cy_reset, cy1);
#endif
    }
  } else if (full) {  // the ordered tick
#ifdef ORX_STAMPS
    ORX_COUNT(dl.n_ordered);
    ORX_CYC_BEGIN(cy1);
#endif
    bool err = false;
    const bool p1_first = first_from_packed(pk_shf, key, game, ep, t0, err);
    Events<false> ev{nullptr, 0};
    tick_game<NCAP, false, GRID>(c, key, game, ep, p1_first, p1, p2, npc, items, hp, tick,
                                 status, err, dl, ev, sep);
#ifdef ORX_STAMPS
    ORX_CYC_END(dl.cy_ordered, cy1);
#endif
  } else {
    // the common path's rules, then the one-sided events: a player that
    // hits an NPC, descends or meets the other does not move freely
    const bool lean = meet;
    const bool s1 = !lean & !hit1 & !st1, s2 = !lean & !hit2 & !st2;
    const int32_t x1o = p1.x, y1o = p1.y, x2o = p2.x, y2o = p2.y;  // for a descend-meet
    p1.x = s1 ? t1x : p1.x;
    p1.y = s1 ? t1y : p1.y;
    p2.x = s2 ? t2x : p2.x;
    p2.y = s2 ? t2y : p2.y;
    tick = ft;
    status = end ? ORX_TIE : ORX_IN_PROGRESS;
    dl.eps += end ? 1 : 0;
    bool desc_done = false;  // fast_descend finished it
    if constexpr (!GRID) {
      if (!lean & (st1 | st2)) {
#ifdef ORX_STAMPS
        ORX_CYC_BEGIN(cyf);
#endif
        // the other player has made its move above
        desc_done = fast_descend<NCAP>(c, key, game, ep, t0, st1, p1, p2,
                                       st1 ? x2o : x1o, st1 ? y2o : y1o,
                                       st1 ? p2.x : p1.x, st1 ? p2.y : p1.y, npc, dl);
#ifdef ORX_STAMPS
        if (desc_done) ORX_COUNT(dl.n_desc);
        ORX_CYC_END(dl.cy_desc, cyf);
#endif
      }
    }
    if (!lean & (st1 | st2) & !desc_done) {  // one player descends: the general form
#ifdef ORX_STAMPS
      ORX_COUNT(dl.n_desc);
      ORX_CYC_BEGIN(cy1);
#endif
      PhiloxSrc src{key, game, ep};
      auto spawn = src.spawn(t0);
      Events<false> ev{nullptr, 0};
      bool err = false;
      Player S = pick(st1, p1, p2);
      Player O = pick(st1, p2, p1);  // after its own move
      // into the other's depth (desc_meet), the drawn order matters: moving
      // first, the descender's spawn cell is tested against the other's
      // cell before that player's move, which may then attack it
      bool s_first = false;
      if (desc_meet) {
        const uint32_t pk = need > 0 ? pk_shf : tick_block(key, game, ep, t0).a;
        s_first = first_from_packed(pk, key, game, ep, t0, err) == st1;
      }
      const int32_t ox0 = st1 ? x2o : x1o, oy0 = st1 ? y2o : y1o;
      Player Ot = O;
      Ot.x = s_first ? ox0 : O.x;
      Ot.y = s_first ? oy0 : O.y;
      descend<NCAP, false, GRID>(c, key, src, S, Ot, st1 ? c.d2 : c.d1, npc, spawn, dl, err,
                                 st1 ? 1 : 2, ev);
      const bool clash = s_first & ((O.x != ox0) | (O.y != oy0)) & (O.x == S.x) & (O.y == S.y);
      O.x = clash ? ox0 : O.x;
      O.y = clash ? oy0 : O.y;
      S.hp -= (clash && c.player_dmg_net > 0) ? c.player_dmg_net : 0;
      dl.combat += clash ? 1 : 0;
      p1 = pick(st1, S, O);
      p2 = pick(st1, O, S);
      if (err) {  // an exhausted spawn stream stops the game (never observed)
        dl.eps -= end ? 1 : 0;
        status = ORX_STATUS_RNG_EXHAUSTED;
      }
      if (clash) deaths_over(p1, p2, end, status, dl);
#ifdef ORX_STAMPS
      ORX_CYC_END(dl.cy_desc, cy1);
#endif
    }
    bool kc1 = false, kc2 = false;  // ORX_EXT_LEVELING: each player's kill this tick
    if (NCAP > 0 && (hit1 | hit2)) {  // NPCs are swept after both moves
#ifdef ORX_STAMPS
      ORX_COUNT(dl.n_hits);
#endif
      Events<false> ev{nullptr, 0};
      dl.combat += (hit1 ? 1 : 0) + (hit2 ? 1 : 0);
      int32_t d1 = c.player_dmg_net > 0 ? c.player_dmg_net : 0, d2 = d1;
      if (c.ext & ORX_EXT_RPG) {  // each attacker's own damage and mana
        d1 = hit1 ? rpg_attack(c, p1) : 0;
        d2 = hit2 ? rpg_attack(c, p2) : 0;
      }
      const int h1 = hit1 ? npc.find(k1) : -1, h2 = hit2 ? npc.find(k2) : -1;
      if (c.ext & ORX_EXT_RPG) {
        // hits in the drawn order: one NPC hit by both (a meet) credits the
        // hit that takes it to zero
        bool sw = false;
        if (lean) {
          const uint32_t sa = ~(pk_shf >> 1) & 0x55555555u;
          sw = ((pk_shf >> __builtin_ctz(sa)) & 1u) == 0;
        }
        bool ka = false, kb = false;
        npc_hits(c, npc, hp, sw ? h2 : h1, sw ? h1 : h2, sw ? d2 : d1, sw ? d1 : d2, dl, ev,
                 ka, kb, sw ? k2 : k1, sw ? k1 : k2);
        kc1 = sw ? kb : ka;
        kc2 = sw ? ka : kb;
        if ((c.ext & ORX_EXT_ITEMS) && kc1) drop_item(c, key, game, ep, t0, h1, k1, npc, items);
        if ((c.ext & ORX_EXT_ITEMS) && kc2) drop_item(c, key, game, ep, t0, h2, k2, npc, items);
      } else {
        // two hits are then order-free: only the health left matters
        npc_hits(c, npc, hp, h1, h2, d1, d2, dl, ev, kc1, kc2, k1, k2);
      }
    }
    if (lean) {  // a meet: the two moves in the drawn order
#ifdef ORX_STAMPS
      ORX_COUNT(dl.n_meet);
#endif
      const uint32_t sa = ~(pk_shf >> 1) & 0x55555555u;  // nonzero: all-reject is ordered
      const bool p1_first = ((pk_shf >> __builtin_ctz(sa)) & 1u) != 0;
      const int32_t ax = p1_first ? t1x : t2x, ay = p1_first ? t1y : t2y;
      const int32_t bx = p1_first ? t2x : t1x, by = p1_first ? t2y : t1y;
      const int32_t fx0 = p1_first ? p1.x : p2.x, fy0 = p1_first ? p1.y : p2.y;
      const int32_t sx0 = p1_first ? p2.x : p1.x, sy0 = p1_first ? p2.y : p1.y;
      const bool hf = p1_first ? hit1 : hit2, hs = p1_first ? hit2 : hit1;
      const bool occf = (ax == sx0) & (ay == sy0);
      const int32_t fx = (occf | hf) ? fx0 : ax, fy = (occf | hf) ? fy0 : ay;
      const bool occs = (bx == fx) & (by == fy);
      const int32_t sx = (occs | hs) ? sx0 : bx, sy = (occs | hs) ? sy0 : by;
      const int32_t dmg = c.player_dmg_net > 0 ? c.player_dmg_net : 0;
      p1.x = p1_first ? fx : sx;
      p1.y = p1_first ? fy : sy;
      p2.x = p1_first ? sx : fx;
      p2.y = p1_first ? sy : fy;
      if (NCAP > 0 && (c.ext & ORX_EXT_ITEMS)) {  // the meet's steps onto items (a
        // health item may save a player hit in the tick: before the win check)
        if ((p1.d == c.d1) & ((p1.x != x1o) | (p1.y != y1o))) pick_up(c, p1, npc, items);
        if ((p2.d == c.d1) & ((p2.x != x2o) | (p2.y != y2o))) pick_up(c, p2, npc, items);
      }
      if (c.ext & ORX_EXT_RPG) {  // each attacker's own damage and mana
        const bool a1 = p1_first ? occf : occs, a2 = p1_first ? occs : occf;
        const int32_t e1 = a1 ? rpg_attack(c, p1) : 0, e2 = a2 ? rpg_attack(c, p2) : 0;
        p2.hp -= e1;
        p1.hp -= e2;
      } else {
        p1.hp -= (p1_first ? occs : occf) ? dmg : 0;
        p2.hp -= (p1_first ? occf : occs) ? dmg : 0;
      }
      dl.combat += (occf ? 1 : 0) + (occs ? 1 : 0);
      deaths_over(p1, p2, end, status, dl);
    }
    // the sweep's experience after every combat of the tick: a player the
    // other killed in a meet is not refilled
    if (NCAP > 0 && (c.ext & ORX_EXT_LEVELING)) {
      if (kc1) gain_xp(c, p1);
      if (kc2) gain_xp(c, p2);
    }
    if (NCAP > 0 && (c.ext & ORX_EXT_ITEMS) && !lean) {  // a step onto an item takes it
      // (readme.md:44; a meet's steps were taken above)
      if (!st1 & (p1.d == c.d1) & ((p1.x != x1o) | (p1.y != y1o))) pick_up(c, p1, npc, items);
      if (!st2 & (p2.d == c.d1) & ((p2.x != x2o) | (p2.y != y2o))) pick_up(c, p2, npc, items);
    }
  }
  return took_ordered;
}

// One rollout tick of one game (the hot loop of server/main.py:110-113,
// fused): the bots' moves (randombot.py:20-21, staircasebot.py:9-21), then
// Updater.update (updater.py:76-162) -- or, for a finished game, the next
// episode's setup (autoreset).
//
// Common path.  The initiative shuffle (updater.py:114) orders the two
// handle_move calls (:133-134, :180-243), but the order is observable only
// when the moves can interact: both players on one depth with a target equal
// to the other's cell or to the other's target (a "meet").  Otherwise each
// move resolves against the other's unchanged cell; NPCs never move and are
// swept only after both moves (:136-145), so an NPC hit does not depend on
// the order either; and a descend into a depth the other player is not on
// reads nothing the other's move changes.  So the common path resolves both
// moves independently from their effective targets (the own cell when
// staying or blocked), and its status is the max_ticks test alone: health
// changes only in combat.  Invariants used: two players on one depth never
// share a cell; no player stands on its depth's staircase or on an NPC.
//
// Every rare case sits in ONE out-of-line block -- a lone wave per SIMD pays
// ~40 cycles per branch instruction, taken or not, so a
// common tick carries that block's branch and the loop's:
//  * a finished game: the next episode's setup_game (autoreset);
//  * the ordered tick, tick_game, the reference's sequence literally: a meet
//    involving a staircase, both players descending (SPAWN stream order),
//    extension flags other than separation damage, shuffle bits that all
//    reject (their stream fallback can stop the game), bot draws beyond the
//    tick block's two segments;
//  * on the common path's tick: one player's descend (handle_descend,
//    :259-296) -- into the other's depth in the drawn order: descending
//    first, the spawn cell is tested against the other's old cell and the
//    other's move into it is a combat --; NPC hits (npc_hits), after the
//    descend, whose spawn test sees every NPC alive; and a meet without
//    staircases -- the two
//    moves in the drawn order, the first against the second's cell, the
//    second against the first's new cell; an occupied target is a combat
//    (every CombatFlag deals damage - armor: no Modifier exists) and the
//    attacker stays; deaths override the status.
//
// LOG (a replay, orx_step_n): the moves are given in a1 / a2 (pol1 = pol2 =
// ORX_POLICY_NONE) -- a game in progress with a pair outside the Move codes
// stops with ORX_STATUS_BAD_ACTION (the rare block, nothing else changes), and
// a heal move (ORX_EXT_HEAL) takes the ordered tick, the only one that heals.
template <int NCAP, bool GRID, class M, bool LOG = false>
__device__ __forceinline__ void rollout_tick(const Cfg& c, const orx_state_t& st, uint32_t B,
                                             uint32_t i, Key key, uint32_t game, uint32_t& ep,
                                             int32_t pol1, int32_t pol2, Player& p1,
                                             Player& p2, Npcs<NCAP>& npc, Items<NCAP>& items,
                                             M& hp, int32_t& tick, int32_t& status, Deltas& dl,
                                             int32_t& sep, bool& restarted, int32_t& a1,
                                             int32_t& a2) {
  // one tick block: the bots' bits and the initiative bits (§4).  Without a
  // RandomBot the block's only reader is the initiative order, which matters
  // only to rare games: the rare block draws it then (C5's StaircaseBots).
  const int need = (pol1 == ORX_POLICY_RANDOM ? 1 : 0) + (pol2 == ORX_POLICY_RANDOM ? 1 : 0);
  W4 tb = {0u, 0u, 0u, 0u};
  if (need > 0) tb = tick_block(key, game, ep, tick);  // uniform
  // RandomBot draws: the first two accepted 3-bit fields of bits 0-29 of
  // word b; the rare games whose word b holds fewer take word c and then the
  // POLICY stream in a separate unlikely block (moves_from_block), so the
  // common decode is 32-bit and loop-free
  int32_t r0 = ORX_MOVE_STAY, r1 = ORX_MOVE_STAY;
  if (need > 0) {  // uniform: skipped for StaircaseBot pairs (C5)
    const uint32_t acc = accepted3(tb.b);
    const uint32_t acc2 = acc & (acc - 1u);
    r0 = (int32_t)((tb.b >> (ffbl(acc) & 31u)) & 7u) + 1;
    r1 = (int32_t)((tb.b >> (ffbl(acc2) & 31u)) & 7u) + 1;
    if (ORX_UNLIKELY((need > 1 ? acc2 : acc) == 0u)) {
      bool err = false;  // (the rollout, like orx_policy's fused form, ignores exhaustion)
      moves_from_block(tb, need, key, game, ep, tick, r0, r1, err);
    }
  }
  assign_moves(pol1, pol2, r0, r1, p1, p2, a1, a2);
  p1.move = a1;
  p2.move = a2;
  const bool bad = LOG && status == ORX_IN_PROGRESS && !(valid_move(c, a1) && valid_move(c, a2));
  const bool heal = LOG && (c.ext & ORX_EXT_HEAL) && (a1 == ORX_MOVE_HEAL || a2 == ORX_MOVE_HEAL);
  const bool in_progress = status == ORX_IN_PROGRESS && !bad;

  // effective targets: the player's own cell when staying or blocked.  Empty
  // dungeons: a move changes one coordinate by one, so a blocked target is
  // the border and clamping it to the interior gives back the own cell
  calc_pos(p1.x, p1.y, p1.move, p1.tx, p1.ty);
  calc_pos(p2.x, p2.y, p2.move, p2.tx, p2.ty);
  int32_t t1x, t1y, t2x, t2y;
  bool g_st1 = false, g_st2 = false;  // bank: the target tile is a staircase
  if constexpr (GRID) {
    // one tile read per player: a Wall blocks, a staircase descends (a
    // blocked player's own cell is never a staircase)
    const bool in1 = (uint32_t)p1.tx < (uint32_t)c.W && (uint32_t)p1.ty < (uint32_t)c.H;
    const bool in2 = (uint32_t)p2.tx < (uint32_t)c.W && (uint32_t)p2.ty < (uint32_t)c.H;
    const uint32_t tile1 = bank_tile(c, p1.lay, in1 ? p1.tx : p1.x, in1 ? p1.ty : p1.y);
    const uint32_t tile2 = bank_tile(c, p2.lay, in2 ? p2.tx : p2.x, in2 ? p2.ty : p2.y);
    const bool b1 = !in1 || tile1 == ORX_TILE_WALL, b2 = !in2 || tile2 == ORX_TILE_WALL;
    g_st1 = !b1 && tile1 == ORX_TILE_STAIRCASE_DOWN;
    g_st2 = !b2 && tile2 == ORX_TILE_STAIRCASE_DOWN;
    t1x = b1 ? p1.x : p1.tx; t1y = b1 ? p1.y : p1.ty;
    t2x = b2 ? p2.x : p2.tx; t2y = b2 ? p2.y : p2.ty;
  } else {
    t1x = med3_i32(p1.tx, 1, c.W - 2); t1y = med3_i32(p1.ty, 1, c.H - 2);
    t2x = med3_i32(p2.tx, 1, c.W - 2); t2y = med3_i32(p2.ty, 1, c.H - 2);
  }
  // meet: same depth and (target 1 == cell 2 or target 2 == cell 1 or
  // target 1 == target 2), as one zero test over xor differences
  const uint32_t e12 = (uint32_t)(t1x ^ p2.x) | (uint32_t)(t1y ^ p2.y);
  const uint32_t e21 = (uint32_t)(t2x ^ p1.x) | (uint32_t)(t2y ^ p1.y);
  const uint32_t e11 = (uint32_t)(t1x ^ t2x) | (uint32_t)(t1y ^ t2y);
  const bool meet = ((uint32_t)(p1.d ^ p2.d) | min(e12, min(e21, e11))) == 0u;
  // NPC keys x | y << 8 (W, H <= 256 with NPCs; effective targets are in the grid)
  const uint32_t k1 = (uint32_t)t1x | ((uint32_t)t1y << 8);
  const uint32_t k2 = (uint32_t)t2x | ((uint32_t)t2y << 8);
  bool n1 = false, n2 = false;
  npc_any2(npc, k1, k2, n1, n2);
  const bool hit1 = NCAP > 0 && ((p1.d == c.d1) & n1);
  const bool hit2 = NCAP > 0 && ((p2.d == c.d1) & n2);
  const bool st1 = GRID ? g_st1 : stair_tile<GRID>(c, p1, t1x, t1y);
  const bool st2 = GRID ? g_st2 : stair_tile<GRID>(c, p2, t2x, t2y);
  const bool ext_ordered =  // uniform
      (c.ext & ~(ORX_EXT_SEPARATION_DAMAGE | ORX_EXT_CHARACTER)) != 0;
  // (ORX_EXT_ITEMS: items sit in their NPCs' slot registers, so hit1 / hit2
  // also flag a target holding an item -- a rare game, sorted out below)
  // The rare games: finished, or a meet, an NPC hit, a staircase, an item, an
  // extension that needs the literal sequence.  Only this union is formed
  // here; the rare block re-derives its parts (from laundered inputs, so they
  // are not kept live across the common path as 0/1 values).  The initiative
  // order is unobservable in a common tick, so its draw -- and the SHUFFLE
  // stream fallback of an all-reject word, whose 4,096-word cap is the only
  // way it could matter there (p < 2^-4000) -- is consulted by the rare
  // block only, where the order is used.
  const bool rare = !in_progress | meet | hit1 | hit2 | st1 | st2 | ext_ordered | heal;
  const int32_t ft = tick + 1;
  const bool end = c.max_ticks && ft >= c.max_ticks;

  // The rare block runs first, from the pre-tick state, and finishes its
  // games in place; the common tick's update follows as selects over the same
  // registers (applied after the block, the old and new values of a field
  // are never live together, so the loop carries no register copies).
  bool took_ordered = false;  // the ordered tick ran (it applies its own extensions)
  if (ORX_UNLIKELY(rare)) {
#ifdef ORX_STAMPS
    ORX_COUNT(dl.n_rare);
    ORX_CYC_BEGIN(cy0);
#endif
    took_ordered = rare_tick<NCAP, GRID>(c, st, B, i, key, game, ep, p1, p2, npc, items, hp,
                                         tick, status, dl, sep, restarted, tb, need, t1x,
                                         t1y, t2x, t2y, ext_ordered | heal, bad);
#ifdef ORX_STAMPS
    ORX_CYC_END(dl.cy_rare, cy0);
#endif
  }
  // the common tick: both players move to their effective targets
  p1.x = rare ? p1.x : t1x;
  p1.y = rare ? p1.y : t1y;
  p2.x = rare ? p2.x : t2x;
  p2.y = rare ? p2.y : t2y;
  dl.eps += (!rare & end) ? 1 : 0;
  status = rare ? status : (end ? ORX_TIE : ORX_IN_PROGRESS);
  tick = rare ? tick : ft;
  const int32_t t0 = ft - 1;  // the pre-tick tick of every game
  if (c.ext & ORX_EXT_README_COMBAT) {  // cooldowns run down (the ordered tick runs its own)
    const bool base = in_progress & !took_ordered;
    p1.cool = base ? max(p1.cool - 1, 0) : p1.cool;
    p2.cool = base ? max(p2.cool - 1, 0) : p2.cool;
  }
  if (c.ext & ORX_EXT_MANA) {  // the end of the tick: mana regeneration (readme.md:72)
    // (the in-progress games of the common path's rules; the ordered tick has its own)
    const bool base = in_progress & !took_ordered;
    p1.mana = base ? min(p1.mana + c.mana_regen, c.mana_max) : p1.mana;
    p2.mana = base ? min(p2.mana + c.mana_regen, c.mana_max) : p2.mana;
  }
  if (c.ext & ORX_EXT_SEPARATION_DAMAGE) {  // build extension (readme.md:46-47), C5's ladder
    // base: the in-progress games whose tick took the common path's rules
    // (free moves, or a hit, a descend or a meet in the rare block)
    // base: the in-progress games whose tick took the common path's rules
    // (free moves, or a hit, a descend or a meet in the rare block)
    const bool base = in_progress & !took_ordered;
    if (base) {
      if (p1.d != p2.d) {
        if (sep < 0) sep = t0;
        const int32_t k = t0 - sep + 1;
        const int32_t dmg = sep_ceil(c, k);
        if (p1.d < p2.d) p1.hp -= dmg; else p2.hp -= dmg;
        deaths_over(p1, p2, end, status, dl);
      } else {
        sep = -1;
      }
    }
  }
}

// Fused rollout: n_ticks x (policy, step); state and NPC positions stay in
// registers; tick t's observation row is streamed out to obs/act.  At the
// headline batch (65,536 games) this is ONE wave per SIMD, so the tick loop is
// bound by that wave's own issue and stalls: the common path is laid out
// straight (rare blocks -- descends, NPC hits, resets, RNG fallbacks -- marked
// unlikely and placed out of line: -13%), and every per-tick decision that
// can be a select is one.  (Rejected, measured: splitting a game over two
// lanes; a producer wave drawing the RNG ahead through an LDS ring -- won
// while a tick took four Philox blocks, lost once it took one.)

// One tick's trajectory rows: obs[t][f][i] (ORX_OBS_* fields) and act[t][i].
// FAST (both present): buffer stores from a running row pointer -- the 14
// per-lane field offsets i*4 + f*B*4 live in VGPRs for the whole launch (an
// opaque copy, so the compiler cannot rematerialize them per tick), so a
// tick's 15 stores need no per-field address arithmetic at all (the lone
// wave issues every instruction, scalar ones included, at one per 4 cycles);
// otherwise per-pointer checks and flat stores.  Nontemporal: the rows are
// written once and read by the caller later (measured -4% per launch).
constexpr int32_t kBufferDword3 = 0x00020000;  // gfx9 raw buffer, 32-bit elements
#ifndef ORX_STREAM_AUX
#define ORX_STREAM_AUX 2
#endif
constexpr int32_t kStreamAux = ORX_STREAM_AUX;  // cache policy: nt (measured)
// ... for rows whose per-wave segments are whole 128-B lines.  Narrower
// segments (fewer than 32 games per wave) are partial lines, which several
// waves complete: there nt stores cost up to 2x (C5 at 8 games per wave: 165
// us per launch with nt, 79 plain), so those launches store with the default
// policy (kPartialAux)
constexpr int32_t kPartialAux = 0;
// the launch tables pick an instance by (AUX == kStreamAux) == nt: equal
// policies would leave one store form with no instance
static_assert(kStreamAux != kPartialAux, "ORX_STREAM_AUX must differ from the partial-line policy");
// ORX_OBS_COMPACT rows (include/orx.h): a cell as x | y << 8 (x, y < 256),
// two int16 healths in a word, tick | status << 27
__device__ __forceinline__ uint32_t cell8(int32_t x, int32_t y) {
  return (uint32_t)x | ((uint32_t)y << 8);
}
__device__ __forceinline__ uint32_t compact_hp(int32_t hp1, int32_t hp2) {
  return ((uint32_t)hp1 & 0xFFFFu) | ((uint32_t)hp2 << 16);
}
__device__ __forceinline__ uint32_t compact_ts(int32_t tick, int32_t status) {
  return (uint32_t)tick | ((uint32_t)status << 27);
}

// CF: the compact row format (FAST writers; the generic writer reads `fmt`);
// ACT: a FAST writer also stores the action pair (a replay has its actions)
template <bool FAST, int AUX = kStreamAux, bool CF = false, bool ACT = true>
struct TrajWriter {
  static constexpr int kRows = CF ? ORX_OBS_COMPACT_FIELDS : ORX_OBS_FIELDS;
  int32_t* obs;
  int8_t* act;
  uint32_t B, i;
  int32_t fmt;  // the generic writer's row format
  uint32_t vo[kRows], va;
  __device__ __forceinline__ TrajWriter(int32_t* o, int8_t* a, uint32_t B_, uint32_t i_,
                                        int32_t fmt_ = ORX_OBS_INT32)
      : obs(o), act(a), B(B_), i(i_), fmt(fmt_) {
    if constexpr (FAST) {
#pragma unroll
      for (int f = 0; f < kRows; ++f) {
#ifdef ORX_OBS_TILED  // diagnostic: [T][B/64][14][64] tiles (B a multiple of 64)
        vo[f] = ((i >> 6) * (uint32_t)kRows * 64u + (uint32_t)f * 64u + (i & 63u)) * 4u;
#else
        vo[f] = i * 4u + (uint32_t)f * B * 4u;
#endif
        asm volatile("" : "+v"(vo[f]));
      }
      va = i * 2u;
      asm volatile("" : "+v"(va));
    }
  }
  // a FAST writer's next rows
  __device__ __forceinline__ void skip() {
    obs += (size_t)kRows * B;
    if constexpr (ACT) act += (size_t)2 * B;
  }
  // row t, the next row of a FAST writer
  __device__ __forceinline__ void write(int32_t t, const Player& p1, const Player& p2,
                                        int32_t tick, int32_t status, int32_t a1, int32_t a2) {
    if constexpr (FAST) {
      const auto ro = __builtin_amdgcn_make_buffer_rsrc(obs, 0, (int32_t)(kRows * B * 4u),
                                                        kBufferDword3);
      if constexpr (CF) {
        const uint32_t vals[kRows] = {cell8(p1.x, p1.y) | (cell8(p2.x, p2.y) << 16),
                                      cell8(p1.sx, p1.sy) | (cell8(p2.sx, p2.sy) << 16),
                                      compact_hp(p1.hp, p2.hp), (uint32_t)p1.d, (uint32_t)p2.d,
                                      compact_ts(tick, status)};
#pragma unroll
        for (int f = 0; f < kRows; ++f)
          __builtin_amdgcn_raw_buffer_store_b32(vals[f], ro, (int32_t)vo[f], 0, AUX);
      } else {
        const int32_t vals[kRows] = {p1.x, p1.y, p1.d, p1.hp, p2.x, p2.y, p2.d, p2.hp,
                                     tick, status, p1.sx, p1.sy, p2.sx, p2.sy};
#pragma unroll
        for (int f = 0; f < kRows; ++f)
          __builtin_amdgcn_raw_buffer_store_b32(vals[f], ro, (int32_t)vo[f], 0, AUX);
      }
      if constexpr (ACT) {
        const auto ra = __builtin_amdgcn_make_buffer_rsrc(act, 0, (int32_t)(B * 2u),
                                                          kBufferDword3);
        __builtin_amdgcn_raw_buffer_store_b16(pack_actions(a1, a2), ra, (int32_t)va, 0, AUX);
      }
      skip();
    } else {
      if (obs) {
        if (fmt == ORX_OBS_COMPACT) {
          const uint32_t vals[ORX_OBS_COMPACT_FIELDS] = {
              cell8(p1.x, p1.y) | (cell8(p2.x, p2.y) << 16),
              cell8(p1.sx, p1.sy) | (cell8(p2.sx, p2.sy) << 16), compact_hp(p1.hp, p2.hp),
              (uint32_t)p1.d, (uint32_t)p2.d, compact_ts(tick, status)};
          uint32_t* o = reinterpret_cast<uint32_t*>(obs) + (size_t)t * ORX_OBS_COMPACT_FIELDS * B;
#pragma unroll
          for (int f = 0; f < ORX_OBS_COMPACT_FIELDS; ++f)
            __builtin_nontemporal_store(vals[f], (o + (size_t)f * B) + i);
        } else {
          const int32_t vals[ORX_OBS_FIELDS] = {p1.x, p1.y, p1.d, p1.hp, p2.x, p2.y, p2.d, p2.hp,
                                                tick, status, p1.sx, p1.sy, p2.sx, p2.sy};
          int32_t* o = obs + (size_t)t * ORX_OBS_FIELDS * B;  // uniform row base + lane index
#pragma unroll
          for (int f = 0; f < ORX_OBS_FIELDS; ++f)
            __builtin_nontemporal_store(vals[f], (o + (size_t)f * B) + i);
        }
      }
      if (act)
        __builtin_nontemporal_store(pack_actions(a1, a2),
                                    reinterpret_cast<uint16_t*>(act) + (size_t)t * B + i);
    }
  }
};

// PM (policy mode, compile-time): 0 generic; 1 both players RandomBot, obs
// and act given, no extension flags (the headline C3/C2 form); 2 both
// StaircaseBot, obs and act given, at most separation damage (C5); 3 both
// RandomBot, obs and act given, the character mechanics on (configs[2]'s
// "enemies + items": mana, experience and items, heal optional).  The
// specialized forms carry no per-tick uniform branches on policy codes or
// pointers and write the trajectory with buffer stores.
template <int NCAP, int PM, bool GRID, int AUX = kStreamAux, bool CF = false>
__global__ void __launch_bounds__(kRolloutBlock) rollout_kernel(orx_cfg_t hc, orx_state_t st,
                                                                int32_t pol1_,
                                                      int32_t pol2_, int32_t n_ticks,
                                                      int32_t* __restrict__ obs,
                                                      int8_t* __restrict__ act, uint32_t B,
                                                      Key key, uint32_t off, uint32_t lanes,
                                                      uint32_t lds_n, uint32_t lds_bits,
                                                      int32_t fmt) {
  constexpr bool kTraj = PM != 0;
  const int32_t pol1 = (PM == 1 || PM == 3) ? (int32_t)ORX_POLICY_RANDOM
                       : PM == 2 ? (int32_t)ORX_POLICY_STAIRCASE : pol1_;
  const int32_t pol2 = (PM == 1 || PM == 3) ? (int32_t)ORX_POLICY_RANDOM
                       : PM == 2 ? (int32_t)ORX_POLICY_STAIRCASE : pol2_;
  bool lds_tiles = false;
  if constexpr (GRID) {  // stage the bank's tiles in LDS (the whole block, before any exit)
    const uint32_t n = lds_n;  // the bank's bytes, or 0: not staged (too large, or disabled)
    if (n > 0u) {
      const uint8_t* src = st.bank_tiles;
      for (uint32_t k = threadIdx.x * 4u; k < n; k += blockDim.x * 4u) {
        if (k + 4u <= n) {
          uint32_t v;
          __builtin_memcpy(&v, src + k, 4);
          __builtin_memcpy(orx_lds_tiles + k, &v, 4);
        } else {
          for (uint32_t j = k; j < n; ++j) orx_lds_tiles[j] = src[j];
        }
      }
      __syncthreads();
      lds_tiles = true;
    }
  }
  uint32_t i = xcd_block() * blockDim.x + threadIdx.x;
  if (lanes < 64u) {  // uniform: lanes >= `lanes` of every wave idle
    if ((threadIdx.x & 63u) >= lanes) return;
    i = (i >> 6) * lanes + (threadIdx.x & 63u);
  }
  if (i >= B) return;
  Cfg c = make_cfg(hc, st);
  c.lds_tiles = lds_tiles;
  if (PM == 1) c.ext = 0;                           // launched only with flags == 0
  if (PM == 2) c.ext &= ORX_EXT_SEPARATION_DAMAGE;  // launched only with flags <= that
  // launched only with MANA, LEVELING and ITEMS on (HEAL is inert here: the
  // bots never heal), nothing else
  if (PM == 3) c.ext = ORX_EXT_MANA | ORX_EXT_LEVELING | ORX_EXT_ITEMS;
  const uint32_t game = off + i;
  ORX_STAMP(0);
  Player p1, p2;
  load_players<GRID>(st, B, i, p1, p2);
  int32_t tick = st.tick[i];
  int32_t status = st.status[i];
  uint32_t ep = (uint32_t)st.episode[i];
  Npcs<NCAP> npc;
  npc.bind(st, c, B, i);
  load_npcs(st, c, B, i, npc);
  if constexpr (NCAP == kDense) {
    // lds_bits: bytes of one game's occupancy bitmap (0: not staged), after
    // the bank's tiles; a lane's bitmap is its own (no barrier)
    if (lds_bits) {
      const uint32_t li = (threadIdx.x >> 6) * lanes + (threadIdx.x & 63u);
      npc.stage((((lds_n + 15u) & ~15u) + li * lds_bits) >> 2);
    }
  }
  // NPC health: registers, loaded and stored once per launch; the dense form's
  // rows stay in HBM
  std::conditional_t<NCAP == kDense, NpcMem, NpcHpRegs<NCAP>> hp;
  if constexpr (NCAP == kDense) hp = NpcMem{st.npc_pos, st.npc_health, B, i};
  else if constexpr (NCAP > 0) hp.load(st.npc_health, c.K, B, i);
  Items<NCAP> items;
  load_rpg(st, c, B, i, p1, p2, npc, items);
  Deltas dl = {0, 0, 0, 0, 0, 0};
  int32_t sep = (c.ext & ORX_EXT_SEPARATION_DAMAGE) ? st.sep_start[i] : -1;
  bool restarted = false;
  TrajWriter<kTraj, AUX, CF> traj(obs, act, B, i, fmt);
  // every state load resolved before the tick loop (pair_rollout_kernel)
  if constexpr (GRID) {
    launder(p1.x, p1.y, p1.d, p1.hp);
    launder(p2.x, p2.y, p2.d, p2.hp);
    launder(p1.sx, p1.sy, p2.sx, p2.sy);
    launder(p1.lay, p2.lay, tick, status);
    asm volatile("" : "+v"(sep), "+v"(ep));
  }
#ifdef ORX_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  ORX_STAMP(1);
  int32_t t = 0;
  // the FAST writers' exit test on the row pointer (a scalar register; a test
  // on t gets t a VGPR: 2 VALU a tick, as in pair_rollout_kernel)
  const int32_t* const obs_end =
      kTraj ? obs + (size_t)n_ticks * TrajWriter<kTraj, AUX, CF>::kRows * B : nullptr;
  do {  // n_ticks >= 1: orx_rollout returns before launching 0 ticks
#ifdef ORX_STAMPS
    if (t == 64) { ORX_STAMP(2); }
#endif
    int32_t a1 = ORX_MOVE_STAY, a2 = ORX_MOVE_STAY;
    if (!(ORX_DIAG & 32))
      rollout_tick<NCAP, GRID>(c, st, B, i, key, game, ep, pol1, pol2, p1, p2, npc, items, hp,
                               tick, status, dl, sep, restarted, a1, a2);
    if (!(ORX_DIAG & 16)) traj.write(t, p1, p2, tick, status, a1, a2);
    else if constexpr (kTraj) traj.skip();
    ++t;
  } while (kTraj ? traj.obs != obs_end : t < n_ticks);
  ORX_STAMP(3);
  store_players<GRID>(st, B, i, p1, p2, restarted || dl.descend != 0);
  store_rpg(st, c, B, i, p1, p2, npc, items);
  st.tick[i] = tick;
  st.status[i] = status;
  st.episode[i] = (int32_t)ep;
  if (c.ext & ORX_EXT_SEPARATION_DAMAGE) st.sep_start[i] = sep;
  if constexpr (NCAP > 0) {
    if (restarted || dl.npc_death) npc.store_alive(st.npc_alive, B, i);
    if constexpr (NCAP != kDense)
      if (restarted || dl.combat) hp.store(st.npc_health, c.K, B, i);
  }
  flush_deltas(st, B, i, dl);
#ifdef ORX_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  ORX_STAMP(4);
#ifdef ORX_STAMPS
  uint32_t r[11] = {dl.n_rare, dl.n_ordered, dl.n_hits, dl.n_desc, dl.n_meet, dl.n_reset,
                    dl.cy_rare, dl.cy_reset, dl.cy_ordered, dl.cy_desc, dl.n_lean};
#pragma unroll
  for (int j = 0; j < 11; ++j)
    for (int o = 32; o > 0; o >>= 1) r[j] += __shfl_xor(r[j], o);
  if ((threadIdx.x & 63) == 0) {
    const size_t w = (size_t)((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 16;
#pragma unroll
    for (int j = 0; j < 11; ++j) g_stamps[w + 5 + j] = r[j];
  }
#endif
}

// ---------------------------------------------------------------------------
// Paired rollout: two lanes per game
// ---------------------------------------------------------------------------
// A batch too small to fill the chip runs at most 32 games per wave (lanes =
// orx_rollout_lanes < 64), and a lone wave per SIMD pays per instruction, not
// per lane (a wave whose exec mask lies in its low 32 lanes issues each VALU
// instruction in one pass: DESIGN.md s7).  Without NPCs and dungeon banks
// (C5's StaircaseBots, C2's RandomBots) those idle lanes take the second
// player: lane 2j is player 1 of game j, lane 2j+1 its player 2, so the
// per-player half of the tick -- the bot's move, the target and its clamp,
// the staircase test, the common move, and half of the observation row's
// stores -- is ONE instruction stream for both players.  The pair exchanges
// the other player's cell, depth and target through DPP (quad_perm
// [1,0,3,2]: one VALU op each) for the meet test, which is symmetric, so both
// lanes reach the same decision.  A rare tick rebuilds the game's two Player
// records in BOTH lanes and runs rollout_tick's scalar rare block (rare_tick)
// redundantly -- the same instructions in two lanes cost what one lane costs
// -- so every rare case keeps the single-lane form's exact semantics; each
// lane then keeps its own player.  Game-level state (tick, status, episode,
// separation timer, counters) is identical in both lanes; lane 2j writes it.
__device__ __forceinline__ int32_t pair_swap(int32_t v) {
  return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);  // quad_perm [1, 0, 3, 2]
}

// The paired common path's exchange terms, each ONE VOP2 instruction whose
// DPP source operand reads the other lane (quad_perm [1,0,3,2]) instead of a
// v_mov_b32_dpp and the op: swap(kp) ^ kt, swap(kt) ^ kp, swap(kt) ^ kt and
// swap(d) ^ d for the meet test; min(swap(z), z) for the staircase / NPC test.
// (The compiler fuses such xors into three-input v_bitop3, which takes no DPP
// operand on gfx950, so they are written out; the leading s_nop 1 gives the
// two wait states a DPP read needs after a VALU write of its source.)
__device__ __forceinline__ void meet_terms(uint32_t kp, uint32_t kt, uint32_t d, uint32_t& e_mo,
                                           uint32_t& e_om, uint32_t& e_tt, uint32_t& e_d) {
  asm("s_nop 1\n"
      "v_xor_b32_dpp %0, %4, %5 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_xor_b32_dpp %1, %5, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_xor_b32_dpp %2, %5, %5 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_xor_b32_dpp %3, %6, %6 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
      : "=&v"(e_mo), "=&v"(e_om), "=&v"(e_tt), "=&v"(e_d)
      : "v"(kp), "v"(kt), "v"(d));
}
__device__ __forceinline__ uint32_t min_swapped(uint32_t z) {
  uint32_t r;
  asm("s_nop 1\n"
      "v_min_u32_dpp %0, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
      : "=v"(r) : "v"(z));
  return r;
}
__device__ __forceinline__ uint32_t pack_cell(int32_t x, int32_t y) {
  return (uint32_t)x | ((uint32_t)y << 8);  // the NPC slots' key form (x, y < 256)
}

// One tick's trajectory rows from a pair of lanes: each lane stores its own
// player's x, y, depth, health and staircase (rows f and f + 4, 10/11 and
// 12/13), lane 2j the tick and lane 2j+1 the status (rows 8 and 9), and its
// own action byte: 7 dword stores and one byte store per tick, each covering
// two rows, instead of 14 and a 16-bit store.
// CF (ORX_OBS_COMPACT): three dword rows per lane -- lane 2j the cells (row 0),
// player 1's depth (3) and tick | status << 27 (5), lane 2j+1 the staircases
// (1), player 2's depth (4) and the healths (2) -- each cell pair and health
// pair assembled from the lane's own value and its partner's (DPP).
template <int AUX, bool CF = false, bool ACT = true>
struct PairWriter {
  static constexpr int kStores = CF ? 3 : 7;
  static constexpr int kRows = CF ? ORX_OBS_COMPACT_FIELDS : ORX_OBS_FIELDS;
  int32_t* obs;
  int8_t* act;
  uint32_t B;
  uint32_t vo[kStores], va;
  __device__ __forceinline__ PairWriter(int32_t* o, int8_t* a, uint32_t B_, uint32_t i,
                                        uint32_t who)
      : obs(o), act(a), B(B_) {
    if constexpr (CF) {
      const uint32_t rows[3] = {who, 3u + who, who ? 2u : 5u};
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        vo[k] = (rows[k] * B + i) * 4u;
        asm volatile("" : "+v"(vo[k]));
      }
    } else {
      const uint32_t rows[7] = {0u + 4u * who, 1u + 4u * who, 2u + 4u * who, 3u + 4u * who,
                                (uint32_t)ORX_OBS_TICK + who,
                                (uint32_t)ORX_OBS_P1_STAIR_X + 2u * who,
                                (uint32_t)ORX_OBS_P1_STAIR_Y + 2u * who};
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        vo[k] = (rows[k] * B + i) * 4u;
        asm volatile("" : "+v"(vo[k]));
      }
    }
    va = 2u * i + who;
    asm volatile("" : "+v"(va));
  }
  // me: this lane's player; kp / ks: its cell and staircase as x | y << 8
  // (compact only); tick and status: the game's (identical in both lanes)
  __device__ __forceinline__ void write(const Player& me, uint32_t kp, uint32_t ks, bool isB,
                                        int32_t tick, int32_t status, int32_t move) {
    const auto ro = __builtin_amdgcn_make_buffer_rsrc(obs, 0, (int32_t)(kRows * B * 4u),
                                                      kBufferDword3);
    if constexpr (CF) {
      // lane 2j assembles the cells, so it takes its partner's cell; lane
      // 2j+1 the staircases, so it takes its partner's staircase: each lane
      // offers its partner what the partner assembles
      const uint32_t a = isB ? ks : kp, give = isB ? kp : ks;
      const uint32_t sw = (uint32_t)pair_swap((int32_t)give);
      const uint32_t lo = isB ? sw : a, hi = isB ? a : sw;
      const int32_t ohp = pair_swap(me.hp);
      const uint32_t vals[3] = {lo | (hi << 16), (uint32_t)me.d,
                                isB ? compact_hp(ohp, me.hp) : compact_ts(tick, status)};
#pragma unroll
      for (int k = 0; k < 3; ++k)
        __builtin_amdgcn_raw_buffer_store_b32(vals[k], ro, (int32_t)vo[k], 0, AUX);
    } else {
      const int32_t vals[7] = {me.x, me.y, me.d, me.hp, isB ? status : tick, me.sx, me.sy};
#pragma unroll
      for (int k = 0; k < 7; ++k)
        __builtin_amdgcn_raw_buffer_store_b32(vals[k], ro, (int32_t)vo[k], 0, AUX);
    }
    if constexpr (ACT) {
      const auto ra = __builtin_amdgcn_make_buffer_rsrc(act, 0, (int32_t)(B * 2u), kBufferDword3);
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)move, ra, (int32_t)va, 0, AUX);
    }
    skip();
  }
  __device__ __forceinline__ void skip() {  // the next tick's rows
    obs += (size_t)kRows * B;
    if constexpr (ACT) act += (size_t)2 * B;
  }
};

// PM 1: both players RandomBot (no extension flags); PM 2: both StaircaseBot
// (at most separation damage).  NCAP 0 / 8 / 16 (register NPCs, no dense
// grid), empty dungeons, obs and act given.  The bench's C3 shards run
// pair_rollout_kernel<8, 1, 2, false>.
// PM 6 (round 6): a replay of a move log (orx_step_n; flags 0, empty
// dungeons, observation rows given) -- each lane's move is its player's byte
// of `act`, which is then the log [n_ticks][B][2] (read, never written; no
// action rows are stored: the log is the actions); a pair outside the Move
// codes stops the game in the rare block (orx_step's rule), and the
// initiative block is drawn only by a rare tick that needs the order.
// (diagnostic builds may add attributes, e.g. an occupancy target)
#ifndef ORX_PAIR_ATTR
#define ORX_PAIR_ATTR
#endif
// the StaircaseBot form with separation damage held to four waves per SIMD
// (128 VGPRs; 131 otherwise, three waves): C5's 131,072 games as two paired
// shards are four 32-game waves per SIMD
#ifndef ORX_SEP_WAVES
#define ORX_SEP_WAVES 1
#endif
// GRID (round 4): a dungeon bank -- each lane reads its target's tile (its
// player's layout; LDS-staged when the bank fits, lds_n bytes), a Wall or the
// grid's edge blocks, ANY staircase tile makes the tick rare; descends and
// resets take rare_tick's bank forms (the closed-form fast paths are for
// empty dungeons).
// The paired rollout's fallback rare tick, out of line (-DORX_RARE_OUTLINE=1,
// build variant `routl`; measured and rejected): its state goes through a
// stack frame on the (rare) call, so the common tick and the lean rare
// branches would not carry the merges of an inlined rare_tick's values.  The
// call makes the kernel take the callee's registers (196-248 VGPRs, two
// waves per SIMD) and 464-788 B of scratch per lane, and every paired form
// slows by a third or more (C3 85 -> 110 us, c3_mixed 155 -> 243, C5's share
// 64 -> 102; profiles/r06_v7/ab_rare_outline_rejected.jsonl).
#ifndef ORX_RARE_OUTLINE
#define ORX_RARE_OUTLINE 0
#endif
template <int NCAP, bool GRID, class M>
__device__ __noinline__ bool rare_tick_ool(const Cfg c, const orx_state_t st, uint32_t B,
                                           uint32_t i, Key key, uint32_t game, uint32_t& ep,
                                           Player& p1, Player& p2, Npcs<NCAP>& npc,
                                           Items<NCAP>& items, M& hp, int32_t& tick,
                                           int32_t& status, Deltas& dl, int32_t& sep,
                                           bool& restarted, const W4 tb, int need, int32_t t1x,
                                           int32_t t1y, int32_t t2x, int32_t t2y) {
  return rare_tick<NCAP, GRID>(c, st, B, i, key, game, ep, p1, p2, npc, items, hp, tick, status,
                               dl, sep, restarted, tb, need, t1x, t1y, t2x, t2y, false);
}

template <int NCAP, int PM, int AUX, bool SEP, bool CF = false, bool GRID = false>
__global__ void __launch_bounds__(GRID ? 512 : kRolloutBlock) ORX_PAIR_ATTR
    __attribute__((amdgpu_waves_per_eu(ORX_SEP_WAVES && PM == 2 && SEP ? 4 : 1)))
    pair_rollout_kernel(orx_cfg_t hc, orx_state_t st,
                                                                     int32_t n_ticks,
                                                                     int32_t* __restrict__ obs,
                                                                     int8_t* __restrict__ act,
                                                                     uint32_t B, Key key,
                                                                     uint32_t off, uint32_t lanes,
                                                                     uint32_t lds_n) {
  bool lds_tiles = false;
  if constexpr (GRID) {  // stage the bank's tiles in LDS (the whole block, before any exit)
    if (lds_n > 0u) {
      const uint8_t* src = st.bank_tiles;
      for (uint32_t k = threadIdx.x * 4u; k < lds_n; k += blockDim.x * 4u) {
        if (k + 4u <= lds_n) {
          uint32_t v;
          __builtin_memcpy(&v, src + k, 4);
          __builtin_memcpy(orx_lds_tiles + k, &v, 4);
        } else {
          for (uint32_t j = k; j < lds_n; ++j) orx_lds_tiles[j] = src[j];
        }
      }
      __syncthreads();
      lds_tiles = true;
    }
  }
  const uint32_t lane = threadIdx.x & 63u;
  if (lane >= 2u * lanes) return;  // uniform per wave
  const uint32_t i = ((xcd_block() * blockDim.x + threadIdx.x) >> 6) * lanes + (lane >> 1);
  if (i >= B) return;              // both lanes of a game together
  const uint32_t who = lane & 1u;  // 0: player 1, 1: player 2
  const bool isB = who != 0u;
  Cfg c = make_cfg(hc, st);
  // PM 1: no extension; PM 2: at most separation damage; PM 3: mana,
  // experience and items (HEAL is inert: the bots never heal)
  c.ext = PM == 3 ? (ORX_EXT_MANA | ORX_EXT_LEVELING | ORX_EXT_ITEMS)
                  : SEP ? ORX_EXT_SEPARATION_DAMAGE : 0;
  c.lds_tiles = lds_tiles;
  const uint32_t game = off + i;
  ORX_STAMP(0);
  Player me;
  me.x = st.p_x[who * B + i];
  me.y = st.p_y[who * B + i];
  me.d = st.p_depth[who * B + i];
  me.hp = st.p_health[who * B + i];
  me.sx = st.st_x[who * B + i];
  me.sy = st.st_y[who * B + i];
  me.lay = GRID ? st.p_layout[who * B + i] : -1;
  me.move = ORX_MOVE_STAY;
  me.tx = me.ty = 0;
  me.mana = me.xp = me.dmg = me.mhp = me.nitems = me.cool = me.heal = me.hd = 0;
  if constexpr (PM == 3) {  // this lane's player's attributes (p_rpg [field][2][B])
    const int32_t* r = st.p_rpg + who * B + i;
    const size_t f = 2 * (size_t)B;
    me.mana = r[ORX_RPG_MANA * f];
    me.xp = r[ORX_RPG_XP * f];
    me.dmg = r[ORX_RPG_DAMAGE * f];
    me.mhp = r[ORX_RPG_MAX_HEALTH * f];
    me.nitems = r[ORX_RPG_ITEMS * f];
  }
  uint32_t kp = pack_cell(me.x, me.y), ks = pack_cell(me.sx, me.sy);  // packed cells
  uint32_t dk = me.d == c.d1 ? 0u : 0x80008000u;  // off the NPCs' depth (npc_any1_dk)
  int32_t tick = st.tick[i];
  int32_t status = st.status[i];
  uint32_t ep = (uint32_t)st.episode[i];
  int32_t sep = SEP ? st.sep_start[i] : -1;
  // NPCs (register slots): the game's in both lanes, kept identical -- every
  // change to them happens in the rare block, which both lanes run
  Npcs<NCAP> npc;
  npc.bind(st, c, B, i);
  load_npcs(st, c, B, i, npc);
  NpcHpRegs<NCAP> hp;
  if constexpr (NCAP > 0) hp.load(st.npc_health, c.K, B, i);
  Items<NCAP> items;
  items.clear();
  if constexpr (PM == 3 && NCAP > 0) {  // the game's items, in their NPCs' slots (both lanes)
    items.on = st.item_mask[i];
    items.kind = st.item_mask[B + i];
    for (int k = 0; k < c.K; ++k)
      if ((items.on >> k) & 1u) npc.set(k, st.item_pos[(size_t)k * B + i]);
  }
  Deltas dl = {0, 0, 0, 0, 0, 0};
  bool restarted = false;
  // PM 4 / 5 (round 5): one RandomBot and one StaircaseBot -- 4: player 1
  // is the RandomBot, 5: player 2 -- (a learner's baseline evaluation);
  // the RandomBot lane takes the tick block's first accepted field, as
  // rollout_tick's single random player
  constexpr bool kMixed = PM == 4 || PM == 5;
  constexpr bool kLog = PM == 6;
  const bool rb_lane = kMixed && (isB == (PM == 5));
  constexpr int need = (PM == 1 || PM == 3) ? 2 : kMixed ? 1 : 0;
  PairWriter<AUX, CF, !kLog> traj(obs, act, B, i, who);
  const int32_t* const obs_end = obs + (size_t)n_ticks * PairWriter<AUX, CF, !kLog>::kRows * B;
  // PM 6: this lane's byte of the log, the next tick's prefetched while this
  // tick runs (the last tick re-reads its own instead of branching)
  const int8_t* const lg = act + 2u * i + who;
  int32_t a_next = 0;
  if constexpr (kLog) {
    a_next = lg[0];
    asm volatile("" : "+v"(a_next));
  }
  // every state load resolved before the tick loop: a value first read in the
  // loop leaves its load pending at the loop head, and that wait then also
  // covers the previous ticks' row stores (vmcnt counts both) -- each tick
  launder(me.x, me.y, me.d, me.hp);
  launder(me.sx, me.sy, me.lay, tick);
  launder(status, sep, me.mana, me.xp);
  launder(me.dmg, me.mhp, me.nitems, reinterpret_cast<int32_t&>(ep));
#ifdef ORX_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  ORX_STAMP(1);
  // Lean spans (StaircaseBots on an empty dungeon, C5): both bots walk
  // greedily to their staircases, so a game's next ticks are plain moves until
  // a player's target is its staircase (its distance to it, less one), the
  // two could meet (same depth: the distance between them shrinks by at most
  // 2 a tick, a meet needs at most 2), the episode ends or, with separation
  // damage across depths, the next tick's damage would kill.  `span` counts
  // those ticks from the state a general tick leaves; while every game of the
  // wave has one left, the wave runs lean ticks: the move, the step, the
  // separation damage (its ceil(k / period) carried as quotient and remainder,
  // no division) and the row, nothing else.
  constexpr bool kLean = ORX_LEAN && PM == 2 && NCAP == 0 && !GRID && (ORX_DIAG & (16 | 32 | 64 | 128)) == 0;
  // split tick blocks (ORX_SPLIT_TICK): the held block of the next tick and
  // its key (episode, tick); n_tick -1: none held
  constexpr bool kSplit = PM == 1 && (ORX_DIAG & 64) == 0 &&
                          (ORX_SPLIT_TICK == 2 || (ORX_SPLIT_TICK == 1 && CF));
  W4 nb = {0u, 0u, 0u, 0u};
  uint32_t nh0 = 0u, nh3 = 0u, n_ep = 0u;
  int32_t n_tick = -1;
  int32_t span = 0;
  int32_t l_od = 0, l_q = 0, l_r = 0;  // SEP: the other's depth; the next tick's damage and phase
  int32_t t = 0;
  do {
#ifdef ORX_STAMPS
    if (t == 64) { ORX_STAMP(2); }
#endif
    if constexpr ((ORX_DIAG & 32) != 0) {  // diagnostic: the trajectory stores alone
      tick += 1;
      traj.write(me, kp, ks, isB, tick, status, ORX_MOVE_STAY);
      continue;
    }
    if constexpr (kLean) {
      // the lean ticks as a loop of their own (its values stay in the tick
      // loop's registers: no copies at a join with the general tick)
      if (__builtin_amdgcn_ballot_w64(span <= 0) == 0) {  // uniform
        do {
          const int32_t dx = me.sx - me.x, dy = me.sy - me.y;
          const int32_t adx = dx < 0 ? -dx : dx, ady = dy < 0 ? -dy : dy;
          const int32_t mv = adx > ady ? (dx > 0 ? ORX_MOVE_RIGHT : ORX_MOVE_LEFT)
                                       : (dy > 0 ? ORX_MOVE_DOWN : ORX_MOVE_UP);
          calc_pos(me.x, me.y, mv, me.x, me.y);
          span -= 1;
          if constexpr (SEP) {  // as the common tick's block (readme.md:46-47)
            if (me.d != l_od) {
              sep = sep < 0 ? tick : sep;
              const bool shallow = me.d < l_od;
              me.hp -= shallow ? l_q : 0;  // ceil(k / period), k = t0 - sep + 1
              const bool wrap = l_r + 1 == c.sep_period;
              l_q += wrap ? 1 : 0;
              l_r = wrap ? 0 : l_r + 1;
              if (shallow & (me.hp - l_q <= 0)) span = 0;  // the next tick's damage kills
            } else {
              sep = -1;
            }
          }
          tick += 1;
#ifdef ORX_STAMPS
          ORX_COUNT(dl.n_lean);
#endif
          traj.write(me, pack_cell(me.x, me.y), ks, isB, tick, status, mv);
        } while (++t < n_ticks && __builtin_amdgcn_ballot_w64(span <= 0) == 0);
        kp = pack_cell(me.x, me.y);
        if (t >= n_ticks) break;
      }
    }
    // the bot's move (randombot.py:20-21 / staircasebot.py:9-21)
    W4 tb = {0u, 0u, 0u, 0u};
    uint32_t h0 = 0u, h3 = 0u;  // PM 1: the tick block's deferred words c, d
    int32_t move;
    if constexpr (PM == 1 || PM == 3) {
      // the tick block in both lanes; player 1 takes the first accepted 3-bit
      // field of word b, player 2 the second (as rollout_tick)
      if constexpr ((ORX_DIAG & 64) != 0) {  // diagnostic: a cheap hash for the tick block
        const uint32_t hsh = (game * 0x9E3779B9u) ^ ((uint32_t)tick * 0x85EBCA6Bu) ^ ep;
        tb = W4{hsh * 0xC2B2AE35u, hsh ^ (hsh >> 15), 0u, 0u};
      } else if constexpr (kSplit) {
        const bool have = (ep == n_ep) & (tick == n_tick);
        if (__builtin_amdgcn_ballot_w64(!have) == 0) {  // uniform: every game holds its block
          tb = nb;
          h0 = nh0;
          h3 = nh3;
          n_tick = -1;
        } else {  // one pass for two ticks: lane 2j this tick's block, lane 2j+1 the next's
          uint32_t m0, m3;
          const W4 m = philox_ab(game, ep, (uint32_t)(tick + (int32_t)who), tag(PUR_TICK, 0),
                                 key, m0, m3);
          const uint32_t oa = (uint32_t)pair_swap((int32_t)m.a), ob = (uint32_t)pair_swap((int32_t)m.b);
          const uint32_t o0 = (uint32_t)pair_swap((int32_t)m0), o3 = (uint32_t)pair_swap((int32_t)m3);
          tb = W4{isB ? oa : m.a, isB ? ob : m.b, 0u, 0u};
          h0 = isB ? o0 : m0;
          h3 = isB ? o3 : m3;
          nb = W4{isB ? m.a : oa, isB ? m.b : ob, 0u, 0u};
          nh0 = isB ? m0 : o0;
          nh3 = isB ? m3 : o3;
          n_ep = ep;
          n_tick = tick + 1;
        }
      } else {
        tb = philox_ab(game, ep, (uint32_t)tick, tag(PUR_TICK, 0), key, h0, h3);
      }
      const uint32_t acc = accepted3(tb.b);
      const uint32_t acc2 = acc & (acc - 1u);
      // (v_bfe_u32 reads its offset's low 5 bits: ffbl's 0xFFFFFFFF for an
      // empty mask needs no mask, the value is then replaced below)
      move = (int32_t)__builtin_amdgcn_ubfe(tb.b, ffbl(isB ? acc2 : acc), 3u) + 1;
      if (ORX_UNLIKELY(acc2 == 0u)) {  // the game's word b holds fewer than two
        int32_t r0 = ORX_MOVE_STAY, r1 = ORX_MOVE_STAY;
        bool err = false;
        finish_cd(tb, h0, h3, key);
        moves_from_block(tb, 2, key, game, ep, tick, r0, r1, err);
        move = isB ? r1 : r0;
      }
    } else if constexpr (kMixed) {
      tb = philox_ab(game, ep, (uint32_t)tick, tag(PUR_TICK, 0), key, h0, h3);
      const uint32_t acc = accepted3(tb.b);
      const int32_t rmove = (int32_t)__builtin_amdgcn_ubfe(tb.b, ffbl(acc), 3u) + 1;
      const int32_t dx = me.sx - me.x, dy = me.sy - me.y;
      const int32_t adx = dx < 0 ? -dx : dx, ady = dy < 0 ? -dy : dy;
      const int32_t smove = adx > ady ? (dx > 0 ? ORX_MOVE_RIGHT : ORX_MOVE_LEFT)
                                      : (dy > 0 ? ORX_MOVE_DOWN : ORX_MOVE_UP);
      move = rb_lane ? rmove : smove;
      if (ORX_UNLIKELY(acc == 0u)) {  // the game's word b holds no accepted field
        int32_t r0 = ORX_MOVE_STAY, r1 = ORX_MOVE_STAY;
        bool err = false;
        finish_cd(tb, h0, h3, key);
        moves_from_block(tb, 1, key, game, ep, tick, r0, r1, err);
        move = rb_lane ? r0 : smove;
      }
    } else if constexpr (kLog) {
      move = a_next;
      a_next = lg[(size_t)(t + 1 < n_ticks ? t + 1 : t) * 2u * B];
    } else {
      const int32_t dx = me.sx - me.x, dy = me.sy - me.y;
      const int32_t adx = dx < 0 ? -dx : dx, ady = dy < 0 ? -dy : dy;
      move = adx > ady ? (dx > 0 ? ORX_MOVE_RIGHT : ORX_MOVE_LEFT)
                       : (dy > 0 ? ORX_MOVE_DOWN : ORX_MOVE_UP);
    }
    // PM 6: a pair outside the Move codes stops the game (rare); its
    // targets are computed as Stays
    bool bad = false;
    if constexpr (kLog) {
      const bool ok_me = (uint32_t)(move - ORX_MOVE_UP) <= (uint32_t)(ORX_MOVE_STAY - ORX_MOVE_UP);
      bad = (status == ORX_IN_PROGRESS) & !(ok_me & (pair_swap(ok_me ? 1 : 0) != 0));
      move = ok_me ? move : ORX_MOVE_STAY;
    }
    me.move = move;
    const bool in_progress = status == ORX_IN_PROGRESS && !bad;
    // effective target (own cell when blocked: the border, clamped)
    int32_t tx, ty;
    calc_pos(me.x, me.y, move, tx, ty);
    bool st_tile = false;  // GRID: the target tile is a staircase
    bool hit_me = false;   // an NPC on my target
    if constexpr (GRID) {
      // one tile read: a Wall or the grid's edge blocks (a blocked player's
      // own cell is never a staircase)
      const bool in = (uint32_t)tx < (uint32_t)c.W && (uint32_t)ty < (uint32_t)c.H;
      const int32_t cx = in ? tx : me.x, cy = in ? ty : me.y;
      const uint32_t tile = bank_tile_lds(c, me.lay, cx, cy);  // (staged: plan_rollout)
      // the NPC test on the in-grid cell while the tile read is in flight (a
      // blocked move's target is the player's own cell, which holds no NPC)
      if constexpr (NCAP > 0) hit_me = npc_any1_dk(npc, pack_cell(cx, cy), dk);
      const bool blk = !in || tile == ORX_TILE_WALL;
      hit_me = hit_me & !blk;
      st_tile = !blk && tile == ORX_TILE_STAIRCASE_DOWN;
      tx = blk ? me.x : tx;
      ty = blk ? me.y : ty;
    } else {
      tx = med3_1(tx, c.W - 2);
      ty = med3_1(ty, c.H - 2);
    }
    const uint32_t kt = pack_cell(tx, ty);
    // The rare test on packed cells (x | y << 8): a meet is both players on
    // one depth with my target on the other's cell, the other's target on
    // mine, or one target for both -- symmetric, so both lanes decide alike
    // -- and either player's target holding its staircase or an NPC (NPC keys
    // x | y << 8, all NPCs on depth d1).  Each term reads the other lane
    // through its own DPP source operand.
    uint32_t e_mo, e_om, e_tt, e_d;
    meet_terms(kp, kt, (uint32_t)me.d, e_mo, e_om, e_tt, e_d);
    const uint32_t mt = min(e_mo, min(e_om, e_tt)) | e_d;  // 0: a meet
    if constexpr (NCAP > 0 && !GRID) hit_me = npc_any1_dk(npc, kt, dk);
    // 0: my staircase (GRID: any staircase tile) or an NPC on my target
    const uint32_t z = (hit_me | st_tile) ? 0u : GRID ? 1u : (kt ^ ks);
    // (ORX_DIAG & 128: no rare block -- an ISA census of the common tick only,
    // never run)
    const bool rare = (ORX_DIAG & 128) ? false : (!in_progress | (min(mt, min_swapped(z)) == 0u));
    // (PM 6: a bad pair is !in_progress with status still InProgress)
    const int32_t ft = tick + 1;
    const bool end = c.max_ticks && ft >= c.max_ticks;
    bool took_ordered = false;
    if (ORX_UNLIKELY(rare)) {
#ifdef ORX_STAMPS
      ORX_COUNT(dl.n_rare);
      ORX_CYC_BEGIN(cy0);
#endif
      if constexpr (PM == 1 || PM == 3 || kMixed) {  // the tick block's words c, d (rare_tick's fallbacks)
        asm volatile("" : "+v"(h0), "+v"(h3));
        finish_cd(tb, h0, h3, key);
      }
      // The pre-tick cell and tick, rebuilt from kp and ft: the common path
      // then needs neither past its target and the next tick's values take
      // their registers (no copies at the loop's back edge).
      {
        uint32_t k0 = kp;
        int32_t f0 = ft;
        asm volatile("" : "+v"(k0), "+v"(f0));
        me.x = (int32_t)(k0 & 0xFFu);
        me.y = (int32_t)(k0 >> 8);
        tick = f0 - 1;
      }
      // the terms one by one, from laundered copies (the common path's
      // swaps stay folded into their ops)
      int32_t lx = me.x, ly = me.y, ld = me.d, ltx = tx, lty = ty, lsx = me.sx, lsy = me.sy;
      launder(lx, ly, ld, ltx);
      asm volatile("" : "+v"(lty), "+v"(lsx), "+v"(lsy));
      const int32_t ox = pair_swap(lx), oy = pair_swap(ly), od = pair_swap(ld);
      const int32_t otx = pair_swap(ltx), oty = pair_swap(lty);
      const bool meet = mt == 0u;
      bool st_me = (ltx == lsx) & (lty == lsy);
      if constexpr (GRID) {
        int32_t sl = st_tile ? 1 : 0;
        asm volatile("" : "+v"(sl));
        st_me = sl != 0;
      }
      const int32_t st_o = pair_swap(st_me ? 1 : 0);
      const int32_t hit_o = pair_swap(hit_me ? 1 : 0);
      // One player descends (C5's common rare tick; StaircaseBots only),
      // fast_descend's rules split over the pair: the descender's lane draws the tick's SPAWN
      // block, the other lane the new depth's DUNGEON block -- one Philox
      // instruction stream for both -- and the lanes swap them.
      bool fast = false;
      const int32_t osx = pair_swap(me.sx), osy = pair_swap(me.sy);
      if constexpr (kLog) {
        if (bad) {  // orx_step's rule: the game stops, nothing else changes
          status = ORX_STATUS_BAD_ACTION;
          fast = true;
        }
        // the initiative bits for a meet (the lean meet below; the ordered
        // tick draws them itself)
        if (meet & !bad) tb.a = tick_block(key, game, ep, tick).a;
      }
      if constexpr ((PM == 2 || kMixed || kLog) && NCAP == 0 && !GRID) {
        if (!in_progress & !bad & (c.autoreset != 0)) {  // uniform over the pair
          // The next episode (setup_game's keyed first-block form), its two
          // starting dungeons split over the pair: each lane draws its own
          // player's DUNGEON block beside the INIT block, and the lanes swap
          // staircases (Together: both draw depth 0's).  Anything the first
          // blocks do not settle takes the general form below.
          const uint32_t ep1 = ep + 1u;
          const bool sepm = c.start_mode == ORX_START_SEPARATED;
          const int32_t dme = sepm ? (isB ? c.d2 : c.d1) : 0;
          W4 wd = philox(game, ep1, (uint32_t)dme, tag(PUR_DUNGEON, 0), key);
          W4 wi = philox(game, ep1, 0u, tag(PUR_INIT, 0), key);
          launder_w4(wd);
          launder_w4(wi);
          int32_t sx, sy;
          const bool okd = stair_from_block(c, wd, sx, sy);
          const int32_t osx1 = pair_swap(sx), osy1 = pair_swap(sy);
          const int32_t s1x = isB ? osx1 : sx, s1y = isB ? osy1 : sy;
          const int32_t s2x = isB ? sx : osx1, s2y = isB ? sy : osy1;
          // both players from the INIT block's four words, as setup_game
          const NpBound g = c.ground;
          int n = 0;
          int32_t x1 = 0, y1 = 0, x2 = 0, y2 = 0;
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t word = j == 0 ? wi.a : j == 1 ? wi.b : j == 2 ? wi.c : wi.d;
            const bool is_p2 = n == 1;
            const uint32_t v = word & g.mask;
            int32_t x, y;
            ground_cell<false>(c, v, -1, is_p2 ? s2x : s1x, is_p2 ? s2y : s1y, x, y);
            const bool take = n < 2 && v <= g.rng && !(is_p2 && !sepm && x == x1 && y == y1);
            x1 = (take && n == 0) ? x : x1;
            y1 = (take && n == 0) ? y : y1;
            x2 = (take && is_p2) ? x : x2;
            y2 = (take && is_p2) ? y : y2;
            n += take ? 1 : 0;
          }
          const bool ok = okd & (pair_swap(okd ? 1 : 0) != 0) & (n == 2) & (g.rng != 0u);
          if (ok) {
            ep = ep1;
            me.d = dme;
            me.sx = sx;
            me.sy = sy;
            me.x = isB ? x2 : x1;
            me.y = isB ? y2 : y1;
            me.hp = c.player_hp;
            tick = kStartTick;
            status = ORX_IN_PROGRESS;
            sep = -1;
            restarted = true;
            fast = true;
#ifdef ORX_STAMPS
            ORX_COUNT(dl.n_reset);
#endif
          }
        }
      }
      if constexpr ((PM == 1 || kMixed || kLog) && NCAP > 0) {
        // NPC hits without a meet or a staircase (C3's common rare tick): the
        // attackers stay, the other player moves; both lanes apply both hits
        // to their identical NPC registers (npc_hits: order-free without the
        // character mechanics, which PM 1 excludes)
        if (in_progress & !meet & !st_me & (st_o == 0) & (hit_me | (hit_o != 0))) {
          const uint32_t kme = (uint32_t)tx | ((uint32_t)ty << 8);
          const int h_me = hit_me ? npc.find(kme) : -1;
          const int h_o = pair_swap(h_me);
          const uint32_t k_o = (uint32_t)pair_swap((int32_t)kme);
          const int h1 = isB ? h_o : h_me, h2 = isB ? h_me : h_o;
          const int32_t dmg = c.player_dmg_net > 0 ? c.player_dmg_net : 0;
          Events<false> ev{nullptr, 0};
          bool k1 = false, k2 = false;
          dl.combat += (h1 >= 0 ? 1 : 0) + (h2 >= 0 ? 1 : 0);
          npc_hits(c, npc, hp, h1, h2, dmg, dmg, dl, ev, k1, k2, isB ? k_o : kme,
                   isB ? kme : k_o);
          me.x = hit_me ? me.x : tx;
          me.y = hit_me ? me.y : ty;
          dl.eps += end ? 1 : 0;
          tick = ft;
          status = end ? ORX_TIE : ORX_IN_PROGRESS;
          fast = true;
#ifdef ORX_STAMPS
          ORX_COUNT(dl.n_hits);
#endif
        }
      }
      if constexpr (PM == 3 && NCAP > 0) {
        // The character mechanics' common rare tick: NPC hits and steps onto
        // items without a meet or a staircase (rare_tick's rules, in its
        // order: moves, hits, the kills' drops, experience, pickups).  Each
        // lane spends its own player's mana on its own hit and takes its own
        // item; both lanes apply both hits, drops and pickups to their
        // identical NPC and item registers (no meet: the two targets differ,
        // so the hits are order-free).
        if (in_progress & !meet & !st_me & (st_o == 0) & (hit_me | (hit_o != 0))) {
          const uint32_t kme = pack_cell(tx, ty);
          const int s_me = hit_me ? npc.find(kme) : -1;
          const bool item_me = s_me >= 0 && ((items.on >> s_me) & 1u) != 0u;
          const int h_me = item_me ? -1 : s_me;                    // the NPC I attack
          const int32_t d_me = h_me >= 0 ? rpg_attack(c, me) : 0;  // my damage and mana
          const int h_o = pair_swap(h_me);
          const int32_t d_o = pair_swap(d_me);
          const uint32_t k_o = (uint32_t)pair_swap((int32_t)kme);
          const int h1 = isB ? h_o : h_me, h2 = isB ? h_me : h_o;
          const uint32_t key1 = isB ? k_o : kme, key2 = isB ? kme : k_o;
          Events<false> ev{nullptr, 0};
          bool k1 = false, k2 = false;
          dl.combat += (h1 >= 0 ? 1 : 0) + (h2 >= 0 ? 1 : 0);
          npc_hits(c, npc, hp, h1, h2, isB ? d_o : d_me, isB ? d_me : d_o, dl, ev, k1, k2, key1,
                   key2);
          if (k1) drop_item(c, key, game, ep, tick, h1, key1, npc, items);
          if (k2) drop_item(c, key, game, ep, tick, h2, key2, npc, items);
          if (isB ? k2 : k1) gain_xp(c, me);
          me.x = h_me >= 0 ? me.x : tx;  // attackers stay
          me.y = h_me >= 0 ? me.y : ty;
          // pickups, player 1's then player 2's (a free item spot takes it)
          const int p_me = (item_me && me.nitems < c.item_slots) ? s_me : -1;
          const int p_o = pair_swap(p_me);
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const bool mine = (j == 1) == isB;
            const int k = mine ? p_me : p_o;
            if (k >= 0) {
              const bool health_item = ((items.kind >> k) & 1u) != 0u;
              items.on &= ~(1u << k);
              items.kind &= ~(1u << k);
              npc.kill(k);
              if (mine) {
                me.nitems += 1;
                me.mhp += health_item ? c.item_bonus : 0;
                me.hp += health_item ? c.item_bonus : 0;
                me.dmg += health_item ? 0 : c.item_bonus;
              }
            }
          }
          dl.eps += end ? 1 : 0;
          tick = ft;
          status = end ? ORX_TIE : ORX_IN_PROGRESS;
          fast = true;
#ifdef ORX_STAMPS
          ORX_COUNT(dl.n_hits);
#endif
        }
      }
      if constexpr (PM == 1 || PM == 3 || kMixed || kLog) {
        // a meet without a staircase or an NPC hit: rare_tick's lean meet,
        // the two moves in the drawn order (the tick block's word a; an
        // all-reject word takes the ordered tick), from each lane's side;
        // PM 3: each attacker's own damage and mana (rpg_attack), no item
        // underfoot (an item rides in an NPC slot, so hit_me / hit_o cover it)
        const uint32_t sa = ~(tb.a >> 1) & 0x55555555u;
        if (in_progress & meet & !st_me & (st_o == 0) & !hit_me & (hit_o == 0) & (sa != 0u)) {
          const bool p1_first = ((tb.a >> __builtin_ctz(sa)) & 1u) != 0;
          const bool me_first = p1_first != isB;
          const int32_t ax = me_first ? tx : otx, ay = me_first ? ty : oty;
          const int32_t bx = me_first ? otx : tx, by = me_first ? oty : ty;
          const int32_t fx0 = me_first ? me.x : ox, fy0 = me_first ? me.y : oy;
          const int32_t sx0 = me_first ? ox : me.x, sy0 = me_first ? oy : me.y;
          const bool occf = (ax == sx0) & (ay == sy0);  // the first attacks the second
          const int32_t fx = occf ? fx0 : ax, fy = occf ? fy0 : ay;
          const bool occs = (bx == fx) & (by == fy);    // the second attacks the first
          me.x = me_first ? fx : (occs ? sx0 : bx);
          me.y = me_first ? fy : (occs ? sy0 : by);
          if constexpr (PM == 3) {  // my attack spends my mana; the other's hits me
            const bool i_attack = me_first ? occf : occs;
            const int32_t d_me = i_attack ? rpg_attack(c, me) : 0;
            me.hp -= pair_swap(d_me);
          } else {
            const int32_t dmg = c.player_dmg_net > 0 ? c.player_dmg_net : 0;
            me.hp -= (me_first ? occs : occf) ? dmg : 0;
          }
          dl.combat += (occf ? 1 : 0) + (occs ? 1 : 0);
          dl.eps += end ? 1 : 0;
          tick = ft;
          status = end ? ORX_TIE : ORX_IN_PROGRESS;
          const int32_t ohp = pair_swap(me.hp);
          const bool d1 = (isB ? ohp : me.hp) <= 0, d2 = (isB ? me.hp : ohp) <= 0;
          if (d1 | d2) {  // deaths_over
            const int32_t sw = d1 ? (d2 ? ORX_TIE : ORX_PLAYER2_WIN) : ORX_PLAYER1_WIN;
            dl.eps += end ? 0 : 1;
            dl.ret += (sw == ORX_PLAYER1_WIN ? 1 : 0) - (sw == ORX_PLAYER2_WIN ? 1 : 0);
            status = sw;
          }
          fast = true;
#ifdef ORX_STAMPS
          ORX_COUNT(dl.n_meet);
#endif
        }
      }
      if ((PM == 2 || kMixed || kLog) && !GRID &&
          (in_progress & !meet & (st_me != (st_o != 0)) & !hit_me & (hit_o == 0))) {
#ifdef ORX_STAMPS
        ORX_CYC_BEGIN(cyf);
#endif
        const bool dIsB = st_me ? isB : !isB;       // the descender is player 2
        const int32_t sd = st_me ? me.d : od, odep = st_me ? od : me.d;
        const int32_t o_start = dIsB ? c.d1 : c.d2;
        const int32_t nd = sd + 1;
        bool present;
        uint32_t gen = 0;
        if (c.despawn == ORX_DESPAWN_UNREACHABLE) {
          present = o_start <= nd && nd <= odep;
        } else {
          present = odep == nd;
          gen = (!present && o_start <= nd && nd < odep) ? 1u : 0u;
        }
        const bool other_on = odep == nd;
        W4 w = philox(game, ep, st_me ? (uint32_t)tick : (uint32_t)nd,
                      st_me ? tag(PUR_SPAWN, 0) : tag(PUR_DUNGEON, gen), key);
        const W4 wo = {(uint32_t)pair_swap((int32_t)w.a), (uint32_t)pair_swap((int32_t)w.b),
                       (uint32_t)pair_swap((int32_t)w.c), (uint32_t)pair_swap((int32_t)w.d)};
        const W4 ws = st_me ? w : wo, wd = st_me ? wo : w;
        int32_t sx, sy;
        bool ok = stair_from_block(c, wd, sx, sy);
        const bool o_stairs = present & other_on;
        sx = o_stairs ? (st_me ? osx : me.sx) : sx;  // the other player's staircase
        sy = o_stairs ? (st_me ? osy : me.sy) : sy;
        ok |= o_stairs;
        const uint32_t v = ws.a & c.ground.mask;
        int32_t x, y;
        ground_cell<false>(c, v, -1, sx, sy, x, y);
        // the other player's cell before and after its move
        const int32_t ox0 = st_me ? ox : me.x, oy0 = st_me ? oy : me.y;
        const int32_t ox1 = st_me ? otx : tx, oy1 = st_me ? oty : ty;
        const bool touch = other_on & (((x == ox1) & (y == oy1)) | ((x == ox0) & (y == oy0)));
        const bool npc_depth = NCAP > 0 && nd == c.d1 && npc.any_alive();
        ok = ok & (c.ground.rng != 0u) & (v <= c.ground.rng) & !touch & !npc_depth;
        if (ok) {
          me.d = st_me ? nd : me.d;
          me.x = st_me ? x : tx;
          me.y = st_me ? y : ty;
          me.sx = st_me ? sx : me.sx;
          me.sy = st_me ? sy : me.sy;
          dl.descend += 1;
          dl.dungeon += present ? 0 : 1;
          dl.eps += end ? 1 : 0;
          tick = ft;
          status = end ? ORX_TIE : ORX_IN_PROGRESS;
          fast = true;
#ifdef ORX_STAMPS
          ORX_COUNT(dl.n_desc);
#endif
        }
#ifdef ORX_STAMPS
        ORX_CYC_END(dl.cy_desc, cyf);
#endif
      }
      if (!fast) {
        // both lanes rebuild the game's players and run the scalar rare block
        Player o = me;
        o.x = ox;
        o.y = oy;
        o.d = od;
        o.hp = pair_swap(me.hp);
        o.sx = osx;
        o.sy = osy;
        o.move = pair_swap(move);
        if constexpr (GRID) o.lay = pair_swap(me.lay);
        if constexpr (PM == 3) {  // the other player's attributes
          o.mana = pair_swap(me.mana);
          o.xp = pair_swap(me.xp);
          o.dmg = pair_swap(me.dmg);
          o.mhp = pair_swap(me.mhp);
          o.nitems = pair_swap(me.nitems);
        }
        Player p1 = pick(isB, o, me), p2 = pick(isB, me, o);
        if constexpr (ORX_RARE_OUTLINE != 0) {
          // the call's copies: only they live in the frame
          uint32_t q_ep = ep;
          Npcs<NCAP> q_npc = npc;
          Items<NCAP> q_items = items;
          auto q_hp = hp;
          int32_t q_tick = tick, q_status = status, q_sep = sep;
          Deltas q_dl = dl;
          bool q_restarted = restarted;
          took_ordered = rare_tick_ool<NCAP, GRID>(c, st, B, i, key, game, q_ep, p1, p2, q_npc,
                                                   q_items, q_hp, q_tick, q_status, q_dl, q_sep,
                                                   q_restarted, tb, need, isB ? otx : tx,
                                                   isB ? oty : ty, isB ? tx : otx,
                                                   isB ? ty : oty);
          ep = q_ep;
          npc = q_npc;
          items = q_items;
          hp = q_hp;
          tick = q_tick;
          status = q_status;
          sep = q_sep;
          dl = q_dl;
          restarted = q_restarted;
        } else {
          took_ordered = rare_tick<NCAP, GRID>(c, st, B, i, key, game, ep, p1, p2, npc, items, hp,
                                            tick, status, dl, sep, restarted, tb, need,
                                            isB ? otx : tx, isB ? oty : ty, isB ? tx : otx,
                                            isB ? ty : oty, false);
        }
        me = pick(isB, p2, p1);
        me.move = move;
      }
      kp = pack_cell(me.x, me.y);
      ks = pack_cell(me.sx, me.sy);
      dk = me.d == c.d1 ? 0u : 0x80008000u;
#ifdef ORX_STAMPS
      ORX_CYC_END(dl.cy_rare, cy0);
#endif
    } else {
      kp = kt;
    }
    // the common tick: the move to the effective target
    me.x = rare ? me.x : tx;
    me.y = rare ? me.y : ty;
    dl.eps += (!rare & end) ? 1 : 0;
    status = rare ? status : (end ? ORX_TIE : ORX_IN_PROGRESS);
    tick = rare ? tick : ft;
    if constexpr (PM == 3) {  // the end of the tick: mana regeneration, as rollout_tick
      const bool base = in_progress & !took_ordered;
      me.mana = base ? min(me.mana + c.mana_regen, c.mana_max) : me.mana;
    }
    if constexpr (SEP) {  // as rollout_tick (readme.md:46-47)
      const bool base = in_progress & !took_ordered;
      const int32_t od2 = pair_swap(me.d);
      if (base) {
        if (me.d != od2) {
          const int32_t t0 = ft - 1;
          if (sep < 0) sep = t0;
          const int32_t k = t0 - sep + 1;
          const int32_t dmg = sep_ceil(c, k);
          me.hp -= me.d < od2 ? dmg : 0;
          const int32_t ohp = pair_swap(me.hp);
          const bool d1 = (isB ? ohp : me.hp) <= 0, d2 = (isB ? me.hp : ohp) <= 0;
          if ((d1 | d2) && status != ORX_STATUS_RNG_EXHAUSTED) {  // deaths_over
            const int32_t s = d1 ? (d2 ? ORX_TIE : ORX_PLAYER2_WIN) : ORX_PLAYER1_WIN;
            dl.eps += end ? 0 : 1;
            dl.ret += (s == ORX_PLAYER1_WIN ? 1 : 0) - (s == ORX_PLAYER2_WIN ? 1 : 0);
            status = s;
          }
        } else {
          sep = -1;
        }
      }
    }
    if constexpr (kLean) {  // the lean ticks from this state on
      const int32_t ox = pair_swap(me.x), oy = pair_swap(me.y), od = pair_swap(me.d);
      const int32_t ex = me.sx - me.x, ey = me.sy - me.y;
      const int32_t dme = (ex < 0 ? -ex : ex) + (ey < 0 ? -ey : ey);  // to my staircase
      const int32_t dot = pair_swap(dme);
      const int32_t mx = me.x - ox, my = me.y - oy;
      const int32_t m = (mx < 0 ? -mx : mx) + (my < 0 ? -my : my);  // between the players
      int32_t sp = min(dme, dot) - 1;
      if (me.d == od) sp = min(sp, (m - 1) >> 1);
      if constexpr (SEP) {
        l_od = od;
        if (me.d != od) {  // the next tick's k = t0 - sep + 1 (sep set there if unset)
          const int32_t P = c.sep_period;
          const int32_t kn = tick - (sep < 0 ? tick : sep) + 1;
          l_q = (kn + P - 1) / P;
          l_r = kn - 1 - (l_q - 1) * P;
          if ((me.d < od) & (me.hp - l_q <= 0)) sp = 0;
        }
      }
      if (c.max_ticks) sp = min(sp, c.max_ticks - tick - 1);
      span = status == ORX_IN_PROGRESS ? sp : 0;
    }
    if (!(ORX_DIAG & 16)) traj.write(me, kp, ks, isB, tick, status, move);
    else traj.skip();
    ++t;
    // the loop's exit test on the row pointer (a scalar register): a test on
    // t alone gets t a VGPR and costs 2 VALU a tick (the compiler takes the
    // counter for divergent in this loop)
    } while (traj.obs != obs_end);
  ORX_STAMP(3);
  st.p_x[who * B + i] = me.x;
  st.p_y[who * B + i] = me.y;
  st.p_depth[who * B + i] = me.d;
  st.p_health[who * B + i] = me.hp;
  if (restarted || dl.descend != 0) {
    st.st_x[who * B + i] = me.sx;
    st.st_y[who * B + i] = me.sy;
    if constexpr (GRID) st.p_layout[who * B + i] = (int16_t)me.lay;
  }
  if constexpr (PM == 3) {
    int32_t* r = st.p_rpg + who * B + i;
    const size_t f = 2 * (size_t)B;
    r[ORX_RPG_MANA * f] = me.mana;
    r[ORX_RPG_XP * f] = me.xp;
    r[ORX_RPG_DAMAGE * f] = me.dmg;
    r[ORX_RPG_MAX_HEALTH * f] = me.mhp;
    r[ORX_RPG_ITEMS * f] = me.nitems;
    r[ORX_RPG_COOLDOWN * f] = 0;
    if constexpr (NCAP > 0) {
      if (!isB) {  // the game's items (identical in both lanes)
        st.item_mask[i] = items.on;
        st.item_mask[B + i] = items.kind;
        for (int k = 0; k < c.K; ++k)
          if ((items.on >> k) & 1u) st.item_pos[(size_t)k * B + i] = (uint16_t)npc.get(k);
      }
    }
  }
  if (!isB) {
    st.tick[i] = tick;
    st.status[i] = status;
    st.episode[i] = (int32_t)ep;
    if constexpr (SEP) st.sep_start[i] = sep;
    if constexpr (NCAP > 0) {
      if (restarted || dl.npc_death) npc.store_alive(st.npc_alive, B, i);
      if (restarted || dl.combat) hp.store(st.npc_health, c.K, B, i);
    }
    flush_deltas(st, B, i, dl);
  }
#ifdef ORX_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  ORX_STAMP(4);
#ifdef ORX_STAMPS
  uint32_t r[11] = {dl.n_rare, dl.n_ordered, dl.n_hits, dl.n_desc, dl.n_meet, dl.n_reset,
                    dl.cy_rare, dl.cy_reset, dl.cy_ordered, dl.cy_desc, dl.n_lean};
#pragma unroll
  for (int j = 0; j < 11; ++j)
    for (int o = 32; o > 0; o >>= 1) r[j] += __shfl_xor(r[j], o);
  if ((threadIdx.x & 63) == 0) {
    const size_t w = (size_t)((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 16;
#pragma unroll
    for (int j = 0; j < 11; ++j) g_stamps[w + 5 + j] = r[j];
  }
#endif
}

// Staircases of arbitrary (game, episode, depth, generation) dungeons, for
// materializing World.dungeons (compat views, wire codec).

// ---------------------------------------------------------------------------
// Stock-seed mode kernels (cfg.rng = ORX_RNG_MT19937)
// ---------------------------------------------------------------------------
// random.seed(n) (CPython random_seed -> init_by_array over the 32-bit words
// of n) and np.random.seed(n) (numpy mt19937_seed = init_genrand) for
// n = seed + global game id; both indices at 624 (the first draw twists).
#if ORX_HOST_TU
__global__ void __launch_bounds__(256) mt_seed_kernel(orx_state_t st, uint32_t B, uint64_t seed,
                                                      uint32_t off, uint32_t dstore_n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const uint64_t n = seed + off + i;
  uint32_t* np = st.mt_np + i;
  uint32_t x = (uint32_t)n;
  for (uint32_t k = 0; k < 624; ++k) {
    np[(size_t)k * B] = x;
    x = 1812433253u * (x ^ (x >> 30)) + k + 1u;
  }
  np[624 * (size_t)B] = 624;
  uint32_t* py = st.mt_py + i;
  const uint32_t key[2] = {(uint32_t)n, (uint32_t)(n >> 32)};
  const uint32_t klen = key[1] ? 2u : 1u;
  x = 19650218u;  // init_genrand(19650218)
  for (uint32_t k = 0; k < 624; ++k) {
    py[(size_t)k * B] = x;
    x = 1812433253u * (x ^ (x >> 30)) + k + 1u;
  }
  uint32_t idx = 1, j = 0, prev = py[0];
  for (uint32_t k = 624; k; --k) {
    const uint32_t v = (py[(size_t)idx * B] ^ ((prev ^ (prev >> 30)) * 1664525u)) + key[j] + j;
    py[(size_t)idx * B] = v;
    prev = v;
    ++idx; ++j;
    if (idx >= 624) { py[0] = prev; idx = 1; }
    if (j >= klen) j = 0;
  }
  for (uint32_t k = 623; k; --k) {
    const uint32_t v = (py[(size_t)idx * B] ^ ((prev ^ (prev >> 30)) * 1566083941u)) - idx;
    py[(size_t)idx * B] = v;
    prev = v;
    ++idx;
    if (idx >= 624) { py[0] = prev; idx = 1; }
  }
  py[0] = 0x80000000u;
  py[624 * (size_t)B] = 624;
  for (uint32_t k = 0; k < 2u * dstore_n; ++k) st.dstore[(size_t)(2 * k) * B + i] = -1;
}
#endif  // ORX_HOST_TU

// RandomBot.move = random.choice(list(Move)) = Move(1 + _randbelow(5))
// (randombot.py:21) from the game's CPython stream; StaircaseBot as usual.
__device__ __forceinline__ void mt_policy_pair(MtStream& py, int32_t pol1, int32_t pol2,
                                               const Player& p1, const Player& p2, int32_t& a1,
                                               int32_t& a2, bool& err) {
  int32_t r[2] = {ORX_MOVE_STAY, ORX_MOVE_STAY};
  int nr = 0;
  if (pol1 == ORX_POLICY_RANDOM) r[nr++] = 1 + (int32_t)py_randbelow(py, Key{0, 0}, 5u, err);
  if (pol2 == ORX_POLICY_RANDOM) r[nr++] = 1 + (int32_t)py_randbelow(py, Key{0, 0}, 5u, err);
  assign_moves(pol1, pol2, r[0], r[1], p1, p2, a1, a2);
}

// random.shuffle of the two players (updater.py:114: player 1 first iff
// _randbelow(2) == 1), then of the NPC updents (:127), whose order cannot
// matter (they Stay) but whose draws advance the stream.
template <int NCAP>
__device__ __forceinline__ bool mt_shuffles(MtStream& py, const Npcs<NCAP>& npc, bool& err) {
  const bool p1_first = py_randbelow(py, Key{0, 0}, 2u, err) == 1u;
  if constexpr (NCAP > 0)
    for (int32_t n = npc.count_alive() - 1; n >= 1; --n)
      py_randbelow(py, Key{0, 0}, (uint32_t)n + 1u, err);
  return p1_first;
}

template <int NCAP, bool GRID>
__global__ void __launch_bounds__(256) mt_reset_kernel(orx_cfg_t hc, orx_state_t st,
                                                       const uint8_t* __restrict__ mask,
                                                       uint32_t B) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  if (mask && !mask[i]) return;
  const Cfg c = make_cfg(hc, st);
  MtSrc src;
  src.open(st, c, B, i);
  Player p1, p2;
  Npcs<NCAP> npc;
  npc.bind(st, c, B, i);
  int32_t tick, status;
  setup_game<NCAP, GRID>(c, Key{0, 0}, src, p1, p2, npc, tick, status);
  src.close();
  store_players<GRID>(st, B, i, p1, p2, true);
  Items<NCAP> items;
  items.clear();
  store_rpg(st, c, B, i, p1, p2, npc, items);
  st.tick[i] = tick;
  st.status[i] = status;
  if (c.ext & ORX_EXT_SEPARATION_DAMAGE) st.sep_start[i] = -1;
  if constexpr (NCAP > 0) {
    npc.store_alive(st.npc_alive, B, i);
    store_new_npcs(st, c, B, i, npc);
  }
}

#if ORX_HOST_TU
__global__ void __launch_bounds__(256) mt_policy_kernel(orx_state_t st, int32_t pol1,
                                                        int32_t pol2,
                                                        int8_t* __restrict__ actions,
                                                        uint32_t B) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  Player p1, p2;
  p1.x = st.p_x[i]; p2.x = st.p_x[B + i];
  p1.y = st.p_y[i]; p2.y = st.p_y[B + i];
  p1.sx = st.st_x[i]; p2.sx = st.st_x[B + i];
  p1.sy = st.st_y[i]; p2.sy = st.st_y[B + i];
  uint16_t* out = reinterpret_cast<uint16_t*>(actions);
  int32_t a1 = ORX_MOVE_STAY, a2 = ORX_MOVE_STAY;
  if (pol1 == ORX_POLICY_NONE || pol2 == ORX_POLICY_NONE) {
    const uint16_t prev = out[i];
    a1 = (int8_t)(prev & 0xFF);
    a2 = (int8_t)(prev >> 8);
  }
  MtStream py;
  py.open(st.mt_py, B, i);
  bool err = false;
  mt_policy_pair(py, pol1, pol2, p1, p2, a1, a2, err);
  py.close();
  out[i] = pack_actions(a1, a2);
}
#endif  // ORX_HOST_TU

template <int NCAP, bool EV, bool GRID, bool MOV = false>
__global__ void __launch_bounds__(256) mt_step_kernel(orx_cfg_t hc, orx_state_t st,
                                                      const int8_t* __restrict__ actions,
                                                      uint32_t B, Key key, uint32_t off,
                                                      int32_t* __restrict__ events,
                                                      int32_t* __restrict__ n_events) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const Cfg c = make_cfg(hc, st);
  const uint32_t game = off + i;
  int32_t status = st.status[i];
  Npcs<NCAP> npc;
  npc.bind(st, c, B, i);
  Player p1, p2;
  if (status != ORX_IN_PROGRESS) {
    if (EV) n_events[i] = 0;
    if (!c.autoreset) return;
    MtSrc src;
    src.open(st, c, B, i);
    const uint32_t ep = (uint32_t)st.episode[i] + 1u;
    int32_t tick;
    setup_game<NCAP, GRID>(c, key, src, p1, p2, npc, tick, status);
    src.close();
    store_players<GRID>(st, B, i, p1, p2, true);
    Items<NCAP> items;
    items.clear();
    store_rpg(st, c, B, i, p1, p2, npc, items);
    st.tick[i] = tick;
    st.status[i] = status;
    st.episode[i] = (int32_t)ep;
    if (c.ext & ORX_EXT_SEPARATION_DAMAGE) st.sep_start[i] = -1;
    if constexpr (NCAP > 0) {
      npc.store_alive(st.npc_alive, B, i);
      store_new_npcs(st, c, B, i, npc);
    }
    return;
  }
  const uint16_t a = reinterpret_cast<const uint16_t*>(actions)[i];
  p1.move = (int8_t)(a & 0xFF);
  p2.move = (int8_t)(a >> 8);
  if (!valid_move(c, p1.move) || !valid_move(c, p2.move)) {
    st.status[i] = ORX_STATUS_BAD_ACTION;
    if (EV) n_events[i] = 0;
    return;
  }
  const uint32_t ep = (uint32_t)st.episode[i];
  int32_t tick = st.tick[i];
  load_players<GRID>(st, B, i, p1, p2);
  load_npcs(st, c, B, i, npc);
  Items<NCAP> items;
  load_rpg(st, c, B, i, p1, p2, npc, items);
  NpcMem m{st.npc_pos, st.npc_health, B, i};
  Deltas dl = {0, 0, 0, 0, 0, 0};
  const int32_t ev_cap = MOV ? max_events_for(c.npc_pol, c.K) : ORX_MAX_EVENTS;
  Events<EV> ev{EV ? events + (size_t)i * (size_t)ev_cap * 4 : nullptr, 0, ev_cap};
  bool err = false;
  MtSrc src;
  src.open(st, c, B, i);
  int32_t sep = (c.ext & ORX_EXT_SEPARATION_DAMAGE) ? st.sep_start[i] : -1;
  if constexpr (MOV) {
    tick_moving<NCAP, EV, GRID>(c, key, src, game, ep, p1, p2, npc, m, tick, status, err, dl, ev,
                                sep);
    store_npc_cells(st, c, B, i, npc);
  } else {
    const bool p1_first = mt_shuffles(src.py, npc, err);
    tick_game<NCAP, EV, GRID>(c, key, src, game, ep, p1_first, p1, p2, npc, items, m, tick,
                              status, err, dl, ev, sep);
  }
  src.close();
  store_rpg(st, c, B, i, p1, p2, npc, items);
  if (c.ext & ORX_EXT_SEPARATION_DAMAGE) st.sep_start[i] = sep;
  store_players<GRID>(st, B, i, p1, p2, dl.descend != 0);
  st.tick[i] = tick;
  st.status[i] = status;
  if (NCAP > 0 && dl.npc_death) npc.store_alive(st.npc_alive, B, i);
  flush_deltas(st, B, i, dl);
  if (EV) n_events[i] = ev.n;
}

template <int NCAP, bool GRID>
__global__ void __launch_bounds__(256) mt_rollout_kernel(orx_cfg_t hc, orx_state_t st,
                                                         int32_t pol1, int32_t pol2,
                                                         int32_t n_ticks,
                                                         int32_t* __restrict__ obs,
                                                         int8_t* __restrict__ act, uint32_t B,
                                                         Key key, uint32_t off, int32_t fmt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const Cfg c = make_cfg(hc, st);
  const uint32_t game = off + i;
  Player p1, p2;
  load_players<GRID>(st, B, i, p1, p2);
  int32_t tick = st.tick[i];
  int32_t status = st.status[i];
  uint32_t ep = (uint32_t)st.episode[i];
  Npcs<NCAP> npc;
  npc.bind(st, c, B, i);
  load_npcs(st, c, B, i, npc);
  NpcMem m{st.npc_pos, st.npc_health, B, i};
  Items<NCAP> items;
  load_rpg(st, c, B, i, p1, p2, npc, items);
  Deltas dl = {0, 0, 0, 0, 0, 0};
  int32_t sep = (c.ext & ORX_EXT_SEPARATION_DAMAGE) ? st.sep_start[i] : -1;
  bool stairs_dirty = false, npc_dirty = false;
  MtSrc src;
  src.open(st, c, B, i);
  TrajWriter<false> traj(obs, act, B, i, fmt);
  for (int32_t t = 0; t < n_ticks; ++t) {
    int32_t a1 = ORX_MOVE_STAY, a2 = ORX_MOVE_STAY;
    bool err = false;
    mt_policy_pair(src.py, pol1, pol2, p1, p2, a1, a2, err);
    if (status == ORX_IN_PROGRESS) {
      p1.move = a1; p2.move = a2;
      const int32_t descents = dl.descend;
      const bool p1_first = mt_shuffles(src.py, npc, err);
      Events<false> ev{nullptr, 0};
      tick_game<NCAP, false, GRID>(c, key, src, game, ep, p1_first, p1, p2, npc, items, m, tick,
                                   status, err, dl, ev, sep);
      stairs_dirty |= dl.descend != descents;
    } else if (c.autoreset) {
      ep += 1;
      setup_game<NCAP, GRID>(c, key, src, p1, p2, npc, tick, status);
      items.clear();
      if constexpr (NCAP > 0) store_new_npcs(st, c, B, i, npc);
      stairs_dirty = true;
      npc_dirty = true;
      sep = -1;
    }
    traj.write(t, p1, p2, tick, status, a1, a2);
  }
  src.close();
  store_players<GRID>(st, B, i, p1, p2, stairs_dirty);
  store_rpg(st, c, B, i, p1, p2, npc, items);
  st.tick[i] = tick;
  st.status[i] = status;
  st.episode[i] = (int32_t)ep;
  if (c.ext & ORX_EXT_SEPARATION_DAMAGE) st.sep_start[i] = sep;
  if (NCAP > 0 && (npc_dirty || dl.npc_death)) npc.store_alive(st.npc_alive, B, i);
  flush_deltas(st, B, i, dl);
}

// orx_step_n: n_ticks x orx_step with given actions (actions[t][b] = the
// pair of tick t, player 1 in the low byte) in one launch, the state in
// registers between ticks -- the multi-tick Updater.update loop of a replay
// (server/main.py:110-113 fed from a recorded or precomputed move log):
// per tick a game in progress validates its pair (a non-Move value stops it
// with ORX_STATUS_BAD_ACTION, as orx_step), draws its initiative from the
// tick block and runs tick_game; a finished game is reset to its next
// episode when cfg.autoreset.  obs (may be NULL): each tick's post-step row,
// in format fmt.  One lane per game (any dungeon, any NPC count, any
// extension flag: the generic tick).
//
// ROWS (0 none, 1 int32, 2 compact) is a compile-time copy of (obs, fmt):
// every path through the tick then issues the same row stores, so the wait
// for the next tick's prefetched pair (issued before this tick's stores)
// leaves this tick's stores in flight -- with the row branch at run time the
// compiler's wait at the loop head has to assume a path without stores and
// drains them all every tick.
template <int NCAP, bool GRID, int ROWS, bool MOV = false>
__device__ __forceinline__ void step_n_game(const orx_cfg_t& hc, const orx_state_t& st,
                                            const int8_t* __restrict__ actions, int32_t n_ticks,
                                            int32_t* __restrict__ obs, uint32_t B, uint32_t i,
                                            Key key, uint32_t off) {
  const Cfg c = make_cfg(hc, st);
  const uint32_t game = off + i;
  Player p1, p2;
  load_players<GRID>(st, B, i, p1, p2);
  int32_t tick = st.tick[i];
  int32_t status = st.status[i];
  uint32_t ep = (uint32_t)st.episode[i];
  Npcs<NCAP> npc;
  npc.bind(st, c, B, i);
  load_npcs(st, c, B, i, npc);
  NpcMem m{st.npc_pos, st.npc_health, B, i};
  Items<NCAP> items;
  load_rpg(st, c, B, i, p1, p2, npc, items);
  Deltas dl = {0, 0, 0, 0, 0, 0};
  int32_t sep = (c.ext & ORX_EXT_SEPARATION_DAMAGE) ? st.sep_start[i] : -1;
  bool stairs_dirty = false, npc_dirty = false;
  if constexpr (ROWS != 0) __builtin_assume(obs != nullptr);
  TrajWriter<false> traj(ROWS != 0 ? obs : nullptr, nullptr, B, i,
                         ROWS == 2 ? ORX_OBS_COMPACT : ORX_OBS_INT32);
  const uint16_t* a16 = reinterpret_cast<const uint16_t*>(actions) + i;
  // the next tick's pair is loaded while this tick runs (a lone wave per SIMD
  // would otherwise wait one HBM round trip per tick); the last tick re-reads
  // its own pair instead of branching
  uint16_t a_next = a16[0];
  // settled before the loop (with the state loads), so that the loop head's
  // wait sees only the back edge: the pair loaded one tick earlier, that
  // tick's row stores issued after it
  asm volatile("" : "+v"(a_next));
  for (int32_t t = 0; t < n_ticks; ++t) {
    const uint16_t a = a_next;
    a_next = a16[(size_t)(t + 1 < n_ticks ? t + 1 : t) * B];
    const int32_t a1 = (int8_t)(a & 0xFF), a2 = (int8_t)(a >> 8);
    if (status == ORX_IN_PROGRESS) {
      p1.move = a1;
      p2.move = a2;
      if (!valid_move(c, a1) || !valid_move(c, a2)) {
        status = ORX_STATUS_BAD_ACTION;
      } else {
        bool err = false;
        const int32_t descents = dl.descend;
        Events<false> ev{nullptr, 0};
        if constexpr (MOV) {
          PhiloxSrc src{key, game, ep};
          tick_moving<NCAP, false, GRID>(c, key, src, game, ep, p1, p2, npc, m, tick, status, err,
                                         dl, ev, sep);
          npc_dirty = true;
        } else {
          const bool p1_first = p1_first_draw(key, game, ep, tick, err);
          tick_game<NCAP, false, GRID>(c, key, game, ep, p1_first, p1, p2, npc, items, m, tick,
                                       status, err, dl, ev, sep);
        }
        stairs_dirty |= dl.descend != descents;
      }
    } else if (c.autoreset) {
      ep += 1;
      setup_game<NCAP, GRID>(c, key, game, ep, p1, p2, npc, tick, status);
      items.clear();
      if constexpr (NCAP > 0) store_new_npcs(st, c, B, i, npc);
      stairs_dirty = true;
      npc_dirty = true;
      sep = -1;
    }
    if constexpr (ROWS != 0) traj.write(t, p1, p2, tick, status, a1, a2);
  }
  store_players<GRID>(st, B, i, p1, p2, stairs_dirty);
  store_rpg(st, c, B, i, p1, p2, npc, items);
  st.tick[i] = tick;
  st.status[i] = status;
  st.episode[i] = (int32_t)ep;
  if (c.ext & ORX_EXT_SEPARATION_DAMAGE) st.sep_start[i] = sep;
  if (NCAP > 0 && (npc_dirty || dl.npc_death)) npc.store_alive(st.npc_alive, B, i);
  if (MOV && npc_dirty) store_npc_cells(st, c, B, i, npc);
  flush_deltas(st, B, i, dl);
}

template <int NCAP, bool GRID, bool MOV = false>
__global__ void __launch_bounds__(256) step_n_kernel(orx_cfg_t hc, orx_state_t st,
                                                     const int8_t* __restrict__ actions,
                                                     int32_t n_ticks, int32_t* __restrict__ obs,
                                                     uint32_t B, Key key, uint32_t off,
                                                     int32_t fmt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  if (obs == nullptr)  // (uniform)
    step_n_game<NCAP, GRID, 0, MOV>(hc, st, actions, n_ticks, obs, B, i, key, off);
  else if (fmt == ORX_OBS_COMPACT)
    step_n_game<NCAP, GRID, 2, MOV>(hc, st, actions, n_ticks, obs, B, i, key, off);
  else
    step_n_game<NCAP, GRID, 1, MOV>(hc, st, actions, n_ticks, obs, B, i, key, off);
}

// orx_rollout with moving NPCs (cfg.npc_policy): n_ticks x (the bots' moves,
// then the moving-NPC tick or the autoreset), one lane per game, each tick's
// observation row (format fmt) and actions written when obs / act are given.
// MT: stock-seed mode (the bots and the tick draw from the game's CPython
// random in the reference's call order, as mt_rollout_kernel).
template <int NCAP, bool GRID, bool MT>
__global__ void __launch_bounds__(256) mov_rollout_kernel(orx_cfg_t hc, orx_state_t st,
                                                          int32_t pol1, int32_t pol2,
                                                          int32_t n_ticks,
                                                          int32_t* __restrict__ obs,
                                                          int8_t* __restrict__ act, uint32_t B,
                                                          Key key, uint32_t off, int32_t fmt,
                                                          uint32_t lanes) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (lanes < 64u) {  // uniform: lanes >= `lanes` of every wave idle (as rollout_kernel)
    if ((threadIdx.x & 63u) >= lanes) return;
    i = (i >> 6) * lanes + (threadIdx.x & 63u);
  }
  if (i >= B) return;
  const Cfg c = make_cfg(hc, st);
  const uint32_t game = off + i;
  Player p1, p2;
  load_players<GRID>(st, B, i, p1, p2);
  int32_t tick = st.tick[i];
  int32_t status = st.status[i];
  uint32_t ep = (uint32_t)st.episode[i];
  Npcs<NCAP> npc;
  npc.bind(st, c, B, i);
  load_npcs(st, c, B, i, npc);
  // register NPCs keep their health in registers for the launch (as the
  // rollout's NpcHpRegs), stored once at the end; dense NPCs' stays in HBM
  constexpr bool kRegHp = NCAP > 0 && NCAP != kDense;
  std::conditional_t<kRegHp, NpcHpRegs<NCAP>, NpcMem> m;
  if constexpr (kRegHp) m.load(st.npc_health, c.K, B, i);
  else m = NpcMem{st.npc_pos, st.npc_health, B, i};
  Items<NCAP> items;
  load_rpg(st, c, B, i, p1, p2, npc, items);
  Deltas dl = {0, 0, 0, 0, 0, 0};
  int32_t sep = (c.ext & ORX_EXT_SEPARATION_DAMAGE) ? st.sep_start[i] : -1;
  bool stairs_dirty = false, npc_dirty = false;
  std::conditional_t<MT, MtSrc, PhiloxSrc> src;
  if constexpr (MT) src.open(st, c, B, i);
  else src = PhiloxSrc{key, game, ep};
  TrajWriter<false> traj(obs, act, B, i, fmt);
  ORX_MCYC_BEGIN(cyl);
  for (int32_t t = 0; t < n_ticks; ++t) {
    int32_t a1 = ORX_MOVE_STAY, a2 = ORX_MOVE_STAY;
    bool err = false;
    ORX_MCYC_BEGIN(cy6);
    // the tick block serves the RandomBots and the moving tick's first draws
    W4 tb{0u, 0u, 0u, 0u};
    if constexpr (MT) {
      mt_policy_pair(src.py, pol1, pol2, p1, p2, a1, a2, err);
    } else {
      tb = tick_block(key, game, ep, tick);
      policy_pair(key, game, ep, tick, pol1, pol2, tb, p1, p2, a1, a2);
    }
    ORX_MCYC_END(6, cy6);
    if (status == ORX_IN_PROGRESS) {
      ORX_MCYC_BEGIN(cyt);
      p1.move = a1;
      p2.move = a2;
      const int32_t descents = dl.descend;
      Events<false> ev{nullptr, 0};
      tick_moving<NCAP, false, GRID>(c, key, src, game, ep, p1, p2, npc, m, tick, status, err, dl,
                                     ev, sep, MT ? nullptr : &tb);
      stairs_dirty |= dl.descend != descents;
      npc_dirty = true;
      ORX_MCYC_END(10, cyt);
    } else if (c.autoreset) {
      ORX_MCYC_BEGIN(cy7);
      ep += 1;
      if constexpr (!MT) src.ep = ep;
      setup_game<NCAP, GRID>(c, key, src, p1, p2, npc, tick, status);
      if constexpr (kRegHp) m.fill(c.npc_hp);  // (the cells: store_npc_cells at the end)
      else if constexpr (NCAP > 0) store_new_npcs(st, c, B, i, npc);
      stairs_dirty = true;
      npc_dirty = true;
      sep = -1;
      ORX_MCYC_END(7, cy7);
    }
    ORX_MCYC_BEGIN(cy8);
    traj.write(t, p1, p2, tick, status, a1, a2);
    ORX_MCYC_END(8, cy8);
  }
  ORX_MCYC_END(9, cyl);
  if constexpr (MT) src.close();
  store_players<GRID>(st, B, i, p1, p2, stairs_dirty);
  st.tick[i] = tick;
  st.status[i] = status;
  st.episode[i] = (int32_t)ep;
  if (c.ext & ORX_EXT_SEPARATION_DAMAGE) st.sep_start[i] = sep;
  if (NCAP > 0 && npc_dirty) {
    npc.store_alive(st.npc_alive, B, i);
    store_npc_cells(st, c, B, i, npc);
    if constexpr (kRegHp) m.store(st.npc_health, c.K, B, i);
  }
  flush_deltas(st, B, i, dl);
}

// orx_step_n's fast form (register NPCs, empty dungeons: NCAP 0 / 8 / 16,
// no bank): the rollout's tick (rollout_tick, LOG) on the logged pair -- the
// order-free common path, every rare case in its out-of-line block, no policy
// draw at all (the initiative block is drawn only by a game whose order
// matters) -- with the rollout's register-resident NPC health and buffer-store
// rows (ROWS 0 none, 1 int32, 2 compact; no action rows: the log is the
// actions).  The next tick's pair is prefetched as in step_n_kernel.
template <int NCAP, int ROWS, bool EXT>
__global__ void __launch_bounds__(kRolloutBlock) replay_kernel(orx_cfg_t hc, orx_state_t st,
                                                               const int8_t* __restrict__ actions,
                                                               int32_t n_ticks,
                                                               int32_t* __restrict__ obs,
                                                               uint32_t B, Key key, uint32_t off,
                                                               uint32_t lanes) {
  uint32_t i = xcd_block() * blockDim.x + threadIdx.x;
  if (lanes < 64u) {  // uniform: lanes >= `lanes` of every wave idle (as rollout_kernel)
    if ((threadIdx.x & 63u) >= lanes) return;
    i = (i >> 6) * lanes + (threadIdx.x & 63u);
  }
  if (i >= B) return;
  Cfg c = make_cfg(hc, st);
  if constexpr (!EXT) c.ext = 0;  // launched only with flags == 0
  const uint32_t game = off + i;
  Player p1, p2;
  load_players<false>(st, B, i, p1, p2);
  int32_t tick = st.tick[i];
  int32_t status = st.status[i];
  uint32_t ep = (uint32_t)st.episode[i];
  Npcs<NCAP> npc;
  npc.bind(st, c, B, i);
  load_npcs(st, c, B, i, npc);
  NpcHpRegs<NCAP> hp;
  if constexpr (NCAP > 0) hp.load(st.npc_health, c.K, B, i);
  Items<NCAP> items;
  load_rpg(st, c, B, i, p1, p2, npc, items);
  Deltas dl = {0, 0, 0, 0, 0, 0};
  int32_t sep = (c.ext & ORX_EXT_SEPARATION_DAMAGE) ? st.sep_start[i] : -1;
  bool restarted = false;
  TrajWriter<true, kStreamAux, ROWS == 2, false> traj(ROWS != 0 ? obs : nullptr, nullptr, B, i);
  const uint16_t* a16 = reinterpret_cast<const uint16_t*>(actions) + i;
  uint16_t a_next = a16[0];   // (issued after the state loads: its wait covers them)
  asm volatile("" : "+v"(a_next));
  int32_t t = 0;
  do {  // n_ticks >= 1: orx_step_n returns before launching 0 ticks
    const uint16_t a = a_next;
    a_next = a16[(size_t)(t + 1 < n_ticks ? t + 1 : t) * B];
    int32_t a1 = (int8_t)(a & 0xFF), a2 = (int8_t)(a >> 8);
    rollout_tick<NCAP, false, NpcHpRegs<NCAP>, true>(
        c, st, B, i, key, game, ep, ORX_POLICY_NONE, ORX_POLICY_NONE, p1, p2, npc, items, hp,
        tick, status, dl, sep, restarted, a1, a2);
    if constexpr (ROWS != 0) traj.write(t, p1, p2, tick, status, a1, a2);
  } while (++t < n_ticks);
  store_players<false>(st, B, i, p1, p2, restarted || dl.descend != 0);
  store_rpg(st, c, B, i, p1, p2, npc, items);
  st.tick[i] = tick;
  st.status[i] = status;
  st.episode[i] = (int32_t)ep;
  if (c.ext & ORX_EXT_SEPARATION_DAMAGE) st.sep_start[i] = sep;
  if constexpr (NCAP > 0) {
    if (restarted || dl.npc_death) npc.store_alive(st.npc_alive, B, i);
    if (restarted || dl.combat) hp.store(st.npc_health, c.K, B, i);
  }
  flush_deltas(st, B, i, dl);
}

template <bool GRID>
__global__ void __launch_bounds__(256) stairs_kernel(orx_cfg_t hc, orx_state_t st,
                                                     const uint32_t* __restrict__ games,
                                                     const int32_t* __restrict__ episodes,
                                                     const int32_t* __restrict__ depths,
                                                     const int32_t* __restrict__ gens,
                                                     int32_t* __restrict__ sx,
                                                     int32_t* __restrict__ sy,
                                                     int32_t* __restrict__ layout, uint32_t n,
                                                     Key key) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Cfg c = make_cfg(hc, st);
  bool err = false;
  int32_t x, y, lay;
  dungeon_stair<GRID>(c, key, games[i], (uint32_t)episodes[i], depths[i], (uint32_t)gens[i], x, y,
                      lay,
                      err);
  sx[i] = err ? -1 : x;
  sy[i] = err ? -1 : y;
  if (layout) layout[i] = err ? -1 : lay;
}

// ---------------------------------------------------------------------------
// Kernel instances: every template instance the host side launches, as
// X-macro lists shared by the host dispatch (below) and the split build's
// explicit instantiations, so the two cannot drift apart.
// ---------------------------------------------------------------------------
// (NCAP, GRID): reset_kernel, mt_reset_kernel, mt_rollout_kernel, step_n_kernel
#define ORX_NG_LIST(X)                                                                          \
  X(0, false) X(8, false) X(16, false) X(kDense, false)                                         \
  X(0, true) X(8, true) X(16, true) X(kDense, true)
// (NCAP, EV, GRID): step_kernel (all rules) and mt_step_kernel
#define ORX_STEP_LIST(X)                                                                        \
  X(0, false, false) X(0, true, false) X(8, false, false) X(8, true, false)                     \
  X(16, false, false) X(16, true, false) X(0, false, true) X(0, true, true)                     \
  X(8, false, true) X(8, true, true) X(16, false, true) X(16, true, true)                       \
  X(kDense, false, false) X(kDense, true, false) X(kDense, false, true) X(kDense, true, true)
// NCAP: step_kernel<NCAP, false, false, false> (the reference's rules only)
#define ORX_STEP_REF_LIST(X) X(0) X(8) X(16)
// (NCAP, ROWS, EXT): replay_kernel (EXT false: flags 0, the extension tests
// compiled out of the common tick)
#define ORX_REPLAY_LIST_E(X, E)                                                                 \
  X(0, 0, E) X(0, 1, E) X(0, 2, E) X(8, 0, E) X(8, 1, E) X(8, 2, E) X(16, 0, E) X(16, 1, E)      \
  X(16, 2, E)
#define ORX_REPLAY_LIST(X) ORX_REPLAY_LIST_E(X, false) ORX_REPLAY_LIST_E(X, true)
// (NCAP, GRID, EXT): env_step_kernel
#define ORX_ENV_LIST(X)                                                                         \
  X(0, false, false) X(8, false, false) X(16, false, false)                                     \
  X(0, false, true) X(8, false, true) X(16, false, true)                                        \
  X(kDense, false, true) X(0, true, true) X(8, true, true) X(16, true, true) X(kDense, true, true)
// (NCAP, PM, AUX, SEP, CF, GRID): pair_rollout_kernel, per NCAP in two halves
// -- A: PM 1 / 2 on empty dungeons in both row formats; B: PM 3 and the banks
#define ORX_PAIR_LIST_C(X, N, C)                                                                \
  X(N, 1, kStreamAux, false, C, false) X(N, 1, kPartialAux, false, C, false)                    \
  X(N, 2, kStreamAux, false, C, false) X(N, 2, kPartialAux, false, C, false)                    \
  X(N, 2, kStreamAux, true, C, false) X(N, 2, kPartialAux, true, C, false)
#define ORX_PAIR_LIST_A(X, N) ORX_PAIR_LIST_C(X, N, false) ORX_PAIR_LIST_C(X, N, true)
#define ORX_PAIR_LIST_B(X, N)                                                                   \
  X(N, 3, kStreamAux, false, false, false) X(N, 3, kPartialAux, false, false, false)            \
  X(N, 3, kStreamAux, false, false, true) X(N, 3, kPartialAux, false, false, true)              \
  X(N, 1, kStreamAux, false, false, true) X(N, 1, kPartialAux, false, false, true)              \
  X(N, 2, kStreamAux, false, false, true) X(N, 2, kPartialAux, false, false, true)
// PM 4 / 5 (a RandomBot against a StaircaseBot), empty dungeons, int32 rows
#define ORX_PAIR_LIST_M(X, N)                                                                   \
  X(N, 4, kStreamAux, false, false, false) X(N, 4, kPartialAux, false, false, false)            \
  X(N, 5, kStreamAux, false, false, false) X(N, 5, kPartialAux, false, false, false)
// PM 6 (a move log's replay, orx_step_n), empty dungeons, int32 / compact rows
#define ORX_PAIR_LIST_L(X, N)                                                                   \
  X(N, 6, kStreamAux, false, false, false) X(N, 6, kPartialAux, false, false, false)            \
  X(N, 6, kStreamAux, false, true, false) X(N, 6, kPartialAux, false, true, false)
#define ORX_PAIR_LIST(X)                                                                        \
  ORX_PAIR_LIST_A(X, 0) ORX_PAIR_LIST_B(X, 0) ORX_PAIR_LIST_A(X, 8) ORX_PAIR_LIST_B(X, 8)       \
  ORX_PAIR_LIST_A(X, 16) ORX_PAIR_LIST_B(X, 16) ORX_PAIR_LIST_M(X, 0) ORX_PAIR_LIST_M(X, 8)     \
  ORX_PAIR_LIST_M(X, 16)
// (NCAP, PM, GRID, AUX, CF): rollout_kernel -- the generic form (PM 0) in one
// store policy and any row format; the buffer-store forms (PM 1 / 2 / 3) in
// both policies; PM 1 / 2 without a bank or dense NPCs also in compact rows
#define ORX_ROLLOUT_LIST_NG(X, N, G)                                                            \
  X(N, 0, G, kStreamAux, false)                                                                 \
  X(N, 1, G, kStreamAux, false) X(N, 1, G, kPartialAux, false)                                  \
  X(N, 2, G, kStreamAux, false) X(N, 2, G, kPartialAux, false)                                  \
  X(N, 3, G, kStreamAux, false) X(N, 3, G, kPartialAux, false)
#define ORX_ROLLOUT_LIST_N(X, N)                                                                \
  ORX_ROLLOUT_LIST_NG(X, N, false) ORX_ROLLOUT_LIST_NG(X, N, true)                              \
  X(N, 1, false, kStreamAux, true) X(N, 1, false, kPartialAux, true)                            \
  X(N, 2, false, kStreamAux, true) X(N, 2, false, kPartialAux, true)
#define ORX_ROLLOUT_LIST_DENSE(X)                                                               \
  X(kDense, 0, false, kStreamAux, false) X(kDense, 0, true, kStreamAux, false)                  \
  X(kDense, 1, false, kStreamAux, false) X(kDense, 1, false, kPartialAux, false)                \
  X(kDense, 2, false, kStreamAux, false) X(kDense, 2, false, kPartialAux, false)                \
  X(kDense, 1, true, kStreamAux, false) X(kDense, 1, true, kPartialAux, false)                  \
  X(kDense, 2, true, kStreamAux, false) X(kDense, 2, true, kPartialAux, false)
#define ORX_ROLLOUT_LIST(X)                                                                     \
  ORX_ROLLOUT_LIST_N(X, 0) ORX_ROLLOUT_LIST_N(X, 8) ORX_ROLLOUT_LIST_N(X, 16)                   \
  ORX_ROLLOUT_LIST_DENSE(X)

// moving NPCs (cfg.npc_policy != ORX_NPC_STAY): (NCAP, GRID) of
// step_n_kernel<N, G, true> and env_step_kernel<N, G, true, true>, (NCAP, EV,
// GRID) of step_kernel<N, E, G, true, true> and mt_step_kernel<N, E, G, true>,
// (NCAP, GRID, MT) of mov_rollout_kernel
#define ORX_MOV_NG_LIST(X)                                                                      \
  X(8, false) X(16, false) X(kDense, false) X(8, true) X(16, true) X(kDense, true)
#define ORX_MOV_STEP_LIST(X)                                                                    \
  X(8, false, false) X(8, true, false) X(16, false, false) X(16, true, false)                   \
  X(kDense, false, false) X(kDense, true, false) X(8, false, true) X(8, true, true)             \
  X(16, false, true) X(16, true, true) X(kDense, false, true) X(kDense, true, true)
#define ORX_MOV_ROLLOUT_LIST(X)                                                                 \
  X(8, false, false) X(16, false, false) X(kDense, false, false) X(8, true, false)              \
  X(16, true, false) X(kDense, true, false) X(8, false, true) X(16, false, true)                \
  X(kDense, false, true) X(8, true, true) X(16, true, true) X(kDense, true, true)

#ifdef ORX_NPARTS
// ORX_INST: `extern` in the host part (an explicit instantiation
// declaration: the part that owns the instance emits it), empty in the
// instance parts (an explicit instantiation definition)
#if ORX_PART == 0
#define ORX_INST extern
#else
#define ORX_INST
#endif
#define ORX_I_RESET(N, G)                                                                       \
  ORX_INST template __global__ void reset_kernel<N, G>(orx_cfg_t, orx_state_t, const uint8_t*,  \
                                                       uint32_t, Key, uint32_t);
#define ORX_I_MT_RESET(N, G)                                                                    \
  ORX_INST template __global__ void mt_reset_kernel<N, G>(orx_cfg_t, orx_state_t,               \
                                                          const uint8_t*, uint32_t);
#define ORX_I_MT_ROLLOUT(N, G)                                                                  \
  ORX_INST template __global__ void mt_rollout_kernel<N, G>(orx_cfg_t, orx_state_t, int32_t,    \
                                                            int32_t, int32_t, int32_t*, int8_t*, \
                                                            uint32_t, Key, uint32_t, int32_t);
#define ORX_I_STEP(N, E, G)                                                                     \
  ORX_INST template __global__ void step_kernel<N, E, G, true>(orx_cfg_t, orx_state_t,          \
                                                               const int8_t*, uint32_t, Key,    \
                                                               uint32_t, int32_t*, int32_t*);
#define ORX_I_STEP_REF(N)                                                                       \
  ORX_INST template __global__ void step_kernel<N, false, false, false>(                        \
      orx_cfg_t, orx_state_t, const int8_t*, uint32_t, Key, uint32_t, int32_t*, int32_t*);
#define ORX_I_MT_STEP(N, E, G)                                                                  \
  ORX_INST template __global__ void mt_step_kernel<N, E, G>(orx_cfg_t, orx_state_t,             \
                                                            const int8_t*, uint32_t, Key,       \
                                                            uint32_t, int32_t*, int32_t*);
#define ORX_I_ENV(N, G, X)                                                                      \
  ORX_INST template __global__ void env_step_kernel<N, G, X>(                                   \
      orx_cfg_t, orx_state_t, const void*, int32_t, int32_t, int32_t, int8_t*, int32_t*, float*, \
      uint8_t*, int32_t*, uint32_t*, uint32_t, Key, uint32_t, int32_t, uint32_t);
#define ORX_I_PAIR(N, P, A, S, C, G)                                                            \
  ORX_INST template __global__ void pair_rollout_kernel<N, P, A, S, C, G>(                      \
      orx_cfg_t, orx_state_t, int32_t, int32_t*, int8_t*, uint32_t, Key, uint32_t, uint32_t,     \
      uint32_t);
#define ORX_I_ROLLOUT(N, P, G, A, C)                                                            \
  ORX_INST template __global__ void rollout_kernel<N, P, G, A, C>(                              \
      orx_cfg_t, orx_state_t, int32_t, int32_t, int32_t, int32_t*, int8_t*, uint32_t, Key,      \
      uint32_t, uint32_t, uint32_t, uint32_t, int32_t);
#define ORX_I_STEP_N(N, G)                                                                      \
  ORX_INST template __global__ void step_n_kernel<N, G>(orx_cfg_t, orx_state_t, const int8_t*,  \
                                                        int32_t, int32_t*, uint32_t, Key,       \
                                                        uint32_t, int32_t);
#define ORX_I_REPLAY(N, R, E)                                                                   \
  ORX_INST template __global__ void replay_kernel<N, R, E>(orx_cfg_t, orx_state_t,              \
                                                           const int8_t*, int32_t, int32_t*,    \
                                                           uint32_t, Key, uint32_t, uint32_t);
#define ORX_I_MOV_STEP(N, E, G)                                                                 \
  ORX_INST template __global__ void step_kernel<N, E, G, true, true>(                           \
      orx_cfg_t, orx_state_t, const int8_t*, uint32_t, Key, uint32_t, int32_t*, int32_t*);      \
  ORX_INST template __global__ void mt_step_kernel<N, E, G, true>(                              \
      orx_cfg_t, orx_state_t, const int8_t*, uint32_t, Key, uint32_t, int32_t*, int32_t*);
#define ORX_I_MOV_NG(N, G)                                                                      \
  ORX_INST template __global__ void step_n_kernel<N, G, true>(orx_cfg_t, orx_state_t,           \
                                                              const int8_t*, int32_t, int32_t*, \
                                                              uint32_t, Key, uint32_t, int32_t); \
  ORX_INST template __global__ void env_step_kernel<N, G, true, true>(                          \
      orx_cfg_t, orx_state_t, const void*, int32_t, int32_t, int32_t, int8_t*, int32_t*, float*, \
      uint8_t*, int32_t*, uint32_t*, uint32_t, Key, uint32_t, int32_t, uint32_t);
#define ORX_I_MOV_ROLLOUT(N, G, M)                                                              \
  ORX_INST template __global__ void mov_rollout_kernel<N, G, M>(                                \
      orx_cfg_t, orx_state_t, int32_t, int32_t, int32_t, int32_t*, int8_t*, uint32_t, Key,      \
      uint32_t, int32_t, uint32_t);
#define ORX_I_STAIRS(G)                                                                         \
  ORX_INST template __global__ void stairs_kernel<G>(orx_cfg_t, orx_state_t, const uint32_t*,    \
                                                     const int32_t*, const int32_t*,            \
                                                     const int32_t*, int32_t*, int32_t*,        \
                                                     int32_t*, uint32_t, Key);
// the parts: 1-6 the paired rollouts (NCAP 0 / 8 / 16, halves A and B), 7-9
// the one-lane rollouts per NCAP, 10 the dense rollouts and env_step, 11 the
// step kernels, 12 the rest, 13 the mixed-bot paired rollouts, 14 the
// moving-NPC kernels, 15 the paired replays; each costs a few tens of
// seconds of hipcc
#define ORX_OWNS(k) (ORX_PART == 0 || ORX_PART == (k))
#if ORX_OWNS(1)
ORX_PAIR_LIST_A(ORX_I_PAIR, 0)
#endif
#if ORX_OWNS(2)
ORX_PAIR_LIST_B(ORX_I_PAIR, 0)
#endif
#if ORX_OWNS(3)
ORX_PAIR_LIST_A(ORX_I_PAIR, 8)
#endif
#if ORX_OWNS(4)
ORX_PAIR_LIST_B(ORX_I_PAIR, 8)
#endif
#if ORX_OWNS(5)
ORX_PAIR_LIST_A(ORX_I_PAIR, 16)
#endif
#if ORX_OWNS(6)
ORX_PAIR_LIST_B(ORX_I_PAIR, 16)
#endif
#if ORX_OWNS(7)
ORX_ROLLOUT_LIST_N(ORX_I_ROLLOUT, 0)
#endif
#if ORX_OWNS(8)
ORX_ROLLOUT_LIST_N(ORX_I_ROLLOUT, 8)
#endif
#if ORX_OWNS(9)
ORX_ROLLOUT_LIST_N(ORX_I_ROLLOUT, 16)
#endif
#if ORX_OWNS(10)
ORX_ROLLOUT_LIST_DENSE(ORX_I_ROLLOUT)
ORX_ENV_LIST(ORX_I_ENV)
#endif
#if ORX_OWNS(11)
ORX_STEP_LIST(ORX_I_STEP)
ORX_STEP_REF_LIST(ORX_I_STEP_REF)
ORX_STEP_LIST(ORX_I_MT_STEP)
#endif
#if ORX_OWNS(13)
ORX_PAIR_LIST_M(ORX_I_PAIR, 0)
ORX_PAIR_LIST_M(ORX_I_PAIR, 8)
ORX_PAIR_LIST_M(ORX_I_PAIR, 16)
#endif
#if ORX_OWNS(15)
ORX_PAIR_LIST_L(ORX_I_PAIR, 0)
ORX_PAIR_LIST_L(ORX_I_PAIR, 8)
ORX_PAIR_LIST_L(ORX_I_PAIR, 16)
#endif
#if ORX_OWNS(14)
ORX_MOV_STEP_LIST(ORX_I_MOV_STEP)
ORX_MOV_NG_LIST(ORX_I_MOV_NG)
ORX_MOV_ROLLOUT_LIST(ORX_I_MOV_ROLLOUT)
#endif
#if ORX_OWNS(12)
ORX_NG_LIST(ORX_I_RESET)
ORX_NG_LIST(ORX_I_MT_RESET)
ORX_NG_LIST(ORX_I_MT_ROLLOUT)
ORX_NG_LIST(ORX_I_STEP_N)
ORX_REPLAY_LIST(ORX_I_REPLAY)
ORX_I_STAIRS(false)
ORX_I_STAIRS(true)
#endif
#endif  // ORX_NPARTS

#if ORX_HOST_TU
// ---------------------------------------------------------------------------
// Host side of the C-ABI
// ---------------------------------------------------------------------------
thread_local char g_err[512] = "";

int fail(int code, const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return code;
}

int check_cfg(const orx_cfg_t* c) {
  if (!c) return fail(ORX_EINVAL, "cfg is NULL");
  if (c->width < 4 || c->height < 4)
    return fail(ORX_EINVAL, "width and height must be >= 4 (np.random.randint(1, W-2))");
  if ((int64_t)(c->width - 2) * (c->height - 2) > (1 << 30))
    return fail(ORX_EINVAL, "grid too large");
  if (c->despawn != ORX_DESPAWN_UNREACHABLE && c->despawn != ORX_DESPAWN_UNUSED)
    return fail(ORX_EINVAL, "unknown despawn strategy");
  if (c->max_ticks < 0) return fail(ORX_EINVAL, "max_ticks must be >= 0");
  if (c->start_mode != ORX_START_TOGETHER && c->start_mode != ORX_START_SEPARATED)
    return fail(ORX_EINVAL, "unknown start mode");
  if (c->start_mode == ORX_START_SEPARATED &&
      (c->p1_depth == c->p2_depth || c->p1_depth < 0 || c->p2_depth < 0))
    return fail(ORX_EINVAL, "SeparatedGameStartGenerator needs p1_depth != p2_depth, both >= 0");
  if (c->n_npcs < 0 || c->n_npcs > ORX_MAX_NPCS)
    return fail(ORX_EINVAL, "n_npcs must be in [0, 255]");
  if (c->n_npcs > ORX_MAX_REG_NPCS && (c->flags & ORX_EXT_ITEMS))
    return fail(ORX_EINVAL, "ORX_EXT_ITEMS needs n_npcs <= 16");
  if (c->n_npcs > 0 && (c->width > ORX_MAX_GRID_NPC || c->height > ORX_MAX_GRID_NPC))
    return fail(ORX_EINVAL, "NPC positions pack 8+8 bits: W, H <= 256 when n_npcs > 0");
  if (c->n_npcs > 0 && (c->npc_health < 1 || c->npc_health > 127))
    return fail(ORX_EINVAL, "npc_health must be in [1, 127]");
  if (c->n_layouts < 0 || c->n_layouts > 32767)
    return fail(ORX_EINVAL, "n_layouts must be in [0, 32767]");
  if (c->n_layouts > 0 && (int64_t)c->width * c->height > 65536)
    return fail(ORX_EINVAL, "a dungeon bank needs W * H <= 65536 (u16 Ground lists)");
  const int64_t n_ground = (int64_t)(c->width - 2) * (c->height - 2) - 1;
  if (c->n_layouts == 0 && n_ground < (int64_t)c->n_npcs + 2)
    return fail(ORX_EINVAL, "board too small for the players and NPCs");
  if (c->player_health < 1) return fail(ORX_EINVAL, "player_health must be >= 1");
  if (c->autoreset != 0 && c->autoreset != 1) return fail(ORX_EINVAL, "autoreset must be 0 or 1");
  if (c->flags & ~(ORX_EXT_SEPARATION_DAMAGE | ORX_EXT_RANDOM_DOUBLE_DEATH | ORX_EXT_CHARACTER))
    return fail(ORX_EINVAL, "unknown extension flag");
  if ((c->flags & ORX_EXT_README_COMBAT) && c->combat_cooldown < 0)
    return fail(ORX_EINVAL, "the readme's combat needs combat_cooldown >= 0");
  if ((c->flags & ORX_EXT_HEAL) && !(c->flags & ORX_EXT_MANA))
    return fail(ORX_EINVAL, "ORX_EXT_HEAL needs ORX_EXT_MANA");
  if ((c->flags & ORX_EXT_MANA) &&
      (c->mana_max < 3 || c->mana_regen < 0 || c->mana_per_point < 1))
    return fail(ORX_EINVAL, "mana needs mana_max >= 3, mana_regen >= 0, mana_per_point >= 1");
  if ((c->flags & ORX_EXT_LEVELING) && (c->xp_per_kill < 0 || c->xp_per_level < 1))
    return fail(ORX_EINVAL, "leveling needs xp_per_kill >= 0, xp_per_level >= 1");
  if ((c->flags & ORX_EXT_ITEMS) && (c->item_drop_pct < 0 || c->item_drop_pct > 100 ||
                                     c->item_bonus < 0 || c->item_slots < 0))
    return fail(ORX_EINVAL, "items need item_drop_pct in [0, 100], item_bonus >= 0, "
                            "item_slots >= 0");
  if ((c->flags & ORX_EXT_SEPARATION_DAMAGE) &&
      (c->sep_period < 1 || c->sep_period > ORX_SEP_PERIOD_MAX))
    return fail(ORX_EINVAL, "separation damage needs 1 <= sep_period <= ORX_SEP_PERIOD_MAX");
  if (c->rng != ORX_RNG_PHILOX && c->rng != ORX_RNG_MT19937)
    return fail(ORX_EINVAL, "unknown rng mode");
  if (c->rng == ORX_RNG_MT19937 && (c->width > 256 || c->height > 256))
    return fail(ORX_EINVAL, "stock-seed mode stores staircases 8+8 bits: W, H <= 256");
  if (c->npc_policy < ORX_NPC_STAY || c->npc_policy > ORX_NPC_CHASE)
    return fail(ORX_EINVAL, "unknown npc_policy");
  if (c->npc_policy != ORX_NPC_STAY &&
      (c->flags & ~(ORX_EXT_SEPARATION_DAMAGE | ORX_EXT_RANDOM_DOUBLE_DEATH)))
    return fail(ORX_EINVAL, "moving NPCs (npc_policy) need flags within "
                            "ORX_EXT_SEPARATION_DAMAGE | ORX_EXT_RANDOM_DOUBLE_DEATH");
  return ORX_OK;
}

// The moving-NPC kernels serve this configuration (NPCs that move)
inline bool moving_npcs(const orx_cfg_t* c) {
  return c->npc_policy != ORX_NPC_STAY && c->n_npcs > 0;
}

int check_state(const orx_cfg_t* c, const orx_state_t* s, bool full) {
  if (!s) return fail(ORX_EINVAL, "state is NULL");
  if (!s->p_x || !s->p_y || !s->p_depth || !s->p_health || !s->st_x || !s->st_y || !s->tick ||
      !s->status || !s->episode)
    return fail(ORX_EINVAL, "a required state pointer is NULL");
  if (full && (!s->ret_sum || !s->ep_count))
    return fail(ORX_EINVAL, "ret_sum / ep_count are NULL");
  if (c->n_npcs > 0 && (!s->npc_pos || !s->npc_health || !s->npc_alive))
    return fail(ORX_EINVAL, "n_npcs > 0 needs npc_pos, npc_health and npc_alive");
  if (c->n_npcs > ORX_MAX_REG_NPCS && !s->npc_grid)
    return fail(ORX_EINVAL, "n_npcs > 16 needs npc_grid ([B][W * H] uint8)");
  if (c->n_layouts > 0 && (!s->p_layout || !s->bank_tiles || !s->bank_ground || !s->bank_meta))
    return fail(ORX_EINVAL, "n_layouts > 0 needs p_layout and the bank_* arrays");
  if ((c->flags & ORX_EXT_SEPARATION_DAMAGE) && !s->sep_start)
    return fail(ORX_EINVAL, "separation damage needs sep_start");
  if (c->rng == ORX_RNG_MT19937 && (!s->mt_py || !s->mt_np || !s->dstore))
    return fail(ORX_EINVAL, "stock-seed mode needs mt_py, mt_np and dstore");
  if ((c->flags & ORX_EXT_CHARACTER) && !s->p_rpg)
    return fail(ORX_EINVAL, "the character mechanics need p_rpg");
  if ((c->flags & ORX_EXT_ITEMS) && c->n_npcs > 0 && (!s->item_pos || !s->item_mask))
    return fail(ORX_EINVAL, "ORX_EXT_ITEMS needs item_pos and item_mask");
  return ORX_OK;
}

int check_policy(int32_t p) {
  if (p < ORX_POLICY_NONE || p > ORX_POLICY_STAY) return fail(ORX_EINVAL, "unknown policy");
  return ORX_OK;
}

// ORX_OBS_COMPACT's field widths (include/orx.h): u8 cells, int16 healths,
// a 27-bit tick
int check_compact(const orx_cfg_t* c) {
  if (c->width > 256 || c->height > 256)
    return fail(ORX_EINVAL, "compact rows: width and height must be <= 256");
  if (c->max_ticks < 1 || c->max_ticks >= (1 << 27))
    return fail(ORX_EINVAL, "compact rows: max_ticks must be in [1, 2^27)");
  const int32_t m = ORX_COMPACT_MAX_STAT;
  bool ok = c->player_health <= m && c->player_damage <= m && c->player_armor >= -m &&
            (c->n_npcs == 0 || c->npc_damage <= m);
  if (c->flags & ORX_EXT_MANA) ok = ok && c->mana_max <= m;
  if (c->flags & ORX_EXT_ITEMS)
    ok = ok && (int64_t)c->item_bonus * (int64_t)c->item_slots <= m;
  if (c->flags & ORX_EXT_SEPARATION_DAMAGE)
    ok = ok && c->max_ticks / (c->sep_period > 0 ? c->sep_period : 1) <= m;
  if (!ok)
    return fail(ORX_EINVAL, "compact rows: a health, damage or separation-damage bound above "
                            "ORX_COMPACT_MAX_STAT (health must fit int16)");
  return ORX_OK;
}

int launch_status(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "%s launch failed: %s", what, hipGetErrorString(e));
    return ORX_EIO;
  }
  g_err[0] = 0;
  return ORX_OK;
}

constexpr int kBlock = 256;

inline dim3 grid_for(int64_t B) { return dim3((unsigned)((B + kBlock - 1) / kBlock)); }

inline Key make_key(uint64_t seed) { return Key{(uint32_t)seed, (uint32_t)(seed >> 32)}; }

int check_sizes(int64_t B, int64_t off) {
  if (B < 0) return fail(ORX_EINVAL, "n_games < 0");
  if (B > 0x7FFFFFFFLL - kBlock) return fail(ORX_EINVAL, "n_games must be < 2^31");
  if (off < 0 || off + B > ((int64_t)1 << 32))
    return fail(ORX_EINVAL, "global game ids (game_offset + index) must fit 32 bits");
  return ORX_OK;
}

// NPC slot capacity of the kernel instance for K NPCs.
inline int ncap_for(int K) {
  return K == 0 ? 0 : K <= 8 ? 8 : K <= ORX_MAX_REG_NPCS ? 16 : kDense;
}

// Games per rollout wave.  A rollout lane runs its game's whole tick stream,
// so a wave's time is set by its instruction stream, not by how many of its
// lanes are busy: a batch too small to put a wave on every SIMD (4 per CU) is
// spread over more, narrower waves, which also take the rare block on fewer
// ticks (C5 at 16,384 games: 232 us per 128-tick launch at 64 games per wave,
// 158 at 16).  Not below 16: narrower waves share each 128-B trajectory line
// among four or more waves, and launches took twice as long (C2 at 4,096
// games: 77 us at 16, 155 at 8).  Two half-full waves per SIMD lose to one
// full one (C3: 101 us at 64, 130 at 32), so the rule is "at most one wave per
// SIMD until the wave is full".  The environment variable ORX_ROLLOUT_LANES
// (1..64, a power of two) overrides it for measurements.
constexpr int kMaxDevices = 64;
constexpr uint32_t kMinLanes = 16;
std::atomic<int> g_cu_count[kMaxDevices];

int device_simds() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return 1024;
  int n = g_cu_count[dev].load(std::memory_order_relaxed);
  if (n <= 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
    g_cu_count[dev].store(n, std::memory_order_relaxed);
  }
  return 4 * n;
}

// Dynamic LDS one workgroup may declare on the current device with the
// opt-in limit raise (160 KiB on gfx950): the opt-in attribute, else the
// default per-block one, else kMaxLdsBlock; read once per device.
std::atomic<int> g_lds_block[kMaxDevices];

uint32_t device_lds_per_block() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return kMaxLdsBlock;
  int n = g_lds_block[dev].load(std::memory_order_relaxed);
  if (n <= 0) {
    int optin = 0, plain = 0;
    if (hipDeviceGetAttribute(&optin, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess)
      optin = 0;
    if (hipDeviceGetAttribute(&plain, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess)
      plain = 0;
    n = optin > 0 ? optin : plain > 0 ? plain : (int)kMaxLdsBlock;
    g_lds_block[dev].store(n, std::memory_order_relaxed);
  }
  return (uint32_t)n;
}

bool paired_enabled() {  // read per launch (ORX_ROLLOUT_PAIRED=0: the one-lane form)
  const char* e = getenv("ORX_ROLLOUT_PAIRED");
  return !(e && e[0] == '0');
}

int lanes_override() {  // read per launch, so a sweep can change it in-process
  const char* e = getenv("ORX_ROLLOUT_LANES");
  const int x = e ? atoi(e) : 0;
  return (x >= 1 && x <= 64 && (x & (x - 1)) == 0) ? x : 0;
}

// Games per wave of mov_rollout_kernel: 64 (its tick is issue-bound, so
// fewer games per wave only add waves: 32 / 16 / 8 measured equal or slower,
// profiles/r06_v4/ab_mov_lanes_regs.jsonl); env ORX_MOV_LANES = 1..64, a
// power of two, overrides, for measurements and tests
uint32_t mov_lanes() {
  const char* e = getenv("ORX_MOV_LANES");
  const int x = e ? atoi(e) : 0;
  return (x >= 1 && x <= 64 && (x & (x - 1)) == 0) ? (uint32_t)x : 64u;
}

// Threads per rollout workgroup: kRolloutBlock (env ORX_ROLLOUT_THREADS = 64
// / 128 / 256 overrides, for measurements).
uint32_t rollout_threads(uint32_t B, uint32_t lanes) {
  const char* e = getenv("ORX_ROLLOUT_THREADS");
  const int x = e ? atoi(e) : 0;
  if (x == 64 || x == 128 || x == 256) return (uint32_t)x;
  (void)B; (void)lanes;  // single-wave workgroups for small batches measured within
                         // +-3% (profiles/r02_v6/threads_ab.jsonl): not the default
  return (uint32_t)kRolloutBlock;
}

uint32_t rollout_lanes(uint32_t B) {
  if (const int o = lanes_override()) return (uint32_t)o;
  const uint64_t simds = (uint64_t)device_simds();
  uint32_t L = 64;
  while (L > kMinLanes && (uint64_t)B < simds * L) L >>= 1;
  return L;
}

// The policy mode (rollout_kernel's PM) of an orx_rollout launch: the
// buffer-addressed trajectory forms need both buffers and one tick's obs rows
// below 2 GiB.
int rollout_pm(const orx_cfg_t* cfg, int32_t p1, int32_t p2, uint32_t B, bool traj) {
  const bool traj_fast = traj && (uint64_t)B * ORX_OBS_FIELDS * 4u < (1ull << 31);
  const bool both_random = p1 == ORX_POLICY_RANDOM && p2 == ORX_POLICY_RANDOM;
  return !traj_fast ? 0
         : (cfg->flags == 0 && both_random) ? 1
         : ((cfg->flags & ~ORX_EXT_SEPARATION_DAMAGE) == 0 && p1 == ORX_POLICY_STAIRCASE &&
            p2 == ORX_POLICY_STAIRCASE) ? 2
         : ((cfg->flags | ORX_EXT_HEAL) == ORX_EXT_RPG && both_random &&
            ncap_for(cfg->n_npcs) != kDense) ? 3   // (no dense-NPC instance of PM 3)
         // one RandomBot against one StaircaseBot: paired forms only (PM 4 /
         // 5; a launch that does not pair takes the generic form)
         : (cfg->flags == 0 && p1 == ORX_POLICY_RANDOM && p2 == ORX_POLICY_STAIRCASE) ? 4
         : (cfg->flags == 0 && p1 == ORX_POLICY_STAIRCASE && p2 == ORX_POLICY_RANDOM) ? 5
         : 0;
}

// A bank's tiles staged in LDS by the rollout kernels: up to the device's
// per-workgroup limit (160 KiB on gfx950; above the default 64 KiB the launch
// raises the kernel's limit, raise_lds).  Env ORX_NO_LDS_TILES: never, for
// measurements.
bool bank_in_lds(const orx_cfg_t* cfg) {
  const uint64_t tiles = (uint64_t)cfg->n_layouts * (uint64_t)(cfg->width * cfg->height);
  return tiles && tiles <= device_lds_per_block() && !getenv("ORX_NO_LDS_TILES");
}

// Raises kernel `fn`'s dynamic-LDS limit to `bytes` when they exceed the
// default 64 KiB; false when the device or the runtime refuses (env
// ORX_REFUSE_LDS_RAISE=1 simulates a refusal, for tests), so the caller
// launches a form that does not need them.
bool raise_lds(const void* fn, uint32_t bytes) {
  if (bytes <= kMaxLdsTiles) return true;
  if (bytes > device_lds_per_block()) return false;
  const char* e = getenv("ORX_REFUSE_LDS_RAISE");
  if (e && e[0] == '1') return false;
  if (!fn) return true;  // (orx_rollout_shape: whether a raise is needed and allowed)
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) !=
      hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return true;
}

// Threads per paired-rollout workgroup: kRolloutBlock, or 512 for a bank
// whose tiles leave room for one workgroup per CU (more than half the LDS):
// then the CU's one copy of the tiles serves 8 waves, two per SIMD, the
// occupancy the paired plan's games per wave assume.  Env
// ORX_ROLLOUT_THREADS (64 / 128 / 256, and 512 for banks) overrides.
uint32_t pair_threads(const orx_cfg_t* cfg, uint32_t lanes, uint32_t lds_n) {
  (void)lanes;
  const char* e = getenv("ORX_ROLLOUT_THREADS");
  const int x = e ? atoi(e) : 0;
  if (x == 64 || x == 128 || x == 256 || (x == 512 && cfg->n_layouts > 0)) return (uint32_t)x;
  if (cfg->n_layouts > 0 && 2ull * lds_n > device_lds_per_block()) return 512u;
  return (uint32_t)kRolloutBlock;
}

// The form, games per wave and store policy of an orx_rollout launch.
struct RolloutPlan {
  bool paired;     // pair_rollout_kernel: two lanes per game
  uint32_t lanes;  // games per wave
  bool nt;         // nontemporal trajectory stores (whole-line row segments)
};

// The paired form: no dense NPCs (K <= 16), no bank, the RandomBot or StaircaseBot trajectory
// forms (PM 1 / 2) and the RandomBot form with the character mechanics (PM 3,
// round 4: each lane its own player's mana, experience, damage, max health
// and items held; the game's items beside its NPCs in both lanes; every rare
// tick through rare_tick), for batches the one-lane rule leaves below 64 games per
// wave; its games per wave: two waves per SIMD -- counting the `concurrency`
// launches that share the device (StreamShardedEngine's shards) -- until the
// wave holds 32 games, at least 8 (C5's 8-GPU share, 16,384 games: 8 per
// wave, 79 us per launch against 89 at 16 and 112 at 32; C2 at 4,096: 50
// against 51; the bench's two 32,768-game C3 shards: 32 per wave, 96.6 us
// per step against 158 at 16, four waves per SIMD where 156 VGPRs fit three).
// ORX_ROLLOUT_LANES (games per wave) and ORX_ROLLOUT_PAIRED=0 override.
RolloutPlan plan_rollout(const orx_cfg_t* cfg, int pm, uint32_t B, uint32_t concurrency) {
  RolloutPlan p;
  p.lanes = rollout_lanes(B);
  // (its packed cells x | y << 8 need x, y < 256)
  // a dungeon bank: PM 1 / 3, and PM 2 without separation damage, with the
  // tiles staged in LDS (the paired form reads them only there)
  const bool bank_ok = cfg->n_layouts == 0 ||
                       (!(pm == 2 && (cfg->flags & ORX_EXT_SEPARATION_DAMAGE) != 0) && pm <= 3 &&
                        bank_in_lds(cfg));
  // StaircaseBots (PM 2) also pair where the one-lane rule fills whole
  // waves, when the batch shares the device with another launch and the
  // device's games come to at most four 32-game waves per SIMD: C5's 131,072
  // games as two 65,536-game stream shards, 177-179 us per 128-tick step
  // paired against 183-192 one-lane (242 / 254 with separation damage;
  // profiles/r05_v1/c5_forms.jsonl)
  const uint64_t simds4 = 4ull * 32ull * (uint64_t)device_simds();
  const bool pm2_full = pm == 2 && p.lanes == 64u && concurrency >= 2 &&
                        (uint64_t)B * concurrency <= simds4 && !lanes_override();
  p.paired = ncap_for(cfg->n_npcs) != kDense && bank_ok && pm >= 1 && pm <= 6 &&
             cfg->width <= 256 && cfg->height <= 256 && (p.lanes <= 32u || pm2_full) &&
             paired_enabled();
  if (p.paired) {
    if (const int o = lanes_override()) {
      p.lanes = o < 32 ? (uint32_t)o : 32u;
    } else {
      const uint64_t simds = (uint64_t)device_simds();
      uint32_t L = 32;
      while (L > 8 && (uint64_t)B * concurrency < 2 * simds * L) L >>= 1;
      p.lanes = L;
    }
  }
  p.nt = p.lanes * 4u >= 128u;  // a wave's row segment is a whole line
  return p;
}
#endif  // ORX_HOST_TU

}  // namespace orx_dev

#if ORX_HOST_TU
using namespace orx_dev;

extern "C" {

int orx_abi_version(void) { return ORX_ABI_VERSION; }

#ifndef ORX_BUILD_ID
#define ORX_BUILD_ID "unknown"
#endif
const char* orx_build_id(void) { return ORX_BUILD_ID; }

int orx_rollout_lanes(int64_t n_games) {
  if (n_games <= 0 || n_games > 0x7FFFFFFFLL) return fail(ORX_EINVAL, "bad n_games");
  return (int)rollout_lanes((uint32_t)n_games);
}

const char* orx_last_error(void) { return g_err; }

int orx_rollout_shape(const orx_cfg_t* cfg, int32_t policy_p1, int32_t policy_p2,
                      int64_t n_games, int32_t trajectory, int32_t concurrency,
                      orx_rollout_shape_t* out) {
  int r;
  if (concurrency < 1) return fail(ORX_EINVAL, "concurrency must be >= 1");
  if ((r = check_cfg(cfg)) || (r = check_policy(policy_p1)) || (r = check_policy(policy_p2)))
    return r;
  if (n_games <= 0 || n_games > 0x7FFFFFFFLL) return fail(ORX_EINVAL, "bad n_games");
  if (!out) return fail(ORX_EINVAL, "out is NULL");
  const uint32_t B = (uint32_t)n_games;
  out->threads_per_block = kBlock;
  out->lds_bytes = 0;
  if (moving_npcs(cfg)) {  // mov_rollout_kernel: one game per lane, mov_lanes per wave
    out->games_per_wave = (int32_t)mov_lanes();
    out->lanes_per_game = 1;
    out->nontemporal = 1;
    return ORX_OK;
  }
  if (cfg->rng == ORX_RNG_MT19937) {  // mt_rollout_kernel: one game per lane, full waves
    out->games_per_wave = 64;
    out->lanes_per_game = 1;
    out->nontemporal = 1;
    return ORX_OK;
  }
  int pm = rollout_pm(cfg, policy_p1, policy_p2, B, trajectory != 0);
  RolloutPlan p = plan_rollout(cfg, pm, B, (uint32_t)concurrency);
  if (!p.paired && pm >= 4) pm = 0;  // (the mixed-bot forms are paired only)
  const uint64_t tiles = (uint64_t)cfg->n_layouts * (uint64_t)(cfg->width * cfg->height);
  uint32_t lds_n = (cfg->n_layouts > 0 && bank_in_lds(cfg)) ? (uint32_t)tiles : 0u;
  if (p.paired && !raise_lds(nullptr, lds_n)) {  // the launch's fallback (one lane, global tiles)
    p.paired = false;
    p.lanes = rollout_lanes(B);
    p.nt = p.lanes * 4u >= 128u;
    lds_n = 0u;
  }
  out->games_per_wave = (int32_t)p.lanes;
  out->lanes_per_game = p.paired ? 2 : 1;
  out->nontemporal = (pm != 0 && !p.nt) ? 0 : 1;
  out->threads_per_block = (int32_t)(p.paired ? pair_threads(cfg, p.lanes, lds_n)
                                              : rollout_threads(B, p.lanes));
  uint32_t lds = p.paired ? lds_n : (uint32_t)((lds_n + 15u) & ~15u);
  if (!p.paired) {  // as the one-lane launch: bitmaps, then tiles, dropped on a refused raise
    uint32_t bits = 0;
    if (ncap_for(cfg->n_npcs) == kDense && !getenv("ORX_NO_LDS_BITS")) {
      const uint32_t bb = (uint32_t)((cfg->width * cfg->height + 31) / 32) * 4u;
      const uint32_t per_block = (uint32_t)out->threads_per_block / 64u * p.lanes;
      if ((uint64_t)lds + (uint64_t)per_block * bb <= device_lds_per_block()) bits = per_block * bb;
    }
    if (raise_lds(nullptr, lds + bits)) lds += bits;
    if (!raise_lds(nullptr, lds)) lds = 0u;
  }
  out->lds_bytes = (int32_t)lds;
  return ORX_OK;
}

int orx_max_events(const orx_cfg_t* cfg) {
  if (const int r = check_cfg(cfg)) return r;
  return max_events_for(cfg->npc_policy, cfg->n_npcs);
}

int orx_dstore_depths(const orx_cfg_t* cfg) {
  if (const int r = check_cfg(cfg)) return r;
  return (int)dstore_depths(cfg->max_ticks);
}

int orx_validate_cfg(const orx_cfg_t* cfg) {
  int r = check_cfg(cfg);
  if (r == ORX_OK) g_err[0] = 0;
  return r;
}

int orx_seed_mt(const orx_cfg_t* cfg, const orx_state_t* st, int64_t n_games, uint64_t seed,
                int64_t game_offset, void* stream) {
  int r;
  if ((r = check_cfg(cfg)) || (r = check_sizes(n_games, game_offset))) return r;
  if (cfg->rng != ORX_RNG_MT19937) return fail(ORX_EINVAL, "orx_seed_mt needs cfg->rng = ORX_RNG_MT19937");
  if (seed + (uint64_t)game_offset + (uint64_t)n_games < seed)
    return fail(ORX_EINVAL, "seed + game id overflows 64 bits");
  if (n_games == 0) return ORX_OK;
  if ((r = check_state(cfg, st, false))) return r;
  hipLaunchKernelGGL(mt_seed_kernel, grid_for(n_games), dim3(kBlock), 0, (hipStream_t)stream, *st,
                     (uint32_t)n_games, seed, (uint32_t)game_offset,
                     dstore_depths(cfg->max_ticks));
  return launch_status("orx_seed_mt");
}

int orx_reset(const orx_cfg_t* cfg, const orx_state_t* st, const uint8_t* mask, int64_t n_games,
              uint64_t seed, int64_t game_offset, void* stream) {
  int r;
  if ((r = check_cfg(cfg)) || (r = check_sizes(n_games, game_offset))) return r;
  if (n_games == 0) return ORX_OK;
  if ((r = check_state(cfg, st, false))) return r;
  const uint32_t B = (uint32_t)n_games, off = (uint32_t)game_offset;
  const hipStream_t s = (hipStream_t)stream;
  const Key k = make_key(seed);
  const int nc = ncap_for(cfg->n_npcs);
  const bool grid = cfg->n_layouts > 0;
  if (cfg->rng == ORX_RNG_MT19937) {
#define ORX_RESET(N, G)                                                                         \
  if (nc == N && grid == G)                                                                     \
    hipLaunchKernelGGL((mt_reset_kernel<N, G>), grid_for(B), dim3(kBlock), 0, s, *cfg, *st, mask, B);
    ORX_NG_LIST(ORX_RESET)
#undef ORX_RESET
    return launch_status("orx_reset");
  }
#define ORX_RESET(N, G)                                                                         \
  if (nc == N && grid == G)                                                                     \
    hipLaunchKernelGGL((reset_kernel<N, G>), grid_for(B), dim3(kBlock), 0, s, *cfg, *st, mask, B, \
                       k, off);
  ORX_NG_LIST(ORX_RESET)
#undef ORX_RESET
  return launch_status("orx_reset");
}

static int launch_step(const orx_cfg_t* cfg, const orx_state_t* st, const int8_t* actions,
                       int32_t* events, int32_t* n_events, int64_t n_games, uint64_t seed,
                       int64_t game_offset, void* stream, const char* name) {
  int r;
  if ((r = check_cfg(cfg)) || (r = check_sizes(n_games, game_offset))) return r;
  if (n_games == 0) return ORX_OK;
  if ((r = check_state(cfg, st, true))) return r;
  if (!actions) return fail(ORX_EINVAL, "actions is NULL");
  const bool ev = events != nullptr;
  if (ev != (n_events != nullptr)) return fail(ORX_EINVAL, "events and n_events go together");
  const uint32_t B = (uint32_t)n_games, off = (uint32_t)game_offset;
  const hipStream_t s = (hipStream_t)stream;
  const Key k = make_key(seed);
  const int nc = ncap_for(cfg->n_npcs);
  const bool grid = cfg->n_layouts > 0;
  const bool mt = cfg->rng == ORX_RNG_MT19937;
  if (moving_npcs(cfg)) {  // the ordered tick with the enemy AI
#define ORX_STEP(NC, E, G)                                                                      \
  if (nc == NC && ev == E && grid == G) {                                                      \
    if (mt)                                                                                     \
      hipLaunchKernelGGL((mt_step_kernel<NC, E, G, true>), grid_for(B), dim3(kBlock), 0, s,     \
                         *cfg, *st, actions, B, k, off, events, n_events);                      \
    else                                                                                        \
      hipLaunchKernelGGL((step_kernel<NC, E, G, true, true>), grid_for(B), dim3(kBlock), 0, s,  \
                         *cfg, *st, actions, B, k, off, events, n_events);                      \
    return launch_status(name);                                                                \
  }
    ORX_MOV_STEP_LIST(ORX_STEP)
#undef ORX_STEP
    return fail(ORX_EIO, "orx_step: no moving-NPC kernel instance for this configuration");
  }
  if (!ev && !grid && !mt && cfg->flags == 0 && nc != kDense) {  // the reference's rules
    if (nc == 0)
      hipLaunchKernelGGL((step_kernel<0, false, false, false>), grid_for(B), dim3(kBlock), 0, s,
                         *cfg, *st, actions, B, k, off, events, n_events);
    else if (nc == 8)
      hipLaunchKernelGGL((step_kernel<8, false, false, false>), grid_for(B), dim3(kBlock), 0, s,
                         *cfg, *st, actions, B, k, off, events, n_events);
    else
      hipLaunchKernelGGL((step_kernel<16, false, false, false>), grid_for(B), dim3(kBlock), 0, s,
                         *cfg, *st, actions, B, k, off, events, n_events);
    return launch_status(name);
  }
#define ORX_STEP(NC, E, G)                                                                      \
  if (nc == NC && ev == E && grid == G) {                                                      \
    if (mt)                                                                                     \
      hipLaunchKernelGGL((mt_step_kernel<NC, E, G>), grid_for(B), dim3(kBlock), 0, s, *cfg, *st, \
                         actions, B, k, off, events, n_events);                                 \
    else                                                                                        \
      hipLaunchKernelGGL((step_kernel<NC, E, G>), grid_for(B), dim3(kBlock), 0, s, *cfg, *st,   \
                         actions, B, k, off, events, n_events);                                 \
  }
  ORX_STEP_LIST(ORX_STEP)
#undef ORX_STEP
  return launch_status(name);
}

int orx_step(const orx_cfg_t* cfg, const orx_state_t* st, const int8_t* actions, int64_t n_games,
             uint64_t seed, int64_t game_offset, void* stream) {
  return launch_step(cfg, st, actions, nullptr, nullptr, n_games, seed, game_offset, stream,
                     "orx_step");
}

int orx_step_events(const orx_cfg_t* cfg, const orx_state_t* st, const int8_t* actions,
                    int32_t* events, int32_t* n_events, int64_t n_games, uint64_t seed,
                    int64_t game_offset, void* stream) {
  if (n_games > 0 && (!events || !n_events))
    return fail(ORX_EINVAL, "orx_step_events needs events and n_events");
  return launch_step(cfg, st, actions, events, n_events, n_games, seed, game_offset, stream,
                     "orx_step_events");
}

int orx_step_n(const orx_cfg_t* cfg, const orx_state_t* st, const int8_t* actions,
               int32_t n_ticks, int32_t* obs, int32_t obs_format, int64_t n_games, uint64_t seed,
               int64_t game_offset, void* stream) {
  return orx_step_n_ex(cfg, st, actions, n_ticks, obs, obs_format, n_games, seed, game_offset, 1,
                       stream);
}

int orx_step_n_ex(const orx_cfg_t* cfg, const orx_state_t* st, const int8_t* actions,
                  int32_t n_ticks, int32_t* obs, int32_t obs_format, int64_t n_games,
                  uint64_t seed, int64_t game_offset, int32_t concurrency, void* stream) {
  int r;
  if (concurrency < 1) return fail(ORX_EINVAL, "concurrency must be >= 1");
  if ((r = check_cfg(cfg)) || (r = check_sizes(n_games, game_offset))) return r;
  if (n_ticks < 0) return fail(ORX_EINVAL, "n_ticks < 0");
  if (obs_format != ORX_OBS_INT32 && obs_format != ORX_OBS_COMPACT)
    return fail(ORX_EINVAL, "unknown obs_format");
  if (obs && obs_format == ORX_OBS_COMPACT && (r = check_compact(cfg))) return r;
  if (cfg->rng == ORX_RNG_MT19937)
    return fail(ORX_EINVAL, "orx_step_n: stock-seed mode steps tick by tick (orx_step)");
  if (n_games == 0 || n_ticks == 0) return ORX_OK;
  if ((r = check_state(cfg, st, true))) return r;
  if (!actions) return fail(ORX_EINVAL, "actions is NULL");
  const uint32_t B = (uint32_t)n_games, off = (uint32_t)game_offset;
  const hipStream_t s = (hipStream_t)stream;
  const Key k = make_key(seed);
  const int nc = ncap_for(cfg->n_npcs);
  const bool grid = cfg->n_layouts > 0;
  // register NPCs on empty dungeons: the rollout's tick on the logged pairs
  // (ORX_STEP_N_GENERIC=1 forces the generic one, for A/B runs and tests)
  const char* gen_env = getenv("ORX_STEP_N_GENERIC");
  // (the buffer-store rows address one tick's rows with 32-bit offsets)
  const bool rows_fit = (uint64_t)B * ORX_OBS_FIELDS * 4u < (1ull << 31);
  if (moving_npcs(cfg)) {
#define ORX_STEP_N(N, G)                                                                        \
    if (nc == N && grid == G) {                                                                 \
      hipLaunchKernelGGL((step_n_kernel<N, G, true>), grid_for(B), dim3(kBlock), 0, s, *cfg,    \
                         *st, actions, n_ticks, obs, B, k, off, obs_format);                    \
      return launch_status("orx_step_n");                                                      \
    }
    ORX_MOV_NG_LIST(ORX_STEP_N)
#undef ORX_STEP_N
    return fail(ORX_EIO, "orx_step_n: no moving-NPC kernel instance for this configuration");
  }
  if (!grid && nc != kDense && rows_fit && !(gen_env && gen_env[0] == '1')) {
    const int rows = obs ? (obs_format == ORX_OBS_COMPACT ? 2 : 1) : 0;
    // the paired form (pair_rollout_kernel PM 6: two lanes per game, the
    // rollout's paired tick on the logged moves) for rows given under the
    // reference's rules, at any batch: two waves per SIMD over the device's
    // concurrent launches until the wave holds 32 games (C3, 65,536 games x
    // 128 ticks, int32 rows: 103-104 us against 114-116 for the one-lane
    // replay_kernel; as two 32,768-game stream shards at 32 games per wave
    // 85-86 us, at 16 -- the plan without the concurrency -- 207,
    // profiles/r06_v3 / r06_v4 ab_replay_paired.jsonl).  Env
    // ORX_REPLAY_PAIRED=0 keeps the one-lane form, for measurements.
    const char* pe = getenv("ORX_REPLAY_PAIRED");
    RolloutPlan pl;
    bool paired = rows != 0 && cfg->flags == 0 && cfg->n_layouts == 0 && paired_enabled() &&
                  cfg->width <= 256 && cfg->height <= 256 && !(pe && pe[0] == '0');
    if (paired) {
      const uint64_t simds = (uint64_t)device_simds();
      uint32_t L = 32;
      while (L > 8 && (uint64_t)B * (uint32_t)concurrency < 2 * simds * L) L >>= 1;
      if (const int o = lanes_override()) L = o < 32 ? (uint32_t)o : 32u;
      pl.lanes = L;
      pl.nt = L * 4u >= 128u;
      pl.paired = true;
    }
    if (paired) {
      const uint32_t lanes = pl.lanes, threads = (uint32_t)kRolloutBlock;
      const uint32_t per_block = threads / 64u * lanes;
      const dim3 blocks((B + per_block - 1) / per_block);
      int8_t* log = const_cast<int8_t*>(actions);  // (PM 6 reads it; the form never writes it)
#define ORX_PAIR_LOG(N, A, C)                                                                   \
      if (nc == N && (A == kStreamAux) == pl.nt && C == (rows == 2)) {                          \
        hipLaunchKernelGGL((pair_rollout_kernel<N, 6, A, false, C, false>), blocks,              \
                           dim3(threads), 0, s, *cfg, *st, n_ticks, obs, log, B, k, off, lanes,  \
                           0u);                                                                 \
        return launch_status("orx_step_n");                                                    \
      }
      ORX_PAIR_LOG(0, kStreamAux, false) ORX_PAIR_LOG(0, kPartialAux, false)
      ORX_PAIR_LOG(0, kStreamAux, true) ORX_PAIR_LOG(0, kPartialAux, true)
      ORX_PAIR_LOG(8, kStreamAux, false) ORX_PAIR_LOG(8, kPartialAux, false)
      ORX_PAIR_LOG(8, kStreamAux, true) ORX_PAIR_LOG(8, kPartialAux, true)
      ORX_PAIR_LOG(16, kStreamAux, false) ORX_PAIR_LOG(16, kPartialAux, false)
      ORX_PAIR_LOG(16, kStreamAux, true) ORX_PAIR_LOG(16, kPartialAux, true)
#undef ORX_PAIR_LOG
      return fail(ORX_EIO, "orx_step_n: no paired replay instance for this plan");
    }
    const uint32_t lanes = rollout_lanes(B);  // games per wave, as the rollout's plan
    const uint64_t threads = (((uint64_t)B + lanes - 1) / lanes) * 64u;
    const dim3 g((unsigned)((threads + kRolloutBlock - 1) / kRolloutBlock));
#define ORX_REPLAY(N, R, E)                                                                     \
    if (nc == N && rows == R && (cfg->flags != 0) == E) {                                       \
      hipLaunchKernelGGL((replay_kernel<N, R, E>), g, dim3(kRolloutBlock), 0, s, *cfg, *st,     \
                         actions, n_ticks, obs, B, k, off, lanes);                              \
      return launch_status("orx_step_n");                                                      \
    }
    ORX_REPLAY_LIST(ORX_REPLAY)
#undef ORX_REPLAY
  }
#define ORX_STEP_N(N, G)                                                                        \
  if (nc == N && grid == G) {                                                                   \
    hipLaunchKernelGGL((step_n_kernel<N, G>), grid_for(B), dim3(kBlock), 0, s, *cfg, *st,       \
                       actions, n_ticks, obs, B, k, off, obs_format);                           \
    return launch_status("orx_step_n");                                                        \
  }
  ORX_NG_LIST(ORX_STEP_N)
#undef ORX_STEP_N
  return fail(ORX_EIO, "orx_step_n: no kernel instance for this configuration");
}

int orx_policy(const orx_cfg_t* cfg, const orx_state_t* st, int32_t policy_p1, int32_t policy_p2,
               int8_t* actions, int64_t n_games, uint64_t seed, int64_t game_offset,
               void* stream) {
  int r;
  if ((r = check_cfg(cfg)) || (r = check_sizes(n_games, game_offset)) ||
      (r = check_policy(policy_p1)) || (r = check_policy(policy_p2)))
    return r;
  if (n_games == 0) return ORX_OK;
  if ((r = check_state(cfg, st, false))) return r;
  if (!actions) return fail(ORX_EINVAL, "actions is NULL");
  const uint32_t B = (uint32_t)n_games, off = (uint32_t)game_offset;
  if (cfg->rng == ORX_RNG_MT19937) {
    hipLaunchKernelGGL(mt_policy_kernel, grid_for(B), dim3(kBlock), 0, (hipStream_t)stream, *st,
                       policy_p1, policy_p2, actions, B);
    return launch_status("orx_policy");
  }
  hipLaunchKernelGGL(policy_kernel, grid_for(B), dim3(kBlock), 0, (hipStream_t)stream, *st,
                     policy_p1, policy_p2, actions, B, make_key(seed), off);
  return launch_status("orx_policy");
}

int orx_env_step(const orx_cfg_t* cfg, const orx_state_t* st, const void* actions,
                 int32_t action_bytes, int32_t action_cols, int32_t policy_p2, int8_t* act,
                 int32_t* obs, float* reward, uint8_t* done, int32_t* status, int64_t n_games,
                 uint64_t seed, int64_t game_offset, void* stream) {
  return orx_env_step_ex(cfg, st, actions, action_bytes, action_cols, policy_p2, act, obs, reward,
                         done, status, nullptr, n_games, seed, game_offset, stream);
}

int orx_env_step_args(const orx_env_step_args_t* a) {
  if (!a) return fail(ORX_EINVAL, "args is NULL");
  return orx_env_step_ex(a->cfg, a->st, a->actions, a->action_bytes, a->action_cols,
                         a->policy_p2, a->act, a->obs, a->reward, a->done, a->status,
                         a->bad_actions, a->n_games, a->seed, a->game_offset, a->stream);
}

int orx_env_step_ex(const orx_cfg_t* cfg, const orx_state_t* st, const void* actions,
                    int32_t action_bytes, int32_t action_cols, int32_t policy_p2, int8_t* act,
                    int32_t* obs, float* reward, uint8_t* done, int32_t* status,
                    uint32_t* bad_actions, int64_t n_games, uint64_t seed, int64_t game_offset,
                    void* stream) {
  int r;
  if ((r = check_cfg(cfg)) || (r = check_sizes(n_games, game_offset)) ||
      (r = check_policy(policy_p2)))
    return r;
  if (action_bytes != 1 && action_bytes != 2 && action_bytes != 4 && action_bytes != 8)
    return fail(ORX_EINVAL, "action_bytes must be 1, 2, 4 or 8");
  if (action_cols != 1 && action_cols != 2) return fail(ORX_EINVAL, "action_cols must be 1 or 2");
  if (action_cols == 1 && policy_p2 == ORX_POLICY_NONE)
    return fail(ORX_EINVAL, "action_cols 1 needs a policy for player 2 (ORX_POLICY_NONE: pass "
                            "both players' actions, action_cols 2)");
  if (cfg->rng == ORX_RNG_MT19937)
    return fail(ORX_EINVAL, "orx_env_step: stock-seed mode draws the bots' moves from the "
                            "games' own streams; use orx_policy + orx_step");
  if (n_games == 0) return ORX_OK;
  if ((r = check_state(cfg, st, true))) return r;
  if (!actions || !act || !obs || !reward || !done)
    return fail(ORX_EINVAL, "a pointer is NULL (only status and bad_actions may be)");
  const uint32_t B = (uint32_t)n_games, off = (uint32_t)game_offset;
  const hipStream_t s = (hipStream_t)stream;
  const Key k = make_key(seed);
  const int nc = ncap_for(cfg->n_npcs);
  const bool grid = cfg->n_layouts > 0;
  // the rows through LDS and 16-byte stores when obs is 16-byte aligned (a
  // torch allocation is; a view may not be: then direct stores), env
  // ORX_ENV_DIRECT_ROWS=1: direct stores, for measurements
  const char* dr = getenv("ORX_ENV_DIRECT_ROWS");
  const int32_t lds_rows = ((dr && dr[0] == '1') || ((uintptr_t)obs & 15u) != 0) ? 0 : 1;
  // games per wave: 64, or 32 where that still leaves at most two waves per
  // SIMD (env ORX_ENV_LANES = 64 / 32 overrides, for measurements)
  const char* le = getenv("ORX_ENV_LANES");
  const int lo = le ? atoi(le) : 0;
  const uint32_t env_lanes = (lo == 32 || lo == 64) ? (uint32_t)lo : 64u;
  const uint32_t per_blk = (uint32_t)kBlock / 64u * env_lanes;
  const dim3 env_grid((unsigned)((B + per_blk - 1) / per_blk));
  if (moving_npcs(cfg)) {
#define ORX_ENV(N, G)                                                                           \
    if (nc == N && grid == G) {                                                                 \
      hipLaunchKernelGGL((env_step_kernel<N, G, true, true>), env_grid, dim3(kBlock), 0, s,     \
                         *cfg, *st, actions, action_bytes, action_cols, policy_p2, act, obs,    \
                         reward, done, status, bad_actions, B, k, off, lds_rows, env_lanes);    \
      return launch_status("orx_env_step");                                                    \
    }
    ORX_MOV_NG_LIST(ORX_ENV)
#undef ORX_ENV
    return fail(ORX_EIO, "orx_env_step: no moving-NPC kernel instance for this configuration");
  }
#define ORX_ENV(N, G, X)                                                                        \
  if (nc == N && grid == G && (cfg->flags == 0 || X)) {                                        \
    hipLaunchKernelGGL((env_step_kernel<N, G, X>), env_grid, dim3(kBlock), 0, s, *cfg, *st,      \
                       actions, action_bytes, action_cols, policy_p2, act, obs, reward, done,   \
                       status, bad_actions, B, k, off, lds_rows, env_lanes);                    \
    return launch_status("orx_env_step");                                                      \
  }
  ORX_ENV_LIST(ORX_ENV)
#undef ORX_ENV
  return fail(ORX_EIO, "orx_env_step: no kernel instance for this configuration");
}

int orx_rollout(const orx_cfg_t* cfg, const orx_state_t* st, int32_t policy_p1, int32_t policy_p2,
                int32_t n_ticks, int32_t* obs, int8_t* act, int64_t n_games, uint64_t seed,
                int64_t game_offset, void* stream) {
  return orx_rollout_concurrent(cfg, st, policy_p1, policy_p2, n_ticks, obs, act, n_games, seed,
                                game_offset, 1, stream);
}

int orx_rollout_concurrent(const orx_cfg_t* cfg, const orx_state_t* st, int32_t policy_p1,
                           int32_t policy_p2, int32_t n_ticks, int32_t* obs, int8_t* act,
                           int64_t n_games, uint64_t seed, int64_t game_offset,
                           int32_t concurrency, void* stream) {
  return orx_rollout_ex(cfg, st, policy_p1, policy_p2, n_ticks, obs, act, ORX_OBS_INT32, n_games,
                        seed, game_offset, concurrency, stream);
}

int orx_rollout_ex(const orx_cfg_t* cfg, const orx_state_t* st, int32_t policy_p1,
                   int32_t policy_p2, int32_t n_ticks, int32_t* obs, int8_t* act,
                   int32_t obs_format, int64_t n_games, uint64_t seed, int64_t game_offset,
                   int32_t concurrency, void* stream) {
  int r;
  if (concurrency < 1) return fail(ORX_EINVAL, "concurrency must be >= 1");
  if ((r = check_cfg(cfg)) || (r = check_sizes(n_games, game_offset)) ||
      (r = check_policy(policy_p1)) || (r = check_policy(policy_p2)))
    return r;
  if (obs_format != ORX_OBS_INT32 && obs_format != ORX_OBS_COMPACT)
    return fail(ORX_EINVAL, "unknown obs_format");
  const bool cf = obs_format == ORX_OBS_COMPACT;
  if (cf && (r = check_compact(cfg))) return r;
  if (policy_p1 == ORX_POLICY_NONE || policy_p2 == ORX_POLICY_NONE)
    return fail(ORX_EINVAL, "orx_rollout needs an action producer for both players");
  if (n_ticks < 0) return fail(ORX_EINVAL, "n_ticks < 0");
  if (n_games == 0 || n_ticks == 0) return ORX_OK;
  if ((r = check_state(cfg, st, true))) return r;
  const uint32_t B = (uint32_t)n_games, off = (uint32_t)game_offset;
  const hipStream_t s = (hipStream_t)stream;
  const Key k = make_key(seed);
  // the buffer-addressed trajectory forms need one tick's obs rows below 2 GiB
  const bool grid = cfg->n_layouts > 0;
  const int nc = ncap_for(cfg->n_npcs);
  if (moving_npcs(cfg)) {  // the ordered tick with the enemy AI, one lane per game
    const bool mt = cfg->rng == ORX_RNG_MT19937;
    const uint32_t lanes = mov_lanes();
    const uint64_t threads = (((uint64_t)B + lanes - 1) / lanes) * 64u;
    const dim3 g((unsigned)((threads + kBlock - 1) / kBlock));
#define ORX_ROLLOUT(N, G, M)                                                                    \
    if (nc == N && grid == G && mt == M) {                                                      \
      hipLaunchKernelGGL((mov_rollout_kernel<N, G, M>), g, dim3(kBlock), 0, s, *cfg, *st,       \
                         policy_p1, policy_p2, n_ticks, obs, act, B, k, off, obs_format, lanes); \
      return launch_status("orx_rollout");                                                     \
    }
    ORX_MOV_ROLLOUT_LIST(ORX_ROLLOUT)
#undef ORX_ROLLOUT
    return fail(ORX_EIO, "orx_rollout: no moving-NPC kernel instance for this configuration");
  }
  if (cfg->rng == ORX_RNG_MT19937) {
#define ORX_ROLLOUT(N, G)                                                                       \
  if (nc == N && grid == G)                                                                     \
    hipLaunchKernelGGL((mt_rollout_kernel<N, G>), grid_for(B), dim3(kBlock), 0, s, *cfg, *st,   \
                       policy_p1, policy_p2, n_ticks, obs, act, B, k, off, obs_format);
    ORX_NG_LIST(ORX_ROLLOUT)
#undef ORX_ROLLOUT
    return launch_status("orx_rollout");
  }
  int pm = rollout_pm(cfg, policy_p1, policy_p2, B, obs && act);
  // compact rows: the buffer-store forms of PM 1 / 2 without a bank or dense
  // NPCs have compact instances; every other launch takes the generic form,
  // whose writer reads the format at run time
  if (cf && (pm >= 3 || grid || nc == kDense)) pm = 0;
  RolloutPlan plan = plan_rollout(cfg, pm, B, (uint32_t)concurrency);
  if (!plan.paired && pm >= 4) pm = 0;  // (the mixed-bot forms are paired only)
  // dynamic LDS: the bank's tiles when they fit the device's per-workgroup
  // limit (160 KiB on gfx950, above 64 KiB with the opt-in raise)
  const uint64_t tiles = grid ? (uint64_t)cfg->n_layouts * (uint64_t)(cfg->width * cfg->height) : 0;
  uint32_t lds_n = (grid && bank_in_lds(cfg)) ? (uint32_t)tiles : 0u;
  const uint32_t lds_max = device_lds_per_block();
  // the paired form (two lanes per game, pair_rollout_kernel): K <= 16 NPCs
  // in registers, a bank only with its tiles in LDS (the paired tick reads
  // them nowhere else), the RandomBot / StaircaseBot / character trajectory
  // forms, at most 32 games per wave (env ORX_ROLLOUT_PAIRED=0 turns it off)
  if (plan.paired) {
    if (grid && !lds_n) return fail(ORX_EIO, "orx_rollout: a paired bank launch without LDS tiles");
    const uint32_t lanes = plan.lanes;
    const uint32_t threads = pair_threads(cfg, lanes, lds_n);
    const uint32_t per_block = threads / 64u * lanes;
    const bool nt = plan.nt;
    const dim3 blocks((B + per_block - 1) / per_block);
    const bool sepd = pm == 2 && (cfg->flags & ORX_EXT_SEPARATION_DAMAGE) != 0;
    // a refused limit raise (above the default 64 KiB) drops the launch to
    // the one-lane form below with the tiles in global memory -- never a
    // paired launch without them
    bool refused = false;
#define ORX_PAIR(N, P, A, S, C, G)                                                              \
    if (nc == N && pm == P && (A == kStreamAux) == nt && S == sepd && C == cf && G == grid) {   \
      auto* kfn = &pair_rollout_kernel<N, P, A, S, C, G>;                                       \
      if (!raise_lds(reinterpret_cast<const void*>(kfn), lds_n)) {                              \
        refused = true;                                                                         \
      } else {                                                                                  \
        hipLaunchKernelGGL(kfn, blocks, dim3(threads), lds_n, s, *cfg, *st, n_ticks, obs, act, B, \
                           k, off, lanes, lds_n);                                               \
        return launch_status("orx_rollout");                                                    \
      }                                                                                         \
    }
    ORX_PAIR_LIST(ORX_PAIR)
#undef ORX_PAIR
    if (!refused) return fail(ORX_EIO, "orx_rollout: no paired kernel instance for this plan");
    plan.paired = false;
    if (pm >= 4) pm = 0;
    plan.lanes = rollout_lanes(B);
    plan.nt = plan.lanes * 4u >= 128u;
    lds_n = 0u;
  }
  const uint32_t lanes = plan.lanes;
  const uint32_t threads = rollout_threads(B, lanes);
  const uint32_t per_block = threads / 64u * lanes;
  const bool nt = plan.nt;
  uint32_t lds = (uint32_t)((lds_n + 15u) & ~15u);
  // dense NPCs: one occupancy bitmap per game of the block after the tiles,
  // when they fit the device's per-workgroup LDS (a workgroup may take all
  // 160 KiB on gfx950); the bitmaps are an optimization -- without them the
  // kernel reads the occupancy grid from HBM -- so a part with less LDS, or
  // a refused limit raise, launches without them instead of failing
  uint32_t lds_bits = 0;
  if (nc == kDense && !getenv("ORX_NO_LDS_BITS")) {
    const uint32_t bb = (uint32_t)((cfg->width * cfg->height + 31) / 32) * 4u;
    if ((uint64_t)lds + (uint64_t)per_block * bb <= lds_max) {
      lds_bits = bb;
      lds += per_block * bb;
    }
  }
  // a refused limit raise: first without the bitmaps, then without the tiles
  // (rollout_kernel reads a bank's tiles from global memory when lds_n is 0)
#define ORX_ROLLOUT_AC(N, P, G, A, C)                                                           \
  if (nc == N && pm == P && grid == G && (P == 0 || (A == kStreamAux) == nt) &&                 \
      (P == 0 || C == cf)) {                                                                    \
    const void* kfn = reinterpret_cast<const void*>(&rollout_kernel<N, P, G, A, C>);            \
    if (!raise_lds(kfn, lds) && lds_bits) {                                                     \
      lds -= per_block * lds_bits;                                                              \
      lds_bits = 0;                                                                             \
    }                                                                                           \
    if (!raise_lds(kfn, lds)) {                                                                 \
      lds_n = 0u;                                                                               \
      lds = 0u;                                                                                 \
    }                                                                                           \
    hipLaunchKernelGGL((rollout_kernel<N, P, G, A, C>), dim3((B + per_block - 1) / per_block),  \
                       dim3(threads), lds, s, *cfg, *st,                                        \
                       policy_p1, policy_p2, n_ticks, obs, act, B, k, off, lanes, lds_n,        \
                       lds_bits, obs_format);                                                   \
    return launch_status("orx_rollout");                                                        \
  }
  ORX_ROLLOUT_LIST(ORX_ROLLOUT_AC)
#undef ORX_ROLLOUT_AC
  return fail(ORX_EIO, "orx_rollout: no rollout kernel instance for this plan");
}

#ifdef ORX_STAMPS
int orx_diag_stamps_clear(void) {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_stamps)) != hipSuccess) return -1;
  return hipMemset(p, 0, sizeof(g_stamps)) == hipSuccess ? 0 : -1;
}
int orx_diag_stamps(uint64_t* host, int64_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost)
             == hipSuccess ? 0 : -1;
}
#endif

int orx_dungeon_spawn(const orx_cfg_t* cfg, const orx_state_t* st, const uint32_t* game_ids,
                      const int32_t* episodes, const int32_t* depths, const int32_t* gens,
                      int32_t* sx, int32_t* sy, int32_t* layout, int64_t n, uint64_t seed,
                      void* stream) {
  int r;
  if ((r = check_cfg(cfg))) return r;
  if (n < 0 || n > 0x7FFFFFFFLL - kBlock) return fail(ORX_EINVAL, "bad n");
  if (cfg->rng == ORX_RNG_MT19937)
    return fail(ORX_EINVAL, "stock-seed dungeons come from the games' numpy streams, not keys");
  if (n == 0) return ORX_OK;
  if (!game_ids || !episodes || !depths || !gens || !sx || !sy)
    return fail(ORX_EINVAL, "a pointer is NULL");
  orx_state_t bank{};
  if (cfg->n_layouts > 0) {
    if (!st || !st->bank_tiles || !st->bank_ground || !st->bank_meta)
      return fail(ORX_EINVAL, "n_layouts > 0 needs the bank_* arrays");
    bank.bank_tiles = st->bank_tiles;
    bank.bank_ground = st->bank_ground;
    bank.bank_meta = st->bank_meta;
  }
  if (cfg->n_layouts > 0)
    hipLaunchKernelGGL(stairs_kernel<true>, grid_for(n), dim3(kBlock), 0, (hipStream_t)stream,
                       *cfg, bank, game_ids, episodes, depths, gens, sx, sy, layout, (uint32_t)n,
                       make_key(seed));
  else
    hipLaunchKernelGGL(stairs_kernel<false>, grid_for(n), dim3(kBlock), 0, (hipStream_t)stream,
                       *cfg, bank, game_ids, episodes, depths, gens, sx, sy, layout, (uint32_t)n,
                       make_key(seed));
  return launch_status("orx_dungeon_spawn");
}

int orx_dungeon_stairs(const orx_cfg_t* cfg, const uint32_t* game_ids, const int32_t* episodes,
                       const int32_t* depths, const int32_t* gens, int32_t* sx, int32_t* sy,
                       int64_t n, uint64_t seed, void* stream) {
  if (cfg && cfg->n_layouts > 0)
    return fail(ORX_EINVAL, "a dungeon bank needs orx_dungeon_spawn");
  return orx_dungeon_spawn(cfg, nullptr, game_ids, episodes, depths, gens, sx, sy, nullptr, n, seed,
                           stream);
}

}  // extern "C"
#endif  // ORX_HOST_TU
