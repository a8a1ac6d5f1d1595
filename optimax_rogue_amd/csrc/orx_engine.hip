// orx_engine.hip -- MI355X (gfx950) batched tick engine for Optimax Rogue.
//
// One lane = one game.  All per-game state is struct-of-arrays with the batch
// axis contiguous, so every field load/store of a wavefront is one coalesced
// 256-byte access.  The tick is integer/branch work; there is nothing for the
// matrix cores.  The kernels are HBM-bound (step, policy) or issue-bound
// (rollout with state held in registers); see DESIGN.md for the byte
// accounting.
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
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../../include/orx.h"

namespace {

// ---------------------------------------------------------------------------
// Philox4x32-10 and the reference's bounded-integer transforms
// ---------------------------------------------------------------------------
enum : uint32_t { PUR_INIT = 1, PUR_DUNGEON = 2, PUR_SHUFFLE = 3, PUR_SPAWN = 4, PUR_POLICY = 5 };
constexpr uint32_t kWordCap = 4096;  // per stream; exceeding it stops the game

struct Key {
  uint32_t k0, k1;
};

__device__ __forceinline__ void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                       Key key, uint32_t& o0, uint32_t& o1, uint32_t& o2,
                                       uint32_t& o3) {
  uint32_t k0 = key.k0, k1 = key.k1;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0);
    const uint32_t lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2);
    const uint32_t lo1 = 0xCD9E8D57u * c2;
    c0 = hi1 ^ c1 ^ k0;
    c1 = lo1;
    c2 = hi0 ^ c3 ^ k1;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  o0 = c0; o1 = c1; o2 = c2; o3 = c3;
}

// A word stream: counter (game, episode, c2, purpose<<28 | gen<<24 | block).
struct Stream {
  uint32_t c0, c1, c2, c3;
  uint32_t idx;
  uint32_t w0, w1, w2, w3;

  __device__ __forceinline__ void init(uint32_t game, uint32_t ep, uint32_t cc2, uint32_t purpose,
                                       uint32_t gen) {
    c0 = game; c1 = ep; c2 = cc2; c3 = (purpose << 28) | (gen << 24); idx = 0;
  }
  __device__ __forceinline__ uint32_t next(Key key) {
    const uint32_t j = idx & 3u;
    if (j == 0) philox(c0, c1, c2, c3 | (idx >> 2), key, w0, w1, w2, w3);
    ++idx;
    return j == 0 ? w0 : j == 1 ? w1 : j == 2 ? w2 : w3;
  }
};

__device__ __forceinline__ int bit_length(uint32_t n) { return n ? 32 - __clz(n) : 0; }

// CPython Random._randbelow_with_getrandbits(n): getrandbits(k) = w >> (32-k).
__device__ __forceinline__ uint32_t py_randbelow(Stream& s, Key key, uint32_t n, bool& err) {
  const int k = bit_length(n);
  for (uint32_t t = 0; t < kWordCap; ++t) {
    const uint32_t r = s.next(key) >> (32 - k);
    if (r < n) return r;
  }
  err = true;
  return 0;
}

// numpy legacy RandomState.randint(low, high), masked rejection on 32-bit words.
__device__ __forceinline__ int32_t np_randint(Stream& s, Key key, int32_t low, int32_t high,
                                              bool& err) {
  const uint32_t rng = (uint32_t)(high - 1 - low);
  if (rng == 0) return low;
  const uint32_t mask = 0xFFFFFFFFu >> __clz(rng);
  for (uint32_t t = 0; t < kWordCap; ++t) {
    const uint32_t v = s.next(key) & mask;
    if (v <= rng) return low + (int32_t)v;
  }
  err = true;
  return low;
}

// ---------------------------------------------------------------------------
// Per-game registers
// ---------------------------------------------------------------------------
struct Player {
  int32_t x, y, d, hp, sx, sy;
  int32_t move;   // validated move for this tick
  int32_t start;  // start depth of the episode (dungeon presence rule)
};

struct Cfg {  // device copy of orx_cfg_t plus derived constants
  int32_t W, H, despawn, max_ticks, start_mode, d1, d2, K;
  int32_t npc_hp, player_hp, player_dmg_net, autoreset;
  int32_t n_ground;  // (W-2)(H-2) - 1 Ground tiles per dungeon
};

struct Deltas {  // counter / return increments, flushed once per launch
  int32_t c0, c1, c2, c3, ret, eps;
};

// NPC slots: positions either cached in registers (rollout) or read from HBM
// on demand (step).  Dead slots are never consulted (alive mask).
template <bool kReg>
struct Npcs {
  uint32_t alive;
  uint32_t pos[kReg ? ORX_MAX_NPCS / 2 : 1];  // two packed u16 per register
  const uint16_t* gpos;
  int8_t* ghp;
  int64_t B, i;
  int32_t K;

  __device__ __forceinline__ void load(const orx_state_t& st, int32_t KK, int64_t BB, int64_t ii) {
    K = KK; B = BB; i = ii;
    gpos = st.npc_pos; ghp = st.npc_health;
    alive = K ? st.npc_alive[i] : 0u;
    if constexpr (kReg) {
#pragma unroll
      for (int k = 0; k < ORX_MAX_NPCS / 2; ++k) pos[k] = 0xFFFFFFFFu;
#pragma unroll
      for (int k = 0; k < ORX_MAX_NPCS; ++k)
        if (k < K) set_pos_reg(k, gpos[(int64_t)k * B + i]);
    }
  }
  __device__ __forceinline__ void set_pos_reg(int k, uint32_t v) {
    if constexpr (kReg) {
      const int r = k >> 1, sh = (k & 1) * 16;
      pos[r] = (pos[r] & ~(0xFFFFu << sh)) | ((v & 0xFFFFu) << sh);
    }
  }
  // Slot of the NPC at (x, y) on the NPC depth, or -1.
  __device__ __forceinline__ int find(int32_t x, int32_t y) const {
    if (!alive) return -1;
    const uint32_t key = (uint32_t)(x & 0xFF) | ((uint32_t)(y & 0xFF) << 8);
    if (x < 0 || y < 0 || x > 255 || y > 255) return -1;
    int hit = -1;
    if constexpr (kReg) {
#pragma unroll
      for (int k = 0; k < ORX_MAX_NPCS; ++k) {
        const uint32_t v = (pos[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu;
        if (k < K && ((alive >> k) & 1u) && v == key) hit = k;
      }
    } else {
      for (int k = 0; k < K; ++k)
        if (((alive >> k) & 1u) && (uint32_t)gpos[(int64_t)k * B + i] == key) hit = k;
    }
    return hit;
  }
  __device__ __forceinline__ void store_pos(int k, uint32_t v) {
    const_cast<uint16_t*>(gpos)[(int64_t)k * B + i] = (uint16_t)v;
    set_pos_reg(k, v);
  }
};

// Dungeon staircase from the keyed stream (episode, depth, generation):
// EmptyDungeonGenerator.spawn_dungeon draws randint(1, W-2) then randint(1, H-2).
__device__ __forceinline__ void dungeon_stair(const Cfg& c, Key key, uint32_t game, uint32_t ep,
                                              int32_t depth, uint32_t gen, int32_t& sx,
                                              int32_t& sy, bool& err) {
  Stream s;
  s.init(game, ep, (uint32_t)depth, PUR_DUNGEON, gen);
  sx = np_randint(s, key, 1, c.W - 2, err);
  sy = np_randint(s, key, 1, c.H - 2, err);
}

// get_random_unblocked on the dungeon with staircase (sx, sy).
__device__ __forceinline__ void random_ground(const Cfg& c, Stream& s, Key key, int32_t sx,
                                              int32_t sy, int32_t& x, int32_t& y, bool& err) {
  const int32_t ih = c.H - 2;
  const int32_t ch = np_randint(s, key, 0, c.n_ground, err);
  const int32_t s_idx = (sx - 1) * ih + (sy - 1);
  const int32_t ci = ch + (ch >= s_idx ? 1 : 0);
  x = 1 + ci / ih;
  y = 1 + ci - (ci / ih) * ih;
}

__device__ __forceinline__ void calc_pos(int32_t x, int32_t y, int32_t m, int32_t& nx, int32_t& ny) {
  nx = x + (m == ORX_MOVE_RIGHT) - (m == ORX_MOVE_LEFT);
  ny = y + (m == ORX_MOVE_DOWN) - (m == ORX_MOVE_UP);
}

__device__ __forceinline__ bool blocked(const Cfg& c, int32_t x, int32_t y) {
  return x <= 0 || x >= c.W - 1 || y <= 0 || y >= c.H - 1;
}

// ---------------------------------------------------------------------------
// Game start (setup_game + NPC spawner)
// ---------------------------------------------------------------------------
template <bool kReg>
__device__ __forceinline__ void setup_game(const Cfg& c, Key key, uint32_t game, uint32_t ep,
                                           Player& p1, Player& p2, Npcs<kReg>& npc,
                                           int32_t& tick, int32_t& status) {
  bool err = false;
  Stream s;
  s.init(game, ep, 0, PUR_INIT, 0);
  if (c.start_mode == ORX_START_SEPARATED) {
    p1.d = c.d1; p2.d = c.d2;
    dungeon_stair(c, key, game, ep, c.d1, 0, p1.sx, p1.sy, err);
    dungeon_stair(c, key, game, ep, c.d2, 0, p2.sx, p2.sy, err);
    random_ground(c, s, key, p1.sx, p1.sy, p1.x, p1.y, err);
    random_ground(c, s, key, p2.sx, p2.sy, p2.x, p2.y, err);
  } else {
    p1.d = 0; p2.d = 0;
    dungeon_stair(c, key, game, ep, 0, 0, p1.sx, p1.sy, err);
    p2.sx = p1.sx; p2.sy = p1.sy;
    random_ground(c, s, key, p1.sx, p1.sy, p1.x, p1.y, err);
    for (uint32_t t = 0; t < kWordCap; ++t) {
      random_ground(c, s, key, p2.sx, p2.sy, p2.x, p2.y, err);
      if (p2.x != p1.x || p2.y != p1.y) break;
      if (t + 1 == kWordCap) err = true;
    }
  }
  p1.start = p1.d; p2.start = p2.d;
  p1.hp = c.player_hp; p2.hp = c.player_hp;
  // NPC spawner: K NPCs on player 1's start depth, redrawn while occupied.
  uint32_t alive = 0;
  for (int k = 0; k < c.K; ++k) {
    int32_t x = 0, y = 0;
    for (uint32_t t = 0; t < kWordCap; ++t) {
      random_ground(c, s, key, p1.sx, p1.sy, x, y, err);
      bool occ = (x == p1.x && y == p1.y) || (p2.d == p1.d && x == p2.x && y == p2.y);
      for (int j = 0; j < k; ++j) {
        const uint32_t v = npc.gpos[(int64_t)j * npc.B + npc.i];
        occ = occ || (v == ((uint32_t)x | ((uint32_t)y << 8)));
      }
      if (!occ) break;
      if (t + 1 == kWordCap) err = true;
    }
    npc.store_pos(k, (uint32_t)x | ((uint32_t)y << 8));
    npc.ghp[(int64_t)k * npc.B + npc.i] = (int8_t)c.npc_hp;
    alive |= 1u << k;
  }
  npc.alive = alive;
  tick = 1;
  status = err ? ORX_STATUS_RNG_EXHAUSTED : ORX_IN_PROGRESS;
}

// ---------------------------------------------------------------------------
// The tick
// ---------------------------------------------------------------------------
// Dungeon presence when `self` enters depth nd (derivation in DESIGN.md):
//   Unreachable: World has nd iff the other player has been on nd
//                (other.start <= nd <= other.d); generation is always 0.
//   Unused:      World == {p1.d, p2.d}, so nd is present iff other.d == nd;
//                a fresh copy is generation 1 iff the other player already
//                passed through nd (other.start <= nd < other.d).
template <bool kReg>
__device__ __forceinline__ void descend(const Cfg& c, Key key, uint32_t game, uint32_t ep,
                                        Player& self, const Player& other, Npcs<kReg>& npc,
                                        Stream& spawn, Deltas& dl, bool& err) {
  const int32_t nd = self.d + 1;
  bool present;
  uint32_t gen = 0;
  if (c.despawn == ORX_DESPAWN_UNREACHABLE) {
    present = other.start <= nd && nd <= other.d;
  } else {
    present = other.d == nd;
    gen = (!present && other.start <= nd && nd < other.d) ? 1u : 0u;
  }
  int32_t sx, sy;
  if (present && other.d == nd) {
    sx = other.sx; sy = other.sy;
  } else {
    dungeon_stair(c, key, game, ep, nd, gen, sx, sy, err);
  }
  if (!present) dl.c2 += 1;
  const bool npc_depth = nd == c.d1 && npc.alive;
  int32_t x = 0, y = 0;
  for (uint32_t t = 0; t < kWordCap; ++t) {
    random_ground(c, spawn, key, sx, sy, x, y, err);
    bool occ = other.d == nd && other.x == x && other.y == y;
    if (!occ && npc_depth) occ = npc.find(x, y) >= 0;
    if (!occ) break;
    if (t + 1 == kWordCap) err = true;
  }
  self.d = nd; self.x = x; self.y = y; self.sx = sx; self.sy = sy;
  dl.c1 += 1;
}

// handle_move for `self`; `self_first` = self acted before `other`.
template <bool kReg>
__device__ __forceinline__ void handle_move(const Cfg& c, Key key, uint32_t game, uint32_t ep,
                                            Player& self, Player& other, Npcs<kReg>& npc,
                                            Stream& spawn, Deltas& dl, int& hit0, int& hit1,
                                            bool& err) {
  if (self.move == ORX_MOVE_STAY) return;
  int32_t tx, ty;
  calc_pos(self.x, self.y, self.move, tx, ty);
  const bool occ_other = other.d == self.d && other.x == tx && other.y == ty;
  int slot = -1;
  if (!occ_other && self.d == c.d1) slot = npc.find(tx, ty);
  if (!occ_other && slot < 0) {
    if (tx == self.sx && ty == self.sy) {
      descend(c, key, game, ep, self, other, npc, spawn, dl, err);
    } else {
      self.x = tx; self.y = ty;
    }
    return;
  }
  // Occupied: Block / Parry / Ambush / Flee (updater.py:222-243).  Without a
  // Modifier subclass every flag deals og_dmg = damage - armor of the attacker.
  dl.c0 += 1;
  const int32_t dmg = c.player_dmg_net;
  if (occ_other) {
    if (dmg > 0) other.hp -= dmg;
  } else {
    if (dmg > 0) {
      int8_t* h = &npc.ghp[(int64_t)slot * npc.B + npc.i];
      *h = (int8_t)(*h - dmg);
    }
    if (hit0 < 0) hit0 = slot; else hit1 = slot;
  }
}

// One Updater.update for an in-progress game with validated raw moves a1, a2.
template <bool kReg>
__device__ __forceinline__ void tick_game(const Cfg& c, Key key, uint32_t game, uint32_t ep,
                                          Player& p1, Player& p2, Npcs<kReg>& npc,
                                          int32_t& tick, int32_t& status, Deltas& dl) {
  bool err = false;
  // illegal moves become Stay (updater.py:89-98)
  int32_t nx, ny;
  calc_pos(p1.x, p1.y, p1.move, nx, ny);
  if (blocked(c, nx, ny)) p1.move = ORX_MOVE_STAY;
  calc_pos(p2.x, p2.y, p2.move, nx, ny);
  if (blocked(c, nx, ny)) p2.move = ORX_MOVE_STAY;

  // random.shuffle of the two players: p1 first iff randbelow(2) == 1
  // (updater.py:114).  The NPC shuffle (:127) draws later words of the same
  // per-tick stream and only orders Stay-ing NPCs, so it has no observable
  // effect and is not evaluated.
  Stream sh;
  sh.init(game, ep, (uint32_t)tick, PUR_SHUFFLE, 0);
  const bool p1_first = py_randbelow(sh, key, 2, err) == 1;

  Stream spawn;
  spawn.init(game, ep, (uint32_t)tick, PUR_SPAWN, 0);
  int hit0 = -1, hit1 = -1;
  // Resolve in initiative order with static register indices: A acts first.
  Player A = p1_first ? p1 : p2;
  Player Bp = p1_first ? p2 : p1;
  handle_move(c, key, game, ep, A, Bp, npc, spawn, dl, hit0, hit1, err);
  handle_move(c, key, game, ep, Bp, A, npc, spawn, dl, hit0, hit1, err);
  p1 = p1_first ? A : Bp;
  p2 = p1_first ? Bp : A;

  // NPC death sweep (updater.py:136-145): only NPCs hit this tick can die.
  if (hit0 >= 0) {
    const int8_t h0 = npc.ghp[(int64_t)hit0 * npc.B + npc.i];
    if (h0 <= 0 && ((npc.alive >> hit0) & 1u)) { npc.alive &= ~(1u << hit0); dl.c3 += 1; }
    if (hit1 >= 0) {
      const int8_t h1 = npc.ghp[(int64_t)hit1 * npc.B + npc.i];
      if (h1 <= 0 && ((npc.alive >> hit1) & 1u)) { npc.alive &= ~(1u << hit1); dl.c3 += 1; }
    }
  }
  tick += 1;
  if (p1.hp <= 0)
    status = p2.hp <= 0 ? ORX_TIE : ORX_PLAYER2_WIN;
  else if (p2.hp <= 0)
    status = ORX_PLAYER1_WIN;
  else if (c.max_ticks && tick >= c.max_ticks)
    status = ORX_TIE;
  else
    status = ORX_IN_PROGRESS;
  if (err) status = ORX_STATUS_RNG_EXHAUSTED;
  if (status != ORX_IN_PROGRESS) {
    if (status == ORX_PLAYER1_WIN) dl.ret += 1;
    if (status == ORX_PLAYER2_WIN) dl.ret -= 1;
    if (status >= ORX_PLAYER1_WIN && status <= ORX_TIE) dl.eps += 1;
  }
}

// RandomBot / StaircaseBot for both players (stream POLICY keyed by tick).
__device__ __forceinline__ void policy_pair(Key key, uint32_t game, uint32_t ep, int32_t tick,
                                            int32_t pol1, int32_t pol2, const Player& p1,
                                            const Player& p2, int32_t& a1, int32_t& a2) {
  Stream s;
  s.init(game, ep, (uint32_t)tick, PUR_POLICY, 0);
  bool err = false;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int32_t pol = p == 0 ? pol1 : pol2;
    const Player& me = p == 0 ? p1 : p2;
    int32_t a = p == 0 ? a1 : a2;
    if (pol == ORX_POLICY_RANDOM) {
      a = 1 + (int32_t)py_randbelow(s, key, 5, err);
    } else if (pol == ORX_POLICY_STAIRCASE) {
      const int32_t dx = me.sx - me.x, dy = me.sy - me.y;
      const int32_t adx = dx < 0 ? -dx : dx, ady = dy < 0 ? -dy : dy;
      if (adx > ady) a = dx > 0 ? ORX_MOVE_RIGHT : ORX_MOVE_LEFT;
      else a = dy > 0 ? ORX_MOVE_DOWN : ORX_MOVE_UP;
    } else if (pol == ORX_POLICY_STAY) {
      a = ORX_MOVE_STAY;
    }
    if (p == 0) a1 = a; else a2 = a;
  }
}

// ---------------------------------------------------------------------------
// SoA load / store helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load_players(const orx_state_t& st, int64_t B, int64_t i,
                                             Player& p1, Player& p2) {
  p1.x = st.p_x[i];           p2.x = st.p_x[B + i];
  p1.y = st.p_y[i];           p2.y = st.p_y[B + i];
  p1.d = st.p_depth[i];       p2.d = st.p_depth[B + i];
  p1.hp = st.p_health[i];     p2.hp = st.p_health[B + i];
  p1.sx = st.st_x[i];         p2.sx = st.st_x[B + i];
  p1.sy = st.st_y[i];         p2.sy = st.st_y[B + i];
}

__device__ __forceinline__ void store_players(const orx_state_t& st, int64_t B, int64_t i,
                                              const Player& p1, const Player& p2,
                                              bool stairs) {
  st.p_x[i] = p1.x;           st.p_x[B + i] = p2.x;
  st.p_y[i] = p1.y;           st.p_y[B + i] = p2.y;
  st.p_depth[i] = p1.d;       st.p_depth[B + i] = p2.d;
  st.p_health[i] = p1.hp;     st.p_health[B + i] = p2.hp;
  if (stairs) {
    st.st_x[i] = p1.sx;       st.st_x[B + i] = p2.sx;
    st.st_y[i] = p1.sy;       st.st_y[B + i] = p2.sy;
  }
}

__device__ __forceinline__ void flush_deltas(const orx_state_t& st, int64_t B, int64_t i,
                                             const Deltas& dl) {
  if (st.counters && (dl.c0 | dl.c1 | dl.c2 | dl.c3)) {
    st.counters[i] += dl.c0;
    st.counters[B + i] += dl.c1;
    st.counters[2 * B + i] += dl.c2;
    st.counters[3 * B + i] += dl.c3;
  }
  if (dl.eps) {
    st.ret_sum[i] += dl.ret;
    st.ep_count[i] += dl.eps;
  }
}

__device__ __forceinline__ Cfg make_cfg(const orx_cfg_t& h) {
  Cfg c;
  c.W = h.width; c.H = h.height; c.despawn = h.despawn; c.max_ticks = h.max_ticks;
  c.start_mode = h.start_mode;
  c.d1 = h.start_mode == ORX_START_SEPARATED ? h.p1_depth : 0;
  c.d2 = h.start_mode == ORX_START_SEPARATED ? h.p2_depth : 0;
  c.K = h.n_npcs; c.npc_hp = h.npc_health; c.player_hp = h.player_health;
  c.player_dmg_net = h.player_damage - h.player_armor;
  c.autoreset = h.autoreset;
  c.n_ground = (h.width - 2) * (h.height - 2) - 1;
  return c;
}

__device__ __forceinline__ bool valid_move(int32_t m) {
  return m >= ORX_MOVE_UP && m <= ORX_MOVE_STAY;
}

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) reset_kernel(orx_cfg_t hc, orx_state_t st,
                                                    const uint8_t* __restrict__ mask, int64_t B,
                                                    Key key, int64_t off) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  if (mask && !mask[i]) return;
  const Cfg c = make_cfg(hc);
  const uint32_t game = (uint32_t)(off + i);
  const uint32_t ep = (uint32_t)st.episode[i];
  Player p1, p2;
  Npcs<false> npc;
  npc.load(st, 0, B, i);
  npc.K = c.K;
  int32_t tick, status;
  setup_game(c, key, game, ep, p1, p2, npc, tick, status);
  store_players(st, B, i, p1, p2, true);
  st.tick[i] = tick;
  st.status[i] = status;
  if (c.K) st.npc_alive[i] = npc.alive;
}

__global__ void __launch_bounds__(256) step_kernel(orx_cfg_t hc, orx_state_t st,
                                                   const int8_t* __restrict__ actions, int64_t B,
                                                   Key key, int64_t off) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const Cfg c = make_cfg(hc);
  const uint32_t game = (uint32_t)(off + i);
  int32_t status = st.status[i];
  Npcs<false> npc;
  Player p1, p2;
  if (status != ORX_IN_PROGRESS) {
    if (!c.autoreset) return;
    const uint32_t ep = (uint32_t)st.episode[i] + 1u;
    npc.load(st, 0, B, i);
    npc.K = c.K;
    int32_t tick;
    setup_game(c, key, game, ep, p1, p2, npc, tick, status);
    store_players(st, B, i, p1, p2, true);
    st.tick[i] = tick;
    st.status[i] = status;
    st.episode[i] = (int32_t)ep;
    if (c.K) st.npc_alive[i] = npc.alive;
    return;
  }
  const uint16_t a = reinterpret_cast<const uint16_t*>(actions)[i];
  p1.move = (int8_t)(a & 0xFF);
  p2.move = (int8_t)(a >> 8);
  if (!valid_move(p1.move) || !valid_move(p2.move)) {
    st.status[i] = ORX_STATUS_BAD_ACTION;
    return;
  }
  const uint32_t ep = (uint32_t)st.episode[i];
  int32_t tick = st.tick[i];
  load_players(st, B, i, p1, p2);
  p1.start = c.d1; p2.start = c.d2;
  npc.load(st, c.K, B, i);
  Deltas dl = {0, 0, 0, 0, 0, 0};
  tick_game(c, key, game, ep, p1, p2, npc, tick, status, dl);
  store_players(st, B, i, p1, p2, dl.c1 != 0);
  st.tick[i] = tick;
  st.status[i] = status;
  if (dl.c3) st.npc_alive[i] = npc.alive;
  flush_deltas(st, B, i, dl);
}

__global__ void __launch_bounds__(256) policy_kernel(orx_cfg_t hc, orx_state_t st, int32_t pol1,
                                                     int32_t pol2, int8_t* __restrict__ actions,
                                                     int64_t B, Key key, int64_t off) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const uint32_t game = (uint32_t)(off + i);
  Player p1, p2;
  const bool need_pos = pol1 == ORX_POLICY_STAIRCASE || pol2 == ORX_POLICY_STAIRCASE;
  if (need_pos) {
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
  policy_pair(key, game, ep, tick, pol1, pol2, p1, p2, a1, a2);
  out[i] = (uint16_t)((uint32_t)(uint8_t)a1 | ((uint32_t)(uint8_t)a2 << 8));
}

// Fused rollout: n_ticks x (policy, step); state and NPC positions stay in
// registers; tick t's observation is streamed out to obs/act.
__global__ void __launch_bounds__(256) rollout_kernel(orx_cfg_t hc, orx_state_t st, int32_t pol1,
                                                      int32_t pol2, int32_t n_ticks,
                                                      int32_t* __restrict__ obs,
                                                      int8_t* __restrict__ act, int64_t B,
                                                      Key key, int64_t off) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const Cfg c = make_cfg(hc);
  const uint32_t game = (uint32_t)(off + i);
  Player p1, p2;
  load_players(st, B, i, p1, p2);
  p1.start = c.d1; p2.start = c.d2;
  int32_t tick = st.tick[i];
  int32_t status = st.status[i];
  uint32_t ep = (uint32_t)st.episode[i];
  Npcs<true> npc;
  npc.load(st, c.K, B, i);
  Deltas dl = {0, 0, 0, 0, 0, 0};
  bool stairs_dirty = false;
  for (int32_t t = 0; t < n_ticks; ++t) {
    int32_t a1 = ORX_MOVE_STAY, a2 = ORX_MOVE_STAY;
    policy_pair(key, game, ep, tick, pol1, pol2, p1, p2, a1, a2);
    if (status != ORX_IN_PROGRESS) {
      if (c.autoreset) {
        ep += 1;
        setup_game(c, key, game, ep, p1, p2, npc, tick, status);
        stairs_dirty = true;
      }
    } else if (!valid_move(a1) || !valid_move(a2)) {
      status = ORX_STATUS_BAD_ACTION;
    } else {
      p1.move = a1; p2.move = a2;
      const int32_t descents = dl.c1;
      tick_game(c, key, game, ep, p1, p2, npc, tick, status, dl);
      stairs_dirty |= dl.c1 != descents;
    }
    if (obs) {
      int32_t* o = obs + (int64_t)t * ORX_OBS_FIELDS * B + i;
      o[ORX_OBS_P1_X * B] = p1.x;
      o[ORX_OBS_P1_Y * B] = p1.y;
      o[ORX_OBS_P1_DEPTH * B] = p1.d;
      o[ORX_OBS_P1_HEALTH * B] = p1.hp;
      o[ORX_OBS_P2_X * B] = p2.x;
      o[ORX_OBS_P2_Y * B] = p2.y;
      o[ORX_OBS_P2_DEPTH * B] = p2.d;
      o[ORX_OBS_P2_HEALTH * B] = p2.hp;
      o[ORX_OBS_TICK * B] = tick;
      o[ORX_OBS_STATUS * B] = status;
      o[ORX_OBS_P1_STAIR_X * B] = p1.sx;
      o[ORX_OBS_P1_STAIR_Y * B] = p1.sy;
      o[ORX_OBS_P2_STAIR_X * B] = p2.sx;
      o[ORX_OBS_P2_STAIR_Y * B] = p2.sy;
    }
    if (act) {
      reinterpret_cast<uint16_t*>(act)[(int64_t)t * B + i] =
          (uint16_t)((uint32_t)(uint8_t)a1 | ((uint32_t)(uint8_t)a2 << 8));
    }
  }
  store_players(st, B, i, p1, p2, stairs_dirty);
  st.tick[i] = tick;
  st.status[i] = status;
  st.episode[i] = (int32_t)ep;
  if (c.K) st.npc_alive[i] = npc.alive;
  flush_deltas(st, B, i, dl);
}

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
    return fail(ORX_EINVAL, "n_npcs must be in [0, 16]");
  if (c->n_npcs > 0 && (c->width > ORX_MAX_GRID_NPC || c->height > ORX_MAX_GRID_NPC))
    return fail(ORX_EINVAL, "NPC positions pack 8+8 bits: W, H <= 256 when n_npcs > 0");
  if (c->n_npcs > 0 && (c->npc_health < 1 || c->npc_health > 127))
    return fail(ORX_EINVAL, "npc_health must be in [1, 127]");
  const int64_t n_ground = (int64_t)(c->width - 2) * (c->height - 2) - 1;
  if (n_ground < (int64_t)c->n_npcs + 2)
    return fail(ORX_EINVAL, "board too small for the players and NPCs");
  if (c->player_health < 1) return fail(ORX_EINVAL, "player_health must be >= 1");
  if (c->autoreset != 0 && c->autoreset != 1) return fail(ORX_EINVAL, "autoreset must be 0 or 1");
  if (c->flags != 0) return fail(ORX_EINVAL, "no extension flags are implemented");
  return ORX_OK;
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
  return ORX_OK;
}

int check_policy(int32_t p) {
  if (p < ORX_POLICY_NONE || p > ORX_POLICY_STAY) return fail(ORX_EINVAL, "unknown policy");
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
  if (off < 0 || off + B > ((int64_t)1 << 32))
    return fail(ORX_EINVAL, "global game ids (game_offset + index) must fit 32 bits");
  if ((B + kBlock - 1) / kBlock > 0x7FFFFFFFLL) return fail(ORX_EINVAL, "n_games too large");
  return ORX_OK;
}

}  // namespace

extern "C" {

int orx_abi_version(void) { return ORX_ABI_VERSION; }

const char* orx_last_error(void) { return g_err; }

int orx_validate_cfg(const orx_cfg_t* cfg) {
  int r = check_cfg(cfg);
  if (r == ORX_OK) g_err[0] = 0;
  return r;
}

int orx_reset(const orx_cfg_t* cfg, const orx_state_t* st, const uint8_t* mask, int64_t n_games,
              uint64_t seed, int64_t game_offset, void* stream) {
  int r;
  if ((r = check_cfg(cfg)) || (r = check_sizes(n_games, game_offset))) return r;
  if (n_games == 0) return ORX_OK;
  if ((r = check_state(cfg, st, false))) return r;
  hipLaunchKernelGGL(reset_kernel, grid_for(n_games), dim3(kBlock), 0, (hipStream_t)stream, *cfg,
                     *st, mask, n_games, make_key(seed), game_offset);
  return launch_status("orx_reset");
}

int orx_step(const orx_cfg_t* cfg, const orx_state_t* st, const int8_t* actions, int64_t n_games,
             uint64_t seed, int64_t game_offset, void* stream) {
  int r;
  if ((r = check_cfg(cfg)) || (r = check_sizes(n_games, game_offset))) return r;
  if (n_games == 0) return ORX_OK;
  if ((r = check_state(cfg, st, true))) return r;
  if (!actions) return fail(ORX_EINVAL, "actions is NULL");
  hipLaunchKernelGGL(step_kernel, grid_for(n_games), dim3(kBlock), 0, (hipStream_t)stream, *cfg,
                     *st, actions, n_games, make_key(seed), game_offset);
  return launch_status("orx_step");
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
  hipLaunchKernelGGL(policy_kernel, grid_for(n_games), dim3(kBlock), 0, (hipStream_t)stream, *cfg,
                     *st, policy_p1, policy_p2, actions, n_games, make_key(seed), game_offset);
  return launch_status("orx_policy");
}

int orx_rollout(const orx_cfg_t* cfg, const orx_state_t* st, int32_t policy_p1, int32_t policy_p2,
                int32_t n_ticks, int32_t* obs, int8_t* act, int64_t n_games, uint64_t seed,
                int64_t game_offset, void* stream) {
  int r;
  if ((r = check_cfg(cfg)) || (r = check_sizes(n_games, game_offset)) ||
      (r = check_policy(policy_p1)) || (r = check_policy(policy_p2)))
    return r;
  if (policy_p1 == ORX_POLICY_NONE || policy_p2 == ORX_POLICY_NONE)
    return fail(ORX_EINVAL, "orx_rollout needs an action producer for both players");
  if (n_ticks < 0) return fail(ORX_EINVAL, "n_ticks < 0");
  if (n_games == 0 || n_ticks == 0) return ORX_OK;
  if ((r = check_state(cfg, st, true))) return r;
  hipLaunchKernelGGL(rollout_kernel, grid_for(n_games), dim3(kBlock), 0, (hipStream_t)stream,
                     *cfg, *st, policy_p1, policy_p2, n_ticks, obs, act, n_games, make_key(seed),
                     game_offset);
  return launch_status("orx_rollout");
}

}  // extern "C"
