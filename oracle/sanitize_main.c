/* TEST INFRASTRUCTURE ONLY: drives the C oracle (orx_oracle.c) through every
 * mode it has -- NPCs (dense and at the K cap), both despawn strategies,
 * Separated starts, a dungeon bank, the build extensions, stock-seed (MT19937)
 * mode, event recording, invalid actions -- so that a build with
 * -fsanitize=address,undefined (tests/test_sanitize.py) checks the oracle
 * itself for memory errors and undefined behaviour. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/orx.h"

void* oracle_new(const orx_cfg_t* cfg, int64_t n_games, uint64_t seed, int64_t game_offset,
                 int record_events);
void oracle_set_bank(void* h, const uint8_t* tiles, int32_t n_layouts);
void oracle_free(void* h);
void oracle_reset(void* h, const uint8_t* mask, const int32_t* episode);
void oracle_step(void* h, const int8_t* actions);
void oracle_policy(void* h, int32_t pol1, int32_t pol2, int8_t* actions);
void oracle_seed_mt(void* h, uint64_t seed);
int32_t oracle_events(void* h, int64_t game, int32_t* out, int32_t cap);
int32_t oracle_entities(void* h, int64_t game, int32_t* out, int32_t cap);
int32_t oracle_world(void* h, int64_t game, int32_t* out, int32_t cap);

static orx_cfg_t base(int w, int h) {
  orx_cfg_t c;
  memset(&c, 0, sizeof c);
  c.width = w; c.height = h; c.despawn = ORX_DESPAWN_UNREACHABLE; c.max_ticks = 60;
  c.start_mode = ORX_START_TOGETHER; c.npc_health = 3; c.npc_damage = 1;
  c.player_health = 10; c.player_damage = 2; c.player_armor = 1; c.autoreset = 1;
  return c;
}

static void run(const char* name, orx_cfg_t c, int64_t B, int pol1, int pol2, int ticks,
                const uint8_t* bank, int L) {
  void* o = oracle_new(&c, B, 7, 3, 1);
  if (bank) oracle_set_bank(o, bank, L);
  if (c.rng == ORX_RNG_MT19937) oracle_seed_mt(o, 11);
  oracle_reset(o, NULL, NULL);
  int8_t* a = (int8_t*)malloc((size_t)B * 2);
  int32_t buf[4096];
  for (int t = 0; t < ticks; ++t) {
    oracle_policy(o, pol1, pol2, a);
    if (t == ticks / 2) a[0] = 9;  /* an invalid action stops that game */
    oracle_step(o, a);
    for (int64_t g = 0; g < B; g += 7) {
      oracle_events(o, g, buf, 1024);
      oracle_entities(o, g, buf, 512);
      oracle_world(o, g, buf, 1024);
    }
  }
  free(a);
  oracle_free(o);
  printf("%s ok\n", name);
}

int main(void) {
  orx_cfg_t c = base(6, 6);
  c.n_npcs = 4;
  run("npc_small", c, 64, 1, 1, 300, NULL, 0);
  c = base(8, 8);
  c.n_npcs = 16; c.max_ticks = 0;
  run("npc_cap", c, 32, 1, 2, 300, NULL, 0);
  c = base(7, 8);
  c.despawn = ORX_DESPAWN_UNUSED; c.n_npcs = 2;
  run("stairs_unused", c, 32, 2, 2, 400, NULL, 0);
  c = base(6, 7);
  c.start_mode = ORX_START_SEPARATED; c.p2_depth = 3;
  run("separated", c, 32, 2, 1, 300, NULL, 0);
  c = base(4, 4);
  c.n_npcs = 1; c.max_ticks = 30;
  run("tiny", c, 32, 1, 2, 200, NULL, 0);
  c = base(9, 8);
  c.flags = ORX_EXT_SEPARATION_DAMAGE | ORX_EXT_RANDOM_DOUBLE_DEATH; c.sep_period = 4;
  c.n_npcs = 2; c.max_ticks = 0;
  run("extensions", c, 32, 2, 1, 300, NULL, 0);
  c = base(7, 8);
  c.rng = ORX_RNG_MT19937; c.n_npcs = 3; c.despawn = ORX_DESPAWN_UNUSED;
  run("stock_mt", c, 16, 2, 1, 300, NULL, 0);
  /* a bank of 3 layouts, 9x8: border walls, a few interior walls, 1-2 stairs */
  enum { W = 9, H = 8, L = 3 };
  static uint8_t tiles[L * W * H];
  for (int l = 0; l < L; ++l)
    for (int x = 0; x < W; ++x)
      for (int y = 0; y < H; ++y) {
        uint8_t t = (x == 0 || y == 0 || x == W - 1 || y == H - 1) ? ORX_TILE_WALL
                                                                      : ORX_TILE_GROUND;
        if (t == ORX_TILE_GROUND && (x * 3 + y * 5 + l) % 11 == 0) t = ORX_TILE_WALL;
        tiles[(l * W + x) * H + y] = t;
      }
  for (int l = 0; l < L; ++l) {
    tiles[(l * W + 2 + l) * H + 3] = ORX_TILE_STAIRCASE_DOWN;
    if (l == 1) tiles[(l * W + 6) * H + 5] = ORX_TILE_STAIRCASE_DOWN;
  }
  c = base(W, H);
  c.n_npcs = 2; c.despawn = ORX_DESPAWN_UNUSED;
  run("bank", c, 32, 2, 1, 300, tiles, L);
  return 0;
}
