/*
 * orx.h -- C-ABI of the MI355X batched Optimax Rogue tick engine (liborx.so).
 *
 * This is the drop-in boundary for the reference's per-tick updater.  Every
 * entry point below replaces one reference interface; the citation after each
 * declaration is the reference file:line (paths relative to the reference
 * repository root, optimax_rogue @ v0).
 *
 * Conventions
 *  - Plain pointers and sizes only; no C++ or torch types cross the boundary.
 *  - Every device pointer is owned by the caller (PyTorch tensors in the Python
 *    host layer); the library never allocates device memory.
 *  - Calls are asynchronous on the caller's HIP stream (`stream`, a
 *    hipStream_t passed as void*; NULL = the legacy default stream).  The
 *    library is stateless and re-entrant; the caller selects the device.
 *  - Return value: ORX_OK (0) or a negative error code; orx_last_error() gives
 *    a thread-local message for the most recent failure on the calling thread.
 *  - Randomness is Philox4x32-10 keyed by (seed) with the counter
 *    (global game id, episode, tick-or-depth, purpose|block); global game id =
 *    game_offset + local index, so results do not depend on how games are
 *    sharded across GPUs.  The words are consumed through the exact CPython
 *    random._randbelow / numpy RandomState.randint transforms used at the
 *    reference's draw sites; a tick's CPython-random draws (bots, shuffles)
 *    first take bits of one "tick block" ("Random streams").
 */
#ifndef ORX_H
#define ORX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORX_ABI_VERSION 7

/* ---- error codes -------------------------------------------------------- */
#define ORX_OK 0
#define ORX_EINVAL (-22) /* bad config, pointer, size or argument            */
#define ORX_EIO (-5)     /* HIP runtime error (launch failure, bad stream)    */

/* ---- enums: same integer values as the reference ------------------------ */
/* Move            optimax_rogue/logic/moves.py:6-12                         */
#define ORX_MOVE_UP 1
#define ORX_MOVE_RIGHT 2
#define ORX_MOVE_DOWN 3
#define ORX_MOVE_LEFT 4
#define ORX_MOVE_STAY 5
/* UpdateResult    optimax_rogue/logic/updater.py:16-21                      */
#define ORX_IN_PROGRESS 1
#define ORX_PLAYER1_WIN 2
#define ORX_PLAYER2_WIN 3
#define ORX_TIE 4
/* build-only per-game status codes (>= 16): the game is stopped            */
#define ORX_STATUS_BAD_ACTION 16   /* an action outside 1..5 (1..6 with
                                      ORX_EXT_HEAL; the reference would
                                      attack itself, updater.py:229-234)     */
#define ORX_STATUS_RNG_EXHAUSTED 17 /* a rejection loop ran past its word cap
                                      (probability < 1e-180; never observed) */
/* DungeonDespawningStrategy  optimax_rogue/logic/updater.py:47-50           */
#define ORX_DESPAWN_UNREACHABLE 1
#define ORX_DESPAWN_UNUSED 2
/* GameStartGenerator plugins optimax_rogue/logic/worldgen.py:61-135         */
#define ORX_START_TOGETHER 1
#define ORX_START_SEPARATED 2
/* Tile            optimax_rogue/game/world.py:10-17                         */
#define ORX_TILE_GROUND 1
#define ORX_TILE_WALL 2
#define ORX_TILE_STAIRCASE_DOWN 3
/* CombatFlag      optimax_rogue/game/modifiers.py:7-12                      */
#define ORX_FLAG_BLOCK 1
#define ORX_FLAG_AMBUSH 2
#define ORX_FLAG_FLEE 3
#define ORX_FLAG_PARRY 4
/* action producers (bots) optimax_rogue_bots/{randombot,staircasebot}.py   */
#define ORX_POLICY_NONE 0      /* leave the action untouched                  */
#define ORX_POLICY_RANDOM 1    /* RandomBot.move   randombot.py:20-21          */
#define ORX_POLICY_STAIRCASE 2 /* StaircaseBot.move staircasebot.py:9-21       */
#define ORX_POLICY_STAY 3      /* always Move.Stay                            */

/* enemy AI (orx_cfg_t.npc_policy): the reference's override hook
 * Updater.decide_npc_move (updater.py:165-178), whose default is Stay.  Every
 * NPC's move is decided at the start of the tick, in GameState.entities order,
 * before any move is resolved (updater.py:116-126); then the reference's NPC
 * shuffle (:127) orders them after the players and handle_move resolves each
 * one (:133-134, 180-243: Block / Ambush / Flee against players and NPCs; an
 * NPC stepping onto a staircase dies, :263-270); the dead are swept
 * (:136-145).  The policies (the same rules as tests/golden/make_golden.py's
 * NpcAiUpdater, which pins them against the reference):
 *   an NPC on a depth without a dungeon (despawned), or on a depth where a
 *   player stands next to a staircase tile, stays -- the second rule keeps
 *   the reference from raising KeyError (a descend that despawns the depth
 *   earlier in the tick, :295-296, then an NPC stepping onto a free cell,
 *   :203); otherwise
 *   ORX_NPC_RANDOM: random.choice(list(Move)), its getrandbits from the NPC
 *     stream (Philox purpose 9, c2 = tick: bits 0-29 of each word, 3-bit
 *     fields, >= 5 rejected) or, in stock-seed mode, the game's CPython random
 *     between the player shuffle and the NPC shuffle;
 *   ORX_NPC_CHASE: a greedy step toward the nearer player on its depth
 *     (Manhattan; player 1 on a tie): |dx| > |dy| -> Right / Left, else Down /
 *     Up (StaircaseBot's rule); no player there -> Stay;
 *   a move into a blocked cell (Dungeon.is_blocked, world.py:41-46) -> Stay.
 * Needs flags within ORX_EXT_SEPARATION_DAMAGE | ORX_EXT_RANDOM_DOUBLE_DEATH;
 * the rollout runs such games one lane per game (the generic ordered tick). */
#define ORX_NPC_STAY 0
#define ORX_NPC_RANDOM 1
#define ORX_NPC_CHASE 2

/* word sources (orx_cfg_t.rng)                                             */
#define ORX_RNG_PHILOX 0  /* keyed Philox4x32-10 streams (default; stateless,
                             shard-invariant, DESIGN.md "Random streams")   */
#define ORX_RNG_MT19937 1 /* stock-seed mode: per game the two MT19937 states
                             of a reference process seeded random.seed(n) and
                             np.random.seed(n), n = seed + global game id
                             (orx_seed_mt), consumed in the reference's call
                             order: CPython random for the bots and shuffles
                             (randombot.py:21, updater.py:114,127), numpy for
                             dungeons and spawn cells (worldgen.py:39-40,
                             world.py:62)                                   */
#define ORX_DSTORE_MIN 256        /* stock-seed mode: the dungeons each player
                                     remembers (orx_dstore_depths) are the
                                     smallest power of two >= max(max_ticks,
                                     ORX_DSTORE_MIN); ORX_DSTORE_UNBOUNDED when
                                     max_ticks == 0, at most ORX_DSTORE_MAX   */
#define ORX_DSTORE_UNBOUNDED 4096
#define ORX_DSTORE_MAX 65536

/* build extensions (orx_cfg_t.flags): mechanics the reference's readme
 * describes but its code does not implement (readme.md:44-48); off = parity.
 * No reference output pins them ("parity unpinned").        */
#define ORX_EXT_SEPARATION_DAMAGE 1 /* "if the agents are on separate levels
   the agent further behind begins taking damage that scales linearly with
   time since separation": at the end of the k-th consecutive separated
   tick the shallower player loses ceil(k / sep_period) health            */
#define ORX_EXT_RANDOM_DOUBLE_DEATH 2 /* "If both agents die during the same
   tick then one wins at random": one word of stream purpose 6 (c2 = tick)
   instead of Tie; top bit 0 = Player1Win                                  */
/* The readme's character mechanics (readme.md:44, 72, 74).  Every free
 * parameter is an orx_cfg_t field; the player attributes live in
 * orx_state_t.p_rpg, items in item_pos / item_mask.       */
#define ORX_EXT_MANA 4 /* "if A has mana then up to 1/3 the manabar is
   converted into damage and spent": players start with mana_max mana; each
   attack (handle_combat with a player attacker, vs a player or an NPC)
   spends s = min(mana, mana_max / 3) rounded down to a multiple of
   mana_per_point and deals s / mana_per_point extra damage; at the end of
   every tick each player regains mana_regen, capped at mana_max          */
#define ORX_EXT_HEAL 8 /* "A player may heal by spending up to 1/3 their
   manabar and converting it to health.  They cannot move while healing":
   action ORX_MOVE_HEAL (6) is a Stay (a Block for attackers) that, at the
   player's turn in the initiative order and if it is alive, converts up to
   min(mana, mana_max / 3) mana into health at mana_per_point per point,
   never above its max health; reported as EntityHealthUpdate (+amount).
   Needs ORX_EXT_MANA                                                      */
#define ORX_EXT_LEVELING 16 /* "Enemies ... may be killed for experience.
   Leveling refills health and mana": the player whose hit takes an NPC to
   health <= 0 gains xp_per_kill; each time its xp crosses a multiple of
   xp_per_level a living player's health is set to its max health and its
   mana to mana_max (after the death sweep)                               */
#define ORX_EXT_ITEMS 32 /* "Enemies may drop items, which provide flat
   attribute bonuses if picked up.  There are a finite number of item
   spots": an NPC removed by the death sweep drops an item on its cell with
   probability item_drop_pct / 100 (Philox purpose 8, c2 = tick, block =
   NPC slot: word a * 100 >> 32 < item_drop_pct; word b bit 0 = kind:
   0 damage, 1 max health); a player whose move steps onto an item's cell
   takes it if it holds fewer than item_slots items: damage or max health
   (and health) += item_bonus                                              */
#define ORX_EXT_RPG (ORX_EXT_MANA | ORX_EXT_HEAL | ORX_EXT_LEVELING | ORX_EXT_ITEMS)
#define ORX_EXT_README_COMBAT 64 /* the readme's combat table (readme.md:69-70)
   instead of handle_move's player-vs-player rules (updater.py:218-243), as
   one simultaneous resolution before the moves (NPC combat unchanged).  With
   a, b the players' cells and ta, tb their targets on one depth (a move
   attacks the other's cell, or the cell both move into):
     both attack each other's cell       -> each takes half the other's
                                            damage, both stay, both get
                                            combat_cooldown ticks of cooldown;
     both move into one cell             -> each takes the other's full
                                            damage, both stay;
     A attacks b, B stays (or heals)     -> negated and A is stunned (1 tick
                                            of cooldown), unless B is on
                                            cooldown: then full damage;
     A attacks b, B moves elsewhere      -> no damage.
   An attacker never moves.  A player on cooldown cannot attack (an attack is
   a Stay) nor defend.  Damage = damage - armor (+ mana with ORX_EXT_MANA,
   spent only by an attack that deals damage).  Combat events: both-attack
   PARRY, one-cell AMBUSH, stay BLOCK, moved-away FLEE.  State:
   p_rpg row ORX_RPG_COOLDOWN                                              */
/* the extensions that keep per-player attributes in orx_state_t.p_rpg       */
#define ORX_EXT_CHARACTER (ORX_EXT_RPG | ORX_EXT_README_COMBAT)

/* player attributes of the character mechanics: rows of orx_state_t.p_rpg  */
#define ORX_RPG_MANA 0
#define ORX_RPG_XP 1
#define ORX_RPG_DAMAGE 2      /* Entity.damage (base + damage items)         */
#define ORX_RPG_MAX_HEALTH 3  /* Entity.max_health (base + health items)     */
#define ORX_RPG_ITEMS 4       /* items held                                  */
#define ORX_RPG_COOLDOWN 5    /* ORX_EXT_README_COMBAT: ticks of cooldown left */
#define ORX_RPG_FIELDS 6
#define ORX_MOVE_HEAL 6       /* ORX_EXT_HEAL only                           */

/* per-game event counters (rows of orx_state_t.counters)                    */
#define ORX_CNT_COMBAT 0        /* handle_combat calls       updater.py:298  */
#define ORX_CNT_DESCEND 1       /* player descents           updater.py:259  */
#define ORX_CNT_DUNGEON 2       /* spawn_dungeon calls in ticks updater.py:274 */
#define ORX_CNT_NPC_DEATH 3     /* EntityDeathUpdate sweeps  updater.py:136  */
#define ORX_NCOUNTERS 4

/* update events (orx_step_events), int32 records {type, iden, a, b}:
 *   COMBAT   {1, attacker, defender, CombatFlag}  EntityCombatUpdate   updates.py:71-139
 *   DEATH    {2, npc iden, 0, 0}                  EntityDeathUpdate    updates.py:167-184
 *   POSITION {3, iden, new depth, x | y << 16}    EntityPositionUpdate updates.py:186-220
 *   DUNGEON  {4, 0, depth, 0}                     DungeonCreatedUpdate updates.py:308-335
 * Entity idens: player 1 = 1, player 2 = 2, NPC slot k = 3 + k.           */
#define ORX_EV_COMBAT 1
#define ORX_EV_DEATH 2
#define ORX_EV_POSITION 3
#define ORX_EV_DUNGEON 4
#define ORX_EV_HEALTH 5  /* {5, iden, amount, 0}  EntityHealthUpdate updates.py:222-253
                            (separation damage -dmg, ORX_EXT_SEPARATION_DAMAGE;
                            a heal +amount, ORX_EXT_HEAL)                   */
#define ORX_MAX_EVENTS 8 /* per game per tick with Stay NPCs (at most 6
                            occur); orx_max_events(cfg) for any config    */

#define ORX_MAX_NPCS 255     /* NPCs per game                                 */
#define ORX_MAX_REG_NPCS 16  /* up to this many the kernels keep the NPCs in
                                registers; above, in an occupancy grid in HBM
                                (orx_state_t.npc_grid; ORX_EXT_ITEMS needs
                                n_npcs <= ORX_MAX_REG_NPCS)                   */
#define ORX_MAX_GRID_NPC 256 /* NPC (x,y) pack into 8+8 bits when K > 0    */

/* trajectory fields, rows of one orx_rollout tick record                    */
#define ORX_OBS_P1_X 0
#define ORX_OBS_P1_Y 1
#define ORX_OBS_P1_DEPTH 2
#define ORX_OBS_P1_HEALTH 3
#define ORX_OBS_P2_X 4
#define ORX_OBS_P2_Y 5
#define ORX_OBS_P2_DEPTH 6
#define ORX_OBS_P2_HEALTH 7
#define ORX_OBS_TICK 8
#define ORX_OBS_STATUS 9
#define ORX_OBS_P1_STAIR_X 10
#define ORX_OBS_P1_STAIR_Y 11
#define ORX_OBS_P2_STAIR_X 12
#define ORX_OBS_P2_STAIR_Y 13
#define ORX_OBS_FIELDS 14

/* ---- configuration (POD) ------------------------------------------------ */
/* Mirrors the reference's construction arguments:
 *   Updater(dgen, despawn_strat, max_ticks)        updater.py:65-69
 *   EmptyDungeonGenerator(width, height)           worldgen.py:29-43
 *   Together/SeparatedGameStartGenerator(...)      worldgen.py:61-135
 *   Entity(iden, depth, x, y, 10, 10, 2, 1, ...)   worldgen.py:85-86        */
/* sep_period's bound: the damage ceil(k / sep_period) stays exact in 31-bit
 * arithmetic for every tick count below 2^31 - 2^24 */
#define ORX_SEP_PERIOD_MAX 16777216 /* 2^24 */

typedef struct orx_cfg {
  int32_t width;          /* W >= 4  (np.random.randint(1, W-2) needs W > 3) */
  int32_t height;         /* H >= 4                                          */
  int32_t despawn;        /* ORX_DESPAWN_*                                   */
  int32_t max_ticks;      /* 0 = no limit ("if self.max_ticks and ...")      */
  int32_t start_mode;     /* ORX_START_*                                     */
  int32_t p1_depth;       /* Separated start depths (Together: both 0)       */
  int32_t p2_depth;
  int32_t n_npcs;         /* K NPCs at reset on player 1's start depth       */
  int32_t npc_health;     /* 1..127                                          */
  int32_t npc_damage;
  int32_t npc_armor;
  int32_t player_health;  /* 10 */
  int32_t player_damage;  /* 2  */
  int32_t player_armor;   /* 1  */
  int32_t autoreset;      /* 1: a finished game is reset by the next step    */
  int32_t flags;          /* ORX_EXT_* build extensions; 0 = reference parity */
  int32_t n_layouts;      /* dungeon generator: 0 = EmptyDungeonGenerator
                             (closed forms, worldgen.py:28-44); L > 0 = a
                             layout bank: spawn_dungeon(depth) returns layout
                             randint(L) of orx_state_t.bank_* (an explicit-
                             grid DungeonGenerator plugin, worldgen.py:9-26) */
  int32_t sep_period;     /* ORX_EXT_SEPARATION_DAMAGE: ticks per +1 damage,
                             1..ORX_SEP_PERIOD_MAX                           */
  int32_t rng;            /* ORX_RNG_*                                       */
  /* character mechanics (ORX_EXT_MANA / HEAL / LEVELING / ITEMS)            */
  int32_t mana_max;       /* manabar size (>= 3 with MANA)                   */
  int32_t mana_regen;     /* mana regained per tick                          */
  int32_t mana_per_point; /* mana per point of damage or health (>= 1)       */
  int32_t xp_per_kill;    /* experience per NPC kill                         */
  int32_t xp_per_level;   /* experience per level (>= 1 with LEVELING)       */
  int32_t item_drop_pct;  /* 0..100: chance a dying NPC drops an item        */
  int32_t item_bonus;     /* flat attribute bonus of an item                 */
  int32_t item_slots;     /* items a player can hold                         */
  int32_t combat_cooldown;/* ORX_EXT_README_COMBAT: ticks after a mutual
                             attack (readme.md:69: 3)                        */
  int32_t npc_policy;     /* (ABI 7) ORX_NPC_*: the enemy AI, Updater.
                             decide_npc_move (updater.py:165-178); 0 = Stay */
} orx_cfg_t;

/* ---- batch state (SoA, batch axis contiguous; all device pointers) ------- */
/* Shapes use B = games in this call.  "[2][B]" = player 1 row then player 2. */
typedef struct orx_state {
  int32_t* p_x;        /* [2][B] Entity.x        entities.py:36-59           */
  int32_t* p_y;        /* [2][B] Entity.y                                    */
  int32_t* p_depth;    /* [2][B] Entity.depth                                */
  int32_t* p_health;   /* [2][B] Entity.health                               */
  int32_t* st_x;       /* [2][B] Dungeon.staircase() of each player's depth  */
  int32_t* st_y;       /* [2][B]                     world.py:52-55          */
  int32_t* tick;       /* [B]    GameState.tick      state.py:25-29          */
  int32_t* status;     /* [B]    last UpdateResult (or ORX_STATUS_*)         */
  int32_t* episode;    /* [B]    episode index (Philox counter word 1)       */
  int32_t* ret_sum;    /* [B]    sum of finished-episode outcomes, p1 view:
                                 +1 Player1Win, -1 Player2Win, 0 Tie         */
  int32_t* ep_count;   /* [B]    finished episodes                           */
  int32_t* counters;   /* [ORX_NCOUNTERS][B] event counters (may be NULL)    */
  uint16_t* npc_pos;   /* [K][B] x | y << 8  (NULL when K == 0)              */
  int8_t* npc_health;  /* [K][B]                                             */
  uint32_t* npc_alive; /* [ceil(K/32)][B] bit k % 32 of row k / 32 = NPC k
                                 still in GameState.entities ([B] for K <= 32) */
  /* dungeon bank (cfg->n_layouts = L > 0; all NULL otherwise)               */
  int16_t* p_layout;            /* [2][B] layout of each player's depth       */
  const uint8_t* bank_tiles;    /* [L][W][H] Tile codes, Dungeon.tiles layout
                                   (flat x * H + y)       world.py:19-39     */
  const uint16_t* bank_ground;  /* [L][W*H] flat indices of the Ground tiles
                                   in ascending order (get_random_unblocked's
                                   candidate list, world.py:57-66)           */
  const int32_t* bank_meta;     /* [L][4] {n_ground, staircase x, staircase y,
                                   0}: first StaircaseDown in x-major order
                                   (Dungeon.staircase, world.py:52-55)       */
  int32_t* sep_start;           /* [B] ORX_EXT_SEPARATION_DAMAGE: tick the
                                   current separation began, -1 = together
                                   (NULL when the extension is off)          */
  /* stock-seed mode (cfg->rng = ORX_RNG_MT19937; NULL otherwise)            */
  uint32_t* mt_py;              /* [625][B] CPython random: mt[624] + index   */
  uint32_t* mt_np;              /* [625][B] numpy RandomState: key[624] + pos */
  int32_t* dstore;              /* [2][N][2][B], N = orx_dstore_depths(cfg):
                                   per player, {depth, sx | sy << 8 |
                                   (layout + 1) << 16} of each dungeon it
                                   entered, slot (depth - its start depth)
                                   mod N -- the staircases a keyed stream
                                   would regenerate.  A player descends at
                                   most once per tick, so a ring of N >=
                                   max_ticks depths still holds every depth
                                   the other player can yet enter from it
                                   (Unreachable, updater.py:245-257)         */
  /* character mechanics (any ORX_EXT_CHARACTER flag; NULL otherwise)        */
  int32_t* p_rpg;               /* [ORX_RPG_FIELDS][2][B] player attributes   */
  uint16_t* item_pos;           /* [K][B] ORX_EXT_ITEMS: item dropped by NPC
                                   slot k, x | y << 8 (on the NPCs' depth)    */
  uint32_t* item_mask;          /* [2][B] ORX_EXT_ITEMS: row 0 bit k = item k
                                   lies on the floor, row 1 bit k = its kind
                                   (0 damage, 1 max health)                  */
  /* dense NPCs (n_npcs > ORX_MAX_REG_NPCS; NULL otherwise)                   */
  uint8_t* npc_grid;            /* [B][W * H] occupancy of the NPCs' depth:
                                   slot + 1 per cell (x * H + y), 0 = empty   */
} orx_state_t;

/* ---- entry points --------------------------------------------------------- */

/* ORX_ABI_VERSION of the loaded library. */
int orx_abi_version(void);

/* Source hash the library was built from: the first 16 hex digits of the
 * SHA-256 of orx_engine.hip followed by include/orx.h (build.py), so a test
 * can prove the loaded library is the tree's own kernel ("unknown" for a
 * build made outside build.py).  No reference counterpart. */
const char* orx_build_id(void);

/* Games per wave orx_rollout launches for a batch of n_games (1..64, a power
 * of two; < 64 when the batch is too small to give every SIMD of the current
 * device a wave; env ORX_ROLLOUT_LANES overrides).  Results do not depend on
 * it.  No reference counterpart (the reference runs one game per process). */
int orx_rollout_lanes(int64_t n_games);

/* The shape of an orx_rollout launch with these arguments (trajectory:
 * obs and act both given): games per wave (1..64), lanes per game (2 for the
 * paired form -- no dense NPCs (n_npcs <= ORX_MAX_REG_NPCS, held in
 * registers), grids up to 256 x 256, two RandomBots (also with the character
 * mechanics: mana, experience, items) or two StaircaseBots, a dungeon bank
 * only when its tiles fit the device's per-workgroup LDS (160 KiB on gfx950;
 * above 64 KiB the launch raises the kernel's limit, and a refused raise
 * takes the one-lane form with the tiles in global memory) and for
 * StaircaseBots without separation damage, batches below 64 games per wave:
 * one lane per player; the bench's C3 shards run
 * pair_rollout_kernel<8, 1, 2, false>), whether the trajectory rows are
 * stored nontemporal (whole-line row segments) or with the default policy,
 * the threads per workgroup (256; 512 for a paired bank above half the LDS:
 * one workgroup per CU then holds two waves per SIMD) and the dynamic LDS
 * bytes per workgroup (a bank's tiles, dense NPCs' occupancy bitmaps);
 * concurrency as in orx_rollout_concurrent (1 for orx_rollout).  Results
 * never depend on it.  No reference counterpart. */
typedef struct orx_rollout_shape {
  int32_t games_per_wave;
  int32_t lanes_per_game;
  int32_t nontemporal;
  int32_t threads_per_block;  /* (ABI 6) */
  int32_t lds_bytes;          /* (ABI 6) */
} orx_rollout_shape_t;
int orx_rollout_shape(const orx_cfg_t* cfg, int32_t policy_p1, int32_t policy_p2,
                      int64_t n_games, int32_t trajectory, int32_t concurrency,
                      orx_rollout_shape_t* out);

/* Stock-seed mode: N, the depths each player's dstore ring holds for this
 * configuration (orx_state_t.dstore is [2][N][2][B] int32), or ORX_EINVAL
 * for an invalid configuration.  N >= max_ticks, so every game the
 * reference can play to max_ticks is played; with max_ticks == 0 (no limit)
 * or max_ticks > ORX_DSTORE_MAX a game whose lagging player still has to
 * enter a dungeon more than N levels behind the other stops with
 * ORX_STATUS_RNG_EXHAUSTED instead of inventing a staircase.  Cost: 16 * N
 * bytes per game (16 KiB at max_ticks 1000, 64 KiB with no limit, 1 MiB at
 * the 65,536-depth cap), all of it cleared by orx_seed_mt -- size stock-seed
 * batches for it (BatchedEngine warns above a quarter of the device's
 * memory).  Replaces nothing: the reference keeps World.dungeons in a dict
 * (world.py:101-180). */
int orx_dstore_depths(const orx_cfg_t* cfg);

/* (ABI 7) Event records per game per tick orx_step_events writes for this
 * configuration (its events buffer is [B][orx_max_events(cfg)][4]):
 * ORX_MAX_EVENTS with Stay NPCs; with moving NPCs (npc_policy) 6 + 2 * n_npcs
 * (each NPC's own move, combat or staircase death, plus its sweep), or
 * ORX_EINVAL for an invalid configuration.  No reference counterpart (the
 * reference returns a Python list, updater.py:76-162). */
int orx_max_events(const orx_cfg_t* cfg);

/* Message for the last non-zero return on this thread ("" if none). */
const char* orx_last_error(void);

/* Validates a configuration without touching the device.
 * Replaces the constructor checks of Updater / generators
 * (updater.py:65-69, worldgen.py:61-135; ValueError -> ORX_EINVAL). */
int orx_validate_cfg(const orx_cfg_t* cfg);

/* Stock-seed mode: seeds game b's two MT19937 states as a reference
 * process would after random.seed(n); np.random.seed(n) with n = seed +
 * game_offset + b (CPython random_seed -> init_by_array, _randommodule.c;
 * numpy RandomState._legacy_seeding -> mt19937_seed; n < 2^32).  Call once
 * before the first orx_reset; later episodes continue the streams. */
int orx_seed_mt(const orx_cfg_t* cfg, const orx_state_t* st, int64_t n_games, uint64_t seed,
                int64_t game_offset, void* stream);

/* Starts episode st->episode[b] for every game b with mask[b] != 0
 * (mask == NULL: all games).  Replaces GameStartGenerator.setup_game:
 * TogetherGameStartGenerator.setup_game  worldgen.py:77-87
 * SeparatedGameStartGenerator.setup_game worldgen.py:124-135
 * plus the NPC spawner (build-defined). */
int orx_reset(const orx_cfg_t* cfg, const orx_state_t* st, const uint8_t* mask,
              int64_t n_games, uint64_t seed, int64_t game_offset, void* stream);

/* Advances every game one tick with actions[b][0] (player 1) and
 * actions[b][1] (player 2), values Move 1..5 (and ORX_MOVE_HEAL with
 * ORX_EXT_HEAL).  Replaces
 * Updater.update(game_state, player1_move, player2_move)  updater.py:76-162
 * (with GameState.on_tick, state.py:46-51, folded in).  A game whose status
 * is not ORX_IN_PROGRESS is reset to its next episode when cfg->autoreset,
 * else left unchanged. */
int orx_step(const orx_cfg_t* cfg, const orx_state_t* st, const int8_t* actions,
             int64_t n_games, uint64_t seed, int64_t game_offset, void* stream);

/* n_ticks x orx_step in one launch (ABI 6): tick t plays actions[(t * n_games
 * + b) * 2 + p] (int8, [n_ticks][n_games][2]: a recorded or precomputed move
 * log), the state kept in registers between ticks; a non-Move value stops
 * that game with ORX_STATUS_BAD_ACTION and a finished game is reset to its
 * next episode when cfg->autoreset, as orx_step does tick by tick (results
 * are identical, tested).  obs (may be NULL) receives each tick's post-step
 * observation as orx_rollout_ex writes it, in obs_format.  Philox mode only
 * (stock-seed mode: orx_step per tick).  Replaces the server loop
 * server/main.py:110-113 over Updater.update (updater.py:76-162) fed from a
 * move log -- SURVEY.md s8(b)'s orx_step(..., n_ticks). */
int orx_step_n(const orx_cfg_t* cfg, const orx_state_t* st, const int8_t* actions,
               int32_t n_ticks, int32_t* obs, int32_t obs_format, int64_t n_games, uint64_t seed,
               int64_t game_offset, void* stream);

/* orx_step_n with the number of launches sharing the device (ABI 7, as
 * orx_rollout_ex's concurrency): a batch replayed as stream shards passes the
 * shard count, so each launch's games per wave are planned for the device's
 * total (orx_step_n = concurrency 1).  Results do not depend on it. */
int orx_step_n_ex(const orx_cfg_t* cfg, const orx_state_t* st, const int8_t* actions,
                  int32_t n_ticks, int32_t* obs, int32_t obs_format, int64_t n_games,
                  uint64_t seed, int64_t game_offset, int32_t concurrency, void* stream);

/* orx_step plus the update-event list of the tick: for game b,
 * events[(b * ORX_MAX_EVENTS + j) * 4 + 0..3], j < n_events[b], in the order
 * Updater.update appends them to its result list (updater.py:133-145).
 * Steps that reset a game (autoreset) or reject an action record none. */
int orx_step_events(const orx_cfg_t* cfg, const orx_state_t* st, const int8_t* actions,
                    int32_t* events, int32_t* n_events, int64_t n_games, uint64_t seed,
                    int64_t game_offset, void* stream);

/* Writes actions[b][p] from the stock bots.  Replaces
 * RandomBot.move    optimax_rogue_bots/randombot.py:20-21
 * StaircaseBot.move optimax_rogue_bots/staircasebot.py:9-21 */
int orx_policy(const orx_cfg_t* cfg, const orx_state_t* st, int32_t policy_p1,
               int32_t policy_p2, int8_t* actions, int64_t n_games,
               uint64_t seed, int64_t game_offset, void* stream);

/* A learner's tick in one launch (VecEnv.step): player 1's actions from
 * `actions` (action_cols 1: [B], player 2 moved by policy_p2 as orx_policy
 * would; 2: [B][2], both players), elements of action_bytes bytes (1, 2, 4
 * or 8: int8 .. int64, read at full width -- any value outside the Move
 * codes, e.g. a 0-based argmax or 257, becomes an invalid move, which stops
 * that game with ORX_STATUS_BAD_ACTION as orx_step does); the pair played is
 * written to act[b][2]; then orx_step; then per game the post-step
 * observation row obs[b * ORX_OBS_FIELDS + f] (the orx_rollout fields), the
 * status, reward[b] (player 1's view: +1 Player1Win, -1 Player2Win, 0
 * otherwise, on the tick the episode ends) and done[b] (1 on that tick; an
 * engine stop code >= 16 ends it as a truncation); status may be NULL (it is
 * also the observation row's field ORX_OBS_STATUS).  No host sync.  Philox
 * mode only (stock-seed mode: orx_policy + orx_step).  action_cols 1 needs a
 * policy for player 2 (ORX_POLICY_NONE is refused).  Replaces the bot
 * loop's per-tick exchange, optimax_rogue_bots/main.py:118-155, and
 * server/main.py:110-113 for a learner. */
int orx_env_step(const orx_cfg_t* cfg, const orx_state_t* st, const void* actions,
                 int32_t action_bytes, int32_t action_cols, int32_t policy_p2, int8_t* act,
                 int32_t* obs, float* reward, uint8_t* done, int32_t* status, int64_t n_games,
                 uint64_t seed, int64_t game_offset, void* stream);

/* orx_env_step plus a refused-action count (ABI 6): when bad_actions (a
 * device uint32) is not NULL, the number of games stopped with
 * ORX_STATUS_BAD_ACTION by this tick is added to it (device atomics, no
 * host sync), so a host can detect a learner's out-of-range actions -- e.g.
 * a 0-based argmax -- without synchronizing every tick (VecEnv reads it
 * asynchronously).  action_cols 1 with policy_p2 ORX_POLICY_NONE is refused
 * (ORX_EINVAL): player 2 then has no move; pass both players' actions. */
int orx_env_step_ex(const orx_cfg_t* cfg, const orx_state_t* st, const void* actions,
                    int32_t action_bytes, int32_t action_cols, int32_t policy_p2, int8_t* act,
                    int32_t* obs, float* reward, uint8_t* done, int32_t* status,
                    uint32_t* bad_actions, int64_t n_games, uint64_t seed, int64_t game_offset,
                    void* stream);

/* orx_env_step_ex with its arguments in one block (ABI 7): a host that
 * calls it every tick (VecEnv.step) builds a block per output set once and
 * per call updates only what changed -- through ctypes one pointer argument
 * instead of sixteen (1.7 -> 0.5 us of host time per call, measured).  Same
 * checks, same results. */
typedef struct orx_env_step_args {
  const orx_cfg_t* cfg;
  const orx_state_t* st;
  const void* actions;
  int32_t action_bytes;
  int32_t action_cols;
  int32_t policy_p2;
  int32_t pad0;       /* (zero) */
  int8_t* act;
  int32_t* obs;
  float* reward;
  uint8_t* done;
  int32_t* status;
  uint32_t* bad_actions;
  int64_t n_games;
  uint64_t seed;
  int64_t game_offset;
  void* stream;
} orx_env_step_args_t;
int orx_env_step_args(const orx_env_step_args_t* args);

/* Fused rollout: n_ticks x (orx_policy then orx_step) in one launch, state
 * kept in registers between ticks.  If obs != NULL, tick t's post-step
 * observation is written to obs[(t * ORX_OBS_FIELDS + f) * n_games + b]
 * (int32) and its actions to act[(t * n_games + b) * 2 + p] (int8, may be
 * NULL).  Bit-identical to the unfused sequence (tested).  Replaces the
 * server hot loop server/main.py:110-113 around Updater.update. */
int orx_rollout(const orx_cfg_t* cfg, const orx_state_t* st, int32_t policy_p1,
                int32_t policy_p2, int32_t n_ticks, int32_t* obs, int8_t* act,
                int64_t n_games, uint64_t seed, int64_t game_offset,
                void* stream);

/* Trajectory row formats (orx_rollout_ex obs_format).
 * ORX_OBS_INT32: obs int32 [n_ticks][ORX_OBS_FIELDS][n_games], as orx_rollout.
 * ORX_OBS_COMPACT: obs uint32 [n_ticks][ORX_OBS_COMPACT_FIELDS][n_games], the
 * same observation in 24 bytes instead of 56 (GameState fields, state.py:25-34):
 *   row 0  p1.x | p1.y << 8 | p2.x << 16 | p2.y << 24        (u8 each)
 *   row 1  p1 staircase x | y << 8 | p2 staircase x << 16 | y << 24
 *   row 2  (uint16)p1.health | (uint16)p2.health << 16      (int16 each)
 *   row 3  p1.depth, row 4 p2.depth                        (int32)
 *   row 5  tick | status << 27                             (tick < 2^27)
 * It needs width, height <= 256, 1 <= max_ticks < 2^27, and health that
 * stays within int16: player_health, player_damage, npc_damage, mana_max
 * (ORX_EXT_MANA), item_bonus * item_slots (ORX_EXT_ITEMS) and max_ticks /
 * sep_period (ORX_EXT_SEPARATION_DAMAGE) each <= ORX_COMPACT_MAX_STAT;
 * otherwise orx_rollout_ex returns ORX_EINVAL. */
#define ORX_OBS_INT32 0
#define ORX_OBS_COMPACT 1
#define ORX_OBS_COMPACT_FIELDS 6
#define ORX_COMPACT_MAX_STAT 8000

/* orx_rollout_concurrent with a trajectory row format (obs_format:
 * ORX_OBS_INT32 or ORX_OBS_COMPACT; act is unchanged).  Results other than
 * the rows' encoding do not depend on it.  No reference counterpart (the
 * reference's observation is a GameState view, state.py:53-58). */
int orx_rollout_ex(const orx_cfg_t* cfg, const orx_state_t* st, int32_t policy_p1,
                   int32_t policy_p2, int32_t n_ticks, int32_t* obs, int8_t* act,
                   int32_t obs_format, int64_t n_games, uint64_t seed, int64_t game_offset,
                   int32_t concurrency, void* stream);

/* orx_rollout as one of `concurrency` (>= 1) launches that run on the device
 * together -- a GPU's batch split over concurrent streams, as
 * StreamShardedEngine does: the launch shape (orx_rollout_shape) is chosen
 * for the device's whole load.  Results do not depend on it; orx_rollout is
 * concurrency 1.  No reference counterpart. */
int orx_rollout_concurrent(const orx_cfg_t* cfg, const orx_state_t* st, int32_t policy_p1,
                           int32_t policy_p2, int32_t n_ticks, int32_t* obs, int8_t* act,
                           int64_t n_games, uint64_t seed, int64_t game_offset,
                           int32_t concurrency, void* stream);

/* Staircase (sx[j], sy[j]) of dungeon `depths[j]`, generation `gens[j]`, of
 * episode `episodes[j]` of global game `game_ids[j]`: the keyed
 * EmptyDungeonGenerator.spawn_dungeon (worldgen.py:33-43).  Used to
 * materialize World.dungeons (world.py:101-135) for depths no player stands
 * on; device arrays of length n. */
int orx_dungeon_stairs(const orx_cfg_t* cfg, const uint32_t* game_ids, const int32_t* episodes,
                       const int32_t* depths, const int32_t* gens, int32_t* sx, int32_t* sy,
                       int64_t n, uint64_t seed, void* stream);

/* orx_dungeon_stairs for any generator: also writes layout[j] (the bank
 * layout, or -1 for EmptyDungeonGenerator; layout may be NULL).  Only the
 * bank_* pointers of st are read. */
int orx_dungeon_spawn(const orx_cfg_t* cfg, const orx_state_t* st, const uint32_t* game_ids,
                      const int32_t* episodes, const int32_t* depths, const int32_t* gens,
                      int32_t* sx, int32_t* sy, int32_t* layout, int64_t n, uint64_t seed,
                      void* stream);

#ifdef __cplusplus
}
#endif

#endif /* ORX_H */
