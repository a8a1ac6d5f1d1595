/* Plain-C consumer of the C-ABI (include/orx.h): proves the boundary is
 * callable without C++, torch or HIP headers -- the way a cgo / JNI / N-API /
 * ctypes binding sees it.  Built and run by tests/test_abi.py (no GPU calls). */
#include <stddef.h>
#include <stdio.h>
#include <string.h>

#include "orx.h"

int main(void) {
  if (orx_abi_version() != ORX_ABI_VERSION) { printf("abi mismatch\n"); return 1; }
  orx_cfg_t c;
  memset(&c, 0, sizeof c);
  c.width = 64; c.height = 64; c.despawn = ORX_DESPAWN_UNREACHABLE; c.max_ticks = 1000;
  c.start_mode = ORX_START_TOGETHER; c.n_npcs = 8; c.npc_health = 3; c.npc_damage = 1;
  c.player_health = 10; c.player_damage = 2; c.player_armor = 1; c.autoreset = 1;
  if (orx_validate_cfg(&c) != ORX_OK) { printf("valid cfg rejected: %s\n", orx_last_error()); return 2; }
  c.width = 3;
  if (orx_validate_cfg(&c) != ORX_EINVAL) { printf("bad cfg accepted\n"); return 3; }
  if (strlen(orx_last_error()) == 0) { printf("no error message\n"); return 4; }
  c.width = 64;
  c.n_layouts = 40000; /* dungeon bank: at most 32767 layouts */
  if (orx_validate_cfg(&c) != ORX_EINVAL) { printf("bad bank accepted\n"); return 8; }
  c.n_layouts = 0;
  /* zero games: no device work, no pointers needed */
  if (orx_step(&c, NULL, NULL, 0, 1, 0, NULL) != ORX_OK) { printf("empty step failed\n"); return 5; }
  if (orx_rollout(&c, NULL, ORX_POLICY_RANDOM, ORX_POLICY_RANDOM, 5, NULL, NULL, 0, 1, 0, NULL) != ORX_OK) return 6;
  if (orx_step(&c, NULL, NULL, 16, 1, 0, NULL) != ORX_EINVAL) { printf("NULL state accepted\n"); return 7; }
  /* ABI 5: the learner's tick and the row formats -- argument checks only */
  if (orx_env_step(&c, NULL, NULL, 8, 1, ORX_POLICY_RANDOM, NULL, NULL, NULL, NULL, NULL, 0, 1, 0,
                   NULL) != ORX_OK) { printf("empty env step failed\n"); return 9; }
  if (orx_env_step(&c, NULL, NULL, 3, 1, ORX_POLICY_RANDOM, NULL, NULL, NULL, NULL, NULL, 16, 1, 0,
                   NULL) != ORX_EINVAL) { printf("3-byte actions accepted\n"); return 10; }
  /* ABI 6: the refused-action count; one action column needs a policy for player 2 */
  if (orx_env_step_ex(&c, NULL, NULL, 8, 1, ORX_POLICY_RANDOM, NULL, NULL, NULL, NULL, NULL, NULL,
                      0, 1, 0, NULL) != ORX_OK) { printf("empty env step ex failed\n"); return 13; }
  if (orx_env_step_ex(&c, NULL, NULL, 8, 1, ORX_POLICY_NONE, NULL, NULL, NULL, NULL, NULL, NULL,
                      16, 1, 0, NULL) != ORX_EINVAL) { printf("player 2 without a move accepted\n"); return 14; }
  /* ABI 6: n ticks of given actions in one launch */
  if (orx_step_n(&c, NULL, NULL, 5, NULL, ORX_OBS_INT32, 0, 1, 0, NULL) != ORX_OK) {
    printf("empty step_n failed\n"); return 16;
  }
  if (orx_step_n(&c, NULL, NULL, -1, NULL, ORX_OBS_INT32, 16, 1, 0, NULL) != ORX_EINVAL) {
    printf("negative n_ticks accepted\n"); return 17;
  }
  if (orx_step_n_ex(&c, NULL, NULL, 5, NULL, ORX_OBS_INT32, 16, 1, 0, 0, NULL) != ORX_EINVAL) {
    printf("orx_step_n_ex accepted concurrency 0\n"); return 20;
  }
  {
    orx_rollout_shape_t sh;
    if (orx_rollout_shape(&c, ORX_POLICY_RANDOM, ORX_POLICY_RANDOM, 65536, 1, 1, &sh) != ORX_OK ||
        sh.threads_per_block <= 0 || sh.lds_bytes != 0) { printf("rollout shape failed\n"); return 15; }
  }
  if (orx_rollout_ex(&c, NULL, ORX_POLICY_RANDOM, ORX_POLICY_RANDOM, 5, NULL, NULL, ORX_OBS_COMPACT,
                     0, 1, 0, 1, NULL) != ORX_OK) { printf("empty compact rollout failed\n"); return 11; }
  if (orx_rollout_ex(&c, NULL, ORX_POLICY_RANDOM, ORX_POLICY_RANDOM, 5, NULL, NULL, 7, 16, 1, 0, 1,
                     NULL) != ORX_EINVAL) { printf("unknown row format accepted\n"); return 12; }
  /* ABI 7: the enemy AI and its event-record bound */
  c.n_npcs = 8;
  c.npc_policy = ORX_NPC_RANDOM;
  if (orx_validate_cfg(&c) != ORX_OK || orx_max_events(&c) != 6 + 2 * 8) {
    printf("moving NPCs refused or their event bound wrong\n"); return 18;
  }
  c.npc_policy = ORX_NPC_STAY;
  if (orx_max_events(&c) != ORX_MAX_EVENTS) { printf("event bound wrong\n"); return 19; }
  /* ABI 7: orx_env_step_ex's arguments as one block */
  {
    orx_env_step_args_t ea;
    memset(&ea, 0, sizeof ea);
    ea.cfg = &c;
    ea.action_bytes = 8;
    ea.action_cols = 1;
    ea.policy_p2 = ORX_POLICY_RANDOM;
    ea.seed = 1;
    if (orx_env_step_args(&ea) != ORX_OK) { printf("empty env step args failed\n"); return 21; }
    ea.policy_p2 = ORX_POLICY_NONE;
    ea.n_games = 16;
    if (orx_env_step_args(&ea) != ORX_EINVAL) { printf("env step args unchecked\n"); return 22; }
    if (orx_env_step_args(NULL) != ORX_EINVAL) { printf("NULL env step args accepted\n"); return 23; }
  }
  c.n_npcs = 8;
  printf("sizeof(orx_cfg_t)=%zu sizeof(orx_state_t)=%zu off_flags=%zu off_npc_alive=%zu "
         "sizeof(orx_env_step_args_t)=%zu off_stream=%zu\n",
         sizeof(orx_cfg_t), sizeof(orx_state_t), offsetof(orx_cfg_t, flags),
         offsetof(orx_state_t, npc_alive), sizeof(orx_env_step_args_t),
         offsetof(orx_env_step_args_t, stream));
  return 0;
}
