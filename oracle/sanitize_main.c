/* TEST INFRASTRUCTURE ONLY — the §5 sanitizer leg: drives the CPU oracle (nmmo_oracle.c) through
 * every entry point the parity tests use, built with -fsanitize=address,undefined
 * (tests/test_oracle_sanitize.py). Any out-of-bounds access, leak, signed overflow, misaligned
 * access or shift error aborts the run with a report.
 *
 * Workloads: the BASELINE system sets (C2 Resource, C3 + Combat/NPC/Progression, C4 all) at full
 * player/NPC counts with a short horizon (episodes end, are culled and auto-reset inside the run),
 * scripted masked-uniform actions, then uniformly random in-range actions (the tick must accept
 * any index a policy can emit), a forced end of episode, a state get/set round trip, the event
 * log and the flat obs of every step. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/nmmo_hip.h"

void* oracle_create(const NmmoConfig* cfg, int n_envs, uint64_t seed, const uint16_t* task_emb);
void oracle_destroy(void* h);
int oracle_reset(void* h, const uint64_t* env_seeds, float* obs, uint8_t* mask);
int oracle_end_episodes(void* h, const uint8_t* env_mask);
int oracle_step(void* h, const int32_t* actions, float* obs, float* rew, uint8_t* term,
                uint8_t* trunc, uint8_t* mask);
int oracle_scripted_actions(void* h, uint64_t pseed, int32_t* actions);
int oracle_get_state(void* h, void* buf, size_t nbytes);
int oracle_set_state(void* h, const void* buf, size_t nbytes);
int oracle_get_events(void* h, int env, int32_t* rows, int max_rows, int* n_rows);
int oracle_set_task_weights(void* h, const double* w, int n_tasks);
int oracle_obs_elems(int task_dim);
size_t oracle_state_bytes_per_env(int slots, int players);

static const int kDims[NMMO_N_ACTION_HEADS] = {3, 101, 1025, 13, 13, 101, 99, 101, 5, 13, 99, 13};

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t next_u32(void) {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (uint32_t)(rng >> 16);
}

static int run(const char* name, uint32_t systems, int ticks) {
  NmmoConfig cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.abi_version = NMMO_ABI_VERSION;
  cfg.player_n = 128;
  cfg.npc_n = 256;
  cfg.horizon = 48;
  cfg.map_n = 3;
  cfg.spawn_immunity = 20;
  cfg.early_stop_agent_num = 8;
  cfg.resilient_u32 = 0x33333333u;
  cfg.systems = systems;
  cfg.obs_layout = NMMO_OBS_FLAT;
  cfg.task_embed_dim = 2048;
  cfg.task_num_tick = 30;
  cfg.event_cap = 4096;
  const int n = 2, P = cfg.player_n;
  void* h = oracle_create(&cfg, n, 7, NULL);
  if (!h) return fprintf(stderr, "%s: create failed\n", name), 1;
  const int S = P + ((systems & NMMO_SYS_NPC) ? cfg.npc_n : 0);
  const size_t elems = (size_t)oracle_obs_elems(cfg.task_embed_dim);
  float* obs = malloc((size_t)n * P * elems * sizeof(float));
  float* rew = malloc((size_t)n * P * sizeof(float));
  uint8_t *term = malloc((size_t)n * P), *trunc = malloc((size_t)n * P), *mask = malloc((size_t)n * P);
  int32_t* act = malloc((size_t)n * P * NMMO_N_ACTION_HEADS * sizeof(int32_t));
  int32_t* rows = malloc((size_t)cfg.event_cap * NMMO_EVENT_COLS * sizeof(int32_t));
  const size_t sb = oracle_state_bytes_per_env(S, P) * n;
  unsigned char *st = malloc(sb), *st2 = malloc(sb);
  const double w[1] = {1.0};
  int rc = oracle_set_task_weights(h, w, 1);
  rc |= oracle_reset(h, NULL, obs, mask);
  long events = 0;
  for (int t = 0; t < ticks && !rc; t++) {
    if (t < ticks / 2) {
      rc |= oracle_scripted_actions(h, 1000 + (uint64_t)t, act);
    } else {
      for (int i = 0; i < n * P; i++)
        for (int k = 0; k < NMMO_N_ACTION_HEADS; k++)
          act[i * NMMO_N_ACTION_HEADS + k] = (int32_t)(next_u32() % (uint32_t)kDims[k]);
    }
    if (t == ticks / 3) {
      const uint8_t em[2] = {0, 1};
      rc |= oracle_end_episodes(h, em);
    }
    rc |= oracle_step(h, act, obs, rew, term, trunc, mask);
    for (int e = 0; e < n; e++) {
      int nr = 0;
      rc |= oracle_get_events(h, e, rows, cfg.event_cap, &nr);
      events += nr;
    }
    if (t == ticks / 2) {  // snapshot round trip
      rc |= oracle_get_state(h, st, sb);
      rc |= oracle_set_state(h, st, sb);
      rc |= oracle_get_state(h, st2, sb);
      if (memcmp(st, st2, sb)) return fprintf(stderr, "%s: state round trip differs\n", name), 1;
    }
  }
  double acc = 0;
  for (size_t i = 0; i < (size_t)n * P * elems; i += 4099) acc += obs[i];
  printf("%s: %d ticks x %d envs, %ld event rows, obs probe %.1f, rc %d\n", name, ticks, n, events, acc, rc);
  oracle_destroy(h);
  free(obs); free(rew); free(term); free(trunc); free(mask); free(act); free(rows); free(st); free(st2);
  return rc != 0;
}

int main(int argc, char** argv) {
  const int ticks = argc > 1 ? atoi(argv[1]) : 120;
  int bad = 0;
  bad |= run("C2", NMMO_SYS_RESOURCE, ticks);
  bad |= run("C3", NMMO_SYS_RESOURCE | NMMO_SYS_COMBAT | NMMO_SYS_NPC | NMMO_SYS_PROGRESSION, ticks);
  bad |= run("C4", NMMO_SYS_ALL, ticks);
  return bad;
}
