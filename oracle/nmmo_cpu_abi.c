/* nmmo_cpu_abi.c — TEST INFRASTRUCTURE ONLY: the CPU oracle behind the product's C-ABI.
 *
 * libnmmo_cpu.so exports every entry point include/nmmo_hip.h declares, implemented over the
 * serial CPU restatement in nmmo_oracle.c ("The C++ CPU stepper exports the same
 * symbols (libnmmo_cpu.so, with host pointers and `stream` ignored), so tests can swap backends").
 * Every buffer is HOST memory here; `stream` and `device` are ignored; the calls the oracle has
 * no counterpart for (the native / wire layouts, the device experience storage, the wrapper
 * layer, device allocations, kernel timing and device counters) return NMMO_E_INVALID with a
 * message. Like the rest of oracle/, nothing in the product path loads it: tests do
 * (tests/test_cpu_abi.py), against the HIP library's host-side results.
 */
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/nmmo_hip.h"

/* the oracle's own API (nmmo_oracle.c) */
void* oracle_create(const NmmoConfig* cfg, int n_envs, uint64_t seed, const uint16_t* task_emb);
void oracle_destroy(void* h);
int oracle_reset(void* h, const uint64_t* env_seeds, float* obs, uint8_t* mask);
int oracle_end_episodes(void* h, const uint8_t* env_mask);
int oracle_write_obs(void* h, int env, float* obs_env);
int oracle_step(void* h, const int32_t* actions, float* obs, float* rew, uint8_t* term, uint8_t* trunc,
                uint8_t* mask);
int oracle_step_range(void* h, int env_lo, int env_hi, const int32_t* actions, float* obs, float* rew,
                      uint8_t* term, uint8_t* trunc, uint8_t* mask);
int oracle_scripted_actions(void* h, uint64_t pseed, int32_t* actions);
int oracle_get_state(void* h, void* buf, size_t nbytes);
int oracle_set_state(void* h, const void* buf, size_t nbytes);
int oracle_set_tasks(void* h, const NmmoTask* tasks, int n_tasks, const uint16_t* emb, const int32_t* assign);
int oracle_set_task_weights(void* h, const double* w, int n_tasks);
int oracle_get_events(void* h, int env, int32_t* rows, int max_rows, int* n_rows);
int oracle_set_map_bank(void* h, const uint8_t* buf, size_t nbytes);
int oracle_get_map_bank(void* h, uint8_t* buf, size_t nbytes);
int oracle_obs_elems(int task_dim);

struct NmmoHandle {
  void* o;
  NmmoConfig cfg;
  NmmoLayout layout;
  int n_envs;
  int32_t fault;  /* nmmo_step_envs' dropped ids, nmmo_inject_fault */
};

static _Thread_local char g_err[512];

static int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
static int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return code;
}
#define UNSUPPORTED(name) return fail(NMMO_E_INVALID, "%s: not in the CPU stepper (libnmmo_cpu.so)", name)

NMMO_API int32_t nmmo_abi_version(void) { return NMMO_ABI_VERSION; }
NMMO_API const char* nmmo_last_error(void) { return g_err; }
NMMO_API const char* nmmo_build_info(void) { return "src=cpu-oracle arch=host"; }

NMMO_API void nmmo_default_config(NmmoConfig* c) {
  memset(c, 0, sizeof *c);
  c->abi_version = NMMO_ABI_VERSION;
  c->player_n = 128;
  c->npc_n = 256;
  c->horizon = 1024;
  c->map_n = 256;
  c->spawn_immunity = 20;
  c->resilient_u32 = 858993459u; /* 0.2 * 2^32 */
  c->systems = NMMO_SYS_ALL;
  c->obs_layout = NMMO_OBS_FLAT;
  c->task_embed_dim = 2048;
  c->task_num_tick = 1024;
  c->event_cap = 4096;
}

/* SPEC §8's flat layout, pufferlib sorted-key order */
NMMO_API int nmmo_layout(const NmmoConfig* cfg, NmmoLayout* L) {
  if (!cfg || !L) return fail(NMMO_E_INVALID, "null argument");
  memset(L, 0, sizeof *L);
  static const int dims[NMMO_N_ACTION_HEADS] = {3, 101, 1025, 13, 13, 101, 99, 101, 5, 13, 99, 13};
  int32_t* offs[NMMO_N_ACTION_HEADS] = {
      &L->off_mask_attack_style, &L->off_mask_attack_target, &L->off_mask_buy, &L->off_mask_destroy,
      &L->off_mask_give_item, &L->off_mask_give_target, &L->off_mask_givegold_price,
      &L->off_mask_givegold_target, &L->off_mask_move, &L->off_mask_sell_item, &L->off_mask_sell_price,
      &L->off_mask_use};
  int o = 0;
  L->act_heads = NMMO_N_ACTION_HEADS;
  for (int h = 0; h < NMMO_N_ACTION_HEADS; h++) {
    L->act_dims[h] = dims[h];
    *offs[h] = o;
    o += dims[h];
  }
  L->off_agent_id = o++;
  L->off_current_tick = o++;
  L->off_entity = o; o += 100 * NMMO_N_ENTITY_COLS;
  L->off_inventory = o; o += NMMO_INV_SLOTS * 16;
  L->off_market = o; o += NMMO_MARKET_ROWS * 16;
  L->off_task = o; o += cfg->task_embed_dim;
  L->off_tile = o; o += 225 * 3;
  L->obs_elems = o;
  L->entity_rows = 100; L->entity_cols = NMMO_N_ENTITY_COLS;
  L->inventory_rows = NMMO_INV_SLOTS; L->item_cols = 16; L->market_rows = NMMO_MARKET_ROWS;
  L->tile_rows = 225; L->tile_cols = 3;
  L->slots = cfg->player_n + ((cfg->systems & NMMO_SYS_NPC) ? cfg->npc_n : 0);
  L->nf = NMMO_NF;
  L->ne = NMMO_NE;
  L->state_bytes_per_env = (size_t)NMMO_NE * 4 + (size_t)NMMO_NF * L->slots * 2 + (size_t)L->slots * 2 +
                           NMMO_MAP_TILES + (size_t)cfg->player_n * NMMO_INV_SLOTS * 8 +
                           (size_t)NMMO_INV_SLOTS * cfg->player_n * 2 + (size_t)cfg->player_n * 4 +
                           (size_t)cfg->player_n * sizeof(NmmoTaskState);
  if (L->obs_elems != oracle_obs_elems(cfg->task_embed_dim)) return fail(NMMO_E_INVALID, "layout mismatch");
  return NMMO_OK;
}

NMMO_API int nmmo_create(const NmmoConfig* cfg, int32_t n_envs, uint64_t seed, int32_t device,
                         const uint16_t* task_embedding, NmmoHandle** out) {
  (void)device;
  if (!cfg || !out) return fail(NMMO_E_INVALID, "null argument");
  *out = NULL;
  if (cfg->abi_version != NMMO_ABI_VERSION)
    return fail(NMMO_E_INVALID, "abi_version %d != %d", cfg->abi_version, NMMO_ABI_VERSION);
  if (cfg->obs_layout != NMMO_OBS_NONE && cfg->obs_layout != NMMO_OBS_FLAT)
    return fail(NMMO_E_INVALID, "obs_layout %d: the CPU stepper writes the flat layout only", cfg->obs_layout);
  void* o = oracle_create(cfg, n_envs, seed, task_embedding);
  if (!o) return fail(NMMO_E_INVALID, "invalid config or n_envs");
  NmmoHandle* h = (NmmoHandle*)calloc(1, sizeof *h);
  h->o = o;
  h->cfg = *cfg;
  h->n_envs = n_envs;
  nmmo_layout(cfg, &h->layout);
  *out = h;
  return NMMO_OK;
}

NMMO_API void nmmo_destroy(NmmoHandle* h) {
  if (!h) return;
  oracle_destroy(h->o);
  free(h);
}

NMMO_API int32_t nmmo_n_envs(const NmmoHandle* h) { return h ? h->n_envs : 0; }

static float* flat_or_null(const NmmoHandle* h, void* obs) {
  return h->cfg.obs_layout == NMMO_OBS_FLAT ? (float*)obs : NULL;
}

NMMO_API int nmmo_reset(NmmoHandle* h, const uint64_t* env_seeds, void* obs, uint8_t* mask, void* stream) {
  (void)stream;
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  return oracle_reset(h->o, env_seeds, flat_or_null(h, obs), mask);
}

NMMO_API int nmmo_end_episodes(NmmoHandle* h, const uint8_t* env_mask, void* stream) {
  (void)stream;
  if (!h || !env_mask) return fail(NMMO_E_INVALID, "null argument");
  return oracle_end_episodes(h->o, env_mask);
}

NMMO_API int nmmo_step(NmmoHandle* h, const int32_t* actions, void* obs, float* rew, uint8_t* term, uint8_t* trunc,
                       uint8_t* mask, void* stream) {
  (void)stream;
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  if (!actions || !rew || !term || !trunc || !mask)
    return fail(NMMO_E_INVALID, "actions/rew/term/trunc/mask must be host pointers");
  return oracle_step(h->o, actions, flat_or_null(h, obs), rew, term, trunc, mask);
}

/* host env_ids; the listed envs step in list order (envs are independent, so any order gives the
 * same state) */
NMMO_API int nmmo_step_envs(NmmoHandle* h, const int32_t* env_ids, int32_t n_ids, const int32_t* actions, void* obs,
                            float* rew, uint8_t* term, uint8_t* trunc, uint8_t* mask, void* stream) {
  (void)stream;
  if (!h || !env_ids) return fail(NMMO_E_INVALID, "null handle / env_ids");
  if (n_ids < 0 || n_ids > h->n_envs) return fail(NMMO_E_INVALID, "n_ids %d not in 0..%d", n_ids, h->n_envs);
  if (!actions || !rew || !term || !trunc || !mask)
    return fail(NMMO_E_INVALID, "actions/rew/term/trunc/mask must be host pointers");
  for (int i = 0; i < n_ids; i++) {
    const int e = env_ids[i];
    if (e < 0 || e >= h->n_envs) {
      if (!h->fault) h->fault = NMMO_FAULT_ENV_LIST | i << 8;
      continue;
    }
    int rc = oracle_step_range(h->o, e, e + 1, actions, flat_or_null(h, obs), rew, term, trunc, mask);
    if (rc) return rc;
  }
  return NMMO_OK;
}

NMMO_API int nmmo_observe(NmmoHandle* h, void* obs, void* stream) {
  (void)stream;
  if (!h || !obs) return fail(NMMO_E_INVALID, "null argument");
  if (h->cfg.obs_layout != NMMO_OBS_FLAT) return fail(NMMO_E_INVALID, "handle built without flat obs");
  const size_t per_env = (size_t)h->cfg.player_n * h->layout.obs_elems;
  for (int e = 0; e < h->n_envs; e++) oracle_write_obs(h->o, e, (float*)obs + per_env * e);
  return NMMO_OK;
}

NMMO_API int nmmo_scripted_actions(NmmoHandle* h, uint64_t policy_seed, int32_t* actions, void* stream) {
  (void)stream;
  if (!h || !actions) return fail(NMMO_E_INVALID, "null argument");
  return oracle_scripted_actions(h->o, policy_seed, actions);
}

NMMO_API int nmmo_get_state(NmmoHandle* h, void* host_buf, size_t nbytes) {
  if (!h || !host_buf) return fail(NMMO_E_INVALID, "null argument");
  if (nbytes != h->layout.state_bytes_per_env * h->n_envs) return fail(NMMO_E_SIZE, "state buffer size");
  return oracle_get_state(h->o, host_buf, nbytes);
}
NMMO_API int nmmo_set_state(NmmoHandle* h, const void* host_buf, size_t nbytes) {
  if (!h || !host_buf) return fail(NMMO_E_INVALID, "null argument");
  if (nbytes != h->layout.state_bytes_per_env * h->n_envs) return fail(NMMO_E_SIZE, "state buffer size");
  return oracle_set_state(h->o, host_buf, nbytes);
}
NMMO_API int nmmo_get_map_bank(NmmoHandle* h, uint8_t* host_buf, size_t nbytes) {
  if (!h || !host_buf) return fail(NMMO_E_INVALID, "null argument");
  return oracle_get_map_bank(h->o, host_buf, nbytes);
}
NMMO_API int nmmo_set_map_bank(NmmoHandle* h, const uint8_t* host_buf, size_t nbytes) {
  if (!h || !host_buf) return fail(NMMO_E_INVALID, "null argument");
  return oracle_set_map_bank(h->o, host_buf, nbytes);
}
NMMO_API int nmmo_set_tasks(NmmoHandle* h, const NmmoTask* tasks, int32_t n_tasks, const uint16_t* embeddings,
                            const int32_t* assign) {
  if (!h || !tasks) return fail(NMMO_E_INVALID, "null argument");
  if (n_tasks < 1 || n_tasks > NMMO_MAX_TASKS) return fail(NMMO_E_INVALID, "n_tasks %d", n_tasks);
  for (int i = 0; i < n_tasks; i++)  /* the HIP tick packs a term's a in 24 bits (capi.hip nmmo_set_tasks) */
    for (int k = 0; k < 2; k++)
      if (tasks[i].term[k].a < -(1 << 23) || tasks[i].term[k].a >= (1 << 23))
        return fail(NMMO_E_INVALID, "task %d term %d: a outside +/-2^23", i, k);
  return oracle_set_tasks(h->o, tasks, n_tasks, embeddings, assign);
}
NMMO_API int nmmo_set_task_weights(NmmoHandle* h, const double* weights, int32_t n_tasks) {
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  return oracle_set_task_weights(h->o, weights, n_tasks);
}
NMMO_API int nmmo_get_events(NmmoHandle* h, int32_t env, int32_t* host_rows, int32_t max_rows, int32_t* n_rows) {
  if (!h || !n_rows) return fail(NMMO_E_INVALID, "null argument");
  if (env < 0 || env >= h->n_envs) return fail(NMMO_E_INVALID, "env %d out of range", env);
  return oracle_get_events(h->o, env, host_rows, max_rows, n_rows);
}

/* ---- the device-only parts of the ABI ---- */
NMMO_API int nmmo_set_wrapper(NmmoHandle* h, const NmmoWrapperConfig* wc, NmmoAgentInfo* dev_info) {
  (void)h; (void)wc; (void)dev_info;
  UNSUPPORTED("nmmo_set_wrapper");
}
NMMO_API int nmmo_get_wrapper_state(NmmoHandle* h, NmmoWrapState* s, uint32_t* u) {
  (void)h; (void)s; (void)u;
  UNSUPPORTED("nmmo_get_wrapper_state");
}
NMMO_API int nmmo_get_wrapper_dropped(NmmoHandle* h, int64_t* total) {
  (void)h; (void)total;
  UNSUPPORTED("nmmo_get_wrapper_dropped");
}
NMMO_API int nmmo_expand_obs(NmmoHandle* h, const void* native, float* flat, int32_t n_envs, void* stream) {
  (void)h; (void)native; (void)flat; (void)n_envs; (void)stream;
  UNSUPPORTED("nmmo_expand_obs");
}
NMMO_API int nmmo_dev_alloc(int32_t device, uint64_t bytes, void** out) {
  (void)device; (void)bytes; (void)out;
  UNSUPPORTED("nmmo_dev_alloc");
}
NMMO_API int nmmo_dev_free(void* ptr) {
  (void)ptr;
  UNSUPPORTED("nmmo_dev_free");
}
NMMO_API int64_t nmmo_wire_header_bytes(int32_t n_envs, int32_t player_n) {
  if (n_envs <= 0 || player_n <= 0 || player_n > 128) return fail(NMMO_E_INVALID, "n_envs > 0, player_n in 1..128");
  return ((8 + 8 * (int64_t)n_envs + 2 * (int64_t)n_envs * player_n + 4 * (int64_t)n_envs) + 15) & ~(int64_t)15;
}
NMMO_API int64_t nmmo_wire_max_bytes(int32_t n_envs, int32_t player_n) {
  const int64_t hdr = nmmo_wire_header_bytes(n_envs, player_n);
  if (hdr < 0) return hdr;
  /* SPEC §8c v4 record: head, 100 indices, 12 Inventory rows, 114 B of materials, the mask stream */
  const int64_t rec = (16 + 2 * 100 + 32 * NMMO_INV_SLOTS + 114 + 2 * ((3 * 100 + 4 * NMMO_INV_SLOTS + 15) / 16) + 15) & ~15;
  const int64_t table = (62 * 384 + 15) & ~15; /* a full entity table (kMaxSlots rows) */
  return hdr + (int64_t)n_envs * (table + (int64_t)player_n * rec + NMMO_NATIVE_MARKET_BYTES);
}
NMMO_API int nmmo_wire_pack(NmmoHandle* h, const void* native, void* wire, void* stream) {
  (void)h; (void)native; (void)wire; (void)stream;
  UNSUPPORTED("nmmo_wire_pack");
}
NMMO_API int nmmo_sizes_row(const void* const* w, int32_t n, int32_t* f, int64_t* row, void* stream) {
  (void)w; (void)n; (void)f; (void)row; (void)stream;
  UNSUPPORTED("nmmo_sizes_row");
}
NMMO_API int nmmo_p2p_load(const char* path) { (void)path; UNSUPPORTED("nmmo_p2p_load"); }
NMMO_API int nmmo_p2p_unique_id(void* id) { (void)id; UNSUPPORTED("nmmo_p2p_unique_id"); }
NMMO_API int nmmo_p2p_init(const void* id, int32_t world, int32_t rank, void** comm) {
  (void)id; (void)world; (void)rank; (void)comm;
  UNSUPPORTED("nmmo_p2p_init");
}
NMMO_API int nmmo_p2p_group(void* comm, const NmmoP2POp* ops, int32_t n_ops, void* stream) {
  (void)comm; (void)ops; (void)n_ops; (void)stream;
  UNSUPPORTED("nmmo_p2p_group");
}
NMMO_API int nmmo_p2p_destroy(void* comm) { (void)comm; UNSUPPORTED("nmmo_p2p_destroy"); }
NMMO_API int nmmo_wire_unpack(int32_t n, int32_t p, const void* wire, void* native, void* stream) {
  (void)n; (void)p; (void)wire; (void)native; (void)stream;
  UNSUPPORTED("nmmo_wire_unpack");
}
NMMO_API int nmmo_wire_check(const void* wire, int32_t n, int32_t p, const int64_t* e, int32_t* s, void* stream) {
  (void)wire; (void)n; (void)p; (void)e; (void)s; (void)stream;
  UNSUPPORTED("nmmo_wire_check");
}
NMMO_API int nmmo_wire_check_many(const void* const* w, const int32_t* n, const int64_t* const* e, int32_t nb,
                                  int32_t p, int32_t* s, void* stream) {
  (void)w; (void)n; (void)e; (void)nb; (void)p; (void)s; (void)stream;
  UNSUPPORTED("nmmo_wire_check_many");
}
NMMO_API int nmmo_set_timing(NmmoHandle* h, int32_t enable) {
  (void)h; (void)enable;
  UNSUPPORTED("nmmo_set_timing");
}
NMMO_API int nmmo_read_timing(NmmoHandle* h, double* ms, int32_t* n) {
  (void)h; (void)ms; (void)n;
  UNSUPPORTED("nmmo_read_timing");
}
NMMO_API int nmmo_get_fault(NmmoHandle* h, int32_t* fault) {  /* the serial oracle has no round loops */
  if (!h || !fault) return fail(NMMO_E_INVALID, "null argument");
  *fault = h->fault;
  h->fault = 0;
  return NMMO_OK;
}
NMMO_API int nmmo_exp_store_records(NmmoHandle* h, const NmmoExperience* x, const NmmoRecordStore* rs,
                                    const NmmoStoreInput* in, int32_t* scratch, void* stream) {
  (void)h; (void)x; (void)rs; (void)in; (void)scratch; (void)stream;
  UNSUPPORTED("nmmo_exp_store_records");
}
NMMO_API int nmmo_exp_store_records_many(NmmoHandle* h, const NmmoExperience* x, const NmmoRecordStore* rs,
                                         const NmmoStoreInput* ins, int32_t n_inputs, int32_t field_stride,
                                         int32_t* scratch, void* stream) {
  (void)h; (void)x; (void)rs; (void)ins; (void)n_inputs; (void)field_stride; (void)scratch; (void)stream;
  UNSUPPORTED("nmmo_exp_store_records_many");
}
NMMO_API int nmmo_exp_store_records_checked(NmmoHandle* h, const NmmoExperience* x, const NmmoRecordStore* rs,
                                            const NmmoStoreInput* ins, int32_t n_inputs, int32_t field_stride,
                                            const int64_t* const* e, uint32_t m, int32_t* cs, int32_t* ctl,
                                            int32_t* scratch, void* stream) {
  (void)h; (void)x; (void)rs; (void)ins; (void)n_inputs; (void)field_stride; (void)e; (void)m; (void)cs; (void)ctl;
  (void)scratch; (void)stream;
  UNSUPPORTED("nmmo_exp_store_records_checked");
}
NMMO_API int nmmo_exp_gather_records(NmmoHandle* h, const NmmoExperience* x, const NmmoRecordStore* rs,
                                     const int32_t* idx, int32_t n, float* out, void* stream) {
  (void)h; (void)x; (void)rs; (void)idx; (void)n; (void)out; (void)stream;
  UNSUPPORTED("nmmo_exp_gather_records");
}
NMMO_API int nmmo_fault_into(NmmoHandle* h, int32_t* dst, void* stream) {  /* host dst */
  (void)stream;
  if (!h || !dst) return fail(NMMO_E_INVALID, "null argument");
  if (h->fault && !*dst) *dst = h->fault;
  return NMMO_OK;
}
NMMO_API int nmmo_inject_fault(NmmoHandle* h, int32_t fault) {
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  h->fault = fault;
  return NMMO_OK;
}
NMMO_API int nmmo_obs_bind(NmmoHandle* h, const void* obs) {
  (void)obs;
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  return NMMO_OK;  /* every obs call writes every row here */
}
NMMO_API int nmmo_obs_invalidate(NmmoHandle* h, void* stream) {
  (void)stream;
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  return NMMO_OK;  /* every obs call writes every row here */
}
NMMO_API int nmmo_obs_invalidate_envs(NmmoHandle* h, const int32_t* env_ids, int32_t n_ids, void* stream) {
  (void)env_ids; (void)n_ids; (void)stream;
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  return NMMO_OK;  /* every obs call writes every row here */
}
NMMO_API int nmmo_obs_invalidate_sections(NmmoHandle* h, const int32_t* env_ids, int32_t n_ids, uint32_t sections,
                                          void* stream) {
  (void)env_ids; (void)n_ids; (void)sections; (void)stream;
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  return NMMO_OK;  /* every obs call writes every row here */
}
NMMO_API int nmmo_set_obs_counter(NmmoHandle* h, uint64_t* c) {
  (void)h; (void)c;
  UNSUPPORTED("nmmo_set_obs_counter");
}
NMMO_API int nmmo_set_step_records(NmmoHandle* h, uint8_t* r, int32_t* f) {
  (void)h; (void)r; (void)f;
  UNSUPPORTED("nmmo_set_step_records");
}
NMMO_API int nmmo_set_counters(NmmoHandle* h, uint64_t* c) {
  (void)h; (void)c;
  UNSUPPORTED("nmmo_set_counters");
}
NMMO_API int64_t nmmo_exp_scratch_ints(int32_t max_rows, int32_t n_slots) {
  (void)max_rows; (void)n_slots;
  UNSUPPORTED("nmmo_exp_scratch_ints");
}
NMMO_API int64_t nmmo_exp_scratch_ints_many(int32_t n_inputs, int32_t max_rows, int32_t n_slots) {
  (void)n_inputs; (void)max_rows; (void)n_slots;
  UNSUPPORTED("nmmo_exp_scratch_ints_many");
}
NMMO_API int nmmo_exp_store(NmmoHandle* h, const NmmoExperience* x, const NmmoStoreInput* in, int32_t* s, void* st) {
  (void)h; (void)x; (void)in; (void)s; (void)st;
  UNSUPPORTED("nmmo_exp_store");
}
NMMO_API int nmmo_exp_sort(const NmmoExperience* x, int32_t* i, int32_t* s, void* st) {
  (void)x; (void)i; (void)s; (void)st;
  UNSUPPORTED("nmmo_exp_sort");
}
NMMO_API int nmmo_exp_gae(const NmmoExperience* x, const int32_t* i, int32_t b, double g, double l, float* a, void* st) {
  (void)x; (void)i; (void)b; (void)g; (void)l; (void)a; (void)st;
  UNSUPPORTED("nmmo_exp_gae");
}
NMMO_API int nmmo_gather_rows(const void* src, int64_t rb, const int32_t* idx, int32_t n, void* out, void* st) {
  (void)src; (void)rb; (void)idx; (void)n; (void)out; (void)st;
  UNSUPPORTED("nmmo_gather_rows");
}
