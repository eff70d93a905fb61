// capi.hip — the C-ABI of libnmmo_hip.so (include/nmmo_hip.h). Host side only: owns the
// device state (SoA over env x slot in HBM), enqueues the gfx950 kernels on the caller's
// stream, never synchronises inside nmmo_step (graph-capturable, no allocation).
#include <math.h>
#include <stdlib.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "kernels.h"
#include "wire.h"



using namespace nmmo;

static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
static int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
#define HIP_TRY(expr)                                                                    \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess) return fail(NMMO_E_HIP, "%s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

struct NmmoHandle {
  NmmoConfig cfg;
  NmmoLayout layout;
  DevState st;
  int device;
  int32_t* d_env = nullptr;
  int16_t* d_ent = nullptr;
  int16_t* d_ring = nullptr;
  uint8_t* d_mat = nullptr;
  uint32_t* d_dep = nullptr;
  int32_t* d_foreign = nullptr;  // DevState::foreign
  uint8_t* d_bank = nullptr;
  float* d_task = nullptr;
  uint64_t* d_seeds = nullptr;
  uint2* d_items = nullptr;
  int16_t* d_iring = nullptr;
  int32_t* d_mlist = nullptr;
  int32_t* d_mcount = nullptr;
  int32_t* d_events = nullptr;
  NmmoTask* d_tasks = nullptr;
  int32_t* d_assign = nullptr;
  NmmoTaskState* d_tstate = nullptr;
  uint16_t* d_wcount = nullptr;  // native obs: per-agent wire count words of the last obs (wire.hip)
  int32_t* d_wmcount = nullptr;  // native obs: per-env listing count of the last obs
  uint16_t* d_wrank = nullptr;   // wire obs: per-slot entity-table index (wire_count_kernel)
  uint32_t* d_wpk = nullptr;     // wire obs: per-env packed datastore-row words (wire_count_kernel)
  // flat / native obs: per agent row, the tag of the buffer the row state describes and the state
  // (ObsParams::zrow / zst); NMMO_OBS_REZERO=1 at create time writes every row in full
  uint64_t* d_zrow = nullptr;
  uint64_t* d_zext = nullptr;  // flat rows' extended state (ObsParams::zext)
  bool zskip = true;
  bool wire_fuse = true;  // the tick writes the wire count words (DevState::wf); NMMO_WIRE_FUSE=0 at create: off
  const void* zbuf = nullptr;  // the bound obs buffer (nmmo_obs_bind) and its tag
  uint64_t ztag = 0;
  unsigned long long* d_rows_out = nullptr;  // nmmo_set_obs_counter
  uint8_t* d_recs = nullptr;                 // nmmo_set_step_records
  int32_t* d_recs_fault = nullptr;
  // the native buffer the last obs gather wrote, and whether no tick ran since (nmmo_wire_pack)
  const void* last_native = nullptr;
  bool native_fresh = false;
  // wrapper layer (nmmo_set_wrapper, SPEC §13)
  bool wrap_on = false;
  NmmoWrapperConfig wc{};
  NmmoWrapState* d_ws = nullptr;
  uint32_t* d_uniq = nullptr;
  int32_t* d_wenv = nullptr;
  uint64_t* d_task_cum = nullptr;
  unsigned long long* d_wdrop = nullptr;
  NmmoAgentInfo* d_info = nullptr;  // caller-owned
  // bench timing (nmmo_set_timing): event pairs around the tick and obs kernels
  bool timing = false;
  int t_count = 0;
  std::vector<hipEvent_t> ev;  // [kTimingCap][4]: tick begin, tick end, wrapper end, obs end
};
static constexpr int kTimingCap = 8192;

static float half_to_float(uint16_t h) {
  uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 31, m = h & 1023, bits;
  if (e == 0) {
    if (m == 0) {
      bits = s;
    } else {
      int sh = 0;
      while (!(m & 1024)) { m <<= 1; sh++; }
      m &= 1023;
      bits = s | ((uint32_t)(127 - 15 - sh + 1) << 23) | (m << 13);
    }
  } else if (e == 31) {
    bits = s | 0x7F800000u | (m << 13);
  } else {
    bits = s | ((e + 112) << 23) | (m << 13);
  }
  float f;
  memcpy(&f, &bits, 4);
  return f;
}

extern "C" {

int32_t nmmo_abi_version(void) { return NMMO_ABI_VERSION; }
#ifndef NMMO_SRC_HASH
#define NMMO_SRC_HASH "unknown"
#endif
const char* nmmo_build_info(void) {
  return "src=" NMMO_SRC_HASH " arch=gfx950 fp_contract=off"
#ifdef NMMO_STAMPS
         " stamps=1"
#endif
      ;
}
const char* nmmo_last_error(void) { return g_err.c_str(); }

void nmmo_default_config(NmmoConfig* c) {
  memset(c, 0, sizeof(*c));
  c->abi_version = NMMO_ABI_VERSION;
  c->player_n = 128;
  c->npc_n = 256;
  c->horizon = 1024;
  c->map_n = 256;
  c->spawn_immunity = 20;
  c->early_stop_agent_num = 0;
  c->resilient_u32 = 858993459u;  // 0.2 * 2^32
  c->systems = NMMO_SYS_ALL;
  c->obs_layout = NMMO_OBS_FLAT;
  c->task_embed_dim = 2048;
  c->task_num_tick = 1024;
  c->event_cap = 4096;
  c->map_seed = 0;
  c->env_index_base = 0;
}

int nmmo_layout(const NmmoConfig* cfg, NmmoLayout* L) {
  if (!cfg || !L) return fail(NMMO_E_INVALID, "null argument");
  memset(L, 0, sizeof(*L));
  const int dims[NMMO_N_ACTION_HEADS] = {3, 101, 1025, 13, 13, 101, 99, 101, 5, 13, 99, 13};
  L->act_heads = NMMO_N_ACTION_HEADS;
  int o = 0;
  int* offs[NMMO_N_ACTION_HEADS] = {
      &L->off_mask_attack_style, &L->off_mask_attack_target, &L->off_mask_buy,
      &L->off_mask_destroy, &L->off_mask_give_item, &L->off_mask_give_target,
      &L->off_mask_givegold_price, &L->off_mask_givegold_target, &L->off_mask_move,
      &L->off_mask_sell_item, &L->off_mask_sell_price, &L->off_mask_use};
  for (int h = 0; h < NMMO_N_ACTION_HEADS; h++) {
    L->act_dims[h] = dims[h];
    *offs[h] = o;
    o += dims[h];
  }
  L->off_agent_id = o; o += 1;
  L->off_current_tick = o; o += 1;
  L->off_entity = o; o += 100 * NMMO_N_ENTITY_COLS;
  L->off_inventory = o; o += 12 * 16;
  L->off_market = o; o += 1024 * 16;
  L->off_task = o; o += cfg->task_embed_dim;
  L->off_tile = o; o += 225 * 3;
  L->obs_elems = o;
  L->entity_rows = 100; L->entity_cols = NMMO_N_ENTITY_COLS;
  L->inventory_rows = 12; L->item_cols = 16; L->market_rows = 1024;
  L->tile_rows = 225; L->tile_cols = 3;
  const int npc = (cfg->systems & NMMO_SYS_NPC) ? cfg->npc_n : 0;
  L->slots = cfg->player_n + npc;
  L->nf = NMMO_NF;
  L->ne = NMMO_NE;
  L->state_bytes_per_env = (size_t)NMMO_NE * 4 + (size_t)NMMO_NF * L->slots * 2 +
                           (size_t)L->slots * 2 + NMMO_MAP_TILES +
                           (size_t)cfg->player_n * NMMO_INV_SLOTS * 8 +
                           (size_t)NMMO_INV_SLOTS * cfg->player_n * 2 + (size_t)cfg->player_n * 4 +
                           (size_t)cfg->player_n * sizeof(NmmoTaskState);
  return NMMO_OK;
}

int32_t nmmo_n_envs(const NmmoHandle* h) { return h ? h->st.n_envs : 0; }

void nmmo_destroy(NmmoHandle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
  void* bufs[] = {h->d_env,  h->d_ent,   h->d_ring,  h->d_mat,   h->d_dep,   h->d_bank,
                  h->d_task, h->d_seeds, h->d_items, h->d_iring, h->d_mlist, h->d_mcount,
                  h->d_events, h->d_tasks, h->d_assign, h->d_tstate, h->d_ws, h->d_uniq, h->d_wenv, h->d_wdrop, h->d_task_cum,
                  h->d_wcount, h->d_wmcount, h->d_wrank, h->d_wpk, h->d_foreign, h->d_zrow, h->d_zext};  // d_zst lives in d_zrow's allocation
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  delete h;
}

int nmmo_create(const NmmoConfig* cfg, int32_t n_envs, uint64_t seed, int32_t device,
                const uint16_t* task_embedding, NmmoHandle** out) {
  if (!cfg || !out) return fail(NMMO_E_INVALID, "null argument");
  *out = nullptr;
  if (cfg->abi_version != NMMO_ABI_VERSION)
    return fail(NMMO_E_INVALID, "abi_version %d != %d", cfg->abi_version, NMMO_ABI_VERSION);
  if (n_envs <= 0) return fail(NMMO_E_INVALID, "n_envs must be > 0");
  if (cfg->player_n <= 0 || cfg->player_n > 128) return fail(NMMO_E_INVALID, "player_n in 1..128");
  if (cfg->npc_n < 0 || cfg->npc_n > 256) return fail(NMMO_E_INVALID, "npc_n in 0..256");
  if (cfg->map_n <= 0) return fail(NMMO_E_INVALID, "map_n must be > 0");
  if (cfg->horizon <= 0 || cfg->task_num_tick <= 0) return fail(NMMO_E_INVALID, "horizon/task_num_tick");
  if (cfg->task_embed_dim < 0 || cfg->task_embed_dim > 65536) return fail(NMMO_E_INVALID, "task_embed_dim");
  if (cfg->event_cap < 0 || cfg->event_cap > (1 << 24)) return fail(NMMO_E_INVALID, "event_cap in 0..2^24");
  if (cfg->obs_layout != NMMO_OBS_NONE && cfg->obs_layout != NMMO_OBS_FLAT && cfg->obs_layout != NMMO_OBS_NATIVE &&
      cfg->obs_layout != NMMO_OBS_WIRE)
    return fail(NMMO_E_INVALID, "obs_layout %d", cfg->obs_layout);
  NmmoHandle* h = new NmmoHandle();
  h->cfg = *cfg;
  h->device = device;
  nmmo_layout(cfg, &h->layout);
  const int P = cfg->player_n, N = (cfg->systems & NMMO_SYS_NPC) ? cfg->npc_n : 0, S = P + N;
  auto cleanup_fail = [&](int code) { nmmo_destroy(h); return code; };
  if (hipSetDevice(device) != hipSuccess) return cleanup_fail(fail(NMMO_E_HIP, "hipSetDevice(%d)", device));
  const size_t n = (size_t)n_envs;
#define ALLOC(ptr, bytes)                                                               \
  if (hipMalloc((void**)&(ptr), (bytes)) != hipSuccess)                                  \
    return cleanup_fail(fail(NMMO_E_NOMEM, "hipMalloc %zu bytes for %s", (size_t)(bytes), #ptr)); \
  if (hipMemset((ptr), 0, (bytes)) != hipSuccess) return cleanup_fail(fail(NMMO_E_HIP, "hipMemset"));
  ALLOC(h->d_env, n * NMMO_NE * 4);
  ALLOC(h->d_ent, n * NMMO_NF * S * 2);
  ALLOC(h->d_ring, n * S * 2);
  ALLOC(h->d_mat, n * NMMO_MAP_TILES);
  ALLOC(h->d_dep, n * kBitmapWords * 4);
  ALLOC(h->d_foreign, 8);  // [0] DevState::foreign, [1] DevState::fault
  ALLOC(h->d_bank, (size_t)cfg->map_n * NMMO_MAP_TILES);
  ALLOC(h->d_task, (size_t)(cfg->task_embed_dim > 0 ? cfg->task_embed_dim : 1) * 4);
  ALLOC(h->d_seeds, n * 8);
  ALLOC(h->d_items, n * P * NMMO_INV_SLOTS * 8);
  ALLOC(h->d_iring, n * NMMO_INV_SLOTS * P * 2);
  ALLOC(h->d_mlist, n * NMMO_MARKET_ROWS * 4);
  ALLOC(h->d_mcount, n * 4);
  if (cfg->event_cap > 0) ALLOC(h->d_events, n * (size_t)cfg->event_cap * NMMO_EVENT_COLS * 4);
  ALLOC(h->d_tasks, sizeof(NmmoTask));
  ALLOC(h->d_assign, n * P * 4);
  ALLOC(h->d_tstate, n * P * sizeof(NmmoTaskState));
  if (cfg->obs_layout == NMMO_OBS_NATIVE) {
    ALLOC(h->d_wcount, n * P * 2);
    ALLOC(h->d_wmcount, n * 4);
  }
  if (cfg->obs_layout == NMMO_OBS_FLAT || cfg->obs_layout == NMMO_OBS_NATIVE) {
    ALLOC(h->d_zrow, n * P * 16);  // (two statements)
  }
  if (cfg->obs_layout == NMMO_OBS_FLAT) {
    ALLOC(h->d_zext, n * P * kZext * 8);
  }
  {
    const char* rz = getenv("NMMO_OBS_REZERO");  // A/B: rewrite the zero rows every launch
    h->zskip = !(rz && rz[0] == '1');
    const char* wf = getenv("NMMO_WIRE_FUSE");  // A/B: the count kernel instead of the tick-fused count
    h->wire_fuse = !(wf && wf[0] == '0');
  }
  if (cfg->obs_layout == NMMO_OBS_WIRE) {
    ALLOC(h->d_wrank, n * (size_t)kMaxSlots * 2);
    ALLOC(h->d_wpk, n * (size_t)kMaxSlots * 4);
  }
#undef ALLOC
  if (init_kernels() != hipSuccess) return cleanup_fail(fail(NMMO_E_HIP, "kernel attributes"));
  if (task_embedding && cfg->task_embed_dim > 0) {
    std::vector<float> t(cfg->task_embed_dim);
    for (int k = 0; k < cfg->task_embed_dim; k++) t[k] = half_to_float(task_embedding[k]);
    if (hipMemcpy(h->d_task, t.data(), t.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
      return cleanup_fail(fail(NMMO_E_HIP, "task upload"));
  }
  h->st = DevState{h->d_env,   h->d_ent,   h->d_ring,  h->d_mat,    h->d_dep, h->d_bank,
                   h->d_items, h->d_iring, h->d_mlist, h->d_mcount, h->d_events,
                   h->d_tasks, h->d_assign, nullptr, h->d_tstate, 1,            0,           0, 0, n_envs, P,
                   N,          S,          seed,       nullptr,     *cfg,      h->d_foreign,
                   h->d_foreign + 1, nullptr, 0};
  {  // default task table: everyone runs TickGE(task_num_tick) (SPEC §12)
    NmmoTask t;
    memset(&t, 0, sizeof(t));
    t.term[0].pred = PRED_TICK_GE;
    t.term[0].a = cfg->task_num_tick;
    if (hipMemcpy(h->d_tasks, &t, sizeof(t), hipMemcpyHostToDevice) != hipSuccess)
      return cleanup_fail(fail(NMMO_E_HIP, "task table upload"));
  }
  if (launch_mapgen(cfg->map_seed, cfg->map_n, h->d_bank, nullptr) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess)
    return cleanup_fail(fail(NMMO_E_HIP, "map generation failed: %s", hipGetErrorString(hipGetLastError())));
  *out = h;
  return NMMO_OK;
}

static ObsParams obs_params(NmmoHandle* h, void* obs) {
  const NmmoLayout& L = h->layout;
  ObsParams p;
  const bool native = h->cfg.obs_layout == NMMO_OBS_NATIVE, wire = h->cfg.obs_layout == NMMO_OBS_WIRE;
  p.env = h->d_env; p.ent = h->d_ent; p.mat = h->d_mat; p.task = h->d_task;
  p.obs = native || wire ? nullptr : (float*)obs;
  p.nat = native ? (uint8_t*)obs : nullptr;
  p.wire = wire ? (uint8_t*)obs : nullptr;
  p.items = h->d_items; p.mlist = h->d_mlist; p.mcount = h->d_mcount; p.assign = h->d_assign;
  p.n_envs = h->st.n_envs; p.P = h->st.P; p.S = h->st.S; p.elems = L.obs_elems;
  p.task_dim = h->cfg.task_embed_dim; p.systems = h->cfg.systems;
  p.spawn_immunity = h->cfg.spawn_immunity;
  p.o_style = L.off_mask_attack_style; p.o_target = L.off_mask_attack_target;
  p.o_buy = L.off_mask_buy; p.o_destroy = L.off_mask_destroy;
  p.o_give_item = L.off_mask_give_item; p.o_give_target = L.off_mask_give_target;
  p.o_gg_price = L.off_mask_givegold_price; p.o_gg_target = L.off_mask_givegold_target;
  p.o_move = L.off_mask_move; p.o_sell_item = L.off_mask_sell_item;
  p.o_sell_price = L.off_mask_sell_price; p.o_use = L.off_mask_use;
  p.o_agent_id = L.off_agent_id; p.o_tick = L.off_current_tick; p.o_entity = L.off_entity;
  p.o_inventory = L.off_inventory; p.o_market = L.off_market; p.o_task = L.off_task;
  p.o_tile = L.off_tile;
  p.row_map = nullptr;
  p.env_list = nullptr;
  p.n_list = 0;
  p.wcount = native ? h->d_wcount : nullptr;
  p.wmcount = native ? h->d_wmcount : nullptr;
  p.wrank = wire ? h->d_wrank : nullptr;
  p.wpk = wire ? h->d_wpk : nullptr;
  p.fault = h->d_foreign + 1;
  // only the bound buffer (nmmo_obs_bind) is written incrementally
  p.zrow = h->d_zrow;
  p.zst = h->d_zrow ? h->d_zrow + (size_t)h->st.n_envs * h->st.P : nullptr;
  p.zext = h->d_zext;
  p.ztag = h->d_zrow && h->zskip && obs && obs == h->zbuf ? h->ztag : 0;
  p.rows_out = h->d_rows_out;
  p.counted = 0;
  p.recs = nullptr;  // (a step's outputs: step_impl sets them)
  p.fault_dst = nullptr;
  p.rew = nullptr;
  p.term = p.trunc = p.mask = nullptr;
  p.ws = h->wrap_on ? h->d_ws : nullptr;
  p.wflags = 0;
  if (h->wrap_on) {
    if (h->wc.kind == NMMO_WRAP_START_KIT) p.wflags |= kWrapObsPrice;
    if (h->wc.disable_give) p.wflags |= kWrapObsNoGive;
    if (h->wc.donot_attack_dangerous_npc) p.wflags |= kWrapObsNoDangerous;
  }
  return p;
}

static WrapParams wrap_params(NmmoHandle* h, const int32_t* actions, float* rew, const uint8_t* term,
                              const uint8_t* trunc, const uint8_t* mask) {
  WrapParams p;
  p.env = h->d_env; p.ent = h->d_ent; p.items = h->d_items; p.events = h->d_events;
  p.tstate = h->d_tstate; p.actions = actions; p.rew = rew; p.term = term; p.trunc = trunc;
  p.mask = mask; p.ws = h->d_ws; p.uniq = h->d_uniq; p.wenv = h->d_wenv; p.wdrop = h->d_wdrop; p.info = h->d_info;
  p.wc = h->wc; p.n_envs = h->st.n_envs; p.P = h->st.P; p.S = h->st.S; p.evcap = h->cfg.event_cap;
  p.items_on = (h->cfg.systems & NMMO_SYS_ITEM) != 0;
  p.env_list = nullptr;
  p.n_list = 0;
  return p;
}

int nmmo_reset(NmmoHandle* h, const uint64_t* env_seeds, void* obs, uint8_t* mask, void* stream) {
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipSetDevice(h->device));
  if (env_seeds) {
    HIP_TRY(hipMemcpyAsync(h->d_seeds, env_seeds, (size_t)h->st.n_envs * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));  // host seeds may go away after return
  }
  HIP_TRY(launch_tick(h->st, nullptr, env_seeds ? h->d_seeds : nullptr, nullptr, nullptr, nullptr,
                      mask, 1, s));
  HIP_TRY(hipMemsetAsync(h->d_foreign, 0, 4, s));  // every env's tiles now match its bank
  if (h->wrap_on) HIP_TRY(launch_wrap(wrap_params(h, nullptr, nullptr, nullptr, nullptr, nullptr), 0, s));
  const bool do_obs = obs && h->cfg.obs_layout != NMMO_OBS_NONE;
  if (do_obs) HIP_TRY(launch_obs(obs_params(h, obs), s));
  if (do_obs) h->last_native = obs;  // kept across a tick without obs: the pack check then says stale
  h->native_fresh = do_obs;
  return NMMO_OK;
}

__global__ void end_episodes_kernel(int32_t* env, const uint8_t* m, int n) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n && m[e]) env[(size_t)e * NMMO_NE + E_DONE] = 1;
}

int nmmo_end_episodes(NmmoHandle* h, const uint8_t* dev_env_mask, void* stream) {
  if (!h || !dev_env_mask) return fail(NMMO_E_INVALID, "null argument");
  const int n = h->st.n_envs;
  HIP_TRY(hipSetDevice(h->device));
  hipLaunchKernelGGL(end_episodes_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, h->d_env,
                     dev_env_mask, n);
  HIP_TRY(hipGetLastError());
  return NMMO_OK;
}

// nmmo_step over every env (env_ids = NULL) or over the listed envs (nmmo_step_envs)
static int step_impl(NmmoHandle* h, const int32_t* env_ids, int32_t n_ids, const int32_t* actions, void* obs,
                     float* rew, uint8_t* term, uint8_t* trunc, uint8_t* mask, void* stream) {
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  if (!actions || !rew || !term || !trunc || !mask)
    return fail(NMMO_E_INVALID, "actions/rew/term/trunc/mask must be device pointers");
  HIP_TRY(hipSetDevice(h->device));
  hipStream_t s = (hipStream_t)stream;
  const bool rec = h->timing && h->t_count < kTimingCap;
  hipEvent_t* ev = rec ? &h->ev[(size_t)h->t_count * 4] : nullptr;
  DevState st = h->st;
  st.env_list = env_ids;
  st.n_list = n_ids;
  const bool do_obs = obs && h->cfg.obs_layout != NMMO_OBS_NONE;
  // a whole-handle step into a wire buffer without the wrapper (which rewrites the rewards the
  // records carry after the tick): the C4 tick writes the count words itself (tick.hip
  // wire_count_fused, the 384-slot / 128-player specialisation launch_tick picks for these shapes)
  if (do_obs && h->cfg.obs_layout == NMMO_OBS_WIRE && !env_ids && !h->wrap_on && h->wire_fuse &&
      st.cfg.systems == NMMO_SYS_ALL && st.S == 384 && st.P == 128) {
    st.wf.wire = (uint8_t*)obs;
    st.wf.wrank = h->d_wrank;
    st.wf.wpk = h->d_wpk;
    st.wf.n_envs = st.n_envs;
    st.wf.spawn_immunity = h->cfg.spawn_immunity;
  }
  if (rec) HIP_TRY(hipEventRecord(ev[0], s));
  HIP_TRY(launch_tick(st, actions, nullptr, rew, term, trunc, mask, 0, s));
  if (rec) HIP_TRY(hipEventRecord(ev[1], s));
  if (h->wrap_on) {
    WrapParams wp = wrap_params(h, actions, rew, term, trunc, mask);
    wp.env_list = env_ids;
    wp.n_list = n_ids;
    HIP_TRY(launch_wrap(wp, 0, s));
  }
  if (rec) HIP_TRY(hipEventRecord(ev[2], s));  // wrapper span = ev[1]..ev[2] (empty when off)
  if (do_obs) {
    ObsParams op = obs_params(h, obs);
    op.env_list = env_ids;
    op.n_list = n_ids;
    op.counted = st.wf.wire != nullptr;
    if (op.wire && h->d_recs) {
      op.recs = h->d_recs;
      op.fault_dst = h->d_recs_fault;
      op.rew = rew;
      op.term = term;
      op.trunc = trunc;
      op.mask = mask;
    }
    HIP_TRY(launch_obs(op, s));
  }
  if (do_obs) h->last_native = obs;  // kept across a tick without obs: the pack check then says stale
  // a subset step leaves the other envs' native rows (and their wire counts) as they were, so the
  // buffer describes no single state: nmmo_wire_pack refuses it until a whole-handle gather
  h->native_fresh = do_obs && !env_ids;
  if (rec) {
    HIP_TRY(hipEventRecord(ev[3], s));  // obs span = ev[2]..ev[3] (empty when no obs)
    h->t_count++;
  }
  return NMMO_OK;
}

int nmmo_step(NmmoHandle* h, const int32_t* actions, void* obs, float* rew, uint8_t* term,
              uint8_t* trunc, uint8_t* mask, void* stream) {
  return step_impl(h, nullptr, 0, actions, obs, rew, term, trunc, mask, stream);
}

int nmmo_step_envs(NmmoHandle* h, const int32_t* env_ids, int32_t n_ids, const int32_t* actions, void* obs,
                   float* rew, uint8_t* term, uint8_t* trunc, uint8_t* mask, void* stream) {
  if (!h || !env_ids) return fail(NMMO_E_INVALID, "null handle / env_ids");
  if (n_ids < 0 || n_ids > h->st.n_envs) return fail(NMMO_E_INVALID, "n_ids %d not in 0..%d", n_ids, h->st.n_envs);
  if (h->cfg.obs_layout == NMMO_OBS_WIRE && obs)
    return fail(NMMO_E_INVALID, "nmmo_step_envs: the wire layout packs every env of the handle (use nmmo_step)");
  return step_impl(h, env_ids, n_ids, actions, obs, rew, term, trunc, mask, stream);
}

__global__ void fault_into_kernel(const int32_t* word, int32_t* dst) {
  const int32_t w = *word;
  if (w) atomicCAS(dst, 0, w);
}

int nmmo_fault_into(NmmoHandle* h, int32_t* dev_dst, void* stream) {
  if (!h || !dev_dst) return fail(NMMO_E_INVALID, "null argument");
  HIP_TRY(hipSetDevice(h->device));
  hipLaunchKernelGGL(fault_into_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, h->d_foreign + 1, dev_dst);
  HIP_TRY(hipGetLastError());
  return NMMO_OK;
}

int nmmo_inject_fault(NmmoHandle* h, int32_t fault) {
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(h->d_foreign + 1, &fault, 4, hipMemcpyHostToDevice));
  return NMMO_OK;
}

int nmmo_observe(NmmoHandle* h, void* obs, void* stream) {
  if (!h || !obs) return fail(NMMO_E_INVALID, "null argument");
  if (h->cfg.obs_layout == NMMO_OBS_NONE) return fail(NMMO_E_INVALID, "handle built with NMMO_OBS_NONE");
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(launch_obs(obs_params(h, obs), (hipStream_t)stream));
  h->last_native = obs;
  h->native_fresh = true;
  return NMMO_OK;
}

int nmmo_expand_obs(NmmoHandle* h, const void* native, float* flat, int32_t n_envs, void* stream) {
  if (!h || !native || !flat) return fail(NMMO_E_INVALID, "null argument");
  if (n_envs <= 0) return fail(NMMO_E_INVALID, "n_envs must be > 0");
  ObsParams p = obs_params(h, nullptr);
  p.nat = (uint8_t*)native;
  p.obs = flat;
  p.n_envs = n_envs;
  HIP_TRY(launch_expand(p, (hipStream_t)stream));
  return NMMO_OK;
}

// ---------------------------------------------------------------- observation buffers
// Large HBM buffers (the 12.6-GB flat obs of 1,024 envs) mapped from 64-MB physical chunks into
// one virtual range. Measured with the obs kernel's store pattern (tools/fill_patterns.hip, same
// box): hipMalloc'd buffers of this size wrote at 5.4-6.5 TB/s from one allocation to the next,
// chunk-mapped ones at 6.54-6.58 TB/s every time (any chunk size from 2 to 256 MB).
namespace {
struct VmmAlloc {
  size_t bytes;
  std::vector<hipMemGenericAllocationHandle_t> chunks;
};
std::mutex g_vmm_mu;
std::map<void*, VmmAlloc> g_vmm;
constexpr size_t kVmmChunk = (size_t)64 << 20;
}  // namespace

int nmmo_dev_alloc(int32_t device, uint64_t bytes, void** out) {
  if (!out || bytes == 0) return fail(NMMO_E_INVALID, "null out / zero bytes");
  *out = nullptr;
  HIP_TRY(hipSetDevice(device));
  int vmm = 0;
  HIP_TRY(hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, device));
  if (!vmm) return fail(NMMO_E_INVALID, "device %d has no virtual memory management (hipMemCreate / hipMemMap)", device);
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = device;
  size_t gran = 0;
  HIP_TRY(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
  const size_t chunk = gran > kVmmChunk ? gran : (kVmmChunk / gran) * gran;
  const size_t total = (bytes + chunk - 1) / chunk * chunk;
  void* va = nullptr;
  HIP_TRY(hipMemAddressReserve(&va, total, chunk, nullptr, 0));
  VmmAlloc a{total, {}};
  size_t mapped = 0;  // chunks mapped so far
  auto undo = [&]() {  // one unmap per mapped chunk, as they were mapped (and as nmmo_dev_free does)
    for (size_t i = 0; i < mapped; i++) (void)hipMemUnmap((char*)va + i * chunk, chunk);
    for (auto c : a.chunks) (void)hipMemRelease(c);
    (void)hipMemAddressFree(va, total);
  };
  for (size_t off = 0; off < total; off += chunk) {
    hipMemGenericAllocationHandle_t hdl;
    if (hipMemCreate(&hdl, chunk, &prop, 0) != hipSuccess) {
      undo();
      return fail(NMMO_E_NOMEM, "hipMemCreate of a %zu-byte chunk (%zu of %zu mapped)", chunk, off, total);
    }
    a.chunks.push_back(hdl);
    if (hipMemMap((char*)va + off, chunk, 0, hdl, 0) != hipSuccess) {
      undo();
      return fail(NMMO_E_HIP, "hipMemMap at offset %zu", off);
    }
    mapped++;
  }
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  if (hipMemSetAccess(va, total, &acc, 1) != hipSuccess) {
    undo();
    return fail(NMMO_E_HIP, "hipMemSetAccess");
  }
  std::lock_guard<std::mutex> lk(g_vmm_mu);
  g_vmm[va] = std::move(a);
  *out = va;
  return NMMO_OK;
}

int nmmo_dev_free(void* ptr) {
  if (!ptr) return NMMO_OK;
  VmmAlloc a;
  {
    std::lock_guard<std::mutex> lk(g_vmm_mu);
    auto it = g_vmm.find(ptr);
    if (it == g_vmm.end()) return fail(NMMO_E_INVALID, "pointer was not returned by nmmo_dev_alloc");
    a = std::move(it->second);
    g_vmm.erase(it);
  }
  HIP_TRY(hipDeviceSynchronize());  // no kernel may still use the range
  // Unmapped chunk by chunk as it was mapped and the physical chunks released; the virtual range
  // stays reserved for the life of the process (NMMO_DEVMEM_FREE_VA=1 frees it, for A/B). Cause,
  // isolated with no build code (tools/vmm_repro.hip, profiles/r05/vmm_repro.txt): after
  // hipMemAddressFree, hipMemAddressReserve hands the same range out again, and a later hipMalloc
  // (torch's caching allocator, here) can return addresses inside it too -- the two allocations
  // alias, so a buffer reads back what the other wrote (187 of 187 reused ranges with hipMalloc'd
  // temporaries alive, either unmap form; 0 of 192 with ranges kept reserved). A range never
  // reused cannot alias; the address space is 128 TB.
  const size_t chunk = a.chunks.empty() ? a.bytes : a.bytes / a.chunks.size();
  for (size_t i = 0; i < a.chunks.size(); i++) HIP_TRY(hipMemUnmap((char*)ptr + i * chunk, chunk));
  for (auto c : a.chunks) HIP_TRY(hipMemRelease(c));
  const char* fr = getenv("NMMO_DEVMEM_FREE_VA");
  if (fr && fr[0] == '1') HIP_TRY(hipMemAddressFree(ptr, a.bytes));
  return NMMO_OK;
}

int nmmo_set_step_records(NmmoHandle* h, uint8_t* dev_records, int32_t* dev_fault) {
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  if (dev_records && h->cfg.obs_layout != NMMO_OBS_WIRE)
    return fail(NMMO_E_INVALID, "nmmo_set_step_records: step records come with the wire obs layout");
  if (dev_fault && !dev_records) return fail(NMMO_E_INVALID, "nmmo_set_step_records: dev_fault without records");
  h->d_recs = dev_records;
  h->d_recs_fault = dev_fault;
  return NMMO_OK;
}

int nmmo_obs_bind(NmmoHandle* h, const void* obs) {
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  if (!h->d_zrow) return obs ? fail(NMMO_E_INVALID, "nmmo_obs_bind: flat or native obs layouts only") : NMMO_OK;
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipDeviceSynchronize());  // no gather of the previous binding is in flight
  HIP_TRY(hipMemset(h->d_zrow, 0, (size_t)h->st.n_envs * h->st.P * 8));
  h->zbuf = obs;
  h->ztag = obs ? h->ztag + 1 : h->ztag;  // never 0 for a bound buffer
  return NMMO_OK;
}

int nmmo_obs_invalidate(NmmoHandle* h, void* stream) {
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  if (!h->d_zrow) return NMMO_OK;
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipMemsetAsync(h->d_zrow, 0, (size_t)h->st.n_envs * h->st.P * 8, (hipStream_t)stream));  // the tags
  return NMMO_OK;
}

// the row-state tags of the listed envs' rows (zrow[e * P + a] = 0: nothing known about the row)
__global__ void obs_forget_envs_kernel(uint64_t* zrow, const int32_t* ids, int n_ids, int n_envs, int P) {
  const int i = blockIdx.x, e = ids[i];
  if ((unsigned)e >= (unsigned)n_envs) return;
  for (int a = threadIdx.x; a < P; a += blockDim.x) zrow[(size_t)e * P + a] = 0;
}

int nmmo_obs_invalidate_envs(NmmoHandle* h, const int32_t* env_ids, int32_t n_ids, void* stream) {
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  if (n_ids < 0 || n_ids > h->st.n_envs) return fail(NMMO_E_INVALID, "n_ids %d not in 0..%d", n_ids, h->st.n_envs);
  if (n_ids > 0 && !env_ids) return fail(NMMO_E_INVALID, "null env_ids");
  if (!h->d_zrow || n_ids == 0) return NMMO_OK;
  HIP_TRY(hipSetDevice(h->device));
  hipLaunchKernelGGL(obs_forget_envs_kernel, dim3(n_ids), dim3(128), 0, (hipStream_t)stream, h->d_zrow, env_ids,
                     n_ids, h->st.n_envs, h->st.P);
  HIP_TRY(hipGetLastError());
  return NMMO_OK;
}

// the Tile sections of the listed envs' rows (all envs when ids is NULL): kZsTile in their state
__global__ void obs_forget_tile_kernel(uint64_t* zst, const int32_t* ids, int n_envs, int P) {
  const int e = ids ? ids[blockIdx.x] : (int)blockIdx.x;
  if ((unsigned)e >= (unsigned)n_envs) return;
  for (int a = threadIdx.x; a < P; a += blockDim.x) zst[(size_t)e * P + a] |= kZsTile;
}

int nmmo_obs_invalidate_sections(NmmoHandle* h, const int32_t* env_ids, int32_t n_ids, uint32_t sections,
                                 void* stream) {
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  if (!env_ids) n_ids = h->st.n_envs;
  if (n_ids < 0 || n_ids > h->st.n_envs) return fail(NMMO_E_INVALID, "n_ids %d not in 0..%d", n_ids, h->st.n_envs);
  if (!h->d_zrow || n_ids == 0 || sections == 0) return NMMO_OK;
  HIP_TRY(hipSetDevice(h->device));
  // the Tile section alone is tracked per row by the flat rows of flat_obs.hip (slots a multiple of
  // 8); any other section, layout or kernel forgets the listed envs' whole rows
  const bool tile_only = sections == NMMO_OBS_SEC_TILE && h->cfg.obs_layout == NMMO_OBS_FLAT && h->st.S % 8 == 0;
  if (!tile_only) {
    if (!env_ids) {
      HIP_TRY(hipMemsetAsync(h->d_zrow, 0, (size_t)h->st.n_envs * h->st.P * 8, (hipStream_t)stream));
      return NMMO_OK;
    }
    return nmmo_obs_invalidate_envs(h, env_ids, n_ids, stream);
  }
  hipLaunchKernelGGL(obs_forget_tile_kernel, dim3(n_ids), dim3(128), 0, (hipStream_t)stream,
                     h->d_zrow + (size_t)h->st.n_envs * h->st.P, env_ids, h->st.n_envs, h->st.P);
  HIP_TRY(hipGetLastError());
  return NMMO_OK;
}

int nmmo_set_obs_counter(NmmoHandle* h, uint64_t* dev_rows) {
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  if (dev_rows) {  // the kernels add into it: it must be device memory of the handle's device
    HIP_TRY(hipSetDevice(h->device));
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, dev_rows) != hipSuccess || at.type != hipMemoryTypeDevice ||
        at.device != h->device) {
      (void)hipGetLastError();
      return fail(NMMO_E_INVALID, "nmmo_set_obs_counter: not device memory of device %d", h->device);
    }
  }
  h->d_rows_out = reinterpret_cast<unsigned long long*>(dev_rows);
  return NMMO_OK;
}

// ---------------------------------------------------------------- wire codec (SPEC §8c)
int64_t nmmo_wire_header_bytes(int32_t n_envs, int32_t player_n) {
  if (n_envs <= 0 || player_n <= 0 || player_n > 128) return fail(NMMO_E_INVALID, "n_envs > 0, player_n in 1..128");
  return wire_header_bytes(n_envs, player_n);
}

int64_t nmmo_wire_max_bytes(int32_t n_envs, int32_t player_n) {
  const int64_t hdr = nmmo_wire_header_bytes(n_envs, player_n);
  if (hdr < 0) return hdr;
  // every agent in the realm with full windows and inventories, a full entity table, every listing
  const int64_t rec = wire_record_bytes(wire_count_word(kNObs, kInv));
  return hdr + (int64_t)n_envs * (wire_table_bytes(kMaxSlots) + (int64_t)player_n * rec + NMMO_NATIVE_MARKET_BYTES);
}

int nmmo_wire_pack(NmmoHandle* h, const void* native, void* wire, void* stream) {
  if (!h || !native || !wire) return fail(NMMO_E_INVALID, "null argument");
  if (h->cfg.obs_layout != NMMO_OBS_NATIVE || !h->d_wcount)
    return fail(NMMO_E_INVALID, "nmmo_wire_pack needs a handle created with NMMO_OBS_NATIVE");
  if (native != h->last_native)
    return fail(NMMO_E_INVALID, "nmmo_wire_pack: `native` is not the buffer the handle's last obs gather wrote");
  if (!h->native_fresh)
    return fail(NMMO_E_INVALID, "nmmo_wire_pack: a tick ran after the last obs gather without one (stale native obs)");
  HIP_TRY(hipSetDevice(h->device));
  const int exch = (h->cfg.systems & NMMO_SYS_ITEM) && (h->cfg.systems & NMMO_SYS_EXCHANGE);
  HIP_TRY(launch_wire_pack(h->d_wcount, h->d_wmcount, (const uint8_t*)native, (uint8_t*)wire, h->st.n_envs, h->st.P,
                           h->d_ent, h->st.S, exch, (hipStream_t)stream));
  return NMMO_OK;
}

int nmmo_wire_check(const void* wire, int32_t n_envs, int32_t player_n, const int64_t* dev_expect_total,
                    int32_t* dev_status, void* stream) {
  if (!wire || !dev_status) return fail(NMMO_E_INVALID, "null argument");
  if (n_envs <= 0 || player_n <= 0 || player_n > 128) return fail(NMMO_E_INVALID, "n_envs > 0, player_n in 1..128");
  HIP_TRY(launch_wire_check((const uint8_t*)wire, n_envs, player_n, dev_expect_total, dev_status, (hipStream_t)stream));
  return NMMO_OK;
}

int nmmo_wire_check_many(const void* const* wires, const int32_t* n_envs, const int64_t* const* dev_expect_totals,
                         int32_t n_bufs, int32_t player_n, int32_t* dev_status, void* stream) {
  if (!wires || !n_envs || !dev_status) return fail(NMMO_E_INVALID, "null argument");
  if (n_bufs < 1 || n_bufs > kMaxCheckBufs) return fail(NMMO_E_INVALID, "n_bufs %d not in 1..%d", n_bufs, kMaxCheckBufs);
  if (player_n <= 0 || player_n > 128) return fail(NMMO_E_INVALID, "player_n in 1..128");
  WireCheckBatch b;
  memset(&b, 0, sizeof(b));
  b.count = n_bufs;
  for (int i = 0; i < n_bufs; i++) {
    if (!wires[i] || n_envs[i] <= 0) return fail(NMMO_E_INVALID, "buffer %d: null wire / n_envs <= 0", i);
    b.wire[i] = (const uint8_t*)wires[i];
    b.n[i] = n_envs[i];
    b.expect[i] = dev_expect_totals ? dev_expect_totals[i] : nullptr;
  }
  HIP_TRY(launch_wire_check_many(b, player_n, dev_status, (hipStream_t)stream));
  return NMMO_OK;
}

// the learner gather's sizes row of one step (nmmo_sizes_row): one launch instead of a copy per
// buffer, a copy and a zero for the fault word
struct SizesRowArgs {
  const int64_t* w[kMaxCheckBufs];
  int n;
};
__global__ void sizes_row_kernel(SizesRowArgs a, int32_t* fault, int64_t* row) {
  const int j = threadIdx.x;
  if (j < a.n) row[j] = *a.w[j];
  if (j == a.n) {
    row[j] = fault ? *fault : 0;
    if (fault) *fault = 0;
  }
}

int nmmo_sizes_row(const void* const* wires, int32_t n_bufs, int32_t* dev_fault, int64_t* dev_row, void* stream) {
  if (!wires || !dev_row) return fail(NMMO_E_INVALID, "null argument");
  if (n_bufs < 1 || n_bufs > kMaxCheckBufs) return fail(NMMO_E_INVALID, "n_bufs %d not in 1..%d", n_bufs, kMaxCheckBufs);
  SizesRowArgs a;
  memset(&a, 0, sizeof(a));
  a.n = n_bufs;
  for (int j = 0; j < n_bufs; j++) {
    if (!wires[j] || ((uintptr_t)wires[j] & 7)) return fail(NMMO_E_INVALID, "buffer %d: null / not 8-B aligned", j);
    a.w[j] = (const int64_t*)wires[j];
  }
  hipLaunchKernelGGL(sizes_row_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a, dev_fault, dev_row);
  HIP_TRY(hipGetLastError());
  return NMMO_OK;
}

// ---------------------------------------------------------------- gather point-to-point (p2p.hip)
int nmmo_p2p_load(const char* librccl_path) {
  char err[512];
  if (p2p_load(librccl_path, err, sizeof(err))) return fail(NMMO_E_INVALID, "%s", err);
  return NMMO_OK;
}
int nmmo_p2p_unique_id(void* id) {
  char err[512];
  if (!id) return fail(NMMO_E_INVALID, "null id");
  if (p2p_load(nullptr, err, sizeof(err))) return fail(NMMO_E_INVALID, "nmmo_p2p_load first");
  if (p2p_unique_id(id, err, sizeof(err))) return fail(NMMO_E_HIP, "%s", err);
  return NMMO_OK;
}
int nmmo_p2p_init(const void* id, int32_t world, int32_t rank, void** comm) {
  char err[512];
  if (!id || !comm) return fail(NMMO_E_INVALID, "null argument");
  if (world < 1 || rank < 0 || rank >= world) return fail(NMMO_E_INVALID, "rank %d of %d", rank, world);
  if (p2p_load(nullptr, err, sizeof(err))) return fail(NMMO_E_INVALID, "nmmo_p2p_load first");
  if (p2p_init(id, world, rank, comm, err, sizeof(err))) return fail(NMMO_E_HIP, "%s", err);
  return NMMO_OK;
}
int nmmo_p2p_group(void* comm, const NmmoP2POp* ops, int32_t n_ops, void* stream) {
  char err[512];
  if (!comm || (n_ops > 0 && !ops) || n_ops < 0) return fail(NMMO_E_INVALID, "null communicator / ops");
  for (int i = 0; i < n_ops; i++)
    if (!ops[i].buf || ops[i].bytes < 0 || ops[i].peer < 0) return fail(NMMO_E_INVALID, "op %d: buffer / size / peer", i);
  if (n_ops == 0) return NMMO_OK;
  if (p2p_group(comm, ops, n_ops, (hipStream_t)stream, err, sizeof(err))) return fail(NMMO_E_HIP, "%s", err);
  return NMMO_OK;
}
int nmmo_p2p_destroy(void* comm) { return p2p_destroy(comm) ? fail(NMMO_E_HIP, "ncclCommDestroy") : NMMO_OK; }

int nmmo_wire_unpack(int32_t n_envs, int32_t player_n, const void* wire, void* native, void* stream) {
  if (!wire || !native) return fail(NMMO_E_INVALID, "null argument");
  if (n_envs <= 0 || player_n <= 0 || player_n > 128) return fail(NMMO_E_INVALID, "n_envs > 0, player_n in 1..128");
  HIP_TRY(launch_wire_unpack((const uint8_t*)wire, (uint8_t*)native, n_envs, player_n, (hipStream_t)stream));
  return NMMO_OK;
}

// ---------------------------------------------------------------- experience storage (§8f row 3)
int64_t nmmo_exp_scratch_ints(int32_t max_rows, int32_t n_slots) {
  const int64_t a = (int64_t)max_rows + store_blocks(max_rows) + 8;
  return a > n_slots ? a : (int64_t)n_slots;
}

int64_t nmmo_exp_scratch_ints_many(int32_t n_inputs, int32_t max_rows, int32_t n_slots) {
  if (n_inputs < 1 || n_inputs > kMaxStoreInputs || max_rows < 0)
    return fail(NMMO_E_INVALID, "n_inputs %d not in 1..%d / max_rows < 0", n_inputs, kMaxStoreInputs);
  const int64_t a = nmmo_exp_scratch_ints((int32_t)std::min<int64_t>((int64_t)n_inputs * max_rows, INT32_MAX), n_slots);
  const int64_t b = store_many_scratch_ints(n_inputs, max_rows);
  return a > b ? a : b;
}

static int check_exp(const NmmoExperience* x, bool need_obs = true) {
  if (!x) return fail(NMMO_E_INVALID, "null experience");
  if (x->capacity <= 0 || x->obs_elems <= 0 || x->n_slots <= 0)
    return fail(NMMO_E_INVALID, "capacity/obs_elems/n_slots must be > 0");
  if ((need_obs && !x->obs) || !x->actions || !x->logprobs || !x->rewards || !x->dones || !x->values || !x->env_id ||
      !x->step || !x->seq || !x->slot_count || !x->ptr)
    return fail(NMMO_E_INVALID, "experience buffers must be device pointers");
  return NMMO_OK;
}

static int check_records(const NmmoRecordStore* rs) {
  if (!rs || !rs->arena || !rs->arena_used || !rs->row_buf || !rs->row_agent)
    return fail(NMMO_E_INVALID, "record store buffers must be device pointers");
  if (rs->arena_bytes <= 0 || ((uintptr_t)rs->arena & 15)) return fail(NMMO_E_INVALID, "arena must be 16-B aligned, > 0 bytes");
  return NMMO_OK;
}

int nmmo_exp_store_records(NmmoHandle* h, const NmmoExperience* x, const NmmoRecordStore* rs, const NmmoStoreInput* in,
                           int32_t* scratch, void* stream) {
  if (int rc = check_exp(x, false)) return rc;
  if (int rc = check_records(rs)) return rc;
  if (!h || !in || !scratch) return fail(NMMO_E_INVALID, "null handle/input/scratch");
  if (!in->wire || in->obs || in->native) return fail(NMMO_E_INVALID, "record storage takes a wire input only");
  if (in->n_rows <= 0 || in->n_rows % h->st.P) return fail(NMMO_E_SIZE, "n_rows must be whole envs of player_n rows");
  if (!in->rewards || !in->dones || !in->mask || !in->actions || !in->logprobs || !in->values)
    return fail(NMMO_E_INVALID, "store inputs must be device pointers");
  if (!in->env_id && (in->env_id_base < 0 || (int64_t)in->env_id_base + in->n_rows > x->n_slots))
    return fail(NMMO_E_INVALID, "env_id_base + n_rows exceeds n_slots");
  if (((uintptr_t)in->wire & 15)) return fail(NMMO_E_INVALID, "wire buffer must be 16-B aligned");
  HIP_TRY(hipSetDevice(h->device));
  const int64_t cap = nmmo_wire_max_bytes(in->n_rows / h->st.P, h->st.P);
  HIP_TRY(launch_store_records(*x, *rs, *in, h->st.P, cap, scratch, (hipStream_t)stream));
  return NMMO_OK;
}

static int store_records_many(NmmoHandle* h, const NmmoExperience* x, const NmmoRecordStore* rs, const NmmoStoreInput* ins,
                              int32_t n_inputs, int32_t field_stride, int32_t* scratch, void* stream,
                              const StoreCheck* chk) {
  if (int rc = check_exp(x, false)) return rc;
  if (int rc = check_records(rs)) return rc;
  if (!h || !ins || !scratch) return fail(NMMO_E_INVALID, "null handle/inputs/scratch");
  if (n_inputs < 1 || n_inputs > kMaxStoreInputs) return fail(NMMO_E_INVALID, "n_inputs %d not in 1..%d", n_inputs, kMaxStoreInputs);
  if (field_stride < 0) return fail(NMMO_E_INVALID, "field_stride < 0");
  StoreBatch b;
  memset(&b, 0, sizeof(b));
  b.n = n_inputs;
  b.P = h->st.P;
  b.stride = field_stride;
  for (int i = 0; i < n_inputs; i++) {
    const NmmoStoreInput& in = ins[i];
    if (!in.wire || in.obs || in.native) return fail(NMMO_E_INVALID, "input %d: record storage takes a wire input only", i);
    if (in.n_rows <= 0 || in.n_rows % h->st.P) return fail(NMMO_E_SIZE, "input %d: n_rows must be whole envs", i);
    if (!in.rewards || !in.dones || !in.mask || !in.actions || !in.logprobs || !in.values)
      return fail(NMMO_E_INVALID, "input %d: store inputs must be device pointers", i);
    if (!in.env_id && (in.env_id_base < 0 || (int64_t)in.env_id_base + in.n_rows > x->n_slots))
      return fail(NMMO_E_INVALID, "input %d: env_id_base + n_rows exceeds n_slots", i);
    if (((uintptr_t)in.wire & 15)) return fail(NMMO_E_INVALID, "input %d: wire buffer must be 16-B aligned", i);
    b.in[i] = in;
    b.wire_cap[i] = nmmo_wire_max_bytes(in.n_rows / h->st.P, h->st.P);
  }
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(launch_store_records_many(*x, *rs, b, scratch, (hipStream_t)stream, chk));
  return NMMO_OK;
}

int nmmo_exp_store_records_many(NmmoHandle* h, const NmmoExperience* x, const NmmoRecordStore* rs,
                                const NmmoStoreInput* ins, int32_t n_inputs, int32_t field_stride, int32_t* scratch,
                                void* stream) {
  return store_records_many(h, x, rs, ins, n_inputs, field_stride, scratch, stream, nullptr);
}

int nmmo_exp_store_records_checked(NmmoHandle* h, const NmmoExperience* x, const NmmoRecordStore* rs,
                                   const NmmoStoreInput* ins, int32_t n_inputs, int32_t field_stride,
                                   const int64_t* const* dev_expect_totals, uint32_t check_mask,
                                   int32_t* dev_check_status, int32_t* dev_ctl, int32_t* scratch, void* stream) {
  if (!dev_ctl) return fail(NMMO_E_INVALID, "dev_ctl must be a device int32 [%d]", NMMO_STORE_CTL_INTS);
  StoreCheck chk;
  memset(&chk, 0, sizeof(chk));
  for (int i = 0; i < n_inputs && i < kMaxStoreInputs; i++) chk.expect[i] = dev_expect_totals ? dev_expect_totals[i] : nullptr;
  chk.status = dev_check_status;
  chk.ctl = dev_ctl;
  chk.mask = check_mask;
  return store_records_many(h, x, rs, ins, n_inputs, field_stride, scratch, stream, &chk);
}

int nmmo_exp_gather_records(NmmoHandle* h, const NmmoExperience* x, const NmmoRecordStore* rs, const int32_t* idx,
                            int32_t n, float* out, void* stream) {
  if (int rc = check_exp(x, false)) return rc;
  if (int rc = check_records(rs)) return rc;
  if (!h || !idx || !out) return fail(NMMO_E_INVALID, "null handle/idx/out");
  if (n < 0) return fail(NMMO_E_INVALID, "n must be >= 0");
  if (x->obs_elems != h->layout.obs_elems) return fail(NMMO_E_SIZE, "obs_elems != the handle's layout");
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(launch_record_gather(obs_params(h, nullptr), *rs, idx, n, out, (hipStream_t)stream));
  return NMMO_OK;
}

int nmmo_exp_store(NmmoHandle* h, const NmmoExperience* x, const NmmoStoreInput* in, int32_t* scratch,
                   void* stream) {
  if (int rc = check_exp(x)) return rc;
  if (!in || !scratch) return fail(NMMO_E_INVALID, "null input/scratch");
  if (in->n_rows <= 0) return fail(NMMO_E_INVALID, "n_rows must be > 0");
  if (!in->rewards || !in->dones || !in->mask || !in->actions || !in->logprobs || !in->values)
    return fail(NMMO_E_INVALID, "store inputs must be device pointers");
  if (!in->env_id && (in->env_id_base < 0 || (int64_t)in->env_id_base + in->n_rows > x->n_slots))
    return fail(NMMO_E_INVALID, "env_id_base + n_rows exceeds n_slots");
  if ((in->obs != nullptr) + (in->native != nullptr) + (in->wire != nullptr) != 1)
    return fail(NMMO_E_INVALID, "exactly one of obs / native / wire");
  if (in->native || in->wire) {
    if (!h) return fail(NMMO_E_INVALID, "native / wire obs need a handle with their layout and task table");
    if (in->native && h->cfg.obs_layout != NMMO_OBS_NATIVE) return fail(NMMO_E_INVALID, "handle is not NMMO_OBS_NATIVE");
    if (in->n_rows % h->st.P) return fail(NMMO_E_SIZE, "n_rows must be whole envs of player_n rows");
    if (x->obs_elems != h->layout.obs_elems) return fail(NMMO_E_SIZE, "obs_elems != the handle's layout");
    HIP_TRY(hipSetDevice(h->device));
    ObsParams p = obs_params(h, nullptr);
    p.nat = (uint8_t*)in->native;
    p.wire = (uint8_t*)in->wire;
    p.n_envs = in->n_rows / h->st.P;
    HIP_TRY(launch_store(*x, *in, &p, scratch, (hipStream_t)stream));
  } else {
    HIP_TRY(launch_store(*x, *in, nullptr, scratch, (hipStream_t)stream));
  }
  return NMMO_OK;
}

int nmmo_exp_sort(const NmmoExperience* x, int32_t* idxs, int32_t* scratch, void* stream) {
  if (int rc = check_exp(x)) return rc;
  if (!idxs || !scratch) return fail(NMMO_E_INVALID, "null idxs/scratch");
  HIP_TRY(launch_sort(*x, idxs, scratch, (hipStream_t)stream));
  return NMMO_OK;
}

int nmmo_exp_gae(const NmmoExperience* x, const int32_t* idxs, int32_t batch_size, double gamma, double gae_lambda,
                 float* advantages, void* stream) {
  if (int rc = check_exp(x)) return rc;
  if (!idxs || !advantages) return fail(NMMO_E_INVALID, "null idxs/advantages");
  if (batch_size <= 0 || batch_size >= x->capacity)
    return fail(NMMO_E_SIZE, "batch_size must be in [1, capacity - 1]");
  // the reference multiplies float32 tensors by the Python floats gamma and gamma*gae_lambda
  // (a double product), each cast to float32 by the op (clean_pufferl.py:431-435)
  HIP_TRY(launch_gae(*x, idxs, batch_size, (float)gamma, (float)(gamma * gae_lambda), advantages,
                     (hipStream_t)stream));
  return NMMO_OK;
}

int nmmo_gather_rows(const void* src, int64_t row_bytes, const int32_t* idx, int32_t n, void* out, void* stream) {
  if (!src || !idx || !out) return fail(NMMO_E_INVALID, "null argument");
  if (row_bytes <= 0 || row_bytes % 4) return fail(NMMO_E_INVALID, "row_bytes must be a positive multiple of 4");
  if (n < 0) return fail(NMMO_E_INVALID, "n must be >= 0");
  if (n) HIP_TRY(launch_gather_rows(src, row_bytes / 4, idx, n, out, (hipStream_t)stream));
  return NMMO_OK;
}

int nmmo_set_timing(NmmoHandle* h, int32_t enable) {
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  HIP_TRY(hipSetDevice(h->device));
  if (enable && h->ev.empty()) {
    h->ev.resize((size_t)kTimingCap * 4);
    for (auto& e : h->ev) HIP_TRY(hipEventCreate(&e));
  }
  h->timing = enable != 0;
  h->t_count = 0;
  return NMMO_OK;
}

int nmmo_get_fault(NmmoHandle* h, int32_t* fault) {
  if (!h || !fault) return fail(NMMO_E_INVALID, "null argument");
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipMemcpy(fault, h->d_foreign + 1, 4, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemset(h->d_foreign + 1, 0, 4));
  return NMMO_OK;
}

int nmmo_set_counters(NmmoHandle* h, uint64_t* dev_counters) {
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  h->st.counters = reinterpret_cast<unsigned long long*>(dev_counters);
  return NMMO_OK;
}

int nmmo_read_timing(NmmoHandle* h, double* ms, int32_t* n) {
  if (!h || !ms || !n) return fail(NMMO_E_INVALID, "null argument");
  ms[0] = ms[1] = ms[2] = 0.0;
  *n = h->t_count;
  for (int i = 0; i < h->t_count; i++) {
    hipEvent_t* ev = &h->ev[(size_t)i * 4];
    float a = 0.f, b = 0.f, c = 0.f;
    HIP_TRY(hipEventSynchronize(ev[3]));
    HIP_TRY(hipEventElapsedTime(&a, ev[0], ev[1]));
    HIP_TRY(hipEventElapsedTime(&b, ev[2], ev[3]));
    HIP_TRY(hipEventElapsedTime(&c, ev[1], ev[2]));
    ms[0] += a;
    ms[1] += b;
    ms[2] += c;
  }
  h->t_count = 0;
  return NMMO_OK;
}

int nmmo_scripted_actions(NmmoHandle* h, uint64_t policy_seed, int32_t* actions, void* stream) {
  if (!h || !actions) return fail(NMMO_E_INVALID, "null argument");
  PolicyParams p;
  p.env = h->d_env; p.ent = h->d_ent; p.mat = h->d_mat; p.actions = actions;
  p.items = h->d_items; p.mlist = h->d_mlist; p.mcount = h->d_mcount;
  p.n_envs = h->st.n_envs; p.P = h->st.P; p.S = h->st.S; p.systems = h->cfg.systems;
  p.spawn_immunity = h->cfg.spawn_immunity; p.seed = policy_seed;
  HIP_TRY(launch_policy(p, (hipStream_t)stream));
  return NMMO_OK;
}

int nmmo_get_state(NmmoHandle* h, void* host_buf, size_t nbytes) {
  if (!h || !host_buf) return fail(NMMO_E_INVALID, "null argument");
  const size_t n = (size_t)h->st.n_envs, S = (size_t)h->st.S;
  const size_t per = h->layout.state_bytes_per_env;
  if (nbytes != per * n) return fail(NMMO_E_SIZE, "state buffer %zu != %zu", nbytes, per * n);
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipDeviceSynchronize());
  std::vector<int32_t> env(n * NMMO_NE);
  std::vector<int16_t> ent(n * NMMO_NF * S), ring(n * S);
  std::vector<uint8_t> mat(n * NMMO_MAP_TILES);
  const size_t IP = (size_t)NMMO_INV_SLOTS * h->st.P;  // items per env
  std::vector<uint32_t> items(n * IP * 2);
  std::vector<int16_t> iring(n * IP);
  const size_t P = (size_t)h->st.P;
  std::vector<int32_t> assign(n * P);
  std::vector<NmmoTaskState> tstate(n * P);
  HIP_TRY(hipMemcpy(items.data(), h->d_items, items.size() * 4, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(iring.data(), h->d_iring, iring.size() * 2, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(assign.data(), h->d_assign, assign.size() * 4, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(tstate.data(), h->d_tstate, tstate.size() * sizeof(NmmoTaskState), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(env.data(), h->d_env, env.size() * 4, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(ent.data(), h->d_ent, ent.size() * 2, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(ring.data(), h->d_ring, ring.size() * 2, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(mat.data(), h->d_mat, mat.size(), hipMemcpyDeviceToHost));
  uint8_t* b = (uint8_t*)host_buf;
  for (size_t e = 0; e < n; e++) {
    memcpy(b, env.data() + e * NMMO_NE, NMMO_NE * 4); b += NMMO_NE * 4;
    memcpy(b, ent.data() + e * NMMO_NF * S, NMMO_NF * S * 2); b += NMMO_NF * S * 2;
    memcpy(b, ring.data() + e * S, S * 2); b += S * 2;
    memcpy(b, mat.data() + e * NMMO_MAP_TILES, NMMO_MAP_TILES); b += NMMO_MAP_TILES;
    memcpy(b, items.data() + e * IP * 2, IP * 8); b += IP * 8;
    memcpy(b, iring.data() + e * IP, IP * 2); b += IP * 2;
    memcpy(b, assign.data() + e * P, P * 4); b += P * 4;
    memcpy(b, tstate.data() + e * P, P * sizeof(NmmoTaskState)); b += P * sizeof(NmmoTaskState);
  }
  return NMMO_OK;
}

int nmmo_set_state(NmmoHandle* h, const void* host_buf, size_t nbytes) {
  if (!h || !host_buf) return fail(NMMO_E_INVALID, "null argument");
  const size_t n = (size_t)h->st.n_envs, S = (size_t)h->st.S;
  const size_t per = h->layout.state_bytes_per_env;
  if (nbytes != per * n) return fail(NMMO_E_SIZE, "state buffer %zu != %zu", nbytes, per * n);
  std::vector<int32_t> env(n * NMMO_NE);
  std::vector<int16_t> ent(n * NMMO_NF * S), ring(n * S);
  std::vector<uint8_t> mat(n * NMMO_MAP_TILES);
  const size_t IP = (size_t)NMMO_INV_SLOTS * h->st.P;
  std::vector<uint32_t> items(n * IP * 2);
  std::vector<int16_t> iring(n * IP);
  const size_t P = (size_t)h->st.P;
  std::vector<int32_t> assign(n * P);
  std::vector<NmmoTaskState> tstate(n * P);
  const uint8_t* b = (const uint8_t*)host_buf;
  for (size_t e = 0; e < n; e++) {
    memcpy(env.data() + e * NMMO_NE, b, NMMO_NE * 4); b += NMMO_NE * 4;
    memcpy(ent.data() + e * NMMO_NF * S, b, NMMO_NF * S * 2); b += NMMO_NF * S * 2;
    memcpy(ring.data() + e * S, b, S * 2); b += S * 2;
    memcpy(mat.data() + e * NMMO_MAP_TILES, b, NMMO_MAP_TILES); b += NMMO_MAP_TILES;
    memcpy(items.data() + e * IP * 2, b, IP * 8); b += IP * 8;
    memcpy(iring.data() + e * IP, b, IP * 2); b += IP * 2;
    memcpy(assign.data() + e * P, b, P * 4); b += P * 4;
    memcpy(tstate.data() + e * P, b, P * sizeof(NmmoTaskState)); b += P * sizeof(NmmoTaskState);
  }
  for (int32_t a : assign)
    if (a < 0 || a >= h->st.n_tasks) return fail(NMMO_E_INVALID, "state blob: task index %d outside the task table", a);
  if (slim_systems(h->st.cfg.systems)) {  // the tick keeps these fields in HBM as reset wrote them
    for (size_t e = 0; e < n; e++)
      for (int f = 0; f < NMMO_NF_USED; f++)
        for (size_t sl = 0; !slim_staged(f) && sl < S; sl++)
          if (ent[(e * NMMO_NF + f) * S + sl] != slim_const(f, sl < P))
            return fail(NMMO_E_INVALID,
                        "state blob: env %zu slot %zu field %d = %d, but without the Item/Equipment/Profession/"
                        "Exchange systems it must hold its reset value %d", e, sl, f,
                        (int)ent[(e * NMMO_NF + f) * S + sl], slim_const(f, sl < P));
  }
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(h->d_env, env.data(), env.size() * 4, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(h->d_ent, ent.data(), ent.size() * 2, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(h->d_ring, ring.data(), ring.size() * 2, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(h->d_mat, mat.data(), mat.size(), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(h->d_items, items.data(), items.size() * 4, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(h->d_iring, iring.data(), iring.size() * 2, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(h->d_assign, assign.data(), assign.size() * 4, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(h->d_tstate, tstate.data(), tstate.size() * sizeof(NmmoTaskState), hipMemcpyHostToDevice));
  HIP_TRY(launch_rebuild_dep(h->st, nullptr));
  HIP_TRY(hipDeviceSynchronize());
  h->native_fresh = false;  // the last native obs no longer describes the state (nmmo_wire_pack)
  return NMMO_OK;
}

int nmmo_set_tasks(NmmoHandle* h, const NmmoTask* tasks, int32_t n_tasks, const uint16_t* embeddings,
                   const int32_t* assign) {
  if (!h || !tasks) return fail(NMMO_E_INVALID, "null argument");
  if (n_tasks < 1 || n_tasks > NMMO_MAX_TASKS) return fail(NMMO_E_INVALID, "n_tasks %d not in 1..%d", n_tasks, NMMO_MAX_TASKS);
  int tev = 0, tmap = 0, tsee = 0;
  for (int i = 0; i < n_tasks; i++)
    for (int k = 0; k < 2; k++) {
      const int pr = tasks[i].term[k].pred;
      if (pr < 0 || pr >= NMMO_N_PREDICATES) return fail(NMMO_E_INVALID, "task %d term %d: predicate %d", i, k, pr);
      const int64_t ta = tasks[i].term[k].a;  // the tick's 8-B descriptor holds a in 24 bits
      if (ta < -(1 << 23) || ta >= (1 << 23)) return fail(NMMO_E_INVALID, "task %d term %d: a %lld outside +/-2^23", i, k, (long long)ta);
      tev |= (pr >= PRED_COUNT_EVENT && pr <= PRED_DEFEAT_ENTITY) || pr == PRED_PRACTICE_EATING;
      tmap |= pr == PRED_CAN_SEE_TILE;
      tsee |= pr == PRED_CAN_SEE_AGENT || pr == PRED_CAN_SEE_GROUP;
    }
  const size_t nP = (size_t)h->st.n_envs * h->st.P;
  if (assign)
    for (size_t i = 0; i < nP; i++)
      if (assign[i] < 0 || assign[i] >= n_tasks) return fail(NMMO_E_INVALID, "assign[%zu] = %d", i, assign[i]);
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipDeviceSynchronize());
  const int D = h->cfg.task_embed_dim > 0 ? h->cfg.task_embed_dim : 1;
  std::vector<float> emb((size_t)n_tasks * D);
  std::vector<float> first(D);
  HIP_TRY(hipMemcpy(first.data(), h->d_task, (size_t)D * 4, hipMemcpyDeviceToHost));
  for (int i = 0; i < n_tasks; i++)
    for (int k = 0; k < D; k++)
      emb[(size_t)i * D + k] = embeddings && h->cfg.task_embed_dim > 0 ? half_to_float(embeddings[(size_t)i * D + k])
                                                                       : first[k];
  float* d_task = nullptr;
  NmmoTask* d_tasks = nullptr;
  if (hipMalloc((void**)&d_task, emb.size() * 4) != hipSuccess ||
      hipMalloc((void**)&d_tasks, (size_t)n_tasks * sizeof(NmmoTask)) != hipSuccess) {
    if (d_task) (void)hipFree(d_task);
    return fail(NMMO_E_NOMEM, "task table allocation");
  }
  HIP_TRY(hipMemcpy(d_task, emb.data(), emb.size() * 4, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(d_tasks, tasks, (size_t)n_tasks * sizeof(NmmoTask), hipMemcpyHostToDevice));
  if (assign) HIP_TRY(hipMemcpy(h->d_assign, assign, nP * 4, hipMemcpyHostToDevice));
  else HIP_TRY(hipMemset(h->d_assign, 0, nP * 4));
  (void)hipFree(h->d_task);
  (void)hipFree(h->d_tasks);
  h->d_task = d_task;
  h->d_tasks = d_tasks;
  h->st.tasks = d_tasks;
  h->st.n_tasks = n_tasks;
  h->st.tev = tev;
  h->st.tmap = tmap;
  h->st.tsee = tsee;
  h->st.task_cum = nullptr;  // weights belong to the previous table
  h->native_fresh = false;   // task indices of the last native obs may be out of date
  // flat rows keep a task's embedding by index (ObsParams::zst): the new table may differ
  if (h->d_zrow) HIP_TRY(hipMemset(h->d_zrow, 0, (size_t)h->st.n_envs * h->st.P * 8));
  return NMMO_OK;
}

// SPEC §12 sampling thresholds: cum[i] = floor(2^32 * (w_0 + .. + w_i) / sum(w)), summed in
// order in double; the last is exactly 2^32 so every draw u < 2^32 selects a task.
static void task_thresholds(const double* w, int n, uint64_t* cum) {
  double sum = 0.0;
  for (int i = 0; i < n; i++) sum += w[i];
  double acc = 0.0;
  for (int i = 0; i < n; i++) {
    acc += w[i];
    const double f = floor(acc / sum * 4294967296.0);
    cum[i] = f >= 4294967296.0 ? (1ull << 32) : (uint64_t)f;
  }
  cum[n - 1] = 1ull << 32;
}

int nmmo_set_task_weights(NmmoHandle* h, const double* weights, int32_t n_tasks) {
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipDeviceSynchronize());
  if (!weights) {
    h->st.task_cum = nullptr;
    return NMMO_OK;
  }
  if (n_tasks != h->st.n_tasks) return fail(NMMO_E_SIZE, "n_tasks %d != the task table's %d", n_tasks, h->st.n_tasks);
  double sum = 0.0;
  for (int i = 0; i < n_tasks; i++) {
    if (!(weights[i] >= 0.0) || weights[i] > 1e300) return fail(NMMO_E_INVALID, "weight %d = %g", i, weights[i]);
    sum += weights[i];
  }
  if (!(sum > 0.0)) return fail(NMMO_E_INVALID, "weights must have a positive sum");
  std::vector<uint64_t> cum((size_t)n_tasks);
  task_thresholds(weights, n_tasks, cum.data());
  if (!h->d_task_cum) {
    if (hipMalloc((void**)&h->d_task_cum, (size_t)NMMO_MAX_TASKS * 8) != hipSuccess)
      return fail(NMMO_E_NOMEM, "task weight allocation");
  }
  HIP_TRY(hipMemcpy(h->d_task_cum, cum.data(), cum.size() * 8, hipMemcpyHostToDevice));
  h->st.task_cum = h->d_task_cum;
  return NMMO_OK;
}

int nmmo_set_wrapper(NmmoHandle* h, const NmmoWrapperConfig* wc, NmmoAgentInfo* dev_info) {
  if (!h) return fail(NMMO_E_INVALID, "null handle");
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipDeviceSynchronize());
  if (!wc) {
    h->wrap_on = false;
    h->d_info = nullptr;
    return NMMO_OK;
  }
  if (h->cfg.event_cap <= 0) return fail(NMMO_E_INVALID, "the wrapper layer needs the event log (event_cap > 0)");
  if (wc->kind < NMMO_WRAP_BASE || wc->kind > NMMO_WRAP_YAOFENG) return fail(NMMO_E_INVALID, "wrapper kind %d", wc->kind);
  if (wc->clip_unique_event < 0) return fail(NMMO_E_INVALID, "clip_unique_event < 0");
  const size_t nP = (size_t)h->st.n_envs * h->st.P;
  if (!h->d_ws) {
    if (hipMalloc((void**)&h->d_ws, nP * sizeof(NmmoWrapState)) != hipSuccess ||
        hipMalloc((void**)&h->d_uniq, nP * NMMO_UNIQ_WORDS * 4) != hipSuccess ||
        hipMalloc((void**)&h->d_wenv, (size_t)h->st.n_envs * 4) != hipSuccess ||
        hipMalloc((void**)&h->d_wdrop, sizeof(unsigned long long)) != hipSuccess)
      return fail(NMMO_E_NOMEM, "wrapper state allocation");
  }
  HIP_TRY(hipMemset(h->d_wdrop, 0, sizeof(unsigned long long)));
  h->wc = *wc;
  h->d_info = dev_info;
  h->wrap_on = true;
  HIP_TRY(launch_wrap(wrap_params(h, nullptr, nullptr, nullptr, nullptr, nullptr), 1, nullptr));
  HIP_TRY(hipDeviceSynchronize());
  return NMMO_OK;
}

int nmmo_get_wrapper_state(NmmoHandle* h, NmmoWrapState* host_state, uint32_t* host_uniq) {
  if (!h || !host_state) return fail(NMMO_E_INVALID, "null argument");
  if (!h->d_ws) return fail(NMMO_E_INVALID, "the wrapper layer was never enabled");
  const size_t nP = (size_t)h->st.n_envs * h->st.P;
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(host_state, h->d_ws, nP * sizeof(NmmoWrapState), hipMemcpyDeviceToHost));
  if (host_uniq) HIP_TRY(hipMemcpy(host_uniq, h->d_uniq, nP * NMMO_UNIQ_WORDS * 4, hipMemcpyDeviceToHost));
  return NMMO_OK;
}

int nmmo_get_wrapper_dropped(NmmoHandle* h, int64_t* total) {
  if (!h || !total) return fail(NMMO_E_INVALID, "null argument");
  if (!h->d_wdrop) return fail(NMMO_E_INVALID, "the wrapper layer was never enabled");
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipDeviceSynchronize());
  unsigned long long v = 0;
  HIP_TRY(hipMemcpy(&v, h->d_wdrop, sizeof(v), hipMemcpyDeviceToHost));
  *total = (int64_t)v;
  return NMMO_OK;
}

int nmmo_get_events(NmmoHandle* h, int32_t env, int32_t* host_rows, int32_t max_rows, int32_t* n_rows) {
  if (!h || !n_rows || (max_rows > 0 && !host_rows)) return fail(NMMO_E_INVALID, "null argument");
  if (env < 0 || env >= h->st.n_envs) return fail(NMMO_E_INVALID, "env %d out of range", env);
  *n_rows = 0;
  const int cap = h->cfg.event_cap;
  if (cap <= 0 || max_rows <= 0) return NMMO_OK;
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipDeviceSynchronize());
  int32_t cnt = 0;
  HIP_TRY(hipMemcpy(&cnt, h->d_env + (size_t)env * NMMO_NE + E_EVENT_COUNT, 4, hipMemcpyDeviceToHost));
  int n = cnt < cap ? cnt : cap;
  if (n > max_rows) n = max_rows;
  const int32_t* ring = h->d_events + (size_t)env * cap * NMMO_EVENT_COLS;
  const int first = (int)((cnt - n) % cap);  // ring index of the oldest copied row
  const int n1 = n < cap - first ? n : cap - first;
  HIP_TRY(hipMemcpy(host_rows, ring + (size_t)first * NMMO_EVENT_COLS, (size_t)n1 * NMMO_EVENT_COLS * 4,
                    hipMemcpyDeviceToHost));
  if (n > n1)
    HIP_TRY(hipMemcpy(host_rows + (size_t)n1 * NMMO_EVENT_COLS, ring, (size_t)(n - n1) * NMMO_EVENT_COLS * 4,
                      hipMemcpyDeviceToHost));
  *n_rows = n;
  return NMMO_OK;
}

int nmmo_set_map_bank(NmmoHandle* h, const uint8_t* host_buf, size_t nbytes) {
  if (!h || !host_buf) return fail(NMMO_E_INVALID, "null argument");
  const size_t need = (size_t)h->cfg.map_n * NMMO_MAP_TILES;
  if (nbytes != need) return fail(NMMO_E_SIZE, "map bank buffer %zu != %zu", nbytes, need);
  for (size_t i = 0; i < need; i++)
    if (host_buf[i] >= 16) return fail(NMMO_E_INVALID, "map %zu tile %zu: material %d >= 16", i / NMMO_MAP_TILES,
                                       i % NMMO_MAP_TILES, (int)host_buf[i]);
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(h->d_bank, host_buf, need, hipMemcpyHostToDevice));
  HIP_TRY(launch_rebuild_dep(h->st, nullptr));
  HIP_TRY(hipDeviceSynchronize());
  h->native_fresh = false;
  return NMMO_OK;
}

int nmmo_get_map_bank(NmmoHandle* h, uint8_t* host_buf, size_t nbytes) {
  if (!h || !host_buf) return fail(NMMO_E_INVALID, "null argument");
  const size_t need = (size_t)h->cfg.map_n * NMMO_MAP_TILES;
  if (nbytes != need) return fail(NMMO_E_SIZE, "map bank buffer %zu != %zu", nbytes, need);
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(host_buf, h->d_bank, need, hipMemcpyDeviceToHost));
  return NMMO_OK;
}

}  // extern "C"
