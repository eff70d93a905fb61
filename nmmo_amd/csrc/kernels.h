// kernels.h — launch interface shared by the kernel translation units and the C-ABI host code.
#pragma once

#include "common.h"

namespace nmmo {

// Slim entity table (tick.hip): system sets whose tick never changes 15 of the entity fields
constexpr int kSlimNF = 30;
__host__ __device__ constexpr bool slim_systems(uint32_t sy) {
  return (sy & (NMMO_SYS_ITEM | NMMO_SYS_EQUIPMENT | NMMO_SYS_PROFESSION | NMMO_SYS_EXCHANGE)) == 0;
}
__host__ __device__ constexpr bool slim_staged(int f) {
  return f != F_ITEM_LEVEL && f != F_MESSAGE && f != F_GOLD && !(f >= F_FISHING_LEVEL && f <= F_ALCHEMY_EXP) &&
         f != F_EQUIP_OFFENSE && f != F_EQUIP_DEFENSE;
}
// value of an unstaged field (slim only): profession levels are 1 for players, all else 0
__host__ __device__ constexpr int slim_const(int f, bool player) {
  return player && f >= F_FISHING_LEVEL && f <= F_ALCHEMY_EXP && ((f - F_FISHING_LEVEL) & 1) == 0 ? 1 : 0;
}

struct DevState {
  int32_t* env;          // [n][NMMO_NE]
  int16_t* ent;          // [n][NMMO_NF][S]
  int16_t* ring;         // [n][S]
  uint8_t* mat;          // [n][kTiles]
  uint32_t* dep;         // [n][kBitmapWords]
  const uint8_t* bank;   // [map_n][kTiles]
  uint2* items;          // [n][P][kInv] (SPEC §9)
  int16_t* iring;        // [n][kInv*P] free item rows
  int32_t* mlist;        // [n][NMMO_MARKET_ROWS] end-of-tick listings, ascending row: row | owner<<16 | slot<<24
  int* mcount;           // [n] listings in mlist (<= NMMO_MARKET_ROWS)
  int32_t* events;       // [n][cfg.event_cap][NMMO_EVENT_COLS] event-log rings (SPEC §11)
  const NmmoTask* tasks; // [n_tasks] task programs (SPEC §12)
  int32_t* assign;       // [n][P] task index of each player
  const uint64_t* task_cum;  // [n_tasks] sampling thresholds (nmmo_set_task_weights) or NULL
  NmmoTaskState* tstate; // [n][P] progress / event accumulators
  int n_tasks, tev;      // tev: some task term counts events
  int tmap;              // some task term reads the material map (CanSeeTile)
  int tsee;              // some task term counts window entities (CanSeeAgent / CanSeeGroup)
  int n_envs, P, N, S;   // N = NPC capacity (0 when the NPC system is off), S = P + N
  uint64_t seed;         // create seed (first-episode seeds)
  unsigned long long* counters;  // optional device u64 [3]: agent-steps, finished episodes, event rows
  NmmoConfig cfg;
  // device int: 1 when some env may hold a depleted tile whose map-bank material is not Foilage
  // (only nmmo_set_state / nmmo_set_map_bank can make one without the Profession system; a full
  // nmmo_reset clears it). While 0, the tick's respawn of a system set without professions needs
  // no map-bank read: its only depletion is Foilage eaten to Scrub.
  int32_t* foreign;
  // device int: the first bounded tick loop that hit its bound (kFault* | env << 8), 0 = none
  // (nmmo_get_fault). Every round loop stops at a bound the serial argument never reaches, so a
  // state outside the tick's invariants ends the launch instead of hanging it.
  int32_t* fault;
  // launch-local env list (nmmo_step_envs): workgroup b steps env env_list[b] for b < n_list;
  // NULL = every env (workgroup b steps env b). Ids outside [0, n_envs) are dropped (fault word).
  const int32_t* env_list;
  int n_list;
  // The wire header's count words written by the tick (wire_count_kernel's outputs from the
  // workgroup's LDS state after the store, tick_kernel<NMMO_SYS_ALL, 384, 128> only): set by a
  // whole-handle nmmo_step into a wire buffer without the wrapper layer; wire == NULL = off
  struct WireFuse {
    uint8_t* wire;
    uint16_t* wrank;  // [n][kMaxSlots] (ObsParams::wrank)
    uint32_t* wpk;    // [n][kMaxSlots] (ObsParams::wpk)
    int n_envs;
    int spawn_immunity;
  } wf;
};
// grid size and env of workgroup b of a launch over an env list (NULL = all n envs)
__host__ __device__ inline int list_grid(const int32_t* list, int n_list, int n) { return list ? n_list : n; }

struct ObsParams {
  const int32_t* env;   // [n][NE]
  const int16_t* ent;   // [n][NF][S]
  const uint8_t* mat;   // [n][kTiles]
  const uint2* items;   // [n][P][kInv]
  const int32_t* mlist; // [n][NMMO_MARKET_ROWS] row | owner<<16 | slot<<24
  const int* mcount;    // [n]
  const float* task;    // [n_tasks][task_dim] Task obs per task
  const int32_t* assign; // [n][P]
  float* obs;           // [n][P][elems] (flat layout)
  uint8_t* nat;         // native layout (SPEC §8b) instead of obs when non-NULL
  uint8_t* wire;        // wire layout (SPEC §8c, NMMO_OBS_WIRE) instead of obs / nat when non-NULL;
                        // expand: the wire buffer the flat rows are decoded from
  const int* row_map;   // expand only: flat row of agent row e*P+a (< 0 = skip); NULL = identity
  int n_envs, P, S, elems, task_dim;
  uint32_t systems;
  int spawn_immunity;
  // flat offsets (NmmoLayout)
  int o_style, o_target, o_buy, o_destroy, o_give_item, o_give_target, o_gg_price, o_gg_target,
      o_move, o_sell_item, o_sell_price, o_use, o_agent_id, o_tick, o_entity, o_inventory,
      o_market, o_task, o_tile;
  // wrapper observation edits (SPEC §13): kWrapObs* bits, prev_price from the wrapper state
  const NmmoWrapState* ws;  // [n][P] or NULL
  int wflags;
  uint16_t* wcount;     // native only, or NULL: per agent 0x8000 | nv | ninv << 7 (0 = not in the realm), wire.hip
  int* wmcount;         // native only, or NULL: [n] the listing count of this obs launch (nmmo_wire_pack)
  uint16_t* wrank;      // wire only: [n][kMaxSlots] entity-table index of each slot (0xFFFF = none),
                        // wire_count_kernel -> wire_obs_kernel
  const int32_t* env_list;  // flat / native obs: gather only these envs (DevState::env_list), or NULL
  int n_list;
  uint32_t* wpk;        // wire only: [n][kMaxSlots] packed datastore-row words (agent_obs.h ao_pack),
                        // wire_count_kernel -> wire_obs_kernel
  int32_t* fault;             // DevState::fault (a look-back that never resolves records kFaultWireScan)
  // flat / native obs row state (nmmo_hip.h nmmo_obs_invalidate). zrow[e * P + a] holds the tag
  // of the buffer that zst[e * P + a] describes row (e, a) of (0 = none); a launch whose buffer has
  // tag ztag (nmmo_dev_alloc serial | offset, capi.hip obs_zero_tag; 0 = untracked buffer: every
  // row written in full, the state untouched) leaves alone what the state says is there already:
  // an all-zero row (kZsZero) of an agent out of the realm; in flat rows also the zero Entity rows
  // >= zs_hv, the zero Market rows and Buy.MarketItem entries >= zs_hm, and the Task embedding of
  // task zs_task.
  uint64_t* zrow;
  uint64_t* zst;
  uint64_t ztag;
  // flat rows (flat_obs.hip), per row kZext u64 (valid when zst has kZsExt): the 64-bit masks of
  // the 10 tracked ActionTargets chunks, the position (row | col << 8) the Tile section was written
  // for, and the 12 item words the Inventory section was written from
  uint64_t* zext;
  // wire layout only (nmmo_set_step_records): per agent 8 B reward | term | trunc | mask | 0,
  // written by wire_obs_kernel from the step's outputs (NULL = off)
  uint8_t* recs;
  int32_t* fault_dst;  // with recs: *fault's nonzero word CAS-ed into it (nmmo_fault_into's effect)
  const float* rew;
  const uint8_t* term;
  const uint8_t* trunc;
  const uint8_t* mask;
  unsigned long long* rows_out;  // optional [n][2]: += rows this launch wrote, bytes it stored, per env
  int counted;  // wire layout: the tick wrote the header's count words (DevState::wf), no count launch
};
constexpr uint64_t kZsZero = 1ull << 20;
constexpr uint64_t kZsExt = 1ull << 21;  // the row's extended state (ObsParams::zext) is valid
// the row's Tile section holds unknown values (a consumer wrote into it, nmmo_obs_invalidate_sections):
// the next flat gather rewrites the whole section (an all-zero row: zeroes it), and forgets the bit
constexpr uint64_t kZsTile = 1ull << 22;
constexpr int kZext = 10 + 1 + 12;       // u64 per row: chunk masks | position | item words
__host__ __device__ inline int zs_hv(uint64_t s) { return (int)(s & 255u); }
__host__ __device__ inline int zs_hm(uint64_t s) { return (int)((s >> 8) & 4095u); }
__host__ __device__ inline int zs_task(uint64_t s) { return (int)(uint32_t)(s >> 32); }
__host__ __device__ inline uint64_t zs_pack(int hv, int hm, int task) {
  return (uint64_t)hv | (uint64_t)hm << 8 | (uint64_t)(uint32_t)task << 32;
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int j) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, j) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), j) << 32;
}
constexpr int kWrapObsPrice = 1, kWrapObsNoGive = 2, kWrapObsNoDangerous = 4;

struct WrapParams {
  const int32_t* env;        // [n][NE]
  const int16_t* ent;        // [n][NF][S]
  const uint2* items;        // [n][P][kInv]
  const int32_t* events;     // [n][evcap][NMMO_EVENT_COLS]
  const NmmoTaskState* tstate;  // [n][P]
  const int32_t* actions;    // [n][P][12] of this step, NULL on reset
  float* rew;                // [n][P] shaped in place
  const uint8_t* term;
  const uint8_t* trunc;
  const uint8_t* mask;
  NmmoWrapState* ws;         // [n][P]
  uint32_t* uniq;            // [n][P][NMMO_UNIQ_WORDS]
  int32_t* wenv;             // [n] event rows already processed
  unsigned long long* wdrop; // [1] event rows overwritten before the wrapper read them
  NmmoAgentInfo* info;       // [n][P] caller-owned, may be NULL
  NmmoWrapperConfig wc;
  int n_envs, P, S, evcap, items_on;
  const int32_t* env_list;   // step only: the stepped envs (DevState::env_list), or NULL
  int n_list;
};

struct PolicyParams {
  const int32_t* env;
  const int16_t* ent;
  const uint8_t* mat;
  const uint2* items;
  const int32_t* mlist;
  const int* mcount;
  int32_t* actions;  // [n][P][12]
  int n_envs, P, S;
  uint32_t systems;
  int spawn_immunity;
  uint64_t seed;
};

hipError_t init_kernels();  // one-time function attributes (dynamic LDS above 64 KB)
hipError_t launch_mapgen(uint64_t seed, int map_n, uint8_t* bank, hipStream_t stream);
hipError_t launch_tick(const DevState& st, const int32_t* actions, const uint64_t* env_seeds,
                       float* rew, uint8_t* term, uint8_t* trunc, uint8_t* mask, int mode,
                       hipStream_t stream);
hipError_t launch_rebuild_dep(const DevState& st, hipStream_t stream);
hipError_t launch_obs(const ObsParams& p, hipStream_t stream);
hipError_t launch_expand(const ObsParams& p, hipStream_t stream);  // native -> flat (SPEC §8b)
// wire codec (wire.hip, SPEC §8c): native <-> compact transport records
hipError_t launch_wire_pack(const uint16_t* counts, const int* mcount, const uint8_t* native, uint8_t* wire, int n,
                            int P, const int16_t* ent, int S, int exch, hipStream_t s);
hipError_t launch_wire_unpack(const uint8_t* wire, uint8_t* native, int n, int P, hipStream_t s);
// NMMO_OBS_WIRE: per-agent count words + per-env payload sizes (wire_count_kernel) and their
// scan, ahead of obs_kernel's record writes (obs.hip launch_obs)
hipError_t launch_wire_header(const ObsParams& p, hipStream_t s);
// NMMO_OBS_WIRE obs gather (wire_obs.hip): header pre-pass + wire_obs_kernel
hipError_t launch_wire_obs(const ObsParams& p, hipStream_t s);
// flat obs rows into the handle's bound buffer, incrementally (flat_obs.hip; p.ztag != 0)
hipError_t launch_flat_obs(const ObsParams& p, hipStream_t s);
bool flat_obs_ok(const ObsParams& p);  // launch_flat_obs takes p (else obs_kernel<kWrap, false>)
// NMMO_OBS_NATIVE obs gather (native_obs.hip)
hipError_t launch_native_obs(const ObsParams& p, hipStream_t s);
// header + record-head consistency of a wire buffer; bits into *status (0 = valid)
hipError_t launch_wire_check(const uint8_t* wire, int n, int P, const int64_t* expect_total, int* status,
                             hipStream_t s);
// several buffers' checks as one launch (nmmo_wire_check_many)
constexpr int kMaxCheckBufs = 16;
struct WireCheckBatch {
  const uint8_t* wire[kMaxCheckBufs];
  const int64_t* expect[kMaxCheckBufs];
  int n[kMaxCheckBufs];
  int count;
};
hipError_t launch_wire_check_many(const WireCheckBatch& b, int P, int* status, hipStream_t s);
// wire records -> flat float32 rows (p.wire, p.obs, p.row_map as in launch_expand)
hipError_t launch_wire_expand(const ObsParams& p, hipStream_t s);
hipError_t launch_store(const NmmoExperience& x, const NmmoStoreInput& in, const ObsParams* native,
                        int* scratch, hipStream_t stream);  // storage.hip
// compact record storage (storage.hip): the store's wire buffer into rs's arena, row references
hipError_t launch_store_records(const NmmoExperience& x, const NmmoRecordStore& rs, const NmmoStoreInput& in,
                                int P, int64_t wire_cap, int* scratch, hipStream_t stream);
// several wire buffers in one record store (storage.hip)
constexpr int kMaxStoreInputs = 16;
struct StoreBatch {
  NmmoStoreInput in[kMaxStoreInputs];
  int64_t wire_cap[kMaxStoreInputs];  // each buffer's capacity bound (nmmo_wire_max_bytes)
  int n, P;
  int stride;  // bytes between consecutive rows' reward / done / mask (0: packed float / u8 arrays)
};
// the fused received-buffer check of the learner root's store (nmmo_exp_store_records_checked)
struct StoreCheck {
  const int64_t* expect[kMaxStoreInputs];  // each input's announced total (device), or NULL
  int* status;                             // the check bits of every input (nmmo_wire_check's), or NULL
  int* ctl;                                // [kMaxStoreInputs] per-input check bits; zero, left zero
  uint32_t mask;                           // bit i: check input i (an unchecked input counts as clean)
};
// the learner gather's native point-to-point groups (p2p.hip; RCCL resolved at run time)
int p2p_load(const char* path, char* err, size_t n);
int p2p_unique_id(void* id, char* err, size_t n);
int p2p_init(const void* id, int world, int rank, void** comm, char* err, size_t n);
int p2p_group(void* comm, const NmmoP2POp* ops, int n_ops, hipStream_t stream, char* err, size_t n);
int p2p_destroy(void* comm);
int store_many_scratch_ints(int n_inputs, int max_rows);
hipError_t launch_store_records_many(const NmmoExperience& x, const NmmoRecordStore& rs, const StoreBatch& b,
                                     int* scratch, hipStream_t stream, const StoreCheck* chk = nullptr);
// flat rows of stored record rows (wire.hip)
hipError_t launch_record_gather(const ObsParams& p, const NmmoRecordStore& rs, const int32_t* idx, int n,
                                float* out, hipStream_t stream);
int store_blocks(int n_rows);
hipError_t launch_sort(const NmmoExperience& x, int32_t* idxs, int* scratch, hipStream_t stream);
hipError_t launch_gae(const NmmoExperience& x, const int32_t* idxs, int B, float g, float gl, float* adv,
                      hipStream_t stream);
hipError_t launch_gather_rows(const void* src, int64_t row_words, const int32_t* idx, int n, void* out,
                              hipStream_t stream);
hipError_t launch_policy(const PolicyParams& p, hipStream_t stream);
hipError_t launch_wrap(const WrapParams& p, int mode, hipStream_t stream);

}  // namespace nmmo
