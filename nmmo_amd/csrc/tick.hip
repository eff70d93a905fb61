// tick.hip — the Realm tick (SPEC.md §4-§6) as one gfx950 workgroup per env.
//
// Replaces nmmo.Env.step / Env.reset behind the reference's call sites
// (reinforcement_learning/stat_wrapper.py:51,64; clean_pufferl.py:175,293,357).
//
// Execution model: thread s owns entity slot s (players 0..P-1, NPCs P.. in spawn order); the
// env's whole entity table (43 int16 fields x slots, ~33 KB at 384 slots), the free-row ring
// and the depleted-tile bitmap live in LDS for the duration of the tick; the material map stays
// in HBM/L2 (sparse per-entity accesses). nmmo's Python executes every phase one entity at a
// time in insertion order; each phase here is parallel over slots, and the order dependence is
// resolved exactly:
//   * food harvest: a player eats iff its tile is Foilage at phase start and no lower slot in
//     the realm stands on it (first-in-slot-order wins, later ones see Scrub);
//   * attacks: two attacks conflict iff their {attacker, target} sets intersect; rounds run, in
//     parallel, every remaining attack that is the lowest-slot remaining attack on both of its
//     entities, which is exactly the serial result (no earlier conflicting attack is pending);
//   * cull, free-row FIFO, NPC compaction and NPC spawn use wave ballots + block prefix counts;
//   * items (SPEC §9): every player's 12-slot inventory, the item-row FIFO, a listed-row bitmap
//     and row->owner map live in LDS too. Per-player item work (harvest, Use, Destroy, Sell,
//     expiry, death cleanup) runs in parallel and touches the item FIFO through block prefix
//     sums, so rows are allocated/freed in exactly the serial slot order; the cross-player
//     steps (Buy in shuffled order, Give/GiveGold, and ammunition + loot of executed attacks,
//     deferred to after the attack phase — equipment sums cannot change inside it) are
//     replayed by thread 0 in serial order.
#include "agent_obs.h"  // ao_pack / ao_in_window / ao_slot, wire.h (the tick-fused wire count)
#include "kernels.h"

namespace nmmo {

struct Ctx {
  int16_t* T;        // [nf][S] staged entity fields (all kNFLive, or the slim set: ent_row)
  int16_t* ent_g;    // global, this env's [NMMO_NF][S] entity table (slim reset writes)
  uint64_t* vism;    // [P][NW] visibility bitmap: bit j of word w = row 64w+j+1 visible to player
  int* gstart;       // [kGridCells+1] grid cell -> first glist index (after vism, union region)
  uint32_t* glist;   // [S] in-realm entities by cell: slot<<25 (players) | (ds_row-1)<<16 | r<<8 | c
  int16_t* rslot;    // [S+1] datastore row -> slot (set for the rows of in-realm entities)
  uint32_t* pp;      // [128] player -> r<<16 | c (0x80008000 when not in the realm): window tests
  int* hkey;         // [kHash] Foilage-tile hash: tile index (-1 = empty)
  int* hmin;         // [kHash] lowest player slot standing on that tile
  int16_t* amove;    // [S]
  int16_t* atgt;     // [S]
  int16_t* asty;     // [S]
  int* ft;           // [2][S] per-entity scratch (closest-player keys; round keys, double-buffered)
  int16_t* clist;    // [S] scratch list (hostile NPCs searching for a target)
  int16_t* ring;     // [S]
  uint32_t* dep;     // [kBitmapWords]
  int* E;            // [NMMO_NE]
  int* wtot;         // [32] wave totals: two alternating 8-wave buffers | attack-round flags
  int wsel;          // block-uniform: offset of the wave-total buffer the last prefix used
  int* misc;         // [16]
  uint8_t* pres;     // [128] present at tick start
  uint8_t* died;     // [128]
  uint8_t* mat;      // global, this env
  const uint8_t* bank;
  // items (SPEC §9), allocated only when the Item system is on
  uint2* inv;        // [P][kInv]
  int16_t* iring;    // [IC] free item rows (FIFO)
  int16_t* rmap;     // [IC+1] listed row -> owner | slot<<8
  uint64_t* lbits;   // [kLWords] listed-row bitmap (bit = row)
  int16_t* a_buy;    // [128] decoded Buy row
  int16_t* a_give;   // [128] decoded Give item row
  int16_t* a_givet;  // [128] Give target slot
  int16_t* a_ggt;    // [128] GiveGold target slot
  int16_t* a_gga;    // [128] GiveGold amount
  int16_t* kill;     // [128] slot killed by this player's attack (deferred loot)
  int16_t* order;    // [128] Buy order / serial replay lists
  uint8_t* fired;    // [128] executed attack (ammunition)
  uint32_t* ikey;    // [128] Buy sort keys
  int16_t* ev_dmg;   // [128] damage of the player's executed attack (-1 none): SCORE_HIT
  int16_t* ev_lvl;   // [128] combat level reached by that attack's XP (0 none): LEVEL_UP
  int32_t* evg;      // this env's event ring (global), evcap rows (SPEC §11)
  // tasks (SPEC §12)
  const NmmoTask* tasks;   // global task table
  int32_t* assign;         // global [P] task index of this env's players (written at reset when sampling)
  const uint64_t* task_cum;  // global [n_tasks] sampling thresholds, or NULL (fixed assignment)
  int n_tasks;
  NmmoTaskState* ts;    // [P] task state: == tsl when staged (task events on), else in HBM
  NmmoTaskState* tsl;   // LDS staging of ts (meaningful only when tev)
  NmmoTaskState* tsg;   // this env's task state in HBM. Accessed through tsl/tsg, never ts, on the
                        // hot path: ts may point to either, so its accesses are flat, and a flat
                        // load makes the next LDS wait (lgkmcnt) wait for HBM too
  int2* tdesc;             // LDS [128][2] (pred | a << 8, b) of each player's terms (when tev): what
                           // task_accumulate reads; 8 B, so C4's task staging keeps 2 workgroups per CU
  bool tev;
  bool tmap;         // DevState::tmap: a task reads the material map at the rewards
  bool tsee;         // DevState::tsee: a task counts window entities (the rewards' slot words in ft)
  int evcap, tick1;  // ring rows (0 = no event log); tick + 1 (the events' tick column)
  int S, P, N, IC;
  bool items, exch, prof, equip;
  bool foreign;      // !prof and DevState::foreign is set: respawn reads the map bank
  bool foreign_any;  // DevState::foreign is set: a respawn may change a tile's passability
  bool slim;         // no Item/Equipment/Profession/Exchange: the fields only they change stay in HBM
  int nf;            // staged entity fields (LDS rows of T)
  const NmmoConfig* cfg;
  uint32_t sysm;     // enabled systems: a compile-time constant in the specialised kernels
  int32_t* fault;    // DevState::fault
  int env;           // this workgroup's env (local index)
};

// Slim entity table (system sets without Item, Equipment, Profession and Exchange, e.g. BASELINE
// config 3): the 15 fields only those systems change -- ITEM_LEVEL, MESSAGE, GOLD, the 10
// profession levels/exps and the NPC equipment pair -- hold per-kind constants for the whole
// episode (players: profession levels 1, the rest 0; NPCs: 0), written to HBM at reset and never
// staged. The other 30 fields keep their order in 30 LDS rows: 45 -> 30 x S x 2 B of LDS
// (C3: 34.6 -> 23.0 KB, so 4 workgroups fit a CU instead of 3).
// LDS row of a staged field: its index minus the unstaged fields below it
__host__ __device__ constexpr int slim_row(int f) {
  return f - (f > F_ITEM_LEVEL) - (f > F_MESSAGE) - (f > F_GOLD) - (f > F_ALCHEMY_EXP ? 10 : 0) -
         (f > F_EQUIP_DEFENSE ? 2 : 0);
}
static_assert(slim_row(F_DROP_TOOL) == kSlimNF - 1, "slim rows");
__device__ __forceinline__ int ent_row(bool slim, int f) { return slim ? slim_row(f) : f; }
#define TF(f, s) c.T[ent_row(c.slim, (f)) * c.S + (s)]

// Diagnostic build only (-DNMMO_STAMPS, tools/stamps.py): thread NMMO_STAMP_TID (0) stamps the
// shader clock right after phase barriers; never compiled into the product library.
#ifdef NMMO_STAMPS
#ifndef NMMO_STAMP_TID  // the stamping thread (64: wave 1's timeline)
#define NMMO_STAMP_TID 0
#endif
__device__ unsigned long long g_stamps[4096 * 32];
#define NMMO_STAMP(k)                                                        \
  do {                                                                       \
    if (threadIdx.x == NMMO_STAMP_TID && blockIdx.x < 4096)                  \
      g_stamps[blockIdx.x * 32 + (k)] = __builtin_amdgcn_s_memtime();        \
  } while (0)
// a launch's stamps start from zero: a phase a system set compiles out reads as absent
#define NMMO_STAMP_CLEAR()                                                  \
  do {                                                                       \
    if (threadIdx.x < 32 && blockIdx.x < 4096) g_stamps[blockIdx.x * 32 + threadIdx.x] = 0ull; \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");                   \
    __builtin_amdgcn_wave_barrier();                                         \
  } while (0)
#else
#define NMMO_STAMP(k) \
  do {               \
  } while (0)
#define NMMO_STAMP_CLEAR() \
  do {                    \
  } while (0)
#endif

__device__ __forceinline__ bool sys(const Ctx& c, uint32_t b) { return (c.sysm & b) != 0; }
// a bounded loop hit its bound (NMMO_FAULT_*): the first one of a launch is kept (nmmo_get_fault)
__device__ __forceinline__ void tick_fault(const Ctx& c, int code) { atomicCAS(c.fault, 0, code | c.env << 8); }
// field of LDS row `row` of T (the inverse of ent_row)
__device__ __forceinline__ int row_field(bool slim, int row) {
  return slim ? row + (row >= 7) + 2 * (row >= 9) + 10 * (row >= 18) + 2 * (row >= 25) : row;
}
// read of any field, staged or not (the slim constants for the unstaged ones)
__device__ __forceinline__ int ent_get(const Ctx& c, int f, int s) {
  return c.slim && !slim_staged(f) ? slim_const(f, s < c.P) : (int)TF(f, s);
}
// the wave-total buffer for the next block prefix (alternates; see block_prefix_sum)
__device__ __forceinline__ int* wtot_next(Ctx& c) {
  c.wsel ^= 8;
  return c.wtot + c.wsel;
}
__device__ __forceinline__ uint64_t env_seed(const Ctx& c) {
  return (uint64_t)(uint32_t)c.E[E_SEED_LO] | ((uint64_t)(uint32_t)c.E[E_SEED_HI] << 32);
}

constexpr int kHash = 256;  // >= 2x players: open addressing never fills
constexpr int kLWords = 32;  // listed-row bitmap words (rows 1..12*128)

// item system: inventories, item FIFO, row map, listed bitmap, decoded Buy/Give actions
__host__ __device__ constexpr size_t item_lds_bytes(int P) {
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  const size_t ic = (size_t)kInv * P;
  return (size_t)P * kInv * 8 + al(ic * 2) + al((ic + 1) * 2) + kLWords * 8 + 5 * 256 + 512;
}
constexpr size_t kPlayerArrBytes = 4 * 256 + 128;  // kill, order, ev_dmg, ev_lvl, fired
// One LDS region, three lifetimes: the decode bitmap (phase 0; reused as the respawn group list
// in phase 6), the position hash (update/harvest) and the attack first-touch arrays.
__host__ __device__ inline bool uses_grid(uint32_t systems) {
  return (systems & (NMMO_SYS_COMBAT | NMMO_SYS_ITEM | NMMO_SYS_NPC)) != 0;
}
__host__ __device__ constexpr size_t union_lds_bytes(int S, bool grid) {
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  size_t u = (size_t)128 * ((S + 63) / 64) * 8 + (grid ? grid_lds_bytes(S) : 0);
  u = u > 2 * kHash * 4 ? u : 2 * kHash * 4;
  const size_t atk = al((size_t)S * 8) + al((size_t)S * 2);  // round keys [2][S] | clist
  return u > atk ? u : atk;
}

__host__ __device__ constexpr size_t tick_lds_bytes(int S, int P, bool items, bool tev, bool grid, bool slim) {
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  // task state is staged in LDS only when events feed its accumulators (else read in place)
  size_t b = (items ? item_lds_bytes(P) : 0) + kPlayerArrBytes;
  b += al((size_t)(slim ? kSlimNF : kNFLive) * S * 2);  // T
  b += union_lds_bytes(S, grid);     // vism + grid | hkey,hmin | ft,clist
  b += al((size_t)(S + 1) * 2);      // rslot
  b += 128 * 4;                      // pp
  b += 3 * al((size_t)S * 2);        // amove atgt asty
  b += al((size_t)S * 2);            // ring
  b += (size_t)kBitmapWords * 4;     // dep
  b += NMMO_NE * 4 + 32 * 4 + 16 * 4 + 128 + 128;
  // task state staging last (make_ctx): 16-B aligned
  if (tev) b = al(b) + al((size_t)P * sizeof(NmmoTaskState)) + 128 * 2 * 8;
  return b;
}
// C4 (384 slots, items) with task events staged (a curriculum with event-counting terms) must keep
// two workgroups per CU: at 82,000 B (80 B over half the CU's LDS) it ran one, and a tick took twice as long
static_assert(tick_lds_bytes(384, 128, true, true, true, false) <= 80 * 1024, "C4 tick LDS: 2 workgroups per CU");

// kS / kP: the slot / player counts when known at compile time (0 = st's)
template <int kS = 0, int kP = 0>
__device__ __forceinline__ Ctx make_ctx(unsigned char* smem, const DevState& st, int e, uint32_t sy) {
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  Ctx c;
  const int S = kS ? kS : st.S, P = kP ? kP : st.P;
  size_t o = 0;
  c.sysm = sy;
  c.items = (sy & NMMO_SYS_ITEM) != 0;
  c.exch = c.items && (sy & NMMO_SYS_EXCHANGE) != 0;
  c.prof = c.items && (sy & NMMO_SYS_PROFESSION) != 0;
  c.equip = c.items && (sy & NMMO_SYS_EQUIPMENT) != 0;
  // DevState::foreign is loaded with the env state (load_env): a scalar load of it here was
  // waited on by the next kernel-argument wait (SMEM returns out of order, so the compiler waits
  // lgkmcnt(0)), one HBM round trip ahead of the state copy
  c.foreign_any = false;
  c.foreign = false;
  c.IC = kInv * P;
  if (c.items) {  // 16-B aligned block first (inventories are copied with 16-B accesses)
    c.inv = reinterpret_cast<uint2*>(smem + o); o += (size_t)P * kInv * 8;
    c.iring = reinterpret_cast<int16_t*>(smem + o); o += al((size_t)c.IC * 2);
    c.rmap = reinterpret_cast<int16_t*>(smem + o); o += al((size_t)(c.IC + 1) * 2);
    c.lbits = reinterpret_cast<uint64_t*>(smem + o); o += kLWords * 8;
    c.a_buy = reinterpret_cast<int16_t*>(smem + o); o += 256;
    c.a_give = reinterpret_cast<int16_t*>(smem + o); o += 256;
    c.a_givet = reinterpret_cast<int16_t*>(smem + o); o += 256;
    c.a_ggt = reinterpret_cast<int16_t*>(smem + o); o += 256;
    c.a_gga = reinterpret_cast<int16_t*>(smem + o); o += 256;
    c.ikey = reinterpret_cast<uint32_t*>(smem + o); o += 512;
  } else {
    c.inv = nullptr;
    c.iring = nullptr;
    c.rmap = nullptr;
    c.lbits = nullptr;
    c.a_buy = c.a_give = c.a_givet = c.a_ggt = c.a_gga = nullptr;
    c.ikey = nullptr;
  }
  c.tev = st.tev != 0;
  c.tmap = st.tmap != 0;
  c.tsee = st.tsee != 0;
  c.tasks = st.tasks;
  c.assign = st.assign + (size_t)e * P;
  c.task_cum = st.task_cum;
  c.n_tasks = st.n_tasks;
  c.tsg = st.tstate + (size_t)e * P;
  c.kill = reinterpret_cast<int16_t*>(smem + o); o += 256;
  c.order = reinterpret_cast<int16_t*>(smem + o); o += 256;
  c.ev_dmg = reinterpret_cast<int16_t*>(smem + o); o += 256;
  c.ev_lvl = reinterpret_cast<int16_t*>(smem + o); o += 256;
  c.fired = smem + o; o += 128;
  c.slim = slim_systems(sy);
  c.nf = c.slim ? kSlimNF : kNFLive;
  c.T = reinterpret_cast<int16_t*>(smem + o); o += al((size_t)c.nf * S * 2);
  c.ent_g = st.ent + (size_t)e * NMMO_NF * S;
  {  // the union region (see union_lds_bytes)
    unsigned char* u = smem + o;
    c.vism = reinterpret_cast<uint64_t*>(u);
    {  // grid_lds_bytes
      const size_t vb = (size_t)128 * ((S + 63) / 64) * 8;
      c.gstart = reinterpret_cast<int*>(u + vb);
      c.glist = reinterpret_cast<uint32_t*>(u + vb + al((size_t)(kGridCells + 1) * 4));
    }
    c.hkey = reinterpret_cast<int*>(u);
    c.hmin = reinterpret_cast<int*>(u + kHash * 4);
    c.ft = reinterpret_cast<int*>(u);
    c.clist = reinterpret_cast<int16_t*>(u + al((size_t)S * 8));
    o += union_lds_bytes(S, uses_grid(sy));
  }
  c.rslot = reinterpret_cast<int16_t*>(smem + o); o += al((size_t)(S + 1) * 2);
  c.pp = reinterpret_cast<uint32_t*>(smem + o); o += 128 * 4;
  c.amove = reinterpret_cast<int16_t*>(smem + o); o += al((size_t)S * 2);
  c.atgt = reinterpret_cast<int16_t*>(smem + o); o += al((size_t)S * 2);
  c.asty = reinterpret_cast<int16_t*>(smem + o); o += al((size_t)S * 2);
  c.ring = reinterpret_cast<int16_t*>(smem + o); o += al((size_t)S * 2);
  c.dep = reinterpret_cast<uint32_t*>(smem + o); o += (size_t)kBitmapWords * 4;
  c.E = reinterpret_cast<int*>(smem + o); o += NMMO_NE * 4;
  c.wtot = reinterpret_cast<int*>(smem + o); o += 32 * 4;
  c.wsel = 0;
  c.misc = reinterpret_cast<int*>(smem + o); o += 16 * 4;
  c.pres = smem + o; o += 128;
  c.died = smem + o; o += 128;
  // task state last: its LDS staging exists only with task events (a run-time flag), so every
  // offset above is a compile-time constant in the specialised kernels
  o = al(o);  // (16-B words: copy_segs)
  c.tsl = reinterpret_cast<NmmoTaskState*>(smem + o);  // an LDS address either way
  if (c.tev) {
    c.ts = c.tsl;
    o += al((size_t)P * sizeof(NmmoTaskState));
    c.tdesc = reinterpret_cast<int2*>(smem + o); o += 128 * 2 * 8;
  } else {
    c.ts = c.tsg;  // HBM, touched once per player at the rewards
    c.tdesc = nullptr;
  }
  c.mat = st.mat + (size_t)e * kTiles;
  c.bank = st.bank;
  c.evcap = st.cfg.event_cap > 0 ? st.cfg.event_cap : 0;
  c.evg = c.evcap ? st.events + (size_t)e * c.evcap * NMMO_EVENT_COLS : nullptr;
  c.tick1 = 0;
  c.S = S;
  c.P = P;
  c.N = st.N;
  c.cfg = &st.cfg;
  c.fault = st.fault;
  c.env = e;
  return c;
}

// ---------------------------------------------------------------- load / store
// HBM -> LDS copy of up to 6 segments of 16-byte words as one flat index space, 8 loads in
// flight per thread before their LDS stores (a plain strided copy loop keeps one dependent
// load in flight per iteration: the state load was a quarter of a C2 tick). Segment 0 is the
// entity table; with `slim` its LDS rows are gathered from the staged fields' HBM rows
// (w = 16-B words per field row).
struct Seg16 {
  uint4* d;
  const uint4* s;
  int n;
};
__device__ __forceinline__ void copy_segs(const Seg16 (&sg)[6], int tid, int nt, bool slim, int w) {
  // segment lookup by selects (a runtime index into sg[] would put the array in scratch)
  const int e0 = sg[0].n, e1 = e0 + sg[1].n, e2 = e1 + sg[2].n, e3 = e2 + sg[3].n, e4 = e3 + sg[4].n,
            total = e4 + sg[5].n;
  auto src0 = [&](int i) -> const uint4* {
    if (!slim) return sg[0].s + i;
    const int row = i / w;
    return sg[0].s + row_field(true, row) * w + (i - row * w);
  };
  auto src = [&](int i) -> const uint4* {
    return i < e0 ? src0(i)
           : i < e1 ? sg[1].s + (i - e0)
           : i < e2 ? sg[2].s + (i - e1)
           : i < e3 ? sg[3].s + (i - e2)
           : i < e4 ? sg[4].s + (i - e3)
                    : sg[5].s + (i - e4);
  };
  auto dst = [&](int i) -> uint4* {
    return i < e0 ? sg[0].d + i
           : i < e1 ? sg[1].d + (i - e0)
           : i < e2 ? sg[2].d + (i - e1)
           : i < e3 ? sg[3].d + (i - e2)
           : i < e4 ? sg[4].d + (i - e3)
                    : sg[5].d + (i - e4);
  };
  // Full batches of U words per thread issue all U loads before the first LDS store. The
  // remainder (the whole copy at C2/C3: 3.7 and 6.3 words per thread) goes in batches of 4 whose
  // loads read a clamped index instead of branching around them, so 4 loads are in flight at once
  // at a quarter of the full batch's registers.
  // The loaded words pass through an empty asm before any LDS store: without it the compiler sank
  // each load into its store's branch (the segment selects lower to branches), and the batch
  // became load, wait, store, load, wait, ... -- one HBM round trip per word.
  auto hold = [](uint4& v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); };
  constexpr int U = 8;
  int b = tid;
  for (; b + (U - 1) * nt < total; b += U * nt) {
    uint4 r[U];
#pragma unroll
    for (int k = 0; k < U; k++) r[k] = *src(b + k * nt);
#pragma unroll
    for (int k = 0; k < U; k++) hold(r[k]);
#pragma unroll
    for (int k = 0; k < U; k++) *dst(b + k * nt) = r[k];
  }
  constexpr int T = 4;
  for (; b < total; b += T * nt) {
    uint4 r[T];
#pragma unroll
    for (int k = 0; k < T; k++) r[k] = *src(min(b + k * nt, total - 1));
#pragma unroll
    for (int k = 0; k < T; k++) hold(r[k]);
#pragma unroll
    for (int k = 0; k < T; k++)
      if (b + k * nt < total) *dst(b + k * nt) = r[k];
  }
}

// The depleted-tile bitmap (3.2 KB of a C2 env's 11 KB of state) held in registers from the
// state load until the update phase, when the C2 tick defers it (defer_dep): the tick's first
// barrier then waits on the entity table alone, and the bitmap, first touched by the harvest,
// arrives behind it.
constexpr int kDepU4 = kBitmapWords / 4;
struct DepQ {
  uint4 v0, v1;
};
// every state segment a whole number of 16-B words (task state: 40 B per player)
__device__ __forceinline__ bool state_v16(const Ctx& c) { return (c.S & 7) == 0 && (c.IC & 7) == 0 && (c.P & 1) == 0; }
__device__ __forceinline__ bool defer_dep(const Ctx& c, uint32_t ksys) {
  return ksys == NMMO_SYS_RESOURCE && state_v16(c) && 2 * (int)blockDim.x >= kDepU4;
}

__device__ __forceinline__ void load_env_arrays(Ctx& c, const DevState& st, int e, bool defer);
// may_defer: a compile-time constant (the C2 kernel), so the bitmap loads are unconditional: a
// conditional load leaves a register merge at the branch join that waits on it
__device__ __forceinline__ DepQ load_env(Ctx& c, const DevState& st, int e, bool may_defer, bool defer) {
  const int tid = threadIdx.x, nt = blockDim.x;
  // env scalars: loaded first, written to LDS after the copy has issued its loads (stored right
  // away, their wait put a whole HBM round trip ahead of the state copy)
  int ev = st.env[(size_t)e * NMMO_NE + min(tid, NMMO_NE - 1)];  // every thread: no branch join
  int fg = *st.foreign;  // (a vector load: vmcnt retires in order, waited with the copy's loads)
  load_env_arrays(c, st, e, defer);
  DepQ dq = {};
  if (may_defer) {  // clamped indices: the tick writes only the in-range words, and only if defer
    const uint4* dep4 = reinterpret_cast<const uint4*>(st.dep + (size_t)e * kBitmapWords);
    dq.v0 = dep4[min(tid, kDepU4 - 1)];
    dq.v1 = dep4[min(tid + nt, kDepU4 - 1)];
  }
  asm volatile("" : "+v"(ev), "+v"(fg));
  if (tid < NMMO_NE) c.E[tid] = ev;
  c.foreign_any = __builtin_amdgcn_readfirstlane(fg) != 0;  // uniform, read before any store
  c.foreign = !c.prof && c.foreign_any;
  return dq;
}

__device__ __forceinline__ void load_env_arrays(Ctx& c, const DevState& st, int e, bool defer) {
  const int tid = threadIdx.x, nt = blockDim.x, S = c.S;
  const int16_t* src = st.ent + (size_t)e * NMMO_NF * S;
  const bool v16 = state_v16(c);
  NmmoTaskState* tsg = st.tstate + (size_t)e * c.P;
  const uint4* ring4 = reinterpret_cast<const uint4*>(st.ring + (size_t)e * S);
  const uint4* dep4 = reinterpret_cast<const uint4*>(st.dep + (size_t)e * kBitmapWords);
  const int ntask = c.tev ? c.P * (int)sizeof(NmmoTaskState) / 16 : 0;
  if (v16) {
    Seg16 sg[6] = {
        {reinterpret_cast<uint4*>(c.T), reinterpret_cast<const uint4*>(src), c.nf * S / 8},
        {reinterpret_cast<uint4*>(c.ring), ring4, S / 8},
        {reinterpret_cast<uint4*>(c.dep), dep4, defer ? 0 : kDepU4},
        {reinterpret_cast<uint4*>(c.inv), reinterpret_cast<const uint4*>(st.items + (size_t)e * c.P * kInv),
         c.items ? c.P * kInv / 2 : 0},
        {reinterpret_cast<uint4*>(c.iring), reinterpret_cast<const uint4*>(st.iring + (size_t)e * c.IC),
         c.items ? c.IC / 8 : 0},
        {reinterpret_cast<uint4*>(c.tsl), reinterpret_cast<const uint4*>(tsg), ntask}};
    copy_segs(sg, tid, nt, c.slim, S / 8);
    return;
  }
  for (int i = tid; i < (c.tev ? c.P * (int)sizeof(NmmoTaskState) / 4 : 0); i += nt)
    reinterpret_cast<int*>(c.tsl)[i] = reinterpret_cast<const int*>(tsg)[i];
  for (int i = tid; i < c.nf * S; i += nt) {  // field by field (slim: staged fields only)
    const int row = i / S;
    c.T[i] = src[row_field(c.slim, row) * S + i - row * S];
  }
  for (int i = tid; i < S; i += nt) c.ring[i] = st.ring[(size_t)e * S + i];
  for (int i = tid; i < kBitmapWords; i += nt) c.dep[i] = st.dep[(size_t)e * kBitmapWords + i];
  if (c.items) {
    const uint4* s4 = reinterpret_cast<const uint4*>(st.items + (size_t)e * c.P * kInv);
    uint4* d4 = reinterpret_cast<uint4*>(c.inv);
    for (int i = tid; i < c.P * kInv / 2; i += nt) d4[i] = s4[i];
    for (int i = tid; i < c.IC; i += nt) c.iring[i] = st.iring[(size_t)e * c.IC + i];
  }
}

__device__ __forceinline__ void store_env(const Ctx& c, const DevState& st, int e) {
  const int tid = threadIdx.x, nt = blockDim.x, S = c.S;
  if (tid < NMMO_NE) st.env[(size_t)e * NMMO_NE + tid] = c.E[tid];
  int16_t* dst = st.ent + (size_t)e * NMMO_NF * S;
  if ((S & 7) == 0) {  // 16-B words, field runs contiguous in both layouts
    const int w = S / 8;
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    const uint4* s4 = reinterpret_cast<const uint4*>(c.T);
    for (int i = tid; i < c.nf * w; i += nt) {
      const int row = i / w;
      d4[row_field(c.slim, row) * w + i - row * w] = s4[i];
    }
  } else {
    for (int i = tid; i < c.nf * S; i += nt) {
      const int row = i / S;
      dst[row_field(c.slim, row) * S + i - row * S] = c.T[i];
    }
  }
  if (state_v16(c)) {  // the ring, bitmap and item ring as 16-B words too (2-B stores wrote partial lines)
    auto copy16 = [&](void* d, const void* s, int n) {
      for (int i = tid; i < n; i += nt) reinterpret_cast<uint4*>(d)[i] = reinterpret_cast<const uint4*>(s)[i];
    };
    copy16(st.ring + (size_t)e * S, c.ring, S / 8);
    copy16(st.dep + (size_t)e * kBitmapWords, c.dep, kDepU4);
    if (c.items) copy16(st.iring + (size_t)e * c.IC, c.iring, c.IC / 8);
  } else {
    for (int i = tid; i < S; i += nt) st.ring[(size_t)e * S + i] = c.ring[i];
    for (int i = tid; i < kBitmapWords; i += nt) st.dep[(size_t)e * kBitmapWords + i] = c.dep[i];
    if (c.items)
      for (int i = tid; i < c.IC; i += nt) st.iring[(size_t)e * c.IC + i] = c.iring[i];
  }
  if (c.items) {
    const uint4* s4 = reinterpret_cast<const uint4*>(c.inv);
    uint4* d4 = reinterpret_cast<uint4*>(st.items + (size_t)e * c.P * kInv);
    for (int i = tid; i < c.P * kInv / 2; i += nt) d4[i] = s4[i];
  }
  if (c.tev) {  // task state (SPEC §12), when staged
    if (state_v16(c)) {
      uint4* d4 = reinterpret_cast<uint4*>(st.tstate + (size_t)e * c.P);
      const uint4* s4 = reinterpret_cast<const uint4*>(c.tsl);
      for (int i = tid; i < c.P * (int)sizeof(NmmoTaskState) / 16; i += nt) d4[i] = s4[i];
    } else {
      int* dsti = reinterpret_cast<int*>(st.tstate + (size_t)e * c.P);
      const int* srci = reinterpret_cast<const int*>(c.tsl);
      for (int i = tid; i < c.P * (int)sizeof(NmmoTaskState) / 4; i += nt) dsti[i] = srci[i];
    }
  }
}

// ---------------------------------------------------------------- items (SPEC §9)
// Serial item-row FIFO operations (one thread at a time).
__device__ __forceinline__ void ifree(Ctx& c, int row) {
  c.iring[(c.E[E_ITEM_FREE_HEAD] + c.E[E_ITEM_FREE_COUNT]) % c.IC] = (int16_t)row;
  c.E[E_ITEM_FREE_COUNT] += 1;
}
__device__ __forceinline__ int ialloc(Ctx& c) {
  const int row = c.iring[c.E[E_ITEM_FREE_HEAD]];
  c.E[E_ITEM_FREE_HEAD] = (c.E[E_ITEM_FREE_HEAD] + 1) % c.IC;
  c.E[E_ITEM_FREE_COUNT] -= 1;
  return row;
}
__device__ __forceinline__ void update_item_level(Ctx& c, int p) {
  const uint2* inv = c.inv + p * kInv;
  int l = 0;
  for (int k = 0; k < kInv; k++) {
    const uint2 w = inv[k];
    if (!it_type(w)) break;
    l += it_equipped(w) ? it_level(w) : 0;
  }
  TF(F_ITEM_LEVEL, p) = (int16_t)l;
}
// a brand-new item (NPC drop): stacks onto ammunition, else a new row if there is room
__device__ __forceinline__ void receive_new(Ctx& c, int p, int type, int level) {
  uint2* inv = c.inv + p * kInv;
  const int k = inv_stack(inv, type, level);
  if (k >= 0) {
    inv[k].y += 1u;
    return;
  }
  if (inv_count(inv) >= kInv) return;
  const int row = ialloc(c);
  inv_insert(inv, make_uint2((uint32_t)type | ((uint32_t)level << 5), 1u | ((uint32_t)row << 16)));
}
// an existing (unequipped, unlisted) item moving into p's inventory; returns false if its row was freed
__device__ __forceinline__ bool receive_moved(Ctx& c, int p, uint2 w) {
  uint2* inv = c.inv + p * kInv;
  const int k = inv_stack(inv, it_type(w), it_level(w));
  if (k >= 0) {
    inv[k].y += (uint32_t)it_qty(w);
    ifree(c, it_row(w));
    return false;
  }
  if (inv_count(inv) >= kInv) {
    ifree(c, it_row(w));
    return false;
  }
  inv_insert(inv, w);
  return true;
}
// receive_moved without touching the item FIFO: a row stacking frees is returned in `freed`
// (-1 if none) for the caller to append in serial order
__device__ __forceinline__ bool receive_moved_deferred(Ctx& c, int p, uint2 w, int& freed) {
  uint2* inv = c.inv + p * kInv;
  const int k = inv_stack(inv, it_type(w), it_level(w));
  if (k >= 0) {
    inv[k].y += (uint32_t)it_qty(w);
    freed = it_row(w);
    return false;
  }
  if (inv_count(inv) >= kInv) {
    freed = it_row(w);
    return false;
  }
  inv_insert(inv, w);
  return true;
}
__device__ __forceinline__ bool has_room(const Ctx& c, int p, uint2 w) {
  const uint2* inv = c.inv + p * kInv;
  return inv_stack(inv, it_type(w), it_level(w)) >= 0 || inv_count(inv) < kInv;
}
__device__ __forceinline__ int inv_offense(const Ctx& c, int p, int style) {
  const uint2* inv = c.inv + p * kInv;
  int a = 0;
  for (int k = 0; k < kInv; k++) {
    const uint2 w = inv[k];
    if (!it_type(w)) break;
    a += it_equipped(w) ? item_attack(it_type(w), it_level(w), style) : 0;
  }
  return a;
}
__device__ __forceinline__ int inv_defense(const Ctx& c, int p) {
  const uint2* inv = c.inv + p * kInv;
  int d = 0;
  for (int k = 0; k < kInv; k++) {
    const uint2 w = inv[k];
    if (!it_type(w)) break;
    d += it_equipped(w) ? item_defense(it_type(w), it_level(w)) : 0;
  }
  return d;
}
// Frees up to one row per thread (row < 0: none), appended to the item FIFO in thread order.
// Every thread of the block must call this.
__device__ __forceinline__ void ring_append_ordered(Ctx& c, int row) {
  int tot;
  const int pre = block_prefix_sum(row >= 0 ? 1 : 0, wtot_next(c), &tot);
  if (row >= 0) c.iring[(c.E[E_ITEM_FREE_HEAD] + c.E[E_ITEM_FREE_COUNT] + pre) % c.IC] = (int16_t)row;
  __syncthreads();
  if (threadIdx.x == 0) c.E[E_ITEM_FREE_COUNT] += tot;
  __syncthreads();
}
// Item.Query.for_sale: listed-row bitmap + row -> owner | slot<<8 (block-wide, barriers inside)
__device__ __forceinline__ void build_market(Ctx& c) {
  const int tid = threadIdx.x;
  if (tid < kLWords) c.lbits[tid] = 0;
  __syncthreads();
  if (tid < c.P) {
    const uint2* inv = c.inv + tid * kInv;
    for (int k = 0; k < kInv; k++) {
      const uint2 w = inv[k];
      if (!it_type(w)) break;
      if (it_price(w)) {
        const int row = it_row(w);
        c.rmap[row] = (int16_t)(tid | (k << 8));
        atomicOr((unsigned long long*)&c.lbits[row >> 6], 1ull << (row & 63));
      }
    }
  }
  __syncthreads();
}
// row of the k-th listing (ascending row), or -1
__device__ __forceinline__ int kth_listed(const Ctx& c, int k) {
  for (int w = 0; w < kLWords; w++) {
    uint64_t m = c.lbits[w];
    const int pc = __popcll(m);
    if (k < pc) {
      for (int i = 0; i < k; i++) m &= m - 1;
      return (w << 6) + __builtin_ctzll(m);
    }
    k -= pc;
  }
  return -1;
}

// ---------------------------------------------------------------- event log (SPEC §11)
// Row of the episode's event `idx` (0-based) for player p.
// an event of player p feeds the event accumulators of p's task terms (SPEC §12)
static_assert(NMMO_N_PREDICATES <= 256, "the 8-B task descriptor packs the predicate in 8 bits");
__device__ __forceinline__ void task_accumulate(const Ctx& c, int p, int code, int type, int level, int number,
                                                int gold, int target) {
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int2 qd = c.tdesc[p * 2 + k];
    const int4 q = make_int4(qd.x & 255, qd.x >> 8, qd.y, 0);  // pred, a, b (c: not read here)
    int* acc = c.tsl[p].acc + 2 * k;  // called only when tev (staged)
    int add0 = 0, add1 = 0;
    switch (q.x) {
      case PRED_COUNT_EVENT: add0 = code == q.y; break;
      case PRED_PRACTICE_EATING: add0 = code == EV_EAT_FOOD; break;
      case PRED_SCORE_HIT: add0 = code == EV_SCORE_HIT && type == q.y; break;
      case PRED_HARVEST_ITEM: add0 = code == EV_HARVEST_ITEM && type == q.y && level >= q.z ? number : 0; break;
      case PRED_CONSUME_ITEM: add0 = code == EV_CONSUME_ITEM && type == q.y && level >= q.z ? number : 0; break;
      case PRED_LIST_ITEM: add0 = code == EV_LIST_ITEM && type == q.y && level >= q.z ? number : 0; break;
      case PRED_BUY_ITEM: add0 = code == EV_BUY_ITEM && type == q.y && level >= q.z ? number : 0; break;
      case PRED_EARN_GOLD: add0 = code == EV_EARN_GOLD ? gold : 0; break;
      case PRED_SPEND_GOLD: add0 = code == EV_BUY_ITEM ? gold : 0; break;
      case PRED_MAKE_PROFIT:
        add0 = code == EV_EARN_GOLD ? gold : 0;
        add1 = code == EV_BUY_ITEM ? gold : 0;
        break;
      case PRED_DEFEAT_ENTITY:
        add0 = code == EV_PLAYER_KILL && ((q.y == 0 && target < 0) || (q.y == 1 && target > 0)) && level >= q.z;
        break;
      default: break;
    }
    if (add0) atomicAdd(&acc[0], add0);
    if (add1) atomicAdd(&acc[1], add1);
  }
}

// Event `idx` (0-based in the episode) of player p: written to the ring when the log is on, and
// counted by p's task when some task counts events.
__device__ __forceinline__ void ev_put(const Ctx& c, int idx, int p, int code, int type, int level,
                                       int number, int gold, int target) {
  if (c.tev) task_accumulate(c, p, code, type, level, number, gold, target);
  if (!c.evcap) return;
  // ring row: a mask for power-of-two rings (the default 4,096; a uniform branch), else a
  // division, ~20 dependent instructions per event on this latency-bound path
  const int row = (c.evcap & (c.evcap - 1)) == 0 ? (idx & (c.evcap - 1)) : idx % c.evcap;
  int32_t* r = c.evg + (size_t)row * NMMO_EVENT_COLS;
  r[0] = idx + 1;
  r[1] = p + 1;
  r[2] = c.tick1;
  r[3] = code;
  r[4] = type;
  r[5] = level;
  r[6] = number;
  r[7] = gold;
  r[8] = target;
}
// Appends each thread's n events in thread (= slot) order: emit(first_index) writes them.
// evn is the block-uniform running count. Every thread must call (barriers inside).
template <typename F>
__device__ __forceinline__ void ev_append(Ctx& c, int& evn, int n, F&& emit) {
  int tot;
  const int pre = block_prefix_sum(n, wtot_next(c), &tot);
  if (n) emit(evn + pre);
  evn += tot;
}

// ring_append_ordered and ev_append in one prefix sum (one barrier fewer each): every thread
// reads the FIFO tail before the scan's barrier, thread 0 moves it after.
template <class F>
__device__ __forceinline__ void ring_ev_append(Ctx& c, int row, int& evn, int nev, F&& emit) {
  const int fb = c.E[E_ITEM_FREE_HEAD] + c.E[E_ITEM_FREE_COUNT];
  int tot;
  const int pre = block_prefix_sum((row >= 0 ? 1 : 0) | nev << 16, wtot_next(c), &tot);
  if (row >= 0) c.iring[(fb + (pre & 0xFFFF)) % c.IC] = (int16_t)row;
  if (nev) emit(evn + (pre >> 16));
  evn += tot >> 16;
  if (threadIdx.x == 0) c.E[E_ITEM_FREE_COUNT] += tot & 0xFFFF;
  __syncthreads();
}

// ---------------------------------------------------------------- NPC spawn (SPEC §5.7)
// Spawn attempt a (thread a < 25 of wave 0): its draw and its tile's material, taken early in the
// tick (npc_spawn_pre) so the spawn neither waits on HBM nor recomputes Philox on its critical path
struct SpawnPre {
  U4 u;          // draw(seed, tick + 1, P_NPC_SPAWN, a) (valid when `drawn`)
  uint32_t mat;  // the tile's material
};
// 25 attempts evaluated by lanes 0..24 of wave 0; accepted in attempt order up to capacity.
// pre: lane a's early draw and tile material (npc_spawn_pre); drawn = pre.u is set (the C3
// variant at <= 64 VGPRs does not keep it through the tick and draws again).
__device__ __forceinline__ void npc_spawn(Ctx& c, uint32_t tick, const SpawnPre& pre, bool drawn) {
  if (wave_id() == 0) {
    const int a = lane_id();
    const uint64_t seed = env_seed(c);
    bool valid = false;
    int r = 0, col = 0, type = 0, style = 0, level = 0;
    uint32_t u3 = 0;
    if (a < 25) {
      const U4 u = drawn ? pre.u : draw(seed, tick, P_NPC_SPAWN, (uint32_t)a, 0);
      r = kLo + (int)uniform_n(u.x, kCenter);
      col = kLo + (int)uniform_n(u.y, kCenter);
      valid = !impassable(c.foreign_any ? (int)c.mat[r * kSize + col] : (int)pre.mat);
      int dist = r - kLo;
      dist = min(dist, kHi - r);
      dist = min(dist, col - kLo);
      dist = min(dist, kHi - col);
      type = 20 * dist >= 1024 ? 3 : 20 * dist >= 640 ? 2 : 1;
      style = (int)uniform_n(u.z, 3);
      level = sys(c, NMMO_SYS_PROGRESSION) ? (9 * dist) / 64 + 1 : 0;
      u3 = u.w;
    }
    const uint64_t b = __ballot(valid);
    const int rank = __popcll(b & lanes_below());
    const int cnt = c.E[E_NPC_COUNT], room = c.N - cnt, head = c.E[E_FREE_HEAD];
    const int nacc = min(__popcll(b), room);
    if (valid && rank < room) {
      const int s = c.P + cnt + rank;
      for (int row = 0; row < c.nf; row++) c.T[row * c.S + s] = 0;
      TF(F_ID, s) = (int16_t)(c.E[E_NPC_NEXT_ID] - rank);
      TF(F_NPC_TYPE, s) = (int16_t)type;
      TF(F_ROW, s) = (int16_t)r;
      TF(F_COL, s) = (int16_t)col;
      TF(F_HEALTH, s) = 100;
      TF(F_FOOD, s) = 100;
      TF(F_WATER, s) = 100;
      TF(F_MELEE_LEVEL, s) = 1;
      TF(F_RANGE_LEVEL, s) = 1;
      TF(F_MAGE_LEVEL, s) = 1;
      if (level > 0) {
        TF(F_MELEE_LEVEL + 2 * style, s) = (int16_t)level;
        TF(F_MELEE_EXP + 2 * style, s) = (int16_t)exp_at_level(level);
      }
      if (sys(c, NMMO_SYS_EXCHANGE)) TF(F_GOLD, s) = (int16_t)level;
      TF(F_ALIVE, s) = 1;
      TF(F_DS_ROW, s) = c.ring[(head + rank) % c.S];
      TF(F_STYLE, s) = (int16_t)style;
      TF(F_NPC_LEVEL, s) = (int16_t)level;
      TF(F_DROP_ARMOR, s) = (int16_t)uniform_n(u3, 3);
      TF(F_DROP_TOOL, s) = (int16_t)uniform_n(u3 >> 2, 5);
      if (sys(c, NMMO_SYS_EQUIPMENT) && level > 0) {  // int(8 * (level - U[0,1)))
        const int eq = (int)(((((uint64_t)level << 32) - u3) * 8) >> 32);
        TF(F_EQUIP_OFFENSE, s) = (int16_t)eq;
        TF(F_EQUIP_DEFENSE, s) = (int16_t)eq;
      }
    }
    if (lane_id() == 0 && nacc > 0) {
      c.E[E_FREE_HEAD] = (head + nacc) % c.S;
      c.E[E_FREE_COUNT] -= nacc;
      c.E[E_NPC_NEXT_ID] -= nacc;
      c.E[E_NPC_COUNT] = cnt + nacc;
    }
  }
  __syncthreads();
}

// Thread a < 25 (wave 0): the material of NPC spawn attempt a's tile at tick + 1, loaded at tick
// start: the spawn only tests passability, which no phase of the tick changes -- unless a
// set_state / set_map_bank installed depleted tiles whose bank material is impassable
// (DevState::foreign: the respawn before the spawn may restore it; npc_spawn reads the map then) --
// and a load issued at the spawn waits for every tile and event store of the tick (vmcnt counts
// stores).
__device__ __forceinline__ SpawnPre npc_spawn_pre(const Ctx& c, uint32_t tick1, const uint8_t* map) {
  SpawnPre x = {{0u, 0u, 0u, 0u}, 0u};
  if (threadIdx.x >= 25) return x;
  x.u = draw(env_seed(c), tick1, P_NPC_SPAWN, threadIdx.x, 0);
  const int r = kLo + (int)uniform_n(x.u.x, kCenter), col = kLo + (int)uniform_n(x.u.y, kCenter);
  x.mat = map[r * kSize + col];
  return x;
}

// ---------------------------------------------------------------- reset (SPEC §4)
__device__ __forceinline__ void reset_env(Ctx& c, uint64_t seed, int episode, int env_global) {
  const int tid = threadIdx.x, nt = blockDim.x, S = c.S, P = c.P;
  for (int i = tid; i < c.nf * S; i += nt) c.T[i] = 0;
  if (c.slim) {  // the unstaged fields' per-kind constants, straight to HBM (never change after)
    for (int i = tid; i < (NMMO_NF_USED - kSlimNF) * S; i += nt) {
      const int k = i / S, slot = i - k * S;
      const int f = k == 0 ? F_ITEM_LEVEL : k == 1 ? F_MESSAGE : k == 2 ? F_GOLD
                  : k < 13 ? F_FISHING_LEVEL + (k - 3) : F_EQUIP_OFFENSE + (k - 13);
      c.ent_g[f * S + slot] = (int16_t)slim_const(f, slot < P);
    }
  }
  for (int i = tid; i < kBitmapWords; i += nt) c.dep[i] = 0;
  for (int i = tid; i < S; i += nt) c.ring[i] = i < c.N ? (int16_t)(P + 1 + i) : (int16_t)0;
  if (tid < NMMO_NE) c.E[tid] = 0;
  if (c.items) {
    for (int i = tid; i < P * kInv; i += nt) c.inv[i] = make_uint2(0u, 0u);
    for (int i = tid; i < c.IC; i += nt) c.iring[i] = (int16_t)(i + 1);
  }
  __syncthreads();
  if (tid == 0) {
    c.E[E_SEED_LO] = (int)(uint32_t)seed;
    c.E[E_SEED_HI] = (int)(uint32_t)(seed >> 32);
    c.E[E_EPISODE] = episode;
    c.E[E_ENV_INDEX] = env_global;
    c.E[E_MAP_ID] = (int)uniform_n(draw(seed, 0, P_MAPSEL, 0, 0).x, (uint32_t)c.cfg->map_n);
    c.E[E_FREE_COUNT] = c.N;
    c.E[E_NPC_NEXT_ID] = -1;
    c.E[E_PLAYERS_ALIVE] = P;
    c.E[E_ITEM_FREE_COUNT] = c.IC;
  }
  __syncthreads();
  {  // copy the bank map into the env's mutable map (16 B per lane)
    const uint4* src = reinterpret_cast<const uint4*>(c.bank + (size_t)c.E[E_MAP_ID] * kTiles);
    uint4* dst = reinterpret_cast<uint4*>(c.mat);
    for (int i = tid; i < kTiles / 16; i += nt) dst[i] = src[i];
  }
  if (tid < P) {
    const uint32_t off = uniform_n(draw(seed, 0, P_SPAWN_OFFSET, 0, 0).x, 508);
    const uint32_t p = (off + (uint32_t)(tid * 508 / P)) % 508, side = p / 127, k = p % 127;
    const int r = side == 0 ? kLo : side == 1 ? kLo + (int)k : side == 2 ? kHi : kHi - (int)k;
    const int col = side == 0 ? kLo + (int)k : side == 1 ? kHi : side == 2 ? kHi - (int)k : kLo;
    const uint32_t u = draw(seed, 0, P_RESILIENT, (uint32_t)tid, 0).x;
    TF(F_ID, tid) = (int16_t)(tid + 1);
    TF(F_ROW, tid) = (int16_t)r;
    TF(F_COL, tid) = (int16_t)col;
    TF(F_HEALTH, tid) = 100;
    TF(F_FOOD, tid) = 100;
    TF(F_WATER, tid) = 100;
#pragma unroll
    for (int sk = 0; sk < (c.slim ? 3 : 8); sk++) TF(F_MELEE_LEVEL + 2 * sk, tid) = 1;
    TF(F_ALIVE, tid) = 1;
    TF(F_DS_ROW, tid) = (int16_t)(tid + 1);
    TF(F_RESILIENT, tid) = u < c.cfg->resilient_u32 ? 1 : 0;
    if (c.task_cum) {  // curriculum sampling (SPEC §12): first i with u < cum[i], cum[n-1] = 2^32
      const uint64_t ut = draw(seed, 0, P_TASK, (uint32_t)tid, 0).x;
      int lo = 0, hi = c.n_tasks - 1;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (ut < c.task_cum[mid]) hi = mid; else lo = mid + 1;
      }
      c.assign[tid] = lo;
    }
  }
  __syncthreads();
  // (the map is the bank's copy just written: the bank holds the same material)
  if (sys(c, NMMO_SYS_NPC)) npc_spawn(c, 0, npc_spawn_pre(c, 0, c.bank + (size_t)c.E[E_MAP_ID] * kTiles), true);
}

// ---------------------------------------------------------------- NPC AI (SPEC §6)
__device__ __forceinline__ bool player_valid(const Ctx& c, int id, int r, int col) {
  if (id <= 0 || id > c.P) return false;
  const int s = id - 1;
  return TF(F_ALIVE, s) && TF(F_HEALTH, s) > 0 && linf(r, col, TF(F_ROW, s), TF(F_COL, s)) <= kVision;
}

// behavior.update: drop an attacker/target that is gone, dead or out of vision; true if this
// NPC is hostile with no target (it then needs the closest-player search)
__device__ __forceinline__ bool npc_validate(Ctx& c, int n) {
  const int r = TF(F_ROW, n), col = TF(F_COL, n);
  if (!player_valid(c, TF(F_ATTACKER_ID, n), r, col)) TF(F_ATTACKER_ID, n) = 0;
  if (!player_valid(c, TF(F_TARGET_ID, n), r, col)) TF(F_TARGET_ID, n) = 0;
  return TF(F_NPC_TYPE, n) == 3 && !TF(F_TARGET_ID, n);
}

// SPEC §6 v2 pathing, bit-parallel: the 15x15 window around the NPC as 15 row masks (bit j =
// window column j passable), a breadth-first wave grown from the target tile one 4-neighbour
// step per iteration with shifts and ORs, until it covers the NPC's tile (window centre) or
// stops growing. The NPC steps to the first of N, S, E, W that the previous wave covered, i.e.
// a neighbour one step closer to the target. -1 = unreachable inside the window. The window
// (rows r-7..r+7, cols c-7..c+7) lies inside the map: NPCs stay in the playable area 16..143.
// NPC hunt pathing (SPEC §6 v2): the first step of a shortest path from the NPC to its target
// inside the NPC's 15x15 window, by a breadth-first wave from the target over the window's
// passable tiles, stopping when it reaches the NPC's tile (then N, S, E, W: the first neighbour
// at distance - 1). Wave-cooperative: 16 lanes per request (lane i holds window row i as a 15-bit
// row of reached / passable tiles; rows i - 1 and i + 1 come from the neighbouring lanes by DPP),
// 4 requests per wave at once; the requests are the hunting NPCs farther than one tile from
// their target (a 256-bit slot mask in c.misc). Result per NPC slot in c.amove (direction, or -1
// = unreachable in the window, so the greedy step applies). Same iteration as the serial
// restatement in the oracle, so the same step.
constexpr int kBfsPending = -2;
__device__ __forceinline__ uint32_t dpp_row_up(uint32_t x) {    // lane i <- lane i - 1 in its 16-lane row (0 at row start)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t dpp_row_down(uint32_t x) {  // lane i <- lane i + 1 in its row (0 at row end)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x101, 0xF, 0xF, true);
}
// returns the number of requests (block-uniform: every thread counts the same LDS mask)
__device__ __forceinline__ int npc_bfs_phase(Ctx& c) {
  constexpr int W = 2 * kVision + 1;
  constexpr uint32_t kImp = (1u << M_VOID) | (1u << M_WATER) | (1u << M_STONE) | (1u << M_OCEAN) | (1u << M_FISH);
  constexpr uint32_t kMid = 1u << kVision;
  const uint32_t* req = reinterpret_cast<const uint32_t*>(c.misc);
  int nreq = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) nreq += __popc(req[k]);
  const int lane = lane_id(), grp = lane >> 4, row = lane & 15;
  const int nw = blockDim.x >> 6;
  const uint64_t gmask = 0xFFFFull << (16 * grp);
  for (int q0 = wave_id() * 4; q0 < nreq; q0 += nw * 4) {  // wave-uniform loop
    const int q = q0 + grp;
    const bool on = q < nreq;
    int n = -1;
    if (on) {  // the q-th requested NPC slot
      int k = q, wd = 0;
      while (k >= __popc(req[wd])) k -= __popc(req[wd++]);
      uint32_t m = req[wd];
      for (int i = 0; i < k; i++) m &= m - 1;
      n = c.P + 32 * wd + __builtin_ctz(m);
    }
    uint32_t pass = 0u, R = 0u;
    if (on && row < W) {
      const int r = TF(F_ROW, n), col = TF(F_COL, n), ts = TF(F_TARGET_ID, n) - 1;
      const int base = (r - kVision + row) * kSize + col - kVision;  // 15 bytes of this window row
      const uint32_t* wp = reinterpret_cast<const uint32_t*>(c.mat + (base & ~3));
      const int sh = base & 3;
      const uint32_t d[5] = {wp[0], wp[1], wp[2], wp[3], wp[4]};
#pragma unroll
      for (int j = 0; j < W; j++) {
        const int k = sh + j;
        const uint32_t mt = (d[k >> 2] >> ((k & 3) * 8)) & 15u;
        pass |= ((kImp >> mt) & 1u) ? 0u : (1u << j);
      }
      const int si = TF(F_ROW, ts) - r + kVision, sj = TF(F_COL, ts) - col + kVision;
      R = row == si ? (1u << sj) : 0u;
    }
    int result = -1;
    bool done = !on;
    for (int it = 0; it < W * W; it++) {
      const uint32_t up = dpp_row_up(R), dn = dpp_row_down(R);
      const uint32_t N = (R | (R << 1) | (R >> 1) | up | dn) & pass;
      const uint64_t grew = __ballot(N != R) & gmask;
      const uint64_t hit = __ballot(row == kVision && (N & kMid)) & gmask;
      const uint64_t rn = __ballot(row == kVision - 1 && (R & kMid)) & gmask;
      const uint64_t rs = __ballot(row == kVision + 1 && (R & kMid)) & gmask;
      const uint64_t re = __ballot(row == kVision && (R & (kMid << 1))) & gmask;
      if (!done) {
        if (hit) {  // the NPC's tile is reached at distance it + 1: R = distance <= it
          result = rn ? 0 : rs ? 1 : re ? 2 : 3;
          done = true;
        } else if (!grew) {
          done = true;
        }
      }
      if (__ballot(!done) == 0) break;
      R = N;
    }
    if (on && row == 0) c.amove[n] = (int16_t)result;
  }
  return nreq;
}
// greedy step toward (dr, dc) over the passable neighbours in nbm (SPEC §6 v1 rule)
__device__ __forceinline__ int greedy_step(int dr, int dc, uint32_t nbm) {
  const int dir_r = dr > 0 ? 1 : 0, dir_c = dc > 0 ? 2 : 3;
  const bool rows_first = iabs(dr) >= iabs(dc);
  const int first = rows_first ? dir_r : dir_c, second = rows_first ? dir_c : dir_r;
  const bool second_nz = rows_first ? dc != 0 : dr != 0;
  if ((nbm >> first) & 1u) return first;
  if (second_nz && ((nbm >> second) & 1u)) return second;
  return -1;
}
__device__ __forceinline__ void npc_decide(Ctx& c, int n, int closest, uint32_t nbm, int& move, int& tgt,
                                           int& sty) {
  const int r = TF(F_ROW, n), col = TF(F_COL, n), id = TF(F_ID, n);
  const U4 u = draw(env_seed(c), (uint32_t)c.E[E_TICK], P_NPC_MOVE, (uint32_t)(-id), 0);
  move = -1;
  tgt = -1;
  sty = TF(F_STYLE, n);
  const int type = TF(F_NPC_TYPE, n);
  bool hunt = false;
  if (type == 2 && TF(F_ATTACKER_ID, n)) {
    TF(F_TARGET_ID, n) = TF(F_ATTACKER_ID, n);
    hunt = true;
  } else if (type == 3) {
    if (!TF(F_TARGET_ID, n) && closest >= 0) TF(F_TARGET_ID, n) = TF(F_ID, closest);
    hunt = TF(F_TARGET_ID, n) != 0;
  }
  if (!hunt) {
    int cand[4], k = 0;
#pragma unroll
    for (int d = 0; d < 4; d++)
      if ((nbm >> d) & 1u) cand[k++] = d;
    if (k) move = cand[uniform_n(u.x, (uint32_t)k)];
    return;
  }
  const int ts = TF(F_TARGET_ID, n) - 1;
  const int tr = TF(F_ROW, ts), tc = TF(F_COL, ts);
  const int dist = linf(r, col, tr, tc);
  if (dist == 0) {
    move = (int)uniform_n(u.y, 4);
  } else if (dist > 1) {  // move.pathfind: npc_bfs_phase, then greedy if unreachable in the window
    move = kBfsPending;
    atomicOr(reinterpret_cast<uint32_t*>(c.misc) + ((n - c.P) >> 5), 1u << ((n - c.P) & 31));
  }
  if (dist <= 3) tgt = ts;
}

// ---------------------------------------------------------------- combat (SPEC §5.3)
__device__ __forceinline__ int combat_level(const Ctx& c, int s) {
  const int nsk = s < c.P && !c.slim ? 8 : 3;  // slim: profession levels are 1 <= melee level
  int l = 0;
  for (int k = 0; k < nsk; k++) l = max(l, (int)TF(F_MELEE_LEVEL + 2 * k, s));
  return l;
}

// Attack.call validity + combat.attack damage on the current LDS state; -1 = no attack.
// eq_off: x's equipment offense in this style; eq_def: t's equipment defense (both constant
// through the attack rounds: ammunition is fired after them)
__device__ __forceinline__ int eval_attack(const Ctx& c, int x, int sty, int t, int eq_off, int eq_def) {
  if (!TF(F_ALIVE, x) || TF(F_HEALTH, x) <= 0) return -1;
  if (!TF(F_ALIVE, t) || TF(F_HEALTH, t) <= 0 || t == x) return -1;
  if (x < c.P && t < c.P && TF(F_TIME_ALIVE, t) < c.cfg->spawn_immunity) return -1;
  if (x >= c.P && t >= c.P) return -1;
  if (linf(TF(F_ROW, x), TF(F_COL, x), TF(F_ROW, t), TF(F_COL, t)) > 3) return -1;
  const bool prog = sys(c, NMMO_SYS_PROGRESSION);
  int offense = prog ? 10 + 5 * TF(F_MELEE_LEVEL + 2 * sty, x) : 30;
  int defense = prog ? 5 * combat_level(c, t) : 0;
  offense += eq_off;
  defense += eq_def;
  const int e0 = TF(F_MELEE_EXP, t), e1 = TF(F_RANGE_EXP, t), e2 = TF(F_MAGE_EXP, t);
  const int mx = max(e0, max(e1, e2)), mn = min(e0, min(e1, e2));
  int mult4 = 4;
  if (mx != mn) {
    const int dom = e0 == mx ? 0 : e1 == mx ? 1 : 2;
    const int weak = dom == 0 ? 2 : dom == 1 ? 0 : 1;  // melee<-mage, range<-melee, mage<-range
    if (sty == weak) mult4 = 6;
  }
  const int d4 = max(mult4 * offense - 4 * defense, offense);
  return d4 >> 2;
}

__device__ __forceinline__ void apply_attack(Ctx& c, int x, int sty, int t, int dmg, int tick) {
  TF(F_ATTACKER_ID, t) = TF(F_ID, x);
  int lvl_up = 0;
  if (x < c.P && sys(c, NMMO_SYS_PROGRESSION)) {
    const int f = F_MELEE_EXP + 2 * sty;
    const int ex = TF(f, x) + 6;
    TF(f, x) = (int16_t)ex;
    const int nl = level_at_exp(ex);
    if (nl > TF(f - 1, x)) {
      TF(f - 1, x) = (int16_t)nl;
      lvl_up = nl;
    }
  }
  TF(F_DAMAGE, t) = (int16_t)dmg;
  const int h = max(0, (int)TF(F_HEALTH, t) - dmg);
  TF(F_HEALTH, t) = (int16_t)h;
  if (h == 0) TF(F_PLAYER_KILLS, x) += 1;
  TF(F_LATEST_COMBAT_TICK, x) = (int16_t)(tick + 1);
  TF(F_LATEST_COMBAT_TICK, t) = (int16_t)(tick + 1);
  if (x < c.P) {  // ammunition, loot and the events are applied after the phase, in slot order
    if (c.equip) c.fired[x] = 1;
    if (h == 0) c.kill[x] = (int16_t)t;
    c.ev_dmg[x] = (int16_t)dmg;
    c.ev_lvl[x] = (int16_t)lvl_up;
  }
}

// fire one unit of x's equipped ammunition of this style (serial)
__device__ __forceinline__ void fire_ammo(Ctx& c, int x, int style) {
  uint2* inv = c.inv + x * kInv;
  for (int k = 0; k < kInv; k++) {
    const uint2 w = inv[k];
    if (!it_type(w)) break;
    if (!it_equipped(w) || it_type(w) != T_WHETSTONE + style) continue;
    inv[k].y -= 1u;
    if (it_qty(inv[k]) == 0) {
      ifree(c, it_row(w));
      inv_remove(inv, k);
      update_item_level(c, x);
    }
    break;
  }
}

// fire_ammo without touching the item FIFO: the row freed by the last unit is returned (-1 if
// none) for the caller to append in serial order
__device__ __forceinline__ int fire_ammo_deferred(Ctx& c, int x, int style) {
  uint2* inv = c.inv + x * kInv;
  for (int k = 0; k < kInv; k++) {
    const uint2 w = inv[k];
    if (!it_type(w)) break;
    if (!it_equipped(w) || it_type(w) != T_WHETSTONE + style) continue;
    inv[k].y -= 1u;
    if (it_qty(inv[k]) == 0) {
      inv_remove(inv, k);
      update_item_level(c, x);
      return it_row(w);
    }
    break;
  }
  return -1;
}

// a player killed t: gold, then t's items (player) or drops (NPC) (serial; SPEC §9 Death)
__device__ __forceinline__ void loot(Ctx& c, int x, int t, int& evn) {
  if (sys(c, NMMO_SYS_EXCHANGE)) {
    TF(F_GOLD, x) = (int16_t)(TF(F_GOLD, x) + TF(F_GOLD, t));
    TF(F_GOLD, t) = 0;
  }
  if (!c.items) return;
  if (t < c.P) {
    uint2* inv = c.inv + t * kInv;
    while (it_type(inv[0])) {
      uint2 w = inv[0];
      if (c.evcap) ev_put(c, evn++, x, EV_LOOT_ITEM, it_type(w), it_level(w), it_qty(w), 0, TF(F_ID, t));
      w.x &= 0x1FFu;  // unequipped, unlisted
      inv_remove(inv, 0);
      receive_moved(c, x, w);
    }
    update_item_level(c, t);
  } else {
    const int lvl = TF(F_NPC_LEVEL, t) > 0 ? TF(F_NPC_LEVEL, t) : 1;
    if (sys(c, NMMO_SYS_EQUIPMENT)) {
      receive_new(c, x, T_HAT + TF(F_DROP_ARMOR, t), lvl);
      if (c.evcap) ev_put(c, evn++, x, EV_LOOT_ITEM, T_HAT + TF(F_DROP_ARMOR, t), lvl, 1, 0, TF(F_ID, t));
    }
    if (sys(c, NMMO_SYS_PROFESSION)) {
      receive_new(c, x, T_ROD + TF(F_DROP_TOOL, t), lvl);
      if (c.evcap) ev_put(c, evn++, x, EV_LOOT_ITEM, T_ROD + TF(F_DROP_TOOL, t), lvl, 1, 0, TF(F_ID, t));
    }
  }
}

// ---------------------------------------------------------------- task progress (SPEC §12)
__device__ __forceinline__ double per_d(int num, int den) { return (double)num / (double)(den > 0 ? den : 1); }
__device__ __forceinline__ double clip01(double x) { return x < 0.0 ? 0.0 : x > 1.0 ? 1.0 : x; }

// Is material `m` on any tile of the 15x15 window around (r, col) (this tick's materials, in
// HBM)? The window rows are loaded as aligned dwords, a row's 5 loads before its tests: a
// byte-by-byte early-exit scan waited, per byte, for every store the tick had queued before it
// (vmcnt counts stores too and retires in order). Bytes 0..14 of a row come out of its 5 dwords
// by v_alignbyte; a zero byte of row ^ (m x 4) is a match.
#ifndef NMMO_SEE_ROWS  // window rows loaded per batch (A/B knob; divides 15)
#define NMMO_SEE_ROWS 1  // (5 rows: same curricula times, more spills in every tick variant: C3 tick +1.3%)
#endif
constexpr int kSeeRows = NMMO_SEE_ROWS;
static_assert(15 % kSeeRows == 0, "window rows per batch");
__device__ __forceinline__ bool can_see_tile(const Ctx& c, int r, int col, int m) {
  if ((unsigned)m > 255u) return false;  // no tile byte holds it
  const uint32_t* m32 = reinterpret_cast<const uint32_t*>(c.mat);
  const uint32_t rep = (uint32_t)(m & 255) * 0x01010101u;
  auto zero_byte = [](uint32_t x) { return ((x - 0x01010101u) & ~x & 0x80808080u) != 0u; };
  bool hit = false;
  for (int r0 = 0; r0 < 15; r0 += kSeeRows) {
    uint32_t w[kSeeRows][5];
    int off[kSeeRows];
#pragma unroll
    for (int i = 0; i < kSeeRows; i++) {
      const int b = (r - kVision + r0 + i) * kSize + col - kVision;  // the row's first window byte
      off[i] = b & 3;
#pragma unroll
      for (int k = 0; k < 5; k++) w[i][k] = m32[min(max((b >> 2) + k, 0), kTiles / 4 - 1)];
    }
#pragma unroll
    for (int i = 0; i < kSeeRows; i++) {
      uint32_t v[4];
#pragma unroll
      for (int k = 0; k < 4; k++) v[k] = __builtin_amdgcn_alignbyte(w[i][k + 1], w[i][k], off[i]) ^ rep;
      // (byte 15 lies outside the window: forced nonzero)
      hit = hit || zero_byte(v[0]) || zero_byte(v[1]) || zero_byte(v[2]) || zero_byte(v[3] | 0xFF000000u);
    }
    if (hit) break;
  }
  return hit;
}

__device__ __forceinline__ double term_progress(const Ctx& c, int p, const NmmoTaskTerm& q, const int* acc) {
  const int sk = q.a >= 1 && q.a <= 8 ? q.a - 1 : -1;
  const uint2* inv = c.items ? c.inv + p * kInv : nullptr;
  switch (q.pred) {
    case PRED_TICK_GE: return per_d(c.tick1, q.a);
    case PRED_PRACTICE_EATING: {  // curriculum_tutorial.py:45-57, Python float arithmetic
      double pr = __dmul_rn((double)acc[0], 0.06);
      if (acc[0] >= 1) pr = __dadd_rn(pr, 0.1);
      if (acc[0] >= 3) pr = __dadd_rn(pr, 0.3);
      return pr;
    }
    case PRED_COUNT_EVENT: case PRED_SCORE_HIT: return per_d(acc[0], q.b);
    case PRED_HARVEST_ITEM: case PRED_CONSUME_ITEM: case PRED_LIST_ITEM: case PRED_BUY_ITEM:
    case PRED_DEFEAT_ENTITY: return per_d(acc[0], q.c);
    case PRED_EARN_GOLD: case PRED_SPEND_GOLD: return per_d(acc[0], q.a);
    case PRED_MAKE_PROFIT: return per_d(acc[0] - acc[1], q.a);
    case PRED_HOARD_GOLD: return per_d(ent_get(c, F_GOLD, p), q.a);
    case PRED_ATTAIN_SKILL: return sk >= 0 && ent_get(c, F_MELEE_LEVEL + 2 * sk, p) >= q.b ? 1.0 : 0.0;
    case PRED_GAIN_EXPERIENCE: return sk >= 0 ? per_d(ent_get(c, F_MELEE_EXP + 2 * sk, p), q.b) : 0.0;
    case PRED_EQUIP_ITEM:
      for (int k = 0; inv && k < kInv && it_type(inv[k]); k++)
        if (it_equipped(inv[k]) && it_type(inv[k]) == q.a && it_level(inv[k]) >= q.b) return 1.0;
      return 0.0;
    case PRED_OWN_ITEM: {
      int n = 0;
      for (int k = 0; inv && k < kInv && it_type(inv[k]); k++)
        if (it_type(inv[k]) == q.a && it_level(inv[k]) >= q.b) n += it_qty(inv[k]);
      return per_d(n, q.c);
    }
    case PRED_INVENTORY_SPACE_GE: return kInv - (inv ? inv_count(inv) : 0) >= q.a ? 1.0 : 0.0;
    case PRED_OCCUPY_TILE: return TF(F_ROW, p) == q.a && TF(F_COL, p) == q.b ? 1.0 : 0.0;
    case PRED_CAN_SEE_TILE: return can_see_tile(c, TF(F_ROW, p), TF(F_COL, p), q.a) ? 1.0 : 0.0;
    case PRED_CAN_SEE_AGENT: case PRED_CAN_SEE_GROUP: {
      // the target agent is one of the Entity obs rows of p's observation after this tick: in
      // the realm, within the 15x15 window, and among the first 100 such entities in datastore
      // row order (SPEC §12; teams: singletons in id order, left of agent id i is i - 1)
      const int id = q.a > 0 ? q.a : q.a == -1 ? (p == 0 ? c.P : p) : (p + 1 == c.P ? 1 : p + 2);
      const int t = id - 1;
      if (t < 0 || t >= c.P || !TF(F_ALIVE, t)) return 0.0;
      const int r = TF(F_ROW, p), col = TF(F_COL, p);
      if (linf(r, col, TF(F_ROW, t), TF(F_COL, t)) > kVision) return 0.0;
      const int dt = TF(F_DS_ROW, t);
      // over the slots' packed words (ds_row << 16 | row << 8 | col, dead: ds_row 511; built once
      // per tick in c.ft when a task counts window entities), four per LDS read: the per-slot
      // loop read four staged fields per slot, and one player's scan was most of a tick
      const uint4* sw = reinterpret_cast<const uint4*>(c.ft);
      int before = 0;
      for (int s4 = 0; s4 < (c.S + 3) >> 2; s4++) {
        const uint4 q4 = sw[s4];
        const uint32_t qs[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
        for (int k = 0; k < 4; k++)
          before += (int)(qs[k] >> 16) < dt && linf(r, col, (int)((qs[k] >> 8) & 255u), (int)(qs[k] & 255u)) <= kVision;
      }
      return before < kNObs ? 1.0 : 0.0;
    }
    case PRED_FULLY_ARMED: {
      if (q.a < 1 || q.a > 3 || !inv) return 0.0;
      const int need[5] = {T_HAT, T_TOP, T_BOTTOM, T_SPEAR + q.a - 1, T_WHETSTONE + q.a - 1};
      for (int j = 0; j < 5; j++) {
        bool ok = false;
        for (int k = 0; k < kInv && it_type(inv[k]); k++)
          ok = ok || (it_equipped(inv[k]) && it_type(inv[k]) == need[j] && it_level(inv[k]) >= q.b);
        if (!ok) return 0.0;
      }
      return 1.0;
    }
    default: return 0.0;
  }
}

// clipped progress of player p's task; SUM without fused multiply-adds (bit-exact with the oracle)
__device__ __forceinline__ double task_progress(const Ctx& c, int p, const NmmoTask& t, const int* acc) {
  const double p0 = clip01(term_progress(c, p, t.term[0], acc));
  if (t.combine == NMMO_TASK_SINGLE) return p0;
  const double p1 = clip01(term_progress(c, p, t.term[1], acc + 2));
  const double v = t.combine == NMMO_TASK_SUM
                       ? __dadd_rn(__dmul_rn((double)t.term[0].weight, p0), __dmul_rn((double)t.term[1].weight, p1))
                       : __dmul_rn(p0, p1);
  return clip01(v);
}

// ---------------------------------------------------------------- the tick (SPEC §5)
__device__ __forceinline__ bool acts(const Ctx& c, int s) { return TF(F_ALIVE, s) && TF(F_HEALTH, s) > 0; }
__device__ __forceinline__ bool same_tile(const Ctx& c, int a, int b) {
  return TF(F_ROW, a) == TF(F_ROW, b) && TF(F_COL, a) == TF(F_COL, b);
}
// slot of player s's k-th visible entity (previous obs' Entity row k), or -1
__device__ __forceinline__ int vis_kth(const Ctx& c, int s, int NW, int k) {
  for (int w = 0; w < NW; w++) {
    uint64_t m = c.vism[s * NW + w];
    const int pc = __popcll(m);
    if (k < pc) {
      for (int i = 0; i < k; i++) m &= m - 1;  // clear the k lowest set bits
      return c.rslot[(w << 6) + __builtin_ctzll(m) + 1];
    }
    k -= pc;
  }
  return -1;
}
// lowest player slot standing on `tile` (position hash), 0x7FFF if none
__device__ __forceinline__ int hash_min(const Ctx& c, int tile) {
  int hh = (int)(h32((uint32_t)tile) & (kHash - 1));
  for (int probe = 0; probe < kHash; probe++) {
    const int k = c.hkey[hh];
    if (k == tile) return c.hmin[hh];
    if (k == -1) return 0x7FFF;
    hh = (hh + 1) & (kHash - 1);
  }
  return 0x7FFF;  // (a full table: the insertion recorded NMMO_FAULT_HASH_PROBE)
}

// system sets with a specialised tick kernel: BASELINE configs 2 and 3 (config 4 = all)
constexpr uint32_t kSysC2 = NMMO_SYS_RESOURCE;
constexpr uint32_t kSysC3 = NMMO_SYS_RESOURCE | NMMO_SYS_COMBAT | NMMO_SYS_NPC | NMMO_SYS_PROGRESSION;

// Make a prefetched task / task state opaque at this point, field by field (an address-taken
// copy would go to scratch): nothing computed from them can be scheduled above the call, so the
// loads issued before the respawn are waited on at the rewards, not next to their issue.
__device__ __forceinline__ void launder(NmmoTask& t) {
#pragma unroll
  for (int k = 0; k < 2; k++)
    asm volatile("" : "+v"(t.term[k].pred), "+v"(t.term[k].a), "+v"(t.term[k].b), "+v"(t.term[k].c),
                 "+v"(t.term[k].weight));
  asm volatile("" : "+v"(t.combine));
}
__device__ __forceinline__ void launder(NmmoTaskState& t) {
  asm volatile("" : "+v"(t.last), "+v"(t.max_progress), "+v"(t.signals), "+v"(t.completed_tick));
  asm volatile("" : "+v"(t.acc[0]), "+v"(t.acc[1]), "+v"(t.acc[2]), "+v"(t.acc[3]));
}

// a player's 12 action heads (kHeads), loaded at kernel start
struct Heads {
  int v[kHeads];
};
__device__ __forceinline__ void tick_env(Ctx& c, Heads hd, bool defer, DepQ dq, float* rew, uint8_t* term,
                         uint8_t* trunc, uint8_t* mask) {
  const int tid = threadIdx.x, nt = blockDim.x, S = c.S, P = c.P;
  const int s = tid;
  const int tick = c.E[E_TICK];
  const int nslots = P + c.E[E_NPC_COUNT];
  const bool inslot = s < nslots;
  const bool items = c.items;
  const uint64_t seed = env_seed(c);
  c.tick1 = tick + 1;
  const bool evon = c.evcap > 0 || c.tev;
  int evn = c.E[E_EVENT_COUNT];  // block-uniform running event count (SPEC §11)

  if (s < P) c.pres[s] = (uint8_t)TF(F_ALIVE, s);
  if (tid < 8) c.misc[tid] = 0;  // hunt-pathing request mask (npc_bfs_phase)
  if (c.exch && tid < kLWords) c.lbits[tid] = 0;
  if (c.tev && s < P) {  // this player's task terms and event accumulators
    const NmmoTask& tk = c.tasks[c.assign[s]];
#pragma unroll
    // pred | a << 8 as unsigned bits (nmmo_set_tasks keeps |a| < 2^23), decoded by an arithmetic shift
    for (int k = 0; k < 2; k++)
      c.tdesc[s * 2 + k] = make_int2((int)((uint32_t)(tk.term[k].pred & 255) | (uint32_t)tk.term[k].a << 8), tk.term[k].b);
  }
  // only the listed-row bitmap's zeroing must precede this phase's writes (its atomicOr); pres,
  // misc and tdesc are read after the phase's closing barrier
  if (c.exch) __syncthreads();
  // Materials around this slot's tile at tick start, loaded here so their latency hides behind
  // the decode; used after it through `nbm`. Passability and Water never change within a tick
  // (every depletion/regrowth maps passable to passable and impassable to impassable), and no
  // entity moves before the move phase, so these stay exact for NPC steering, drinking,
  // foilage eating (the own tile is read before any harvest) and the move check.
  const int my_task = s < P ? c.assign[s] : 0;  // HBM; first used before the respawn phase
  const bool in_realm = s < S && inslot && TF(F_ALIVE, s);  // => health > 0 at tick start
  const int pos_r = s < S ? TF(F_ROW, s) : 0, pos_c = s < S ? TF(F_COL, s) : 0;
  if (in_realm) c.rslot[TF(F_DS_ROW, s)] = (int16_t)s;
  // Loaded as whole dwords by every thread (the map centre for slots not in the realm): row r's
  // 8 aligned bytes holding columns c-1..c+1, and the dwords holding column c in rows r-1 and
  // r+1. They stay opaque until the decode is done: byte loads let the compiler merge two of
  // them and split the result right after the load, which waited on HBM here.
  const int qr = in_realm ? pos_r : kSize / 2, qc = in_realm ? pos_c : kSize / 2;
  const uint32_t* mrow = reinterpret_cast<const uint32_t*>(c.mat + qr * kSize);
  const int mcw = (qc - 1) >> 2;
  uint32_t mw0 = mrow[mcw], mw1 = mrow[mcw + 1], mup = mrow[(qc >> 2) - kSize / 4],
           mdn = mrow[(qc >> 2) + kSize / 4];
  if (tid < 128) c.pp[tid] = (tid < P && TF(F_ALIVE, tid)) ? ((uint32_t)TF(F_ROW, tid) << 16) | (uint32_t)TF(F_COL, tid)
                                                        : 0x80008000u;
  if (c.exch && s < P) {  // listings of the previous observation (Buy.MarketItem index space)
    const uint2* inv = c.inv + s * kInv;
    for (int k = 0; k < kInv; k++) {
      const uint2 w = inv[k];
      if (!it_type(w)) break;
      if (it_price(w)) {
        const int row = it_row(w);
        c.rmap[row] = (int16_t)(s | (k << 8));
        atomicOr((unsigned long long*)&c.lbits[row >> 6], 1ull << (row & 63));
      }
    }
  }
  __syncthreads();
  NMMO_STAMP(1);

  // 0. decode (Env._validate_actions) against the previous observation's state.
  // Target indices select the k-th visible entity in datastore-row order (the previous obs'
  // Entity row k). Every wave builds the player x row visibility bitmap for its 64 rows with one
  // ballot per player; each player then selects its k-th set bit with popcounts.
  const int NW = (S + 63) >> 6;
  const bool combat = sys(c, NMMO_SYS_COMBAT);
  if (uses_grid(c.sysm)) {
    // Uniform grid (common.h): each player tests only the entities of the <= 3x3 cells its
    // 15x15 window touches. Bit (row-1) of the player's bitmap is set iff the entity in
    // datastore row `row` is in the realm and within L-inf 7 -- the same set an all-pairs test
    // gives, at a small fraction of the pair tests.
    uint32_t* vis32 = reinterpret_cast<uint32_t*>(c.vism);
    for (int k = tid; k < P * NW * 2; k += nt) vis32[k] = 0;
    int cell = -1;
    uint32_t gv = 0;
    if (in_realm) {  // players: slot in bits 25-31 (P <= 128)
      cell = (s < P ? 0 : kCells) + (pos_r >> kCellShift) * kGrid + (pos_c >> kCellShift);
      gv = ((uint32_t)(TF(F_DS_ROW, s) - 1) << 16) | (uint32_t)(pos_r << 8) | (uint32_t)pos_c |
           (s < P ? (uint32_t)s << 25 : 0u);
    }
    grid_build(c.gstart, c.glist, cell, gv);
    // kWinRows threads per player, one grid row of its window each; bits land with no-return
    // LDS atomics (ds_or_b32), so only the candidate loads are waited on, four at a time
    for (int t = tid; t < kWinRows * P; t += nt) {
      const int p = t / kWinRows;
      if (!c.pres[p]) continue;
      const int r = (int)(c.pp[p] >> 16), col = (int)(c.pp[p] & 0xFFFF);
      const int4 wdw = grid_window(r, col);
      const int cr = wdw.x + (t - kWinRows * p);
      if (cr > wdw.y) continue;
      uint32_t* mine = vis32 + p * NW * 2;
      auto setbit = [&](uint32_t v, int, int) {
        atomicOr(&mine[(v >> 21) & 15], 1u << ((v >> 16) & 31));
      };
      const int g = cr * kGrid;
      grid_scan(c.glist, c.gstart[g + wdw.z], c.gstart[g + wdw.w + 1], r, col, setbit);
      grid_scan(c.glist, c.gstart[kCells + g + wdw.z], c.gstart[kCells + g + wdw.w + 1], r, col, setbit);
    }
  }
  if (uses_grid(c.sysm)) __syncthreads();  // (without the grid the prep's barrier ordered all)
  NMMO_STAMP(13);
  // bits 0-3: neighbour d passable; 4-7: neighbour d is Water; 8-15: own tile material; 16-19:
  // neighbour (row - 1, row + 1, col - 1, col + 1) is Fish (the professions' order). Fish and
  // the own tile's material are read here, at tick start, by the harvest too: no harvest earlier
  // in the tick turns a tile into or out of Fish or a profession resource, and a load after the
  // tick's first tile store would wait for it (vmcnt counts stores).
  asm volatile("" : "+v"(mw0), "+v"(mw1), "+v"(mup), "+v"(mdn));
  const uint64_t mrow8 = (uint64_t)mw0 | ((uint64_t)mw1 << 32);
  const int msh = 8 * ((qc - 1) & 3), mcol = 8 * (qc & 3);
  const uint32_t m_n3 = in_realm ? (uint32_t)(mrow8 >> msh) & 255u : 0u;  // column c-1
  const uint32_t m_own = in_realm ? (uint32_t)(mrow8 >> (msh + 8)) & 255u : 0u;
  const uint32_t m_n2 = in_realm ? (uint32_t)(mrow8 >> (msh + 16)) & 255u : 0u;  // column c+1
  const uint32_t m_n0 = in_realm ? (mup >> mcol) & 255u : 0u;                    // row r-1
  const uint32_t m_n1 = in_realm ? (mdn >> mcol) & 255u : 0u;                    // row r+1
  const uint32_t nbm = (impassable(m_n0) ? 0u : 1u) | (impassable(m_n1) ? 0u : 2u) |
                       (impassable(m_n2) ? 0u : 4u) | (impassable(m_n3) ? 0u : 8u) |
                       (m_n0 == M_WATER ? 16u : 0u) | (m_n1 == M_WATER ? 32u : 0u) |
                       (m_n2 == M_WATER ? 64u : 0u) | (m_n3 == M_WATER ? 128u : 0u) | (m_own << 8) |
                       (m_n0 == M_FISH ? 1u << 16 : 0u) | (m_n1 == M_FISH ? 1u << 17 : 0u) |
                       (m_n3 == M_FISH ? 1u << 18 : 0u) | (m_n2 == M_FISH ? 1u << 19 : 0u);
  int my_move = -1, my_tgt = -1, my_sty = 0;
  int use_row = -1, destroy_row = -1, sell_row = -1, sell_price = 0;
  if (s < P) {
    if (items) {
      c.a_buy[s] = c.a_give[s] = c.a_givet[s] = c.a_ggt[s] = -1;
      c.a_gga[s] = 0;
    }
    c.kill[s] = -1;
    c.fired[s] = 0;
    c.ev_dmg[s] = -1;
    c.ev_lvl[s] = 0;
  }
  if (s < P && c.pres[s]) {
#pragma unroll
    for (int k = 0; k < kHeads; k++) asm volatile("" : "+v"(hd.v[k]));  // loaded before the state
    const int* a = hd.v;
    const int dmove = a[8], dsty = a[0], dk = a[1];
    if (dmove >= 0 && dmove < 5) my_move = dmove;
    if (combat && dsty >= 0 && dsty < 3 && dk >= 0 && dk < kNObs) {
      my_tgt = vis_kth(c, s, NW, dk);
      my_sty = my_tgt >= 0 ? dsty : 0;
    }
    if (items) {  // InventoryItem k -> item row of the previous obs' inventory slot k
      const uint2* inv = c.inv + s * kInv;
      const int n = inv_count(inv);
      auto row_of = [&](int k) { return (k >= 0 && k < n) ? it_row(inv[k]) : -1; };
      use_row = row_of(a[11]);
      destroy_row = row_of(a[3]);
      if (a[5] >= 0 && a[5] < kNObs) {
        const int gr = row_of(a[4]);
        const int t = gr >= 0 ? vis_kth(c, s, NW, a[5]) : -1;
        if (t >= 0) {
          c.a_give[s] = (int16_t)gr;
          c.a_givet[s] = (int16_t)t;
        }
      }
      if (c.exch) {
        if (a[7] >= 0 && a[7] < kNObs && a[6] >= 0 && a[6] < 99) {
          const int t = vis_kth(c, s, NW, a[7]);
          if (t >= 0) {
            c.a_ggt[s] = (int16_t)t;
            c.a_gga[s] = (int16_t)(a[6] + 1);
          }
        }
        if (a[10] >= 0 && a[10] < 99) {
          sell_row = row_of(a[9]);
          sell_price = a[10] + 1;
        }
        if (a[2] >= 0 && a[2] < NMMO_MARKET_ROWS) c.a_buy[s] = (int16_t)kth_listed(c, a[2]);
      }
    }
  }
#ifdef NMMO_STAMPS
  __syncthreads();
  NMMO_STAMP(12);
#endif
  // 1. npcs.actions. A hostile NPC without a target takes the closest player within vision
  // (ties to the lowest slot) from the players in the grid cells of its window.
  const bool npc_on = sys(c, NMMO_SYS_NPC);
  int closest = -1;
  if (npc_on && s >= P && inslot && npc_validate(c, s)) {
    const int r = TF(F_ROW, s), col = TF(F_COL, s);
    const int4 wdw = grid_window(r, col);
    int best = 0x7FFFFFFF;
    for (int cr = wdw.x; cr <= wdw.y; cr++)  // player cells only
      grid_scan(c.glist, c.gstart[cr * kGrid + wdw.z], c.gstart[cr * kGrid + wdw.w + 1], r, col,
                [&](uint32_t v, int d, int) { best = min(best, (d << 8) | (int)(v >> 25)); });
    closest = best == 0x7FFFFFFF ? -1 : (best & 255);
  }
  if (npc_on && s >= P && inslot) npc_decide(c, s, closest, nbm, my_move, my_tgt, my_sty);
  // wave 0 (players) has no NPC to decide: it draws the spawn attempts' tiles meanwhile (before
  // the tick's first global store)
  SpawnPre spawn = {{0u, 0u, 0u, 0u}, 0u};
  const bool spawn_drawn = c.sysm != kSysC3;
  if (npc_on) spawn = npc_spawn_pre(c, (uint32_t)(tick + 1), c.mat);
  asm volatile("" : "+v"(spawn.mat));  // opaque: waited on at the spawn, not here
  if (npc_on) {  // hunt pathing for the NPCs that asked (block-uniform)
    __syncthreads();
    // the results' barrier only when some NPC asked (no request: nothing was written)
    if (npc_bfs_phase(c) > 0) __syncthreads();
    if (my_move == kBfsPending) {
      const int r = c.amove[s];
      const int ts = TF(F_TARGET_ID, s) - 1;
      my_move = r >= 0 ? r : greedy_step(TF(F_ROW, ts) - TF(F_ROW, s), TF(F_COL, ts) - TF(F_COL, s), nbm);
    }
  }
  if (s < S) {
    c.amove[s] = (int16_t)my_move;
    c.atgt[s] = (int16_t)my_tgt;
    c.asty[s] = (int16_t)my_sty;
  }
  const bool grid = uses_grid(c.sysm);
  if (!grid) {  // the position hash's LDS held nothing this tick: initialised before the barrier
    for (int k = tid; k < kHash; k += nt) {
      c.hkey[k] = -1;
      c.hmin[k] = 0x7FFF;
    }
  }
  __syncthreads();
  NMMO_STAMP(2);
  // This player's task state (when it lives in HBM) and task, for the rewards. Loaded by every
  // thread from valid addresses (a conditional load leaves a register merge at the branch join
  // that waits on it); used only for present, surviving players. Issued here, a whole tick ahead
  // of the rewards, except in the <= 64-VGPR C3 variant, which cannot hold 24 more registers
  // through the middle phases and issues them after the respawn draws instead (issued before
  // them, the draw loop's head waits on them).
  const bool task_early = c.sysm != kSysC3;
  NmmoTaskState tsr = {};
  NmmoTask tk = {};
  if (task_early) {
    tsr = c.tsg[s < P ? s : 0];
    tk = c.tasks[my_task];
  }
  if (grid) {
    for (int k = tid; k < kHash; k += nt) {  // position hash (its LDS held the decode bitmap and grid)
      c.hkey[k] = -1;
      c.hmin[k] = 0x7FFF;
    }
    __syncthreads();
  }

  // 2. players.update / npcs.update. Every player in the realm registers its tile in the
  // position hash (lowest slot per tile via atomicMin): first-in-slot-order harvests.
  const bool resource = sys(c, NMMO_SYS_RESOURCE);
  int tile = 0, hslot = -1;
  // this player's update-phase events: EAT_FOOD, DRINK_WATER, harvests and level-ups
  bool e_eat = false, e_drink = false;
  int e_fish = 0, e_fish_nl = 0, e_on_q = -1, e_on_type = 0, e_on_lvl = 0, e_on_nl = 0;
  if (inslot && TF(F_ALIVE, s)) {
    if (TF(F_DAMAGE, s) == 0) TF(F_ATTACKER_ID, s) = 0;
    TF(F_DAMAGE, s) = 0;
    TF(F_TIME_ALIVE, s) += 1;
    if (s >= P) {
      TF(F_HEALTH, s) = (int16_t)min(100, TF(F_HEALTH, s) + 1);
    } else {
      const int r = TF(F_ROW, s), col = TF(F_COL, s);
      tile = r * kSize + col;
      if (resource) {
        const int org = TF(F_HEALTH, s);
        int h = org;
        const int food = TF(F_FOOD, s), water = TF(F_WATER, s);
        if (food > 50 && water > 50) h = min(100, h + 10);
        const int dmg = TF(F_RESILIENT, s) ? 5 : 10;
        if (food == 0) h = max(0, h - dmg);
        if (water == 0) h = max(0, h - dmg);
        TF(F_HEALTH, s) = (int16_t)h;
        TF(F_HEALTH_RESTORE, s) = (int16_t)(h - org);
        TF(F_FOOD, s) = (int16_t)max(0, food - 5);
        const bool drink = (nbm & 0xF0u) != 0;
        TF(F_WATER, s) = (int16_t)(drink ? 100 : max(0, water - 5));
        e_drink = drink;
      }
      if ((resource && ((nbm >> 8) & 255u) == M_FOILAGE) || c.prof) {
        int hh = (int)(h32((uint32_t)tile) & (kHash - 1));
        for (int probe = 0;; probe++) {  // kHash >= 2 P: never full
          if (probe == kHash) {
            tick_fault(c, NMMO_FAULT_HASH_PROBE);
            break;
          }
          const int old = atomicCAS(&c.hkey[hh], -1, tile);
          if (old == -1 || old == tile) break;
          hh = (hh + 1) & (kHash - 1);
        }
        atomicMin(&c.hmin[hh], s);
        hslot = hh;
      }
    }
  }
  if (defer) {  // the deferred bitmap into LDS, ahead of the harvest's first atomicOr
    uint4* d4 = reinterpret_cast<uint4*>(c.dep);
    if (tid < kDepU4) d4[tid] = dq.v0;
    if (tid + nt < kDepU4) d4[tid + nt] = dq.v1;
  }
  __syncthreads();
  NMMO_STAMP(3);
  // The prefetched task words are waited on here, before the tick's first global store (the
  // harvest's depletion): gfx9 counts stores in vmcnt, so waited on at the rewards, behind the
  // harvest and respawn stores, they held each tick a store round trip longer.
  if (task_early) {
    launder(tk);
    launder(tsr);
  }
  const bool first_on_tile = hslot >= 0 && c.hmin[hslot] == s;
  if (resource && first_on_tile && ((nbm >> 8) & 255u) == M_FOILAGE) {
    e_eat = true;
    TF(F_FOOD, s) = 100;
    c.mat[tile] = M_SCRUB;
    atomicOr(&c.dep[tile >> 5], 1u << (tile & 31));
  }
  if (c.prof) {
    // Professions: adjacent Fish (depleted by the lowest adjacent slot; every Fish 4-neighbour
    // of a player is depleted) then the on-tile Herb/Ore/Tree/Crystal (first on the tile).
    int fishm = 0, q_on = -1;
    bool got = false;
    if (hslot >= 0) {
      const int nb[4] = {tile - kSize, tile + kSize, tile - 1, tile + 1};
#pragma unroll
      for (int q = 0; q < 4; q++) {
        if (!((nbm >> (16 + q)) & 1u)) continue;
        fishm |= 1 << q;
        const int f = nb[q];
        const int w = min(min(hash_min(c, f - kSize), hash_min(c, f + kSize)),
                          min(hash_min(c, f - 1), hash_min(c, f + 1)));
        got = got || w == s;
      }
      if (first_on_tile) {  // (a tile eaten this tick was Foilage: no profession resource either way)
        const int m = (int)((nbm >> 8) & 255u);
        q_on = m == M_HERB ? 0 : m == M_ORE ? 1 : m == M_TREE ? 2 : m == M_CRYSTAL ? 3 : -1;
      }
    }
    int held = -1, held_lvl = 1, need = 0, n = 0;
    uint2* inv = c.inv + (s < P ? s : 0) * kInv;
    const int out_type = q_on == 0 ? T_POTION : q_on == 1 ? T_WHETSTONE : q_on == 2 ? T_ARROW : T_RUNES;
    if (got || q_on >= 0) {
      for (int k = 0; k < kInv; k++) {
        const uint2 w = inv[k];
        if (!it_type(w)) break;
        n++;
        if (it_equipped(w) && equip_slot(it_type(w)) == 3) {
          held = it_type(w);
          held_lvl = it_level(w);
        }
      }
    }
    const int lvl_f = held == T_ROD ? held_lvl : 1;
    const int lvl_on = q_on >= 0 && held == T_GLOVES + q_on ? held_lvl : 1;
    const bool new_f = got && n < kInv;
    const bool stack_on = q_on >= 0 && inv_stack(inv, out_type, lvl_on) >= 0;
    const bool new_on = q_on >= 0 && !stack_on && n + (new_f ? 1 : 0) < kInv;
    need = (new_f ? 1 : 0) + (new_on ? 1 : 0);
    int tot;
    const int pre = block_prefix_sum(need, wtot_next(c), &tot);  // rows in slot order (barriers inside)
    const int head = c.E[E_ITEM_FREE_HEAD];
    if (fishm) {
      const int nb[4] = {tile - kSize, tile + kSize, tile - 1, tile + 1};
#pragma unroll
      for (int q = 0; q < 4; q++)
        if (fishm & (1 << q)) {
          c.mat[nb[q]] = M_OCEAN;
          atomicOr(&c.dep[nb[q] >> 5], 1u << (nb[q] & 31));
        }
    }
    int ri = pre;
    if (got) {
      if (new_f) {
        const int row = c.iring[(head + ri++) % c.IC];
        inv_insert(inv, make_uint2((uint32_t)T_RATION | ((uint32_t)lvl_f << 5), 1u | ((uint32_t)row << 16)));
      }
      const int ex = TF(F_FISHING_EXP, s) + 30 * lvl_f;
      TF(F_FISHING_EXP, s) = (int16_t)ex;
      const int nl = level_at_exp(ex);
      if (nl > TF(F_FISHING_LEVEL, s)) {
        TF(F_FISHING_LEVEL, s) = (int16_t)nl;
        e_fish_nl = nl;
      }
      e_fish = lvl_f;
    }
    if (q_on >= 0) {
      const int to = q_on == 0 ? M_WEEDS : q_on == 1 ? M_SLAG : q_on == 2 ? M_STUMP : M_FRAGMENT;
      c.mat[tile] = (uint8_t)to;
      atomicOr(&c.dep[tile >> 5], 1u << (tile & 31));
      if (stack_on) {
        inv[inv_stack(inv, out_type, lvl_on)].y += 1u;
      } else if (new_on) {
        const int row = c.iring[(head + ri++) % c.IC];
        inv_insert(inv, make_uint2((uint32_t)out_type | ((uint32_t)lvl_on << 5), 1u | ((uint32_t)row << 16)));
      }
      const int fe = F_HERBALISM_EXP + 2 * q_on;
      const int ex = TF(fe, s) + (q_on == 0 ? 30 : 15) * lvl_on;
      TF(fe, s) = (int16_t)ex;
      const int nl = level_at_exp(ex);
      if (nl > TF(fe - 1, s)) {
        TF(fe - 1, s) = (int16_t)nl;
        e_on_nl = nl;
      }
      e_on_q = q_on;
      e_on_type = out_type;
      e_on_lvl = lvl_on;
    }
    __syncthreads();
    if (tid == 0 && tot) {
      c.E[E_ITEM_FREE_HEAD] = (head + tot) % c.IC;
      c.E[E_ITEM_FREE_COUNT] -= tot;
    }
  }
  // Without items the next phase that touches another slot's data or the hash's LDS is behind the
  // harvest events' scan barrier (the tile writes are read after the cull's)
  if (c.prof || items || !evon) __syncthreads();
  NMMO_STAMP(15);
  if (evon) {
    const int n = (int)e_eat + (int)e_drink + (e_fish > 0) + (e_fish_nl > 0) + (e_on_q >= 0) + (e_on_nl > 0);
    ev_append(c, evn, n, [&](int i) {
      if (e_eat) ev_put(c, i++, s, EV_EAT_FOOD, 0, 0, 0, 0, 0);
      if (e_drink) ev_put(c, i++, s, EV_DRINK_WATER, 0, 0, 0, 0, 0);
      if (e_fish) ev_put(c, i++, s, EV_HARVEST_ITEM, T_RATION, e_fish, 1, 0, 0);
      if (e_fish_nl) ev_put(c, i++, s, EV_LEVEL_UP, 4, e_fish_nl, 0, 0, 0);
      if (e_on_q >= 0) ev_put(c, i++, s, EV_HARVEST_ITEM, e_on_type, e_on_lvl, 1, 0, 0);
      if (e_on_nl) ev_put(c, i++, s, EV_LEVEL_UP, 5 + e_on_q, e_on_nl, 0, 0, 0);
    });
  }
  NMMO_STAMP(21);

  if (items) {
    // 3. Use (priority 10): own inventory only -> parallel; consumed rows freed in slot order
    int freed = -1, u_code = 0, u_type = 0, u_lvl = 0, u_num = 0;
    if (s < P && use_row >= 0 && acts(c, s)) {
      uint2* inv = c.inv + s * kInv;
      const int k = inv_find(inv, use_row);
      if (k >= 0 && !it_price(inv[k])) {
        const uint2 w = inv[k];
        const int type = it_type(w), lvl = it_level(w), slot = equip_slot(type);
        if (slot >= 0) {
          if (it_equipped(w)) {
            inv[k].x &= ~(1u << 9);
          } else if (lvl <= requirement_level(c.T, S, s, type)) {
            for (int j = 0; j < kInv; j++) {
              if (!it_type(inv[j])) break;
              if (it_equipped(inv[j]) && equip_slot(it_type(inv[j])) == slot) inv[j].x &= ~(1u << 9);
            }
            inv[k].x |= 1u << 9;
            u_code = EV_EQUIP_ITEM;
            u_type = type;
            u_lvl = lvl;
            u_num = it_qty(w);
          }
          update_item_level(c, s);
        } else if (lvl <= requirement_level(c.T, S, s, type)) {
          const int rs = 50 + 5 * lvl;
          if (type == T_RATION) {
            TF(F_FOOD, s) = (int16_t)min(100, TF(F_FOOD, s) + rs);
            TF(F_WATER, s) = (int16_t)min(100, TF(F_WATER, s) + rs);
          } else {
            TF(F_HEALTH, s) = (int16_t)min(100, TF(F_HEALTH, s) + rs);
          }
          inv[k].y -= 1u;
          u_code = EV_CONSUME_ITEM;
          u_type = type;
          u_lvl = lvl;
          u_num = 1;
          if (it_qty(inv[k]) == 0) {
            freed = it_row(w);
            inv_remove(inv, k);
          }
        }
      }
    }
    ring_ev_append(c, freed, evn, evon && u_code ? 1 : 0,
                   [&](int i) { ev_put(c, i, s, u_code, u_type, u_lvl, u_num, 0, 0); });
  NMMO_STAMP(22);

    // Buy (priority 20): buyers in shuffled order (key draw(tick, BUY_ORDER, id), ties by id).
    // A buy touches two players -- its buyer (gold, inventory room) and the listing's owner at
    // tick start (gold, inventory); a later buy of a row an earlier buy took finds it unlisted in
    // the new owner's inventory and fails, and both buys share that first owner -- so buys run
    // in rounds like the attacks: each round executes every remaining buy that is the earliest
    // (in shuffled order) remaining buy of both its players, all in parallel, which is the
    // serial result. The events (BUY_ITEM + EARN_GOLD per success) and the rows freed by
    // stacking go to the event log and the item FIFO in shuffled order: ranks by popcounts of
    // per-position bit masks.
    if (c.exch) {
      const bool isb = s < P && c.a_buy[s] >= 0;
      int nbuy;
      block_prefix_count(isb, wtot_next(c), &nbuy);
      NMMO_STAMP(28);
      if (nbuy > 0) {
        int* mi = c.ft;  // [2][S] round keys (see the attack rounds); attack init zeroes them again
        uint32_t* okm = reinterpret_cast<uint32_t*>(c.wtot + 20);  // [4] succeeded, by position
        uint32_t* frm = reinterpret_cast<uint32_t*>(c.wtot + 24);  // [4] freed a row, by position
        int16_t* frow = c.order;                                   // [128] that row, by position
        uint32_t* tgm = reinterpret_cast<uint32_t*>(c.wtot + 28);  // [4] owners of some buy's row
        int* anyf = c.wtot + 16;
        // sort keys, ~0 for the slots without a buy (up to a multiple of 4: read as uint4 below)
        if (s < ((P + 3) & ~3)) c.ikey[s] = isb ? draw(seed, (uint32_t)tick, P_BUY_ORDER, (uint32_t)(s + 1), 0).x : ~0u;
        if (tid < P) mi[tid] = mi[S + tid] = 0;
        if (tid < 12) okm[tid] = 0u;  // okm, frm and tgm
        if (tid < 3) anyf[tid] = 0;
        __syncthreads();
        int pos = 0, owner0 = -1, rm0 = -1;
        const int brow = isb ? c.a_buy[s] : -1;
        if (isb) {
          // pos = buys with a smaller (key, slot): the keys below this one, 4 per LDS read; only
          // when another slot holds the same key (a ~0 key, or a 32-bit draw collision) the
          // exact per-slot count
          const uint32_t key = c.ikey[s];
          const uint4* k4 = reinterpret_cast<const uint4*>(c.ikey);
          int eq = 0;
          for (int q4 = 0; q4 < ((P + 3) >> 2); q4++) {
            const uint4 v = k4[q4];
            pos += (v.x < key) + (v.y < key) + (v.z < key) + (v.w < key);
            eq += (v.x == key) + (v.y == key) + (v.z == key) + (v.w == key);
          }
          if (eq > 1) {
            pos = 0;
            for (int q = 0; q < P; q++)
              if (c.a_buy[q] >= 0) pos += (c.ikey[q] < key || (c.ikey[q] == key && q < s)) ? 1 : 0;
          }
          rm0 = c.rmap[brow];
          owner0 = rm0 & 255;  // a listed row at tick start (kth_listed)
        }
        bool active = isb && acts(c, s) && owner0 != s;  // the others fail without effect
        // Whether the buy would succeed on the tick-start state (no buy has run yet: every thread
        // passes round 1's barrier before any executes). A buyer whose own row no buy targets
        // keeps its gold and inventory through the phase, so if it fails now it fails at its turn.
        bool elig0 = false;
        if (active) {
          const uint2* oinv = c.inv + owner0 * kInv;
          const int k = inv_find(oinv, brow);
          if (k >= 0) {
            const uint2 w = oinv[k];
            elig0 = it_price(w) && TF(F_GOLD, s) >= it_price(w) && has_room(c, s, w);
          }
        }
        bool ok = false;
        uint2 bw = make_uint2(0u, 0u);
        int bprice = 0, bowner = -1;
        NMMO_STAMP(29);
        for (int round = 1;; round++) {
          if (round > P + 1) {  // <= nbuy rounds (the earliest pending buy runs in every round)
            if (tid == 0) tick_fault(c, NMMO_FAULT_BUY_ROUNDS);
            break;
          }
          const int key = (round << 16) | (0xFFFF - pos);
          int* mr = mi + (round & 1) * S;
          if (active) {
            atomicMax(&mr[s], key);
            atomicMax(&mr[owner0], key);
            anyf[round % 3] = 1;
            if (round == 1) atomicOr(&tgm[owner0 >> 5], 1u << (owner0 & 31));
          }
          if (tid == 0) anyf[(round + 1) % 3] = 0;
          __syncthreads();
          if (!anyf[round % 3]) break;
          // (round 1) the buys that fail on the tick-start state and whose buyer owns no bought
          // row fail at their turn too: they retire without a round of owner0's (a full
          // inventory or short gold chained one round per buyer of a popular seller)
          if (round == 1 && active && !elig0 && !((tgm[s >> 5] >> (s & 31)) & 1u)) active = false;
          // A buy whose row has left its tick-start owner fails whenever its turn comes: only a
          // buy of the same row moves it, that buy shares owner0 and so ran earlier in the order,
          // and it leaves the row unlisted. Such a buy retires now instead of taking a round of
          // owner0's (the buyers of one popular listing used to chain one round each: p99 26k
          // cycles). A row moved in this round's executions is seen now or next round.
          if (active && c.rmap[brow] != rm0 && !(mr[s] == key && mr[owner0] == key)) active = false;
          if (active && mr[s] == key && mr[owner0] == key) {
            active = false;
            const int owner = c.rmap[brow] < 0 ? -1 : (c.rmap[brow] & 255);
            uint2* oinv = c.inv + (owner >= 0 ? owner : 0) * kInv;
            const int k = owner >= 0 && owner != s ? inv_find(oinv, brow) : -1;
            if (k >= 0) {
              uint2 w = oinv[k];
              const int price = it_price(w);
              if (price && TF(F_GOLD, s) >= price && has_room(c, s, w)) {
                TF(F_GOLD, s) = (int16_t)(TF(F_GOLD, s) - price);
                TF(F_GOLD, owner) = (int16_t)(TF(F_GOLD, owner) + price);
                bw = w;
                bprice = price;
                bowner = owner;
                ok = true;
                w.x &= 0x1FFu;
                inv_remove(oinv, k);
                int freed = -1;
                c.rmap[brow] = receive_moved_deferred(c, s, w, freed) ? (int16_t)s : (int16_t)-1;
                atomicOr(&okm[pos >> 5], 1u << (pos & 31));
                if (freed >= 0) {
                  frow[pos] = (int16_t)freed;
                  atomicOr(&frm[pos >> 5], 1u << (pos & 31));
                }
              }
            }
          }
        }
        NMMO_STAMP(30);
        // (the loop's last barrier published okm / frm / frow)
        auto below = [&](const uint32_t* m) {
          int n = 0;
#pragma unroll
          for (int i = 0; i < 4; i++)
            n += i < (pos >> 5) ? __popc(m[i]) : i == (pos >> 5) ? __popc(m[i] & ((1u << (pos & 31)) - 1u)) : 0;
          return n;
        };
        const int nok = __popc(okm[0]) + __popc(okm[1]) + __popc(okm[2]) + __popc(okm[3]);
        const int nfr = __popc(frm[0]) + __popc(frm[1]) + __popc(frm[2]) + __popc(frm[3]);
        if (ok) {
          const int i = evn + 2 * below(okm);
          if (evon) {
            ev_put(c, i, s, EV_BUY_ITEM, it_type(bw), it_level(bw), it_qty(bw), bprice, 0);
            ev_put(c, i + 1, bowner, EV_EARN_GOLD, 0, 0, 0, bprice, 0);
          }
        }
        if (isb && ((frm[pos >> 5] >> (pos & 31)) & 1u))
          c.iring[(c.E[E_ITEM_FREE_HEAD] + c.E[E_ITEM_FREE_COUNT] + below(frm)) % c.IC] = frow[pos];
        if (evon) evn += 2 * nok;
        __syncthreads();
        if (tid == 0) {
          c.E[E_ITEM_FREE_COUNT] += nfr;
          c.E[E_EVENT_COUNT] = evn;
        }
        __syncthreads();
      }
    }

    NMMO_STAMP(23);
    // Give / GiveGold (priority 30), in slot order. Player p's gives touch p, its item target t
    // and its gold target t2 (inventories and gold); like the buys, they run in rounds: each
    // round executes every remaining give that is the lowest-slot remaining give of all its
    // players, all in parallel, which is the serial result. Events (GIVE_ITEM, then GIVE_GOLD per
    // player) and the rows freed by stacking go out in slot order by one prefix sum afterwards.
    {
      const bool isg = s < P && (c.a_givet[s] >= 0 || c.a_ggt[s] >= 0);
      int ng;
      block_prefix_count(isg, wtot_next(c), &ng);
      if (ng > 0) {
        int* mi = c.ft;  // [2][S] round keys (see the attack rounds); attack init zeroes them again
        int* anyf = c.wtot + 16;
        if (tid < P) mi[tid] = mi[S + tid] = 0;
        if (tid < 3) anyf[tid] = 0;
        __syncthreads();
        const int tg = isg ? c.a_givet[s] : -1, tg2 = isg ? c.a_ggt[s] : -1;
        const bool r1 = tg >= 0 && tg < P && tg != s, r2 = tg2 >= 0 && tg2 < P && tg2 != s;
        bool active = isg && acts(c, s) && (r1 || r2);  // the others fail without effect
        bool did_item = false, did_gold = false;
        uint2 gw = make_uint2(0u, 0u);
        int freed = -1;
        for (int round = 1;; round++) {
          if (round > P + 1) {  // <= ng rounds (the lowest pending give runs in every round)
            if (tid == 0) tick_fault(c, NMMO_FAULT_GIVE_ROUNDS);
            break;
          }
          const int key = (round << 16) | (0xFFFF - s);
          int* mr = mi + (round & 1) * S;
          if (active) {
            atomicMax(&mr[s], key);
            if (r1) atomicMax(&mr[tg], key);
            if (r2) atomicMax(&mr[tg2], key);
            anyf[round % 3] = 1;
          }
          if (tid == 0) anyf[(round + 1) % 3] = 0;
          __syncthreads();
          if (!anyf[round % 3]) break;
          if (active && mr[s] == key && (!r1 || mr[tg] == key) && (!r2 || mr[tg2] == key)) {
            active = false;
            if (r1 && acts(c, tg) && same_tile(c, tg, s)) {
              uint2* inv = c.inv + s * kInv;
              const int k = inv_find(inv, c.a_give[s]);
              if (k >= 0 && !it_equipped(inv[k]) && !it_price(inv[k]) && has_room(c, tg, inv[k])) {
                gw = inv[k];
                did_item = true;
                inv_remove(inv, k);
                receive_moved_deferred(c, tg, gw, freed);
              }
            }
            if (r2 && acts(c, tg2) && c.a_gga[s] <= TF(F_GOLD, s) && same_tile(c, tg2, s)) {
              TF(F_GOLD, s) = (int16_t)(TF(F_GOLD, s) - c.a_gga[s]);
              TF(F_GOLD, tg2) = (int16_t)(TF(F_GOLD, tg2) + c.a_gga[s]);
              did_gold = true;
            }
          }
        }
        // (the loop's last barrier ordered every give before these reads)
        const int fb = c.E[E_ITEM_FREE_HEAD] + c.E[E_ITEM_FREE_COUNT];
        const int nev = evon ? (int)did_item + (int)did_gold : 0;
        int tot;
        const int pre = block_prefix_sum((freed >= 0 ? 1 : 0) | nev << 16, wtot_next(c), &tot);
        if (freed >= 0) c.iring[(fb + (pre & 0xFFFF)) % c.IC] = (int16_t)freed;
        if (nev) {
          int i = evn + (pre >> 16);
          if (did_item) ev_put(c, i++, s, EV_GIVE_ITEM, it_type(gw), it_level(gw), it_qty(gw), 0, TF(F_ID, tg));
          if (did_gold) ev_put(c, i, s, EV_GIVE_GOLD, 0, 0, 0, c.a_gga[s], TF(F_ID, tg2));
        }
        evn += tot >> 16;
        if (tid == 0) {
          c.E[E_ITEM_FREE_COUNT] += tot & 0xFFFF;
          c.E[E_EVENT_COUNT] = evn;
        }
        __syncthreads();
      }
    }
    NMMO_STAMP(24);

    // Destroy (priority 40): own inventory, rows freed in slot order
    freed = -1;
    uint2 dw = make_uint2(0u, 0u);
    if (s < P && destroy_row >= 0 && acts(c, s)) {
      uint2* inv = c.inv + s * kInv;
      const int k = inv_find(inv, destroy_row);
      if (k >= 0 && !it_equipped(inv[k]) && !it_price(inv[k])) {
        freed = destroy_row;
        dw = inv[k];
        inv_remove(inv, k);
      }
    }
    ring_ev_append(c, freed, evn, evon && freed >= 0 ? 1 : 0,
                   [&](int i) { ev_put(c, i, s, EV_DESTROY_ITEM, it_type(dw), it_level(dw), it_qty(dw), 0, 0); });
  }

  NMMO_STAMP(14);
  // 3a. Attack (priority 50), in rounds. An attack (attacker slot s -> target t) touches the
  // entities {s, t}; two attacks with disjoint sets have disjoint read/write sets. Each round
  // runs every remaining attack that is the lowest-slot remaining attack on both of its
  // entities (so it follows every earlier attack it conflicts with), all in parallel; round 1
  // is all attacks no earlier attack conflicts with. The per-entity minimum is an atomicMax of
  // round << 16 | (0xFFFF - slot), so no reset between rounds is needed. The keys alternate
  // between two arrays by round parity: between barriers r and r + 1 a fast wave already bids
  // for round r + 1 while a slow one still checks round r, and with one array a check could see
  // a round-(r + 1) key, miss its turn, and -- repeated every round -- never finish (a launch
  // that hung on MI355X). A round-(r + 2) bid needs barrier r + 1, after every round-r check.
  int* mi = c.ft;
  int eq_off = 0;
  if (combat || sys(c, NMMO_SYS_NPC)) {
    for (int k = tid; k < 2 * S; k += nt) mi[k] = 0;
    if (tid < 3) c.wtot[16 + tid] = 0;  // attack-round flags
    // equipment bonuses, once (players: equipped items; NPCs: spawn-time equipment): this slot's
    // offense in its attack style (a register) and its defense (c.clist, read by its attackers)
    if (sys(c, NMMO_SYS_EQUIPMENT) && s < S) {
      const int sty0 = c.asty[s];
      eq_off = s < P ? (items ? inv_offense(c, s, sty0) : 0) : TF(F_EQUIP_OFFENSE, s);
      c.clist[s] = (int16_t)(s < P ? (items ? inv_defense(c, s) : 0) : TF(F_EQUIP_DEFENSE, s));
    }
    __syncthreads();
  }
  NMMO_STAMP(4);
  if (combat || sys(c, NMMO_SYS_NPC)) {
    // One barrier per round: pending attackers raise flag r % 3 before it, and thread 0 clears
    // flag (r + 1) % 3 -- last read in round r - 2 -- for the next round.
    int* anyf = c.wtot + 16;
    const int t = s < S ? c.atgt[s] : -1;
    bool active = inslot && t >= 0;
    const int sty = s < S ? c.asty[s] : 0;
    for (int round = 1;; round++) {
      if (round > S + 1) {  // <= attacks rounds (the lowest pending attack runs in every round)
        if (tid == 0) tick_fault(c, NMMO_FAULT_ATTACK_ROUNDS);
        break;
      }
      const int key = (round << 16) | (0xFFFF - s);
      int* mr = mi + (round & 1) * S;
      if (active) {
        atomicMax(&mr[s], key);
        atomicMax(&mr[t], key);
        anyf[round % 3] = 1;
      }
      if (tid == 0) anyf[(round + 1) % 3] = 0;
      __syncthreads();
      if (!anyf[round % 3]) break;
      if (active && mr[s] == key && mr[t] == key) {
        const int dmg = eval_attack(c, s, sty, t, eq_off, sys(c, NMMO_SYS_EQUIPMENT) ? c.clist[t] : 0);
        if (dmg >= 0) apply_attack(c, s, sty, t, dmg, tick);
        active = false;
      }
    }
  }
  NMMO_STAMP(25);
  if (evon && combat) {  // SCORE_HIT, LEVEL_UP, PLAYER_KILL per player attacker in slot order
    const int dm = s < P ? c.ev_dmg[s] : -1, lv = s < P ? c.ev_lvl[s] : 0, kv = s < P ? c.kill[s] : -1;
    ev_append(c, evn, (dm >= 0) + (lv > 0) + (kv >= 0), [&](int i) {
      const int sk = c.asty[s] + 1;
      if (dm >= 0) ev_put(c, i++, s, EV_SCORE_HIT, sk, 0, dm, 0, 0);
      if (lv > 0) ev_put(c, i++, s, EV_LEVEL_UP, sk, lv, 0, 0, 0);
      if (kv >= 0) {
        const int vl = max((int)TF(F_MELEE_LEVEL, kv), max((int)TF(F_RANGE_LEVEL, kv), (int)TF(F_MAGE_LEVEL, kv)));
        ev_put(c, i++, s, EV_PLAYER_KILL, 0, vl, 0, 0, TF(F_ID, kv));
      }
    });
  }
  NMMO_STAMP(26);
  if (items || sys(c, NMMO_SYS_EXCHANGE)) {
    // ammunition and loot of the executed player attacks, in slot order (equipment sums and
    // every attack's validity are unaffected by them, so deferring is exact). A shot touches
    // only its shooter's inventory, and a loot its killer's and victim's: the shots of players
    // no player killed this tick commute with every other shot and loot (their own loot comes
    // after their shot in both orders), so they fire in parallel; only the FIFO rows a shot
    // frees (its last unit) keep their serial place, appended by thread 0's slot-order walk
    // with the remaining shots (of victims) and the loots.
    uint32_t* victim = reinterpret_cast<uint32_t*>(c.misc);  // [16] slot bitmask (hunt mask: dead now)
    if (tid < 16) victim[tid] = 0u;
    __syncthreads();
    if (s < P && c.kill[s] >= 0) atomicOr(&victim[c.kill[s] >> 5], 1u << (c.kill[s] & 31));
    __syncthreads();
    int16_t* shot_row = c.clist;  // [S] scratch (the hostile-NPC list of the decode: dead now)
    int freed = -1;
    const bool is_victim = s < S && ((victim[s >> 5] >> (s & 31)) & 1u);
    if (s < P && c.fired[s] && !is_victim) {
      freed = fire_ammo_deferred(c, s, c.asty[s]);
      c.fired[s] = 0;  // done
    }
    if (s < P) shot_row[s] = (int16_t)freed;
    const bool nd = s < P && (c.fired[s] || c.kill[s] >= 0 || freed >= 0);
    int nn;
    const int pos = block_prefix_count(nd, wtot_next(c), &nn);
    if (nd) c.order[pos] = (int16_t)s;
    __syncthreads();
    NMMO_STAMP(27);
    if (tid == 0) {
      for (int i = 0; i < nn; i++) {
        const int x = c.order[i];
        if (shot_row[x] >= 0) ifree(c, shot_row[x]);
        if (c.fired[x]) fire_ammo(c, x, c.asty[x]);
        if (c.kill[x] >= 0) loot(c, x, c.kill[x], evn);
      }
      c.E[E_EVENT_COUNT] = evn;
    }
    __syncthreads();
    evn = c.E[E_EVENT_COUNT];
  }
  NMMO_STAMP(5);

  // 3b. Move (priority 60)
  int gf = 0;  // GO_FARTHEST record
  if (inslot && c.amove[s] >= 0 && TF(F_ALIVE, s) && TF(F_HEALTH, s) > 0) {
    const int d = c.amove[s];
    const int nr = TF(F_ROW, s) + dir_dr(d), nc = TF(F_COL, s) + dir_dc(d);
    if ((d == 4 || ((nbm >> d) & 1u)) && TF(F_FREEZE, s) <= 0) {  // d == 4: own tile
      TF(F_ROW, s) = (int16_t)nr;
      TF(F_COL, s) = (int16_t)nc;
      const int progress = 64 - linf(80, 80, nr, nc);
      if (progress > TF(F_EXPLORATION, s)) {
        TF(F_EXPLORATION, s) = (int16_t)progress;
        gf = s < P ? progress : 0;
      }
    }
  }
  // Sell (priority 70): own inventory
  uint2 sw = make_uint2(0u, 0u);
  if (c.exch && s < P && sell_row >= 0 && acts(c, s)) {
    uint2* inv = c.inv + s * kInv;
    const int k = inv_find(inv, sell_row);
    if (k >= 0 && !it_equipped(inv[k])) {
      inv[k].x = (inv[k].x & 0x3FFu) | ((uint32_t)sell_price << 10) | ((uint32_t)tick << 17);
      sw = inv[k];
    }
  }
  if (evon) {  // GO_FARTHEST (Move) events, then LIST_ITEM (Sell) events: both counts in one scan
    const int nl = it_type(sw) ? 1 : 0;
    int tot;
    const int pre = block_prefix_sum((gf > 0 ? 1 : 0) | (nl << 16), wtot_next(c), &tot);
    if (gf > 0) ev_put(c, evn + (pre & 0xFFFF), s, EV_GO_FARTHEST, 0, 0, gf, 0, 0);
    if (nl)
      ev_put(c, evn + (tot & 0xFFFF) + (pre >> 16), s, EV_LIST_ITEM, it_type(sw), it_level(sw), it_qty(sw),
             sell_price, 0);
    evn += (tot & 0xFFFF) + (tot >> 16);
  }
  // (no barrier: the cull reads only this slot's own fields, which only this thread wrote since
  // the attack rounds' last barrier)
  NMMO_STAMP(6);

  // 4. cull: rows appended to the free ring in slot order; NPC slots compacted. One prefix sum
  // places the dead slots' rows (bits 0-9), the dead players' events (10-17) and the dead
  // players' freed item rows (18-31); every thread reads the ring tails before its barrier and
  // thread 0 moves them after.
  const bool dead = inslot && TF(F_ALIVE, s) && TF(F_HEALTH, s) <= 0;
  const int ring_tail = c.E[E_FREE_HEAD] + c.E[E_FREE_COUNT];
  const int iring_tail = items ? c.E[E_ITEM_FREE_HEAD] + c.E[E_ITEM_FREE_COUNT] : 0;
  uint2* dinv = items ? c.inv + (s < P ? s : 0) * kInv : nullptr;
  const int nitem = (items && dead && s < P) ? inv_count(dinv) : 0;
  static_assert(kMaxSlots < 1024 && kInv * 128 < (1 << 14), "cull scan fields");
  int ctot;
  const int cpre = block_prefix_sum((dead ? 1 : 0) | ((dead && s < P) ? 1 << 10 : 0) | nitem << 18, wtot_next(c), &ctot);
  const int dpos = cpre & 1023, ppos = (cpre >> 10) & 255;
  const int ndead = ctot & 1023, npdead = (ctot >> 10) & 255;
  if (s < P) c.died[s] = dead ? 1 : 0;
  if (evon) {  // AGENT_CULLED in slot order (players are slots 0..P-1: the same prefix)
    if (dead && s < P) ev_put(c, evn + ppos, s, EV_AGENT_CULLED, 0, 0, 0, 0, 0);
    evn += npdead;
  }
  if (dead) {
    c.ring[(ring_tail + dpos) % S] = TF(F_DS_ROW, s);
    TF(F_ALIVE, s) = 0;
    if (s < P) TF(F_DIED_TICK, s) = (int16_t)(tick + 1);
  }
  if (nitem) {  // unlooted items of the dead are destroyed: rows freed in (slot, inventory) order
    const int base = iring_tail + (cpre >> 18);
    for (int k = 0; k < nitem; k++) {
      c.iring[(base + k) % c.IC] = (int16_t)it_row(dinv[k]);
      dinv[k] = make_uint2(0u, 0u);
    }
    TF(F_ITEM_LEVEL, s) = 0;
  }
  if (tid == 0) {
    c.E[E_FREE_COUNT] += ndead;
    c.E[E_PLAYERS_ALIVE] -= npdead;
    if (items) c.E[E_ITEM_FREE_COUNT] += ctot >> 18;
  }
  if (sys(c, NMMO_SYS_NPC) && ndead > npdead) {  // compaction only when an NPC left the realm
    const bool keep = s >= P && inslot && TF(F_ALIVE, s);
    int nkeep;
    const int kpos = block_prefix_count(keep, wtot_next(c), &nkeep);
    int16_t v[kNFLive];
    if (keep) {
#pragma unroll
      for (int row = 0; row < kNFLive; row++)
        if (row < c.nf) v[row] = c.T[row * S + s];
    }
    __syncthreads();
    if (keep) {
#pragma unroll
      for (int row = 0; row < kNFLive; row++)
        if (row < c.nf) c.T[row * S + P + kpos] = v[row];
    }
    if (s >= P + nkeep && inslot) {
#pragma unroll
      for (int row = 0; row < kNFLive; row++)
        if (row < c.nf) c.T[row * S + s] = 0;
    }
    if (tid == 0) c.E[E_NPC_COUNT] = nkeep;
  }
  __syncthreads();
  NMMO_STAMP(7);

  // 5-6. tick += 1; map.step respawn of depleted tiles; exchange.step listing expiry.
  // One Philox call serves a group of 4 consecutive tiles (SPEC §5.6). Each wave takes every
  // nwv-th chunk of 64 bitmap words, compacts the groups holding a depleted tile into its own
  // list (wave scan; in LDS space the decode bitmap no longer needs) and draws them one group
  // per lane: ~one Philox per lane instead of the busiest lane's tile count, and no block-wide
  // prefix sum or barrier. A wave whose groups overflow its list share uses the per-word loop.
  // Without the NPC system (whose spawn closes with a barrier) and with 4+ waves, the players'
  // two waves leave the respawn to the others and go on to the listing expiry and the rewards,
  // which read neither the bitmap nor (without a map-reading task, where a barrier follows) the
  // materials the draws write (same box: C2 tick 14.5 -> 14.3 us; C3 0.6 % slower with it).
  const int rskip = !sys(c, NMMO_SYS_NPC) && (nt >> 6) >= 4 && P <= 128 ? 2 : 0;
  if ((tid >> 6) >= rskip) {
    const uint8_t* base = c.bank + (size_t)c.E[E_MAP_ID] * kTiles;
    const uint32_t* base4 = reinterpret_cast<const uint32_t*>(base);  // 4 tiles per word
    // Without professions the only depletion is Foilage eaten to Scrub, so every depleted tile's
    // bank material is Foilage unless a set_state / set_map_bank installed another (c.foreign,
    // loaded at kernel start): no bank read, so the draws do not wait on HBM -- with stores in
    // flight a load's wait is a store round trip as well (gfx9 counts both in vmcnt).
    const bool foilage_only = !c.prof && !c.foreign;
    const int lane = lane_id(), wv = (tid >> 6) - rskip, nwv = (nt >> 6) - rskip;
    const int wcap = (128 * NW * 4) / nwv;                              // int16 entries per wave
    int16_t* wlist = reinterpret_cast<int16_t*>(c.vism) + wv * wcap;  // vism: dead after decode
    const uint32_t rtick = (uint32_t)(tick + 1);
    auto groups_of = [&](int w) {  // bit 4q of the result: group q of word w holds a depleted tile
      uint32_t nz = w < kBitmapWords ? c.dep[w] : 0u;
      nz |= nz >> 1;
      nz |= nz >> 2;
      return nz & 0x11111111u;
    };
    // one pass counts and lists (entries past wcap are dropped; the per-word loop then runs)
    int ng = 0;  // this wave's groups (wave-uniform)
    for (int ch = wv * 64; ch < kBitmapWords; ch += nwv * 64) {
      const int w = ch + lane;
      uint32_t nz = groups_of(w);
      const int n = __popc(nz);
      const int inc = wave_incl_scan(n);
      int k = ng + inc - n;
      ng += __builtin_amdgcn_readlane(inc, 63);
      while (nz) {
        const int b = __builtin_ctz(nz);
        nz &= nz - 1;
        if (k < wcap) wlist[k] = (int16_t)(w * 8 + (b >> 2));
        k++;
      }
    }
    NMMO_STAMP(16);
    if (ng <= wcap) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      NMMO_STAMP(18);
      // a lane's groups in batches of 4: the 4 bank words are loaded (clamped index, no branch)
      // before the first draw, so one HBM round trip serves 4 draws
      constexpr int kB = 4;
      for (int i0 = lane; i0 < ng; i0 += kB * 64) {
        int gb[kB];
        uint32_t b4[kB];
#pragma unroll
        for (int q = 0; q < kB; q++) {
          gb[q] = wlist[min(i0 + 64 * q, ng - 1)];
          b4[q] = foilage_only ? (uint32_t)M_FOILAGE * 0x01010101u : base4[gb[q]];
        }
#pragma unroll
        for (int q = 0; q < kB; q++) {
          if (i0 + 64 * q >= ng) break;
          const int g = gb[q], w = g >> 3, sh = (g & 7) * 4;
          const uint32_t nib = (c.dep[w] >> sh) & 15u;
          const U4 u = draw(seed, rtick, P_RESPAWN, (uint32_t)g, 0);
          const uint32_t uu[4] = {u.x, u.y, u.z, u.w};
          uint32_t clear = 0;
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const int bm = (int)((b4[q] >> (8 * j)) & 255u);
            if (((nib >> j) & 1u) && uu[j] < respawn_u32(bm)) {
              c.mat[4 * g + j] = (uint8_t)bm;
              clear |= 1u << (sh + j);
            }
          }
          if (clear) atomicAnd(&c.dep[w], ~clear);  // lanes may share a word
        }
      }
    } else {
      for (int ch = wv * 64; ch < kBitmapWords; ch += nwv * 64) {
        const int w = ch + lane;
        if (w >= kBitmapWords) continue;
        uint32_t bits = c.dep[w], keepb = bits;
        while (bits) {
          const int b = __builtin_ctz(bits);
          bits &= bits - 1;
          const int tt = w * 32 + b;
          const int bm = foilage_only ? (int)M_FOILAGE : base[tt];
          const U4 u = draw(seed, rtick, P_RESPAWN, (uint32_t)(tt >> 2), 0);
          const uint32_t ut = (tt & 3) == 0 ? u.x : (tt & 3) == 1 ? u.y : (tt & 3) == 2 ? u.z : u.w;
          if (ut < respawn_u32(bm)) {
            c.mat[tt] = (uint8_t)bm;
            keepb &= ~(1u << b);
          }
        }
        c.dep[w] = keepb;
      }
    }
  }
  if (!task_early) {
    tsr = c.tsg[s < P ? s : 0];
    tk = c.tasks[my_task];
  }
  if (c.exch && s < P) {
    uint2* inv = c.inv + s * kInv;
    for (int k = 0; k < kInv; k++) {
      if (!it_type(inv[k])) break;
      if (it_price(inv[k]) && tick + 1 - it_ltick(inv[k]) > 5) inv[k].x &= 0x3FFu;
    }
  }
  NMMO_STAMP(19);
  // The NPC spawn tests its tiles' passability from their tick-start materials (npc_spawn_pre),
  // and nothing else it touches (free ring, NPC slots, E) is written by the respawn or the
  // expiry: it follows the respawn without a barrier, except under foreign depletion, where it
  // reads the respawned tiles. The rewards read the respawned tiles only through CanSeeTile
  // (task_progress reads c.mat, which the respawn's other waves write): with the NPC system they
  // follow the spawn's closing barrier, without it they need this one when a task reads the map.
  if (sys(c, NMMO_SYS_NPC) ? c.foreign_any : c.tmap) __syncthreads();
  if (tid == 0) c.E[E_TICK] = tick + 1;  // read only at the tick's start (and by store_env)
  NMMO_STAMP(8);
  // 7. NPC refill
  if (sys(c, NMMO_SYS_NPC)) npc_spawn(c, (uint32_t)(tick + 1), spawn, spawn_drawn);
  NMMO_STAMP(9);

  // 8. rewards / dones (every thread evaluates `done`: E_PLAYERS_ALIVE was last written before
  // the respawn barrier)
  const int alive_n = c.E[E_PLAYERS_ALIVE];
  const bool done = alive_n == 0 || tick + 1 >= c.cfg->horizon || alive_n <= c.cfg->early_stop_agent_num;
  if (tid == 0) {
    c.E[E_DONE] = done;
    if (c.evcap) c.E[E_EVENT_COUNT] = evn;
  }
  if (c.tsee) {  // the slots' packed words for CanSeeAgent / CanSeeGroup (the union region is free here)
    uint32_t* sw = reinterpret_cast<uint32_t*>(c.ft);
    for (int k = tid; k < ((c.S + 3) & ~3); k += blockDim.x)
      sw[k] = k < c.S && TF(F_ALIVE, k) ? (uint32_t)(TF(F_DS_ROW, k) & 511) << 16 | (uint32_t)(TF(F_ROW, k) & 255) << 8 |
                                              (uint32_t)(TF(F_COL, k) & 255)
                                        : 511u << 16;
    __syncthreads();
  }
  if (s < P) {  // Task.compute_rewards: progress delta, death penalty (SPEC §12)
    float rw = 0.f;
    // the prefetched task words stay opaque until here, or the compiler hoists their conversions
    // (float weight -> double) up to the loads and waits on HBM before the respawn
    launder(tk);
    if (!c.tev) launder(tsr);
    if (c.pres[s] && c.died[s]) {
      rw = -1.f;
    } else if (c.pres[s]) {
      NmmoTaskState ts = c.tev ? c.tsl[s] : tsr;  // staged in LDS, or prefetched from HBM
      const double np = task_progress(c, s, tk, ts.acc), d = np - ts.last;
      ts.last = np;
      if (np > ts.max_progress) ts.max_progress = np;
      if (d > 0.0) ts.signals += 1;
      if (np >= 1.0 && ts.completed_tick == 0) ts.completed_tick = tick + 1;
      if (c.tev)
        c.tsl[s] = ts;
      else
        c.tsg[s] = ts;
      rw = (float)d;
    }
    rew[s] = rw;
    term[s] = c.died[s];
    trunc[s] = (uint8_t)(done && TF(F_ALIVE, s));
    mask[s] = c.pres[s];
  }
}

// The tick-fused wire count (DevState::wf): wire.hip wire_count_kernel's outputs -- per agent in
// the realm its count word (visible entities, the first kNObs, and its occupied inventory prefix),
// the env's entity-table ranks and size, its listing count and payload bytes, the packed word of
// every datastore row into wf.wpk -- computed the same way from the workgroup's LDS state after
// the store instead of from HBM by a launch of its own (C5: the count kernel was ~14 us per 512
// envs, most of it loading what the tick held). Scratch: the item ring and row map (free after the
// store) hold the packed rows, positions, shown set and prefixes; the union .. died range holds
// the id set and its prefix.
template <int kS, int kP>
__device__ __forceinline__ void wire_count_fused(Ctx& c, const DevState& st, int e) {
  static_assert(kS > 0 && kS <= kMaxSlots && kP > 0 && kP <= 128, "a specialised shape");
  auto al16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  constexpr size_t kIdBytes = (size_t)kIdWords * 4 * 2;  // ids | pre
  constexpr size_t kRegion = union_lds_bytes(kS, true) + al16((size_t)(kS + 1) * 2) + 128 * 4 + 4 * al16((size_t)kS * 2) +
                             (size_t)kBitmapWords * 4 + NMMO_NE * 4 + 32 * 4 + 16 * 4 + 128 + 128;
  static_assert(kRegion >= kIdBytes, "the id set fits the union .. died range");
  constexpr size_t kSmall = (size_t)kMaxSlots * 8 + kMaxSlots / 8 + 128 + 16 * 4 + 4;
  static_assert(kSmall <= al16((size_t)kInv * kP * 2) + al16((size_t)(kInv * kP + 1) * 2), "the item ring and row map");
  constexpr uint32_t kOut = 0xFFFFFFFFu;
  const int tid = threadIdx.x, lane = lane_id(), S = kS, P = kP;
  const int w = __builtin_amdgcn_readfirstlane(wave_id()), nw = blockDim.x >> 6;
  int nm = 0;  // store_market's listing count
  if (c.exch && tid == 0) {
    for (int j = 0; j < kLWords; j++) nm += __popcll(c.lbits[j]);
    nm = min(nm, NMMO_MARKET_ROWS);
  }
  // this thread's slot (blockDim >= S), read before the barrier that frees the scratch
  const int s = tid;
  const bool in = s < S && TF(F_ALIVE, s);
  const int ds = s < S ? TF(F_DS_ROW, s) : 0, r = s < S ? TF(F_ROW, s) : 0, col = s < S ? TF(F_COL, s) : 0;
  const int id = s < S ? TF(F_ID, s) : 0, ta = s < S ? TF(F_TIME_ALIVE, s) : 0, npc = s < S ? TF(F_NPC_TYPE, s) : 0;
  int ninv = 0;
  if (tid < P) {  // the occupied inventory prefix
    const uint2* inv = c.inv + tid * kInv;
#pragma unroll
    for (int k = kInv - 1; k >= 0; k--) ninv = it_type(inv[k]) ? ninv + 1 : 0;
  }
  __syncthreads();  // the store's LDS reads are done: the scratch below overwrites what they read
  uint32_t* pk = reinterpret_cast<uint32_t*>(c.iring);  // datastore row - 1 -> ao_pack word
  uint32_t* pos = pk + kMaxSlots;                       // slot -> row << 16 | col
  uint32_t* tab = pos + kMaxSlots;                      // slots some record shows
  uint8_t* nin = reinterpret_cast<uint8_t*>(tab + kMaxSlots / 32);
  int* wsum = reinterpret_cast<int*>(nin + 128);
  int* bytes = wsum + 16;
  uint32_t* ids = reinterpret_cast<uint32_t*>(c.vism);
  int* pre = reinterpret_cast<int*>(ids + kIdWords);
  for (int k = tid; k < kMaxSlots; k += blockDim.x) pk[k] = kOut;
  if (tid < kMaxSlots / 32) tab[tid] = 0u;
  idset_clear(ids);
  if (tid < P) nin[tid] = (uint8_t)ninv;
  if (tid == 0) *bytes = 0;
  __syncthreads();
  if (s < kMaxSlots) {
    pos[s] = in ? ((uint32_t)(uint16_t)r << 16) | (uint32_t)(uint16_t)col : kOut;
    if (in && (unsigned)(ds - 1) < (unsigned)S) {
      const bool player = s < P;
      pk[ds - 1] = ao_pack(s, r, col, player && ta < st.wf.spawn_immunity, npc > 1, player);
    }
  }
  __syncthreads();
  const WireView v = wire_view(st.wf.wire, st.wf.n_envs, P);
  uint32_t pr[kMaxSlots / 64];  // this lane's datastore rows 1 + lane + 64 i
#pragma unroll
  for (int i = 0; i < kMaxSlots / 64; i++) {
    pr[i] = pk[lane + 64 * i];
    if (w == 0) st.wf.wpk[(size_t)e * kMaxSlots + lane + 64 * i] = pr[i];
  }
  int mine = 0;
  for (int a = w; a < P; a += nw) {
    const uint32_t pa = pos[a];
    uint32_t word = 0u;
    if (pa != kOut) {  // wave-uniform
      const uint32_t rc = (pa >> 16) | (pa & 0xFFFFu) << 16;  // r | c << 16
      int nvis = 0;
#pragma unroll
      for (int i = 0; i < kMaxSlots / 64; i++) {
        const uint32_t x = pr[i];
        const bool iw = ao_in_window(x, rc);  // (an empty row is at (255, 255): outside)
        const uint64_t b = __ballot(iw);
        if (iw && nvis + __popcll(b & lanes_below()) < kNObs) {
          const int q = ao_slot(x);
          atomicOr(&tab[q >> 5], 1u << (q & 31));
        }
        nvis += __popcll(b);
      }
      word = wire_count_word(min(nvis, kNObs), nin[a]);
    }
    if (lane == 0) {
      v.cnt[(size_t)e * P + a] = (uint16_t)word;
      mine += wire_record_bytes(word);
    }
  }
  if (lane == 0) atomicAdd(bytes, mine);
  __syncthreads();
  const bool shown = s < S && ((tab[s >> 5] >> (s & 31)) & 1u);
  if (shown) idset_add(ids, id);
  const int ne = idset_prefix(ids, pre, wsum);  // (barriers inside)
  if (s < kMaxSlots) st.wf.wrank[(size_t)e * kMaxSlots + s] = shown ? (uint16_t)idrank(ids, pre, id) : (uint16_t)0xFFFF;
  if (tid == 0) {
    v.mcount[e] = (uint16_t)nm;
    v.ecount[e] = (uint16_t)ne;
    v.env_off[e] = wire_table_bytes(ne) + *bytes + 32 * nm;
  }
}

// End-of-tick listings for the obs and policy kernels (Market rows, Buy mask): ascending row.
__device__ __forceinline__ void store_market(Ctx& c, const DevState& st, int e) {
  const int tid = threadIdx.x;
  if (!c.exch) {
    if (tid == 0) st.mcount[e] = 0;
    return;
  }
  build_market(c);
  int32_t* ml = st.mlist + (size_t)e * NMMO_MARKET_ROWS;
  for (int row = tid + 1; row <= c.IC; row += blockDim.x) {
    const int w = row >> 6;
    const uint64_t m = c.lbits[w];
    if (!((m >> (row & 63)) & 1)) continue;
    int rank = __popcll(m & ((1ull << (row & 63)) - 1ull));
    for (int j = 0; j < w; j++) rank += __popcll(c.lbits[j]);
    if (rank < NMMO_MARKET_ROWS) {
      const int rm = c.rmap[row];
      ml[rank] = row | ((rm & 255) << 16) | ((rm >> 8) << 24);
    }
  }
  if (tid == 0) {
    int n = 0;
    for (int j = 0; j < kLWords; j++) n += __popcll(c.lbits[j]);
    st.mcount[e] = min(n, NMMO_MARKET_ROWS);
  }
}

// ---------------------------------------------------------------- kernel
// mode 0: step (auto-reset envs that are done); mode 1: reset every env.
// kSys != 0: specialised for exactly that system set (launch_tick dispatches on
// cfg.systems), so disabled systems compile out; kSys == 0 reads the set at run time.
template <uint32_t kSys, int kS, int kP>
__device__ __forceinline__ void tick_body(const DevState& st, const int32_t* __restrict__ actions,
                                          const uint64_t* __restrict__ env_seeds, float* rew, uint8_t* term,
                                          uint8_t* trunc, uint8_t* mask, int mode) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int e = st.env_list ? st.env_list[blockIdx.x] : (int)blockIdx.x;
  if ((unsigned)e >= (unsigned)st.n_envs) {  // a bad id of an env list: drop it, say so
    if (threadIdx.x == 0) atomicCAS(st.fault, 0, NMMO_FAULT_ENV_LIST | (int)blockIdx.x << 8);
    return;
  }
  NMMO_STAMP_CLEAR();
  NMMO_STAMP(0);
  Ctx c = make_ctx<kS, kP>(smem, st, e, kSys ? kSys : st.cfg.systems);
  // a step's action heads of this thread's player (a valid row for every thread; Move /
  // AttackStyle / AttackTarget, and the item heads with the Item system), loaded ahead of the
  // state so their latency hides under its load
  Heads hd = {};
  if (mode == 0) {
    const int32_t* a = actions + ((size_t)e * c.P + min((int)threadIdx.x, c.P - 1)) * kHeads;
#pragma unroll
    for (int k = 0; k < kHeads; k++)
      if (k == 0 || k == 1 || k == 8 || c.items) hd.v[k] = a[k];
  }
  const bool defer = defer_dep(c, kSys);
  const DepQ dq = load_env(c, st, e, kSys == NMMO_SYS_RESOURCE, defer);
  __syncthreads();
  NMMO_STAMP(20);
  const size_t o = (size_t)e * c.P;
  const bool reset_path = mode == 1 || c.E[E_DONE];
  const int alive0 = c.E[E_PLAYERS_ALIVE];  // players in the realm at tick start (sum of pres)
  const int ev_start = c.E[E_EVENT_COUNT];  // event rows this tick appends (counters[2])
  if (reset_path) {
    const int env_global = (int)(st.cfg.env_index_base + (uint64_t)e);
    uint64_t seed;
    int episode;
    if (mode == 1) {
      seed = env_seeds ? env_seeds[e] : splitmix64(st.seed ^ splitmix64((uint64_t)env_global));
      episode = 0;
    } else {
      seed = splitmix64(env_seed(c) ^ (0xD1B54A32D192ED03ull * (uint64_t)(c.E[E_EPISODE] + 1)));
      episode = c.E[E_EPISODE] + 1;
    }
    __syncthreads();
    reset_env(c, seed, episode, env_global);
    for (int i = threadIdx.x; i < c.P * (int)sizeof(NmmoTaskState) / 4; i += blockDim.x) {
      if (c.tev)  // task progress restarts with the episode
        reinterpret_cast<int*>(c.tsl)[i] = 0;
      else
        reinterpret_cast<int*>(c.tsg)[i] = 0;
    }
    if (!c.items) {  // item state is not staged in LDS without the Item system; reset it in HBM
      for (int i = threadIdx.x; i < c.P * kInv; i += blockDim.x) st.items[(size_t)e * c.P * kInv + i] = make_uint2(0u, 0u);
      for (int i = threadIdx.x; i < c.IC; i += blockDim.x) st.iring[(size_t)e * c.IC + i] = (int16_t)(i + 1);
    }
    for (int p = threadIdx.x; p < c.P; p += blockDim.x) {
      if (rew) rew[o + p] = 0.f;
      if (term) term[o + p] = 0;
      if (trunc) trunc[o + p] = 0;
      if (mask) mask[o + p] = 1;
    }
  } else {
    tick_env(c, hd, defer, dq, rew + o, term + o, trunc + o, mask + o);
  }
  __syncthreads();
  if (st.counters && threadIdx.x == 0) {  // sum(mask) of this launch + done envs + event rows, one
    // thread (no barrier; one atomic per counter and workgroup: per-wave atomics on one address
    // serialise in L2 and held C3 launches ~5 us longer). sum(mask) = the players present at
    // tick start (pres = alive = E_PLAYERS_ALIVE then), or all players on a reset.
    const bool reset = mode == 1 || reset_path;
    atomicAdd(&st.counters[0], (unsigned long long)(reset ? c.P : alive0));
    if (!reset && c.E[E_DONE]) atomicAdd(&st.counters[1], 1ull);
    if (!reset && c.evcap) atomicAdd(&st.counters[2], (unsigned long long)(c.E[E_EVENT_COUNT] - ev_start));
  }
  NMMO_STAMP(10);
  store_market(c, st, e);
  store_env(c, st, e);
  if constexpr (kSys == NMMO_SYS_ALL && kS > 0 && kP > 0)
    if (st.wf.wire) wire_count_fused<kS, kP>(c, st, e);
#ifdef NMMO_STAMPS
  __syncthreads();
#endif
  NMMO_STAMP(11);
}

// kS / kP != 0: specialised for that slot / player count too (the bench configs: C2 128 / 128,
// C3 and C4 384 / 128), so the staged arrays' LDS offsets are immediates rather than uniform values
// held across the whole tick (the generic C4 kernel spilled 960 SGPRs to VGPR lanes)
template <uint32_t kSys, int kS = 0, int kP = 0>
__global__ void tick_kernel(DevState st, const int32_t* __restrict__ actions,
                            const uint64_t* __restrict__ env_seeds, float* rew, uint8_t* term,
                            uint8_t* trunc, uint8_t* mask, int mode) {
  tick_body<kSys, kS, kP>(st, actions, env_seeds, rew, term, trunc, mask, mode);
}
// The C3 specialisation at <= 64 VGPRs: a 6-wave workgroup puts 2 waves on two SIMDs, so 4
// workgroups per CU (the 1,024 envs of C3 in one round on 256 CUs) need 8 wave slots there.
#ifndef NMMO_TICK_C3_WPE  // (A/B knob: tools/debug/variants.py)
#define NMMO_TICK_C3_WPE 8
#endif
template <uint32_t kSys, int kS = 0, int kP = 0>
__global__ void __attribute__((amdgpu_waves_per_eu(NMMO_TICK_C3_WPE, NMMO_TICK_C3_WPE)))
tick_kernel_w8(DevState st, const int32_t* __restrict__ actions, const uint64_t* __restrict__ env_seeds,
               float* rew, uint8_t* term, uint8_t* trunc, uint8_t* mask, int mode) {
  tick_body<kSys, kS, kP>(st, actions, env_seeds, rew, term, trunc, mask, mode);
}


hipError_t launch_tick(const DevState& st, const int32_t* actions, const uint64_t* env_seeds,
                       float* rew, uint8_t* term, uint8_t* trunc, uint8_t* mask, int mode,
                       hipStream_t stream) {
  // >= 8 waves: the block-wide loops (state copies, respawn draws, the wave-split phases) get two
  // waves per SIMD; slot phases leave threads >= S idle (same box: C2 tick 15.3 -> 14.9 us, C3
  // 34.9 -> 34.3, C4 58.9 -> 58.1 against >= 4 waves)
#ifndef NMMO_TICK_MIN_THREADS  // (A/B knob: tools/debug/variants.py; at most 8 waves: wtot)
#define NMMO_TICK_MIN_THREADS 512
#endif
  const int threads = max(((st.S + 63) / 64) * 64, NMMO_TICK_MIN_THREADS);
  const size_t lds = tick_lds_bytes(st.S, st.P, (st.cfg.systems & NMMO_SYS_ITEM) != 0, st.tev != 0,
                                    uses_grid(st.cfg.systems), slim_systems(st.cfg.systems));
  void (*k)(DevState, const int32_t*, const uint64_t*, float*, uint8_t*, uint8_t*, uint8_t*, int);
  const bool s128 = st.S == 128 && st.P == 128, s384 = st.S == 384 && st.P == 128;
  switch (st.cfg.systems) {
    case kSysC2: k = s128 ? tick_kernel<kSysC2, 128, 128> : tick_kernel<kSysC2>; break;
    case kSysC3: k = s384 ? tick_kernel_w8<kSysC3, 384, 128> : tick_kernel_w8<kSysC3>; break;
    case NMMO_SYS_ALL: k = s384 ? tick_kernel<NMMO_SYS_ALL, 384, 128> : tick_kernel<NMMO_SYS_ALL>; break;
    default: k = tick_kernel<0>; break;
  }
  const int grid = list_grid(st.env_list, st.n_list, st.n_envs);
  if (grid <= 0) return hipSuccess;
  hipLaunchKernelGGL(k, dim3(grid), dim3(threads), lds, stream,
                     st, actions, env_seeds, rew, term, trunc, mask, mode);
  return hipGetLastError();
}

hipError_t init_kernels() {
  // dynamic LDS may use what the kernel's static LDS leaves of 160 KB
  const void* ks[7] = {reinterpret_cast<const void*>(tick_kernel<kSysC2>),
                       reinterpret_cast<const void*>(tick_kernel_w8<kSysC3>),
                       reinterpret_cast<const void*>(tick_kernel<NMMO_SYS_ALL>),
                       reinterpret_cast<const void*>(tick_kernel<0>),
                       reinterpret_cast<const void*>(tick_kernel<kSysC2, 128, 128>),
                       reinterpret_cast<const void*>(tick_kernel_w8<kSysC3, 384, 128>),
                       reinterpret_cast<const void*>(tick_kernel<NMMO_SYS_ALL, 384, 128>)};
  for (const void* k : ks) {
    hipFuncAttributes fa;
    hipError_t err = hipFuncGetAttributes(&fa, k);
    if (err != hipSuccess) return err;
    err = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(160 * 1024 - fa.sharedSizeBytes));
    if (err != hipSuccess) return err;
  }
  return hipSuccess;
}

// set_state support: derived state is rebuilt from the blob — the depleted-tile bitmap
// (bit <=> material != bank) and the end-of-tick market list (listed rows, ascending).
__global__ void rebuild_dep_kernel(DevState st) {
  __shared__ uint64_t lbits[kLWords];
  __shared__ int16_t rmap[kInv * 128 + 1];
  const int e = blockIdx.x, tid = threadIdx.x;
  const int32_t* E = st.env + (size_t)e * NMMO_NE;
  const uint8_t* mat = st.mat + (size_t)e * kTiles;
  const uint8_t* base = st.bank + (size_t)E[E_MAP_ID] * kTiles;
  bool foreign = false;  // a depleted tile whose bank material is not Foilage (DevState::foreign)
  for (int w = tid; w < kBitmapWords; w += blockDim.x) {
    uint32_t bits = 0;
    for (int b = 0; b < 32; b++) {
      const bool d = mat[w * 32 + b] != base[w * 32 + b];
      bits |= (d ? 1u : 0u) << b;
      foreign = foreign || (d && base[w * 32 + b] != M_FOILAGE);
    }
    st.dep[(size_t)e * kBitmapWords + w] = bits;
  }
  if (__ballot(foreign) && lane_id() == 0) atomicOr(st.foreign, 1);
  if (tid < kLWords) lbits[tid] = 0;
  __syncthreads();
  const bool exch = (st.cfg.systems & NMMO_SYS_ITEM) && (st.cfg.systems & NMMO_SYS_EXCHANGE);
  if (exch && tid < st.P) {
    const uint2* inv = st.items + ((size_t)e * st.P + tid) * kInv;
    for (int k = 0; k < kInv && it_type(inv[k]); k++)
      if (it_price(inv[k])) {
        const int row = it_row(inv[k]);
        rmap[row] = (int16_t)(tid | (k << 8));
        atomicOr((unsigned long long*)&lbits[row >> 6], 1ull << (row & 63));
      }
  }
  __syncthreads();
  if (tid == 0) {
    int n = 0;
    for (int row = 1; row <= kInv * st.P; row++)
      if ((lbits[row >> 6] >> (row & 63)) & 1) {
        if (n < NMMO_MARKET_ROWS)
          st.mlist[(size_t)e * NMMO_MARKET_ROWS + n] = row | ((rmap[row] & 255) << 16) | ((rmap[row] >> 8) << 24);
        n++;
      }
    st.mcount[e] = min(n, NMMO_MARKET_ROWS);
  }
}

hipError_t launch_rebuild_dep(const DevState& st, hipStream_t stream) {
  const hipError_t err = hipMemsetAsync(st.foreign, 0, 4, stream);
  if (err != hipSuccess) return err;
  hipLaunchKernelGGL(rebuild_dep_kernel, dim3(st.n_envs), dim3(256), 0, stream, st);
  return hipGetLastError();
}

}  // namespace nmmo

#ifdef NMMO_STAMPS
extern "C" __attribute__((visibility("default"))) int nmmo_debug_read_stamps(unsigned long long* out,
                                                                              int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(nmmo::g_stamps), (size_t)n * 8, 0,
                                  hipMemcpyDeviceToHost);
}
#endif
