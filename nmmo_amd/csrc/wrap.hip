// wrap.hip — the wrapper layer (SPEC.md §13) as a device pass after the tick.
//
// Replaces the per-agent Python loop that env_creator's RewardWrapper(BaseStatWrapper) runs on
// every env step (reinforcement_learning/stat_wrapper.py:57-97: unique-event counting per agent
// through an event-log query per agent per tick, :120-126; the episode stats of :128-185 and
// process_event_log :216-293; the reward shaping of agent_zoo/*/reward_wrapper.py).
//
// One workgroup per env. Phase 1 walks only the event rows this tick appended to the env's ring
// (thread per row): every term is order-free — a per-agent fetch-or into the agent's
// `experienced` bitset in HBM returns whether the (event, type, level) tuple is new (exactly one
// row wins per tuple), counts/sums/maxima/ORs go into per-agent LDS slots with LDS atomics —
// so the parallel result is the serial one. Phase 2 (thread per agent) merges them into the
// agent's wrapper state, shapes the reward in double (explicit __dadd_rn/__dmul_rn so no FMA
// contraction differs from the oracle), and writes the episode record on the final step.
// Roofline: HBM; per env-step it reads the tick's rows (9 x 4 B each), the agents' 88-B wrapper
// states and writes them back — a few KB per env, latency-bound like the tick kernel.
#include "kernels.h"

namespace nmmo {

#ifndef NMMO_WRAP_THREADS  // (A/B knob: tools/debug/variants.py; >= 128 = the player cap)
#define NMMO_WRAP_THREADS 256  // (same box: wrapper 16.4 -> 16.0 us per 512 envs against 128)
#endif
constexpr int kWrapThreads = NMMO_WRAP_THREADS;
static_assert(kWrapThreads >= 128 && kWrapThreads % 64 == 0, "thread a owns agent a");

// event code -> dense index 0..16 (SPEC §11 code list), -1 otherwise
__host__ __device__ inline int ev_index(int code) {
  if (code >= 1 && code <= 3) return code - 1;
  if (code == 11 || code == 12) return code - 8;            // 3, 4
  if (code >= 21 && code <= 26) return code - 16;           // 5..10
  if (code >= 31 && code <= 34) return code - 20;           // 11..14
  if (code == 41) return 15;
  if (code == 91) return 16;
  return -1;
}
// ITEM_TYPE categories of stat_wrapper.py:207-213: armor, weapon, tool, ammo, consumable
__host__ __device__ inline int item_category(int type) {
  return (type >= T_HAT && type <= T_BOTTOM) ? 0 : (type >= T_SPEAR && type <= T_WAND) ? 1
         : (type >= T_ROD && type <= T_CHISEL) ? 2 : (type >= T_WHETSTONE && type <= T_RUNES) ? 3
         : (type >= T_RATION && type <= T_POTION) ? 4 : -1;
}
// performed bit of a KEY_EVENT code (stat_wrapper.py:196-205), -1 otherwise
__host__ __device__ inline int key_event_bit(int code) {
  switch (code) {
    case EV_EAT_FOOD: return 0;
    case EV_DRINK_WATER: return 1;
    case EV_SCORE_HIT: return 2;
    case EV_PLAYER_KILL: return 3;
    case EV_CONSUME_ITEM: return 4;
    case EV_HARVEST_ITEM: return 5;
    case EV_LIST_ITEM: return 6;
    case EV_BUY_ITEM: return 7;
    default: return -1;
  }
}

// entity fields phase 2 reads (skill levels/exps in nmmo skill order melee..alchemy)
enum : int {
  WF_ALIVE, WF_HEALTH_RESTORE, WF_HEALTH, WF_GOLD, WF_DAMAGE, WF_FOOD, WF_WATER, WF_LVL0,
  WF_EXP0 = WF_LVL0 + 8, kWrapFields = WF_EXP0 + 8
};
__constant__ const int kWrapField[kWrapFields] = {
    F_ALIVE, F_HEALTH_RESTORE, F_HEALTH, F_GOLD, F_DAMAGE, F_FOOD, F_WATER,
    F_MELEE_LEVEL, F_RANGE_LEVEL, F_MAGE_LEVEL, F_FISHING_LEVEL, F_HERBALISM_LEVEL,
    F_PROSPECTING_LEVEL, F_CARVING_LEVEL, F_ALCHEMY_LEVEL,
    F_MELEE_EXP, F_RANGE_EXP, F_MAGE_EXP, F_FISHING_EXP, F_HERBALISM_EXP,
    F_PROSPECTING_EXP, F_CARVING_EXP, F_ALCHEMY_EXP};

__device__ inline void ws_init(NmmoWrapState& w) {
  w.cum_reward = 0.0;
  w.prev_count = w.curr_count = 0;
  w.prev_price = 0;
  w.hp = 100;
  w.exp = 0;
  w.gold = 0;
  w.dmg_inflicted_prev = w.dmg_inflicted = 0;
  w.performed = 0;
  w.max_dist = w.earned_gold = w.max_damage = 0;
  for (int k = 0; k < 5; k++) w.max_item_level[k] = -1;
  w.agent_kills = w.npc_kills = 0;
  w.reserved = 0;
}

// mode 0: after a step / reset launch of the tick kernel (an env whose tick is 0 was reset);
// mode 1: (re)initialise every env's wrapper state (nmmo_set_wrapper).
__global__ void __launch_bounds__(kWrapThreads) wrap_kernel(WrapParams p, int mode) {
  __shared__ int cnt[128], dmg[128], maxdist[128], earned[128], maxdmg[128], ak[128], nk[128];
  __shared__ int lvl[5][128];
  __shared__ unsigned int perf[128];
  const int e = p.env_list ? p.env_list[blockIdx.x] : (int)blockIdx.x, tid = threadIdx.x, P = p.P, S = p.S;
  if ((unsigned)e >= (unsigned)p.n_envs) return;  // a bad list id (the tick records it)
  const int32_t* E = p.env + (size_t)e * NMMO_NE;
  const int tick = E[E_TICK], evc = E[E_EVENT_COUNT];
  NmmoWrapState* ws = p.ws + (size_t)e * P;
  uint32_t* uq = p.uniq + (size_t)e * P * NMMO_UNIQ_WORDS;
  NmmoAgentInfo* info = p.info + (size_t)e * P;
  if (mode == 1 || tick == 0) {  // _reset_episode_stats / _reset_reward_vars
    for (int a = tid; a < P; a += blockDim.x) {
      NmmoWrapState w;
      ws_init(w);
      ws[a] = w;
      if (info) info[a].done = 0;
    }
    uint4* u4 = reinterpret_cast<uint4*>(uq);  // P * 153 words: 16-B aligned per env when P % 4 == 0
    const int nw = P * NMMO_UNIQ_WORDS;
    if ((nw & 3) == 0 && ((reinterpret_cast<uintptr_t>(uq) & 15) == 0)) {
      for (int i = tid; i < nw / 4; i += blockDim.x) u4[i] = make_uint4(0u, 0u, 0u, 0u);
    } else {
      for (int i = tid; i < nw; i += blockDim.x) uq[i] = 0u;
    }
    if (tid == 0) p.wenv[e] = mode == 1 ? evc : 0;  // rows logged before this point are not ours
    return;
  }
  // the agent's inputs are loaded before the event walk so their latency overlaps it
  // (blockDim = 128 >= P: thread a owns agent a)
  const int a = tid;
  const bool mine = a < P;
  const size_t o = (size_t)e * P + (mine ? a : 0);
  const int16_t* T = p.ent + (size_t)e * NMMO_NF * S;
  NmmoWrapState w;
  NmmoTaskState ts;
  int f[kWrapFields];
  uint8_t present = 0, term8 = 0, trunc8 = 0;
  float raw = 0.f;
  int price = 0;
  if (mine) {
    w = ws[a];
    present = p.mask[o];
    term8 = p.term[o];
    trunc8 = p.trunc[o];
    raw = p.rew[o];
    ts = p.tstate[o];
    if (p.actions) price = p.actions[o * kHeads + 10];
#pragma unroll
    for (int k = 0; k < kWrapFields; k++) f[k] = T[kWrapField[k] * S + a];
  }
  for (int i = tid; i < 128; i += blockDim.x) {
    cnt[i] = dmg[i] = maxdist[i] = earned[i] = maxdmg[i] = ak[i] = nk[i] = 0;
    perf[i] = 0u;
    for (int k = 0; k < 5; k++) lvl[k][i] = -1;
  }
  __syncthreads();
  // phase 1: this tick's rows (env ring, SPEC §11) -> per-agent terms
  const int cap = p.evcap;
  int lo = p.wenv[e];
  if (evc - lo > cap) {  // rows the ring already overwrote are lost (event_cap too small): counted
    if (tid == 0) atomicAdd(p.wdrop, (unsigned long long)(evc - lo - cap));
    lo = evc - cap;
  }
  const int32_t* ring = p.events + (size_t)e * cap * NMMO_EVENT_COLS;
  for (int i = lo + tid; i < evc; i += blockDim.x) {
    const int32_t* r = ring + (size_t)(i % cap) * NMMO_EVENT_COLS;
    const int ag = r[1] - 1, code = r[3], type = r[4], level = r[5], num = r[6], gold = r[7], tgt = r[8];
    if (ag < 0 || ag >= P) continue;
    const int ci = ev_index(code);
    bool fresh = false;
    if (ci >= 0 && type >= 0 && type < 18 && level >= 0 && level < 16) {
      const int b = (ci * 18 + type) * 16 + level;
      const uint32_t bit = 1u << (b & 31);
      fresh = (atomicOr(&uq[ag * NMMO_UNIQ_WORDS + (b >> 5)], bit) & bit) == 0u;
    }
    if (fresh || code == EV_PLAYER_KILL || code == EV_EARN_GOLD) atomicAdd(&cnt[ag], 1);
    unsigned int pb = 0u;
    const int kb = key_event_bit(code);
    if (kb >= 0) pb |= 1u << kb;
    const int cat = item_category(type);
    if (code == EV_EQUIP_ITEM && cat >= 0 && cat < 4) pb |= 1u << (8 + cat);
    if (code == EV_HARVEST_ITEM && cat == 1) pb |= 1u << 12;
    if (pb) atomicOr(&perf[ag], pb);
    switch (code) {
      case EV_GO_FARTHEST: atomicMax(&maxdist[ag], num); break;
      case EV_EARN_GOLD: atomicAdd(&earned[ag], gold); break;
      case EV_SCORE_HIT:
        atomicMax(&maxdmg[ag], num);
        atomicAdd(&dmg[ag], num);
        break;
      case EV_PLAYER_KILL:
        if (tgt > 0) atomicAdd(&ak[ag], 1);
        if (tgt < 0) atomicAdd(&nk[ag], 1);
        break;
      default: break;
    }
    if ((code == EV_HARVEST_ITEM || code == EV_LOOT_ITEM || code == EV_BUY_ITEM) && cat >= 0)
      atomicMax(&lvl[cat][ag], level);
  }
  __syncthreads();
  // phase 2: thread per agent
  const NmmoWrapperConfig& wc = p.wc;
  if (mine) {
    // event accumulators: every row of this tick belongs to an agent present at tick start
    w.performed |= perf[a];
    w.max_dist = max(w.max_dist, maxdist[a]);
    w.earned_gold += earned[a];
    w.max_damage = max(w.max_damage, maxdmg[a]);
    for (int k = 0; k < 5; k++) w.max_item_level[k] = max(w.max_item_level[k], lvl[k][a]);
    w.agent_kills += ak[a];
    w.npc_kills += nk[a];
    w.dmg_inflicted += dmg[a];
  }
  if (mine && !present) {
    ws[a] = w;
    if (info) info[a].done = 0;
  } else if (mine) {
    w.prev_count = w.curr_count;
    w.curr_count += cnt[a];
    const bool term = term8 != 0, trunc = trunc8 != 0, done = term || trunc;
    if (!done) w.cum_reward = __dadd_rn(w.cum_reward, (double)raw);
    const bool in_realm = f[WF_ALIVE] != 0;
    double rd = (double)raw;
    if (!wc.use_custom_reward) {
      rd = term ? 0.0 : rd;
    } else if (wc.kind == NMMO_WRAP_START_KIT) {
      double heal = 0.0, explore = 0.0;
      if (wc.heal_bonus_weight > 0.0 && in_realm && f[WF_HEALTH_RESTORE] > 0) heal = wc.heal_bonus_weight;
      if (wc.explore_bonus_weight > 0.0 && w.curr_count > w.prev_count)
        explore = __dmul_rn((double)min(wc.clip_unique_event, w.curr_count - w.prev_count), wc.explore_bonus_weight);
      rd = __dadd_rn(rd, __dadd_rn(heal, explore));
    } else if (wc.kind == NMMO_WRAP_TAKERU) {
      if (!done && wc.explore_bonus_weight > 0.0 && w.curr_count > w.prev_count)
        rd = __dadd_rn(rd, __dmul_rn((double)min(wc.clip_unique_event, w.curr_count - w.prev_count),
                                     wc.explore_bonus_weight));
    } else if (wc.kind == NMMO_WRAP_YAOFENG) {
      if (!done) {
        const int hp = f[WF_HEALTH];
        const double hp_b = __dmul_rn((double)(hp - w.hp), wc.hp_bonus_weight);
        w.hp = hp;
        int xp = f[WF_EXP0];
        for (int k = 1; k < 8; k++) xp = max(xp, f[WF_EXP0 + k]);
        const double exp_b = __dmul_rn((double)(xp - w.exp), wc.exp_bonus_weight);
        w.exp = xp;
        int D = 0;
        if (p.items_on) {
          const uint2* inv = p.items + o * kInv;
          for (int k = 0; k < kInv; k++) {
            const uint2 it = inv[k];
            if (it_type(it) && it_equipped(it)) D += item_defense(it_type(it), it_level(it));
          }
        }
        const double def_b = __dmul_rn(wc.defense_bonus_weight, __ddiv_rn((double)(3 * D), 45.0));
        const double atk_b = __dmul_rn((double)(w.dmg_inflicted - w.dmg_inflicted_prev), wc.attack_bonus_weight);
        w.dmg_inflicted_prev = w.dmg_inflicted;
        const int gold = f[WF_GOLD];
        const double gold_b = __dmul_rn((double)(gold - w.gold), wc.gold_bonus_weight);
        w.gold = gold;
        const double sum = __dadd_rn(__dadd_rn(__dadd_rn(__dadd_rn(hp_b, exp_b), def_b), atk_b), gold_b);
        rd = __dadd_rn(rd, __dmul_rn(sum, wc.custom_bonus_scale));
      }
    }
    p.rew[o] = (float)rd;
    if (p.actions) w.prev_price = price;  // start kit action(): the Sell.Price index of this step
    if (info) {
      if (done) {
        NmmoAgentInfo r;
        r.done = 1;
        r.length = tick;
        r.ret = wc.eval_mode ? ts.max_progress : w.cum_reward;
        r.max_progress = ts.max_progress;
        r.reward_signal_count = ts.signals;
        r.task_completed = ts.completed_tick != 0;
        r.cod_attacked = term && f[WF_DAMAGE] > 0;
        r.cod_starved = term && f[WF_FOOD] == 0;
        r.cod_dehydrated = term && f[WF_WATER] == 0;
        r.max_combat_level = max(f[WF_LVL0], max(f[WF_LVL0 + 1], f[WF_LVL0 + 2]));
        r.max_harvest_skill_ammo = max(f[WF_LVL0 + 5], max(f[WF_LVL0 + 6], f[WF_LVL0 + 7]));
        r.max_harvest_skill_consum = max(f[WF_LVL0 + 3], f[WF_LVL0 + 4]);
        r.performed = w.performed;
        r.max_progress_to_center = w.max_dist;
        r.earned_gold = w.earned_gold;
        r.max_damage = w.max_damage;
        for (int k = 0; k < 5; k++) r.max_item_level[k] = w.max_item_level[k];
        r.agent_kill_count = w.agent_kills;
        r.npc_kill_count = w.npc_kills;
        r.unique_events = w.curr_count;
        info[a] = r;
      } else {
        info[a].done = 0;
      }
    }
    ws[a] = w;
  }
  if (tid == 0) p.wenv[e] = evc;
}

hipError_t launch_wrap(const WrapParams& p, int mode, hipStream_t stream) {
  if (p.P > 128 || p.evcap <= 0) return hipErrorInvalidValue;
  const int ne = list_grid(p.env_list, p.n_list, p.n_envs);
  if (ne <= 0) return hipSuccess;
  hipLaunchKernelGGL(wrap_kernel, dim3(ne), dim3(kWrapThreads), 0, stream, p, mode);
  return hipGetLastError();
}

}  // namespace nmmo
