// obs.hip — per-agent observation gather (SPEC.md §8) and the scripted masked-uniform policy
// (SPEC.md §10).
//
// Replaces Env._compute_observations + pufferlib's flatten/pad (the buffer the reference
// receives from pool.recv(), clean_pufferl.py:293, and decodes with unpack_batched_obs,
// baseline_policy.py:41). Output: float32 [n_envs][P][23,987] in pufferlib sorted-key order.
//
// Roofline: this kernel is HBM-write-bound — 95,948 B written per agent row against ~0.3 KB of
// reads (the env's entity columns are staged once per workgroup in LDS and shared by its 16
// agents; the 225 map bytes per agent come from L2). One wave owns one agent row at a time:
// it compacts the agent's visible entities with a ballot/prefix-popcount over datastore rows
// (the nmmo window order) into LDS, then streams the row with coalesced stores — 16-byte
// stores for the long constant runs (Inventory+Market), dword stores elsewhere.
#include "kernels.h"

namespace nmmo {

constexpr int kObsAgentsPerBlock = 16;
constexpr int kObsWaves = 4;
constexpr int kObsFields = F_DS_ROW + 1;  // 0..30 obs columns, alive, ds_row

__host__ __device__ inline size_t obs_lds_bytes(int S) {
  return (((size_t)kObsFields * S * 2 + 15) & ~(size_t)15) + (((size_t)(S + 1) * 2 + 15) & ~(size_t)15) +
         (size_t)kObsWaves * 128 * 2;
}

// zero [lo, hi) of a row with 16-byte stores on the aligned body (wave-cooperative)
__device__ inline void wave_zero(float* row, int lo, int hi) {
  const int lane = lane_id();
  const uintptr_t a = reinterpret_cast<uintptr_t>(row + lo);
  int head = (int)(((16 - (a & 15)) & 15) >> 2);
  if (head > hi - lo) head = hi - lo;
  if (lane < head) row[lo + lane] = 0.f;
  const int body = (hi - lo - head) >> 2;
  float4* p4 = reinterpret_cast<float4*>(row + lo + head);
  for (int i = lane; i < body; i += 64) p4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  const int tail0 = lo + head + body * 4;
  if (tail0 + lane < hi) row[tail0 + lane] = 0.f;
}

__global__ void __launch_bounds__(256) obs_kernel(ObsParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int S = p.S;
  int16_t* T = reinterpret_cast<int16_t*>(smem);
  int16_t* rowslot = reinterpret_cast<int16_t*>(smem + (((size_t)kObsFields * S * 2 + 15) & ~(size_t)15));
  int16_t* vis_all = rowslot + ((((size_t)(S + 1) * 2 + 15) & ~(size_t)15) / 2);
  const int e = blockIdx.x, g = blockIdx.y;
  const int tid = threadIdx.x;
  {
    const int16_t* src = p.ent + (size_t)e * NMMO_NF * S;
    const int n16 = kObsFields * S;
    if ((S & 7) == 0) {
      const uint4* s4 = reinterpret_cast<const uint4*>(src);
      uint4* d4 = reinterpret_cast<uint4*>(T);
      for (int i = tid; i < n16 / 8; i += blockDim.x) d4[i] = s4[i];
    } else {
      for (int i = tid; i < n16; i += blockDim.x) T[i] = src[i];
    }
    for (int k = tid; k <= S; k += blockDim.x) rowslot[k] = -1;
  }
  __syncthreads();
  for (int s = tid; s < S; s += blockDim.x)
    if (T[F_ALIVE * S + s]) rowslot[T[F_DS_ROW * S + s]] = (int16_t)s;
  __syncthreads();

  const int lane = lane_id(), w = wave_id();
  int16_t* vis = vis_all + w * 128;
  const uint8_t* mat = p.mat + (size_t)e * kTiles;
  const int tick = p.env[(size_t)e * NMMO_NE + E_TICK];
  const bool combat = (p.systems & NMMO_SYS_COMBAT) != 0;
  for (int i = w; i < kObsAgentsPerBlock; i += kObsWaves) {
    const int a = g * kObsAgentsPerBlock + i;
    if (a >= p.P) break;
    float* row = p.obs + ((size_t)e * p.P + a) * p.elems;
    if (!T[F_ALIVE * S + a]) {
      wave_zero(row, 0, p.elems);
      continue;
    }
    const int r = T[F_ROW * S + a], c = T[F_COL * S + a];
    // Entity.Query.window: ascending datastore rows within L-inf <= 7, first 100
    int nv = 0;
    for (int base = 1; base <= S; base += 64) {
      const int k = base + lane;
      bool v = false;
      int q = -1;
      if (k <= S) {
        q = rowslot[k];
        v = q >= 0 && linf(r, c, T[F_ROW * S + q], T[F_COL * S + q]) <= kVision;
      }
      const uint64_t b = __ballot(v);
      const int pos = nv + __popcll(b & lanes_below());
      if (v && pos < kNObs) vis[pos] = (int16_t)q;
      nv += __popcll(b);
    }
    nv = min(nv, kNObs);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");

    // ActionTargets [0, o_agent_id)
    for (int j = lane; j < p.o_agent_id; j += 64) {
      float v = 0.f;
      if (j < p.o_target) {
        v = combat ? 1.f : 0.f;
      } else if (j < p.o_buy) {
        const int k = j - p.o_target;
        if (k == kNObs) v = 1.f;
        else if (combat && k < nv) {
          const int q = vis[k];
          const bool ok = q != a && linf(r, c, T[F_ROW * S + q], T[F_COL * S + q]) <= 3 &&
                          !(q < p.P && T[F_TIME_ALIVE * S + q] < p.spawn_immunity);
          v = ok ? 1.f : 0.f;
        }
      } else if (j >= p.o_move && j < p.o_sell_item) {
        const int d = j - p.o_move;
        v = impassable(mat[(r + dir_dr(d)) * kSize + c + dir_dc(d)]) ? 0.f : 1.f;
      } else {
        // noop (last) index of every other Target / InventoryItem / MarketItem mask
        v = (j == p.o_destroy - 1 || j == p.o_give_item - 1 || j == p.o_give_target - 1 ||
             j == p.o_gg_price - 1 || j == p.o_move - 1 || j == p.o_sell_price - 1 ||
             j == p.o_agent_id - 1)
                ? 1.f
                : 0.f;
      }
      row[j] = v;
    }
    if (lane == 0) row[p.o_agent_id] = (float)T[F_ID * S + a];
    if (lane == 1) row[p.o_tick] = (float)tick;
    // Entity rows (31 columns each)
    const int ne = kNObs * NMMO_N_ENTITY_COLS;
    for (int j = lane; j < ne; j += 64) {
      const int k = j / NMMO_N_ENTITY_COLS, f = j - k * NMMO_N_ENTITY_COLS;
      row[p.o_entity + j] = k < nv ? (float)T[f * S + vis[k]] : 0.f;
    }
    // Inventory + Market (v1: no items, no listings)
    wave_zero(row, p.o_inventory, p.o_task);
    for (int j = lane; j < p.task_dim; j += 64) row[p.o_task + j] = p.task[j];
    for (int j = lane; j < 225 * 3; j += 64) {
      const int t = j / 3, comp = j - 3 * t;
      const int tr = r + t / 15 - kVision, tc = c + t % 15 - kVision;
      row[p.o_tile + j] = comp == 0 ? (float)tr : comp == 1 ? (float)tc : (float)mat[tr * kSize + tc];
    }
    __builtin_amdgcn_wave_barrier();
  }
}

hipError_t launch_obs(const ObsParams& p, hipStream_t stream) {
  dim3 grid(p.n_envs, (p.P + kObsAgentsPerBlock - 1) / kObsAgentsPerBlock);
  hipLaunchKernelGGL(obs_kernel, grid, dim3(64 * kObsWaves), obs_lds_bytes(p.S), stream, p);
  return hipGetLastError();
}

// ---------------------------------------------------------------- scripted policy (SPEC §10)
// One workgroup per env, one thread per player. The env's entities are first packed per
// datastore row into one int32 (r | c<<8 | slot<<16 | immune<<25, -1 = absent), so the two
// visibility passes over the rows are one broadcast LDS load per row with no dependent loads.
__global__ void __launch_bounds__(128) policy_kernel(PolicyParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int S = p.S, e = blockIdx.x, tid = threadIdx.x;
  int* rp = reinterpret_cast<int*>(smem);  // by datastore row (row 0 unused), int4-padded
  const int16_t* E = p.ent + (size_t)e * NMMO_NF * S;
  for (int k = tid; k < rp_groups(S) * 4; k += blockDim.x) rp[k] = -1;
  __syncthreads();
  for (int s = tid; s < S; s += blockDim.x) {
    if (!E[F_ALIVE * S + s]) continue;
    const bool immune = s < p.P && E[F_TIME_ALIVE * S + s] < p.spawn_immunity;
    rp[E[F_DS_ROW * S + s]] = E[F_ROW * S + s] | (E[F_COL * S + s] << 8) | (s << 16) | ((int)immune << 25);
  }
  __syncthreads();
  const int32_t* env = p.env + (size_t)e * NMMO_NE;
  const uint8_t* mat = p.mat + (size_t)e * kTiles;
  for (int a = tid; a < p.P; a += blockDim.x) {
    int32_t* out = p.actions + ((size_t)e * p.P + a) * kHeads;
    int32_t h[kHeads] = {0, kNObs, 1024, 12, 12, kNObs, 0, kNObs, 0, 12, 0, 12};
    if (!E[F_ALIVE * S + a]) {
#pragma unroll
      for (int k = 0; k < kHeads; k++) out[k] = 0;
      continue;
    }
    const uint32_t c0 = (uint32_t)env[E_TICK] + 2048u * (uint32_t)env[E_EPISODE];
    const uint32_t c1 = (uint32_t)env[E_ENV_INDEX];
    const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
    const int r = E[F_ROW * S + a], c = E[F_COL * S + a];
    if (p.systems & NMMO_SYS_COMBAT) {
      h[0] = (int)uniform_n(philox(c0, c1, (uint32_t)a, 0, k0, k1).x, 3);
      // attack mask over the first 100 visible rows: count, draw, then select the k-th set bit
      const int4* rp4 = reinterpret_cast<const int4*>(rp);
      const int ng = rp_groups(S);
      int nb = 0, nv = 0;
      for (int g = 0; g < ng; g++) {  // pass 1: count targets among the first 100 visible
        const int4 q = rp4[g];
        const int vv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int v = vv[j];
          const int d = linf(r, c, v & 255, (v >> 8) & 255);
          const bool vis = v >= 0 && d <= kVision && nv < kNObs;
          nb += vis && ((v >> 16) & 511) != a && d <= 3 && !((v >> 25) & 1);
          nv += vis;
        }
      }
      const int pick = (int)uniform_n(philox(c0, c1, (uint32_t)a, 1, k0, k1).x, (uint32_t)(nb + 1));
      int sel = kNObs;
      if (pick < nb) {  // pass 2: visible index of the pick-th target
        int seen = 0;
        nv = 0;
        for (int g = 0; g < ng && sel == kNObs; g++) {
          const int4 q = rp4[g];
          const int vv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const int v = vv[j];
            const int d = linf(r, c, v & 255, (v >> 8) & 255);
            const bool vis = v >= 0 && d <= kVision;
            const bool ok = vis && ((v >> 16) & 511) != a && d <= 3 && !((v >> 25) & 1);
            sel = (ok && seen == pick && sel == kNObs) ? nv : sel;
            seen += ok;
            nv += vis;
          }
        }
      }
      h[1] = sel;
    }
    int mv[5], nm = 0;
#pragma unroll
    for (int d = 0; d < 5; d++)
      if (!impassable(mat[(r + dir_dr(d)) * kSize + c + dir_dc(d)])) mv[nm++] = d;
    h[8] = mv[uniform_n(philox(c0, c1, (uint32_t)a, 8, k0, k1).x, (uint32_t)nm)];
#pragma unroll
    for (int k = 0; k < kHeads; k++) out[k] = h[k];
  }
}

hipError_t launch_policy(const PolicyParams& p, hipStream_t stream) {
  const size_t lds = (size_t)rp_groups(p.S) * 16;
  hipLaunchKernelGGL(policy_kernel, dim3(p.n_envs), dim3(128), lds, stream, p);
  return hipGetLastError();
}

}  // namespace nmmo
