// wire_obs.hip — NMMO_OBS_WIRE: the per-agent observation gather written straight as wire
// records (SPEC.md §8c), the C5 sender's obs kernel.
//
// Same observation as the native layout (SPEC §8b; `nmmo_wire_pack` of it is byte-identical,
// tests/test_gpu_wire.py), built for what a record is: ~0.3 KB per agent of bits, entity-table
// indices and a few rows, so the kernel is bound by the per-agent dependency chain, not bytes.
// Staging, window compaction and the ActionTargets bit fields are agent_obs.h's (shared with
// the native kernel); the 561-bit image is assembled with scalar ops and goes out with the head
// as one dword store, the Entity rows as u16 entity-table indices, then u16 stores for the
// Inventory rows, the 4-bit materials and the zero pad. The env's entity table (the rows some
// record shows, one 62-B row each) is written once per env from the staged columns.
// The header's count words, entity-table ranks and per-env offsets come from wire_count_kernel +
// wire_scan_kernel (wire.hip): record sizes are taken from the count words, so records never
// overlap whatever the state holds.
#include "agent_obs.h"

namespace nmmo {

// 32 agents per workgroup, 8 waves (the native kernel's 16 / 4): the per-workgroup prologue
// (entity staging, record offsets, table indices) is long next to ~0.3 KB records, so twice the
// agents per prologue: same box, 0.089 -> 0.083 ms per 512 envs, C5 at N = 1 368 -> 375 M.
#ifndef NMMO_WO_WAVES  // (A/B knobs: tools/debug/variants.py)
#define NMMO_WO_WAVES 8
#define NMMO_WO_AGENTS 32
#endif
constexpr int kWoWaves = NMMO_WO_WAVES, kWoAgents = NMMO_WO_AGENTS;

// LDS: agent_obs.h's entity staging | per-wave visible rows | per-wave window materials | the
// env's record offsets | the slots' entity-table indices. 34 KB at S = 384.
__host__ __device__ inline size_t wo_lds_bytes(int S) {
  return ao_entity_lds(S) + (size_t)kWoWaves * (128 * 4 + 256) + (size_t)(128 + 4) * 4 + (size_t)kMaxSlots * 2;
}

template <bool kWrap>
__global__ void __launch_bounds__(64 * kWoWaves) wire_obs_kernel(ObsParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int S = p.S, P = p.P, Sp = ao_stride(S);
  int16_t* T = reinterpret_cast<int16_t*>(smem);  // [31][Sp]
  uint32_t* pk = reinterpret_cast<uint32_t*>(smem + ao_entity_lds(S) - (size_t)(kMaxSlots + 64) * 4);
  uint32_t* visw_all = pk + kMaxSlots + 64;               // [kWoWaves][128] packed words of the visible rows
  uint8_t* wmat_all = reinterpret_cast<uint8_t*>(visw_all + kWoWaves * 128);  // [kWoWaves][256] window materials
  int* woff = reinterpret_cast<int*>(wmat_all + kWoWaves * 256);            // [P + 1] record offsets
  uint16_t* rk = reinterpret_cast<uint16_t*>(woff + 128 + 4);                // [kMaxSlots] table index
  int e, g;
  ao_env_group(p.n_envs, (P + kWoAgents - 1) / kWoAgents, e, g);
  const int tid = threadIdx.x, lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane(wave_id());  // wave-uniform values in SGPRs
  const WireView v = wire_view(p.wire, p.n_envs, P);
  const uint16_t* cnt = v.cnt + (size_t)e * P;
  const int ne = v.ecount[e];
  record_offsets_wave0(cnt, P, woff, wire_table_bytes(ne));
  for (int s = tid; s < kMaxSlots; s += blockDim.x) rk[s] = p.wrank[(size_t)e * kMaxSlots + s];
  ao_stage(p, e, T, pk);  // (publishes woff and rk too)

  uint8_t* wenv = p.wire + v.env_off[e];
  const int nm = min(max(p.mcount[e], 0), NMMO_MARKET_ROWS);
  if (g == 0) {  // the env's listings (Market rows), one 32-B row per thread
    uint4* mk = reinterpret_cast<uint4*>(wenv + woff[P]);
    for (int k = tid; k < nm; k += blockDim.x) {
      const int x = p.mlist[(size_t)e * NMMO_MARKET_ROWS + k];
      const int own = (x >> 16) & 255, slot = (x >> 24) & 15;
      const uint2 wd = p.items[((size_t)e * P + own) * kInv + slot];
      uint32_t q[8];
#pragma unroll
      for (int i = 0; i < 8; i++)
        q[i] = i16pack((int)item_col(wd, own + 1, 2 * i), (int)item_col(wd, own + 1, 2 * i + 1));
      mk[2 * k] = make_uint4(q[0], q[1], q[2], q[3]);
      mk[2 * k + 1] = make_uint4(q[4], q[5], q[6], q[7]);
    }
    // the entity table: the 31 columns of each shown slot at its index (a thread per slot), then
    // the table's zero pad
    int16_t* tab = reinterpret_cast<int16_t*>(wenv);
    for (int s = tid; s < S; s += blockDim.x) {
      const int x = rk[s];
      if (x == 0xFFFF) continue;
#pragma unroll
      for (int f = 0; f < NMMO_N_ENTITY_COLS; f++) tab[x * NMMO_N_ENTITY_COLS + f] = T[f * Sp + s];
    }
    for (int b = kEntRow * ne + tid; b < wire_table_bytes(ne); b += blockDim.x) wenv[b] = 0;
  }

  uint32_t pr[kAoRows];  // this lane's datastore rows 1 + lane + 64 i
#pragma unroll
  for (int i = 0; i < kAoRows; i++) pr[i] = pk[lane + 64 * i];
  uint32_t* visw = visw_all + w * 128;
  uint8_t* wmat = wmat_all + w * 256;
  if (lane < 256 - 225) wmat[225 + lane] = 0;  // materials 225.. read as zero nibbles
  const uint8_t* mat = p.mat + (size_t)e * kTiles;
  const int tick = p.env[(size_t)e * NMMO_NE + E_TICK];
  const bool item = (p.systems & NMMO_SYS_ITEM) != 0;
  const bool exch = item && (p.systems & NMMO_SYS_EXCHANGE) != 0;

  const int per_wave = (kWoAgents + kWoWaves - 1) / kWoWaves;
  const int abase = g * kWoAgents + w;
  int my_task = 0, my_prev = -1;  // lane j: agent abase + 4 j
  if (lane < per_wave && abase + kWoWaves * lane < P) {
    const size_t ai = (size_t)e * P + abase + kWoWaves * lane;
    my_task = p.assign[ai];
    if constexpr (kWrap)
      if (p.ws) my_prev = p.ws[ai].prev_price;
  }
  uint2 iv = make_uint2(0u, 0u);
  uint32_t wm[4] = {0u, 0u, 0u, 0u};
  int mo[2];
  ao_window_offsets(mo);
  auto prefetch = [&](int a) {
    const int at = T[F_ROW * Sp + a] * kSize + T[F_COL * Sp + a];
    iv = lane < kInv ? p.items[((size_t)e * P + a) * kInv + lane] : make_uint2(0u, 0u);
#pragma unroll
    for (int i = 0; i < 4; i++) wm[i] = lane + 64 * i < 225 ? mat[at + ao_window_off(mo, i)] : 0u;
  };
  auto in_realm = [&](int j) {
    const int a = abase + kWoWaves * j;
    return j < per_wave && a < P && (cnt[a] & 0x8000u);
  };
  if (in_realm(0)) prefetch(abase);

#ifdef NMMO_WO_ABLATE_LOOP  // diagnostic timing only (no records written): the prologue alone
  if (p.S != 12345) return;
#endif
  for (int j = 0; j < per_wave; j++) {
    const int a = abase + kWoWaves * j;
    if (a >= P) break;
    const uint32_t cw = (uint32_t)__builtin_amdgcn_readfirstlane((int)cnt[a]);
    if (!(cw & 0x8000u)) {  // not in the realm: no record
      if (in_realm(j + 1)) prefetch(a + kWoWaves);
      continue;
    }
    const int nv = cw & 127, ninv = (cw >> 7) & 15;
    const int r = __builtin_amdgcn_readfirstlane(T[F_ROW * Sp + a]);
    const int c = __builtin_amdgcn_readfirstlane(T[F_COL * Sp + a]);
    const int gold = __builtin_amdgcn_readfirstlane(T[F_GOLD * Sp + a]);
    const int aid = __builtin_amdgcn_readfirstlane(T[F_ID * Sp + a]);
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (lane + 64 * i < 225) wmat[lane + 64 * i] = (uint8_t)wm[i];
    const uint2 it = iv;  // this agent's item word (lanes 0..11)
    const uint32_t mv = ao_move_bits(wm[1]);
    if (in_realm(j + 1)) prefetch(a + kWoWaves);  // the next agent's loads, ahead of the stores

    ao_compact(pr, S, r, c, visw);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    AoAgent ag;
    ag.a = a;
    ag.r = r;
    ag.c = c;
    ag.gold = gold;
    ag.aid = aid;
    ag.nv = nv;
    ag.ninv = ninv;
    ag.prev_price = kWrap ? __builtin_amdgcn_readlane(my_prev, j) : -1;
    ag.mv = mv;
    uint32_t img[(kWireMaskBits + 31) / 32];  // the 561-bit image, wave-uniform
    ao_image<false>(ao_sections<kWrap>(p, T, Sp, visw, ag, it), img);
    // record: head (4 dwords) | mask image (18 + 2 zero dwords): lane i holds dword i, one store
    uint8_t* rec = wenv + woff[a];
    {
      const int task = __builtin_amdgcn_readlane(my_task, j);
      const uint32_t head[4] = {i16pack(aid, tick), i16pack(task, r - kVision), i16pack(c - kVision, nv),
                                i16pack(ninv | (exch ? 1 << 8 : 0), gold)};
      int x = 0;  // lanes 22, 23: the image's zero pad
      x = writelanes<0, 0, 4>(head, x);
      x = writelanes<4, 0, (kWireMaskBits + 31) / 32>(img, x);
      if (lane < (kWireBody >> 2)) reinterpret_cast<int*>(rec)[lane] = x;
    }
    // Entity rows: each visible row's entity-table index
    if (lane < nv) reinterpret_cast<uint16_t*>(rec + kWireBody)[lane] = rk[ao_slot(visw[lane])];
    if (lane + 64 < nv) reinterpret_cast<uint16_t*>(rec + kWireBody)[lane + 64] = rk[ao_slot(visw[lane + 64])];
    // Inventory rows | materials (4 bits, 4 per int16) | zero pad, as int16 stores
    {
      const int R = kWireBody + 2 * nv;
      const int H = (wire_record_bytes(cw) - R) >> 1;
      const int ni = 16 * ninv;
      const uint32_t* wm32 = reinterpret_cast<const uint32_t*>(wmat);
      int16_t* dst = reinterpret_cast<int16_t*>(rec + R);
      for (int h0 = 0; h0 < H; h0 += 64) {
        const int h = h0 + lane;
        const int q = min(h >> 4, kInv - 1);
        const uint2 iw = make_uint2((uint32_t)__shfl((int)it.x, q), (uint32_t)__shfl((int)it.y, q));
        int x = 0;
        if (h < ni) {
          x = (int)item_col(iw, aid, h & 15);
        } else if (h - ni < (kWireTiles + 1) / 2) {
          const uint32_t m4 = wm32[h - ni] & 0x0F0F0F0Fu;
          x = (int)((m4 & 15u) | (m4 >> 4 & 0xF0u) | (m4 >> 8 & 0xF00u) | (m4 >> 12 & 0xF000u));
        }
        if (h < H) dst[h] = (int16_t)x;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the next agent reuses visw / wmat
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// ---------------------------------------------------------------- fused: one workgroup per env
// The whole wire gather of an env in one workgroup, one kernel per launch: the env is staged
// once; its agents' window compactions give the count words, the shown slots and (by their ids)
// the entity table; the env's payload offset comes from a decoupled look-back over the
// preceding envs' payload sizes (the separate count / scan kernels re-read the state and added
// two launches); then the table, the listings and the records. An A/B with the prologue alone
// (tools/debug/variants.py wonoloop) put the three-kernel path's staging and header passes at 57%
// of its time. kWeWaves waves, kWeWaves / 128 of the agents each.
// Measured slower, so it is built only with -DNMMO_WIRE_FUSED (same box, C5, 512-env launches,
// profiles/r04/ab/ab_wire_fused.txt): 0.167 ms per launch at 16 waves, 0.222 at 8, 0.255 at 4,
// against 0.086 for count + scan + records. One workgroup per env holds the whole env's
// critical path (staging, 128 compactions, the id set's prefix, the look-back, 128 records) on
// one CU, where the record kernel spreads an env over 4 workgroups; at 16 waves LDS and VGPRs
// leave one workgroup per CU, so 512 envs run in two rounds.
#ifndef NMMO_WE_WAVES
#define NMMO_WE_WAVES 16
#endif
constexpr int kWeWaves = NMMO_WE_WAVES;
constexpr int kLookSpin = 1 << 22;  // bounded wait for a predecessor's payload size (fault beyond)
__host__ __device__ inline size_t we_lds_bytes(int S) {
  return ao_entity_lds(S) + (size_t)kWeWaves * (128 * 4 + 256) + (size_t)(128 + 4) * 4 + (size_t)kMaxSlots * 2 +
         128 * 2 + 128 + 128 + (size_t)(kMaxSlots / 32) * 4 + (size_t)kIdWords * 8 + 16 * 4 + 16;
}
// look-back word: status << 62 | value (1 = this env's payload bytes, 2 = payload bytes of envs
// 0..e inclusive)
constexpr unsigned long long kLookAgg = 1ull << 62, kLookInc = 2ull << 62, kLookVal = (1ull << 62) - 1;

template <bool kWrap>
__global__ void __launch_bounds__(64 * kWeWaves) wire_env_kernel(ObsParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int S = p.S, P = p.P, Sp = ao_stride(S);
  int16_t* T = reinterpret_cast<int16_t*>(smem);  // [31][Sp]
  uint32_t* pk = reinterpret_cast<uint32_t*>(smem + ao_entity_lds(S) - (size_t)(kMaxSlots + 64) * 4);
  uint32_t* visw_all = pk + kMaxSlots + 64;                                   // [kWeWaves][128]
  uint8_t* wmat_all = reinterpret_cast<uint8_t*>(visw_all + kWeWaves * 128);  // [kWeWaves][256]
  int* woff = reinterpret_cast<int*>(wmat_all + kWeWaves * 256);              // [P + 1] record offsets
  uint16_t* rk = reinterpret_cast<uint16_t*>(woff + 128 + 4);                 // [kMaxSlots] table index
  uint16_t* cntw = rk + kMaxSlots;                                            // [128] count words
  uint8_t* nin = reinterpret_cast<uint8_t*>(cntw + 128);                      // [128] occupied inventory prefix
  uint8_t* aliv = nin + 128;                                                  // [128] in the realm
  uint32_t* tab = reinterpret_cast<uint32_t*>(aliv + 128);                    // [kMaxSlots / 32] shown slots
  uint32_t* ids = tab + kMaxSlots / 32;                                       // [kIdWords]
  int* pre = reinterpret_cast<int*>(ids + kIdWords);                          // [kIdWords]
  int* wsum = pre + kIdWords;                                                 // [16]
  long long* shb = reinterpret_cast<long long*>(wsum + 16);                   // [2] env payload base
  const int e = blockIdx.x, tid = threadIdx.x, lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane(wave_id());
  const WireView v = wire_view(p.wire, p.n_envs, P);
  const int16_t* E = p.ent + (size_t)e * NMMO_NF * S;
  const int nm = min(max(p.mcount[e], 0), NMMO_MARKET_ROWS);

  // 1. staging: the entity columns and packed row words (ao_stage), per agent its occupied
  // inventory prefix and whether it is in the realm; the shown-slot and id sets cleared
  if (tid < P) {
    const uint2* it = p.items + ((size_t)e * P + tid) * kInv;
    uint32_t ty[kInv];
#pragma unroll
    for (int k = 0; k < kInv; k++) ty[k] = it[k].x & 31u;
    int n = 0;
#pragma unroll
    for (int k = kInv - 1; k >= 0; k--) n = ty[k] ? n + 1 : 0;
    nin[tid] = (uint8_t)n;
    aliv[tid] = E[F_ALIVE * S + tid] != 0;
  }
  if (tid < kMaxSlots / 32) tab[tid] = 0u;
  idset_clear(ids);
  ao_stage(p, e, T, pk);  // (two barriers: publishes the above too)

  // 2. count words: each wave compacts its agents' windows (the first kNObs rows in datastore
  // order), marks the shown slots
  uint32_t pr[kAoRows];  // this lane's datastore rows 1 + lane + 64 i
#pragma unroll
  for (int i = 0; i < kAoRows; i++) pr[i] = pk[lane + 64 * i];
  uint32_t* visw = visw_all + w * 128;
  for (int a = w; a < P; a += kWeWaves) {
    uint32_t word = 0u;
    if (aliv[a]) {  // wave-uniform
      const int r = T[F_ROW * Sp + a], c = T[F_COL * Sp + a];
      const int nv = min(ao_compact(pr, S, r, c, visw), kNObs);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int k = lane + 64 * h;
        if (k < nv) {
          const int q = ao_slot(visw[k]);
          atomicOr(&tab[q >> 5], 1u << (q & 31));
        }
      }
      word = wire_count_word(nv, nin[a]);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the next agent reuses visw
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (lane == 0) {
      cntw[a] = (uint16_t)word;
      v.cnt[(size_t)e * P + a] = (uint16_t)word;
    }
  }
  __syncthreads();
  // 3. the entity table: the shown slots' ids as a set, ranks by id
  bool shown[(kMaxSlots + 64 * kWeWaves - 1) / (64 * kWeWaves)];
#pragma unroll
  for (int u = 0; u < (int)(sizeof(shown) / sizeof(bool)); u++) {
    const int s = tid + 64 * kWeWaves * u;
    shown[u] = s < S && ((tab[s >> 5] >> (s & 31)) & 1u);
    if (shown[u]) idset_add(ids, T[F_ID * Sp + s]);
  }
  const int ne = idset_prefix(ids, pre, wsum);  // (barriers inside)
#pragma unroll
  for (int u = 0; u < (int)(sizeof(shown) / sizeof(bool)); u++) {
    const int s = tid + 64 * kWeWaves * u;
    if (s < kMaxSlots) rk[s] = shown[u] ? (uint16_t)idrank(ids, pre, T[F_ID * Sp + s]) : (uint16_t)0xFFFF;
  }
  record_offsets_wave0(cntw, P, woff, wire_table_bytes(ne));
  __syncthreads();
  // 4. this env's payload offset: decoupled look-back over the preceding envs' payload sizes
  // (workgroups of lower index are dispatched first, so the lowest unfinished one always runs)
  if (tid == 0) {
    const long long payload = (long long)woff[P] + 32 * nm;
    long long before = 0;
    if (e == 0) {
      __hip_atomic_store(&p.wlook[0], kLookInc | (unsigned long long)payload, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_store(&p.wlook[e], kLookAgg | (unsigned long long)payload, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      int k = e - 1, spin = 0;
      while (k >= 0) {
        const unsigned long long x = __hip_atomic_load(&p.wlook[k], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if ((x & ~kLookVal) == 0ull) {  // not published yet
          if (++spin > kLookSpin) {
            atomicCAS(p.fault, 0, NMMO_FAULT_WIRE_SCAN | e << 8);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        before += (long long)(x & kLookVal);
        if ((x & ~kLookVal) == kLookInc) break;
        k--;
      }
      __hip_atomic_store(&p.wlook[e], kLookInc | (unsigned long long)(before + payload), __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    const long long base = wire_header_bytes(p.n_envs, P) + before;
    shb[0] = base;
    v.env_off[e] = base;
    v.ecount[e] = (uint16_t)ne;
    v.mcount[e] = (uint16_t)nm;
    if (e == p.n_envs - 1) *v.total = base + payload;
  }
  if (e == p.n_envs - 1) {  // the header's zero pad
    const int64_t used = wire_header_used(p.n_envs, P);
    if (used + tid < wire_header_bytes(p.n_envs, P)) p.wire[used + tid] = 0;
  }
  __syncthreads();
  uint8_t* wenv = p.wire + shb[0];
  // 5. listings (one 32-B row per thread), the entity table (a thread per shown slot) and its pad
  {
    uint4* mk = reinterpret_cast<uint4*>(wenv + woff[P]);
    for (int k = tid; k < nm; k += blockDim.x) {
      const int x = p.mlist[(size_t)e * NMMO_MARKET_ROWS + k];
      const int own = (x >> 16) & 255, slot = (x >> 24) & 15;
      const uint2 wd = p.items[((size_t)e * P + own) * kInv + slot];
      uint32_t q[8];
#pragma unroll
      for (int i = 0; i < 8; i++)
        q[i] = i16pack((int)item_col(wd, own + 1, 2 * i), (int)item_col(wd, own + 1, 2 * i + 1));
      mk[2 * k] = make_uint4(q[0], q[1], q[2], q[3]);
      mk[2 * k + 1] = make_uint4(q[4], q[5], q[6], q[7]);
    }
    int16_t* tabw = reinterpret_cast<int16_t*>(wenv);
    for (int s = tid; s < S; s += blockDim.x) {
      const int x = rk[s];
      if (x == 0xFFFF) continue;
#pragma unroll
      for (int f = 0; f < NMMO_N_ENTITY_COLS; f++) tabw[x * NMMO_N_ENTITY_COLS + f] = T[f * Sp + s];
    }
    for (int b = kEntRow * ne + tid; b < wire_table_bytes(ne); b += blockDim.x) wenv[b] = 0;
  }
  // 6. the records (wire_obs_kernel's per-agent body)
  uint8_t* wmat = wmat_all + w * 256;
  if (lane < 256 - 225) wmat[225 + lane] = 0;  // materials 225.. read as zero nibbles
  const uint8_t* mat = p.mat + (size_t)e * kTiles;
  const int tick = p.env[(size_t)e * NMMO_NE + E_TICK];
  const bool exch = (p.systems & NMMO_SYS_ITEM) && (p.systems & NMMO_SYS_EXCHANGE);
  constexpr int per_wave = (128 + kWeWaves - 1) / kWeWaves;
  int my_task = 0, my_prev = -1;  // lane j: agent w + kWeWaves j
  if (lane < per_wave && w + kWeWaves * lane < P) {
    const size_t ai = (size_t)e * P + w + kWeWaves * lane;
    my_task = p.assign[ai];
    if constexpr (kWrap)
      if (p.ws) my_prev = p.ws[ai].prev_price;
  }
  uint2 iv = make_uint2(0u, 0u);
  uint32_t wm[4] = {0u, 0u, 0u, 0u};
  int mo[2];
  ao_window_offsets(mo);
  auto prefetch = [&](int a) {
    const int at = T[F_ROW * Sp + a] * kSize + T[F_COL * Sp + a];
    iv = lane < kInv ? p.items[((size_t)e * P + a) * kInv + lane] : make_uint2(0u, 0u);
#pragma unroll
    for (int i = 0; i < 4; i++) wm[i] = lane + 64 * i < 225 ? mat[at + ao_window_off(mo, i)] : 0u;
  };
  auto in_realm = [&](int j) {
    const int a = w + kWeWaves * j;
    return j < per_wave && a < P && (cntw[a] & 0x8000u);
  };
  if (in_realm(0)) prefetch(w);
  for (int j = 0; j < per_wave; j++) {
    const int a = w + kWeWaves * j;
    if (a >= P) break;
    const uint32_t cw = (uint32_t)__builtin_amdgcn_readfirstlane((int)cntw[a]);
    if (!(cw & 0x8000u)) {  // not in the realm: no record
      if (in_realm(j + 1)) prefetch(a + kWeWaves);
      continue;
    }
    const int nv = cw & 127, ninv = (cw >> 7) & 15;
    const int r = __builtin_amdgcn_readfirstlane(T[F_ROW * Sp + a]);
    const int c = __builtin_amdgcn_readfirstlane(T[F_COL * Sp + a]);
    const int gold = __builtin_amdgcn_readfirstlane(T[F_GOLD * Sp + a]);
    const int aid = __builtin_amdgcn_readfirstlane(T[F_ID * Sp + a]);
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (lane + 64 * i < 225) wmat[lane + 64 * i] = (uint8_t)wm[i];
    const uint2 it = iv;  // this agent's item word (lanes 0..11)
    const uint32_t mv = ao_move_bits(wm[1]);
    if (in_realm(j + 1)) prefetch(a + kWeWaves);  // the next agent's loads, ahead of the stores

    ao_compact(pr, S, r, c, visw);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    AoAgent ag;
    ag.a = a;
    ag.r = r;
    ag.c = c;
    ag.gold = gold;
    ag.aid = aid;
    ag.nv = nv;
    ag.ninv = ninv;
    ag.prev_price = kWrap ? __builtin_amdgcn_readlane(my_prev, j) : -1;
    ag.mv = mv;
    uint32_t img[(kWireMaskBits + 31) / 32];  // the 561-bit image, wave-uniform
    ao_image<false>(ao_sections<kWrap>(p, T, Sp, visw, ag, it), img);
    uint8_t* rec = wenv + woff[a];
    {
      const int task = __builtin_amdgcn_readlane(my_task, j);
      const uint32_t head[4] = {i16pack(aid, tick), i16pack(task, r - kVision), i16pack(c - kVision, nv),
                                i16pack(ninv | (exch ? 1 << 8 : 0), gold)};
      int x = 0;  // lanes 22, 23: the image's zero pad
      x = writelanes<0, 0, 4>(head, x);
      x = writelanes<4, 0, (kWireMaskBits + 31) / 32>(img, x);
      if (lane < (kWireBody >> 2)) reinterpret_cast<int*>(rec)[lane] = x;
    }
    if (lane < nv) reinterpret_cast<uint16_t*>(rec + kWireBody)[lane] = rk[ao_slot(visw[lane])];
    if (lane + 64 < nv) reinterpret_cast<uint16_t*>(rec + kWireBody)[lane + 64] = rk[ao_slot(visw[lane + 64])];
    {
      const int R = kWireBody + 2 * nv;
      const int H = (wire_record_bytes(cw) - R) >> 1;
      const int ni = 16 * ninv;
      const uint32_t* wm32 = reinterpret_cast<const uint32_t*>(wmat);
      int16_t* dst = reinterpret_cast<int16_t*>(rec + R);
      for (int h0 = 0; h0 < H; h0 += 64) {
        const int h = h0 + lane;
        const int q = min(h >> 4, kInv - 1);
        const uint2 iw = make_uint2((uint32_t)__shfl((int)it.x, q), (uint32_t)__shfl((int)it.y, q));
        int x = 0;
        if (h < ni) {
          x = (int)item_col(iw, aid, h & 15);
        } else if (h - ni < (kWireTiles + 1) / 2) {
          const uint32_t m4 = wm32[h - ni] & 0x0F0F0F0Fu;
          x = (int)((m4 & 15u) | (m4 >> 4 & 0xF0u) | (m4 >> 8 & 0xF00u) | (m4 >> 12 & 0xF000u));
        }
        if (h < H) dst[h] = (int16_t)x;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the next agent reuses visw / wmat
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

hipError_t launch_wire_obs(const ObsParams& p, hipStream_t stream) {
  if (p.S % 8 || p.S > kMaxSlots || p.P > 128 || !p.wire) return hipErrorInvalidValue;
  if (!ao_layout_ok(p)) return hipErrorInvalidValue;  // the wire format's fixed sections
#ifndef NMMO_WIRE_FUSED  // the three-kernel path (the fused one-kernel path is an A/B variant)
  const hipError_t err = launch_wire_header(p, stream);  // count words, sizes, offsets
  if (err != hipSuccess) return err;
  const dim3 grid(p.n_envs * ((p.P + kWoAgents - 1) / kWoAgents)), block(64 * kWoWaves);  // ao_env_group
  const size_t lds = wo_lds_bytes(p.S);
  if (p.wflags) hipLaunchKernelGGL(wire_obs_kernel<true>, grid, block, lds, stream, p);
  else hipLaunchKernelGGL(wire_obs_kernel<false>, grid, block, lds, stream, p);
#else
  if (!p.wlook || !p.fault) return hipErrorInvalidValue;
  const hipError_t err = hipMemsetAsync(p.wlook, 0, (size_t)p.n_envs * 8, stream);
  if (err != hipSuccess) return err;
  const size_t lds = we_lds_bytes(p.S);
  if (p.wflags) hipLaunchKernelGGL(wire_env_kernel<true>, dim3(p.n_envs), dim3(64 * kWeWaves), lds, stream, p);
  else hipLaunchKernelGGL(wire_env_kernel<false>, dim3(p.n_envs), dim3(64 * kWeWaves), lds, stream, p);
#endif
  return hipGetLastError();
}

}  // namespace nmmo
