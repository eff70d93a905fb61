// wire_obs.hip — NMMO_OBS_WIRE: the per-agent observation gather written straight as wire
// records (SPEC.md §8c), the C5 sender's obs kernel.
//
// Same observation as the native layout (SPEC §8b; `nmmo_wire_pack` of it is byte-identical,
// tests/test_gpu_wire.py), built for what a record is: ~0.3 KB per agent of bits, entity-table
// indices and a few rows, so the kernel is bound by the per-agent dependency chain, not bytes.
// Window compaction (over wire_count_kernel's packed row words) and the ActionTargets bit fields
// are agent_obs.h's (shared with the native kernel); the head (with the Style / Move / GoldPrice /
// SellPrice sections folded into two of its words) goes out as one dword store, the Entity rows as
// u16 entity-table indices, then u16 stores for the Inventory rows, the 4-bit materials, the
// mask bit stream (3 nv + 4 ninv bits from ballots) and the zero pad. The env's entity table (the rows some
// record shows, one 62-B row each) is written once per env from the columns in HBM.
// The header's count words, entity-table ranks and per-env offsets come from wire_count_kernel +
// wire_scan_kernel (wire.hip): record sizes are taken from the count words, so records never
// overlap whatever the state holds.
#include "agent_obs.h"

namespace nmmo {

// 16 agents per workgroup, 4 waves. Round 3 (each workgroup staging the env's 24 KB of
// columns) took 32 agents / 8 waves to amortise that prologue (0.089 -> 0.083 ms per 512 envs);
// without the staging, 16 / 4 is faster again (same box: 0.0797 vs 0.0835 ms; 64 / 8 0.086,
// profiles/r04/ab/ab_wire_nostage.txt).
#ifndef NMMO_WO_WAVES  // (A/B knobs: tools/debug/variants.py)
#define NMMO_WO_WAVES 4
#define NMMO_WO_AGENTS 16
#endif
constexpr int kWoWaves = NMMO_WO_WAVES, kWoAgents = NMMO_WO_AGENTS;

// LDS: the workgroup's agents' 31 Entity columns | per-wave visible rows | per-wave window
// materials | the env's record offsets | the slots' entity-table indices. 9.6 KB.
// The env's other slots are read only as wire_count_kernel's packed row words (p.wpk: slot, row,
// col, flags), loaded straight into registers, and the entity table (workgroup 0) is written from
// the columns in HBM: the kernel used to stage all 24 KB of the env's columns in LDS per
// workgroup, once for each of an env's 4 workgroups, and that prologue was over half its time.
// + the workgroup's staged window rows and item words (agent_obs.h ao_stage_windows): 15.9 KB.
__host__ __device__ inline size_t wo_lds_bytes() {
  return (size_t)NMMO_N_ENTITY_COLS * kWoAgents * 2 + (size_t)kWoWaves * (128 * 4 + 256) + (size_t)(128 + 4) * 4 +
         (size_t)kMaxSlots * 2 + ao_win_lds();
}
static_assert(kWoAgents == kAoAgents, "ao_stage_windows stages kAoAgents agents per workgroup");

#ifndef NMMO_WO_STAMPS  // diagnostic: s_memtime per wave phase and per record section (tools/debug/wo_stamps.py)
#define NMMO_WO_STAMPS 0
#endif
#if NMMO_WO_STAMPS
constexpr int kWoStamps = 6;  // record: start, window materials, compaction, sections, stream, stores
__device__ uint64_t wo_stamp_buf[1 << 17][kWoStamps];
__device__ uint64_t wo_wave_buf[1 << 15][6];  // wave: start, prologue, windows, loop, end, env | records << 32
#define WO_STAMP(arr, k) arr[k] = __builtin_amdgcn_s_memtime()
#else
#define WO_STAMP(arr, k) \
  do {                   \
  } while (0)
#endif
template <bool kWrap>
__global__ void __launch_bounds__(64 * kWoWaves) wire_obs_kernel(ObsParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
#if NMMO_WO_STAMPS
  uint64_t wv_[6], rs_[kWoStamps];
  int nrec = 0;
  WO_STAMP(wv_, 0);
#endif
  const int S = p.S, P = p.P;
  constexpr int Sp = kWoAgents;  // T's stride: column f of the workgroup's agent la at T[f * Sp + la]
  int16_t* T = reinterpret_cast<int16_t*>(smem);  // [31][kWoAgents]
  uint32_t* visw_all = reinterpret_cast<uint32_t*>(T + NMMO_N_ENTITY_COLS * kWoAgents);  // [kWoWaves][128] packed words of the visible rows
  uint8_t* wmat_all = reinterpret_cast<uint8_t*>(visw_all + kWoWaves * 128);  // [kWoWaves][256] window materials
  int* woff = reinterpret_cast<int*>(wmat_all + kWoWaves * 256);            // [P + 1] record offsets
  uint16_t* rk = reinterpret_cast<uint16_t*>(woff + 128 + 4);                // [kMaxSlots] table index
  uint32_t* wst = reinterpret_cast<uint32_t*>(rk + kMaxSlots);                 // [16][15][5] window rows
  uint2* ist = reinterpret_cast<uint2*>(wst + kAoAgents * kAoWinAgentBytes / 4);  // [16][12] item words
  int e, g;
  ao_env_group(p.n_envs, (P + kWoAgents - 1) / kWoAgents, e, g);
  const int tid = threadIdx.x, lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane(wave_id());  // wave-uniform values in SGPRs
  const WireView v = wire_view(p.wire, p.n_envs, P);
  const uint16_t* cnt = v.cnt + (size_t)e * P;
  const int ne = v.ecount[e];
  const int a0 = g * kWoAgents;  // the workgroup's first agent
  const int16_t* E = p.ent + (size_t)e * NMMO_NF * S;
  // Every global load of the kernel is issued here or in the agent loop's prefetch, ahead of any
  // store (vmcnt counts stores too and retires in issue order: a load after a store waits for
  // it). Lane j of a wave holds its agent abase + kWoWaves j's count word, task and last price.
  int my_task = 0, my_prev = -1, my_cnt = 0;
  uint2 my_rec = make_uint2(0u, 0u);  // its step record (nmmo_set_step_records), stored after the loop
  const int my_a = g * kWoAgents + wave_id() + kWoWaves * lane;
  const bool my_on = lane < (kWoAgents + kWoWaves - 1) / kWoWaves && my_a < P;
  {
    if (my_on) {
      const size_t ai = (size_t)e * P + my_a;
      my_cnt = cnt[my_a];
      my_task = p.assign[ai];
      if constexpr (kWrap)
        if (p.ws) my_prev = p.ws[ai].prev_price;
      if (p.recs)  // reward | term | trunc | mask | 0
        my_rec = make_uint2(__float_as_uint(p.rew[ai]),
                            (uint32_t)p.term[ai] | (uint32_t)p.trunc[ai] << 8 | (uint32_t)p.mask[ai] << 16);
    }
  }
  const int tick = p.env[(size_t)e * NMMO_NE + E_TICK];
  uint8_t* const wenv = p.wire + v.env_off[e];
  // the table ranks and the agents' columns: every load of the thread before its LDS writes
  constexpr int kRk = (kMaxSlots + 64 * kWoWaves - 1) / (64 * kWoWaves);
  constexpr int kTc = (NMMO_N_ENTITY_COLS * kWoAgents + 64 * kWoWaves - 1) / (64 * kWoWaves);
  uint16_t rkv[kRk];
  int16_t tcv[kTc];
#pragma unroll
  for (int k = 0; k < kRk; k++) {
    const int sl = tid + 64 * kWoWaves * k;
    rkv[k] = sl < kMaxSlots ? p.wrank[(size_t)e * kMaxSlots + sl] : (uint16_t)0;
  }
#pragma unroll
  for (int k = 0; k < kTc; k++) {
    const int i = tid + 64 * kWoWaves * k, f = i / kWoAgents, la = i - f * kWoAgents;
    tcv[k] = i < NMMO_N_ENTITY_COLS * kWoAgents && a0 + la < P ? E[f * S + a0 + la] : (int16_t)0;
  }
  record_offsets_wave0(cnt, P, woff, wire_table_bytes(ne));
#pragma unroll
  for (int k = 0; k < kRk; k++)
    if (tid + 64 * kWoWaves * k < kMaxSlots) rk[tid + 64 * kWoWaves * k] = rkv[k];
#pragma unroll
  for (int k = 0; k < kTc; k++)
    if (tid + 64 * kWoWaves * k < NMMO_N_ENTITY_COLS * kWoAgents) T[tid + 64 * kWoWaves * k] = tcv[k];
  uint32_t pr[kAoRows];  // this lane's datastore rows 1 + lane + 64 i
#pragma unroll
  for (int i = 0; i < kAoRows; i++) pr[i] = p.wpk[(size_t)e * kMaxSlots + lane + 64 * i];
  __syncthreads();
  // the workgroup's window rows and item words into LDS (T is per workgroup: agent a at a - a0),
  // so the agent loop issues no global load: an in-loop prefetch after the previous record's
  // stores waited for them (vmcnt retires in order)
#if NMMO_WO_STAMPS
  WO_STAMP(wv_, 1);
#endif
  ao_stage_windows(p, e, g, T - a0, Sp, wst, ist);  // (barrier inside)
#if NMMO_WO_STAMPS
  WO_STAMP(wv_, 2);
#endif
  const uint8_t* wsb = reinterpret_cast<const uint8_t*>(wst);

  uint32_t* visw = visw_all + w * 128;
  uint8_t* wmat = wmat_all + w * 256;
  if (lane < 256 - 225) wmat[225 + lane] = 0;  // materials 225.. read as zero nibbles
  const bool item = (p.systems & NMMO_SYS_ITEM) != 0;
  const bool exch = item && (p.systems & NMMO_SYS_EXCHANGE) != 0;

  const int per_wave = (kWoAgents + kWoWaves - 1) / kWoWaves;
  const int abase = g * kWoAgents + w;
  int wo[2];
  ao_win_offsets(wo);

#ifdef NMMO_WO_ABLATE_LOOP  // diagnostic timing only (no records written): the prologue alone
  if (p.S != 12345) return;
#endif
  for (int j = 0; j < per_wave; j++) {
    const int a = abase + kWoWaves * j;
    if (a >= P) break;
    const uint32_t cw = (uint32_t)__builtin_amdgcn_readlane(my_cnt, j);
    if (!(cw & 0x8000u)) continue;  // not in the realm: no record
    const int nv = cw & 127, ninv = (cw >> 7) & 15;
    const int la = a - a0;
    const int r = __builtin_amdgcn_readfirstlane(T[F_ROW * Sp + la]);
    const int c = __builtin_amdgcn_readfirstlane(T[F_COL * Sp + la]);
    const int gold = __builtin_amdgcn_readfirstlane(T[F_GOLD * Sp + la]);
    const int aid = __builtin_amdgcn_readfirstlane(T[F_ID * Sp + la]);
    const uint8_t* wa = wsb + la * kAoWinAgentBytes + ((c - kVision) & 3);
    uint32_t wm[4];
#pragma unroll
    for (int i = 0; i < 4; i++) wm[i] = lane + 64 * i < 225 ? wa[ao_win_off(wo, i)] : 0u;
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (lane + 64 * i < 225) wmat[lane + 64 * i] = (uint8_t)wm[i];
    const uint2 it = lane < kInv ? ist[la * kInv + lane] : make_uint2(0u, 0u);  // lanes 0..11
    const uint32_t mv = ao_move_bits(wm[1]);

#if NMMO_WO_STAMPS
    WO_STAMP(rs_, 0);
    asm volatile("" ::"v"(wm[0]), "v"(wm[3]));
    WO_STAMP(rs_, 1);
#endif
    ao_compact(pr, S, r, c, visw);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    AoAgent ag;
    ag.a = a;
    ag.ti = a - a0;
    ag.r = r;
    ag.c = c;
    ag.gold = gold;
    ag.aid = aid;
    ag.nv = nv;
    ag.ninv = ninv;
    ag.prev_price = kWrap ? __builtin_amdgcn_readlane(my_prev, j) : -1;
    ag.mv = mv;
    // the ActionTargets as what they are made of (wire.h v4): head words m5 / m6 and a bit stream
    // of the first nv entries of the 3 target sections and the first ninv of the 4 inventory ones
#if NMMO_WO_STAMPS
    WO_STAMP(rs_, 2);
#endif
    const AoSections x = ao_sections<kWrap>(p, T, Sp, visw, ag, it);
#if NMMO_WO_STAMPS
    asm volatile("" ::"s"(x.s0), "s"(x.s3));
    WO_STAMP(rs_, 3);
#endif
    int pp1 = 0;  // 1 + the SellPrice entry the wrapper cleared
    if (exch) {
      const uint64_t z0 = ~x.s10[0], z1 = ~x.s10[1] & low_bits(kSecN[10] - 64);
      pp1 = z0 ? __builtin_ctzll(z0) + 1 : z1 ? 65 + __builtin_ctzll(z1) : 0;
    }
    const int ng = __popcll(x.s6[0]) + __popcll(x.s6[1]);
    const int B = 3 * nv + 4 * ninv;  // stream bits
    uint64_t W[6];                    // the stream, 64 bits per word (B <= 348)
#pragma unroll
    for (int q = 0; q < 6; q++) W[q] = 0ull;
    if (B <= 64) {  // the common case (nv <= 21 with ninv <= 0, ...): one word, scalar shifts and ors
      const uint64_t mv = low_bits(nv), mi = low_bits(ninv);
      const int o = 3 * nv;
      W[0] = (x.s1[0] & mv) | (x.s5[0] & mv) << nv | (x.s7[0] & mv) << (2 * nv) | (x.s3 & mi) << o |
             (x.s4 & mi) << (o + ninv) | (x.s9 & mi) << (o + 2 * ninv) | (x.s11 & mi) << (o + 3 * ninv);
    }
#pragma unroll
    for (int q = 0; q < 6; q++) {
      if (B <= 64 || 64 * q >= B) continue;  // wave-uniform: the long streams a lane per bit
      int k = 64 * q + lane;
      uint64_t lo = 0ull, hi = 0ull;
      if (k < nv) {
        lo = x.s1[0], hi = x.s1[1];
      } else if ((k -= nv) < nv) {
        lo = x.s5[0], hi = x.s5[1];
      } else if ((k -= nv) < nv) {
        lo = x.s7[0], hi = x.s7[1];
      } else {
        k -= nv;
        lo = k < ninv ? x.s3 : k < 2 * ninv ? x.s4 : k < 3 * ninv ? x.s9 : x.s11;
        k -= k < ninv ? 0 : k < 2 * ninv ? ninv : k < 3 * ninv ? 2 * ninv : 3 * ninv;
      }
      const uint64_t wd = k < 64 ? lo : hi;
      W[q] = __ballot(64 * q + lane < B && ((wd >> (k & 63)) & 1ull));
    }
#if NMMO_WO_STAMPS
    asm volatile("" ::"s"(W[0]), "s"(W[5]));
    WO_STAMP(rs_, 4);
#endif
    uint8_t* rec = wenv + woff[a];
    {
      const int task = __builtin_amdgcn_readlane(my_task, j);
      const uint32_t head[4] = {i16pack(aid, tick), i16pack(task, r - kVision),
                                i16pack(c - kVision, (int)wire_m5(nv, ninv, exch, pp1)),
                                i16pack((int)wire_m6(x.s0 != 0ull, x.s8, ng, pp1), gold)};
      int hx = 0;
      hx = writelanes<0, 0, 4>(head, hx);
      if (lane < 4) reinterpret_cast<int*>(rec)[lane] = hx;
    }
    // Entity rows: each visible row's entity-table index
    if (lane < nv) reinterpret_cast<uint16_t*>(rec + kWireHead)[lane] = rk[ao_slot(visw[lane])];
    if (lane + 64 < nv) reinterpret_cast<uint16_t*>(rec + kWireHead)[lane + 64] = rk[ao_slot(visw[lane + 64])];
    // Inventory rows | materials (4 bits, 4 per int16) | the mask stream | zero pad, as int16 stores
    {
      const int R = wire_off_inv(nv);
      const int H = (wire_record_bytes(cw) - R) >> 1;
      const int ni = 16 * ninv, nt = kWireTiles / 2, ns = wire_stream_bytes(nv, ninv) / 2;
      const uint32_t* wm32 = reinterpret_cast<const uint32_t*>(wmat);
      int16_t* dst = reinterpret_cast<int16_t*>(rec + R);
      for (int h0 = 0; h0 < H; h0 += 64) {
        const int h = h0 + lane;
        const int q = min(h >> 4, kInv - 1);
        const uint2 iw = make_uint2((uint32_t)__shfl((int)it.x, q), (uint32_t)__shfl((int)it.y, q));
        int v16 = 0;
        if (h < ni) {
          v16 = (int)item_col(iw, aid, h & 15);
        } else if (h - ni < nt) {
          const uint32_t m4 = wm32[h - ni] & 0x0F0F0F0Fu;
          v16 = (int)((m4 & 15u) | (m4 >> 4 & 0xF0u) | (m4 >> 8 & 0xF00u) | (m4 >> 12 & 0xF000u));
        } else if (h - ni - nt < ns) {
          const int m = h - ni - nt;
          uint64_t wv = W[0];
#pragma unroll
          for (int u = 1; u < 6; u++) wv = (m >> 2) == u ? W[u] : wv;
          v16 = (int)((wv >> (16 * (m & 3))) & 0xFFFFu);
        }
        if (h < H) dst[h] = (int16_t)v16;
      }
    }
#if NMMO_WO_STAMPS
    WO_STAMP(rs_, 5);
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < kWoStamps; k++) wo_stamp_buf[(size_t)e * P + a][k] = rs_[k];
    }
    nrec++;
#endif
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the next agent reuses visw / wmat
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
#if NMMO_WO_STAMPS
  WO_STAMP(wv_, 3);
#endif
  if (p.recs && my_on) reinterpret_cast<uint2*>(p.recs)[(size_t)e * P + my_a] = my_rec;
  if (p.fault_dst && e == 0 && g == 0 && tid == 0) {  // nmmo_fault_into's effect (the tick ran before)
    const int32_t fw = *p.fault;
    if (fw) atomicCAS(p.fault_dst, 0, fw);
  }
  // the env's listings (Market rows, one 32-B row per thread) and its entity table (the 31
  // columns of each shown slot at its index, a thread per slot, the columns from HBM; then the
  // table's zero pad): workgroup 0, after its records, so no record waits on these stores
  if (g == 0) {
    const int nm = min(max(p.mcount[e], 0), NMMO_MARKET_ROWS);
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
    int16_t* tab = reinterpret_cast<int16_t*>(wenv);
    for (int s = tid; s < S; s += blockDim.x) {
      const int x = rk[s];
      if (x == 0xFFFF) continue;
      int16_t col[NMMO_N_ENTITY_COLS];
#pragma unroll
      for (int f = 0; f < NMMO_N_ENTITY_COLS; f++) col[f] = E[f * S + s];
#pragma unroll
      for (int f = 0; f < NMMO_N_ENTITY_COLS; f++) tab[x * NMMO_N_ENTITY_COLS + f] = col[f];
    }
    for (int b = kEntRow * ne + tid; b < wire_table_bytes(ne); b += blockDim.x) wenv[b] = 0;
  }
#if NMMO_WO_STAMPS
  WO_STAMP(wv_, 4);
  wv_[5] = (uint64_t)e | (uint64_t)nrec << 32;
  if (lane == 0) {
    const int wi = blockIdx.x * kWoWaves + w;
    if (wi < (1 << 15))
      for (int k = 0; k < 6; k++) wo_wave_buf[wi][k] = wv_[k];
  }
#endif
}

hipError_t launch_wire_obs(const ObsParams& p, hipStream_t stream) {
  if (p.S % 8 || p.S > kMaxSlots || p.P > 128 || !p.wire) return hipErrorInvalidValue;
  if (!ao_layout_ok(p)) return hipErrorInvalidValue;  // the wire format's fixed sections
  const hipError_t err = launch_wire_header(p, stream);  // count words, sizes, offsets
  if (err != hipSuccess) return err;
  const dim3 grid(p.n_envs * ((p.P + kWoAgents - 1) / kWoAgents)), block(64 * kWoWaves);  // ao_env_group
  const size_t lds = wo_lds_bytes();
  if (p.wflags) hipLaunchKernelGGL(wire_obs_kernel<true>, grid, block, lds, stream, p);
  else hipLaunchKernelGGL(wire_obs_kernel<false>, grid, block, lds, stream, p);
  return hipGetLastError();
}

}  // namespace nmmo

#if NMMO_WO_STAMPS
extern "C" __attribute__((visibility("default"))) int nmmo_debug_wo_stamps(void* rec, size_t rec_bytes, void* wave,
                                                                         size_t wave_bytes) {
  if (rec_bytes > sizeof(nmmo::wo_stamp_buf)) rec_bytes = sizeof(nmmo::wo_stamp_buf);
  if (wave_bytes > sizeof(nmmo::wo_wave_buf)) wave_bytes = sizeof(nmmo::wo_wave_buf);
  if (hipMemcpyFromSymbol(rec, HIP_SYMBOL(nmmo::wo_stamp_buf), rec_bytes) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(wave, HIP_SYMBOL(nmmo::wo_wave_buf), wave_bytes) != hipSuccess) return -1;
  void* d = nullptr;
  if (hipGetSymbolAddress(&d, HIP_SYMBOL(nmmo::wo_stamp_buf)) != hipSuccess || hipMemset(d, 0, sizeof(nmmo::wo_stamp_buf)) != hipSuccess)
    return -1;
  if (hipGetSymbolAddress(&d, HIP_SYMBOL(nmmo::wo_wave_buf)) != hipSuccess || hipMemset(d, 0, sizeof(nmmo::wo_wave_buf)) != hipSuccess)
    return -1;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
#endif
