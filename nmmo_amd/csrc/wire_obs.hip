// wire_obs.hip — NMMO_OBS_WIRE: the per-agent observation gather written straight as wire
// records (SPEC.md §8c), the C5 sender's obs kernel.
//
// Same observation as obs_kernel's native layout (SPEC §8b; `nmmo_wire_pack` of it is
// byte-identical, tests/test_gpu_wire.py), built for what a record is: ~0.55 KB per agent of
// bits and a few rows, so the kernel is bound by the per-agent dependency chain, not bytes.
// Per workgroup (env e, a group of agents; 4 waves, one agent per wave at a time):
//  - the env's 31 Entity columns are staged in LDS with an odd dword stride (a lane per field
//    reads one slot's row conflict-free; the field-major stride of S = 384 puts all 31 fields
//    of a slot in one bank), and one packed word per datastore row: slot | row << 10 |
//    col << 18 | spawn-immune << 26 | dangerous << 27 | player << 28 (0xFFFFFFFF = empty row);
//  - every lane keeps the packed words of its 6 datastore rows in registers, so an agent's
//    window compaction (Entity.Query.window order) is 6 ballots with no LDS read;
//  - the 11 sent ActionTargets sections are built as wave-uniform bit fields (ballots over the
//    visible rows and the 12 inventory slots, closed forms for Style / GoldPrice / Move /
//    SellPrice) and lane d assembles dword d of the 561-bit image in registers: no LDS atomics;
//  - the record goes out as one dword store for head + mask, one dword store per 4 Entity rows
//    (row pairs are 31 dwords), and u16 stores for the Inventory rows, the 4-bit materials and
//    the zero pad.
// The header's count words and per-env offsets come from wire_count_kernel + wire_scan_kernel
// (wire.hip): record sizes are taken from the count words, so records never overlap.
#include "kernels.h"
#include "wire.h"

namespace nmmo {

constexpr int kWoWaves = 4;
constexpr int kWoAgents = 16;                 // agents per workgroup
constexpr int kWoRows = kMaxSlots / 64;       // packed datastore-row words per lane
constexpr uint32_t kWoEmpty = 0xFFFFFFFFu;
static_assert(kSize <= 256 && kMaxSlots <= 2 * 256, "packed entity word; two slots per thread");
__host__ __device__ inline int wo_stride(int S) { return ((S + 1) >> 1 | 1) << 1; }  // int16, odd dword count
__host__ __device__ inline size_t wo_lds_bytes(int S) {
  return (((size_t)NMMO_N_ENTITY_COLS * wo_stride(S) * 2 + 15) & ~(size_t)15) + (size_t)(kMaxSlots + 64) * 4 +
         (size_t)kWoWaves * (128 * 4 + 256) + (size_t)(128 + 4) * 4;
}

__device__ __forceinline__ int wo_slot(uint32_t w) { return (int)(w & 1023u); }
__device__ __forceinline__ int wo_row(uint32_t w) { return (int)((w >> 10) & 255u); }
__device__ __forceinline__ int wo_col(uint32_t w) { return (int)((w >> 18) & 255u); }

// The 12 ActionTargets sections (nmmo_layout's dims, flat order) and the wire bit offset of
// each sent one: compile-time, so a section's bits land in the record's bit image with constant
// scalar shifts (the launcher checks the handle's layout against them).
constexpr int kSecN[12] = {3, 101, NMMO_MARKET_ROWS + 1, kInv + 1, kInv + 1, kNObs + 1, 99, kNObs + 1, 5, kInv + 1, 99, kInv + 1};
__host__ __device__ constexpr int sec_flat(int k) { return k == 0 ? 0 : sec_flat(k - 1) + kSecN[k - 1]; }
__host__ __device__ constexpr int sec_wire(int k) { return k < 2 ? sec_flat(k) : sec_flat(k) - kWireBuyN; }
static_assert(sec_flat(2) == kWireBuyLo && sec_flat(12) == kMaskN && sec_wire(12) == kWireMaskBits, "sections");
constexpr int kImgWords = (kWireMaskBits + 31) / 32;  // 18

// OR the kN-bit field lo | hi << 64 (bits >= kN zero) into the image at wire bit sec_wire(kSec)
template <int kSec>
__device__ __forceinline__ void put_field(uint32_t (&img)[kImgWords], uint64_t lo, uint64_t hi) {
  constexpr int kOff = sec_wire(kSec), kN = kSecN[kSec];
#pragma unroll
  for (int d = kOff / 32; d <= (kOff + kN - 1) / 32; d++) {
    const int st = 32 * d - kOff;  // field bit on the dword's bit 0
    uint32_t x;
    if (st < 0) x = (uint32_t)(lo << (-st));
    else if (st == 0) x = (uint32_t)lo;
    else if (st < 64) x = (uint32_t)((lo >> st) | (hi << (64 - st)));
    else x = (uint32_t)(hi >> (st - 64));
    img[d] |= x;
  }
}
// x with lane L's value replaced by the wave-uniform v
__device__ __forceinline__ int writelane(int v, int L, int x) { return lane_id() == L ? v : x; }
__device__ __forceinline__ uint64_t low_bits(int n) { return n >= 64 ? ~0ull : n <= 0 ? 0ull : (1ull << n) - 1ull; }

template <bool kWrap>
__global__ void __launch_bounds__(256) wire_obs_kernel(ObsParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int S = p.S, P = p.P, Sp = wo_stride(S);
  int16_t* T = reinterpret_cast<int16_t*>(smem);  // [31][Sp]
  uint32_t* pk = reinterpret_cast<uint32_t*>(smem + (((size_t)NMMO_N_ENTITY_COLS * Sp * 2 + 15) & ~(size_t)15));
  uint32_t* visw_all = pk + kMaxSlots + 64;               // [4][128] packed words of the visible rows
  uint8_t* wmat_all = reinterpret_cast<uint8_t*>(visw_all + kWoWaves * 128);  // [4][256] window materials
  int* woff = reinterpret_cast<int*>(wmat_all + kWoWaves * 256);            // [P + 1] record offsets
  const int e = blockIdx.x, g = blockIdx.y, tid = threadIdx.x, lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane(wave_id());  // wave-uniform values in SGPRs
  const WireView v = wire_view(p.wire, p.n_envs, P);
  const uint16_t* cnt = v.cnt + (size_t)e * P;
  record_offsets_wave0(cnt, P, woff);
  const int16_t* E = p.ent + (size_t)e * NMMO_NF * S;
  {  // the 31 Entity columns: 16-B global loads, dword LDS writes (the padded rows are 4-B aligned)
    const int w4 = S / 8;  // 16-B words per field (S % 8 == 0: checked by the launcher)
    for (int i = tid; i < NMMO_N_ENTITY_COLS * w4; i += blockDim.x) {
      const int f = i / w4, j = i - f * w4;
      const uint4 x = reinterpret_cast<const uint4*>(E + (size_t)f * S)[j];
      uint32_t* d = reinterpret_cast<uint32_t*>(T + f * Sp) + 4 * j;
      d[0] = x.x;
      d[1] = x.y;
      d[2] = x.z;
      d[3] = x.w;
    }
    for (int k = tid; k < kMaxSlots + 64; k += blockDim.x) pk[k] = kWoEmpty;
  }
  // alive / datastore row of slots tid and tid + 256, loaded ahead of the barrier
  int al[2], ds[2];
#pragma unroll
  for (int u = 0; u < 2; u++) {
    const int s = tid + 256 * u;
    al[u] = s < S ? E[F_ALIVE * S + s] : 0;
    ds[u] = s < S ? E[F_DS_ROW * S + s] : 0;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 2; u++) {  // datastore row k (1..S) -> packed entity word at pk[k - 1]
    const int s = tid + 256 * u;
    if (al[u] && (unsigned)(ds[u] - 1) < (unsigned)S) {
      const bool player = s < P;
      const bool immune = player && T[F_TIME_ALIVE * Sp + s] < p.spawn_immunity;
      const bool danger = T[F_NPC_TYPE * Sp + s] > 1;
      pk[ds[u] - 1] = (uint32_t)s | (uint32_t)(uint16_t)T[F_ROW * Sp + s] << 10 |
                      (uint32_t)(uint16_t)T[F_COL * Sp + s] << 18 | (immune ? 1u << 26 : 0u) |
                      (danger ? 1u << 27 : 0u) | (player ? 1u << 28 : 0u);
    }
  }
  __syncthreads();

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
  }

  uint32_t pr[kWoRows];  // this lane's datastore rows 1 + lane + 64 i
#pragma unroll
  for (int i = 0; i < kWoRows; i++) pr[i] = pk[lane + 64 * i];
  uint32_t* visw = visw_all + w * 128;
  uint8_t* wmat = wmat_all + w * 256;
  if (lane < 256 - 225) wmat[225 + lane] = 0;  // materials 225.. read as zero nibbles
  const uint8_t* mat = p.mat + (size_t)e * kTiles;
  const int tick = p.env[(size_t)e * NMMO_NE + E_TICK];
  const bool combat = (p.systems & NMMO_SYS_COMBAT) != 0;
  const bool item = (p.systems & NMMO_SYS_ITEM) != 0;
  const bool exch = item && (p.systems & NMMO_SYS_EXCHANGE) != 0;
  const bool no_give = kWrap && (p.wflags & kWrapObsNoGive);
  const bool no_danger = kWrap && (p.wflags & kWrapObsNoDangerous);
  constexpr int n6 = kSecN[6], n10 = kSecN[10];

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
  auto prefetch = [&](int a) {
    const int r = T[F_ROW * Sp + a], c = T[F_COL * Sp + a];
    iv = lane < kInv ? p.items[((size_t)e * P + a) * kInv + lane] : make_uint2(0u, 0u);
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int t = lane + 64 * i;
      wm[i] = t < 225 ? mat[(r + t / 15 - kVision) * kSize + c + t % 15 - kVision] : 0u;
    }
  };
  auto in_realm = [&](int j) {
    const int a = abase + kWoWaves * j;
    return j < per_wave && a < P && (cnt[a] & 0x8000u);
  };
  if (in_realm(0)) prefetch(abase);

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
    const uint32_t mv = [&] {  // Move targets passable (the centre's neighbours are in wm[1])
      uint32_t b = 0u;
#pragma unroll
      for (int d = 0; d < 5; d++) {
        const int t = (kVision + dir_dr(d)) * 15 + kVision + dir_dc(d);
        if (!impassable((int)__builtin_amdgcn_readlane((int)wm[1], t - 64))) b |= 1u << d;
      }
      return b;
    }();
    if (in_realm(j + 1)) prefetch(a + kWoWaves);  // the next agent's loads, ahead of the stores

    // window compaction: ascending datastore rows within L-inf <= kVision, the first kNObs
    int nvis = 0;
#pragma unroll
    for (int i = 0; i < kWoRows; i++) {
      if (64 * i >= S) break;
      const uint32_t x = pr[i];
      const bool in = x != kWoEmpty && linf(r, c, wo_row(x), wo_col(x)) <= kVision;
      const uint64_t b = __ballot(in);
      const int pos = nvis + __popcll(b & lanes_below());
      if (in && pos < kNObs) visw[pos] = x;
      nvis += __popcll(b);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // sections over the visible rows: 1 AttackTarget, 5 GiveTarget, 7 GoldTarget (+ noop k = 100)
    uint64_t s1[2] = {0ull, 0ull}, s5[2] = {0ull, 0ull}, s7[2] = {0ull, 0ull};
#pragma unroll
    for (int h = 0; h < 2; h++) {
      if (64 * h >= nv) break;
      const int k = 64 * h + lane;
      bool tgt = false, st = false;
      if (k < nv) {
        const uint32_t x = visw[k];
        const int q = wo_slot(x);
        tgt = combat && q != a && linf(r, c, wo_row(x), wo_col(x)) <= 3 && !((x >> 26) & 1u) &&
              !(no_danger && ((x >> 27) & 1u));
        st = ((x >> 28) & 1u) && q != a && wo_row(x) == r && wo_col(x) == c;
      }
      s1[h] = __ballot(tgt);
      const uint64_t sb = __ballot(st);
      if (item && !no_give) s5[h] = sb;
      if (exch && !no_give) s7[h] = sb;
    }
    s1[1] |= 1ull << (kNObs - 64);
    s5[1] |= 1ull << (kNObs - 64);
    s7[1] |= 1ull << (kNObs - 64);
    // sections over the inventory: 3 Destroy, 4 GiveItem, 9 SellItem, 11 Use (+ noop k = 12)
    const bool have = lane < ninv;
    const bool fr = have && !it_equipped(it) && !it_price(it);
    const uint64_t s3 = (item ? __ballot(fr) : 0ull) | 1ull << kInv;
    const uint64_t s4 = (item && !no_give ? __ballot(fr) : 0ull) | 1ull << kInv;
    const uint64_t s9 = (exch ? __ballot(have && !it_equipped(it)) : 0ull) | 1ull << kInv;
    const uint64_t s11 = (item ? __ballot(have && item_usable(T, Sp, a, it)) : 0ull) | 1ull << kInv;
    // closed forms: 0 Style, 6 GoldPrice (k < gold), 8 Move, 10 SellPrice (all but the
    // wrapper's last price)
    const uint64_t s0 = combat ? low_bits(kSecN[0]) : 0ull;
    uint64_t s6[2] = {0ull, 0ull};
    if (exch) {
      const int ng = no_give ? min(gold, 1) : min(gold, n6);
      s6[0] = low_bits(ng);
      s6[1] = low_bits(ng - 64);
    }
    uint64_t s10[2] = {0ull, 0ull};
    if (exch) {
      s10[0] = low_bits(n10);
      s10[1] = low_bits(n10 - 64);
      if constexpr (kWrap) {
        const int pp = __builtin_amdgcn_readlane(my_prev, j);
        if ((p.wflags & kWrapObsPrice) && pp >= 0 && pp < n10) s10[pp >> 6] &= ~(1ull << (pp & 63));
      }
    }
    // the 561-bit image, wave-uniform (scalar ops with constant shifts)
    uint32_t img[kImgWords];
#pragma unroll
    for (int d = 0; d < kImgWords; d++) img[d] = 0u;
    put_field<0>(img, s0, 0ull);
    put_field<1>(img, s1[0], s1[1]);
    put_field<3>(img, s3, 0ull);
    put_field<4>(img, s4, 0ull);
    put_field<5>(img, s5[0], s5[1]);
    put_field<6>(img, s6[0], s6[1]);
    put_field<7>(img, s7[0], s7[1]);
    put_field<8>(img, (uint64_t)mv, 0ull);
    put_field<9>(img, s9, 0ull);
    put_field<10>(img, s10[0], s10[1]);
    put_field<11>(img, s11, 0ull);
    // record: head (4 dwords) | mask image (18 + 2 zero dwords): lane i holds dword i, one store
    uint8_t* rec = wenv + woff[a];
    {
      const int task = __builtin_amdgcn_readlane(my_task, j);
      int x = 0;
      x = writelane((int)i16pack(aid, tick), 0, x);
      x = writelane((int)i16pack(task, r - kVision), 1, x);
      x = writelane((int)i16pack(c - kVision, nv), 2, x);
      x = writelane((int)i16pack(ninv | (exch ? 1 << 8 : 0), gold), 3, x);
#pragma unroll
      for (int d = 0; d < kImgWords; d++) x = writelane((int)img[d], 4 + d, x);
      if (lane < (kWireBody >> 2)) reinterpret_cast<int*>(rec)[lane] = x;
    }
    // Entity rows, four per pass: a row pair is 31 dwords (4-B aligned: 96 + 124 j), lanes
    // 0-30 the pair (k, k + 1), lanes 32-62 the pair (k + 2, k + 3); a pair's last dword holds
    // the next region's first int16 when k + 1 == nv (then only its low half is stored)
    {
      const int i = lane & 31, hp = lane >> 5;
      const int c0 = 2 * i, c1 = 2 * i + 1;
      const int r0 = c0 >= NMMO_N_ENTITY_COLS, r1 = c1 >= NMMO_N_ENTITY_COLS;
      const int f0 = c0 - r0 * NMMO_N_ENTITY_COLS, f1 = c1 - r1 * NMMO_N_ENTITY_COLS;
#pragma unroll 1
      for (int k0 = 0; k0 < nv; k0 += 4) {
        const int k = k0 + 2 * hp, ka = k + r0, kb = k + r1;
        if (i < NMMO_N_ENTITY_COLS && ka < nv) {
          const int lo = T[f0 * Sp + wo_slot(visw[ka])];
          uint8_t* dst = rec + kWireBody + 62 * k + 4 * i;
          if (kb < nv) {
            const int hi = T[f1 * Sp + wo_slot(visw[kb])];
            *reinterpret_cast<uint32_t*>(dst) = i16pack(lo, hi);
          } else {
            *reinterpret_cast<int16_t*>(dst) = (int16_t)lo;
          }
        }
      }
    }
    // Inventory rows | materials (4 bits, 4 per int16) | zero pad, as int16 stores
    {
      const int R = kWireBody + 62 * nv;
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
  const int offs[12] = {p.o_style, p.o_target, p.o_buy, p.o_destroy, p.o_give_item, p.o_give_target,
                        p.o_gg_price, p.o_gg_target, p.o_move, p.o_sell_item, p.o_sell_price, p.o_use};
  for (int k = 0; k < 12; k++)
    if (offs[k] != sec_flat(k)) return hipErrorInvalidValue;  // the wire format's fixed sections
  const hipError_t err = launch_wire_header(p, stream);  // count words, sizes, offsets
  if (err != hipSuccess) return err;
  const dim3 grid(p.n_envs, (p.P + kWoAgents - 1) / kWoAgents), block(64 * kWoWaves);
  const size_t lds = wo_lds_bytes(p.S);
  if (p.wflags) hipLaunchKernelGGL(wire_obs_kernel<true>, grid, block, lds, stream, p);
  else hipLaunchKernelGGL(wire_obs_kernel<false>, grid, block, lds, stream, p);
  return hipGetLastError();
}

}  // namespace nmmo
