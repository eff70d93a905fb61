// storage.hip — GPU-resident experience storage: the trainer-side
// buffers of the reference's clean_pufferl kept in HBM, so the rollout never leaves the device.
//
//   store_count / store_place / store_rows  <- evaluate(): learner_mask, the alive-row indices
//       truncated to the room left, the obs/values/actions/logprobs/rewards/dones row stores
//       and the (env_id, step) sort keys      reinforcement_learning/clean_pufferl.py:331-346
//   sort_scan / sort_scatter  <- sorted(range(len(sort_keys)), key=sort_keys.__getitem__)  :414
//   gae_kernel                <- the reversed advantage loop (float32, serial order)   :424-436
//   gather_rows_kernel        <- b_obs = obs_ary[b_idxs] and the per-minibatch copies  :439-458
//
// Byte work, HBM-bound: a stored row moves 95,948 B of obs (flat) or is expanded straight from
// the native layout (SPEC §8b: 9,552 B read per row) or decoded from its wire record (SPEC §8c,
// ~1.3 KB read per row; wire.hip wire_expand_kernel) into its experience slot; every other
// field is a few bytes per row.
#include <algorithm>

#include "kernels.h"
#include "wire.h"

namespace nmmo {

constexpr int kStoreBlock = 512;  // rows per workgroup in the count/place passes (8 waves)

// A row is stored iff the learner mask selects it and its env id is a valid slot; a selected
// row with an env id outside [0, n_slots) is dropped (never indexes slot_count / offset) and
// raises bit 0 of x.status.
__device__ __forceinline__ bool row_selected(const NmmoExperience& x, const NmmoStoreInput& in, int r) {
  if (r >= in.n_rows || in.mask[r] == 0) return false;
  const int eid = in.env_id ? in.env_id[r] : in.env_id_base + r;
  if (eid >= 0 && eid < x.n_slots) return true;
  if (x.status) atomicOr(x.status, 1);
  return false;
}

// Pass 1: selected rows per block of kStoreBlock rows.
__global__ void __launch_bounds__(kStoreBlock) store_count_kernel(NmmoExperience x, NmmoStoreInput in, int* blk_cnt) {
  __shared__ int wt[8];
  const int r = blockIdx.x * kStoreBlock + threadIdx.x;
  const uint64_t b = __ballot(row_selected(x, in, r));
  if (lane_id() == 0) wt[wave_id()] = __popcll(b);
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int i = 0; i < kStoreBlock / 64; i++) s += wt[i];
    blk_cnt[blockIdx.x] = s;
  }
}

// Pass 2: each alive row's rank in row order (clean_pufferl.py:333 torch.where(learner_mask)),
// its experience slot ptr + rank if that is below the capacity (the [: batch_size - ptr + 1]
// cut, :333), and the small per-row fields. dst[r] = slot or -1 (read by store_rows).
// gate: NULL, or a device int that is 0 when the store keeps no row (record storage without arena
// room); rs.row_buf non-NULL: record storage, each stored row's buffer descriptor (at arena offset
// *rbase) and agent index are recorded.
__global__ void __launch_bounds__(kStoreBlock) store_place_kernel(NmmoExperience x, NmmoStoreInput in,
                                                                  const int* blk_cnt, int* dst, int* total,
                                                                  const int* gate, NmmoRecordStore rs,
                                                                  const int64_t* rbase) {
  __shared__ int wt[2][8];
  const int b = blockIdx.x, tid = threadIdx.x, r = b * kStoreBlock + tid;
  int part = 0;  // rows of the blocks before this one
  for (int i = tid; i < b; i += kStoreBlock) part += blk_cnt[i];
  int base_total;
  (void)block_prefix_sum(part, wt[0], &base_total);
  const bool alive = row_selected(x, in, r);
  int blk_total;
  const int rank = base_total + block_prefix_count(alive, wt[1], &blk_total);
  const int ptr0 = *x.ptr;
  const int room = gate && !*gate ? 0 : x.capacity - ptr0;
  if (r < in.n_rows) dst[r] = (alive && rank < room) ? ptr0 + rank : -1;
  if (alive && rank < room) {
    const int s = ptr0 + rank;
    const int eid = in.env_id ? in.env_id[r] : in.env_id_base + r;
    x.rewards[s] = in.rewards[r];
    x.dones[s] = (float)in.dones[r];
    x.logprobs[s] = in.logprobs[r];
    x.values[s] = in.values[r];
    const int32_t* a = in.actions + (size_t)r * kHeads;
    long long* o = reinterpret_cast<long long*>(x.actions) + (size_t)s * kHeads;
#pragma unroll
    for (int h = 0; h < kHeads; h++) o[h] = a[h];
    x.env_id[s] = eid;
    x.step[s] = in.step;
    if (rs.row_buf) {
      rs.row_buf[s] = *rbase;
      rs.row_agent[s] = r;
    }
    // rank of this row among its env_id's rows (stores arrive in step order). Env ids are
    // distinct within one store (ABI precondition), so the counter has one writer; the atomic
    // keeps a violating caller's rows at distinct sorted positions instead of corrupting them.
    x.seq[s] = atomicAdd(&x.slot_count[eid], 1);
  }
  if (b == gridDim.x - 1 && tid == 0) *total = min(base_total + blk_total, room);  // rows placed
}

// Pass 3 (flat obs): one wave copies one 95,948-B row (4-B aligned rows, so dword accesses;
// eight loads in flight per lane).
__global__ void __launch_bounds__(256) store_rows_kernel(const float* __restrict__ src, int n, int elems,
                                                        const int* __restrict__ dst, float* __restrict__ out) {
  const int r = blockIdx.x * 4 + wave_id();
  if (r >= n) return;
  const int s = dst[r];
  if (s < 0) return;
  const float* a = src + (size_t)r * elems;
  float* o = out + (size_t)s * elems;
  const int lane = lane_id();
  int j = lane;
  for (; j + 7 * 64 < elems; j += 8 * 64) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = a[j + k * 64];
#pragma unroll
    for (int k = 0; k < 8; k++) o[j + k * 64] = v[k];
  }
  for (; j < elems; j += 64) o[j] = a[j];
}

__global__ void store_commit_kernel(int* ptr, const int* total, int capacity) {
  const int p = *ptr + *total;
  *ptr = p < capacity ? p : capacity;
}

// ---------------------------------------------------------------- sort by (env_id, step)
// Rows of one env_id arrive in step order, so the stable order of clean_pufferl.py:414 is
// position = (rows of all smaller env ids) + the row's rank among its env id's rows: an
// exclusive scan of the per-env-id counts (one workgroup) and a scatter. No comparison sort.
__global__ void __launch_bounds__(512) sort_scan_kernel(const int* slot_count, int n_slots, int* offset) {
  __shared__ int wt[2][8];
  int carry = 0;
  for (int base = 0, k = 0; base < n_slots; base += 512, k ^= 1) {
    const int i = base + threadIdx.x;
    const int v = i < n_slots ? slot_count[i] : 0;
    int t;
    const int ex = block_prefix_sum(v, wt[k], &t);
    if (i < n_slots) offset[i] = carry + ex;
    carry += t;
  }
}

__global__ void __launch_bounds__(256) sort_scatter_kernel(NmmoExperience x, const int* offset, int32_t* idxs) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= *x.ptr) return;
  idxs[offset[x.env_id[r]] + x.seq[r]] = r;
}

// ---------------------------------------------------------------- advantages (:424-436)
// for t = B-1 .. 0 with i = idxs[t], j = idxs[t+1]:
//   nnt = 1 - dones[j]; delta = rewards[j] + g*values[j]*nnt - values[i]
//   adv[t] = last = delta + gl*nnt*last           (g = gamma, gl = gamma*gae_lambda, float32)
// The reference evaluates this on float32 CPU tensors one op at a time (left to right, each op
// rounded); delta and gl*nnt do not depend on `last`, so all 64 lanes form them for a chunk of
// 64 t's in parallel and only the two-op recurrence walks the chunk serially (operands read
// with v_readlane). FP contraction is off here: no FMA, bit-identical to the reference.
__global__ void __launch_bounds__(64) gae_kernel(NmmoExperience x, const int32_t* idxs, int B, float g, float gl,
                                                 float* adv) {
#pragma clang fp contract(off)
  const int lane = lane_id();
  float last = 0.f;
  for (int hi = B - 1; hi >= 0; hi -= 64) {
    const int t = hi - lane;  // lane 0 walks first (largest t)
    float delta = 0.f, k = 0.f;
    if (t >= 0) {
      const int i = idxs[t], j = idxs[t + 1];
      const float nnt = 1.0f - x.dones[j];
      delta = x.rewards[j] + g * x.values[j] * nnt - x.values[i];
      k = gl * nnt;
    }
    float mine = 0.f;
    // lanes past t = 0 in the last chunk carry delta = k = 0: they only overwrite `last` after
    // the final stored element
#pragma unroll
    for (int l = 0; l < 64; l++) {
      const float d = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, delta), l));
      const float kk = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, k), l));
      last = d + kk * last;
      mine = lane == l ? last : mine;
    }
    if (t >= 0) adv[t] = mine;
  }
}

// ---------------------------------------------------------------- row gather (:439-458)
// out[k] = src[idx[k]] for rows of `words` dwords; one wave per row, eight loads in flight.
__global__ void __launch_bounds__(256) gather_rows_kernel(const uint32_t* __restrict__ src, int64_t words,
                                                         const int32_t* __restrict__ idx, int n,
                                                         uint32_t* __restrict__ out) {
  const int k = blockIdx.x * 4 + wave_id();
  if (k >= n) return;
  const uint32_t* a = src + (size_t)idx[k] * words;
  uint32_t* o = out + (size_t)k * words;
  int64_t j = lane_id();
  for (; j + 7 * 64 < words; j += 8 * 64) {
    uint32_t v[8];
#pragma unroll
    for (int q = 0; q < 8; q++) v[q] = a[j + q * 64];
#pragma unroll
    for (int q = 0; q < 8; q++) o[j + q * 64] = v[q];
  }
  for (; j < words; j += 64) o[j] = a[j];
}

// ---------------------------------------------------------------- launches
int store_blocks(int n_rows) { return (n_rows + kStoreBlock - 1) / kStoreBlock; }

hipError_t launch_store(const NmmoExperience& x, const NmmoStoreInput& in, const ObsParams* native,
                        int* scratch, hipStream_t stream) {
  const int nb = store_blocks(in.n_rows);
  int* dst = scratch;                // [n_rows]
  int* blk = scratch + in.n_rows;    // [nb]
  int* total = blk + nb;             // [1]
  hipLaunchKernelGGL(store_count_kernel, dim3(nb), dim3(kStoreBlock), 0, stream, x, in, blk);
  hipLaunchKernelGGL(store_place_kernel, dim3(nb), dim3(kStoreBlock), 0, stream, x, in, blk, dst, total,
                     (const int*)nullptr, NmmoRecordStore{}, (const int64_t*)nullptr);
  if (native) {
    ObsParams p = *native;
    p.obs = x.obs;
    p.row_map = dst;
    hipError_t e = p.wire ? launch_wire_expand(p, stream) : launch_expand(p, stream);
    if (e != hipSuccess) return e;
  } else {
    hipLaunchKernelGGL(store_rows_kernel, dim3((in.n_rows + 3) / 4), dim3(256), 0, stream, in.obs, in.n_rows,
                       x.obs_elems, dst, x.obs);
  }
  hipLaunchKernelGGL(store_commit_kernel, dim3(1), dim3(1), 0, stream, x.ptr, total, x.capacity);
  return hipGetLastError();
}

// ---------------------------------------------------------------- compact record storage
// One thread: the wire buffer's announced total, its place in the arena (16-B aligned, after a
// 16-B descriptor n_envs | player_n) if it fits and is a plausible buffer (>= its header, <= the
// caller's capacity bound). gate[0] = fits; rbase[0] = descriptor offset; the arena grows.
__global__ void record_reserve_kernel(NmmoExperience x, NmmoRecordStore rs, const uint8_t* wire, int n_envs, int P,
                                      int64_t wire_cap, int* gate, int64_t* rbase) {
  const int64_t total = *reinterpret_cast<const int64_t*>(wire);
  const int64_t base = (*rs.arena_used + 15) & ~(int64_t)15;
  const bool sane = total >= wire_header_bytes(n_envs, P) && total <= wire_cap && (total & 15) == 0 &&
                    base + 16 + total <= rs.arena_bytes;
  // a buffer inside the arena is stored only at its own slot (record_reserve_wave)
  const bool inside = wire >= rs.arena && wire < rs.arena + rs.arena_bytes, placed = wire == rs.arena + base + 16;
  const bool ok = sane && (!inside || placed);
  *gate = ok ? (placed ? 2 : 1) : 0;  // 2: the buffer is in place already
  *rbase = base;
  if (ok) {
    int64_t* d = reinterpret_cast<int64_t*>(rs.arena + base);
    d[0] = n_envs;
    d[1] = P;
    *rs.arena_used = base + 16 + total;
  } else if (x.status) {
    atomicOr(x.status, sane ? 16 : 2);
  }
}

// the buffer's `total` bytes behind its descriptor, 16 B per lane, grid-stride (the length is read
// on the device)
__global__ void __launch_bounds__(256) record_copy_kernel(NmmoRecordStore rs, const uint4* __restrict__ wire,
                                                         const int* gate, const int64_t* rbase) {
  if (*gate != 1) return;  // not stored, or received in place
  const int64_t words = *reinterpret_cast<const int64_t*>(wire) / 16;
  uint4* dst = reinterpret_cast<uint4*>(rs.arena + *rbase + 16);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = wire[i];
}

hipError_t launch_store_records(const NmmoExperience& x, const NmmoRecordStore& rs, const NmmoStoreInput& in,
                                int P, int64_t wire_cap, int* scratch, hipStream_t stream) {
  const int nb = store_blocks(in.n_rows);
  int* dst = scratch;                // [n_rows]
  int* blk = scratch + in.n_rows;    // [nb]
  int* total = blk + nb;             // [1]
  int* gate = total + 1;             // [1]
  int64_t* rbase = reinterpret_cast<int64_t*>(scratch + ((in.n_rows + nb + 2 + 1) & ~1));  // [1], 8-B aligned
  const uint8_t* wire = (const uint8_t*)in.wire;
  hipLaunchKernelGGL(record_reserve_kernel, dim3(1), dim3(1), 0, stream, x, rs, wire, in.n_rows / P, P, wire_cap,
                     gate, rbase);
  hipLaunchKernelGGL(store_count_kernel, dim3(nb), dim3(kStoreBlock), 0, stream, x, in, blk);
  hipLaunchKernelGGL(store_place_kernel, dim3(nb), dim3(kStoreBlock), 0, stream, x, in, blk, dst, total,
                     (const int*)gate, rs, (const int64_t*)rbase);
  const int64_t words = wire_cap / 16;
  const int grid = (int)std::min<int64_t>((words + 255) / 256, 4096);
  hipLaunchKernelGGL(record_copy_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, stream, rs,
                     (const uint4*)wire, (const int*)gate, (const int64_t*)rbase);
  hipLaunchKernelGGL(store_commit_kernel, dim3(1), dim3(1), 0, stream, x.ptr, total, x.capacity);
  return hipGetLastError();
}

// ---- several wire buffers in one store (the root of the C5 gather: every rank's buffers of a
// step, kept as one batch of rows in input order; five launches whatever the input count)
__device__ __forceinline__ int sb_mask(const StoreBatch& b, const NmmoStoreInput& in, int r) {
  return b.stride ? in.mask[(size_t)r * b.stride] : in.mask[r];
}
__device__ __forceinline__ bool sb_selected(const NmmoExperience& x, const StoreBatch& b, int i, const int* gates,
                                            int r) {
  const NmmoStoreInput& in = b.in[i];
  if (r >= in.n_rows || !gates[i] || sb_mask(b, in, r) == 0) return false;
  const int eid = in.env_id ? in.env_id[r] : in.env_id_base + r;
  if (eid >= 0 && eid < x.n_slots) return true;
  if (x.status) atomicOr(x.status, 1);
  return false;
}

// The reservation of every input, in input order, by one wave: lane i loads input i's announced
// total and check word (every load in flight at once -- one thread walking 16 inputs waited a
// memory round trip per input), then lane 0 places them serially from registers. An input is
// stored when its announced total is a plausible buffer (>= its header, <= its capacity bound,
// 16-B multiple), it fits, and (ist, the check's per-input bits, when given) it passed its check.
// gates[i]: 2 = the buffer already sits where it is to be stored (received straight into the
// arena), 1 = copy it there, 0 = not stored (x.status bit 1: no room / not plausible; bit 3:
// failed its check; bit 4: the buffer lies inside the arena but not at its reserved slot -- a
// copy would read arena bytes that earlier inputs of this store overwrite, so it is refused,
// never copied).
__device__ void record_reserve_wave(const NmmoExperience& x, const NmmoRecordStore& rs, const StoreBatch& b,
                                    int* gates, int64_t* rbase, const int* ist) {
  const int lane = threadIdx.x;
  int64_t tot = 0;
  int chk = 0;
  if (lane < b.n) {
    tot = *reinterpret_cast<const int64_t*>(b.in[lane].wire);
    chk = ist ? ist[lane] : 0;
  }
  int64_t used = *rs.arena_used;
  if (lane != 0) return;
  const uint8_t* a0 = rs.arena;
  for (int i = 0; i < b.n; i++) {
    const NmmoStoreInput& in = b.in[i];
    const int n_envs = in.n_rows / b.P;
    const uint8_t* w = reinterpret_cast<const uint8_t*>(in.wire);
    const int64_t total = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)tot, i) |
                          (int64_t)__builtin_amdgcn_readlane((int)(tot >> 32), i) << 32;
    const int64_t base = (used + 15) & ~(int64_t)15;
    const bool sane = total >= wire_header_bytes(n_envs, b.P) && total <= b.wire_cap[i] && (total & 15) == 0 &&
                      base + 16 + total <= rs.arena_bytes;
    const bool checked = __builtin_amdgcn_readlane(chk, i) == 0;
    const bool inside = w >= a0 && w < a0 + rs.arena_bytes;
    const bool placed = w == a0 + base + 16;
    const bool ok = sane && checked && (!inside || placed);
    gates[i] = ok ? (placed ? 2 : 1) : 0;
    rbase[i] = base;
    if (ok) {
      int64_t* d = reinterpret_cast<int64_t*>(rs.arena + base);
      d[0] = n_envs;
      d[1] = b.P;
      used = base + 16 + total;
    } else if (x.status) {
      atomicOr(x.status, !sane ? 2 : !checked ? 8 : 16);
    }
  }
  *rs.arena_used = used;
}

__global__ void __launch_bounds__(64) record_reserve_many_kernel(NmmoExperience x, NmmoRecordStore rs, StoreBatch b,
                                                                  int* gates, int64_t* rbase) {
  record_reserve_wave(x, rs, b, gates, rbase, nullptr);
}

// The root's received-buffer check inside its store (nmmo_exp_store_records_checked): wave (env,
// input) runs the check of one env (wire_check_env, the bits of nmmo_wire_check_many) and ORs
// what it finds into the input's status word c.ctl[i] and the caller's; the reservation that
// follows (record_reserve_checked_kernel) stores only the inputs whose word stayed 0 and zeroes
// the words again. (A last-block ticket that reserved inside this launch measured ~1 ms per step
// at C5's 16 inputs x 512 envs: one agent-scope atomic per block on a single word.)
__global__ void __launch_bounds__(64 * kCheckEnvsPerBlock) record_check_kernel(StoreBatch b, StoreCheck c) {
  const int i = blockIdx.y, e = blockIdx.x * kCheckEnvsPerBlock + wave_id();
  const int n_envs = b.in[i].n_rows / b.P;
  if (e >= n_envs || !((c.mask >> i) & 1u)) return;  // wave-uniform
  const int bad = wire_check_env(reinterpret_cast<const uint8_t*>(b.in[i].wire), n_envs, b.P, c.expect[i], e);
  if (bad) {
    atomicOr(&c.ctl[i], bad);
    if (c.status) atomicOr(c.status, bad);
  }
}

__global__ void __launch_bounds__(64) record_reserve_checked_kernel(NmmoExperience x, NmmoRecordStore rs, StoreBatch b,
                                                                     StoreCheck c, int* gates, int64_t* rbase) {
  record_reserve_wave(x, rs, b, gates, rbase, c.ctl);
  if (threadIdx.x < kMaxStoreInputs) c.ctl[threadIdx.x] = 0;  // (every lane read its word above)
}

__global__ void __launch_bounds__(kStoreBlock) store_count_many_kernel(NmmoExperience x, StoreBatch b,
                                                                       const int* gates, int* blk_cnt) {
  __shared__ int wt[8];
  const int i = blockIdx.y, r = blockIdx.x * kStoreBlock + threadIdx.x;
  const uint64_t m = __ballot(sb_selected(x, b, i, gates, r));
  if (lane_id() == 0) wt[wave_id()] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int k = 0; k < kStoreBlock / 64; k++) s += wt[k];
    blk_cnt[i * gridDim.x + blockIdx.x] = s;
  }
}

__global__ void __launch_bounds__(kStoreBlock) store_place_many_kernel(NmmoExperience x, NmmoRecordStore rs,
                                                                       StoreBatch b, const int* gates,
                                                                       const int64_t* rbase, const int* blk_cnt,
                                                                       int* total) {
  __shared__ int wt[2][8];
  const int i = blockIdx.y, tid = threadIdx.x, r = blockIdx.x * kStoreBlock + tid;
  const int gb = i * gridDim.x + blockIdx.x;  // this block's place in input order
  int part = 0;
  for (int k = tid; k < gb; k += kStoreBlock) part += blk_cnt[k];
  int base_total;
  (void)block_prefix_sum(part, wt[0], &base_total);
  const bool alive = sb_selected(x, b, i, gates, r);
  int blk_total;
  const int rank = base_total + block_prefix_count(alive, wt[1], &blk_total);
  const int ptr0 = *x.ptr;
  const int room = x.capacity - ptr0;
  if (alive && rank < room) {
    const NmmoStoreInput& in = b.in[i];
    const int s = ptr0 + rank;
    const int eid = in.env_id ? in.env_id[r] : in.env_id_base + r;
    const uint8_t* rw = reinterpret_cast<const uint8_t*>(in.rewards);
    x.rewards[s] = b.stride ? *reinterpret_cast<const float*>(rw + (size_t)r * b.stride) : in.rewards[r];
    x.dones[s] = (float)(b.stride ? in.dones[(size_t)r * b.stride] : in.dones[r]);
    x.logprobs[s] = in.logprobs[r];
    x.values[s] = in.values[r];
    const int32_t* a = in.actions + (size_t)r * kHeads;
    long long* o = reinterpret_cast<long long*>(x.actions) + (size_t)s * kHeads;
#pragma unroll
    for (int h = 0; h < kHeads; h++) o[h] = a[h];
    x.env_id[s] = eid;
    x.step[s] = in.step;
    // env ids are distinct within one store (nmmo_hip.h precondition): a plain read and write, no
    // atomic round trip per row
    const int q = x.slot_count[eid];
    x.seq[s] = q;
    x.slot_count[eid] = q + 1;
    rs.row_buf[s] = rbase[i];
    rs.row_agent[s] = r;
  }
  if (gb == (int)(gridDim.x * gridDim.y) - 1 && tid == 0) *total = min(base_total + blk_total, room);
}

// The inputs with gate 1, each copied behind its descriptor (16 B per lane, grid-stride over a 1-D
// grid that walks every input: a store whose inputs are all in place costs one short launch).
__global__ void __launch_bounds__(256) record_copy_many_kernel(NmmoRecordStore rs, StoreBatch b, const int* gates,
                                                              const int64_t* rbase) {
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
  for (int i = 0; i < b.n; i++) {
    if (gates[i] != 1) continue;  // not stored, or received in place
    const uint4* wire = reinterpret_cast<const uint4*>(b.in[i].wire);
    const int64_t words = *reinterpret_cast<const int64_t*>(wire) / 16;
    uint4* dst = reinterpret_cast<uint4*>(rs.arena + rbase[i] + 16);
    for (int64_t k = t0; k < words; k += stride) dst[k] = wire[k];
  }
}

int store_many_scratch_ints(int n_inputs, int max_rows) {
  return n_inputs * store_blocks(max_rows) + 1 + n_inputs + 2 * n_inputs + 4;
}

hipError_t launch_store_records_many(const NmmoExperience& x, const NmmoRecordStore& rs, const StoreBatch& b,
                                     int* scratch, hipStream_t stream, const StoreCheck* chk) {
  int max_rows = 0;
  for (int i = 0; i < b.n; i++) max_rows = max(max_rows, b.in[i].n_rows);
  const int nb = store_blocks(max_rows);
  int* blk = scratch;              // [n][nb]
  int* total = blk + b.n * nb;     // [1]
  int* gates = total + 1;          // [n]
  int64_t* rbase = reinterpret_cast<int64_t*>(scratch + ((b.n * nb + 1 + b.n + 1) & ~1));  // [n], 8-B aligned
  if (chk) {
    hipLaunchKernelGGL(record_check_kernel, dim3((max_rows / b.P + kCheckEnvsPerBlock - 1) / kCheckEnvsPerBlock, b.n),
                       dim3(64 * kCheckEnvsPerBlock), 0, stream, b, *chk);
    hipLaunchKernelGGL(record_reserve_checked_kernel, dim3(1), dim3(64), 0, stream, x, rs, b, *chk, gates, rbase);
  } else {
    hipLaunchKernelGGL(record_reserve_many_kernel, dim3(1), dim3(64), 0, stream, x, rs, b, gates, rbase);
  }
  hipLaunchKernelGGL(store_count_many_kernel, dim3(nb, b.n), dim3(kStoreBlock), 0, stream, x, b, (const int*)gates,
                     blk);
  hipLaunchKernelGGL(store_place_many_kernel, dim3(nb, b.n), dim3(kStoreBlock), 0, stream, x, rs, b,
                     (const int*)gates, (const int64_t*)rbase, (const int*)blk, total);
  int64_t words = 0;
  for (int i = 0; i < b.n; i++) words = std::max(words, b.wire_cap[i] / 16);
  const int grid = (int)std::min<int64_t>((words + 255) / 256, 2048);
  hipLaunchKernelGGL(record_copy_many_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, stream, rs, b,
                     (const int*)gates, (const int64_t*)rbase);
  hipLaunchKernelGGL(store_commit_kernel, dim3(1), dim3(1), 0, stream, x.ptr, total, x.capacity);
  return hipGetLastError();
}

hipError_t launch_sort(const NmmoExperience& x, int32_t* idxs, int* scratch, hipStream_t stream) {
  hipLaunchKernelGGL(sort_scan_kernel, dim3(1), dim3(512), 0, stream, x.slot_count, x.n_slots, scratch);
  hipLaunchKernelGGL(sort_scatter_kernel, dim3((x.capacity + 255) / 256), dim3(256), 0, stream, x, scratch, idxs);
  return hipGetLastError();
}

hipError_t launch_gae(const NmmoExperience& x, const int32_t* idxs, int B, float g, float gl, float* adv,
                      hipStream_t stream) {
  hipLaunchKernelGGL(gae_kernel, dim3(1), dim3(64), 0, stream, x, idxs, B, g, gl, adv);
  return hipGetLastError();
}

hipError_t launch_gather_rows(const void* src, int64_t row_words, const int32_t* idx, int n, void* out,
                              hipStream_t stream) {
  hipLaunchKernelGGL(gather_rows_kernel, dim3((n + 3) / 4), dim3(256), 0, stream, (const uint32_t*)src,
                     row_words, idx, n, (uint32_t*)out);
  return hipGetLastError();
}

}  // namespace nmmo
