// p2p.hip — the learner gather's point-to-point transfers posted natively (nmmo_p2p_*): one RCCL
// group of ncclSend / ncclRecv per call on the caller's stream, over a communicator of this
// library's own (its unique id shared through torch.distributed by the caller).
//
// Why native: the gather root posts 2 x (N - 1) x batches receives per step (C5 at N = 8: 28,
// plus the 7 size rows). Through torch.distributed.batch_isend_irecv each op costs ~13.5 us of host
// time on the GPU box (tools/debug/p2p_host_cost.py: 435 us for a 32-op group), more than the
// whole ~0.27-ms step; a group posted here costs ~1 us per op. The RCCL functions are resolved
// from the librccl the process already loaded (torch's, by path, RTLD_NOLOAD), so there is one
// RCCL instance in the process.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>

#include "kernels.h"

namespace nmmo {
namespace {

struct Rccl {
  void* so = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};
Rccl g_rccl;

template <typename F>
bool sym(void* so, const char* name, F& f) {
  f = reinterpret_cast<F>(dlsym(so, name));
  return f != nullptr;
}

}  // namespace

// 0 on success; a message into err otherwise
int p2p_load(const char* path, char* err, size_t n) {
  if (g_rccl.so) return 0;
  void* so = path && *path ? dlopen(path, RTLD_NOW | RTLD_NOLOAD) : nullptr;
  if (!so && path && *path) so = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!so) {
    snprintf(err, n, "librccl not loadable from '%s': %s", path ? path : "", dlerror());
    return -1;
  }
  Rccl r;
  r.so = so;
  if (!sym(so, "ncclGetUniqueId", r.get_unique_id) || !sym(so, "ncclCommInitRank", r.comm_init_rank) ||
      !sym(so, "ncclCommDestroy", r.comm_destroy) || !sym(so, "ncclSend", r.send) || !sym(so, "ncclRecv", r.recv) ||
      !sym(so, "ncclGroupStart", r.group_start) || !sym(so, "ncclGroupEnd", r.group_end) ||
      !sym(so, "ncclGetErrorString", r.error_string)) {
    snprintf(err, n, "librccl at '%s' lacks an entry point", path);
    return -1;
  }
  g_rccl = r;
  return 0;
}

int p2p_unique_id(void* id, char* err, size_t n) {
  ncclUniqueId u;
  const ncclResult_t rc = g_rccl.get_unique_id(&u);
  if (rc != ncclSuccess) {
    snprintf(err, n, "ncclGetUniqueId: %s", g_rccl.error_string(rc));
    return -1;
  }
  memcpy(id, &u, sizeof(u));
  return 0;
}

int p2p_init(const void* id, int world, int rank, void** comm, char* err, size_t n) {
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  const ncclResult_t rc = g_rccl.comm_init_rank(&c, world, u, rank);
  if (rc != ncclSuccess) {
    snprintf(err, n, "ncclCommInitRank(world %d, rank %d): %s", world, rank, g_rccl.error_string(rc));
    return -1;
  }
  *comm = c;
  return 0;
}

int p2p_group(void* comm, const NmmoP2POp* ops, int n_ops, hipStream_t stream, char* err, size_t n) {
  ncclComm_t c = static_cast<ncclComm_t>(comm);
  ncclResult_t rc = g_rccl.group_start();
  for (int i = 0; i < n_ops && rc == ncclSuccess; i++) {
    const NmmoP2POp& o = ops[i];
    rc = o.recv ? g_rccl.recv(o.buf, (size_t)o.bytes, ncclUint8, o.peer, c, stream)
                : g_rccl.send(o.buf, (size_t)o.bytes, ncclUint8, o.peer, c, stream);
  }
  const ncclResult_t re = g_rccl.group_end();  // always closes the group it opened
  if (rc == ncclSuccess) rc = re;
  if (rc != ncclSuccess) {
    snprintf(err, n, "RCCL group of %d ops: %s", n_ops, g_rccl.error_string(rc));
    return -1;
  }
  return 0;
}

int p2p_destroy(void* comm) {
  return comm && g_rccl.comm_destroy && g_rccl.comm_destroy(static_cast<ncclComm_t>(comm)) == ncclSuccess ? 0 : -1;
}

}  // namespace nmmo
