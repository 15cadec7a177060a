// Library-owned RCCL communicator (include/ptzba.h ptzba_comm_*): "a handle per rank, created with an RCCL
// unique id" (SURVEY §8b), so a plain ctypes caller -- the reference's rf_map_wrapper.py style -- can run a
// sharded solve without torch.  RCCL is loaded at run time (dlopen): the library itself does not depend
// on it, a process that never builds a communicator never loads it, and PTZBA_RCCL_LIB can point at another
// build (the CPU plumbing test points it at a stub).  If the process already holds an RCCL (torch's), the
// loader returns that one for the same soname.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/ptzba.h"
#include "host_util.h"

namespace {

// the RCCL (NCCL 2.x) ABI this file uses: opaque communicator, 128-byte unique id, ncclFloat64 = 8,
// ncclSum = 0, ncclSuccess = 0
typedef void* nccl_comm_t;
struct nccl_uid {
  char internal[PTZBA_UNIQUE_ID_BYTES];
};
constexpr int NCCL_FLOAT64 = 8, NCCL_SUM = 0;

struct Rccl {
  void* so = nullptr;
  int (*get_unique_id)(nccl_uid*) = nullptr;
  int (*comm_init_rank)(nccl_comm_t*, int, nccl_uid, int) = nullptr;
  int (*comm_destroy)(nccl_comm_t) = nullptr;
  int (*comm_split)(nccl_comm_t, int, int, nccl_comm_t*, void*) = nullptr;
  int (*all_reduce)(const void*, void*, size_t, int, int, nccl_comm_t, hipStream_t) = nullptr;
  int (*user_rank)(nccl_comm_t, int*) = nullptr;
  int (*count)(nccl_comm_t, int*) = nullptr;
  const char* (*error_string)(int) = nullptr;
  std::string err;
};

Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* path = getenv("PTZBA_RCCL_LIB");
    const char* names[] = {path, "librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : names) {
      if (!n || !*n) continue;
      r.so = dlopen(n, RTLD_NOW | RTLD_LOCAL);
      if (r.so) break;
      r.err = dlerror();
      if (path && n == path) break;  // an explicit path must load
    }
    if (!r.so) return;
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(r.so, "ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(r.so, "ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(r.so, "ncclCommDestroy"));
    r.comm_split = reinterpret_cast<decltype(r.comm_split)>(dlsym(r.so, "ncclCommSplit"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(r.so, "ncclAllReduce"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(r.so, "ncclGetErrorString"));
    r.user_rank = reinterpret_cast<decltype(r.user_rank)>(dlsym(r.so, "ncclCommUserRank"));
    r.count = reinterpret_cast<decltype(r.count)>(dlsym(r.so, "ncclCommCount"));
    if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.all_reduce) {
      r.err = "RCCL library lacks ncclGetUniqueId / ncclCommInitRank / ncclCommDestroy / ncclAllReduce";
      r.so = nullptr;
    }
  });
  return r;
}

int rccl_fail(const char* what, int code) {
  Rccl& r = rccl();
  return ptzba::fail("%s failed: RCCL error %d (%s)", what, code, r.error_string ? r.error_string(code) : "?");
}

}  // namespace

struct ptzba_comm_s {
  nccl_comm_t comm = nullptr;
  int rank = 0, world = 1, device = -1;
};

int ptzba_comm_unique_id(void* id_out) {
  if (!id_out) return ptzba::fail("null id buffer");
  Rccl& r = rccl();
  if (!r.so) return ptzba::fail("RCCL not available: %s", r.err.c_str());
  nccl_uid id;
  std::memset(&id, 0, sizeof(id));
  if (int e = r.get_unique_id(&id)) return rccl_fail("ncclGetUniqueId", e);
  std::memcpy(id_out, &id, sizeof(id));
  return 0;
}

ptzba_comm ptzba_comm_new(int device, const void* unique_id, int32_t rank, int32_t world) {
  if (!unique_id || world < 1 || rank < 0 || rank >= world) {
    ptzba::fail("bad communicator arguments (rank %d, world %d)", rank, world);
    return nullptr;
  }
  Rccl& r = rccl();
  if (!r.so) {
    ptzba::fail("RCCL not available: %s", r.err.c_str());
    return nullptr;
  }
  if (device >= 0 && ptzba::select_device(device)) return nullptr;
  nccl_uid id;
  std::memcpy(&id, unique_id, sizeof(id));
  nccl_comm_t c = nullptr;
  if (int e = r.comm_init_rank(&c, world, id, rank)) {
    rccl_fail("ncclCommInitRank", e);
    return nullptr;
  }
  auto* pc = new ptzba_comm_s();
  pc->comm = c;
  pc->rank = rank;
  pc->world = world;
  pc->device = device;
  return pc;
}

void ptzba_comm_delete(ptzba_comm c) {
  if (!c) return;
  Rccl& r = rccl();
  if (c->comm && r.so) (void)r.comm_destroy(c->comm);
  delete c;
}

ptzba_comm ptzba_comm_split(ptzba_comm parent, int32_t color, int32_t key) {
  if (!parent || !parent->comm) {
    ptzba::fail("null communicator");
    return nullptr;
  }
  Rccl& r = rccl();
  if (!r.comm_split) {
    ptzba::fail("this RCCL has no ncclCommSplit");
    return nullptr;
  }
  nccl_comm_t c = nullptr;
  if (int e = r.comm_split(parent->comm, color, key, &c, nullptr)) {
    rccl_fail("ncclCommSplit", e);
    return nullptr;
  }
  // the new communicator's rank / size (ranks of this color ordered by key), as RCCL reports them; -1 when
  // this RCCL lacks ncclCommUserRank / ncclCommCount
  auto* pc = new ptzba_comm_s();
  pc->comm = c;
  pc->rank = -1;
  pc->world = -1;
  pc->device = parent->device;
  int v = 0;
  if (r.user_rank && r.user_rank(c, &v) == 0) pc->rank = v;
  if (r.count && r.count(c, &v) == 0) pc->world = v;
  return pc;
}

int ptzba_comm_info(ptzba_comm c, int32_t* rank, int32_t* world) {
  if (!c) return ptzba::fail("null communicator");
  if (rank) *rank = c->rank;
  if (world) *world = c->world;
  return 0;
}

int ptzba_comm_allreduce(ptzba_comm c, double* dev_buf, int64_t count, void* hip_stream) {
  if (!c || !c->comm) return ptzba::fail("null communicator");
  if (count < 0 || (count > 0 && !dev_buf)) return ptzba::fail("bad buffer");
  if (count == 0) return 0;
  Rccl& r = rccl();
  if (int e = r.all_reduce(dev_buf, dev_buf, (size_t)count, NCCL_FLOAT64, NCCL_SUM, c->comm, (hipStream_t)hip_stream))
    return rccl_fail("ncclAllReduce", e);
  return 0;
}
