/* Test double of the RCCL entry points libptzba's communicator loads at run time (csrc/comm.cpp), for the CPU
 * plumbing test (tests/test_comm_stub.py): no GPU, buffers are host memory, and an all-reduce of a rank's
 * buffer returns it times the communicator size (the sum of `world` identical contributions). */
#include <stdlib.h>
#include <string.h>

typedef struct { char internal[128]; } ncclUniqueId;
typedef struct { int nranks, rank, color; } stub_comm;
static int uid_calls = 0;

int ncclGetUniqueId(ncclUniqueId* id) {
  memset(id, 0, sizeof(*id));
  strcpy(id->internal, "stub-rccl-unique-id");
  id->internal[100] = (char)(++uid_calls);
  return 0;
}
int ncclCommInitRank(void** comm, int nranks, ncclUniqueId id, int rank) {
  if (strcmp(id.internal, "stub-rccl-unique-id") != 0) return 4; /* ncclInvalidArgument */
  if (rank < 0 || rank >= nranks) return 4;
  stub_comm* c = (stub_comm*)malloc(sizeof(stub_comm));
  c->nranks = nranks; c->rank = rank; c->color = -1;
  *comm = c;
  return 0;
}
int ncclCommSplit(void* comm, int color, int key, void** newcomm, void* config) {
  (void)config;
  stub_comm* p = (stub_comm*)comm;
  stub_comm* c = (stub_comm*)malloc(sizeof(stub_comm));
  c->nranks = (p->nranks + 1) / 2; c->rank = key % c->nranks; c->color = color;
  *newcomm = c;
  return 0;
}
int ncclCommDestroy(void* comm) { free(comm); return 0; }
int ncclCommUserRank(void* comm, int* rank) { *rank = ((stub_comm*)comm)->rank; return 0; }
int ncclCommCount(void* comm, int* count) { *count = ((stub_comm*)comm)->nranks; return 0; }
int ncclAllReduce(const void* send, void* recv, size_t count, int dtype, int op, void* comm, void* stream) {
  (void)stream;
  if (dtype != 8 || op != 0) return 4; /* ncclFloat64, ncclSum */
  const double* s = (const double*)send;
  double* r = (double*)recv;
  const int n = ((stub_comm*)comm)->nranks;
  for (size_t i = 0; i < count; ++i) r[i] = s[i] * n;
  return 0;
}
const char* ncclGetErrorString(int e) { return e == 4 ? "invalid argument (stub)" : "stub error"; }
