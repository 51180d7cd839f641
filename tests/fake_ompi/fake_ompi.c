/* TEST INFRASTRUCTURE ONLY -- never shipped, never loaded by the product except in its tests.
 *
 * A one-rank stand-in for an Open MPI library, exporting the Open MPI ABI symbol set that the
 * product's fcomm bridge resolves at run time (iterative-solver_amd/host/mpi_bridge.cpp, the
 * Impl<void*> branch): handles are the addresses of predefined objects (ompi_mpi_comm_world,
 * ompi_mpi_double, ompi_mpi_op_sum, ...), MPI_IN_PLACE is (void*)1, MPI_COMM_TYPE_SHARED is 0,
 * MPI_Comm_f2c / MPI_Comm_c2f are functions with the Fortran handles 0 (world), 1 (self), 2 (null).
 * The reference converts the caller's Fortran handle with MPI_Comm_f2c
 * (src/molpro/linalg/IterativeSolverCMPI.cpp:169); Open MPI is a common Molpro MPI.
 *
 * Every call checks that it received this ABI's handles (a predefined object of the right kind, the
 * in-place marker, the shared split type, a live communicator) and counts it; fake_ompi_count()
 * reports the counters, and "bad" counts the calls that did not hold to the ABI.  One rank: sums and
 * gathers are copies. */
#include <string.h>

struct fake_obj {
  char body[256]; /* Open MPI's predefined objects are structs; only their addresses are handles */
};

struct fake_obj ompi_mpi_comm_world, ompi_mpi_comm_self, ompi_mpi_comm_null;
struct fake_obj ompi_mpi_double, ompi_mpi_byte, ompi_mpi_op_sum, ompi_mpi_info_null;

#define NSPLIT 64
static struct fake_obj split_comms[NSPLIT];
static int split_live[NSPLIT];
static int nsplit;
static int initialized, finalized;
static long c_allreduce, c_in_place, c_allgather, c_bcast, c_split, c_free, c_f2c, c_c2f, c_init, c_finalize, c_bad;

static int live_split(const void* c) {
  for (int i = 0; i < nsplit; ++i)
    if (c == &split_comms[i]) return split_live[i];
  return 0;
}
static int is_comm(const void* c) { return c == &ompi_mpi_comm_world || c == &ompi_mpi_comm_self || live_split(c); }
static int bad(void) {
  ++c_bad;
  return 1;
}
static int usable(void) { return initialized && !finalized; }

long fake_ompi_count(const char* what) {
  const char* names[] = {"allreduce", "in_place", "allgather", "bcast", "split", "free",
                         "f2c", "c2f", "init", "finalize", "bad"};
  long* vals[] = {&c_allreduce, &c_in_place, &c_allgather, &c_bcast, &c_split, &c_free,
                  &c_f2c, &c_c2f, &c_init, &c_finalize, &c_bad};
  for (unsigned i = 0; i < sizeof(names) / sizeof(names[0]); ++i)
    if (!strcmp(what, names[i])) return *vals[i];
  return -1;
}

int MPI_Initialized(int* flag) {
  *flag = initialized;
  return 0;
}
int MPI_Finalized(int* flag) {
  *flag = finalized;
  return 0;
}
int MPI_Init(int* argc, char*** argv) {
  (void)argc;
  (void)argv;
  if (initialized) return bad();
  ++c_init;
  initialized = 1;
  return 0;
}
int MPI_Finalize(void) {
  if (!usable()) return bad();
  ++c_finalize;
  finalized = 1;
  return 0;
}
int MPI_Comm_size(void* comm, int* size) {
  if (!usable() || !is_comm(comm)) return bad();
  *size = 1;
  return 0;
}
int MPI_Comm_rank(void* comm, int* rank) {
  if (!usable() || !is_comm(comm)) return bad();
  *rank = 0;
  return 0;
}
int MPI_Allreduce(const void* send, void* recv, int count, void* dtype, void* op, void* comm) {
  if (!usable() || count < 0 || dtype != &ompi_mpi_double || op != &ompi_mpi_op_sum || !is_comm(comm)) return bad();
  ++c_allreduce;
  if (send == (const void*)1)
    ++c_in_place; /* MPI_IN_PLACE: recv holds this rank's contribution, and the sum of one rank */
  else
    memcpy(recv, send, (size_t)count * sizeof(double));
  return 0;
}
int MPI_Allgather(const void* send, int scount, void* stype, void* recv, int rcount, void* rtype, void* comm) {
  if (!usable() || scount < 0 || scount != rcount || stype != &ompi_mpi_byte || rtype != &ompi_mpi_byte ||
      !is_comm(comm) || send == (const void*)1)
    return bad();
  ++c_allgather;
  memcpy(recv, send, (size_t)scount);
  return 0;
}
int MPI_Bcast(void* buf, int count, void* dtype, int root, void* comm) {
  (void)buf;
  if (!usable() || count < 0 || dtype != &ompi_mpi_byte || root != 0 || !is_comm(comm)) return bad();
  ++c_bcast;
  return 0;
}
int MPI_Comm_split_type(void* comm, int split_type, int key, void* info, void** newcomm) {
  (void)key;
  if (!usable() || !is_comm(comm) || split_type != 0 /* MPI_COMM_TYPE_SHARED */ || info != &ompi_mpi_info_null ||
      nsplit == NSPLIT)
    return bad();
  ++c_split;
  split_live[nsplit] = 1;
  *newcomm = &split_comms[nsplit++];
  return 0;
}
int MPI_Comm_free(void** comm) {
  if (!usable() || !live_split(*comm)) return bad(); /* predefined communicators are never freed */
  ++c_free;
  split_live[(struct fake_obj*)*comm - split_comms] = 0;
  *comm = &ompi_mpi_comm_null;
  return 0;
}
void* MPI_Comm_f2c(int f) {
  ++c_f2c;
  if (f == 0) return &ompi_mpi_comm_world;
  if (f == 1) return &ompi_mpi_comm_self;
  if (f == 2) return &ompi_mpi_comm_null;
  if (f >= 3 && f < 3 + nsplit && split_live[f - 3]) return &split_comms[f - 3];
  return 0; /* Open MPI's f2c of an unknown index: NULL */
}
int MPI_Comm_c2f(void* c) {
  ++c_c2f;
  if (c == &ompi_mpi_comm_world) return 0;
  if (c == &ompi_mpi_comm_self) return 1;
  if (c == &ompi_mpi_comm_null) return 2;
  for (int i = 0; i < nsplit; ++i)
    if (c == &split_comms[i]) return 3 + i;
  return -1;
}
