// The reference's MPI communicator argument (`fcomm`, a Fortran handle: IterativeSolverCMPI.cpp:169
// MPI_Comm comm = MPI_Comm_f2c(fcomm)) on the HBM back end, without a link-time MPI dependency.
//
// libitsolv_hbm.so does not link libmpi.  When the calling process has loaded an MPI library and
// initialised it (a Fortran/C program linked with MPI, Python with mpi4py, ctypes with RTLD_GLOBAL),
// the bridge finds its C entry points at run time (dlsym) and:
//  - resolves fcomm to that library's MPI_Comm (MPI_Comm_f2c), and its size and rank;
//  - attaches an ssp context to the communicator's ranks over one of three transports:
//      "mpi"  (default) reductions and gathers are MPI_Allreduce(MPI_SUM) / MPI_Allgather on the
//             communicator itself -- the reference's own collectives (DistrArray.cpp:133-135,
//             gemm.h:179-182, gather_all.h:15-25), so the sum of the ranks' partials has MPI's
//             association, whatever algorithm the library picks;
//      "p2p"  the peer-memory device exchange (ssp_ctx_attach_p2p; one node, any device sharing), its
//             id broadcast from rank 0 with MPI_Bcast;
//      "rccl" RCCL over xGMI (ssp_ctx_attach_comm; one rank per device), id broadcast likewise;
//  - selects the device from the rank's position among the communicator's ranks on its node
//    (MPI_Comm_split_type(MPI_COMM_TYPE_SHARED)), modulo the visible device count.
//
// Two ABIs exist for the handle types: the MPICH ABI (MPICH, Intel MPI, MVAPICH, Cray MPICH; integer
// handles with fixed values) and Open MPI's (pointers to exported objects).  The MPICH ABI is what this
// image carries (/opt/conda, MPICH 3.3.2) and what the tests run; the Open MPI form follows that
// library's documented handle symbols and is untested here.
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>

#include "subspace_hip.h"

namespace molpro::linalg::hbm::mpi {

class Bridge {
 public:
  virtual ~Bridge() = default;
  //! MPI_Init has run and MPI_Finalize has not.
  virtual bool active() = 0;
  //! fcomm names a communicator (not MPI_COMM_NULL, not a non-communicator handle).
  virtual bool valid(int64_t fcomm) = 0;
  virtual int size(int64_t fcomm) = 0;
  virtual int rank(int64_t fcomm) = 0;
  //! This rank's index and the rank count among fcomm's ranks on this node (collective).
  virtual void node(int64_t fcomm, int* node_rank, int* node_size) = 0;
  //! In-place sum of n doubles over fcomm's ranks; 0 on success.
  virtual int allreduce_sum(int64_t fcomm, double* buf, size_t n) = 0;
  //! `bytes` from every rank into recv (size * bytes), rank order; 0 on success.
  virtual int allgather(int64_t fcomm, const void* send, void* recv, size_t bytes) = 0;
  virtual int bcast(int64_t fcomm, void* buf, size_t bytes, int root) = 0;
  //! Fortran handles of MPI_COMM_WORLD / MPI_COMM_SELF (MPI_Comm_c2f).
  virtual int64_t world() = 0;
  virtual int64_t self() = 0;
  //! MPI_Init when not yet initialised (remembered for finalize); MPI_Finalize when initialised here.
  virtual int init() = 0;
  virtual int finalize() = 0;
  virtual const char* abi() const = 0;
};

//! The MPI library loaded in this process, or nullptr when there is none.
Bridge* bridge();

//! Attaches ctx to fcomm's ranks over `transport` ("mpi", "p2p", "rccl"; null or "" -> the
//! ITSOLV_HBM_COMM environment variable, else "mpi").  Collective over fcomm.  The returned object
//! carries the callback state of the "mpi" transport and must outlive every use of ctx; throws
//! std::runtime_error on failure.
std::shared_ptr<void> attach(ssp_ctx* ctx, int64_t fcomm, const char* transport);

//! The device for this rank of fcomm: its node-local index modulo the visible device count.
int device_for(int64_t fcomm);

}  // namespace molpro::linalg::hbm::mpi
