/*
 * iterative_solver_c.h — the reference's reverse-communication C API (what Molpro's Fortran and
 * the Python extension bind) on the MI355X back end, exported by libitsolv_hbm.so.
 *
 * Every declaration below has the name, argument list and meaning of the reference's
 * src/molpro/linalg/IterativeSolverC.h:6-73 (implementation IterativeSolverCMPI.cpp:158-534):
 *  - R vectors are the caller's host arrays, `buffer_size` vectors of length `dimension` stored
 *    one after the other; this rank works on [range_begin, range_end) of each (the reference's
 *    make_distribution_spread_remainder layout), returned by the *Initialize calls;
 *  - with `sync` != 0 the updated vectors are gathered in full on every rank;
 *  - Q (and D) vectors live in HBM instead of DistrArrayFile: every subspace operation runs on the
 *    device, and R crosses PCIe once per call in each direction;
 *  - the solver instances form a stack; only the top one is active (as in the reference).
 *
 * Differences:
 *  - `fcomm` (a Fortran MPI communicator, reference IterativeSolverCMPI.cpp:169 MPI_Comm_f2c(fcomm))
 *    is bridged at run time to the MPI library the calling process has loaded and initialised
 *    (libitsolv_hbm.so does not link MPI; iterative-solver_amd/host/mpi_bridge.h).  With more than
 *    one rank the instance's vectors are sharded over the communicator's ranks exactly as the
 *    reference distributes them (make_distribution_spread_remainder, :79-105), each rank's shard in
 *    the HBM of the device matching its place among the communicator's ranks on its node, and the
 *    reductions / sync gathers run over the transport ITSOLV_HBM_COMM names: "mpi" (default:
 *    MPI_Allreduce / MPI_Allgather on the communicator, the reference's own collectives), "p2p"
 *    (peer-memory device exchange, one node) or "rccl" (RCCL over xGMI, one rank per device).
 *    Precedence: a context set by IterativeSolverHbmSetContext; else fcomm when MPI is initialised in
 *    the process and fcomm names a communicator; else a single-rank context on the device of the
 *    node-local rank the launcher exports (LOCAL_RANK, OMPI_COMM_WORLD_LOCAL_RANK, MPI_LOCALRANKID or
 *    SLURM_LOCALID, first one set, modulo the visible device count; device 0 without any of them).
 *  - Supported algorithms: LinearEigensystem and LinearEquations "Davidson" (or ""),
 *    NonLinearEquations "DIIS" (or ""), Optimize "BFGS" (or "") and "SD"; `minimize` is ignored,
 *    as in the reference (IterativeSolverCMPI.cpp:250-268).
 *  - Davidson instances (LinearEigensystem, LinearEquations) orthogonalise new R vectors by block
 *    Gram-Schmidt (coefficients by forward substitution through the stored overlaps, one gemm_outer
 *    per space): the same projection as the reference's sequential MGS in exact
 *    arithmetic, not bit-identical.  "BLOCK_GRAM_SCHMIDT=false" in the options string restores
 *    the reference's MGS.
 *  - IterativeSolverAddVector on a non-linear solver (DIIS) passes the vector through the solver's
 *    own add_vector (residual norm, convergence flag, least-important-vector deletion), as the
 *    reference's solve() driver does; the reference's C layer reaches the generic vector-list
 *    overload, which skips that logic.
 *  - Errors are thrown as C++ exceptions, exactly as the reference's extern "C" functions do,
 *    unless IterativeSolverHbmSetThrow(0) selects recorded errors (IterativeSolverHbmLastError).
 */
#ifndef ITERATIVE_SOLVER_C_H
#define ITERATIVE_SOLVER_C_H
#include <stddef.h>
#include <stdint.h>

#include "subspace_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

void IterativeSolverLinearEigensystemInitialize(size_t nQ, size_t nroot, size_t* range_begin, size_t* range_end,
                                                double thresh, double thresh_value, int hermitian, int verbosity,
                                                const char* fname, int64_t fcomm, const char* algorithm,
                                                const char* options);
void IterativeSolverLinearEquationsInitialize(size_t n, size_t nroot, size_t* range_begin, size_t* range_end,
                                              const double* rhs, double aughes, double thresh, double thresh_value,
                                              int hermitian, int verbosity, const char* fname, int64_t fcomm,
                                              const char* algorithm, const char* options);
void IterativeSolverNonLinearEquationsInitialize(size_t n, size_t* range_begin, size_t* range_end, double thresh,
                                                 int verbosity, const char* fname, int64_t fcomm,
                                                 const char* algorithm, const char* options);
void IterativeSolverOptimizeInitialize(size_t n, size_t* range_begin, size_t* range_end, double thresh,
                                       double thresh_value, int verbosity, int minimize, const char* fname,
                                       int64_t fcomm, const char* algorithm, const char* options);
void IterativeSolverFinalize(void);
size_t IterativeSolverAddVector(size_t buffer_size, double* parameters, double* action, int sync);
void IterativeSolverSolution(int nroot, int* roots, double* parameters, double* action, int sync);
size_t IterativeSolverAddValue(double value, double* parameters, double* action, int sync);
size_t IterativeSolverEndIteration(size_t buffer_size, double* solution, double* residual, int sync);
int IterativeSolverEndIterationNeeded(void);
size_t IterativeSolverAddP(size_t buffer_size, size_t nP, const size_t* offsets, const size_t* indices,
                           const double* coefficients, const double* pp, double* parameters, double* action, int sync,
                           void (*func)(const double*, double*, const size_t, const size_t*));
void IterativeSolverErrors(double* errors);
void IterativeSolverEigenvalues(double* eigenvalues);
void IterativeSolverWorkingSetEigenvalues(double* eigenvalues);
size_t IterativeSolverSuggestP(const double* solution, const double* residual, size_t maximumNumber, double threshold,
                               size_t* indices);
void IterativeSolverPrintStatistics(void);
int IterativeSolverNonLinear(void);
int IterativeSolverHasValues(void);
int IterativeSolverHasEigenvalues(void);
void IterativeSolverSetDiagonals(const double* diagonals);
void IterativeSolverDiagonals(double* diagonals);
double IterativeSolverValue(void);
int IterativeSolverVerbosity(void);
int IterativeSolverMaxIter(void);
void IterativeSolverSetMaxIter(int max_iter);
int64_t mpicomm_self(void);
int64_t mpicomm_global(void);
int64_t IterativeSolver_mpicomm_global(void);
int64_t IterativeSolver_mpicomm_self(void);
/* IterativeSolverCMPI.cpp:481-534 through the caller's MPI library when it has one: the Fortran
 * handles of MPI_COMM_WORLD / MPI_COMM_SELF (0 without MPI), the world's size and rank (without MPI:
 * those of the context set by IterativeSolverHbmSetContext, else 1 and 0), MPI_Init when MPI is
 * loaded but not initialised, and MPI_Finalize of an MPI initialised that way (0 otherwise).  The
 * _mpi_size_/_mpi_rank_ spellings are the names the reference's Fortran module binds
 * (IterativeSolverF.F90:50-57). */
int64_t IterativeSolver_mpisize_global(void);
int64_t IterativeSolver_mpirank_global(void);
int64_t IterativeSolver_mpi_size_global(void);
int64_t IterativeSolver_mpi_rank_global(void);
int IterativeSolver_mpi_init(void);
int IterativeSolver_mpi_finalize(void);

/* ---- extension: device / communicator selection ----------------------------------------- */
/* Use `ctx` (not owned) for the instances initialised after this call; NULL restores the
 * default (a private single-rank context on the node-local rank's device, see above).  Returns 0. */
int IterativeSolverHbmSetContext(ssp_ctx* ctx);
/* enable = 0: errors are recorded (IterativeSolverHbmLastError, cleared by every call) instead of
 * thrown, and the failing call returns 0 -- for callers that cannot unwind C++ exceptions
 * (ctypes, Fortran).  Default 1 (throw, as the reference does).  Returns 0. */
int IterativeSolverHbmSetThrow(int enable);
/* Statistics of the top instance: iterations, R and Q creations (for tests and reports). */
int IterativeSolverHbmStatistics(int* iterations, int* r_creations, int* q_creations);
const char* IterativeSolverHbmLastError(void);
/* Id (> 0) of the top instance, 0 when there is none.  Ids are unique within the process. */
uint64_t IterativeSolverHbmInstanceId(void);
/* Removes the instance with this id wherever it sits in the stack (a binding whose solver object
 * is destroyed after a newer one was created must not pop the newer one, which
 * IterativeSolverFinalize would).  Returns 0, or 1 when no instance has that id. */
int IterativeSolverHbmFinalizeInstance(uint64_t id);
/* 1 when the process has an MPI library loaded and initialised (MPI_Init done, MPI_Finalize not),
 * i.e. when the *Initialize calls bridge `fcomm`; 0 otherwise. */
int IterativeSolverHbmMpiActive(void);
/* Attaches `ctx` to the ranks of the Fortran MPI communicator `fcomm` over `transport` ("mpi", "p2p",
 * "rccl"; NULL or "" -> ITSOLV_HBM_COMM, else "mpi") -- the attach the *Initialize calls perform for
 * their own contexts, for callers that drive ssp contexts directly.  Collective over fcomm.  Returns
 * 0, or 1 (IterativeSolverHbmLastError) in no-throw mode. */
int IterativeSolverHbmMpiAttach(ssp_ctx* ctx, int64_t fcomm, const char* transport);
/* Number of roots of the top instance (0 when there is none): the length of the arrays
 * IterativeSolverErrors / IterativeSolverEigenvalues fill (used by the Fortran module). */
size_t IterativeSolverHbmNRoots(void);

#ifdef __cplusplus
}
#endif
#endif
