// The reference's reverse-communication C API (src/molpro/linalg/IterativeSolverC.h:6-73,
// IterativeSolverCMPI.cpp:158-534) over the HBM handlers: R arrives as host arrays and is staged
// into HBM vectors for each call; Q, D and every subspace operation stay on the device.
#include "iterative_solver_c.h"

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <limits>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <tuple>
#include <type_traits>
#include <vector>

#include "itsolv_hbm/hbm_handlers.h"
#include "itsolv_hbm/solver_factory.h"
#include "itsolv_hbm/solvers.h"
#include "mpi_bridge.h"

using molpro::linalg::hbm::check;
using molpro::linalg::hbm::Device;
using molpro::linalg::hbm::SparseP;
using molpro::linalg::hbm::Vec;
namespace it = molpro::linalg::itsolv;

namespace {

using Solver = it::IterativeSolverTemplate<Vec, Vec, SparseP>;
using Davidson = it::LinearEigensystemDavidson<Vec, Vec, SparseP>;
using RSPT = it::LinearEigensystemRSPT<Vec, Vec, SparseP>;
using DIIS = it::NonLinearEquationsDIIS<Vec, Vec, SparseP>;
using LinEq = it::LinearEquationsDavidson<Vec, Vec, SparseP>;
using BFGS = it::OptimizeBFGS<Vec, Vec, SparseP>;
using SD = it::OptimizeSD<Vec, Vec, SparseP>;
typedef void (*Apply_on_p_fort)(const double*, double*, const size_t, const size_t*);

thread_local std::string g_error;
ssp_ctx* g_user_ctx = nullptr;
bool g_throw = true;

struct Instance {
  uint64_t id = 0;  // IterativeSolverHbmInstanceId: lets a binding finalize its own instance
  std::shared_ptr<Device> dev;
  std::unique_ptr<Solver> solver;
  size_t dimension = 0, offset = 0, local = 0;
  std::vector<Vec> rp, ra;  // HBM staging of the caller's R vectors (grown on demand)
  Apply_on_p_fort apply_on_p_fort = nullptr;
  std::unique_ptr<Vec> diagonals;
  bool has_values = false;
  bool has_eigenvalues = false;
};
// The instance stack (reference IterativeSolverCMPI.cpp: std::stack<Instance>); the back is the top,
// the only active instance.  A vector, so that IterativeSolverHbmFinalizeInstance can also remove
// an instance below the top whose owner has gone away.  Instances are heap-held: the P-space
// callback keeps a pointer to its instance across pushes and erasures.
std::vector<std::unique_ptr<Instance>> instances;
uint64_t g_next_id = 1;

Instance& top() {
  if (instances.empty()) throw std::runtime_error("IterativeSolver not initialised properly");
  return *instances.back();
}
void push(Instance&& in) {
  in.id = g_next_id++;
  instances.push_back(std::make_unique<Instance>(std::move(in)));
}

// Without IterativeSolverHbmSetContext the node-local rank a launcher exports (torchrun, Open MPI,
// MPICH, Slurm) picks the device, so independent processes on one node spread over its GPUs
// instead of all landing on device 0.
int default_device() {
  for (const char* var : {"LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", "SLURM_LOCALID"}) {
    const char* s = std::getenv(var);
    if (!s || !*s) continue;
    const int r = std::atoi(s), n = ssp_device_count();
    return (r >= 0 && n > 0) ? r % n : 0;
  }
  return 0;
}

// A context attached to the ranks of an MPI communicator (mpi_bridge.h), with the transport's state.
class BridgedDevice : public Device {
 public:
  BridgedDevice(int device, int64_t fcomm) : Device(device) {
    m_link = molpro::linalg::hbm::mpi::attach(ctx(), fcomm, nullptr);
  }

 private:
  std::shared_ptr<void> m_link;
};
// One bridged context per communicator, shared by the instances that use it and released with the
// last of them (every rank creates and finalizes instances in the same order, so the collective
// attach happens on all ranks together).
std::map<int64_t, std::weak_ptr<Device>> g_bridged;

// The instance's device and ranks.  In order:
//  - the context set by IterativeSolverHbmSetContext;
//  - the communicator fcomm names, when the process has an initialised MPI library (reference
//    IterativeSolverCMPI.cpp:169, :205, :234, :254 -- MPI_Comm_f2c(fcomm)): a context attached to its
//    ranks, on the device of the rank's place among them on its node (one rank: a private context);
//  - otherwise a private single-rank context on the node-local rank's device.
std::shared_ptr<Device> make_device(int64_t fcomm) {
  namespace mpi = molpro::linalg::hbm::mpi;
  if (g_user_ctx) return std::make_shared<Device>(g_user_ctx, true);
  mpi::Bridge* b = mpi::bridge();
  if (b && b->active() && b->valid(fcomm)) {
    if (b->size(fcomm) <= 1) return std::make_shared<Device>(mpi::device_for(fcomm));
    if (auto d = g_bridged[fcomm].lock()) return d;
    auto d = std::make_shared<BridgedDevice>(mpi::device_for(fcomm), fcomm);
    g_bridged[fcomm] = d;
    return d;
  }
  return std::make_shared<Device>(default_device());
}

void setup(Instance& in, size_t n, size_t* range_begin, size_t* range_end) {
  in.dimension = n;
  std::tie(in.offset, in.local) = in.dev->shard(n);
  // reference DistrArrayDefaultRange (IterativeSolverCMPI.cpp:80-89)
  if (range_begin) *range_begin = in.offset;
  if (range_end) *range_end = in.offset + in.local;
}

void ensure_r(Instance& in, size_t nvec) {
  while (in.rp.size() < nvec) {
    in.rp.emplace_back(in.dev, in.dimension);
    in.ra.emplace_back(in.dev, in.dimension);
  }
}

// This rank's range of host vectors [k*dimension + offset, +local) <-> HBM.
void upload(Instance& in, std::vector<Vec>& v, size_t nvec, const double* host) {
  for (size_t k = 0; k < nvec; ++k)
    check(ssp_upload(in.dev->ctx(), v[k].data_wo(), host + k * in.dimension + in.offset, in.local), "ssp_upload");
}
void download(Instance& in, std::vector<Vec>& v, size_t nvec, double* host) {
  for (size_t k = 0; k < nvec; ++k)
    check(ssp_download(in.dev->ctx(), host + k * in.dimension + in.offset, v[k].data(), in.local), "ssp_download");
}

// reference DistrArraySynchronize / gather_all (IterativeSolverCMPI.cpp:133-139): every rank
// receives every rank's range of each vector.
void synchronize(Instance& in, size_t nvec, double* host) {
  const int nr = in.dev->nranks();
  if (nr <= 1 || nvec == 0) return;
  const size_t chunk = (in.dimension + size_t(nr) - 1) / size_t(nr);  // >= the largest shard
  std::vector<double> send(chunk), recv(chunk * size_t(nr));
  for (size_t k = 0; k < nvec; ++k) {
    double* vec = host + k * in.dimension;
    std::memcpy(send.data(), vec + in.offset, in.local * sizeof(double));
    check(ssp_allgather_host(in.dev->ctx(), send.data(), recv.data(), chunk * sizeof(double)), "ssp_allgather_host");
    for (int r = 0; r < nr; ++r) {
      size_t off = 0, len = 0;
      check(ssp_shard_range(in.dimension, nr, r, &off, &len), "ssp_shard_range");
      std::memcpy(vec + off, recv.data() + size_t(r) * chunk, len * sizeof(double));
    }
  }
}

it::VecRef<Vec> first(std::vector<Vec>& v, size_t n) { return it::wrap(v.begin(), v.begin() + long(n)); }

it::Verbosity verbosity_of(int v) {
  return v <= 0 ? it::Verbosity::None : v == 1 ? it::Verbosity::Summary : v == 2 ? it::Verbosity::Iteration
                                                                                : it::Verbosity::Detailed;
}

// Runs one API call.  Errors are thrown as the reference's extern "C" functions throw; with
// IterativeSolverHbmSetThrow(0) they are recorded for IterativeSolverHbmLastError() instead and the
// call returns a zero value (for callers that cannot unwind C++ exceptions: ctypes, Fortran).
template <class F>
auto guarded(F&& f) -> decltype(f()) {
  using T = decltype(f());
  g_error.clear();
  try {
    return f();
  } catch (const std::exception& e) {
    g_error = e.what();
    if (g_throw) throw;
  }
  if constexpr (!std::is_void_v<T>) return T{};
}

molpro::linalg::hbm::mpi::Bridge* active_mpi() {
  auto* b = molpro::linalg::hbm::mpi::bridge();
  return b && b->active() ? b : nullptr;
}

}  // namespace

extern "C" {

int IterativeSolverHbmSetThrow(int enable) {
  g_throw = enable != 0;
  return 0;
}

int IterativeSolverHbmSetContext(ssp_ctx* ctx) {
  g_user_ctx = ctx;
  return 0;
}

const char* IterativeSolverHbmLastError(void) { return g_error.c_str(); }

int IterativeSolverHbmStatistics(int* iterations, int* r_creations, int* q_creations) {
  if (instances.empty()) return 1;
  const auto& s = instances.back()->solver->statistics();
  if (iterations) *iterations = s.iterations;
  if (r_creations) *r_creations = s.r_creations;
  if (q_creations) *q_creations = s.q_creations;
  return 0;
}

void IterativeSolverLinearEigensystemInitialize(size_t nQ, size_t nroot, size_t* range_begin, size_t* range_end,
                                                double thresh, double thresh_value, int hermitian, int verbosity,
                                                const char* fname, int64_t fcomm, const char* algorithm,
                                                const char* options) {
  guarded([&] {
    (void)fname;
    Instance in;
    in.dev = make_device(fcomm);
    // method dispatch and option parsing as the reference's create_LinearEigensystem (SolverFactory.h:114-125)
    auto solver = it::create_LinearEigensystem(algorithm ? algorithm : "", options ? options : "",
                                               molpro::linalg::hbm::make_handlers());
    solver->set_n_roots(nroot);  // every method (reference IterativeSolverCMPI.cpp:176)
    if (auto* d = dynamic_cast<Davidson*>(solver.get())) d->set_hermiticity(hermitian != 0);
    solver->set_verbosity(verbosity_of(verbosity));
    solver->set_convergence_threshold(thresh);
    solver->set_convergence_threshold_value(thresh_value);
    in.solver = std::move(solver);
    in.has_eigenvalues = true;
    setup(in, nQ, range_begin, range_end);
    push(std::move(in));
  });
}

void IterativeSolverLinearEquationsInitialize(size_t n, size_t nroot, size_t* range_begin, size_t* range_end,
                                              const double* rhs, double aughes, double thresh, double thresh_value,
                                              int hermitian, int verbosity, const char* fname, int64_t fcomm,
                                              const char* algorithm, const char* options) {
  guarded([&] {
    (void)fname;
    auto made = it::create_LinearEquations(algorithm ? algorithm : "", options ? options : "",
                                           molpro::linalg::hbm::make_handlers());
    std::unique_ptr<LinEq> solver(static_cast<LinEq*>(made.release()));
    Instance in;
    in.dev = make_device(fcomm);
    setup(in, n, range_begin, range_end);
    // reference IterativeSolverCMPI.cpp:199-225: rhs as R vectors, then options
    std::vector<Vec> b;
    for (size_t r = 0; r < nroot; ++r) {
      b.emplace_back(in.dev, n);
      check(ssp_upload(in.dev->ctx(), b.back().data_wo(), rhs + r * n + in.offset, in.local), "ssp_upload");
    }
    solver->set_hermiticity(hermitian != 0);
    solver->set_n_roots(nroot);
    solver->add_equations(b);
    solver->set_convergence_threshold(thresh);
    solver->set_convergence_threshold_value(thresh_value);
    if (aughes > 0) solver->set_augmented_hessian(aughes);
    solver->set_verbosity(verbosity_of(verbosity));
    in.solver = std::move(solver);
    push(std::move(in));
  });
}

void IterativeSolverNonLinearEquationsInitialize(size_t n, size_t* range_begin, size_t* range_end, double thresh,
                                                 int verbosity, const char* fname, int64_t fcomm,
                                                 const char* algorithm, const char* options) {
  guarded([&] {
    (void)fname;
    Instance in;
    in.dev = make_device(fcomm);
    auto solver = it::create_NonLinearEquations(algorithm ? algorithm : "", options ? options : "",
                                                molpro::linalg::hbm::make_handlers());
    solver->set_convergence_threshold(thresh);
    solver->set_verbosity(verbosity_of(verbosity));
    in.solver = std::move(solver);
    setup(in, n, range_begin, range_end);
    push(std::move(in));
  });
}

void IterativeSolverOptimizeInitialize(size_t n, size_t* range_begin, size_t* range_end, double thresh,
                                       double thresh_value, int verbosity, int minimize, const char* fname,
                                       int64_t fcomm, const char* algorithm, const char* options) {
  guarded([&] {
    (void)fname;
    (void)minimize;  // ignored, as the reference does (IterativeSolverCMPI.cpp:250-268)
    Instance in;
    in.dev = make_device(fcomm);
    auto solver = it::create_Optimize(algorithm ? algorithm : "", options ? options : "",
                                      molpro::linalg::hbm::make_handlers());
    // reference IterativeSolverCMPI.cpp:245-264
    solver->set_n_roots(1);
    solver->set_convergence_threshold(thresh);
    solver->set_convergence_threshold_value(thresh_value);
    solver->set_verbosity(verbosity_of(verbosity));
    in.solver = std::move(solver);
    in.has_values = true;
    setup(in, n, range_begin, range_end);
    push(std::move(in));
  });
}

void IterativeSolverFinalize(void) {
  guarded([] {
    if (!instances.empty()) instances.pop_back();
  });
}

uint64_t IterativeSolverHbmInstanceId(void) { return instances.empty() ? 0 : instances.back()->id; }

int IterativeSolverHbmFinalizeInstance(uint64_t id) {
  for (auto it = instances.begin(); it != instances.end(); ++it)
    if ((*it)->id == id) {
      instances.erase(it);
      return 0;
    }
  return 1;
}

size_t IterativeSolverAddVector(size_t buffer_size, double* parameters, double* action, int sync) {
  return guarded([&] {
    auto& in = top();
    ensure_r(in, buffer_size);
    upload(in, in.rp, buffer_size, parameters);
    upload(in, in.ra, buffer_size, action);
    // Non-linear solvers take one vector through their own add_vector (for DIIS: the residual norm,
    // the convergence flag and the least-important-vector deletion, NonLinearEquationsDIIS.h:83-102),
    // as IterativeSolverTemplate::solve does for them (:379-382).  The reference's C layer reaches
    // the generic vector-list overload instead, which skips that logic.
    const size_t nwork = in.solver->nonlinear() && buffer_size >= 1
                             ? size_t(in.solver->add_vector(in.rp[0], in.ra[0], 0.0))
                             : size_t(in.solver->add_vector(first(in.rp, buffer_size), first(in.ra, buffer_size)));
    // The reference's R vectors are views of these host arrays, so every vector the solver wrote
    // (solutions and residuals of all roots, batch by batch) reaches the caller; sync gathers the
    // working set (IterativeSolverCMPI.cpp:302-306).
    download(in, in.rp, buffer_size, parameters);
    download(in, in.ra, buffer_size, action);
    const size_t nws = std::min(in.solver->working_set().size(), buffer_size);
    if (sync) {
      synchronize(in, nws, parameters);
      synchronize(in, nws, action);
    }
    return nwork;
  });
}

void IterativeSolverSolution(int nroot, int* roots, double* parameters, double* action, int sync) {
  guarded([&] {
    auto& in = top();
    const size_t n = size_t(nroot);
    ensure_r(in, n);
    std::vector<int> r(roots, roots + nroot);
    in.solver->solution(r, first(in.rp, n), first(in.ra, n));
    download(in, in.rp, n, parameters);
    download(in, in.ra, n, action);
    if (sync) {
      synchronize(in, n, parameters);
      synchronize(in, n, action);
    }
  });
}

size_t IterativeSolverAddValue(double value, double* parameters, double* action, int sync) {
  return guarded([&]() -> size_t {
    auto& in = top();
    ensure_r(in, 1);
    upload(in, in.rp, 1, parameters);
    upload(in, in.ra, 1, action);
    // reference IterativeSolverCMPI.cpp:270-298: working set of one, or none when line-searching
    const int r = in.solver->add_vector(in.rp[0], in.ra[0], value);
    download(in, in.rp, 1, parameters);
    download(in, in.ra, 1, action);
    if (sync) {
      synchronize(in, 1, parameters);
      synchronize(in, 1, action);
    }
    return r > 0 ? 1 : 0;
  });
}

size_t IterativeSolverEndIteration(size_t buffer_size, double* solution, double* residual, int sync) {
  return guarded([&] {
    auto& in = top();
    ensure_r(in, buffer_size);
    upload(in, in.rp, buffer_size, solution);
    upload(in, in.ra, buffer_size, residual);
    const size_t result = in.solver->end_iteration(first(in.rp, buffer_size), first(in.ra, buffer_size));
    download(in, in.rp, buffer_size, solution);
    download(in, in.ra, buffer_size, residual);
    const size_t nws = std::min(in.solver->working_set().size(), buffer_size);
    if (sync) {
      synchronize(in, nws, solution);
      synchronize(in, nws, residual);
    }
    return result;
  });
}

int IterativeSolverEndIterationNeeded(void) {
  return guarded([] { return top().solver->end_iteration_needed() ? 1 : 0; });
}

size_t IterativeSolverAddP(size_t buffer_size, size_t nP, const size_t* offsets, const size_t* indices,
                           const double* coefficients, const double* pp, double* parameters, double* action, int sync,
                           void (*func)(const double*, double*, const size_t, const size_t*)) {
  return guarded([&] {
    auto& in = top();
    in.apply_on_p_fort = func;
    ensure_r(in, buffer_size);
    upload(in, in.rp, buffer_size, parameters);
    upload(in, in.ra, buffer_size, action);
    std::vector<SparseP> pvectors(nP);
    for (size_t p = 0; p < nP; ++p)
      for (size_t k = offsets[p]; k < offsets[p + 1]; ++k) pvectors[p].emplace(indices[k], coefficients[k]);
    const size_t npp = (in.solver->dimensions().oP + nP) * nP;  // reference IterativeSolverCMPI.cpp:417
    std::vector<double> ppm(pp, pp + npp);
    Instance* ip = &in;
    // reference apply_on_p_c (IterativeSolverCMPI.cpp:141-157): the caller's routine adds the
    // P-space contributions to this rank's range of the action vectors, laid out as host arrays.
    auto apply = [ip](const std::vector<std::vector<double>>& pvecs, const it::CVecRef<SparseP>&,
                      const it::VecRef<Vec>& act) {
      Instance& I = *ip;
      const size_t nu = pvecs.size();
      std::vector<double> flat;
      for (const auto& v : pvecs) flat.insert(flat.end(), v.begin(), v.end());
      std::vector<size_t> ranges;
      for (size_t k = 0; k < nu; ++k) {
        ranges.push_back(I.offset);
        ranges.push_back(I.offset + I.local);
      }
      std::vector<double> host(nu * I.dimension, 0.0);
      for (size_t k = 0; k < nu; ++k)
        check(ssp_download(I.dev->ctx(), host.data() + k * I.dimension + I.offset, act[k].get().data(), I.local),
              "ssp_download");
      I.apply_on_p_fort(flat.data(), host.data() + I.offset, nu, ranges.data());
      for (size_t k = 0; k < nu; ++k)
        check(ssp_upload(I.dev->ctx(), act[k].get().data_wo(), host.data() + k * I.dimension + I.offset, I.local),
              "ssp_upload");
    };
    const size_t nwork =
        in.solver->add_p(it::cwrap(pvectors), ppm, first(in.rp, buffer_size), first(in.ra, buffer_size), apply);
    download(in, in.rp, buffer_size, parameters);
    download(in, in.ra, buffer_size, action);
    if (sync) {
      synchronize(in, std::min(nwork, buffer_size), parameters);
      synchronize(in, std::min(nwork, buffer_size), action);
    }
    return nwork;
  });
}

void IterativeSolverErrors(double* errors) {
  guarded([&] {
    size_t k = 0;
    for (double e : top().solver->errors()) errors[k++] = e;
  });
}

void IterativeSolverEigenvalues(double* eigenvalues) {
  guarded([&] {
    if (auto* d = dynamic_cast<Davidson*>(top().solver.get())) {
      size_t k = 0;
      for (double e : d->eigenvalues()) eigenvalues[k++] = e;
    } else if (auto* r = dynamic_cast<RSPT*>(top().solver.get())) {
      size_t k = 0;
      for (double e : r->eigenvalues()) eigenvalues[k++] = e;
    }
  });
}

void IterativeSolverWorkingSetEigenvalues(double* eigenvalues) {
  guarded([&] {
    if (auto* d = dynamic_cast<Davidson*>(top().solver.get())) {
      size_t k = 0;
      for (double e : d->working_set_eigenvalues()) eigenvalues[k++] = e;
    } else if (auto* r = dynamic_cast<RSPT*>(top().solver.get())) {
      size_t k = 0;
      for (double e : r->working_set_eigenvalues()) eigenvalues[k++] = e;
    }
  });
}

// reference IterativeSolverTemplate::suggest_p (IterativeSolverTemplate.h:238-241) returns no indices.
size_t IterativeSolverSuggestP(const double*, const double*, size_t, double, size_t*) { return 0; }

void IterativeSolverPrintStatistics(void) {
  guarded([] { std::cout << top().solver->statistics() << std::endl; });
}

int IterativeSolverNonLinear(void) {
  return guarded([] { return top().solver->nonlinear() ? 1 : 0; });
}
int IterativeSolverHasValues(void) {
  return guarded([] { return top().has_values ? 1 : 0; });
}
int IterativeSolverHasEigenvalues(void) {
  return guarded([] { return top().has_eigenvalues ? 1 : 0; });
}

void IterativeSolverSetDiagonals(const double* diagonals) {
  guarded([&] {
    auto& in = top();
    in.diagonals = std::make_unique<Vec>(in.dev, in.dimension);
    check(ssp_upload(in.dev->ctx(), in.diagonals->data_wo(), diagonals + in.offset, in.local), "ssp_upload");
  });
}

void IterativeSolverDiagonals(double* diagonals) {
  guarded([&] {
    auto& in = top();
    if (!in.diagonals) throw std::runtime_error("IterativeSolverDiagonals: no diagonals set");
    check(ssp_download(in.dev->ctx(), diagonals + in.offset, in.diagonals->data(), in.local), "ssp_download");
  });
}

// reference IterativeSolverTemplate::value (IterativeSolverTemplate.h:312-315): NaN unless the
// subspace carries a value block (Optimize only).
double IterativeSolverValue(void) {
  return guarded([] { return top().solver->value(); });
}

int IterativeSolverVerbosity(void) {
  return guarded([] {
    switch (top().solver->get_verbosity()) {
      case it::Verbosity::None: return 0;
      case it::Verbosity::Summary: return 1;
      case it::Verbosity::Iteration: return 2;
      case it::Verbosity::Detailed: return 3;
    }
    return -1;
  });
}

int IterativeSolverMaxIter(void) {
  return guarded([] { return top().solver->get_max_iter(); });
}
void IterativeSolverSetMaxIter(int max_iter) {
  guarded([&] { top().solver->set_max_iter(max_iter); });
}

size_t IterativeSolverHbmNRoots(void) {
  return instances.empty() ? 0 : instances.back()->solver->n_roots();
}

// reference IterativeSolverCMPI.cpp:481-534 (mpi::comm_global / comm_self / size_global /
// rank_global / init / finalize), through the caller's MPI library when the process has one
// (mpi_bridge.h).  Without MPI the handles are 0 and size and rank are those of the context the next
// instance will use.  init calls MPI_Init when MPI is loaded but not initialised, and finalize undoes
// only that; both return 0 (MPI_SUCCESS) without MPI.  The reference's Fortran module binds the
// size/rank functions as IterativeSolver_mpi_size_global / _mpi_rank_global (IterativeSolverF.F90:50-57)
// while its C++ defines IterativeSolver_mpisize_global / _mpirank_global: both spellings exist here.
int64_t IterativeSolver_mpicomm_global(void) { return active_mpi() ? active_mpi()->world() : 0; }
int64_t IterativeSolver_mpicomm_self(void) { return active_mpi() ? active_mpi()->self() : 0; }
int64_t mpicomm_global(void) { return IterativeSolver_mpicomm_global(); }
int64_t mpicomm_self(void) { return IterativeSolver_mpicomm_self(); }
int64_t IterativeSolver_mpisize_global(void) {
  if (g_user_ctx) return ssp_ctx_nranks(g_user_ctx);
  auto* b = active_mpi();
  return b ? b->size(b->world()) : 1;
}
int64_t IterativeSolver_mpirank_global(void) {
  if (g_user_ctx) return ssp_ctx_rank(g_user_ctx);
  auto* b = active_mpi();
  return b ? b->rank(b->world()) : 0;
}
int64_t IterativeSolver_mpi_size_global(void) { return IterativeSolver_mpisize_global(); }
int64_t IterativeSolver_mpi_rank_global(void) { return IterativeSolver_mpirank_global(); }
int IterativeSolver_mpi_init(void) {
  auto* b = molpro::linalg::hbm::mpi::bridge();
  return b ? b->init() : 0;
}
int IterativeSolver_mpi_finalize(void) {
  auto* b = molpro::linalg::hbm::mpi::bridge();
  return b ? b->finalize() : 0;
}

int IterativeSolverHbmMpiActive(void) { return active_mpi() ? 1 : 0; }

int IterativeSolverHbmMpiAttach(ssp_ctx* ctx, int64_t fcomm, const char* transport) {
  return guarded([&] {
    if (!ctx) throw std::invalid_argument("IterativeSolverHbmMpiAttach: null context");
    auto link = molpro::linalg::hbm::mpi::attach(ctx, fcomm, transport);
    // The caller owns ctx and detaches it by destroying it; the transport's callback state stays
    // with the process (a few bytes per attach).
    static std::vector<std::shared_ptr<void>> keep;
    if (link) keep.push_back(std::move(link));
    return 0;
  }) == 0 && g_error.empty() ? 0 : 1;
}

}  // extern "C"
