// Solver construction by family and method name (reference itsolv/SolverFactory.h:73-185 and
// SolverFactory-implementation.h:16-100).
//
//   create_LinearEigensystem("Davidson" | "RSPT", options, handlers)
//   create_LinearEquations("Davidson", options, handlers)
//   create_NonLinearEquations("DIIS", options, handlers)
//   create_Optimize("BFGS" | "SD", options, handlers)
//   SolverFactory<R,Q,P>{}.create("LinearEigensystem" | "LinearEquations", options_map, handlers)
//
// Same method names, defaults (an empty method selects the family's default), option strings
// ("key=value,..." with case-insensitive keys) and errors (std::runtime_error "Unimplemented method
// <m>" for an unknown method name) as the reference.  Differences: every solver here derives from
// IterativeSolverTemplate (there are no separate family interfaces), so the factory returns that;
// the handlers are a required argument (the reference defaults them to its CPU handlers, and the
// HBM back end's are hbm::make_handlers(), see hbm::create_* in hbm_handlers.h's callers).
#pragma once
#include <memory>
#include <stdexcept>
#include <string>

#include "common.h"
#include "solvers.h"

namespace molpro::linalg::itsolv {

template <class R, class Q = R, class P = std::map<size_t, typename R::value_type>>
class SolverFactory {
 public:
  using Solver = IterativeSolverTemplate<R, Q, P>;
  using Handlers = std::shared_ptr<ArrayHandlers<R, Q, P>>;
  virtual ~SolverFactory() = default;

  // SolverFactory-implementation.h:30-47: the option set's type selects the method
  virtual std::unique_ptr<Solver> create_linear_eigensystem(const Options& options, const Handlers& handlers) {
    if (auto* o = dynamic_cast<const LinearEigensystemDavidsonOptions*>(&options)) {
      auto s = std::make_unique<LinearEigensystemDavidson<R, Q, P>>(handlers);
      s->set_options(*o);
      return s;
    }
    if (auto* o = dynamic_cast<const LinearEigensystemRSPTOptions*>(&options)) {
      auto s = std::make_unique<LinearEigensystemRSPT<R, Q, P>>(handlers);
      s->set_options(*o);
      return s;
    }
    throw std::logic_error("SolverFactory failed to cast to solver");
  }

  // :49-56
  virtual std::unique_ptr<Solver> create_linear_equations(const LinearEquationsDavidsonOptions& options,
                                                          const Handlers& handlers) {
    auto s = std::make_unique<LinearEquationsDavidson<R, Q, P>>(handlers);
    s->set_options(options);
    return s;
  }

  // :58-69
  virtual std::unique_ptr<Solver> create_non_linear_equations(const Options& options, const Handlers& handlers) {
    if (auto* o = dynamic_cast<const NonLinearEquationsDIISOptions*>(&options)) {
      auto s = std::make_unique<NonLinearEquationsDIIS<R, Q, P>>(handlers);
      s->set_options(*o);
      return s;
    }
    throw std::runtime_error("Unimplemented solver method");
  }

  // :71-87
  virtual std::unique_ptr<Solver> create_optimize(const Options& options, const Handlers& handlers) {
    if (auto* o = dynamic_cast<const OptimizeBFGSOptions*>(&options)) {
      auto s = std::make_unique<OptimizeBFGS<R, Q, P>>(handlers);
      s->set_options(*o);
      return s;
    }
    if (auto* o = dynamic_cast<const OptimizeSDOptions*>(&options)) {
      auto s = std::make_unique<OptimizeSD<R, Q, P>>(handlers);
      s->set_options(*o);
      return s;
    }
    throw std::runtime_error("Unimplemented solver method");
  }

  // :89-99: by family name, with that family's default method
  virtual std::unique_ptr<Solver> create(const std::string& family, const options_map& options,
                                         const Handlers& handlers) {
    if (family == "LinearEigensystem") return create_linear_eigensystem(LinearEigensystemDavidsonOptions{options}, handlers);
    if (family == "LinearEquations") return create_linear_equations(LinearEquationsDavidsonOptions{options}, handlers);
    throw std::runtime_error("Method = " + family + ", is not implemented");
  }
};

// Free functions by method name (SolverFactory.h:114-185).
template <class R, class Q, class P>
std::unique_ptr<IterativeSolverTemplate<R, Q, P>>
create_LinearEigensystem(const std::string& method, const std::string& options,
                         const std::shared_ptr<ArrayHandlers<R, Q, P>>& handlers) {
  const auto m = parse_options(options);
  if (method == "Davidson" || method.empty())
    return SolverFactory<R, Q, P>{}.create_linear_eigensystem(LinearEigensystemDavidsonOptions{m}, handlers);
  if (method == "RSPT") return SolverFactory<R, Q, P>{}.create_linear_eigensystem(LinearEigensystemRSPTOptions{m}, handlers);
  throw std::runtime_error("Unimplemented method " + method);
}

template <class R, class Q, class P>
std::unique_ptr<IterativeSolverTemplate<R, Q, P>>
create_LinearEquations(const std::string& method, const std::string& options,
                       const std::shared_ptr<ArrayHandlers<R, Q, P>>& handlers) {
  if (method == "Davidson" || method.empty())
    return SolverFactory<R, Q, P>{}.create_linear_equations(LinearEquationsDavidsonOptions{parse_options(options)},
                                                            handlers);
  throw std::runtime_error("Unimplemented method " + method);
}

template <class R, class Q, class P>
std::unique_ptr<IterativeSolverTemplate<R, Q, P>>
create_NonLinearEquations(const std::string& method, const std::string& options,
                          const std::shared_ptr<ArrayHandlers<R, Q, P>>& handlers) {
  if (method == "DIIS" || method.empty())
    return SolverFactory<R, Q, P>{}.create_non_linear_equations(NonLinearEquationsDIISOptions{parse_options(options)},
                                                                handlers);
  throw std::runtime_error("Unimplemented method " + method);
}

template <class R, class Q, class P>
std::unique_ptr<IterativeSolverTemplate<R, Q, P>>
create_Optimize(const std::string& method, const std::string& options,
                const std::shared_ptr<ArrayHandlers<R, Q, P>>& handlers) {
  const auto m = parse_options(options);
  if (method == "BFGS" || method.empty())
    return SolverFactory<R, Q, P>{}.create_optimize(OptimizeBFGSOptions{m}, handlers);
  if (method == "SD") return SolverFactory<R, Q, P>{}.create_optimize(OptimizeSDOptions{m}, handlers);
  throw std::runtime_error("Unimplemented method " + method);
}

}  // namespace molpro::linalg::itsolv
