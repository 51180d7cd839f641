// Drop-in for the reference: the MI355X HBM handlers derived from the reference's OWN abstract
// handler, molpro::linalg::array::ArrayHandler<AL, AR> (reference src/molpro/linalg/array/
// ArrayHandler.h:161-437).
//
// Include this from a translation unit of the reference tree (include path: the reference's src/
// and this package's include/ plus the repository's include/), then inject the handlers into the
// reference's solvers exactly as its own handlers are injected (reference itsolv/ArrayHandlers.h:57-103,
// LinearEigensystemDavidson.h:34, NonLinearEquationsDIIS.h:37):
//
//   #include <molpro/linalg/itsolv/ArrayHandlers.h>
//   #include <molpro/linalg/array/ArrayHandlerSparse.h>
//   #include <itsolv_hbm/reference_handler.h>
//   using molpro::linalg::hbm::Vec;  using P = std::map<size_t, double>;
//   auto dense = [] { return std::make_shared<molpro::linalg::hbm::ArrayHandlerHbm>(); };
//   auto sparse = [] { return std::make_shared<molpro::linalg::hbm::ArrayHandlerHbmSparse>(); };
//   auto handlers = molpro::linalg::itsolv::ArrayHandlers<Vec, Vec, P>::create()
//       .rr(dense()).qq(dense()).rq(dense()).qr(dense())
//       .rp(sparse()).qp(sparse())
//       .pp(std::make_shared<molpro::linalg::array::ArrayHandlerSparse<P, P>>())
//       .build();
//   molpro::linalg::itsolv::LinearEigensystemDavidson<Vec, Vec, P> solver(handlers);
//
// R and Q are hbm::Vec (itsolv_hbm/hbm_vec.h): the solver's Q space then lives in HBM and every
// handler operation is one libsubspace_hip.so call; link with -lsubspace_hip.  The classes are the
// ones this package's own solvers use (itsolv_hbm/hbm_handler_impl.h), compiled here against the
// reference's base: lazy_handle() is implemented (ArrayHandler.h:436) and the protected
// fused_dot / fused_axpy (:271-292) evaluate a lazy register as one gemm_inner / gemm_outer launch.
//
// Do not include this together with itsolv_hbm/array_handler.h (the package's restatement of the
// same base) in one translation unit.  libitsolv_hbm.so keeps its restated C++ symbols local
// (host/exports.map), so the two coexist in one process.
#pragma once
#include <molpro/linalg/array/ArrayHandler.h>

#include "hbm_handler_impl.h"
