﻿!mod$ v1 sum:c5bf272f067226ea
!need$ 0bde2ac47243ead2 i iso_c_binding
module iterative_solver
use,intrinsic::iso_c_binding,only:c_associated
use,intrinsic::iso_c_binding,only:c_funloc
use,intrinsic::iso_c_binding,only:c_funptr
use,intrinsic::iso_c_binding,only:c_f_pointer
use,intrinsic::iso_c_binding,only:c_loc
use,intrinsic::iso_c_binding,only:c_null_funptr
use,intrinsic::iso_c_binding,only:c_null_ptr
use,intrinsic::iso_c_binding,only:c_ptr
use,intrinsic::iso_c_binding,only:c_sizeof
use,intrinsic::iso_c_binding,only:operator(==)
use,intrinsic::iso_c_binding,only:operator(/=)
use,intrinsic::iso_c_binding,only:c_int8_t
use,intrinsic::iso_c_binding,only:c_int16_t
use,intrinsic::iso_c_binding,only:c_int32_t
use,intrinsic::iso_c_binding,only:c_int64_t
use,intrinsic::iso_c_binding,only:c_int128_t
use,intrinsic::iso_c_binding,only:c_int
use,intrinsic::iso_c_binding,only:c_short
use,intrinsic::iso_c_binding,only:c_long
use,intrinsic::iso_c_binding,only:c_long_long
use,intrinsic::iso_c_binding,only:c_signed_char
use,intrinsic::iso_c_binding,only:c_size_t
use,intrinsic::iso_c_binding,only:c_intmax_t
use,intrinsic::iso_c_binding,only:c_intptr_t
use,intrinsic::iso_c_binding,only:c_ptrdiff_t
use,intrinsic::iso_c_binding,only:c_int_least8_t
use,intrinsic::iso_c_binding,only:c_int_fast8_t
use,intrinsic::iso_c_binding,only:c_int_least16_t
use,intrinsic::iso_c_binding,only:c_int_fast16_t
use,intrinsic::iso_c_binding,only:c_int_least32_t
use,intrinsic::iso_c_binding,only:c_int_fast32_t
use,intrinsic::iso_c_binding,only:c_int_least64_t
use,intrinsic::iso_c_binding,only:c_int_fast64_t
use,intrinsic::iso_c_binding,only:c_int_least128_t
use,intrinsic::iso_c_binding,only:c_int_fast128_t
use,intrinsic::iso_c_binding,only:c_float
use,intrinsic::iso_c_binding,only:c_double
use,intrinsic::iso_c_binding,only:c_long_double
use,intrinsic::iso_c_binding,only:c_float_complex
use,intrinsic::iso_c_binding,only:c_double_complex
use,intrinsic::iso_c_binding,only:c_long_double_complex
use,intrinsic::iso_c_binding,only:c_bool
use,intrinsic::iso_c_binding,only:c_char
use,intrinsic::iso_c_binding,only:c_null_char
use,intrinsic::iso_c_binding,only:c_alert
use,intrinsic::iso_c_binding,only:c_backspace
use,intrinsic::iso_c_binding,only:c_form_feed
use,intrinsic::iso_c_binding,only:c_new_line
use,intrinsic::iso_c_binding,only:c_carriage_return
use,intrinsic::iso_c_binding,only:c_horizontal_tab
use,intrinsic::iso_c_binding,only:c_vertical_tab
use,intrinsic::iso_c_binding,only:c_float128
use,intrinsic::iso_c_binding,only:c_float128_complex
use,intrinsic::iso_c_binding,only:c_uint8_t
use,intrinsic::iso_c_binding,only:c_uint16_t
use,intrinsic::iso_c_binding,only:c_uint32_t
use,intrinsic::iso_c_binding,only:c_uint64_t
use,intrinsic::iso_c_binding,only:c_uint128_t
use,intrinsic::iso_c_binding,only:c_unsigned_char
use,intrinsic::iso_c_binding,only:c_unsigned_short
use,intrinsic::iso_c_binding,only:c_unsigned
use,intrinsic::iso_c_binding,only:c_unsigned_long
use,intrinsic::iso_c_binding,only:c_unsigned_long_long
use,intrinsic::iso_c_binding,only:c_uintmax_t
use,intrinsic::iso_c_binding,only:c_uint_fast8_t
use,intrinsic::iso_c_binding,only:c_uint_fast16_t
use,intrinsic::iso_c_binding,only:c_uint_fast32_t
use,intrinsic::iso_c_binding,only:c_uint_fast64_t
use,intrinsic::iso_c_binding,only:c_uint_fast128_t
use,intrinsic::iso_c_binding,only:c_uint_least8_t
use,intrinsic::iso_c_binding,only:c_uint_least16_t
use,intrinsic::iso_c_binding,only:c_uint_least32_t
use,intrinsic::iso_c_binding,only:c_uint_least64_t
use,intrinsic::iso_c_binding,only:c_uint_least128_t
use,intrinsic::iso_c_binding,only:c_f_procpointer
private::c_associated
private::c_funloc
private::c_funptr
private::c_f_pointer
private::c_loc
private::c_null_funptr
private::c_null_ptr
private::c_ptr
private::c_sizeof
private::operator(==)
private::operator(/=)
private::c_int8_t
private::c_int16_t
private::c_int32_t
private::c_int64_t
private::c_int128_t
private::c_int
private::c_short
private::c_long
private::c_long_long
private::c_signed_char
private::c_size_t
private::c_intmax_t
private::c_intptr_t
private::c_ptrdiff_t
private::c_int_least8_t
private::c_int_fast8_t
private::c_int_least16_t
private::c_int_fast16_t
private::c_int_least32_t
private::c_int_fast32_t
private::c_int_least64_t
private::c_int_fast64_t
private::c_int_least128_t
private::c_int_fast128_t
private::c_float
private::c_double
private::c_long_double
private::c_float_complex
private::c_double_complex
private::c_long_double_complex
private::c_bool
private::c_char
private::c_null_char
private::c_alert
private::c_backspace
private::c_form_feed
private::c_new_line
private::c_carriage_return
private::c_horizontal_tab
private::c_vertical_tab
private::c_float128
private::c_float128_complex
private::c_uint8_t
private::c_uint16_t
private::c_uint32_t
private::c_uint64_t
private::c_uint128_t
private::c_unsigned_char
private::c_unsigned_short
private::c_unsigned
private::c_unsigned_long
private::c_unsigned_long_long
private::c_uintmax_t
private::c_uint_fast8_t
private::c_uint_fast16_t
private::c_uint_fast32_t
private::c_uint_fast64_t
private::c_uint_fast128_t
private::c_uint_least8_t
private::c_uint_least16_t
private::c_uint_least32_t
private::c_uint_least64_t
private::c_uint_least128_t
private::c_f_procpointer
integer(4),parameter::mpicomm_kind=4_4
intrinsic::kind
private::kind
integer(4),private,save::compute_comm
logical(4),private,save::compute_comm_set
private::c_eigensystem_init
interface
subroutine c_eigensystem_init(n,nroot,range_begin,range_end,thresh,thresh_value,hermitian,verbosity,fname,fcomm,algorithm,options) bind(c,name="IterativeSolverLinearEigensystemInitialize")
integer(8),value::n
integer(8),value::nroot
integer(8),intent(inout)::range_begin
integer(8),intent(inout)::range_end
real(8),value::thresh
real(8),value::thresh_value
integer(4),value::hermitian
integer(4),value::verbosity
character(1_8,1),intent(in)::fname(1_8:*)
integer(8),value::fcomm
character(1_8,1),intent(in)::algorithm(1_8:*)
character(1_8,1),intent(in)::options(1_8:*)
end
end interface
private::c_equations_init
interface
subroutine c_equations_init(n,nroot,range_begin,range_end,rhs,aughes,thresh,thresh_value,hermitian,verbosity,fname,fcomm,algorithm,options) bind(c,name="IterativeSolverLinearEquationsInitialize")
integer(8),value::n
integer(8),value::nroot
integer(8),intent(inout)::range_begin
integer(8),intent(inout)::range_end
real(8),intent(in)::rhs(1_8:*)
real(8),value::aughes
real(8),value::thresh
real(8),value::thresh_value
integer(4),value::hermitian
integer(4),value::verbosity
character(1_8,1),intent(in)::fname(1_8:*)
integer(8),value::fcomm
character(1_8,1),intent(in)::algorithm(1_8:*)
character(1_8,1),intent(in)::options(1_8:*)
end
end interface
private::c_diis_init
interface
subroutine c_diis_init(n,range_begin,range_end,thresh,verbosity,fname,fcomm,algorithm,options) bind(c,name="IterativeSolverNonLinearEquationsInitialize")
integer(8),value::n
integer(8),intent(inout)::range_begin
integer(8),intent(inout)::range_end
real(8),value::thresh
integer(4),value::verbosity
character(1_8,1),intent(in)::fname(1_8:*)
integer(8),value::fcomm
character(1_8,1),intent(in)::algorithm(1_8:*)
character(1_8,1),intent(in)::options(1_8:*)
end
end interface
private::c_optimize_init
interface
subroutine c_optimize_init(n,range_begin,range_end,thresh,thresh_value,verbosity,minimize,fname,fcomm,algorithm,options) bind(c,name="IterativeSolverOptimizeInitialize")
integer(8),value::n
integer(8),intent(inout)::range_begin
integer(8),intent(inout)::range_end
real(8),value::thresh
real(8),value::thresh_value
integer(4),value::verbosity
integer(4),value::minimize
character(1_8,1),intent(in)::fname(1_8:*)
integer(8),value::fcomm
character(1_8,1),intent(in)::algorithm(1_8:*)
character(1_8,1),intent(in)::options(1_8:*)
end
end interface
interface
subroutine iterative_solver_finalize() bind(c,name="IterativeSolverFinalize")
end
end interface
private::c_add_vector
interface
function c_add_vector(buffer_size,parameters,action,sync) bind(c,name="IterativeSolverAddVector")
import::c_ptr
integer(8),value::buffer_size
type(c_ptr),value::parameters
type(c_ptr),value::action
integer(4),value::sync
integer(8)::c_add_vector
end
end interface
private::c_add_value
interface
function c_add_value(value,parameters,action,sync) bind(c,name="IterativeSolverAddValue")
import::c_ptr
real(8),value::value
type(c_ptr),value::parameters
type(c_ptr),value::action
integer(4),value::sync
integer(8)::c_add_value
end
end interface
private::c_end_iteration
interface
function c_end_iteration(buffer_size,solution,residual,sync) bind(c,name="IterativeSolverEndIteration")
import::c_ptr
integer(8),value::buffer_size
type(c_ptr),value::solution
type(c_ptr),value::residual
integer(4),value::sync
integer(8)::c_end_iteration
end
end interface
private::c_end_iteration_needed
interface
function c_end_iteration_needed() bind(c,name="IterativeSolverEndIterationNeeded")
integer(4)::c_end_iteration_needed
end
end interface
private::c_solution
interface
subroutine c_solution(nroot,roots,parameters,action,sync) bind(c,name="IterativeSolverSolution")
import::c_ptr
integer(4),value::nroot
integer(4),intent(in)::roots(1_8:*)
type(c_ptr),value::parameters
type(c_ptr),value::action
integer(4),value::sync
end
end interface
private::c_add_p
interface
function c_add_p(buffer_size,np,offsets,indices,coefficients,pp,parameters,action,sync,func) bind(c,name="IterativeSolverAddP")
import::c_funptr
import::c_ptr
integer(8),value::buffer_size
integer(8),value::np
integer(8),intent(in)::offsets(1_8:*)
integer(8),intent(in)::indices(1_8:*)
real(8),intent(in)::coefficients(1_8:*)
real(8),intent(in)::pp(1_8:*)
type(c_ptr),value::parameters
type(c_ptr),value::action
integer(4),value::sync
type(c_funptr),value::func
integer(8)::c_add_p
end
end interface
private::c_suggest_p
interface
function c_suggest_p(solution,residual,maximum_number,threshold,indices) bind(c,name="IterativeSolverSuggestP")
real(8),intent(in)::solution(1_8:*)
real(8),intent(in)::residual(1_8:*)
integer(8),value::maximum_number
real(8),value::threshold
integer(8),intent(inout)::indices(1_8:*)
integer(8)::c_suggest_p
end
end interface
private::c_errors
interface
subroutine c_errors(errors) bind(c,name="IterativeSolverErrors")
real(8),intent(inout)::errors(1_8:*)
end
end interface
private::c_eigenvalues
interface
subroutine c_eigenvalues(eigenvalues) bind(c,name="IterativeSolverEigenvalues")
real(8),intent(inout)::eigenvalues(1_8:*)
end
end interface
private::c_working_set_eigenvalues
interface
subroutine c_working_set_eigenvalues(eigenvalues) bind(c,name="IterativeSolverWorkingSetEigenvalues")
real(8),intent(inout)::eigenvalues(1_8:*)
end
end interface
private::c_nroots
interface
function c_nroots() bind(c,name="IterativeSolverHbmNRoots")
integer(8)::c_nroots
end
end interface
interface
subroutine iterative_solver_print_statistics() bind(c,name="IterativeSolverPrintStatistics")
end
end interface
interface
function iterative_solver_value() bind(c,name="IterativeSolverValue")
real(8)::iterative_solver_value
end
end interface
interface
function iterative_solver_verbosity() bind(c,name="IterativeSolverVerbosity")
integer(4)::iterative_solver_verbosity
end
end interface
private::c_nonlinear
interface
function c_nonlinear() bind(c,name="IterativeSolverNonLinear")
integer(4)::c_nonlinear
end
end interface
private::c_has_values
interface
function c_has_values() bind(c,name="IterativeSolverHasValues")
integer(4)::c_has_values
end
end interface
private::c_has_eigenvalues
interface
function c_has_eigenvalues() bind(c,name="IterativeSolverHasEigenvalues")
integer(4)::c_has_eigenvalues
end
end interface
private::c_max_iter
interface
function c_max_iter() bind(c,name="IterativeSolverMaxIter")
integer(4)::c_max_iter
end
end interface
private::c_set_max_iter
interface
subroutine c_set_max_iter(max_iter) bind(c,name="IterativeSolverSetMaxIter")
integer(4),value::max_iter
end
end interface
private::c_set_diagonals
interface
subroutine c_set_diagonals(diagonals) bind(c,name="IterativeSolverSetDiagonals")
real(8),intent(in)::diagonals(1_8:*)
end
end interface
private::c_diagonals
interface
subroutine c_diagonals(diagonals) bind(c,name="IterativeSolverDiagonals")
real(8),intent(inout)::diagonals(1_8:*)
end
end interface
private::c_mpicomm_global
interface
function c_mpicomm_global() bind(c,name="IterativeSolver_mpicomm_global")
integer(8)::c_mpicomm_global
end
end interface
private::c_mpicomm_self
interface
function c_mpicomm_self() bind(c,name="IterativeSolver_mpicomm_self")
integer(8)::c_mpicomm_self
end
end interface
private::c_mpi_init
interface
function c_mpi_init() bind(c,name="IterativeSolver_mpi_init")
integer(4)::c_mpi_init
end
end interface
private::c_mpi_finalize
interface
function c_mpi_finalize() bind(c,name="IterativeSolver_mpi_finalize")
integer(4)::c_mpi_finalize
end
end interface
interface
function mpi_size_global() bind(c,name="IterativeSolver_mpisize_global")
integer(8)::mpi_size_global
end
end interface
interface
function mpi_rank_global() bind(c,name="IterativeSolver_mpirank_global")
integer(8)::mpi_rank_global
end
end interface
private::c_string
private::real_or
private::int_or
private::flag_or
private::comm_or_compute
private::columns
private::range_in
private::range_out
private::eigensystem_init_sizet
private::eigensystem_init_default
private::equations_init_sizet
private::equations_init_default
private::diis_init_sizet
private::diis_init_default
private::optimize_init_sizet
private::optimize_init_default
interface iterative_solver_linear_eigensystem_initialize
procedure::eigensystem_init_default
procedure::eigensystem_init_sizet
end interface
interface iterative_solver_linear_equations_initialize
procedure::equations_init_default
procedure::equations_init_sizet
end interface
interface iterative_solver_diis_initialize
procedure::diis_init_default
procedure::diis_init_sizet
end interface
interface iterative_solver_optimize_initialize
procedure::optimize_init_default
procedure::optimize_init_sizet
end interface
contains
function mpicomm_global()
integer(4)::mpicomm_global
end
function mpicomm_self()
integer(4)::mpicomm_self
end
function mpicomm_compute()
integer(4)::mpicomm_compute
end
subroutine set_mpicomm_compute(comm)
integer(4),intent(in)::comm
end
subroutine mpi_init()
end
subroutine mpi_finalize()
end
function c_string(s) result(c)
character(*,1),intent(in),optional::s
character(:,1),allocatable::c
end
function real_or(x,default)
real(8),intent(in),optional::x
real(8),intent(in)::default
real(8)::real_or
end
function int_or(i,default)
integer(4),intent(in),optional::i
integer(4),intent(in)::default
integer(4)::int_or
end
function flag_or(l,default)
logical(4),intent(in),optional::l
logical(4),intent(in)::default
integer(4)::flag_or
end
function comm_or_compute(comm)
integer(4),intent(in),optional::comm
integer(8)::comm_or_compute
end
function columns(a)
real(8),intent(in)::a(..)
integer(8)::columns
end
subroutine range_in(range,b,e)
integer(4),intent(in),optional::range(1_8:2_8)
integer(8),intent(out)::b
integer(8),intent(out)::e
end
subroutine range_out(range,b,e)
integer(4),intent(inout),optional::range(1_8:2_8)
integer(8),intent(in)::b
integer(8),intent(in)::e
end
subroutine eigensystem_init_sizet(nq,nroot,thresh,thresh_value,hermitian,verbosity,pname,mpicomm,algorithm,range,options)
integer(8),intent(in)::nq
integer(8),intent(in)::nroot
real(8),intent(in),optional::thresh
real(8),intent(in),optional::thresh_value
logical(4),intent(in),optional::hermitian
integer(4),intent(in),optional::verbosity
character(*,1),intent(in),optional::pname
integer(4),intent(in),optional::mpicomm
character(*,1),intent(in),optional::algorithm
integer(4),intent(inout),optional::range(1_8:2_8)
character(*,1),intent(in),optional::options
end
subroutine eigensystem_init_default(nq,nroot,thresh,thresh_value,hermitian,verbosity,pname,mpicomm,algorithm,range,options)
integer(4),intent(in)::nq
integer(4),intent(in)::nroot
real(8),intent(in),optional::thresh
real(8),intent(in),optional::thresh_value
logical(4),intent(in),optional::hermitian
integer(4),intent(in),optional::verbosity
character(*,1),intent(in),optional::pname
integer(4),intent(in),optional::mpicomm
character(*,1),intent(in),optional::algorithm
integer(4),intent(inout),optional::range(1_8:2_8)
character(*,1),intent(in),optional::options
end
subroutine equations_init_sizet(nq,nroot,rhs,augmented_hessian,thresh,thresh_value,hermitian,verbosity,pname,mpicomm,algorithm,range,options)
integer(8),intent(in)::nq
integer(8),intent(in)::nroot
real(8),intent(in)::rhs(1_8:nq,1_8:nroot)
real(8),intent(in),optional::augmented_hessian
real(8),intent(in),optional::thresh
real(8),intent(in),optional::thresh_value
logical(4),intent(in),optional::hermitian
integer(4),intent(in),optional::verbosity
character(*,1),intent(in),optional::pname
integer(4),intent(in),optional::mpicomm
character(*,1),intent(in),optional::algorithm
integer(4),intent(inout),optional::range(1_8:2_8)
character(*,1),intent(in),optional::options
end
subroutine equations_init_default(nq,nroot,rhs,augmented_hessian,thresh,thresh_value,hermitian,verbosity,pname,mpicomm,algorithm,range,options)
integer(4),intent(in)::nq
integer(4),intent(in)::nroot
real(8),intent(in)::rhs(1_8:int(nq,kind=8),1_8:int(nroot,kind=8))
real(8),intent(in),optional::augmented_hessian
real(8),intent(in),optional::thresh
real(8),intent(in),optional::thresh_value
logical(4),intent(in),optional::hermitian
integer(4),intent(in),optional::verbosity
character(*,1),intent(in),optional::pname
integer(4),intent(in),optional::mpicomm
character(*,1),intent(in),optional::algorithm
integer(4),intent(inout),optional::range(1_8:2_8)
character(*,1),intent(in),optional::options
end
subroutine diis_init_sizet(nq,thresh,verbosity,pname,mpicomm,algorithm,range,options)
integer(8),intent(in)::nq
real(8),intent(in),optional::thresh
integer(4),intent(in),optional::verbosity
character(*,1),intent(in),optional::pname
integer(4),intent(in),optional::mpicomm
character(*,1),intent(in),optional::algorithm
integer(4),intent(inout),optional::range(1_8:2_8)
character(*,1),intent(in),optional::options
end
subroutine diis_init_default(nq,thresh,verbosity,pname,mpicomm,algorithm,range,options)
integer(4),intent(in)::nq
real(8),intent(in),optional::thresh
integer(4),intent(in),optional::verbosity
character(*,1),intent(in),optional::pname
integer(4),intent(in),optional::mpicomm
character(*,1),intent(in),optional::algorithm
integer(4),intent(inout),optional::range(1_8:2_8)
character(*,1),intent(in),optional::options
end
subroutine optimize_init_sizet(nq,thresh,verbosity,minimize,pname,mpicomm,algorithm,range,thresh_value,options)
integer(8),intent(in)::nq
real(8),intent(in),optional::thresh
integer(4),intent(in),optional::verbosity
logical(4),intent(in),optional::minimize
character(*,1),intent(in),optional::pname
integer(4),intent(in),optional::mpicomm
character(*,1),intent(in),optional::algorithm
integer(4),intent(inout),optional::range(1_8:2_8)
real(8),intent(in),optional::thresh_value
character(*,1),intent(in),optional::options
end
subroutine optimize_init_default(nq,thresh,verbosity,minimize,pname,mpicomm,algorithm,range,thresh_value,options)
integer(4),intent(in)::nq
real(8),intent(in),optional::thresh
integer(4),intent(in),optional::verbosity
logical(4),intent(in),optional::minimize
character(*,1),intent(in),optional::pname
integer(4),intent(in),optional::mpicomm
character(*,1),intent(in),optional::algorithm
integer(4),intent(inout),optional::range(1_8:2_8)
real(8),intent(in),optional::thresh_value
character(*,1),intent(in),optional::options
end
function iterative_solver_add_vector(parameters,action,synchronize,value)
real(8),contiguous,intent(inout),target::parameters(..)
real(8),contiguous,intent(inout),target::action(..)
logical(4),intent(in),optional::synchronize
real(8),intent(in),optional::value
integer(4)::iterative_solver_add_vector
end
subroutine iterative_solver_solution(roots,parameters,action,synchronize)
integer(4),intent(in)::roots(:)
real(8),contiguous,intent(inout),target::parameters(..)
real(8),contiguous,intent(inout),target::action(..)
logical(4),intent(in),optional::synchronize
end
function iterative_solver_end_iteration(solution,residual,synchronize)
real(8),contiguous,intent(inout),target::solution(..)
real(8),contiguous,intent(inout),target::residual(..)
logical(4),intent(in),optional::synchronize
integer(4)::iterative_solver_end_iteration
end
function iterative_solver_end_iteration_needed()
logical(4)::iterative_solver_end_iteration_needed
end
function iterative_solver_add_p(np,offsets,indices,coefficients,pp,parameters,action,fproc,synchronize)
integer(4),intent(in)::np
integer(4),intent(in)::offsets(0_8:int(np,kind=8))
integer(4),intent(in)::indices(1_8:int(offsets(int(np,kind=8)),kind=8))
real(8),intent(in)::coefficients(1_8:int(offsets(int(np,kind=8)),kind=8))
real(8),intent(in)::pp(1_8:*)
real(8),contiguous,intent(inout),target::parameters(:,:)
real(8),contiguous,intent(inout),target::action(:,:)
procedure()::fproc
logical(4),intent(in),optional::synchronize
integer(4)::iterative_solver_add_p
end
function iterative_solver_suggest_p(solution,residual,indices,threshold)
real(8),intent(in)::solution(1_8:*)
real(8),intent(in)::residual(1_8:*)
integer(4),intent(inout)::indices(:)
real(8),intent(in),optional::threshold
integer(4)::iterative_solver_suggest_p
end
function iterative_solver_errors() result(errors)
real(8),allocatable::errors(:)
end
function iterative_solver_eigenvalues() result(eigenvalues)
real(8),allocatable::eigenvalues(:)
end
function iterative_solver_working_set_eigenvalues(working_set_size) result(eigenvalues)
integer(4),intent(in)::working_set_size
real(8)::eigenvalues(1_8:int(working_set_size,kind=8))
end
subroutine iterative_solver_solve(parameters,actions,problem,generate_initial_guess,max_iter)
use iterative_solver_problem,only:problem_class=>problem
real(8),contiguous,intent(inout),target::parameters(..)
real(8),contiguous,intent(inout),target::actions(..)
class(problem_class),intent(in)::problem
logical(4),intent(in),optional::generate_initial_guess
integer(4),intent(in),optional::max_iter
end
end
