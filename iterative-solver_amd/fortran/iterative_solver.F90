!> Fortran binding of the reverse-communication C API of libitsolv_hbm.so (include/iterative_solver_c.h).
!>
!> Module Iterative_Solver with the public names, argument lists, defaults and index conventions of
!> the reference's Fortran module (src/molpro/linalg/IterativeSolverF.F90:1-935), so that Molpro-style
!> Fortran callers switch by relinking: the solvers behind it keep Q, D and every subspace operation
!> in HBM, R crosses PCIe once per call (DESIGN.md §5).
!>
!> Conventions kept from the reference:
!>  - thresh defaults to 1e-10, thresh_value to 1e50, verbosity to 0, hermitian to .false.;
!>  - range(1:2) receives this rank's [begin, end) of every vector, 0-based, as the C layer returns it;
!>  - root numbers (Solution) and P-space indices (Add_P, Suggest_P) are 1-based here, 0-based in C;
!>  - Add_Vector with `value` goes through IterativeSolverAddValue (Optimize), otherwise through
!>    IterativeSolverAddVector with the number of columns of `parameters` as the buffer size;
!>  - mpicomm arguments are integers of kind mpicomm_kind (= KIND(c_int64_t), the default integer
!>    kind, as in the reference) and are passed on, widened, as the C API's int64 communicator.
!> Differences (each a defect of the reference module, fixed here):
!>  - Optimize: minimize defaults to 1 (the reference sets an unrelated variable and passes an
!>    uninitialised one, IterativeSolverF.F90:321, :362-364); the C layer ignores it anyway;
!>  - DIIS: the algorithm string is NUL-terminated (the reference passes the Fortran string,
!>    IterativeSolverF.F90:462-463);
!>  - Initialize accepts nq and nroot as default integers or as c_size_t/c_int64_t integers (generic
!>    interfaces), as the reference's own tests call it (test/itsolv/test_LinearEigensystemF.f90:23);
!>  - Errors / Eigenvalues are sized by the top instance's number of roots (the reference keeps one
!>    module variable, which a nested instance overwrites);
!>  - Working_Set_Eigenvalues is zero for solvers without eigenvalues (the reference leaves it
!>    undefined), so the default preconditioner then divides by the bare diagonals;
!>  - Add_Vector and End_Iteration count buffer columns from the array's shape for any rank (the
!>    reference reads ubound(parameters, 2) of rank-1 arrays);
!>  - mpi_size_global / mpi_rank_global bind symbols that exist (see iterative_solver_c.h).
module Iterative_Solver
  use, intrinsic :: iso_c_binding
  implicit none
  private

  public :: Iterative_Solver_Linear_Eigensystem_Initialize, Iterative_Solver_Linear_Equations_Initialize
  public :: Iterative_Solver_DIIS_Initialize, Iterative_Solver_Optimize_Initialize
  public :: Iterative_Solver_Finalize
  public :: Iterative_Solver_Add_Vector, Iterative_Solver_End_Iteration, Iterative_Solver_End_Iteration_Needed
  public :: Iterative_Solver_Solution, Iterative_Solver_Add_P, Iterative_Solver_Suggest_P
  public :: Iterative_Solver_Errors, Iterative_Solver_Eigenvalues, Iterative_Solver_Working_Set_Eigenvalues
  public :: Iterative_Solver_Print_Statistics, Iterative_Solver_Solve
  public :: Iterative_Solver_Value, Iterative_Solver_Verbosity
  public :: mpicomm_global, mpicomm_self, mpicomm_compute, set_mpicomm_compute
  public :: mpi_init, mpi_finalize, mpi_rank_global, mpi_size_global

  integer, public, parameter :: mpicomm_kind = kind(c_int64_t)

  integer(kind=mpicomm_kind), save :: compute_comm = 0
  logical, save :: compute_comm_set = .false.

  interface Iterative_Solver_Linear_Eigensystem_Initialize
    module procedure eigensystem_init_default, eigensystem_init_sizet
  end interface
  interface Iterative_Solver_Linear_Equations_Initialize
    module procedure equations_init_default, equations_init_sizet
  end interface
  interface Iterative_Solver_DIIS_Initialize
    module procedure diis_init_default, diis_init_sizet
  end interface
  interface Iterative_Solver_Optimize_Initialize
    module procedure optimize_init_default, optimize_init_sizet
  end interface

  ! ---- the C API (include/iterative_solver_c.h) -------------------------------------------------
  interface
    subroutine c_eigensystem_init(n, nroot, range_begin, range_end, thresh, thresh_value, hermitian, verbosity, &
        fname, fcomm, algorithm, options) bind(c, name='IterativeSolverLinearEigensystemInitialize')
      import :: c_size_t, c_double, c_int, c_int64_t, c_char
      integer(c_size_t), value :: n, nroot
      integer(c_size_t), intent(inout) :: range_begin, range_end
      real(c_double), value :: thresh, thresh_value
      integer(c_int), value :: hermitian, verbosity
      character(kind=c_char), dimension(*), intent(in) :: fname, algorithm, options
      integer(c_int64_t), value :: fcomm
    end subroutine c_eigensystem_init
    subroutine c_equations_init(n, nroot, range_begin, range_end, rhs, aughes, thresh, thresh_value, hermitian, &
        verbosity, fname, fcomm, algorithm, options) bind(c, name='IterativeSolverLinearEquationsInitialize')
      import :: c_size_t, c_double, c_int, c_int64_t, c_char
      integer(c_size_t), value :: n, nroot
      integer(c_size_t), intent(inout) :: range_begin, range_end
      real(c_double), dimension(*), intent(in) :: rhs
      real(c_double), value :: aughes, thresh, thresh_value
      integer(c_int), value :: hermitian, verbosity
      character(kind=c_char), dimension(*), intent(in) :: fname, algorithm, options
      integer(c_int64_t), value :: fcomm
    end subroutine c_equations_init
    subroutine c_diis_init(n, range_begin, range_end, thresh, verbosity, fname, fcomm, algorithm, options) &
        bind(c, name='IterativeSolverNonLinearEquationsInitialize')
      import :: c_size_t, c_double, c_int, c_int64_t, c_char
      integer(c_size_t), value :: n
      integer(c_size_t), intent(inout) :: range_begin, range_end
      real(c_double), value :: thresh
      integer(c_int), value :: verbosity
      character(kind=c_char), dimension(*), intent(in) :: fname, algorithm, options
      integer(c_int64_t), value :: fcomm
    end subroutine c_diis_init
    subroutine c_optimize_init(n, range_begin, range_end, thresh, thresh_value, verbosity, minimize, fname, fcomm, &
        algorithm, options) bind(c, name='IterativeSolverOptimizeInitialize')
      import :: c_size_t, c_double, c_int, c_int64_t, c_char
      integer(c_size_t), value :: n
      integer(c_size_t), intent(inout) :: range_begin, range_end
      real(c_double), value :: thresh, thresh_value
      integer(c_int), value :: verbosity, minimize
      character(kind=c_char), dimension(*), intent(in) :: fname, algorithm, options
      integer(c_int64_t), value :: fcomm
    end subroutine c_optimize_init
    subroutine Iterative_Solver_Finalize() bind(c, name='IterativeSolverFinalize')
    end subroutine Iterative_Solver_Finalize
    integer(c_size_t) function c_add_vector(buffer_size, parameters, action, sync) &
        bind(c, name='IterativeSolverAddVector')
      import :: c_size_t, c_ptr, c_int
      integer(c_size_t), value :: buffer_size
      type(c_ptr), value :: parameters, action
      integer(c_int), value :: sync
    end function c_add_vector
    integer(c_size_t) function c_add_value(value, parameters, action, sync) bind(c, name='IterativeSolverAddValue')
      import :: c_size_t, c_ptr, c_int, c_double
      real(c_double), value :: value
      type(c_ptr), value :: parameters, action
      integer(c_int), value :: sync
    end function c_add_value
    integer(c_size_t) function c_end_iteration(buffer_size, solution, residual, sync) &
        bind(c, name='IterativeSolverEndIteration')
      import :: c_size_t, c_ptr, c_int
      integer(c_size_t), value :: buffer_size
      type(c_ptr), value :: solution, residual
      integer(c_int), value :: sync
    end function c_end_iteration
    integer(c_int) function c_end_iteration_needed() bind(c, name='IterativeSolverEndIterationNeeded')
      import :: c_int
    end function c_end_iteration_needed
    subroutine c_solution(nroot, roots, parameters, action, sync) bind(c, name='IterativeSolverSolution')
      import :: c_int, c_ptr
      integer(c_int), value :: nroot
      integer(c_int), dimension(*), intent(in) :: roots
      type(c_ptr), value :: parameters, action
      integer(c_int), value :: sync
    end subroutine c_solution
    integer(c_size_t) function c_add_p(buffer_size, np, offsets, indices, coefficients, pp, parameters, action, &
        sync, func) bind(c, name='IterativeSolverAddP')
      import :: c_size_t, c_double, c_ptr, c_int, c_funptr
      integer(c_size_t), value :: buffer_size, np
      integer(c_size_t), dimension(*), intent(in) :: offsets, indices
      real(c_double), dimension(*), intent(in) :: coefficients, pp
      type(c_ptr), value :: parameters, action
      integer(c_int), value :: sync
      type(c_funptr), value :: func
    end function c_add_p
    integer(c_size_t) function c_suggest_p(solution, residual, maximum_number, threshold, indices) &
        bind(c, name='IterativeSolverSuggestP')
      import :: c_size_t, c_double
      real(c_double), dimension(*), intent(in) :: solution, residual
      integer(c_size_t), value :: maximum_number
      real(c_double), value :: threshold
      integer(c_size_t), dimension(*), intent(inout) :: indices
    end function c_suggest_p
    subroutine c_errors(errors) bind(c, name='IterativeSolverErrors')
      import :: c_double
      real(c_double), dimension(*), intent(inout) :: errors
    end subroutine c_errors
    subroutine c_eigenvalues(eigenvalues) bind(c, name='IterativeSolverEigenvalues')
      import :: c_double
      real(c_double), dimension(*), intent(inout) :: eigenvalues
    end subroutine c_eigenvalues
    subroutine c_working_set_eigenvalues(eigenvalues) bind(c, name='IterativeSolverWorkingSetEigenvalues')
      import :: c_double
      real(c_double), dimension(*), intent(inout) :: eigenvalues
    end subroutine c_working_set_eigenvalues
    integer(c_size_t) function c_nroots() bind(c, name='IterativeSolverHbmNRoots')
      import :: c_size_t
    end function c_nroots
    subroutine Iterative_Solver_Print_Statistics() bind(c, name='IterativeSolverPrintStatistics')
    end subroutine Iterative_Solver_Print_Statistics
    real(c_double) function Iterative_Solver_Value() bind(c, name='IterativeSolverValue')
      import :: c_double
    end function Iterative_Solver_Value
    integer(c_int) function Iterative_Solver_Verbosity() bind(c, name='IterativeSolverVerbosity')
      import :: c_int
    end function Iterative_Solver_Verbosity
    integer(c_int) function c_nonlinear() bind(c, name='IterativeSolverNonLinear')
      import :: c_int
    end function c_nonlinear
    integer(c_int) function c_has_values() bind(c, name='IterativeSolverHasValues')
      import :: c_int
    end function c_has_values
    integer(c_int) function c_has_eigenvalues() bind(c, name='IterativeSolverHasEigenvalues')
      import :: c_int
    end function c_has_eigenvalues
    integer(c_int) function c_max_iter() bind(c, name='IterativeSolverMaxIter')
      import :: c_int
    end function c_max_iter
    subroutine c_set_max_iter(max_iter) bind(c, name='IterativeSolverSetMaxIter')
      import :: c_int
      integer(c_int), value :: max_iter
    end subroutine c_set_max_iter
    subroutine c_set_diagonals(diagonals) bind(c, name='IterativeSolverSetDiagonals')
      import :: c_double
      real(c_double), dimension(*), intent(in) :: diagonals
    end subroutine c_set_diagonals
    subroutine c_diagonals(diagonals) bind(c, name='IterativeSolverDiagonals')
      import :: c_double
      real(c_double), dimension(*), intent(inout) :: diagonals
    end subroutine c_diagonals
    integer(c_int64_t) function c_mpicomm_global() bind(c, name='IterativeSolver_mpicomm_global')
      import :: c_int64_t
    end function c_mpicomm_global
    integer(c_int64_t) function c_mpicomm_self() bind(c, name='IterativeSolver_mpicomm_self')
      import :: c_int64_t
    end function c_mpicomm_self
    integer(c_int) function c_mpi_init() bind(c, name='IterativeSolver_mpi_init')
      import :: c_int
    end function c_mpi_init
    integer(c_int) function c_mpi_finalize() bind(c, name='IterativeSolver_mpi_finalize')
      import :: c_int
    end function c_mpi_finalize
    integer(c_int64_t) function mpi_size_global() bind(c, name='IterativeSolver_mpisize_global')
      import :: c_int64_t
    end function mpi_size_global
    integer(c_int64_t) function mpi_rank_global() bind(c, name='IterativeSolver_mpirank_global')
      import :: c_int64_t
    end function mpi_rank_global
  end interface

contains

  ! ---- communicators (IterativeSolverF.F90:20-73) ------------------------------------------------
  integer(kind=mpicomm_kind) function mpicomm_global()
    mpicomm_global = int(c_mpicomm_global(), mpicomm_kind)
  end function mpicomm_global

  integer(kind=mpicomm_kind) function mpicomm_self()
    mpicomm_self = int(c_mpicomm_self(), mpicomm_kind)
  end function mpicomm_self

  !> The communicator Initialize uses when none is passed: set_mpicomm_compute's, else the global one.
  integer(kind=mpicomm_kind) function mpicomm_compute()
    if (.not. compute_comm_set) then
      compute_comm = mpicomm_global()
      compute_comm_set = .true.
    end if
    mpicomm_compute = compute_comm
  end function mpicomm_compute

  subroutine set_mpicomm_compute(comm)
    integer(kind=mpicomm_kind), intent(in) :: comm
    compute_comm = comm
    compute_comm_set = .true.
  end subroutine set_mpicomm_compute

  subroutine mpi_init()
    integer(c_int) :: status
    status = c_mpi_init()
  end subroutine mpi_init

  subroutine mpi_finalize()
    integer(c_int) :: status
    status = c_mpi_finalize()
  end subroutine mpi_finalize

  ! ---- argument helpers ----------------------------------------------------------------------------
  !> NUL-terminated copy of a Fortran string (trailing blanks dropped); "" when absent.
  function c_string(s) result(c)
    character(len=*), intent(in), optional :: s
    character(kind=c_char, len=:), allocatable :: c
    if (present(s)) then
      c = trim(s)//c_null_char
    else
      c = c_null_char
    end if
  end function c_string

  real(c_double) function real_or(x, default)
    double precision, intent(in), optional :: x
    double precision, intent(in) :: default
    real_or = default
    if (present(x)) real_or = x
  end function real_or

  integer(c_int) function int_or(i, default)
    integer, intent(in), optional :: i
    integer, intent(in) :: default
    int_or = int(default, c_int)
    if (present(i)) int_or = int(i, c_int)
  end function int_or

  integer(c_int) function flag_or(l, default)
    logical, intent(in), optional :: l
    logical, intent(in) :: default
    logical :: v
    v = default
    if (present(l)) v = l
    flag_or = merge(1_c_int, 0_c_int, v)
  end function flag_or

  integer(c_int64_t) function comm_or_compute(comm)
    integer(kind=mpicomm_kind), intent(in), optional :: comm
    if (present(comm)) then
      comm_or_compute = int(comm, c_int64_t)
    else
      comm_or_compute = int(mpicomm_compute(), c_int64_t)
    end if
  end function comm_or_compute

  !> Number of vectors an R buffer holds: 1 for a scalar or a single vector, else the product of
  !> the extents beyond the first (columns of a matrix).
  integer(c_size_t) function columns(a)
    double precision, dimension(..), intent(in) :: a
    if (rank(a) <= 1 .or. size(a, 1) == 0) then
      columns = 1
    else
      columns = int(size(a, kind=c_size_t) / size(a, 1, kind=c_size_t), c_size_t)
    end if
  end function columns

  subroutine range_in(range, b, e)
    integer, dimension(2), intent(in), optional :: range
    integer(c_size_t), intent(out) :: b, e
    b = 0
    e = 0
    if (present(range)) then
      b = int(range(1), c_size_t)
      e = int(range(2), c_size_t)
    end if
  end subroutine range_in

  subroutine range_out(range, b, e)
    integer, dimension(2), intent(inout), optional :: range
    integer(c_size_t), intent(in) :: b, e
    if (present(range)) range = [int(b), int(e)]
  end subroutine range_out

  ! ---- Initialize (IterativeSolverF.F90:75-468) ----------------------------------------------------
  !> Lowest eigensolutions of a matrix (Davidson by default).
  subroutine eigensystem_init_sizet(nq, nroot, thresh, thresh_value, hermitian, verbosity, pname, mpicomm, &
      algorithm, range, options)
    integer(c_int64_t), intent(in) :: nq, nroot
    double precision, intent(in), optional :: thresh, thresh_value
    logical, intent(in), optional :: hermitian
    integer, intent(in), optional :: verbosity
    character(len=*), intent(in), optional :: pname, algorithm, options
    integer(kind=mpicomm_kind), intent(in), optional :: mpicomm
    integer, dimension(2), intent(inout), optional :: range
    integer(c_size_t) :: b, e
    call range_in(range, b, e)
    call c_eigensystem_init(int(nq, c_size_t), int(nroot, c_size_t), b, e, real_or(thresh, 1d-10), &
        real_or(thresh_value, 1d50), flag_or(hermitian, .false.), int_or(verbosity, 0), c_string(pname), &
        comm_or_compute(mpicomm), c_string(algorithm), c_string(options))
    call range_out(range, b, e)
  end subroutine eigensystem_init_sizet

  subroutine eigensystem_init_default(nq, nroot, thresh, thresh_value, hermitian, verbosity, pname, mpicomm, &
      algorithm, range, options)
    integer, intent(in) :: nq, nroot
    double precision, intent(in), optional :: thresh, thresh_value
    logical, intent(in), optional :: hermitian
    integer, intent(in), optional :: verbosity
    character(len=*), intent(in), optional :: pname, algorithm, options
    integer(kind=mpicomm_kind), intent(in), optional :: mpicomm
    integer, dimension(2), intent(inout), optional :: range
    call eigensystem_init_sizet(int(nq, c_int64_t), int(nroot, c_int64_t), thresh, thresh_value, hermitian, &
        verbosity, pname, mpicomm, algorithm, range, options)
  end subroutine eigensystem_init_default

  !> Linear equations A x = rhs (one column of rhs per root); augmented_hessian 0 (default) solves
  !> them unmodified, 1 the augmented-Hessian problem, other values scale its damping.
  subroutine equations_init_sizet(nq, nroot, rhs, augmented_hessian, thresh, thresh_value, hermitian, verbosity, &
      pname, mpicomm, algorithm, range, options)
    integer(c_int64_t), intent(in) :: nq, nroot
    double precision, intent(in), dimension(nq, nroot) :: rhs
    double precision, intent(in), optional :: augmented_hessian, thresh, thresh_value
    logical, intent(in), optional :: hermitian
    integer, intent(in), optional :: verbosity
    character(len=*), intent(in), optional :: pname, algorithm, options
    integer(kind=mpicomm_kind), intent(in), optional :: mpicomm
    integer, dimension(2), intent(inout), optional :: range
    integer(c_size_t) :: b, e
    call range_in(range, b, e)
    call c_equations_init(int(nq, c_size_t), int(nroot, c_size_t), b, e, rhs, real_or(augmented_hessian, 0d0), &
        real_or(thresh, 1d-10), real_or(thresh_value, 1d50), flag_or(hermitian, .false.), int_or(verbosity, 0), &
        c_string(pname), comm_or_compute(mpicomm), c_string(algorithm), c_string(options))
    call range_out(range, b, e)
  end subroutine equations_init_sizet

  subroutine equations_init_default(nq, nroot, rhs, augmented_hessian, thresh, thresh_value, hermitian, verbosity, &
      pname, mpicomm, algorithm, range, options)
    integer, intent(in) :: nq, nroot
    double precision, intent(in), dimension(nq, nroot) :: rhs
    double precision, intent(in), optional :: augmented_hessian, thresh, thresh_value
    logical, intent(in), optional :: hermitian
    integer, intent(in), optional :: verbosity
    character(len=*), intent(in), optional :: pname, algorithm, options
    integer(kind=mpicomm_kind), intent(in), optional :: mpicomm
    integer, dimension(2), intent(inout), optional :: range
    call equations_init_sizet(int(nq, c_int64_t), int(nroot, c_int64_t), rhs, augmented_hessian, thresh, &
        thresh_value, hermitian, verbosity, pname, mpicomm, algorithm, range, options)
  end subroutine equations_init_default

  !> Non-linear equations accelerated by DIIS (the default) or a related method.
  subroutine diis_init_sizet(nq, thresh, verbosity, pname, mpicomm, algorithm, range, options)
    integer(c_int64_t), intent(in) :: nq
    double precision, intent(in), optional :: thresh
    integer, intent(in), optional :: verbosity
    character(len=*), intent(in), optional :: pname, algorithm, options
    integer(kind=mpicomm_kind), intent(in), optional :: mpicomm
    integer, dimension(2), intent(inout), optional :: range
    integer(c_size_t) :: b, e
    call range_in(range, b, e)
    call c_diis_init(int(nq, c_size_t), b, e, real_or(thresh, 1d-10), int_or(verbosity, 0), c_string(pname), &
        comm_or_compute(mpicomm), c_string(algorithm), c_string(options))
    call range_out(range, b, e)
  end subroutine diis_init_sizet

  subroutine diis_init_default(nq, thresh, verbosity, pname, mpicomm, algorithm, range, options)
    integer, intent(in) :: nq
    double precision, intent(in), optional :: thresh
    integer, intent(in), optional :: verbosity
    character(len=*), intent(in), optional :: pname, algorithm, options
    integer(kind=mpicomm_kind), intent(in), optional :: mpicomm
    integer, dimension(2), intent(inout), optional :: range
    call diis_init_sizet(int(nq, c_int64_t), thresh, verbosity, pname, mpicomm, algorithm, range, options)
  end subroutine diis_init_default

  !> Minimisation (L-BFGS by default, or "SD").
  subroutine optimize_init_sizet(nq, thresh, verbosity, minimize, pname, mpicomm, algorithm, range, thresh_value, &
      options)
    integer(c_int64_t), intent(in) :: nq
    double precision, intent(in), optional :: thresh, thresh_value
    integer, intent(in), optional :: verbosity
    logical, intent(in), optional :: minimize
    character(len=*), intent(in), optional :: pname, algorithm, options
    integer(kind=mpicomm_kind), intent(in), optional :: mpicomm
    integer, dimension(2), intent(inout), optional :: range
    integer(c_size_t) :: b, e
    call range_in(range, b, e)
    call c_optimize_init(int(nq, c_size_t), b, e, real_or(thresh, 1d-10), real_or(thresh_value, 1d50), &
        int_or(verbosity, 0), flag_or(minimize, .true.), c_string(pname), comm_or_compute(mpicomm), &
        c_string(algorithm), c_string(options))
    call range_out(range, b, e)
  end subroutine optimize_init_sizet

  subroutine optimize_init_default(nq, thresh, verbosity, minimize, pname, mpicomm, algorithm, range, thresh_value, &
      options)
    integer, intent(in) :: nq
    double precision, intent(in), optional :: thresh, thresh_value
    integer, intent(in), optional :: verbosity
    logical, intent(in), optional :: minimize
    character(len=*), intent(in), optional :: pname, algorithm, options
    integer(kind=mpicomm_kind), intent(in), optional :: mpicomm
    integer, dimension(2), intent(inout), optional :: range
    call optimize_init_sizet(int(nq, c_int64_t), thresh, verbosity, minimize, pname, mpicomm, algorithm, range, &
        thresh_value, options)
  end subroutine optimize_init_default

  ! ---- the iteration (IterativeSolverF.F90:480-770) ------------------------------------------------
  !> Add the current parameters and their action (linear) or residual (non-linear; with `value`,
  !> the objective function for Optimize) to the subspace.  On exit parameters and action hold the
  !> working set's solutions and residuals; returns the working-set size (for Optimize with value:
  !> 1, or 0 when the solver line-searches and the residual must not be preconditioned).
  integer function Iterative_Solver_Add_Vector(parameters, action, synchronize, value)
    double precision, dimension(..), contiguous, target, intent(inout) :: parameters, action
    logical, intent(in), optional :: synchronize
    double precision, intent(in), optional :: value
    if (present(value)) then
      Iterative_Solver_Add_Vector = int(c_add_value(value, c_loc(parameters), c_loc(action), &
          flag_or(synchronize, .true.)))
    else
      Iterative_Solver_Add_Vector = int(c_add_vector(columns(parameters), c_loc(parameters), c_loc(action), &
          flag_or(synchronize, .true.)))
    end if
  end function Iterative_Solver_Add_Vector

  !> Solutions and residuals of the given roots (1-based), one column each.
  subroutine Iterative_Solver_Solution(roots, parameters, action, synchronize)
    integer, intent(in), dimension(:) :: roots
    double precision, dimension(..), contiguous, target, intent(inout) :: parameters, action
    logical, intent(in), optional :: synchronize
    integer(c_int), dimension(size(roots)) :: roots0
    roots0 = int(roots - 1, c_int)
    call c_solution(int(size(roots), c_int), roots0, c_loc(parameters), c_loc(action), flag_or(synchronize, .true.))
  end subroutine Iterative_Solver_Solution

  !> Take the preconditioned residuals, return the next working set's parameters; returns its size.
  integer function Iterative_Solver_End_Iteration(solution, residual, synchronize)
    double precision, dimension(..), contiguous, target, intent(inout) :: solution, residual
    logical, intent(in), optional :: synchronize
    Iterative_Solver_End_Iteration = int(c_end_iteration(columns(solution), c_loc(solution), c_loc(residual), &
        flag_or(synchronize, .true.)))
  end function Iterative_Solver_End_Iteration

  logical function Iterative_Solver_End_Iteration_Needed()
    Iterative_Solver_End_Iteration_Needed = c_end_iteration_needed() /= 0
  end function Iterative_Solver_End_Iteration_Needed

  !> Add nP P-space vectors: vector k has the coefficients(offsets(k-1)+1 : offsets(k)) at the
  !> (1-based) indices of the same positions; pp is the P-P block (existing P + nP) x nP.  fproc is
  !> a bind(c) routine (p, g, nvec, ranges) that adds the P-space part of the action to g.
  integer function Iterative_Solver_Add_P(nP, offsets, indices, coefficients, pp, parameters, action, fproc, &
      synchronize)
    integer, intent(in) :: nP
    integer, intent(in), dimension(0:nP) :: offsets
    integer, intent(in), dimension(offsets(nP)) :: indices
    double precision, dimension(offsets(nP)), intent(in) :: coefficients
    double precision, dimension(*), intent(in) :: pp
    double precision, dimension(:, :), contiguous, target, intent(inout) :: parameters, action
    external :: fproc
    logical, intent(in), optional :: synchronize
    integer(c_size_t), dimension(0:nP) :: offsets_c
    integer(c_size_t), dimension(max(1, offsets(nP))) :: indices_c
    offsets_c = int(offsets, c_size_t)
    indices_c = 0
    if (offsets(nP) > 0) indices_c(1:offsets(nP)) = int(indices - 1, c_size_t)
    Iterative_Solver_Add_P = int(c_add_p(int(size(parameters, 2), c_size_t), int(nP, c_size_t), offsets_c, &
        indices_c, coefficients, pp, c_loc(parameters), c_loc(action), flag_or(synchronize, .true.), &
        c_funloc(fproc)))
  end function Iterative_Solver_Add_P

  !> Suggested P-space indices (1-based) for the current solution; returns how many were filled.
  integer function Iterative_Solver_Suggest_P(solution, residual, indices, threshold)
    double precision, dimension(*), intent(in) :: solution, residual
    integer, intent(inout), dimension(:) :: indices
    double precision, intent(in), optional :: threshold
    integer(c_size_t), dimension(max(1, size(indices))) :: indices_c
    integer :: k
    indices_c = 0
    Iterative_Solver_Suggest_P = int(c_suggest_p(solution, residual, int(size(indices), c_size_t), &
        real_or(threshold, 0d0), indices_c))
    do k = 1, Iterative_Solver_Suggest_P
      indices(k) = int(indices_c(k)) + 1
    end do
  end function Iterative_Solver_Suggest_P

  !> Residual norm of each root.
  function Iterative_Solver_Errors() result(errors)
    double precision, dimension(:), allocatable :: errors
    allocate (errors(max(1_c_size_t, c_nroots())))
    errors = 0d0
    call c_errors(errors)
    errors = errors(1:c_nroots())
  end function Iterative_Solver_Errors

  !> Current eigenvalues of all the roots sought.
  function Iterative_Solver_Eigenvalues() result(eigenvalues)
    double precision, dimension(:), allocatable :: eigenvalues
    allocate (eigenvalues(max(1_c_size_t, c_nroots())))
    eigenvalues = 0d0
    call c_eigenvalues(eigenvalues)
    eigenvalues = eigenvalues(1:c_nroots())
  end function Iterative_Solver_Eigenvalues

  !> Eigenvalues of the working set (the roots not yet converged); zero for solvers without.
  function Iterative_Solver_Working_Set_Eigenvalues(working_set_size) result(eigenvalues)
    integer, intent(in) :: working_set_size
    double precision, dimension(working_set_size) :: eigenvalues
    double precision, dimension(:), allocatable :: buffer
    allocate (buffer(max(1_c_size_t, c_nroots(), int(working_set_size, c_size_t))))
    buffer = 0d0
    call c_working_set_eigenvalues(buffer)
    eigenvalues = buffer(1:working_set_size)
  end function Iterative_Solver_Working_Set_Eigenvalues

  ! ---- the simplified driver (IterativeSolverF.F90:814-924) ----------------------------------------
  !> Iterate the solver initialised last to convergence (or max_iter iterations) on `problem`.
  !> parameters/actions: one column per root (a vector for a single root).  With
  !> generate_initial_guess, the parameters start as unit vectors on the smallest diagonals (the
  !> problem must provide them).  Linear solvers call problem%action, non-linear ones
  !> problem%residual; the preconditioner is problem%precondition, given the working-set
  !> eigenvalues as shifts and, when the problem has them, the diagonals.
  subroutine Iterative_Solver_Solve(parameters, actions, problem, generate_initial_guess, max_iter)
    use Iterative_Solver_Problem, only: problem_class => Problem
    double precision, dimension(..), contiguous, target, intent(inout) :: parameters, actions
    class(problem_class), intent(in) :: problem
    logical, intent(in), optional :: generate_initial_guess
    integer, intent(in), optional :: max_iter
    double precision, dimension(:, :), pointer :: x, g
    double precision :: value
    integer :: n, nbuffer, nwork, iter, verbosity, i, k
    logical :: use_diagonals, reported, nonlinear

    n = 1
    if (rank(parameters) >= 1) n = size(parameters, 1)
    nbuffer = int(columns(parameters))
    call c_f_pointer(c_loc(parameters), x, [n, nbuffer])
    call c_f_pointer(c_loc(actions), g, [n, nbuffer])
    verbosity = Iterative_Solver_Verbosity()
    if (present(max_iter)) call c_set_max_iter(int(max_iter, c_int))
    nonlinear = c_nonlinear() > 0

    ! the first action column is scratch for the diagonals (as in the reference)
    use_diagonals = problem%diagonals(g(:, 1))
    if (use_diagonals) call c_set_diagonals(g(:, 1))
    if (verbosity >= 3) write (6, *) 'IterativeSolver_Solve nonlinear=', c_nonlinear(), ' use_diagonals=', &
        use_diagonals
    if (present(generate_initial_guess)) then
      if (generate_initial_guess) then
        if (.not. use_diagonals) error stop 'Default initial guess requested, but diagonal elements are not available'
        x = 0d0
        do i = 1, nbuffer
          k = minloc(g(:, 1), 1)
          x(k, i) = 1d0
          g(k, 1) = 1d50
        end do
      end if
    end if

    nwork = nbuffer
    value = 0d0
    do iter = 1, c_max_iter()
      if (nonlinear) then
        value = problem%residual(x, g)
        nwork = Iterative_Solver_Add_Vector(x, g, value=value)
      else
        call problem%action(x, g)
        nwork = Iterative_Solver_Add_Vector(x, g)
      end if
      do while (Iterative_Solver_End_Iteration_Needed())
        if (nwork > 0) then
          if (use_diagonals) then
            ! the first parameter column is scratch for the diagonals (as in the reference)
            call c_diagonals(x(:, 1))
            call problem%precondition(g(:, :nwork), Iterative_Solver_Working_Set_Eigenvalues(nwork), x(:, 1))
          else
            call problem%precondition(g(:, :nwork), Iterative_Solver_Working_Set_Eigenvalues(nwork))
          end if
        end if
        nwork = Iterative_Solver_End_Iteration(x, g)
      end do
      if (nwork <= 0) verbosity = verbosity + 1
      if (c_has_values() /= 0) then
        reported = problem%report(iter, verbosity, Iterative_Solver_Errors(), value=Iterative_Solver_Value())
      else if (c_has_eigenvalues() /= 0) then
        reported = problem%report(iter, verbosity, Iterative_Solver_Errors(), eigenvalues=Iterative_Solver_Eigenvalues())
      else
        reported = problem%report(iter, verbosity, Iterative_Solver_Errors())
      end if
      if (.not. reported .and. verbosity >= 2) then
        write (6, '(A,I3,1X,A,(T32,10F7.2))') 'Iteration', iter, 'log10(|residual|)=', log10(Iterative_Solver_Errors())
        if (c_has_values() > 0) write (6, *) 'Objective function value ', Iterative_Solver_Value()
      end if
      if (nwork < 1) exit
    end do
    if (c_has_values() /= 0) then
      reported = problem%report(-nwork, verbosity, Iterative_Solver_Errors(), value=Iterative_Solver_Value())
    else
      reported = problem%report(-nwork, verbosity, Iterative_Solver_Errors())
    end if
  end subroutine Iterative_Solver_Solve

end module Iterative_Solver
