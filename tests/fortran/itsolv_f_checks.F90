! Fortran callers of module Iterative_Solver for tests/test_fortran.py (test infrastructure).
!
! Each check is a bind(c) function driving one solver family through the Fortran binding the way the
! reference's Fortran tests and examples do, and returning what the Python side compares: iteration
! counts, eigenvalues, errors, solutions.  They restate
!   test/itsolv/test_LinearEigensystemF.f90:1-74  (f_eigensystem: lowest-diagonal guess, Add_Vector,
!                                                  Working_Set_Eigenvalues shift, End_Iteration)
!   test/itsolv/test_LinearEquationsF.f90:1-86    (f_linear_equations: -rhs/diag guess, Solution)
!   test/itsolv/test_OptimizeF.f90:1-45           (f_optimize: f = (x-1).H.(x-1)/2 with its value)
!   examples/LinearEigensystemExampleF-problem.F90 (f_solve_matrix: Iterative_Solver_Solve, Matrix_Problem)
!   examples/OptimizeExampleF-problem.F90          (f_solve_forced: Solve with a Problem extension)
!   examples/LinearEigensystemExampleF-Pspace.F90  (f_pspace: Add_P with a bind(c) P-space action)
! plus a DIIS loop (f_diis: r = H(x-1), the reference's C++ test_NonLinearEquations.cpp:60-85; its
! Fortran file test_NonLinearEquationsF.f90 defines test_OptimizeF again).
module itsolv_f_checks
  use, intrinsic :: iso_c_binding
  use Iterative_Solver
  use Iterative_Solver_Problem, only: Problem, Matrix_Problem
  implicit none

  ! P-space action callback state (f_pspace)
  double precision, pointer, dimension(:, :) :: p_matrix => null()
  integer, allocatable, dimension(:) :: p_indices

  ! objective (1/2) c.m.c - sum(c), m(i,j) = 1 + (3i-1) delta(i,j) (OptimizeExampleF-problem.F90)
  type, extends(Problem) :: forced_problem
  contains
    procedure, pass :: residual => forced_residual
    procedure, pass :: diagonals => forced_diagonals
  end type forced_problem

contains

  ! ---- helpers ---------------------------------------------------------------------------------
  !> Index of the smallest diagonal element not yet taken (first one on ties), as the reference test.
  subroutine lowest_diagonals(matrix, picks)
    double precision, dimension(:, :), intent(in) :: matrix
    integer, dimension(:), intent(out) :: picks
    double precision, dimension(size(matrix, 1)) :: d
    integer :: i, k
    d = [(matrix(k, k), k = 1, size(matrix, 1))]
    do i = 1, size(picks)
      picks(i) = minloc(d, 1)
      d(picks(i)) = huge(1d0)
    end do
  end subroutine lowest_diagonals

  function forced_residual(this, parameters, residuals) result(e)
    class(forced_problem), intent(in) :: this
    double precision, intent(in), dimension(:, :) :: parameters
    double precision, intent(inout), dimension(:, :) :: residuals
    double precision :: e
    integer :: i
    ! m.c, then the objective and its gradient m.c - 1 (the reference example subtracts the 1 twice
    ! from its gradient, which then disagrees with its value)
    do i = 1, size(residuals, 1)
      residuals(i, 1) = sum(parameters(:, 1)) + (3 * i - 1) * parameters(i, 1)
    end do
    e = 0.5d0 * dot_product(parameters(:, 1), residuals(:, 1)) - sum(parameters(:, 1))
    residuals = residuals - 1
  end function forced_residual

  logical function forced_diagonals(this, d)
    class(forced_problem), intent(in) :: this
    double precision, intent(inout), dimension(:) :: d
    integer :: i
    d = [(3d0 * i, i = 1, size(d))]
    forced_diagonals = .true.
  end function forced_diagonals

  ! ---- LinearEigensystem -----------------------------------------------------------------------
  !> Davidson on a dense column-major matrix; returns the number of Add_Vector calls made.
  integer(c_int) function f_eigensystem(matrix, n, nroot, hermitian, thresh, options, eigenvalues, errors, &
      range_out) bind(c)
    integer(c_size_t), value :: n, nroot
    real(c_double), dimension(n, n), intent(in) :: matrix
    integer(c_int), value :: hermitian
    real(c_double), value :: thresh
    character(kind=c_char), dimension(*), intent(in) :: options
    real(c_double), dimension(nroot), intent(out) :: eigenvalues, errors
    integer(c_int), dimension(2), intent(out) :: range_out
    double precision, dimension(n, nroot) :: c, g
    double precision, allocatable, dimension(:) :: shift
    integer, dimension(nroot) :: guess
    integer, dimension(2) :: range
    integer :: nwork, it, k
    call Iterative_Solver_Linear_Eigensystem_Initialize(n, nroot, thresh=thresh, hermitian=hermitian /= 0, &
        range=range, options=fstring(options))
    range_out = range
    call lowest_diagonals(matrix, guess)
    c = 0
    do k = 1, int(nroot)
      c(guess(k), k) = 1
    end do
    f_eigensystem = 0
    do it = 1, 1000
      g = matmul(matrix, c)
      nwork = Iterative_Solver_Add_Vector(c, g)
      f_eigensystem = f_eigensystem + 1
      if (nwork <= 0) exit
      shift = Iterative_Solver_Working_Set_Eigenvalues(nwork)
      do k = 1, nwork
        g(:, k) = -g(:, k) / (diag(matrix) + 1d-12 - shift(k))
      end do
      nwork = Iterative_Solver_End_Iteration(c, g)
      if (nwork <= 0) exit
    end do
    eigenvalues = Iterative_Solver_Eigenvalues()
    errors = Iterative_Solver_Errors()
    call Iterative_Solver_Finalize
  end function f_eigensystem

  pure function diag(m) result(d)
    double precision, dimension(:, :), intent(in) :: m
    double precision, dimension(size(m, 1)) :: d
    integer :: k
    d = [(m(k, k), k = 1, size(m, 1))]
  end function diag

  !> Fortran string from a NUL-terminated C string.
  function fstring(s) result(f)
    character(kind=c_char), dimension(*), intent(in) :: s
    character(len=:), allocatable :: f
    integer :: k
    k = 0
    do while (s(k + 1) /= c_null_char)
      k = k + 1
    end do
    allocate (character(len=k) :: f)
    do k = 1, len(f)
      f(k:k) = s(k)
    end do
  end function fstring

  ! ---- LinearEquations -------------------------------------------------------------------------
  !> Solves matrix.x = rhs (column-major n x nroot); returns the number of Add_Vector calls.
  integer(c_int) function f_linear_equations(matrix, rhs, n, nroot, augmented_hessian, thresh, solution, &
      residual_norm) bind(c)
    integer(c_size_t), value :: n, nroot
    real(c_double), dimension(n, n), intent(in) :: matrix
    real(c_double), dimension(n, nroot), intent(in) :: rhs
    real(c_double), value :: augmented_hessian, thresh
    real(c_double), dimension(n, nroot), intent(out) :: solution
    real(c_double), intent(out) :: residual_norm
    double precision, dimension(n, nroot) :: c, g
    integer, dimension(nroot) :: roots
    integer :: nwork, it, k
    call Iterative_Solver_Linear_Equations_Initialize(n, nroot, rhs, augmented_hessian=augmented_hessian, &
        hermitian=.true., thresh=thresh, thresh_value=1d50)
    c = 0
    do k = 1, int(nroot)
      c(k:, k) = -rhs(k:, k) / diag(matrix(k:, k:))
    end do
    f_linear_equations = 0
    do it = 1, 1000
      g = matmul(matrix, c)
      nwork = Iterative_Solver_Add_Vector(c, g)
      f_linear_equations = f_linear_equations + 1
      if (nwork <= 0) exit
      do k = 1, nwork
        g(:, k) = -g(:, k) / diag(matrix)
      end do
      nwork = Iterative_Solver_End_Iteration(c, g)
      if (nwork <= 0) exit
    end do
    roots = [(k, k = 1, int(nroot))]
    call Iterative_Solver_Solution(roots, c, g)
    solution = c
    residual_norm = 0
    do k = 1, int(nroot)
      residual_norm = max(residual_norm, norm2(matmul(matrix, c(:, k)) - rhs(:, k)))
    end do
    call Iterative_Solver_Finalize
  end function f_linear_equations

  ! ---- Optimize --------------------------------------------------------------------------------
  !> Minimises (x-1).H.(x-1)/2 from x = e_1 with "BFGS" (algorithm 0) or "SD" (1).  Returns the
  !> number of Add_Vector calls; x and the final value on exit.
  integer(c_int) function f_optimize(matrix, n, algorithm, thresh, x, value) bind(c)
    integer(c_size_t), value :: n
    real(c_double), dimension(n, n), intent(in) :: matrix
    integer(c_int), value :: algorithm
    real(c_double), value :: thresh
    real(c_double), dimension(n), intent(out) :: x
    real(c_double), intent(out) :: value
    double precision, dimension(n) :: c, g
    double precision, dimension(n, 1) :: xs, gs
    integer :: nwork, it
    call Iterative_Solver_Optimize_Initialize(n, thresh=thresh, mpicomm=mpicomm_compute(), &
        algorithm=merge('BFGS', 'SD  ', algorithm == 0), minimize=.true.)
    c = 0
    c(1) = 1
    f_optimize = 0
    do it = 1, 1000
      g = matmul(matrix, c - 1)
      value = 0.5d0 * dot_product(g, c - 1)
      f_optimize = f_optimize + 1
      if (Iterative_Solver_Add_Vector(c, g, value=value) > 0) g = g / diag(matrix)
      nwork = Iterative_Solver_End_Iteration(c, g)
      if (nwork <= 0) exit
    end do
    call Iterative_Solver_Solution([1], xs, gs)
    x = xs(:, 1)
    value = Iterative_Solver_Value()
    call Iterative_Solver_Finalize
  end function f_optimize

  ! ---- NonLinearEquations (DIIS) ---------------------------------------------------------------
  !> Solves H(x-1) = 0 from x = e_1 with DIIS; returns the number of Add_Vector calls.
  integer(c_int) function f_diis(matrix, n, thresh, options, x, error) bind(c)
    integer(c_size_t), value :: n
    real(c_double), dimension(n, n), intent(in) :: matrix
    real(c_double), value :: thresh
    character(kind=c_char), dimension(*), intent(in) :: options
    real(c_double), dimension(n), intent(out) :: x
    real(c_double), intent(out) :: error
    double precision, dimension(n) :: c, g
    double precision, dimension(n, 1) :: xs, gs
    double precision, allocatable, dimension(:) :: errs
    integer :: nwork, it
    call Iterative_Solver_DIIS_Initialize(n, thresh=thresh, algorithm='DIIS', options=fstring(options))
    c = 0
    c(1) = 1
    f_diis = 0
    do it = 1, 1000
      g = matmul(matrix, c - 1)
      nwork = Iterative_Solver_Add_Vector(c, g)
      f_diis = f_diis + 1
      if (nwork <= 0) exit
      g = g / diag(matrix)
      nwork = Iterative_Solver_End_Iteration(c, g)
      if (nwork <= 0) exit
    end do
    call Iterative_Solver_Solution([1], xs, gs)
    x = xs(:, 1)
    errs = Iterative_Solver_Errors()
    error = errs(1)
    call Iterative_Solver_Finalize
  end function f_diis

  ! ---- the simplified driver -------------------------------------------------------------------
  !> Iterative_Solver_Solve on Matrix_Problem(matrix) with the generated initial guess.
  integer(c_int) function f_solve_matrix(matrix, n, nroot, thresh, max_iter, eigenvalues, errors) bind(c)
    integer(c_size_t), value :: n, nroot
    real(c_double), dimension(n, n), intent(in), target :: matrix
    real(c_double), value :: thresh
    integer(c_int), value :: max_iter
    real(c_double), dimension(nroot), intent(out) :: eigenvalues, errors
    double precision, dimension(n, nroot) :: c, g
    double precision, pointer, dimension(:, :) :: m
    integer(c_int) :: iterations, rcreate, qcreate
    interface
      integer(c_int) function statistics(it, r, q) bind(c, name='IterativeSolverHbmStatistics')
        import :: c_int
        integer(c_int), intent(out) :: it, r, q
      end function statistics
    end interface
    m => matrix
    call Iterative_Solver_Linear_Eigensystem_Initialize(int(n), int(nroot), thresh=thresh, hermitian=.true., &
        options='max_size_qspace=10')
    call Iterative_Solver_Solve(c, g, Matrix_Problem(m), max_iter=int(max_iter), generate_initial_guess=.true.)
    eigenvalues = Iterative_Solver_Eigenvalues()
    errors = Iterative_Solver_Errors()
    f_solve_matrix = -1
    if (statistics(iterations, rcreate, qcreate) == 0) f_solve_matrix = iterations
    call Iterative_Solver_Finalize
  end function f_solve_matrix

  !> Iterative_Solver_Solve minimising the forced quadratic of OptimizeExampleF-problem.F90.
  integer(c_int) function f_solve_forced(n, thresh, x, value) bind(c)
    integer(c_size_t), value :: n
    real(c_double), value :: thresh
    real(c_double), dimension(n), intent(out) :: x
    real(c_double), intent(out) :: value
    double precision, dimension(n) :: c, g
    type(forced_problem) :: problem
    call Iterative_Solver_Optimize_Initialize(int(n), thresh=thresh, algorithm='BFGS', options='max_size_qspace=3')
    c = 0
    c(1) = 1
    call Iterative_Solver_Solve(c, g, problem)
    call Iterative_Solver_Solution([1], c, g)
    x = c
    value = Iterative_Solver_Value()
    f_solve_forced = 0
    if (Iterative_Solver_Verbosity() == 0) f_solve_forced = 1
    call Iterative_Solver_Finalize
  end function f_solve_forced

  ! ---- P space ---------------------------------------------------------------------------------
  !> P-space action for f_pspace: g(:, i) += sum_k m(:, indices(k)) p(k, i) on this rank's range.
  subroutine apply_p(p, g, nvec, ranges) bind(c)
    integer(c_size_t), value :: nvec
    real(c_double), dimension(size(p_indices), nvec), intent(in) :: p
    real(c_double), dimension(size(p_matrix, 1), nvec), intent(inout) :: g
    integer(c_size_t), dimension(2, nvec), intent(in) :: ranges
    integer :: i, k
    integer(c_size_t) :: j0, j1
    do i = 1, int(nvec)
      j0 = ranges(1, i) + 1
      j1 = ranges(2, i)
      do k = 1, size(p_indices)
        g(j0:j1, i) = g(j0:j1, i) + p_matrix(j0:j1, p_indices(k)) * p(k, i)
      end do
    end do
  end subroutine apply_p

  !> Davidson with the first np unit vectors of the lowest diagonals as P space (Add_P), then
  !> Add_Vector/End_Iteration; returns the number of iterations.
  integer(c_int) function f_pspace(matrix, n, nroot, np, thresh, eigenvalues, errors) bind(c)
    integer(c_size_t), value :: n, nroot, np
    real(c_double), dimension(n, n), intent(in), target :: matrix
    real(c_double), value :: thresh
    real(c_double), dimension(nroot), intent(out) :: eigenvalues, errors
    double precision, dimension(n, nroot) :: c, g
    double precision, dimension(np, np) :: pp
    double precision, dimension(np) :: coefficients
    integer, dimension(0:np) :: offsets
    double precision, allocatable, dimension(:) :: e
    integer :: nwork, it, k, i
    p_matrix => matrix
    if (allocated(p_indices)) deallocate (p_indices)
    allocate (p_indices(np))
    call lowest_diagonals(matrix, p_indices)
    offsets = [(k, k = 0, int(np))]
    coefficients = 1
    do k = 1, int(np)
      do i = 1, int(np)
        pp(i, k) = matrix(p_indices(i), p_indices(k))
      end do
    end do
    call Iterative_Solver_Linear_Eigensystem_Initialize(n, nroot, thresh=thresh, hermitian=.true., &
        options='max_size_qspace=' // itoa(max(6 * int(nroot), min(int(n), min(1000, 6 * int(nroot))) - int(np))) &
        // ',reset_D=8')
    c = 0
    g = 0
    nwork = Iterative_Solver_Add_P(int(np), offsets, p_indices, coefficients, pp, c, g, apply_p, .true.)
    f_pspace = 1
    do it = 1, 1000
      e = Iterative_Solver_Working_Set_Eigenvalues(max(nwork, 1))
      do k = 1, nwork
        g(:, k) = -g(:, k) / (diag(matrix) + 1d-12 - e(k))
      end do
      nwork = Iterative_Solver_End_Iteration(c, g)
      if (nwork <= 0) exit
      g = matmul(matrix, c)
      nwork = Iterative_Solver_Add_Vector(c, g)
      f_pspace = f_pspace + 1
      if (nwork <= 0) exit
    end do
    eigenvalues = Iterative_Solver_Eigenvalues()
    errors = Iterative_Solver_Errors()
    call Iterative_Solver_Finalize
  end function f_pspace

  function itoa(i) result(s)
    integer, intent(in) :: i
    character(len=:), allocatable :: s
    character(len=24) :: buf
    write (buf, '(I0)') i
    s = trim(buf)
  end function itoa

  ! ---- communicator helpers --------------------------------------------------------------------
  !> mpi_init, size, rank, the communicators and mpi_finalize; returns size * 1000 + rank.
  integer(c_int) function f_mpi() bind(c)
    integer(kind=mpicomm_kind) :: comm
    call mpi_init
    comm = mpicomm_compute()
    call set_mpicomm_compute(mpicomm_self())
    comm = mpicomm_compute()
    call set_mpicomm_compute(mpicomm_global())
    f_mpi = int(mpi_size_global() * 1000 + mpi_rank_global(), c_int)
    call mpi_finalize
  end function f_mpi

end module itsolv_f_checks
