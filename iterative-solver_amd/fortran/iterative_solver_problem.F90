!> Problem class of the simplified Fortran driver Iterative_Solver_Solve (module Iterative_Solver).
!>
!> Restates the reference's Iterative_Solver_Problem module
!> (src/molpro/linalg/Iterative_Solver_Problem.F90:1-139): a base type whose type-bound procedures a
!> caller overrides (action for the linear solvers, residual for the non-linear ones, diagonals and
!> precondition, report), and Matrix_Problem, whose action and diagonals come from an explicit
!> matrix.  Same names, argument meaning and defaults as the reference:
!>  - diagonals() returns .false. (no diagonal preconditioner);
!>  - precondition(action, shift, diagonals) divides by (diagonals + shift + 1e-14) when diagonals
!>    are passed, and does nothing otherwise (reference :56-75 -- note the + shift; the C++
!>    default preconditioner, IterativeSolver.h:47-55, uses d - shift);
!>  - residual() zeroes the residuals and returns an undefined value, action() does nothing;
!>  - report() prints the reference's progress lines and returns .true.
module Iterative_Solver_Problem
  implicit none
  private

  type, public :: Problem
  contains
    procedure, pass :: diagonals
    procedure, pass :: precondition
    procedure, pass :: residual
    procedure, pass :: action
    procedure, pass :: report
  end type Problem

  !> A problem given by its (dense, column-major) matrix: action = matrix . parameters.
  type, public, extends(Problem) :: Matrix_Problem
    double precision, pointer, dimension(:, :) :: matrix => null()
  contains
    procedure, pass :: diagonals => matrix_diagonals
    procedure, pass :: action => matrix_action
  end type Matrix_Problem

  double precision, parameter :: precondition_floor = 1d-14

contains

  !> Diagonal elements of the kernel, if the problem can provide them (then .true.).
  logical function diagonals(this, d)
    class(Problem), intent(in) :: this
    double precision, intent(inout), dimension(:) :: d
    diagonals = .false.
  end function diagonals

  logical function matrix_diagonals(this, d)
    class(Matrix_Problem), intent(in) :: this
    double precision, intent(inout), dimension(:) :: d
    integer :: i, i0
    i0 = lbound(this%matrix, 1)
    do i = 1, size(d)
      d(i) = this%matrix(i0 + i - 1, lbound(this%matrix, 2) + i - 1)
    end do
    matrix_diagonals = .true.
  end function matrix_diagonals

  !> Turn residuals into (minus) predicted steps; with `diagonals`, divide element-wise by
  !> diagonals + shift(column) (+ a small floor).
  subroutine precondition(this, action, shift, diagonals)
    class(Problem), intent(in) :: this
    double precision, intent(inout), dimension(:, :) :: action
    double precision, intent(in), dimension(:), optional :: shift
    double precision, intent(in), dimension(:), optional :: diagonals
    integer :: k
    double precision :: s
    if (.not. present(diagonals)) return
    do k = 1, size(action, 2)
      s = 0d0
      if (present(shift)) s = shift(k)
      action(:, k) = action(:, k) / (diagonals(1:size(action, 1)) + s + precondition_floor)
    end do
  end subroutine precondition

  !> Residual of the non-linear solvers; returns the objective function value where one exists.
  function residual(this, parameters, residuals) result(value)
    class(Problem), intent(in) :: this
    double precision, intent(in), dimension(:, :) :: parameters
    double precision, intent(inout), dimension(:, :) :: residuals
    double precision :: value
    residuals = 0d0
    value = 0d0
  end function residual

  !> Action of the kernel on each column of parameters (linear solvers).
  subroutine action(this, parameters, actions)
    class(Problem), intent(in) :: this
    double precision, intent(in), dimension(:, :) :: parameters
    double precision, intent(inout), dimension(:, :) :: actions
  end subroutine action

  subroutine matrix_action(this, parameters, actions)
    class(Matrix_Problem), intent(in) :: this
    double precision, intent(in), dimension(:, :) :: parameters
    double precision, intent(inout), dimension(:, :) :: actions
    actions = matmul(this%matrix, parameters)
  end subroutine matrix_action

  !> Progress report: iteration > 0 during the iterations, 0 on convergence, < 0 when unconverged.
  !> Prints at verbosity >= 2 every iteration and at verbosity >= 1 at the end; returns .true.
  logical function report(this, iteration, verbosity, errors, value, eigenvalues)
    class(Problem), intent(in) :: this
    integer, intent(in) :: iteration
    integer, intent(in) :: verbosity
    double precision, intent(in), dimension(:) :: errors
    double precision, intent(in), optional :: value
    double precision, dimension(:), intent(in), optional :: eigenvalues
    report = .true.
    if (verbosity < 2 .and. .not. (iteration <= 0 .and. verbosity >= 1)) return
    if (iteration > 0) then
      write (6, '(A,I3,1X,A,(T32,10F7.2))') 'Iteration', iteration, 'log10(|residual|)=', log10(errors)
    else if (iteration == 0) then
      write (6, '(A,(T32,10F7.2))') 'Converged,   log10(|residual|)=', log10(errors)
    else
      write (6, '(A,(T32,10F7.2))') 'Unconverged, log10(|residual|)=', log10(errors)
    end if
    if (present(value)) write (6, *) 'Objective function value ', value
    if (present(eigenvalues)) write (6, *) 'Eigenvalues ', eigenvalues
  end function report

end module Iterative_Solver_Problem
