﻿!mod$ v1 sum:f580f73b9999a0d8
module iterative_solver_problem
type::problem
contains
procedure,pass::diagonals
procedure,pass::precondition
procedure,pass::residual
procedure,pass::action
procedure,pass::report
end type
type,extends(problem)::matrix_problem
real(8),pointer::matrix(:,:)=>NULL()
contains
procedure,pass::diagonals=>matrix_diagonals
procedure,pass::action=>matrix_action
end type
intrinsic::null
private::null
real(8),parameter,private::precondition_floor=9.999999999999999988193093545598986971343290729163921781719182035885751247406005859375e-15_8
private::diagonals
private::matrix_diagonals
private::precondition
private::residual
private::action
private::matrix_action
private::report
contains
function diagonals(this,d)
class(problem),intent(in)::this
real(8),intent(inout)::d(:)
logical(4)::diagonals
end
function matrix_diagonals(this,d)
class(matrix_problem),intent(in)::this
real(8),intent(inout)::d(:)
logical(4)::matrix_diagonals
end
subroutine precondition(this,action,shift,diagonals)
class(problem),intent(in)::this
real(8),intent(inout)::action(:,:)
real(8),intent(in),optional::shift(:)
real(8),intent(in),optional::diagonals(:)
end
function residual(this,parameters,residuals) result(value)
class(problem),intent(in)::this
real(8),intent(in)::parameters(:,:)
real(8),intent(inout)::residuals(:,:)
real(8)::value
end
subroutine action(this,parameters,actions)
class(problem),intent(in)::this
real(8),intent(in)::parameters(:,:)
real(8),intent(inout)::actions(:,:)
end
subroutine matrix_action(this,parameters,actions)
class(matrix_problem),intent(in)::this
real(8),intent(in)::parameters(:,:)
real(8),intent(inout)::actions(:,:)
end
function report(this,iteration,verbosity,errors,value,eigenvalues)
class(problem),intent(in)::this
integer(4),intent(in)::iteration
integer(4),intent(in)::verbosity
real(8),intent(in)::errors(:)
real(8),intent(in),optional::value
real(8),intent(in),optional::eigenvalues(:)
logical(4)::report
end
end
