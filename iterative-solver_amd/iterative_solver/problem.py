"""Problem: what a user of the iterative solvers supplies (mirror of the reference's Python API,
python/iterative_solver/problem.py; the same method names, arguments and defaults)."""
import sys

import numpy as np


class Problem:
    """Base class for the problem to be solved.  Linear solvers call action(); non-linear ones call
    residual(); diagonals() enables the default preconditioner and the P-space selection."""

    def __init__(self):
        self.dimension = None

    def residual(self, parameters, residual):
        """Fill `residual` for trial `parameters`; return the objective value (Optimize) or 0."""
        raise NotImplementedError

    def action(self, parameters, action):
        """Fill `action` (rows) with the kernel applied to `parameters` (rows)."""
        raise NotImplementedError

    def diagonals(self, diagonals):
        """Optionally fill `diagonals` with the kernel's diagonal and return True."""
        return False

    def precondition(self, residual, shift=None, diagonals=None):
        """Turn residual rows into update steps in place.  Default: divide by the diagonals plus
        the shift plus 1e-14, row by row (reference problem.py:55-82 uses exactly this form)."""
        small = 1e-14
        if residual.ndim > 1:
            for i in range(residual.shape[0]):
                self.precondition(residual[i, :], float(shift[i]) if shift is not None else None, diagonals)
            return
        if diagonals is None:
            raise NotImplementedError
        denom = diagonals + (shift if shift is not None else 0.0) + small
        residual[:] = residual / denom

    def pp_action_matrix(self, pparams):
        return np.array([], dtype=np.double)

    def p_action(self, p_coefficients, pparams, actions):
        raise NotImplementedError("P-space unavailable: p_action() not implemented by this Problem")

    def test_parameters(self, instance, parameters):
        return False

    def report(self, iteration, verbosity, errors, value=None, eigenvalues=None):
        if not ((iteration <= 0 and verbosity >= 1) or verbosity >= 2):
            return False
        err = np.log10(np.asarray(errors) + sys.float_info.min)
        if iteration > 0 and verbosity >= 2:
            print("Iteration", iteration, "log10(|residual|)=", err)
        else:
            print("Converged" if iteration == 0 else "Unconverged", "log10(|residual|)=", err)
        if value is not None:
            print("Objective function value", value)
        if eigenvalues is not None:
            print("Eigenvalues", eigenvalues)
        return True
