"""Reverse-communication loops of the reference's solver tests, written once and driven through
either back end: oracle.RcSolver (the reference CPU path) or the iterative_solver package (the
C API on the HIP handlers).  Each driver returns a trace (per-iteration return values and
parameters) so the two paths can be compared step by step.

Problems and loops follow the reference's tests:
  quadratic form     test_Optimize.cpp:20-112 / test_NonLinearEquations.cpp:20-110
                     (h = 1 + diag((i + 2) param), minimum / root at x = 1, start x = e_0)
  Rosenbrock         test_Optimize.cpp:124-156
  trig1d             test_Optimize.cpp:158-176, test_NonLinearEquations.cpp:252-270
  trig (n = 1, 2)    test_NonLinearEquations.cpp:160-250 (calc, trigProblem)
  test_eigen         test_LinearEigensystem.cpp:60-330 (file, n, small, symmetry and
                     non-hermitian matrices; P space through add_p; preconditioner
                     g *= -1 / (1e-12 - shift + h_ii))
  RSPT               test_RSPT.cpp:31-190: <file>.hamiltonian with H0 = diag(<file>.h0);
                     Rayleigh-Schroedinger perturbation series (file_eigen) and the
                     second-order energy as the Hylleraas minimum by BFGS / DIIS (file_Hylleraas)
"""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def quadratic_matrix(n, param):
    h = np.ones((n, n))
    h[np.diag_indices(n)] = (np.arange(n) + 2) * param
    return h


def quadratic_action(h, x, g):
    """f = 0.5 (x - 1).h.(x - 1), g = h (x - 1) (test_Optimize.cpp:32-46)."""
    d = x - 1.0
    g[:] = h @ d
    return 0.5 * d @ (h @ d)


def loop_quadratic(solver, h, optimize, max_iter=1000):
    """test_Optimize.cpp:60-88 (optimize) / test_NonLinearEquations.cpp:62-86 (DIIS)."""
    n = h.shape[0]
    x, g = np.zeros(n), np.zeros(n)
    x[0] = 1.0
    trace, nwork, n_iter = [], 1, 1
    for _ in range(1, max_iter):
        if nwork <= 0:
            break
        value = quadratic_action(h, x, g)
        precon = solver.add_value(value, x, g) if optimize else solver.add_vector(x, g)
        if precon > 0:
            g /= np.diag(h)
        nwork = solver.end_iteration(x, g)
        trace.append((precon, nwork, x.copy()))
        n_iter += 1
    return trace, n_iter


def rosenbrock(x, a=1.0, b=100.0):
    """test_Optimize.cpp:124-133"""
    f, f1 = 0.0, np.zeros_like(x)
    for i in range(x.size - 1):
        f += (a - x[i]) ** 2 + b * (x[i] ** 2 - x[i + 1]) ** 2
        f1[i] -= 2 * (a - x[i])
        f1[i] += 4 * b * x[i] * (x[i] ** 2 - x[i + 1])
        f1[i + 1] -= 2 * b * (x[i] ** 2 - x[i + 1])
    return f, f1


def loop_rosenbrock(solver, n, max_iter=10000):
    """test_Optimize.cpp:135-156: x = (-3, -4, ..., -4), preconditioner g / 2."""
    x = np.full(n, -4.0)
    x[0] = -3.0
    g = np.zeros(n)
    trace = []
    for _ in range(max_iter):
        value, g[:] = rosenbrock(x)
        precon = solver.add_value(value, x, g) > 0
        if precon:
            g /= 2
        nwork = solver.end_iteration(x, g)
        trace.append((int(precon), nwork, x.copy()))
        if nwork == 0:
            break
    return trace, x


def loop_trig1d(solver, optimize, max_iter=100):
    """test_Optimize.cpp:158-176 / test_NonLinearEquations.cpp:252-270: f = sin x, g = cos x, x = 1."""
    x, g = np.ones(1), np.zeros(1)
    trace = []
    for _ in range(max_iter):
        value = np.sin(x[0])
        g[0] = np.cos(x[0])
        precon = solver.add_value(value, x, g) if optimize else solver.add_vector(x, g)
        nwork = solver.end_iteration(x, g)
        trace.append((precon, nwork, x.copy()))
        if nwork == 0:
            break
    return trace, x


def trig_calc(x, g):
    """test_NonLinearEquations.cpp:160-173"""
    n = x.size
    value = 0.0
    couple = 1e-2
    for i in range(n):
        value += np.sin((i + 1) * x[i]) ** 2
        g[i] = 2 * (i + 1) * np.sin((i + 1) * x[i]) * np.cos((i + 1) * x[i])
        for j in range(n):
            value += couple * x[i] * x[j]
            g[i] += 2 * couple * x[j]
    return value


def loop_trig(solver, n, max_iter=100):
    """test_NonLinearEquations.cpp:215-250 through IterativeSolverTemplate::solve's loop for a
    non-linear problem (IterativeSolverTemplate.h:371-405): residual, add_vector, precondition when
    asked, end_iteration.  The reference trigProblem's precondition divides a COPY of each residual
    (`auto g = gr.get()`, :186), so it leaves the residual unchanged; so does this loop."""
    x, g = np.full(n, 0.05), np.zeros(n)
    trace = []
    for _ in range(max_iter):
        trig_calc(x, g)
        nwork = solver.add_vector(x, g)
        nwork = solver.end_iteration(x, g)
        trace.append((nwork, x.copy()))
        if nwork == 0:
            break
    return trace, x


# ---- LinearEigensystem: test_LinearEigensystem.cpp:60-330 ---------------------------------------
def eigen_matrix(n, param=1.0, non_hermiticity=0.0):
    """load_matrix(n, "", param, non_hermiticity) (test_LinearEigensystem.cpp:41-51)."""
    h = np.ones((n, n))
    h[np.diag_indices(n)] = np.arange(n) * param
    if non_hermiticity:
        h[np.tril_indices(n, -1)] *= 1 - non_hermiticity
    return h


def symmetry_matrix(n, param=1.0):
    """symmetry_eigen (test_LinearEigensystem.cpp:387-406): couplings between i % 3 == 0 and the rest removed."""
    h = eigen_matrix(n, param)
    for i in range(n):
        for j in range(n):
            if (i % 3 == 0 and j % 3 != 0) or (j % 3 == 0 and i % 3 != 0):
                h[j, i] = 0.0
    return h


def eigen_options(n, nroot, np_, hermitian):
    """set_options (test_LinearEigensystem.cpp:192-215)."""
    qmax = max(6 * nroot, min(n, min(1000, 6 * nroot)) - np_)
    return (f"convergence_threshold=1e-8,max_size_qspace={qmax},reset_D=8,"
            f"hermiticity={'true' if hermitian else 'false'}")


def _lowest_diagonals(h, count):
    d = list(np.diag(h).copy())
    out = []
    for _ in range(count):
        k = int(np.argmin(d))  # first minimum, as std::min_element
        out.append(k)
        d[k] = 1e99
    return out


def eigen_update(h, g, shift):
    """update(): g_k *= -1 / (1e-12 - shift_k + h_ii) (test_LinearEigensystem.cpp:91-102)."""
    d = np.diag(h)
    for k in range(min(g.shape[0], len(shift))):
        g[k] *= -1.0 / (1e-12 - shift[k] + d)


def loop_eigen(solver, h, nroot, np_, max_iter=100):
    """initialize_subspace + the test_eigen loop (test_LinearEigensystem.cpp:217-283).  Returns the
    trace of add_vector / end_iteration returns and the iteration count n_iter."""
    n = h.shape[0]
    x, g = np.zeros((nroot, n)), np.zeros((nroot, n))
    trace = []
    if np_:
        pidx = _lowest_diagonals(h, np_)
        pspace = [{k: 1.0} for k in pidx]
        pp = h[np.ix_(pidx, pidx)].copy()

        def apply_p(pc, gl, ranges):
            # adds to this rank's range [r0, r1) of each action row, rows n apart (the reference's
            # apply_on_p_c contract, IterativeSolverCMPI.cpp:141-157; one rank: the whole row)
            for i in range(pc.shape[0]):
                r0, r1 = int(ranges[i, 0]), int(ranges[i, 1])
                for pi, k in enumerate(pidx):
                    gl[i * n:i * n + r1 - r0] += h[r0:r1, k] * pc[i, pi]

        nwork = solver.add_p(pspace, pp, x, g, apply_p)
        trace.append(("p", nwork))
    else:
        for root, k in enumerate(_lowest_diagonals(h, nroot)):
            x[root, k] = 1.0
        g[:] = x @ h.T
        nwork = solver.add_vector(x, g)
        trace.append(("v", nwork))
    eigen_update(h, g, solver.working_set_eigenvalues(nwork))
    trace.append(("e", solver.end_iteration(x, g)))
    n_iter = 2
    for _ in range(1, max_iter):
        g[:] = x @ h.T
        nwork = solver.add_vector(x, g)
        trace.append(("v", nwork))
        if nwork == 0:
            break
        eigen_update(h, g, solver.working_set_eigenvalues(nwork))
        nwork = solver.end_iteration(x, g)
        trace.append(("e", nwork))
        n_iter += 1
        if nwork == 0:
            break
    return trace, n_iter


def expected_eigen(h, hermitian):
    if hermitian:
        w, v = np.linalg.eigh(h)
    else:
        w, v = np.linalg.eig(h)
        o = np.argsort(w.real, kind="stable")
        w, v = w[o].real, v[:, o].real
        v /= np.linalg.norm(v, axis=0)
    return w, v


def eigen_cases(n, hermitian=True):
    """(nroot, np) pairs of test_eigen (test_LinearEigensystem.cpp:226-229)."""
    for nroot in range(1, min(n, 28) + 1, max(1, n // 10)):
        for np_ in range(0, min(n, 100) + 1, max(nroot, n // 5)):
            if hermitian or np_ == 0:
                yield nroot, np_


# ---- RSPT (test_RSPT.cpp) ------------------------------------------------------------------------
def rspt_problem(name, degeneracy_split=1e-8):
    """test_RSPT.cpp:31-50: H read row by row, diagonal split by degeneracy_split * i, H0 diagonal."""
    t = open(os.path.join(GOLDEN, name + ".hamiltonian")).read().split()
    n = int(t[0])
    h = np.array(t[1:1 + n * n], dtype=float).reshape(n, n) + np.diag(degeneracy_split * np.arange(n))
    h0 = np.array(open(os.path.join(GOLDEN, name + ".h0")).read().split()[:n], dtype=float)
    return h, h0


def rspt_update(h0, g):
    """test_RSPT.cpp:58-66: g /= (1e-12 - e0 + h0), e0 = min h0."""
    g /= 1e-12 - h0.min() + h0


def rspt_initial_guess(h0):
    x = np.zeros(h0.size)
    x[int(np.argmin(h0))] = 1.0  # test_RSPT.cpp:68-74
    return x


def loop_rspt(solver, h, h0, niter=9):
    """test_RSPT.cpp:99-125 (file_eigen): x = psi(k), g = H x; add_vector, update, end_iteration."""
    x, g = rspt_initial_guess(h0), np.zeros(h0.size)
    trace = []
    for _ in range(niter):
        g[:] = h @ x
        nwork = solver.add_vector(x, g)
        rspt_update(h0, g)
        nend = solver.end_iteration(x, g)
        trace.append((nwork, nend, x.copy()))
    return trace


def rspt_second_order_energy(h, h0):
    """Closed form (independent of the solvers): E2 = -sum_{i != 0} H1_{i0}^2 / (h0_i - e0 + 1e-12) with
    psi(0) = e_0 the minimum of h0 and H1 = H - diag(h0)."""
    i0 = int(np.argmin(h0))
    col = h[:, i0].copy()
    col[i0] = 0.0
    return -np.sum(col * col / (1e-12 - h0[i0] + h0))


def loop_hylleraas(solver, h, h0, optimize, precondition=True, max_iter=20):
    """test_RSPT.cpp:134-188: minimise the Hylleraas functional
    e2(x) = 2 x0.(H1 x - e1 x) + x.(H0 x - e0 x) (BFGS: add_value(e2 / 2), DIIS: add_vector) from
    x = 0 with gradient r = H1 x0 - e1 x0 + H0 x - e0 x; returns the last e2 and the trace."""
    n = h0.size
    ham0 = np.diag(h0)
    ham1 = h - ham0
    x0 = rspt_initial_guess(h0)
    e0 = h0 @ x0
    e1 = x0 @ (ham1 @ x0)
    x, g = np.zeros(n), np.zeros(n)
    trace, e2 = [], None
    for _ in range(1, max_iter):
        e2 = 2 * (x0 @ (ham1 @ x - e1 * x)) + x @ (ham0 @ x - e0 * x)
        g[:] = ham1 @ x0 - e1 * x0 + ham0 @ x - e0 * x
        nwork = solver.add_value(e2 / 2, x, g) if optimize else solver.add_vector(x, g)
        if precondition:
            rspt_update(h0, g)
        nwork = solver.end_iteration(x, g)
        trace.append((nwork, x.copy()))
        if nwork < 1:
            break
    return e2, trace
