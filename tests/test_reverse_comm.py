"""Reverse-communication solver loops of the reference's tests (test_Optimize.cpp,
test_NonLinearEquations.cpp) on problems defined in Python (tests/rc_problems.py).

CPU: the reference CPU path (oracle.RcSolver: the restated solvers over the CPU handlers, called
     as the C API calls them) must satisfy the reference tests' own assertions.
GPU: the same loops through the C API on the HIP handlers (iterative_solver package) take the
     same steps as the CPU path -- identical per-iteration return values and iteration counts,
     parameters within 1e-10 (1e-6 mid-trajectory on Rosenbrock) -- and satisfy the same
     assertions.  At these sizes the HIP path computes in the reference's arithmetic by default
     (ssp_ctx_set_exact_max), and the *_bit_for_bit tests hold every loop to the CPU path exactly.
"""
import numpy as np
import pytest

import oracle
import rc_problems as rp

THRESH = 1e-8
OPTS6 = "convergence_threshold=1e-8,max_size_qspace=6"


def cpu(kind, n, algorithm="", options=OPTS6):
    return oracle.RcSolver(kind, n, thresh=THRESH, algorithm=algorithm, options=options)


def gpu(kind, n, algorithm="", options=OPTS6):
    import iterative_solver

    if kind == "Optimize":
        return iterative_solver.Optimize(n, thresh=THRESH, algorithm=algorithm, options=options)
    return iterative_solver.NonLinearEquations(n, thresh=THRESH, options=options)


def check_quadratic(s, trace, n_iter, n, stats):
    # test_Optimize.cpp:89-110 / test_NonLinearEquations.cpp:87-108
    assert np.all(np.abs(stats["errors"]) <= 2 * THRESH)
    assert stats["r_creations"] <= 2 * n_iter
    x, g = np.zeros(n), np.zeros(n)
    s.solution([0], x, g)
    assert np.linalg.norm(g) <= THRESH
    np.testing.assert_allclose(x, 1.0, rtol=0, atol=THRESH)


def gpu_stats(s):
    import iterative_solver

    st = iterative_solver.statistics()
    return {"iterations": st["iterations"], "r_creations": st["r_creations"], "errors": s.errors, "value": s.value}


def same_trace(a, b, xtol=1e-10):
    assert len(a) == len(b), (len(a), len(b))
    for sa, sb in zip(a, b):
        assert sa[:-1] == sb[:-1]
        np.testing.assert_allclose(sa[-1], sb[-1], rtol=xtol, atol=xtol)


# ---- CPU: the reference path reproduces the reference tests' assertions ----------------------
@pytest.mark.parametrize("n", [2, 11, 20, 29])
@pytest.mark.parametrize("alg", ["BFGS", "SD"])
def test_optimize_quadratic_form_cpu(n, alg):
    h = rp.quadratic_matrix(n, 10.0)
    s = cpu("Optimize", n, alg)
    trace, n_iter = rp.loop_quadratic(s, h, optimize=True)
    st = s.stats()
    assert abs(st["value"]) <= 2e-9  # test_Optimize.cpp:91
    check_quadratic(s, trace, n_iter, n, st)


@pytest.mark.parametrize("n", [2, 7, 20, 50])
def test_diis_quadratic_form_cpu(n):
    h = rp.quadratic_matrix(n, 10.0)
    s = cpu("NonLinearEquations", n)
    trace, n_iter = rp.loop_quadratic(s, h, optimize=False)
    check_quadratic(s, trace, n_iter, n, s.stats())


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6])
def test_optimize_rosenbrock_cpu(n):
    s = cpu("Optimize", n, "BFGS")
    trace, x = rp.loop_rosenbrock(s, n)
    assert trace[-1][1] == 0
    np.testing.assert_allclose(x, 1.0, rtol=0, atol=THRESH)  # test_Optimize.cpp:153-154


@pytest.mark.parametrize("optimize", [True, False])
def test_trig1d_cpu(optimize):
    # test_Optimize.cpp:158-176 / test_NonLinearEquations.cpp:252-270 (no assertion there: the loop runs)
    s = cpu("Optimize" if optimize else "NonLinearEquations", 1, "BFGS" if optimize else "",
            "convergence_threshold=1e-8,max_size_qspace=2")
    trace, x = rp.loop_trig1d(s, optimize)
    assert trace and np.isfinite(x).all()


@pytest.mark.parametrize("n", [1, 2])
def test_diis_trig_cpu(n):
    s = cpu("NonLinearEquations", n, options="convergence_threshold=1e-8,max_size_qspace=5")
    trace, x = rp.loop_trig(s, n)
    xs, gs = np.zeros(n), np.zeros(n)
    s.solution([0], xs, gs)
    np.testing.assert_allclose(xs, 0.0, rtol=0, atol=THRESH)  # test_NonLinearEquations.cpp:246-247


# ---- GPU: the C API on the HIP handlers takes the reference path's steps -----------------------
@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 11, 20, 29])
@pytest.mark.parametrize("alg", ["BFGS", "SD"])
def test_optimize_quadratic_form_gpu(n, alg):
    h = rp.quadratic_matrix(n, 10.0)
    ref = rp.loop_quadratic(cpu("Optimize", n, alg), h, optimize=True)
    g = gpu("Optimize", n, alg)
    trace, n_iter = rp.loop_quadratic(g, h, optimize=True)
    same_trace(trace, ref[0])
    check_quadratic(g, trace, n_iter, n, gpu_stats(g))
    g.finalize()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 7, 20, 50])
def test_diis_quadratic_form_gpu(n):
    h = rp.quadratic_matrix(n, 10.0)
    ref = rp.loop_quadratic(cpu("NonLinearEquations", n), h, optimize=False)
    g = gpu("NonLinearEquations", n)
    trace, n_iter = rp.loop_quadratic(g, h, optimize=False)
    same_trace(trace, ref[0])
    check_quadratic(g, trace, n_iter, n, gpu_stats(g))
    g.finalize()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 3, 4, 5, 6])
def test_optimize_rosenbrock_gpu(n):
    ref, xr = rp.loop_rosenbrock(cpu("Optimize", n, "BFGS"), n)
    g = gpu("Optimize", n, "BFGS")
    trace, x = rp.loop_rosenbrock(g, n)
    np.testing.assert_allclose(x, 1.0, rtol=0, atol=THRESH)
    # identical step sequence; mid-trajectory parameters agree to 1e-6: the GPU dots differ from the
    # sequential CPU sums in the last bits and Rosenbrock's valley (Hessian condition ~1e3) amplifies
    # them until the end, where both reach x = 1 within the threshold
    same_trace(trace, ref, xtol=1e-6)
    g.finalize()


@pytest.mark.gpu
@pytest.mark.parametrize("optimize", [True, False])
def test_trig1d_gpu(optimize):
    opts = "convergence_threshold=1e-8,max_size_qspace=2"
    kind, alg = ("Optimize", "BFGS") if optimize else ("NonLinearEquations", "")
    ref, _ = rp.loop_trig1d(cpu(kind, 1, alg, opts), optimize)
    g = gpu(kind, 1, alg, opts)
    trace, _ = rp.loop_trig1d(g, optimize)
    same_trace(trace, ref)
    g.finalize()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2])
def test_diis_trig_gpu(n):
    opts = "convergence_threshold=1e-8,max_size_qspace=5"
    ref, _ = rp.loop_trig(cpu("NonLinearEquations", n, options=opts), n)
    g = gpu("NonLinearEquations", n, options=opts)
    trace, _ = rp.loop_trig(g, n)
    same_trace(trace, ref)
    xs, gs = np.zeros(n), np.zeros(n)
    g.solution([0], xs, gs)
    np.testing.assert_allclose(xs, 0.0, rtol=0, atol=THRESH)
    g.finalize()


# ---- LinearEigensystem: test_LinearEigensystem.cpp test_eigen on every matrix family -----------
BIG = 1.7976931348623157e308


def _hamiltonian(name, split):
    import os

    t = open(os.path.join(os.path.dirname(__file__), "golden", name + ".hamiltonian")).read().split()
    n = int(t[0])
    return np.array(t[1:1 + n * n], dtype=float).reshape(n, n) + np.diag(split * np.arange(n))


# file_eigen uses phenol, bh, hf (:347-352); phenol.hamiltonian is not in the reference tree.
EIGEN_FAMILIES = {
    "file_bh": lambda: [_hamiltonian("bh", 1e-8)],
    "file_hf": lambda: [_hamiltonian("hf", 1e-8)],
    "n_eigen_100": lambda: [rp.eigen_matrix(100, 1.0)],
    "nonhermitian_6": lambda: [rp.eigen_matrix(6, p, nh) for p in (1.0, 0.1) for nh in (0.0, 0.1, 0.2)],
    "small_1_4": lambda: [rp.eigen_matrix(n, 1.0) for n in range(1, 5)],
    "symmetry_1_5": lambda: [rp.symmetry_matrix(n, 1.0) for n in range(1, 6)],
}


def run_eigen(make, h, nroot, np_):
    n = h.shape[0]
    hermitian = bool(np.linalg.norm(h - h.T) < 1e-10)
    s = make(n, nroot, hermitian, rp.eigen_options(n, nroot, np_, hermitian))
    trace, n_iter = rp.loop_eigen(s, h, nroot, np_)
    return s, trace, n_iter, hermitian


def check_eigen(s, h, nroot, n_iter, hermitian, errors, eigenvalues, r_creations, tag):
    # test_LinearEigensystem.cpp:296-329
    n = h.shape[0]
    w, v = rp.expected_eigen(h, hermitian)
    assert np.all(np.abs(errors) <= 2e-8), (tag, errors)
    np.testing.assert_allclose(eigenvalues, w[:nroot], rtol=0, atol=2e-9, err_msg=tag)
    assert r_creations <= (nroot + 1) * n_iter, tag
    x, g = np.zeros((nroot, n)), np.zeros((nroot, n))
    s.solution(list(range(nroot)), x, g)
    r = x @ h.T - eigenvalues[:, None] * x
    assert np.all(np.linalg.norm(r, axis=1) <= 1e-8), tag
    for k in range(nroot):
        gap = np.min(np.abs(np.delete(w, k) - w[k])) if n > 1 else 1.0
        if gap > 1e-6:  # the reference's map of eigenvectors keyed by eigenvalue assumes no degeneracy
            assert abs(abs(x[k] @ v[:, k]) - 1) <= 1e-8, tag


def cpu_eigen(n, nroot, hermitian, options):
    return oracle.RcSolver("LinearEigensystem", n, nroot=nroot, thresh=THRESH, thresh_value=BIG,
                           hermitian=hermitian, options=options)


def gpu_eigen(n, nroot, hermitian, options):
    import iterative_solver

    return iterative_solver.LinearEigensystem(n, nroot, thresh=THRESH, thresh_value=BIG, hermitian=hermitian,
                                              options=options)


@pytest.mark.parametrize("family", list(EIGEN_FAMILIES))
def test_eigen_cpu(family):
    for h in EIGEN_FAMILIES[family]():
        hermitian = bool(np.linalg.norm(h - h.T) < 1e-10)
        for nroot, np_ in rp.eigen_cases(h.shape[0], hermitian):
            s, trace, n_iter, herm = run_eigen(cpu_eigen, h, nroot, np_)
            st = s.stats()
            check_eigen(s, h, nroot, n_iter, herm, st["errors"], st["eigenvalues"], st["r_creations"],
                        f"{family} n={h.shape[0]} nroot={nroot} np={np_}")


def rounding_sensitive(h, nroot, np_, trace):
    """True when the reference CPU path itself takes different steps after a relative perturbation
    of 2^-50 in H: then the step sequence is decided by rounding (for example the redundancy screen's
    choice inside a null space of several singular values ~1e-16, propose_rspace.h:481-512) and only
    the converged results are compared."""
    s2, t2, _, _ = run_eigen(cpu_eigen, h * (1 + 2.0 ** -50), nroot, np_)
    return t2 != trace


# n_eigen (n = 100, H = 1 + diag(i)): the reference CPU path changes its step sequence in 8 of the 17
# cases when H is scaled by 1 + 2^-50 (the redundancy screen picks residuals inside null spaces of
# several singular values ~1e-16), so only the converged results are compared there.
ROUNDING_CHAOTIC = {"n_eigen_100"}


@pytest.mark.gpu
@pytest.mark.parametrize("family", list(EIGEN_FAMILIES))
def test_eigen_gpu(family):
    import iterative_solver

    sensitive = []

    for h in EIGEN_FAMILIES[family]():
        hermitian = bool(np.linalg.norm(h - h.T) < 1e-10)
        for nroot, np_ in rp.eigen_cases(h.shape[0], hermitian):
            tag = f"{family} n={h.shape[0]} nroot={nroot} np={np_}"
            c, ctrace, c_iter, _ = run_eigen(cpu_eigen, h, nroot, np_)
            cst = c.stats()
            g, gtrace, g_iter, herm = run_eigen(gpu_eigen, h, nroot, np_)
            st = iterative_solver.statistics()
            if family in ROUNDING_CHAOTIC or rounding_sensitive(h, nroot, np_, ctrace):
                sensitive.append(tag)
            else:
                assert gtrace == ctrace, tag  # same add_p / add_vector / end_iteration returns, call for call
                assert st["iterations"] == cst["iterations"], tag
            np.testing.assert_allclose(g.eigenvalues, cst["eigenvalues"], rtol=0, atol=1e-10, err_msg=tag)
            check_eigen(g, h, nroot, g_iter, herm, g.errors, g.eigenvalues, st["r_creations"], tag)
            g.finalize()
    if family not in ROUNDING_CHAOTIC:
        # Outside n_eigen the exact-trace bar applies to all but the cases whose steps the reference
        # CPU path itself changes under a 2^-50 perturbation of H -- with the restated dsyev-type
        # eigensolver (dense.h sym_eigen, tridiagonal QL) that is bh at nroot = 23 of n = 28 (82 % of
        # the full space, the overlap's smallest eigenvalues at the rank threshold), with and without
        # P space -- and those must stay the exception.
        assert len(sensitive) <= 2, sensitive
        print(family, "rounding-sensitive in the CPU path itself:", sensitive)


def _solution_case(make, h, nroot, np_):
    """test_LinearEigensystem.cpp:408-433: after initialize_subspace, solution(working set) gives the
    residuals the solver handed back."""
    n = h.shape[0]
    s = make(n, nroot, True, rp.eigen_options(n, nroot, np_, True))
    x, g = np.zeros((nroot, n)), np.zeros((nroot, n))
    if np_:
        pidx = rp._lowest_diagonals(h, np_)
        pp = h[np.ix_(pidx, pidx)].copy()

        def apply_p(pc, gl, ranges):
            for i in range(pc.shape[0]):
                for pi, k in enumerate(pidx):
                    gl[i * n:(i + 1) * n] += h[:, k] * pc[i, pi]

        nwork = s.add_p([{k: 1.0} for k in pidx], pp, x, g, apply_p)
    else:
        for root, k in enumerate(rp._lowest_diagonals(h, nroot)):
            x[root, k] = 1.0
        g[:] = x @ h.T
        nwork = s.add_vector(x, g)
    ev = s.working_set_eigenvalues(nwork)
    rp.eigen_update(h, g, ev)
    s.end_iteration(x, g)
    return s, nwork, ev


@pytest.mark.parametrize("backend", ["cpu", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_eigen_solution_matches_residual(backend):
    h = rp.eigen_matrix(10, 1.0)
    make = cpu_eigen if backend == "cpu" else gpu_eigen
    for nroot in range(1, 10):
        for np_ in (0, nroot):
            s, nwork, _ = _solution_case(make, h, nroot, np_)
            roots = list(range(nroot))
            x, g = np.zeros((nroot, 10)), np.zeros((nroot, 10))
            s.solution(roots, x, g)
            ev = (s.stats()["eigenvalues"] if backend == "cpu" else s.eigenvalues)[:nroot]
            r = x @ h.T - ev[:, None] * x
            # the solver's residual for each root is H x - e x (reference: |g - residual| <= 1e-6)
            np.testing.assert_allclose(g, r, rtol=0, atol=1e-6, err_msg=f"nroot={nroot} np={np_}")
            if backend == "gpu":
                s.finalize()


# ---- RSPT and the Hylleraas functional (test_RSPT.cpp) -------------------------------------------
RSPT_FILES = ["he", "bh", "hf"]


def rspt_cpu(n):
    return oracle.RcSolver("LinearEigensystem", n, thresh=THRESH, algorithm="RSPT", options="")


def rspt_gpu(n):
    import iterative_solver

    return iterative_solver.LinearEigensystem(n, 1, thresh=THRESH, hermitian=True, algorithm="RSPT")


def hylleraas_solver(factory, n, method):
    if factory is cpu:
        return cpu("Optimize", n, "BFGS", options="") if method == "BFGS" else cpu("NonLinearEquations", n, options="")
    return gpu("Optimize", n, "BFGS", options="") if method == "BFGS" else gpu("NonLinearEquations", n, options="")


def check_rspt_trace(trace, h, h0):
    # x after the first end_iteration is psi(1): its energy <psi(0)|H|psi(1)> is E(2) (the Hylleraas
    # minimum), and psi(1) is orthogonal to psi(0).
    x0 = rp.rspt_initial_guess(h0)
    psi1 = trace[0][-1]
    assert abs(x0 @ psi1) <= 1e-14 * np.linalg.norm(psi1)
    e2 = x0 @ (h @ psi1)
    assert abs(e2 - rp.rspt_second_order_energy(h, h0)) <= 1e-12 * max(1.0, abs(e2))
    # The series E(0) + E(1) + ... (E(k+1) = <psi(0)|H|psi(k)>) approaches the lowest eigenvalue;
    # for He (the reference's FCI energy -2.878990189612, examples/he.molpro/run/5.molpro/5.out:408)
    # nine orders are within 1e-7.
    series = np.cumsum([x0 @ (h @ x0)] + [x0 @ (h @ t[-1]) for t in trace[:-1]])
    exact = np.linalg.eigvalsh(h)[0]
    assert abs(series[-1] - exact) < abs(series[1] - exact)
    if h0.size == 4:
        assert abs(series[-1] - exact) < 1e-7 and abs(series[-1] - (-2.878990189612)) < 1e-7
    return e2


def rspt_recurrence(h, h0, norders=9, shift=1e-12):
    """Textbook Rayleigh-Schroedinger recurrence in numpy, independent of solvers.h: H = H0 + V with
    H0 = diag(h0), psi(0) = e_i0 (min h0), intermediate normalisation, E(j) = <psi(0)|V|psi(j-1)>,
    (H0 - E0 + shift) psi(n) = -[(V - E1) psi(n-1) - sum_{j=2..n} E(j) psi(n-j)] off i0 (the shift is
    the reference test's preconditioner, test_RSPT.cpp:58-66). Returns [E(0), E(1), ...] and psi."""
    i0 = int(np.argmin(h0))
    v = h - np.diag(h0)
    psi = [np.zeros(h0.size)]
    psi[0][i0] = 1.0
    e = [h0[i0], v[i0, i0]]
    den = shift - h0[i0] + h0
    for n in range(1, norders):
        rhs = v @ psi[n - 1] - e[1] * psi[n - 1] - sum(e[j] * psi[n - j] for j in range(2, n + 1))
        rhs[i0] = 0.0
        psi.append(-rhs / den)
        e.append(psi[0] @ (v @ psi[n]))
    return np.array(e), psi


@pytest.mark.parametrize("name", RSPT_FILES)
def test_rspt_orders_match_textbook_recurrence(name):
    # Pins LinearEigensystemRSPT (LinearEigensystemRSPT.h:63-73 end_iteration, :165-185
    # construct_residual) independently of the restated solver headers: the product CPU path's
    # psi(k) and <psi(0)|H psi(k)> are the textbook recurrence's (measured: energies to 2e-14,
    # vectors to 4e-11 relative over eight orders).
    h, h0 = rp.rspt_problem(name)
    trace = rp.loop_rspt(rspt_cpu(h0.size), h, h0)
    e, psi = rspt_recurrence(h, h0)
    x0 = rp.rspt_initial_guess(h0)
    got = np.array([x0 @ (h @ x0)] + [x0 @ (h @ t[-1]) for t in trace[:-1]])
    want = np.array([e[0] + e[1]] + list(e[2:len(got) + 1]))  # <psi0|H psi(k)> = E(k+1), k >= 1
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-13)
    for k, t in enumerate(trace[:-1], start=1):
        assert np.max(np.abs(t[-1] - psi[k])) <= 1e-9 * np.max(np.abs(psi[k]))


@pytest.mark.parametrize("name", RSPT_FILES)
def test_rspt_file_eigen_cpu(name):
    # test_RSPT.cpp:191-196 (file_eigen): nine orders of the perturbation series on the product's
    # CPU path (restated solvers over the CPU handlers); the orders themselves are pinned by
    # test_rspt_orders_match_textbook_recurrence
    h, h0 = rp.rspt_problem(name)
    trace = rp.loop_rspt(rspt_cpu(h0.size), h, h0)
    assert len(trace) == 9
    check_rspt_trace(trace, h, h0)


@pytest.mark.parametrize("name", RSPT_FILES)
def test_rspt_file_hylleraas_cpu(name):
    # test_RSPT.cpp:198-206 (file_Hylleraas_BFGS): the preconditioned BFGS minimum is the expected
    # E(2); unpreconditioned BFGS and preconditioned DIIS reach it within 1e-11; it is the closed-form
    # second-order energy and the RSPT series' E(2).
    h, h0 = rp.rspt_problem(name)
    n = h0.size
    expected, _ = rp.loop_hylleraas(hylleraas_solver(cpu, n, "BFGS"), h, h0, optimize=True)
    e_bfgs, _ = rp.loop_hylleraas(hylleraas_solver(cpu, n, "BFGS"), h, h0, optimize=True, precondition=False)
    e_diis, _ = rp.loop_hylleraas(hylleraas_solver(cpu, n, "DIIS"), h, h0, optimize=False)
    assert abs(e_bfgs - expected) <= 1e-11
    assert abs(e_diis - expected) <= 1e-11
    assert abs(expected - rp.rspt_second_order_energy(h, h0)) <= 1e-10


@pytest.mark.gpu
@pytest.mark.parametrize("name", RSPT_FILES)
def test_rspt_file_eigen_gpu(name):
    # product CPU path vs the GPU path, order for order (the CPU path is pinned to the textbook
    # recurrence above)
    h, h0 = rp.rspt_problem(name)
    ref = rp.loop_rspt(rspt_cpu(h0.size), h, h0)
    g = rspt_gpu(h0.size)
    trace = rp.loop_rspt(g, h, h0)
    # higher orders grow (|psi(k)| ~ ratio^k): relative agreement per order
    assert [t[:-1] for t in trace] == [t[:-1] for t in ref]
    for a, b in zip(trace, ref):
        np.testing.assert_allclose(a[-1], b[-1], rtol=1e-9, atol=1e-10 * np.max(np.abs(b[-1])))
    check_rspt_trace(trace, h, h0)
    g.finalize()


@pytest.mark.gpu
@pytest.mark.parametrize("name", RSPT_FILES)
@pytest.mark.parametrize("method,precondition", [("BFGS", True), ("BFGS", False), ("DIIS", True)])
def test_rspt_file_hylleraas_gpu(name, method, precondition):
    h, h0 = rp.rspt_problem(name)
    n = h0.size
    opt = method == "BFGS"
    e_ref, ref = rp.loop_hylleraas(hylleraas_solver(cpu, n, method), h, h0, optimize=opt, precondition=precondition)
    s = hylleraas_solver(gpu, n, method)
    e_gpu, trace = rp.loop_hylleraas(s, h, h0, optimize=opt, precondition=precondition)
    if precondition:
        assert [t[0] for t in trace] == [t[0] for t in ref]
    else:
        # Unpreconditioned BFGS on hf reaches a knife-edge line-search decision: measured on MI355X
        # (tools/rspt_diverge.py), x agrees to 1e-17 for three steps, then one branch flips on a
        # last-bit difference of the GPU's reductions and the paths take different (both
        # convergent) trajectories, 15 vs 13 steps, e2 equal to 5e-17; he and bh agree step for
        # step.  The reference's own assertion for this case (test_RSPT.cpp:198-206: e2 within
        # 1e-11 of the preconditioned minimum) is the bar, on both paths.
        e_min, _ = rp.loop_hylleraas(hylleraas_solver(cpu, n, "BFGS"), h, h0, optimize=True)
        assert abs(e_gpu - e_min) <= 1e-11
        return s.finalize()
    assert abs(e_gpu - e_ref) <= 1e-11
    assert abs(e_gpu - rp.rspt_second_order_energy(h, h0)) <= 1e-10
    s.finalize()


def rspt_dense_problem(n=2000, seed=7):
    # A perturbation problem at a size the fixtures do not reach: H0 = diag(i / 10 + 1), a weak
    # symmetric perturbation (|H1| ~ 1e-3), so the series converges fast to the lowest eigenvalue.
    rng = np.random.default_rng(seed)
    h0 = 1.0 + 0.1 * np.arange(n)
    v = rng.uniform(-1e-3, 1e-3, (n, n))
    return np.diag(h0) + (v + v.T) / 2, h0


def rspt_series(trace, h, h0):
    x0 = rp.rspt_initial_guess(h0)
    return np.cumsum([x0 @ (h @ x0)] + [x0 @ (h @ t[-1]) for t in trace[:-1]])


def test_rspt_dense_2000_cpu():
    h, h0 = rspt_dense_problem()
    trace = rp.loop_rspt(rspt_cpu(h0.size), h, h0)
    series = rspt_series(trace, h, h0)
    exact = np.linalg.eigvalsh(h)[0]
    assert abs(series[1] - series[0] - rp.rspt_second_order_energy(h, h0)) <= 1e-15
    assert abs(series[-1] - exact) < 1e-12


@pytest.mark.gpu
def test_rspt_dense_2000_gpu():
    # the HBM path (C API, host R buffers) against the CPU path: same steps, each order's energy
    # and vector to the last digits the reductions' order leaves
    h, h0 = rspt_dense_problem()
    ref = rp.loop_rspt(rspt_cpu(h0.size), h, h0)
    g = rspt_gpu(h0.size)
    trace = rp.loop_rspt(g, h, h0)
    assert [t[:-1] for t in trace] == [t[:-1] for t in ref]
    for a, b in zip(trace, ref):
        np.testing.assert_allclose(a[-1], b[-1], rtol=0, atol=1e-12 * max(1e-300, np.max(np.abs(b[-1]))))
    np.testing.assert_allclose(rspt_series(trace, h, h0), rspt_series(ref, h, h0), rtol=1e-14, atol=0)
    g.finalize()


# ---- the reference's arithmetic: every reverse-communication loop bit for bit ------------------------
# These problems have at most 1000 elements, where the HIP path computes as the reference's loops do by
# default (sequential sums, no fused multiply-adds; ssp_ctx_set_exact_max): the GPU then
# takes the CPU path's steps with bit-identical parameters and values in every case -- including the
# cases above whose steps the CPU path itself changes under a 2^-50 perturbation, and n_eigen.
@pytest.mark.gpu
@pytest.mark.parametrize("family", list(EIGEN_FAMILIES))
def test_eigen_gpu_is_the_cpu_path_bit_for_bit(family):
    import iterative_solver

    for h in EIGEN_FAMILIES[family]():
        hermitian = bool(np.linalg.norm(h - h.T) < 1e-10)
        for nroot, np_ in rp.eigen_cases(h.shape[0], hermitian):
            tag = f"{family} n={h.shape[0]} nroot={nroot} np={np_}"
            c, ctrace, _, _ = run_eigen(cpu_eigen, h, nroot, np_)
            cst = c.stats()
            g, gtrace, _, _ = run_eigen(gpu_eigen, h, nroot, np_)
            st = iterative_solver.statistics()
            assert gtrace == ctrace, tag
            assert st["iterations"] == cst["iterations"], tag
            assert np.array_equal(np.asarray(g.eigenvalues), np.asarray(cst["eigenvalues"])), tag
            g.finalize()


@pytest.mark.gpu
def test_optimizer_and_diis_loops_gpu_are_the_cpu_path_bit_for_bit():
    for n in (2, 11, 20, 29):
        for alg in ("BFGS", "SD"):
            h = rp.quadratic_matrix(n, 10.0)
            ref = rp.loop_quadratic(cpu("Optimize", n, alg), h, optimize=True)
            g = gpu("Optimize", n, alg)
            same_trace(rp.loop_quadratic(g, h, optimize=True)[0], ref[0], xtol=0)
            g.finalize()
    for n in (2, 7, 20, 50):
        h = rp.quadratic_matrix(n, 10.0)
        ref = rp.loop_quadratic(cpu("NonLinearEquations", n), h, optimize=False)
        g = gpu("NonLinearEquations", n)
        same_trace(rp.loop_quadratic(g, h, optimize=False)[0], ref[0], xtol=0)
        g.finalize()
    for n in (2, 3, 4, 5, 6):  # Rosenbrock: above, 1e-6 mid-trajectory with the bandwidth kernels
        ref, _ = rp.loop_rosenbrock(cpu("Optimize", n, "BFGS"), n)
        g = gpu("Optimize", n, "BFGS")
        same_trace(rp.loop_rosenbrock(g, n)[0], ref, xtol=0)
        g.finalize()
    opts = "convergence_threshold=1e-8,max_size_qspace=5"
    for n in (1, 2):
        ref, _ = rp.loop_trig(cpu("NonLinearEquations", n, options=opts), n)
        g = gpu("NonLinearEquations", n, options=opts)
        same_trace(rp.loop_trig(g, n)[0], ref, xtol=0)
        g.finalize()
