"""Reverse-communication solver loops of the reference's tests (test_Optimize.cpp,
test_NonLinearEquations.cpp) on problems defined in Python (tests/rc_problems.py).

CPU: the reference CPU path (oracle.RcSolver: the restated solvers over the CPU handlers, called
     as the C API calls them) must satisfy the reference tests' own assertions.
GPU: the same loops through the C API on the HIP handlers (iterative_solver package) take the
     same steps as the CPU path -- identical per-iteration return values and iteration counts,
     parameters within 1e-10 (1e-6 mid-trajectory on Rosenbrock) -- and satisfy the same
     assertions.
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
