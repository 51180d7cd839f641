"""Component pins of the restated host layer (the solver code the GPU path and the oracle share):
the reference's own component tests restated in C++ (tests/cpp/host_layer_test.cpp,
tests/cpp/matrix_test.cpp), compiled with g++ and run on CPU.

* subspace::Matrix runs the cases of the reference's testMatrix.cpp twice: on the restated
  itsolv_hbm/matrix.h and on the reference's own subspace/Matrix.h (where /root/reference exists),
  so the restatement is checked against the reference code itself;
* host_layer_test: subspace/test_util.cpp (overlap, parameter_batches), testDSpaceResetter.cpp,
  itsolv/test_util.cpp (is_iota, construct_zeroed_copy, delete_parameters, StringFacet),
  test_SolverFactory.cpp (option strings -> get_options()), QSpace/XSpace update semantics;
* test_svd_system.cpp:64-90: the restated eigensolver_lapacke_dsyev / svd_system on the reference
  test's rand()-built matrix against LAPACK through numpy (the reference compares with Eigen at 1e-4;
  here 1e-12).
"""
import json
import os
import subprocess
import tempfile

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SAN = os.environ.get("ITSOLV_SAN_FLAGS", "").split()  # tools/asan_cpu.sh: the sanitizer build
ROOT = os.path.dirname(HERE)
REF_SRC = "/root/reference/src"
INC = ["-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "iterative-solver_amd", "include"),
       "-I" + os.path.join(ROOT, "oracle")]
ORACLE_BUILD = os.path.join(ROOT, "oracle", "build")


def build(src, extra=(), libs=()):
    d = tempfile.mkdtemp()
    exe = os.path.join(d, "t")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", *extra, *SAN, *INC, os.path.join(HERE, "cpp", src), "-o", exe,
                        *libs], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    return exe


def run_cases(exe, *args):
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OK 0 failure(s)" in r.stdout, r.stdout[-4000:] + r.stderr[-2000:]
    return r.stdout


@pytest.fixture(scope="module")
def host_exe():
    if not os.path.exists(os.path.join(ORACLE_BUILD, "liboracle_ops.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    return build("host_layer_test.cpp", libs=["-L" + ORACLE_BUILD, "-loracle_ops", "-Wl,-rpath," + ORACLE_BUILD])


def test_matrix_restated():
    out = run_cases(build("matrix_test.cpp"))
    assert "base: restated" in out and out.count("PASS ") == 18


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference tree not present")
def test_matrix_reference_header_same_cases():
    out = run_cases(build("matrix_test.cpp", ["-DWITH_REFERENCE_BASE", "-I" + REF_SRC]))
    assert "base: reference" in out and out.count("PASS ") == 18


def test_host_layer_components(host_exe):
    out = run_cases(host_exe)
    for name in ("overlap_reverse_params", "parameter_batches", "resize_qspace", "max_overlap_with_R_qparams_0",
                 "StringFacet_parse_keyval_string", "solver_factory_string_constructor", "qspace_prepend_and_blocks",
                 "ordered_gemm_is_the_triple_loop", "eigenproblem_kept_vectors", "screen_cholesky_proof"):
        assert "PASS " + name in out
    assert out.count("PASS ") == 30


def test_svd_system_against_lapack(host_exe):
    r = subprocess.run([host_exe, "svd"], capture_output=True, text=True, timeout=60)
    d = json.loads(r.stdout)
    n = d["dim"]
    m = np.array(d["matrix"]).reshape(n, n)  # column-major as the reference builds it; symmetric
    assert np.array_equal(m, m.T)
    w, v = np.linalg.eigh(m)
    np.testing.assert_allclose(d["eigenvalues"], w, rtol=1e-12, atol=0)
    vecs = np.array(d["eigenvectors"]).reshape(n, n).T  # eigenvector i in column i (LAPACK layout)
    np.testing.assert_allclose(np.abs(vecs), np.abs(v), atol=1e-10)
    # svd_system(hermitian): eigenpairs largest first (helper-implementation.h:263-296)
    np.testing.assert_allclose(d["svd_values"], np.sort(np.linalg.svd(m, compute_uv=False))[::-1], rtol=1e-12)
    sv = np.array(d["svd_vectors"]).reshape(n, n)
    np.testing.assert_allclose(np.abs(sv), np.abs(v[:, ::-1].T), atol=1e-10)


def sym_eigen(exe, a):
    n = a.shape[0]
    inp = f"{n}\n" + "\n".join(repr(float(x)) for x in a.ravel()) + "\n"
    r = subprocess.run([exe, "sym_eigen"], input=inp, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    v = np.array(r.stdout.split(), dtype=float)
    return v[:n], v[n:].reshape(n, n).T  # eigenvector i in column i


def sym_cases():
    r = np.random.default_rng(3)
    for n in (1, 2, 3, 7, 24, 48, 72, 100):
        m = r.standard_normal((n, n))
        yield f"random{n}", m + m.T
    yield "identity", np.eye(9)
    yield "zero", np.zeros((5, 5))
    yield "repeated", np.diag([1.0, 2.0, 2.0, 2.0, 5.0, 5.0])
    u = r.standard_normal(20)
    yield "rank_one", np.outer(u, u)
    w = np.diag(np.abs(np.arange(-10, 11)).astype(float)) + np.diag(np.ones(20), 1) + np.diag(np.ones(20), -1)
    yield "wilkinson21", w
    q, _ = np.linalg.qr(r.standard_normal((30, 30)))
    yield "clustered", q @ np.diag(1 + 1e-12 * np.arange(30)) @ q.T
    yield "graded", q @ np.diag(10.0 ** np.linspace(-10, 10, 30)) @ q.T
    x = r.standard_normal((60, 12))
    yield "overlap_rank12", x.T @ x  # a Davidson overlap matrix shape (full rank)
    y = r.standard_normal((40, 8))
    yield "overlap_rank_deficient", np.hstack([y, y[:, :3]]).T @ np.hstack([y, y[:, :3]])


@pytest.mark.parametrize("name,a", list(sym_cases()), ids=[c[0] for c in sym_cases()])
def test_sym_eigen_tridiagonal_ql_against_lapack(host_exe, name, a):
    # dense::sym_eigen (Householder + implicit QL, as dsyev / Eigen's SelfAdjointEigenSolver) against
    # LAPACK through numpy: eigenvalues, residuals and orthonormality to backward-stable accuracy.
    n = a.shape[0]
    ev, vec = sym_eigen(host_exe, a)
    w = np.linalg.eigvalsh(a)
    scale = max(np.linalg.norm(a, 2), 1e-300)
    tol = 1e-14 * max(n, 4) * scale
    assert np.all(np.diff(ev) >= 0), "ascending"
    np.testing.assert_allclose(ev, w, rtol=0, atol=tol)
    assert np.max(np.abs(a @ vec - vec * ev)) <= 10 * tol
    assert np.max(np.abs(vec.T @ vec - np.eye(n))) <= 1e-14 * max(n, 4) * 10
