"""The drop-in boundary: the C-ABI libraries load here (no GPU) and export every symbol the headers
in include/ declare.  No compute calls are made without a GPU."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INCLUDE = os.path.join(ROOT, "include")
LIBDIR = os.path.join(ROOT, "iterative-solver_amd", "lib")

HEADERS = {
    "subspace_hip.h": "libsubspace_hip.so",
    "itsolv_hbm.h": "libitsolv_hbm.so",
    "iterative_solver_c.h": "libitsolv_hbm.so",
}
# The reverse-communication API keeps the reference's names (src/molpro/linalg/IterativeSolverC.h).
REFERENCE_C_API = [
    "IterativeSolverLinearEigensystemInitialize", "IterativeSolverLinearEquationsInitialize",
    "IterativeSolverNonLinearEquationsInitialize", "IterativeSolverOptimizeInitialize", "IterativeSolverFinalize",
    "IterativeSolverAddVector", "IterativeSolverSolution", "IterativeSolverAddValue", "IterativeSolverEndIteration",
    "IterativeSolverEndIterationNeeded", "IterativeSolverAddP", "IterativeSolverErrors", "IterativeSolverEigenvalues",
    "IterativeSolverWorkingSetEigenvalues", "IterativeSolverSuggestP", "IterativeSolverPrintStatistics",
    "IterativeSolverNonLinear", "IterativeSolverHasValues", "IterativeSolverHasEigenvalues",
    "IterativeSolverSetDiagonals", "IterativeSolverDiagonals", "IterativeSolverValue", "IterativeSolverVerbosity",
    "IterativeSolverMaxIter", "IterativeSolverSetMaxIter", "mpicomm_self", "mpicomm_global",
    "IterativeSolver_mpicomm_global", "IterativeSolver_mpicomm_self",
    # IterativeSolverCMPI.cpp:516-534, and the spellings IterativeSolverF.F90:46-57 binds
    "IterativeSolver_mpisize_global", "IterativeSolver_mpirank_global", "IterativeSolver_mpi_init",
    "IterativeSolver_mpi_finalize", "IterativeSolver_mpi_size_global", "IterativeSolver_mpi_rank_global",
]


def declared_functions(header):
    text = open(os.path.join(INCLUDE, header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b((?:ssp|sspx|itsolv)_\w+|IterativeSolver\w+|mpicomm_\w+)\s*\(",
                       text, flags=re.M)
    return sorted(set(names))


@pytest.mark.parametrize("header,lib", sorted(HEADERS.items()))
def test_library_exports_every_declared_symbol(header, lib):
    if not os.path.exists(os.path.join(INCLUDE, header)):
        pytest.skip(f"{header} not present")
    path = os.path.join(LIBDIR, lib)
    assert os.path.exists(path), f"{path} not built (run __graft_entry__.build())"
    so = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    names = declared_functions(header)
    assert len(names) > 5
    missing = [n for n in names if not hasattr(so, n)]
    assert not missing, f"{lib} lacks {missing}"


def test_reverse_communication_api_is_the_reference_name_set():
    declared = declared_functions("iterative_solver_c.h")
    assert set(REFERENCE_C_API) <= set(declared)
    extra = sorted(set(declared) - set(REFERENCE_C_API))
    assert all(n.startswith("IterativeSolverHbm") for n in extra), extra


def test_python_binding_lists_every_symbol():
    import subspace_hip as sh

    assert sorted(sh.EXPORTS) == declared_functions("subspace_hip.h")


def test_library_loads_without_gpu_and_reports_errors():
    import subspace_hip as sh

    lib = sh.load_library()
    assert b"gfx950" in lib.ssp_version()
    if sh.device_count() == 0:
        h = ctypes.c_void_p()
        code = lib.ssp_ctx_create(0, ctypes.byref(h))
        assert code != 0 and h.value is None
        assert len(lib.ssp_last_error()) > 0


def test_code_object_targets_gfx950():
    data = open(os.path.join(LIBDIR, "libsubspace_hip.so"), "rb").read()
    assert b"gfx950" in data
