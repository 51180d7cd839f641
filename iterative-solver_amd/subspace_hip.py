"""ctypes binding of libsubspace_hip.so (C ABI: include/subspace_hip.h).

Host-side plumbing for tests, smoke and bench: every operation here is a direct call into the HIP
library; nothing is computed on the CPU.  Importing works without a GPU (the library only needs the
HIP runtime to load); creating a Context requires a visible MI355X and raises otherwise.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libsubspace_hip.so")

STATUS = {
    0: "SSP_OK",
    1: "SSP_ERR_SIZE",
    2: "SSP_ERR_RANGE",
    3: "SSP_ERR_ARG",
    4: "SSP_ERR_HIP",
    5: "SSP_ERR_COMM",
    6: "SSP_ERR_NOMEM",
    7: "SSP_ERR_UNSUPPORTED",
}

# Every symbol include/subspace_hip.h declares (checked by tests/test_boundary.py).
EXPORTS = [
    "ssp_last_error", "ssp_version", "ssp_device_count", "ssp_ctx_create", "ssp_ctx_destroy", "ssp_ctx_stream",
    "ssp_synchronize", "ssp_alloc", "ssp_free", "ssp_release_cached", "ssp_memory_stats", "ssp_upload",
    "ssp_download", "ssp_comm_unique_id", "ssp_ctx_attach_comm", "ssp_ctx_rank", "ssp_ctx_nranks",
    "ssp_allreduce_sum", "ssp_allgather_host", "ssp_ledger_enable", "ssp_ledger_reset", "ssp_ledger_count",
    "ssp_ledger_entry", "ssp_fill", "ssp_scal", "ssp_copy", "ssp_axpy", "ssp_dot",
    "ssp_gemm_inner", "ssp_gemm_outer", "ssp_precondition", "ssp_select", "ssp_select_max_dot",
    "ssp_sparse_copy", "ssp_sparse_axpy", "ssp_sparse_dot", "ssp_gemm_inner_sparse", "ssp_gemm_outer_sparse",
    "sspx_synthetic_action", "sspx_synthetic_add_lowrank", "sspx_synthetic_diagonal", "sspx_fill_random", "sspx_dense_action",
]


class SspError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{STATUS.get(code, code)}: {what}")
        self.code = code


_lib = None


def load_library() -> C.CDLL:
    """Loads the in-tree HIP library; raises loudly if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C iterative-solver_amd` (or __graft_entry__.build())")
        lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        _declare(lib)
        _lib = lib
    return _lib


P = C.c_void_p
D = C.c_double
Z = C.c_size_t
I = C.c_int
PD = C.POINTER(C.c_double)
PZ = C.POINTER(C.c_size_t)


def _declare(lib):
    sig = {
        "ssp_last_error": (C.c_char_p, []),
        "ssp_version": (C.c_char_p, []),
        "ssp_device_count": (I, []),
        "ssp_ctx_create": (I, [I, C.POINTER(P)]),
        "ssp_ctx_destroy": (I, [P]),
        "ssp_ctx_stream": (P, [P]),
        "ssp_synchronize": (I, [P]),
        "ssp_alloc": (I, [P, Z, C.POINTER(P)]),
        "ssp_free": (I, [P, P]),
        "ssp_release_cached": (I, [P]),
        "ssp_memory_stats": (I, [P, PZ, PZ]),
        "ssp_upload": (I, [P, P, P, Z]),
        "ssp_download": (I, [P, P, P, Z]),
        "ssp_comm_unique_id": (I, [C.c_char_p]),
        "ssp_ctx_attach_comm": (I, [P, I, I, C.c_char_p]),
        "ssp_ctx_rank": (I, [P]),
        "ssp_ctx_nranks": (I, [P]),
        "ssp_allreduce_sum": (I, [P, P, Z]),
        "ssp_allgather_host": (I, [P, P, P, Z]),
        "ssp_ledger_enable": (I, [P, I]),
        "ssp_ledger_reset": (I, [P]),
        "ssp_ledger_count": (I, [P]),
        "ssp_ledger_entry": (I, [P, I, C.POINTER(C.c_char_p), C.POINTER(C.c_longlong), PD, PD]),
        "ssp_fill": (I, [P, D, P, Z]),
        "ssp_scal": (I, [P, D, P, Z]),
        "ssp_copy": (I, [P, P, P, Z]),
        "ssp_axpy": (I, [P, D, P, P, Z]),
        "ssp_dot": (I, [P, P, P, Z, PD]),
        "ssp_gemm_inner": (I, [P, P, I, P, I, Z, PD]),
        "ssp_gemm_outer": (I, [P, PD, P, I, P, I, Z]),
        "ssp_precondition": (I, [P, P, I, P, PD, Z]),
        "ssp_select": (I, [P, P, Z, Z, Z, I, I, PZ, PD, PZ]),
        "ssp_select_max_dot": (I, [P, P, P, Z, Z, Z, PZ, PD, PZ]),
        "ssp_sparse_copy": (I, [P, P, Z, Z, PZ, PD, Z]),
        "ssp_sparse_axpy": (I, [P, D, PZ, PD, Z, P, Z, Z]),
        "ssp_sparse_dot": (I, [P, P, Z, Z, PZ, PD, Z, PD]),
        "ssp_gemm_inner_sparse": (I, [P, P, I, Z, Z, PZ, PZ, PD, I, PD]),
        "ssp_gemm_outer_sparse": (I, [P, PD, PZ, PZ, PD, I, P, I, Z, Z]),
        "sspx_synthetic_action": (I, [P, P, P, I, Z, Z, D, I, C.c_ulonglong]),
        "sspx_synthetic_add_lowrank": (I, [P, P, I, Z, Z, D, I, C.c_ulonglong, PD]),
        "sspx_synthetic_diagonal": (I, [P, P, Z, Z, D, I]),
        "sspx_fill_random": (I, [P, P, Z, Z, C.c_ulonglong, C.c_ulonglong]),
        "sspx_dense_action": (I, [P, P, Z, P, P, I, Z, Z]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args


def _check(code: int):
    if code != 0:
        raise SspError(code, load_library().ssp_last_error().decode())


def _ptrs(vecs: Sequence["DeviceVector"]):
    arr = (C.c_void_p * max(1, len(vecs)))(*[v.ptr for v in vecs])
    return arr


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(PD)


def _zptr(a: np.ndarray):
    return a.ctypes.data_as(PZ)


class DeviceVector:
    """One HBM shard of n doubles, owned by a Context's arena."""

    def __init__(self, ctx: "Context", n: int, ptr: int, owner: bool = True):
        self.ctx, self.n, self.ptr, self.owner = ctx, n, ptr, owner

    def free(self):
        if self.owner and self.ptr:
            _check(self.ctx.lib.ssp_free(self.ctx.handle, self.ptr))
        self.ptr = 0

    def numpy(self) -> np.ndarray:
        return self.ctx.download(self)

    def __len__(self):
        return self.n


class Context:
    """One HIP device + stream (+ optional RCCL communicator): the unit the C ABI works on."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = C.c_void_p()
        _check(self.lib.ssp_ctx_create(device, C.byref(h)))
        self.handle = h.value
        self.device = device

    def close(self):
        if getattr(self, "handle", None):
            self.lib.ssp_ctx_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def stream(self) -> int:
        return self.lib.ssp_ctx_stream(self.handle)

    def synchronize(self):
        _check(self.lib.ssp_synchronize(self.handle))

    # -- memory -----------------------------------------------------------------------------
    def alloc(self, n: int) -> DeviceVector:
        p = C.c_void_p()
        _check(self.lib.ssp_alloc(self.handle, n, C.byref(p)))
        return DeviceVector(self, n, p.value)

    def upload(self, a: np.ndarray) -> DeviceVector:
        a = np.ascontiguousarray(a, dtype=np.float64)
        v = self.alloc(a.size)
        _check(self.lib.ssp_upload(self.handle, v.ptr, a.ctypes.data, a.size))
        return v

    def upload_into(self, v: DeviceVector, a: np.ndarray):
        a = np.ascontiguousarray(a, dtype=np.float64)
        assert a.size == v.n
        _check(self.lib.ssp_upload(self.handle, v.ptr, a.ctypes.data, a.size))

    def download(self, v: DeviceVector) -> np.ndarray:
        out = np.empty(v.n, dtype=np.float64)
        _check(self.lib.ssp_download(self.handle, out.ctypes.data, v.ptr, v.n))
        return out

    def memory_stats(self):
        a, b = C.c_size_t(), C.c_size_t()
        _check(self.lib.ssp_memory_stats(self.handle, C.byref(a), C.byref(b)))
        return a.value, b.value

    def release_cached(self):
        _check(self.lib.ssp_release_cached(self.handle))

    # -- communicator -------------------------------------------------------------------------
    @staticmethod
    def unique_id() -> bytes:
        lib = load_library()
        buf = C.create_string_buffer(128)
        _check(lib.ssp_comm_unique_id(buf))
        return buf.raw

    def attach_comm(self, nranks: int, rank: int, uid: bytes):
        _check(self.lib.ssp_ctx_attach_comm(self.handle, nranks, rank, uid))

    # -- ledger (HIP-event kernel times + algorithmic bytes per operation) --------------------------
    def ledger_enable(self, on: bool = True):
        _check(self.lib.ssp_ledger_enable(self.handle, int(on)))

    def ledger_reset(self):
        _check(self.lib.ssp_ledger_reset(self.handle))

    def ledger(self) -> dict:
        """{op: {"calls": c, "ms": kernel milliseconds, "bytes": algorithmic bytes}}"""
        cnt = self.lib.ssp_ledger_count(self.handle)
        if cnt < 0:
            _check(4)
        out = {}
        for i in range(cnt):
            name, calls, ms, nb = C.c_char_p(), C.c_longlong(), C.c_double(), C.c_double()
            _check(self.lib.ssp_ledger_entry(self.handle, i, C.byref(name), C.byref(calls), C.byref(ms), C.byref(nb)))
            out[name.value.decode()] = {"calls": calls.value, "ms": ms.value, "bytes": nb.value}
        return out

    # -- ops ----------------------------------------------------------------------------------
    def fill(self, alpha: float, x: DeviceVector):
        _check(self.lib.ssp_fill(self.handle, alpha, x.ptr, x.n))

    def scal(self, alpha: float, x: DeviceVector):
        _check(self.lib.ssp_scal(self.handle, alpha, x.ptr, x.n))

    def copy(self, x: DeviceVector, y: DeviceVector):
        _check(self.lib.ssp_copy(self.handle, x.ptr, y.ptr, x.n))

    def axpy(self, alpha: float, x: DeviceVector, y: DeviceVector):
        _check(self.lib.ssp_axpy(self.handle, alpha, x.ptr, y.ptr, y.n))

    def dot(self, x: DeviceVector, y: DeviceVector) -> float:
        out = C.c_double()
        _check(self.lib.ssp_dot(self.handle, x.ptr, y.ptr, x.n, C.byref(out)))
        return out.value

    def gemm_inner(self, xx: Sequence[DeviceVector], yy: Sequence[DeviceVector]) -> np.ndarray:
        m, k = len(xx), len(yy)
        out = np.zeros((m, k))
        n = xx[0].n if m else 0
        _check(self.lib.ssp_gemm_inner(self.handle, _ptrs(xx), m, _ptrs(yy), k, n, _dptr(out)))
        return out

    def gemm_outer(self, alphas: np.ndarray, xx: Sequence[DeviceVector], yy: Sequence[DeviceVector]):
        alphas = np.ascontiguousarray(alphas, dtype=np.float64)
        k, m = len(xx), len(yy)
        assert alphas.shape == (k, m)
        n = yy[0].n if m else 0
        _check(self.lib.ssp_gemm_outer(self.handle, _dptr(alphas), _ptrs(xx), k, _ptrs(yy), m, n))

    def precondition(self, aa: Sequence[DeviceVector], d: DeviceVector, shift: Sequence[float]):
        sh = np.ascontiguousarray(shift, dtype=np.float64)
        _check(self.lib.ssp_precondition(self.handle, _ptrs(aa), len(aa), d.ptr, _dptr(sh), d.n))

    def select(self, x: DeviceVector, nsel: int, max: bool = False, ignore_sign: bool = False, offset: int = 0):
        idx = np.zeros(max_(nsel), dtype=np.uint64)
        val = np.zeros(max_(nsel))
        nout = C.c_size_t()
        _check(self.lib.ssp_select(self.handle, x.ptr, x.n, offset, nsel, int(max), int(ignore_sign), _zptr(idx),
                                   _dptr(val), C.byref(nout)))
        return idx[: nout.value].astype(np.int64), val[: nout.value]

    def select_max_dot(self, x: DeviceVector, y: DeviceVector, nsel: int, offset: int = 0):
        idx = np.zeros(max_(nsel), dtype=np.uint64)
        val = np.zeros(max_(nsel))
        nout = C.c_size_t()
        _check(self.lib.ssp_select_max_dot(self.handle, x.ptr, y.ptr, x.n, offset, nsel, _zptr(idx), _dptr(val),
                                           C.byref(nout)))
        return idx[: nout.value].astype(np.int64), val[: nout.value]

    def sparse_copy(self, x: DeviceVector, idx, val, offset: int = 0):
        idx = np.ascontiguousarray(idx, dtype=np.uint64)
        val = np.ascontiguousarray(val, dtype=np.float64)
        _check(self.lib.ssp_sparse_copy(self.handle, x.ptr, x.n, offset, _zptr(idx), _dptr(val), idx.size))

    def sparse_axpy(self, alpha: float, idx, val, x: DeviceVector, offset: int = 0):
        idx = np.ascontiguousarray(idx, dtype=np.uint64)
        val = np.ascontiguousarray(val, dtype=np.float64)
        _check(self.lib.ssp_sparse_axpy(self.handle, alpha, _zptr(idx), _dptr(val), idx.size, x.ptr, x.n, offset))

    def sparse_dot(self, x: DeviceVector, idx, val, offset: int = 0) -> float:
        idx = np.ascontiguousarray(idx, dtype=np.uint64)
        val = np.ascontiguousarray(val, dtype=np.float64)
        out = C.c_double()
        _check(self.lib.ssp_sparse_dot(self.handle, x.ptr, x.n, offset, _zptr(idx), _dptr(val), idx.size,
                                       C.byref(out)))
        return out.value

    @staticmethod
    def _pack_sparse(ps):
        ptr = np.zeros(len(ps) + 1, dtype=np.uint64)
        idx, val = [], []
        for j, p in enumerate(ps):
            keys = sorted(p)
            idx.extend(keys)
            val.extend(p[k] for k in keys)
            ptr[j + 1] = len(idx)
        return ptr, np.asarray(idx, dtype=np.uint64), np.asarray(val, dtype=np.float64)

    def gemm_inner_sparse(self, xx: Sequence[DeviceVector], ps: Sequence[dict], offset: int = 0) -> np.ndarray:
        ptr, idx, val = self._pack_sparse(ps)
        m, k = len(xx), len(ps)
        out = np.zeros((m, k))
        n = xx[0].n if m else 0
        _check(self.lib.ssp_gemm_inner_sparse(self.handle, _ptrs(xx), m, n, offset, _zptr(ptr), _zptr(idx),
                                              _dptr(val), k, _dptr(out)))
        return out

    def gemm_outer_sparse(self, alphas: np.ndarray, ps: Sequence[dict], yy: Sequence[DeviceVector], offset: int = 0):
        ptr, idx, val = self._pack_sparse(ps)
        alphas = np.ascontiguousarray(alphas, dtype=np.float64)
        k, m = len(ps), len(yy)
        assert alphas.shape == (k, m)
        n = yy[0].n if m else 0
        _check(self.lib.ssp_gemm_outer_sparse(self.handle, _dptr(alphas), _zptr(ptr), _zptr(idx), _dptr(val), k,
                                              _ptrs(yy), m, n, offset))

    # -- synthetic problem (harness) ------------------------------------------------------------
    def synthetic_action(self, xx, yy, rho: float, rank: int, seed: int, offset: int = 0):
        _check(self.lib.sspx_synthetic_action(self.handle, _ptrs(xx), _ptrs(yy), len(xx), xx[0].n, offset, rho, rank,
                                              seed))

    def synthetic_diagonal(self, d: DeviceVector, rho: float, rank: int, offset: int = 0):
        _check(self.lib.sspx_synthetic_diagonal(self.handle, d.ptr, d.n, offset, rho, rank))

    def fill_random(self, x: DeviceVector, seed: int, vec: int, offset: int = 0):
        _check(self.lib.sspx_fill_random(self.handle, x.ptr, x.n, offset, seed, vec))


def max_(n: int) -> int:
    return n if n > 0 else 1


def device_count() -> int:
    return load_library().ssp_device_count()
