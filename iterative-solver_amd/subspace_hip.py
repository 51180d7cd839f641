"""ctypes binding of libsubspace_hip.so (C ABI: include/subspace_hip.h).

Host-side plumbing for tests, smoke and bench: every operation here is a direct call into the HIP
library; nothing is computed on the CPU.  Importing works without a GPU (the library only needs the
HIP runtime to load); creating a Context requires a visible MI355X and raises otherwise.
"""
from __future__ import annotations

import builtins
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
    8: "SSP_ERR_COMM_ABANDONED",
}

# Every symbol include/subspace_hip.h declares (checked by tests/test_boundary.py).
EXPORTS = [
    "ssp_last_error", "ssp_version", "ssp_device_count", "ssp_ctx_create", "ssp_ctx_destroy", "ssp_ctx_stream",
    "ssp_synchronize", "ssp_alloc", "ssp_free", "ssp_release_cached", "ssp_memory_stats", "ssp_upload",
    "ssp_download", "ssp_comm_unique_id", "ssp_ctx_attach_comm", "ssp_ctx_rank", "ssp_ctx_nranks",
    "ssp_allreduce_sum", "ssp_allgather_host", "ssp_ctx_attach_host_comm", "ssp_shard_range", "ssp_select_merge",
    "ssp_p2p_unique_id", "ssp_ctx_attach_p2p", "ssp_ctx_set_comm_timeout", "sspx_debug_stall",
    "ssp_ctx_set_exact_max",
    "ssp_ledger_enable", "ssp_ledger_reset", "ssp_ledger_count", "ssp_ledger_reserve",
    "ssp_ledger_entry", "ssp_fill", "ssp_scal", "ssp_copy", "ssp_axpy", "ssp_dot",
    "ssp_gemm_inner", "ssp_gemm_outer", "ssp_gemm_outer_set", "ssp_axpy_inner", "ssp_scal_inner", "ssp_axpy_norm", "ssp_axpy_gram", "ssp_transform_gram", "ssp_transform_norms", "ssp_axpy_pairs_norm", "ssp_precondition", "ssp_precondition_norms", "ssp_select", "ssp_select_max_dot",
    "ssp_sparse_copy", "ssp_sparse_axpy", "ssp_sparse_axpy_batch", "ssp_sparse_dot", "ssp_gemm_inner_sparse", "ssp_gemm_outer_sparse",
    "ssp_construct_solution",
    "sspx_synthetic_action", "sspx_synthetic_add_lowrank", "sspx_synthetic_diagonal", "sspx_fill_random", "sspx_dense_action",
    "sspx_synth_action", "sspx_synth_add_lowrank", "sspx_synth_diagonal",
    # deferred scal (hbm_vec.h): operands with pending scales
    "ssp_scal_copy", "ssp_axpy_scaled", "ssp_dot_scaled", "ssp_gemm_inner_scaled", "ssp_gemm_outer_scaled",
    "ssp_gemm_outer_set_scaled", "ssp_gemm_inner_sparse_scaled", "ssp_construct_solution_scaled", "ssp_block_update",
    "sspx_synth_action_scaled",
    # a sparse inner product queued ahead of other work
    "ssp_gemm_inner_sparse_begin", "ssp_gemm_inner_sparse_end",
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
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, PD, C.c_size_t, C.c_void_p)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)


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
        "ssp_ctx_attach_host_comm": (I, [P, I, I, ALLREDUCE_FN, ALLGATHER_FN, P]),
        "ssp_p2p_unique_id": (I, [C.c_char_p]),
        "ssp_ctx_attach_p2p": (I, [P, I, I, C.c_char_p]),
        "ssp_ctx_set_comm_timeout": (I, [P, D]),
        "sspx_debug_stall": (I, [P, D]),
        "ssp_ctx_set_exact_max": (I, [P, Z]),
        "ssp_shard_range": (I, [Z, I, I, PZ, PZ]),
        "ssp_select_merge": (I, [I, PZ, Z, PZ, PD, Z, I, PZ, PD, PZ]),
        "ssp_ledger_enable": (I, [P, I]),
        "ssp_ledger_reset": (I, [P]),
        "ssp_ledger_count": (I, [P]),
        "ssp_ledger_reserve": (I, [P, I]),
        "ssp_ledger_entry": (I, [P, I, C.POINTER(C.c_char_p), C.POINTER(C.c_longlong), PD, PD]),
        "ssp_fill": (I, [P, D, P, Z]),
        "ssp_scal": (I, [P, D, P, Z]),
        "ssp_copy": (I, [P, P, P, Z]),
        "ssp_axpy": (I, [P, D, P, P, Z]),
        "ssp_dot": (I, [P, P, P, Z, PD]),
        "ssp_gemm_inner": (I, [P, P, I, P, I, Z, PD]),
        "ssp_gemm_outer": (I, [P, PD, P, I, P, I, Z]),
        "ssp_gemm_outer_set": (I, [P, PD, P, I, P, I, Z]),
        "ssp_axpy_inner": (I, [P, PD, P, P, I, P, Z, PD]),
        "ssp_scal_inner": (I, [P, C.c_double, P, P, I, Z, PD]),
        "ssp_axpy_norm": (I, [P, PD, P, P, I, Z, PD]),
        "ssp_axpy_gram": (I, [P, PD, P, D, I, P, I, Z, PD]),
        "ssp_transform_gram": (I, [P, PD, P, PD, I, Z, PD]),
        "ssp_transform_norms": (I, [P, PD, P, PD, I, Z, PD]),
        "ssp_axpy_pairs_norm": (I, [P, PD, P, PD, P, PD, I, Z, PD]),
        "ssp_precondition": (I, [P, P, I, P, PD, Z]),
        "ssp_precondition_norms": (I, [P, P, I, P, PD, Z, PD]),
        "ssp_select": (I, [P, P, Z, Z, Z, I, I, PZ, PD, PZ]),
        "ssp_select_max_dot": (I, [P, P, P, Z, Z, Z, PZ, PD, PZ]),
        "ssp_sparse_copy": (I, [P, P, Z, Z, PZ, PD, Z]),
        "ssp_sparse_axpy": (I, [P, D, PZ, PD, Z, P, Z, Z]),
        "ssp_sparse_axpy_batch": (I, [P, I, PZ, PZ, PD, P, Z, Z]),
        "ssp_sparse_dot": (I, [P, P, Z, Z, PZ, PD, Z, PD]),
        "ssp_gemm_inner_sparse": (I, [P, P, I, Z, Z, PZ, PZ, PD, I, PD]),
        "ssp_gemm_outer_sparse": (I, [P, PD, PZ, PZ, PD, I, P, I, Z, Z]),
        "ssp_construct_solution": (I, [P, PD, PZ, PZ, PD, I, PD, P, I, P, I, Z, Z]),
        "sspx_synthetic_action": (I, [P, P, P, I, Z, Z, D, I, C.c_ulonglong]),
        "sspx_synthetic_add_lowrank": (I, [P, P, I, Z, Z, D, I, C.c_ulonglong, PD]),
        "sspx_synthetic_diagonal": (I, [P, P, Z, Z, D, I]),
        "sspx_synth_action": (I, [P, P, P, P, I, Z, Z]),
        "sspx_synth_add_lowrank": (I, [P, P, P, I, Z, Z, PD]),
        "sspx_synth_diagonal": (I, [P, P, P, Z, Z]),
        "sspx_fill_random": (I, [P, P, Z, Z, C.c_ulonglong, C.c_ulonglong]),
        "sspx_dense_action": (I, [P, P, Z, P, P, I, Z, Z]),
        "ssp_scal_copy": (I, [P, D, P, P, Z]),
        "ssp_axpy_scaled": (I, [P, D, P, D, P, D, Z]),
        "ssp_dot_scaled": (I, [P, P, D, P, D, Z, PD]),
        "ssp_gemm_inner_scaled": (I, [P, P, PD, I, P, PD, I, Z, PD]),
        "ssp_gemm_outer_scaled": (I, [P, PD, P, PD, I, P, PD, I, Z]),
        "ssp_gemm_outer_set_scaled": (I, [P, PD, P, PD, I, P, I, Z]),
        "ssp_gemm_inner_sparse_scaled": (I, [P, P, PD, I, Z, Z, PZ, PZ, PD, I, PD]),
        "ssp_gemm_inner_sparse_begin": (I, [P, P, PD, I, Z, Z, PZ, PZ, PD, I]),
        "ssp_gemm_inner_sparse_end": (I, [P, PD]),
        "ssp_construct_solution_scaled": (I, [P, PD, PZ, PZ, PD, I, PD, P, PD, I, P, I, Z, Z]),
        "ssp_block_update": (I, [P, PD, PZ, PZ, PD, I, PD, P, PD, I, P, PD, I, Z, Z]),
        "sspx_synth_action_scaled": (I, [P, P, P, PD, P, I, Z, Z]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args


def shard_range(n: int, nranks: int, rank: int):
    """(offset, length) of rank's shard (ssp_shard_range: the reference's
    make_distribution_spread_remainder).  Host only."""
    off, ln = C.c_size_t(), C.c_size_t()
    _check(load_library().ssp_shard_range(n, nranks, rank, C.byref(off), C.byref(ln)))
    return off.value, ln.value


def select_merge(parts, nsel: int, max: bool = False):
    """ssp_select_merge over per-rank (idx, val) selections, as ssp_select merges its all-gathered
    candidates.  Host only.  Returns (idx, val) ordered by index."""
    nr = len(parts)
    stride = max_(builtins.max((len(i) for i, _ in parts), default=0))
    counts = np.array([len(i) for i, _ in parts], dtype=np.uint64)
    idx = np.zeros(nr * stride, dtype=np.uint64)
    val = np.zeros(nr * stride)
    for r, (i, v) in enumerate(parts):
        idx[r * stride:r * stride + len(i)] = i
        val[r * stride:r * stride + len(v)] = v
    oi, ov, cnt = np.zeros(max_(nsel), dtype=np.uint64), np.zeros(max_(nsel)), C.c_size_t()
    _check(load_library().ssp_select_merge(nr, _zptr(counts), stride, _zptr(idx), _dptr(val), nsel, int(max),
                                           _zptr(oi), _dptr(ov), C.byref(cnt)))
    return oi[:cnt.value].astype(np.int64), ov[:cnt.value]


class TorchHostComm:
    """Host-side callbacks for ssp_ctx_attach_host_comm over a torch.distributed (gloo) group:
    allreduce(sum) of doubles and allgather of raw bytes.  Plumbing for running the sharded
    path with several ranks where RCCL is unavailable (several ranks on one device, CPU tests)."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist

        self.torch, self.dist, self.group = torch, dist, group
        self.nranks = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.allreduce_cb = ALLREDUCE_FN(self._allreduce)
        self.allgather_cb = ALLGATHER_FN(self._allgather)

    def _allreduce(self, buf, n, _user):
        try:
            a = np.ctypeslib.as_array(buf, shape=(n,))
            t = self.torch.from_numpy(a.copy())
            self.dist.all_reduce(t, group=self.group)
            a[:] = t.numpy()
            return 0
        except Exception:  # noqa: BLE001 - reported to the C side as a status
            return 1

    def _allgather(self, send, recv, nbytes, _user):
        try:
            src = np.frombuffer((C.c_char * nbytes).from_address(send), dtype=np.uint8).copy() if nbytes else \
                np.zeros(0, dtype=np.uint8)
            outs = [self.torch.zeros(nbytes, dtype=self.torch.uint8) for _ in range(self.nranks)]
            self.dist.all_gather(outs, self.torch.from_numpy(src), group=self.group)
            dst = (C.c_char * (nbytes * self.nranks)).from_address(recv)
            for r, o in enumerate(outs):
                dst[r * nbytes:(r + 1) * nbytes] = o.numpy().tobytes()
            return 0
        except Exception:  # noqa: BLE001
            return 1


class HubComm:
    """Host communicator over plain TCP sockets (stdlib only, no torch): rank 0 is the hub, every
    collective gathers the ranks' buffers there in rank order and sends the result back, so all
    ranks receive bit-identical sums.  Used to run the sharded path with several ranks on ONE
    device (RCCL refuses duplicate devices) and in multi-process CPU tests."""

    def __init__(self, rank: int, nranks: int, addr: str = "127.0.0.1", port: int = 0, timeout: float = 120.0):
        import socket
        import struct
        import time

        self.rank, self.nranks, self._struct = rank, nranks, struct
        self.peers = {}
        if nranks > 1:
            if rank == 0:
                srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
                srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
                srv.bind((addr, port))
                srv.listen(nranks)
                srv.settimeout(timeout)
                for _ in range(nranks - 1):
                    c, _a = srv.accept()
                    c.settimeout(timeout)
                    (r,) = struct.unpack("<i", self._recv(c, 4))
                    self.peers[r] = c
                srv.close()
            else:
                t0 = time.time()
                while True:
                    try:
                        c = socket.create_connection((addr, port), timeout=timeout)
                        break
                    except OSError:
                        if time.time() - t0 > timeout:
                            raise
                        time.sleep(0.05)
                c.sendall(struct.pack("<i", rank))
                self.peers[0] = c
        self.allreduce_cb = ALLREDUCE_FN(self._allreduce_cb)
        self.allgather_cb = ALLGATHER_FN(self._allgather_cb)

    @staticmethod
    def _recv(c, n):
        out = bytearray()
        while len(out) < n:
            b = c.recv(n - len(out))
            if not b:
                raise ConnectionError("HubComm: peer closed")
            out += b
        return bytes(out)

    def _send_msg(self, c, data: bytes):
        c.sendall(self._struct.pack("<Q", len(data)) + data)

    def _recv_msg(self, c):
        (n,) = self._struct.unpack("<Q", self._recv(c, 8))
        return self._recv(c, n)

    def allgather(self, data: bytes) -> list:
        if self.nranks == 1:
            return [data]
        if self.rank == 0:
            parts = [data] + [self._recv_msg(self.peers[r]) for r in range(1, self.nranks)]
            blob = b"".join(self._struct.pack("<Q", len(p)) + p for p in parts)
            for r in range(1, self.nranks):
                self._send_msg(self.peers[r], blob)
        else:
            self._send_msg(self.peers[0], data)
            blob = self._recv_msg(self.peers[0])
            parts, o = [], 0
            while o < len(blob):
                (n,) = self._struct.unpack_from("<Q", blob, o)
                parts.append(blob[o + 8:o + 8 + n])
                o += 8 + n
        return parts

    def allreduce(self, a: np.ndarray) -> np.ndarray:
        parts = self.allgather(np.ascontiguousarray(a, dtype=np.float64).tobytes())
        s = np.frombuffer(parts[0], dtype=np.float64).copy()
        for p in parts[1:]:
            s += np.frombuffer(p, dtype=np.float64)
        return s

    def barrier(self):
        self.allgather(b"")

    def close(self):
        for c in self.peers.values():
            c.close()
        self.peers = {}

    def _allreduce_cb(self, buf, n, _user):
        try:
            a = np.ctypeslib.as_array(buf, shape=(n,))
            a[:] = self.allreduce(a)
            return 0
        except Exception:  # noqa: BLE001 - reported to the C side as a status
            return 1

    def _allgather_cb(self, send, recv, nbytes, _user):
        try:
            data = C.string_at(send, nbytes) if nbytes else b""
            parts = self.allgather(data)
            C.memmove(recv, b"".join(parts), nbytes * self.nranks)
            return 0
        except Exception:  # noqa: BLE001
            return 1


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

    @staticmethod
    def p2p_unique_id() -> bytes:
        """Name of a new peer-memory communicator (made on rank 0, distributed by the caller)."""
        buf = C.create_string_buffer(128)
        _check(load_library().ssp_p2p_unique_id(buf))
        return buf.raw

    def attach_p2p(self, nranks: int, rank: int, uid: bytes):
        """Peer-memory communicator (ssp_ctx_attach_p2p): IPC-shared device inboxes, no RCCL; several
        ranks may share one device.  Collective."""
        _check(self.lib.ssp_ctx_attach_p2p(self.handle, nranks, rank, uid))

    def set_comm_timeout(self, seconds: float):
        """Deadline of every wait that depends on other ranks (SSP_COMM_TIMEOUT_S)."""
        _check(self.lib.ssp_ctx_set_comm_timeout(self.handle, float(seconds)))

    def set_exact_max(self, n: int):
        """Vectors of at most n local elements use the reference's arithmetic bit for bit: sequential
        dots, no fused multiply-adds (ssp_ctx_set_exact_max; default 2048, 0 = off)."""
        _check(self.lib.ssp_ctx_set_exact_max(self.handle, int(n)))

    def debug_stall(self, ms: float):
        """Test harness: holds the stream for ms milliseconds (sspx_debug_stall)."""
        _check(self.lib.sspx_debug_stall(self.handle, float(ms)))

    def allgather_bytes(self, data: bytes) -> list:
        """Every rank's `data` (equal lengths), rank order, over the attached communicator."""
        nr = self.lib.ssp_ctx_nranks(self.handle)
        send = C.create_string_buffer(data, len(data))
        recv = C.create_string_buffer(len(data) * nr)
        _check(self.lib.ssp_allgather_host(self.handle, send, recv, len(data)))
        return [recv.raw[r * len(data):(r + 1) * len(data)] for r in range(nr)]

    def barrier(self):
        """Device-ordered barrier: a one-element allreduce on the context stream, then a sync."""
        if not hasattr(self, "_barrier_buf"):
            self._barrier_buf = self.alloc(1)
        _check(self.lib.ssp_allreduce_sum(self.handle, self._barrier_buf.ptr, 1))
        self.synchronize()

    # -- ledger (HIP-event kernel times + algorithmic bytes per operation) --------------------------
    def attach_host_comm(self, comm):
        """Reductions over ranks through host callbacks (e.g. gloo) instead of RCCL."""
        self._host_comm = comm  # keep the ctypes callbacks alive
        _check(self.lib.ssp_ctx_attach_host_comm(self.handle, comm.nranks, comm.rank, comm.allreduce_cb,
                                                  comm.allgather_cb, None))

    def ledger_enable(self, on: bool = True):
        _check(self.lib.ssp_ledger_enable(self.handle, int(on)))

    def ledger_reset(self):
        _check(self.lib.ssp_ledger_reset(self.handle))

    def ledger_reserve(self, n_events: int):
        """Pre-create HIP events for a ledger of n_events / 2 ops (none created while it records)."""
        _check(self.lib.ssp_ledger_reserve(self.handle, int(n_events)))

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

    def gemm_outer_set(self, alphas: np.ndarray, xx: Sequence[DeviceVector], yy: Sequence[DeviceVector]):
        """yy[j] = sum_i alphas[i, j] xx[i] (fill(0) + gemm_outer in one pass)."""
        alphas = np.ascontiguousarray(alphas, dtype=np.float64).reshape(len(xx), len(yy))
        n = yy[0].n if yy else 0
        _check(self.lib.ssp_gemm_outer_set(self.handle, _dptr(alphas), _ptrs(xx), len(xx), _ptrs(yy), len(yy), n))

    def axpy_inner(self, c: Sequence[float], x: DeviceVector, yy: Sequence[DeviceVector], z: DeviceVector) -> np.ndarray:
        """yy[j] += c[j] x, then returns <yy[j], z> (fused MGS step)."""
        cc = np.ascontiguousarray(c, dtype=np.float64)
        out = np.zeros(max_(len(yy)))
        _check(self.lib.ssp_axpy_inner(self.handle, _dptr(cc), x.ptr, _ptrs(yy), len(yy), z.ptr, x.n, _dptr(out)))
        return out[:len(yy)]

    def scal_inner(self, alpha: float, x: DeviceVector, yy: Sequence[DeviceVector]) -> np.ndarray:
        """x *= alpha, then returns <x, yy[j]> (fused orthonormalisation step)."""
        out = np.zeros(max_(len(yy)))
        _check(self.lib.ssp_scal_inner(self.handle, float(alpha), x.ptr, _ptrs(yy), len(yy), x.n, _dptr(out)))
        return out[:len(yy)]

    def axpy_norm(self, c: Sequence[float], x: DeviceVector, yy: Sequence[DeviceVector]) -> float:
        """yy[j] += c[j] x, then returns <yy[0], yy[0]> (fused orthonormalisation step)."""
        cc = np.ascontiguousarray(c, dtype=np.float64)
        out = np.zeros(1)
        _check(self.lib.ssp_axpy_norm(self.handle, _dptr(cc), x.ptr, _ptrs(yy), len(yy), x.n, _dptr(out)))
        return float(out[0])

    def axpy_gram(self, c: Sequence[float], x: DeviceVector, xs: float, yy: Sequence[DeviceVector],
                  store_x: bool = True) -> np.ndarray:
        """x_s = x * xs (stored when store_x), yy[j] += c[j] x_s, then returns <yy[0], yy[j]> (one-pass
        orthonormalisation step with the next vector's Gram row)."""
        cc = np.ascontiguousarray(c, dtype=np.float64)
        out = np.zeros(max_(len(yy)))
        _check(self.lib.ssp_axpy_gram(self.handle, _dptr(cc), x.ptr, float(xs), int(store_x), _ptrs(yy), len(yy),
                                      x.n, _dptr(out)))
        return out[:len(yy)]

    def transform_gram(self, t: np.ndarray, xx: Sequence[DeviceVector], xs: Sequence[float] = None,
                       gram: bool = True):
        """xx[j] <- sum_i t[i, j] xs[i] xx[i] in place (ssp_transform_gram); returns the m x m Gram
        matrix of the new vectors (None when gram is False)."""
        m = len(xx)
        tt = np.ascontiguousarray(t, dtype=np.float64).reshape(m, m)
        sx = None if xs is None else np.ascontiguousarray(xs, dtype=np.float64)
        g = np.zeros((m, m)) if gram else None
        _check(self.lib.ssp_transform_gram(self.handle, _dptr(tt), _ptrs(xx), None if sx is None else _dptr(sx), m,
                                           xx[0].n if m else 0, None if g is None else _dptr(g)))
        return g

    def transform_norms(self, t: np.ndarray, xx: Sequence[DeviceVector], xs: Sequence[float] = None) -> np.ndarray:
        """The same transform; returns the self-dots of the new vectors, formed in the same pass."""
        m = len(xx)
        tt = np.ascontiguousarray(t, dtype=np.float64).reshape(m, m)
        sx = None if xs is None else np.ascontiguousarray(xs, dtype=np.float64)
        out = np.zeros(max(1, m))
        _check(self.lib.ssp_transform_norms(self.handle, _dptr(tt), _ptrs(xx), None if sx is None else _dptr(sx), m,
                                            xx[0].n if m else 0, _dptr(out)))
        return out[:m]

    def axpy_pairs_norm(self, c: Sequence[float], xx: Sequence[DeviceVector], yy: Sequence[DeviceVector],
                        xs: Sequence[float] = None, ys: Sequence[float] = None) -> np.ndarray:
        """yy[j] = ys[j] yy[j] + c[j] xs[j] xx[j], then returns <yy[j], yy[j]> (residuals and their norms)."""
        cc = np.ascontiguousarray(c, dtype=np.float64)
        sx = None if xs is None else np.ascontiguousarray(xs, dtype=np.float64)
        sy = None if ys is None else np.ascontiguousarray(ys, dtype=np.float64)
        out = np.zeros(max_(len(yy)))
        _check(self.lib.ssp_axpy_pairs_norm(self.handle, _dptr(cc), _ptrs(xx), None if sx is None else _dptr(sx),
                                            _ptrs(yy), None if sy is None else _dptr(sy), len(yy),
                                            yy[0].n if yy else 0, _dptr(out)))
        return out[:len(yy)]

    def precondition(self, aa: Sequence[DeviceVector], d: DeviceVector, shift: Sequence[float]):
        sh = np.ascontiguousarray(shift, dtype=np.float64)
        _check(self.lib.ssp_precondition(self.handle, _ptrs(aa), len(aa), d.ptr, _dptr(sh), d.n))

    def precondition_norms(self, aa: Sequence[DeviceVector], d: DeviceVector, shift: Sequence[float]) -> np.ndarray:
        """ssp_precondition plus the self-dots of the results, formed in the same pass."""
        sh = np.ascontiguousarray(shift, dtype=np.float64)
        out = np.zeros(max(1, len(aa)))
        _check(self.lib.ssp_precondition_norms(self.handle, _ptrs(aa), len(aa), d.ptr, _dptr(sh), d.n, _dptr(out)))
        return out[: len(aa)]

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

    def sparse_axpy_batch(self, ps: Sequence[dict], xx: Sequence[DeviceVector], offset: int = 0):
        """xx[k] += p_k for each sparse vector p_k (ssp_sparse_axpy_batch: one launch)."""
        ptr, idx, val = self._pack_sparse(ps)
        n = xx[0].n if xx else 0
        _check(self.lib.ssp_sparse_axpy_batch(self.handle, len(ps), _zptr(ptr), _zptr(idx), _dptr(val), _ptrs(xx), n,
                                              offset))

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

    def construct_solution(self, palphas: np.ndarray, ps: Sequence[dict], alphas: np.ndarray,
                           xx: Sequence[DeviceVector], yy: Sequence[DeviceVector], offset: int = 0):
        """yy[j] = sum_i palphas[i, j] p_i + sum_s alphas[s, j] xx[s] (fill(0) + sparse and dense
        gemm_outer in one pass, reference construct_solution)."""
        m = len(yy)
        pa = np.ascontiguousarray(palphas, dtype=np.float64).reshape(len(ps), m)
        al = np.ascontiguousarray(alphas, dtype=np.float64).reshape(len(xx), m)
        ptr, idx, val = self._pack_sparse(ps)
        n = yy[0].n if m else 0
        _check(self.lib.ssp_construct_solution(self.handle, _dptr(pa), _zptr(ptr), _zptr(idx), _dptr(val), len(ps),
                                               _dptr(al), _ptrs(xx), len(xx), _ptrs(yy), m, n, offset))

    def gemm_outer_sparse(self, alphas: np.ndarray, ps: Sequence[dict], yy: Sequence[DeviceVector], offset: int = 0):
        ptr, idx, val = self._pack_sparse(ps)
        alphas = np.ascontiguousarray(alphas, dtype=np.float64)
        k, m = len(ps), len(yy)
        assert alphas.shape == (k, m)
        n = yy[0].n if m else 0
        _check(self.lib.ssp_gemm_outer_sparse(self.handle, _dptr(alphas), _zptr(ptr), _zptr(idx), _dptr(val), k,
                                              _ptrs(yy), m, n, offset))

    # -- deferred scal (include/subspace_hip.h *_scaled): each operand with a pending scale ---------
    @staticmethod
    def _scales(s, cnt):
        return np.ascontiguousarray(np.ones(cnt) if s is None else s, dtype=np.float64).reshape(cnt)

    def scal_copy(self, alpha: float, x: DeviceVector, y: DeviceVector):
        _check(self.lib.ssp_scal_copy(self.handle, float(alpha), x.ptr, y.ptr, x.n))

    def axpy_scaled(self, alpha: float, x: DeviceVector, xs: float, y: DeviceVector, ys: float):
        _check(self.lib.ssp_axpy_scaled(self.handle, float(alpha), x.ptr, float(xs), y.ptr, float(ys), y.n))

    def dot_scaled(self, x: DeviceVector, xs: float, y: DeviceVector, ys: float) -> float:
        out = np.zeros(1)
        _check(self.lib.ssp_dot_scaled(self.handle, x.ptr, float(xs), y.ptr, float(ys), x.n, _dptr(out)))
        return float(out[0])

    def gemm_inner_scaled(self, xx, xs, yy, ys) -> np.ndarray:
        m, k = len(xx), len(yy)
        out = np.zeros((m, k))
        a, b = self._scales(xs, m), self._scales(ys, k)
        n = xx[0].n if m else 0
        _check(self.lib.ssp_gemm_inner_scaled(self.handle, _ptrs(xx), _dptr(a), m, _ptrs(yy), _dptr(b), k, n,
                                              _dptr(out)))
        return out

    def gemm_outer_scaled(self, alphas, xx, xs, yy, ys):
        alphas = np.ascontiguousarray(alphas, dtype=np.float64).reshape(len(xx), len(yy))
        a, b = self._scales(xs, len(xx)), self._scales(ys, len(yy))
        n = yy[0].n if yy else 0
        _check(self.lib.ssp_gemm_outer_scaled(self.handle, _dptr(alphas), _ptrs(xx), _dptr(a), len(xx), _ptrs(yy),
                                              _dptr(b), len(yy), n))

    def gemm_outer_set_scaled(self, alphas, xx, xs, yy):
        alphas = np.ascontiguousarray(alphas, dtype=np.float64).reshape(len(xx), len(yy))
        a = self._scales(xs, len(xx))
        n = yy[0].n if yy else 0
        _check(self.lib.ssp_gemm_outer_set_scaled(self.handle, _dptr(alphas), _ptrs(xx), _dptr(a), len(xx),
                                                  _ptrs(yy), len(yy), n))

    def gemm_inner_sparse_scaled(self, xx, xs, ps, offset: int = 0) -> np.ndarray:
        ptr, idx, val = self._pack_sparse(ps)
        m, k = len(xx), len(ps)
        out = np.zeros((m, k))
        a = self._scales(xs, m)
        n = xx[0].n if m else 0
        _check(self.lib.ssp_gemm_inner_sparse_scaled(self.handle, _ptrs(xx), _dptr(a), m, n, offset, _zptr(ptr),
                                                     _zptr(idx), _dptr(val), k, _dptr(out)))
        return out

    def gemm_inner_sparse_begin(self, xx, ps, xs=None, offset: int = 0) -> tuple:
        """Queues gemm_inner_sparse(xx, ps); gemm_inner_sparse_end() delivers it."""
        ptr, idx, val = self._pack_sparse(ps)
        m, k = len(xx), len(ps)
        a = self._scales(xs, m)
        n = xx[0].n if m else 0
        _check(self.lib.ssp_gemm_inner_sparse_begin(self.handle, _ptrs(xx), _dptr(a), m, n, offset, _zptr(ptr),
                                                    _zptr(idx), _dptr(val), k))
        return (m, k)

    def gemm_inner_sparse_end(self, shape: tuple) -> np.ndarray:
        out = np.zeros(shape)
        _check(self.lib.ssp_gemm_inner_sparse_end(self.handle, _dptr(out)))
        return out

    def construct_solution_scaled(self, palphas, ps, alphas, xx, xs, yy, offset: int = 0):
        m = len(yy)
        pa = np.ascontiguousarray(palphas, dtype=np.float64).reshape(len(ps), m)
        al = np.ascontiguousarray(alphas, dtype=np.float64).reshape(len(xx), m)
        a = self._scales(xs, len(xx))
        ptr, idx, val = self._pack_sparse(ps)
        n = yy[0].n if m else 0
        _check(self.lib.ssp_construct_solution_scaled(self.handle, _dptr(pa), _zptr(ptr), _zptr(idx), _dptr(val),
                                                      len(ps), _dptr(al), _ptrs(xx), _dptr(a), len(xx), _ptrs(yy), m,
                                                      n, offset))

    def block_update(self, palphas, ps, alphas, xx, xs, yy, ys, offset: int = 0):
        """yy[j] = ys[j] yy[j] + sum_i palphas[i, j] p_i + sum_s alphas[s, j] xs[s] xx[s]."""
        m = len(yy)
        pa = np.ascontiguousarray(palphas, dtype=np.float64).reshape(len(ps), m)
        al = np.ascontiguousarray(alphas, dtype=np.float64).reshape(len(xx), m)
        a, b = self._scales(xs, len(xx)), self._scales(ys, m)
        ptr, idx, val = self._pack_sparse(ps)
        n = yy[0].n if m else 0
        _check(self.lib.ssp_block_update(self.handle, _dptr(pa), _zptr(ptr), _zptr(idx), _dptr(val), len(ps),
                                         _dptr(al), _ptrs(xx), _dptr(a), len(xx), _ptrs(yy), _dptr(b), m, n, offset))

    def synth_action_scaled(self, xx, xs, yy, spec, offset: int = 0):
        a = self._scales(xs, len(xx))
        _check(self.lib.sspx_synth_action_scaled(self.handle, C.byref(spec), _ptrs(xx), _dptr(a), _ptrs(yy), len(xx),
                                                 xx[0].n, offset))

    # -- synthetic problem (harness) ------------------------------------------------------------
    def synthetic_action(self, xx, yy, rho: float, rank: int, seed: int, offset: int = 0):
        _check(self.lib.sspx_synthetic_action(self.handle, _ptrs(xx), _ptrs(yy), len(xx), xx[0].n, offset, rho, rank,
                                              seed))

    def synthetic_diagonal(self, d: DeviceVector, rho: float, rank: int, offset: int = 0):
        _check(self.lib.sspx_synthetic_diagonal(self.handle, d.ptr, d.n, offset, rho, rank))

    def synth_action(self, xx, yy, spec, offset: int = 0):
        """Any synthetic family; spec = itsolv_hbm.Synth."""
        _check(self.lib.sspx_synth_action(self.handle, C.byref(spec), _ptrs(xx), _ptrs(yy), len(xx), xx[0].n,
                                          offset))

    def synth_diagonal(self, d: DeviceVector, spec, offset: int = 0):
        _check(self.lib.sspx_synth_diagonal(self.handle, C.byref(spec), d.ptr, d.n, offset))

    def fill_random(self, x: DeviceVector, seed: int, vec: int, offset: int = 0):
        _check(self.lib.sspx_fill_random(self.handle, x.ptr, x.n, offset, seed, vec))


def max_(n: int) -> int:
    return n if n > 0 else 1


def device_count() -> int:
    return load_library().ssp_device_count()
