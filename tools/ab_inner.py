#!/usr/bin/env python3
"""Same-process A/B of gemm_inner (8 x 48, N = 1e8) between builds of libsubspace_hip.so on the SAME
vectors (raw ctypes, HIP-event ledger of each build; device pointers are process-wide, so the
vectors allocated through the first build serve every build).
usage: python tools/ab_inner.py LIB [LIB ...]"""
import ctypes as C
import sys

P, PD = C.c_void_p, C.POINTER(C.c_double)
paths = sys.argv[1:]
libs = [C.CDLL(p) for p in paths]
ctxs = []
for lib in libs:
    c = P()
    assert lib.ssp_ctx_create(0, C.byref(c)) == 0
    ctxs.append(c)
n, m, k = 100_000_000, 8, 48
l0, c0 = libs[0], ctxs[0]
vec = []
for i in range(m + k):
    p = PD()
    assert l0.ssp_alloc(c0, C.c_size_t(n), C.byref(p)) == 0
    l0.sspx_fill_random(c0, p, C.c_size_t(n), C.c_size_t(0), C.c_ulonglong(7), C.c_ulonglong(i))
    vec.append(p)
l0.ssp_synchronize(c0)
xs = (PD * m)(*vec[:m])
ys = (PD * k)(*vec[m:])
out = (C.c_double * (m * k))()
ref = None
for rnd in range(4):
    for path, lib, ctx in zip(paths, libs, ctxs):
        assert lib.ssp_gemm_inner(ctx, xs, m, ys, k, C.c_size_t(n), out) == 0
        if ref is None:
            ref = list(out)
        err = max(abs(a - b) for a, b in zip(out, ref))
        lib.ssp_ledger_reset(ctx)
        lib.ssp_ledger_enable(ctx, 1)
        for _ in range(10):
            assert lib.ssp_gemm_inner(ctx, xs, m, ys, k, C.c_size_t(n), out) == 0
        lib.ssp_synchronize(ctx)
        lib.ssp_ledger_enable(ctx, 0)
        name, calls, ms, by = C.c_char_p(), C.c_longlong(), C.c_double(), C.c_double()
        for i in range(lib.ssp_ledger_count(ctx)):
            lib.ssp_ledger_entry(ctx, i, C.byref(name), C.byref(calls), C.byref(ms), C.byref(by))
            if name.value == b"gemm_inner":
                print(f"round {rnd} {path.split('/')[-1]:12s} gemm_inner 8x48 {ms.value / calls.value:7.3f} ms "
                      f"{by.value / (ms.value / 1e3) / 1e9:8.1f} GB/s  max|diff| vs first build {err:.2e}", flush=True)
