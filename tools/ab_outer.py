#!/usr/bin/env python3
"""Same-box A/B of gemm_outer (48 -> 8, N = 1e8) between two builds of libsubspace_hip.so
(raw ctypes, HIP-event ledger).  usage: python tools/ab_outer.py LIB [reps]"""
import ctypes as C
import sys

lib = C.CDLL(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
P, PD = C.c_void_p, C.POINTER(C.c_double)
ctx = P()
assert lib.ssp_ctx_create(0, C.byref(ctx)) == 0
n, m, k = 100_000_000, 8, 48
vec = []
for i in range(m + k):
    p = PD()
    assert lib.ssp_alloc(ctx, C.c_size_t(n), C.byref(p)) == 0
    lib.sspx_fill_random(ctx, p, C.c_size_t(n), C.c_size_t(0), C.c_ulonglong(7), C.c_ulonglong(i))
    vec.append(p)
al = (C.c_double * (k * m))(*[1e-3 * (i % 17) for i in range(k * m)])
xs = (PD * k)(*vec[m:])
ys = (PD * m)(*vec[:m])
lib.ssp_gemm_outer(ctx, al, xs, k, ys, m, C.c_size_t(n))
lib.ssp_synchronize(ctx)
for rnd in range(3):
    lib.ssp_ledger_reset(ctx)
    lib.ssp_ledger_enable(ctx, 1)
    for _ in range(reps):
        assert lib.ssp_gemm_outer(ctx, al, xs, k, ys, m, C.c_size_t(n)) == 0
    lib.ssp_synchronize(ctx)
    lib.ssp_ledger_enable(ctx, 0)
    name, calls, ms, by = C.c_char_p(), C.c_longlong(), C.c_double(), C.c_double()
    for i in range(lib.ssp_ledger_count(ctx)):
        lib.ssp_ledger_entry(ctx, i, C.byref(name), C.byref(calls), C.byref(ms), C.byref(by))
        if name.value == b"gemm_outer":
            print(f"{sys.argv[1].split('/')[-1]:28s} gemm_outer 48->8 {by.value / (ms.value / 1e3) / 1e9:8.1f} GB/s",
                  flush=True)
