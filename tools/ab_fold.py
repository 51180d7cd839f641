#!/usr/bin/env python3
"""Same-process A/B of the fused reduction tail's hand-off (ssp_internal.h fold_tail): the library
build (write-through sc1 form) against a build with -DSSP_FOLD_RELACQ (release / acq_rel arrivals,
agent-scope acquire fence).  Host-visible latency per call at small N (the tail dominates) and
HIP-event kernel time at N = 1e8, on the SAME vectors, rounds interleaved; results compared bitwise.
usage: python tools/ab_fold.py LIB_A LIB_B"""
import ctypes as C
import sys
import time

P, PD = C.c_void_p, C.POINTER(C.c_double)
paths = sys.argv[1:]
libs = [C.CDLL(p) for p in paths]
ctxs = []
for lib in libs:
    c = P()
    assert lib.ssp_ctx_create(0, C.byref(c)) == 0
    ctxs.append(c)
l0, c0 = libs[0], ctxs[0]


def alloc(n, count, seed):
    out = []
    for i in range(count):
        p = PD()
        assert l0.ssp_alloc(c0, C.c_size_t(n), C.byref(p)) == 0
        l0.sspx_fill_random(c0, p, C.c_size_t(n), C.c_size_t(0), C.c_ulonglong(seed), C.c_ulonglong(i))
        out.append(p)
    l0.ssp_synchronize(c0)
    return out


def ledger_ms(lib, ctx, name):
    nm, calls, ms, by = C.c_char_p(), C.c_longlong(), C.c_double(), C.c_double()
    for i in range(lib.ssp_ledger_count(ctx)):
        lib.ssp_ledger_entry(ctx, i, C.byref(nm), C.byref(calls), C.byref(ms), C.byref(by))
        if nm.value == name:
            return ms.value / calls.value
    return float("nan")


results = {}
for n in (1000, 100_000_000):
    vec = alloc(n, 56, 11)
    xs, ys = (PD * 8)(*vec[:8]), (PD * 48)(*vec[8:])
    out = (C.c_double * (8 * 48))()
    d = C.c_double()
    ref = {}
    for rnd in range(4):
        for path, lib, ctx in zip(paths, libs, ctxs):
            tag = path.split("/")[-2]
            # correctness: bitwise identical across builds
            assert lib.ssp_dot(ctx, vec[0], vec[1], C.c_size_t(n), C.byref(d)) == 0
            assert lib.ssp_gemm_inner(ctx, xs, 8, ys, 48, C.c_size_t(n), out) == 0
            key = (n, "dot")
            ref.setdefault(key, d.value)
            ref.setdefault((n, "gi"), list(out))
            same = ref[key] == d.value and ref[(n, "gi")] == list(out)
            if n <= 1000:
                reps = 5000
                t0 = time.perf_counter()
                for _ in range(reps):
                    lib.ssp_dot(ctx, vec[0], vec[1], C.c_size_t(n), C.byref(d))
                t_dot = (time.perf_counter() - t0) / reps * 1e6
                t0 = time.perf_counter()
                for _ in range(reps // 2):
                    lib.ssp_gemm_inner(ctx, xs, 8, ys, 48, C.c_size_t(n), out)
                t_gi = (time.perf_counter() - t0) / (reps // 2) * 1e6
                line = f"n={n:>9} round {rnd} {tag:14s} dot {t_dot:7.2f} us/call  gemm_inner 8x48 {t_gi:7.2f} us/call"
            else:
                lib.ssp_ledger_reset(ctx)
                lib.ssp_ledger_enable(ctx, 1)
                for _ in range(20):
                    lib.ssp_dot(ctx, vec[0], vec[1], C.c_size_t(n), C.byref(d))
                for _ in range(5):
                    lib.ssp_gemm_inner(ctx, xs, 8, ys, 48, C.c_size_t(n), out)
                lib.ssp_synchronize(ctx)
                lib.ssp_ledger_enable(ctx, 0)
                t_dot, t_gi = ledger_ms(lib, ctx, b"dot"), ledger_ms(lib, ctx, b"gemm_inner")
                line = f"n={n:>9} round {rnd} {tag:14s} dot {t_dot * 1e3:9.1f} us  gemm_inner 8x48 {t_gi * 1e3:9.1f} us"
            results.setdefault((n, tag), []).append((t_dot, t_gi))
            print(line + f"  bitwise-same {same}", flush=True)
    for p in vec:
        l0.ssp_free(c0, p)
print("medians:")
for (n, tag), v in sorted(results.items()):
    a = sorted(x[0] for x in v)
    b = sorted(x[1] for x in v)
    print(f"n={n:>9} {tag:14s} dot {a[len(a) // 2]:.4g}  gemm_inner {b[len(b) // 2]:.4g}")
