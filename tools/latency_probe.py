#!/usr/bin/env python3
"""Per-call latency of the C-ABI ops at small and shard-sized N (development tool).

Times many back-to-back calls from Python (ctypes) so the figure is host-visible latency per call:
launch + kernel + (for reductions) the second pass, the D2H of the result and the stream sync.
Usage: python tools/latency_probe.py [--rccl] [--out file.json]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "iterative-solver_amd"))
import subspace_hip as sh  # noqa: E402


def per_call(f, reps):
    f()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--rccl", action="store_true",
                    help="attach a one-rank RCCL communicator: reductions take the multi-rank path "
                         "(fold -> ncclAllReduce -> publish) instead of the fused host publish")
    ap.add_argument("--p2p", action="store_true",
                    help="attach a one-rank peer-memory communicator: fold -> k_p2p_allreduce (push, flag "
                         "wait, rank-order sum, host publish)")
    args = ap.parse_args()
    res = {}
    with sh.Context(0) as ctx:
        if args.rccl:
            ctx.attach_comm(1, 0, sh.Context.unique_id())
        if args.p2p:
            ctx.attach_p2p(1, 0, sh.Context.p2p_unique_id())
        for n in (1024, 1_000_000, 12_500_000):
            reps = 2000 if n <= 1_000_000 else 200
            x = [ctx.alloc(n) for _ in range(56)]
            for i, v in enumerate(x):
                ctx.fill_random(v, 1, i, 0)
            ctx.synchronize()
            r = {
                "fill (async)": per_call(lambda: ctx.fill(0.0, x[0]), reps),
                "fill + sync": per_call(lambda: (ctx.fill(0.0, x[0]), ctx.synchronize()), reps),
                "dot(x,x)": per_call(lambda: ctx.dot(x[1], x[1]), reps),
                "dot(x,y)": per_call(lambda: ctx.dot(x[1], x[2]), reps),
                "gemm_inner 8x48": per_call(lambda: ctx.gemm_inner(x[:8], x[8:56]), max(20, reps // 10)),
                "sync only": per_call(ctx.synchronize, reps),
                "barrier": per_call(ctx.barrier, reps),
            }
            res[str(n)] = {k: round(v, 2) for k, v in r.items()}
            print(n, json.dumps(res[str(n)]), flush=True)
            del x
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
