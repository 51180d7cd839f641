"""Runs bench.py (or its RCCL-id rendezvous) over the host-memory emulation of the device ABI
(oracle/ssp_emul.cpp, test infrastructure), so that the driver's multi-rank launch
(`torch.distributed.run --nproc-per-node 8 ... bench.py --gpus 8`) can be rehearsed on CPU with the
world size of the 8-GPU scaling run.  The GPU runs of bench.py are tests/test_bench.py (-m gpu).

  python -m torch.distributed.run --nproc-per-node 8 ... tests/bench_emul.py bench <bench args>
  RANK=r WORLD_SIZE=w MASTER_ADDR=a MASTER_PORT=p python tests/bench_emul.py uid
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "iterative-solver_amd")):
    sys.path.insert(0, p)

import subspace_hip as sh  # noqa: E402

sh.LIB_PATH = os.path.join(ROOT, "oracle", "build", "libssp_emul.so")
import itsolv_hbm as ih  # noqa: E402

ih.LIB_PATH = os.path.join(ROOT, "oracle", "build", "libitsolv_emul.so")

import bench  # noqa: E402

if __name__ == "__main__":
    mode = sys.argv[1]
    if mode == "bench":
        sys.argv = ["bench.py"] + sys.argv[2:]
        bench.main()
    elif mode == "uid":
        # rank 0's id must reach every rank unchanged (the emulation's own id is all zeros)
        sh.Context.unique_id = staticmethod(lambda: bytes(range(7, 7 + 128)))
        rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
        uid, path = bench.rendezvous_uid(rank, world, timeout=60.0)
        print("uid", rank, uid.hex(), flush=True)
        if path:  # rank 0 removes the file once every rank has reported (the test waits on all)
            import time

            time.sleep(2.0)
            os.remove(path)
    else:
        raise SystemExit(f"unknown mode {mode}")
