"""Diagnostic: one rank of a two-rank RCCL communicator joins alone (SSP_COMM_TRACE stage lines on
stderr), with a short deadline.  Prints the outcome and how long it took."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "iterative-solver_amd"))
import subspace_hip as sh  # noqa: E402

c = sh.Context(0)
c.set_comm_timeout(float(sys.argv[1]) if len(sys.argv) > 1 else 8.0)
t0 = time.time()
try:
    c.attach_comm(2, 0, sh.Context.unique_id())
    print("ATTACHED", flush=True)
except sh.SspError as e:
    print(f"FAILED {e.code} {time.time() - t0:.2f} {e}", flush=True)
print("closing", flush=True)
c.close()
print("closed", time.time() - t0, flush=True)
