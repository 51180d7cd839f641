import sys, numpy as np
sys.path[:0] = ["tests", ".", "oracle", "iterative-solver_amd"]
import rc_problems as rp
from test_reverse_comm import hylleraas_solver, cpu, gpu
for name in ["he", "bh", "hf"]:
    h, h0 = rp.rspt_problem(name)
    n = h0.size
    e_ref, ref = rp.loop_hylleraas(hylleraas_solver(cpu, n, "BFGS"), h, h0, optimize=True, precondition=False)
    s = hylleraas_solver(gpu, n, "BFGS")
    e_gpu, tr = rp.loop_hylleraas(s, h, h0, optimize=True, precondition=False)
    print(name, len(ref), len(tr), e_ref, e_gpu, e_ref - e_gpu)
    for k, (a, b) in enumerate(zip(tr, ref)):
        print("  step", k, a[0], b[0], np.max(np.abs(a[1] - b[1])), np.linalg.norm(b[1]))
    s.finalize()
