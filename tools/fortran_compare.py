"""Probe: every case of tests/fortran_cases.py on the GPU library and on the CPU emulation (own
process), listing each case whose iteration count or values differ."""
import json, os, subprocess, sys, tempfile
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import fortran_cases as fc  # noqa: E402

out = os.path.join(tempfile.mkdtemp(), "emul.json")
subprocess.run([sys.executable, os.path.join(HERE, "..", "tests", "fortran_cases.py"), "--emul", out], check=True,
               capture_output=True)
cpu = json.load(open(out))
gpu = fc.run_all(fc.load(fc.LIB_GPU))
for k, g in gpu.items():
    c = cpu[k]
    diffs = {}
    if g.get("iterations") != c.get("iterations"):
        diffs["iterations"] = (g.get("iterations"), c.get("iterations"))
    for f in ("eigenvalues", "x", "solution", "errors"):
        if f in g:
            d = float(np.max(np.abs(np.array(g[f]) - np.array(c[f])))) if len(g[f]) else 0.0
            if d > 1e-10 or f == "errors" and diffs:
                diffs[f] = (d, g[f][:4], c[f][:4])
    if diffs:
        print(k, diffs)
print("compared", len(gpu))
