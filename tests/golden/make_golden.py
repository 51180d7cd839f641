"""Generates tests/golden/*.json / *.npz — golden vectors pinning the oracle.

Inputs are the reference's own fixtures (examples/{he,hf,bh}.hamiltonian, copied here as data) and
seeded synthetic vectors.  Expected outputs are computed INDEPENDENTLY of the oracle (numpy/LAPACK
eigensolvers, numpy dot products in extended-precision-free float64, lexicographic sorts), so the
oracle's restatement of the reference loops is checked against them, not against itself.

Reference anchors recorded here:
  * FCI ground state of he: -2.878990189612 (reference examples/he.molpro/run/5.molpro/5.out:408)
  * degeneracy split 1e-8 * i applied to bh/hf as reference test_LinearEigensystem.cpp:347-352 does
Run: python tests/golden/make_golden.py
"""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def load_hamiltonian(name, split=0.0):
    t = open(os.path.join(HERE, name + ".hamiltonian")).read().split()
    n = int(t[0])
    h = np.array(t[1 : 1 + n * n], dtype=np.float64).reshape(n, n)
    h = h + np.diag(split * np.arange(n))
    return h


def main():
    out = {}
    for name, split in (("he", 0.0), ("hf", 1e-8), ("bh", 1e-8)):
        h = load_hamiltonian(name, split)
        w = np.linalg.eigvalsh(h)
        out[name] = {"n": int(h.shape[0]), "degeneracy_split": split, "eigenvalues": [float(x) for x in w]}
    out["he"]["fci_energy"] = -2.878990189612
    # reference test_LinearEigensystem.cpp:41-51: H = 1 off-diagonal, H_ii = i * param (n = 100, param = 1)
    n = 100
    h = np.ones((n, n)) + np.diag(np.arange(n) - 1.0)
    out["ones_100"] = {"n": n, "eigenvalues": [float(x) for x in np.linalg.eigvalsh(h)[:10]]}
    # reference test_rayleigh_quotient.cpp:37-42: H_ij = (i == j) ? i + 1 + rho : rho, n = 4, rho = 0.01
    n, rho = 4, 0.01
    h = np.full((n, n), rho) + np.diag(np.arange(n) + 1.0)
    w, v = np.linalg.eigh(h)
    out["rayleigh_4"] = {"n": n, "rho": rho, "eigenvalues": [float(x) for x in w],
                         "lowest_eigenvector_abs": [float(abs(x)) for x in v[:, 0]]}
    # reference test_simplified.cpp:24 / examples/ExampleProblem.h:8: i == j ? i + 1 : 0.001 * ((i + j) % n)
    n = 20
    i, j = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    h = np.where(i == j, i + 1.0, 0.001 * ((i + j) % n))
    out["example_20"] = {"n": n, "eigenvalues": [float(x) for x in np.linalg.eigvals(h).real[np.argsort(np.linalg.eigvals(h).real)][:4]]}
    with open(os.path.join(HERE, "eigen_golden.json"), "w") as f:
        json.dump(out, f, indent=1)

    # Handler-op golden vectors: seeded inputs, expected outputs from numpy.
    rng = np.random.default_rng(20251015)
    n, m, k = 1003, 5, 7
    xs = rng.uniform(-1, 1, (m, n))
    ys = rng.uniform(-1, 1, (k, n))
    alphas = rng.uniform(-1, 1, (k, m))
    diag = 1.0 + np.arange(n) + 0.3
    shift = rng.uniform(-2, 0, m)
    sel = np.round(rng.uniform(-50, 50, n))  # many ties: exercises the larger-index-wins rule
    gi = xs @ ys.T  # gemm_inner(xs, ys)
    go = xs.copy()
    for j in range(m):  # gemm_outer(alphas (k x m), ys -> xs)
        for i in range(k):
            go[j] = go[j] + alphas[i, j] * ys[i]
    prec = xs / (diag[None, :] - shift[:, None] + 1e-15)

    def lex_select(v, nsel):
        order = sorted(range(len(v)), key=lambda t: (v[t], t), reverse=True)[:nsel]
        return sorted(order)

    sel_min = lex_select(-sel, 9)
    sel_max_abs = lex_select(np.abs(sel), 9)
    np.savez(os.path.join(HERE, "ops_golden.npz"), xs=xs, ys=ys, alphas=alphas, diag=diag, shift=shift, sel=sel,
             gemm_inner=gi, gemm_outer=go, precondition=prec, select_min_idx=np.array(sel_min),
             select_max_abs_idx=np.array(sel_max_abs))


if __name__ == "__main__":
    main()
