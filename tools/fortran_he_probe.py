"""Probe: the he (n = 4) Davidson loop of tests/fortran/itsolv_f_checks.F90 through a C API library
(argv[2]: the product libitsolv_hbm.so or the emulation), printing errors after every call."""
import ctypes, numpy as np, sys
import os; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests'))
import fortran_cases as fc
L = ctypes.CDLL(sys.argv[2])
D=ctypes.POINTER(ctypes.c_double); S=ctypes.c_size_t
h = fc.hamiltonian('he'); n=4; nroot=int(sys.argv[1])
rb, re_ = S(0), S(0)
L.IterativeSolverLinearEigensystemInitialize.argtypes=[S,S,ctypes.POINTER(S),ctypes.POINTER(S),ctypes.c_double,ctypes.c_double,ctypes.c_int,ctypes.c_int,ctypes.c_char_p,ctypes.c_int64,ctypes.c_char_p,ctypes.c_char_p]
L.IterativeSolverLinearEigensystemInitialize(n,nroot,ctypes.byref(rb),ctypes.byref(re_),1e-8,1e50,1,0,b"",0,b"",b"")
d = np.diag(h).copy(); c = np.zeros((nroot,n))
dd=d.copy()
for k in range(nroot):
    i=int(np.argmin(dd)); c[k,i]=1; dd[i]=np.inf
for it in range(10):
    g = c @ h.T
    nw = L.IterativeSolverAddVector(S(nroot), c.ctypes.data_as(D), g.ctypes.data_as(D), 1)
    e = np.zeros(nroot); L.IterativeSolverErrors(e.ctypes.data_as(D))
    ev = np.zeros(nroot); L.IterativeSolverEigenvalues(ev.ctypes.data_as(D))
    print('add', it, nw, e, ev)
    if nw==0: break
    ws = np.zeros(nroot); L.IterativeSolverWorkingSetEigenvalues(ws.ctypes.data_as(D))
    for k in range(nw): g[k] = -g[k]/(d+1e-12-ws[k])
    nw = L.IterativeSolverEndIteration(S(nroot), c.ctypes.data_as(D), g.ctypes.data_as(D), 1)
    print('end', it, nw)
    if nw==0: break

import json
