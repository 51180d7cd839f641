"""Independent numpy restatement of the reference's LinearEigensystemDavidson and NonLinearEquationsDIIS.

TEST INFRASTRUCTURE (only tests/ import it).  It shares no code with the product's host layer
(iterative-solver_amd/include/itsolv_hbm/{solvers,rspace,subspace,dense}.h) or with the C++ oracle
that compiles those headers over CPU handlers: it is a second, separate reading of the reference, in
numpy, so that a restatement error in the product's host C++ shows up as a disagreement between the
two (tests/test_davidson_independent.py).  Vectors are dense numpy arrays; the subspace matrices are
kept exactly as the reference keeps them (blocks computed when a vector enters the subspace, the
same transposes for the hermitian case), so the two implementations differ only in rounding
(numpy's summation order, LAPACK's dsyevd/dgeev for dsyev/Eigen::EigenSolver).

Followed, file:line under /root/reference/src/molpro/linalg/itsolv/:
  IterativeSolverTemplate.h:21-31 parameter_batches, :33-65 construct_solution, :95-117 update_errors /
      select_working_set, :140-166 add_vector, :176-187 add_p, :191-215 solution, :322-408 solve,
      :518-563 solve_and_generate_working_set
  LinearEigensystemDavidson.h:63-83 end_iteration, :106-113 set_value_errors, :186-192 construct_residual
  IterativeSolver.h:46-55 precondition_default
  propose_rspace.h:17-28 normalise, :39-256 dspace helpers, :271-300 append_overlap_with_r,
      :310-336 limit_qspace_size, :349-403 construct_dspace, :421-466 modified_gram_schmidt,
      :481-512 redundant_parameters, :553-624 propose_rspace
  DSpaceResetter.h:14-24 resize_qspace, :33-54 max_overlap_with_R, :72-145 DSpaceResetter
  subspace/XSpace.h:30-83 update_qspace_data, :86-134 D-space data, :136-151 copy_dspace_eqn_data,
      :176-205 update_dspace / update_pspace, :241-245 eraseq, :293-300 remove_data
  subspace/QSpace.h:77-116 QSpace::update (new vectors prepended, in order)
  subspace/SubspaceSolverLinEig.h:32-57 solve_eigenvalue
  helper-implementation.h:221-231 get_rank, :263-296 svd_system (hermitian), :318-543 eigenproblem
  util.h:70-100 construct_solutions / delete_parameters; array/util/select.h:28-55 select
  LinearEquationsDavidson.h:46-60 end_iteration, :170-181 construct_residual; XSpace.h:218-230
      add_rhs_equations, :273-276 update_rhs_with_pspace; SubspaceSolverLinEig.h:59-79
      solve_linear_equations; helper-implementation.h:555-614 solve_LinearEquations (incl. augmented Hessian)
  OptimizeBFGS.h:40-185 (Wolfe tests, cubic line search, two-loop BFGS update), OptimizeSD.h:37-95,
      subspace/SubspaceSolverOptBFGS.h / SubspaceSolverOptSD.h, Interpolate.cpp:51-66 cubic, :115-134
      minimize_cubic (Interpolate.h:46: analytic by default)
  NonLinearEquationsDIIS.h:52-83 least_important_vector, :86-102 add_vector, :103-119 end_iteration;
      subspace/SubspaceSolverDIIS.h:27-66; helper-implementation.h:619-669 solve_DIIS;
      XSpace.h:45-50 (action . action H for DIIS)
"""
from __future__ import annotations

import numpy as np

INT_MAX = 2**31 - 1
DBL_MAX = np.finfo(np.float64).max


# ---- dense helpers -------------------------------------------------------------------------------
def sym_eig_ascending(m):
    """dsyev: eigenpairs of a symmetric matrix (lower triangle), ascending (helper-implementation.h:122-158)."""
    return np.linalg.eigh(m, UPLO="L")


def svd_system_hermitian(m, threshold):
    """svd_system(hermitian=true, reduce_to_rank=false): the eigenpairs of m with value <= threshold,
    ascending (helper-implementation.h:263-283)."""
    if m.size == 0:
        return []
    w, v = sym_eig_ascending(m)
    return [(float(w[i]), v[:, i].copy()) for i in range(len(w)) if not w[i] > threshold]


def eigenproblem_hermitian(h, s, svd_threshold=1e-14):
    """helper-implementation.h:318-543 for hermitian = true: returns (eigenvalues, solutions as rows)."""
    dim = h.shape[0]
    if dim == 0:
        return np.zeros(0), np.zeros((0, 0))
    ev, vecs = sym_eig_ascending(s)
    rank = int(np.count_nonzero(ev >= svd_threshold * np.max(ev)))  # get_rank :221-231
    sv = ev[:rank]  # singularValues.head(rank): the head of dsyev's ascending order (:368)
    svmh = np.where(sv > 1e-14, 1.0 / np.sqrt(np.where(sv > 0, sv, 1.0)), 0.0)
    v = vecs[:, :rank]
    hbar = (svmh[:, None] * (v.T @ h @ v)) * svmh[None, :]
    w, y = np.linalg.eig(hbar)
    if np.linalg.norm(np.imag(w)) >= 1e-10:
        raise RuntimeError("complex subspace eigenvalues (not restated)")
    w, y = np.real(w), np.real(y)
    x = v @ (svmh[:, None] * y)  # back-transform before sorting (:394)
    order = np.argsort(w, kind="stable")  # selection sort, ties to the lower index (:409-428)
    w, x = w[order], x[:, order]
    for k in range(rank):  # sign: the largest |component| among the first Hbar.cols() positive
        maxcomp = 0
        for l in range(rank):
            if abs(x[l, k]) > abs(x[maxcomp, k]):
                maxcomp = l
        if x[maxcomp, k] < 0:
            x[:, k] = -x[:, k]
    return w, x.T.copy()


def select_smallest(values, n):
    """util::select(n, x, max=false): the n smallest values, ties to the larger index, returned in
    index order (array/util/select.h:28-55)."""
    idx = sorted(range(len(values)), key=lambda i: (values[i], -i))[:n]
    return sorted(idx)


def sym_overlap(vecs):
    """subspace::util::overlap(params, handler): lower triangle by dots, mirrored (subspace/util.h:55-62)."""
    n = len(vecs)
    m = np.zeros((n, n))
    for i in range(n):
        for j in range(i + 1):
            m[i, j] = m[j, i] = vecs[i] @ vecs[j]
    return m


def cross(left, right):
    """subspace::util::overlap(left, right, handler) = gemm_inner: (i, j) = <left_i, right_j>."""
    m = np.zeros((len(left), len(right)))
    for i, a in enumerate(left):
        for j, b in enumerate(right):
            m[i, j] = a @ b
    return m


# ---- problems ------------------------------------------------------------------------------------
class DenseProblem:
    """Problem<R> over a dense matrix (action = H x, diagonals, P space of unit vectors)."""

    def __init__(self, h):
        self.h = np.asarray(h, dtype=np.float64)
        self.n = self.h.shape[0]

    def action(self, x):
        return self.h @ x

    def diagonals(self):
        return np.diag(self.h).copy()

    def pp_action_matrix(self, p):
        return self.h[np.ix_(p, p)].copy()

    def p_column(self, i):
        return self.h[:, i].copy()

    def residual(self, x):
        return self.h @ (x - 1.0)


def splitmix64(z):
    z = (z + np.uint64(0x9E3779B97F4A7C15)).astype(np.uint64)
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)).astype(np.uint64)
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)).astype(np.uint64)
    return z ^ (z >> np.uint64(31))


class SyntheticProblem:
    """H = diag(d) + rho sum_l u_l u_l^T, u_0 = 1, u_l(g) = +-1 from splitmix64 (the
    rank-one case is test_rayleigh_quotient.cpp:37-42).  d_g = 1 + g (diag_kind 0), or for C5's
    well-posed DIIS instance (diag_kind 1) d_g = 1 + 2 frac(g phi1) with the preconditioner handed the
    approximate diagonal d_g (1 + alpha (2 frac(g phi2) - 1))."""

    PHI1, PHI2 = float.fromhex("0x1.3c6ef372fe950p-1"), float.fromhex("0x1.827f5352054c6p-1")

    def __init__(self, n, rho, rank, seed, diag_kind=0, alpha=0.0, target=1.0):
        self.n, self.rho, self.rank, self.diag_kind = n, rho, rank, diag_kind
        self.target = target  # r = H (x - target 1)
        g = np.arange(n, dtype=np.uint64)
        with np.errstate(over="ignore"):
            self.u = np.empty((rank, n))
            for l in range(rank):
                if l == 0:
                    self.u[l] = 1.0
                    continue
                key = splitmix64(np.array([np.uint64(seed) ^ np.uint64((1000 + l) * 0xD1B54A32D192ED03 % 2**64)],
                                          dtype=np.uint64))[0]
                self.u[l] = np.where(splitmix64(np.uint64(key) ^ g) & np.uint64(1), -1.0, 1.0)
        g = np.arange(n, dtype=np.float64)
        if diag_kind == 1:
            f1, f2 = g * self.PHI1, g * self.PHI2
            self.d0 = 1.0 + 2.0 * (f1 - np.floor(f1))
            self.pre = self.d0 * (1.0 + alpha * (2.0 * (f2 - np.floor(f2)) - 1.0))
        else:
            self.d0 = 1.0 + g
            self.pre = self.d0 + self.rank * self.rho

    def action(self, x):
        return self.d0 * x + self.rho * (self.u.T @ (self.u @ x))

    def diagonals(self):
        return self.pre

    def pp_action_matrix(self, p):
        up = self.u[:, p]
        return np.diag(self.d0[p]) + self.rho * (up.T @ up)

    def p_column(self, i):
        c = self.rho * (self.u.T @ self.u[:, i])
        c[i] += self.d0[i]
        return c

    def residual(self, x):
        return self.action(x - self.target)


# ---- the solver ----------------------------------------------------------------------------------
class Davidson:
    """LinearEigensystemDavidson (hermitian) with the reference's option semantics."""

    def __init__(self, nroots, convergence_threshold=1e-8, max_size_qspace=INT_MAX, reset_D=INT_MAX,
                 reset_D_max_Q_size=INT_MAX, max_p=0, p_threshold=DBL_MAX, max_iter=100):
        self.nroots = nroots
        self.thresh = convergence_threshold
        self.max_size_qspace = max_size_qspace
        self.reset_D = reset_D
        # set_max_size_qspace caps the resetter's limit (LinearEigensystemDavidson.h:137-141)
        self.max_Q_after_reset = min(reset_D_max_Q_size, max_size_qspace)
        self.max_p, self.p_threshold, self.max_iter = max_p, p_threshold, max_iter
        self.norm_thresh, self.svd_thresh = 1e-10, 1e-12
        self.P = []  # unit-vector indices
        self.q = []  # (param, action), newest first
        self.d = []  # (param, action)
        self.S = np.zeros((0, 0))
        self.H = np.zeros((0, 0))
        self.eigvals = np.zeros(0)
        self.solutions = np.zeros((0, 0))
        self.sub_errors = []
        self.errors = []
        self.value_errors = []
        self.last_values = []
        self.resetting = False
        self.working_set = list(range(nroots))
        self.iterations = 0
        self.r_creations = 0
        self.solution_params = []  # DSpaceResetter's pending solutions
        self.action_dot_action = False
        self.hermitian = True
        self.record_eigenvalues = True
        self.screened = 0  # new R vectors removed by the redundancy screen and as null, in all
        self.trace = {"eigenvalues": [], "errors": [], "nq": [], "nwork": [], "screened": []}

    # -- dimensions
    @property
    def nP(self):
        return len(self.P)

    @property
    def nQ(self):
        return len(self.q)

    @property
    def nD(self):
        return len(self.d)

    @property
    def nX(self):
        return self.nP + self.nQ + self.nD

    # -- subspace data
    def _p_vec(self, i):
        v = np.zeros(self.n)
        v[self.P[i]] = 1.0
        return v

    def update_qspace(self, params, actions):
        """XSpace::update_qspace (XSpace.h:176-183 -> update_qspace_data :30-83, QSpace::update :77-110)."""
        nP, nQ, nD, nX = self.nP, self.nQ, self.nD, self.nX
        oQ = nP
        qp = [p for p, _ in self.q]
        qa = [a for _, a in self.q]
        dp = [p for p, _ in self.d]
        da = [a for _, a in self.d]
        pv = [self._p_vec(i) for i in range(nP)]
        k = len(params)
        qq_s = sym_overlap(params)
        qx_s = np.hstack([cross(params, pv), cross(params, qp), cross(params, dp)]) if nX else np.zeros((k, 0))
        left = actions if self.action_dot_action else params  # XSpace.h:45-50
        qq_h = sym_overlap(actions) if self.action_dot_action else cross(params, actions)
        qx_h = np.zeros((k, nX))
        qx_h[:, nP:nP + nQ] = cross(left, qa)
        qx_h[:, nP + nQ:] = cross(left, da)
        xq_h = np.zeros((nX, k))
        if self.hermitian:  # XSpace.h:52-60
            xq_h[:nP, :] = cross(pv, actions)
            xq_h[nP:nP + nQ, :] = qx_h[:, nP:nP + nQ].T
            xq_h[nP + nQ:, :] = qx_h[:, nP + nQ:].T
            qx_h[:, :nP] = xq_h[:nP, :].T
        else:  # XSpace.h:61-64: <x_old, action_new>
            xq_h[nP:nP + nQ, :] = cross(qp, actions)
            xq_h[nP + nQ:, :] = cross(dp, actions)
        xq_s = qx_s.T
        for name, qq, qx, xq in (("S", qq_s, qx_s, xq_s), ("H", qq_h, qx_h, xq_h)):
            old = getattr(self, name)
            new = np.zeros((nX + k, nX + k))
            new[oQ + k:, oQ + k:] = old[oQ:, oQ:]
            new[oQ:oQ + k, oQ:oQ + k] = qq
            new[oQ:oQ + k, :oQ] = qx[:, :oQ]
            new[oQ:oQ + k, oQ + k:] = qx[:, oQ:]
            new[:oQ, oQ:oQ + k] = xq[:oQ, :]
            new[oQ + k:, oQ:oQ + k] = xq[oQ:, :]
            new[:oQ, :oQ] = old[:oQ, :oQ]
            new[:oQ, oQ + k:] = old[:oQ, oQ:]
            new[oQ + k:, :oQ] = old[oQ:, :oQ]
            setattr(self, name, new)
        self.q = [(params[i].copy(), actions[i].copy()) for i in range(k)] + self.q

    def update_dspace(self, dparams, dactions):
        """XSpace::update_dspace (XSpace.h:185-200): D replaced; its S and H blocks recomputed."""
        self.d = list(zip(dparams, dactions))
        nX = self.nX
        for name in ("S", "H"):
            m = getattr(self, name)
            new = np.zeros((nX, nX))
            c = min(nX, m.shape[0])
            new[:c, :c] = m[:c, :c]  # Matrix::resize keeps the leading block
            setattr(self, name, new)
        nP, nQ, nD = self.nP, self.nQ, self.nD
        oD = nP + nQ
        if nD == 0:
            return
        pv = [self._p_vec(i) for i in range(nP)]
        qp = [p for p, _ in self.q]
        qa = [a for _, a in self.q]
        dp = [p for p, _ in self.d]
        da = [a for _, a in self.d]
        # overlap data (:86-106): dd, dx = [dP, dQ], xd = dx^T
        dd = sym_overlap(dp)
        dx = np.hstack([cross(dp, pv), cross(dp, qp)])
        self.S[oD:, oD:] = dd
        self.S[oD:, :nP] = dx[:, :nP]
        self.S[oD:, nP:oD] = dx[:, nP:]
        self.S[:nP, oD:] = dx[:, :nP].T
        self.S[nP:oD, oD:] = dx[:, nP:].T
        # action data (:109-134)
        hdd = cross(dp, da)
        hxd = np.vstack([cross(pv, da), cross(qp, da)])
        hdx = np.zeros((nD, nP + nQ))
        hdx[:, nP:] = cross(dp, qa)
        hdx[:, :nP] = hxd[:nP, :].T
        self.H[oD:, oD:] = hdd
        self.H[oD:, :nP] = hdx[:, :nP]
        self.H[oD:, nP:oD] = hdx[:, nP:]
        self.H[:nP, oD:] = hxd[:nP, :]
        self.H[nP:oD, oD:] = hxd[nP:, :]

    def update_pspace(self, pidx, pp_action):
        """XSpace::update_pspace (XSpace.h:203-216), on an empty subspace."""
        self.P = list(pidx)
        self.S = sym_overlap([self._p_vec(i) for i in range(self.nP)])
        self.H = np.array(pp_action, dtype=np.float64).reshape(self.nP, self.nP)

    def _remove(self, i):
        for name in ("S", "H"):
            m = getattr(self, name)
            setattr(self, name, np.delete(np.delete(m, i, axis=0), i, axis=1))

    def eraseq(self, i):
        del self.q[i]
        self._remove(self.nP + i)

    # -- subspace solver
    def subspace_solve(self, nroots_max):
        w, sol = eigenproblem_hermitian(self.H, self.S)
        nr = min(nroots_max, sol.shape[0])
        self.eigvals = w[:nr].copy()
        self.solutions = sol[:nr].copy()
        self.sub_errors = [DBL_MAX] * nr

    # -- IterativeSolverTemplate
    def construct_solution(self, roots, with_p=True, actions=False):
        oP, oQ, oD = 0, self.nP, self.nP + self.nQ
        out = []
        for r in roots:
            x = np.zeros(self.n)
            if with_p:
                for j, i in enumerate(self.P):
                    x[i] += self.solutions[r, oP + j]
            vq = [a if actions else p for p, a in self.q]
            vd = [a if actions else p for p, a in self.d]
            for j, v in enumerate(vq):
                x += self.solutions[r, oQ + j] * v
            for j, v in enumerate(vd):
                x += self.solutions[r, oD + j] * v
            out.append(x)
        return out

    def solution(self, roots, params, actions):
        xs = self.construct_solution(roots)
        gs = self.construct_solution(roots, with_p=False, actions=True)
        for k, r in enumerate(roots):  # apply_p: the P-space part of the action (:210-211)
            for j, i in enumerate(self.P):
                gs[k] = gs[k] + self.problem.p_column(i) * self.solutions[r, j]
        for k, r in enumerate(roots):
            gs[k] = self.construct_residual(r, xs[k], gs[k])
        for k in range(len(roots)):
            params[k] = xs[k]
            actions[k] = gs[k]

    def construct_residual(self, root, x, g):
        """LinearEigensystemDavidson.h:186-192: g -= lambda x."""
        return g - self.eigvals[root] * x

    def set_value_errors(self):
        """LinearEigensystemDavidson.h:106-113."""
        cur = list(self.eigvals)
        self.value_errors = [DBL_MAX] * len(cur)
        for i in range(min(len(self.last_values), len(cur))):
            self.value_errors[i] = abs(cur[i] - self.last_values[i])
        if not self.resetting:
            self.last_values = cur

    def shifts(self):
        """working_set_eigenvalues (LinearEigensystemDavidson.h:98-104)."""
        return [self.eigvals[i] for i in self.working_set]

    def solve_and_generate_working_set(self, params, actions):
        self.subspace_solve(self.nroots)
        nsol = self.solutions.shape[0]
        nbuf = len(params)
        for start in range(0, nsol, nbuf):
            roots = list(range(start, min(start + nbuf, nsol)))
            if nsol > nbuf:
                raise NotImplementedError("more solutions than parameter buffers (not restated)")
            self.solution(roots, params, actions)
            for k, r in enumerate(roots):
                self.sub_errors[r] = float(np.sqrt(abs(actions[k] @ actions[k])))
        self.set_value_errors()
        self.errors = list(self.sub_errors)
        # select_working_set (:104-117): value threshold is DBL_MAX, so only errors decide
        cand = [i for i, e in enumerate(self.errors)
                if e > self.thresh or (i < len(self.value_errors) and self.value_errors[i] > DBL_MAX)]
        cand.sort(key=lambda i: -self.errors[i])  # multimap<greater>: equal keys keep insertion order
        ws = sorted(cand[:nbuf])
        self.working_set = ws
        for i, root in enumerate(ws):
            if root < i:
                raise RuntimeError("incorrect ordering of roots")
            if root > i:
                params[i] = params[root].copy()
                actions[i] = actions[root].copy()
        return len(ws)

    def add_vector(self, params, actions):
        nw = min(len(self.working_set), len(params))
        self.r_creations += nw
        self.update_qspace(params[:nw], actions[:nw])
        return self.solve_and_generate_working_set(params, actions)

    # -- propose_rspace and helpers
    def limit_qspace_size(self, max_size, solutions, nP):
        q_delete, q_indices = [], list(range(self.nQ))
        while len(q_indices) > max_size:
            contrib = [max(abs(solutions[j, nP + i]) for j in range(solutions.shape[0])) for i in q_indices]
            i = int(np.argmin(contrib))  # min_element: first minimum
            q_delete.append(q_indices.pop(i))
        return q_delete

    def _projected(self, solutions, q_delete):
        """construct_projected_solution + overlap + the two normalise/null-space passes (:39-179)."""
        nP, nQ, nD = self.nP, self.nQ, self.nD
        cols = [nP + j for j in q_delete] + [nP + nQ + j for j in range(nD)]
        sp = solutions[:, cols].copy()
        sblk = self.S[np.ix_(cols, cols)]

        def overlap(c):
            return c @ sblk @ c.T

        def remove_null_norm_and_normalise(c, ov):
            norms = np.sqrt(np.abs(np.diag(ov)))
            keep = []
            for i in range(c.shape[0]):
                if norms[i] > self.norm_thresh:
                    keep.append(i)
            c = c[keep] / norms[keep][:, None]
            ov = ov[np.ix_(keep, keep)] / np.outer(norms[keep], norms[keep])
            return c, ov

        ov = overlap(sp)
        sp, ov = remove_null_norm_and_normalise(sp, ov)
        svd = [(val, vec) for val, vec in svd_system_hermitian(ov, DBL_MAX) if not val < self.svd_thresh]
        svd.sort(key=lambda t: t[0])
        sp = np.array([vec @ sp for _, vec in svd]).reshape(len(svd), sp.shape[1])
        ov = overlap(sp)
        sp, ov = remove_null_norm_and_normalise(sp, ov)
        return sp

    def construct_dspace(self, solutions, q_delete):
        sp = self._projected(solutions, q_delete)
        nQd = len(q_delete)
        dp_new, da_new = [], []
        for i in range(sp.shape[0]):
            x, g = np.zeros(self.n), np.zeros(self.n)
            for j, iq in enumerate(q_delete):
                x += sp[i, j] * self.q[iq][0]
                g += sp[i, j] * self.q[iq][1]
            for j, (p, a) in enumerate(self.d):
                x += sp[i, nQd + j] * p
                g += sp[i, nQd + j] * a
            norm = np.sqrt(abs(x @ x))
            dp_new.append(x / norm)
            da_new.append(g / norm)
        return dp_new, da_new

    def propose_rspace(self, params, residuals):
        solutions = self.solutions.copy()
        q_delete = self.limit_qspace_size(self.max_size_qspace, solutions, self.nP)
        if q_delete:
            dp, da = self.construct_dspace(solutions, q_delete)
            for iq in sorted(q_delete, reverse=True):
                self.eraseq(iq)
            self.update_dspace(dp, da)
            self.subspace_solve(solutions.shape[0])
        idx = list(range(len(self.working_set)))  # wresidual: references into residuals
        for i in idx:  # normalise (:17-28)
            nrm = np.sqrt(abs(residuals[i] @ residuals[i]))
            if nrm > 1e-14:
                residuals[i] = residuals[i] / nrm
        # append_overlap_with_r + redundant_parameters (:271-300, :481-512)
        nX, nR = self.nX, len(idx)
        rv = [residuals[i] for i in idx]
        pv = [self._p_vec(i) for i in range(self.nP)]
        full = np.zeros((nX + nR, nX + nR))
        full[:nX, :nX] = self.S
        full[nX:, nX:] = sym_overlap(rv)
        full[nX:, :nX] = np.hstack([cross(rv, pv), cross(rv, [p for p, _ in self.q]), cross(rv, [p for p, _ in self.d])])
        full[:nX, nX:] = full[nX:, :nX].T
        redundant, rind = [], list(range(nR))
        for _, v in svd_system_hermitian(full, self.svd_thresh):
            if rind:
                contrib = [abs(v[nX + i]) for i in rind]
                k = int(np.argmax(contrib))
                redundant.append(rind.pop(k))
        for k in sorted(redundant, reverse=True):
            del idx[k]
        # modified_gram_schmidt (:421-466)
        spaces = [(pv, 0), ([p for p, _ in self.q], self.nP), ([p for p, _ in self.d], self.nP + self.nQ)]
        for vecs, off in spaces:
            for i, x in enumerate(vecs):
                norm = abs(self.S[off + i, off + i])
                if idx:
                    c = [-(residuals[j] @ x) / norm for j in idx]
                    for cj, j in zip(c, idx):
                        residuals[j] = residuals[j] + cj * x
        null = []
        for a, i in enumerate(idx):
            nrm = np.sqrt(abs(residuals[i] @ residuals[i]))
            if nrm > self.norm_thresh:
                residuals[i] = residuals[i] * (1.0 / nrm)
                for j in idx[a + 1:]:
                    ov = residuals[i] @ residuals[j]
                    residuals[j] = residuals[j] - ov * residuals[i]
            else:
                null.append(a)
        for k in sorted(null, reverse=True):
            del idx[k]
        self.screened += len(redundant) + len(null)
        for i in idx:
            nrm = np.sqrt(abs(residuals[i] @ residuals[i]))
            if nrm > 1e-14:
                residuals[i] = residuals[i] / nrm
        for k, i in enumerate(idx):
            params[k] = residuals[i].copy()
        return [self.working_set[i] for i in idx]

    def dspace_reset_run(self, params):
        """DSpaceResetter::run (DSpaceResetter.h:84-144)."""
        solutions = self.solutions.copy()
        if not self.solution_params and params:
            sp = self._projected(solutions, list(range(self.nQ)))
            nQ = self.nQ
            for i in range(sp.shape[0]):
                x = np.zeros(self.n)
                for j, (p, _) in enumerate(self.q):
                    x += sp[i, j] * p
                for j, (p, _) in enumerate(self.d):
                    x += sp[i, nQ + j] * p
                self.solution_params.append(x)
            self.update_dspace([], [])
        nr = min(len(params), len(self.solution_params))
        for i in range(nr):
            params[i] = self.solution_params.pop(0)
        ov = cross(params[:nr], [p for p, _ in self.q])
        q_ind, q_max = list(range(self.nQ)), []
        for i in range(nr):
            if not q_ind:
                break
            k = int(np.argmax([abs(ov[i, j]) for j in q_ind]))
            q_max.append(q_ind.pop(k))
        for iq in sorted(q_max, reverse=True):
            self.eraseq(iq)
        if self.nQ + nr > self.max_Q_after_reset:
            limit = self.max_Q_after_reset - nr if self.max_Q_after_reset > nr else 0
            # resize_qspace reads the (pre-reset) solution matrix with the current dimensions
            for iq in sorted(self.limit_qspace_size(limit, solutions, self.nP), reverse=True):
                self.eraseq(iq)
        return list(range(nr))

    def end_iteration(self, params, actions):
        do_reset = ((self.iterations + 1) % self.reset_D == 0 and self.nD > 0) or bool(self.solution_params)
        if do_reset:
            self.resetting = True
            self.working_set = self.dspace_reset_run(params)
        else:
            self.resetting = False
            self.working_set = self.propose_rspace(params, actions)
        self.iterations += 1
        return len(self.working_set)

    # -- solve (IterativeSolverTemplate.h:322-408)
    def solve(self, problem, generate_initial_guess=True):
        self.problem, self.n = problem, problem.n
        nbuf = self.nroots
        params = [np.zeros(self.n) for _ in range(nbuf)]
        actions = [np.zeros(self.n) for _ in range(nbuf)]
        diag = problem.diagonals()
        if generate_initial_guess:
            for root, g in enumerate(select_smallest(diag, nbuf)):
                params[root] = np.zeros(self.n)
                params[root][g] = 1.0
        nwork = nbuf
        pspace = []
        if self.max_p > 0:
            sel = select_smallest(diag, self.max_p)
            first = diag[sel[0]] if sel else 0.0
            for k, i in enumerate(sel):
                if diag[i] > first + self.p_threshold:
                    sel = sel[:k]
                    break
            pspace = sel
            if pspace and len(pspace) < self.nroots:
                raise RuntimeError("P space must be empty or at least as large as number of roots sought")
            self.update_pspace(pspace, problem.pp_action_matrix(pspace))
            nwork = self.solve_and_generate_working_set(params, actions)
        end_needed = True
        for it in range(self.max_iter):
            if nwork <= 0:
                break
            if it > 0 or not pspace:
                for k in range(nwork):
                    actions[k] = problem.action(params[k])
                nwork = self.add_vector(params, actions)
                end_needed = True
            while end_needed:
                if nwork > 0:
                    shifts = self.shifts()
                    for k in range(nwork):
                        actions[k] = actions[k] / (diag - shifts[k] + 1e-15)
                nwork = self.end_iteration(params, actions)
                end_needed = False
            if self.record_eigenvalues:
                self.trace["eigenvalues"].append(list(self.eigvals))
            self.trace["errors"].append(list(self.errors))
            self.trace["nq"].append(self.nQ)
            self.trace["nwork"].append(len(self.working_set))
            self.trace["screened"].append(self.screened)
        converged = nwork == 0 and max(self.errors) <= self.thresh
        return {"converged": converged, "iterations": self.iterations, "r_creations": self.r_creations,
                "eigenvalues": list(self.eigvals), "errors": list(self.errors), "trace": self.trace}


def solve_diis(h):
    """helper-implementation.h:619-669: the augmented B matrix [[H, -1], [-1, 0]] solved for
    rhs (0, ..., 0, -1) by a JacobiSVD with threshold 0 (a full-rank solve); the first dim entries."""
    dim = h.shape[0]
    b = np.zeros((dim + 1, dim + 1))
    b[:dim, :dim] = h
    b[dim, :dim] = b[:dim, dim] = -1.0
    rhs = np.zeros(dim + 1)
    rhs[dim] = -1.0
    u, sv, vt = np.linalg.svd(b)
    coeffs = vt.T @ (np.where(sv > 0, 1.0 / np.where(sv > 0, sv, 1.0), 0.0) * (u.T @ rhs))
    if np.any(np.isnan(coeffs)):
        raise OverflowError("NaN detected in DIIS submatrix solution")
    return coeffs[:dim]


class DIIS(Davidson):
    """NonLinearEquationsDIIS (hermitian X space, H = action . action) over the shared X-space code."""

    def __init__(self, convergence_threshold=1e-8, max_size_qspace=INT_MAX, max_iter=100):
        super().__init__(1, convergence_threshold, max_iter=max_iter)
        self.diis_max_q = max_size_qspace
        self.action_dot_action = True
        self.converged_flag = False

    def least_important_vector(self):
        h = self.H
        result = (0, DBL_MAX)
        if h.shape[1] < 2:
            return result
        w, v = sym_eig_ascending(h)
        evmax, second, first = 0.0, DBL_MAX, 0
        for i in range(len(w)):
            evmax = max(evmax, w[i])
            if w[i] < second:
                second, first = w[i], 1
                for j in range(1, h.shape[0]):
                    if abs(v[j, i]) > abs(v[first, i]):
                        first = j
        second /= evmax
        if second > self.svd_thresh:
            return h.shape[1] - 1, DBL_MAX
        return first, second

    def subspace_solve(self, nroots_max):
        dim = self.H.shape[0]
        self.solutions = np.zeros((1, dim))
        if self.converged_flag:
            self.solutions[0, 0] = 1.0
            return  # errors kept (SubspaceSolverDIIS.h:40-44)
        self.solutions[0] = solve_diis(self.H)
        self.sub_errors = [self.H[0, 0]]

    def solve_and_generate_working_set(self, params, actions):
        self.subspace_solve(1)
        self.solution([0], params, actions)
        if not self.sub_errors:
            self.sub_errors = [0.0]
        self.sub_errors[0] = float(np.sqrt(abs(actions[0] @ actions[0])))
        self.errors = list(self.sub_errors)  # set_value_errors is the base no-op: no value errors
        ws = [0] if self.errors[0] > self.thresh else []
        self.working_set = ws
        return len(ws)

    def solution(self, roots, params, actions):
        xs = self.construct_solution(roots)
        gs = self.construct_solution(roots, with_p=False, actions=True)  # residual: no construct_residual
        for k in range(len(roots)):
            params[k] = xs[k]
            actions[k] = gs[k]

    def add_vector(self, params, actions):
        x, r = params[0], actions[0]
        error = float(np.sqrt(r @ r))
        self.converged_flag = error < self.thresh
        d = self.least_important_vector()
        while self.nX >= self.diis_max_q or d[1] < self.svd_thresh:
            self.eraseq(d[0])
            d = self.least_important_vector()
        nw = min(len(self.working_set), 1)
        self.r_creations += nw
        self.update_qspace([x][:nw], [r][:nw])
        nwork = self.solve_and_generate_working_set(params, actions)
        self.errors[0] = error
        return nwork

    def end_iteration(self, params, actions):
        if self.working_set:
            params[0] = self.construct_solution(self.working_set)[0]
        if self.errors[0] < self.thresh:
            self.working_set = []
            return 0
        self.working_set = [0]
        params[0] = params[0] - actions[0]
        self.iterations += 1
        return 1

    def solve(self, problem, generate_initial_guess=False):
        """IterativeSolverTemplate::solve for a nonlinear solver: x starts at e_0 (the product's DIIS
        driver), r = residual(x), preconditioner shift 0 (IterativeSolver.h:320-322)."""
        self.problem, self.n = problem, problem.n
        x = np.zeros(self.n)
        x[0] = 1.0
        params, actions = [x], [np.zeros(self.n)]
        diag = problem.diagonals()
        nwork = 1
        for it in range(self.max_iter):
            if nwork <= 0:
                break
            actions[0] = problem.residual(params[0])
            nwork = self.add_vector(params, actions)
            end_needed = True
            while end_needed:
                if nwork > 0:
                    actions[0] = actions[0] / (diag - 0.0 + 1e-15)
                nwork = self.end_iteration(params, actions)
                end_needed = False
            self.trace["errors"].append(list(self.errors))
            self.trace["nq"].append(self.nQ)
            self.trace["nwork"].append(len(self.working_set))
        converged = nwork == 0 and max(self.errors) <= self.thresh
        return {"converged": converged, "iterations": self.iterations, "r_creations": self.r_creations,
                "errors": list(self.errors), "x": params[0], "trace": self.trace}


class LinearEquations(Davidson):
    """LinearEquationsDavidson (hermitian by default): A x_r = b_r for the given right-hand sides."""

    def __init__(self, rhs, convergence_threshold=1e-8, max_size_qspace=INT_MAX, reset_D=INT_MAX,
                 reset_D_max_Q_size=INT_MAX, augmented_hessian=0.0, max_p=0, max_iter=100):
        super().__init__(len(rhs), convergence_threshold, max_size_qspace, reset_D, reset_D_max_Q_size, max_p,
                         max_iter=max_iter)
        self.b = [np.array(r, dtype=np.float64) for r in rhs]
        self.b_norm = []
        for r in self.b:  # XSpace::add_rhs_equations
            d = abs(r @ r)
            if d == 0:
                raise RuntimeError("RHS vector cannot be zero")
            self.b_norm.append(np.sqrt(d))
        self.ah = augmented_hessian
        self.RHS = np.zeros((0, len(self.b)))  # data[rhs]: nX x nRHS
        self.record_eigenvalues = False

    # the rhs block follows every change of the X space
    def update_qspace(self, params, actions):
        nP, k = self.nP, len(params)
        rows = cross(params, self.b)  # XSpace.h:65
        self.RHS = np.vstack([self.RHS[:nP], rows, self.RHS[nP:]])
        super().update_qspace(params, actions)

    def update_dspace(self, dparams, dactions):
        super().update_dspace(dparams, dactions)
        keep = self.RHS[: self.nP + self.nQ]
        self.RHS = np.vstack([keep, cross([p for p, _ in self.d], self.b)]) if self.nD else keep.copy()

    def update_pspace(self, pidx, pp_action):
        super().update_pspace(pidx, pp_action)
        self.RHS = cross([self._p_vec(i) for i in range(self.nP)], self.b)

    def eraseq(self, i):
        self.RHS = np.delete(self.RHS, self.nP + i, axis=0)
        super().eraseq(i)

    def subspace_solve(self, nroots_max):
        """SubspaceSolverLinEig::solve_linear_equations -> solve_LinearEquations."""
        nx, nr = self.H.shape[0], len(self.b)
        self.eigvals = np.zeros(nr)
        sol = np.zeros((nr, nx))
        if self.ah > 0:
            import scipy.linalg

            flat = self.RHS.reshape(-1)  # rhs[i + nX * root] of the row-major nX x nRHS block
            for root in range(nr):
                a = np.zeros((nx + 1, nx + 1))
                b = np.zeros((nx + 1, nx + 1))
                a[:nx, :nx] = self.H.T  # column-major Map of the row-major H (helper-implementation.h:571)
                b[:nx, :nx] = self.S.T
                col = -self.ah * flat[np.arange(nx) + nx * root]
                a[:nx, nx] = a[nx, :nx] = col
                b[nx, nx] = 1.0
                w, v = scipy.linalg.eig(a, b)
                imax = 0
                for i in range(nx + 1):
                    if w[i].real < w[imax].real:
                        imax = i
                self.eigvals[root] = w[imax].real
                sol[root] = v[:nx, imax].real / (self.ah * v[nx, imax].real)
        else:
            sol = np.linalg.solve(self.H, self.RHS).T
        self.solutions = sol
        self.sub_errors = [DBL_MAX] * nr

    def construct_residual(self, root, x, g):
        """LinearEquationsDavidson.h:170-181: g = (g - b_root) / |b_root|."""
        g = g - self.b[root]
        if self.b_norm[root] != 0:
            g = g * (1.0 / self.b_norm[root])
        return g

    def set_value_errors(self):
        self.value_errors = []  # the base no-op: LinearEquationsDavidson has no value errors

    def shifts(self):
        return [0.0] * len(self.working_set)  # IterativeSolver.h:320-322

    def end_iteration(self, params, actions):
        do_reset = ((self.iterations + 1) % self.reset_D == 0 and self.nD > 0) or bool(self.solution_params)
        if do_reset:
            self.working_set = self.dspace_reset_run(params)
        else:
            self.working_set = self.propose_rspace(params, actions)
        self.iterations += 1
        return len(self.working_set)


class Cubic:
    """Interpolate(p0, p1, "cubic") and its analytic minimum (Interpolate.cpp:56-66, :101-134);
    points are (x, f, f1)."""

    def __init__(self, p0, p1):
        self.x0, self.x1 = p0[0], p1[0]
        x1mx0 = p1[0] - p0[0]
        f1pf0, f1mf0 = p1[1] + p0[1], p1[1] - p0[1]
        g1pg0, g1mg0 = p1[2] + p0[2], p1[2] - p0[2]
        self.c = [0.5 * f1pf0 - 0.125 * g1mg0 * x1mx0, -0.25 * g1pg0 + 1.5 * f1mf0 / x1mx0, 0.5 * g1mg0 / x1mx0,
                  (-2 * f1mf0 + g1pg0 * x1mx0) / x1mx0 ** 3]

    def __call__(self, x):
        c, xb = self.c, 0.5 * (self.x1 + self.x0)
        t = x - xb
        return x, c[0] + t * (c[1] + t * (c[2] + t * c[3])), c[1] + t * (2 * c[2] + 3 * t * c[3])

    def minimize_cubic(self):
        cc, b, a = self.c[1], 2 * self.c[2], 3 * self.c[3]
        with np.errstate(all="ignore"):
            disc = b * b / (4 * a * a) - cc / a
        if np.isnan(disc) or disc < 0:
            return float("nan")
        xb = 0.5 * (self.x1 + self.x0)
        pm = self(xb - (b / (2 * a)) + np.sqrt(disc))
        pp = self(xb - (b / (2 * a)) - np.sqrt(disc))
        return pm[0] if pm[1] < pp[1] else pp[0]


class Optimize(Davidson):
    """OptimizeBFGS (bfgs = True) / OptimizeSD over a non-hermitian X space; value data as the reference
    keeps it (BFGS shifts it with the Q space, SD overwrites its first row)."""

    def __init__(self, bfgs=True, convergence_threshold=1e-8, max_size_qspace=INT_MAX, max_iter=100):
        super().__init__(1, convergence_threshold, max_iter=max_iter)
        self.bfgs = bfgs
        self.hermitian = False
        self.opt_max_q = max_size_qspace
        self.value = np.zeros(0)
        self.alpha = []
        self.linesearch = False
        self.last_linesearching = False
        self.strong_wolfe, self.wolfe1, self.wolfe2 = True, 1e-4, 0.9
        self.ls_tol, self.ls_grow = 0.2, 2.0
        self.record_eigenvalues = False
        self.line_searches = 0

    def eraseq(self, i):
        self.value = np.delete(self.value, self.nP + i)
        super().eraseq(i)

    def subspace_solve(self, nroots_max):
        dim = self.H.shape[0]
        self.solutions = np.zeros((1, dim))
        self.solutions[0, 0] = 1.0
        self.sub_errors = [self.H[0, 0]]

    def set_value_errors(self):
        self.value_errors = [DBL_MAX]
        if self.nX > 1 and self.value[0] < self.value[1]:
            self.value_errors[0] = self.value[1] - self.value[0]

    def solution(self, roots, params, actions):
        xs = self.construct_solution(roots)
        gs = self.construct_solution(roots, with_p=False, actions=True)
        for k in range(len(roots)):
            params[k] = xs[k]
            actions[k] = gs[k]

    def solve_and_generate_working_set(self, params, actions):
        self.subspace_solve(1)
        self.solution([0], params, actions)
        self.sub_errors[0] = float(np.sqrt(abs(actions[0] @ actions[0])))
        self.set_value_errors()
        self.errors = list(self.sub_errors)
        ws = [0] if (self.errors[0] > self.thresh or self.value_errors[0] > DBL_MAX) else []
        self.working_set = ws
        return len(ws)

    def base_add_vector(self, params, actions):
        nw = min(len(self.working_set), 1)
        self.r_creations += nw
        self.update_qspace(params[:nw], actions[:nw])
        return self.solve_and_generate_working_set(params, actions)

    def _h4(self, a):
        h = self.H
        return h[a, a] - h[a, a + 1] - h[a + 1, a] + h[a + 1, a + 1]

    def add_vector(self, params, actions, value):
        if not self.bfgs:  # OptimizeSD.h:79-87
            v = np.zeros(self.nX + 1)
            v[: len(self.value)] = self.value[: self.nX + 1]
            v[0] = value
            self.value = v
            return self.base_add_vector(params, actions)
        while self.nX >= self.opt_max_q:
            self.eraseq(self.nX - 1)
        self.value = np.r_[value, self.value]
        nwork = self.base_add_vector(params, actions)
        if self.nX > 1:
            fprev, fcur = self.value[1], self.value[0]
            gprev, gcur = self.H[0, 1] - self.H[1, 1], self.H[0, 0] - self.H[1, 0]
            w1 = fcur <= fprev + self.wolfe1 * gprev
            w2 = gcur >= self.wolfe2 * gprev if self.strong_wolfe else abs(gcur) <= self.wolfe2 * abs(gprev)
            if not (w1 and w2):
                x = Cubic((-1.0, fprev, gprev), (0.0, fcur, gcur)).minimize_cubic()
                if abs(x) > self.ls_tol:
                    params[0] = params[0] * (1 + x)
                    params[0] = params[0] + (-x) * self.q[1][0]
                    self.eraseq(0 if fprev < fcur else 1)
                    self.linesearch = True
                    return -1
        self.linesearch = False
        while True:  # accept: drop a Q pair that makes a BFGS denominator vanish
            # (the reference indexes past the shrunken H when an erase leaves fewer pairs than alphas;
            # the loop stops at the last pair, as the product's restatement does)
            for a in range(min(len(self.alpha), self.nX - 1)):
                if abs(self._h4(a)) < max(5e-14 * abs(self.H[a, a]), 1e-15):
                    self.eraseq(a + 1)
                    break
            else:
                break
        g = actions[0]  # BFGS_update_1 (OptimizeBFGS.h:135-146)
        self.alpha = [0.0] * (self.nX - 1)
        for a in range(len(self.alpha)):
            qa, qb = self.q[a][0], self.q[a + 1][0]
            self.alpha[a] = ((g @ qa) - (g @ qb)) / self._h4(a)
            g = g + (-self.alpha[a]) * self.q[a][1]
            g = g + self.alpha[a] * self.q[a + 1][1]
        actions[0] = g
        return nwork

    def end_iteration(self, params, actions):
        if not self.bfgs:  # OptimizeSD.h:37-47
            if self.working_set:
                params[0] = self.construct_solution(self.working_set)[0]
            if self.errors[0] < self.thresh:
                self.working_set = []
                return 0
            self.working_set = [0]
            params[0] = params[0] - actions[0]
            self.iterations += 1
            return 1
        self.working_set = [0]
        if not self.linesearch:
            self.last_linesearching = False
            params[0] = self.construct_solution([0])[0]
            if self.errors[0] < self.thresh:
                self.working_set = []
                return 0
            z = actions[0]  # BFGS_update_2 (:148-157)
            for a in range(len(self.alpha) - 1, -1, -1):
                beta = ((z @ self.q[a][1]) - (z @ self.q[a + 1][1])) / self._h4(a)
                z = z + (self.alpha[a] - beta) * self.q[a][0]
                z = z + (-self.alpha[a] + beta) * self.q[a + 1][0]
            params[0] = params[0] - z
        else:
            if not self.last_linesearching:
                self.line_searches += 1
            self.last_linesearching = True
        self.iterations += 1
        return 0 if self.errors[0] < self.thresh else 1

    def solve(self, problem, generate_initial_guess=False):
        """IterativeSolverTemplate::solve, nonlinear branch: value = residual(x, g); add_vector; the
        diagonal preconditioner with shift 0 when nwork > 0; end_iteration.  x starts at e_0."""
        self.problem, self.n = problem, problem.n
        x = np.zeros(self.n)
        x[0] = 1.0
        params, actions = [x], [np.zeros(self.n)]
        diag = problem.diagonals()
        nwork = 1
        for it in range(self.max_iter):
            if nwork <= 0 and it > 0:
                break
            f, actions[0] = problem.value_gradient(params[0])
            nwork = self.add_vector(params, actions, f)
            if nwork > 0:
                actions[0] = actions[0] / (diag - 0.0 + 1e-15)
            nwork = self.end_iteration(params, actions)
            self.trace["eigenvalues"].append([self.value[0]])
            self.trace["errors"].append(list(self.errors))
            self.trace["nq"].append(self.nQ)
            self.trace["nwork"].append(len(self.working_set))
        converged = nwork == 0 and max(self.errors) <= self.thresh
        return {"converged": converged, "iterations": self.iterations, "r_creations": self.r_creations,
                "errors": list(self.errors), "x": params[0], "value": self.value[0], "trace": self.trace}


class RayleighProblem(DenseProblem):
    """f(x) = x.Hx / x.x, g = 2 (Hx - f x) / x.x (the product's optimize_dense problem,
    test_Optimize.cpp's Rayleigh-quotient form)."""

    def value_gradient(self, x):
        g = self.h @ x
        xx, xg = x @ x, x @ g
        f = xg / xx
        return f, (g - f * x) * (2 / xx)
