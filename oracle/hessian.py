"""Second-order (HessianLearner) restatement over the oracle's ENUM path
matrices -- TEST INFRASTRUCTURE ONLY (tests/ may import it; the product never
does).

Dense numpy restatement of the reference's default optimizer
(src/HessianLearner.cpp), used to check the GPU HessianLearner epoch by epoch:

* AssembleH (:381-496): the H_f pattern of an equivocal string (more than one
  path) is every pair of parameters whose counts are not identical on all of
  its paths; unique-path strings contribute nothing.
* ComputeHf (:498-547): H_f[j,k] += p_s (E[c_j] E[c_k] - E[c_j c_k]) under the
  string's relative path probabilities -- minus the count covariance.
* ComputeHg (:589-607), ComputeRhs (:580-587), InitSlackVariables (:554-563),
  LambdaUpdate (src/Learner.cpp:438-462): the KKT system
  [[H_f + diag(e^x lambda_c), J_g], [J_g^T, 0]] [dx; dl] = [grad + J_g lambda; C^T e^x - 1],
  x -= eta dx, lambda -= eta dl (or the exponential update, flag 32).
* GetOptimizationInfo (:293-350): KL, graderr, g_min, g_max, inertia (+, -),
  lambda_min, rmin (smallest relative path probability), its path index.
* ComputeLogDetHessian (:219-260) + RealSymmetricLogDet (src/Utils.cpp:296-350):
  log det of (H_f - diag(grad)) / (e^x_j e^x_k), the objective's Hessian in
  weight space; +inf when the determinant is not positive.

The factorisation is numpy's (LAPACK), not MKL DSS: solves agree to rounding.
A determinant of an (exactly) singular Hessian is rounding noise and differs
between factorisations -- see DESIGN.md, "Hessian" (talk is such a case).
"""
import numpy as np

from .oracle import Oracle, OracleError


def _log_simplex_volume(d):
    """src/Utils.cpp:221-227"""
    if d <= 0:
        return 0.0
    return 0.5 * np.log(d) - sum(np.log(i) for i in range(2, d))


def _mxlogx(x):
    return -x * np.log(x) if x > 0 else 0.0


class HessianOracle:
    def __init__(self, oracle: Oracle):
        self.o = oracle
        self.n, self.k = oracle.n, oracle.info["n_constraints"]
        self.ccol = oracle.ccol()
        prow, pcol, pdata, mrow = oracle.paths()
        self.p = oracle.p()
        self.S = len(self.p)
        self.mrow = mrow
        self.n_paths = len(prow) - 1
        # dense path-count matrix (paths x params): the oracle cases are small
        self.P = np.zeros((self.n_paths, self.n))
        for l in range(self.n_paths):
            for q in range(prow[l], prow[l + 1]):
                self.P[l, pcol[q]] += pdata[q]
        self.unique = self.n_paths == self.S
        self.plogp = float(np.sum(self.p * np.log(self.p)))
        self.x = np.zeros(self.n)
        self.lam = np.ones(self.k)
        self.include_hf = False
        self.exp_lambda = False
        self.degenerate = False
        self.error = np.inf
        # equivocal parameter sets per string (AssembleH)
        self.equivocal = []
        for s in range(self.S):
            a, b = mrow[s], mrow[s + 1]
            if b - a > 1:
                rows = self.P[a:b]
                eq = np.flatnonzero(np.any(rows != rows[0], axis=0) & np.any(rows != 0, axis=0))
                self.equivocal.append((s, eq))

    # -- Learner pieces -----------------------------------------------------
    def renormalize(self):
        """src/Learner.cpp:23-42"""
        for c in range(self.k):
            m = self.ccol == c
            self.x[m] -= np.log(np.exp(self.x[m]).sum())

    def modeled(self):
        """ComputeModeledProbs (src/Learner.cpp:515-547): logq, relative path probs"""
        lw = self.P @ self.x
        logq = np.zeros(self.S)
        rpp = np.zeros(self.n_paths)
        for s in range(self.S):
            a, b = self.mrow[s], self.mrow[s + 1]
            m = lw[a:b].max()
            e = np.exp(lw[a:b] - m)
            q = e.sum()
            logq[s] = m + np.log(q)
            rpp[a:b] = e / q
        return logq, rpp

    def grad(self, rpp):
        """ComputeGrad (:620-653): -P^T (M^T p * rpp)"""
        pl = np.repeat(self.p, np.diff(self.mrow))
        return -(self.P.T @ (pl * rpp))

    def hf(self, rpp):
        """ComputeHf (:498-547), dense, symmetric"""
        H = np.zeros((self.n, self.n))
        for s, eq in self.equivocal:
            a, b = self.mrow[s], self.mrow[s + 1]
            c = self.P[a:b][:, eq]
            r = rpp[a:b]
            m = r @ c
            H[np.ix_(eq, eq)] += self.p[s] * (np.outer(m, m) - (c * r[:, None]).T @ c)
        return H

    def kkt(self, grad, hf):
        ex = np.exp(self.x)
        n, k = self.n, self.k
        K = np.zeros((n + k, n + k))
        if self.include_hf:
            K[:n, :n] = hf
        K[np.arange(n), np.arange(n)] += ex * self.lam[self.ccol]
        K[np.arange(n), n + self.ccol] = ex
        K[n + self.ccol, np.arange(n)] = ex
        g = np.bincount(self.ccol, weights=ex, minlength=k) - 1.0
        rhs = np.concatenate([grad + ex * self.lam[self.ccol], g])
        return K, rhs

    # -- the optimizer ------------------------------------------------------
    def init(self, flags):
        """InitCallback (:125-180)"""
        self.exp_lambda = bool(flags & 32)
        if flags & 1:
            self.x = np.zeros(self.n)
            self.lam = np.ones(self.k)
        if flags & 2:
            self.renormalize()
        if flags & 4:
            _, rpp = self.modeled()
            g = self.grad(rpp)
            self.lam = -np.bincount(self.ccol, weights=g, minlength=self.k)
        self.include_hf = bool(flags & 8)
        self.degenerate = False

    def step(self, eta=1.0):
        """OptimizationStep (:62-123) + GetOptimizationInfo: returns the 9-value info row"""
        logq, rpp = self.modeled()
        grad = self.grad(rpp)
        kl = self.plogp - float(self.p @ logq)
        K, rhs = self.kkt(grad, self.hf(rpp) if self.include_hf else None)
        lambda_min = float(self.lam.min()) if self.k else 0.0
        try:
            d = np.linalg.solve(K, rhs)
        except np.linalg.LinAlgError:
            d = np.full_like(rhs, np.nan)
        if not np.all(np.isfinite(d)):
            self.degenerate = True
        else:
            self.x -= eta * d[:self.n]
            if self.exp_lambda:
                self.lam *= np.exp(-eta * d[self.n:] / self.lam)
            else:
                self.lam -= eta * d[self.n:]
        info = np.zeros(9)
        info[0] = kl
        info[1] = np.abs(rhs[:self.n]).max()
        info[2] = rhs[self.n:].min()
        info[3] = rhs[self.n:].max()
        self.error = max(info[1], abs(info[2]), abs(info[3]))
        if not self.degenerate:
            ev = np.linalg.eigvalsh(K)
            tol = np.abs(ev).max() * len(ev) * np.finfo(float).eps
            info[4] = float(np.sum(ev > tol))
            info[5] = float(np.sum(ev < -tol))
        info[6] = lambda_min
        if not self.unique:
            i = int(np.argmin(np.abs(rpp)))
            info[7], info[8] = rpp[i], i
        return info

    def halt(self, tol):
        """HaltCondition (:371-377)"""
        if self.degenerate:
            raise OracleError("Unable to continue!")
        return self.error <= tol

    def run(self, flags=31, epochs=20, eta=1.0, tol=1e-6):
        """main.cpp epoch loop (src/main.cpp:276-303)"""
        self.init(flags)
        rows = []
        for _ in range(epochs):
            rows.append(self.step(eta))
            if self.halt(tol):
                break
        return rows

    def weight_hessian(self):
        """ComputeLogDetHessian's matrix: (H_f - diag(grad)) / (e^x_j e^x_k)"""
        _, rpp = self.modeled()
        grad = self.grad(rpp)
        ex = np.exp(self.x)
        return (self.hf(rpp) - np.diag(grad)) / np.outer(ex, ex)

    def log_det_hessian(self):
        H = self.weight_hessian()
        if not any(len(eq) > 1 for _, eq in self.equivocal):
            d = np.diag(H)    # diagonal pattern: RealSymmetricLogDet's n == nnz rule
            return float(np.sum(np.log(d))) if np.all(d > 0) else np.inf
        sign, logdet = np.linalg.slogdet(H)
        return float(logdet) if sign > 0 else np.inf

    def result(self):
        """GetOptimizationResult (:352-369): 8 values"""
        logq, _ = self.modeled()
        info = self.o.info
        return np.array([
            self.plogp - float(self.p @ logq),
            _mxlogx(info["common_support"]),
            info["model_volume"],
            _log_simplex_volume(int(info["aux_params"])),
            self.log_det_hessian(),
            info["aux_hessian"],
            float(self.n - self.k),
            float(max(0, info["aux_params"] - 1)),
        ])
