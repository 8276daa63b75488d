"""ctypes wrapper of oracle/_build/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of the reference w-fsa objective/gradient
path (see wfsa_oracle.c).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module; the product never does.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

ENUM, TRELLIS = 0, 1


class _Info(C.Structure):
    _fields_ = [
        ("n_corpus", C.c_int64), ("n_strings", C.c_int64), ("n_paths", C.c_int64),
        ("n_full", C.c_int), ("n_params", C.c_int), ("n_constraints", C.c_int), ("unique", C.c_int),
        ("aux_params", C.c_int64),
        ("plogp", C.c_double), ("common_support", C.c_double), ("model_volume", C.c_double),
        ("aux_hessian", C.c_double),
        ("n_states", C.c_int),
    ]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, i64, dbl = C.c_void_p, C.c_int64, C.c_double
        pd = C.POINTER(C.c_double)
        L.oracle_build_text.restype = vp
        L.oracle_build_text.argtypes = [C.c_char_p, C.c_char_p, C.c_int, i64, C.c_char_p, C.c_int]
        L.oracle_build_arrays.restype = vp
        L.oracle_build_arrays.argtypes = [C.c_char_p, vp, vp, vp, i64, C.c_int, i64, C.c_char_p, C.c_int]
        L.oracle_free.argtypes = [vp]
        L.oracle_get_info.argtypes = [vp, C.POINTER(_Info)]
        L.oracle_param_name.argtypes = [vp, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_int), C.POINTER(C.c_char_p)]
        L.oracle_full_param_name.argtypes = L.oracle_param_name.argtypes
        L.oracle_trimmed_index.argtypes = [vp, C.c_int]
        L.oracle_trimmed_index.restype = C.c_int
        for name in ("oracle_path_counts", "oracle_get_x", "oracle_set_x", "oracle_get_logq",
                     "oracle_get_p", "oracle_get_grad", "oracle_get_w_full"):
            getattr(L, name).argtypes = [vp, vp]
        L.oracle_kl.argtypes = [vp]
        L.oracle_kl.restype = dbl
        L.oracle_objective_grad.argtypes = [vp, pd, pd]
        L.oracle_renormalize.argtypes = [vp]
        L.oracle_qn_init.argtypes = [vp, C.c_int]
        L.oracle_qn_step.argtypes = [vp, dbl, vp]
        L.oracle_qn_halt.argtypes = [vp, dbl]
        L.oracle_qn_halt.restype = C.c_int
        L.oracle_trellis_eval.argtypes = [vp, vp, vp, vp, pd, C.c_char_p, C.c_int]
        L.oracle_set_threads.argtypes = [vp, C.c_int]
        L.oracle_path_nnz.argtypes = [vp]
        L.oracle_path_nnz.restype = i64
        L.oracle_get_paths.argtypes = [vp, vp, vp, vp, vp]
        L.oracle_get_paths.restype = C.c_int
        L.oracle_get_ccol.argtypes = [vp, vp]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


class OracleError(RuntimeError):
    pass


class Oracle:
    """One built learner: automaton + corpus -> p, P/M (ENUM) or trellis."""

    def __init__(self, handle):
        self._h = handle
        info = _Info()
        lib().oracle_get_info(self._h, C.byref(info))
        self.info = {f: getattr(info, f) for f, _ in _Info._fields_}

    @classmethod
    def from_text(cls, wfsa_text, corpus_text, mode=ENUM, max_paths=1_000_000):
        err = C.create_string_buffer(512)
        h = lib().oracle_build_text(wfsa_text.encode("latin-1") if isinstance(wfsa_text, str) else wfsa_text,
                                    corpus_text.encode("latin-1") if isinstance(corpus_text, str) else corpus_text,
                                    mode, max_paths, err, 512)
        if not h:
            raise OracleError(err.value.decode("latin-1"))
        return cls(h)

    @classmethod
    def from_files(cls, wfsa_path, corpus_path, **kw):
        with open(wfsa_path, "rb") as f:
            a = f.read()
        with open(corpus_path, "rb") as f:
            c = f.read()
        return cls.from_text(a, c, **kw)

    @classmethod
    def from_arrays(cls, wfsa_text, sym, off, weights, mode=ENUM, max_paths=1_000_000):
        sym = np.ascontiguousarray(sym, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.int64)
        weights = np.ascontiguousarray(weights, dtype=np.float64)
        err = C.create_string_buffer(512)
        h = lib().oracle_build_arrays(wfsa_text.encode("latin-1") if isinstance(wfsa_text, str) else wfsa_text,
                                      _ptr(sym), _ptr(off), _ptr(weights), len(off) - 1, mode, max_paths, err, 512)
        if not h:
            raise OracleError(err.value.decode("latin-1"))
        return cls(h)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oracle_free(self._h)
            self._h = None

    # -- accessors ---------------------------------------------------------
    @property
    def n(self):
        return self.info["n_params"]

    def param_names(self):
        """trimmed index -> (state, kind, label); kind 'E' emission / 'T' transition"""
        out = []
        s, k, l = C.c_char_p(), C.c_int(), C.c_char_p()
        for t in range(self.n):
            lib().oracle_param_name(self._h, t, C.byref(s), C.byref(k), C.byref(l))
            out.append((s.value.decode("latin-1"), "ET"[k.value], l.value.decode("latin-1")))
        return out

    def full_param_names(self):
        out = []
        s, k, l = C.c_char_p(), C.c_int(), C.c_char_p()
        for j in range(self.info["n_full"]):
            lib().oracle_full_param_name(self._h, j, C.byref(s), C.byref(k), C.byref(l))
            out.append((s.value.decode("latin-1"), "ET"[k.value], l.value.decode("latin-1")))
        return out

    def trimmed_index(self):
        return np.array([lib().oracle_trimmed_index(self._h, j) for j in range(self.info["n_full"])], dtype=np.int64)

    def path_counts(self):
        a = np.zeros(self.info["n_corpus"], dtype=np.int64)
        lib().oracle_path_counts(self._h, _ptr(a))
        return a

    def paths(self):
        """ENUM path matrices: (Prow, Pcol, Pdata, Mrow) -- path l's parameter
        counts are Pcol/Pdata[Prow[l]:Prow[l+1]], string s's paths Mrow[s]:Mrow[s+1]"""
        nnz = lib().oracle_path_nnz(self._h)
        if nnz < 0:
            raise OracleError("path matrices exist in ENUM mode only")
        prow = np.zeros(self.info["n_paths"] + 1, dtype=np.int64)
        pcol = np.zeros(max(nnz, 1), dtype=np.int32)
        pdata = np.zeros(max(nnz, 1), dtype=np.float64)
        mrow = np.zeros(self.info["n_strings"] + 1, dtype=np.int64)
        lib().oracle_get_paths(self._h, _ptr(prow), _ptr(pcol), _ptr(pdata), _ptr(mrow))
        return prow, pcol[:nnz], pdata[:nnz], mrow

    def ccol(self):
        """constraint (normalisation group) of each trimmed parameter"""
        a = np.zeros(max(self.n, 1), dtype=np.int32)
        lib().oracle_get_ccol(self._h, _ptr(a))
        return a[:self.n].astype(np.int64)

    def x(self):
        a = np.zeros(self.n, dtype=np.float64)
        lib().oracle_get_x(self._h, _ptr(a))
        return a

    def set_x(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        assert x.shape == (self.n,)
        lib().oracle_set_x(self._h, _ptr(x))

    def p(self):
        a = np.zeros(self.info["n_strings"], dtype=np.float64)
        lib().oracle_get_p(self._h, _ptr(a))
        return a

    def logq(self):
        a = np.zeros(self.info["n_strings"], dtype=np.float64)
        lib().oracle_get_logq(self._h, _ptr(a))
        return a

    def grad(self):
        a = np.zeros(self.n, dtype=np.float64)
        lib().oracle_get_grad(self._h, _ptr(a))
        return a

    def w_full(self):
        a = np.zeros(self.info["n_full"], dtype=np.float64)
        lib().oracle_get_w_full(self._h, _ptr(a))
        return a

    # -- the hot path ------------------------------------------------------
    def objective_grad(self):
        """(KL, loglik) at the current x; grad() / logq() hold the rest."""
        kl, ll = C.c_double(), C.c_double()
        lib().oracle_objective_grad(self._h, C.byref(kl), C.byref(ll))
        return kl.value, ll.value

    def set_threads(self, n):
        """OpenMP threads of objective_grad / trellis_eval (1 = serial, the default)"""
        lib().oracle_set_threads(self._h, int(n))

    def renormalize(self):
        lib().oracle_renormalize(self._h)

    def qn_init(self, flags):
        lib().oracle_qn_init(self._h, flags)

    def qn_step(self, eta=1.0):
        info = np.zeros(7, dtype=np.float64)
        lib().oracle_qn_step(self._h, eta, _ptr(info))
        return info

    def qn_halt(self, tol):
        return bool(lib().oracle_qn_halt(self._h, tol))

    def qn_run(self, flags=7, epochs=20, eta=1.0, tol=1e-6):
        """main.cpp epoch loop (src/main.cpp:276-303): returns list of info rows."""
        self.qn_init(flags)
        rows = []
        for _ in range(epochs):
            info = self.qn_step(eta)
            rows.append(info)
            if not np.all(np.isfinite(info)):
                raise OracleError("non-finite epoch info")
            if self.qn_halt(tol):
                break
        return rows

    def trellis_eval(self, w_full):
        """dense trellis at Fsa-indexed weights: (loglik, logq per corpus string, grad_full)"""
        w_full = np.ascontiguousarray(w_full, dtype=np.float64)
        logq = np.zeros(self.info["n_corpus"], dtype=np.float64)
        grad = np.zeros(self.info["n_full"], dtype=np.float64)
        ll = C.c_double()
        err = C.create_string_buffer(256)
        rc = lib().oracle_trellis_eval(self._h, _ptr(w_full), _ptr(logq), _ptr(grad), C.byref(ll), err, 256)
        if rc != 0:
            raise OracleError(err.value.decode())
        return ll.value, logq, grad
