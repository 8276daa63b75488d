"""MI355X-native objective/gradient path of w-fsa (weighted FSA weight learning).

Python mirror of the reference's host interface (Fsa, Corpus, Learner,
QuasiNewtonLearner; inc/*.h of gaebor/w-fsa) over the C ABI in
include/wfsa_host.h, plus direct access to the device boundary
(include/wfsa_dev.h) through `Device`.  All compute runs in the HIP library
libwfsa_amd.so on a gfx950 GPU; there is no CPU fallback.
"""
import ctypes as C
import os
import sys
import time

import numpy as np

from . import _lib
from ._lib import WfsaError, check_dev, check_host, load

_RUN_TRACE = bool(os.environ.get("WFSA_RUN_TRACE"))   # (diagnostics: Run's host-side timestamps on stderr)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


__all__ = ["Fsa", "Corpus", "QuasiNewtonLearner", "Device", "Synthetic", "WfsaError", "load", "shard_range",
           "sym_sparse_solve", "trellis_stats"]


def shard_range(off, nranks, rank):
    """[begin, end) of the strings rank `rank` keeps (balanced on total length)"""
    off = np.ascontiguousarray(off, dtype=np.int64)
    b, e = C.c_int64(), C.c_int64()
    check_host(load().wfsa_shard_range(_ptr(off), len(off) - 1, nranks, rank, C.byref(b), C.byref(e)))
    return b.value, e.value


def sym_sparse_solve(i, j, v, n, b=None, order=0):
    """the HessianLearner's sparse LDL^T on the upper-triangle coordinates
    (i <= j): (x or None, dict of the factorisation's statistics)"""
    i = np.ascontiguousarray(i, dtype=np.int32)
    j = np.ascontiguousarray(j, dtype=np.int32)
    v = np.ascontiguousarray(v, dtype=np.float64)
    bb = None if b is None else np.ascontiguousarray(b, dtype=np.float64)
    x = None if b is None else np.zeros(n)
    oi = np.zeros(8, dtype=np.int64)
    od = np.zeros(3)
    check_host(load().wfsa_sym_sparse_solve(n, len(v), _ptr(i), _ptr(j), _ptr(v), order, _ptr(bb), _ptr(x),
                                            _ptr(oi), _ptr(od)))
    return x, dict(positive=int(oi[0]), negative=int(oi[1]), nnz_l=int(oi[2]), ordered=bool(oi[3]),
                   supernodes=int(oi[4]), two_by_two=int(oi[5]), max_front=int(oi[6]), delayed=int(oi[7]),
                   log_abs_det=float(od[0]), det_sign=int(od[1]), min_pivot_ratio=float(od[2]))


def trellis_stats(fsa):
    """(nodes, byte edges, end edges, parameter-list entries) of the compiled trellis"""
    d = fsa.desc()
    out = np.zeros(4, dtype=np.int64)
    check_host(load().wfsa_trellis_compile_stats(C.byref(d), _ptr(out)))
    return tuple(int(v) for v in out)


def _b(s):
    return s if isinstance(s, bytes) else s.encode("latin-1")


class Fsa:
    """The automaton (inc/Fsa.h): .wfsa reader, parameter numbering, Dump."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def read_text(cls, text):
        h = C.c_void_p()
        check_host(load().wfsa_fsa_read_text(_b(text), C.byref(h)))
        return cls(h)

    @classmethod
    def read_file(cls, path):
        h = C.c_void_p()
        check_host(load().wfsa_fsa_read_file(_b(path), C.byref(h)))
        return cls(h)

    def __del__(self):
        if getattr(self, "_h", None):
            load().wfsa_fsa_free(self._h)
            self._h = None

    def counts(self):
        a = np.zeros(6, dtype=np.int64)
        check_host(load().wfsa_fsa_counts(self._h, _ptr(a)))
        keys = ("states", "transitions", "emissions", "parameters", "constraints", "free_parameters")
        return dict(zip(keys, (int(v) for v in a)))

    def desc(self):
        d = _lib.ModelDesc()
        check_host(load().wfsa_fsa_desc(self._h, C.byref(d)))
        return d

    def param_name(self, j):
        s, k, l = C.c_char_p(), C.c_int32(), C.c_char_p()
        check_host(load().wfsa_fsa_param_name(self._h, j, C.byref(s), C.byref(k), C.byref(l)))
        return s.value.decode("latin-1"), "ET"[k.value], l.value.decode("latin-1")

    def param_names(self):
        return [self.param_name(j) for j in range(self.counts()["parameters"])]


class Corpus:
    """The string store (inc/Corpus.h): .corpus reader; weights as read."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def read_text(cls, text):
        h = C.c_void_p()
        check_host(load().wfsa_corpus_read_text(_b(text), C.byref(h)))
        return cls(h)

    @classmethod
    def read_file(cls, path):
        h = C.c_void_p()
        check_host(load().wfsa_corpus_read_file(_b(path), C.byref(h)))
        return cls(h)

    def __del__(self):
        if getattr(self, "_h", None):
            load().wfsa_corpus_free(self._h)
            self._h = None

    def packed(self):
        """(sym uint8[], off int64[n+1], weights float64[n]) copies"""
        sym, off, w, n = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_int64()
        check_host(load().wfsa_corpus_view(self._h, C.byref(sym), C.byref(off), C.byref(w), C.byref(n)))
        n = n.value
        off_a = np.ctypeslib.as_array(C.cast(off, C.POINTER(C.c_int64)), shape=(n + 1,)).copy()
        w_a = np.ctypeslib.as_array(C.cast(w, C.POINTER(C.c_double)), shape=(max(n, 1),))[:n].copy()
        total = int(off_a[-1])
        sym_a = (np.ctypeslib.as_array(C.cast(sym, C.POINTER(C.c_uint8)), shape=(total,)).copy()
                 if total else np.zeros(0, dtype=np.uint8))
        return sym_a, off_a, w_a

    def strings(self):
        sym, off, w = self.packed()
        return [bytes(sym[off[i]:off[i + 1]]).decode("latin-1") for i in range(len(w))], w


class Synthetic:
    """Synthetic automaton + corpus (SURVEY.md 8d families)."""

    def __init__(self, n_states=1024, degree=8, vocab=64, emissions=1, dense=False, n_strings=1000,
                 max_len=128, seed=1):
        h = C.c_void_p()
        check_host(load().wfsa_synth_make(n_states, degree, vocab, emissions, int(dense), n_strings, max_len,
                                          seed, C.byref(h)))
        self._h = h
        self.wfsa_text = load().wfsa_synth_wfsa_text(h).decode("latin-1")

    def __del__(self):
        if getattr(self, "_h", None):
            load().wfsa_synth_free(self._h)
            self._h = None

    def corpus(self):
        sym, off, w, n = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_int64()
        check_host(load().wfsa_synth_corpus(self._h, C.byref(sym), C.byref(off), C.byref(w), C.byref(n)))
        n = n.value
        off_a = np.ctypeslib.as_array(C.cast(off, C.POINTER(C.c_int64)), shape=(n + 1,)).copy()
        w_a = np.ctypeslib.as_array(C.cast(w, C.POINTER(C.c_double)), shape=(n,)).copy()
        sym_a = np.ctypeslib.as_array(C.cast(sym, C.POINTER(C.c_uint8)), shape=(int(off_a[-1]),)).copy()
        return sym_a, off_a, w_a


class QuasiNewtonLearner:
    """inc/QuasiNewtonLearner.h: BuildFrom -> Finalize -> Init -> OptimizationStep*.
    optimizer="Hessian" gives the reference's HessianLearner (see HessianLearner)."""

    def __init__(self, device=0, optimizer="QuasiNewton"):
        h = C.c_void_p()
        check_host(load().wfsa_learner_create(_b(optimizer), device, C.byref(h)))
        self._h = h
        self._fsa = None
        self.width = load().wfsa_learner_info_width(h)   # values per info row

    def __del__(self):
        if getattr(self, "_h", None):
            load().wfsa_learner_destroy(self._h)
            self._h = None

    def SetCommunicator(self, nranks, rank, unique_id):
        buf = (C.c_uint8 * _lib.COMM_ID_BYTES).from_buffer_copy(bytes(unique_id))
        check_host(load().wfsa_learner_set_comm(self._h, nranks, rank, buf))

    def AbortCommunicator(self, why="aborted by the caller"):
        """this rank failed: the other ranks' current or next collective
        fails at once (wfsa_learner_comm_abort)"""
        check_host(load().wfsa_learner_comm_abort(self._h, why.encode()))

    def BuildFrom(self, fsa, corpus):
        self._fsa = fsa
        check_host(load().wfsa_learner_build(self._h, fsa._h, corpus._h))

    def set_info_rmin(self, on):
        """the rmin info column on (default) / off"""
        check_host(load().wfsa_learner_set_info_rmin(self._h, int(bool(on))))

    def LoadMatrices(self, prefix):
        """matrix-file mode (Learner::LoadMatrices): prefix.{C,M,P,prob,aux}"""
        self._fsa = None
        check_host(load().wfsa_learner_load_matrices(self._h, os.fsencode(prefix)))

    def SaveMatrices(self, prefix):
        check_host(load().wfsa_learner_save_matrices(self._h, os.fsencode(prefix)))

    def SetHostCommunicator(self, nranks, rank, allreduce):
        """a communicator over a host callback (wfsa_learner_set_comm_host):
        allreduce(array, op) reduces a numpy array in place over the ranks,
        op "sum" / "min" (float64) or "max" (uint8) -- e.g. torch_allreduce
        over a gloo process group"""
        self._host_cb = _host_callback(allreduce)
        check_host(load().wfsa_learner_set_comm_host(self._h, nranks, rank, self._host_cb, None))

    def BuildFromPacked(self, fsa, sym, off, weights):
        self._fsa = fsa
        sym = np.ascontiguousarray(sym, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.int64)
        weights = np.ascontiguousarray(weights, dtype=np.float64)
        check_host(load().wfsa_learner_build_packed(self._h, fsa._h, _ptr(sym), _ptr(off), _ptr(weights),
                                                    len(off) - 1))

    def Finalize(self):
        check_host(load().wfsa_learner_finalize(self._h))

    def info(self):
        i = _lib.LearnerInfo()
        check_host(load().wfsa_learner_info_get(self._h, C.byref(i)))
        return {f: getattr(i, f) for f, _ in _lib.LearnerInfo._fields_}

    @property
    def n(self):
        return self.info()["n_params"]

    def Init(self, flags, x0=None):
        x0 = None if x0 is None else np.ascontiguousarray(x0, dtype=np.float64)
        check_host(load().wfsa_learner_init(self._h, flags, _ptr(x0)))

    def OptimizationStep(self, eta=1.0, tol=1e-6):
        info = np.zeros(self.width, dtype=np.float64)
        halt = C.c_int32()
        check_host(load().wfsa_learner_step(self._h, eta, tol, _ptr(info), C.byref(halt)))
        return info, bool(halt.value)

    def objective_grad(self, want_logq=False):
        """(KL, grad[n_params], logq or None) at the current x"""
        inf = self.info()
        grad = np.zeros(inf["n_params"], dtype=np.float64)
        logq = np.zeros(inf["n_local_strings"], dtype=np.float64) if want_logq else None
        kl = C.c_double()
        check_host(load().wfsa_learner_objective_grad(self._h, C.byref(kl), _ptr(grad), _ptr(logq)))
        return kl.value, grad, logq

    def x(self):
        a = np.zeros(self.n, dtype=np.float64)
        check_host(load().wfsa_learner_get_x(self._h, _ptr(a)))
        return a

    def last_grad(self):
        """gradient (trimmed) of the last evaluation; after Run, of its last step"""
        a = np.zeros(self.n, dtype=np.float64)
        check_host(load().wfsa_learner_get_grad(self._h, _ptr(a)))
        return a

    def set_x(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        assert x.shape == (self.n,)
        check_host(load().wfsa_learner_set_x(self._h, _ptr(x)))

    def p(self):
        a = np.zeros(self.info()["n_local_strings"], dtype=np.float64)
        check_host(load().wfsa_learner_get_p(self._h, _ptr(a)))
        return a

    def trimmed_index(self):
        a = np.zeros(self.info()["n_full"], dtype=np.int32)
        check_host(load().wfsa_learner_trimmed_index(self._h, _ptr(a)))
        return a

    def path_counts(self):
        inf = self.info()
        m = inf["shard_end"] - inf["shard_begin"]
        pc = np.zeros(m, dtype=np.float64)
        rec = np.zeros(m, dtype=np.uint8)
        check_host(load().wfsa_learner_path_counts(self._h, _ptr(pc), _ptr(rec)))
        return pc, rec

    def Renormalize(self):
        check_host(load().wfsa_learner_renormalize(self._h))

    def Dump(self, path, fsa=None):
        check_host(load().wfsa_learner_dump(self._h, (fsa or self._fsa)._h, _b(path)))

    def stats(self):
        s = _lib.DevStats()
        check_host(load().wfsa_learner_stats(self._h, C.byref(s)))
        return {f: getattr(s, f) for f, _ in _lib.DevStats._fields_}

    def param_names(self):
        """trimmed index -> (state, kind, label)"""
        fsa = self._fsa
        tw = self.trimmed_index()
        names = [None] * self.n
        for j, t in enumerate(tw):
            if t >= 0:
                names[t] = fsa.param_name(j)
        return names

    def run(self, flags=7, epochs=20, eta=1.0, tol=1e-6):
        """main.cpp's epoch loop (src/main.cpp:276-303), run natively by
        wfsa_learner_run: list of info rows (the epochs actually run)"""
        self.Init(flags)
        return self.Run(epochs, eta, tol)

    def result(self):
        """GetOptimizationResult (the -eval line): KL, mxlogx(support),
        LogModelVolume, LogAuxVolume, logdetHessian, LogDetAuxHessian, n-k, aux-1"""
        out = np.zeros(8, dtype=np.float64)
        check_host(load().wfsa_learner_result(self._h, _ptr(out)))
        return out

    def Run(self, epochs, eta=1.0, tol=1e-6):
        """up to `epochs` OptimizationSteps in one native call (no Init)"""
        t0 = time.monotonic_ns() if _RUN_TRACE else 0
        n = max(int(epochs), 0)
        rb = self.__dict__.get("_run_rows")
        if rb is None or rb[0].shape[0] < n:   # (one rows buffer per learner, grown on demand: no allocation per Run)
            rows = np.zeros((max(n, 256), self.width))
            done = C.c_int32(0)
            rb = self._run_rows = (rows, _ptr(rows), done, C.byref(done), load().wfsa_learner_run)
        rows, ptr, done, done_ref, fn = rb
        t1 = time.monotonic_ns() if _RUN_TRACE else 0
        rc = fn(self._h, eta, tol, n, ptr, done_ref)
        t2 = time.monotonic_ns() if _RUN_TRACE else 0
        check_host(rc)
        out = rows[:done.value].tolist()
        if _RUN_TRACE:
            print(f"[wfsa.py] Run: entry {t0} ns, native call at {t1}, back at {t2}, out at {time.monotonic_ns()}",
                  file=sys.stderr, flush=True)
        return out


_OPS = ("sum", "min", "max")


def _host_callback(allreduce):
    """wrap a Python all-reduce as a wfsa_host_allreduce_fn"""
    def cb(user, buf, count, op):
        try:
            ct = C.c_uint8 if op == 2 else C.c_double
            arr = np.ctypeslib.as_array((ct * int(count)).from_address(buf))
            allreduce(arr, _OPS[op])
            return 0
        except Exception:   # reported to the library as a failed transport
            import traceback
            traceback.print_exc()
            return 1
    return _lib.HOST_ALLREDUCE_FN(cb)


def torch_allreduce(arr, op):
    """all-reduce a numpy array in place over the default torch.distributed
    process group (gloo for host buffers).  A member that stalls without
    aborting: the wait gives up after WFSA_COMM_TIMEOUT_S (default 300 s, the
    library's host watchdog limit) and raises -- the library then fails the
    call and treats the group as broken (collective.hip HostCollective)"""
    import datetime
    import torch
    import torch.distributed as dist
    red = {"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX}[op]
    t = torch.from_numpy(arr)
    limit = float(os.environ.get("WFSA_COMM_TIMEOUT_S", "300"))
    dist.all_reduce(t, op=red, async_op=True).wait(timeout=datetime.timedelta(seconds=limit))


class Device:
    """Direct handle on the device boundary (include/wfsa_dev.h)."""

    def __init__(self, device=0):
        h = C.c_void_p()
        check_dev(load().wfsa_dev_create(device, C.byref(h)))
        self._h = h
        self.n_params = 0
        self.n_strings = 0

    def __del__(self):
        if getattr(self, "_h", None):
            load().wfsa_dev_destroy(self._h)
            self._h = None

    def load_model(self, fsa):
        d = fsa.desc()
        self._fsa = fsa   # keeps the desc arrays alive
        check_dev(load().wfsa_dev_load_model(self._h, C.byref(d)))
        self.n_params = d.n_params

    def load_corpus(self, sym, off, p):
        self._sym = np.ascontiguousarray(sym, dtype=np.uint8)
        self._off = np.ascontiguousarray(off, dtype=np.int64)
        self._p = np.ascontiguousarray(p, dtype=np.float64)
        check_dev(load().wfsa_dev_load_corpus(self._h, _ptr(self._sym), _ptr(self._off), _ptr(self._p),
                                              len(self._off) - 1))
        self.n_strings = len(self._off) - 1

    def recognize(self):
        rec = np.zeros(self.n_strings, dtype=np.uint8)
        pc = np.zeros(self.n_strings, dtype=np.float64)
        used = np.zeros(max(self.n_params, 1), dtype=np.uint8)
        check_dev(load().wfsa_dev_recognize(self._h, _ptr(rec), _ptr(pc), _ptr(used)))
        return rec, pc, used[:self.n_params]

    def sym_factor(self, a):
        """Bunch-Kaufman LDL^T of symmetric a in HBM: ((pos, neg, zero), log|det|, sign)"""
        a = np.ascontiguousarray(a, dtype=np.float64)
        n = a.shape[0]
        inertia = np.zeros(3, dtype=np.int64)
        lad, sign = C.c_double(), C.c_int32()
        check_dev(load().wfsa_dev_sym_factor(self._h, n, _ptr(a), _ptr(inertia), C.byref(lad), C.byref(sign)))
        return tuple(int(v) for v in inertia), lad.value, sign.value

    def sym_factor_coo(self, n, i, j, v, b=None):
        """the blocked LDL^T from upper-triangle entries (wfsa_dev_sym_factor_coo):
        ((pos, neg, zero), log|det|, sign, method (1 blocked, 2 full BK), x or None)"""
        i = np.ascontiguousarray(i, dtype=np.int32)
        j = np.ascontiguousarray(j, dtype=np.int32)
        v = np.ascontiguousarray(v, dtype=np.float64)
        x = None if b is None else np.array(b, dtype=np.float64)
        inertia = np.zeros(3, dtype=np.int64)
        lad, sign, method = C.c_double(), C.c_int32(), C.c_int32()
        check_dev(load().wfsa_dev_sym_factor_coo(self._h, int(n), len(v), _ptr(i), _ptr(j), _ptr(v), _ptr(x),
                                                 _ptr(inertia), C.byref(lad), C.byref(sign), C.byref(method)))
        return tuple(int(q) for q in inertia), lad.value, sign.value, method.value, x

    def sym_solve(self, b):
        x = np.array(b, dtype=np.float64)
        check_dev(load().wfsa_dev_sym_solve(self._h, _ptr(x)))
        return x

    def load_paths(self, n_params, prow, pcol, pdata, mrow, mcol, p):
        """matrix-file mode on the device: P (paths x params CSR), M (strings x paths)"""
        prow = np.ascontiguousarray(prow, dtype=np.int64)
        pcol = np.ascontiguousarray(pcol, dtype=np.int32)
        pdata = np.ascontiguousarray(pdata, dtype=np.float64)
        mrow = np.ascontiguousarray(mrow, dtype=np.int64)
        mcol = np.ascontiguousarray(mcol, dtype=np.int64)
        p = np.ascontiguousarray(p, dtype=np.float64)
        check_dev(load().wfsa_dev_load_paths(self._h, int(n_params), len(prow) - 1, _ptr(prow), _ptr(pcol), _ptr(pdata),
                                             len(mrow) - 1, _ptr(mrow), _ptr(mcol), _ptr(p)))
        self.n_params = int(n_params)
        self.n_strings = len(mrow) - 1

    def string_tiers(self):
        """per string: -1 compiled stream, 0/1 LDS traversal, 2 wide traversal, 3 dense"""
        t = np.zeros(max(self.n_strings, 1), dtype=np.int8)
        check_dev(load().wfsa_dev_string_tiers(self._h, _ptr(t)))
        return t[:self.n_strings]

    def objective_grad(self, w_full, want_logq=True):
        w = np.ascontiguousarray(w_full, dtype=np.float64)
        grad = np.zeros(max(self.n_params, 1), dtype=np.float64)
        logq = np.zeros(self.n_strings, dtype=np.float64) if want_logq else None
        ll = C.c_double()
        check_dev(load().wfsa_dev_objective_grad(self._h, _ptr(w), C.byref(ll), _ptr(grad), _ptr(logq)))
        return ll.value, grad[:self.n_params], logq

    def objective_grad_begin(self, w_full, want_logq=True):
        """enqueue the evaluation and return (wfsa_dev_objective_grad_begin)"""
        self._w_keep = np.ascontiguousarray(w_full, dtype=np.float64)
        self._want_logq = want_logq
        check_dev(load().wfsa_dev_objective_grad_begin(self._h, _ptr(self._w_keep), int(want_logq)))

    def objective_grad_end(self):
        grad = np.zeros(max(self.n_params, 1), dtype=np.float64)
        logq = np.zeros(self.n_strings, dtype=np.float64) if getattr(self, "_want_logq", False) else None
        ll = C.c_double()
        check_dev(load().wfsa_dev_objective_grad_end(self._h, C.byref(ll), _ptr(grad), _ptr(logq)))
        return ll.value, grad[:self.n_params], logq

    def hf_setup(self):
        """pattern of the Hessian's second-order term: (j, k) Fsa parameter pairs"""
        n = C.c_int64()
        check_dev(load().wfsa_dev_hf_setup(self._h, C.byref(n)))
        pairs = np.zeros(max(2 * n.value, 1), dtype=np.int32)
        check_dev(load().wfsa_dev_hf_pairs(self._h, _ptr(pairs)))
        self._hf_n = n.value
        return pairs[:2 * n.value].reshape(-1, 2)

    def hf_eval(self, w_full):
        """sum_s p_s Cov_s(count_j, count_k) for the hf_setup pairs"""
        w = np.ascontiguousarray(w_full, dtype=np.float64)
        vals = np.zeros(max(self._hf_n, 1), dtype=np.float64)
        check_dev(load().wfsa_dev_hf_eval(self._h, _ptr(w), _ptr(vals)))
        return vals[:self._hf_n]

    def rmin(self):
        """(smallest relative path probability, string holding it) at the
        weights of the last objective_grad; string -1 when none is ambiguous"""
        r, i = C.c_double(), C.c_int64()
        check_dev(load().wfsa_dev_rmin(self._h, C.byref(r), C.byref(i)))
        return r.value, i.value

    def comm_init(self, nranks, rank, unique_id):
        buf = (C.c_uint8 * _lib.COMM_ID_BYTES).from_buffer_copy(bytes(unique_id))
        check_dev(load().wfsa_dev_comm_init(self._h, nranks, rank, buf))

    @staticmethod
    def comm_unique_id():
        buf = (C.c_uint8 * _lib.COMM_ID_BYTES)()
        check_dev(load().wfsa_dev_comm_unique_id(buf))
        return bytes(buf)

    @staticmethod
    def comm_local_id(nranks):
        """id of an in-process group: `nranks` contexts of this process, one
        thread each (wfsa_dev_comm_local_id)"""
        buf = (C.c_uint8 * _lib.COMM_ID_BYTES)()
        check_dev(load().wfsa_dev_comm_local_id(nranks, buf))
        return bytes(buf)

    def comm_init_host(self, nranks, rank, allreduce):
        """wfsa_dev_comm_init_host (see QuasiNewtonLearner.SetHostCommunicator)"""
        self._host_cb = _host_callback(allreduce)
        check_dev(load().wfsa_dev_comm_init_host(self._h, nranks, rank, self._host_cb, None))

    def comm_abort(self, why="aborted by the caller"):
        """wfsa_dev_comm_abort: every other member's current or next
        collective fails at once"""
        check_dev(load().wfsa_dev_comm_abort(self._h, why.encode()))

    @staticmethod
    def peer_selftest(nranks, n, timeout_s, mode, device=0):
        """the peer all-reduce kernel on one device (wfsa_dev_peer_selftest):
        returns (metric, status, poisoned areas, seconds)"""
        out = (C.c_double * 4)()
        check_dev(load().wfsa_dev_peer_selftest(device, nranks, n, timeout_s, mode, out))
        return tuple(out)

    def allreduce(self, values):
        a = np.ascontiguousarray(values, dtype=np.float64).copy()
        check_dev(load().wfsa_dev_allreduce(self._h, _ptr(a), len(a)))
        return a

    def stats(self):
        s = _lib.DevStats()
        check_dev(load().wfsa_dev_get_stats(self._h, C.byref(s)))
        return {f: getattr(s, f) for f, _ in _lib.DevStats._fields_}


class HessianLearner(QuasiNewtonLearner):
    """inc/HessianLearner.h: the reference's default optimizer (augmented
    Newton/KKT steps with the count covariance H_f from the device)."""

    def __init__(self, device=0):
        super().__init__(device, optimizer="Hessian")
