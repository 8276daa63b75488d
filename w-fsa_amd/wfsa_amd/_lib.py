"""ctypes bindings of libwfsa_amd.so (include/wfsa_dev.h, include/wfsa_host.h).

The library is built in-tree by `make -C w-fsa_amd/csrc` (or
__graft_entry__.build()).  There is no CPU fallback: if the library or a
gfx950 device is missing, every call fails loudly.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# WFSA_LIB: the timing-experiment build (make -C w-fsa_amd/csrc exp) for tools/;
# bench.py refuses to measure with it
LIB_PATH = os.environ.get("WFSA_LIB") or os.path.join(HERE, "libwfsa_amd.so")

WFSA_OK = 0
WFSA_ERR_ARG = -1
WFSA_ERR_HIP = -2
WFSA_ERR_MODEL = -3
WFSA_ERR_CAPACITY = -4
WFSA_ERR_RCCL = -5
WFSA_ERR_NODEV = -6
COMM_ID_BYTES = 128

vp = C.c_void_p
i32, i64, u8, dbl = C.c_int32, C.c_int64, C.c_uint8, C.c_double
P = C.POINTER


class ModelDesc(C.Structure):
    _fields_ = [
        ("n_states", i32), ("start", i32), ("end", i32), ("n_params", i32),
        ("em_ptr", P(i32)), ("em_off", P(i64)), ("em_len", P(i32)), ("em_param", P(i32)),
        ("em_bytes", P(u8)), ("tr_ptr", P(i32)), ("tr_dst", P(i32)), ("tr_param", P(i32)),
    ]


class DevStats(C.Structure):
    _fields_ = [
        ("n_strings", i64), ("total_symbols", i64), ("max_len", i32), ("n_nodes", i32),
        ("n_edges", i64), ("n_end_edges", i64), ("compiled_strings", i64), ("fallback_strings", i64),
        ("stream_words", i64), ("stream_bytes", i64), ("bubble_words", i64), ("n_bubbles", i64), ("fb_launches", i64), ("fb_kernel_ms", dbl),
        ("last_fb_kernel_ms", dbl), ("last_compiled_ms", dbl), ("last_call_ms", dbl),
        ("last_live_edges", i64), ("tier1_strings", i32), ("waves_per_block", i32), ("prepare_ms", dbl),
        ("compiled_kernel_ms", dbl), ("graph", i32), ("dense", i32),
        ("host_steps", i64), ("host_begin_ms", dbl), ("host_overlap_ms", dbl), ("host_wait_ms", dbl),
        ("host_post_ms", dbl),
        ("dense_rows", i32), ("dense_steps", i32), ("dense_np", i32), ("tier2_strings", i32),
        ("wave_strings", i32), ("wave_row_entries", i64), ("wave_pair_edges", i64),
        ("comm_ranks", i32), ("comm_peer", i32),
        ("slot_chunks", i64), ("max_group_chunks", i32), ("wave_pull", i32),
        ("dense_blas", i32), ("qn_inkernel_waves", i32), ("qn_batches", i32),
    ]


# int fn(void* user, void* buf, int64_t count, int32_t op) (wfsa_host_allreduce_fn)
HOST_ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, vp, vp, i64, i32)


class LearnerInfo(C.Structure):
    _fields_ = [
        ("n_strings", i64), ("n_local_strings", i64), ("n_paths", i64),
        ("n_full", i32), ("n_params", i32), ("n_constraints", i32), ("unique_paths", i32),
        ("aux_params", i64),
        ("common_support", dbl), ("plogp", dbl), ("model_volume", dbl), ("aux_hessian", dbl),
        ("kl", dbl), ("loglik", dbl), ("shard_begin", i64), ("shard_end", i64),
    ]


# name -> (restype, argtypes)
_SIGS = {
    # device boundary (wfsa_dev.h)
    "wfsa_dev_create": (C.c_int, [C.c_int, P(vp)]),
    "wfsa_dev_destroy": (None, [vp]),
    "wfsa_dev_last_error": (C.c_char_p, []),
    "wfsa_dev_load_model": (C.c_int, [vp, P(ModelDesc)]),
    "wfsa_dev_load_corpus": (C.c_int, [vp, vp, vp, vp, i64]),
    "wfsa_dev_recognize": (C.c_int, [vp, vp, vp, vp]),
    "wfsa_dev_string_tiers": (C.c_int, [vp, vp]),
    "wfsa_dev_rmin": (C.c_int, [vp, vp, vp]),
    "wfsa_dev_sym_factor": (C.c_int, [vp, C.c_int64, vp, vp, vp, vp]),
    "wfsa_dev_sym_solve": (C.c_int, [vp, vp]),
    "wfsa_dev_sym_factor_coo": (C.c_int, [vp, C.c_int64, C.c_int64, vp, vp, vp, vp, vp, vp, vp, vp]),
    "wfsa_dev_load_paths": (C.c_int, [vp, C.c_int32, C.c_int64, vp, vp, vp, C.c_int64, vp, vp, vp]),
    "wfsa_learner_load_matrices": (C.c_int, [vp, C.c_char_p]),
    "wfsa_learner_set_info_rmin": (C.c_int, [vp, C.c_int]),
    "wfsa_learner_save_matrices": (C.c_int, [vp, C.c_char_p]),
    "wfsa_dev_objective_grad": (C.c_int, [vp, vp, P(dbl), vp, vp]),
    "wfsa_dev_objective_grad_begin": (C.c_int, [vp, vp, C.c_int]),
    "wfsa_dev_weights_staging": (vp, [vp]),
    "wfsa_dev_objective_grad_end": (C.c_int, [vp, P(dbl), vp, vp]),
    "wfsa_dev_qn_setup": (C.c_int, [vp, vp]),
    "wfsa_dev_qn_set_state": (C.c_int, [vp, vp, vp]),
    "wfsa_dev_qn_get_state": (C.c_int, [vp, vp, vp, vp]),
    "wfsa_dev_qn_run": (C.c_int, [vp, dbl, dbl, i32, vp, P(i32), P(i32)]),
    "wfsa_dev_hf_setup": (C.c_int, [vp, P(C.c_int64)]),
    "wfsa_dev_hf_pairs": (C.c_int, [vp, vp]),
    "wfsa_dev_hf_eval": (C.c_int, [vp, vp, vp]),
    "wfsa_dev_comm_unique_id": (C.c_int, [vp]),
    "wfsa_dev_comm_init": (C.c_int, [vp, C.c_int, C.c_int, vp]),
    "wfsa_dev_comm_local_id": (C.c_int, [C.c_int, vp]),
    "wfsa_dev_allreduce": (C.c_int, [vp, vp, i64]),
    "wfsa_dev_comm_abort": (C.c_int, [vp, C.c_char_p]),
    "wfsa_dev_peer_selftest": (C.c_int, [C.c_int, C.c_int, i64, C.c_double, C.c_int, vp]),
    "wfsa_dev_comm_init_host": (C.c_int, [vp, C.c_int, C.c_int, vp, vp]),
    "wfsa_dev_get_stats": (C.c_int, [vp, P(DevStats)]),
    # host mirror (wfsa_host.h)
    "wfsa_host_last_error": (C.c_char_p, []),
    "wfsa_fsa_read_text": (C.c_int, [C.c_char_p, P(vp)]),
    "wfsa_fsa_read_file": (C.c_int, [C.c_char_p, P(vp)]),
    "wfsa_fsa_free": (None, [vp]),
    "wfsa_fsa_desc": (C.c_int, [vp, P(ModelDesc)]),
    "wfsa_fsa_counts": (C.c_int, [vp, vp]),
    "wfsa_fsa_param_name": (C.c_int, [vp, i32, P(C.c_char_p), P(i32), P(C.c_char_p)]),
    "wfsa_corpus_read_text": (C.c_int, [C.c_char_p, P(vp)]),
    "wfsa_corpus_read_file": (C.c_int, [C.c_char_p, P(vp)]),
    "wfsa_corpus_free": (None, [vp]),
    "wfsa_corpus_view": (C.c_int, [vp, P(vp), P(vp), P(vp), P(i64)]),
    "wfsa_learner_create": (C.c_int, [C.c_char_p, C.c_int, P(vp)]),
    "wfsa_learner_destroy": (None, [vp]),
    "wfsa_learner_set_comm": (C.c_int, [vp, C.c_int, C.c_int, vp]),
    "wfsa_learner_set_comm_host": (C.c_int, [vp, C.c_int, C.c_int, vp, vp]),
    "wfsa_learner_comm_abort": (C.c_int, [vp, C.c_char_p]),
    "wfsa_learner_build": (C.c_int, [vp, vp, vp]),
    "wfsa_learner_build_packed": (C.c_int, [vp, vp, vp, vp, vp, i64]),
    "wfsa_learner_finalize": (C.c_int, [vp]),
    "wfsa_learner_info_get": (C.c_int, [vp, P(LearnerInfo)]),
    "wfsa_learner_init": (C.c_int, [vp, C.c_int, vp]),
    "wfsa_learner_info_width": (C.c_int, [vp]),
    "wfsa_learner_step": (C.c_int, [vp, dbl, dbl, vp, P(i32)]),
    "wfsa_learner_result": (C.c_int, [vp, vp]),
    "wfsa_learner_run": (C.c_int, [vp, dbl, dbl, i32, vp, P(i32)]),
    "wfsa_learner_objective_grad": (C.c_int, [vp, P(dbl), vp, vp]),
    "wfsa_learner_get_x": (C.c_int, [vp, vp]),
    "wfsa_learner_get_grad": (C.c_int, [vp, vp]),
    "wfsa_learner_set_x": (C.c_int, [vp, vp]),
    "wfsa_learner_get_p": (C.c_int, [vp, vp]),
    "wfsa_learner_trimmed_index": (C.c_int, [vp, vp]),
    "wfsa_learner_path_counts": (C.c_int, [vp, vp, vp]),
    "wfsa_learner_renormalize": (C.c_int, [vp]),
    "wfsa_learner_dump": (C.c_int, [vp, vp, C.c_char_p]),
    "wfsa_learner_stats": (C.c_int, [vp, P(DevStats)]),
    "wfsa_shard_range": (C.c_int, [vp, i64, C.c_int, C.c_int, P(i64), P(i64)]),
    "wfsa_sym_sparse_solve": (C.c_int, [i64, i64, vp, vp, vp, C.c_int, vp, vp, vp, vp]),
    "wfsa_trellis_compile_stats": (C.c_int, [P(ModelDesc), vp]),
    "wfsa_synth_make": (C.c_int, [i32, i32, i32, i32, i32, i64, i32, C.c_uint64, P(vp)]),
    "wfsa_synth_free": (None, [vp]),
    "wfsa_synth_wfsa_text": (C.c_char_p, [vp]),
    "wfsa_synth_corpus": (C.c_int, [vp, P(vp), P(vp), P(vp), P(i64)]),
}

EXPORTS = tuple(_SIGS)

_lib = None


class WfsaError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def load():
    """Load the in-tree library; raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `make -C w-fsa_amd/csrc` "
                              "(or __graft_entry__.build()); there is no CPU fallback")
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check_dev(rc):
    if rc != WFSA_OK:
        raise WfsaError(rc, load().wfsa_dev_last_error().decode(errors="replace"))


def check_host(rc):
    if rc != WFSA_OK:
        raise WfsaError(rc, load().wfsa_host_last_error().decode(errors="replace"))
