#!/usr/bin/env python3
"""Benchmark of the MI355X forward-backward / objective-gradient path.

Headline workload (BASELINE.json configs[2], SURVEY.md 8d "c3"): synthetic
family-A automaton (1024 states, out-degree 8 + end, one symbol per state out
of 64), 1M distinct strings sampled from it (mean length ~36, capped at 128).
With N > 1 GPUs the per-GPU shard is c4's (configs[3]: 10M strings over 8
GPUs = 1.25M per GPU), weak scaling.

One step = one QuasiNewtonLearner::OptimizationStep over the whole corpus,
run DEVICE-RESIDENT: main.cpp's epoch loop is wfsa_learner_run ->
wfsa_dev_qn_run, which enqueues per step the forward-backward kernels (stream
+ bubble + traversal tiers), [the RCCL all-reduce of the gradient], and the QN
update (x, lambda and the next weights stay in HBM; each step's info row lands
in host-mapped memory).  At c3 that is ONE launch per step: the stream kernel
with the bubbles and the QN update inside; across ranks too, the
QN batches' partials then summed over the ranks through the peer areas inside
that launch.  Inputs are resident in HBM.  The same steps
through the host binding of INTEGRATION.md section 2 (wfsa_dev_objective_grad
per step: H2D weights, D2H [LL, grad], host QN update) are timed beside it
(`boundary`).

Multi-GPU: launched by torch.distributed.run, one process per GPU (`--gpus N`
without a launcher starts the N ranks itself, or refuses when the node has
fewer GPUs); every rank builds the same global corpus and keeps a contiguous
shard (Learner::BuildFrom); the gradient + log-likelihood are summed once per
step over xGMI through the peer areas, inside the stream kernel's QN waves
(the two-kernel step: the one-shot peer all-reduce kernel; RCCL's own
all-reduce if the peer path's set-up check fails -- `comm` in the line says
which).

After the headline (one GPU only) two sub-records run in the same process,
each with its own roofline and CPU baseline: `dense_c5` (configs[4], the
fp64 MFMA path) and `famB` (SURVEY 8d family B, the ambiguous automaton that
runs on the traversal tiers).

Prints ONE JSON line (rank 0).
"""
import argparse
import gc
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
F64_MFMA_PEAK_TFS = 78.6     # MI355X spec: FP64 matrix (dense) 78.6 TF (= the FP64 vector rate)
METRIC = "forward-backward strings/sec @1/2/4/8 GPU; log-lik rel-err vs MKL ref"

# SURVEY.md 8d families: automaton, corpus size per GPU, default steps/warmup, CPU sample
WORKLOADS = {
    "c3": dict(states=1024, degree=8, vocab=64, emissions=1, dense=False, strings_per_gpu=1_000_000,
               steps=200, warmup=10, cpu_sample=200_000),
    "c5": dict(states=4096, degree=8, vocab=16, emissions=16, dense=True, strings_per_gpu=4096,
               steps=10, warmup=2, cpu_sample=1),
    "famB": dict(states=1024, degree=8, vocab=16, emissions=4, dense=False, strings_per_gpu=100_000,
                 steps=10, warmup=2, cpu_sample=400),
}
C4_STRINGS_PER_GPU = 1_250_000   # configs[3]: 10M strings over 8 GPUs


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", choices=tuple(WORKLOADS), default="c3",
                    help="c3: 1024-state sparse family A, 1M strings/GPU (the headline; c4 sizing with N > 1); "
                         "c5: dense 4096-state automaton on the fp64 MFMA path; famB: SURVEY 8d family B")
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--strings-per-gpu", type=int, default=None)
    ap.add_argument("--states", type=int, default=None)
    ap.add_argument("--degree", type=int, default=None)
    ap.add_argument("--vocab", type=int, default=None)
    ap.add_argument("--emissions", type=int, default=None)
    ap.add_argument("--max-len", type=int, default=128)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--info-rmin", action="store_true",
                    help="time the headline steps with the rmin info column on (default: measured in a "
                         "second pass and reported as info_rmin; SURVEY 8d's timed region leaves it out)")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="strings timed through the CPU oracle (0 = skip)")
    ap.add_argument("--no-sub", action="store_true", help="skip the dense_c5 / famB sub-records")
    ap.add_argument("--boundary-steps", type=int, default=50,
                    help="steps timed through the host binding (wfsa_dev_objective_grad per step; 0 = skip)")
    ap.add_argument("--profile-traffic", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="committed PMC traffic measurement to quote (if present)")
    return ap.parse_args()


def workload_args(args, name, world):
    """the workload's parameters, command-line overrides applied to the headline only"""
    w = dict(WORKLOADS[name])
    w["name"] = name
    if name == "c3" and world > 1:
        w["strings_per_gpu"] = C4_STRINGS_PER_GPU
        w["name"] = "c4"
    if name == args.workload:
        for k in ("steps", "warmup", "strings_per_gpu", "states", "degree", "vocab", "emissions", "cpu_sample"):
            v = getattr(args, k)
            if v is not None:
                w[k] = v
    w["max_len"] = args.max_len
    w["seed"] = args.seed
    return w


def host_cpu():
    """CPU model, logical CPUs of the machine, CPUs this process may use, and
    the OpenMP threads the multi-core baselines use (OMP_NUM_THREADS, capped
    by the CPUs available; the GPU box grants 16 per GPU)"""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 1
    want = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or avail
    return {"cpu_model": model, "nproc": os.cpu_count(), "cpus_available": avail,
            "omp_threads": max(1, min(want, avail, 16))}


def cpu_baseline_enum(syn_text, sym, off, wt, n_sample):
    """Reference algorithm restated in C (oracle/): BFS path enumeration once,
    then the SpMV chain per iteration, one core.  Also the log-likelihood of
    the same sample through the device path, for the rel-err column."""
    from oracle import ENUM, Oracle, TRELLIS
    import wfsa_amd as W
    n = min(n_sample, len(wt))
    s_off = off[: n + 1].copy()
    s_sym = sym[: s_off[-1]].copy()
    s_wt = wt[:n].copy()
    t0 = time.perf_counter()
    os.environ["ORACLE_BUILD_THREADS"] = "1"   # the reference's enumeration is sequential (mkl_sequential build)
    try:
        o = Oracle.from_arrays(syn_text, s_sym, s_off, s_wt, mode=ENUM, max_paths=1_000_000)
    finally:
        os.environ.pop("ORACLE_BUILD_THREADS", None)
    t_build = time.perf_counter() - t0
    o.qn_init(7)
    iters = 3
    t0 = time.perf_counter()
    for _ in range(iters):
        kl_ref, ll_ref = o.objective_grad()
    t_iter = (time.perf_counter() - t0) / iters
    S = o.info["n_strings"]
    host = host_cpu()
    nt = host["omp_threads"]
    # the same SpMV chain on every granted core (OpenMP over paths / strings)
    o.set_threads(nt)
    o.objective_grad()
    t0 = time.perf_counter()
    for _ in range(iters):
        o.objective_grad()
    t_iter_mt = (time.perf_counter() - t0) / iters
    o.set_threads(1)
    # the trellis restatement (oracle TRELLIS: forward-backward per string,
    # OpenMP over strings) on a hundredth of the sample (it visits every state
    # at every position: ~1 ms per family-A string on one core)
    nt_s = max(1, n // 100)
    t_off = off[: nt_s + 1].copy()
    ot = Oracle.from_arrays(syn_text, sym[: t_off[-1]].copy(), t_off, wt[:nt_s].copy(), mode=TRELLIS)
    ot.set_threads(nt)
    wt_full = np.array(ot.w_full())
    ot.trellis_eval(wt_full)
    t0 = time.perf_counter()
    ot.trellis_eval(wt_full)
    t_trel = time.perf_counter() - t0
    # the same sample through the device
    fsa = W.Fsa.read_text(syn_text)
    lrn = W.QuasiNewtonLearner(0)
    lrn.BuildFromPacked(fsa, s_sym, s_off, s_wt)
    lrn.Finalize()
    lrn.Init(7)
    lrn.objective_grad()
    ll_dev = lrn.info()["loglik"]
    rel = abs(ll_dev - ll_ref) / abs(ll_ref)
    return {
        "value": S / t_iter, "unit": "strings/s", "cores": 1, "kind": "port",
        "sample": (f"first {n} strings of the same corpus; oracle/wfsa_oracle.c ENUM = the reference "
                   f"algorithm (BFS path enumeration {t_build:.2f} s once = {S / t_build:.0f} strings/s, "
                   f"then the P/M SpMV chain: {t_iter * 1e3:.1f} ms per objective+gradient)"),
        "enumeration_s": t_build, "iteration_s": t_iter, "paths": o.info["n_paths"],
        "multi_core": {"value": S / t_iter_mt, "unit": "strings/s", "cores": nt, "kind": "port",
                       "iteration_s": t_iter_mt,
                       "sample": f"the same {n} strings, ENUM SpMV chain with {nt} OpenMP threads"},
        "trellis_omp": {"value": nt_s / t_trel, "unit": "strings/s", "cores": nt, "kind": "port",
                        "iteration_s": t_trel,
                        "sample": f"first {nt_s} strings, oracle TRELLIS forward-backward, {nt} OpenMP threads"},
        "host": host,
    }, rel


def cpu_baseline_trellis(syn_text, sym, off, wt, n_sample, why):
    """The oracle's trellis restatement (oracle/wfsa_oracle.c TRELLIS: dense
    float64 forward-backward per string, one core) on the first strings of the
    corpus, for automata whose paths the reference algorithm cannot enumerate."""
    from oracle import Oracle, TRELLIS
    n = min(n_sample, len(wt))
    s_off = off[: n + 1].copy()
    s_sym = sym[: s_off[-1]].copy()
    t0 = time.perf_counter()
    o = Oracle.from_arrays(syn_text, s_sym, s_off, wt[:n].copy(), mode=TRELLIS)
    t_build = time.perf_counter() - t0
    w = np.array(o.w_full())
    t0 = time.perf_counter()
    o.trellis_eval(w)
    t_eval = time.perf_counter() - t0
    return {
        "value": n / t_eval, "unit": "strings/s", "cores": 1, "kind": "port",
        "sample": (f"first {n} string(s) ({int(s_off[-1])} symbols) of the same corpus through oracle/wfsa_oracle.c "
                   f"TRELLIS (dense fp64 forward-backward, one core): {t_eval:.2f} s per evaluation; "
                   f"build incl. its structural pass {t_build:.1f} s; {why}"),
        "iteration_s": t_eval,
        "host": host_cpu(),
    }


def run_workload(wl, world, rank, local_rank, distributed, dist, torch, info_rmin=False):
    """build, warm up, time `steps` device-resident QN steps; returns the
    measurement and the objects the extras need"""
    import wfsa_amd as W
    # torch's own HIP start-up (its first CUDA call) here rather than in the
    # barrier between the warmup and the timed steps: it idles the GPU for
    # long enough that the timed steps start at a lower clock (measured: a
    # 50 ms pause before the timed Run costs 35 -> 45 us per c3 step,
    # tools/bench_like.py)
    torch.cuda.synchronize()
    total = wl["strings_per_gpu"] * world
    syn = W.Synthetic(n_states=wl["states"], degree=wl["degree"], vocab=wl["vocab"], emissions=wl["emissions"],
                      dense=wl["dense"], n_strings=total, max_len=wl["max_len"], seed=wl["seed"])
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    lrn = W.QuasiNewtonLearner(device=local_rank)
    if distributed:
        uid = [W.Device.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        lrn.SetCommunicator(world, rank, uid[0])
    t0 = time.perf_counter()
    lrn.BuildFromPacked(fsa, sym, off, wt)
    t_build = time.perf_counter() - t0
    lrn.Finalize()
    lrn.Init(7)
    lrn.set_info_rmin(info_rmin)
    info = lrn.info()

    def barrier():
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()

    # main.cpp's epoch loop runs natively (wfsa_learner_run); tol < 0 never
    # halts, so exactly `steps` OptimizationSteps run.  No cyclic garbage
    # collection from the warmup to the end of the timed region: a collection
    # pass over torch's heap costs tens of microseconds of host time inside it,
    # and milliseconds between the warmup and the timed steps idle the GPU
    # long enough for its clock to drop (the timed steps then start slow)
    gc.collect()
    gc.disable()
    if wl["warmup"]:
        lrn.Run(wl["warmup"], 1.0, -1.0)
    st0 = lrn.stats()
    barrier()
    t0 = time.perf_counter()
    ns0 = time.monotonic_ns()
    rows = lrn.Run(wl["steps"], 1.0, -1.0)
    ns1 = time.monotonic_ns()
    t_run = time.perf_counter()
    barrier()
    dt = time.perf_counter() - t0
    gc.enable()
    if os.environ.get("WFSA_BENCH_TRACE"):   # (diagnostics: where the timed region's wall time goes)
        print(f"[bench] timed region {dt * 1e6:.1f} us: Run {1e6 * (t_run - t0):.1f}, barrier {1e6 * (t0 + dt - t_run):.1f}"
              f" (Run call at {ns0} ns, returned at {ns1} ns)", file=sys.stderr, flush=True)
    assert len(rows) == wl["steps"]
    st1 = lrn.stats()
    if distributed:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dict(wl=wl, syn=syn, sym=sym, off=off, wt=wt, fsa=fsa, lrn=lrn, info=info, st0=st0, st1=st1, dt=dt,
                t_build=t_build, barrier=barrier,
                value=info["n_strings"] * wl["steps"] / dt, ms_per_step=dt * 1e3 / wl["steps"],
                local_sym=int(off[info["shard_end"]] - off[info["shard_begin"]]))


def workload_label(wl, off):
    mean = float(np.diff(off).mean())
    if wl["dense"]:
        return (f"{wl['name']} dense: {wl['states']}-state WFSA, full transition matrix (every S->T and S->$), every "
                f"state emits every one of {wl['vocab']} symbols, {wl['strings_per_gpu']} distinct strings per GPU "
                f"sampled from it (mean len {mean:.1f}, max {wl['max_len']})")
    fam = "family A" if wl["emissions"] == 1 else "family B"
    return (f"{wl['name']} {fam}: {wl['states']}-state sparse WFSA, out-degree {wl['degree']}+end, "
            f"{wl['emissions']} of {wl['vocab']} symbols/state, {wl['strings_per_gpu']} distinct strings per GPU "
            f"(mean len {mean:.1f}, max {wl['max_len']})")


def roofline_of(m, traffic):
    """the dominant kernel's roofline: fbs_kernel (compiled streams, c3/c4),
    the dense GEMM evaluation (c5), the traversal tiers (family B)"""
    wl, st0, st1 = m["wl"], m["st0"], m["st1"]
    timed = max(st1["fb_launches"] - st0["fb_launches"], 1)
    kern_ms = (st1["compiled_kernel_ms"] - st0["compiled_kernel_ms"]) / timed   # k0..kc: the stream kernel
    fb_ms = (st1["fb_kernel_ms"] - st0["fb_kernel_ms"]) / timed                 # k0..k2: every evaluation kernel
    local_strings = max(m["info"]["n_local_strings"], 1)
    mean_sym = m["local_sym"] / local_strings
    if wl["dense"]:
        # 3 GEMM-equivalents of 2 N^2 flops per string
        # position (forward, backward, gradient); every evaluation kernel is
        # inside the timed span (weights, GEMMs, log q, reductions)
        N = wl["states"]
        alg_flops = 6.0 * N * N * m["local_sym"]
        npd, R, T = st1["dense_np"], st1["dense_rows"], st1["dense_steps"]
        tf = alg_flops / (fb_ms * 1e-3) / 1e12 if fb_ms > 0 else None
        return {"bound": "mfma", "achieved": tf, "peak": F64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                "frac": tf / F64_MFMA_PEAK_TFS if tf else None, "traffic": None,
                "kernel": {1: "rocblas_dgemm (library fp64 MFMA GEMMs) + our epilogue kernels, one evaluation",
                           2: "dense_gemm_kernel<RAW> (hand-written v_mfma_f64_16x16x4f64, 8-wave 128x128 blocks, K in "
                              "two halves) + dense_gemm_kernel<GRAD> + our epilogue kernels, one evaluation",
                           3: "dense GEMMs with LDS-DMA pipelined tiles (hand-written v_mfma_f64_16x16x4f64, "
                              "WFSA_DENSE_ENGINE=dma) + our epilogue kernels, one evaluation"}.get(
                               st1.get("dense_blas", 0),
                               "dense_gemm_kernel<FWD/BWD/GRAD> (hand-written v_mfma_f64_16x16x4f64, epilogues "
                               "fused), one evaluation"),
                "timed_launches": timed, "evaluation_ms": fb_ms, "algorithmic_flops_per_evaluation": alg_flops,
                "issued_flops_per_evaluation": 6.0 * npd * npd * R * max(T - 1, 0), "row_slots": R, "trellis_steps": T}
    comp = st1["compiled_strings"]
    trav = st1["fallback_strings"]
    live = st1["last_live_edges"]
    if comp >= trav:   # the stream kernel dominates (c3/c4)
        alg_bytes = int(mean_sym * comp) + 16 * comp   # string bytes + offset + p per string
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else None   # None: WFSA_TIMING=0
        return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS if achieved else None, "traffic": traffic,
                "traffic_source": ("a committed lease measurement, not taken in this run: "
                                   "profiles/traffic_latest.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes "
                                   "over bench.py on this kernel, corrected per MI355X_MICROARCH.md, per launch)")
                if traffic else None,
                "kernel": "fbs_kernel (compiled-stream forward pass + fused bubbles, per step)",
                "timed_launches": timed, "kernel_ms_per_launch": kern_ms, "all_fb_kernels_ms_per_step": fb_ms,
                "algorithmic_bytes_per_launch": alg_bytes,
                "note": ("one launch per QN step: staging of the weight table (~4.3 us), the fused bubbles "
                         "(write-through slots, an arrival counter), the delta-format stream pass, and the QN "
                         "update's waves after the last bubble arrival (profiles/r05/fbs_trace_fit.log).  PMC "
                         "(profiles/r05/profile/pmc.txt, profiles/traffic_latest.json): 86.2 MB of HBM traffic "
                         "per launch (1.67x the algorithmic bytes), waves waiting 66% of their cycles, LDS bank "
                         "conflicts 53% of LDS-active cycles; the launch's end is the QN tail and the slowest "
                         "stream waves, not the stream's bytes.  The kernel time is from HIP events attached to "
                         "its dispatch (hipExtLaunchKernelGGL start/stop); rocprof's average is ~1-3 us lower "
                         "(DESIGN 6)")}
    # family B: the traversal strings (k_c..k_2 of the evaluation)
    trav_ms = max(fb_ms - kern_ms, 1e-9)
    rows, pedges = st1.get("wave_row_entries", 0), st1.get("wave_pair_edges", 0)
    alg_bytes = int(mean_sym * trav) + 16 * trav   # string bytes + offset + p per string
    extra = {}
    if st1.get("wave_strings", 0) > 0:
        pull = st1.get("wave_pull", 0)
        kernel = ("wave_pull_kernel (traversal strings: a wavefront per string, each step's nodes pulled lane by "
                  "lane over the byte-pair edge lists)" if pull else
                  "wide2_kernel (traversal strings: a wavefront per string over byte-pair edge lists, LDS rows)")
        note = ("frac is against the algorithmic bytes (SURVEY 8d: string bytes + offset + p), which this pass "
                "is far from: a dependent per-position chain of L2 loads, LDS gathers and LDS fixed-point "
                "gradient adds per string, 16 strings in flight per CU.  PMC (profiles/r05/famb/pmc.txt): waves "
                "wait 55% of their cycles, LDS bank conflicts 61% of LDS-active cycles, L2 hit rate 69%, and "
                "2.7-4.7 TB/s of HBM traffic (raw / calibrated FETCH_SIZE + WRITE_SIZE): the alpha history "
                "(every row written and read back, alpha_history_bytes) and L2 misses on the byte-pair entry "
                "tables, so the pass is HBM-loaded as well as latency-bound")
        extra = {"alpha_history_bytes": 16 * rows, "nodes_per_lane": pull}
    else:
        kernel = "traversal tiers (trav_kernel<MODE_WEIGHTED> tiers 0/1 + wide_kernel tier 2), per step"
        note = "HBM is not the binding level here (SURVEY 8d: a dependent L-step chain + LDS/L2 gathers)"
    achieved = alg_bytes / (trav_ms * 1e-3) / 1e9
    out = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": kernel,
           "timed_launches": timed, "kernel_ms_per_launch": trav_ms, "all_fb_kernels_ms_per_step": fb_ms,
           "algorithmic_bytes_per_launch": alg_bytes, "traversal_strings": trav, "note": note, **extra}
    if pedges > 0:
        out.update({"alpha_entries_per_evaluation": rows, "pair_edges_per_pass": pedges,
                    "pair_edge_visits_per_s": 2.0 * pedges / (trav_ms * 1e-3)})
    if live > 0:   # ~6 fp64 flops per live trellis edge (forward FMA, backward FMA, posterior mul+add)
        eps = live / (fb_ms * 1e-3)
        out.update({"live_edges_per_evaluation": live, "edge_ops_per_s": eps,
                    "fp64_flops_frac": 6.0 * eps / (F64_MFMA_PEAK_TFS * 1e12)})
    return out


def boundary_steps(m, k):
    """the same steps through the host binding (INTEGRATION.md section 2:
    wfsa_dev_objective_grad per step, H2D weights, D2H [LL, grad], host QN update)"""
    lrn = m["lrn"]
    lrn.Init(7)
    for _ in range(3):
        lrn.OptimizationStep(1.0, -1.0)
    m["barrier"]()
    s0 = lrn.stats()
    t0 = time.perf_counter()
    for _ in range(k):
        lrn.OptimizationStep(1.0, -1.0)
    m["barrier"]()
    dt = time.perf_counter() - t0
    s1 = lrn.stats()
    host = {f: (s1[f] - s0[f]) / k for f in ("host_begin_ms", "host_overlap_ms", "host_wait_ms", "host_post_ms")}
    return {"ms_per_step": dt * 1e3 / k, "value": m["info"]["n_strings"] * k / dt, "steps": k,
            "host_ms_per_step": host,
            "note": "QuasiNewtonLearner::OptimizationStep through the C ABI a maintainer binds (wfsa_dev_objective_grad: "
                    "host weights in over PCIe, [LL, grad] out, the QN update on the host)"}


def record(m, traffic, cpu):
    wl = m["wl"]
    return {"metric": METRIC, "value": m["value"], "unit": "strings/s", "steps": wl["steps"], "warmup": wl["warmup"],
            "ms_per_step": m["ms_per_step"], "dtype": "f64",
            "config": {"workload": workload_label(wl, m["off"]), "strings_per_gpu": wl["strings_per_gpu"],
                       "step": "device-resident QN loop (wfsa_dev_qn_run: evaluation kernels + the QN update per step)"},
            "roofline": roofline_of(m, traffic), "cpu_baseline": cpu,
            "compiled_strings": m["st1"]["compiled_strings"], "fallback_strings": m["st1"]["fallback_strings"],
            "tier2_strings": m["st1"]["tier2_strings"], "build_s": m["t_build"]}


def launch_ranks(n):
    """`bench.py --gpus N` (N > 1) started without a launcher: start the N rank
    processes as fresh children through torch.distributed.run, before this
    process touches the GPU, and exit with their status.  Refuses (exit 2)
    when the node has fewer than N GPUs -- it never reports N GPUs from one."""
    import socket
    import subprocess
    import torch   # device_count() does not initialise the GPU on this image
    have = torch.cuda.device_count()
    if have < n:
        print(f"bench.py: --gpus {n} needs {n} GPUs on this node, {have} visible; refusing", file=sys.stderr)
        sys.exit(2)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def main():
    args = parse()
    knobs = sorted(k for k in os.environ if (k.startswith("WFSA_") and k.endswith("_DBG")) or k == "WFSA_LIB")
    if knobs:   # timing experiments that skip work: never inside a measurement
        print(f"bench.py: refusing to measure with {', '.join(knobs)} set", file=sys.stderr)
        sys.exit(2)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        launch_ranks(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus not in (1, world):   # (a launcher without --gpus: the default 1 means "one per rank")
        print(f"bench.py: --gpus {args.gpus} but {world} rank process(es); refusing", file=sys.stderr)
        sys.exit(2)
    n_gpus = world   # the rank processes actually running, one GPU each
    import torch
    import torch.distributed as dist
    distributed = world > 1
    if distributed:
        dist.init_process_group("gloo")   # rendezvous / timing barrier only; the data path is RCCL
    torch.cuda.set_device(local_rank)

    wl = workload_args(args, args.workload, world)
    m = run_workload(wl, world, rank, local_rank, distributed, dist, torch, info_rmin=args.info_rmin)
    lrn, st1 = m["lrn"], m["st1"]
    traffic = None
    if not wl["dense"] and wl["emissions"] == 1 and os.path.exists(args.profile_traffic):
        try:
            tj = json.load(open(args.profile_traffic))
            traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    # the same steps with the rmin info column (QuasiNewtonLearner::
    # GetOptimizationInfo's smallest relative path probability), which the
    # reference prints each epoch but computes outside OptimizationStep
    rmin_pass = None
    if not args.info_rmin and not distributed and not wl["dense"] and not args.no_sub:
        lrn.set_info_rmin(True)
        lrn.Run(max(wl["warmup"], 10), 1.0, -1.0)   # (its set-up, then the clock back up: as the headline's warmup)
        m["barrier"]()
        t1 = time.perf_counter()
        rrows = lrn.Run(wl["steps"], 1.0, -1.0)
        m["barrier"]()
        dtr = time.perf_counter() - t1
        rmin_pass = {"ms_per_step": dtr * 1e3 / wl["steps"], "value": m["info"]["n_strings"] * wl["steps"] / dtr,
                     "last_rmin": float(rrows[-1][5]) if len(rrows) else None,
                     "note": "the headline steps plus the rmin info column (the (min, x) passes fused into "
                             "the evaluation's bubble / traversal kernels)"}
        lrn.set_info_rmin(False)
    # (one GPU only: a sub-record must never leave ranks waiting in a collective)
    boundary = boundary_steps(m, args.boundary_steps) if args.boundary_steps > 0 and not distributed else None

    out = {
        "metric": METRIC,
        "value": m["value"],
        "unit": "strings/s",
        "n_gpus": n_gpus,
        "steps": wl["steps"],
        "warmup": wl["warmup"],
        "ms_per_step": m["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": workload_label(wl, m["off"]),
            "global_strings": m["info"]["n_strings"],
            "strings_per_gpu": wl["strings_per_gpu"],
            "parallelism": f"dp{n_gpus}",
            "step": ("device-resident QN loop: wfsa_learner_run -> wfsa_dev_qn_run enqueues per step " +
                     ("the forward-backward kernels, the RCCL all-reduce and the QN step kernel"
                      if distributed or not st1.get("qn_inkernel_waves") else
                      "ONE stream kernel with the bubbles and the QN update inside (%d QN waves)"
                      % st1.get("qn_inkernel_waves", 0)) +
                     " (x, lambda, weights stay in HBM; info rows to host-mapped memory)"),
            "info_rmin": bool(args.info_rmin),
        },
        "roofline": roofline_of(m, traffic),
        "info_rmin": rmin_pass,
        "boundary": boundary,
        "comm": ({"transport": "rccl", "ranks": st1.get("comm_ranks", world),
                  "per_step_sum": ("the QN batches' partials through the peer areas (xGMI), inside the stream kernel"
                                   if st1.get("qn_inkernel_waves") else
                                   {1: "one-shot peer all-reduce (xGMI)", 0: "ncclAllReduce",
                                    -1: "ncclAllReduce (peer set-up check failed)"}.get(st1.get("comm_peer", 0)))}
                 if distributed else None),
        "experiment_knobs": "none (WFSA_*_DBG refused; compiled out of the release library)",
        "live_edges_per_step": st1["last_live_edges"],
        "build_s": m["t_build"],
        "tier1_strings": st1["tier1_strings"],
        "tier2_strings": st1["tier2_strings"],
        "compiled_strings": st1["compiled_strings"],
        "fallback_strings": st1["fallback_strings"],
        "stream_words": st1["stream_words"],
        "n_bubbles": st1["n_bubbles"],
        "bubble_words": st1["bubble_words"],
        "prepare_ms": st1["prepare_ms"],
    }
    cpu_n = wl["cpu_sample"]
    if rank == 0 and world == 1 and cpu_n > 0:
        if wl["dense"]:
            out["cpu_baseline"] = cpu_baseline_trellis(m["syn"].wfsa_text, m["sym"], m["off"], m["wt"], cpu_n,
                                                       "path enumeration (the reference algorithm) is infeasible here")
        elif wl["emissions"] == 1:
            cb, rel = cpu_baseline_enum(m["syn"].wfsa_text, m["sym"], m["off"], m["wt"], cpu_n)
            out["cpu_baseline"] = cb
            out["ll_rel_err_vs_reference_algorithm"] = rel
        else:
            out["cpu_baseline"] = cpu_baseline_trellis(m["syn"].wfsa_text, m["sym"], m["off"], m["wt"], cpu_n,
                                                       "the reference's BFS truncates or drops these ambiguous strings")
    else:
        out["cpu_baseline"] = None
    del m, lrn
    # the sub-records: configs[4] (dense, MFMA) and family B (traversal tiers)
    # (dense_c5_rocblas: the same c5 run with rocBLAS dgemm for the GEMMs, the
    # library reference for the hand-written engine's roofline fraction)
    if not distributed and not args.no_sub and args.workload == "c3":
        for key in ("dense_c5", "famB", "dense_c5_rocblas"):
            name = "famB" if key == "famB" else "c5"
            sw = workload_args(args, name, 1)
            engine = os.environ.get("WFSA_DENSE_ENGINE")
            if key == "dense_c5_rocblas":
                os.environ["WFSA_DENSE_ENGINE"] = "blas"
            try:
                sm = run_workload(sw, 1, 0, local_rank, False, dist, torch)
                cpu = None
                if sw["cpu_sample"] > 0 and args.cpu_sample != 0 and key != "dense_c5_rocblas":
                    why = ("path enumeration (the reference algorithm) is infeasible here" if sw["dense"] else
                           "the reference's BFS truncates or drops these ambiguous strings")
                    cpu = cpu_baseline_trellis(sm["syn"].wfsa_text, sm["sym"], sm["off"], sm["wt"], sw["cpu_sample"],
                                               why)
                out[key] = record(sm, None, cpu)
                del sm
            except Exception as e:   # a sub-record never takes the headline down
                out[key] = {"error": f"{type(e).__name__}: {e}"}
            finally:
                if engine is None:
                    os.environ.pop("WFSA_DENSE_ENGINE", None)
                else:
                    os.environ["WFSA_DENSE_ENGINE"] = engine
    if rank == 0:
        print(json.dumps(out), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
