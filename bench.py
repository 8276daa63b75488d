#!/usr/bin/env python3
"""Benchmark of the MI355X forward-backward / objective-gradient path.

Workload (BASELINE.json configs[2], SURVEY.md 8d "c3"): synthetic family-A
automaton (1024 states, out-degree 8 + end, one symbol per state out of 64),
1M distinct strings per GPU sampled from it (mean length ~32, capped at 128).
One step = one QuasiNewtonLearner::OptimizationStep over the whole corpus:
H2D of the weights, the forward-backward kernels, (RCCL all-reduce),
D2H of [loglik, grad], the host O(n) update.  Inputs are resident in HBM.

Multi-GPU (weak scaling): launched by torch.distributed.run, one process per
GPU; every rank builds the same global corpus and keeps a contiguous shard;
the gradient + log-likelihood are summed with one RCCL all-reduce per step.

Prints ONE JSON line (rank 0).
"""
import argparse
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", choices=("c3", "c5"), default="c3",
                    help="c3: 1024-state sparse family A, 1M strings/GPU (the headline); "
                         "c5: dense 4096-state automaton on the fp64 MFMA path")
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--strings-per-gpu", type=int, default=None)
    ap.add_argument("--states", type=int, default=None)
    ap.add_argument("--degree", type=int, default=8)
    ap.add_argument("--vocab", type=int, default=None)
    ap.add_argument("--emissions", type=int, default=None)
    ap.add_argument("--max-len", type=int, default=128)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--info-rmin", action="store_true",
                    help="time the headline steps with the rmin info column on (default: measured in a "
                         "second pass and reported as info_rmin; SURVEY 8d's timed region leaves it out)")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="strings timed through the CPU oracle (0 = skip)")
    ap.add_argument("--profile-traffic", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="committed PMC traffic measurement to quote (if present)")
    a = ap.parse_args()
    dense = a.workload == "c5"
    defaults = dict(steps=(10 if dense else 200), warmup=(2 if dense else 10),
                    strings_per_gpu=(4096 if dense else 1_000_000), states=(4096 if dense else 1024),
                    vocab=(16 if dense else 64), emissions=(16 if dense else 1),
                    cpu_sample=(1 if dense else 200_000))
    for k, v in defaults.items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    return a


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


def cpu_baseline(syn_text, sym, off, wt, n_sample):
    """Reference algorithm restated in C (oracle/): BFS path enumeration once,
    then the SpMV chain per iteration, one core.  Also the log-likelihood of
    the same sample through the device path, for the rel-err column."""
    from oracle import ENUM, Oracle
    import wfsa_amd as W
    n = min(n_sample, len(wt))
    s_off = off[: n + 1].copy()
    s_sym = sym[: s_off[-1]].copy()
    s_wt = wt[:n].copy()
    t0 = time.perf_counter()
    o = Oracle.from_arrays(syn_text, s_sym, s_off, s_wt, mode=ENUM, max_paths=1_000_000)
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
    from oracle import TRELLIS
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
    kl_dev, _, _ = lrn.objective_grad()
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
    }, rel, ll_ref, ll_dev


def cpu_baseline_dense(syn_text, sym, off, wt, n_sample):
    """The oracle's trellis restatement (oracle/wfsa_oracle.c TRELLIS: dense
    float64 forward-backward, one core) on the first strings of the corpus.
    The reference algorithm (BFS path enumeration) cannot run this model:
    a length-32 string has ~4096^32 paths."""
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
    host = host_cpu()
    return {
        "value": n / t_eval, "unit": "strings/s", "cores": 1, "kind": "port",
        "sample": (f"first {n} string(s) ({int(s_off[-1])} symbols) of the same corpus through oracle/wfsa_oracle.c "
                   f"TRELLIS (dense fp64 forward-backward, one core): {t_eval:.1f} s per evaluation; "
                   f"build incl. its structural pass {t_build:.1f} s; path enumeration (the reference "
                   f"algorithm) is infeasible here"),
        "iteration_s": t_eval,
        "host": host,
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    n_gpus = max(args.gpus, world)
    import torch
    import torch.distributed as dist
    distributed = world > 1
    if distributed:
        dist.init_process_group("gloo")   # rendezvous / timing barrier only; the data path is RCCL
    torch.cuda.set_device(local_rank)

    import wfsa_amd as W

    total = args.strings_per_gpu * world
    dense = args.workload == "c5"
    syn = W.Synthetic(n_states=args.states, degree=args.degree, vocab=args.vocab, emissions=args.emissions,
                      dense=dense, n_strings=total, max_len=args.max_len, seed=args.seed)
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
    lrn.set_info_rmin(args.info_rmin)
    info = lrn.info()
    local_sym = int(off[info["shard_end"]] - off[info["shard_begin"]])
    local_strings = info["n_local_strings"]

    def barrier():
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()

    # main.cpp's epoch loop runs natively (wfsa_learner_run); tol < 0 never
    # halts, so exactly `steps` OptimizationSteps run
    if args.warmup:
        lrn.Run(args.warmup, 1.0, -1.0)
    st0 = lrn.stats()
    barrier()
    t0 = time.perf_counter()
    rows = lrn.Run(args.steps, 1.0, -1.0)
    barrier()
    assert len(rows) == args.steps
    dt = time.perf_counter() - t0
    st1 = lrn.stats()
    if distributed:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    strings_all = info["n_strings"]
    value = strings_all * args.steps / dt
    # the same steps with the rmin info column (QuasiNewtonLearner::
    # GetOptimizationInfo's smallest relative path probability), which the
    # reference prints each epoch but computes outside OptimizationStep
    rmin_pass = None
    if not args.info_rmin and not distributed and not dense:
        lrn.set_info_rmin(True)
        lrn.Run(2, 1.0, -1.0)
        barrier()
        t1 = time.perf_counter()
        rrows = lrn.Run(args.steps, 1.0, -1.0)
        barrier()
        dtr = time.perf_counter() - t1
        rmin_pass = {"ms_per_step": dtr * 1e3 / args.steps, "value": strings_all * args.steps / dtr,
                     "last_rmin": float(rrows[-1][5]) if len(rrows) else None,
                     "note": "the headline steps plus the rmin info column (the (min, x) passes fused into "
                             "the evaluation's bubble / traversal kernels)"}
        lrn.set_info_rmin(False)
    # the device times a sample of the steps' kernels with HIP events (every
    # 4th step: an event between two kernels idles the device for a few us)
    timed = max(st1["fb_launches"] - st0["fb_launches"], 1)
    kern_ms = (st1["compiled_kernel_ms"] - st0["compiled_kernel_ms"]) / timed
    fb_ms = (st1["fb_kernel_ms"] - st0["fb_kernel_ms"]) / timed
    # algorithmic bytes: string bytes + offset + p per string,
    # for the strings the compiled kernel serves
    comp = st1["compiled_strings"]
    alg_bytes = int(local_sym * comp / max(local_strings, 1)) + 16 * comp
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else None   # None: WFSA_TIMING=0
    traffic = None
    if not dense and os.path.exists(args.profile_traffic):
        try:
            traffic = json.load(open(args.profile_traffic)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    if dense:
        # 3 GEMM-equivalents of 2 N^2 flops per string
        # position (forward, backward, gradient); every evaluation kernel is
        # inside the timed span (weights, GEMMs, log q, reductions)
        N = args.states
        alg_flops = 6.0 * N * N * local_sym
        npd, R, T = st1["dense_np"], st1["dense_rows"], st1["dense_steps"]
        issued = 6.0 * npd * npd * R * max(T - 1, 0)
        tf = alg_flops / (fb_ms * 1e-3) / 1e12 if fb_ms > 0 else None
        workload = (f"c5 dense: {N}-state WFSA, full transition matrix (every S->T and S->$), every state "
                    f"emits every one of {args.vocab} symbols, {args.strings_per_gpu} distinct strings per GPU "
                    f"sampled from it (mean len {np.diff(off).mean():.1f}, max {args.max_len})")
        roofline = {
            "bound": "mfma",
            "achieved": tf,
            "peak": F64_MFMA_PEAK_TFS,
            "unit": "TFLOP/s",
            "frac": tf / F64_MFMA_PEAK_TFS if tf else None,
            "traffic": None,
            "kernel": "dense_gemm_kernel<FWD/BWD/GRAD> (v_mfma_f64_16x16x4f64) + its epilogue kernels, one evaluation",
            "timed_launches": timed,
            "evaluation_ms": fb_ms,
            "algorithmic_flops_per_evaluation": alg_flops,
            "issued_flops_per_evaluation": issued,
            "row_slots": R,
            "trellis_steps": T,
        }
    else:
        workload = (f"c3 family A: {args.states}-state sparse WFSA, out-degree {args.degree}+end, "
                    f"{args.emissions} of {args.vocab} symbols/state, {args.strings_per_gpu} distinct "
                    f"strings per GPU (mean len {np.diff(off).mean():.1f}, max {args.max_len})")
        roofline = {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS if achieved else None,
            "traffic": traffic,
            "kernel": "fbs_kernel (compiled-stream forward pass, per-iteration)",
            "timed_launches": timed,
            "kernel_ms_per_launch": kern_ms,
            "all_fb_kernels_ms_per_step": fb_ms,
            "algorithmic_bytes_per_launch": alg_bytes,
        }

    out = {
        "metric": METRIC,
        "value": value,
        "unit": "strings/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": workload,
            "global_strings": strings_all,
            "strings_per_gpu": args.strings_per_gpu,
            "parallelism": f"dp{n_gpus}",
            "step": "QuasiNewtonLearner::OptimizationStep (H2D w, forward-backward, all-reduce, D2H grad, host update; epoch loop in wfsa_learner_run)",
            "info_rmin": bool(args.info_rmin),
        },
        "info_rmin": rmin_pass,
        "roofline": roofline,
        "host_ms_per_step": {k: (st1["host_" + k + "_ms"] - st0["host_" + k + "_ms"]) /
                             max(st1["host_steps"] - st0["host_steps"], 1)
                             for k in ("begin", "overlap", "wait", "post")},
        "device_call_ms_last": st1["last_call_ms"],
        "live_edges_per_step": st1["last_live_edges"],
        "build_s": t_build,
        "tier1_strings": st1["tier1_strings"],
        "compiled_strings": st1["compiled_strings"],
        "fallback_strings": st1["fallback_strings"],
        "stream_words": st1["stream_words"],
        "n_bubbles": st1["n_bubbles"],
        "bubble_words": st1["bubble_words"],
        "prepare_ms": st1["prepare_ms"],
    }
    if rank == 0 and world == 1 and args.cpu_sample > 0 and dense:
        out["cpu_baseline"] = cpu_baseline_dense(syn.wfsa_text, sym, off, wt, args.cpu_sample)
    elif rank == 0 and world == 1 and args.cpu_sample > 0:
        cb, rel, ll_ref, ll_dev = cpu_baseline(syn.wfsa_text, sym, off, wt, args.cpu_sample)
        out["cpu_baseline"] = cb
        out["ll_rel_err_vs_reference_algorithm"] = rel
    else:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
