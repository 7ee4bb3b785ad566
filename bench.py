#!/usr/bin/env python3
"""bench.py -- queries/sec of the KNN classify hot path on MI355X.

Metric (BASELINE.json): queries/sec (node) + % MFMA peak on configs[1] =
1M train x 10k queries, d=128, k=10 (L2), per GPU.  A step is one
knn_classify_device call over the rank's 10k queries: fused MFMA distance +
top-R candidate kernel, fp64 exact re-rank + certification + first-to-max
vote, exact rescan of uncertified queries if any.  Inputs are synthetic
(seeded Gaussian mixture, min-max normalised, fp64 like the reference's
Data_train) and resident in HBM before timing starts.

Multi-GPU (--mode query, default; north_star mode a): the train set is
broadcast from rank 0 with torch.distributed (RCCL over xGMI) before timing;
every rank classifies its own 10k queries (weak scaling, no data-path
collective).  --mode train (mode b, cfg4 shape: --n-train 100000000 --dim 96):
rank r holds train rows [n r/W, n (r+1)/W); a step = local exact top-(k+1)
+ RCCL all-gather of the lists + k-way merge/vote of the rank's query slice.

Run: python bench.py [--gpus N --steps K --warmup W]
     (N>1: python -m torch.distributed.run --nproc-per-node N bench.py ...)
"""
import argparse
import importlib.util
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "-mpi-knn-_amd")
PEAK_FP32_TFLOPS = 157.3   # MI355X dense fp32 MFMA (= vector) peak, MI355X_MICROARCH.md
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA peak (no sparsity), MI355X_MICROARCH.md
METRIC = "queries/sec (node) + % MFMA peak, 1M train x 10k query d=128 k=10, 1/2/4/8 GPU"


def log(*a):
    """Progress to stderr (the JSON result line is the only stdout output)."""
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench %.1fs]" % (time.perf_counter() - T0), *a, file=sys.stderr, flush=True)


T0 = time.perf_counter()


def _load(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(PKG, name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def load_knn():
    return _load("knn_amd")


def pad_dim(d):
    for v in (16, 32, 48, 64, 96, 128, 160, 192, 256):
        if d <= v:
            return v
    return d


def _grid(x, lo, hi):
    """Scale into [0,1) and quantise to the 8-bit grid k/256 (SIFT-like byte
    features): exact in fp64 and in an 8-digit decimal CSV, so the reference
    program reads back the identical values (oracle/ref_runner.py)."""
    return ((x - lo) / (hi - lo) * 256.0).floor_().clamp_(0.0, 255.0).div_(256.0)


def synth(n, m, d, classes, seed_train, seed_query, device, row0=0, n_total=None):
    """Gaussian mixture (class = cluster), values scaled into [0,1) like the
    reference's min-max normalisation (cpp:229-306) and quantised to 8-bit
    grid values k/256, fp64.  Rows [row0, row0+n) of a virtual n_total-row
    train set (train sharding), generated in chunks so a 100M-row shard
    needs no temporaries of its size."""
    g = torch.Generator(device=device)
    g.manual_seed(seed_train)
    centres = torch.rand((classes, d), generator=g, device=device, dtype=torch.float64) * 4 - 2
    lo, hi = -2.0 - 4.5, 2.0 + 4.5  # fixed scale (centres in [-2,2] + N(0,1) tails)
    X = torch.empty((n, d), device=device, dtype=torch.float64)
    lab = torch.empty(n, device=device, dtype=torch.int32)
    chunk = 1 << 20
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        gc = torch.Generator(device=device)
        gc.manual_seed(seed_train * 1000003 + (row0 + c0) // chunk)
        lc = torch.randint(0, classes, (c1 - c0,), generator=gc, device=device, dtype=torch.int32)
        xc = centres[lc.long()] + torch.randn((c1 - c0, d), generator=gc, device=device,
                                              dtype=torch.float64)
        X[c0:c1] = _grid(xc, lo, hi)
        lab[c0:c1] = lc
    gq = torch.Generator(device=device)
    gq.manual_seed(seed_query)
    qlab = torch.randint(0, classes, (m,), generator=gq, device=device, dtype=torch.int32)
    Q = centres[qlab.long()] + torch.randn((m, d), generator=gq, device=device, dtype=torch.float64)
    Q = _grid(Q, lo, hi).contiguous()
    return X, lab, Q, qlab


def pmc_traffic(kernel, n, m, d, k):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC pass
    (profiles/*_traffic_*.json, made by tools/traffic_json.py: 2*FETCH_SIZE +
    WRITE_SIZE, KiB -> B) when it profiled this exact workload; else None.
    Counters cannot be read from inside the timed process itself."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic_*.json")), reverse=True):
        try:
            rec = json.load(open(path))
        except (OSError, ValueError):
            continue
        wl = rec.get("workload", {})
        if (wl.get("n_train"), wl.get("queries"), wl.get("dim"), wl.get("k")) != (n, m, d, k):
            continue
        kr = rec.get("kernels", {}).get(kernel)
        if kr:
            return kr["hbm_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None, None


def cpu_baseline(X, lab, Q, k, classes, gpu_labels, budget_s=12.0):
    """Oracle (CPU restatement of the reference, bit-identical on the golden
    fixtures) on a bounded query sample using all host cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    cores = max(1, min(cores, 16))
    Xh, lh, Qh = X.cpu().numpy(), lab.cpu().numpy(), Q.cpu().numpy()
    t0 = time.perf_counter()
    oracle.knn(Xh, lh, Qh[:cores], k, True, classes, nthreads=cores)  # calibrate
    per_round = time.perf_counter() - t0
    rounds = int(max(1, min(32, (budget_s - per_round) / max(per_round, 1e-6))))
    sample = min(Qh.shape[0], cores * rounds)
    t0 = time.perf_counter()
    want, _, _ = oracle.knn(Xh, lh, Qh[:sample], k, True, classes, nthreads=cores)
    el = time.perf_counter() - t0
    match = bool((want == gpu_labels[:sample]).all())
    return {"value": sample / el, "unit": "queries/s", "cores": cores, "kind": "port",
            "sample": "%d of the %d queries (first ones) against all %d train rows, "
                      "oracle/knn_oracle.cpp with %d threads, %.1f s; labels match GPU: %s"
                      % (sample, Qh.shape[0], Xh.shape[0], cores, el, match),
            "labels_match_gpu": match}


REF_SAMPLE = 512  # queries the reference program classifies in the bench's baseline leg


def ref_config(n, d, k, classes, sample=REF_SAMPLE):
    """Constants of the reference build timed as the CPU baseline (cpp:108-116);
    __graft_entry__.build() compiles it (oracle/_ref travels to the GPU box)."""
    return dict(dim=d, K=k, N_train=n, N_test=sample, N_val=sample, class_cnt=classes,
                Validation=False, Normalize=False, Euclidean_distance=True)


def cpu_baseline_reference(X, lab, Q, k, classes, gpu_labels):
    """The reference program itself (knn_mpi.cpp, compiled unmodified apart
    from its constants and a timer around the test-query loop) under mpirun
    on the host cores, on the first REF_SAMPLE queries against the full train
    set.  value = queries / test-loop seconds (max over ranks); the CSV parse
    and MPI_Bcast are in running_time_s."""
    import shutil
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import build_ref
    import ref_runner
    n, d = X.shape
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    nprocs = next(p for p in (16, 8, 4, 2) if p <= max(2, cores) and n % p == 0
                  and REF_SAMPLE % p == 0)
    exe = build_ref.build_ref(ref_config(n, d, k, classes), instrument=False, timing=True)
    codes = (X * 256.0).round().to(torch.uint8).cpu().numpy()
    qcodes = (Q[:REF_SAMPLE] * 256.0).round().to(torch.uint8).cpu().numpy()
    assert np.array_equal(ref_runner.grid_values(codes), X.cpu().numpy()), "bench data off-grid"
    wd = tempfile.mkdtemp(prefix="knn_ref_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        ref_runner.write_grid_csv(os.path.join(wd, "mnist_train.csv"), codes, lab.cpu().numpy())
        ref_runner.write_grid_csv(os.path.join(wd, "mnist_test.csv"), qcodes)
        labels, loop_s, run_s = ref_runner.run_reference(exe, wd, nprocs)
    finally:
        shutil.rmtree(wd, ignore_errors=True)
    match = bool((labels == gpu_labels[:REF_SAMPLE]).all())
    return {"value": REF_SAMPLE / loop_s, "unit": "queries/s", "cores": nprocs, "kind": "reference",
            "sample": "%d of the %d queries (first ones) against all %d train rows: "
                      "/root/reference/knn_mpi.cpp (constants set, Normalize=false, timer around "
                      "the test loop) under mpirun -np %d; test loop %.2f s, whole run %.1f s "
                      "incl. CSV parse + MPI_Bcast; labels match GPU: %s"
                      % (REF_SAMPLE, Q.shape[0], n, nprocs, loop_s, run_s, match),
            "running_time_s": run_s, "labels_match_gpu": match}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--mode", choices=("query", "train"), default="query")
    ap.add_argument("--n-train", type=int, default=1_000_000, help="train rows (whole job)")
    ap.add_argument("--queries", type=int, default=10_000,
                    help="queries per GPU (query mode) / in total (train mode)")
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--classes", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fp32-path", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    kd = _load("knn_dist")
    knn = load_knn()
    n, m, d, k, C = args.n_train, args.queries, args.dim, args.k, args.classes
    sync = torch.cuda.synchronize
    stream = torch.cuda.current_stream().cuda_stream
    clf = knn.Classifier(local)
    clf.set_timing(True)

    if args.mode == "query":
        # train generated on rank 0 and RCCL-broadcast (≙ MPI_Bcast cpp:224-225)
        X, lab, Q, _ = synth(n, m, d, C, 1234, 5678 + rank, dev)
        kd.broadcast_train(X, lab)
        sync()
        log("synthetic train ready: %d rows x %d" % (n, d))
        clf.set_train_device(X.data_ptr(), lab.data_ptr(), n, d, C, keep=(X, lab))
        out_lab = torch.empty(m, dtype=torch.int32, device=dev)
        out_flags = torch.empty(m, dtype=torch.int32, device=dev)
        stats = {"cand": [], "rr": [], "resc": 0}

        def step():
            clf.classify_device(Q.data_ptr(), m, k, knn.L2, out_lab.data_ptr(), None, None,
                                out_flags.data_ptr(), stream)
            stats["cand"].append(clf.last_phase_ms(knn.PHASE_CANDIDATE))
            stats["rr"].append(clf.last_phase_ms(knn.PHASE_RERANK))
            stats["resc"] += clf.last_rescan_count()

        def run(precision, steps, warmup):
            clf.set_precision(precision)
            for key in ("cand", "rr"):
                stats[key] = []
            stats["resc"] = 0
            el = kd.timed(step, steps, warmup, sync, dev)
            cand = stats["cand"][warmup:]
            return dict(el=el, t_cand=float(np.mean(cand)) * 1e-3,
                        rr=float(np.mean(stats["rr"][warmup:])), resc=stats["resc"],
                        path=clf.last_candidate_path(), geom=clf.last_geometry())

        n_rank, m_rank = n, m
        flops = 2.0 * n * d * m  # algorithmic, per launch per GPU (norm terms excluded)
        main_r = run(knn.PRECISION_AUTO, args.steps, args.warmup)
        log("default path done: %.3f ms/step" % (main_r["el"] / args.steps * 1e3))
        labels_auto = out_lab.clone()
        fp32_r = None
        if not args.no_fp32_path:
            fp32_r = run(knn.PRECISION_FP32, max(3, args.steps // 2), 1)
        same = bool(torch.equal(labels_auto, out_lab))
        total_q = m * world * args.steps
        tag = {(1_000_000, 128, 10): "cfg2", (1_000_000, 960, 100): "cfg5"}.get(
            (n, d, k), "custom")
        workload = ("%s: %d train x %d queries per GPU, d=%d, k=%d, L2, %d classes"
                    % (tag, n, m, d, k, C))
        parallelism = "query-sharded dp%d" % world
    else:
        # train-sharded: this rank's rows only; the same queries on every rank
        r0, r1 = kd.shard_range(n, world, rank)
        X, lab, Q, _ = synth(r1 - r0, m, d, C, 1234, 5678, dev, row0=r0, n_total=n)
        sync()
        log("synthetic shard ready: %d rows x %d" % (r1 - r0, d))
        clf.set_train_device(X.data_ptr(), lab.data_ptr(), r1 - r0, d, C, idx_offset=r0,
                             keep=(X, lab))
        w = k + 1
        pd_ = torch.empty((m, w), dtype=torch.float64, device=dev)
        pi_ = torch.empty((m, w), dtype=torch.int64, device=dev)
        pl_ = torch.empty((m, w), dtype=torch.int32, device=dev)
        q0, q1 = kd.shard_range(m, world, rank)
        out_lab = torch.empty(max(1, q1 - q0), dtype=torch.int32, device=dev)
        stats = {"cand": [], "rr": [], "resc": 0}

        def search_partial(Qt):
            clf.search_partial_device(Qt.data_ptr(), m, w, knn.L2, pd_.data_ptr(), pi_.data_ptr(),
                                      pl_.data_ptr(), stream)
            stats["cand"].append(clf.last_phase_ms(knn.PHASE_CANDIDATE))
            stats["rr"].append(clf.last_phase_ms(knn.PHASE_RERANK))
            stats["resc"] += clf.last_rescan_count()
            return pd_, pi_, pl_

        def merge_vote(gd, gi, gl, parts, a, b):  # k-way merge + vote of this rank's slice
            clf.merge_vote_device(gd.data_ptr(), gi.data_ptr(), gl.data_ptr(), parts, m, w, k,
                                  out_lab.data_ptr(), stream=stream, q0=a, mq=b - a)
            return out_lab

        def step():
            kd.train_sharded(search_partial, merge_vote, Q, m, w, k, dev)
            log("train-sharded step: cand %.2f ms rerank %.2f ms rescans %d"
                % (stats["cand"][-1], stats["rr"][-1], stats["resc"]))

        def run(precision, steps, warmup):
            clf.set_precision(precision)
            for key in ("cand", "rr"):
                stats[key] = []
            stats["resc"] = 0
            el = kd.timed(step, steps, warmup, sync, dev)
            return dict(el=el, t_cand=float(np.mean(stats["cand"][warmup:])) * 1e-3,
                        rr=float(np.mean(stats["rr"][warmup:])), resc=stats["resc"],
                        path=clf.last_candidate_path(), geom=clf.last_geometry())

        n_rank, m_rank = r1 - r0, m
        flops = 2.0 * (r1 - r0) * d * m
        main_r = run(knn.PRECISION_AUTO, args.steps, args.warmup)
        fp32_r, same = None, None
        total_q = m * args.steps
        workload = ("cfg4-shape: %d train (sharded) x %d queries, d=%d, k=%d, L2, %d classes"
                    % (n, m, d, k, C))
        parallelism = "train-sharded tp%d" % world

    path = main_r["path"]
    bf16 = path in (2, 3)
    # fp16 / bf16 MFMA share the dense peak; bf16x3 issues 3 MFMA flops per
    # algorithmic flop, fp16 and fp32 one
    peak = PEAK_BF16_TFLOPS if path in (2, 3, 4) else PEAK_FP32_TFLOPS
    mfma_mult = 3.0 if bf16 else 1.0
    cand_desc = {
        0: "fp32 MFMA 32x32x2",
        2: "bf16x3 split (qh.xh+ql.xh+qh.xl) on MFMA 32x32x16 bf16",
        3: "bf16x3 split (qh.xh+ql.xh+qh.xl) on MFMA 16x16x32 bf16",
        4: "fp16 operands (power-of-two scaled, centred) on MFMA 16x16x32 f16",
    }.get(path, "kernel metric %d" % path)
    achieved = flops / main_r["t_cand"] / 1e12
    geom = main_r["geom"]
    n_qt = max(1, geom["workgroups"] // max(1, geom["splits"]))
    nw = 8 if -(-m_rank // n_qt) > 128 else 4  # waves per workgroup (32 queries each)
    kname = ("cand_kernel<%d,%d,%d,%d>" % (pad_dim(d), geom["lists"], main_r["path"], nw)
             if d <= 256 else "cand_stream_kernel<32,%d,%d>" % (geom["lists"], main_r["path"]))
    traffic, traffic_src = pmc_traffic(kname, n_rank, m_rank, d, k)
    result = {
        "metric": METRIC,
        "value": total_q / main_r["el"],
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": main_r["el"] / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak" if args.mode == "query" else "strong",
        "vs_baseline": None,
        "dtype": {2: "bf16x3", 3: "bf16x3", 4: "fp16"}.get(path, "fp32"),
        "data": "synthetic (seeded Gaussian mixture scaled to [0,1) on the 8-bit grid k/256, "
                "SIFT-like; fp64 inputs)",
        "config": {"workload": workload, "n_train": n, "queries": m, "dim": d, "k": k,
                   "parallelism": parallelism,
                   "candidate_pass": cand_desc + " + fused top-R per lane, certified bound",
                   "rerank": "fp64 exact (reference arithmetic), certified; labels exact",
                   "geometry": geom, "rescanned_queries": main_r["resc"]},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                     "frac": achieved / peak, "traffic": traffic,
                     "traffic_unit": "bytes per launch (HBM, PMC)", "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": (n_rank + m_rank) * d * 4 + m_rank * k * 8,
                     "kernel": kname,
                     "kernel_ms": main_r["t_cand"] * 1e3, "rerank_ms": main_r["rr"],
                     "algorithmic_flops_per_launch": flops,
                     "mfma_flops_per_algorithmic_flop": mfma_mult,
                     "frac_of_issued_mfma": achieved * mfma_mult / peak},
        "cpu_baseline": None,
    }
    if fp32_r is not None:
        a32 = flops / fp32_r["t_cand"] / 1e12
        result["fp32_path"] = {
            "value": m * world * max(3, args.steps // 2) / fp32_r["el"], "unit": "queries/s",
            "kernel_ms": fp32_r["t_cand"] * 1e3, "achieved": a32, "peak": PEAK_FP32_TFLOPS,
            "frac": a32 / PEAK_FP32_TFLOPS, "rescanned_queries": fp32_r["resc"],
            "geometry": fp32_r["geom"], "labels_equal_default_path": same}
    if rank == 0 and world == 1 and args.mode == "query" and not args.no_cpu_baseline:
        log("cpu baseline (oracle port) ...")
        port = cpu_baseline(X, lab, Q, k, C, labels_auto.cpu().numpy(), budget_s=6.0)
        result["cpu_baseline"] = port
        try:
            log("cpu baseline (reference program under mpirun) ...")
            result["cpu_baseline"] = cpu_baseline_reference(X, lab, Q, k, C,
                                                            labels_auto.cpu().numpy())
            result["cpu_baseline_port"] = port
        except (OSError, RuntimeError, StopIteration, subprocess.SubprocessError) as e:
            log("reference baseline unavailable (%s); reporting the oracle port" % e)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
