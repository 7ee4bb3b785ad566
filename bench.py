#!/usr/bin/env python3
"""bench.py -- queries/sec of the KNN classify hot path on MI355X.

Metric (BASELINE.json): queries/sec (node) + % MFMA peak on configs[1] =
1M train x 10k queries, d=128, k=10 (L2), per GPU.  A step is one
knn_classify_device call over the rank's 10k queries: fused MFMA distance +
top-R candidate kernel, fp64 exact re-rank + certification + first-to-max
vote, and the device-driven exact rescan of uncertified queries.  Inputs are
synthetic (seeded Gaussian mixture, fp64 like the reference's Data_train)
and resident in HBM before timing starts.

Multi-GPU: `--gpus N` launches N ranks itself (one process per GPU through
torch.distributed.run, started before anything touches the GPU) unless it
already runs under a launcher (WORLD_SIZE set, e.g. the driver's own
torch.distributed.run).
  --mode query (default; north_star mode a, ≙ MPI_Bcast + MPI_Scatter,
    cpp:224-227): the train set is RCCL-broadcast from rank 0 (timed and
    reported separately: train_broadcast_ms) and every rank classifies its
    own 10k queries -- weak scaling, no data-path collective.  The same line
    carries the configs[2] strong-scaling leg (`cfg3_strong`): a fixed 1M
    queries split 1M/N per rank (≙ the batch split cpp:136-138).
  --mode train (mode b, cfg4 shape: --n-train 100000000 --dim 96): rank r
    holds train rows [n r/N, n (r+1)/N); a step = local exact top-(k+1) + RCCL
    all-gather of the lists + k-way merge/vote of the rank's query slice.
`--dry-run` (CPU, gloo): plumbing check of the launcher and the
decomposition only -- a plain torch brute force stands in for the HIP
library and the line reports value null.

Run: python bench.py [--gpus N --steps K --warmup W]
"""
import argparse
import glob
import hashlib
import importlib.util
import json
import os
import socket
import subprocess
import sys
import time
import traceback
from datetime import timedelta

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "-mpi-knn-_amd")
PEAK_FP32_TFLOPS = 157.3   # MI355X dense fp32 MFMA (= vector) peak, MI355X_MICROARCH.md
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16/fp16 MFMA peak (no sparsity), MI355X_MICROARCH.md
PEAK_I8_TOPS = 5000.0      # MI355X dense int8 MFMA peak: 2x bf16 per clock (16x16x64), same guide


def peak_of(path):
    """Dense MFMA peak of a candidate path (knn_last_candidate_path)."""
    return {2: PEAK_BF16_TFLOPS, 3: PEAK_BF16_TFLOPS, 4: PEAK_BF16_TFLOPS,
            5: PEAK_I8_TOPS, 6: PEAK_I8_TOPS}.get(path, PEAK_FP32_TFLOPS)
METRIC = "queries/sec (node) + % MFMA peak, 1M train x 10k query d=128 k=10, 1/2/4/8 GPU"
REF_SAMPLE = 512  # queries the reference program classifies in the bench's baseline leg


PHASE = ["start"]  # what this rank is doing (named in a failure report)


def phase(name):
    PHASE[0] = name
    log("phase: %s" % name)


def _world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def gather_per_rank(vals, dev=None):
    """This rank's numbers -> one list per rank (rank order), on every rank."""
    world, _ = _world()
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=dev)
    if world == 1:
        return [t.tolist()]
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def labels_sha1(t):
    return hashlib.sha1(t.detach().to("cpu").to(torch.int32).numpy().tobytes()).hexdigest()


def per_rank_report(dev, fields, labels=None):
    """{field: [value of rank 0, rank 1, ...]} for the N-GPU line (every rank
    must call it); labels: this rank's label slice, reported as one sha1 per
    rank (the 1-GPU line's rank-0 sha1 is comparable with every N's: rank r
    classifies the same query rows at every N)."""
    names = list(fields)
    vals = gather_per_rank([fields[k] for k in names], dev)
    out = {k: [v[i] for v in vals] for i, k in enumerate(names)}
    if labels is not None:
        h = hashlib.sha1(labels.detach().to("cpu").to(torch.int32).numpy().tobytes()).digest()
        ht = torch.tensor(list(h), dtype=torch.uint8, device=dev)
        world, _ = _world()
        if world > 1:
            parts = [torch.empty_like(ht) for _ in range(world)]
            dist.all_gather(parts, ht)
        else:
            parts = [ht]
        out["labels_sha1"] = [bytes(p.cpu().tolist()).hex() for p in parts]
    return out


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


def _grid(x, lo, hi):
    """Scale into [0,1) and quantise to the 8-bit grid k/256 (SIFT-like byte
    features): exact in fp64 and in an 8-digit decimal CSV, so the reference
    program reads back the identical values (oracle/ref_runner.py)."""
    return ((x - lo) / (hi - lo) * 256.0).floor_().clamp_(0.0, 255.0).div_(256.0)


CHUNK = 1 << 20  # rows per generator chunk (a chunk's values depend only on its index)
QCHUNK = 1 << 13  # the query sets' chunk: rank r's queries at every N (rows r m .. (r+1) m)


def _rows(centres, n, row0, seed, device, classes, n_total=None, chunk=CHUNK):
    """Rows [row0, row0+n) of a virtual Gaussian-mixture set, raw (unscaled)
    fp64, generated by global chunks of `chunk` rows whose values depend only
    on the chunk's index: every chunk draws all its `chunk` rows, whatever
    n_total, so any shard of the set -- and any prefix, e.g. rank 0's queries
    at 1 and at 8 GPUs -- is reproduced exactly whatever the shard boundaries
    (a shard starting or ending inside a chunk generates that chunk and keeps
    its part).  n_total is accepted for the callers' bookkeeping only."""
    d = centres.shape[1]
    X = torch.empty((n, d), device=device, dtype=torch.float64)
    lab = torch.empty(n, device=device, dtype=torch.int32)
    for ci in range(row0 // chunk, (row0 + n + chunk - 1) // chunk):
        g0 = ci * chunk                       # the chunk's global rows [g0, g0 + chunk)
        a, b = max(row0, g0), min(row0 + n, g0 + chunk)
        if a >= b:
            continue
        gc = torch.Generator(device=device)
        gc.manual_seed(seed * 1000003 + ci)
        lc = torch.randint(0, classes, (chunk,), generator=gc, device=device, dtype=torch.int32)
        xc = torch.randn((chunk, d), generator=gc, device=device, dtype=torch.float64)
        X[a - row0:b - row0] = centres[lc[a - g0:b - g0].long()] + xc[a - g0:b - g0]
        lab[a - row0:b - row0] = lc[a - g0:b - g0]
        del xc
    return X, lab


def minmax_normalize_(sets, reduce=None):
    """The reference's transductive min-max normalisation (cpp:229-306) on
    device tensors, in place: per-dim max/min over every set, starting from
    the quirky -1 / 999999 (cpp:239-243), then (x - min) / (max - min) on
    dims with max != min (cpp:279-305) -- the same fp64 subtract and divide.
    reduce(mx, mn): optional cross-rank MAX / MIN all-reduce (≙ cpp:276-277)."""
    d = sets[0].shape[1]
    dev = sets[0].device
    mx = torch.full((d,), -1.0, dtype=torch.float64, device=dev)
    mn = torch.full((d,), 999999.0, dtype=torch.float64, device=dev)
    for s in sets:
        for c0 in range(0, s.shape[0], CHUNK):
            c = s[c0:c0 + CHUNK]
            mx = torch.maximum(mx, c.amax(0))
            mn = torch.minimum(mn, c.amin(0))
    if reduce is not None:
        reduce(mx, mn)
    rng = mx - mn
    keep = rng != 0
    rng = torch.where(keep, rng, torch.ones_like(rng))
    for s in sets:
        for c0 in range(0, s.shape[0], CHUNK):
            c = s[c0:c0 + CHUNK]
            c.copy_(torch.where(keep, (c - mn) / rng, c))
    return mx, mn


def synth(n, m, d, classes, seed_train, seed_query, device, row0=0, n_total=None, data="grid",
          q0=0, reduce=None, q_total=None):
    """Gaussian mixture (class = cluster), fp64.  Train rows [row0, row0+n)
    and query rows [q0, q0+m) of virtual sets (train / query sharding),
    generated in chunks so a 100M-row shard needs no temporaries of its size.
      data="grid":       scaled into [0,1) with a fixed range and quantised to
                         the 8-bit grid k/256 (SIFT-like byte features);
      data="continuous": min-max normalised exactly as the reference does
                         (cpp:229-306, over train and queries), no quantisation:
                         values are not on any power-of-two grid (MNIST-style
                         (x - min) / (max - min) features).  With sharded sets
                         pass reduce= for the cross-rank MAX/MIN."""
    g = torch.Generator(device=device)
    g.manual_seed(seed_train)
    centres = torch.rand((classes, d), generator=g, device=device, dtype=torch.float64) * 4 - 2
    X, lab = _rows(centres, n, row0, seed_train, device, classes, n_total)
    Q, qlab = _rows(centres, m, q0, seed_query, device, classes, q_total, chunk=QCHUNK)
    if data == "grid":
        lo, hi = -2.0 - 4.5, 2.0 + 4.5  # fixed scale (centres in [-2,2] + N(0,1) tails)
        for s in (X, Q):
            for c0 in range(0, s.shape[0], CHUNK):
                s[c0:c0 + CHUNK] = _grid(s[c0:c0 + CHUNK], lo, hi)
    elif data == "continuous":
        minmax_normalize_([X, Q], reduce)
    else:
        raise ValueError("data must be grid or continuous")
    return X, lab, Q, qlab


def kernel_src_sha():
    """Identity of the kernel build: sha1 over the library's sources.  PMC
    traffic files record it, and a bench line only cites a profile of the
    same sources (profiles/*_traffic_*.json, tools/traffic_json.py)."""
    h = hashlib.sha1()
    for p in sorted(glob.glob(os.path.join(PKG, "csrc", "*"))):
        h.update(os.path.basename(p).encode())
        h.update(open(p, "rb").read())
    return h.hexdigest()[:16]


def pmc_traffic(kernel, workload, src_sha):
    """HBM bytes per launch of `kernel` from a committed rocprofv3 PMC pass of
    this exact workload and kernel build (2*FETCH_SIZE + WRITE_SIZE, KiB -> B);
    (None, reason) when no such profile exists.  Counters cannot be read from
    inside the timed process itself."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic_*.json"))):
        try:
            rec = json.load(open(path))
        except (OSError, ValueError):
            continue
        wl = rec.get("workload", {})
        if any(wl.get(key) != workload[key] for key in ("n_train", "queries", "dim", "k")):
            continue
        if wl.get("data", "grid") != workload.get("data", "grid"):
            continue
        if wl.get("tuning") != workload.get("tuning"):  # (a profiled tuning variant)
            continue
        if rec.get("kernel_src_sha") != src_sha:
            continue
        kr = rec.get("kernels", {}).get(kernel)
        if kr:
            return kr["hbm_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None, "no PMC profile of %s for this workload and kernel build (%s)" % (kernel, src_sha)


def host_cores():
    """(CPUs this process may run on, the CPU share granted to it): on the GPU
    box the affinity mask shows the whole machine while the share is set in
    OMP_NUM_THREADS (16 per GPU)."""
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    share = int(os.environ.get("OMP_NUM_THREADS") or cores)
    return cores, max(1, min(cores, share))


def cpu_baseline(X, lab, Q, k, classes, gpu_labels, budget_s=12.0):
    """Oracle (CPU restatement of the reference, bit-identical on the golden
    fixtures) on a bounded query sample using the granted host cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    cores, share = host_cores()
    Xh, lh, Qh = X.cpu().numpy(), lab.cpu().numpy(), Q.cpu().numpy()
    t0 = time.perf_counter()
    oracle.knn(Xh, lh, Qh[:share], k, True, classes, nthreads=share)  # calibrate
    per_round = time.perf_counter() - t0
    rounds = int(max(1, min(32, (budget_s - per_round) / max(per_round, 1e-6))))
    sample = min(Qh.shape[0], share * rounds)
    t0 = time.perf_counter()
    want, _, _ = oracle.knn(Xh, lh, Qh[:sample], k, True, classes, nthreads=share)
    el = time.perf_counter() - t0
    match = bool((want == gpu_labels[:sample]).all())
    return {"value": sample / el, "unit": "queries/s", "cores": share, "host_cores": cores,
            "cpu_share": share, "kind": "port",
            "sample": "%d of the %d queries (first ones) against all %d train rows, "
                      "oracle/knn_oracle.cpp with %d threads (%d host CPUs visible, share %d), "
                      "%.1f s; labels match GPU: %s"
                      % (sample, Qh.shape[0], Xh.shape[0], share, cores, share, el, match),
            "labels_match_gpu": match}


def ref_config(n, d, k, classes, sample=REF_SAMPLE):
    """Constants of the reference build timed as the CPU baseline (cpp:108-116);
    __graft_entry__.build() compiles it (oracle/_ref travels to the GPU box)."""
    return dict(dim=d, K=k, N_train=n, N_test=sample, N_val=sample, class_cnt=classes,
                Validation=False, Normalize=False, Euclidean_distance=True)


def cpu_baseline_reference(X, lab, Q, k, classes, gpu_labels):
    """The reference program itself (knn_mpi.cpp, compiled unmodified apart
    from its constants and a timer around the test-query loop) under mpirun
    on the granted host cores, on the first REF_SAMPLE queries against the
    full train set.  Ranks = the largest P <= the CPU share that divides
    N_train and the sample (the reference aborts otherwise, cpp:127-129).
    value = queries / test-loop seconds (max over ranks); the CSV parse and
    MPI_Bcast are in running_time_s."""
    import shutil
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import build_ref
    import ref_runner
    n, d = X.shape
    cores, share = host_cores()
    nprocs = max(p for p in range(2, max(2, share) + 1) if n % p == 0 and REF_SAMPLE % p == 0)
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
    return {"value": REF_SAMPLE / loop_s, "unit": "queries/s", "cores": nprocs,
            "host_cores": cores, "cpu_share": share, "ranks": nprocs, "kind": "reference",
            "sample": "%d of the %d queries (first ones) against all %d train rows: "
                      "/root/reference/knn_mpi.cpp (constants set, Normalize=false, timer around "
                      "the test loop) under mpirun -np %d on the box's host CPUs (%d visible, "
                      "share %d); test loop %.2f s, whole run %.1f s incl. CSV parse + "
                      "MPI_Bcast; labels match GPU: %s"
                      % (REF_SAMPLE, Q.shape[0], n, nprocs, cores, share, loop_s, run_s, match),
            "running_time_s": run_s, "labels_match_gpu": match}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n):
    """One process per GPU: re-run this script under torch.distributed.run as
    a CHILD process (nothing here has touched the GPU) and return its exit
    code.  The env (HSA_ENABLE_IPC_MODE_LEGACY=0 etc.) is inherited."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
           str(n), "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


class CpuStandIn:
    """--dry-run only: a plain torch fp64 brute force in place of the HIP
    library, so the launcher and the decomposition can be exercised on CPU
    (gloo).  Not a measurement; the bench line reports value null."""
    L2 = 0
    PRECISION_AUTO = PRECISION_FP32 = 0

    def set_train(self, X, lab, classes):
        self.X, self.lab = X, lab

    def classify(self, Q, k):
        d2 = (Q * Q).sum(1)[:, None] + (self.X * self.X).sum(1)[None, :] - 2.0 * Q @ self.X.T
        nb = torch.topk(d2, k, dim=1, largest=False).indices
        nl = self.lab[nb]
        return self.vote(nl, k)

    @staticmethod
    def vote(nl, k):
        out = torch.empty(nl.shape[0], dtype=torch.int32)
        for q in range(nl.shape[0]):  # cpp:324-337
            cnt, best, bl = {}, 0, -1
            for t in range(k):
                lb = int(nl[q, t])
                cnt[lb] = cnt.get(lb, 0) + 1
                if cnt[lb] > best:
                    best, bl = cnt[lb], lb
            out[q] = bl
        return out

    def search_partial(self, Q, w, r0):
        """This shard's top-w (dist, global idx, label), ascending."""
        d2 = (Q * Q).sum(1)[:, None] + (self.X * self.X).sum(1)[None, :] - 2.0 * Q @ self.X.T
        v, i = torch.topk(d2, min(w, d2.shape[1]), dim=1, largest=False)
        return v, i + r0, self.lab[i]

    def merge_vote(self, gd, gi, gl, k, a, b):
        """[parts][m][w] lists -> labels of queries [a, b): by (dist, idx)."""
        d = gd[:, a:b].permute(1, 0, 2).reshape(b - a, -1)
        i = gi[:, a:b].permute(1, 0, 2).reshape(b - a, -1)
        lb = gl[:, a:b].permute(1, 0, 2).reshape(b - a, -1)
        o = torch.argsort(i, dim=1, stable=True)
        d, i, lb = d.gather(1, o), i.gather(1, o), lb.gather(1, o)
        o = torch.argsort(d, dim=1, stable=True)
        return self.vote(lb.gather(1, o)[:, :k], k)


def timed_run(kd, clf, step, steps, warmup, sync, dev, precision=None):
    """W untimed steps, then exactly K timed steps bracketed by barrier + sync
    (max over ranks); the candidate kernel's HIP-event times and the rescan
    counts of the K timed calls are read back only after the timed region.
    The timed calls record only the two events around the candidate kernel
    (each event record holds the stream ~6 us: 5 per call cost ~2 % of a
    cfg2 step, profiles/ab_log.md r5u); the other phases' times (prep,
    re-rank, rescan) come from up to 5 further, untimed calls with every
    phase's events."""
    if precision is not None:
        clf.set_precision(precision)
    for _ in range(warmup):
        step()
    sync()
    clf.set_timing(True, kernel_only=True)
    clf.timing_totals(reset=True)
    clf.rescan_totals(reset=True)
    clf.tie_totals(reset=True)
    el = kd.timed(step, steps, 0, sync, dev)
    ms, calls = clf.timing_totals(reset=True)
    resc = clf.rescan_totals(reset=True)
    ties = clf.tie_totals(reset=True)
    calls = max(1, calls)
    clf.set_timing(True)
    for _ in range(min(steps, 5)):
        step()
    sync()
    ph, pcalls = clf.timing_totals(reset=True)
    pcalls = max(1, pcalls)
    clf.set_timing(True, kernel_only=True)  # (the mode the timed calls ran in)
    return dict(el=el, t_cand=ms[1] / calls * 1e-3, rr=ph[2] / pcalls, rescan_ms=ph[3] / pcalls,
                prep_ms=ph[0] / pcalls, phase_calls=pcalls, calls=calls, resc=resc[0],
                full_scans=resc[1],
                tie_reordered=ties,
                path=clf.last_candidate_path(), geom=clf.last_geometry(),
                kernel=clf.last_kernel_name())


# ---------------------------------------------------------------------------
# The native drop-in (bin/knn_mpi_amd) as the reference is run: CSV in,
# Test_label.csv out, one process driving every GPU through knn_group (RCCL
# ncclBroadcast / ncclAllGather / ncclAllReduce, ≙ cpp:224-227, 276-277, 340,
# 383).  Runs as a child process before this process touches any GPU.
DROPIN = dict(n=1_000_000, m=10_000, d=128, k=10, classes=10)  # configs[1] shape
_GRID_TXT = np.frombuffer(b"".join(("%.8f," % (c / 256.0)).encode() for c in range(256)),
                          dtype=np.uint8).reshape(256, 11)


def write_grid_csv(path, codes, labels=None, chunk=1 << 16):
    """8-bit grid values k/256 in the reference's CSV formats (cpp:154-222):
    "label,x1,..,xd" rows (train / validation) or "x1,..,xd" rows (test),
    every value printed with its exact 8-digit expansion (labels 0-9)."""
    rows, dim = codes.shape
    with open(path, "wb") as f:
        for r0 in range(0, rows, chunk):
            c = codes[r0:r0 + chunk]
            body = _GRID_TXT[c].reshape(c.shape[0], dim * 11)
            body[:, -1] = ord("\n")
            if labels is not None:
                pre = np.empty((c.shape[0], 2), np.uint8)
                pre[:, 0] = ord("0") + labels[r0:r0 + chunk]
                pre[:, 1] = ord(",")
                body = np.concatenate([pre, body], axis=1)
            f.write(body.tobytes())


def dropin_inputs(wd, n, m, d, classes, seed=97):
    """Seeded Gaussian mixture on the 8-bit grid (numpy, no GPU): train,
    validation (m rows) and test (m rows) CSVs under the reference's file
    names (cpp:117-119)."""
    assert classes <= 10
    rng = np.random.default_rng(seed)
    centres = rng.uniform(0.2, 0.8, (classes, d)).astype(np.float32)

    def block(rows):
        lab = rng.integers(0, classes, rows).astype(np.int32)
        x = centres[lab] + 0.12 * rng.standard_normal((rows, d), dtype=np.float32)
        return np.clip(np.floor(x * 256.0), 0, 255).astype(np.uint8), lab

    parts = [block(min(1 << 18, n - r0)) for r0 in range(0, n, 1 << 18)]
    tr = np.concatenate([p[0] for p in parts])
    trl = np.concatenate([p[1] for p in parts])
    va, val_ = block(m)
    te, _ = block(m)
    write_grid_csv(os.path.join(wd, "mnist_train.csv"), tr, trl)
    write_grid_csv(os.path.join(wd, "mnist_validation.csv"), va, val_)
    write_grid_csv(os.path.join(wd, "mnist_test.csv"), te)


def dropin_cmd(wd, gpus, mode, n, m, d, k, classes, out):
    return [os.path.join(PKG, "bin", "knn_mpi_amd"), "--dim", str(d), "--K", str(k),
            "--N_train", str(n), "--N_test", str(m), "--N_val", str(m), "--class_cnt",
            str(classes), "--Euclidean_distance", "true", "--Normalize", "true",
            "--Validation", "true", "--gpus", str(gpus), "--mode", mode, "--output", out,
            "--timings"]


def run_dropin(wd, gpus, mode, shape, timeout=600):
    out = os.path.join(wd, "Test_label_%s_%d.csv" % (mode, gpus))
    cmd = dropin_cmd(wd, gpus, mode, out=out, **shape)
    t0 = time.perf_counter()
    r = subprocess.run(cmd, cwd=wd, capture_output=True, text=True, timeout=timeout)
    wall = time.perf_counter() - t0
    if r.returncode != 0:
        raise RuntimeError("knn_mpi_amd --gpus %d --mode %s failed (%d): %s"
                           % (gpus, mode, r.returncode, r.stderr[-1500:]))
    phases = {}
    for line in r.stderr.splitlines():
        if line.startswith("[knn_mpi_amd]"):
            f = line.split()
            phases[f[1]] = float(f[2])
    run_s = acc = None
    for line in r.stdout.splitlines():
        if line.startswith("Running time is "):
            run_s = float(line.split()[3])
        elif line.startswith("accuracy = "):
            acc = line
    body = open(out, "rb").read()
    return {"gpus": gpus, "mode": mode, "running_time_s": run_s, "process_wall_s": wall,
            "phases_s": phases, "accuracy_line": acc,
            "test_label_sha1": hashlib.sha1(body).hexdigest(), "labels": body.count(b"\n"),
            "queries_per_s_test_pass": shape["m"] / phases["test"] if phases.get("test") else None}


def dropin_legs(world, shape=DROPIN, dry=False):
    """The drop-in driver at 1 GPU and at `world` GPUs in both modes; the
    Test_label.csv bytes of every multi-GPU run must equal the 1-GPU run's.
    dry: write the inputs and report the planned commands only (no GPU)."""
    import shutil
    import tempfile
    wd = tempfile.mkdtemp(prefix="knn_dropin_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        t0 = time.perf_counter()
        dropin_inputs(wd, shape["n"], shape["m"], shape["d"], shape["classes"])
        gen_s = time.perf_counter() - t0
        legs = [(1, "query")] + ([(world, "query")] if world > 1 else []) + [(world, "train")]
        desc = ("native drop-in bin/knn_mpi_amd on generated CSVs (%d train x %d validation + "
                "%d test, d=%d, K=%d, Normalize=true, Validation=true), one process over the "
                "GPUs via knn_group (RCCL)" % (shape["n"], shape["m"], shape["m"], shape["d"],
                                                shape["k"]))
        if dry:
            return {"group_query": {"cmd": " ".join(dropin_cmd(wd, world, "query", out="-", **shape)),
                                    "value": None},
                    "group_train": {"cmd": " ".join(dropin_cmd(wd, world, "train", out="-", **shape)),
                                    "value": None},
                    "inputs_written": sorted(os.listdir(wd)), "dry_run": True}
        # each leg's own time limit (a 1M x 128 leg runs ~1 s of GPU work plus
        # the CSV parse); a failed multi-GPU leg is reported, not retried, and
        # ends the drop-in phase so the measured legs of the line still run
        res, err = {}, None
        for g, mode in legs:
            try:
                res[(g, mode)] = run_dropin(wd, g, mode, shape, timeout=180)
            except (OSError, RuntimeError, subprocess.SubprocessError) as e:
                err = "knn_mpi_amd --gpus %d --mode %s: %s" % (g, mode, str(e)[-800:])
                break
        base = res.get((1, "query"))
        out = {"workload": desc, "input_generation_s": gen_s, "group_1gpu": base}
        if err:
            out["error"] = err
        for key, (g, mode) in (("group_query", (world, "query")), ("group_train", (world, "train"))):
            r = res.get((g, mode))
            if r is None or base is None:
                continue
            r["labels_match"] = r["test_label_sha1"] == base["test_label_sha1"]
            r["accuracy_match"] = r["accuracy_line"] == base["accuracy_line"]
            out[key] = r
        return out
    finally:
        shutil.rmtree(wd, ignore_errors=True)


# ---------------------------------------------------------------------------
# The reference's own published workload (pdf p.12-13, cpp:108-119): the MNIST
# shape 60k train x (10k validation + 10k test), d=784, K=50, L2, normalised,
# validation on.  Inputs: the golden fixture f11_mnist_shape's CSVs
# (tests/golden, regenerated from its spec and checked against the sha256 of
# the bytes the reference itself read), so the drop-in's Test_label.csv and
# accuracy line are compared with the reference's own outputs.
MNIST_FIXTURE = "f11_mnist_shape"
MNIST_PUBLISHED = {"1_process_s": 2921.11, "1000_processes_s": 8.270078,
                   "source": "pdf p.13 (whole-program wall time, mean of 5 runs, unspecified "
                             "supercomputer; BASELINE.md section 1)"}
MNIST_REF_SAMPLE = 256  # test queries of the reference's timed sample run


def mnist_reference_sample(wd, fx, sets):
    """The reference program at the MNIST shape on a sample: N_test =
    MNIST_REF_SAMPLE (the first rows of the test CSV), Validation off, under
    mpirun on the granted host cores; its timed test loop extrapolated
    linearly to the 20k queries of the published run (every query costs the
    same: 60k distances + a 60k-record std::sort).  The sample's min-max
    bounds come from train + sample rows, so its labels are not compared."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import build_ref
    import datagen
    import ref_runner
    s = fx.spec
    S = MNIST_REF_SAMPLE
    cores, share = host_cores()
    nprocs = max(p for p in range(2, max(2, share) + 1)
                 if s["N_train"] % p == 0 and S % p == 0)
    exe = build_ref.build_ref(mnist_ref_config(fx), instrument=False, timing=True)
    rd = os.path.join(wd, "ref_sample")
    os.makedirs(rd)
    os.symlink(os.path.join(wd, "mnist_train.csv"), os.path.join(rd, "mnist_train.csv"))
    tr, trl, te, tel, va, val_ = sets
    with open(os.path.join(rd, "mnist_test.csv"), "w") as f:  # exactly N_test rows (cpp:180-194)
        f.write(datagen._fmt_rows(te[:S], None, s["kind"]))
    with open(os.path.join(rd, "mnist_validation.csv"), "w") as f:
        f.write(datagen._fmt_rows(va[:S], val_[:S], s["kind"]))
    _, loop_s, run_s = ref_runner.run_reference(exe, rd, nprocs, timeout=300)
    q = s["N_test"] + s["N_val"]
    per_q = loop_s / S
    return {"kind": "reference", "ranks": nprocs, "cores": nprocs, "host_cores": cores,
            "cpu_share": share, "sample_queries": S, "test_loop_s": loop_s,
            "running_time_s": run_s,
            "extrapolated_running_time_s": run_s - loop_s + per_q * q,
            "queries_per_s": S / loop_s,
            "sample": "/root/reference/knn_mpi.cpp (constants: the MNIST shape with N_test = %d, "
                      "Validation off, timer around the test loop) under mpirun -np %d on the "
                      "box's host CPUs (%d visible, share %d): test loop %.2f s for %d queries, "
                      "whole run %.1f s incl. the 60k-row CSV parse, MPI_Bcast and normalisation; "
                      "the published run's %d queries extrapolated linearly"
                      % (S, nprocs, cores, share, loop_s, S, run_s, q)}


def mnist_ref_config(fx):
    s = fx.spec
    return dict(dim=s["dim"], K=s["K"], N_train=s["N_train"], N_test=MNIST_REF_SAMPLE,
                N_val=MNIST_REF_SAMPLE, class_cnt=s["class_cnt"], Validation=False,
                Normalize=bool(s["Normalize"]), Euclidean_distance=bool(s["Euclidean_distance"]))


def mnist_leg(world):
    """bin/knn_mpi_amd at the reference's published workload on one GPU; its
    labels and accuracy line against the golden fixture (the reference's own
    outputs on these CSVs), beside pdf p.13's times and the reference timed
    on this box's host cores (N=1 lines only)."""
    import shutil
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import golden_io
    fx = golden_io.Fixture(MNIST_FIXTURE)
    s = fx.spec
    wd = tempfile.mkdtemp(prefix="knn_mnist_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        t0 = time.perf_counter()
        sets = fx.write_inputs(wd, names=("mnist_train.csv", "mnist_validation.csv",
                                          "mnist_test.csv"))
        gen_s = time.perf_counter() - t0
        shape = dict(n=s["N_train"], m=s["N_test"], d=s["dim"], k=s["K"], classes=s["class_cnt"])
        r = run_dropin(wd, 1, "query", shape, timeout=300)
        got = np.loadtxt(os.path.join(wd, "Test_label_query_1.csv"), dtype=np.int64, ndmin=1)
        want = fx.test_labels
        out = {"workload": "the reference's published run (pdf p.12-13, cpp:108-119): %d train x "
                           "(%d validation + %d test) queries, d=%d, K=%d, L2, normalised, "
                           "validation on; bin/knn_mpi_amd on 1 GPU, inputs = golden fixture %s "
                           "(synthetic Gaussian mixture of the MNIST shape, CSV sha256 checked)"
                           % (s["N_train"], s["N_val"], s["N_test"], s["dim"], s["K"],
                              MNIST_FIXTURE),
               "running_time_s": r["running_time_s"], "process_wall_s": r["process_wall_s"],
               "phases_s": r["phases_s"], "input_generation_s": gen_s,
               "queries_per_s": (s["N_test"] + s["N_val"]) / r["running_time_s"]
               if r["running_time_s"] else None,
               "accuracy_line": r["accuracy_line"],
               "labels_match_reference": bool(got.shape == want.shape and (got == want).all()),
               "accuracy_matches_reference": r["accuracy_line"] == str(fx.accuracy_line),
               "test_label_sha1": r["test_label_sha1"],
               "published": MNIST_PUBLISHED,
               "speedup_vs_published_1_process": MNIST_PUBLISHED["1_process_s"] / r["running_time_s"]
               if r["running_time_s"] else None,
               "speedup_vs_published_1000_processes": MNIST_PUBLISHED["1000_processes_s"]
               / r["running_time_s"] if r["running_time_s"] else None}
        if world == 1:
            try:
                out["cpu_reference"] = mnist_reference_sample(wd, fx, sets)
            except (OSError, RuntimeError, ValueError, subprocess.SubprocessError) as e:
                out["cpu_reference"] = {"error": "reference sample run unavailable: %s" % e}
        return out
    finally:
        shutil.rmtree(wd, ignore_errors=True)


# ---------------------------------------------------------------------------
# configs[3] in the N-rank run: train-sharded, 100M x 96 split over the ranks,
# 10k queries on every rank, local exact top-(k+1) -> ONE all-gather of the
# packed lists -> k-way merge + vote of each rank's query slice.
def _local_topk(X, r0, Qs, k, chunk=1 << 22):
    """Independent fp64 brute force (GEMM form) over this rank's rows:
    (distances [S, k], global indices [S, k])."""
    qn = (Qs * Qs).sum(1, keepdim=True)
    bd = bi = None
    for c0 in range(0, X.shape[0], chunk):
        Xc = X[c0:c0 + chunk]
        D2 = (qn + (Xc * Xc).sum(1)[None, :] - 2.0 * (Qs @ Xc.T)).clamp_(min=0.0)
        v, i = torch.topk(D2, min(k, D2.shape[1]), dim=1, largest=False)
        i = i + (r0 + c0)
        if bd is not None:
            v, j = torch.topk(torch.cat([bd, v], 1), k, dim=1, largest=False)
            i = torch.gather(torch.cat([bi, i], 1), 1, j)
        bd, bi = v, i
    return bd.sqrt(), bi


def verify_train_sharded(kd, X, lab, r0, r1, Q, k, got, idx, dist, sample, world):
    """The full-size cfg4 test's checks on a query sample, across ranks:
    reported distances = the reference formula for the reported rows
    (cpp:33-50, dims added in order in fp64, recomputed where the row lives),
    vote = cpp:324-337 over the reported rows' labels, optimality against an
    independent fp64 brute force over all n rows (1e-10 relative)."""
    Qs = Q[sample]
    ids = idx[sample]                                   # [S, k] global rows
    mine = (ids >= r0) & (ids < r1)
    loc = (ids - r0).clamp_(0, r1 - r0 - 1)
    rows = X[loc]                                       # [S, k, d]
    r = torch.zeros(ids.shape, dtype=torch.float64, device=X.device)
    for j in range(X.shape[1]):
        t = Qs[:, None, j] - rows[:, :, j]
        r = r + t * t
    r = torch.where(mine, r, torch.zeros_like(r))
    labs = torch.where(mine, lab[loc].long(), torch.zeros_like(ids))
    bv, bi = _local_topk(X, r0, Qs, k)
    if world > 1:
        dist.all_reduce(r)
        dist.all_reduce(labs)
        allv = [torch.empty_like(bv) for _ in range(world)]
        dist.all_gather(allv, bv)
        bv = torch.topk(torch.cat(allv, 1), k, dim=1, largest=False).values
    dist_ok = bool((r.sqrt().view(torch.int64) == dist[sample].view(torch.int64)).all())
    ln = labs.cpu().numpy()
    want = np.empty(ln.shape[0], np.int32)
    for q in range(ln.shape[0]):
        cnt, best, bl = {}, 0, -1
        for t in range(k):
            cnt[ln[q, t]] = cnt.get(ln[q, t], 0) + 1
            if cnt[ln[q, t]] > best:
                best, bl = cnt[ln[q, t]], int(ln[q, t])
        want[q] = bl
    vote_ok = bool((want == got[sample].cpu().numpy()).all())
    opt_ok = bool(torch.allclose(dist[sample], bv, rtol=1e-10, atol=0.0))
    return {"sample_queries": int(len(sample)), "distances_bit_exact": dist_ok,
            "vote_consistent": vote_ok, "optimal_vs_fp64_brute_force": opt_ok,
            "labels_match": dist_ok and vote_ok and opt_ok}


def train_sharded_leg(args, kd, knn, world, rank, local, dev, sync):
    n, m, d, k, C = args.ts_n_train, args.ts_queries, 96, args.k, args.classes
    r0, r1 = kd.shard_range(n, world, rank)
    X, lab, Q, _ = synth(r1 - r0, m, d, C, 2468, 1357, dev, row0=r0, n_total=n)
    sync()
    ctx = knn.Classifier(local)
    ctx.set_timing(True)
    t0 = time.perf_counter()
    ctx.set_train_device(X.data_ptr(), lab.data_ptr(), r1 - r0, d, C, idx_offset=r0, keep=(X, lab))
    sync()
    set_train_ms = (time.perf_counter() - t0) * 1e3
    w = k + 1
    pd_ = torch.empty((m, w), dtype=torch.float64, device=dev)
    pi_ = torch.empty((m, w), dtype=torch.int64, device=dev)
    pl_ = torch.empty((m, w), dtype=torch.int32, device=dev)
    q0, q1 = kd.shard_range(m, world, rank)
    mq = max(1, q1 - q0)
    o_lab = torch.empty(mq, dtype=torch.int32, device=dev)
    o_idx = torch.empty((mq, k), dtype=torch.int64, device=dev)
    o_dist = torch.empty((mq, k), dtype=torch.float64, device=dev)
    o_flg = torch.empty(mq, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream

    def search_partial(Qt):
        ctx.search_partial_device(Qt.data_ptr(), m, w, knn.L2, pd_.data_ptr(), pi_.data_ptr(),
                                  pl_.data_ptr(), stream)
        return pd_, pi_, pl_

    def merge_vote(gd, gi, gl, parts, a, b):
        ctx.merge_vote_device(gd.data_ptr(), gi.data_ptr(), gl.data_ptr(), parts, m, w, k,
                              o_lab.data_ptr(), o_idx.data_ptr(), o_dist.data_ptr(),
                              o_flg.data_ptr(), stream=stream, q0=a, mq=b - a)
        return o_lab

    # queries whose label the reference's tie order decides: every shard's
    # distances to their owner, re-sorted as the reference's std::sort
    ties = kd.HipTies(ctx, Q, lab, n, k, (o_lab, o_idx, o_dist, o_flg), q1 - q0, stream=stream,
                      device=dev)

    def step():
        kd.train_sharded(search_partial, merge_vote, Q, m, w, k, dev, ties=ties)

    steps = max(2, args.steps // 3)
    r = timed_run(kd, ctx, step, steps, 1, sync, dev, knn.PRECISION_AUTO)
    got = kd.gather_slices(o_lab[:q1 - q0], m, dev)
    idx = kd.gather_slices(o_idx[:q1 - q0], m, dev)
    dst = kd.gather_slices(o_dist[:q1 - q0], m, dev)
    flg = kd.gather_slices(o_flg[:q1 - q0], m, dev)
    sample = torch.arange(0, m, max(1, m // 64), device=dev)
    chk = verify_train_sharded(kd, X, lab, r0, r1, Q, k, got, idx, dst, sample, world)
    pr = per_rank_report(dev, {"kernel_ms": r["t_cand"] * 1e3, "rescanned_queries": r["resc"],
                               "tie_resolved_queries": ties.resolved,
                               "tie_pending_queries": int(((o_flg[:q1 - q0] & ties.FLAG_TIE_PENDING)
                                                           != 0).sum().item())})
    flops = 2.0 * (r1 - r0) * d * m
    ach = flops / r["t_cand"] / 1e12
    out = {
        "workload": "configs[3]: %d train rows sharded over %d GPU(s) (%d per rank) x %d queries, "
                    "d=%d, k=%d; local exact top-%d, one packed all-gather, k-way merge + vote"
                    % (n, world, r1 - r0, m, d, k, w),
        "value": m * steps / r["el"], "unit": "queries/s", "n_gpus": world, "steps": steps,
        "ms_per_step": r["el"] / steps * 1e3, "scaling": "strong",
        "kernel": r["kernel"], "kernel_ms_max_over_ranks": max(pr["kernel_ms"]),
        "per_rank": pr, "labels_sha1": labels_sha1(got),
        "roofline_rank0": {"achieved": ach, "peak": peak_of(r["path"]), "unit": "TFLOP/s",
                           "frac": ach / peak_of(r["path"]), "candidate_path": r["path"]},
        "allgather_bytes_per_rank": (m * w * 20 + 15) // 16 * 16 if world > 1 else 0,
        "set_train_ms": set_train_ms, "rescanned_queries": r["resc"],
        "tie_vote_queries": int(((flg & knn.FLAG_TIE_VOTE) != 0).sum().item()),
        "tie_resolved_queries_rank0": ties.resolved,
        "check": chk, "labels_match": chk["labels_match"]}
    ctx.close()
    del X, lab, Q, pd_, pi_, pl_
    torch.cuda.empty_cache()
    return out


def cfg5_leg(args, kd, knn, dev, sync, stream):
    """configs[4]: 1M train x 10k queries, d=960 (GIST-like), k=100 on one GPU:
    the fp16 candidate pass on the streamed S3 kernel + the exact fp64
    re-rank; roofline against the fp16 MFMA peak, PMC traffic of the same
    kernel build when profiled, and the oracle port on a query sample."""
    n, m, d, k, C = 1_000_000, 10_000, 960, 100, args.classes
    X, lab, Q, _ = synth(n, m, d, C, 4321, 8765, dev)
    sync()
    ctx = knn.Classifier(torch.cuda.current_device())
    ctx.set_timing(True)
    t0 = time.perf_counter()
    ctx.set_train_device(X.data_ptr(), lab.data_ptr(), n, d, C, keep=(X, lab))
    sync()
    set_train_ms = (time.perf_counter() - t0) * 1e3
    out = torch.empty(m, dtype=torch.int32, device=dev)

    def step():
        ctx.classify_device(Q.data_ptr(), m, k, knn.L2, out.data_ptr(), None, None, None, stream)

    steps = max(3, args.steps // 4)
    r = timed_run(kd, ctx, step, steps, 1, sync, dev, knn.PRECISION_AUTO)
    flops = 2.0 * n * d * m
    ach = flops / r["t_cand"] / 1e12
    peak = peak_of(r["path"])
    tr, tr_src = pmc_traffic(r["kernel"], {"n_train": n, "queries": m, "dim": d, "k": k},
                             kernel_src_sha())
    res = {"workload": "cfg5: %d train x %d queries, d=%d, k=%d, L2, %d classes" % (n, m, d, k, C),
           "value": m * steps / r["el"], "unit": "queries/s", "n_gpus": 1, "steps": steps,
           "ms_per_step": r["el"] / steps * 1e3, "set_train_ms": set_train_ms,
           "kernel": r["kernel"], "kernel_ms": r["t_cand"] * 1e3, "rerank_ms": r["rr"],
           "rescanned_queries": r["resc"], "candidate_path": r["path"],
           "roofline": {"bound": "mfma", "achieved": ach, "peak": peak, "unit": "TFLOP/s",
                        "frac": ach / peak, "traffic": tr,
                        "traffic_unit": "bytes per launch (HBM, PMC)", "traffic_source": tr_src,
                        "algorithmic_bytes_per_launch": (n + m) * d * 4 + m * k * 8,
                        "algorithmic_flops_per_launch": flops, "kernel": r["kernel"]}}
    if not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(X, lab, Q, k, C, out.cpu().numpy(), budget_s=5.0)
    ctx.close()
    del X, lab, Q
    torch.cuda.empty_cache()
    return res


def main():
    """Runs the bench; any failure on any rank exits non-zero naming the rank
    and the phase it was in (a hung collective fails after the process
    group's timeout, KNN_BENCH_COLL_TIMEOUT_S, default 600 s)."""
    try:
        _main()
    except SystemExit:
        raise
    except BaseException as e:  # noqa: B902 -- report and exit 1 on anything
        print("[bench.py] rank %s of %s FAILED in phase '%s': %s: %s"
              % (os.environ.get("RANK", "0"), os.environ.get("WORLD_SIZE", "1"), PHASE[0],
                 type(e).__name__, e), file=sys.stderr, flush=True)
        traceback.print_exc()
        sys.stderr.flush()
        os._exit(1)


def _main():
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
    ap.add_argument("--data", choices=("grid", "continuous"), default="grid")
    ap.add_argument("--cfg3-queries", type=int, default=1_000_000,
                    help="configs[2] strong-scaling leg: total queries split over the ranks "
                         "(0 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fp32-path", action="store_true")
    ap.add_argument("--no-continuous", action="store_true",
                    help="skip the continuous-data leg of the default run")
    ap.add_argument("--no-dropin", action="store_true",
                    help="skip the native drop-in legs (bin/knn_mpi_amd through knn_group)")
    ap.add_argument("--no-train-sharded", action="store_true",
                    help="skip the configs[3] train-sharded leg")
    ap.add_argument("--ts-n-train", type=int, default=100_000_000,
                    help="train-sharded leg: train rows split over the ranks (d=96)")
    ap.add_argument("--ts-queries", type=int, default=10_000,
                    help="train-sharded leg: queries (the same on every rank)")
    ap.add_argument("--no-mnist", action="store_true",
                    help="skip the reference's published workload (MNIST shape through bin/knn_mpi_amd)")
    ap.add_argument("--no-cfg5", action="store_true",
                    help="skip the configs[4] leg (1M x 10k, d=960, k=100)")
    ap.add_argument("--precision", choices=("auto", "fp32", "fp16"), default="auto",
                    help="candidate pass of the main leg (profiling of the fp32 / fp16 kernels)")
    ap.add_argument("--order", type=int, default=-1,
                    help="region order of the train layout (tuning key 'order': -1 auto, 0 off)")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="extra knn_set_tuning key of the main leg (profiling of a variant, "
                         "e.g. qres=1 for the query-resident d > 256 kernel); repeatable")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU/gloo plumbing check with a torch stand-in (no measurement)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("note: --gpus %d but the launcher started %d ranks; reporting %d"
            % (args.gpus, world, world))
    kd = _load("knn_dist")
    if args.dry_run:
        return dry_run(args, kd, world, rank)
    # the native drop-in over all N GPUs, as a child process, before this
    # process (or any other rank) touches a GPU
    dropin = None if args.no_dropin or args.mode != "query" else dropin_phase(
        world, rank, mnist=not args.no_mnist)

    phase("device %d setup" % local)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        phase("init_process_group (nccl = RCCL) over %d ranks" % world)
        dist.init_process_group("nccl", device_id=dev, timeout=timedelta(
            seconds=float(os.environ.get("KNN_BENCH_COLL_TIMEOUT_S", "600"))))
    knn = load_knn()
    n, m, d, k, C = args.n_train, args.queries, args.dim, args.k, args.classes
    sync = torch.cuda.synchronize
    stream = torch.cuda.current_stream().cuda_stream
    clf = knn.Classifier(local)
    clf.set_timing(True)
    extra = {}

    def allreduce_minmax(mx, mn):
        if world > 1:
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
            dist.all_reduce(mn, op=dist.ReduceOp.MIN)

    if args.mode == "query":
        # train generated on rank 0 and RCCL-broadcast (≙ MPI_Bcast cpp:224-225);
        # rank r's weak-scaling queries are rows [r m, (r+1) m) of one query set
        phase("synthetic data (query mode)")
        X, lab, Q, _ = synth(n, m, d, C, 1234, 5678, dev, data=args.data, q0=rank * m,
                             reduce=allreduce_minmax, q_total=m * world)
        sync()
        if world > 1:
            phase("train broadcast (RCCL, rank 0 -> all)")
            dist.barrier()
            sync()
            t0 = time.perf_counter()
            kd.broadcast_train(X, lab)
            sync()
            dist.barrier()
            bt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
            dist.all_reduce(bt, op=dist.ReduceOp.MAX)
            extra["train_broadcast_ms"] = float(bt.item()) * 1e3
            extra["train_broadcast_gbps"] = (X.numel() * 8 + lab.numel() * 4) / float(bt.item()) / 1e9
        log("synthetic train ready: %d rows x %d (%s data)" % (n, d, args.data))
        phase("set_train (main leg)")
        t0 = time.perf_counter()
        clf.set_tuning("order", args.order)
        for kv in args.tune:
            key, val = kv.split("=")
            clf.set_tuning(key, int(val))
        clf.set_train_device(X.data_ptr(), lab.data_ptr(), n, d, C, keep=(X, lab))
        sync()
        extra["set_train_ms"] = (time.perf_counter() - t0) * 1e3
        out_lab = torch.empty(m, dtype=torch.int32, device=dev)
        out_flags = torch.empty(m, dtype=torch.int32, device=dev)

        def step():
            clf.classify_device(Q.data_ptr(), m, k, knn.L2, out_lab.data_ptr(), None, None,
                                out_flags.data_ptr(), stream)

        n_rank, m_rank = n, m
        flops = 2.0 * n * d * m  # algorithmic, per launch per GPU (norm terms excluded)
        prec_main = {"auto": knn.PRECISION_AUTO, "fp32": knn.PRECISION_FP32,
                     "fp16": knn.PRECISION_FP16}[args.precision]
        phase("main leg (query-sharded, %d queries per rank)" % m)
        main_r = timed_run(kd, clf, step, args.steps, args.warmup, sync, dev, prec_main)
        clf.set_precision(knn.PRECISION_AUTO)
        log("default path done: %.3f ms/step" % (main_r["el"] / args.steps * 1e3))
        labels_auto = out_lab.clone()
        flags_auto = out_flags.clone()
        tie_vote = int(((flags_auto & knn.FLAG_TIE_VOTE) != 0).sum().item())
        phase("main leg per-rank report")
        pr = per_rank_report(dev, {"kernel_ms": main_r["t_cand"] * 1e3,
                                   "rescanned_queries": main_r["resc"],
                                   "tie_vote_queries": tie_vote,
                                   "tie_reordered_queries": main_r["tie_reordered"]}, labels_auto)
        extra["per_rank"] = pr
        extra["labels_sha1_rank0"] = pr["labels_sha1"][0]
        tie_vote = int(sum(pr["tie_vote_queries"]))
        extra["tie_vote_queries"] = tie_vote
        fp32_r = same = fp16_r = same16 = None
        if not args.no_fp32_path and world == 1:
            fp32_r = timed_run(kd, clf, step, max(3, args.steps // 2), 1, sync, dev,
                               knn.PRECISION_FP32)
            same = bool(torch.equal(labels_auto, out_lab))
            clf.set_precision(knn.PRECISION_AUTO)
            if main_r["path"] in (5, 6):
                # the fp16 candidate pass on the same data (the int8 pass off)
                clf.set_tuning("i8", 0)
                fp16_r = timed_run(kd, clf, step, max(3, args.steps // 2), 1, sync, dev,
                                   knn.PRECISION_AUTO)
                same16 = bool(torch.equal(labels_auto, out_lab))
                clf.set_tuning("i8", -1)
        total_q = m * world * args.steps
        tag = {(1_000_000, 128, 10): "cfg2", (1_000_000, 960, 100): "cfg5"}.get((n, d, k), "custom")
        workload = ("%s: %d train x %d queries per GPU, d=%d, k=%d, L2, %d classes"
                    % (tag, n, m, d, k, C))
        parallelism = "query-sharded dp%d" % world
        scaling = "weak"

        if args.cfg3_queries > 0 and d == 128 and n == 1_000_000:
            # configs[2]: a fixed query count split over the ranks (strong scaling)
            M = args.cfg3_queries
            q0, q1 = kd.shard_range(M, world, rank)
            _, _, Q3, _ = synth(0, q1 - q0, d, C, 1234, 91011, dev, data=args.data, q0=q0,
                                q_total=M)
            if args.data == "continuous":  # the train set's normalisation bounds are already applied
                Q3 = None
            if Q3 is not None:
                lab3 = torch.empty(q1 - q0, dtype=torch.int32, device=dev)
                flg3 = torch.empty(q1 - q0, dtype=torch.int32, device=dev)

                def step3():
                    clf.classify_device(Q3.data_ptr(), q1 - q0, k, knn.L2, lab3.data_ptr(), None,
                                        None, flg3.data_ptr(), stream)

                s3 = max(2, args.steps // 4)
                phase("cfg3 strong-scaling leg (%d of %d queries)" % (q1 - q0, M))
                r3 = timed_run(kd, clf, step3, s3, 1, sync, dev, knn.PRECISION_AUTO)
                extra["cfg3_strong"] = {
                    "workload": "cfg3: %d train x %d queries in total split over %d GPU(s) "
                                "(%d per rank), d=%d, k=%d" % (n, M, world, q1 - q0, d, k),
                    "value": M * s3 / r3["el"], "unit": "queries/s", "n_gpus": world,
                    "steps": s3, "ms_per_step": r3["el"] / s3 * 1e3, "scaling": "strong",
                    "kernel_ms": r3["t_cand"] * 1e3, "rescanned_queries": r3["resc"],
                    "tie_reordered_queries": r3["tie_reordered"],
                    "candidate_path": r3["path"]}
                tv3 = torch.tensor([int(((flg3 & knn.FLAG_TIE_VOTE) != 0).sum().item())],
                                   dtype=torch.int64, device=dev)
                if world > 1:
                    dist.all_reduce(tv3)
                extra["cfg3_strong"]["tie_vote_queries"] = int(tv3.item())
                # every N classifies the same M queries: one sha1 of all M labels
                all3 = kd.gather_slices(lab3, M, dev)
                extra["cfg3_strong"]["labels_sha1"] = labels_sha1(all3)
                extra["cfg3_strong"]["per_rank"] = per_rank_report(
                    dev, {"kernel_ms": r3["t_cand"] * 1e3, "rescanned_queries": r3["resc"]})
                del all3
                log("cfg3 strong leg: %.1f ms/step" % (r3["el"] / s3 * 1e3))
                del Q3, lab3, flg3

        if not args.no_continuous and args.data == "grid" and world == 1:
            # the same workload on continuous (min-max normalised, off-grid) data
            Xc, labc, Qc, _ = synth(n, m, d, C, 4242, 2424, dev, data="continuous")
            clf.set_train_device(Xc.data_ptr(), labc.data_ptr(), n, d, C, keep=(Xc, labc))
            outc = torch.empty(m, dtype=torch.int32, device=dev)

            def stepc():
                clf.classify_device(Qc.data_ptr(), m, k, knn.L2, outc.data_ptr(), None, None,
                                    None, stream)

            sc = max(3, args.steps // 2)
            rc = timed_run(kd, clf, stepc, sc, 1, sync, dev, knn.PRECISION_AUTO)
            ac = flops / rc["t_cand"] / 1e12
            wlc = {"n_train": n, "queries": m, "dim": d, "k": k, "data": "continuous"}
            trc, trc_src = pmc_traffic(rc["kernel"], wlc, kernel_src_sha())
            extra["continuous_data"] = {
                "data": "same Gaussian mixture, min-max normalised as cpp:229-306 (train and "
                        "queries), not quantised: values on no power-of-two grid",
                "value": m * sc / rc["el"], "unit": "queries/s", "ms_per_step": rc["el"] / sc * 1e3,
                "kernel_ms": rc["t_cand"] * 1e3, "frac": ac / peak_of(rc["path"]),
                "candidate_path": rc["path"], "rescanned_queries": rc["resc"],
                "rescanned_per_step": rc["resc"] / rc["calls"], "full_scans": rc["full_scans"],
                "tie_reordered_queries": rc["tie_reordered"],
                "roofline": {"bound": "mfma", "achieved": ac, "peak": peak_of(rc["path"]),
                             "unit": "TFLOP/s", "frac": ac / peak_of(rc["path"]), "traffic": trc,
                             "traffic_unit": "bytes per launch (HBM, PMC)",
                             "traffic_source": trc_src, "kernel": rc["kernel"],
                             "algorithmic_bytes_per_launch": (n + m) * d * 4 + m * k * 8,
                             "algorithmic_flops_per_launch": flops}}
            if not args.no_cpu_baseline:
                log("cpu baseline of the continuous-data leg (oracle port) ...")
                extra["continuous_data"]["cpu_baseline"] = cpu_baseline(
                    Xc, labc, Qc, k, C, outc.cpu().numpy(), budget_s=4.0)
            log("continuous-data leg: %.3f ms/step, %d rescans" % (rc["el"] / sc * 1e3, rc["resc"]))
            del Xc, labc, Qc
            clf.set_train_device(X.data_ptr(), lab.data_ptr(), n, d, C, keep=(X, lab))
        if not args.no_cfg5 and world == 1 and (n, d, k) == (1_000_000, 128, 10):
            log("cfg5 leg (1M x 10k, d=960, k=100) ...")
            extra["cfg5"] = cfg5_leg(args, kd, knn, dev, sync, stream)
            log("cfg5 leg: %.2f ms/step" % extra["cfg5"]["ms_per_step"])
    else:
        # train-sharded: this rank's rows only; the same queries on every rank
        r0, r1 = kd.shard_range(n, world, rank)
        X, lab, Q, _ = synth(r1 - r0, m, d, C, 1234, 5678, dev, row0=r0, n_total=n,
                             data=args.data, reduce=allreduce_minmax)
        sync()
        log("synthetic shard ready: %d rows x %d" % (r1 - r0, d))
        t0 = time.perf_counter()
        clf.set_train_device(X.data_ptr(), lab.data_ptr(), r1 - r0, d, C, idx_offset=r0,
                             keep=(X, lab))
        sync()
        extra["set_train_ms"] = (time.perf_counter() - t0) * 1e3
        w = k + 1
        pd_ = torch.empty((m, w), dtype=torch.float64, device=dev)
        pi_ = torch.empty((m, w), dtype=torch.int64, device=dev)
        pl_ = torch.empty((m, w), dtype=torch.int32, device=dev)
        q0, q1 = kd.shard_range(m, world, rank)
        out_lab = torch.empty(max(1, q1 - q0), dtype=torch.int32, device=dev)
        out_flg = torch.empty(max(1, q1 - q0), dtype=torch.int32, device=dev)

        def search_partial(Qt):
            clf.search_partial_device(Qt.data_ptr(), m, w, knn.L2, pd_.data_ptr(), pi_.data_ptr(),
                                      pl_.data_ptr(), stream)
            return pd_, pi_, pl_

        def merge_vote(gd, gi, gl, parts, a, b):  # k-way merge + vote of this rank's slice
            clf.merge_vote_device(gd.data_ptr(), gi.data_ptr(), gl.data_ptr(), parts, m, w, k,
                                  out_lab.data_ptr(), d_flags=out_flg.data_ptr(), stream=stream,
                                  q0=a, mq=b - a)
            return out_lab

        ties = kd.HipTies(clf, Q, lab, n, k, (out_lab, None, None, out_flg), q1 - q0,
                          stream=stream, device=dev)

        def step():
            kd.train_sharded(search_partial, merge_vote, Q, m, w, k, dev, ties=ties)

        n_rank, m_rank = r1 - r0, m
        flops = 2.0 * (r1 - r0) * d * m
        main_r = timed_run(kd, clf, step, args.steps, args.warmup, sync, dev, knn.PRECISION_AUTO)
        fp32_r, same, fp16_r, same16 = None, None, None, None
        total_q = m * args.steps
        workload = ("cfg4-shape: %d train (sharded) x %d queries, d=%d, k=%d, L2, %d classes"
                    % (n, m, d, k, C))
        parallelism = "train-sharded tp%d" % world
        scaling = "strong"

    ts = None
    if args.mode == "query" and not args.no_train_sharded:
        log("train-sharded leg: %d rows over %d rank(s) ..." % (args.ts_n_train, world))
        phase("train-sharded leg (%d rows over %d ranks)" % (args.ts_n_train, world))
        ts = train_sharded_leg(args, kd, knn, world, rank, local, dev, sync)
        log("train-sharded leg: %.2f ms/step, labels_match %s" % (ts["ms_per_step"],
                                                                ts["labels_match"]))

    path = main_r["path"]
    bf16 = path in (2, 3)
    # fp16 / bf16 MFMA share the dense peak; bf16x3 issues 3 MFMA flops per
    # algorithmic flop, fp16 and fp32 one
    peak = peak_of(path)
    mfma_mult = 3.0 if bf16 else 1.0
    cand_desc = {
        0: "fp32 MFMA 32x32x2",
        2: "bf16x3 split (qh.xh+ql.xh+qh.xl) on MFMA 32x32x16 bf16",
        3: "bf16x3 split (qh.xh+ql.xh+qh.xl) on MFMA 16x16x32 bf16",
        4: "fp16 operands (power-of-two scaled, centred) on MFMA 16x16x32 f16",
        5: "int8 codes of the data's 8-bit grid (exact integer arithmetic) on MFMA 16x16x64 i8",
        6: "int8 codes of the data's 8-bit grid (exact integer arithmetic) on MFMA 32x32x32 i8",
    }.get(path, "kernel metric %d" % path)
    achieved = flops / main_r["t_cand"] / 1e12
    kname = main_r["kernel"]
    src_sha = kernel_src_sha()
    wl = {"n_train": n_rank, "queries": m_rank, "dim": d, "k": k, "data": args.data}
    if args.tune:
        wl["tuning"] = ",".join(args.tune)
    traffic, traffic_src = pmc_traffic(kname, wl, src_sha)
    result = {
        "metric": METRIC,
        "value": total_q / main_r["el"],
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": main_r["el"] / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": {2: "bf16x3", 3: "bf16x3", 4: "fp16", 5: "int8", 6: "int8"}.get(path, "fp32"),
        "data": ("synthetic (seeded Gaussian mixture scaled to [0,1) on the 8-bit grid k/256, "
                 "SIFT-like; fp64 inputs)" if args.data == "grid" else
                 "synthetic (seeded Gaussian mixture, min-max normalised as cpp:229-306, "
                 "continuous values; fp64 inputs)"),
        "config": {"workload": workload, "n_train": n, "queries": m, "dim": d, "k": k,
                   "parallelism": parallelism,
                   "candidate_pass": cand_desc + " + fused top-R per lane, certified bound",
                   "rerank": "fp64 exact (reference arithmetic), certified; labels exact",
                   "geometry": main_r["geom"], "rescanned_queries": main_r["resc"],
                   "full_scan_queries": main_r["full_scans"],
                   "tie_reordered_queries": main_r["tie_reordered"],
                   **({"tuning": list(args.tune)} if args.tune else {})},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                     "frac": achieved / peak, "traffic": traffic,
                     "traffic_unit": "bytes per launch (HBM, PMC)", "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": (n_rank + m_rank) * d * 4 + m_rank * k * 8,
                     "kernel": kname, "kernel_src_sha": src_sha,
                     "kernel_ms": main_r["t_cand"] * 1e3, "rerank_ms": main_r["rr"],
                     "rescan_ms": main_r["rescan_ms"], "prep_ms": main_r["prep_ms"],
                     "timed_launches": main_r["calls"],
                     "phase_ms_source": ("kernel_ms: HIP events around the candidate kernel of "
                                         "the %d timed calls; prep/rerank/rescan_ms: %d further "
                                         "untimed calls after the timed region with every "
                                         "phase's events" % (main_r["calls"], main_r["phase_calls"])),
                     "algorithmic_flops_per_launch": flops,
                     "mfma_flops_per_algorithmic_flop": mfma_mult,
                     "frac_of_issued_mfma": achieved * mfma_mult / peak},
        "cpu_baseline": None,
    }
    result.update(extra)
    if dropin is not None:
        for key in ("group_query", "group_train", "group_1gpu", "error", "mnist_shape"):
            if key in dropin:
                result[key] = dropin[key]
        result["group_workload"] = dropin.get("workload")
    if ts is not None:
        result["train_sharded"] = ts
    if args.mode == "query":
        result["scaling_note"] = (
            "value is weak scaling (10k queries per GPU); north_star's >=7x-at-8-GPUs claim "
            "rests on cfg3_strong (a fixed 1M queries split over the ranks) and the "
            "train_sharded leg (a fixed 100M x 96 train set split over the ranks)")
        if world > 1:
            result["cpu_baseline_note"] = ("measured at N=1 only (rank 0, host cores of one "
                                           "GPU's share); see the N=1 line")
    if fp32_r is not None:
        a32 = flops / fp32_r["t_cand"] / 1e12
        tr32, tr32_src = pmc_traffic(fp32_r["kernel"], wl, src_sha)
        result["fp32_path"] = {
            "value": m * world * fp32_r["calls"] / fp32_r["el"], "unit": "queries/s",
            "kernel": fp32_r["kernel"], "kernel_ms": fp32_r["t_cand"] * 1e3, "achieved": a32,
            "peak": PEAK_FP32_TFLOPS, "frac": a32 / PEAK_FP32_TFLOPS,
            "traffic": tr32, "traffic_unit": "bytes per launch (HBM, PMC)",
            "traffic_source": tr32_src,
            "rescanned_queries": fp32_r["resc"], "geometry": fp32_r["geom"],
            "labels_equal_default_path": same}
    if fp16_r is not None:
        a16 = flops / fp16_r["t_cand"] / 1e12
        result["fp16_path"] = {
            "value": m * world * fp16_r["calls"] / fp16_r["el"], "unit": "queries/s",
            "ms_per_step": fp16_r["el"] / fp16_r["calls"] * 1e3,
            "kernel": fp16_r["kernel"], "kernel_ms": fp16_r["t_cand"] * 1e3, "achieved": a16,
            "peak": peak_of(fp16_r["path"]), "frac": a16 / peak_of(fp16_r["path"]),
            "candidate_path": fp16_r["path"], "rescanned_queries": fp16_r["resc"],
            "labels_equal_default_path": same16}
    if rank == 0 and world == 1 and args.mode == "query" and not args.no_cpu_baseline:
        log("cpu baseline (oracle port) ...")
        port = cpu_baseline(X, lab, Q, k, C, labels_auto.cpu().numpy(), budget_s=6.0)
        result["cpu_baseline"] = port
        if args.data == "grid":
            try:
                log("cpu baseline (reference program under mpirun) ...")
                result["cpu_baseline"] = cpu_baseline_reference(X, lab, Q, k, C,
                                                                labels_auto.cpu().numpy())
                result["cpu_baseline_port"] = port
            except (OSError, RuntimeError, ValueError, subprocess.SubprocessError) as e:
                log("reference baseline unavailable (%s); reporting the oracle port" % e)
        cb = result["cpu_baseline"]
        if "cfg3_strong" in result and cb:
            # configs[2] has configs[1]'s train set and k: the CPU's per-query
            # cost is the same, so its rate carries over (1M queries would take
            # hours on the CPU; the extrapolation is linear in the query count)
            M = args.cfg3_queries
            result["cfg3_strong"]["cpu_baseline"] = {
                "value": cb["value"], "unit": "queries/s", "cores": cb["cores"],
                "kind": cb["kind"],
                "sample": "the cfg2 measurement of this line (%s; same 1M x 128 train set and "
                          "k = 10, so the same per-query cost); %d queries extrapolated "
                          "linearly: %.0f s on %d cores"
                          % (cb["sample"][:80], M, M / cb["value"], cb["cores"]),
                "extrapolated_seconds": M / cb["value"],
                "labels_match_gpu": cb["labels_match_gpu"]}
    if rank == 0:
        print(json.dumps(result), flush=True)
        dropin_marker_cleanup()
    if world > 1:
        dist.destroy_process_group()


def _dropin_marker():
    return os.path.join(os.environ.get("TMPDIR", "/tmp"), "knn_bench_dropin_%s_%s.json" % (
        os.environ.get("MASTER_PORT", "0"), os.environ.get("TORCHELASTIC_RUN_ID", "none")))


def dropin_phase(world, rank, mnist=True):
    """Rank 0 runs the drop-in legs (and the MNIST-shape leg); the other ranks
    wait for its marker file (one node; nothing here has touched a GPU, so no
    rank's HIP runtime is up while the child drives every GPU of the node)."""
    marker = _dropin_marker()
    if rank == 0:
        log("drop-in legs (bin/knn_mpi_amd, 1 and %d GPU(s)) ..." % world)
        try:
            res = dropin_legs(world)
        except (OSError, RuntimeError, KeyError, ValueError, subprocess.SubprocessError) as e:
            res = {"error": "drop-in legs failed: %s" % e}
        if mnist:
            log("MNIST-shape leg (the reference's published workload) ...")
            try:
                res["mnist_shape"] = mnist_leg(world)
            except (OSError, RuntimeError, KeyError, ValueError, AssertionError,
                    subprocess.SubprocessError) as e:
                res["mnist_shape"] = {"error": "MNIST-shape leg failed: %s" % e}
        log("drop-in legs done: %s" % {k: (v.get("labels_match"), v.get("running_time_s"))
                                       for k, v in res.items() if isinstance(v, dict)})
        if world > 1:
            with open(marker + ".tmp", "w") as f:
                json.dump({"done": True}, f)
            os.replace(marker + ".tmp", marker)
        return res
    t0 = time.time()
    while not os.path.exists(marker) and time.time() - t0 < 1800:
        time.sleep(0.2)
    return None


def dropin_marker_cleanup():
    try:
        os.remove(_dropin_marker())
    except OSError:
        pass


def dry_run(args, kd, world, rank):
    """Launcher + decomposition on CPU (gloo) with the torch stand-in: the
    line carries n_gpus and a checksum of the gathered labels, value null."""
    if world > 1:
        phase("dry run: init_process_group (gloo) over %d ranks" % world)
        dist.init_process_group("gloo")
    phase("dry run: synthetic data")
    n, m, d, k, C = args.n_train, args.queries, args.dim, args.k, args.classes
    cpu = torch.device("cpu")
    X, lab, Q, _ = synth(n, m * world, d, C, 1234, 5678, cpu, data=args.data)
    kd.broadcast_train(X, lab)
    q0, q1 = kd.shard_range(m * world, world, rank)
    clf = CpuStandIn()
    clf.set_train(X, lab, C)
    out = {}

    def step():
        out["lab"] = clf.classify(Q[q0:q1], k)

    el = kd.timed(step, args.steps, args.warmup, lambda: None, None)
    labels = kd.gather_slices(out["lab"], m * world)
    # the train-sharded decomposition: rank r's rows only, one all-gather of
    # the packed lists, merge + vote of the rank's query slice
    r0, r1 = kd.shard_range(n, world, rank)
    part = CpuStandIn()
    part.set_train(X[r0:r1], lab[r0:r1], C)
    w = k + 1
    Qa = Q[:m]
    mine, (a, b) = kd.train_sharded(lambda Qt: part.search_partial(Qt, w, r0),
                                    lambda gd, gi, gl, parts, a, b: part.merge_vote(gd, gi, gl, k, a, b),
                                    Qa, m, w, k)
    ts_labels = kd.gather_slices(mine, m)
    ts_ok = bool(torch.equal(ts_labels, labels[:m]))
    # the N-GPU line's per-rank fields, through the same code as the GPU run
    pr = per_rank_report(None, {"kernel_ms": el / args.steps * 1e3, "rescanned_queries": 0,
                                "tie_vote_queries": 0, "tie_reordered_queries": 0}, out["lab"])
    ts_pr = per_rank_report(None, {"kernel_ms": 0.0, "rescanned_queries": 0,
                                   "tie_resolved_queries": 0, "tie_pending_queries": 0})
    dropin = dropin_legs(world, shape=dict(n=3000, m=64, d=24, k=k, classes=min(C, 10)),
                         dry=True) if rank == 0 else None
    if rank == 0:
        print(json.dumps({
            "group_query": dropin["group_query"], "group_train": dropin["group_train"],
            "dropin_inputs": dropin["inputs_written"],
            "train_sharded": {"value": None, "labels_match": ts_ok, "n_gpus": world,
                              "per_rank": ts_pr, "labels_sha1": labels_sha1(ts_labels),
                              "workload": "dry-run: %d train rows over %d rank(s) x %d queries"
                                          % (n, world, m)},
            "per_rank": pr, "labels_sha1_rank0": pr["labels_sha1"][0],
            "metric": METRIC, "value": None, "unit": "queries/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (%s)" % args.data, "dry_run": True,
            "note": "CPU plumbing check (torch stand-in, gloo); not a measurement",
            "config": {"workload": "dry-run: %d train x %d queries per rank, d=%d, k=%d"
                                   % (n, m, d, k), "parallelism": "query-sharded dp%d" % world},
            "labels_sha1": hashlib.sha1(labels.numpy().astype(np.int32).tobytes()).hexdigest(),
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
