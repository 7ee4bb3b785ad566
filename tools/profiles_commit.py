#!/usr/bin/env python3
"""Turn the rocprofv3 outputs of tools/profile_all.sh (gpurun_out/prof_<tag>/)
into the committed evidence under profiles/:

  <tag>_kernel_stats_<cfg>.csv  rocprofv3 --stats rows of the knnk:: kernels
  <tag>_kernels_<cfg>.json      per knnk:: kernel: dispatches, mean duration over
                                all dispatches and over the timed ones (the
                                bench's last `steps` launches of the candidate
                                kernel), the profiled run's own bench line, and
                                the roofline fraction recomputed from the profile
  <tag>_traffic_<cfg>.json      HBM bytes per launch (tools/traffic_json.py:
                                2*FETCH_SIZE + WRITE_SIZE, separate passes) and
                                the kernel_src_sha of the profiled build
  <tag>_hip_api_cfg2.json       the HIP API calls made between the first and the
                                last candidate-kernel launch of the timed loop
                                (knn_classify_device is enqueue-only: no stream
                                or event synchronisation in there)
Usage: python tools/profiles_commit.py [--tag r2]"""
import argparse
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import traffic_json  # noqa: E402

# bench arguments of each profiled workload (tools/profile_all.sh)
WORKLOADS = {
    "cfg2": dict(steps=10, warmup=2, n_train=1_000_000, queries=10_000, dim=128, k=10),
    "cfg4": dict(steps=3, warmup=1, n_train=100_000_000, queries=10_000, dim=96, k=10),
    "cfg5": dict(steps=4, warmup=1, n_train=1_000_000, queries=10_000, dim=960, k=100),
    # cfg5 on the query-resident fp16 kernel (tuning "qres" 1)
    "cfg5q": dict(steps=4, warmup=1, n_train=1_000_000, queries=10_000, dim=960, k=100,
                  tuning="qres=1"),
    "cfg4s": dict(steps=5, warmup=1, n_train=12_500_000, queries=10_000, dim=96, k=10),
    "cfg2c": dict(steps=10, warmup=2, n_train=1_000_000, queries=10_000, dim=128, k=10,
                  data="continuous"),
    "cfg2f32": dict(steps=4, warmup=1, n_train=1_000_000, queries=10_000, dim=128, k=10,
                    precision="fp32"),
}


def short(name):
    return name.split("(")[0].replace("void ", "").replace("knnk::", "").replace(" ", "")


def bench_line(log):
    for line in open(log):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    return None


def kernels(trace):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(trace)):
        if "knnk::" in r["Kernel_Name"]:
            per[short(r["Kernel_Name"])].append(
                (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Correlation_Id"])))
    return per


def timed_slice(launches, steps):
    """The candidate launches of bench.timed_run's K timed calls: they are
    followed by min(K, 5) untimed calls that record every phase's events."""
    tail = min(steps, 5)
    return launches[-(steps + tail):-tail]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r2")
    a = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", "prof_" + a.tag)
    dst = os.path.join(ROOT, "profiles")
    # the profiled build must be this tree's (tools/profile_all.sh records it)
    rec = os.path.join(src, "src_sha.txt")
    if not os.path.exists(rec) or open(rec).read().strip() != bench.kernel_src_sha():
        sys.exit("profiles_commit: %s was not profiled from this tree's sources (%s); re-run "
                 "tools/profile_all.sh" % (src, bench.kernel_src_sha()))
    for cfg, wl in WORKLOADS.items():
        sdir = os.path.join(src, "stats_" + cfg)
        if not os.path.isdir(sdir):
            continue
        rows = [r for r in csv.reader(open(os.path.join(sdir, "run_kernel_stats.csv")))]
        with open(os.path.join(dst, "%s_kernel_stats_%s.csv" % (a.tag, cfg)), "w", newline="") as f:
            w = csv.writer(f, quoting=csv.QUOTE_ALL)
            w.writerow(rows[0])
            for r in rows[1:]:
                if "knnk::" in r[0]:
                    w.writerow(r)
        line = bench_line(os.path.join(src, "stats_%s.log" % cfg))
        per = kernels(os.path.join(sdir, "run_kernel_trace.csv"))
        cand = line["roofline"]["kernel"] if line else None
        out = {"workload": wl, "bench_line": line, "kernels": {}}
        for k, v in sorted(per.items()):
            d = [e - s for s, e, _ in v]
            rec = {"dispatches": len(d), "mean_ns_all": sum(d) / len(d), "min_ns": min(d)}
            if k == cand:
                timed = timed_slice(d, wl["steps"])
                rec["mean_ns_timed"] = sum(timed) / len(timed)
                flops = line["roofline"]["algorithmic_flops_per_launch"]
                ach = flops / (rec["mean_ns_timed"] * 1e-9) / 1e12
                rec["achieved_tflops_profile"] = ach
                rec["frac_profile"] = ach / line["roofline"]["peak"]
                rec["frac_bench_line"] = line["roofline"]["frac"]
            out["kernels"][k] = rec
        json.dump(out, open(os.path.join(dst, "%s_kernels_%s.json" % (a.tag, cfg)), "w"),
                  indent=1)
        fdir, wdir = os.path.join(src, "fetch_" + cfg), os.path.join(src, "write_" + cfg)
        if os.path.isdir(fdir) and os.path.isdir(wdir):
            fetch = traffic_json.per_launch(fdir, "FETCH_SIZE")
            write = traffic_json.per_launch(wdir, "WRITE_SIZE")
            tr = {"workload": {key: wl[key] for key in ("n_train", "queries", "dim", "k", "data", "tuning")
                               if key in wl},
                  "kernel_src_sha": bench.kernel_src_sha(),
                  "formula": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE half-count "
                             "correction; KiB units)", "kernels": {}}
            for k in sorted(set(fetch) | set(write)):
                fv, nf = fetch.get(k, (0.0, 0))
                wv, nw = write.get(k, (0.0, 0))
                tr["kernels"][k] = {"fetch_kib": fv, "write_kib": wv, "dispatches": [nf, nw],
                                    "hbm_bytes_per_launch": 2 * fv * 1024 + wv * 1024}
            json.dump(tr, open(os.path.join(dst, "%s_traffic_%s.json" % (a.tag, cfg)), "w"),
                      indent=1)
    adir = os.path.join(src, "api_cfg2")
    if os.path.isdir(adir):
        per = kernels(os.path.join(adir, "run_kernel_trace.csv"))
        line = bench_line(os.path.join(src, "api_cfg2.log"))
        cand = line["roofline"]["kernel"]
        launches = sorted(per[cand], key=lambda x: x[0])
        timed = timed_slice(launches, WORKLOADS["cfg2"]["steps"])
        corr = {c for _, _, c in timed}
        api = list(csv.DictReader(open(os.path.join(adir, "run_hip_api_trace.csv"))))
        by_corr = {int(r["Correlation_Id"]): r for r in api}
        t0 = int(by_corr[min(corr)]["Start_Timestamp"])
        t1 = int(by_corr[max(corr)]["End_Timestamp"])
        calls = collections.Counter(r["Function"] for r in api
                                    if t0 <= int(r["Start_Timestamp"]) <= t1)
        syncs = {f: n for f, n in calls.items() if re.search(r"Synchronize|Query", f)}
        json.dump({"what": "HIP API calls between the launch of the first and of the last "
                           "candidate kernel of the timed loop (%d knn_classify_device calls)"
                           % len(timed),
                   "kernel": cand, "calls": dict(calls.most_common()),
                   "synchronising_calls": syncs,
                   "window_us": (t1 - t0) / 1e3}, open(
                       os.path.join(dst, "%s_hip_api_cfg2.json" % a.tag), "w"), indent=1)


if __name__ == "__main__":
    main()
