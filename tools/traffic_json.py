#!/usr/bin/env python3
"""Per-launch HBM traffic of each knnk:: kernel from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE collected separately, MI355X_MICROARCH.md "HBM"):

  bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024

FETCH_SIZE/WRITE_SIZE are KiB; on gfx950 FETCH_SIZE tallies exactly half the
bytes of a 16-B-per-lane streaming read (global_load and LDS-DMA alike), so it
is doubled; WRITE_SIZE is exact for 16-B stores.  Values are summed over the
TCC instances of a dispatch and averaged over dispatches.

Usage: traffic_json.py <fetch-dir> <write-dir> <workload-json> > profiles/rN_traffic.json
  workload-json: '{"n_train":..,"queries":..,"dim":..,"k":..}' of the profiled run.
The file records kernel_src_sha (bench.kernel_src_sha() of the tree that was
profiled): bench.py cites a traffic file only for the same kernel build.
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def per_launch(d, counter):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
        if "knnk::" not in r["Kernel_Name"] or r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("knnk::", "")
        per[(name.replace(" ", ""), r["Dispatch_Id"])] += float(r["Counter_Value"])
    agg = collections.defaultdict(list)
    for (k, _), v in per.items():
        agg[k].append(v)
    return {k: (sum(v) / len(v), len(v)) for k, v in agg.items()}


def main():
    fetch = per_launch(sys.argv[1], "FETCH_SIZE")
    write = per_launch(sys.argv[2], "WRITE_SIZE")
    wl = json.loads(sys.argv[3])
    out = {"workload": wl, "kernel_src_sha": bench.kernel_src_sha(), "formula": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE "
           "half-count correction; KiB units)", "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f, nf = fetch.get(k, (0.0, 0))
        w, nw = write.get(k, (0.0, 0))
        out["kernels"][k] = {"fetch_kib": f, "write_kib": w, "dispatches": [nf, nw],
                             "hbm_bytes_per_launch": 2 * f * 1024 + w * 1024}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
