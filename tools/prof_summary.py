"""Summarise a rocprofv3 run of bench.py into profiles/ (committed evidence).

    python tools/prof_summary.py gpurun_out/r01 r01 [--kernel ws_piece_unmask_kernel,ws_piece_walk_kernel]

The first --kernel name is the dominant kernel; traffic per step sums every listed kernel.

Inputs (written by tools/profile.sh on the GPU box):
  <dir>/trace/run_kernel_stats.csv       rocprofv3 --kernel-trace --stats
  <dir>/pmc_fetch/run_counter_collection.csv   rocprofv3 --pmc FETCH_SIZE
  <dir>/pmc_write/run_counter_collection.csv   rocprofv3 --pmc WRITE_SIZE
  <dir>/bench.json                        the bench line of the same code
Outputs: profiles/<tag>_kernel_stats.csv (copy), profiles/<tag>_pmc.json,
profiles/<tag>_bench.json (the traced run's own line), profiles/<tag>_bench_full.json (an
untraced run with the CPU baseline and end-to-end fields).

HBM traffic per launch (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are
in KiB; on gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced
streaming read, so traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import csv
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path, kernel, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def main():
    src, tag = sys.argv[1], sys.argv[2]
    names = (sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv
             else "ws_piece_unmask_kernel,ws_piece_walk_kernel").split(",")
    kernel = names[0]
    out = os.path.join(REPO, "profiles")
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(out, tag + "_kernel_stats.csv"))
    rows = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    stats = [r for r in rows if kernel in r["Name"]]
    per_kernel = {}
    fetch_kib = write_kib = 0.0
    nf = nw = 0
    for k in names:
        st = [r for r in rows if k in r["Name"]]
        if not st and k != kernel:                      # a listed kernel that did not run here
            continue
        f, a = per_launch(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), k, "FETCH_SIZE")
        w, b = per_launch(os.path.join(src, "pmc_write", "run_counter_collection.csv"), k, "WRITE_SIZE")
        per_kernel[k] = {"avg_ns": float(st[0]["AverageNs"]) if st else None, "calls": int(st[0]["Calls"]) if st else 0,
                         "fetch_kib": f, "write_kib": w}
        if f is None or w is None:
            fetch_kib = write_kib = None
        elif fetch_kib is not None:
            fetch_kib += f
            write_kib += w
        if k == kernel:
            nf, nw = a, b
    bench = json.load(open(os.path.join(src, "bench.json")))
    rf = bench["roofline"]
    algo = rf.get("algo_bytes_per_launch") or rf.get("algo_bytes_per_step")
    rec = {
        "kernel": stats[0]["Name"] if stats else kernel,
        "rocprof_calls": int(stats[0]["Calls"]) if stats else 0,
        "rocprof_avg_ns": float(stats[0]["AverageNs"]) if stats else None,
        "rocprof_min_ns": float(stats[0]["MinNs"]) if stats else None,
        "bench_kernel_ms_mean": rf.get("kernel_ms_mean"),
        "bench_ms_per_step": bench.get("ms_per_step"),
        "kernels_summed": names,
        "per_kernel": per_kernel,
        "per_kernel_avg_ns": {k: v["avg_ns"] for k, v in per_kernel.items()},
        "fetch_size_kib_per_launch": fetch_kib, "fetch_dispatches": nf,
        "write_size_kib_per_launch": write_kib, "write_dispatches": nw,
        "fetch_bytes_corrected": 2 * fetch_kib * 1024 if fetch_kib is not None else None,
        "write_bytes": write_kib * 1024 if write_kib is not None else None,
        "algo_bytes_per_launch": algo,
        "bench_metric": bench.get("metric"),
        "correction": "FETCH_SIZE x2 (gfx950 reports half of wide streaming reads), KiB -> bytes",
    }
    if fetch_kib is not None and write_kib is not None:
        rec["traffic_bytes_per_launch"] = (2 * fetch_kib + write_kib) * 1024
        rec["traffic_over_algo"] = rec["traffic_bytes_per_launch"] / algo
    if "traffic_bytes_per_launch" in rec:
        # the bench line ran before this profile's counter passes: its traffic field is filled
        # from them (the same code and workload)
        rf["traffic"] = int(rec["traffic_bytes_per_launch"])
        rf["traffic_source"] = "profiles/%s_pmc.json" % tag
        rf["traffic_kernels"] = names
        if "per_kernel_ns_profiled" in rf:
            rf["per_kernel_ns_profiled"] = rec["per_kernel_avg_ns"]
    # consistency: the step's kernels (each launched once per step) against the bench line of
    # the same traced process — a kernel cannot take longer than the step that contains it
    ks = [v["avg_ns"] for v in per_kernel.values() if v["avg_ns"] is not None]
    rec["rocprof_kernel_sum_ms"] = round(sum(ks) / 1e6, 4) if ks else None
    rec["same_run_ms_per_step"] = bench.get("ms_per_step")
    if ks and bench.get("ms_per_step"):
        rec["kernel_sum_le_step"] = sum(ks) / 1e6 <= bench["ms_per_step"]
        rec["kernel_sum_frac_of_step"] = round(sum(ks) / 1e6 / bench["ms_per_step"], 4)
    rec["bench_source"] = "the JSON line printed by the rocprofv3 --kernel-trace run itself (tools/profile.sh)"
    json.dump(rec, open(os.path.join(out, tag + "_pmc.json"), "w"), indent=1)
    full = os.path.join(src, "bench_full.json")
    if os.path.exists(full) and os.path.getsize(full):
        shutil.copy(full, os.path.join(out, tag + "_bench_full.json"))
    json.dump(bench, open(os.path.join(out, tag + "_bench.json"), "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
