"""Summarise a rocprofv3 run of bench.py into profiles/ (committed evidence).

    python tools/prof_summary.py gpurun_out/r01 r01 [--kernel ws_piece_unmask_kernel,ws_piece_walk_kernel]
                                 [--launches-per-step N]

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
streaming read (the guide's ×2), so a STREAMING kernel's traffic = (2 * FETCH_SIZE +
WRITE_SIZE) * 1024. The ×2 applies to that access pattern only: the walk kernels (K1's
16-lane scattered 32-B header reads, the raw stream's candidate / owner / emit walks, the
encode front's random edge windows) fetch about one 64-B line per request and are
reported raw, FETCH_SIZE * 1024 (cfg2 K1: 76.7 MB raw ≈ one 64-B line per 4 KiB frame).
"""

# kernels whose reads are wide coalesced streams (16 B per lane over whole pieces / segments):
# the only ones FETCH_SIZE is doubled for
STREAMING = ("ws_piece_unmask_kernel", "ws_enc_copy_kernel", "ws_segfuse_kernel", "ws_reasm_seg_kernel",
             "ws_reasm_gather_kernel", "ws_walker_kernel")


def fetch_factor(kernel):
    return 2.0 if any(kernel.startswith(k) or k in kernel for k in STREAMING) else 1.0
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


def region_kernel_ms(src, names, kernel, warmup, steps, lps=1):
    """every listed kernel's dispatch time inside the bench's timed region, per step: from the end
    of the dominant kernel's last warm-up dispatch to the end of its last timed one (lps: its
    launches per step — the raw stream's split unmask launches twice)"""
    path = os.path.join(src, "trace", "run_kernel_trace.csv")
    if not os.path.exists(path) or steps <= 0:
        return None
    rows = list(csv.DictReader(open(path)))
    dom = sorted((r for r in rows if kernel in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
    if len(dom) < (warmup + steps) * lps:
        return None
    t0 = int(dom[warmup * lps - 1]["End_Timestamp"]) if warmup else 0
    t1 = int(dom[(warmup + steps) * lps - 1]["End_Timestamp"])
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                if any(n in r["Kernel_Name"] for n in names) and t0 <= int(r["Start_Timestamp"]) < t1)
    # the union of the dispatch intervals (kernels on a side stream overlap the call's own: the
    # device is busy once for both)
    busy, cur_s, cur_e = 0, None, None
    for a, b in iv:
        if cur_e is None or a > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    if cur_e is not None:
        busy += cur_e - cur_s
    return busy / steps / 1e6


def main():
    src, tag = sys.argv[1], sys.argv[2]
    names = (sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv
             else "ws_piece_unmask_kernel,ws_piece_walk_kernel").split(",")
    kernel = names[0]
    # launches of the dominant kernel per step (the raw stream's split unmask: 2)
    lps = int(sys.argv[sys.argv.index("--launches-per-step") + 1]) if "--launches-per-step" in sys.argv else 1
    out = os.path.join(REPO, "profiles")
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(out, tag + "_kernel_stats.csv"))
    rows = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    stats = [r for r in rows if kernel in r["Name"]]
    per_kernel = {}
    fetch_kib = write_kib = fetch_corr = 0.0
    nf = nw = 0
    for k in names:
        st = [r for r in rows if k in r["Name"]]
        if not st and k != kernel:                      # a listed kernel that did not run here
            continue
        f, a = per_launch(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), k, "FETCH_SIZE")
        w, b = per_launch(os.path.join(src, "pmc_write", "run_counter_collection.csv"), k, "WRITE_SIZE")
        per_kernel[k] = {"avg_ns": float(st[0]["AverageNs"]) if st else None, "calls": int(st[0]["Calls"]) if st else 0,
                         "fetch_kib": f, "write_kib": w, "fetch_factor": fetch_factor(k)}
        m = lps if k == kernel else 1                   # per step
        if f is None or w is None:
            fetch_kib = write_kib = None
            fetch_corr = None
        elif fetch_kib is not None:
            fetch_kib += m * f
            write_kib += m * w
            fetch_corr += m * fetch_factor(k) * f
        if k == kernel:
            nf, nw = a, b
    bench = json.load(open(os.path.join(src, "bench.json")))
    rf = bench["roofline"]
    algo = rf.get("algo_bytes_per_launch") or rf.get("algo_bytes_per_step")
    rec = {
        "kernel": stats[0]["Name"] if stats else kernel,
        "launches_per_step": lps,
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
        "fetch_bytes_corrected": fetch_corr * 1024 if fetch_kib is not None else None,
        "write_bytes": write_kib * 1024 if write_kib is not None else None,
        "algo_bytes_per_launch": algo,
        "bench_metric": bench.get("metric"),
        "bench_frac": rf.get("frac"),
        "bench_hip_graph": bool(bench.get("config", {}).get("hip_graph")),
        "bench_config": bench.get("config"),
        "correction": "FETCH_SIZE x2 for the streaming kernels only (%s: gfx950 reports half of wide coalesced "
                      "streaming reads), x1 for walk kernels (scattered line requests), KiB -> bytes"
                      % ", ".join(k for k in names if fetch_factor(k) == 2.0),
    }
    if fetch_kib is not None and write_kib is not None:
        rec["traffic_bytes_per_launch"] = (fetch_corr + write_kib) * 1024
        rec["traffic_over_algo"] = rec["traffic_bytes_per_launch"] / algo
    if "traffic_bytes_per_launch" in rec:
        # the bench line ran before this profile's counter passes: its traffic field is filled
        # from them (the same code and workload)
        rf["traffic"] = int(rec["traffic_bytes_per_launch"])
        rf["traffic_source"] = "profiles/%s_pmc.json" % tag
        rf["traffic_kernels"] = names
        if "per_kernel_ns_profiled" in rf:
            rf["per_kernel_ns_profiled"] = rec["per_kernel_avg_ns"]
    # consistency: the step's kernels against the bench line of the same traced process — a
    # kernel cannot take longer than the step that contains it (dispatches that overlap, on a
    # side stream, count once: the union of their intervals). rocprof's averages cover every
    # dispatch of the process (warm-up calls too), so the check uses the dispatches inside the
    # timed region: from the end of the dominant kernel's last warm-up dispatch to the end of
    # its last timed one (kernel trace), every listed kernel's durations summed, / steps.
    ks = [v["avg_ns"] * (lps if k == kernel else 1) for k, v in per_kernel.items() if v["avg_ns"] is not None]
    rec["rocprof_kernel_sum_ms"] = round(sum(ks) / 1e6, 4) if ks else None
    step = bench.get("ms_per_step")
    rec["same_run_ms_per_step"] = step
    region = region_kernel_ms(src, names, kernel, int(bench.get("warmup") or 0), int(bench.get("steps") or 0), lps)
    rec["timed_region_kernel_ms_per_step"] = round(region, 4) if region is not None else None
    if bench.get("scaling") == "strong" and step:                  # cfg4: the step sums the rounds
        rounds = int(bench.get("config", {}).get("rounds_per_rank") or 1)
        rec["same_run_ms_per_round"] = round(step / rounds, 4)
        # the last round's timed dispatches (kernel trace) when found, else every dispatch's
        # average (warm-up dispatches included, which can sit a few us above the timed ones)
        v = region if region is not None else sum(ks) / 1e6
        rec["kernel_sum_le_step"] = v <= step / rounds
        rec["check"] = ("kernels of the last round's timed calls (kernel trace), per call, <= the round's per-call time"
                        if region is not None else "rocprof average per dispatch <= the round's per-call time")
    elif step and (region is not None or ks):
        v = region if region is not None else sum(ks) / 1e6
        rec["kernel_sum_le_step"] = v <= step
        rec["kernel_sum_frac_of_step"] = round(v / step, 4)
        rec["check"] = ("kernels inside the timed region (kernel trace, union of their intervals) <= the step"
                        if region is not None
                        else "rocprof averages <= the step")
    rec["bench_source"] = "the JSON line printed by the rocprofv3 --kernel-trace run itself (tools/profile.sh)"
    json.dump(rec, open(os.path.join(out, tag + "_pmc.json"), "w"), indent=1)
    full = os.path.join(src, "bench_full.json")
    if os.path.exists(full) and os.path.getsize(full):
        shutil.copy(full, os.path.join(out, tag + "_bench_full.json"))
    json.dump(bench, open(os.path.join(out, tag + "_bench.json"), "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
