"""Print one call's kernel timeline from a rocprofv3 --kernel-trace CSV (CPU side).

    python tools/trace_timeline.py <run_kernel_trace.csv> <first-kernel-substring> [call_index]

A call starts at each dispatch of the first kernel (e.g. ws_rw_plan_kernel); prints every kernel
that starts before the next call: start offset, duration (us), the queue/stream id."""
import csv
import sys


def main():
    path, first = sys.argv[1], sys.argv[2]
    idx = int(sys.argv[3]) if len(sys.argv) > 3 else -2
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    a = starts[idx]
    b = starts[idx + 1] if idx + 1 < len(starts) and idx != -1 else len(rows)
    t0 = int(rows[a]["Start_Timestamp"])
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
        q = r.get("Stream_Id") or r.get("Queue_Id") or ""
        print("%9.1f %9.1f %8.1f  q%-3s %s" % (s / 1e3, e / 1e3, (e - s) / 1e3, q, name))


if __name__ == "__main__":
    main()
