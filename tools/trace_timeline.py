"""Per-position timeline of a repeated kernel sequence (one latency-plan graph replay) from a
rocprofv3 kernel trace: for each kernel of the sequence, the median duration and the median gap
from the previous dispatch's end to its start, over the last `--reps` replays.

  python tools/trace_timeline.py <kernel_trace.csv> --len 12 [--reps 100]

The sequence is taken as the last `--len` dispatches of the trace (the run must end with the
replays, e.g. tools/lat_ab.py with one arm)."""
import csv
import re
import statistics
import sys


def main():
    path = sys.argv[1]
    L = int(sys.argv[sys.argv.index("--len") + 1])
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 100
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if "at::native" in r["Kernel_Name"] or "__amd_rocclr" in r["Kernel_Name"]:
                continue  # torch / runtime kernels around the replays
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         re.sub(r"\(.*$", "", r["Kernel_Name"]).replace("dnnhip::", "")[:70],
                         r.get("Grid_Size", r.get("Grid_Size_X", ""))))
    rows.sort()
    seq = [(n, g) for _, _, n, g in rows[-L:]]
    # walk back over whole replays that match the sequence
    reps_found = []
    i = len(rows) - L
    while i >= 0 and len(reps_found) < reps:
        if [(n, g) for _, _, n, g in rows[i:i + L]] == seq:
            reps_found.append(i)
            i -= L
        else:
            i -= 1
    print("replays matched: %d" % len(reps_found))
    tot = []
    print("%3s %9s %9s  %-8s %s" % ("pos", "dur_us", "gap_us", "grid", "kernel"))
    sd, sg = 0.0, 0.0
    for p in range(L):
        d = [(rows[i + p][1] - rows[i + p][0]) / 1e3 for i in reps_found]
        g = [(rows[i + p][0] - rows[i + p - 1][1]) / 1e3 for i in reps_found if i + p - 1 >= 0 and p > 0]
        md, mg = statistics.median(d), (statistics.median(g) if g else 0.0)
        sd += md
        sg += mg
        print("%3d %9.2f %9.2f  %-8s %s" % (p, md, mg, seq[p][1], seq[p][0]))
    for i in reps_found:
        tot.append((rows[i + L - 1][1] - rows[i][0]) / 1e3)
    print("sum of durations %.2f us, sum of gaps %.2f us, first start to last end median %.2f us" %
          (sd, sg, statistics.median(tot)))


if __name__ == "__main__":
    main()
