"""Group a rocprofv3 kernel trace (CSV, one row per dispatch) by (kernel, grid size): dispatch
count and mean / median duration in us, largest total first.  Tells the latency plan's kernels
(200 single-frame graph replays per bench run) apart from the batch-64 ones that share a kernel
name but not a grid.

  python tools/trace_by_grid.py gpurun_out/<dir>/.../*_kernel_trace.csv [--min-count N]
"""
import csv
import re
import statistics
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*$", "", name)  # drop the argument list
    name = name.replace("dnnhip::", "")
    return name[:90]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    min_count = 1
    if "--min-count" in sys.argv:
        min_count = int(sys.argv[sys.argv.index("--min-count") + 1])
        args = [a for a in args if a != str(min_count)]
    groups = defaultdict(list)
    for path in args:
        with open(path) as f:
            for row in csv.DictReader(f):
                grid = tuple(row.get(k, "") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z", "Grid_Size"))
                grid = "x".join(g for g in grid if g)
                dur = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1000.0
                groups[(short(row["Kernel_Name"]), grid)].append(dur)
    rows = [(k, v) for k, v in groups.items() if len(v) >= min_count]
    rows.sort(key=lambda kv: -sum(kv[1]))
    print("%6s %9s %9s  %-14s %s" % ("count", "mean_us", "med_us", "grid", "kernel"))
    for (name, grid), v in rows:
        print("%6d %9.2f %9.2f  %-14s %s" % (len(v), statistics.mean(v), statistics.median(v), grid, name))


if __name__ == "__main__":
    main()
