"""Summarise rocprofv3 CSV output of `bench.py` per PLAN kernel (conv0.im2col ... conv8.gemm).

rocprofv3 --stats aggregates by kernel template, and one template serves several layers, so
this maps every dispatch to its plan kernel by position inside each forward (a forward
starts at the conv0 im2col dispatch and has a fixed kernel order).

  python tools/prof_summary.py --trace DIR/trace_kernel_trace.csv \
      [--fetch DIR/fetch_counter_collection.csv --write DIR/write_counter_collection.csv] \
      [--out profiles/pmc_summary.json]

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reads exactly
half the bytes of a wide (16 B/lane) coalesced streaming read on gfx950, so it is doubled;
WRITE_SIZE is exact for 16 B/lane stores.  bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import argparse
import csv
import json
from collections import defaultdict

# kernel order of one YOLOv2-tiny forward in the default (fused) plan: conv5-7's split-K
# partials are combined inside their GEMMs (DNN_HIP_SPLITK_FUSED=0 / --reduce: a separate
# convN.reduce kernel after each)
ORDER = ["conv0.direct", "conv1.gemm", "conv2.gemm", "conv3.gemm", "conv4.gemm", "conv5.gemm", "pool5",
         "conv6.gemm", "conv7.gemm", "conv8.gemm"]
# (round 5: pool5 fused into conv5's whole-image x3 kernel -- the same list without "pool5";
# dispatch_sequence picks the variant whose length matches the trace's forward period)
# (the same kernel list with DNN_HIP_X3=0: conv5-7 split-K combined in the GEMM)
# ... the fp16 plan (dnn_plan_set_precision 1): conv1 patch kernel, f16->f32 output conversion
ORDER_FP16 = ["conv0.direct", "conv1.patch", "conv2.gemm", "conv3.gemm", "conv4.gemm", "conv5.gemm", "pool5",
              "conv6.gemm", "conv7.gemm", "conv8.gemm", "output.cvt"]
# ... and with DNN_HIP_FUSE=0 (explicit im2col + GEMM, separate pools)
ORDER_UNFUSED = []
for _i in range(9):
    if _i < 8:
        ORDER_UNFUSED.append(f"conv{_i}.im2col")
    ORDER_UNFUSED.append(f"conv{_i}.gemm")
    if _i < 6:
        ORDER_UNFUSED.append(f"pool{_i}")

def with_reduces(order):
    """the same plan with a separate split-K reduce kernel after conv5/6/7's GEMM"""
    out = []
    for n in order:
        out.append(n)
        if n in ("conv5.gemm", "conv6.gemm", "conv7.gemm"):
            out.append(n.replace(".gemm", ".reduce"))
    return out


# every kernel of the plan lives in namespace dnnhip; weight packing (finalize) and the
# postprocessing kernels (after the forward) are not plan kernels
_NOT_PLAN = ("pack_weights", "yolo_", "f32_to_f16_kernel", "preprocess_kernel", "clock_stamp")


def _ours(name):
    # rocprofv3 leaves names with _Float16 parameters mangled (..6dnnhip..)
    return ("dnnhip::" in name or "6dnnhip" in name) and not any(t in name for t in _NOT_PLAN)


def dispatch_sequence(rows, key_start="Start_Timestamp", key_end="End_Timestamp"):
    """[(plan_kernel, row)] for every dispatch inside a recognised forward."""
    seq = [r for r in rows if _ours(r["Kernel_Name"])]
    seq.sort(key=lambda r: int(r.get("Dispatch_Id") or 0))
    out, i = [], 0
    first = None
    order = ORDER
    while i < len(seq):
        name = seq[i]["Kernel_Name"]
        if first is None:
            first = name  # the first dispatch of the first forward defines the start marker
            starts = [j for j in range(i, len(seq)) if seq[j]["Kernel_Name"] == first]
            if len(starts) > 1 and starts[1] - starts[0] == len(order) - 1 and "pool5" in order:
                order = [k for k in order if k != "pool5"]  # pool5 fused into conv5 (x3_img)
            elif len(starts) > 1 and starts[1] - starts[0] == len(order) - 2 and "output.cvt" in order:
                # fp16, round 5: pool5 fused into conv5, conv8 writes the fp32 output itself
                order = [k for k in order if k not in ("pool5", "output.cvt")]
        if name == first and i + len(order) <= len(seq):
            for j, pk in enumerate(order):
                out.append((pk, seq[i + j]))
            i += len(order)
        else:
            i += 1
    return out


def summarise(trace=None, fetch=None, write=None, skip=0):
    """skip: leading (warm-up) dispatches per plan kernel left out of avg_us / median_us
    (bench.py's roofline averages only its timed steps); avg_all_us keeps every call."""
    res = defaultdict(lambda: {"calls": 0})
    if trace:
        rows = list(csv.DictReader(open(trace)))
        for pk, r in dispatch_sequence(rows):
            d = res[pk]
            d["calls"] += 1
            d.setdefault("_ns", []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            d["template"] = r["Kernel_Name"].split("(")[0]
            d["grid"] = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
            d["vgpr"] = int(r.get("VGPR_Count") or 0)
            d["agpr"] = int(r.get("Accum_VGPR_Count") or 0)
            d["lds"] = int(r.get("LDS_Block_Size") or 0)
    for path, key in ((fetch, "FETCH_SIZE"), (write, "WRITE_SIZE")):
        if not path:
            continue
        rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == key]
        for pk, r in dispatch_sequence(rows):
            res[pk].setdefault("_" + key, []).append(float(r["Counter_Value"]))
    out = {}
    for pk in ORDER:
        if pk not in res:
            continue
        d = dict(res[pk])
        if "_ns" in d:
            allns = d.pop("_ns")
            ns = sorted(allns[skip:] if len(allns) > skip else allns)
            d["avg_us"] = round(sum(ns) / len(ns) / 1e3, 2)
            d["median_us"] = round(ns[len(ns) // 2] / 1e3, 2)
            d["avg_all_us"] = round(sum(allns) / len(allns) / 1e3, 2)
            d["timed_calls"] = len(ns)
        for key in ("FETCH_SIZE", "WRITE_SIZE"):
            v = d.pop("_" + key, None)
            if v:
                d[key.lower() + "_kib"] = round(sum(v) / len(v), 1)
        if "fetch_size_kib" in d and "write_size_kib" in d:
            d["hbm_bytes_per_launch"] = round((2 * d["fetch_size_kib"] + d["write_size_kib"]) * 1024)
        out[pk] = d
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--out")
    ap.add_argument("--note", default="")
    ap.add_argument("--skip", type=int, default=0, help="warm-up dispatches per kernel to leave out of avg_us")
    ap.add_argument("--unfused", action="store_true", help="trace of a DNN_HIP_FUSE=0 run")
    ap.add_argument("--fp16", action="store_true", help="trace of a --precision fp16 run")
    ap.add_argument("--reduce", action="store_true", help="trace of a DNN_HIP_SPLITK_FUSED=0 run (fp32)")
    a = ap.parse_args()
    if a.unfused:
        ORDER[:] = ORDER_UNFUSED
    if a.reduce:
        ORDER[:] = with_reduces(ORDER)
    if a.fp16:
        ORDER[:] = with_reduces(ORDER_FP16) if a.reduce else ORDER_FP16
    s = summarise(a.trace, a.fetch, a.write, a.skip)
    doc = {"note": a.note or __doc__.strip().splitlines()[0], "kernels": s}
    text = json.dumps(doc, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")
    for k, d in s.items():
        print(f"{k:14s} calls={d.get('calls', 0):4d} avg_us={d.get('avg_us', 0):9.2f} "
              f"fetch={d.get('fetch_size_kib', 0):12.1f}KiB write={d.get('write_size_kib', 0):12.1f}KiB "
              f"{d.get('template', '')[:60]}")


if __name__ == "__main__":
    main()
