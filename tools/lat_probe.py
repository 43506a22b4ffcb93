"""Batch-1 latency probe (BASELINE config 2): one JSON line with the latency plan's graph
replay time, its per-kernel event times and the plan description.  Environment switches of
choose_latency_plan (DNN_HIP_LAT_UNITS / _MINSTEPS / _CAND, DNN_HIP_SPLIT) apply."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dnn-inference-engine_amd")]


def main():
    import torch
    import bench
    import dnn_hip
    import synth
    import yolo_graph
    dev = torch.device("cuda", 0)
    ws = synth.yolo_weights()
    lat = os.environ.get("LAT", "1") == "1"
    r = bench.latency_b1(dnn_hip, yolo_graph, ws, dev, iters=int(os.environ.get("ITERS", "200")), latency=lat)
    r.pop("_x", None)
    r.pop("_y", None)
    g, _ = yolo_graph.build_graph(dnn_hip.DnnGraphBuilder, synth.yolo_zero_weights(), in_shape=(1, 416, 416, 3))
    r["env"] = {k: v for k, v in os.environ.items() if k.startswith("DNN_HIP_")}
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
