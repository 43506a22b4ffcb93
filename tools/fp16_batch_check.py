"""fp16 YOLOv2-tiny: batch-64 rows vs batch-1 runs and batch-64 run-to-run, per DNN_HIP_* arm
(debugging aid: prints max |diff| per checked frame)."""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "dnn-inference-engine_amd"))
import dnn_hip  # noqa: E402
import synth  # noqa: E402
import yolo_graph  # noqa: E402

ws = synth.yolo_weights()
g1, _ = yolo_graph.build_graph(dnn_hip.DnnGraphBuilder, ws, in_shape=(1, 416, 416, 3))
e1 = dnn_hip.DnnInferenceEngine(g1, False, precision="fp16")
x = synth.frames([0, 1, 2, 3] + [100 + i for i in range(60)])
g64, _ = yolo_graph.build_graph(dnn_hip.DnnGraphBuilder, ws, in_shape=(64, 416, 416, 3))
e64 = dnn_hip.DnnInferenceEngine(g64, False, precision="fp16")
print(e64.plan().describe())
y64 = e64.run(x)
y64b = e64.run(x)
print("batch-64 run-to-run max diff", float(np.abs(y64 - y64b).max()))
for pos in (0, 3, 17, 63):
    y1 = e1.run(x[pos:pos + 1])
    d = np.abs(y64[pos:pos + 1] - y1)
    print("frame", pos, "max diff", float(d.max()), "count", int((d > 0).sum()))
