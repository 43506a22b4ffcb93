"""Write the YOLOv2-tiny output (batch argv[2], default 16; precision argv[3], default fp32) of
the default plan to argv[1] (.npy), for
variant A/B runs (one process per arm of a switch read once per process)."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "dnn-inference-engine_amd"))
import numpy as np  # noqa: E402

import dnn_hip  # noqa: E402
import synth  # noqa: E402
import yolo_graph  # noqa: E402

B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
g, _ = yolo_graph.build_graph(dnn_hip.DnnGraphBuilder, synth.yolo_weights(), in_shape=(B, 416, 416, 3))
prec = sys.argv[3] if len(sys.argv) > 3 else "fp32"
eng = dnn_hip.DnnInferenceEngine(g, False, device=0, precision=prec)
np.save(sys.argv[1], eng.run(synth.frames(list(range(B)))))
