"""YOLOv2-tiny model front-end on the MI355X engine — the reference's
`cs492-projects/proj3/yolov2tiny.py` interface for this path:

    y2t = YOLO_V2_TINY([1, 416, 416, 3], "y2t_weights.pickle", debug)   # yolov2tiny.py:7-13
    out = y2t.inference(frame)                                           # :80-82
    boxes = postprocessing(np.squeeze(out))                              # :94-176

The graph is the reference's node chain (yolo_graph.build_graph = yolov2tiny.py:25-79) on
dnn_hip's DnnGraphBuilder / DnnInferenceEngine; the weights come from the pickle through the
safe loader (yolo_weights.py; the reference's own get_y2t_w raises on Python 3.10), or a
list of layer dicts in the same format may be passed directly.  `postprocessing` runs on the
GPU (yolo_post.py).
"""
import dnn_hip
import yolo_graph
import yolo_post
import yolo_weights

postprocessing = yolo_post.postprocessing


class YOLO_V2_TINY(object):
    """yolov2tiny.py:7-82 with the MI355X engine underneath."""

    def __init__(self, in_shape, weight_pickle, debug, device=None):
        self.weight_pickle = weight_pickle
        self.g = dnn_hip.DnnGraphBuilder()
        self.build_graph(in_shape)
        self.sess = dnn_hip.DnnInferenceEngine(self.g, debug, device=device)

    def get_y2t_w(self):
        if isinstance(self.weight_pickle, (list, tuple)):
            return yolo_weights.validate(self.weight_pickle)
        return yolo_weights.load_y2t_weights(self.weight_pickle)

    def build_graph(self, in_shape):
        y2t_w = self.get_y2t_w()
        self.g, self.nodes = yolo_graph.build_graph(lambda: self.g, y2t_w, in_shape=tuple(in_shape))

    def inference(self, im):
        return self.sess.run(im)
