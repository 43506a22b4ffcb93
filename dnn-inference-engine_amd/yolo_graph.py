"""YOLOv2-tiny node chain: the caller side of the path (SURVEY.md §8b "caller contract").

`build_graph` mirrors `YOLO_V2_TINY.build_graph` (proj3/yolov2tiny.py:25-79): 9 Conv2D
(3x3 stride 1 SAME, the last 1x1), 9 BiasAdd, 8 BatchNorm (eps 1e-5), 8 LeakyReLU and 6
MaxPool2D (five 2x2/s2 SAME, then one 2x2/s1 SAME after the 6th conv).  It works on any
module exposing the reference's DnnGraphBuilder API (dnn_hip, or the reference's own
wrappers), taking the weight list in the pickle's format
(proj3/yolov2tiny.py:30-77: dicts with kernel / biases / moving_mean / moving_variance /
gamma).  The pickle itself is read by yolo_weights.load_y2t_weights (the reference's
get_y2t_w rejects Python 3.10, proj3/yolov2tiny.py:17-22) and the reference's model class is
mirrored by yolov2tiny.YOLO_V2_TINY.
"""
import numpy as np

EPS = 1e-5


def build_graph(builder_cls, weights, in_shape=(1, 416, 416, 3)):
    """Return (graph, nodes) with nodes in creation order (40 nodes for YOLOv2-tiny)."""
    g = builder_cls()
    nodes = []
    x = g.create_input(list(in_shape))
    s1 = [1, 1, 1, 1]
    last = len(weights) - 1
    for i, w in enumerate(weights):
        x = g.create_conv2d(x, w["kernel"], strides=s1, padding="SAME")
        nodes.append(x)
        x = g.create_bias_add(x, w["biases"])
        nodes.append(x)
        if i == last:  # conv22 + bias only (proj3/yolov2tiny.py:76-77)
            break
        x = g.create_batch_norm(x, w["moving_mean"], w["moving_variance"], w["gamma"], EPS)
        nodes.append(x)
        x = g.create_leaky_relu(x)
        nodes.append(x)
        if i < 5:
            x = g.create_max_pool2d(x, ksize=[1, 2, 2, 1], strides=[1, 2, 2, 1], padding="SAME")
            nodes.append(x)
        elif i == 5:
            x = g.create_max_pool2d(x, ksize=[1, 2, 2, 1], strides=[1, 1, 1, 1], padding="SAME")
            nodes.append(x)
    g.set_out_node(x)
    return g, nodes


def conv_flops_per_image(weights, in_hw=(416, 416)):
    """Algorithmic conv FLOPs per image, 2*M*N*K summed over the 9 convs (6.971 GFLOP for
    the tiny-yolo-voc plan at 416x416)."""
    h, w = in_hw
    total = 0.0
    for i, wt in enumerate(weights):
        kh, kw, ic, od = wt["kernel"].shape
        total += 2.0 * h * w * od * kh * kw * ic
        if i < 5:
            h, w = (h + 1) // 2, (w + 1) // 2
    return total


def zero_weights_like(weights):
    """Same shapes, zero values: lets a non-root rank build its plan layout before the
    weight broadcast overwrites the packed buffer."""
    return [{k: np.zeros_like(v) for k, v in w.items()} for w in weights]
