"""YOLOv2 postprocessing on the GPU — drop-in for the reference's host-side
`postprocessing(predictions)` (cs492-projects/proj3/yolov2tiny.py:94-234).

    from yolo_post import postprocessing          # same name, argument and return value
    label_boxes = postprocessing(engine.run(frame))  # [(name, (l, t), (r, b), color)]

The work runs in `dnn_yolo_postprocess` (include/dnn_hip_post.h, csrc/postprocess.hip):
decode + threshold + sort + greedy NMS, one workgroup per image.  `detect_batch` handles a
whole [B,13,13,125] batch in one launch, and `DetectionBuffers` keeps the outputs on the
device for the multi-GPU detection gather (dist.py).  There is no CPU fallback: a missing
library raises (dnn_hip.load_library).
"""
import ctypes

import numpy as np

import dnn_hip

N_BOXES = 845  # DNN_YOLO_BOXES: 13 * 13 * 5, the most detections an image can have
PRED_FLOATS = 13 * 13 * 125

# yolov2tiny.py:102-112 (data)
CLASSES = ("aeroplane", "bicycle", "bird", "boat", "bottle", "bus", "car", "cat", "chair", "cow", "diningtable",
           "dog", "horse", "motorbike", "person", "pottedplant", "sheep", "sofa", "train", "tvmonitor")
COLORS = ((254.0, 254.0, 254), (239.88888888888889, 211.66666666666669, 127),
          (225.77777777777777, 169.33333333333334, 0), (211.66666666666669, 127.0, 254),
          (197.55555555555557, 84.66666666666667, 127), (183.44444444444443, 42.33333333333332, 0),
          (169.33333333333334, 0.0, 254), (155.22222222222223, -42.33333333333335, 127),
          (141.11111111111111, -84.66666666666664, 0), (127.0, 254.0, 254),
          (112.88888888888889, 211.66666666666669, 127), (98.77777777777777, 169.33333333333334, 0),
          (84.66666666666667, 127.0, 254), (70.55555555555556, 84.66666666666667, 127),
          (56.44444444444444, 42.33333333333332, 0), (42.33333333333332, 0.0, 254),
          (28.222222222222236, -42.33333333333335, 127), (14.111111111111118, -84.66666666666664, 0),
          (0.0, 254.0, 254), (-14.111111111111118, 211.66666666666669, 127))


class Detection(ctypes.Structure):
    """dnn_detection (include/dnn_hip_post.h), 40 bytes."""
    _fields_ = [("cls", ctypes.c_int), ("score", ctypes.c_float), ("left", ctypes.c_longlong),
                ("top", ctypes.c_longlong), ("right", ctypes.c_longlong), ("bottom", ctypes.c_longlong)]


DETECTION_DTYPE = np.dtype([("cls", "<i4"), ("score", "<f4"), ("left", "<i8"), ("top", "<i8"), ("right", "<i8"),
                            ("bottom", "<i8")])
assert DETECTION_DTYPE.itemsize == ctypes.sizeof(Detection) == 40


def _bind(lib):
    vp, i = ctypes.c_void_p, ctypes.c_int
    lib.dnn_yolo_postprocess.restype = i
    lib.dnn_yolo_postprocess.argtypes = [vp, i, vp, i, vp, vp]
    lib.dnn_yolo_postprocess_host.restype = i
    lib.dnn_yolo_postprocess_host.argtypes = [vp, i, vp, i, vp]
    lib.dnn_yolo_pack_detections.restype = i
    lib.dnn_yolo_pack_detections.argtypes = [vp, vp, i, i, vp, vp, vp]
    return lib


_lib = _bind(dnn_hip.mylib)


ERRORS = {-1: "a box corner is not finite or out of int64 range (the reference's int() raises there)",
          -2: "an IoU denominator is zero (the reference raises ZeroDivisionError)"}


def _rows(dets, counts, max_det, raise_errors=True):
    out = []
    for i, n in enumerate(counts):
        if n < 0:
            if not raise_errors:
                out.append(int(n))
                continue
            raise dnn_hip.DnnHipError(f"image {i}: " + ERRORS.get(int(n), f"error {n}"))
        if n > max_det:
            raise dnn_hip.DnnHipError(f"image {i}: {n} detections > max_det {max_det}")
        out.append([(int(d["cls"]), int(d["left"]), int(d["top"]), int(d["right"]), int(d["bottom"]),
                     float(d["score"])) for d in dets[i, :n]])
    return out


def detect_batch(predictions, max_det=N_BOXES, raise_errors=True):
    """[B,13,13,125] (or [13,13,125]) fp32 host predictions -> per image a list of
    (class, left, top, right, bottom, score) in the reference's output order.  An image on
    which the reference raises raises DnnHipError, or with raise_errors=False yields its
    negative error code (ERRORS) in place of the list."""
    p = np.ascontiguousarray(predictions, dtype=np.float32)
    if p.size % PRED_FLOATS:
        raise ValueError(f"predictions of shape {p.shape} are not [B,13,13,125]")
    n = p.size // PRED_FLOATS
    dets = np.zeros((n, max_det), DETECTION_DTYPE)
    counts = np.zeros(n, np.int32)
    dnn_hip._check(_lib.dnn_yolo_postprocess_host(p.ctypes.data, n, dets.ctypes.data, max_det,
                                                  counts.ctypes.data), "dnn_yolo_postprocess_host")
    return _rows(dets, counts, max_det, raise_errors)


def label_boxes(rows):
    """(class, l, t, r, b, score) rows -> the reference's label_boxes tuples."""
    return [(CLASSES[c], (l, t), (r, b), COLORS[c]) for c, l, t, r, b, _ in rows]


def postprocessing(predictions):
    """yolov2tiny.py:94-176: one image's [1,13,13,125] output -> [(class name, (left, top),
    (right, bottom), color)] after the 0.3 threshold and greedy NMS."""
    p = np.asarray(predictions, dtype=np.float32)
    if p.size != PRED_FLOATS:
        raise ValueError(f"postprocessing expects one 13x13x125 prediction, got shape {p.shape}")
    return label_boxes(detect_batch(p)[0])


class DetectionBuffers(object):
    """Device-side outputs for `n` images (torch tensors on `device`): dets [n, max_det, 40 B]
    as uint8 and counts [n] int32, filled by `run(pred_ptr, n, stream)` asynchronously;
    `pack(n, stream)` then compacts them image-major into packed [n * max_det, 40] with the
    row count in total[0] (dnn_yolo_pack_detections), ready for dist.gather_detections."""

    def __init__(self, n, device, max_det=N_BOXES):
        import torch
        self.n, self.max_det = n, max_det
        self.dets = torch.zeros((n, max_det, DETECTION_DTYPE.itemsize), dtype=torch.uint8, device=device)
        self.counts = torch.zeros(n, dtype=torch.int32, device=device)
        self.packed = torch.zeros((n * max_det, DETECTION_DTYPE.itemsize), dtype=torch.uint8, device=device)
        self.total = torch.zeros(1, dtype=torch.int32, device=device)

    def run(self, pred_ptr, n, stream):
        dnn_hip._check(_lib.dnn_yolo_postprocess(pred_ptr, n, self.dets.data_ptr(), self.max_det,
                                                 self.counts.data_ptr(), stream), "dnn_yolo_postprocess")

    def pack(self, n, stream):
        dnn_hip._check(_lib.dnn_yolo_pack_detections(self.dets.data_ptr(), self.counts.data_ptr(), n, self.max_det,
                                                     self.packed.data_ptr(), self.total.data_ptr(), stream),
                       "dnn_yolo_pack_detections")
        return self.packed, self.total, self.counts

    @staticmethod
    def to_rows(dets_u8, counts, max_det=N_BOXES, raise_errors=True):
        """Host copies (numpy uint8 [n, max_det, 40], int32 [n]) -> per-image rows."""
        d = np.ascontiguousarray(dets_u8).view(DETECTION_DTYPE).reshape(len(counts), max_det)
        return _rows(d, np.asarray(counts), max_det, raise_errors)
