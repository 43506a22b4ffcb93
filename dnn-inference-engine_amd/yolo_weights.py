"""The YOLOv2-tiny weight pickle: format, safe loader, writer.

Format (cs492-projects/proj3/yolov2tiny.py:15-77): a pickled list of 9 dicts, one per
conv layer, with fp32 numpy arrays
    "kernel"          HWIO [kh, kw, in_c, out_c]   (3x3 for convs 0-7, 1x1 for conv 8)
    "biases"          [out_c]
    "moving_mean", "moving_variance", "gamma"   [out_c]   (convs 0-7; BatchNorm eps 1e-5)
The reference reads it with `pickle.load(h)` on Python 2.7 or `pickle.load(h,
encoding='latin1')` on 3.5 and raises on anything else (yolov2tiny.py:15-22).  Here the file
is read by a restricted unpickler that can only rebuild numpy arrays / dtypes / scalars and
plain containers — nothing else in the file can run — on any Python 3, with latin1 for
Python-2 pickles, then validated (layer count, keys, shapes chaining from 3 input channels)
and converted to contiguous fp32.  `dnn_hip.Plan` packs the result into the device layouts
(Bt[Npad][Kpad] + epilogue vectors) once at finalize.
"""
import io
import pickle

import numpy as np

N_LAYERS = 9
BN_KEYS = ("moving_mean", "moving_variance", "gamma")

# the only globals a numpy-array pickle needs (protocols 0-5, numpy 1.x or 2.x writers)
_ALLOWED = {
    ("numpy.core.multiarray", "_reconstruct"): ("numpy._core.multiarray", "_reconstruct"),
    ("numpy._core.multiarray", "_reconstruct"): ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"): ("numpy._core.multiarray", "scalar"),
    ("numpy._core.multiarray", "scalar"): ("numpy._core.multiarray", "scalar"),
    ("numpy", "ndarray"): ("numpy", "ndarray"),
    ("numpy", "dtype"): ("numpy", "dtype"),
    ("_codecs", "encode"): ("_codecs", "encode"),
}


class WeightFileError(ValueError):
    pass


class _ArrayUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        target = _ALLOWED.get((module, name))
        if target is None:
            raise WeightFileError(f"weight pickle references {module}.{name}: only numpy arrays are allowed")
        return super().find_class(*target)


def _safe_load(data):
    try:
        return _ArrayUnpickler(io.BytesIO(data), encoding="latin1").load()
    except WeightFileError:
        raise
    except Exception as e:
        raise WeightFileError(f"not a readable weight pickle: {e!r}") from e


def validate(weights):
    """Check the 9-layer structure and return it as fp32 contiguous arrays (new dicts)."""
    if not isinstance(weights, (list, tuple)) or len(weights) != N_LAYERS:
        raise WeightFileError(f"expected a list of {N_LAYERS} layer dicts, got {type(weights).__name__} "
                              f"of length {len(weights) if hasattr(weights, '__len__') else '?'}")
    out, in_c = [], 3
    for i, w in enumerate(weights):
        if not isinstance(w, dict):
            raise WeightFileError(f"layer {i}: expected a dict, got {type(w).__name__}")
        keys = ("kernel", "biases") + (BN_KEYS if i < N_LAYERS - 1 else ())
        missing = [k for k in keys if k not in w]
        if missing:
            raise WeightFileError(f"layer {i}: missing {missing}")
        d = {}
        for k in keys:
            a = np.asarray(w[k])
            if a.dtype.kind not in "fiu":
                raise WeightFileError(f"layer {i} {k}: non-numeric dtype {a.dtype}")
            d[k] = np.ascontiguousarray(a, dtype=np.float32)
        k = d["kernel"]
        kk = 1 if i == N_LAYERS - 1 else 3
        if k.ndim != 4 or k.shape[0] != kk or k.shape[1] != kk or k.shape[2] != in_c:
            raise WeightFileError(f"layer {i}: kernel shape {k.shape}, expected ({kk}, {kk}, {in_c}, out)")
        od = k.shape[3]
        for key in keys[1:]:
            if d[key].shape != (od,):
                raise WeightFileError(f"layer {i} {key}: shape {d[key].shape}, expected ({od},)")
        out.append(d)
        in_c = od
    if in_c != 125:
        raise WeightFileError(f"last layer has {in_c} outputs; YOLOv2-tiny VOC needs 125 (yolov2tiny.py:120)")
    return out


def load_y2t_weights(path):
    """Read and validate a YOLOv2-tiny weight pickle (Python-2 or -3 written)."""
    with open(path, "rb") as f:
        return validate(_safe_load(f.read()))


def save_y2t_weights(weights, path, protocol=2):
    """Write `weights` in the reference's pickle format (protocol 2 is readable by the
    reference's Python 2.7 and 3.5 loaders too)."""
    w = validate(weights)
    with open(path, "wb") as f:
        pickle.dump([dict(d) for d in w], f, protocol=protocol)
