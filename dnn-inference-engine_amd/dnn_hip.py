"""dnn_hip — MI355X (gfx950) drop-in for proj3's `dnn_openblas.py` / `dnn_cublas.py`.

Same public surface as the reference wrapper (proj3/dnn_openblas.py:23-300):
`DnnGraphBuilder` with `create_input / create_conv2d / create_bias_add /
create_batch_norm / create_leaky_relu / create_max_pool2d / set_out_node`, the node
classes `Conv2D, BiasAdd, MaxPool2D, BatchNorm, LeakyReLU, Input` with the same
constructor arguments and `ValueError` shape checks, `get_out_pads`, and
`DnnInferenceEngine(graph, debug).run(tin) -> np.ndarray`.  `yolov2tiny.py` switches
engines by its import line (proj3/yolov2tiny.py:5):

    from dnn_hip import DnnGraphBuilder, DnnInferenceEngine

Execution.  `run` lowers the node chain ONCE to a device-resident plan
(include/dnn_hip_plan.h): every Conv2D -> BiasAdd -> BatchNorm -> LeakyReLU run becomes
one im2col + fp32-MFMA GEMM with the element-wise ops in its epilogue, every MaxPool2D
one pool kernel; weights are uploaded once and activations stay in HBM.  With
`debug=True` (or a graph the plan cannot express) it instead runs node by node through
the per-op C-ABI (`conv2d_mul`, `bias_add`, ... in libdnn_hip.so, include/dnn_hip.h),
exactly like the reference, and saves every layer to ./intermediate/layer_{k}.npy
(counter from 1, proj3/dnn_openblas.py:47-50; the reference saves unconditionally, the
AVX wrapper only in debug mode, proj3/dnn_avx.py:55-57 — we follow the latter).

Numerics are the reference's correct semantics: fp32 everywhere, the
conv accumulation order differs from OpenBLAS, so outputs match within the stated
normwise tolerance max|d| <= 1e-4 * max|ref|; the element-wise ops and max pool are
bit-exact.  There is no CPU fallback: a missing or broken HIP library raises.
"""
import ctypes
import math
import os

import numpy as np

try:  # the reference's graph container (proj3/dnn_openblas.py:1-4)
    import networkx as nx
except ImportError:  # pragma: no cover - networkx ships in the image
    nx = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = os.environ.get("DNN_HIP_LIB", "libdnn_hip.so")

c_float_pointer_type = ctypes.POINTER(ctypes.c_float)
c_int_pointer_type = ctypes.POINTER(ctypes.c_int)


class DnnHipError(RuntimeError):
    pass


def _bind_plan_api(lib):
    vp, i, f, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
    P = ctypes.POINTER
    sig = {
        "dnn_last_error": (ctypes.c_char_p, []),
        "dnn_plan_create": (i, [i, i, i, i, P(vp)]),
        "dnn_plan_destroy": (None, [vp]),
        "dnn_plan_add_conv": (i, [vp, i, i, i, i, i, i, vp, vp, vp, vp, vp, f, i]),
        "dnn_plan_add_max_pool": (i, [vp, i, i, i, i, i]),
        "dnn_plan_output_shape": (i, [vp, P(i), P(i), P(i), P(i)]),
        "dnn_plan_describe": (i, [vp, ctypes.c_char_p, i]),
        "dnn_plan_memory": (i, [vp, P(sz), P(sz)]),
        "dnn_plan_finalize": (i, [vp, i, vp, vp]),
        "dnn_plan_weight_buffer": (i, [vp, P(vp), P(sz)]),
        "dnn_plan_run": (i, [vp, i, vp, vp, vp]),
        "dnn_plan_run_host": (i, [vp, i, vp, vp]),
        "dnn_plan_run_graph": (i, [vp, i, vp, vp, vp]),
        "dnn_plan_set_precision": (i, [vp, i]),
        "dnn_plan_set_latency_mode": (i, [vp, i]),
        "dnn_plan_num_kernels": (i, [vp]),
        "dnn_plan_kernel_info": (i, [vp, i, ctypes.c_char_p, i, P(ctypes.c_double), P(ctypes.c_double)]),
        "dnn_plan_timing_begin": (i, [vp, i]),
        "dnn_plan_timing_begin_only": (i, [vp, i, i]),
        "dnn_plan_timing_end": (i, [vp, P(ctypes.c_double), P(ctypes.c_longlong)]),
        "dnn_clock_stamp": (i, [vp, vp, i]),
        "dnn_plan_clock_begin": (i, [vp, i, vp, i, i]),
        "dnn_plan_clock_end": (i, [vp, P(i)]),
        "dnn_plan_set_mark": (i, [vp, i]),
        "dnn_plan_wait_mark": (i, [vp, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def _one_hip_runtime():
    """PyTorch-ROCm bundles its own libamdhip64.so (SONAME libamdhip64.so.7).  If torch is
    importable, import it BEFORE our library so that our NEEDED libamdhip64.so.7 resolves to
    that already-loaded runtime by SONAME: one HIP runtime per process, and device pointers
    and streams from torch are valid here.  Without torch the system ROCm runtime is used."""
    if os.environ.get("DNN_HIP_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load_library(name=LIB_NAME):
    """Load one of the in-tree C-ABI libraries (built by csrc/Makefile).  Fails loudly:
    there is no CPU fallback for the product path."""
    _one_hip_runtime()
    path = name if os.path.isabs(name) else os.path.join(_HERE, name)
    if not os.path.exists(path):
        raise DnnHipError(f"{path} not found: build it with `make -C {os.path.join(_HERE, 'csrc')}` "
                          "(or __graft_entry__.build())")
    return _bind_plan_api(ctypes.CDLL(path))


mylib = load_library()


def last_error(lib=None):
    msg = (lib or mylib).dnn_last_error()
    return msg.decode() if msg else ""


def _check(rc, what, lib=None):
    if rc != 0:
        raise DnnHipError(f"{what} failed ({rc}): {last_error(lib)}")


def _check_legacy(what):
    msg = last_error()
    if msg:
        raise DnnHipError(f"{what} failed: {msg}")


def _fp(a):
    return a.ctypes.data_as(c_float_pointer_type)


def _vp(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


PRECISIONS = {"fp32": 0, "fp16": 1}


def _precision(p):
    p = (os.environ.get("DNN_HIP_PRECISION", "fp32") if p is None else p).lower()
    if p not in PRECISIONS:
        raise ValueError(f"precision must be one of {sorted(PRECISIONS)}, got {p!r}")
    return p


class DnnInferenceEngine(object):
    """proj3/dnn_openblas.py:23-57.  `device` picks the GPU (default $DNN_HIP_DEVICE or 0);
    `precision` "fp32" (default, the reference's arithmetic) or "fp16" (fp16 MFMA conv path,
    BASELINE config 5; default from $DNN_HIP_PRECISION); `latency` True builds a latency plan
    (dnn_plan_set_latency_mode: K splits chosen for the graph's batch, for single-frame
    inference as proj3/__init__.py:24-26 runs it; fp32 only).  Unset, $DNN_HIP_LATENCY=1 turns
    it on for fp32 engines and is ignored by fp16 ones; latency=True with fp16 is an error."""

    def __init__(self, graph, debug, device=None, precision=None, latency=None):
        self.g = graph
        self.debug = debug
        self.precision = _precision(precision)
        if latency is None:  # the environment default applies where latency plans exist (fp32)
            latency = os.environ.get("DNN_HIP_LATENCY") == "1" and self.precision == "fp32"
        self.latency = bool(latency)
        self.device = int(os.environ.get("DNN_HIP_DEVICE", "0")) if device is None else device
        self.save_dir = os.path.join(os.getcwd(), "intermediate")
        self._plan = None
        self._chain = None

    # -- fused, device-resident path ------------------------------------------------
    def plan(self):
        """The lowered plan (built on first use; weights uploaded once)."""
        if self._plan is None:
            self._plan = Plan.from_graph(self.g, device=self.device, precision=self.precision,
                                         latency=self.latency)
        return self._plan

    def run(self, tin):
        self.g.in_node.set_input(tin)
        if not self.debug and lower_graph(self.g) is not None:
            x = np.ascontiguousarray(tin, dtype=np.float32)
            out = self.plan().run_host(x)
            self.g.out_node.result = out
            return out
        return self._run_nodes()

    # -- node-by-node path through the per-op ABI (the reference's traversal) --------
    def _run_nodes(self):
        out = {}
        currents = [self.g.in_node]
        done = set()
        counter = 0
        if self.debug:
            os.makedirs(self.save_dir, exist_ok=True)
        while len(currents) != 0:
            nexts = []
            for current in currents:
                if current in done:
                    continue
                if any(p not in done for p in self.g.predecessors(current)):
                    nexts.extend(p for p in self.g.predecessors(current) if p not in done)
                    continue
                current.run()
                if not isinstance(current, Input):
                    counter += 1
                    if self.debug:
                        np.save(os.path.join(self.save_dir, "layer_{}.npy".format(counter)), current.result)
                if self.g.is_out_node(current):
                    out = current.result
                done.add(current)
                nexts.extend(self.g.successors(current))
            currents = nexts
        return out


class _DiGraph(object):
    """Minimal stand-in for networkx.DiGraph when networkx is unavailable."""

    def __init__(self):
        self._succ, self._pred = {}, {}

    def add_node(self, n):
        self._succ.setdefault(n, [])
        self._pred.setdefault(n, [])

    def add_edge(self, a, b):
        self.add_node(a)
        self.add_node(b)
        self._succ[a].append(b)
        self._pred[b].append(a)

    def successors(self, n):
        return iter(self._succ.get(n, []))

    def predecessors(self, n):
        return iter(self._pred.get(n, []))


class DnnGraphBuilder(object):
    """proj3/dnn_openblas.py:59-114."""

    def __init__(self):
        self.G = nx.DiGraph() if nx is not None else _DiGraph()
        self.name_num = {"conv2d": 0, "bias_add": 0, "max_pool2d": 0, "batch_norm": 0, "leaky_relu": 0,
                         "input": 0}
        self.in_node = None
        self.out_node = None

    def set_in_node(self, node):
        self.in_node = node

    def set_out_node(self, node):
        self.out_node = node

    def is_out_node(self, node):
        return self.out_node is node

    def successors(self, node):
        return list(self.G.successors(node))

    def predecessors(self, node):
        return list(self.G.predecessors(node))

    def get_name(self, layer_name):
        name = layer_name + "_" + str(self.name_num[layer_name])
        self.name_num[layer_name] += 1
        return name

    def create_conv2d(self, in_node, kernel, strides, padding):
        out_node = Conv2D(self.get_name("conv2d"), in_node, kernel, strides, padding)
        self.G.add_edge(in_node, out_node)
        return out_node

    def create_bias_add(self, in_node, biases):
        out_node = BiasAdd(self.get_name("bias_add"), in_node, biases)
        self.G.add_edge(in_node, out_node)
        return out_node

    def create_max_pool2d(self, in_node, ksize, strides, padding):
        out_node = MaxPool2D(self.get_name("max_pool2d"), in_node, ksize, strides, padding)
        self.G.add_edge(in_node, out_node)
        return out_node

    def create_batch_norm(self, in_node, mean, variance, gamma, epsilon):
        out_node = BatchNorm(self.get_name("batch_norm"), in_node, mean, variance, gamma, epsilon)
        self.G.add_edge(in_node, out_node)
        return out_node

    def create_leaky_relu(self, in_node):
        out_node = LeakyReLU(self.get_name("leaky_relu"), in_node)
        self.G.add_edge(in_node, out_node)
        return out_node

    def create_input(self, in_shape):
        out_node = Input(self.get_name("input"), in_shape)
        self.G.add_node(out_node)
        self.set_in_node(out_node)  # Assume there's only one input
        return out_node


class DnnNode(object):
    def __init__(self):
        pass

    def run(self):
        self.result = None


def get_out_pads(in_size, filter_size, stride_size, padding):
    """TF SAME/VALID output size and pads (proj3/dnn_openblas.py:127-142)."""
    assert padding == 'SAME' or padding == 'VALID'
    if padding == 'SAME':
        out_size = math.ceil(float(in_size) / float(stride_size))
        pad_size = max((out_size - 1) * stride_size + filter_size - in_size, 0)
        pad_front = pad_size // 2
        pad_back = pad_size - pad_front
    else:
        out_size = math.ceil(float(in_size - filter_size + 1) / float(stride_size))
        pad_front = 0
        pad_back = 0
    return out_size, pad_front, pad_back


class Conv2D(DnnNode):
    """proj3/dnn_openblas.py:144-188; run() -> conv2d_mul on the device."""

    def __init__(self, name, in_node, kernel, strides, padding):
        batch, np_ih, np_iw, ic = in_node.result.shape
        kh, kw, kernel_ic, od = kernel.shape
        if kernel_ic != ic:
            raise ValueError
        if not (padding == 'SAME' or padding == 'VALID'):
            raise ValueError
        oh, self.pad_top, self.pad_bottom = get_out_pads(np_ih, kh, strides[1], padding)
        ow, self.pad_left, self.pad_right = get_out_pads(np_iw, kw, strides[2], padding)
        self.in_node = in_node
        self.kernel = np.ascontiguousarray(kernel).astype(np.float32)
        self.strides = strides
        self.padding = padding
        self.result = np.zeros((batch, oh, ow, od), dtype='float32')
        # K order (ic, kh, kw), the layout conv2d_mul expects (dnn_openblas.py:166-167)
        self.kernel_r = np.ascontiguousarray(self.kernel.transpose(2, 0, 1, 3).reshape(-1, od))
        # the host im2col scratch of the reference is not needed: the device has its own
        self.col = np.zeros((0,), dtype=np.float32)
        self.name = name

    def run(self):
        in_layer = np.ascontiguousarray(np.pad(
            self.in_node.result,
            [(0, 0), (self.pad_top, self.pad_bottom), (self.pad_left, self.pad_right), (0, 0)],
            'constant'), dtype=np.float32)
        mylib.conv2d_mul(
            _fp(in_layer), _fp(self.col), _fp(self.kernel_r), _fp(self.result),
            *map(ctypes.c_int, self.result.shape),
            *map(ctypes.c_int, in_layer.shape[1:]),
            *map(ctypes.c_int, self.kernel.shape[:2]),
            *map(ctypes.c_int, self.strides[1:3]))
        _check_legacy(self.name)


class BiasAdd(DnnNode):
    """proj3/dnn_openblas.py:190-209; run() -> bias_add."""

    def __init__(self, name, in_node, biases):
        if not (biases.ndim == 1 and in_node.result.shape[-1] == biases.shape[0]):
            raise ValueError
        self.in_node = in_node
        self.biases = np.ascontiguousarray(biases, dtype=np.float32)
        self.result = np.zeros(in_node.result.shape, dtype='float32')
        self.name = name

    def run(self):
        x = np.ascontiguousarray(self.in_node.result, dtype=np.float32)
        mylib.bias_add(_fp(x), _fp(self.biases), _fp(self.result), *map(ctypes.c_int, self.result.shape))
        _check_legacy(self.name)


class MaxPool2D(DnnNode):
    """proj3/dnn_openblas.py:211-242; run() -> max_pool2d on a -FLT_MAX padded input."""

    def __init__(self, name, in_node, ksize, strides, padding):
        if not (padding == 'SAME' or padding == 'VALID'):
            raise ValueError
        batch, in_height, in_width, in_channels = in_node.result.shape
        out_height, self.pad_top, self.pad_bottom = get_out_pads(in_height, ksize[1], strides[1], padding)
        out_width, self.pad_left, self.pad_right = get_out_pads(in_width, ksize[2], strides[2], padding)
        self.in_node = in_node
        self.ksize = ksize
        self.strides = strides
        self.padding = padding
        self.result = np.zeros((batch, out_height, out_width, in_channels), dtype='float32')
        self.name = name

    def run(self):
        in_layer = np.ascontiguousarray(np.pad(
            self.in_node.result,
            [(0, 0), (self.pad_top, self.pad_bottom), (self.pad_left, self.pad_right), (0, 0)],
            'constant', constant_values=np.finfo('float32').min), dtype=np.float32)
        mylib.max_pool2d(_fp(in_layer), _fp(self.result),
                         *map(ctypes.c_int, self.result.shape),
                         *map(ctypes.c_int, in_layer.shape[1:]),
                         *map(ctypes.c_int, self.ksize[1:3]),
                         *map(ctypes.c_int, self.strides[1:3]))
        _check_legacy(self.name)


class BatchNorm(DnnNode):
    """proj3/dnn_openblas.py:244-270; run() -> batch_norm (variance is never mutated)."""

    def __init__(self, name, in_node, mean, variance, gamma, epsilon):
        if not all(arg.ndim == 1 and in_node.result.shape[-1] == arg.shape[0] for arg in [mean, variance, gamma]):
            raise ValueError
        self.in_node = in_node
        self.mean = np.ascontiguousarray(mean, dtype=np.float32)
        self.variance = np.ascontiguousarray(variance, dtype=np.float32)
        self.gamma = np.ascontiguousarray(gamma, dtype=np.float32)
        self.epsilon = epsilon
        self.result = np.zeros(in_node.result.shape, dtype='float32')
        self.name = name

    def run(self):
        x = np.ascontiguousarray(self.in_node.result, dtype=np.float32)
        mylib.batch_norm(_fp(x), _fp(self.mean), _fp(self.variance), _fp(self.gamma),
                         ctypes.c_float(self.epsilon), _fp(self.result), *map(ctypes.c_int, self.result.shape))
        _check_legacy(self.name)


class LeakyReLU(DnnNode):
    """proj3/dnn_openblas.py:272-284; run() -> leaky_relu."""

    def __init__(self, name, in_node):
        self.in_node = in_node
        self.result = np.zeros(in_node.result.shape, dtype='float32')
        self.name = name

    def run(self):
        x = np.ascontiguousarray(self.in_node.result, dtype=np.float32)
        mylib.leaky_relu(_fp(x), _fp(self.result), *map(ctypes.c_int, self.result.shape))
        _check_legacy(self.name)


class Input(DnnNode):
    """proj3/dnn_openblas.py:287-300 (unchanged contract)."""

    def __init__(self, name, in_shape):
        self.name = name
        self.in_shape = in_shape
        self.result = np.ndarray(self.in_shape)

    def set_input(self, tensor):
        assert tuple(self.in_shape) == tuple(tensor.shape)
        self.result = tensor

    def run(self):
        pass


# ---------------------------------------------------------------------------------------
# Graph -> plan lowering
# ---------------------------------------------------------------------------------------
class ConvEntry(object):
    """One fused plan conv: Conv2D [-> BiasAdd] [-> BatchNorm] [-> LeakyReLU]."""

    def __init__(self, conv):
        self.conv, self.bias, self.bn, self.leaky = conv, None, None, False
        self.nodes = [conv]


class PoolEntry(object):
    def __init__(self, pool):
        self.pool = pool
        self.nodes = [pool]


def lower_graph(g):
    """Lower a builder graph to fused plan entries, or None if the graph is not a plain
    chain the plan can express (then the node-by-node path runs)."""
    if g.in_node is None or g.out_node is None:
        return None
    entries = []
    node = g.in_node
    succ = list(g.G.successors(node))
    while True:
        if len(succ) != 1 or g.is_out_node(node):
            break
        nxt = succ[0]
        if len(list(g.G.predecessors(nxt))) != 1:
            return None
        if isinstance(nxt, Conv2D):
            e = ConvEntry(nxt)
            cur = nxt
            for kind in (BiasAdd, BatchNorm, LeakyReLU):
                nn = list(g.G.successors(cur))
                if g.is_out_node(cur) or len(nn) != 1 or not isinstance(nn[0], kind):
                    continue
                cur = nn[0]
                if kind is BiasAdd:
                    e.bias = cur
                elif kind is BatchNorm:
                    e.bn = cur
                else:
                    e.leaky = True
                e.nodes.append(cur)
            entries.append(e)
            node = cur
        elif isinstance(nxt, MaxPool2D):
            entries.append(PoolEntry(nxt))
            node = nxt
        else:
            return None  # a standalone element-wise op: not expressible as a fused entry
        succ = list(g.G.successors(node))
    if not g.is_out_node(node) or not entries:
        return None
    return entries


def clock_stamp(dev_ptr, nwg, stream_ptr, lib=None):
    """Launch the clock-stamp kernel (dnn_clock_stamp): nwg workgroups, 4 uint64 each at dev_ptr."""
    lib = lib or mylib
    _check(lib.dnn_clock_stamp(ctypes.c_void_p(stream_ptr), ctypes.c_void_p(dev_ptr), int(nwg)), "clock_stamp", lib)


def sclk_from_stamps(start, end):
    """Mean shader clock per XCD between two stamp launches (arrays [nwg][4] of uint64:
    s_memtime, s_memrealtime (100 MHz), XCC_ID, HW_ID): per XCD the median of each counter over
    its workgroups, then d(memtime) / d(memrealtime) x 100 MHz.  Returns {"mean", "min", "max",
    "per_xcd": {xcd: GHz}, "window_us"} (GHz, the mean over XCDs)."""
    import numpy as np
    a, b = np.asarray(start, dtype=np.uint64), np.asarray(end, dtype=np.uint64)
    per = {}
    win = []
    for x in sorted(set(int(v) for v in a[:, 2]) & set(int(v) for v in b[:, 2])):
        sa, sb = a[a[:, 2] == x], b[b[:, 2] == x]
        dt = float(np.median(sb[:, 0].astype(np.float64))) - float(np.median(sa[:, 0].astype(np.float64)))
        dr = float(np.median(sb[:, 1].astype(np.float64))) - float(np.median(sa[:, 1].astype(np.float64)))
        if dr > 0 and dt > 0:
            per[x] = dt / dr * 0.1  # memrealtime ticks at 100 MHz: GHz = (dt / dr) x 0.1
            win.append(dr * 0.01)   # microseconds
    if not per:
        return None
    v = list(per.values())
    return {"mean": sum(v) / len(v), "min": min(v), "max": max(v), "per_xcd": per,
            "window_us": sum(win) / len(win)}


def _pad_code(padding):
    return 1 if padding == 'SAME' else 0


class Plan(object):
    """Owner of a dnn_plan handle (include/dnn_hip_plan.h)."""

    def __init__(self, batch, in_shape, entries, device=0, weights_ptr=None, workspace_ptr=None, upload=True,
                 leaky_variant=1, lib=None, precision="fp32", latency=False):
        self.lib = lib or mylib
        self.batch = int(batch)
        self.in_shape = tuple(int(v) for v in in_shape)
        self.precision = _precision(precision)
        h = ctypes.c_void_p()
        _check(self.lib.dnn_plan_create(self.batch, *self.in_shape, ctypes.byref(h)), "dnn_plan_create", self.lib)
        self.h = h
        _check(self.lib.dnn_plan_set_precision(self.h, PRECISIONS[self.precision]), "dnn_plan_set_precision",
               self.lib)
        self.latency = bool(latency)
        if self.latency:
            _check(self.lib.dnn_plan_set_latency_mode(self.h, 1), "dnn_plan_set_latency_mode", self.lib)
        self.entries = entries
        for e in entries:
            if isinstance(e, ConvEntry):
                c = e.conv
                kh, kw, _, od = c.kernel.shape
                bias = e.bias.biases if e.bias is not None else None
                if e.bn is not None:
                    mean, var, gamma, eps = e.bn.mean, e.bn.variance, e.bn.gamma, float(e.bn.epsilon)
                else:
                    mean = var = gamma = None
                    eps = 0.0
                keep = (c.kernel, bias, mean, var, gamma)  # noqa: F841 (alive across the call)
                rc = self.lib.dnn_plan_add_conv(
                    self.h, kh, kw, od, int(c.strides[1]), int(c.strides[2]), _pad_code(c.padding),
                    # without upload only the kernel is withheld: the epilogue pointers still
                    # declare which of bias / BN the layer has (the values arrive with the arena)
                    _vp(c.kernel) if upload else None, _vp(bias), _vp(mean), _vp(var), _vp(gamma), eps,
                    leaky_variant if e.leaky else 0)
                _check(rc, "dnn_plan_add_conv", self.lib)
            else:
                p = e.pool
                _check(self.lib.dnn_plan_add_max_pool(self.h, int(p.ksize[1]), int(p.ksize[2]), int(p.strides[1]),
                                                      int(p.strides[2]), _pad_code(p.padding)),
                       "dnn_plan_add_max_pool", self.lib)
        b, oh, ow, oc = (ctypes.c_int() for _ in range(4))
        _check(self.lib.dnn_plan_output_shape(self.h, ctypes.byref(b), ctypes.byref(oh), ctypes.byref(ow),
                                              ctypes.byref(oc)), "dnn_plan_output_shape", self.lib)
        self.out_shape = (oh.value, ow.value, oc.value)
        self.device = device
        _check(self.lib.dnn_plan_finalize(self.h, device, weights_ptr, workspace_ptr), "dnn_plan_finalize",
               self.lib)

    @classmethod
    def from_graph(cls, g, device=0, **kw):
        entries = lower_graph(g)
        if entries is None:
            raise DnnHipError("graph is not a conv/pool chain the fused plan can express")
        return cls(g.in_node.in_shape[0], tuple(g.in_node.in_shape[1:]), entries, device=device, **kw)

    @staticmethod
    def memory(batch, in_shape, entries, lib=None, precision="fp32", latency=False):
        """(weight_bytes, workspace_bytes) a plan of this shape needs, without finalizing."""
        lib = lib or mylib
        h = ctypes.c_void_p()
        _check(lib.dnn_plan_create(int(batch), *in_shape, ctypes.byref(h)), "dnn_plan_create", lib)
        try:
            _check(lib.dnn_plan_set_precision(h, PRECISIONS[_precision(precision)]), "dnn_plan_set_precision", lib)
            if latency:
                _check(lib.dnn_plan_set_latency_mode(h, 1), "dnn_plan_set_latency_mode", lib)
            for e in entries:
                if isinstance(e, ConvEntry):
                    kh, kw, _, od = e.conv.kernel.shape
                    _check(lib.dnn_plan_add_conv(h, kh, kw, od, int(e.conv.strides[1]), int(e.conv.strides[2]),
                                                 _pad_code(e.conv.padding), None, None, None, None, None, 0.0,
                                                 1 if e.leaky else 0), "dnn_plan_add_conv", lib)
                else:
                    p = e.pool
                    _check(lib.dnn_plan_add_max_pool(h, int(p.ksize[1]), int(p.ksize[2]), int(p.strides[1]),
                                                     int(p.strides[2]), _pad_code(p.padding)),
                           "dnn_plan_add_max_pool", lib)
            wb, sb = ctypes.c_size_t(), ctypes.c_size_t()
            _check(lib.dnn_plan_memory(h, ctypes.byref(wb), ctypes.byref(sb)), "dnn_plan_memory", lib)
            return wb.value, sb.value
        finally:
            lib.dnn_plan_destroy(h)

    def describe(self):
        buf = ctypes.create_string_buffer(8192)
        _check(self.lib.dnn_plan_describe(self.h, buf, 8192), "dnn_plan_describe", self.lib)
        return buf.value.decode()

    def weight_buffer(self):
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        _check(self.lib.dnn_plan_weight_buffer(self.h, ctypes.byref(p), ctypes.byref(n)), "weight_buffer", self.lib)
        return p.value, n.value

    def run_host(self, x):
        x = np.ascontiguousarray(x, dtype=np.float32)
        n = x.shape[0]
        if tuple(x.shape[1:]) != self.in_shape or n > self.batch:
            raise ValueError(f"input {x.shape} does not fit plan [{self.batch}, {self.in_shape}]")
        out = np.empty((n,) + self.out_shape, dtype=np.float32)
        _check(self.lib.dnn_plan_run_host(self.h, n, _vp(x), _vp(out)), "dnn_plan_run_host", self.lib)
        return out

    def run_device(self, n, in_ptr, out_ptr, stream_ptr=None):
        _check(self.lib.dnn_plan_run(self.h, int(n), ctypes.c_void_p(in_ptr), ctypes.c_void_p(out_ptr),
                                     ctypes.c_void_p(stream_ptr) if stream_ptr else None),
               "dnn_plan_run", self.lib)

    def run_graph(self, n, in_ptr, out_ptr, stream_ptr):
        """run_device through a captured HIP graph (dnn_plan_run_graph): one submission per
        forward after the first call for these (n, in, out)."""
        _check(self.lib.dnn_plan_run_graph(self.h, int(n), ctypes.c_void_p(in_ptr), ctypes.c_void_p(out_ptr),
                                           ctypes.c_void_p(stream_ptr)), "dnn_plan_run_graph", self.lib)

    def kernels(self):
        out = []
        for i in range(self.lib.dnn_plan_num_kernels(self.h)):
            name = ctypes.create_string_buffer(64)
            fl, by = ctypes.c_double(), ctypes.c_double()
            _check(self.lib.dnn_plan_kernel_info(self.h, i, name, 64, ctypes.byref(fl), ctypes.byref(by)),
                   "kernel_info", self.lib)
            out.append({"name": name.value.decode(), "flops": fl.value, "bytes": by.value})
        return out

    def timing_begin(self, max_runs, only=None):
        """Per-kernel HIP events over the next runs; `only` = a kernel name: events around that
        kernel alone (dnn_plan_timing_begin_only)."""
        if only is None:
            _check(self.lib.dnn_plan_timing_begin(self.h, int(max_runs)), "timing_begin", self.lib)
            return
        idx = [k["name"] for k in self.kernels()].index(only)
        _check(self.lib.dnn_plan_timing_begin_only(self.h, int(max_runs), idx), "timing_begin_only", self.lib)

    def timing_end(self):
        nk = self.lib.dnn_plan_num_kernels(self.h)
        ms = (ctypes.c_double * nk)()
        cnt = (ctypes.c_longlong * nk)()
        _check(self.lib.dnn_plan_timing_end(self.h, ms, cnt), "timing_end", self.lib)
        return list(ms), list(cnt)

    def clock_begin(self, kernel, dev_buf_ptr, max_runs, nwg):
        """Shader-clock stamps around `kernel` (a kernel name) in the next runs, into a device
        buffer of max_runs x 8 x nwg uint64 (dnn_plan_clock_begin; sclk_from_stamps reads them)."""
        idx = [k["name"] for k in self.kernels()].index(kernel)
        _check(self.lib.dnn_plan_clock_begin(self.h, idx, ctypes.c_void_p(dev_buf_ptr), int(max_runs), int(nwg)),
               "clock_begin", self.lib)

    def clock_end(self):
        runs = ctypes.c_int()
        _check(self.lib.dnn_plan_clock_end(self.h, ctypes.byref(runs)), "clock_end", self.lib)
        return runs.value

    def set_mark(self, kernel):
        """Record an event right before `kernel` (a kernel name; None: off) in every later run
        (dnn_plan_set_mark); wait_mark(stream) makes a stream wait for the latest run's mark."""
        idx = -1 if kernel is None else [k["name"] for k in self.kernels()].index(kernel)
        _check(self.lib.dnn_plan_set_mark(self.h, idx), "set_mark", self.lib)

    def wait_mark(self, stream_ptr):
        _check(self.lib.dnn_plan_wait_mark(self.h, ctypes.c_void_p(stream_ptr)), "wait_mark", self.lib)

    def close(self):
        if getattr(self, "h", None):
            self.lib.dnn_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
