"""CPU-only checks of the drop-in boundary and the host logic (no GPU compute):
  * both C-ABI libraries load and export every function include/*.h declares;
  * the Python mirror keeps the reference's API and ValueError checks;
  * graph lowering fuses conv->bias->bn->leaky and keeps pools;
  * the plan's shape inference / memory / algorithmic-FLOP bookkeeping (pure host code)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import PKG, REPO

import dnn_hip
import synth
import yolo_graph
import ref_numpy as R

HEADERS = {
    "libdnn_hip.so": ["dnn_hip_plan.h", "dnn_hip.h", "dnn_hip_post.h", "dnn_hip_ingest.h"],
    "libdnn_hip_avx.so": ["dnn_hip_plan.h", "dnn_hip_avx.h", "dnn_hip_post.h", "dnn_hip_ingest.h"],
}


def declared_functions(header):
    text = open(os.path.join(REPO, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?(?:void|int|char|size_t)\s*\**\s*(\w+)\s*\(", text, flags=re.M)
    return set(names)


@pytest.mark.parametrize("lib", sorted(HEADERS))
def test_library_exports_every_declared_symbol(lib):
    so = ctypes.CDLL(os.path.join(PKG, lib))
    names = set()
    for h in HEADERS[lib]:
        names |= declared_functions(h)
    assert len(names) >= 15
    missing = [n for n in sorted(names) if not hasattr(so, n)]
    assert not missing, missing


def test_reference_symbol_sets_present():
    """The exact symbol names the reference wrappers bind."""
    ob = declared_functions("dnn_hip.h")
    assert {"conv2d_mul", "conv2d_cublas", "bias_add", "batch_norm", "max_pool2d", "leaky_relu", "im2col"} <= ob
    av = declared_functions("dnn_hip_avx.h")
    assert {"conv2d_pthread", "conv2d_cuda_pthread", "bias_add_pthread", "max_pool2d_pthread", "max_pool2d_avx",
            "batch_norm", "batch_norm_cuda", "leaky_relu"} <= av


def test_get_out_pads_matches_reference_rule():
    for n in range(1, 40):
        for k in (1, 2, 3):
            for s in (1, 2, 3):
                for p in ("SAME", "VALID"):
                    if p == "VALID" and n < k:
                        continue
                    assert dnn_hip.get_out_pads(n, k, s, p) == R.get_out_pads(n, k, s, p)


def test_node_value_errors():
    g = dnn_hip.DnnGraphBuilder()
    x = g.create_input([1, 5, 5, 3])
    with pytest.raises(ValueError):
        g.create_conv2d(x, np.zeros((3, 3, 4, 8), np.float32), [1, 1, 1, 1], "SAME")
    with pytest.raises(ValueError):
        g.create_conv2d(x, np.zeros((3, 3, 3, 8), np.float32), [1, 1, 1, 1], "FULL")
    with pytest.raises(ValueError):
        g.create_bias_add(x, np.zeros(4, np.float32))
    with pytest.raises(ValueError):
        g.create_batch_norm(x, np.zeros(3), np.zeros(4), np.zeros(3), 1e-5)
    with pytest.raises(ValueError):
        g.create_max_pool2d(x, [1, 2, 2, 1], [1, 2, 2, 1], "full")
    c = g.create_conv2d(x, np.zeros((3, 3, 3, 8), np.float32), [1, 2, 2, 1], "SAME")
    assert c.result.shape == (1, 3, 3, 8)
    assert c.kernel_r.shape == (27, 8)
    names = [c.name, g.create_bias_add(c, np.zeros(8, np.float32)).name]
    # as in the reference, get_name() advances the counter before a constructor raises
    # (proj3/dnn_openblas.py:81-89): two failed convs and one failed bias_add came first
    assert names == ["conv2d_2", "bias_add_1"]


def test_yolo_graph_lowering():
    ws = synth.yolo_weights()
    g, nodes = yolo_graph.build_graph(dnn_hip.DnnGraphBuilder, ws)
    assert len(nodes) == 40
    entries = dnn_hip.lower_graph(g)
    kinds = ["C" if isinstance(e, dnn_hip.ConvEntry) else "P" for e in entries]
    assert "".join(kinds) == "CPCPCPCPCPCPCCC"
    convs = [e for e in entries if isinstance(e, dnn_hip.ConvEntry)]
    assert all(e.bias is not None for e in convs)
    assert all(e.bn is not None and e.leaky for e in convs[:-1])
    assert convs[-1].bn is None and not convs[-1].leaky
    assert sum(len(e.nodes) for e in entries) == 40
    assert yolo_graph.conv_flops_per_image(ws) == pytest.approx(6.971e9, rel=1e-3)


def test_lowering_rejects_unfusable_graph():
    g = dnn_hip.DnnGraphBuilder()
    x = g.create_input([1, 4, 4, 8])
    y = g.create_leaky_relu(x)  # element-wise op with no producing conv
    g.set_out_node(y)
    assert dnn_hip.lower_graph(g) is None


@pytest.mark.parametrize("fuse,splitk", [("1", "1"), ("0", "1"), ("1", "0")])
def test_plan_shape_memory_and_flops_host_only(monkeypatch, fuse, splitk):
    """The fp32-MFMA plan (DNN_HIP_X3=0; the x3 plan: test_plan_x3_structure_host_only)."""
    monkeypatch.setenv("DNN_HIP_FUSE", fuse)
    monkeypatch.setenv("DNN_HIP_SPLITK_FUSED", splitk)
    monkeypatch.setenv("DNN_HIP_X3", "0")
    ws = synth.yolo_weights()
    g, _ = yolo_graph.build_graph(dnn_hip.DnnGraphBuilder, ws, in_shape=(64, 416, 416, 3))
    entries = dnn_hip.lower_graph(g)
    wb, sb = dnn_hip.Plan.memory(64, (416, 416, 3), entries)
    nparams = sum(w["kernel"].size for w in ws)
    assert wb >= 4 * nparams and wb < 4 * nparams * 1.2
    if splitk == "1":
        # fused combine: partial tiles in the accumulator-native layout, 85 x 2 tiles of 128 x 512
        # (conv6/conv7 at M = 64*169 = 10,816), + one ticket per tile (170 -> 192 words)
        slab = 85 * 2 * 128 * 512 * 3 * 4 + 192 * 4
    else:
        slab = 3 * 64 * 13 * 13 * 1024 * 4  # split-K partials of conv5/conv6/conv7 (3 splits)
    if fuse == "0":
        # two activation buffers (conv0 output, 64x416x416x16) + the largest col buffer
        assert sb >= 2 * 64 * 416 * 416 * 16 * 4 + slab
    else:
        # pools fused into the convs, no col buffer: the largest activation is conv0's pooled output
        act2 = 2 * 64 * 208 * 208 * 16 * 4
        assert act2 + slab <= sb < act2 + slab + 4096
    lib = dnn_hip.mylib
    h = ctypes.c_void_p()
    assert lib.dnn_plan_create(64, 416, 416, 3, ctypes.byref(h)) == 0
    try:
        for e in entries:
            if isinstance(e, dnn_hip.ConvEntry):
                kh, kw, _, od = e.conv.kernel.shape
                assert lib.dnn_plan_add_conv(h, kh, kw, od, 1, 1, 1, None, None, None, None, None, 0.0, 1) == 0
            else:
                assert lib.dnn_plan_add_max_pool(h, 2, 2, e.pool.strides[1], e.pool.strides[2], 1) == 0
        b, oh, ow, oc = (ctypes.c_int() for _ in range(4))
        lib.dnn_plan_output_shape(h, ctypes.byref(b), ctypes.byref(oh), ctypes.byref(ow), ctypes.byref(oc))
        assert (b.value, oh.value, ow.value, oc.value) == (64, 13, 13, 125)
        nk = lib.dnn_plan_num_kernels(h)
        names, flops = [], 0.0
        for i in range(nk):
            nm = ctypes.create_string_buffer(64)
            fl, by = ctypes.c_double(), ctypes.c_double()
            assert lib.dnn_plan_kernel_info(h, i, nm, 64, ctypes.byref(fl), ctypes.byref(by)) == 0
            names.append(nm.value.decode())
            flops += fl.value
        assert flops == pytest.approx(64 * 6.971e9, rel=1e-3)
        # the 1x1 conv8 reads its input directly (no im2col)
        assert "conv8.im2col" not in names and "conv8.gemm" in names and "conv7.gemm" in names
        # conv5-7 (N >= 512, K >= 2048) run split-K = 3: combined inside the GEMM by the last
        # split of each tile, or (DNN_HIP_SPLITK_FUSED=0) by an ordered reduce kernel
        nred = 0 if splitk == "1" else 3
        assert sum(n.endswith(".reduce") for n in names) == nred
        if splitk == "0":
            assert "conv5.reduce" in names and "conv6.reduce" in names and "conv7.reduce" in names
        if fuse == "0":  # explicit im2col for every 3x3 conv, every pool separate
            assert len(names) == 23 + nred
            assert sum(n.endswith(".im2col") for n in names) == 8
            assert sum(n.startswith("pool") for n in names) == 6
        else:  # conv0 direct + pool, conv1 patch + pool, conv2-7 implicit GEMM (2-5 with the pool), pool5 (s1)
            want = ["conv0.direct", "conv1.patch", "conv2.gemm", "conv3.gemm", "conv4.gemm", "conv5.gemm",
                    "conv5.reduce", "pool5", "conv6.gemm", "conv6.reduce", "conv7.gemm", "conv7.reduce", "conv8.gemm"]
            assert names == [n for n in want if splitk == "0" or not n.endswith(".reduce")]
        buf = ctypes.create_string_buffer(8192)
        assert lib.dnn_plan_describe(h, buf, 8192) == 0
        desc = buf.value.decode()
        assert desc.count("\n") == len(names) - nred - (8 if fuse == "0" else 0)
        assert desc.count("splitK=3") == 3
        assert desc.count(" combine") == (3 if splitk == "1" else 0)
    finally:
        lib.dnn_plan_destroy(h)


def test_plan_x3_structure_host_only(monkeypatch):
    """Default fp32 batch plan: conv1-conv7 on the x3 conv (exact 3-way bf16 splits; conv1 on the
    16-channel kernel reading conv0's fp32 output, conv2 and conv3 on the 2-D tile kernel, N = 64 /
    128), conv1-conv4 with their 2x2 pools fused; conv5 (N = 512) on whole-image tiles over all of
    K with pool5 fused (x3_img; DNN_HIP_X3_IMG=0: 2 K slices whose partials pool5 combines); conv8
    (1x1) on the 1x1 x3 conv reading conv7's split planes; weights of those layers in 3 bf16
    pieces."""
    monkeypatch.delenv("DNN_HIP_X3", raising=False)
    monkeypatch.delenv("DNN_HIP_X3_TILE", raising=False)
    monkeypatch.delenv("DNN_HIP_X3_C16", raising=False)
    ws = synth.yolo_weights()
    g, _ = yolo_graph.build_graph(dnn_hip.DnnGraphBuilder, ws, in_shape=(64, 416, 416, 3))
    entries = dnn_hip.lower_graph(g)
    wb, sb = dnn_hip.Plan.memory(64, (416, 416, 3), entries)
    nparams = sum(w["kernel"].size for w in ws)
    x3params = 9 * (16 * 32 + 32 * 64 + 64 * 128 + 128 * 256 + 256 * 512 + 512 * 1024 + 1024 * 1024) + 1024 * 125
    assert wb >= 4 * nparams + 2 * x3params and wb < (4 * nparams + 2 * x3params) * 1.2
    act2 = 2 * 64 * 208 * 208 * 16 * 4
    # one zero-bordered split-plane region per producer: conv1 (pooled 104x104x32), conv2
    # (pooled 52x52x64), conv3 (pooled 26x26x128), conv4 (pooled 13x13x256), conv5 + pool5
    # (13x13x512), conv6 and conv7 (13x13x1024 each), 6 B per element; no split-K slab
    pad = sum(64 * 6 * (h + 2) ** 2 * c
              for h, c in ((104, 32), (52, 64), (26, 128), (13, 256), (13, 512), (13, 1024), (13, 1024)))
    assert act2 + pad <= sb < act2 + pad + 16384
    lines = _describe_yolo(64, False)
    conv = [ln for ln in lines if ln.startswith("conv")]
    assert [i for i, ln in enumerate(conv) if "patch_x3" in ln] == [1, 2, 3, 4, 6, 7]
    assert "mode=x3_img" in conv[5] and "+pool2x2s1" in conv[5], conv[5]
    assert "mode=x3_1x1" in conv[8]
    assert sum("splitK" in ln for ln in lines) == 0
    assert all("+pool2x2s2" in conv[i] for i in (1, 2, 3, 4))  # pools fused into the x3 convs
    assert sum(ln.startswith("pool") for ln in lines) == 0  # pool5 fused into conv5
    # DNN_HIP_X3_IMG=0: conv5 in 2 K slices of the wide kernel, pool5 combining their partials
    monkeypatch.setenv("DNN_HIP_X3_IMG", "0")
    wb0, sb0 = dnn_hip.Plan.memory(64, (416, 416, 3), entries)
    slab = 2 * 64 * 13 * 13 * 512 * 4  # conv5's two raw K-slice partials
    assert act2 + pad + slab <= sb0 < act2 + pad + slab + 16384
    lines0 = _describe_yolo(64, False)
    conv0 = [ln for ln in lines0 if ln.startswith("conv")]
    assert "splitK=2 x3-combine" in conv0[5] and sum("splitK" in ln for ln in lines0) == 1
    assert sum(ln.startswith("pool") for ln in lines0) == 1  # pool5 (s1, combines conv5's slices)
    monkeypatch.delenv("DNN_HIP_X3_IMG")
    # latency plans (one frame): conv1 / conv2 on the narrow x3 kernels (small tiles), conv3-conv5
    # and conv8 on the K-split x3 kernels (pool5 fused into conv5), conv6 / conv7 on the small-M
    # x3 kernel; conv0 stays on its fp32 direct kernel
    latl = _describe_yolo(1, True)
    lat = [ln for ln in latl if ln.startswith("conv")]
    assert [i for i, ln in enumerate(lat) if "mode=patch_x3" in ln] == [1, 2]
    assert [i for i, ln in enumerate(lat) if "mode=x3_ktile" in ln] == [3, 4, 5, 8]
    assert [i for i, ln in enumerate(lat) if "mode=x3_lat" in ln] == [6, 7]
    assert "+pool2x2s1" in lat[5] and not any(ln.startswith("pool") for ln in latl)
    # DNN_HIP_X3_TILE=0: conv2/conv3 back on the fp32 MFMA, conv3's pooled epilogue splits;
    # DNN_HIP_X3_C16=0: conv1 on the fp32 patch kernel (its pooled epilogue splits for conv2)
    monkeypatch.setenv("DNN_HIP_X3_TILE", "0")
    conv = [ln for ln in _describe_yolo(64, False) if ln.startswith("conv")]
    assert [i for i, ln in enumerate(conv) if "patch_x3" in ln] == [1, 4, 6, 7] and "mode=x3_img" in conv[5]
    monkeypatch.setenv("DNN_HIP_X3_TILE", "1")
    monkeypatch.setenv("DNN_HIP_X3_C16", "0")
    conv = [ln for ln in _describe_yolo(64, False) if ln.startswith("conv")]
    assert [i for i, ln in enumerate(conv) if "patch_x3" in ln] == [2, 3, 4, 6, 7] and "mode=patch " in conv[1] + " "


def test_plan_errors_are_reported():
    lib = dnn_hip.mylib
    h = ctypes.c_void_p()
    assert lib.dnn_plan_create(1, 4, 4, 3, ctypes.byref(h)) == 0
    try:
        rc = lib.dnn_plan_add_conv(h, 5, 5, 8, 1, 1, 0, None, None, None, None, None, 0.0, 0)  # VALID 5x5 on 4x4
        assert rc != 0 and "empty output" in dnn_hip.last_error()
        rc = lib.dnn_plan_add_conv(h, 3, 3, 8, 1, 1, 1, None, None, ctypes.c_void_p(1), None, None, 0.0, 0)
        assert rc != 0 and "mean/var/gamma" in dnn_hip.last_error()
        assert lib.dnn_plan_run(h, 1, None, None, None) != 0  # not finalized
    finally:
        lib.dnn_plan_destroy(h)
    assert lib.dnn_plan_create(-1, 4, 4, 3, ctypes.byref(h)) != 0
    # a batch whose activation region reaches 2 GiB (the fused kernels' 32-bit store offsets) is
    # refused at finalize, before any device call
    assert lib.dnn_plan_create(2048, 416, 416, 3, ctypes.byref(h)) == 0
    try:
        assert lib.dnn_plan_add_conv(h, 3, 3, 16, 1, 1, 1, None, None, None, None, None, 0.0, 1) == 0
        assert lib.dnn_plan_finalize(h, 0, None, None) != 0 and "2 GiB" in dnn_hip.last_error()
    finally:
        lib.dnn_plan_destroy(h)


def test_postprocess_api_host_checks():
    import yolo_post
    assert ctypes.sizeof(yolo_post.Detection) == 40
    assert "dnn_yolo_postprocess" in declared_functions("dnn_hip_post.h")
    with pytest.raises(ValueError):
        yolo_post.postprocessing(np.zeros((13, 13, 124), np.float32))
    with pytest.raises(ValueError):
        yolo_post.detect_batch(np.zeros((2, 13, 13, 120), np.float32))
    # argument validation happens before any GPU call
    assert dnn_hip.mylib.dnn_yolo_postprocess_host(None, -1, None, 0, None) != 0
    assert "bad arguments" in dnn_hip.last_error()


def test_weight_pickle_round_trip_and_safety(tmp_path):
    import pickle
    import yolo_weights as YW
    ws = synth.yolo_weights()
    p = tmp_path / "y2t_weights.pickle"
    YW.save_y2t_weights(ws, p)
    back = YW.load_y2t_weights(p)
    assert len(back) == 9
    for a, b in zip(ws, back):
        for k in a:
            assert b[k].dtype == np.float32 and np.array_equal(a[k], b[k])
    # protocol 0 / 4 writers and float64 arrays load too (converted to fp32)
    for proto in (0, 4):
        q = tmp_path / f"w{proto}.pickle"
        with open(q, "wb") as f:
            pickle.dump([{k: v.astype(np.float64) for k, v in d.items()} for d in ws], f, protocol=proto)
        assert all(np.array_equal(x["kernel"], y["kernel"]) for x, y in zip(ws, YW.load_y2t_weights(q)))

    # a pickle that would run code is refused before anything executes
    class Evil(object):
        def __reduce__(self):
            return (os.system, ("touch " + str(tmp_path / "pwned"),))
    e = tmp_path / "evil.pickle"
    with open(e, "wb") as f:
        pickle.dump([Evil()], f, protocol=2)
    with pytest.raises(YW.WeightFileError):
        YW.load_y2t_weights(e)
    assert not (tmp_path / "pwned").exists()
    # structure checks
    with pytest.raises(YW.WeightFileError):
        YW.validate(ws[:8])
    bad = [dict(d) for d in ws]
    bad[3] = dict(bad[3], kernel=np.zeros((3, 3, 7, 256), np.float32))
    with pytest.raises(YW.WeightFileError):
        YW.validate(bad)
    bad = [dict(d) for d in ws]
    del bad[2]["gamma"]
    with pytest.raises(YW.WeightFileError):
        YW.validate(bad)


def _describe_yolo(batch, latency, env=None):
    """Plan layout of YOLOv2-tiny at `batch` (shapes only, no GPU): describe() lines."""
    import synth
    import yolo_graph
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        g, _ = yolo_graph.build_graph(dnn_hip.DnnGraphBuilder, synth.yolo_zero_weights(),
                                      in_shape=(batch, 416, 416, 3))
        lib = dnn_hip.mylib
        h = ctypes.c_void_p()
        assert lib.dnn_plan_create(batch, 416, 416, 3, ctypes.byref(h)) == 0
        try:
            assert lib.dnn_plan_set_latency_mode(h, 1 if latency else 0) == 0
            for e in dnn_hip.lower_graph(g):
                if isinstance(e, dnn_hip.ConvEntry):
                    kh, kw, _, od = e.conv.kernel.shape
                    assert lib.dnn_plan_add_conv(h, kh, kw, od, 1, 1, 1, None, None, None, None, None, 0.0, 1) == 0
                else:
                    assert lib.dnn_plan_add_max_pool(h, 2, 2, e.pool.strides[1], e.pool.strides[2], 1) == 0
            buf = ctypes.create_string_buffer(8192)
            assert lib.dnn_plan_describe(h, buf, 8192) == 0
            return buf.value.decode().splitlines()
        finally:
            lib.dnn_plan_destroy(h)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_latency_plan_layout():
    """dnn_plan_set_latency_mode: at batch 1 conv1 / conv2 on the narrow x3 kernels (small tiles
    chosen at launch), conv3-conv5 on the x3 kernel with the K split inside the workgroup (conv3 /
    conv4 with their 2x2/s2 pools, conv5 with pool5), conv6/conv7 on the small-M x3 kernel, conv8 on the
    1x1 K-split kernel, conv0 on its direct kernel; batch plans are unchanged."""
    lat = _describe_yolo(1, True)
    base = _describe_yolo(1, False)
    assert all(l.endswith(" latency") for l in lat if l.startswith("conv"))
    conv = [l for l in lat if l.startswith("conv")]
    assert "mode=direct" in conv[0] and all("mode=patch_x3" in conv[i] for i in (1, 2))
    for i in (3, 4, 5):
        assert "mode=x3_ktile" in conv[i] and " splitK=" not in conv[i], conv[i]
    assert "+pool2x2s2" in conv[4] and "+pool2x2s1" in conv[5]
    # conv6 / conv7: the small-M x3 kernel in 16 K slices; conv8 the 1x1 K-split kernel
    for i in (6, 7):
        assert "mode=x3_lat" in conv[i] and " splitK=16 x3-combine latency" in conv[i], conv[i]
    assert "mode=x3_ktile" in conv[8] and " splitK=" not in conv[8], conv[8]
    # the batch plan at batch 1: conv1-conv7 on the x3 conv (conv5 + pool5 on whole-image tiles, as
    # at batch 64), no K split
    assert not any(" splitK=" in l for l in base) and sum("patch_x3" in l for l in base) == 6 and \
        sum("mode=x3_img" in l for l in base) == 1
    assert sum(" splitK=16 " in l for l in conv) == 2  # conv6/conv7 at batch 1: 48 tiles x 16
    # batch 64: latency mode leaves the (N, K)-only rule in charge of every layer that fills the chip
    assert [l.replace(" latency", "") for l in _describe_yolo(64, True)] == _describe_yolo(64, False)
    # without the in-GEMM combine (DNN_HIP_SPLITK_FUSED=0) latency mode adds no split
    assert [l.replace(" latency", "") for l in _describe_yolo(1, True, {"DNN_HIP_SPLITK_FUSED": "0"})] == \
        _describe_yolo(1, False, {"DNN_HIP_SPLITK_FUSED": "0"})


def test_latency_mode_errors():
    lib = dnn_hip.mylib
    h = ctypes.c_void_p()
    assert lib.dnn_plan_create(1, 8, 8, 32, ctypes.byref(h)) == 0
    try:
        assert lib.dnn_plan_set_latency_mode(h, 2) != 0
        assert lib.dnn_plan_set_precision(h, 1) == 0
        assert lib.dnn_plan_set_latency_mode(h, 1) != 0  # fp32 plans only
        assert lib.dnn_plan_set_precision(h, 0) == 0
        assert lib.dnn_plan_add_conv(h, 3, 3, 64, 1, 1, 1, None, None, None, None, None, 0.0, 1) == 0
        assert lib.dnn_plan_set_latency_mode(h, 1) != 0  # after a layer
    finally:
        lib.dnn_plan_destroy(h)


def test_latency_env_default_only_for_fp32(monkeypatch):
    """$DNN_HIP_LATENCY=1 turns latency plans on for fp32 engines only (fp16 plans
    have none); an explicit latency argument wins."""
    g = dnn_hip.DnnGraphBuilder()
    g.set_out_node(g.create_input([1, 4, 4, 8]))
    monkeypatch.setenv("DNN_HIP_LATENCY", "1")
    assert dnn_hip.DnnInferenceEngine(g, False).latency
    assert not dnn_hip.DnnInferenceEngine(g, False, precision="fp16").latency
    assert not dnn_hip.DnnInferenceEngine(g, False, latency=False).latency
    monkeypatch.setenv("DNN_HIP_LATENCY", "0")
    assert not dnn_hip.DnnInferenceEngine(g, False).latency


@pytest.mark.parametrize("c_mid,want_x3", [(384, False), (512, True), (640, False), (1024, True)])
def test_latency_1x1_ktile_only_for_launchable_widths(c_mid, want_x3):
    """a latency plan's 1x1 head after an x3 conv takes the K-split x3 kernel only for
    the widths its launcher instantiates (K / 128 = 1, 2, 4, 8 chunk quads); other widths (C = 384
    after a kind-2 tile conv, 640, ...) stay on the fp32 GEMM instead of failing at run time."""
    lib = dnn_hip.mylib
    h = ctypes.c_void_p()
    assert lib.dnn_plan_create(1, 13, 13, 256, ctypes.byref(h)) == 0
    try:
        assert lib.dnn_plan_set_latency_mode(h, 1) == 0
        assert lib.dnn_plan_add_max_pool(h, 2, 2, 1, 1, 1) == 0  # split-plane producer of the 3x3 conv
        assert lib.dnn_plan_add_conv(h, 3, 3, c_mid, 1, 1, 1, None, None, None, None, None, 0.0, 1) == 0
        assert lib.dnn_plan_add_conv(h, 1, 1, 125, 1, 1, 1, None, None, None, None, None, 0.0, 0) == 0
        buf = ctypes.create_string_buffer(4096)
        assert lib.dnn_plan_describe(h, buf, 4096) == 0
        conv = [ln for ln in buf.value.decode().splitlines() if ln.startswith("conv")]
        assert "mode=patch_x3" in conv[0] or "mode=x3_" in conv[0], conv
        assert ("mode=x3_ktile" in conv[1]) == want_x3, conv
        if not want_x3:
            assert "mode=direct_a" in conv[1], conv
    finally:
        lib.dnn_plan_destroy(h)


@pytest.mark.parametrize("hw,want_patch", [((64, 3), False), ((64, 2), False), ((64, 4), True), ((13, 13), True)])
def test_fp16_patch_kernel_only_where_its_patch_fits(hw, want_patch):
    """the fp16 patch kernel's row-skewed LDS patch holds span * 10 + 12 (span / Wp + 2)
    16-B units; narrow frames whose tiles span more (W = 3: 306 rows, 3,816 units) or more than
    its 320 rows (W = 2) stay on the fp16 implicit GEMM instead of failing at launch."""
    H, W = hw
    lib = dnn_hip.mylib
    h = ctypes.c_void_p()
    assert lib.dnn_plan_create(2, H, W, 64, ctypes.byref(h)) == 0
    try:
        assert lib.dnn_plan_set_precision(h, 1) == 0
        assert lib.dnn_plan_add_max_pool(h, 2, 2, 1, 1, 1) == 0  # a pool producer (zero-bordered output)
        assert lib.dnn_plan_add_conv(h, 3, 3, 256, 1, 1, 1, None, None, None, None, None, 0.0, 1) == 0
        buf = ctypes.create_string_buffer(4096)
        assert lib.dnn_plan_describe(h, buf, 4096) == 0
        conv = [ln for ln in buf.value.decode().splitlines() if ln.startswith("conv")]
        assert ("mode=patch16" in conv[0]) == want_patch, conv
    finally:
        lib.dnn_plan_destroy(h)


def test_sclk_from_stamps_host_only():
    """The bench's shader-clock arithmetic (dnn_hip.sclk_from_stamps): per XCD the medians of the
    two counters over its workgroups, d(memtime) / d(memrealtime) x 100 MHz; XCDs present in only
    one of the two stamp sets are left out."""
    nwg = 64
    start = np.zeros((nwg, 4), dtype=np.int64)
    end = np.zeros((nwg, 4), dtype=np.int64)
    for w in range(nwg):
        x = w % 8
        ghz = 1.8 + 0.05 * x
        start[w] = [1_000_000 + 37 * w, 500_000 + w, x, 0]
        end[w] = [start[w, 0] + int(round(ghz * 1e4)), start[w, 1] + 1000, x, 0]  # 10 us at 100 MHz
    c = dnn_hip.sclk_from_stamps(start, end)
    assert set(c["per_xcd"]) == set(range(8))
    for x in range(8):
        assert abs(c["per_xcd"][x] - (1.8 + 0.05 * x)) < 1e-9
    assert abs(c["min"] - 1.8) < 1e-9 and abs(c["max"] - 2.15) < 1e-9
    assert abs(c["window_us"] - 10.0) < 1e-9
    end[:, 2] = 9  # no XCD in common
    assert dnn_hip.sclk_from_stamps(start, end) is None
