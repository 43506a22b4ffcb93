"""Frame ingest: host uint8 BGR frames -> the engine's fp32 NHWC input on the GPU
(the reference's `resize_input`, cs492-projects/proj3/__init__.py:8-12).

`resize_input_gpu(im)` is the drop-in for one frame (returns the numpy array the reference
returns).  `FrameIngest` is the batched pipeline: frames are copied into one of two pinned
host buffers, uploaded as 8-bit data on a copy stream (4x fewer PCIe bytes than fp32), then
resized / scaled / channel-flipped on the GPU (`dnn_preprocess_frames`,
include/dnn_hip_ingest.h) on the compute stream, so the upload of batch k+1 overlaps the
forward of batch k.  No CPU fallback: the library must be present.
"""
import ctypes

import numpy as np

import dnn_hip

_lib = dnn_hip.mylib
_lib.dnn_preprocess_frames.restype = ctypes.c_int
_lib.dnn_preprocess_frames.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_void_p]

IN_SIZE = 416


def preprocess_device(d_bgr_ptr, n, h, w, d_out_ptr, stream_ptr, out_hw=(IN_SIZE, IN_SIZE)):
    dnn_hip._check(_lib.dnn_preprocess_frames(d_bgr_ptr, int(n), int(h), int(w), d_out_ptr, int(out_hw[0]),
                                              int(out_hw[1]), stream_ptr), "dnn_preprocess_frames")


def resize_input_gpu(im, device=0):
    """__init__.py:8-12 for one HxWx3 uint8 BGR frame -> [416,416,3] fp32 RGB (numpy)."""
    import torch
    im = np.ascontiguousarray(im, dtype=np.uint8)
    if im.ndim != 3 or im.shape[2] != 3:
        raise ValueError(f"expected an HxWx3 uint8 BGR frame, got shape {im.shape}")
    dev = torch.device("cuda", device)
    src = torch.from_numpy(im).to(dev)
    out = torch.empty((IN_SIZE, IN_SIZE, 3), dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream(dev)
    preprocess_device(src.data_ptr(), 1, im.shape[0], im.shape[1], out.data_ptr(), s.cuda_stream)
    return out.cpu().numpy()


class FrameIngest(object):
    """Double-buffered uint8 upload + GPU preprocessing for batches of `batch` frames of
    h x w x 3 uint8 BGR.  submit(frames) returns the fp32 [n,416,416,3] device tensor for
    that batch; it is ready in stream order on `compute_stream`.

    Slot reuse is ordered without any call from the caller: before slot k is refilled,
      * the host waits until the previous upload out of pinned host[k] has completed
        (next_host_buffer / submit_host), so the CPU never rewrites a buffer the copy
        engine is still reading;
      * the copy stream waits for the previous preprocess that read dev_u8[k], so an upload
        never overwrites 8-bit frames that are still being resized;
      * the preprocess writing out[k] runs on the compute stream after everything enqueued
        there before it (the forward that read out[k] two batches ago).
    release(stream) is needed only when the returned tensor is consumed on ANOTHER stream:
    it records that consumption so the preprocess that next overwrites the slot waits for it."""

    def __init__(self, batch, h, w, device, compute_stream=None, out_hw=(IN_SIZE, IN_SIZE)):
        import torch
        self.torch = torch
        self.batch, self.h, self.w, self.out_hw = int(batch), int(h), int(w), tuple(out_hw)
        self.dev = torch.device(device) if not isinstance(device, torch.device) else device
        shape = (self.batch, self.h, self.w, 3)
        self.host = [torch.empty(shape, dtype=torch.uint8).pin_memory() for _ in range(2)]
        self.dev_u8 = [torch.empty(shape, dtype=torch.uint8, device=self.dev) for _ in range(2)]
        self.out = [torch.empty((self.batch,) + self.out_hw + (3,), dtype=torch.float32, device=self.dev)
                    for _ in range(2)]
        self.copy_stream = torch.cuda.Stream(self.dev)
        self.compute = compute_stream or torch.cuda.current_stream(self.dev)
        self.uploaded = [None, None]   # upload out of host[k] (copy stream)
        self.prepped = [None, None]    # preprocess that read dev_u8[k] (compute stream)
        self.consumed = [None, None]   # off-stream consumer of out[k] (release())
        self.slot = 0
        self.last = None

    def next_host_buffer(self):
        """The pinned uint8 [batch, h, w, 3] buffer the next submit_host() uploads: a frame
        decoder can write into it directly (no extra host copy).  Waits (host) until the
        previous upload out of that buffer has completed."""
        if self.uploaded[self.slot] is not None:
            self.uploaded[self.slot].synchronize()
        return self.host[self.slot]

    def submit(self, frames):
        """frames: [n, h, w, 3] uint8 BGR (numpy), n <= batch: copied into the next pinned
        slot, then submit_host(n)."""
        f = np.asarray(frames, dtype=np.uint8)
        n = f.shape[0]
        if n > self.batch or f.shape[1:] != (self.h, self.w, 3):
            raise ValueError(f"frames of shape {f.shape} do not fit [{self.batch},{self.h},{self.w},3]")
        self.next_host_buffer()[:n].numpy()[...] = f
        return self.submit_host(n)

    def submit_host(self, n):
        """Upload the first n frames of the current pinned slot and preprocess them."""
        torch = self.torch
        if not 0 <= n <= self.batch:  # (before the slot flips: a rejected call changes nothing)
            raise ValueError(f"n={n} outside [0, {self.batch}]")
        k = self.slot
        self.slot ^= 1
        up = torch.cuda.Event()
        with torch.cuda.stream(self.copy_stream):
            if self.prepped[k] is not None:
                self.copy_stream.wait_event(self.prepped[k])  # dev_u8[k]'s last reader is done
            self.dev_u8[k][:n].copy_(self.host[k][:n], non_blocking=True)
            up.record(self.copy_stream)
        self.uploaded[k] = up
        self.compute.wait_event(up)
        if self.consumed[k] is not None:
            self.compute.wait_event(self.consumed[k])  # an off-stream reader of out[k]
            self.consumed[k] = None
        preprocess_device(self.dev_u8[k].data_ptr(), n, self.h, self.w, self.out[k].data_ptr(),
                          self.compute.cuda_stream, self.out_hw)
        pe = torch.cuda.Event()
        pe.record(self.compute)
        self.prepped[k] = pe
        self.last = k
        return self.out[k][:n]

    def release(self, stream=None):
        """The most recently returned batch is being read on `stream` (default: the compute
        stream, where nothing needs recording): call after that work has been enqueued, so
        the preprocess that reuses the slot waits for it.  Optional on the compute stream."""
        if self.last is None:
            return
        if stream is None or stream == self.compute:
            return
        e = self.torch.cuda.Event()
        e.record(stream)
        self.consumed[self.last] = e
