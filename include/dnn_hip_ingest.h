/* dnn_hip_ingest.h — frame preprocessing on the GPU, exported by both libraries.
 *
 * Replaces the host `resize_input(im)` of the reference driver
 * (cs492-projects/proj3/__init__.py:8-12: cv2.resize to 416x416, / 255., BGR -> RGB,
 * float32) for a batch of frames already on the device, so a caller uploads 8-bit frames
 * (0.52 MB for a 416x416 frame instead of 2.08 MB of fp32) and the engine reads the fp32
 * NHWC tensor the reference would have produced.  The Python pipeline with pinned host
 * buffers and copy/compute overlap is dnn-inference-engine_amd/ingest.py.
 *
 * Resize: OpenCV's scalar fixed-point INTER_LINEAR for 8-bit images restated (11-bit
 * coefficients, see csrc/ingest.hip); parity with cv2 itself is unpinned (cv2 is not
 * importable in the build image).  /255, the channel order and the fp32 rounding are exact.
 */
#ifndef DNN_HIP_INGEST_H
#define DNN_HIP_INGEST_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif
#pragma GCC visibility push(default)

/* d_bgr: [n][h][w][3] uint8 BGR (device); d_out: [n][out_h][out_w][3] fp32 RGB in [0, 1]
 * (device); asynchronous on `stream` (hipStream_t, NULL = default). */
int dnn_preprocess_frames(const uint8_t* d_bgr, int n, int h, int w, float* d_out, int out_h, int out_w,
                          void* stream);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif
