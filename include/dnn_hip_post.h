/* dnn_hip_post.h — on-GPU YOLOv2 postprocessing (decode, score threshold, sort, greedy NMS)
 * exported by both libdnn_hip.so and libdnn_hip_avx.so.
 *
 * Replaces the host-side `postprocessing(predictions)` of the reference
 * (cs492-projects/proj3/yolov2tiny.py:94-234, with iou :179-195 and
 * non_maximal_suppression :197-226), which runs after DnnInferenceEngine.run() on the
 * [1,13,13,125] output.  The Python mirror keeps that name and return value
 * (dnn-inference-engine_amd/yolo_post.py); this C-ABI is what it binds, and what a
 * multi-GPU caller uses to gather detections instead of whole output tensors.
 *
 * Semantics (oracle/post_numpy.py restates them; tests/golden/post_golden.json pins them):
 * per image, all 13*13*5 boxes decoded in (row, col, anchor) order in fp32, kept when
 * conf * p(best class) > 0.3f, sorted by score descending (ties: lower box index first,
 * = Python's stable sort), then greedy NMS at IoU > 0.3 against every kept box.  Corners are
 * the truncated int() of fp32 values; IoU uses exact integer areas (+1 widths, no clamp).
 *
 * Error channel: int return (0 ok, < 0 error, message from dnn_last_error()).
 * Per image, counts[i] = number of detections (only the first max_det are written), or
 *   -1 when a box corner is not finite or beyond +-2^61 (the reference's int() raises), or
 *   -2 when an evaluated IoU has a zero denominator (the reference raises ZeroDivisionError;
 *      possible because its overlaps are not clamped).
 */
#ifndef DNN_HIP_POST_H
#define DNN_HIP_POST_H

#ifdef __cplusplus
extern "C" {
#endif

#pragma GCC visibility push(default)

/* one detection, 40 bytes: class index into the 20 VOC names, fp32 score, corners */
typedef struct dnn_detection {
  int cls;
  float score;
  long long left, top, right, bottom;
} dnn_detection;

#define DNN_YOLO_BOXES 845 /* 13 * 13 * 5: no image can have more detections */

/* Device pointers, asynchronous on `stream` (hipStream_t, NULL = default stream).
 * pred: [n_images][13][13][125] fp32; dets: [n_images][max_det]; counts: [n_images]. */
int dnn_yolo_postprocess(const float* pred, int n_images, dnn_detection* dets, int max_det, int* counts,
                         void* stream);

/* Device pointers, asynchronous: image-major compaction of the per-image lists written by
 * dnn_yolo_postprocess, packed = dets[0][:counts[0]] ++ dets[1][:counts[1]] ++ ... (images
 * with an error code contribute nothing; counts are clamped to max_det), total[0] = rows.
 * packed needs room for n_images * max_det rows.  Used before a multi-GPU gather so only
 * the detections travel. */
int dnn_yolo_pack_detections(const dnn_detection* dets, const int* counts, int n_images, int max_det,
                             dnn_detection* packed, int* total, void* stream);

/* Host pointers, synchronous (copies in, runs, copies out). */
int dnn_yolo_postprocess_host(const float* pred, int n_images, dnn_detection* dets, int max_det, int* counts);

#pragma GCC visibility pop

#ifdef __cplusplus
}
#endif

#endif /* DNN_HIP_POST_H */
