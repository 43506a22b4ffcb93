/* dnn_hip_plan.h — device-resident, fused execution plan for the YOLOv2-tiny Conv2D path.
 *
 * The reference has no plan object: `DnnInferenceEngine.run` (proj3/dnn_openblas.py:29-57)
 * walks the networkx graph and calls one host-pointer C function per node
 * (conv2d_mul / bias_add / batch_norm / leaky_relu / max_pool2d, dnn_openblas.c).  The
 * plan is the device-resident lowering of that same node chain: each
 * Conv2D -> BiasAdd -> BatchNorm -> LeakyReLU run becomes ONE conv entry (im2col + fp32
 * MFMA GEMM with the three element-wise ops as its epilogue, evaluated in the reference's
 * operation order), each MaxPool2D one pool entry, and activations never leave HBM.
 * It is what `dnn_hip.DnnInferenceEngine.run` (the Python mirror of dnn_openblas.py)
 * lowers the graph to.
 *
 * Conventions: plain C ABI, cdecl, no torch types.  All tensors NHWC fp32 contiguous,
 * conv kernels HWIO (the pickle layout of proj3/yolov2tiny.py:30-77).  Functions return
 * 0 on success and a negative code on error; dnn_last_error() describes the last error
 * of the calling thread.  Padding: 0 = VALID, 1 = SAME with TF semantics
 * (get_out_pads, proj3/dnn_openblas.py:127-142).
 */
#ifndef DNN_HIP_PLAN_H
#define DNN_HIP_PLAN_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif
#pragma GCC visibility push(default)

typedef struct dnn_plan dnn_plan;

/* Last error message of the calling thread ("" if none). */
const char* dnn_last_error(void);

/* First 16 hex digits of the SHA-256 of the sources this library was built from
 * (csrc/Makefile SRCS); tests/conftest.py refuses a library whose id does not match. */
const char* dnn_build_id(void);

/* Create an empty plan for inputs [batch, in_h, in_w, in_c]. */
int dnn_plan_create(int batch, int in_h, int in_w, int in_c, dnn_plan** out);
void dnn_plan_destroy(dnn_plan* plan);

/* Precision of the plan (call before adding layers): 0 = fp32 everywhere (default, the
 * reference's arithmetic); 1 = fp16 conv path (BASELINE config 5): fp16 activations and
 * weights, v_mfma_f32_32x32x16_f16 with fp32 accumulation and fp32 epilogue, fp32 frames in
 * and fp32 predictions out.  fp16 plans need C % 8 == 0 for every conv except a <= 4-channel
 * 3x3 first conv followed by a 2x2/s2 pool; tolerance vs fp32: DESIGN.md. */
int dnn_plan_set_precision(dnn_plan* plan, int precision);

/* Latency mode (call before adding layers; fp32 plans): on = 1 lets the K split of a GEMM
 * layer depend on M, so a small-M forward (one frame: BASELINE config 2, the single timed
 * frame of proj3/__init__.py:24-26) spreads conv4-conv8 over the whole chip (2..16 K splits,
 * combined in split order inside the GEMM).  Outputs stay within the fp32 tolerance of the
 * reference but are no longer bit-equal to the same frame's row of a batch plan (whose
 * summation order depends on (N, K) only).  Default 0. */
int dnn_plan_set_latency_mode(dnn_plan* plan, int on);

/* Append a Conv2D (proj3/dnn_openblas.py:144-188) with its trailing BiasAdd / BatchNorm /
 * LeakyReLU fused.  kernel: [kh][kw][in_c][od] HWIO.  biases may be NULL (no BiasAdd);
 * mean/var/gamma all NULL means no BatchNorm (else all three, eps as in
 * proj3/dnn_openblas.py:263-270); leaky: 0 none, 1 = dnn_openblas.c leaky_relu
 * (t<0 ? 0.1*t in double : t), 2 = dnn_avx.c leaky_relu (max(t, 0.1f*t)).
 * Host weight pointers are copied; pass kernel == NULL to declare the layer's shape only
 * (weights then arrive through dnn_plan_weight_buffer, e.g. an RCCL broadcast). */
int dnn_plan_add_conv(dnn_plan* plan, int kh, int kw, int od, int stride_h, int stride_w, int padding,
                      const float* kernel, const float* biases, const float* mean, const float* var,
                      const float* gamma, float eps, int leaky);

/* Append a MaxPool2D (proj3/dnn_openblas.py:213-242). */
int dnn_plan_add_max_pool(dnn_plan* plan, int kh, int kw, int stride_h, int stride_w, int padding);

/* Output shape of the plan so far (per image, plus the planned batch). */
int dnn_plan_output_shape(const dnn_plan* plan, int* batch, int* h, int* w, int* c);

/* Human-readable lowering, one line per plan entry: shapes, execution mode (gemm =
 * explicit im2col + GEMM, direct_a = 1x1 GEMM on the input, implicit = implicit GEMM,
 * direct = direct conv, patch = LDS-patch MFMA conv), GEMM config, whether a 2x2/s2 max
 * pool is fused and whether the GEMM is split along K (splitK=3: partials + an ordered
 * reduce/epilogue kernel).  A 2x2/s2 MaxPool2D directly after an implicit, patch or direct
 * conv is folded into it; set DNN_HIP_FUSE=0 in the environment before dnn_plan_create to
 * keep every conv explicit and every pool separate (DNN_HIP_PATCH=0: no patch mode). */
int dnn_plan_describe(const dnn_plan* plan, char* buf, int buf_len);

/* Device bytes the plan needs: packed weights + epilogue params, and workspace
 * (two activation buffers + the im2col buffer) for the planned batch. */
int dnn_plan_memory(const dnn_plan* plan, size_t* weight_bytes, size_t* workspace_bytes);

/* Bind device memory and upload weights.  weights / workspace may be NULL, in which case
 * the plan hipMallocs its own.  If every conv was added with host weights they are packed
 * into the weight buffer here (hipMemcpy + pack kernel, synchronous). */
int dnn_plan_finalize(dnn_plan* plan, int device, void* weights, void* workspace);

/* Device pointer and size of the packed weight buffer (for a broadcast from rank 0). */
int dnn_plan_weight_buffer(const dnn_plan* plan, void** ptr, size_t* bytes);

/* Run n <= batch images: d_in [n,in_h,in_w,in_c] -> d_out [n,oh,ow,oc], both device
 * pointers, asynchronously on `stream` (a hipStream_t; NULL = default stream). */
int dnn_plan_run(dnn_plan* plan, int n, const float* d_in, float* d_out, void* stream);

/* Host-pointer convenience: H2D copy, run, D2H copy, synchronise. */
int dnn_plan_run_host(dnn_plan* plan, int n, const float* h_in, float* h_out);

/* dnn_plan_run through a HIP graph: the first call for a given (n, d_in, d_out) captures the
 * plan's kernel sequence on `stream` (hipStreamBeginCapture) and instantiates it; every call
 * then submits the whole forward with one hipGraphLaunch — the launch-bound batch-1 case.
 * A different (n, d_in, d_out) re-captures.  `stream` must be a created stream (the NULL
 * stream cannot be captured); per-kernel timing must be off. */
int dnn_plan_run_graph(dnn_plan* plan, int n, const float* d_in, float* d_out, void* stream);

/* Per-kernel timing with HIP events recorded on the run stream.
 * begin: allocate events for up to max_runs runs and start recording;
 * end: synchronise, write per-kernel summed milliseconds and launch counts (arrays of
 * dnn_plan_num_kernels() entries), stop recording. */
int dnn_plan_num_kernels(const dnn_plan* plan);
int dnn_plan_kernel_info(const dnn_plan* plan, int idx, char* name, int name_len, double* flops,
                         double* bytes);
int dnn_plan_timing_begin(dnn_plan* plan, int max_runs);
/* As dnn_plan_timing_begin, but events are recorded only around kernel `kernel_idx` (two per
 * forward instead of one per kernel: no event packets between the other kernels); the other
 * kernels report 0 launches at dnn_plan_timing_end. */
int dnn_plan_timing_begin_only(dnn_plan* plan, int max_runs, int kernel_idx);
int dnn_plan_timing_end(dnn_plan* plan, double* ms_sum, long long* launches);

/* Shader-clock measurement (rooflines against the measured clock).
 * dnn_clock_stamp: launches `nwg` one-wave workgroups on `stream`; workgroup w stores four
 * uint64 at dev_out[4 w ..]: s_memtime (shader clock counter), s_memrealtime (100 MHz), XCC_ID,
 * HW_ID.  Two stamps bracketing a region give, per XCD, the mean shader clock over it:
 * d(memtime) / d(memrealtime) x 100 MHz.
 * dnn_plan_clock_begin: the next runs (up to max_runs) bracket kernel `kernel_idx` with two such
 * launches each — run r's opening stamps at dev_buf[8 r nwg], closing ones at [(8 r + 4) nwg];
 * dev_buf holds max_runs x 8 x nwg uint64.  The stamps sit outside the kernel's HIP-event window.
 * dnn_plan_clock_end: stops stamping and returns the number of stamped runs. */
int dnn_clock_stamp(void* stream, unsigned long long* dev_out, int nwg);
int dnn_plan_clock_begin(dnn_plan* plan, int kernel_idx, unsigned long long* dev_buf, int max_runs, int nwg);
int dnn_plan_clock_end(dnn_plan* plan, int* runs);

/* Mark inside a run (scheduling other streams' work beside a forward's later layers).
 * dnn_plan_set_mark: from now on every run records an event on its stream right before kernel
 * `kernel_idx` (-1: off; not with dnn_plan_run_graph).
 * dnn_plan_wait_mark: makes `stream` wait for the mark of the most recent run enqueued (the
 * usual stream-wait-event semantics: a later run's mark does not affect an earlier wait). */
int dnn_plan_set_mark(dnn_plan* plan, int kernel_idx);
int dnn_plan_wait_mark(dnn_plan* plan, void* stream);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif
