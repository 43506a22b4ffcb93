// Device-resident execution plan (include/dnn_hip_plan.h).
//
// The reference walks its graph node by node and round-trips every intermediate through
// host numpy arrays (proj3/dnn_openblas.py:29-57; each CUDA/cuBLAS call even mallocs and
// copies per image, dnn_cuda.cu:193-210).  Here the same node chain is lowered once to a
// list of device steps.  Each conv entry (Conv2D + its BiasAdd / BatchNorm / LeakyReLU as
// the GEMM epilogue) runs in one of four modes:
//   GEMM      explicit im2col into a col buffer + LDS-tiled fp32-MFMA GEMM (the reference's
//             im2col + sgemm structure, dnn_openblas.c:160-194; generic fallback)
//   DIRECT_A  1x1 / stride 1 / unpadded: the NHWC input IS the col matrix, GEMM only
//   IMPLICIT  implicit GEMM: the LDS-DMA loader gathers the im2col rows straight from the
//             input (per-lane source addresses), no col buffer
//   DIRECT    3x3 conv with <= 4 input channels (conv0): direct FMA conv, weights in LDS
//   PATCH     3x3 SAME conv with 16/32 input channels + 2x2 pool (conv1): input patch and
//             weights DMA'd to LDS once per tile, taps are constant LDS offsets (conv_patch.hip)
// and a following 2x2/stride-2 MaxPool2D is fused into the IMPLICIT / DIRECT epilogue
// (pool-window-major rows), otherwise it is its own pool entry.  Weights are packed once
// into a device arena as Bt[Npad][Kpad] (K order kh,kw,ic; HWIO as-is for DIRECT) plus four
// Npad-long epilogue vectors (bias, mean, sqrt(var+eps), gamma).  Activations ping-pong
// between two workspace buffers.  DNN_HIP_FUSE=0 in the environment at plan creation
// forces the explicit GEMM path with separate pools (for A/B checks); DNN_HIP_PATCH=0 keeps
// PATCH-eligible layers on the implicit GEMM.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include "dnn_common.h"
#include "../../include/dnn_hip_plan.h"

namespace dnnhip {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}
const char* last_error() { return g_last_error.c_str(); }

bool getenv_flag_off(const char* name) {
  const char* e = getenv(name);
  return e && e[0] == '0';
}

int device_cu_count() {
  // compute units of the current device (256 on MI355X), cached per device
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

void out_pads(int in, int k, int s, int same, int* out, int* pad_front) {
  // proj3/dnn_openblas.py:127-142 (TensorFlow SAME / VALID)
  if (same) {
    int o = (in + s - 1) / s;
    int pad = (o - 1) * s + k - in;
    if (pad < 0) pad = 0;
    *out = o;
    *pad_front = pad / 2;
  } else {
    int span = in - k + 1;
    *out = span > 0 ? (span + s - 1) / s : 0;
    *pad_front = 0;
  }
}

static size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

}  // namespace dnnhip

using namespace dnnhip;

// MODE_PATCH16: fp16 3x3 conv on a zero-bordered input (conv3x3_f16_acc_kernel; conv6/conv7)
// MODE_TILE16: fp16 3x3 conv + 2x2/s2 pool on 2-D tiles of a zero-bordered input
//   (conv3x3_f16_tile_kernel; conv2-conv4)
// MODE_X3: fp32 3x3 conv on the bf16 MFMA with exact 3-way splits, split zero-bordered input
// (conv3x3_x3_patch_kernel; conv6/conv7 of the fp32 path)
// MODE_X3_1X1: fp32 1x1 conv with the same arithmetic on its producer's split planes
// (conv1x1_x3_kernel; conv8 of the fp32 path)
enum ConvMode : int { MODE_GEMM = 0, MODE_DIRECT_A = 1, MODE_IMPLICIT = 2, MODE_DIRECT = 3, MODE_PATCH = 4,
                      MODE_PATCH16 = 5, MODE_X3 = 6, MODE_X3_1X1 = 7, MODE_TILE16 = 8 };
static const char* kModeName[] = {"gemm", "direct_a", "implicit", "direct", "patch", "patch16", "patch_x3", "x3_1x1",
                                  "tile16"};

struct PlanLayer {
  int type = 0;  // 0 conv, 1 pool
  // shapes (per image): input H,W,C -> conv/pool output OH,OW,OC (-> fused pool PH,PW)
  int H = 0, W = 0, C = 0, OH = 0, OW = 0, OC = 0;
  int kh = 0, kw = 0, sh = 1, sw = 1, pt = 0, pl = 0;
  // conv
  int mode = MODE_GEMM;
  int K = 0, Kpad = 0, Npad = 0, cfg = 0, epi_flags = 0;
  int splits = 1;  // split-K partial count (> 1: GEMM writes partials, a reduce kernel finishes)
  bool pool = false;  // a 2x2/stride-2 max pool fused into this conv
  bool x3lat = false;  // MODE_X3 on the small-M kernel (latency plans: launch_conv_x3_lat)
  bool x3k = false;    // MODE_X3 with the K split inside the workgroup (latency plans: launch_conv_x3_ktile)
  bool pool1 = false;  // x3k / x3img: a 2x2/stride-1 SAME pool fused (same output frame)
  bool x3img = false;  // MODE_X3 on whole-image tiles over all of K (launch_conv_x3_img), pool1 fused
  bool out_padded = false;  // output written zero-bordered (the next layer is MODE_PATCH16 / MODE_X3;
                            // fp32 plans: as x3 split planes)
  size_t pad_off = 0;       // its zero-bordered output region: float offset inside the pad area
  int PH = 0, PW = 0;
  size_t w_off = 0, epi_off = 0;  // float offsets in the weight arena
  bool have_host = false;
  std::vector<float> w, bias, mean, sq, gamma;
  int kernel_idx = 0;  // index of this layer's first kernel in the kernel list
  int out_h() const { return pool ? PH : OH; }
  int out_w() const { return pool ? PW : OW; }
};

struct KernelDesc {
  std::string name;
  int layer;
  int kind;             // 0 im2col, 1 gemm / conv, 2 pool
  double flops, bytes;  // algorithmic, full planned batch
};

struct dnn_plan {
  int batch = 0, in_h = 0, in_w = 0, in_c = 0;
  int cur_h = 0, cur_w = 0, cur_c = 0;
  bool fuse = true;
  bool patch = true;
  bool splitk_fused = true;  // fp32 split-K layers combine in the GEMM (no reduce kernel)
  int fp16 = 0;  // 1: fp16 activations/weights, fp16 MFMA, fp32 accumulate + epilogue
  bool direct_out = false;  // fp16: the last layer writes the fp32 output itself (fp16_direct_out)
  bool latency = false;  // split K by M too (dnn_plan_set_latency_mode): batch-1 latency plans
  std::vector<PlanLayer> layers;
  std::vector<KernelDesc> kernels;
  int device = -1;
  bool finalized = false;
  float* weights = nullptr;
  size_t weight_floats = 0;
  bool own_weights = false;
  float* ws = nullptr;
  size_t ws_floats = 0;
  bool own_ws = false;
  size_t act_floats = 0, col_floats = 0, slab_floats = 0, ticket_floats = 0, pad_floats = 0;
  static constexpr size_t kZeroFloats = 64;  // zero page: source of padding taps (implicit GEMM)
  // staging for dnn_plan_run_host
  float* h_in_dev = nullptr;
  size_t h_in_floats = 0;
  // timing
  bool timing = false;
  int ev_cap = 0, ev_used = 0;
  int timing_only = -1;  // >= 0: events only around that kernel (dnn_plan_timing_begin_only)
  std::vector<hipEvent_t> ev;
  std::vector<int> ev_kernel;
  // shader-clock stamps around one kernel (dnn_plan_clock_begin): run r's stamps of the opening
  // launch at clk_buf + 2 r nwg 4, of the closing launch 4 nwg further (clock.hip)
  int clk_kernel = -1, clk_cap = 0, clk_used = 0, clk_nwg = 0;
  // mark: an event recorded on the run stream right before kernel `mark_kernel` of every run
  // (dnn_plan_set_mark / dnn_plan_wait_mark)
  int mark_kernel = -1;
  hipEvent_t mark_ev = nullptr;
  bool clk_open = false;
  unsigned long long* clk_buf = nullptr;
  // captured forward (dnn_plan_run_graph)
  hipGraph_t graph = nullptr;
  hipGraphExec_t gexec = nullptr;
  int g_n = -1;
  const float* g_in = nullptr;
  float* g_out = nullptr;
};

static void drop_graph(dnn_plan* p) {
  if (p->gexec) (void)hipGraphExecDestroy(p->gexec);
  if (p->graph) (void)hipGraphDestroy(p->graph);
  p->gexec = nullptr;
  p->graph = nullptr;
  p->g_n = -1;
}

static bool fused_splitk(const dnn_plan* p) { return p->splitk_fused; }

// fp16 plans whose last layer is a dense GEMM the fp32-output launcher covers (conv8): it writes
// the plan's fp32 output itself, no output conversion kernel.  DNN_HIP_F16_DIRECT_OUT=0: off.
static bool fp16_direct_out(const dnn_plan* p) {
  if (!p->fp16 || p->layers.empty() || getenv_flag_off("DNN_HIP_F16_DIRECT_OUT")) return false;
  const PlanLayer& L = p->layers.back();
  return L.type == 0 && L.mode == MODE_DIRECT_A && gemm16_f32out_supported(L.splits, L.Npad) && !L.out_padded;
}

static void layout(dnn_plan* p) {
  p->direct_out = fp16_direct_out(p);
  size_t off = 0, act = (size_t)p->in_h * p->in_w * p->in_c, col = 0, slab = 0, slab_fused = 0, tickets = 0;
  int nconv = 0, npool = 0;  // kernel names use conv / pool ordinals: "conv7.gemm" is YOLO's conv7
  p->kernels.clear();
  const double B = p->batch;
  for (size_t i = 0; i < p->layers.size(); ++i) {
    PlanLayer& L = p->layers[i];
    act = std::max(act, (size_t)L.out_h() * L.out_w() * L.OC);
    const double M = B * L.OH * L.OW;
    const double in_b = 4.0 * B * L.H * L.W * L.C, out_b = 4.0 * B * L.out_h() * L.out_w() * L.OC;
    L.kernel_idx = (int)p->kernels.size();
    char nm[64];
    if (L.type == 0) {
      L.w_off = off;
      // fp16 GEMM layers hold Bt in halves (2 per float slot); conv0's direct kernel reads fp32
      const bool half_w = p->fp16 && L.mode != MODE_DIRECT;
      if (L.mode == MODE_X3 || L.mode == MODE_X3_1X1)  // three bf16 pieces per weight
        off = align_up(off + (size_t)L.Npad * L.Kpad * 3 / 2, 64);
      else
        off = align_up(off + ((size_t)L.Npad * L.Kpad + (half_w ? 1 : 0)) / (half_w ? 2 : 1), 64);
      L.epi_off = off;
      off = align_up(off + 4 * (size_t)L.Npad, 64);
      const double flops = 2.0 * M * L.OC * L.K, w_b = 4.0 * L.K * L.OC;
      if (L.mode == MODE_GEMM) {
        col = std::max(col, (size_t)L.OH * L.OW * L.Kpad);
        snprintf(nm, sizeof(nm), "conv%d.im2col", nconv);
        // algorithmic bytes: col written once + input read once
        p->kernels.push_back({nm, (int)i, 0, 0.0, 4.0 * M * L.K + in_b});
        snprintf(nm, sizeof(nm), "conv%d.gemm", nconv++);
        p->kernels.push_back({nm, (int)i, 1, flops, 4.0 * M * L.K + w_b + out_b});
      } else if (L.mode == MODE_DIRECT || L.mode == MODE_PATCH) {
        snprintf(nm, sizeof(nm), L.mode == MODE_DIRECT ? "conv%d.direct" : "conv%d.patch", nconv++);
        p->kernels.push_back({nm, (int)i, 1, flops, in_b + w_b + out_b});
      } else {  // DIRECT_A reads the input as A; IMPLICIT reads it once per tap in the ideal
        snprintf(nm, sizeof(nm), "conv%d.gemm", nconv);
        p->kernels.push_back({nm, (int)i, 1, flops, in_b + w_b + out_b});
        ++nconv;
      }
      if (L.mode == MODE_X3 && L.splits > 1) {  // raw partials; combined by the next pool, or:
        slab = std::max(slab, (size_t)L.splits * L.OH * L.OW * L.OC);
        const bool pool_next = i + 1 < p->layers.size() && p->layers[i + 1].type == 1;
        if (!pool_next) {
          snprintf(nm, sizeof(nm), "conv%d.combine", nconv - 1);
          p->kernels.push_back({nm, (int)i, 3, (L.splits - 1) * M * L.OC, 4.0 * (L.splits + 1) * M * L.OC});
        }
      }
      if (L.mode == MODE_X3) {
        // (split-K partials: below)
      } else if (L.splits > 1 && fused_splitk(p)) {  // partials combined by the GEMM's last-arriving split
        const long long Mg = L.pool ? 4LL * p->batch * L.PH * L.PW : (long long)M;  // the GEMM's rows
        slab_fused = std::max(slab_fused, (size_t)(p->fp16 ? splitk16_fused_slab_floats(L.cfg, Mg, L.OC, L.splits)
                                                           : splitk_fused_slab_floats(L.cfg, Mg, L.OC, L.splits)));
        tickets = std::max(tickets, (size_t)(p->fp16 ? splitk16_tiles(L.cfg, Mg, L.OC)
                                                     : splitk_tiles(L.cfg, Mg, L.OC)));
        if (p->fp16 && L.cfg == GEMM16_128x512_W16)  // the launcher's 128x128 fallback has more tiles
          tickets = std::max(tickets, (size_t)splitk16_tiles(GEMM16_128x128, (long long)M, L.OC));
      } else if (L.splits > 1) {  // partials written by the GEMM, summed + epilogue by the reduce kernel
        slab = std::max(slab, (size_t)L.splits * L.OH * L.OW * L.OC);
        snprintf(nm, sizeof(nm), "conv%d.reduce", nconv - 1);
        p->kernels.push_back({nm, (int)i, 3, (L.splits - 1) * M * L.OC, 4.0 * (L.splits + 1) * M * L.OC});
      }
      if (L.pool) npool++;
    } else {
      snprintf(nm, sizeof(nm), "pool%d", npool++);
      p->kernels.push_back({nm, (int)i, 2, 0.0, in_b + out_b});
    }
  }
  if (p->fp16) {  // fp16 plans convert at the edges: fp32 frames in (unless conv0 is direct), fp32 out
    if (p->layers.empty() || p->layers[0].mode != MODE_DIRECT)
      p->kernels.insert(p->kernels.begin(), {"input.cvt", -1, 4, 0.0, 6.0 * B * p->in_h * p->in_w * p->in_c});
    if (!p->direct_out)
      p->kernels.push_back({"output.cvt", -1, 4, 0.0, 6.0 * B * p->cur_h * p->cur_w * p->cur_c});
    for (auto& L : p->layers) L.kernel_idx += (p->layers.empty() || p->layers[0].mode != MODE_DIRECT) ? 1 : 0;
  }
  p->weight_floats = align_up(off, 64);
  // activation buffers hold fp16 elements on the fp16 path
  p->act_floats = align_up((act * (size_t)p->batch + (p->fp16 ? 1 : 0)) / (p->fp16 ? 2 : 1), 64);
  p->col_floats = align_up(col * (size_t)p->batch, 64);
  p->slab_floats = align_up(std::max(slab * (size_t)p->batch, slab_fused), 64);
  p->ticket_floats = align_up(tickets, 64);  // unsigned tickets of the fused split-K layers
  // zero-bordered activations feeding MODE_PATCH16 (fp16, 2 B per element) / MODE_X3 (3 bf16
  // pieces, 6 B) layers: one region per producer (zeroed once at finalize; each producer
  // rewrites only its own interior, so its borders stay zero whatever the layers' shapes)
  size_t pad_total = 0;
  for (auto& L : p->layers)
    if (L.out_padded) {
      const size_t elems = (size_t)p->batch * (L.out_h() + 2) * (L.out_w() + 2) * L.OC;
      L.pad_off = pad_total;
      pad_total += align_up(p->fp16 ? (elems + 1) / 2 : elems * 3 / 2, 64);
    }
  p->pad_floats = pad_total;
  p->ws_floats = 2 * p->act_floats + p->col_floats + p->slab_floats + p->ticket_floats + p->pad_floats +
                 dnn_plan::kZeroFloats;
}

extern "C" {

const char* dnn_last_error(void) { return last_error(); }

int dnn_plan_create(int batch, int in_h, int in_w, int in_c, dnn_plan** out) {
  DNN_REQUIRE(out != nullptr, "dnn_plan_create: out is NULL");
  DNN_REQUIRE(batch >= 0 && in_h > 0 && in_w > 0 && in_c > 0, "dnn_plan_create: bad shape %d,%d,%d,%d", batch,
              in_h, in_w, in_c);
  dnn_plan* p = new dnn_plan();
  p->batch = batch;
  p->in_h = p->cur_h = in_h;
  p->in_w = p->cur_w = in_w;
  p->in_c = p->cur_c = in_c;
  const char* f = getenv("DNN_HIP_FUSE");
  p->fuse = !(f && f[0] == '0');
  const char* pe = getenv("DNN_HIP_PATCH");
  p->patch = !(pe && pe[0] == '0');
  p->splitk_fused = !getenv_flag_off("DNN_HIP_SPLITK_FUSED");
  *out = p;
  return 0;
}

void dnn_plan_destroy(dnn_plan* p) {
  if (!p) return;
  if (p->device >= 0) (void)hipSetDevice(p->device);
  drop_graph(p);
  for (auto e : p->ev) (void)hipEventDestroy(e);
  if (p->mark_ev) (void)hipEventDestroy(p->mark_ev);
  if (p->own_weights && p->weights) (void)hipFree(p->weights);
  if (p->own_ws && p->ws) (void)hipFree(p->ws);
  if (p->h_in_dev) (void)hipFree(p->h_in_dev);
  delete p;
}

static void set_cfg(dnn_plan* p, PlanLayer& L) {
  const long long M = (long long)p->batch * L.OH * L.OW;
  if (!p->fp16 && L.mode == MODE_X3_1X1) {  // one config: 32 x 128 tiles over all of K
    L.cfg = 0;
    L.Kpad = L.K;
    L.Npad = (int)align_up(L.OC, 128);
    L.splits = 1;
    return;
  }
  if (!p->fp16 && L.mode == MODE_X3) {  // one config per width (kernels_x3.hip); split-K by (N, K) only
    L.cfg = 0;
    L.Kpad = L.C == 16 ? 160 : L.K;  // (16 channels: 5 steps of two taps)
    L.Npad = L.OC;  // (a multiple of 256, or of 32 / 64 / 128 for the tile kernels)
    L.splits = L.x3k ? 1 : L.x3lat ? x3_lat_splits(L.OC, L.K) : x3_splits(L.OC, L.K);
    return;
  }
  if (p->fp16 && L.mode == MODE_PATCH16) {  // one config: 192x256 tiles, no split
    L.cfg = 0;
    L.Kpad = L.K;
    L.Npad = (int)align_up(L.OC, 256);
    L.splits = 1;
    return;
  }
  if (p->fp16) {  // fp16 MFMA configs: BK = 64 halves, split rule on (N, K) only
    L.cfg = choose_gemm16_cfg(M, L.OC, L.K);
    L.Kpad = (int)align_up(L.K, 64);
    L.Npad = (int)align_up(L.OC, gemm16_cfg_bn(L.cfg));
    L.splits = (L.Kpad == L.K) ? choose_splitk16(L.OC, L.K) : 1;
    return;
  }
  L.cfg = L.mode == MODE_IMPLICIT ? choose_gemm_cfg_implicit(M, L.OC, L.K) : choose_gemm_cfg(M, L.OC, L.K);
  if (const char* e = getenv("DNN_HIP_CFG")) {  // tuning experiments: "K:cfg,K:cfg,..."
    for (const char* q = e; *q;) {
      int k = 0, c = 0, n = 0;
      if (sscanf(q, "%d:%d%n", &k, &c, &n) != 2) break;
      if (k == L.K && c >= GEMM_128x128_K32 && c < GEMM_NUM_CFGS && c != GEMM_G64x32_K32) L.cfg = c;
      q += n;
      if (*q == ',') ++q;
    }
  }
  L.Kpad = (int)align_up(L.K, gemm_cfg_bk(L.cfg));
  L.Npad = (int)align_up(L.OC, gemm_cfg_bn(L.cfg));
  L.splits = (L.cfg >= GEMM_128x128_K32 && L.Kpad == L.K) ? choose_splitk(L.OC, L.K, fused_splitk(p)) : 1;
  if (p->latency && fused_splitk(p) && L.Kpad == L.K) {
    // a tile config and split for this M when the batch rule leaves the chip idle
    int cfg = L.cfg, sp = L.splits;
    choose_latency_plan(M, L.OC, L.K, &cfg, &sp, false);
    if (const char* e = getenv("DNN_HIP_SPLIT")) {  // tuning experiments: "K:splits,..."
      for (const char* q = e; *q;) {
        int k = 0, v = 0, n = 0;
        if (sscanf(q, "%d:%d%n", &k, &v, &n) != 2) break;
        if (k == L.K && v >= 1 && v <= 32 && (L.Kpad / gemm_cfg_bk(cfg)) % v == 0 && cfg >= GEMM_128x128_K32) sp = v;
        q += n;
        if (*q == ',') ++q;
      }
    }
    L.cfg = cfg;
    L.splits = sp;
    L.Npad = (int)align_up(L.OC, gemm_cfg_bn(L.cfg));
  }
}

int dnn_plan_set_precision(dnn_plan* p, int precision) {
  DNN_REQUIRE(p && !p->finalized && p->layers.empty(), "dnn_plan_set_precision: call before adding layers");
  DNN_REQUIRE(precision == 0 || precision == 1, "dnn_plan_set_precision: precision must be 0 (fp32) or 1 (fp16)");
  p->fp16 = precision;
  return 0;
}

int dnn_plan_set_latency_mode(dnn_plan* p, int on) {
  DNN_REQUIRE(p && !p->finalized && p->layers.empty(), "dnn_plan_set_latency_mode: call before adding layers");
  DNN_REQUIRE(on == 0 || on == 1, "dnn_plan_set_latency_mode: on must be 0 or 1");
  DNN_REQUIRE(!on || !p->fp16, "dnn_plan_set_latency_mode: fp32 plans only");
  p->latency = on != 0;
  return 0;
}

int dnn_plan_add_conv(dnn_plan* p, int kh, int kw, int od, int stride_h, int stride_w, int padding,
                      const float* kernel, const float* biases, const float* mean, const float* var,
                      const float* gamma, float eps, int leaky) {
  DNN_REQUIRE(p && !p->finalized, "dnn_plan_add_conv: plan is NULL or finalized");
  DNN_REQUIRE(kh > 0 && kw > 0 && od > 0 && stride_h > 0 && stride_w > 0, "dnn_plan_add_conv: bad args");
  DNN_REQUIRE((mean == nullptr) == (var == nullptr) && (var == nullptr) == (gamma == nullptr),
              "dnn_plan_add_conv: mean/var/gamma must be all set or all NULL");
  DNN_REQUIRE(leaky >= 0 && leaky <= 2, "dnn_plan_add_conv: leaky must be 0, 1 or 2");
  PlanLayer L;
  L.type = 0;
  L.H = p->cur_h;
  L.W = p->cur_w;
  L.C = p->cur_c;
  L.kh = kh;
  L.kw = kw;
  L.sh = stride_h;
  L.sw = stride_w;
  out_pads(L.H, kh, stride_h, padding, &L.OH, &L.pt);
  out_pads(L.W, kw, stride_w, padding, &L.OW, &L.pl);
  DNN_REQUIRE(L.OH > 0 && L.OW > 0, "dnn_plan_add_conv: empty output (%dx%d input, %dx%d kernel)", L.H, L.W, kh,
              kw);
  L.OC = od;
  L.K = kh * kw * L.C;
  const bool one_by_one = kh == 1 && kw == 1 && stride_h == 1 && stride_w == 1 && L.pt == 0 && L.pl == 0 &&
                          L.OH == L.H && L.OW == L.W && L.C % (p->fp16 ? 8 : 32) == 0;
  if (p->fp16) {
    // fp16 path: 1x1 on the input, implicit GEMM (C % 8 == 0), or conv0's direct kernel (set
    // when its 2x2/s2 pool arrives); anything else is rejected at finalize
    L.mode = one_by_one ? MODE_DIRECT_A : (L.C % 8 == 0 && kh * kw <= 30) ? MODE_IMPLICIT : MODE_GEMM;
    // 3x3 wide layers whose producer (a separate pool or another such conv) can write a
    // zero-bordered output: the patch kernel (input staged once per 64-channel chunk)
    if (L.mode == MODE_IMPLICIT && !p->layers.empty() &&
        conv_patch16_supported(L.C, od, L.H, L.W, L.OH, L.OW, kh, kw, stride_h, stride_w, L.pt, L.pl)) {
      PlanLayer& prev = p->layers.back();
      if (prev.type == 1 || (prev.mode == MODE_PATCH16 && !prev.pool) || prev.mode == MODE_TILE16) {
        L.mode = MODE_PATCH16;
        prev.out_padded = true;
      }
    }
  } else if (one_by_one)
    L.mode = MODE_DIRECT_A;
  else if (p->fuse && implicit_conv_supported(L.C, kh, kw) &&
           choose_gemm_cfg_implicit((long long)p->batch * L.OH * L.OW, od, L.K) >= 0)
    L.mode = MODE_IMPLICIT;
  else
    L.mode = MODE_GEMM;  // may become MODE_DIRECT when a 2x2/s2 pool follows (conv0)
  // fp32 3x3 wide layers fed by a separate pool or another such conv: the x3 conv (its producer
  // writes the split planes).  Batch plans choose it by the layer alone, so a batch-1 plan and a
  // batch-64 plan run the same arithmetic.  Latency plans (with the in-GEMM split-K combine) take
  // the batch kernel only where its tiles fill half the chip (at batch 1 a 176 x 256 tile's
  // one-chunk K slice alone takes ~26 us), elsewhere the small-M x3 kernel (gemm_x3_lat.h: 64
  // columns x one or two chunks per workgroup, 8 waves splitting rows / columns / chunks;
  // conv6 / conv7 of a one-frame plan) when it makes at least two K slices
  bool x3_cand = false, x3_lat = false, x3_k = false;
  if (!p->fp16 && L.mode == MODE_IMPLICIT && !p->layers.empty()) {
    const bool batch_ok = conv_x3_supported(L.C, od, L.H, L.W, L.OH, L.OW, kh, kw, stride_h, stride_w, L.pt, L.pl);
    // (the narrow kernels take small tiles in latency plans: batch_ok is enough.  conv1 at one
    // frame: the 16-channel kernel's 4 x 26 tiles 10.6 us, its 16 x 26 ones 11.7, the fp32 patch
    // conv 13.8 (HIP events, same box))
    const int xk = conv_x3_kind(od, L.C);
    const bool lat = p->latency && fused_splitk(p);
    // latency plans: conv3-conv5 of a frame with the K split inside the workgroup (one launch, no
    // partials), first; conv1 / conv2 on the narrow kernels' small tiles; conv6 / conv7 on the
    // small-M kernel's K slices + combine
    const bool fills = batch_ok && x3_tiles(p->batch, L.OH, L.OW, od, L.C, L.K) >= 128;  // the batch tiles fill the chip
    x3_k = lat && !fills &&
           conv_x3_ktile_supported(p->batch, L.C, od, L.H, L.W, L.OH, L.OW, kh, kw, stride_h, stride_w, L.pt, L.pl, 0);
    if (x3_k) {
      x3_cand = true;
    } else if (lat && !(batch_ok && (xk > 0 || x3_tiles(p->batch, L.OH, L.OW, od, L.C, L.K) >= 128))) {
      x3_lat = conv_x3_lat_supported(p->batch, L.C, od, L.H, L.W, L.OH, L.OW, kh, kw, stride_h, stride_w, L.pt,
                                     L.pl) &&
               x3_lat_splits(od, L.K) >= 2;
      x3_cand = x3_lat;
    } else {
      x3_cand = batch_ok;
    }
  }
  // fp32 1x1 layers right after an x3 conv (conv8 after conv7): the 1x1 x3 conv on the split
  // planes that producer writes instead of its fp32 output.  Chosen by the layer alone (batch
  // plans of any size run the same arithmetic).  Latency plans keep the fp32 GEMM split over the
  // chip where this kernel's 32 x 128 tiles would not fill it (one frame's 169 rows are 6 tiles:
  // 21 us against 14)
  // (latency plans whose frame leaves those tiles few: the K-split 1x1 form, 16 x 32 tiles)
  const long long t1x1 = ((long long)p->batch * L.OH * L.OW + 31) / 32 * ((od + 127) / 128);
  const bool lat1x1 = p->latency && fused_splitk(p) && t1x1 < 256;
  if (!p->fp16 && L.mode == MODE_DIRECT_A && !p->layers.empty() && p->layers.back().type == 0 &&
      p->layers.back().mode == MODE_X3 &&
      (lat1x1 ? conv_x3_1x1_ktile_supported(L.C, od, L.H, L.W) : conv_x3_1x1_supported(L.C, od, L.H, L.W))) {
    L.mode = MODE_X3_1X1;
    L.x3k = lat1x1;
    p->layers.back().out_padded = true;
  }
  if (x3_cand) {
    // producers that can write the split planes: a separate pool, another x3 conv, a pool-fused
    // implicit GEMM without split-K (its epilogue splits, EPI_OUT_X3) or the pool-fused patch
    // conv (conv1)
    PlanLayer& prev = p->layers.back();
    if (L.C == 16) {  // the 16-channel x3 kernel reads the producer's fp32 output (conv1)
      L.mode = MODE_X3;
    } else if ((prev.type == 1 && prev.C % 32 == 0) || (prev.type == 0 && prev.mode == MODE_X3) ||
        (prev.type == 0 && prev.mode == MODE_IMPLICIT && prev.pool && prev.splits == 1) ||
        (prev.type == 0 && prev.mode == MODE_PATCH && prev.pool)) {
      L.mode = MODE_X3;
      L.x3lat = x3_lat;
      L.x3k = x3_k;
      prev.out_padded = true;
    }
  }
  set_cfg(p, L);
  L.epi_flags = (biases ? EPI_BIAS : 0) | (mean ? EPI_BN : 0) |
                (leaky == 1 ? EPI_LEAKY_F64 : leaky == 2 ? EPI_LEAKY_F32 : 0);
  // fp16 plans (tolerance, not bit parity): BiasAdd + BatchNorm folded into v * alpha - beta
  // (alpha = gamma / sqrt(var + eps), beta = (mean - bias) * alpha) and the leaky as
  // max(v, 0.1f v): 4 VALU per output instead of ~30 for the reference's exact division and
  // double-rounded leaky (the VALU-bound small-channel kernels run on the epilogue)
  const bool fold16 = p->fp16 && mean;
  if (fold16)
    L.epi_flags = EPI_BN_AB | ((L.epi_flags & (EPI_LEAKY_F64 | EPI_LEAKY_F32)) ? EPI_LEAKY_F32 : 0);
  if (kernel) {
    L.have_host = true;
    L.w.assign(kernel, kernel + (size_t)L.K * od);
    const int np = std::max(L.Npad, 32);
    L.bias.assign(np, 0.f);
    L.mean.assign(np, 0.f);
    L.sq.assign(np, 1.f);
    L.gamma.assign(np, 1.f);
    for (int d = 0; d < od; ++d) {
      if (biases) L.bias[d] = biases[d];
      if (mean) {
        L.mean[d] = mean[d];
        // sqrt(variance + epsilon) in fp32 as the reference (dnn_openblas.c:48-50; dnn.py:325-327)
        volatile float s = var[d] + eps;
        L.sq[d] = sqrtf(s);
        L.gamma[d] = gamma[d];
      }
      if (fold16) {  // EPI_BN_AB: mean slot = alpha, sq slot = beta
        const float alpha = L.gamma[d] / L.sq[d];
        const float beta = (L.mean[d] - (biases ? biases[d] : 0.f)) * alpha;
        L.mean[d] = alpha;
        L.sq[d] = beta;
        L.bias[d] = 0.f;
        L.gamma[d] = 1.f;
      }
    }
  }
  p->layers.push_back(std::move(L));
  p->cur_h = p->layers.back().OH;
  p->cur_w = p->layers.back().OW;
  p->cur_c = od;
  return 0;
}

int dnn_plan_add_max_pool(dnn_plan* p, int kh, int kw, int stride_h, int stride_w, int padding) {
  DNN_REQUIRE(p && !p->finalized, "dnn_plan_add_max_pool: plan is NULL or finalized");
  DNN_REQUIRE(kh > 0 && kw > 0 && stride_h > 0 && stride_w > 0, "dnn_plan_add_max_pool: bad args");
  PlanLayer L;
  L.type = 1;
  L.H = p->cur_h;
  L.W = p->cur_w;
  L.C = L.OC = p->cur_c;
  L.kh = kh;
  L.kw = kw;
  L.sh = stride_h;
  L.sw = stride_w;
  out_pads(L.H, kh, stride_h, padding, &L.OH, &L.pt);
  out_pads(L.W, kw, stride_w, padding, &L.OW, &L.pl);
  DNN_REQUIRE(L.OH > 0 && L.OW > 0, "dnn_plan_add_max_pool: empty output");
  // fuse a 2x2/stride-2 pool (front pads are 0 for both SAME and VALID) into the conv before it
  if (p->fuse && !p->layers.empty() && kh == 2 && kw == 2 && stride_h == 2 && stride_w == 2 && L.pt == 0 &&
      L.pl == 0) {
    PlanLayer& prev = p->layers.back();
    // (latency plans: a split implicit conv keeps its split, the combine pools)
    if (prev.type == 0 && !prev.pool &&
        (prev.splits == 1 ||
         (prev.mode == MODE_IMPLICIT && !p->fp16 && fused_splitk(p) && generic_combine_cfg(prev.cfg)))) {
      bool ok = false;
      if (prev.mode == MODE_IMPLICIT) {
        ok = true;
        if (!p->fp16 && p->patch && prev.splits == 1 && patch_conv_pool_supported(prev.C, prev.OC, prev.H, prev.W, prev.OH, prev.OW, prev.kh, prev.kw,
                                                  prev.sh, prev.sw, prev.pt, prev.pl) &&
            prev.Kpad == patch_conv_kpad(prev.C))
          prev.mode = MODE_PATCH;  // same packed weights (Bt[Npad][Kpad]) as the implicit GEMM
        if (p->fp16 && p->patch &&
            conv1_patch_f16_supported(prev.C, prev.OC, prev.H, prev.W, prev.OH, prev.OW, prev.kh, prev.kw, prev.sh,
                                      prev.sw, prev.pt, prev.pl))
          prev.mode = MODE_PATCH;  // fp16 patch kernel on the same fp16 Bt
        // fp16 3x3 layers whose producer can write a zero-bordered output (a separate pool, the
        // conv1 patch kernel, another tile or patch16 conv): the 2-D tile kernel (its weights
        // packed in order 5 into the same Npad x Kpad slot)
        if (p->fp16 && prev.mode == MODE_IMPLICIT && prev.splits == 1 && p->layers.size() >= 2 &&
            conv_tile16_supported(prev.C, prev.OC, prev.H, prev.W, prev.OH, prev.OW, prev.kh, prev.kw, prev.sh,
                                  prev.sw, prev.pt, prev.pl) &&
            prev.Kpad % 32 == 0) {
          PlanLayer& q = p->layers[p->layers.size() - 2];
          if (q.type == 1 || (q.type == 0 && (q.mode == MODE_PATCH16 || q.mode == MODE_TILE16 ||
                                              (q.mode == MODE_PATCH && q.pool)))) {
            prev.mode = MODE_TILE16;
            q.out_padded = true;
          }
        }
      } else if (p->fp16 && prev.mode == MODE_PATCH16 &&
                 conv_tile16_supported(prev.C, prev.OC, prev.H, prev.W, prev.OH, prev.OW, prev.kh, prev.kw, prev.sh,
                                       prev.sw, prev.pt, prev.pl)) {
        prev.mode = MODE_TILE16;  // (its producer already writes the zero-bordered input) the pool fused
        ok = true;
      } else if (prev.mode == MODE_GEMM && direct_conv_pool_supported(prev.C, prev.OC, prev.kh, prev.kw, prev.sh,
                                                                      prev.sw)) {
        prev.mode = MODE_DIRECT;
        ok = true;
      } else if (prev.mode == MODE_X3 && !p->fp16 &&
                 (prev.x3k ? conv_x3_ktile_supported(p->batch, prev.C, prev.OC, prev.H, prev.W, prev.OH, prev.OW,
                                                     prev.kh, prev.kw, prev.sh, prev.sw, prev.pt, prev.pl, 1)
                           : conv_x3_pool_supported(prev.OC, prev.C, prev.H, prev.W))) {
        ok = true;  // pool-window-major rows, pooled before the epilogue in the x3 kernel
      }
      if (ok) {
        prev.pool = true;
        prev.PH = L.OH;
        prev.PW = L.OW;
        p->cur_h = L.OH;
        p->cur_w = L.OW;
        return 0;
      }
    }
  }
  // a 2x2/stride-1 SAME pool (YOLO's pool5) into a single-frame x3k conv before it: the conv
  // computes the row below each tile too and pools before its epilogue
  if (p->fuse && !p->layers.empty() && kh == 2 && kw == 2 && stride_h == 1 && stride_w == 1 && L.pt == 0 &&
      L.pl == 0 && L.OH == L.H && L.OW == L.W) {
    PlanLayer& prev = p->layers.back();
    if (prev.type == 0 && prev.mode == MODE_X3 && prev.x3k && !prev.pool && !prev.pool1 &&
        conv_x3_ktile_supported(p->batch, prev.C, prev.OC, prev.H, prev.W, prev.OH, prev.OW, prev.kh, prev.kw,
                                prev.sh, prev.sw, prev.pt, prev.pl, 2)) {
      prev.pool1 = true;
      return 0;
    }
    // ... into an fp16 conv of a 13 x 13 frame fed by a zero-bordered producer (conv5 + pool5 of
    // the fp16 path): the tile kernel's whole-frame form, pool taken from its fp16 stage
    if (p->fp16 && prev.type == 0 && (prev.mode == MODE_IMPLICIT || prev.mode == MODE_PATCH16) && !prev.pool &&
        !prev.pool1 && p->layers.size() >= 2 &&
        prev.kh == 3 && prev.kw == 3 && prev.sh == 1 && prev.sw == 1 && prev.pt == 1 && prev.pl == 1 &&
        prev.OH == prev.H && prev.OW == prev.W && prev.Kpad % 32 == 0 &&
        conv_img16_supported(prev.C, prev.OC, prev.H, prev.W)) {
      PlanLayer& q = p->layers[p->layers.size() - 2];
      if (q.type == 1 || (q.type == 0 && (q.mode == MODE_PATCH16 || q.mode == MODE_TILE16 ||
                                          (q.mode == MODE_PATCH && q.pool)))) {
        prev.mode = MODE_TILE16;
        prev.pool1 = true;
        prev.splits = 1;
        q.out_padded = true;
        return 0;
      }
    }
    // ... into a batch-tile x3 conv of a small frame (conv5 + pool5): whole-image tiles over all
    // of K (gemm_x3_img.h) instead of K slices whose partials the pool combines
    if (prev.type == 0 && prev.mode == MODE_X3 && !prev.x3k && !prev.x3lat && !prev.pool && !prev.pool1 &&
        prev.C != 16 && conv_x3_img_supported(prev.C, prev.OC, prev.H, prev.W)) {
      prev.pool1 = true;
      prev.x3img = true;
      prev.splits = 1;
      return 0;
    }
  }
  p->layers.push_back(std::move(L));
  p->cur_h = p->layers.back().OH;
  p->cur_w = p->layers.back().OW;
  return 0;
}

int dnn_plan_output_shape(const dnn_plan* p, int* batch, int* h, int* w, int* c) {
  DNN_REQUIRE(p, "dnn_plan_output_shape: plan is NULL");
  if (batch) *batch = p->batch;
  if (h) *h = p->cur_h;
  if (w) *w = p->cur_w;
  if (c) *c = p->cur_c;
  return 0;
}

int dnn_plan_memory(const dnn_plan* pc, size_t* weight_bytes, size_t* workspace_bytes) {
  DNN_REQUIRE(pc, "dnn_plan_memory: plan is NULL");
  dnn_plan* p = const_cast<dnn_plan*>(pc);
  layout(p);
  if (weight_bytes) *weight_bytes = p->weight_floats * sizeof(float);
  if (workspace_bytes) *workspace_bytes = p->ws_floats * sizeof(float);
  return 0;
}

static int upload_weights(dnn_plan* p) {
  size_t maxw = 0, maxp = 0;
  for (auto& L : p->layers)
    if (L.type == 0) {
      maxw = std::max(maxw, L.w.size());
      maxp = std::max(maxp, (size_t)L.Npad * L.Kpad);
    }
  float* tmp = nullptr;
  DNN_HIP_TRY(hipMalloc(&tmp, (std::max<size_t>(maxw, 1) + (p->fp16 ? maxp : 0)) * sizeof(float)));
  float* packed32 = tmp + std::max<size_t>(maxw, 1);  // fp16 plans: fp32 pack, then convert
  int rc = 0;
  for (auto& L : p->layers) {
    if (L.type != 0) continue;
    const size_t wb = L.w.size() * sizeof(float);
    if (L.mode == MODE_DIRECT) {  // HWIO [K][N] as is: one 16-float row per (tap, cin)
      if (hipMemcpy(p->weights + L.w_off, L.w.data(), wb, hipMemcpyHostToDevice) != hipSuccess) rc = -1;
    } else {
      if (hipMemcpy(tmp, L.w.data(), wb, hipMemcpyHostToDevice) != hipSuccess) rc = -1;
      if (p->fp16) {
        if (!rc)
          rc = launch_pack_weights(tmp, packed32, L.K, L.OC, L.Kpad, L.Npad, L.mode == MODE_TILE16 ? 5 : L.mode == MODE_PATCH16 ? patch16_pack_order() : 0, L.kh,
                                   L.kw, L.C, 0);
        if (!rc)
          rc = launch_f32_to_f16(packed32, reinterpret_cast<half_t*>(p->weights + L.w_off),
                                 (long long)L.Npad * L.Kpad, 0);
      } else if (!rc && (L.mode == MODE_X3 || L.mode == MODE_X3_1X1)) {
        rc = launch_pack_weights_x3(tmp, reinterpret_cast<unsigned short*>(p->weights + L.w_off), L.K, L.OC, L.Npad,
                                    L.C, 0);
      } else if (!rc) {
        rc = launch_pack_weights(tmp, p->weights + L.w_off, L.K, L.OC, L.Kpad, L.Npad, 0, L.kh, L.kw, L.C, 0);
      }
    }
    float* e = p->weights + L.epi_off;
    const size_t nb = (size_t)L.Npad * sizeof(float);
    if (!rc && (hipMemcpy(e, L.bias.data(), nb, hipMemcpyHostToDevice) != hipSuccess ||
                hipMemcpy(e + L.Npad, L.mean.data(), nb, hipMemcpyHostToDevice) != hipSuccess ||
                hipMemcpy(e + 2 * L.Npad, L.sq.data(), nb, hipMemcpyHostToDevice) != hipSuccess ||
                hipMemcpy(e + 3 * L.Npad, L.gamma.data(), nb, hipMemcpyHostToDevice) != hipSuccess))
      rc = -1;
    if (!rc && hipDeviceSynchronize() != hipSuccess) rc = -1;
    if (rc) {
      if (last_error()[0] == 0) set_error("dnn_plan_finalize: weight upload failed");
      break;
    }
  }
  (void)hipFree(tmp);
  if (rc) return rc;
  for (auto& L : p->layers) std::vector<float>().swap(L.w);  // host copies no longer needed
  return 0;
}

int dnn_plan_finalize(dnn_plan* p, int device, void* weights, void* workspace) {
  DNN_REQUIRE(p && !p->finalized, "dnn_plan_finalize: plan is NULL or already finalized");
  DNN_REQUIRE(!p->layers.empty(), "dnn_plan_finalize: plan has no layers");
  if (p->fp16)
    for (auto& L : p->layers) {
      DNN_REQUIRE(L.type != 0 || L.mode != MODE_GEMM,
                  "dnn_plan_finalize: fp16 plan cannot run conv %dx%dx%d k%dx%d (needs C %% 8 == 0, or <= 4 "
                  "input channels with a fused 2x2/s2 pool)", L.H, L.W, L.C, L.kh, L.kw);
      DNN_REQUIRE(L.type != 1 || L.C % 8 == 0, "dnn_plan_finalize: fp16 pool needs C %% 8 == 0 (C=%d)", L.C);
    }
  layout(p);
  // the fused kernels' output stores take 32-bit byte offsets from their region's base (the
  // write-through buffer stores of gemm_f32.h store16_at): every region a kernel writes, the
  // caller's output included (at most one activation), must stay below 2 GiB
  {
    const unsigned long long lim = 0x80000000ULL;
    bool ok = (unsigned long long)p->act_floats * 4 < lim && (unsigned long long)p->slab_floats * 4 < lim;
    for (auto& L : p->layers)
      if (L.out_padded)
        ok = ok && (unsigned long long)p->batch * (L.out_h() + 2) * (L.out_w() + 2) * L.OC * (p->fp16 ? 2 : 6) < lim;
    DNN_REQUIRE(ok, "dnn_plan_finalize: batch %d makes an activation region >= 2 GiB; split the batch over plans",
                p->batch);
  }
  DNN_HIP_TRY(hipSetDevice(device));
  p->device = device;
  if (weights) {
    p->weights = static_cast<float*>(weights);
  } else {
    DNN_HIP_TRY(hipMalloc(&p->weights, p->weight_floats * sizeof(float)));
    p->own_weights = true;
  }
  if (workspace) {
    p->ws = static_cast<float*>(workspace);
  } else {
    DNN_HIP_TRY(hipMalloc(&p->ws, p->ws_floats * sizeof(float)));
    p->own_ws = true;
  }
  // zero page at the end of the workspace (padding taps of the implicit GEMM read it)
  DNN_HIP_TRY(hipMemset(p->ws + p->ws_floats - dnn_plan::kZeroFloats, 0, dnn_plan::kZeroFloats * sizeof(float)));
  if (p->pad_floats)  // zero borders of the padded activations (interiors are rewritten every run)
    DNN_HIP_TRY(hipMemset(p->ws + 2 * p->act_floats + p->col_floats + p->slab_floats + p->ticket_floats, 0,
                          p->pad_floats * sizeof(float)));
  if (p->ticket_floats)  // fused split-K tickets start at zero; every launch leaves them zero
    DNN_HIP_TRY(hipMemset(p->ws + 2 * p->act_floats + p->col_floats + p->slab_floats, 0,
                          p->ticket_floats * sizeof(float)));
  bool all_host = true;
  for (auto& L : p->layers)
    if (L.type == 0 && !L.have_host) all_host = false;
  if (all_host) {
    int rc = upload_weights(p);
    if (rc) return rc;
  }
  DNN_HIP_TRY(hipDeviceSynchronize());
  p->finalized = true;
  return 0;
}

int dnn_plan_weight_buffer(const dnn_plan* p, void** ptr, size_t* bytes) {
  DNN_REQUIRE(p && p->finalized, "dnn_plan_weight_buffer: plan not finalized");
  if (ptr) *ptr = p->weights;
  if (bytes) *bytes = p->weight_floats * sizeof(float);
  return 0;
}

static int record_events(dnn_plan* p, int kernel, hipStream_t s);

// before each kernel (its plan index) and after the last one (-1): HIP events (timing) and the
// clock stamps around the stamped kernel — the opening stamp before its opening event, the closing
// stamp after the event that closes it, so an event-timed kernel never contains a stamp launch
static int record(dnn_plan* p, int kernel, hipStream_t s) {
  int rc;
  if (p->mark_kernel >= 0 && kernel == p->mark_kernel) DNN_HIP_TRY(hipEventRecord(p->mark_ev, s));
  const bool close_now = p->clk_open;
  if (!close_now && p->clk_kernel >= 0 && kernel == p->clk_kernel && p->clk_used < p->clk_cap) {
    if ((rc = launch_clock_stamp(s, p->clk_buf + (size_t)p->clk_used * 8 * p->clk_nwg, p->clk_nwg))) return rc;
    p->clk_open = true;
  }
  if ((rc = record_events(p, kernel, s))) return rc;
  if (close_now) {
    if ((rc = launch_clock_stamp(s, p->clk_buf + ((size_t)p->clk_used * 8 + 4) * p->clk_nwg, p->clk_nwg))) return rc;
    p->clk_open = false;
    p->clk_used++;
  }
  return 0;
}

static int record_events(dnn_plan* p, int kernel, hipStream_t s) {
  if (!p->timing) return 0;
  if (p->timing_only >= 0) {  // one kernel: its opening event and the next one (which closes it)
    const bool closes = p->ev_used > 0 && p->ev_kernel[p->ev_used - 1] == p->timing_only;
    if (kernel != p->timing_only && !closes) return 0;
    if (kernel != p->timing_only) kernel = -1;  // a pure closer opens nothing
  }
  if (p->ev_used + 1 >= p->ev_cap) return 0;  // capacity exhausted: stop recording silently
  DNN_HIP_TRY(hipEventRecord(p->ev[p->ev_used], s));
  p->ev_kernel[p->ev_used] = kernel;
  p->ev_used++;
  return 0;
}

// fp16 path: fp16 activations between layers, fp32 frames in / predictions out
static int run_fp16(dnn_plan* p, int n, const float* d_in, float* d_out, hipStream_t s) {
  half_t* act[2] = {reinterpret_cast<half_t*>(p->ws), reinterpret_cast<half_t*>(p->ws + p->act_floats)};
  float* slab = p->ws + 2 * p->act_floats + p->col_floats;
  unsigned* tickets = fused_splitk(p) ? reinterpret_cast<unsigned*>(slab + p->slab_floats) : nullptr;
  const float* zero = p->ws + p->ws_floats - dnn_plan::kZeroFloats;
  const int nl = (int)p->layers.size();
  const half_t* cur = nullptr;
  int rc = 0;
  if (p->layers[0].mode != MODE_DIRECT) {  // convert the frames once (into act[1]: layer 0 writes act[0])
    if ((rc = record(p, 0, s))) return rc;
    if ((rc = launch_f32_to_f16(d_in, act[1], (long long)n * p->in_h * p->in_w * p->in_c, s))) return rc;
    cur = act[1];
  }
  half_t* padr = reinterpret_cast<half_t*>(p->ws + 2 * p->act_floats + p->col_floats + p->slab_floats +
                                            p->ticket_floats);
  for (int i = 0; i < nl; ++i) {
    PlanLayer& L = p->layers[i];
    half_t* dst = L.out_padded ? padr + L.pad_off * 2 : act[i & 1];
    int k = L.kernel_idx;
    if (L.type == 0) {
      const float* e = p->weights + L.epi_off;
      const EpiParams epi{e, e + L.Npad, e + 2 * L.Npad, e + 3 * L.Npad, L.epi_flags};
      const half_t* wt = reinterpret_cast<const half_t*>(p->weights + L.w_off);
      if ((rc = record(p, k, s))) return rc;
      const long long Mc = (long long)n * L.OH * L.OW;
      switch (L.mode) {
        case MODE_DIRECT: {
          DirectGeom g{n, L.H, L.W, L.OH, L.OW, L.PH, L.PW, L.pt, L.pl};
          rc = conv0_mfma_supported(L.C, L.OC, L.kh, L.kw, L.sh, L.sw)
                   ? launch_conv0_mfma_f16(d_in, p->weights + L.w_off, dst, g, L.C, epi, s)
                   : launch_conv3x3_pool2_direct_f16out(d_in, p->weights + L.w_off, dst, g, L.C, L.OC, epi, s);
          break;
        }
        case MODE_PATCH: {
          DirectGeom g{n, L.H, L.W, L.OH, L.OW, L.PH, L.PW, L.pt, L.pl};
          rc = launch_conv1_patch_f16(cur, wt, L.Kpad, dst, g, zero, epi, s, L.out_padded ? 1 : 0);
          break;
        }
        case MODE_DIRECT_A:
          if (i == nl - 1 && p->direct_out) {
            rc = launch_gemm16_f32out(cur, L.C, wt, L.Kpad, L.Npad, d_out, L.OC, Mc, L.OC, L.Kpad, epi, s);
            if (rc) return rc;
            return record(p, -1, s);
          }
          rc = launch_gemm16(L.cfg, GEMM_DENSE, cur, L.C, ImplicitConv{}, wt, L.Kpad, dst, L.OC, Mc, L.OC, L.Kpad,
                             epi, s, L.splits, slab, tickets);
          break;
        case MODE_PATCH16:
          rc = launch_conv_patch16(cur, wt, L.Kpad, dst, L.out_padded ? 1 : 0, Mc, L.OC, L.K, L.H, L.W, L.C, epi, s);
          break;
        case MODE_TILE16:
          rc = launch_conv_tile16(cur, wt, L.Kpad, dst, L.out_padded ? 1 : 0, n, L.OC, L.K, L.H, L.W, L.C, epi, s,
                                  L.pool1 ? 2 : 1);
          break;
        case MODE_IMPLICIT: {
          ImplicitConv ic{zero, L.H, L.W, L.C, L.OH, L.OW, L.PH, L.PW, L.kh, L.kw, L.sh, L.sw, L.pt, L.pl,
                          L.pool ? 1 : 0};
          const long long M = L.pool ? 4LL * n * L.PH * L.PW : Mc;
          rc = launch_gemm16(L.cfg, L.pool ? GEMM_IMPLICIT_POOL : GEMM_IMPLICIT, cur, 0, ic, wt, L.Kpad, dst, L.OC,
                             M, L.OC, L.Kpad, epi, s, L.splits, slab, tickets);
          break;
        }
        default:
          set_error("dnn_plan_run: fp16 plan has an unsupported conv mode %d", L.mode);
          return -2;
      }
      if (rc) return rc;
      if (L.splits > 1 && !tickets) {
        if ((rc = record(p, ++k, s))) return rc;
        if ((rc = launch_splitk_reduce16(slab, L.splits, Mc, L.OC, dst, L.OC, epi, s))) return rc;
      }
    } else {
      PoolGeom g{n, L.H, L.W, L.C, L.OH, L.OW, L.kh, L.kw, L.sh, L.sw, L.pt, L.pl, 0};
      if ((rc = record(p, k, s))) return rc;
      if ((rc = launch_maxpool16(cur, dst, g, s, L.out_padded ? 1 : 0))) return rc;
    }
    cur = dst;
  }
  if ((rc = record(p, (int)p->kernels.size() - 1, s))) return rc;
  if ((rc = launch_f16_to_f32(cur, d_out, (long long)n * p->cur_h * p->cur_w * p->cur_c, s))) return rc;
  return record(p, -1, s);
}

int dnn_plan_run(dnn_plan* p, int n, const float* d_in, float* d_out, void* stream) {
  DNN_REQUIRE(p && p->finalized, "dnn_plan_run: plan not finalized");
  DNN_REQUIRE(n >= 0 && n <= p->batch, "dnn_plan_run: n=%d outside [0, %d]", n, p->batch);
  if (n == 0) return 0;
  DNN_REQUIRE(d_in && d_out, "dnn_plan_run: NULL tensor");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (p->fp16) return run_fp16(p, n, d_in, d_out, s);
  float* act[2] = {p->ws, p->ws + p->act_floats};
  float* col = p->ws + 2 * p->act_floats;
  float* slab = col + p->col_floats;
  unsigned* tickets = fused_splitk(p) ? reinterpret_cast<unsigned*>(slab + p->slab_floats) : nullptr;
  const float* zero = p->ws + p->ws_floats - dnn_plan::kZeroFloats;
  const float* cur = d_in;
  const int nl = (int)p->layers.size();
  unsigned short* padr = reinterpret_cast<unsigned short*>(slab + p->slab_floats + p->ticket_floats);
  for (int i = 0; i < nl; ++i) {
    PlanLayer& L = p->layers[i];
    float* dst = (i == nl - 1) ? d_out : act[i & 1];
    // output in x3 split planes (the next layer is MODE_X3)
    unsigned short* dsplit = L.out_padded ? padr + L.pad_off * 2 : nullptr;
    int k = L.kernel_idx;
    int rc = 0;
    if (L.type == 0) {
      const float* e = p->weights + L.epi_off;
      const EpiParams epi{e, e + L.Npad, e + 2 * L.Npad, e + 3 * L.Npad, L.epi_flags};
      const float* wt = p->weights + L.w_off;
      if ((rc = record(p, k, s))) return rc;
      const long long Mc = (long long)n * L.OH * L.OW;
      switch (L.mode) {
        case MODE_GEMM: {
          ConvGeom g{n, L.H, L.W, L.C, L.OH, L.OW, L.kh, L.kw, L.sh, L.sw, L.pt, L.pl, L.K, L.Kpad};
          if ((rc = launch_im2col(cur, col, g, s))) return rc;
          if ((rc = record(p, ++k, s))) return rc;
          rc = launch_gemm(L.cfg, col, L.Kpad, wt, L.Kpad, dst, L.OC, Mc, L.OC, L.Kpad, epi, s, L.splits, slab,
                           tickets);
          break;
        }
        case MODE_DIRECT_A:
          rc = launch_gemm(L.cfg, cur, L.C, wt, L.Kpad, dst, L.OC, Mc, L.OC, L.Kpad, epi, s, L.splits, slab,
                           tickets);
          break;
        case MODE_IMPLICIT: {
          ImplicitConv ic{zero, L.H, L.W, L.C, L.OH, L.OW, L.PH, L.PW, L.kh, L.kw, L.sh, L.sw, L.pt, L.pl,
                          L.pool ? 1 : 0};
          const long long M = L.pool ? 4LL * n * L.PH * L.PW : Mc;
          const int gm = L.pool ? GEMM_IMPLICIT_POOL : GEMM_IMPLICIT;
          // feeding an x3 conv: the pooled epilogue stores the split planes (EPI_OUT_X3)
          EpiParams ep = epi;
          float* o = dst;
          if (dsplit) {
            ep.flags |= EPI_OUT_X3;
            o = reinterpret_cast<float*>(dsplit);
          }
          // unsplit layers: the persistent kernel (same bits) when it covers the config
          rc = L.splits == 1 ? launch_gemm_persist(L.cfg, gm, cur, ic, wt, L.Kpad, o, L.OC, M, L.OC, L.Kpad, ep, s)
                             : -3;
          if (rc == -3)
            rc = launch_gemm_implicit(L.cfg, gm, cur, ic, wt, L.Kpad, o, L.OC, M, L.OC, L.Kpad, ep, s, L.splits,
                                      slab, tickets);
          break;
        }
        case MODE_DIRECT: {
          DirectGeom g{n, L.H, L.W, L.OH, L.OW, L.PH, L.PW, L.pt, L.pl};
          rc = conv0_mfma_supported(L.C, L.OC, L.kh, L.kw, L.sh, L.sw)
                   ? launch_conv0_mfma(cur, wt, dst, g, L.C, zero, epi, s)
                   : launch_conv3x3_pool2_direct(cur, wt, dst, g, L.C, L.OC, epi, s);
          break;
        }
        case MODE_PATCH: {
          DirectGeom g{n, L.H, L.W, L.OH, L.OW, L.PH, L.PW, L.pt, L.pl};
          rc = launch_conv3x3_patch_pool(cur, wt, L.Kpad, dst, g, L.C, L.OC, zero, epi, s, dsplit);
          break;
        }
        case MODE_X3_1X1:
          rc = L.x3k ? launch_conv_x3_1x1_ktile(reinterpret_cast<const unsigned short*>(cur),
                                                reinterpret_cast<const unsigned short*>(wt), dst, Mc, L.OC, L.Npad,
                                                L.K, L.H, L.W, L.C, epi, s)
                     : launch_conv_x3_1x1(reinterpret_cast<const unsigned short*>(cur),
                                          reinterpret_cast<const unsigned short*>(wt), dst, Mc, L.OC, L.Npad, L.K, L.H,
                                          L.W, L.C, epi, s);
          break;
        case MODE_X3:
          if (L.x3img) {
            rc = launch_conv_x3_img(reinterpret_cast<const unsigned short*>(cur),
                                    reinterpret_cast<const unsigned short*>(wt), dsplit ? nullptr : dst, dsplit, n,
                                    L.OC, L.Npad, L.K, L.H, L.W, L.C, epi, s);
          } else if (L.x3k) {
            rc = launch_conv_x3_ktile(reinterpret_cast<const unsigned short*>(cur),
                                      reinterpret_cast<const unsigned short*>(wt), dsplit ? nullptr : dst, dsplit,
                                      L.pool ? 4LL * n * L.PH * L.PW : Mc, L.OC, L.Npad, L.K, L.H, L.W, L.C, epi, s,
                                      L.pool ? 1 : L.pool1 ? 2 : 0);
          } else if (L.splits > 1) {  // raw partials into the slab; the next pool or a combine kernel finishes
            rc = L.x3lat ? launch_conv_x3_lat(reinterpret_cast<const unsigned short*>(cur),
                                              reinterpret_cast<const unsigned short*>(wt), slab, Mc, L.OC, L.Npad, L.K,
                                              L.H, L.W, L.C, L.splits, s)
                         : launch_conv_x3(reinterpret_cast<const unsigned short*>(cur),
                                          reinterpret_cast<const unsigned short*>(wt), slab, nullptr, Mc, L.OC, L.Npad,
                                          L.K, L.H, L.W, L.C, epi, s, L.splits);
            if (!rc && !(i + 1 < nl && p->layers[i + 1].type == 1)) {
              PoolGeom id{n, L.OH, L.OW, L.OC, L.OH, L.OW, 1, 1, 1, 1, 0, 0, 0};
              if ((rc = record(p, ++k, s))) return rc;
              rc = launch_x3_combine(slab, L.splits, Mc * L.OC, epi, id, dsplit ? nullptr : dst, dsplit, s);
            }
          } else {
            rc = launch_conv_x3(reinterpret_cast<const unsigned short*>(cur),
                                reinterpret_cast<const unsigned short*>(wt), dsplit ? nullptr : dst, dsplit,
                                L.pool ? 4LL * n * L.PH * L.PW : Mc, L.OC, L.Npad, L.K, L.H, L.W, L.C, epi, s, 1,
                                L.pool ? 1 : 0, p->latency && fused_splitk(p));
          }
          break;
        default:
          set_error("dnn_plan_run: fp32 plan has an unsupported conv mode %d", L.mode);
          return -2;
      }
      if (rc) return rc;
      if (L.splits > 1 && !tickets && L.mode != MODE_X3) {
        if ((rc = record(p, ++k, s))) return rc;
        if ((rc = launch_splitk_reduce(slab, L.splits, Mc, L.OC, dst, L.OC, epi, s))) return rc;
      }
    } else {
      PoolGeom g{n, L.H, L.W, L.C, L.OH, L.OW, L.kh, L.kw, L.sh, L.sw, L.pt, L.pl, 0};
      if ((rc = record(p, k, s))) return rc;
      const PlanLayer* pv = i > 0 ? &p->layers[i - 1] : nullptr;
      if (pv && pv->type == 0 && pv->mode == MODE_X3 && pv->splits > 1) {  // combine the x3 partials + pool
        const float* e = p->weights + pv->epi_off;
        const EpiParams pe{e, e + pv->Npad, e + 2 * pv->Npad, e + 3 * pv->Npad, pv->epi_flags};
        rc = launch_x3_combine(slab, pv->splits, (long long)n * pv->OH * pv->OW * pv->OC, pe, g, dsplit ? nullptr : dst,
                               dsplit, s);
      } else {
        rc = dsplit ? launch_maxpool_x3(cur, dsplit, g, s) : launch_maxpool(cur, dst, g, s);
      }
      if (rc) return rc;
    }
    cur = dsplit ? reinterpret_cast<const float*>(dsplit) : dst;
  }
  return record(p, -1, s);
}

int dnn_plan_run_host(dnn_plan* p, int n, const float* h_in, float* h_out) {
  DNN_REQUIRE(p && p->finalized, "dnn_plan_run_host: plan not finalized");
  DNN_REQUIRE(n >= 0 && n <= p->batch, "dnn_plan_run_host: n=%d outside [0, %d]", n, p->batch);
  if (n == 0) return 0;
  DNN_HIP_TRY(hipSetDevice(p->device));
  const size_t in_f = (size_t)n * p->in_h * p->in_w * p->in_c;
  const size_t out_f = (size_t)n * p->cur_h * p->cur_w * p->cur_c;
  if (p->h_in_floats < in_f + out_f) {
    if (p->h_in_dev) DNN_HIP_TRY(hipFree(p->h_in_dev));
    p->h_in_dev = nullptr;
    DNN_HIP_TRY(hipMalloc(&p->h_in_dev, (in_f + out_f) * sizeof(float)));
    p->h_in_floats = in_f + out_f;
  }
  float* d_in = p->h_in_dev;
  float* d_out = p->h_in_dev + in_f;
  DNN_HIP_TRY(hipMemcpy(d_in, h_in, in_f * sizeof(float), hipMemcpyHostToDevice));
  int rc = dnn_plan_run(p, n, d_in, d_out, nullptr);
  if (rc) return rc;
  DNN_HIP_TRY(hipMemcpy(h_out, d_out, out_f * sizeof(float), hipMemcpyDeviceToHost));
  return 0;
}

int dnn_plan_run_graph(dnn_plan* p, int n, const float* d_in, float* d_out, void* stream) {
  DNN_REQUIRE(p && p->finalized, "dnn_plan_run_graph: plan not finalized");
  DNN_REQUIRE(stream != nullptr, "dnn_plan_run_graph: needs a created stream (NULL cannot be captured)");
  DNN_REQUIRE(!p->timing, "dnn_plan_run_graph: per-kernel timing is active");
  DNN_REQUIRE(p->clk_kernel < 0, "dnn_plan_run_graph: clock stamping is active");
  DNN_REQUIRE(p->mark_kernel < 0, "dnn_plan_run_graph: a mark is set");
  DNN_REQUIRE(n >= 0 && n <= p->batch, "dnn_plan_run_graph: n=%d outside [0, %d]", n, p->batch);
  if (n == 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (!p->gexec || p->g_n != n || p->g_in != d_in || p->g_out != d_out) {
    drop_graph(p);
    DNN_HIP_TRY(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    const int rc = dnn_plan_run(p, n, d_in, d_out, stream);
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(s, &g);
    if (rc) {
      if (e == hipSuccess && g) (void)hipGraphDestroy(g);
      return rc;
    }
    DNN_HIP_TRY(e);
    p->graph = g;
    DNN_HIP_TRY(hipGraphInstantiate(&p->gexec, g, nullptr, nullptr, 0));
    p->g_n = n;
    p->g_in = d_in;
    p->g_out = d_out;
  }
  DNN_HIP_TRY(hipGraphLaunch(p->gexec, s));
  return 0;
}

int dnn_plan_num_kernels(const dnn_plan* pc) {
  if (!pc) return -2;
  dnn_plan* p = const_cast<dnn_plan*>(pc);
  if (!p->finalized) layout(p);
  return (int)p->kernels.size();
}

int dnn_plan_kernel_info(const dnn_plan* pc, int idx, char* name, int name_len, double* flops, double* bytes) {
  DNN_REQUIRE(pc, "dnn_plan_kernel_info: plan is NULL");
  dnn_plan* p = const_cast<dnn_plan*>(pc);
  if (!p->finalized) layout(p);
  DNN_REQUIRE(idx >= 0 && idx < (int)p->kernels.size(), "dnn_plan_kernel_info: bad index %d", idx);
  const KernelDesc& k = p->kernels[idx];
  if (name && name_len > 0) snprintf(name, name_len, "%s", k.name.c_str());
  if (flops) *flops = k.flops;
  if (bytes) *bytes = k.bytes;
  return 0;
}

int dnn_plan_describe(const dnn_plan* p, char* buf, int buf_len) {
  DNN_REQUIRE(p && buf && buf_len > 0, "dnn_plan_describe: bad args");
  std::string s;
  char line[256];
  for (size_t i = 0; i < p->layers.size(); ++i) {
    const PlanLayer& L = p->layers[i];
    if (L.type == 0) {
      char sk[32] = "";
      if (L.splits > 1) snprintf(sk, sizeof(sk), " splitK=%d", L.splits);
      snprintf(line, sizeof(line), "conv %dx%dx%d -> %dx%dx%d k%dx%d s%d mode=%s cfg=%d K=%d Kpad=%d%s%s%s%s%s\n", L.H,
               L.W, L.C, L.out_h(), L.out_w(), L.OC, L.kh, L.kw, L.sh, L.x3lat ? "x3_lat" : L.x3k ? "x3_ktile" : L.x3img ? "x3_img" : kModeName[L.mode], L.cfg, L.K, L.Kpad,
               L.pool ? " +pool2x2s2" : L.pool1 ? " +pool2x2s1" : "", sk,
               L.splits > 1 ? (L.mode == MODE_X3 ? " x3-combine" : fused_splitk(p) ? " combine" : "") : "",
               p->fp16 ? " fp16" : "", p->latency ? " latency" : "");
    } else
      snprintf(line, sizeof(line), "pool %dx%dx%d -> %dx%dx%d k%dx%d s%d%s\n", L.H, L.W, L.C, L.OH, L.OW, L.OC, L.kh,
               L.kw, L.sh, p->fp16 ? " fp16" : "");
    s += line;
  }
  snprintf(buf, buf_len, "%s", s.c_str());
  return 0;
}

int dnn_plan_timing_begin(dnn_plan* p, int max_runs) {
  DNN_REQUIRE(p && p->finalized, "dnn_plan_timing_begin: plan not finalized");
  DNN_REQUIRE(max_runs > 0, "dnn_plan_timing_begin: max_runs must be > 0");
  DNN_HIP_TRY(hipSetDevice(p->device));
  int need = max_runs * ((int)p->kernels.size() + 1) + 1;
  while ((int)p->ev.size() < need) {
    hipEvent_t e;
    DNN_HIP_TRY(hipEventCreate(&e));
    p->ev.push_back(e);
  }
  p->ev_kernel.assign(p->ev.size(), -1);
  p->ev_cap = (int)p->ev.size();
  p->ev_used = 0;
  p->timing_only = -1;
  p->timing = true;
  return 0;
}

int dnn_plan_timing_begin_only(dnn_plan* p, int max_runs, int kernel_idx) {
  DNN_REQUIRE(p && kernel_idx >= 0 && kernel_idx < (int)p->kernels.size(),
              "dnn_plan_timing_begin_only: bad kernel index %d", kernel_idx);
  int rc = dnn_plan_timing_begin(p, max_runs);
  if (rc) return rc;
  p->timing_only = kernel_idx;
  return 0;
}

int dnn_plan_clock_begin(dnn_plan* p, int kernel_idx, unsigned long long* dev_buf, int max_runs, int nwg) {
  DNN_REQUIRE(p && p->finalized, "dnn_plan_clock_begin: plan not finalized");
  DNN_REQUIRE(kernel_idx >= 0 && kernel_idx < (int)p->kernels.size(), "dnn_plan_clock_begin: bad kernel index %d",
              kernel_idx);
  DNN_REQUIRE(dev_buf && max_runs > 0 && nwg > 0 && nwg <= 65536, "dnn_plan_clock_begin: bad buffer / runs / nwg");
  p->clk_kernel = kernel_idx;
  p->clk_buf = dev_buf;
  p->clk_cap = max_runs;
  p->clk_nwg = nwg;
  p->clk_used = 0;
  p->clk_open = false;
  return 0;
}

int dnn_plan_set_mark(dnn_plan* p, int kernel_idx) {
  DNN_REQUIRE(p && p->finalized, "dnn_plan_set_mark: plan not finalized");
  DNN_REQUIRE(kernel_idx >= -1 && kernel_idx < (int)p->kernels.size(), "dnn_plan_set_mark: bad kernel index %d",
              kernel_idx);
  if (kernel_idx >= 0 && !p->mark_ev) {
    DNN_HIP_TRY(hipSetDevice(p->device));
    DNN_HIP_TRY(hipEventCreateWithFlags(&p->mark_ev, hipEventDisableTiming));
  }
  p->mark_kernel = kernel_idx;
  return 0;
}

int dnn_plan_wait_mark(dnn_plan* p, void* stream) {
  DNN_REQUIRE(p && p->mark_kernel >= 0 && p->mark_ev, "dnn_plan_wait_mark: no mark set");
  DNN_HIP_TRY(hipStreamWaitEvent(static_cast<hipStream_t>(stream), p->mark_ev, 0));
  return 0;
}

int dnn_plan_clock_end(dnn_plan* p, int* runs) {
  DNN_REQUIRE(p && p->clk_kernel >= 0, "dnn_plan_clock_end: clock stamping not active");
  DNN_REQUIRE(!p->clk_open, "dnn_plan_clock_end: a stamped kernel was not closed");
  if (runs) *runs = p->clk_used;
  p->clk_kernel = -1;
  p->clk_buf = nullptr;
  p->clk_used = p->clk_cap = 0;
  return 0;
}

int dnn_plan_timing_end(dnn_plan* p, double* ms_sum, long long* launches) {
  DNN_REQUIRE(p && p->timing, "dnn_plan_timing_end: timing not active");
  p->timing = false;
  const int nk = (int)p->kernels.size();
  for (int i = 0; i < nk; ++i) {
    if (ms_sum) ms_sum[i] = 0.0;
    if (launches) launches[i] = 0;
  }
  if (p->ev_used > 0) DNN_HIP_TRY(hipEventSynchronize(p->ev[p->ev_used - 1]));
  // event i opens kernel ev_kernel[i]; it is closed by event i+1 (same stream, in order)
  for (int i = 0; i + 1 < p->ev_used; ++i) {
    int k = p->ev_kernel[i];
    if (k < 0) continue;
    float ms = 0.f;
    DNN_HIP_TRY(hipEventElapsedTime(&ms, p->ev[i], p->ev[i + 1]));
    if (ms_sum) ms_sum[k] += ms;
    if (launches) launches[k] += 1;
  }
  p->ev_used = 0;
  return 0;
}

}  // extern "C"
