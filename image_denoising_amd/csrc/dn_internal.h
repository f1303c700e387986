// Internal declarations shared by the HIP kernels and the host orchestration.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace dn {

// Makes the device of stream s current for the lifetime of the guard (and restores the caller's
// on exit): the executors launch onto side streams and create per-device objects, which must
// happen on the device of the caller's stream, not whichever device the thread had selected.
struct StreamDeviceGuard {
  int prev = -1;
  explicit StreamDeviceGuard(hipStream_t s) {
    hipDevice_t dev = 0;
    int cur = 0;
    if (hipStreamGetDevice(s, &dev) == hipSuccess && hipGetDevice(&cur) == hipSuccess &&
        cur != dev && hipSetDevice(dev) == hipSuccess)
      prev = cur;
  }
  ~StreamDeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  StreamDeviceGuard(const StreamDeviceGuard&) = delete;
  StreamDeviceGuard& operator=(const StreamDeviceGuard&) = delete;
};

// In-step launch profiler (profile.cpp, dn_profile_ops): prof_on() while enabled; an OpTimer
// brackets one launch on its stream with HIP events and records op / shape / algorithmic FLOPs;
// launchers name the kernel they picked with prof_kernel() (a string literal).
bool prof_on();
void prof_kernel(const char* k);
struct OpTimer {
  int idx = -1;
  hipStream_t s = nullptr;
  OpTimer(hipStream_t st, const char* op, double flops, int K = 0, int NOUT = 0, int H = 0,
          int W = 0, int N = 0);
  ~OpTimer();
  OpTimer(const OpTimer&) = delete;
  OpTimer& operator=(const OpTimer&) = delete;
};

// DN_TRY(call) bracketed by an OpTimer (statement form)
#define DN_TIMED(st, op, flops, K, NO, h, w, n, call)          \
  do {                                                        \
    const ::dn::OpTimer dn_timer_(st, op, flops, K, NO, h, w, n); \
    DN_TRY(call);                                             \
  } while (0)

// How an output pixel of the implicit-GEMM kernel gathers its input pixels.
enum Gather {
  G_C3 = 0,   // 3x3, stride 1, pad 1: in(y+ky-1, x+kx-1), 9 taps     (conv fwd / conv dgrad)
  G_C1 = 1,   // 1x1: in(y, x), 1 tap                                  (1x1 conv, deconv fwd)
  G_DN2 = 2,  // in(2y+a, 2x+b), 4 taps                                (deconv data-grad)
  G_UP = 3,   // in(y, x), 1 tap, the 4 waves take the 4 (a,b) parities (deconv forward)
};

// How the weight-gradient kernel pairs its two operands over the pixel (K) dimension.
enum WMode {
  W_C3 = 0,   // dW[co][ci][t] = sum_p G[p][co] * X[p + off(t)][ci]
  W_C1 = 1,   // dW[co][ci]    = sum_p G[p][co] * X[p][ci]
  W_UP2 = 2,  // dW[ci][co][t] = sum_p X[p][ci] * G[2p + ab(t)][co]   (deconv)
};

enum Epi {
  EPI_BIAS = 0,      // acc + bias
  EPI_BIAS_ACT = 1,  // leaky_relu(acc + bias, 0.2)
  EPI_PLAIN = 2,     // acc
  EPI_MASK = 3,      // acc * (mask > 0 ? 1 : 0.2)   (LeakyReLU backward through the saved output)
  EPI_ACCUM = 4,     // out += acc
  EPI_BIAS_ADD = 5,  // acc + bias + res  (residual source read through the mask view)
};

enum OutLayout {
  OUT_NHWC = 0,  // out[((n*OH+y)*OW+x)*stride + off + c]
  OUT_NCHW = 1,  // out[((n*NOUT+c)*OH+y)*OW+x]
  OUT_UP2 = 2,   // deconv scatter: out[((n*2OH+2y+a)*2OW+2x+b)*stride + off + c], ab = blockIdx.z
  OUT_PS = 3,    // PixelShuffle(2) of the conv output: channel 4c+2i+j -> pixel (2y+i, 2x+j), channel c
};

// Strided view of the weight tensor as B[t][k][n] (t = tap, k = reduction channel, n = output).
struct WView {
  const float* w;
  long off, sK, sN, sT, sZ;  // idx = off + k*sK + n*sN + tap(t)*sT + blockIdx.z*sZ
  int taps;
  int flip;                  // tap(t) = flip ? taps-1-t : t; 2 (PK_W6 only): 3x3 taps transposed
};

struct FwdArgs {
  const float* in; int in_stride, in_off; int IHt, IWt;  // NHWC input, spatial dims
  int N, OH, OW;                                         // output domain (deconv: input res)
  int K, NOUT;                                           // reduction channels, output channels
  const float* wp; long wp_z;                            // packed weights (k_pack_batch), z stride
  const float* bias;
  int epi;
  float* out; int out_stride, out_off; int out_layout;
  const float* mask; int mask_stride, mask_off;
  // optional fused 2x2 max-pool of the activated output (EPI_BIAS_ACT, x6 kernels with an even
  // number of tile rows per wave): pooled NHWC pixel (OH/2, OW/2) at pool_out[pix * pool_stride +
  // pool_off + channel], in the window order of k_pool_fwd (bit-identical to pooling `out`)
  float* pool_out; int pool_stride, pool_off;
  int pool_only;  // with pool_out: the full-resolution output is not stored (forward-only plans)
  int zc;        // > 0: blockIdx.z selects output channels [z*zc, z*zc+zc) (wide layers)
  int x6_tail;   // split-bf16 kernels: packing of the last K chunk, x6_tail_mode(K) (0: plain)
  // split-bf16 3x3 forward, "selected pixels" mode (launch_fwd_x6_sel): per 2x2 output cell the
  // N2N pair choice rd (0..7, [N][OH/2][OW/2]); only the cell's two pair pixels are computed
  const unsigned char* sel_rd;
  // mixed-precision bf16 forward (conv_bf16.hip): the input / output activations are stored as
  // bf16 (RNE of the fp32 value; strides and offsets in elements) instead of fp32
  int in_bf16, out_bf16;
  // X6_T1 (k_c3w6's one-channel tail): that channel read from this compact [N][IHt][IWt] image
  // (the network input) instead of channel K - 4 of `in` -- its concat slice need not be written
  const float* in_t1;
};

// Fused output head (arch_unet.py:186-190, 253-257): the dec_conv1b kernel keeps its
// 96-channel tile in registers and runs nin_a -> nin_b -> nin_c on it.
struct HeadArgs {
  const float* wp;                    // packed [nin_a | nin_b] images, HEAD_LW floats each
  const float* ba; const float* bb;   // nin_a / nin_b biases
  const float* wc; const float* bc;   // nin_c weight [oc][96], bias [oc]
  int oc;
  float* y;                           // [N, oc, H, W]
  float* d1b; float* na; float* nb;   // optional NHWC (stride 96) saves for the backward
  // the input is a pair image (launch_fwd_x6_sel): output pixel (i, 2j + s) of the head goes to
  // y's pixel pair[rd[n][i][j]][s] of cell (i, j), y itself [N, oc, 2 * OH, OW]
  const unsigned char* rd;
};
// Backward of the head: g_nb = leaky'(nb) * (Wc^T dy), g_na = leaky'(na) * (Wb^T g_nb),
// g_d1b = leaky'(d1b) * (Wa^T g_na) over npx pixels (all NHWC stride 96, dy stride dy_stride)
struct HeadBwdArgs {
  const float* wp;                    // packed [nin_b^T | nin_a^T] images, HEAD_LW floats each
  const float* wc; int oc;            // nin_c weight [oc][96]
  const float* dy; int dy_stride;
  const float* nb; const float* na; const float* d1b;
  float* g_nb; float* g_na; float* g_d1b;
  long npx;
};
constexpr int HEAD_WS = 100;   // k-row stride of a head weight image (conflict-free A reads)
constexpr int HEAD_LW = 9728;  // 96 * HEAD_WS rounded up to 256 floats
constexpr int X6_HEAD_BF = 3 * 3 * 96 * 32;  // bf16 per layer of the bf16x6 head image (54 KiB)
constexpr int X6_HEAD_OCMAX = 16;  // most nin_c outputs of the bf16x6 head (kept in its LDS)
constexpr int X6_HEAD_BWD_OCMAX = 4;  // most nin_c outputs of its backward (k_head_bwd_x6)

struct WgradArgs {
  const float* g; int g_stride, g_off;  // gradient operand (rows = co), NHWC
  const float* x; int x_stride, x_off;  // input operand (cols = ci), NHWC
  int N, KH, KW;                        // pixel (K) domain; for W_UP2 g is at 2KH x 2KW
  int Cout, Cin;
  float* slab; long slab_stride;        // one [W ; b] image per split
  int wlayout;                          // 0: [co][ci][t]  1: [ci][co][t]
  int cin_total, ci_base;               // weight tensor's Cin and this launch's first ci
  int bias;                             // also produce the bias gradient
  const float* zeros;                   // >= 16 zero bytes (LDS-DMA source for padding)
  int co_base, cout_total;              // this launch's first output channel / the layer's Cout
  int zc;                               // > 0: blockIdx.z = output-channel block of zc channels
  // k_wgrad1p of nin_b with the gradient operand recomputed (head_gnb > 0 = nin_c's outputs):
  // g = leaky'(nb) (Wc^T dy) per pixel, with g pointing at nb (k_head_bwd_x6's order and result)
  int head_gnb; const float* hd_dy; int hd_dy_stride; const float* hd_wc;
  // (head_gnb) nin_c's weight gradient from the same nb / dy reads: one slab row per workgroup,
  // [oc][96] then the bias [oc] (k_wgrad_thin's layout), or null
  float* hd_slab_c; float* hd_dwc;  // (and its reduction's destination: nin_c's [W | b])
};

// strided NHWC view: element (pixel, c) at p[pixel * stride + off + c]
struct View {
  float* p;
  int stride;
  int off;
};

// geometry of the packed per-chunk weight image of the forward-family kernel
struct FwdGeom { int KC, TAPS, WNS, LW; };

// ---- batched weight packing (conv_x6.hip) ----
// Every weight image a pass needs is written by ONE launch: blockIdx.y = job, each job a
// grid-stride loop over its image.  The kinds: the fp32 per-chunk image of the forward-family
// kernel ([chunk][tap][k][n]), the pre-split bf16x6 image of a 3x3 layer, the four bf16x6 parity
// images of a 96-channel deconv, the two bf16x6 head images, and a zero fill (the weight
// gradients' 64-float DMA padding).  Strides of the weight view are element strides (< 2^31).
enum PackKind { PK_F32 = 0, PK_X6 = 1, PK_DECONV_X6 = 2, PK_HEAD_X6 = 3, PK_ZERO = 4,
                PK_DECONV_DGRAD_X6 = 5, PK_BF16 = 6, PK_W6 = 7 };
struct PackJob {
  const float* w;   // view origin (WView.w + off); PK_HEAD_X6: nin_a, PK_DECONV_X6: raw weight
  const float* w2;  // PK_HEAD_X6: nin_b
  void* out;
  int sK, sN, sT, sZ, taps, flip;
  int kind, K, NOUT, nz, zc, ntot, nch, tail;
  int g0, g1, g2, g3;  // PK_F32: KC, TAPS, WNS, LW; PK_X6: NP; PK_ZERO: floats;
                       // PK_BF16: NP, stage elements, 3x3?, image elements
};
constexpr int kPackJobs = 24;  // 24 x 104 B of kernel arguments
struct PackBatch {
  PackJob j[kPackJobs];
  int n = 0;
};
static_assert(sizeof(PackBatch) <= 3072, "pack batch exceeds the kernel-argument budget");
// elements (= threads of work) of one job
__host__ __device__ inline long pack_job_elems(const PackJob& j) {
  switch (j.kind) {
    case PK_F32: return (long)j.nch * j.g3 * j.nz;
    case PK_X6: return (long)j.nz * j.nch * 9 * j.g0 * 32;
    case PK_W6: return (long)j.nz * j.nch * 12 * j.g0 * 32;
    case PK_DECONV_X6: return 4L * 3 * 3 * 96 * 32;
    case PK_HEAD_X6: return 2L * 3 * 3 * 96 * 32;
    case PK_DECONV_DGRAD_X6: return 4L * 3 * 3 * 96 * 32;
    case PK_BF16: return j.g3;
    default: return j.g0;
  }
}
hipError_t pack_flush(PackBatch& b, hipStream_t s);  // one launch; empties b
hipError_t pack_add(PackBatch& b, const PackJob& j, hipStream_t s);  // flushes a full batch first
bool pack_job_x6(const WView& wv, int K, int nout, int zc, void* out, int tail, PackJob& j);
PackJob pack_job_head_x6(const float* wa, const float* wb, void* out);
PackJob pack_job_head_bwd_x6(const float* wa, const float* wb, void* out);  // Wb^T | Wa^T
hipError_t launch_head_bwd_x6(const HeadBwdArgs& h, const void* wimg, hipStream_t s);
PackJob pack_job_deconv_x6(const float* w, void* out);
PackJob pack_job_deconv_dgrad_x6(const float* w, void* out);
PackJob pack_job_zero(float* out, int n);
// the bf16 image of launch_pack_bf16 (conv_bf16.hip) as a job of the pass's pack launch
bool pack_job_bf16(const WView& wv, int K, int nout, int ksize, void* out, PackJob& j);

// ---- batched fixed-order reduction of weight-gradient slabs (conv.hip) ----
// out[omap(e)] = sum_s slab[s * stride + imap(e)], e < n, rows summed in a fixed order
// (bit-reproducible); imap(e) = (e / ig) * is1 + (e % ig) * is2, omap(e) = (e / og) * os1 +
// e % og + ooff.  A backward queues every layer's reduction (each layer owns its slab) and
// launches them together.
struct RedJob {
  const float* slab;
  float* out;
  int stride, splits, n, ig, is1, is2, og, os1, ooff, b0;  // b0: first workgroup of the job
  int vec;  // set by red_add: four contiguous 16-B aligned elements per lane (k_reduce_batch)
};
constexpr int kRedJobs = 40;
struct RedBatch {
  RedJob j[kRedJobs];
  int n = 0, blocks = 0;
};
static_assert(sizeof(RedBatch) <= 3072, "reduction batch exceeds the kernel-argument budget");
RedJob red_job(const float* slab, long stride, int splits, long n, float* out);  // identity maps
hipError_t red_add(RedBatch* b, const RedJob& j, hipStream_t s);  // b == nullptr: launched alone
hipError_t red_flush(RedBatch& b, hipStream_t s);                 // one launch; empties b

// ---- launchers (conv.hip) ----
bool fwd_geometry(int gather, int nout, FwdGeom& g);
long pack_floats(int gather, int nout, int K, int nz);  // floats of a packed weight set
bool pack_job(int gather, const WView& wv, int K, int nout, int nz, float* out, int zc, int ntot,
              PackJob& j);
hipError_t launch_pack(int gather, const WView& wv, int K, int nout, int nz, float* out,
                       hipStream_t s, int zc = 0, int ntot = 0);
// forward-family launch with explicit tile width NT (16*NT output channels per z-block) and
// a.zc = 16*NT output-channel blocks over blockIdx.z
hipError_t launch_fwd_nt(int gather, int nt, const FwdArgs& a, hipStream_t s);
hipError_t launch_fwd(int gather, const FwdArgs& a, hipStream_t s);
hipError_t launch_enc0_fwd(const float* x, int N, int C, int H, int W, const float* w,
                           const float* b, float* out, float* cat, int cat_stride, int cat_off,
                           int cat_zero_to, float* xcopy, hipStream_t s, bool out_bf16 = false);
int enc0_wgrad_splits(int N, int H, int W);
hipError_t launch_enc0_wgrad(const float* g, int g_stride, const float* x, int N, int C, int H,
                             int W, float* slab, int splits, float* dwb, hipStream_t s,
                             RedBatch* rb = nullptr);
// dL/dx (NCHW) of the network input from enc_conv0's (48 ch) and dec_conv1a's (96 ch, input
// channels [c1_base, c1_base + C) of c1_total) pre-activation gradients
hipError_t launch_dgrad_input(const float* g0, const float* w0, const float* g1, const float* w1,
                              int c1_total, int c1_base, int N, int C, int H, int W, float* dx,
                              hipStream_t s);
constexpr int EVAL_PARTS = 1024;
hipError_t launch_u8_to_unit(const uint8_t* x, long n, float* y, hipStream_t s);
hipError_t launch_tile_extract(const uint8_t* img, int C, int H, int W, int ps, int stride,
                               int nti, int ntj, float* tiles, hipStream_t s);
hipError_t launch_tile_blend(const float* pred, int C, int H, int W, int ps, int stride, int nti,
                             int ntj, const float* wmask, float* out_unit, uint8_t* out_u8,
                             hipStream_t s);
hipError_t launch_quantize_u8(const float* x, long n, int plus_half, uint8_t* y, hipStream_t s);
hipError_t launch_psnr(const uint8_t* a, const uint8_t* b, long n, double* part, double* out,
                       hipStream_t s);
hipError_t launch_ssim(const uint8_t* a, const uint8_t* b, int C, int H, int W, int hwc,
                       double* part, double* out, hipStream_t s);
hipError_t launch_l1_batched(const float* a, const float* b, long P, long n, double* out,
                             hipStream_t s);
hipError_t launch_l1(const float* a, const float* b, long n, double* part, double* out,
                     hipStream_t s);
hipError_t launch_head_bwd(const HeadBwdArgs& h, hipStream_t s);
int wgrad_thin_splits(long npx);
hipError_t launch_wgrad_c3_thin(const float* g, int cout, const float* x, int N, int C, int H,
                                int W, float* slab, long slab_stride, int cin_total, int ci_base,
                                int with_bias, int splits, hipStream_t s);
hipError_t launch_wgrad_thin(const float* g, int g_stride, int cout, const float* x, long npx,
                             float* slab, int splits, float* dwb, hipStream_t s,
                             RedBatch* rb = nullptr);
hipError_t launch_accumulate(float* dst, const float* src, long n, hipStream_t s);
hipError_t launch_head(const FwdArgs& a, const HeadArgs& h, hipStream_t s);
// nin_a -> nin_b -> nin_c on an activated dec_conv1b output (a.in, a.K = 96); h.d1b unused
hipError_t launch_nin_head(const FwdArgs& a, const HeadArgs& h, hipStream_t s);
hipError_t launch_pack_head(const WView& wa, const WView& wb, float* out, hipStream_t s,
                            PackBatch* pb = nullptr);  // pb: queued, not launched
// bf16x6 nin head (conv_x6.hip): pre-split nin_a | nin_b images (2 x X6_HEAD_BF bf16)
hipError_t launch_pack_head_x6(const float* wa, const float* wb, void* out, hipStream_t s);
// bf16: plain bf16 products (the bf16 base; no saved activations, no pair image)
hipError_t launch_nin_head_x6(const FwdArgs& a, const HeadArgs& h, const void* wimg, hipStream_t s,
                              bool bf16 = false);
// dec_conv1b-shaped 3x3 forward (K = NOUT = 96, EPI_BIAS_ACT) on the two N2N pair pixels of every
// 2x2 cell only (a.sel_rd): output = the "pair image" [N][OH/2][OW][96] NHWC, column 2j + s = pixel
// pair[rd][s] of cell j (s = 0, 1), i.e. exactly the pixels training_script.md:141-144 reads
hipError_t launch_fwd_x6_sel(const FwdArgs& a, hipStream_t s);
// bf16x6 ConvTranspose2d(96, 96, 2, 2) forward: four pre-split parity images (4 x X6_HEAD_BF bf16)
bool deconv_x6_ok(const FwdArgs& a);
hipError_t launch_pack_deconv_x6(const float* w, void* out, hipStream_t s);
hipError_t launch_deconv_x6(const FwdArgs& a, const void* wimg, hipStream_t s, bool b1 = false);
// its data gradient: a.in = dy (IHt x IWt = 2 OH x 2 OW, stride in_stride), a.out = dx (OH x OW,
// stride out_stride), a.mask (EPI_MASK) / EPI_PLAIN; K = NOUT = 96; wimg = the pre-split images
// (pack_job_deconv_dgrad_x6, 4 x X6_HEAD_BF bf16)
bool deconv_dgrad_x6_ok(const FwdArgs& a);
hipError_t launch_deconv_dgrad_x6(const FwdArgs& a, const void* wimg, hipStream_t s);
int wgrad_splits(int mode, int N, int KH, int KW, int Cin, int Cout);
hipError_t launch_wgrad(int mode, const WgradArgs& a, int splits, hipStream_t s, bool x6 = false);
// bf16x6 3x3 weight gradient (conv_x6.hip, k_wgrad3s): 96 or 48 outputs, Cin >= 32
bool wgrad3_x6_ok(const WgradArgs& a);
int wgrad_splits_x6(const WgradArgs& a, int splits);  // split count when the x6 kernel is taken
hipError_t launch_wgrad3_x6(const WgradArgs& a, int splits, hipStream_t s);
// ... its 96-output form with the operands split once per stage into LDS planes (wgrad_x6p.hip,
// k_wgrad3p; nz = output-channel blocks of a.zc == 96 over blockIdx.z, else 1)
bool wgrad3p_ok(const WgradArgs& a);
hipError_t launch_wgrad3p(const WgradArgs& a, int splits, hipStream_t s, int nz);
bool wgrad1p_ok(const WgradArgs& a);  // 96 -> 96 1x1 on k_wgrad1p (bf16x6)
hipError_t launch_wgrad1p(const WgradArgs& a, int splits, hipStream_t s, bool up2 = false);
bool wgrad1_ok(int mode, const WgradArgs& a);
long wgrad_slab_floats(int mode, int N, int KH, int KW, int cin, int cout);
int wgrad1_splits(int mode, int N, int KH, int KW);  // k_wgrad1 / k_wgrad1p split count
hipError_t launch_wgrad1(int mode, const WgradArgs& a, float* dwb, hipStream_t s,
                         RedBatch* rb = nullptr, bool x6 = false);
hipError_t launch_reduce_scatter(const float* slab, long slab_stride, int splits, long n,
                                 float* out, long grp, long ostride, long ooff, hipStream_t s,
                                 RedBatch* rb = nullptr);
hipError_t launch_reduce(const float* slab, long slab_stride, int splits, long n, float* out,
                         hipStream_t s, RedBatch* rb = nullptr);
bool fwd_supported(int gather, int nout);
int gwgrad_splits(int mode, int N, int KH, int KW, int Cin, int Cout);
bool gwgrad_ok(int mode, int Cin, int Cout, const View& g, const View& x);
hipError_t launch_gwgrad(int mode, const WgradArgs& a, int splits, hipStream_t s);
// the same 3x3 weight gradient on the bf16x6 kernel (conv_x6.hip)
bool gwgrad_x6_ok(const WgradArgs& a);
int gwgrad_x6_splits(const WgradArgs& a, int splits);
hipError_t launch_gwgrad_x6(const WgradArgs& a, int splits, hipStream_t s);
bool wgrad_supported(int mode, int cout, int cin);

// ---- elementwise launchers (elementwise.hip) ----
hipError_t launch_pool_fwd(const float* a, int N, int H, int W, int C, float* out, int os, int oo,
                           hipStream_t s);
hipError_t launch_pool_bwd(const float* a, int N, int H, int W, int C, const float* dp, int ds,
                           int doff, int act, float* da, hipStream_t s);
hipError_t launch_nchw_to_slice(const float* x, int N, int C, int H, int W, float* dst, int ds,
                                int doff, int zero_to, hipStream_t s);
hipError_t launch_subsample(const float* img, int N, int C, int H, int W, const uint8_t* rd_in,
                            uint64_t seed, uint64_t offset, uint64_t cell_base, float* sub1,
                            float* sub2, uint8_t* rd_out, hipStream_t s);
hipError_t launch_masks(const uint8_t* rd, int64_t ncells, uint8_t* m1, uint8_t* m2, hipStream_t s);
hipError_t launch_subimage_from_mask(const float* img, int N, int C, int H, int W,
                                     const uint8_t* mask, float* sub, hipStream_t s);
hipError_t launch_noise(const float* clean, int N, int64_t per_image, float std_,
                        const float* std_per_image, uint64_t seed, uint64_t offset,
                        uint64_t elem_base, float* noisy, hipStream_t s);
hipError_t launch_poisson(const float* clean, int N, int64_t per_image, float lam,
                          const float* lam_per_image, uint64_t seed, uint64_t offset,
                          uint64_t elem_base, float* noisy, hipStream_t s);
size_t loss_partials_bytes();
hipError_t launch_n2n_loss(const float* out, const float* sub2, const float* den,
                           const uint8_t* rd, int N, int C, int h, int w, float lambda,
                           float* dout, float* loss3, void* partials, hipStream_t s);
hipError_t launch_structure_loss(const float* pred, const float* pred2, const float* tgt, int N,
                                 int C, int H, int W, float alpha, float beta, float gamma,
                                 float* dpred, float* dpred2, float* loss5, void* partials,
                                 hipStream_t s);
hipError_t launch_adam(float* p, const float* g, float* m, float* v, int64_t n, float w1,
                       float b2, float w2, float step_size, float bc2s, float eps, float gscale,
                       hipStream_t s);

// ---- mixed-precision (bf16 MFMA) 3x3 forward (conv_bf16.hip) ----
long bf16_pack_elems(int K, int nout, int ksize = 3);
long bf16_stage_elems(int nout, int ksize);  // bf16 per weight stage of the image (-1: no tile)
// ---- fp32 3x3 conv on the bf16 matrix cores by three-way operand splitting (conv_x6.hip) ----
long x6_pack_elems(int K, int nout, int zc);  // bf16 elements of a pre-split weight image
hipError_t launch_pack_x6(const WView& wv, int K, int nout, int zc, void* out, hipStream_t s,
                          int tail = 0);
// packing of a partial last 32-channel chunk for the pipelined kernel: 1 = <= 4 channels,
// im2col over the 9 taps (2 stages); 2 = <= 16 channels, two taps per stage (5 stages); else 0
int x6_tail_mode(int K);
// the launch takes the pipelined kernel (large grid), so a tail-packed image may be used
bool x6_pipelined(int N, int H, int W, int nout, int zc);
hipError_t launch_fwd_x6(const FwdArgs& a, hipStream_t s);
// k_c3w6 (conv_w6.hip): the 1-D Winograd F(2,3) bf16x6 kernel for 96 output channels, on a PK_W6
// image; FwdArgs::x6_tail carries X6_W6 | x6_tail_mode(K) for it (see x6_image_mode)
constexpr int X6_W6 = 8;
// | X6_T1 (with X6_W6 and tail mode 1): the last chunk holds ONE live channel (the rest zero
// weights / zero pad channels), packed and consumed in k_c3w6's six-slot tail layout (TAIL 3)
constexpr int X6_T1 = 16;
hipError_t launch_fwd_w6(const FwdArgs& a, hipStream_t s);
// the N2N pair-pixel dec_conv1b on the Winograd kernel (conv_w6.hip k_c3w6s): the cells of rd
// listed per tile orientation (list: 2 N (OH/2)(OW/2) uint32, cnt: 2 N int), then the pass over
// them; a.wp = PK_W6 image, wpv = the tap-transposed PK_W6 image (WView flip = 2)
hipError_t launch_w6s_lists(const unsigned char* rd, int N, int OH, int OW, unsigned* list, int* cnt,
                            hipStream_t s);
hipError_t launch_fwd_w6s(const FwdArgs& a, const unsigned* list, const int* cnt, const void* wpv,
                          hipStream_t s);
// the weight-image mode of a split-bf16 3x3 launch (pack and launch agree on it): the tail
// packing of the last chunk on large grids with aligned views, | X6_W6 for the Winograd kernel
int x6_image_mode(int N, int H, int W, int K, int nout, int zc, bool aligned);
hipError_t launch_pack_bf16(const WView& wv, int K, int nout, void* out, hipStream_t s,
                            int ksize = 3);
hipError_t launch_fwd_bf16(const FwdArgs& a, hipStream_t s, int ksize = 3);
hipError_t launch_pack_bf16_deconv(const float* w, int cin, int cout, void* out, hipStream_t s);

// ---- adapter finetune (adapter.hip) ----
long adapter_param_count(int C);
int adapter_bwd_blocks(int N, int H, int W);
hipError_t launch_adapter_fwd(const float* prm, const float* noisy, const float* base, int N, int C,
                              int H, int W, float* out, hipStream_t s);
hipError_t launch_adapter_bwd(const float* prm, const float* noisy, const float* base,
                              const float* dout, int N, int C, int H, int W, float* dprm,
                              float* slab, hipStream_t s);
hipError_t launch_ft_loss(const float* pred, const float* tgt, int N, int C, int H, int W,
                          float lam, float* dpred, float* loss3, void* partials, hipStream_t s);

}  // namespace dn
