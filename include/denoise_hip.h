/*
 * denoise_hip.h — C-ABI of libdenoise_hip.so, the MI355X (gfx950) Neighbor2Neighbor
 * U-Net training path.
 *
 * The reference (lmh9507/image_denoising) is pure Python/PyTorch and has no FFI; its
 * "interface" is a set of Python callables.  Every entry point below names the
 * reference callable it replaces (file:line in the reference tree).  The Python
 * package `image_denoising_amd` binds these with ctypes.
 *
 * Conventions (all entry points):
 *   - every pointer is a caller-owned DEVICE buffer (PyTorch tensors are used only as
 *     containers); the library never allocates device memory — sizes come from the
 *     *_size queries;
 *   - all work is enqueued asynchronously on `stream` (a hipStream_t passed as void*;
 *     NULL = the legacy default stream); nothing synchronises the host;
 *   - the return value is a dn_status: 0 = ok, < 0 = error.  The message of the last
 *     error on the calling thread is available from dn_last_error();
 *   - network tensors at the boundary are NCHW fp32 contiguous, exactly like the
 *     reference's torch tensors; activations inside the workspace are NHWC fp32;
 *   - parameters live in ONE flat fp32 buffer in the reference's state_dict order
 *     (arch_unet.py:100-192, e.g. enc_conv0.weight, enc_conv0.bias, ..., nin_c.bias)
 *     with PyTorch layouts (Conv2d OIHW, ConvTranspose2d (in,out,kh,kw)), so
 *     checkpoints round-trip without repacking.  Gradients use the same layout.
 */
#ifndef DENOISE_HIP_H
#define DENOISE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int dn_status;
#define DN_OK 0
#define DN_ERR_ARG (-1)         /* bad shape / unsupported configuration */
#define DN_ERR_WORKSPACE (-2)   /* workspace too small */
#define DN_ERR_HIP (-3)         /* a HIP runtime call failed */

/* Arithmetic of the U-Net's 3x3 convolutions (dn_unet_forward_prec / dn_unet_backward_prec):
   DN_PREC_FP32     fp32 operands on the fp32 matrix cores (v_mfma_f32_16x16x4_f32);
   DN_PREC_FP32_X6  fp32 operands split exactly into three bf16 pieces, the six piece products of
                    order <= 2 on the bf16 matrix cores with fp32 accumulation: fp32-accurate
                    (error of an fp32 dot product), 2.67x the matrix-core ceiling;
   DN_PREC_BF16     forward only: bf16-rounded operands (the adapter-finetune frozen base). */
#define DN_PREC_FP32 0
#define DN_PREC_BF16 1
#define DN_PREC_FP32_X6 2

/* U-Net configuration: arch_unet.py:101-106 UNet(in_nc, out_nc, n_feature, blindspot=False). */
typedef struct dn_unet_cfg {
  int in_nc;      /* input channels  (1 or 3)  */
  int out_nc;     /* output channels (1 or 3)  */
  int n_feature;  /* 48 (the only width the reference trains, train.py:30) */
} dn_unet_cfg;

/* ---- library / errors ---------------------------------------------------------- */
/* "denoise_hip <version> gfx950 src=<16 hex>": the hash identifies the sources the library was
   built from (image_denoising_amd/_build.py source_hash) */
const char* dn_version(void);
/* The ABI revision of this header; a caller compiled against another revision must not bind.
   Revision 3 (library 0.3.x): dn_unet_backward / dn_unet_backward_prec gained the nullable
   `float* dx` argument after `dparams` (revision 2 had no dx: an old caller's arguments would
   be shifted, so check dn_abi_version() == DN_ABI_VERSION before binding).  Revision 4
   (library 0.4.x): dn_unet_backward_split added.  Revision 5 (library 0.5.x):
   dn_unet_pack_weights / dn_unet_forward_prepacked added (existing signatures unchanged). */
#define DN_ABI_VERSION 5
int dn_abi_version(void);
/* copies the last error message of this thread into buf (NUL-terminated); returns its length */
int dn_last_error(char* buf, size_t len);

/* ---- parameters ---------------------------------------------------------------- */
/* number of floats of the flat parameter buffer (1,256,689 for in=out=1, nf=48) */
dn_status dn_unet_param_count(const dn_unet_cfg* cfg, size_t* count);
/* offset (floats) and size of the weight of layer `index` (0..24, state_dict order);
   the bias follows the weight directly.  Used by the host mirror for state_dict views. */
dn_status dn_unet_param_info(const dn_unet_cfg* cfg, int index, size_t* w_off, size_t* w_count,
                             size_t* b_count);

/* ---- in-step launch profiler (bench.py's per-shape roofline) ------------------------- */
/* One launch recorded while profiling is enabled: op ("fwd3", "fwd3sel", "dgrad3", "wgrad3",
   "fwd1", "deconv", "deconv_dgrad", "wgrad1", "wgrad_up", "head", "head_bwd", "enc0", "pool",
   "pool_bwd", "pack", "reduce", "noise", "subsample", "loss", "adam", ...), the kernel the
   launcher picked (may be empty), the GEMM shape (K reduction channels -> NOUT outputs over N x H
   x W pixels), its algorithmic FLOPs (0 for byte-moving ops) and its HIP-event time on the
   stream it was launched on. */
typedef struct dn_op_record {
  char op[24];
  char kernel[48];
  int K, NOUT, H, W, N;
  double flops;
  double ms;
} dn_op_record;
/* enable (1) / disable (0) recording; either call drops earlier records.  While enabled the
   U-Net executors run every launch on the caller's stream (no side streams), so each record's
   event pair brackets one kernel.  Not for production steps (one event pair per launch). */
dn_status dn_profile_ops(int enable);
/* waits for the recorded events, copies up to cap records into out, sets *count to the number
   recorded (may exceed cap) and drops them. */
dn_status dn_profile_ops_read(dn_op_record* out, int cap, int* count);

/* ---- streams ---------------------------------------------------------------------- */
/* Creates the backward's side streams for the device of `stream` (the weight-gradient and
   reduction streams every U-Net / ImprovedUNet backward on this host thread uses) and submits a
   marker on each, so they take their hardware queues now.  HIP binds a stream to one of
   GPU_MAX_HW_QUEUES (default 4) hardware queues at its first submission and shares queues beyond
   that; a data-parallel caller runs this (and touches its own step streams) before
   torch.distributed / RCCL create their streams, so the step's concurrent streams keep queues of
   their own (image_denoising_amd.dist.prepare_streams).  Optional: the backward creates them
   on first use otherwise.  No reference counterpart (the reference runs one stream). */
dn_status dn_prepare_streams(void* stream);

/* ---- U-Net forward / backward: arch_unet.py:194-260 (UNet.forward) + autograd ---- */
/* bytes of workspace for a batch N x H x W (H, W multiples of 32).  with_backward=1 sizes the
   saved activations, gradient buffers and weight-gradient slabs needed by dn_unet_backward.
   The LAYOUT inside the workspace depends on with_backward (forward-only plans pad the concat
   buffers' pixel strides to 128-B lines; backward plans keep them dense), so offsets read with
   dn_unet_debug_buffers apply only to a workspace of the same with_backward. */
dn_status dn_unet_workspace_size(const dn_unet_cfg* cfg, int N, int H, int W, int with_backward,
                                 size_t* bytes);
/* y[N,out_nc,H,W] = UNet(x[N,in_nc,H,W]).  Activations are kept in ws for a later backward
   when ws was sized with with_backward=1. */
dn_status dn_unet_forward(const dn_unet_cfg* cfg, const float* params, const float* x, float* y,
                          int N, int H, int W, void* ws, size_t ws_bytes, void* stream);
/* The N2N step's no-grad pass (training_script.md:141-144): den = UNet(x) needed only at the
   two pixels of every 2x2 cell that generate_subimages' mask1 / mask2 pick (train.py:141-190),
   given by rd_idx (one byte per cell, [N][H/2][W/2], values 0..7 as for dn_n2n_subsample).  den
   (NCHW [N,out_nc,H,W]) is written at exactly those pixels; the others are left untouched.  With
   DN_PREC_FP32_X6 dec_conv1b and the head are evaluated on those pixels only (half their work;
   per-pixel arithmetic unchanged, so den at the pair pixels is bit-identical to
   dn_unet_forward_prec's); with DN_PREC_FP32 the whole image is computed.  Same workspace as
   dn_unet_forward (with_backward = 0); saves nothing for a backward. */
dn_status dn_unet_forward_n2n(const dn_unet_cfg* cfg, const float* params, const float* x,
                              float* den, const uint8_t* rd_idx, int N, int H, int W, void* ws,
                              size_t ws_bytes, int precision, void* stream);
/* Mixed-precision inference forward (the frozen base of the adapter finetune, BASELINE
   configs[4]): every 3x3 layer multiplies bf16-rounded activations and weights on the bf16
   matrix cores with fp32 accumulation; bias, activations, 1x1 layers, deconvs and storage stay
   fp32.  Same workspace as dn_unet_forward; saves nothing for a backward. */
dn_status dn_unet_forward_bf16(const dn_unet_cfg* cfg, const float* params, const float* x,
                               float* y, int N, int H, int W, void* ws, size_t ws_bytes,
                               void* stream);
/* dparams = dL/dparams given dy = dL/dy, for the activations saved by the last
   dn_unet_forward on the same ws (same N,H,W).  dparams is overwritten (not accumulated).
   dx (nullable) receives dL/dx of the network input, NCHW [N,in_nc,H,W] (overwritten): the
   input gradient autograd gives the reference module (arch_unet.py:194-260; x feeds enc_conv0
   and, as pool0, the last in_nc channels of dec_conv1a's input). */
dn_status dn_unet_backward(const dn_unet_cfg* cfg, const float* params, const float* dy,
                           float* dparams, float* dx, int N, int H, int W, void* ws,
                           size_t ws_bytes, void* stream);
/* dn_unet_forward / dn_unet_backward with the 3x3 convolutions' arithmetic chosen by
   precision (DN_PREC_*; the backward takes DN_PREC_FP32 or DN_PREC_FP32_X6). */
dn_status dn_unet_forward_prec(const dn_unet_cfg* cfg, const float* params, const float* x,
                               float* y, int N, int H, int W, void* ws, size_t ws_bytes,
                               int precision, void* stream);
dn_status dn_unet_backward_prec(const dn_unet_cfg* cfg, const float* params, const float* dy,
                                float* dparams, float* dx, int N, int H, int W, void* ws,
                                size_t ws_bytes, int precision, void* stream);
/* Persistent packed weights (SURVEY §8b dn_unet_pack_weights; replaces the per-call weight
   relayout that arch_unet.UNet's nn.Conv2d modules never need, arch_unet.py:115-192): packs the
   forward's weight images for (N, H, W, precision) into ws -- the plan is chosen by ws_bytes as
   in dn_unet_forward_prec -- and dn_unet_forward_prepacked then runs the forward on them without
   re-packing (inference over many batches with fixed weights: evaluation.py:66-108).  The
   prepacked forward still reads the biases and the thin layers (enc_conv0, nin_c) from params,
   which must be the buffer that was packed; its output equals dn_unet_forward_prec's bit for
   bit.  Any forward or backward with packing (every other entry point) overwrites the images. */
dn_status dn_unet_pack_weights(const dn_unet_cfg* cfg, const float* params, int N, int H, int W,
                               void* ws, size_t ws_bytes, int precision, void* stream);
dn_status dn_unet_forward_prepacked(const dn_unet_cfg* cfg, const float* params, const float* x,
                                    float* y, int N, int H, int W, void* ws, size_t ws_bytes,
                                    int precision, void* stream);
/* dn_unet_backward_prec for a data-parallel step that overlaps the gradient all-reduce with
   the backward (train.py:324-326 reduces inside the backward too).  The backward finishes the
   head's and the decoder's parameter gradients first: dparams[*tail_begin ..] (the state_dict
   tail from dec_conv5a on: every decoder layer except upsample5, the head) is final once
   tail_ready (a hipEvent_t the caller created on the device of stream, passed as void*) fires;
   the library records it on the stream that finishes that range.  dparams[0 .. *tail_begin)
   (the encoder and upsample5) is final when the work queued on `stream` completes, as for
   dn_unet_backward_prec.  A caller then all-reduces the tail on a stream that waits on
   tail_ready while the encoder's gradients are still being computed.  tail_ready may be NULL
   (then only *tail_begin is set); tail_begin may be NULL. */
dn_status dn_unet_backward_split(const dn_unet_cfg* cfg, const float* params, const float* dy,
                                 float* dparams, float* dx, int N, int H, int W, void* ws,
                                 size_t ws_bytes, int precision, void* stream, void* tail_ready,
                                 int64_t* tail_begin);

/* Debug/introspection: (offset_floats, channel_stride, level) of every NHWC buffer of the
   workspace plan, in the order c1 a0 a1 c2..c5 a2..a5 p5 a6 d{2..5}a d{2..5}b d1a d1b nin_a nin_b
   [g_nb g_na g_d1b g_d1a g_c1 g_c2..g_c5 g_d{2..5}a g_d{2..5}b g_a2..g_a5 g_a6 g_p5 g_a0 g_a1].
   c1 = [up1 (2*nf) | image (C) | pad] is reported with its full pixel stride, but only the up1
   channels [0, 2*nf) are guaranteed to be written: when the bf16x6 Winograd dec_conv1a reads the
   image channel from the network input itself (C = 1, unet.cpp X6_T1), enc_conv0 does not copy
   the image into c1 and channels [2*nf, stride) hold stale workspace data. */
dn_status dn_unet_debug_buffers(const dn_unet_cfg* cfg, int N, int H, int W, int with_backward,
                                int64_t* desc, int max_entries, int* n_entries);

/* ---- Neighbor2Neighbor sub-sampler: train.py:134-190 ------------------------------ */
/* One call replaces generate_mask_pair + 2x generate_subimages (train.py:141-190,
   training_script.md:137-139).  img is NCHW [N,C,H,W]; sub1/sub2 are NCHW [N,C,H/2,W/2].
   rd_idx (one byte per 2x2 cell, values 0..7 indexing the pair table of train.py:151-154):
     - rd_idx_in != NULL: parity mode, the caller's per-cell choices are used;
     - rd_idx_in == NULL: counter-based Philox4x32-10 keyed on (seed, offset) and the GLOBAL
       cell index cell_base + (n*H/2 + i)*W/2 + j, so the mask stream does not depend on how
       a batch is sharded over ranks.
   rd_idx_out (nullable) receives the choices actually used. */
dn_status dn_n2n_subsample(const float* img, int N, int C, int H, int W, const uint8_t* rd_idx_in,
                           uint64_t seed, uint64_t offset, uint64_t cell_base, float* sub1,
                           float* sub2, uint8_t* rd_idx_out, void* stream);
/* generate_mask_pair output format (train.py:141-172): two bool[N*H/2*W/2*4] masks from rd_idx */
dn_status dn_n2n_masks(const uint8_t* rd_idx, int64_t ncells, uint8_t* mask1, uint8_t* mask2,
                       void* stream);
/* generate_subimages(img, mask) (train.py:175-190) for a single bool mask */
dn_status dn_n2n_subimage_from_mask(const float* img, int N, int C, int H, int W,
                                    const uint8_t* mask, float* sub, void* stream);

/* ---- noise synthesis: train.py:84-101 AugmentNoise.add_train_noise (gauss) -------- */
/* noisy = clean + std_n * N(0,1); std_per_image (nullable, [N]) overrides std (gauss_range).
   Normals come from Philox4x32-10 + Box-Muller keyed on (seed, offset, elem_base + e). */
dn_status dn_add_gauss_noise(const float* clean, int N, int64_t per_image, float std_,
                             const float* std_per_image, uint64_t seed, uint64_t offset,
                             uint64_t elem_base, float* noisy, void* stream);
/* Poisson noise, train.py:102-111 (AugmentNoise poisson_fix / poisson_range; replaces
   torch.poisson(lam * x, generator) / lam): noisy = Poisson(lam * clean) / lam, lam per image
   from lam_per_image when not null.  Counts by fp64 CDF inversion of one 53-bit Philox uniform
   per element (same global-index stream convention as the Gaussian).  0 < lam <= 500 and clean
   in [0, 1] (lam * clean <= 500): a scalar lam outside that range is rejected (DN_ERR_ARG); a
   per-image lam outside it (device memory, not checked by the host) makes that image NaN. */
dn_status dn_add_poisson_noise(const float* clean, int N, int64_t per_image, float lam,
                               const float* lam_per_image, uint64_t seed, uint64_t offset,
                               uint64_t elem_base, float* noisy, void* stream);

/* ---- losses ------------------------------------------------------------------------ */
/* N2N regularised loss, training_script.md:141-153.  out, sub2: [N,C,h,w]; den: [N,C,2h,2w]
   (the no-grad full-resolution denoised image, sub-sampled in-kernel with rd_idx).
     loss1 = mean((out-sub2)^2); loss2 = lambda * mean(((out-sub2) - (den1-den2))^2)
   Writes dout = d(loss1+loss2)/d out and loss3 = {loss1, loss2, loss1+loss2} (device floats).
   partial_ws must hold dn_loss_partials_size() bytes. */
size_t dn_loss_partials_size(void);
dn_status dn_n2n_loss(const float* out, const float* sub2, const float* den, const uint8_t* rd_idx,
                      int N, int C, int h, int w, float lambda, float* dout, float* loss3,
                      void* partial_ws, void* stream);
/* Structure_loss, util.py:41-70 (alpha=1, beta=.5, gamma=.5, reduction='mean'):
   L = alpha*L1(pred,tgt) + beta*(L1 TV of pred2 over H + over W)/2 + gamma*L1(pred2,tgt).
   Writes dpred, dpred2 and loss5 = {pixel, tv1, tv2, cst, total}. */
dn_status dn_structure_loss(const float* pred, const float* pred2, const float* target, int N, int C,
                            int H, int W, float alpha, float beta, float gamma, float* dpred,
                            float* dpred2, float* loss5, void* partial_ws, void* stream);

/* ---- optimiser: torch.optim.Adam as used at train.py:332, :368 --------------------- */
/* One fused Adam step over n floats (torch _single_tensor_adam math, amsgrad=False,
   weight_decay=0).  step is the 1-based step count after increment.  grad_scale multiplies
   the gradient first (1/world_size after an all-reduce sum). */
dn_status dn_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                       float lr, float beta1, float beta2, float eps, int64_t step,
                       float grad_scale, void* stream);

/* dst += src over n floats (sums the parameter gradients of several backward passes, e.g.
   the two network evaluations of the Structure_loss step, train.py:361-367) */
dn_status dn_accumulate(float* dst, const float* src, int64_t n, void* stream);

/* ---- op-level entry points (NHWC), used by the tests and the tiled-inference path ---- */
/* The forward-family kernels read weights pre-packed into per-chunk LDS images; the caller
   provides that scratch (pack_ws, pack_bytes >= the *_pack_size query).  backward_data=1
   sizes the flipped/transposed image used by the data gradient. */
size_t dn_conv2d_pack_size(int Cin, int Cout, int ksize, int backward_data);
size_t dn_deconv2x2_pack_size(int Cin, int Cout, int backward_data);
/* 3x3/pad1 (ksize=3) or 1x1 (ksize=1) convolution + bias (+ LeakyReLU(0.2) if act).
   x: [N,H,W,*] with channel stride x_stride; y: [N,H,W,*] stride y_stride.
   w: [Cout,Cin,k,k] (PyTorch OIHW), b: [Cout].  arch_unet.py:65-78 conv_func, :113 act. */
dn_status dn_conv2d_forward(const float* x, int x_stride, int N, int H, int W, int Cin,
                            const float* w, const float* b, int Cout, int ksize, int act, float* y,
                            int y_stride, void* pack_ws, size_t pack_bytes, void* stream);
/* 3x3/pad1 forward on the bf16 matrix cores (bf16-rounded x and w, fp32 accumulate, fp32 bias /
   LeakyReLU / output); Cout <= 96 and a multiple of 4.  Used by dn_unet_forward_bf16. */
size_t dn_conv2d_bf16_pack_size(int Cin, int Cout);
dn_status dn_conv2d_forward_bf16(const float* x, int x_stride, int N, int H, int W, int Cin,
                                 const float* w, const float* b, int Cout, int act, float* y,
                                 int y_stride, void* pack_ws, size_t pack_bytes, void* stream);
/* 3x3/pad1 forward and data gradient at fp32 accuracy on the bf16 matrix cores (DN_PREC_FP32_X6:
   operands split exactly into three bf16 pieces, six piece products accumulated in fp32).
   Forward: Cout <= 96.  Data gradient: any Cin (blocks of 48 channels past 96).  Same argument
   meaning as dn_conv2d_forward (ksize 3) / dn_conv2d_backward_data. */
size_t dn_conv2d_x6_pack_size(int Cin, int Cout, int backward_data);
dn_status dn_conv2d_forward_x6(const float* x, int x_stride, int N, int H, int W, int Cin,
                               const float* w, const float* b, int Cout, int act, float* y,
                               int y_stride, void* pack_ws, size_t pack_bytes, void* stream);
dn_status dn_conv2d_backward_data_x6(const float* dz, int N, int H, int W, int Cout,
                                     const float* w, int Cin, const float* mask, int mask_stride,
                                     int accumulate, float* dx, int dx_stride, void* pack_ws,
                                     size_t pack_bytes, void* stream);
/* dx = conv^T(dz) [* leaky'(mask)] : data gradient (mask nullable; mask_stride). If accumulate,
   dx += result.  dx stride dx_stride. */
dn_status dn_conv2d_backward_data(const float* dz, int N, int H, int W, int Cout, const float* w,
                                  int Cin, int ksize, const float* mask, int mask_stride,
                                  int accumulate, float* dx, int dx_stride, void* pack_ws,
                                  size_t pack_bytes, void* stream);
/* dw [Cout,Cin,k,k] and db [Cout] (contiguous after dw) from dz [N,H,W,Cout] and x.
   slab must hold dn_conv2d_wgrad_slab_size() bytes. */
size_t dn_conv2d_wgrad_slab_size(int N, int H, int W, int Cin, int Cout, int ksize);
dn_status dn_conv2d_backward_weight(const float* dz, const float* x, int x_stride, int N, int H,
                                    int W, int Cin, int Cout, int ksize, float* dwb, void* slab,
                                    void* stream);
/* The same 3x3 weight gradient at fp32 accuracy on the bf16 matrix cores (DN_PREC_FP32_X6: each
   32-pixel K block as six split-bf16 products, summed from zero, added in fp32).  96 output
   channels with Cin >= 32 take the split kernel; other shapes run the fp32 kernel.  Same slab. */
dn_status dn_conv2d_backward_weight_x6(const float* dz, const float* x, int x_stride, int N,
                                       int H, int W, int Cin, int Cout, float* dwb, void* slab,
                                       void* stream);
/* ConvTranspose2d(Cin, Cout, 2, 2) (arch_unet.py:57): x [N,H,W,Cin] -> y [N,2H,2W,*]
   (written at channel offset y_off of stride y_stride, i.e. directly into a concat buffer). */
dn_status dn_deconv2x2_forward(const float* x, int N, int H, int W, int Cin, const float* w,
                               const float* b, int Cout, float* y, int y_stride, int y_off,
                               void* pack_ws, size_t pack_bytes, void* stream);
/* The same ConvTranspose2d(96, 96, 2, 2) at fp32 accuracy on the bf16 matrix cores
   (DN_PREC_FP32_X6); pack_bytes >= dn_deconv2x2_x6_pack_size().  x channel stride 96. */
size_t dn_deconv2x2_x6_pack_size(void);
dn_status dn_deconv2x2_forward_x6(const float* x, int N, int H, int W, const float* w,
                                  const float* b, float* y, int y_stride, int y_off, void* pack_ws,
                                  size_t pack_bytes, void* stream);
/* Its data gradient (same pack size): dx [N,H,W,96] (contiguous) from dy [N,2H,2W,*] (channel
   stride dy_stride), times LeakyReLU'(mask) when mask [N,H,W,96] is not null. */
dn_status dn_deconv2x2_backward_data_x6(const float* dy, int dy_stride, int N, int H, int W,
                                        const float* w, const float* mask, float* dx,
                                        void* pack_ws, size_t pack_bytes, void* stream);
dn_status dn_deconv2x2_backward_data(const float* dy, int dy_stride, int N, int H, int W, int Cout,
                                     const float* w, int Cin, const float* mask, float* dx,
                                     void* pack_ws, size_t pack_bytes, void* stream);
size_t dn_deconv2x2_wgrad_slab_size(int N, int H, int W, int Cin, int Cout);
dn_status dn_deconv2x2_backward_weight(const float* dy, int dy_stride, const float* x, int N, int H,
                                       int W, int Cin, int Cout, float* dwb, void* slab,
                                       void* stream);
/* MaxPool2d(2) (arch_unet.py:120-135) on NHWC x [N,H,W,C] -> y (channel stride y_stride, offset y_off) */
dn_status dn_maxpool2x2_forward(const float* x, int N, int H, int W, int C, float* y, int y_stride,
                                int y_off, void* stream);
/* dx = route(dy -> argmax, first max in row-major wins) * leaky'(x) if act else route only */
dn_status dn_maxpool2x2_backward(const float* x, int N, int H, int W, int C, const float* dy,
                                 int dy_stride, int dy_off, int act, float* dx, void* stream);

/* ---- evaluation path: evaluation.py:23-114, evaluation_704.py:57-115, utils_eval.py:19-53 ----
   Images are uint8 [C,H,W] (CHW) unless stated.  Metrics are written to a device double and
   computed from fixed-order block partials (deterministic); part must hold
   dn_eval_partials_size() bytes. */
size_t dn_eval_partials_size(void);
/* y = x / 255 (fp32)  -- evaluation.py:69 `noisy / 255.0` */
dn_status dn_u8_to_unit(const uint8_t* x, int64_t n, float* y, void* stream);
/* number of tiles per axis of the overlapping-tile loop (evaluation_704.py:80-81) */
int dn_tile_count(int extent, int patch, int stride);
/* tiles [nti*ntj, C, patch, patch] = img[:, r0:r0+patch, c0:c0+patch] / 255 with numpy 'reflect'
   padding of edge tiles, r0 = ti*stride, c0 = tj*stride (evaluation_704.py:84-93) */
dn_status dn_tile_extract(const uint8_t* img, int C, int H, int W, int patch, int stride,
                          float* tiles, void* stream);
/* out = sum_tiles clamp(pred,0,1)*wmask / sum wmask (0 -> 1), tiles in loop order; out_u8 =
   clip(out*255, 0, 255) truncated (evaluation_704.py:100-115).  Either output may be NULL. */
dn_status dn_tile_blend(const float* pred, int C, int H, int W, int patch, int stride,
                        const float* wmask, float* out, uint8_t* out_u8, void* stream);
/* y = uint8(clip(clamp(x,0,1)*255 [+ 0.5], 0, 255))  (evaluation.py:81-82 uses plus_half=1) */
dn_status dn_quantize_u8(const float* x, int64_t n, int plus_half, uint8_t* y, void* stream);
/* psnr = 10 log10(255^2 / mean((a-b)^2))  (utils_eval.py:49-53) over n uint8 values */
dn_status dn_psnr_u8(const uint8_t* a, const uint8_t* b, int64_t n, void* part, double* psnr,
                     void* stream);
/* mean SSIM (utils_eval.py:19-46): 11x11 Gaussian sigma 1.5, valid region [5,H-5)x[5,W-5),
   averaged over channels; hwc=1 for [H,W,C] images.  H, W > 10. */
dn_status dn_ssim_u8(const uint8_t* a, const uint8_t* b, int C, int H, int W, int hwc, void* part,
                     double* ssim, void* stream);
/* mean |a - b| (nn.L1Loss, evaluation.py:74) */
dn_status dn_l1_mean(const float* a, const float* b, int64_t n, void* part, double* l1,
                     void* stream);
/* l1[p] = mean |a[p] - b[p]| for P consecutive items of n floats (evaluation_704.py:98's
   criterion(prediction_patch, noisy_input) for every tile at once, one launch; fp64 sums) */
dn_status dn_l1_mean_batched(const float* a, const float* b, int64_t P, int64_t n, double* l1,
                             void* stream);

/* ---- adapter finetune: adapter.py:5-67 (OutputAdapter / DenoiserWithAdapter),
   finetune.py:153-162 (gradient_loss), finetune.py:269-289 (the step) ------------------------
   Adapter parameters are one flat fp32 buffer in OutputAdapter's state_dict order:
   net.0.weight [16,2C,3,3], net.0.bias [16], net.2.weight [C,16,3,3], net.2.bias [C]
   (449 floats for C=1, 1315 for C=3).  Only hidden_channels=16 (adapter.py:13) is built. */
dn_status dn_adapter_param_count(int in_channels, int hidden_channels, size_t* count);
/* out = base_out + conv2(relu(conv1(cat[noisy, base_out])))   (adapter.py:22-26); all NCHW */
dn_status dn_adapter_forward(const float* params, const float* noisy, const float* base_out,
                             float* out, int N, int C, int H, int W, int hidden_channels,
                             void* stream);
/* bytes of slab dn_adapter_backward needs (0 = unsupported arguments) */
size_t dn_adapter_slab_size(int N, int C, int H, int W, int hidden_channels);
/* dparams = dL/dparams of the adapter for dout = dL/dout (the base is frozen: no gradient
   flows into base_out or noisy, finetune.py:255-262).  Overwrites dparams; deterministic. */
dn_status dn_adapter_backward(const float* params, const float* noisy, const float* base_out,
                              const float* dout, float* dparams, int N, int C, int H, int W,
                              int hidden_channels, void* slab, size_t slab_bytes, void* stream);
/* loss = L1(pred, target) + lambda_grad * gradient_loss(pred, target)  (finetune.py:283-285);
   writes dpred = dloss/dpred and loss3 = {loss_l1, loss_grad, loss}.  partial_ws holds
   dn_loss_partials_size() bytes. */
dn_status dn_finetune_loss(const float* pred, const float* target, int N, int C, int H, int W,
                           float lambda_grad, float* dpred, float* loss3, void* partial_ws,
                           void* stream);

/* ---- ImprovedUNet: arch_unet.py:421-531 ImprovedUNet(in_nc, out_nc, n_feature=48, depth=4,
   noise=True) — the model train.sh / evaluation.py default to (train.py:311-313) --------------
   Same conventions as the UNet entry points: NCHW fp32 at the boundary, ONE flat fp32 parameter
   buffer in ImprovedUNet's state_dict order (noise_estimator.*, downs.*, bottle.*, ups.*,
   final.*; GroupNorm weight/bias included), H and W multiples of 16.  cfg->n_feature must be 48
   (the width train.py:30 uses); in_nc 1..3, out_nc 1..4. */
dn_status dn_iunet_param_count(const dn_unet_cfg* cfg, size_t* count);
dn_status dn_iunet_workspace_size(const dn_unet_cfg* cfg, int N, int H, int W, int with_backward,
                                  size_t* bytes);
/* y = sigmoid(...) = ImprovedUNet(x); keeps the activations for a backward when ws was sized
   with with_backward=1 */
dn_status dn_iunet_forward(const dn_unet_cfg* cfg, const float* params, const float* x, float* y,
                           int N, int H, int W, void* ws, size_t ws_bytes, void* stream);
/* dparams = dL/dparams for dy = dL/dy, using the activations the last dn_iunet_forward on ws
   saved.  Overwrites dparams; deterministic. */
dn_status dn_iunet_backward(const dn_unet_cfg* cfg, const float* params, const float* dy,
                            float* dparams, int N, int H, int W, void* ws, size_t ws_bytes,
                            void* stream);
/* dn_iunet_forward / dn_iunet_backward with the 3x3 convolutions' arithmetic chosen by
   precision: DN_PREC_FP32 or DN_PREC_FP32_X6 (forward and data gradient as exact split-bf16
   products; weight gradients, 1x1 convs and the noise estimator stay on the fp32 kernels). */
dn_status dn_iunet_forward_prec(const dn_unet_cfg* cfg, const float* params, const float* x,
                                float* y, int N, int H, int W, void* ws, size_t ws_bytes,
                                int precision, void* stream);
dn_status dn_iunet_backward_prec(const dn_unet_cfg* cfg, const float* params, const float* dy,
                                 float* dparams, int N, int H, int W, void* ws, size_t ws_bytes,
                                 int precision, void* stream);
/* Debug/introspection: (offset_floats, channel_stride, level) of the main NHWC activations:
   x0 h | down level i = 0..3: F r z1 a1 z2 | bottle: F r z1 a1 z2 | up k = 0..3: cc F r z1 a1 z2 |
   xb cf */
dn_status dn_iunet_debug_buffers(const dn_unet_cfg* cfg, int N, int H, int W, int with_backward,
                                 int64_t* desc, int max_entries, int* n_entries);

#ifdef __cplusplus
}
#endif

#endif /* DENOISE_HIP_H */
