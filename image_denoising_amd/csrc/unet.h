// Host-side U-Net plan and orchestration (internal).
#pragma once
#include <string>

#include "../../include/denoise_hip.h"
#include "dn_internal.h"

namespace dn {

enum LayerIdx {
  ENC0, ENC1, ENC2, ENC3, ENC4, ENC5, ENC6,
  UP5, D5A, D5B, UP4, D4A, D4B, UP3, D3A, D3B, UP2, D2A, D2B, UP1, D1A, D1B,
  NINA, NINB, NINC, NL
};

struct Layer {
  int cout, cin, k;
  bool deconv;   // ConvTranspose2d: weight [cin][cout][2][2]
  long woff;     // float offset of the weight in the flat buffer (bias follows)
  long wcount;
};

struct ParamLayout {
  Layer L[NL];
  long total;
};


struct Plan {
  ParamLayout P;
  int N, H, W, C, OC, nf;
  bool with_bwd;
  // forward activations (NHWC, offsets in floats)
  int c1s, c1k, c1kp;           // up1 concat: pixel stride, real channels, float4-padded K
  long c1, a0, a1;
  long c[5]; int cs[5], ck[5];  // concat buffers at levels 1..4: pixel stride, channels
  long a[5];                    // a2..a5 at levels 1..4
  long p5, a6;
  long da[5], db[5];            // decoder conv outputs at levels 1..4
  long d1a, d1b, na, nb;
  long packF[NL];               // packed forward weight images
  long packH;                   // fused head: nin_a | nin_b images (2 x HEAD_LW)
  long packUX[NL];              // bf16x6 parity images of the 96-channel deconvs (-1: none)
  long packBF[NL];              // bf16 images of the 3x3 layers (mixed-precision forward)
  long packX[NL];               // pre-split bf16x6 images of the 3x3 layers (forward)
  // forward-only plans, the N2N pair-pixel pass on the Winograd kernel (k_c3w6s): dec_conv1b's
  // tap-transposed PK_W6 image (y tiles) and the per-orientation cell lists (2 N cells uint32)
  // with their counts (2 N int); -1 in plans with a backward
  long packXV, w6s_list, w6s_cnt;
  long fwd_floats;
  // gradients
  long g_nb, g_na, g_d1b, g_d1a, g_c1;
  long g_c[5], g_da[5], g_db[5], g_a[5];
  long g_a6, g_p5, g_a0, g_a1;
  long xin;                     // compact NCHW copy of the network input (weight gradients)
  long packB[NL];               // packed data-gradient weight images
  long packXB[NL];              // pre-split bf16x6 data-gradient images of the 3x3 layers
  long packHB;                  // fused head backward: nin_b^T | nin_a^T images
  long packUXB[NL];             // bf16x6 data-gradient images of the 96-channel deconvs (-1: none)
  long zeros;                   // 64 zero floats (weight-gradient DMA padding)
  long slab[NL];                // per-layer weight-gradient slabs: [64 | splits x (W + b)]
  long slab_floats;             // all slabs
  int splits[NL];
  long total_floats;
};

void set_error(const std::string& s);
extern thread_local std::string g_last_error;
const char* layer_name(int i);
int layer_level(int i);
int dgrad_nout(const Plan& p, int i);
bool build_params(const dn_unet_cfg& c, ParamLayout& P, std::string& err);
bool build_plan(const dn_unet_cfg& c, int N, int H, int W, bool bwd, Plan& p, std::string& err);
// prec: DN_PREC_FP32 (fp32 matrix cores), DN_PREC_FP32_X6 (3x3 layers on the bf16 matrix cores
// by three-way operand splitting, fp32-accurate), DN_PREC_BF16 (forward only, bf16 operands)
// sel_rd (nullable, DN_PREC_FP32_X6 and no backward only): dec_conv1b and the head run on the
// two N2N pair pixels of every 2x2 cell only; y is written at those pixels and nowhere else
// pack: PACK_RUN packs the weight images into ws and runs; PACK_ONLY packs and returns (x, y
// unused; dn_unet_pack_weights); RUN_ONLY runs on the images a PACK_ONLY call left in ws
// (dn_unet_forward_prepacked: the same params, shape and precision; biases and the thin layers
// are still read from prm)
enum { PACK_RUN = 0, PACK_ONLY = 1, RUN_ONLY = 2 };
dn_status unet_forward(const Plan& p, const float* prm, const float* x, float* y, float* ws,
                       hipStream_t s, int prec = DN_PREC_FP32, const uint8_t* sel_rd = nullptr,
                       int pack = PACK_RUN);
// dx (nullable): dL/dx of the network input, NCHW [N, in_nc, H, W]
// tail_ready (nullable): recorded once dprm[tail_begin(p) ..] is final (dn_unet_backward_split)
dn_status unet_backward(const Plan& p, const float* prm, const float* dy, float* dprm, float* dx,
                        float* ws, hipStream_t s, int prec = DN_PREC_FP32,
                        hipEvent_t tail_ready = nullptr);
// first float of the parameter range the backward finishes early (dec_conv5a .. nin_c)
// The backward's side streams (unet.cpp): weight gradients on `st`, slab reductions on `rst`,
// with their fork / join events; one set per host thread and device (nullptr when creating them
// failed: run on one stream).  Shared by the UNet and ImprovedUNet executors.
struct SideStream {
  hipStream_t st = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  // the slab reductions' own stream (round 6): a flush there overlaps both the data-gradient
  // chain and the remaining weight gradients instead of delaying the latter on `st`
  hipStream_t rst = nullptr;
  hipEvent_t rfork = nullptr, rjoin = nullptr;
};
SideStream* side_stream(hipStream_t s);

long tail_begin(const Plan& p);
// zc of the bf16x6 data gradient of a 3x3 layer producing nout channels (0: one block)
int x6_dgrad_zc(int nout);

WView conv_fwd_view(const float* w, int K, int ksize);
WView conv_dgrad_view(const float* w, int cin_total, int ksize);
WView deconv_fwd_view(const float* w, int cout);
WView deconv_dgrad_view(const float* w, int cout);
long conv_fwd_pack_size(int K, int cout, int ksize);
long conv_dgrad_pack_size(int cout, int nout, int ksize);
long deconv_fwd_pack_size(int cin, int cout);
long deconv_dgrad_pack_size(int cout, int cin);
hipError_t pack_conv_fwd(const float* w, int K, int cout, int ksize, float* out, hipStream_t s);
hipError_t pack_conv_dgrad(const float* w, int cin_total, int nout, int cout, int ksize, float* out,
                           hipStream_t s);
hipError_t pack_deconv_fwd(const float* w, int cin, int cout, float* out, hipStream_t s);
hipError_t pack_deconv_dgrad(const float* w, int cout, int cin, float* out, hipStream_t s);
hipError_t conv_forward(const View& in, int N, int H, int W, int K, const float* wp,
                        const float* b, int cout, int ksize, int act, const View& out,
                        int out_layout, hipStream_t s);
hipError_t conv_dgrad(const View& dz, int N, int H, int W, int cout, const float* wp, int nout,
                      int ksize, int epi, const View& mask, const View& dx, hipStream_t s);
hipError_t deconv_forward(const View& x, int N, int h, int w, int cin, const float* wp,
                          const float* b, int cout, const View& out, hipStream_t s);
hipError_t deconv_dgrad(const View& dy, int N, int h, int w, int cout, const float* wp, int cin,
                        const View& mask, int epi, const View& dx, hipStream_t s);
// slab: [64 floats | splits x (W + b)]; zeros == nullptr: the 64 floats are zeroed here and
// serve as the DMA padding; rb: the reduction is queued, not launched
hipError_t wgrad(int mode, const View& g, const View& x, int N, int KH, int KW, int cout, int cin,
                 float* dwb, float* slab, int splits, hipStream_t s, bool x6 = false,
                 const float* zeros = nullptr, RedBatch* rb = nullptr, int head_gnb = 0,
                 const float* hd_dy = nullptr, int hd_dy_stride = 0, const float* hd_wc = nullptr,
                 float* hd_slab_c = nullptr, float* hd_dwc = nullptr);

}  // namespace dn
