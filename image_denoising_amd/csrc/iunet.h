// Host-side plan and orchestration of ImprovedUNet (arch_unet.py:421-531) — internal.
#pragma once
#include <string>

#include "../../include/denoise_hip.h"
#include "dn_internal.h"

namespace dn {

// offsets (floats) of one layer's tensors in the flat parameter buffer
struct IConv { long w = -1, b = -1; int cout = 0, cin = 0, k = 3; };
struct IGN { long g = -1, b = -1; int C = 0, G = 0; };
struct IRdb { IConv conv[4]; IConv lff; int C = 0; };
struct IRes { IConv c1, c2; IGN n1, n2; int C = 0; };
struct ILevel { IConv conv; IRdb rdb; IRes res; };
struct IUp { IConv ps, fuse; IRdb rdb; IRes res; int in = 0, out = 0; };

struct IParams {
  int C = 1, OC = 1, nf = 48;
  IConv ne0, ne2;
  ILevel down[4];
  IRdb brdb;
  IRes bres;
  IUp up[4];
  IConv fin;
  long total = 0;
};

// activations of one RDB + ResBlock pair at one resolution
struct IBlockBufs {
  long F = 0;          // [x | o0..o3]  (C + 128 channels)
  long r = 0;          // RDB output (C)
  long z1 = 0, a1 = 0, z2 = 0;  // ResBlock conv1 out, leaky(GN1), conv2 out
  long st1 = 0, st2 = 0;        // GN stats (mean, rstd) per (n, group)
  // gradients
  // (dzj per growth conv, dzf = the up block's fuse-conv gradient: the weight gradients read
  // them on the side stream while the data-gradient chain goes on)
  long dF = 0, dr = 0, dz2 = 0, dg1 = 0, dz1 = 0, dzj[4] = {0, 0, 0, 0}, dzf = 0;
};

struct IPlan {
  IParams P;
  int N = 0, H = 0, W = 0;
  bool with_bwd = false;
  long x0 = 0, h = 0;                 // [x, sigma, 0] (stride 4); noise-estimator hidden (48)
  long xin = 0, yout = 0, sig = 0;    // NCHW copies of the input / output, sigma map (NCHW)
  IBlockBufs dl[4], bb, ul[4];        // down levels, bottle, up blocks
  long pool[4] = {0, 0, 0, 0};        // pooled input of down level i (i >= 1)
  long cc[4] = {0, 0, 0, 0};          // up-block concat [u | skip]  (3*out)
  long xb = 0;                        // bottle output (384)
  long xu[3] = {0, 0, 0};             // up-block outputs 0..2
  long cf = 0;                        // final concat [x_up3 (24) | x (C) | 0]  stride 28
  long sc = 0, sh = 0;                // GN scale / shift scratch [N * 384]
  long gpart = 0;                     // GN partial sums (doubles)
  long pack = 0, pack_floats = 0;     // packed-weight arena (one slot per conv of a pass)
  // gradients
  long dzfin = 0, dcc[4] = {0, 0, 0, 0}, dps[4] = {0, 0, 0, 0}, dxu[3] = {0, 0, 0}, dxb = 0, dpool = 0;
  long dza[4] = {0, 0, 0, 0}, dsg = 0, dh = 0, ca = 0, cb = 0, ccf = 0;
  long slab = 0, slab_floats = 0;
  long total_floats = 0;
};

bool iunet_build_params(const dn_unet_cfg& c, IParams& P, std::string& err);
bool iunet_build_plan(const dn_unet_cfg& c, int N, int H, int W, bool bwd, IPlan& p,
                      std::string& err);
// prec: DN_PREC_FP32, or DN_PREC_FP32_X6 (the 3x3 convs' forward and data gradient as split
// bf16 products, conv_x6.hip)
dn_status iunet_forward(const IPlan& p, const float* prm, const float* x, float* y, float* ws,
                        hipStream_t s, int prec = DN_PREC_FP32);
dn_status iunet_backward(const IPlan& p, const float* prm, const float* dy, float* dprm,
                         float* ws, hipStream_t s, int prec = DN_PREC_FP32);

}  // namespace dn
