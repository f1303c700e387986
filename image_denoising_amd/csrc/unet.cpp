// U-Net orchestration for the N2N training path: parameter layout (reference state_dict
// order), workspace plan (NHWC activation arena, gradient buffers, weight-gradient slabs),
// and the forward / backward launch sequences.  Mirrors arch_unet.py:100-260 (UNet) and
// the autograd graph that `loss.backward()` replays for it.
#include "unet.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>

namespace dn {

thread_local std::string g_last_error;

void set_error(const std::string& s) { g_last_error = s; }

// ------------------------------------------------------------------------------------
// parameters: arch_unet.py:115-192 registration order (== state_dict order)
// ------------------------------------------------------------------------------------
static const char* kNames[NL] = {
    "enc_conv0", "enc_conv1", "enc_conv2", "enc_conv3", "enc_conv4", "enc_conv5", "enc_conv6",
    "up5.deconv", "dec_conv5a", "dec_conv5b", "up4.deconv", "dec_conv4a", "dec_conv4b",
    "up3.deconv", "dec_conv3a", "dec_conv3b", "up2.deconv", "dec_conv2a", "dec_conv2b",
    "up1.deconv", "dec_conv1a", "dec_conv1b", "nin_a", "nin_b", "nin_c"};

const char* layer_name(int i) { return (i >= 0 && i < NL) ? kNames[i] : ""; }

bool build_params(const dn_unet_cfg& c, ParamLayout& P, std::string& err) {
  const int C = c.in_nc, OC = c.out_nc, nf = c.n_feature;
  if (C < 1 || C > 4 || OC < 1 || OC > 16) {
    err = "in_nc must be in [1,4] and out_nc in [1,16]";
    return false;
  }
  if (nf != 48) {
    err = "n_feature must be 48 (kernel tiles are instantiated for the reference width)";
    return false;
  }
  auto conv = [&](int i, int cout, int cin, int k) { P.L[i] = {cout, cin, k, false, 0, 0}; };
  auto dec = [&](int i, int cin, int cout) { P.L[i] = {cout, cin, 2, true, 0, 0}; };
  conv(ENC0, nf, C, 3);
  for (int i = ENC1; i <= ENC6; ++i) conv(i, nf, nf, 3);
  dec(UP5, nf, nf);
  conv(D5A, 2 * nf, 2 * nf, 3);
  conv(D5B, 2 * nf, 2 * nf, 3);
  dec(UP4, 2 * nf, 2 * nf);
  conv(D4A, 2 * nf, 3 * nf, 3);
  conv(D4B, 2 * nf, 2 * nf, 3);
  dec(UP3, 2 * nf, 2 * nf);
  conv(D3A, 2 * nf, 3 * nf, 3);
  conv(D3B, 2 * nf, 2 * nf, 3);
  dec(UP2, 2 * nf, 2 * nf);
  conv(D2A, 2 * nf, 3 * nf, 3);
  conv(D2B, 2 * nf, 2 * nf, 3);
  dec(UP1, 2 * nf, 2 * nf);
  conv(D1A, 96, 2 * nf + C, 3);  // arch_unet.py:177 (hard-wired 96)
  conv(D1B, 96, 96, 3);
  conv(NINA, 96, 96, 1);
  conv(NINB, 96, 96, 1);
  conv(NINC, OC, 96, 1);
  long off = 0;
  for (int i = 0; i < NL; ++i) {
    Layer& L = P.L[i];
    L.wcount = (long)L.cout * L.cin * L.k * L.k;
    L.woff = off;
    off += L.wcount + L.cout;
  }
  P.total = off;
  return true;
}

// ------------------------------------------------------------------------------------
// workspace plan (offsets in floats, 256-byte aligned)
// ------------------------------------------------------------------------------------
int dgrad_nout(const Plan& p, int i);

bool build_plan(const dn_unet_cfg& c, int N, int H, int W, bool bwd, Plan& p, std::string& err) {
  if (N < 1 || H < 32 || W < 32 || (H % 32) || (W % 32)) {
    err = "N >= 1 and H, W must be positive multiples of 32 (5 pooling levels)";
    return false;
  }
  if (!build_params(c, p.P, err)) return false;
  p.N = N; p.H = H; p.W = W;
  p.C = c.in_nc; p.OC = c.out_nc; p.nf = c.n_feature;
  const int nf = p.nf;
  long off = 0;
  auto px = [&](int lvl) { return (long)N * (H >> lvl) * (W >> lvl); };
  auto alloc = [&](int lvl, int ch) {
    long o = off;
    off += (px(lvl) * ch + 63) / 64 * 64;
    return o;
  };
  p.c1k = 2 * nf + p.C;             // [up1 | x] channels
  p.c1kp = (p.c1k + 3) / 4 * 4;     // ... padded to float4 (pad channels kept at zero)
  // pixel stride of forward-only plans (the N2N target pass, the frozen finetune base, eval): a
  // multiple of 32 channels (128 B), so the deconv's 384-B pixel writes and dec_conv1a's 128-B
  // chunk reads stay line-aligned (stride 100: 400-B pixels, every 64-B piece split over two
  // lines; the 256^2 deconv measured 0.88 ms at stride 100, 0.64 at 96); channels [c1kp, c1s)
  // are never written or read.  Plans with a backward keep the float4 stride (measured faster
  // there).  DN_C1S_ALIGN=4 / 32 forces either.
  static const int c1s_env = getenv("DN_C1S_ALIGN") ? atoi(getenv("DN_C1S_ALIGN")) : 0;
  const int c1s_align = c1s_env > 0 ? c1s_env : (bwd ? 4 : 32);
  p.c1s = (p.c1k + c1s_align - 1) / c1s_align * c1s_align;
  p.c1 = alloc(0, p.c1s);
  p.a0 = alloc(0, nf);
  p.a1 = alloc(0, nf);
  for (int l = 1; l <= 4; ++l) {  // c2..c5 concat buffers (c5 is [u5 | p4] = 2nf)
    p.ck[l] = (l == 4) ? 2 * nf : 3 * nf;
    // forward-only plans: pixel stride a multiple of 32 channels like c1 (144 -> 160: 640-B
    // pixels, the deconv / pool writes and the 128-B chunk reads line-aligned)
    const int a = c1s_env > 0 ? c1s_env : (bwd ? 1 : 32);
    p.cs[l] = (p.ck[l] + a - 1) / a * a;
    p.c[l] = alloc(l, p.cs[l]);
  }
  for (int l = 1; l <= 4; ++l) p.a[l] = alloc(l, nf);  // a2..a5 live at levels 1..4
  p.p5 = alloc(5, nf);
  p.a6 = alloc(5, nf);
  for (int l = 1; l <= 4; ++l) {
    p.da[l] = alloc(l, 2 * nf);
    p.db[l] = alloc(l, 2 * nf);
  }
  p.d1a = alloc(0, 96);
  p.d1b = alloc(0, 96);
  p.na = alloc(0, 96);
  p.nb = alloc(0, 96);
  // packed forward weights (rebuilt by every dn_unet_forward from the flat parameters)
  auto alloc_f = [&](long n) {
    long o = off;
    off += (n + 63) / 64 * 64;
    return o;
  };
  for (int i = 0; i < NL; ++i) {
    const Layer& L = p.P.L[i];
    const long n = L.deconv ? deconv_fwd_pack_size(L.cin, L.cout)
                            : conv_fwd_pack_size(L.cin, L.cout, L.k);
    if (n < 0) {
      err = std::string("no forward kernel tile for layer ") + kNames[i];
      return false;
    }
    p.packF[i] = alloc_f(n);
  }
  p.packH = alloc_f(2 * HEAD_LW > X6_HEAD_BF ? 2 * HEAD_LW : X6_HEAD_BF);  // fp32 | bf16x6 head images
  for (int i = 0; i < NL; ++i) {  // 4 x X6_HEAD_BF bf16 per 96-channel deconv
    const Layer& L = p.P.L[i];
    p.packUX[i] = (L.deconv && L.cin == 96 && L.cout == 96) ? alloc_f(2 * X6_HEAD_BF) : -1;
  }
  for (int i = 0; i < NL; ++i) {  // bf16 images (2 bytes each) of the 3x3 layers
    const Layer& L = p.P.L[i];
    p.packBF[i] = -1;
    if (i == ENC0 || i == NINC) continue;  // 3x3 layers, deconvs, nin_a / nin_b
    const long e = L.deconv ? 4 * bf16_pack_elems(L.cin, L.cout, 1) : bf16_pack_elems(L.cin, L.cout, L.k);
    if (e < 0) {
      err = std::string("no bf16 forward tile for layer ") + kNames[i];
      return false;
    }
    p.packBF[i] = alloc_f((e + 1) / 2);
  }
  for (int i = 0; i < NL; ++i) {  // bf16x6 (split fp32) images of the 3x3 layers
    const Layer& L = p.P.L[i];
    p.packX[i] = -1;
    if (i == ENC0 || L.deconv || L.k != 3) continue;
    const long e = x6_pack_elems(L.cin, L.cout, 0);
    if (e < 0) {
      err = std::string("no bf16x6 forward tile for layer ") + kNames[i];
      return false;
    }
    p.packX[i] = alloc_f((e + 1) / 2);
  }
  p.packXV = p.w6s_list = p.w6s_cnt = -1;
  if (!bwd) {
    p.packXV = alloc_f((x6_pack_elems(96, 96, 0) + 1) / 2);
    p.w6s_list = alloc_f(2L * N * (H / 2) * (W / 2));
    p.w6s_cnt = alloc_f(2L * N);
  }
  p.fwd_floats = off;
  if (bwd) {
    p.g_nb = alloc(0, 96);
    p.g_na = alloc(0, 96);
    p.g_d1b = alloc(0, 96);
    p.g_d1a = alloc(0, 96);
    p.g_c1 = alloc(0, 2 * nf);
    for (int l = 1; l <= 4; ++l) {
      p.g_c[l] = alloc(l, p.cs[l]);
      p.g_da[l] = alloc(l, 2 * nf);
      p.g_db[l] = alloc(l, 2 * nf);
      p.g_a[l] = alloc(l, nf);
    }
    p.g_a6 = alloc(5, nf);
    p.g_p5 = alloc(5, nf);
    p.g_a0 = alloc(0, nf);
    p.g_a1 = alloc(0, nf);
    p.xin = alloc(0, p.C);
    for (int i = 0; i < NL; ++i) {  // packed data-gradient weights
      const Layer& L = p.P.L[i];
      long n = 0;
      if (i == ENC0) n = 0;  // the network input needs no gradient
      else if (L.deconv) n = deconv_dgrad_pack_size(L.cout, L.cin);
      else n = conv_dgrad_pack_size(L.cout, dgrad_nout(p, i), L.k);
      if (n < 0) {
        err = std::string("no data-gradient kernel tile for layer ") + kNames[i];
        return false;
      }
      p.packB[i] = alloc_f(n);
    }
    p.packHB = alloc_f(2 * HEAD_LW > X6_HEAD_BF ? 2 * HEAD_LW : X6_HEAD_BF);  // fp32 | bf16x6 (Wb^T | Wa^T)
    for (int i = 0; i < NL; ++i)  // 4 x X6_HEAD_BF bf16 per 96-channel deconv
      p.packUXB[i] = p.packUX[i] >= 0 ? alloc_f(2 * X6_HEAD_BF) : -1;
    for (int i = 0; i < NL; ++i) {  // bf16x6 data-gradient images of the 3x3 layers
      const Layer& L = p.P.L[i];
      p.packXB[i] = -1;
      if (i == ENC0 || L.deconv || L.k != 3) continue;
      const int nout = dgrad_nout(p, i);
      const long e = x6_pack_elems(L.cout, nout, x6_dgrad_zc(nout));
      if (e < 0) {
        err = std::string("no bf16x6 data-gradient tile for layer ") + kNames[i];
        return false;
      }
      p.packXB[i] = alloc_f((e + 1) / 2);
    }
    // weight-gradient slabs, one per layer (the backward queues every layer's reduction and
    // launches them together at its end): splits * (W + b) after 64 floats
    p.zeros = alloc_f(64);
    p.slab_floats = 0;
    for (int i = 0; i < NL; ++i) {
      const Layer& L = p.P.L[i];
      int lvl = layer_level(i);
      int KH = H >> lvl, KW = W >> lvl;
      int mode = L.deconv ? W_UP2 : (L.k == 3 ? W_C3 : W_C1);
      if (L.deconv) { KH = H >> (lvl + 1); KW = W >> (lvl + 1); }
      int sp = i == ENC0   ? enc0_wgrad_splits(N, KH, KW)
               : (i == NINC && p.OC <= 4) ? wgrad_thin_splits((long)N * KH * KW)
                           : wgrad_splits(mode, N, KH, KW, i == D1A ? 2 * nf : L.cin, L.cout);
      p.splits[i] = sp;
      long need = (i == ENC0 || i == D1A || (i == NINC && p.OC <= 4))
                      ? (long)sp * (L.wcount + L.cout)
                      : wgrad_slab_floats(mode, N, KH, KW, L.cin, L.cout);
      // (nin_c: also the rows nin_b's k_wgrad1p<., GNB> writes its weight gradient into)
      if (i == NINC && p.OC <= 4) {
        const long s1 = wgrad1_splits(W_C1, N, KH, KW);
        if (s1 * (L.wcount + L.cout) > need) need = s1 * (L.wcount + L.cout);
      }
      if (i == D1A) need += (long)enc0_wgrad_splits(N, KH, KW) * 96 * p.C * 9;  // input slice
      p.slab[i] = alloc_f(64 + need);
      p.slab_floats += 64 + need;
    }
  }
  p.total_floats = off;
  p.with_bwd = bwd;
  return true;
}

int x6_dgrad_zc(int nout) { return nout <= 96 ? 0 : 48; }

// channels of the data gradient a layer's backward must produce
int dgrad_nout(const Plan& p, int i) {
  if (i == D1A) return 2 * p.nf;  // only the up1 part of [up1 | x]
  return p.P.L[i].cin;
}

// output level of every layer (deconvs: level of their OUTPUT)
int layer_level(int i) {
  switch (i) {
    case ENC0: case ENC1: return 0;
    case ENC2: return 1;
    case ENC3: return 2;
    case ENC4: return 3;
    case ENC5: return 4;
    case ENC6: return 5;
    case UP5: case D5A: case D5B: return 4;
    case UP4: case D4A: case D4B: return 3;
    case UP3: case D3A: case D3B: return 2;
    case UP2: case D2A: case D2B: return 1;
    default: return 0;  // UP1, D1A, D1B, NIN*
  }
}

// ------------------------------------------------------------------------------------
// op helpers
// ------------------------------------------------------------------------------------
#define DN_TRY(x)                                                         \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      set_error(std::string("HIP error in ") + #x + ": " + hipGetErrorString(e_)); \
      return DN_ERR_HIP;                                                  \
    }                                                                     \
  } while (0)

WView conv_fwd_view(const float* w, int K, int ksize) {
  return ksize == 3 ? WView{w, 0, 9, (long)K * 9, 1, 0, 9, 0} : WView{w, 0, 1, (long)K, 0, 0, 1, 0};
}
WView conv_dgrad_view(const float* w, int cin_total, int ksize) {  // flipped + transposed
  return ksize == 3 ? WView{w, 0, (long)cin_total * 9, 9, 1, 0, 9, 1}
                    : WView{w, 0, (long)cin_total, 1, 0, 0, 1, 0};
}
WView deconv_fwd_view(const float* w, int cout) { return WView{w, 0, (long)cout * 4, 4, 0, 1, 1, 0}; }
WView deconv_dgrad_view(const float* w, int cout) { return WView{w, 0, 4, (long)cout * 4, 1, 0, 4, 0}; }

long conv_fwd_pack_size(int K, int cout, int ksize) {
  return pack_floats(ksize == 3 ? G_C3 : G_C1, cout, K, 1);
}
long conv_dgrad_pack_size(int cout, int nout, int ksize) {
  return pack_floats(ksize == 3 ? G_C3 : G_C1, nout, cout, 1);
}
long deconv_fwd_pack_size(int cin, int cout) { return pack_floats(G_UP, cout, cin, 4); }
long deconv_dgrad_pack_size(int cout, int cin) { return pack_floats(G_DN2, cin, cout, 1); }

hipError_t pack_conv_fwd(const float* w, int K, int cout, int ksize, float* out, hipStream_t s) {
  return launch_pack(ksize == 3 ? G_C3 : G_C1, conv_fwd_view(w, K, ksize), K, cout, 1, out, s);
}
hipError_t pack_conv_dgrad(const float* w, int cin_total, int nout, int cout, int ksize, float* out,
                           hipStream_t s) {
  return launch_pack(ksize == 3 ? G_C3 : G_C1, conv_dgrad_view(w, cin_total, ksize), cout, nout, 1,
                     out, s);
}
hipError_t pack_deconv_fwd(const float* w, int cin, int cout, float* out, hipStream_t s) {
  return launch_pack(G_UP, deconv_fwd_view(w, cout), cin, cout, 4, out, s);
}
hipError_t pack_deconv_dgrad(const float* w, int cout, int cin, float* out, hipStream_t s) {
  return launch_pack(G_DN2, deconv_dgrad_view(w, cout), cout, cin, 1, out, s);
}

hipError_t conv_forward(const View& in, int N, int H, int W, int K, const float* wp,
                        const float* b, int cout, int ksize, int act, const View& out,
                        int out_layout, hipStream_t s) {
  FwdArgs a{};
  a.in = in.p; a.in_stride = in.stride; a.in_off = in.off; a.IHt = H; a.IWt = W;
  a.N = N; a.OH = H; a.OW = W; a.K = K; a.NOUT = cout;
  a.wp = wp; a.wp_z = 0;
  a.bias = b; a.epi = act ? EPI_BIAS_ACT : EPI_BIAS;
  a.out = out.p; a.out_stride = out.stride; a.out_off = out.off; a.out_layout = out_layout;
  return launch_fwd(ksize == 3 ? G_C3 : G_C1, a, s);
}

// dx (channels [0, nout)) from dz [N,H,W,cout]; wp = pack_conv_dgrad(...)
hipError_t conv_dgrad(const View& dz, int N, int H, int W, int cout, const float* wp, int nout,
                      int ksize, int epi, const View& mask, const View& dx, hipStream_t s) {
  FwdArgs a{};
  a.in = dz.p; a.in_stride = dz.stride; a.in_off = dz.off; a.IHt = H; a.IWt = W;
  a.N = N; a.OH = H; a.OW = W; a.K = cout; a.NOUT = nout;
  a.wp = wp; a.wp_z = 0;
  a.bias = nullptr; a.epi = epi;
  a.out = dx.p; a.out_stride = dx.stride; a.out_off = dx.off; a.out_layout = OUT_NHWC;
  a.mask = mask.p; a.mask_stride = mask.stride; a.mask_off = mask.off;
  return launch_fwd(ksize == 3 ? G_C3 : G_C1, a, s);
}

// ConvTranspose2d(cin, cout, 2, 2): x [N,h,w,cin] -> out at (2y+a, 2x+b); wp = pack_deconv_fwd
hipError_t deconv_forward(const View& x, int N, int h, int w, int cin, const float* wp,
                          const float* b, int cout, const View& out, hipStream_t s) {
  FwdArgs a{};
  a.in = x.p; a.in_stride = x.stride; a.in_off = x.off; a.IHt = h; a.IWt = w;
  a.N = N; a.OH = h; a.OW = w; a.K = cin; a.NOUT = cout;
  a.wp = wp; a.wp_z = pack_floats(G_UP, cout, cin, 1);
  a.bias = b; a.epi = EPI_BIAS;
  a.out = out.p; a.out_stride = out.stride; a.out_off = out.off; a.out_layout = OUT_UP2;
  return launch_fwd(G_UP, a, s);
}

// dx [N,h,w,cin] = sum_{ab,co} dy[2y+a][2x+b][co] * W[ci][co][ab]  (* leaky'(mask));
// wp = pack_deconv_dgrad
hipError_t deconv_dgrad(const View& dy, int N, int h, int w, int cout, const float* wp, int cin,
                        const View& mask, int epi, const View& dx, hipStream_t s) {
  FwdArgs a{};
  a.in = dy.p; a.in_stride = dy.stride; a.in_off = dy.off; a.IHt = 2 * h; a.IWt = 2 * w;
  a.N = N; a.OH = h; a.OW = w; a.K = cout; a.NOUT = cin;
  a.wp = wp; a.wp_z = 0;
  a.bias = nullptr; a.epi = epi;
  a.out = dx.p; a.out_stride = dx.stride; a.out_off = dx.off; a.out_layout = OUT_NHWC;
  a.mask = mask.p; a.mask_stride = mask.stride; a.mask_off = mask.off;
  return launch_fwd(G_DN2, a, s);
}

hipError_t wgrad(int mode, const View& g, const View& x, int N, int KH, int KW, int cout, int cin,
                 float* dwb, float* slab, int splits, hipStream_t s, bool x6, const float* zeros,
                 RedBatch* rb, int head_gnb, const float* hd_dy, int hd_dy_stride,
                 const float* hd_wc, float* hd_slab_c, float* hd_dwc) {
  WgradArgs a{};
  a.head_gnb = head_gnb; a.hd_dy = hd_dy; a.hd_dy_stride = hd_dy_stride; a.hd_wc = hd_wc;
  a.hd_slab_c = hd_slab_c; a.hd_dwc = hd_dwc;
  a.g = g.p; a.g_stride = g.stride; a.g_off = g.off;
  a.x = x.p; a.x_stride = x.stride; a.x_off = x.off;
  a.N = N; a.KH = KH; a.KW = KW; a.Cout = cout; a.Cin = cin;
  const int taps = mode == W_C3 ? 9 : (mode == W_UP2 ? 4 : 1);
  const long n = (long)cout * cin * taps + cout;
  const OpTimer timer(s, mode == W_C3 ? "wgrad3" : (mode == W_UP2 ? "wgrad_up" : "wgrad1"),
                      2.0 * N * KH * KW * cout * cin * taps, cin, cout, KH, KW, N);
  // slab scratch layout: [64 floats | splits x (W + b)]
  a.zeros = zeros ? zeros : slab;
  a.slab = slab + 64; a.slab_stride = n;
  a.wlayout = mode == W_UP2 ? 1 : 0;
  a.cin_total = cin; a.ci_base = 0; a.bias = 1;
  if (!zeros) {
    hipError_t e = hipMemsetAsync(slab, 0, 64 * sizeof(float), s);
    if (e != hipSuccess) return e;
  }
  // 1x1 / deconv, own splits (x6: the 96 x 96 1x1 layers on k_wgrad1p)
  if (wgrad1_ok(mode, a)) return launch_wgrad1(mode, a, dwb, s, rb, x6);
  if (x6 && mode == W_C3) splits = wgrad_splits_x6(a, splits);
  hipError_t e = launch_wgrad(mode, a, splits, s, x6);
  if (e != hipSuccess) return e;
  return launch_reduce(slab + 64, n, splits, n, dwb, s, rb);
}

// ------------------------------------------------------------------------------------
// forward: arch_unet.py:194-260 (non-blind-spot branch)
// ------------------------------------------------------------------------------------
dn_status unet_forward(const Plan& p, const float* prm, const float* x, float* y, float* ws,
                       hipStream_t s, int prec, const uint8_t* sel_rd, int pack) {
  const StreamDeviceGuard device_guard(s);
  const bool bf16 = prec == DN_PREC_BF16, x6 = prec == DN_PREC_FP32_X6;
  // (bf16x6 96-channel deconvs: k_deconv_x6)
  const int N = p.N, nf = p.nf, C = p.C;
  auto H = [&](int l) { return p.H >> l; };
  auto Wd = [&](int l) { return p.W >> l; };
  auto Wt = [&](int i) { return ws + p.packF[i]; };  // packed forward weights
  auto Bs = [&](int i) { return prm + p.P.L[i].woff + p.P.L[i].wcount; };
  auto V = [&](long off, int stride, int coff = 0) { return View{ws + off, stride, coff}; };
  // every 3x3 layer (enc_conv1..dec_conv1b): the fp32 kernel, the bf16x6 one (split fp32
  // operands on the bf16 matrix cores), or the bf16 one (bf16 operands, fp32 accumulation /
  // bias / activation / storage)
  // the pipelined split-bf16 kernel takes a partial last K chunk (dec_conv1a's x channels,
  // the 48-channel encoder's second chunk) packed over fewer stages (x6_tail_mode)
  // (x6_image_mode: | X6_W6 for the Winograd kernel on the 96- and 48-output layers from one
  // round of 8 x 16 tiles)
  // the encoder's 2x2 max-pools fused into the x6 convs' epilogues (DN_POOL_FUSE=0: separate
  // k_pool_fwd launches, A/B)
  static const bool pool_fuse = !getenv("DN_POOL_FUSE") || atoi(getenv("DN_POOL_FUSE")) != 0;
  // (the N2N pair-pixel pass's dec_conv1b runs the Winograd kernel k_c3w6s wherever the full
  // forward's dec_conv1b has a Winograd image; the direct k_c3x6s below one round of tiles)
  auto x6_tail_f = [&](int i) -> int {
    const Layer& L = p.P.L[i];
    const int l = layer_level(i);
    const int m = x6_image_mode(N, H(l), Wd(l), i == D1A ? p.c1kp : L.cin, L.cout, 0, true);
    // dec_conv1a at C = 1 on the Winograd kernel: the image channel alone in the last chunk
    return m | (i == D1A && (m & X6_W6) && (m & 7) == 1 && L.cin % 32 == 1 && L.cout == 96 ? X6_T1 : 0);
  };
  // bf16 base (forward-only plans): bf16 storage of the decoder's a-conv outputs, whose only
  // reader is the matching b-conv
  const bool bf16_store = bf16 && !p.with_bwd;
  // (bf16 base: the fused head kernel in plain bf16 products, see below; it reads d1b as bf16)
  const bool bf16_head_x6 = bf16 && !p.with_bwd && p.OC <= X6_HEAD_OCMAX;
  auto bf16_store_out = [&](int i) {
    if (i == D1B) return bf16_store && bf16_head_x6 && p.packBF[i] >= 0;
    return bf16_store && (i == D1A || i == D2A || i == D3A || i == D4A || i == D5A) &&
           p.packBF[i] >= 0 && p.packBF[i + 1] >= 0;
  };
  // enc_conv0's output too: only enc_conv1 reads it in a forward-only plan
  const bool enc0_bf16 = bf16_store && p.packBF[ENC1] >= 0;
  auto bf16_store_in = [&](int i) {
    if (i == ENC1) return enc0_bf16;
    return bf16_store && (i == D1B || i == D2B || i == D3B || i == D4B || i == D5B) &&
           bf16_store_out(i - 1);
  };
  // (dec_conv1b -> the bf16 head: bf16_store_out(D1B))
  // pool (x6 path, EPI_BIAS_ACT): the 2x2 max-pool of `out` fused into the conv's epilogue into
  // that view (*pooled set); otherwise the caller pools
  // forward-only plans: an encoder conv whose pool is fused stores only the pooled output
  // (its full-resolution activation is read by nothing but that pool; the backward's pool
  // routing reads it in plans with a backward)
  const int pool_only = !p.with_bwd ? 1 : 0;
  auto conv_forward = [&](const View& in, int Nn, int h, int w, int K, const float* wp,
                          const float* b, int cout, int ksize, int act, const View& out,
                          int layout, hipStream_t st, const View* pool = nullptr,
                          bool* pooled = nullptr) -> hipError_t {
    if (pooled) *pooled = false;
    const OpTimer timer(st, ksize == 3 ? "fwd3" : "fwd1",
                        2.0 * Nn * h * w * K * cout * ksize * ksize, K, cout, h, w, Nn);
    int i = ENC1;
    while (i < NL && Wt(i) != wp) ++i;
    if (x6 && i < NL && p.packX[i] >= 0) {
      FwdArgs a{};
      a.in = in.p; a.in_stride = in.stride; a.in_off = in.off; a.IHt = h; a.IWt = w;
      a.N = Nn; a.OH = h; a.OW = w; a.K = K; a.NOUT = cout;
      // dec_conv1a reads [up1 | x | zero pad] (c1kp = c1k rounded to 4): taking the zero pad
      // channel as a reduction channel (its packed weights are zero) keeps K % 4 == 0
      if (i == D1A) a.K = p.c1kp;
      a.x6_tail = x6_tail_f(i);  // a partial last K chunk packed over fewer stages
      if (a.x6_tail & X6_T1) a.in_t1 = x;  // the image channel straight from the network input
      a.wp = ws + p.packX[i]; a.bias = b; a.epi = act ? EPI_BIAS_ACT : EPI_BIAS;
      a.out = out.p; a.out_stride = out.stride; a.out_off = out.off; a.out_layout = layout;
      if (pool && pool_fuse && act && layout == OUT_NHWC) {
        a.pool_out = pool->p; a.pool_stride = pool->stride; a.pool_off = pool->off;
        a.pool_only = pool_only;
        if (pooled) *pooled = true;
      }
      return launch_fwd_x6(a, st);
    }
    if (!bf16 || i == NL || p.packBF[i] < 0)
      return dn::conv_forward(in, Nn, h, w, K, wp, b, cout, ksize, act, out, layout, st);
    FwdArgs a{};
    a.in = in.p; a.in_stride = in.stride; a.in_off = in.off; a.IHt = h; a.IWt = w;
    a.N = Nn; a.OH = h; a.OW = w; a.K = K; a.NOUT = cout;
    if (i == D1A) a.K = p.c1kp;  // the zero pad channel as in the x6 path: K % 4 == 0 (pipelined)
    a.wp = ws + p.packBF[i]; a.bias = b; a.epi = act ? EPI_BIAS_ACT : EPI_BIAS;
    a.out = out.p; a.out_stride = out.stride; a.out_off = out.off; a.out_layout = layout;
    // the activations that only a bf16 3x3 conv reads (d_l a -> d_l b, d1a -> d1b) stored as
    // bf16: the consumer rounds its staged operands to bf16 anyway, so the result is
    // bit-identical and those tensors move half the bytes
    a.out_bf16 = bf16_store_out(i);
    a.in_bf16 = bf16_store_in(i);
    // the encoder's pools fused as in the x6 path
    if (pool && pool_fuse && act && ksize == 3 && layout == OUT_NHWC && !a.out_bf16) {
      a.pool_out = pool->p; a.pool_stride = pool->stride; a.pool_off = pool->off;
      a.pool_only = pool_only;
      if (pooled) *pooled = true;
    }
    return launch_fwd_bf16(a, st, ksize);
  };

  // the bf16x6 nin head (k_nin_head_x6), also at the pair pixels
  const bool sel = x6 && sel_rd && !p.with_bwd && p.OC <= X6_HEAD_OCMAX;
  const bool w6_sel = sel && p.packXV >= 0 && (x6_tail_f(D1B) & X6_W6);
  const bool head_x6 = x6 && p.OC <= X6_HEAD_OCMAX;
  // bf16 base (inference only): the fused head kernel in plain bf16 products instead of nin_a /
  // nin_b as two bf16 1x1 launches + an fp32 nin_c (two 96-channel round trips through HBM
  // saved; bf16_head_x6 above)
  // the 96-channel deconvs on the persistent bf16x6 kernel, also in the bf16 base (one pass over
  // the input instead of a bf16 1x1 launch per output parity)
  auto deconv_x6_layer = [&](int i) { return (x6 || bf16) && p.packUX[i] >= 0; };
  // ConvTranspose2d(2,2): fp32 kernel, or the bf16 1x1 kernel per output parity
  auto deconv_forward = [&](const View& xin, int Nn, int h, int w, int cin, const float* wp,
                            const float* b, int cout, const View& out, hipStream_t st) -> hipError_t {
    const OpTimer timer(st, "deconv", 2.0 * Nn * h * w * cin * cout * 4, cin, cout, h, w, Nn);
    int i = ENC1;
    while (i < NL && Wt(i) != wp) ++i;
    if (i < NL && deconv_x6_layer(i)) {  // bf16x6 parity GEMMs on the layer's pre-split images
      FwdArgs a{};
      a.in = xin.p; a.in_stride = xin.stride; a.in_off = xin.off; a.IHt = h; a.IWt = w;
      a.N = Nn; a.OH = h; a.OW = w; a.K = cin; a.NOUT = cout; a.bias = b;
      a.out = out.p; a.out_stride = out.stride; a.out_off = out.off;
      if (!deconv_x6_ok(a)) return hipErrorInvalidValue;
      // (the bf16 base: plain bf16 products, as its convs)
      return launch_deconv_x6(a, ws + p.packUX[i], st, bf16);
    }
    if (!bf16 || i == NL || p.packBF[i] < 0)
      return dn::deconv_forward(xin, Nn, h, w, cin, wp, b, cout, out, st);
    FwdArgs a{};
    a.in = xin.p; a.in_stride = xin.stride; a.in_off = xin.off; a.IHt = h; a.IWt = w;
    a.N = Nn; a.OH = h; a.OW = w; a.K = cin; a.NOUT = cout;
    a.wp = ws + p.packBF[i]; a.wp_z = bf16_pack_elems(cin, cout, 1);
    a.bias = b; a.epi = EPI_BIAS;
    a.out = out.p; a.out_stride = out.stride; a.out_off = out.off; a.out_layout = OUT_UP2;
    return launch_fwd_bf16(a, st, 1);
  };

  // every weight image of the pass (fp32, bf16x6 and bf16 alike) in one pack launch (not for a
  // prepacked forward: dn_unet_pack_weights left them in ws)
  if (pack != RUN_ONLY) {
    PackBatch pb;
    auto add = [&](bool ok, const PackJob& j) { return ok ? pack_add(pb, j, s) : hipErrorInvalidValue; };
    for (int i = ENC1; i < NINA; ++i) {
      const Layer& L = p.P.L[i];
      const float* w = prm + L.woff;
      PackJob j;
      if (L.deconv && deconv_x6_layer(i)) {
        DN_TRY(add(true, pack_job_deconv_x6(w, ws + p.packUX[i])));
      } else if (L.deconv && bf16) {  // ConvTranspose2d [cin][cout][2][2]: a 1x1 image per parity
        const long img = bf16_pack_elems(L.cin, L.cout, 1);
        for (int ab = 0; ab < 4; ++ab) {
          WView v{};
          v.w = w; v.off = ab; v.sK = (long)L.cout * 4; v.sN = 4; v.taps = 1;
          DN_TRY(add(pack_job_bf16(v, L.cin, L.cout, 1,
                                   reinterpret_cast<unsigned short*>(ws + p.packBF[i]) + ab * img, j), j));
        }
      } else if (L.deconv) {
        DN_TRY(add(pack_job(G_UP, deconv_fwd_view(w, L.cout), L.cin, L.cout, 4, ws + p.packF[i], 0, 0, j),
                   j));
      } else if (bf16) DN_TRY(add(pack_job_bf16(conv_fwd_view(w, L.cin, 3), L.cin, L.cout, 3,
                                              ws + p.packBF[i], j), j));
      else if (x6) DN_TRY(add(pack_job_x6(conv_fwd_view(w, L.cin, 3), L.cin, L.cout, 0,
                                          ws + p.packX[i], x6_tail_f(i), j), j));
      else DN_TRY(add(pack_job(L.k == 3 ? G_C3 : G_C1, conv_fwd_view(w, L.cin, L.k), L.cin, L.cout, 1,
                               ws + p.packF[i], 0, 0, j), j));
      // dec_conv1b's y-tile image for the Winograd pair pass: PK_W6 over the transposed taps
      if (i == D1B && w6_sel) {
        WView v = conv_fwd_view(w, L.cin, 3);
        v.flip = 2;
        DN_TRY(add(pack_job_x6(v, L.cin, L.cout, 0, ws + p.packXV, X6_W6, j), j));
      }
    }
    if (bf16_head_x6) {
      DN_TRY(add(true, pack_job_head_x6(prm + p.P.L[NINA].woff, prm + p.P.L[NINB].woff, ws + p.packH)));
    } else if (bf16) {  // nin_a, nin_b on the bf16 kernel, nin_c (96 -> out_nc) on the fp32 one
      for (int i = NINA; i <= NINB; ++i)
        DN_TRY(launch_pack_bf16(conv_fwd_view(prm + p.P.L[i].woff, 96, 1), 96, 96,
                                ws + p.packBF[i], s, 1));
      PackJob j;
      DN_TRY(add(pack_job(G_C1, conv_fwd_view(prm + p.P.L[NINC].woff, 96, 1), 96, p.OC, 1,
                          ws + p.packF[NINC], 0, 0, j), j));
    } else if (head_x6) {
      DN_TRY(add(true, pack_job_head_x6(prm + p.P.L[NINA].woff, prm + p.P.L[NINB].woff, ws + p.packH)));
    } else {
      DN_TRY(launch_pack_head(conv_fwd_view(prm + p.P.L[NINA].woff, 96, 1),
                              conv_fwd_view(prm + p.P.L[NINB].woff, 96, 1), ws + p.packH, s, &pb));
    }
    {
      const OpTimer timer(s, "pack", 0);
      DN_TRY(pack_flush(pb, s));
    }
  }
  if (pack == PACK_ONLY) return DN_OK;
  // the pair pass's cell lists first: they depend on the pair choices only, and built here they
  // run beside the other stream's work instead of alone right before the pair pass (~20 us of a
  // step in which nothing else ran, profiles/r6_step_timeline.txt)
  if (w6_sel)
    DN_TIMED(s, "sel_lists", 0, 0, 0, 0, 0, 0,
             launch_w6s_lists(sel_rd, N, H(0), Wd(0), reinterpret_cast<unsigned*>(ws + p.w6s_list),
                              reinterpret_cast<int*>(ws + p.w6s_cnt), s));
  // enc_conv0, fused with pool0 = x -> channels [2nf, 2nf+C) of the up1 concat buffer
  DN_TIMED(s, "enc0", 2.0 * N * p.H * p.W * C * nf * 9, C, nf, p.H, p.W, N,
           launch_enc0_fwd(x, N, C, p.H, p.W, prm + p.P.L[ENC0].woff, Bs(ENC0), ws + p.a0,
                           // (dec_conv1a reading x itself, X6_T1: the concat slice is never read --
                           // 16 scattered bytes per 512-B pixel cost the launch 0.19 ms/step; c1's
                           // channels [2nf, c1s) then hold stale data, which the debug-buffer
                           // contract in denoise_hip.h states)
                           x6 && (x6_tail_f(D1A) & X6_T1) ? nullptr : ws + p.c1, p.c1s, 2 * nf,
                           p.c1kp, p.with_bwd ? ws + p.xin : nullptr, s, enc0_bf16));
  {  // enc_conv1 + pool1 -> skip slice of c2
    const View pv = V(p.c[1], p.cs[1], 2 * nf);
    bool pooled = false;
    DN_TRY(conv_forward(V(p.a0, nf), N, H(0), Wd(0), nf, Wt(ENC1), Bs(ENC1), nf, 3, 1,
                        V(p.a1, nf), OUT_NHWC, s, &pv, &pooled));
    if (!pooled)
      DN_TIMED(s, "pool", 0, 0, 0, 0, 0, 0, launch_pool_fwd(ws + p.a1, N, H(0), Wd(0), nf, ws + p.c[1], p.cs[1], 2 * nf, s));
  }
  // enc_conv2..5 + pool2..5 (pool_k -> skip slice of c_{k+1}; pool5 -> p5)
  for (int l = 1; l <= 4; ++l) {
    const int li = ENC2 + (l - 1);
    const View in = (l == 4) ? V(p.c[4], p.cs[4], nf) : V(p.c[l], p.cs[l], 2 * nf);
    const View pv = l < 4 ? V(p.c[l + 1], p.cs[l + 1], (l + 1 == 4) ? nf : 2 * nf) : V(p.p5, nf, 0);
    bool pooled = false;
    DN_TRY(conv_forward(in, N, H(l), Wd(l), nf, Wt(li), Bs(li), nf, 3, 1, V(p.a[l], nf), OUT_NHWC,
                        s, &pv, &pooled));
    if (pooled) continue;
    DN_TIMED(s, "pool", 0, 0, 0, 0, 0, 0,
             launch_pool_fwd(ws + p.a[l], N, H(l), Wd(l), nf, pv.p, pv.stride, pv.off, s));
  }
  DN_TRY(conv_forward(V(p.p5, nf), N, H(5), Wd(5), nf, Wt(ENC6), Bs(ENC6), nf, 3, 1, V(p.a6, nf),
                      OUT_NHWC, s));
  // decoder: up5 (a6 -> c5[0:nf]); dec5a/b at level 4
  DN_TRY(deconv_forward(V(p.a6, nf), N, H(5), Wd(5), nf, Wt(UP5), Bs(UP5), nf, V(p.c[4], p.cs[4], 0),
                        s));
  const int up_idx[6] = {0, UP1, UP2, UP3, UP4, UP5};  // up_idx[k]: level k -> level k-1
  const int da_idx[5] = {0, D2A, D3A, D4A, D5A};
  for (int l = 4; l >= 1; --l) {
    if (l < 4) {  // up_{l+1}: d_{l+1}b -> c_l[0:2nf]
      DN_TRY(deconv_forward(V(p.db[l + 1], 2 * nf), N, H(l + 1), Wd(l + 1), 2 * nf,
                            Wt(up_idx[l + 1]), Bs(up_idx[l + 1]), 2 * nf, V(p.c[l], p.cs[l], 0),
                            s));
    }
    const int ia = da_idx[l], ib = da_idx[l] + 1;
    DN_TRY(conv_forward(V(p.c[l], p.cs[l]), N, H(l), Wd(l), p.ck[l], Wt(ia), Bs(ia), 2 * nf, 3, 1,
                        V(p.da[l], 2 * nf), OUT_NHWC, s));
    DN_TRY(conv_forward(V(p.da[l], 2 * nf), N, H(l), Wd(l), 2 * nf, Wt(ib), Bs(ib), 2 * nf, 3, 1,
                        V(p.db[l], 2 * nf), OUT_NHWC, s));
  }
  // up1: d2b -> c1[0:2nf]
  DN_TRY(deconv_forward(V(p.db[1], 2 * nf), N, H(1), Wd(1), 2 * nf, Wt(UP1), Bs(UP1), 2 * nf,
                        V(p.c1, p.c1s, 0), s));
  DN_TRY(conv_forward(V(p.c1, p.c1s), N, H(0), Wd(0), p.c1k, Wt(D1A), Bs(D1A), 96, 3, 1,
                      V(p.d1a, 96), OUT_NHWC, s));
  if (bf16) {  // dec_conv1b, nin_a, nin_b on the bf16 kernel, then nin_c (96 -> out_nc, fp32)
    DN_TRY(conv_forward(V(p.d1a, 96), N, H(0), Wd(0), 96, Wt(D1B), Bs(D1B), 96, 3, 1,
                        V(p.d1b, 96), OUT_NHWC, s));
    if (bf16_head_x6) {
      FwdArgs a{};
      a.in = ws + p.d1b; a.in_stride = 96; a.in_off = 0; a.IHt = H(0); a.IWt = Wd(0);
      a.N = N; a.OH = H(0); a.OW = Wd(0); a.K = 96; a.NOUT = 96;
      HeadArgs h{};
      h.wp = ws + p.packH;
      h.ba = Bs(NINA); h.bb = Bs(NINB);
      h.wc = prm + p.P.L[NINC].woff; h.bc = Bs(NINC); h.oc = p.OC;
      h.y = y;
      a.in_bf16 = bf16_store_out(D1B);  // d1b stored as bf16 by dec_conv1b
      DN_TIMED(s, "head", 2.0 * N * H(0) * Wd(0) * 96 * (2 * 96 + p.OC), 96, p.OC, H(0), Wd(0), N,
               launch_nin_head_x6(a, h, ws + p.packH, s, /*bf16=*/true));
      return DN_OK;
    }
    DN_TRY(conv_forward(V(p.d1b, 96), N, H(0), Wd(0), 96, Wt(NINA), Bs(NINA), 96, 1, 1,
                        V(p.na, 96), OUT_NHWC, s));
    DN_TRY(conv_forward(V(p.na, 96), N, H(0), Wd(0), 96, Wt(NINB), Bs(NINB), 96, 1, 1,
                        V(p.nb, 96), OUT_NHWC, s));
    DN_TRY(dn::conv_forward(V(p.nb, 96), N, H(0), Wd(0), 96, Wt(NINC), Bs(NINC), p.OC, 1, 0,
                            View{y, p.OC, 0}, OUT_NCHW, s));
    return DN_OK;
  }
  // N2N no-grad pass (training_script.md:141-144 reads den at the pair pixels only): dec_conv1b
  // and the head on those pixels, through the [N, H/2, W, 96] pair image in d1b's storage
  if (sel) {
    FwdArgs a{};
    a.in = ws + p.d1a; a.in_stride = 96; a.in_off = 0; a.IHt = H(0); a.IWt = Wd(0);
    a.N = N; a.OH = H(0); a.OW = Wd(0); a.K = 96; a.NOUT = 96;
    a.wp = ws + p.packX[D1B]; a.bias = Bs(D1B); a.epi = EPI_BIAS_ACT;
    a.out = ws + p.d1b; a.out_stride = 96; a.out_off = 0; a.out_layout = OUT_NHWC;
    if (w6_sel) {  // the cells listed per tile orientation, then the Winograd pass over them
      unsigned* list = reinterpret_cast<unsigned*>(ws + p.w6s_list);
      int* cnt = reinterpret_cast<int*>(ws + p.w6s_cnt);
      DN_TIMED(s, "fwd3sel", 2.0 * N * (H(0) / 2) * Wd(0) * 96 * 96 * 9, 96, 96, H(0) / 2, Wd(0), N,
               launch_fwd_w6s(a, list, cnt, ws + p.packXV, s));
    } else {
      a.sel_rd = sel_rd;
      DN_TIMED(s, "fwd3sel", 2.0 * N * (H(0) / 2) * Wd(0) * 96 * 96 * 9, 96, 96, H(0) / 2, Wd(0), N,
               launch_fwd_x6_sel(a, s));
    }
    FwdArgs ah{};
    ah.in = ws + p.d1b; ah.in_stride = 96; ah.in_off = 0; ah.IHt = H(0) / 2; ah.IWt = Wd(0);
    ah.N = N; ah.OH = H(0) / 2; ah.OW = Wd(0); ah.K = 96; ah.NOUT = 96;
    HeadArgs h{};
    h.ba = Bs(NINA); h.bb = Bs(NINB);
    h.wc = prm + p.P.L[NINC].woff; h.bc = Bs(NINC); h.oc = p.OC;
    h.y = y;
    h.rd = sel_rd;
    DN_TIMED(s, "head", 2.0 * N * (H(0) / 2) * Wd(0) * 96 * (2 * 96 + p.OC), 96, p.OC, H(0) / 2,
             Wd(0), N, launch_nin_head_x6(ah, h, ws + p.packH, s));
    return DN_OK;
  }
  if (x6) {  // dec_conv1b on the bf16x6 kernel, then the fused nin_a -> nin_b -> nin_c head
    DN_TRY(conv_forward(V(p.d1a, 96), N, H(0), Wd(0), 96, Wt(D1B), Bs(D1B), 96, 3, 1,
                        V(p.d1b, 96), OUT_NHWC, s));
    FwdArgs a{};
    a.in = ws + p.d1b; a.in_stride = 96; a.in_off = 0; a.IHt = H(0); a.IWt = Wd(0);
    a.N = N; a.OH = H(0); a.OW = Wd(0); a.K = 96; a.NOUT = 96;
    HeadArgs h{};
    h.wp = ws + p.packH;
    h.ba = Bs(NINA); h.bb = Bs(NINB);
    h.wc = prm + p.P.L[NINC].woff; h.bc = Bs(NINC); h.oc = p.OC;
    h.y = y;
    if (p.with_bwd) { h.na = ws + p.na; h.nb = ws + p.nb; }
    DN_TIMED(s, "head", 2.0 * N * H(0) * Wd(0) * 96 * (2 * 96 + p.OC), 96, p.OC, H(0), Wd(0), N,
             head_x6 ? launch_nin_head_x6(a, h, ws + p.packH, s) : launch_nin_head(a, h, s));
    return DN_OK;
  }
  // dec_conv1b + nin_a + nin_b + nin_c in one kernel (arch_unet.py:251-257); the
  // intermediate activations are written only when a backward will read them
  {
    FwdArgs a{};
    a.in = ws + p.d1a; a.in_stride = 96; a.in_off = 0; a.IHt = H(0); a.IWt = Wd(0);
    a.N = N; a.OH = H(0); a.OW = Wd(0); a.K = 96; a.NOUT = 96;
    a.wp = Wt(D1B); a.wp_z = 0; a.bias = Bs(D1B); a.epi = EPI_BIAS_ACT;
    a.out = ws + p.d1b; a.out_stride = 96; a.out_off = 0; a.out_layout = OUT_NHWC;
    HeadArgs h{};
    h.wp = ws + p.packH;
    h.ba = Bs(NINA); h.bb = Bs(NINB);
    h.wc = prm + p.P.L[NINC].woff; h.bc = Bs(NINC); h.oc = p.OC;
    h.y = y;
    if (p.with_bwd) { h.d1b = ws + p.d1b; h.na = ws + p.na; h.nb = ws + p.nb; }
    DN_TIMED(s, "fwd3+head", 2.0 * N * H(0) * Wd(0) * 96 * (9 * 96 + 2 * 96 + p.OC), 96, 96, H(0),
             Wd(0), N, launch_head(a, h, s));
  }
  return DN_OK;
}

// ------------------------------------------------------------------------------------
// backward: the autograd graph of the forward above, in reverse.  Data gradients fuse
// LeakyReLU' into their epilogue (mask = the layer input, which is the previous layer's
// post-activation output); skip gradients are accumulated into the concat-gradient buffers.
// ------------------------------------------------------------------------------------
// The weight gradients of the backward run on a second stream (DN_BWD_STREAMS=0: one stream):
// they only read gradients and forward activations that nothing later in the backward rewrites
// (the accumulations into a concat gradient's skip slice touch channels no weight gradient
// reads) and write their own slabs, so they overlap the data-gradient chain; each is forked
// from the main stream after the kernel that produced its gradient, and the branch is joined
// before the batched reduction.  (struct SideStream: unet.h)
//
// One side stream (and its fork / join events) per host thread and device: keyed on the
// device of the caller's stream (not hipGetDevice(), which a caller need not have set to it) and
// created under a guard for that device; thread-local, so two host threads running backwards on
// one device never share the events between a record and its wait.  The owner destroys them when
// its thread exits (executors called from short-lived threads do not leak streams).
struct SideStreams {
  std::map<int, SideStream> per_device;
  ~SideStreams() {
    for (auto& kv : per_device) {
      SideStream& ss = kv.second;
      if (!ss.st) continue;
      // (HIP releases a stream / event with work still pending once that work completes)
      (void)hipEventDestroy(ss.fork);
      (void)hipEventDestroy(ss.join);
      (void)hipEventDestroy(ss.rfork);
      (void)hipEventDestroy(ss.rjoin);
      (void)hipStreamDestroy(ss.st);
      (void)hipStreamDestroy(ss.rst);
    }
  }
};

SideStream* side_stream(hipStream_t s) {
  thread_local SideStreams owner;
  std::map<int, SideStream>& per_device = owner.per_device;
  hipDevice_t dev = 0;
  if (hipStreamGetDevice(s, &dev) != hipSuccess) return nullptr;
  SideStream& ss = per_device[dev];
  if (!ss.st) {
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return nullptr;
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return nullptr;
    if (hipStreamCreateWithFlags(&ss.st, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&ss.fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ss.join, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&ss.rst, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&ss.rfork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ss.rjoin, hipEventDisableTiming) != hipSuccess)
      ss = SideStream{};
    if (cur != dev) (void)hipSetDevice(cur);
    if (!ss.st) return nullptr;
  }
  return &ss;
}

long tail_begin(const Plan& p) { return p.P.L[D5A].woff; }

dn_status unet_backward(const Plan& p, const float* prm, const float* dy, float* dprm, float* dx,
                        float* ws, hipStream_t s, int prec, hipEvent_t tail_ready) {
  const StreamDeviceGuard device_guard(s);
  const bool x6 = prec == DN_PREC_FP32_X6;
  // bf16x6 3x3 weight gradients (k_wgrad3p / k_wgrad3q)
  const bool x6w = x6;
  const int N = p.N, nf = p.nf, C = p.C;
  auto H = [&](int l) { return p.H >> l; };
  auto Wd = [&](int l) { return p.W >> l; };
  auto Wt = [&](int i) { return ws + p.packB[i]; };  // packed data-gradient weights
  auto G = [&](int i) { return dprm + p.P.L[i].woff; };
  auto V = [&](long off, int stride, int coff = 0) { return View{ws + off, stride, coff}; };
  auto x6_tail_b = [&](int i) -> int {  // as x6_tail_f in the forward, for the data gradients
    const int l = layer_level(i), nout = dgrad_nout(p, i);
    return x6_image_mode(N, H(l), Wd(l), p.P.L[i].cout, nout, x6_dgrad_zc(nout), true);
  };
  // bf16x6 data gradients of the 96-channel deconvs
  auto x6_dgrad_deconv = [&](int i) { return x6 && p.packUXB[i] >= 0; };
  auto deconv_dgrad = [&](const View& dy, int Nn, int h, int w, int cout, int i, int cin,
                          const View& mask, int epi, const View& dx, hipStream_t st) -> hipError_t {
    const OpTimer timer(st, "deconv_dgrad", 2.0 * Nn * h * w * cin * cout * 4, cout, cin, h, w, Nn);
    if (!x6_dgrad_deconv(i))
      return dn::deconv_dgrad(dy, Nn, h, w, cout, Wt(i), cin, mask, epi, dx, st);
    FwdArgs a{};
    a.in = dy.p; a.in_stride = dy.stride; a.in_off = dy.off; a.IHt = 2 * h; a.IWt = 2 * w;
    a.N = Nn; a.OH = h; a.OW = w; a.K = cout; a.NOUT = cin;
    a.epi = epi; a.mask = mask.p; a.mask_stride = mask.stride; a.mask_off = mask.off;
    a.out = dx.p; a.out_stride = dx.stride; a.out_off = dx.off;
    return launch_deconv_dgrad_x6(a, ws + p.packUXB[i], st);
  };
  // the head's data gradients in the bf16x6 arithmetic (k_head_bwd_x6)
  const bool head_bwd_x6 = x6 && p.OC <= X6_HEAD_BWD_OCMAX;
  // g_nb (the nin_b output's gradient) recomputed by nin_b's weight gradient (k_wgrad1p<., GNB>)
  // from nb and dy instead of being stored by k_head_bwd_x6 and read back (384 B per pixel less)
  const bool head_gnb = head_bwd_x6;
  // flipped/transposed weight images for the data gradients, the head's images and the
  // weight gradients' zero padding: one launch
  {
    PackBatch pb;
    auto add = [&](bool ok, const PackJob& j) { return ok ? pack_add(pb, j, s) : hipErrorInvalidValue; };
    for (int i = ENC1; i < NINA; ++i) {
      const Layer& L = p.P.L[i];
      const float* w = prm + L.woff;
      PackJob j;
      if (L.deconv && x6_dgrad_deconv(i)) {
        DN_TRY(add(true, pack_job_deconv_dgrad_x6(w, ws + p.packUXB[i])));
      } else if (L.deconv) {
        DN_TRY(add(pack_job(G_DN2, deconv_dgrad_view(w, L.cout), L.cout, L.cin, 1, ws + p.packB[i],
                            0, 0, j), j));
      } else if (x6 && p.packXB[i] >= 0) {
        const int nout = dgrad_nout(p, i);
        DN_TRY(add(pack_job_x6(conv_dgrad_view(w, L.cin, 3), L.cout, nout, x6_dgrad_zc(nout),
                               ws + p.packXB[i], x6_tail_b(i), j), j));
      } else {
        DN_TRY(add(pack_job(L.k == 3 ? G_C3 : G_C1, conv_dgrad_view(w, L.cin, L.k), L.cout,
                            dgrad_nout(p, i), 1, ws + p.packB[i], 0, 0, j), j));
      }
    }
    if (head_bwd_x6)
      DN_TRY(add(true, pack_job_head_bwd_x6(prm + p.P.L[NINA].woff, prm + p.P.L[NINB].woff, ws + p.packHB)));
    else
      DN_TRY(launch_pack_head(conv_dgrad_view(prm + p.P.L[NINB].woff, 96, 1),
                              conv_dgrad_view(prm + p.P.L[NINA].woff, 96, 1), ws + p.packHB, s, &pb));
    DN_TRY(add(true, pack_job_zero(ws + p.zeros, 64)));
    DN_TIMED(s, "pack", 0, 0, 0, 0, 0, 0, pack_flush(pb, s));
  }
  RedBatch rb;  // every weight gradient's reduction, launched together at the end
  const float* Z = ws + p.zeros;
  static const bool two_env = !getenv("DN_BWD_STREAMS") || atoi(getenv("DN_BWD_STREAMS")) != 0;
  // (profiling: one stream, so each launch's event pair brackets that kernel alone)
  SideStream* side = two_env && !prof_on() ? side_stream(s) : nullptr;
  hipStream_t s2 = side ? side->st : s;
  auto fork = [&]() -> hipError_t {  // the side stream continues after main's work so far
    if (!side) return hipSuccess;
    hipError_t e = hipEventRecord(side->fork, s);
    return e != hipSuccess ? e : hipStreamWaitEvent(side->st, side->fork, 0);
  };
  // the queued slab reductions on the reduction stream, behind the weight gradients queued on
  // the side stream so far (one stream: on s, in order)
  auto flush_side = [&]() -> hipError_t {
    if (!side) return red_flush(rb, s);
    hipError_t e = hipEventRecord(side->rfork, s2);
    if (e == hipSuccess) e = hipStreamWaitEvent(side->rst, side->rfork, 0);
    if (e == hipSuccess) e = red_flush(rb, side->rst);
    return e;
  };
  auto SL = [&](int i) { return ws + p.slab[i]; };
  // 3x3 data gradients: the fp32 kernel or the bf16x6 one
  auto conv_dgrad = [&](const View& dz, int Nn, int h, int w, int cout, const float* wp, int nout,
                        int ksize, int epi, const View& mask, const View& dx,
                        hipStream_t st) -> hipError_t {
    const OpTimer timer(st, ksize == 3 ? "dgrad3" : "dgrad1",
                        2.0 * Nn * h * w * cout * nout * ksize * ksize, cout, nout, h, w, Nn);
    int i = ENC1;
    while (i < NL && Wt(i) != wp) ++i;
    if (!x6 || i == NL || p.packXB[i] < 0 || ksize != 3)
      return dn::conv_dgrad(dz, Nn, h, w, cout, wp, nout, ksize, epi, mask, dx, st);
    FwdArgs a{};
    a.in = dz.p; a.in_stride = dz.stride; a.in_off = dz.off; a.IHt = h; a.IWt = w;
    a.N = Nn; a.OH = h; a.OW = w; a.K = cout; a.NOUT = nout;
    a.zc = x6_dgrad_zc(nout);
    a.wp = ws + p.packXB[i];
    a.wp_z = a.zc ? x6_pack_elems(cout, nout, a.zc) / ((nout + a.zc - 1) / a.zc) : 0;
    a.bias = nullptr; a.epi = epi;
    a.out = dx.p; a.out_stride = dx.stride; a.out_off = dx.off; a.out_layout = OUT_NHWC;
    a.mask = mask.p; a.mask_stride = mask.stride; a.mask_off = mask.off;
    a.x6_tail = x6_tail_b(i);
    return launch_fwd_x6(a, st);
  };
  const View none{nullptr, 0, 0};
  const int OC = p.OC;

  // dy arrives NCHW [N, OC, H, W]; for OC == 1 that equals NHWC.  For OC > 1 transpose
  // into g_c1's storage first (free at this point).
  View dyv{const_cast<float*>(dy), OC, 0};
  if (OC > 1) {
    DN_TRY(launch_nchw_to_slice(dy, N, OC, p.H, p.W, ws + p.g_c1, OC, 0, OC, s));
    dyv = V(p.g_c1, OC);
  }
  // nin_c -> nin_b -> nin_a data gradients in one kernel (g_nb, g_na, g_d1b), then the three
  // 1x1 weight gradients from them
  {
    HeadBwdArgs h{};
    h.wp = ws + p.packHB;
    h.wc = prm + p.P.L[NINC].woff; h.oc = OC;
    h.dy = dyv.p; h.dy_stride = dyv.stride;
    h.nb = ws + p.nb; h.na = ws + p.na; h.d1b = ws + p.d1b;
    // (head_gnb: nin_b's weight gradient recomputes g_nb, nothing reads a stored one)
    h.g_nb = head_gnb ? nullptr : ws + p.g_nb;
    h.g_na = ws + p.g_na; h.g_d1b = ws + p.g_d1b;
    h.npx = (long)N * H(0) * Wd(0);
    DN_TIMED(s, "head_bwd", 2.0 * h.npx * 96 * (2 * 96 + OC), OC, 96, H(0), Wd(0), N,
             head_bwd_x6 ? launch_head_bwd_x6(h, ws + p.packHB, s) : launch_head_bwd(h, s));
  }
  const bool fold_c = head_gnb && OC == 1;  // nin_c's weight gradient inside nin_b's (k_wgrad1p)
  if (!fold_c) {
    DN_TRY(fork());
    if (OC <= 4)
      DN_TIMED(s2, "wgrad1", 2.0 * N * H(0) * Wd(0) * 96 * OC, 96, OC, H(0), Wd(0), N,
               launch_wgrad_thin(dyv.p, dyv.stride, OC, ws + p.nb, (long)N * H(0) * Wd(0),
                               SL(NINC) + 64, p.splits[NINC], G(NINC), s2, &rb));
    else
      DN_TRY(wgrad(W_C1, dyv, V(p.nb, 96), N, H(0), Wd(0), OC, 96, G(NINC), SL(NINC),
                   p.splits[NINC], s2, false, Z, &rb));
  }
  DN_TRY(fork());
  // (head_gnb: the gradient operand g_nb recomputed from nb and dy inside k_wgrad1p, which also
  // forms nin_c's weight gradient from those reads into nin_c's slab)
  DN_TRY(wgrad(W_C1, head_gnb ? V(p.nb, 96) : V(p.g_nb, 96), V(p.na, 96), N, H(0), Wd(0), 96, 96,
               G(NINB), SL(NINB), p.splits[NINB], s2, x6, Z, &rb,
               head_gnb ? OC : 0, dyv.p, dyv.stride, prm + p.P.L[NINC].woff,
               fold_c ? SL(NINC) + 64 : nullptr, G(NINC)));
  DN_TRY(fork());
  DN_TRY(wgrad(W_C1, V(p.g_na, 96), V(p.d1b, 96), N, H(0), Wd(0), 96, 96, G(NINA), SL(NINA),
               p.splits[NINA], s2, x6, Z, &rb));
  DN_TRY(fork());
  DN_TRY(wgrad(W_C3, V(p.g_d1b, 96), V(p.d1a, 96), N, H(0), Wd(0), 96, 96, G(D1B), SL(D1B),
               p.splits[D1B], s2, x6w, Z, &rb));
  DN_TRY(conv_dgrad(V(p.g_d1b, 96), N, H(0), Wd(0), 96, Wt(D1B), 96, 3, EPI_MASK,
                    V(p.d1a, 96), V(p.g_d1a, 96), s));
  // dec_conv1a weight gradient: the MFMA kernel over the up1 channels [0, 2nf) and the thin
  // kernel over the network-input channels [2nf, 2nf + C), each into its own slab rows and
  // reduced into its own columns of W[co][c1k][9]
  {
    const long n = (long)96 * p.c1k * 9 + 96;
    float* slab = SL(D1A) + 64;
    WgradArgs a{};
    a.g = ws + p.g_d1a; a.g_stride = 96; a.g_off = 0;
    a.x = ws + p.c1; a.x_stride = p.c1s; a.x_off = 0;
    a.N = N; a.KH = H(0); a.KW = Wd(0); a.Cout = 96; a.Cin = 2 * nf;
    a.zeros = Z; a.slab = slab; a.slab_stride = n;
    a.wlayout = 0; a.cin_total = p.c1k; a.ci_base = 0; a.bias = 1;
    const int sp = x6w ? wgrad_splits_x6(a, p.splits[D1A]) : p.splits[D1A];
    DN_TRY(fork());
    DN_TIMED(s2, "wgrad3", 2.0 * N * H(0) * Wd(0) * 96 * 2 * nf * 9, 2 * nf, 96, H(0), Wd(0), N,
             launch_wgrad(W_C3, a, sp, s2, x6w));
    RedJob j = red_job(slab, n, sp, 96L * 2 * nf * 9, G(D1A));  // W[co][ci < 2nf][t]
    j.ig = j.og = 2 * nf * 9;
    j.is1 = j.os1 = p.c1k * 9;
    DN_TRY(red_add(&rb, j, s2));  // (a full batch flushes on s2, behind the wgrads it reads)
    DN_TRY(red_add(&rb, red_job(slab + 96L * p.c1k * 9, n, sp, 96, G(D1A) + 96L * p.c1k * 9), s2));
    // input-channel slice: compact [co][C][9] rows after the MFMA kernel's, own split count,
    // scattered into W[co][2nf + ci][t]
    float* thin = slab + (long)p.splits[D1A] * n;
    const long nt = 96L * C * 9;
    const int st = enc0_wgrad_splits(N, H(0), Wd(0));
    DN_TIMED(s2, "wgrad3_thin", 2.0 * N * H(0) * Wd(0) * 96 * C * 9, C, 96, H(0), Wd(0), N,
             launch_wgrad_c3_thin(ws + p.g_d1a, 96, ws + p.xin, N, C, H(0), Wd(0), thin, nt, C, 0,
                                  0, st, s2));
    DN_TRY(launch_reduce_scatter(thin, nt, st, nt, G(D1A), 9L * C, 9L * p.c1k, 9L * 2 * nf, s2,
                                 &rb));
  }
  // only the up1 part of the concat needs a gradient (pool0 is the network input)
  DN_TRY(conv_dgrad(V(p.g_d1a, 96), N, H(0), Wd(0), 96, Wt(D1A), 2 * nf, 3, EPI_PLAIN, none,
                    V(p.g_c1, 2 * nf), s));

  // decoder levels 1..4: up_{l}(d_{l+1}b ...) ; here "dU" for level l-1's deconv
  const int up_idx[6] = {UP1, UP2, UP3, UP4, UP5, 0};
  const int da_idx[5] = {0, D2A, D3A, D4A, D5A};
  View dU = V(p.g_c1, 2 * nf);  // gradient of up1's output
  for (int l = 1; l <= 4; ++l) {
    const int iu = up_idx[l - 1];  // deconv producing level l-1 from level l
    // deconv wgrad: x = d_l b (level l), dU at level l-1
    DN_TRY(fork());
    DN_TRY(wgrad(W_UP2, dU, V(p.db[l], 2 * nf), N, H(l), Wd(l), 2 * nf, 2 * nf, G(iu), SL(iu),
                 p.splits[iu], s2, x6, Z, &rb));
    DN_TRY(deconv_dgrad(dU, N, H(l), Wd(l), 2 * nf, iu, 2 * nf, V(p.db[l], 2 * nf), EPI_MASK,
                        V(p.g_db[l], 2 * nf), s));
    const int ia = da_idx[l], ib = ia + 1;
    DN_TRY(fork());
    DN_TRY(wgrad(W_C3, V(p.g_db[l], 2 * nf), V(p.da[l], 2 * nf), N, H(l), Wd(l), 2 * nf, 2 * nf,
                 G(ib), SL(ib), p.splits[ib], s2, x6w, Z, &rb));
    DN_TRY(conv_dgrad(V(p.g_db[l], 2 * nf), N, H(l), Wd(l), 2 * nf, Wt(ib), 2 * nf, 3,
                      EPI_MASK, V(p.da[l], 2 * nf), V(p.g_da[l], 2 * nf), s));
    DN_TRY(fork());
    // channel count ck (the layer's cin, what G(ia) and the dgrad pack are sized for); cs is
    // only the pixel stride (larger under a DN_C1S_ALIGN override)
    DN_TRY(wgrad(W_C3, V(p.g_da[l], 2 * nf), V(p.c[l], p.cs[l]), N, H(l), Wd(l), 2 * nf, p.ck[l],
                 G(ia), SL(ia), p.splits[ia], s2, x6w, Z, &rb));
    DN_TRY(conv_dgrad(V(p.g_da[l], 2 * nf), N, H(l), Wd(l), 2 * nf, Wt(ia), p.ck[l], 3,
                      EPI_PLAIN, none, V(p.g_c[l], p.cs[l]), s));
    dU = V(p.g_c[l], p.cs[l], 0);  // [u_{l+1} grad | skip grad]
  }
  // the head's and the decoder's reductions on the side stream now, behind their weight
  // gradients, overlapping the encoder's data gradients
  if (side) {
    DN_TIMED(side->rst, "reduce", 0, 0, 0, 0, 0, 0, flush_side());
    // dprm[tail_begin ..] (dec_conv5a .. nin_c) is final behind this flush
    if (tail_ready) DN_TRY(hipEventRecord(tail_ready, side->rst));
    tail_ready = nullptr;
  }
  // up5: x = a6 (level 5), dU = g_c5[0:nf]
  DN_TRY(fork());
  DN_TRY(wgrad(W_UP2, V(p.g_c[4], p.cs[4], 0), V(p.a6, nf), N, H(5), Wd(5), nf, nf, G(UP5), SL(UP5),
               p.splits[UP5], s2, false, Z, &rb));
  DN_TRY(deconv_dgrad(V(p.g_c[4], p.cs[4], 0), N, H(5), Wd(5), nf, UP5, nf, V(p.a6, nf),
                      EPI_MASK, V(p.g_a6, nf), s));
  // enc_conv6 (input p5, level 5)
  DN_TRY(fork());
  DN_TRY(wgrad(W_C3, V(p.g_a6, nf), V(p.p5, nf), N, H(5), Wd(5), nf, nf, G(ENC6), SL(ENC6),
               p.splits[ENC6], s2, x6w, Z, &rb));
  DN_TRY(conv_dgrad(V(p.g_a6, nf), N, H(5), Wd(5), nf, Wt(ENC6), nf, 3, EPI_PLAIN, none,
                    V(p.g_p5, nf), s));
  // pool5 backward -> g_a5 (level 4)
  DN_TIMED(s, "pool_bwd", 0, 0, 0, 0, 0, 0, launch_pool_bwd(ws + p.a[4], N, H(4), Wd(4), nf, ws + p.g_p5, nf, 0, 1, ws + p.g_a[4], s));
  // enc_conv5..2: input p_{l} = skip slice of c_l; gradient accumulates into g_c_l's skip slice
  for (int l = 4; l >= 1; --l) {
    const int li = ENC2 + (l - 1);
    const int skip = (l == 4) ? nf : 2 * nf;
    DN_TRY(fork());
    DN_TRY(wgrad(W_C3, V(p.g_a[l], nf), V(p.c[l], p.cs[l], skip), N, H(l), Wd(l), nf, nf, G(li),
                 SL(li), p.splits[li], s2, x6w, Z, &rb));
    DN_TRY(conv_dgrad(V(p.g_a[l], nf), N, H(l), Wd(l), nf, Wt(li), nf, 3, EPI_ACCUM, none,
                      V(p.g_c[l], p.cs[l], skip), s));
    // pool_l backward: d p_l (skip slice) -> gradient of the level l-1 activation
    if (l > 1) {
      DN_TIMED(s, "pool_bwd", 0, 0, 0, 0, 0, 0, launch_pool_bwd(ws + p.a[l - 1], N, H(l - 1), Wd(l - 1), nf, ws + p.g_c[l], p.cs[l],
                             skip, 1, ws + p.g_a[l - 1], s));
    } else {
      DN_TIMED(s, "pool_bwd", 0, 0, 0, 0, 0, 0, launch_pool_bwd(ws + p.a1, N, H(0), Wd(0), nf, ws + p.g_c[1], p.cs[1], skip, 1,
                             ws + p.g_a1, s));
    }
  }
  // the encoder's deep-level reductions (up5, enc_conv6 .. enc_conv2) on the side stream now,
  // beside enc_conv1's data gradient, so the serial tail of the step (after the last data
  // gradient) only reduces enc_conv1's and enc_conv0's slabs
  if (side) DN_TIMED(side->rst, "reduce", 0, 0, 0, 0, 0, 0, flush_side());
  // enc_conv1 (input a0), enc_conv0 (input x = c1 slice; no data gradient needed).  Two
  // streams: enc_conv1's weight gradient on the main stream behind its data gradient and
  // enc_conv0's beside it on the side stream, which is still working through the encoder's
  // weight gradients (both streams end together instead of the side stream alone for ~0.5 ms,
  // profiles/r6_step_timeline.txt)
  DN_TRY(conv_dgrad(V(p.g_a1, nf), N, H(0), Wd(0), nf, Wt(ENC1), nf, 3, EPI_MASK, V(p.a0, nf),
                    V(p.g_a0, nf), s));
  DN_TRY(fork());
  DN_TIMED(s2, "wgrad3_thin", 2.0 * N * H(0) * Wd(0) * nf * C * 9, C, nf, H(0), Wd(0), N,
           launch_enc0_wgrad(ws + p.g_a0, nf, ws + p.xin, N, C, H(0), Wd(0), SL(ENC0) + 64,
                             p.splits[ENC0], G(ENC0), s2, &rb));
  DN_TRY(wgrad(W_C3, V(p.g_a1, nf), V(p.a0, nf), N, H(0), Wd(0), nf, nf, G(ENC1), SL(ENC1),
               p.splits[ENC1], s, x6w, Z, &rb));
  if (side) {  // join the weight-gradient and reduction branches before the last reduction
    DN_TRY(hipEventRecord(side->join, s2));
    DN_TRY(hipStreamWaitEvent(s, side->join, 0));
    DN_TRY(hipEventRecord(side->rjoin, side->rst));
    DN_TRY(hipStreamWaitEvent(s, side->rjoin, 0));
  }
  DN_TIMED(s, "reduce", 0, 0, 0, 0, 0, 0, red_flush(rb, s));
  if (tail_ready) DN_TRY(hipEventRecord(tail_ready, s));  // one stream: everything is final here
  // dL/dx: the network input feeds enc_conv0 and (as pool0) dec_conv1a's last C channels
  if (dx)
    DN_TIMED(s, "dgrad_input", 0, 0, 0, 0, 0, 0, launch_dgrad_input(ws + p.g_a0, prm + p.P.L[ENC0].woff, ws + p.g_d1a,
                              prm + p.P.L[D1A].woff, p.c1k, 2 * nf, N, C, H(0), Wd(0), dx, s));
  return DN_OK;
}

}  // namespace dn
