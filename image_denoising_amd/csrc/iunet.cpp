// ImprovedUNet (arch_unet.py:421-531, noise=True, depth=4) forward and backward on the gfx950
// kernels: every 3x3 / 1x1 convolution with >= 16 channels on both sides runs on the fp32
// MFMA implicit-GEMM kernel (k_fwd, output-channel blocks over blockIdx.z; data gradients
// through the flipped weight view), thin ones (noise estimator, final conv, sigma-map
// gradient) on VALU kernels; GroupNorm, pooling and PixelShuffle are HBM-bound passes.
//
// Dataflow (NHWC fp32 in one workspace; "[a | b]" = one buffer, channel slices):
//   x0 = [x | sigma]            sigma = sigmoid(ne2(leaky(ne0(x))))          arch_unet.py:519-521
//   level i (C_i = 48 * 2^i, res H/2^i):
//     F_i = [leaky(conv_i(x_i)) | o0 | o1 | o2 | o3]   o_j = leaky(conv_j(F_i[:, :C_i+32j]))
//     r_i = F_i[:, :C_i] + lff(F_i)                      RDB, arch_unet.py:436-451
//     s_i = r_i + GN2(conv2(leaky(GN1(conv1(r_i)))))     ResBlock, arch_unet.py:422-433
//           written straight into the skip slice of up block 3-i's concat buffer
//     x_{i+1} = maxpool(s_i)                             arch_unet.py:524-526
//   bottle: ResBlock(RDB(x_4)) at H/16, 384 channels    arch_unet.py:507, 527
//   up k (in 384/2^k -> out 192/2^k):  cc_k = [PixelShuffle(conv_ps(x)) | s_{3-k}]
//     f = leaky(fuse(cc_k)), then ResBlock(RDB(f))      UpBlock, arch_unet.py:454-472
//   y = sigmoid(final([x_up3 | x]))                      arch_unet.py:530-531
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "iunet.h"
#include "iunet_ops.h"
#include "unet.h"

namespace dn {

namespace {

#define IU_TRY(x)                                                         \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      set_error(std::string("HIP error in ") + #x + ": " + hipGetErrorString(e_)); \
      return DN_ERR_HIP;                                                  \
    }                                                                     \
  } while (0)

// a launch of a pass body, skipped in its dry run (Ctx::dry)
#define IU_RUN(c, x)                 \
  do {                               \
    if (!(c).dry) IU_TRY(x);         \
  } while (0)

constexpr int GROWTH = 32;  // RDB growth (arch_unet.py:437)
constexpr float GN_EPS = 1e-5f;

int gn_groups(int ch) {  // norm2d('gn', ch, groups=32), arch_unet.py:12-15
  int g = std::min(32, ch);
  while (ch % g != 0 && g > 1) --g;
  return g;
}

// ---- generic convolution on the MFMA kernel --------------------------------------------
struct GGeom {
  int gather = G_C3, nt = 6, np = 96, nz = 1;
  long img = 0;  // floats of one z-block's packed image
};

bool ggeom(int ksize, int K, int nout, GGeom& g) {
  g.gather = ksize == 3 ? G_C3 : G_C1;
  const int nts[3] = {6, 3, 2};
  // relative cost per output channel of the tile widths; with few reduction channels (K < 64:
  // at most 16 four-channel chunks) the 96-wide tile's fixed per-tile cost dominates
  const double eff[3] = {K < 64 ? 1.6 : 1.0, 1.3, 1.6};
  double best = 1e30;
  for (int i = 0; i < 3; ++i) {
    const int np = 16 * nts[i], nz = (nout + np - 1) / np;
    const double c = nz * np * eff[i];
    if (c < best) { best = c; g.nt = nts[i]; g.np = np; g.nz = nz; }
  }
  g.img = pack_floats(g.gather, g.np, K, 1);
  return g.img > 0;
}

// split-bf16 (DN_PREC_FP32_X6) 3x3 convs: the kernels tile 32, 48 or 96 output channels and
// 32 reduction channels (on large grids a partial last chunk of <= 16 channels costs 5 of 9
// stages, `tail`), so they take the convs that fill those tiles; small-grid K = 48 and the
// level conv (K = 4) stay on the fp32 kernels, where the padding would cost more than the
// faster matrix cores give (measured per shape)
bool x6_shape(int nout) { return nout == 32 || nout % 48 == 0; }
bool x6_takes(int K, int nout, int tail) {
  // 32-wide tiles with K < 80 were staging-bound on round 2's 8-row kernels (no gain for 32x48,
  // 32x56); the 16-row ones take K >= 48 at 0.33-0.37 of the x6 peak against the fp32 kernel's
  // 0.25-0.27 (48->32 @256^2: 1.05 -> 0.79 ms)
  if (nout == 32 && K < 80 && !(K % 4 == 0 && K >= 48)) return false;
  // 32-wide RDB growth convs with K >= 80 take a zero-padded last chunk when it cannot be
  // tail-packed (88, 120: 3 / 4 chunks, 9 / 7 % padding; on the fp32 kernel they ran at ~60 %
  // of the x6 rate of their 80- / 112-channel neighbours)
  if (nout == 32 && K % 4 == 0) return true;
  // likewise the data gradients of those convs (K = 32 = the growth, nout = 80..144 of the dense
  // concatenation: 48-channel output blocks, the last one partial) and the 24-channel top
  // level's 72 -> 24 (a 32-wide tile, 8 outputs idle): the fp32 kernel ran them at 0.19-0.22 of
  // the x6 ceiling
  if (K == 32 && nout >= 80 && nout % 8 == 0) return true;
  if (nout == 24 && K >= 72 && K % 4 == 0) return true;
  // round 6: the top level's 24 -> 24 (ResBlock) and 24 -> 32 (first growth conv) too, one
  // zero-padded chunk: fwd3 -0.25 ms/step against the fp32 kernel (profiles/r6_iunet_x624_ab.log)
  if (K == 24 && (nout == 24 || nout == 32)) return true;
  return x6_shape(nout) && (K % 32 == 0 || K >= 128 || tail) && (K > 32 || nout % 96 == 0);
}
// output-channel blocks of the wide layers: 96, or 48 where 96 would pad (144 = 3 x 48)
int x6_zc(int nout) { return nout <= 96 ? 0 : (nout % 96 == 0 ? 96 : 48); }

long gpack_floats(int ksize, int K, int nout) {
  GGeom g;
  if (!ggeom(ksize, K, nout, g)) return -1;
  return g.img * g.nz;
}

// forward image of conv weight [cout][cin][k][k] (reduction K = cin, outputs = cout)
bool gjob_fwd(const float* w, int ksize, int cin, int cout, float* out, PackJob& j) {
  GGeom g;
  if (!ggeom(ksize, cin, cout, g)) return false;
  WView wv = conv_fwd_view(w, cin, ksize);
  wv.sZ = (long)g.np * wv.sN;
  return pack_job(g.gather, wv, cin, g.np, g.nz, out, g.np, cout, j);
}

// data-gradient image: reduction over the layer's cout, outputs = its first nout input channels
bool gjob_dgrad(const float* w, int ksize, int cin_total, int cout, int nout, float* out,
                PackJob& j) {
  GGeom g;
  if (!ggeom(ksize, cout, nout, g)) return false;
  WView wv = conv_dgrad_view(w, cin_total, ksize);
  wv.sZ = (long)g.np * wv.sN;
  return pack_job(g.gather, wv, cout, g.np, g.nz, out, g.np, nout, j);
}

hipError_t grun(int ksize, const View& in, int N, int H, int W, int K, const float* wp, int nout,
                const float* bias, int epi, const View& out, int layout, const View& aux,
                hipStream_t s) {
  GGeom g;
  if (!ggeom(ksize, K, nout, g)) return hipErrorInvalidValue;
  FwdArgs a{};
  a.in = in.p; a.in_stride = in.stride; a.in_off = in.off; a.IHt = H; a.IWt = W;
  a.N = N; a.OH = H; a.OW = W; a.K = K; a.NOUT = nout;
  a.wp = wp; a.wp_z = g.img;
  a.bias = bias; a.epi = epi;
  a.out = out.p; a.out_stride = out.stride; a.out_off = out.off; a.out_layout = layout;
  a.mask = aux.p; a.mask_stride = aux.stride; a.mask_off = aux.off;
  a.zc = g.np;
  return launch_fwd_nt(g.gather, g.nt, a, s);
}

// the same 3x3 conv on the split-bf16 kernels (image from launch_pack_x6 with zc = x6_zc(nout))
// tail packing of a partial last K chunk when the launch takes the pipelined kernel
// (w6_ok: the launch's output / auxiliary views allow the Winograd kernel's float4 NHWC
// epilogue; then x6_image_mode may add X6_W6 for the 96-channel blocks)
int x6_tail_for(const View& in, int N, int H, int W, int K, int nout, bool w6_ok) {
  const bool aligned = ((in.stride | in.off | K) & 3) == 0;
  if (w6_ok && aligned) return x6_image_mode(N, H, W, K, nout, x6_zc(nout), true);
  return aligned && x6_pipelined(N, H, W, nout, x6_zc(nout)) ? x6_tail_mode(K) : 0;
}
static bool w6_views(const View& out, int layout, const View& aux, int nout) {
  return layout == OUT_NHWC && ((out.stride | out.off | nout) & 3) == 0 &&
         (!aux.p || ((aux.stride | aux.off) & 3) == 0);
}

hipError_t x6run(const View& in, int N, int H, int W, int K, const float* wp, int nout,
                 const float* bias, int epi, const View& out, int layout, const View& aux,
                 int tail, hipStream_t s) {
  FwdArgs a{};
  a.x6_tail = tail;
  a.in = in.p; a.in_stride = in.stride; a.in_off = in.off; a.IHt = H; a.IWt = W;
  a.N = N; a.OH = H; a.OW = W; a.K = K; a.NOUT = nout;
  a.zc = x6_zc(nout);
  a.wp = wp; a.wp_z = a.zc ? x6_pack_elems(K, nout, a.zc) / ((nout + a.zc - 1) / a.zc) : 0;
  a.bias = bias; a.epi = epi;
  a.out = out.p; a.out_stride = out.stride; a.out_off = out.off; a.out_layout = layout;
  a.mask = aux.p; a.mask_stride = aux.stride; a.mask_off = aux.off;
  return launch_fwd_x6(a, s);
}

// ---- parameter layout (state_dict order of ImprovedUNet) ---------------------------------
struct Alloc {
  long off = 0;
  IConv conv(int cout, int cin, int k, bool bias = true) {
    IConv c;
    c.cout = cout; c.cin = cin; c.k = k;
    c.w = off; off += (long)cout * cin * k * k;
    if (bias) { c.b = off; off += cout; }
    return c;
  }
  IGN gn(int ch) {
    IGN n;
    n.C = ch; n.G = gn_groups(ch);
    n.g = off; off += ch;
    n.b = off; off += ch;
    return n;
  }
  IRdb rdb(int ch) {
    IRdb r;
    r.C = ch;
    for (int j = 0; j < 4; ++j) r.conv[j] = conv(GROWTH, ch + GROWTH * j, 3);
    r.lff = conv(ch, ch + 4 * GROWTH, 1);
    return r;
  }
  IRes res(int ch) {  // block = [conv(no bias), GN, LeakyReLU, conv(no bias), GN]
    IRes r;
    r.C = ch;
    r.c1 = conv(ch, ch, 3, false);
    r.n1 = gn(ch);
    r.c2 = conv(ch, ch, 3, false);
    r.n2 = gn(ch);
    return r;
  }
};

// every conv the backward runs a weight gradient for: (mode, level resolution shift, cin, cout)
struct WJob { int mode, lvl, cin, cout; };

void wgrad_jobs(const IParams& P, std::vector<WJob>& v) {
  auto rdb = [&](const IRdb& r, int l) {
    for (int j = 0; j < 4; ++j) v.push_back({W_C3, l, r.conv[j].cin, GROWTH});
    v.push_back({W_C1, l, r.lff.cin, r.C});
  };
  auto res = [&](const IRes& r, int l) {
    v.push_back({W_C3, l, r.C, r.C});
    v.push_back({W_C3, l, r.C, r.C});
  };
  v.push_back({W_C3, 0, 48, 1});  // ne2
  for (int i = 0; i < 4; ++i) {
    if (i > 0) v.push_back({W_C3, i, P.down[i].conv.cin, P.down[i].conv.cout});
    rdb(P.down[i].rdb, i);
    res(P.down[i].res, i);
  }
  rdb(P.brdb, 4);
  res(P.bres, 4);
  for (int k = 0; k < 4; ++k) {
    const IUp& u = P.up[k];
    v.push_back({W_C3, 4 - k, u.ps.cin, u.ps.cout});
    v.push_back({W_C3, 3 - k, u.fuse.cin, u.fuse.cout});
    rdb(u.rdb, 3 - k);
    res(u.res, 3 - k);
  }
  v.push_back({W_C3, 0, P.fin.cin, P.fin.cout});
}

}  // namespace

bool iunet_build_params(const dn_unet_cfg& c, IParams& P, std::string& err) {
  if (c.in_nc < 1 || c.in_nc > 3 || c.out_nc < 1 || c.out_nc > 4) {
    err = "ImprovedUNet: in_nc must be 1..3 and out_nc 1..4";
    return false;
  }
  if (c.n_feature != 48) {
    err = "ImprovedUNet: only n_feature=48 is built (train.py:30 default)";
    return false;
  }
  P = IParams{};
  P.C = c.in_nc; P.OC = c.out_nc; P.nf = 48;
  Alloc A;
  P.ne0 = A.conv(48, P.C, 3);  // noise_estimator.0 (arch_unet.py:483)
  P.ne2 = A.conv(1, 48, 3);    // noise_estimator.2 (:485)
  int nf = 48;
  for (int i = 0; i < 4; ++i) {  // downs.i = [conv, LeakyReLU, RDB, ResBlock] (:499-503)
    const int inc = i == 0 ? P.C + 1 : nf / 2;
    P.down[i].conv = A.conv(nf, inc, 3);
    P.down[i].rdb = A.rdb(nf);
    P.down[i].res = A.res(nf);
    nf *= 2;
  }
  P.brdb = A.rdb(nf / 2);  // bottle (:507)
  P.bres = A.res(nf / 2);
  nf /= 2;
  for (int k = 0; k < 4; ++k) {  // ups.k = UpBlock(nf, nf/2) (:511-513, 454-461)
    IUp& u = P.up[k];
    u.in = nf; u.out = nf / 2;
    u.ps = A.conv(4 * u.out, u.in, 3);
    u.fuse = A.conv(u.out, 3 * u.out, 3);
    u.rdb = A.rdb(u.out);
    u.res = A.res(u.out);
    nf /= 2;
  }
  P.fin = A.conv(P.OC, 24 + P.C, 3);  // final (:515)
  P.total = A.off;
  return true;
}

bool iunet_build_plan(const dn_unet_cfg& c, int N, int H, int W, bool bwd, IPlan& p,
                      std::string& err) {
  if (!iunet_build_params(c, p.P, err)) return false;
  if (N < 1 || H < 16 || W < 16 || (H % 16) || (W % 16)) {
    err = "ImprovedUNet needs N >= 1 and H, W multiples of 16 (4 pooling levels)";
    return false;
  }
  p.N = N; p.H = H; p.W = W; p.with_bwd = bwd;
  const IParams& P = p.P;
  long off = 0;
  auto px = [&](int l) { return (long)N * (H >> l) * (W >> l); };
  auto alloc = [&](int l, int ch) {
    long o = off;
    off += (px(l) * ch + 63) / 64 * 64;
    return o;
  };
  auto allocf = [&](long n) {
    long o = off;
    off += (n + 63) / 64 * 64;
    return o;
  };
  auto block = [&](IBlockBufs& b, int l, int ch) {
    b.F = alloc(l, ch + 4 * GROWTH);
    b.r = alloc(l, ch);
    b.z1 = alloc(l, ch);
    b.a1 = alloc(l, ch);
    b.z2 = alloc(l, ch);
    b.st1 = allocf(2L * N * gn_groups(ch));
    b.st2 = allocf(2L * N * gn_groups(ch));
  };
  p.x0 = alloc(0, 4);
  p.h = alloc(0, 48);
  p.xin = alloc(0, P.C);
  p.yout = alloc(0, P.OC);
  p.sig = alloc(0, 1);
  for (int i = 0; i < 4; ++i) {
    block(p.dl[i], i, 48 << i);
    if (i > 0) p.pool[i] = alloc(i, 48 << (i - 1));
  }
  block(p.bb, 4, 384);
  for (int k = 0; k < 4; ++k) {
    const int out = P.up[k].out, l = 3 - k;
    p.cc[k] = alloc(l, 3 * out);
    block(p.ul[k], l, out);
    if (k < 3) p.xu[k] = alloc(l, out);
  }
  p.xb = alloc(4, 384);
  p.cf = alloc(0, 28);
  p.sc = allocf((long)N * 384);
  p.sh = allocf((long)N * 384);
  p.gpart = allocf(2L * 2 * std::max(2048L, (long)N) * 384);  // N*S splits x 384 ch x 2 doubles
  // packed-weight arena: one slot per conv of a pass (forward images; the backward's
  // data-gradient images reuse the region), each sized for the fp32 or the split-bf16 image,
  // whichever the launch takes.  A pass packs every slot in a few batched launches first.
  long fsum = 0, bsum = 0;
  auto slot = [](int k, int K, int nout) {
    long f = gpack_floats(k, K, nout);
    if (k == 3)  // every shape x6_takes may route (-1 where the x6 kernels have no tile)
      f = std::max(f, (x6_pack_elems(K, nout, x6_zc(nout)) + 1) / 2);
    return (std::max(f, 0L) + 63) / 64 * 64;
  };
  auto pf = [&](int k, int K, int nout) { fsum += slot(k, K, nout); };
  auto pb = [&](int k, int K, int nout) { bsum += slot(k, K, nout); };
  for (int i = 0; i < 4; ++i) {
    const ILevel& L = P.down[i];
    pf(3, L.conv.cin, L.conv.cout);
    if (i > 0) pb(3, L.conv.cout, L.conv.cin);
  }
  auto rdbp = [&](const IRdb& r) {
    for (int j = 0; j < 4; ++j) { pf(3, r.conv[j].cin, GROWTH); pb(3, GROWTH, r.conv[j].cin); }
    pf(1, r.lff.cin, r.C); pb(1, r.C, r.lff.cin);
  };
  auto resp = [&](const IRes& r) {
    for (int t = 0; t < 2; ++t) { pf(3, r.C, r.C); pb(3, r.C, r.C); }
  };
  for (int i = 0; i < 4; ++i) { rdbp(P.down[i].rdb); resp(P.down[i].res); }
  rdbp(P.brdb); resp(P.bres);
  for (int k = 0; k < 4; ++k) {
    const IUp& u = P.up[k];
    pf(3, u.ps.cin, u.ps.cout); pb(3, u.ps.cout, u.ps.cin);
    pf(3, u.fuse.cin, u.fuse.cout); pb(3, u.fuse.cout, u.fuse.cin);
    rdbp(u.rdb); resp(u.res);
  }
  pb(3, 1, 48);         // ne2 data gradient
  pb(3, P.OC, 24);      // final data gradient (x_up3 part)
  const long arena = bwd ? std::max(fsum, bsum) : fsum;
  p.pack = allocf(arena);
  p.pack_floats = arena;
  if (bwd) {
    auto gblock = [&](IBlockBufs& b, int l, int ch) {
      b.dF = alloc(l, ch + 4 * GROWTH);
      b.dr = alloc(l, ch);
      b.dz2 = alloc(l, ch);
      b.dg1 = alloc(l, ch);
      b.dz1 = alloc(l, ch);
      for (int j = 0; j < 4; ++j) b.dzj[j] = alloc(l, GROWTH);
      b.dzf = alloc(l, ch);
    };
    for (int i = 0; i < 4; ++i) gblock(p.dl[i], i, 48 << i);
    gblock(p.bb, 4, 384);
    for (int k = 0; k < 4; ++k) {
      const int out = P.up[k].out, l = 3 - k;
      p.dcc[k] = alloc(l, 3 * out);
      gblock(p.ul[k], l, out);
      if (k < 3) p.dxu[k] = alloc(l, out);
    }
    p.dxb = alloc(4, 384);
    p.dzfin = alloc(0, 4);
    for (int k = 0; k < 4; ++k)  // unshuffled PixelShuffle gradient of up block k (4 x out ch)
      p.dps[k] = alloc(4 - k, 4 * P.up[k].out);
    p.dpool = alloc(1, 48);     // largest pooled-input gradient: level 1 (48 ch at H/2)
    for (int i = 0; i < 4; ++i)  // level-conv pre-activation gradients
      p.dza[i] = alloc(i, 48 << i);
    p.dsg = alloc(0, 4);
    p.dh = alloc(0, 48);
    p.ca = allocf((long)N * 384);
    p.cb = allocf((long)N * 384);
    p.ccf = allocf((long)N * 384);
    // weight-gradient slab: 64 zero floats + max over layers of splits x (W + b)
    std::vector<WJob> jobs;
    wgrad_jobs(P, jobs);
    long slab = 0;
    for (const WJob& j : jobs) {
      const int taps = j.mode == W_C3 ? 9 : 1;
      const int sp = gwgrad_splits(j.mode, N, H >> j.lvl, W >> j.lvl, j.cin, j.cout);
      slab = std::max(slab, (long)sp * ((long)j.cout * j.cin * taps + j.cout));
    }
    const int st = enc0_wgrad_splits(N, H, W);
    slab = std::max(slab, (long)st * (48L * (P.C + 1) * 9 + 48));
    p.slab = off;
    off += 64 + (slab + 63) / 64 * 64;
    p.slab_floats = slab;
  }
  p.total_floats = off;
  return true;
}

// ------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------
namespace {

// Optional per-op timing (DN_PROFILE_OPS=1): HIP events around every conv / weight gradient /
// GroupNorm call, aggregated by shape and printed to stderr at the end of each pass.  One record
// list per host thread (thread_local g_prof below: no state shared between callers); a failing
// HIP event call switches this thread's profiling off with a message, it never fails a pass.
struct OpProf {
  struct Rec { std::string label; double flops; hipEvent_t a, b; };
  bool on = getenv("DN_PROFILE_OPS") != nullptr;
  std::vector<Rec> recs;
  bool ok(hipError_t e, const char* what) {
    if (e == hipSuccess) return true;
    fprintf(stderr, "[dn ops] %s failed (%s): per-op timing off\n", what, hipGetErrorString(e));
    on = false;
    return false;
  }
  void drop() {
    for (auto& r : recs) {
      if (r.a) (void)hipEventDestroy(r.a);
      if (r.b) (void)hipEventDestroy(r.b);
    }
    recs.clear();
  }
  void flush(const char* pass) {
    if (!on || recs.empty()) return;
    if (!ok(hipEventSynchronize(recs.back().b), "hipEventSynchronize")) return drop();
    struct Agg { double ms = 0, flops = 0; int n = 0; };
    std::vector<std::pair<std::string, Agg>> agg;
    double total = 0;
    for (auto& r : recs) {
      float ms = 0;
      if (!ok(hipEventElapsedTime(&ms, r.a, r.b), "hipEventElapsedTime")) return drop();
      total += ms;
      auto it = std::find_if(agg.begin(), agg.end(), [&](auto& x) { return x.first == r.label; });
      if (it == agg.end()) { agg.push_back({r.label, Agg{}}); it = agg.end() - 1; }
      it->second.ms += ms; it->second.flops += r.flops; it->second.n += 1;
    }
    const size_t nrec = recs.size();
    drop();
    std::sort(agg.begin(), agg.end(), [](auto& x, auto& y) { return x.second.ms > y.second.ms; });
    fprintf(stderr, "[dn ops] %s: %.3f ms in %zu ops\n", pass, total, nrec);
    for (auto& [l, a] : agg)
      fprintf(stderr, "  %8.3f ms  %7.1f TF/s  x%-3d %s\n", a.ms,
              a.flops > 0 ? a.flops / (a.ms * 1e-3) / 1e12 : 0.0, a.n, l.c_str());
  }
};
thread_local OpProf g_prof;

// dn_profile_ops op name of an OpScope kind ("fwd" + k = 3 -> "fwd3", the bench's 3x3 ops)
inline const char* prof_op(const char* kind, int k) {
  const std::string kd(kind);
  if (kd == "fwd") return k == 3 ? "fwd3" : "fwd1";
  if (kd == "wgrad") return k == 3 ? "wgrad3" : "wgrad1";
  if (kd == "dgrad") return k == 3 ? "dgrad3" : "dgrad1";
  return kind;
}

struct OpScope {
  hipStream_t s;
  bool on;
  OpTimer timer;  // the in-step launch record (dn_profile_ops), when enabled
  OpScope(hipStream_t st, const char* kind, int cout, int cin, int k, int h, int w, int N,
          double flop_mult)
      : s(st), on(g_prof.on),
        timer(st, prof_op(kind, k), flop_mult * 2.0 * N * h * w * (double)cout * cin * k * k,
              cin, cout, h, w, N) {
    if (!on) return;
    char b[128];
    snprintf(b, sizeof(b), "%-6s %dx%d k%d @%dx%d", kind, cout, cin, k, h, w);
    OpProf::Rec r{b, flop_mult * 2.0 * N * h * w * (double)cout * cin * k * k, nullptr, nullptr};
    if (!g_prof.ok(hipEventCreate(&r.a), "hipEventCreate") ||
        !g_prof.ok(hipEventCreate(&r.b), "hipEventCreate") ||
        !g_prof.ok(hipEventRecord(r.a, s), "hipEventRecord")) {
      if (r.a) (void)hipEventDestroy(r.a);
      if (r.b) (void)hipEventDestroy(r.b);
      on = false;
      g_prof.drop();
      return;
    }
    g_prof.recs.push_back(r);
  }
  ~OpScope() {
    if (on && g_prof.on && !g_prof.recs.empty() &&
        !g_prof.ok(hipEventRecord(g_prof.recs.back().b, s), "hipEventRecord"))
      g_prof.drop();
  }
};

struct Ctx {
  const IPlan& p;
  const float* prm;
  float* ws;
  hipStream_t s;
  int prec;
  // backward: the weight gradients' stream (s when running on one stream) and its fork event
  hipStream_t s2 = nullptr;
  hipEvent_t fork = nullptr;
  // A pass runs twice: dry (every conv queues its weight image into the next arena slot, nothing
  // else launches), then the batched packs, then for real (each conv takes the same slot).
  bool dry = false;
  PackBatch* pb = nullptr;
  long* next = nullptr;
  View V(long o, int stride, int off = 0) const { return View{ws + o, stride, off}; }
  float* slot(long floats) const {  // the next conv's arena slot (nullptr: arena overrun)
    const long o = *next;
    *next += (floats + 63) / 64 * 64;
    return *next <= p.pack_floats ? ws + p.pack + o : nullptr;
  }
  const float* Wt(const IConv& c) const { return prm + c.w; }
  const float* Bs(const IConv& c) const { return c.b >= 0 ? prm + c.b : nullptr; }
};

const View kNone{nullptr, 0, 0};

dn_status conv_fwd(const Ctx& c, const IConv& L, const View& in, int h, int w, int epi,
                   const View& out, int layout = OUT_NHWC, const View& aux = kNone) {
  const int tail = x6_tail_for(in, c.p.N, h, w, L.cin, L.cout, w6_views(out, layout, aux, L.cout));
  const bool x6 = c.prec == DN_PREC_FP32_X6 && L.k == 3 && x6_takes(L.cin, L.cout, tail);
  float* pk = c.slot(x6 ? (x6_pack_elems(L.cin, L.cout, x6_zc(L.cout)) + 1) / 2
                        : gpack_floats(L.k, L.cin, L.cout));
  if (!pk) {
    set_error("ImprovedUNet: packed-weight arena overrun (forward)");
    return DN_ERR_ARG;
  }
  if (c.dry) {
    PackJob j;
    const bool ok = x6 ? pack_job_x6(conv_fwd_view(c.Wt(L), L.cin, 3), L.cin, L.cout,
                                     x6_zc(L.cout), pk, tail, j)
                       : gjob_fwd(c.Wt(L), L.k, L.cin, L.cout, pk, j);
    if (!ok) {
      set_error("ImprovedUNet: no weight image for a forward conv");
      return DN_ERR_ARG;
    }
    IU_TRY(pack_add(*c.pb, j, c.s));
    return DN_OK;
  }
  OpScope prof(c.s, "fwd", L.cout, L.cin, L.k, h, w, c.p.N, 1.0);
  if (x6)
    IU_TRY(x6run(in, c.p.N, h, w, L.cin, pk, L.cout, c.Bs(L), epi, out, layout, aux, tail, c.s));
  else
    IU_TRY(grun(L.k, in, c.p.N, h, w, L.cin, pk, L.cout, c.Bs(L), epi, out, layout, aux, c.s));
  return DN_OK;
}

dn_status gn_fwd(const Ctx& c, const IGN& g, const View& z, int h, int w, float* stats, int act,
                 const View* res, const View& out) {
  if (c.dry) return DN_OK;
  OpScope prof(c.s, "gn", g.C, 1, 1, h, w, c.p.N, 0.0);
  const int N = c.p.N;
  const long P = (long)h * w;
  const int S = chan_sums_splits(N, P);
  double* part = reinterpret_cast<double*>(c.ws + c.p.gpart);
  IU_TRY(launch_chan_sums(z, nullptr, N, P, g.C, S, part, c.s));
  IU_TRY(launch_gn_fwd_fin(part, S, N, g.C, g.G, P, GN_EPS, c.prm + g.g, c.prm + g.b, stats,
                           c.ws + c.p.sc, c.ws + c.p.sh, c.s));
  IU_TRY(launch_affine(z, nullptr, c.ws + c.p.sc, nullptr, c.ws + c.p.sh, act, res, out, N, P, g.C,
                       c.s));
  return DN_OK;
}

// F[:, :C] holds the block input; writes the RDB output to b.r
dn_status rdb_fwd(const Ctx& c, const IRdb& R, const IBlockBufs& b, int h, int w) {
  const int C = R.C, FS = C + 4 * GROWTH;
  for (int j = 0; j < 4; ++j)
    if (dn_status st = conv_fwd(c, R.conv[j], c.V(b.F, FS), h, w, EPI_BIAS_ACT,
                                c.V(b.F, FS, C + GROWTH * j)))
      return st;
  return conv_fwd(c, R.lff, c.V(b.F, FS), h, w, EPI_BIAS_ADD, c.V(b.r, C), OUT_NHWC, c.V(b.F, FS));
}

dn_status res_fwd(const Ctx& c, const IRes& R, const IBlockBufs& b, int h, int w, const View& out) {
  const int C = R.C;
  const View r = c.V(b.r, C);
  if (dn_status st = conv_fwd(c, R.c1, r, h, w, EPI_PLAIN, c.V(b.z1, C))) return st;
  if (dn_status st = gn_fwd(c, R.n1, c.V(b.z1, C), h, w, c.ws + b.st1, 1, nullptr, c.V(b.a1, C)))
    return st;
  if (dn_status st = conv_fwd(c, R.c2, c.V(b.a1, C), h, w, EPI_PLAIN, c.V(b.z2, C))) return st;
  return gn_fwd(c, R.n2, c.V(b.z2, C), h, w, c.ws + b.st2, 0, &r, out);
}

WView thin_view(const float* w, int cin) {  // weight [o][cin][3][3] as W(o, k, t)
  WView v{};
  v.w = w; v.off = 0; v.sN = (long)cin * 9; v.sK = 9; v.sT = 1; v.taps = 9; v.flip = 0;
  return v;
}

// the forward's launches (Ctx::dry: only the convs' weight images are queued)
dn_status forward_body(const Ctx& c, const float* x, float* y) {
  const IPlan& p = c.p;
  const float* prm = c.prm;
  float* ws = c.ws;
  const hipStream_t s = c.s;
  const IParams& P = p.P;
  const int N = p.N, H = p.H, W = p.W, C = P.C;
  // noise estimator: h = leaky(ne0(x)) (also writes x into x0[:, :C], zeros x0[:, C:4])
  IU_RUN(c, launch_enc0_fwd(x, N, C, H, W, prm + P.ne0.w, prm + P.ne0.b, ws + p.h, ws + p.x0, 4,
                            0, 4, nullptr, s));
  IU_RUN(c, launch_conv3_thin(c.V(p.h, 48), N, H, W, 48, thin_view(prm + P.ne2.w, 48),
                              prm + P.ne2.b, TE_SIGMOID, kNone, c.V(p.x0, 4, C), 0, 1, s));
  if (p.with_bwd) {
    IU_RUN(c, hipMemcpyAsync(ws + p.xin, x, sizeof(float) * (size_t)N * C * H * W,
                             hipMemcpyDeviceToDevice, s));
    IU_RUN(c, launch_conv3_thin(c.V(p.h, 48), N, H, W, 48, thin_view(prm + P.ne2.w, 48),
                                prm + P.ne2.b, TE_SIGMOID, kNone, View{ws + p.sig, 0, 0}, 1, 1, s));
  }
  IU_RUN(c, launch_nchw_to_slice(x, N, C, H, W, ws + p.cf, 28, 24, 28, s));  // final concat input
                                 // encoder
                                 View xi = c.V(p.x0, 4);
  for (int i = 0; i < 4; ++i) {
    const ILevel& L = P.down[i];
    const int h = H >> i, w = W >> i, nf = L.conv.cout, FS = nf + 4 * GROWTH;
    const IBlockBufs& b = p.dl[i];
    if (dn_status st = conv_fwd(c, L.conv, xi, h, w, EPI_BIAS_ACT, c.V(b.F, FS))) return st;
    if (dn_status st = rdb_fwd(c, L.rdb, b, h, w)) return st;
    const int k = 3 - i, out = P.up[k].out;  // skip slice of up block k's concat
    const View skip = c.V(p.cc[k], 3 * out, out);
    if (dn_status st = res_fwd(c, L.res, b, h, w, skip)) return st;
    const View dst = i < 3 ? c.V(p.pool[i + 1], nf) : c.V(p.bb.F, 384 + 4 * GROWTH);
    IU_RUN(c, launch_vpool_fwd(skip, N, h, w, nf, dst, s));
    xi = dst;
  }
  // bottleneck
  if (dn_status st = rdb_fwd(c, P.brdb, p.bb, H >> 4, W >> 4)) return st;
  if (dn_status st = res_fwd(c, P.bres, p.bb, H >> 4, W >> 4, c.V(p.xb, 384))) return st;
  // decoder
  View xk = c.V(p.xb, 384);
  for (int k = 0; k < 4; ++k) {
    const IUp& u = P.up[k];
    const int l = 3 - k, h = H >> l, w = W >> l, out = u.out, FS = out + 4 * GROWTH;
    const IBlockBufs& b = p.ul[k];
    if (dn_status st = conv_fwd(c, u.ps, xk, h / 2, w / 2, EPI_BIAS, c.V(p.cc[k], 3 * out), OUT_PS))
      return st;
    if (dn_status st = conv_fwd(c, u.fuse, c.V(p.cc[k], 3 * out), h, w, EPI_BIAS_ACT, c.V(b.F, FS)))
      return st;
    if (dn_status st = rdb_fwd(c, u.rdb, b, h, w)) return st;
    const View o = k < 3 ? c.V(p.xu[k], out) : c.V(p.cf, 28);
    if (dn_status st = res_fwd(c, u.res, b, h, w, o)) return st;
    xk = o;
  }
  IU_RUN(c, launch_conv3_thin(c.V(p.cf, 28), N, H, W, 24 + C, thin_view(prm + P.fin.w, 24 + C),
                              prm + P.fin.b, TE_SIGMOID, kNone, View{y, 0, 0}, 1, P.OC, s));
  if (p.with_bwd)
    IU_RUN(c, hipMemcpyAsync(ws + p.yout, y, sizeof(float) * (size_t)N * P.OC * H * W,
                             hipMemcpyDeviceToDevice, s));
  return DN_OK;
}

}  // namespace

// Every pass: a dry run queues the weight image of each conv into its arena slot, the queued
// packs launch (24 images per launch), then the pass runs on them.
dn_status iunet_forward(const IPlan& p, const float* prm, const float* x, float* y, float* ws,
                        hipStream_t s, int prec) {
  const StreamDeviceGuard device_guard(s);
  if (prec != DN_PREC_FP32 && prec != DN_PREC_FP32_X6) return DN_ERR_ARG;
  PackBatch pb;
  long next = 0;
  Ctx c{p, prm, ws, s, prec};
  c.pb = &pb; c.next = &next; c.dry = true;
  if (dn_status st = forward_body(c, x, y)) return st;
  IU_TRY(pack_flush(pb, s));
  next = 0; c.dry = false;
  if (dn_status st = forward_body(c, x, y)) return st;
  g_prof.flush("iunet forward");
  return DN_OK;
}

// ------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------
namespace {

// dW (+ db) of a conv from g = dL/d(conv output) and its input x; written into dprm
dn_status wgrad_g(const Ctx& c, float* dprm, int mode, const IConv& L, const View& g, const View& x,
                  int h, int w) {
  if (c.dry) return DN_OK;
  // on the side stream, behind the main stream's work so far (g is its latest output)
  const hipStream_t s2 = c.s2 ? c.s2 : c.s;
  if (s2 != c.s) {
    IU_TRY(hipEventRecord(c.fork, c.s));
    IU_TRY(hipStreamWaitEvent(s2, c.fork, 0));
  }
  OpScope prof(s2, "wgrad", L.cout, L.cin, L.k, h, w, c.p.N, 1.0);
  const int taps = mode == W_C3 ? 9 : 1;
  const bool bias = L.b >= 0;
  if (bias && L.b != L.w + (long)L.cout * L.cin * taps) {
    set_error("ImprovedUNet: bias does not follow its weight");
    return DN_ERR_ARG;
  }
  if (!gwgrad_ok(mode, L.cin, L.cout, g, x)) {
    set_error("ImprovedUNet: no weight-gradient kernel for this layer shape");
    return DN_ERR_ARG;
  }
  float* slab = c.ws + c.p.slab;
  const long n = (long)L.cout * L.cin * taps + (bias ? L.cout : 0);
  WgradArgs a{};
  a.g = g.p; a.g_stride = g.stride; a.g_off = g.off;
  a.x = x.p; a.x_stride = x.stride; a.x_off = x.off;
  a.N = c.p.N; a.KH = h; a.KW = w; a.Cout = L.cout; a.Cin = L.cin;
  a.zeros = slab; a.slab = slab + 64; a.slab_stride = n;
  a.wlayout = 0; a.cin_total = L.cin; a.ci_base = 0; a.bias = bias ? 1 : 0;
  int sp = gwgrad_splits(mode, c.p.N, h, w, L.cin, L.cout);
  IU_TRY(hipMemsetAsync(slab, 0, 64 * sizeof(float), s2));
  // fp32_x6: the 3x3 weight gradients on the bf16x6 kernel too
  if (c.prec == DN_PREC_FP32_X6 && mode == W_C3 && gwgrad_x6_ok(a)) {
    sp = gwgrad_x6_splits(a, sp);
    IU_TRY(launch_gwgrad_x6(a, sp, s2));
  } else {
    IU_TRY(launch_gwgrad(mode, a, sp, s2));
  }
  IU_TRY(launch_reduce(slab + 64, n, sp, n, dprm + L.w, s2));
  return DN_OK;
}

// dx (first nout input channels) = conv^T(g) with epilogue epi (aux = mask / residual)
dn_status dgrad_g(const Ctx& c, const IConv& L, const View& g, int h, int w, int nout, int epi,
                  const View& aux, const View& dx) {
  const int tail = x6_tail_for(g, c.p.N, h, w, L.cout, nout, w6_views(dx, OUT_NHWC, aux, nout));
  const bool x6 = c.prec == DN_PREC_FP32_X6 && L.k == 3 && x6_takes(L.cout, nout, tail);
  float* pk = c.slot(x6 ? (x6_pack_elems(L.cout, nout, x6_zc(nout)) + 1) / 2
                        : gpack_floats(L.k, L.cout, nout));
  if (!pk) {
    set_error("ImprovedUNet: packed-weight arena overrun (backward)");
    return DN_ERR_ARG;
  }
  if (c.dry) {
    PackJob j;
    const bool ok = x6 ? pack_job_x6(conv_dgrad_view(c.Wt(L), L.cin, 3), L.cout, nout,
                                     x6_zc(nout), pk, tail, j)
                       : gjob_dgrad(c.Wt(L), L.k, L.cin, L.cout, nout, pk, j);
    if (!ok) {
      set_error("ImprovedUNet: no weight image for a data gradient");
      return DN_ERR_ARG;
    }
    IU_TRY(pack_add(*c.pb, j, c.s));
    return DN_OK;
  }
  OpScope prof(c.s, "dgrad", nout, L.cout, L.k, h, w, c.p.N, 1.0);
  if (x6)
    IU_TRY(x6run(g, c.p.N, h, w, L.cout, pk, nout, nullptr, epi, dx, OUT_NHWC, aux, tail, c.s));
  else
    IU_TRY(grun(L.k, g, c.p.N, h, w, L.cout, pk, nout, nullptr, epi, dx, OUT_NHWC, aux, c.s));
  return DN_OK;
}

dn_status gn_bwd(const Ctx& c, float* dprm, const IGN& g, const View& dy, const View& z, int h,
                 int w, const float* stats, const View& dz) {
  if (c.dry) return DN_OK;
  OpScope prof(c.s, "gnbwd", g.C, 1, 1, h, w, c.p.N, 0.0);
  const int N = c.p.N;
  const long P = (long)h * w;
  const int S = chan_sums_splits(N, P);
  double* part = reinterpret_cast<double*>(c.ws + c.p.gpart);
  IU_TRY(launch_chan_sums(dy, &z, N, P, g.C, S, part, c.s));
  IU_TRY(launch_gn_bwd_fin(part, S, N, g.C, g.G, P, c.prm + g.g, stats, c.ws + c.p.ca,
                           c.ws + c.p.cb, c.ws + c.p.ccf, dprm + g.g, dprm + g.b, c.s));
  IU_TRY(launch_affine(dy, &z, c.ws + c.p.ca, c.ws + c.p.cb, c.ws + c.p.ccf, 0, nullptr, dz, N, P,
                       g.C, c.s));
  return DN_OK;
}

// ResBlock backward: dout -> b.dr (gradient of the block input r)
dn_status res_bwd(const Ctx& c, float* dprm, const IRes& R, const IBlockBufs& b, const View& dout,
                  int h, int w) {
  const int C = R.C;
  if (dn_status st = gn_bwd(c, dprm, R.n2, dout, c.V(b.z2, C), h, w, c.ws + b.st2, c.V(b.dz2, C)))
    return st;
  if (dn_status st = wgrad_g(c, dprm, W_C3, R.c2, c.V(b.dz2, C), c.V(b.a1, C), h, w)) return st;
  if (dn_status st = dgrad_g(c, R.c2, c.V(b.dz2, C), h, w, C, EPI_MASK, c.V(b.a1, C), c.V(b.dg1, C)))
    return st;
  if (dn_status st = gn_bwd(c, dprm, R.n1, c.V(b.dg1, C), c.V(b.z1, C), h, w, c.ws + b.st1,
                            c.V(b.dz1, C)))
    return st;
  if (dn_status st = wgrad_g(c, dprm, W_C3, R.c1, c.V(b.dz1, C), c.V(b.r, C), h, w)) return st;
  // d r = conv1^T(dz1) + dout  (the residual), EPI_BIAS_ADD with no bias
  return dgrad_g(c, R.c1, c.V(b.dz1, C), h, w, C, EPI_BIAS_ADD, dout, c.V(b.dr, C));
}

// RDB backward: b.dr (gradient of the RDB output) -> b.dF[:, :C] (gradient of the block input)
dn_status rdb_bwd(const Ctx& c, float* dprm, const IRdb& R, const IBlockBufs& b, int h, int w) {
  const int C = R.C, FS = C + 4 * GROWTH;
  const long npx = (long)c.p.N * h * w;
  const View dr = c.V(b.dr, C);
  if (dn_status st = wgrad_g(c, dprm, W_C1, R.lff, dr, c.V(b.F, FS), h, w)) return st;
  if (dn_status st = dgrad_g(c, R.lff, dr, h, w, FS, EPI_PLAIN, kNone, c.V(b.dF, FS))) return st;
  IU_RUN(c, launch_vadd(c.V(b.dF, FS), dr, npx, C, c.s));  // out = x + lff(...)
                        for (int j = 3; j >= 0; --j) {
                        const int o = C + GROWTH * j;
    const View dzj = c.V(b.dzj[j], GROWTH);
    IU_RUN(c, launch_vmask(dzj, c.V(b.dF, FS, o), c.V(b.F, FS, o), npx, GROWTH, c.s));
    if (dn_status st = wgrad_g(c, dprm, W_C3, R.conv[j], dzj, c.V(b.F, FS), h, w)) return st;
    if (dn_status st = dgrad_g(c, R.conv[j], dzj, h, w, o, EPI_ACCUM, kNone,
                               c.V(b.dF, FS)))
      return st;
  }
  return DN_OK;
}

// the backward's launches (Ctx::dry: only the data gradients' weight images are queued)
dn_status backward_body(const Ctx& c, const float* dy, float* dprm, SideStream* side) {
  const IPlan& p = c.p;
  const float* prm = c.prm;
  float* ws = c.ws;
  const hipStream_t s = c.s;
  const hipStream_t s2 = side ? side->st : s;
  auto fork = [&]() -> hipError_t {
    if (!side) return hipSuccess;
    hipError_t e = hipEventRecord(side->fork, s);
    return e != hipSuccess ? e : hipStreamWaitEvent(s2, side->fork, 0);
  };
  const IParams& P = p.P;
  const int N = p.N, H = p.H, W = p.W, C = P.C, OC = P.OC;
  const long HW = (long)H * W;
  // final: dz = dy * y(1-y)  (stride-4 NHWC), then its weight / data gradients
  IU_RUN(c, launch_dsigmoid_nchw(ws + p.yout, dy, N, OC, HW, ws + p.dzfin, 4, s));
  if (dn_status st = wgrad_g(c, dprm, W_C3, P.fin, c.V(p.dzfin, 4), c.V(p.cf, 28), H, W)) return st;
  // gradient of x_up3 = the first 24 channels of the final concat (the input slice needs
  // none); dh (48 channels) is free until the noise estimator's backward
  IU_RUN(c, hipMemsetAsync(ws + p.dsg, 0, sizeof(float) * 4 * (size_t)N * HW, s));
  const View dfin = c.V(p.dh, 24);
  if (dn_status st = dgrad_g(c, P.fin, c.V(p.dzfin, 4), H, W, 24, EPI_PLAIN, kNone, dfin)) return st;
  // decoder, last block first
  View dcur = dfin;
  for (int k = 3; k >= 0; --k) {
    const IUp& u = P.up[k];
    const int l = 3 - k, h = H >> l, w = W >> l, out = u.out, FS = out + 4 * GROWTH;
    const IBlockBufs& b = p.ul[k];
    if (dn_status st = res_bwd(c, dprm, u.res, b, dcur, h, w)) return st;
    if (dn_status st = rdb_bwd(c, dprm, u.rdb, b, h, w)) return st;
    // f = leaky(fuse(cc)): dz = dF[:, :out] * leaky'(f)
    const View dzf = c.V(b.dzf, out);
    IU_RUN(c, launch_vmask(dzf, c.V(b.dF, FS), c.V(b.F, FS), (long)N * h * w, out, s));
    if (dn_status st = wgrad_g(c, dprm, W_C3, u.fuse, dzf, c.V(p.cc[k], 3 * out), h, w)) return st;
    if (dn_status st = dgrad_g(c, u.fuse, dzf, h, w, 3 * out, EPI_PLAIN, kNone,
                               c.V(p.dcc[k], 3 * out)))
      return st;
    // PixelShuffle backward, then conv_ps (input: bottle output or the previous up block)
    float* gps = ws + p.dps[k];
    IU_RUN(c, launch_unshuffle(c.V(p.dcc[k], 3 * out), N, h / 2, w / 2, out, gps, s));
    const View xin = k == 0 ? c.V(p.xb, 384) : c.V(p.xu[k - 1], u.in);
    if (dn_status st = wgrad_g(c, dprm, W_C3, u.ps, View{gps, 4 * out, 0}, xin, h / 2, w / 2))
      return st;
    const View dxin = k == 0 ? c.V(p.dxb, 384) : c.V(p.dxu[k - 1], u.in);
    if (dn_status st = dgrad_g(c, u.ps, View{gps, 4 * out, 0}, h / 2, w / 2, u.in, EPI_PLAIN,
                               kNone, dxin))
      return st;
    dcur = dxin;
  }
  // bottleneck: its input is pool(s_3), living in bb.F[:, :384]
  if (dn_status st = res_bwd(c, dprm, P.bres, p.bb, c.V(p.dxb, 384), H >> 4, W >> 4)) return st;
  if (dn_status st = rdb_bwd(c, dprm, P.brdb, p.bb, H >> 4, W >> 4)) return st;
  View dpooled = c.V(p.bb.dF, 384 + 4 * GROWTH);  // d x_4 (first 384 channels)
  // encoder, deepest level first
  for (int i = 3; i >= 0; --i) {
    const ILevel& L = P.down[i];
    const int h = H >> i, w = W >> i, nf = L.conv.cout, FS = nf + 4 * GROWTH;
    const IBlockBufs& b = p.dl[i];
    const int k = 3 - i, out = P.up[k].out;
    const View skip = c.V(p.cc[k], 3 * out, out), dskip = c.V(p.dcc[k], 3 * out, out);
    // d s_i = (skip gradient from the fuse conv) + maxpool backward of d x_{i+1}
    IU_RUN(c, launch_vpool_bwd_acc(skip, N, h, w, nf, dpooled, dskip, s));
    if (dn_status st = res_bwd(c, dprm, L.res, b, dskip, h, w)) return st;
    if (dn_status st = rdb_bwd(c, dprm, L.rdb, b, h, w)) return st;
    const View dza = c.V(p.dza[i], nf);
    IU_RUN(c, launch_vmask(dza, c.V(b.dF, FS), c.V(b.F, FS), (long)N * h * w, nf, s));
    if (i > 0) {
      const View xi = c.V(p.pool[i], L.conv.cin);
      if (dn_status st = wgrad_g(c, dprm, W_C3, L.conv, dza, xi, h, w)) return st;
      if (dn_status st = dgrad_g(c, L.conv, dza, h, w, L.conv.cin, EPI_PLAIN, kNone,
                                 c.V(p.dpool, L.conv.cin)))
        return st;
      dpooled = c.V(p.dpool, L.conv.cin);
    } else {
      // level-0 conv: input x0 = [x | sigma] with C+1 < 16 channels -> the thin wgrad kernel on
      // the NCHW input (channels [0, C)) and sigma map (channel C), into one slab
      float* slab = ws + p.slab;
      const long n = 48L * (C + 1) * 9 + 48;
      const int st = enc0_wgrad_splits(N, H, W);
      IU_RUN(c, fork());
      IU_RUN(c, launch_wgrad_c3_thin(ws + p.dza[0], 48, ws + p.xin, N, C, H, W, slab, n, C + 1, 0,
                                     1, st, s2));
      IU_RUN(c, launch_wgrad_c3_thin(ws + p.dza[0], 48, ws + p.sig, N, 1, H, W, slab, n, C + 1, C,
                                     0, st, s2));
      IU_RUN(c, launch_reduce(slab, n, st, n, dprm + L.conv.w, s2));
      // d sigma (channel C of x0) through the sigmoid: flipped weight column ci = C
      WView fv{};
      fv.w = prm + L.conv.w; fv.off = (long)C * 9; fv.sN = 9; fv.sK = (long)(C + 1) * 9;
      fv.sT = 1; fv.taps = 9; fv.flip = 1;
      IU_RUN(c, launch_conv3_thin(dza, N, H, W, 48, fv, nullptr, TE_DSIG, c.V(p.x0, 4, C),
                                  c.V(p.dsg, 4), 0, 1, s));
    }
  }
  // noise estimator: ne2 (48 -> 1) and ne0 (C -> 48)
  if (dn_status st = wgrad_g(c, dprm, W_C3, P.ne2, c.V(p.dsg, 4), c.V(p.h, 48), H, W)) return st;
  if (dn_status st = dgrad_g(c, P.ne2, c.V(p.dsg, 4), H, W, 48, EPI_MASK, c.V(p.h, 48),
                             c.V(p.dh, 48)))
    return st;
  {
    float* slab = ws + p.slab;
    const long n = 48L * C * 9 + 48;
    const int st = enc0_wgrad_splits(N, H, W);
    IU_RUN(c, fork());
    IU_RUN(c, launch_wgrad_c3_thin(ws + p.dh, 48, ws + p.xin, N, C, H, W, slab, n, C, 0, 1, st,
                                   s2));
    IU_RUN(c, launch_reduce(slab, n, st, n, dprm + P.ne0.w, s2));
  }
  if (side) {  // the caller's stream continues after every weight gradient
    IU_RUN(c, hipEventRecord(side->join, s2));
    IU_RUN(c, hipStreamWaitEvent(s, side->join, 0));
  }
  return DN_OK;
}

}  // namespace

dn_status iunet_backward(const IPlan& p, const float* prm, const float* dy, float* dprm, float* ws,
                         hipStream_t s, int prec) {
  const StreamDeviceGuard device_guard(s);
  if (prec != DN_PREC_FP32 && prec != DN_PREC_FP32_X6) return DN_ERR_ARG;
  // The weight gradients (and their slab reductions) run on a side stream beside the
  // data-gradient chain (DN_BWD_STREAMS=0 or per-op profiling: one stream).  Each is forked after
  // the launch that produced its output gradient; every buffer one reads (the forward's
  // activations, dz2 / dz1 / dr / dzf of a block, dzj[j], dps[k], dza[i], dzfin, dsg, dh once
  // written) is not rewritten later in the pass, and only they use the slab.  Joined at the end.
  static const bool two_env = !getenv("DN_BWD_STREAMS") || atoi(getenv("DN_BWD_STREAMS")) != 0;
  SideStream* side = two_env && !prof_on() && !g_prof.on ? side_stream(s) : nullptr;
  PackBatch pb;
  long next = 0;
  Ctx c{p, prm, ws, s, prec};
  if (side) { c.s2 = side->st; c.fork = side->fork; }
  c.pb = &pb; c.next = &next; c.dry = true;
  if (dn_status st = backward_body(c, dy, dprm, side)) return st;
  IU_TRY(pack_flush(pb, s));
  next = 0; c.dry = false;
  if (dn_status st = backward_body(c, dy, dprm, side)) return st;
  g_prof.flush("iunet backward");
  return DN_OK;
}

}  // namespace dn
