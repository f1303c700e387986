// bf16x6 3x3 convolution (forward / data gradient) with the weights in registers (k_c3x6r):
// the 96-output-channel shapes of the N2N step without a workgroup barrier per tap.
//
// k_c3x6p shares each tap's 18 KiB weight stage between its 8 waves through an LDS ring, so every
// tap ends on a workgroup barrier (measured with stage stamps: ~650 barrier + ~400 tail cycles
// of a ~3700-cycle stage whose MFMA floor is 2304).  Here the 16 x 16 x 96 tile is split over the
// waves by output channels as well as rows: wave (mq, nh) = (w & 3, w >> 2) computes tile rows
// 4mq .. 4mq+3 (four M fragments) for output channels 48nh .. 48nh+47 (three N fragments), and
// loads ITS weights of a tap -- 3 fragments x 3 planes, one 16-B buffer load per lane each --
// straight from the pre-split image (L2 / L1) into registers, one tap ahead.  Only the x tile is
// shared: double-buffered in LDS (the next chunk's tile loaded into registers at the chunk's
// first tap, split into the other buffer at its fourth), so the waves meet at one barrier per
// 32-channel chunk instead of one per tap, and each tap reads 4 x 3 A fragments from LDS for its
// 72 MFMAs (k_c3x6p: 2 x 3 A + 6 x 3 B for 72).  The weight image and its packing (pk_x6, the
// tail modes of the last chunk) are k_c3x6p's.
#include <cstdlib>
#include <string>
#include <type_traits>

#include "conv_epi.h"
#include "x6_core.h"

namespace dn {

struct RCfg {
  static constexpr int WAVES = 8, MT = 4, NTW = 3, NP = 96;
  static constexpr int TW = 16, TH = 16, IH = TH + 2, IW = TW + 2, KC = 32;
  static constexpr int XPIX = IH * IW;
  static constexpr int XPL = XPIX * KC;      // bf16 per plane of an x buffer
  static constexpr int XBUF = 3 * XPL;       // bf16 per x buffer (three planes)
  static constexpr int WPL = NP * KC;        // bf16 per plane of a weight stage
  static constexpr int WSTP = x6_wst(NP);    // stage stride of the packed image (bf16)
  static constexpr int XQ = XPIX * (KC / 4);
  static constexpr int XITEMS = (XQ + WAVES * 64 - 1) / (WAVES * 64);
  static constexpr int PS = 16 * NTW + 4;    // epilogue staging pixel stride (floats)
  static constexpr int LEPI = 16 * PS;       // floats of one wave's staging area
  static constexpr int LBYTES = 2 * XBUF * 2 + WAVES * LEPI * 4;
  static_assert(LBYTES <= 163840, "one workgroup per CU");
};

__device__ __forceinline__ void x6r_barrier() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);  // no compiler motion of LDS accesses across it
  __builtin_amdgcn_s_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// f(integral_constant<I>) for I in [I0, N): compile-time tap indices, so the alternating weight
// register sets are never indexed at run time
template <int I0, int N, class F>
__device__ __forceinline__ void x6r_for(F&& f) {
  if constexpr (I0 < N) {
    f(std::integral_constant<int, I0>{});
    x6r_for<I0 + 1, N>(f);
  }
}

// per-block sums (x6_block: the five corrections summed from zero per block, 8 VALU adds per
// fragment) by default: the carried form's 48 extra accumulators do not fit beside the two
// weight register sets at 2 waves per SIMD
#ifndef DN_X6R_CARRY
#define DN_X6R_CARRY 0
#endif
#ifndef DN_X6R_MH
#define DN_X6R_MH 2
#endif
#ifndef DN_X6R_XG
#define DN_X6R_XG 3  // groups the next chunk's x tile is staged in (see k_c3x6r)
#endif
#ifndef DN_X6R_DEFAULT
#define DN_X6R_DEFAULT 0  // DN_X6_REG unset: k_c3x6r off (0) / on (1)
#endif

template <int TAIL>
__global__ __launch_bounds__(512, 1) void k_c3x6r(FwdArgs a) {
  using C = RCfg;
  constexpr int MT = C::MT, NTW = C::NTW;
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[C::LBYTES];
  __bf16* lx = reinterpret_cast<__bf16*>(lds_raw);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lg = lane >> 4;
  const int mq = wave & 3, nh = wave >> 2;
  const int tiles_x = (a.OW + C::TW - 1) / C::TW;
  int bxr, byr;  // XCD-aware tile order (conv_epi.h xcd_tile)
  xcd_tile(bxr, byr);
  const int ty0 = (bxr / tiles_x) * C::TH, tx0 = (bxr % tiles_x) * C::TW, n = byr;
  const int iy0 = ty0 - 1, ix0 = tx0 - 1;
  const float* inb = a.in + (long)n * a.IHt * a.IWt * a.in_stride + a.in_off;
  const int nch = (a.K + C::KC - 1) / C::KC;
  constexpr int tail_st = TAIL == 1 ? 2 : 5;
  const int nst = 9 * nch - (TAIL ? 9 - tail_st : 0);

  constexpr int MH = DN_X6R_MH;  // M fragments whose A operands are in registers at once
  f32x4 acc[MT][NTW], accl[DN_X6R_CARRY ? MT : 1][NTW];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < NTW; ++q) acc[m][q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int m = 0; m < (DN_X6R_CARRY ? MT : 1); ++m)
#pragma unroll
    for (int q = 0; q < NTW; ++q) accl[m][q] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the tile's input rows through a 32-bit buffer resource (out-of-range offsets read zeros)
  const int ry0 = iy0 > 0 ? iy0 : 0, ry1 = iy0 + C::IH < a.IHt ? iy0 + C::IH : a.IHt;
  const long row_floats = (long)a.IWt * a.in_stride;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(inb + ry0 * row_floats), (short)0, (int)((ry1 - ry0) * row_floats * 4),
      0x00020000);
  // the next chunk's x tile moves in XG groups of XPG items (registers of one group at a time):
  // group g is loaded at tap 2g and split into the other buffer at tap 2g + 2
  constexpr int XG = DN_X6R_XG, XPG = (C::XITEMS + XG - 1) / XG;
  static_assert(2 * XG + 1 <= 8, "the last group is stored before the chunk's last tap");
  f32x4 xr[C::XITEMS];
  auto load_x = [&](int k0, int tid, int g0 = 0, int g1 = C::XITEMS) {
#pragma unroll
    for (int it = g0; it < g1; ++it) {
      const int e = tid + it * C::WAVES * 64;
      const int q = e % (C::KC / 4), pix = e / (C::KC / 4);
      const int iy = pix / C::IW, ix = pix - iy * C::IW;
      const int gy = iy0 + iy, gx = ix0 + ix, k = k0 + 4 * q;
      const bool ok = e < C::XQ && gy >= 0 && gy < a.IHt && gx >= 0 && gx < a.IWt && k < a.K;
      const int off = ok ? (((gy - ry0) * a.IWt + gx) * a.in_stride + k) * 4 : 0x7fffffff;
      xr[it] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
    }
  };
  auto store_x = [&](__bf16* xb, int tid, int g0 = 0, int g1 = C::XITEMS) {
#pragma unroll
    for (int it = g0; it < g1; ++it) {
      const int e = tid + it * C::WAVES * 64;
      if (e < C::XQ) {
        const int q = e % (C::KC / 4), pix = e / (C::KC / 4);
        const float f[4] = {xr[it][0], xr[it][1], xr[it][2], xr[it][3]};
        bf16x4 h, m, l;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          __bf16 hj, mj, lj;
          split3(f[j], hj, mj, lj);
          h[j] = hj; m[j] = mj; l[j] = lj;
        }
        const int off = pix * C::KC + x6_swz(pix, q >> 1) * 8 + (q & 1) * 4;
        *reinterpret_cast<bf16x4*>(xb + off) = h;
        *reinterpret_cast<bf16x4*>(xb + C::XPL + off) = m;
        *reinterpret_cast<bf16x4*>(xb + 2 * C::XPL + off) = l;
      }
    }
  };
  // this wave's weights of stage st: fragment j = output channels 48nh + 16j .. +15, plane p;
  // lane (li, lg) holds row 48nh + 16j + li, k = 8lg .. 8lg+7 (quad x6_swz(row, lg) of the row)
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.wp), (short)0, nst * C::WSTP * 2, 0x00020000);
  int woff[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int row = (NTW * nh + j) * 16 + li;
    woff[j] = (row * C::KC + x6_swz(row, lg) * 8) * 2;
  }
  auto load_w = [&](int st, bf16x8 (&w)[3][NTW]) {
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int j = 0; j < NTW; ++j)
        w[p][j] = __builtin_bit_cast(
            bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, (st * C::WSTP + p * C::WPL) * 2 + woff[j], 0, 0));
  };

  // one tap of this wave's 4 x 3 fragments: MODE 0 = a full chunk's tap t; 1 / 2 = stage t of a
  // tail-packed last chunk (x6_tail_mode: im2col of <= 4 channels / tap pairs of <= 16 channels)
  auto tap = [&](auto mode_tag, const __bf16* xb, int t, const bf16x8 (&w)[3][NTW], int li, int lg) {
    constexpr int MODE = decltype(mode_tag)::value;
#pragma unroll
    for (int mh = 0; mh < MT / MH; ++mh) {
    bf16x8 av[3][MH];
    if constexpr (MODE == 1) {
      const int ta = 8 * t + 2 * lg, tb = ta + 1;
      const int ca = ta < 9 ? ta : 8, cb = tb < 9 ? tb : 8;
      const int da = (ca / 3) * C::IW + ca % 3, db = (cb / 3) * C::IW + cb % 3;
      const bf16x4 z4 = {(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
#pragma unroll
      for (int m = 0; m < MH; ++m) {
        const int p0 = (mq * MT + mh * MH + m) * C::IW + li;
        const int pa = p0 + da, pb = p0 + db;
        const int oa = pa * C::KC + x6_swz(pa, 0) * 8, ob = pb * C::KC + x6_swz(pb, 0) * 8;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          bf16x4 va = *reinterpret_cast<const bf16x4*>(xb + p * C::XPL + oa);
          bf16x4 vb = *reinterpret_cast<const bf16x4*>(xb + p * C::XPL + ob);
          if (ta > 8) va = z4;
          if (tb > 8) vb = z4;
          av[p][m] = __builtin_shufflevector(va, vb, 0, 1, 2, 3, 4, 5, 6, 7);
        }
      }
    } else if constexpr (MODE == 2) {
      const int ta = 2 * t + (lg >> 1);
      const int ca = ta < 9 ? ta : 8;
      const int da = (ca / 3) * C::IW + ca % 3;
      const bf16x8 z8 = {};
#pragma unroll
      for (int m = 0; m < MH; ++m) {
        const int pa = (mq * MT + mh * MH + m) * C::IW + li + da;
        const int oa = pa * C::KC + x6_swz(pa, lg & 1) * 8;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(xb + p * C::XPL + oa);
          av[p][m] = ta > 8 ? z8 : v;
        }
      }
    } else {
      const int ky = t / 3, kx = t - 3 * ky;
#pragma unroll
      for (int m = 0; m < MH; ++m) {
        const int pix = (mq * MT + mh * MH + m + ky) * C::IW + li + kx;
        const int off = pix * C::KC + x6_swz(pix, lg) * 8;
#pragma unroll
        for (int p = 0; p < 3; ++p) av[p][m] = *reinterpret_cast<const bf16x8*>(xb + p * C::XPL + off);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    f32x4(&ah)[MH][NTW] = *reinterpret_cast<f32x4(*)[MH][NTW]>(&acc[mh * MH]);
    // one output fragment at a time, its adds into acc pinned right behind its MFMAs (the
    // compiler otherwise sinks every group's adds to the end and spills the block sums)
#pragma unroll
    for (int g = 0; g < NTW; ++g) {
#if DN_X6R_CARRY
      f32x4(&alh)[MH][NTW] = *reinterpret_cast<f32x4(*)[MH][NTW]>(&accl[mh * MH]);
      x6_group_c<MH, NTW, 1>(ah, alh, av, w, g);
#else
      x6_group<MH, NTW, 1>(ah, av, w, g);
#endif
#pragma unroll
      for (int i = 0; i < MH; ++i) asm volatile("" : "+v"(ah[i][g]));
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_sched_barrier(0);
    }
  };

  bf16x8 w0[3][NTW], w1[3][NTW];
  load_w(0, w0);
  load_x(0, tid);
  store_x(lx, tid);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own x-tile stores done
  x6r_barrier();

  using M0 = std::integral_constant<int, 0>;
#pragma unroll 1
  for (int c = 0; c < nch; ++c) {
    // the lane's tile coordinates re-derived per chunk from opaque copies: otherwise the compiler
    // hoists every tap's LDS offsets (and the x loads' bounds masks) out of the chunk loop and
    // spills them
    int liv = li, lgv = lg, tidv = tid;
    asm volatile("" : "+v"(liv), "+v"(lgv), "+v"(tidv));
    const __bf16* xb = lx + (c & 1) * C::XBUF;
    __bf16* xn = lx + ((c + 1) & 1) * C::XBUF;
    const bool more = c + 1 < nch;
    const int st0 = 9 * c;
    if (TAIL && !more) {  // the tail-packed last chunk: tail_st stages, nothing to prefetch after
      using MT_ = std::integral_constant<int, TAIL == 1 ? 1 : 2>;
      x6r_for<0, tail_st>([&](auto ti) {
        constexpr int t = decltype(ti)::value;
        if constexpr (t + 1 < tail_st) {
          if constexpr (t & 1) load_w(st0 + t + 1, w0);
          else load_w(st0 + t + 1, w1);
        }
        if constexpr (t & 1) tap(MT_{}, xb, t, w1, liv, lgv);
        else tap(MT_{}, xb, t, w0, liv, lgv);
      });
      break;
    }
    // a full chunk: taps 0..8 alternate w0 / w1 (tap t + 1's weights requested before tap t)
    x6r_for<0, 9>([&](auto ti) {
      constexpr int t = decltype(ti)::value;
      const int nxt = st0 + t + 1;
      if (nxt < nst) {
        if constexpr (t & 1) load_w(nxt, w0);
        else load_w(nxt, w1);
      }
      if constexpr (t % 2 == 0 && t / 2 < XG) {
        constexpr int g = t / 2;
        if (more) load_x((c + 1) * C::KC, tidv, g * XPG, (g + 1) * XPG < C::XITEMS ? (g + 1) * XPG : C::XITEMS);
      }
      if constexpr (t & 1) tap(M0{}, xb, t, w1, liv, lgv);
      else tap(M0{}, xb, t, w0, liv, lgv);
      if constexpr (t % 2 == 0 && t >= 2 && t / 2 - 1 < XG) {
        constexpr int g = t / 2 - 1;
        if (more) store_x(xn, tidv, g * XPG, (g + 1) * XPG < C::XITEMS ? (g + 1) * XPG : C::XITEMS);
      }
    });
    // tap 8 read w0 and requested the next chunk's tap 0 into w1: move it (the waves' own copies)
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int j = 0; j < NTW; ++j) w0[p][j] = w1[p][j];
    if (more) {
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own stores of the next x tile done
      x6r_barrier();                       // the next tile complete; this one's readers done
    }
  }
#if DN_X6R_CARRY
  x6_fold(acc, accl);
#endif
  // the staging areas sit past the two x buffers: no barrier before the epilogue
  float* st = reinterpret_cast<float*>(lds_raw + 2 * C::XBUF * 2) + wave * C::LEPI;
  fwd_epilogue_at<NTW, MT, C::PS>(a, acc, st, ty0, tx0, n, mq * MT, nh * 16 * NTW, 16 * NTW);
}

// A/B switch DN_X6_REG (default 0 until measured): the 96-channel shapes on k_c3x6r
bool x6r_enabled() {
  static const bool on = getenv("DN_X6_REG") ? atoi(getenv("DN_X6_REG")) != 0 : DN_X6R_DEFAULT != 0;
  return on;
}

// k_c3x6r for a 96-output-channel forward / data gradient: NHWC float4 output with a vec epilogue
// kind, float4-aligned input views, one channel block (zc = 0); false = not taken
bool launch_fwd_x6r(const FwdArgs& a, hipStream_t s, hipError_t& err) {
  using C = RCfg;
  const bool aux = a.epi == EPI_MASK || a.epi == EPI_BIAS_ADD;
  if (a.NOUT != 96 || a.zc || a.out_layout != OUT_NHWC || a.sel_rd ||
      ((a.out_stride | a.out_off | a.NOUT) & 3) || (aux && ((a.mask_stride | a.mask_off) & 3)) ||
      a.epi < EPI_BIAS || a.epi > EPI_BIAS_ADD || ((a.in_stride | a.in_off | a.K) & 3) ||
      (long)C::IH * a.IWt * a.in_stride * 4 >= 0x7fffffffL || a.x6_tail > 2)
    return false;
  const int tx = (a.OW + C::TW - 1) / C::TW, ty = (a.OH + C::TH - 1) / C::TH;
  const dim3 grid(tx * ty, a.N, 1), block(C::WAVES * 64);
  static const char* kn[3] = {"k_c3x6r<0>", "k_c3x6r<1>", "k_c3x6r<2>"};
  prof_kernel(kn[a.x6_tail]);
  if (a.x6_tail == 1)
    hipLaunchKernelGGL(k_c3x6r<1>, grid, block, 0, s, a);
  else if (a.x6_tail == 2)
    hipLaunchKernelGGL(k_c3x6r<2>, grid, block, 0, s, a);
  else
    hipLaunchKernelGGL(k_c3x6r<0>, grid, block, 0, s, a);
  err = hipGetLastError();
  return true;
}

}  // namespace dn
