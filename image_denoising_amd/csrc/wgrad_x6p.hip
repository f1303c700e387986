// 3x3 weight gradient at fp32 accuracy on the bf16 matrix cores, operands split ONCE per stage
// into bf16 planes (k_wgrad3p: 96 output channels).
//
// GEMM M = output channels, N = input channels x 9 taps, K = pixels (as k_wgrad3s,
// conv_x6.hip).  k_wgrad3s splits each fp32 operand at the read, so every value is split by
// each of the two waves that share it, and the three horizontal taps need funnel shifts of the
// split window: its stage loop is vector-issue bound (SQ counters: every issue slot of a SIMD
// taken, MFMA busy 0.46).  Here the next stage's fp32 operands are loaded into registers (buffer
// loads, out-of-range offsets read zeros) while the current stage computes, split once by the
// workgroup's threads and written into three bf16 planes of the other LDS buffer; the MFMA
// operands are read from the planes with ds_read_b64_tr_b16, the hardware transpose that turns
// pixel-major (NHWC) bf16 rows into the K-contiguous fragment a lane needs.  A tap offset is
// then only a different starting row of the X plane.  One barrier per stage.
//
//   Workgroup = 4 waves (two workgroups per CU), wave (wm, wn): output channels 48wm .. +47
//   (three 16-row fragments) x input channels ci0 + 16wn .. +15 x 9 taps; acc[9][3] fp32.
//   K stage = 32 pixels: 32 >> SWL rows of sw = 1 << SWL pixels (sw >= 8).
//   LDS: two buffers of three bf16 planes, each [G: 32 px x 96 co | X: (sh+2)(sw+2) px x 32 ci].
//   The 16 channels (32 B) of block b of pixel row r sit in block b ^ ((r >> 3) & 1) of the row: the two 16-lane groups of a 32-lane half read rows 8 apart,
//   which the flip puts on the other 32 banks (conflict-free transposed reads).
//   Each 32-pixel block of the six products is summed from zero and added to the running fp32
//   sum with a round-to-nearest add (x6_block), as in k_wgrad3s.
#include <cstdlib>

#include "conv_epi.h"
#include "x6_core.h"


namespace dn {

typedef short i16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ i16x4 lds_tr16(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) i16x4*)(p));
}

// eight K-consecutive bf16 of a lane (two transposed 4-row reads)
__device__ __forceinline__ bf16x8 tr_frag(const __bf16* p0, const __bf16* p1) {
  const i16x4 a = lds_tr16(p0), b = lds_tr16(p1);
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

// CO = 96: 4 waves (wm, wn) = 48 output channels x 16 of 32 input channels each.  CO = 48 (the
// encoder's 48 -> 48 layers): 3 waves, wn = 16 of 48 input channels, all 48 outputs; the G and X
// plane rows are padded to 64 channels (the block flip pairs blocks 2 and 3).
template <int SWL, int CO = 96>
struct Wp3Cfg {
  static constexpr int COUT = CO, MFW = 3, CIB = CO == 96 ? 32 : 48, NW = CO == 96 ? 4 : 3;
  static constexpr int NTHR = 64 * NW;
  static constexpr int GRW = CO == 96 ? 96 : 64, XRW = CO == 96 ? 32 : 64;  // plane row widths
  static constexpr int SW = 1 << SWL, SH = 32 >> SWL, XW = SW + 2, XPIX = (SH + 2) * XW;
  static constexpr int GQ = 32 * COUT / 4, XQ = XPIX * CIB / 4, NQ = GQ + XQ;  // float4 items
  static constexpr int NIT = (NQ + NTHR - 1) / NTHR;
  static constexpr int GPL = 32 * GRW, XPL = XPIX * XRW;   // bf16 of G / X per plane
  static constexpr int PL = GPL + XPL;                     // plane stride: [G | X]
  static constexpr int BUF = 3 * PL;                       // bf16 per stage buffer
  static_assert(CO == 96 || CO == 48, "96 or 48 output channels");
  static_assert(GQ % NTHR == 0, "items 0 .. GQ/NTHR - 1 of every thread are G items");
  static_assert(2 * BUF * 2 <= 81920, "two workgroups per CU");
};

// the swizzle of a 64-channel (128-B) plane row: a 16-lane group of ds_read_b64_tr_b16 reads
// rows s .. s+3 and the other group of its half-wave rows s+8 .. s+11, but a 128-B row covers
// only half of the 64 banks, so rows two apart collide; block b of row r sits in block
// b ^ (bit 1 of r | bit 3 of r << 1), which puts those eight rows on eight distinct 8-bank sets
// for any s (adding 8 toggles bit 3 only, adding 2 to an even row toggles bit 1)
__device__ __forceinline__ int wp_flip64(int r) { return ((r >> 1) & 1) | ((r >> 2) & 2); }

// plane index of channel block `blk` (16 channels) of row r (row width `rw` channels: 96 and
// 32 keep the bit-3 flip of two 32-B blocks, 64 the two-bit flip above)
__device__ __forceinline__ int wp_idx(int r, int rw, int blk) {
  if (rw == 64) return r * 64 + ((blk ^ wp_flip64(r)) << 4);
  return r * rw + ((blk ^ ((r >> 3) & 1)) << 4);
}

// diagnostic ablations of k_wgrad3p (wrong results, timing only; tools/probes/r5_wgabl.sh,
// profiles/r5_wgrad_ablation.log): NOS = no next-stage loads / splits / plane writes, NOLD = no
// next-stage global loads (the stale registers are split and written), NOBAR = no barrier
#ifndef DN_WG_ABL_NOS
#define DN_WG_ABL_NOS 0
#endif
#ifndef DN_WG_ABL_NOLD
#define DN_WG_ABL_NOLD 0
#endif
#ifndef DN_WG_ABL_NOBAR
#define DN_WG_ABL_NOBAR 0
#endif

// The next stage's G and X operands are loaded at the start of the stage and split into the other
// buffer at its end (a whole stage of load latency for both)
template <int SWL, int CO = 96>
__global__ __launch_bounds__(CO == 96 ? 256 : 192, 2) void k_wgrad3p(WgradArgs a0) {
  using C = Wp3Cfg<SWL, CO>;
  constexpr int MFW = C::MFW, SW = C::SW, SH = C::SH, XW = C::XW;
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * C::BUF];
  const WgradArgs a = wg_block(a0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = CO == 96 ? wave >> 1 : 0, wn = CO == 96 ? wave & 1 : wave;
  const int li = lane & 15, lg = lane >> 4;
  const int ci0 = blockIdx.y * C::CIB;
  const int ux = (a.KW + SW - 1) / SW, uy = (a.KH + SH - 1) / SH;
  const long U = (long)a.N * uy * ux;
  const long u_beg = U * blockIdx.x / gridDim.x, u_end = U * (blockIdx.x + 1) / gridDim.x;
  const bool do_bias = a.bias && blockIdx.y == 0 && wn == 0;

  f32x4 acc[9][MFW][1];
  f32x4 accb[MFW][1];
#pragma unroll
  for (int i = 0; i < MFW; ++i) {
    accb[i][0] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t][i][0] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // ---- the split pass: item q (a float4 of 4 channels of one pixel) of this thread ----------
  // Items 0 .. NG-1 of a thread are G items, NG .. NIT-1 X items.  Stage-invariant parts: the
  // offset relative to the stage origin, the LDS plane index of the 4 channels (low 16 bits) and
  // the halo-edge class (bits 16..: 0 top row, 1 bottom row, 2 left column, 3 right column,
  // 5 no data)
  constexpr int NG = C::GQ / C::NTHR, NX = C::NIT - NG;
  int ioff[C::NIT], ilde[C::NIT];
#pragma unroll
  for (int it = 0; it < C::NIT; ++it) {
    const int q = tid + it * C::NTHR;
    ioff[it] = 0; ilde[it] = 32 << 16;
    if (it < NG) {
      const int px = q / (C::COUT / 4), c = 4 * (q % (C::COUT / 4));
      ioff[it] = ((px >> SWL) * a.KW + (px & (SW - 1))) * a.g_stride + c;
      ilde[it] = (wp_idx(px, C::GRW, c >> 4) + (c & 15)) | ((c < a.Cout ? 0 : 32) << 16);
    } else if (q < C::NQ) {
      const int r = q - C::GQ, xp = r / (C::CIB / 4), c = 4 * (r % (C::CIB / 4));
      const int yy = xp / XW, xx = xp - yy * XW;
      ioff[it] = ((yy - 1) * a.KW + xx - 1) * a.x_stride + ci0 + c;
      const int e = (yy == 0) | ((yy == SH + 1) << 1) | ((xx == 0) << 2) | ((xx == SW + 1) << 3) |
                    ((ci0 + c < a.Cin ? 0 : 1) << 5);
      ilde[it] = (C::GPL + wp_idx(xp, C::XRW, c >> 4) + (c & 15)) | (e << 16);
    }
  }
  const bool exact = a.KW % SW == 0 && a.KH % SH == 0;
  f32x4 pg[NG], px_[NX];  // the next stage's G / X operands in flight
  // stage u = (image n, row block iy, column block ix), decoded incrementally
  struct Pos { int n, iy, ix; };
  auto pos_of = [&](long u) {
    Pos p;
    p.n = (int)(u / ((long)uy * ux));
    const int rem = (int)(u - (long)p.n * uy * ux);
    p.iy = rem / ux; p.ix = rem - p.iy * ux;
    return p;
  };
  auto next = [&](Pos p) {
    if (++p.ix == ux) { p.ix = 0; if (++p.iy == uy) { p.iy = 0; ++p.n; } }
    return p;
  };
  auto emask_of = [&](Pos p) {
    const int py0 = p.iy * SH, px0 = p.ix * SW;
    return (py0 == 0) | ((py0 + SH >= a.KH) << 1) | ((px0 == 0) << 2) | ((px0 + SW >= a.KW) << 3) |
           (1 << 5);
  };
  // item it's byte offset in its operand image (0x7fffffff: zeros)
  auto item_off = [&](Pos p, int it, bool isg, int base) {
    const int q = tid + it * C::NTHR;
    const int py0 = p.iy * SH, px0 = p.ix * SW;
    bool ok = !((ilde[it] >> 16) & emask_of(p));
    if (!exact && q < C::NQ) {  // sides that are not whole stage blocks: per-item bounds
      if (isg) {
        const int pxl = q / (C::COUT / 4);
        ok = ok && py0 + (pxl >> SWL) < a.KH && px0 + (pxl & (SW - 1)) < a.KW;
      } else {
        const int xp = (q - C::GQ) / (C::CIB / 4), yy = xp / XW, xx = xp - yy * XW;
        ok = ok && py0 - 1 + yy < a.KH && px0 - 1 + xx < a.KW;
      }
    }
    return ok ? (base + ioff[it]) * 4 : 0x7fffffff;
  };
  auto load_g = [&](Pos p) {
    const long img = (long)p.n * a.KH * a.KW;
    const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.g + img * a.g_stride + a.g_off), (short)0,
        (int)((long)a.KH * a.KW * a.g_stride * 4), 0x00020000);
    const int base = (p.iy * SH * a.KW + p.ix * SW) * a.g_stride;
#pragma unroll
    for (int it = 0; it < NG; ++it)
      pg[it] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                             gr, item_off(p, it, true, base), 0, 0));
  };
  auto load_x = [&](Pos p) {
    const long img = (long)p.n * a.KH * a.KW;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.x + img * a.x_stride + a.x_off), (short)0,
        (int)((long)a.KH * a.KW * a.x_stride * 4), 0x00020000);
    const int base = (p.iy * SH * a.KW + p.ix * SW) * a.x_stride;
#pragma unroll
    for (int it = 0; it < NX; ++it)
      px_[it] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                              xr, item_off(p, NG + it, false, base), 0, 0));
  };
  auto store4 = [&](__bf16* buf, int it, const f32x4& v) {
    const int o = ilde[it] & 0xffff;
    unsigned h0, m0, l0, h1, m1, l1;
    split3x2(v[0], v[1], h0, m0, l0);
    split3x2(v[2], v[3], h1, m1, l1);
    typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
    *reinterpret_cast<u32x2_t*>(buf + o) = u32x2_t{h0, h1};
    *reinterpret_cast<u32x2_t*>(buf + o + C::PL) = u32x2_t{m0, m1};
    *reinterpret_cast<u32x2_t*>(buf + o + 2 * C::PL) = u32x2_t{l0, l1};
  };
  auto store_g = [&](__bf16* buf) {
#pragma unroll
    for (int it = 0; it < NG; ++it) store4(buf, it, pg[it]);
  };
  auto store_x = [&](__bf16* buf) {
#pragma unroll
    for (int it = 0; it < NX; ++it)
      if (tid + (NG + it) * C::NTHR < C::NQ) store4(buf, NG + it, px_[it]);
  };

  // ---- MFMA operand addresses (stage-invariant) ----------------------------------------------
  // A (G planes [px][96]): lane 4q+p of group lg supplies row 8lg + 4t + q, columns 4p..4p+3
  // of block 3wm + i, i.e. block (3wm + i) ^ (lg & 1) of the row
  const int abase = (8 * lg + (li >> 2)) * C::GRW + 4 * (li & 3);
  const int aflip = C::GRW == 64 ? wp_flip64(8 * lg + (li >> 2)) : lg & 1;  // (+4t: same flip)
  // B (X planes [xp][32]): stage pixel 8lg + j = (row pr0, column pc0 + j); tap (ky, kx), read t
  // -> X row r0 + d, d = ky*XW + kx + 4t, r0 = pr0*XW + pc0 + (li >> 2), in block wn ^ bit 3 of
  // the row.  Bit k of bmask: that flip for the k-th (ky, kx, t)
  const int pr0 = (8 * lg) >> SWL, pc0 = (8 * lg) & (SW - 1);
  const int r0 = pr0 * XW + pc0 + (li >> 2);
  const int bbase = C::GPL + r0 * C::XRW + 16 * wn + 4 * (li & 3);
  const int bsgn = (wn & 1) ? -16 : 16;
  unsigned bmask0 = 0;
  // 64-channel rows (CO = 48): the block wn ^ flip of the k-th read, two bits per read
  const int bbase64 = C::GPL + r0 * C::XRW + 4 * (li & 3);
  unsigned bm64[2] = {0u, 0u};
#pragma unroll
  for (int k = 0; k < 18; ++k) {
    const int d = (k >> 1) / 3 * XW + (k >> 1) % 3 + 4 * (k & 1);
    bmask0 |= (unsigned)(((r0 + d) >> 3) & 1) << k;
    bm64[k >> 4] |= (unsigned)(wn ^ wp_flip64(r0 + d)) << (2 * (k & 15));
  }
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;

  Pos pn = pos_of(u_beg);
  if (u_beg < u_end) {
    load_g(pn);
    load_x(pn);
    store_g(lds);
    store_x(lds);
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own plane writes done
  __syncthreads();
#pragma unroll 1
  for (long u = u_beg; u < u_end; ++u) {
    const int cb = (int)((u - u_beg) & 1);
    const __bf16* buf = lds + cb * C::BUF;
    __bf16* nbuf = lds + (cb ^ 1) * C::BUF;
    pn = next(pn);
    const bool more = u + 1 < u_end;
    if (more && !DN_WG_ABL_NOS && !DN_WG_ABL_NOLD) {  // in flight during the whole stage
      load_g(pn);
      load_x(pn);
    }
    int aoff = abase;
    unsigned bmask = bmask0, bml = bm64[0], bmh = bm64[1];
    asm volatile("" : "+v"(aoff), "+v"(bmask));  // (addresses formed here, not held across stages)
    if (C::XRW == 64) asm volatile("" : "+v"(bml), "+v"(bmh));
    bf16x8 av[3][MFW];
#pragma unroll
    for (int i = 0; i < MFW; ++i) {
      const int o = aoff + (((3 * wm + i) ^ aflip) << 4);
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        const __bf16* p = buf + pl * C::PL + o;
        av[pl][i] = tr_frag(p, p + 4 * C::GRW);
      }
    }
    // B fragments of tap t (three planes), read one tap ahead of their MFMAs: the reads of tap
    // t + 1 are in flight during tap t's 18 MFMAs instead of being waited for at the head of
    // every tap (96->96 @64 x 128^2 0.963 -> 0.934 ms, profiles/r5_wg_ab.log)
    auto read_b = [&](int t, bf16x8 (&bv)[3]) {
      const int ky = t / 3, kx = t - 3 * (t / 3), k = 2 * t, d = ky * XW + kx;
      int oa, ob;
      if (C::XRW == 64) {
        const unsigned m = k < 16 ? bml : bmh;
        oa = bbase64 + d * 64 + (int)(((m >> (2 * (k & 15))) & 3) << 4);
        ob = bbase64 + (d + 4) * 64 + (int)(((m >> (2 * ((k + 1) & 15))) & 3) << 4);
      } else {
        oa = bbase + d * C::XRW + (int)((bmask >> k) & 1) * bsgn;
        ob = bbase + (d + 4) * C::XRW + (int)((bmask >> (k + 1)) & 1) * bsgn;
      }
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) bv[pl] = tr_frag(buf + pl * C::PL + oa, buf + pl * C::PL + ob);
    };
    bf16x8 bvs[2][3];
    read_b(0, bvs[0]);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t + 1 < 9) {
        read_b(t + 1, bvs[(t + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
      }
      const int sl = t & 1;
      bf16x8 bv[3][1];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) bv[pl][0] = bvs[sl][pl];
      // the six products of a fragment, one fragment at a time (a dependent 16x16x32 chain
      // issues back-to-back, MI355X_MICROARCH.md): the five corrections chained from zero,
      // the leading product a0 b0 last on top of them, so the 32-pixel block reaches the
      // running sum through ONE round-to-nearest add (4 VALU per fragment instead of 8).  The
      // block sum is still fresh per stage: the chain's accumulator is at most the block's
      // own magnitude, as for a leading product summed from zero.
#pragma unroll
      for (int i = 0; i < MFW; ++i) {
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        f32x4 lo = mfma_bf16(av[0][i], bv[1][0], z);
        lo = mfma_bf16(av[1][i], bv[0][0], lo);
        lo = mfma_bf16(av[0][i], bv[2][0], lo);
        lo = mfma_bf16(av[1][i], bv[1][0], lo);
        lo = mfma_bf16(av[2][i], bv[0][0], lo);
        const f32x4 blk = mfma_bf16(av[0][i], bv[0][0], lo);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[t][i][0][r] = acc[t][i][0][r] + blk[r];
        asm volatile("" : "+v"(acc[t][i][0]));
      }
    }
    if (do_bias) {
#pragma unroll
      for (int i = 0; i < MFW; ++i) {
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        const f32x4 hi = mfma_bf16(av[0][i], ones, z);
        f32x4 lo = mfma_bf16(av[1][i], ones, z);
        lo = mfma_bf16(av[2][i], ones, lo);
        x6_acc_add(accb[i][0], hi, lo);
      }
    }
    if (more && !DN_WG_ABL_NOS) {  // (waits for its loads itself)
      store_g(nbuf);
      store_x(nbuf);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own plane writes done
    if (!DN_WG_ABL_NOBAR) __syncthreads();  // next buffer complete; everyone done with this one
  }

  float* slab = a.slab + (long)blockIdx.x * a.slab_stride;
  const int ci = ci0 + 16 * wn + li;
  const int cot = a.cout_total ? a.cout_total : a.Cout;
#pragma unroll
  for (int i = 0; i < MFW; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = (3 * wm + i) * 16 + 4 * lg + r;
        if (co < a.Cout && ci < a.Cin)
          slab[((long)(a.co_base + co) * a.cin_total + a.ci_base + ci) * 9 + t] = acc[t][i][0][r];
      }
  if (do_bias && li == 0) {
#pragma unroll
    for (int i = 0; i < MFW; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = (3 * wm + i) * 16 + 4 * lg + r;
        if (co < a.Cout) slab[(long)cot * a.cin_total * 9 + a.co_base + co] = accb[i][0][r];
      }
  }
}

// ------------------------------------------------------------------------------------
// The encoder's 48 -> 48 weight gradients (k_wgrad3q; arch_unet.py:201-221, enc_conv1..5):
// k_wgrad3p's plane scheme with FOUR waves.  The 3-wave form (one 16-channel input block per
// wave) left two of a CU's four SIMDs with one wave and two with two (two 192-thread workgroups),
// so the busier SIMDs set the pace with half the MFMA pipes idle (MFMA busy 0.30).  Here the
// 27 B fragments of a stage (3 input-channel blocks j x 9 taps t, p = 9 j + t) are dealt to the
// four waves 7 / 7 / 7 / 6 (p = 7 w + k), every wave multiplying each against all three output
// fragments (acc[7][3]); the bias gradient goes to wave 3, which has one fragment fewer.
//   K stage = 32 pixels (SH rows of SW), G [32 px][64] and X [XPIX][64] bf16 planes (48 channels
//   used; 128-B rows, wp_flip64), two buffers, two workgroups per CU (78 KiB each).
//   Split-pass items: 16 quad slots per pixel (4 blocks x 4 quads; block 3 is the row padding,
//   its lanes neither load nor store), G's 512 slots = items 0 and 1 of every thread, then X's.
//   A 16-lane group of a ds_write_b64 (banks mod 32 dwords) thus writes the four blocks of ONE
//   pixel row, which the row swizzle keeps on four distinct 32-B bank sets: conflict-free
//   writes (12 real quads per pixel dealt 16 lanes at a time put blocks of two pixels on the same
//   banks: 25 % of the LDS-active cycles in conflicts, profiles/r5_pmc_sq_n2n.txt).
//   B reads one fragment ahead of their MFMAs (as k_wgrad3p).
// ------------------------------------------------------------------------------------
template <int SWL>
struct Wq3Cfg {
  static constexpr int NTHR = 256, RW = 64, CIB = 48;
  static constexpr int SW = 1 << SWL, SH = 32 >> SWL, XW = SW + 2, XPIX = (SH + 2) * XW;
  static constexpr int GQ = 32 * 16, XQ = XPIX * 16, NQ = GQ + XQ;  // float4 slots
  static constexpr int NIT = (NQ + NTHR - 1) / NTHR;
  static constexpr int GPL = 32 * RW, PL = GPL + XPIX * RW, BUF = 3 * PL;  // bf16
  static constexpr int KMAX = 7;                                         // B fragments per wave
  static_assert(GQ == 2 * NTHR, "items 0 and 1 of every thread are G");
  static_assert(2 * BUF * 2 <= 81920, "two workgroups per CU");
};

template <int SWL>
__global__ __launch_bounds__(256, 2) void k_wgrad3q(WgradArgs a) {
  using C = Wq3Cfg<SWL>;
  constexpr int SW = C::SW, SH = C::SH, XW = C::XW, NIT = C::NIT, KMAX = C::KMAX;
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * C::BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lg = lane >> 4;
  const int ci0 = blockIdx.y * C::CIB;
  const int ux = (a.KW + SW - 1) / SW, uy = (a.KH + SH - 1) / SH;
  const long U = (long)a.N * uy * ux;
  const long u_beg = U * blockIdx.x / gridDim.x, u_end = U * (blockIdx.x + 1) / gridDim.x;
  const bool do_bias = a.bias && blockIdx.y == 0 && wave == 3;
  const int nk = wave == 3 ? 6 : 7;  // B fragments of this wave: p = 7 wave + k, k < nk

  f32x4 acc[KMAX][3], accb[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KMAX; ++k) acc[k][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // ---- split-pass items (as k_wgrad3p): offset in the operand image relative to the stage
  // origin; LDS index (low 16 bits) | halo-edge class (bits 16..)
  auto is_g = [&](int it) { return it < 2; };
  // (bit 21: no data -- loads zeros; bit 22: padding slot -- not stored either)
  int ioff[NIT], ilde[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int q = tid + it * C::NTHR;
    ioff[it] = 0; ilde[it] = (32 | 64) << 16;
    if (q < C::GQ) {
      const int px = q >> 4, c = 4 * (q & 15);
      ioff[it] = ((px >> SWL) * a.KW + (px & (SW - 1))) * a.g_stride + c;
      ilde[it] = (wp_idx(px, 64, c >> 4) + (c & 15)) |
                 ((c >= 48 ? 32 | 64 : (c < a.Cout ? 0 : 32)) << 16);
    } else if (q < C::NQ) {
      const int r = q - C::GQ, xp = r >> 4, c = 4 * (r & 15);
      const int yy = xp / XW, xx = xp - yy * XW;
      ioff[it] = ((yy - 1) * a.KW + xx - 1) * a.x_stride + ci0 + c;
      const int e = (yy == 0) | ((yy == SH + 1) << 1) | ((xx == 0) << 2) | ((xx == SW + 1) << 3) |
                    (c >= 48 ? 32 | 64 : ((ci0 + c < a.Cin ? 0 : 1) << 5));
      ilde[it] = (C::GPL + wp_idx(xp, 64, c >> 4) + (c & 15)) | (e << 16);
    }
  }
  const bool exact = a.KW % SW == 0 && a.KH % SH == 0;
  f32x4 pv[NIT];  // the next stage's operands in flight
  struct Pos { int n, iy, ix; };
  auto pos_of = [&](long u) {
    Pos p;
    p.n = (int)(u / ((long)uy * ux));
    const int rem = (int)(u - (long)p.n * uy * ux);
    p.iy = rem / ux; p.ix = rem - p.iy * ux;
    return p;
  };
  auto next = [&](Pos p) {
    if (++p.ix == ux) { p.ix = 0; if (++p.iy == uy) { p.iy = 0; ++p.n; } }
    return p;
  };
  auto load_all = [&](Pos p) {
    const long img = (long)p.n * a.KH * a.KW;
    const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.g + img * a.g_stride + a.g_off), (short)0,
        (int)((long)a.KH * a.KW * a.g_stride * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.x + img * a.x_stride + a.x_off), (short)0,
        (int)((long)a.KH * a.KW * a.x_stride * 4), 0x00020000);
    const int py0 = p.iy * SH, px0 = p.ix * SW;
    const int em = (py0 == 0) | ((py0 + SH >= a.KH) << 1) | ((px0 == 0) << 2) |
                   ((px0 + SW >= a.KW) << 3) | (1 << 5);
    const int gbase = (py0 * a.KW + px0) * a.g_stride, xbase = (py0 * a.KW + px0) * a.x_stride;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int q = tid + it * C::NTHR;
      bool ok = !((ilde[it] >> 16) & em);
      if (is_g(it)) {
        if (!exact) {
          const int pxl = q >> 4;
          ok = ok && py0 + (pxl >> SWL) < a.KH && px0 + (pxl & (SW - 1)) < a.KW;
        }
        pv[it] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                               gr, ok ? (gbase + ioff[it]) * 4 : 0x7fffffff, 0, 0));
      } else {
        if (!exact && q < C::NQ) {
          const int xp = (q - C::GQ) >> 4, yy = xp / XW, xx = xp - yy * XW;
          ok = ok && py0 - 1 + yy < a.KH && px0 - 1 + xx < a.KW;
        }
        pv[it] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                               xr, ok ? (xbase + ioff[it]) * 4 : 0x7fffffff, 0, 0));
      }
    }
  };
  auto store_all = [&](__bf16* buf) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      if (tid + it * C::NTHR >= C::NQ || ((ilde[it] >> 22) & 1)) continue;  // (padding slots)
      const int o = ilde[it] & 0xffff;
      unsigned h0, m0, l0, h1, m1, l1;
      split3x2(pv[it][0], pv[it][1], h0, m0, l0);
      split3x2(pv[it][2], pv[it][3], h1, m1, l1);
      typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
      *reinterpret_cast<u32x2_t*>(buf + o) = u32x2_t{h0, h1};
      *reinterpret_cast<u32x2_t*>(buf + o + C::PL) = u32x2_t{m0, m1};
      *reinterpret_cast<u32x2_t*>(buf + o + 2 * C::PL) = u32x2_t{l0, l1};
    }
  };

  // ---- MFMA operand addresses -----------------------------------------------------------
  // A (G planes): lane 4q+p of group lg: row 8lg + 4t + q, columns 4p .. of block i ^ flip
  const int abase = (8 * lg + (li >> 2)) * 64 + 4 * (li & 3);
  const int aflip = wp_flip64(8 * lg + (li >> 2));  // (+4t leaves bits 1 and 3 alone)
  // B (X planes): stage pixel 8lg + jj = (row pr0, column pc0 + jj); fragment (j, t): X row
  // r0 + d (+4 for the second read), d = ky XW + kx, block j ^ flip(row); two bits per read
  const int pr0 = (8 * lg) >> SWL, pc0 = (8 * lg) & (SW - 1);
  const int r0 = pr0 * XW + pc0 + (li >> 2);
  const int bbase = C::GPL + r0 * 64 + 4 * (li & 3);
  unsigned bm0 = 0;
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    const int p = 7 * wave + k, j = p / 9, t = p - 9 * j;
    const int d = (t / 3) * XW + t % 3;
    bm0 |= (unsigned)(((j ^ wp_flip64(r0 + d)) & 3) | (((j ^ wp_flip64(r0 + d + 4)) & 3) << 2)) << (4 * k);
  }
  bf16x8 ones;
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) ones[jj] = (__bf16)1.0f;

  Pos pn = pos_of(u_beg);
  if (u_beg < u_end) {
    load_all(pn);
    store_all(lds);
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own plane writes done
  __syncthreads();
#pragma unroll 1
  for (long u = u_beg; u < u_end; ++u) {
    const int cb = (int)((u - u_beg) & 1);
    const __bf16* buf = lds + cb * C::BUF;
    __bf16* nbuf = lds + (cb ^ 1) * C::BUF;
    pn = next(pn);
    const bool more = u + 1 < u_end;
    if (more) load_all(pn);  // in flight during the whole stage
    int aoff = abase;
    unsigned bm = bm0;
    asm volatile("" : "+v"(aoff), "+v"(bm));
    bf16x8 av[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int o = aoff + ((i ^ aflip) << 4);
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        const __bf16* pp = buf + pl * C::PL + o;
        av[pl][i] = tr_frag(pp, pp + 4 * 64);
      }
    }
    auto read_b = [&](int k, bf16x8 (&bv)[3]) {
      const int p = 7 * wave + k, j = p / 9, t = p - 9 * j;  // (uniform)
      const int d = (t / 3) * XW + t % 3;
      const int oa = bbase + d * 64 + (int)(((bm >> (4 * k)) & 3) << 4);
      const int ob = bbase + (d + 4) * 64 + (int)(((bm >> (4 * k + 2)) & 3) << 4);
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) bv[pl] = tr_frag(buf + pl * C::PL + oa, buf + pl * C::PL + ob);
    };
    bf16x8 bvs[2][3];
    read_b(0, bvs[0]);
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k + 1 < KMAX && k + 1 < nk) read_b(k + 1, bvs[(k + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
      if (k < nk) {
        const bf16x8(&bv)[3] = bvs[k & 1];
#pragma unroll
        for (int i = 0; i < 3; ++i) {  // k_wgrad3p's fold: five corrections, then a0 b0, one add
          const f32x4 z = {0.f, 0.f, 0.f, 0.f};
          f32x4 lo = mfma_bf16(av[0][i], bv[1], z);
          lo = mfma_bf16(av[1][i], bv[0], lo);
          lo = mfma_bf16(av[0][i], bv[2], lo);
          lo = mfma_bf16(av[1][i], bv[1], lo);
          lo = mfma_bf16(av[2][i], bv[0], lo);
          const f32x4 blk = mfma_bf16(av[0][i], bv[0], lo);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[k][i][r] = acc[k][i][r] + blk[r];
          asm volatile("" : "+v"(acc[k][i]));
        }
      }
    }
    if (do_bias) {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        const f32x4 hi = mfma_bf16(av[0][i], ones, z);
        f32x4 lo = mfma_bf16(av[1][i], ones, z);
        lo = mfma_bf16(av[2][i], ones, lo);
        x6_acc_add(accb[i], hi, lo);
      }
    }
    if (more) store_all(nbuf);  // (waits for its loads itself)
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own plane writes done
    __syncthreads();                     // next buffer complete; everyone done with this one
  }

  float* slab = a.slab + (long)blockIdx.x * a.slab_stride;
  const int cot = a.cout_total ? a.cout_total : a.Cout;
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    if (k >= nk) continue;
    const int p = 7 * wave + k, j = p / 9, t = p - 9 * j;
    const int ci = ci0 + 16 * j + li;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = i * 16 + 4 * lg + r;
        if (co < a.Cout && ci < a.Cin)
          slab[((long)(a.co_base + co) * a.cin_total + a.ci_base + ci) * 9 + t] = acc[k][i][r];
      }
  }
  if (do_bias && li == 0) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = i * 16 + 4 * lg + r;
        if (co < a.Cout) slab[(long)cot * a.cin_total * 9 + a.co_base + co] = accb[i][r];
      }
  }
}

// 96 output channels (or 96-channel blocks, a.zc == 96), 32 input channels per workgroup,
// 16-byte aligned NHWC views, images under 2 GiB per operand (32-bit buffer offsets)
bool wgrad3p_ok(const WgradArgs& a) {
  if ((a.zc ? a.zc != 96 : (a.Cout != 96 && a.Cout != 48)) || a.Cin < 32 || a.KW < 8) return false;
  if ((a.g_stride | a.g_off | a.x_stride | a.x_off) & 3) return false;
  if (a.x_off + ((a.Cin + 3) & ~3) > a.x_stride) return false;
  return (long)a.KH * a.KW * a.g_stride * 4 < 0x7fffffffL &&
         (long)a.KH * a.KW * a.x_stride * 4 < 0x7fffffffL;
}

// Stage rows of at most 16 pixels (2 rows of 16: 72 X pixels per stage instead of 102 for one
// row of 32) and the late G split measured best (profiles/r4_wgp2_ab.log).  The encoder's
// 48 -> 48 layers take the 4-wave k_wgrad3q at 128^2 (0.35-0.36 -> 0.31-0.33 ms); below that
// the 3-wave k_wgrad3p<.., 48> measured faster (@64^2 0.120-0.127 vs 0.131-0.133 ms,
// profiles/r5_wg_ab.log; @32^2 0.050 vs 0.065 ms in-step): with 7 fragments per wave the
// shorter stages no longer hide the next stage's loads.
hipError_t launch_wgrad3p(const WgradArgs& a, int splits, hipStream_t s, int nz) {
  if (!wgrad3p_ok(a)) return hipErrorInvalidValue;
  if (!a.zc && a.Cout == 48) {
    const dim3 grid(splits, (a.Cin + 47) / 48, nz);
    if (a.KW >= 128) {
      prof_kernel("k_wgrad3q<4>");
      hipLaunchKernelGGL(k_wgrad3q<4>, grid, dim3(256), 0, s, a);
    } else if (a.KW >= 16) {
      prof_kernel("k_wgrad3p<4,48>");
      hipLaunchKernelGGL((k_wgrad3p<4, 48>), grid, dim3(192), 0, s, a);
    } else {
      prof_kernel("k_wgrad3p<3,48>");
      hipLaunchKernelGGL((k_wgrad3p<3, 48>), grid, dim3(192), 0, s, a);
    }
    return hipGetLastError();
  }
  const dim3 grid(splits, (a.Cin + 31) / 32, nz), block(256);
  if (a.KW >= 16) {
    prof_kernel("k_wgrad3p<4,96>");
    hipLaunchKernelGGL((k_wgrad3p<4>), grid, block, 0, s, a);
  } else {
    prof_kernel("k_wgrad3p<3,96>");
    hipLaunchKernelGGL((k_wgrad3p<3>), grid, block, 0, s, a);
  }
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// 1x1 weight gradient of the 96 x 96 head layers (nin_a, nin_b: arch_unet.py:186-189) and of
// the 96-channel deconvs (UP2: UpsampleCat's ConvTranspose2d(2, 2), arch_unet.py:57) in the
// same arithmetic (k_wgrad1p; k_wgrad1 does them on the fp32 matrix cores).  UP2: blockIdx.z =
// parity (a, b); the gradient operand of low-res pixel (y, x) is g at (2y + a, 2x + b), so its
// rows are gathered per pixel (64-bit addresses, plain loads) while x stays a flat range.  K = pixels of the
// flattened N x H x W range (a 1x1 conv has no halo), 32 per stage: G [32 px][96 co] and X
// [32 px][96 ci] split once into three bf16 planes of the stage buffer, the next stage's fp32
// operands in registers meanwhile, one barrier per stage.  Wave (wm, wn): output channels
// 48wm .. +47 x input channels 48wn .. +47 (3 x 3 fragments, six products each, the fold of
// k_wgrad3p); both operands are read with ds_read_b64_tr_b16 in the same pattern (pixel-major
// rows, 16-channel blocks flipped by bit 3 of the row).  The bias gradient is G against a ones
// fragment in the wn = 0 waves.  Each workgroup writes its partial [W | b] to a slab row.
// ------------------------------------------------------------------------------------
struct Wp1Cfg {
  static constexpr int C = 96, NTHR = 256, PX = 32;
  static constexpr int GQ = PX * C / 4, NQ = 2 * GQ, NIT = NQ / NTHR;  // float4 items
  static constexpr int GPL = PX * C, PL = 2 * GPL, BUF = 3 * PL;     // bf16
  static_assert(NQ % NTHR == 0 && GQ % NTHR == 0, "whole items per thread");
  static_assert(2 * BUF * 2 <= 81920, "two workgroups per CU");
};

#ifndef DN_WG1_PD
#define DN_WG1_PD 2
#endif
// WG1_PD = 2: stage u + 2's loads are issued at the head of stage u into a second register set
// (pv2), stage u + 1's operands (pv) are split into the other LDS buffer at the end of stage u,
// then pv = pv2.  That copy waits for the u + 2 loads inside stage u, so load latency is still
// hidden behind ONE stage only; what the form buys is that the split / plane writes of stage u + 1
// no longer wait for their own loads (issued a whole stage earlier).  Measured: the deconv weight
// gradients 0.346-0.348 -> 0.298-0.305 ms/step, the 1x1 ones unchanged
// (profiles/r5_wgrad1_pd_ab.log).
constexpr int WG1_PD = DN_WG1_PD;
// GNB > 0 (nin_b's weight gradient, GNB = nin_c's outputs): the gradient operand is recomputed
// from the nin_b activation (a.g) and dL/dy as g = leaky'(nb) (Wc^T dy) -- k_head_bwd_x6's
// fmaf order, the same values -- so the data-gradient pass does not store g_nb (384 B per pixel).
// With a.hd_slab_c it also forms nin_c's weight gradient dWc[o][c] = sum dy[o] nb[c] and
// dbc[o] = sum dy[o] from the same registers (per-thread sums of its three channel quads, then
// a fixed-order sum over the workgroup's threads): the separate k_wgrad_thin pass and its
// 388 B per pixel of reads go away.
template <bool UP2, int GNB = 0>
__global__ __launch_bounds__(256, 2) void k_wgrad1p(WgradArgs a, long npx) {
  using C = Wp1Cfg;
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * C::BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 15, lg = lane >> 4;
  // UP2: one flat grid of 4 x splits blocks; block b = (split, parity) with parity (b >> 3) & 3,
  // so the four parity blocks of a split are dispatched within 32 blocks of each other onto the
  // same XCD (b % 8) and three of the four reads of its low-res input rows hit that XCD's L2
  // (parity-major z launches read them at four different times: 1.27x the operand bytes)
  const int nsp = UP2 ? (int)gridDim.x / 4 : (int)gridDim.x;
  const int bsp = UP2 ? (int)((blockIdx.x & 7) | ((blockIdx.x >> 5) << 3)) : (int)blockIdx.x;
  const int bz = UP2 ? (int)((blockIdx.x >> 3) & 3) : 0;
  const long U = (npx + C::PX - 1) / C::PX;
  const long u_beg = U * bsp / nsp, u_end = U * (bsp + 1) / nsp;
  const bool do_bias = wn == 0;

  f32x4 acc[3][3], accb[3][1];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    accb[i][0] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // item it of this thread: operand (G for it < NIT/2), pixel, 4 channels; its LDS index
  constexpr int NG = C::GQ / C::NTHR;
  int ioff[C::NIT], ipx[C::NIT], ilds[C::NIT];
#pragma unroll
  for (int it = 0; it < C::NIT; ++it) {
    const int q = tid + it * C::NTHR, r = it < NG ? q : q - C::GQ;
    const int px = r / (C::C / 4), c = 4 * (r % (C::C / 4));
    ipx[it] = px;
    ioff[it] = px * (it < NG ? a.g_stride : a.x_stride) + c;
    ilds[it] = (it < NG ? 0 : C::GPL) + wp_idx(px, C::C, c >> 4) + (c & 15);
  }
  f32x4 pv[C::NIT], pv2[WG1_PD == 2 ? C::NIT : 1];
  constexpr int GO = GNB > 0 ? GNB : 1;
  float dv[NG][GO], dv2[WG1_PD == 2 ? NG : 1][GO];  // (GNB) dy of the G items' pixels
  f32x4 wcr[NG][GO];                                   // (GNB) Wc[o][c .. c + 3] of the G items
  // (the nin_c fold for one nin_c output only -- the N2N head of C = 1: more outputs' partial
  // sums do not fit beside the operands, and k_wgrad_thin keeps them)
  constexpr bool FOLDC = GNB == 1;
  f32x4 gwc[NG][GO];                                   // (FOLDC) dWc partial sums of the G items
  float gbc[GO];                                       // (FOLDC) dbc partial sums (quad 0 items)
#pragma unroll
  for (int o = 0; o < GO; ++o) {
    gbc[o] = 0.f;
#pragma unroll
    for (int it = 0; it < NG; ++it) gwc[it][o] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if constexpr (GNB > 0) {
#pragma unroll
    for (int it = 0; it < NG; ++it)
#pragma unroll
      for (int o = 0; o < GNB; ++o)
        wcr[it][o] = *reinterpret_cast<const f32x4*>(a.hd_wc + o * 96 + (ioff[it] - ipx[it] * a.g_stride));
  }
  const int pa = bz >> 1, pb = bz & 1;
  auto load = [&](long u, f32x4* dst, float (*ddst)[GO]) {
    const long p0 = u * C::PX;
    const int np = npx - p0 < C::PX ? (int)(npx - p0) : C::PX;
    if constexpr (GNB > 0) {
      const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(a.hd_dy + p0 * a.hd_dy_stride), (short)0, np * a.hd_dy_stride * 4, 0x00020000);
#pragma unroll
      for (int it = 0; it < NG; ++it)
#pragma unroll
        for (int o = 0; o < GNB; ++o)
          ddst[it][o] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                      dr, (ipx[it] * a.hd_dy_stride + o) * 4, 0, 0));
    }
    const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.g + p0 * a.g_stride + a.g_off), (short)0, np * a.g_stride * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.x + p0 * a.x_stride + a.x_off), (short)0, np * a.x_stride * 4, 0x00020000);
#pragma unroll
    for (int it = 0; it < C::NIT; ++it) {
      if (UP2 && it < NG) {  // low-res pixel p -> g pixel (2y + a, 2x + b) of its image
        const long p = p0 + ipx[it], r = p / a.KW;  // r = n KH + y
        const int xx = (int)(p - r * a.KW);
        const float* src = a.g + ((2 * r + pa) * 2 * a.KW + 2 * xx + pb) * a.g_stride + a.g_off +
                           (ioff[it] - ipx[it] * a.g_stride);
        dst[it] = ipx[it] < np ? *reinterpret_cast<const f32x4*>(src) : f32x4{0.f, 0.f, 0.f, 0.f};
        continue;
      }
      const int off = ipx[it] < np ? ioff[it] * 4 : 0x7fffffff;
      dst[it] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(it < NG ? gr : xr, off, 0, 0));
    }
  };
  auto store = [&](__bf16* buf) {
#pragma unroll
    for (int it = 0; it < C::NIT; ++it) {
      const int o = ilds[it];
      f32x4 v = pv[it];
      if constexpr (GNB > 0) {
        if (it < NG) {  // g_nb = leaky'(nb) (Wc^T dy)
          f32x4 t = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int oo = 0; oo < GNB; ++oo) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              t[e] = fmaf(wcr[it][oo][e], dv[it][oo], t[e]);
              if (FOLDC) gwc[it][oo][e] = fmaf(dv[it][oo], pv[it][e], gwc[it][oo][e]);  // dWc
            }
            if (FOLDC && ioff[it] - ipx[it] * a.g_stride == 0) gbc[oo] += dv[it][oo];  // dbc
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = pv[it][e] > 0.f ? t[e] : t[e] * 0.2f;
        }
      }
      unsigned h0, m0, l0, h1, m1, l1;
      split3x2(v[0], v[1], h0, m0, l0);
      split3x2(v[2], v[3], h1, m1, l1);
      typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
      *reinterpret_cast<u32x2_t*>(buf + o) = u32x2_t{h0, h1};
      *reinterpret_cast<u32x2_t*>(buf + o + C::PL) = u32x2_t{m0, m1};
      *reinterpret_cast<u32x2_t*>(buf + o + 2 * C::PL) = u32x2_t{l0, l1};
    }
  };
  // lane 4q+p of group lg: row 8lg + 4t + q, columns 4p .. 4p+3 of its block (see k_wgrad3p)
  const int abase = (8 * lg + (li >> 2)) * C::C + 4 * (li & 3);
  const int aflip = lg & 1;
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;

  if (u_beg < u_end) {
    load(u_beg, pv, dv);
    store(lds);
  }
  if (WG1_PD == 2 && u_beg + 1 < u_end) load(u_beg + 1, pv, dv);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own plane writes done
  __syncthreads();
#pragma unroll 1
  for (long u = u_beg; u < u_end; ++u) {
    const int cb = (int)((u - u_beg) & 1);
    const __bf16* buf = lds + cb * C::BUF;
    const bool more = u + 1 < u_end;
    if (u + WG1_PD < u_end) load(u + WG1_PD, WG1_PD == 2 ? pv2 : pv, WG1_PD == 2 ? dv2 : dv);  // in flight during this stage
    int aoff = abase;
    asm volatile("" : "+v"(aoff));
    bf16x8 av[3][3], bv[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int oa = aoff + (((3 * wm + i) ^ aflip) << 4);
      const int ob = C::GPL + aoff + (((3 * wn + i) ^ aflip) << 4);
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        const __bf16* pa = buf + pl * C::PL + oa;
        const __bf16* pb = buf + pl * C::PL + ob;
        av[pl][i] = tr_frag(pa, pa + 4 * C::C);
        bv[pl][i] = tr_frag(pb, pb + 4 * C::C);
      }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        // the five corrections chained from zero, the leading product last (k_wgrad3p's fold)
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        f32x4 lo = mfma_bf16(av[0][i], bv[1][j], z);
        lo = mfma_bf16(av[1][i], bv[0][j], lo);
        lo = mfma_bf16(av[0][i], bv[2][j], lo);
        lo = mfma_bf16(av[1][i], bv[1][j], lo);
        lo = mfma_bf16(av[2][i], bv[0][j], lo);
        const f32x4 blk = mfma_bf16(av[0][i], bv[0][j], lo);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = acc[i][j][r] + blk[r];
        asm volatile("" : "+v"(acc[i][j]));
      }
    if (do_bias) {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        const f32x4 hi = mfma_bf16(av[0][i], ones, z);
        f32x4 lo = mfma_bf16(av[1][i], ones, z);
        lo = mfma_bf16(av[2][i], ones, lo);
        x6_acc_add(accb[i][0], hi, lo);
      }
    }
    if (more) store(lds + (cb ^ 1) * C::BUF);  // (waits for its loads itself)
    if (WG1_PD == 2) {  // (waits for the u + 2 loads issued at this stage's head)
#pragma unroll
      for (int it = 0; it < C::NIT; ++it) pv[it] = pv2[it];
      if constexpr (GNB > 0) {
#pragma unroll
        for (int it = 0; it < NG; ++it)
#pragma unroll
          for (int o = 0; o < GNB; ++o) dv[it][o] = dv2[it][o];
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __syncthreads();  // next buffer complete; everyone done with this one
  }
  // slab row (UP2: parity z's block of gridDim.x rows, the deconv layout [ci][co])
  float* slab = a.slab + ((long)bz * nsp + bsp) * a.slab_stride;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = (3 * wm + i) * 16 + 4 * lg + r, ci = (3 * wn + j) * 16 + li;
        slab[UP2 ? ci * C::C + co : co * C::C + ci] = acc[i][j][r];
      }
  if (do_bias && li == 0) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) slab[C::C * C::C + (3 * wm + i) * 16 + 4 * lg + r] = accb[i][0][r];
  }
  if constexpr (FOLDC) {
    if (a.hd_slab_c) {
      // item it of thread t holds channel quad (t + 16 it) % 24 (q = t + 256 it, 256 = 10 x 24 +
      // 16); every thread's partials into LDS (the stage buffers are free after the loop's last
      // barrier), then output (o, c) sums the (it, t) whose quad is c / 4, it-major, t ascending
      float* red = reinterpret_cast<float*>(lds);
#pragma unroll
      for (int it = 0; it < NG; ++it)
#pragma unroll
        for (int o = 0; o < GNB; ++o)
#pragma unroll
          for (int e = 0; e < 4; ++e) red[((it * C::NTHR + tid) * GNB + o) * 4 + e] = gwc[it][o][e];
      float* redb = red + NG * C::NTHR * GNB * 4;
#pragma unroll
      for (int o = 0; o < GNB; ++o) redb[tid * GNB + o] = gbc[o];
      __syncthreads();
      float* slc = a.hd_slab_c + (long)blockIdx.x * (GNB * 96 + GNB);
      for (int oc = tid; oc < GNB * 96 + GNB; oc += C::NTHR) {
        float sum = 0.f;
        if (oc < GNB * 96) {
          const int o = oc / 96, c = oc % 96, k = c >> 2, e = c & 3;
          for (int it = 0; it < NG; ++it)  // the threads t = k - 16 it (mod 24), ascending
            for (int t = (k + 48 - 16 * it) % 24; t < C::NTHR; t += 24)
              sum += red[((it * C::NTHR + t) * GNB + o) * 4 + e];
        } else {
          const int o = oc - GNB * 96;
          for (int t = 0; t < C::NTHR; ++t) sum += redb[t * GNB + o];
        }
        slc[oc] = sum;
      }
    }
  }
}

// 96 -> 96 1x1, NHWC views with 16-byte aligned pixels (g / x stride and offset % 4 == 0)
bool wgrad1p_ok(const WgradArgs& a) {
  if (a.Cout != 96 || a.Cin != 96 || a.zc > 0) return false;
  if ((a.g_stride | a.g_off | a.x_stride | a.x_off) & 3) return false;
  return a.g_off + 96 <= a.g_stride && a.x_off + 96 <= a.x_stride &&
         32L * a.g_stride * 4 < 0x7fffffffL && 32L * a.x_stride * 4 < 0x7fffffffL;
}

// k_wgrad1p over `splits` slab rows of [W (co, ci) | b] (a.slab, a.slab_stride >= 96*96 + 96);
// up2: 4 x splits rows of [W (ci, co) | b], parity-major (a.KH x a.KW = the low-res input)
hipError_t launch_wgrad1p(const WgradArgs& a, int splits, hipStream_t s, bool up2) {
  if (!wgrad1p_ok(a) || splits < 1 || a.slab_stride < 96 * 96 + 96) return hipErrorInvalidValue;
  const long npx = (long)a.N * a.KH * a.KW;
  if (up2) {
    // (the flat grid's block -> (split, parity) map needs whole groups of 32 blocks)
    if (splits % 8) return hipErrorInvalidValue;
    prof_kernel("k_wgrad1p<true>");
    hipLaunchKernelGGL(k_wgrad1p<true>, dim3(4 * splits), dim3(256), 0, s, a, npx);
  } else if (a.head_gnb > 0) {
    if (a.head_gnb > 4 || !a.hd_dy || !a.hd_wc || a.g_stride != 96 || a.g_off ||
        (a.hd_slab_c && a.head_gnb != 1))  // (the nin_c fold: one output only)
      return hipErrorInvalidValue;
    prof_kernel("k_wgrad1p<false,gnb>");
#define DN_GNB(K) hipLaunchKernelGGL((k_wgrad1p<false, K>), dim3(splits), dim3(256), 0, s, a, npx)
    if (a.head_gnb == 1) DN_GNB(1);
    else if (a.head_gnb == 2) DN_GNB(2);
    else if (a.head_gnb == 3) DN_GNB(3);
    else DN_GNB(4);
#undef DN_GNB
  } else {
    prof_kernel("k_wgrad1p<false>");
    hipLaunchKernelGGL(k_wgrad1p<false>, dim3(splits), dim3(256), 0, s, a, npx);
  }
  return hipGetLastError();
}


}  // namespace dn
