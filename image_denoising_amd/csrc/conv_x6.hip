// fp32 3x3 convolution on the gfx950 bf16 matrix cores by three-way operand splitting
// ("bf16x6"): the training-path conv forward / data gradient at fp32 accuracy.
//
// Every fp32 operand v is split exactly into three bf16 pieces, v = v0 + v1 + v2 (each piece
// is the round-to-nearest-even bf16 of what the previous ones left; 3 x 8 significand bits
// cover fp32's 24).  A product a*b is the sum of the nine piece products a_i*b_j of weight
// 2^-8(i+j); the six with i+j <= 2 are kept (a0b0, a0b1, a1b0, a0b2, a1b1, a2b0), the dropped
// three are below 2^-23 |ab|, i.e. one fp32 rounding.  Each piece product is exact in the
// MFMA's fp32 accumulator, so the result has the error of an fp32 dot product (measured
// against fp64: the same rms error as the fp32 MFMA path).  Six
// v_mfma_f32_16x16x32_bf16 (16 cycles each) replace eight v_mfma_f32_16x16x4_f32 (32 cycles)
// per 16x16x32 block: a 2.67x higher matrix-core ceiling for the same fp32-accurate result.
//
//   Workgroup = 4 waves, tile = 4*MT rows x 16 pixels x 16*NT output channels; wave w owns
//   rows [w*MT, w*MT+MT).  K is staged 32 input channels (one MFMA K) at a time: the x tile
//   (with halo) is split as it is staged (fp32 registers -> three bf16 planes in LDS, once
//   per chunk), the pre-split weights arrive one tap per stage by LDS DMA, double
//   buffered, one barrier per stage.  LDS rows are 32 bf16 (64 B) with the 16-B quad index
//   XOR-swizzled by (row >> 1) & 3, which makes the per-lane ds_read_b128 operand reads
//   conflict-free for every tap offset.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "conv_epi.h"
#include "x6_core.h"

namespace dn {

// profiling label of a template instantiation ("k_c3x6p<6,0>"; -1 = parameter absent)
static std::string x6_kname(const char* k, int p0, int p1, int p2) {
  std::string n = std::string(k) + "<" + std::to_string(p0);
  for (int v : {p1, p2})
    if (v >= 0) n += "," + std::to_string(v);
  return n + ">";
}
// the same with one more template argument spelled out: x6_kmore(x6_kname(...), "false")
static std::string x6_kmore(std::string n, const char* last) {
  n.back() = ',';
  return n.append(last).append(">");
}

#ifndef DN_X6_GDMA
#define DN_X6_GDMA 0  // A/B switch: 1 = the 3x3 kernels' weight DMA as global_load_lds
#endif

template <int NT, int MT>
struct XCfg {
  static constexpr int TW = 16, TH = 4 * MT, IH = TH + 2, IW = TW + 2, KC = 32, NP = 16 * NT;
  static constexpr int XPIX = IH * IW;
  static constexpr int XPL = XPIX * KC;        // bf16 per plane of the x tile
  static constexpr int WPL = NP * KC;          // bf16 per plane of a weight stage
  static constexpr int WST = 3 * WPL;          // bf16 per stage (one tap, three planes)
  static constexpr int WSTP = x6_wst(NP);      // stage stride in the packed image
  static_assert(WST % 512 == 0, "weight stages are copied in whole KiBs");
  static constexpr int XQ = XPIX * (KC / 4);   // float4 items of the x tile
  static constexpr int XITEMS = (XQ + 255) / 256;
  static constexpr int PS = NP + 4;            // epilogue staging pixel stride (floats)
  static constexpr int LBYTES_MAIN = 2 * 3 * XPL + 2 * 2 * WST;
  static constexpr int LBYTES = LBYTES_MAIN > 4 * 4 * 16 * PS ? LBYTES_MAIN : 4 * 4 * 16 * PS;
  // resident workgroups per CU (LDS-limited; the register budget allows 2 waves per SIMD)
  static constexpr int OCC = (163840 / LBYTES) < 2 ? (163840 / LBYTES) : 2;
};

template <int NT, int MT>
__global__ __launch_bounds__(256, 2) void k_c3x6(FwdArgs a) {
  using C = XCfg<NT, MT>;
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[C::LBYTES];
  __bf16* lx = reinterpret_cast<__bf16*>(lds_raw);
  __bf16* lw0 = lx + 3 * C::XPL;
  __bf16* lw1 = lw0 + C::WST;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  const int li = lane & 15, lg = lane >> 4;
  const int tiles_x = (a.OW + C::TW - 1) / C::TW;
  int bxr, byr;  // XCD-aware tile order (conv_epi.h xcd_tile)
  xcd_tile(bxr, byr);
  const int ty0 = (bxr / tiles_x) * C::TH;
  const int tx0 = (bxr % tiles_x) * C::TW;
  const int n = byr;
  const int iy0 = ty0 - 1, ix0 = tx0 - 1;
  const float* inb = a.in + (long)n * a.IHt * a.IWt * a.in_stride + a.in_off;
  const __bf16* wimg = reinterpret_cast<const __bf16*>(a.wp) + (long)blockIdx.z * a.wp_z;
  const bool vec = ((a.in_stride | a.in_off) & 3) == 0;
  const int nch = (a.K + C::KC - 1) / C::KC;
  const int nst = 9 * nch;

  f32x4 acc[MT][NT], accl[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < NT; ++q) acc[m][q] = accl[m][q] = f32x4{0.f, 0.f, 0.f, 0.f};

  float4 xr[C::XITEMS];
  auto load_x = [&](int k0) {
#pragma unroll
    for (int it = 0; it < C::XITEMS; ++it) {
      const int e = tid + it * 256;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < C::XQ) {
        const int q = e % (C::KC / 4), pix = e / (C::KC / 4);
        const int iy = pix / C::IW, ix = pix - iy * C::IW;
        const int gy = iy0 + iy, gx = ix0 + ix, k = k0 + 4 * q;
        if (gy >= 0 && gy < a.IHt && gx >= 0 && gx < a.IWt && k < a.K) {
          const float* p = inb + ((long)gy * a.IWt + gx) * a.in_stride + k;
          if (vec && k + 4 <= a.K) {
            v = *reinterpret_cast<const float4*>(p);
          } else {
            v.x = p[0];
            if (k + 1 < a.K) v.y = p[1];
            if (k + 2 < a.K) v.z = p[2];
            if (k + 3 < a.K) v.w = p[3];
          }
        }
      }
      xr[it] = v;
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int it = 0; it < C::XITEMS; ++it) {
      const int e = tid + it * 256;
      if (e < C::XQ) {
        const int q = e % (C::KC / 4), pix = e / (C::KC / 4);
        const float f[4] = {xr[it].x, xr[it].y, xr[it].z, xr[it].w};
        bf16x4 h, m, l;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          __bf16 hj, mj, lj;
          split3(f[j], hj, mj, lj);
          h[j] = hj; m[j] = mj; l[j] = lj;
        }
        const int off = pix * C::KC + x6_swz(pix, q >> 1) * 8 + (q & 1) * 4;
        *reinterpret_cast<bf16x4*>(lx + off) = h;
        *reinterpret_cast<bf16x4*>(lx + C::XPL + off) = m;
        *reinterpret_cast<bf16x4*>(lx + 2 * C::XPL + off) = l;
      }
    }
  };
  // (buffer loads to LDS, not global_load_lds: see k_c3x6p's load_w)
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__bf16*>(wimg), (short)0, nst * C::WSTP * 2, 0x00020000);
  auto load_w = [&](int st, __bf16* dst) {  // stage st = chunk * 9 + tap, whole KiB pieces
#pragma unroll
    for (int p = wave; p < C::WST / 512; p += 4) {
#if DN_X6_GDMA
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(wimg + (long)st * C::WSTP + p * 512 + lane * 8),
          (__attribute__((address_space(3))) void*)(dst + p * 512), 16, 0, 0);
#else
      buf_lds16(wrs, dst + p * 512, (st * C::WSTP + p * 512 + lane * 8) * 2);
#endif
    }
  };

  load_w(0, lw0);
  load_x(0);
  store_x();
  __syncthreads();

  for (int st = 0; st < nst; ++st) {
    const int c = st / 9, t = st - 9 * c, ky = t / 3, kx = t - 3 * ky;
    const __bf16* lw = (st & 1) ? lw1 : lw0;
    // the buffer of stage st+1 was last read in stage st-1, which every wave has left
    if (st + 1 < nst) load_w(st + 1, (st & 1) ? lw0 : lw1);
    if (t == 0 && c + 1 < nch) load_x((c + 1) * C::KC);
    bf16x8 av[3][MT], bv[3][NT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int pix = (wave * MT + m + ky) * C::IW + li + kx;
      const int off = pix * C::KC + x6_swz(pix, lg) * 8;
#pragma unroll
      for (int p = 0; p < 3; ++p) av[p][m] = *reinterpret_cast<const bf16x8*>(lx + p * C::XPL + off);
    }
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      const int row = q * 16 + li;
      const int off = row * C::KC + x6_swz(row, lg) * 8;
#pragma unroll
      for (int p = 0; p < 3; ++p) bv[p][q] = *reinterpret_cast<const bf16x8*>(lw + p * C::WPL + off);
    }
    x6_block_c<MT, NT, x6_qgc(MT, NT)>(acc, accl, av, bv);
    if (t == 8 && c + 1 < nch) {  // every wave is done with this chunk's x tile
      __syncthreads();
      store_x();
    }
    __syncthreads();  // next stage's weights landed (vmcnt(0)); next x tile written
  }
  x6_fold(acc, accl);
  fwd_epilogue<NT, MT, C::PS, false>(a, acc, reinterpret_cast<float*>(lds_raw), ty0, tx0, n);
}

// ------------------------------------------------------------------------------------
// Pipelined variant for large grids: 8 waves (2 per SIMD) share one 16 x 16 x 16*NT tile
// (wave w: rows 2w, 2w+1), one workgroup per CU.  The weight stages stream through an
// S-deep LDS ring by 1 KiB DMAs (buffer_load_dwordx4 ... lds, PPW per wave per stage),
// so a stage's weights are requested S-2 stages (~2 us) before they are read; the wait before
// each stage's barrier counts only this wave's own DMAs (s_waitcnt vmcnt(N)), not the next
// chunk's x tile, which is loaded into registers when a chunk starts and split into the
// three LDS planes when it ends.  Requires float4-aligned input views with K % 4 == 0.
// ------------------------------------------------------------------------------------
template <int NT, int WV = 8>
struct PCfg {
  // WV = 8: two waves per SIMD, MT = 2 rows each.  WV = 4 (one wave per SIMD, 4 rows, 392-462
  // registers with the accumulators in AGPRs, no spills) measured 8-15 % slower on the 96-channel
  // shapes (profiles/r3_ab_w4_not_kept.log): not launched
  static constexpr int WAVES = WV, MT = 16 / WV, S = 4;
  static constexpr int TW = 16, TH = WAVES * MT, IH = TH + 2, IW = TW + 2, KC = 32, NP = 16 * NT;
  static constexpr int XPIX = IH * IW;
  static constexpr int XPL = XPIX * KC;
  static constexpr int WPL = NP * KC;
  static constexpr int WSTP = x6_wst(NP);              // bf16 per stage (padded)
  static constexpr int PPW = WSTP * 2 / (WAVES * 1024);  // 1 KiB DMAs per wave per stage
  static_assert(PPW * WAVES * 1024 == WSTP * 2, "stage = whole DMA rounds");
  static constexpr int XQ = XPIX * (KC / 4);
  static constexpr int XITEMS = (XQ + WAVES * 64 - 1) / (WAVES * 64);
  static constexpr int PS = NP + 4;
  static constexpr int LBYTES_MAIN = 2 * 3 * XPL + 2 * S * WSTP;
  static constexpr int LEPI = 4 * WAVES * 16 * PS;
  static constexpr int LBYTES = LBYTES_MAIN > LEPI ? LBYTES_MAIN : LEPI;
  static_assert(LBYTES <= 163840, "one workgroup per CU");
};

#define X6_WAITCNT_VM(n) \
  __builtin_amdgcn_s_waitcnt(((n) & 0xF) | (((n) >> 4) << 14) | (0x7 << 4) | (0xF << 8))
// the same with lgkmcnt(0): at a stage's end every LDS read has been consumed, so the wait is
// free, and it clears the compiler's view of the stage's weight DMAs as pending LGKM events --
// otherwise the next stage's first MFMA waits lgkmcnt(0) for all of its operand reads instead
// of the counted lgkmcnt(N) for the first few (the waitcnt pass treats global_load_lds as an
// out-of-order LGKM event)
#define X6_WAITCNT_VM_LGKM0(n) \
  __builtin_amdgcn_s_waitcnt(((n) & 0xF) | (((n) >> 4) << 14) | (0x7 << 4))

__device__ __forceinline__ void x6_barrier() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);  // no compiler motion of LDS accesses across it
  __builtin_amdgcn_s_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// SEL: a.sel_rd's N2N pair pixels only (launch_fwd_x6_sel): the 16 selected pixels (2 per cell)
// of one row of 2x2 cells form ONE M fragment (the lane of fragment row 2j + s reads its A
// operand at the pixel pair[rd][s] of cell j): half the MFMAs, the same staging, per-pixel
// arithmetic unchanged (bit-identical outputs).  Wave w computes cell rows 2(w&3), 2(w&3)+1 of
// the tile for output channels [NT/2 * 16 (w>>2), +NT/2 * 16): two M fragments x NT/2 B
// fragments per stage (6 + 9 operand reads) instead of one cell row x NT (3 + 18) -- the B
// reads had made the LDS array, not the matrix core, the limit.  The epilogue writes row
// ty0/2 + 2(w&3) + m of the [OH/2][OW] pair image, channels of the wave's half.
#ifndef DN_X6P_STAGED
#define DN_X6P_STAGED 1  // A/B switch: the pipelined first fragment group of a k_c3x6p stage
#endif
#ifndef DN_X6P_LOOK
#define DN_X6P_LOOK 2  // B fragment groups read ahead of their MFMAs in k_c3x6p
#endif
// A/B switches of the k_c3x6p stage schedule (full chunks): DMAI = the next weight stage's DMA
// pieces issued between the first fragment groups instead of after the last MFMA; PIN = each
// group's round-to-nearest hi adds pinned behind its MFMAs instead of sunk to the stage end
#ifndef DN_X6P_DMAI
#define DN_X6P_DMAI 1
#endif
#ifndef DN_X6P_PIN
#define DN_X6P_PIN 1
#endif
#ifndef DN_X6P_ABL_NODMA
#define DN_X6P_ABL_NODMA 0  // diagnostic ablation: no weight DMA in the stage loop (wrong results)
#endif
// DN_X6_STAMPS=1 (diagnostic builds only): s_memtime stamps of waves 0 and 4 (one per SIMD pair
// half) of the first 64 tiles of image 0 -- kernel start, per stage after its opening barrier /
// after its last MFMA / before its closing barrier, end of the main loop, end of the epilogue --
// read back with dn_debug_x6_stamps (tools/x6_stamps.py).  Stamps sit where no LDS read is in
// flight, so the counted lgkmcnt waits of the stage are unchanged.
#ifndef DN_X6_STAMPS
#define DN_X6_STAMPS 0
#endif
// A/B switch: static priority 1 for waves 4-7 (the second-dispatched half, the arbitration
// loser of every stage) before the main loop (MI355X_MICROARCH.md, two waves per SIMD, item 4)
#if DN_X6_STAMPS
constexpr int X6_STAMP_SLOTS = 128;
__device__ unsigned long long g_x6_stamps[64 * 2 * X6_STAMP_SLOTS];
#define X6_STAMP(slot)                                                                         \
  do {                                                                                         \
    if (blockIdx.y == 0 && blockIdx.z == 0 && blockIdx.x < 64 && (wave & 3) == 0 &&            \
        (slot) < X6_STAMP_SLOTS) {                                                             \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                              \
      if (lane == 0) g_x6_stamps[(blockIdx.x * 2 + (wave >> 2)) * X6_STAMP_SLOTS + (slot)] = t_; \
    }                                                                                          \
  } while (0)
#else
#define X6_STAMP(slot) \
  do {                 \
  } while (0)
#endif

template <int NT, int TAIL, bool SEL = false, int WV = 8>
__global__ __launch_bounds__(64 * WV, 1) void k_c3x6p(FwdArgs a) {
  using C = PCfg<NT, WV>;
  static_assert(!SEL || (TAIL == 0 && NT % 2 == 0 && C::MT == 2 && C::WAVES == 8),
                "selected pixels: full 32-channel chunks, 8 waves of two cell rows x NT/2");
  constexpr int MTC = C::MT;               // M fragments computed per wave
  constexpr int NTW = SEL ? NT / 2 : NT;   // B fragments per wave
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[C::LBYTES];
  __bf16* lx = reinterpret_cast<__bf16*>(lds_raw);
  __bf16* ring = lx + 3 * C::XPL;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  const int li = lane & 15, lg = lane >> 4;
  const int tiles_x = (a.OW + C::TW - 1) / C::TW;
  int bxr, byr;  // XCD-aware tile order (conv_epi.h xcd_tile)
  xcd_tile(bxr, byr);
  const int ty0 = (bxr / tiles_x) * C::TH;
  const int tx0 = (bxr % tiles_x) * C::TW;
  const int n = byr;
  const int iy0 = ty0 - 1, ix0 = tx0 - 1;
  const float* inb = a.in + (long)n * a.IHt * a.IWt * a.in_stride + a.in_off;
  const __bf16* wimg = reinterpret_cast<const __bf16*>(a.wp) + (long)blockIdx.z * a.wp_z;
  const int nch = (a.K + C::KC - 1) / C::KC;
  // last chunk packed by x6_tail_mode: 2 im2col stages (mode 1) or 5 tap-pair stages (mode 2)
  constexpr int tail = TAIL;
  constexpr int tail_st = tail == 1 ? 2 : 5;
  const int nst = 9 * nch - (tail ? 9 - tail_st : 0);

  f32x4 acc[MTC][NTW], accl[MTC][NTW];
#pragma unroll
  for (int m = 0; m < MTC; ++m)
#pragma unroll
    for (int q = 0; q < NTW; ++q) acc[m][q] = accl[m][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int qoff = SEL ? (wave >> 2) * NTW : 0;  // first B fragment (16 channels) of this wave
  // SEL: x-tile pixel of this lane's row of fragment m (tile cell row 2(w&3) + m, cell
  // j = li / 2, pair member s = li % 2)
  int selpix[MTC] = {};
  if constexpr (SEL) {
#pragma unroll
    for (int m = 0; m < MTC; ++m) {
      const int lc = 2 * (wave & 3) + m;
      const int ci = ty0 / 2 + lc, cj = tx0 / 2 + (li >> 1);
      const int r = (ci < a.OH / 2 && cj < a.OW / 2)
                        ? a.sel_rd[((long)n * (a.OH / 2) + ci) * (a.OW / 2) + cj] & 7 : 0;
      constexpr unsigned kPair = 0xB721ED84u;  // train.py:151-154, 4 bits (a | b << 2) per rd
      const int k = (kPair >> (4 * r + 2 * (li & 1))) & 3;
      selpix[m] = (2 * lc + (k >> 1)) * C::IW + 2 * (li >> 1) + (k & 1);
    }
  }

  // Exactly XITEMS buffer loads per thread per chunk (items outside the tile or the image get
  // an out-of-range offset, for which the buffer unit returns zeros) and exactly PPW DMAs per
  // wave per stage (past the last stage: a harmless re-load into a retired ring slot), so the
  // vmcnt counts below are compile-time constants.
  // The resource covers only this tile's input rows [ry0, ry1) (based at row ry0), so its
  // 32-bit byte extent and offsets stay below 2^31 for any image height (launch_fwd_x6 checks
  // IH * IWt * in_stride * 4 < 2^31); 0x7fffffff is then always out of range.
  const int ry0 = iy0 > 0 ? iy0 : 0, ry1 = iy0 + C::IH < a.IHt ? iy0 + C::IH : a.IHt;
  const long row_floats = (long)a.IWt * a.in_stride;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(inb + ry0 * row_floats), (short)0,
      (int)((ry1 - ry0) * row_floats * 4), 0x00020000);
  f32x4 xr[C::XITEMS];
  auto load_x = [&](int k0) {
#pragma unroll
    for (int it = 0; it < C::XITEMS; ++it) {
      const int e = tid + it * C::WAVES * 64;
      const int q = e % (C::KC / 4), pix = e / (C::KC / 4);
      const int iy = pix / C::IW, ix = pix - iy * C::IW;
      const int gy = iy0 + iy, gx = ix0 + ix, k = k0 + 4 * q;
      const bool ok = e < C::XQ && gy >= 0 && gy < a.IHt && gx >= 0 && gx < a.IWt && k < a.K;
      const int off = ok ? (((gy - ry0) * a.IWt + gx) * a.in_stride + k) * 4 : 0x7fffffff;
      xr[it] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int it = 0; it < C::XITEMS; ++it) {
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
        *reinterpret_cast<bf16x4*>(lx + off) = h;
        *reinterpret_cast<bf16x4*>(lx + C::XPL + off) = m;
        *reinterpret_cast<bf16x4*>(lx + 2 * C::XPL + off) = l;
      }
    }
  };
  // weights of stage `src_st` into ring slot `slot`: PPW DMAs of 1 KiB per wave, as buffer loads
  // to LDS (MUBUF): the FLAT-encoded global_load_lds counts as a pending FLAT access, which makes
  // the compiler's waitcnt pass treat every later LDS-read wait as out of order (lgkmcnt(0)
  // instead of the counted wait) as long as any of those DMAs is outstanding -- i.e. always
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__bf16*>(wimg), (short)0, nst * C::WSTP * 2, 0x00020000);
  auto load_w_piece = [&](int src_st, int slot, int j) {
    if (DN_X6P_ABL_NODMA) return;  // diagnostic ablation only: stale weights
    unsigned char* dst = reinterpret_cast<unsigned char*>(ring + slot * C::WSTP);
    const int piece = wave * C::PPW + j;
    buf_lds16(wrs, dst + piece * 1024, src_st * C::WSTP * 2 + piece * 1024 + lane * 16);
  };
  auto load_w = [&](int src_st, int slot) {
    unsigned char* dst = reinterpret_cast<unsigned char*>(ring + slot * C::WSTP);
#pragma unroll
    for (int j = 0; j < C::PPW; ++j) {
      const int piece = wave * C::PPW + j;
#if DN_X6_GDMA
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(reinterpret_cast<const unsigned char*>(wimg) +
                                                          (long)src_st * C::WSTP * 2 + piece * 1024 + lane * 16),
          (__attribute__((address_space(3))) void*)(dst + piece * 1024), 16, 0, 0);
#else
      buf_lds16(wrs, dst + piece * 1024, src_st * C::WSTP * 2 + piece * 1024 + lane * 16);
#endif
    }
  };

  // prologue: weight stages 0 .. S-2 requested first (L2-resident), then the x tile of chunk 0
  // (HBM) split into LDS -- the two latencies overlap -- and chunk 1's x into registers, which
  // is not waited for (the first two stages allow its loads in flight)
#pragma unroll
  for (int j = 0; j < C::S - 1; ++j) load_w(j < nst ? j : nst - 1, j);
  load_x(0);
  store_x();
  load_x((nch > 1 ? 1 : 0) * C::KC);
  X6_WAITCNT_VM(C::XITEMS);            // own DMAs of stages 0 .. S-2 landed (older than x1)
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own x-tile stores done
  x6_barrier();

  // Stage st computes from ring slot st % S, then (after the chunk's last tap: splits the next
  // chunk's x tile into LDS and loads the one after into registers) requests stage st+S-1 into
  // slot (st-1) % S, which every wave left at the previous barrier.  The compiler's own waits
  // for the x registers then only ever cover DMAs issued a stage or more earlier.
  // MODE 0: a full 32-channel chunk tap, with the operand reads of a stage in one basic block
  // (the MFMAs then wait for them with counted lgkmcnt); MODE 3: the tail instantiations.
  X6_STAMP(0);
  auto stage = [&](auto mode_tag, int c, int t) {
    constexpr int MODE = decltype(mode_tag)::value;
    const bool more = c + 1 < nch;
    const int st = 9 * c + t;
    X6_STAMP(1 + 3 * st);
    const __bf16* lw = ring + (st % C::S) * C::WSTP;
    bf16x8 av[3][MTC], bv[3][NTW];
    // MODE 3: the last chunk's mode decided at run time (tail instantiations: one A-read path
    // with branches keeps them at <= 256 VGPRs; two peeled paths would spill)
    const int mode = MODE == 3 ? ((tail && c + 1 == nch) ? tail : 0) : MODE;
    constexpr int QG = x6_qgc(MTC, NTW), NG = NTW / QG, LOOK = NG < DN_X6P_LOOK ? NG : DN_X6P_LOOK;
    // STAGED (full chunks, carried form): the stage's first fragment group is issued as a
    // read/compute pipeline -- A plane p and B plane p of group 0 requested one step before the
    // MFMAs that use them -- so the first MFMA waits for 3 reads, not for all 6 A + 6 B reads
    // of a stage that all 8 waves issue together after the barrier (384 LDS cycles); the MFMA
    // order per accumulator is that of x6_group_c (results unchanged bit for bit)
    constexpr bool STAGED = MODE == 0 && QG == 1 && NG >= 3 && DN_X6P_STAGED;
    if constexpr (STAGED) {
    } else if (mode == 1) {
      // im2col stage t: lane group lg holds k = 8lg..8lg+7 = channels 0..3 of taps
      // 8t+2lg and 8t+2lg+1 (taps past 8 are zero), read as 8 B from quad 0 of the pixel
      const int ta = 8 * t + 2 * lg, tb = ta + 1;
      const int ca = ta < 9 ? ta : 8, cb = tb < 9 ? tb : 8;
      const int da = (ca / 3) * C::IW + ca % 3, db = (cb / 3) * C::IW + cb % 3;
      const bf16x4 z4 = {(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
#pragma unroll
      for (int m = 0; m < C::MT; ++m) {
        const int p0 = (wave * C::MT + m) * C::IW + li;
        const int pa = p0 + da, pb = p0 + db;
        const int oa = pa * C::KC + x6_swz(pa, 0) * 8, ob = pb * C::KC + x6_swz(pb, 0) * 8;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          bf16x4 va = *reinterpret_cast<const bf16x4*>(lx + p * C::XPL + oa);
          bf16x4 vb = *reinterpret_cast<const bf16x4*>(lx + p * C::XPL + ob);
          if (ta > 8) va = z4;
          if (tb > 8) vb = z4;
          av[p][m] = __builtin_shufflevector(va, vb, 0, 1, 2, 3, 4, 5, 6, 7);
        }
      }
    } else if (mode == 2) {
      // tap-pair stage t: lane groups 0,1 hold channels 0..15 of tap 2t, groups 2,3 those of
      // tap 2t+1 (zero past tap 8): quad lg & 1 of the pixel at that tap
      const int ta = 2 * t + (lg >> 1);
      const int ca = ta < 9 ? ta : 8;
      const int da = (ca / 3) * C::IW + ca % 3;
      const bf16x8 z8 = {};
#pragma unroll
      for (int m = 0; m < C::MT; ++m) {
        const int pa = (wave * C::MT + m) * C::IW + li + da;
        const int oa = pa * C::KC + x6_swz(pa, lg & 1) * 8;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(lx + p * C::XPL + oa);
          av[p][m] = ta > 8 ? z8 : v;
        }
      }
    } else if constexpr (SEL) {
      const int ky = t / 3, kx = t - 3 * ky;
#pragma unroll
      for (int m = 0; m < MTC; ++m) {
        const int pix = selpix[m] + ky * C::IW + kx;
        const int off = pix * C::KC + x6_swz(pix, lg) * 8;
#pragma unroll
        for (int p = 0; p < 3; ++p)
          av[p][m] = *reinterpret_cast<const bf16x8*>(lx + p * C::XPL + off);
      }
    } else {
      const int ky = t / 3, kx = t - 3 * ky;
#pragma unroll
      for (int m = 0; m < C::MT; ++m) {
        const int pix = (wave * C::MT + m + ky) * C::IW + li + kx;
        const int off = pix * C::KC + x6_swz(pix, lg) * 8;
#pragma unroll
        for (int p = 0; p < 3; ++p)
          av[p][m] = *reinterpret_cast<const bf16x8*>(lx + p * C::XPL + off);
      }
    }
    // B fragment groups in the order x6_group consumes them, read LOOK groups ahead of the
    // MFMAs: the reads of group g + LOOK are issued after group g's MFMAs (into its freed
    // registers), so every MFMA finds its operands in flight long enough, and the stage's
    // operands never all live at once (the kernel is at 2 waves per SIMD, 256 VGPRs)
    auto read_b = [&](int g) {
#pragma unroll
      for (int q = g * QG; q < (g + 1) * QG; ++q) {
        const int row = (qoff + q) * 16 + li;
        const int off = row * C::KC + x6_swz(row, lg) * 8;
#pragma unroll
        for (int p = 0; p < 3; ++p)
          bv[p][q] = *reinterpret_cast<const bf16x8*>(lw + p * C::WPL + off);
      }
    };
    // next weight stage (st + S - 1) into the slot every wave left at the previous barrier
    const int wsrc = st + C::S - 1 < nst ? st + C::S - 1 : nst - 1, wslot = (st + C::S - 1) % C::S;
    // the group's hi adds materialised here (an empty asm reading and writing the sums): the
    // compiler had sunk all of them to the stage end, behind the last MFMA, keeping 12 hi
    // temporaries live and adding 48 dependent adds to the tail the partner wave waits on
    auto pin_group = [&](int g) {
      if constexpr (DN_X6P_PIN) {
#pragma unroll
        for (int m = 0; m < MTC; ++m)
#pragma unroll
          for (int q = g * QG; q < (g + 1) * QG; ++q) asm volatile("" : "+v"(acc[m][q]));
      }
    };
    if constexpr (STAGED) {
      static_assert(!DN_X6P_DMAI || C::PPW <= NG, "one DMA piece per early fragment group");
      const int ky = t / 3, kx = t - 3 * ky;
      auto read_a = [&](int p) {
#pragma unroll
        for (int m = 0; m < MTC; ++m) {
          int pix;
          if constexpr (SEL) pix = selpix[m] + ky * C::IW + kx;
          else pix = (wave * C::MT + m + ky) * C::IW + li + kx;
          const int off = pix * C::KC + x6_swz(pix, lg) * 8;
          av[p][m] = *reinterpret_cast<const bf16x8*>(lx + p * C::XPL + off);
        }
      };
      auto read_bp = [&](int p) {  // plane p of B fragment 0
        const int row = qoff * 16 + li;
        const int off = row * C::KC + x6_swz(row, lg) * 8;
        bv[p][0] = *reinterpret_cast<const bf16x8*>(lw + p * C::WPL + off);
      };
      auto lo = [&](int pa, int pb) {
#pragma unroll
        for (int m = 0; m < MTC; ++m) accl[m][0] = mfma_bf16(av[pa][m], bv[pb][0], accl[m][0]);
      };
      read_a(0); read_bp(0); read_bp(1);
      __builtin_amdgcn_sched_barrier(0);
      read_a(1); read_bp(2);
      __builtin_amdgcn_sched_barrier(0);
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      f32x4 hi[MTC];
#pragma unroll
      for (int m = 0; m < MTC; ++m)
        hi[m] = mfma_bf16(av[0][m], bv[0][0], z);
      lo(0, 1);
      __builtin_amdgcn_sched_barrier(0);
      read_a(2); read_b(1);
      __builtin_amdgcn_sched_barrier(0);
      lo(1, 0); lo(0, 2); lo(1, 1);
      __builtin_amdgcn_sched_barrier(0);
      read_b(2);
      __builtin_amdgcn_sched_barrier(0);
      lo(2, 0);
#pragma unroll
      for (int m = 0; m < MTC; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[m][0][r] = acc[m][0][r] + hi[m][r];
      pin_group(0);
      __builtin_amdgcn_sched_barrier(0);
      if (DN_X6P_DMAI) load_w_piece(wsrc, wslot, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int g = 1; g < NG; ++g) {
        x6_group_c<MTC, NTW, QG>(acc, accl, av, bv, g * QG);
        pin_group(g);
        __builtin_amdgcn_sched_barrier(0);
        if (DN_X6P_DMAI && g < C::PPW) load_w_piece(wsrc, wslot, g);
        if (g + 2 < NG) read_b(g + 2);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int g = 0; g < LOOK; ++g) read_b(g);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        x6_group_c<MTC, NTW, QG>(acc, accl, av, bv, g * QG);
        __builtin_amdgcn_sched_barrier(0);
        if (g + LOOK < NG) read_b(g + LOOK);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    X6_STAMP(2 + 3 * st);
    const bool xstep = t == 8 && more;
    if (xstep) {
      x6_barrier();  // every wave is done with this chunk's x tile
      store_x();
      load_x((c + 2 < nch ? c + 2 : nch - 1) * C::KC);  // uniform count: re-load at the end
    }
    constexpr bool DMAI = STAGED && DN_X6P_DMAI;
    if (!DMAI) load_w(wsrc, wslot);
    // own DMAs of stage st+1 landed: issued after them are those of stages st+2, st+S-1 and the
    // next-but-one chunk's x loads when issued in this stage (xstep) or the previous one (a
    // chunk's first stage) -- the x loads are not waited for here
    // (stages 0 and 1: the prologue's chunk-1 x loads are younger than their DMAs)
    // DMAI: a stage's weight DMAs precede its x loads, so the x loads of stage st-2 (a chunk's
    // second stage, t == 1) are younger than stage st+1's DMAs too
    if (xstep || (t == 0 && c > 0) || (DMAI && t == 1 && c > 0) || (c == 0 && t < 2))
      X6_WAITCNT_VM_LGKM0(C::PPW * (C::S - 2) + C::XITEMS);
    else
      X6_WAITCNT_VM_LGKM0(C::PPW * (C::S - 2));
    if (xstep) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own x-tile stores done
    X6_STAMP(3 + 3 * st);
    x6_barrier();
  };
  // TAIL: the instantiation's last-chunk packing (the host passes a.x6_tail == TAIL)
  for (int c = 0; c < nch; ++c) {
    if constexpr (TAIL == 0) {
#pragma unroll 1
      for (int t = 0; t < 9; ++t) stage(std::integral_constant<int, 0>{}, c, t);
    } else {
      const int ns = c + 1 < nch ? 9 : tail_st;
#pragma unroll 1
      for (int t = 0; t < ns; ++t) stage(std::integral_constant<int, 3>{}, c, t);
    }
  }
  X6_WAITCNT_VM(0);  // the trailing re-load DMAs must land before the LDS is reused
  x6_barrier();
  X6_STAMP(1 + 3 * nst);
  x6_fold(acc, accl);
  if constexpr (SEL) {
    // the pair image: OH/2 rows, row ty0/2 + 2(w&3) + m, column tx0 + fragment row, the wave's
    // NTW*16 channels (the epilogue places wave w's rows at its ty0 argument + w*MT + m)
    FwdArgs ap = a;
    ap.OH = a.OH / 2;
    ap.NOUT = NTW * 16;
    ap.out_off = a.out_off + qoff * 16;
    ap.bias = a.bias ? a.bias + qoff * 16 : nullptr;
    fwd_epilogue<NTW, MTC, C::PS, false>(ap, acc, reinterpret_cast<float*>(lds_raw),
                                         ty0 / 2 + 2 * (wave & 3) - MTC * wave, tx0, n);
  } else {
    fwd_epilogue<NT, C::MT, C::PS, false>(a, acc, reinterpret_cast<float*>(lds_raw), ty0, tx0, n);
  }
#if DN_X6_STAMPS
  X6_STAMP(3 + 3 * nst);  // epilogue issued (stores in flight)
  __builtin_amdgcn_s_waitcnt(0);
  X6_STAMP(2 + 3 * nst);  // stores complete
#endif
}

#if DN_X6_STAMPS
// host copy of the stamp buffer (diagnostic builds only; not part of include/denoise_hip.h)
extern "C" int dn_debug_x6_stamps(unsigned long long* host, int n) {
  const int cap = 64 * 2 * X6_STAMP_SLOTS;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_x6_stamps),
                                  sizeof(unsigned long long) * (n < cap ? n : cap));
}
#endif

// ------------------------------------------------------------------------------------
// The N2N pair-pixel pass with 32-row tiles (k_c3x6s, launch_fwd_x6_sel): the 16-row SEL tile of
// k_c3x6p has half the MFMAs of a full tile for the same x staging, barriers and weight DMAs per
// stage (measured 0.34 of the bf16/6 ceiling against the full kernel's 0.47).  Here a 32 x 16
// tile's 16 cell rows give every wave two M fragments (cell rows 2w, 2w+1) of all 96 channels,
// as many MFMAs per stage as the full kernel; the 34-row x tile (117.5 KB, three planes) leaves
// room for a 2-slot ring of unpadded 18 KiB weight stages: stage st+1's 18 DMA pieces (3 per
// wave, the short waves repeating one) are issued during stage st, between its first fragment
// groups, and waited for at its end.
// ------------------------------------------------------------------------------------
struct SCfg {
  static constexpr int WAVES = 8, MT = 2, S = 2, NT = 6;
  static constexpr int TW = 16, TH = 32, IH = TH + 2, IW = TW + 2, KC = 32, NP = 96;
  static constexpr int XPIX = IH * IW;
  static constexpr int XPL = XPIX * KC;
  static constexpr int WPL = NP * KC;
  static constexpr int WST = 3 * WPL;                 // bf16 per LDS stage (unpadded)
  static constexpr int WSTP = x6_wst(NP);             // stage stride of the packed image
  static constexpr int PIECES = WST * 2 / 1024;       // 18
  static constexpr int PPW = (PIECES + WAVES - 1) / WAVES;
  static_assert(PIECES * 1024 == WST * 2 && PPW == 3, "stage = 18 whole KiB pieces");
  static constexpr int XQ = XPIX * (KC / 4);
  static constexpr int XITEMS = (XQ + WAVES * 64 - 1) / (WAVES * 64);
  static constexpr int PS = NP + 4;
  static constexpr int LBYTES_MAIN = 2 * 3 * XPL + 2 * S * WST;
  static constexpr int LEPI = 4 * WAVES * 16 * PS;
  static constexpr int LBYTES = LBYTES_MAIN > LEPI ? LBYTES_MAIN : LEPI;
  static_assert(LBYTES <= 163840, "one workgroup per CU");
};

__global__ __launch_bounds__(512, 1) void k_c3x6s(FwdArgs a) {
  using C = SCfg;
  constexpr int MT = C::MT, NT = C::NT;
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[C::LBYTES];
  __bf16* lx = reinterpret_cast<__bf16*>(lds_raw);
  __bf16* ring = lx + 3 * C::XPL;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lg = lane >> 4;
  const int tiles_x = (a.OW + C::TW - 1) / C::TW;
  int bxr, byr;  // XCD-aware tile order (conv_epi.h xcd_tile)
  xcd_tile(bxr, byr);
  const int ty0 = (bxr / tiles_x) * C::TH;
  const int tx0 = (bxr % tiles_x) * C::TW;
  const int n = byr;
  const int iy0 = ty0 - 1, ix0 = tx0 - 1;
  const float* inb = a.in + (long)n * a.IHt * a.IWt * a.in_stride + a.in_off;
  const __bf16* wimg = reinterpret_cast<const __bf16*>(a.wp);
  const int nch = a.K / C::KC;
  const int nst = 9 * nch;

  f32x4 acc[MT][NT], accl[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < NT; ++q) acc[m][q] = accl[m][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  // x-tile pixel of this lane's row of fragment m: tile cell row 2w + m, cell j = li / 2, pair
  // member s = li % 2 at pair[rd][s] of the cell (train.py:151-154)
  int selpix[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int lc = 2 * wave + m;
    const int ci = ty0 / 2 + lc, cj = tx0 / 2 + (li >> 1);
    const int r = (ci < a.OH / 2 && cj < a.OW / 2)
                      ? a.sel_rd[((long)n * (a.OH / 2) + ci) * (a.OW / 2) + cj] & 7 : 0;
    constexpr unsigned kPair = 0xB721ED84u;  // 4 bits (a | b << 2) per rd
    const int k = (kPair >> (4 * r + 2 * (li & 1))) & 3;
    selpix[m] = (2 * lc + (k >> 1)) * C::IW + 2 * (li >> 1) + (k & 1);
  }

  // x tile rows through a 32-bit buffer resource (see k_c3x6p)
  const int ry0 = iy0 > 0 ? iy0 : 0, ry1 = iy0 + C::IH < a.IHt ? iy0 + C::IH : a.IHt;
  const long row_floats = (long)a.IWt * a.in_stride;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(inb + ry0 * row_floats), (short)0,
      (int)((ry1 - ry0) * row_floats * 4), 0x00020000);
  f32x4 xr[C::XITEMS];
  auto load_x = [&](int k0) {
#pragma unroll
    for (int it = 0; it < C::XITEMS; ++it) {
      const int e = tid + it * C::WAVES * 64;
      const int q = e % (C::KC / 4), pix = e / (C::KC / 4);
      const int iy = pix / C::IW, ix = pix - iy * C::IW;
      const int gy = iy0 + iy, gx = ix0 + ix, k = k0 + 4 * q;
      const bool ok = e < C::XQ && gy >= 0 && gy < a.IHt && gx >= 0 && gx < a.IWt && k < a.K;
      const int off = ok ? (((gy - ry0) * a.IWt + gx) * a.in_stride + k) * 4 : 0x7fffffff;
      xr[it] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int it = 0; it < C::XITEMS; ++it) {
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
        *reinterpret_cast<bf16x4*>(lx + off) = h;
        *reinterpret_cast<bf16x4*>(lx + C::XPL + off) = m;
        *reinterpret_cast<bf16x4*>(lx + 2 * C::XPL + off) = l;
      }
    }
  };
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__bf16*>(wimg), (short)0, nst * C::WSTP * 2, 0x00020000);
  // piece j of stage src_st into slot `slot`: pieces w, w + 8, w + 16 (waves 2..7 repeat w + 8:
  // the same bytes to the same place), so every wave issues PPW DMAs per stage
  auto load_w_piece = [&](int src_st, int slot, int j) {
    int piece = wave + j * C::WAVES;
    if (piece >= C::PIECES) piece -= C::WAVES;
    unsigned char* dst = reinterpret_cast<unsigned char*>(ring + slot * C::WST);
    buf_lds16(wrs, dst + piece * 1024, src_st * C::WSTP * 2 + piece * 1024 + lane * 16);
  };

  // prologue: stage 0's weights, chunk 0's x tile into LDS, chunk 1's x into registers
#pragma unroll
  for (int j = 0; j < C::PPW; ++j) load_w_piece(0, 0, j);
  load_x(0);
  store_x();
  load_x((nch > 1 ? 1 : 0) * C::KC);
  X6_WAITCNT_VM(C::XITEMS);            // own stage-0 DMAs landed (older than the x loads)
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own x-tile stores done
  x6_barrier();

  constexpr int NG = NT;  // fragment groups of one B fragment (carried form, QG = 1)
#pragma unroll 1
  for (int st = 0; st < nst; ++st) {
    const int c = st / 9, t = st - 9 * c;
    const bool more = c + 1 < nch;
    const int ky = t / 3, kx = t - 3 * ky;
    const __bf16* lw = ring + (st % C::S) * C::WST;
    const int wsrc = st + 1 < nst ? st + 1 : nst - 1, wslot = (st + 1) % C::S;
    bf16x8 av[3][MT], bv[3][NT];
    auto read_a = [&](int p) {
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int pix = selpix[m] + ky * C::IW + kx;
        av[p][m] = *reinterpret_cast<const bf16x8*>(lx + p * C::XPL + pix * C::KC + x6_swz(pix, lg) * 8);
      }
    };
    auto read_b = [&](int q) {
      const int row = q * 16 + li;
      const int off = row * C::KC + x6_swz(row, lg) * 8;
#pragma unroll
      for (int p = 0; p < 3; ++p) bv[p][q] = *reinterpret_cast<const bf16x8*>(lw + p * C::WPL + off);
    };
    auto read_bp = [&](int p) {
      const int off = li * C::KC + x6_swz(li, lg) * 8;
      bv[p][0] = *reinterpret_cast<const bf16x8*>(lw + p * C::WPL + off);
    };
    auto lo = [&](int pa, int pb) {
#pragma unroll
      for (int m = 0; m < MT; ++m) accl[m][0] = mfma_bf16(av[pa][m], bv[pb][0], accl[m][0]);
    };
    auto pin_group = [&](int g) {
#pragma unroll
      for (int m = 0; m < MT; ++m) asm volatile("" : "+v"(acc[m][g]));
    };
    // group 0 as a read/compute pipeline (k_c3x6p's STAGED order), then groups 1..5 with B read
    // two groups ahead; the next stage's DMA pieces after groups 0, 1, 2
    read_a(0); read_bp(0); read_bp(1);
    __builtin_amdgcn_sched_barrier(0);
    read_a(1); read_bp(2);
    __builtin_amdgcn_sched_barrier(0);
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    f32x4 hi[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) hi[m] = mfma_bf16(av[0][m], bv[0][0], z);
    lo(0, 1);
    __builtin_amdgcn_sched_barrier(0);
    read_a(2); read_b(1);
    __builtin_amdgcn_sched_barrier(0);
    lo(1, 0); lo(0, 2); lo(1, 1);
    __builtin_amdgcn_sched_barrier(0);
    read_b(2);
    __builtin_amdgcn_sched_barrier(0);
    lo(2, 0);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[m][0][r] = acc[m][0][r] + hi[m][r];
    pin_group(0);
    __builtin_amdgcn_sched_barrier(0);
    load_w_piece(wsrc, wslot, 0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int g = 1; g < NG; ++g) {
      x6_group_c<MT, NT, 1>(acc, accl, av, bv, g);
      pin_group(g);
      __builtin_amdgcn_sched_barrier(0);
      if (g < C::PPW) load_w_piece(wsrc, wslot, g);
      if (g + 2 < NG) read_b(g + 2);
      __builtin_amdgcn_sched_barrier(0);
    }
    const bool xstep = t == 8 && more;
    if (xstep) {
      x6_barrier();  // every wave is done with this chunk's x tile
      store_x();
      load_x((c + 2 < nch ? c + 2 : nch - 1) * C::KC);  // uniform count: re-load at the end
    }
    // own DMAs of stage st+1 landed (issued in this stage); the x loads issued after them (an
    // xstep) are not waited for -- those of the previous xstep are (one stage after their issue)
    if (xstep)
      X6_WAITCNT_VM_LGKM0(C::XITEMS);
    else
      X6_WAITCNT_VM_LGKM0(0);
    if (xstep) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own x-tile stores done
    x6_barrier();
  }
  X6_WAITCNT_VM(0);  // trailing re-load DMAs / x loads land before the LDS is reused
  x6_barrier();
  x6_fold(acc, accl);
  // the pair image: OH/2 rows, row ty0/2 + 2w + m (the epilogue places wave w's rows at its ty0
  // argument + w*MT + m), all 96 channels
  FwdArgs ap = a;
  ap.OH = a.OH / 2;
  fwd_epilogue<NT, MT, C::PS, false>(ap, acc, reinterpret_cast<float*>(lds_raw), ty0 / 2, tx0, n);
}

// ------------------------------------------------------------------------------------
// Two-workgroups-per-CU variant for large grids (k_c3x6h): 4 waves on an 8 x 16 x 16*NT tile
// (wave w: rows 2w, 2w+1), 70 KB of LDS (the x tile's three planes + a 2-slot ring of unpadded
// 18 KiB weight stages), so two workgroups share a CU and one's prologue (x tile from HBM) and
// epilogue overlap the other's main loop -- the per-tile cost the one-workgroup-per-CU kernel
// pays in series (k_c3x6p: ~4 us prologue + ~3 us epilogue per 16-row tile).  Stage st+1's
// weights are DMA'd at the start of stage st (5 x 1 KiB per wave; the 18 pieces of a stage are
// spread over the 4 waves, the two short waves re-load one of theirs, so every wave waits on a
// constant count); the next chunk's x tile is loaded into registers at the start of a chunk,
// after that stage's DMA, and split into LDS at its end.  Stage reads and MFMAs as k_c3x6p.
// ------------------------------------------------------------------------------------
template <int NT, int MT_ = 2, int S_ = 2>
struct HCfg {
  static constexpr int WAVES = 4, MT = MT_, S = S_;
  static constexpr int TW = 16, TH = WAVES * MT, IH = TH + 2, IW = TW + 2, KC = 32, NP = 16 * NT;
  static constexpr int XPIX = IH * IW;
  static constexpr int XPL = XPIX * KC;
  static constexpr int WPL = NP * KC;
  static constexpr int WST = 3 * WPL;                 // bf16 per stage (unpadded)
  static constexpr int WSTP = x6_wst(NP);             // stage stride of the packed image
  static constexpr int PIECES = WST * 2 / 1024;       // 1 KiB DMA pieces per stage
  static constexpr int PPW = (PIECES + WAVES - 1) / WAVES;
  static_assert(PIECES * 1024 == WST * 2, "stage = whole KiB pieces");
  static constexpr int XQ = XPIX * (KC / 4);
  static constexpr int XITEMS = (XQ + WAVES * 64 - 1) / (WAVES * 64);
  static constexpr int PS = NP + 4;
  static constexpr int LBYTES_MAIN = 2 * 3 * XPL + 2 * S * WST;
  static constexpr int LEPI = 4 * WAVES * 16 * PS;
  static constexpr int LBYTES = LBYTES_MAIN > LEPI ? LBYTES_MAIN : LEPI;
  static_assert(2 * LBYTES <= 163840, "two workgroups per CU");
};

#ifndef DN_X6H_LOOK
#define DN_X6H_LOOK 2  // B fragment groups read ahead of their MFMAs in k_c3x6h
#endif
#ifndef DN_X6H_CARRY4
#define DN_X6H_CARRY4 1  // A/B switch: 1 = MT = 4 with NT <= 3 carries the corrections too (96 acc VGPRs)
#endif
#ifndef DN_X6H_PIN
#define DN_X6H_PIN 0  // A/B switch: 1 = MT = 2's hi adds pinned per group (100->96 @256^2: 1-2 % slower)
#endif
// S_ = 3 (small grids, MT = 1): a 3-slot weight ring, stage st + 2 requested at the start of st,
// so a stage waits on neither the L2 latency of its weights nor that of the next stage's
template <int NT, int TAIL, int MT_ = 2, int S_ = 2>
__global__ __launch_bounds__(256, 2) void k_c3x6h(FwdArgs a) {
  using C = HCfg<NT, MT_, S_>;
  constexpr int MT = C::MT;
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[C::LBYTES];
  __bf16* lx = reinterpret_cast<__bf16*>(lds_raw);
  __bf16* ring = lx + 3 * C::XPL;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  const int li = lane & 15, lg = lane >> 4;
  const int tiles_x = (a.OW + C::TW - 1) / C::TW;
  int bxr, byr;  // XCD-aware tile order (conv_epi.h xcd_tile)
  xcd_tile(bxr, byr);
  const int ty0 = (bxr / tiles_x) * C::TH;
  const int tx0 = (bxr % tiles_x) * C::TW;
  const int n = byr;
  const int iy0 = ty0 - 1, ix0 = tx0 - 1;
  const float* inb = a.in + (long)n * a.IHt * a.IWt * a.in_stride + a.in_off;
  const __bf16* wimg = reinterpret_cast<const __bf16*>(a.wp) + (long)blockIdx.z * a.wp_z;
  const int nch = (a.K + C::KC - 1) / C::KC;
  constexpr int tail = TAIL;
  constexpr int tail_st = tail == 1 ? 2 : 5;
  const int nst = 9 * nch - (tail ? 9 - tail_st : 0);

  f32x4 acc[MT][NT], accl[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < NT; ++q) acc[m][q] = accl[m][q] = f32x4{0.f, 0.f, 0.f, 0.f};

  // input rows of this tile through a 32-bit buffer resource (see k_c3x6p)
  const int ry0 = iy0 > 0 ? iy0 : 0, ry1 = iy0 + C::IH < a.IHt ? iy0 + C::IH : a.IHt;
  const long row_floats = (long)a.IWt * a.in_stride;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(inb + ry0 * row_floats), (short)0, (int)((ry1 - ry0) * row_floats * 4),
      0x00020000);
  f32x4 xr[C::XITEMS];
  auto load_x = [&](int k0) {
#pragma unroll
    for (int it = 0; it < C::XITEMS; ++it) {
      const int e = tid + it * C::WAVES * 64;
      const int q = e % (C::KC / 4), pix = e / (C::KC / 4);
      const int iy = pix / C::IW, ix = pix - iy * C::IW;
      const int gy = iy0 + iy, gx = ix0 + ix, k = k0 + 4 * q;
      const bool ok = e < C::XQ && gy >= 0 && gy < a.IHt && gx >= 0 && gx < a.IWt && k < a.K;
      const int off = ok ? (((gy - ry0) * a.IWt + gx) * a.in_stride + k) * 4 : 0x7fffffff;
      xr[it] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int it = 0; it < C::XITEMS; ++it) {
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
        *reinterpret_cast<bf16x4*>(lx + off) = h;
        *reinterpret_cast<bf16x4*>(lx + C::XPL + off) = m;
        *reinterpret_cast<bf16x4*>(lx + 2 * C::XPL + off) = l;
      }
    }
  };
  // stage src_st's 18 pieces into slot `slot`: wave w copies pieces w, w+4, ...; a wave with
  // fewer than PPW repeats its last piece (same bytes, same place) so every wave issues PPW
  // (buffer loads to LDS, not global_load_lds: see k_c3x6p's load_w)
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__bf16*>(wimg), (short)0, nst * C::WSTP * 2, 0x00020000);
  auto load_w = [&](int src_st, int slot) {
    unsigned char* dst = reinterpret_cast<unsigned char*>(ring + slot * C::WST);
#pragma unroll
    for (int j = 0; j < C::PPW; ++j) {
      int piece = wave + j * C::WAVES;
      if (piece >= C::PIECES) piece -= C::WAVES;
#if DN_X6_GDMA
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(reinterpret_cast<const unsigned char*>(wimg) +
                                                          (long)src_st * C::WSTP * 2 + piece * 1024 + lane * 16),
          (__attribute__((address_space(3))) void*)(dst + piece * 1024), 16, 0, 0);
#else
      buf_lds16(wrs, dst + piece * 1024, src_st * C::WSTP * 2 + piece * 1024 + lane * 16);
#endif
    }
  };

  // prologue: the first S - 1 stages' weights (L2) and chunk 0's x tile (HBM) in flight together
#pragma unroll
  for (int j = 0; j + 1 < C::S; ++j) load_w(j < nst ? j : nst - 1, j);
  load_x(0);
  store_x();                           // waits for the x loads (and the older DMA)
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own x-tile stores done
  x6_barrier();

  auto stage = [&](int c, int t) {
    const bool more = c + 1 < nch;
    const int st = 9 * c + t;
    const __bf16* lw = ring + (st % C::S) * C::WST;
    // stage st+S-1's weights into the slot of stage st-1 (every wave left it at the last
    // barrier); past the end a re-load of the last stage
    load_w(st + C::S - 1 < nst ? st + C::S - 1 : nst - 1, (st + C::S - 1) % C::S);
    if (t == 0 && more) load_x((c + 1) * C::KC);  // the next chunk, after this stage's DMA
    const int mode = (tail && c + 1 == nch) ? tail : 0;
    // MT = 4: the A pieces of two rows at a time (registers), the B fragments read once for all
    constexpr int MH = MT >= 4 ? 2 : MT;
    // MT = 4 keeps the per-block form (its 2 x 48 accumulators at NT = 6 leave no room for accl)
    constexpr bool BLK = MT >= 4 && !(DN_X6H_CARRY4 && NT <= 3);
    constexpr int QG = MT >= 4 ? 1 : x6_qgc(MT, NT), NG = NT / QG,
                  LOOK = NG < DN_X6H_LOOK ? NG : DN_X6H_LOOK;
    bf16x8 bv[3][NT];
    auto read_b = [&](int g) {
#pragma unroll
      for (int q = g * QG; q < (g + 1) * QG; ++q) {
        const int row = q * 16 + li;
        const int off = row * C::KC + x6_swz(row, lg) * 8;
#pragma unroll
        for (int p = 0; p < 3; ++p)
          bv[p][q] = *reinterpret_cast<const bf16x8*>(lw + p * C::WPL + off);
      }
    };
#pragma unroll
    for (int mh = 0; mh < MT / MH; ++mh) {
      bf16x8 av[3][MH];
      if (mode == 1) {
        const int ta = 8 * t + 2 * lg, tb = ta + 1;
        const int ca = ta < 9 ? ta : 8, cb = tb < 9 ? tb : 8;
        const int da = (ca / 3) * C::IW + ca % 3, db = (cb / 3) * C::IW + cb % 3;
        const bf16x4 z4 = {(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
#pragma unroll
        for (int i = 0; i < MH; ++i) {
          const int p0 = (wave * MT + mh * MH + i) * C::IW + li;
          const int pa = p0 + da, pb = p0 + db;
          const int oa = pa * C::KC + x6_swz(pa, 0) * 8, ob = pb * C::KC + x6_swz(pb, 0) * 8;
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            bf16x4 va = *reinterpret_cast<const bf16x4*>(lx + p * C::XPL + oa);
            bf16x4 vb = *reinterpret_cast<const bf16x4*>(lx + p * C::XPL + ob);
            if (ta > 8) va = z4;
            if (tb > 8) vb = z4;
            av[p][i] = __builtin_shufflevector(va, vb, 0, 1, 2, 3, 4, 5, 6, 7);
          }
        }
      } else if (mode == 2) {
        const int ta = 2 * t + (lg >> 1);
        const int ca = ta < 9 ? ta : 8;
        const int da = (ca / 3) * C::IW + ca % 3;
        const bf16x8 z8 = {};
#pragma unroll
        for (int i = 0; i < MH; ++i) {
          const int pa = (wave * MT + mh * MH + i) * C::IW + li + da;
          const int oa = pa * C::KC + x6_swz(pa, lg & 1) * 8;
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            const bf16x8 v = *reinterpret_cast<const bf16x8*>(lx + p * C::XPL + oa);
            av[p][i] = ta > 8 ? z8 : v;
          }
        }
      } else {
        const int ky = t / 3, kx = t - 3 * ky;
#pragma unroll
        for (int i = 0; i < MH; ++i) {
          const int pix = (wave * MT + mh * MH + i + ky) * C::IW + li + kx;
          const int off = pix * C::KC + x6_swz(pix, lg) * 8;
#pragma unroll
          for (int p = 0; p < 3; ++p)
            av[p][i] = *reinterpret_cast<const bf16x8*>(lx + p * C::XPL + off);
        }
      }
      if (mh == 0) {
#pragma unroll
        for (int g = 0; g < LOOK; ++g) read_b(g);
      }
      __builtin_amdgcn_sched_barrier(0);
      f32x4(&acch)[MH][NT] = *reinterpret_cast<f32x4(*)[MH][NT]>(&acc[mh * MH]);
      f32x4(&acclh)[MH][NT] = *reinterpret_cast<f32x4(*)[MH][NT]>(&accl[mh * MH]);
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        if constexpr (BLK) x6_group<MH, NT, QG>(acch, av, bv, g * QG);
        else x6_group_c<MH, NT, QG>(acch, acclh, av, bv, g * QG);
        if constexpr (MT >= 4 || DN_X6H_PIN) {  // the block sums' adds here, not sunk to the stage end
#pragma unroll
          for (int i = 0; i < MH; ++i)
#pragma unroll
            for (int q = g * QG; q < (g + 1) * QG; ++q) asm volatile("" : "+v"(acch[i][q]));
        }
        __builtin_amdgcn_sched_barrier(0);
        if (mh == 0 && g + LOOK < NG) read_b(g + LOOK);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    const int ns = (tail && c + 1 == nch) ? tail_st : 9;
    const bool xstep = t == ns - 1 && more;
    if (xstep) {
      x6_barrier();  // every wave is done with this chunk's x tile
      store_x();
    }
    // own DMAs of stage st+1 landed; younger: those of stages st+2 .. st+S-1 and the chunk's x
    // loads while they were issued after it (t <= S-2); after the last stage none in flight
    // (the epilogue reuses the ring)
    if constexpr (C::S == 2) {
      if (t == 0 && more) X6_WAITCNT_VM(C::XITEMS);
      else X6_WAITCNT_VM(0);
    } else {
      if (st + 1 == nst) X6_WAITCNT_VM(0);
      else if (t <= C::S - 2 && more) X6_WAITCNT_VM((C::S - 2) * C::PPW + C::XITEMS);
      else X6_WAITCNT_VM((C::S - 2) * C::PPW);
    }
    if (xstep) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own x-tile stores done
    x6_barrier();
  };
  for (int c = 0; c < nch; ++c) {
    const int ns = (tail && c + 1 == nch) ? tail_st : 9;
#pragma unroll 1
    for (int t = 0; t < ns; ++t) stage(c, t);
  }
  x6_fold(acc, accl);
  fwd_epilogue<NT, MT, C::PS, false>(a, acc, reinterpret_cast<float*>(lds_raw), ty0, tx0, n);
}

template <int NT, int MT = 2>
static hipError_t run_x6h(const FwdArgs& a, int nz, hipStream_t s) {
  using C = HCfg<NT, MT>;
  const int tx = (a.OW + C::TW - 1) / C::TW, ty = (a.OH + C::TH - 1) / C::TH;
  const dim3 grid(tx * ty, a.N, nz), block(C::WAVES * 64);
  static const std::string kn[3] = {x6_kname("k_c3x6h", NT, 0, MT), x6_kname("k_c3x6h", NT, 1, MT),
                                    x6_kname("k_c3x6h", NT, 2, MT)};
  prof_kernel(kn[a.x6_tail > 2 ? 0 : a.x6_tail].c_str());
  if (a.x6_tail == 1)
    hipLaunchKernelGGL((k_c3x6h<NT, 1, MT>), grid, block, 0, s, a);
  else if (a.x6_tail == 2)
    hipLaunchKernelGGL((k_c3x6h<NT, 2, MT>), grid, block, 0, s, a);
  else
    hipLaunchKernelGGL((k_c3x6h<NT, 0, MT>), grid, block, 0, s, a);
  return hipGetLastError();
}

// small grids (below one round of 16 x 16 tiles), plain image: the 3-slot ring
template <int NT, int MT>
static hipError_t run_x6h3(const FwdArgs& a, int nz, hipStream_t s) {
  using C = HCfg<NT, MT, 3>;
  const int tx = (a.OW + C::TW - 1) / C::TW, ty = (a.OH + C::TH - 1) / C::TH;
  static const std::string kn = x6_kmore(x6_kname("k_c3x6h", NT, 0, MT), "3");
  prof_kernel(kn.c_str());
  hipLaunchKernelGGL((k_c3x6h<NT, 0, MT, 3>), dim3(tx * ty, a.N, nz), dim3(C::WAVES * 64), 0, s, a);
  return hipGetLastError();
}

// Pre-split weight image, one per output-channel block z: [chunk][tap][piece][n < NP][32 k],
// bf16, 16-B quads swizzled by n (see x6_swz); zero padded past K / NOUT.
// Each stage is x6_wst(NP) elements (the tail past 3*NP*32 is zero).
// tail (x6_tail_mode, for k_c3x6p): the last chunk's channels packed over its first stages:
// 1: (<= 4 channels) im2col, k = 4*tap + channel (stage 0: taps 0..7, stage 1: tap 8);
// 2: (<= 16 channels) two taps per stage, k = 16*(tap - 2*stage) + channel (5 stages).
__device__ __forceinline__ void pk_x6(const PackJob& j, long e) {
  const int NP = j.g0, nch = j.nch, wst = x6_wst(NP), pad = wst - 3 * NP * 32;
  const long per_z = (long)nch * 9 * NP * 32;
  const int z = (int)(e / per_z);
  const long r = e - (long)z * per_z;
  const int kk = (int)(r % 32), nn = (int)((r / 32) % NP);
  const int ct = (int)(r / (32L * NP)), c = ct / 9;
  int t = ct % 9, k = c * 32 + kk;
  bool live = true;
  if (j.tail == 1 && c == nch - 1) {
    const int kg = 32 * t + kk;  // im2col index of the tail stage: 4 * tap + channel
    live = t < 2 && kg < 36;
    t = kg >> 2;
    k = c * 32 + (kg & 3);
  } else if (j.tail == 2 && c == nch - 1) {  // tap pair: 16 * (tap - 2t) + channel
    const int tap = 2 * t + (kk >> 4);
    live = t < 5 && tap < 9;
    t = tap < 9 ? tap : 8;
    k = c * 32 + (kk & 15);
  }
  float v = 0.f;
  if (live && k < j.K && nn < j.NOUT && (j.zc == 0 || z * j.zc + nn < j.ntot)) {
    const int tm = j.flip ? j.taps - 1 - t : t;
    v = j.w[(long)z * j.sZ + (long)k * j.sK + (long)nn * j.sN + (long)tm * j.sT];
  }
  __bf16 h, m, l;
  split3(v, h, m, l);
  // (block z's image starts at z x x6_pack_elems / nz: 12 stage slots per chunk for 96- and
  // 48-wide blocks, which have room for the Winograd image too)
  __bf16* st = static_cast<__bf16*>(j.out) + ((long)z * nch * (NP == 96 || NP == 48 ? 12 : 9) + ct) * wst;
  const int o = nn * 32 + x6_swz(nn, kk >> 3) * 8 + (kk & 7);
  st[o] = h;
  st[NP * 32 + o] = m;
  st[2 * NP * 32 + o] = l;
  if ((int)(r % (32L * NP)) < pad) st[3 * NP * 32 + (int)(r % (32L * NP))] = (__bf16)0.f;
}

// Winograd F(2,3) image of k_c3w6 (conv_w6.hip): [chunk][stage][piece][n < 96][32 k] as pk_x6,
// stage 4 ky + p holding u_p = G g of kernel row ky (g = the three kx taps of (k, n)):
// u = (g0, (g0 + g1 + g2) / 2, (g0 - g1 + g2) / 2, g2), each rounded once from fp64, then split.
// Last chunk (tail): 1: stage p, k = 4 ky + channel (k < 16; k = 16 + 4 ky + channel with planes
// (h, h, m)); 2: stage 2p + h, k = 16 (ky - 2h) + channel
// for h = 0, h = 1: kernel row 2, k = channel with planes (h, m, l) and k = 16 + channel with
// planes (h, h, m) (k_c3w6's stage mode 4);
// 3 (X6_T1): stage p, k = 8 ky + slot, plane 0 = u's piece of each of the six products (k_c3w6).
__device__ __forceinline__ void pk_w6(const PackJob& j, long e0) {
  const int NP = j.g0, nch = j.nch, wst = x6_wst(NP), pad = wst - 3 * NP * 32;
  const long per_z = (long)nch * 12 * NP * 32;  // one image per output-channel block z (zc)
  const int z = (int)(e0 / per_z);
  const long e = e0 - (long)z * per_z;
  const int kk = (int)(e % 32), nn = (int)((e / 32) % NP);
  const int cs = (int)(e / (32L * NP)), c = cs / 12, s = cs % 12;
  int ky = s >> 2, p = s & 3, k = c * 32 + kk, slot = -1;
  bool live = true, dup = false;
  if (j.tail == 3 && c == nch - 1) {  // X6_T1: k = 8 ky + product slot, channel c * 32 only
    p = s; ky = kk >> 3; slot = kk & 7; k = c * 32;
    live = s < 4 && ky < 3 && slot < 6;
  } else if (j.tail == 1 && c == nch - 1) {  // both K halves k = 4 ky + channel, upper (h, h, m)
    p = s; ky = (kk & 15) >> 2; k = c * 32 + (kk & 3);
    live = s < 4 && (kk & 15) < 12;
    dup = kk >= 16;
  } else if (j.tail == 2 && c == nch - 1) {
    p = s >> 1; ky = 2 * (s & 1) + (kk >> 4); k = c * 32 + (kk & 15);
    live = s < 8 && ky < 3;
    if ((s & 1) && kk >= 16) { ky = 2; live = s < 8; dup = true; }
  }
  float v = 0.f;
  if (live && k < j.K && nn < j.NOUT && (j.zc == 0 || z * j.zc + nn < j.ntot)) {
    double g[3];
    for (int kx = 0; kx < 3; ++kx) {
      // flip 2: the transposed taps (u along ky for each kx: the y-tile image of k_c3w6s)
      const int t = 3 * ky + kx, tm = j.flip == 2 ? 3 * kx + ky : (j.flip ? j.taps - 1 - t : t);
      g[kx] = j.w[(long)z * j.sZ + (long)k * j.sK + (long)nn * j.sN + (long)tm * j.sT];
    }
    const double u = p == 0 ? g[0] : (p == 1 ? (g[0] + g[1] + g[2]) * 0.5
                                             : (p == 2 ? (g[0] - g[1] + g[2]) * 0.5 : g[2]));
    v = (float)u;
  }
  __bf16 h, m, l;
  split3(v, h, m, l);
  if (slot >= 0) {  // u's piece of product slot (h,h) (h,m) (m,h) (h,l) (l,h) (m,m), plane 0 only
    h = slot == 1 || slot == 5 ? m : (slot == 3 ? l : h);
    m = l = (__bf16)0.f;
  }
  if (dup) {  // tail 2, kernel row 2, upper half: planes (h, h, m)
    l = m;
    m = h;
  }
  __bf16* st = static_cast<__bf16*>(j.out) + ((long)z * nch * 12 + cs) * wst;
  const int o = nn * 32 + x6_swz(nn, kk >> 3) * 8 + (kk & 7);
  st[o] = h;
  st[NP * 32 + o] = m;
  st[2 * NP * 32 + o] = l;
  if ((int)(e % (32L * NP)) < pad) st[3 * NP * 32 + (int)(e % (32L * NP))] = (__bf16)0.f;
}

// the forward-family kernel's per-chunk LDS image [chunk][tap][k][n] (zero padded), one image
// set per z (deconv forward: one per (a,b))
__device__ __forceinline__ void pk_f32(const PackJob& j, long e) {
  const int KC = j.g0, TAPS = j.g1, WNS = j.g2, LW = j.g3;
  const long per_z = (long)j.nch * LW;
  const int z = (int)(e / per_z);
  const long r = e - (long)z * per_z;
  const int c = (int)(r / LW), q = (int)(r % LW);
  float v = 0.f;
  if (q < TAPS * KC * WNS) {
    const int t = q / (KC * WNS), kk = (q / WNS) % KC, nn = q % WNS, k = c * KC + kk;
    if (k < j.K && nn < j.NOUT && (j.zc == 0 || z * j.zc + nn < j.ntot)) {
      const int tm = j.flip ? (j.taps - 1 - t) : t;
      v = j.w[(long)z * j.sZ + (long)k * j.sK + (long)nn * j.sN + (long)tm * j.sT];
    }
  }
  static_cast<float*>(j.out)[e] = v;
}

// nin_a / nin_b (OIHW 96x96x1x1) -> the two pre-split head images: [plane][b][out][32] in the
// head kernel's permuted K order (see k_nin_head_x6); j.flip: the transposed matrices (row o of
// the image = column o of the weight), the backward's Wb^T | Wa^T (k_head_bwd_x6)
__device__ __forceinline__ void pk_head_x6(const PackJob& j, long e) {
  const int layer = (int)(e / X6_HEAD_BF), r0 = (int)(e % X6_HEAD_BF);
  const int p = r0 / (3 * 96 * 32), row = (r0 / 32) % (3 * 96), k = r0 % 32;  // row = b*96 + o
  const int b = row / 96, o = row % 96, g = k >> 3, jj = k & 7;
  const int ch = 32 * b + (jj < 4 ? 4 * g + jj : 16 + 4 * g + (jj - 4));
  __bf16 h, m, l;
  split3((layer ? j.w2 : j.w)[j.flip ? ch * 96 + o : o * 96 + ch], h, m, l);
  static_cast<__bf16*>(j.out)[layer * X6_HEAD_BF + (p * 3 * 96 + row) * 32 + x6_swz(row, g) * 8 + jj] =
      p == 0 ? h : (p == 1 ? m : l);
}

// raw deconv weight W[ci][co][a][b] (96, 96, 2, 2) -> four pre-split parity images
__device__ __forceinline__ void pk_deconv_x6(const PackJob& j, long e) {
  const int par = (int)(e / X6_HEAD_BF), r0 = (int)(e % X6_HEAD_BF);
  const int p = r0 / (3 * 96 * 32), row = (r0 / 32) % (3 * 96), k = r0 % 32;  // row = b*96 + co
  const int b = row / 96, co = row % 96;
  __bf16 h, m, l;
  split3(j.w[((32 * b + k) * 96 + co) * 4 + par], h, m, l);  // par = 2a + b
  static_cast<__bf16*>(j.out)[par * X6_HEAD_BF + (p * 3 * 96 + row) * 32 + x6_swz(row, k >> 3) * 8 + (k & 7)] =
      p == 0 ? h : (p == 1 ? m : l);
}

// raw deconv weight W[ci][co][a][b] (96, 96, 2, 2) -> the data gradient's pre-split images: per
// input-channel half h and parity, [plane][K block (32 co)][row = ci - 48h][32 co] (X6_DG_BF each)
constexpr int X6_DG_BF = 3 * 3 * 48 * 32;
__device__ __forceinline__ void pk_deconv_dgrad_x6(const PackJob& j, long e) {
  const int h = (int)(e / (4 * X6_DG_BF)), par = (int)(e / X6_DG_BF) % 4, r0 = (int)(e % X6_DG_BF);
  const int p = r0 / (3 * 48 * 32), row = (r0 / 32) % (3 * 48), k = r0 % 32;  // row = kb*48 + ci'
  const int kb = row / 48, ci = 48 * h + row % 48, co = 32 * kb + k;
  __bf16 hh, m, l;
  split3(j.w[((long)ci * 96 + co) * 4 + par], hh, m, l);
  static_cast<__bf16*>(j.out)[(long)(h * 4 + par) * X6_DG_BF + (p * 3 * 48 + row) * 32 +
                              x6_swz(row, k >> 3) * 8 + (k & 7)] = p == 0 ? hh : (p == 1 ? m : l);
}

// launch_pack_bf16's image (k_pack_bf16, conv_bf16.hip): [chunk][ky][kx][n][40], zero padded
__device__ __forceinline__ void pk_bf16(const PackJob& j, long e) {
  const int NP = j.g0, WST = j.g1, spc = j.g2 ? 3 : 1;
  const long st = e / WST;
  const int r = (int)(e - st * WST);
  const int c = (int)(st / spc), ky = (int)(st % spc);
  float v = 0.f;
  if (r < spc * NP * 32) {  // conv_bf16.hip's image: 32-bf16 rows, quads swizzled (x6_swz)
    const int row = r / 32, kx = row / NP, nn = row % NP;
    const int kk = x6_swz(row, (r % 32) / 8) * 8 + r % 8;
    const int k = c * 32 + kk;
    if (k < j.K && nn < j.NOUT) {
      const int t = j.g2 ? ky * 3 + kx : 0;
      const int tm = j.flip ? j.taps - 1 - t : t;
      v = j.w[(long)k * j.sK + (long)nn * j.sN + (long)tm * j.sT];
    }
  }
  static_cast<__bf16*>(j.out)[e] = (__bf16)v;
}

__global__ __launch_bounds__(256) void k_pack_batch(PackBatch b) {
  const PackJob& j = b.j[blockIdx.y];
  const long total = pack_job_elems(j);
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    switch (j.kind) {
      case PK_F32: pk_f32(j, e); break;
      case PK_X6: pk_x6(j, e); break;
      case PK_W6: pk_w6(j, e); break;
      case PK_DECONV_X6: pk_deconv_x6(j, e); break;
      case PK_HEAD_X6: pk_head_x6(j, e); break;
      case PK_DECONV_DGRAD_X6: pk_deconv_dgrad_x6(j, e); break;
      case PK_BF16: pk_bf16(j, e); break;
      default: static_cast<float*>(j.out)[e] = 0.f; break;
    }
  }
}

hipError_t pack_flush(PackBatch& b, hipStream_t s) {
  if (b.n == 0) return hipSuccess;
  long blocks = 1;
  for (int i = 0; i < b.n; ++i) blocks = std::max(blocks, (pack_job_elems(b.j[i]) + 255) / 256);
  hipLaunchKernelGGL(k_pack_batch, dim3((unsigned)std::min(blocks, 1024L), (unsigned)b.n), dim3(256),
                     0, s, b);
  b.n = 0;
  return hipGetLastError();
}

hipError_t pack_add(PackBatch& b, const PackJob& j, hipStream_t s) {
  if (b.n == kPackJobs) {
    hipError_t e = pack_flush(b, s);
    if (e != hipSuccess) return e;
  }
  b.j[b.n++] = j;
  return hipSuccess;
}

// a WView's element strides as the job's ints (false when one does not fit)
static bool pack_view(const WView& wv, PackJob& j) {
  const long lim = 1L << 31;
  if (wv.sK >= lim || wv.sN >= lim || wv.sT >= lim || wv.sZ >= lim) return false;
  j.w = wv.w + wv.off;
  j.sK = (int)wv.sK; j.sN = (int)wv.sN; j.sT = (int)wv.sT; j.sZ = (int)wv.sZ;
  j.taps = wv.taps; j.flip = wv.flip;
  return true;
}

PackJob pack_job_head_x6(const float* wa, const float* wb, void* out) {
  PackJob j{};
  j.kind = PK_HEAD_X6; j.w = wa; j.w2 = wb; j.out = out;
  return j;
}

PackJob pack_job_head_bwd_x6(const float* wa, const float* wb, void* out) {
  PackJob j{};
  j.kind = PK_HEAD_X6; j.w = wb; j.w2 = wa; j.out = out; j.flip = 1;  // Wb^T | Wa^T
  return j;
}

PackJob pack_job_deconv_x6(const float* w, void* out) {
  PackJob j{};
  j.kind = PK_DECONV_X6; j.w = w; j.out = out;
  return j;
}

PackJob pack_job_deconv_dgrad_x6(const float* w, void* out) {
  PackJob j{};
  j.kind = PK_DECONV_DGRAD_X6; j.w = w; j.out = out;
  return j;
}

bool pack_job_bf16(const WView& wv, int K, int nout, int ksize, void* out, PackJob& j) {
  j = PackJob{};
  const long st = bf16_stage_elems(nout, ksize), tot = bf16_pack_elems(K, nout, ksize);
  if (st < 0 || tot < 0 || tot >= (1L << 31) || !pack_view(wv, j)) return false;
  j.kind = PK_BF16; j.out = out; j.K = K; j.NOUT = nout;
  j.g0 = nout <= 48 ? 48 : 96; j.g1 = (int)st; j.g2 = ksize == 3; j.g3 = (int)tot;
  return true;
}

PackJob pack_job_zero(float* out, int n) {
  PackJob j{};
  j.kind = PK_ZERO; j.out = out; j.g0 = n;
  return j;
}

template <int NT, int MT>
static hipError_t run_x6(const FwdArgs& a, int nz, hipStream_t s) {
  using C = XCfg<NT, MT>;
  const int tx = (a.OW + C::TW - 1) / C::TW, ty = (a.OH + C::TH - 1) / C::TH;
  static const std::string kn = x6_kname("k_c3x6", NT, MT, -1);
  prof_kernel(kn.c_str());
  hipLaunchKernelGGL((k_c3x6<NT, MT>), dim3(tx * ty, a.N, nz), dim3(256), 0, s, a);
  return hipGetLastError();
}

// output channels per workgroup: 32, 48 or 96 (wider layers run zc-blocks of 48 or 96)
static int x6_np(int nout, int zc) {
  const int np = zc > 0 ? zc : nout;
  return np <= 32 ? 32 : (np <= 48 ? 48 : (np <= 96 ? 96 : 0));
}

long x6_pack_elems(int K, int nout, int zc) {
  const int np = x6_np(nout, zc);
  if (np == 0 || (zc > 0 && zc != np)) return -1;
  const int nz = zc > 0 ? (nout + zc - 1) / zc : 1;
  // 96- and 48-output blocks: room for the Winograd image (12 stages per chunk) as well
  const int spc = np == 96 || np == 48 ? 12 : 9;
  return (long)nz * ((K + 31) / 32) * spc * x6_wst(np);
}

// DN_X6_W6=1/0: 96- and 48-output-channel large-grid launches on the Winograd kernel or not
// (default DN_X6_W6_DEFAULT)
#ifndef DN_X6_W6_DEFAULT
#define DN_X6_W6_DEFAULT 1
#endif
static bool w6_enabled() {
  static const bool on = getenv("DN_X6_W6") ? atoi(getenv("DN_X6_W6")) != 0 : DN_X6_W6_DEFAULT != 0;
  return on;
}

int x6_image_mode(int N, int H, int W, int K, int nout, int zc, bool aligned) {
  if (!aligned) return 0;
  // k_c3w6 (8 x 16 tiles, two workgroups per CU) from one full round of resident workgroups
  const long t8 = (long)N * ((H + 7) / 8) * ((W + 15) / 16);
  const int nz = zc > 0 ? (nout + zc - 1) / zc : 1;
  // DN_W6_MIN_TILES: tuning probe for the smallest Winograd launch (default one full round)
  static const long min_t = getenv("DN_W6_MIN_TILES") ? atol(getenv("DN_W6_MIN_TILES")) : 512;
  const int np = x6_np(nout, zc);
  const bool w6 = w6_enabled() && (np == 96 || np == 48) && (zc == 0 ? nout == np : zc == np) &&
                  t8 * nz >= min_t;
  if (!w6 && !x6_pipelined(N, H, W, nout, zc)) return 0;
  return x6_tail_mode(K) | (w6 ? X6_W6 : 0);
}

int x6_tail_mode(int K) {
  const int r = K % 32;
  return r == 0 ? 0 : (r <= 4 ? 1 : (r <= 16 ? 2 : 0));
}

bool pack_job_x6(const WView& wv, int K, int nout, int zc, void* out, int mode, PackJob& j) {
  const long total = x6_pack_elems(K, nout, zc);
  const int tail = mode & 7;
  const bool w6 = (mode & X6_W6) != 0;
  const int npw = x6_np(nout, zc);
  if (total < 0 || wv.taps != 9 || (tail && tail != x6_tail_mode(K)) ||
      (w6 && ((npw != 96 && npw != 48) || (zc == 0 ? nout != npw : zc != npw))))
    return false;
  WView v = wv;
  if (zc > 0) v.sZ = (long)zc * wv.sN;  // block z = output channels [z*zc, z*zc + zc)
  j = PackJob{};
  if (!pack_view(v, j)) return false;
  j.kind = PK_X6; j.out = out;
  j.K = K; j.NOUT = zc > 0 ? zc : nout; j.g0 = x6_np(nout, zc); j.nch = (K + 31) / 32;
  j.nz = zc > 0 ? (nout + zc - 1) / zc : 1; j.zc = zc; j.ntot = nout; j.tail = tail;
  if (w6) j.kind = PK_W6;
  if (mode & X6_T1) {  // one live channel in the last chunk: k_c3w6's six-slot tail
    if (!w6 || tail != 1 || npw != 96 || K % 32 != 1) return false;
    j.tail = 3;
  }
  return true;
}

hipError_t launch_pack_x6(const WView& wv, int K, int nout, int zc, void* out, hipStream_t s,
                          int tail) {
  PackBatch b;
  PackJob j;
  if (!pack_job_x6(wv, K, nout, zc, out, tail, j)) return hipErrorInvalidValue;
  b.j[b.n++] = j;
  return pack_flush(b, s);
}

// Tile height 8/4 rows: the fewest rounds of resident workgroups, each weighed by its length
// (as pick_mt in conv.hip; per-tile efficiency of the shorter tiles from the halo overhead).
template <int NT>
static int x6_pick_mt(const FwdArgs& a, int nz) {
  const int mts[2] = {2, 1};
  const int occ[2] = {XCfg<NT, 2>::OCC, XCfg<NT, 1>::OCC};
  const double eff[2] = {1.0, 1.2};
  int mt = 1;
  double best = 1e30;
  for (int i = 0; i < 2; ++i) {
    const long blocks = (long)a.N * ((a.OH + 4 * mts[i] - 1) / (4 * mts[i])) * ((a.OW + 15) / 16) * nz;
    const long slots = 256L * occ[i];
    const double cost = (double)((blocks + slots - 1) / slots) * occ[i] * mts[i] * eff[i];
    if (cost < best - 1e-9) { best = cost; mt = mts[i]; }
  }
  return mt;
}

template <int NT>
static hipError_t run_x6p(const FwdArgs& a, int nz, hipStream_t s) {
  using C = PCfg<NT>;
  const int tx = (a.OW + C::TW - 1) / C::TW, ty = (a.OH + C::TH - 1) / C::TH;
  const dim3 grid(tx * ty, a.N, nz), block(C::WAVES * 64);
  // (labels as rocprofv3 prints the instantiations: SEL = false spelled out)
  static const std::string kn[3] = {x6_kmore(x6_kname("k_c3x6p", NT, 0, -1), "false"),
                                    x6_kmore(x6_kname("k_c3x6p", NT, 1, -1), "false"),
                                    x6_kmore(x6_kname("k_c3x6p", NT, 2, -1), "false")};
  prof_kernel(kn[a.x6_tail > 2 ? 0 : a.x6_tail].c_str());
  if (a.x6_tail == 1)
    hipLaunchKernelGGL((k_c3x6p<NT, 1>), grid, block, 0, s, a);
  else if (a.x6_tail == 2)
    hipLaunchKernelGGL((k_c3x6p<NT, 2>), grid, block, 0, s, a);
  else
    hipLaunchKernelGGL((k_c3x6p<NT, 0>), grid, block, 0, s, a);
  return hipGetLastError();
}

hipError_t launch_fwd_x6_sel(const FwdArgs& a, hipStream_t s) {
  using C = PCfg<6>;
  if (x6_np(a.NOUT, a.zc) != 96 || a.zc || a.K % 32 || a.x6_tail || !a.sel_rd ||
      a.out_layout != OUT_NHWC || a.epi != EPI_BIAS_ACT || (a.OH | a.OW) & 1 ||
      ((a.in_stride | a.in_off) & 3) || (long)C::IH * a.IWt * a.in_stride * 4 >= 0x7fffffffL)
    return hipErrorInvalidValue;
  // 32-row tiles (k_c3x6s), else the 16-row k_c3x6p<6,0,true>
  if ((long)SCfg::IH * a.IWt * a.in_stride * 4 < 0x7fffffffL) {
    const int tx = (a.OW + SCfg::TW - 1) / SCfg::TW, ty = (a.OH + SCfg::TH - 1) / SCfg::TH;
    prof_kernel("k_c3x6s");
    hipLaunchKernelGGL(k_c3x6s, dim3(tx * ty, a.N, 1), dim3(SCfg::WAVES * 64), 0, s, a);
    return hipGetLastError();
  }
  const int tx = (a.OW + C::TW - 1) / C::TW, ty = (a.OH + C::TH - 1) / C::TH;
  prof_kernel("k_c3x6p<6,0,true>");
  hipLaunchKernelGGL((k_c3x6p<6, 0, true>), dim3(tx * ty, a.N, 1), dim3(C::WAVES * 64), 0, s, a);
  return hipGetLastError();
}

bool x6_pipelined(int N, int H, int W, int nout, int zc) {
  const int nz = zc > 0 ? (nout + zc - 1) / zc : 1;
  return (long)N * ((H + 15) / 16) * ((W + 15) / 16) * nz >= 512;
}

// a.wp = the launch_pack_x6 image (a.wp_z = its per-block size when a.zc > 0); every epilogue
// and output layout of k_fwd
hipError_t launch_fwd_x6(const FwdArgs& a, hipStream_t s) {
  const int np = x6_np(a.NOUT, a.zc);
  if (np == 0 || (a.zc > 0 && a.zc != np)) return hipErrorInvalidValue;
  // a fused pool: the float4 epilogue of a tiled kernel, even sides
  if (a.pool_out && (a.epi != EPI_BIAS_ACT || a.out_layout != OUT_NHWC ||
                     ((a.out_stride | a.out_off | a.NOUT) & 3) || ((a.OH | a.OW) & 1)))
    return hipErrorInvalidValue;
  const int nz = a.zc > 0 ? (a.NOUT + a.zc - 1) / a.zc : 1;
  if (a.x6_tail & X6_W6) return launch_fwd_w6(a, s);  // a Winograd image (x6_image_mode)
  // large grids: the pipelined 16-row kernel (one workgroup per CU, >= 2 rounds of tiles)
  // the pipelined kernel addresses one tile's 18 input rows through a 32-bit buffer resource
  const bool aligned = ((a.in_stride | a.in_off | a.K) & 3) == 0 &&
                       (long)PCfg<6>::IH * a.IWt * a.in_stride * 4 < 0x7fffffffL;
  auto pipe = [&]() {
    return np == 32 ? run_x6p<2>(a, nz, s) : (np == 48 ? run_x6p<3>(a, nz, s) : run_x6p<6>(a, nz, s));
  };
  // large grids: the two-workgroups-per-CU kernel where it measured faster (48 / 32 output
  // channels: -6..-11 %; a 4-channel tail chunk: -3.6 %), else the one-per-CU kernel (equal
  // within noise on the 96-channel shapes; tools/x6_micro.py)
  const bool half_fits = (long)HCfg<6>::IH * a.IWt * a.in_stride * 4 < 0x7fffffffL;
  const bool half = half_fits && (np <= 48 || a.x6_tail == 1);
  // 48 / 32 output channels: 16-row tiles (4 rows per wave, twice the MFMAs per operand read
  // and per stage barrier) when they fill two rounds of resident workgroups
  const long tiles16 = (long)a.N * nz * ((a.OH + 15) / 16) * ((a.OW + 15) / 16);
  const bool h4 = np <= 48 && tiles16 >= 1024 &&
                  (long)HCfg<3, 4>::IH * a.IWt * a.in_stride * 4 < 0x7fffffffL;
  auto run = [&]() {
    if (half && h4) return np == 32 ? run_x6h<2, 4>(a, nz, s) : run_x6h<3, 4>(a, nz, s);
    if (half)
      return np == 32 ? run_x6h<2>(a, nz, s) : (np == 48 ? run_x6h<3>(a, nz, s) : run_x6h<6>(a, nz, s));
    return pipe();
  };
  if (a.x6_tail) {  // tail-packed last chunk: only the pipelined kernels read it
    if (!aligned || a.x6_tail != x6_tail_mode(a.K)) return hipErrorInvalidValue;
    return run();
  }
  if (x6_pipelined(a.N, a.OH, a.OW, a.NOUT, a.zc) && aligned) return run();
  // (a fused pool needs an even number of tile rows per wave: MT = 2)
  const bool pool = a.pool_out != nullptr;
  // small grids: k_c3x6h with the 3-slot weight ring where the shape allows (float4 rows; two
  // workgroups per CU: MT = 1 at 96 channels); DN_X6_RING3=0 keeps k_c3x6
  static const bool ring3 = !getenv("DN_X6_RING3") || atoi(getenv("DN_X6_RING3")) != 0;
  if (ring3 && aligned && half_fits) {
    if (np == 96 && !pool) return run_x6h3<6, 1>(a, nz, s);
    if (np == 48) return pool || x6_pick_mt<3>(a, nz) == 2 ? run_x6h3<3, 2>(a, nz, s) : run_x6h3<3, 1>(a, nz, s);
    if (np == 32) return pool || x6_pick_mt<2>(a, nz) == 2 ? run_x6h3<2, 2>(a, nz, s) : run_x6h3<2, 1>(a, nz, s);
  }
  if (np == 32)
    return pool || x6_pick_mt<2>(a, nz) == 2 ? run_x6<2, 2>(a, nz, s) : run_x6<2, 1>(a, nz, s);
  if (np == 48)
    return pool || x6_pick_mt<3>(a, nz) == 2 ? run_x6<3, 2>(a, nz, s) : run_x6<3, 1>(a, nz, s);
  return pool || x6_pick_mt<6>(a, nz) == 2 ? run_x6<6, 2>(a, nz, s) : run_x6<6, 1>(a, nz, s);
}


// ------------------------------------------------------------------------------------
// 3x3 weight gradient at fp32 accuracy on the bf16 matrix cores (k_wgrad3s: 96 or 48 output
// channels).  GEMM M = output channels, N = input channels x 9 taps, K = pixels.  Each 32-pixel
// K stage of the gradient G [px][GS] and of the input X [(sh+2) rows][sw+2][XS] (halo included;
// GS / XS = channels + 4, so lane groups 8 pixels apart fall on opposite bank halves) is copied
// by per-lane global_load_lds into double-buffered LDS (padding slots load zeros), one barrier
// per stage -- no staging registers.  The split happens at the operand read: lane group lg's 8 K
// values are the stage pixels 8lg .. 8lg+7, read as fp32 and split into three bf16 pieces in
// registers.  For X that makes the three horizontal taps of a kernel row sliding windows of ONE
// 10-pixel read: kx = 0 and 2 are whole-register offsets of its split pieces, kx = 1 a 16-bit
// funnel shift.  Each (output fragment, tap) runs the six piece products of x6_block from zero,
// added to the fp32 accumulators.  Wave (wm, wn): MFW output-channel fragments x 16 input
// channels x 9 taps; the bias gradient is the G pieces against a ones fragment.
// ------------------------------------------------------------------------------------
template <int CO_FR, int WM, int WN>
struct Ws3Cfg {
  static constexpr int COUT = 16 * CO_FR, MFW = CO_FR / WM, CIB = 16 * WN;
  static constexpr int NW = WM * WN, NTHR = 64 * NW;
  static constexpr int PC = 32, GS = COUT + 4, XS = CIB + 4;
  static constexpr int XPIX = 3 * 34;                              // widest stage: 3 rows x 34
  static constexpr int LGF = (PC * GS + 255) / 256 * 256;          // G floats per stage
  static constexpr int LXF = (XPIX * XS + 255) / 256 * 256;        // X floats per stage
  static constexpr int LGP = LGF / 256, LXP = LXF / 256;           // 1 KiB DMA pieces
  static constexpr int LBUF = LGF + LXF;
};

// (the 96-output layers and the encoder's 48-output ones run k_wgrad3p / k_wgrad3q,
// wgrad_x6p.hip; this kernel serves the output-channel-blocked launches of ImprovedUNet)
template <int CO_FR, int WM, int WN, int SWL>
__global__ __launch_bounds__(64 * WM * WN, 2) void k_wgrad3s(WgradArgs a0) {
  using C = Ws3Cfg<CO_FR, WM, WN>;
  constexpr int MFW = C::MFW;
  const WgradArgs a = wg_block(a0);
  __shared__ __attribute__((aligned(16))) float lds[2 * C::LBUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int li = lane & 15, lg = lane >> 4;
  const int ci0 = blockIdx.y * C::CIB;
  // K stage = 32 pixels: one row segment of 32, or 32/sw whole rows of sw >= 8 pixels
  constexpr int sw = 1 << SWL, sh = C::PC >> SWL, xw = sw + 2;
  static_assert(sw >= 8, "a lane group's 8 K pixels lie in one stage row");
  const int ux = (a.KW + sw - 1) / sw, uy = (a.KH + sh - 1) / sh;
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
  auto glds = [](const float* g, float* l) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)l, 16, 0, 0);
  };
  // stage u = (image n, stage row block iy, column block ix), decoded incrementally (no 64-bit
  // divisions per stage)
  struct Pos { int n, iy, ix; };
  auto pos_of = [&](long u) {
    Pos q;
    q.n = (int)(u / ((long)uy * ux));
    const int rem = (int)(u - (long)q.n * uy * ux);
    q.iy = rem / ux; q.ix = rem - q.iy * ux;
    return q;
  };
  auto next = [&](Pos q) {
    if (++q.ix == ux) { q.ix = 0; if (++q.iy == uy) { q.iy = 0; ++q.n; } }
    return q;
  };
  // images whose sides are whole stage blocks (every UNet level): the per-lane parts of the DMA
  // addresses are stage-invariant and precomputed; only the halo edges need a per-stage test
  const bool exact = a.KW % sw == 0 && a.KH % sh == 0;
  constexpr int JG = (C::LGP + C::NW - 1) / C::NW, JX = (C::LXP + C::NW - 1) / C::NW;
  int goff[JG], xoff[JX], xedge[JX];
#pragma unroll
  for (int j = 0; j < JG; ++j) {
    const int idx = (wave + j * C::NW) * 256 + lane * 4;
    const int px = idx / C::GS, co = idx - px * C::GS;
    goff[j] = (px < C::PC && co < a.Cout) ? ((px >> SWL) * a.KW + (px & (sw - 1))) * a.g_stride + co : -1;
  }
#pragma unroll
  for (int j = 0; j < JX; ++j) {
    const int idx = (wave + j * C::NW) * 256 + lane * 4;
    const int px = idx / C::XS, q = idx - px * C::XS;
    const int yy = px / xw, xx = px - yy * xw;
    const bool ok = px < (sh + 2) * xw && q < C::CIB && ci0 + q < a.Cin;
    xoff[j] = ((yy - 1) * a.KW + xx - 1) * a.x_stride + ci0 + q;
    // halo edges: bit 0 top row, 1 bottom row, 2 left column, 3 right column; bit 4 unused slot
    xedge[j] = (yy == 0) | ((yy == sh + 1) << 1) | ((xx == 0) << 2) | ((xx == sw + 1) << 3) | ((!ok) << 4);
  }
  auto issue = [&](Pos q, float* buf) {
    const int py0 = q.iy * sh, px0 = q.ix * sw;
    const float* gb = a.g + (long)q.n * a.KH * a.KW * a.g_stride + a.g_off;
    const float* xb = a.x + (long)q.n * a.KH * a.KW * a.x_stride + a.x_off;
    if (exact) {
      const float* gs = gb + ((long)py0 * a.KW + px0) * a.g_stride;
      const float* xs = xb + ((long)py0 * a.KW + px0) * a.x_stride;
      const int emask = (py0 == 0) | ((py0 + sh >= a.KH) << 1) | ((px0 == 0) << 2) |
                        ((px0 + sw >= a.KW) << 3) | (1 << 4);
#pragma unroll
      for (int j = 0; j < JG; ++j) {
        const int p = wave + j * C::NW;
        if (p < C::LGP) glds(goff[j] >= 0 ? gs + goff[j] : a.zeros, buf + p * 256);
      }
#pragma unroll
      for (int j = 0; j < JX; ++j) {
        const int p = wave + j * C::NW;
        if (p < C::LXP) glds((xedge[j] & emask) ? a.zeros : xs + xoff[j], buf + C::LGF + p * 256);
      }
      return;
    }
    for (int p = wave; p < C::LGP; p += C::NW) {
      const int idx = p * 256 + lane * 4;
      const int px = idx / C::GS, co = idx - px * C::GS;
      const int gy = py0 + (px >> SWL), gx = px0 + (px & (sw - 1));
      const float* src = (px < C::PC && co < a.Cout && gy < a.KH && gx < a.KW)
                             ? gb + ((long)gy * a.KW + gx) * a.g_stride + co : a.zeros;
      glds(src, buf + p * 256);
    }
    const int xpix = (sh + 2) * xw;
    for (int p = wave; p < C::LXP; p += C::NW) {
      const int idx = p * 256 + lane * 4;
      const int px = idx / C::XS, q4 = idx - px * C::XS;
      const int yy = px / xw, xx = px - yy * xw;
      const int gy = py0 - 1 + yy, gx = px0 - 1 + xx, ci = ci0 + q4;
      const bool ok = px < xpix && q4 < C::CIB && gy >= 0 && gy < a.KH && gx >= 0 && gx < a.KW &&
                      ci < a.Cin;
      const float* src = ok ? xb + ((long)gy * a.KW + gx) * a.x_stride + ci : a.zeros;
      glds(src, buf + C::LGF + p * 256);
    }
  };
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;
  // this lane group's 8 K pixels: stage row pr0, columns pc0 .. pc0 + 7
  const int pr0 = (8 * lg) >> SWL, pc0 = (8 * lg) & (sw - 1);

  Pos pn = pos_of(u_beg);
  if (u_beg < u_end) issue(pn, lds);
  __syncthreads();
  for (long u = u_beg; u < u_end; ++u) {
    const int cb = (int)((u - u_beg) & 1);
    const float* lgs = lds + cb * C::LBUF;
    const float* lxs = lgs + C::LGF;
    pn = next(pn);
    if (u + 1 < u_end) issue(pn, lds + (cb ^ 1) * C::LBUF);
    // A: the wave's MFW gradient fragments
    bf16x8 av[3][MFW];
#pragma unroll
    for (int i = 0; i < MFW; ++i) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = lgs[(8 * lg + j) * C::GS + (wm * MFW + i) * 16 + li];
      split3x8(v, av[0][i], av[1][i], av[2][i]);
#pragma unroll
      for (int p = 0; p < 3; ++p) asm volatile("" : "+v"(av[p][i]));  // kept, not re-split per tap
    }
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      // the kernel row's 10-pixel window, split once: P[plane][d] = pieces of pixels 2d, 2d+1
      unsigned P[3][5];
      {
      const float* xr = lxs + ((pr0 + ky) * xw + pc0) * C::XS + wn * 16 + li;
      float w[10];
#pragma unroll
      for (int m = 0; m < 10; ++m) w[m] = xr[m * C::XS];
#pragma unroll
      for (int d = 0; d < 5; ++d) {
        split3x2(w[2 * d], w[2 * d + 1], P[0][d], P[1][d], P[2][d]);
      }
      }
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        bf16x8 bv[3][1];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          u32x4_t q;
#pragma unroll
          for (int d = 0; d < 4; ++d)
            q[d] = kx == 0 ? P[pl][d]
                           : (kx == 2 ? P[pl][d + 1] : __builtin_amdgcn_alignbit(P[pl][d + 1], P[pl][d], 16));
          bv[pl][0] = __builtin_bit_cast(bf16x8, q);
        }
        const int t = 3 * ky + kx;
        x6_block<MFW, 1, 1>(acc[t], av, bv);
        // the tap's running sums materialised here (a deferred add keeps its MFMA results live)
#pragma unroll
        for (int i = 0; i < MFW; ++i) asm volatile("" : "+v"(acc[t][i][0]));
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
    __syncthreads();  // next stage landed (vmcnt(0)); everyone done with this buffer
  }

  float* slab = a.slab + (long)blockIdx.x * a.slab_stride;
  const int ci = ci0 + wn * 16 + li;
  const int cot = a.cout_total ? a.cout_total : a.Cout;
#pragma unroll
  for (int i = 0; i < MFW; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = (wm * MFW + i) * 16 + 4 * lg + r;
        if (co < a.Cout && ci < a.Cin)
          slab[((long)(a.co_base + co) * a.cin_total + a.ci_base + ci) * 9 + t] = acc[t][i][0][r];
      }
  if (do_bias && li == 0) {
#pragma unroll
    for (int i = 0; i < MFW; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = (wm * MFW + i) * 16 + 4 * lg + r;
        if (co < a.Cout) slab[(long)cot * a.cin_total * 9 + a.co_base + co] = accb[i][0][r];
      }
  }
}

// 96 or 48 output channels, Cin >= 32, rows >= 8 wide, 16-byte aligned NHWC views whose
// channel quads stay inside each pixel (the staging of k_wgrad3)
bool wgrad3_x6_ok(const WgradArgs& a) {
  if ((a.Cout != 96 && a.Cout != 48) || a.Cin < 32 || a.KW < 8 || !a.zeros || a.zc > 0) return false;
  if ((a.g_stride | a.g_off | a.x_stride | a.x_off) & 3) return false;
  return a.x_off + ((a.Cin + 3) & ~3) <= a.x_stride;
}

// two workgroups per CU: splits x input-channel blocks fill one round of 512
int wgrad_splits_x6(const WgradArgs& a, int splits) {
  if (!wgrad3_x6_ok(a)) return splits;
  const int cib = a.Cout == 96 ? 32 : 48;
  const int cap = 512 / ((a.Cin + cib - 1) / cib);
  return splits < cap ? splits : (cap < 1 ? 1 : cap);
}

template <int CO_FR, int WM, int WN>
static hipError_t run_wgrad3s(const WgradArgs& a, int splits, hipStream_t s, int nz = 1) {
  using C = Ws3Cfg<CO_FR, WM, WN>;
  const dim3 grid(splits, (a.Cin + C::CIB - 1) / C::CIB, nz), block(C::NTHR);
  static const std::string kn[3] = {x6_kmore(x6_kname("k_wgrad3s", CO_FR, WM, WN), "3"),
                                    x6_kmore(x6_kname("k_wgrad3s", CO_FR, WM, WN), "4"),
                                    x6_kmore(x6_kname("k_wgrad3s", CO_FR, WM, WN), "5")};
  prof_kernel(kn[a.KW >= 32 ? 2 : (a.KW >= 16 ? 1 : 0)].c_str());
  if (a.KW >= 32) hipLaunchKernelGGL((k_wgrad3s<CO_FR, WM, WN, 5>), grid, block, 0, s, a);
  else if (a.KW >= 16) hipLaunchKernelGGL((k_wgrad3s<CO_FR, WM, WN, 4>), grid, block, 0, s, a);
  else hipLaunchKernelGGL((k_wgrad3s<CO_FR, WM, WN, 3>), grid, block, 0, s, a);
  return hipGetLastError();
}

hipError_t launch_wgrad3_x6(const WgradArgs& a, int splits, hipStream_t s) {
  if (!wgrad3_x6_ok(a)) return hipErrorInvalidValue;
  if (wgrad3p_ok(a)) return launch_wgrad3p(a, splits, s, 1);  // k_wgrad3p (96) / k_wgrad3q (48)
  return a.Cout == 96 ? run_wgrad3s<6, 2, 2>(a, splits, s) : run_wgrad3s<3, 1, 3>(a, splits, s);
}

// The blocked 3x3 weight gradient (the ImprovedUNet executor: any Cout, output-channel blocks of
// 96 / 48 / 32 over blockIdx.z, as launch_gwgrad) on the bf16x6 kernel.  32-wide blocks (the RDB
// growth convs, the 24-channel level) take 32 / 48 / 64 input channels per workgroup, whichever
// pads Cin least; every block of a layer uses the same split count.
static int gw6_block(int cout) { return cout <= 32 ? 32 : (cout <= 48 ? 48 : 96); }
static int gw6_cib(int cb, int Cin) {
  if (cb == 96) return 32;
  if (cb == 48) return 48;
  int best = 48;
  long pad = 1L << 30;
  for (int t : {64, 48, 32}) {
    const long p = (long)(Cin + t - 1) / t * t;
    if (p < pad) { pad = p; best = t; }
  }
  return best;
}

bool gwgrad_x6_ok(const WgradArgs& a) {
  if (a.Cin < 16 || a.KW < 8 || !a.zeros || a.zc > 0) return false;
  if ((a.g_stride | a.g_off | a.x_stride | a.x_off) & 3) return false;
  return a.x_off + ((a.Cin + 3) & ~3) <= a.x_stride && a.g_off + ((a.Cout + 3) & ~3) <= a.g_stride;
}

// split count of the x6 launch: at most `splits` (what the slab was sized for), and splits x
// input-channel blocks x output blocks within one round of 512 resident workgroups
int gwgrad_x6_splits(const WgradArgs& a, int splits) {
  const int cb = gw6_block(a.Cout), nz = (a.Cout + cb - 1) / cb;
  const int cib = gw6_cib(cb, a.Cin);
  const int cap = 512 / (nz * ((a.Cin + cib - 1) / cib));
  return splits < cap ? splits : (cap < 1 ? 1 : cap);
}

hipError_t launch_gwgrad_x6(const WgradArgs& a0, int splits, hipStream_t s) {
  if (!gwgrad_x6_ok(a0)) return hipErrorInvalidValue;
  const int cb = gw6_block(a0.Cout), nz = (a0.Cout + cb - 1) / cb;
  WgradArgs a = a0;
  a.zc = cb;
  a.cout_total = a0.Cout;
  a.co_base = 0;
  if (cb == 96 && wgrad3p_ok(a)) return launch_wgrad3p(a, splits, s, nz);
  if (cb == 96) return run_wgrad3s<6, 2, 2>(a, splits, s, nz);
  if (cb == 48) return run_wgrad3s<3, 1, 3>(a, splits, s, nz);
  const int ct = gw6_cib(cb, a.Cin);
  if (ct == 64) return run_wgrad3s<2, 1, 4>(a, splits, s, nz);
  if (ct == 32) return run_wgrad3s<2, 1, 2>(a, splits, s, nz);
  return run_wgrad3s<2, 1, 3>(a, splits, s, nz);
}

// ------------------------------------------------------------------------------------
// The nin head (nin_a -> nin_b -> nin_c, arch_unet.py:186-190, 257-259) on the activated
// dec_conv1b output, with the two 96x96 1x1 GEMMs in the bf16x6 arithmetic.  As in k_nin_head
// the tile lives in the 16x16 MFMA C/D map (rows = channels, columns = 16 pixels), which is
// directly the B operand of the next GEMM: for K block b (32 channels) lane group g supplies
// channels {32b + 4g + r, 32b + 16 + 4g + r} (r < 4) = registers 2b and 2b+1 of its tile
// fragment, split into three bf16x8 planes in registers.  The weight images are pre-split
// in the same permuted K order (pk_head_x6: [plane][b][out][32], 64-B rows, quads
// swizzled) and DMA'd into LDS once per workgroup (54 KiB per layer).
// ------------------------------------------------------------------------------------
// Persistent: one 8-wave workgroup per CU keeps both images (108 KiB) and the biases / nin_c
// weights in LDS for the whole launch; wave-tiles are single 16-pixel rows, taken in a wave-
// strided loop, the next row's input loaded into registers while the current one computes
// (the images are read from L2 once per CU, not once per tile).
// SAVE: na / nb written for the backward; PAIR: the input is a pair image (hd.rd); B1: plain
// bf16 products (the bf16 base's autocast arithmetic): the input rounded to bf16, the images'
// leading planes (the weights rounded to bf16), one MFMA per block chained in fp32
// IBF (with B1): the input activation is stored as bf16 (FwdArgs::in_bf16), 8 bytes per lane and
// 4 channels, taken as the operand without conversion
template <bool SAVE, bool PAIR, bool B1 = false, bool IBF = false>
__global__ __launch_bounds__(512, 1) void k_nin_head_x6(FwdArgs a, HeadArgs hd, const __bf16* wimg,
                                                      int nwt) {
  static_assert(!IBF || B1, "bf16 input only in the plain-bf16 head");
  __shared__ __attribute__((aligned(16))) __bf16 lw[2 * X6_HEAD_BF];
  __shared__ __attribute__((aligned(16))) float lb[2 * 96 + X6_HEAD_OCMAX * 97];  // ba|bb|wc|bc
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, lg = lane >> 4;
  for (int q = wave; q < 2 * X6_HEAD_BF * 2 / 1024; q += 8)
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(wimg + q * 512 + lane * 8),
        (__attribute__((address_space(3))) void*)(lw + q * 512), 16, 0, 0);
  for (int e = threadIdx.x; e < 2 * 96 + hd.oc * 97; e += 512) {
    float v;
    if (e < 96) v = hd.ba[e];
    else if (e < 192) v = hd.bb[e - 96];
    else if (e < 192 + hd.oc * 96) v = hd.wc[e - 192];
    else v = hd.bc[e - 192 - hd.oc * 96];
    lb[e] = v;
  }
  const float* lbc = lb + 192 + hd.oc * 96;
  const int tiles_x = (a.OW + 15) / 16;
  const int wstride = gridDim.x * 8;
  // per-row buffer resources, out-of-range offsets instead of branches (see k_deconv_x6)
  const long in_row = (long)a.IWt * a.in_stride;
  auto load = [&](int wt, f32x4 (&v)[6], int& rd) {
    const int n = wt / (a.OH * tiles_x), r = wt - n * a.OH * tiles_x;
    const int gy = r / tiles_x, gx = (r - gy * tiles_x) * 16 + li;
    const bool ok = wt < nwt && gx < a.OW;
    constexpr int EB = IBF ? 2 : 4;  // bytes per stored activation
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned char*>(reinterpret_cast<const unsigned char*>(a.in) +
                                   (((long)n * a.IHt + gy) * in_row + a.in_off) * EB),
        (short)0, (int)(in_row * EB), 0x00020000);
    const int off = ok ? (gx * a.in_stride + 4 * lg) * EB : 0x7fffffff;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      if constexpr (IBF) {  // bf16 bits of channels 16q + 4lg .. +3 in v[q][0..1]
        typedef unsigned u32x2h __attribute__((ext_vector_type(2)));
        const u32x2h d = __builtin_bit_cast(u32x2h, __builtin_amdgcn_raw_buffer_load_b64(rs, off + 32 * q, 0, 0));
        v[q] = f32x4{__uint_as_float(d[0]), __uint_as_float(d[1]), 0.f, 0.f};
      } else {
        v[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 64 * q, 0, 0));
      }
    }
    if constexpr (PAIR) {  // the cell's pair choice, loaded with the row (no wait of its own later)
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<unsigned char*>(hd.rd + ((long)n * a.OH + gy) * (a.OW / 2)), (short)0,
          a.OW / 2, 0x00020000);
      rd = __builtin_amdgcn_raw_buffer_load_b8(rr, ok ? gx >> 1 : 0x7fffffff, 0, 0);
    }
  };
  auto bias_act = [](f32x4& v, float4 b) {
    v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * 0.2f;
  };
  auto save = [&](float* dst, long row, int off, const f32x4& v, int q) {  // 16 px x 96 ch
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst + row * a.OW * 96, (short)0,
                                                                        a.OW * 96 * 4, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rs, off + 64 * q, 0, 0);
  };
  // out = W (LDS image at `img`) x in, three 32-channel K blocks of six split products each
  // (INB: `in` holds bf16 bits as loaded by load() under IBF)
  auto gemm96 = [&](auto inb_tag, const __bf16* img, const f32x4 (&in)[6], f32x4 (&out)[6][1]) {
    constexpr bool INB = decltype(inb_tag)::value;
#pragma unroll
    for (int f = 0; f < 6; ++f) out[f][0] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      bf16x8 xv[3][1];
      const float v8[8] = {in[2 * b][0], in[2 * b][1], in[2 * b][2], in[2 * b][3],
                           in[2 * b + 1][0], in[2 * b + 1][1], in[2 * b + 1][2], in[2 * b + 1][3]};
      if constexpr (B1) {
        if constexpr (INB) {
          const u32x4_t d = {__float_as_uint(in[2 * b][0]), __float_as_uint(in[2 * b][1]),
                             __float_as_uint(in[2 * b + 1][0]), __float_as_uint(in[2 * b + 1][1])};
          xv[0][0] = __builtin_bit_cast(bf16x8, d);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) xv[0][0][j] = (__bf16)v8[j];
        }
#pragma unroll
        for (int f = 0; f < 6; ++f) {
          const int row = b * 96 + f * 16 + li;
          const bf16x8 w0 = *reinterpret_cast<const bf16x8*>(img + row * 32 + x6_swz(row, lg) * 8);
          out[f][0] = mfma_bf16(w0, xv[0][0], out[f][0]);
        }
        continue;
      }
      split3x8(v8, xv[0][0], xv[1][0], xv[2][0]);
      bf16x8 wv[3][6];
#pragma unroll
      for (int f = 0; f < 6; ++f) {
        const int row = b * 96 + f * 16 + li;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          wv[pl][f] = *reinterpret_cast<const bf16x8*>(img + (pl * 3 * 96 + row) * 32 + x6_swz(row, lg) * 8);
      }
      x6_block<6, 1, 1>(out, wv, xv);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // one wave-tile; two register sets (xa, xb) alternate so that the next tile's loads are in
  // flight while this one computes and no copy forces a wait for them (or for the stores)
  auto tile = [&](int wt, const f32x4 (&xin)[6], int rd) {
    const int n = wt / (a.OH * tiles_x), r = wt - n * a.OH * tiles_x;
    const int gy = r / tiles_x, gx = (r - gy * tiles_x) * 16 + li;
    const bool ok = gx < a.OW;
    const long row = (long)n * a.OH + gy;
    const int soff = ok ? (gx * 96 + 4 * lg) * 4 : 0x7fffffff;
    f32x4 u[6][1], h[6];
    gemm96(std::integral_constant<bool, IBF>{}, lw, xin, u);  // nin_a
#pragma unroll
    for (int f = 0; f < 6; ++f) {
      bias_act(u[f][0], *reinterpret_cast<const float4*>(lb + f * 16 + 4 * lg));
      h[f] = u[f][0];
    }
    if constexpr (SAVE)
#pragma unroll
      for (int f = 0; f < 6; ++f) save(hd.na, row, soff, h[f], f);
    gemm96(std::false_type{}, lw + X6_HEAD_BF, h, u);  // nin_b
#pragma unroll
    for (int f = 0; f < 6; ++f) {
      bias_act(u[f][0], *reinterpret_cast<const float4*>(lb + 96 + f * 16 + 4 * lg));
      if constexpr (SAVE) save(hd.nb, row, soff, u[f][0], f);
    }
    // nin_c (fp32 VALU): per-lane partial over its 24 channels, then across the lane groups;
    // lane group 0 stores (the others get an out-of-range offset)
    // PAIR: pair image pixel (gy, gx) -> pixel pair[rd][gx & 1] of cell (gy, gx / 2), i.e. y's
    // rows 2gy, 2gy + 1
    int yoff = 0x7fffffff;
    if (lg == 0 && ok) {
      if constexpr (PAIR) {
        constexpr unsigned kPair = 0xB721ED84u;
        const int k = (kPair >> (4 * (rd & 7) + 2 * (gx & 1))) & 3;
        yoff = ((k >> 1) * a.OW + (gx & ~1) + (k & 1)) * 4;
      } else {
        yoff = gx * 4;
      }
    }
    constexpr int YR = PAIR ? 2 : 1;  // y rows per wave-tile
    for (int o = 0; o < hd.oc; ++o) {
      float t = 0.f;
#pragma unroll
      for (int f = 0; f < 6; ++f) {
        const float4 w = *reinterpret_cast<const float4*>(lb + 192 + o * 96 + f * 16 + 4 * lg);
        t = fmaf(w.x, u[f][0][0], t); t = fmaf(w.y, u[f][0][1], t);
        t = fmaf(w.z, u[f][0][2], t); t = fmaf(w.w, u[f][0][3], t);
      }
      t += __shfl_xor(t, 16);
      t += __shfl_xor(t, 32);
      const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
          hd.y + (((long)n * hd.oc + o) * YR * a.OH + YR * gy) * a.OW, (short)0, YR * a.OW * 4,
          0x00020000);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, t + lbc[o]), ry, yoff, 0, 0);
    }
  };
  int wt = blockIdx.x * 8 + wave;
  f32x4 xa[6], xb[6];
  int ra = 0, rb = 0;
  load(wt, xa, ra);
  __syncthreads();  // images, biases and nin_c weights landed
  for (; wt < nwt; wt += 2 * wstride) {
    load(wt + wstride, xb, rb);
    tile(wt, xa, ra);
    if (wt + wstride >= nwt) break;
    load(wt + 2 * wstride, xa, ra);
    tile(wt + wstride, xb, rb);
  }
}


// ------------------------------------------------------------------------------------
// Backward of the fused head in the bf16x6 arithmetic (k_head_bwd's products on the fp32
// matrix cores, arch_unet.py:186-190 differentiated):
//   g_nb = leaky'(nb) * (Wc^T dy)      (fp32 VALU, K = oc, nin_c's weights in LDS)
//   g_na = leaky'(na) * (Wb^T g_nb)    (bf16x6 GEMM, image Wb^T)
//   g_d1b = leaky'(d1b) * (Wa^T g_na)  (bf16x6 GEMM, image Wa^T)
// The tile stays in the MFMA C/D map (rows = channels, columns = 16 pixels), which is the B
// operand of the next GEMM as in k_nin_head_x6; the transposed images (pk_head_x6 with flip) are
// DMA'd into LDS once per workgroup.  One 8-wave workgroup per CU walks 16-pixel wave-tiles of
// the flattened pixel range; a tile's nb / dy / na / d1b loads are issued together at its start
// (the other wave on the SIMD computes meanwhile).  Every 16-pixel tile addresses its rows
// through its own buffer resource (pixel ranges beyond 2 GiB, out-of-range lanes read zeros and
// drop their stores).
// ------------------------------------------------------------------------------------
template <int OCM>  // nin_c outputs at most (registers of dy)
__global__ __launch_bounds__(512, 1) void k_head_bwd_x6(HeadBwdArgs h, const __bf16* wimg, long nwt) {
  __shared__ __attribute__((aligned(16))) __bf16 lw[2 * X6_HEAD_BF];
  __shared__ __attribute__((aligned(16))) float lc[X6_HEAD_OCMAX * 96];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, lg = lane >> 4;
  for (int q = wave; q < 2 * X6_HEAD_BF * 2 / 1024; q += 8)
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(wimg + q * 512 + lane * 8),
        (__attribute__((address_space(3))) void*)(lw + q * 512), 16, 0, 0);
  for (int e = threadIdx.x; e < h.oc * 96; e += 512) lc[e] = h.wc[e];
  __syncthreads();
  auto rsrc = [&](const float* base, long px0, int npx_t) {  // 16 pixels x 96 channels
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base + px0 * 96), (short)0,
                                             npx_t * 96 * 4, 0x00020000);
  };
  auto mask = [](f32x4& v, const f32x4& m) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = m[r] > 0.f ? v[r] : v[r] * 0.2f;
  };
  // out = W (LDS image at `img`) x in: three 32-channel K blocks of six split products each
  // (k_nin_head_x6's gemm96)
  auto gemm96 = [&](const __bf16* img, const f32x4 (&in)[6], f32x4 (&out)[6][1]) {
#pragma unroll
    for (int f = 0; f < 6; ++f) out[f][0] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      bf16x8 xv[3][1];
      const float v8[8] = {in[2 * b][0], in[2 * b][1], in[2 * b][2], in[2 * b][3],
                           in[2 * b + 1][0], in[2 * b + 1][1], in[2 * b + 1][2], in[2 * b + 1][3]};
      split3x8(v8, xv[0][0], xv[1][0], xv[2][0]);
      bf16x8 wv[3][6];
#pragma unroll
      for (int f = 0; f < 6; ++f) {
        const int row = b * 96 + f * 16 + li;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          wv[pl][f] = *reinterpret_cast<const bf16x8*>(img + (pl * 3 * 96 + row) * 32 + x6_swz(row, lg) * 8);
      }
      x6_block<6, 1, 1>(out, wv, xv);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  const int loff = (li * 96 + 4 * lg) * 4;  // lane's bytes within a tile row set
  for (long wt = (long)blockIdx.x * 8 + wave; wt < nwt; wt += (long)gridDim.x * 8) {
    const long px0 = wt * 16;
    const int npx_t = h.npx - px0 < 16 ? (int)(h.npx - px0) : 16;
    const bool ok = li < npx_t;
    const int off = ok ? loff : 0x7fffffff;
    const __amdgpu_buffer_rsrc_t rnb = rsrc(h.nb, px0, npx_t), rna = rsrc(h.na, px0, npx_t),
                                 rd1 = rsrc(h.d1b, px0, npx_t);
    f32x4 nb[6], na[6], d1[6];
#pragma unroll
    for (int q = 0; q < 6; ++q)
      nb[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rnb, off + 64 * q, 0, 0));
    float dy[OCM];
    const __amdgpu_buffer_rsrc_t rdy = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(h.dy + px0 * h.dy_stride), (short)0, npx_t * h.dy_stride * 4, 0x00020000);
#pragma unroll
    for (int o = 0; o < OCM; ++o)
      if (o < h.oc)
        dy[o] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                              rdy, ok ? (li * h.dy_stride + o) * 4 : 0x7fffffff, 0, 0));
#pragma unroll
    for (int q = 0; q < 6; ++q)
      na[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rna, off + 64 * q, 0, 0));
    // g_nb (K = oc, k_head_bwd's order)
    f32x4 t[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) t[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int o = 0; o < OCM; ++o) {
      if (o >= h.oc) break;
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        const float4 w = *reinterpret_cast<const float4*>(lc + o * 96 + q * 16 + 4 * lg);
        t[q][0] = fmaf(w.x, dy[o], t[q][0]); t[q][1] = fmaf(w.y, dy[o], t[q][1]);
        t[q][2] = fmaf(w.z, dy[o], t[q][2]); t[q][3] = fmaf(w.w, dy[o], t[q][3]);
      }
    }
    // (h.g_nb null: k_head_wgrad_x6 recomputes g_nb from dy and nb, nothing stores it)
    const __amdgpu_buffer_rsrc_t wnb = rsrc(h.g_nb ? h.g_nb : h.nb, px0, h.g_nb ? npx_t : 0);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      mask(t[q], nb[q]);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, t[q]), wnb, off + 64 * q, 0, 0);
    }
    f32x4 u[6][1];
    gemm96(lw, t, u);  // Wb^T g_nb
    // d1b's loads behind the first GEMM (registers), in flight during the second
#pragma unroll
    for (int q = 0; q < 6; ++q)
      d1[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rd1, off + 64 * q, 0, 0));
    const __amdgpu_buffer_rsrc_t wna = rsrc(h.g_na, px0, npx_t);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      mask(u[q][0], na[q]);
      t[q] = u[q][0];
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, t[q]), wna, off + 64 * q, 0, 0);
    }
    gemm96(lw + X6_HEAD_BF, t, u);  // Wa^T g_na
    const __amdgpu_buffer_rsrc_t wd1 = rsrc(h.g_d1b, px0, npx_t);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      mask(u[q][0], d1[q]);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, u[q][0]), wd1, off + 64 * q, 0, 0);
    }
  }
}

// wimg = pack_job_head_bwd_x6's images; every tensor NHWC stride 96 (dy: dy_stride, oc <=
// X6_HEAD_BWD_OCMAX: dy in registers; more outputs spill, k_head_bwd takes them)
hipError_t launch_head_bwd_x6(const HeadBwdArgs& h, const void* wimg, hipStream_t s) {
  if (h.oc < 1 || h.oc > X6_HEAD_BWD_OCMAX || h.npx < 1 || h.dy_stride < h.oc) return hipErrorInvalidValue;
  const long nwt = (h.npx + 15) / 16;
  const long blocks = (nwt + 7) / 8 < 256 ? (nwt + 7) / 8 : 256;  // one workgroup per CU
  prof_kernel("k_head_bwd_x6<4>");
  hipLaunchKernelGGL(k_head_bwd_x6<4>, dim3((unsigned)blocks), dim3(512), 0, s, h,
                     static_cast<const __bf16*>(wimg), nwt);
  return hipGetLastError();
}

// nin_a / nin_b weights (OIHW 96x96x1x1, contiguous) -> the two pre-split head images
hipError_t launch_pack_head_x6(const float* wa, const float* wb, void* out, hipStream_t s) {
  PackBatch b;
  b.j[b.n++] = pack_job_head_x6(wa, wb, out);
  return pack_flush(b, s);
}

hipError_t launch_nin_head_x6(const FwdArgs& a, const HeadArgs& h, const void* wimg, hipStream_t s,
                              bool bf16) {
  if ((bf16 && (h.rd || (h.na && h.nb))) || (a.in_bf16 && !bf16) || a.K != 96 || h.oc < 1 ||
      h.oc > X6_HEAD_OCMAX || ((a.in_stride | a.in_off) & 3) ||
      (long)a.IWt * a.in_stride * 4 >= 0x7fffffffL || (long)a.OW * 96 * 4 * 2 >= 0x7fffffffL)
    return hipErrorInvalidValue;
  const long nwt = (long)a.N * a.OH * ((a.OW + 15) / 16);  // one 16-pixel row per wave-tile
  if (nwt >= (1L << 31) - (1L << 20)) return hipErrorInvalidValue;
  long blocks = (nwt + 7) / 8;
  if (blocks > 256) blocks = 256;  // one workgroup per CU
  const __bf16* w = static_cast<const __bf16*>(wimg);
  const dim3 grid((unsigned)blocks), block(512);
  const bool save = h.na && h.nb;
  if (save && h.rd) return hipErrorInvalidValue;  // the pair pass saves nothing
  if (h.rd) hipLaunchKernelGGL((k_nin_head_x6<false, true>), grid, block, 0, s, a, h, w, (int)nwt);
  else if (save) hipLaunchKernelGGL((k_nin_head_x6<true, false>), grid, block, 0, s, a, h, w, (int)nwt);
  else if (bf16 && a.in_bf16)
    hipLaunchKernelGGL((k_nin_head_x6<false, false, true, true>), grid, block, 0, s, a, h, w, (int)nwt);
  else if (bf16) hipLaunchKernelGGL((k_nin_head_x6<false, false, true>), grid, block, 0, s, a, h, w, (int)nwt);
  else hipLaunchKernelGGL((k_nin_head_x6<false, false>), grid, block, 0, s, a, h, w, (int)nwt);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// ConvTranspose2d(96, 96, 2, 2) forward (UpsampleCat's deconv, arch_unet.py:51-62) in the
// bf16x6 arithmetic: out(2y+a, 2x+b, co) = bias[co] + sum_ci x(y, x, ci) W[ci][co][a][b].
// Each parity's 96x96 weight matrix is pre-split ([plane][K block][co][32 ci], 64-B rows,
// swizzled quads; 54 KiB) and DMA'd into LDS.  A lane's B operand is 8 consecutive input
// channels of its pixel (two float4 loads, split in registers); the 16x16 C/D tile (rows =
// output channels, columns = pixels) is stored as float4 channel quads at the scattered
// output pixel.
// ------------------------------------------------------------------------------------
// Persistent: one 8-wave workgroup per CU holds two parity images, (a, 0) and (a, 1), waves 0-3 /
// 4-7 computing those parities; the two workgroups of a group (blockIdx.x bit 3 = a, the other
// bits = group; same XCD) cover the four parities of the same wave-tiles -- one low-res row of
// 16 pixels -- so three of the four reads of an input row hit that XCD's L2.  The next row's
// input is loaded into registers while the current one computes; the images are read from L2
// once per workgroup.
// B1: plain bf16 products (the bf16 base's autocast arithmetic, as k_nin_head_x6's B1): the input
// rounded to bf16, the images' leading planes (the weights rounded to bf16), one MFMA per block
// chained in fp32 -- a sixth of the MFMAs, so the launch is bound by its output stores
template <bool B1 = false>
__global__ __launch_bounds__(512, 1) void k_deconv_x6(FwdArgs a, const __bf16* wimg, int nwt) {
  __shared__ __attribute__((aligned(16))) __bf16 lw[2 * X6_HEAD_BF];
  __shared__ __attribute__((aligned(16))) float lbias[96];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, lg = lane >> 4;
  const int pa = (blockIdx.x >> 3) & 1, pb = wave >> 2, wq = wave & 3;
  const int grp = ((blockIdx.x >> 4) << 3) | (blockIdx.x & 7), ngrp = gridDim.x >> 1;
  const __bf16* src = wimg + 2 * pa * X6_HEAD_BF;  // parities 2a, 2a + 1
  for (int q = wave; q < 2 * X6_HEAD_BF * 2 / 1024; q += 8)
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(src + q * 512 + lane * 8),
        (__attribute__((address_space(3))) void*)(lw + q * 512), 16, 0, 0);
  if (threadIdx.x < 96) lbias[threadIdx.x] = a.bias[threadIdx.x];
  const __bf16* img = lw + pb * X6_HEAD_BF;
  const int tiles_x = (a.OW + 15) / 16;
  const int wstride = ngrp * 4;
  // loads and stores through per-row buffer resources: out-of-range lanes (past the row or the
  // last wave-tile) get an out-of-range offset instead of a branch, so every wave-tile issues the
  // same 6 loads and 6 stores and the compiler's counted waits cover exactly the loads they need.
  // Constant offsets go into the vector offset (folded into the instruction's offset field), never
  // into soffset: a 16-byte buffer store with an SGPR soffset whose data registers were rewritten
  // by the very next instruction (an LDS read) stored a corrupted last dword on some lanes.
  const long in_row = (long)a.IWt * a.in_stride, out_row = 2L * a.OW * a.out_stride;
  auto load = [&](int wt, float4 (&v)[6]) {
    const int n = wt / (a.OH * tiles_x), r = wt - n * a.OH * tiles_x;
    const int gy = r / tiles_x, gx = (r - gy * tiles_x) * 16 + li;
    const bool ok = wt < nwt && gx < a.OW;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.in + ((long)n * a.IHt + gy) * in_row + a.in_off), (short)0,
        (int)(in_row * 4), 0x00020000);
    const int off = ok ? (gx * a.in_stride + 8 * lg) * 4 : 0x7fffffff;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      v[2 * b] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 128 * b, 0, 0));
      v[2 * b + 1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 128 * b + 16, 0, 0));
    }
  };
  // one wave-tile; two register sets alternate (see k_nin_head_x6)
  auto tile = [&](int wt, const float4 (&xin)[6]) {
    const int n = wt / (a.OH * tiles_x), r = wt - n * a.OH * tiles_x;
    const int gy = r / tiles_x, gx = (r - gy * tiles_x) * 16 + li;
    f32x4 out[6][1];
#pragma unroll
    for (int f = 0; f < 6; ++f) out[f][0] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      const float4 u0 = xin[2 * b], u1 = xin[2 * b + 1];
      const float v8[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
      if constexpr (B1) {
        bf16x8 x0;
#pragma unroll
        for (int j = 0; j < 8; ++j) x0[j] = (__bf16)v8[j];
#pragma unroll
        for (int f = 0; f < 6; ++f) {
          const int row = b * 96 + f * 16 + li;
          const bf16x8 w0 = *reinterpret_cast<const bf16x8*>(img + row * 32 + x6_swz(row, lg) * 8);
          out[f][0] = mfma_bf16(w0, x0, out[f][0]);
        }
        continue;
      }
      bf16x8 xv[3][1];
      split3x8(v8, xv[0][0], xv[1][0], xv[2][0]);
      // one output fragment at a time, its three weight planes read one fragment ahead: 24
      // operand registers live instead of 72, which leaves room for the third input set below
      bf16x8 wv[2][3];
      auto read_w = [&](int f, bf16x8 (&w)[3]) {
        const int row = b * 96 + f * 16 + li;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          w[pl] = *reinterpret_cast<const bf16x8*>(img + (pl * 3 * 96 + row) * 32 + x6_swz(row, lg) * 8);
      };
      read_w(0, wv[0]);
#pragma unroll
      for (int f = 0; f < 6; ++f) {
        if (f + 1 < 6) read_w(f + 1, wv[(f + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        // x6_group's product order (hi = w0 x0; lo = w0 x1, w1 x0, w0 x2, w1 x1, w2 x0)
        const bf16x8(&w)[3] = wv[f & 1];
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        const f32x4 hi = mfma_bf16(w[0], xv[0][0], z);
        f32x4 lo = mfma_bf16(w[0], xv[1][0], z);
        lo = mfma_bf16(w[1], xv[0][0], lo);
        lo = mfma_bf16(w[0], xv[2][0], lo);
        lo = mfma_bf16(w[1], xv[1][0], lo);
        lo = mfma_bf16(w[2], xv[0][0], lo);
        x6_acc_add(out[f][0], hi, lo);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        a.out + ((long)n * 2 * a.OH + 2 * gy + pa) * out_row + a.out_off, (short)0,
        (int)(out_row * 4), 0x00020000);
    // Whole 128-B lines per store: a lane holds 4 channels of fragments f and f + 1 of its own
    // pixel, so one store per fragment wrote only 64 B of each pixel's 32-channel line, and the
    // L2 filled the other half from HBM before the second store came (0.75 GB of extra fetch per
    // 256^2 launch, profiles/r5a_pmc_step.json).  Adjacent lanes (pixels 2p, 2p + 1 of the
    // wave-tile) swap one fragment's registers (DPP quad_perm [1,0,3,2]), and each store
    // instruction writes the full line (channels 32k .. 32k + 31) of one pixel per lane pair:
    // the even lane its fragment-f quad, the odd lane the even pixel's fragment-(f + 1) quad.
    const bool ev = (li & 1) == 0;
    const int gxa = gx - (li & 1);  // the pair's even pixel; gxa + 1 the odd one
    const int offa = gxa < a.OW ? ((2 * gxa + pb) * a.out_stride + 4 * lg + (ev ? 0 : 16)) * 4 : 0x7fffffff;
    const int offb = gxa + 1 < a.OW ? ((2 * gxa + 2 + pb) * a.out_stride + 4 * lg + (ev ? 0 : 16)) * 4
                                     : 0x7fffffff;
#pragma unroll
    for (int f = 0; f < 6; f += 2) {
      const float4 b0 = *reinterpret_cast<const float4*>(lbias + f * 16 + 4 * lg);
      const float4 b1 = *reinterpret_cast<const float4*>(lbias + f * 16 + 16 + 4 * lg);
      const f32x4 o0 = {out[f][0][0] + b0.x, out[f][0][1] + b0.y, out[f][0][2] + b0.z, out[f][0][3] + b0.w};
      const f32x4 o1 = {out[f + 1][0][0] + b1.x, out[f + 1][0][1] + b1.y, out[f + 1][0][2] + b1.z,
                        out[f + 1][0][3] + b1.w};
      f32x4 t;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        t[r] = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(
                                             __builtin_bit_cast(int, ev ? o1[r] : o0[r]), 0xB1, 0xF, 0xF, false));
      const f32x4 va = ev ? o0 : t, vb = ev ? t : o1;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, va), rs, offa + 64 * f, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, vb), rs, offb + 64 * f, 0, 0);
    }
  };
  // three input register sets: a wave-tile's input is requested two tiles before it is used
  // (one tile of MFMA work did not cover the HBM latency: 0.8 ms at 64 x 128^2 -> 256^2 against
  // ~0.4 ms of HBM traffic)
  int wt = grp * 4 + wq;
  float4 xa[6], xb[6], xc[6];
  load(wt, xa);
  load(wt + wstride, xb);
  __syncthreads();  // parity images and bias landed
  for (; wt < nwt; wt += 3 * wstride) {
    load(wt + 2 * wstride, xc);
    tile(wt, xa);
    if (wt + wstride >= nwt) break;
    load(wt + 3 * wstride, xa);
    tile(wt + wstride, xb);
    if (wt + 2 * wstride >= nwt) break;
    load(wt + 4 * wstride, xb);
    tile(wt + 2 * wstride, xc);
  }
}

bool deconv_x6_ok(const FwdArgs& a) {  // float4 views; per-row buffer extents below 2^31 bytes
  return a.K == 96 && a.NOUT == 96 && !((a.in_stride | a.in_off | a.out_stride | a.out_off) & 3) &&
         (long)a.IWt * a.in_stride * 4 < 0x7fffffffL && 2L * a.OW * a.out_stride * 4 < 0x7fffffffL;
}

// raw deconv weight (96, 96, 2, 2) -> four pre-split parity images (4 x X6_HEAD_BF bf16)
hipError_t launch_pack_deconv_x6(const float* w, void* out, hipStream_t s) {
  PackBatch b;
  b.j[b.n++] = pack_job_deconv_x6(w, out);
  return pack_flush(b, s);
}

// a: in = x (IHt = OH = h, IWt = OW = w), out = the 2h x 2w view, bias; K = NOUT = 96; b1: plain
// bf16 products (the bf16 base)
hipError_t launch_deconv_x6(const FwdArgs& a, const void* wimg, hipStream_t s, bool b1) {
  if (!deconv_x6_ok(a)) return hipErrorInvalidValue;
  const long nwt = (long)a.N * a.OH * ((a.OW + 15) / 16);  // one low-res 16-pixel row per wave-tile
  if (nwt >= (1L << 31) - (1L << 20)) return hipErrorInvalidValue;
  // groups of two workgroups (one per parity row a), a multiple of 8 groups (one per XCD)
  long groups = (nwt + 3) / 4;
  if (groups > 128) groups = 128;
  groups = (groups + 7) / 8 * 8;
  if (b1) {
    prof_kernel("k_deconv_x6<true>");
    hipLaunchKernelGGL(k_deconv_x6<true>, dim3((unsigned)(2 * groups)), dim3(512), 0, s, a,
                       static_cast<const __bf16*>(wimg), (int)nwt);
  } else {
    prof_kernel("k_deconv_x6<false>");
    hipLaunchKernelGGL(k_deconv_x6<false>, dim3((unsigned)(2 * groups)), dim3(512), 0, s, a,
                       static_cast<const __bf16*>(wimg), (int)nwt);
  }
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// Data gradient of the 96-channel ConvTranspose2d(2, 2) (arch_unet.py:51-62) in the bf16x6
// arithmetic: dx(y, x, ci) = sum_{a,b} sum_co dy(2y+a, 2x+b, co) W[ci][co][a][b] (x leaky'(mask)),
// a GEMM with K = 4 parities x 96.  Persistent, one 8-wave workgroup per CU holding the images of
// one input-channel half h for all four parities (4 x 27 KiB; the two halves' workgroups of a
// group share an XCD and the same wave-tiles, so the second read of dy hits L2); a wave-tile is
// one row of 16 output pixels x 48 channels, computed in four parity steps whose dy rows are
// loaded one step ahead (two alternating register sets), the mask with the last step.
// ------------------------------------------------------------------------------------
template <bool MASKED>
__global__ __launch_bounds__(512, 1) void k_deconv_dgrad_x6(FwdArgs a, const __bf16* wimg, int nwt) {
  __shared__ __attribute__((aligned(16))) __bf16 lw[4 * X6_DG_BF];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, lg = lane >> 4;
  const int h = (blockIdx.x >> 3) & 1;
  const int grp = ((blockIdx.x >> 4) << 3) | (blockIdx.x & 7), ngrp = gridDim.x >> 1;
  const __bf16* src = wimg + (long)h * 4 * X6_DG_BF;
  for (int q = wave; q < 4 * X6_DG_BF * 2 / 1024; q += 8)
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(src + q * 512 + lane * 8),
        (__attribute__((address_space(3))) void*)(lw + q * 512), 16, 0, 0);
  const int tiles_x = (a.OW + 15) / 16;
  const int wstride = ngrp * 8;
  // per-row buffer resources, constant offsets in the vector offset (see k_deconv_x6)
  const long in_row = (long)a.IWt * a.in_stride;
  auto load = [&](int wt, int par, float4 (&v)[6]) {  // dy row 2gy + a, pixels 2gx + b
    const int n = wt / (a.OH * tiles_x), r = wt - n * a.OH * tiles_x;
    const int gy = r / tiles_x, gx = (r - gy * tiles_x) * 16 + li;
    const bool ok = wt < nwt && gx < a.OW;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.in + ((long)n * a.IHt + 2 * gy + (par >> 1)) * in_row + a.in_off),
        (short)0, (int)(in_row * 4), 0x00020000);
    const int off = ok ? ((2 * gx + (par & 1)) * a.in_stride + 8 * lg) * 4 : 0x7fffffff;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      v[2 * b] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 128 * b, 0, 0));
      v[2 * b + 1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 128 * b + 16, 0, 0));
    }
  };
  auto row_rsrc = [&](const float* base, int stride, int wt) {  // output-resolution row of wt
    const int n = wt / (a.OH * tiles_x), r = wt - n * a.OH * tiles_x;
    const int gy = r / tiles_x;
    return __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(base + ((long)n * a.OH + gy) * a.OW * stride), (short)0,
        a.OW * stride * 4, 0x00020000);
  };
  auto pix_off = [&](int wt, int stride, int coff) {  // this lane's channel quad, or out of range
    const int r = wt % (a.OH * tiles_x), gx = (r % tiles_x) * 16 + li;
    return wt < nwt && gx < a.OW ? (gx * stride + coff + 48 * h + 4 * lg) * 4 : 0x7fffffff;
  };
  auto mload = [&](int wt, float4 (&m)[3]) {
    const __amdgpu_buffer_rsrc_t rs = row_rsrc(a.mask, a.mask_stride, wt);
    const int off = pix_off(wt, a.mask_stride, a.mask_off);
#pragma unroll
    for (int f = 0; f < 3; ++f)
      m[f] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 64 * f, 0, 0));
  };
  auto step = [&](int par, const float4 (&xin)[6], f32x4 (&acc)[3][1]) {
    const __bf16* img = lw + par * X6_DG_BF;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      const float4 u0 = xin[2 * b], u1 = xin[2 * b + 1];
      const float v8[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
      bf16x8 xv[3][1];
      split3x8(v8, xv[0][0], xv[1][0], xv[2][0]);
      bf16x8 wv[3][3];
#pragma unroll
      for (int f = 0; f < 3; ++f) {
        const int row = b * 48 + f * 16 + li;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          wv[pl][f] = *reinterpret_cast<const bf16x8*>(img + (pl * 3 * 48 + row) * 32 + x6_swz(row, lg) * 8);
      }
      x6_block<3, 1, 1>(acc, wv, xv);
      __builtin_amdgcn_sched_barrier(0);
    }
    // the running sums materialised here: otherwise the compiler defers the fp32 adds of the
    // block sums to the epilogue and keeps every step's MFMA results live (it spills)
#pragma unroll
    for (int f = 0; f < 3; ++f) asm volatile("" : "+v"(acc[f][0]));
  };
  auto epilogue = [&](int wt, const f32x4 (&acc)[3][1], const float4 (&m)[3]) {
    const __amdgpu_buffer_rsrc_t rs = row_rsrc(a.out, a.out_stride, wt);
    const int off = pix_off(wt, a.out_stride, a.out_off);
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      float4 o = make_float4(acc[f][0][0], acc[f][0][1], acc[f][0][2], acc[f][0][3]);
      if constexpr (MASKED) {
        o.x *= m[f].x > 0.f ? 1.f : 0.2f; o.y *= m[f].y > 0.f ? 1.f : 0.2f;
        o.z *= m[f].z > 0.f ? 1.f : 0.2f; o.w *= m[f].w > 0.f ? 1.f : 0.2f;
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, o), rs, off + 64 * f, 0, 0);
    }
  };
  int wt = grp * 8 + wave;
  float4 xa[6], xb[6], m[3] = {};
  load(wt, 0, xa);
  __syncthreads();  // images landed
  for (; wt < nwt; wt += wstride) {
    f32x4 acc[3][1];
#pragma unroll
    for (int f = 0; f < 3; ++f) acc[f][0] = f32x4{0.f, 0.f, 0.f, 0.f};
    load(wt, 1, xb);
    step(0, xa, acc);
    load(wt, 2, xa);
    step(1, xb, acc);
    load(wt, 3, xb);
    if constexpr (MASKED) mload(wt, m);
    step(2, xa, acc);
    load(wt + wstride, 0, xa);
    step(3, xb, acc);
    epilogue(wt, acc, m);
  }
}

bool deconv_dgrad_x6_ok(const FwdArgs& a) {  // float4 views; per-row buffer extents below 2^31
  return a.K == 96 && a.NOUT == 96 && a.IHt == 2 * a.OH && a.IWt == 2 * a.OW &&
         !((a.in_stride | a.in_off | a.out_stride | a.out_off) & 3) &&
         (a.epi == EPI_PLAIN || (a.epi == EPI_MASK && a.mask && !((a.mask_stride | a.mask_off) & 3))) &&
         (long)a.IWt * a.in_stride * 4 < 0x7fffffffL && (long)a.OW * a.out_stride * 4 < 0x7fffffffL &&
         (a.epi != EPI_MASK || (long)a.OW * a.mask_stride * 4 < 0x7fffffffL);
}

hipError_t launch_deconv_dgrad_x6(const FwdArgs& a, const void* wimg, hipStream_t s) {
  if (!deconv_dgrad_x6_ok(a)) return hipErrorInvalidValue;
  const long nwt = (long)a.N * a.OH * ((a.OW + 15) / 16);  // one 16-pixel output row per wave-tile
  if (nwt >= (1L << 31) - (1L << 20)) return hipErrorInvalidValue;
  // groups of two workgroups (one per input-channel half), a multiple of 8 groups (one per XCD)
  long groups = (nwt + 7) / 8;
  if (groups > 128) groups = 128;
  groups = (groups + 7) / 8 * 8;
  const dim3 grid((unsigned)(2 * groups)), block(512);
  const __bf16* w = static_cast<const __bf16*>(wimg);
  if (a.epi == EPI_MASK) hipLaunchKernelGGL(k_deconv_dgrad_x6<true>, grid, block, 0, s, a, w, (int)nwt);
  else hipLaunchKernelGGL(k_deconv_dgrad_x6<false>, grid, block, 0, s, a, w, (int)nwt);
  return hipGetLastError();
}

}  // namespace dn
