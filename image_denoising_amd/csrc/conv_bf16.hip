// Mixed-precision 3x3 / 1x1 convolution forward on the gfx950 bf16 matrix cores
// (v_mfma_f32_16x16x32_bf16): the frozen-base forward of the adapter finetune (BASELINE
// configs[4], "mixed-precision bf16"; finetune.py:255-262 runs the base under no_grad).
//
// Activations stay fp32 NHWC in HBM; each input tile is rounded to bf16 (round-to-nearest-even)
// as it is staged into LDS, weights are pre-packed in bf16, products accumulate in fp32 and the
// epilogue (bias, LeakyReLU) and output are fp32 — the numerics of torch.autocast(bfloat16) for
// a conv, except that the output is not rounded to bf16.
//
//   Workgroup = 4 waves, tile = 4*MT rows x 16 pixels x 16*NT output channels; wave w owns rows
//   [w*MT, w*MT+MT).  K is staged 32 input channels at a time (one MFMA K): the x tile (with
//   halo) once per chunk, the weights one kernel row (3 taps; 1x1: the single tap) per stage,
//   double-buffered by global_load_lds.  Per stage a wave issues 3*MT*NT MFMAs of 16x16x32.
//   LDS rows are 32 bf16 (64 B) per pixel / per (tap, output channel), the 16-B quad q of row r
//   stored at quad x6_swz(r, q) = q ^ ((r >> 1) & 3) (the bf16x6 kernels' layout): a lane's
//   8-element operand (k = 8*(lane>>4) .. +7) is one ds_read_b128, conflict-free over gfx950's
//   ds_read_b128 lane groups for every tap offset.  (The unswizzled 80-B rows of round 2 were
//   2-way on a third of those groups: SQ_LDS_BANK_CONFLICT 47 % of the LDS-active cycles.)
#include <cstdlib>

#include "conv_epi.h"
#include "dn_internal.h"
#include "x6_core.h"

namespace dn {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4b __attribute__((ext_vector_type(4)));

template <int NT, int MT, bool K3 = true>
struct BCfg {
  static constexpr int HALO = K3 ? 2 : 0, TPS = K3 ? 3 : 1;  // taps per weight stage
  static constexpr int SPC = K3 ? 3 : 1;                     // weight stages per K chunk
  static constexpr int TW = 16, TH = 4 * MT, IH = TH + HALO, IW = TW + HALO;
  static constexpr int KC = 32;                       // input channels per chunk
  static constexpr int XS = 32;                       // bf16 per pixel row of the x tile
  static constexpr int NP = 16 * NT;
  static constexpr int WS = 32;                       // bf16 per (tap, n) row of a weight stage
  static constexpr int WST = (TPS * NP * WS + 511) / 512 * 512;  // bf16 per stage, whole KiBs
  static constexpr int LXB = (IH * IW * XS + 511) / 512 * 512;  // bf16 of the x tile
  static constexpr int XQ = IH * IW * (KC / 4);       // float4 items of the x tile
  static constexpr int XITEMS = (XQ + 255) / 256;
  static constexpr int PS = NP + 4;                   // epilogue staging pixel stride (floats)
  static constexpr int LST = 4 * 16 * PS;             // floats
  static constexpr int LBYTES_MAIN = 2 * LXB + 2 * 2 * WST;
  static constexpr int LBYTES = LBYTES_MAIN > 4 * LST ? LBYTES_MAIN : 4 * LST;
};

__device__ __forceinline__ void glds16b(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// the same as a buffer load to LDS (k_fwd_bf16p): a pending global_load_lds (FLAT) keeps the
// compiler's waitcnt pass from counting LDS-read waits (every wait becomes lgkmcnt(0)); the
// builtin exists only for the device pass (see x6_core.h buf_lds16)
__device__ __forceinline__ void blds16b(__amdgpu_buffer_rsrc_t rs, void* l, int voffset) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)l, 16,
                                           voffset, 0, 0, 0);
#else
  (void)rs; (void)l; (void)voffset;
#endif
}

template <int NT, int MT, bool K3, bool IB = false>
__global__ __launch_bounds__(256, 2) void k_fwd_bf16(FwdArgs a) {
  using C = BCfg<NT, MT, K3>;
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[C::LBYTES];
  __bf16* lx = reinterpret_cast<__bf16*>(lds_raw);
  __bf16* lw0 = lx + C::LXB;
  __bf16* lw1 = lw0 + C::WST;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const int tiles_x = (a.OW + C::TW - 1) / C::TW;
  int bxr, byr;  // XCD-aware tile order (conv_epi.h xcd_tile)
  xcd_tile(bxr, byr);
  const int ty0 = (bxr / tiles_x) * C::TH;
  const int tx0 = (bxr % tiles_x) * C::TW;
  const int n = byr;
  const int iy0 = ty0 - (K3 ? 1 : 0), ix0 = tx0 - (K3 ? 1 : 0);
  const float* inb = a.in + (long)n * a.IHt * a.IWt * a.in_stride + a.in_off;
  const bool vec = ((a.in_stride | a.in_off) & 3) == 0;
  const int nch = (a.K + C::KC - 1) / C::KC;
  const int nst = C::SPC * nch;

  f32x4b acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < NT; ++q) acc[m][q] = f32x4b{0.f, 0.f, 0.f, 0.f};

  float4 xr[C::XITEMS];
  typedef unsigned u32x2b __attribute__((ext_vector_type(2)));
  u32x2b xh[IB ? C::XITEMS : 1];  // (IB) bf16 input: 4 channels = 8 bytes, stored as loaded
  auto load_x = [&](int k0) {
#pragma unroll
    for (int it = 0; it < C::XITEMS; ++it) {
      const int e = tid + it * 256;
      if constexpr (IB) {  // channel quads whole (K % 4 == 0, aligned views: the launcher)
        u32x2b v = {0u, 0u};
        if (e < C::XQ) {
          const int q = e % (C::KC / 4), pix = e / (C::KC / 4);
          const int iy = pix / C::IW, ix = pix - iy * C::IW;
          const int gy = iy0 + iy, gx = ix0 + ix, k = k0 + 4 * q;
          if (gy >= 0 && gy < a.IHt && gx >= 0 && gx < a.IWt && k < a.K)
            v = *reinterpret_cast<const u32x2b*>(reinterpret_cast<const __bf16*>(a.in) +
                                                 ((long)n * a.IHt * a.IWt + (long)gy * a.IWt + gx) *
                                                     a.in_stride + a.in_off + k);
        }
        xh[it] = v;
        continue;
      }
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
        __bf16* dst = lx + pix * C::XS + x6_swz(pix, q >> 1) * 8 + (q & 1) * 4;
        if constexpr (IB) {
          *reinterpret_cast<u32x2b*>(dst) = xh[it];
          continue;
        }
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        bf16x4 h;
        h[0] = (__bf16)xr[it].x; h[1] = (__bf16)xr[it].y;
        h[2] = (__bf16)xr[it].z; h[3] = (__bf16)xr[it].w;
        *reinterpret_cast<bf16x4*>(dst) = h;
      }
    }
  };
  auto load_w = [&](int st, __bf16* dst) {  // stage st = chunk * 3 + ky, whole 1 KiB pieces
    // (deconv: blockIdx.z = output parity (a,b), one image of wp_z bf16 elements each)
    const __bf16* src = reinterpret_cast<const __bf16*>(a.wp) + (long)blockIdx.z * a.wp_z +
                        (long)st * C::WST;
    for (int p = wave; p < C::WST / 512; p += 4) glds16b(src + p * 512 + lane * 8, dst + p * 512);
  };

  load_w(0, lw0);
  load_x(0);
  store_x();
  __syncthreads();

  for (int st = 0; st < nst; ++st) {
    const int c = st / C::SPC, ky = st - C::SPC * c;
    const __bf16* lw = (st & 1) ? lw1 : lw0;
    if (st + 1 < nst) load_w(st + 1, (st & 1) ? lw0 : lw1);
    if (ky == 0 && c + 1 < nch) load_x((c + 1) * C::KC);
#pragma unroll
    for (int kx = 0; kx < C::TPS; ++kx) {
      bf16x8 av[MT], bv[NT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int r = wave * MT + m;
        const int pix = (r + ky) * C::IW + li + kx;
        av[m] = *reinterpret_cast<const bf16x8*>(lx + pix * C::XS + x6_swz(pix, lg) * 8);
      }
#pragma unroll
      for (int q = 0; q < NT; ++q)
        bv[q] = *reinterpret_cast<const bf16x8*>(lw + (kx * C::NP + q * 16 + li) * C::WS +
                                                 x6_swz(kx * C::NP + q * 16 + li, lg) * 8);
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int q = 0; q < NT; ++q)
          acc[m][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[m], bv[q], acc[m][q], 0, 0, 0);
    }
    __syncthreads();  // all waves done with this weight stage (and the x tile at ky == 2)
    if (ky == C::SPC - 1 && c + 1 < nch) store_x();
    __syncthreads();  // next stage's weights landed (vmcnt(0)), next x tile written
  }

  // the shared LDS-staged epilogue (conv_epi.h): loads of all rows before any store, no
  // per-row barriers (each wave stages its own rows)
  fwd_epilogue<NT, MT, C::PS, false>(a, acc, reinterpret_cast<float*>(lds_raw), ty0, tx0, n);
}

// ------------------------------------------------------------------------------------
// Pipelined 3x3 variant (float4-aligned input views, K % 4 == 0): the tile and LDS layout of
// k_fwd_bf16, but ONE barrier per weight stage and the waits counted per wave.  Stage st+1's
// weights are DMA'd into the other ring slot at the start of stage st (every wave issues the
// same PPW pieces; short waves re-load their last one); the next chunk's x tile is requested
// into registers at its first stage (buffer loads with out-of-range offsets for the halo and
// the image border, so the count is fixed) and rounded into LDS at its last.  The wait before
// a stage's barrier is vmcnt(XITEMS) at a chunk's first stage (the x loads younger than the
// weight DMAs stay in flight across the chunk), vmcnt(0) otherwise: the x tile's HBM latency
// is hidden behind two weight stages instead of stalling the stage it was issued in (k_fwd_bf16
// waits for it at that stage's barrier).
// ------------------------------------------------------------------------------------
#define BF_WAITCNT_VM(n) \
  __builtin_amdgcn_s_waitcnt(((n) & 0xF) | (((n) >> 4) << 14) | (0x7 << 4) | (0xF << 8))

__device__ __forceinline__ void bf_barrier() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);  // no compiler motion of LDS accesses across it
  __builtin_amdgcn_s_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// (MT = 6 with NT = 6: the larger wave tile -- fewer LDS fragment reads per MFMA -- needs the
// whole register file, one workgroup per CU; DN_BF16_MT / DN_BF16_MT3 select it)
template <int NT, int MT, bool IB = false>
__global__ __launch_bounds__(256, (NT * MT > 24) ? 1 : 2) void k_fwd_bf16p(FwdArgs a) {
  using C = BCfg<NT, MT, true>;
  constexpr int PIECES = C::WST / 512, PPW = (PIECES + 3) / 4;
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[C::LBYTES];
  __bf16* lx = reinterpret_cast<__bf16*>(lds_raw);
  __bf16* ring = lx + C::LXB;

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
  constexpr int EB = IB ? 2 : 4;  // bytes per stored activation
  const unsigned char* inb = reinterpret_cast<const unsigned char*>(a.in) +
                             ((long)n * a.IHt * a.IWt * a.in_stride + a.in_off) * EB;
  const __bf16* wimg = reinterpret_cast<const __bf16*>(a.wp);
  const int nch = (a.K + C::KC - 1) / C::KC;
  const int nst = 3 * nch;

  f32x4b acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < NT; ++q) acc[m][q] = f32x4b{0.f, 0.f, 0.f, 0.f};

  // this tile's input rows through a 32-bit buffer resource (host: < 2 GiB per tile's rows)
  const int ry0 = iy0 > 0 ? iy0 : 0, ry1 = iy0 + C::IH < a.IHt ? iy0 + C::IH : a.IHt;
  const long row_elems = (long)a.IWt * a.in_stride;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char*>(inb + ry0 * row_elems * EB), (short)0,
      (int)((ry1 - ry0) * row_elems * EB), 0x00020000);
  typedef unsigned u32x2b __attribute__((ext_vector_type(2)));
  f32x4b xr[IB ? 1 : C::XITEMS];
  u32x2b xh[IB ? C::XITEMS : 1];  // (IB) bf16 input: 4 channels = 8 bytes, stored as loaded
  auto load_x = [&](int k0) {
#pragma unroll
    for (int it = 0; it < C::XITEMS; ++it) {
      const int e = tid + it * 256;
      const int q = e % (C::KC / 4), pix = e / (C::KC / 4);
      const int iy = pix / C::IW, ix = pix - iy * C::IW;
      const int gy = iy0 + iy, gx = ix0 + ix, k = k0 + 4 * q;
      const bool ok = e < C::XQ && gy >= 0 && gy < a.IHt && gx >= 0 && gx < a.IWt && k < a.K;
      const int off = ok ? (((gy - ry0) * a.IWt + gx) * a.in_stride + k) * EB : 0x7fffffff;
      if constexpr (IB)
        xh[it] = __builtin_bit_cast(u32x2b, __builtin_amdgcn_raw_buffer_load_b64(xrs, off, 0, 0));
      else
        xr[it] = __builtin_bit_cast(f32x4b, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int it = 0; it < C::XITEMS; ++it) {
      const int e = tid + it * 256;
      if (e < C::XQ) {
        const int q = e % (C::KC / 4), pix = e / (C::KC / 4);
        __bf16* dst = lx + pix * C::XS + x6_swz(pix, q >> 1) * 8 + (q & 1) * 4;
        if constexpr (IB) {
          *reinterpret_cast<u32x2b*>(dst) = xh[it];
        } else {
          typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
          bf16x4 h;
          h[0] = (__bf16)xr[it][0]; h[1] = (__bf16)xr[it][1];
          h[2] = (__bf16)xr[it][2]; h[3] = (__bf16)xr[it][3];
          *reinterpret_cast<bf16x4*>(dst) = h;
        }
      }
    }
  };
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__bf16*>(wimg), (short)0, nst * C::WST * 2, 0x00020000);
  auto load_w = [&](int st, int slot) {  // stage st = chunk * 3 + ky: PPW 1 KiB pieces per wave
    __bf16* dst = ring + slot * C::WST;
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      int p = wave + 4 * j;
      if (p >= PIECES) p -= 4;
      blds16b(wrs, dst + p * 512, (st * C::WST + p * 512 + lane * 8) * 2);
    }
  };

  load_w(0, 0);
  load_x(0);
  store_x();                           // waits for the x loads (and the older DMAs)
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own x-tile stores done
  bf_barrier();

#pragma unroll 1
  for (int st = 0; st < nst; ++st) {
    const int c = st / 3, ky = st - 3 * c;
    const bool more = c + 1 < nch;
    const __bf16* lw = ring + (st & 1) * C::WST;
    load_w(st + 1 < nst ? st + 1 : nst - 1, (st + 1) & 1);  // past the end: a re-load
    if (ky == 0 && more) load_x((c + 1) * C::KC);
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      bf16x8 av[MT], bv[NT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int r = wave * MT + m;
        const int pix = (r + ky) * C::IW + li + kx;
        av[m] = *reinterpret_cast<const bf16x8*>(lx + pix * C::XS + x6_swz(pix, lg) * 8);
      }
#pragma unroll
      for (int q = 0; q < NT; ++q)
        bv[q] = *reinterpret_cast<const bf16x8*>(lw + (kx * C::NP + q * 16 + li) * C::WS +
                                                 x6_swz(kx * C::NP + q * 16 + li, lg) * 8);
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int q = 0; q < NT; ++q)
          acc[m][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[m], bv[q], acc[m][q], 0, 0, 0);
    }
    const bool xstep = ky == 2 && more;
    if (xstep) {
      bf_barrier();  // every wave is done with this chunk's x tile
      store_x();
    }
    // own DMAs of stage st+1 landed; younger: the next chunk's x loads (issued at ky == 0)
    if (ky == 0 && more) BF_WAITCNT_VM(C::XITEMS);
    else BF_WAITCNT_VM(0);
    if (xstep) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own x-tile stores done
    bf_barrier();
  }
  __syncthreads();
  // the shared LDS-staged epilogue (conv_epi.h): loads of all rows before any store, no
  // per-row barriers (each wave stages its own rows)
  fwd_epilogue<NT, MT, C::PS, false>(a, acc, reinterpret_cast<float*>(lds_raw), ty0, tx0, n);
}

// bf16 weight image: [chunk][ky][kx][n][32] (k = chunk*32 + kk; zero padded), the quads of row
// kx*NP + n swizzled as the LDS image (x6_swz), each (chunk, ky) stage rounded up to whole KiB
__global__ __launch_bounds__(256) void k_pack_bf16(WView wv, int K, int NOUT, int NP, int WST,
                                                   int k3, long total, __bf16* __restrict__ out) {
  const int spc = k3 ? 3 : 1;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const long st = e / WST;
    const int r = (int)(e - st * WST);
    const int c = (int)(st / spc), ky = (int)(st % spc);
    float v = 0.f;
    if (r < spc * NP * 32) {
      const int row = r / 32, kx = row / NP, nn = row % NP;
      const int kk = x6_swz(row, (r % 32) / 8) * 8 + r % 8;  // the swizzle is an involution
      const int k = c * 32 + kk;
      if (k < K && nn < NOUT) {
        const int t = k3 ? ky * 3 + kx : 0;
        const int tm = wv.flip ? wv.taps - 1 - t : t;
        v = wv.w[wv.off + (long)k * wv.sK + (long)nn * wv.sN + (long)tm * wv.sT];
      }
    }
    out[e] = (__bf16)v;
  }
}

template <int NT, int MT, bool K3>
static hipError_t run_bf16(const FwdArgs& a, hipStream_t s) {
  using C = BCfg<NT, MT, K3>;
  const int tx = (a.OW + C::TW - 1) / C::TW, ty = (a.OH + C::TH - 1) / C::TH;
  const int nz = a.out_layout == OUT_UP2 ? 4 : 1;
  if (a.in_bf16)
    hipLaunchKernelGGL((k_fwd_bf16<NT, MT, K3, true>), dim3(tx * ty, a.N, nz), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((k_fwd_bf16<NT, MT, K3>), dim3(tx * ty, a.N, nz), dim3(256), 0, s, a);
  return hipGetLastError();
}

static int bf16_nt(int nout) { return nout <= 48 ? 3 : (nout <= 96 ? 6 : 0); }

static long bf16_stage(int nt, int ksize) {
  if (ksize == 3) return nt == 3 ? BCfg<3, 4, true>::WST : BCfg<6, 4, true>::WST;
  return nt == 3 ? BCfg<3, 4, false>::WST : BCfg<6, 4, false>::WST;
}

long bf16_stage_elems(int nout, int ksize) {
  const int nt = bf16_nt(nout);
  return nt == 0 || (ksize != 1 && ksize != 3) ? -1 : bf16_stage(nt, ksize);
}

// bf16 elements of the packed image of a 3x3 (ksize 3) or 1x1 layer (K inputs, nout <= 96)
long bf16_pack_elems(int K, int nout, int ksize) {
  const int nt = bf16_nt(nout);
  if (nt == 0 || (ksize != 1 && ksize != 3)) return -1;
  return (long)((K + 31) / 32) * (ksize == 3 ? 3 : 1) * bf16_stage(nt, ksize);
}

hipError_t launch_pack_bf16(const WView& wv, int K, int nout, void* out, hipStream_t s, int ksize) {
  const int nt = bf16_nt(nout);
  if (nt == 0) return hipErrorInvalidValue;
  const long total = bf16_pack_elems(K, nout, ksize);
  if (total < 0) return hipErrorInvalidValue;
  long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(k_pack_bf16, dim3((unsigned)blocks), dim3(256), 0, s, wv, K, nout, 16 * nt,
                     (int)bf16_stage(nt, ksize), ksize == 3 ? 1 : 0, total,
                     static_cast<__bf16*>(out));
  return hipGetLastError();
}

// ConvTranspose2d(cin, cout, 2, 2) weight [cin][cout][2][2] as four 1x1 images (one per output
// parity ab), each bf16_pack_elems(cin, cout, 1) elements
hipError_t launch_pack_bf16_deconv(const float* w, int cin, int cout, void* out, hipStream_t s) {
  const long img = bf16_pack_elems(cin, cout, 1);
  if (img < 0) return hipErrorInvalidValue;
  for (int ab = 0; ab < 4; ++ab) {
    WView v{};
    v.w = w; v.off = ab; v.sK = (long)cout * 4; v.sN = 4; v.sT = 0; v.sZ = 0; v.taps = 1; v.flip = 0;
    hipError_t e = launch_pack_bf16(v, cin, cout, static_cast<__bf16*>(out) + ab * img, s, 1);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// a.wp = the launch_pack_bf16 image; epilogue EPI_BIAS / EPI_BIAS_ACT; NHWC fp32 output with
// float4-aligned views and NOUT % 4 == 0
hipError_t launch_fwd_bf16(const FwdArgs& a, hipStream_t s, int ksize) {
  const int nt = bf16_nt(a.NOUT);
  if (nt == 0 || (a.NOUT & 3) || ((a.out_stride | a.out_off) & 3) ||
      (a.out_layout != OUT_NHWC && !(a.out_layout == OUT_UP2 && ksize == 1)) ||
      (a.epi != EPI_BIAS && a.epi != EPI_BIAS_ACT) || !a.bias || (ksize != 1 && ksize != 3))
    return hipErrorInvalidValue;
  // bf16 activation storage: whole channel quads (8-byte loads / stores), the float4 epilogue
  if ((a.in_bf16 && ((a.K | a.in_stride | a.in_off) & 3)) || (a.out_bf16 && a.out_layout != OUT_NHWC))
    return hipErrorInvalidValue;
  // a fused 2x2 max-pool (the float4 epilogue's, as the x6 kernels): 3x3, activated, NHWC
  // fp32 output, even sides, an even number of rows per wave (MT = 4 even on small grids)
  if (a.pool_out && (ksize != 3 || a.epi != EPI_BIAS_ACT || a.out_layout != OUT_NHWC || a.out_bf16 ||
                     ((a.pool_stride | a.pool_off) & 3) || ((a.OH | a.OW) & 1)))
    return hipErrorInvalidValue;
  const long tiles = (long)a.N * ((a.OH + 15) / 16) * ((a.OW + 15) / 16) *
                     (a.out_layout == OUT_UP2 ? 4 : 1);
  const bool small = tiles < 1024 && !a.pool_out;
  if (ksize == 1) {
    if (nt == 3) return small ? run_bf16<3, 1, false>(a, s) : run_bf16<3, 4, false>(a, s);
    return small ? run_bf16<6, 1, false>(a, s) : run_bf16<6, 4, false>(a, s);
  }
  // pipelined kernel: aligned views, whole channel quads, < 2 GiB of input rows per tile
  // rows per wave: 96-output convs 4 (6 needs the whole register file: one workgroup per CU,
  // slower); 48-output convs 8 -- fewer LDS fragment reads per MFMA at the
  // same occupancy -- where the grid still has >= 4096 such tiles (8 rounds of 512 resident
  // workgroups), else 4.  The accumulation order does not depend on MT: bit-identical results.
  const long tiles8 = (long)a.N * ((a.OH + 31) / 32) * ((a.OW + 15) / 16);
  const int mt = nt == 3 ? (tiles8 >= 4096 ? 8 : 4) : 4;
  const bool pipe = !small && a.out_layout == OUT_NHWC && a.K % 4 == 0 &&
                    ((a.in_stride | a.in_off) & 3) == 0 &&
                    (long)BCfg<6, 8, true>::IH * a.IWt * a.in_stride * 4 < 0x7fffffffL;
  if (pipe) {
    const int tx = (a.OW + 15) / 16, ty = (a.OH + 4 * mt - 1) / (4 * mt);
    const dim3 grid(tx * ty, a.N, 1);
#define DN_BF16P_LAUNCH(NT_, MT_)                                                              \
  do {                                                                                         \
    prof_kernel(a.in_bf16 ? "k_fwd_bf16p<" #NT_ "," #MT_ ",true>"                              \
                          : "k_fwd_bf16p<" #NT_ "," #MT_ ",false>");  /* (rocprofv3 names) */  \
    if (a.in_bf16) hipLaunchKernelGGL((k_fwd_bf16p<NT_, MT_, true>), grid, dim3(256), 0, s, a); \
    else hipLaunchKernelGGL((k_fwd_bf16p<NT_, MT_, false>), grid, dim3(256), 0, s, a);          \
  } while (0)
    if (nt == 3) {
      if (mt == 8) DN_BF16P_LAUNCH(3, 8);
      else DN_BF16P_LAUNCH(3, 4);
    } else {
      DN_BF16P_LAUNCH(6, 4);
    }
#undef DN_BF16P_LAUNCH
    return hipGetLastError();
  }
  if (nt == 3) return small ? run_bf16<3, 1, true>(a, s) : run_bf16<3, 4, true>(a, s);
  return small ? run_bf16<6, 1, true>(a, s) : run_bf16<6, 4, true>(a, s);
}

}  // namespace dn
