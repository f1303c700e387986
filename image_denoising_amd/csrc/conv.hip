// Convolution kernels of the N2N U-Net for gfx950 (MI355X).
//
// Every arithmetic op of arch_unet.py's UNet that reduces over channels (3x3 conv
// arch_unet.py:116-181, 1x1 "nin" convs :186-190, ConvTranspose2d(2,2) :57) and its
// autograd backward is expressed as one of two implicit-GEMM kernels on the fp32 matrix
// cores (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 accumulation, the same
// 157.3 TFLOP/s peak as the fp32 vector ALUs):
//
//   k_fwd   output-stationary: out[p][n] = epi( sum_t sum_k in[gather(p,t)][k] * W[t][k][n] )
//           -> conv forward, conv data-gradient (flipped/transposed weight view),
//              deconv forward (1x1 GEMM + scatter epilogue), deconv data-gradient.
//   k_wgrad weight-gradient: partial dW over a slice of pixels, one slab per split,
//           then k_reduce_batch sums the slabs in a fixed order (deterministic, no atomics).
//
// Data layout: activations NHWC fp32 (channels contiguous), weights in the reference's
// PyTorch layout read through a strided view (no repacking pass).
#include <cstdlib>

#include "conv_epi.h"

namespace dn {

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// smallest x >= v with x % mod == res  (LDS strides chosen for conflict-free ds_read_b32)
constexpr int cround(int v, int mod, int res) { return v + (((res - v % mod) % mod) + mod) % mod; }

// ------------------------------------------------------------------------------------
// Forward-style implicit GEMM.
//   Workgroup = 4 waves; tile = TH x 16 output pixels x NP output channels.
//   Wave w owns tile rows [w*MT, w*MT+MT); fragment m = one row of 16 pixels (MFMA M),
//   fragment n = 16 output channels (MFMA N).  K = taps x input channels, staged through
//   LDS KC channels at a time:
//     - weights come pre-packed (k_pack_batch) as one LDS image per chunk, [tap][k][n] padded to
//       WNS, and are copied by global_load_lds_dwordx4 into a double-buffered slab;
//     - the input tile (with halo) is prefetched into registers (float4 along channels)
//       while the previous chunk computes, then written channel-major [k][pixel].
//   MFMA k-lane group g (lane>>4) takes channel 4s+g of the stage.
// ------------------------------------------------------------------------------------
template <int GATHER, int NT, int MT>
struct FwdCfg {
  // G_UP: every wave covers all MT rows of the tile and wave w takes parity (a,b) = w
  static constexpr int TW = 16, TH = GATHER == G_UP ? MT : 4 * MT;
  static constexpr int KC = GATHER == G_C1 ? 32 : (GATHER == G_UP ? 16 : (NT >= 6 ? 4 : 8));
  static constexpr int NZ = GATHER == G_UP ? 4 : 1;  // weight images per chunk in LDS
  static constexpr int TAPS = GATHER == G_C3 ? 9 : (GATHER == G_DN2 ? 4 : 1);
  static constexpr int IH = GATHER == G_C3 ? TH + 2 : (GATHER == G_DN2 ? 2 * TH : TH);
  static constexpr int IW = GATHER == G_C3 ? TW + 2 : (GATHER == G_DN2 ? 2 * TW : TW);
  // channel stride of the input tile: lanes (i, g) of a 32-lane half hit distinct banks
  static constexpr int XCS = cround(IH * IW, 32, GATHER == G_DN2 ? 1 : 16);
  static constexpr int NP = NT * 16;
  static constexpr int WNS = cround(NP, 32, 16);
  static constexpr int LW = (TAPS * KC * WNS + 255) / 256 * 256;  // one chunk's weight image
  static constexpr int LX = KC * XCS;
  static constexpr int QPP = KC / 4;                              // float4 quads per pixel
  static constexpr int XQ = IH * IW * QPP;
  static constexpr int XITEMS = (XQ + 255) / 256;
  static constexpr int PS = NP + 4;             // epilogue staging: pixel stride (floats)
  static constexpr int LST = 4 * 16 * PS;       // 4 waves x 16 pixels x PS
  static constexpr int LT0 = (LX + 2 * NZ * LW) > LST ? (LX + 2 * NZ * LW) : LST;
  static constexpr int LTOT = LT0 > HEAD_LW ? LT0 : HEAD_LW;  // HEAD: one 1x1 image at a time
};

__device__ __forceinline__ void glds16(const float* g, float* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// Tail of the fused output head (arch_unet.py:251-257) for k_nin_head: acc holds a 4*MT x
// 16-pixel tile of the 96 dec_conv1b channels in the 16x16 MFMA C/D map (PRE_ACT: before its
// bias + LeakyReLU, which are applied here and optionally saved to hd.d1b; else the activated
// values).  lds must hold HEAD_LW floats and be free.  k_fwd<..., HEAD> keeps its own inline copy
// of the PRE_ACT form: through this function its 168-register budget (3 workgroups per CU)
// spills.
template <int MT, bool PRE_ACT>
__device__ __forceinline__ void head_tail(const FwdArgs& a, const HeadArgs& hd,
                                          f32x4 (&acc)[MT][6], float* lds, int ty0, int tx0,
                                          int n) {
  constexpr int NT = 6;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lg = lane >> 4;
    // acc[m][q][r] = dec_conv1b pre-activation at pixel (row m, x = li), channel
    // q*16 + 4*lg + r.  As the B operand of the next 16x16x4 MFMA, register r of fragment q
    // supplies k = channel q*16 + 4g + r for lane group g: nin_a/nin_b consume the tile
    // where it is, with the k order permuted the same way in their weight reads.
    // Two phases through ONE image slot (38 KiB, so three workgroups fit a CU): nin_a for
    // all rows in place (acc <- na), then nin_b + nin_c.
    for (int p = wave; p < HEAD_LW / 256; p += 4) glds16(hd.wp + p * 256 + lane * 4, lds + p * 256);
    auto bias_act = [](f32x4& v, float4 b) {
      v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * 0.2f;
    };
    auto save = [&](float* dst, long pix, int q, const f32x4& v) {
      *reinterpret_cast<float4*>(dst + pix * 96 + q * 16 + 4 * lg) = make_float4(v[0], v[1], v[2], v[3]);
    };
    // 1x1 GEMM on the transposed tile: out[f] = W^T-image x in (k order = the tile's)
    auto gemm96 = [&](const float* w, const f32x4 (&in)[NT], f32x4 (&out)[NT]) {
#pragma unroll
      for (int f = 0; f < NT; ++f) out[f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < NT; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float* wr = w + (q * 16 + 4 * lg + r) * HEAD_WS + li;
#pragma unroll
          for (int f = 0; f < NT; ++f) out[f] = mfma4(wr[f * 16], in[q][r], out[f]);
        }
    };
    if (PRE_ACT) {
#pragma unroll
      for (int q = 0; q < NT; ++q) {
        const float4 b = *reinterpret_cast<const float4*>(a.bias + q * 16 + 4 * lg);
#pragma unroll
        for (int m = 0; m < MT; ++m) bias_act(acc[m][q], b);
      }
    }
    const int gx = tx0 + li;
    if (PRE_ACT && hd.d1b) {
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int gy = ty0 + wave * MT + m;
        if (gy < a.OH && gx < a.OW)
#pragma unroll
          for (int q = 0; q < NT; ++q) save(hd.d1b, ((long)n * a.OH + gy) * a.OW + gx, q, acc[m][q]);
      }
    }
    __syncthreads();  // nin_a image landed
#pragma unroll
    for (int m = 0; m < MT; ++m) {  // phase 1: acc[m] <- na
      const int gy = ty0 + wave * MT + m;
      f32x4 u[NT];
      gemm96(lds, acc[m], u);
#pragma unroll
      for (int f = 0; f < NT; ++f) {
        bias_act(u[f], *reinterpret_cast<const float4*>(hd.ba + f * 16 + 4 * lg));
        acc[m][f] = u[f];
      }
      if (hd.na && gy < a.OH && gx < a.OW)
#pragma unroll
        for (int f = 0; f < NT; ++f) save(hd.na, ((long)n * a.OH + gy) * a.OW + gx, f, acc[m][f]);
    }
    __syncthreads();  // everyone done with nin_a
    for (int p = wave; p < HEAD_LW / 256; p += 4)
      glds16(hd.wp + HEAD_LW + p * 256 + lane * 4, lds + p * 256);
    __syncthreads();  // nin_b image landed
#pragma unroll
    for (int m = 0; m < MT; ++m) {  // phase 2: nb, then nin_c
      const int gy = ty0 + wave * MT + m;
      const bool ok = gy < a.OH && gx < a.OW;
      const long pix = ((long)n * a.OH + gy) * a.OW + gx;
      f32x4 v[NT];
      gemm96(lds, acc[m], v);
#pragma unroll
      for (int f = 0; f < NT; ++f) {
        bias_act(v[f], *reinterpret_cast<const float4*>(hd.bb + f * 16 + 4 * lg));
        if (hd.nb && ok) save(hd.nb, pix, f, v[f]);
      }
      // nin_c: per-lane partial over its 24 channels, then across the 4 lane groups
      for (int o = 0; o < hd.oc; ++o) {
        float t = 0.f;
#pragma unroll
        for (int f = 0; f < NT; ++f) {
          const float4 w = *reinterpret_cast<const float4*>(hd.wc + o * 96 + f * 16 + 4 * lg);
          t = fmaf(w.x, v[f][0], t); t = fmaf(w.y, v[f][1], t);
          t = fmaf(w.z, v[f][2], t); t = fmaf(w.w, v[f][3], t);
        }
        t += __shfl_xor(t, 16);
        t += __shfl_xor(t, 32);
        if (lg == 0 && ok) hd.y[(((long)n * hd.oc + o) * a.OH + gy) * a.OW + gx] = t + hd.bc[o];
      }
    }
}

template <int GATHER, int NT, int MT, bool HEAD = false>
__global__ __launch_bounds__(256, (GATHER == G_C3 && NT == 6) ? 3 : 2) void k_fwd(
    FwdArgs a, HeadArgs hd) {
  using C = FwdCfg<GATHER, NT, MT>;
  __shared__ __attribute__((aligned(16))) float lds[HEAD ? C::LTOT : C::LT0];
  float* lx = lds;
  float* lw0 = lds + C::LX;
  float* lw1 = lw0 + C::NZ * C::LW;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const int tiles_x = (a.OW + C::TW - 1) / C::TW;
  int bxr, byr;  // XCD-aware tile order (conv_epi.h xcd_tile)
  xcd_tile(bxr, byr);
  const int ty0 = (bxr / tiles_x) * C::TH;
  const int tx0 = (bxr % tiles_x) * C::TW;
  const int n = byr;
  const int iy0 = GATHER == G_C3 ? ty0 - 1 : (GATHER == G_DN2 ? 2 * ty0 : ty0);
  const int ix0 = GATHER == G_C3 ? tx0 - 1 : (GATHER == G_DN2 ? 2 * tx0 : tx0);
  const float* inb = a.in + (long)n * a.IHt * a.IWt * a.in_stride + a.in_off;
  const float* wp = a.wp + (long)blockIdx.z * a.wp_z;
  const bool vec = ((a.in_stride | a.in_off) & 3) == 0;
  const int nch = (a.K + C::KC - 1) / C::KC;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < NT; ++q) acc[m][q] = f32x4{0.f, 0.f, 0.f, 0.f};

  float4 xr[C::XITEMS];
  auto load_x = [&](int k0) {
#pragma unroll
    for (int it = 0; it < C::XITEMS; ++it) {
      const int e = tid + it * 256;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < C::XQ) {
        const int q = e % C::QPP, pix = e / C::QPP;
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
        const int q = e % C::QPP, pix = e / C::QPP;
        float* d = lx + 4 * q * C::XCS + pix;
        d[0] = xr[it].x;
        d[C::XCS] = xr[it].y;
        d[2 * C::XCS] = xr[it].z;
        d[3 * C::XCS] = xr[it].w;
      }
    }
  };
  auto load_w = [&](int c, float* dst) {
    if constexpr (GATHER == G_UP) {  // the 4 parity images of chunk c, back to back
      constexpr int PP = C::LW / 256;
#pragma unroll
      for (int p = wave; p < C::NZ * PP; p += 4)
        glds16(a.wp + (long)(p / PP) * a.wp_z + (long)c * C::LW + (p % PP) * 256 + lane * 4,
               dst + p * 256);
    } else {
      const float* src = wp + (long)c * C::LW;
#pragma unroll
      for (int p = wave; p < C::LW / 256; p += 4) glds16(src + p * 256 + lane * 4, dst + p * 256);
    }
  };

  load_w(0, lw0);
  load_x(0);
  store_x();
  __syncthreads();

  for (int c = 0; c < nch; ++c) {
    const float* lw = (c & 1) ? lw1 : lw0;
    if (c + 1 < nch) {  // prefetch the next chunk while this one computes
      load_w(c + 1, (c & 1) ? lw0 : lw1);
      load_x((c + 1) * C::KC);
    }
#pragma unroll
    for (int t = 0; t < C::TAPS; ++t) {
#pragma unroll
      for (int s = 0; s < C::KC / 4; ++s) {
        const int kk = 4 * s + lg;
        float av[MT], bv[NT];
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const int r = GATHER == G_UP ? m : wave * MT + m;
          int off;
          if (GATHER == G_C3) off = (r + t / 3) * C::IW + li + t % 3;
          else if (GATHER == G_DN2) off = (2 * r + t / 2) * C::IW + 2 * li + (t & 1);
          else off = r * C::IW + li;
          av[m] = lx[kk * C::XCS + off];
        }
#pragma unroll
        for (int q = 0; q < NT; ++q)
          bv[q] = lw[(GATHER == G_UP ? wave * C::LW : 0) + (t * C::KC + kk) * C::WNS + q * 16 + li];
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int q = 0; q < NT; ++q)  // HEAD keeps the transposed tile (rows = channels)
            acc[m][q] = HEAD ? mfma4(bv[q], av[m], acc[m][q]) : mfma4(av[m], bv[q], acc[m][q]);
      }
    }
    __syncthreads();  // all waves done with lx and this weight buffer
    if (c + 1 < nch) store_x();
    __syncthreads();  // next chunk's input tile written, its weight DMA landed (vmcnt(0))
  }

  if constexpr (HEAD) {
    // acc[m][q][r] = dec_conv1b pre-activation at pixel (row m, x = li), channel
    // q*16 + 4*lg + r.  As the B operand of the next 16x16x4 MFMA, register r of fragment q
    // supplies k = channel q*16 + 4g + r for lane group g: nin_a/nin_b consume the tile
    // where it is, with the k order permuted the same way in their weight reads.
    static_assert(GATHER == G_C3 && NT == 6, "head fusion is for the 96-channel dec_conv1b");
    // Two phases through ONE image slot (38 KiB, so three workgroups fit a CU): nin_a for
    // all rows in place (acc <- na), then nin_b + nin_c.
    for (int p = wave; p < HEAD_LW / 256; p += 4) glds16(hd.wp + p * 256 + lane * 4, lds + p * 256);
    auto bias_act = [](f32x4& v, float4 b) {
      v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * 0.2f;
    };
    auto save = [&](float* dst, long pix, int q, const f32x4& v) {
      *reinterpret_cast<float4*>(dst + pix * 96 + q * 16 + 4 * lg) = make_float4(v[0], v[1], v[2], v[3]);
    };
    // 1x1 GEMM on the transposed tile: out[f] = W^T-image x in (k order = the tile's)
    auto gemm96 = [&](const float* w, const f32x4 (&in)[NT], f32x4 (&out)[NT]) {
#pragma unroll
      for (int f = 0; f < NT; ++f) out[f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < NT; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float* wr = w + (q * 16 + 4 * lg + r) * HEAD_WS + li;
#pragma unroll
          for (int f = 0; f < NT; ++f) out[f] = mfma4(wr[f * 16], in[q][r], out[f]);
        }
    };
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      const float4 b = *reinterpret_cast<const float4*>(a.bias + q * 16 + 4 * lg);
#pragma unroll
      for (int m = 0; m < MT; ++m) bias_act(acc[m][q], b);
    }
    const int gx = tx0 + li;
    if (hd.d1b) {
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int gy = ty0 + wave * MT + m;
        if (gy < a.OH && gx < a.OW)
#pragma unroll
          for (int q = 0; q < NT; ++q) save(hd.d1b, ((long)n * a.OH + gy) * a.OW + gx, q, acc[m][q]);
      }
    }
    __syncthreads();  // nin_a image landed
#pragma unroll
    for (int m = 0; m < MT; ++m) {  // phase 1: acc[m] <- na
      const int gy = ty0 + wave * MT + m;
      f32x4 u[NT];
      gemm96(lds, acc[m], u);
#pragma unroll
      for (int f = 0; f < NT; ++f) {
        bias_act(u[f], *reinterpret_cast<const float4*>(hd.ba + f * 16 + 4 * lg));
        acc[m][f] = u[f];
      }
      if (hd.na && gy < a.OH && gx < a.OW)
#pragma unroll
        for (int f = 0; f < NT; ++f) save(hd.na, ((long)n * a.OH + gy) * a.OW + gx, f, acc[m][f]);
    }
    __syncthreads();  // everyone done with nin_a
    for (int p = wave; p < HEAD_LW / 256; p += 4)
      glds16(hd.wp + HEAD_LW + p * 256 + lane * 4, lds + p * 256);
    __syncthreads();  // nin_b image landed
#pragma unroll
    for (int m = 0; m < MT; ++m) {  // phase 2: nb, then nin_c
      const int gy = ty0 + wave * MT + m;
      const bool ok = gy < a.OH && gx < a.OW;
      const long pix = ((long)n * a.OH + gy) * a.OW + gx;
      f32x4 v[NT];
      gemm96(lds, acc[m], v);
#pragma unroll
      for (int f = 0; f < NT; ++f) {
        bias_act(v[f], *reinterpret_cast<const float4*>(hd.bb + f * 16 + 4 * lg));
        if (hd.nb && ok) save(hd.nb, pix, f, v[f]);
      }
      // nin_c: per-lane partial over its 24 channels, then across the 4 lane groups
      for (int o = 0; o < hd.oc; ++o) {
        float t = 0.f;
#pragma unroll
        for (int f = 0; f < NT; ++f) {
          const float4 w = *reinterpret_cast<const float4*>(hd.wc + o * 96 + f * 16 + 4 * lg);
          t = fmaf(w.x, v[f][0], t); t = fmaf(w.y, v[f][1], t);
          t = fmaf(w.z, v[f][2], t); t = fmaf(w.w, v[f][3], t);
        }
        t += __shfl_xor(t, 16);
        t += __shfl_xor(t, 32);
        if (lg == 0 && ok) hd.y[(((long)n * hd.oc + o) * a.OH + gy) * a.OW + gx] = t + hd.bc[o];
      }
    }
    return;
  } else {
    fwd_epilogue<NT, MT, C::PS, GATHER == G_UP>(a, acc, lds, ty0, tx0, n);
  }
}

// The same head on an already activated dec_conv1b output (hd.d1b ignored; a.in = d1b NHWC,
// stride 96): the head of a forward whose dec_conv1b ran on another kernel (bf16x6).
template <int MT>
__global__ __launch_bounds__(256, 2) void k_nin_head(FwdArgs a, HeadArgs hd) {
  __shared__ __attribute__((aligned(16))) float lds[HEAD_LW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const int tiles_x = (a.OW + 15) / 16;
  const int ty0 = (blockIdx.x / tiles_x) * 4 * MT, tx0 = (blockIdx.x % tiles_x) * 16;
  const int n = blockIdx.y, gx = tx0 + li;
  f32x4 acc[MT][6];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int gy = ty0 + wave * MT + m;
    const bool ok = gy < a.OH && gx < a.OW;
    const float* p = a.in + (((long)n * a.IHt + gy) * a.IWt + gx) * a.in_stride + a.in_off + 4 * lg;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const float4 v = ok ? *reinterpret_cast<const float4*>(p + q * 16) : make_float4(0.f, 0.f, 0.f, 0.f);
      acc[m][q] = f32x4{v.x, v.y, v.z, v.w};
    }
  }
  head_tail<MT, false>(a, hd, acc, lds, ty0, tx0, n);
}

// Backward of the fused head (see HeadBwdArgs).  A workgroup loads the two transposed 1x1
// images once and walks 64*MT-pixel chunks; per 16-pixel fragment the three data gradients
// stay in registers in the transposed (channel-row) MFMA layout, as in the forward head.
template <int MT, int NWV>
__global__ __launch_bounds__(NWV * 64, 2) void k_head_bwd(HeadBwdArgs h) {
  __shared__ __attribute__((aligned(16))) float lds[2 * HEAD_LW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;
  for (int p = wave; p < 2 * HEAD_LW / 256; p += NWV) glds16(h.wp + p * 256 + lane * 4, lds + p * 256);
  __syncthreads();
  auto ld4 = [](const float* p) { return *reinterpret_cast<const float4*>(p); };
  auto st4 = [](float* p, const f32x4& v) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  };
  auto mask = [](f32x4& v, float4 m) {
    v[0] = m.x > 0.f ? v[0] : v[0] * 0.2f; v[1] = m.y > 0.f ? v[1] : v[1] * 0.2f;
    v[2] = m.z > 0.f ? v[2] : v[2] * 0.2f; v[3] = m.w > 0.f ? v[3] : v[3] * 0.2f;
  };
  const long nchunks = (h.npx + 16 * NWV * MT - 1) / (16 * NWV * MT);
  for (long ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
#pragma unroll 1
    for (int m = 0; m < MT; ++m) {
      // loop-variant zero: keeps the (loop-invariant) LDS weight reads inside the loop
      // instead of hoisting 144 of them into registers
      int lz = 0;
      asm volatile("" : "+v"(lz));
      const float* wbT = lds + lz;
      const float* waT = lds + HEAD_LW + lz;
      const long px = ch * 16 * NWV * MT + (wave * MT + m) * 16 + li;
      const bool ok = px < h.npx;
      const long pc = ok ? px : 0;
      // g_nb (VALU: K = oc)
      f32x4 t[6];
#pragma unroll
      for (int q = 0; q < 6; ++q) t[q] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int o = 0; o < h.oc; ++o) {
        const float d = ok ? h.dy[pc * h.dy_stride + o] : 0.f;
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          const float4 w = ld4(h.wc + o * 96 + q * 16 + 4 * lg);
          t[q][0] = fmaf(w.x, d, t[q][0]); t[q][1] = fmaf(w.y, d, t[q][1]);
          t[q][2] = fmaf(w.z, d, t[q][2]); t[q][3] = fmaf(w.w, d, t[q][3]);
        }
      }
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        mask(t[q], ld4(h.nb + pc * 96 + q * 16 + 4 * lg));
        if (ok) st4(h.g_nb + px * 96 + q * 16 + 4 * lg, t[q]);
      }
      // g_na = leaky'(na) * Wb^T g_nb
      f32x4 u[6];
#pragma unroll
      for (int f = 0; f < 6; ++f) u[f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 6; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float* wr = wbT + (q * 16 + 4 * lg + r) * HEAD_WS + li;
#pragma unroll
          for (int f = 0; f < 6; ++f) u[f] = mfma4(wr[f * 16], t[q][r], u[f]);
        }
#pragma unroll
      for (int f = 0; f < 6; ++f) {
        mask(u[f], ld4(h.na + pc * 96 + f * 16 + 4 * lg));
        if (ok) st4(h.g_na + px * 96 + f * 16 + 4 * lg, u[f]);
      }
      // g_d1b = leaky'(d1b) * Wa^T g_na
#pragma unroll
      for (int f = 0; f < 6; ++f) t[f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 6; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float* wr = waT + (q * 16 + 4 * lg + r) * HEAD_WS + li;
#pragma unroll
          for (int f = 0; f < 6; ++f) t[f] = mfma4(wr[f * 16], u[q][r], t[f]);
        }
#pragma unroll
      for (int f = 0; f < 6; ++f) {
        mask(t[f], ld4(h.d1b + pc * 96 + f * 16 + 4 * lg));
        if (ok) st4(h.g_d1b + px * 96 + f * 16 + 4 * lg, t[f]);
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// Weight gradient.  MFMA M = output channels (gradient operand G), N = input channels x
// taps (input operand X), K = pixels.  One workgroup = all output channels x 16*CIF input
// channels x all taps, accumulated over a contiguous range of pixel chunks (a "split");
// it writes its partial dW/db into slab[split]; k_reduce_batch sums the slabs in a fixed order.
//   LDS keeps both operands in their natural NHWC order: G chunk [pixel][GS] and the input
//   chunk (with halo for 3x3) [pixel][XS]; the strides make the 16x16x4 fragment reads
//   conflict-free.  The next chunk is prefetched into registers (float4 along channels)
//   while the current one computes.  The bias gradient rides along as one extra MFMA per
//   k-step against a ones vector (only in the workgroups of input-channel block 0).
// ------------------------------------------------------------------------------------
template <int MODE, int MF, int NW, int CIF>
struct WgCfg {
  static constexpr int TAPS = MODE == W_C3 ? 9 : (MODE == W_UP2 ? 4 : 1);
  static constexpr int PR = (MODE == W_UP2 || MF >= 2) ? 1 : 2;
  static constexpr int PC = MODE == W_UP2 ? 16 : 32;
  static constexpr int NPIX = PR * PC;                 // K-pixels per chunk
  static constexpr int COP = MF * NW * 16;             // output channels (padded)
  static constexpr int GH = MODE == W_UP2 ? 2 * PR : PR, GW = MODE == W_UP2 ? 2 * PC : PC;
  static constexpr int GS = cround(COP, 32, MODE == W_UP2 ? 8 : 16);
  static constexpr int XH = MODE == W_C3 ? PR + 2 : PR, XW = MODE == W_C3 ? PC + 2 : PC;
  static constexpr int CIN_T = 16 * CIF;
  static constexpr int XS = cround(CIN_T, 32, 16);
  static constexpr int NF = TAPS * CIF;
  static constexpr int LG = GH * GW * GS, LX = XH * XW * XS;
  static constexpr int NTHR = NW * 64;
  static constexpr int GQ = GH * GW * (COP / 4), XQ = XH * XW * (CIN_T / 4);  // float4 items
  static constexpr int GITEMS = (GQ + NTHR - 1) / NTHR, XITEMS = (XQ + NTHR - 1) / NTHR;
};

template <int MODE, int MF, int NW, int CIF>
// (occupancy targets the register allocation reaches: k_wgrad<W_C1, 1, 1, 2> holds two input-
// channel fragments per wave and gets 3 waves per SIMD, not 4)
__global__ __launch_bounds__(NW * 64, MF >= 2 || CIF >= 2 ? 3 : 4) void k_wgrad(WgradArgs a0) {
  using C = WgCfg<MODE, MF, NW, CIF>;
  const WgradArgs a = wg_block(a0);
  __shared__ __attribute__((aligned(16))) float lds[C::LG + C::LX];
  float* lg_ = lds;
  float* lx = lds + C::LG;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lgp = lane >> 4;
  const int ci0 = blockIdx.y * C::CIN_T;
  const int ux = (a.KW + C::PC - 1) / C::PC, uy = (a.KH + C::PR - 1) / C::PR;
  const long U = (long)a.N * uy * ux;
  const long u_beg = U * blockIdx.x / gridDim.x, u_end = U * (blockIdx.x + 1) / gridDim.x;
  const int GHt = MODE == W_UP2 ? 2 * a.KH : a.KH, GWt = MODE == W_UP2 ? 2 * a.KW : a.KW;
  const bool do_bias = a.bias && blockIdx.y == 0;
  const bool gvec = ((a.g_stride | a.g_off) & 3) == 0;
  const bool xvec = ((a.x_stride | a.x_off) & 3) == 0;

  f32x4 acc[MF][C::NF];
  f32x4 accb[MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) {
    accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int f = 0; f < C::NF; ++f) acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  float4 gr[C::GITEMS], xr[C::XITEMS];
  auto load = [&](long u) {
    const int n = (int)(u / ((long)uy * ux));
    const int rem = (int)(u - (long)n * uy * ux);
    const int py0 = (rem / ux) * C::PR, px0 = (rem % ux) * C::PC;
    const int gy0 = MODE == W_UP2 ? 2 * py0 : py0, gx0 = MODE == W_UP2 ? 2 * px0 : px0;
    const float* gb = a.g + (long)n * GHt * GWt * a.g_stride + a.g_off;
#pragma unroll
    for (int it = 0; it < C::GITEMS; ++it) {
      const int e = tid + it * C::NTHR;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < C::GQ) {
        const int q = e % (C::COP / 4), pix = e / (C::COP / 4);
        const int y = pix / C::GW, x = pix - y * C::GW;
        const int gy = gy0 + y, gx = gx0 + x, co = 4 * q;
        if (gy < GHt && gx < GWt && co < a.Cout) {
          const float* p = gb + ((long)gy * GWt + gx) * a.g_stride + co;
          if (gvec && co + 4 <= a.Cout) {
            v = *reinterpret_cast<const float4*>(p);
          } else {
            v.x = p[0];
            if (co + 1 < a.Cout) v.y = p[1];
            if (co + 2 < a.Cout) v.z = p[2];
            if (co + 3 < a.Cout) v.w = p[3];
          }
        }
      }
      gr[it] = v;
    }
    const int xy0 = MODE == W_C3 ? py0 - 1 : py0, xx0 = MODE == W_C3 ? px0 - 1 : px0;
    const float* xb = a.x + (long)n * a.KH * a.KW * a.x_stride + a.x_off;
#pragma unroll
    for (int it = 0; it < C::XITEMS; ++it) {
      const int e = tid + it * C::NTHR;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < C::XQ) {
        const int q = e % (C::CIN_T / 4), pix = e / (C::CIN_T / 4);
        const int y = pix / C::XW, x = pix - y * C::XW;
        const int gy = xy0 + y, gx = xx0 + x, ci = ci0 + 4 * q;
        if (gy >= 0 && gy < a.KH && gx >= 0 && gx < a.KW && ci < a.Cin) {
          const float* p = xb + ((long)gy * a.KW + gx) * a.x_stride + ci;
          if (xvec && ci + 4 <= a.Cin) {
            v = *reinterpret_cast<const float4*>(p);
          } else {
            v.x = p[0];
            if (ci + 1 < a.Cin) v.y = p[1];
            if (ci + 2 < a.Cin) v.z = p[2];
            if (ci + 3 < a.Cin) v.w = p[3];
          }
        }
      }
      xr[it] = v;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int it = 0; it < C::GITEMS; ++it) {
      const int e = tid + it * C::NTHR;
      if (e < C::GQ) {
        const int q = e % (C::COP / 4), pix = e / (C::COP / 4);
        *reinterpret_cast<float4*>(lg_ + pix * C::GS + 4 * q) = gr[it];
      }
    }
#pragma unroll
    for (int it = 0; it < C::XITEMS; ++it) {
      const int e = tid + it * C::NTHR;
      if (e < C::XQ) {
        const int q = e % (C::CIN_T / 4), pix = e / (C::CIN_T / 4);
        *reinterpret_cast<float4*>(lx + pix * C::XS + 4 * q) = xr[it];
      }
    }
  };

  if (u_beg < u_end) {
    load(u_beg);
    store();
  }
  __syncthreads();
  for (long u = u_beg; u < u_end; ++u) {
    if (u + 1 < u_end) load(u + 1);
#pragma unroll 1
    for (int ks = 0; ks < C::NPIX / 4; ++ks) {
      const int pr = (4 * ks) / C::PC;
      const int pc = (4 * ks) % C::PC + lgp;  // this lane's pixel (k = lane>>4)
      float av[MF][MODE == W_UP2 ? 4 : 1];
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        const int co = (wave * MF + i) * 16 + li;
        if (MODE == W_UP2) {
#pragma unroll
          for (int t = 0; t < 4; ++t)
            av[i][t] = lg_[((2 * pr + (t >> 1)) * C::GW + 2 * pc + (t & 1)) * C::GS + co];
        } else {
          av[i][0] = lg_[(pr * C::PC + pc) * C::GS + co];
        }
      }
#pragma unroll
      for (int f = 0; f < C::NF; ++f) {
        const int tap = f / CIF, cf = f % CIF;
        float bv;
        if (MODE == W_C3)
          bv = lx[((pr + tap / 3) * C::XW + pc + tap % 3) * C::XS + cf * 16 + li];
        else
          bv = lx[(pr * C::XW + pc) * C::XS + cf * 16 + li];
#pragma unroll
        for (int i = 0; i < MF; ++i)
          acc[i][f] = mfma4(av[i][MODE == W_UP2 ? tap : 0], bv, acc[i][f]);
      }
      if (do_bias) {
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
          for (int t = 0; t < (MODE == W_UP2 ? 4 : 1); ++t) accb[i] = mfma4(av[i][t], 1.0f, accb[i]);
      }
    }
    __syncthreads();
    if (u + 1 < u_end) store();
    __syncthreads();
  }

  float* slab = a.slab + (long)blockIdx.x * a.slab_stride;
  const int cot = a.cout_total ? a.cout_total : a.Cout;
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int f = 0; f < C::NF; ++f) {
      const int tap = f / CIF, cf = f % CIF;
      const int ci = ci0 + cf * 16 + li;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = (wave * MF + i) * 16 + 4 * lgp + r;
        if (co < a.Cout && ci < a.Cin) {
          const long widx =
              a.wlayout == 0 ? ((long)(a.co_base + co) * a.cin_total + a.ci_base + ci) * C::TAPS + tap
                             : ((long)(a.ci_base + ci) * cot + a.co_base + co) * C::TAPS + tap;
          slab[widx] = acc[i][f][r];
        }
      }
    }
  if (do_bias && li == 0) {
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = (wave * MF + i) * 16 + 4 * lgp + r;
        if (co < a.Cout) slab[(long)cot * a.cin_total * C::TAPS + a.co_base + co] = accb[i][r];
      }
  }
}

// ------------------------------------------------------------------------------------
// 3x3 weight gradient, asynchronous staging.  Workgroup = all Cout (16*CO_FR) x CIB = 16*WN
// input channels x 9 taps; wave (wm, wn) owns CO_FR/WM output-channel fragments x the 16
// input channels wn x 9 taps = 27 MFMA tiles.  Each K stage is one image row segment of 32
// pixels: both operands are copied by per-lane-addressed global_load_lds_dwordx4 (padding
// and out-of-image halo read a zero buffer) into one of two LDS buffers while the other is
// consumed -- one barrier per stage, no staging registers.
// ------------------------------------------------------------------------------------
template <int CO_FR, int WM, int WN>
struct Wg3Cfg {
  static constexpr int COUT = 16 * CO_FR, MFW = CO_FR / WM, CIB = 16 * WN;
  static constexpr int NW = WM * WN, NTHR = 64 * NW;
  static constexpr int PC = 32, XW = PC + 2, XH = 3;
  static constexpr int LGF = PC * COUT;                               // G floats per stage
  static constexpr int LXF = (XH * XW * CIB + 255) / 256 * 256;       // X floats per stage
  static constexpr int LGP = LGF / 256, LXP = LXF / 256;              // 1 KiB DMA pieces
  static constexpr int LBUF = LGF + LXF;
  static_assert(LGF % 256 == 0, "G stage must be whole 1 KiB pieces");
};

template <int CO_FR, int WM, int WN, int SWL = 5>
// (k_wgrad3<2, 1, 2 or 4, *>, the 32-output ImprovedUNet blocks with 32 / 64 input channels per
// workgroup: 2 waves per SIMD is what its registers allow)
__global__ __launch_bounds__(64 * WM * WN, CO_FR == 2 && WN != 3 ? 2 : 3) void k_wgrad3(WgradArgs a0) {
  using C = Wg3Cfg<CO_FR, WM, WN>;
  const WgradArgs a = wg_block(a0);
  __shared__ __attribute__((aligned(16))) float lds[2 * C::LBUF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int li = lane & 15, lgp = lane >> 4;
  const int ci0 = blockIdx.y * C::CIB;
  // K stage = 32 pixels: one row segment of 32, or (images narrower than 32 with KW a power of
  // two) a block of 32/KW whole rows, so narrow deep levels do not run 3/4 empty stages
  constexpr int swl = SWL, sw = 1 << SWL, sh = C::PC >> SWL, xw = sw + 2;
  const int ux = (a.KW + sw - 1) / sw, uy = (a.KH + sh - 1) / sh;
  const long U = (long)a.N * uy * ux;
  const long u_beg = U * blockIdx.x / gridDim.x, u_end = U * (blockIdx.x + 1) / gridDim.x;
  const bool do_bias = a.bias && blockIdx.y == 0 && wn == 0;

  f32x4 acc[C::MFW][9];
  f32x4 accb[C::MFW];
#pragma unroll
  for (int i = 0; i < C::MFW; ++i) {
    accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  auto issue = [&](long u, float* buf) {
    const int n = (int)(u / ((long)uy * ux));
    const int rem = (int)(u - (long)n * uy * ux);
    const int py0 = (rem / ux) * sh, px0 = (rem % ux) * sw;
    const float* gb = a.g + (long)n * a.KH * a.KW * a.g_stride + a.g_off;
    for (int p = wave; p < C::LGP; p += C::NW) {
      const int idx = p * 256 + lane * 4;
      const int px = idx / C::COUT, co = idx - px * C::COUT;
      const int gy = py0 + (px >> swl), gx = px0 + (px & (sw - 1));
      const float* src = (gy < a.KH && gx < a.KW && co < a.Cout)
                             ? gb + ((long)gy * a.KW + gx) * a.g_stride + co : a.zeros;
      glds16(src, buf + p * 256);
    }
    const float* xb = a.x + (long)n * a.KH * a.KW * a.x_stride + a.x_off;
    const int xpix = (sh + 2) * xw;
    for (int p = wave; p < C::LXP; p += C::NW) {
      const int idx = p * 256 + lane * 4;
      const int px = idx / C::CIB, q = idx - px * C::CIB;
      const int yy = px / xw, xx = px - yy * xw;
      const int gy = py0 - 1 + yy, gx = px0 - 1 + xx, ci = ci0 + q;
      const bool ok = px < xpix && gy >= 0 && gy < a.KH && gx >= 0 && gx < a.KW && ci < a.Cin;
      const float* src = ok ? xb + ((long)gy * a.KW + gx) * a.x_stride + ci : a.zeros;
      glds16(src, buf + C::LGF + p * 256);
    }
  };

  if (u_beg < u_end) issue(u_beg, lds);
  __syncthreads();
  for (long u = u_beg; u < u_end; ++u) {
    const int cb = (int)((u - u_beg) & 1);
    const float* lg_ = lds + cb * C::LBUF;
    const float* lx = lg_ + C::LGF;
    if (u + 1 < u_end) issue(u + 1, lds + (cb ^ 1) * C::LBUF);
#pragma unroll 2
    for (int ks = 0; ks < C::PC / 4; ++ks) {
      const int pc = 4 * ks + lgp;  // this lane's pixel (k = lane>>4)
      const int pr = pc >> swl, pcc = pc & (sw - 1);
      float av[C::MFW];
#pragma unroll
      for (int i = 0; i < C::MFW; ++i)
        av[i] = lg_[pc * C::COUT + (wm * C::MFW + i) * 16 + li];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const float bv = lx[((pr + t / 3) * xw + pcc + t % 3) * C::CIB + wn * 16 + li];
#pragma unroll
        for (int i = 0; i < C::MFW; ++i) acc[i][t] = mfma4(av[i], bv, acc[i][t]);
      }
      if (do_bias) {
#pragma unroll
        for (int i = 0; i < C::MFW; ++i) accb[i] = mfma4(av[i], 1.0f, accb[i]);
      }
    }
    __syncthreads();  // next stage landed (vmcnt(0)); everyone done with this buffer
  }

  float* slab = a.slab + (long)blockIdx.x * a.slab_stride;
  const int ci = ci0 + wn * 16 + li;
  const int cot = a.cout_total ? a.cout_total : a.Cout;
#pragma unroll
  for (int i = 0; i < C::MFW; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = (wm * C::MFW + i) * 16 + 4 * lgp + r;
        if (co < a.Cout && ci < a.Cin)
          slab[((long)(a.co_base + co) * a.cin_total + a.ci_base + ci) * 9 + t] = acc[i][t][r];
      }
  if (do_bias && li == 0) {
#pragma unroll
    for (int i = 0; i < C::MFW; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = (wm * C::MFW + i) * 16 + 4 * lgp + r;
        if (co < a.Cout) slab[(long)cot * a.cin_total * 9 + a.co_base + co] = accb[i][r];
      }
  }
}

// ------------------------------------------------------------------------------------
// 1x1 / deconv-2x2 weight gradient (nin_a, nin_b: arch_unet.py:186-189; up_k.deconv:
// arch_unet.py:57).  M = output channels, N = ALL input channels, K = pixels: one workgroup
// owns the whole Cout x Cin matrix for a contiguous range of 32-pixel row segments, so each
// operand byte is read from HBM once.  Both operands are copied by per-lane addressed
// global_load_lds_dwordx4 into double-buffered LDS ([px][Cout] and [px][Cin]), one barrier
// per stage; the bias rides along as an MFMA against ones.
//   deconv (up2 != 0): blockIdx.z = (a,b) parity; the gradient operand of low-res pixel
//   (y, x) is g at (2y+a, 2x+b) of the 2KH x 2KW image.  Slab row r = z*splits + split holds
//   [W_ab | b_ab] and the launcher reduces per parity (scattered into (in,out,2,2)) and the
//   bias over all rows.
// ------------------------------------------------------------------------------------
template <int CO_FR, int CI_FR, int WM, int WN>
struct Wg1Cfg {
  static constexpr int COUT = 16 * CO_FR, CIN = 16 * CI_FR;
  static constexpr int MFW = CO_FR / WM, NFW = CI_FR / WN;
  static constexpr int NW = WM * WN, NTHR = 64 * NW;
  static constexpr int PC = 32;
  static constexpr int LGF = PC * COUT, LXF = PC * CIN;
  static constexpr int LGP = LGF / 256, LXP = LXF / 256;
  static constexpr int LBUF = LGF + LXF;
  static_assert(LGF % 256 == 0 && LXF % 256 == 0, "whole 1 KiB DMA pieces");
};

template <int CO_FR, int CI_FR, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN, 3) void k_wgrad1(WgradArgs a0, int up2) {
  using C = Wg1Cfg<CO_FR, CI_FR, WM, WN>;
  // 1x1 (up2 == 0) with a.zc > 0: blockIdx.z = output-channel block, blockIdx.y = input-channel
  // block of C::CIN; all blocks of a split write one slab row
  const WgradArgs a = up2 ? a0 : wg_block(a0);
  const int ci0 = up2 ? 0 : (int)blockIdx.y * C::CIN;
  __shared__ __attribute__((aligned(16))) float lds[2 * C::LBUF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int li = lane & 15, lgp = lane >> 4;
  const int ux = (a.KW + C::PC - 1) / C::PC;
  const long U = (long)a.N * a.KH * ux;
  const long u_beg = U * blockIdx.x / gridDim.x, u_end = U * (blockIdx.x + 1) / gridDim.x;
  const bool do_bias = wn == 0 && blockIdx.y == 0;
  const int pa = up2 ? (int)(blockIdx.z >> 1) : 0, pb = up2 ? (int)(blockIdx.z & 1) : 0;
  const int GH = up2 ? 2 * a.KH : a.KH, GW = up2 ? 2 * a.KW : a.KW, sc = up2 ? 2 : 1;

  f32x4 acc[C::MFW][C::NFW];
  f32x4 accb[C::MFW];
#pragma unroll
  for (int i = 0; i < C::MFW; ++i) {
    accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < C::NFW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  auto issue = [&](long u, float* buf) {
    const int n = (int)(u / ((long)a.KH * ux));
    const int rem = (int)(u - (long)n * a.KH * ux);
    const int py = rem / ux, px0 = (rem % ux) * C::PC;
    const float* gb = a.g + ((long)n * GH + sc * py + pa) * GW * a.g_stride + a.g_off;
    for (int p = wave; p < C::LGP; p += C::NW) {
      const int idx = p * 256 + lane * 4;
      const int px = idx / C::COUT, co = idx - px * C::COUT;
      const int gx = px0 + px;
      const float* src = (gx < a.KW && co < a.Cout) ? gb + (long)(sc * gx + pb) * a.g_stride + co
                                                     : a.zeros;
      glds16(src, buf + p * 256);
    }
    const float* xb = a.x + ((long)n * a.KH + py) * a.KW * a.x_stride + a.x_off;
    for (int p = wave; p < C::LXP; p += C::NW) {
      const int idx = p * 256 + lane * 4;
      const int px = idx / C::CIN, ci = ci0 + idx - px * C::CIN;
      const int gx = px0 + px;
      const float* src = (gx < a.KW && ci < a.Cin) ? xb + (long)gx * a.x_stride + ci : a.zeros;
      glds16(src, buf + C::LGF + p * 256);
    }
  };

  if (u_beg < u_end) issue(u_beg, lds);
  __syncthreads();
  for (long u = u_beg; u < u_end; ++u) {
    const int cb = (int)((u - u_beg) & 1);
    const float* lg_ = lds + cb * C::LBUF;
    const float* lx = lg_ + C::LGF;
    if (u + 1 < u_end) issue(u + 1, lds + (cb ^ 1) * C::LBUF);
#pragma unroll 2
    for (int ks = 0; ks < C::PC / 4; ++ks) {
      const int pc = 4 * ks + lgp;  // this lane's pixel (k = lane>>4)
      float av[C::MFW], bv[C::NFW];
#pragma unroll
      for (int i = 0; i < C::MFW; ++i) av[i] = lg_[pc * C::COUT + (wm * C::MFW + i) * 16 + li];
#pragma unroll
      for (int j = 0; j < C::NFW; ++j) bv[j] = lx[pc * C::CIN + (wn * C::NFW + j) * 16 + li];
#pragma unroll
      for (int i = 0; i < C::MFW; ++i)
#pragma unroll
        for (int j = 0; j < C::NFW; ++j) acc[i][j] = mfma4(av[i], bv[j], acc[i][j]);
      if (do_bias) {
#pragma unroll
        for (int i = 0; i < C::MFW; ++i) accb[i] = mfma4(av[i], 1.0f, accb[i]);
      }
    }
    __syncthreads();  // next stage landed (vmcnt(0)); everyone done with this buffer
  }

  const long row = up2 ? (long)blockIdx.z * gridDim.x + blockIdx.x : (long)blockIdx.x;
  float* slab = a.slab + row * a.slab_stride;
  const int cot = a.zc > 0 ? a.cout_total : a.Cout;
#pragma unroll
  for (int i = 0; i < C::MFW; ++i)
#pragma unroll
    for (int j = 0; j < C::NFW; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = (wm * C::MFW + i) * 16 + 4 * lgp + r;
        const int ci = ci0 + (wn * C::NFW + j) * 16 + li;
        if (co < a.Cout && ci < a.Cin)
          slab[a.wlayout ? (long)ci * a.Cout + co : (long)(a.co_base + co) * a.Cin + ci] = acc[i][j][r];
      }
  if (do_bias && li == 0) {
#pragma unroll
    for (int i = 0; i < C::MFW; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = (wm * C::MFW + i) * 16 + 4 * lgp + r;
        if (co < a.Cout) slab[(long)cot * a.Cin + a.co_base + co] = accb[i][r];
      }
  }
}

// out[omap(e)] = sum_s slab[s][imap(e)] in a fixed order (bit-reproducible): a workgroup owns
// 64 elements of one job, its four waves sum interleaved quarters of the rows (four loads in
// flight per lane), then wave 0 adds the four partials.  blockIdx.x -> job by the jobs' first
// workgroups (b0, increasing).
constexpr int RED_VF = 12;  // 16-B rows a lane keeps in flight (vector jobs)
// Vector jobs (j.vec, red_add): a lane owns FOUR consecutive elements, contiguous in every slab
// row, and reads them with one 16-byte load per row -- the same per-element summation order as
// the scalar form (bit-identical results) with a quarter of the load instructions and 4x the bytes
// in flight (the scalar form waited on its loads: SQ_WAIT_ANY 0.86, profiles/r5zz_pmc_sq_n2n.txt).
__global__ __launch_bounds__(256) void k_reduce_batch(RedBatch b) {
  __shared__ float part[4][64];
  __shared__ f32x4 part4[4][64];
  int jj = 0;
  for (int q = 1; q < b.n; ++q)
    if ((int)blockIdx.x >= b.j[q].b0) jj = q;
  const RedJob& j = b.j[jj];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (j.vec) {
    const long e = ((long)((int)blockIdx.x - j.b0) * 64 + lane) * 4;
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    if (e < j.n) {
      const f32x4* src = reinterpret_cast<const f32x4*>(j.slab + (e / j.ig) * j.is1 + e % j.ig);
      const long stride = j.stride / 4;
      int i = wave;
      for (; i + 4 * (RED_VF - 1) < j.splits; i += 4 * RED_VF) {  // RED_VF rows in flight
        f32x4 v[RED_VF];
#pragma unroll
        for (int k = 0; k < RED_VF; ++k) v[k] = src[(long)(i + 4 * k) * stride];
#pragma unroll
        for (int k = 0; k < RED_VF; ++k)
#pragma unroll
          for (int r = 0; r < 4; ++r) s[r] += v[k][r];
      }
      for (; i < j.splits; i += 4) {
        const f32x4 v = src[(long)i * stride];
#pragma unroll
        for (int r = 0; r < 4; ++r) s[r] += v[r];
      }
    }
    part4[wave][lane] = s;
    __syncthreads();
    if (wave == 0 && e < j.n) {
      const f32x4 p0 = part4[0][lane], p1 = part4[1][lane], p2 = part4[2][lane], p3 = part4[3][lane];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long er = e + r;
        j.out[(er / j.og) * j.os1 + j.ooff + er % j.og] = ((p0[r] + p1[r]) + p2[r]) + p3[r];
      }
    }
    return;
  }
  const long e = (long)((int)blockIdx.x - j.b0) * 64 + lane;
  float s = 0.f;
  if (e < j.n) {
    const float* src = j.slab + (e / j.ig) * j.is1 + (e % j.ig) * j.is2;
    const long stride = j.stride;
    int i = wave;
    for (; i + 12 < j.splits; i += 16) {  // four loads in flight per lane
      const float v0 = src[(long)i * stride], v1 = src[(long)(i + 4) * stride];
      const float v2 = src[(long)(i + 8) * stride], v3 = src[(long)(i + 12) * stride];
      s += v0; s += v1; s += v2; s += v3;
    }
    for (; i < j.splits; i += 4) s += src[(long)i * stride];
  }
  part[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && e < j.n)
    j.out[(e / j.og) * j.os1 + j.ooff + e % j.og] =
        ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
}

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
template <int GATHER, int NT, int MT>
static hipError_t run_fwd(const FwdArgs& a, hipStream_t s) {
  using C = FwdCfg<GATHER, NT, MT>;
  const int tx = (a.OW + C::TW - 1) / C::TW, ty = (a.OH + C::TH - 1) / C::TH;
  const int nz = a.zc ? (a.NOUT + a.zc - 1) / a.zc : ((a.out_layout == OUT_UP2 && GATHER != G_UP) ? 4 : 1);
  dim3 grid(tx * ty, a.N, nz);
  prof_kernel("k_fwd");
  hipLaunchKernelGGL((k_fwd<GATHER, NT, MT>), grid, dim3(256), 0, s, a, HeadArgs{});
  return hipGetLastError();
}

template <int MT>
static hipError_t run_head(const FwdArgs& a, const HeadArgs& h, hipStream_t s) {
  using C = FwdCfg<G_C3, 6, MT>;
  const int tx = (a.OW + C::TW - 1) / C::TW, ty = (a.OH + C::TH - 1) / C::TH;
  dim3 grid(tx * ty, a.N, 1);
  hipLaunchKernelGGL((k_fwd<G_C3, 6, MT, true>), grid, dim3(256), 0, s, a, h);
  return hipGetLastError();
}

hipError_t launch_head(const FwdArgs& a, const HeadArgs& h, hipStream_t s) {
  if (a.NOUT != 96 || h.oc < 1) return hipErrorInvalidValue;
  const long tiles = (long)a.N * ((a.OH + 15) / 16) * ((a.OW + 15) / 16);
  return tiles < 1024 ? run_head<1>(a, h, s) : run_head<4>(a, h, s);
}

hipError_t launch_nin_head(const FwdArgs& a, const HeadArgs& h, hipStream_t s) {
  if (a.K != 96 || h.oc < 1 || ((a.in_stride | a.in_off) & 3)) return hipErrorInvalidValue;
  const long tiles = (long)a.N * ((a.OH + 15) / 16) * ((a.OW + 15) / 16);
  const int mt = tiles < 1024 ? 1 : 2;
  const dim3 grid(((a.OW + 15) / 16) * ((a.OH + 4 * mt - 1) / (4 * mt)), a.N, 1);
  if (mt == 1) hipLaunchKernelGGL((k_nin_head<1>), grid, dim3(256), 0, s, a, h);
  else hipLaunchKernelGGL((k_nin_head<2>), grid, dim3(256), 0, s, a, h);
  return hipGetLastError();
}

hipError_t launch_head_bwd(const HeadBwdArgs& h, hipStream_t s) {
  if (h.oc < 1 || h.npx < 1) return hipErrorInvalidValue;
  const long nchunks = (h.npx + 511) / 512;
  const unsigned grid = (unsigned)(nchunks < 512 ? nchunks : 512);  // 2 per CU, weights loaded once
  hipLaunchKernelGGL((k_head_bwd<4, 8>), dim3(grid), dim3(512), 0, s, h);
  return hipGetLastError();
}

template <int GATHER, int NT, int MT>
static void geom(FwdGeom& g) {
  using C = FwdCfg<GATHER, NT, MT>;
  g.KC = C::KC; g.TAPS = C::TAPS; g.WNS = C::WNS; g.LW = C::LW;
}

bool fwd_supported(int gather, int nout) {
  const int nt = (nout + 15) / 16;
  if (gather == G_C3) return nt == 2 || nt == 3 || nt == 6 || nt == 9;
  if (gather == G_C1) return nt == 1 || nt == 2 || nt == 3 || nt == 6;
  if (gather == G_DN2 || gather == G_UP) return nt == 3 || nt == 6;
  return false;
}

bool fwd_geometry(int gather, int nout, FwdGeom& g) {
  const int nt = (nout + 15) / 16;
  if (gather == G_C3) {
    if (nt == 2) { geom<G_C3, 2, 4>(g); return true; }
    if (nt == 3) { geom<G_C3, 3, 4>(g); return true; }
    if (nt == 6) { geom<G_C3, 6, 4>(g); return true; }
    if (nt == 9) { geom<G_C3, 9, 2>(g); return true; }
  } else if (gather == G_C1) {
    if (nt == 1) { geom<G_C1, 1, 4>(g); return true; }
    if (nt == 2) { geom<G_C1, 2, 4>(g); return true; }
    if (nt == 3) { geom<G_C1, 3, 4>(g); return true; }
    if (nt == 6) { geom<G_C1, 6, 4>(g); return true; }
  } else if (gather == G_DN2) {
    if (nt == 3) { geom<G_DN2, 3, 4>(g); return true; }
    if (nt == 6) { geom<G_DN2, 6, 4>(g); return true; }
  } else if (gather == G_UP) {
    if (nt == 3) { geom<G_UP, 3, 4>(g); return true; }
    if (nt == 6) { geom<G_UP, 6, 4>(g); return true; }
  }
  return false;
}

long pack_floats(int gather, int nout, int K, int nz) {
  FwdGeom g;
  if (!fwd_geometry(gather, nout, g)) return -1;
  const long nch = (K + g.KC - 1) / g.KC;
  return nch * g.LW * nz;
}

bool pack_job(int gather, const WView& wv, int K, int nout, int nz, float* out, int zc, int ntot,
              PackJob& j) {
  FwdGeom g;
  const long lim = 1L << 31;
  if (!fwd_geometry(gather, nout, g) || wv.sK >= lim || wv.sN >= lim || wv.sT >= lim ||
      wv.sZ >= lim)
    return false;
  j = PackJob{};
  j.kind = PK_F32; j.w = wv.w + wv.off; j.out = out;
  j.sK = (int)wv.sK; j.sN = (int)wv.sN; j.sT = (int)wv.sT; j.sZ = (int)wv.sZ;
  j.taps = wv.taps; j.flip = wv.flip;
  j.K = K; j.NOUT = nout; j.nz = nz; j.zc = zc; j.ntot = ntot; j.nch = (K + g.KC - 1) / g.KC;
  j.g0 = g.KC; j.g1 = g.TAPS; j.g2 = g.WNS; j.g3 = g.LW;
  return true;
}

hipError_t launch_pack(int gather, const WView& wv, int K, int nout, int nz, float* out,
                       hipStream_t s, int zc, int ntot) {
  PackBatch b;
  if (!pack_job(gather, wv, K, nout, nz, out, zc, ntot, b.j[0])) return hipErrorInvalidValue;
  b.n = 1;
  return pack_flush(b, s);
}

// nin_a / nin_b as two single-chunk images [k][n] with row stride HEAD_WS
static PackJob head_job(const WView& w, float* out) {
  PackJob j{};
  j.kind = PK_F32; j.w = w.w + w.off; j.out = out;
  j.sK = (int)w.sK; j.sN = (int)w.sN; j.sT = (int)w.sT; j.sZ = (int)w.sZ;
  j.taps = w.taps; j.flip = w.flip;
  j.K = 96; j.NOUT = 96; j.nz = 1; j.nch = 1;
  j.g0 = 96; j.g1 = 1; j.g2 = HEAD_WS; j.g3 = HEAD_LW;
  return j;
}

hipError_t launch_pack_head(const WView& wa, const WView& wb, float* out, hipStream_t s,
                            PackBatch* pb) {
  PackBatch local;
  PackBatch& b = pb ? *pb : local;
  hipError_t e = pack_add(b, head_job(wa, out), s);
  if (e == hipSuccess) e = pack_add(b, head_job(wb, out + HEAD_LW), s);
  if (e != hipSuccess || pb) return e;
  return pack_flush(b, s);
}

// Tile height for a G_C3 launch: 16/8/4 rows (MT = 4/2/1) -- the fewest rounds of resident
// workgroups, each round weighed by its length (occupancy x tile height x per-tile efficiency
// of the shorter tiles).  E.g. a 1024-tile grid of the 96-channel kernel (3 resident per CU =
// 768 slots) runs 2 rounds of which the second is a third full at 16 rows, but 2048 tiles of
// 8 rows fill 2 rounds of 1024 slots.  Occupancy per
// variant: the compiler's waves/SIMD (one wave of each workgroup per SIMD).
static int c3_occupancy(int nt, int mt) {
  if (nt == 6) return mt == 4 ? 3 : 4;
  if (nt == 9) return 3;
  if (nt == 3) return mt == 1 ? 5 : 4;
  return mt == 1 ? 5 : 4;  // nt == 2
}

static int pick_mt(int nt, const FwdArgs& a, int nz, bool allow4) {
  const int mts[3] = {4, 2, 1};
  const double eff[3] = {1.0, 1.08, 1.25};
  int mt = 1;
  double best = 1e30;
  for (int i = allow4 ? 0 : 1; i < 3; ++i) {
    const long blocks = (long)a.N * ((a.OH + 4 * mts[i] - 1) / (4 * mts[i])) * ((a.OW + 15) / 16) * nz;
    // a round keeps occ workgroups per CU busy: it lasts ~occ * MT tile-rows of MFMA work
    const int occ = c3_occupancy(nt, mts[i]);
    const long slots = 256L * occ;
    const double cost = (double)((blocks + slots - 1) / slots) * occ * mts[i] * eff[i];
    if (cost < best - 1e-9) { best = cost; mt = mts[i]; }
  }
  return mt;
}

hipError_t launch_fwd(int gather, const FwdArgs& a, hipStream_t s) {
  const int nt = (a.NOUT + 15) / 16;
  // small images: 4-row tiles so that the grid still fills the chip
  const long big_tiles = (long)a.N * ((a.OH + 15) / 16) * ((a.OW + 15) / 16) *
                         (a.out_layout == OUT_UP2 ? 4 : 1);
  const bool small = big_tiles < 1024;
  if (gather == G_C3) {
    const int mt = pick_mt(nt, a, 1, nt != 9);
    if (nt == 3) return mt == 4 ? run_fwd<G_C3, 3, 4>(a, s) : mt == 2 ? run_fwd<G_C3, 3, 2>(a, s) : run_fwd<G_C3, 3, 1>(a, s);
    if (nt == 6) return mt == 4 ? run_fwd<G_C3, 6, 4>(a, s) : mt == 2 ? run_fwd<G_C3, 6, 2>(a, s) : run_fwd<G_C3, 6, 1>(a, s);
    if (nt == 9) return mt == 2 ? run_fwd<G_C3, 9, 2>(a, s) : run_fwd<G_C3, 9, 1>(a, s);
  } else if (gather == G_C1) {
    if (nt == 1) return run_fwd<G_C1, 1, 4>(a, s);
    if (nt == 3) return small ? run_fwd<G_C1, 3, 1>(a, s) : run_fwd<G_C1, 3, 4>(a, s);
    if (nt == 6) return small ? run_fwd<G_C1, 6, 1>(a, s) : run_fwd<G_C1, 6, 2>(a, s);
  } else if (gather == G_UP) {
    if (a.out_layout != OUT_UP2) return hipErrorInvalidValue;
    if (nt == 3) return run_fwd<G_UP, 3, 4>(a, s);
    if (nt == 6) return run_fwd<G_UP, 6, 4>(a, s);
  } else if (gather == G_DN2) {
    if (nt == 3) return small ? run_fwd<G_DN2, 3, 1>(a, s) : run_fwd<G_DN2, 3, 4>(a, s);
    if (nt == 6) return small ? run_fwd<G_DN2, 6, 1>(a, s) : run_fwd<G_DN2, 6, 4>(a, s);
  }
  return hipErrorInvalidValue;
}

// explicit tile width; a.zc must be 16*nt (or 0 for a single block of NOUT <= 16*nt)
hipError_t launch_fwd_nt(int gather, int nt, const FwdArgs& a, hipStream_t s) {
  const int nz = a.zc ? (a.NOUT + a.zc - 1) / a.zc : 1;
  const long big_tiles = (long)a.N * ((a.OH + 15) / 16) * ((a.OW + 15) / 16) * nz;
  const bool small = big_tiles < 1024;
  if (gather == G_C3) {
    const int mt = pick_mt(nt, a, nz, true);
    if (nt == 2) return mt == 4 ? run_fwd<G_C3, 2, 4>(a, s) : mt == 2 ? run_fwd<G_C3, 2, 2>(a, s) : run_fwd<G_C3, 2, 1>(a, s);
    if (nt == 3) return mt == 4 ? run_fwd<G_C3, 3, 4>(a, s) : mt == 2 ? run_fwd<G_C3, 3, 2>(a, s) : run_fwd<G_C3, 3, 1>(a, s);
    if (nt == 6) return mt == 4 ? run_fwd<G_C3, 6, 4>(a, s) : mt == 2 ? run_fwd<G_C3, 6, 2>(a, s) : run_fwd<G_C3, 6, 1>(a, s);
  } else if (gather == G_C1) {
    if (nt == 2) return small ? run_fwd<G_C1, 2, 1>(a, s) : run_fwd<G_C1, 2, 4>(a, s);
    if (nt == 3) return small ? run_fwd<G_C1, 3, 1>(a, s) : run_fwd<G_C1, 3, 4>(a, s);
    if (nt == 6) return small ? run_fwd<G_C1, 6, 1>(a, s) : run_fwd<G_C1, 6, 2>(a, s);
  }
  return hipErrorInvalidValue;
}

template <int MODE, int MF, int NW, int CIF>
static hipError_t run_wgrad(const WgradArgs& a, int splits, hipStream_t s) {
  using C = WgCfg<MODE, MF, NW, CIF>;
  const int nz = a.zc > 0 ? (a.cout_total + a.zc - 1) / a.zc : 1;
  dim3 grid(splits, (a.Cin + C::CIN_T - 1) / C::CIN_T, nz);
  hipLaunchKernelGGL((k_wgrad<MODE, MF, NW, CIF>), grid, dim3(C::NTHR), 0, s, a);
  return hipGetLastError();
}

template <int CO_FR, int WM, int WN>
static hipError_t run_wgrad3(const WgradArgs& a, int splits, hipStream_t s) {
  using C = Wg3Cfg<CO_FR, WM, WN>;
  const int nz = a.zc > 0 ? (a.cout_total + a.zc - 1) / a.zc : 1;
  dim3 grid(splits, (a.Cin + C::CIB - 1) / C::CIB, nz);
  // K stage width: 32-pixel row segments, or 16 / 8 / 4 pixels x 2 / 4 / 8 rows for narrow images
  prof_kernel("k_wgrad3");
  if (a.KW >= 32) hipLaunchKernelGGL((k_wgrad3<CO_FR, WM, WN, 5>), grid, dim3(C::NTHR), 0, s, a);
  else if (a.KW >= 16) hipLaunchKernelGGL((k_wgrad3<CO_FR, WM, WN, 4>), grid, dim3(C::NTHR), 0, s, a);
  else if (a.KW >= 8) hipLaunchKernelGGL((k_wgrad3<CO_FR, WM, WN, 3>), grid, dim3(C::NTHR), 0, s, a);
  else hipLaunchKernelGGL((k_wgrad3<CO_FR, WM, WN, 2>), grid, dim3(C::NTHR), 0, s, a);
  return hipGetLastError();
}

// the asynchronous 3x3 kernel needs 16-byte aligned pixels and channel quads that stay
// inside each pixel's row (reads past Cin land on padding or a neighbouring slice)
static bool wgrad3_ok(const WgradArgs& a) {
  if (a.Cout != 48 && a.Cout != 96) return false;
  if (a.Cin < 32) return false;  // a 32/48-channel block would be mostly padding
  if ((a.g_stride | a.g_off | a.x_stride | a.x_off) & 3) return false;
  if (a.x_off + ((a.Cin + 3) & ~3) > a.x_stride) return false;
  return a.zeros != nullptr;
}

// (CIN_T, PR, PC) of the template that launch_wgrad picks for (mode, cout)
static void wgrad_tile(int mode, int cout, int& cin_t, int& pr, int& pc) {
  const int cf = (cout + 15) / 16;
  pc = 32;
  if (mode == W_C3) { cin_t = cf >= 6 ? 32 : 48; pr = 1; }
  else if (mode == W_UP2) { cin_t = 16; pr = 1; pc = 16; }
  else { cin_t = cf == 1 ? 32 : 96; pr = cf >= 6 ? 1 : 2; }
}

bool wgrad_supported(int mode, int cout, int cin) {
  (void)cin;
  const int cf = (cout + 15) / 16;
  if (mode == W_C3 || mode == W_UP2) return cf == 3 || cf == 6;
  if (mode == W_C1) return cf == 1 || cf == 6;
  return false;
}

// Splits: splits x input-channel blocks fills ONE round of resident workgroups (3 per CU on
// 256 CUs) without a straggler round (floor, not ceil: 770 workgroups on 768 slots would
// double the time), at least two pixel chunks each, and a slab of at most 256 MB.
int wgrad_splits(int mode, int N, int KH, int KW, int Cin, int Cout) {
  int cin_t, pr, pc;
  wgrad_tile(mode, Cout, cin_t, pr, pc);
  const int taps = mode == W_C3 ? 9 : (mode == W_UP2 ? 4 : 1);
  long units = (long)N * ((KH + pr - 1) / pr) * ((KW + pc - 1) / pc);
  if (mode == W_C3 && KW < 32) {  // k_wgrad3 stages rows of narrow images together
    const int sw = KW >= 16 ? 16 : (KW >= 8 ? 8 : 4), sh = 32 / sw;
    units = (long)N * ((KH + sh - 1) / sh) * ((KW + sw - 1) / sw);
  }
  const long cib = (Cin + cin_t - 1) / cin_t;
  long want = 768 / cib;
  const long slab_cap = (64L << 20) / ((long)Cout * Cin * taps + Cout);  // <= 256 MB of slab
  if (want > slab_cap) want = slab_cap;
  // at least 2 pixel chunks per split: on the small levels the per-workgroup slab (up to 110 KB
  // written, then re-read by the reduction) outweighs the work of a 1-chunk split
  if (want > units / 2) want = units / 2;
  if (want < 1) want = 1;
  return (int)want;
}

hipError_t launch_wgrad(int mode, const WgradArgs& a, int splits, hipStream_t s, bool x6) {
  const int cf = (a.Cout + 15) / 16;
  if (x6 && mode == W_C3 && wgrad3_x6_ok(a)) return launch_wgrad3_x6(a, splits, s);
  if (mode == W_C3 && wgrad3_ok(a)) {
    if (cf == 6) return run_wgrad3<6, 2, 2>(a, splits, s);
    if (cf == 3) return run_wgrad3<3, 1, 3>(a, splits, s);
  }
  if (mode == W_C3) {
    if (cf == 3) return run_wgrad<W_C3, 1, 3, 1>(a, splits, s);
    if (cf == 6) return run_wgrad<W_C3, 2, 3, 1>(a, splits, s);
  } else if (mode == W_C1) {
    if (cf == 1) return run_wgrad<W_C1, 1, 1, 2>(a, splits, s);
    if (cf == 6) return run_wgrad<W_C1, 2, 3, 6>(a, splits, s);
  } else if (mode == W_UP2) {
    if (cf == 3) return run_wgrad<W_UP2, 1, 3, 1>(a, splits, s);
    if (cf == 6) return run_wgrad<W_UP2, 2, 3, 1>(a, splits, s);
  }
  return hipErrorInvalidValue;
}

// ---- general weight gradient (any Cout via output-channel blocks) ----------------------
// 3x3: k_wgrad3 in blocks of 96 / 48 / 32 output channels (Cin >= 16, float4-aligned views);
// 1x1: k_wgrad<W_C1> in blocks of 96 / 48.  Every block of one layer uses the same split count,
// so each slab row ends up holding the whole [W ; b] image and one reduction job finishes it.
static int gw_block(int mode, int cout) {
  if (mode == W_C3) return cout <= 32 ? 32 : (cout <= 48 ? 48 : 96);
  return cout <= 48 ? 48 : 96;
}

// input channels per workgroup of the 3x3 kernel: 32 for 96-wide output blocks; for 32-wide
// blocks (RDB growth convs, 24-channel layers) 32 / 48 / 64, whichever pads Cin least (ties:
// the wider block, fewer workgroups re-reading the gradient operand); else 48
static int gw_cin_t(int cb, int Cin) {
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

int gwgrad_splits(int mode, int N, int KH, int KW, int Cin, int Cout) {
  const int cb = gw_block(mode, Cout);
  const int nblk = (Cout + cb - 1) / cb;
  const int cin_t = mode == W_C3 ? gw_cin_t(cb, Cin) : 96;
  if (mode == W_C1) {  // k_wgrad1: one 32-pixel row segment per K stage
    const long units = (long)N * KH * ((KW + 31) / 32);
    long want = 768 / ((long)nblk * ((Cin + 95) / 96));
    const long slab_cap = (64L << 20) / ((long)Cout * Cin + Cout);
    if (want > slab_cap) want = slab_cap;
    if (want > units / 2) want = units / 2;
    return (int)(want < 1 ? 1 : want);
  }
  const long cib = (long)nblk * ((Cin + cin_t - 1) / cin_t);
  const int taps = mode == W_C3 ? 9 : 1;
  const int sw = KW >= 32 ? 32 : (KW >= 16 ? 16 : (KW >= 8 ? 8 : 4));  // k_wgrad3 segments
  const long units = mode == W_C3 ? (long)N * ((KH + 32 / sw - 1) / (32 / sw)) * ((KW + sw - 1) / sw)
                                  : (long)N * ((KH + (cb == 96 ? 0 : 1)) / (cb == 96 ? 1 : 2)) * ((KW + 31) / 32);
  long want = 768 / cib;
  const long slab_cap = (64L << 20) / ((long)Cout * Cin * taps + Cout);
  if (want > slab_cap) want = slab_cap;
  if (want > units / 2) want = units / 2;
  return (int)(want < 1 ? 1 : want);
}

// operands are read as channel quads: every quad that starts inside [0, C) must lie inside
// the view's row (padding channels of a wider buffer are fine, they meet masked rows/columns)
bool gwgrad_ok(int mode, int Cin, int Cout, const View& g, const View& x) {
  if (mode != W_C3 && mode != W_C1) return false;
  if ((g.stride | g.off | x.stride | x.off) & 3) return false;
  if (mode == W_C3 && Cin < 16) return false;
  if (x.off + ((Cin + 3) & ~3) > x.stride || g.off + ((Cout + 3) & ~3) > g.stride) return false;
  return Cout >= 1 && Cin >= 1;
}

hipError_t launch_gwgrad(int mode, const WgradArgs& a0, int splits, hipStream_t s) {
  const int cb = gw_block(mode, a0.Cout);
  WgradArgs a = a0;  // all output-channel blocks in ONE launch (blockIdx.z)
  a.zc = cb;
  a.cout_total = a0.Cout;
  a.co_base = 0;
  if (mode == W_C3) {
    if (cb == 96) return run_wgrad3<6, 2, 2>(a, splits, s);
    if (cb == 48) return run_wgrad3<3, 1, 3>(a, splits, s);
    const int ct = gw_cin_t(cb, a.Cin);
    if (ct == 64) return run_wgrad3<2, 1, 4>(a, splits, s);
    if (ct == 32) return run_wgrad3<2, 1, 2>(a, splits, s);
    return run_wgrad3<2, 1, 3>(a, splits, s);
  }
  // 1x1: the asynchronous k_wgrad1 tiled over (input-channel block of 96, output-channel block)
  const dim3 grid(splits, (a.Cin + 95) / 96, (a.Cout + cb - 1) / cb);
  if (cb == 96) hipLaunchKernelGGL((k_wgrad1<6, 6, 2, 2>), grid, dim3(256), 0, s, a, 0);
  else hipLaunchKernelGGL((k_wgrad1<3, 6, 1, 3>), grid, dim3(192), 0, s, a, 0);
  return hipGetLastError();
}

// ---- k_wgrad1 routing --------------------------------------------------------------
static bool wgrad1_shape(int mode, int cin, int cout) {
  return (mode == W_C1 || mode == W_UP2) && cin == cout && (cin == 96 || cin == 48);
}

bool wgrad1_ok(int mode, const WgradArgs& a) {
  if (!wgrad1_shape(mode, a.Cin, a.Cout) || !a.zeros) return false;
  if ((a.g_stride | a.g_off | a.x_stride | a.x_off) & 3) return false;
  return a.g_off + a.Cout <= a.g_stride && a.x_off + a.Cin <= a.x_stride;
}

// one round of resident workgroups (3 per CU) over splits x parities, >= 2 segments each
int wgrad1_splits(int mode, int N, int KH, int KW) {
  const int z = mode == W_UP2 ? 4 : 1;
  const long units = (long)N * KH * ((KW + 31) / 32);
  long sp = 768 / z;
  if (sp > units / 2) sp = units / 2;
  // UP2: whole groups of 8 (k_wgrad1p's XCD map of the four parity blocks; splits past the
  // pixel count write zero rows)
  if (z == 4) sp = sp < 8 ? 8 : sp / 8 * 8;
  return (int)(sp < 1 ? 1 : sp);
}

long wgrad_slab_floats(int mode, int N, int KH, int KW, int cin, int cout) {
  const int taps = mode == W_C3 ? 9 : (mode == W_UP2 ? 4 : 1);
  long f = (long)wgrad_splits(mode, N, KH, KW, cin, cout) * ((long)cout * cin * taps + cout);
  if (wgrad1_shape(mode, cin, cout)) {
    const long f1 = (long)(mode == W_UP2 ? 4 : 1) * wgrad1_splits(mode, N, KH, KW) *
                    ((long)cout * cin + cout);
    if (f1 > f) f = f1;
  }
  return f;
}

// k_wgrad1 + its reductions straight into dwb (PyTorch layout, bias after the weight); x6: the
// 96 x 96 1x1 on k_wgrad1p (bf16x6), the same splits and slab rows
hipError_t launch_wgrad1(int mode, const WgradArgs& a0, float* dwb, hipStream_t s,
                         RedBatch* rb, bool x6) {
  const bool up2 = mode == W_UP2;
  const int sp = wgrad1_splits(mode, a0.N, a0.KH, a0.KW), z = up2 ? 4 : 1;
  const long W = (long)a0.Cout * a0.Cin, row = W + a0.Cout;
  WgradArgs a = a0;
  a.slab_stride = row;
  a.wlayout = up2 ? 1 : 0;  // deconv weight (in, out, 2, 2): [ci][co] per parity
  const dim3 grid(sp, 1, z);
  hipError_t e;
  if (x6 && wgrad1p_ok(a)) {
    e = launch_wgrad1p(a, sp, s, up2);
  } else {
    if (a.Cout == 96)
      hipLaunchKernelGGL((k_wgrad1<6, 6, 2, 2>), grid, dim3(256), 0, s, a, (int)up2);
    else
      hipLaunchKernelGGL((k_wgrad1<3, 3, 1, 3>), grid, dim3(192), 0, s, a, (int)up2);
    e = hipGetLastError();
  }
  if (e != hipSuccess) return e;
  if (!up2 && a.hd_slab_c) {  // nin_c's weight gradient formed by the same launch (k_wgrad1p GNB)
    const long rc = (long)a.head_gnb * 96 + a.head_gnb;
    e = launch_reduce(a.hd_slab_c, rc, sp, rc, a.hd_dwc, s, rb);
    if (e != hipSuccess) return e;
  }
  if (!up2) return launch_reduce(a.slab, row, sp, row, dwb, s, rb);
  // W[ci][co][a][b] in output order: element e = 4 (ci*Cout + co) + ab lives in parity ab's
  // block of sp rows
  RedJob j = red_job(a.slab, row, sp, 4 * W, dwb);
  j.ig = 4; j.is1 = 1; j.is2 = (int)(sp * row);
  e = red_add(rb, j, s);
  if (e != hipSuccess) return e;
  return launch_reduce(a.slab + W, row, 4 * sp, a.Cout, dwb + 4 * W, s, rb);  // bias: all rows
}

RedJob red_job(const float* slab, long stride, int splits, long n, float* out) {
  RedJob j{};
  j.slab = slab; j.out = out;
  j.stride = (int)stride; j.splits = splits; j.n = (int)n;
  j.ig = (int)n; j.is1 = 0; j.is2 = 1;
  j.og = (int)n; j.os1 = 0; j.ooff = 0;
  return j;
}

hipError_t red_flush(RedBatch& b, hipStream_t s) {
  if (b.n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_reduce_batch, dim3((unsigned)b.blocks), dim3(256), 0, s, b);
  b.n = 0;
  b.blocks = 0;
  return hipGetLastError();
}

hipError_t red_add(RedBatch* b, const RedJob& j, hipStream_t s) {
  if (j.n <= 0) return hipSuccess;
  RedBatch local;
  RedBatch& r = b ? *b : local;
  if (r.n == kRedJobs) {
    hipError_t e = red_flush(r, s);
    if (e != hipSuccess) return e;
  }
  r.j[r.n] = j;
  r.j[r.n].b0 = r.blocks;
  // four elements per lane where they are contiguous and 16-B aligned in every slab row
  const int vec = j.is2 == 1 && j.ig % 4 == 0 && j.is1 % 4 == 0 && j.stride % 4 == 0 &&
                  j.n % 4 == 0 && (reinterpret_cast<uintptr_t>(j.slab) & 15) == 0;
  r.j[r.n].vec = vec;
  r.blocks += vec ? (j.n + 255) / 256 : (j.n + 63) / 64;
  ++r.n;
  return b ? hipSuccess : red_flush(r, s);
}

hipError_t launch_reduce(const float* slab, long slab_stride, int splits, long n, float* out,
                         hipStream_t s, RedBatch* rb) {
  return red_add(rb, red_job(slab, slab_stride, splits, n, out), s);
}

hipError_t launch_reduce_scatter(const float* slab, long slab_stride, int splits, long n,
                                 float* out, long grp, long ostride, long ooff, hipStream_t s,
                                 RedBatch* rb) {
  RedJob j = red_job(slab, slab_stride, splits, n, out);
  j.og = (int)grp; j.os1 = (int)ostride; j.ooff = (int)ooff;
  return red_add(rb, j, s);
}

}  // namespace dn
