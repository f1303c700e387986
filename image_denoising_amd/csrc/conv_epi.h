// Device helpers shared by the conv kernels (conv.hip, conv_x6.hip): the weight-gradient
// output-channel blocking and the output epilogue of the output-stationary kernels (k_fwd and
// the split-bf16 fp32 kernels).  Those keep a wave's tile as acc[m][q] in the 16x16 MFMA C/D map
// (col = lane&15 -> output channel q*16 + col, row = 4*(lane>>4) + reg -> pixel x of tile row m),
// so one LDS-staged epilogue serves every layout and fused op (FwdArgs::epi / out_layout).
#pragma once

#include "dn_internal.h"

namespace dn {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// XCD-aware tile order of the tiled conv kernels: the hardware deals workgroups round-robin
// over the 8 XCDs (linear block b -> XCD b % 8, MI355X_MICROARCH.md §Workgroup dispatch), so in
// launch order neighbouring tiles land on different XCDs and each re-fetches the halo rows the
// other already holds in its own L2.  Remapped, XCD x walks one contiguous run of
// (tile, image) indices -- vertical and horizontal neighbours are in flight on the same XCD --
// without changing which tiles are computed.  Over (blockIdx.x, blockIdx.y) of one z slab
// (the epilogue reads blockIdx.z itself); a bijection for any slab size (uneven runs when it
// is not a multiple of 8).  DN_XCD_REMAP=0 builds the launch order (A/B).
#ifndef DN_XCD_REMAP
#define DN_XCD_REMAP 1
#endif
__device__ __forceinline__ void xcd_tile(int& bx, int& by) {
  const unsigned gx = gridDim.x, tot = gx * gridDim.y;
  const unsigned l = blockIdx.x + gx * blockIdx.y;
  if (!DN_XCD_REMAP || tot < 16) {
    bx = (int)blockIdx.x; by = (int)blockIdx.y;
    return;
  }
  // global block l + z*tot sits on XCD (l + z0) % 8; XCD x holds the slab blocks
  // first(x), first(x) + 8, ... and gets the run [start(x), start(x) + count(x)) of the order
  const unsigned z0 = (blockIdx.z * tot) % 8, x = (l + z0) % 8;
  unsigned start = 0;
  for (unsigned xx = 0; xx < x; ++xx) {
    const unsigned f = (xx + 8 - z0) % 8;
    start += f < tot ? (tot - 1 - f) / 8 + 1 : 0u;
  }
  const unsigned lp = start + (l - (x + 8 - z0) % 8) / 8;
  bx = (int)(lp % gx); by = (int)(lp / gx);
}

// weight gradients: output-channel block of a wide layer (a.zc > 0): blockIdx.z selects
// channels [z*zc, z*zc+zc)
__device__ __forceinline__ WgradArgs wg_block(const WgradArgs& a0) {
  WgradArgs a = a0;
  if (a0.zc > 0) {
    a.co_base = (int)blockIdx.z * a0.zc;
    a.Cout = min(a0.zc, a0.cout_total - a.co_base);
    a.g_off = a0.g_off + a.co_base;
  }
  return a;
}

// Stage each 16-pixel row of the wave's tile through LDS, then write whole pixels: as float4
// (NOUT contiguous channels, 1 KiB contiguous per wave store) when the layout allows, else
// element by element (NCHW, PixelShuffle, unaligned views).  `lds` must hold waves*16*PS floats
// and be free (the caller's main loop ended on a barrier); each wave uses only its own 16*PS.
// UP: deconv forward, wave = parity (a,b) and every wave covers all MT rows; else wave w owns
// rows [w*MT, w*MT+MT) and blockIdx.z is the output-channel block (zc) or the scatter parity.
template <int NT, int MT, int PS, bool UP>
__device__ __forceinline__ void fwd_epilogue_generic(const FwdArgs& a, const f32x4 (&acc)[MT][NT],
                                                     float* lds, int ty0, int tx0, int n) {
  constexpr int NP = 16 * NT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const int ab = UP ? wave : (int)blockIdx.z;
  const int wrow = UP ? 0 : wave * MT;  // first tile row of this wave
  // output-channel block of a wide layer: channels [cz, cz + nout) of NOUT
  const int cz = a.zc ? (int)blockIdx.z * a.zc : 0;
  const int nout = a.zc ? min(NP, a.NOUT - cz) : a.NOUT;
  const bool aux = a.epi == EPI_MASK || a.epi == EPI_BIAS_ADD;
  const bool vec_out = (a.out_layout == OUT_NHWC || a.out_layout == OUT_UP2) &&
                       ((a.out_stride | a.out_off | a.NOUT) & 3) == 0 &&
                       (!aux || ((a.mask_stride | a.mask_off) & 3) == 0);
  float* st = lds + wave * 16 * PS;
  const bool bias_epi = (a.epi == EPI_BIAS || a.epi == EPI_BIAS_ACT || a.epi == EPI_BIAS_ADD) &&
                        a.bias != nullptr;
  // float4 path: every load of a row (staged tile, bias, mask / old output) is issued before its
  // stores -- a load after a store would wait for that store's completion (in-order vmcnt), which
  // serialised the epilogue on one L2 round trip per float4 (6 us per 16x16x96 tile)
  constexpr int NIT = (16 * NP / 4 + 63) / 64;  // float4 items per lane per row
  const int NQv = nout >> 2;
  float4 bvec[NIT];
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    const int e = lane + 64 * k;
    bvec[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (vec_out && bias_epi && e < 16 * NQv)
      bvec[k] = *reinterpret_cast<const float4*>(a.bias + cz + 4 * (e - (e / NQv) * NQv));
  }
#pragma unroll
  for (int m = 0; m < MT; ++m) {
#pragma unroll
    for (int q = 0; q < NT; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) st[(4 * lg + r) * PS + q * 16 + li] = acc[m][q][r];
    // st is this wave's own staging area and a wave's LDS accesses complete in order: no
    // barrier (a __syncthreads here would also drain the previous row's global stores)
    const int gy = ty0 + wrow + m;
    if (gy < a.OH && vec_out) {
      const int NQ = NQv;
      float4 vv[NIT], rr[NIT];
      long oiv[NIT];
      bool okv[NIT];
#pragma unroll
      for (int k = 0; k < NIT; ++k) {  // phase 1: loads
        const int e = lane + 64 * k;
        const int p = e / NQ, c = 4 * (e - p * NQ);
        const int gx = tx0 + p;
        okv[k] = e < 16 * NQ && gx < a.OW;
        vv[k] = rr[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        oiv[k] = 0;
        if (!okv[k]) continue;
        vv[k] = *reinterpret_cast<const float4*>(st + p * PS + c);
        const long pix = ((long)n * a.OH + gy) * a.OW + gx;
        if (a.out_layout == OUT_NHWC)
          oiv[k] = pix * a.out_stride + a.out_off + cz + c;
        else
          oiv[k] = (((long)n * 2 * a.OH + 2 * gy + (ab >> 1)) * 2 * a.OW + 2 * gx + (ab & 1)) *
                       a.out_stride + a.out_off + c;
        if (aux)
          rr[k] = *reinterpret_cast<const float4*>(a.mask + pix * a.mask_stride + a.mask_off + cz + c);
        else if (a.epi == EPI_ACCUM)
          rr[k] = *reinterpret_cast<const float4*>(a.out + oiv[k]);
      }
#pragma unroll
      for (int k = 0; k < NIT; ++k) {  // phase 2: arithmetic and stores
        if (!okv[k]) continue;
        float4 v = vv[k];
        if (bias_epi) {
          v.x += bvec[k].x; v.y += bvec[k].y; v.z += bvec[k].z; v.w += bvec[k].w;
        }
        const float4 r = rr[k];
        if (a.epi == EPI_BIAS_ACT) {
          v.x = v.x > 0.f ? v.x : v.x * 0.2f; v.y = v.y > 0.f ? v.y : v.y * 0.2f;
          v.z = v.z > 0.f ? v.z : v.z * 0.2f; v.w = v.w > 0.f ? v.w : v.w * 0.2f;
        } else if (a.epi == EPI_BIAS_ADD) {
          v.x = r.x + v.x; v.y = r.y + v.y; v.z = r.z + v.z; v.w = r.w + v.w;
        } else if (a.epi == EPI_MASK) {
          v.x = r.x > 0.f ? v.x : v.x * 0.2f; v.y = r.y > 0.f ? v.y : v.y * 0.2f;
          v.z = r.z > 0.f ? v.z : v.z * 0.2f; v.w = r.w > 0.f ? v.w : v.w * 0.2f;
        } else if (a.epi == EPI_ACCUM) {
          v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
        }
        *reinterpret_cast<float4*>(a.out + oiv[k]) = v;
      }
    } else if (gy < a.OH) {
      for (int e = lane; e < 16 * nout; e += 64) {
        const int p = e / nout, c = e - p * nout;
        const int gx = tx0 + p;
        if (gx >= a.OW) continue;
        const int cg = cz + c;  // channel of the layer
        float v = st[p * PS + c];
        const long pix = ((long)n * a.OH + gy) * a.OW + gx;
        if (bias_epi) v = v + a.bias[cg];
        if (a.epi == EPI_BIAS_ACT) {
          v = v > 0.f ? v : v * 0.2f;
        } else if (a.epi == EPI_BIAS_ADD) {
          v = a.mask[pix * a.mask_stride + a.mask_off + cg] + v;
        } else if (a.epi == EPI_MASK) {
          v = a.mask[pix * a.mask_stride + a.mask_off + cg] > 0.f ? v : v * 0.2f;
        }
        long oi;
        if (a.out_layout == OUT_NHWC) {
          oi = pix * a.out_stride + a.out_off + cg;
        } else if (a.out_layout == OUT_NCHW) {
          oi = (((long)n * a.NOUT + cg) * a.OH + gy) * a.OW + gx;
        } else if (a.out_layout == OUT_PS) {  // PixelShuffle(2): cg = 4*c' + 2*i + j
          oi = (((long)n * 2 * a.OH + 2 * gy + ((cg >> 1) & 1)) * 2 * a.OW + 2 * gx + (cg & 1)) *
                   a.out_stride + a.out_off + (cg >> 2);
        } else {
          oi = (((long)n * 2 * a.OH + 2 * gy + (ab >> 1)) * 2 * a.OW + 2 * gx + (ab & 1)) *
                   a.out_stride + a.out_off + c;
        }
        if (a.epi == EPI_ACCUM) v += a.out[oi];
        a.out[oi] = v;
      }
    }
  }
}


// NHWC float4 epilogue specialised on the epilogue kind EPI (compile time): every load of the
// wave's rows -- the staged tile read back from LDS, the mask / residual / old output -- is
// issued before the first global store.  The generic epilogue decides the kind at run time, so
// the compiler had to place a conservative s_waitcnt vmcnt(0) at the merge of each row's
// conditional loads -- behind the previous row's stores, i.e. one full store round trip per row
// (~15k cycles of a ~115k-cycle 16x16x96 tile with every CU storing at once, DN_X6_STAMPS).
// Requires vec_out (OUT_NHWC, float4-aligned strides / offsets); rows are staged one at a time
// through the wave's own LDS area (a wave's LDS accesses complete in order).
// (fwd_epilogue_vec_at: the wave's rows start at tile row wrow, its channels at cz (nout of
// them), its staging area is `st` (16 * PS floats) -- for kernels whose waves split the channels)
template <int NT, int MT, int PS, int EPI>
__device__ __forceinline__ void fwd_epilogue_vec_at(const FwdArgs& a, const f32x4 (&acc)[MT][NT],
                                                    float* st, int ty0, int tx0, int n, int wrow,
                                                    int cz, int nout) {
  constexpr int NP = 16 * NT;
  constexpr bool BIAS = EPI == EPI_BIAS || EPI == EPI_BIAS_ACT || EPI == EPI_BIAS_ADD;
  constexpr bool MASKL = EPI == EPI_MASK || EPI == EPI_BIAS_ADD;  // reads a.mask
  constexpr bool OLDL = EPI == EPI_ACCUM;                         // reads a.out
  constexpr int NIT = (16 * NP / 4 + 63) / 64;  // float4 items per lane per row
  const int lane = threadIdx.x & 63;
  const int li = lane & 15, lg = lane >> 4;
  const int NQ = nout >> 2;
  if constexpr (EPI == EPI_BIAS_ACT && MT % 2 == 0) {
    // fused 2x2 max-pool (FwdArgs::pool_out): rows m, m+1 of the wave and pixels 4lg + 2h, +1
    // of a lane are one window; each member activated exactly as below, then k_pool_fwd's
    // window order (TL, TR, BL, BR; a later member wins only if greater or NaN)
    if (a.pool_out) {
      const int OH2 = a.OH >> 1, OW2 = a.OW >> 1;
#pragma unroll
      for (int q = 0; q < NT; ++q) {
        const int c = 16 * q + li;
        const float b = (c < nout && a.bias) ? a.bias[cz + c] : 0.f;
#pragma unroll
        for (int m = 0; m < MT; m += 2)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            float v[4] = {acc[m][q][2 * h], acc[m][q][2 * h + 1], acc[m + 1][q][2 * h],
                          acc[m + 1][q][2 * h + 1]};
            float mx = 0.f;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              float x = v[t] + b;
              x = x > 0.f ? x : x * 0.2f;
              mx = (t == 0 || x > mx || __builtin_isnan(x)) ? x : mx;
            }
            const int gy2 = (ty0 + wrow + m) >> 1, gx2 = (tx0 >> 1) + 2 * lg + h;
            if (c < nout && gy2 < OH2 && gx2 < OW2)
              a.pool_out[((long)n * OH2 + gy2) * OW2 * a.pool_stride + (long)gx2 * a.pool_stride +
                         a.pool_off + cz + c] = mx;
          }
      }
      if (a.pool_only) return;  // nothing reads the full-resolution activation
    }
  }
  const bool has_bias = BIAS && a.bias != nullptr;
  float4 bvec[NIT];
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    const int e = lane + 64 * k;
    bvec[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (has_bias && e < 16 * NQ)
      bvec[k] = *reinterpret_cast<const float4*>(a.bias + cz + 4 * (e - (e / NQ) * NQ));
  }
  float4 vv[MT][NIT], rr[MT][NIT];
  long oi[MT][NIT];
  bool ok[MT][NIT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {  // phase 1: stage, read back, auxiliary loads
#pragma unroll
    for (int q = 0; q < NT; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) st[(4 * lg + r) * PS + q * 16 + li] = acc[m][q][r];
    const int gy = ty0 + wrow + m;
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int e = lane + 64 * k;
      const int p = e / NQ, c = 4 * (e - p * NQ);
      const int gx = tx0 + p;
      ok[m][k] = e < 16 * NQ && gx < a.OW && gy < a.OH;
      vv[m][k] = rr[m][k] = make_float4(0.f, 0.f, 0.f, 0.f);
      const long pix = ((long)n * a.OH + gy) * a.OW + gx;
      oi[m][k] = pix * a.out_stride + a.out_off + cz + c;
      if (e < 16 * NQ) vv[m][k] = *reinterpret_cast<const float4*>(st + p * PS + c);
      if (MASKL && ok[m][k])
        rr[m][k] = *reinterpret_cast<const float4*>(a.mask + pix * a.mask_stride + a.mask_off + cz + c);
      if (OLDL && ok[m][k]) rr[m][k] = *reinterpret_cast<const float4*>(a.out + oi[m][k]);
    }
  }
#pragma unroll
  for (int m = 0; m < MT; ++m)  // phase 2: arithmetic and stores
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      if (!ok[m][k]) continue;
      float4 v = vv[m][k];
      const float4 r = rr[m][k];
      if (BIAS) {
        v.x += bvec[k].x; v.y += bvec[k].y; v.z += bvec[k].z; v.w += bvec[k].w;
      }
      if (EPI == EPI_BIAS_ACT) {
        v.x = v.x > 0.f ? v.x : v.x * 0.2f; v.y = v.y > 0.f ? v.y : v.y * 0.2f;
        v.z = v.z > 0.f ? v.z : v.z * 0.2f; v.w = v.w > 0.f ? v.w : v.w * 0.2f;
      } else if (EPI == EPI_BIAS_ADD) {
        v.x = r.x + v.x; v.y = r.y + v.y; v.z = r.z + v.z; v.w = r.w + v.w;
      } else if (EPI == EPI_MASK) {
        v.x = r.x > 0.f ? v.x : v.x * 0.2f; v.y = r.y > 0.f ? v.y : v.y * 0.2f;
        v.z = r.z > 0.f ? v.z : v.z * 0.2f; v.w = r.w > 0.f ? v.w : v.w * 0.2f;
      } else if (EPI == EPI_ACCUM) {
        v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
      }
      if (a.out_bf16) {  // (uniform) bf16 activation storage: RNE, 8 bytes per 4 channels
        typedef __bf16 bf16x4e __attribute__((ext_vector_type(4)));
        const bf16x4e h = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
        *reinterpret_cast<bf16x4e*>(reinterpret_cast<__bf16*>(a.out) + oi[m][k]) = h;
      } else {
        *reinterpret_cast<float4*>(a.out + oi[m][k]) = v;
      }
    }
}

template <int NT, int MT, int PS, int EPI>
__device__ __forceinline__ void fwd_epilogue_vec(const FwdArgs& a, const f32x4 (&acc)[MT][NT],
                                                 float* lds, int ty0, int tx0, int n) {
  const int wave = threadIdx.x >> 6;
  const int cz = a.zc ? (int)blockIdx.z * a.zc : 0;
  const int nout = a.zc ? min(16 * NT, a.NOUT - cz) : a.NOUT;
  fwd_epilogue_vec_at<NT, MT, PS, EPI>(a, acc, lds + wave * 16 * PS, ty0, tx0, n, wave * MT, cz,
                                       nout);
}

// the float4 NHWC epilogue of a wave that owns rows [wrow, wrow + MT) and channels [cz, cz +
// nout) of the tile, the kind dispatched at run time (the caller checked vec_nhwc)
template <int NT, int MT, int PS>
__device__ __forceinline__ void fwd_epilogue_at(const FwdArgs& a, const f32x4 (&acc)[MT][NT],
                                                float* st, int ty0, int tx0, int n, int wrow,
                                                int cz, int nout) {
  switch (a.epi) {
    case EPI_BIAS: return fwd_epilogue_vec_at<NT, MT, PS, EPI_BIAS>(a, acc, st, ty0, tx0, n, wrow, cz, nout);
    case EPI_BIAS_ACT: return fwd_epilogue_vec_at<NT, MT, PS, EPI_BIAS_ACT>(a, acc, st, ty0, tx0, n, wrow, cz, nout);
    case EPI_PLAIN: return fwd_epilogue_vec_at<NT, MT, PS, EPI_PLAIN>(a, acc, st, ty0, tx0, n, wrow, cz, nout);
    case EPI_MASK: return fwd_epilogue_vec_at<NT, MT, PS, EPI_MASK>(a, acc, st, ty0, tx0, n, wrow, cz, nout);
    case EPI_ACCUM: return fwd_epilogue_vec_at<NT, MT, PS, EPI_ACCUM>(a, acc, st, ty0, tx0, n, wrow, cz, nout);
    case EPI_BIAS_ADD: return fwd_epilogue_vec_at<NT, MT, PS, EPI_BIAS_ADD>(a, acc, st, ty0, tx0, n, wrow, cz, nout);
    default: break;
  }
}

// the epilogue: the specialised float4 NHWC path where it applies, else the generic one
template <int NT, int MT, int PS, bool UP>
__device__ __forceinline__ void fwd_epilogue(const FwdArgs& a, const f32x4 (&acc)[MT][NT],
                                             float* lds, int ty0, int tx0, int n) {
  const bool aux = a.epi == EPI_MASK || a.epi == EPI_BIAS_ADD;
  const bool vec_nhwc = !UP && a.out_layout == OUT_NHWC &&
                        ((a.out_stride | a.out_off | a.NOUT) & 3) == 0 &&
                        (!aux || ((a.mask_stride | a.mask_off) & 3) == 0);
#ifndef DN_EPI_VEC
#define DN_EPI_VEC 1  // A/B switch: 0 = the generic run-time-kind epilogue everywhere
#endif
  if (DN_EPI_VEC && vec_nhwc) {
    switch (a.epi) {
      case EPI_BIAS: return fwd_epilogue_vec<NT, MT, PS, EPI_BIAS>(a, acc, lds, ty0, tx0, n);
      case EPI_BIAS_ACT: return fwd_epilogue_vec<NT, MT, PS, EPI_BIAS_ACT>(a, acc, lds, ty0, tx0, n);
      case EPI_PLAIN: return fwd_epilogue_vec<NT, MT, PS, EPI_PLAIN>(a, acc, lds, ty0, tx0, n);
      case EPI_MASK: return fwd_epilogue_vec<NT, MT, PS, EPI_MASK>(a, acc, lds, ty0, tx0, n);
      case EPI_ACCUM: return fwd_epilogue_vec<NT, MT, PS, EPI_ACCUM>(a, acc, lds, ty0, tx0, n);
      case EPI_BIAS_ADD: return fwd_epilogue_vec<NT, MT, PS, EPI_BIAS_ADD>(a, acc, lds, ty0, tx0, n);
      default: break;
    }
  }
  fwd_epilogue_generic<NT, MT, PS, UP>(a, acc, lds, ty0, tx0, n);
}

}  // namespace dn
