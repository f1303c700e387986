// HBM-bound building blocks of ImprovedUNet (arch_unet.py:421-531) for gfx950:
//
//   GroupNorm  (norm2d('gn'), arch_unet.py:7-15 / ResBlock :422-433)
//     k_chan_sums     per (image, channel) partial sums  S1 = sum a,  S2 = sum a*b  over a pixel
//                     range (fp64, fixed order); forward: a = b = z; backward: a = dy, b = z
//     k_gn_fwd_fin    per (image, group) mean / rstd, folded with gamma/beta into a per
//                     (image, channel) scale & shift   (y = z*scale + shift, as ATen's CPU kernel)
//     k_gn_bwd_fin    per (image, channel) coefficients of dz = A*dy + B*z + C and the
//                     gamma / beta gradients (fixed order over images)
//     k_affine        y = x*A[n,c] (+ B[n,c]*x2) + C[n,c]  [+ LeakyReLU] [+ residual]   (float4)
//   MaxPool2d(2) on strided views (fwd, bwd accumulating into the skip-gradient slice)
//   PixelShuffle(2) backward (gradient gather into the conv_ps output layout)
//   k_conv3_thin    3x3 conv with <= 4 output channels on the vector ALUs (noise estimator's
//                   second conv, the final conv; with a flipped view: the sigma-map data gradient)
//   small elementwise ops: view add, LeakyReLU' mask, sigmoid' of the output
#include <math.h>

#include "dn_internal.h"
#include "iunet_ops.h"

namespace dn {

static inline unsigned nblocks(long n, long cap = 8192) {
  long b = (n + 255) / 256;
  if (b > cap) b = cap;
  return (unsigned)(b < 1 ? 1 : b);
}

// ---- GroupNorm statistics ---------------------------------------------------------------
// grid (S, N): block (s, n) sums pixels [P*s/S, P*(s+1)/S) of image n for all C channels.
// Thread t: channel quad q = t % QC, pixel lane l = t / QC (PL = 256 / QC lanes).
__global__ __launch_bounds__(256) void k_chan_sums(const float* __restrict__ a, int as, int ao,
                                                   const float* __restrict__ b, int bs, int bo,
                                                   long P, int C, double* __restrict__ part) {
  __shared__ double red[256 * 8];
  const int QC = C >> 2, PL = 256 / QC;
  const int t = threadIdx.x, q = t % QC, l = t / QC;
  const int S = gridDim.x, s = blockIdx.x, n = blockIdx.y;
  const long p0 = P * s / S, p1 = P * (s + 1) / S;
  double v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (l < PL) {
    const float* an = a + (long)n * P * as + ao + 4 * q;
    const float* bn = b ? b + (long)n * P * bs + bo + 4 * q : nullptr;
    // four pixels' loads in flight per thread, summed in the same order as one at a time
    constexpr int UB = 4;
    for (long p = p0 + l; p < p1; p += UB * PL) {
      float4 x[UB], y[UB];
#pragma unroll
      for (int j = 0; j < UB; ++j) {
        const long pj = p + (long)j * PL;
        x[j] = pj < p1 ? *reinterpret_cast<const float4*>(an + pj * as) : make_float4(0.f, 0.f, 0.f, 0.f);
        y[j] = bn && pj < p1 ? *reinterpret_cast<const float4*>(bn + pj * bs) : x[j];
      }
#pragma unroll
      for (int j = 0; j < UB; ++j) {
        if (p + (long)j * PL >= p1) break;
        v[0] += x[j].x; v[1] += x[j].y; v[2] += x[j].z; v[3] += x[j].w;
        v[4] += (double)x[j].x * y[j].x; v[5] += (double)x[j].y * y[j].y;
        v[6] += (double)x[j].z * y[j].z; v[7] += (double)x[j].w * y[j].w;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[t * 8 + k] = v[k];
  __syncthreads();
  if (t < QC) {
    double r[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int ll = 0; ll < PL; ++ll)
#pragma unroll
      for (int k = 0; k < 8; ++k) r[k] += red[(ll * QC + t) * 8 + k];
    double* o = part + (((long)n * S + s) * C + 4 * t) * 2;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o[2 * k] = r[k];
      o[2 * k + 1] = r[4 + k];
    }
  }
}

// sums of channel c over the S splits of image n (fixed order)
__device__ __forceinline__ void split_sum(const double* part, int S, int C, int n, int c, double& s1,
                                          double& s2) {
  s1 = 0.0; s2 = 0.0;
  for (int s = 0; s < S; ++s) {
    const double* o = part + (((long)n * S + s) * C + c) * 2;
    s1 += o[0]; s2 += o[1];
  }
}

// one thread per (n, g): mean/rstd over M = cpg*P values; scale/shift per (n, c)
__global__ __launch_bounds__(256) void k_gn_fwd_fin(const double* __restrict__ part, int S, int N,
                                                    int C, int G, long P, float eps,
                                                    const float* __restrict__ gamma,
                                                    const float* __restrict__ beta,
                                                    float* __restrict__ stats,
                                                    float* __restrict__ scale,
                                                    float* __restrict__ shift) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N * G) return;
  const int n = i / G, g = i % G, cpg = C / G;
  double s1 = 0.0, s2 = 0.0;
  for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
    double a1, a2;
    split_sum(part, S, C, n, c, a1, a2);
    s1 += a1; s2 += a2;
  }
  const double M = (double)cpg * (double)P;
  const double mean = s1 / M;
  double var = s2 / M - mean * mean;
  if (var < 0.0) var = 0.0;
  const float meanf = (float)mean;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  stats[2 * i] = meanf;
  stats[2 * i + 1] = rstd;
  for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
    const float sc = rstd * gamma[c];
    scale[(long)n * C + c] = sc;
    shift[(long)n * C + c] = -sc * meanf + beta[c];
  }
}

// one thread per (n, g): dz = A*dy + B*z + C with (ATen GroupNormBackward)
//   ds = sum_c gamma_c * sum(dy*z),  db = sum_c gamma_c * sum(dy)
//   A = rstd*gamma_c,  B = (db*mean - ds) * rstd^3 / M,  C = -B*mean - db*rstd/M
__global__ __launch_bounds__(256) void k_gn_bwd_fin(const double* __restrict__ part, int S, int N,
                                                    int C, int G, long P,
                                                    const float* __restrict__ gamma,
                                                    const float* __restrict__ stats,
                                                    float* __restrict__ ca, float* __restrict__ cb,
                                                    float* __restrict__ cc) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N * G) return;
  const int n = i / G, g = i % G, cpg = C / G;
  double ds = 0.0, db = 0.0;
  for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
    double a1, a2;
    split_sum(part, S, C, n, c, a1, a2);
    db += (double)gamma[c] * a1;
    ds += (double)gamma[c] * a2;
  }
  const double mean = stats[2 * i], rstd = stats[2 * i + 1];
  const double M = (double)cpg * (double)P;
  const double B = (db * mean - ds) * rstd * rstd * rstd / M;
  const double Cc = -B * mean - db * rstd / M;
  for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
    ca[(long)n * C + c] = (float)(rstd * gamma[c]);
    cb[(long)n * C + c] = (float)B;
    cc[(long)n * C + c] = (float)Cc;
  }
}

// one 64-lane block per channel: dgamma[c] = sum_n (S2 - mean*S1)*rstd, dbeta[c] = sum_n S1;
// lane l takes images l, l+64, ... (splits in order), then a fixed xor-tree over the wave
__global__ __launch_bounds__(64) void k_gn_dparams(const double* __restrict__ part, int S, int N,
                                                   int C, int G, const float* __restrict__ stats,
                                                   float* __restrict__ dgamma,
                                                   float* __restrict__ dbeta) {
  const int c = blockIdx.x, l = threadIdx.x;
  const int g = c / (C / G);
  double dg = 0.0, dbt = 0.0;
  for (int n = l; n < N; n += 64) {
    double s1, s2;
    split_sum(part, S, C, n, c, s1, s2);
    const double mean = stats[2 * (n * G + g)], rstd = stats[2 * (n * G + g) + 1];
    dg += (s2 - mean * s1) * rstd;
    dbt += s1;
  }
  for (int o = 32; o > 0; o >>= 1) {
    dg += __shfl_xor(dg, o, 64);
    dbt += __shfl_xor(dbt, o, 64);
  }
  if (l == 0) {
    dgamma[c] = (float)dg;
    dbeta[c] = (float)dbt;
  }
}

// y = x*A + (x2 ? x2*B : 0) + Cc  (per (n, c) coefficients)  [+ LeakyReLU]  [+ res]
// (IDX = unsigned when every index fits 32 bits: 64-bit division per element cost more than the
// float4 it addresses)
template <typename IDX>
__global__ __launch_bounds__(256) void k_affine(const float* __restrict__ x, int xs, int xo,
                                                const float* __restrict__ x2, int x2s, int x2o,
                                                const float* __restrict__ A,
                                                const float* __restrict__ B,
                                                const float* __restrict__ Cc, int act,
                                                const float* __restrict__ res, int rs, int ro,
                                                float* __restrict__ y, int ys, int yo, long P,
                                                int C, long total4) {
  const IDX C4 = (IDX)(C >> 2), PP = (IDX)P;
  for (IDX e = (IDX)blockIdx.x * 256 + threadIdx.x; e < (IDX)total4; e += (IDX)gridDim.x * 256) {
    const int q = (int)(e % C4);
    const long pix = (long)(e / C4);  // n*P + p
    const long n = (long)((IDX)pix / PP);
    const long ci = n * C + 4 * q;
    const float4 v = *reinterpret_cast<const float4*>(x + pix * xs + xo + 4 * q);
    const float4 a = *reinterpret_cast<const float4*>(A + ci);
    const float4 c = *reinterpret_cast<const float4*>(Cc + ci);
    float4 o;
    if (x2) {
      const float4 v2 = *reinterpret_cast<const float4*>(x2 + pix * x2s + x2o + 4 * q);
      const float4 b = *reinterpret_cast<const float4*>(B + ci);
      o.x = v.x * a.x + v2.x * b.x + c.x; o.y = v.y * a.y + v2.y * b.y + c.y;
      o.z = v.z * a.z + v2.z * b.z + c.z; o.w = v.w * a.w + v2.w * b.w + c.w;
    } else {
      o.x = v.x * a.x + c.x; o.y = v.y * a.y + c.y; o.z = v.z * a.z + c.z; o.w = v.w * a.w + c.w;
    }
    if (act) {
      o.x = o.x > 0.f ? o.x : o.x * 0.2f; o.y = o.y > 0.f ? o.y : o.y * 0.2f;
      o.z = o.z > 0.f ? o.z : o.z * 0.2f; o.w = o.w > 0.f ? o.w : o.w * 0.2f;
    }
    if (res) {
      const float4 r = *reinterpret_cast<const float4*>(res + pix * rs + ro + 4 * q);
      o.x = r.x + o.x; o.y = r.y + o.y; o.z = r.z + o.z; o.w = r.w + o.w;
    }
    *reinterpret_cast<float4*>(y + pix * ys + yo + 4 * q) = o;
  }
}

// ---- MaxPool2d(2) on strided views (first max in row-major order wins, NaN propagates) ------
__device__ __forceinline__ bool take(float v, float m) { return v > m || isnan(v); }

__global__ __launch_bounds__(256) void k_vpool_fwd(const float* __restrict__ a, int as, int ao,
                                                   int N, int H, int W, int C,
                                                   float* __restrict__ y, int ys, int yo) {
  const int H2 = H >> 1, W2 = W >> 1, C4 = C >> 2;
  const long total = (long)N * H2 * W2 * C4;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int q = (int)(e % C4);
    const long pix = e / C4;
    const int x2 = (int)(pix % W2);
    const long t = pix / W2;
    const int y2 = (int)(t % H2);
    const long n = t / H2;
    const long p00 = (n * H + 2 * y2) * W + 2 * x2;
    const float* b = a + ao + 4 * q;
    float4 v[4];
    v[0] = *reinterpret_cast<const float4*>(b + p00 * as);
    v[1] = *reinterpret_cast<const float4*>(b + (p00 + 1) * as);
    v[2] = *reinterpret_cast<const float4*>(b + (p00 + W) * as);
    v[3] = *reinterpret_cast<const float4*>(b + (p00 + W + 1) * as);
    float4 m = v[0];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      m.x = take(v[k].x, m.x) ? v[k].x : m.x; m.y = take(v[k].y, m.y) ? v[k].y : m.y;
      m.z = take(v[k].z, m.z) ? v[k].z : m.z; m.w = take(v[k].w, m.w) ? v[k].w : m.w;
    }
    *reinterpret_cast<float4*>(y + pix * ys + yo + 4 * q) = m;
  }
}

__device__ __forceinline__ int argmax4(float a0, float a1, float a2, float a3) {
  int k = 0;
  float m = a0;
  if (take(a1, m)) { m = a1; k = 1; }
  if (take(a2, m)) { m = a2; k = 2; }
  if (take(a3, m)) { k = 3; }
  return k;
}

// dx (view, same layout as the pool input a) += route(dy)
__global__ __launch_bounds__(256) void k_vpool_bwd(const float* __restrict__ a, int as, int ao,
                                                   int N, int H, int W, int C,
                                                   const float* __restrict__ dy, int ds, int dof,
                                                   float* __restrict__ dx, int xs, int xo) {
  const int H2 = H >> 1, W2 = W >> 1;
  const long total = (long)N * H2 * W2 * C;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int c = (int)(e % C);
    const long pix = e / C;
    const int x2 = (int)(pix % W2);
    const long t = pix / W2;
    const int y2 = (int)(t % H2);
    const long n = t / H2;
    const long p[4] = {(n * H + 2 * y2) * W + 2 * x2, (n * H + 2 * y2) * W + 2 * x2 + 1,
                       (n * H + 2 * y2 + 1) * W + 2 * x2, (n * H + 2 * y2 + 1) * W + 2 * x2 + 1};
    const int k = argmax4(a[p[0] * as + ao + c], a[p[1] * as + ao + c], a[p[2] * as + ao + c],
                          a[p[3] * as + ao + c]);
    const float d = dy[pix * ds + dof + c];
    float* o = dx + p[k] * xs + xo + c;
    *o = *o + d;
  }
}

// ---- PixelShuffle(2) backward: g[(n,y,x), 4c+2i+j] = du[(n,2y+i,2x+j), c] --------------------
__global__ __launch_bounds__(256) void k_unshuffle(const float* __restrict__ du, int ds, int dof,
                                                   int N, int h, int w, int C,
                                                   float* __restrict__ g) {
  const long total = (long)N * h * w * C;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int c = (int)(e % C);
    const long pix = e / C;
    const int x = (int)(pix % w);
    const long t = pix / w;
    const int y = (int)(t % h);
    const long n = t / h;
    const long q0 = (n * 2 * h + 2 * y) * 2 * w + 2 * x;
    float4 v;
    v.x = du[q0 * ds + dof + c];
    v.y = du[(q0 + 1) * ds + dof + c];
    v.z = du[(q0 + 2 * w) * ds + dof + c];
    v.w = du[(q0 + 2 * w + 1) * ds + dof + c];
    *reinterpret_cast<float4*>(g + pix * 4 * C + 4 * c) = v;
  }
}

// ---- elementwise on views ----------------------------------------------------------------
// dst += src
__global__ __launch_bounds__(256) void k_vadd(float* __restrict__ d, int dsr, int dof,
                                              const float* __restrict__ s, int ss, int so, int C,
                                              long total4) {
  const int C4 = C >> 2;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total4; e += (long)gridDim.x * 256) {
    const int q = (int)(e % C4);
    const long pix = e / C4;
    float4* o = reinterpret_cast<float4*>(d + pix * dsr + dof + 4 * q);
    const float4 v = *reinterpret_cast<const float4*>(s + pix * ss + so + 4 * q);
    float4 r = *o;
    r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
    *o = r;
  }
}

// dst = src * leaky'(act)   (LeakyReLU(0.2) backward through the saved output)
__global__ __launch_bounds__(256) void k_vmask(float* __restrict__ d, int dsr, int dof,
                                               const float* __restrict__ s, int ss, int so,
                                               const float* __restrict__ m, int ms, int mo, int C,
                                               long total4) {
  const int C4 = C >> 2;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total4; e += (long)gridDim.x * 256) {
    const int q = (int)(e % C4);
    const long pix = e / C4;
    const float4 v = *reinterpret_cast<const float4*>(s + pix * ss + so + 4 * q);
    const float4 k = *reinterpret_cast<const float4*>(m + pix * ms + mo + 4 * q);
    float4 r;
    r.x = k.x > 0.f ? v.x : v.x * 0.2f; r.y = k.y > 0.f ? v.y : v.y * 0.2f;
    r.z = k.z > 0.f ? v.z : v.z * 0.2f; r.w = k.w > 0.f ? v.w : v.w * 0.2f;
    *reinterpret_cast<float4*>(d + pix * dsr + dof + 4 * q) = r;
  }
}

// sigmoid output y (NCHW [N,C,H,W]) and dy (NCHW): dz (NHWC stride ds, channels [0,C)) =
// dy * y * (1 - y); channels [C, ds) zeroed
__global__ __launch_bounds__(256) void k_dsigmoid_nchw(const float* __restrict__ y,
                                                       const float* __restrict__ dy, int N, int C,
                                                       long HW, float* __restrict__ dz, int ds) {
  const long total = (long)N * HW;
  for (long p = (long)blockIdx.x * 256 + threadIdx.x; p < total; p += (long)gridDim.x * 256) {
    const long n = p / HW, r = p - n * HW;
    for (int c = 0; c < ds; ++c) {
      float v = 0.f;
      if (c < C) {
        const float s = y[(n * C + c) * HW + r];
        v = dy[(n * C + c) * HW + r] * (s * (1.f - s));
      }
      dz[p * ds + c] = v;
    }
  }
}

// ---- thin-output 3x3 conv (VALU) ------------------------------------------------------------
// out[p][o] = sum_{k<K} sum_t W(o, k, t) * in[p + off(t)][k]  for o < CO (<= 4), 16x16 tile per
// block, input staged through LDS 16 channels at a time, weights read through a strided view:
// W(o, k, t) = w[woff + o*wso + k*wsk + tap(t)*wst], tap(t) = flip ? 8 - t : t.
// Epilogue: TE_BIAS: acc + b[o];  TE_SIGMOID: sigmoid(acc + b[o]);  TE_DSIG: acc * s(1-s) with s
// read from aux (NHWC view).  Output: NHWC view (o at yo + o) or NCHW [N, CO, H, W].
constexpr int TKC = 16;
template <int CO>
__global__ __launch_bounds__(256) void k_conv3_thin(const float* __restrict__ in, int is, int io,
                                                    int N, int H, int W, int K,
                                                    const float* __restrict__ w, long woff,
                                                    long wso, long wsk, long wst, int flip,
                                                    const float* __restrict__ bias, int epi,
                                                    const float* __restrict__ aux, int auxs,
                                                    int auxo, float* __restrict__ out, int os,
                                                    int oo, int nchw, int nout) {
  __shared__ float sx[TKC * 18 * 18];
  __shared__ float sw[CO * TKC * 9];
  const int tiles_x = (W + 15) / 16;
  const int ty0 = (blockIdx.x / tiles_x) * 16, tx0 = (blockIdx.x % tiles_x) * 16;
  const int n = blockIdx.y, t = threadIdx.x;
  const int py = t / 16, px = t % 16;
  float acc[CO];
#pragma unroll
  for (int o = 0; o < CO; ++o) acc[o] = 0.f;
  const float* inb = in + (long)n * H * W * is + io;
  // quads must not straddle K: whole quads of real channels, or padding inside the row
  const bool vec = ((is | io) & 3) == 0 && (K % 4 == 0 || io + ((K + 3) & ~3) <= is);
  for (int k0 = 0; k0 < K; k0 += TKC) {
    const int kc = K - k0 < TKC ? K - k0 : TKC;
    if (vec) {  // float4 along channels: consecutive lanes read consecutive quads of a pixel
      for (int e = t; e < 324 * (TKC / 4); e += 256) {
        const int r = e / (TKC / 4), q = e % (TKC / 4);
        const int gy = ty0 - 1 + r / 18, gx = tx0 - 1 + r % 18;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (4 * q < kc && gy >= 0 && gy < H && gx >= 0 && gx < W)
          v = *reinterpret_cast<const float4*>(inb + ((long)gy * W + gx) * is + k0 + 4 * q);
        sx[(4 * q) * 324 + r] = v.x;
        sx[(4 * q + 1) * 324 + r] = v.y;
        sx[(4 * q + 2) * 324 + r] = v.z;
        sx[(4 * q + 3) * 324 + r] = v.w;
      }
    } else {
      for (int e = t; e < TKC * 324; e += 256) {
        const int k = e / 324, r = e % 324;
        const int gy = ty0 - 1 + r / 18, gx = tx0 - 1 + r % 18;
        float v = 0.f;
        if (k < kc && gy >= 0 && gy < H && gx >= 0 && gx < W) v = inb[((long)gy * W + gx) * is + k0 + k];
        sx[e] = v;
      }
    }
    for (int e = t; e < CO * TKC * 9; e += 256) {
      const int o = e / (TKC * 9), k = (e / 9) % TKC, tp = e % 9;
      float v = 0.f;
      if (o < nout && k < kc) v = w[woff + o * wso + (long)(k0 + k) * wsk + (flip ? 8 - tp : tp) * wst];
      sw[e] = v;
    }
    __syncthreads();
    for (int k = 0; k < kc; ++k) {
      float xv[9];
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) xv[tp] = sx[k * 324 + (py + tp / 3) * 18 + px + tp % 3];
#pragma unroll
      for (int o = 0; o < CO; ++o)
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) acc[o] = fmaf(sw[(o * TKC + k) * 9 + tp], xv[tp], acc[o]);
    }
    __syncthreads();
  }
  const int gy = ty0 + py, gx = tx0 + px;
  if (gy >= H || gx >= W) return;
  const long pix = ((long)n * H + gy) * W + gx;
#pragma unroll
  for (int o = 0; o < CO; ++o) {
    if (o >= nout) break;
    float v = acc[o];
    if (epi == TE_BIAS) {
      v += bias[o];
    } else if (epi == TE_SIGMOID) {
      v = 1.f / (1.f + expf(-(v + bias[o])));
    } else if (epi == TE_DSIG) {
      const float s = aux[pix * auxs + auxo + o];
      v = v * (s * (1.f - s));
    }
    if (nchw) out[(((long)n * nout + o) * H + gy) * W + gx] = v;
    else out[pix * os + oo + o] = v;
  }
}

// ---- launchers ------------------------------------------------------------------------------
int chan_sums_splits(int N, long P) {
  long s = 2048 / (N > 0 ? N : 1);
  const long cap = P / 256;
  if (s > cap) s = cap;
  return (int)(s < 1 ? 1 : s);
}

hipError_t launch_chan_sums(const View& a, const View* b, int N, long P, int C, int S,
                            double* part, hipStream_t s) {
  if ((C & 3) || C / 4 > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_chan_sums, dim3(S, N), dim3(256), 0, s, a.p, a.stride, a.off,
                     b ? b->p : nullptr, b ? b->stride : 0, b ? b->off : 0, P, C, part);
  return hipGetLastError();
}

hipError_t launch_gn_fwd_fin(const double* part, int S, int N, int C, int G, long P, float eps,
                             const float* gamma, const float* beta, float* stats, float* scale,
                             float* shift, hipStream_t s) {
  hipLaunchKernelGGL(k_gn_fwd_fin, dim3((N * G + 255) / 256), dim3(256), 0, s, part, S, N, C, G, P,
                     eps, gamma, beta, stats, scale, shift);
  return hipGetLastError();
}

hipError_t launch_gn_bwd_fin(const double* part, int S, int N, int C, int G, long P,
                             const float* gamma, const float* stats, float* ca, float* cb,
                             float* cc, float* dgamma, float* dbeta, hipStream_t s) {
  hipLaunchKernelGGL(k_gn_bwd_fin, dim3((N * G + 255) / 256), dim3(256), 0, s, part, S, N, C, G, P,
                     gamma, stats, ca, cb, cc);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_gn_dparams, dim3(C), dim3(64), 0, s, part, S, N, C, G, stats, dgamma, dbeta);
  return hipGetLastError();
}

hipError_t launch_affine(const View& x, const View* x2, const float* A, const float* B,
                         const float* Cc, int act, const View* res, const View& y, int N, long P,
                         int C, hipStream_t s) {
  const long total4 = (long)N * P * (C / 4);
  // (32-bit indices: total4 plus one grid stride below 2^32)
  if (total4 + (long)nblocks(total4) * 256 < (1L << 32))
    hipLaunchKernelGGL(k_affine<unsigned>, dim3(nblocks(total4)), dim3(256), 0, s, x.p, x.stride, x.off,
                       x2 ? x2->p : nullptr, x2 ? x2->stride : 0, x2 ? x2->off : 0, A, B, Cc, act,
                       res ? res->p : nullptr, res ? res->stride : 0, res ? res->off : 0, y.p,
                       y.stride, y.off, P, C, total4);
  else
    hipLaunchKernelGGL(k_affine<unsigned long>, dim3(nblocks(total4)), dim3(256), 0, s, x.p, x.stride,
                       x.off, x2 ? x2->p : nullptr, x2 ? x2->stride : 0, x2 ? x2->off : 0, A, B, Cc,
                       act, res ? res->p : nullptr, res ? res->stride : 0, res ? res->off : 0, y.p,
                       y.stride, y.off, P, C, total4);
  return hipGetLastError();
}

hipError_t launch_vpool_fwd(const View& a, int N, int H, int W, int C, const View& y, hipStream_t s) {
  const long total = (long)N * (H / 2) * (W / 2) * (C / 4);
  hipLaunchKernelGGL(k_vpool_fwd, dim3(nblocks(total)), dim3(256), 0, s, a.p, a.stride, a.off, N, H,
                     W, C, y.p, y.stride, y.off);
  return hipGetLastError();
}

hipError_t launch_vpool_bwd_acc(const View& a, int N, int H, int W, int C, const View& dy,
                                const View& dx, hipStream_t s) {
  const long total = (long)N * (H / 2) * (W / 2) * C;
  hipLaunchKernelGGL(k_vpool_bwd, dim3(nblocks(total)), dim3(256), 0, s, a.p, a.stride, a.off, N, H,
                     W, C, dy.p, dy.stride, dy.off, dx.p, dx.stride, dx.off);
  return hipGetLastError();
}

hipError_t launch_unshuffle(const View& du, int N, int h, int w, int C, float* g, hipStream_t s) {
  const long total = (long)N * h * w * C;
  hipLaunchKernelGGL(k_unshuffle, dim3(nblocks(total)), dim3(256), 0, s, du.p, du.stride, du.off, N,
                     h, w, C, g);
  return hipGetLastError();
}

hipError_t launch_vadd(const View& d, const View& src, long npx, int C, hipStream_t s) {
  const long total4 = npx * (C / 4);
  hipLaunchKernelGGL(k_vadd, dim3(nblocks(total4)), dim3(256), 0, s, d.p, d.stride, d.off, src.p,
                     src.stride, src.off, C, total4);
  return hipGetLastError();
}

hipError_t launch_vmask(const View& d, const View& src, const View& act, long npx, int C,
                        hipStream_t s) {
  const long total4 = npx * (C / 4);
  hipLaunchKernelGGL(k_vmask, dim3(nblocks(total4)), dim3(256), 0, s, d.p, d.stride, d.off, src.p,
                     src.stride, src.off, act.p, act.stride, act.off, C, total4);
  return hipGetLastError();
}

hipError_t launch_dsigmoid_nchw(const float* y, const float* dy, int N, int C, long HW, float* dz,
                                int ds, hipStream_t s) {
  hipLaunchKernelGGL(k_dsigmoid_nchw, dim3(nblocks((long)N * HW)), dim3(256), 0, s, y, dy, N, C, HW,
                     dz, ds);
  return hipGetLastError();
}

hipError_t launch_conv3_thin(const View& in, int N, int H, int W, int K, const WView& wv,
                             const float* bias, int epi, const View& aux, const View& out, int nchw,
                             int nout, hipStream_t s) {
  const dim3 grid(((W + 15) / 16) * ((H + 15) / 16), N);
#define DN_CT(CO)                                                                               \
  hipLaunchKernelGGL(k_conv3_thin<CO>, grid, dim3(256), 0, s, in.p, in.stride, in.off, N, H, W, K, \
                     wv.w, wv.off, wv.sN, wv.sK, wv.sT, wv.flip, bias, epi, aux.p, aux.stride,     \
                     aux.off, out.p, out.stride, out.off, nchw, nout)
  if (nout == 1) DN_CT(1);
  else if (nout <= 4) DN_CT(4);
  else return hipErrorInvalidValue;
#undef DN_CT
  return hipGetLastError();
}

}  // namespace dn
