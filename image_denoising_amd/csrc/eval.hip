// Evaluation path: full-image and tiled inference around dn_unet_forward,
// and the image metrics, all on the device.
//
//   k_u8_to_unit     x / 255 in fp32                             evaluation.py:69, evaluation_704.py:89
//   k_tile_extract   overlapping patch x patch tiles, numpy 'reflect' padding of short edge
//                    tiles, as one batch for the forward          evaluation_704.py:80-93
//   k_tile_blend     clamp(0,1) * weight mask, accumulated per pixel over the covering tiles
//                    in the reference's loop order (row-major tile order, fp32 mul then add,
//                    no contraction), / contribution (0 -> 1), then uint8 quantisation
//                                                                 evaluation_704.py:100-115
//   k_quantize_u8    clip(x*255 [+0.5], 0, 255) -> uint8 (trunc) evaluation.py:81-82
//   k_psnr_part      exact integer sum of squared uint8 differences utils_eval.py:49-53
//   k_ssim_part      11x11 Gaussian (sigma 1.5) window statistics in fp64 over the valid
//                    region [5, H-5) x [5, W-5), SSIM map summed per block utils_eval.py:19-33
//   k_l1_part        sum |a - b| in fp64                           evaluation.py:74 (nn.L1Loss)
//   k_eval_finalize  fixed-order sum of the block partials -> metric (deterministic)
#include <cstdint>

#include "dn_internal.h"

namespace dn {

constexpr int EVAL_BLOCKS = EVAL_PARTS;  // partial slots per metric (caller workspace)

__global__ __launch_bounds__(256) void k_u8_to_unit(const uint8_t* __restrict__ x, long n,
                                                    float* __restrict__ y) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    y[i] = (float)x[i] / 255.0f;
}

// numpy.pad(mode='reflect') index for an axis of length n (period 2(n-1))
__device__ __forceinline__ int reflect_idx(int i, int n) {
  if (n == 1) return 0;
  const int period = 2 * (n - 1);
  int j = i % period;
  return j < n ? j : period - j;
}

// img [C,H,W] uint8 -> tiles [P,C,ps,ps] fp32 (/255), tile p = (ti, tj) at (ti*stride, tj*stride)
__global__ __launch_bounds__(256) void k_tile_extract(const uint8_t* __restrict__ img, int C,
                                                      int H, int W, int ps, int stride, int nti,
                                                      int ntj, float* __restrict__ tiles) {
  const long per = (long)C * ps * ps, total = per * nti * ntj;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int p = (int)(e / per);
    const long r = e - (long)p * per;
    const int c = (int)(r / ((long)ps * ps)), q = (int)(r % ((long)ps * ps));
    const int i = q / ps, j = q - i * ps;
    const int r0 = (p / ntj) * stride, c0 = (p % ntj) * stride;
    const int ph = (r0 + ps < H ? r0 + ps : H) - r0, pw = (c0 + ps < W ? c0 + ps : W) - c0;
    const int si = reflect_idx(i, ph), sj = reflect_idx(j, pw);
    tiles[e] = (float)img[((long)c * H + r0 + si) * W + c0 + sj] / 255.0f;
  }
}

// out_unit [C,H,W] = blended prediction; out_u8 = clip(out*255, 0, 255) truncated
__global__ __launch_bounds__(256) void k_tile_blend(const float* __restrict__ pred, int C, int H,
                                                    int W, int ps, int stride, int nti, int ntj,
                                                    const float* __restrict__ wmask,
                                                    float* __restrict__ out_unit,
                                                    uint8_t* __restrict__ out_u8) {
#pragma clang fp contract(off)
  const long total = (long)C * H * W;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int c = (int)(e / ((long)H * W));
    const int q = (int)(e % ((long)H * W));
    const int y = q / W, x = q - y * W;
    float acc = 0.f, cm = 0.f;
    // tiles covering (y, x), in the reference's (r_start, c_start) loop order
    int ti_lo = y >= ps ? (y - ps) / stride + 1 : 0;
    int ti_hi = y / stride; if (ti_hi > nti - 1) ti_hi = nti - 1;
    int tj_lo = x >= ps ? (x - ps) / stride + 1 : 0;
    int tj_hi = x / stride; if (tj_hi > ntj - 1) tj_hi = ntj - 1;
    for (int ti = ti_lo; ti <= ti_hi; ++ti) {
      const int dy = y - ti * stride;
      for (int tj = tj_lo; tj <= tj_hi; ++tj) {
        const int dx = x - tj * stride;
        float v = pred[(((long)(ti * ntj + tj) * C + c) * ps + dy) * ps + dx];
        v = fminf(fmaxf(v, 0.f), 1.f);
        const float wm = wmask[dy * ps + dx];
        acc = acc + v * wm;
        cm = cm + wm;
      }
    }
    if (cm == 0.f) cm = 1.f;
    const float o = acc / cm;
    if (out_unit) out_unit[e] = o;
    if (out_u8) {
      float s = o * 255.0f;
      s = fminf(fmaxf(s, 0.f), 255.f);
      out_u8[e] = (uint8_t)s;
    }
  }
}

__global__ __launch_bounds__(256) void k_quantize_u8(const float* __restrict__ x, long n,
                                                     int plus_half, uint8_t* __restrict__ y) {
#pragma clang fp contract(off)
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float v = fminf(fmaxf(x[i], 0.f), 1.f);  // prediction.clamp(0, 1)
    float s = v * 255.0f;
    if (plus_half) s = s + 0.5f;
    s = fminf(fmaxf(s, 0.f), 255.f);
    y[i] = (uint8_t)s;
  }
}

// block-level sums (fixed shape: 256 threads, tree in LDS) -----------------------------
__device__ __forceinline__ double block_sum_d(double v, double* sh) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) sh[t] += sh[t + s];
    __syncthreads();
  }
  return sh[0];
}

__global__ __launch_bounds__(256) void k_psnr_part(const uint8_t* __restrict__ a,
                                                   const uint8_t* __restrict__ b, long n,
                                                   double* __restrict__ part) {
  __shared__ unsigned long long sh[256];
  unsigned long long s = 0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int d = (int)a[i] - (int)b[i];
    s += (unsigned long long)(d * d);
  }
  const int t = threadIdx.x;
  sh[t] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (t < k) sh[t] += sh[t + k];
    __syncthreads();
  }
  if (t == 0) part[blockIdx.x] = (double)sh[0];  // exact below 2^53
}

__global__ __launch_bounds__(256) void k_l1_part(const float* __restrict__ a,
                                                 const float* __restrict__ b, long n,
                                                 double* __restrict__ part) {
  __shared__ double sh[256];
  double s = 0.0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    s += fabs((double)a[i] - (double)b[i]);
  const double tot = block_sum_d(s, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// mean |a_p - b_p| of P items of n floats each (the per-tile criterion of evaluation_704.py:98),
// one workgroup per item: fp64 per-thread sums in a fixed order, fixed-tree block sum
__global__ __launch_bounds__(256) void k_l1_batched(const float* __restrict__ a,
                                                    const float* __restrict__ b, long n,
                                                    double* __restrict__ out) {
  __shared__ double sh[256];
  const float* pa = a + (long)blockIdx.x * n;
  const float* pb = b + (long)blockIdx.x * n;
  double s = 0.0;
  for (long i = threadIdx.x; i < n; i += 256) s += fabs((double)pa[i] - (double)pb[i]);
  const double tot = block_sum_d(s, sh);
  if (threadIdx.x == 0) out[blockIdx.x] = tot / (double)n;
}

// img [C,H,W] or [H,W,C] (hwc=1) uint8; one SSIM map per channel over the valid region
__global__ __launch_bounds__(256) void k_ssim_part(const uint8_t* __restrict__ a,
                                                   const uint8_t* __restrict__ b, int C, int H,
                                                   int W, int hwc, double* __restrict__ part) {
  __shared__ double g[11];
  __shared__ double sh[256];
  if (threadIdx.x == 0) {  // cv2.getGaussianKernel(11, 1.5): t_i = exp(-(i-5)^2 / (2 sigma^2))
    double sum = 0.0, t[11];
    const double scale2x = -0.5 / (1.5 * 1.5);
    for (int i = 0; i < 11; ++i) {
      const double x = i - 5.0;
      t[i] = exp(scale2x * x * x);
      sum += t[i];
    }
    const double inv = 1.0 / sum;
    for (int i = 0; i < 11; ++i) g[i] = t[i] * inv;
  }
  __syncthreads();
  const double C1 = (0.01 * 255) * (0.01 * 255), C2 = (0.03 * 255) * (0.03 * 255);
  const int vh = H - 10, vw = W - 10;
  const long per = (long)vh * vw, total = per * C;
  double s = 0.0;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int c = (int)(e / per);
    const long r = e - (long)c * per;
    const int y = (int)(r / vw) + 5, x = (int)(r % vw) + 5;
    double m1 = 0, m2 = 0, s11 = 0, s22 = 0, s12 = 0;
    for (int i = 0; i < 11; ++i) {
      const int yy = y + i - 5;
      for (int j = 0; j < 11; ++j) {
        const int xx = x + j - 5;
        const long idx = hwc ? ((long)yy * W + xx) * C + c : ((long)c * H + yy) * W + xx;
        const double w = g[i] * g[j];
        const double p = a[idx], q = b[idx];
        m1 += w * p;
        m2 += w * q;
        s11 += w * (p * p);
        s22 += w * (q * q);
        s12 += w * (p * q);
      }
    }
    const double mu1_sq = m1 * m1, mu2_sq = m2 * m2, mu12 = m1 * m2;
    const double sg1 = s11 - mu1_sq, sg2 = s22 - mu2_sq, sg12 = s12 - mu12;
    s += ((2 * mu12 + C1) * (2 * sg12 + C2)) / ((mu1_sq + mu2_sq + C1) * (sg1 + sg2 + C2));
  }
  const double tot = block_sum_d(s, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// kind 0: PSNR from the squared-error sum; 1: mean (SSIM, L1) of the partials over `count`
__global__ __launch_bounds__(256) void k_eval_finalize(const double* __restrict__ part, int nparts,
                                                       double count, int kind,
                                                       double* __restrict__ out) {
  __shared__ double sh[256];
  double v = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 256) v += part[i];  // fixed order per thread
  const double s = block_sum_d(v, sh);
  if (threadIdx.x != 0) return;
  const double mean = s / count;
  out[0] = kind == 0 ? 10.0 * log10(255.0 * 255.0 / mean) : mean;
}

static unsigned blocks_for(long n) {
  long b = (n + 255) / 256;
  if (b > EVAL_BLOCKS) b = EVAL_BLOCKS;
  return (unsigned)(b < 1 ? 1 : b);
}

hipError_t launch_u8_to_unit(const uint8_t* x, long n, float* y, hipStream_t s) {
  hipLaunchKernelGGL(k_u8_to_unit, dim3(blocks_for(n) * 4), dim3(256), 0, s, x, n, y);
  return hipGetLastError();
}

hipError_t launch_tile_extract(const uint8_t* img, int C, int H, int W, int ps, int stride,
                               int nti, int ntj, float* tiles, hipStream_t s) {
  const long total = (long)C * ps * ps * nti * ntj;
  hipLaunchKernelGGL(k_tile_extract, dim3(blocks_for(total) * 4), dim3(256), 0, s, img, C, H, W, ps,
                     stride, nti, ntj, tiles);
  return hipGetLastError();
}

hipError_t launch_tile_blend(const float* pred, int C, int H, int W, int ps, int stride, int nti,
                             int ntj, const float* wmask, float* out_unit, uint8_t* out_u8,
                             hipStream_t s) {
  const long total = (long)C * H * W;
  hipLaunchKernelGGL(k_tile_blend, dim3(blocks_for(total) * 4), dim3(256), 0, s, pred, C, H, W, ps,
                     stride, nti, ntj, wmask, out_unit, out_u8);
  return hipGetLastError();
}

hipError_t launch_quantize_u8(const float* x, long n, int plus_half, uint8_t* y, hipStream_t s) {
  hipLaunchKernelGGL(k_quantize_u8, dim3(blocks_for(n) * 4), dim3(256), 0, s, x, n, plus_half, y);
  return hipGetLastError();
}

hipError_t launch_psnr(const uint8_t* a, const uint8_t* b, long n, double* part, double* out,
                       hipStream_t s) {
  const unsigned nb = blocks_for(n);
  hipLaunchKernelGGL(k_psnr_part, dim3(nb), dim3(256), 0, s, a, b, n, part);
  hipLaunchKernelGGL(k_eval_finalize, dim3(1), dim3(256), 0, s, part, (int)nb, (double)n, 0, out);
  return hipGetLastError();
}

hipError_t launch_ssim(const uint8_t* a, const uint8_t* b, int C, int H, int W, int hwc,
                       double* part, double* out, hipStream_t s) {
  const long total = (long)C * (H - 10) * (W - 10);
  const unsigned nb = blocks_for(total);
  hipLaunchKernelGGL(k_ssim_part, dim3(nb), dim3(256), 0, s, a, b, C, H, W, hwc, part);
  hipLaunchKernelGGL(k_eval_finalize, dim3(1), dim3(256), 0, s, part, (int)nb, (double)total, 1,
                     out);
  return hipGetLastError();
}

hipError_t launch_l1_batched(const float* a, const float* b, long P, long n, double* out,
                             hipStream_t s) {
  hipLaunchKernelGGL(k_l1_batched, dim3((unsigned)P), dim3(256), 0, s, a, b, n, out);
  return hipGetLastError();
}

hipError_t launch_l1(const float* a, const float* b, long n, double* part, double* out,
                     hipStream_t s) {
  const unsigned nb = blocks_for(n);
  hipLaunchKernelGGL(k_l1_part, dim3(nb), dim3(256), 0, s, a, b, n, part);
  hipLaunchKernelGGL(k_eval_finalize, dim3(1), dim3(256), 0, s, part, (int)nb, (double)n, 1, out);
  return hipGetLastError();
}

}  // namespace dn
