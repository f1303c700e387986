// HBM-bound kernels of the N2N training step for gfx950: 2x2 max-pool fwd/bwd, the
// neighbour sub-sampler, Gaussian noise synthesis, the loss reductions and Adam.
#include <math.h>
#include <cstdint>

#include "dn_internal.h"
#include "philox.h"

namespace dn {

static inline unsigned grid_for(long n, int per_block = 256, long cap = 1L << 30) {
  long b = (n + per_block - 1) / per_block;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (unsigned)b;
}

// ------------------------------------------------------------------------------------
// MaxPool2d(2): arch_unet.py:120-135.  NaN propagates and the first maximum in row-major
// window order (TL, TR, BL, BR) wins, as ATen's max_pool2d_with_indices does.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ bool pool_take(float v, float m) { return v > m || isnan(v); }

__global__ __launch_bounds__(256) void k_pool_fwd(const float* __restrict__ a, int N, int H, int W,
                                                  int C, float* __restrict__ out, int os, int oo) {
  const int H2 = H >> 1, W2 = W >> 1, C4 = C >> 2;
  const long total = (long)N * H2 * W2 * C4;
  for (long idx = (long)blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (long)gridDim.x * 256) {
    const int c4 = (int)(idx % C4);
    const long pix = idx / C4;
    const int x2 = (int)(pix % W2);
    const long t = pix / W2;
    const int y2 = (int)(t % H2);
    const int n = (int)(t / H2);
    const long base = (((long)n * H + 2 * y2) * W + 2 * x2) * C + 4 * c4;
    const float4 v0 = *reinterpret_cast<const float4*>(a + base);
    const float4 v1 = *reinterpret_cast<const float4*>(a + base + C);
    const float4 v2 = *reinterpret_cast<const float4*>(a + base + (long)W * C);
    const float4 v3 = *reinterpret_cast<const float4*>(a + base + (long)W * C + C);
    float4 m = v0;
    m.x = pool_take(v1.x, m.x) ? v1.x : m.x; m.y = pool_take(v1.y, m.y) ? v1.y : m.y;
    m.z = pool_take(v1.z, m.z) ? v1.z : m.z; m.w = pool_take(v1.w, m.w) ? v1.w : m.w;
    m.x = pool_take(v2.x, m.x) ? v2.x : m.x; m.y = pool_take(v2.y, m.y) ? v2.y : m.y;
    m.z = pool_take(v2.z, m.z) ? v2.z : m.z; m.w = pool_take(v2.w, m.w) ? v2.w : m.w;
    m.x = pool_take(v3.x, m.x) ? v3.x : m.x; m.y = pool_take(v3.y, m.y) ? v3.y : m.y;
    m.z = pool_take(v3.z, m.z) ? v3.z : m.z; m.w = pool_take(v3.w, m.w) ? v3.w : m.w;
    *reinterpret_cast<float4*>(out + pix * os + oo + 4 * c4) = m;
  }
}

__device__ __forceinline__ void pool_bwd1(float a0, float a1, float a2, float a3, float d, int act,
                                          float& o0, float& o1, float& o2, float& o3) {
  int k = 0;
  float m = a0;
  if (pool_take(a1, m)) { m = a1; k = 1; }
  if (pool_take(a2, m)) { m = a2; k = 2; }
  if (pool_take(a3, m)) { m = a3; k = 3; }
  o0 = k == 0 ? d : 0.f; o1 = k == 1 ? d : 0.f; o2 = k == 2 ? d : 0.f; o3 = k == 3 ? d : 0.f;
  if (act) {  // LeakyReLU(0.2) backward through the saved (post-activation) value
    o0 = a0 > 0.f ? o0 : o0 * 0.2f; o1 = a1 > 0.f ? o1 : o1 * 0.2f;
    o2 = a2 > 0.f ? o2 : o2 * 0.2f; o3 = a3 > 0.f ? o3 : o3 * 0.2f;
  }
}

__global__ __launch_bounds__(256) void k_pool_bwd(const float* __restrict__ a, int N, int H, int W,
                                                  int C, const float* __restrict__ dp, int ds,
                                                  int doff, int act, float* __restrict__ da) {
  const int H2 = H >> 1, W2 = W >> 1, C4 = C >> 2;
  const long total = (long)N * H2 * W2 * C4;
  for (long idx = (long)blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (long)gridDim.x * 256) {
    const int c4 = (int)(idx % C4);
    const long pix = idx / C4;
    const int x2 = (int)(pix % W2);
    const long t = pix / W2;
    const int y2 = (int)(t % H2);
    const int n = (int)(t / H2);
    const long b0 = (((long)n * H + 2 * y2) * W + 2 * x2) * C + 4 * c4;
    const long b1 = b0 + C, b2 = b0 + (long)W * C, b3 = b2 + C;
    const float4 v0 = *reinterpret_cast<const float4*>(a + b0);
    const float4 v1 = *reinterpret_cast<const float4*>(a + b1);
    const float4 v2 = *reinterpret_cast<const float4*>(a + b2);
    const float4 v3 = *reinterpret_cast<const float4*>(a + b3);
    const float4 d = *reinterpret_cast<const float4*>(dp + pix * ds + doff + 4 * c4);
    float4 o0, o1, o2, o3;
    pool_bwd1(v0.x, v1.x, v2.x, v3.x, d.x, act, o0.x, o1.x, o2.x, o3.x);
    pool_bwd1(v0.y, v1.y, v2.y, v3.y, d.y, act, o0.y, o1.y, o2.y, o3.y);
    pool_bwd1(v0.z, v1.z, v2.z, v3.z, d.z, act, o0.z, o1.z, o2.z, o3.z);
    pool_bwd1(v0.w, v1.w, v2.w, v3.w, d.w, act, o0.w, o1.w, o2.w, o3.w);
    *reinterpret_cast<float4*>(da + b0) = o0;
    *reinterpret_cast<float4*>(da + b1) = o1;
    *reinterpret_cast<float4*>(da + b2) = o2;
    *reinterpret_cast<float4*>(da + b3) = o3;
  }
}

// NCHW network input -> channels [doff, doff+C) of an NHWC buffer (the up1 concat buffer,
// arch_unet.py:240 `self.up1(x, pool0)` where pool0 is the raw input); channels
// [doff+C, zero_to) are the float4 padding of that buffer and are written as zeros.
__global__ __launch_bounds__(256) void k_nchw_to_slice(const float* __restrict__ x, int N, int C,
                                                       int H, int W, float* __restrict__ dst,
                                                       int ds, int doff, int zero_to) {
  const long total = (long)N * H * W;
  const long hw = (long)H * W;
  for (long p = (long)blockIdx.x * 256 + threadIdx.x; p < total; p += (long)gridDim.x * 256) {
    const long n = p / hw, r = p - n * hw;
    for (int c = 0; c < C; ++c) dst[p * ds + doff + c] = x[(n * C + c) * hw + r];
    for (int c = doff + C; c < zero_to; ++c) dst[p * ds + c] = 0.f;
  }
}

// ------------------------------------------------------------------------------------
// Neighbour sub-sampler: train.py:134-190.  Pair table train.py:151-154, within-cell
// index k = 2*dy + dx (space_to_depth/unfold order, train.py:134-138).
// ------------------------------------------------------------------------------------
__constant__ int kPairA[8] = {0, 0, 1, 2, 1, 2, 3, 3};
__constant__ int kPairB[8] = {1, 2, 3, 3, 0, 0, 1, 2};

__global__ __launch_bounds__(256) void k_subsample(const float* __restrict__ img, int N, int C,
                                                   int H, int W, const uint8_t* __restrict__ rd_in,
                                                   uint64_t seed, uint64_t offset,
                                                   uint64_t cell_base, float* __restrict__ sub1,
                                                   float* __restrict__ sub2,
                                                   uint8_t* __restrict__ rd_out) {
  const int h = H >> 1, w = W >> 1;
  const long cells = (long)N * h * w;
  for (long cell = (long)blockIdx.x * 256 + threadIdx.x; cell < cells;
       cell += (long)gridDim.x * 256) {
    int rd;
    if (rd_in) rd = rd_in[cell] & 7;
    else rd = (int)(philox_cell_u32(seed, offset, cell_base + (uint64_t)cell) & 7u);
    if (rd_out) rd_out[cell] = (uint8_t)rd;
    const int j = (int)(cell % w);
    const long t = cell / w;
    const int i = (int)(t % h);
    const int n = (int)(t / h);
    const int k1 = kPairA[rd], k2 = kPairB[rd];
    for (int c = 0; c < C; ++c) {
      const float* p = img + ((long)n * C + c) * H * W;
      const long o = (((long)n * C + c) * h + i) * w + j;
      sub1[o] = p[(long)(2 * i + (k1 >> 1)) * W + 2 * j + (k1 & 1)];
      sub2[o] = p[(long)(2 * i + (k2 >> 1)) * W + 2 * j + (k2 & 1)];
    }
  }
}

// Four cells per thread (cells 4b .. 4b + 3 of one sub-image row share Philox block b: one
// Philox evaluation instead of four), float4 / uchar4 stores; the same values as k_subsample.
// Needs w % 4 == 0 and cell_base % 4 == 0 (launch_subsample checks).
__global__ __launch_bounds__(256) void k_subsample4(const float* __restrict__ img, int N, int C,
                                                    int H, int W, const uint8_t* __restrict__ rd_in,
                                                    uint64_t seed, uint64_t offset,
                                                    uint64_t cell_base, float* __restrict__ sub1,
                                                    float* __restrict__ sub2,
                                                    uint8_t* __restrict__ rd_out) {
  const int h = H >> 1, w = W >> 1;
  const long quads = (long)N * h * w / 4;
  for (long qd = (long)blockIdx.x * 256 + threadIdx.x; qd < quads; qd += (long)gridDim.x * 256) {
    const long cell = 4 * qd;
    int rd[4];
    if (rd_in) {
      const uchar4 r4 = reinterpret_cast<const uchar4*>(rd_in)[qd];
      rd[0] = r4.x & 7; rd[1] = r4.y & 7; rd[2] = r4.z & 7; rd[3] = r4.w & 7;
    } else {
      const uint64_t blk = (cell_base + (uint64_t)cell) >> 2;
      const U32x4 o = philox4x32_10((uint32_t)blk, (uint32_t)(blk >> 32), (uint32_t)offset,
                                    (uint32_t)(offset >> 32), (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
      for (int k = 0; k < 4; ++k) rd[k] = (int)(o.v[k] & 7u);
    }
    if (rd_out) reinterpret_cast<uchar4*>(rd_out)[qd] =
        make_uchar4((uint8_t)rd[0], (uint8_t)rd[1], (uint8_t)rd[2], (uint8_t)rd[3]);
    const int j = (int)(cell % w);
    const long t = cell / w;
    const int i = (int)(t % h);
    const int n = (int)(t / h);
    for (int c = 0; c < C; ++c) {
      const float* p = img + ((long)n * C + c) * H * W + (long)(2 * i) * W + 2 * j;
      const float4 r0a = *reinterpret_cast<const float4*>(p), r0b = *reinterpret_cast<const float4*>(p + 4);
      const float4 r1a = *reinterpret_cast<const float4*>(p + W), r1b = *reinterpret_cast<const float4*>(p + W + 4);
      const float cellv[4][4] = {{r0a.x, r0a.y, r1a.x, r1a.y}, {r0a.z, r0a.w, r1a.z, r1a.w},
                                 {r0b.x, r0b.y, r1b.x, r1b.y}, {r0b.z, r0b.w, r1b.z, r1b.w}};
      float4 o1, o2;
      float* a1 = &o1.x;
      float* a2 = &o2.x;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        a1[k] = cellv[k][kPairA[rd[k]]];
        a2[k] = cellv[k][kPairB[rd[k]]];
      }
      const long o = (((long)n * C + c) * h + i) * w + j;
      *reinterpret_cast<float4*>(sub1 + o) = o1;
      *reinterpret_cast<float4*>(sub2 + o) = o2;
    }
  }
}

// generate_mask_pair output format: mask[4*cell + k] (train.py:163-171)
__global__ __launch_bounds__(256) void k_masks(const uint8_t* __restrict__ rd, int64_t ncells,
                                               uint8_t* __restrict__ m1, uint8_t* __restrict__ m2) {
  for (long cell = (long)blockIdx.x * 256 + threadIdx.x; cell < ncells;
       cell += (long)gridDim.x * 256) {
    const int r = rd[cell] & 7;
    const int a = kPairA[r], b = kPairB[r];
    uchar4 x1, x2;
    x1.x = a == 0; x1.y = a == 1; x1.z = a == 2; x1.w = a == 3;
    x2.x = b == 0; x2.y = b == 1; x2.z = b == 2; x2.w = b == 3;
    reinterpret_cast<uchar4*>(m1)[cell] = x1;
    reinterpret_cast<uchar4*>(m2)[cell] = x2;
  }
}

// generate_subimages(img, mask) for an arbitrary one-hot-per-cell bool mask
__global__ __launch_bounds__(256) void k_subimage_from_mask(const float* __restrict__ img, int N,
                                                            int C, int H, int W,
                                                            const uint8_t* __restrict__ mask,
                                                            float* __restrict__ sub) {
  const int h = H >> 1, w = W >> 1;
  const long cells = (long)N * h * w;
  for (long cell = (long)blockIdx.x * 256 + threadIdx.x; cell < cells;
       cell += (long)gridDim.x * 256) {
    const uchar4 mk = reinterpret_cast<const uchar4*>(mask)[cell];
    const int k = mk.x ? 0 : (mk.y ? 1 : (mk.z ? 2 : 3));
    const int j = (int)(cell % w);
    const long t = cell / w;
    const int i = (int)(t % h);
    const int n = (int)(t / h);
    for (int c = 0; c < C; ++c) {
      const float* p = img + ((long)n * C + c) * H * W;
      sub[(((long)n * C + c) * h + i) * w + j] = p[(long)(2 * i + (k >> 1)) * W + 2 * j + (k & 1)];
    }
  }
}

// ------------------------------------------------------------------------------------
// Gaussian noise: train.py:84-101 (gauss_fix / gauss_range).  Element e of the global
// stream uses Philox block e>>2 and Box-Muller pair (e>>1)&1.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_noise(const float* __restrict__ clean, int N,
                                               int64_t per_image, float std_,
                                               const float* __restrict__ std_img, uint64_t seed,
                                               uint64_t offset, uint64_t elem_base,
                                               float* __restrict__ noisy) {
  const long total = (long)N * per_image;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const float z = philox_normal(seed, offset, elem_base + (uint64_t)e);
    const float s = std_img ? std_img[e / per_image] : std_;
    noisy[e] = clean[e] + s * z;
  }
}

// Four elements per thread (elements 4b .. 4b + 3 are Philox block b's two Box-Muller pairs):
// one Philox evaluation and two logs / square roots instead of four, float4 loads and stores;
// the same values as k_noise (philox_normal's operations, sinf / cosf separately).  Needs
// per_image % 4 == 0, elem_base % 4 == 0 and 16-B aligned buffers (launch_noise checks).
__global__ __launch_bounds__(256) void k_noise4(const float* __restrict__ clean, int N,
                                                int64_t per_image, float std_,
                                                const float* __restrict__ std_img, uint64_t seed,
                                                uint64_t offset, uint64_t elem_base,
                                                float* __restrict__ noisy) {
  const long quads = (long)N * per_image / 4;
  for (long qd = (long)blockIdx.x * 256 + threadIdx.x; qd < quads; qd += (long)gridDim.x * 256) {
    const long e = 4 * qd;
    const uint64_t blk = (elem_base + (uint64_t)e) >> 2;
    const U32x4 o = philox4x32_10((uint32_t)blk, (uint32_t)(blk >> 32), (uint32_t)offset,
                                  (uint32_t)(offset >> 32), (uint32_t)seed, (uint32_t)(seed >> 32));
    float z[4];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const uint32_t a = o.v[2 * p], b = o.v[2 * p + 1];
      const float u1 = ((float)(a >> 8) + 1.0f) * (1.0f / 16777216.0f);
      const float u2 = (float)(b >> 8) * (1.0f / 16777216.0f);
      const float r = sqrtf(-2.0f * logf(u1));
      const float th = 6.283185307179586f * u2;
      z[2 * p] = r * cosf(th);
      z[2 * p + 1] = r * sinf(th);
    }
    const float sd = std_img ? std_img[e / per_image] : std_;
    const float4 c4 = reinterpret_cast<const float4*>(clean)[qd];
    reinterpret_cast<float4*>(noisy)[qd] =
        make_float4(c4.x + sd * z[0], c4.y + sd * z[1], c4.z + sd * z[2], c4.w + sd * z[3]);
  }
}

// Poisson noise: train.py:102-111 (poisson_fix / poisson_range), noisy = Poisson(lam x) / lam.
// The count is drawn by inversion of the Poisson CDF in fp64 with one 53-bit uniform per element
// (philox_uniform53): k = min{k : u <= F(k)}, F accumulated from p_0 = exp(-mu),
// p_k = p_{k-1} mu / k.  mu = lam x is formed in fp32 as torch.poisson receives it; mu <= 500
// (the host checks a scalar lam; a per-image lam outside (0, 500] makes that image's output NaN;
// the images are in [0, 1]), the loop is bounded at mu + 20 sqrt(mu) + 40.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_poisson(const float* __restrict__ clean, int N,
                                                 int64_t per_image, float lam,
                                                 const float* __restrict__ lam_img, uint64_t seed,
                                                 uint64_t offset, uint64_t elem_base,
                                                 float* __restrict__ noisy) {
  const long total = (long)N * per_image;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const float l = lam_img ? lam_img[e / per_image] : lam;
    if (!(l > 0.f && l <= 500.f)) {  // a per-image lam the host could not check: NaN, loudly
      noisy[e] = __builtin_nanf("");
      continue;
    }
    const float muf = l * clean[e];
    const double mu = muf > 0.f ? (double)muf : 0.0;
    const double u = philox_uniform53(seed, offset, elem_base + (uint64_t)e);
    double p = exp(-mu), F = p;
    const int kmax = (int)(mu + 20.0 * sqrt(mu)) + 40;
    int k = 0;
    while (u > F && k < kmax) {
      ++k;
      p *= mu / k;
      F += p;
    }
    noisy[e] = (float)k / l;
  }
}

// ------------------------------------------------------------------------------------
// Loss reductions: fixed grid, per-block fp64 partial sums, one finalize block.
// ------------------------------------------------------------------------------------
constexpr int kLossBlocks = 1024;
constexpr int kLossTerms = 4;
size_t loss_partials_bytes() { return sizeof(double) * kLossBlocks * kLossTerms; }

__device__ __forceinline__ double wave_sum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int T>
__device__ __forceinline__ void block_store_partials(double (&v)[T], double* partials) {
  __shared__ double red[4][T];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int t = 0; t < T; ++t) v[t] = wave_sum(v[t]);
  if (lane == 0)
#pragma unroll
    for (int t = 0; t < T; ++t) red[wv][t] = v[t];
  __syncthreads();
  if (threadIdx.x == 0)
#pragma unroll
    for (int t = 0; t < T; ++t)
      partials[blockIdx.x * kLossTerms + t] = ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t];
}

// training_script.md:141-153.  den1/den2 are the sub-images of the no-grad denoised output
// (training_script.md:143-144), gathered here with the same rd_idx.
__global__ __launch_bounds__(256) void k_n2n_loss(const float* __restrict__ out,
                                                  const float* __restrict__ sub2,
                                                  const float* __restrict__ den,
                                                  const uint8_t* __restrict__ rd, int N, int C,
                                                  int h, int w, float invM, float lamM,
                                                  float* __restrict__ dout,
                                                  double* __restrict__ partials) {
  const long total = (long)N * C * h * w;
  const int H = 2 * h, W = 2 * w;
  double v[2] = {0.0, 0.0};
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int j = (int)(e % w);
    long t = e / w;
    const int i = (int)(t % h);
    t /= h;
    const int c = (int)(t % C);
    const int n = (int)(t / C);
    const int r = rd[((long)n * h + i) * w + j] & 7;
    const int k1 = kPairA[r], k2 = kPairB[r];
    const float* dp = den + ((long)n * C + c) * H * W;
    const float d1 = dp[(long)(2 * i + (k1 >> 1)) * W + 2 * j + (k1 & 1)];
    const float d2 = dp[(long)(2 * i + (k2 >> 1)) * W + 2 * j + (k2 & 1)];
    const float diff = out[e] - sub2[e];
    const float ed = d1 - d2;
    const float q = diff - ed;
    v[0] += (double)diff * diff;
    v[1] += (double)q * q;
    // autograd of mean(diff^2) + lambda*mean(q^2): (1/M)*(2*diff) + (lambda/M)*(2*q)
    dout[e] = __fadd_rn(__fmul_rn(invM, __fmul_rn(2.f, diff)), __fmul_rn(lamM, __fmul_rn(2.f, q)));
  }
  block_store_partials<2>(v, partials);
}

// Sum of the first T terms of the block partials by one 256-thread block: thread t adds
// blocks t, t+256, ... in order, then a fixed tree (deterministic; result valid in thread 0).
template <int T>
__device__ __forceinline__ void sum_partials(const double* __restrict__ partials, int nblk,
                                             double (&out)[T]) {
  __shared__ double sh[T][256];
  const int t = threadIdx.x;
  double v[T];
#pragma unroll
  for (int k = 0; k < T; ++k) v[k] = 0.0;
  for (int b = t; b < nblk; b += 256)
#pragma unroll
    for (int k = 0; k < T; ++k) v[k] += partials[b * kLossTerms + k];
#pragma unroll
  for (int k = 0; k < T; ++k) sh[k][t] = v[k];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w)
#pragma unroll
      for (int k = 0; k < T; ++k) sh[k][t] += sh[k][t + w];
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < T; ++k) out[k] = sh[k][0];
}

__global__ __launch_bounds__(256) void k_n2n_finalize(const double* __restrict__ partials, int nblk,
                                                      double M, float lambda,
                                                      float* __restrict__ loss3) {
  double sums[2];
  sum_partials<2>(partials, nblk, sums);
  if (threadIdx.x != 0) return;
  const double s1 = sums[0], s2 = sums[1];
  const float l1 = (float)(s1 / M);
  const float l2 = lambda * (float)(s2 / M);
  loss3[0] = l1;
  loss3[1] = l2;
  loss3[2] = l1 + l2;
}

__device__ __forceinline__ float sgnf(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

// util.py:56-70 Structure_loss.  Per-element gradients are computed in gather form (each
// element looks at its TV neighbours), so no atomics are needed.
__global__ __launch_bounds__(256) void k_structure_loss(
    const float* __restrict__ pred, const float* __restrict__ pred2,
    const float* __restrict__ tgt, int N, int C, int H, int W, float ga, float gtv1, float gtv2,
    float gc, float* __restrict__ dpred, float* __restrict__ dpred2,
    double* __restrict__ partials) {
  const long total = (long)N * C * H * W;
  double v[4] = {0.0, 0.0, 0.0, 0.0};
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int x = (int)(e % W);
    const int y = (int)((e / W) % H);
    const float p = pred[e], p2 = pred2[e], tg = tgt[e];
    const float d0 = p - tg, dc = p2 - tg;
    v[0] += fabs((double)d0);
    v[3] += fabs((double)dc);
    float g2 = gc * sgnf(dc);
    if (y + 1 < H) {
      const float dv = pred2[e + W] - p2;  // tv1 term (y+1, y)
      v[1] += fabs((double)dv);
      g2 -= gtv1 * sgnf(dv);
    }
    if (y > 0) g2 += gtv1 * sgnf(p2 - pred2[e - W]);
    if (x + 1 < W) {
      const float dh = pred2[e + 1] - p2;  // tv2 term (x+1, x)
      v[2] += fabs((double)dh);
      g2 -= gtv2 * sgnf(dh);
    }
    if (x > 0) g2 += gtv2 * sgnf(p2 - pred2[e - 1]);
    dpred[e] = ga * sgnf(d0);
    dpred2[e] = g2;
  }
  block_store_partials<4>(v, partials);
}

__global__ __launch_bounds__(256) void k_structure_finalize(const double* __restrict__ partials,
                                                            int nblk, double M, double M1,
                                                            double M2, float alpha, float beta,
                                                            float gamma, float* __restrict__ loss5) {
  double s[4];
  sum_partials<4>(partials, nblk, s);
  if (threadIdx.x != 0) return;
  const float pix = (float)(s[0] / M), tv1 = (float)(s[1] / M1), tv2 = (float)(s[2] / M2),
              cst = (float)(s[3] / M);
  loss5[0] = pix;
  loss5[1] = tv1;
  loss5[2] = tv2;
  loss5[3] = cst;
  loss5[4] = alpha * pix + beta * ((tv1 + tv2) / 2.f) + gamma * cst;
}

// ------------------------------------------------------------------------------------
// Adam (torch/optim/adam.py _single_tensor_adam, amsgrad=False, weight_decay=0):
//   m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, value=1-b2)   (lerp as ATen's vectorised fmadd)
//   denom = v.sqrt() / sqrt(bc2) + eps; p.addcdiv_(m, denom, value=-lr/bc1)
// Contraction is disabled so every op rounds like the eager CPU kernels.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_adam(float* __restrict__ p, const float* __restrict__ g,
                                              float* __restrict__ m, float* __restrict__ v,
                                              int64_t n, float w1, float b2, float w2,
                                              float step_size, float bc2s, float eps,
                                              float gscale) {
#pragma clang fp contract(off)
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float gg = gscale == 1.f ? g[i] : g[i] * gscale;
    const float mo = m[i];
    const float mm = fmaf(w1, gg - mo, mo);     // ATen lerp_vec: fmadd(weight, end-start, start)
    const float vv = v[i] * b2 + (w2 * gg) * gg;  // addcmul: self + (value*t1)*t2
    const float denom = sqrtf(vv) / bc2s + eps;
    p[i] = p[i] + (-step_size * mm) / denom;      // addcdiv: self + (value*t1)/t2
    m[i] = mm;
    v[i] = vv;
  }
}

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
hipError_t launch_pool_fwd(const float* a, int N, int H, int W, int C, float* out, int os, int oo,
                           hipStream_t s) {
  const long total = (long)N * (H / 2) * (W / 2) * (C / 4);
  hipLaunchKernelGGL(k_pool_fwd, dim3(grid_for(total, 256, 65536)), dim3(256), 0, s, a, N, H, W,
                     C, out, os, oo);
  return hipGetLastError();
}

hipError_t launch_pool_bwd(const float* a, int N, int H, int W, int C, const float* dp, int ds,
                           int doff, int act, float* da, hipStream_t s) {
  const long total = (long)N * (H / 2) * (W / 2) * (C / 4);
  hipLaunchKernelGGL(k_pool_bwd, dim3(grid_for(total, 256, 65536)), dim3(256), 0, s, a, N, H, W,
                     C, dp, ds, doff, act, da);
  return hipGetLastError();
}

hipError_t launch_nchw_to_slice(const float* x, int N, int C, int H, int W, float* dst, int ds,
                                int doff, int zero_to, hipStream_t s) {
  const long total = (long)N * H * W;
  hipLaunchKernelGGL(k_nchw_to_slice, dim3(grid_for(total, 256, 65536)), dim3(256), 0, s, x, N, C,
                     H, W, dst, ds, doff, zero_to);
  return hipGetLastError();
}

hipError_t launch_subsample(const float* img, int N, int C, int H, int W, const uint8_t* rd_in,
                            uint64_t seed, uint64_t offset, uint64_t cell_base, float* sub1,
                            float* sub2, uint8_t* rd_out, hipStream_t s) {
  const long cells = (long)N * (H / 2) * (W / 2);
  const bool v4 = (W / 2) % 4 == 0 && cell_base % 4 == 0 && W % 4 == 0 &&
                  ((reinterpret_cast<uintptr_t>(img) | reinterpret_cast<uintptr_t>(sub1) |
                    reinterpret_cast<uintptr_t>(sub2) | reinterpret_cast<uintptr_t>(rd_in) |
                    reinterpret_cast<uintptr_t>(rd_out)) & 15) == 0;
  if (v4)
    hipLaunchKernelGGL(k_subsample4, dim3(grid_for(cells / 4, 256, 65536)), dim3(256), 0, s, img,
                       N, C, H, W, rd_in, seed, offset, cell_base, sub1, sub2, rd_out);
  else
    hipLaunchKernelGGL(k_subsample, dim3(grid_for(cells, 256, 65536)), dim3(256), 0, s, img, N, C,
                       H, W, rd_in, seed, offset, cell_base, sub1, sub2, rd_out);
  return hipGetLastError();
}

hipError_t launch_masks(const uint8_t* rd, int64_t ncells, uint8_t* m1, uint8_t* m2,
                        hipStream_t s) {
  hipLaunchKernelGGL(k_masks, dim3(grid_for(ncells, 256, 65536)), dim3(256), 0, s, rd, ncells, m1,
                     m2);
  return hipGetLastError();
}

hipError_t launch_subimage_from_mask(const float* img, int N, int C, int H, int W,
                                     const uint8_t* mask, float* sub, hipStream_t s) {
  const long cells = (long)N * (H / 2) * (W / 2);
  hipLaunchKernelGGL(k_subimage_from_mask, dim3(grid_for(cells, 256, 65536)), dim3(256), 0, s,
                     img, N, C, H, W, mask, sub);
  return hipGetLastError();
}

hipError_t launch_noise(const float* clean, int N, int64_t per_image, float std_,
                        const float* std_per_image, uint64_t seed, uint64_t offset,
                        uint64_t elem_base, float* noisy, hipStream_t s) {
  const long total = (long)N * per_image;
  if (per_image % 4 == 0 && elem_base % 4 == 0 &&
      ((reinterpret_cast<uintptr_t>(clean) | reinterpret_cast<uintptr_t>(noisy)) & 15) == 0)
    hipLaunchKernelGGL(k_noise4, dim3(grid_for(total / 4, 256, 65536)), dim3(256), 0, s, clean, N,
                       per_image, std_, std_per_image, seed, offset, elem_base, noisy);
  else
    hipLaunchKernelGGL(k_noise, dim3(grid_for(total, 256, 65536)), dim3(256), 0, s, clean, N,
                       per_image, std_, std_per_image, seed, offset, elem_base, noisy);
  return hipGetLastError();
}

hipError_t launch_poisson(const float* clean, int N, int64_t per_image, float lam,
                          const float* lam_per_image, uint64_t seed, uint64_t offset,
                          uint64_t elem_base, float* noisy, hipStream_t s) {
  const long total = (long)N * per_image;
  hipLaunchKernelGGL(k_poisson, dim3(grid_for(total, 256, 65536)), dim3(256), 0, s, clean, N,
                     per_image, lam, lam_per_image, seed, offset, elem_base, noisy);
  return hipGetLastError();
}

hipError_t launch_n2n_loss(const float* out, const float* sub2, const float* den,
                           const uint8_t* rd, int N, int C, int h, int w, float lambda,
                           float* dout, float* loss3, void* partials, hipStream_t s) {
  const double M = (double)N * C * h * w;
  const float Mf = (float)M;
  const float invM = 1.0f / Mf;       // mean backward: grad / numel
  const float lamM = lambda / Mf;     // (lambda * mean)' : lambda / numel
  double* part = static_cast<double*>(partials);
  hipLaunchKernelGGL(k_n2n_loss, dim3(kLossBlocks), dim3(256), 0, s, out, sub2, den, rd, N, C, h,
                     w, invM, lamM, dout, part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_n2n_finalize, dim3(1), dim3(256), 0, s, part, kLossBlocks, M, lambda, loss3);
  return hipGetLastError();
}

hipError_t launch_structure_loss(const float* pred, const float* pred2, const float* tgt, int N,
                                 int C, int H, int W, float alpha, float beta, float gamma,
                                 float* dpred, float* dpred2, float* loss5, void* partials,
                                 hipStream_t s) {
  const double M = (double)N * C * H * W;
  const double M1 = (double)N * C * (H - 1) * W, M2 = (double)N * C * H * (W - 1);
  // d/dx of alpha*mean|.|  = alpha/M * sgn ; of beta*(tv1+tv2)/2 = beta/2/M1 * sgn, ...
  const float ga = alpha / (float)M;
  const float gtv1 = (beta / 2.f) / (float)M1, gtv2 = (beta / 2.f) / (float)M2;
  const float gc = gamma / (float)M;
  double* part = static_cast<double*>(partials);
  hipLaunchKernelGGL(k_structure_loss, dim3(kLossBlocks), dim3(256), 0, s, pred, pred2, tgt, N, C,
                     H, W, ga, gtv1, gtv2, gc, dpred, dpred2, part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_structure_finalize, dim3(1), dim3(256), 0, s, part, kLossBlocks, M, M1, M2,
                     alpha, beta, gamma, loss5);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_accumulate_tail(float* __restrict__ dst,
                                                         const float* __restrict__ src, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    dst[i] += src[i];
}

__global__ __launch_bounds__(256) void k_accumulate(float* __restrict__ dst,
                                                    const float* __restrict__ src, long n) {
  const long n4 = n >> 2;
  float4* d4 = reinterpret_cast<float4*>(dst);
  const float4* s4 = reinterpret_cast<const float4*>(src);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float4 a = d4[i];
    const float4 b = s4[i];
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    d4[i] = a;
  }
  for (long i = 4 * n4 + (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    dst[i] += src[i];
}

hipError_t launch_accumulate(float* dst, const float* src, long n, hipStream_t s) {
  const bool vec = ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) == 0;
  long blocks = ((vec ? n / 4 : n) + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  if (vec) {
    hipLaunchKernelGGL(k_accumulate, dim3((unsigned)blocks), dim3(256), 0, s, dst, src, n);
  } else {  // unaligned views: the scalar tail loop covers everything
    hipLaunchKernelGGL(k_accumulate, dim3((unsigned)blocks), dim3(256), 0, s, dst, src, 0L);
    hipLaunchKernelGGL(k_accumulate_tail, dim3((unsigned)blocks), dim3(256), 0, s, dst, src, n);
  }
  return hipGetLastError();
}

hipError_t launch_adam(float* p, const float* g, float* m, float* v, int64_t n, float w1,
                       float b2, float w2, float step_size, float bc2s, float eps, float gscale,
                       hipStream_t s) {
  hipLaunchKernelGGL(k_adam, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, p, g, m, v, n, w1, b2,
                     w2, step_size, bc2s, eps, gscale);
  return hipGetLastError();
}

}  // namespace dn
