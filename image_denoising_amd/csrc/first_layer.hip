// Thin layers of the N2N U-Net for gfx950: enc_conv0 (arch_unet.py:116-117, 196:
// Conv2d(in_nc, 48, 3, padding=1) + LeakyReLU(0.2)) and the weight gradient of nin_c
// (arch_unet.py:190: Conv2d(96, out_nc, 1)).  With in_nc in {1, 3} the layer has 9 or 27 MACs per output channel: as an MFMA
// implicit GEMM its K would be padded to 8 (fwd) / 16 (wgrad) channels, so it is written as a
// direct VALU kernel that is HBM-bound on its 48-channel output instead.
//
//   k_enc0_fwd    one pixel per thread, all 48 output channels; weights (transposed, 4-channel
//                 vectors) in LDS, broadcast reads; the 256 pixels x 48 channels of a block are
//                 staged in LDS and written as one contiguous 48 KiB run of the NHWC output.
//                 The same pass copies the network input into its slice of the up1 concat
//                 buffer (the "pool0" skip of arch_unet.py:197, 247-248), zero-padding it to a
//                 float4 boundary.
//   k_enc0_wgrad  dW[co][ci][t] and db[co] as partial sums over a pixel range per block
//                 (fixed order), one slab row per block; the batched reduction adds the rows in order.
#include "dn_internal.h"

namespace dn {

constexpr int E0_CO = 48;
// k_enc0_fwd's output stage keeps 48 floats per pixel, channel quad q of pixel p at quad
// q ^ ((p >> 2) & 3): a 16-lane float4 write then covers all 16 four-bank groups (unswizzled, pixels
// p and p + 4 shared groups: 31 % of the launch's LDS-active cycles in conflicts,
// profiles/r4_pmc_sq_n2n.txt)
__device__ __forceinline__ int e0_quad(int p, int q) { return p * (E0_CO / 4) + (q ^ ((p >> 2) & 3)); }

template <int C>
__global__ __launch_bounds__(256) void k_enc0_fwd(const float* __restrict__ x, int N, int H,
                                                  int W, const float* __restrict__ w,
                                                  const float* __restrict__ b,
                                                  float* __restrict__ out, float* __restrict__ cat,
                                                  int cat_stride, int cat_off, int cat_zero_to,
                                                  float* __restrict__ xcopy, int obf) {
  constexpr int KT = 9 * C;
  __shared__ __attribute__((aligned(16))) float wl[(KT + 1) * E0_CO];  // [tap*C+ci | bias][co]
  __shared__ __attribute__((aligned(16))) float st[256 * E0_CO];
  const int tid = threadIdx.x;
  for (int e = tid; e < KT * E0_CO; e += 256) {
    const int co = e % E0_CO, j = e / E0_CO, t = j / C, ci = j - t * C;
    wl[e] = w[(co * C + ci) * 9 + t];
  }
  if (tid < E0_CO) wl[KT * E0_CO + tid] = b[tid];
  __syncthreads();

  const long total = (long)N * H * W, hw = (long)H * W;
  const long p0 = (long)blockIdx.x * 256;
  const long p = p0 + tid;
  if (p < total) {
    const long n = p / hw;
    const int r = (int)(p - n * hw), y = r / W, xx = r - y * W;
    const float* xn = x + n * C * hw;
    float xin[KT];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int yy = y + t / 3 - 1, xc = xx + t % 3 - 1;
      const bool in = yy >= 0 && yy < H && xc >= 0 && xc < W;
#pragma unroll
      for (int ci = 0; ci < C; ++ci) xin[t * C + ci] = in ? xn[ci * hw + (long)yy * W + xc] : 0.f;
    }
    const float4* w4 = reinterpret_cast<const float4*>(wl);
#pragma unroll
    for (int cq = 0; cq < E0_CO / 4; ++cq) {
      float4 v = w4[KT * (E0_CO / 4) + cq];
#pragma unroll
      for (int j = 0; j < KT; ++j) {
        const float4 ww = w4[j * (E0_CO / 4) + cq];
        v.x = fmaf(ww.x, xin[j], v.x); v.y = fmaf(ww.y, xin[j], v.y);
        v.z = fmaf(ww.z, xin[j], v.z); v.w = fmaf(ww.w, xin[j], v.w);
      }
      v.x = v.x > 0.f ? v.x : v.x * 0.2f; v.y = v.y > 0.f ? v.y : v.y * 0.2f;
      v.z = v.z > 0.f ? v.z : v.z * 0.2f; v.w = v.w > 0.f ? v.w : v.w * 0.2f;
      reinterpret_cast<float4*>(st)[e0_quad(tid, cq)] = v;
    }
    // the input's slice of the up1 concat buffer (centre tap = the pixel itself), and the
    // compact NCHW copy the weight gradients read (only when a backward follows)
    if (xcopy)
#pragma unroll
      for (int ci = 0; ci < C; ++ci) xcopy[(n * C + ci) * hw + r] = xin[4 * C + ci];
    float* d = cat + p * cat_stride + cat_off;
    // (no concat buffer: the plan's dec_conv1a reads the input itself, X6_T1)
    if (!cat) {
    } else if (C == 1 && cat_zero_to - cat_off == 4 && ((cat_stride | cat_off) & 3) == 0) {
      *reinterpret_cast<float4*>(d) = make_float4(xin[4], 0.f, 0.f, 0.f);
    } else {
#pragma unroll
      for (int ci = 0; ci < C; ++ci) d[ci] = xin[4 * C + ci];
      for (int c = cat_off + C; c < cat_zero_to; ++c) cat[p * cat_stride + c] = 0.f;
    }
  }
  __syncthreads();
  const long npx = total - p0 < 256 ? total - p0 : 256;
  const float4* s4 = reinterpret_cast<const float4*>(st);
  if (obf) {  // bf16 storage (RNE, the value the bf16 base's enc_conv1 stages anyway)
    typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
    u16x4* o2 = reinterpret_cast<u16x4*>(reinterpret_cast<unsigned short*>(out) + p0 * E0_CO);
    for (int e = tid; e < npx * (E0_CO / 4); e += 256) {
      const float4 v = s4[e0_quad(e / (E0_CO / 4), e % (E0_CO / 4))];
      const __bf16 q[4] = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
      o2[e] = u16x4{__builtin_bit_cast(unsigned short, q[0]), __builtin_bit_cast(unsigned short, q[1]),
                    __builtin_bit_cast(unsigned short, q[2]), __builtin_bit_cast(unsigned short, q[3])};
    }
    return;
  }
  float4* o4 = reinterpret_cast<float4*>(out + p0 * E0_CO);
  for (int e = tid; e < npx * (E0_CO / 4); e += 256) o4[e] = s4[e0_quad(e / (E0_CO / 4), e % (E0_CO / 4))];
}

// Weight gradient of a 3x3 conv with few input channels C and CO output channels:
// enc_conv0 (C = in_nc, CO = 48) and the network-input slice of dec_conv1a (C = in_nc,
// CO = 96, into its own compact slab).  The input operand is the network input itself, NCHW
// (a compact copy the forward keeps), so its rows stage with contiguous loads.  Block b owns
// image rows [R*b/splits, R*(b+1)/splits) of the flattened N*H rows (possibly none: it then
// writes zeros, so every slab row is defined) and walks them in 128-pixel segments: the
// gradient segment [128][CO] is staged in LDS with float4 loads, the input rows y-1..y+1
// (+halo) likewise, from registers the previous segment's loads filled; then NG = 256/CO pixel
// phases x CO output channels accumulate W[co][ci][t] and b[co] from broadcast LDS reads
// (threads past NG*CO only load).
// Slab row = W[co][cin_total][3][3] then b[co]; this kernel fills input channels
// [ci_base, ci_base + C) (+ b if with_bias).
constexpr int E0_SEG = 128;
template <int C, int CO>
__global__ __launch_bounds__(256) void k_wgrad_c3_thin(const float* __restrict__ g,
                                                       const float* __restrict__ x, int N, int H,
                                                       int W, float* __restrict__ slab,
                                                       long slab_stride, int cin_total,
                                                       int ci_base, int with_bias) {
  constexpr int KT = 9 * C, NG = 256 / CO;
  constexpr int SEG = E0_SEG * 48 / CO;  // 24 KiB gradient stage whatever CO
  __shared__ __attribute__((aligned(16))) float gr[SEG * CO];
  __shared__ float xr[3][C][SEG + 2];
  __shared__ float red[NG - 1][CO][KT + 1];
  const int tid = threadIdx.x, co = tid % CO, grp = tid / CO;
  float acc[KT + 1];
#pragma unroll
  for (int j = 0; j <= KT; ++j) acc[j] = 0.f;
  const long R = (long)N * H, HW = (long)H * W;
  const int rb = (int)(R * blockIdx.x / gridDim.x), re = (int)(R * (blockIdx.x + 1) / gridDim.x);
  // the block's segments k = (row rb + k / nseg, columns (k % nseg) * SEG ..); segment k + 1's
  // gradient and input values are loaded into registers while segment k computes
  const int nseg = (W + SEG - 1) / SEG;
  const long nk = (long)(re - rb) * nseg;
  constexpr int GI = (SEG * CO / 4 + 255) / 256, XI = (3 * C * (SEG + 2) + 255) / 256;
  float4 pgv[GI];
  float pxv[XI];
  auto seg_w = [&](long k) { const int x0 = (int)(k % nseg) * SEG; return W - x0 < SEG ? W - x0 : SEG; };
  auto load = [&](long k) {
    const int row = rb + (int)(k / nseg), x0 = (int)(k % nseg) * SEG, seg = seg_w(k);
    const int n = row / H, y = row - n * H;
    const float4* g4 = reinterpret_cast<const float4*>(g + ((long)row * W + x0) * CO);
#pragma unroll
    for (int i = 0; i < GI; ++i) {
      const int e = tid + 256 * i;
      pgv[i] = e < seg * (CO / 4) ? g4[e] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int e = tid + 256 * i;
      const int dy = e / (C * (seg + 2)), r = e - dy * (C * (seg + 2));
      const int ci = r / (seg + 2), xx = r - ci * (seg + 2);
      const int gy = y + dy - 1, gx = x0 + xx - 1;
      pxv[i] = (e < 3 * C * (seg + 2) && gy >= 0 && gy < H && gx >= 0 && gx < W)
                   ? x[((long)n * C + ci) * HW + (long)gy * W + gx]
                   : 0.f;
    }
  };
  auto store = [&](int seg) {
#pragma unroll
    for (int i = 0; i < GI; ++i) {
      const int e = tid + 256 * i;
      if (e < seg * (CO / 4)) reinterpret_cast<float4*>(gr)[e] = pgv[i];
    }
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int e = tid + 256 * i;
      const int dy = e / (C * (seg + 2)), r = e - dy * (C * (seg + 2));
      const int ci = r / (seg + 2), xx = r - ci * (seg + 2);
      if (e < 3 * C * (seg + 2)) xr[dy][ci][xx] = pxv[i];
    }
  };
  if (nk > 0) load(0);
  for (long k = 0; k < nk; ++k) {
    const int seg = seg_w(k);
    __syncthreads();  // every thread is done with segment k - 1's stage
    store(seg);
    if (k + 1 < nk) load(k + 1);
    __syncthreads();
    if (grp < NG) {
      for (int px = grp; px < seg; px += NG) {
        const float gv = gr[px * CO + co];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int ci = 0; ci < C; ++ci)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx)
              acc[ci * 9 + dy * 3 + dx] = fmaf(gv, xr[dy][ci][px + dx], acc[ci * 9 + dy * 3 + dx]);
        acc[KT] += gv;
      }
    }
  }
  if (grp >= 1 && grp < NG)
#pragma unroll
    for (int j = 0; j <= KT; ++j) red[grp - 1][co][j] = acc[j];
  __syncthreads();
  if (grp == 0) {
#pragma unroll
    for (int j = 0; j <= KT; ++j)
#pragma unroll
      for (int q = 0; q < NG - 1; ++q) acc[j] += red[q][co][j];
    float* row = slab + (long)blockIdx.x * slab_stride;
#pragma unroll
    for (int ci = 0; ci < C; ++ci)
#pragma unroll
      for (int t = 0; t < 9; ++t) row[((long)co * cin_total + ci_base + ci) * 9 + t] = acc[ci * 9 + t];
    if (with_bias) row[(long)CO * cin_total * 9 + co] = acc[KT];
  }
}

hipError_t launch_enc0_fwd(const float* x, int N, int C, int H, int W, const float* w,
                           const float* b, float* out, float* cat, int cat_stride, int cat_off,
                           int cat_zero_to, float* xcopy, hipStream_t s, bool out_bf16) {
  if (C < 1 || C > 4) return hipErrorInvalidValue;
  const long total = (long)N * H * W;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (C == 1)
    hipLaunchKernelGGL(k_enc0_fwd<1>, grid, dim3(256), 0, s, x, N, H, W, w, b, out, cat, cat_stride,
                       cat_off, cat_zero_to, xcopy, (int)out_bf16);
  else if (C == 2)
    hipLaunchKernelGGL(k_enc0_fwd<2>, grid, dim3(256), 0, s, x, N, H, W, w, b, out, cat, cat_stride,
                       cat_off, cat_zero_to, xcopy, (int)out_bf16);
  else if (C == 3)
    hipLaunchKernelGGL(k_enc0_fwd<3>, grid, dim3(256), 0, s, x, N, H, W, w, b, out, cat, cat_stride,
                       cat_off, cat_zero_to, xcopy, (int)out_bf16);
  else
    hipLaunchKernelGGL(k_enc0_fwd<4>, grid, dim3(256), 0, s, x, N, H, W, w, b, out, cat, cat_stride,
                       cat_off, cat_zero_to, xcopy, (int)out_bf16);
  return hipGetLastError();
}

int enc0_wgrad_splits(int N, int H, int W) {
  (void)W;
  const int rows = N * H;
  return rows < 1024 ? rows : 1024;
}

template <int CO>
static hipError_t run_c3_thin(const float* g, const float* x, int N, int C, int H, int W,
                              float* slab, long slab_stride, int cin_total, int ci_base,
                              int with_bias, int splits, hipStream_t s) {
#define DN_C3T(CC)                                                                          \
  hipLaunchKernelGGL((k_wgrad_c3_thin<CC, CO>), dim3(splits), dim3(256), 0, s, g, x, N, H, W, \
                     slab, slab_stride, cin_total, ci_base, with_bias)
  if (C == 1) DN_C3T(1);
  else if (C == 2) DN_C3T(2);
  else if (C == 3) DN_C3T(3);
  else if (C == 4) DN_C3T(4);
  else return hipErrorInvalidValue;
#undef DN_C3T
  return hipGetLastError();
}

// g: NHWC [N,H,W,cout] contiguous; x: NCHW [N,C,H,W] (the network input)
hipError_t launch_wgrad_c3_thin(const float* g, int cout, const float* x, int N, int C, int H,
                                int W, float* slab, long slab_stride, int cin_total, int ci_base,
                                int with_bias, int splits, hipStream_t s) {
  if (C < 1 || C > 4 || splits < 1) return hipErrorInvalidValue;
  if (cout == 48)
    return run_c3_thin<48>(g, x, N, C, H, W, slab, slab_stride, cin_total, ci_base, with_bias,
                           splits, s);
  if (cout == 96)
    return run_c3_thin<96>(g, x, N, C, H, W, slab, slab_stride, cin_total, ci_base, with_bias,
                           splits, s);
  return hipErrorInvalidValue;
}

hipError_t launch_enc0_wgrad(const float* g, int g_stride, const float* x, int N, int C, int H,
                             int W, float* slab, int splits, float* dwb, hipStream_t s,
                             RedBatch* rb) {
  if (g_stride != E0_CO) return hipErrorInvalidValue;
  const long n_el = (long)E0_CO * 9 * C + E0_CO;
  hipError_t e = launch_wgrad_c3_thin(g, E0_CO, x, N, C, H, W, slab, n_el, C, 0, 1, splits, s);
  if (e != hipSuccess) return e;
  return launch_reduce(slab, n_el, splits, n_el, dwb, s, rb);
}

// ------------------------------------------------------------------------------------
// dL/dx of the network input (the reference's autograd, arch_unet.py:196-248): x feeds
// enc_conv0 (C -> 48) and, as pool0, the last C channels of dec_conv1a's input (97 -> 96 for
// C = 1), so
//   dx[n][c][y][x] = sum_{t, co} W0[co][c][t] g0[n][y+1-ky][x+1-kx][co]
//                  + sum_{t, co} W1[co][c1 + c][t] g1[n][y+1-ky][x+1-kx][co]
// with g0 / g1 the gradients of the two layers' pre-activations (NHWC, 48 / 96 channels),
// out-of-image taps skipped.  One output pixel per thread, all C channels; the weights of the
// C input channels live transposed in LDS ([c][t][co], broadcast float4 reads); the 144
// gradient channels of the 9 neighbours come through L1/L2 as float4 rows.  Fixed summation
// order (taps, then enc_conv0's channels, then dec_conv1a's): deterministic.
template <int C>
__global__ __launch_bounds__(256) void k_dgrad_input(const float* __restrict__ g0,
                                                     const float* __restrict__ w0,
                                                     const float* __restrict__ g1,
                                                     const float* __restrict__ w1, int c1_total,
                                                     int c1_base, int N, int H, int W,
                                                     float* __restrict__ dx) {
  constexpr int C0 = 48, C1 = 96;
  __shared__ __attribute__((aligned(16))) float wl[C][9][C0 + C1];
  for (int e = threadIdx.x; e < C * 9 * (C0 + C1); e += 256) {
    const int co = e % (C0 + C1), r = e / (C0 + C1), t = r % 9, c = r / 9;
    wl[c][t][co] = co < C0 ? w0[((long)co * C + c) * 9 + t]
                           : w1[((long)(co - C0) * c1_total + c1_base + c) * 9 + t];
  }
  __syncthreads();
  const long hw = (long)H * W, total = (long)N * hw;
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= total) return;
  const long n = p / hw;
  const int r = (int)(p - n * hw), y = r / W, x = r - y * W;
  float acc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) acc[c] = 0.f;
#pragma unroll 1
  for (int t = 0; t < 9; ++t) {
    const int ky = t / 3, kx = t - 3 * ky, sy = y + 1 - ky, sx = x + 1 - kx;
    if (sy < 0 || sy >= H || sx < 0 || sx >= W) continue;
    const long q = n * hw + (long)sy * W + sx;
    const float4* a0 = reinterpret_cast<const float4*>(g0 + q * C0);
    const float4* a1 = reinterpret_cast<const float4*>(g1 + q * C1);
#pragma unroll
    for (int j = 0; j < (C0 + C1) / 4; ++j) {
      const float4 gv = j < C0 / 4 ? a0[j] : a1[j - C0 / 4];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float4 wv = *reinterpret_cast<const float4*>(&wl[c][t][4 * j]);
        acc[c] = fmaf(gv.x, wv.x, acc[c]);
        acc[c] = fmaf(gv.y, wv.y, acc[c]);
        acc[c] = fmaf(gv.z, wv.z, acc[c]);
        acc[c] = fmaf(gv.w, wv.w, acc[c]);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < C; ++c) dx[(n * C + c) * hw + r] = acc[c];
}

hipError_t launch_dgrad_input(const float* g0, const float* w0, const float* g1, const float* w1,
                              int c1_total, int c1_base, int N, int C, int H, int W, float* dx,
                              hipStream_t s) {
  const long total = (long)N * H * W;
  const dim3 grid((unsigned)((total + 255) / 256));
#define DN_DGI(CC)                                                                           \
  hipLaunchKernelGGL(k_dgrad_input<CC>, grid, dim3(256), 0, s, g0, w0, g1, w1, c1_total,    \
                     c1_base, N, H, W, dx)
  if (C == 1) DN_DGI(1);
  else if (C == 2) DN_DGI(2);
  else if (C == 3) DN_DGI(3);
  else if (C == 4) DN_DGI(4);
  else return hipErrorInvalidValue;
#undef DN_DGI
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// Weight gradient of a thin 1x1 conv with 96 input and few output channels (nin_c,
// arch_unet.py:190): dW[co][ci] = sum_p g[p][co] x[p][ci], db[co] = sum_p g[p][co].
// 240 threads = 10 pixel phases x 24 float4 channel quads; per block a contiguous pixel range;
// the phases are summed in a fixed order into one slab row in PyTorch layout (W[co][ci] then
// b[co]); the batched reduction sums the rows in order.
template <int CO>
__global__ __launch_bounds__(256) void k_wgrad_thin(const float* __restrict__ g, int g_stride,
                                                    const float* __restrict__ x, long npx, long per,
                                                    float* __restrict__ slab) {
  constexpr int NE = CO * 96 + CO;
  __shared__ float red[10][NE];
  const int tid = threadIdx.x, cq = tid % 24, ph = tid / 24;
  const long pb = (long)blockIdx.x * per;
  const long pe = pb + per < npx ? pb + per : npx;
  float4 acc[CO];
  float accb[CO];
#pragma unroll
  for (int o = 0; o < CO; ++o) { acc[o] = make_float4(0.f, 0.f, 0.f, 0.f); accb[o] = 0.f; }
  if (ph < 10) {
    const float4* x4 = reinterpret_cast<const float4*>(x);
#pragma unroll 2
    for (long p = pb + ph; p < pe; p += 10) {
      const float4 xv = x4[p * 24 + cq];
#pragma unroll
      for (int o = 0; o < CO; ++o) {
        const float gv = g[p * g_stride + o];
        acc[o].x = fmaf(gv, xv.x, acc[o].x); acc[o].y = fmaf(gv, xv.y, acc[o].y);
        acc[o].z = fmaf(gv, xv.z, acc[o].z); acc[o].w = fmaf(gv, xv.w, acc[o].w);
        accb[o] += gv;
      }
    }
#pragma unroll
    for (int o = 0; o < CO; ++o) {
      red[ph][o * 96 + 4 * cq] = acc[o].x; red[ph][o * 96 + 4 * cq + 1] = acc[o].y;
      red[ph][o * 96 + 4 * cq + 2] = acc[o].z; red[ph][o * 96 + 4 * cq + 3] = acc[o].w;
      if (cq == 0) red[ph][CO * 96 + o] = accb[o];
    }
  }
  __syncthreads();
  float* row = slab + (long)blockIdx.x * NE;
  for (int e = tid; e < NE; e += 256) {
    float t = red[0][e];
#pragma unroll
    for (int q = 1; q < 10; ++q) t += red[q][e];
    row[e] = t;
  }
}

int wgrad_thin_splits(long npx) {
  long sp = (npx + 511) / 512;  // >= 512 pixels per block
  if (sp > 2048) sp = 2048;
  return (int)(sp < 1 ? 1 : sp);
}

hipError_t launch_wgrad_thin(const float* g, int g_stride, int cout, const float* x, long npx,
                             float* slab, int splits, float* dwb, hipStream_t s, RedBatch* rb) {
  const long per = (npx + splits - 1) / splits;
  if (cout == 1)
    hipLaunchKernelGGL(k_wgrad_thin<1>, dim3(splits), dim3(256), 0, s, g, g_stride, x, npx, per, slab);
  else if (cout == 2)
    hipLaunchKernelGGL(k_wgrad_thin<2>, dim3(splits), dim3(256), 0, s, g, g_stride, x, npx, per, slab);
  else if (cout == 3)
    hipLaunchKernelGGL(k_wgrad_thin<3>, dim3(splits), dim3(256), 0, s, g, g_stride, x, npx, per, slab);
  else if (cout == 4)
    hipLaunchKernelGGL(k_wgrad_thin<4>, dim3(splits), dim3(256), 0, s, g, g_stride, x, npx, per, slab);
  else
    return hipErrorInvalidValue;
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const long n_el = (long)cout * 96 + cout;
  return launch_reduce(slab, n_el, splits, n_el, dwb, s, rb);
}

}  // namespace dn
