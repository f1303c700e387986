// Adapter finetune path (adapter.py:5-67, finetune.py:153-162, :269-289) for gfx950.
//
// OutputAdapter: out = base + conv2(relu(conv1(cat[noisy, base])))  with conv1 2C->16 3x3 and
// conv2 16->C 3x3 (pad 1).  Both convolutions are thin (<= 6 input or 16 output channels), so
// they run on the vector ALUs as ONE fused tile kernel: the 16 hidden channels live only in
// LDS (recomputed by the backward instead of being written to HBM).  Traffic per pixel: read
// noisy + base, write out (12*C bytes) -- HBM-bound, far below the MFMA roof.
//
// The backward produces only the adapter's parameter gradients (the base is frozen and run
// under no_grad, finetune.py:255-262; the noisy input needs none): a workgroup walks a fixed
// set of 16x16 tiles, keeps its share of the 449 (C=1) / 1315 (C=3) parameter sums in
// registers, writes one slab row, and the batched reduction adds the rows in a fixed order.
//
// The loss kernel fuses L1(pred, clean) + lambda * gradient_loss(pred, clean)
// (finetune.py:153-162) with its gradient in gather form (no atomics).
#include "dn_internal.h"

namespace dn {

constexpr int AD_T = 16;    // output tile edge
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int AD_HID = 16;  // hidden channels (adapter.py:13 default, finetune.py --adapter_hidden)

template <int C>
struct AdCfg {
  static constexpr int CI = 2 * C;
  // float offsets in the flat buffer (state_dict order: net.0.weight, net.0.bias, net.2.weight,
  // net.2.bias); net.0.weight starts at 0
  static constexpr int B1 = AD_HID * CI * 9, W2 = B1 + AD_HID, B2 = W2 + C * AD_HID * 9;
  static constexpr int NP = B2 + C;                  // parameter count
  static constexpr int PPT = (NP + 255) / 256;       // parameters per thread (backward)
  static constexpr int XE = AD_T + 4, HE = AD_T + 2; // input tile (halo 2), hidden tile (halo 1)
};

// noisy/base channel i of the concatenated adapter input at (gy, gx), zero outside the image
template <int C>
__device__ __forceinline__ void load_cat_tile(const float* __restrict__ noisy,
                                              const float* __restrict__ base, int n, int H, int W,
                                              int y0, int x0, float* sx) {
  using A = AdCfg<C>;
  for (int e = threadIdx.x; e < A::CI * A::XE * A::XE; e += 256) {
    const int i = e / (A::XE * A::XE), r = e - i * A::XE * A::XE;
    const int gy = y0 + r / A::XE, gx = x0 + r % A::XE;
    float v = 0.f;
    if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
      const float* src = i < C ? noisy : base;
      v = src[(((long)n * C + (i % C)) * H + gy) * W + gx];
    }
    sx[e] = v;
  }
}

// hidden = relu(conv1(x) + b1) on the (AD_T+2)^2 grid around the tile, 0 outside the image
// (conv2's zero padding)
template <int C>
__device__ __forceinline__ void hidden_tile(const float* __restrict__ prm, const float* sx, int H,
                                            int W, int y0, int x0, float* sh) {
  using A = AdCfg<C>;
  for (int e = threadIdx.x; e < A::HE * A::HE; e += 256) {
    const int yy = e / A::HE, xx = e - yy * A::HE;
    const int gy = y0 + yy, gx = x0 + xx;
    const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
    float xin[A::CI][9];
#pragma unroll
    for (int i = 0; i < A::CI; ++i)
#pragma unroll
      for (int t = 0; t < 9; ++t) xin[i][t] = sx[i * A::XE * A::XE + (yy + t / 3) * A::XE + xx + t % 3];
#pragma unroll 4
    for (int h = 0; h < AD_HID; ++h) {
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < A::CI; ++i)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc = fmaf(prm[(h * A::CI + i) * 9 + t], xin[i][t], acc);
      acc += prm[A::B1 + h];
      sh[h * A::HE * A::HE + e] = in ? fmaxf(acc, 0.f) : 0.f;
    }
  }
}

template <int C>
__global__ __launch_bounds__(256) void k_adapter_fwd(const float* __restrict__ prm,
                                                     const float* __restrict__ noisy,
                                                     const float* __restrict__ base, int N, int H,
                                                     int W, float* __restrict__ out) {
  using A = AdCfg<C>;
  __shared__ float sx[A::CI * A::XE * A::XE];
  __shared__ float sh[AD_HID * A::HE * A::HE];
  const int tiles_x = (W + AD_T - 1) / AD_T;
  const int ty0 = (blockIdx.x / tiles_x) * AD_T, tx0 = (blockIdx.x % tiles_x) * AD_T;
  const int n = blockIdx.y;
  load_cat_tile<C>(noisy, base, n, H, W, ty0 - 2, tx0 - 2, sx);
  __syncthreads();
  hidden_tile<C>(prm, sx, H, W, ty0 - 1, tx0 - 1, sh);
  __syncthreads();
  const int py = threadIdx.x / AD_T, px = threadIdx.x % AD_T;
  const int gy = ty0 + py, gx = tx0 + px;
  if (gy >= H || gx >= W) return;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    float acc = 0.f;
#pragma unroll 4
    for (int h = 0; h < AD_HID; ++h)
#pragma unroll
      for (int t = 0; t < 9; ++t)
        acc = fmaf(prm[A::W2 + (c * AD_HID + h) * 9 + t],
                   sh[h * A::HE * A::HE + (py + t / 3) * A::HE + px + t % 3], acc);
    const long o = (((long)n * C + c) * H + gy) * W + gx;
    out[o] = base[o] + (acc + prm[A::B2 + c]);  // adapter.py:26 base_out + delta
  }
}

// Parameter-gradient tasks of a tile, each a kernel row of one sum (its three horizontal taps
// share the row reads): dW1 (h, i, ky), dW2 (c, h, ky), then db1 (h) and db2 (c).  A task reads
// 16-float rows as float4 / float2 vectors and sums in the pixel order q = 16 r + col.
template <int C>
struct AdTasks {
  static constexpr int T1 = AD_HID * 2 * C * 3, T2 = C * AD_HID * 3, TB1 = AD_HID, TB2 = C;
  // slots: each task type starts on a wave boundary, so no wave runs two types' loops in turn
  static constexpr int S2 = (T1 + 63) / 64 * 64, SB = (S2 + T2 + 63) / 64 * 64;
  static constexpr int NS = SB + TB1 + TB2;     // slots used
  static constexpr int TPT = (NS + 255) / 256;  // slots per thread
};

template <int C>
__global__ __launch_bounds__(256, 3) void k_adapter_bwd(const float* __restrict__ prm,
                                                     const float* __restrict__ noisy,
                                                     const float* __restrict__ base,
                                                     const float* __restrict__ dout, int N, int H,
                                                     int W, float* __restrict__ slab) {
  using A = AdCfg<C>;
  using T = AdTasks<C>;
  // TP: dpre row pitch, padded so that the 16-float row reads of tasks with different h start
  // on different banks (h * 256 floats would all hit the same ones)
  constexpr int XA = A::XE * A::XE, HA = A::HE * A::HE, TA = AD_T * AD_T, TP = TA + 4;
  __shared__ __attribute__((aligned(16))) float sx[A::CI * XA];
  __shared__ __attribute__((aligned(16))) float sh[AD_HID * HA];
  __shared__ __attribute__((aligned(16))) float sdo[C * HA];
  __shared__ __attribute__((aligned(16))) float sdp[AD_HID * TP];
  const int tid = threadIdx.x;
  const int tiles_x = (W + AD_T - 1) / AD_T, tiles_y = (H + AD_T - 1) / AD_T;
  const long ntiles = (long)N * tiles_x * tiles_y;
  float acc[T::TPT][3];
#pragma unroll
  for (int j = 0; j < T::TPT; ++j) acc[j][0] = acc[j][1] = acc[j][2] = 0.f;

  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int n = (int)(tile / ((long)tiles_x * tiles_y));
    const int r = (int)(tile - (long)n * tiles_x * tiles_y);
    const int ty0 = (r / tiles_x) * AD_T, tx0 = (r % tiles_x) * AD_T;
    // the weights re-read per tile (scalar loads): an opaque copy of the pointer keeps the
    // compiler from hoisting all of them out of the tile loop into vector registers
    const float* pw = prm;
    asm volatile("" : "+s"(pw));
    int tt = tid;  // likewise for the per-thread LDS addresses (hoisted, they spill for C = 3)
    asm volatile("" : "+v"(tt));
    load_cat_tile<C>(noisy, base, n, H, W, ty0 - 2, tx0 - 2, sx);
    for (int e = tid; e < C * HA; e += 256) {  // dout with a 1-pixel halo, 0 outside the image
      const int c = e / HA, q = e - c * HA;
      const int gy = ty0 - 1 + q / A::HE, gx = tx0 - 1 + q % A::HE;
      sdo[e] = (gy >= 0 && gy < H && gx >= 0 && gx < W)
                   ? dout[(((long)n * C + c) * H + gy) * W + gx] : 0.f;
    }
    __syncthreads();
    hidden_tile<C>(pw, sx, H, W, ty0 - 1, tx0 - 1, sh);
    __syncthreads();
    {  // d pre-activation of the hidden layer at the tile's own pixels
      const int qy = tt / AD_T, qx = tt % AD_T;
#pragma unroll 2
      for (int h = 0; h < AD_HID; ++h) {
        float g = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
          for (int t = 0; t < 9; ++t)  // hidden q feeds out p = q - (dy-1, dx-1)
            g = fmaf(pw[A::W2 + (c * AD_HID + h) * 9 + t],
                     sdo[c * HA + (qy + 2 - t / 3) * A::HE + qx + 2 - t % 3], g);
        const bool on = sh[h * HA + (qy + 1) * A::HE + qx + 1] > 0.f;  // relu'
        sdp[h * TP + tt] = on ? g : 0.f;
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < T::TPT; ++j) {
      const int k = tt + 256 * j;
      if (k >= T::NS || (k >= T::T1 && k < T::S2) || (k >= T::S2 + T::T2 && k < T::SB)) continue;
      float a0 = acc[j][0], a1 = acc[j][1], a2 = acc[j][2];
      if (k < T::T1) {  // dW1[h][i][ky][kx] = sum_q dpre[h][q] * x[i][q + (ky-1, kx-1)]
        const int h = k / (A::CI * 3), i = (k / 3) % A::CI, ky = k % 3;
        const float* xs = sx + i * XA + (ky + 1) * A::XE;  // input row r+ky+1 (halo 2), cols 0..19
        const float* ds = sdp + h * TP;
#pragma unroll 1
        for (int rr = 0; rr < AD_T; ++rr) {
          f4 d[4], x[5];
#pragma unroll
          for (int v = 0; v < 4; ++v) d[v] = *reinterpret_cast<const f4*>(ds + rr * AD_T + 4 * v);
#pragma unroll
          for (int v = 0; v < 5; ++v) x[v] = *reinterpret_cast<const f4*>(xs + rr * A::XE + 4 * v);
#pragma unroll
          for (int c = 0; c < AD_T; ++c) {
            const float dc = d[c >> 2][c & 3];
            a0 = fmaf(dc, x[(c + 1) >> 2][(c + 1) & 3], a0);
            a1 = fmaf(dc, x[(c + 2) >> 2][(c + 2) & 3], a1);
            a2 = fmaf(dc, x[(c + 3) >> 2][(c + 3) & 3], a2);
          }
        }
      } else if (k < T::SB) {  // dW2[c][h][ky][kx] = sum_p dout[c][p] * hid[h][p + (ky-1, kx-1)]
        const int kk = k - T::S2;
        const int c = kk / (AD_HID * 3), h = (kk / 3) % AD_HID, ky = kk % 3;
        const float* hs = sh + h * HA + ky * A::HE;  // hidden row r+ky (halo 1), cols 0..17
        const float* os = sdo + c * HA + A::HE;      // dout row r+1, cols 0..17 (1..16 used)
#pragma unroll 1
        for (int rr = 0; rr < AD_T; ++rr) {
          f2 o[9], hv[9];
#pragma unroll
          for (int v = 0; v < 9; ++v) {
            o[v] = *reinterpret_cast<const f2*>(os + rr * A::HE + 2 * v);
            hv[v] = *reinterpret_cast<const f2*>(hs + rr * A::HE + 2 * v);
          }
#pragma unroll
          for (int cc = 0; cc < AD_T; ++cc) {
            const float oc = o[(cc + 1) >> 1][(cc + 1) & 1];
            a0 = fmaf(oc, hv[cc >> 1][cc & 1], a0);
            a1 = fmaf(oc, hv[(cc + 1) >> 1][(cc + 1) & 1], a1);
            a2 = fmaf(oc, hv[(cc + 2) >> 1][(cc + 2) & 1], a2);
          }
        }
      } else if (k < T::SB + T::TB1) {  // db1
        const float* ds = sdp + (k - T::SB) * TP;
        for (int q = 0; q < TA; q += 4) {
          const f4 v = *reinterpret_cast<const f4*>(ds + q);
          a0 += v[0]; a0 += v[1]; a0 += v[2]; a0 += v[3];
        }
      } else {  // db2
        const float* os = sdo + (k - T::SB - T::TB1) * HA + A::HE;
        for (int rr = 0; rr < AD_T; ++rr)
#pragma unroll
          for (int cc = 1; cc <= AD_T; ++cc) a0 += os[rr * A::HE + cc];
      }
      acc[j][0] = a0; acc[j][1] = a1; acc[j][2] = a2;
    }
    __syncthreads();
  }
  // the slab row in state_dict order (AdCfg offsets)
  float* row = slab + (long)blockIdx.x * A::NP;
#pragma unroll
  for (int j = 0; j < T::TPT; ++j) {
    const int k = tid + 256 * j;
    if (k >= T::NS || (k >= T::T1 && k < T::S2) || (k >= T::S2 + T::T2 && k < T::SB)) continue;
    if (k < T::T1) {
      const int h = k / (A::CI * 3), i = (k / 3) % A::CI, ky = k % 3;
      for (int kx = 0; kx < 3; ++kx) row[(h * A::CI + i) * 9 + ky * 3 + kx] = acc[j][kx];
    } else if (k < T::SB) {
      const int kk = k - T::S2;
      const int c = kk / (AD_HID * 3), h = (kk / 3) % AD_HID, ky = kk % 3;
      for (int kx = 0; kx < 3; ++kx) row[A::W2 + (c * AD_HID + h) * 9 + ky * 3 + kx] = acc[j][kx];
    } else if (k < T::SB + T::TB1) {
      row[A::B1 + k - T::SB] = acc[j][0];
    } else {
      row[A::B2 + k - T::SB - T::TB1] = acc[j][0];
    }
  }
}

// ---- finetune loss (finetune.py:153-162, :283-285) ---------------------------------------
constexpr int kFtBlocks = 1024;

__device__ __forceinline__ float sgn1(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

__device__ __forceinline__ double wsum64(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(256) void k_ft_loss(const float* __restrict__ p,
                                                 const float* __restrict__ t, int N, int C, int H,
                                                 int W, float g0, float gx, float gy,
                                                 float* __restrict__ dp,
                                                 double* __restrict__ partials) {
  const long total = (long)N * C * H * W;
  double v[3] = {0.0, 0.0, 0.0};
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int x = (int)(e % W);
    const int y = (int)((e / W) % H);
    const float pe = p[e], te = t[e];
    const float d0 = pe - te;
    v[0] += fabs((double)d0);
    float g = g0 * sgn1(d0);
    // gradient(x) = (x[..., 1:] - x[..., :-1], x[:, :, 1:] - x[:, :, :-1])  (finetune.py:153-156)
    if (x + 1 < W) {
      const float a = (p[e + 1] - pe) - (t[e + 1] - te);
      v[1] += fabs((double)a);
      g -= gx * sgn1(a);
    }
    if (x > 0) g += gx * sgn1((pe - p[e - 1]) - (te - t[e - 1]));
    if (y + 1 < H) {
      const float b = (p[e + W] - pe) - (t[e + W] - te);
      v[2] += fabs((double)b);
      g -= gy * sgn1(b);
    }
    if (y > 0) g += gy * sgn1((pe - p[e - W]) - (te - t[e - W]));
    dp[e] = g;
  }
  __shared__ double red[4][3];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 3; ++k) v[k] = wsum64(v[k]);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < 3; ++k) red[wv][k] = v[k];
  __syncthreads();
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < 3; ++k)
      partials[blockIdx.x * 4 + k] = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
}

__global__ __launch_bounds__(256) void k_ft_finalize(const double* __restrict__ partials, int nblk,
                                                     double M, double Mx, double My, float lam,
                                                     float* __restrict__ loss3) {
  __shared__ double sh[3][256];
  const int t = threadIdx.x;
  double v[3] = {0.0, 0.0, 0.0};
  for (int b = t; b < nblk; b += 256)
#pragma unroll
    for (int k = 0; k < 3; ++k) v[k] += partials[b * 4 + k];
#pragma unroll
  for (int k = 0; k < 3; ++k) sh[k][t] = v[k];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w)
#pragma unroll
      for (int k = 0; k < 3; ++k) sh[k][t] += sh[k][t + w];
    __syncthreads();
  }
  if (t != 0) return;
  const float l1 = (float)(sh[0][0] / M);
  const float lg = (float)(sh[1][0] / Mx) + (float)(sh[2][0] / My);
  loss3[0] = l1;
  loss3[1] = lg;
  loss3[2] = l1 + lam * lg;
}

// ---- launchers ------------------------------------------------------------------------------
long adapter_param_count(int C) {
  if (C == 1) return AdCfg<1>::NP;
  if (C == 3) return AdCfg<3>::NP;
  return -1;
}

// one round of resident workgroups (3 per CU, bound by LDS): 1024 left a second round of 256
int adapter_bwd_blocks(int N, int H, int W) {
  const long tiles = (long)N * ((H + AD_T - 1) / AD_T) * ((W + AD_T - 1) / AD_T);
  return (int)(tiles < 768 ? tiles : 768);
}

hipError_t launch_adapter_fwd(const float* prm, const float* noisy, const float* base, int N, int C,
                              int H, int W, float* out, hipStream_t s) {
  const dim3 grid(((W + AD_T - 1) / AD_T) * ((H + AD_T - 1) / AD_T), N);
  if (C == 1) hipLaunchKernelGGL(k_adapter_fwd<1>, grid, dim3(256), 0, s, prm, noisy, base, N, H, W, out);
  else if (C == 3) hipLaunchKernelGGL(k_adapter_fwd<3>, grid, dim3(256), 0, s, prm, noisy, base, N, H, W, out);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_adapter_bwd(const float* prm, const float* noisy, const float* base,
                              const float* dout, int N, int C, int H, int W, float* dprm,
                              float* slab, hipStream_t s) {
  const int nb = adapter_bwd_blocks(N, H, W);
  if (C == 1) hipLaunchKernelGGL(k_adapter_bwd<1>, dim3(nb), dim3(256), 0, s, prm, noisy, base, dout, N, H, W, slab);
  else if (C == 3) hipLaunchKernelGGL(k_adapter_bwd<3>, dim3(nb), dim3(256), 0, s, prm, noisy, base, dout, N, H, W, slab);
  else return hipErrorInvalidValue;
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const long np = adapter_param_count(C);
  return launch_reduce(slab, np, nb, np, dprm, s);
}

hipError_t launch_ft_loss(const float* pred, const float* tgt, int N, int C, int H, int W,
                          float lam, float* dpred, float* loss3, void* partials, hipStream_t s) {
  const double M = (double)N * C * H * W;
  const double Mx = (double)N * C * H * (W - 1), My = (double)N * C * (H - 1) * W;
  // d/dp of mean|.| = sgn / numel; gradient_loss terms carry lambda_grad (finetune.py:285)
  const float g0 = 1.0f / (float)M, gx = lam / (float)Mx, gy = lam / (float)My;
  double* part = static_cast<double*>(partials);
  hipLaunchKernelGGL(k_ft_loss, dim3(kFtBlocks), dim3(256), 0, s, pred, tgt, N, C, H, W, g0, gx, gy,
                     dpred, part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_ft_finalize, dim3(1), dim3(256), 0, s, part, kFtBlocks, M, Mx, My, lam, loss3);
  return hipGetLastError();
}

}  // namespace dn
