// Shared bf16x6 building blocks: exact three-way bf16 split of fp32 operands and the
// six-product 16x16x32 MFMA block (used by the conv forward / data-gradient kernels in
// conv_x6.hip and by the 3x3 weight-gradient kernel in conv.hip).  See conv_x6.hip's header.
#pragma once

#include "conv_epi.h"

namespace dn {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// bf16 elements of one weight stage (one tap, three planes of NP x 32) in the packed image,
// padded to whole rounds of the pipelined kernel's DMA (8 waves x 1 KiB dwordx4 LDS loads;
// the 12-byte form would fit 18 KiB exactly, but it writes lane x 16 B in LDS, not lane x 12)
__host__ __device__ constexpr int x6_wst(int np) {
  return (3 * np * 32 * 2 + 8191) / 8192 * 8192 / 2;
}

// 16-B quad q of LDS row `row` lives at quad q ^ ((row >> 1) & 3)
__device__ __forceinline__ int x6_swz(int row, int q) { return q ^ ((row >> 1) & 3); }

// v = h + m + l exactly (normal fp32 v); each step's remainder is exact in fp32
__device__ __forceinline__ void split3(float v, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)v;
  const float r = v - (float)h;
  m = (__bf16)r;
  l = (__bf16)(r - (float)m);
}

typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

// split3 of two values at once (v_cvt_pk_bf16_f32 for the conversions, scalar subtractions): the
// three 32-bit words each hold the (a, b) pieces of one plane, low half = a
__device__ __forceinline__ void split3x2(float a, float b, unsigned& h, unsigned& m,
                                         unsigned& l) {
  const f32x2_t v = {a, b};
  h = __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2_t));
  // scalar subtractions (see x6_acc_add)
  const float ra = a - __uint_as_float(h << 16), rb = b - __uint_as_float(h & 0xffff0000u);
  const f32x2_t r = {ra, rb};
  m = __builtin_bit_cast(unsigned, __builtin_convertvector(r, bf16x2_t));
  const f32x2_t r2 = {ra - __uint_as_float(m << 16), rb - __uint_as_float(m & 0xffff0000u)};
  l = __builtin_bit_cast(unsigned, __builtin_convertvector(r2, bf16x2_t));
}

// the three bf16x8 planes of eight fp32 values (element e = v[e])
__device__ __forceinline__ void split3x8(const float (&v)[8], bf16x8& p0, bf16x8& p1,
                                         bf16x8& p2) {
  u32x4_t h, m, l;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    unsigned hh, mm, ll;
    split3x2(v[2 * j], v[2 * j + 1], hh, mm, ll);
    h[j] = hh; m[j] = mm; l[j] = ll;
  }
  p0 = __builtin_bit_cast(bf16x8, h);
  p1 = __builtin_bit_cast(bf16x8, m);
  p2 = __builtin_bit_cast(bf16x8, l);
}

// 16 bytes per lane from a buffer resource into LDS at lds + 16 * lane (buffer_load_dwordx4 ...
// lds).  The builtin exists only for the device pass: in the host pass it would invalidate the
// calling kernel templates and drop their host stubs without a diagnostic.
__device__ __forceinline__ void buf_lds16(__amdgpu_buffer_rsrc_t rs, void* lds, int voffset) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds, 16,
                                           voffset, 0, 0, 0);
#else
  (void)rs; (void)lds; (void)voffset;
#endif
}

__device__ __forceinline__ f32x4 mfma_bf16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// acc += hi + lo as scalar v_add_f32 (conv_x6.hip is built with -fno-slp-vectorize): a packed
// v_pk_add_f32 beside MFMAs costs more issue cycles than the two scalar adds it replaces
// (A/B on one box: k_wgrad3s 96->96 at 64 x 128^2 1.127 -> 1.050 ms, the step 25.2 -> 24.8-25.1 ms)
__device__ __forceinline__ void x6_acc_add(f32x4& acc, const f32x4& hi, const f32x4& lo) {
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r] = acc[r] + (hi[r] + lo[r]);
}

// One 16x16x32 block of every fragment of a wave: acc[m][q] += sum_k A[m] B[q] at fp32 accuracy.
// The leading product a0*b0 and the five corrections are summed by the matrix core from zero
// (hi, lo) and only then added to the running fp32 sum with a round-to-nearest VALU add: the
// matrix core's internal alignment rounds toward -inf, which on a long running sum (6 x 27
// MFMAs per output for K = 96) leaves a small negative bias that the weight-gradient sums over
// ~1e5 pixels would turn into a visible error; on a fresh 32-term block it is ~50x smaller.
// QG output-channel fragments are processed together (temporaries 8*MT*QG registers) so that
// the lo chain has MT*QG - 1 independent MFMAs between dependent ones.
// fragment-group width: >= 4 independent lo chains within the register budget
constexpr int x6_qg(int mt, int nt) { return mt >= 4 ? 1 : (mt == 2 ? (nt % 2 ? 3 : 2) : nt); }

// the fragment group [q0, q0 + QG) of x6_block
template <int MT, int NT, int QG>
__device__ __forceinline__ void x6_group(f32x4 (&acc)[MT][NT], const bf16x8 (&av)[3][MT],
                                         const bf16x8 (&bv)[3][NT], int q0) {
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  constexpr int PA[4] = {1, 0, 1, 2}, PB[4] = {0, 2, 1, 0};
  f32x4 hi[MT][QG], lo[MT][QG];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int g = 0; g < QG; ++g) hi[m][g] = mfma_bf16(av[0][m], bv[0][q0 + g], z);
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int g = 0; g < QG; ++g) lo[m][g] = mfma_bf16(av[0][m], bv[1][q0 + g], z);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int g = 0; g < QG; ++g)
        lo[m][g] = mfma_bf16(av[PA[j]][m], bv[PB[j]][q0 + g], lo[m][g]);
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int g = 0; g < QG; ++g) x6_acc_add(acc[m][q0 + g], hi[m][g], lo[m][g]);
}

template <int MT, int NT, int QG>
__device__ __forceinline__ void x6_block(f32x4 (&acc)[MT][NT], const bf16x8 (&av)[3][MT],
                                         const bf16x8 (&bv)[3][NT]) {
  static_assert(NT % QG == 0, "whole fragment groups");
#pragma unroll
  for (int q0 = 0; q0 < NT; q0 += QG) x6_group<MT, NT, QG>(acc, av, bv, q0);
}

// Carried-correction form (the 3x3 forward / data-gradient kernels): the leading product a0*b0
// of a block is still summed from zero and added to the running sum `acc` by a round-to-nearest
// VALU add, but the five corrections chain across blocks in their own accumulator `accl`
// (added to acc once, before the epilogue).  The corrections are <= 2^-7 of the products they
// correct, so the matrix core's alignment bias on that chain is <= 2^-7 of the bias a chained
// leading sum would carry -- below one fp32 rounding of the output over a K = 864 dot product --
// while the block costs 4 VALU adds per fragment instead of 8 and no fresh lo chain.
// fragment-group width of the carried form: one chain per fragment (a single 16x16x32 bf16
// accumulation chain issues back-to-back, MI355X_MICROARCH.md); the narrow group keeps the hi
// temporaries and the B look-ahead small enough for the extra accl registers
constexpr int x6_qgc(int, int) { return 1; }
template <int MT, int NT, int QG>
__device__ __forceinline__ void x6_group_c(f32x4 (&acc)[MT][NT], f32x4 (&accl)[MT][NT],
                                           const bf16x8 (&av)[3][MT], const bf16x8 (&bv)[3][NT],
                                           int q0) {
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  constexpr int PA[5] = {0, 1, 0, 1, 2}, PB[5] = {1, 0, 2, 1, 0};
  f32x4 hi[MT][QG];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int g = 0; g < QG; ++g) hi[m][g] = mfma_bf16(av[0][m], bv[0][q0 + g], z);
#pragma unroll
  for (int j = 0; j < 5; ++j)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int g = 0; g < QG; ++g)
        accl[m][q0 + g] = mfma_bf16(av[PA[j]][m], bv[PB[j]][q0 + g], accl[m][q0 + g]);
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int g = 0; g < QG; ++g)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[m][q0 + g][r] = acc[m][q0 + g][r] + hi[m][g][r];
}

template <int MT, int NT, int QG>
__device__ __forceinline__ void x6_block_c(f32x4 (&acc)[MT][NT], f32x4 (&accl)[MT][NT],
                                           const bf16x8 (&av)[3][MT], const bf16x8 (&bv)[3][NT]) {
  static_assert(NT % QG == 0, "whole fragment groups");
#pragma unroll
  for (int q0 = 0; q0 < NT; q0 += QG) x6_group_c<MT, NT, QG>(acc, accl, av, bv, q0);
}

// acc += accl (the carried corrections), once before the epilogue
template <int MT, int NT>
__device__ __forceinline__ void x6_fold(f32x4 (&acc)[MT][NT], const f32x4 (&accl)[MT][NT]) {
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < NT; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[m][q][r] = acc[m][q][r] + accl[m][q][r];
}

}  // namespace dn
