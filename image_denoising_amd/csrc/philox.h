// Counter-based Philox4x32-10 (Salmon et al., SC'11) for the in-kernel random streams of the
// N2N step.  Replaces train.py:56-61 get_generator() + torch.randint/torch.normal: every
// random value is a pure function of (seed, offset, global index), so results do not depend
// on grid shape or on how the batch is sharded over ranks.  oracle/philox.py restates it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dn {

struct U32x4 { uint32_t v[4]; };

__host__ __device__ inline U32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                               uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)M0 * c0;
    const uint64_t p1 = (uint64_t)M1 * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += W0; k1 += W1;
  }
  U32x4 o;
  o.v[0] = c0; o.v[1] = c1; o.v[2] = c2; o.v[3] = c3;
  return o;
}

// 32-bit word for global index q: block q>>2, word q&3; counter = (blk lo, blk hi, off lo, off hi)
__host__ __device__ inline uint32_t philox_cell_u32(uint64_t seed, uint64_t offset, uint64_t q) {
  const uint64_t blk = q >> 2;
  const U32x4 o = philox4x32_10((uint32_t)blk, (uint32_t)(blk >> 32), (uint32_t)offset,
                                (uint32_t)(offset >> 32), (uint32_t)seed, (uint32_t)(seed >> 32));
  return o.v[q & 3];
}

// standard normal for global element q: Box-Muller on words (2p, 2p+1) of block q>>2,
// p = (q>>1)&1; even q -> cos branch, odd q -> sin branch.
__host__ __device__ inline float philox_normal(uint64_t seed, uint64_t offset, uint64_t q) {
  const uint64_t blk = q >> 2;
  const U32x4 o = philox4x32_10((uint32_t)blk, (uint32_t)(blk >> 32), (uint32_t)offset,
                                (uint32_t)(offset >> 32), (uint32_t)seed, (uint32_t)(seed >> 32));
  const int p = (int)((q >> 1) & 1);
  const uint32_t a = o.v[2 * p], b = o.v[2 * p + 1];
  const float u1 = ((float)(a >> 8) + 1.0f) * (1.0f / 16777216.0f);  // (0, 1]
  const float u2 = (float)(b >> 8) * (1.0f / 16777216.0f);           // [0, 1)
  const float r = sqrtf(-2.0f * logf(u1));
  const float th = 6.283185307179586f * u2;
  return (q & 1) ? r * sinf(th) : r * cosf(th);
}

// uniform double in (0, 1) for global element q: 53 bits from words (2p, 2p+1) of block q>>1,
// p = q & 1 (the Poisson sampler's draw)
__host__ __device__ inline double philox_uniform53(uint64_t seed, uint64_t offset, uint64_t q) {
  const uint64_t blk = q >> 1;
  const U32x4 o = philox4x32_10((uint32_t)blk, (uint32_t)(blk >> 32), (uint32_t)offset,
                                (uint32_t)(offset >> 32), (uint32_t)seed, (uint32_t)(seed >> 32));
  const int p = (int)(q & 1);
  const uint32_t a = o.v[2 * p] >> 5, b = o.v[2 * p + 1] >> 6;  // 27 + 26 bits
  return ((double)a * 67108864.0 + (double)b + 0.5) * (1.0 / 9007199254740992.0);
}

}  // namespace dn
