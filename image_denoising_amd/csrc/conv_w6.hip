// bf16x6 3x3 convolution through the 1-D Winograd transform F(2,3) along x (k_c3w6): the
// 96-output-channel forward / data-gradient shapes of the N2N step with 2/3 of the MFMAs.
//
// Along x, two outputs of a kernel row are y0 = d0 g0 + d1 g1 + d2 g2 and y1 = d1 g0 + d2 g1 +
// d3 g2 (d = four consecutive inputs of a tile of two output pixels, g = the row's three taps).
// F(2,3) computes them from four products of transformed operands,
//   v = (d0 - d2, d1 + d2, d2 - d1, d1 - d3),   u = (g0, (g0 + g1 + g2) / 2, (g0 - g1 + g2) / 2, g2),
//   m_p = v_p u_p,   y0 = m0 + m1 + m2,   y1 = m1 - m2 - m3,
// so a tile row costs 3 kernel rows x 4 positions = 12 products per two output pixels instead of
// 18 (every product here a 32-channel dot product on the matrix cores).  The four positions are
// four independent GEMMs over (input channel, kernel row): M = tiles, N = output channels,
// K = 32 channels x 3 rows; y is formed in registers after the last K chunk.
// Arithmetic: v (fp32 adds) and u (rounded once from fp64 by the packer) are split exactly into
// three bf16 pieces and multiplied as in the bf16x6 kernels (six piece products, fp32 sums), so
// each m_p has the accuracy of an fp32 dot product; the transforms add one rounding of v and u
// (measured against fp64 in tests/test_gpu_x6.py like the direct kernels).
//
//   Workgroup = 4 waves, two workgroups per CU, tile = 8 rows x 16 pixels (8 Winograd tiles per
//   row) x 96 output channels.  Wave (nh, ph) = (w & 1, w >> 1): all 8 tile rows (four M
//   fragments of 16 Winograd tiles = two rows each) x output channels 48nh .. +47 (three N
//   fragments) x positions 2ph, 2ph+1.  Per K chunk a wave runs 6 stages (kernel row ky,
//   position p) of 4 x 3 fragments x 6 products = 72 MFMAs.
//   * Per chunk the workgroup first builds the transformed x tile V (10 input rows x 8 tiles x 4
//     positions x 32 channels, three bf16 planes, 60 KiB) straight from global loads, between two
//     barriers; the other workgroup on the CU keeps the matrix cores busy meanwhile.
//   * Weights come straight from the pre-split image (k_pack_batch PK_W6) into registers: each
//     N fragment of the next stage is requested right after its last use in this one.
//   * After the last chunk the two position halves exchange partial output sums through LDS.
#include <cstdlib>
#include <string>
#include <type_traits>

#include "conv_epi.h"
#include "x6_core.h"

namespace dn {

// NO = 96 output channels: wave (nh, ph) = output channels 48nh .. +47 x all 4 M fragments x
// positions 2ph, 2ph + 1.  NO = 48 (the encoder's 48 -> 48 convs, the 96 -> 144 data gradient's
// 48-channel blocks): wave p = all 48 output channels x all 4 M fragments x position p (P1: each
// weight fragment feeds four MFMA groups; the four positions' partial sums meet in LDS after the
// last chunk; 48->48 @256^2 0.99-1.01 -> 0.96 ms, @128^2 data gradient 0.248 -> 0.240 ms,
// profiles/r5_w48p1_ab.log).  The four-channel tail mode keeps the two-position form (wave (mh,
// ph) = M fragments 2mh, 2mh + 1 x positions 2ph, 2ph + 1); DN_W6_48P1 = 0 selects it throughout.
#ifndef DN_W6_48P1
#define DN_W6_48P1 1
#endif
template <int NO = 96, bool P1_ = false>
struct WCfg {
  static constexpr bool P1 = NO == 48 && P1_;
  static constexpr int WAVES = 4, MT = NO == 96 || P1 ? 4 : 2, NTW = 3, NP = NO, NPOS = 4, NJ = 8;
  static constexpr int NPW = P1 ? 1 : 2;               // positions per wave
  static constexpr int HF = P1 ? 1 : MT / 2;           // M fragments a wave keeps after the exchange
  static constexpr int TW = 16, TH = 8, IH = TH + 2, IW = TW + 2, KC = 32;
  static constexpr int SPC = 12;                       // weight stages per full chunk (ky, p)
  static constexpr int VPL = IH * 4 * NJ * NPOS * 8;   // bf16 per plane of V (quads of 8)
  static constexpr int VBYTES = 3 * VPL * 2;
  static constexpr int WPL = NP * KC;
  static constexpr int WSTP = x6_wst(NP);
  static constexpr int VITEMS = (IH * NJ * 8 + WAVES * 64 - 1) / (WAVES * 64);  // transform items
  static constexpr int PS = 16 * NTW + 4;
  static constexpr int XCH = P1 ? WAVES * MT * NTW * 4 * 64       // floats of the exchange area
                                : WAVES * HF * NTW * 2 * 4 * 64;
  static constexpr int LEND = (XCH + WAVES * 16 * PS) * 4;  // exchange + epilogue staging (over V)
  static constexpr int LBYTES = VBYTES > LEND ? VBYTES : LEND;
  static_assert(2 * LBYTES <= 163840, "two workgroups per CU");
  static_assert(NO == 96 || NO == 48, "96 or 48 output channels");
};

// 16-B quad index of V element (row, kq, j, p): p is XOR-swizzled by row & 1 and the bit-reversed
// kq, so that every ds_read_b128 lane group of the stage reads (lanes {0-3, 12-15, 20-27}, ...:
// two tile rows, two kq, four tiles each) and every 16-lane group of the transform's 8-B writes
// (one row, two tiles, four kq x two halves) falls on distinct banks.  Found by a brute-force search
// over XOR swizzles in the bits of j, row and a permutation of kq against gfx950's LDS lane groups
// (MI355X_MICROARCH.md); the round-3 swizzle p ^ (j >> 2) ^ ((row & 1) << 1) ^ kq left the reads
// 2-way (SQ_LDS_BANK_CONFLICT 37 % of the LDS-active cycles of k_c3w6<1>, profiles/r4_pmc_sq_n2n.txt).
__device__ __forceinline__ int w6_vq(int row, int kq, int j, int p) {
  return ((row * 4 + kq) * 8 + j) * 4 + (p ^ (row & 1) ^ (((kq & 1) << 1) | (kq >> 1)));
}

// 8-B slot of V element (row, j, p) of a tail-mode-1 chunk (<= 4 channels: one bf16x4 per
// plane): p XOR-swizzled by row & 3, so the transform's 16-lane writes (two rows x 8 tiles) and
// the stage's 8-B reads (a half-wave: four rows x 8 tiles) fall on distinct banks.  (In the
// quad layout above these were 2- and 4-way conflicts: k_c3w6<1> 24 % of its LDS-active cycles
// against 7 % for the kernels without this chunk.)
__device__ __forceinline__ int w6_vt(int row, int j, int p) {
  return (row * 8 + j) * 4 + (p ^ (row & 3));
}

// transform item e -> (channel quad c4, Winograd tile j, input row).  C4 = 4 (the 16-channel
// tail chunk): a 16-lane group of the 8-B V writes covers two rows x two tiles x four quads
// (c4 = e & 3, j = 2 (e >> 4 & 3) + (e >> 2 & 1), row = 2 (e >> 6) + (e >> 3 & 1)), so the row
// bit of w6_vq's swizzle separates what the tile pairs j, j + 2 of one row put on the same banks
// (the one-row order c4 + 4 j was 2-way); otherwise c4 fastest, then j, then row.
template <int C4>
__device__ __forceinline__ void w6_item(int e, int& c4, int& j, int& row) {
  if constexpr (C4 == 4) {
    c4 = e & 3;
    j = 2 * ((e >> 4) & 3) + ((e >> 2) & 1);
    row = 2 * (e >> 6) + ((e >> 3) & 1);
  } else {
    c4 = e % C4; j = (e / C4) & 7; row = e / (8 * C4);
  }
}

__device__ __forceinline__ void w6_barrier() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// diagnostic ablations (wrong results, timing only; tools/probes/r5_w6abl.sh): NOT = V built for
// the first chunk only, NOW = no weight loads in the stage loop
#ifndef DN_W6_ABL_NOT
#define DN_W6_ABL_NOT 0
#endif
#ifndef DN_W6_ABL_NOW
#define DN_W6_ABL_NOW 0
#endif
constexpr int W6_TG = 3;  // transform items whose x loads are in flight together

template <int I0, int N, class F>
__device__ __forceinline__ void w6_for(F&& f) {
  if constexpr (I0 < N) {
    f(std::integral_constant<int, I0>{});
    w6_for<I0 + 1, N>(f);
  }
}

// TAIL (x6_tail_mode of K) packs the last chunk's channels: 1 (<= 4 channels): one stage per
// position, k = 4 ky + channel in each K half, the products paired as in mode 4 below; 2 (<= 16 channels): two stages per position, k = 16 (ky - 2s) +
// channel for s = 0; s = 1 holds kernel row 2 alone, its six products in three MFMAs (stage mode
// 4): k < 16 pairs v's (h, h, h) with u's (h, m, l), k >= 16 the same channels' (m, l, m) with
// (h, h, m), so the three sums are hh + mh, hm + lh, hl + mm.  Full chunks: stage 4 ky + p,
// k = channel.
// TAIL 3 (X6_T1: the last chunk has ONE live channel, dec_conv1a's image channel at C = 1, read
// from the compact network input a.in_t1 rather than the concat buffer): one
// stage per position whose single MFMA per fragment pair holds all six split products of the
// three kernel rows, k = 8 ky + slot, slot = (h,h) (h,m) (m,h) (h,l) (l,h) (m,m) of (v, u):
// lane group ky reads its row's (h, m, l) of v as one 8-B slot, the packer lays u's pieces out
// in slot order (pk_w6).  1 MFMA instead of 6, summed from zero and added to the running sum
// as the other blocks' hi + lo.
template <int TAIL, int NO = 96>
__global__ __launch_bounds__(256, 2) void k_c3w6(FwdArgs a) {
  using C = WCfg<NO, NO == 48 && DN_W6_48P1 && TAIL != 1>;
  constexpr int MT = C::MT, NTW = C::NTW, HF = C::HF, NPW = C::NPW;
  constexpr bool P1 = C::P1;
  static_assert(!P1 || TAIL == 0 || TAIL == 2, "one position per wave: tail modes 0 and 2");
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[C::LBYTES];
  __bf16* lv = reinterpret_cast<__bf16*>(lds_raw);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lg = lane >> 4;
  const int nh = NO == 96 ? wave & 1 : 0, ph = P1 ? 0 : wave >> 1;
  const int mb = NO == 96 || P1 ? 0 : 2 * (wave & 1);  // the wave's first M fragment
  const int tiles_x = (a.OW + C::TW - 1) / C::TW;
  int bxr, byr;
  xcd_tile(bxr, byr);
  const int ty0 = (bxr / tiles_x) * C::TH, tx0 = (bxr % tiles_x) * C::TW, n = byr;
  const int iy0 = ty0 - 1, ix0 = tx0 - 1;
  const float* inb = a.in + (long)n * a.IHt * a.IWt * a.in_stride + a.in_off;
  const int nch = (a.K + C::KC - 1) / C::KC;

  // acc[pi][f][q]: position 2ph + pi (P1: position wave), M fragment f, N fragment q
  f32x4 acc[NPW][MT][NTW];
#pragma unroll
  for (int pi = 0; pi < NPW; ++pi)
#pragma unroll
    for (int f = 0; f < MT; ++f)
#pragma unroll
      for (int q = 0; q < NTW; ++q) acc[pi][f][q] = f32x4{0.f, 0.f, 0.f, 0.f};

  // x rows of the tile through a 32-bit buffer resource (out-of-range offsets read zeros)
  const int ry0 = iy0 > 0 ? iy0 : 0, ry1 = iy0 + C::IH < a.IHt ? iy0 + C::IH : a.IHt;
  const long row_floats = (long)a.IWt * a.in_stride;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(inb + ry0 * row_floats), (short)0, (int)((ry1 - ry0) * row_floats * 4),
      0x00020000);
  // (TAIL 3: the tail channel's compact image rows, a.in_t1)
  const __amdgpu_buffer_rsrc_t trs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(TAIL == 3 ? a.in_t1 + ((long)n * a.IHt + ry0) * a.IWt : a.in), (short)0,
      TAIL == 3 ? (int)((ry1 - ry0) * (long)a.IWt * 4) : 0, 0x00020000);
  // chunk k0's V: item (row, j, c4) = channels 4c4 .. 4c4+3 of Winograd tile j of input row row,
  // from the four input pixels 2j .. 2j+3 of the halo tile (loaded for all of a thread's items
  // first, so their latencies overlap)
  // (C4: channel quads transformed -- 8 for a full chunk, the ones a tail stage reads for the
  // tail chunk: 1 for mode 1, 4 for mode 2)
  auto transform = [&](auto c4tag, int k0, int tid) {
    constexpr int C4 = decltype(c4tag)::value, NIT = C::IH * C::NJ * C4;
    constexpr int VIT = (NIT + C::WAVES * 64 - 1) / (C::WAVES * 64);
#pragma unroll
    for (int ig = 0; ig < VIT; ig += W6_TG) {
    f32x4 d[C::VITEMS][4];
#pragma unroll
    for (int it = ig; it < ig + W6_TG && it < VIT; ++it) {
      const int e = tid + it * C::WAVES * 64;
      int c4, j, row;
      w6_item<C4>(e, c4, j, row);
      const int gy = iy0 + row, k = k0 + 4 * c4;
      const bool rok = e < NIT && gy >= 0 && gy < a.IHt && k < a.K;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int gx = ix0 + 2 * j + i;
        const bool ok = rok && gx >= 0 && gx < a.IWt;
        if constexpr (TAIL == 3 && C4 == 1) {  // the one live channel from the compact image
          const int off = ok ? ((gy - ry0) * a.IWt + gx) * 4 : 0x7fffffff;
          d[it][i] = f32x4{__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(trs, off, 0, 0)),
                           0.f, 0.f, 0.f};
          continue;
        }
        const int off = ok ? (((gy - ry0) * a.IWt + gx) * a.in_stride + k) * 4 : 0x7fffffff;
        d[it][i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
      }
    }
#pragma unroll
    for (int it = ig; it < ig + W6_TG && it < VIT; ++it) {
      const int e = tid + it * C::WAVES * 64;
      if (e < NIT) {
        int c4, j, row;
        w6_item<C4>(e, c4, j, row);
        f32x4 v[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          v[0][c] = d[it][0][c] - d[it][2][c];
          v[1][c] = d[it][1][c] + d[it][2][c];
          v[2][c] = d[it][2][c] - d[it][1][c];
          v[3][c] = d[it][1][c] - d[it][3][c];
        }
        typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
        if constexpr (TAIL == 3 && C4 == 1) {
          // one live channel: the (h, m, l) of v_p as one 8-B slot of plane 0
#pragma unroll
          for (int p = 0; p < 4; p += 2) {
            unsigned h, m, l;
            split3x2(v[p][0], v[p + 1][0], h, m, l);
            *reinterpret_cast<u32x2_t*>(lv + w6_vt(row, j, p) * 4) =
                u32x2_t{(h & 0xffffu) | (m << 16), l & 0xffffu};
            *reinterpret_cast<u32x2_t*>(lv + w6_vt(row, j, p + 1) * 4) =
                u32x2_t{(h >> 16) | (m & 0xffff0000u), l >> 16};
          }
          continue;
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          unsigned h0, m0, l0, h1, m1, l1;
          split3x2(v[p][0], v[p][1], h0, m0, l0);
          split3x2(v[p][2], v[p][3], h1, m1, l1);
          // bf16 index in a plane (tail mode 1: the 8-B slot layout w6_vt)
          const int o = C4 == 1 ? w6_vt(row, j, p) * 4 : w6_vq(row, c4 >> 1, j, p) * 8 + (c4 & 1) * 4;
          *reinterpret_cast<u32x2_t*>(lv + o) = u32x2_t{h0, h1};
          *reinterpret_cast<u32x2_t*>(lv + C::VPL + o) = u32x2_t{m0, m1};
          *reinterpret_cast<u32x2_t*>(lv + 2 * C::VPL + o) = u32x2_t{l0, l1};
        }
      }
    }
    }
  };

  // weights: fragment q = output channels 48nh + 16q .. +15 of stage st, plane pl
  // (output-channel block z = blockIdx.z of 96 channels when a.zc: its own image, a.wp_z bf16)
  const int nst_img = nch * C::SPC;
  const __bf16* wimg = reinterpret_cast<const __bf16*>(a.wp) + (long)blockIdx.z * a.wp_z;
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__bf16*>(wimg), (short)0, nst_img * C::WSTP * 2, 0x00020000);
  int woff[NTW];
#pragma unroll
  for (int q = 0; q < NTW; ++q) {
    const int row = (NTW * nh + q) * 16 + li;
    woff[q] = (row * C::KC + x6_swz(row, lg) * 8) * 2;
  }
  bf16x8 w[3][NTW];
  auto load_wq = [&](int st, int q) {
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
      w[pl][q] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, (st * C::WSTP + pl * C::WPL) * 2 + woff[q], 0, 0));
  };

  // stage list of this wave for chunk c (image stage index); tail chunks per TAIL
  auto stage_of = [&](int c, int s, bool tailc) -> int {
    if (P1) return tailc ? c * C::SPC + 2 * wave + s : c * C::SPC + 4 * s + wave;  // s = half / ky
    if (!tailc) return c * C::SPC + (s >> 1) * 4 + 2 * ph + (s & 1);  // s = 2 ky + pi
    if (TAIL == 1 || TAIL == 3) return c * C::SPC + 2 * ph + s;       // s = pi
    return c * C::SPC + 2 * (2 * ph + (s >> 1)) + (s & 1);             // s = 2 pi + half
  };

  // one stage: A fragments of the 4 M fragments (three planes each) read from V, then per N
  // fragment q: 2 x 2 M fragments x 6 products, its adds pinned, and the next stage's fragment q
  // requested into the registers it frees
  auto stage = [&](auto mode_tag, int s, int nxt, int liv, int lgv) {
    constexpr int MODE = decltype(mode_tag)::value;  // 0 full, 1 / 2 / 3 / 4 tail
    int pi, ky0;
    if (P1) { pi = 0; ky0 = MODE == 0 ? s : 2 * (s & 1); }
    else if (MODE == 0) { pi = s & 1; ky0 = s >> 1; }
    else if (MODE == 1 || MODE == 3) { pi = s; ky0 = 0; }
    else { pi = s >> 1; ky0 = 2 * (s & 1); }
    const int p = P1 ? wave : 2 * ph + pi;
    bf16x8 av[3][MT];  // (mode 4: av[0] = A of the (h | m) halves, av[1] = A of (h | l))
#pragma unroll
    for (int f = 0; f < MT; ++f) {
      const int row0 = 2 * (mb + f) + (liv >> 3), j = liv & 7;
      if constexpr (MODE == 0) {
        const int o = w6_vq(row0 + ky0, lgv, j, p) * 8;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) av[pl][f] = *reinterpret_cast<const bf16x8*>(lv + pl * C::VPL + o);
      } else if constexpr (MODE == 4) {
        // kernel row 2 of a tail-2 chunk: lane groups 0, 1 read channels 0..15 from plane h,
        // groups 2, 3 the same channels from plane m (av[0]) and plane l (av[1])
        const int o = w6_vq(row0 + 2, lgv & 1, j, p) * 8, up = lgv >> 1;
        av[0][f] = *reinterpret_cast<const bf16x8*>(lv + up * C::VPL + o);
        av[1][f] = *reinterpret_cast<const bf16x8*>(lv + 2 * up * C::VPL + o);
      } else if constexpr (MODE == 3) {
        // lane group ky: (h, m, l, 0) of kernel row ky -> A slots (h, h, m, h, l, m, 0, 0)
        const int ky = lgv;
        const bf16x4 q4 = *reinterpret_cast<const bf16x4*>(lv + w6_vt(row0 + (ky < 3 ? ky : 0), j, p) * 4);
        const bf16x8 z8 = {};
        const bf16x8 v8 = __builtin_shufflevector(q4, q4, 0, 0, 1, 0, 2, 1, 3, 3);
        av[0][f] = ky > 2 ? z8 : v8;
      } else if constexpr (MODE == 1) {
        // lane groups 0 / 2: channels 0..3 of ky 0 and 1; 1 / 3: ky 2 and zeros; groups 0, 1
        // from plane h, groups 2, 3 from plane m (av[0]) and plane l (av[1]) (the paired
        // products of stage mode 4)
        const int ka = 2 * (lgv & 1), kb = ka + 1, up = lgv >> 1;
        const int oa = w6_vt(row0 + ka, j, p) * 4;
        const int ob = w6_vt(row0 + (kb < 3 ? kb : 0), j, p) * 4;
        const bf16x4 z4 = {(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int pl = (1 + i) * up;
          const bf16x4 va = *reinterpret_cast<const bf16x4*>(lv + pl * C::VPL + oa);
          bf16x4 vb = *reinterpret_cast<const bf16x4*>(lv + pl * C::VPL + ob);
          if (kb > 2) vb = z4;
          av[i][f] = __builtin_shufflevector(va, vb, 0, 1, 2, 3, 4, 5, 6, 7);
        }
      } else {
        // lane groups 0, 1: channels 0..15 of ky0 (quads 0, 1); 2, 3: those of ky0 + 1
        const int ky = ky0 + (lgv >> 1);
        const int o = w6_vq(row0 + (ky < 3 ? ky : 0), lgv & 1, j, p) * 8;
        const bf16x8 z8 = {};
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(lv + pl * C::VPL + o);
          av[pl][f] = ky > 2 ? z8 : v;
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    auto run = [&](auto pic) {
      constexpr int PI = decltype(pic)::value;
#pragma unroll
      for (int q = 0; q < NTW; ++q) {
#pragma unroll
        for (int mp = 0; mp < MT; ++mp) {  // one M fragment per MFMA group
          if constexpr (MODE == 3) {
            const f32x4 t = mfma_bf16(av[0][mp], w[0][q], f32x4{0.f, 0.f, 0.f, 0.f});
            acc[PI][mp][q] = acc[PI][mp][q] + t;
            continue;
          }
          if constexpr (MODE == 4 || MODE == 1) {  // (hl + mm) + (hm + lh) from zero, then hh + mh
            const f32x4 z = {0.f, 0.f, 0.f, 0.f};
            f32x4 lo = mfma_bf16(av[0][mp], w[2][q], z);
            lo = mfma_bf16(av[1][mp], w[1][q], lo);
            const f32x4 hi = mfma_bf16(av[0][mp], w[0][q], z);
            x6_acc_add(acc[PI][mp][q], hi, lo);
            asm volatile("" : "+v"(acc[PI][mp][q]));
            __builtin_amdgcn_sched_barrier(0);
            continue;
          }
          f32x4(&ah)[1][NTW] = *reinterpret_cast<f32x4(*)[1][NTW]>(&acc[PI][mp]);
          bf16x8 a2[3][1];
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) a2[pl][0] = av[pl][mp];
          x6_group<1, NTW, 1>(ah, a2, w, q);
          asm volatile("" : "+v"(ah[0][q]));
          __builtin_amdgcn_sched_barrier(0);
        }
        if (nxt >= 0 && !DN_W6_ABL_NOW) load_wq(nxt, q);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    if constexpr (P1) run(std::integral_constant<int, 0>{});
    else if (pi == 0) run(std::integral_constant<int, 0>{});
    else run(std::integral_constant<int, 1>{});
  };

  // first stage's weights; then per chunk: V built between two barriers, then its stages
  const bool tail_only = TAIL && nch == 1;
#pragma unroll
  for (int q = 0; q < NTW; ++q) load_wq(stage_of(0, 0, tail_only), q);
  const int nfull = TAIL ? nch - 1 : nch;  // full chunks; a tail-packed last one after the loop
#pragma unroll 1
  for (int c = 0; c < nfull; ++c) {
    int liv = li, lgv = lg, tidv = tid;
    asm volatile("" : "+v"(liv), "+v"(lgv), "+v"(tidv));
    const bool more = c + 1 < nch;
    const bool next_tail = TAIL && c + 2 == nch;
    if (c > 0) w6_barrier();  // every wave is done with the previous chunk's V
    if (!DN_W6_ABL_NOT || c == 0) transform(std::integral_constant<int, 8>{}, c * C::KC, tidv);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own V stores done
    w6_barrier();
    constexpr int NSF = P1 ? 3 : 6;  // stages of a full chunk per wave
    w6_for<0, NSF>([&](auto si) {
      constexpr int s = decltype(si)::value;
      const int nxt = s + 1 < NSF ? stage_of(c, s + 1, false) : (more ? stage_of(c + 1, 0, next_tail) : -1);
      stage(std::integral_constant<int, 0>{}, s, nxt, liv, lgv);
    });
  }
  if constexpr (TAIL != 0) {
    const int c = nch - 1;
    int liv = li, lgv = lg, tidv = tid;
    asm volatile("" : "+v"(liv), "+v"(lgv), "+v"(tidv));
    if (c > 0) w6_barrier();
    transform(std::integral_constant<int, TAIL == 2 ? 4 : 1>{}, c * C::KC, tidv);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    w6_barrier();
    constexpr int NS = TAIL == 2 ? (P1 ? 2 : 4) : 2;
    using MD = std::integral_constant<int, TAIL>;
    w6_for<0, NS>([&](auto si) {
      constexpr int s = decltype(si)::value;
      const int nxt = s + 1 < NS ? stage_of(c, s + 1, true) : -1;
      if constexpr (TAIL == 2 && (s & 1)) stage(std::integral_constant<int, 4>{}, s, nxt, liv, lgv);
      else stage(MD{}, s, nxt, liv, lgv);
    });
  }

  f32x4 y[HF][2][NTW];  // [kept fragment][output parity][q]
  if constexpr (P1) {
    // one position per wave: every wave's m_p of all four M fragments into LDS, then wave w
    // forms M fragment w from the four: y0 = (m0 + m1) + m2, y1 = m1 + (-m2 - m3) (the order of
    // the two-position form below)
    __builtin_amdgcn_s_waitcnt(0xC07F);
    w6_barrier();  // every wave is done with V: it becomes the exchange area
    float* xa = reinterpret_cast<float*>(lds_raw);
#pragma unroll
    for (int f = 0; f < MT; ++f)
#pragma unroll
      for (int q = 0; q < NTW; ++q)
        *reinterpret_cast<f32x4*>(xa + (((wave * MT + f) * NTW + q) * 64 + lane) * 4) = acc[0][f][q];
    __builtin_amdgcn_s_waitcnt(0xC07F);
    w6_barrier();
#pragma unroll
    for (int q = 0; q < NTW; ++q) {
      f32x4 m[4];
#pragma unroll
      for (int pp = 0; pp < 4; ++pp)
        m[pp] = *reinterpret_cast<const f32x4*>(xa + (((pp * MT + wave) * NTW + q) * 64 + lane) * 4);
      y[0][0][q] = (m[0] + m[1]) + m[2];
      y[0][1][q] = m[1] + (-m[2] - m[3]);
    }
  } else {
  // output transform: ph 0 holds m0, m1, ph 1 holds m2, m3.  Partial sums per tile:
  //   ph 0: (y0, y1) += (m0 + m1, m1);   ph 1: (y0, y1) += (m2, -m2 - m3)
  // wave ph keeps HF of its MT M fragments (96: 2ph, 2ph+1 = tile rows 4ph .. 4ph+3; 48: its
  // fragment mb + ph) and hands the other HF's partials to its partner (wave ^ 2) through LDS
  __builtin_amdgcn_s_waitcnt(0xC07F);
  w6_barrier();  // every wave is done with V: it becomes the exchange area
  {
    float* xo = reinterpret_cast<float*>(lds_raw) + (wave * HF * NTW * 2) * 4 * 64;  // mine, out
    const int pw = wave ^ 2;                                                         // partner
    const float* xi = reinterpret_cast<const float*>(lds_raw) + (pw * HF * NTW * 2) * 4 * 64;
    // compile-time fragment indices per position half (a run-time index would put acc in memory)
    auto part = [&](auto phc) {
      constexpr int PH = decltype(phc)::value;
#pragma unroll
      for (int ff = 0; ff < HF; ++ff)
#pragma unroll
        for (int q = 0; q < NTW; ++q) {
          constexpr int FO = HF * (1 - PH), FK = HF * PH;  // the partner's fragments, mine
          f32x4 o0, o1, k0, k1;
          if constexpr (PH == 0) {
            o0 = acc[0][FO + ff][q] + acc[1][FO + ff][q]; o1 = acc[1][FO + ff][q];
            k0 = acc[0][FK + ff][q] + acc[1][FK + ff][q]; k1 = acc[1][FK + ff][q];
          } else {
            o0 = acc[0][FO + ff][q]; o1 = -acc[0][FO + ff][q] - acc[1][FO + ff][q];
            k0 = acc[0][FK + ff][q]; k1 = -acc[0][FK + ff][q] - acc[1][FK + ff][q];
          }
          *reinterpret_cast<f32x4*>(xo + ((ff * NTW + q) * 2 + 0) * 256 + lane * 4) = o0;
          *reinterpret_cast<f32x4*>(xo + ((ff * NTW + q) * 2 + 1) * 256 + lane * 4) = o1;
          y[ff][0][q] = k0;
          y[ff][1][q] = k1;
        }
    };
    if (ph == 0) part(std::integral_constant<int, 0>{});
    else part(std::integral_constant<int, 1>{});
    __builtin_amdgcn_s_waitcnt(0xC07F);
    w6_barrier();
#pragma unroll
    for (int ff = 0; ff < HF; ++ff)
#pragma unroll
      for (int q = 0; q < NTW; ++q) {
        // y0 = (m0 + m1) + m2, y1 = m1 + (-m2 - m3): ph 0's part first in both
        const f32x4 i0 = *reinterpret_cast<const f32x4*>(xi + ((ff * NTW + q) * 2 + 0) * 256 + lane * 4);
        const f32x4 i1 = *reinterpret_cast<const f32x4*>(xi + ((ff * NTW + q) * 2 + 1) * 256 + lane * 4);
        if (ph == 0) { y[ff][0][q] = y[ff][0][q] + i0; y[ff][1][q] = y[ff][1][q] + i1; }
        else { y[ff][0][q] = i0 + y[ff][0][q]; y[ff][1][q] = i1 + y[ff][1][q]; }
      }
  }
  }
  // epilogue: this wave's 2 HF tile rows wrow + r (kept fragment r/2, half r%2), channels
  // 48nh .. +47; the fragment's lane (li, lg) holds tiles 4lg .. 4lg+3 of the fragment's 16,
  // i.e. row half lg >> 1, tiles 4 (lg & 1) + e -> pixels 2 (4 (lg & 1) + e) + parity
  float* st = reinterpret_cast<float*>(lds_raw) + C::XCH + wave * 16 * C::PS;
  f32x4 outr[2 * HF][NTW];  // rows as the vec epilogue's acc: pixel 4lg' + r of row m
  // stage each row through LDS in the C/D map the epilogue expects: write the row's 16 pixels
  // x 48 channels, read back as acc-layout registers
#pragma unroll
  for (int r4 = 0; r4 < 2 * HF; ++r4) {
    const int ff = r4 >> 1, hf = r4 & 1;
    if ((lg >> 1) == hf) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int t = 4 * (lg & 1) + e;
#pragma unroll
        for (int q = 0; q < NTW; ++q) {
          st[(2 * t) * C::PS + 16 * q + li] = y[ff][0][q][e];
          st[(2 * t + 1) * C::PS + 16 * q + li] = y[ff][1][q][e];
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll
    for (int q = 0; q < NTW; ++q)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) outr[r4][q][rr] = st[(4 * lg + rr) * C::PS + 16 * q + li];
    __builtin_amdgcn_s_waitcnt(0xC07F);
  }
  {
    const int cz = (a.zc ? (int)blockIdx.z * a.zc : 0) + nh * 16 * NTW;
    const int nout = a.NOUT - cz < 16 * NTW ? a.NOUT - cz : 16 * NTW;
    const int wrow = P1 ? 2 * wave : 2 * (mb + HF * ph);  // (even: a fused 2x2 pool sees whole windows)
    if (nout > 0) fwd_epilogue_at<NTW, 2 * HF, C::PS>(a, outr, st, ty0, tx0, n, wrow, cz, nout);
  }
}

// ------------------------------------------------------------------------------------
// The N2N no-grad pass's dec_conv1b at the pair pixels only, on the Winograd transform
// (k_c3w6s).  train.py:151-154's pair table makes every cell's two pixels an aligned F(2,3)
// tile: horizontal neighbours (rd 0, 3, 4, 7: row 2ci + r, columns 2cj, 2cj + 1) are a tile along
// x, vertical ones (rd 1, 2, 5, 6: rows 2ci, 2ci + 1 of column 2cj + c) a tile along y.  The cells
// are listed per orientation (k_w6s_lists, raster order), and a workgroup takes 64 consecutive
// cells of one list: M = those cells, N = 96 output channels, K = 32 input channels x the three
// rows (x tiles) or columns (y tiles) of the kernel, four positions p: 12 instead of 18 products
// per cell and input chunk.  Each cell's V (its four input pixels along the tile, for one kernel
// row k3) is gathered straight from global memory (no halo sharing: cells are not adjacent in a
// list), transformed, split into three bf16 planes in LDS, between two barriers per (chunk, k3)
// phase; the other workgroup on the CU keeps the matrix cores busy meanwhile.  Weights: the
// layer's PK_W6 image (u along kx for each ky) for x tiles, the same with the taps transposed
// (u along ky for each kx; WView flip = 2) for y tiles, straight into registers as in k_c3w6.
// Output: the pair image [N][OH/2][OW][96] (column 2cj + s = pixel pair[rd][s] of cell (ci, cj)),
// bias + LeakyReLU, as k_c3x6s writes it for the head.
// ------------------------------------------------------------------------------------
struct SCfgW {
  static constexpr int WAVES = 4, MT = 4, NTW = 3, NP = 96, CELLS = 64, KC = 32;
  static constexpr int VPL = 4 * CELLS * KC;        // bf16 per plane of V: [p][cell][32 ch]
  static constexpr int VBYTES = 3 * VPL * 2;        // 48 KiB
  static constexpr int WSTP = x6_wst(NP);
  static constexpr int XCH = WAVES * 2 * NTW * 2 * 4 * 64;  // floats of the exchange area
  // output stage: [cell][pixel s][96 ch], cells 208 floats apart (the four cells a 4-byte write
  // instruction covers land 16 banks apart)
  static constexpr int OCS = 208, OBYTES = CELLS * OCS * 4;
  static constexpr int LB0 = VBYTES > XCH * 4 ? VBYTES : XCH * 4;
  static constexpr int LBYTES = LB0 > OBYTES ? LB0 : OBYTES;
  static_assert(2 * (LBYTES + CELLS * 4) <= 163840, "two workgroups per CU");
};

// list entry: cj | ci << 15 | (r or c) << 30 | swap << 31
__device__ __forceinline__ unsigned w6s_entry(int ci, int cj, int rd) {
  const unsigned rc = (rd == 2 || rd == 3 || rd == 6 || rd == 7) ? 1u : 0u;
  return (unsigned)cj | ((unsigned)ci << 15) | (rc << 30) | ((rd >= 4 ? 1u : 0u) << 31);
}

// per image n: the cells of orientation o (0: x tiles, rd 0/3/4/7; 1: y tiles, rd 1/2/5/6) in
// raster order -> list[(n * 2 + o) * cells + i], their number -> cnt[n * 2 + o]
__global__ __launch_bounds__(1024) void k_w6s_lists(const unsigned char* __restrict__ rd, int ch,
                                                     int cw, unsigned* __restrict__ list,
                                                     int* __restrict__ cnt) {
  __shared__ int part[2][1024];
  const int n = blockIdx.x, tid = threadIdx.x;
  const long cells = (long)ch * cw;
  const unsigned char* r = rd + (long)n * cells;
  unsigned* lo[2] = {list + (long)(2 * n) * cells, list + (long)(2 * n + 1) * cells};
  int base[2] = {0, 0};
  for (long c0 = 0; c0 < cells; c0 += 16L * 1024) {
    // 16 consecutive cells per thread
    int k[2] = {0, 0};
    const long e0 = c0 + 16L * tid;
    for (int j = 0; j < 16; ++j) {
      const long e = e0 + j;
      if (e < cells) {
        const int v = r[e] & 7;
        ++k[(v == 1 || v == 2 || v == 5 || v == 6) ? 1 : 0];
      }
    }
    part[0][tid] = k[0];
    part[1][tid] = k[1];
    __syncthreads();
    // inclusive scan of the two count arrays (Hillis-Steele over 1024 threads)
    for (int d = 1; d < 1024; d <<= 1) {
      const int a0 = tid >= d ? part[0][tid - d] : 0, a1 = tid >= d ? part[1][tid - d] : 0;
      __syncthreads();
      part[0][tid] += a0;
      part[1][tid] += a1;
      __syncthreads();
    }
    int o0 = base[0] + part[0][tid] - k[0], o1 = base[1] + part[1][tid] - k[1];
    for (int j = 0; j < 16; ++j) {
      const long e = e0 + j;
      if (e < cells) {
        const int v = r[e] & 7;
        const int ci = (int)(e / cw), cj = (int)(e - (long)ci * cw);
        const unsigned en = w6s_entry(ci, cj, v);
        if (v == 1 || v == 2 || v == 5 || v == 6) lo[1][o1++] = en;
        else lo[0][o0++] = en;
      }
    }
    base[0] += part[0][1023];
    base[1] += part[1][1023];
    __syncthreads();
  }
  if (tid == 0) {
    cnt[2 * n] = base[0];
    cnt[2 * n + 1] = base[1];
  }
}

// Block order: workgroup b runs on XCD b % 8; XCD x gets a contiguous run of
// the logical order (image, 64-cell chunk, orientation), so the x-tile and y-tile workgroups of
// the same cell rows, and the neighbouring chunks that share their input rows, run on one L2 at
// about the same time (otherwise each input row is fetched from HBM by up to four workgroups
// on different XCDs: 5.25 GB per launch for 1.6 GB of input, profiles/r4_n2n_pmc_step.json).
__device__ __forceinline__ void w6s_block(int nchunk, int& o, int& n, int& chunk) {
  const unsigned b = blockIdx.x, tot = gridDim.x;
  unsigned l = b;
  if (tot >= 8) {
    const unsigned x = b % 8, base = tot / 8, extra = tot % 8;
    l = x * base + (x < extra ? x : extra) + b / 8;  // XCD x: (tot - x + 7) / 8 blocks
  }
  o = (int)(l & 1);
  l >>= 1;
  chunk = (int)(l % (unsigned)nchunk);
  n = (int)(l / (unsigned)nchunk);
}

__global__ __launch_bounds__(256, 2) void k_c3w6s(FwdArgs a, const unsigned* __restrict__ list,
                                                  const int* __restrict__ cnt,
                                                  const __bf16* __restrict__ wpv, int nchunk) {
  using C = SCfgW;
  constexpr int MT = C::MT, NTW = C::NTW;
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[C::LBYTES];
  __shared__ unsigned lent[C::CELLS];
  __bf16* lv = reinterpret_cast<__bf16*>(lds_raw);
  int o, n, chunk;
  w6s_block(nchunk, o, n, chunk);
  const int cbase = chunk * C::CELLS;
  const int ncell = cnt[2 * n + o];
  if (cbase >= ncell) return;  // (uniform: the list is shorter than the grid allows)
  const long cells = (long)(a.OH / 2) * (a.OW / 2);
  const unsigned* lst = list + (long)(2 * n + o) * cells;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lg = lane >> 4;
  const int nh = wave & 1, ph = wave >> 1;
  if (tid < C::CELLS) lent[tid] = cbase + tid < ncell ? lst[cbase + tid] : 0xffffffffu;
  __syncthreads();

  f32x4 acc[2][MT][NTW];
#pragma unroll
  for (int pi = 0; pi < 2; ++pi)
#pragma unroll
    for (int f = 0; f < MT; ++f)
#pragma unroll
      for (int q = 0; q < NTW; ++q) acc[pi][f][q] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the image through a 32-bit buffer resource (host: < 2 GiB), out-of-range offsets read zeros
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.in + (long)n * a.IHt * a.IWt * a.in_stride + a.in_off), (short)0,
      (int)((long)a.IHt * a.IWt * a.in_stride * 4), 0x00020000);
  // transform items: (cell, channel quad c4) = tid + 256 it -> cells tid >> 3 and +32, quad tid & 7
  const int c4 = tid & 7;
  unsigned ent[2];
#pragma unroll
  for (int it = 0; it < 2; ++it) ent[it] = lent[(tid >> 3) + 32 * it];
  // tload: the phase's input pixels into d (tload_phase), twrite: V from them
  f32x4 d[2][4];
  auto tload = [&](int k0, int k3) {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const unsigned e = ent[it];
      const bool live = e != 0xffffffffu;
      const int cj = e & 0x7fff, ci = (e >> 15) & 0x7fff, rc = (e >> 30) & 1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // x tiles: row 2ci + r + k3 - 1, column 2cj - 1 + i; y tiles: row 2ci - 1 + i, column
        // 2cj + c + k3 - 1
        const int gy = o == 0 ? 2 * ci + rc + k3 - 1 : 2 * ci - 1 + i;
        const int gx = o == 0 ? 2 * cj - 1 + i : 2 * cj + rc + k3 - 1;
        const bool ok = live && gy >= 0 && gy < a.IHt && gx >= 0 && gx < a.IWt;
        const int off = ok ? (((gy * a.IWt + gx) * a.in_stride) + k0 + 4 * c4) * 4 : 0x7fffffff;
        d[it][i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
      }
    }
  };
  auto twrite = [&]() {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int cell = (tid >> 3) + 32 * it;
      f32x4 v[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        v[0][c] = d[it][0][c] - d[it][2][c];
        v[1][c] = d[it][1][c] + d[it][2][c];
        v[2][c] = d[it][2][c] - d[it][1][c];
        v[3][c] = d[it][1][c] - d[it][3][c];
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        unsigned h0, m0, l0, h1, m1, l1;
        split3x2(v[p][0], v[p][1], h0, m0, l0);
        split3x2(v[p][2], v[p][3], h1, m1, l1);
        const int row = p * C::CELLS + cell;
        const int off = row * C::KC + x6_swz(row, c4 >> 1) * 8 + (c4 & 1) * 4;  // bf16 index
        typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
        *reinterpret_cast<u32x2_t*>(lv + off) = u32x2_t{h0, h1};
        *reinterpret_cast<u32x2_t*>(lv + C::VPL + off) = u32x2_t{m0, m1};
        *reinterpret_cast<u32x2_t*>(lv + 2 * C::VPL + off) = u32x2_t{l0, l1};
      }
    }
  };

  // weights: fragment q = output channels 48nh + 16q .. +15 of stage st (= c*12 + k3*4 + p)
  const int nch = a.K / C::KC;
  const __bf16* wimg = o == 0 ? reinterpret_cast<const __bf16*>(a.wp) : wpv;
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__bf16*>(wimg), (short)0, nch * 12 * C::WSTP * 2, 0x00020000);
  int woff[NTW];
#pragma unroll
  for (int q = 0; q < NTW; ++q) {
    const int row = (NTW * nh + q) * 16 + li;
    woff[q] = (row * C::KC + x6_swz(row, lg) * 8) * 2;
  }
  bf16x8 w[3][NTW];
  auto load_wq = [&](int st, int q) {
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
      w[pl][q] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, (st * C::WSTP + pl * 96 * 32) * 2 + woff[q], 0, 0));
  };
  // one stage: position p = 2ph + pi of this phase, its A fragments from V
  auto stage = [&](auto pic, int nxt, int liv, int lgv) {
    constexpr int PI = decltype(pic)::value;
    const int p = 2 * ph + PI;
    bf16x8 av[3][MT];
#pragma unroll
    for (int f = 0; f < MT; ++f) {
      const int row = p * C::CELLS + 16 * f + liv;
      const int off = row * C::KC + x6_swz(row, lgv) * 8;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) av[pl][f] = *reinterpret_cast<const bf16x8*>(lv + pl * C::VPL + off);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < NTW; ++q) {
#pragma unroll
      for (int f = 0; f < MT; ++f) {
        f32x4(&ah)[1][NTW] = *reinterpret_cast<f32x4(*)[1][NTW]>(&acc[PI][f]);
        bf16x8 a2[3][1];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) a2[pl][0] = av[pl][f];
        x6_group<1, NTW, 1>(ah, a2, w, q);
        asm volatile("" : "+v"(ah[0][q]));
        __builtin_amdgcn_sched_barrier(0);
      }
      if (nxt >= 0) load_wq(nxt, q);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
#pragma unroll
  for (int q = 0; q < NTW; ++q) load_wq(2 * ph, q);
  // the next phase's input pixels are requested right after this phase's V is written, so their
  // latency runs under this phase's MFMAs instead of between the two barriers of the next
  // transform (a tile has three phases per input chunk, each with its own gather from L2)
  const int nph = nch * 3;
  tload(0, 0);
#pragma unroll 1
  for (int ph3 = 0; ph3 < nph; ++ph3) {
    const int c = ph3 / 3, k3 = ph3 - 3 * c;
    int liv = li, lgv = lg;
    asm volatile("" : "+v"(liv), "+v"(lgv));
    if (ph3 > 0) w6_barrier();  // every wave is done with the previous phase's V
    twrite();
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own V stores done
    w6_barrier();
    if (ph3 + 1 < nph) {
      const int c1 = (ph3 + 1) / 3;
      tload(c1 * C::KC, ph3 + 1 - 3 * c1);
    }
    const int st0 = ph3 * 4 + 2 * ph;  // c*12 + k3*4 + 2ph
    stage(std::integral_constant<int, 0>{}, st0 + 1, liv, lgv);
    stage(std::integral_constant<int, 1>{}, ph3 + 1 < nph ? st0 + 4 : -1, liv, lgv);
  }

  // output transform (as k_c3w6): ph 0 holds m0, m1, ph 1 holds m2, m3;
  //   ph 0: (y0, y1) += (m0 + m1, m1);   ph 1: (y0, y1) += (m2, -m2 - m3)
  // wave ph keeps M fragments 2ph, 2ph+1 and hands the other two's partials to its partner
  __builtin_amdgcn_s_waitcnt(0xC07F);
  w6_barrier();  // every wave is done with V: it becomes the exchange area
  f32x4 y[2][2][NTW];
  {
    float* xo = reinterpret_cast<float*>(lds_raw) + (wave * 2 * NTW * 2) * 4 * 64;
    const int pw = wave ^ 2;
    const float* xi = reinterpret_cast<const float*>(lds_raw) + (pw * 2 * NTW * 2) * 4 * 64;
    auto part = [&](auto phc) {
      constexpr int PH = decltype(phc)::value;
#pragma unroll
      for (int ff = 0; ff < 2; ++ff)
#pragma unroll
        for (int q = 0; q < NTW; ++q) {
          constexpr int FO = 2 * (1 - PH), FK = 2 * PH;
          f32x4 o0, o1, k0, k1;
          if constexpr (PH == 0) {
            o0 = acc[0][FO + ff][q] + acc[1][FO + ff][q]; o1 = acc[1][FO + ff][q];
            k0 = acc[0][FK + ff][q] + acc[1][FK + ff][q]; k1 = acc[1][FK + ff][q];
          } else {
            o0 = acc[0][FO + ff][q]; o1 = -acc[0][FO + ff][q] - acc[1][FO + ff][q];
            k0 = acc[0][FK + ff][q]; k1 = -acc[0][FK + ff][q] - acc[1][FK + ff][q];
          }
          *reinterpret_cast<f32x4*>(xo + ((ff * NTW + q) * 2 + 0) * 256 + lane * 4) = o0;
          *reinterpret_cast<f32x4*>(xo + ((ff * NTW + q) * 2 + 1) * 256 + lane * 4) = o1;
          y[ff][0][q] = k0;
          y[ff][1][q] = k1;
        }
    };
    if (ph == 0) part(std::integral_constant<int, 0>{});
    else part(std::integral_constant<int, 1>{});
    __builtin_amdgcn_s_waitcnt(0xC07F);
    w6_barrier();
#pragma unroll
    for (int ff = 0; ff < 2; ++ff)
#pragma unroll
      for (int q = 0; q < NTW; ++q) {
        const f32x4 i0 = *reinterpret_cast<const f32x4*>(xi + ((ff * NTW + q) * 2 + 0) * 256 + lane * 4);
        const f32x4 i1 = *reinterpret_cast<const f32x4*>(xi + ((ff * NTW + q) * 2 + 1) * 256 + lane * 4);
        if (ph == 0) { y[ff][0][q] = y[ff][0][q] + i0; y[ff][1][q] = y[ff][1][q] + i1; }
        else { y[ff][0][q] = i0 + y[ff][0][q]; y[ff][1][q] = i1 + y[ff][1][q]; }
      }
  }
  // epilogue: lane (li, lg) of fragment 2ph + ff holds cells 16(2ph + ff) + 4lg + e (e < 4),
  // output channel 48nh + 16q + li; bias + LeakyReLU into the output stage (pixel s = 0 takes
  // pair[rd][0]: y0 unless the entry's swap bit), then every cell's two pixels (columns 2cj,
  // 2cj + 1 of pair-image row ci: 768 contiguous bytes) leave as whole 128-B lines, float4 per
  // lane (per-lane 4-byte stores had the two waves of a pixel write halves of one line at
  // different times)
  __builtin_amdgcn_s_waitcnt(0xC07F);
  w6_barrier();  // every wave has read its partner's partial sums: the area becomes the stage
  float* ost = reinterpret_cast<float*>(lds_raw);
#pragma unroll
  for (int q = 0; q < NTW; ++q) {
    const int ch = 48 * nh + 16 * q + li;
    const float b = a.bias[ch];
#pragma unroll
    for (int ff = 0; ff < 2; ++ff)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int cell = 16 * (2 * ph + ff) + 4 * lg + e;
        const int sw = (int)(lent[cell] >> 31);
        float v0 = y[ff][0][q][e] + b, v1 = y[ff][1][q][e] + b;
        v0 = v0 > 0.f ? v0 : v0 * 0.2f;
        v1 = v1 > 0.f ? v1 : v1 * 0.2f;
        ost[cell * C::OCS + (sw ? 96 : 0) + ch] = v0;
        ost[cell * C::OCS + (sw ? 0 : 96) + ch] = v1;
      }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  w6_barrier();
#pragma unroll
  for (int i = 0; i < C::CELLS * 48 / 256; ++i) {
    const int e = tid + 256 * i, cell = e / 48, w = e - 48 * cell;  // w: float4 of the two pixels
    const unsigned en = lent[cell];
    if (en == 0xffffffffu) continue;
    const int cj = en & 0x7fff, ci = (en >> 15) & 0x7fff;
    const f32x4 v = *reinterpret_cast<const f32x4*>(ost + cell * C::OCS + 4 * w);
    float* dst = a.out + (((long)n * (a.OH / 2) + ci) * a.OW + 2 * cj + (w >= 24)) * a.out_stride + a.out_off +
                 4 * (w >= 24 ? w - 24 : w);
    *reinterpret_cast<f32x4*>(dst) = v;
  }
}

// the cell lists of k_c3w6s for rd [N][OH/2][OW/2]: list (2 * N * cells uint32), cnt (2 * N int)
hipError_t launch_w6s_lists(const unsigned char* rd, int N, int OH, int OW, unsigned* list, int* cnt,
                            hipStream_t s) {
  if (N < 1 || (OH | OW) & 1 || OH / 2 >= 32768 || OW / 2 >= 32768) return hipErrorInvalidValue;
  prof_kernel("k_w6s_lists");
  hipLaunchKernelGGL(k_w6s_lists, dim3(N), dim3(1024), 0, s, rd, OH / 2, OW / 2, list, cnt);
  return hipGetLastError();
}

// dec_conv1b at the pair pixels on the Winograd kernel: a.wp = the layer's PK_W6 image (x tiles),
// wpv = the tap-transposed one (y tiles), list / cnt from launch_w6s_lists on the same rd
hipError_t launch_fwd_w6s(const FwdArgs& a, const unsigned* list, const int* cnt, const void* wpv,
                          hipStream_t s) {
  if (a.NOUT != 96 || a.K % 32 || a.K <= 0 || a.zc || a.epi != EPI_BIAS_ACT || !a.bias ||
      a.out_layout != OUT_NHWC || ((a.in_stride | a.in_off | a.out_stride | a.out_off) & 3) ||
      a.out_stride < 96 || (a.OH | a.OW) & 1 ||
      a.IHt != a.OH || a.IWt != a.OW || (long)a.IHt * a.IWt * a.in_stride * 4 >= 0x7fffffffL ||
      (a.x6_tail & 7) != 0)
    return hipErrorInvalidValue;
  const long cells = (long)(a.OH / 2) * (a.OW / 2);
  const long nchunk = (cells + SCfgW::CELLS - 1) / SCfgW::CELLS;
  if (nchunk * a.N * 2 >= (1L << 31)) return hipErrorInvalidValue;
  const dim3 grid((unsigned)(nchunk * a.N * 2));
  prof_kernel("k_c3w6s");
  hipLaunchKernelGGL(k_c3w6s, grid, dim3(SCfgW::WAVES * 64), 0, s, a, list, cnt,
                     static_cast<const __bf16*>(wpv), (int)nchunk);
  return hipGetLastError();
}

int w6_stages_per_chunk() { return WCfg<96>::SPC; }

// k_c3w6 for a 96- or 48-output-channel forward / data gradient on a PK_W6 image (a.x6_tail &
// X6_W6); a fused 2x2 max-pool (a.pool_out) through the float4 epilogue as the direct kernels
hipError_t launch_fwd_w6(const FwdArgs& a, hipStream_t s) {
  using C = WCfg<96>;  // (tile geometry: both widths)
  const bool aux = a.epi == EPI_MASK || a.epi == EPI_BIAS_ADD;
  const int tail = a.x6_tail & 7;
  const int nz = a.zc ? (a.NOUT + a.zc - 1) / a.zc : 1;
  const int np = a.zc ? a.zc : a.NOUT;
  if ((np != 96 && np != 48) || a.out_layout != OUT_NHWC || a.sel_rd ||
      ((a.out_stride | a.out_off | a.NOUT) & 3) || (aux && ((a.mask_stride | a.mask_off) & 3)) ||
      a.epi < EPI_BIAS || a.epi > EPI_BIAS_ADD || ((a.in_stride | a.in_off | a.K) & 3) ||
      (long)C::IH * a.IWt * a.in_stride * 4 >= 0x7fffffffL || tail != x6_tail_mode(a.K))
    return hipErrorInvalidValue;
  if (a.pool_out && (a.epi != EPI_BIAS_ACT || ((a.pool_stride | a.pool_off) & 3) || ((a.OH | a.OW) & 1)))
    return hipErrorInvalidValue;
  const int tx = (a.OW + C::TW - 1) / C::TW, ty = (a.OH + C::TH - 1) / C::TH;
  const dim3 grid(tx * ty, a.N, nz), block(C::WAVES * 64);
  // X6_T1: a one-channel tail chunk in the six-slot layout (96 outputs only)
  const bool t1 = (a.x6_tail & X6_T1) != 0;
  if (t1 && (tail != 1 || np != 96 || !a.in_t1 || (long)a.IHt * a.IWt * 4 >= 0x7fffffffL))
    return hipErrorInvalidValue;
  static const char* kn[2][4] = {{"k_c3w6<0,96>", "k_c3w6<1,96>", "k_c3w6<2,96>", "k_c3w6<3,96>"},
                                 {"k_c3w6<0,48>", "k_c3w6<1,48>", "k_c3w6<2,48>", ""}};
  prof_kernel(kn[np == 48][t1 ? 3 : tail]);
  if (np == 48) {
    if (tail == 1) hipLaunchKernelGGL((k_c3w6<1, 48>), grid, block, 0, s, a);
    else if (tail == 2) hipLaunchKernelGGL((k_c3w6<2, 48>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((k_c3w6<0, 48>), grid, block, 0, s, a);
  } else {
    if (t1) hipLaunchKernelGGL(k_c3w6<3>, grid, block, 0, s, a);
    else if (tail == 1) hipLaunchKernelGGL(k_c3w6<1>, grid, block, 0, s, a);
    else if (tail == 2) hipLaunchKernelGGL(k_c3w6<2>, grid, block, 0, s, a);
    else hipLaunchKernelGGL(k_c3w6<0>, grid, block, 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace dn
