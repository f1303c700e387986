// ImprovedUNet building blocks (iunet_ops.hip) — internal.
#pragma once
#include "dn_internal.h"

namespace dn {

enum ThinEpi { TE_BIAS = 0, TE_SIGMOID = 1, TE_DSIG = 2, TE_PLAIN = 3 };

int chan_sums_splits(int N, long P);
// partials [N][S][C][2] doubles
hipError_t launch_chan_sums(const View& a, const View* b, int N, long P, int C, int S,
                            double* part, hipStream_t s);
hipError_t launch_gn_fwd_fin(const double* part, int S, int N, int C, int G, long P, float eps,
                             const float* gamma, const float* beta, float* stats, float* scale,
                             float* shift, hipStream_t s);
hipError_t launch_gn_bwd_fin(const double* part, int S, int N, int C, int G, long P,
                             const float* gamma, const float* stats, float* ca, float* cb,
                             float* cc, float* dgamma, float* dbeta, hipStream_t s);
hipError_t launch_affine(const View& x, const View* x2, const float* A, const float* B,
                         const float* Cc, int act, const View* res, const View& y, int N, long P,
                         int C, hipStream_t s);
hipError_t launch_vpool_fwd(const View& a, int N, int H, int W, int C, const View& y, hipStream_t s);
hipError_t launch_vpool_bwd_acc(const View& a, int N, int H, int W, int C, const View& dy,
                                const View& dx, hipStream_t s);
hipError_t launch_unshuffle(const View& du, int N, int h, int w, int C, float* g, hipStream_t s);
hipError_t launch_vadd(const View& d, const View& src, long npx, int C, hipStream_t s);
hipError_t launch_vmask(const View& d, const View& src, const View& act, long npx, int C,
                        hipStream_t s);
hipError_t launch_dsigmoid_nchw(const float* y, const float* dy, int N, int C, long HW, float* dz,
                                int ds, hipStream_t s);
hipError_t launch_conv3_thin(const View& in, int N, int H, int W, int K, const WView& wv,
                             const float* bias, int epi, const View& aux, const View& out, int nchw,
                             int nout, hipStream_t s);

}  // namespace dn
