// extern "C" boundary of libdenoise_hip.so (declared in include/denoise_hip.h).
// Validates arguments, maps failures to dn_status + a thread-local message, never throws.
#include <cmath>
#include <cstring>
#include <string>

#include "iunet.h"
#include "unet.h"

using namespace dn;

namespace {

dn_status fail(int code, const std::string& msg) {
  set_error(msg);
  return code;
}

dn_status hip_status(hipError_t e, const char* what) {
  if (e == hipSuccess) return DN_OK;
  return fail(DN_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define DN_GUARD_BEGIN try {
#define DN_GUARD_END                                              \
  }                                                               \
  catch (const std::exception& ex) { return fail(DN_ERR_ARG, ex.what()); } \
  catch (...) { return fail(DN_ERR_ARG, "unknown C++ exception"); }

}  // namespace

extern "C" {

#ifndef DN_SRC_HASH
#define DN_SRC_HASH "unknown"
#endif
// src= the sha256 prefix of the sources this library was compiled from (_build.source_hash)
const char* dn_version(void) { return "denoise_hip 0.5.0 gfx950 src=" DN_SRC_HASH; }

int dn_abi_version(void) { return DN_ABI_VERSION; }

int dn_last_error(char* buf, size_t len) {
  const std::string& s = g_last_error;
  if (buf && len) {
    size_t n = s.size() < len - 1 ? s.size() : len - 1;
    std::memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return (int)s.size();
}

dn_status dn_prepare_streams(void* stream) {
  DN_GUARD_BEGIN
  const hipStream_t s = static_cast<hipStream_t>(stream);
  const StreamDeviceGuard device_guard(s);
  SideStream* ss = side_stream(s);
  if (!ss) return fail(DN_ERR_HIP, "creating the backward's side streams failed");
  // one marker on each (its first submission binds it to a hardware queue), ordered after the
  // caller's stream and joined back into it
  if (hipEventRecord(ss->fork, s) != hipSuccess ||
      hipStreamWaitEvent(ss->st, ss->fork, 0) != hipSuccess ||
      hipStreamWaitEvent(ss->rst, ss->fork, 0) != hipSuccess ||
      hipEventRecord(ss->join, ss->st) != hipSuccess ||
      hipEventRecord(ss->rjoin, ss->rst) != hipSuccess ||
      hipStreamWaitEvent(s, ss->join, 0) != hipSuccess ||
      hipStreamWaitEvent(s, ss->rjoin, 0) != hipSuccess)
    return fail(DN_ERR_HIP, "marker on the backward's side streams failed");
  return DN_OK;
  DN_GUARD_END
}

dn_status dn_unet_param_count(const dn_unet_cfg* cfg, size_t* count) {
  DN_GUARD_BEGIN
  if (!cfg || !count) return fail(DN_ERR_ARG, "null argument");
  ParamLayout P;
  std::string err;
  if (!build_params(*cfg, P, err)) return fail(DN_ERR_ARG, err);
  *count = (size_t)P.total;
  return DN_OK;
  DN_GUARD_END
}

dn_status dn_unet_param_info(const dn_unet_cfg* cfg, int index, size_t* w_off, size_t* w_count,
                             size_t* b_count) {
  DN_GUARD_BEGIN
  if (!cfg || !w_off || !w_count || !b_count) return fail(DN_ERR_ARG, "null argument");
  ParamLayout P;
  std::string err;
  if (!build_params(*cfg, P, err)) return fail(DN_ERR_ARG, err);
  if (index < 0 || index >= NL) return fail(DN_ERR_ARG, "layer index out of range");
  *w_off = (size_t)P.L[index].woff;
  *w_count = (size_t)P.L[index].wcount;
  *b_count = (size_t)P.L[index].cout;
  return DN_OK;
  DN_GUARD_END
}

dn_status dn_unet_workspace_size(const dn_unet_cfg* cfg, int N, int H, int W, int with_backward,
                                 size_t* bytes) {
  DN_GUARD_BEGIN
  if (!cfg || !bytes) return fail(DN_ERR_ARG, "null argument");
  Plan p;
  std::string err;
  if (!build_plan(*cfg, N, H, W, with_backward != 0, p, err)) return fail(DN_ERR_ARG, err);
  *bytes = (size_t)p.total_floats * sizeof(float);
  return DN_OK;
  DN_GUARD_END
}

dn_status dn_unet_forward(const dn_unet_cfg* cfg, const float* params, const float* x, float* y,
                          int N, int H, int W, void* ws, size_t ws_bytes, void* stream) {
  return dn_unet_forward_prec(cfg, params, x, y, N, H, W, ws, ws_bytes, DN_PREC_FP32, stream);
}

dn_status dn_unet_forward_prec(const dn_unet_cfg* cfg, const float* params, const float* x,
                               float* y, int N, int H, int W, void* ws, size_t ws_bytes,
                               int precision, void* stream) {
  DN_GUARD_BEGIN
  if (precision == DN_PREC_BF16)
    return dn_unet_forward_bf16(cfg, params, x, y, N, H, W, ws, ws_bytes, stream);
  if (precision != DN_PREC_FP32 && precision != DN_PREC_FP32_X6)
    return fail(DN_ERR_ARG, "unknown precision");
  if (!cfg || !params || !x || !y || !ws) return fail(DN_ERR_ARG, "null argument");
  Plan p;
  std::string err;
  // The workspace's size decides the plan: one sized with_backward=1 gets the backward plan
  // (dense concat strides, the layout dn_unet_backward reads) and the forward saves the
  // activations the backward needs (the fused head writes d1b/na/nb); a smaller one gets the
  // forward-only plan, whose concat strides are padded to 128-B lines (a different layout).
  if (!build_plan(*cfg, N, H, W, true, p, err)) return fail(DN_ERR_ARG, err);
  if (ws_bytes < (size_t)p.total_floats * sizeof(float) &&
      !build_plan(*cfg, N, H, W, false, p, err))
    return fail(DN_ERR_ARG, err);
  if (ws_bytes < (size_t)p.total_floats * sizeof(float))
    return fail(DN_ERR_WORKSPACE, "workspace smaller than dn_unet_workspace_size()");
  return unet_forward(p, params, x, y, static_cast<float*>(ws), (hipStream_t)stream, precision);
  DN_GUARD_END
}

// the plan a forward entry point runs on this workspace (dn_unet_forward_prec's rule; bf16:
// the forward-only plan)
static dn_status forward_plan(const dn_unet_cfg* cfg, int N, int H, int W, size_t ws_bytes,
                              int precision, Plan& p) {
  std::string err;
  if (precision != DN_PREC_FP32 && precision != DN_PREC_FP32_X6 && precision != DN_PREC_BF16)
    return fail(DN_ERR_ARG, "unknown precision");
  const bool bwd_ok = precision != DN_PREC_BF16;
  if (!bwd_ok || !build_plan(*cfg, N, H, W, true, p, err) ||
      ws_bytes < (size_t)p.total_floats * sizeof(float))
    if (!build_plan(*cfg, N, H, W, false, p, err)) return fail(DN_ERR_ARG, err);
  if (ws_bytes < (size_t)p.total_floats * sizeof(float))
    return fail(DN_ERR_WORKSPACE, "workspace smaller than dn_unet_workspace_size()");
  if (!bwd_ok) p.with_bwd = false;
  return DN_OK;
}

dn_status dn_unet_pack_weights(const dn_unet_cfg* cfg, const float* params, int N, int H, int W,
                               void* ws, size_t ws_bytes, int precision, void* stream) {
  DN_GUARD_BEGIN
  if (!cfg || !params || !ws) return fail(DN_ERR_ARG, "null argument");
  Plan p;
  const dn_status st = forward_plan(cfg, N, H, W, ws_bytes, precision, p);
  if (st != DN_OK) return st;
  return unet_forward(p, params, nullptr, nullptr, static_cast<float*>(ws), (hipStream_t)stream,
                      precision, nullptr, PACK_ONLY);
  DN_GUARD_END
}

dn_status dn_unet_forward_prepacked(const dn_unet_cfg* cfg, const float* params, const float* x,
                                    float* y, int N, int H, int W, void* ws, size_t ws_bytes,
                                    int precision, void* stream) {
  DN_GUARD_BEGIN
  if (!cfg || !params || !x || !y || !ws) return fail(DN_ERR_ARG, "null argument");
  Plan p;
  const dn_status st = forward_plan(cfg, N, H, W, ws_bytes, precision, p);
  if (st != DN_OK) return st;
  return unet_forward(p, params, x, y, static_cast<float*>(ws), (hipStream_t)stream, precision,
                      nullptr, RUN_ONLY);
  DN_GUARD_END
}

dn_status dn_unet_forward_n2n(const dn_unet_cfg* cfg, const float* params, const float* x,
                              float* den, const uint8_t* rd_idx, int N, int H, int W, void* ws,
                              size_t ws_bytes, int precision, void* stream) {
  DN_GUARD_BEGIN
  if (precision != DN_PREC_FP32 && precision != DN_PREC_FP32_X6)
    return fail(DN_ERR_ARG, "precision must be DN_PREC_FP32 or DN_PREC_FP32_X6");
  if (!cfg || !params || !x || !den || !rd_idx || !ws) return fail(DN_ERR_ARG, "null argument");
  Plan p;
  std::string err;
  if (!build_plan(*cfg, N, H, W, false, p, err)) return fail(DN_ERR_ARG, err);
  if (ws_bytes < (size_t)p.total_floats * sizeof(float))
    return fail(DN_ERR_WORKSPACE, "workspace smaller than dn_unet_workspace_size()");
  p.with_bwd = false;  // no-grad pass: nothing is saved
  return unet_forward(p, params, x, den, static_cast<float*>(ws), (hipStream_t)stream, precision,
                      rd_idx);
  DN_GUARD_END
}

dn_status dn_unet_forward_bf16(const dn_unet_cfg* cfg, const float* params, const float* x,
                               float* y, int N, int H, int W, void* ws, size_t ws_bytes,
                               void* stream) {
  DN_GUARD_BEGIN
  if (!cfg || !params || !x || !y || !ws) return fail(DN_ERR_ARG, "null argument");
  Plan p;
  std::string err;
  if (!build_plan(*cfg, N, H, W, false, p, err)) return fail(DN_ERR_ARG, err);
  if (ws_bytes < (size_t)p.total_floats * sizeof(float))
    return fail(DN_ERR_WORKSPACE, "workspace smaller than dn_unet_workspace_size()");
  p.with_bwd = false;  // inference only: nothing is saved for a backward
  return unet_forward(p, params, x, y, static_cast<float*>(ws), (hipStream_t)stream,
                      DN_PREC_BF16);
  DN_GUARD_END
}

dn_status dn_unet_backward(const dn_unet_cfg* cfg, const float* params, const float* dy,
                           float* dparams, float* dx, int N, int H, int W, void* ws,
                           size_t ws_bytes, void* stream) {
  return dn_unet_backward_prec(cfg, params, dy, dparams, dx, N, H, W, ws, ws_bytes, DN_PREC_FP32,
                               stream);
}

dn_status dn_unet_backward_prec(const dn_unet_cfg* cfg, const float* params, const float* dy,
                                float* dparams, float* dx, int N, int H, int W, void* ws,
                                size_t ws_bytes, int precision, void* stream) {
  DN_GUARD_BEGIN
  if (precision != DN_PREC_FP32 && precision != DN_PREC_FP32_X6)
    return fail(DN_ERR_ARG, "backward precision must be DN_PREC_FP32 or DN_PREC_FP32_X6");
  if (!cfg || !params || !dy || !dparams || !ws) return fail(DN_ERR_ARG, "null argument");
  Plan p;
  std::string err;
  if (!build_plan(*cfg, N, H, W, true, p, err)) return fail(DN_ERR_ARG, err);
  if (ws_bytes < (size_t)p.total_floats * sizeof(float))
    return fail(DN_ERR_WORKSPACE,
                "workspace smaller than dn_unet_workspace_size(with_backward=1)");
  return unet_backward(p, params, dy, dparams, dx, static_cast<float*>(ws), (hipStream_t)stream,
                       precision);
  DN_GUARD_END
}

dn_status dn_unet_backward_split(const dn_unet_cfg* cfg, const float* params, const float* dy,
                                 float* dparams, float* dx, int N, int H, int W, void* ws,
                                 size_t ws_bytes, int precision, void* stream, void* tail_ready,
                                 int64_t* tail_begin_out) {
  DN_GUARD_BEGIN
  if (precision != DN_PREC_FP32 && precision != DN_PREC_FP32_X6)
    return fail(DN_ERR_ARG, "backward precision must be DN_PREC_FP32 or DN_PREC_FP32_X6");
  if (!cfg) return fail(DN_ERR_ARG, "null argument");
  Plan p;
  std::string err;
  if (!build_plan(*cfg, N, H, W, true, p, err)) return fail(DN_ERR_ARG, err);
  if (tail_begin_out) *tail_begin_out = tail_begin(p);
  if (!params || !dy || !dparams || !ws) {
    if (!params && !dy && !dparams && !ws && !tail_ready) return DN_OK;  // a tail_begin query
    return fail(DN_ERR_ARG, "null argument");
  }
  if (ws_bytes < (size_t)p.total_floats * sizeof(float))
    return fail(DN_ERR_WORKSPACE,
                "workspace smaller than dn_unet_workspace_size(with_backward=1)");
  return unet_backward(p, params, dy, dparams, dx, static_cast<float*>(ws), (hipStream_t)stream,
                       precision, static_cast<hipEvent_t>(tail_ready));
  DN_GUARD_END
}

dn_status dn_unet_debug_buffers(const dn_unet_cfg* cfg, int N, int H, int W, int with_backward,
                                int64_t* desc, int max_entries, int* n_entries) {
  DN_GUARD_BEGIN
  if (!cfg || !desc || !n_entries) return fail(DN_ERR_ARG, "null argument");
  Plan p;
  std::string err;
  if (!build_plan(*cfg, N, H, W, with_backward != 0, p, err)) return fail(DN_ERR_ARG, err);
  int n = 0;
  auto add = [&](long off, int stride, int level) {
    if (n < max_entries) {
      desc[3 * n] = off;
      desc[3 * n + 1] = stride;
      desc[3 * n + 2] = level;
    }
    ++n;
  };
  const int nf = p.nf;
  add(p.c1, p.c1s, 0); add(p.a0, nf, 0); add(p.a1, nf, 0);
  for (int l = 1; l <= 4; ++l) add(p.c[l], p.cs[l], l);
  for (int l = 1; l <= 4; ++l) add(p.a[l], nf, l);
  add(p.p5, nf, 5); add(p.a6, nf, 5);
  for (int l = 1; l <= 4; ++l) add(p.da[l], 2 * nf, l);
  for (int l = 1; l <= 4; ++l) add(p.db[l], 2 * nf, l);
  add(p.d1a, 96, 0); add(p.d1b, 96, 0); add(p.na, 96, 0); add(p.nb, 96, 0);
  if (with_backward) {
    add(p.g_nb, 96, 0); add(p.g_na, 96, 0); add(p.g_d1b, 96, 0); add(p.g_d1a, 96, 0);
    add(p.g_c1, 2 * nf, 0);
    for (int l = 1; l <= 4; ++l) add(p.g_c[l], p.cs[l], l);
    for (int l = 1; l <= 4; ++l) add(p.g_da[l], 2 * nf, l);
    for (int l = 1; l <= 4; ++l) add(p.g_db[l], 2 * nf, l);
    for (int l = 1; l <= 4; ++l) add(p.g_a[l], nf, l);
    add(p.g_a6, nf, 5); add(p.g_p5, nf, 5); add(p.g_a0, nf, 0); add(p.g_a1, nf, 0);
  }
  *n_entries = n;
  return DN_OK;
  DN_GUARD_END
}

dn_status dn_n2n_subsample(const float* img, int N, int C, int H, int W, const uint8_t* rd_idx_in,
                           uint64_t seed, uint64_t offset, uint64_t cell_base, float* sub1,
                           float* sub2, uint8_t* rd_idx_out, void* stream) {
  if (N < 0 || C < 1 || H < 0 || W < 0 || (H & 1) || (W & 1))
    return fail(DN_ERR_ARG, "H and W must be even");
  if ((long)N * H * W == 0) return DN_OK;
  if (!img || !sub1 || !sub2) return fail(DN_ERR_ARG, "null argument");
  const OpTimer timer((hipStream_t)stream, "subsample", 0, C, C, H, W, N);
  return hip_status(launch_subsample(img, N, C, H, W, rd_idx_in, seed, offset, cell_base, sub1,
                                     sub2, rd_idx_out, (hipStream_t)stream),
                    "dn_n2n_subsample");
}

dn_status dn_n2n_masks(const uint8_t* rd_idx, int64_t ncells, uint8_t* mask1, uint8_t* mask2,
                       void* stream) {
  if (ncells < 0) return fail(DN_ERR_ARG, "ncells < 0");
  if (ncells == 0) return DN_OK;
  if (!rd_idx || !mask1 || !mask2) return fail(DN_ERR_ARG, "null argument");
  return hip_status(launch_masks(rd_idx, ncells, mask1, mask2, (hipStream_t)stream),
                    "dn_n2n_masks");
}

dn_status dn_n2n_subimage_from_mask(const float* img, int N, int C, int H, int W,
                                    const uint8_t* mask, float* sub, void* stream) {
  if (N < 0 || C < 1 || (H & 1) || (W & 1)) return fail(DN_ERR_ARG, "H and W must be even");
  if ((long)N * H * W == 0) return DN_OK;
  if (!img || !mask || !sub) return fail(DN_ERR_ARG, "null argument");
  return hip_status(launch_subimage_from_mask(img, N, C, H, W, mask, sub, (hipStream_t)stream),
                    "dn_n2n_subimage_from_mask");
}

dn_status dn_add_gauss_noise(const float* clean, int N, int64_t per_image, float std_,
                             const float* std_per_image, uint64_t seed, uint64_t offset,
                             uint64_t elem_base, float* noisy, void* stream) {
  if (N < 0 || per_image < 0) return fail(DN_ERR_ARG, "negative size");
  if ((long)N * per_image == 0) return DN_OK;
  if (!clean || !noisy) return fail(DN_ERR_ARG, "null argument");
  const OpTimer timer((hipStream_t)stream, "noise", 0);
  return hip_status(launch_noise(clean, N, per_image, std_, std_per_image, seed, offset, elem_base,
                                 noisy, (hipStream_t)stream),
                    "dn_add_gauss_noise");
}

dn_status dn_add_poisson_noise(const float* clean, int N, int64_t per_image, float lam,
                               const float* lam_per_image, uint64_t seed, uint64_t offset,
                               uint64_t elem_base, float* noisy, void* stream) {
  if (N < 0 || per_image < 0) return fail(DN_ERR_ARG, "negative size");
  if (!lam_per_image && !(lam > 0.f && lam <= 500.f)) return fail(DN_ERR_ARG, "lam must be in (0, 500]");
  if ((long)N * per_image == 0) return DN_OK;
  if (!clean || !noisy) return fail(DN_ERR_ARG, "null argument");
  const OpTimer timer((hipStream_t)stream, "noise", 0);
  return hip_status(launch_poisson(clean, N, per_image, lam, lam_per_image, seed, offset, elem_base,
                                   noisy, (hipStream_t)stream),
                    "dn_add_poisson_noise");
}

size_t dn_loss_partials_size(void) { return loss_partials_bytes(); }

dn_status dn_n2n_loss(const float* out, const float* sub2, const float* den, const uint8_t* rd_idx,
                      int N, int C, int h, int w, float lambda, float* dout, float* loss3,
                      void* partial_ws, void* stream) {
  if (!out || !sub2 || !den || !rd_idx || !dout || !loss3 || !partial_ws)
    return fail(DN_ERR_ARG, "null argument");
  if (N < 1 || C < 1 || h < 1 || w < 1) return fail(DN_ERR_ARG, "empty loss input");
  const OpTimer timer((hipStream_t)stream, "loss", 0);
  return hip_status(launch_n2n_loss(out, sub2, den, rd_idx, N, C, h, w, lambda, dout, loss3,
                                    partial_ws, (hipStream_t)stream),
                    "dn_n2n_loss");
}

dn_status dn_structure_loss(const float* pred, const float* pred2, const float* target, int N, int C,
                            int H, int W, float alpha, float beta, float gamma, float* dpred,
                            float* dpred2, float* loss5, void* partial_ws, void* stream) {
  if (!pred || !pred2 || !target || !dpred || !dpred2 || !loss5 || !partial_ws)
    return fail(DN_ERR_ARG, "null argument");
  if (N < 1 || C < 1 || H < 2 || W < 2) return fail(DN_ERR_ARG, "Structure_loss needs H, W >= 2");
  const OpTimer timer((hipStream_t)stream, "loss", 0);
  return hip_status(launch_structure_loss(pred, pred2, target, N, C, H, W, alpha, beta, gamma,
                                          dpred, dpred2, loss5, partial_ws, (hipStream_t)stream),
                    "dn_structure_loss");
}

dn_status dn_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                       float lr, float beta1, float beta2, float eps, int64_t step,
                       float grad_scale, void* stream) {
  if (n < 0 || step < 1) return fail(DN_ERR_ARG, "n >= 0 and step >= 1 required");
  if (n == 0) return DN_OK;
  if (!param || !grad || !exp_avg || !exp_avg_sq) return fail(DN_ERR_ARG, "null argument");
  // scalars exactly as torch/optim/adam.py _single_tensor_adam computes them (python floats)
  const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
  const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
  const double step_size = (double)lr / bc1;
  const double bc2s = std::sqrt(bc2);
  const OpTimer timer((hipStream_t)stream, "adam", 0);
  return hip_status(launch_adam(param, grad, exp_avg, exp_avg_sq, n, (float)(1.0 - (double)beta1),
                                beta2, (float)(1.0 - (double)beta2), (float)step_size,
                                (float)bc2s, eps, grad_scale, (hipStream_t)stream),
                    "dn_adam_step");
}

dn_status dn_accumulate(float* dst, const float* src, int64_t n, void* stream) {
  if (n < 0) return fail(DN_ERR_ARG, "n < 0");
  if (n == 0) return DN_OK;
  if (!dst || !src) return fail(DN_ERR_ARG, "null argument");
  const OpTimer timer((hipStream_t)stream, "accumulate", 0);
  return hip_status(launch_accumulate(dst, src, n, (hipStream_t)stream), "dn_accumulate");
}

// ---- evaluation path ----------------------------------------------------------------------
size_t dn_eval_partials_size(void) { return EVAL_PARTS * sizeof(double); }

dn_status dn_u8_to_unit(const uint8_t* x, int64_t n, float* y, void* stream) {
  if (n < 0) return fail(DN_ERR_ARG, "n < 0");
  if (n == 0) return DN_OK;
  if (!x || !y) return fail(DN_ERR_ARG, "null argument");
  return hip_status(launch_u8_to_unit(x, n, y, (hipStream_t)stream), "dn_u8_to_unit");
}

int dn_tile_count(int extent, int patch, int stride) {
  if (extent < 1 || patch < 1 || stride < 1) return 0;
  return (extent + stride - 1) / stride;  // range(0, extent, stride)
}

static bool tile_args_ok(int C, int H, int W, int patch, int stride) {
  return C >= 1 && H >= 1 && W >= 1 && patch >= 1 && stride >= 1 && stride <= patch;
}

dn_status dn_tile_extract(const uint8_t* img, int C, int H, int W, int patch, int stride,
                          float* tiles, void* stream) {
  if (!img || !tiles) return fail(DN_ERR_ARG, "null argument");
  if (!tile_args_ok(C, H, W, patch, stride))
    return fail(DN_ERR_ARG, "need C,H,W,patch >= 1 and 1 <= stride <= patch");
  return hip_status(launch_tile_extract(img, C, H, W, patch, stride, dn_tile_count(H, patch, stride),
                                        dn_tile_count(W, patch, stride), tiles, (hipStream_t)stream),
                    "dn_tile_extract");
}

dn_status dn_tile_blend(const float* pred, int C, int H, int W, int patch, int stride,
                        const float* wmask, float* out, uint8_t* out_u8, void* stream) {
  if (!pred || !wmask || (!out && !out_u8)) return fail(DN_ERR_ARG, "null argument");
  if (!tile_args_ok(C, H, W, patch, stride))
    return fail(DN_ERR_ARG, "need C,H,W,patch >= 1 and 1 <= stride <= patch");
  return hip_status(launch_tile_blend(pred, C, H, W, patch, stride, dn_tile_count(H, patch, stride),
                                      dn_tile_count(W, patch, stride), wmask, out, out_u8,
                                      (hipStream_t)stream),
                    "dn_tile_blend");
}

dn_status dn_quantize_u8(const float* x, int64_t n, int plus_half, uint8_t* y, void* stream) {
  if (n < 0) return fail(DN_ERR_ARG, "n < 0");
  if (n == 0) return DN_OK;
  if (!x || !y) return fail(DN_ERR_ARG, "null argument");
  return hip_status(launch_quantize_u8(x, n, plus_half, y, (hipStream_t)stream), "dn_quantize_u8");
}

dn_status dn_psnr_u8(const uint8_t* a, const uint8_t* b, int64_t n, void* part, double* psnr,
                     void* stream) {
  if (n < 1) return fail(DN_ERR_ARG, "n >= 1 required");
  if (!a || !b || !part || !psnr) return fail(DN_ERR_ARG, "null argument");
  return hip_status(launch_psnr(a, b, n, static_cast<double*>(part), psnr, (hipStream_t)stream),
                    "dn_psnr_u8");
}

dn_status dn_ssim_u8(const uint8_t* a, const uint8_t* b, int C, int H, int W, int hwc, void* part,
                     double* ssim, void* stream) {
  if (C < 1 || H <= 10 || W <= 10) return fail(DN_ERR_ARG, "need C >= 1 and H, W > 10");
  if (!a || !b || !part || !ssim) return fail(DN_ERR_ARG, "null argument");
  return hip_status(launch_ssim(a, b, C, H, W, hwc, static_cast<double*>(part), ssim,
                                (hipStream_t)stream),
                    "dn_ssim_u8");
}

dn_status dn_l1_mean(const float* a, const float* b, int64_t n, void* part, double* l1,
                     void* stream) {
  if (n < 1) return fail(DN_ERR_ARG, "n >= 1 required");
  if (!a || !b || !part || !l1) return fail(DN_ERR_ARG, "null argument");
  return hip_status(launch_l1(a, b, n, static_cast<double*>(part), l1, (hipStream_t)stream),
                    "dn_l1_mean");
}

dn_status dn_l1_mean_batched(const float* a, const float* b, int64_t P, int64_t n, double* l1,
                             void* stream) {
  if (P < 0 || n < 1) return fail(DN_ERR_ARG, "P >= 0 and n >= 1 required");
  if (P == 0) return DN_OK;
  if (P > 0x7fffffffL) return fail(DN_ERR_ARG, "P too large");
  if (!a || !b || !l1) return fail(DN_ERR_ARG, "null argument");
  return hip_status(launch_l1_batched(a, b, P, n, l1, (hipStream_t)stream), "dn_l1_mean_batched");
}

// ---- op-level entry points ------------------------------------------------------------
size_t dn_conv2d_pack_size(int Cin, int Cout, int ksize, int backward_data) {
  if ((ksize != 1 && ksize != 3) || Cin < 1 || Cout < 1) return 0;
  const long n = backward_data ? conv_dgrad_pack_size(Cout, Cin, ksize)
                               : conv_fwd_pack_size(Cin, Cout, ksize);
  return n < 0 ? 0 : sizeof(float) * (size_t)n;
}

size_t dn_deconv2x2_pack_size(int Cin, int Cout, int backward_data) {
  if (Cin < 1 || Cout < 1) return 0;
  const long n = backward_data ? deconv_dgrad_pack_size(Cout, Cin) : deconv_fwd_pack_size(Cin, Cout);
  return n < 0 ? 0 : sizeof(float) * (size_t)n;
}

static dn_status need_pack(void* ws, size_t have, size_t need) {
  if (need == 0) return fail(DN_ERR_ARG, "unsupported channel count for this kernel build");
  if (!ws || have < need) return fail(DN_ERR_WORKSPACE, "pack scratch smaller than *_pack_size()");
  return DN_OK;
}

dn_status dn_conv2d_forward(const float* x, int x_stride, int N, int H, int W, int Cin,
                            const float* w, const float* b, int Cout, int ksize, int act, float* y,
                            int y_stride, void* pack_ws, size_t pack_bytes, void* stream) {
  if (!x || !w || !b || !y) return fail(DN_ERR_ARG, "null argument");
  if (ksize != 1 && ksize != 3) return fail(DN_ERR_ARG, "ksize must be 1 or 3");
  if (N < 1 || H < 1 || W < 1 || Cin < 1 || x_stride < Cin || y_stride < Cout)
    return fail(DN_ERR_ARG, "bad shape");
  if (dn_status st = need_pack(pack_ws, pack_bytes, dn_conv2d_pack_size(Cin, Cout, ksize, 0))) return st;
  hipStream_t s = (hipStream_t)stream;
  float* wp = static_cast<float*>(pack_ws);
  hipError_t e = pack_conv_fwd(w, Cin, Cout, ksize, wp, s);
  if (e == hipSuccess)
    e = conv_forward(View{const_cast<float*>(x), x_stride, 0}, N, H, W, Cin, wp, b, Cout, ksize,
                     act, View{y, y_stride, 0}, OUT_NHWC, s);
  return hip_status(e, "dn_conv2d_forward");
}

size_t dn_conv2d_bf16_pack_size(int Cin, int Cout) {
  if (Cin < 1 || Cout < 1) return 0;
  const long e = bf16_pack_elems(Cin, Cout);
  return e < 0 ? 0 : 2 * (size_t)e;
}

dn_status dn_conv2d_forward_bf16(const float* x, int x_stride, int N, int H, int W, int Cin,
                                 const float* w, const float* b, int Cout, int act, float* y,
                                 int y_stride, void* pack_ws, size_t pack_bytes, void* stream) {
  if (!x || !w || !b || !y) return fail(DN_ERR_ARG, "null argument");
  if (N < 1 || H < 1 || W < 1 || Cin < 1 || x_stride < Cin || y_stride < Cout || (Cout & 3) ||
      (y_stride & 3))
    return fail(DN_ERR_ARG, "bad shape (Cout and y_stride must be multiples of 4)");
  if (dn_status st = need_pack(pack_ws, pack_bytes, dn_conv2d_bf16_pack_size(Cin, Cout))) return st;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = launch_pack_bf16(conv_fwd_view(w, Cin, 3), Cin, Cout, pack_ws, s);
  if (e == hipSuccess) {
    FwdArgs a{};
    a.in = x; a.in_stride = x_stride; a.in_off = 0; a.IHt = H; a.IWt = W;
    a.N = N; a.OH = H; a.OW = W; a.K = Cin; a.NOUT = Cout;
    a.wp = static_cast<const float*>(pack_ws); a.bias = b; a.epi = act ? EPI_BIAS_ACT : EPI_BIAS;
    a.out = y; a.out_stride = y_stride; a.out_off = 0; a.out_layout = OUT_NHWC;
    e = launch_fwd_bf16(a, s);
  }
  return hip_status(e, "dn_conv2d_forward_bf16");
}

size_t dn_conv2d_x6_pack_size(int Cin, int Cout, int backward_data) {
  if (Cin < 1 || Cout < 1) return 0;
  const long e = backward_data ? x6_pack_elems(Cout, Cin, x6_dgrad_zc(Cin))
                               : x6_pack_elems(Cin, Cout, 0);
  return e < 0 ? 0 : 2 * (size_t)e;
}

dn_status dn_conv2d_forward_x6(const float* x, int x_stride, int N, int H, int W, int Cin,
                               const float* w, const float* b, int Cout, int act, float* y,
                               int y_stride, void* pack_ws, size_t pack_bytes, void* stream) {
  if (!x || !w || !b || !y) return fail(DN_ERR_ARG, "null argument");
  if (N < 1 || H < 1 || W < 1 || Cin < 1 || x_stride < Cin || y_stride < Cout)
    return fail(DN_ERR_ARG, "bad shape");
  const size_t need = dn_conv2d_x6_pack_size(Cin, Cout, 0);
  if (need == 0) return fail(DN_ERR_ARG, "bf16x6 forward supports Cout <= 96");
  if (dn_status st = need_pack(pack_ws, pack_bytes, need)) return st;
  hipStream_t s = (hipStream_t)stream;
  // large grids with a partial last 32-channel chunk: the pipelined kernel's tail packing
  const int tail = x6_image_mode(N, H, W, Cin, Cout, 0,
                                 x_stride % 4 == 0 && Cin % 4 == 0 && y_stride % 4 == 0);
  hipError_t e = launch_pack_x6(conv_fwd_view(w, Cin, 3), Cin, Cout, 0, pack_ws, s, tail);
  if (e == hipSuccess) {
    FwdArgs a{};
    a.x6_tail = tail;
    a.in = x; a.in_stride = x_stride; a.in_off = 0; a.IHt = H; a.IWt = W;
    a.N = N; a.OH = H; a.OW = W; a.K = Cin; a.NOUT = Cout;
    a.wp = static_cast<const float*>(pack_ws); a.bias = b; a.epi = act ? EPI_BIAS_ACT : EPI_BIAS;
    a.out = y; a.out_stride = y_stride; a.out_off = 0; a.out_layout = OUT_NHWC;
    e = launch_fwd_x6(a, s);
  }
  return hip_status(e, "dn_conv2d_forward_x6");
}

dn_status dn_conv2d_backward_data_x6(const float* dz, int N, int H, int W, int Cout,
                                     const float* w, int Cin, const float* mask, int mask_stride,
                                     int accumulate, float* dx, int dx_stride, void* pack_ws,
                                     size_t pack_bytes, void* stream) {
  if (!dz || !w || !dx) return fail(DN_ERR_ARG, "null argument");
  if (N < 1 || H < 1 || W < 1 || Cout < 1 || dx_stride < Cin) return fail(DN_ERR_ARG, "bad shape");
  if (mask && accumulate) return fail(DN_ERR_ARG, "mask and accumulate are exclusive");
  const size_t need = dn_conv2d_x6_pack_size(Cin, Cout, 1);
  if (need == 0) return fail(DN_ERR_ARG, "bf16x6 data gradient: unsupported Cin");
  if (dn_status st = need_pack(pack_ws, pack_bytes, need)) return st;
  hipStream_t s = (hipStream_t)stream;
  const int zc = x6_dgrad_zc(Cin);
  const int tail = x6_image_mode(N, H, W, Cout, Cin, zc,
                                 Cout % 4 == 0 && dx_stride % 4 == 0 && (!mask || mask_stride % 4 == 0));
  hipError_t e = launch_pack_x6(conv_dgrad_view(w, Cin, 3), Cout, Cin, zc, pack_ws, s, tail);
  if (e == hipSuccess) {
    FwdArgs a{};
    a.x6_tail = tail;
    a.in = dz; a.in_stride = Cout; a.in_off = 0; a.IHt = H; a.IWt = W;
    a.N = N; a.OH = H; a.OW = W; a.K = Cout; a.NOUT = Cin;
    a.zc = zc;
    a.wp = static_cast<const float*>(pack_ws);
    a.wp_z = zc ? x6_pack_elems(Cout, Cin, zc) / ((Cin + zc - 1) / zc) : 0;
    a.epi = mask ? EPI_MASK : (accumulate ? EPI_ACCUM : EPI_PLAIN);
    a.out = dx; a.out_stride = dx_stride; a.out_off = 0; a.out_layout = OUT_NHWC;
    a.mask = mask; a.mask_stride = mask_stride; a.mask_off = 0;
    e = launch_fwd_x6(a, s);
  }
  return hip_status(e, "dn_conv2d_backward_data_x6");
}

dn_status dn_conv2d_backward_data(const float* dz, int N, int H, int W, int Cout, const float* w,
                                  int Cin, int ksize, const float* mask, int mask_stride,
                                  int accumulate, float* dx, int dx_stride, void* pack_ws,
                                  size_t pack_bytes, void* stream) {
  if (!dz || !w || !dx) return fail(DN_ERR_ARG, "null argument");
  if (ksize != 1 && ksize != 3) return fail(DN_ERR_ARG, "ksize must be 1 or 3");
  if (N < 1 || H < 1 || W < 1 || Cout < 1 || dx_stride < Cin) return fail(DN_ERR_ARG, "bad shape");
  if (mask && accumulate) return fail(DN_ERR_ARG, "mask and accumulate are exclusive");
  if (dn_status st = need_pack(pack_ws, pack_bytes, dn_conv2d_pack_size(Cin, Cout, ksize, 1))) return st;
  const int epi = mask ? EPI_MASK : (accumulate ? EPI_ACCUM : EPI_PLAIN);
  hipStream_t s = (hipStream_t)stream;
  float* wp = static_cast<float*>(pack_ws);
  hipError_t e = pack_conv_dgrad(w, Cin, Cin, Cout, ksize, wp, s);
  if (e == hipSuccess)
    e = conv_dgrad(View{const_cast<float*>(dz), Cout, 0}, N, H, W, Cout, wp, Cin, ksize, epi,
                   View{const_cast<float*>(mask), mask_stride, 0}, View{dx, dx_stride, 0}, s);
  return hip_status(e, "dn_conv2d_backward_data");
}

size_t dn_conv2d_wgrad_slab_size(int N, int H, int W, int Cin, int Cout, int ksize) {
  const int mode = ksize == 3 ? W_C3 : W_C1;
  return sizeof(float) * (64 + (size_t)wgrad_slab_floats(mode, N, H, W, Cin, Cout));
}

dn_status dn_conv2d_backward_weight(const float* dz, const float* x, int x_stride, int N, int H,
                                    int W, int Cin, int Cout, int ksize, float* dwb, void* slab,
                                    void* stream) {
  if (!dz || !x || !dwb || !slab) return fail(DN_ERR_ARG, "null argument");
  if (ksize != 1 && ksize != 3) return fail(DN_ERR_ARG, "ksize must be 1 or 3");
  const int mode = ksize == 3 ? W_C3 : W_C1;
  if (!wgrad_supported(mode, Cout, Cin)) return fail(DN_ERR_ARG, "unsupported Cout");
  if (mode == W_C1 && Cin > 96) return fail(DN_ERR_ARG, "1x1 wgrad supports Cin <= 96");
  const int sp = wgrad_splits(mode, N, H, W, Cin, Cout);
  return hip_status(wgrad(mode, View{const_cast<float*>(dz), Cout, 0},
                          View{const_cast<float*>(x), x_stride, 0}, N, H, W, Cout, Cin, dwb,
                          static_cast<float*>(slab), sp, (hipStream_t)stream),
                    "dn_conv2d_backward_weight");
}

dn_status dn_conv2d_backward_weight_x6(const float* dz, const float* x, int x_stride, int N,
                                       int H, int W, int Cin, int Cout, float* dwb, void* slab,
                                       void* stream) {
  if (!dz || !x || !dwb || !slab) return fail(DN_ERR_ARG, "null argument");
  if (!wgrad_supported(W_C3, Cout, Cin)) return fail(DN_ERR_ARG, "unsupported Cout");
  const int sp = wgrad_splits(W_C3, N, H, W, Cin, Cout);
  return hip_status(wgrad(W_C3, View{const_cast<float*>(dz), Cout, 0},
                          View{const_cast<float*>(x), x_stride, 0}, N, H, W, Cout, Cin, dwb,
                          static_cast<float*>(slab), sp, (hipStream_t)stream, true),
                    "dn_conv2d_backward_weight_x6");
}

dn_status dn_deconv2x2_forward(const float* x, int N, int H, int W, int Cin, const float* w,
                               const float* b, int Cout, float* y, int y_stride, int y_off,
                               void* pack_ws, size_t pack_bytes, void* stream) {
  if (!x || !w || !b || !y) return fail(DN_ERR_ARG, "null argument");
  if (N < 1 || H < 1 || W < 1 || Cin < 1 || y_stride < y_off + Cout)
    return fail(DN_ERR_ARG, "bad shape");
  if (dn_status st = need_pack(pack_ws, pack_bytes, dn_deconv2x2_pack_size(Cin, Cout, 0))) return st;
  hipStream_t s = (hipStream_t)stream;
  float* wp = static_cast<float*>(pack_ws);
  hipError_t e = pack_deconv_fwd(w, Cin, Cout, wp, s);
  if (e == hipSuccess)
    e = deconv_forward(View{const_cast<float*>(x), Cin, 0}, N, H, W, Cin, wp, b, Cout,
                       View{y, y_stride, y_off}, s);
  return hip_status(e, "dn_deconv2x2_forward");
}

size_t dn_deconv2x2_x6_pack_size(void) { return 4 * sizeof(uint16_t) * (size_t)X6_HEAD_BF; }

dn_status dn_deconv2x2_forward_x6(const float* x, int N, int H, int W, const float* w,
                                  const float* b, float* y, int y_stride, int y_off, void* pack_ws,
                                  size_t pack_bytes, void* stream) {
  if (!x || !w || !b || !y) return fail(DN_ERR_ARG, "null argument");
  if (N < 1 || H < 1 || W < 1 || y_stride < y_off + 96 || ((y_stride | y_off) & 3))
    return fail(DN_ERR_ARG, "bad shape");
  if (dn_status st = need_pack(pack_ws, pack_bytes, dn_deconv2x2_x6_pack_size())) return st;
  hipStream_t s = (hipStream_t)stream;
  FwdArgs a{};
  a.in = x; a.in_stride = 96; a.in_off = 0; a.IHt = H; a.IWt = W;
  a.N = N; a.OH = H; a.OW = W; a.K = 96; a.NOUT = 96; a.bias = b;
  a.out = y; a.out_stride = y_stride; a.out_off = y_off;
  if (!deconv_x6_ok(a)) return fail(DN_ERR_ARG, "shape outside the bf16x6 deconv kernel");
  hipError_t e = launch_pack_deconv_x6(w, pack_ws, s);
  if (e == hipSuccess) e = launch_deconv_x6(a, pack_ws, s);
  return hip_status(e, "dn_deconv2x2_forward_x6");
}

dn_status dn_deconv2x2_backward_data_x6(const float* dy, int dy_stride, int N, int H, int W,
                                        const float* w, const float* mask, float* dx,
                                        void* pack_ws, size_t pack_bytes, void* stream) {
  if (!dy || !w || !dx) return fail(DN_ERR_ARG, "null argument");
  if (N < 1 || H < 1 || W < 1 || dy_stride < 96 || (dy_stride & 3)) return fail(DN_ERR_ARG, "bad shape");
  if (dn_status st = need_pack(pack_ws, pack_bytes, dn_deconv2x2_x6_pack_size())) return st;
  hipStream_t s = (hipStream_t)stream;
  FwdArgs a{};
  a.in = dy; a.in_stride = dy_stride; a.in_off = 0; a.IHt = 2 * H; a.IWt = 2 * W;
  a.N = N; a.OH = H; a.OW = W; a.K = 96; a.NOUT = 96;
  a.epi = mask ? EPI_MASK : EPI_PLAIN; a.mask = mask; a.mask_stride = 96; a.mask_off = 0;
  a.out = dx; a.out_stride = 96; a.out_off = 0;
  if (!deconv_dgrad_x6_ok(a)) return fail(DN_ERR_ARG, "shape outside the bf16x6 deconv kernel");
  PackBatch b;
  b.j[b.n++] = pack_job_deconv_dgrad_x6(w, pack_ws);
  hipError_t e = pack_flush(b, s);
  if (e == hipSuccess) e = launch_deconv_dgrad_x6(a, pack_ws, s);
  return hip_status(e, "dn_deconv2x2_backward_data_x6");
}

dn_status dn_deconv2x2_backward_data(const float* dy, int dy_stride, int N, int H, int W, int Cout,
                                     const float* w, int Cin, const float* mask, float* dx,
                                     void* pack_ws, size_t pack_bytes, void* stream) {
  if (!dy || !w || !dx) return fail(DN_ERR_ARG, "null argument");
  if (N < 1 || H < 1 || W < 1 || Cout < 1 || dy_stride < Cout) return fail(DN_ERR_ARG, "bad shape");
  if (dn_status st = need_pack(pack_ws, pack_bytes, dn_deconv2x2_pack_size(Cin, Cout, 1))) return st;
  hipStream_t s = (hipStream_t)stream;
  float* wp = static_cast<float*>(pack_ws);
  hipError_t e = pack_deconv_dgrad(w, Cout, Cin, wp, s);
  if (e == hipSuccess)
    e = deconv_dgrad(View{const_cast<float*>(dy), dy_stride, 0}, N, H, W, Cout, wp, Cin,
                     View{const_cast<float*>(mask), Cin, 0}, mask ? EPI_MASK : EPI_PLAIN,
                     View{dx, Cin, 0}, s);
  return hip_status(e, "dn_deconv2x2_backward_data");
}

size_t dn_deconv2x2_wgrad_slab_size(int N, int H, int W, int Cin, int Cout) {
  return sizeof(float) * (64 + (size_t)wgrad_slab_floats(W_UP2, N, H, W, Cin, Cout));
}

dn_status dn_deconv2x2_backward_weight(const float* dy, int dy_stride, const float* x, int N, int H,
                                       int W, int Cin, int Cout, float* dwb, void* slab,
                                       void* stream) {
  if (!dy || !x || !dwb || !slab) return fail(DN_ERR_ARG, "null argument");
  if (!wgrad_supported(W_UP2, Cout, Cin)) return fail(DN_ERR_ARG, "unsupported Cout");
  const int sp = wgrad_splits(W_UP2, N, H, W, Cin, Cout);
  return hip_status(wgrad(W_UP2, View{const_cast<float*>(dy), dy_stride, 0},
                          View{const_cast<float*>(x), Cin, 0}, N, H, W, Cout, Cin, dwb,
                          static_cast<float*>(slab), sp, (hipStream_t)stream),
                    "dn_deconv2x2_backward_weight");
}

dn_status dn_maxpool2x2_forward(const float* x, int N, int H, int W, int C, float* y, int y_stride,
                                int y_off, void* stream) {
  if (!x || !y) return fail(DN_ERR_ARG, "null argument");
  if ((H & 1) || (W & 1) || (C & 3) || (y_stride & 3) || (y_off & 3))
    return fail(DN_ERR_ARG, "H, W even and C, y_stride, y_off multiples of 4 required");
  return hip_status(launch_pool_fwd(x, N, H, W, C, y, y_stride, y_off, (hipStream_t)stream),
                    "dn_maxpool2x2_forward");
}

dn_status dn_maxpool2x2_backward(const float* x, int N, int H, int W, int C, const float* dy,
                                 int dy_stride, int dy_off, int act, float* dx, void* stream) {
  if (!x || !dy || !dx) return fail(DN_ERR_ARG, "null argument");
  if ((H & 1) || (W & 1) || (C & 3) || (dy_stride & 3) || (dy_off & 3))
    return fail(DN_ERR_ARG, "H, W even and C, dy_stride, dy_off multiples of 4 required");
  return hip_status(launch_pool_bwd(x, N, H, W, C, dy, dy_stride, dy_off, act, dx,
                                    (hipStream_t)stream),
                    "dn_maxpool2x2_backward");
}

// ---- adapter finetune (adapter.py:5-67, finetune.py:153-162) ---------------------------------
dn_status dn_adapter_param_count(int in_channels, int hidden_channels, size_t* count) {
  if (!count) return fail(DN_ERR_ARG, "null argument");
  if (hidden_channels != 16) return fail(DN_ERR_ARG, "hidden_channels must be 16 (adapter.py default)");
  const long n = adapter_param_count(in_channels);
  if (n < 0) return fail(DN_ERR_ARG, "in_channels must be 1 or 3");
  *count = (size_t)n;
  return DN_OK;
}

static dn_status adapter_args(int N, int C, int H, int W, int hidden) {
  if (hidden != 16) return fail(DN_ERR_ARG, "hidden_channels must be 16 (adapter.py default)");
  if (C != 1 && C != 3) return fail(DN_ERR_ARG, "in_channels must be 1 or 3");
  if (N < 1 || H < 1 || W < 1) return fail(DN_ERR_ARG, "empty adapter input");
  return DN_OK;
}

size_t dn_adapter_slab_size(int N, int C, int H, int W, int hidden_channels) {
  if (hidden_channels != 16 || adapter_param_count(C) < 0 || N < 1 || H < 1 || W < 1) return 0;
  return sizeof(float) * (size_t)adapter_bwd_blocks(N, H, W) * (size_t)adapter_param_count(C);
}

dn_status dn_adapter_forward(const float* params, const float* noisy, const float* base_out,
                             float* out, int N, int C, int H, int W, int hidden_channels,
                             void* stream) {
  if (!params || !noisy || !base_out || !out) return fail(DN_ERR_ARG, "null argument");
  if (dn_status st = adapter_args(N, C, H, W, hidden_channels)) return st;
  return hip_status(launch_adapter_fwd(params, noisy, base_out, N, C, H, W, out, (hipStream_t)stream),
                    "dn_adapter_forward");
}

dn_status dn_adapter_backward(const float* params, const float* noisy, const float* base_out,
                              const float* dout, float* dparams, int N, int C, int H, int W,
                              int hidden_channels, void* slab, size_t slab_bytes, void* stream) {
  if (!params || !noisy || !base_out || !dout || !dparams || !slab)
    return fail(DN_ERR_ARG, "null argument");
  if (dn_status st = adapter_args(N, C, H, W, hidden_channels)) return st;
  if (slab_bytes < dn_adapter_slab_size(N, C, H, W, hidden_channels))
    return fail(DN_ERR_WORKSPACE, "slab smaller than dn_adapter_slab_size()");
  return hip_status(launch_adapter_bwd(params, noisy, base_out, dout, N, C, H, W, dparams,
                                       static_cast<float*>(slab), (hipStream_t)stream),
                    "dn_adapter_backward");
}

dn_status dn_finetune_loss(const float* pred, const float* target, int N, int C, int H, int W,
                           float lambda_grad, float* dpred, float* loss3, void* partial_ws,
                           void* stream) {
  if (!pred || !target || !dpred || !loss3 || !partial_ws) return fail(DN_ERR_ARG, "null argument");
  if (N < 1 || C < 1 || H < 2 || W < 2) return fail(DN_ERR_ARG, "gradient_loss needs H, W >= 2");
  return hip_status(launch_ft_loss(pred, target, N, C, H, W, lambda_grad, dpred, loss3, partial_ws,
                                   (hipStream_t)stream),
                    "dn_finetune_loss");
}

// ---- ImprovedUNet (arch_unet.py:421-531) ------------------------------------------------------
dn_status dn_iunet_param_count(const dn_unet_cfg* cfg, size_t* count) {
  DN_GUARD_BEGIN
  if (!cfg || !count) return fail(DN_ERR_ARG, "null argument");
  IParams P;
  std::string err;
  if (!iunet_build_params(*cfg, P, err)) return fail(DN_ERR_ARG, err);
  *count = (size_t)P.total;
  return DN_OK;
  DN_GUARD_END
}

dn_status dn_iunet_workspace_size(const dn_unet_cfg* cfg, int N, int H, int W, int with_backward,
                                  size_t* bytes) {
  DN_GUARD_BEGIN
  if (!cfg || !bytes) return fail(DN_ERR_ARG, "null argument");
  IPlan p;
  std::string err;
  if (!iunet_build_plan(*cfg, N, H, W, with_backward != 0, p, err)) return fail(DN_ERR_ARG, err);
  *bytes = (size_t)p.total_floats * sizeof(float);
  return DN_OK;
  DN_GUARD_END
}

dn_status dn_iunet_forward(const dn_unet_cfg* cfg, const float* params, const float* x, float* y,
                           int N, int H, int W, void* ws, size_t ws_bytes, void* stream) {
  return dn_iunet_forward_prec(cfg, params, x, y, N, H, W, ws, ws_bytes, DN_PREC_FP32, stream);
}

dn_status dn_iunet_forward_prec(const dn_unet_cfg* cfg, const float* params, const float* x,
                                float* y, int N, int H, int W, void* ws, size_t ws_bytes,
                                int precision, void* stream) {
  DN_GUARD_BEGIN
  if (precision != DN_PREC_FP32 && precision != DN_PREC_FP32_X6)
    return fail(DN_ERR_ARG, "ImprovedUNet precision must be DN_PREC_FP32 or DN_PREC_FP32_X6");
  if (!cfg || !params || !x || !y || !ws) return fail(DN_ERR_ARG, "null argument");
  IPlan p;
  std::string err;
  // the plan with the backward buffers has the same forward offsets: a workspace that large
  // makes the forward keep what the backward reads
  if (!iunet_build_plan(*cfg, N, H, W, true, p, err)) return fail(DN_ERR_ARG, err);
  if (ws_bytes < (size_t)p.total_floats * sizeof(float) &&
      !iunet_build_plan(*cfg, N, H, W, false, p, err))
    return fail(DN_ERR_ARG, err);
  if (ws_bytes < (size_t)p.total_floats * sizeof(float))
    return fail(DN_ERR_WORKSPACE, "workspace smaller than dn_iunet_workspace_size()");
  return iunet_forward(p, params, x, y, static_cast<float*>(ws), (hipStream_t)stream, precision);
  DN_GUARD_END
}

dn_status dn_iunet_backward(const dn_unet_cfg* cfg, const float* params, const float* dy,
                            float* dparams, int N, int H, int W, void* ws, size_t ws_bytes,
                            void* stream) {
  return dn_iunet_backward_prec(cfg, params, dy, dparams, N, H, W, ws, ws_bytes, DN_PREC_FP32,
                                stream);
}

dn_status dn_iunet_backward_prec(const dn_unet_cfg* cfg, const float* params, const float* dy,
                                 float* dparams, int N, int H, int W, void* ws, size_t ws_bytes,
                                 int precision, void* stream) {
  DN_GUARD_BEGIN
  if (precision != DN_PREC_FP32 && precision != DN_PREC_FP32_X6)
    return fail(DN_ERR_ARG, "ImprovedUNet precision must be DN_PREC_FP32 or DN_PREC_FP32_X6");
  if (!cfg || !params || !dy || !dparams || !ws) return fail(DN_ERR_ARG, "null argument");
  IPlan p;
  std::string err;
  if (!iunet_build_plan(*cfg, N, H, W, true, p, err)) return fail(DN_ERR_ARG, err);
  if (ws_bytes < (size_t)p.total_floats * sizeof(float))
    return fail(DN_ERR_WORKSPACE, "workspace smaller than dn_iunet_workspace_size(with_backward=1)");
  return iunet_backward(p, params, dy, dparams, static_cast<float*>(ws), (hipStream_t)stream,
                        precision);
  DN_GUARD_END
}

/* (offset_floats, channel_stride, level) of the main ImprovedUNet activations, in the order
   x0 h | per down level i: F r z1 a1 z2 | bottle: F r z1 a1 z2 | per up k: cc F r z1 a1 z2 | xb cf */
dn_status dn_iunet_debug_buffers(const dn_unet_cfg* cfg, int N, int H, int W, int with_backward,
                                 int64_t* desc, int max_entries, int* n_entries) {
  DN_GUARD_BEGIN
  if (!cfg || !desc || !n_entries) return fail(DN_ERR_ARG, "null argument");
  IPlan p;
  std::string err;
  if (!iunet_build_plan(*cfg, N, H, W, with_backward != 0, p, err)) return fail(DN_ERR_ARG, err);
  int n = 0;
  auto add = [&](long off, int stride, int level) {
    if (n < max_entries) {
      desc[3 * n] = off;
      desc[3 * n + 1] = stride;
      desc[3 * n + 2] = level;
    }
    ++n;
  };
  auto blk = [&](const IBlockBufs& b, int ch, int l) {
    add(b.F, ch + 128, l); add(b.r, ch, l); add(b.z1, ch, l); add(b.a1, ch, l); add(b.z2, ch, l);
  };
  add(p.x0, 4, 0); add(p.h, 48, 0);
  for (int i = 0; i < 4; ++i) blk(p.dl[i], 48 << i, i);
  blk(p.bb, 384, 4);
  for (int k = 0; k < 4; ++k) {
    const int out = p.P.up[k].out;
    add(p.cc[k], 3 * out, 3 - k);
    blk(p.ul[k], out, 3 - k);
  }
  add(p.xb, 384, 4); add(p.cf, 28, 0);
  if (with_backward) {  // | per down level: dr dz2 dg1 dz1 | per up k: dcc | dpool
    for (int i = 0; i < 4; ++i) {
      const int ch = 48 << i;
      add(p.dl[i].dr, ch, i); add(p.dl[i].dz2, ch, i); add(p.dl[i].dg1, ch, i);
      add(p.dl[i].dz1, ch, i);
    }
    for (int k = 0; k < 4; ++k) add(p.dcc[k], 3 * p.P.up[k].out, 3 - k);
  }
  *n_entries = n;
  return DN_OK;
  DN_GUARD_END
}

}  // extern "C"
