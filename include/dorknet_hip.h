/*
 * dorknet_hip.h -- C ABI of libdorknet_hip.so, the MI355X (gfx950) implementation of
 * Dorknet's convolution training hot path (reference: WJGiles/Dorknet).
 *
 * Conventions (every entry point):
 *   - pointers are DEVICE pointers owned by the caller; nothing here allocates;
 *   - activations are NHWC fp32 ([P][C] with P = N*H*W pixels, channels innermost);
 *   - scratch memory comes from a caller-provided workspace (ws, ws_bytes); each user of
 *     one has a matching *_workspace_bytes() query with the same shape arguments;
 *   - `stream` is a hipStream_t passed as void*; all work is stream-ordered on it;
 *   - the int return value is a hipError_t (0 = success); 10001 = bad arguments,
 *     10002 = workspace too small.  Nothing is checked on the device.  Exceptions: the
 *     count queries (*_blocks, *_rows, *_count, dk_abi_version, dk_debug_*) return a count;
 *   - reentrant: no global mutable state (except the dk_debug_* tuning knob).
 *
 * Each block cites the reference interface it replaces (file:line under the reference
 * repository).  In the reference these are CuPy RawKernel launches (NVRTC CUDA strings),
 * cuBLAS SGEMM through cp.dot, and CuPy elementwise / reduction kernels, called from the
 * Layer classes; here the Layer classes (dorknet_amd/layers/) call these entry points
 * through ctypes (dorknet_amd/_hip.py).  Parsed by dorknet_amd/_hip.py to declare the
 * ctypes prototypes: keep one declaration per statement, `int|size_t name(args);`.
 */
#ifndef DORKNET_HIP_H
#define DORKNET_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int dk_abi_version(void);

/* ---------------------------------------------------------------------------------------
 * Device-side input pipeline (dorknet_amd/csrc/input_pipeline.hip),
 * replacing the per-image CPU work of data_loading/image_preprocessor.py:16-39 and the mixup
 * of data_loading/image_data_loader.py:101-111 for a whole batch:
 *  - dk_resize_bilinear_u8: cv2.resize(im, (OW, OH)) INTER_LINEAR geometry (half-pixel centres,
 *    edge replication), fp32 interpolation rounded to nearest-even, uint8 NHWC in and out;
 *  - dk_u8_nhwc_to_nchw_f32: im[r:r+OH, c:c+OW, :].astype(float32).transpose(2,0,1) - shift for
 *    every image; crop_rc = device int32 [N][2] (row, col) offsets (NULL: 0, 0; clamped into the
 *    image); dst fp32 NCHW [N][C][OH][OW];
 *  - dk_mixup_f32: ab = p*b + (1-p)*a and ba = p*a + (1-p)*b elementwise, with p and 1-p
 *    passed as the fp32 values numpy multiplies by (X_batch = a, X_batch_m = b). */
int dk_resize_bilinear_u8(const uint8_t* src, int N, int H, int W, int C, int OH, int OW, uint8_t* dst, void* stream);
int dk_u8_nhwc_to_nchw_f32(const uint8_t* src, int N, int H, int W, int C, const int* crop_rc, int OH, int OW, float shift, float* dst, void* stream);
int dk_mixup_f32(const float* a, const float* b, long long n, float p, float one_minus_p, float* ab, float* ba, void* stream);

/* Path selectors and tuning knobs for tests and A/B runs (dorknet_amd/csrc/knobs.hip: one registry
 * of atomics holding built-in defaults; no environment variable reaches them; not for production
 * use).  cfg = -1 restores the default.  Returns the number of configurations for kinds 0 / 1, 0 for
 * the others, -1 for an unknown or retired kind (5, 12, 15-17, 20, 22).
 * kind 0 / 1: force GEMM tile configuration `cfg` for forward/dgrad problems / split-K
 * weight-gradient problems (-1 = the built-in heuristic);
 * kind 2: split-K grids sized to one round of resident blocks (1 = default) or the fixed ~1024-block
 * split (0);
 * kind 3: the streaming pointwise kernels for K = C = 64 / 128 (1 = default; 0 = the tiled engine for
 * every shape);
 * kind 4: nontemporal output stores, a bitmask over kernel families (NtFam in csrc/dk_common.h);
 * kind 7: blocks the fused stride-1 depthwise backward aims for (its batch is dealt into image runs
 * above that; 0 = one image per block; default 768);
 * kind 8: output rows per thread of the depthwise forward / stride-1 dgrad (-1 = the shape rule);
 * kind 9: the bf16 streaming pointwise kernels (1 = default; 0 = the tiled engine);
 * kind 11: the fp32 weight-stationary deep pointwise kernels (1 = default);
 * kind 13: the bf16 weight-stationary deep pointwise kernels (1 = default);
 * kind 14: the fused deep pointwise backward, dgrad + weight gradient in one pass (1 = default);
 * kind 18: blocks a split-K weight gradient aims for (default 1024);
 * kind 21: output columns per thread of the fused stride-1 depthwise backward (2 = default where the
 * width allows, 1 = one); the dk_dwconv_bwd_bnbwd*_stats_rows / _workspace_bytes follow it. */
int dk_debug_set_gemm_config(int kind, int cfg);

/* Bandwidth ceiling probe (not on the training path; scripts/stream_ceiling.py): reads nin
 * (1..3) fp32 arrays a, b, c and writes nout (0..2) arrays o0, o1 of numel elements each, 16
 * bytes per lane per access, on `blocks` blocks of 256 threads (<= 0: 2048); nout + 10 = the same
 * with nontemporal stores. */
int dk_debug_stream_mix(const float* a, const float* b, const float* c, float* o0, float* o1, int nin, int nout, long long numel, int blocks, void* stream);
/* Tuning knob (same caveats): launch variant of dk_bn_bwd_apply_f32 (bits 0-1: rows in flight
 * 4/8 x plain/nontemporal stores; bits 2-3: rows per lane 16/8/32/64; bit 4: block cap 16384);
 * -1 restores the default (22).  Returns the number of variants. */
int dk_debug_set_ew_variant(int v);

/* ---------------------------------------------------------------------------------------
 * Dense convolution, implicit GEMM on fp32 MFMA.
 * Replaces ConvLayer.forward GPU branch (layers/convolution.py:58-87: pad_input :144-151,
 * CUDA im2col :187-203, cp.dot :75) and ConvLayer.backward (:90-117: wgrad cp.dot :96,
 * l2 :99-100, dgrad cp.dot :104, CUDA row2im :205-222).
 * Weights stay in the reference layout W[K][C][R][S]; the *_krsc / *_crsk helpers produce
 * the GEMM-friendly copies (C padded to Cp, a multiple of 4, with zeros).
 * OH/OW are passed in: the caller computes them with the reference formula
 * int((H + 2*pad - R)/stride + 1) (convolution.py:67-68).
 * ------------------------------------------------------------------------------------- */
int dk_conv_weight_krsc_f32(const float* w_kcrs, int K, int C, int R, int S, int Cp, float* w_krsc, void* stream);
int dk_conv_weight_crsk_f32(const float* w_kcrs, int K, int C, int R, int S, float* w_crsk, void* stream);
int dk_conv2d_fwd_f32(const float* x, int N, int H, int W, int C, const float* w_krsc, int K, int R, int S, int stride, int pad, const float* bias, float* y, int OH, int OW, void* stream);
int dk_conv2d_dgrad_f32(const float* dy, int N, int OH, int OW, int K, const float* w_crsk, int C, int R, int S, int pad, float* dx, int H, int W, void* stream);
/* Strided dgrad without a column matrix (sub-pixel decomposition; conv_subpixel.hip), for
 * narrow inputs (C <= 16) and the instantiated (R, S, stride, pad) geometries: (5,5,2,1), (5,5,2,2),
 * (3,3,2,1), (4,4,2,1), (7,7,2,3), (3,3,2,0), (2,2,2,0) (replaces convolution.py:101-111 +
 * row2im :205-222).  The workspace query returns 0 when the geometry is not covered (use
 * dk_conv2d_dgrad_phase_f32). */
size_t dk_conv2d_dgrad_subpixel_workspace_bytes(int K, int C, int R, int S, int stride, int pad);
int dk_conv2d_dgrad_subpixel_f32(const float* dy, int N, int OH, int OW, int K, const float* w_kcrs, int C, int R, int S, int stride, int pad, float* dx, int H, int W, void* ws, size_t ws_bytes, void* stream);
/* Any-stride input gradient as one implicit GEMM per sub-pixel phase (no column matrix, no atomics;
 * replaces cp.dot(dy, W_flat) + row2im, layers/convolution.py:101-117, :205-222).  dy: NHWC with
 * Kp = K rounded up to 4 channels (zero-padded when K % 4 != 0); w_kcrs: the reference layout;
 * dx: NHWC (N, H, W, C).  Workspace: dk_conv2d_dgrad_phase_workspace_bytes(). */
size_t dk_conv2d_dgrad_phase_workspace_bytes(int K, int C, int R, int S, int stride);
int dk_conv2d_dgrad_phase_f32(const float* dy, int N, int OH, int OW, int Kp, int K, const float* w_kcrs, int C, int R, int S, int stride, int pad, float* dx, int H, int W, void* ws, size_t ws_bytes, void* stream);
size_t dk_conv2d_wgrad_workspace_bytes(int N, int OH, int OW, int K, int Cp, int R, int S);
int dk_conv2d_wgrad_f32(const float* dy, const float* x, int N, int H, int W, int Cp, int C, int K, int R, int S, int stride, int pad, int OH, int OW, const float* w_kcrs, float l2, float* dw_kcrs, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * Pointwise (1x1) convolution = the R=S=1 case of the GEMM engine.
 * Replaces PointwiseConvLayer.forward/backward (layers/pointwise_convolution.py:46-75):
 * the X[:, :, ::s, ::s] subsample (:48-49) is a strided gather, the NHWC transpose copy
 * (:50) disappears, and the stride-s backward widen (:68-72) is fused into dgrad.
 * Weights W[K][C] as in the reference.
 * ------------------------------------------------------------------------------------- */
int dk_pwconv_fwd_f32(const float* x, int N, int H, int W, int C, const float* w_kc, int K, int stride, const float* bias, float* y, int OH, int OW, void* stream);
int dk_pwconv_dgrad_f32(const float* dy, int N, int OH, int OW, int K, const float* w_kc, int C, int stride, float* dx, void* stream);
size_t dk_pwconv_wgrad_workspace_bytes(int N, int OH, int OW, int K, int C);
int dk_pwconv_wgrad_f32(const float* dy, const float* x, int N, int H, int W, int C, int K, int stride, int OH, int OW, const float* w_kc, float l2, float* dw_kc, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * "BN on load" variants (*_bnx_*): the input operand is bn(x) (+ReLU if bn_relu), computed
 * from the raw x of the layer before the BatchNormLayer as each tile is loaded, so the BN
 * output is never written to HBM.  Replaces the pair BatchNormLayer.forward (apply,
 * layers/batch_norm.py:91-96) [+ ReLu.forward, activations.py:37-42] -> consumer forward /
 * weight gradient; the values the consumer sees are bit-identical to dk_bn_apply_f32's
 * output (same bn_out arithmetic), and padding stays exactly 0.
 * bn_*: per-channel mean, 1/std, gamma, beta (C floats each, 16-byte aligned).
 * ------------------------------------------------------------------------------------- */
int dk_conv2d_fwd_bnx_f32(const float* x, int N, int H, int W, int C, const float* w_krsc, int K, int R, int S, int stride, int pad, const float* bias, float* y, int OH, int OW, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, void* stream);
/* Weight gradient with the following BatchNorm's backward applied as dy is loaded (g: the
 * gradient w.r.t. that BN's (+ReLU) output; bn_x: its raw input = this layer's output; out_* /
 * k12: its parameters and folded coefficients): dy = dk_bn_bwd_apply_f32(bn_x, g) bit for bit,
 * never stored.  Replaces dk_bn_bwd_apply_f32 -> dk_conv2d_wgrad[_bnx]_f32 for a layer whose
 * input gradient is not needed (the stem: feed_forward_network.py:64-70 drops it).  bn_* (optional):
 * this layer's input BatchNorm, as dk_conv2d_wgrad_bnx_f32.  Workspace: dk_conv2d_wgrad_workspace_bytes. */
int dk_conv2d_wgrad_bnbwd_f32(const float* g, const float* bn_x, const float* x, int N, int H, int W, int Cp, int C, int K, int R, int S, int stride, int pad, int OH, int OW, const float* out_mean, const float* out_invstd, const float* out_gamma, const float* out_beta, int out_relu, const float* k12, const float* w_kcrs, float l2, float* dw_kcrs, void* ws, size_t ws_bytes, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, void* stream);
int dk_conv2d_wgrad_bnx_f32(const float* dy, const float* x, int N, int H, int W, int Cp, int C, int K, int R, int S, int stride, int pad, int OH, int OW, const float* w_kcrs, float l2, float* dw_kcrs, void* ws, size_t ws_bytes, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, void* stream);
int dk_pwconv_fwd_bnx_f32(const float* x, int N, int H, int W, int C, const float* w_kc, int K, int stride, const float* bias, float* y, int OH, int OW, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, void* stream);
int dk_pwconv_wgrad_bnx_f32(const float* dy, const float* x, int N, int H, int W, int C, int K, int stride, int OH, int OW, const float* w_kc, float l2, float* dw_kc, void* ws, size_t ws_bytes, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, void* stream);
/* Narrow-input convolution (dorknet_amd/csrc/conv_narrow.hip): the stem -- conv0, 64 x 3 x 5 x 5
 * stride 2 on the NCHW image (convolution.py:58-100, examples/imagenet_dogs_225_resnet_18_depsep.py
 * :112-116) -- forward and weight gradient read the NCHW input directly (no NHWC copy, no channel
 * padding: the reduction is k = (c, r, s), the reference's KCRS order, padded only to 4).
 * dk_conv2d_narrow_preferred: 1 when these entry points take the shape (C <= 4, K % 4 == 0,
 * K <= 64, R, S <= 7, C*R*S <= 160, stride <= 2, st*(16*ceil(OW/16) - 1) + S <= 256).
 * dk_conv2d_fwd_narrow_f32: y NHWC; bias optional; stats (optional) = the output BatchNorm's
 * partial rows [dk_conv2d_fwd_narrow_stats_rows()][2][K] (in-launch fold: dk_bn_fold_arm_stats).
 * dk_conv2d_wgrad_narrow_f32 / _bnbwd_narrow_f32: as dk_conv2d_wgrad_f32 /
 * dk_conv2d_wgrad_bnbwd_f32 (dy given, or formed on load from the following BatchNorm's
 * deferred gradient), x NCHW; workspace: dk_conv2d_wgrad_narrow_workspace_bytes.  g_lattice = 2: g is
 * given compact on the even (oh, ow) lattice only ([N][ceil(OH/2)][ceil(OW/2)][K], zero elsewhere: the
 * un-widened gradient of a following stride-2 pointwise layer, dk_pwconv_dgrad_lattice_f32); 1: dense. */
int dk_conv2d_narrow_preferred(int N, int C, int H, int W, int K, int R, int S, int stride, int pad, int OH, int OW);
int dk_conv2d_fwd_narrow_stats_rows(int N, int C, int H, int W, int K, int R, int S, int stride, int pad, int OH, int OW);
int dk_conv2d_fwd_narrow_f32(const float* x_nchw, int N, int C, int H, int W, const float* w_kcrs, int K, int R, int S, int stride, int pad, const float* bias, float* y, int OH, int OW, double* stats, void* stream);
size_t dk_conv2d_wgrad_narrow_workspace_bytes(int N, int C, int H, int W, int K, int R, int S, int stride, int pad, int OH, int OW);
int dk_conv2d_wgrad_narrow_f32(const float* dy, const float* x_nchw, int N, int C, int H, int W, int K, int R, int S, int stride, int pad, int OH, int OW, const float* w_kcrs, float l2, float* dw_kcrs, void* ws, size_t ws_bytes, void* stream);
int dk_conv2d_wgrad_bnbwd_narrow_f32(const float* g, const float* bn_x, const float* x_nchw, int N, int C, int H, int W, int K, int R, int S, int stride, int pad, int OH, int OW, const float* out_mean, const float* out_invstd, const float* out_gamma, const float* out_beta, int out_relu, const float* k12, int g_lattice, const float* w_kcrs, float l2, float* dw_kcrs, void* ws, size_t ws_bytes, void* stream);
/* Producer side of the same fusion: *_fwd_ex_f32 = forward with an optional input BN
 * (bn_mean == NULL: raw input) and, when stats != NULL, the BatchNorm statistics of the
 * output y (fp64 sum and sum of squares per output channel, per tile: stats[rows][2][K],
 * rows = the matching *_fwd_stats_rows()).  dk_bn_stats_from_partials_f32 turns them into
 * mean/std -- the separate statistics pass over y (batch_norm.py:76-80) disappears.
 * dk_dwconv_fwd_stats_rows returns 0 when C/4 does not divide 256 (no statistics variant).
 * dk_dwconv_fwd_ex_f32 takes the filters in the reference layout W[C][R][S] (no re-layout). */
int dk_conv2d_fwd_stats_rows(int N, int OH, int OW, int K, int C, int R, int S);
int dk_conv2d_fwd_ex_f32(const float* x, int N, int H, int W, int C, const float* w_krsc, int K, int R, int S, int stride, int pad, const float* bias, float* y, int OH, int OW, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* stats, void* stream);
int dk_pwconv_fwd_stats_rows(int N, int OH, int OW, int K, int C);
int dk_pwconv_fwd_ex_f32(const float* x, int N, int H, int W, int C, const float* w_kc, int K, int stride, const float* bias, float* y, int OH, int OW, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* stats, void* stream);
int dk_dwconv_fwd_stats_rows(int N, int OH, int OW, int C, int stride);
/* The same for dk_dwconv_fwd_ex_bf16 (whole output columns per thread: fewer blocks, fewer rows). */
int dk_dwconv_fwd_bf16_stats_rows(int N, int OH, int OW, int C, int stride);
int dk_dwconv_fwd_ex_f32(const float* x, int N, int H, int W, int C, const float* w_crs, int R, int S, int stride, int pad, const float* bias, float* y, int OH, int OW, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* stats, void* stream);
/* Depthwise forward whose input is a residual block's output y = ReLU(bnA(a) + bnB(b))
 * (residual_block.py:75; the operands of dk_bn_add_f32, bnX = identity when its mean is NULL): the
 * join is formed as the window rows are loaded and stored once into y_join (+ its ReLU mask, uint8,
 * nullable) -- bit-identical to dk_bn_add_f32 -- and the depthwise output / statistics are those of
 * dk_dwconv_fwd_ex_f32 on y_join.  3 x 3, pad 1, stride 1 or 2, fp32, C % 4 == 0.  Replaces the
 * separate join pass + this layer's re-read of its output. */
int dk_dwconv_fwd_join_f32(const float* a, const float* a_mean, const float* a_invstd, const float* a_gamma, const float* a_beta, int a_relu, const float* b, const float* b_mean, const float* b_invstd, const float* b_gamma, const float* b_beta, int b_relu, float* y_join, uint8_t* mask, int N, int H, int W, int C, const float* w_crs, int stride, const float* bias, float* y, int OH, int OW, double* stats, void* stream);
/* Backward side: *_dgrad_ex_f32 = the input gradient plus stage 1 of the backward of the
 * BatchNorm whose output this layer consumed (the BN-on-load input of its forward): with
 * g = dx masked by that BN's fused ReLU (recomputed from bn_x, the BN's raw input, laid out
 * like dx), part[rows][2][C] = per-tile (sum g, sum g * x_hat) -- what dk_bn_bwd_partial_f64
 * computes in a separate pass over x and dx (batch_norm.py:125-174).  Consume with
 * dk_bn_bwd_from_partials_f32.  dk_dwconv_dgrad_stats_rows returns 0 (no fused variant)
 * unless stride == 1 and C/4 divides 256.  The dgrad_ex entries also take an optional
 * `residual` addend (dx = dgrad + residual: the residual join's other gradient term,
 * residual_block.py:94-97; NULL = none) and make the BN part optional (bn_x == NULL). */
int dk_pwconv_dgrad_stats_rows(int N, int OH, int OW, int K, int C);
int dk_pwconv_dgrad_ex_f32(const float* dy, int N, int OH, int OW, int K, const float* w_kc, int C, int stride, float* dx, const float* residual, const float* bn_x, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* part, void* stream);
/* dk_pwconv_dgrad_ex_f32 (with the input BN's partials) for stride > 1, the widened gradient kept
 * compact: dx_lat[n][oh][ow][c] = the widened dx (pointwise_convolution.py:68-72) at (n, s*oh, s*ow, c);
 * every other point of the widened grid is zero and is neither written nor handed on (the
 * consumer is dk_conv2d_wgrad_bnbwd_narrow_f32 with g_lattice = 2).  Rows: dk_pwconv_dgrad_stats_rows. */
int dk_pwconv_dgrad_lattice_f32(const float* dy, int N, int OH, int OW, int K, const float* w_kc, int C, int stride, float* dx_lat, const float* bn_x, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* part, void* stream);
int dk_dwconv_dgrad_stats_rows(int N, int H, int W, int C, int stride);
int dk_dwconv_dgrad_ex_f32(const float* dy, int N, int OH, int OW, int C, const float* w_crs, int R, int S, int stride, int pad, float* dx, int H, int W, void* ws, size_t ws_bytes, const float* residual, const float* bn_x, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* part, void* stream);
/* The other side of the same BatchNorm pair: *_dgrad_bnbwd_f32 = a stride-1 layer's input
 * gradient when its OUTPUT fed a BatchNorm (+ReLU).  g is the gradient w.r.t. that BN's
 * output, bn_x its raw input (= this layer's output), out_* its parameters and k12 its
 * folded backward coefficients (dk_bn_bwd_from_partials_f32).  The layer's gradient
 * dy = dk_bn_bwd_apply_f32(bn_x, g) is formed as the operand is loaded (stage 3 of
 * batch_norm.py:125-174) and, when dy_out != NULL, also stored there (bit-identical to the
 * separate pass) for the layer's weight gradient.  The remaining arguments are those of the
 * matching *_dgrad_ex_f32 (x / bn_* / part: the BN before this layer; residual addend).
 * (No depthwise form: that dgrad is HBM-bound, and forming dy on load costs it more than
 * the separate apply pass saves -- measured, DESIGN.md.) */
int dk_pwconv_dgrad_bnbwd_stats_rows(int N, int OH, int OW, int K, int C);
int dk_pwconv_dgrad_bnbwd_f32(const float* g, const float* bn_x, int N, int OH, int OW, int K, const float* out_mean, const float* out_invstd, const float* out_gamma, const float* out_beta, int out_relu, const float* k12, float* dy_out, const float* w_kc, int C, float* dx, const float* residual, const float* x, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* part, void* stream);
/* Fused stride-1 pointwise backward (dorknet_amd/csrc/pw_bwd_fused.hip), replacing
 * dk_pwconv_dgrad_bnbwd_f32 + dk_pwconv_wgrad_bnx_f32 (pointwise_convolution.py:57-75 with the
 * following BatchNorm's backward, batch_norm.py:125-174, applied as dy is formed): one pass
 * reads g, bn_x (the following BN's raw input) and x (this layer's raw input) and writes dx
 * (+ residual), the weight gradient dw_kc = dy^T . bn_in(x) + l2 * w_kc (fixed-order reduce of
 * per-block partials in ws) and, when part != NULL, the input BN's backward partials
 * part[rows][2][C], rows = dk_pwconv_bwd_fused_rows().  dy itself is never stored.
 * K, C in {64, 128}, or K in {128, 256} with C a multiple of 128 (the weight-stationary deep kernel;
 * dk_pwconv_bwd_fused_rows() returns 0 for other shapes); fp32 NHWC.  At the deep kernel's shapes an
 * input BN (bn_*) must come with its partials (part), else DK_ERR_ARGS. */
int dk_pwconv_bwd_fused_rows(int N, int OH, int OW, int K, int C);
/* 1 when the fused backward is the faster path for the shape (K = C = 64: the streaming kernel;
 * the layers then take it by default), else 0. */
int dk_pwconv_bwd_fused_preferred(int N, int OH, int OW, int K, int C);
size_t dk_pwconv_bwd_fused_workspace_bytes(int N, int OH, int OW, int K, int C);
/* The stride-s form for the compact-lattice input gradient (pointwise_convolution.py:57-75 with
 * the widen's zeros never stored; dk_pwconv_dgrad_lattice_f32's output): one pass over the N x OH x OW
 * output pixels, x = the layer input N x H x W x C read at the stride-s lattice with its BatchNorm
 * (bn_*, required) applied on load, dx compact N x OH x OW x C, part (optional) that BN's partials,
 * dk_pwconv_bwd_fused_rows(N, OH, OW, K, C) rows.  K = C = 64. */
int dk_pwconv_bwd_bnbwd_lattice_f32(const float* g, const float* bn_x, int N, int OH, int OW, int K, const float* out_mean, const float* out_invstd, const float* out_gamma, const float* out_beta, int out_relu, const float* k12, const float* w_kc, int C, float l2, float* dw_kc, float* dx, const float* x, int H, int W, int stride, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* part, void* ws, size_t ws_bytes, void* stream);
int dk_pwconv_bwd_bnbwd_f32(const float* g, const float* bn_x, int N, int OH, int OW, int K, const float* out_mean, const float* out_invstd, const float* out_gamma, const float* out_beta, int out_relu, const float* k12, const float* w_kc, int C, float l2, float* dw_kc, float* dx, const float* residual, const float* x, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* part, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * bf16 storage twins (BASELINE config 5: the depthwise-separable stack with bf16 activations).
 * Same contracts as the _f32 entries above, except that every activation / activation-
 * gradient tensor (x, y, dy, dx, bn_x, residual) is bf16 (raw uint16_t bits, NHWC, C % 4 == 0);
 * weights, biases, BatchNorm parameters / statistics and weight gradients stay fp32, and all
 * arithmetic is fp32 (bf16 -> fp32 on load; fp32 -> bf16 round-to-nearest-even on store, the
 * BatchNorm statistics / partials are taken over the rounded stored values).  Reference:
 * the same layer methods as the _f32 twins (depthwise_convolution.py:85-102, :198-221;
 * pointwise_convolution.py:46-75; batch_norm.py:54-174), which compute in fp32 throughout.
 * ------------------------------------------------------------------------------------- */
int dk_cast_f32_to_bf16(const float* x, long long n, uint16_t* y, void* stream);
int dk_cast_bf16_to_f32(const uint16_t* x, long long n, float* y, void* stream);
int dk_bn_stats_bf16(const uint16_t* x, int P, int C, float eps, float momentum, int first, float* mean, float* std_, float* invstd, float* run_mean, float* run_std, void* ws, size_t ws_bytes, void* stream);
int dk_bn_apply_bf16(const uint16_t* x, long long numel, int C, const float* mean, const float* invstd, const float* gamma, const float* beta, int relu, uint16_t* y, uint8_t* mask, void* stream);
int dk_bn_bwd_apply_bf16(const uint16_t* x, const uint16_t* dy, long long numel, int C, const float* mean, const float* invstd, const float* gamma, const float* beta, int relu, const float* k12, uint16_t* dx, void* stream);
int dk_bn_bwd_bf16(const uint16_t* x, const uint16_t* dy, int P, int C, const float* mean, const float* invstd, const float* gamma, const float* beta, int relu, float* dgamma, float* dbeta, uint16_t* dx, void* ws, size_t ws_bytes, void* stream);
int dk_relu_fwd_bf16(const uint16_t* x, long long n, uint16_t* y, uint8_t* mask, void* stream);
int dk_relu_bwd_bf16(const uint16_t* dy, const uint8_t* mask, long long n, uint16_t* dx, void* stream);
int dk_pwconv_fwd_bf16_stats_rows(int N, int OH, int OW, int K, int C);
int dk_pwconv_fwd_ex_bf16(const uint16_t* x, int N, int H, int W, int C, const float* w_kc, int K, int stride, const float* bias, uint16_t* y, int OH, int OW, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* stats, void* stream);
int dk_pwconv_dgrad_ex_bf16(const uint16_t* dy, int N, int OH, int OW, int K, const float* w_kc, int C, int stride, uint16_t* dx, const uint16_t* residual, const uint16_t* bn_x, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* part, void* stream);
int dk_pwconv_wgrad_bnx_bf16(const uint16_t* dy, const uint16_t* x, int N, int H, int W, int C, int K, int stride, int OH, int OW, const float* w_kc, float l2, float* dw_kc, void* ws, size_t ws_bytes, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, void* stream);
int dk_dwconv_fwd_ex_bf16(const uint16_t* x, int N, int H, int W, int C, const float* w_crs, int R, int S, int stride, int pad, const float* bias, uint16_t* y, int OH, int OW, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* stats, void* stream);
int dk_dwconv_dgrad_ex_bf16(const uint16_t* dy, int N, int OH, int OW, int C, const float* w_crs, int R, int S, int stride, int pad, uint16_t* dx, int H, int W, void* ws, size_t ws_bytes, const uint16_t* residual, const uint16_t* bn_x, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* part, void* stream);

/* BatchNorm-backward-on-load fusions for bf16 storage (as dk_pwconv_dgrad_bnbwd_f32 and
 * dk_dwconv_bwd_bnbwd_f32; reference layers/pointwise_convolution.py:57-75,
 * layers/depthwise_convolution.py:198-221, layers/batch_norm.py:125-174): dy is formed in fp32
 * from the following BN's gradient g and input bn_x; the pointwise dgrad rounds it to bf16 as its
 * MFMA operand and as written to dy_out; the depthwise backward keeps it fp32. */
int dk_pwconv_dgrad_bnbwd_bf16_stats_rows(int N, int OH, int OW, int K, int C);
int dk_pwconv_dgrad_bnbwd_bf16(const uint16_t* g, const uint16_t* bn_x, int N, int OH, int OW, int K, const float* out_mean, const float* out_invstd, const float* out_gamma, const float* out_beta, int out_relu, const float* k12, uint16_t* dy_out, const float* w_kc, int C, uint16_t* dx, const uint16_t* residual, const uint16_t* x, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* part, void* stream);
/* Fused pointwise backward for bf16 storage (the twin of dk_pwconv_bwd_bnbwd_f32; BASELINE config 5's
 * 56 x 56 units, K = C = 64, stride 1): dx as dk_pwconv_dgrad_bnbwd_bf16 (bit-identical) plus the
 * weight gradient dW = dy^T bn_relu(x) + l2 w (fp32, bf16 MFMA operands: dy as the dgrad rounds it,
 * bn_relu(x) rounded to bf16) in one pass; dy is never stored.  Replaces the dgrad + the separate
 * weight gradient (layers/pointwise_convolution.py:57-75).  *_rows: the partial rows of part (0 = shape
 * not taken); the workspace holds that many fp32 [K][C] weight-gradient partial rows. */
int dk_pwconv_bwd_fused_bf16_rows(int N, int OH, int OW, int K, int C);
size_t dk_pwconv_bwd_fused_bf16_workspace_bytes(int N, int OH, int OW, int K, int C);
int dk_pwconv_bwd_bnbwd_bf16(const uint16_t* g, const uint16_t* bn_x, int N, int OH, int OW, int K, const float* out_mean, const float* out_invstd, const float* out_gamma, const float* out_beta, int out_relu, const float* k12, const float* w_kc, int C, float l2, float* dw_kc, uint16_t* dx, const uint16_t* residual, const uint16_t* x, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* part, void* ws, size_t ws_bytes, void* stream);
int dk_dwconv_bwd_bnbwd_bf16(const uint16_t* g, const uint16_t* bn_x, int N, int H, int W, int C, const float* out_mean, const float* out_invstd, const float* out_gamma, const float* out_beta, int out_relu, const float* k12, const uint16_t* x, const float* w_crs, int R, int S, int pad, float l2, float* dw_crs, uint16_t* dx, const uint16_t* residual, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* part, void* ws, size_t ws_bytes, void* stream);
/* rows / workspace of dk_dwconv_bwd_bnbwd_bf16 (its block geometry: two output columns per thread
 * where the width allows, knob 21) */
int dk_dwconv_bwd_bnbwd_bf16_stats_rows(int N, int H, int W, int C);
size_t dk_dwconv_bwd_bnbwd_bf16_workspace_bytes(int N, int H, int W, int C, int R, int S);
int dk_dwconv_wgrad_bnx_bf16(const uint16_t* dy, const uint16_t* x, int N, int H, int W, int C, int R, int S, int stride, int pad, int OH, int OW, const float* w_crs, float l2, float* dw_crs, void* ws, size_t ws_bytes, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, void* stream);

/* ---------------------------------------------------------------------------------------
 * Depthwise convolution, direct (no MFMA).
 * Replaces DepthwiseConvLayer.forward_cp (layers/depthwise_convolution.py:85-102, CUDA
 * forward_conv :105-121) and backward_cp (:198-221, CUDA backward_conv :122-140).
 * Weights W[C][R][S] as in the reference; dk_dw_weight_rsc_f32 makes the [R][S][C] copy
 * the forward kernel reads (dgrad takes W[C][R][S] and re-lays it out in its workspace).
 * R x S in {1x1, 3x3, 5x5}; stride 1 or 2 for forward / wgrad.
 * ------------------------------------------------------------------------------------- */
int dk_dw_weight_rsc_f32(const float* w_crs, int C, int R, int S, float* w_rsc, void* stream);
int dk_dwconv_fwd_f32(const float* x, int N, int H, int W, int C, const float* w_rsc, int R, int S, int stride, int pad, const float* bias, float* y, int OH, int OW, void* stream);
size_t dk_dwconv_dgrad_workspace_bytes(int C, int R, int S);
int dk_dwconv_dgrad_f32(const float* dy, int N, int OH, int OW, int C, const float* w_crs, int R, int S, int stride, int pad, float* dx, int H, int W, void* ws, size_t ws_bytes, void* stream);
size_t dk_dwconv_wgrad_workspace_bytes(int N, int OH, int OW, int C, int R, int S);
int dk_dwconv_wgrad_f32(const float* dy, const float* x, int N, int H, int W, int C, int R, int S, int stride, int pad, int OH, int OW, const float* w_crs, float l2, float* dw_crs, void* ws, size_t ws_bytes, void* stream);
/* BN-on-load variants (see the *_bnx_* note after the pointwise block). */
int dk_dwconv_fwd_bnx_f32(const float* x, int N, int H, int W, int C, const float* w_rsc, int R, int S, int stride, int pad, const float* bias, float* y, int OH, int OW, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, void* stream);
int dk_dwconv_wgrad_bnx_f32(const float* dy, const float* x, int N, int H, int W, int C, int R, int S, int stride, int pad, int OH, int OW, const float* w_crs, float l2, float* dw_crs, void* ws, size_t ws_bytes, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, void* stream);
/* Fused stride-1 depthwise backward for a layer whose OUTPUT fed a BatchNorm (+ReLU): replaces
 * dk_bn_bwd_apply_f32 -> dk_dwconv_dgrad_ex_f32 + dk_dwconv_wgrad_bnx_f32 (batch_norm.py:125-174
 * stage 3; depthwise_convolution.py:198-221 backward_cp) with one pass.  g: gradient w.r.t. that
 * BN's output; bn_x: its raw input (= this layer's output, N x H x W x C: stride 1, same size as
 * the input); out_* / k12: its parameters and folded coefficients.  dy is formed as it is loaded
 * and never stored.  x: this layer's stored input, with bn_* its input BatchNorm applied on load
 * (bn_mean NULL: none); part (NULL: none; needs bn_*): that input BN's backward partial sums,
 * dk_dwconv_bwd_bnbwd_stats_rows rows [rows][2][C] (fp64).  dx NULL: weight gradient only.
 * dw_crs = weight gradient (+ l2 * w_crs).  3x3 filters, pad 1, C % 4 == 0.  dx is bit-identical
 * to the unfused sequence; part and dw_crs differ from it by summation order only. */
int dk_dwconv_bwd_bnbwd_stats_rows(int N, int H, int W, int C);
size_t dk_dwconv_bwd_bnbwd_workspace_bytes(int N, int H, int W, int C, int R, int S);
int dk_dwconv_bwd_bnbwd_f32(const float* g, const float* bn_x, int N, int H, int W, int C, const float* out_mean, const float* out_invstd, const float* out_gamma, const float* out_beta, int out_relu, const float* k12, const float* x, const float* w_crs, int R, int S, int pad, float l2, float* dw_crs, float* dx, const float* residual, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* part, void* ws, size_t ws_bytes, void* stream);
/* dk_dwconv_bwd_bnbwd_f32 for a layer whose input is a residual block's output ReLU(bn_j(join_x) + skip)
 * (residual_block.py:75, no input BN): dx = (dgrad + residual) * join_mask -- the join's ReLU backward
 * (activations.py:44-47) -- and part (dk_dwconv_bwd_bnbwd_stats_rows x 2 x C) = stage 1 of bn_j's
 * backward over that dx (batch_norm.py:125-147), replacing dk_relu_bwd_bn_partial_f64's pass over it.
 * join_mask may be NULL when x IS the join's output: the mask is then x > 0 (bit-identical to the
 * stored one, y = max(v, 0) > 0 iff v > 0) and is not read.
 * Takes an in-launch fold arming (dk_bn_fold_arm_bwd). */
int dk_dwconv_bwd_bnbwd_join_f32(const float* g, const float* bn_x, int N, int H, int W, int C, const float* out_mean, const float* out_invstd, const float* out_gamma, const float* out_beta, int out_relu, const float* k12, const float* x, const float* w_crs, int R, int S, int pad, float l2, float* dw_crs, float* dx, const float* residual, const uint8_t* join_mask, const float* join_x, const float* join_mean, const float* join_invstd, double* part, void* ws, size_t ws_bytes, void* stream);
/* The strided (sub-pixel) depthwise input gradient with the same join fusion (the first layer of a
 * downsampling residual block); rows: dk_dwconv_dgrad_join_rows (0 = no join variant for the geometry).
 * residual_lattice = stride: the residual is the skip projection's un-widened gradient, compact on the
 * stride lattice ([N][ceil(H/s)][ceil(W/s)][C], zero elsewhere); 0: dense [N][H][W][C]. */
int dk_dwconv_dgrad_join_rows(int N, int H, int W, int C, int R, int S, int stride, int pad);
/* Fused stride-2 depthwise backward (3x3, pad 1): dk_dwconv_bwd_bnbwd_f32's one pass for a stride-2
 * layer (replaces dk_bn_bwd_apply -> dk_dwconv_dgrad_ex + dk_dwconv_wgrad_bnx; batch_norm.py:125-174
 * stage 3, depthwise_convolution.py:198-221).  g / bn_x: the following BN's output gradient and raw
 * input, N x OH x OW x C (OH = ceil(H / 2), OW = ceil(W / 2)); x: this layer's input N x H x W x C
 * with bn_* applied on load (bn_mean NULL: none); dx (NULL: weight gradient only) = dgrad
 * (+ residual); part (needs bn_*): that input BN's backward partials, dk_dwconv_bwd_s2_stats_rows
 * rows [rows][2][C].  C / 4 must divide 256.  dx is bit-identical to the unfused sequence (fp32). */
int dk_dwconv_bwd_s2_stats_rows(int N, int H, int W, int C);
size_t dk_dwconv_bwd_s2_workspace_bytes(int N, int H, int W, int C);
int dk_dwconv_bwd_s2_bnbwd_f32(const float* g, const float* bn_x, int N, int H, int W, int C, int OH, int OW, const float* out_mean, const float* out_invstd, const float* out_gamma, const float* out_beta, int out_relu, const float* k12, const float* x, const float* w_crs, float l2, float* dw_crs, float* dx, const float* residual, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* part, void* ws, size_t ws_bytes, void* stream);
/* The join form (fp32): x = a residual block's output y = ReLU(bn_j(join_x) + skip) (no input BN):
 * dx = (dgrad + residual) * (y > 0), part (required) = stage 1 of bn_j's backward over dx;
 * residual_lattice 2: the residual is the compact stride-2 lattice N x OH x OW x C (0: dense). */
int dk_dwconv_bwd_s2_bnbwd_join_f32(const float* g, const float* bn_x, int N, int H, int W, int C, int OH, int OW, const float* out_mean, const float* out_invstd, const float* out_gamma, const float* out_beta, int out_relu, const float* k12, const float* x, const float* w_crs, float l2, float* dw_crs, float* dx, const float* residual, int residual_lattice, const float* join_x, const float* join_mean, const float* join_invstd, double* part, void* ws, size_t ws_bytes, void* stream);
int dk_dwconv_bwd_s2_bnbwd_bf16(const uint16_t* g, const uint16_t* bn_x, int N, int H, int W, int C, int OH, int OW, const float* out_mean, const float* out_invstd, const float* out_gamma, const float* out_beta, int out_relu, const float* k12, const uint16_t* x, const float* w_crs, float l2, float* dw_crs, uint16_t* dx, const uint16_t* residual, const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu, double* part, void* ws, size_t ws_bytes, void* stream);
int dk_dwconv_dgrad_join_f32(const float* dy, int N, int OH, int OW, int C, const float* w_crs, int R, int S, int stride, int pad, float* dx, int H, int W, void* ws, size_t ws_bytes, const float* residual, int residual_lattice, const uint8_t* join_mask, const float* join_x, const float* join_mean, const float* join_invstd, double* part, void* stream);

/* ---------------------------------------------------------------------------------------
 * Dense layer (layers/dense_layer.py:46-67; W stored (in, out) as the reference).
 * ------------------------------------------------------------------------------------- */
int dk_dense_fwd_f32(const float* x, int B, int IN, const float* w_io, int OUT, const float* bias, float* y, void* stream);
int dk_dense_dgrad_f32(const float* dy, int B, int OUT, const float* w_io, int IN, float* dx, void* stream);
size_t dk_dense_wgrad_workspace_bytes(int B, int IN, int OUT);
int dk_dense_wgrad_f32(const float* x, const float* dy, int B, int IN, int OUT, const float* w_io, float l2, float* dw_io, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * Batch norm, training mode with batch statistics (layers/batch_norm.py:54-174).
 * Forward: partial sums -> (optional SyncBN all-reduce of the collapsed [2][C] sums) ->
 * finalize (mean, std, invstd, running mean/std as batch_norm.py:76-89) -> apply
 * (gamma*x_hat + beta, optionally fused with the following ReLU, activations.py:37-42).
 * Backward: partials of (sum dy, sum dy*x_hat) -> finalize (dgamma, dbeta from the local
 * sums, the dx coefficients k12 = [k1[C], k2[C]] from the global sums) -> apply.
 * Partial buffers are fp64 [nblk][2][C], nblk = dk_bn_partial_blocks(P, C).
 * ------------------------------------------------------------------------------------- */
int dk_bn_partial_blocks(int P, int C);
size_t dk_bn_workspace_bytes(int P, int C);
size_t dk_bn_bwd_workspace_bytes(int P, int C);
int dk_bn_stats_partial_f64(const float* x, int P, int C, void* ws, size_t ws_bytes, void* stream);
int dk_bn_collapse_f64(const void* part, int nblk, int C, void* out, void* stream);
int dk_bn_stats_finalize_f32(const void* part, int nblk, int C, double count, float eps, float momentum, int first, float* mean, float* std_, float* invstd, float* run_mean, float* run_std, void* stream);
size_t dk_bn_stats_workspace_bytes(int P, int C);
int dk_bn_stats_f32(const float* x, int P, int C, float eps, float momentum, int first, float* mean, float* std_, float* invstd, float* run_mean, float* run_std, void* ws, size_t ws_bytes, void* stream);
/* Statistics from a producer's partial sums (stats of *_fwd_ex_f32): fixed-order fold of
 * part[nblk][2][C] (workspace: dk_bn_partials_workspace_bytes) then the finalize above.
 * tickets (optional, here and in dk_bn_bwd_from_partials_f32): >= dk_bn_fold_tickets_count(C)
 * words that the caller zeroed once; every call leaves them zero.  With them a fold of more
 * than 256 rows runs in ONE launch (the last block to arrive at an agent-scope ticket folds
 * the level-2 rows), without them in one launch per level.  Calls sharing ticket words must
 * not run concurrently (e.g. on two streams);
 * dk_bn_reduce_partials_f64 gives the [2][C] sums a SyncBN rank all-reduces. */
size_t dk_bn_partials_workspace_bytes(int nblk, int C);
int dk_bn_fold_tickets_count(int C);
int dk_bn_stats_from_partials_f32(const void* part, int nblk, int C, double count, float eps, float momentum, int first, float* mean, float* std_, float* invstd, float* run_mean, float* run_std, void* ws, size_t ws_bytes, unsigned* tickets, void* stream);
int dk_bn_reduce_partials_f64(const void* part, int nblk, int C, void* out, void* ws, size_t ws_bytes, void* stream);
/* Backward stage 2 from partials of any origin ([nblk][2][C]: dk_bn_bwd_partial_f64, a
 * consumer's *_dgrad_ex_f32, dk_relu_bwd_bn_partial_f64): dgamma, dbeta and k12 for
 * dk_bn_bwd_apply_f32.  The fused post-residual ReLU backward (residual_block.py:85-86) +
 * stage 1 of the backward of the BN feeding the join: dx = mask ? dy : 0 and part (sized
 * dk_bn_workspace_bytes(P, C), dk_bn_partial_blocks(P, C) rows). */
int dk_bn_bwd_from_partials_f32(const void* part, int nblk, int C, double count, float* dgamma, float* dbeta, float* k12, void* ws, size_t ws_bytes, unsigned* tickets, void* stream);
/* In-launch folds.  Arm a partials buffer before the entry point that writes it: that launch's
 * last-arriving blocks then fold the rows (two ticketed levels, fixed order) and finalize
 * exactly what dk_bn_stats_from_partials_f32 (arm_stats) or dk_bn_bwd_from_partials_f32
 * (arm_bwd) would, and the entry point returns DK_FOLDED (10100) instead of 0 -- the caller
 * skips the separate fold launch.  Entry points that take an arming: dk_pwconv_fwd_ex_f32,
 * dk_dwconv_fwd_ex_f32, dk_conv2d_fwd_ex_f32, dk_conv2d_fwd_narrow_f32, dk_pwconv_dgrad_bnbwd_f32, dk_pwconv_dgrad_ex_f32,
 * dk_pwconv_bwd_bnbwd_f32, dk_dwconv_bwd_bnbwd_f32, dk_dwconv_dgrad_ex_f32,
 * dk_relu_bwd_bn_partial_f64 (for the paths that implement it; otherwise they return 0 and
 * the caller folds as before and calls dk_bn_fold_disarm).  One arming per host thread; the
 * next entry point that writes that buffer consumes it.  tickets: >= ntickets zeroed words
 * (dk_bn_fold_tickets_needed_count(nrows, channel slices of the producer), left zero), not shared
 * with concurrent launches; scratch: >= dk_bn_fold_scratch_bytes(nrows, C). */
int dk_bn_fold_arm_stats(const void* part, int nrows, int C, double count, float eps, float momentum, int first, float* mean, float* std_, float* invstd, float* run_mean, float* run_std, unsigned* tickets, int ntickets, void* scratch, size_t scratch_bytes);
int dk_bn_fold_arm_bwd(const void* part, int nrows, int C, double count, float* dgamma, float* dbeta, float* k12, unsigned* tickets, int ntickets, void* scratch, size_t scratch_bytes);
int dk_bn_fold_disarm(void);
/* Deferred weight-gradient reduce.  dk_wgrad_reduce_defer(1): the fused backward entry points
 * called next on this host thread (dk_dwconv_bwd_bnbwd_f32 / _bf16, dk_dwconv_bwd_bnbwd_join_f32,
 * dk_dwconv_bwd_s2_bnbwd_*, dk_pwconv_bwd_bnbwd_f32 / _bf16) leave the weight-gradient partial slab in their workspace and record its
 * fixed-order reduce instead of launching it; dk_wgrad_reduce_flush(stream) launches the recorded
 * ones, in order, on `stream` (the caller orders that stream after the entry points' and keeps the
 * workspaces untouched until the reduces have run).  (0): reduce in the entry point again; (-1):
 * as 0, dropping the recorded reduces.  Up to 64 recorded per host thread (then DK_ERR_ARGS until
 * flushed); dk_wgrad_reduce_pending() = how many. */
int dk_wgrad_reduce_defer(int mode);
int dk_wgrad_reduce_pending(void);
int dk_wgrad_reduce_flush(void* stream);
/* Cross-stream ordering between the host's HIP streams (main / weight-gradient side / skip branch)
 * with events created without the system-scope fence and without timing (the hand-overs are
 * device-internal).  dk_stream_wait_stream(waiter, src, event): work enqueued on `waiter` from now on
 * starts after everything enqueued on `src` so far; `event` (from dk_sync_event_create) may be
 * recorded again once the call has returned.  dk_sync_event_record + dk_stream_wait_event: the same
 * split in two (a branch's completion recorded now, waited on later).  Return 0 or the hipError_t. */
int dk_sync_event_create(void** event);
int dk_sync_event_destroy(void* event);
int dk_sync_event_record(void* event, void* stream);
int dk_stream_wait_event(void* stream, void* event);
int dk_stream_wait_stream(void* waiter, void* src, void* event);
size_t dk_bn_fold_scratch_bytes(int nrows, int C);
int dk_bn_fold_tickets_needed_count(int nrows, int nslices);
int dk_relu_bwd_bn_partial_f64(const float* dy, const uint8_t* mask, const float* x, int P, int C, const float* mean, const float* invstd, const float* gamma, const float* beta, int relu, float* dx, void* part, size_t part_bytes, void* stream);
int dk_bn_infer_params_f32(const float* run_std, int C, float* invstd, void* stream);
int dk_bn_apply_f32(const float* x, long long numel, int C, const float* mean, const float* invstd, const float* gamma, const float* beta, int relu, float* y, uint8_t* mask, void* stream);
int dk_bn_bwd_partial_f64(const float* x, const float* dy, int P, int C, const float* mean, const float* invstd, const float* gamma, const float* beta, int relu, void* ws, size_t ws_bytes, void* stream);
int dk_bn_bwd_finalize_f32(const void* part_local, int nblk_local, const void* part_global, int nblk_global, int C, double count, float* dgamma, float* dbeta, float* k12, void* stream);
int dk_bn_bwd_apply_f32(const float* x, const float* dy, long long numel, int C, const float* mean, const float* invstd, const float* gamma, const float* beta, int relu, const float* k12, float* dx, void* stream);
int dk_bn_bwd_f32(const float* x, const float* dy, int P, int C, const float* mean, const float* invstd, const float* gamma, const float* beta, int relu, float* dgamma, float* dbeta, float* dx, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * Activation, residual join, pooling head, loss.
 *   ReLU: layers/activations.py:14-47 (mask is uint8 here, fp32 in the reference).
 *   add (+ReLU): ResidualBlock.forward/backward joins (layers/residual_block.py:75, :94-97).
 *   GAP: layers/pooling.py:23-36.   softmax + CE: layers/losses.py:13-34.
 * ------------------------------------------------------------------------------------- */
/* dk_relu_fwd_*: y = max(x, 0) and mask = (x > 0) as uint8; either output may be NULL (a mask-only pass). */
int dk_relu_fwd_f32(const float* x, long long n, float* y, uint8_t* mask, void* stream);
int dk_relu_bwd_f32(const float* dy, const uint8_t* mask, long long n, float* dx, void* stream);
int dk_mask_to_f32(const uint8_t* mask, long long n, float* out, void* stream);
int dk_add_f32(const float* a, const float* b, long long n, int relu, float* y, uint8_t* mask, void* stream);
/* Residual join with BN on load (see *_bnx_*): y = [ReLU](bnA(a) + bnB(b)) over NHWC rows of C
 * channels; a_mean (b_mean) == NULL: that input is used as is.  Replaces BatchNormLayer
 * apply + ResidualBlock join + post-activation (residual_block.py:65-75). */
int dk_bn_add_f32(const float* a, const float* a_mean, const float* a_invstd, const float* a_gamma, const float* a_beta, int a_relu, const float* b, const float* b_mean, const float* b_invstd, const float* b_gamma, const float* b_beta, int b_relu, long long n, int C, int relu, float* y, uint8_t* mask, void* stream);
int dk_gap_fwd_f32(const float* x, int N, int HW, int C, float* out, void* stream);
/* The global average pooling of a residual join y = ReLU(bnA(a) + bnB(b)) (dk_bn_add_f32's operands;
 * residual_block.py:75 then pooling.py:23-30) without storing y: out[N][C] bit-identical to
 * dk_bn_add_f32 followed by dk_gap_fwd_f32, y's ReLU mask (N*HW*C bytes, NHWC) written when non-NULL. */
int dk_gap_join_fwd_f32(const float* a, const float* a_mean, const float* a_invstd, const float* a_gamma, const float* a_beta, int a_relu, const float* b, const float* b_mean, const float* b_invstd, const float* b_gamma, const float* b_beta, int b_relu, int N, int HW, int C, uint8_t* mask, float* out, void* stream);
int dk_gap_bwd_f32(const float* dy, int N, int HW, int C, float* dx, void* stream);
int dk_softmax_xent_fwd_f32(const float* x, const float* y_onehot, int B, int K, float* p, float* loss, void* stream);
int dk_softmax_xent_bwd_f32(const float* p, const float* y_onehot, int B, int K, float* dx, void* stream);

/* ---------------------------------------------------------------------------------------
 * Optimiser / regulariser / utilities.
 *   SGD momentum over a table of tensors in ONE launch (optimisers/SGDMomentum.py:31-39;
 *   the reference issues ~4 CuPy kernels per tensor).  Table entry (40 bytes):
 *   { float* w; const float* g; float* v; int64 n; int64 first_block }, first_block =
 *   sum of ceil(n/256) over the preceding entries; total_blocks = that sum over all.
 *   l2 loss term: regularisers/l2.py:12-14; scale: l2.py:16-17 and DP averaging.
 *   colsum: bias gradients, np.sum(upstream_dx, axis=(0,2,3)) (convolution.py:91-92 etc.).
 * ------------------------------------------------------------------------------------- */
int dk_sgd_momentum_multi_f32(const void* table, int ntens, long long total_blocks, float lr, float momentum, float grad_scale, void* stream);
int dk_l2_loss_f32(const float* w, long long n, float strength, int accumulate, float* out, void* stream);
size_t dk_l2_multi_workspace_bytes(long long total_blocks);
int dk_l2_loss_multi_f32(const void* table, int ntens, long long total_blocks, const float* add_to, float* out, void* ws, size_t ws_bytes, void* stream);
int dk_scale_f32(const float* x, long long n, float s, float* y, void* stream);
size_t dk_colsum_workspace_bytes(int M, int N);
int dk_colsum_f32(const float* in, int M, int N, float* out, void* ws, size_t ws_bytes, void* stream);
int dk_nchw_to_nhwc_f32(const float* x, int N, int C, int H, int W, int Cp, float* y, void* stream);
int dk_nhwc_unpad_f32(const float* x, long long P, int Cp, int C, float* y, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DORKNET_HIP_H */
