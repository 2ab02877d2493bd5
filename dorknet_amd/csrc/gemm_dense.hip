// Dense layer entry points (layers/dense_layer.py) on the implicit-GEMM engine (gemm_engine.h).
#include "gemm_engine.h"

using namespace dk;

// Dense (dense_layer.py:46-55): y[b][o] = sum_i x[b][i] * w[i][o] (+ bias[o]);  w stored (in, out).
DK_API int dk_dense_fwd_f32(const float* x, int B, int IN, const float* w_io, int OUT, const float* bias, float* y,
                            void* stream) {
  MatDesc a = mat(x, B, IN, B);
  MatDesc b = mat(w_io, IN, OUT, OUT);
  EpStore ep = ep_store(y, OUT, bias);
  const hipStream_t st = as_stream(stream);
  const bool va = vec_ok(a, IN, 4), vb = vec_ok(b, 4, OUT);
  if (va && vb) return igemm_rows<LdMatKC, MatDesc, LdMatIC, MatDesc, EpStore>(a, b, ep, B, OUT, IN, st);
  return igemm_rows<LdMatKC1, MatDesc, LdMatIC1, MatDesc, EpStore>(a, b, ep, B, OUT, IN, st);
}

// dx[b][i] = sum_o dy[b][o] * w[i][o]   (dense_layer.py:67)
DK_API int dk_dense_dgrad_f32(const float* dy, int B, int OUT, const float* w_io, int IN, float* dx, void* stream) {
  MatDesc a = mat(dy, B, OUT, B);
  MatDesc b = mat(w_io, IN, OUT, IN);
  EpStore ep = ep_store(dx, IN, nullptr);
  const hipStream_t st = as_stream(stream);
  if (vec_ok(a, OUT, 4) && vec_ok(b, OUT, 4))
    return igemm_rows<LdMatKC, MatDesc, LdMatKC, MatDesc, EpStore>(a, b, ep, B, IN, OUT, st);
  return igemm_rows<LdMatKC1, MatDesc, LdMatKC1, MatDesc, EpStore>(a, b, ep, B, IN, OUT, st);
}

DK_API size_t dk_dense_wgrad_workspace_bytes(int B, int IN, int OUT) { return splitk_ws_bytes(IN, OUT, B); }

// dw[i][o] = sum_b x[b][i] * dy[b][o] (+ l2 * w)   (dense_layer.py:61-66)
DK_API int dk_dense_wgrad_f32(const float* x, const float* dy, int B, int IN, int OUT, const float* w_io, float l2,
                              float* dw_io, void* ws, size_t ws_bytes, void* stream) {
  if (ws_bytes < splitk_ws_bytes(IN, OUT, B)) return DK_ERR_WORKSPACE;
  MatDesc a = mat(x, B, IN, IN);
  MatDesc b = mat(dy, B, OUT, OUT);
  int splits = 1;
  const hipStream_t st = as_stream(stream);
  int rc;
  if (vec_ok(a, 4, IN) && vec_ok(b, 4, OUT))
    rc = igemm_splitk<LdMatIC, MatDesc, LdMatIC, MatDesc>(a, b, static_cast<float*>(ws), IN, OUT, B, st, &splits);
  else
    rc = igemm_splitk<LdMatIC1, MatDesc, LdMatIC1, MatDesc>(a, b, static_cast<float*>(ws), IN, OUT, B, st, &splits);
  if (rc) return rc;
  return splitk_reduce(static_cast<float*>(ws), splits, IN, OUT, dw_io, w_io, l2, 0, OUT, OUT, 1, 1, st);
}

