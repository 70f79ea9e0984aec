// PyTorch bindings for the dstack_amd HIP kernels. The kernels themselves (elementwise.hip,
// flash_attn.hip) are plain HIP translation units with C launchers; this file only validates
// tensors, allocates outputs and forwards the current HIP stream.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

extern "C" {
hipError_t dsa_rmsnorm_fwd(const void*, const void*, const void*, void*, void*, float*, int, int, float,
                           hipStream_t);
int dsa_rmsnorm_bwd_grid(int rows);
hipError_t dsa_rmsnorm_bwd(const void*, const void*, const void*, const float*, const void*, void*, float*,
                           float*, void*, int, int, int, hipStream_t);
hipError_t dsa_swiglu_fwd(const void*, void*, int, int, hipStream_t);
bool dsa_transpose2d_supported(int, int);
hipError_t dsa_swiglu_fwd_t(const void*, void*, void*, int, int, hipStream_t);
hipError_t dsa_transpose2d(const void*, void*, int, int, hipStream_t);
hipError_t dsa_swiglu_bwd(const void*, const void*, void*, int, int, hipStream_t);
hipError_t dsa_swiglu_bwd_t(const void*, const void*, void*, void*, int, int, hipStream_t);
hipError_t dsa_rope_qkv(const void*, void*, const float*, const float*, int, int, int, int, int, int,
                        hipStream_t);
hipError_t dsa_ce_fwd(const void*, const int64_t*, float*, float*, int, int, hipStream_t);
hipError_t dsa_ce_bwd(const void*, const int64_t*, const float*, const float*, void*, int, int, hipStream_t);
hipError_t dsa_adamw(void*, const void*, float*, float*, float*, size_t, float, float, float, float, float,
                     float, float, float, int, hipStream_t);
hipError_t dsa_embedding_bwd(const void*, const int64_t*, const int64_t*, void*, int, int, int, hipStream_t);
hipError_t dsa_fa_fwd(const void*, void*, float*, int, int, int, int, int, float, int, hipStream_t);
size_t dsa_fa_bwd_workspace(int, int, int);
hipError_t dsa_fa_bwd(const void*, const void*, const void*, const float*, void*, void*, int, int, int, int,
                      int, float, int, const float*, const float*, hipStream_t);
int dsa_paged_page_size();
hipError_t dsa_rope_cache_write(void*, const int*, const int*, const float*, const float*, void*, void*, int, int,
                                int, int, float, float, const float*, const float*, hipStream_t);
hipError_t dsa_paged_decode(const void*, long, const void*, const void*, const int*, int, const int*, void*, float*,
                            float*, int, int, int, int, int, float, int, float, float, hipStream_t);
hipError_t dsa_sample(const void*, long, int, int, const float*, const int64_t*, const int*, int*, float*,
                      hipStream_t);
bool dsa_gemm_tn_supported(int, int, int);
bool dsa_gemv_supported(int, int);
hipError_t dsa_gemv(const void*, long, const void*, void*, long, int, int, int, hipStream_t);
bool dsa_quant_fp8_supported(int);
bool dsa_rmsnorm_fwd_fp8_supported(int, int);
hipError_t dsa_rmsnorm_fwd_fp8(const void*, const void*, const void*, void*, void*, float*, float*, int, int, float,
                               const float*, const float*, hipStream_t);
hipError_t dsa_quant_fp8_rows(const void*, long, void*, long, float*, int, int, hipStream_t);
hipError_t dsa_swiglu_quant_fp8_rows(const void*, long, void*, long, float*, int, int, const float*, const float*,
                                     hipStream_t);
hipError_t dsa_scale_rows_cols(void*, long, int, int, const float*, const float*, hipStream_t);
bool dsa_gemv_fp8_supported(int, int);
hipError_t dsa_gemv_fp8(const void*, long, const void*, const float*, void*, long, int, int, int, hipStream_t);
hipError_t dsa_gemm_tn(const void*, const void*, void*, int, int, int, long, long, long, int, hipStream_t);
bool dsa_gemm_nt_supported(int, int, int);
hipError_t dsa_gemm_nt(const void*, const void*, void*, int, int, int, long, long, long, int, hipStream_t);
bool dsa_gemm_nt_rope_supported(int, int, int, int, int);
bool dsa_gemm_nt_f8_supported(int, int, int);
void dsa_gemm_nt_set_grid(int);
bool dsa_gemm_nt_f8_swiglu_supported(int, int, int);
hipError_t dsa_gemm_nt_f8_swiglu(const void*, const void*, void*, float*, const float*, const float*, int, int, int,
                                 long, long, hipStream_t);
hipError_t dsa_quant_fp8_rows_pmax(const void*, long, const float*, int, void*, long, float*, int, int, hipStream_t);
hipError_t dsa_gemm_nt_f8(const void*, const void*, void*, int, int, int, long, long, long, hipStream_t);
hipError_t dsa_gemm_nt_rope(const void*, const void*, void*, const float*, const float*, int, int, int, long, long,
                            long, int, int, hipStream_t);
bool dsa_gemm_nt_swiglu_supported(int, int, int);
hipError_t dsa_gemm_nt_trace(const void*, const void*, void*, int, int, int, unsigned long long*, hipStream_t);
hipError_t dsa_gemm_nt_swiglu(const void*, const void*, void*, void*, void*, int, int, int, long, long, hipStream_t);
bool dsa_gemm_nt_swiglu_bwd_supported(int, int, int);
bool dsa_gemm_km_supported(int, int, int);
hipError_t dsa_fa_dkdv_trace(const void*, const void*, const float*, const float*, float*, float*, unsigned long long*,
                             int, int, int, int, float, hipStream_t);
bool dsa_fp8_rows_gemm_supported(int, int, int, int, int);
bool dsa_fp8_stream_gemm_supported(int, int, int, int, int);
hipError_t dsa_fp8_stream_gemm(const void*, const float*, const void*, const float*, void*, float*, int, int, int,
                               long, long, long, int, int, int, int, hipStream_t);
hipError_t dsa_fp8_rows_gemm(const void*, const float*, const void*, const float*, void*, float*, int*, int, int, int,
                             long, long, long, int, int, int, hipStream_t);
hipError_t dsa_gemm_km(const void*, const void*, void*, int, int, int, long, long, long, int, hipStream_t);
hipError_t dsa_cu_hog(int, int, int, double, int*, hipStream_t);
hipError_t dsa_synthetic_tokens(const double*, const int64_t*, const int64_t*, const int64_t*, int64_t*, int64_t*,
                                uint64_t, float, int, int, int, hipStream_t);
hipError_t dsa_gemm_km_f32(const void*, const void*, void*, float*, int, int, int, long, long, long, long, int,
                           hipStream_t);
hipError_t dsa_gemm_nt_swiglu_bwd(const void*, const void*, const void*, void*, void*, int, int, int, long, long,
                                  hipStream_t);
}

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "dstack_amd kernel ", what, " failed: ", hipGetErrorString(e));
}

void check_bf16(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a ROCm tensor");
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16, name, " must be bf16");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

std::vector<torch::Tensor> rms_norm_fwd(torch::Tensor x, torch::Tensor w, double eps) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  const int rows = x.size(0), D = x.size(1);
  auto y = torch::empty_like(x);
  auto rstd = torch::empty({rows}, x.options().dtype(torch::kFloat32));
  check(dsa_rmsnorm_fwd(x.data_ptr(), nullptr, w.data_ptr(), nullptr, y.data_ptr(), rstd.data_ptr<float>(),
                        rows, D, (float)eps, stream()),
        "rms_norm_fwd");
  return {y, rstd};
}

std::vector<torch::Tensor> add_rms_norm_fwd(torch::Tensor x, torch::Tensor delta, torch::Tensor w, double eps) {
  check_bf16(x, "x");
  check_bf16(delta, "delta");
  check_bf16(w, "w");
  TORCH_CHECK(x.sizes() == delta.sizes(), "x/delta shape mismatch");
  const int rows = x.size(0), D = x.size(1);
  auto h = torch::empty_like(x);
  auto y = torch::empty_like(x);
  auto rstd = torch::empty({rows}, x.options().dtype(torch::kFloat32));
  check(dsa_rmsnorm_fwd(x.data_ptr(), delta.data_ptr(), w.data_ptr(), h.data_ptr(), y.data_ptr(),
                        rstd.data_ptr<float>(), rows, D, (float)eps, stream()),
        "add_rms_norm_fwd");
  return {h, y, rstd};
}

bool rms_norm_fp8_supported(int64_t rows, int64_t D) { return dsa_rmsnorm_fwd_fp8_supported((int)rows, (int)D); }

// (x + delta) -> RMSNorm -> e4m3 [rows, D] (uint8) + per-row scales; returns {h (x + delta, or an
// empty tensor without delta), q, s}.  Serving decode (rows <= 1024).
// dr / dc (optional, with delta): delta is a raw fp8 GEMM product whose row-wise scales (dr [rows]
// per token, dc [D] per output channel) are applied before the residual add
std::vector<torch::Tensor> rms_norm_fp8(torch::Tensor x, c10::optional<torch::Tensor> delta, torch::Tensor w,
                                        double eps, c10::optional<torch::Tensor> dr, c10::optional<torch::Tensor> dc) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  const int rows = x.size(0), D = x.size(1);
  TORCH_CHECK(dsa_rmsnorm_fwd_fp8_supported(rows, D), "rms_norm_fp8: D % 8 == 0, D <= 8192");
  TORCH_CHECK(dr.has_value() == dc.has_value() && (!dr.has_value() || delta.has_value()),
              "rms_norm_fp8: dr and dc go together, with delta");
  const float* drp = nullptr;
  const float* dcp = nullptr;
  if (dr.has_value()) {
    TORCH_CHECK(dr->scalar_type() == torch::kFloat32 && dr->is_contiguous() && dr->numel() == rows,
                "rms_norm_fp8: dr must be fp32 [rows]");
    TORCH_CHECK(dc->scalar_type() == torch::kFloat32 && dc->is_contiguous() && dc->numel() == D &&
                    reinterpret_cast<uintptr_t>(dc->data_ptr()) % 16 == 0,
                "rms_norm_fp8: dc must be fp32 [D], 16-byte aligned");
    drp = dr->data_ptr<float>();
    dcp = dc->data_ptr<float>();
  }
  torch::Tensor h;
  if (delta.has_value()) {
    check_bf16(*delta, "delta");
    TORCH_CHECK(delta->sizes() == x.sizes(), "x/delta shape mismatch");
    h = torch::empty_like(x);
  }
  auto q = torch::empty({rows, D}, x.options().dtype(torch::kUInt8));
  auto qs = torch::empty({rows}, x.options().dtype(torch::kFloat32));
  auto rstd = torch::empty({rows}, x.options().dtype(torch::kFloat32));
  check(dsa_rmsnorm_fwd_fp8(x.data_ptr(), delta.has_value() ? delta->data_ptr() : nullptr, w.data_ptr(),
                            delta.has_value() ? h.data_ptr() : nullptr, q.data_ptr(), qs.data_ptr<float>(),
                            rstd.data_ptr<float>(), rows, D, (float)eps, drp, dcp, stream()),
        "rms_norm_fp8");
  return {delta.has_value() ? h : torch::Tensor(), q, qs};
}

// dw_out (bf16 [D], optional): write the weight gradient there (accumulating when `accumulate`)
// instead of returning an fp32 dw -- the optimizer's flat-buffer view of the norm weight's grad
std::vector<torch::Tensor> rms_norm_bwd(torch::Tensor dy, torch::Tensor h, torch::Tensor w, torch::Tensor rstd,
                                        c10::optional<torch::Tensor> dres, c10::optional<torch::Tensor> dw_out,
                                        bool accumulate) {
  check_bf16(dy, "dy");
  check_bf16(h, "h");
  check_bf16(w, "w");
  const int rows = h.size(0), D = h.size(1);
  const void* dres_ptr = nullptr;
  if (dres.has_value()) {
    check_bf16(*dres, "dres");
    dres_ptr = dres->data_ptr();
  }
  void* dw_out_ptr = nullptr;
  if (dw_out.has_value()) {
    check_bf16(*dw_out, "dw_out");
    TORCH_CHECK(dw_out->numel() == D, "dw_out must hold D elements");
    dw_out_ptr = dw_out->data_ptr();
  }
  auto dx = torch::empty_like(h);
  const int grid = dsa_rmsnorm_bwd_grid(rows);
  auto part = torch::empty({grid, D}, h.options().dtype(torch::kFloat32));
  auto dw = dw_out_ptr ? torch::Tensor() : torch::empty({D}, h.options().dtype(torch::kFloat32));
  check(dsa_rmsnorm_bwd(dy.data_ptr(), h.data_ptr(), w.data_ptr(), rstd.data_ptr<float>(), dres_ptr,
                        dx.data_ptr(), part.data_ptr<float>(), dw_out_ptr ? nullptr : dw.data_ptr<float>(),
                        dw_out_ptr, accumulate ? 1 : 0, rows, D, stream()),
        "rms_norm_bwd");
  return {dx, dw};
}

bool transpose2d_supported(int64_t R, int64_t C) { return dsa_transpose2d_supported((int)R, (int)C); }

// out[C, R] = x[R, C]^T for a row-contiguous 2-D bf16 x (row stride may exceed C)
torch::Tensor transpose2d(torch::Tensor x) {
  check_bf16(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) == x.size(1), "transpose2d: contiguous 2-D input");
  const int R = (int)x.size(0), C = (int)x.size(1);
  TORCH_CHECK(dsa_transpose2d_supported(R, C), "transpose2d: shape not tiled (R % 128, C % 64)");
  auto out = torch::empty({C, R}, x.options());
  check(dsa_transpose2d(x.data_ptr(), out.data_ptr(), R, C, stream()), "transpose2d");
  return out;
}

torch::Tensor swiglu_fwd(torch::Tensor gu) {
  check_bf16(gu, "gu");
  const int F = gu.size(-1) / 2;
  const int rows = gu.numel() / gu.size(-1);
  auto sizes = gu.sizes().vec();
  sizes.back() = F;
  auto out = torch::empty(sizes, gu.options());
  check(dsa_swiglu_fwd(gu.data_ptr(), out.data_ptr(), rows, F, stream()), "swiglu_fwd");
  return out;
}

// (a, aT): a = silu(gate) * up [..., F] and its transpose aT [F, T] (T = rows)
std::vector<torch::Tensor> swiglu_fwd_t(torch::Tensor gu) {
  check_bf16(gu, "gu");
  const int F = gu.size(-1) / 2;
  const int T = gu.numel() / gu.size(-1);
  TORCH_CHECK(T % 128 == 0 && F % 64 == 0, "swiglu_fwd_t: rows % 128 and F % 64 must be 0");
  auto sizes = gu.sizes().vec();
  sizes.back() = F;
  auto out = torch::empty(sizes, gu.options());
  auto outT = torch::empty({F, T}, gu.options());
  check(dsa_swiglu_fwd_t(gu.data_ptr(), out.data_ptr(), outT.data_ptr(), T, F, stream()), "swiglu_fwd_t");
  return {out, outT};
}

torch::Tensor swiglu_bwd(torch::Tensor da, torch::Tensor gu) {
  check_bf16(da, "da");
  check_bf16(gu, "gu");
  const int F = gu.size(-1) / 2;
  const int rows = gu.numel() / gu.size(-1);
  auto dgu = torch::empty_like(gu);
  check(dsa_swiglu_bwd(da.data_ptr(), gu.data_ptr(), dgu.data_ptr(), rows, F, stream()), "swiglu_bwd");
  return dgu;
}

// returns {dgu [.., 2F], dgu^T [2F, T]}
std::vector<torch::Tensor> swiglu_bwd_t(torch::Tensor da, torch::Tensor gu) {
  check_bf16(da, "da");
  check_bf16(gu, "gu");
  const int F = gu.size(-1) / 2;
  const int T = gu.numel() / gu.size(-1);
  TORCH_CHECK(T % 128 == 0 && F % 64 == 0, "swiglu_bwd_t: rows % 128 and F % 64 must be 0");
  TORCH_CHECK(da.numel() == (int64_t)T * F, "swiglu_bwd_t: da must be [T, F]");
  auto dgu = torch::empty_like(gu);
  auto dguT = torch::empty({2 * F, T}, gu.options());
  check(dsa_swiglu_bwd_t(da.data_ptr(), gu.data_ptr(), dgu.data_ptr(), dguT.data_ptr(), T, F, stream()),
        "swiglu_bwd_t");
  return {dgu, dguT};
}

torch::Tensor rope_qkv(torch::Tensor qkv, torch::Tensor cos, torch::Tensor sin, int64_t n_rot, int64_t head_dim,
                       bool inverse) {
  check_bf16(qkv, "qkv");
  TORCH_CHECK(qkv.dim() == 3, "qkv must be [B, S, NH*D]");
  TORCH_CHECK(cos.scalar_type() == torch::kFloat32 && sin.scalar_type() == torch::kFloat32, "cos/sin fp32");
  TORCH_CHECK(cos.is_contiguous() && sin.is_contiguous(), "cos/sin contiguous");
  const int B = qkv.size(0), S = qkv.size(1);
  const int NH = qkv.size(2) / head_dim;
  TORCH_CHECK(cos.size(0) >= S && cos.size(1) == head_dim / 2, "rope table shape");
  auto out = torch::empty_like(qkv);
  check(dsa_rope_qkv(qkv.data_ptr(), out.data_ptr(), cos.data_ptr<float>(), sin.data_ptr<float>(), B * S, S, NH,
                     (int)n_rot, (int)head_dim, inverse ? 1 : 0, stream()),
        "rope_qkv");
  return out;
}

std::vector<torch::Tensor> cross_entropy_fwd(torch::Tensor logits, torch::Tensor target) {
  check_bf16(logits, "logits");
  TORCH_CHECK(target.scalar_type() == torch::kInt64 && target.is_contiguous(), "target int64");
  const int rows = logits.size(0), V = logits.size(1);
  TORCH_CHECK(V % 8 == 0, "vocab must be a multiple of 8");
  auto loss = torch::empty({rows}, logits.options().dtype(torch::kFloat32));
  auto lse = torch::empty({rows}, logits.options().dtype(torch::kFloat32));
  check(dsa_ce_fwd(logits.data_ptr(), target.data_ptr<int64_t>(), loss.data_ptr<float>(), lse.data_ptr<float>(),
                   rows, V, stream()),
        "cross_entropy_fwd");
  return {loss, lse};
}

torch::Tensor cross_entropy_bwd(torch::Tensor logits, torch::Tensor target, torch::Tensor lse, torch::Tensor scale,
                                bool inplace) {
  check_bf16(logits, "logits");
  const int rows = logits.size(0), V = logits.size(1);
  auto out = inplace ? logits : torch::empty_like(logits);
  check(dsa_ce_bwd(logits.data_ptr(), target.data_ptr<int64_t>(), lse.data_ptr<float>(), scale.data_ptr<float>(),
                   out.data_ptr(), rows, V, stream()),
        "cross_entropy_bwd");
  return out;
}

// grad (bf16 [V, D]) (+)= scatter-sum of dy rows by token id; the ids come stably sorted with their
// original positions (torch.sort(stable=True)).  accumulate=false clears the whole table first.
void embedding_bwd(torch::Tensor dy, torch::Tensor sorted_tok, torch::Tensor order, torch::Tensor grad,
                   bool accumulate) {
  check_bf16(dy, "dy");
  check_bf16(grad, "grad");
  TORCH_CHECK(dy.dim() == 2 && grad.dim() == 2 && dy.size(1) == grad.size(1), "embedding_bwd: dy [T, D], grad [V, D]");
  for (auto* t : {&sorted_tok, &order}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kInt64 && t->is_contiguous() && t->numel() == dy.size(0),
                "embedding_bwd: sorted ids / order must be int64 [T]");
  }
  if (!accumulate) check(hipMemsetAsync(grad.data_ptr(), 0, grad.numel() * 2, stream()), "embedding_bwd memset");
  check(dsa_embedding_bwd(dy.data_ptr(), sorted_tok.data_ptr<int64_t>(), order.data_ptr<int64_t>(), grad.data_ptr(),
                          (int)dy.size(0), (int)dy.size(1), accumulate ? 1 : 0, stream()),
        "embedding_bwd");
}

void adamw(torch::Tensor param, torch::Tensor grad, torch::Tensor master, torch::Tensor m, torch::Tensor v,
           double lr, double b1, double b2, double eps, double wd, double bc1, double bc2, double gscale,
           int64_t max_blocks) {
  check_bf16(param, "param");
  check_bf16(grad, "grad");
  for (auto* t : {&master, &m, &v}) {
    TORCH_CHECK(t->scalar_type() == torch::kFloat32 && t->is_contiguous(), "adam state must be fp32 contiguous");
    TORCH_CHECK(t->numel() == param.numel(), "adam state numel mismatch");
  }
  check(dsa_adamw(param.data_ptr(), grad.data_ptr(), master.data_ptr<float>(), m.data_ptr<float>(),
                  v.data_ptr<float>(), param.numel(), lr, b1, b2, eps, wd, bc1, bc2, gscale, (int)max_blocks,
                  stream()),
        "adamw");
}

std::vector<torch::Tensor> flash_attn_fwd(torch::Tensor qkv, int64_t H, int64_t KVH, bool causal) {
  check_bf16(qkv, "qkv");
  TORCH_CHECK(qkv.dim() == 3, "qkv must be [B, S, (H+2KVH)*D]");
  const int B = qkv.size(0), S = qkv.size(1);
  const int D = qkv.size(2) / (H + 2 * KVH);
  auto out = torch::empty({B, S, H * D}, qkv.options());
  auto lse = torch::empty({B, H, S}, qkv.options().dtype(torch::kFloat32));
  check(dsa_fa_fwd(qkv.data_ptr(), out.data_ptr(), lse.data_ptr<float>(), B, S, H, KVH, D, 1.0f / std::sqrt((float)D),
                   causal ? 1 : 0, stream()),
        "flash_attn_fwd");
  return {out, lse};
}

// rope_cos / rope_sin ([>= S, 64] fp32, optional): q and k of `qkv` were rotated by RoPE; the
// returned gradient is w.r.t. the unrotated projection (the RoPE backward fused in)
torch::Tensor flash_attn_bwd(torch::Tensor dout, torch::Tensor qkv, torch::Tensor out, torch::Tensor lse, int64_t H,
                             int64_t KVH, bool causal, c10::optional<torch::Tensor> rope_cos,
                             c10::optional<torch::Tensor> rope_sin) {
  check_bf16(dout, "dout");
  check_bf16(qkv, "qkv");
  check_bf16(out, "out");
  const int B = qkv.size(0), S = qkv.size(1);
  const int D = qkv.size(2) / (H + 2 * KVH);
  const float *rc = nullptr, *rs = nullptr;
  TORCH_CHECK(rope_cos.has_value() == rope_sin.has_value(), "flash_attn_bwd: rope_cos and rope_sin go together");
  if (rope_cos.has_value()) {
    for (const auto& t : {*rope_cos, *rope_sin}) {
      TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kFloat32 && t.is_contiguous() && t.dim() == 2 &&
                      t.size(0) >= S && t.size(1) == D / 2,
                  "flash_attn_bwd: rope tables must be contiguous fp32 [>= S, head_dim / 2]");
    }
    rc = rope_cos->data_ptr<float>();
    rs = rope_sin->data_ptr<float>();
  }
  auto dqkv = torch::empty_like(qkv);
  auto ws = torch::empty({(int64_t)dsa_fa_bwd_workspace(B, S, H)}, qkv.options().dtype(torch::kUInt8));
  check(dsa_fa_bwd(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(), dqkv.data_ptr(),
                   ws.data_ptr(), B, S, H, KVH, D, 1.0f / std::sqrt((float)D), causal ? 1 : 0, rc, rs, stream()),
        "flash_attn_bwd");
  return dqkv;
}

// diagnostic: per-phase s_memtime stamps of the causal 8-wave dK/dV pass (waves 0 and 4 of
// workgroup 0, q-tiles 8..11, 5 points each) -> int64 [2, 64]
torch::Tensor fa_dkdv_trace(torch::Tensor qkv, torch::Tensor dout, torch::Tensor lse, torch::Tensor delta, int64_t H,
                            int64_t KVH) {
  check_bf16(qkv, "qkv");
  check_bf16(dout, "dout");
  const int B = qkv.size(0), S = qkv.size(1);
  auto f32 = qkv.options().dtype(torch::kFloat32);
  auto dkp = torch::empty({B, S, H, 128}, f32), dvp = torch::empty({B, S, H, 128}, f32);
  auto tr = torch::zeros({2, 64}, qkv.options().dtype(torch::kInt64));
  const float sl2 = 1.4426950408889634f / std::sqrt(128.f);
  check(dsa_fa_dkdv_trace(qkv.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(), delta.data_ptr<float>(),
                          dkp.data_ptr<float>(), dvp.data_ptr<float>(),
                          reinterpret_cast<unsigned long long*>(tr.data_ptr()), B, S, (int)H, (int)KVH, sl2, stream()),
        "fa_dkdv_trace");
  return tr;
}

bool gemm_tn_supported(int64_t P, int64_t Q, int64_t T) { return dsa_gemm_tn_supported(P, Q, T); }

bool gemv_supported(int64_t M, int64_t K) { return dsa_gemv_supported((int)M, (int)K); }

// y [M, N] = x [M, K] @ w[N, K]^T for M <= 4 (decode projections, csrc/gemv.hip)
torch::Tensor gemv(torch::Tensor x, torch::Tensor w) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kBFloat16 && x.dim() == 2 && x.stride(1) == 1,
              "gemv: x must be bf16 [M, K] with contiguous rows");
  check_bf16(w, "w");
  TORCH_CHECK(w.dim() == 2 && w.size(1) == x.size(1), "gemv: w must be [N, K]");
  TORCH_CHECK(x.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "gemv: x alignment");
  const int64_t M = x.size(0), N = w.size(0), K = x.size(1);
  TORCH_CHECK(dsa_gemv_supported((int)M, (int)K), "gemv: M <= 4 and K % 512 == 0");
  auto y = torch::empty({M, N}, x.options());
  check(dsa_gemv(x.data_ptr(), x.stride(0), w.data_ptr(), y.data_ptr(), N, (int)M, (int)N, (int)K, stream()),
        "gemv");
  return y;
}

// FP8 (e4m3) rows: q [M, K] uint8 (view as float8_e4m3fn) and s [M] fp32, x[m] ~= q[m] * s[m]
// gu [M, 2F] bf16 -> (q [M, F] e4m3 bytes, s [M] fp32) of bf16(silu(gate) * up), per-row scales
// rs / cs (optional, together): gu is the raw product of a tensor-wise-scaled fp8 GEMM; the per-token
// scale rs [M] and per-output-channel scale cs [2F] are applied before the SwiGLU
std::vector<torch::Tensor> swiglu_quant_fp8_rows(torch::Tensor gu, c10::optional<torch::Tensor> rs,
                                                 c10::optional<torch::Tensor> cs) {
  TORCH_CHECK(gu.is_cuda() && gu.scalar_type() == torch::kBFloat16 && gu.dim() == 2 && gu.stride(1) == 1,
              "swiglu_quant_fp8_rows: gu must be bf16 [M, 2F] with contiguous rows");
  TORCH_CHECK(gu.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(gu.data_ptr()) % 16 == 0 && gu.size(1) % 16 == 0,
              "swiglu_quant_fp8_rows: alignment (2F % 16 == 0)");
  const int64_t M = gu.size(0), F = gu.size(1) / 2;
  TORCH_CHECK(rs.has_value() == cs.has_value(), "swiglu_quant_fp8_rows: rs and cs go together");
  const float* rp = nullptr;
  const float* cp = nullptr;
  if (rs.has_value()) {
    TORCH_CHECK(rs->scalar_type() == torch::kFloat32 && rs->is_contiguous() && rs->numel() == M,
                "swiglu_quant_fp8_rows: rs must be fp32 [M]");
    TORCH_CHECK(cs->scalar_type() == torch::kFloat32 && cs->is_contiguous() && cs->numel() == 2 * F &&
                    reinterpret_cast<uintptr_t>(cs->data_ptr()) % 16 == 0,
                "swiglu_quant_fp8_rows: cs must be fp32 [2F], 16-byte aligned");
    rp = rs->data_ptr<float>();
    cp = cs->data_ptr<float>();
  }
  auto q = torch::empty({M, F}, gu.options().dtype(torch::kUInt8));
  auto sc = torch::empty({M}, gu.options().dtype(torch::kFloat32));
  if (M > 0)
    check(dsa_swiglu_quant_fp8_rows(gu.data_ptr(), gu.stride(0), q.data_ptr(), F, sc.data_ptr<float>(), (int)M,
                                    (int)F, rp, cp, stream()),
          "swiglu_quant_fp8_rows");
  return {q, sc};
}

// y [M, N] bf16 (+ row stride) *= rs[:, None] * cs[None, :] in place
torch::Tensor scale_rows_cols_(torch::Tensor y, torch::Tensor rs, torch::Tensor cs) {
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == torch::kBFloat16 && y.dim() == 2 && y.stride(1) == 1 &&
                  y.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0 && y.size(1) % 8 == 0,
              "scale_rows_cols_: y must be bf16 [M, N], contiguous 16-byte-aligned rows, N % 8 == 0");
  TORCH_CHECK(rs.scalar_type() == torch::kFloat32 && rs.is_contiguous() && rs.numel() == y.size(0),
              "scale_rows_cols_: rs must be fp32 [M]");
  TORCH_CHECK(cs.scalar_type() == torch::kFloat32 && cs.is_contiguous() && cs.numel() == y.size(1) &&
                  reinterpret_cast<uintptr_t>(cs.data_ptr()) % 16 == 0,
              "scale_rows_cols_: cs must be fp32 [N], 16-byte aligned");
  if (y.size(0) > 0)
    check(dsa_scale_rows_cols(y.data_ptr(), y.stride(0), (int)y.size(0), (int)y.size(1), rs.data_ptr<float>(),
                              cs.data_ptr<float>(), stream()),
          "scale_rows_cols_");
  return y;
}

std::vector<torch::Tensor> quant_fp8_rows(torch::Tensor x) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kBFloat16 && x.dim() == 2 && x.stride(1) == 1,
              "quant_fp8_rows: x must be bf16 [M, K] with contiguous rows");
  TORCH_CHECK(x.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "quant_fp8_rows: alignment");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(dsa_quant_fp8_supported((int)K), "quant_fp8_rows: K % 8 == 0");
  auto q = torch::empty({M, K}, x.options().dtype(torch::kUInt8));
  auto sc = torch::empty({M}, x.options().dtype(torch::kFloat32));
  if (M > 0)
    check(dsa_quant_fp8_rows(x.data_ptr(), x.stride(0), q.data_ptr(), K, sc.data_ptr<float>(), (int)M, (int)K,
                             stream()),
          "quant_fp8_rows");
  return {q, sc};
}

bool gemv_fp8_supported(int64_t M, int64_t K) { return dsa_gemv_fp8_supported((int)M, (int)K); }

// y [M, N] = (x [M, K] @ q[N, K]^T) * s[N] for M <= 4, q e4m3 bytes (decode, csrc/fp8.hip)
torch::Tensor gemv_fp8(torch::Tensor x, torch::Tensor q, torch::Tensor sc) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kBFloat16 && x.dim() == 2 && x.stride(1) == 1,
              "gemv_fp8: x must be bf16 [M, K] with contiguous rows");
  TORCH_CHECK(x.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "gemv_fp8: x alignment");
  TORCH_CHECK(q.is_cuda() && q.element_size() == 1 && q.dim() == 2 && q.is_contiguous() && q.size(1) == x.size(1),
              "gemv_fp8: q must be contiguous 1-byte [N, K]");
  TORCH_CHECK(sc.is_cuda() && sc.scalar_type() == torch::kFloat32 && sc.numel() == q.size(0) && sc.is_contiguous(),
              "gemv_fp8: s must be fp32 [N]");
  const int64_t M = x.size(0), N = q.size(0), K = x.size(1);
  TORCH_CHECK(dsa_gemv_fp8_supported((int)M, (int)K), "gemv_fp8: M <= 4 and K % 1024 == 0");
  auto y = torch::empty({M, N}, x.options());
  check(dsa_gemv_fp8(x.data_ptr(), x.stride(0), q.data_ptr(), sc.data_ptr<float>(), y.data_ptr(), N, (int)M,
                     (int)N, (int)K, stream()),
        "gemv_fp8");
  return y;
}

void check_rows(const torch::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kBFloat16 && t.dim() == 2, what, ": 2-D bf16 ROCm tensors");
  TORCH_CHECK(t.stride(1) == 1 && t.stride(0) % 8 == 0, what, ": rows must be contiguous, row stride % 8 == 0");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, what, ": 16-byte aligned base");
}

bool gemm_nt_supported(int64_t M, int64_t N, int64_t K) { return dsa_gemm_nt_supported(M, N, K); }

// out[M][N] (+)= a[M][K] b[N][K]^T  (csrc/gemm_nt.hip); mode 2 = timing-only (no stores, diagnostics)
void gemm_nt_mode(torch::Tensor a, torch::Tensor b, torch::Tensor out, int64_t mode);
void gemm_nt(torch::Tensor a, torch::Tensor b, torch::Tensor out, bool accumulate) {
  gemm_nt_mode(a, b, out, accumulate ? 1 : 0);
}
void gemm_nt_mode(torch::Tensor a, torch::Tensor b, torch::Tensor out, int64_t mode) {
  check_rows(a, "gemm_nt");
  check_rows(b, "gemm_nt");
  check_rows(out, "gemm_nt");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K && out.size(0) == M && out.size(1) == N, "gemm_nt: shape mismatch");
  TORCH_CHECK(dsa_gemm_nt_supported(M, N, K), "gemm_nt: M % 256, N % 256, K % 128 must be 0");
  check(dsa_gemm_nt(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, a.stride(0), b.stride(0), out.stride(0),
                    (int)mode, stream()),
        "gemm_nt");
}

bool gemm_nt_swiglu_supported(int64_t T, int64_t F, int64_t K) { return dsa_gemm_nt_swiglu_supported(T, F, K); }

bool gemm_nt_f8_supported(int64_t M, int64_t N, int64_t K) { return dsa_gemm_nt_f8_supported(M, N, K); }

// out[M][N] = bf16(a[M][K] w[N][K]^T) for e4m3 a / w (uint8 or float8_e4m3fn storage), unscaled
void gemm_nt_f8(torch::Tensor a, torch::Tensor w, torch::Tensor out) {
  for (const auto& t : {a, w}) {
    TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.stride(1) == 1 && t.element_size() == 1,
                "gemm_nt_f8: operands must be 2-D row-major 1-byte (e4m3) tensors");
  }
  check_rows(out, "gemm_nt_f8");
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && out.size(0) == M && out.size(1) == N, "gemm_nt_f8: shape mismatch");
  TORCH_CHECK(dsa_gemm_nt_f8_supported(M, N, K), "gemm_nt_f8: M % 256, N % 256, K % 256 must be 0");
  check(dsa_gemm_nt_f8(a.data_ptr(), w.data_ptr(), out.data_ptr(), M, N, K, a.stride(0), w.stride(0), out.stride(0),
                       stream()),
        "gemm_nt_f8");
}

bool gemm_nt_f8_swiglu_supported(int64_t M, int64_t F, int64_t K) { return dsa_gemm_nt_f8_swiglu_supported(M, F, K); }

// Serving fp8 gate/up + SwiGLU + per-token e4m3 quantization: x [M][K] e4m3 with row scales xs [M],
// w [2F][K] e4m3 (gate rows then up rows) with per-output-channel scales ws [2F] ->
// (q [M][F] e4m3, s [M]) -- what swiglu_quant_fp8_rows(raw, xs, ws) gives for the raw product,
// with a = silu(g) u (bf16) as the only intermediate in HBM.  Also returns a (diagnostics).
std::vector<torch::Tensor> gemm_nt_f8_swiglu_quant(torch::Tensor x, torch::Tensor w, torch::Tensor xs,
                                                   torch::Tensor ws) {
  for (const auto& t : {x, w}) {
    TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.stride(1) == 1 && t.element_size() == 1,
                "gemm_nt_f8_swiglu_quant: operands must be 2-D row-major e4m3 tensors");
  }
  const int64_t M = x.size(0), K = x.size(1), F = w.size(0) / 2;
  TORCH_CHECK(w.size(1) == K && w.size(0) == 2 * F, "gemm_nt_f8_swiglu_quant: shape mismatch");
  TORCH_CHECK(xs.scalar_type() == torch::kFloat32 && xs.is_contiguous() && xs.numel() == M &&
                  ws.scalar_type() == torch::kFloat32 && ws.is_contiguous() && ws.numel() == 2 * F,
              "gemm_nt_f8_swiglu_quant: fp32 scales xs [M], ws [2F]");
  TORCH_CHECK(dsa_gemm_nt_f8_swiglu_supported(M, F, K), "gemm_nt_f8_swiglu_quant: M % 256, F % 128, K % 256 must be 0");
  auto a = torch::empty({M, F}, x.options().dtype(torch::kBFloat16));
  auto pmax = torch::empty({M, F / 32}, x.options().dtype(torch::kFloat32));
  auto q = torch::empty({M, F}, x.options().dtype(torch::kUInt8));
  auto s = torch::empty({M}, x.options().dtype(torch::kFloat32));
  check(dsa_gemm_nt_f8_swiglu(x.data_ptr(), w.data_ptr(), a.data_ptr(), pmax.data_ptr<float>(), xs.data_ptr<float>(),
                              ws.data_ptr<float>(), M, F, K, x.stride(0), w.stride(0), stream()),
        "gemm_nt_f8_swiglu");
  check(dsa_quant_fp8_rows_pmax(a.data_ptr(), F, pmax.data_ptr<float>(), F / 32, q.data_ptr(), F,
                                s.data_ptr<float>(), M, F, stream()),
        "quant_fp8_rows_pmax");
  return {q, s, a};
}

bool gemm_nt_rope_supported(int64_t M, int64_t N, int64_t K, int64_t S, int64_t rot_cols) {
  return dsa_gemm_nt_rope_supported(M, N, K, S, rot_cols);
}

// qkv[M][N] = a[M][K] w[N][K]^T with RoPE (rotate-half, head_dim 128) on columns [0, rot_cols), in
// the GEMM's epilogue before the bf16 rounding; row m is position m % S (csrc/gemm_nt.hip EPI_ROPE)
torch::Tensor gemm_nt_rope(torch::Tensor a, torch::Tensor w, torch::Tensor cos, torch::Tensor sin, int64_t S,
                           int64_t rot_cols) {
  check_rows(a, "gemm_nt_rope");
  check_rows(w, "gemm_nt_rope");
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "gemm_nt_rope: shape mismatch");
  for (const auto& t : {cos, sin}) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kFloat32 && t.is_contiguous() && t.dim() == 2 &&
                    t.size(0) >= S && t.size(1) == 64,
                "gemm_nt_rope: rope tables must be contiguous fp32 [>= S, 64]");
  }
  TORCH_CHECK(dsa_gemm_nt_rope_supported(M, N, K, S, rot_cols),
              "gemm_nt_rope: M % S == 0, S % 256, N % 256, K % 128 must be 0, rot_cols % 128 == 0");
  auto out = torch::empty({M, N}, a.options());
  check(dsa_gemm_nt_rope(a.data_ptr(), w.data_ptr(), out.data_ptr(), cos.data_ptr<float>(), sin.data_ptr<float>(),
                         M, N, K, a.stride(0), w.stride(0), out.stride(0), S, rot_cols, stream()),
        "gemm_nt_rope");
  return out;
}

// diagnostic: per-phase s_memtime stamps of workgroup 0 (waves 0 and 4) -> int64 [2, 64]
torch::Tensor gemm_nt_trace(torch::Tensor a, torch::Tensor b, torch::Tensor out) {
  check_rows(a, "gemm_nt_trace");
  check_rows(b, "gemm_nt_trace");
  check_rows(out, "gemm_nt_trace");
  TORCH_CHECK(a.is_contiguous() && b.is_contiguous() && out.is_contiguous(), "gemm_nt_trace: contiguous operands");
  auto tr = torch::zeros({2, 64}, a.options().dtype(torch::kInt64));
  check(dsa_gemm_nt_trace(a.data_ptr(), b.data_ptr(), out.data_ptr(), a.size(0), b.size(0), a.size(1),
                          reinterpret_cast<unsigned long long*>(tr.data_ptr()), stream()),
        "gemm_nt_trace");
  return tr;
}

bool gemm_km_supported(int64_t M, int64_t N, int64_t K) { return dsa_gemm_km_supported(M, N, K); }

bool fp8_rows_gemm_supported(int64_t M, int64_t N, int64_t K, int64_t bm, int64_t S) {
  return dsa_fp8_rows_gemm_supported((int)M, (int)N, (int)K, (int)bm, (int)S);
}

// y[M][N] = bf16(xs[m] ws[n] (xq wq^T)) for a decode batch (M <= 256), e4m3 operands
// (csrc/fp8_gemm.hip); bm = 64 | 128 batch rows per workgroup; S > 1 splits K, with fp32 slabs
// `part` (S * 256 * N floats) and tickets `cnt` ((N / 128) * ceil(M / bm) int32, zero; left zero);
// wimg: wq holds ops.serving.fp8_rows_shuffle(w), the weights as per-tile LDS images
torch::Tensor fp8_rows_gemm(torch::Tensor xq, torch::Tensor xs, torch::Tensor wq, torch::Tensor ws, int64_t bm,
                            int64_t S, c10::optional<torch::Tensor> part, c10::optional<torch::Tensor> cnt,
                            bool wimg) {
  for (auto* t : {&xq, &wq}) {
    TORCH_CHECK(t->is_cuda() && t->element_size() == 1 && t->dim() == 2 && t->stride(1) == 1,
                "fp8_rows_gemm: 1-byte 2-D operands with contiguous rows");
    TORCH_CHECK(t->stride(0) % 16 == 0 && reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                "fp8_rows_gemm: 16-byte aligned rows");
  }
  const int64_t M = xq.size(0), K = xq.size(1), N = wq.size(0);
  TORCH_CHECK(wq.size(1) == K, "fp8_rows_gemm: K mismatch");
  TORCH_CHECK(!wimg || wq.is_contiguous(), "fp8_rows_gemm: an LDS-image weight is one contiguous block");
  TORCH_CHECK(xs.is_cuda() && xs.scalar_type() == torch::kFloat32 && xs.is_contiguous() && xs.numel() == M,
              "fp8_rows_gemm: xs fp32 [M]");
  TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == torch::kFloat32 && ws.is_contiguous() && ws.numel() == N,
              "fp8_rows_gemm: ws fp32 [N]");
  TORCH_CHECK(dsa_fp8_rows_gemm_supported((int)M, (int)N, (int)K, (int)bm, (int)S),
              "fp8_rows_gemm: M <= 256, N % 128 == 0, bm 64 | 128, K % (128 S) == 0");
  float* pp = nullptr;
  int* cp = nullptr;
  if (S > 1) {
    TORCH_CHECK(part.has_value() && cnt.has_value(), "fp8_rows_gemm: split-K needs part and cnt");
    TORCH_CHECK(part->is_cuda() && part->scalar_type() == torch::kFloat32 && part->numel() >= S * 256 * N,
                "fp8_rows_gemm: part needs S * 256 * N floats");
    TORCH_CHECK(cnt->is_cuda() && cnt->scalar_type() == torch::kInt32 &&
                    cnt->numel() >= (N / 128) * ((M + bm - 1) / bm),
                "fp8_rows_gemm: cnt needs one int32 per output tile");
    pp = part->data_ptr<float>();
    cp = cnt->data_ptr<int>();
  }
  auto y = torch::empty({M, N}, xq.options().dtype(torch::kBFloat16));
  check(dsa_fp8_rows_gemm(xq.data_ptr(), xs.data_ptr<float>(), wq.data_ptr(), ws.data_ptr<float>(), y.data_ptr(), pp,
                          cp, (int)M, (int)N, (int)K, xq.stride(0), wq.stride(0), y.stride(0), (int)bm, (int)S,
                          (int)wimg, stream()),
        "fp8_rows_gemm");
  return y;
}

bool fp8_stream_gemm_supported(int64_t M, int64_t N, int64_t K, int64_t rw, int64_t S) {
  return dsa_fp8_stream_gemm_supported((int)M, (int)N, (int)K, (int)rw, (int)S);
}

// y[M][N] = bf16(xs[m] ws[n] (xq wq^T)) for a decode batch of up to 256 rows with the weights streamed
// straight into registers (csrc/fp8_gemm.hip fp8_stream_gemm); rw = 64 | 32 weight rows per wave,
// S > 1 splits K (fp32 partials allocated here, added by a second kernel); shuffled 1 | 2: wq [N][K] holds
// the weights in ops.serving.fp8_stream_shuffle(wq, group=16 | 256) order
torch::Tensor fp8_stream_gemm(torch::Tensor xq, torch::Tensor xs, torch::Tensor wq, torch::Tensor ws, int64_t rw,
                              int64_t S, int64_t shuffled, int64_t depth) {
  for (auto* t : {&xq, &wq}) {
    TORCH_CHECK(t->is_cuda() && t->element_size() == 1 && t->dim() == 2 && t->stride(1) == 1,
                "fp8_stream_gemm: 1-byte 2-D operands with contiguous rows");
    TORCH_CHECK(t->stride(0) % 16 == 0 && reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                "fp8_stream_gemm: 16-byte aligned rows");
  }
  const int64_t M = xq.size(0), K = xq.size(1), N = wq.size(0);
  TORCH_CHECK(wq.size(1) == K, "fp8_stream_gemm: K mismatch");
  TORCH_CHECK(shuffled >= 0 && shuffled <= 2 && (!shuffled || wq.is_contiguous()),
              "fp8_stream_gemm: shuffled 0 | 1 | 2, a shuffled weight one contiguous block");
  TORCH_CHECK(xs.is_cuda() && xs.scalar_type() == torch::kFloat32 && xs.is_contiguous() && xs.numel() == M,
              "fp8_stream_gemm: xs fp32 [M]");
  TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == torch::kFloat32 && ws.is_contiguous() && ws.numel() == N,
              "fp8_stream_gemm: ws fp32 [N]");
  TORCH_CHECK(dsa_fp8_stream_gemm_supported((int)M, (int)N, (int)K, (int)rw, (int)S),
              "fp8_stream_gemm: M <= 256, rw 32 (or 64 without split), N % 256 == 0, K % (512 S) == 0");
  auto y = torch::empty({M, N}, xq.options().dtype(torch::kBFloat16));
  torch::Tensor part;
  if (S > 1) part = torch::empty({S, M, N}, xq.options().dtype(torch::kFloat32));
  check(dsa_fp8_stream_gemm(xq.data_ptr(), xs.data_ptr<float>(), wq.data_ptr(), ws.data_ptr<float>(), y.data_ptr(),
                            S > 1 ? part.data_ptr<float>() : nullptr, (int)M, (int)N, (int)K, xq.stride(0),
                            wq.stride(0), y.stride(0), (int)rw, (int)S, (int)shuffled, (int)depth, stream()),
        "fp8_stream_gemm");
  return y;
}

// out[M][N] (+)= a[K][M]^T b[K][N]  (csrc/gemm_nt.hip KM form: dW = dY^T X, token-major operands);
// mode 2 = timing-only
void gemm_km(torch::Tensor a, torch::Tensor b, torch::Tensor out, int64_t mode) {
  check_rows(a, "gemm_km");
  check_rows(b, "gemm_km");
  check_rows(out, "gemm_km");
  const int64_t K = a.size(0), M = a.size(1), N = b.size(1);
  TORCH_CHECK(b.size(0) == K && out.size(0) == M && out.size(1) == N, "gemm_km: shape mismatch");
  TORCH_CHECK(dsa_gemm_km_supported(M, N, K), "gemm_km: M % 256, N % 256, K % 128 must be 0");
  check(dsa_gemm_km(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, a.stride(0), b.stride(0), out.stride(0),
                    (int)mode, stream()),
        "gemm_km");
}

// weight gradient with an fp32 accumulator acc [M][N]: mode 0 acc = a^T b, 1 acc += a^T b, 2 out (bf16)
// = acc + a^T b (the last micro-batch, one rounding)
void gemm_km_f32(torch::Tensor a, torch::Tensor b, torch::Tensor acc, c10::optional<torch::Tensor> out, int64_t mode) {
  check_rows(a, "gemm_km_f32");
  check_rows(b, "gemm_km_f32");
  TORCH_CHECK(acc.is_cuda() && acc.scalar_type() == torch::kFloat32 && acc.dim() == 2 && acc.stride(1) == 1,
              "gemm_km_f32: acc must be a row-major fp32 CUDA matrix");
  const int64_t K = a.size(0), M = a.size(1), N = b.size(1);
  TORCH_CHECK(b.size(0) == K && acc.size(0) == M && acc.size(1) == N, "gemm_km_f32: shape mismatch");
  TORCH_CHECK(dsa_gemm_km_supported(M, N, K), "gemm_km_f32: M % 256, N % 256, K % 128 must be 0");
  void* o = nullptr;
  long ldo = 0;
  if (mode == 2) {
    TORCH_CHECK(out.has_value(), "gemm_km_f32: mode 2 writes the bf16 `out`");
    check_rows(*out, "gemm_km_f32");
    TORCH_CHECK(out->size(0) == M && out->size(1) == N, "gemm_km_f32: out shape mismatch");
    o = out->data_ptr();
    ldo = out->stride(0);
  }
  check(dsa_gemm_km_f32(a.data_ptr(), b.data_ptr(), o, acc.data_ptr<float>(), M, N, K, a.stride(0), b.stride(0), ldo,
                        acc.stride(0), (int)mode, stream()),
        "gemm_km_f32");
}

// diagnostic: hold `blocks` workgroup slots for `us` microseconds on the current stream
void cu_hog(int64_t blocks, int64_t threads, int64_t lds_bytes, double us, torch::Tensor sink) {
  TORCH_CHECK(sink.is_cuda() && sink.scalar_type() == torch::kInt32, "cu_hog: int32 CUDA sink");
  check(dsa_cu_hog((int)blocks, (int)threads, (int)lds_bytes, us, sink.data_ptr<int>(), stream()), "cu_hog");
}

// the bench's synthetic token stream (workloads/data.py, csrc/data.hip): out [n] int64, ws [n] int64
void synthetic_tokens(torch::Tensor cdf, torch::Tensor perm, torch::Tensor pow_a, torch::Tensor geo_b,
                      torch::Tensor out, torch::Tensor ws, int64_t key, double copy_p, int64_t row_len) {
  TORCH_CHECK(cdf.is_cuda() && cdf.scalar_type() == torch::kFloat64 && cdf.is_contiguous(), "synthetic_tokens: cdf");
  for (auto* t : {&perm, &pow_a, &geo_b, &out, &ws})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kInt64 && t->is_contiguous(),
                "synthetic_tokens: int64 CUDA tensors expected");
  const int64_t n = out.numel(), V = cdf.numel();
  TORCH_CHECK(perm.numel() == V && ws.numel() >= n && pow_a.numel() > n && geo_b.numel() > n,
              "synthetic_tokens: shape mismatch");
  check(dsa_synthetic_tokens(cdf.data_ptr<double>(), perm.data_ptr<int64_t>(), pow_a.data_ptr<int64_t>(),
                             geo_b.data_ptr<int64_t>(), out.data_ptr<int64_t>(), ws.data_ptr<int64_t>(), (uint64_t)key,
                             (float)copy_p, (int)n, (int)row_len, (int)V, stream()),
        "synthetic_tokens");
}

// gu = x w^T (w = [gate; up] [2F][K]) -> (gu [T][2F], a = silu(g) * u [T][F], a^T [F][T]); with
// transposed = false a^T is not written (returned empty)
std::vector<torch::Tensor> gemm_nt_swiglu(torch::Tensor x, torch::Tensor w, bool transposed) {
  check_rows(x, "gemm_nt_swiglu");
  check_rows(w, "gemm_nt_swiglu");
  const int64_t T = x.size(0), K = x.size(1), F = w.size(0) / 2;
  TORCH_CHECK(w.size(1) == K && w.size(0) == 2 * F, "gemm_nt_swiglu: shape mismatch");
  TORCH_CHECK(dsa_gemm_nt_swiglu_supported(T, F, K), "gemm_nt_swiglu: T % 256, F % 128, K % 128 must be 0");
  auto gu = torch::empty({T, 2 * F}, x.options());
  auto a = torch::empty({T, F}, x.options());
  auto aT = transposed ? torch::empty({F, T}, x.options()) : torch::empty({0}, x.options());
  check(dsa_gemm_nt_swiglu(x.data_ptr(), w.data_ptr(), gu.data_ptr(), a.data_ptr(), transposed ? aT.data_ptr() : nullptr, T, F, K,
                           x.stride(0), w.stride(0), stream()),
        "gemm_nt_swiglu");
  return {gu, a, aT};
}

bool gemm_nt_swiglu_bwd_supported(int64_t T, int64_t F, int64_t K) {
  return dsa_gemm_nt_swiglu_bwd_supported(T, F, K);
}

// da = dy wdT^T (wdT = W_down^T [F][K]) fused with the SwiGLU backward -> (dgu [T][2F], dgu^T [2F][T])
std::vector<torch::Tensor> gemm_nt_swiglu_bwd(torch::Tensor dy, torch::Tensor wdT, torch::Tensor gu, bool transposed) {
  check_rows(dy, "gemm_nt_swiglu_bwd");
  check_rows(wdT, "gemm_nt_swiglu_bwd");
  const int64_t T = dy.size(0), K = dy.size(1), F = wdT.size(0);
  TORCH_CHECK(wdT.size(1) == K, "gemm_nt_swiglu_bwd: shape mismatch");
  TORCH_CHECK(gu.is_cuda() && gu.scalar_type() == torch::kBFloat16 && gu.is_contiguous() && gu.numel() == T * 2 * F,
              "gemm_nt_swiglu_bwd: gu must be a contiguous bf16 [T, 2F]");
  TORCH_CHECK(dsa_gemm_nt_swiglu_bwd_supported(T, F, K), "gemm_nt_swiglu_bwd: T % 256, F % 256, K % 128 must be 0");
  auto dgu = torch::empty({T, 2 * F}, dy.options());
  auto dguT = transposed ? torch::empty({2 * F, T}, dy.options()) : torch::empty({0}, dy.options());
  check(dsa_gemm_nt_swiglu_bwd(dy.data_ptr(), wdT.data_ptr(), gu.data_ptr(), dgu.data_ptr(), transposed ? dguT.data_ptr() : nullptr, T, F,
                               K, dy.stride(0), wdT.stride(0), stream()),
        "gemm_nt_swiglu_bwd");
  return {dgu, dguT};
}

// out[P][Q] (+)= a^T b ; a = [T][P], b = [T][Q] (weight gradient dW = dY^T X)
void gemm_tn(torch::Tensor a, torch::Tensor b, torch::Tensor out, bool accumulate) {
  for (auto* t : {&a, &b, &out}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kBFloat16 && t->dim() == 2, "gemm_tn: 2-D bf16 tensors");
    TORCH_CHECK(t->stride(1) == 1, "gemm_tn: rows must be contiguous");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "gemm_tn: 16-byte aligned base");
  }
  const int64_t T = a.size(0), P = a.size(1), Q = b.size(1);
  TORCH_CHECK(b.size(0) == T && out.size(0) == P && out.size(1) == Q, "gemm_tn: shape mismatch");
  check(dsa_gemm_tn(a.data_ptr(), b.data_ptr(), out.data_ptr(), P, Q, T, a.stride(0), b.stride(0), out.stride(0),
                    accumulate ? 1 : 0, stream()),
        "gemm_tn");
}

// ---- serving: paged KV cache (k [P][KVH][64][128], v [P][KVH][128][64]) ----
void check_i32(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kInt32 && t.is_contiguous(), name,
              " must be a contiguous int32 ROCm tensor");
}

// returns true for an fp8 (e4m3) cache, false for bf16
bool check_cache(const torch::Tensor& k, const torch::Tensor& v, int64_t KVH) {
  const bool fp8 = k.scalar_type() == torch::kFloat8_e4m3fn;
  if (fp8) {
    TORCH_CHECK(k.is_cuda() && k.is_contiguous() && v.is_cuda() && v.is_contiguous() &&
                    v.scalar_type() == torch::kFloat8_e4m3fn,
                "fp8 k_cache / v_cache must both be contiguous float8_e4m3fn");
  } else {
    check_bf16(k, "k_cache");
    check_bf16(v, "v_cache");
  }
  const int64_t P = dsa_paged_page_size();
  TORCH_CHECK(k.dim() == 4 && k.size(1) == KVH && k.size(2) == P && k.size(3) == 128,
              "k_cache must be [pages, KVH, 64, 128]");
  TORCH_CHECK(v.dim() == 4 && v.size(0) == k.size(0) && v.size(1) == KVH && v.size(2) == 128 && v.size(3) == P,
              "v_cache must be [pages, KVH, 128, 64]");
  return fp8;
}

// rotates q/k of qkv [T, (H+2KVH)*128] in place and writes k, v of each token to its cache slot;
// rs [T] / cs [(H+2KVH)*128] (optional, together): qkv is a raw fp8 GEMM product whose row-wise
// scales are applied first (and written back for every head)
void rope_cache_write(torch::Tensor qkv, torch::Tensor positions, torch::Tensor slots, torch::Tensor cos,
                      torch::Tensor sin, torch::Tensor k_cache, torch::Tensor v_cache, int64_t H, int64_t KVH,
                      double k_scale, double v_scale, c10::optional<torch::Tensor> rs,
                      c10::optional<torch::Tensor> cs) {
  check_bf16(qkv, "qkv");
  check_i32(positions, "positions");
  check_i32(slots, "slots");
  const bool fp8 = check_cache(k_cache, v_cache, KVH);
  TORCH_CHECK(k_scale > 0 && v_scale > 0, "kv cache scales must be positive");
  const int64_t T = positions.numel();
  TORCH_CHECK(slots.numel() == T && qkv.numel() == T * (H + 2 * KVH) * 128, "rope_cache_write: shape mismatch");
  TORCH_CHECK(cos.scalar_type() == torch::kFloat32 && sin.scalar_type() == torch::kFloat32 && cos.is_contiguous() &&
                  sin.is_contiguous() && cos.size(1) == 64 && sin.sizes() == cos.sizes(),
              "rope tables must be fp32 [max_pos, 64]");
  TORCH_CHECK(rs.has_value() == cs.has_value(), "rope_cache_write: rs and cs go together");
  const float* rp = nullptr;
  const float* cp = nullptr;
  if (rs.has_value()) {
    TORCH_CHECK(qkv.is_contiguous(), "rope_cache_write: a raw product must be contiguous");
    TORCH_CHECK(rs->scalar_type() == torch::kFloat32 && rs->is_contiguous() && rs->numel() == T,
                "rope_cache_write: rs must be fp32 [T]");
    TORCH_CHECK(cs->scalar_type() == torch::kFloat32 && cs->is_contiguous() && cs->numel() == (H + 2 * KVH) * 128 &&
                    reinterpret_cast<uintptr_t>(cs->data_ptr()) % 16 == 0,
                "rope_cache_write: cs must be fp32 [(H+2KVH)*128], 16-byte aligned");
    rp = rs->data_ptr<float>();
    cp = cs->data_ptr<float>();
  }
  check(dsa_rope_cache_write(qkv.data_ptr(), positions.data_ptr<int>(), slots.data_ptr<int>(), cos.data_ptr<float>(),
                             sin.data_ptr<float>(), k_cache.data_ptr(), v_cache.data_ptr(), (int)T, (int)H, (int)KVH,
                             fp8 ? 1 : 0, (float)k_scale, (float)v_scale, rp, cp, stream()),
        "rope_cache_write");
}

// q: [B, >= H*128] rows (e.g. the fused qkv output; its row stride is passed); out [B, H*128] bf16.
// o_part / lse_part: fp32 workspaces of >= B*H*nsplit*128 and B*H*nsplit elements (unused when nsplit == 1)
void paged_decode(torch::Tensor q, torch::Tensor k_cache, torch::Tensor v_cache, torch::Tensor block_tables,
                  torch::Tensor ctx_lens, torch::Tensor out, torch::Tensor o_part, torch::Tensor lse_part, int64_t H,
                  int64_t KVH, int64_t nsplit, int64_t pages_per_split, double scale, double k_scale,
                  double v_scale) {
  TORCH_CHECK(q.is_cuda() && q.scalar_type() == torch::kBFloat16 && q.dim() == 2 && q.stride(1) == 1 &&
                  q.size(1) >= H * 128 && q.stride(0) % 8 == 0,
              "q must be bf16 [B, >= H*128] with contiguous rows");
  const bool fp8 = check_cache(k_cache, v_cache, KVH);
  check_i32(block_tables, "block_tables");
  check_i32(ctx_lens, "ctx_lens");
  check_bf16(out, "out");
  const int64_t B = q.size(0);
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(0) == B && ctx_lens.numel() == B, "batch mismatch");
  TORCH_CHECK(nsplit * pages_per_split >= block_tables.size(1), "splits do not cover the block table");
  TORCH_CHECK(out.numel() == B * H * 128, "out must be [B, H*128]");
  if (nsplit > 1) {
    TORCH_CHECK(o_part.scalar_type() == torch::kFloat32 && o_part.numel() >= B * H * nsplit * 128 &&
                    lse_part.scalar_type() == torch::kFloat32 && lse_part.numel() >= B * H * nsplit,
                "paged_decode: split workspaces too small");
  }
  check(dsa_paged_decode(q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                         block_tables.data_ptr<int>(), (int)block_tables.stride(0), ctx_lens.data_ptr<int>(),
                         out.data_ptr(), nsplit > 1 ? o_part.data_ptr<float>() : nullptr,
                         nsplit > 1 ? lse_part.data_ptr<float>() : nullptr, (int)B, (int)H, (int)KVH, (int)nsplit,
                         (int)pages_per_split, (float)scale, fp8 ? 1 : 0, (float)k_scale, (float)v_scale, stream()),
        "paged_decode");
}

// tokens (int32 [rows]) and log-probs (fp32 [rows]) written in place; temps fp32, seeds int64, steps int32
void sample(torch::Tensor logits, torch::Tensor temps, torch::Tensor seeds, torch::Tensor steps, torch::Tensor tokens,
            torch::Tensor logprobs) {
  TORCH_CHECK(logits.is_cuda() && logits.scalar_type() == torch::kBFloat16 && logits.dim() == 2 &&
                  logits.stride(1) == 1,
              "logits must be bf16 [rows, V] with contiguous rows");
  const int64_t rows = logits.size(0);
  TORCH_CHECK(temps.scalar_type() == torch::kFloat32 && temps.numel() == rows && temps.is_contiguous(), "temps");
  TORCH_CHECK(seeds.scalar_type() == torch::kInt64 && seeds.numel() == rows && seeds.is_contiguous(), "seeds");
  check_i32(steps, "steps");
  check_i32(tokens, "tokens");
  TORCH_CHECK(steps.numel() == rows && tokens.numel() == rows, "sample: rows mismatch");
  TORCH_CHECK(logprobs.scalar_type() == torch::kFloat32 && logprobs.numel() == rows, "logprobs fp32 [rows]");
  check(dsa_sample(logits.data_ptr(), logits.stride(0), (int)rows, (int)logits.size(1), temps.data_ptr<float>(),
                   seeds.data_ptr<int64_t>(), steps.data_ptr<int>(), tokens.data_ptr<int>(), logprobs.data_ptr<float>(),
                   stream()),
        "sample");
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "dstack_amd HIP/CDNA4 kernels (gfx950)";
  m.def("rms_norm_fwd", &rms_norm_fwd);
  m.def("add_rms_norm_fwd", &add_rms_norm_fwd);
  m.def("rms_norm_bwd", &rms_norm_bwd, py::arg("dy"), py::arg("h"), py::arg("w"), py::arg("rstd"),
        py::arg("dres") = py::none(), py::arg("dw_out") = py::none(), py::arg("accumulate") = false);
  m.def("swiglu_fwd", &swiglu_fwd);
  m.def("transpose2d", &transpose2d);
  m.def("swiglu_fwd_t", &swiglu_fwd_t);
  m.def("transpose2d_supported", &transpose2d_supported);
  m.def("swiglu_bwd", &swiglu_bwd);
  m.def("swiglu_bwd_t", &swiglu_bwd_t);
  m.def("rope_qkv", &rope_qkv);
  m.def("cross_entropy_fwd", &cross_entropy_fwd);
  m.def("cross_entropy_bwd", &cross_entropy_bwd);
  m.def("adamw", &adamw);
  m.def("embedding_bwd", &embedding_bwd);
  m.def("flash_attn_fwd", &flash_attn_fwd);
  m.def("flash_attn_bwd", &flash_attn_bwd, py::arg("dout"), py::arg("qkv"), py::arg("out"), py::arg("lse"),
        py::arg("H"), py::arg("KVH"), py::arg("causal"), py::arg("rope_cos") = py::none(),
        py::arg("rope_sin") = py::none());
  m.def("fa_dkdv_trace", &fa_dkdv_trace);
  m.def("quant_fp8_rows", &quant_fp8_rows);
  m.def("rms_norm_fp8", &rms_norm_fp8, py::arg("x"), py::arg("delta"), py::arg("w"), py::arg("eps"),
        py::arg("dr") = py::none(), py::arg("dc") = py::none());
  m.def("rms_norm_fp8_supported", &rms_norm_fp8_supported);
  m.def("gemv_fp8", &gemv_fp8);
  m.def("gemv_fp8_supported", &gemv_fp8_supported);
  m.def("gemm_tn", &gemm_tn);
  m.def("gemm_tn_supported", &gemm_tn_supported);
  m.def("gemm_nt", &gemm_nt);
  m.def("gemm_nt_mode", &gemm_nt_mode);
  m.def("gemm_nt_supported", &gemm_nt_supported);
  m.def("gemm_nt_swiglu", &gemm_nt_swiglu, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("transposed") = true);
  m.def("gemm_km", &gemm_km, pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("out"), pybind11::arg("mode") = 0);
  m.def("gemm_km_supported", &gemm_km_supported);
  m.def("synthetic_tokens", &synthetic_tokens);
  m.def("cu_hog", &cu_hog);
  m.def("gemm_km_f32", &gemm_km_f32, pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("acc"),
        pybind11::arg("out") = pybind11::none(), pybind11::arg("mode") = 0);
  m.def("fp8_rows_gemm", &fp8_rows_gemm, pybind11::arg("xq"), pybind11::arg("xs"), pybind11::arg("wq"),
        pybind11::arg("ws"), pybind11::arg("bm") = 64, pybind11::arg("split") = 1, pybind11::arg("part") = pybind11::none(),
        pybind11::arg("cnt") = pybind11::none(), pybind11::arg("wimg") = false);
  m.def("fp8_rows_gemm_supported", &fp8_rows_gemm_supported);
  m.def("fp8_stream_gemm", &fp8_stream_gemm, pybind11::arg("xq"), pybind11::arg("xs"), pybind11::arg("wq"),
        pybind11::arg("ws"), pybind11::arg("rw") = 64, pybind11::arg("split") = 1, pybind11::arg("shuffled") = 0,
        pybind11::arg("depth") = 2);
  m.def("fp8_stream_gemm_supported", &fp8_stream_gemm_supported);
  m.def("swiglu_quant_fp8_rows", &swiglu_quant_fp8_rows, py::arg("gu"), py::arg("rs") = py::none(),
        py::arg("cs") = py::none());
  m.def("scale_rows_cols_", &scale_rows_cols_);
  m.def("gemm_nt_trace", &gemm_nt_trace);
  m.def("gemm_nt_rope", &gemm_nt_rope);
  m.def("gemm_nt_f8", &gemm_nt_f8);
  m.def("gemm_nt_set_grid", [](int64_t mode) { dsa_gemm_nt_set_grid((int)mode); },
        "in-tree GEMM grid form: -1 environment default, 0 one workgroup per tile, 1 persistent");
  m.def("gemm_nt_f8_supported", &gemm_nt_f8_supported);
  m.def("gemm_nt_f8_swiglu_quant", &gemm_nt_f8_swiglu_quant);
  m.def("gemm_nt_f8_swiglu_supported", &gemm_nt_f8_swiglu_supported);
  m.def("gemm_nt_rope_supported", &gemm_nt_rope_supported);
  m.def("gemm_nt_swiglu_supported", &gemm_nt_swiglu_supported);
  m.def("gemm_nt_swiglu_bwd", &gemm_nt_swiglu_bwd, pybind11::arg("dy"), pybind11::arg("wdT"), pybind11::arg("gu"),
        pybind11::arg("transposed") = true);
  m.def("gemm_nt_swiglu_bwd_supported", &gemm_nt_swiglu_bwd_supported);
  m.def("gemv", &gemv);
  m.def("gemv_supported", &gemv_supported);
  m.def("paged_page_size", &dsa_paged_page_size);
  m.def("rope_cache_write", &rope_cache_write, py::arg("qkv"), py::arg("positions"), py::arg("slots"), py::arg("cos"),
        py::arg("sin"), py::arg("k_cache"), py::arg("v_cache"), py::arg("H"), py::arg("KVH"), py::arg("k_scale"),
        py::arg("v_scale"), py::arg("rs") = py::none(), py::arg("cs") = py::none());
  m.def("paged_decode", &paged_decode);
  m.def("sample", &sample);
}
