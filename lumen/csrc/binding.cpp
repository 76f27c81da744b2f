// Python binding for lumen's native ops (built into lumen/_C*.so by lumen/csrc/build.py).
//
// Every function here only checks arguments, picks the dtype code and the current HIP stream,
// and calls an `extern "C"` launcher from kernels/*.hip.  Allocation and shape logic live in
// lumen/ops/*.py so this translation unit (the only one that includes the heavy torch headers)
// rarely changes.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

extern "C" {
hipError_t lumen_rmsnorm_fwd(int, const void*, const void*, const void*, void*, void*, float*, int,
                             int, float, hipStream_t);
hipError_t lumen_rmsnorm_bwd(int, const void*, const void*, const void*, const float*, const void*,
                             void*, float*, int, int, hipStream_t);
hipError_t lumen_qkv_rope(int, int, void*, void*, void*, void*, const int*, const float*,
                          const float*, int, int, int, int, int, hipStream_t);
hipError_t lumen_rope_inplace(int, void*, const int*, const float*, const float*, int, int, int,
                              int, hipStream_t);
hipError_t lumen_swiglu(int, int, const void*, const void*, void*, int, int, int, int, hipStream_t);
hipError_t lumen_scale_dev(int, void*, long long, const float*, const float*, hipStream_t);
hipError_t lumen_cross_entropy(int, void*, const int64_t*, float*, float*, int, int, int, float,
                               int, const float*, hipStream_t);
hipError_t lumen_grad_norm_sq(int, const void*, long long, float*, hipStream_t);
hipError_t lumen_adamw(float*, int, const void*, float*, float*, int, void*, long long, float, float,
                       float, float, float, float, float, float, const float*, float, float*,
                       const double*, hipStream_t);
hipError_t lumen_lora_gemm(int, int, int, const void*, const void*, void*, long long, long long,
                           long long, long long, float, int, unsigned long long, unsigned int, float,
                           long long, int, const long long*, const long long*, const long long*,
                           const int*, const int*, const int*, hipStream_t);
hipError_t lumen_lora2(int, int, int, const void*, long long, const float*, long long, void*,
                       long long, long long, float, int, int, int, unsigned long long, unsigned int,
                       float, long long, long long, int, const long long*, const long long*,
                       const long long*, const int*, const float*, const float*, const int*, int,
                       hipStream_t);
hipError_t lumen_rmsnorm_fwd_ld(int, const void*, const void*, const void*, void*, void*, float*,
                                int, int, float, long long, hipStream_t);
hipError_t lumen_lora3_z_tail(int, const float*, int, void*, long long, int, int, int, hipStream_t);
hipError_t lumen_lora3_w_tail_batch(int, const long long*, int, long long, hipStream_t);
hipError_t lumen_lora3_w_tail(int, void*, long long, int, const float*, int, int, const long long*,
                              const long long*, const int*, const int*, float, hipStream_t);
hipError_t lumen_lora3_dxa(int, const void*, long long, void*, long long, const float*, const float*,
                           long long, float*, long long, int, int, int, int, unsigned long long,
                           unsigned int, float, long long, long long, float*, float*, unsigned*,
                           hipStream_t);
hipError_t lumen_embedding(const void*, const long long*, void*, int, int, int, hipStream_t);
hipError_t lumen_lora3_down(int, const void*, long long, const float*, long long, float*, long long,
                            int, int, int, float, unsigned long long, unsigned int, float, long long,
                            long long, void*, long long, int, int, unsigned*, float*, hipStream_t);
hipError_t lumen_lora3_up(int, int, void*, long long, const float*, long long, const float*,
                          long long, int, int, float, unsigned long long, unsigned int, float,
                          long long, long long, int, const long long*, const long long*,
                          const long long*, const int*, const float*, const float*, const int*,
                          int, hipStream_t);
hipError_t lumen_lora3_dy(int, const void*, long long, const float*, int, const float*, long long,
                          float*, long long, float*, int, int, float, int, const long long*,
                          const long long*, const long long*, const int*, float*, float*,
                          unsigned*, unsigned*, hipStream_t);
hipError_t lumen_transpose(int, const void*, void*, int, int, long long, long long, hipStream_t);
hipError_t lumen_rope_cache(int, void*, long long, const int*, const float*, const float*, void*,
                            void*, const long long*, int, int, int, int, int, int, hipStream_t);
hipError_t lumen_skinny_swiglu_gemm(int, const void*, const void*, void*, int, int, int, long long,
                                    long long, hipStream_t);
hipError_t lumen_skinny_gemm(int, const void*, const void*, void*, int, int, int, long long,
                             long long, hipStream_t);
hipError_t lumen_decode_gemm(int, const void*, const void*, void*, float*, int*, int, int, int,
                             long long, long long, int, int, int, int, int, hipStream_t);
hipError_t lumen_mlp_gemm(int, int, const void*, long long, const void*, long long, void*, long long,
                          void*, long long, const void*, long long, int, int, int, int, int, float*,
                          int*, int, hipStream_t);
int lumen_mlp_gemm_split(int, int, int, int, int);
hipError_t lumen_hbm_read(const void*, long long, unsigned*, int, hipStream_t);
void lumen_set_gemv_form(int);
void lumen_set_rms_lds(int, int);
hipError_t lumen_paged_attention_decode(int, void*, const void*, const void*, const void*,
                                        const int*, const int*, int, int, int, int, int, int, int,
                                        float, float*, float*, void*, int, unsigned*, int, int,
                                        int, hipStream_t);
hipError_t lumen_kv_dequant(int, const void*, const void*, void*, void*, const int*, int,
                            const int*, int, int, int, int, int, hipStream_t);
hipError_t lumen_reshape_and_cache(int, const void*, const void*, void*, void*, const long long*,
                                   int, int, int, int, long long, long long, int, hipStream_t);
hipError_t lumen_sample(int, const void*, const float*, const float*, const int*,
                        unsigned long long, long long, long long*, float*, float*, int, int,
                        hipStream_t);
hipError_t lumen_flash_attn_paged(int, int, const void*, long long, const void*, const void*, void*,
                                  long long, const int*, const int*, const int*, int, const int*,
                                  int, int, int, int, int, float, hipStream_t);
hipError_t lumen_flash_attn(int, int, int, int, const void*, const void*, const void*, long long,
                            long long, long long, void*, long long, float*, const int*, const int*,
                            int, int, int, int, float, const void*, long long, void*, void*, void*,
                            long long, long long, long long, const float*, const int*, const float*,
                            const float*, hipStream_t);
hipError_t lumen_flash_attn_ds(int, int, int, const void*, const void*, const void*, long long,
                               long long, long long, const float*, const int*, const int*, int, int,
                               int, int, float, const void*, long long, void*, void*, void*,
                               long long, long long, long long, const float*, const int*,
                               const float*, const float*, void*, const int*, int, hipStream_t);
long long lumen_car_signal_bytes();
int lumen_car_max_blocks();
int lumen_car_max_ranks();
hipError_t lumen_car_alloc(long long, int, void**);
hipError_t lumen_car_free(void*);
hipError_t lumen_car_get_handle(void*, void*);
int lumen_car_handle_bytes();
hipError_t lumen_car_open_handle(const void*, void**);
hipError_t lumen_car_close_handle(void*);
hipError_t lumen_car_read_err(void*, unsigned int*);
hipError_t lumen_car_read_diag(void*, unsigned int*);
hipError_t lumen_car_allreduce(int, const long long*, const long long*, int, int, const void*,
                               void*, long long, int, int, double, void*, hipStream_t);
hipError_t lumen_car_allgather(int, const long long*, const long long*, int, int, const void*,
                               void*, long long, long long, int, double, void*, hipStream_t);
hipError_t lumen_car_host_flag_alloc(void**, void**);
hipError_t lumen_car_host_flag_free(void*);
void lumen_cpu_adamw(float*, const float*, float*, float*, long long, float, float, float, float,
                     float, float, float, float);
int lumen_cpu_has_avx512();
}

namespace {

int dcode(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kHalf: return 1;
    case at::kBFloat16: return 2;
    default: throw std::invalid_argument("lumen: unsupported dtype " + std::string(toString(t.scalar_type())));
  }
}

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check(hipError_t e, const char* what) {
  if (e != hipSuccess)
    throw std::runtime_error(std::string("lumen native op ") + what + " failed: " + hipGetErrorString(e));
}

void need_cuda(const at::Tensor& t, const char* name) {
  if (!t.is_cuda()) throw std::invalid_argument(std::string("lumen: ") + name + " must be a GPU tensor");
  if (!t.is_contiguous()) throw std::invalid_argument(std::string("lumen: ") + name + " must be contiguous");
}

template <typename T = void>
T* ptr(const std::optional<at::Tensor>& t) {
  return t.has_value() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

void rmsnorm_fwd(const at::Tensor& x, const std::optional<at::Tensor>& residual, const at::Tensor& w,
                 at::Tensor& y, const std::optional<at::Tensor>& s_out, at::Tensor& rstd, double eps) {
  need_cuda(x, "x"); need_cuda(w, "w");
  if (!y.is_cuda()) throw std::invalid_argument("lumen: y must be a GPU tensor");
  const int H = static_cast<int>(x.size(-1));
  const int rows = static_cast<int>(x.numel() / H);
  // y may be a row-strided view (unit column stride): ldy = its row stride
  if (y.stride(-1) != 1 || y.numel() != x.numel())
    throw std::invalid_argument("lumen: rmsnorm_fwd output must have x's shape and unit column stride");
  const long long ldy = y.dim() >= 2 ? y.stride(-2) : H;
  check(lumen_rmsnorm_fwd_ld(dcode(x), x.data_ptr(), ptr(residual), w.data_ptr(), y.data_ptr(),
                             ptr(s_out), rstd.data_ptr<float>(), rows, H, static_cast<float>(eps),
                             ldy, cur_stream()),
        "rmsnorm_fwd");
}

void rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& s, const at::Tensor& w, const at::Tensor& rstd,
                 const std::optional<at::Tensor>& ds_res, at::Tensor& dx,
                 const std::optional<at::Tensor>& dw) {
  need_cuda(dy, "dy"); need_cuda(s, "s");
  const int H = static_cast<int>(dy.size(-1));
  const int rows = static_cast<int>(dy.numel() / H);
  check(lumen_rmsnorm_bwd(dcode(dy), dy.data_ptr(), s.data_ptr(), w.data_ptr(),
                          rstd.data_ptr<float>(), ptr(ds_res), dx.data_ptr(), ptr<float>(dw), rows,
                          H, cur_stream()),
        "rmsnorm_bwd");
}

void qkv_rope(bool bwd, at::Tensor& qkv, at::Tensor& q, at::Tensor& k, at::Tensor& v,
              const std::optional<at::Tensor>& pos, const at::Tensor& cos_t, const at::Tensor& sin_t,
              int64_t S, int64_t nh, int64_t nkv, int64_t D) {
  need_cuda(qkv, "qkv"); need_cuda(q, "q"); need_cuda(k, "k"); need_cuda(v, "v");
  const int T = static_cast<int>(qkv.numel() / ((nh + 2 * nkv) * D));
  check(lumen_qkv_rope(dcode(qkv), bwd ? 1 : 0, qkv.data_ptr(), q.data_ptr(), k.data_ptr(),
                       v.data_ptr(), ptr<const int>(pos), cos_t.data_ptr<float>(),
                       sin_t.data_ptr<float>(), T, static_cast<int>(S), static_cast<int>(nh),
                       static_cast<int>(nkv), static_cast<int>(D), cur_stream()),
        "qkv_rope");
}

void rope_inplace(at::Tensor& x, const at::Tensor& pos, const at::Tensor& cos_t, const at::Tensor& sin_t,
                  int64_t ntok, int64_t row_stride, int64_t nheads, int64_t D) {
  check(lumen_rope_inplace(dcode(x), x.data_ptr(), pos.data_ptr<int>(), cos_t.data_ptr<float>(),
                           sin_t.data_ptr<float>(), static_cast<int>(ntok),
                           static_cast<int>(row_stride), static_cast<int>(nheads),
                           static_cast<int>(D), cur_stream()),
        "rope_inplace");
}

// c1 < 0: the whole row; else columns [c0, c1) of the activation (contiguous gu / dact / out)
void swiglu(bool bwd, const at::Tensor& gu, const std::optional<at::Tensor>& dact, at::Tensor& out,
            int64_t c0, int64_t c1) {
  need_cuda(gu, "gate_up"); need_cuda(out, "out");
  const int F = static_cast<int>(gu.size(-1) / 2);
  const int rows = static_cast<int>(gu.numel() / (2 * F));
  if (!gu.is_contiguous() || !out.is_contiguous() || (dact && !dact->is_contiguous()) ||
      out.numel() != static_cast<int64_t>(rows) * (bwd ? 2 * F : F) ||
      (dact && dact->numel() != static_cast<int64_t>(rows) * F))
    throw std::invalid_argument("lumen: swiglu shape/layout mismatch");
  if (c1 < 0) { c0 = 0; c1 = F; }
  check(lumen_swiglu(dcode(gu), bwd ? 1 : 0, gu.data_ptr(), ptr(dact), out.data_ptr(), rows, F,
                     static_cast<int>(c0), static_cast<int>(c1), cur_stream()),
        "swiglu");
}

// y [M, N] = swiglu(gu [M, 2K]) @ w [N, K]^T, M <= 4 (batch-1..4 decode down projection)
void skinny_swiglu_gemm(const at::Tensor& gu, const at::Tensor& w, at::Tensor& y) {
  if (!gu.is_cuda() || !y.is_cuda()) throw std::invalid_argument("lumen: skinny_swiglu_gemm needs GPU tensors");
  need_cuda(w, "w");
  if (gu.dim() != 2 || w.dim() != 2 || y.dim() != 2 || gu.stride(1) != 1 || y.stride(1) != 1 ||
      !w.is_contiguous() || gu.size(1) != 2 * w.size(1) || y.size(0) != gu.size(0) ||
      y.size(1) != w.size(0) || gu.scalar_type() != w.scalar_type() ||
      y.scalar_type() != w.scalar_type())
    throw std::invalid_argument("lumen: skinny_swiglu_gemm shape/layout mismatch");
  check(lumen_skinny_swiglu_gemm(dcode(w), gu.data_ptr(), w.data_ptr(), y.data_ptr(),
                                 static_cast<int>(gu.size(0)), static_cast<int>(w.size(0)),
                                 static_cast<int>(w.size(1)), gu.stride(0), y.stride(0),
                                 cur_stream()),
        "skinny_swiglu_gemm");
}

void skinny_gemm(const at::Tensor& x, const at::Tensor& w, at::Tensor& y) {
  if (!x.is_cuda() || !y.is_cuda()) throw std::invalid_argument("lumen: skinny_gemm needs GPU tensors");
  need_cuda(w, "w");  // x / y may be row-strided views (unit column stride checked below)
  if (x.dim() != 2 || w.dim() != 2 || y.dim() != 2 || x.stride(1) != 1 || y.stride(1) != 1 ||
      !w.is_contiguous() || x.size(1) != w.size(1) || y.size(0) != x.size(0) ||
      y.size(1) != w.size(0) || x.scalar_type() != w.scalar_type() ||
      y.scalar_type() != w.scalar_type())
    throw std::invalid_argument("lumen: skinny_gemm shape/layout mismatch");
  check(lumen_skinny_gemm(dcode(w), x.data_ptr(), w.data_ptr(), y.data_ptr(),
                          static_cast<int>(x.size(0)), static_cast<int>(w.size(0)),
                          static_cast<int>(w.size(1)), x.stride(0), y.stride(0), cur_stream()),
        "skinny_gemm");
}

// decode-batch MFMA GEMM (kernels/decode_gemm.hip): y = x @ w^T with block tile (bm, bn) and
// split-K s (s > 1: ws f32 slabs + cnt zeroed tile counters)
void decode_gemm(const at::Tensor& x, const at::Tensor& w, at::Tensor& y,
                 const std::optional<at::Tensor>& ws, const std::optional<at::Tensor>& cnt,
                 int64_t bm, int64_t bn, int64_t s, int64_t nw, int64_t flags) {
  if (!x.is_cuda() || !y.is_cuda()) throw std::invalid_argument("lumen: decode_gemm needs GPU tensors");
  need_cuda(w, "w");
  // flags bit 1: x in the k-tiled layout, a contiguous [K / 64, bm, 64] tensor (M = y rows)
  const bool xt = (flags & 2) != 0;
  if (xt ? (!x.is_contiguous() || x.numel() != w.size(1) / 64 * bm * 64 || bm != 256)
         : (x.dim() != 2 || x.stride(1) != 1 || x.size(1) != w.size(1) ||
            y.size(0) != x.size(0)))
    throw std::invalid_argument("lumen: decode_gemm x shape/layout mismatch");
  if (w.dim() != 2 || y.dim() != 2 || y.stride(1) != 1 || !w.is_contiguous() ||
      y.size(1) != w.size(0) || x.scalar_type() != w.scalar_type() ||
      y.scalar_type() != w.scalar_type())
    throw std::invalid_argument("lumen: decode_gemm shape/layout mismatch");
  const long long tiles = (w.size(0) + bn - 1) / bn;
  if (s > 1) {
    if (!ws || !cnt || !ws->is_cuda() || !cnt->is_cuda() ||
        ws->scalar_type() != at::kFloat || cnt->scalar_type() != at::kInt ||
        ws->numel() < tiles * s * bm * bn || cnt->numel() < tiles)
      throw std::invalid_argument("lumen: decode_gemm split-K workspace too small");
  }
  check(lumen_decode_gemm(dcode(w), x.data_ptr(), w.data_ptr(), y.data_ptr(),
                          s > 1 ? ws->data_ptr<float>() : nullptr,
                          s > 1 ? cnt->data_ptr<int>() : nullptr, static_cast<int>(y.size(0)),
                          static_cast<int>(w.size(0)), static_cast<int>(w.size(1)),
                          xt ? w.size(1) : x.stride(0), y.stride(0), static_cast<int>(bm),
                          static_cast<int>(bn), static_cast<int>(nw), static_cast<int>(s),
                          static_cast<int>(flags), cur_stream()),
        "decode_gemm");
}

// training-shape MLP GEMMs with the SwiGLU in the epilogue (kernels/mlp_gemm.hip):
// epi 0: c = x @ w^T; epi 1: c = gu = x @ w^T (w = [gate | up] rows), act = silu(g) * u;
// epi 2: c = dgu from dact = x @ w^T (x = dout, w = Wd^T) and the saved gu
// tiles of the last wave that would run split in two k halves (0: none)
int64_t mlp_gemm_split(int64_t M, int64_t N, int64_t K, int64_t epi, int64_t cus) {
  return lumen_mlp_gemm_split(static_cast<int>(M), static_cast<int>(N), static_cast<int>(K),
                              static_cast<int>(epi), static_cast<int>(cus));
}

void mlp_gemm(int64_t epi, const at::Tensor& x, const at::Tensor& w, at::Tensor& c,
              const std::optional<at::Tensor>& act, const std::optional<at::Tensor>& gu,
              int64_t group_m, const std::optional<at::Tensor>& ws,
              const std::optional<at::Tensor>& cnt, int64_t split) {
  if (!x.is_cuda() || !w.is_cuda() || !c.is_cuda())
    throw std::invalid_argument("lumen: mlp_gemm needs GPU tensors");
  if (x.dim() != 2 || w.dim() != 2 || c.dim() != 2 || x.stride(1) != 1 || w.stride(1) != 1 ||
      c.stride(1) != 1 || x.size(1) != w.size(1) || c.size(0) != x.size(0) ||
      x.scalar_type() != w.scalar_type() || c.scalar_type() != w.scalar_type())
    throw std::invalid_argument("lumen: mlp_gemm shape/layout mismatch");
  const int64_t M = x.size(0), K = x.size(1), Nw = w.size(0);
  int64_t F = 0;
  const int64_t e = epi & 15;  // bit 4: kernel variant (A/B probes)
  if (e == 0) {
    if (c.size(1) != Nw) throw std::invalid_argument("lumen: mlp_gemm c must be [M, N]");
  } else if (e == 1) {
    F = Nw / 2;
    if (!act || !act->is_cuda() || act->dim() != 2 || act->stride(1) != 1 || act->size(0) != M ||
        act->size(1) != F || c.size(1) != 2 * F || act->scalar_type() != w.scalar_type())
      throw std::invalid_argument("lumen: mlp_gemm swiglu operands mismatch");
  } else if (e == 2) {
    F = Nw;
    if (!gu || !gu->is_cuda() || gu->dim() != 2 || gu->stride(1) != 1 || gu->size(0) != M ||
        gu->size(1) != 2 * F || c.size(1) != 2 * F || gu->scalar_type() != w.scalar_type())
      throw std::invalid_argument("lumen: mlp_gemm swiglu-backward operands mismatch");
  } else {
    throw std::invalid_argument("lumen: mlp_gemm epi must be 0, 1 or 2");
  }
  if (split > 0 && (!ws || !cnt || !ws->is_cuda() || !cnt->is_cuda() ||
                    ws->scalar_type() != at::kFloat || cnt->scalar_type() != at::kInt ||
                    ws->numel() < split * 2 * 65536 || cnt->numel() < split))
    throw std::invalid_argument("lumen: mlp_gemm split workspace too small");
  check(lumen_mlp_gemm(dcode(w), static_cast<int>(epi), x.data_ptr(), x.stride(0), w.data_ptr(),
                       w.stride(0), c.data_ptr(), c.stride(0), act ? act->data_ptr() : nullptr,
                       act ? act->stride(0) : 0, gu ? gu->data_ptr() : nullptr,
                       gu ? gu->stride(0) : 0, static_cast<int>(M), static_cast<int>(Nw),
                       static_cast<int>(K), static_cast<int>(F), static_cast<int>(group_m),
                       split > 0 ? ws->data_ptr<float>() : nullptr,
                       split > 0 ? cnt->data_ptr<int>() : nullptr, static_cast<int>(split),
                       cur_stream()),
        "mlp_gemm");
}

// box calibration: a non-temporal read of all of ``buf`` (kernels/calib.hip)
void hbm_read(const at::Tensor& buf, at::Tensor& out, int64_t blocks) {
  need_cuda(buf, "buf"); need_cuda(out, "out");
  if (out.scalar_type() != at::kInt || out.numel() < 1)
    throw std::invalid_argument("lumen: hbm_read out must be an int32 tensor");
  check(lumen_hbm_read(buf.data_ptr(), buf.numel() * buf.element_size(),
                       reinterpret_cast<unsigned*>(out.data_ptr()), static_cast<int>(blocks),
                       cur_stream()),
        "hbm_read");
}

void cross_entropy(at::Tensor& logits, const at::Tensor& labels, const std::optional<at::Tensor>& loss_sum,
                   const std::optional<at::Tensor>& row_loss, int64_t ignore_index, double scale,
                   bool write_grad, const std::optional<at::Tensor>& gscale) {
  need_cuda(logits, "logits"); need_cuda(labels, "labels");
  if (labels.scalar_type() != at::kLong) throw std::invalid_argument("lumen: labels must be int64");
  const int V = static_cast<int>(logits.size(-1));
  const int rows = static_cast<int>(logits.numel() / V);
  check(lumen_cross_entropy(dcode(logits), logits.data_ptr(), labels.data_ptr<int64_t>(),
                            ptr<float>(loss_sum), ptr<float>(row_loss), rows, V,
                            static_cast<int>(ignore_index), static_cast<float>(scale),
                            write_grad ? 1 : 0, ptr<const float>(gscale), cur_stream()),
        "cross_entropy");
}

// x *= num / den (device f32 scalars; den optional), in place, contiguous x
void scale_dev(at::Tensor& x, const at::Tensor& num, const std::optional<at::Tensor>& den) {
  need_cuda(x, "x"); need_cuda(num, "num");
  if (!x.is_contiguous() || num.scalar_type() != at::kFloat || num.numel() < 1 ||
      (den && (den->scalar_type() != at::kFloat || den->numel() < 1)))
    throw std::invalid_argument("lumen: scale_dev needs a contiguous x and f32 scalars");
  check(lumen_scale_dev(dcode(x), x.data_ptr(), x.numel(), num.data_ptr<float>(),
                        ptr<const float>(den), cur_stream()),
        "scale_dev");
}

void grad_norm_sq(const at::Tensor& g, at::Tensor& out) {
  need_cuda(g, "grad");
  check(lumen_grad_norm_sq(dcode(g), g.data_ptr(), g.numel(), out.data_ptr<float>(), cur_stream()),
        "grad_norm_sq");
}

void adamw(at::Tensor& p, const at::Tensor& g, at::Tensor& m, at::Tensor& v,
           const std::optional<at::Tensor>& out_copy, double lr, double b1, double b2, double eps,
           double wd, double bc1, double bc2, double inv_scale,
           const std::optional<at::Tensor>& norm_sq, double max_norm,
           const std::optional<at::Tensor>& step_state, const std::vector<double>& sched) {
  need_cuda(p, "param"); need_cuda(g, "grad"); need_cuda(m, "exp_avg"); need_cuda(v, "exp_avg_sq");
  if (step_state.has_value() && (step_state->scalar_type() != at::kFloat || step_state->numel() < 2))
    throw std::invalid_argument("lumen: adamw step_state must be f32[2] (applied, skipped)");
  if (step_state.has_value() && (step_state->numel() < 8 || sched.size() < 9))
    throw std::invalid_argument("lumen: adamw step_state needs 8 words and 9 schedule values "
                                "(lr_min, lr_max, warm_n, warm_linear, inv_world, dynamic, "
                                "window, hysteresis, min_scale)");
  if (p.scalar_type() != at::kFloat) throw std::invalid_argument("lumen: adamw master must be f32");
  // optional values 10-12 (decay_total, decay_kind, cos_min_ratio) default to 0
  std::vector<double> sched10 = sched;
  if (!sched10.empty() && sched10.size() < 12) sched10.resize(12, 0.0);
  const int od = out_copy.has_value() ? dcode(*out_copy) : 0;
  check(lumen_adamw(p.data_ptr<float>(), dcode(g), g.data_ptr(), m.data_ptr<float>(),
                    v.data_ptr<float>(), od, ptr(out_copy), p.numel(), static_cast<float>(lr),
                    static_cast<float>(b1), static_cast<float>(b2), static_cast<float>(eps),
                    static_cast<float>(wd), static_cast<float>(bc1), static_cast<float>(bc2),
                    static_cast<float>(inv_scale), ptr<const float>(norm_sq),
                    static_cast<float>(max_norm), ptr<float>(step_state),
                    sched10.empty() ? nullptr : sched10.data(), cur_stream()),
        "adamw");
}

void lora_gemm(int64_t act_dtype, int64_t mode, int64_t bn, const at::Tensor& X, const at::Tensor& W,
               at::Tensor& C, int64_t ldx, int64_t ldw, int64_t cs_m, int64_t cs_n, double alpha,
               int64_t ksplit, int64_t seed, int64_t drop_thresh, double drop_scale, int64_t drop_ld,
               const std::vector<std::vector<int64_t>>& segs) {
  if (!X.is_cuda() || !W.is_cuda() || !C.is_cuda()) throw std::invalid_argument("lumen: lora_gemm needs GPU tensors");
  const int nseg = static_cast<int>(segs.size());
  if (nseg < 1 || nseg > 4) throw std::invalid_argument("lumen: lora_gemm needs 1..4 segments");
  long long xo[4] = {0}, wo[4] = {0}, co[4] = {0};
  int Ms[4] = {0}, Ns[4] = {0}, Ks[4] = {0};
  for (int i = 0; i < nseg; ++i) {
    if (segs[i].size() != 6) throw std::invalid_argument("lumen: segment = (x_off, w_off, c_off, M, N, K)");
    xo[i] = segs[i][0]; wo[i] = segs[i][1]; co[i] = segs[i][2];
    Ms[i] = static_cast<int>(segs[i][3]); Ns[i] = static_cast<int>(segs[i][4]);
    Ks[i] = static_cast<int>(segs[i][5]);
  }
  check(lumen_lora_gemm(static_cast<int>(act_dtype), static_cast<int>(mode), static_cast<int>(bn),
                        X.data_ptr(), W.data_ptr(), C.data_ptr(), ldx, ldw, cs_m, cs_n,
                        static_cast<float>(alpha), static_cast<int>(ksplit),
                        static_cast<unsigned long long>(seed), static_cast<unsigned int>(drop_thresh),
                        static_cast<float>(drop_scale), drop_ld, nseg, xo, wo, co, Ms, Ns, Ks,
                        cur_stream()),
        "lora_gemm");
}

// segs: (big_off, small_off, out_off, ncols) per segment
void lora2(int64_t dtype, int64_t kind, int64_t flag, const at::Tensor& big, int64_t ldb,
           const at::Tensor& small, int64_t lds, at::Tensor& out, int64_t cs0, int64_t cs1,
           double alpha, int64_t T, int64_t J, int64_t split, int64_t seed, int64_t drop_thresh,
           double drop_scale, int64_t drop_ld, int64_t drop_col0,
           const std::vector<std::vector<int64_t>>& segs, const c10::optional<at::Tensor>& rope_cos,
           const c10::optional<at::Tensor>& rope_sin, const c10::optional<at::Tensor>& rope_pos,
           int64_t rope_mask) {
  if (!big.is_cuda() || !small.is_cuda() || !out.is_cuda())
    throw std::invalid_argument("lumen: lora2 needs GPU tensors");
  if (small.scalar_type() != at::kFloat)
    throw std::invalid_argument("lumen: lora2 small operand must be f32");
  if (kind == 2 ? (big.scalar_type() != at::kFloat || out.scalar_type() == at::kFloat)
                : out.scalar_type() != at::kFloat)
    throw std::invalid_argument("lumen: lora2 UP takes f32 adapter weights and a 16-bit output; "
                                "DOWN/WGRAD write f32");
  const int nseg = static_cast<int>(segs.size());
  if (nseg < 1 || nseg > 4) throw std::invalid_argument("lumen: lora2 needs 1..4 segments");
  long long bo[4] = {0}, so[4] = {0}, oo[4] = {0};
  int nc[4] = {0};
  for (int i = 0; i < nseg; ++i) {
    if (segs[i].size() != 4) throw std::invalid_argument("lumen: lora2 segment = (big_off, small_off, out_off, ncols)");
    bo[i] = segs[i][0]; so[i] = segs[i][1]; oo[i] = segs[i][2];
    nc[i] = static_cast<int>(segs[i][3]);
  }
  check(lumen_lora2(static_cast<int>(dtype), static_cast<int>(kind), static_cast<int>(flag),
                    big.data_ptr(), ldb, small.data_ptr<float>(), lds, out.data_ptr(), cs0,
                    cs1, static_cast<float>(alpha), static_cast<int>(T), static_cast<int>(J),
                    static_cast<int>(split), static_cast<unsigned long long>(seed),
                    static_cast<unsigned int>(drop_thresh), static_cast<float>(drop_scale),
                    drop_ld, drop_col0, nseg, bo, so, oo, nc,
                    rope_cos ? rope_cos->data_ptr<float>() : nullptr,
                    rope_sin ? rope_sin->data_ptr<float>() : nullptr,
                    rope_pos ? rope_pos->data_ptr<int>() : nullptr, static_cast<int>(rope_mask),
                    cur_stream()),
        "lora2");
}

bool is_fp8(const at::Tensor& t) { return t.scalar_type() == at::kFloat8_e4m3fn; }

void need_cuda_f32(const at::Tensor& t, const char* what) {
  if (!t.is_cuda() || t.scalar_type() != at::kFloat)
    throw std::invalid_argument(std::string("lumen: ") + what + " must be an f32 GPU tensor");
}

// Z[t, :R] += alpha * drop(x) A^T   (x [T, K] 16-bit, row stride ldx; A [R, K] f32; Z f32)
void lora3_down(const at::Tensor& x, int64_t ldx, const at::Tensor& A, at::Tensor& Z, int64_t ldz,
                int64_t T, int64_t K, int64_t R, double alpha, int64_t seed, int64_t thresh,
                double drop_scale, int64_t drop_ld, int64_t drop_col0,
                const c10::optional<at::Tensor>& xe, int64_t xk, int64_t KP,
                const c10::optional<at::Tensor>& cnt, const c10::optional<at::Tensor>& slab) {
  if (!x.is_cuda()) throw std::invalid_argument("lumen: lora3_down needs GPU tensors");
  need_cuda_f32(A, "lora3_down A");
  need_cuda_f32(Z, "lora3_down Z");
  if (A.stride(1) != 1 || A.size(0) < R || A.size(1) < K || x.size(0) < T || Z.size(0) < T)
    throw std::invalid_argument("lumen: lora3_down shape mismatch");
  void* xp = nullptr;
  long long ldxe = 0;
  unsigned* cp = nullptr;
  if (xe && xe->defined()) {
    // fused fold tail: xe [>= T, >= xk + KP] 16-bit like x, cnt int32 [>= ceil(T / 64)] zeroed
    if (!cnt || !cnt->defined() || cnt->scalar_type() != at::kInt || !cnt->is_cuda() ||
        cnt->numel() < (T + 63) / 64 || xe->scalar_type() != x.scalar_type() || xe->dim() != 2 ||
        xe->stride(1) != 1 || xe->size(0) < T || xe->size(1) < xk + KP || Z.size(1) < R)
      throw std::invalid_argument("lumen: lora3_down fold tail: xe [T, >= xk + KP], cnt int32 [T / 64]");
    xp = xe->data_ptr();
    ldxe = xe->stride(0);
    cp = reinterpret_cast<unsigned*>(cnt->data_ptr<int>());
  }
  float* sp = nullptr;
  if (slab && slab->defined()) {
    // deterministic K-block sum: slab f32 >= ceil(T / 64) * ceil(K / 1024) * 64 * R; with cnt
    // (zeroed) the last-arriving K block sums in the kernel, without it a second launch does
    const bool with_cnt = cnt && cnt->defined();
    if ((with_cnt && (cnt->scalar_type() != at::kInt || !cnt->is_cuda() ||
                      cnt->numel() < (T + 63) / 64)) ||
        slab->scalar_type() != at::kFloat || !slab->is_cuda() ||
        slab->numel() < ((T + 63) / 64) * ((K + 1023) / 1024) * 64 * R)
      throw std::invalid_argument("lumen: lora3_down slab / cnt too small");
    sp = slab->data_ptr<float>();
    cp = with_cnt ? reinterpret_cast<unsigned*>(cnt->data_ptr<int>()) : nullptr;
  }
  check(lumen_lora3_down(dcode(x), x.data_ptr(), ldx, A.data_ptr<float>(), A.stride(0),
                         Z.data_ptr<float>(), ldz, static_cast<int>(T), static_cast<int>(K),
                         static_cast<int>(R), static_cast<float>(alpha),
                         static_cast<unsigned long long>(seed), static_cast<unsigned int>(thresh),
                         static_cast<float>(drop_scale), drop_ld, drop_col0, xp, ldxe,
                         static_cast<int>(xk), static_cast<int>(KP), cp, sp, cur_stream()),
        "lora3_down");
}

// segs: (out_off, s1_off, s2_off, ncols)
void lora3_up(int64_t fwd, at::Tensor& out, int64_t ldo, const at::Tensor& s1, int64_t ld1,
              const at::Tensor& s2, int64_t ld2, int64_t T, int64_t J, double alpha, int64_t seed,
              int64_t thresh, double drop_scale, int64_t drop_ld, int64_t drop_col0,
              const std::vector<std::vector<int64_t>>& segs, const c10::optional<at::Tensor>& rope_cos,
              const c10::optional<at::Tensor>& rope_sin, const c10::optional<at::Tensor>& rope_pos,
              int64_t rope_mask) {
  if (!out.is_cuda()) throw std::invalid_argument("lumen: lora3_up needs GPU tensors");
  need_cuda_f32(s1, "lora3_up s1");
  need_cuda_f32(s2, "lora3_up s2");
  const int nseg = static_cast<int>(segs.size());
  if (nseg < 1 || nseg > 4) throw std::invalid_argument("lumen: lora3_up needs 1..4 segments");
  long long oo[4] = {0}, so1[4] = {0}, so2[4] = {0};
  int nc[4] = {0};
  for (int i = 0; i < nseg; ++i) {
    if (segs[i].size() != 4) throw std::invalid_argument("lumen: lora3_up segment = (out_off, s1_off, s2_off, ncols)");
    oo[i] = segs[i][0]; so1[i] = segs[i][1]; so2[i] = segs[i][2]; nc[i] = static_cast<int>(segs[i][3]);
  }
  check(lumen_lora3_up(dcode(out), static_cast<int>(fwd), out.data_ptr(), ldo, s1.data_ptr<float>(),
                       ld1, s2.data_ptr<float>(), ld2, static_cast<int>(T), static_cast<int>(J),
                       static_cast<float>(alpha), static_cast<unsigned long long>(seed),
                       static_cast<unsigned int>(thresh), static_cast<float>(drop_scale), drop_ld,
                       drop_col0, nseg, oo, so1, so2, nc,
                       rope_cos ? rope_cos->data_ptr<float>() : nullptr,
                       rope_sin ? rope_sin->data_ptr<float>() : nullptr,
                       rope_pos ? rope_pos->data_ptr<int>() : nullptr, static_cast<int>(rope_mask),
                       cur_stream()),
        "lora3_up");
}

// segs: (n_off, r_off, b_off, n_len)
void lora3_dy(const at::Tensor& dy, int64_t ldy, const at::Tensor& B, int64_t r, const at::Tensor& Z,
              int64_t ldz, at::Tensor& dZ, int64_t lddz, at::Tensor& dB, int64_t T, int64_t tw,
              double alpha, const std::vector<std::vector<int64_t>>& segs,
              const c10::optional<at::Tensor>& ws, const c10::optional<at::Tensor>& cnt) {
  if (!dy.is_cuda()) throw std::invalid_argument("lumen: lora3_dy needs GPU tensors");
  need_cuda_f32(B, "lora3_dy B");
  need_cuda_f32(Z, "lora3_dy Z");
  need_cuda_f32(dZ, "lora3_dy dZ");
  need_cuda_f32(dB, "lora3_dy dB");
  const int nseg = static_cast<int>(segs.size());
  if (nseg < 1 || nseg > 4) throw std::invalid_argument("lumen: lora3_dy needs 1..4 segments");
  long long no[4] = {0}, ro[4] = {0}, bo[4] = {0};
  int nl[4] = {0};
  for (int i = 0; i < nseg; ++i) {
    if (segs[i].size() != 4) throw std::invalid_argument("lumen: lora3_dy segment = (n_off, r_off, b_off, n_len)");
    no[i] = segs[i][0]; ro[i] = segs[i][1]; bo[i] = segs[i][2]; nl[i] = static_cast<int>(segs[i][3]);
  }
  // deterministic sums (ws f32): dZ partials [nseg][gy][gx][tw][r], then dB partials
  // [nseg][gx][gy][256][r].  With cnt (int32, zeroed; dZ [nseg][gy], then dB [nseg][gx]) the
  // last-arriving workgroups sum them inside the kernel; without it a second launch does
  float *sz = nullptr, *sb = nullptr;
  unsigned *cz = nullptr, *cb = nullptr;
  if (ws && ws->defined()) {
    int maxl = 0;
    for (int i = 0; i < nseg; ++i) maxl = std::max(maxl, nl[i]);
    const long long gx = (maxl + 255) / 256, gy = (T + tw - 1) / tw;
    const long long nz = nseg * gy * gx * tw * r, nb = nseg * gx * gy * 256 * r;
    const bool with_cnt = cnt && cnt->defined();
    if (!ws->is_cuda() || ws->scalar_type() != at::kFloat || ws->numel() < nz + nb ||
        (with_cnt && (!cnt->is_cuda() || cnt->scalar_type() != at::kInt ||
                      cnt->numel() < nseg * (gx + gy))))
      throw std::invalid_argument("lumen: lora3_dy deterministic workspace too small");
    sz = ws->data_ptr<float>();
    sb = sz + nz;
    if (with_cnt) {
      cz = reinterpret_cast<unsigned*>(cnt->data_ptr<int>());
      cb = cz + nseg * gy;
    }
  }
  check(lumen_lora3_dy(dcode(dy), dy.data_ptr(), ldy, B.data_ptr<float>(), static_cast<int>(r),
                       Z.data_ptr<float>(), ldz, dZ.data_ptr<float>(), lddz, dB.data_ptr<float>(),
                       static_cast<int>(T), static_cast<int>(tw), static_cast<float>(alpha), nseg,
                       no, ro, bo, nl, sz, sb, cz, cb, cur_stream()),
        "lora3_dy");
}

// out[t, :] = W[ids[t], :]  (16-bit table, int64 ids; out of range ids -> zero rows)
void embedding(const at::Tensor& W, const at::Tensor& ids, at::Tensor& out) {
  if (!W.is_cuda() || !ids.is_cuda() || !out.is_cuda() || W.dim() != 2 || !W.is_contiguous() ||
      !out.is_contiguous() || ids.scalar_type() != at::kLong || !ids.is_contiguous() ||
      out.numel() != ids.numel() * W.size(1) || out.scalar_type() != W.scalar_type() ||
      W.element_size() != 2)
    throw std::invalid_argument("lumen: embedding expects a contiguous 16-bit [V, H] table, int64 ids and a [T, H] output");
  check(lumen_embedding(W.data_ptr(), reinterpret_cast<const long long*>(ids.data_ptr<int64_t>()), out.data_ptr(),
                        static_cast<int>(ids.numel()), static_cast<int>(W.size(0)),
                        static_cast<int>(W.size(1)), cur_stream()),
        "embedding");
}

// K-extended LoRA GEMM operands (see kernels/lora_v3.hip): Z tail of the activation buffer
void lora3_z_tail(const at::Tensor& Z, at::Tensor& xe, int64_t K, int64_t KP) {
  need_cuda_f32(Z, "lora3_z_tail Z");
  if (!xe.is_cuda() || xe.dim() != 2 || xe.stride(1) != 1 || !Z.is_contiguous() ||
      Z.size(0) > xe.size(0) || xe.size(1) < K + KP)
    throw std::invalid_argument("lumen: lora3_z_tail: Z [T, R] f32, xe [T, >= K + KP] 16-bit");
  check(lumen_lora3_z_tail(dcode(xe), Z.data_ptr<float>(), static_cast<int>(Z.size(1)),
                           xe.data_ptr(), xe.stride(0), static_cast<int>(K), static_cast<int>(KP),
                           static_cast<int>(Z.size(0)), cur_stream()),
        "lora3_z_tail");
}

// segs: (n_off, b_off, n_len, r_off)
void lora3_w_tail(at::Tensor& w, int64_t K, const at::Tensor& B, int64_t r,
                  const std::vector<std::vector<int64_t>>& segs, double scale) {
  need_cuda_f32(B, "lora3_w_tail B");
  if (!w.is_cuda() || w.dim() != 2 || w.stride(1) != 1 || !B.is_contiguous())
    throw std::invalid_argument("lumen: lora3_w_tail: w [N, K + KP] 16-bit, B [*, r] f32");
  const int nseg = static_cast<int>(segs.size());
  if (nseg < 1 || nseg > 4) throw std::invalid_argument("lumen: lora3_w_tail needs 1..4 segments");
  long long no[4] = {0}, bo[4] = {0};
  int nl[4] = {0}, ro[4] = {0};
  for (int i = 0; i < nseg; ++i) {
    no[i] = segs[i][0]; bo[i] = segs[i][1]; nl[i] = static_cast<int>(segs[i][2]);
    ro[i] = static_cast<int>(segs[i][3]);
  }
  check(lumen_lora3_w_tail(dcode(w), w.data_ptr(), w.stride(0), static_cast<int>(K),
                           B.data_ptr<float>(), static_cast<int>(r), nseg, no, bo, nl, ro,
                           static_cast<float>(scale), cur_stream()),
        "lora3_w_tail");
}

// every folded linear's tail in one launch: desc [n, 24] int64 on the GPU (built by
// lumen.models.layers.FoldTails, which also validates the pointers / shapes it encodes)
void lora3_w_tail_batch(const at::Tensor& desc, int64_t dtype, int64_t max_chunks) {
  need_cuda(desc, "lora3_w_tail_batch desc");
  if (desc.scalar_type() != at::kLong || desc.dim() != 2 || desc.size(1) != 24 ||
      !desc.is_contiguous())
    throw std::invalid_argument("lumen: lora3_w_tail_batch: desc [n, 24] int64");
  check(lumen_lora3_w_tail_batch(static_cast<int>(dtype),
                                 reinterpret_cast<const long long*>(desc.data_ptr<int64_t>()),
                                 static_cast<int>(desc.size(0)), max_chunks, cur_stream()),
        "lora3_w_tail_batch");
}

// fused x-side LoRA backward (kernels/lora_v3.hip dxa3_kernel)
void lora3_dxa(const at::Tensor& x, at::Tensor& dx, const at::Tensor& dZ, const at::Tensor& A,
               at::Tensor& dA, int64_t tw, int64_t seed, int64_t thresh, double drop_scale,
               int64_t drop_ld, int64_t drop_col0, const c10::optional<at::Tensor>& delta,
               const c10::optional<at::Tensor>& ws, const c10::optional<at::Tensor>& cnt) {
  need_cuda_f32(dZ, "lora3_dxa dZ");
  float* dp = nullptr;
  if (delta && delta->defined()) {
    // attention delta hand-off: [K / 128 heads, T] f32, head dim 128, R = 16 (o_proj)
    need_cuda_f32(*delta, "lora3_dxa delta");
    if (!delta->is_contiguous() || delta->dim() != 2 || x.size(1) % 128 != 0 ||
        delta->size(0) != x.size(1) / 128 || delta->size(1) != x.size(0) || dZ.size(1) != 16)
      throw std::invalid_argument("lumen: lora3_dxa delta: [K / 128, T] f32 with R = 16");
    dp = delta->data_ptr<float>();
  }
  need_cuda_f32(A, "lora3_dxa A");
  need_cuda_f32(dA, "lora3_dxa dA");
  if (!x.is_cuda() || !dx.is_cuda() || x.dim() != 2 || dx.dim() != 2 || x.stride(1) != 1 ||
      dx.stride(1) != 1 || x.sizes() != dx.sizes() || dx.scalar_type() != x.scalar_type() ||
      !dZ.is_contiguous() || dZ.size(0) != x.size(0) || A.stride(1) != 1 || dA.stride(1) != 1 ||
      A.size(0) != dZ.size(1) || dA.size(0) != dZ.size(1) || A.size(1) != x.size(1) ||
      dA.size(1) != x.size(1))
    throw std::invalid_argument("lumen: lora3_dxa: x/dx [T, K] 16-bit, dZ [T, R] f32, A/dA [R, K] f32");
  float* sp = nullptr;
  unsigned* cp = nullptr;
  // deterministic dA: partials [gx][gy][R][128]; with counters [gx] the last-arriving row
  // block sums them in the kernel, without them a second launch does
  if (ws && ws->defined()) {
    const long long gx = (x.size(1) + 127) / 128, gy = (x.size(0) + tw - 1) / tw;
    const bool with_cnt = cnt && cnt->defined();
    if (!ws->is_cuda() || ws->scalar_type() != at::kFloat ||
        ws->numel() < gx * gy * 128 * dZ.size(1) ||
        (with_cnt && (!cnt->is_cuda() || cnt->scalar_type() != at::kInt || cnt->numel() < gx)))
      throw std::invalid_argument("lumen: lora3_dxa deterministic workspace too small");
    sp = ws->data_ptr<float>();
    if (with_cnt) cp = reinterpret_cast<unsigned*>(cnt->data_ptr<int>());
  }
  check(lumen_lora3_dxa(dcode(x), x.data_ptr(), x.stride(0), dx.data_ptr(), dx.stride(0),
                        dZ.data_ptr<float>(), A.data_ptr<float>(), A.stride(0),
                        dA.data_ptr<float>(), dA.stride(0), static_cast<int>(x.size(0)),
                        static_cast<int>(x.size(1)), static_cast<int>(dZ.size(1)),
                        static_cast<int>(tw), static_cast<unsigned long long>(seed),
                        static_cast<unsigned int>(thresh), static_cast<float>(drop_scale), drop_ld,
                        drop_col0, dp, sp, cp, cur_stream()),
        "lora3_dxa");
}

void transpose2d(const at::Tensor& in, at::Tensor& out) {
  if (!in.is_cuda() || !out.is_cuda() || in.dim() != 2 || out.dim() != 2)
    throw std::invalid_argument("lumen: transpose2d needs 2-D GPU tensors");
  if (in.stride(1) != 1 || out.stride(1) != 1 || out.size(0) != in.size(1) || out.size(1) != in.size(0))
    throw std::invalid_argument("lumen: transpose2d shape/stride mismatch");
  check(lumen_transpose(dcode(in), in.data_ptr(), out.data_ptr(), static_cast<int>(in.size(0)),
                        static_cast<int>(in.size(1)), in.stride(0), out.stride(0), cur_stream()),
        "transpose2d");
}

void paged_attention_decode(at::Tensor& out, const at::Tensor& q, const at::Tensor& k_cache,
                            const at::Tensor& v_cache, const at::Tensor& block_tables,
                            const at::Tensor& context_lens, int64_t num_kv_heads, int64_t block_size,
                            int64_t max_blocks_per_seq, double scale, at::Tensor& tmp_m,
                            at::Tensor& tmp_l, at::Tensor& tmp_o, int64_t partition_size,
                            const std::optional<at::Tensor>& counters, int64_t one_pass) {
  if (!q.is_cuda()) throw std::invalid_argument("lumen: q must be a GPU tensor");
  need_cuda(out, "out");
  const int num_seqs = static_cast<int>(q.size(0));
  const int nh = static_cast<int>(q.size(1));
  const int D = static_cast<int>(q.size(2));
  // q may be a view into the fused qkv rows: heads contiguous, rows at any multiple of D
  if (q.dim() != 3 || q.stride(2) != 1 || q.stride(1) != D || q.stride(0) % D != 0 ||
      q.stride(0) < static_cast<int64_t>(nh) * D)
    throw std::invalid_argument("lumen: paged_attention_decode q must be [nseq, nh, D] with "
                                "contiguous heads");
  const int qldh = static_cast<int>(q.stride(0) / D);
  unsigned* cnt = nullptr;
  if (counters.has_value()) {
    const at::Tensor& c = *counters;
    need_cuda(c, "counters");
    if (c.scalar_type() != at::kInt || c.numel() < static_cast<int64_t>(num_seqs) * num_kv_heads)
      throw std::invalid_argument("lumen: paged_attention_decode counters must be int32 >= nseq*nkv");
    cnt = reinterpret_cast<unsigned*>(c.data_ptr<int>());
  }
  check(lumen_paged_attention_decode(dcode(q), out.data_ptr(), q.data_ptr(), k_cache.data_ptr(),
                                     v_cache.data_ptr(), block_tables.data_ptr<int>(),
                                     context_lens.data_ptr<int>(), num_seqs, nh,
                                     static_cast<int>(num_kv_heads), D, static_cast<int>(block_size),
                                     static_cast<int>(max_blocks_per_seq),
                                     static_cast<int>(tmp_m.size(-1)), static_cast<float>(scale),
                                     tmp_m.data_ptr<float>(), tmp_l.data_ptr<float>(),
                                     tmp_o.data_ptr(), static_cast<int>(partition_size), cnt,
                                     static_cast<int>(one_pass), is_fp8(k_cache) ? 1 : 0, qldh,
                                     cur_stream()),
        "paged_attention_decode");
}

// fp8 KV cache -> 16-bit scratch for prefill attention: block b of sequence s (b * bs <
// kv_lens[s]) lands at scratch block s * maxb + b
void kv_dequant(const at::Tensor& k_cache, const at::Tensor& v_cache, at::Tensor& k_scr,
                at::Tensor& v_scr, const at::Tensor& tables, const at::Tensor& kv_lens,
                int64_t maxb) {
  need_cuda(k_cache, "k_cache"); need_cuda(v_cache, "v_cache");
  need_cuda(k_scr, "k_scr"); need_cuda(v_scr, "v_scr");
  if (!is_fp8(k_cache) || !is_fp8(v_cache) || k_cache.dim() != 4 || k_scr.dim() != 4 ||
      k_scr.size(1) != k_cache.size(1) || k_scr.size(2) != k_cache.size(2) ||
      k_scr.size(3) != k_cache.size(3) || tables.scalar_type() != at::kInt ||
      kv_lens.scalar_type() != at::kInt || tables.dim() != 2 ||
      k_scr.size(0) < kv_lens.numel() * maxb || !k_scr.is_contiguous() || !v_scr.is_contiguous())
    throw std::invalid_argument("lumen: kv_dequant: fp8 [nb, nkv, bs, D] caches, 16-bit scratch "
                                ">= nseq * maxb blocks, int32 tables / kv_lens");
  check(lumen_kv_dequant(dcode(k_scr), k_cache.data_ptr(), v_cache.data_ptr(), k_scr.data_ptr(),
                         v_scr.data_ptr(), tables.data_ptr<int>(),
                         static_cast<int>(tables.stride(0)), kv_lens.data_ptr<int>(),
                         static_cast<int>(kv_lens.numel()), static_cast<int>(maxb),
                         static_cast<int>(k_cache.size(1)), static_cast<int>(k_cache.size(2)),
                         static_cast<int>(k_cache.size(3)), cur_stream()),
        "kv_dequant");
}

void reshape_and_cache(const at::Tensor& k, const at::Tensor& v, at::Tensor& k_cache, at::Tensor& v_cache,
                       const at::Tensor& slot_mapping, int64_t num_kv_heads, int64_t D,
                       int64_t block_size, int64_t k_stride, int64_t v_stride) {
  const int ntok = static_cast<int>(slot_mapping.numel());
  check(lumen_reshape_and_cache(dcode(k), k.data_ptr(), v.data_ptr(), k_cache.data_ptr(),
                                v_cache.data_ptr(), reinterpret_cast<const long long*>(slot_mapping.data_ptr<int64_t>()), ntok,
                                static_cast<int>(num_kv_heads), static_cast<int>(D),
                                static_cast<int>(block_size), k_stride, v_stride,
                                is_fp8(k_cache) ? 1 : 0, cur_stream()),
        "reshape_and_cache");
}

void rope_cache_write(at::Tensor& qkv, const at::Tensor& pos, const at::Tensor& cos_t,
                      const at::Tensor& sin_t, at::Tensor& k_cache, at::Tensor& v_cache,
                      const at::Tensor& slots, int64_t nh, int64_t nkv, int64_t D,
                      int64_t block_size) {
  if (!qkv.is_cuda() || qkv.dim() != 2 || qkv.stride(1) != 1)
    throw std::invalid_argument("lumen: rope_cache_write needs a 2-D GPU qkv with unit column stride");
  need_cuda(pos, "pos"); need_cuda(cos_t, "cos"); need_cuda(sin_t, "sin");
  need_cuda(k_cache, "k_cache"); need_cuda(v_cache, "v_cache"); need_cuda(slots, "slots");
  if (pos.scalar_type() != at::kInt || slots.scalar_type() != at::kLong ||
      cos_t.scalar_type() != at::kFloat || sin_t.scalar_type() != at::kFloat ||
      qkv.size(1) < (nh + 2 * nkv) * D || pos.numel() < qkv.size(0) ||
      slots.numel() < qkv.size(0))
    throw std::invalid_argument("lumen: rope_cache_write argument mismatch");
  check(lumen_rope_cache(dcode(qkv), qkv.data_ptr(), qkv.stride(0), pos.data_ptr<int>(),
                         cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), k_cache.data_ptr(),
                         v_cache.data_ptr(),
                         reinterpret_cast<const long long*>(slots.data_ptr<int64_t>()),
                         static_cast<int>(qkv.size(0)), static_cast<int>(nh),
                         static_cast<int>(nkv), static_cast<int>(D),
                         static_cast<int>(block_size), is_fp8(k_cache) ? 1 : 0, cur_stream()),
        "rope_cache_write");
}

void sample(const at::Tensor& logits, const at::Tensor& temperature, const at::Tensor& top_p,
            const at::Tensor& top_k, int64_t seed, int64_t offset, at::Tensor& out_tokens,
            const std::optional<at::Tensor>& out_logprob, const std::optional<at::Tensor>& out_tau) {
  need_cuda(logits, "logits");
  const int V = static_cast<int>(logits.size(-1));
  const int rows = static_cast<int>(logits.numel() / V);
  for (const at::Tensor* t :
       std::initializer_list<const at::Tensor*>{&temperature, &top_p, &top_k, &out_tokens})
    if (!t->is_cuda() || t->numel() < rows)
      throw std::invalid_argument("lumen: sample per-row tensors must be GPU tensors of >= rows");
  if (out_tau && (!out_tau->is_cuda() || out_tau->scalar_type() != at::kFloat ||
                  out_tau->numel() < rows))
    throw std::invalid_argument("lumen: sample out_tau must be a float32 GPU tensor of >= rows");
  check(lumen_sample(dcode(logits), logits.data_ptr(), temperature.data_ptr<float>(),
                     top_p.data_ptr<float>(), top_k.data_ptr<int>(),
                     static_cast<unsigned long long>(seed), offset,
                     reinterpret_cast<long long*>(out_tokens.data_ptr<int64_t>()),
                     ptr<float>(out_logprob), ptr<float>(out_tau), rows, V, cur_stream()),
        "sample");
}

// which: 0 fwd, 1 delta, 2 dK/dV, 3 dQ.  q/k/v/o/dout/dq/dk/dv are (possibly strided) 2-D views
// [T, cols]: the kernels address head h at column h*128 with the given row strides.
void flash_attn(int64_t which, bool causal, int64_t mt, const at::Tensor& q, const at::Tensor& k,
                const at::Tensor& v, const at::Tensor& o, const at::Tensor& lse,
                const at::Tensor& cu, const at::Tensor& tiles, int64_t nh, int64_t nkv,
                double scale, const std::optional<at::Tensor>& dout,
                const std::optional<at::Tensor>& dq, const std::optional<at::Tensor>& dk,
                const std::optional<at::Tensor>& dv, const std::optional<at::Tensor>& delta,
                const std::optional<at::Tensor>& rope_pos, const std::optional<at::Tensor>& rope_cos,
                const std::optional<at::Tensor>& rope_sin) {
  if (!q.is_cuda()) throw std::invalid_argument("lumen: flash_attn needs GPU tensors");
  if (rope_pos.has_value() &&
      (!rope_cos.has_value() || !rope_sin.has_value() || rope_pos->scalar_type() != at::kInt ||
       rope_cos->scalar_type() != at::kFloat || rope_sin->scalar_type() != at::kFloat ||
       !rope_pos->is_contiguous() || !rope_cos->is_contiguous() || !rope_sin->is_contiguous() ||
       rope_cos->size(-1) != 64 || rope_pos->numel() < q.size(0)))
    throw std::invalid_argument("lumen: flash_attn rope needs int32 pos [T] and f32 cos/sin [*, 64]");
  auto st = [](const std::optional<at::Tensor>& t) -> long long { return t.has_value() ? t->stride(0) : 0; };
  const int T = static_cast<int>(q.size(0));
  const int ntiles = static_cast<int>(tiles.numel() / ((which & 0x100) ? 3 : 2));
  check(lumen_flash_attn(dcode(q), static_cast<int>(which), causal ? 1 : 0, static_cast<int>(mt),
                         q.data_ptr(), k.data_ptr(), v.data_ptr(), q.stride(0), k.stride(0),
                         v.stride(0), o.data_ptr(), o.stride(0), lse.data_ptr<float>(),
                         cu.data_ptr<int>(), tiles.data_ptr<int>(), ntiles, static_cast<int>(nh),
                         static_cast<int>(nkv), T, static_cast<float>(scale), ptr(dout), st(dout),
                         ptr(dq), ptr(dk), ptr(dv), st(dq), st(dk), st(dv), ptr<const float>(delta),
                         ptr<const int>(rope_pos), ptr<const float>(rope_cos),
                         ptr<const float>(rope_sin), cur_stream()),
        "flash_attn");
}

// Backward with the dS hand-off (which 7 = dK/dV + dS store, 8 = dQ from dS); ds is a
// [nh, ds_total, 64*64] 16-bit buffer, ds_off int32 [nseq] the per-sequence first tile.
void flash_attn_ds(int64_t which, bool causal, const at::Tensor& q, const at::Tensor& k,
                   const at::Tensor& v, const at::Tensor& lse, const at::Tensor& cu,
                   const at::Tensor& tiles, int64_t nh, int64_t nkv, double scale,
                   const at::Tensor& dout, const at::Tensor& dq, const at::Tensor& dk,
                   const at::Tensor& dv, const at::Tensor& delta, const at::Tensor& ds,
                   const at::Tensor& ds_off, int64_t ds_total,
                   const std::optional<at::Tensor>& rope_pos, const std::optional<at::Tensor>& rope_cos,
                   const std::optional<at::Tensor>& rope_sin) {
  if (!q.is_cuda() || !ds.is_cuda() || !ds_off.is_cuda())
    throw std::invalid_argument("lumen: flash_attn_ds needs GPU tensors");
  if (ds_off.scalar_type() != at::kInt || ds.scalar_type() != q.scalar_type() || !ds.is_contiguous() ||
      ds.numel() < nh * ds_total * 4096 || ds_off.numel() + 1 < cu.numel())
    throw std::invalid_argument("lumen: flash_attn_ds needs ds [nh, ds_total, 4096] of q's dtype and "
                                "int32 ds_off [nseq]");
  if (rope_pos.has_value() &&
      (!rope_cos.has_value() || !rope_sin.has_value() || rope_pos->scalar_type() != at::kInt ||
       rope_cos->scalar_type() != at::kFloat || rope_sin->scalar_type() != at::kFloat ||
       rope_cos->size(-1) != 64 || rope_pos->numel() < q.size(0)))
    throw std::invalid_argument("lumen: flash_attn_ds rope needs int32 pos [T] and f32 cos/sin [*, 64]");
  check(lumen_flash_attn_ds(dcode(q), static_cast<int>(which), causal ? 1 : 0, q.data_ptr(),
                            k.data_ptr(), v.data_ptr(), q.stride(0), k.stride(0), v.stride(0),
                            lse.data_ptr<float>(), cu.data_ptr<int>(), tiles.data_ptr<int>(),
                            static_cast<int>(tiles.numel() / ((which & 0x100) ? 3 : 2)),
                            static_cast<int>(nh),
                            static_cast<int>(nkv), static_cast<int>(q.size(0)),
                            static_cast<float>(scale), dout.data_ptr(), dout.stride(0),
                            dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), dq.stride(0), dk.stride(0),
                            dv.stride(0), delta.data_ptr<float>(), ptr<const int>(rope_pos),
                            ptr<const float>(rope_cos), ptr<const float>(rope_sin), ds.data_ptr(),
                            ds_off.data_ptr<int>(), static_cast<int>(ds_total), cur_stream()),
        "flash_attn_ds");
}

// q [T, >= nh*D] token-major rows (any row stride), caches [nblocks, nkv, bs, D], o [T, nh*D]
void flash_attn_paged(bool causal, const at::Tensor& q, const at::Tensor& k_cache,
                      const at::Tensor& v_cache, at::Tensor& o, const at::Tensor& cu_q,
                      const at::Tensor& kv_lens, const at::Tensor& tiles,
                      const at::Tensor& block_tables, int64_t nh, int64_t nkv, double scale) {
  need_cuda(q, "q"); need_cuda(k_cache, "k_cache"); need_cuda(v_cache, "v_cache");
  need_cuda(o, "o");
  if (k_cache.dim() != 4 || k_cache.size(3) != 128 || k_cache.size(1) != nkv ||
      !k_cache.is_contiguous() || !v_cache.is_contiguous() ||
      v_cache.sizes() != k_cache.sizes() || q.scalar_type() != k_cache.scalar_type() ||
      o.scalar_type() != q.scalar_type() || q.stride(1) != 1 || o.stride(1) != 1)
    throw std::invalid_argument("lumen: flash_attn_paged needs [nblocks, nkv, bs, 128] caches "
                                "of the query dtype and row-major q / o");
  for (const at::Tensor* t : {&cu_q, &kv_lens, &tiles, &block_tables})
    if (t->scalar_type() != at::kInt || !t->is_contiguous() || !t->is_cuda())
      throw std::invalid_argument("lumen: flash_attn_paged index tensors must be int32 on GPU");
  if (block_tables.dim() != 2 || block_tables.size(0) < kv_lens.numel() ||
      cu_q.numel() != kv_lens.numel() + 1)
    throw std::invalid_argument("lumen: flash_attn_paged: cu_q [nseq+1], kv_lens [nseq], "
                                "block_tables [nseq, max_blocks]");
  check(lumen_flash_attn_paged(dcode(q), causal ? 1 : 0, q.data_ptr(), q.stride(0),
                               k_cache.data_ptr(), v_cache.data_ptr(), o.data_ptr(), o.stride(0),
                               cu_q.data_ptr<int>(), kv_lens.data_ptr<int>(),
                               tiles.data_ptr<int>(), static_cast<int>(tiles.numel() / 2),
                               block_tables.data_ptr<int>(),
                               static_cast<int>(block_tables.stride(0)),
                               static_cast<int>(k_cache.size(2)), static_cast<int>(nh),
                               static_cast<int>(nkv), static_cast<int>(q.size(0)),
                               static_cast<float>(scale), cur_stream()),
        "flash_attn_paged");
}

void cpu_adamw(at::Tensor& p, const at::Tensor& g, at::Tensor& m, at::Tensor& v, double lr, double b1,
               double b2, double eps, double wd, double bc1, double bc2, double grad_scale) {
  if (p.is_cuda() || g.is_cuda()) throw std::invalid_argument("lumen: cpu_adamw takes host tensors");
  if (p.scalar_type() != at::kFloat || g.scalar_type() != at::kFloat)
    throw std::invalid_argument("lumen: cpu_adamw needs f32");
  lumen_cpu_adamw(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                  p.numel(), static_cast<float>(lr), static_cast<float>(b1), static_cast<float>(b2),
                  static_cast<float>(eps), static_cast<float>(wd), static_cast<float>(bc1),
                  static_cast<float>(bc2), static_cast<float>(grad_scale));
}

}  // namespace

// ---- custom all-reduce (kernels/custom_ar.hip): raw device pointers travel as Python ints
int64_t car_alloc(int64_t bytes, bool cached) {
  void* p = nullptr;
  check(lumen_car_alloc(bytes, cached ? 1 : 0, &p), "car_alloc");
  return reinterpret_cast<int64_t>(p);
}

void car_free(int64_t p) { check(lumen_car_free(reinterpret_cast<void*>(p)), "car_free"); }

py::bytes car_handle(int64_t p) {
  std::string h(lumen_car_handle_bytes(), '\0');
  check(lumen_car_get_handle(reinterpret_cast<void*>(p), h.data()), "car_handle");
  return py::bytes(h);
}

int64_t car_open(const py::bytes& handle) {
  std::string h = handle;
  if ((int)h.size() != lumen_car_handle_bytes()) throw std::invalid_argument("lumen: bad IPC handle");
  void* p = nullptr;
  check(lumen_car_open_handle(h.data(), &p), "car_open");
  return reinterpret_cast<int64_t>(p);
}

void car_close(int64_t p) { check(lumen_car_close_handle(reinterpret_cast<void*>(p)), "car_close"); }

// pinned host-mapped error word: (host address, device address); read with car_host_flag_read
std::vector<int64_t> car_host_flag_alloc() {
  void *h = nullptr, *d = nullptr;
  check(lumen_car_host_flag_alloc(&h, &d), "car_host_flag_alloc");
  return {reinterpret_cast<int64_t>(h), reinterpret_cast<int64_t>(d)};
}

void car_host_flag_free(int64_t h) {
  check(lumen_car_host_flag_free(reinterpret_cast<void*>(h)), "car_host_flag_free");
}

// a plain load of the host word: no device sync (the kernel writes it system-coherently)
int64_t car_host_flag_read(int64_t h) {
  return static_cast<int64_t>(*reinterpret_cast<volatile uint32_t*>(h));
}

void car_host_flag_clear(int64_t h) { *reinterpret_cast<volatile uint32_t*>(h) = 0; }

void car_allgather(const std::vector<int64_t>& data, const std::vector<int64_t>& sig, int rank,
                   const at::Tensor& in, at::Tensor& out, int blocks, double timeout_s,
                   int64_t host_err) {
  need_cuda(in, "in");
  need_cuda(out, "out");
  const int world = (int)data.size();
  if ((int)sig.size() != world || rank < 0 || rank >= world || in.dim() != 2 || out.dim() != 2)
    throw std::invalid_argument("lumen: car_allgather needs 2-D tensors and matching peer tables");
  if (out.size(0) != in.size(0) || out.size(1) != in.size(1) * world || (in.size(1) & 7) ||
      in.scalar_type() != out.scalar_type())
    throw std::invalid_argument("lumen: car_allgather shapes: in [R, Vs], out [R, W*Vs], Vs % 8 == 0");
  std::vector<long long> d(data.begin(), data.end()), s(sig.begin(), sig.end());
  check(lumen_car_allgather(dcode(in), d.data(), s.data(), rank, world, in.data_ptr(),
                            out.data_ptr(), in.size(0), in.size(1), blocks, timeout_s,
                            reinterpret_cast<void*>(host_err), cur_stream()),
        "car_allgather");
}

int64_t car_err(int64_t sig) {
  unsigned int e = 0;
  check(lumen_car_read_err(reinterpret_cast<void*>(sig), &e), "car_err");
  return e;
}

// (err, err_info, long_wait_us, long_waits) of a signal block: synchronous, diagnostics only
std::vector<int64_t> car_diag(int64_t sig) {
  unsigned int v[4] = {0, 0, 0, 0};
  check(lumen_car_read_diag(reinterpret_cast<void*>(sig), v), "car_diag");
  return {v[0], v[1], v[2], v[3]};
}

void car_allreduce(const std::vector<int64_t>& data, const std::vector<int64_t>& sig, int rank,
                   const at::Tensor& in, at::Tensor& out, bool two_shot, int blocks,
                   double timeout_s, int64_t host_err) {
  need_cuda(in, "in");
  need_cuda(out, "out");
  const int world = (int)data.size();
  if ((int)sig.size() != world || rank < 0 || rank >= world)
    throw std::invalid_argument("lumen: car_allreduce peer tables do not match");
  if (in.numel() != out.numel() || in.scalar_type() != out.scalar_type() || (in.numel() & 7))
    throw std::invalid_argument("lumen: car_allreduce needs same-shape tensors with numel % 8 == 0");
  std::vector<long long> d(data.begin(), data.end()), s(sig.begin(), sig.end());
  check(lumen_car_allreduce(dcode(in), d.data(), s.data(), rank, world, in.data_ptr(),
                            out.data_ptr(), in.numel(), two_shot ? 1 : 0, blocks, timeout_s,
                            reinterpret_cast<void*>(host_err), cur_stream()),
        "car_allreduce");
}

PYBIND11_MODULE(_C, m) {
  m.doc() = "lumen native ops for MI355X (gfx950)";
  m.def("rmsnorm_fwd", &rmsnorm_fwd);
  m.def("lora3_down", &lora3_down, py::arg("x"), py::arg("ldx"), py::arg("A"), py::arg("Z"),
        py::arg("ldz"), py::arg("T"), py::arg("K"), py::arg("R"), py::arg("alpha"), py::arg("seed"),
        py::arg("thresh"), py::arg("drop_scale"), py::arg("drop_ld"), py::arg("drop_col0"),
        py::arg("xe") = py::none(), py::arg("xk") = 0, py::arg("KP") = 0,
        py::arg("cnt") = py::none(), py::arg("slab") = py::none());
  m.def("embedding", &embedding);
  m.def("lora3_dy", &lora3_dy, py::arg("dy"), py::arg("ldy"), py::arg("B"), py::arg("r"),
        py::arg("Z"), py::arg("ldz"), py::arg("dZ"), py::arg("lddz"), py::arg("dB"), py::arg("T"),
        py::arg("tw"), py::arg("alpha"), py::arg("segs"), py::arg("ws") = py::none(),
        py::arg("cnt") = py::none());
  m.def("lora3_dxa", &lora3_dxa, py::arg("x"), py::arg("dx"), py::arg("dZ"), py::arg("A"),
        py::arg("dA"), py::arg("tw"), py::arg("seed"), py::arg("thresh"), py::arg("drop_scale"),
        py::arg("drop_ld"), py::arg("drop_col0"), py::arg("delta") = py::none(),
        py::arg("ws") = py::none(), py::arg("cnt") = py::none());
  m.def("lora3_z_tail", &lora3_z_tail);
  m.def("lora3_w_tail", &lora3_w_tail);
  m.def("kv_dequant", &kv_dequant);
  m.def("lora3_up", &lora3_up);
  m.def("rmsnorm_bwd", &rmsnorm_bwd);
  m.def("qkv_rope", &qkv_rope);
  m.def("rope_inplace", &rope_inplace);
  m.def("swiglu", &swiglu, py::arg("bwd"), py::arg("gu"), py::arg("dact"), py::arg("out"),
        py::arg("c0") = 0, py::arg("c1") = -1);
  m.def("cross_entropy", &cross_entropy);
  m.def("scale_dev", &scale_dev);
  m.def("grad_norm_sq", &grad_norm_sq);
  m.def("adamw", &adamw);
  m.def("lora_gemm", &lora_gemm);
  m.def("lora2", &lora2);
  m.def("transpose2d", &transpose2d);
  m.def("skinny_gemm", &skinny_gemm);
  m.def("skinny_swiglu_gemm", &skinny_swiglu_gemm);
  m.def("decode_gemm", &decode_gemm);
  m.def("mlp_gemm", &mlp_gemm, py::arg("epi"), py::arg("x"), py::arg("w"), py::arg("c"),
        py::arg("act") = py::none(), py::arg("gu") = py::none(), py::arg("group_m") = 4,
        py::arg("ws") = py::none(), py::arg("cnt") = py::none(), py::arg("split") = 0);
  m.def("mlp_gemm_split", &mlp_gemm_split);
  m.def("hbm_read", &hbm_read);
  m.def("lora3_w_tail_batch", &lora3_w_tail_batch);
  m.def("set_gemv_form", [](int64_t f) { lumen_set_gemv_form(static_cast<int>(f)); });
  m.def("set_rms_lds", [](int64_t f, int64_t b) {
    lumen_set_rms_lds(static_cast<int>(f), static_cast<int>(b));
  });
  m.def("rope_cache_write", &rope_cache_write);
  m.def("paged_attention_decode", &paged_attention_decode);
  m.def("reshape_and_cache", &reshape_and_cache);
  m.def("sample", &sample, py::arg("logits"), py::arg("temperature"), py::arg("top_p"),
        py::arg("top_k"), py::arg("seed"), py::arg("offset"), py::arg("out_tokens"),
        py::arg("out_logprob") = py::none(), py::arg("out_tau") = py::none());
  m.def("flash_attn", &flash_attn);
  m.def("flash_attn_paged", &flash_attn_paged);
  m.def("flash_attn_ds", &flash_attn_ds);
  m.def("car_alloc", &car_alloc);
  m.def("car_free", &car_free);
  m.def("car_handle", &car_handle);
  m.def("car_open", &car_open);
  m.def("car_close", &car_close);
  m.def("car_err", &car_err);
  m.def("car_diag", &car_diag);
  m.def("car_host_flag_alloc", &car_host_flag_alloc);
  m.def("car_host_flag_free", &car_host_flag_free);
  m.def("car_host_flag_read", &car_host_flag_read);
  m.def("car_host_flag_clear", &car_host_flag_clear);
  m.def("car_allreduce", &car_allreduce);
  m.def("car_allgather", &car_allgather);
  m.def("car_signal_bytes", &lumen_car_signal_bytes);
  m.def("car_max_blocks", &lumen_car_max_blocks);
  m.def("car_max_ranks", &lumen_car_max_ranks);
  // the GIL is released: the async ZeRO-Offload step runs this on a host thread while the
  // main thread keeps launching the next forward
  m.def("cpu_adamw", &cpu_adamw, py::call_guard<py::gil_scoped_release>());
  m.def("cpu_has_avx512", &lumen_cpu_has_avx512);
}
