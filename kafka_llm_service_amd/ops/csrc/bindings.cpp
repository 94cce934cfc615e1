#include <cstring>
// Python bindings for the CDNA4 kernels. Host-side shape / dtype / device checks live here so that a malformed
// call fails with a Python exception instead of launching a kernel on a shape it does not assume.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

typedef unsigned short bf16;  // raw bf16 storage on the host side

extern "C" {
hipError_t kafka_launch_rmsnorm(bf16* out, int64_t os, const bf16* x, int64_t xs, const bf16* w, int T, int d, float eps,
                          hipStream_t st);
hipError_t kafka_launch_fused_add_rmsnorm(bf16* out, int64_t os, const bf16* x, int64_t xs, bf16* resid, int64_t rs,
                                    const bf16* w, int T, int d, float eps, hipStream_t st);
hipError_t kafka_launch_fused_add_rmsnorm_slab(bf16* out, int64_t os, const float* xp, int S, int64_t ps, bf16* resid,
                                               int64_t rs, const bf16* w, int T, int d, float eps, hipStream_t st);
hipError_t kafka_launch_silu_mul(bf16* out, const bf16* x, int64_t xs, int T, int F, hipStream_t st);
hipError_t kafka_launch_silu_mul_slab(bf16* out, const float* xp, int S, int64_t ps, int T, int F, hipStream_t st);
hipError_t kafka_launch_rope_kv(const bf16* qkv, const float* qp, int S, int64_t ps, int64_t qkv_stride,
                                const int64_t* positions, const float* cos_sin, bf16* q_out, int64_t q_stride,
                                bf16* k_cache, bf16* v_cache, const int64_t* slot_mapping, int T, int Hq, int Hkv,
                                int D, int block_size, hipStream_t st);
hipError_t kafka_launch_rope_kv_fp8(const bf16* qkv, const float* qp, int S, int64_t ps, int64_t qkv_stride,
                                    const int64_t* positions, const float* cos_sin, bf16* q_out, int64_t q_stride,
                                    uint8_t* k_cache, uint8_t* v_cache, const int64_t* slot_mapping, int T, int Hq,
                                    int Hkv, int D, hipStream_t st);
hipError_t kafka_launch_attn_decode(const bf16* q, int64_t q_stride, const void* k_cache, const void* v_cache, int fp8,
                                    int n_items, int B, int Hkv, int G, int D, const int* block_tables, int bt_stride,
                                    const int* items, float* out_part, float* lse_part, int S_total, float scale,
                                    bf16* out, int64_t out_stride, int* tickets, const bf16* pre_bf16,
                                    const float* m_part, const float* m_lse, int m_S, int m_rows, bf16* m_out,
                                    int64_t m_out_stride, hipStream_t st);
hipError_t kafka_launch_attn_prefill(const void* items, int n_items, const bf16* q, int64_t q_stride,
                                     const void* k_cache, const void* v_cache, int fp8, int Hkv, int G, int D,
                                     const int* block_tables, int bt_stride, const int* q_limit, bf16* out,
                                     int64_t out_stride, float* out_part, float* lse_part, int S_total, float scale,
                                     int variant, int part_bf16, float* alt_part, float* alt_lse, int alt_S,
                                     int alt_tok_off, hipStream_t st);
hipError_t kafka_launch_attn_merge(const float* part, const float* lse, int rows, int Hq, int S, int D, bf16* out,
                                   int64_t out_stride, float* lse_out, const bf16* pre, int npre, hipStream_t st);
hipError_t kafka_launch_sample(const void* logits, bool is_bf16, int64_t stride, int B, int V, const float* temperature,
                         const float* top_p, const int* top_k, const int64_t* seeds, const int64_t* step,
                         int64_t* out_tokens, int* ws, int nsplit, const int* proc, const uint32_t* mask_tab,
                         int64_t mask_ld, int* counts, int64_t cnt_ld, hipStream_t st);
int kafka_wstream_plan(int M, int N, int K, int max_splits, int* mt, int* kc, int* splits);
hipError_t kafka_launch_wstream_gemm(const bf16* X, int64_t ldx, const bf16* Wt, int M, int N, int K, int mt, int kc,
                                     int splits, int nt, int kw, int pin, int glu, bf16* Y, int64_t ldy, float* P,
                                     hipStream_t st);
hipError_t kafka_launch_slab_reduce(const float* P, int S, int M, int N, bf16* Y, int64_t ldy, hipStream_t st);
// host mirror of wstream_gemm.hip's FinArgs (same field order and types; size cross-checked at first use)
struct FinArgs {
  int* tickets;
  const float* ss_in;
  int nss, ss_ld;
  float inv_d, eps;
  bf16* resid;
  int64_t ldr;
  const bf16* nw;
  bf16* xn;
  int64_t ldxn;
  float* ss_out;
  int ss_out_ld;
  const int64_t* positions;
  const float* cos_sin;
  bf16* q_out;
  int64_t q_stride;
  bf16* k_cache;
  bf16* v_cache;
  const int64_t* slots;
  int Hq, Hkv;
  uint64_t* stamps;
  int* err;
};
int kafka_fin_args_size();
hipError_t kafka_launch_wstream_fin(int fin, const bf16* X, int64_t ldx, const bf16* Wt, int M, int N, int K, int mt,
                                    int kc, int splits, int kw, int pin, bf16* Y, int64_t ldy, float* P,
                                    const FinArgs* fa, hipStream_t st);
hipError_t kafka_launch_wstream_grouped(const bf16* X, int64_t ldx, const bf16* Wt, int e_local, int N, int K,
                                        const int* perm_tok, const float* perm_w, const int* expert_off, int e_lo,
                                        int max_rows, int gather, bf16* Y, int64_t ldy, float* out, int64_t ldo,
                                        int pin, hipStream_t st);
hipError_t kafka_launch_moe_route(const bf16* logits, int64_t ld, int T, int E, int K, int BM, float* topk_w,
                                  int* topk_e, int* perm_tok, float* perm_w, int* expert_off, int* tile_off,
                                  hipStream_t st);
hipError_t kafka_launch_grouped_gemm(const bf16* X, int64_t ldx, const bf16* W, int N, int Kd, const int* perm_tok,
                                     const float* perm_w, const int* expert_off, const int* tile_off, int e_lo,
                                     int e_n, int max_tiles, int gather, bf16* Y, int64_t ldy, float* out,
                                     int64_t ldo, hipStream_t st);
hipError_t kafka_car_alloc(int64_t bytes, void** out);
int64_t kafka_car_header_bytes();
hipError_t kafka_car_timing(const void* own, uint64_t* ring_out, int* epoch_out);
hipError_t kafka_car_ipc_handle(void* p, hipIpcMemHandle_t* h);
hipError_t kafka_car_open(const hipIpcMemHandle_t* h, void** out);
hipError_t kafka_car_close(void* p);
hipError_t kafka_car_free(void* p);
hipError_t kafka_launch_car_allreduce(char* const* bases, int nranks, int rank, const bf16* x, const float* xp, int S,
                                      int64_t ps, bf16* y, int64_t n8, int64_t max_bytes, int nblocks,
                                      hipStream_t st);
hipError_t kafka_launch_car_a2a(char* const* bases, int nranks, int rank, const void* send, int64_t nbytes, void* recv,
                                int64_t bpd, int bcast, int64_t max_bytes, int nblocks, hipStream_t st);
hipError_t kafka_launch_ep_dispatch(const bf16* x, int64_t ldx, const int* topk_e, int lo, int n_pairs, int k, int El,
                                    int ep, int C, int MR, int d, bf16* img, int* slot_map, hipStream_t st);
hipError_t kafka_launch_ep_recv_route(const bf16* img, int ep, int C, int MR, int d, int El, int BM, int* perm_tok,
                                      float* perm_w, int* expert_off, int* tile_off, hipStream_t st);
hipError_t kafka_launch_ep_combine(const bf16* back, const int* slot_map, const float* topk_w, int lo, int n_own,
                                   int k, int d, bf16* out, int64_t ldo, hipStream_t st);
int kafka_skinny_plan(int M, int N, int K, int max_splits, int* splits);
hipError_t kafka_launch_skinny_gemm(const bf16* X, int64_t ldx, const bf16* Wt, int M, int N, int K, int splits,
                                    int glu, bf16* Y, int64_t ldy, float* P, hipStream_t st);
hipError_t kafka_launch_car_allreduce_add_rmsnorm(char* const* bases, int nranks, int rank, const bf16* x,
                                                  const float* xp, int S, int64_t ps, int T, int d, bf16* resid,
                                                  int64_t rs, const bf16* w, float eps, bf16* out, int64_t os,
                                                  int64_t max_bytes, int nblocks, const bf16* pre, int64_t pre_s, int dpre, hipStream_t st);
}  // extern "C"

#define CHECK_CUDA(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_DT(x, dt) TORCH_CHECK((x).scalar_type() == (dt), #x " has wrong dtype")
#define CHECK_LASTDIM(x) TORCH_CHECK((x).stride(-1) == 1, #x " must be contiguous in its last dim")
#define CHECK_HIP(e)                                                                 \
  do {                                                                               \
    hipError_t _e = (e);                                                             \
    TORCH_CHECK(_e == hipSuccess, "HIP launch failed: ", hipGetErrorString(_e));    \
  } while (0)

static hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }
static bf16* bptr(const at::Tensor& t) { return reinterpret_cast<bf16*>(t.data_ptr()); }

static void rmsnorm(at::Tensor out, at::Tensor x, at::Tensor w, double eps) {
  CHECK_CUDA(x); CHECK_DT(x, at::kBFloat16); CHECK_DT(w, at::kBFloat16); CHECK_DT(out, at::kBFloat16);
  CHECK_LASTDIM(x); CHECK_LASTDIM(out);
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2 && w.is_contiguous(), "rmsnorm: x/out must be 2-D");
  const int d = x.size(1);
  TORCH_CHECK(d % 8 == 0 && d <= 16384 && w.numel() == d && out.size(0) == x.size(0) && out.size(1) == d,
              "rmsnorm: bad shapes");
  CHECK_HIP(kafka_launch_rmsnorm(bptr(out), out.stride(0), bptr(x), x.stride(0), bptr(w), x.size(0), d, eps,
                                  cur_stream()));
}

// A split-K slab is an fp32 contiguous [S, T, n] tensor (wstream_gemm output); kernels that accept one sum it on load.
static bool is_slab(const at::Tensor& x) { return x.scalar_type() == at::kFloat && x.dim() == 3; }
static void check_slab(const at::Tensor& x) {
  TORCH_CHECK(x.is_contiguous() && x.size(0) >= 1 && x.size(2) % 8 == 0, "slab must be contiguous fp32 [S, T, n]");
}

// x: bf16 [T, d] or slab [S, T, d]
static void fused_add_rmsnorm(at::Tensor out, at::Tensor x, at::Tensor residual, at::Tensor w, double eps) {
  CHECK_CUDA(x); CHECK_DT(residual, at::kBFloat16); CHECK_DT(w, at::kBFloat16);
  CHECK_DT(out, at::kBFloat16);
  CHECK_LASTDIM(x); CHECK_LASTDIM(out); CHECK_LASTDIM(residual);
  const bool slab = is_slab(x);
  if (slab) check_slab(x); else CHECK_DT(x, at::kBFloat16);
  TORCH_CHECK((slab || x.dim() == 2) && residual.dim() == 2 && out.dim() == 2,
              "fused_add_rmsnorm: 2-D tensors (or a 3-D fp32 slab) expected");
  const int64_t T = x.size(slab ? 1 : 0);
  const int d = x.size(slab ? 2 : 1);
  TORCH_CHECK(d % 8 == 0 && d <= 16384 && w.numel() == d && residual.size(0) == T &&
                  residual.size(1) == d && out.size(0) == T && out.size(1) == d,
              "fused_add_rmsnorm: bad shapes");
  if (slab)
    CHECK_HIP(kafka_launch_fused_add_rmsnorm_slab(bptr(out), out.stride(0), x.data_ptr<float>(), x.size(0),
                                                  T * d, bptr(residual), residual.stride(0), bptr(w), T, d, eps,
                                                  cur_stream()));
  else
    CHECK_HIP(kafka_launch_fused_add_rmsnorm(bptr(out), out.stride(0), bptr(x), x.stride(0), bptr(residual),
                                              residual.stride(0), bptr(w), T, d, eps, cur_stream()));
}

// x: bf16 [T, 2F] or slab [S, T, 2F]
static void silu_mul(at::Tensor out, at::Tensor x) {
  CHECK_CUDA(x); CHECK_DT(out, at::kBFloat16);
  const bool slab = is_slab(x);
  if (slab) check_slab(x); else CHECK_DT(x, at::kBFloat16);
  TORCH_CHECK((slab || (x.dim() == 2 && x.stride(1) == 1)) && out.dim() == 2 && out.is_contiguous(),
              "silu_mul: 2-D (or slab)");
  const int F = out.size(1);
  const int64_t T = x.size(slab ? 1 : 0);
  TORCH_CHECK(x.size(slab ? 2 : 1) == 2 * F && F % 8 == 0 && out.size(0) == T, "silu_mul: bad shapes");
  if (slab)
    CHECK_HIP(kafka_launch_silu_mul_slab(bptr(out), x.data_ptr<float>(), x.size(0), T * 2 * F, T, F, cur_stream()));
  else
    CHECK_HIP(kafka_launch_silu_mul(bptr(out), bptr(x), x.stride(0), T, F, cur_stream()));
}

// Paged KV caches: bf16 K[blocks, Hkv, 16, 128] / V[blocks, Hkv, 128, 16], or fp8 (e4m3 + per-token exponents,
// rope_kv.hip) as uint8 K[blocks, Hkv, 16 * 128 + 32] / V[blocks, Hkv, 128 * 16].
static bool is_fp8_cache(const at::Tensor& k) { return k.scalar_type() == at::kByte; }

static void check_cache_pair(const at::Tensor& k_cache, const at::Tensor& v_cache) {
  TORCH_CHECK(k_cache.is_contiguous() && v_cache.is_contiguous(), "caches must be contiguous");
  TORCH_CHECK(k_cache.is_cuda() && v_cache.is_cuda(), "caches must be GPU tensors");
  if (is_fp8_cache(k_cache)) {
    CHECK_DT(v_cache, at::kByte);
    TORCH_CHECK(k_cache.dim() == 3 && v_cache.dim() == 3 && k_cache.size(2) == 16 * 128 + 32 &&
                    v_cache.size(2) == 128 * 16 && k_cache.size(0) == v_cache.size(0) &&
                    k_cache.size(1) == v_cache.size(1),
                "fp8 paged caches must be uint8 K[blocks,Hkv,2080] / V[blocks,Hkv,2048]");
    return;
  }
  CHECK_DT(k_cache, at::kBFloat16); CHECK_DT(v_cache, at::kBFloat16);
  TORCH_CHECK(k_cache.dim() == 4 && v_cache.dim() == 4 && k_cache.size(2) == 16 && k_cache.size(3) == 128 &&
                  v_cache.size(2) == 128 && v_cache.size(3) == 16 && k_cache.size(0) == v_cache.size(0) &&
                  k_cache.size(1) == v_cache.size(1),
              "paged caches must be K[blocks,Hkv,16,128] / V[blocks,Hkv,128,16]");
}

static void rope_kv_write(at::Tensor qkv, at::Tensor positions, at::Tensor cos_sin, at::Tensor q_out,
                          at::Tensor k_cache, at::Tensor v_cache, c10::optional<at::Tensor> slot_mapping, int64_t Hq,
                          int64_t Hkv) {
  CHECK_CUDA(qkv); CHECK_DT(q_out, at::kBFloat16);
  const bool slab = is_slab(qkv);
  if (slab) check_slab(qkv); else CHECK_DT(qkv, at::kBFloat16);
  CHECK_DT(positions, at::kLong); CHECK_DT(cos_sin, at::kFloat);
  TORCH_CHECK(k_cache.is_contiguous() && v_cache.is_contiguous() && cos_sin.is_contiguous() &&
                  positions.is_contiguous(), "rope_kv_write: caches/positions/cos_sin must be contiguous");
  const bool fp8 = is_fp8_cache(k_cache);
  int D, bs = 16;
  if (fp8) {
    check_cache_pair(k_cache, v_cache);
    D = 128;
    TORCH_CHECK(k_cache.size(1) == Hkv, "rope_kv_write: cache shape mismatch");
  } else {
    CHECK_DT(k_cache, at::kBFloat16); CHECK_DT(v_cache, at::kBFloat16);
    TORCH_CHECK(k_cache.dim() == 4 && v_cache.dim() == 4, "k/v cache must be [blocks, Hkv, ., .]");
    D = k_cache.size(3);
    bs = k_cache.size(2);
    TORCH_CHECK(k_cache.size(1) == Hkv && v_cache.size(1) == Hkv && v_cache.size(2) == D && v_cache.size(3) == bs &&
                    v_cache.size(0) == k_cache.size(0), "rope_kv_write: cache shape mismatch");
    TORCH_CHECK(bs == 16, "page size must be 16");
    TORCH_CHECK(D == 128 || D == 64, "head dim must be 64 or 128");
  }
  const int T = qkv.size(slab ? 1 : 0);
  const int64_t W = (Hq + 2 * Hkv) * D;
  TORCH_CHECK(slab ? qkv.size(2) == W : (qkv.dim() == 2 && qkv.stride(1) == 1 && qkv.size(1) == W), "qkv shape");
  TORCH_CHECK(positions.numel() == T && cos_sin.dim() == 2 && cos_sin.size(1) == D, "positions/cos_sin shape");
  TORCH_CHECK(q_out.dim() == 3 && q_out.size(0) == T && q_out.size(1) == Hq && q_out.size(2) == D &&
                  q_out.stride(2) == 1 && q_out.stride(1) == D, "q_out shape");
  const int64_t* sm = nullptr;
  if (slot_mapping.has_value()) {
    CHECK_DT(slot_mapping.value(), at::kLong);
    TORCH_CHECK(slot_mapping->numel() == T && slot_mapping->is_contiguous(), "slot_mapping shape");
    sm = slot_mapping->data_ptr<int64_t>();
  }
  if (fp8)
    CHECK_HIP(kafka_launch_rope_kv_fp8(slab ? nullptr : bptr(qkv), slab ? qkv.data_ptr<float>() : nullptr,
                                        slab ? qkv.size(0) : 0, slab ? (int64_t)T * W : 0, slab ? W : qkv.stride(0),
                                        positions.data_ptr<int64_t>(), cos_sin.data_ptr<float>(), bptr(q_out),
                                        q_out.stride(0), k_cache.data_ptr<uint8_t>(), v_cache.data_ptr<uint8_t>(), sm,
                                        T, Hq, Hkv, D, cur_stream()));
  else
    CHECK_HIP(kafka_launch_rope_kv(slab ? nullptr : bptr(qkv), slab ? qkv.data_ptr<float>() : nullptr,
                                    slab ? qkv.size(0) : 0, slab ? (int64_t)T * W : 0, slab ? W : qkv.stride(0),
                                    positions.data_ptr<int64_t>(), cos_sin.data_ptr<float>(), bptr(q_out),
                                    q_out.stride(0), bptr(k_cache), bptr(v_cache), sm, T, Hq, Hkv, D, bs,
                                    cur_stream()));
}

// items: int32 [n, 8] decode work items (b, lo, hi, split, nsplit, npre, 0, 0) — see attention.hip DecodeItem.
// Their values are device data; the kernel drops an item whose b / slots fall outside the checked buffer shapes.
static void attn_decode(at::Tensor q, at::Tensor k_cache, at::Tensor v_cache, at::Tensor block_tables,
                        at::Tensor items, at::Tensor out_part, at::Tensor lse_part, double scale,
                        c10::optional<at::Tensor> out, c10::optional<at::Tensor> tickets,
                        c10::optional<at::Tensor> pre_part, c10::optional<at::Tensor> m_part,
                        c10::optional<at::Tensor> m_lse, c10::optional<at::Tensor> m_out) {
  CHECK_CUDA(q); CHECK_DT(q, at::kBFloat16); check_cache_pair(k_cache, v_cache);
  CHECK_DT(block_tables, at::kInt); CHECK_DT(items, at::kInt); CHECK_DT(out_part, at::kFloat);
  CHECK_DT(lse_part, at::kFloat);
  TORCH_CHECK(q.dim() == 3 && q.stride(2) == 1 && q.stride(1) == 128 && q.size(2) == 128, "q must be [B, Hq, 128]");
  const int B = q.size(0), Hq = q.size(1), Hkv = k_cache.size(1);
  TORCH_CHECK(Hq % Hkv == 0 && Hq / Hkv <= 8, "decode kernel needs Hq/Hkv <= 8");
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(0) >= B && block_tables.stride(1) == 1, "block_tables");
  TORCH_CHECK(items.is_cuda() && items.is_contiguous() && items.dim() == 2 && items.size(1) == 8,
              "items must be a device int32 [n, 8]");
  TORCH_CHECK(out_part.is_contiguous() && out_part.dim() == 4 && out_part.size(0) >= B && out_part.size(1) == Hq &&
                  out_part.size(3) == 128, "out_part must be [B, Hq, S_total, 128]");
  const int S_total = out_part.size(2);
  TORCH_CHECK(lse_part.is_contiguous() && lse_part.numel() >= (int64_t)B * Hq * S_total, "lse_part");
  bf16* op = nullptr;
  int64_t ostride = 0;
  int* tp = nullptr;
  if (out.has_value()) {  // fused merge: final bf16 rows [B, Hq, 128]
    CHECK_DT(out.value(), at::kBFloat16);
    TORCH_CHECK(out->dim() == 3 && out->size(0) >= B && out->size(1) == Hq && out->size(2) == 128 &&
                    out->stride(2) == 1 && out->stride(1) == 128,
                "attn_decode: fused-merge out must be [B, Hq, 128]");
    op = bptr(out.value());
    ostride = out->stride(0);
    TORCH_CHECK(tickets.has_value() && tickets->is_cuda() && tickets->scalar_type() == at::kInt &&
                    tickets->numel() >= (int64_t)B * Hkv,
                "attn_decode: the fused merge needs an int32 ticket buffer of >= B * Hkv zeros");
    tp = tickets->data_ptr<int>();
    TORCH_CHECK(out_part.numel() * 4 < 0x7fffffffLL, "attn_decode: the ticket merge addresses out_part as a < 2 GiB buffer");
  }
  const bf16* pre = nullptr;  // bf16 cascade prefix partials (slots < npre), same [B, Hq, S_total, 128] indexing
  if (pre_part.has_value()) {
    CHECK_DT(pre_part.value(), at::kBFloat16);
    TORCH_CHECK(pre_part->is_contiguous() && pre_part->sizes() == out_part.sizes(),
                "attn_decode: pre_part must match out_part's shape");
    pre = bptr(pre_part.value());
  }
  // fused merge of prefill rows (attention.hip FusedMerge): m_part [rows, Hq, S2, 128] / m_lse [rows, Hq, S2] fp32
  // -> m_out [rows, Hq, 128] bf16
  const float *mp = nullptr, *ml = nullptr;
  bf16* mo = nullptr;
  int mS = 0, mrows = 0;
  int64_t mstride = 0;
  if (m_part.has_value()) {
    TORCH_CHECK(m_lse.has_value() && m_out.has_value(), "attn_decode: a fused merge needs m_part, m_lse and m_out");
    CHECK_CUDA(m_part.value()); CHECK_DT(m_part.value(), at::kFloat); CHECK_DT(m_lse.value(), at::kFloat);
    CHECK_DT(m_out.value(), at::kBFloat16);
    TORCH_CHECK(m_part->is_contiguous() && m_part->dim() == 4 && m_part->size(1) == Hq && m_part->size(3) == 128,
                "attn_decode: m_part must be contiguous [rows, Hq, S, 128]");
    mrows = m_part->size(0);
    mS = m_part->size(2);
    TORCH_CHECK(m_lse->is_contiguous() && m_lse->numel() == (int64_t)mrows * Hq * mS, "attn_decode: m_lse");
    TORCH_CHECK(m_out->dim() == 3 && m_out->size(0) == mrows && m_out->size(1) == Hq && m_out->size(2) == 128 &&
                    m_out->stride(2) == 1 && m_out->stride(1) == 128,
                "attn_decode: m_out must be [rows, Hq, 128] with 128-element head rows");
    mp = m_part->data_ptr<float>();
    ml = m_lse->data_ptr<float>();
    mo = bptr(m_out.value());
    mstride = m_out->stride(0);
  }
  CHECK_HIP(kafka_launch_attn_decode(bptr(q), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                                      is_fp8_cache(k_cache) ? 1 : 0, items.size(0), B, Hkv,
                                      Hq / Hkv, 128, block_tables.data_ptr<int>(), block_tables.stride(0),
                                      items.data_ptr<int>(), out_part.data_ptr<float>(), lse_part.data_ptr<float>(),
                                      S_total, scale, op, ostride, tp, pre, mp, ml, mS, mrows, mo, mstride,
                                      cur_stream()));
}

static void attn_prefill(at::Tensor items, at::Tensor q, at::Tensor k_cache, at::Tensor v_cache,
                         at::Tensor block_tables, at::Tensor q_limit, c10::optional<at::Tensor> out,
                         c10::optional<at::Tensor> out_part, c10::optional<at::Tensor> lse_part, double scale,
                         int64_t variant, c10::optional<at::Tensor> alt_part, c10::optional<at::Tensor> alt_lse,
                         int64_t alt_tok_off) {
  CHECK_CUDA(q); CHECK_DT(q, at::kBFloat16); check_cache_pair(k_cache, v_cache);
  CHECK_DT(items, at::kInt); CHECK_DT(block_tables, at::kInt); CHECK_DT(q_limit, at::kInt);
  TORCH_CHECK(items.is_contiguous() && items.dim() == 2 && items.size(1) == 8, "items must be [n, 8] int32");
  TORCH_CHECK(q.dim() == 3 && q.stride(2) == 1 && q.stride(1) == 128 && q.size(2) == 128, "q must be [T, Hq, 128]");
  const int T = q.size(0), Hq = q.size(1), Hkv = k_cache.size(1);
  TORCH_CHECK(Hq % Hkv == 0, "Hq % Hkv");
  const int G = Hq / Hkv;
  TORCH_CHECK(G <= 32 && 128 % G == 0, "prefill kernel needs Hq/Hkv dividing 128");
  TORCH_CHECK(q_limit.numel() >= T && q_limit.is_contiguous(), "q_limit");
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.stride(1) == 1, "block_tables");
  bf16* op = nullptr;
  int64_t os = 0;
  if (out.has_value()) {
    CHECK_DT(out.value(), at::kBFloat16);
    TORCH_CHECK(out->dim() == 3 && out->size(0) >= T && out->size(1) == Hq && out->size(2) == 128 &&
                    out->stride(2) == 1 && out->stride(1) == 128, "out must be [T, Hq, 128]");
    op = bptr(out.value());
    os = out->stride(0);
  }
  float* pp = nullptr;
  float* lp = nullptr;
  int S_total = 0;
  int part_bf16 = 0;
  if (out_part.has_value()) {
    TORCH_CHECK(lse_part.has_value(), "lse_part required with out_part");
    part_bf16 = out_part->scalar_type() == at::kBFloat16 ? 1 : 0;  // bf16 partials: tile variant 3 only
    TORCH_CHECK(!part_bf16 || variant == 3, "attn_prefill: bf16 out_part needs tile variant 3");
    if (!part_bf16) CHECK_DT(out_part.value(), at::kFloat);
    CHECK_DT(lse_part.value(), at::kFloat);
    // (with alt partials the main buffer covers the rows below alt_tok_off: the decode rows of a cascade pass whose
    // prefill rows write the alt buffer)
    const int64_t rows_main = alt_part.has_value() ? std::min<int64_t>(T, alt_tok_off) : T;
    TORCH_CHECK(out_part->is_contiguous() && out_part->dim() == 4 && out_part->size(0) >= rows_main &&
                    out_part->size(1) == Hq && out_part->size(3) == 128, "out_part must be [T, Hq, S, 128]");
    S_total = out_part->size(2);
    TORCH_CHECK(lse_part->is_contiguous() && lse_part->numel() >= rows_main * Hq * S_total, "lse_part");
    pp = reinterpret_cast<float*>(out_part->data_ptr());
    lp = lse_part->data_ptr<float>();
  }
  TORCH_CHECK(op != nullptr || pp != nullptr, "attn_prefill needs out or out_part");
  // alt partials (items with field 6 set, tile variant 3): fp32 [rows, Hq, S2, 128] + lse, row = token - alt_tok_off
  float* ap = nullptr;
  float* al = nullptr;
  int S2 = 0;
  if (alt_part.has_value()) {
    TORCH_CHECK(variant == 3 && alt_lse.has_value(), "attn_prefill: alt partials need tile variant 3 and alt_lse");
    CHECK_DT(alt_part.value(), at::kFloat); CHECK_DT(alt_lse.value(), at::kFloat);
    TORCH_CHECK(alt_part->is_contiguous() && alt_part->dim() == 4 && alt_part->size(1) == Hq &&
                    alt_part->size(3) == 128 && alt_tok_off >= 0 && alt_part->size(0) + alt_tok_off >= T,
                "attn_prefill: alt_part must be [>= T - alt_tok_off, Hq, S, 128]");
    S2 = alt_part->size(2);
    TORCH_CHECK(alt_lse->is_contiguous() && alt_lse->numel() >= alt_part->size(0) * Hq * S2, "attn_prefill: alt_lse");
    ap = alt_part->data_ptr<float>();
    al = alt_lse->data_ptr<float>();
  }
  CHECK_HIP(kafka_launch_attn_prefill(items.data_ptr<int>(), items.size(0), bptr(q), q.stride(0), k_cache.data_ptr(),
                                       v_cache.data_ptr(), is_fp8_cache(k_cache) ? 1 : 0, Hkv, G, 128, block_tables.data_ptr<int>(),
                                       block_tables.stride(0), q_limit.data_ptr<int>(), op, os, pp, lp, S_total,
                                       scale, (int)variant, part_bf16, ap, al, S2, (int)alt_tok_off, cur_stream()));
}

static void attn_merge(at::Tensor part, at::Tensor lse, at::Tensor out, c10::optional<at::Tensor> lse_out,
                       c10::optional<at::Tensor> pre, int64_t npre) {
  CHECK_CUDA(part); CHECK_DT(part, at::kFloat); CHECK_DT(lse, at::kFloat); CHECK_DT(out, at::kBFloat16);
  TORCH_CHECK(part.is_contiguous() && part.dim() == 4 && part.size(3) == 128, "part must be [rows, Hq, S, 128]");
  const int rows = out.size(0), Hq = part.size(1), S = part.size(2);
  TORCH_CHECK(part.size(0) >= rows && out.dim() == 3 && out.size(1) == Hq && out.size(2) == 128 &&
                  out.stride(2) == 1 && out.stride(1) == 128, "out must be [rows, Hq, 128]");
  TORCH_CHECK(lse.is_contiguous() && lse.numel() >= (int64_t)rows * Hq * S, "lse");
  float* lo = nullptr;
  if (lse_out.has_value()) {
    CHECK_DT(lse_out.value(), at::kFloat);
    TORCH_CHECK(lse_out->numel() >= (int64_t)rows * Hq, "lse_out");
    lo = lse_out->data_ptr<float>();
  }
  const bf16* pp = nullptr;
  if (pre.has_value()) {  // bf16 prefix partials in slots [0, npre), part's shape
    CHECK_DT(pre.value(), at::kBFloat16);
    TORCH_CHECK(pre->is_contiguous() && pre->sizes() == part.sizes() && npre >= 0 && npre <= S, "attn_merge: pre");
    pp = bptr(pre.value());
  }
  CHECK_HIP(kafka_launch_attn_merge(part.data_ptr<float>(), lse.data_ptr<float>(), rows, Hq, S, 128, bptr(out),
                                     out.stride(0), lo, pp, (int)npre, cur_stream()));
}

static void sample(at::Tensor logits, c10::optional<at::Tensor> temperature, c10::optional<at::Tensor> top_p,
                   c10::optional<at::Tensor> top_k, c10::optional<at::Tensor> seeds, c10::optional<at::Tensor> step,
                   at::Tensor out, c10::optional<at::Tensor> ws, int64_t nsplit, c10::optional<at::Tensor> proc,
                   c10::optional<at::Tensor> mask_tab, c10::optional<at::Tensor> counts) {
  CHECK_CUDA(logits); CHECK_DT(out, at::kLong);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits must be [B, V]");
  const bool is_bf16 = logits.scalar_type() == at::kBFloat16;
  TORCH_CHECK(is_bf16 || logits.scalar_type() == at::kFloat, "logits must be bf16 or fp32");
  const int B = logits.size(0), V = logits.size(1);
  TORCH_CHECK(out.numel() >= B && out.is_contiguous(), "out");
  TORCH_CHECK(logits.stride(0) % 8 == 0, "logits row stride must be a multiple of 8");
  auto fp = [&](const c10::optional<at::Tensor>& t, at::ScalarType dt) -> void* {
    if (!t.has_value()) return nullptr;
    TORCH_CHECK(t->scalar_type() == dt && t->is_contiguous() && t->numel() >= B, "sampling param dtype/shape");
    return t->data_ptr();
  };
  void* st = nullptr;
  if (step.has_value()) {
    TORCH_CHECK(step->scalar_type() == at::kLong && step->numel() >= 1, "step must be int64[1]");
    st = step->data_ptr();
  }
  int* wp = nullptr;
  if (ws.has_value() && nsplit > 1) {  // split rows: tickets [65536] | partials [B][nsplit][2]
    TORCH_CHECK(ws->is_cuda() && ws->scalar_type() == at::kInt && ws->is_contiguous() &&
                    ws->numel() >= 65536 + 2 * (int64_t)B * nsplit && nsplit <= 64,
                "sample: workspace must be int32 [>= 65536 + 2 * B * nsplit]");
    wp = ws->data_ptr<int>();
  }
  // logits processing: proc int32 [B, 8] (mode, mask row / forced id, penalty slot, presence, frequency), the
  // bitmask table uint32-as-int32 [rows, >= V / 32] and the count table int32 [slots, >= V rounded to 8]. The
  // kernel trusts the row / slot / forced-id values: the host builder (engine/logits_proc.py) range-checks them
  // against these tables before the plan is uploaded
  const int* pp = nullptr;
  const uint32_t* mt = nullptr;
  int* cp = nullptr;
  int64_t mld = 0, cld = 0;
  if (proc.has_value()) {
    TORCH_CHECK(proc->is_cuda() && proc->scalar_type() == at::kInt && proc->is_contiguous() && proc->dim() == 2 &&
                    proc->size(0) >= B && proc->size(1) == 8, "sample: proc must be int32 [>= B, 8] on the GPU");
    TORCH_CHECK(mask_tab.has_value() && mask_tab->is_cuda() && mask_tab->scalar_type() == at::kInt &&
                    mask_tab->is_contiguous() && mask_tab->dim() == 2 && mask_tab->size(1) * 32 >= V,
                "sample: mask_tab must be int32 [rows, >= V / 32] on the GPU");
    pp = proc->data_ptr<int>();
    mt = reinterpret_cast<const uint32_t*>(mask_tab->data_ptr<int>());
    mld = mask_tab->size(1);
    if (counts.has_value()) {
      TORCH_CHECK(counts->is_cuda() && counts->scalar_type() == at::kInt && counts->is_contiguous() &&
                      counts->dim() == 2 && counts->size(1) >= ((V + 7) & ~7) && counts->size(1) % 8 == 0,
                  "sample: counts must be int32 [slots, >= V rounded up to 8]");
      cp = counts->data_ptr<int>();
      cld = counts->size(1);
    }
  }
  CHECK_HIP(kafka_launch_sample(logits.data_ptr(), is_bf16, logits.stride(0), B, V,
                                 (const float*)fp(temperature, at::kFloat), (const float*)fp(top_p, at::kFloat),
                                 (const int*)fp(top_k, at::kInt), (const int64_t*)fp(seeds, at::kLong),
                                 (const int64_t*)st, out.data_ptr<int64_t>(), wp, wp ? (int)nsplit : 1, pp, mt, mld,
                                 cp, cld, cur_stream()));
}

// (mt, kc, splits) of the weight-streaming decode GEMM for a shape, or (0, 0, 0) if unsupported
static std::vector<int64_t> wstream_plan(int64_t M, int64_t N, int64_t K, int64_t max_splits) {
  int mt = 0, kc = 0, s = 0;
  if (kafka_wstream_plan((int)M, (int)N, (int)K, (int)max_splits, &mt, &kc, &s) != 0) return {0, 0, 0};
  return {mt, kc, s};
}

// x [M, K] bf16 . W^T with W given wave-tiled as wt [N/32, K/16, 64, 8] (ops.tile_weight). Writes bf16 y [M, N]
// (splits == 1) or fp32 slabs p [splits, M, N].
static void wstream_gemm(at::Tensor x, at::Tensor wt, c10::optional<at::Tensor> y, c10::optional<at::Tensor> p,
                         int64_t max_splits, bool nt, bool glu) {
  CHECK_CUDA(x); CHECK_DT(x, at::kBFloat16); CHECK_DT(wt, at::kBFloat16); CHECK_LASTDIM(x);
  TORCH_CHECK(x.dim() == 2 && x.stride(0) % 8 == 0, "wstream_gemm: x must be [M, K] with 16-B rows");
  TORCH_CHECK(wt.dim() == 4 && wt.is_contiguous() && wt.size(2) == 64 && wt.size(3) == 8,
              "wstream_gemm: wt must be contiguous [N/32, K/16, 64, 8]");
  const int M = x.size(0), K = x.size(1), N = wt.size(0) * 32;
  TORCH_CHECK(wt.size(1) * 16 == K, "wstream_gemm: K mismatch");
  TORCH_CHECK(!glu || N % 64 == 0, "wstream_gemm: GLU weights need N % 64 == 0");
  int mt = 0, kc = 0, s = 0;
  TORCH_CHECK(kafka_wstream_plan(M, N, K, (int)max_splits, &mt, &kc, &s) == 0, "wstream_gemm: unsupported shape");
  bf16* yp = nullptr;
  int64_t ldy = 0;
  float* pp = nullptr;
  if (s == 1) {
    // glu + one split: y is the activated [M, N/2]; otherwise [M, N] in gate | up column order
    TORCH_CHECK(y.has_value(), "wstream_gemm: y required for a single split");
    CHECK_DT(y.value(), at::kBFloat16); CHECK_LASTDIM(y.value());
    TORCH_CHECK(y->dim() == 2 && y->size(0) == M && y->size(1) == (glu ? N / 2 : N), "wstream_gemm: y shape");
    yp = bptr(y.value());
    ldy = y->stride(0);
  } else {
    TORCH_CHECK(p.has_value(), "wstream_gemm: slab output required");
    CHECK_DT(p.value(), at::kFloat);
    TORCH_CHECK(p->is_contiguous() && p->dim() == 3 && p->size(0) == s && p->size(1) == M && p->size(2) == N,
                "wstream_gemm: slab shape must be [splits, M, N]");
    pp = p->data_ptr<float>();
  }
  // two K halves per chunk (8 waves) for 64-row tiles with >= 6 chunks per split: the long streams (gate_up unsplit
  // with its fused SwiGLU, down) ran 1.6-2.8 % faster in the config sweep, the short ones (qkv, o) slower; headline
  // +0.24 % (3 / 3 interleaved pairs, profiles/r04/bench_ab_wstream_kw2.jsonl)
  const int kw = mt == 2 && kc == 256 && K / s / kc >= 6 ? 2 : 1;
  // weight prefetch pinned ahead of the MFMAs (wstream_gemm_kernel PIN) when a split streams >= 3 chunks: -1..-4 us
  // per projection at 64 rows, -4..-7 us at 97..128 rows; not for 96-row tiles (their 348 registers leave one wave
  // per SIMD and the longer live ranges lose) nor 2-chunk splits (o at 64 rows: +0.9 us)
  // (profiles/r05/wstream_sweep_pin.jsonl)
  const int pin = mt != 3 && K / s / kc >= 3 ? 1 : 0;
  CHECK_HIP(kafka_launch_wstream_gemm(bptr(x), x.stride(0), bptr(wt), M, N, K, mt, kc, s, nt ? 1 : 0, kw, pin,
                                      glu ? 1 : 0,
                                      yp, ldy, pp, cur_stream()));
}

// Fused decode-layer GEMMs (wstream_gemm.hip FIN_*): fin 1 = o / down with the split-K finisher doing the residual
// add, the next RMSNorm's weight and its row partial sums (resid, nw, xn, ss_out); 2 = qkv with RoPE + paged KV
// write in the finisher (positions, cos_sin, q_out, caches, slots, Hq, Hkv); 3 = gate_up with the SwiGLU epilogue
// (one split, y [M, N/2]). ss_in (fp32 [K/128, >= M]): partial sums of squares of X's rows — X is then the
// un-normalised bf16(h * w) and each row is scaled by rsqrt(sum / K + eps) after the GEMM.
static void wstream_fin(int64_t fin, at::Tensor x, at::Tensor wt, c10::optional<at::Tensor> y,
                        c10::optional<at::Tensor> p, at::Tensor tickets, c10::optional<at::Tensor> ss_in, double eps,
                        c10::optional<at::Tensor> resid, c10::optional<at::Tensor> nw, c10::optional<at::Tensor> xn,
                        c10::optional<at::Tensor> ss_out, c10::optional<at::Tensor> positions,
                        c10::optional<at::Tensor> cos_sin, c10::optional<at::Tensor> q_out,
                        c10::optional<at::Tensor> k_cache, c10::optional<at::Tensor> v_cache,
                        c10::optional<at::Tensor> slots, int64_t Hq, int64_t Hkv, int64_t max_splits,
                        c10::optional<at::Tensor> stamps) {
  static const bool abi_ok = kafka_fin_args_size() == (int)sizeof(FinArgs);
  TORCH_CHECK(abi_ok, "wstream_fin: FinArgs layout differs between the kernel and the bindings");
  TORCH_CHECK(fin >= 1 && fin <= 3, "wstream_fin: fin must be 1, 2 or 3");
  CHECK_CUDA(x); CHECK_DT(x, at::kBFloat16); CHECK_DT(wt, at::kBFloat16); CHECK_LASTDIM(x);
  TORCH_CHECK(x.dim() == 2 && x.stride(0) % 8 == 0, "wstream_fin: x must be [M, K] with 16-B rows");
  TORCH_CHECK(wt.dim() == 4 && wt.is_contiguous() && wt.size(2) == 64 && wt.size(3) == 8,
              "wstream_fin: wt must be contiguous [N/32, K/16, 64, 8]");
  const int M = x.size(0), K = x.size(1), N = wt.size(0) * 32;
  TORCH_CHECK(wt.size(1) * 16 == K && M >= 1 && M <= 128 && N % 128 == 0, "wstream_fin: shape");
  int mt = 0, kc = 0, s = 0;
  TORCH_CHECK(kafka_wstream_plan(M, N, K, fin == 3 ? 1 : (int)max_splits, &mt, &kc, &s) == 0,
              "wstream_fin: unsupported shape");
  CHECK_DT(tickets, at::kInt);
  TORCH_CHECK(tickets.is_cuda() && tickets.is_contiguous() && tickets.numel() >= N / 128, "wstream_fin: tickets");
  FinArgs fa{};
  fa.tickets = tickets.data_ptr<int>();
  TORCH_CHECK(tickets.numel() >= N / 128 + 1, "wstream_fin: tickets need N/128 + 1 entries (the last one is the error word)");
  fa.err = tickets.data_ptr<int>() + (tickets.numel() - 1);
  fa.eps = (float)eps;
  fa.inv_d = 1.f / (float)K;
  if (ss_in.has_value()) {
    CHECK_DT(ss_in.value(), at::kFloat);
    TORCH_CHECK(ss_in->is_cuda() && ss_in->dim() == 2 && (ss_in->stride(1) == 1 || ss_in->size(1) == 1) &&
                    ss_in->size(0) * 128 == K && ss_in->size(1) >= M && ss_in->stride(0) >= M,
                "wstream_fin: ss_in must be fp32 [K/128, >= M] with unit column stride");
    fa.ss_in = ss_in->data_ptr<float>();
    fa.nss = ss_in->size(0);
    fa.ss_ld = ss_in->stride(0);
  }
  const int kw = mt == 2 && kc == 256 && K / s / kc >= 6 ? 2 : 1;  // (the wstream_gemm rules above)
  const int pin = mt != 3 && K / s / kc >= 3 ? 1 : 0;
  bf16* yp = nullptr;
  int64_t ldy = 0;
  float* pp = nullptr;
  if (s > 1) {
    TORCH_CHECK(p.has_value(), "wstream_fin: slab scratch required");
    CHECK_DT(p.value(), at::kFloat);
    TORCH_CHECK(p->is_cuda() && p->is_contiguous() && p->dim() == 3 && p->size(0) == s && p->size(1) == M &&
                    p->size(2) == N, "wstream_fin: slab scratch must be [splits, M, N]");
    TORCH_CHECK((int64_t)s * M * N * 4 < 0x7fffffffLL, "wstream_fin: slab scratch beyond 2 GiB");
    pp = p->data_ptr<float>();
  }
  if (fin == 1) {
    TORCH_CHECK(resid.has_value() && nw.has_value() && xn.has_value() && ss_out.has_value(), "wstream_fin: fin 1 args");
    CHECK_DT(resid.value(), at::kBFloat16); CHECK_DT(nw.value(), at::kBFloat16); CHECK_DT(xn.value(), at::kBFloat16);
    CHECK_DT(ss_out.value(), at::kFloat);
    CHECK_LASTDIM(resid.value()); CHECK_LASTDIM(xn.value()); CHECK_LASTDIM(ss_out.value());
    TORCH_CHECK(resid->dim() == 2 && resid->size(0) == M && resid->size(1) == N && resid->stride(0) % 4 == 0 &&
                    xn->dim() == 2 && xn->size(0) == M && xn->size(1) == N && xn->stride(0) % 4 == 0 &&
                    nw->is_contiguous() && nw->numel() == N && ss_out->dim() == 2 && ss_out->size(0) == N / 128 &&
                    ss_out->size(1) >= M, "wstream_fin: fin 1 shapes");
    fa.resid = bptr(resid.value());
    fa.ldr = resid->stride(0);
    fa.nw = bptr(nw.value());
    fa.xn = bptr(xn.value());
    fa.ldxn = xn->stride(0);
    fa.ss_out = ss_out->data_ptr<float>();
    fa.ss_out_ld = ss_out->stride(0);
  } else if (fin == 2) {
    TORCH_CHECK(positions.has_value() && cos_sin.has_value() && q_out.has_value(), "wstream_fin: fin 2 args");
    CHECK_DT(positions.value(), at::kLong); CHECK_DT(cos_sin.value(), at::kFloat); CHECK_DT(q_out.value(), at::kBFloat16);
    TORCH_CHECK(N == (Hq + 2 * Hkv) * 128, "wstream_fin: qkv width must be (Hq + 2 Hkv) * 128");
    TORCH_CHECK(positions->is_contiguous() && positions->numel() == M && cos_sin->is_contiguous() &&
                    cos_sin->dim() == 2 && cos_sin->size(1) == 128, "wstream_fin: positions / cos_sin");
    TORCH_CHECK(q_out->dim() == 3 && q_out->size(0) == M && q_out->size(1) == Hq && q_out->size(2) == 128 &&
                    q_out->stride(2) == 1 && q_out->stride(1) == 128 && q_out->stride(0) % 4 == 0, "wstream_fin: q_out");
    fa.positions = positions->data_ptr<int64_t>();
    fa.cos_sin = cos_sin->data_ptr<float>();
    fa.q_out = bptr(q_out.value());
    fa.q_stride = q_out->stride(0);
    fa.Hq = Hq;
    fa.Hkv = Hkv;
    if (slots.has_value()) {
      TORCH_CHECK(k_cache.has_value() && v_cache.has_value(), "wstream_fin: caches required with slots");
      check_cache_pair(k_cache.value(), v_cache.value());
      TORCH_CHECK(!is_fp8_cache(k_cache.value()) && k_cache->size(1) == Hkv, "wstream_fin: bf16 caches of Hkv heads");
      CHECK_DT(slots.value(), at::kLong);
      TORCH_CHECK(slots->is_contiguous() && slots->numel() == M, "wstream_fin: slots shape");
      fa.slots = slots->data_ptr<int64_t>();
      fa.k_cache = bptr(k_cache.value());
      fa.v_cache = bptr(v_cache.value());
    }
  } else {
    TORCH_CHECK(s == 1 && y.has_value(), "wstream_fin: fin 3 needs one split and y");
    CHECK_DT(y.value(), at::kBFloat16); CHECK_LASTDIM(y.value());
    TORCH_CHECK(y->dim() == 2 && y->size(0) == M && y->size(1) == N / 2, "wstream_fin: y must be [M, N/2]");
    yp = bptr(y.value());
    ldy = y->stride(0);
  }
  if (stamps.has_value()) {
    TORCH_CHECK(stamps->is_cuda() && stamps->scalar_type() == at::kLong && stamps->is_contiguous() &&
                    stamps->numel() >= (int64_t)(N / 128) * s * 8, "wstream_fin: stamps must be int64 [grid * 8]");
    fa.stamps = reinterpret_cast<uint64_t*>(stamps->data_ptr<int64_t>());
  }
  CHECK_HIP(kafka_launch_wstream_fin((int)fin, bptr(x), x.stride(0), bptr(wt), M, N, K, mt, kc, s, kw, pin, yp, ldy, pp,
                                     &fa, cur_stream()));
}

// Skinny MFMA GEMM (csrc/skinny_gemm.hip) for 129..256 rows on the wave-tiled weights: y bf16 for one split
// ([M, N/2] activated with glu), else fp32 slabs p [splits, M, N]
static int64_t skinny_plan(int64_t M, int64_t N, int64_t K, int64_t max_splits) {
  int s = 0;
  return kafka_skinny_plan((int)M, (int)N, (int)K, (int)max_splits, &s) == 0 ? s : 0;
}

static void skinny_gemm(at::Tensor x, at::Tensor wt, c10::optional<at::Tensor> y, c10::optional<at::Tensor> p,
                        int64_t splits, bool glu) {
  CHECK_CUDA(x); CHECK_DT(x, at::kBFloat16); CHECK_DT(wt, at::kBFloat16); CHECK_LASTDIM(x);
  TORCH_CHECK(x.dim() == 2 && x.stride(0) % 8 == 0, "skinny_gemm: x must be [M, K] with 16-B rows");
  TORCH_CHECK(wt.dim() == 4 && wt.is_contiguous() && wt.size(2) == 64 && wt.size(3) == 8,
              "skinny_gemm: wt must be contiguous [N/32, K/16, 64, 8]");
  const int M = x.size(0), K = x.size(1), N = wt.size(0) * 32;
  TORCH_CHECK(wt.size(1) * 16 == K && M > 0 && M <= 256 && N % 128 == 0 && K % (64 * splits) == 0,
              "skinny_gemm: shape");
  bf16* yp = nullptr;
  int64_t ldy = 0;
  float* pp = nullptr;
  if (splits == 1) {
    TORCH_CHECK(y.has_value(), "skinny_gemm: y required for one split");
    CHECK_DT(y.value(), at::kBFloat16); CHECK_LASTDIM(y.value());
    TORCH_CHECK(y->dim() == 2 && y->size(0) == M && y->size(1) == (glu ? N / 2 : N), "skinny_gemm: y shape");
    yp = bptr(y.value());
    ldy = y->stride(0);
  } else {
    TORCH_CHECK(p.has_value(), "skinny_gemm: slab output required");
    CHECK_DT(p.value(), at::kFloat);
    TORCH_CHECK(p->is_contiguous() && p->dim() == 3 && p->size(0) == splits && p->size(1) == M && p->size(2) == N,
                "skinny_gemm: slab shape must be [splits, M, N]");
    pp = p->data_ptr<float>();
  }
  CHECK_HIP(kafka_launch_skinny_gemm(bptr(x), x.stride(0), bptr(wt), M, N, K, (int)splits, glu ? 1 : 0, yp, ldy, pp,
                                     cur_stream()));
}

// explicit-configuration variant (microbenchmark sweeps): (mt, kc, splits) as given, no planning
static void wstream_gemm_cfg(at::Tensor x, at::Tensor wt, c10::optional<at::Tensor> y, c10::optional<at::Tensor> p,
                             int64_t mt, int64_t kc, int64_t s, bool nt, int64_t kw, int64_t pin) {
  CHECK_CUDA(x); CHECK_DT(x, at::kBFloat16); CHECK_DT(wt, at::kBFloat16); CHECK_LASTDIM(x);
  TORCH_CHECK(x.dim() == 2 && x.stride(0) % 8 == 0 && wt.dim() == 4 && wt.is_contiguous(), "wstream_gemm_cfg: x/wt");
  const int M = x.size(0), K = x.size(1), N = wt.size(0) * 32;
  // (M beyond 32 * mt runs as row tiles of 32 * mt rows, as the planned path does above 128 rows)
  TORCH_CHECK(wt.size(1) * 16 == K && M >= 1 && M <= 256 && K % (kc * s) == 0, "wstream_gemm_cfg: shape/config");
  if (s == 1) {
    TORCH_CHECK(y.has_value() && y->dim() == 2 && y->size(0) == M && y->size(1) == N, "wstream_gemm_cfg: y");
    CHECK_DT(y.value(), at::kBFloat16); CHECK_LASTDIM(y.value());
  } else {
    TORCH_CHECK(p.has_value() && p->is_contiguous() && p->numel() == s * M * N, "wstream_gemm_cfg: p");
    CHECK_DT(p.value(), at::kFloat);
  }
  CHECK_HIP(kafka_launch_wstream_gemm(bptr(x), x.stride(0), bptr(wt), M, N, K, (int)mt, (int)kc, (int)s, nt ? 1 : 0,
                                      (int)kw, (int)pin, 0,
                                      s == 1 ? bptr(y.value()) : nullptr, s == 1 ? y->stride(0) : 0,
                                      s == 1 ? nullptr : p->data_ptr<float>(), cur_stream()));
}

// Expert MLP halves on wave-tiled expert weights wt [E_local, N/32, K/16, 64, 8] (ops.tile_experts). glu: gate_up
// with fused SwiGLU into y [n_ent, N/2]; else down with the weighted combine into out f32 [T, N]. max_rows = T
// bounds every expert segment (a token picks an expert at most once).
static void wstream_grouped(at::Tensor x, at::Tensor wt, at::Tensor perm_tok, at::Tensor perm_w, at::Tensor expert_off,
                            int64_t e_lo, int64_t max_rows, bool gather, c10::optional<at::Tensor> y,
                            c10::optional<at::Tensor> out, bool pin) {
  CHECK_CUDA(x); CHECK_DT(x, at::kBFloat16); CHECK_DT(wt, at::kBFloat16); CHECK_LASTDIM(x);
  CHECK_DT(perm_tok, at::kInt); CHECK_DT(perm_w, at::kFloat); CHECK_DT(expert_off, at::kInt);
  TORCH_CHECK(x.dim() == 2 && x.stride(0) % 8 == 0, "wstream_grouped: x must be [rows, K] with 16-B rows");
  TORCH_CHECK(wt.dim() == 5 && wt.is_contiguous() && wt.size(3) == 64 && wt.size(4) == 8,
              "wstream_grouped: wt must be contiguous [E_local, N/32, K/16, 64, 8]");
  const int E_local = wt.size(0), N = wt.size(1) * 32, K = wt.size(2) * 16;
  TORCH_CHECK(x.size(1) == K && K % 256 == 0 && N % 64 == 0, "wstream_grouped: K / N");
  const int64_t n_ent = perm_tok.numel();
  TORCH_CHECK(perm_w.numel() == n_ent && perm_tok.is_contiguous() && perm_w.is_contiguous(), "wstream_grouped: perm");
  TORCH_CHECK(expert_off.is_contiguous() && e_lo >= 0 && expert_off.numel() >= e_lo + E_local + 1,
              "wstream_grouped: expert_off too short for the local experts");
  TORCH_CHECK(max_rows >= 1 && (gather ? x.size(0) == max_rows : x.size(0) >= n_ent),
              "wstream_grouped: x rows (tokens when gathering, entries otherwise)");
  bf16* yp = nullptr;
  int64_t ldy = 0;
  float* op = nullptr;
  int64_t ldo = 0;
  if (y.has_value()) {
    CHECK_DT(y.value(), at::kBFloat16); CHECK_LASTDIM(y.value());
    TORCH_CHECK(!out.has_value() && y->dim() == 2 && y->size(0) >= n_ent && y->size(1) == N / 2,
                "wstream_grouped: y must be [n_ent, N/2]");
    yp = bptr(y.value());
    ldy = y->stride(0);
  } else {
    TORCH_CHECK(out.has_value(), "wstream_grouped: y or out required");
    CHECK_DT(out.value(), at::kFloat); CHECK_LASTDIM(out.value());
    TORCH_CHECK(out->dim() == 2 && out->size(0) == max_rows && out->size(1) == N, "wstream_grouped: out [T, N]");
    op = out->data_ptr<float>();
    ldo = out->stride(0);
  }
  CHECK_HIP(kafka_launch_wstream_grouped(bptr(x), x.stride(0), bptr(wt), E_local, N, K, perm_tok.data_ptr<int>(),
                                         perm_w.data_ptr<float>(), expert_off.data_ptr<int>(), (int)e_lo,
                                         (int)max_rows, gather ? 1 : 0, yp, ldy, op, ldo, pin ? 1 : 0,
                                         cur_stream()));
}

// y [M, N] bf16 = sum over the slabs p [S, M, N]
static void slab_reduce(at::Tensor p, at::Tensor y) {
  CHECK_CUDA(p); CHECK_DT(p, at::kFloat); CHECK_DT(y, at::kBFloat16); CHECK_LASTDIM(y);
  check_slab(p);
  TORCH_CHECK(y.dim() == 2 && y.size(0) == p.size(1) && y.size(1) == p.size(2) && y.stride(0) % 8 == 0,
              "slab_reduce: y must be [M, N]");
  CHECK_HIP(kafka_launch_slab_reduce(p.data_ptr<float>(), p.size(0), p.size(1), p.size(2), bptr(y), y.stride(0),
                                     cur_stream()));
}

// softmax -> top-k -> renormalise + stable expert sort (one kernel, no host sync)
static void moe_route(at::Tensor logits, int64_t k, int64_t bm, at::Tensor topk_w, at::Tensor topk_e,
                      at::Tensor perm_tok, at::Tensor perm_w, at::Tensor expert_off, at::Tensor tile_off) {
  CHECK_CUDA(logits); CHECK_DT(logits, at::kBFloat16); CHECK_LASTDIM(logits);
  CHECK_DT(topk_w, at::kFloat); CHECK_DT(perm_w, at::kFloat);
  CHECK_DT(topk_e, at::kInt); CHECK_DT(perm_tok, at::kInt); CHECK_DT(expert_off, at::kInt); CHECK_DT(tile_off, at::kInt);
  const int T = logits.size(0), E = logits.size(1);
  TORCH_CHECK(T >= 1 && E <= 16 && k >= 1 && k <= 4 && k <= E, "moe_route: unsupported T/E/k");
  TORCH_CHECK(topk_w.numel() == (int64_t)T * k && topk_e.numel() == (int64_t)T * k &&
                  perm_tok.numel() == (int64_t)T * k && perm_w.numel() == (int64_t)T * k &&
                  expert_off.numel() == E + 1 && tile_off.numel() == E + 1,
              "moe_route: output sizes");
  TORCH_CHECK(topk_w.is_contiguous() && topk_e.is_contiguous() && perm_tok.is_contiguous() && perm_w.is_contiguous(),
              "moe_route: contiguous outputs");
  CHECK_HIP(kafka_launch_moe_route(bptr(logits), logits.stride(0), T, E, (int)k, (int)bm, topk_w.data_ptr<float>(),
                                   topk_e.data_ptr<int>(), perm_tok.data_ptr<int>(), perm_w.data_ptr<float>(),
                                   expert_off.data_ptr<int>(), tile_off.data_ptr<int>(), cur_stream()));
}

// Y (or out += w * Y) = X_e . W_e^T per expert segment of the routed entries; W = [e_n, N, K] local experts
static void grouped_gemm(at::Tensor x, at::Tensor w, at::Tensor perm_tok, at::Tensor perm_w, at::Tensor expert_off,
                         at::Tensor tile_off, int64_t e_lo, int64_t max_tiles, bool gather,
                         c10::optional<at::Tensor> y, c10::optional<at::Tensor> out) {
  CHECK_CUDA(x); CHECK_DT(x, at::kBFloat16); CHECK_DT(w, at::kBFloat16); CHECK_LASTDIM(x);
  TORCH_CHECK(w.dim() == 3 && w.is_contiguous(), "grouped_gemm: w must be contiguous [E_local, N, K]");
  const int e_n = w.size(0), N = w.size(1), Kd = w.size(2);
  const int E = expert_off.numel() - 1;
  TORCH_CHECK(x.size(1) == Kd && N % 128 == 0 && Kd % 64 == 0 && x.stride(0) % 8 == 0,
              "grouped_gemm: need N % 128 == 0, K % 64 == 0, 16-B rows");
  TORCH_CHECK(e_lo >= 0 && e_lo + e_n <= E, "grouped_gemm: expert range");
  const int64_t entries = perm_tok.numel();
  TORCH_CHECK(max_tiles >= (entries + 63) / 64 + E, "grouped_gemm: max_tiles below the routing bound");
  TORCH_CHECK(gather || x.size(0) >= entries, "grouped_gemm: direct mode needs one x row per routed entry");
  bf16* yp = nullptr;
  int64_t ldy = 0;
  float* op = nullptr;
  int64_t ldo = 0;
  if (out.has_value()) {
    CHECK_DT(out.value(), at::kFloat); CHECK_LASTDIM(out.value());
    TORCH_CHECK(out.value().size(1) == N, "grouped_gemm: out width");
    op = out.value().data_ptr<float>();
    ldo = out.value().stride(0);
  } else {
    TORCH_CHECK(y.has_value(), "grouped_gemm: y or out required");
    CHECK_DT(y.value(), at::kBFloat16); CHECK_LASTDIM(y.value());
    TORCH_CHECK(y.value().size(0) >= entries && y.value().size(1) == N && y.value().stride(0) % 8 == 0,
                "grouped_gemm: y shape");
    yp = bptr(y.value());
    ldy = y.value().stride(0);
  }
  CHECK_HIP(kafka_launch_grouped_gemm(bptr(x), x.stride(0), bptr(w), N, Kd, perm_tok.data_ptr<int>(),
                                      perm_w.data_ptr<float>(), expert_off.data_ptr<int>(), tile_off.data_ptr<int>(),
                                      (int)e_lo, e_n, (int)max_tiles, gather ? 1 : 0, yp, ldy, op, ldo,
                                      cur_stream()));
}

// ---- CU-masked streams (attention partition: the compute-bound cascade tile and the bandwidth-bound suffix decode
// run side by side on disjoint CU sets). Returns the raw hipStream_t for torch.cuda.ExternalStream; the stream
// lives for the process (one per partition, created once).
static int64_t cu_mask_stream(std::vector<int64_t> mask_words) {
  TORCH_CHECK(!mask_words.empty() && mask_words.size() <= 64, "cu_mask_stream: 1..64 mask words");
  std::vector<uint32_t> m(mask_words.size());
  for (size_t i = 0; i < m.size(); ++i) m[i] = (uint32_t)(mask_words[i] & 0xffffffffll);
  hipStream_t st = nullptr;
  CHECK_HIP(hipExtStreamCreateWithCUMask(&st, (uint32_t)m.size(), m.data()));
  return reinterpret_cast<int64_t>(st);
}
static std::vector<int64_t> stream_cu_mask(int64_t stream, int64_t words) {
  std::vector<uint32_t> m((size_t)words, 0u);
  CHECK_HIP(hipExtStreamGetCUMask(reinterpret_cast<hipStream_t>(stream), (uint32_t)words, m.data()));
  return std::vector<int64_t>(m.begin(), m.end());
}

// ---- custom one-shot all-reduce (csrc/allreduce.hip): raw device allocations + IPC handles
static int64_t car_alloc(int64_t bytes) {
  void* p = nullptr;
  CHECK_HIP(kafka_car_alloc(bytes, &p));
  return reinterpret_cast<int64_t>(p);
}
static py::bytes car_ipc_handle(int64_t ptr) {
  hipIpcMemHandle_t h;
  CHECK_HIP(kafka_car_ipc_handle(reinterpret_cast<void*>(ptr), &h));
  return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
}
static int64_t car_open(py::bytes handle) {
  std::string s = handle;
  TORCH_CHECK(s.size() == sizeof(hipIpcMemHandle_t), "car_open: bad handle size");
  hipIpcMemHandle_t h;
  memcpy(&h, s.data(), sizeof(h));
  void* p = nullptr;
  CHECK_HIP(kafka_car_open(&h, &p));
  return reinterpret_cast<int64_t>(p);
}
static void car_close(int64_t ptr) { CHECK_HIP(kafka_car_close(reinterpret_cast<void*>(ptr))); }
static void car_free(int64_t ptr) { CHECK_HIP(kafka_car_free(reinterpret_cast<void*>(ptr))); }
static int64_t car_error(int64_t own) {
  int v = 0;
  CHECK_HIP(hipMemcpy(&v, reinterpret_cast<char*>(own) + 8 * 128 * 4, sizeof(int), hipMemcpyDeviceToHost));
  return v;
}
// Stream-ordered copy of the error word into out[idx] (pinned int32 host tensor): the engine reads it with the
// step's sampled ids, so a peer that stopped arriving fails the replica instead of yielding wrong tokens.
static void car_error_async(int64_t own, at::Tensor out, int64_t idx) {
  TORCH_CHECK(out.is_pinned() && out.scalar_type() == at::kInt && idx >= 0 && idx < out.numel(),
              "car_error_async: pinned int32 host tensor");
  CHECK_HIP(hipMemcpyAsync(out.data_ptr<int>() + idx, reinterpret_cast<char*>(own) + 8 * 128 * 4, sizeof(int),
                           hipMemcpyDeviceToHost, cur_stream()));
}
// (timing ring [128, 2] of 100 MHz clock stamps, block 0's call counter): SURVEY §5.5 collective time in /metrics
static std::tuple<at::Tensor, int64_t> car_timing(int64_t own) {
  at::Tensor ring = at::empty({128, 2}, at::TensorOptions().dtype(at::kLong));
  int epoch = 0;
  CHECK_HIP(kafka_car_timing(reinterpret_cast<const void*>(own), reinterpret_cast<uint64_t*>(ring.data_ptr<int64_t>()),
                             &epoch));
  return {ring, (int64_t)epoch};
}
static std::vector<char*> car_bases(const std::vector<int64_t>& bases) {
  std::vector<char*> b(bases.size());
  for (size_t i = 0; i < bases.size(); ++i) b[i] = reinterpret_cast<char*>(bases[i]);
  return b;
}

// x: bf16 [.., n] (in place when y is omitted) or an fp32 split-K slab [S, T, n] (then y is required)
static void car_all_reduce(at::Tensor x, c10::optional<at::Tensor> y, std::vector<int64_t> bases, int64_t rank,
                           int64_t max_bytes, int64_t nblocks) {
  CHECK_CUDA(x);
  const bool slab = is_slab(x);
  if (slab) check_slab(x); else CHECK_DT(x, at::kBFloat16);
  TORCH_CHECK(x.is_contiguous(), "car_all_reduce: contiguous input");
  at::Tensor out = y.has_value() ? y.value() : x;
  TORCH_CHECK(!slab || y.has_value(), "car_all_reduce: a slab input needs a bf16 output");
  CHECK_DT(out, at::kBFloat16);
  const int64_t n = slab ? x.size(1) * x.size(2) : x.numel();
  TORCH_CHECK(out.is_contiguous() && out.numel() == n && n % 8 == 0, "car_all_reduce: output shape");
  TORCH_CHECK(n * 2 <= max_bytes, "car_all_reduce: message larger than the registered buffer");
  auto b = car_bases(bases);
  CHECK_HIP(kafka_launch_car_allreduce(b.data(), (int)b.size(), (int)rank, slab ? nullptr : bptr(x),
                                       slab ? x.data_ptr<float>() : nullptr, slab ? x.size(0) : 0,
                                       slab ? x.size(1) * x.size(2) : 0, bptr(out), n / 8, max_bytes, (int)nblocks,
                                       cur_stream()));
}

// residual <- allreduce(x) + residual; out = rmsnorm(residual) * w  (x: bf16 [T, d] or slab [S, T, d])
// pre (optional): bf16 [T, dpre] columns 0 .. dpre-1 of the row, already all-reduced; x then holds only the remaining
// d - dpre columns (the second half of an overlapped TP seam)
static void car_all_reduce_add_rmsnorm(at::Tensor x, at::Tensor residual, at::Tensor w, double eps, at::Tensor out,
                                       std::vector<int64_t> bases, int64_t rank, int64_t max_bytes,
                                       int64_t nblocks, c10::optional<at::Tensor> pre) {
  CHECK_CUDA(x); CHECK_DT(residual, at::kBFloat16); CHECK_DT(w, at::kBFloat16); CHECK_DT(out, at::kBFloat16);
  const bool slab = is_slab(x);
  if (slab) check_slab(x); else CHECK_DT(x, at::kBFloat16);
  TORCH_CHECK(x.is_contiguous() && (slab || x.dim() == 2), "car_all_reduce_add_rmsnorm: x [T, d] or slab");
  const int T = x.size(slab ? 1 : 0), dx = x.size(slab ? 2 : 1);
  int dpre = 0;
  int64_t pre_s = 0;
  const bf16* pp = nullptr;
  if (pre.has_value()) {
    CHECK_CUDA(*pre); CHECK_DT(*pre, at::kBFloat16);
    TORCH_CHECK(pre->dim() == 2 && pre->size(0) == T && pre->stride(1) == 1 && pre->size(1) % 8 == 0 &&
                    pre->stride(0) % 8 == 0, "car_all_reduce_add_rmsnorm: pre [T, dpre] bf16");
    dpre = pre->size(1);
    pre_s = pre->stride(0);
    pp = bptr(*pre);
  }
  const int d = dpre + dx;
  TORCH_CHECK(residual.dim() == 2 && residual.size(0) == T && residual.size(1) == d && residual.stride(1) == 1 &&
                  out.dim() == 2 && out.size(0) == T && out.size(1) == d && out.stride(1) == 1 &&
                  w.is_contiguous() && w.numel() == d && d % 8 == 0 && dx % 8 == 0 && d <= 16384,
              "car_all_reduce_add_rmsnorm: shapes");
  TORCH_CHECK((int64_t)T * dx * 2 <= max_bytes, "car_all_reduce_add_rmsnorm: message larger than the buffer");
  auto b = car_bases(bases);
  CHECK_HIP(kafka_launch_car_allreduce_add_rmsnorm(
      b.data(), (int)b.size(), (int)rank, slab ? nullptr : bptr(x), slab ? x.data_ptr<float>() : nullptr,
      slab ? x.size(0) : 0, slab ? (int64_t)T * dx : 0, T, d, bptr(residual), residual.stride(0), bptr(w),
      (float)eps, bptr(out), out.stride(0), max_bytes, (int)nblocks, pp, pre_s, dpre, cur_stream()));
}

// Expert-parallel all-to-all (bcast = false: part q of `send` [nranks * bpd bytes] goes to rank q) or all-gather
// (bcast = true: `send` is one part) over the IPC-mapped buffers; recv = nranks parts of bpd bytes.
static void car_a2a(at::Tensor send, at::Tensor recv, int64_t bpd, bool bcast, std::vector<int64_t> bases,
                    int64_t rank, int64_t max_bytes, int64_t nblocks) {
  CHECK_CUDA(send); CHECK_CUDA(recv);
  TORCH_CHECK(send.is_contiguous() && recv.is_contiguous(), "car_a2a: contiguous buffers");
  const int64_t nbytes = send.numel() * send.element_size();
  const int64_t nr = (int64_t)bases.size();
  TORCH_CHECK(recv.numel() * recv.element_size() == nr * bpd, "car_a2a: recv must hold nranks parts");
  TORCH_CHECK(nbytes == (bcast ? bpd : nr * bpd) && bpd % 16 == 0 && nbytes <= max_bytes,
              "car_a2a: image size / part size / buffer capacity");
  auto b = car_bases(bases);
  CHECK_HIP(kafka_launch_car_a2a(b.data(), (int)nr, (int)rank, send.data_ptr(), nbytes, recv.data_ptr(), bpd,
                                 bcast ? 1 : 0, max_bytes, (int)nblocks, cur_stream()));
}

// EP send image [ep, C + MR, d] bf16 of the owned (token, expert) pairs [lo * k, (lo + n_own) * k) + slot map
static void ep_dispatch(at::Tensor x, at::Tensor topk_e, int64_t lo, int64_t n_own, int64_t El, int64_t C,
                        at::Tensor img, at::Tensor slot_map) {
  CHECK_CUDA(x); CHECK_DT(x, at::kBFloat16); CHECK_LASTDIM(x); CHECK_DT(topk_e, at::kInt); CHECK_DT(img, at::kBFloat16);
  CHECK_DT(slot_map, at::kInt);
  TORCH_CHECK(topk_e.dim() == 2 && topk_e.is_contiguous() && img.dim() == 3 && img.is_contiguous(),
              "ep_dispatch: topk_e [T, k], img [ep, C + MR, d]");
  const int k = topk_e.size(1), ep = img.size(0), d = img.size(2);
  TORCH_CHECK(x.size(1) == d && x.stride(0) % 8 == 0 && lo >= 0 && lo + n_own <= topk_e.size(0) &&
                  lo + n_own <= x.size(0) && slot_map.numel() >= n_own * k,
              "ep_dispatch: shapes");
  const int MR = img.size(1) - (int)C;  // metadata rows after the C row slots of each destination block
  TORCH_CHECK(C >= 1 && MR >= 1 && 16 + 4 * C <= (int64_t)MR * d * 2 && El >= 1 && (int64_t)ep * El >= 1,
              "ep_dispatch: metadata rows");
  CHECK_HIP(kafka_launch_ep_dispatch(bptr(x), x.stride(0), topk_e.data_ptr<int>(), (int)lo, (int)(n_own * k), k,
                                     (int)El, ep, (int)C, MR, d, bptr(img), slot_map.data_ptr<int>(), cur_stream()));
}

static void ep_recv_route(at::Tensor img, int64_t C, int64_t El, int64_t bm, at::Tensor perm_tok, at::Tensor perm_w,
                          at::Tensor expert_off, at::Tensor tile_off) {
  CHECK_CUDA(img); CHECK_DT(img, at::kBFloat16); CHECK_DT(perm_tok, at::kInt); CHECK_DT(perm_w, at::kFloat);
  CHECK_DT(expert_off, at::kInt); CHECK_DT(tile_off, at::kInt);
  TORCH_CHECK(img.dim() == 3 && img.is_contiguous(), "ep_recv_route: img [ep, C + MR, d]");
  const int ep = img.size(0), d = img.size(2), MR = img.size(1) - (int)C;
  TORCH_CHECK(MR >= 1 && perm_tok.numel() == ep * C && perm_w.numel() == ep * C && expert_off.numel() == El + 1 &&
                  tile_off.numel() == El + 1 && El <= 16,
              "ep_recv_route: sizes");
  CHECK_HIP(kafka_launch_ep_recv_route(bptr(img), ep, (int)C, MR, d, (int)El, (int)bm, perm_tok.data_ptr<int>(),
                                       perm_w.data_ptr<float>(), expert_off.data_ptr<int>(), tile_off.data_ptr<int>(),
                                       cur_stream()));
}

// out[i] = sum_j topk_w[lo + i, j] * back[slot_map[i k + j]]   (back: [rows, d] bf16)
static void ep_combine(at::Tensor back, at::Tensor slot_map, at::Tensor topk_w, int64_t lo, int64_t n_own,
                       at::Tensor out) {
  CHECK_CUDA(back); CHECK_DT(back, at::kBFloat16); CHECK_DT(slot_map, at::kInt); CHECK_DT(topk_w, at::kFloat);
  CHECK_DT(out, at::kBFloat16); CHECK_LASTDIM(out);
  TORCH_CHECK(back.is_contiguous() && topk_w.dim() == 2 && topk_w.is_contiguous(), "ep_combine: layouts");
  const int k = topk_w.size(1), d = back.size(-1);
  TORCH_CHECK(out.size(1) == d && out.size(0) >= n_own && out.stride(0) % 8 == 0 && slot_map.numel() >= n_own * k &&
                  lo + n_own <= topk_w.size(0),
              "ep_combine: shapes");
  CHECK_HIP(kafka_launch_ep_combine(bptr(back), slot_map.data_ptr<int>(), topk_w.data_ptr<float>(), (int)lo,
                                    (int)n_own, k, d, bptr(out), out.stride(0), cur_stream()));
}

PYBIND11_MODULE(_kafka_ops, m) {
  m.doc() = "kafka_llm_service_amd CDNA4 (gfx950) HIP kernels";
  m.def("rmsnorm", &rmsnorm);
  m.def("fused_add_rmsnorm", &fused_add_rmsnorm);
  m.def("silu_mul", &silu_mul);
  m.def("rope_kv_write", &rope_kv_write);
  m.def("attn_decode", &attn_decode, py::arg("q"), py::arg("k_cache"), py::arg("v_cache"), py::arg("block_tables"),
        py::arg("items"), py::arg("out_part"), py::arg("lse_part"), py::arg("scale"), py::arg("out"),
        py::arg("tickets"), py::arg("pre_part") = py::none(), py::arg("m_part") = py::none(),
        py::arg("m_lse") = py::none(), py::arg("m_out") = py::none());
  m.def("attn_prefill", &attn_prefill, py::arg("items"), py::arg("q"), py::arg("k_cache"), py::arg("v_cache"),
        py::arg("block_tables"), py::arg("q_limit"), py::arg("out"), py::arg("out_part"), py::arg("lse_part"),
        py::arg("scale"), py::arg("variant") = 0, py::arg("alt_part") = py::none(), py::arg("alt_lse") = py::none(),
        py::arg("alt_tok_off") = 0);
  m.def("attn_merge", &attn_merge, py::arg("part"), py::arg("lse"), py::arg("out"), py::arg("lse_out") = py::none(),
        py::arg("pre") = py::none(), py::arg("npre") = 0);
  m.def("sample", &sample, py::arg("logits"), py::arg("temperature"), py::arg("top_p"), py::arg("top_k"),
        py::arg("seeds"), py::arg("step"), py::arg("out"), py::arg("ws") = py::none(), py::arg("nsplit") = 1,
        py::arg("proc") = py::none(), py::arg("mask_tab") = py::none(), py::arg("counts") = py::none());
  m.def("wstream_plan", &wstream_plan);
  m.def("wstream_gemm", &wstream_gemm, py::arg("x"), py::arg("wt"), py::arg("y"), py::arg("p"),
        py::arg("max_splits"), py::arg("nt"), py::arg("glu"));
  m.def("wstream_fin", &wstream_fin, py::arg("fin"), py::arg("x"), py::arg("wt"), py::arg("y"), py::arg("p"),
        py::arg("tickets"), py::arg("ss_in"), py::arg("eps"), py::arg("resid"), py::arg("nw"), py::arg("xn"),
        py::arg("ss_out"), py::arg("positions"), py::arg("cos_sin"), py::arg("q_out"), py::arg("k_cache"),
        py::arg("v_cache"), py::arg("slots"), py::arg("Hq"), py::arg("Hkv"), py::arg("max_splits"),
        py::arg("stamps") = py::none());
  m.def("skinny_plan", &skinny_plan);
  m.def("skinny_gemm", &skinny_gemm);
  m.def("wstream_gemm_cfg", &wstream_gemm_cfg);
  m.def("slab_reduce", &slab_reduce);
  m.def("wstream_grouped", &wstream_grouped, py::arg("x"), py::arg("wt"), py::arg("perm_tok"), py::arg("perm_w"),
        py::arg("expert_off"), py::arg("e_lo"), py::arg("max_rows"), py::arg("gather"), py::arg("y"), py::arg("out"),
        py::arg("pin") = true);
  m.def("moe_route", &moe_route);
  m.def("cu_mask_stream", &cu_mask_stream);
  m.def("stream_cu_mask", &stream_cu_mask);
  m.def("car_alloc", &car_alloc);
  m.def("car_ipc_handle", &car_ipc_handle);
  m.def("car_open", &car_open);
  m.def("car_close", &car_close);
  m.def("car_free", &car_free);
  m.def("car_error", &car_error);
  m.def("car_error_async", &car_error_async);
  m.def("car_timing", &car_timing);
  m.def("car_all_reduce", &car_all_reduce);
  m.def("car_all_reduce_add_rmsnorm", &car_all_reduce_add_rmsnorm, py::arg("x"), py::arg("residual"), py::arg("w"),
        py::arg("eps"), py::arg("out"), py::arg("bases"), py::arg("rank"), py::arg("max_bytes"), py::arg("nblocks"),
        py::arg("pre") = py::none());
  m.def("car_a2a", &car_a2a);
  m.def("ep_dispatch", &ep_dispatch);
  m.def("ep_recv_route", &ep_recv_route);
  m.def("ep_combine", &ep_combine);
  m.def("grouped_gemm", &grouped_gemm);
}
