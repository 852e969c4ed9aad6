/*
 * vit_hip.h — C ABI of the MI355X (gfx950) ViT training-step kernels.
 *
 * The reference (sea-with-sakura/ViT-of-Pytorch) has no native code and no FFI: every op
 * on its hot path is a PyTorch ATen call made from src/model.py / src/train.py. Each entry
 * point below replaces the ATen op(s) named in its comment (reference file:line), so the
 * drop-in Python surface (vitmi.model.VisionTransformer etc.) can run the training step on
 * hand-written CDNA4 kernels.
 *
 * Conventions
 *   - all pointers are device pointers; sizes/strides are element counts (int64_t);
 *   - bf16 tensors are passed as `void*` / `const void*` holding IEEE bfloat16 bit patterns;
 *   - `stream` is a hipStream_t passed as an opaque pointer (NULL = default stream);
 *   - the library never allocates or frees device memory: callers own every buffer,
 *     including workspaces; no call synchronises the host;
 *   - every entry point returns VIT_OK (0) or an error code; vit_last_error() returns a
 *     thread-local description of the last failure on the calling thread;
 *   - calls are reentrant and keep no global mutable device state.
 */
#ifndef VIT_HIP_H_
#define VIT_HIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* vit_stream_t;

enum vit_status {
  VIT_OK = 0,
  VIT_ERR_INVALID_ARG = 1,
  VIT_ERR_HIP = 2,
  VIT_ERR_UNSUPPORTED = 3,
};

const char* vit_last_error(void);
int vit_abi_version(void);
/* Source fingerprint the library was built from (16 hex digits, vit-of-pytorch_amd/vitmi/buildid.py over
 * Makefile, csrc/ and this header); the Python binding refuses a library whose id differs from its tree. */
const char* vit_build_id(void);

/* ------------------------------------------------------------------------------------------
 * bf16 MFMA GEMM with fused epilogues.
 *   C[m, n] = sum_k A(m, k) * B(k, n)
 * A(m,k) is A[m*lda + k] when a_layout == VIT_K_CONTIG, A[k*lda + m] when VIT_MN_CONTIG.
 * B(k,n) is B[n*ldb + k] when b_layout == VIT_K_CONTIG, B[k*ldb + n] when VIT_MN_CONTIG.
 * K must be a multiple of 64 (callers zero-pad). M, N are arbitrary.
 * gridDim.z batching: every pointer advances by its *_batch_stride per batch index.
 *
 * Replaces (reference): LinearGeneral.forward tensordot+bias   src/model.py:61-63,86-88,99
 *                       MlpBlock fc1 -> GELU, fc2                src/model.py:43-48
 *                       Conv2d patch embedding + cls + pos-emb  src/model.py:179,197-204, :16-17
 *                       and the autograd dgrad/wgrad of all of them (src/train.py:23)
 * ---------------------------------------------------------------------------------------- */
enum vit_layout { VIT_K_CONTIG = 0, VIT_MN_CONTIG = 1 };

/* Dropout descriptor. nn.Dropout(p) of PositionEmbs (src/model.py:19-20), EncoderBlock
 * (:124-125) and MlpBlock (:46-49) as a counter-based mask that forward and backward regenerate:
 * element (row, col) of dropout site `site` is kept iff the 16-bit half (col % 8) of
 * Philox4x32-10(counter = {col / 8, row, site, offset_lo}, key = {seed_lo, seed_hi ^ offset_hi})
 * is >= round(p * 65536); kept elements are scaled by 1 / (1 - p). A NULL descriptor or p == 0
 * disables it. Sites used by the engine: 0 = position embedding, 1 + 3i / 2 + 3i / 3 + 3i =
 * attention output / MLP dropout1 / MLP dropout2 of encoder layer i. */
typedef struct vit_dropout {
  float p;
  uint32_t site;
  uint64_t seed;
  uint64_t offset;
  int64_t row_stride; /* mask row of a call's row r = r * row_stride (0 is taken as 1); the final
                         LayerNorm backward runs on the cls rows only (row stride N tokens) */
} vit_dropout;

/* mult[r*ld + c] = dropout multiplier (0 or 1/(1-p)) of element (row0 + r, c), c < cols (tests) */
int vit_dropout_mask(const vit_dropout* d, int64_t row0, int64_t rows, int64_t cols, float* mult,
                     int64_t ld, vit_stream_t stream);

enum vit_epilogue {
  VIT_EPI_F32 = 0,            /* C(f32)  = acc                                                */
  VIT_EPI_BF16 = 1,           /* C(bf16) = acc                                                */
  VIT_EPI_BIAS_BF16 = 2,      /* C(bf16) = acc + bias[n]                                       */
  VIT_EPI_BIAS_GELU = 3,      /* u = acc + bias[n]; C(bf16) = u; C2(bf16) = gelu_erf(u)        */
  VIT_EPI_BIAS_RESID_F32 = 4, /* C(f32) = acc + bias[n] + aux_f32[m*ldaux + n] (C may == aux) */
  VIT_EPI_GELU_BWD = 5,       /* C(bf16) = acc * gelu_erf'(aux_bf16[m*ldaux + n])              */
  VIT_EPI_PATCH = 6,          /* C(f32) = (m % tokens == 0) ? aux2[n] + pos[0][n]
                                            : acc + bias[n] + pos[m % tokens][n],
                                 pos = aux_f32 with row stride ldaux                          */
  VIT_EPI_SPLITK = 7,         /* split-K partial: C(f32)[(z*split_k + s)*M*N + m*N + n] = acc  */
  VIT_EPI_BIAS_GELU_DGELU = 8,/* u = acc + bias[n]; C(bf16) = gelu_erf'(u); C2(bf16) = gelu_erf(u)
                                 (the backward then needs no transcendental: VIT_EPI_MUL_BF16)   */
  VIT_EPI_MUL_BF16 = 9,       /* C(bf16) = acc * aux_bf16[m*ldaux + n]                         */
};

typedef struct vit_gemm_args {
  int64_t M, N, K;
  const void* A;
  int64_t lda;
  int64_t a_batch_stride;
  int32_t a_layout;
  int32_t b_layout;
  const void* B;
  int64_t ldb;
  int64_t b_batch_stride;
  void* C;
  int64_t ldc;
  int64_t c_batch_stride;
  void* C2;
  int64_t ldc2;
  const float* bias;
  int64_t bias_batch_stride;
  const void* aux;
  int64_t ldaux;
  const float* aux2;
  int64_t batch;   /* >= 1 */
  int64_t split_k; /* >= 1; > 1 only with VIT_EPI_SPLITK */
  int64_t tokens;  /* VIT_EPI_PATCH: tokens per image */
  float* col_partial; /* optional (batch 1, split_k 1): col_partial[tile_m * N + n] = sum over the
                         tile's rows of the epilogue's output (bias-gradient partials); reduce the
                         vit_gemm_partial_rows() rows with vit_colsum */
  int32_t epilogue;
  int32_t tile;    /* 0 = auto */
  const vit_dropout* dropout; /* optional, on the epilogue's output (row m, col n):
                                 PATCH: C = drop(embedding + pos);  BIAS_RESID_F32: C = drop(acc + bias) + aux;
                                 BIAS_GELU_DGELU: C2 = drop(gelu(u)), C = gelu'(u) * mult (the dropout
                                 backward folded into the saved derivative) */
} vit_gemm_args;

int vit_gemm_bf16(const vit_gemm_args* args, vit_stream_t stream);
/* rows of C covered by one workgroup tile for these arguments */
int64_t vit_gemm_tile_rows(const vit_gemm_args* args);
/* rows of col_partial a call with these arguments writes (the rows to reduce with vit_colsum): one per
 * 256-row tile of the whole-wave part and one per 128-row tile of a wave-split remainder */
int64_t vit_gemm_partial_rows(const vit_gemm_args* args);
/* rows of the whole-wave part of a wave-split call (the 256 x 256 tiles that fill whole waves of the CUs; the
 * remaining rows run on 128 x 128 tiles), 0 when the call runs as one launch */
int64_t vit_gemm_split_rows(const vit_gemm_args* args);
/* one part of vit_gemm_bf16: part 1 = the whole-wave rows [0, split_rows) (the whole GEMM when it does not
 * split), part 2 = the remainder rows [split_rows, M) (nothing when it does not split). Parts 1 and 2 together
 * are exactly vit_gemm_bf16(args); they may run on different streams (the remainder beside a row-local op of
 * the whole-wave rows) */
int vit_gemm_bf16_part(const vit_gemm_args* args, int32_t part, vit_stream_t stream);
/* up to 4 split-K weight-gradient GEMMs in ONE launch (the concatenation of their grids): each member is a
 * vit_gemm_bf16 call with epilogue VIT_EPI_SPLITK and both operands M/N-contiguous, its own split_k / batch, and
 * writes exactly what that call writes (the same f32 slabs; every member on 256 x 256 tiles, M or N below 256 as
 * partial tiles). Fills the CUs where members alone leave a wave partly empty (the out-projection and q|k|v weight
 * gradients of one layer; the Res-ViT router's four weight gradients) */
int vit_gemm_splitk_group(const vit_gemm_args* args, int32_t n, vit_stream_t stream);

/* out[z*out_batch_stride + m*ldo + n] (+)= sum_s ws[((z*split + s)*M + m)*N + n]  (f32) */
int vit_splitk_reduce(const float* ws, int64_t batch, int64_t split, int64_t M, int64_t N,
                      float* out, int64_t ldo, int64_t out_batch_stride, int32_t accumulate,
                      vit_stream_t stream);
/* up to VIT_SPLITK_GROUP_MAX vit_splitk_reduce calls in ONE launch (each job's output bit-identical to its own call;
 * jobs outside the 16-B vector form fall back to one launch each) */
#define VIT_SPLITK_GROUP_MAX 8
typedef struct vit_splitk_job {
  const float* ws;
  int64_t batch, split, M, N;
  float* out;
  int64_t ldo, out_batch_stride;
  int32_t accumulate;
  int32_t reserved;
} vit_splitk_job;
int vit_splitk_reduce_group(const vit_splitk_job* jobs, int32_t njobs, vit_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * LayerNorm over the last dim (eps, biased variance, affine).  nn.LayerNorm src/model.py:108,114,146
 * fwd: y = (x - mean) * rstd * gamma + beta; saves mean/rstd (f32). y is bf16 or f32 (y_f32).
 * bwd: dx = rstd*(g - mean(g) - xhat*mean(g*xhat)), g = dy*gamma; dx_out = dres + dx (dres may
 *      be NULL); optional bf16 copy of dx_out. Per-block partial sums [nblk][3*D] of
 *      (dy*xhat, dy, dx_out) go to `partial` (>= vit_layernorm_bwd_partial_rows(rows) rows of 3*D);
 *      when non-NULL, dgamma_dbeta[0:D] = dgamma, [D:2D] = dbeta, and dx_colsum[0:D] = column sums of
 *      dx_out (= the bias gradient of the linear layer feeding this residual stream). With both NULL
 *      only the partials are written: nblk = vit_layernorm_bwd_blocks(rows) rows, which a caller can
 *      reduce later (vit_colsum3 over [nblk][3*D], e.g. on another stream).
 *      dx_dropout (optional): the bf16 copy and dx_colsum carry dx_out * mult (the gradient of the
 *      dropout-ed branch that fed the residual stream); dx itself stays unmasked.
 * ---------------------------------------------------------------------------------------- */
int vit_layernorm_fwd(const float* x, int64_t ldx, const float* gamma, const float* beta,
                      void* y, int64_t ldy, int32_t y_f32, float* mean, float* rstd,
                      int64_t rows, int64_t D, float eps, vit_stream_t stream);
int64_t vit_layernorm_bwd_partial_rows(int64_t rows);
int64_t vit_layernorm_bwd_blocks(int64_t rows);
int vit_layernorm_bwd(const void* dy, int64_t lddy, int32_t dy_f32, const float* x, int64_t ldx,
                      const float* mean, const float* rstd, const float* gamma,
                      const float* dres, int64_t lddres, float* dx, int64_t lddx,
                      void* dx_bf16, int64_t lddxb, float* partial, float* dgamma_dbeta,
                      float* dx_colsum, int32_t accumulate_params, int64_t rows, int64_t D,
                      const vit_dropout* dx_dropout, vit_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Fused multi-head self-attention, one (image, head) per workgroup, all keys in LDS.
 * qkv: bf16 [B*N, 3, H, hd] (q | k | v);  o: bf16 [B*N, H, hd];  lse: f32 [B, H, N]
 * S = (q k^T) * scale (scale = 1/sqrt(hd)), P = softmax(S), O = P v.
 * Replaces SelfAttention.forward src/model.py:90-97 (matmul, /scale, softmax, matmul, permutes)
 * bwd: dqkv (bf16 [B*N, 3, H, hd]) from dO, recomputing P from lse; when bias_partial != NULL
 *      it also receives per-image column sums of dq | dk | dv (f32 [B][3*H*hd], the q/k/v bias
 *      gradient partials; reduce over B with vit_colsum).
 * Two implementations (`path`): 1 = LDS-resident (all keys of a head on chip, exact softmax;
 * N <= 320: 197 tokens for B/16 and L/16 @224, 257 for H/14 @224), 2 = K/V-tiled (64-key blocks
 * streamed through LDS, online softmax; any N: 577 tokens @384 for B/16 and L/16, 730 for H/14,
 * src/config.py:12,37), 0 = pick by N, 3 = path 1 in its one-workgroup-per-(image, head) kernels only (no
 * persistent forward / backward: same-box A/B and parity checks; 1 bias row per image). hd: multiple of 16,
 * <= 96 (80-wide LDS images for ViT-H/14's hd 80).
 * ---------------------------------------------------------------------------------------- */
int vit_attention_fwd(const void* qkv, void* o, float* lse, int64_t B, int64_t N, int64_t H,
                      int64_t hd, float scale, vit_stream_t stream);
int vit_attention_bwd(const void* qkv, const void* o, const void* dout, const float* lse, void* dqkv,
                      float* bias_partial, int64_t B, int64_t N, int64_t H, int64_t hd, float scale,
                      vit_stream_t stream);
/* as vit_attention_fwd / _bwd for queries [0, q_rows) only (1 <= q_rows <= N; rounded up to whole
 * 32-row pairs): the forward writes o / lse of those rows; the backward assumes dout is zero on every
 * other row (their dQ is written as 0, dK / dV / bias partials are exact). Used for the last encoder
 * layer, whose output reaches the classifier through the cls row only (src/model.py:210). */
int vit_attention_fwd_rows(const void* qkv, void* o, float* lse, int64_t B, int64_t N, int64_t H, int64_t hd,
                           float scale, int64_t q_rows, vit_stream_t stream);
int vit_attention_bwd_rows(const void* qkv, const void* o, const void* dout, const float* lse, void* dqkv,
                           float* bias_partial, int64_t B, int64_t N, int64_t H, int64_t hd, float scale,
                           int64_t q_rows, vit_stream_t stream);
/* Path-explicit forms. bias_partial of the backward holds vit_attention_bias_rows(N, hd, path) rows per
 * image ([B * rows][3*H*hd], reduce all B * rows rows with vit_colsum): on path 1 one per wave of the
 * persistent kernel (8; hd <= 64 and N <= 208 at hd 64) or 1 (the two-stage kernel), ceil(N / 64) on
 * path 2 (one per 64-row block). The tiled backward needs `workspace`, >= vit_attention_workspace_elems
 * floats (the exact per-query delta = sum_j P dP handed from its dQ kernel to its dK/dV kernel);
 * path 1 needs none (NULL). q_rows as for the *_rows forms (path 2 rounds it up to 64-row blocks). */
int64_t vit_attention_bias_rows(int64_t N, int64_t hd, int32_t path);
int64_t vit_attention_workspace_elems(int64_t B, int64_t N, int64_t H, int32_t path);
int vit_attention_fwd_ex(const void* qkv, void* o, float* lse, int64_t B, int64_t N, int64_t H, int64_t hd,
                         float scale, int64_t q_rows, int32_t path, vit_stream_t stream);
int vit_attention_bwd_ex(const void* qkv, const void* o, const void* dout, const float* lse, void* dqkv,
                         float* bias_partial, int64_t B, int64_t N, int64_t H, int64_t hd, float scale,
                         int64_t q_rows, int32_t path, float* workspace, vit_stream_t stream);

/* Ragged-query attention forward (Res-ViT inference, res-vit/model.py:494-529: per sample, queries =
 * its active tokens, keys / values = all its tokens). Sample b's queries are rows [cu_q[b], cu_q[b+1])
 * of q (bf16, row stride ldq, head h at columns h*hd), its keys rows [b*Nkv, (b+1)*Nkv) of k and v
 * (bf16, strides ldk / ldv); o (bf16, stride ldo) rows match q's. cu_q: device int32 [B + 1],
 * max_q >= every sample's query count. o = softmax((q k^T) / sqrt(hd)) v (scale = 1/sqrt(hd)).
 * K/V-tiled online softmax, any Nkv; one launch for the whole batch. Forward only. */
int vit_attention_fwd_varlen(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                             void* o, int64_t ldo, const int32_t* cu_q, int64_t B, int64_t max_q, int64_t Nkv,
                             int64_t H, int64_t hd, float scale, vit_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Patch embedding im2col (Conv2d k=s=P as a GEMM, src/model.py:179,197-200):
 * x f32 NCHW [B,3,img,img] -> out bf16 [B*N, Kpad], N = (img/P)^2 + 1, row b*N (cls) is 0,
 * row b*N+1+(py*g+px), col c*P*P + ky*P + kx; cols >= 3P^2 are 0.
 * ---------------------------------------------------------------------------------------- */
int vit_im2col(const float* x, void* out, int64_t B, int64_t img, int64_t P, int64_t Kpad,
               vit_stream_t stream);

/* ----------------------------------------------------------------------------------------
 * Training-input transform (src/data_loaders.py:66-80 CIFAR train, :100-112 ImageNet):
 * torchvision Resize -> RandomHorizontalFlip -> ToTensor -> Normalize on the device.
 * images uint8 HWC [B][H][W][3] (image b at images + b*image_stride bytes) -> out f32 NCHW
 * [B,3,out_h,out_w] = (resized[c][y][flip ? out_w-1-x : x] / 255 - mean[c]) / std[c], with
 * resized = Pillow Image.resize((out_w, out_h), BILINEAR) bit-exactly (8-bit fixed point,
 * horizontal pass then vertical). flips: uint8 [B] (NULL = no flips). mean_std: host float[6] =
 * {mean0..2, std0..2}. Replaces the reference's CPU DataLoader transform; the caller sizes
 * out_h/out_w (torchvision's int-size rule lives in vitmi.data).
 * ---------------------------------------------------------------------------------------- */
int vit_preprocess_u8(const uint8_t* images, int64_t B, int64_t H, int64_t W, int64_t image_stride,
                      const uint8_t* flips, int64_t out_h, int64_t out_w, const float* mean_std, float* out,
                      vit_stream_t stream);

/* token-level grads of the embedding (src/model.py:17,203-204): from dh0 f32 [B*N, D]:
 * dpos[n][d] = sum_b dh0[b*N+n][d]; dcls = dpos[0]; dconv_bias = sum_{n>=1} dpos[n].
 * dropout (optional): dh0 is taken through the position-embedding dropout's multipliers first. */
int vit_embed_grad(const float* dh0, int64_t B, int64_t N, int64_t D, float* dpos, float* dcls,
                   float* dconv_bias, const vit_dropout* dropout, vit_stream_t stream);

/* column sums: out[n] (+)= sum_r in[r*ld + n], in bf16 (in_bf16=1) or f32. `partial` needs
 * vit_colsum_partial_rows(rows) * cols floats. (bias grads, src/train.py:23 autograd) */
int64_t vit_colsum_partial_rows(int64_t rows);
int vit_colsum(const void* in, int32_t in_bf16, int64_t rows, int64_t cols, int64_t ld,
               float* partial, float* out, int32_t accumulate, vit_stream_t stream);
/* the same over 3*seg columns, segment k (columns [k*seg, (k+1)*seg)) written to out_k (NULL = dropped):
 * q|k|v bias gradients, LayerNorm [dgamma | dbeta | dx column sum] in one reduction. Needs seg % 8 == 0. */
int vit_colsum3(const void* in, int32_t in_bf16, int64_t rows, int64_t seg, int64_t ld, float* partial,
                float* out0, float* out1, float* out2, int32_t accumulate, vit_stream_t stream);

/* Up to VIT_COLSUM_BATCH_MAX f32 column reductions in ONE launch, no workspace: for each job,
 * column c in [0, cols) of in[r*ld + c] summed over r in [0, rows) (a fixed order: deterministic) goes to
 * out_k[c - k*seg], k = c / seg (seg = 0: out0[c]); NULL outputs are dropped; accumulate adds to them.
 * Rows of 16-B multiples (cols % 4 == 0, ld % 4 == 0, `in` 16-B aligned) take vector loads. The engine's backward issues every bias-gradient
 * reduction of one encoder layer (LayerNorm dgamma | dbeta | dx column sums, fc1 bias from the fc2-dgrad
 * epilogue's tile partials, q|k|v biases from the attention backward's per-image partials) as one batch
 * on the compute stream. (bias grads of src/model.py:61-63,108,114 under src/train.py:23 autograd) */
#define VIT_COLSUM_BATCH_MAX 8
typedef struct vit_colsum_job {
  const float* in;
  int64_t rows, cols, ld, seg;
  float* out0;
  float* out1;
  float* out2;
  int32_t accumulate;
  int32_t reserved;
} vit_colsum_job;
int vit_colsum_batch(const vit_colsum_job* jobs, int32_t njobs, vit_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Classifier head helpers (tiny, f32): C = op(A) op(B) (+ bias) (+ C if accumulate).
 * a_trans: A(m,k) = A[k*lda+m]; b_trans: B(k,n) = B[n*ldb+k].  nn.Linear src/model.py:194,210
 * ---------------------------------------------------------------------------------------- */
int vit_gemm_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, int32_t a_trans,
                 const float* B, int64_t ldb, int32_t b_trans, float* C, int64_t ldc,
                 const float* bias, int32_t accumulate, vit_stream_t stream);

/* Cross entropy (mean over the global batch), CrossEntropyLoss src/train.py:151,22, plus
 * accuracy counts (src/utils.py:28-41). dlogits = (softmax - onehot) * grad_scale.
 * row_stats[b] = {loss_b, top1_hit, top5_hit}. A label outside [0, C) is not read through: that row's
 * loss and dlogits are NaN. */
int vit_cross_entropy(const float* logits, const int64_t* labels, int64_t B, int64_t C,
                      float* dlogits, float grad_scale, float* row_stats, vit_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Optimizer / parameter mirrors.  torch.optim.SGD step, src/train.py:24,154-158:
 *   d = g + wd*p; buf = first ? d : momentum*buf + d; p -= lr*buf; p_bf16 = bf16(p) (if != NULL)
 * ---------------------------------------------------------------------------------------- */
int vit_sgd_step(float* p, const float* g, float* buf, void* p_bf16, int64_t n, float lr,
                 float momentum, float weight_decay, int32_t first, vit_stream_t stream);
/* vit_sgd_step with hyper = {lr, momentum, first} read from device memory (a step inside a captured HIP
 * graph; the schedule writes the three floats before each replay) */
int vit_sgd_step_dev(float* p, const float* g, float* buf, void* p_bf16, int64_t n, const float* hyper,
                     float weight_decay, vit_stream_t stream);
int vit_cast_f32_bf16(const float* in, void* out, int64_t n, vit_stream_t stream);
/* out bf16 [rows][ldo] <- in f32 [rows][cols]; columns cols..ldo-1 are zeroed. */
int vit_cast_pad_rows(const float* in, int64_t rows, int64_t cols, void* out, int64_t ldo,
                      vit_stream_t stream);
/* up to VIT_CAST_BATCH_MAX casts in ONE launch: out[r*ldo + c] (bf16) = in[r*ldi + c] for r < rows, c < cols, zero for
 * the rest of [rows_pad][cols_pad] (small weight / operand casts of the Res-ViT nodes, one launch per node) */
#define VIT_CAST_BATCH_MAX 8
typedef struct vit_cast_job {
  const float* in;
  int64_t rows, cols, ldi;
  void* out;
  int64_t ldo, rows_pad, cols_pad;
} vit_cast_job;
int vit_cast_pad_batch(const vit_cast_job* jobs, int32_t njobs, vit_stream_t stream);
/* out[r*ldo + z*cols + c] = in[z*zstride + r*ldi + c]  (z < Z), as bf16 (out_bf16) or f32.
 * Packs q/k/v LinearGeneral weights [D][H,hd] (src/model.py:73-75) into one [D][3D] operand. */
int vit_pack_cols(const float* in, int64_t zstride, int64_t ldi, int64_t rows, int64_t cols, int64_t Z,
                  void* out, int64_t ldo, int32_t out_bf16, vit_stream_t stream);
/* vit_pack_cols over `batch` matrix sets (one per encoder layer): set z reads in + z*in_batch_stride
 * (floats, may be negative) and writes out + z*out_batch_stride (elements). One launch for all layers. */
int vit_pack_cols_batched(const float* in, int64_t in_batch_stride, int64_t zstride, int64_t ldi, int64_t rows,
                          int64_t cols, int64_t Z, void* out, int64_t out_batch_stride, int64_t ldo,
                          int32_t out_bf16, int64_t batch, vit_stream_t stream);
/* out bf16 [cols][ldo] <- transpose of in f32 [rows][ldi]: out[c*ldo + r] = bf16(in[r*ldi + c]), for
 * batch matrices z at in + z*in_batch_stride, out + z*out_batch_stride (strides may be negative).
 * K-contiguous weight copies for the dgrad / projection GEMMs (fc1/fc2 weights src/model.py:31-32,
 * LinearGeneral q/k/v/out src/model.py:73-76). */
int vit_transpose_f32_bf16(const float* in, int64_t rows, int64_t cols, int64_t ldi, void* out, int64_t ldo,
                           int64_t batch, int64_t in_batch_stride, int64_t out_batch_stride, vit_stream_t stream);
/* y = a*x + b*y (f32), used for gradient scaling / accumulation. */
int vit_axpby(const float* x, float* y, int64_t n, float a, float b, vit_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * fp32 ("exact") forward: the reference's arithmetic (f32 operands, f32 accumulation) for the
 * logits-parity gate and fp32 evaluation. Projections use vit_gemm_f32; LayerNorm
 * vit_layernorm_fwd with y_f32 = 1.
 * ---------------------------------------------------------------------------------------- */
/* out f32 [B*N, Kpad]: as vit_im2col (src/model.py:179,197-200) without the bf16 rounding */
int vit_im2col_f32(const float* x, float* out, int64_t B, int64_t img, int64_t P, int64_t Kpad,
                   vit_stream_t stream);
/* h[b*N+t] = (t == 0 ? cls : h[b*N+t]) + pos[t]   (src/model.py:203-204, :16-17) */
int vit_embed_fwd_f32(float* h, int64_t B, int64_t N, int64_t D, const float* pos, const float* cls,
                      vit_stream_t stream);
/* out = 0.5 u (1 + erf(u / sqrt 2))   nn.GELU() src/model.py:33 */
int vit_gelu_f32(const float* in, float* out, int64_t n, vit_stream_t stream);
/* o = softmax((q k^T) * inv_sqrt_hd) v per (image, head), f32: qkv [B*N, 3, H, hd], o [B*N, H, hd]
 * (SelfAttention.forward src/model.py:90-97) */
int vit_attention_fwd_f32(const float* qkv, float* o, int64_t B, int64_t N, int64_t H, int64_t hd,
                          float inv_sqrt_hd, vit_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Standalone sub-module path (vitmi.model Encoder / EncoderBlock / SelfAttention / MlpBlock /
 * LinearGeneral / PositionEmbs .forward on their own, composed from the kernels above plus these):
 * ---------------------------------------------------------------------------------------- */
/* dx = dy * GELU'(u), exact erf (autograd of nn.GELU, src/model.py:33,44) */
int vit_gelu_bwd_f32(const float* u, const float* dy, float* dx, int64_t n, vit_stream_t stream);
/* out[r*cols + c] = in[r*cols + c] * multiplier(r, c) of dropout descriptor d (in == out allowed);
 * forward and backward of nn.Dropout (src/model.py:19-20,46-51,124-125) regenerate the same mask */
int vit_dropout_apply_f32(const vit_dropout* d, const float* in, float* out, int64_t rows, int64_t cols,
                          vit_stream_t stream);
/* out[o*inner + i] = x[o*inner + i] + y[i]  (PositionEmbs: x + pos_embedding, src/model.py:17) */
int vit_add_bcast_f32(const float* x, const float* y, float* out, int64_t outer, int64_t inner, vit_stream_t stream);
/* Res-ViT router backward (res-vit/model.py:186-190, the global half of out_conv's input):
 * vit_segment_colsum: out[s*ldo + c] = scale * sum_{r < seg_rows} in[(s*seg_stride + row0 + r)*ld + c] (per-image
 *   token sums / means; f32 or bf16 in, even ld, fixed order);
 * vit_router_dx_gate: out (bf16 [rows_pad][cols_pad], ld ldo) = bf16((dx[t][c] + [t % N >= reserve] g_scale
 *   g[t / N][c]) * gp[t][c]) for t < T, c < cols, zero elsewhere (in_conv's input-gradient times its saved GELU');
 *   optional col_partial[b*ldp + c] = column sums of the rounded values over row block b
 *   (vit_router_dx_gate_partial_rows(rows_pad) blocks; reduce with vit_colsum_batch) */
int vit_segment_colsum(const void* in, int32_t in_bf16, int64_t ld, int64_t segs, int64_t seg_stride, int64_t row0,
                       int64_t seg_rows, int64_t cols, float scale, float* out, int64_t ldo, vit_stream_t stream);
/* vit_segment_colsum, and each segment's result rounded to bf16 into rows [s*seg_stride, + bc_rows) of bc (ld ldbc):
 * the router's per-image token mean broadcast into the global half of out_conv's operand (res-vit/model.py:188-189) */
int vit_segment_colsum_bcast(const void* in, int32_t in_bf16, int64_t ld, int64_t segs, int64_t seg_stride,
                             int64_t row0, int64_t seg_rows, int64_t cols, float scale, float* out, int64_t ldo,
                             void* bc, int64_t ldbc, int64_t bc_rows, vit_stream_t stream);
int64_t vit_router_dx_gate_partial_rows(int64_t rows_pad);
int vit_router_dx_gate(const float* dx, int64_t ldx, const float* g, int64_t ldg, float g_scale, const void* gp,
                       int64_t ldgp, int64_t T, int64_t N, int64_t reserve, int64_t cols, void* out, int64_t ldo,
                       int64_t rows_pad, int64_t cols_pad, float* col_partial, int64_t ldp, vit_stream_t stream);
/* Res-ViT router head (res-vit/model.py:191-211, RouterModule.forward after out_conv), logits f32 [T][bs][2], T = B*N:
 *   soft = softmax(logits); entropy[0] = -(sum over tokens t % N >= reserve of p log(p + 1e-8)) / norm (per-block
 *   partials in ent_part[vit_router_head_partials(T)], then a fixed-order sum); training: y_soft = softmax(logits + g),
 *   g = noise (noise_mode 1) or -log(noise) (2: exponential draws) or 0 (0), hard = (y_hard - y_soft) + y_soft with
 *   y_hard = yhard_in or the one-hot of argmax y_soft; evaluation: hard = yhard_in or the one-hot of argmax soft;
 *   rows of reserved tokens (t % N < reserve) = (0, 1); indices[t] = sum_i hard[t][i][1] 2^(bs-1-i).
 * vit_router_head_bwd: dlogits from dsoft, the entropy gradient dent[0] and (training) the straight-through
 *   gradients dhard / dind through y_soft; any of dsoft / dhard / dind / dent may be NULL. */
int64_t vit_router_head_partials(int64_t T);
int vit_router_head_fwd(const float* logits, const float* noise, int32_t noise_mode, const float* yhard_in, int64_t T,
                        int64_t N, int32_t bs, int64_t reserve, int32_t training, float norm, float* soft, float* ysoft,
                        float* hard, float* indices, float* ent_part, float* entropy, vit_stream_t stream);
int vit_router_head_bwd(const float* soft, const float* ysoft, const float* dsoft, const float* dhard, const float* dind,
                        const float* dent, float norm, int64_t T, int64_t N, int32_t bs, int64_t reserve,
                        int32_t training, float* dlogits, vit_stream_t stream);
/* Res-ViT routing masks from the pattern index (res-vit/model.py:486-512, 336-368), one workgroup:
 * active[j*T + t] = (long)indices[t] in block position j's transformer set (bit v of active_masks[j], v < 32),
 * sel[k*T + t] = (indices[t] == k) for approximator keys k < nkeys, any[k] = any token with sel; bytes 0 / 1
 * (torch.bool storage). npos <= 8, nkeys <= 32. */
int vit_router_select(const float* indices, int64_t T, int32_t npos, const uint32_t* active_masks, int32_t nkeys,
                      void* active, void* sel, void* any, vit_stream_t stream);
/* out[r*ldo + c] (bf16) = in[r*ldi + c] for rows whose mask byte is non-zero (every row when mask is NULL), zeros for
 * the other rows (not read): a routed layer's output gradient as the bf16 operand of its backward, on the active rows
 * only (res-vit/model.py:507-512). cols, ldi, ldo multiples of 4. */
int vit_cast_rows_masked(const float* in, int64_t ldi, int64_t rows, int64_t cols, const void* mask, void* out,
                         int64_t ldo, vit_stream_t stream);
/* Res-ViT distillation loss on the cls rows (res-vit/model.py:40-59: mse_loss(student[:, 0], teacher[:, 0])):
 * vit_cls_mse: e[b][d] = x[b*ldx + d] - t[b*ldt + d], loss[0] = (sum of e^2, per-row partials part[B] then a fixed
 *   order) / (B D); vit_cls_mse_bwd: dx[b*lddx + d] += ((2 / (B D)) e[b][d]) g[0] (device scalar g). */
int vit_cls_mse(const float* x, int64_t ldx, const float* t, int64_t ldt, int64_t B, int64_t D, float* e, float* part,
                float* loss, vit_stream_t stream);
int vit_cls_mse_bwd(float* dx, int64_t lddx, const float* e, int64_t B, int64_t D, const float* g,
                    vit_stream_t stream);
/* out[r*ldo + c] = f32(in[r*ldi + c]) for bf16 `in` (attention outputs / gradients back to f32 modules) */
int vit_unpack_bf16_f32(const void* in, int64_t ldi, int64_t rows, int64_t cols, float* out, int64_t ldo,
                        vit_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Res-ViT optimizer step (res-vit/train.py:64-66 clip_grad_norm_(params, 1.0, 2) + AdamW.step(),
 * :272-277) over ONE flat f32 buffer of the trainable parameters, one 64-element-aligned segment per
 * parameter (replaces torch.nn.utils.clip_grad_norm_ and torch.optim.AdamW's per-tensor loops).
 * ---------------------------------------------------------------------------------------- */
/* partial[i] (f64) = sum of g[j]^2 over workgroup i's fixed grid-stride slice (nparts workgroups) */
int vit_sqnorm_partial(const float* g, int64_t n, double* partial, int32_t nparts, vit_stream_t stream);
/* one workgroup: norm = sqrt(sum partial) (partial may be NULL: no clipping), clip coefficient
 * min(1, max_norm / (norm + 1e-6)) (1 when max_norm <= 0); norm_out[0..1] = {norm, coef} if non-NULL.
 * For each of nseg segments: if used[s] > 0, steps[s] += 1 and table[s] (float4) = {lr / (1 - beta1^step),
 * sqrt(1 - beta2^step), 1, coef}; otherwise {0, 0, 0, coef} (torch skips parameters without a grad). */
int vit_adamw_prep(const double* partial, int32_t nparts, const float* used, float* steps, int32_t nseg,
                   float lr, float beta1, float beta2, float max_norm, float* table, float* norm_out,
                   vit_stream_t stream);
/* per chunk c (chunks[3c..3c+2] = {segment, start element, length <= vit_adamw_chunk_elems()}), for the
 * segment's active parameters, torch's AdamW (decoupled decay) on the clipped gradient g*coef:
 *   p *= decay; m += (1-beta1)(g - m); v = beta2 v + (1-beta2) g^2;
 *   p -= step_size * m / (sqrt(v) / sqrt(bc2) + eps);   g <- g*coef if write_grad; p_bf16 = bf16(p)
 * decay = 1 - lr*weight_decay and the (1 - beta) factors are rounded from the caller's doubles, as torch's
 * Python scalars are. */
int vit_adamw_update(float* p, float* g, float* m, float* v, void* p_bf16, const int64_t* chunks, int32_t nchunks,
                     const float* table, float decay, float beta1, float beta2, float one_minus_beta1,
                     float one_minus_beta2, float eps, int32_t write_grad, vit_stream_t stream);
int vit_adamw_chunk_elems(void);
/* g[i] *= *coef (device scalar; the in-place scaling of clip_grad_norm_) */
int vit_scale_by_coef(float* g, int64_t n, const float* coef, vit_stream_t stream);
/* bytes of device memory at ptr set to 0 on the stream (hipMemsetAsync) */
int vit_zero(void* ptr, int64_t bytes, vit_stream_t stream);
/* rows whose mask byte (mask[r], e.g. a torch.bool [rows] tensor) is 0: dst + r*dld <- src + r*sld, row_bytes bytes
 * (zeros when src is NULL); other rows untouched. 16-B aligned rows, row_bytes % 16 == 0. Res-ViT's routed-layer
 * selection `where(active, layer(x), x)` (res-vit/model.py:507-512) and its backward masks, inside the fused layer. */
int vit_rows_select(void* dst, int64_t dld, const void* src, int64_t sld, const void* mask, int64_t rows,
                    int64_t row_bytes, vit_stream_t stream);
/* height rows of width bytes: dst + r*dpitch <- src + r*spitch (hipMemcpy2DAsync, device to device) */
int vit_copy2d(void* dst, int64_t dpitch, const void* src, int64_t spitch, int64_t width, int64_t height,
               vit_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* VIT_HIP_H_ */
