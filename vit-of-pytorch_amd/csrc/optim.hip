// Optimizer kernels of the Res-ViT training step (reference res-vit/train.py:64-66,272-277):
// torch.nn.utils.clip_grad_norm_(params, max_norm, 2) followed by torch.optim.AdamW.step(), over ONE
// flat f32 buffer of the trainable parameters (vitmi.flat.FlatParams: 64-element aligned segments,
// one per parameter).
//
//   vit_sqnorm_partial  grid of `nparts` workgroups, each a fixed grid-stride slice of the gradient:
//                       f64 partial sums of squares (deterministic, no atomics)
//   vit_adamw_prep      one workgroup: total norm = sqrt(sum of the partials, fixed order), clip
//                       coefficient min(1, max_norm / (norm + 1e-6)); per segment, if the parameter
//                       received a gradient this step, step += 1 and the bias corrections
//   vit_adamw_update    one workgroup per chunk (a run of <= 8192 elements inside one segment):
//                       clip scale, decoupled weight decay, the two moments and the update, in
//                       torch's single-tensor AdamW order (torch/optim/adamw.py _single_tensor_adam)
//   vit_scale_by_coef   grads *= coef (device scalar): the standalone clip_grad_norm_
//
// HBM work per element of the update: p, g, m, v read + p, m, v (+ g when the clipped gradient is
// written back) written = 28-32 B; the norm pass reads g once (4 B).
#include "common.h"

namespace {

constexpr int kNormThreads = 256;

__global__ void __launch_bounds__(kNormThreads) sqnorm_partial_kernel(const float* __restrict__ g, long n,
                                                                      double* __restrict__ partial) {
  double acc = 0.0;
  const long n4 = n / 4;
  const long stride = (long)gridDim.x * kNormThreads;
  for (long i = (long)blockIdx.x * kNormThreads + threadIdx.x; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(g)[i];
    // f32 squares summed in f64: the order is fixed by the launch shape
    acc += (double)(v.x * v.x) + (double)(v.y * v.y) + (double)(v.z * v.z) + (double)(v.w * v.w);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const float t = g[n4 * 4 + threadIdx.x];
    acc += (double)(t * t);
  }
  __shared__ double red[kNormThreads];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = kNormThreads / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// table[s] = {step_size = lr / bc1, sqrt(bc2), active, clip coefficient}
__global__ void __launch_bounds__(256) adamw_prep_kernel(const double* __restrict__ partial, int nparts,
                                                         const float* __restrict__ used, float* __restrict__ steps,
                                                         int nseg, float lr, float beta1, float beta2,
                                                         float max_norm, float4* __restrict__ table,
                                                         float* __restrict__ norm_out) {
  __shared__ double red[256];
  __shared__ float coef_s;
  double acc = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 256) acc += partial[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float norm = partial ? (float)sqrt(red[0]) : 0.0f;
    // torch.nn.utils.clip_grad_norm_: clip_coef = max_norm / (total_norm + 1e-6), clamped to 1
    float coef = 1.0f;
    if (partial && max_norm > 0.0f) coef = fminf(max_norm / (norm + 1e-6f), 1.0f);
    coef_s = coef;
    if (norm_out) {
      norm_out[0] = norm;
      norm_out[1] = coef;
    }
  }
  __syncthreads();
  const float coef = coef_s;
  for (int s = threadIdx.x; s < nseg; s += 256) {
    const bool act = used[s] > 0.0f;
    float st = steps[s];
    if (act) {
      st += 1.0f;
      steps[s] = st;
    }
    // torch: bias_correction1 = 1 - beta1 ** step; step_size = lr / bias_correction1;
    //        bias_correction2_sqrt = sqrt(1 - beta2 ** step)   (host doubles there; doubles here)
    const double bc1 = 1.0 - pow((double)beta1, (double)st);
    const double bc2 = 1.0 - pow((double)beta2, (double)st);
    table[s] = act ? make_float4((float)((double)lr / bc1), (float)sqrt(bc2), 1.0f, coef)
                   : make_float4(0.0f, 0.0f, 0.0f, coef);
  }
}

constexpr int kChunk = 8192;  // elements per update workgroup (256 threads x 4 x 8)

__global__ void __launch_bounds__(256) adamw_update_kernel(float* __restrict__ p, float* __restrict__ g,
                                                           float* __restrict__ m, float* __restrict__ v,
                                                           bf16_t* __restrict__ pb, const int64_t* __restrict__ chunks,
                                                           const float4* __restrict__ table, float decay, float beta1,
                                                           float beta2, float omb1, float omb2, float eps,
                                                           int write_grad) {
  const int64_t seg = chunks[3 * blockIdx.x], start = chunks[3 * blockIdx.x + 1], len = chunks[3 * blockIdx.x + 2];
  const float4 t = table[seg];
  const float coef = t.w;
  if (t.z == 0.0f) {  // no gradient this step: torch's AdamW skips the parameter entirely
    return;
  }
  const float step_size = t.x, bc2s = t.y;
  // segments start 64-element aligned and chunks are multiples of 4 except a segment's last
  const long n4 = len / 4;
  float4* p4 = reinterpret_cast<float4*>(p + start);
  float4* g4 = reinterpret_cast<float4*>(g + start);
  float4* m4 = reinterpret_cast<float4*>(m + start);
  float4* v4 = reinterpret_cast<float4*>(v + start);
  auto upd = [&](float& pp, float& gg, float& mm, float& vv) {
    gg *= coef;
    pp *= decay;                                        // param.mul_(1 - lr * weight_decay)
    mm += omb1 * (gg - mm);                             // exp_avg.lerp_(grad, 1 - beta1)
    vv = vv * beta2 + omb2 * gg * gg;                   // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
    const float denom = sqrtf(vv) / bc2s + eps;         // (exp_avg_sq.sqrt() / bc2_sqrt).add_(eps)
    pp -= step_size * (mm / denom);                     // param.addcdiv_(exp_avg, denom, -step_size)
  };
  for (long i = threadIdx.x; i < n4; i += 256) {
    float4 pv = p4[i], gv = g4[i], mv = m4[i], vv = v4[i];
    upd(pv.x, gv.x, mv.x, vv.x);
    upd(pv.y, gv.y, mv.y, vv.y);
    upd(pv.z, gv.z, mv.z, vv.z);
    upd(pv.w, gv.w, mv.w, vv.w);
    p4[i] = pv;
    m4[i] = mv;
    v4[i] = vv;
    if (write_grad) g4[i] = gv;
    if (pb) {
      uint2 u;
      u.x = pack2bf(pv.x, pv.y);
      u.y = pack2bf(pv.z, pv.w);
      reinterpret_cast<uint2*>(pb + start)[i] = u;
    }
  }
  const long tail = n4 * 4 + threadIdx.x;
  if (tail < len) {
    float pp = p[start + tail], gg = g[start + tail], mm = m[start + tail], vv = v[start + tail];
    upd(pp, gg, mm, vv);
    p[start + tail] = pp;
    m[start + tail] = mm;
    v[start + tail] = vv;
    if (write_grad) g[start + tail] = gg;
    if (pb) pb[start + tail] = f2bf(pp);
  }
}

__global__ void scale_by_coef_kernel(float* __restrict__ g, long n, const float* __restrict__ coef) {
  const float c = *coef;
  const long n4 = n / 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 v = reinterpret_cast<float4*>(g)[i];
    v.x *= c; v.y *= c; v.z *= c; v.w *= c;
    reinterpret_cast<float4*>(g)[i] = v;
  }
  const long t = n4 * 4 + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && t < n) g[t] *= c;
}

}  // namespace

extern "C" int vit_sqnorm_partial(const float* g, int64_t n, double* partial, int32_t nparts, vit_stream_t stream) {
  VIT_CHECK_ARG(g && partial && n >= 0 && nparts > 0 && nparts <= 65536, "vit_sqnorm_partial: bad args");
  VIT_CHECK_ARG((uintptr_t)g % 16 == 0, "vit_sqnorm_partial: gradient buffer must be 16-B aligned");
  hipLaunchKernelGGL(sqnorm_partial_kernel, dim3(nparts), dim3(kNormThreads), 0, (hipStream_t)stream, g, (long)n,
                     partial);
  VIT_LAUNCH_CHECK("vit_sqnorm_partial");
}

extern "C" int vit_adamw_prep(const double* partial, int32_t nparts, const float* used, float* steps, int32_t nseg,
                              float lr, float beta1, float beta2, float max_norm, float* table, float* norm_out,
                              vit_stream_t stream) {
  VIT_CHECK_ARG(nseg >= 0 && (nseg == 0 || (used && steps && table)) &&
                    (partial ? nparts > 0 && nparts <= 65536 : nparts == 0),
                "vit_adamw_prep: bad args (partial needs nparts in 1..65536, no partial needs nparts 0)");
  VIT_CHECK_ARG(beta1 >= 0.0f && beta1 < 1.0f && beta2 >= 0.0f && beta2 < 1.0f, "vit_adamw_prep: betas must be in [0, 1)");
  hipLaunchKernelGGL(adamw_prep_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, partial, (int)nparts, used, steps,
                     (int)nseg, lr, beta1, beta2, max_norm, (float4*)table, norm_out);
  VIT_LAUNCH_CHECK("vit_adamw_prep");
}

extern "C" int vit_adamw_update(float* p, float* g, float* m, float* v, void* p_bf16, const int64_t* chunks,
                                int32_t nchunks, const float* table, float decay, float beta1, float beta2,
                                float one_minus_beta1, float one_minus_beta2, float eps, int32_t write_grad,
                                vit_stream_t stream) {
  VIT_CHECK_ARG(p && g && m && v && chunks && table && nchunks >= 0, "vit_adamw_update: bad args");
  VIT_CHECK_ARG(((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16 == 0 && (uintptr_t)p_bf16 % 8 == 0,
                "vit_adamw_update: buffers must be 16-B aligned (bf16 mirror 8-B)");
  if (nchunks == 0) return VIT_OK;
  hipLaunchKernelGGL(adamw_update_kernel, dim3(nchunks), dim3(256), 0, (hipStream_t)stream, p, g, m, v,
                     (bf16_t*)p_bf16, chunks, (const float4*)table, decay, beta1, beta2, one_minus_beta1,
                     one_minus_beta2, eps, (int)write_grad);
  VIT_LAUNCH_CHECK("vit_adamw_update");
}

extern "C" int vit_adamw_chunk_elems(void) { return kChunk; }

extern "C" int vit_scale_by_coef(float* g, int64_t n, const float* coef, vit_stream_t stream) {
  VIT_CHECK_ARG(g && coef && n >= 0 && (uintptr_t)g % 16 == 0, "vit_scale_by_coef: bad args");
  if (n == 0) return VIT_OK;
  long blocks = (n / 4 + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
  hipLaunchKernelGGL(scale_by_coef_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, g, (long)n, coef);
  VIT_LAUNCH_CHECK("vit_scale_by_coef");
}

extern "C" int vit_zero(void* ptr, int64_t bytes, vit_stream_t stream) {
  VIT_CHECK_ARG(ptr && bytes >= 0, "vit_zero: bad args");
  if (bytes == 0) return VIT_OK;
  return vit::check_hip(hipMemsetAsync(ptr, 0, (size_t)bytes, (hipStream_t)stream), "vit_zero");
}

// Row selection (Res-ViT's `where(active, layer(x), x)` folded into the layer node): every row r whose mask byte is 0
// gets dst row r <- src row r (zeros when src is null); rows whose mask byte is non-zero are left alone. 16-B chunks.
__global__ void rows_select_kernel(char* __restrict__ dst, long dld, const char* __restrict__ src, long sld,
                                   const unsigned char* __restrict__ mask, long rows, long chunks) {
  const long n = rows * chunks;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / chunks, c = i - r * chunks;
    if (mask[r]) continue;
    const uint4 v = src ? *reinterpret_cast<const uint4*>(src + r * sld + c * 16) : make_uint4(0u, 0u, 0u, 0u);
    *reinterpret_cast<uint4*>(dst + r * dld + c * 16) = v;
  }
}

extern "C" int vit_rows_select(void* dst, int64_t dld, const void* src, int64_t sld, const void* mask, int64_t rows,
                               int64_t row_bytes, vit_stream_t stream) {
  VIT_CHECK_ARG(dst && mask && rows >= 0 && row_bytes >= 0 && row_bytes % 16 == 0 && dld % 16 == 0 &&
                    (src == nullptr || sld % 16 == 0) && ((uintptr_t)dst | (uintptr_t)src) % 16 == 0,
                "vit_rows_select: bad args (16-B aligned rows of a multiple of 16 bytes)");
  VIT_CHECK_ARG(dld >= row_bytes && (src == nullptr || sld >= row_bytes), "vit_rows_select: row pitch below row_bytes");
  const long n = (long)rows * (row_bytes / 16);
  if (n == 0) return VIT_OK;
  long blocks = (n + 255) / 256;
  blocks = blocks > 8192 ? 8192 : blocks;
  hipLaunchKernelGGL(rows_select_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, (char*)dst,
                     (long)dld, (const char*)src, (long)sld, (const unsigned char*)mask, (long)rows, (long)(row_bytes / 16));
  VIT_LAUNCH_CHECK("vit_rows_select");
}

extern "C" int vit_copy2d(void* dst, int64_t dpitch, const void* src, int64_t spitch, int64_t width, int64_t height,
                          vit_stream_t stream) {
  VIT_CHECK_ARG(dst && src && width >= 0 && height >= 0 && dpitch >= width && spitch >= width, "vit_copy2d: bad args");
  if (width == 0 || height == 0) return VIT_OK;
  return vit::check_hip(hipMemcpy2DAsync(dst, (size_t)dpitch, src, (size_t)spitch, (size_t)width, (size_t)height,
                                         hipMemcpyDeviceToDevice, (hipStream_t)stream),
                        "vit_copy2d");
}
