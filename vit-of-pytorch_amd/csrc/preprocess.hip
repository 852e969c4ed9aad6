// GPU-side training-input transform: the reference's loader pipeline
// Resize(size) -> RandomHorizontalFlip -> ToTensor -> Normalize(0.5, 0.5)
// (src/data_loaders.py:66-80, 100-112) as one HBM-bound kernel from uint8 HWC images to the f32
// NCHW batch the model consumes. Resize is Pillow's 8-bit fixed-point bilinear resampling (the
// library under torchvision's PIL path; restated and pinned in oracle/preprocess.py), reproduced
// bit-exactly: coefficients in double without FMA contraction, horizontal pass clipped to uint8,
// then the vertical pass. Ratios up to 4x (at most 9 taps per axis) run the tiled two-pass LDS
// kernel, which computes each column's and row's weights once per block; larger ratios run the
// generic kernel (one thread per output pixel, every weight recomputed - deterministically, so the
// normalising sum and each weight still match Pillow).
#include "common.h"

#include <algorithm>
#include <cmath>

namespace {

constexpr int kPrecisionBits = 32 - 8 - 2;

struct Axis {
  double scale, support, ss;
  int in_size;
};

__host__ __device__ inline Axis make_axis(int in_size, int out_size) {
  Axis a;
  a.scale = (double)in_size / (double)out_size;
  const double filterscale = a.scale < 1.0 ? 1.0 : a.scale;
  a.support = 1.0 * filterscale;
  a.ss = 1.0 / filterscale;
  a.in_size = in_size;
  return a;
}

__device__ inline double tri(double x) {
  if (x < 0.0) x = -x;
  return x < 1.0 ? 1.0 - x : 0.0;
}

// Pillow precompute_coeffs for output index xx: first tap, tap count, centre and weight sum.
__device__ inline void taps(const Axis& a, int xx, int& xmin, int& cnt, double& center, double& ww) {
#pragma clang fp contract(off)
  center = (xx + 0.5) * a.scale;
  xmin = (int)(center - a.support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + a.support + 0.5);
  if (xmax > a.in_size) xmax = a.in_size;
  cnt = xmax - xmin;
  ww = 0.0;
  for (int x = 0; x < cnt; ++x) ww += tri((x + xmin - center + 0.5) * a.ss);
}

// normalize_coeffs_8bpp: fixed-point weight of tap x
__device__ inline int coeff(const Axis& a, int x, int xmin, double center, double ww) {
#pragma clang fp contract(off)
  double w = tri((x + xmin - center + 0.5) * a.ss);
  if (ww != 0.0) w = w / ww;
  return w < 0 ? (int)(-0.5 + w * (double)(1 << kPrecisionBits)) : (int)(0.5 + w * (double)(1 << kPrecisionBits));
}

__device__ inline int clip8(int v) {
  if (v >= (1 << kPrecisionBits << 8)) return 255;
  if (v <= 0) return 0;
  return v >> kPrecisionBits;
}

struct PrepArgs {
  const uint8_t* in;
  long in_bs;  // bytes between images
  int H, W, oh, ow, B;
  const uint8_t* flips;
  float mean[3], stdv[3];
  float* out;
};

__global__ void __launch_bounds__(256) preprocess_kernel(PrepArgs p) {
#pragma clang fp contract(off)
  const Axis ax = make_axis(p.W, p.ow), ay = make_axis(p.H, p.oh);
  const long plane = (long)p.oh * p.ow;
  const long total = (long)p.B * plane;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / plane);
    const int rem = (int)(i - (long)b * plane);
    const int y = rem / p.ow, x = rem - y * p.ow;
    const int xs = (p.flips && p.flips[b]) ? p.ow - 1 - x : x;  // the flip mirrors the resized image
    int xmin, xcnt, ymin, ycnt;
    double xc, xw, yc, yw;
    taps(ax, xs, xmin, xcnt, xc, xw);
    taps(ay, y, ymin, ycnt, yc, yw);
    const uint8_t* img = p.in + (long)b * p.in_bs;
    int acc0 = 1 << (kPrecisionBits - 1), acc1 = acc0, acc2 = acc0;
    for (int j = 0; j < ycnt; ++j) {
      const uint8_t* row = img + ((long)(ymin + j) * p.W + xmin) * 3;
      int h0 = 1 << (kPrecisionBits - 1), h1 = h0, h2 = h0;
      for (int k = 0; k < xcnt; ++k) {
        const int c = coeff(ax, k, xmin, xc, xw);
        h0 += row[3 * k + 0] * c;
        h1 += row[3 * k + 1] * c;
        h2 += row[3 * k + 2] * c;
      }
      const int cy = coeff(ay, j, ymin, yc, yw);
      acc0 += clip8(h0) * cy;
      acc1 += clip8(h1) * cy;
      acc2 += clip8(h2) * cy;
    }
    const int v[3] = {clip8(acc0), clip8(acc1), clip8(acc2)};
    float* o = p.out + (long)b * 3 * plane + rem;
#pragma unroll
    for (int c = 0; c < 3; ++c) o[c * plane] = ((float)v[c] / 255.0f - p.mean[c]) / p.stdv[c];
  }
}

// Fast path (every axis with at most KMAX <= 9 taps, i.e. ratios up to 4x): a block owns 64 output
// columns x 32 output rows of one image and runs Pillow's two passes through LDS. Pass 1: the
// horizontal pass over the band of input rows those 32 output rows read (at most 31 * 4 + 1 + 9
// rows), each thread one output column with its weights in registers (computed once), results
// clipped to 8 bits into LDS. Pass 2: the vertical pass for the 32 rows from LDS with the row
// weights (computed once per block by 32 threads). Every input pixel is gathered once per block
// instead of once per output row that uses it.
constexpr int kColsPerBlock = 64, kRowsPerBlock = 32, kRowLanes = 4, kBandMax = 31 * 4 + 1 + 9;

template <int KMAX>
__global__ void __launch_bounds__(kColsPerBlock* kRowLanes) preprocess_tiled_kernel(PrepArgs p) {
#pragma clang fp contract(off)
  __shared__ int s_ky[kRowsPerBlock][KMAX];
  __shared__ int s_ymin[kRowsPerBlock], s_ycnt[kRowsPerBlock];
  __shared__ uint32_t s_h[kBandMax][kColsPerBlock];  // horizontal pass, (r, g, b) bytes
  const Axis ax = make_axis(p.W, p.ow), ay = make_axis(p.H, p.oh);
  const int b = blockIdx.z;
  const int y0 = blockIdx.y * kRowsPerBlock;
  const int rows = p.oh - y0 < kRowsPerBlock ? p.oh - y0 : kRowsPerBlock;
  const int tid = threadIdx.y * kColsPerBlock + threadIdx.x;
  if (tid < rows) {
    int ymin, ycnt;
    double yc, yw;
    taps(ay, y0 + tid, ymin, ycnt, yc, yw);
    s_ymin[tid] = ymin;
    s_ycnt[tid] = ycnt;
    for (int j = 0; j < KMAX; ++j) s_ky[tid][j] = j < ycnt ? coeff(ay, j, ymin, yc, yw) : 0;
  }
  const int x = blockIdx.x * kColsPerBlock + threadIdx.x;
  const bool live = x < p.ow;
  const int xs = live && p.flips && p.flips[b] ? p.ow - 1 - x : x;
  int xmin = 0, xcnt = 0;
  int kx[KMAX];
  if (live) {
    double xc, xw;
    taps(ax, xs, xmin, xcnt, xc, xw);
#pragma unroll
    for (int k = 0; k < KMAX; ++k) kx[k] = k < xcnt ? coeff(ax, k, xmin, xc, xw) : 0;
  }
  __syncthreads();
  const int band0 = s_ymin[0];
  const int nband = s_ymin[rows - 1] + s_ycnt[rows - 1] - band0;  // <= kBandMax (host: ksize <= 9)
  if (live) {
    const uint8_t* src = p.in + (long)b * p.in_bs + ((long)band0 * p.W + xmin) * 3;
    for (int r = threadIdx.y; r < nband; r += kRowLanes) {
      const uint8_t* row = src + (long)r * p.W * 3;
      int h0 = 1 << (kPrecisionBits - 1), h1 = h0, h2 = h0;
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        if (k < xcnt) {
          h0 += row[3 * k + 0] * kx[k];
          h1 += row[3 * k + 1] * kx[k];
          h2 += row[3 * k + 2] * kx[k];
        }
      }
      s_h[r][threadIdx.x] = (uint32_t)clip8(h0) | ((uint32_t)clip8(h1) << 8) | ((uint32_t)clip8(h2) << 16);
    }
  }
  __syncthreads();
  if (!live) return;
  const long plane = (long)p.oh * p.ow;
  float* o = p.out + (long)b * 3 * plane + x;
  for (int r = threadIdx.y; r < rows; r += kRowLanes) {
    const int ymin = s_ymin[r] - band0, ycnt = s_ycnt[r];
    int acc0 = 1 << (kPrecisionBits - 1), acc1 = acc0, acc2 = acc0;
    for (int j = 0; j < ycnt; ++j) {
      const uint32_t hv = s_h[ymin + j][threadIdx.x];
      const int cy = s_ky[r][j];
      acc0 += (int)(hv & 0xffu) * cy;
      acc1 += (int)((hv >> 8) & 0xffu) * cy;
      acc2 += (int)((hv >> 16) & 0xffu) * cy;
    }
    const long off = (long)(y0 + r) * p.ow;
    o[off] = ((float)clip8(acc0) / 255.0f - p.mean[0]) / p.stdv[0];
    o[plane + off] = ((float)clip8(acc1) / 255.0f - p.mean[1]) / p.stdv[1];
    o[2 * plane + off] = ((float)clip8(acc2) / 255.0f - p.mean[2]) / p.stdv[2];
  }
}

// Pillow's kernel size for one axis: ceil(support) * 2 + 1, support = max(in / out, 1)
int axis_ksize(long in, long out) {
  const double scale = (double)in / (double)out;
  const double support = scale < 1.0 ? 1.0 : scale;
  return (int)std::ceil(support) * 2 + 1;
}

}  // namespace

extern "C" int vit_preprocess_u8(const uint8_t* images, int64_t B, int64_t H, int64_t W, int64_t image_stride,
                                 const uint8_t* flips, int64_t out_h, int64_t out_w, const float* mean_std,
                                 float* out, vit_stream_t stream) {
  VIT_CHECK_ARG(images && out && mean_std && B > 0 && H > 0 && W > 0 && out_h > 0 && out_w > 0,
                "vit_preprocess_u8: bad args");
  VIT_CHECK_ARG(image_stride >= H * W * 3, "vit_preprocess_u8: image_stride %lld < H*W*3", (long long)image_stride);
  VIT_CHECK_ARG(H < (1 << 15) && W < (1 << 15) && out_h < (1 << 15) && out_w < (1 << 15) &&
                    B * out_h * out_w < (1LL << 40),
                "vit_preprocess_u8: sizes too large");
  PrepArgs p;
  p.in = images;
  p.in_bs = image_stride;
  p.H = (int)H; p.W = (int)W; p.oh = (int)out_h; p.ow = (int)out_w; p.B = (int)B;
  p.flips = flips;
  for (int c = 0; c < 3; ++c) {
    p.mean[c] = mean_std[c];
    p.stdv[c] = mean_std[3 + c];
  }
  p.out = out;
  const int ks = std::max(axis_ksize(W, out_w), axis_ksize(H, out_h));
  if (ks <= 9 && B < 65536) {
    const dim3 grid((unsigned)((out_w + kColsPerBlock - 1) / kColsPerBlock),
                    (unsigned)((out_h + kRowsPerBlock - 1) / kRowsPerBlock), (unsigned)B);
    const dim3 block(kColsPerBlock, kRowLanes);
    if (ks <= 3)
      hipLaunchKernelGGL(preprocess_tiled_kernel<3>, grid, block, 0, (hipStream_t)stream, p);
    else if (ks <= 5)
      hipLaunchKernelGGL(preprocess_tiled_kernel<5>, grid, block, 0, (hipStream_t)stream, p);
    else
      hipLaunchKernelGGL(preprocess_tiled_kernel<9>, grid, block, 0, (hipStream_t)stream, p);
    VIT_LAUNCH_CHECK("vit_preprocess_u8");
  }
  // generic path: any ratio, every weight recomputed per pixel
  const long total = B * out_h * out_w;
  long blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(preprocess_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, p);
  VIT_LAUNCH_CHECK("vit_preprocess_u8");
}
