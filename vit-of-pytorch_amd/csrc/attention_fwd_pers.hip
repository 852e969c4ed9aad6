// Attention forward, persistent form (image widths 32 and 64; N up to 208 at hd 64).
//
// Replaces SelfAttention.forward's core (reference src/model.py:90-97: q k^T / sqrt(hd), softmax, P v).
//
// One workgroup per CU (16 waves) walks (image, head) items. The K, V and Q images of the next item come in by
// LDS-DMA (buffer_load ... lds) into the other of two slots while this item's 16-query strips run, so the CU's
// HBM stream does not stop between items; the one-shot kernel (attention.hip attn_fwd2_kernel: one workgroup
// per item, images loaded through registers, then computed) leaves it idle during each workgroup's load and
// tail. The arithmetic per strip is attn_fwd2_kernel's, operation for operation (same MFMA chains, max,
// exp2, sums, rounding), so the two produce identical bits; only the Q fragments come from an LDS image
// instead of straight from HBM, and O leaves from registers (8-B pieces of 16 rows per store).
// LDS: slot 0 and slot 1, each K | V | Q as swizzled [NP][HD] bf16 images (156 KB at N = 197, hd 64). Separate
// LDS objects per slot and a slot-templated item body: hipcc proves that a DMA in flight into one slot cannot
// alias the reads of the other and inserts no vmcnt wait for it.
// Waits: each wave drains only its own DMAs at the item start: its O / lse stores of the previous item were
// issued after them and vmcnt retires in order, so it waits for vmcnt <= (stores issued since), never for the
// stores themselves; their packed words stay live to the end of the item (hipcc protects the source
// registers of an outstanding store with a vmcnt wait before reusing them).
#include "attn_pers.h"
#include <type_traits>

namespace {
using namespace vit_attn;

// waves per workgroup: 16 (four per SIMD, at most one 16-query strip each per item: the strip's dependent
// chains, MFMA -> max -> exp2 -> sum -> P V, are latency-bound and need the other waves to hide them; 8
// waves with two strips each ran 17% slower than the one-shot kernel); 8 past 16 key tiles (hd 32, N > 256),
// where a wave's two strips do not fit 128 registers
template <int NKT>
constexpr int fp_nw = NKT <= 16 ? 16 : 8;

template <int HD, int NKT>
__global__ void __launch_bounds__(fp_nw<NKT> * 64, 1) attn_fwd_pers_kernel(const bf16_t* __restrict__ qkv,
                                                                     bf16_t* __restrict__ o, float* __restrict__ lse,
                                                                     int nitems, int N, int H, int hd, float scale,
                                                                     int nq) {
  constexpr int NW = fp_nw<NKT>;
  constexpr int NP = NKT * 16;
  constexpr int IMG = NP * HD * 2;
  constexpr int T = ImgLane<HD>::TILE;
  constexpr int KK = HD / 32;
  constexpr int ND = HD / 16;
  constexpr int MAXS = (NKT + NW - 1) / NW;  // strips per wave and item
  constexpr int SPS = ND + 1;                // store instructions per strip: ND O pieces + the lse row
  static_assert(MAXS <= 3, "store counts");
  __shared__ __attribute__((aligned(16))) char s0[3 * IMG];  // K | V | Q, slot 0
  __shared__ __attribute__((aligned(16))) char s1[3 * IMG];  // slot 1

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, i = lane & 15;
  const ImgLane<HD> L(lane);
  const int D = H * hd;
  const long rs = 3L * D;
  const float c = scale * LOG2E;
  const int nqa = min(N, (nq + 31) / 32 * 32);  // whole 32-row pairs (the backward's stage 2 reads their lse)
  const int nqt = (nqa + 15) / 16;
  const int qrows = min(NP, nqt * 16);
  constexpr int KV_PIECES = 2 * ((NP + 1024 / (HD * 2) - 1) / (1024 / (HD * 2)));

  int item = blockIdx.x;
  if (item >= nitems) return;
  auto qkv_of = [&](int it_) { return qkv + (long)(it_ / H) * N * rs + (long)(it_ % H) * hd; };
  // K, V (all NP rows: the padding rows of the last key tile land as zeros) and the Q rows of the computed strips
  auto dma_item = [&](lds_t* img, int it_) {
    const bf16_t* b = qkv_of(it_);
    dma_pair<HD>(img, b + D, rs, img + IMG, b + 2 * D, rs, NP, N, hd, 0, wave, lane, NW);
    dma_image<HD>(img + 2 * IMG, b, rs, qrows, N, hd, KV_PIECES % NW, wave, lane, NW);
  };
  dma_item((lds_t*)s0, item);

  int nst = 0;  // store instructions this wave issued after its last DMA
  auto body = [&](auto slot) {
    constexpr int SLOT = decltype(slot)::value;
    lds_t* const Ki = (lds_t*)(SLOT ? s1 : s0);
    lds_t* const Vi = Ki + IMG;
    lds_t* const Qi = Ki + 2 * IMG;
    lds_t* const Kn = (lds_t*)(SLOT ? s0 : s1);
    const int bh = item;
    const int b = bh / H, h = bh % H;
    const int next = __builtin_amdgcn_readfirstlane(item + (int)gridDim.x);

    // this item's images landed (each wave drains its own DMAs, then the barrier), and every wave is past
    // the previous item (the last reader of the other slot)
    switch (nst / SPS) {
      case 0: wait_vmcnt<0>(); break;
      case 1: wait_vmcnt<SPS>(); break;
      case 2: wait_vmcnt<2 * SPS>(); break;
      default: wait_vmcnt<3 * SPS>(); break;
    }
    lds_barrier();
    if (next < nitems) dma_item(Kn, next);

    bf16_t* const ob = o + (long)b * N * D + (long)h * hd;
    const __amdgpu_buffer_rsrc_t rl = make_rsrc(uniform_ptr(lse + (long)bh * N), (uint32_t)N * 4);
    uint2 ow[MAXS][ND];
    float lv[MAXS];
    int ns = 0;
#pragma unroll
    for (int u = 0; u < MAXS; ++u) {
      const int qt = wave + u * NW;
      if (qt >= nqt) break;
      ++ns;
      v8bf qf[KK];
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) qf[kk] = __builtin_bit_cast(v8bf, lds_ld<v8s>(Qi + qt * T + L.row[kk]));
      v4f s[NKT];
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        s[kt] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
          s[kt] = mfma(__builtin_bit_cast(v8bf, lds_ld<v8s>(Ki + kt * T + L.row[kk])), qf[kk], s[kt]);
      }
      if (N < NP) {  // only the last tile holds padded keys
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if ((NKT - 1) * 16 + 4 * g + r >= N) s[NKT - 1][r] = -INFINITY;
      }
      float mx = max3f(s[0][0], s[0][1], s[0][2]);
      mx = fmaxf(mx, s[0][3]);
#pragma unroll
      for (int kt = 1; kt < NKT; ++kt) {
        mx = max3f(mx, s[kt][0], s[kt][1]);
        mx = max3f(mx, s[kt][2], s[kt][3]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mc = mx * c;
      float l = 0.f;  // f32 row sum of the unrounded P (the reference's normalisation)
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s[kt][r] = ex2(fmaf(s[kt][r], c, -mc));
          l += s[kt][r];
        }
      l += __shfl_xor(l, 16, 64);
      l += __shfl_xor(l, 32, 64);
      v4f acc[ND];
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) acc[dt] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKT / 2; ++ks) {
        const v8bf pp = pack8(s[2 * ks], s[2 * ks + 1]);
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) {
          v8s vt;
          vt.lo = lds_tr(Vi + 2 * ks * T + L.tr[dt]);
          vt.hi = lds_tr(Vi + (2 * ks + 1) * T + L.tr[dt]);
          acc[dt] = mfma(__builtin_bit_cast(v8bf, vt), pp, acc[dt]);
        }
      }
      if constexpr (NKT % 2 == 1) {
        const v4s pp = pack4(s[NKT - 1]);
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) acc[dt] = mfma16_add(lds_tr(Vi + (NKT - 1) * T + L.tr[dt]), pp, acc[dt]);
      }
      const int q = qt * 16 + i;
      const float inv_l = 1.0f / l;
      lv[u] = mx * scale + logf(l);
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) ow[u][dt] = pack4bf(acc[dt], inv_l);
      // O rows qt*16 + i, columns 16 dt + 4 g ..: past row N - 1 / column hd the descriptor drops the piece
      const __amdgpu_buffer_rsrc_t ro = rows_rsrc(ob, D, qt * 16, N, hd);
      const int offs = (int)(i * D * 2) + g * 8;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) st_b64(ro, dt * 16 < hd ? offs + dt * 32 : 0x40000000, ow[u][dt]);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, lv[u]), rl,
                                            g == 0 && q < N ? q * 4 : 0x40000000, 0, 0);
    }
    // the stores' source words stay live to the end of the item (no vmcnt wait before their registers are reused)
#pragma unroll
    for (int u = 0; u < MAXS; ++u) {
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) keep_live2(ow[u][dt]);
      asm volatile("" ::"v"(lv[u]));
    }
    nst = ns * SPS;
    item = __builtin_amdgcn_readfirstlane(next);
  };
  while (true) {
    body(std::integral_constant<int, 0>{});
    if (item >= nitems) break;
    body(std::integral_constant<int, 1>{});
    if (item >= nitems) break;
  }
}

template <int HD, int NKT>
hipError_t launch_fwd_pers(const bf16_t* qkv, bf16_t* o, float* lse, int B, int N, int H, int hd, float scale, int nq,
                           hipStream_t s) {
  static_assert((size_t)6 * NKT * 16 * HD * 2 <= 160 * 1024, "LDS budget");
  int cus = 256;
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) {
      int n = 0;
      if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0) cus = n;
    }
  }
  const int items = B * H;
  const int grid = items < cus ? items : cus;
  hipLaunchKernelGGL((attn_fwd_pers_kernel<HD, NKT>), dim3(grid), dim3(fp_nw<NKT> * 64), 0, s, qkv, o, lse, items, N, H, hd,
                     scale, nq);
  return hipGetLastError();
}

}  // namespace

// whether the persistent forward takes (N, head width): both K | V | Q slots fit the LDS
bool vit_attn_fwd_pers_ok(int N, int hd) {
  if (hd > 64) return false;
  const int HD = hd <= 32 ? 32 : 64;
  const int np = (N + 15) / 16 * 16;
  return (size_t)6 * np * HD * 2 <= 160 * 1024;
}

hipError_t vit_attn_fwd_pers(const void* qkv, void* o, float* lse, int B, int N, int H, int hd, float scale, int nq,
                             hipStream_t s) {
  const bf16_t* q = (const bf16_t*)qkv;
  bf16_t* out = (bf16_t*)o;
  const int nkt = (N + 15) / 16;
  if (!vit_attn_fwd_pers_ok(N, hd)) return hipErrorInvalidValue;
  if (hd <= 32) {
    switch (nkt) {
#define C(n) \
  case n: return launch_fwd_pers<32, n>(q, out, lse, B, N, H, hd, scale, nq, s);
      C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9) C(10) C(11) C(12) C(13) C(14) C(15) C(16) C(17) C(18) C(19) C(20)
#undef C
    }
  } else {
    switch (nkt) {
#define C(n) \
  case n: return launch_fwd_pers<64, n>(q, out, lse, B, N, H, hd, scale, nq, s);
      C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9) C(10) C(11) C(12) C(13)
#undef C
    }
  }
  return hipErrorInvalidValue;
}
