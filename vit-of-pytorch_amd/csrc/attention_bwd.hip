// Attention backward, persistent single-load form (head widths up to 64, N up to 208 at hd 64).
//
// Replaces the autograd backward of SelfAttention's core (reference src/model.py:90-97).
//
// One 8-wave workgroup per CU walks (image, head) items. Every byte of Q, K, V, dO and lse leaves HBM
// once per item, always by LDS-DMA (buffer_load ... lds) issued one phase ahead, and dQ | dK | dV are
// written once:
//   Q, dO, lse  into the idle one of two Q / dO slots at the start of the previous item;
//   K, V        into the single K / V slot once the previous item's stage 2 has its K / V rows in registers.
// Nothing is prefetched into registers, so no load is pending across the register-heavy stages (an
// in-flight register load under full register pressure made hipcc split its live range and wait vmcnt(0)
// inside stage 2's loop).
// Per item:
//   stage 1  each wave owns 16-query strips: S^T = K Q^T and dP^T = V dO^T for ALL keys stay in
//            registers, so delta_q = sum_j P_qj dP_qj is exact (not rowsum(dO * O) of the bf16 O: see
//            attention.hip), dS = P (dP - delta) and dQ = dS K come out of the same pass (K^T by
//            ds_read_b64_tr_b16);
//   stage 2  each wave owns one pair of 16-key tiles, K / V rows taken from the images into registers;
//            S, dP recomputed against the Q / dO images, dV = P^T dO, dK = dS^T Q accumulated in
//            registers (no atomics: deterministic);
//   bias     per-wave column sums of dQ, dK, dV (DPP row sums) -> row (b, wave) of bias_partial[b][PB_NW][3 D]
//            (q|k|v bias-gradient partials; no cross-wave step, so no barrier: the column reduction that
//            finishes the bias gradients sums the PB_NW rows of each image).
// LDS: K / V images, Q / dO slot 0, Q / dO slot 1 ([NP][HD] bf16, NP = 16 * ceil(N / 16), 16-B-chunk XOR
// swizzle of attn_common.h), lse slot 0 / 1 (whole 1-KiB DMA pieces) and delta rows (162 KB at N = 197, hd 64). Separate LDS objects per slot and a slot-templated item body: hipcc then proves that an
// in-flight LDS-DMA into one slot cannot alias the accesses to another and inserts no vmcnt wait for it.
#include "attn_pers.h"
#include <type_traits>

namespace {
using namespace vit_attn;

constexpr int PB_NW = 8;

#ifdef VIT_ATTN_STAMPS
// DIAGNOSTIC build only (make ... EXTRA=-DVIT_ATTN_STAMPS): s_memtime stamps of workgroup 0's waves 0 and
// VIT_STAMP_WAVE2 (default 7), first 4 items, 8 points per item; read back with vit_attn_stamps()
#ifndef VIT_STAMP_WAVE2
#define VIT_STAMP_WAVE2 7
#endif
__device__ unsigned long long g_attn_stamps[2][4][8];
#define STAMP(k)                                                                                            \
  do {                                                                                                      \
    if (blockIdx.x == 0 && (wave == 0 || wave == VIT_STAMP_WAVE2) && it < 4) {                                            \
      unsigned long long t_;                                                                                \
      __builtin_amdgcn_sched_barrier(0);                                                                    \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                            \
      __builtin_amdgcn_sched_barrier(0);                                                                    \
      if (lane == 0) g_attn_stamps[wave == VIT_STAMP_WAVE2][it][k] = t_;                                                  \
    }                                                                                                       \
  } while (0)
// sub-phases of the wave's first strip of each item (stage 1)
__device__ unsigned long long g_attn_stamps2[2][4][8];
#define STAMP1(k)                                                                                           \
  do {                                                                                                      \
    if (blockIdx.x == 0 && (wave == 0 || wave == VIT_STAMP_WAVE2) && it < 4 && qt == wave) {                              \
      unsigned long long t_;                                                                                \
      __builtin_amdgcn_sched_barrier(0);                                                                    \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                          \
      __builtin_amdgcn_sched_barrier(0);                                                                    \
      if (lane == 0) g_attn_stamps2[wave == VIT_STAMP_WAVE2][it][k] = t_;                                                 \
    }                                                                                                       \
  } while (0)
#else
#define STAMP(k) \
  do {           \
  } while (0)
#define STAMP1(k) \
  do {            \
  } while (0)
#endif

template <int HD, int NKT>
__global__ void __launch_bounds__(PB_NW * 64, 1) attn_bwd_pers_kernel(const bf16_t* __restrict__ qkv,
                                                                     const bf16_t* __restrict__ dout,
                                                                     const float* __restrict__ lse,
                                                                     bf16_t* __restrict__ dqkv,
                                                                     float* __restrict__ bias_partial, int nitems, int N,
                                                                     int H, int hd, float scale, int nq) {
  constexpr int NW = PB_NW;
  constexpr int NP = NKT * 16;
  constexpr int IMG = NP * HD * 2;
  constexpr int KK = HD / 32;
  constexpr int T = ImgLane<HD>::TILE;
  constexpr int LSEB = (NP * 4 + 1023) / 1024 * 1024;  // lse slot bytes (whole DMA pieces)
  __shared__ __attribute__((aligned(16))) char kv_s[2 * IMG];   // K | V images
  __shared__ __attribute__((aligned(16))) char qo0_s[2 * IMG];  // Q | dO images, slot 0
  __shared__ __attribute__((aligned(16))) char qo1_s[2 * IMG];  // Q | dO images, slot 1
  __shared__ __attribute__((aligned(16))) char ls0_s[LSEB];      // lse rows (natural log), slot 0
  __shared__ __attribute__((aligned(16))) char ls1_s[LSEB];      // lse rows, slot 1
  __shared__ __attribute__((aligned(16))) float dlt_s[NP];       // delta rows of the item
  lds_t* const Ki = (lds_t*)kv_s;
  lds_t* const Vi = Ki + IMG;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, i = lane & 15;
  const ImgLane<HD> L(lane);
  const int D = H * hd;
  const long rs = 3L * D;
  const float c = scale * LOG2E;
  const int npair = (N + 31) / 32;                   // pairs of 16-row tiles holding valid rows
  const bool last_half = (2 * npair - 1) * 16 >= N;  // the last pair's second tile is wholly padding
  // queries [0, nq) carry a gradient (nq < N: the last layer's cls rows); their 32-row pairs are processed
  // and only their Q / dO rows are loaded
  const int nqa = min(N, (nq + 31) / 32 * 32);
  const int npair_q = (nqa + 31) / 32;
  const int nqt = (N + 15) / 16;  // == NKT
  const int qrows = min(NP, 32 * npair_q);
  const int offs = (int)(i * rs * 2) + g * 8;  // 8-B output chunk: row i, columns 16 dt + 4 g ..

  int item = blockIdx.x;
  if (item >= nitems) return;
  auto qkv_of = [&](int it_) { return qkv + (long)(it_ / H) * N * rs + (long)(it_ % H) * hd; };
  auto dout_of = [&](int it_) { return dout + (long)(it_ / H) * N * D + (long)(it_ % H) * hd; };
  // Q / dO / lse of item it_ into a Q / dO slot (waves 0.. take the pieces; the lse piece goes to the last)
  auto dma_qo = [&](lds_t* qo, lds_t* ls, int it_, bool single) {
    dma_floats<NP>(ls, lse + (long)it_ * N, N, wave, lane, single);
    dma_pair<HD>(qo, qkv_of(it_), rs, qo + IMG, dout_of(it_), D, qrows, N, hd, 0, wave, lane, single ? 1 : NW);
  };
  // N <= 16 * NKT leaves at most (16 NKT + 31) / 32 key pairs for stage 2: below NW the last wave has none,
  // and it alone issues the next item's Q / dO / lse DMA during stage 2 instead of every wave at the start
  // of the item (where ~7 DMAs per wave cost 2 500-4 000 cycles of stage 1: attention stamps, round 3)
  constexpr bool IDLE_LAST = (NKT * 16 + 31) / 32 < NW;
  auto dma_kv = [&](int it_) {
    const bf16_t* bq = qkv_of(it_);
    // all NP rows: the padding rows N.. of the images must be zeros (the last key tile reads them)
    dma_pair<HD>(Ki, bq + D, rs, Vi, bq + 2 * D, rs, NP, N, hd, 3, wave, lane);
  };
  // ---- prologue: everything of the first item
  dma_kv(item);
  dma_qo((lds_t*)qo0_s, (lds_t*)ls0_s, item, false);

  int it = 0;
  auto body = [&](auto slot) {
    constexpr int SLOT = decltype(slot)::value;
    lds_t* const Qi = (lds_t*)(SLOT ? qo1_s : qo0_s);
    lds_t* const Oi = Qi + IMG;
    float* const lse_s = reinterpret_cast<float*>(SLOT ? ls1_s : ls0_s);
    lds_t* const Qn = (lds_t*)(SLOT ? qo0_s : qo1_s);
    lds_t* const Ln = (lds_t*)(SLOT ? ls0_s : ls1_s);
    const int b = item / H, h = item % H;
    bf16_t* const dqb = dqkv + (long)b * N * rs + (long)h * hd;
    const int next = __builtin_amdgcn_readfirstlane(item + (int)gridDim.x);

    // (a) this item's K / V, Q / dO, lse landed (every wave drains its own DMAs, then the barrier), and
    // every wave is past the previous item's stage 2 / bias sums (the last readers of the other slot)
    STAMP(0);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) (a builtin: hipcc's own wait tracking sees it)
    STAMP(1);
    lds_barrier();
    STAMP(2);
    // (b) the next item's Q / dO / lse into the other slot
    if (!IDLE_LAST && next < nitems) dma_qo(Qn, Ln, next, false);
#ifdef VIT_ATTN_STAMPS
    {
      const int qt = wave;  // (STAMP1's first-strip filter)
      STAMP1(7);
    }
#endif

    // ---- stage 1: delta, dS, dQ per 16-query strip ----
    float bq16[16];  // the wave's dQ column partials: [4 dt + r] for column 16 dt + 4 g + r (summed over lanes i later)
#pragma unroll
    for (int k = 0; k < 16; ++k) bq16[k] = 0.f;
    for (int qt = wave; qt < nqt; qt += NW) {
      const int q = qt * 16 + i;
      const __amdgpu_buffer_rsrc_t rdq = rows_rsrc(dqb, rs, qt * 16, N, hd);
      if (qt * 16 >= nqa) {  // no gradient reaches these queries: dQ = 0 (delta unused: stage 2 skips them)
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt)
          if (dt * 16 < hd) st_b64(rdq, offs + dt * 32, uint2{0u, 0u});
        continue;
      }
      STAMP1(0);
      v8bf qf[KK], df[KK];
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        qf[kk] = __builtin_bit_cast(v8bf, lds_ld<v8s>(Qi + qt * T + L.row[kk]));
        df[kk] = __builtin_bit_cast(v8bf, lds_ld<v8s>(Oi + qt * T + L.row[kk]));
      }
      const float ls = q < N ? lse_s[q] * LOG2E : 1e30f;  // padded queries: P = 2^-1e30 = 0
      // stage 2 reads the strip's lse in log2 units (one fma per score there); nothing else reads this slot's
      // lse before the stage 1 / stage 2 barrier
      if (g == 0) lse_s[q] = ls;
      STAMP1(1);
      v4f P[NKT], DP[NKT];
      float dlr[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        v4f st = {0.f, 0.f, 0.f, 0.f}, dpt = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          st = mfma(__builtin_bit_cast(v8bf, lds_ld<v8s>(Ki + kt * T + L.row[kk])), qf[kk], st);
          dpt = mfma(__builtin_bit_cast(v8bf, lds_ld<v8s>(Vi + kt * T + L.row[kk])), df[kk], dpt);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = st[r] * c - ls;
          float pv;
          if (kt == NKT - 1) {
            // the last tile may hold padded keys (zero K / V rows: dP = 0, nothing added to delta, and
            // their dS meets zero K rows in dQ): only the exponent is clamped so that P stays finite
            // whatever the query's LSE; nan_of keeps a NaN score visible (v_min returns the non-NaN operand)
            pv = ex2(fminf(e, 0.f) + nan_of(e));
          } else {
            pv = ex2(e);
          }
          P[kt][r] = pv;
          dlr[r] += pv * dpt[r];
        }
        DP[kt] = dpt;
      }
      STAMP1(2);
      float dl = (dlr[0] + dlr[1]) + (dlr[2] + dlr[3]);
      dl += __shfl_xor(dl, 16, 64);
      dl += __shfl_xor(dl, 32, 64);
      if (q >= N) dl = 0.f;
      if (g == 0) dlt_s[q] = dl;
      STAMP1(3);
      v4f dq[HD / 16];
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) dq[dt] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKT / 2; ++ks) {
        v4f d0, d1;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          d0[r] = P[2 * ks][r] * (DP[2 * ks][r] - dl);
          d1[r] = P[2 * ks + 1][r] * (DP[2 * ks + 1][r] - dl);
        }
        const v8bf bD = pack8(d0, d1);
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) {
          v8s kt8;
          kt8.lo = lds_tr(Ki + 2 * ks * T + L.tr[dt]);
          kt8.hi = lds_tr(Ki + (2 * ks + 1) * T + L.tr[dt]);
          dq[dt] = mfma(__builtin_bit_cast(v8bf, kt8), bD, dq[dt]);
        }
      }
      if constexpr (NKT % 2 == 1) {
        v4f d0;
#pragma unroll
        for (int r = 0; r < 4; ++r) d0[r] = P[NKT - 1][r] * (DP[NKT - 1][r] - dl);
        const v4s bD = pack4(d0);
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) dq[dt] = mfma16_add(lds_tr(Ki + (NKT - 1) * T + L.tr[dt]), bD, dq[dt]);
      }
      STAMP1(4);
      {
        uint2 pk[HD / 16];
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) pk[dt] = pack4bf(dq[dt], scale);
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt)
          if (dt * 16 < hd) st_b64(rdq, offs + dt * 32, pk[dt]);
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) keep_live2(pk[dt]);
      }
      if (bias_partial) {  // padded queries: dS = 0
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt)
#pragma unroll
          for (int r = 0; r < 4; ++r) bq16[dt * 4 + r] += dq[dt][r];
      }
    }
    // lane 16 g + 4 dt + r: the wave's sum of dQ column 16 dt + 4 g + r
    const float bq1 = bias_partial ? reduce16(bq16, i) : 0.f;
    STAMP(3);
    lds_barrier();  // delta complete
    STAMP(4);

    // ---- stage 2: dK, dV per pair of 16-key tiles ----
    const ImgLane<HD> L2(lane_now());  // (rebuilt: see lane_now)
    const int kp = wave;
    v8bf kf[2][KK], vf[2][KK];
    const bool have_pair = kp < npair;
    const bool t1_valid = (2 * kp + 1) * 16 < N;  // the pair's second tile holds a valid key
    if (have_pair) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          const bool ok = t == 0 || t1_valid;
          kf[t][kk] = ok ? __builtin_bit_cast(v8bf, lds_ld<v8s>(Ki + (2 * kp + t) * T + L2.row[kk])) : v8bf{};
          vf[t][kk] = ok ? __builtin_bit_cast(v8bf, lds_ld<v8s>(Vi + (2 * kp + t) * T + L2.row[kk])) : v8bf{};
        }
    }
    // every wave has its K / V rows: the next item's K / V into the images, landing during stage 2
    lds_barrier();  // (its lgkmcnt(0): this wave's K / V reads are back)
    if (next < nitems) dma_kv(next);
    if (IDLE_LAST && wave == NW - 1 && next < nitems) dma_qo(Qn, Ln, next, true);  // (b) of IDLE_LAST
    STAMP(7);
    float bk4[HD / 16][4], bv4[HD / 16][4];
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) bk4[dt][r] = bv4[dt][r] = 0.f;
    if (have_pair) {
      v4f dv[2][HD / 16], dk[2][HD / 16];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) dv[t][dt] = dk[t][dt] = v4f{0.f, 0.f, 0.f, 0.f};
      const bool kv0 = (2 * kp) * 16 + i < N, kv1 = (2 * kp + 1) * 16 + i < N;
      // P and dS of the (key pair, query tile 2 qs + u) products, u < NU; MASK: the pair holds padded keys
      // (only the last pair: their P forced to 0). lse_s holds log2 units since stage 1 (padded queries 1e30).
      // NTK: key tiles of the pair that hold a valid key (1: the last pair's second tile is wholly padding, and
      // its products are skipped instead of computed and masked to zero)
      auto scores = [&](int qs, auto nu, auto maskc, auto ntk, v4f (&Pm)[2][2], v4f (&DS)[2][2]) __attribute__((always_inline)) {
        constexpr int NU = decltype(nu)::value;
        constexpr bool MASK = decltype(maskc)::value;
        constexpr int NTK = decltype(ntk)::value;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int qt = 2 * qs + u;
          v8bf qr[KK], orow[KK];
#pragma unroll
          for (int kk = 0; kk < KK; ++kk) {
            qr[kk] = __builtin_bit_cast(v8bf, lds_ld<v8s>(Qi + qt * T + L2.row[kk]));
            orow[kk] = __builtin_bit_cast(v8bf, lds_ld<v8s>(Oi + qt * T + L2.row[kk]));
          }
          // padded queries (rows >= N) have zero Q and dO rows and lse 1e30: P = 0
          const v4f lq = *reinterpret_cast<const v4f*>(lse_s + qt * 16 + 4 * g);
          const v4f dq4 = *reinterpret_cast<const v4f*>(dlt_s + qt * 16 + 4 * g);
#pragma unroll
          for (int t = 0; t < NTK; ++t) {
            v4f sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) {
              sv = mfma(qr[kk], kf[t][kk], sv);
              dp = mfma(orow[kk], vf[t][kk], dp);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float p = ex2(fmaf(sv[r], c, -lq[r]));
              if constexpr (MASK) p = (t == 0 ? kv0 : kv1) ? p : 0.f;
              Pm[t][u][r] = p;
              DS[t][u][r] = p * (dp[r] - dq4[r]);
            }
          }
        }
      };
      struct Packed {
        v8bf bP0, bP1, bD0, bD1;
      };
      // a whole query-tile pair: its products as the B operands of dV / dK (front), then the 16 MFMAs (back)
      auto front = [&](int qs, auto maskc, auto ntk) __attribute__((always_inline)) {
        constexpr int NTK = decltype(ntk)::value;
        v4f Pm[2][2], DS[2][2];  // [key tile][query tile]
        scores(qs, std::integral_constant<int, 2>{}, maskc, ntk, Pm, DS);
        Packed o;
        o.bP0 = pack8(Pm[0][0], Pm[0][1]);
        o.bD0 = pack8(DS[0][0], DS[0][1]);
        if constexpr (NTK == 2) {
          o.bP1 = pack8(Pm[1][0], Pm[1][1]);
          o.bD1 = pack8(DS[1][0], DS[1][1]);
        }
        return o;
      };
      auto back = [&](int qs, const Packed& o, auto ntk) __attribute__((always_inline)) {
        constexpr int NTK = decltype(ntk)::value;
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) {
          v8s ot, qtr;
          ot.lo = lds_tr(Oi + 2 * qs * T + L2.tr[dt]);
          ot.hi = lds_tr(Oi + (2 * qs + 1) * T + L2.tr[dt]);
          qtr.lo = lds_tr(Qi + 2 * qs * T + L2.tr[dt]);
          qtr.hi = lds_tr(Qi + (2 * qs + 1) * T + L2.tr[dt]);
          dv[0][dt] = mfma(__builtin_bit_cast(v8bf, ot), o.bP0, dv[0][dt]);
          dk[0][dt] = mfma(__builtin_bit_cast(v8bf, qtr), o.bD0, dk[0][dt]);
          if constexpr (NTK == 2) {
            dv[1][dt] = mfma(__builtin_bit_cast(v8bf, ot), o.bP1, dv[1][dt]);
            dk[1][dt] = mfma(__builtin_bit_cast(v8bf, qtr), o.bD1, dk[1][dt]);
          }
        }
      };
      // the query pair's second tile wholly padding (past the images): tile 2 qs alone, the 16-deep MFMA
      auto half_unit = [&](int qs, auto maskc, auto ntk) __attribute__((always_inline)) {
        constexpr int NTK = decltype(ntk)::value;
        v4f Pm[2][2], DS[2][2];
        scores(qs, std::integral_constant<int, 1>{}, maskc, ntk, Pm, DS);
        const v4s bP0 = pack4(Pm[0][0]), bD0 = pack4(DS[0][0]);
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) {
          const v4s ot = lds_tr(Oi + 2 * qs * T + L2.tr[dt]);
          const v4s qtr = lds_tr(Qi + 2 * qs * T + L2.tr[dt]);
          dv[0][dt] = mfma16_add(ot, bP0, dv[0][dt]);
          dk[0][dt] = mfma16_add(qtr, bD0, dk[0][dt]);
          if constexpr (NTK == 2) {
            const v4s bP1 = pack4(Pm[1][0]), bD1 = pack4(DS[1][0]);
            dv[1][dt] = mfma16_add(ot, bP1, dv[1][dt]);
            dk[1][dt] = mfma16_add(qtr, bD1, dk[1][dt]);
          }
        }
      };
      const int nfull = last_half && npair_q == npair ? npair_q - 1 : npair_q;
      // software-pipelined over query pairs: the products of pair qs + 1 (LDS reads, 16 MFMAs, the exp / dS
      // VALU) sit in one basic block with pair qs's dV / dK MFMAs, so one wave keeps both pipes busy
      auto run = [&](auto maskc, auto ntk) __attribute__((always_inline)) {
        if (nfull > 0) {
          Packed cur = front(0, maskc, ntk);
          for (int qs = 0; qs + 1 < nfull; ++qs) {
            const Packed nxt = front(qs + 1, maskc, ntk);
            back(qs, cur, ntk);
            cur = nxt;
          }
          back(nfull - 1, cur, ntk);
        }
        if (nfull < npair_q) half_unit(nfull, maskc, ntk);
      };
      // the last pair holds the padded keys (masked); when its second tile is wholly padding (N <= 16 (2 kp + 1))
      // only the first tile's products are computed: that wave had ~25% more stage-2 work than any other
      // (stamps: 18.6 k against 15 k cycles at N = 197) and set the item's pace
      if (kp == npair - 1) {
        if (t1_valid) run(std::true_type{}, std::integral_constant<int, 2>{});
        else run(std::true_type{}, std::integral_constant<int, 1>{});
      } else {
        run(std::false_type{}, std::integral_constant<int, 2>{});
      }
      uint2 pk[2][HD / 16], pv[2][HD / 16];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) {
          pk[t][dt] = pack4bf(dk[t][dt], scale);
          pv[t][dt] = pack4bf(dv[t][dt], 1.0f);
        }
#pragma unroll
      for (int t = 0; t < 2; ++t) {  // rows past N are dropped by the descriptors
        const __amdgpu_buffer_rsrc_t rk = rows_rsrc(dqb + D, rs, (2 * kp + t) * 16, N, hd);
        const __amdgpu_buffer_rsrc_t rv = rows_rsrc(dqb + 2 * D, rs, (2 * kp + t) * 16, N, hd);
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt)
          if (dt * 16 < hd) {
            st_b64(rk, offs + dt * 32, pk[t][dt]);
            st_b64(rv, offs + dt * 32, pv[t][dt]);
          }
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) {
          keep_live2(pk[t][dt]);
          keep_live2(pv[t][dt]);
        }
      if (bias_partial) {
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {  // invalid keys hold exact zeros (P = 0)
            bk4[dt][r] = dk[0][dt][r] + dk[1][dt][r];
            bv4[dt][r] = dv[0][dt][r] + dv[1][dt][r];
          }
      }
    }
    STAMP(5);

    // ---- bias partials: the wave's column sums of dQ, dK, dV -> its own row of bias_partial (every wave
    // writes its row, zeros when it had no strip / pair; vit_colsum_batch sums the PB_NW rows per image)
    if (bias_partial) {
      float tk[16], tv[16];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          tk[dt * 4 + r] = dt < HD / 16 ? bk4[dt][r] : 0.f;
          tv[dt * 4 + r] = dt < HD / 16 ? bv4[dt][r] : 0.f;
        }
      const float bk1 = reduce16(tk, i), bv1 = reduce16(tv, i);
      const int dcol = 16 * (i >> 2) + 4 * g + (i & 3);  // this lane's column (see reduce16)
      if (dcol < hd) {
        float* row = bias_partial + ((long)b * NW + wave) * 3 * D + h * hd + dcol;
        row[0] = bq1 * scale;
        row[D] = bk1 * scale;
        row[2 * D] = bv1;
      }
    }
    STAMP(6);
    item = __builtin_amdgcn_readfirstlane(next);  // (uniform: scalar branches and addresses)
    ++it;
  };
  while (true) {
    body(std::integral_constant<int, 0>{});
    if (item >= nitems) break;
    body(std::integral_constant<int, 1>{});
    if (item >= nitems) break;
  }
}

template <int HD, int NKT>
constexpr size_t pers_lds() {
  return (size_t)6 * NKT * 16 * HD * 2 + 2 * ((NKT * 16 * 4 + 1023) / 1024 * 1024) + NKT * 16 * 4;
}

template <int HD, int NKT>
hipError_t launch_pers(const bf16_t* qkv, const bf16_t* dout, const float* lse, bf16_t* dqkv, float* bias_partial,
                       int B, int N, int H, int hd, float scale, int nq, hipStream_t s) {
  static_assert(pers_lds<HD, NKT>() <= 160 * 1024, "LDS budget");
  auto kern = attn_bwd_pers_kernel<HD, NKT>;
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
  hipLaunchKernelGGL(kern, dim3(grid), dim3(PB_NW * 64), 0, s, qkv, dout, lse, dqkv, bias_partial, items, N, H, hd,
                     scale, nq);
  return hipGetLastError();
}

}  // namespace

// LDS bytes of the persistent backward for (N, head width), 0 when it does not apply (the two-stage
// kernel of attention.hip then runs)
size_t vit_attn_bwd_pers_lds(int N, int hd) {
  if (hd > 64) return 0;
  // stage 2 gives each wave one pair of 16-key tiles (kp = wave): keys past 32 * PB_NW would get no dK / dV
  if ((N + 31) / 32 > PB_NW) return 0;
  const int HD = hd <= 32 ? 32 : 64;
  const int np = (N + 15) / 16 * 16;
  const size_t lds = (size_t)6 * np * HD * 2 + 2 * ((np * 4 + 1023) / 1024 * 1024) + np * 4;
  return lds <= 160 * 1024 ? lds : 0;
}

#ifdef VIT_ATTN_STAMPS
extern "C" int vit_attn_stamps(unsigned long long* out) {  // 128 values: [2][wave 0 / 7][item][point]
  int e = (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_attn_stamps), sizeof(g_attn_stamps));
  if (e) return e;
  return (int)hipMemcpyFromSymbol(out + 64, HIP_SYMBOL(g_attn_stamps2), sizeof(g_attn_stamps2));
}
#endif

int vit_attn_bwd_pers_bias_rows() { return PB_NW; }

hipError_t vit_attn_bwd_pers(const void* qkv, const void* dout, const float* lse, void* dqkv, float* bias_partial,
                             int B, int N, int H, int hd, float scale, int nq, hipStream_t s) {
  const bf16_t *q = (const bf16_t*)qkv, *d = (const bf16_t*)dout;
  bf16_t* dq = (bf16_t*)dqkv;
  const int nkt = (N + 15) / 16;
  if ((N + 31) / 32 > PB_NW) return hipErrorInvalidValue;  // see vit_attn_bwd_pers_lds
  if (hd <= 32) {
    switch (nkt) {
#define C(n) \
  case n: return launch_pers<32, n>(q, d, lse, dq, bias_partial, B, N, H, hd, scale, nq, s);
      C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9) C(10) C(11) C(12) C(13) C(14) C(15) C(16)
#undef C
    }
  } else {
    switch (nkt) {
#define C(n) \
  case n: return launch_pers<64, n>(q, d, lse, dq, bias_partial, B, N, H, hd, scale, nq, s);
      C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9) C(10) C(11) C(12) C(13)
#undef C
    }
  }
  return hipErrorInvalidValue;
}
