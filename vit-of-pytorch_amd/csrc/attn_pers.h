// Helpers of the persistent attention kernels (attention_bwd.hip: backward; attention_fwd_pers.hip: forward):
// whole-image LDS-DMA into swizzled [NP][HD] images, wave-uniform descriptors, a barrier for LDS hand-offs.
#pragma once
#include "attn_common.h"

namespace vit_attn {

// a pointer every lane holds the same value of, moved to SGPRs (the buffer descriptor of an LDS-DMA must be
// wave-uniform: from VGPRs hipcc wraps each DMA in a waterfall loop)
template <class T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const unsigned long long u = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u), hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  return (T*)(((unsigned long long)hi << 32) | lo);
}

// Workgroup barrier for LDS hand-offs only. __syncthreads() also waits vmcnt(0) (global-store visibility),
// which would stall every wave on the LDS-DMA prefetches in flight; LDS-DMA completion is handled explicitly
// (each wave drains its own vmcnt before the item-start barrier).
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// s_waitcnt vmcnt(N) (0 <= N <= 63; lgkmcnt / expcnt left alone). vmcnt retires a wave's vector memory
// operations in issue order, so with N = the number of stores issued after a wave's last LDS-DMA the wait
// covers that DMA and never the stores' own round trip.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt(0x0F70 | (N & 15) | ((N >> 4) << 14));
}

// the lane index, recomputed where it is used (opaque to CSE): lane-derived offsets of a later phase are
// rebuilt from it instead of being kept live (and spilled) across the register-heavy stage before it
__device__ __forceinline__ int lane_now() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// Buffer descriptor over rows [r0, N) of a [rows][stride] bf16 block based at `base` (row 0), up to column hd of
// row N - 1: loads past it read zero, stores past it are dropped, so padded rows need no per-lane branch.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const bf16_t* base, long stride, int r0, int N, int hd) {
  const long rec = ((long)(N - 1 - r0) * stride + hd) * 2;
  return make_rsrc(uniform_ptr(base + (long)r0 * stride), r0 < N && rec > 0 ? (uint32_t)rec : 0u);
}
__device__ __forceinline__ void st_b64(__amdgpu_buffer_rsrc_t r, int off, const uint2& v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, v), r, off, 0, 0);
}

// LDS-DMA of image rows [0, rows) (rows >= N land as zeros) of two [N][stride] bf16 blocks (A, B: 1-KiB pieces, 64 lanes x 16 B, contiguous
// in LDS) into their swizzled [NP][HD] LDS images; pieces are dealt round-robin to the waves from `first`.
// Each piece gets its own (scalar) descriptor based at its first row, so every piece uses the same one
// lane-offset VGPR (per-piece offsets get spilled, and hipcc then waits vmcnt(0) on each reload, i.e. on
// every earlier piece); the record count clips rows past N and columns past hd of row N - 1 to zero.
// nwv = 1: this wave issues every piece (first ignored).
template <int HD>
__device__ __forceinline__ void dma_pair(lds_t* imga, const bf16_t* basea, long stridea, lds_t* imgb,
                                         const bf16_t* baseb, long strideb, int rows, int N, int hd, int first,
                                         int wave, int lane, int nwv = 8) {
  constexpr int RPP = 1024 / (HD * 2);  // image rows per piece
  constexpr int CPR = HD / 8;           // 16-B chunks per row
  static_assert(RPP % 8 == 0, "the swizzle period divides a piece");
  const int npc = (rows + RPP - 1) / RPP;  // pieces per image
  const bf16_t* ba = uniform_ptr(basea);
  const bf16_t* bb = uniform_ptr(baseb);
  const int lr = lane / CPR, pc = lane % CPR;
  const int ch = pc ^ aswz<HD>(lr);  // row bits 1..2 of q * RPP + lr are those of lr
  const bool colok = ch * 8 < hd;
  const int offa = colok ? (int)(lr * stridea * 2 + ch * 16) : 0x40000000;
  const int offb = colok ? (int)(lr * strideb * 2 + ch * 16) : 0x40000000;
  int p = nwv == 1 ? 0 : wave - first;
  if (p < 0) p += nwv;
  for (; p < 2 * npc; p += nwv) {
    const bool isb = p >= npc;
    const int q = isb ? p - npc : p;
    const long stride = isb ? strideb : stridea;
    const long shift = (long)q * RPP * stride;  // elements
    const long rec = (((long)(N - 1) * stride + hd) - shift) * 2;
    const __amdgpu_buffer_rsrc_t r = make_rsrc((isb ? bb : ba) + shift, rec > 0 ? (uint32_t)rec : 0u);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (isb ? imgb : imga) + q * 1024, 16, isb ? offb : offa, 0, 0, 0);
  }
}

// LDS-DMA of n (<= NP) consecutive floats (an item's lse row) into dst; past n reads zero
template <int NP>
__device__ __forceinline__ void dma_floats(lds_t* dst, const float* src, int n, int wave, int lane, bool all = false) {
  constexpr int PCS = (NP * 4 + 1023) / 1024;
  const __amdgpu_buffer_rsrc_t r = make_rsrc(uniform_ptr(src), (uint32_t)n * 4);
  if (all) {
#pragma unroll
    for (int k = 0; k < PCS; ++k)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst + k * 1024, 16, k * 1024 + lane * 16, 0, 0, 0);
  } else if (wave < PCS) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst + wave * 1024, 16, wave * 1024 + lane * 16, 0, 0, 0);
  }
}

// LDS-DMA of image rows [0, rows) of one [N][stride] bf16 block into its swizzled [NP][HD] LDS image (as dma_pair)
template <int HD>
__device__ __forceinline__ void dma_image(lds_t* img, const bf16_t* base, long stride, int rows, int N, int hd,
                                          int first, int wave, int lane, int nwv = 8) {
  constexpr int RPP = 1024 / (HD * 2);
  constexpr int CPR = HD / 8;
  static_assert(RPP % 8 == 0, "the swizzle period divides a piece");
  const int npc = (rows + RPP - 1) / RPP;
  const bf16_t* b = uniform_ptr(base);
  const int lr = lane / CPR, pc = lane % CPR;
  const int ch = pc ^ aswz<HD>(lr);
  const int off = ch * 8 < hd ? (int)(lr * stride * 2 + ch * 16) : 0x40000000;
  int p = wave - first;
  if (p < 0) p += nwv;
  for (; p < npc; p += nwv) {
    const long shift = (long)p * RPP * stride;
    const long rec = (((long)(N - 1) * stride + hd) - shift) * 2;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(make_rsrc(b + shift, rec > 0 ? (uint32_t)rec : 0u), img + p * 1024, 16,
                                             off, 0, 0, 0);
  }
}

}  // namespace vit_attn
