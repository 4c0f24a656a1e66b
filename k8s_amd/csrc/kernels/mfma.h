// MFMA / LDS building blocks shared by the gfx950 matrix kernels (gemm.hip, attention.hip).
//
//  * v_mfma_f32_16x16x32_bf16: A[16 rows][32 k] x B[32 k][16 cols] (+)= C[16][16] fp32. Operand
//    lane map (both operands): lane l holds row/col (l & 15) and k = 8 * (l >> 4) + j, j = 0..7.
//    Result lane map: col = l & 15, rows 4 * (l >> 4) + r, r = 0..3 (4 fp32 per lane).
//    The k order inside one MFMA is free as long as both operands agree -- the attention kernels
//    use that to consume the result of one MFMA as the operand of the next without a shuffle.
//  * global_load_lds: 16 B per lane straight into LDS at (wave-uniform base + lane * 16); the LDS
//    image is lane-linear, so swizzles are applied to the per-lane SOURCE address and the same XOR
//    on the read.
//  * K-major tile [rows][64 k] (128-B rows): 16-B chunk c of row r stored at c ^ ((r >> 1) & 7)
//    -> conflict-free ds_read_b128 fragment reads (frag_kmajor).
//  * MN-major tile [k rows][128 mn] (256-B rows): 16-B unit u of k-row r stored at u ^ mn_swz(r)
//    -> ds_read_b64_tr_b16 transposed reads (4 k x 16 mn per 16 lanes).
#pragma once
#include "common.h"

namespace k8s_amd {

typedef __attribute__((ext_vector_type(8))) __bf16 mfma_bf16x8;
typedef __attribute__((ext_vector_type(4))) short short4_t;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) short4_t lds_short4;

__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (lds_void*)lds_base, 16, 0, 0);
}

__device__ __forceinline__ int mn_swz(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }

__device__ __forceinline__ f32x4_t mfma16(const mfma_bf16x8& a, const mfma_bf16x8& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// operand fragment of a K-major [rows][64 k] tile: row rb + (lane & 15), k = kk*32 + 8*(lane>>4) .. +7
__device__ __forceinline__ mfma_bf16x8 frag_kmajor(const char* tile, int rb, int kk, int lane) {
  const int row = rb + (lane & 15);
  const int c = kk * 4 + (lane >> 4);
  const bf16x8_t v = *reinterpret_cast<const bf16x8_t*>(tile + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
  return __builtin_bit_cast(mfma_bf16x8, v);
}

// 4 bf16 of one LDS column, transposed across 16 lanes (see ds_read_b64_tr_b16)
__device__ __forceinline__ short4_t tr16(const char* addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(addr));
}

// the same from an LDS-address-space base and a byte offset: pointer arithmetic in address space 3, so a constant part
// of the offset can fold into the instruction's 16-bit offset field (the generic-pointer form adds it in VALU)
typedef __attribute__((address_space(3))) char lds_char;
__device__ __forceinline__ const lds_char* lds_ptr(const void* p) {
  return (const lds_char*)(p);
}
__device__ __forceinline__ short4_t tr16l(const lds_char* base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(base + off));
}

// ds_read_b64_tr_b16 as inline asm. hipcc (ROCm 7.2) cannot prove that the builtin's read does not alias an
// in-flight global_load_lds into the same LDS array and puts `s_waitcnt vmcnt(0)` in front of it, which drains a
// counted LDS-DMA pipeline every K step (seen in the .s of gemm256r / wgrad_stream). The asm form is invisible to
// that analysis: the caller's own vmcnt + barrier protocol orders it after the DMA, and its destination is not
// ready until a following lds_tie() wait names it (cdna_hip_programming.md §5.7 item 1, form ii).
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}
__device__ __forceinline__ void tr16_asm(short4_t& r, const char* addr) {
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(lds_addr(addr)));
}
// s_waitcnt lgkmcnt(0) that every listed register depends on (8 per statement; later statements after the wait)
#define K8S_LDS_TIE8(w, a, b, c, d, e, f, g, h) \
  asm volatile(w : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h))

// Sum over each 16-lane DPP row (lanes 16q .. 16q+15); every lane of the row gets the total. Four DPP adds
// (quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror) instead of four ds_bpermute round trips
// through the LDS crossbar, which is what __shfl_xor compiles to.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_mov<0xB1>(v);
  v += dpp_mov<0x4E>(v);
  v += dpp_mov<0x141>(v);
  v += dpp_mov<0x140>(v);
  return v;
}

__device__ __forceinline__ mfma_bf16x8 join8(short4_t lo, short4_t hi) {
  bf16x8_t v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(mfma_bf16x8, v);
}

__device__ __forceinline__ mfma_bf16x8 pack8(const float (&lo)[4], const float (&hi)[4]) {
  bf16x8_t v;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = (short)f2bf(lo[j]);
    v[4 + j] = (short)f2bf(hi[j]);
  }
  return __builtin_bit_cast(mfma_bf16x8, v);
}

}  // namespace k8s_amd
