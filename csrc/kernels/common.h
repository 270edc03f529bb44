// Shared device helpers for the gfx950 (CDNA4) kernels.
//
// Conventions (cdna_hip_programming.md §1, §6 G13):
//  * wave = 64 lanes, blocks are multiples of 64 threads;
//  * bf16 tensors are moved 16 B per lane (8 x bf16) — never scalar bf16 loads;
//  * f32 accumulation everywhere; bf16 rounding by the hardware cvt (RNE, NaN-preserving).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace llmc {

constexpr int kWave = 64;

typedef uint16_t bf16_t;  // storage type for bf16 tensors
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) short bf16x8;  // MFMA A/B fragment (8 bf16)
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

__device__ __forceinline__ float bf16_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ float bf16_to_f32(bf16_t b) { return __uint_as_float(static_cast<uint32_t>(b) << 16); }

__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(bf16_t, b);
}
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return static_cast<uint32_t>(f32_to_bf16(lo)) | (static_cast<uint32_t>(f32_to_bf16(hi)) << 16);
}

// 8 bf16 packed in a u32x4 -> 8 floats
__device__ __forceinline__ void unpack8(const u32x4& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = bf16_lo(v[i]);
    f[2 * i + 1] = bf16_hi(v[i]);
  }
}
__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = pack_bf16x2(f[2 * i], f[2 * i + 1]);
  return v;
}

// f32 += dot(bf16x2 a, bf16x2 b) in one VALU op (v_dot2_f32_bf16).
__device__ __forceinline__ float dot2_bf16(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a), __builtin_bit_cast(bf16x2_t, b), c, false);
}
__device__ __forceinline__ float dot8_bf16(const u32x4& a, const u32x4& b, float c) {
  c = dot2_bf16(a[0], b[0], c);
  c = dot2_bf16(a[1], b[1], c);
  c = dot2_bf16(a[2], b[2], c);
  c = dot2_bf16(a[3], b[3], c);
  return c;
}

template <bool NT>
__device__ __forceinline__ u32x4 load16(const void* p) {
  if constexpr (NT) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  } else {
    return *reinterpret_cast<const u32x4*>(p);
  }
}

// Load of a wave-uniform address through the scalar cache (s_load_dword, counted by lgkmcnt, so
// it does not queue behind the vector loads in flight). Read-only data only.
template <typename T>
__device__ __forceinline__ T ld_scalar(const T* p) {
  static_assert(sizeof(T) == 4, "32-bit scalar loads");
  return *reinterpret_cast<const __attribute__((address_space(4))) T*>(reinterpret_cast<uintptr_t>(p));
}

// Cross-lane exchanges without an LDS round trip. __shfl_xor lowers to ds_bpermute (an LDS access and
// an lgkmcnt wait on every step of a reduction's dependency chain); these run in the VALU:
//  * lanes (l, l ^ 32) / (l, l ^ 16): v_permlane32_swap / v_permlane16_swap of v with itself leaves
//    the pair's two values in the two results, in lane-dependent order -> for a commutative op,
//    op(r0, r1) == op(v, v[l ^ o]) bit for bit;
//  * lanes (l, l ^ 8) inside a 16-lane row: DPP row_ror:8; (l, l ^ 2) / (l, l ^ 1): DPP quad_perm.
// IEEE add and max are commutative, so each step below computes exactly the value of the shuffle
// form it replaces (same association order: the results are bit-identical).
__device__ __forceinline__ uint32_t fbits(float v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ float bitsf(uint32_t v) { return __builtin_bit_cast(float, v); }
__device__ __forceinline__ float fmax_raw(float a, float b) {  // no canonicalising v_max x, x on a and b
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// The swap as inline asm, with the 2 wait states the gfx950 hazard rule wants between a VALU write
// of either operand and the swap inside the string (what hipcc emits for the builtin; the asm keeps
// the instruction where the source puts it)
__device__ __forceinline__ void permlane_swap16(uint32_t& a, uint32_t& b) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void permlane_swap32(uint32_t& a, uint32_t& b) {
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ float xor32_add(float v) {
  uint32_t a = fbits(v), b = fbits(v);
  permlane_swap32(a, b);
  return bitsf(a) + bitsf(b);
}
__device__ __forceinline__ float xor16_add(float v) {
  uint32_t a = fbits(v), b = fbits(v);
  permlane_swap16(a, b);
  return bitsf(a) + bitsf(b);
}
__device__ __forceinline__ float xor32_max(float v) {
  uint32_t a = fbits(v), b = fbits(v);
  permlane_swap32(a, b);
  return fmax_raw(bitsf(a), bitsf(b));
}
__device__ __forceinline__ float xor16_max(float v) {
  uint32_t a = fbits(v), b = fbits(v);
  permlane_swap16(a, b);
  return fmax_raw(bitsf(a), bitsf(b));
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return bitsf(static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(fbits(v)), CTRL, 0xF, 0xF, true)));
}
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E;  // quad_perm [1,0,3,2] / [2,3,0,1]
constexpr int kDppRor8 = 0x128, kDppRor4 = 0x124;  // row_ror:8 = lane ^ 8 within a 16-lane row

// v of lane ^ M for any lane pattern (the exact __shfl_xor(v, M, 64)), in the VALU. DPP row_ror:n
// reads lane (l - n) mod 16 of the row (norm.hip lane_exchange_check_kernel: every helper against
// __shfl_xor, bit for bit, tests/test_kernels_gpu.py).
template <int M>
__device__ __forceinline__ float xor_shfl(float v, int lane) {
  static_assert(M == 1 || M == 2 || M == 4 || M == 8 || M == 16 || M == 32, "lane xor of one bit");
  if constexpr (M == 32) {
    uint32_t a = fbits(v), b = fbits(v);
    permlane_swap32(a, b);
    return bitsf(lane & 32 ? a : b);
  } else if constexpr (M == 16) {
    uint32_t a = fbits(v), b = fbits(v);
    permlane_swap16(a, b);
    return bitsf(lane & 16 ? a : b);
  } else if constexpr (M == 8) {
    return dpp_f<kDppRor8>(v);
  } else if constexpr (M == 4) {
    // both rotations under the full EXEC mask (a select over two DPP reads was lowered to two
    // EXEC-masked DPP moves, which read 0 from the masked-off source lanes): banks 0 / 2 (lanes
    // 0-3, 8-11 of each row) take ror:12 (lane + 4), banks 1 / 3 ror:4 (lane - 4), by the DPP bank mask
    const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(fbits(v)), 0x12C, 0xF, 0x5, false);
    return bitsf(static_cast<uint32_t>(__builtin_amdgcn_update_dpp(lo, static_cast<int>(fbits(v)), kDppRor4, 0xF, 0xA, false)));
  } else {
    return dpp_f<M == 2 ? kDppXor2 : kDppXor1>(v);
  }
}
// sum over the lanes l ^ {M, M/2, ..., 1}: the butterfly M, M/2, ..., 1 (every lane of the group
// ends with the group's sum)
template <int M>
__device__ __forceinline__ float xor_tree_sum(float v, int lane) {
  if constexpr (M >= 1) {
    v += xor_shfl<M>(v, lane);
    return xor_tree_sum<M / 2>(v, lane);
  } else {
    return v;
  }
}

// Full-wave reductions: the xor butterfly 32, 16, 8, 4, 2, 1. After the 32 / 16 / 8 steps every
// lane's value depends on lane % 8 only, so row_ror:4 (lane -> lane +- 4 in its row) reads the
// same value as lane ^ 4 would.
__device__ __forceinline__ float wave_sum(float v) {
  v = xor32_add(v);
  v = xor16_add(v);
  v += dpp_f<kDppRor8>(v);
  v += dpp_f<kDppRor4>(v);
  v += dpp_f<kDppXor2>(v);
  v += dpp_f<kDppXor1>(v);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
  v = xor32_max(v);
  v = xor16_max(v);
  v = fmax_raw(v, dpp_f<kDppRor8>(v));
  v = fmax_raw(v, dpp_f<kDppRor4>(v));
  v = fmax_raw(v, dpp_f<kDppXor2>(v));
  v = fmax_raw(v, dpp_f<kDppXor1>(v));
  return v;
}
// Reduction inside aligned groups of W lanes (W power of two <= 64).
template <int W>
__device__ __forceinline__ float group_sum(float v) {
  return xor_tree_sum<W / 2>(v, static_cast<int>(threadIdx.x) & 63);
}

// Block-wide sum for NT threads (NT multiple of 64, <= 1024). `red` needs NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x / kWave, l = threadIdx.x % kWave;
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / kWave; ++i) t += red[i];
  __syncthreads();
  return t;
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

// Split-KV decode attention, balanced form: a fixed grid of `gc` blocks per (sequence, kv head)
// shares the sequence's L keys evenly in 32-key units (the MFMA sub-tile): n = min(gc,
// ceil(L / min_chunk)) blocks, block c owning units [c*U/n, (c+1)*U/n) of U = ceil(L/32), so
// the grid shape (and a captured graph) is independent of L and every live block gets the same
// work to within one sub-tile. chunk_arg < 0 encodes this form (min_chunk = -chunk_arg);
// chunk_arg >= 0 is the fixed-chunk form (blocks of chunk_arg keys; VALU kernels).
__device__ __forceinline__ int decode_nsplit(int L, int gc, int chunk_arg) {
  if (chunk_arg >= 0) return (L + chunk_arg - 1) / chunk_arg;
  const int n = (L + (-chunk_arg) - 1) / (-chunk_arg);
  return n < 1 ? 1 : (n < gc ? n : gc);
}
__device__ __forceinline__ void decode_range(int L, int n, int c, int chunk_arg, int& start, int& end) {
  if (chunk_arg >= 0) {
    start = c * chunk_arg;
    end = min(start + chunk_arg, L);
    return;
  }
  const int64_t units = (L + 31) / 32;
  start = static_cast<int>(32 * (c * units / n));
  end = min(L, static_cast<int>(32 * ((c + 1) * units / n)));
}

}  // namespace llmc

#define LLMC_CHECK_LAUNCH() (void)0
