// Shared device helpers for the gfx950 (CDNA4, MI355X) recsys kernels.
//
// Storage dtypes: every activation / weight-copy kernel is templated on the
// element type T in {float, __bf16}.  Arithmetic is always fp32 (MFMA fp32
// accumulate; LN / softmax / loss statistics in fp32).  fp32 instantiations use
// the exact f32-input MFMA (v_mfma_f32_16x16x4_f32, a bitwise k-ordered fmaf
// chain) and are the parity mode; bf16 instantiations use v_mfma_f32_16x16x32_bf16.
//
// MFMA operand convention used by every kernel (16x16 output tile, 32-deep k
// chunk): lane l holds A[row = l&15][k = 8*(l>>4) + j] and B[k = 8*(l>>4) + j][col = l&15]
// for j = 0..7; the accumulator holds C[row = 4*(l>>4) + r][col = l&15], r = 0..3.
// For bf16 this is one v_mfma_f32_16x16x32_bf16; for fp32 it is eight
// v_mfma_f32_16x16x4_f32 (MFMA j consumes element j of every lane, i.e. the
// k-subset {8g + j}), so one fragment layout serves both dtypes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <algorithm>

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;

#define RS_DTYPE_F32 0
#define RS_DTYPE_BF16 1

#define RS_OK 0
#define RS_ERR_ARG 1001
#define RS_ERR_UNSUPPORTED 1002

#define WAVE 64

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(__bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ __bf16 from_f<__bf16>(float x) { return (__bf16)x; }

// ---------------------------------------------------------------- fragments
template <typename T> struct Frag;
template <> struct Frag<__bf16> { bf16x8 v; };
template <> struct Frag<float> { float v[8]; };

// 8 contiguous elements (16-B aligned for bf16, 16-B aligned pairs for f32)
__device__ __forceinline__ void frag_load_vec(Frag<__bf16>& f, const __bf16* p) {
  f.v = *reinterpret_cast<const bf16x8*>(p);
}
__device__ __forceinline__ void frag_load_vec(Frag<float>& f, const float* p) {
  float4 a = *reinterpret_cast<const float4*>(p);
  float4 b = *reinterpret_cast<const float4*>(p + 4);
  f.v[0] = a.x; f.v[1] = a.y; f.v[2] = a.z; f.v[3] = a.w;
  f.v[4] = b.x; f.v[5] = b.y; f.v[6] = b.z; f.v[7] = b.w;
}
// 8 elements with a stride
__device__ __forceinline__ void frag_load_strided(Frag<__bf16>& f, const __bf16* p, int stride) {
#pragma unroll
  for (int j = 0; j < 8; ++j) f.v[j] = p[j * stride];
}
__device__ __forceinline__ void frag_load_strided(Frag<float>& f, const float* p, int stride) {
#pragma unroll
  for (int j = 0; j < 8; ++j) f.v[j] = p[j * stride];
}
__device__ __forceinline__ void frag_zero(Frag<__bf16>& f) {
#pragma unroll
  for (int j = 0; j < 8; ++j) f.v[j] = (__bf16)0.0f;
}
__device__ __forceinline__ void frag_zero(Frag<float>& f) {
#pragma unroll
  for (int j = 0; j < 8; ++j) f.v[j] = 0.0f;
}
__device__ __forceinline__ void frag_set(Frag<__bf16>& f, int j, float x) { f.v[j] = (__bf16)x; }
__device__ __forceinline__ void frag_set(Frag<float>& f, int j, float x) { f.v[j] = x; }

__device__ __forceinline__ f32x4 mma(const Frag<__bf16>& a, const Frag<__bf16>& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mma(const Frag<float>& a, const Frag<float>& b, f32x4 c) {
#pragma unroll
  for (int j = 0; j < 8; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[j], b.v[j], c, 0, 0, 0);
  return c;
}

// ---------------------------------------------------------------- vectors
// VEC = elements per 16-byte chunk
template <typename T> struct Vec { static constexpr int N = 16 / sizeof(T); };

template <typename T>
__device__ __forceinline__ void load_chunk(float* out, const T* p);
template <>
__device__ __forceinline__ void load_chunk<float>(float* out, const float* p) {
  float4 a = *reinterpret_cast<const float4*>(p);
  out[0] = a.x; out[1] = a.y; out[2] = a.z; out[3] = a.w;
}
template <>
__device__ __forceinline__ void load_chunk<__bf16>(float* out, const __bf16* p) {
  bf16x8 a = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = (float)a[j];
}
template <typename T>
__device__ __forceinline__ void store_chunk(T* p, const float* in);
template <>
__device__ __forceinline__ void store_chunk<float>(float* p, const float* in) {
  *reinterpret_cast<float4*>(p) = make_float4(in[0], in[1], in[2], in[3]);
}
template <>
__device__ __forceinline__ void store_chunk<__bf16>(__bf16* p, const float* in) {
  bf16x8 a;
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = (__bf16)in[j];
  *reinterpret_cast<bf16x8*>(p) = a;
}

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// reduce over the 16 lanes that share (l>>4) -- i.e. over the accumulator's columns
__device__ __forceinline__ float group16_sum(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float group16_max(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Cross-lane steps without the LDS crossbar, for code that runs with ALL 64 lanes active (DPP and the permlane
// swaps read an inactive lane's register as invalid; __shfl_xor's ds_bpermute_b32 reads it regardless -- but costs
// an LDS round trip each): lane ^ 32 / ^ 16 by the gfx950 permlane swaps (the pair's two values summed in either
// order: the same bits), lane ^ 8 / ^ 4 / ^ 2 / ^ 1 by DPP row moves -- row_ror:8 IS lane ^ 8 within a 16-lane row,
// and once the lanes i, i ^ 8 agree row_ror:4 reads the value lane ^ 4 holds -- so each form returns, in every
// lane, the bits of the xor butterfly it replaces.
template <int CTRL> __device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
#define DPP_XOR1 0xB1    // quad_perm [1, 0, 3, 2]
#define DPP_XOR2 0x4E    // quad_perm [2, 3, 0, 1]
#define DPP_ROR4 0x124   // row_ror:4
#define DPP_ROR8 0x128   // row_ror:8
#define DPP_HALF_MIRROR 0x141
#define DPP_MIRROR 0x140
// v_permlane32_swap_b32 a, b: lanes 32-63 of a <-> lanes 0-31 of b; v_permlane16_swap_b32: the odd 16-lane rows of a
// <-> the even rows of b.  With a = b = v the pair (a, b) then holds, per lane, v and the value of lane ^ 32 (^ 16).
// Inline asm, two distinct registers: hipcc 7.2 folds __builtin_amdgcn_permlane*_swap(u, u) wrongly (the two
// results taken as equal: every lane wrong, tools/micro/xlane_probe.hip).  s_nop 1: the VALU-write -> permlane-read
// hazard's two wait states.
__device__ __forceinline__ void pl32_swap(unsigned& a, unsigned& b) {
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void pl16_swap(unsigned& a, unsigned& b) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ float add_xor32(float v) {
  unsigned a = __builtin_bit_cast(unsigned, v), b = a;
  pl32_swap(a, b);
  return __builtin_bit_cast(float, a) + __builtin_bit_cast(float, b);
}
__device__ __forceinline__ float add_xor16(float v) {
  unsigned a = __builtin_bit_cast(unsigned, v), b = a;
  pl16_swap(a, b);
  return __builtin_bit_cast(float, a) + __builtin_bit_cast(float, b);
}
__device__ __forceinline__ float max_xor32(float v) {
  unsigned a = __builtin_bit_cast(unsigned, v), b = a;
  pl32_swap(a, b);
  return fmaxf(__builtin_bit_cast(float, a), __builtin_bit_cast(float, b));
}
__device__ __forceinline__ float max_xor16(float v) {
  unsigned a = __builtin_bit_cast(unsigned, v), b = a;
  pl16_swap(a, b);
  return fmaxf(__builtin_bit_cast(float, a), __builtin_bit_cast(float, b));
}
// = group16_sum (butterfly order 8, 4, 2, 1), all lanes active
__device__ __forceinline__ float group16_sum_full(float v) {
  v += dpp_mov<DPP_ROR8>(v);
  v += dpp_mov<DPP_ROR4>(v);
  v += dpp_mov<DPP_XOR2>(v);
  v += dpp_mov<DPP_XOR1>(v);
  return v;
}
// the xor butterfly over offsets 1, 2, 4, 8 (that order), all lanes active
__device__ __forceinline__ float row16_sum_up(float v) {
  v += dpp_mov<DPP_XOR1>(v);
  v += dpp_mov<DPP_XOR2>(v);
  v += dpp_mov<DPP_HALF_MIRROR>(v);   // the other quad of the half row
  v += dpp_mov<DPP_MIRROR>(v);        // the other half row
  return v;
}

// ---------------------------------------------------------------- dropout RNG
// Counter-based: keep(seed, idx) is a pure function of (site/step seed, element index), so the
// backward pass regenerates every mask instead of storing it.  One 32-bit avalanche hash
// (lowbias32) per PAIR of elements {2j, 2j+1} gives two 16-bit uniforms; thresholds have 2^-16
// resolution (p = 0.2 keeps 1 - 13107/65536).  Cost: ~6 VALU per element.
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t seed32(uint64_t seed) { return (uint32_t)seed ^ (uint32_t)(seed >> 32) * 0x27d4eb2fU; }
// one 32-bit hash per pair of adjacent elements (16 bits each).  Two multiplies per pair, as lowbias32: the
// element-pair index is XORed into the site seed, and the seed ALSO picks the first multiplier (an odd constant
// derived from it, loop-invariant: formed once per thread / in scalar registers, not per pair).  With the seed
// in the XOR alone, two sites' (or steps') masks were the same sequence shifted by s1 ^ s2 pairs -- copies of each
// other whenever the seeds differed by less than the pair count; a seed-dependent multiplier makes them distinct
// functions of the pair index.  (Pair indices past 2^32 -- 8.6G elements of one site -- would repeat masks; a
// golden-ratio pre-multiply and a high-word term would cost two more 4-pass v_mul_lo_u32 per pair in every site.)
__device__ __forceinline__ uint32_t seed_mult(uint32_t s32) { return ((s32 * 0x9E3779B9u) ^ 0x7feb352dU) | 1u; }
__device__ __forceinline__ uint32_t pair_hash(uint32_t s32, uint64_t idx) {
  uint32_t x = (uint32_t)(idx >> 1) ^ s32;
  x ^= x >> 16;
  x *= seed_mult(s32);
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t drop_thr(float p) { return (uint32_t)fminf(p * 65536.0f, 65535.0f); }
// keep with probability 1-p; returns the multiplier (0 or 1/(1-p))
__device__ __forceinline__ float drop_mul(float p, uint64_t seed, uint64_t idx) {
  if (p <= 0.0f) return 1.0f;
  const uint32_t h = pair_hash(seed32(seed), idx);
  const uint32_t u = (idx & 1) ? (h >> 16) : (h & 0xFFFFu);
  return u >= drop_thr(p) ? 1.0f / (1.0f - p) : 0.0f;
}
// the two multipliers of elements idx, idx+1 (idx even) from one hash
__device__ __forceinline__ void drop_mul2(float p, uint32_t s32, uint64_t idx_even, float& m0, float& m1) {
  const uint32_t h = pair_hash(s32, idx_even);
  const uint32_t thr = drop_thr(p);
  const float k = 1.0f / (1.0f - p);
  m0 = (h & 0xFFFFu) >= thr ? k : 0.0f;
  m1 = (h >> 16) >= thr ? k : 0.0f;
}

// effective per-site seed: host-side site salt mixed with the device-side step
// seed (a device word advanced by rs_seed_advance, so graph replays re-draw masks)
__device__ __forceinline__ uint64_t eff_seed(uint64_t salt, const uint64_t* base) {
  return salt ^ ((base ? *base : 0ull) * 0xD1B54A32D192ED03ull);
}

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k = 0.7978845608028654f;  // sqrt(2/pi)
  return 0.5f * x * (1.0f + tanhf(k * (x + 0.044715f * x * x * x)));
}
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k = 0.7978845608028654f;
  float u = k * (x + 0.044715f * x * x * x);
  float t = tanhf(u);
  return 0.5f * (1.0f + t) + 0.5f * x * (1.0f - t * t) * k * (1.0f + 3.0f * 0.044715f * x * x);
}

// the same GELU in sigmoid form for the bf16 path: 0.5 (1 + tanh u) = 1 / (1 + e^{-2u}), one v_exp and one
// v_rcp instead of libm tanhf (which cost the BERT FFN GEMMs ~40% of their time)
__device__ __forceinline__ float gelu_sig(float x) {
  const float u2 = 1.5957691216057308f * x * (1.0f + 0.044715f * x * x);  // 2u
  return __builtin_amdgcn_rcpf(1.0f + __expf(-u2));
}
__device__ __forceinline__ float gelu_tanh_fast(float x) { return x * gelu_sig(x); }
__device__ __forceinline__ float gelu_tanh_grad_fast(float x) {
  const float s = gelu_sig(x);
  return s + x * s * (1.0f - s) * 1.5957691216057308f * (1.0f + 0.134145f * x * x);
}

__host__ __device__ static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---- kernel stamps (bench.py's in-step timing of the dominant launch; misc.hip rs_kernel_stamps) ----
// buf: [0] base step, [1] steps held, [2] marks per step, [3] W; then per (step slot, mark) a record of
// 1 + W u64: {begin, end lanes 0 .. W-1} in s_memrealtime ticks.  begin = the start of the first
// dispatched workgroup's wave 0 (workgroup 0 is dispatched first); every wave raises end lane
// (wave index mod W) to its exit time with a no-return atomic max -- W distinct words, so waves
// sharing a word are W apart in dispatch order and rarely contend (same-address atomics from
// thousands of waves serialise and cost tens of microseconds) -- and the reader takes the max over
// the lanes.  Slot = the optimizer's step count (*step, a device double advanced by rs_adam_prepare)
// - base.  buf == null: off.
struct KStamp {
  unsigned long long* buf;
  const double* step;
  int mark;
};

__device__ __forceinline__ unsigned long long* kstamp_rec(const KStamp& k) {
  const long long slot = (long long)(*k.step) - (long long)k.buf[0];
  if (slot < 0 || slot >= (long long)k.buf[1] || k.mark >= (int)k.buf[2]) return nullptr;
  return k.buf + 4 + (slot * (long long)k.buf[2] + k.mark) * (1 + (long long)k.buf[3]);
}

__device__ __forceinline__ long long kstamp_wave() {
  return ((long long)blockIdx.x + (long long)gridDim.x * ((long long)blockIdx.y + (long long)gridDim.y * blockIdx.z)) *
             (long long)(blockDim.x >> 6) + (threadIdx.x >> 6);
}

struct KStampBegin {
  __device__ __forceinline__ explicit KStampBegin(const KStamp& k) {
    if (k.buf && threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) {
      unsigned long long* p = kstamp_rec(k);
      if (p) *p = (unsigned long long)wall_clock64();
    }
  }
};

// raises its end lane when the wave leaves the kernel (any return path); the record address is formed
// at exit from the kernel arguments, so nothing stays live in registers across the kernel body
struct KStampEnd {
  const KStamp& k;
  __device__ __forceinline__ explicit KStampEnd(const KStamp& k_) : k(k_) {}
  __device__ __forceinline__ ~KStampEnd() {
    if (k.buf && (threadIdx.x & 63) == 0) {
      unsigned long long* p = kstamp_rec(k);
      if (p) atomicMax(p + 1 + kstamp_wave() % (long long)k.buf[3], (unsigned long long)wall_clock64());
    }
  }
};

// host: the stamp for the next stamped launch (marks numbered in launch order since rs_kernel_stamps);
// kind: RS_STAMP_* of the launch, reported by rs_kernel_stamp_kinds
KStamp kstamp_next(int kind);

// second pass of every two-level reduction (reduce.hip): out0[i] (+)= sum_z slab[z*n+i] for i < n0,
// out1[i-n0] likewise for n0 <= i < n (either output may be null to drop that part).
hipError_t launch_reduce_slabs(const float* slab, int splits, int64_t n, int64_t n0, float* out0, float* out1,
                               int accumulate, hipStream_t s);
