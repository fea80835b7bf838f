// 256-wide LDS-DMA stage machinery shared by the vocabulary head's dE / dh GEMMs (gemm_n256.hip) and the BERT
// weight gradients on 256 x 256 tiles (wgrad.hip wgrad_group256_kernel).  Header-only, namespace g256.
#pragma once
#include "common.h"

namespace g256 {

constexpr int BM = 256, BN = 256, BKT = 64, NTH = 512;
typedef __attribute__((ext_vector_type(4))) __bf16 bf4;

// ---------------------------------------------------------------------------------------------------------------
// 32-deep stages loaded by global_load_lds_dwordx4 straight into FOUR LDS stage buffers,
// three stages in flight -- no staging registers, and the HBM latency (~1-2 us under load) hidden behind three
// stages of MFMAs (~0.4 us each) instead of one.  A DMA writes 1 KB lane-linear, so the images are unpadded and the
// bank-conflict-free layouts are applied to the SOURCE address:
//  * k-major images ([32 k][256] as two halves of [32][128] bf16) in 8-row x 32-column subtiles (km_off) --
//    conflict-free for the transposing fragment reads;
//  * k-contiguous image ([256 m][32 k], 64-B rows): chunk ch of row r at 16 * (ch ^ h(r >> 2 & 3)) (kc_off).
// Every DMA source is clamped into the operand; the last (partial) stage zeroes its k rows / columns past the end in
// LDS before use.  One raw s_barrier per stage (after this wave's counted vmcnt and lgkmcnt(0)) publishes the
// stage and frees the buffer the next DMA overwrites.
#ifndef G256_DIST
#define G256_DIST 3
#endif
constexpr int DBK = 32, DIST = G256_DIST, NBUF = DIST + 1;
constexpr int KM_HALF = DBK * 128 * 2;          // bytes of one [32][128] half image
constexpr int IMG_BYTES = DBK * 256 * 2;        // 16 KB: one operand's stage image
constexpr int DSTAGE = 2 * IMG_BYTES;           // A + B
constexpr int PIECES = IMG_BYTES / 1024;        // 16 DMA pieces per image, 2 per wave

// byte offset of element (k-row r, column c) of a k-major stage image: two halves of [32][128]; within a half the
// guide's 8-row x 32-column subtile layout (cdna_hip_programming.md T10, image (a)): subtile (r >> 3, ch >> 2) of
// 512 B, row r & 7 at 64 B, 16-B chunk (ch & 3) ^ ((r >> 2) & 3).  Conflict-free for the transposing fragment
// reads, and a wave's fragments differ by compile-time offsets except for the (ch & 3) bit pattern (two address
// bases), so the fragment addresses cost almost no VALU (the 256-B-row XOR layout cost ~110 VALU per stage)
__device__ __forceinline__ uint32_t km_off(int r, int c) {
  const int cc = c & 127, ch = cc >> 3;
  return (uint32_t)((c >> 7) * KM_HALF + 2048 * (r >> 3) + 512 * (ch >> 2) + 64 * (r & 7) +
                    16 * ((ch & 3) ^ ((r >> 2) & 3)) + 2 * (cc & 7));
}
// byte offset of element (row m, k) of the k-contiguous stage image: chunk g of row m is stored at position
// g ^ h((m >> 2) & 3), h = {0, 2, 3, 1} -- with ds_read_b128's lane groups ({0-3, 12-15, 20-27}, {4-11, 16-19,
// 28-31}, ...) every group's 16 reads of a 16-row fragment then land on 16 distinct 16-B slots of a 256-B bank
// row (h = identity left 40 % of the LDS cycles as conflicts: SQ_LDS_BANK_CONFLICT 56M of 141M)
__device__ __forceinline__ uint32_t kc_swz(int m) { return (uint32_t)((0x1320u >> (4 * ((m >> 2) & 3))) & 3u); }
__device__ __forceinline__ uint32_t kc_off(int m, int k) {
  return (uint32_t)(64 * m + 16 * ((uint32_t)(k >> 3) ^ kc_swz(m)) + 2 * (k & 7));
}

typedef __attribute__((address_space(3))) void* lds_vptr;
__device__ __forceinline__ uint32_t lds_u32(const void* p) { return (uint32_t)(uintptr_t)(lds_vptr)p; }
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(dst)
               : "memory");
}
template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }
// wait for the oldest stage of a wave's DMAs, `after` later stages (4 pieces each: 2 per operand) left in flight
__device__ __forceinline__ void vm_wait_stages(int after) {
  if (after >= 4) vm_wait<16>();
  else if (after == 3) vm_wait<12>();
  else if (after == 2) vm_wait<8>();
  else if (after == 1) vm_wait<4>();
  else vm_wait<0>();
}
__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// piece j (0..15) of a k-major image: bytes [1024 (j & 7), +1024) of half j >> 3; lane l's 16 B at byte
// b = 1024 (j & 7) + 16 l hold (row r, logical chunk ch) of the subtile layout: source (k0 + r, c0 + 128 half + 8 ch)
__device__ __forceinline__ void km_piece(const __bf16* base, int64_t ld, int64_t k0, int64_t c0, int64_t klim,
                                         int64_t clim, int j, int lane, uint32_t img) {
  const int b = 1024 * (j & 7) + 16 * lane, half = j >> 3;
  const int r = 8 * (b >> 11) + ((b >> 6) & 7);
  const int ch = 4 * ((b >> 9) & 3) + (((b >> 4) & 3) ^ ((r >> 2) & 3));
  const int64_t k = min(k0 + r, klim - 1), c = min(c0 + half * 128 + 8 * ch, clim - 8);
  dma16(base + k * ld + c, __builtin_amdgcn_readfirstlane(img + (uint32_t)j * 1024));
}
// piece j of the k-contiguous image: rows 16 j .. +15; lane l stores chunk l & 3 of row 16 j + (l >> 2)
__device__ __forceinline__ void kc_piece(const __bf16* base, int64_t ld, int64_t m0, int64_t k0, int64_t mlim,
                                         int64_t kcap, int j, int lane, uint32_t img) {
  const int r = 16 * j + (lane >> 2);
  const int ch = (lane & 3) ^ (int)kc_swz(r);
  const int64_t m = min(m0 + r, mlim - 1), k = min(k0 + 8 * ch, kcap - 8);
  dma16(base + m * ld + k, __builtin_amdgcn_readfirstlane(img + (uint32_t)j * 1024));
}

// fragment (16 rows from row0, the stage's 32 k) of a k-major image: two transposing reads
__device__ __forceinline__ bf16x8 km_frag(const char* img, int row0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int c = row0 + 4 * p, r = 8 * g + q;
  const bf4 x = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf4*)(img + km_off(r, c)));
  const bf4 y =
      __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf4*)(img + km_off(r + 4, c)));
  return __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ bf16x8 kc_frag(const char* img, int row0, int lane) {
  const int g = lane >> 4, li = lane & 15;
  return *reinterpret_cast<const bf16x8*>(img + kc_off(row0 + li, 8 * g));
}

}  // namespace g256
