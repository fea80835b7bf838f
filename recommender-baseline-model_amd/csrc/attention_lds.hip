// LDS-resident attention for bf16, T <= 256, head dim 32/64/128 (gfx950).
//
// Same math and masks as attention.hip (the reference call sites are listed
// there): S = scale * q.k^T, causal -inf (SAS) or key-padding -1e9 (BERT),
// P = softmax(S), dropout(P), O = P.v; backward recomputes P from the row
// logsumexp.  Design (CDNA4):
//
//  * one workgroup = 4 waves = one (sequence, head) and a 1/nsplit share of its
//    16-row tiles; the two operands every tile needs (K,V forward and for dQ;
//    Q,dO for dK/dV) are staged ONCE into LDS as row-major images with a
//    32-byte row pad (T*Dh*2 B each: 51 KB at T=200, Dh=128), so HBM/L2 sees
//    each of q,k,v,o,dO about once per split;
//  * "key on the register axis": the first product of each pair is computed
//    transposed (S^T = K.Q^T in the forward / dQ pass, S = Q.K^T in the dK/dV
//    pass) so that its 16x16 accumulator tiles, packed pairwise to bf16, ARE
//    the B operand of the second product (O^T = V^T.P^T, dQ^T = K^T.dS^T,
//    dV^T = dO^T.P, dK^T = Q^T.dS): no P/dS round trip through LDS.  The k order
//    inside a 32-deep step is then {16(j>>2) + 4g + (j&3)}, and the matching A
//    operand (the transposed image) is read with ds_read_b64_tr_b16;
//  * softmax statistics per query live on one lane (+2 cross-group shuffles).
#include "common.h"
#include <algorithm>
#include <cstring>
#include "../../include/recsys_hip.h"

typedef __attribute__((ext_vector_type(4))) __bf16 bf4;
typedef __bf16 bf16;

#define PLAN_S 4
#define PLAN_I 6
struct AttnLdsArgs {
  int64_t B, T, H;
  const bf16* q; int64_t ldq;
  const bf16* k; int64_t ldk;
  const bf16* v; int64_t ldv;
  const bf16* o; int64_t ldo;
  const bf16* dout; int64_t lddo;
  bf16* out; int64_t ldout;     // forward: O
  bf16* dq; int64_t lddq;
  bf16* dk; int64_t lddk;
  bf16* dv; int64_t lddv;
  float* lse;                    // forward writes; backward reads
  float* delta;                  // dQ pass writes, dK/dV pass reads (delta_in: precomputed, both read)
  int delta_in;                  // delta = rowsum(dO * O) given by the caller (rs_sas_block_out_bwd): O is not read
  float scale;
  int mask_kind;                 // 0 causal (-inf), 1 key padding (-1e9)
  const int64_t* ids;
  float drop_p;
  uint64_t seed;
  const uint64_t* seed_base;
  int nsplit;
  KStamp ks;                     // backward: dQ kernel stamps begin, dK/dV kernel end
  // backward work plan (causal): per (split, wave) up to PLAN_I items, 0 = none; unused (use_plan 0) -> one
  // tile per wave round robin.  Item = valid << 31 | slot << 26 | role << 24 | chunk end << 16 | chunk begin
  // << 8 | tile; chunks are 32 keys (dQ) / 32 queries (dK/dV); role 0 = whole tile, 1 = lower half (its
  // partial goes to LDS slot `slot`), 2 = upper half (adds that slot's partial, then writes the tile)
  int use_plan;
  uint32_t plan[PLAN_S][8][PLAN_I];
};
#define DQ_SLOTS 4    // fp32 partial dQ tiles (8 KB each at Dh = 128)
#define DKV_SLOTS 3   // bf16 partial (dK, dV) tiles (8 KB each at Dh = 128)

#define NEG_INF (-__builtin_inff())
// 8 waves per workgroup (2 per SIMD): with ~7 tiles per workgroup every tile gets its own wave,
// and a SIMD always has a second wave to issue while the first waits on LDS / exp / MFMA results
#define NW 8
#define NT (64 * NW)
#define LOG2E 1.4426950408889634f
#define LN2 0.6931471805599453f
// softmax in the log2 domain: scores are scaled by scale*log2(e) once, exponentials are the raw
// v_exp_f32 (2^x); the reference's -1e9 fill (applied after scaling) becomes -1e9*log2(e)
#define MASK2 (-1e9f * LOG2E)
__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

// phase timestamps for tools/micro/attn_phase.hip (compiled out of the library)
#ifdef ATTN_PROF
__device__ unsigned long long g_attn_prof[8192 * NW * 10];
#define APROF(slot)                                                                          \
  do {                                                                                       \
    if ((threadIdx.x & 63) == 0)                                                             \
      g_attn_prof[((blockIdx.x + gridDim.x * blockIdx.y) * NW + (threadIdx.x >> 6)) * 10 + (slot)] = \
          wall_clock64();                                                                    \
  } while (0)
#else
#define APROF(slot) \
  do {              \
  } while (0)
#endif

template <int DH> struct Img { static constexpr int LD = DH + 16; };  // row stride (elements), +32 B pad

__device__ __forceinline__ bf16x8 cat8(bf4 a, bf4 b) {
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

// A operand = X^T for a 32-row k step starting at image row rb, columns c0..c0+15 (X row-major image)
__device__ __forceinline__ bf16x8 tr_frag(const bf16* img, int ld, int rb, int c0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const bf16* a0 = img + (rb + 4 * g + q) * ld + c0 + 4 * p;
  const bf4 x = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf4*)a0);
  const bf4 y = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf4*)(a0 + 16 * ld));
  return cat8(x, y);
}

// row fragment (A or B operand in natural k order) from an LDS image
__device__ __forceinline__ bf16x8 row_frag(const bf16* img, int ld, int row, int col) {
  return *reinterpret_cast<const bf16x8*>(img + row * ld + col);
}

__device__ __forceinline__ bf16x8 pack8(const f32x4& a, const f32x4& b) {
  bf16x8 r;
  r[0] = (bf16)a[0]; r[1] = (bf16)a[1]; r[2] = (bf16)a[2]; r[3] = (bf16)a[3];
  r[4] = (bf16)b[0]; r[5] = (bf16)b[1]; r[6] = (bf16)b[2]; r[7] = (bf16)b[3];
  return r;
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// global row chunk (zero beyond T).  Branch-free: the load always reads a valid row (clamped) and
// the result is masked afterwards -- a branch around the load makes hipcc wait vmcnt(0) per chunk.
__device__ __forceinline__ bf16x8 gload8(const bf16* base, int64_t ld, int64_t row, int64_t T, int col) {
  const int64_t rc = row < T ? row : T - 1;
  typedef __attribute__((ext_vector_type(4))) unsigned u4;
  u4 v = *reinterpret_cast<const u4*>(base + rc * ld + col);
  const unsigned keep = row < T ? 0xffffffffu : 0u;
  v &= keep;
  return __builtin_bit_cast(bf16x8, v);
}

// ------------------------------------------------------------------ progressive staging by LDS-DMA
// The operand images are filled by LDS-DMA (global_load_lds_dwordx4: 64 lanes x 16 B to 1 KB of LDS,
// lane-linear) in 32-row chunks by ONE loader wave (the workgroup's last), which keeps three chunks in flight
// and publishes each chunk (an LDS flag) as soon as its own vmcnt says it has landed; the other waves start on
// the first chunks while the rest stream in, and wait on the loader's flags only where they need a chunk.  The
// loader issues every DMA itself, so one wave's in-order vmcnt covers them all (no cross-wave publication), and
// the computing waves have no DMA in flight, so the compiler's vmcnt waits on their own loads stay exact.  The
// padded image row (DH + 16 elements) is 16-byte granular and a 32-row chunk is a whole number of 1 KB pieces
// (9 KB at DH = 128), so a piece's lanes that land on a row's pad just load some valid 16 B; rows past T load row
// T - 1 (finite values; every product with them is masked to 0).  After its stream the loader computes the
// smaller share the work plan gives it.
typedef __attribute__((address_space(3))) void* lds_ptr_t;
__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)(lds_ptr_t)p; }
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(dst)
               : "memory");
}
template <int N> __device__ __forceinline__ void vm_wait_n() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }
#define LOADER (NW - 1)   // the loader wave
#define NCNT 16           // chunk flags (T <= 256: at most 8 chunks), ints, in LDS
template <int DH> struct DmaStage {
  static constexpr int ROWB = Img<DH>::LD * 2, CHB = 32 * ROWB, PPC = CHB / 1024, PP = 2 * PPC, WIN = 3;
  static_assert(CHB % 1024 == 0, "a 32-row chunk is whole DMA pieces");
  static_assert(WIN * PP <= 63, "chunks in flight fit vmcnt");
  // all pieces of chunk c of both images (A -> LDS byte address la, B -> lb; head slices, row strides ldA / ldB)
  static __device__ __forceinline__ void chunk(const bf16* A, int64_t ldA, uint32_t la, const bf16* B, int64_t ldB,
                                               uint32_t lb, int T, int c, int lane) {
#pragma unroll
    for (int j = 0; j < PP; ++j) {
      const bool second = j >= PPC;
      const int pj = second ? j - PPC : j;
      const int off = c * CHB + pj * 1024 + lane * 16;
      const int row = off / ROWB, o = off - row * ROWB;
      const int col = o < DH * 2 ? o >> 1 : 0;
      const int64_t rr = row < T ? row : T - 1;
      const bf16* src = second ? B + rr * ldB + col : A + rr * ldA + col;
      dma16(src, __builtin_amdgcn_readfirstlane((second ? lb : la) + (uint32_t)(c * CHB + pj * 1024)));
    }
  }
  // loader, before the prologue barrier: the first WIN chunks
  static __device__ __forceinline__ void prime(const bf16* A, int64_t ldA, const bf16* imgA, const bf16* B,
                                               int64_t ldB, const bf16* imgB, int T, int nch, int lane) {
    const uint32_t la = lds_addr(imgA), lb = lds_addr(imgB);
    for (int c = 0; c < min(nch, WIN); ++c) chunk(A, ldA, la, B, ldB, lb, T, c, lane);
  }
  // loader, after the barrier (the flags are zero): publish chunk c once landed, keep WIN chunks in flight
  static __device__ __forceinline__ void stream(const bf16* A, int64_t ldA, const bf16* imgA, const bf16* B,
                                                int64_t ldB, const bf16* imgB, int T, int nch, int* flag, int lane) {
    const uint32_t la = lds_addr(imgA), lb = lds_addr(imgB);
    for (int c = 0; c < nch; ++c) {
      const int later = min(nch, c + WIN) - (c + 1);   // chunks issued after c, still allowed in flight
      if (later >= 2) vm_wait_n<2 * PP>();
      else if (later == 1) vm_wait_n<PP>();
      else vm_wait_n<0>();
      if (lane == 0) __hip_atomic_store(&flag[c], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (c + WIN < nch) chunk(A, ldA, la, B, ldB, lb, T, c + WIN, lane);
    }
  }
};
// a computing wave's view of the loader's flags
struct ChunkWait {
  const int* flag;
  int nch, ready;
  // chunk c (and every earlier one: the loader publishes in order) is in LDS
  __device__ __forceinline__ void ensure(int c) {
    c = min(c, nch - 1);
    if (c <= ready) return;
    // bounded: a missing flag (a bug) ends in wrong values, not a hung GPU
    for (int spin = 0; spin < (1 << 22) &&
                       __hip_atomic_load(&flag[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0;
         ++spin)
      __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
    ready = c;
  }
};
// prologue barrier without a memory fence (the fence's vmcnt(0) would wait for the loader's DMAs): LDS writes
// made before it (flags, key mask, lse / delta rows) are complete and visible after it
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// stage rows [0, rows) of a (T x DH) head slice into an LDS image (rows >= T zero).
// Batches of 8 chunks per thread: all 8 loads are issued before the first LDS store, so a
// 51 KB image takes ~2 dependent HBM round trips instead of one per chunk.
template <int DH>
__device__ __forceinline__ void stage(bf16* img, const bf16* src, int64_t ld, int64_t T, int rows, int tid) {
  constexpr int CPR = DH / 8, LD = Img<DH>::LD, U = 8;
  const int n = rows * CPR;
  for (int i0 = tid; i0 < n; i0 += NT * U) {
    bf16x8 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(i0 + u * NT, n - 1);
      v[u] = gload8(src, ld, i / CPR, T, (i % CPR) * 8);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * NT;
      if (i < n) *reinterpret_cast<bf16x8*>(img + (i / CPR) * LD + (i % CPR) * 8) = v[u];
    }
  }
}

// two images at once: every load of both is issued before the first LDS store (one dependent HBM
// round trip for both operands instead of one each)
template <int DH>
__device__ __forceinline__ void stage2(bf16* imgA, const bf16* srcA, int64_t ldA, bf16* imgB, const bf16* srcB,
                                       int64_t ldB, int64_t T, int rows, int tid) {
  constexpr int CPR = DH / 8, LD = Img<DH>::LD, U = 8;
  const int n = rows * CPR;
  for (int i0 = tid; i0 < n; i0 += NT * U) {
    bf16x8 va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(i0 + u * NT, n - 1);
      va[u] = gload8(srcA, ldA, i / CPR, T, (i % CPR) * 8);
      vb[u] = gload8(srcB, ldB, i / CPR, T, (i % CPR) * 8);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * NT;
      if (i < n) {
        *reinterpret_cast<bf16x8*>(imgA + (i / CPR) * LD + (i % CPR) * 8) = va[u];
        *reinterpret_cast<bf16x8*>(imgB + (i / CPR) * LD + (i % CPR) * 8) = vb[u];
      }
    }
  }
}

// 1.0 where the key is masked by key padding (mask_kind 1), else 0; keys >= T are handled separately
__device__ __forceinline__ void stage_keymask(float* km, const AttnLdsArgs& a, int64_t b, int rows, int tid) {
  for (int i = tid; i < rows; i += NT)
    km[i] = (a.mask_kind == 1 && i < a.T && a.ids[b * a.T + i] == 0) ? 1.f : 0.f;
}

// 0 = live score, 1 = -inf (causal / beyond the sequence), 2 = filled with -1e9 (key padding)
__device__ __forceinline__ int mask_state(const AttnLdsArgs& a, const float* km, int64_t q, int64_t key) {
  if (key >= a.T) return 1;
  if (a.mask_kind == 0) return key > q ? 1 : 0;
  return km[key] != 0.f ? 2 : 0;
}
__device__ __forceinline__ float apply_mask(int st, float s) { return st == 0 ? s : (st == 1 ? NEG_INF : -1e9f); }
__device__ __forceinline__ float masked(const AttnLdsArgs& a, const float* km, int64_t q, int64_t key, float s) {
  return apply_mask(mask_state(a, km, q, key), s);
}

// (sequence-head, split) of this workgroup.  Workgroups are dealt to the 8 XCDs round-robin in dispatch order
// (block b on XCC b % 8, fixed: tools/micro/xcd_probe.hip), so XCD x takes the x-th eighth of the sequence-heads
// -- the rows the row-chain kernels give the same XCD (rowchain.hip tiles_of_wave) -- and the nsplit workgroups of
// one sequence, which stage the same K/V (or Q/dO) rows, land on one XCD too.  The q/k/v the block-input kernel
// just wrote and the o (dO) this launch writes for the block-output kernel then stay in one XCD's L2.
// lin: the workgroup's linear index among the launch's workgroups of this pass (split fastest)
__device__ __forceinline__ void block_coords(const AttnLdsArgs& a, int64_t lin, int64_t& bh, int& split) {
  const int ns = a.nsplit;
  const int64_t BH = a.B * a.H;
  if (BH % 8 == 0) {
    const int64_t xcd = lin & 7, slot = lin >> 3;
    bh = xcd * (BH >> 3) + slot / ns;
    split = (int)(slot % ns);
  } else {
    bh = lin / ns;
    split = (int)(lin % ns);
  }
}
__device__ __forceinline__ void block_coords(const AttnLdsArgs& a, int64_t& bh, int& split) {
  block_coords(a, blockIdx.x + (int64_t)a.nsplit * blockIdx.y, bh, split);
}

// tiles of 16 queries handled by this workgroup: split, split+nsplit, ...
__device__ __forceinline__ int last_tile_of_split(int nq, int split, int nsplit) {
  return split + ((nq - 1 - split) / nsplit) * nsplit;
}

// ------------------------------------------------------------------ forward
template <int DH>
__global__ __launch_bounds__(NT) void attn_fwd_lds_kernel(AttnLdsArgs a) {
  constexpr int LD = Img<DH>::LD, KC = DH / 32, DT = DH / 16, NKT = 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  APROF(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4, cl = lane & 15;
  int64_t bh;
  int split;
  block_coords(a, bh, split);
  const int64_t b = bh / a.H, h = bh % a.H;
  const int T = (int)a.T;
  const int nq = (T + 15) / 16;
  if (split >= nq) return;
  const int lastq = last_tile_of_split(nq, split, a.nsplit);
  const int kneed = a.mask_kind == 0 ? min(T, 16 * (lastq + 1)) : T;
  const int rows = ((kneed + 31) / 32) * 32;
  bf16* Ks = reinterpret_cast<bf16*>(smem);
  bf16* Vs = Ks + rows * LD;
  float* km = reinterpret_cast<float*>(Vs + rows * LD);
  const bf16* Kg = a.k + b * a.T * a.ldk + h * DH;
  const bf16* Vg = a.v + b * a.T * a.ldv + h * DH;
  const bf16* Qg = a.q + b * a.T * a.ldq + h * DH;
  // the first query tile's operands are requested before (and so arrive with) the K/V staging.  (The forward
  // keeps all-wave register staging: its longest query tile needs every key chunk at once, so the loader-wave
  // stream of the backward passes measured slower here: 14.7 vs 12.6 us at B = 128, T = 200.)
  bf16x8 qf[KC];
  {
    const int64_t qrow0 = (split + wave * a.nsplit) * 16 + cl;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) qf[kc] = gload8(Qg, a.ldq, qrow0, a.T, kc * 32 + 8 * g);
  }
  stage2<DH>(Ks, Kg, a.ldk, Vs, Vg, a.ldv, a.T, rows, tid);
  stage_keymask(km, a, b, rows, tid);
  __syncthreads();
  APROF(1);
  const uint64_t seed = eff_seed(a.seed, a.seed_base);
  // the younger half at issue priority 1, as in the backward passes (cfg2 bench, three interleaved rounds: 459.2 /
  // 463.1 / 462.2k -> 462.8 / 463.8 / 466.6k seq/s)
  if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);

  for (int qt = split + wave * a.nsplit; qt < nq; qt += NW * a.nsplit) {
    const int q0 = qt * 16;
    const int64_t qrow = q0 + cl;  // this lane's query
    if (qt != split + wave * a.nsplit) {
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) qf[kc] = gload8(Qg, a.ldq, qrow, a.T, kc * 32 + 8 * g);
    }
    const int nkt = a.mask_kind == 0 ? qt + 1 : nq;
    const float sl2 = a.scale * LOG2E;
    const int qi = q0 + cl;
    f32x4 s[NKT];
    float mx = NEG_INF;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      s[kt] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (kt < nkt) {
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) s[kt] = mfma16(row_frag(Ks, LD, kt * 16 + cl, kc * 32 + 8 * g), qf[kc], s[kt]);
        // per-element masking only where a tile can hold masked scores (wave-uniform test); selects, not
        // exec-mask branches (the key-padding flags are one vector load, 0 when causal)
        const bool need = a.mask_kind != 0 || kt == qt || kt * 16 + 16 > T;
        const int kb = kt * 16 + 4 * g;
        if (need) {
          const f32x4 kmv = *reinterpret_cast<const f32x4*>(km + kb);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int k = kb + r;
            const bool dead = (k >= T) | ((a.mask_kind == 0) & (k > qi));
            const float x = s[kt][r] * sl2;
            s[kt][r] = dead ? NEG_INF : (kmv[r] != 0.f ? MASK2 : x);
            mx = fmaxf(mx, s[kt][r]);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            s[kt][r] *= sl2;
            mx = fmaxf(mx, s[kt][r]);
          }
        }
      }
    }
    mx = max_xor32(max_xor16(mx));
    float sm = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      if (kt < nkt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = ex2(s[kt][r] - mx);
          s[kt][r] = e;
          sm += e;
        }
      }
    }
    sm = add_xor32(add_xor16(sm));
    const float inv = 1.f / sm;
    if (g == 0 && qrow < a.T) a.lse[bh * a.T + qrow] = (mx + __builtin_amdgcn_logf(sm)) * LN2;
    // P^T (+ dropout: one hash per pair of adjacent keys), packed pairwise as the B operand of O^T = V^T P^T
    const uint32_t s32 = seed32(seed);
    const uint32_t rowidx = (uint32_t)(((int)bh * T + qi) * (T + (T & 1)));   // mask row pitch: even
    f32x4 o[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NKT / 2; ++c) {
      if (2 * c < nkt) {
        f32x4 pp[2] = {s[2 * c], s[2 * c + 1]};
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const int t = 2 * c + hf;
          const float sc = t < nkt ? inv : 0.f;
          if (a.drop_p > 0.f) {
            float m[4];
            const uint32_t base = rowidx + (uint32_t)(t * 16 + 4 * g);
            drop_mul2(a.drop_p, s32, base, m[0], m[1]);
            drop_mul2(a.drop_p, s32, base + 2, m[2], m[3]);
#pragma unroll
            for (int r = 0; r < 4; ++r) pp[hf][r] *= sc * m[r];
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) pp[hf][r] *= sc;
          }
        }
        const bf16x8 pb = pack8(pp[0], pp[1]);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) o[dt] = mfma16(tr_frag(Vs, LD, 32 * c, 16 * dt, lane), pb, o[dt]);
      }
    }
    if (qrow < a.T) {
      bf16* O = a.out + (b * a.T + qrow) * a.ldout + h * DH;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        bf4 w;
        w[0] = (bf16)o[dt][0]; w[1] = (bf16)o[dt][1]; w[2] = (bf16)o[dt][2]; w[3] = (bf16)o[dt][3];
        *reinterpret_cast<bf4*>(O + 16 * dt + 4 * g) = w;
      }
    }
  }
  APROF(2);
}

// ------------------------------------------------------------------ backward: delta + dQ
template <int DH>
__device__ __forceinline__ void attn_bwd_dq_body(const AttnLdsArgs& a, int64_t lin) {
  constexpr int LD = Img<DH>::LD, KC = DH / 32, DT = DH / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  APROF(4);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4, cl = lane & 15;
  int64_t bh;
  int split;
  block_coords(a, lin, bh, split);
  const int64_t b = bh / a.H, h = bh % a.H;
  const int T = (int)a.T;
  const int nq = (T + 15) / 16;
  if (split >= nq) return;
  const int lastq = last_tile_of_split(nq, split, a.nsplit);
  const int kneed = a.mask_kind == 0 ? min(T, 16 * (lastq + 1)) : T;
  const int rows = ((kneed + 31) / 32) * 32;
  bf16* Ks = reinterpret_cast<bf16*>(smem);
  bf16* Vs = Ks + rows * LD;
  float* km = reinterpret_cast<float*>(Vs + rows * LD);
  int* cnt = reinterpret_cast<int*>(km + rows);
  float* slots = km + rows + NCNT;                     // plan: fp32 partial dQ tiles [slot][DT*4][64]
  int* flags = reinterpret_cast<int*>(slots + DQ_SLOTS * DT * 4 * 64);
  const bf16* Qg = a.q + b * a.T * a.ldq + h * DH;
  const bf16* Og = a.o + b * a.T * a.ldo + h * DH;
  const bf16* dOg = a.dout + b * a.T * a.lddo + h * DH;
  // this wave's work items: the plan's (tile, key-chunk range, role), else one whole tile per wave round robin
  auto item = [&](int it, int& qt, int& cb, int& ce, int& role, int& slot) -> bool {
    if (a.use_plan) {
      if (it >= PLAN_I) return false;
      const uint32_t e = a.plan[split][wave][it];
      if (!(e >> 31)) return false;
      qt = e & 255; cb = (e >> 8) & 255; ce = (e >> 16) & 255; role = (e >> 24) & 3; slot = (e >> 26) & 15;
      return true;
    }
    qt = split + (wave + it * NW) * a.nsplit;
    if (qt >= nq) return false;
    cb = 0;
    ce = ((a.mask_kind == 0 ? qt + 1 : nq) + 1) / 2;
    role = 0; slot = 0;
    return true;
  };
  if (a.use_plan && tid < DQ_SLOTS) flags[tid] = 0;
  if (tid < NCNT) cnt[tid] = 0;
  const int nch = rows / 32;
  bf16x8 qf[KC], df[KC], of[KC];
  int qt0 = 0, cb0, ce0, role0, slot0;
  const bool any = item(0, qt0, cb0, ce0, role0, slot0);
  const bf16* Kg = a.k + b * a.T * a.ldk + h * DH;
  const bf16* Vg = a.v + b * a.T * a.ldv + h * DH;
  if (wave == LOADER) {
    DmaStage<DH>::prime(Kg, a.ldk, Ks, Vg, a.ldv, Vs, T, nch, lane);
  } else {   // the first item's q, dO (, O) rows
    const int64_t qrow0 = (any ? qt0 : 0) * 16 + cl;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      qf[kc] = gload8(Qg, a.ldq, qrow0, a.T, kc * 32 + 8 * g);
      df[kc] = gload8(dOg, a.lddo, qrow0, a.T, kc * 32 + 8 * g);
      if (!a.delta_in) of[kc] = gload8(Og, a.ldo, qrow0, a.T, kc * 32 + 8 * g);
    }
  }
  stage_keymask(km, a, b, rows, tid);
  lds_barrier();
  if (wave == LOADER) DmaStage<DH>::stream(Kg, a.ldk, Ks, Vg, a.ldv, Vs, T, nch, cnt, lane);
  ChunkWait ch{cnt, nch, wave == LOADER ? nch - 1 : -1};
  APROF(5);
  const uint64_t seed = eff_seed(a.seed, a.seed_base);

  // the second-dispatched half of the workgroup (waves 4-7, each sharing a SIMD with one of waves 0-3) at issue
  // priority 1 for the whole loop: it otherwise loses every arbitration to its older partner (phase stamps, B = 128,
  // T = 200, tools/micro/attn_bwd_phase.hip, two interleaved rounds: span 25.99 / 25.85 -> 24.44 / 23.66 us)
  if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  int qt, cb, ce, role, slot;
  for (int it = 0; item(it, qt, cb, ce, role, slot); ++it) {
    const int q0 = qt * 16;
    const int64_t qrow = q0 + cl;
    if (it > 0 || wave == LOADER) {
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        qf[kc] = gload8(Qg, a.ldq, qrow, a.T, kc * 32 + 8 * g);
        df[kc] = gload8(dOg, a.lddo, qrow, a.T, kc * 32 + 8 * g);
        if (!a.delta_in) of[kc] = gload8(Og, a.ldo, qrow, a.T, kc * 32 + 8 * g);
      }
    }
    float dl = 0.f;
    if (a.delta_in) {
      dl = a.delta[bh * a.T + (qrow < a.T ? qrow : a.T - 1)];
    } else {
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
#pragma unroll
        for (int j = 0; j < 8; ++j) dl += (float)df[kc][j] * (float)of[kc][j];
      }
      dl = add_xor32(add_xor16(dl));  // delta = rowsum(dO * O) for query qrow
      if (role != 1 && g == 0 && qrow < a.T) a.delta[bh * a.T + qrow] = dl;
    }
    const float lq2 = (qrow < a.T ? a.lse[bh * a.T + qrow] : 0.f) * LOG2E;
    const float sl2 = a.scale * LOG2E;
    const int qi = q0 + cl;
    const uint32_t s32 = seed32(seed);
    const uint32_t rowidx = (uint32_t)(((int)bh * T + qi) * (T + (T & 1)));   // mask row pitch: even
    const bool qok = qi < T;
    const int nkt = a.mask_kind == 0 ? qt + 1 : nq;
    f32x4 acc[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) acc[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // two-stage pipeline over 16-key half steps: the S / dP products of the next half step are issued before
    // the softmax-gradient VALU of the current one, so the MFMA chains run under it.  Half steps past the
    // tile's keys (t >= nkt) are computed on a clamped row and masked (branch-free issue).
    const int tmax = rows / 16 - 1;
    auto sdp = [&](int t, f32x4& sv, f32x4& dp) {
      const int tr = min(t, tmax);
      bf16x8 fk[KC], fv[KC];
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        fk[kc] = row_frag(Ks, LD, tr * 16 + cl, kc * 32 + 8 * g);
        fv[kc] = row_frag(Vs, LD, tr * 16 + cl, kc * 32 + 8 * g);
      }
      sv = (f32x4){0.f, 0.f, 0.f, 0.f};
      dp = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        sv = mfma16(fk[kc], qf[kc], sv);
        dp = mfma16(fv[kc], df[kc], dp);
      }
    };
    // dS^T for half step t: P = exp2(S*scale*log2e - lse), dS = P*(dP*mask - delta)*scale; 0 where masked
    // (branch-free per element: the masks are selects; only the wave-uniform `need` picks the masked variant)
    auto dsv = [&](int t, const f32x4& sv, const f32x4& dp, f32x4& ds) {
      const bool need = a.mask_kind != 0 || t >= qt || t * 16 + 16 > T;
      const int kb = t * 16 + 4 * g;
      float m[4] = {1.f, 1.f, 1.f, 1.f};
      if (a.drop_p > 0.f) {
        drop_mul2(a.drop_p, s32, rowidx + (uint32_t)kb, m[0], m[1]);
        drop_mul2(a.drop_p, s32, rowidx + (uint32_t)kb + 2, m[2], m[3]);
      }
      const bool tok = (t < nkt) & qok, causal = a.mask_kind == 0;
      float pe[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) pe[r] = ex2(sv[r] * sl2 - lq2) * a.scale;
      if (need) {
        // masked_fill has no gradient: dS = 0 on masked scores (-inf and -1e9 alike)
        const f32x4 kmv = *reinterpret_cast<const f32x4*>(km + kb);   // key-padding flags (0 when causal)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int k = kb + r;
          // non-short-circuit (&): selects, no exec-mask branches
          const bool live = tok & (k < T) & !(causal & (k > qi)) & (kmv[r] == 0.f);
          const float v = pe[r] * (dp[r] * m[r] - dl);
          ds[r] = live ? v : 0.f;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) ds[r] = tok ? pe[r] * (dp[r] * m[r] - dl) : 0.f;
      }
    };
    f32x4 sA, dA, sB, dB, dsA, dsB;
    ch.ensure(cb);
    sdp(2 * cb, sA, dA);
    for (int c = cb; c < ce; ++c) {
      sdp(2 * c + 1, sB, dB);
      dsv(2 * c, sA, dA, dsA);
      if (c + 1 < ce) ch.ensure(c + 1);   // the next chunk's rows (once per chunk: a scheduling fence)
      sdp(2 * c + 2, sA, dA);      // past the range on the last chunk: clamped, unused
      dsv(2 * c + 1, sB, dB, dsB);
      const bf16x8 bds = pack8(dsA, dsB);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) acc[dt] = mfma16(tr_frag(Ks, LD, 32 * c, 16 * dt, lane), bds, acc[dt]);
    }
    float* sl = slots + slot * (DT * 4 * 64);
    if (role == 1) {
      // upper key half: partial dQ -> LDS slot, then release it to the lower half's wave
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) sl[(dt * 4 + r) * 64 + lane] = acc[dt][r];
      // LDS-only hand-off: the slot writes precede the flag in this wave's in-order LDS stream (a release fence
      // would also wait for this wave's DMAs still in flight)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(&flags[slot], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      continue;
    }
    if (role == 2) {
      for (int spin = 0; spin < (1 << 22) &&
                         __hip_atomic_load(&flags[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0;
           ++spin)
        __builtin_amdgcn_s_sleep(1);
      asm volatile("" ::: "memory");
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[dt][r] += sl[(dt * 4 + r) * 64 + lane];
    }
    if (qrow < a.T) {
      bf16* dQ = a.dq + (b * a.T + qrow) * a.lddq + h * DH;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        bf4 w;
        w[0] = (bf16)acc[dt][0]; w[1] = (bf16)acc[dt][1]; w[2] = (bf16)acc[dt][2]; w[3] = (bf16)acc[dt][3];
        *reinterpret_cast<bf4*>(dQ + 16 * dt + 4 * g) = w;
      }
    }
  }
  APROF(6);
}

// ------------------------------------------------------------------ backward: dK, dV
// Dropout multipliers of P[q0 + r*... ] for this lane's key ki and its 4 queries (row indices rq0 + r*Tp): the
// pair hash of (query, key pair) is shared by the lanes of keys ki and ki^1 (lanes l and l^1), so each lane hashes
// two of the four queries and takes the other two from its partner (one DPP move each) -- the same multipliers as
// drop_mul(p, seed, rowq + ki), one hash per element pair instead of per element.
__device__ __forceinline__ void drop_keys4(float p, uint32_t s32, uint32_t rq0, uint32_t Tp, uint32_t ki, int lane,
                                           float (&m)[4]) {
  const uint32_t odd = (uint32_t)(lane & 1), r0 = 2 * odd;
  const uint32_t h0 = pair_hash(s32, rq0 + r0 * Tp + ki), h1 = pair_hash(s32, rq0 + (r0 + 1) * Tp + ki);
  const uint32_t x0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)h0, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
  const uint32_t x1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)h1, 0xB1, 0xF, 0xF, true);
  uint32_t h[4];
  h[0] = odd ? x0 : h0;
  h[1] = odd ? x1 : h1;
  h[2] = odd ? h0 : x0;
  h[3] = odd ? h1 : x1;
  const uint32_t thr = drop_thr(p);
  const float k = 1.0f / (1.0f - p);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t u = (ki & 1) ? (h[r] >> 16) : (h[r] & 0xFFFFu);
    m[r] = u >= thr ? k : 0.f;
  }
}

// own_delta: delta = rowsum(dO * O) is formed here (from O rows and the staged dO image, in the dQ pass's
// summation order, so bit for bit the same values) instead of read from the dQ pass -- the two passes then
// run as ONE launch (attn_bwd_lds_kernel) with no ordering between their workgroups
template <int DH>
__device__ __forceinline__ void attn_bwd_dkv_body(const AttnLdsArgs& a, int64_t lin, bool own_delta) {
  constexpr int LD = Img<DH>::LD, KC = DH / 32, DT = DH / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  APROF(7);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4, cl = lane & 15;
  int64_t bh;
  int split;
  block_coords(a, lin, bh, split);
  const int64_t b = bh / a.H, h = bh % a.H;
  const int T = (int)a.T;
  const int nk = (T + 15) / 16;  // key tiles
  if (split >= nk) return;
  // queries needed: causal -> from the first key tile of this split on (all queries of the
  // sequence, kept simple: the image always starts at query 0)
  const int rows = ((T + 31) / 32) * 32;
  bf16* Qs = reinterpret_cast<bf16*>(smem);
  bf16* dOs = Qs + rows * LD;
  float* lse_s = reinterpret_cast<float*>(dOs + rows * LD);
  float* dl_s = lse_s + rows;
  float* km = dl_s + rows;
  int* cnt = reinterpret_cast<int*>(km + rows);
  bf16* slots = reinterpret_cast<bf16*>(km + rows + NCNT);   // plan: bf16 partial (dK, dV) tiles [slot][2][DT*4][64]
  int* flags = reinterpret_cast<int*>(slots + DKV_SLOTS * 2 * DT * 4 * 64);
  const bf16* Kg = a.k + b * a.T * a.ldk + h * DH;
  const bf16* Vg = a.v + b * a.T * a.ldv + h * DH;
  const int nqc = (T + 31) / 32;  // 32-query chunks
  // this wave's work items: the plan's (key tile, query-chunk range, role), else one whole key tile per wave
  auto item = [&](int it, int& kt, int& cb, int& ce, int& role, int& slot) -> bool {
    if (a.use_plan) {
      if (it >= PLAN_I) return false;
      const uint32_t e = a.plan[split][wave][it];
      if (!(e >> 31)) return false;
      kt = e & 255; cb = (e >> 8) & 255; ce = (e >> 16) & 255; role = (e >> 24) & 3; slot = (e >> 26) & 15;
      return true;
    }
    kt = split + (wave + it * NW) * a.nsplit;
    if (kt >= nk) return false;
    cb = a.mask_kind == 0 ? kt / 2 : 0;
    ce = nqc;
    role = 0; slot = 0;
    return true;
  };
  if (a.use_plan && tid < DKV_SLOTS) flags[tid] = 0;
  if (tid < NCNT) cnt[tid] = 0;
  const int nch = rows / 32;
  bf16x8 kf[KC], vf[KC];
  int kt0 = 0, cb0, ce0, role0, slot0;
  const bool any = item(0, kt0, cb0, ce0, role0, slot0);
  const bf16* Qg = a.q + b * a.T * a.ldq + h * DH;
  const bf16* dOg = a.dout + b * a.T * a.lddo + h * DH;
  // own_delta: this wave's first two 16-row groups of O, requested with its first operands
  const bf16* Og = a.o + b * a.T * a.ldo + h * DH;
  bf16x8 op[2][KC];
  if (wave == LOADER) {
    DmaStage<DH>::prime(Qg, a.ldq, Qs, dOg, a.lddo, dOs, T, nch, lane);
  } else {   // the first key tile's k/v rows
    const int64_t key0 = (any ? kt0 : 0) * 16 + cl;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      kf[kc] = gload8(Kg, a.ldk, key0, a.T, kc * 32 + 8 * g);
      vf[kc] = gload8(Vg, a.ldv, key0, a.T, kc * 32 + 8 * g);
    }
    if (own_delta) {
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) op[k][kc] = gload8(Og, a.ldo, (wave + k * NW) * 16 + cl, a.T, kc * 32 + 8 * g);
    }
  }
  if (tid < rows) {   // per-query lse / delta (rows <= 256: waves 0..3, never the loader)
    const int ti = min(tid, T - 1);
    const float lse_v = a.lse[bh * a.T + ti] * LOG2E, dl_v = own_delta ? 0.f : a.delta[bh * a.T + ti];
    lse_s[tid] = tid < T ? lse_v : 0.f;
    dl_s[tid] = tid < T ? dl_v : 0.f;
  }
  stage_keymask(km, a, b, rows, tid);
  lds_barrier();
  if (wave == LOADER) DmaStage<DH>::stream(Qg, a.ldq, Qs, dOg, a.lddo, dOs, T, nch, cnt, lane);
  ChunkWait ch{cnt, nch, wave == LOADER ? nch - 1 : -1};
  if (own_delta) {
    ch.ensure(nch - 1);   // the whole dO image
    for (int k = 0, rg = wave; rg * 16 < rows; ++k, rg += NW) {
      const int row = rg * 16 + cl;
      bf16x8 of[KC];
#pragma unroll
      for (int kc = 0; kc < KC; ++kc)
        of[kc] = (k < 2 && wave != LOADER) ? op[k][kc] : gload8(Og, a.ldo, row, a.T, kc * 32 + 8 * g);
      float dl = 0.f;
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        const bf16x8 dfv = *reinterpret_cast<const bf16x8*>(dOs + row * LD + kc * 32 + 8 * g);
#pragma unroll
        for (int j = 0; j < 8; ++j) dl += (float)dfv[j] * (float)of[kc][j];
      }
      dl = add_xor32(add_xor16(dl));
      if (g == 0) dl_s[row] = row < T ? dl : 0.f;
    }
    __syncthreads();
  }
  APROF(8);
  const uint64_t seed = eff_seed(a.seed, a.seed_base);
  const uint32_t s32 = seed32(seed), Tp = (uint32_t)(T + (T & 1));   // mask row pitch: even

  const float sl2 = a.scale * LOG2E;
  if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);   // as the dQ pass
  int kt, cb, ce, role, slot;
  for (int it = 0; item(it, kt, cb, ce, role, slot); ++it) {
    const int64_t key = kt * 16 + cl;  // this lane's key
    const int ki = kt * 16 + cl;
    if (it > 0 || wave == LOADER) {
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        kf[kc] = gload8(Kg, a.ldk, key, a.T, kc * 32 + 8 * g);
        vf[kc] = gload8(Vg, a.ldv, key, a.T, kc * 32 + 8 * g);
      }
    }
    f32x4 dk[DT], dv[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      dk[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
      dv[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    // two-stage pipeline over 16-query half steps (as the dQ pass): the next half step's S / dP MFMAs run under
    // this one's VALU; half steps past the image are computed on a clamped row and unused
    const int tmax = rows / 16 - 1;
    auto sdp = [&](int t, f32x4& sv, f32x4& dp) {
      const int tr = min(t, tmax);
      bf16x8 fq[KC], fo[KC];
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        fq[kc] = row_frag(Qs, LD, tr * 16 + cl, kc * 32 + 8 * g);
        fo[kc] = row_frag(dOs, LD, tr * 16 + cl, kc * 32 + 8 * g);
      }
      sv = (f32x4){0.f, 0.f, 0.f, 0.f};
      dp = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        sv = mfma16(fq[kc], kf[kc], sv);
        dp = mfma16(fo[kc], vf[kc], dp);
      }
    };
    // P (dropped) and dS for this lane's key and the 4 queries t*16 + 4g + r
    // (branch-free per element: masks are selects; the wave-uniform `need` picks the masked variant)
    const bool kdead = ki >= T, kfill = km[min(ki, rows - 1)] != 0.f;   // key beyond T / key padding (-1e9)
    auto pds = [&](int t, const f32x4& sv, const f32x4& dp, f32x4& pd, f32x4& ds) {
      const f32x4 ls = *reinterpret_cast<const f32x4*>(lse_s + t * 16 + 4 * g);
      const f32x4 dd = *reinterpret_cast<const f32x4*>(dl_s + t * 16 + 4 * g);
      float m[4] = {1.f, 1.f, 1.f, 1.f};
      if (a.drop_p > 0.f) drop_keys4(a.drop_p, s32, ((uint32_t)bh * (uint32_t)T + (uint32_t)(t * 16 + 4 * g)) * Tp,
                                     Tp, (uint32_t)ki, lane, m);
      const bool need = a.mask_kind != 0 || t <= kt || t * 16 + 16 > T || kt * 16 + 16 > T;
      if (need) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qr = t * 16 + 4 * g + r;
          const bool dead = kdead | (qr >= T) | ((a.mask_kind == 0) & (ki > qr));   // -inf: P = 0
          const float x2 = kfill ? MASK2 : sv[r] * sl2;                          // -1e9 fill: P from the fill
          const float p = ex2(dead ? NEG_INF : x2 - ls[r]);                      // select, not a branch
          pd[r] = p * m[r];
          const float v = p * (dp[r] * m[r] - dd[r]) * a.scale;
          ds[r] = dead | kfill ? 0.f : v;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = ex2(sv[r] * sl2 - ls[r]);
          pd[r] = p * m[r];
          ds[r] = p * (dp[r] * m[r] - dd[r]) * a.scale;
        }
      }
    };
    f32x4 sA, dA, sB, dB, pdA, dsA, pdB, dsB;
    ch.ensure(cb);
    sdp(2 * cb, sA, dA);
    for (int c = cb; c < ce; ++c) {
      sdp(2 * c + 1, sB, dB);
      pds(2 * c, sA, dA, pdA, dsA);
      if (c + 1 < ce) ch.ensure(c + 1);
      sdp(2 * c + 2, sA, dA);
      pds(2 * c + 1, sB, dB, pdB, dsB);
      const bf16x8 bp = pack8(pdA, pdB);
      const bf16x8 bds = pack8(dsA, dsB);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        dv[dt] = mfma16(tr_frag(dOs, LD, 32 * c, 16 * dt, lane), bp, dv[dt]);
        dk[dt] = mfma16(tr_frag(Qs, LD, 32 * c, 16 * dt, lane), bds, dk[dt]);
      }
    }
    bf16* sl = slots + slot * (2 * DT * 4 * 64);
    if (role == 1) {
      // upper query half: partial (dK, dV) -> LDS slot (bf16), then release it to the lower half's wave
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          sl[(dt * 4 + r) * 64 + lane] = (bf16)dk[dt][r];
          sl[(DT * 4 + dt * 4 + r) * 64 + lane] = (bf16)dv[dt][r];
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // LDS-only hand-off (see the dQ pass)
      if (lane == 0) __hip_atomic_store(&flags[slot], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      continue;
    }
    if (role == 2) {
      for (int spin = 0; spin < (1 << 22) &&
                         __hip_atomic_load(&flags[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0;
           ++spin)
        __builtin_amdgcn_s_sleep(1);
      asm volatile("" ::: "memory");
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dk[dt][r] += (float)sl[(dt * 4 + r) * 64 + lane];
          dv[dt][r] += (float)sl[(DT * 4 + dt * 4 + r) * 64 + lane];
        }
    }
    if (key < a.T) {
      bf16* dK = a.dk + (b * a.T + key) * a.lddk + h * DH;
      bf16* dV = a.dv + (b * a.T + key) * a.lddv + h * DH;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        bf4 wk, wv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          wk[r] = (bf16)dk[dt][r];
          wv[r] = (bf16)dv[dt][r];
        }
        *reinterpret_cast<bf4*>(dK + 16 * dt + 4 * g) = wk;
        *reinterpret_cast<bf4*>(dV + 16 * dt + 4 * g) = wv;
      }
    }
  }
  APROF(9);
}

// both backward passes in one launch: workgroups [0, n_dq) are dQ ones (dispatched first), the rest dK/dV
// ones, which take CUs as dQ workgroups retire -- their Q/dO staging overlaps other CUs' dQ compute instead
// of following a launch boundary with the whole chip loading at once
template <int DH>
__global__ __launch_bounds__(NT) void attn_bwd_lds_kernel(AttnLdsArgs aq, AttnLdsArgs akv) {
  KStampBegin begin_(aq.ks);
  KStampEnd end_(aq.ks);
  const int64_t nq = (int64_t)aq.nsplit * aq.B * aq.H;
  if ((int64_t)blockIdx.x < nq) attn_bwd_dq_body<DH>(aq, blockIdx.x);
  else attn_bwd_dkv_body<DH>(akv, blockIdx.x - nq, !akv.delta_in);
}

// ------------------------------------------------------------------ launchers
template <int DH>
static size_t fwd_lds_bytes(int T) {
  const int rows = ((T + 31) / 32) * 32;
  return (size_t)2 * rows * Img<DH>::LD * 2 + rows * 4 + NCNT * 4;
}
template <int DH>
static size_t dkv_lds_bytes(int T) {
  const int rows = ((T + 31) / 32) * 32;
  return (size_t)2 * rows * Img<DH>::LD * 2 + 3 * rows * 4 + NCNT * 4;
}

static int pick_split(int64_t BH, int ntiles) {
  // aim for >= 256 workgroups (one per CU at T ~ 200), at least 2 tiles per wave group
  int s = 1;
  while (BH * s < 256 && s * 2 <= std::max(1, ntiles / 4)) s *= 2;   // ~7 tiles per 8-wave group at T=200
  return s;
}

// backward: the merged launch runs 2 * nsplit * BH workgroups (dQ + dK/dV); keep them to one round on the
// chip's 256 CUs (one workgroup each) so every dK/dV workgroup runs BESIDE the dQ ones, not after them
static int pick_split_bwd(int64_t BH, int ntiles) {
  int s = 1;
  while (2 * BH * s * 2 <= 256 && s * 2 <= std::max(1, ntiles / 4)) s *= 2;
  return s;
}

bool attn_lds_supported(int64_t T, int64_t Dh) {
  if (T <= 0 || T > 256) return false;
  if (Dh != 32 && Dh != 64 && Dh != 128) return false;
  const size_t need = Dh == 128 ? dkv_lds_bytes<128>((int)T) : Dh == 64 ? dkv_lds_bytes<64>((int)T)
                                                                            : dkv_lds_bytes<32>((int)T);
  return need <= 160 * 1024;
}

template <int DH>
static hipError_t fwd_t(AttnLdsArgs& a, hipStream_t s) {
  const int nq = (int)cdiv(a.T, 16);
  a.nsplit = pick_split(a.B * a.H, nq);
  const size_t lds = fwd_lds_bytes<DH>((int)a.T);
  hipLaunchKernelGGL((attn_fwd_lds_kernel<DH>), dim3((unsigned)a.nsplit, (unsigned)(a.B * a.H)), dim3(NT), lds, s,
                     a);
  return hipGetLastError();
}

// Causal backward work plan.  Round robin gives a wave one whole tile: the dQ tile of the last queries
// scans every key (13 key tiles at T = 200) while the mean is half that, and the workgroup waits for its
// longest wave.  Here the longest tiles (up to `slots` of them) are cut in two halves of their chunk range
// -- the lower half's wave leaves a partial in an LDS slot for the upper half's wave, which adds it and
// writes the tile -- and the items are dealt longest-first to the least-loaded wave, writers first in each
// wave's list (a reader only ever waits for a writer, so there is no cycle).  Measured at B = 128, T = 200
// (tools/micro/attn_bwd_phase.hip): the slowest wave did ~2x the mean work; balanced, the dK/dV pass's
// slowest wave went 14.5 -> 12.5 us, the dQ pass's barely moved -- with every wave busy the workgroup is
// bound by the CU's LDS operand traffic (one 1 KB fragment read per MFMA), not by its longest wave.
#define LOADER_HANDICAP 3   // plan chunks the loader's staging stream is worth
struct PlanItem {
  int tile, cb, ce, role, slot;
};

static bool make_plan(AttnLdsArgs& a, int ntiles, bool dkv, int slots) {
  const int T = (int)a.T, nqc = (T + 31) / 32;
  if (a.nsplit > PLAN_S) return false;
  memset(a.plan, 0, sizeof(a.plan));
  for (int sp = 0; sp < a.nsplit; ++sp) {
    PlanItem items[64];
    int n = 0;
    for (int t = sp; t < ntiles; t += a.nsplit) {
      if (n >= 32) return false;
      items[n++] = dkv ? PlanItem{t, t / 2, nqc, 0, 0} : PlanItem{t, 0, (t + 2) / 2, 0, 0};
    }
    std::sort(items, items + n, [](const PlanItem& x, const PlanItem& y) {
      return x.ce - x.cb != y.ce - y.cb ? x.ce - x.cb > y.ce - y.cb : x.tile < y.tile;
    });
    const int n0 = n;
    for (int k = 0, used = 0; k < n0 && used < slots; ++k) {
      PlanItem& it = items[k];
      const int w = it.ce - it.cb;
      if (w < 2) break;
      const int hmid = it.cb + (w + 1) / 2;
      // lower half: writer (its chunks are staged first, so it starts early); upper half: reader (dealt last)
      items[n++] = PlanItem{it.tile, hmid, it.ce, 2, used};
      it.ce = hmid;
      it.role = 1;
      it.slot = used++;
    }
    std::sort(items, items + n, [](const PlanItem& x, const PlanItem& y) {
      return x.ce - x.cb != y.ce - y.cb ? x.ce - x.cb > y.ce - y.cb : x.tile < y.tile;
    });
    int load[NW] = {0}, cnt[NW] = {0};
    load[LOADER] = LOADER_HANDICAP;   // the loader wave streams the operand images first
    PlanItem lists[NW][PLAN_I];
    for (int k = 0; k < n; ++k) {
      int w = 0;
      for (int j = 1; j < NW; ++j)
        if (load[j] < load[w]) w = j;
      if (cnt[w] == PLAN_I) return false;
      lists[w][cnt[w]++] = items[k];
      load[w] += items[k].ce - items[k].cb;
    }
    for (int w = 0; w < NW; ++w) {
      int o = 0;
      for (int pass = 0; pass < 3; ++pass) {     // writers, whole tiles, readers
        const int want = pass == 0 ? 1 : pass == 1 ? 0 : 2;
        for (int k = 0; k < cnt[w]; ++k) {
          const PlanItem& it = lists[w][k];
          if (it.role != want) continue;
          a.plan[sp][w][o++] = 1u << 31 | (uint32_t)it.slot << 26 | (uint32_t)it.role << 24 |
                               (uint32_t)it.ce << 16 | (uint32_t)it.cb << 8 | (uint32_t)it.tile;
        }
      }
    }
  }
  return true;
}

// host-only view of the causal backward plan (tests/test_attn_plan.py checks its invariants on the CPU)
extern "C" int rs_attn_bwd_plan(int64_t B, int64_t T, int64_t H, int dkv, uint32_t* plan, int* nsplit) {
  if (B <= 0 || T <= 0 || H <= 0 || !plan || !nsplit) return RS_ERR_ARG;
  AttnLdsArgs a = {};
  a.B = B; a.T = T; a.H = H; a.mask_kind = 0;
  const int nq = (int)cdiv(T, 16);
  a.nsplit = pick_split_bwd(B * H, nq);
  *nsplit = a.nsplit;
  const bool ok = nq >= 8 && make_plan(a, nq, dkv != 0, dkv ? DKV_SLOTS : DQ_SLOTS);
  memcpy(plan, a.plan, sizeof(a.plan));
  return ok ? 0 : RS_ERR_UNSUPPORTED;
}

template <int DH>
static hipError_t bwd_t(AttnLdsArgs& a, hipStream_t s) {
  const int nq = (int)cdiv(a.T, 16);
  a.nsplit = pick_split_bwd(a.B * a.H, nq);
  constexpr int DT = DH / 16;
  const size_t lds_q = fwd_lds_bytes<DH>((int)a.T), lds_kv = dkv_lds_bytes<DH>((int)a.T);
  const size_t ext_q = (size_t)DQ_SLOTS * DT * 4 * 64 * 4 + 16, ext_kv = (size_t)DKV_SLOTS * 2 * DT * 4 * 64 * 2 + 16;
  AttnLdsArgs aq = a, akv = a;
  // only long causal sequences: at T = 50 (4 tiles) the split halves cost more than the imbalance they remove
  const bool want = a.mask_kind == 0 && nq >= 8;
  aq.use_plan = want && lds_q + ext_q <= 160 * 1024 && make_plan(aq, nq, false, DQ_SLOTS);
  akv.use_plan = want && lds_kv + ext_kv <= 160 * 1024 && make_plan(akv, nq, true, DKV_SLOTS);
  const size_t bq = lds_q + (aq.use_plan ? ext_q : 0), bkv = lds_kv + (akv.use_plan ? ext_kv : 0);
  hipLaunchKernelGGL((attn_bwd_lds_kernel<DH>), dim3((unsigned)(2 * a.nsplit * a.B * a.H)), dim3(NT),
                     std::max(bq, bkv), s, aq, akv);
  return hipGetLastError();
}

template <int DH>
static void set_lds_limits() {
  hipFuncSetAttribute((const void*)attn_fwd_lds_kernel<DH>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipFuncSetAttribute((const void*)attn_bwd_lds_kernel<DH>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

static void init_once() {
  static bool done = false;
  if (!done) {
    set_lds_limits<32>();
    set_lds_limits<64>();
    set_lds_limits<128>();
    done = true;
  }
}

hipError_t attn_lds_fwd(int64_t B, int64_t T, int64_t H, int64_t Dh, const void* q, int64_t ldq, const void* k,
                        int64_t ldk, const void* v, int64_t ldv, void* o, int64_t ldo, float* lse, float scale,
                        int mask_kind, const int64_t* ids, float drop_p, uint64_t seed, const uint64_t* seed_base,
                        hipStream_t s) {
  init_once();
  AttnLdsArgs a = {};
  a.B = B; a.T = T; a.H = H;
  a.q = (const bf16*)q; a.ldq = ldq; a.k = (const bf16*)k; a.ldk = ldk; a.v = (const bf16*)v; a.ldv = ldv;
  a.out = (bf16*)o; a.ldout = ldo; a.lse = lse; a.scale = scale; a.mask_kind = mask_kind; a.ids = ids;
  a.drop_p = drop_p; a.seed = seed; a.seed_base = seed_base;
  if (Dh == 128) return fwd_t<128>(a, s);
  if (Dh == 64) return fwd_t<64>(a, s);
  return fwd_t<32>(a, s);
}

hipError_t attn_lds_bwd(int64_t B, int64_t T, int64_t H, int64_t Dh, const void* q, int64_t ldq, const void* k,
                        int64_t ldk, const void* v, int64_t ldv, const void* o, int64_t ldo, const void* dout,
                        int64_t lddo, const float* lse, void* dq, int64_t lddq, void* dk, int64_t lddk, void* dv,
                        int64_t lddv, float scale, int mask_kind, const int64_t* ids, float drop_p, uint64_t seed,
                        const uint64_t* seed_base, float* delta, hipStream_t s) {
  init_once();
  AttnLdsArgs a = {};
  a.B = B; a.T = T; a.H = H;
  a.delta_in = (mask_kind & RS_ATTN_DELTA_IN) != 0;
  mask_kind &= ~RS_ATTN_DELTA_IN;
  a.q = (const bf16*)q; a.ldq = ldq; a.k = (const bf16*)k; a.ldk = ldk; a.v = (const bf16*)v; a.ldv = ldv;
  a.o = (const bf16*)o; a.ldo = ldo; a.dout = (const bf16*)dout; a.lddo = lddo;
  a.dq = (bf16*)dq; a.lddq = lddq; a.dk = (bf16*)dk; a.lddk = lddk; a.dv = (bf16*)dv; a.lddv = lddv;
  a.lse = const_cast<float*>(lse); a.delta = delta; a.scale = scale; a.mask_kind = mask_kind; a.ids = ids;
  a.drop_p = drop_p; a.seed = seed; a.seed_base = seed_base;
  a.ks = kstamp_next(RS_STAMP_ATTN_BWD);
  if (Dh == 128) return bwd_t<128>(a, s);
  if (Dh == 64) return bwd_t<64>(a, s);
  return bwd_t<32>(a, s);
}
