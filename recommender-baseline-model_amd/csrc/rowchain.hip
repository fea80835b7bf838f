// Wave-resident row chains for the SASRec sublayers (bf16, gfx950): the kernels behind
// rs_sas_block_in / rs_sas_block_out / rs_sas_block_out_bwd / rs_sas_block_in_bwd.
//
// Everything in a SAS block except the attention core is row-local (BS/models/sas_model/sas.py:73-76 before the
// core: Q = LN1(x), q = Q Wq^T + bq, kv = x Wkv^T + bkv; sas.py:75-84 after it: x1 = Q + O Wo^T + bo, z = LN2(x1),
// h1 = relu(drop(z W1^T + b1)), x' = (drop(h1 W2^T + b2) + z) * (ids != 0), PointWiseFeedForward sas.py:8-24).
// The saved tensors, their layout and every dropout index (m*d + n per site salt) are those of the generic
// kernels (fp32 parity mode, other widths).  Laid out for the CDNA4 execution model:
//
//  * one workgroup per CU (NW = 8 waves) stages the block's three d x d weight matrices ONCE
//    into LDS (110 KB at d = 128), then every wave runs its own 16-token chain with no
//    workgroup barrier: 16-row tiles are dealt round robin over the workgroups of each XCD, each
//    XCD taking one eighth of the rows (tiles_of_wave), so at cfg2 (1,600 tiles) every CU gets 6-7
//    of them instead of one or two 64-row tiles (400 tiles on 256 CUs);
//  * the activations never leave registers: every GEMM is computed TRANSPOSED,
//    Y^T = W . X^T, with the weight as the MFMA A operand (LDS) and the 16 tokens as the B
//    operand, so the accumulator (lane (g, cl) holds feature 16j + 4g + r of token cl) packed
//    pairwise to bf16 IS the next GEMM's B operand: the k order inside a 32-deep step is then
//    {4g + e, 16 + 4g + e}, and the weights are staged into LDS with that permutation
//    (conflict-free ds_read_b128 at a 32-byte row pad);
//  * a token's features sit on one lane group (4 lanes x D/4 values), so LayerNorm's row
//    statistics are 2 cross-group shuffles;
//  * global loads/stores of activations use the same layout (8 bytes per lane per 16
//    features), LayerNorm affine partials accumulate per lane over the wave's tiles and are
//    reduced once per workgroup (partial set = workgroup: rs_sas_block_parts sets).
#include "common.h"
#include "../../include/recsys_hip.h"

namespace rc {

// phase timestamps for tools/micro/rowchain_phase.hip (compiled out of the library)
#ifdef RC_PROF
__device__ unsigned long long g_rc_prof[4096 * 8 * 16];
#define RCPROF(slot)                                                                                 \
  do {                                                                                               \
    if ((threadIdx.x & 63) == 0) g_rc_prof[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 16 + (slot)] = wall_clock64(); \
  } while (0)
#else
#define RCPROF(slot) \
  do {               \
  } while (0)
#endif

#ifndef RC_HEAD_PREFETCH
#define RC_HEAD_PREFETCH 1   // head item-row loads: 0 tile start, 1 mid-chain (A/B 0.2999 vs 0.3020 ms at cfg2), 2 after the chain, 3 ids at the start + rows mid-chain (18 VGPRs spilled: 0.2975 vs 0.2953)
#endif

#ifndef RC_NOSTORE
#define RC_NOSTORE 0   // tools/micro/rowchain_phase.hip: 1 = skip block_out's saved-tensor stores (cost probe)
#endif

typedef __bf16 bf16;
typedef __attribute__((address_space(3))) void* lds_ptr;

constexpr int NW = 8;                 // waves per workgroup
constexpr int NT = 64 * NW;
constexpr int TR = 16;                // tokens per wave tile

template <int D> struct Lay {
  static constexpr int J = D / 16;    // accumulator tiles per token row
  static constexpr int S = D / 32;    // 32-deep k steps = 16-byte chunks per lane per row
  static constexpr int CPR = D / 8;   // 16-byte chunks per weight row
  static constexpr int WBYTES = D * D * 2;
};

// Feature convention: lane (g, cl) holds token cl; accumulator tile j = 2s + h, element r holds feature
// 32s + 8g + 4h + r, i.e. step s's 8 features 32s + 8g .. +7 are contiguous (one 16-byte global access, one
// natural-order B fragment).  The MFMA writes tile j, lane g, element r to output row 16j + 4g + r, so the
// weight rows are staged in the order perm(n) = 32(n >> 5) + 8((n >> 2) & 3) + 4((n >> 4) & 1) + (n & 3).
__device__ __forceinline__ int perm_row(int n) { return 32 * (n >> 5) + 8 * ((n >> 2) & 3) + 4 * ((n >> 4) & 1) + (n & 3); }
// LDS weight image: unpadded rows, 16-byte chunk c of row n stored at chunk c ^ swz(n) (conflict-free
// ds_read_b128 of the A fragments: rows 16j + cl, chunk 4s + g)
template <int D> __device__ __forceinline__ int swz(int n) { return (n / (128 / D)) & (Lay<D>::CPR - 1); }

// stage NM weight matrices ([D rows][D] at row stride ldw each) into LDS by LDS-DMA (global_load_lds_dwordx4:
// lane-linear 1 KB per wave instruction, so the swizzle and row permutation go on the source address)
template <int D, int NM>
__device__ __forceinline__ void stage_w(char* lds, const bf16* const (&W)[NM], const int64_t (&ldw)[NM], int wave,
                                        int lane) {
  constexpr int IPM = Lay<D>::WBYTES / 1024, CPR = Lay<D>::CPR;
  static_assert(NM * IPM % NW == 0, "staging split");
#pragma unroll
  for (int u = 0; u < NM * IPM / NW; ++u) {
    const int q = wave + NW * u, mtx = q / IPM, qi = q % IPM;
    const int idx = qi * 64 + lane, n = idx / CPR, pc = idx % CPR, lc = pc ^ swz<D>(n);
    const bf16* src = W[mtx] + (int64_t)perm_row(n) * ldw[mtx] + 8 * lc;
    __builtin_amdgcn_global_load_lds(src, (lds_ptr)(lds + mtx * Lay<D>::WBYTES + qi * 1024), 16, 0, 0);
  }
}
// NV fp32 vectors of D (bias, LN affine) -> LDS, plain loads
template <int D, int NV>
__device__ __forceinline__ void stage_v(float* lv, const float* const (&V)[NV], int tid) {
  for (int i = tid; i < NV * D; i += NT) lv[i] = V[i / D][i % D];
}

// activations of 16 tokens: Act in fp32 (tile j = 2s + h, element r), Raw as stored (bf16, step s, element
// 4h + r) -- both hold features 32s + 8g + 4h + r of token cl
template <int D> struct Act { f32x4 v[Lay<D>::J]; };
template <int D> struct Raw { bf16x8 v[Lay<D>::S]; };

template <int D>
__device__ __forceinline__ void load_raw(Raw<D>& a, const bf16* base, int64_t ld, int64_t m, int g) {
  const bf16* p = base + m * ld + 8 * g;
#pragma unroll
  for (int s = 0; s < Lay<D>::S; ++s) a.v[s] = *reinterpret_cast<const bf16x8*>(p + 32 * s);
}
template <int D>
__device__ __forceinline__ void to_act(Act<D>& a, const Raw<D>& r) {
#pragma unroll
  for (int j = 0; j < Lay<D>::J; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) a.v[j][e] = (float)r.v[j >> 1][4 * (j & 1) + e];
}
// round to bf16 (the stored value) and keep both forms
template <int D>
__device__ __forceinline__ void round_act(Act<D>& a, Raw<D>& r) {
#pragma unroll
  for (int j = 0; j < Lay<D>::J; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      r.v[j >> 1][4 * (j & 1) + e] = (bf16)a.v[j][e];
      a.v[j][e] = (float)r.v[j >> 1][4 * (j & 1) + e];
    }
}
template <int D>
__device__ __forceinline__ void store_raw(bf16* base, int64_t ld, int64_t m, bool ok, const Raw<D>& r, int g) {
  if (!ok) return;
  bf16* p = base + m * ld + 8 * g;
#pragma unroll
  for (int s = 0; s < Lay<D>::S; ++s) *reinterpret_cast<bf16x8*>(p + 32 * s) = r.v[s];
}
// acc[j] += W[feature of (j, g, r)][:] . x[token cl][:]  (W staged at wl)
// Two-stage pipeline over the output tiles: tile j+1's fragments are read while tile j's MFMAs run, and the
// scheduler may not batch more (all fragments of a chain in flight spill at d = 128).
template <int D>
__device__ __forceinline__ void mm(const bf16* wl, const Raw<D>& b, Act<D>& acc, int lane) {
  constexpr int J = Lay<D>::J, S = Lay<D>::S;
  const int g = lane >> 4, cl = lane & 15;
  auto frag = [&](int j, int s) {
    const int n = 16 * j + cl;
    return *reinterpret_cast<const bf16x8*>(wl + n * D + 8 * ((4 * s + g) ^ swz<D>(n)));
  };
  bf16x8 f[2][S];
#pragma unroll
  for (int s = 0; s < S; ++s) f[0][s] = frag(0, s);
#pragma unroll
  for (int j = 0; j < J; ++j) {
    if (j + 1 < J) {
#pragma unroll
      for (int s = 0; s < S; ++s) f[(j + 1) & 1][s] = frag(j + 1, s);
    }
#pragma unroll
    for (int s = 0; s < S; ++s)
      acc.v[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[j & 1][s], b.v[s], acc.v[j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}
template <int D>
__device__ __forceinline__ void zero(Act<D>& a) {
#pragma unroll
  for (int j = 0; j < Lay<D>::J; ++j) a.v[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
}
// this lane's 4 values of tile j of a staged fp32 vector
template <int D>
__device__ __forceinline__ f32x4 vec4(const float* lv, int j, int g) {
  return *reinterpret_cast<const f32x4*>(lv + 32 * (j >> 1) + 8 * g + 4 * (j & 1));
}
__device__ __forceinline__ int feat(int j, int g, int r) { return 32 * (j >> 1) + 8 * g + 4 * (j & 1) + r; }
// sum over the token's features: this lane's values, then the other 3 lane groups
__device__ __forceinline__ float row_sum(float s) { return add_xor32(add_xor16(s)); }   // xor 16, then 32 (all lanes active)

// torch.nn.LayerNorm (biased variance, eps inside the sqrt), in place; returns (mean, rstd)
template <int D>
__device__ __forceinline__ void ln_fwd(Act<D>& x, const float* gw, const float* gb, float eps, int g, float& mu,
                                       float& rs) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < Lay<D>::J; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) s += x.v[j][e];
  mu = row_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < Lay<D>::J; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float u = x.v[j][e] - mu;
      q += u * u;
    }
  rs = 1.0f / sqrtf(row_sum(q) / (float)D + eps);
#pragma unroll
  for (int j = 0; j < Lay<D>::J; ++j) {
    const f32x4 w = vec4<D>(gw, j, g), b = vec4<D>(gb, j, g);
#pragma unroll
    for (int e = 0; e < 4; ++e) x.v[j][e] = (x.v[j][e] - mu) * rs * w[e] + b[e];
  }
}

// sum over the 16 lanes of a DPP row (the 16 tokens of a lane group): common.h row16_sum_up, the xor butterfly's
// bits from DPP operand moves instead of __shfl_xor's ds_bpermute_b32 (~260 LDS-crossbar round trips per tile in the
// LayerNorm backwards).  Every caller runs with all 64 lanes active (wave-uniform tile loops).
__device__ __forceinline__ float row16_sum(float v) { return row16_sum_up(v); }

// LayerNorm backward (layernorm.hip ln_bwd, VAR 0), in place on dy: t = rstd*(dy*g - mean(dy*g))
// - rstd^3*mean(dy*g*u)*u, u = x - mean (x as stored, bf16); dy zeroed on invalid tokens.  The dgamma/dbeta
// terms of the tile's 16 tokens are summed by an xor tree over the lanes of a group as they are formed and added
// to the wave's own LDS row red[wave][2][D] (no other wave touches it before ln_partials' barrier)
template <int D>
__device__ __forceinline__ void ln_bwd(Act<D>& dy, const Raw<D>& xr, bool valid, const float* gw, float mu, float a,
                                       float* red, int lane, int wave) {
  const int g = lane >> 4, cl = lane & 15;
  float* rw = red + wave * 2 * D;
  float sg = 0.f, sgu = 0.f;
#pragma unroll
  for (int j = 0; j < Lay<D>::J; ++j) {
    const f32x4 w = vec4<D>(gw, j, g);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float gy = valid ? dy.v[j][e] : 0.f;
      const float u = (float)xr.v[j >> 1][4 * (j & 1) + e] - mu;
      const float gq = gy * w[e];
      const float pg = row16_sum(gy * (u * a)), pb = row16_sum(gy);
      if (cl == 0) {
        rw[feat(j, g, e)] += pg;
        rw[D + feat(j, g, e)] += pb;
      }
      sg += gq;
      sgu += gq * u;
      dy.v[j][e] = gq;   // dy*g for now
    }
  }
  sg = row_sum(sg);
  sgu = row_sum(sgu);
  const float mg = sg / (float)D, coef = a * a * a * sgu / (float)D;
#pragma unroll
  for (int j = 0; j < Lay<D>::J; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      dy.v[j][e] = a * (dy.v[j][e] - mg) - coef * ((float)xr.v[j >> 1][4 * (j & 1) + e] - mu);
}

__device__ __forceinline__ void ln_zero(float* red, int D, int lane, int wave) {
  for (int i = lane; i < 2 * D; i += 64) red[wave * 2 * D + i] = 0.f;
}
// the workgroup's partial set (waves summed in order 0..NW-1) -> part[blockIdx.x][2][D]
template <int D>
__device__ __forceinline__ void ln_partials(const float* red, float* part, int tid) {
  __syncthreads();
  if (tid < 2 * D) {
    const int which = tid / D, c = tid % D;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[(w * 2 + which) * D + c];
    part[((int64_t)blockIdx.x * 2 + which) * D + c] = s;
  }
}

__device__ __forceinline__ int64_t n_tiles(int64_t M) { return (M + TR - 1) / TR; }

// The tiles of one wave: first, first + step, ... < end.  XCD-contiguous dealing: workgroup w runs on XCD w % 8
// (blocks are dealt round-robin over the 8 XCDs: measured fixed, block b on XCC b % 8, tools/micro/xcd_probe.hip),
// so XCD x takes the x-th eighth of the tiles -- the rows of sequences [x B / 8, (x + 1) B / 8) when 128 divides
// M -- which is the sequence range the attention kernels give the same XCD (attention_lds.hip block_coords).  A
// tensor one of them writes is then read by the other from that XCD's L2 (a 64 KB burst per workgroup right after
// its producer: 1.24 us XCD-local against 2.6 us from another XCD, xcd_probe).  Placement is for speed only: every
// tile has exactly one owner whatever the placement.
struct TileRange {
  int64_t first, step, end;
};
__device__ __forceinline__ TileRange tiles_of_wave(int64_t nt, int wave) {
  const int64_t G = gridDim.x, w = blockIdx.x;
  if (G >= 8 && G % 8 == 0) {
    const int64_t x = w & 7, Gx = G >> 3;
    return TileRange{x * nt / 8 + (w >> 3) + Gx * wave, Gx * NW, (x + 1) * nt / 8};
  }
  return TileRange{w + G * wave, G * NW, nt};
}

// ------------------------------------------------------------------ LDS layout
// NM weight images, then NV fp32 vectors of D, then NR LayerNorm partial blocks red[NW][2][D]
template <int D, int NM, int NV, int NR> struct Smem {
  static constexpr size_t W = (size_t)NM * Lay<D>::WBYTES;
  static constexpr size_t V = W + (size_t)NV * D * 4;
  static constexpr size_t BYTES = V + (size_t)NR * NW * 2 * D * 4;
};
__device__ __forceinline__ const bf16* wslot(const char* smem, int i, int wbytes) {
  return reinterpret_cast<const bf16*>(smem + (size_t)i * wbytes);
}

// per-tile context: this wave's 16 tokens
struct Tile {
  int64_t m, mc;   // this lane's token row, clamped for loads
  bool ok;         // row < M
};
__device__ __forceinline__ Tile tile_of(int64_t t, int64_t M, int cl) {
  Tile x;
  x.m = t * TR + cl;
  x.ok = x.m < M;
  x.mc = x.ok ? x.m : M - 1;
  return x;
}
// ------------------------------------------------------------------ chain stages (one 16-token tile per wave)
// Forward, block input side (sas.py:73-76): Q = LN1(x) [saved], q = Q Wq^T + bq.  Weights/vectors: Wq at wq;
// lv: ln1_w, ln1_b, bq, bk, bv (5 x D).  Returns nothing; k/v follow in fwd_in_kv.
template <int D>
__device__ __forceinline__ void fwd_in_q(const Raw<D>& xr, const Tile& T, const bf16* wq, const float* lv, float eps,
                                         bf16* Q, float* mean, float* rstd, bf16* q, int lane) {
  const int g = lane >> 4;
  Act<D> y;
  to_act<D>(y, xr);
  float mu, rs;
  ln_fwd<D>(y, lv, lv + D, eps, g, mu, rs);
  Raw<D> Qr;
  round_act<D>(y, Qr);
  store_raw<D>(Q, D, T.m, T.ok, Qr, g);
  if (T.ok && g == 0) {
    mean[T.m] = mu;
    rstd[T.m] = rs;
  }
  Act<D> acc;
  zero<D>(acc);
  mm<D>(wq, Qr, acc, lane);
#pragma unroll
  for (int j = 0; j < Lay<D>::J; ++j) acc.v[j] += vec4<D>(lv + 2 * D, j, g);
  Raw<D> r;
  round_act<D>(acc, r);
  store_raw<D>(q, D, T.m, T.ok, r, g);
}
// k, v = x Wk^T + bk, x Wv^T + bv -> kv [M][2D]
template <int D>
__device__ __forceinline__ void fwd_in_kv(const Raw<D>& xr, const Tile& T, const bf16* wk, const bf16* wv,
                                          const float* lv, bf16* kv, int lane) {
  const int g = lane >> 4;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    Act<D> acc;
    zero<D>(acc);
    mm<D>(h == 0 ? wk : wv, xr, acc, lane);
#pragma unroll
    for (int j = 0; j < Lay<D>::J; ++j) acc.v[j] += vec4<D>(lv + (3 + h) * D, j, g);
    Raw<D> r;
    round_act<D>(acc, r);
    store_raw<D>(kv + h * D, 2 * D, T.m, T.ok, r, g);
  }
}

struct OutFwd {
  bf16 *x1, *z, *h1, *xn;
  float *mean, *rstd;
  const int64_t* ids;
  float drop_p, eps;
  uint32_t s1, s2;
};
// dropout multipliers of this lane's 4 features of tile j (pairs share one hash, as drop_mul2)
__device__ __forceinline__ void drop4(float p, uint32_t s32, int64_t m, int D, int j, int g, float (&dm)[4]) {
  const uint64_t idx = (uint64_t)(m * D + feat(j, g, 0));
  drop_mul2(p, s32, idx, dm[0], dm[1]);
  drop_mul2(p, s32, idx + 2, dm[2], dm[3]);
}
// Forward, block output side part 1 (sas.py:75-80): x1 = Q + o Wo^T + bo [saved], z = LN2(x1) [saved],
// h1 = relu(drop(z W1^T + b1)) [saved].  lv: bo, ln2_w, ln2_b, b1, b2.
template <int D>
__device__ __forceinline__ void fwd_out_a(const Raw<D>& orr, const Raw<D>& Qr, const Tile& T, const bf16* wo,
                                          const bf16* w1, const float* lv, const OutFwd& o, Raw<D>& zr, Raw<D>& hr,
                                          int lane) {
  const int g = lane >> 4;
  Act<D> acc;
  Raw<D> r;
  zero<D>(acc);
  mm<D>(wo, orr, acc, lane);
#pragma unroll
  for (int j = 0; j < Lay<D>::J; ++j) {
    const f32x4 bb = vec4<D>(lv, j, g);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc.v[j][e] = acc.v[j][e] + bb[e] + (float)Qr.v[j >> 1][4 * (j & 1) + e];
  }
  round_act<D>(acc, r);
  if (!RC_NOSTORE) store_raw<D>(o.x1, D, T.m, T.ok, r, g);
  float mu, rs;
  ln_fwd<D>(acc, lv + D, lv + 2 * D, o.eps, g, mu, rs);
  round_act<D>(acc, zr);
  if (!RC_NOSTORE) store_raw<D>(o.z, D, T.m, T.ok, zr, g);
  if (T.ok && g == 0) {
    o.mean[T.m] = mu;
    o.rstd[T.m] = rs;
  }
  zero<D>(acc);
  mm<D>(w1, zr, acc, lane);
  const bool drop = o.drop_p > 0.f;
#pragma unroll
  for (int j = 0; j < Lay<D>::J; ++j) {
    float dm[4] = {1.f, 1.f, 1.f, 1.f};
    if (drop) drop4(o.drop_p, o.s1, T.m, D, j, g, dm);
    const f32x4 bb = vec4<D>(lv + 3 * D, j, g);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc.v[j][e] = fmaxf(acc.v[j][e] + bb[e], 0.f) * dm[e];
  }
  round_act<D>(acc, hr);
  if (!RC_NOSTORE) store_raw<D>(o.h1, D, T.m, T.ok, hr, g);
}
// part 2 (sas.py:81-84): x' = (drop(h1 W2^T + b2) + z) * (ids != 0) [saved] -> xr
template <int D>
__device__ __forceinline__ void fwd_out_b(const Raw<D>& hr, const Raw<D>& zr, const Tile& T, const bf16* w2,
                                          const float* lv, const OutFwd& o, Raw<D>& xr, int lane) {
  const int g = lane >> 4;
  const bool keep = T.ok && o.ids[T.mc] != 0;
  Act<D> acc;
  zero<D>(acc);
  mm<D>(w2, hr, acc, lane);
  const bool drop = o.drop_p > 0.f;
#pragma unroll
  for (int j = 0; j < Lay<D>::J; ++j) {
    float dm[4] = {1.f, 1.f, 1.f, 1.f};
    if (drop) drop4(o.drop_p, o.s2, T.m, D, j, g, dm);
    const f32x4 bb = vec4<D>(lv + 4 * D, j, g);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float v = __builtin_fmaf(acc.v[j][e] + bb[e], dm[e], (float)zr.v[j >> 1][4 * (j & 1) + e]);
      acc.v[j][e] = keep ? v : 0.f;
    }
  }
  round_act<D>(acc, xr);
  store_raw<D>(o.xn, D, T.m, T.ok, xr, g);
}

// Backward, block input side (sas.py:73-76 reversed), part 1: dx_kv = dk Wk + dv Wv (WkT, WvT images)
template <int D>
__device__ __forceinline__ void bwd_in_a(const Raw<D>& kr, const Raw<D>& vr, const bf16* wk, const bf16* wv,
                                         Raw<D>& dxkv, int lane) {
  Act<D> acc;
  zero<D>(acc);
  mm<D>(wk, kr, acc, lane);
  mm<D>(wv, vr, acc, lane);
  round_act<D>(acc, dxkv);
}
// part 2: dQ = dq Wq + dx1; dx = dx_kv + LN1'(x, dQ) (+ affine partials into red) -> dxr
template <int D>
__device__ __forceinline__ void bwd_in_b(const Raw<D>& qr, const Raw<D>& rr, const Raw<D>& xr, const Raw<D>& dxkv,
                                         const Tile& T, float mu, float rs, const bf16* wq, const float* lnw,
                                         float* red, Raw<D>& dxr, int lane, int wave) {
  const int g = lane >> 4;
  Act<D> dQ;
  Raw<D> r;
  to_act<D>(dQ, rr);
  mm<D>(wq, qr, dQ, lane);
  round_act<D>(dQ, r);
  ln_bwd<D>(dQ, xr, T.ok, lnw, mu, rs, red, lane, wave);
#pragma unroll
  for (int j = 0; j < Lay<D>::J; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) dQ.v[j][e] += (float)dxkv.v[j >> 1][4 * (j & 1) + e];
  round_act<D>(dQ, dxr);
}

struct OutBwd {
  bf16 *dy2, *da1, *dx1, *dout;
  float* delta;   // optional: delta[m] = rowsum(dout * o), the attention backward's row term (one head)
  const int64_t* ids;
  float drop_p;
  uint32_t s1, s2;
};
// Backward, block output side (sas.py:75-84 reversed), part 1: dzres = dxn*mask; dy2 = drop2(dzres) [saved];
// da1 = relu'(h1) * drop1(dy2 W2) [saved] -> dz (holding dzres), dar (da1)
template <int D>
__device__ __forceinline__ void bwd_out_a(const Raw<D>& dr, const Raw<D>& hr, const Tile& T, const bf16* w2,
                                          const OutBwd& o, Raw<D>& dzr, Raw<D>& dar, int lane) {
  const int g = lane >> 4;
  const bool keep = T.ok && o.ids[T.mc] != 0;
  const bool drop = o.drop_p > 0.f;
  Act<D> acc;
  Raw<D> r;
#pragma unroll
  for (int j = 0; j < Lay<D>::J; ++j) {
    float dm[4] = {1.f, 1.f, 1.f, 1.f};
    if (drop) drop4(o.drop_p, o.s2, T.m, D, j, g, dm);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bf16 v = keep ? dr.v[j >> 1][4 * (j & 1) + e] : (bf16)0.f;
      dzr.v[j >> 1][4 * (j & 1) + e] = v;
      acc.v[j][e] = (float)v * dm[e];
    }
  }
  round_act<D>(acc, r);
  store_raw<D>(o.dy2, D, T.m, T.ok, r, g);
  zero<D>(acc);
  mm<D>(w2, r, acc, lane);
#pragma unroll
  for (int j = 0; j < Lay<D>::J; ++j) {
    float dm[4] = {1.f, 1.f, 1.f, 1.f};
    if (drop) drop4(o.drop_p, o.s1, T.m, D, j, g, dm);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc.v[j][e] = ((float)hr.v[j >> 1][4 * (j & 1) + e] > 0.f ? acc.v[j][e] : 0.f) * dm[e];
  }
  round_act<D>(acc, dar);
  store_raw<D>(o.da1, D, T.m, T.ok, dar, g);
}
// part 2: dz = da1 W1 + dzres; dx1 = LN2'(x1, dz) [saved, + affine partials into red]; dout = dx1 Wo [saved];
// with o.delta: delta = rowsum(dout * O) of the stored (bf16) values, O = the attention output (orr)
template <int D>
__device__ __forceinline__ void bwd_out_b(const Raw<D>& dar, const Raw<D>& xr, const Raw<D>& dzr, const Raw<D>& orr,
                                          const Tile& T, float mu, float rs, const bf16* w1, const bf16* wo,
                                          const float* lnw, const OutBwd& o, float* red, int lane, int wave) {
  const int g = lane >> 4;
  Raw<D> r;
  Act<D> dz;
  to_act<D>(dz, dzr);
  mm<D>(w1, dar, dz, lane);
  round_act<D>(dz, r);
  ln_bwd<D>(dz, xr, T.ok, lnw, mu, rs, red, lane, wave);
  round_act<D>(dz, r);
  store_raw<D>(o.dx1, D, T.m, T.ok, r, g);
  Act<D> acc;
  zero<D>(acc);
  mm<D>(wo, r, acc, lane);
  round_act<D>(acc, r);
  store_raw<D>(o.dout, D, T.m, T.ok, r, g);
  if (o.delta) {
    float dl = 0.f;
#pragma unroll
    for (int s = 0; s < Lay<D>::S; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) dl = __builtin_fmaf((float)r.v[s][e], (float)orr.v[s][e], dl);
    dl = row_sum(dl);
    if (T.ok && g == 0) o.delta[T.m] = dl;
  }
}

// ------------------------------------------------------------------ single-block kernels
// The SAS embedding stage folded into the first block's input kernel (rs_sas_block_in_embed): the tile's
// x = (item_emb[ids]·scale + pos_emb[t]) → dropout → ·(ids != 0) is formed in registers exactly as
// embed_fwd_kernel forms it (same expression, same hash index r·d + c), stored (x0, the backward's LN1 input) and
// fed to the chain; each workgroup also counts its tiles' valid positions (count_ids != 0) into
// count_parts[workgroup] (the head kernel's 256 workgroups then load one word per thread, not a dependent chain of 8).
struct EmbIn {
  const int64_t* ids; const bf16* etab; const bf16* ptab; int64_t T;
  float scale, drop_p; uint64_t salt; const uint64_t* seed_base;
  bf16* xout; const int64_t* cnt_ids; int* cnt_parts;
};
struct InArgs {
  int64_t M;
  const bf16* x; int64_t ldx;
  const float* ln_w; const float* ln_b; float eps;
  bf16* Q; float* mean; float* rstd;
  const bf16* Wq; const float* bq; bf16* q;
  const bf16* Wkv; const float* bkv; bf16* kv;
  EmbIn e;                                                  // e.etab == nullptr: x is read
};
template <int D>
__device__ __forceinline__ void embed_tile(Raw<D>& xr, const EmbIn& e, const Tile& T, uint32_t s32, int g) {
  const int64_t id = e.ids[T.mc], t = T.mc % e.T;
  const bf16* ep = e.etab + id * D + 8 * g;
  const bf16* pp = e.ptab + t * D + 8 * g;
  bf16x8 ev[Lay<D>::S], pv[Lay<D>::S];
#pragma unroll
  for (int s = 0; s < Lay<D>::S; ++s) {
    ev[s] = *reinterpret_cast<const bf16x8*>(ep + 32 * s);
    pv[s] = *reinterpret_cast<const bf16x8*>(pp + 32 * s);
  }
  const float keep = id == 0 ? 0.f : 1.f;
#pragma unroll
  for (int s = 0; s < Lay<D>::S; ++s)
#pragma unroll
    for (int k = 0; k < 8; k += 2) {
      float x0 = (float)ev[s][k] * e.scale + (float)pv[s][k];
      float x1 = (float)ev[s][k + 1] * e.scale + (float)pv[s][k + 1];
      if (e.drop_p > 0.f) {
        float m0, m1;
        drop_mul2(e.drop_p, s32, (uint64_t)(T.mc * D + 32 * s + 8 * g + k), m0, m1);
        x0 *= m0;
        x1 *= m1;
      }
      xr.v[s][k] = (bf16)(x0 * keep);
      xr.v[s][k + 1] = (bf16)(x1 * keep);
    }
}

// X -> Q = LN1(X) [saved], q = Q Wq^T + bq, kv = X Wkv^T + bkv
template <int D>
__global__ __launch_bounds__(NT) void block_in_kernel(InArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef Smem<D, 3, 5, 0> L;
  constexpr int WB = Lay<D>::WBYTES;
  const float* lv = reinterpret_cast<const float*>(smem + L::W);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4,
            cl = lane & 15;
  const TileRange tr = tiles_of_wave(n_tiles(a.M), wave);
  int64_t t = tr.first;
  const bool emb = a.e.etab != nullptr;
  const uint32_t es32 = emb && a.e.drop_p > 0.f ? seed32(eff_seed(a.e.salt, a.e.seed_base)) : 0u;
  int cnt = 0;
  auto load_x = [&](Raw<D>& xr, const Tile& T) {
    if (!emb) {
      load_raw<D>(xr, a.x, a.ldx, T.mc, g);
      return;
    }
    // the count's id load goes out with the gathers and is consumed before the x0 store: vmcnt retires in order
    // and counts stores too on gfx950, so a load consumed after a store waits for that store
    const int64_t cid = a.e.cnt_ids && T.ok && g == 0 ? a.e.cnt_ids[T.mc] : 0;
    embed_tile<D>(xr, a.e, T, es32, g);
    if (a.e.cnt_ids) cnt += __popcll(__ballot(cid != 0));
    store_raw<D>(a.e.xout, D, T.m, T.ok, xr, g);
  };
  Raw<D> xr;
  if (t < tr.end) load_x(xr, tile_of(t, a.M, cl));
  {
    const bf16* const W[3] = {a.Wq, a.Wkv, a.Wkv + (int64_t)D * D};
    const int64_t ldw[3] = {D, D, D};
    stage_w<D, 3>(smem, W, ldw, wave, lane);
    const float* const V[5] = {a.ln_w, a.ln_b, a.bq, a.bkv, a.bkv + D};
    stage_v<D, 5>(reinterpret_cast<float*>(smem + L::W), V, tid);
  }
  __syncthreads();
  for (; t < tr.end; t += tr.step) {
    asm volatile("" ::: "memory");   // no hoisting of the loop-invariant weight fragment reads
    const Tile T = tile_of(t, a.M, cl);
    if (t != tr.first) load_x(xr, T);
    fwd_in_q<D>(xr, T, wslot(smem, 0, WB), lv, a.eps, a.Q, a.mean, a.rstd, a.q, lane);
    fwd_in_kv<D>(xr, T, wslot(smem, 1, WB), wslot(smem, 2, WB), lv, a.kv, lane);
  }
  if (emb && a.e.cnt_parts) {   // integer counts: exact in any order
    __shared__ int wcnt[NW];
    if (lane == 0) wcnt[wave] = cnt;
    __syncthreads();
    if (tid == 0) {
      int c = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) c += wcnt[w];
      a.e.cnt_parts[blockIdx.x] = c;
    }
  }
}

// The SAS output head riding in the LAST block's output kernel (rs_sas_block_out_head): every quantity of the head
// is token-local once the BCE divisor is known (the valid-position count, summed from the first block's per-wave
// counts), so each tile's x_L = x' goes on, in registers, through the last LayerNorm (f saved), the tied sampled
// logits <f, E[pos]>, <f, E[neg]>, the BCE gradient (dpl, dnl saved), df = dpl E[pos] + dnl E[neg] and the last
// LayerNorm's backward (dx_L saved for the blocks' backward; affine partials per workgroup, BCE partials sp, sn,
// count per workgroup for the loss statistics).  Same math as head.hip's kernels (sums in this layout's order).
struct HeadArgs {
  const bf16* E; const int64_t* pos; const int64_t* neg;
  const float* gl; const float* bl; float eps;
  const int* cnt_parts; int ncnt; const float* divisor;
  bf16* f; float* pl; float* nl; float* dpl; float* dnl; bf16* dx; float* lnpart; float* part;
};
struct OutArgs {
  int64_t M;
  const bf16* o; const bf16* Q;
  const bf16* Wo; const float* bo; bf16* x1;
  const float* ln_w; const float* ln_b; float eps; bf16* z; float* mean; float* rstd;
  const bf16* W1; const float* b1; bf16* h1;
  const bf16* W2; const float* b2; bf16* xn;
  const int64_t* ids;
  float drop_p; uint64_t salt1, salt2; const uint64_t* seed_base;
  HeadArgs h;                                               // h.E == nullptr: no head
};
__device__ __forceinline__ float h_softplus(float z) { return fmaxf(z, 0.f) + log1pf(__expf(-fabsf(z))); }
__device__ __forceinline__ float h_sigmoid(float z) { return 1.f / (1.f + __expf(-z)); }

// the tile's item rows E[pos], E[neg] (issued at the tile's start: their latency hides behind the block's chain)
template <int D>
__device__ __forceinline__ int64_t head_rows(const HeadArgs& h, const Tile& T, Raw<D>& er, Raw<D>& nr, int g) {
  const int64_t ip = h.pos[T.mc], in = h.neg[T.mc];
  load_raw<D>(er, h.E, D, ip, g);
  load_raw<D>(nr, h.E, D, in, g);
  return ip;
}
template <int D>
__device__ __forceinline__ void head_rows_at(const HeadArgs& h, int64_t ip, int64_t in, Raw<D>& er, Raw<D>& nr,
                                             int g) {
  load_raw<D>(er, h.E, D, ip, g);
  load_raw<D>(nr, h.E, D, in, g);
}
template <int D>
__device__ __forceinline__ void head_tile(const Raw<D>& xr, const Raw<D>& er, const Raw<D>& nr, int64_t ip,
                                          const Tile& T, const float* gl, const float* bl, const HeadArgs& h,
                                          float scale, float* red, float (&acc)[3], int lane, int wave) {
  const int g = lane >> 4;
  Act<D> y;
  to_act<D>(y, xr);
  float mu, rs;
  ln_fwd<D>(y, gl, bl, h.eps, g, mu, rs);
  Raw<D> fr;
  round_act<D>(y, fr);                       // the logits read the stored (bf16) features
  store_raw<D>(h.f, D, T.m, T.ok, fr, g);
  float dp = 0.f, dn = 0.f;
#pragma unroll
  for (int j = 0; j < Lay<D>::J; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      dp += y.v[j][e] * (float)er.v[j >> 1][4 * (j & 1) + e];
      dn += y.v[j][e] * (float)nr.v[j >> 1][4 * (j & 1) + e];
    }
  dp = row_sum(dp);
  dn = row_sum(dn);
  const bool valid = T.ok && ip != 0;
  const float gp = valid ? (h_sigmoid(dp) - 1.f) * scale : 0.f;
  const float gn = valid ? h_sigmoid(dn) * scale : 0.f;
  if (T.ok && g == 0) {
    h.pl[T.m] = dp;
    h.nl[T.m] = dn;
    h.dpl[T.m] = gp;
    h.dnl[T.m] = gn;
    if (ip != 0) {
      acc[0] += h_softplus(-dp);
      acc[1] += h_softplus(dn);
      acc[2] += 1.f;
    }
  }
  Act<D> df;
#pragma unroll
  for (int j = 0; j < Lay<D>::J; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      df.v[j][e] = gp * (float)er.v[j >> 1][4 * (j & 1) + e] + gn * (float)nr.v[j >> 1][4 * (j & 1) + e];
  ln_bwd<D>(df, xr, T.ok, gl, mu, rs, red, lane, wave);
  Raw<D> dr;
  round_act<D>(df, dr);
  store_raw<D>(h.dx, D, T.m, T.ok, dr, g);
}
__device__ __forceinline__ OutFwd out_fwd_of(const OutArgs& a) {
  const bool drop = a.drop_p > 0.f;
  return OutFwd{a.x1, a.z, a.h1, a.xn, a.mean, a.rstd, a.ids, a.drop_p, a.eps,
                drop ? seed32(eff_seed(a.salt1, a.seed_base)) : 0u, drop ? seed32(eff_seed(a.salt2, a.seed_base)) : 0u};
}

// O -> x1 = Q + O Wo^T + bo [saved], z = LN2(x1) [saved], h1 = relu(drop(z W1^T + b1)) [saved],
// x' = (drop(h1 W2^T + b2) + z) * (ids != 0)
template <int D, bool HEAD>
__global__ __launch_bounds__(NT) void block_out_kernel(OutArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef Smem<D, 3, 7, 1> L;
  constexpr int WB = Lay<D>::WBYTES;
  const float* lv = reinterpret_cast<const float*>(smem + L::W);   // bo, ln_w, ln_b, b1, b2 (+ head: gl, bl)
  float* red = reinterpret_cast<float*>(smem + L::V);
  constexpr bool head = HEAD;
  __shared__ float hred[4][NW];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4,
            cl = lane & 15;
  RCPROF(0);
  const TileRange tr = tiles_of_wave(n_tiles(a.M), wave);
  const OutFwd of = out_fwd_of(a);
  int64_t t = tr.first;
  Raw<D> orr, Qr;
  if (t < tr.end) {
    const int64_t mc = tile_of(t, a.M, cl).mc;
    load_raw<D>(orr, a.o, D, mc, g);
    load_raw<D>(Qr, a.Q, D, mc, g);
  }
  {
    const bf16* const W[3] = {a.Wo, a.W1, a.W2};
    const int64_t ldw[3] = {D, D, D};
    stage_w<D, 3>(smem, W, ldw, wave, lane);
    if (head) {
      const float* const V[7] = {a.bo, a.ln_w, a.ln_b, a.b1, a.b2, a.h.gl, a.h.bl};
      stage_v<D, 7>(reinterpret_cast<float*>(smem + L::W), V, tid);
    } else {
      const float* const V[5] = {a.bo, a.ln_w, a.ln_b, a.b1, a.b2};
      stage_v<D, 5>(reinterpret_cast<float*>(smem + L::W), V, tid);
    }
  }
  // head: the loss's divisor (the valid count: integer partials, any order is exact) and zeroed LN partial rows
  float hscale = 0.f;
  float hacc[3] = {0.f, 0.f, 0.f};
  if (head) {
    ln_zero(red, D, lane, wave);
    int c = 0;
    for (int i = tid; i < a.h.ncnt; i += NT) c += a.h.cnt_parts[i];
    c = (int)wave_sum((float)c);   // exact: counts < 2^24
    if (lane == 0) hred[3][wave] = (float)c;
  }
  __syncthreads();
  if (head) {
    float c = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) c += hred[3][w];
    hscale = 1.f / (a.h.divisor ? *a.h.divisor : c);
  }
  RCPROF(1);
  for (; t < tr.end; t += tr.step) {
    asm volatile("" ::: "memory");
    const Tile T = tile_of(t, a.M, cl);
    if (t != tr.first) {
      load_raw<D>(orr, a.o, D, T.mc, g);
      load_raw<D>(Qr, a.Q, D, T.mc, g);
    }
    Raw<D> zr, hr, xr, er, nr;
    int64_t ip = 0, in = 0;
    if (head && RC_HEAD_PREFETCH == 0) ip = head_rows<D>(a.h, T, er, nr, g);
    // 3: the tile's item ids at its start (before any store: vmcnt retires in order and counts stores, so an
    // index load issued after the chain's stores would wait for them), the item rows mid-chain
    if (head && RC_HEAD_PREFETCH == 3) {
      ip = a.h.pos[T.mc];
      in = a.h.neg[T.mc];
    }
    fwd_out_a<D>(orr, Qr, T, wslot(smem, 0, WB), wslot(smem, 1, WB), lv, of, zr, hr, lane);
    RCPROF(2);
    if (head && RC_HEAD_PREFETCH == 1) ip = head_rows<D>(a.h, T, er, nr, g);
    if (head && RC_HEAD_PREFETCH == 3) head_rows_at<D>(a.h, ip, in, er, nr, g);
    fwd_out_b<D>(hr, zr, T, wslot(smem, 2, WB), lv, of, xr, lane);
    RCPROF(4);
    if (head && RC_HEAD_PREFETCH == 2) ip = head_rows<D>(a.h, T, er, nr, g);
    if (head) head_tile<D>(xr, er, nr, ip, T, lv + 5 * D, lv + 6 * D, a.h, hscale, red, hacc, lane, wave);
    RCPROF(6);
  }
  RCPROF(5);
  if (head) {
    // BCE partials: lanes -> waves -> the workgroup's row (fixed order); LN affine partials likewise
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float v = wave_sum(hacc[k]);
      if (lane == 0) hred[k][wave] = v;
    }
    ln_partials<D>(red, a.h.lnpart, tid);   // begins with a barrier
    if (tid < 3) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) v += hred[tid][w];
      a.h.part[blockIdx.x * 3 + tid] = v;
    }
  }
}

struct OutBwdArgs {
  int64_t M;
  const bf16* dxn; const int64_t* ids;
  const bf16* h1; const bf16* x1; const float* mean2; const float* rstd2; const float* ln_w;
  const bf16* W2T; const bf16* W1T; const bf16* WoT;      // transposed [in][out] copies
  bf16* dy2; bf16* da1; bf16* dx1; bf16* dout; float* part;
  float drop_p; uint64_t salt1, salt2; const uint64_t* seed_base;
  const bf16* o; float* delta;                              // optional (both or neither)
};
__device__ __forceinline__ OutBwd out_bwd_of(const OutBwdArgs& a) {
  const bool drop = a.drop_p > 0.f;
  return OutBwd{a.dy2, a.da1, a.dx1, a.dout, a.delta, a.ids, a.drop_p,
                drop ? seed32(eff_seed(a.salt1, a.seed_base)) : 0u, drop ? seed32(eff_seed(a.salt2, a.seed_base)) : 0u};
}

// dzres = dxn*mask; dy2 = drop2(dzres) [saved]; da1 = relu'(h1)*drop1(dy2 W2) [saved]; dz = da1 W1 + dzres;
// dx1 = LN2'(x1, dz) [saved, + affine partials]; dout = dx1 Wo
template <int D>
__global__ __launch_bounds__(NT) void block_out_bwd_kernel(OutBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef Smem<D, 3, 1, 1> L;
  constexpr int WB = Lay<D>::WBYTES;
  const float* lv = reinterpret_cast<const float*>(smem + L::W);   // ln_w
  float* red = reinterpret_cast<float*>(smem + L::V);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4,
            cl = lane & 15;
  const TileRange tr = tiles_of_wave(n_tiles(a.M), wave);
  const OutBwd ob = out_bwd_of(a);
  int64_t t = tr.first;
  // every input of the first tile is requested before the weight staging (its ~3 us burst then hides their latency;
  // requested after the barrier they cost a second round trip)
  Raw<D> dr, hr, xr, orr;
  float mu = 0.f, rs = 0.f;
  auto load_tile = [&](int64_t mc) {
    load_raw<D>(dr, a.dxn, D, mc, g);
    load_raw<D>(hr, a.h1, D, mc, g);
    load_raw<D>(xr, a.x1, D, mc, g);
    if (a.delta) load_raw<D>(orr, a.o, D, mc, g);
    mu = a.mean2[mc];
    rs = a.rstd2[mc];
  };
  if (t < tr.end) load_tile(tile_of(t, a.M, cl).mc);
  {
    const bf16* const W[3] = {a.W2T, a.W1T, a.WoT};
    const int64_t ldw[3] = {D, D, D};
    stage_w<D, 3>(smem, W, ldw, wave, lane);
    const float* const V[1] = {a.ln_w};
    stage_v<D, 1>(reinterpret_cast<float*>(smem + L::W), V, tid);
  }
  ln_zero(red, D, lane, wave);
  __syncthreads();
  for (; t < tr.end; t += tr.step) {
    asm volatile("" ::: "memory");
    const Tile T = tile_of(t, a.M, cl);
    if (t != tr.first) load_tile(T.mc);
    Raw<D> dzr, dar;
    bwd_out_a<D>(dr, hr, T, wslot(smem, 0, WB), ob, dzr, dar, lane);
    bwd_out_b<D>(dar, xr, dzr, orr, T, mu, rs, wslot(smem, 1, WB), wslot(smem, 2, WB), lv, ob, red, lane, wave);
  }
  ln_partials<D>(red, a.part, tid);
}

struct InBwdArgs {
  int64_t M;
  const bf16* dq; const bf16* dkv; const bf16* dx1; const bf16* x;
  const float* mean1; const float* rstd1; const float* ln_w;
  const bf16* WinT; int64_t ldwt;                       // in_proj^T [d][3d]
  bf16* dx; float* part;
};

// dx_kv = dk Wk + dv Wv; dQ = dq Wq + dx1; dx = dx_kv + LN1'(x, dQ) (+ affine partials)
template <int D>
__global__ __launch_bounds__(NT) void block_in_bwd_kernel(InBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef Smem<D, 3, 1, 1> L;
  constexpr int WB = Lay<D>::WBYTES;
  const float* lv = reinterpret_cast<const float*>(smem + L::W);   // ln_w
  float* red = reinterpret_cast<float*>(smem + L::V);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4,
            cl = lane & 15;
  const TileRange tr = tiles_of_wave(n_tiles(a.M), wave);
  int64_t t = tr.first;
  // every input of the first tile is requested before the weight staging (as block_out_bwd)
  Raw<D> kr, vr, qr, rr, xr;
  float mu = 0.f, rs = 0.f;
  auto load_tile = [&](int64_t mc) {
    load_raw<D>(kr, a.dkv, 2 * D, mc, g);
    load_raw<D>(vr, a.dkv + D, 2 * D, mc, g);
    load_raw<D>(qr, a.dq, D, mc, g);
    load_raw<D>(rr, a.dx1, D, mc, g);
    load_raw<D>(xr, a.x, D, mc, g);
    mu = a.mean1[mc];
    rs = a.rstd1[mc];
  };
  if (t < tr.end) load_tile(tile_of(t, a.M, cl).mc);
  {
    const bf16* const W[3] = {a.WinT + D, a.WinT + 2 * D, a.WinT};   // Wk^T, Wv^T, Wq^T rows
    const int64_t ldw[3] = {a.ldwt, a.ldwt, a.ldwt};
    stage_w<D, 3>(smem, W, ldw, wave, lane);
    const float* const V[1] = {a.ln_w};
    stage_v<D, 1>(reinterpret_cast<float*>(smem + L::W), V, tid);
  }
  ln_zero(red, D, lane, wave);
  __syncthreads();
  for (; t < tr.end; t += tr.step) {
    asm volatile("" ::: "memory");
    const Tile T = tile_of(t, a.M, cl);
    if (t != tr.first) load_tile(T.mc);
    Raw<D> dxkv, dxr;
    bwd_in_a<D>(kr, vr, wslot(smem, 0, WB), wslot(smem, 1, WB), dxkv, lane);
    bwd_in_b<D>(qr, rr, xr, dxkv, T, mu, rs, wslot(smem, 2, WB), lv, red, dxr, lane, wave);
    store_raw<D>(a.dx, D, T.m, T.ok, dxr, g);
  }
  ln_partials<D>(red, a.part, tid);
}

// ------------------------------------------------------------------ launch geometry
static int g_ncu = 0;
static int64_t grid_for(int64_t M) {
  if (g_ncu == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) ==
                                                 hipSuccess && n > 0)
      g_ncu = n;
    else
      g_ncu = 256;
  }
  const int64_t nt = (M + TR - 1) / TR;
  return nt < g_ncu ? nt : g_ncu;
}
template <int D> static size_t lds_fwd() { return Smem<D, 3, 5, 0>::BYTES; }
template <int D, bool HEAD> static size_t lds_out() {
  return HEAD ? Smem<D, 3, 7, 1>::BYTES : Smem<D, 3, 5, 0>::BYTES;
}
template <int D> static size_t lds_bwd() { return Smem<D, 3, 1, 1>::BYTES; }

template <typename K>
static void set_lds(K kern, size_t bytes) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
template <int D, bool HEAD>
static void launch_out_t(const OutArgs& a, hipStream_t s) {
  constexpr auto k = block_out_kernel<D, HEAD>;
  const size_t lds = lds_out<D, HEAD>();
  set_lds(k, lds);
  hipLaunchKernelGGL(k, dim3((unsigned)grid_for(a.M)), dim3(NT), lds, s, a);
}
static int launch_out(const OutArgs& a, int64_t d, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const bool head = a.h.E != nullptr;
  if (d == 64) head ? launch_out_t<64, true>(a, s) : launch_out_t<64, false>(a, s);
  else if (d == 128) head ? launch_out_t<128, true>(a, s) : launch_out_t<128, false>(a, s);
  else return RS_ERR_UNSUPPORTED;
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------ batched bf16 transpose
// dst[m][c][r] = src[m][r][c] for the SAS block weight matrices (desc: rows, cols, src_off, lds, dst_off, ldd in
// elements; 64x64 tiles through LDS): the [in][out] copies the backward kernels stage as their A operands
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const int64_t* __restrict__ desc, const __bf16* src,
                                                             __bf16* dst) {
  __shared__ __bf16 t[64][66];
  const int64_t* dsc = desc + 6 * blockIdx.y;
  const int64_t rows = dsc[0], cols = dsc[1];
  const int64_t tc = cdiv(cols, 64);
  const int64_t tr = blockIdx.x / tc, tcc = blockIdx.x % tc;
  if (tr * 64 >= rows) return;
  const __bf16* sp = src + dsc[2];
  __bf16* dp = dst + dsc[4];
  const int64_t lds = dsc[3], ldd = dsc[5];
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int r = e / 64, c = e % 64;
    const int64_t gr = tr * 64 + r, gc = tcc * 64 + c;
    t[r][c] = (gr < rows && gc < cols) ? sp[gr * lds + gc] : (__bf16)0.f;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int c = e / 64, r = e % 64;
    const int64_t gr = tr * 64 + r, gc = tcc * 64 + c;
    if (gr < rows && gc < cols) dp[gc * ldd + gr] = t[r][c];
  }
}

}  // namespace rc

extern "C" {

int64_t rs_sas_block_parts(int64_t M) {
  if (M <= 0) return 0;
  return rc::grid_for(M);
}

int rs_sas_block_in(int64_t M, int64_t d, const void* x, int64_t ldx, const float* ln_w, const float* ln_b, float eps,
                    void* Q, float* mean, float* rstd, const void* Wq, const float* bq, void* q, const void* Wkv,
                    const float* bkv, void* kv, void* stream) {
  if (M <= 0 || ldx % 8) return RS_ERR_ARG;
  rc::InArgs a = {M, (const __bf16*)x, ldx, ln_w, ln_b, eps, (__bf16*)Q, mean, rstd, (const __bf16*)Wq, bq,
                  (__bf16*)q, (const __bf16*)Wkv, bkv, (__bf16*)kv};
  const dim3 grid((unsigned)rc::grid_for(M));
  hipStream_t s = (hipStream_t)stream;
  if (d == 64) {
    rc::set_lds(rc::block_in_kernel<64>, rc::lds_fwd<64>());
    hipLaunchKernelGGL(rc::block_in_kernel<64>, grid, dim3(rc::NT), rc::lds_fwd<64>(), s, a);
  } else if (d == 128) {
    rc::set_lds(rc::block_in_kernel<128>, rc::lds_fwd<128>());
    hipLaunchKernelGGL(rc::block_in_kernel<128>, grid, dim3(rc::NT), rc::lds_fwd<128>(), s, a);
  } else {
    return RS_ERR_UNSUPPORTED;
  }
  return (int)hipGetLastError();
}

int64_t rs_sas_block_in_count_parts(int64_t M) { return M > 0 ? rc::grid_for(M) : 0; }

int rs_sas_block_in_embed(int64_t M, int64_t d, const int64_t* ids, int64_t T, const void* item_emb, const void* pos_emb,
                          float scale, float drop_p, uint64_t salt, const uint64_t* seed_base, void* x0,
                          const int64_t* count_ids, int* count_parts, const float* ln_w, const float* ln_b, float eps,
                          void* Q, float* mean, float* rstd, const void* Wq, const float* bq, void* q, const void* Wkv,
                          const float* bkv, void* kv, void* stream) {
  if (M <= 0 || T <= 0 || M % T || !ids || !item_emb || !pos_emb || !x0 || !count_ids != !count_parts)
    return RS_ERR_ARG;
  if (((uintptr_t)item_emb | (uintptr_t)pos_emb | (uintptr_t)x0) % 16 || (d != 64 && d != 128)) return RS_ERR_ARG;
  rc::InArgs a = {M, (const __bf16*)x0, d, ln_w, ln_b, eps, (__bf16*)Q, mean, rstd, (const __bf16*)Wq, bq,
                  (__bf16*)q, (const __bf16*)Wkv, bkv, (__bf16*)kv,
                  rc::EmbIn{ids, (const __bf16*)item_emb, (const __bf16*)pos_emb, T, scale, drop_p, salt, seed_base,
                            (__bf16*)x0, count_ids, count_parts}};
  const dim3 grid((unsigned)rc::grid_for(M));
  hipStream_t s = (hipStream_t)stream;
  if (d == 64) {
    rc::set_lds(rc::block_in_kernel<64>, rc::lds_fwd<64>());
    hipLaunchKernelGGL(rc::block_in_kernel<64>, grid, dim3(rc::NT), rc::lds_fwd<64>(), s, a);
  } else {
    rc::set_lds(rc::block_in_kernel<128>, rc::lds_fwd<128>());
    hipLaunchKernelGGL(rc::block_in_kernel<128>, grid, dim3(rc::NT), rc::lds_fwd<128>(), s, a);
  }
  return (int)hipGetLastError();
}

int rs_sas_block_out(int64_t M, int64_t d, const void* o, const void* Q, const void* Wo, const float* bo, void* x1,
                     const float* ln_w, const float* ln_b, float eps, void* z, float* mean, float* rstd,
                     const void* W1, const float* b1, void* h1, const void* W2, const float* b2, void* xn,
                     const int64_t* ids, float drop_p, uint64_t salt1, uint64_t salt2, const uint64_t* seed_base,
                     void* stream) {
  if (M <= 0) return RS_ERR_ARG;
  rc::OutArgs a = {M, (const __bf16*)o, (const __bf16*)Q, (const __bf16*)Wo, bo, (__bf16*)x1, ln_w, ln_b, eps,
                   (__bf16*)z, mean, rstd, (const __bf16*)W1, b1, (__bf16*)h1, (const __bf16*)W2, b2, (__bf16*)xn,
                   ids, drop_p, salt1, salt2, seed_base};
  return rc::launch_out(a, d, stream);
}

int64_t rs_sas_block_grid(int64_t M) { return M > 0 ? rc::grid_for(M) : 0; }

int rs_sas_block_out_head(int64_t M, int64_t d, const void* o, const void* Q, const void* Wo, const float* bo,
                          void* x1, const float* ln_w, const float* ln_b, float eps, void* z, float* mean, float* rstd,
                          const void* W1, const float* b1, void* h1, const void* W2, const float* b2, void* xn,
                          const int64_t* ids, float drop_p, uint64_t salt1, uint64_t salt2,
                          const uint64_t* seed_base, const void* E, const int64_t* pos, const int64_t* neg,
                          const float* lnl_w, const float* lnl_b, const int* count_parts, int64_t ncount,
                          const float* divisor, void* f, float* pl, float* nl, float* dpl, float* dnl, void* dx,
                          float* lnpart, float* part, void* stream) {
  if (M <= 0 || !E || !pos || !neg || !count_parts || ncount <= 0 || !f || !dx || !lnpart || !part) return RS_ERR_ARG;
  if (d != 64 && d != 128) return RS_ERR_UNSUPPORTED;
  rc::OutArgs a = {M, (const __bf16*)o, (const __bf16*)Q, (const __bf16*)Wo, bo, (__bf16*)x1, ln_w, ln_b, eps,
                   (__bf16*)z, mean, rstd, (const __bf16*)W1, b1, (__bf16*)h1, (const __bf16*)W2, b2, (__bf16*)xn,
                   ids, drop_p, salt1, salt2, seed_base,
                   rc::HeadArgs{(const __bf16*)E, pos, neg, lnl_w, lnl_b, eps, count_parts, (int)ncount, divisor,
                                (__bf16*)f, pl, nl, dpl, dnl, (__bf16*)dx, lnpart, part}};
  return rc::launch_out(a, d, stream);
}

int rs_sas_block_out_bwd(int64_t M, int64_t d, const void* dxn, const int64_t* ids, const void* h1, const void* x1,
                         const float* mean2, const float* rstd2, const float* ln_w, const void* W2T, const void* W1T,
                         const void* WoT, void* dy2, void* da1, void* dx1, void* dout, float* part, float drop_p,
                         uint64_t salt1, uint64_t salt2, const uint64_t* seed_base, void* stream) {
  return rs_sas_block_out_bwd_delta(M, d, dxn, ids, h1, x1, mean2, rstd2, ln_w, W2T, W1T, WoT, dy2, da1, dx1, dout,
                                    part, drop_p, salt1, salt2, seed_base, nullptr, nullptr, stream);
}

int rs_sas_block_out_bwd_delta(int64_t M, int64_t d, const void* dxn, const int64_t* ids, const void* h1,
                               const void* x1, const float* mean2, const float* rstd2, const float* ln_w,
                               const void* W2T, const void* W1T, const void* WoT, void* dy2, void* da1, void* dx1,
                               void* dout, float* part, float drop_p, uint64_t salt1, uint64_t salt2,
                               const uint64_t* seed_base, const void* o, float* delta, void* stream) {
  if (!o != !delta) return RS_ERR_ARG;
  if (M <= 0) return RS_ERR_ARG;
  rc::OutBwdArgs a = {M, (const __bf16*)dxn, ids, (const __bf16*)h1, (const __bf16*)x1, mean2, rstd2, ln_w,
                      (const __bf16*)W2T, (const __bf16*)W1T, (const __bf16*)WoT, (__bf16*)dy2, (__bf16*)da1,
                      (__bf16*)dx1, (__bf16*)dout, part, drop_p, salt1, salt2, seed_base, (const __bf16*)o, delta};
  const dim3 grid((unsigned)rc::grid_for(M));
  hipStream_t s = (hipStream_t)stream;
  if (d == 64) {
    rc::set_lds(rc::block_out_bwd_kernel<64>, rc::lds_bwd<64>());
    hipLaunchKernelGGL(rc::block_out_bwd_kernel<64>, grid, dim3(rc::NT), rc::lds_bwd<64>(), s, a);
  } else if (d == 128) {
    rc::set_lds(rc::block_out_bwd_kernel<128>, rc::lds_bwd<128>());
    hipLaunchKernelGGL(rc::block_out_bwd_kernel<128>, grid, dim3(rc::NT), rc::lds_bwd<128>(), s, a);
  } else {
    return RS_ERR_UNSUPPORTED;
  }
  return (int)hipGetLastError();
}

int rs_sas_block_in_bwd(int64_t M, int64_t d, const void* dq, const void* dkv, const void* dx1, const void* x,
                        const float* mean1, const float* rstd1, const float* ln_w, const void* WinT, void* dx,
                        float* part, void* stream) {
  if (M <= 0) return RS_ERR_ARG;
  rc::InBwdArgs a = {M, (const __bf16*)dq, (const __bf16*)dkv, (const __bf16*)dx1, (const __bf16*)x, mean1, rstd1,
                     ln_w, (const __bf16*)WinT, 3 * d, (__bf16*)dx, part};
  const dim3 grid((unsigned)rc::grid_for(M));
  hipStream_t s = (hipStream_t)stream;
  if (d == 64) {
    rc::set_lds(rc::block_in_bwd_kernel<64>, rc::lds_bwd<64>());
    hipLaunchKernelGGL(rc::block_in_bwd_kernel<64>, grid, dim3(rc::NT), rc::lds_bwd<64>(), s, a);
  } else if (d == 128) {
    rc::set_lds(rc::block_in_bwd_kernel<128>, rc::lds_bwd<128>());
    hipLaunchKernelGGL(rc::block_in_bwd_kernel<128>, grid, dim3(rc::NT), rc::lds_bwd<128>(), s, a);
  } else {
    return RS_ERR_UNSUPPORTED;
  }
  return (int)hipGetLastError();
}

int rs_transpose_bf16(int64_t nmat, const int64_t* desc, int64_t max_tiles, const void* src, void* dst,
                      void* stream) {
  if (nmat <= 0 || max_tiles <= 0) return RS_ERR_ARG;
  hipLaunchKernelGGL(rc::transpose_bf16_kernel, dim3((unsigned)max_tiles, (unsigned)nmat), dim3(256), 0,
                     (hipStream_t)stream, desc, (const __bf16*)src, (__bf16*)dst);
  return (int)hipGetLastError();
}

}  // extern "C"
