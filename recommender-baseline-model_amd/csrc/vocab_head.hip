// BERT4Rec vocabulary head on the labelled rows, vocabulary-tile-stationary (bf16, gfx950).
//
// Reference: BERTModel.out = Linear(d, V+1) on every position (BS/models/bert.py:10,16) and
// CrossEntropyLoss(ignore_index=0) (BS/trainers/bert.py:11,36-40).  The fused step keeps the R
// labelled rows h [R][d] (R ~ 1.8k at the ML-20M / 1M-item shapes) and needs, per step,
//   fwd: per row the log-sum-exp of the logits h E^T + b and the label's logit;
//   bwd: dlogits = (softmax - onehot) * dloss / count (operand of the input gradient dh = dlogits E),
//        dE = dlogits^T h and db = colsum(dlogits).
// With V+1 = 1M these are R x 1M x d products: the generic GEMM ran them as 128x128 output tiles with
// only d / 64 = 4 k-stages each, so every workgroup paid a cold prologue and a full epilogue for 4
// stages of MFMAs (~15 % of the MFMA peak), and dE was a third pass re-reading 3.6 GB of dlogits.
//
// Here one workgroup owns a 128-column vocabulary tile at a time (persistent over tiles) and walks
// ALL row tiles of h against it:
//   * the h row tile [128][d] sits whole in LDS (prefetched into registers during the previous row
//     tile); E's tile streams through double-buffered 64-deep LDS stages from L2 (HBM reads it once);
//   * S^T = E_tile . h_tile^T is accumulated transposed (vocabulary on the accumulator's row axis), so
//     a lane holds 4 consecutive vocabulary entries of one row: per-row softmax statistics reduce in
//     registers + 2 shuffles, and dlogits leave as 8-byte LDS writes;
//   * bwd: dlogits go to LDS [rows][vocab] and, 16-B coalesced, to the global dlogits operand of
//     dh = dlogits.E (split-K rs_gemm) and dE = dlogits^T.h, db = colsum (rs_linear_wgrad).  Forming dE here
//     instead (a second pass over each row tile's h stages, dE^T accumulated in registers per vocabulary
//     tile, db from the dlogits in LDS) was built and measured: the 128 x d fp32 dE tile is 64 more
//     registers per lane on a kernel already near 256 with 8 waves, and it spilled 125 (d = 256) / 64
//     (d = 128) -- not kept.
// The fwd partials have exactly the layout of vocab_ce.hip's EC_CE_PART epilogue, so ce_tiles_kernel /
// ce_sum_kernel finish the loss unchanged (the label logit is formed there as <h, E[label]> + b).
//
// Measured at R = 1750, V+1 = 1M, d = 256 (tools/vhead_bench.py): fwd 1.94 ms = 463 TFLOP/s (the GEMM-epilogue
// form: 2.5 ms).  Where the rest goes (switching parts off): the bare MFMA loop alone runs at 917 TFLOP/s
// (16 MFMAs per wave between barriers, both waves of a SIMD in the same phase), the softmax epilogue costs
// ~0.5 ms (its VALU work per logit equals the MFMA work of a d = 256 product and does not overlap it), the h
// stream ~0.3 ms, the E tiles ~0.1 ms.  The XOR-swizzled images removed all LDS bank conflicts (44 % of the
// LDS cycles with padded rows).
#include "common.h"
#include "../../include/recsys_hip.h"
#include <type_traits>

typedef __attribute__((ext_vector_type(4))) __bf16 bf4;

namespace vh {
typedef __bf16 bf16;

constexpr int BR = 128;   // rows per row tile
constexpr int NTH = 512;  // 8 waves, 2 per SIMD: wave (wm, wn) = vocabulary quarter wm x row half wn
typedef __attribute__((ext_vector_type(4))) unsigned u4;

struct Args {
  int64_t R, V1, ntn;       // ntn: 128-column partial tiles (vocab_ce.hip's ws layout)
  const bf16* h; int64_t ldh;
  const bf16* E; int64_t lde;
  const float* bias;
  const int64_t* labels;
  const int* rows_dev;
  float* part;        // fwd: [R][ntn][2] (max, sum exp) per 128-column tile
  float* tgt;         // fwd: [R] label logits
  const float* lse;   // bwd
  const float* count;
  const float* dloss;
  bf16* dl; int64_t lddl;   // bwd: dlogits [R][V1] (rows >= live count untouched)
  int64_t voff;             // vocabulary index of E's row 0 (a shard of the table; 0 = the whole table)
  KStamp ks;
};

// BV vocabulary entries per workgroup tile (E tile stationary in LDS), h streamed in BK-deep stages
template <int DK, int BV, bool BWD> struct L {
  static constexpr int BK = BWD ? 64 : 32;
  static constexpr int LDE = DK;                   // unpadded rows, 16-B chunks XOR-swizzled (swz)
  static constexpr int LDH = BK;
  static constexpr int LDD = BV + 8;
  static constexpr int E_ELEMS = BV * LDE;
  static constexpr int H_ELEMS = BR * LDH;
  static constexpr int D_ELEMS = BWD ? BR * LDD : 0;
  static constexpr int NKS = DK / BK;
  static constexpr int HPT = BR * BK / 8 / NTH;    // 16-B chunks of an h stage per thread
  static constexpr int EPT = BV * DK / 8 / NTH;    // ... of an E tile
  static constexpr int FV = BV / 64;               // 16-wide vocabulary fragments per wave
  static constexpr int PF = 3;                     // h stages in flight (register ring)
  static constexpr int LDS = (E_ELEMS + 2 * H_ELEMS + D_ELEMS) * 2 + BR * 12 + 4 * BR * 2 * 4;
};

// XOR swizzle of the 16-B chunk index within a row of CPR chunks: the 16 lanes of every ds_read_b128 lane
// group (rows li = lane & 15 of a fragment, chunks c0 + (lane >> 4)) then hit 16 distinct 4-bank sets
template <int CPR>
__device__ __forceinline__ int swz(int row) {
  if constexpr (CPR >= 16) return row & 15;
  else if constexpr (CPR == 8) return ((row >> 1) & 3) << 1;
  else return ((row >> 3) & 1) << 1;
}

// MFMA operand fragment: rows row0 + (lane & 15), 16-B chunk c0 + (lane >> 4) of a swizzled image
template <int CPR>
__device__ __forceinline__ bf16x8 row_frag(const bf16* img, int row0, int c0, int lane) {
  const int row = row0 + (lane & 15), c = (c0 + (lane >> 4)) ^ swz<CPR>(row);
  return *reinterpret_cast<const bf16x8*>(img + row * (CPR * 8) + c * 8);
}

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void comb(float& mx, float& sm, float m2, float s2) {
  const float mm = fmaxf(mx, m2);
  sm = (mm == -__builtin_inff()) ? 0.f : sm * __expf(mx - mm) + s2 * __expf(m2 - mm);
  mx = mm;
}

template <int DK, int BV, bool BWD>
__global__ __launch_bounds__(NTH, 1) void vhead_kernel(Args a) {
  KStampBegin stamp_b_(a.ks);
  KStampEnd stamp_e_(a.ks);
  using C = L<DK, BV, BWD>;
  constexpr int BK = C::BK, FV = C::FV;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* Et = reinterpret_cast<bf16*>(smem);           // E tile [BV][LDE]
  bf16* Hs = Et + C::E_ELEMS;                         // 2 h stages [BR][LDH]
  bf16* Ds = Hs + 2 * C::H_ELEMS;                     // bwd: dlogits [BR][LDD]
  int64_t* labs = reinterpret_cast<int64_t*>(Ds + C::D_ELEMS);
  float* lses = reinterpret_cast<float*>(labs + BR);
  float* red = lses + BR;                             // fwd: [4 quarters][BR][2]

  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, cl = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), wm = wave >> 1, wn = wave & 1;
  const int v0w = wm * (BV / 4);
  const int64_t Rl = a.rows_dev ? min(a.R, (int64_t)*a.rows_dev) : a.R;
  const int nmt = (int)((Rl + BR - 1) / BR);
  // row tiles of this workgroup: all of them, or (small vocabularies: fewer vocabulary tiles than CUs) the
  // gridDim.y-th share blockIdx.y -- every (row, vocabulary tile) still formed by exactly one workgroup
  const int mtb = (int)((int64_t)nmt * blockIdx.y / gridDim.y), mte = (int)((int64_t)nmt * (blockIdx.y + 1) / gridDim.y);
  if (mte <= mtb) return;
  const int NIT = (mte - mtb) * C::NKS;

  float sc = 0.f;
  if constexpr (BWD) sc = (a.dloss ? *a.dloss : 1.f) / *a.count;

  // h stage `it` (row tile it / NKS, k stage it % NKS) -> register slot (a ring of PF stages in flight, so
  // each stage's L2 round trip hides under PF - 1 stages of MFMAs); rows >= Rl read as zero
  constexpr int PF = C::PF;
  bf16x8 hr[PF][C::HPT];
  auto h_load = [&](auto slot, int it) {
    constexpr int sl = decltype(slot)::value;
    const int mo = it / C::NKS, ks = it - mo * C::NKS, mt = mtb + mo;
#pragma unroll
    for (int c = 0; c < C::HPT; ++c) {
      const int ch = tid + NTH * c, r = ch / (BK / 8), k8 = (ch % (BK / 8)) * 8;
      const int64_t row = (int64_t)mt * BR + r;
      const int64_t rc = row < Rl ? row : Rl - 1;
      u4 v = *reinterpret_cast<const u4*>(a.h + rc * a.ldh + ks * BK + k8);
      v &= (row < Rl ? 0xffffffffu : 0u);
      hr[sl][c] = __builtin_bit_cast(bf16x8, v);
    }
  };
  auto h_store = [&](auto slot, int buf) {
    constexpr int sl = decltype(slot)::value;
#pragma unroll
    for (int c = 0; c < C::HPT; ++c) {
      const int ch = tid + NTH * c, r = ch / (BK / 8), k8 = (ch % (BK / 8)) * 8;
      *reinterpret_cast<bf16x8*>(Hs + buf * C::H_ELEMS + r * C::LDH + (((k8 >> 3) ^ swz<BK / 8>(r)) << 3)) =
          hr[sl][c];
    }
  };
  // row metadata of row tile mt -> LDS (labels; lse for the backward)
  auto meta_store = [&](int mt) {
    if (tid < BR) {
      const int64_t row = (int64_t)mt * BR + tid;
      labs[tid] = row < Rl ? a.labels[row] : 0;
      if constexpr (BWD) lses[tid] = row < Rl ? a.lse[row] : 0.f;
    }
  };

  for (int64_t vt = blockIdx.x; vt * BV < a.V1; vt += gridDim.x) {
    const int64_t n0 = vt * BV;
    float bia[FV][4];
#pragma unroll
    for (int i = 0; i < FV; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t v = n0 + v0w + 16 * i + 4 * g + r;
        bia[i][r] = (a.bias && v < a.V1) ? a.bias[v] : 0.f;
      }
    // prologue: E tile (stationary for all row tiles), h stage (0, 0), row tile 0's metadata
    __syncthreads();                    // the previous vocabulary tile's readers are done
    constexpr int EB = C::EPT < 8 ? C::EPT : 8;     // chunks in flight per batch
#pragma unroll
    for (int c0 = 0; c0 < C::EPT; c0 += EB) {
      u4 ex[EB];
#pragma unroll
      for (int c = 0; c < EB; ++c) {
        const int ch = tid + NTH * (c0 + c), r = ch / (DK / 8), k8 = (ch % (DK / 8)) * 8;
        const int64_t v = n0 + r;
        const int64_t vc = v < a.V1 ? v : a.V1 - 1;
        ex[c] = *reinterpret_cast<const u4*>(a.E + vc * a.lde + k8);
        ex[c] &= (v < a.V1 ? 0xffffffffu : 0u);
      }
#pragma unroll
      for (int c = 0; c < EB; ++c) {
        const int ch = tid + NTH * (c0 + c), r = ch / (DK / 8), k8 = (ch % (DK / 8)) * 8;
        *reinterpret_cast<u4*>(Et + r * C::LDE + (((k8 >> 3) ^ swz<DK / 8>(r)) << 3)) = ex[c];
      }
    }
    h_load(std::integral_constant<int, 0>{}, 0);
    if (1 < NIT) h_load(std::integral_constant<int, 1 % PF>{}, 1);
    if (2 < NIT) h_load(std::integral_constant<int, 2 % PF>{}, 2);
    static_assert(PF == 3, "prologue loads PF - 1 stages ahead");
    h_store(std::integral_constant<int, 0>{}, 0);
    meta_store(mtb);
    __syncthreads();

    f32x4 acc[FV][4];
    // iteration `it` (register slot u = it % PF, a compile-time constant in the unrolled ring): MFMAs on LDS
    // stage it & 1; stage it + 1 (slot (u + 1) % PF) -> the other LDS buffer; stage it + PF -> slot u
    auto body = [&](int it, auto U) {
      constexpr int u = decltype(U)::value;
      const int mo = it / C::NKS, ks = it - mo * C::NKS, mt = mtb + mo;
      if (ks == 0) {
#pragma unroll
        for (int i = 0; i < FV; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      }
      const bool more = it + 1 < NIT;
      const bf16* H = Hs + (it & 1) * C::H_ELEMS;
#pragma unroll
      for (int s = 0; s < BK / 32; ++s) {
        bf16x8 fa[FV], fb[4];
#pragma unroll
        for (int i = 0; i < FV; ++i) fa[i] = row_frag<DK / 8>(Et, v0w + 16 * i, (ks * BK + 32 * s) / 8, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = row_frag<BK / 8>(H, wn * 64 + 16 * j, 4 * s, lane);
#pragma unroll
        for (int i = 0; i < FV; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma(fa[i], fb[j], acc[i][j]);
      }
      if (more) h_store(std::integral_constant<int, (u + 1) % PF>{}, (it + 1) & 1);
      if (it + PF < NIT) h_load(std::integral_constant<int, u>{}, it + PF);
      if (ks != C::NKS - 1) {
        __syncthreads();
        return;
      }

      // ---- row tile mt complete: acc[i][j][r] = S^T[vocab v0w+16i+4g+r][row wn*64+16j+cl] (no bias yet)
      const int64_t m0 = (int64_t)mt * BR;
      // vocabulary entries of this lane's accumulator rows are base + 16 i + r, base = n0 + v0w + 4g; only the
      // last tile is ragged (lim < 16 FV): masking there only, as selects
      const int lim = (int)min((int64_t)BV, a.V1 - n0) - v0w - 4 * g;
      const bool ragged = n0 + BV > a.V1;
      if constexpr (!BWD) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int rl = wn * 64 + 16 * j + cl;
          float mx = -__builtin_inff();
#pragma unroll
          for (int i = 0; i < FV; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float x = acc[i][j][r] + bia[i][r];
              if (ragged) x = 16 * i + r < lim ? x : -__builtin_inff();
              acc[i][j][r] = x;
              mx = fmaxf(mx, x);
            }
          float sm = 0.f;
          const float mxl = mx * 1.4426950408889634f;
#pragma unroll
          for (int i = 0; i < FV; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r)     // e^(x - mx) = 2^(x log2e - mx log2e); masked: 2^-inf = 0
              sm += __builtin_amdgcn_exp2f(__builtin_fmaf(acc[i][j][r], 1.4426950408889634f, -mxl));
          if (mx == -__builtin_inff()) sm = 0.f;
#pragma unroll
          for (int o = 16; o < 64; o <<= 1) comb(mx, sm, __shfl_xor(mx, o, 64), __shfl_xor(sm, o, 64));
          if (g == 0) {
            red[(wm * BR + rl) * 2 + 0] = mx;
            red[(wm * BR + rl) * 2 + 1] = sm;
          }
        }
        __syncthreads();
        // per 128-column partial tile: quarters {0,1} (BV = 256) or all four (BV = 128)
        constexpr int QPT = 512 / BV;          // quarters per 128-column partial tile
        if (tid < BR * (4 / QPT) && m0 + (tid % BR) < Rl) {
          const int rl = tid % BR, half = tid / BR;
          float mx = red[((half * QPT) * BR + rl) * 2], sm = red[((half * QPT) * BR + rl) * 2 + 1];
#pragma unroll
          for (int q = 1; q < QPT; ++q)
            comb(mx, sm, red[((half * QPT + q) * BR + rl) * 2], red[((half * QPT + q) * BR + rl) * 2 + 1]);
          const int64_t pt = (n0 >> 7) + half;
          if (pt < a.ntn) {
            a.part[((m0 + rl) * a.ntn + pt) * 2 + 0] = mx;
            a.part[((m0 + rl) * a.ntn + pt) * 2 + 1] = sm;
          }
        }
      } else {
        // dlogits of this tile -> Ds [row][vocab] (bf16, 8-byte writes of 4 vocabulary entries) -> global
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int rl = wn * 64 + 16 * j + cl;
          const int64_t lb = labs[rl];
          const bool live = m0 + rl < Rl && lb != 0;
          const float Lr = lses[rl];
          const float scr = live ? sc : 0.f;
          const int64_t offl = lb - a.voff - (n0 + v0w + 4 * g);   // label's entry in this lane's rows
          const int off = offl < 0 || offl >= 64 ? -1 : (int)offl;
#pragma unroll
          for (int i = 0; i < FV; ++i) {
            bf4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float x = acc[i][j][r] + bia[i][r];
              float gv = (__expf(x - Lr) - (off == 16 * i + r ? 1.f : 0.f)) * scr;
              if (ragged) gv = 16 * i + r < lim ? gv : 0.f;
              o[r] = (bf16)gv;
            }
            *reinterpret_cast<bf4*>(Ds + rl * C::LDD + v0w + 16 * i + 4 * g) = o;
          }
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < BR * BV / 8 / NTH; ++c) {
          const int ch = tid + NTH * c, r = ch / (BV / 8), c8 = (ch % (BV / 8)) * 8;
          const int64_t row = m0 + r, v = n0 + c8;
          if (row < Rl) {
            const bf16x8 x = *reinterpret_cast<const bf16x8*>(Ds + r * C::LDD + c8);
            bf16* dst = a.dl + row * a.lddl + v;
            if (v + 8 <= a.V1) {
              *reinterpret_cast<bf16x8*>(dst) = x;
            } else {
              for (int e = 0; e < 8; ++e)
                if (v + e < a.V1) dst[e] = x[e];
            }
          }
        }
      }
      __syncthreads();                         // labs / red / Ds readers of this row tile are done
      if (mt + 1 < mte) meta_store(mt + 1);    // (visible after the next stage's barrier)
      if constexpr (C::NKS == 1) __syncthreads();
    };
    for (int it0 = 0; it0 < NIT; it0 += PF) {
      body(it0, std::integral_constant<int, 0>{});
      if (it0 + 1 < NIT) body(it0 + 1, std::integral_constant<int, 1>{});
      if (it0 + 2 < NIT) body(it0 + 2, std::integral_constant<int, 2>{});
    }
  }
}

template <int DK, int BV, bool BWD>
hipError_t launch(Args& a, hipStream_t s) {
  using C = L<DK, BV, BWD>;
  static_assert(C::LDS <= 163840, "LDS budget");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)vhead_kernel<DK, BV, BWD>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              C::LDS);
    attr = true;
  }
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t nvt = cdiv(a.V1, BV);
  const int64_t grid = std::min<int64_t>(nvt, (int64_t)cus);
  // fewer vocabulary tiles than CUs (cfg3: 105 / 209 of 256): split the row tiles over gridDim.y groups so that
  // up to one workgroup per CU runs (the 1M-vocabulary shapes keep one group, persistent over vocabulary tiles)
  const int64_t gy = std::max<int64_t>(1, std::min<int64_t>(cdiv(a.R, BR), (int64_t)cus / nvt));
  hipLaunchKernelGGL((vhead_kernel<DK, BV, BWD>), dim3((unsigned)grid, (unsigned)gy), dim3(NTH), C::LDS, s, a);
  return hipGetLastError();
}

// ---- ping-pong forms (forward and backward) -----------------------------------------------------------------
// The forms above run their eight waves in lock step (a barrier per h stage), so the two waves of a SIMD are in
// their softmax epilogue (VALU + transcendental) at the same time and the matrix core idles through it.  Here:
//   * each wave keeps its 64 vocabulary entries x d of E in REGISTERS for the whole vocabulary tile (the A
//     operand; 128 VGPRs at d = 256), so LDS carries only h, and a whole 32-row tile of h (16 KB at d = 256)
//     arrives by LDS-DMA in one piece: one barrier per row tile ("item") instead of one per k stage;
//   * waves 0-3 (group 0) and 4-7 (group 1) -- one of each per SIMD, same vocabulary quarter -- take alternate
//     items and run half an interval apart: in interval n group 0 runs the MFMAs of item 2n and then its
//     epilogue, group 1 the epilogue of item 2n - 1 and then the MFMAs of item 2n + 1, so on every SIMD one
//     wave's MFMAs overlap the other's epilogue;
//   * h tiles are prefetched two intervals ahead (six buffers).  DMA completion is only visible through vmcnt,
//     which retires in order and counts stores too, so every interval issues its global traffic in a fixed order
//     -- the previous interval's stores, then (at a vocabulary-tile change, waited at once) the E reload, then
//     the DMAs two intervals ahead -- and no vector-memory load follows the DMAs: the wait at the next interval
//     is then exactly "all but this wave's DMAs of the last interval" (stores and the previous DMAs had a whole
//     interval to land).  Per-row backward metadata (label entry, lse) sits in LDS for the launch;
//   * fwd: each quarter's per-row (max, sum) pairs combine with the neighbouring quarter's into the 128-column
//     `part` layout above one interval later; bwd: dlogits are staged per wave in LDS and leave as 16-B stores at
//     the next interval's start;
//   * a workgroup walks its (vocabulary tile, row tile) items from a rotated start, so the E reloads of the 256
//     CUs (32 MB when they coincide) are spread over the launch.
namespace pp {
#ifndef VPP_EXPT
#define VPP_EXPT 0   // timing-only builds (tools/build_variant.sh): 1 no exp, 2 no fwd epilogue, 3 no dlogits
#endif               // stores, 4 no MFMAs
constexpr int BV = 256, BRT = 32, NJ = BRT / 16, PD = 2, NBUF = 2 * (PD + 1), SLD = 64 + 8;
constexpr int LDS_MAX = 163840;
template <int DK, bool BWD> struct C {
  static constexpr int KS = DK / 32;                  // 32-deep k steps
  static constexpr int CPR = DK / 8;                  // 16-B chunks per h row
  static constexpr int TILE = BRT * DK;               // h tile elements
  static constexpr int PIECES = TILE * 2 / 1024;      // 1-KB LDS-DMA pieces per h tile
  static constexpr int RPP = 1024 / (DK * 2);         // h rows per piece
  static constexpr int H_BYTES = NBUF * TILE * 2;
  static constexpr int BSL_BYTES = 8 * 64 * 4;        // per wave: its bias quarter
  static constexpr int RED_BYTES = BWD ? 0 : 2 * 2 * 4 * 4 * BRT * 8;   // fwd: [group][parity][quarter][g][BRT]
  static constexpr int STG_BYTES = BWD ? 8 * BRT * SLD * 2 : 0;     // bwd: per wave [BRT][SLD] bf16 dlogits
  static constexpr int FIXED = H_BYTES + BSL_BYTES + RED_BYTES + STG_BYTES;   // + bwd: 8 B per row of the range
};

typedef __attribute__((address_space(3))) void* lds_vptr;
__device__ __forceinline__ uint32_t lds_u32(const void* p) { return (uint32_t)(uintptr_t)(lds_vptr)p; }
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(dst)
               : "memory");
}
// s_waitcnt vmcnt(N) (expcnt / lgkmcnt not waited)
template <int N> __device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}
__device__ __forceinline__ void wait_vm_n(int n) {
  switch (n) {
    case 0: wait_vm<0>(); break;
    case 1: wait_vm<1>(); break;
    case 2: wait_vm<2>(); break;
    case 3: wait_vm<3>(); break;
    default: wait_vm<4>(); break;
  }
}
__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);     // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int DK, bool BWD>
__global__ __launch_bounds__(NTH, 1) void pp_kernel(Args a) {
  KStampBegin stamp_b_(a.ks);
  KStampEnd stamp_e_(a.ks);
  using P = C<DK, BWD>;
  constexpr int KS = P::KS, CPR = P::CPR;
  static_assert(2 * P::PIECES / 8 <= 4, "wait_vm_n covers up to 4 pieces per wave and interval");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* Hb = reinterpret_cast<bf16*>(smem);                                    // NBUF h tiles [BRT][DK], swizzled
  float* bsl = reinterpret_cast<float*>(smem + P::H_BYTES);                    // [wave][64]
  float2* red = reinterpret_cast<float2*>(smem + P::H_BYTES + P::BSL_BYTES);  // fwd
  bf16* stg = reinterpret_cast<bf16*>(smem + P::H_BYTES + P::BSL_BYTES + P::RED_BYTES);   // bwd

  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, cl = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), q = wave & 3, G = wave >> 2;
  const int64_t Rl = a.rows_dev ? min(a.R, (int64_t)*a.rows_dev) : a.R;
  const int nmt = (int)((Rl + BRT - 1) / BRT);
  const int mtb = (int)((int64_t)nmt * blockIdx.y / gridDim.y), mte = (int)((int64_t)nmt * (blockIdx.y + 1) / gridDim.y);
  const int nloc = mte - mtb;
  const int64_t nvt = (a.V1 + BV - 1) / BV;
  if (nloc <= 0 || (int64_t)blockIdx.x >= nvt) return;
  const int nvl = (int)((nvt - 1 - blockIdx.x) / gridDim.x + 1);         // this workgroup's vocabulary tiles
  const int F = nvl * nloc;                                               // items: (vocabulary tile, row tile)
  const int rot = (int)((blockIdx.x * 37u + blockIdx.y * 11u) % (unsigned)F);   // rotated start (see above)
  const int64_t rbase = (int64_t)mtb * BRT;
  const uint32_t hb0 = lds_u32(Hb);
  int* mlab = reinterpret_cast<int*>(smem + P::FIXED);          // bwd: [rows] label entry (-1: none here, -2: dead)
  float* mlse = reinterpret_cast<float*>(mlab + nloc * BRT);    // bwd: [rows] lse * log2(e) (+inf: dead)

  float sc = 0.f;
  if constexpr (BWD) {
    sc = (a.dloss ? *a.dloss : 1.f) / *a.count;
    for (int r = tid; r < nloc * BRT; r += NTH) {
      const int64_t row = rbase + r;
      int le = -2;
      float L = __builtin_inff();
      if (row < Rl) {
        const int64_t lb = a.labels[row];
        if (lb != 0) {
          const int64_t o = lb - a.voff;
          le = (o >= 0 && o < a.V1) ? (int)o : -1;
          L = a.lse[row] * 1.4426950408889634f;
        }
      }
      mlab[r] = le;
      mlse[r] = L;
    }
  }
  // flat item f (in processing order) -> (local vocabulary tile, row tile)
  // ff / nloc by a multiply-shift (nloc is the workgroup's constant; exact while ff * nloc < 2^40, i.e. always here:
  // ff < F = tiles x nloc) instead of an integer division sequence ~10 times per interval per wave
  const uint64_t dmag = (1ull << 40) / (uint64_t)nloc + 1;
  auto div_nloc = [&](int ff) { return (int)(((uint64_t)ff * dmag) >> 40); };
  auto item_vt = [&](int f) { const int ff = f + rot < F ? f + rot : f + rot - F; return div_nloc(ff); };
  auto item_u = [&](int f) { const int ff = f + rot < F ? f + rot : f + rot - F; return ff - div_nloc(ff) * nloc; };

  // items fa, fa + 1 -> h buffers fa % NBUF, (fa + 1) % NBUF: 2 * PIECES DMA pieces dealt over the 8 waves.  A
  // wave's pieces j all have j = wave (mod 8), so its lanes' (row in piece, swizzled chunk) are fixed: lane row
  // lr, source chunk hc; only the piece's first row (scalar) varies
  const int lr = lane / CPR;
  const int hc = 8 * ((lane % CPR) ^ swz<CPR>((wave % P::PIECES) * P::RPP + lr));
  auto issue = [&](int fa) {
#pragma unroll
    for (int p0 = 0; p0 < 2 * P::PIECES; p0 += 8) {
      const int p = p0 + wave, f = fa + p / P::PIECES, j = p % P::PIECES;
      if (f < F) {
        const int64_t rb = (int64_t)(mtb + item_u(f)) * BRT + j * P::RPP;
        const int64_t gr = min(rb + lr, Rl - 1);
        dma16(a.h + gr * a.ldh + hc,
              __builtin_amdgcn_readfirstlane(hb0 + (uint32_t)((f % NBUF) * P::TILE * 2 + j * 1024)));
      }
    }
  };
  // DMA pieces this wave issued for items fa, fa + 1
  auto issued = [&](int fa) {
    int c = 0;
#pragma unroll
    for (int p0 = 0; p0 < 2 * P::PIECES; p0 += 8) c += (fa + (p0 + wave) / P::PIECES < F) ? 1 : 0;
    return c;
  };

  bf16x8 ef[4][KS];          // this wave's E quarter of the current vocabulary tile (A operand fragments)
  f32x4 acc[4][NJ];          // S^T[vocab 64 q + 16 i + 4 g + r][row 16 j + cl] of the wave's last item
  int cur_vtl = -1;

  // E quarter + bias of local vocabulary tile vtl (waited here: no vector load may follow the interval's DMAs).
  // The bias goes to this wave's LDS slot, -inf past the vocabulary, which masks those entries (E rows past it
  // are clamped, so their products are finite)
  auto load_e = [&](int vtl) {
    cur_vtl = vtl;
    const int64_t vt = (int64_t)blockIdx.x + (int64_t)vtl * gridDim.x;
    const int64_t vb = vt * BV + 64 * q + lane;
    const float bv = vb < a.V1 ? (a.bias ? a.bias[vb] : 0.f) : -__builtin_inff();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t v = min(vt * BV + 64 * q + 16 * i + cl, a.V1 - 1);
#pragma unroll
      for (int s = 0; s < KS; ++s) ef[i][s] = *reinterpret_cast<const bf16x8*>(a.E + v * a.lde + 32 * s + 8 * g);
    }
    bsl[wave * 64 + lane] = bv;
    wait_vm<0>();
  };

  auto mfma_item = [&](int f) {
    const bf16* H = Hb + (f % NBUF) * P::TILE;
    // the accumulators start from the bias of their vocabulary rows (-inf past the vocabulary)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(bsl + wave * 64 + 16 * i + 4 * g);
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = b4;
    }
    // h fragments one k step ahead (the MFMA phase of a wave often has the SIMD to itself, so the LDS latency
    // must hide under its own MFMAs); the scheduling fence keeps the compiler from hoisting more steps' reads
    bf16x8 fb[2][NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) fb[0][j] = row_frag<CPR>(H, 16 * j, 0, lane);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (s + 1 < KS) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) fb[(s + 1) & 1][j] = row_frag<CPR>(H, 16 * j, 4 * (s + 1), lane);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          if (VPP_EXPT == 4) acc[i][j][0] += (float)fb[s & 1][j][0] * (float)ef[i][s][0];
          else acc[i][j] = mfma(ef[i][s], fb[s & 1][j], acc[i][j]);
        }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // fwd: softmax statistics of item f: per lane (max, sum) over its 16 entries of each of its rows (four
  // independent sum chains, no cross-lane step) -> red[G][parity][q][g][row]; the combine folds the 4 lane groups
  // x 2 quarters of a 128-column tile
  auto epi_fwd = [&](int f) {
    float2* rd = red + (((G * 2 + ((f >> 1) & 1)) * 4 + q) * 4 + g) * BRT;
    if (VPP_EXPT == 2) {
      rd[cl] = make_float2(acc[0][0][0], acc[3][NJ - 1][3]);
      return;
    }
    // per element: one 3-input max step (chains of v_max3), half a packed FMA and half a packed add (v_pk_fma_f32 /
    // v_pk_add_f32 on element pairs) and the exp -- the epilogue, not the MFMAs, bounds this kernel (timing-only
    // builds at cfg5: no MFMAs 1,119 us, no epilogue 815, all 1,270)
    typedef __attribute__((ext_vector_type(2))) float f2;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      float mx = acc[0][j][0];
#pragma unroll
      for (int t = 1; t + 1 < 16; t += 2)
        mx = fmaxf(fmaxf(mx, acc[t >> 2][j][t & 3]), acc[(t + 1) >> 2][j][(t + 1) & 3]);
      mx = fmaxf(mx, acc[3][j][3]);
      const float mxl = mx * 1.4426950408889634f;
      const f2 l2 = {1.4426950408889634f, 1.4426950408889634f}, nm = {-mxl, -mxl};
      f2 sp[2] = {{0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          const f2 a = {acc[i][j][r], acc[i][j][r + 1]};
          const f2 ea = __builtin_elementwise_fma(a, l2, nm);
          f2 e;
          e.x = VPP_EXPT == 1 ? ea.x : __builtin_amdgcn_exp2f(ea.x);
          e.y = VPP_EXPT == 1 ? ea.y : __builtin_amdgcn_exp2f(ea.y);
          sp[(r >> 1) & 1] += e;
        }
      const float sm = mx == -__builtin_inff() ? 0.f : (sp[0].x + sp[0].y) + (sp[1].x + sp[1].y);
      rd[16 * j + cl] = make_float2(mx, sm);
    }
  };

  // fwd: lane groups x quarters {0, 1} / {2, 3} of item f -> its two 128-column partial tiles (one barrier after
  // epi_fwd(f)); the fold order is fixed
  auto combine = [&](int f) {
    const int tg = tid & 255;
    if (tg < 2 * BRT) {
      const int rl = tg & (BRT - 1), half = tg / BRT;
      const int64_t n0 = ((int64_t)blockIdx.x + (int64_t)item_vt(f) * gridDim.x) * BV;
      const int64_t row = (int64_t)(mtb + item_u(f)) * BRT + rl, pt = (n0 >> 7) + half;
      const float2* rd = red + (G * 2 + ((f >> 1) & 1)) * 16 * BRT + 2 * half * 4 * BRT + rl;
      float2 e[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) e[k] = rd[k * BRT];
      float mx = e[0].x;
#pragma unroll
      for (int k = 1; k < 8; ++k) mx = fmaxf(mx, e[k].x);
      float sm = 0.f;
      if (mx != -__builtin_inff()) {
#pragma unroll
        for (int k = 0; k < 8; ++k) sm += e[k].y * __expf(e[k].x - mx);
      }
      if (row < Rl && pt < a.ntn) *reinterpret_cast<float2*>(a.part + (row * a.ntn + pt) * 2) = make_float2(mx, sm);
    }
  };

  // bwd: dlogits of item f over this wave's quarter -> the wave's LDS stage [row][64 entries] (a lane holds 4
  // consecutive entries of a row: one 8-B write).  Dead rows take lse = +inf and scale 0: exactly 0, no select
  bf16* st = stg + wave * BRT * SLD;
  auto epi_bwd = [&](int f) {
    const int u = item_u(f);
    const int64_t vb = ((int64_t)blockIdx.x + (int64_t)item_vt(f) * gridDim.x) * BV + 64 * q + 4 * g;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int rr = u * BRT + 16 * j + cl;
      const int le = mlab[rr];
      const float Ll = mlse[rr];
      const float scr = le == -2 ? 0.f : sc;
      const int64_t offl = (int64_t)le - vb;             // the label's entry among this lane's rows
      const int off = le < 0 || offl < 0 || offl >= 64 ? -1 : (int)offl;
      // element pairs on packed FMA / add / mul (the same operations per element, so the same bits)
      typedef __attribute__((ext_vector_type(2))) float f2;
      const f2 l2 = {1.4426950408889634f, 1.4426950408889634f}, nl = {-Ll, -Ll}, s2 = {scr, scr};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        bf4 o;
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          const f2 a = {acc[i][j][r], acc[i][j][r + 1]};
          const f2 ea = __builtin_elementwise_fma(a, l2, nl);
          f2 e;
          e.x = VPP_EXPT == 1 ? ea.x : __builtin_amdgcn_exp2f(ea.x);
          e.y = VPP_EXPT == 1 ? ea.y : __builtin_amdgcn_exp2f(ea.y);
          const f2 oh = {off == 16 * i + r ? 1.f : 0.f, off == 16 * i + r + 1 ? 1.f : 0.f};
          const f2 t = (e - oh) * s2;
          o[r] = (bf16)t.x;
          o[r + 1] = (bf16)t.y;
        }
        *reinterpret_cast<bf4*>(st + (16 * j + cl) * SLD + 16 * i + 4 * g) = o;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // bwd: the stage of item f -> dlogits, 16-B stores (8 rows x 128 B per instruction); rows >= the live count are
  // not written; a chunk starting below V1 may run into the row's padding up to lddl (zeros there)
  auto flush = [&](int f) {
    const int u = item_u(f);
    const int64_t c0 = ((int64_t)blockIdx.x + (int64_t)item_vt(f) * gridDim.x) * BV + 64 * q;
#pragma unroll
    for (int k = 0; k < BRT / 8; ++k) {
      const int r = 8 * k + (lane >> 3), ch = lane & 7;
      const int64_t row = (int64_t)(mtb + u) * BRT + r, v = c0 + 8 * ch;
      const bf16x8 x = *reinterpret_cast<const bf16x8*>(st + r * SLD + 8 * ch);
      if (row < Rl && v < a.V1 && (VPP_EXPT != 3 || a.V1 < 0)) *reinterpret_cast<bf16x8*>(a.dl + row * a.lddl + v) = x;
    }
  };

  const int NI = (F + 1) / 2;
  issue(0);
  issue(2);
#pragma unroll 1
  for (int n = 0; n <= NI + 1; ++n) {
    wait_vm_n(issued(2 * n + 2));      // items 2n, 2n + 1 landed (this wave's); interval n + 1's may be in flight
    raw_barrier();                     // ... everyone's; interval n - 1's readers are done
    const int fm = 2 * n + G, fe = 2 * n - G, fc = fe - 2;
    if constexpr (BWD) {
      if (fc >= 0 && fc < F) flush(fc);
    } else {
      if (fc >= 0 && fc < F) combine(fc);
    }
    if (fm < F && item_vt(fm) != cur_vtl) load_e(item_vt(fm));
    if (2 * n + 4 < F) issue(2 * n + 4);
    // group 0: MFMAs of item 2n, then its epilogue; group 1: epilogue of item 2n - 1, then the MFMAs of 2n + 1
    // (one copy of each phase in the code: phase ph runs the MFMAs where ph == G)
#pragma unroll 1
    for (int ph = 0; ph < 2; ++ph) {
      if (ph == G) {
        if (fm < F) mfma_item(fm);
      } else if (fe >= 0 && fe < F) {
        if constexpr (BWD) epi_bwd(fe);
        else epi_fwd(fe);
      }
    }
  }
}

// returns hipErrorNotSupported when the backward's per-row metadata would not fit LDS (the caller falls back)
template <int DK, bool BWD>
hipError_t launch_pp(Args& a, hipStream_t s) {
  using P = C<DK, BWD>;
  static_assert(P::FIXED <= LDS_MAX, "LDS budget");
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t nvt = cdiv(a.V1, BV);
  const int64_t grid = std::min<int64_t>(nvt, (int64_t)cus);
  const int64_t nmt = cdiv(a.R, BRT);
  const int64_t gy = std::max<int64_t>(1, std::min<int64_t>(nmt, (int64_t)cus / nvt));
  const int64_t lds = P::FIXED + (BWD ? 8 * BRT * cdiv(nmt, gy) : 0);
  if (lds > LDS_MAX) return hipErrorNotSupported;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)pp_kernel<DK, BWD>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    attr = true;
  }
  hipLaunchKernelGGL((pp_kernel<DK, BWD>), dim3((unsigned)grid, (unsigned)gy), dim3(NTH), (unsigned)lds, s, a);
  return hipGetLastError();
}
}  // namespace pp

// RS_VHEAD_PP=0 selects the lock-step forms (read per launch, for A/B); default: the ping-pong forms
// (R = 1,750, 1M + 1 classes, d = 256: fwd 1,876 -> 1,427 us, bwd 3,064 -> 1,715 us; cfg3's 26,745 classes:
// 74.1 -> 62.6 / 86.8 -> 61.1 us; tools/vhead_bench.py, same session)
inline bool use_pp() {
  const char* e = getenv("RS_VHEAD_PP");
  return e ? atoi(e) != 0 : true;
}

// lock-step forms: fwd 256-entry vocabulary tiles (E tile 132 KB at d = 256); bwd 128 (room for the dlogits
// staging tile)
template <bool BWD>
hipError_t dispatch(Args& a, int64_t d, hipStream_t s) {
  constexpr int BV = BWD ? 128 : 256;
  if (use_pp()) {
    const hipError_t e = d == 256 ? pp::launch_pp<256, BWD>(a, s)
                         : d == 128 ? pp::launch_pp<128, BWD>(a, s) : pp::launch_pp<64, BWD>(a, s);
    if (e != hipErrorNotSupported) return e;
  }
  if (d == 256) return launch<256, BV, BWD>(a, s);
  if (d == 128) return launch<128, BV, BWD>(a, s);
  return launch<64, BV, BWD>(a, s);
}

}  // namespace vh

// partials -> lse / loss (vocab_ce.hip); with h != null the label logits are formed there (<h, E[label]> + b)
hipError_t vce_finish(const float* part, int64_t ntn, int64_t R, const int64_t* labels, const float* tgt,
                      const int* rows_dev, float* lse, float* rowp, const float* count_override, float* out,
                      hipStream_t s, const void* h, int64_t ldh, const void* E, int64_t lde, const float* bias,
                      int64_t d);

extern "C" {

int rs_vocab_head_supported(int64_t d) { return d == 64 || d == 128 || d == 256; }

int rs_vocab_head_fwd(int64_t R, int64_t V1, int64_t d, const void* h, int64_t ldh, const void* E, int64_t lde,
                      const float* bias, const int64_t* labels, const int* rows_dev, const float* count_override,
                      float* ws, float* out, void* stream) {
  if (!rs_vocab_head_supported(d) || R <= 0 || V1 <= 0 || ldh % 8 || lde % 8 || ((uintptr_t)h | (uintptr_t)E) % 16 ||
      !labels || !ws || !out)
    return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  vh::Args a{};
  a.R = R; a.V1 = V1; a.ntn = cdiv(V1, 128);
  a.h = (const __bf16*)h; a.ldh = ldh; a.E = (const __bf16*)E; a.lde = lde;
  a.bias = bias; a.labels = labels; a.rows_dev = rows_dev;
  // ws layout = vocab_ce.hip's: part [R][ntn][2] | tgt [R] | lse [R] | rowp [R][2]
  a.part = ws;
  a.tgt = ws + R * a.ntn * 2;
  a.ks = kstamp_next(RS_STAMP_VOCAB_CE_FWD);
  hipError_t e = vh::dispatch<false>(a, d, s);
  if (e != hipSuccess) return (int)e;
  return (int)vce_finish(a.part, a.ntn, R, labels, a.tgt, rows_dev, a.tgt + R, a.tgt + 2 * R, count_override, out, s,
                         h, ldh, E, lde, bias, d);
}

int rs_vocab_head_bwd(int64_t R, int64_t V1, int64_t d, const void* h, int64_t ldh, const void* E, int64_t lde,
                      const float* bias, const int64_t* labels, const int* rows_dev, const float* count,
                      const float* dloss, const float* ws, void* dlogits, int64_t lddl, int64_t voff, void* stream) {
  if (!rs_vocab_head_supported(d) || R <= 0 || V1 <= 0 || ldh % 8 || lde % 8 || lddl % 8 ||
      ((uintptr_t)h | (uintptr_t)E | (uintptr_t)dlogits) % 16 || !labels || !ws || !count || !dlogits)
    return RS_ERR_ARG;
  vh::Args a{};
  a.R = R; a.V1 = V1; a.ntn = cdiv(V1, 128);
  a.h = (const __bf16*)h; a.ldh = ldh; a.E = (const __bf16*)E; a.lde = lde;
  a.bias = bias; a.labels = labels; a.rows_dev = rows_dev;
  a.lse = ws + R * a.ntn * 2 + R;
  a.count = count; a.dloss = dloss;
  a.dl = (__bf16*)dlogits; a.lddl = lddl;
  a.voff = voff;
  return (int)vh::dispatch<true>(a, d, (hipStream_t)stream);
}

}  // extern "C"

// ---- vocabulary-sharded head (data-parallel ranks each own a slice of E = out.weight) ---------------
namespace vh {

// one wave per row: log-sum-exp of the row's 128-column partials over this shard (0 for dead rows)
__global__ __launch_bounds__(256) void shard_lse_kernel(const float* __restrict__ part, int64_t ntn, int64_t R,
                                                        const int64_t* __restrict__ labels, float* __restrict__ lse) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  if (labels[r] == 0) {
    if (lane == 0) lse[r] = 0.f;
    return;
  }
  float mx = -__builtin_inff(), sm = 0.f;
  const float2* pr = reinterpret_cast<const float2*>(part + r * ntn * 2);
  int64_t t = lane;
  constexpr int U = 8;   // eight tiles in flight per lane, folded against their common max (vocab_ce.hip's finish)
  for (; t + 64 * (U - 1) < ntn; t += 64 * U) {
    float2 q[U];
#pragma unroll
    for (int u = 0; u < U; ++u) q[u] = pr[t + 64 * u];
    float mm = mx;
#pragma unroll
    for (int u = 0; u < U; ++u) mm = fmaxf(mm, q[u].x);
    if (mm != -__builtin_inff()) {
      float acc = sm * __expf(mx - mm);
#pragma unroll
      for (int u = 0; u < U; ++u) acc += q[u].y * __expf(q[u].x - mm);
      sm = acc;
      mx = mm;
    }
  }
  for (; t < ntn; t += 64) comb(mx, sm, pr[t].x, pr[t].y);
  for (int o = 32; o > 0; o >>= 1) comb(mx, sm, __shfl_xor(mx, o, 64), __shfl_xor(sm, o, 64));
  if (lane == 0) lse[r] = mx + __logf(sm);
}

// one wave per row: the label's logit <h, E[label - v0]> + b when this shard holds the label, else 0
__global__ __launch_bounds__(256) void shard_label_kernel(int64_t R, int64_t d, const bf16* __restrict__ h,
                                                          int64_t ldh, const bf16* __restrict__ E, int64_t lde,
                                                          const float* __restrict__ bias,
                                                          const int64_t* __restrict__ labels, int64_t v0, int64_t v1,
                                                          float* __restrict__ tgt) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const int64_t lb = labels[r];
  if (lb == 0 || lb < v0 || lb >= v1) {
    if (lane == 0) tgt[r] = 0.f;
    return;
  }
  float dot = 0.f;
  for (int64_t k = lane; k < d; k += 64) dot += (float)h[r * ldh + k] * (float)E[(lb - v0) * lde + k];
  dot = wave_sum(dot);
  if (lane == 0) tgt[r] = dot + (bias ? bias[lb - v0] : 0.f);
}

// every shard's per-row lse [N][R] -> the row's lse over the whole vocabulary; loss over live rows
__global__ __launch_bounds__(256) void shard_combine_kernel(int N, int64_t R, const float* __restrict__ lse_parts,
                                                            const float* __restrict__ tgt,
                                                            const int64_t* __restrict__ labels,
                                                            float* __restrict__ lse, float* __restrict__ out) {
  float s = 0.f, c = 0.f;
  for (int64_t r = threadIdx.x; r < R; r += blockDim.x) {
    if (labels[r] == 0) {
      lse[r] = 0.f;
      continue;
    }
    float mx = -__builtin_inff();
    for (int q = 0; q < N; ++q) mx = fmaxf(mx, lse_parts[q * R + r]);
    float sm = 0.f;
    for (int q = 0; q < N; ++q) sm += __expf(lse_parts[q * R + r] - mx);
    const float L = mx + __logf(sm);
    lse[r] = L;
    s += L - tgt[r];
    c += 1.f;
  }
  __shared__ float rs[4], rc[4];
  s = wave_sum(s);
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0) { rs[threadIdx.x >> 6] = s; rc[threadIdx.x >> 6] = c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float S = rs[0] + rs[1] + rs[2] + rs[3], Cn = rc[0] + rc[1] + rc[2] + rc[3];
    out[0] = S;
    out[1] = Cn;
    out[2] = Cn > 0.f ? S / Cn : 0.f;
  }
}

}  // namespace vh

extern "C" {

int rs_vocab_shard_lse(int64_t R, int64_t V1s, int64_t d, const void* h, int64_t ldh, const void* E, int64_t lde,
                       const float* bias, const int64_t* labels, float* ws, float* lse, void* stream) {
  if (!rs_vocab_head_supported(d) || R <= 0 || V1s <= 0 || ldh % 8 || lde % 8 || ((uintptr_t)h | (uintptr_t)E) % 16 ||
      !labels || !ws || !lse)
    return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  vh::Args a{};
  a.R = R; a.V1 = V1s; a.ntn = cdiv(V1s, 128);
  a.h = (const __bf16*)h; a.ldh = ldh; a.E = (const __bf16*)E; a.lde = lde;
  a.bias = bias; a.labels = labels;
  a.part = ws;
  a.tgt = ws + R * a.ntn * 2;
  hipError_t e = vh::dispatch<false>(a, d, s);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(vh::shard_lse_kernel, dim3((unsigned)cdiv(R, 4)), dim3(256), 0, s, a.part, a.ntn, R, labels, lse);
  return (int)hipGetLastError();
}

int rs_vocab_shard_label_logits(int64_t R, int64_t d, const void* h, int64_t ldh, const void* E, int64_t lde,
                                const float* bias, const int64_t* labels, int64_t v0, int64_t v1, float* tgt,
                                void* stream) {
  if (R <= 0 || d <= 0 || !h || !E || !labels || !tgt) return RS_ERR_ARG;
  hipLaunchKernelGGL(vh::shard_label_kernel, dim3((unsigned)cdiv(R, 4)), dim3(256), 0, (hipStream_t)stream, R, d,
                     (const __bf16*)h, ldh, (const __bf16*)E, lde, bias, labels, v0, v1, tgt);
  return (int)hipGetLastError();
}

int rs_vocab_shard_combine(int N, int64_t R, const float* lse_parts, const float* tgt, const int64_t* labels,
                           float* lse, float* out, void* stream) {
  if (N <= 0 || R <= 0 || !lse_parts || !tgt || !labels || !lse || !out) return RS_ERR_ARG;
  hipLaunchKernelGGL(vh::shard_combine_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, N, R, lse_parts, tgt, labels,
                     lse, out);
  return (int)hipGetLastError();
}

}  // extern "C"
