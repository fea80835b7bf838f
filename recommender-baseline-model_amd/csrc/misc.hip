// Optimizer and elementwise helpers (gfx950), all HBM-bound streaming kernels.
//
//   rs_adam_prepare / rs_adam_step   torch.optim.Adam as built in BS/trainers/base.py:225-228
//                                    (one fused sweep over the flat fp32 parameter buffer;
//                                    optionally emits the bf16 weight copy the GEMMs read)
//   rs_cast_bf16                     fp32 master weights -> bf16 compute copy
//   rs_colsum                        bias gradients (sum over token rows), deterministic
//   rs_dropout_rowmask               dropout/timeline-mask backward for SAS FFN dropout2
//                                    (BS/models/sas_model/sas.py:17,84)
#include "adam_math.h"
#include "common.h"
#include "../../include/recsys_hip.h"

__device__ __forceinline__ void adam_commit(double* state, double t, AdamScalars c, uint64_t* seed_base) {
  if (seed_base) *seed_base += 1;   // next step's dropout masks (rs_seed_advance folded in)
  state[0] = t;
  state[1] = c.step_size;
  state[2] = c.bc2s;
  state[3] = c.gs;
}

__global__ void adam_prepare_kernel(double* state, const double* hyper, const float* divisor, uint64_t* seed_base) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const double t = state[0] + 1.0;
  adam_commit(state, t, adam_scalars(t, hyper, divisor), seed_base);
}

// PREP: the launch also does rs_adam_prepare's work -- every workgroup derives step t = state[0] + 1's
// scalars itself, and the LAST workgroup to finish (arrival counter in state[7]) writes them back, advances
// the step count and the dropout seed, and re-arms the counter.  One launch instead of two on the step's
// critical path.
// streaming float4 access; NT: nontemporal (slc / nt) loads and stores for the optimizer's single-use sweeps
typedef float f4v __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ float4 ld4(const float* a, int64_t i) {
  if (NT) {
    const f4v x = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(a) + i);
    return make_float4(x[0], x[1], x[2], x[3]);
  }
  return reinterpret_cast<const float4*>(a)[i];
}
template <bool NT>
__device__ __forceinline__ void st4(float* a, int64_t i, float4 v) {
  if (NT) {
    const f4v x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<f4v*>(a) + i);
  } else {
    reinterpret_cast<float4*>(a)[i] = v;
  }
}

// one float4 of the Adam update (torch.optim.Adam, BS/trainers/base.py:225-228) + its stores
template <bool BF16OUT, bool NT>
__device__ __forceinline__ void adam4(int64_t i, float4 pp, float4 gg, float4 mm, float4 vv, float* __restrict__ p,
                                      float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
                                      __bf16* __restrict__ pb, AdamElem h,
                                      float step_size, float bc2s, float gs, int zero_grad,
                                      const int64_t* __restrict__ tdesc, int ntd, int64_t tbase,
                                      __bf16* __restrict__ wT, int64_t tlo, int64_t thi) {
  float* P = &pp.x; float* G = &gg.x; float* Mv = &mm.x; float* Vv = &vv.x;
#pragma unroll
  for (int j = 0; j < 4; ++j) adam_elem_update(P[j], G[j], Mv[j], Vv[j], h, step_size, bc2s, gs);
  st4<NT>(p, i, pp);
  st4<NT>(m, i, mm);
  st4<NT>(v, i, vv);
  // zero_grad: only where the gradient is not already zero -- the table rows no token of the step touched (most of
  // a large item / token table) keep their zeros without a store (4 of the 34 bytes per element)
  if (zero_grad && (__float_as_uint(gg.x) | __float_as_uint(gg.y) | __float_as_uint(gg.z) | __float_as_uint(gg.w)))
    reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (BF16OUT) {
    bf16x4 o;
    o[0] = (__bf16)P[0]; o[1] = (__bf16)P[1]; o[2] = (__bf16)P[2]; o[3] = (__bf16)P[3];
    if (NT) {
      uint64_t w;
      __builtin_memcpy(&w, &o, 8);
      __builtin_nontemporal_store(w, reinterpret_cast<uint64_t*>(pb) + i);
    } else {
      reinterpret_cast<bf16x4*>(pb)[i] = o;
    }
    // transposed bf16 copies of matrices inside the buffer (the SAS backward's [in][out] block weights,
    // rs_transpose_bf16's desc layout): the 4 elements share a row (host checks lds % 4 == 0)
    // the descriptors' element span [tlo, thi) first: most of the buffer (the tables) is outside every matrix
    const int64_t e0 = tbase + 4 * i;
    const int nk = (e0 >= tlo && e0 < thi) ? ntd : 0;
    for (int k = 0; k < nk; ++k) {
      const int64_t* dk = tdesc + 6 * k;
      const int64_t rel = tbase + 4 * i - dk[2];
      if (rel >= 0 && rel < dk[0] * dk[3]) {
        // 32-bit division (a weight matrix: rows * row stride < 2^31, host-checked); the 64-bit one is a
        // ~60-instruction sequence per float4 of every transposed weight
        const uint32_t ru = (uint32_t)rel, ld = (uint32_t)dk[3];
        const int64_t r = ru / ld, c = ru - (uint32_t)r * ld;
        if (c < dk[1]) {
          __bf16* t = wT + dk[4] + c * dk[5] + r;
#pragma unroll
          for (int j = 0; j < 4; ++j) t[j * dk[5]] = o[j];
        }
      }
    }
  }
}

// rows of a table whose gradient only the item-gradient kernels write (rs_item_grad_marked): marks[row] == *epoch for
// every row they wrote this step (and possibly for rows of an old step: harmless, their gradient reads as zero), so a
// row without the mark has a zero gradient and the sweep skips its load -- 4 of the 30 bytes per element of a table
// whose rows a batch mostly does not touch (cfg5's 1M-row token table, cfg4's 54k-row item table)
struct RowMarks {
  const uint8_t* marks;
  const uint8_t* epoch;
  const float* zeros;   // 1 KB of zeros after the marks (16-B aligned)
  int64_t moff;       // launch element index of the table's row 0 (may be negative: the launch starts inside it)
  int64_t mlo, mhi;   // launch element range covered by the table
  int dshift;         // log2(row width)
};

// The marks of a wave's rows by SCALAR loads (constant address space, wave-uniform address): lgkmcnt-counted, so
// consuming them does not wait for the wave's vector loads in flight (vmcnt retires in order -- a per-lane byte
// load before the gradient load made every group wait for all earlier loads: two round trips per group).  A
// wave's 64 float4 span 256 elements, at most 3 rows of >= 128: the 16 mark bytes from the row of its first
// active lane (rounded down to 8) cover them (row_marks arrays carry 16 bytes of padding).
typedef __attribute__((address_space(4))) const uint64_t* const_u64p;
template <bool MK>
__device__ __forceinline__ bool row_touched(int64_t i, const RowMarks& rm, uint8_t ep) {
  if (!MK) return true;
  const int64_t e = 4 * i;
  const bool inside = e >= rm.mlo && e < rm.mhi;
  // lanes outside the table take row 0: every scalar load stays inside [0, mrows + 15] (a wave straddling the
  // table's start holds rows 0..2 inside it; one straddling its end starts inside)
  const int64_t r = inside ? (e - rm.moff) >> rm.dshift : 0;
  const int rf = __builtin_amdgcn_readfirstlane((int)r) & ~7;
  const const_u64p w = (const_u64p)(rm.marks + rf);
  const uint64_t lo = w[0], hi = w[1];
  const int k = (int)r - rf;
  const uint64_t word = k < 8 ? lo : hi;
  const uint8_t mk = (uint8_t)(word >> (8 * (k & 7)));
  return !inside || mk == ep;
}

template <bool BF16OUT, bool PREP, int U, bool NT, bool MK>
__global__ __launch_bounds__(256) void adam_step_kernel(int64_t n, float* __restrict__ p, float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        __bf16* __restrict__ pb, double* __restrict__ state,
                                                        const double* __restrict__ hyper, int zero_grad,
                                                        const float* __restrict__ divisor, uint64_t* seed_base,
                                                        const int64_t* __restrict__ tdesc, int ntd, int64_t tbase,
                                                        __bf16* __restrict__ wT, const float* __restrict__ lsum,
                                                        float* __restrict__ lout, RowMarks rm) {
  const AdamElem h = adam_elem(hyper);
  const uint8_t ep = MK ? *rm.epoch : 0;
  // data parallel: the step's reported loss = all-reduced loss sum / all-reduced count (the division torch.div did
  // in its own launch), by one thread: both inputs are final before this launch
  if (PREP && lout && blockIdx.x == 0 && threadIdx.x == 0) *lout = lsum[0] / divisor[0];
  float step_size, bc2s, gs;
  double t = 0.0;
  AdamScalars c;
  if (PREP) {
    t = state[0] + 1.0;
    c = adam_scalars(t, hyper, divisor);
    step_size = c.step_size; bc2s = c.bc2s; gs = c.gs;
  } else {
    step_size = (float)state[1];
    bc2s = (float)state[2];
    gs = (float)state[3];
  }
  int64_t tlo = 0, thi = 0;
  if (BF16OUT && ntd > 0) {
    tlo = INT64_MAX;
    for (int k = 0; k < ntd; ++k) {
      const int64_t* dk = tdesc + 6 * k;
      tlo = min(tlo, dk[2]);
      thi = max(thi, dk[2] + dk[0] * dk[3]);
    }
  }
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  // U float4 per thread in flight: every load of the group is issued before the first store
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    float4 pq[U], gq[U], mq[U], vq[U];
    bool tq[U];
#pragma unroll
    for (int u = 0; u < U; ++u) tq[u] = row_touched<MK>(i + u * stride, rm, ep);
    if (MK) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      pq[u] = ld4<NT>(p, i + u * stride);
      // an unstamped row's lanes read zeros from the marks' zero tail (a hot 1 KB) instead of HBM: one load either
      // way, no branch around it
      gq[u] = MK ? *(tq[u] ? reinterpret_cast<const float4*>(g) + i + u * stride
                           : reinterpret_cast<const float4*>(rm.zeros) + (threadIdx.x & 63))
                 : ld4<NT>(g, i + u * stride);
      mq[u] = ld4<NT>(m, i + u * stride);
      vq[u] = ld4<NT>(v, i + u * stride);
    }
    // marked: all U groups' loads issued before the first use (the scheduler otherwise sinks group u+1's loads and
    // its mark loads below group u's update).  Unmarked: left to the scheduler, which issues group u+1's loads after
    // group u's -- forcing all eight in flight measured slower (256M elements at 256 / 512 workgroups: 1,460-1,472
    // -> 1,486-1,491 / 1,508-1,519 -> 1,621-1,624 us)
    if (MK) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u)
      adam4<BF16OUT, NT>(i + u * stride, pq[u], gq[u], mq[u], vq[u], p, g, m, v, pb, h, step_size, bc2s, gs,
                     zero_grad, tdesc, ntd, tbase, wT, tlo, thi);
  }
  for (; i < n4; i += stride) {
    float4 pp = ld4<NT>(p, i);
    const bool tt = row_touched<MK>(i, rm, ep);
    float4 gg = MK ? *(tt ? reinterpret_cast<const float4*>(g) + i
                          : reinterpret_cast<const float4*>(rm.zeros) + (threadIdx.x & 63))
                   : ld4<NT>(g, i);
    float4 mm = ld4<NT>(m, i);
    float4 vv = ld4<NT>(v, i);
    adam4<BF16OUT, NT>(i, pp, gg, mm, vv, p, g, m, v, pb, h, step_size, bc2s, gs, zero_grad, tdesc, ntd,
                   tbase, wT, tlo, thi);
  }
  // tail
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const int64_t j = n4 * 4 + threadIdx.x;
    adam_elem_update(p[j], g[j], m[j], v[j], h, step_size, bc2s, gs);
    if (BF16OUT) pb[j] = (__bf16)p[j];
    if (zero_grad) g[j] = 0.f;
  }
  if (PREP) {
    // every lane of this workgroup has read state[0] above; once all workgroups have arrived, the
    // last one publishes step t.  A relaxed counter suffices: nothing the other workgroups wrote is read
    // by the last one (the kernel boundary publishes the parameters), only the order "all reads of state
    // before its overwrite" matters, and each workgroup's reads complete before its arrival.  (A
    // __threadfence() here -- an L2 writeback per workgroup on gfx950 -- made the launch 30 us.)
    // Arrivals count per XCD group first (workgroup b runs on XCD b % 8; one counter per 128-B line), the
    // last of each group then counts at the top: ~80 same-address atomics per line in parallel instead of
    // every workgroup serialising on one address (13.8 us for the launch with a single counter).
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned x = blockIdx.x & 7u;
      const unsigned in_x = (gridDim.x >> 3) + (x < (gridDim.x & 7u) ? 1u : 0u);
      unsigned int* local = reinterpret_cast<unsigned int*>(state + 16 + 16 * x);
      unsigned int* top = reinterpret_cast<unsigned int*>(state + 7);
      const unsigned groups = gridDim.x < 8u ? gridDim.x : 8u;
      if (__hip_atomic_fetch_add(local, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == in_x - 1) {
        *local = 0u;
        if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == groups - 1) {
          adam_commit(state, t, c, seed_base);
          *top = 0u;
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void cast_bf16_kernel(int64_t n, const float* __restrict__ src, __bf16* __restrict__ dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = (__bf16)src[i];
}

#define COLSUM_BLOCKS 64
// block = 256 threads = CPR chunk-columns (16 B each) x (256/CPR) row groups; every block sums
// a contiguous range of rows, the row groups are combined in LDS in a fixed order.
template <typename T, int CPR>
__global__ __launch_bounds__(256) void colsum_partial_v_kernel(const T* __restrict__ X, int64_t M, int64_t N,
                                                               int64_t ldx, float* __restrict__ ws) {
  constexpr int V = Vec<T>::N, RG = 256 / CPR;
  const int cc = threadIdx.x % CPR, rg = threadIdx.x / CPR;
  const int64_t rows_per = cdiv(M, (int64_t)gridDim.x);
  const int64_t r0 = blockIdx.x * rows_per, r1 = min(M, r0 + rows_per);
  float acc[V];
#pragma unroll
  for (int j = 0; j < V; ++j) acc[j] = 0.f;
  const bool active = cc * V < N;
  if (active) {
    for (int64_t r = r0 + rg; r < r1; r += RG) {
      float v[V];
      load_chunk<T>(v, X + r * ldx + cc * V);
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] += v[j];
    }
  }
  __shared__ float red[RG][CPR * V];
#pragma unroll
  for (int j = 0; j < V; ++j) red[rg][cc * V + j] = acc[j];
  __syncthreads();
  for (int c = threadIdx.x; c < N; c += 256) {
    float t = 0.f;
    for (int g = 0; g < RG; ++g) t += red[g][c];
    ws[blockIdx.x * N + c] = t;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void colsum_partial_kernel(const T* __restrict__ X, int64_t M, int64_t N, int64_t ldx,
                                                             float* __restrict__ ws) {
  const int64_t rows_per = cdiv(M, (int64_t)gridDim.x);
  const int64_t r0 = blockIdx.x * rows_per, r1 = min(M, r0 + rows_per);
  for (int64_t c = threadIdx.x; c < N; c += blockDim.x) {
    float s = 0.f;
    for (int64_t r = r0; r < r1; ++r) s += to_f(X[r * ldx + c]);
    ws[blockIdx.x * N + c] = s;
  }
}

template <typename T>
static hipError_t colsum_partial(const T* X, int64_t M, int64_t N, int64_t ldx, float* ws, int nblk, hipStream_t s) {
  constexpr int V = Vec<T>::N;
  const bool vec = (N % V == 0) && (ldx % V == 0) && ((uintptr_t)X % 16 == 0);
  const int64_t cpr = N / V;
  if (vec && cpr <= 16)
    hipLaunchKernelGGL((colsum_partial_v_kernel<T, 16>), dim3(nblk), dim3(256), 0, s, X, M, N, ldx, ws);
  else if (vec && cpr <= 32)
    hipLaunchKernelGGL((colsum_partial_v_kernel<T, 32>), dim3(nblk), dim3(256), 0, s, X, M, N, ldx, ws);
  else if (vec && cpr <= 64)
    hipLaunchKernelGGL((colsum_partial_v_kernel<T, 64>), dim3(nblk), dim3(256), 0, s, X, M, N, ldx, ws);
  else
    hipLaunchKernelGGL((colsum_partial_kernel<T>), dim3(nblk), dim3(256), 0, s, X, M, N, ldx, ws);
  return hipGetLastError();
}

template <typename T>
__global__ __launch_bounds__(256) void dropout_rowmask_kernel(const T* __restrict__ x, int64_t M, int64_t N, int64_t ld,
                                                              float p, uint64_t salt, const uint64_t* seed_base,
                                                              int64_t drop_ld, const int64_t* __restrict__ ids,
                                                              T* __restrict__ out, T* __restrict__ out_masked) {
  const uint64_t seed = eff_seed(salt, seed_base);
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= M * N) return;
  const int64_t m = i / N, c = i % N;
  float v = to_f(x[m * ld + c]);
  if (ids && ids[m] == 0) v = 0.f;
  if (out_masked) out_masked[m * ld + c] = from_f<T>(v);
  if (p > 0.f) v *= drop_mul(p, seed, (uint64_t)(m * drop_ld + c));
  out[m * ld + c] = from_f<T>(v);
}


// 8 columns per thread (N, ld, drop_ld multiples of 8; 16-B aligned rows): the same masks as
// dropout_rowmask_kernel (element m*drop_ld+c, drop_mul2 pairs = drop_mul).  TWO: the chained
// backward of two stacked dropouts, out = round(x * m1) and out2 = round(out * m2) in one pass
// (BERT's block-output and residual dropouts, bert.py encode_backward).
template <typename T, bool TWO>
__global__ __launch_bounds__(256) void dropout_v8_kernel(const T* __restrict__ x, int64_t M, int64_t N, int64_t ld,
                                                         float p, uint64_t salt, uint64_t salt2,
                                                         const uint64_t* seed_base, int64_t drop_ld,
                                                         const int64_t* __restrict__ ids, T* __restrict__ out,
                                                         T* __restrict__ out2) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t n8 = N >> 3;
  if (i >= M * n8) return;
  const int64_t m = i / n8, c = (i - m * n8) * 8;
  const bool keep = !ids || ids[m] != 0;
  float v[8];
  if (sizeof(T) == 2) {
    load_chunk<__bf16>(v, reinterpret_cast<const __bf16*>(x) + m * ld + c);
  } else {
    load_chunk<float>(v, reinterpret_cast<const float*>(x) + m * ld + c);
    load_chunk<float>(v + 4, reinterpret_cast<const float*>(x) + m * ld + c + 4);
  }
  auto put = [&](T* dst, const float* w) {
    if (sizeof(T) == 2) {
      store_chunk<__bf16>(reinterpret_cast<__bf16*>(dst) + m * ld + c, w);
    } else {
      store_chunk<float>(reinterpret_cast<float*>(dst) + m * ld + c, w);
      store_chunk<float>(reinterpret_cast<float*>(dst) + m * ld + c + 4, w + 4);
    }
  };
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = keep ? v[j] : 0.f;
  if (!TWO && out2) put(out2, v);   // the single-mask form's out_masked
  const uint64_t base = (uint64_t)(m * drop_ld + c);
  if (p > 0.f) {
    const uint32_t s1 = seed32(eff_seed(salt, seed_base));
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      float a, b;
      drop_mul2(p, s1, base + j, a, b);
      v[j] = to_f(from_f<T>(v[j] * a));
      v[j + 1] = to_f(from_f<T>(v[j + 1] * b));
    }
  }
  put(out, v);
  if (TWO) {
    if (p > 0.f) {
      const uint32_t s2 = seed32(eff_seed(salt2, seed_base));
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        float a, b;
        drop_mul2(p, s2, base + j, a, b);
        v[j] *= a;
        v[j + 1] *= b;
      }
    }
    put(out2, v);
  }
}

extern "C" {

int rs_adam_prepare(double* state, const double* hyper, const float* grad_divisor, uint64_t* seed_base,
                    void* stream) {
  hipLaunchKernelGGL(adam_prepare_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, state, hyper, grad_divisor,
                     seed_base);
  return (int)hipGetLastError();
}

// two float4 groups in flight per thread (1 and 4 measured slower)
// nontemporal sweeps only for ranges far beyond the 256 MB Infinity Cache (cfg5's 256M-element out.weight and token
// table: 1,535 -> 1,460-1,472 us per sweep alone, cfg5 7.03-7.11k -> 7.26-7.28k seq/s); below that the next step's
// optimizer re-reads the masters / moments from that cache (cfg4's item table with nt hints: 636-639k -> 604-608k)
#define ADAM_NT_MIN (64ll << 20)
#define ADAM_LAUNCH(BO, PR, ...)                                                                         \
  do {                                                                                                   \
    if (rm.marks) {                                                                                      \
      if (n >= ADAM_NT_MIN) hipLaunchKernelGGL((adam_step_kernel<BO, PR, 2, true, true>), __VA_ARGS__, rm);  \
      else hipLaunchKernelGGL((adam_step_kernel<BO, PR, 2, false, true>), __VA_ARGS__, rm);                \
    } else {                                                                                             \
      if (n >= ADAM_NT_MIN) hipLaunchKernelGGL((adam_step_kernel<BO, PR, 2, true, false>), __VA_ARGS__, rm); \
      else hipLaunchKernelGGL((adam_step_kernel<BO, PR, 2, false, false>), __VA_ARGS__, rm);               \
    }                                                                                                    \
  } while (0)

// row_marks layout: mrows stamps, padding to 16 B + 16 (the scalar loads' overrun), then 1 KB of zeros
#define ROW_MARKS_ZEROS(rows) ((((rows) + 15) / 16) * 16 + 16)
// the marked table's rows inside launch elements [0, n): row r of the table is launch element moff + r << dshift.
// A wave's mark test reads ONE 16-byte scalar window from its first active lane's row rounded down to 8: that
// covers the wave's 256 elements only while they span <= 9 rows, i.e. rows of >= 32 elements (dshift >= 5)
#define ROW_MARKS_MIN_DSHIFT 5
static int row_marks(int64_t n, const uint8_t* marks, const uint8_t* epoch, int64_t moff, int64_t mrows, int dshift,
                     RowMarks& rm) {
  rm = RowMarks{nullptr, nullptr, nullptr, 0, 0, 0, 0};
  if (!marks) return 0;
  if (!epoch || mrows <= 0 || dshift < ROW_MARKS_MIN_DSHIFT || dshift > 16 || moff % 4 || (uintptr_t)marks % 16) return RS_ERR_ARG;
  rm.marks = marks; rm.epoch = epoch; rm.moff = moff; rm.dshift = dshift;
  rm.zeros = reinterpret_cast<const float*>(marks + ROW_MARKS_ZEROS(mrows));
  rm.mlo = std::max<int64_t>(0, moff);
  rm.mhi = std::min<int64_t>(n, moff + (mrows << dshift));
  if (rm.mhi <= rm.mlo) rm.marks = nullptr;   // no overlap: the plain sweep
  return 0;
}

int rs_adam_step(int64_t n, float* p, float* g, float* m, float* v, void* p_bf16, const double* state,
                 const double* hyper, int zero_grad, void* stream) {
  return rs_adam_step_wg(n, p, g, m, v, p_bf16, state, hyper, zero_grad, 8192, stream);
}

int rs_adam_step_wg(int64_t n, float* p, float* g, float* m, float* v, void* p_bf16, const double* state,
                    const double* hyper, int zero_grad, int max_wg, void* stream) {
  return rs_adam_step_marked(n, p, g, m, v, p_bf16, state, hyper, zero_grad, max_wg, nullptr, nullptr, 0, 0, 0,
                             stream);
}

int rs_adam_step_marked(int64_t n, float* p, float* g, float* m, float* v, void* p_bf16, const double* state,
                        const double* hyper, int zero_grad, int max_wg, const uint8_t* row_marks_, const uint8_t* epoch,
                        int64_t moff, int64_t mrows, int dshift, void* stream) {
  if (n <= 0 || max_wg <= 0 || ((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16) return RS_ERR_ARG;
  RowMarks rm;
  if (int e = row_marks(n, row_marks_, epoch, moff, mrows, dshift, rm)) return e;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(cdiv(n / 4, 256), max_wg));
  hipStream_t s = (hipStream_t)stream;
  double* st = const_cast<double*>(state);   // read only without PREP
  if (p_bf16)
    ADAM_LAUNCH(true, false, dim3((unsigned)blocks), dim3(256), 0, s, n, p, g, m, v,
                       (__bf16*)p_bf16, st, hyper, zero_grad, nullptr, nullptr, nullptr, 0, 0,
                       nullptr, nullptr, nullptr);
  else
    ADAM_LAUNCH(false, false, dim3((unsigned)blocks), dim3(256), 0, s, n, p, g, m, v,
                       (__bf16*)nullptr, st, hyper, zero_grad, nullptr, nullptr, nullptr, 0, 0,
                       nullptr, nullptr, nullptr);
  return (int)hipGetLastError();
}

int rs_adam_prepare_step(int64_t n, float* p, float* g, float* m, float* v, void* p_bf16, double* state,
                         const double* hyper, int zero_grad, const float* grad_divisor, uint64_t* seed_base,
                         const int64_t* tdesc, int ntd, int64_t tbase, void* wT, void* stream) {
  return rs_adam_prepare_step_loss(n, p, g, m, v, p_bf16, state, hyper, zero_grad, grad_divisor, seed_base, tdesc, ntd,
                                   tbase, wT, nullptr, nullptr, stream);
}

int rs_adam_prepare_step_loss(int64_t n, float* p, float* g, float* m, float* v, void* p_bf16, double* state,
                              const double* hyper, int zero_grad, const float* grad_divisor, uint64_t* seed_base,
                              const int64_t* tdesc, int ntd, int64_t tbase, void* wT, const float* loss_sum,
                              float* loss_out, void* stream) {
  return rs_adam_prepare_step_marked(n, p, g, m, v, p_bf16, state, hyper, zero_grad, grad_divisor, seed_base, tdesc,
                                     ntd, tbase, wT, loss_sum, loss_out, nullptr, nullptr, 0, 0, 0, stream);
}

int rs_adam_prepare_step_marked(int64_t n, float* p, float* g, float* m, float* v, void* p_bf16, double* state,
                                const double* hyper, int zero_grad, const float* grad_divisor, uint64_t* seed_base,
                                const int64_t* tdesc, int ntd, int64_t tbase, void* wT, const float* loss_sum,
                                float* loss_out, const uint8_t* row_marks_, const uint8_t* epoch, int64_t moff,
                                int64_t mrows, int dshift, void* stream) {
  if (n <= 0 || !state || ((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16) return RS_ERR_ARG;
  RowMarks rm;
  if (int e = row_marks(n, row_marks_, epoch, moff, mrows, dshift, rm)) return e;
  if (!loss_out != !loss_sum || (loss_out && !grad_divisor)) return RS_ERR_ARG;
  if (ntd < 0 || (ntd > 0 && (!tdesc || !wT || !p_bf16))) return RS_ERR_ARG;
  // at most 2048 workgroups: every workgroup pays an arrival atomic (the PREP step-count publication); 7k of
  // them cost ~13 us at 7.4M parameters (kbench: 56 -> 40 us for the launch; flat at 0.66M and 20M; the
  // cfg4 step within noise, 560k vs 567k seq/s)
#ifndef ADAM_PREP_MAX_WG
#define ADAM_PREP_MAX_WG 2048
#endif
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(cdiv(n / 4, 256), ADAM_PREP_MAX_WG));
  hipStream_t s = (hipStream_t)stream;
  if (p_bf16)
    ADAM_LAUNCH(true, true, dim3((unsigned)blocks), dim3(256), 0, s, n, p, g, m, v,
                       (__bf16*)p_bf16, state, hyper, zero_grad, grad_divisor, seed_base, tdesc, ntd,
                       tbase, (__bf16*)wT, loss_sum, loss_out);
  else
    ADAM_LAUNCH(false, true, dim3((unsigned)blocks), dim3(256), 0, s, n, p, g, m, v,
                       (__bf16*)nullptr, state, hyper, zero_grad, grad_divisor, seed_base, nullptr, 0,
                       0, nullptr, loss_sum, loss_out);
  return (int)hipGetLastError();
}

int rs_cast_bf16(int64_t n, const float* src, void* dst, void* stream) {
  if (n <= 0) return RS_ERR_ARG;
  const int64_t blocks = std::min<int64_t>(cdiv(n, 256), 8192);
  hipLaunchKernelGGL(cast_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n, src,
                     (__bf16*)dst);
  return (int)hipGetLastError();
}

int rs_colsum(int dtype, const void* X, int64_t M, int64_t N, int64_t ldx, float* ws, float* out, int accumulate,
              void* stream) {
  if (M <= 0 || N <= 0) return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int nblk = (int)std::min<int64_t>(COLSUM_BLOCKS, cdiv(M, 64));
  hipError_t e = dtype == RS_DTYPE_BF16 ? colsum_partial<__bf16>((const __bf16*)X, M, N, ldx, ws, nblk, s)
                                        : colsum_partial<float>((const float*)X, M, N, ldx, ws, nblk, s);
  if (e != hipSuccess) return (int)e;
  return (int)launch_reduce_slabs(ws, nblk, N, N, out, nullptr, accumulate, s);
}

int rs_dropout_rowmask(int dtype, const void* x, int64_t M, int64_t N, int64_t ld, float drop_p, uint64_t seed,
                       const uint64_t* seed_base, int64_t drop_ld, const int64_t* rowmask_ids, void* out,
                       void* out_masked, void* stream) {
  if (M <= 0 || N <= 0) return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int es = dtype == RS_DTYPE_BF16 ? 2 : 4;
  if (N % 8 == 0 && ld % 8 == 0 && drop_ld % 2 == 0 && ((uintptr_t)x | (uintptr_t)out | (uintptr_t)out_masked) % 16 == 0) {
    dim3 g8((unsigned)cdiv(M * (N / 8), 256));
    if (es == 2)
      hipLaunchKernelGGL((dropout_v8_kernel<__bf16, false>), g8, dim3(256), 0, s, (const __bf16*)x, M, N, ld, drop_p,
                         seed, 0ull, seed_base, drop_ld, rowmask_ids, (__bf16*)out, (__bf16*)out_masked);
    else
      hipLaunchKernelGGL((dropout_v8_kernel<float, false>), g8, dim3(256), 0, s, (const float*)x, M, N, ld, drop_p,
                         seed, 0ull, seed_base, drop_ld, rowmask_ids, (float*)out, (float*)out_masked);
    return (int)hipGetLastError();
  }
  dim3 grid((unsigned)cdiv(M * N, 256));
  if (dtype == RS_DTYPE_BF16)
    hipLaunchKernelGGL((dropout_rowmask_kernel<__bf16>), grid, dim3(256), 0, s, (const __bf16*)x, M, N, ld, drop_p,
                       seed, seed_base, drop_ld, rowmask_ids, (__bf16*)out, (__bf16*)out_masked);
  else
    hipLaunchKernelGGL((dropout_rowmask_kernel<float>), grid, dim3(256), 0, s, (const float*)x, M, N, ld, drop_p,
                       seed, seed_base, drop_ld, rowmask_ids, (float*)out, (float*)out_masked);
  return (int)hipGetLastError();
}

int rs_dropout2(int dtype, const void* x, int64_t M, int64_t N, int64_t ld, float drop_p, uint64_t salt1,
                uint64_t salt2, const uint64_t* seed_base, int64_t drop_ld, void* out1, void* out2, void* stream) {
  if (M <= 0 || N <= 0 || N % 8 || ld % 8 || drop_ld % 2 || !x || !out1 || !out2 ||
      ((uintptr_t)x | (uintptr_t)out1 | (uintptr_t)out2) % 16)
    return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  dim3 g8((unsigned)cdiv(M * (N / 8), 256));
  if (dtype == RS_DTYPE_BF16)
    hipLaunchKernelGGL((dropout_v8_kernel<__bf16, true>), g8, dim3(256), 0, s, (const __bf16*)x, M, N, ld, drop_p,
                       salt1, salt2, seed_base, drop_ld, (const int64_t*)nullptr, (__bf16*)out1, (__bf16*)out2);
  else
    hipLaunchKernelGGL((dropout_v8_kernel<float, true>), g8, dim3(256), 0, s, (const float*)x, M, N, ld, drop_p,
                       salt1, salt2, seed_base, drop_ld, (const int64_t*)nullptr, (float*)out1, (float*)out2);
  return (int)hipGetLastError();
}

__global__ void seed_advance_kernel(uint64_t* s) {
  if (threadIdx.x == 0) *s += 1;
}

int rs_graph_upload(void* graph_exec, void* stream) {
  if (!graph_exec) return RS_ERR_ARG;
  return (int)hipGraphUpload((hipGraphExec_t)graph_exec, (hipStream_t)stream);
}

int rs_seed_advance(uint64_t* seed_base, void* stream) {
  hipLaunchKernelGGL(seed_advance_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, seed_base);
  return (int)hipGetLastError();
}

// ---- kernel stamps (see common.h) ------------------------------------------------------------
static unsigned long long* g_kstamp_buf = nullptr;
static const double* g_kstamp_step = nullptr;
static int g_kstamp_next = 0, g_kstamp_mask = 0;
static int g_kstamp_kind[256];

}  // extern "C"

KStamp kstamp_next(int kind) {
  KStamp k{nullptr, nullptr, 0};
  if (g_kstamp_buf && (g_kstamp_mask >> kind & 1)) {
    k.buf = g_kstamp_buf;
    k.step = g_kstamp_step;
    if (g_kstamp_next < 256) g_kstamp_kind[g_kstamp_next] = kind;
    k.mark = g_kstamp_next++;
  }
  return k;
}

extern "C" {

int rs_kernel_stamps(uint64_t* buf, const double* step, int kind_mask) {
  if ((buf == nullptr) != (step == nullptr)) return RS_ERR_ARG;
  g_kstamp_buf = (unsigned long long*)buf;
  g_kstamp_step = step;
  g_kstamp_mask = kind_mask;
  if (buf) g_kstamp_next = 0;      // disabling keeps the launch log of the last enabled period
  return 0;
}

int rs_kernel_stamp_kinds(int* kinds, int n) {
  const int m = g_kstamp_next < 256 ? g_kstamp_next : 256;
  for (int i = 0; i < n && i < m; ++i) kinds[i] = g_kstamp_kind[i];
  return 0;
}

int rs_kernel_stamp_count(void) { return g_kstamp_next; }

int rs_wall_clock_khz(int* khz) {
  if (!khz) return RS_ERR_ARG;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  return (int)hipDeviceGetAttribute(khz, hipDeviceAttributeWallClockRate, dev);
}

int rs_abi_version(void) { return 1; }

}  // extern "C"
