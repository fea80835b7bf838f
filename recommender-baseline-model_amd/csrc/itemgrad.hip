// rs-build: included by grad_tail.hip (compiled once, as part of that translation unit)
// Item-embedding gradient by inverted index (deterministic, no float atomics).
//
// The item table receives, per training step, one gradient row per token of the input sequence
// (the embedding lookup, sas.py:59-66: scale * dropout-mask * dx[m]) and one per positive and
// negative logit (sas.py:91-98: dpl[m] * f[m], dnl[m] * f[m]), keyed by the item id -- Zipf
// distributed, so a handful of ids own thousands of rows.  Float atomics into the table run at
// the memory-side atomic rate and serialise on the hot rows.  Instead:
//
//   rs_item_index_build: keys (ids | pos | neg) -> stable counting sort of the entries by key:
//                        per-512-entry-block key histograms (LDS), per-key exclusive prefix over
//                        blocks, a two-level scan over keys (group sums of 64 keys, one workgroup
//                        scanning the groups, a wave scan per group), then each block places its
//                        entries by a bitonic sort of (key, index) words in LDS for the in-block
//                        rank -- all hand-written -- for tables whose per-block histograms fit LDS
//                        (<= 32k rows: cfg2, cfg3).  Larger tables (cfg4's 54.5k items, cfg5's 1M tokens)
//                        take a hand-written LSD radix sort instead (the counting sort's nb x V global
//                        histogram was 33-100 MB of traffic beside the forward): per pass of <= 8 key
//                        bits, a count launch (per-tile digit histograms) and a scatter launch (stable
//                        per-wave ranks from 8 ballots, wave x digit counters, each tile's digit offsets
//                        scanned by the tile itself).  The workgroups are thin on purpose: a one-CU
//                        LDS-resident sort (tried) held a CU for 42-51 us, and every forward kernel runs
//                        one workgroup per CU, so its last workgroup waited behind it (+9 us per step
//                        at cfg4); these co-reside with the forward's workgroups instead.  No per-key start table (a 1M-row table's
//                        4 MB of it was a launch of its own): the gradient kernels find a key run's
//                        extent from the neighbouring sorted keys
//   rs_item_grad:        chunks of 64 sorted entries: contribution rows summed per key run in
//                        LDS; a key wholly inside one chunk is written by that chunk (+=); a
//                        key spanning chunks leaves per-chunk partials that the chunk holding
//                        its first entry sums in chunk order (second kernel).
//
// Every destination row has exactly one writer and a fixed summation order: bitwise
// reproducible.  Rows with key 0 (padding_idx) are skipped.
#include "common.h"
#include "../../include/recsys_hip.h"

namespace ig {

#ifndef IG_CH
#define IG_CH 32   // A/B against 64: cfg2 0.2962 vs 0.2991, cfg4 0.2258 vs 0.2322 ms/step (more, shorter chunk workgroups beside the weight-gradient tiles); 128 slower
#endif
constexpr int CH = IG_CH;       // sorted entries per gradient chunk
constexpr int BE = 512;         // entries per counting-sort block (512: 150 blocks at cfg2, 1024 took 75)
#ifndef IG_COUNT_VMAX
#define IG_COUNT_VMAX 32768
#endif
constexpr int VMAX_LDS = IG_COUNT_VMAX;     // largest table for the counting sort's LDS histogram
constexpr int64_t HMAX = (int64_t)1 << 26;  // largest per-block histogram table (ints) for the counting sort
constexpr int IBITS = 9;                    // BE = 2^IBITS: an entry's block index in the sort word's low bits
constexpr int KBITS_MAX = 32 - IBITS - 1;   // key bits the counting-sort path's (key, index) sort word holds
static_assert(BE == 1 << IBITS, "sort word layout");
// LSD radix sort (tables past the counting sort's limits): thin workgroups that co-reside with the forward's
// one-workgroup-per-CU kernels (~20 VGPRs of words, 5 KB LDS), so the side-queue sort takes no CU from them
constexpr int RT = 256;                    // threads of a sort workgroup
constexpr int RW = RT / 64;                // its waves
constexpr int RB = 8;                      // widest digit (bits): one digit per thread in the scans
constexpr int NBIN = 1 << RB;
constexpr int CPAD = NBIN + 1;             // per-wave counter row pitch: rows start on different banks
constexpr int ITB = 8;                     // words per thread of a tile
constexpr int TB = RT * ITB;               // entries per tile (2,048: cfg4's 19,200 entries are 10 tiles)
constexpr int64_t FUSED_SCAN_TILES = 64;   // up to this many tiles each scatter workgroup scans the counts itself
static_assert(NBIN == RT, "one thread per digit");
enum SortPath { SORT_COUNT = 0, SORT_TILES = 3 };

struct Layout {
  int64_t n, nchunks, nb, V;
  int path, kb;              // SortPath; key bits
  bool cs;
  size_t sk, sv, start, part, H, total, ping, pong, hist, temp, temp_bytes, total_bytes;
};

static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

static int key_bits(int64_t table_rows) {
  int b = 1;
  while (b < 32 && ((int64_t)1 << b) < table_rows) ++b;
  return b;
}

static hipError_t layout(int nsrc, int64_t rows, int64_t table_rows, int64_t d, Layout& L) {
  L.n = nsrc * rows;
  L.nchunks = cdiv(L.n, CH);
  L.nb = cdiv(L.n, BE);
  L.V = table_rows;
  // counting sort only where the per-block histograms live in LDS; a larger table's nb x V global histogram
  // (cfg4: 150 x 54.5k ints = 33 MB zeroed, scanned and re-read; cfg5: 100 MB) ran beside the forward and slowed
  // it more than the sort costs: cfg4 0.2226 -> 0.2148 ms/step, cfg5 12.20 -> 12.09 with the radix sort
  L.cs = table_rows <= VMAX_LDS && L.nb * table_rows <= HMAX && key_bits(table_rows) <= KBITS_MAX;
  L.kb = key_bits(table_rows);
  L.path = L.cs ? SORT_COUNT : SORT_TILES;
  size_t o = 0;
  L.sk = o; o = al256(o + L.n * 4);
  L.sv = o; o = al256(o + L.n * 4);
  L.start = 0;
  if (L.cs) { L.start = o; o = al256(o + (table_rows + 1) * 4); }   // the counting sort's placement offsets
  L.part = o; o = al256(o + L.nchunks * 2 * d * 4);
  L.temp_bytes = 0;
  L.H = L.total = L.ping = L.pong = L.hist = L.temp = 0;
  if (L.cs) {
    L.H = o; o = al256(o + L.nb * table_rows * 4);
    L.total = o; o = al256(o + (table_rows + 1) * 4);   // [V] = 0: the scan's last entry is the total
    L.temp = o;                                          // group sums of the key scan: cdiv(V, 64) + 1 ints
    L.temp_bytes = (size_t)(cdiv(table_rows, 64) + 1) * 4;
    o = al256(o + L.temp_bytes);
  } else if (L.path == SORT_TILES) {                     // word ping-pong + per-(digit, tile) counts
    L.ping = o; o = al256(o + L.n * 8);
    L.pong = o; o = al256(o + L.n * 8);
    L.hist = o; o = al256(o + (size_t)NBIN * cdiv(L.n, TB) * 4);
  }
  L.total_bytes = o;
  return hipSuccess;
}

struct Keys {
  const int64_t* k[3];
  int64_t rows, n, V;
  __device__ __forceinline__ const int64_t* addr(int64_t e) const {   // source by comparison: no 64-bit division
    const int src = (e >= rows) + (e >= 2 * rows);
    return k[src] + (e - src * rows);
  }
  __device__ __forceinline__ uint32_t key_of(int64_t v) const { return (v < 0 || v >= V) ? 0u : (uint32_t)v; }
  __device__ __forceinline__ uint32_t get(int64_t e) const { return key_of(*addr(e)); }
};

// ---- counting sort ------------------------------------------------------------------------
// H[b][v] = number of entries of block b with key v
// LDS sized to the table (dynamic, V ints): a 3.4k-row table takes 14 KB, so the block fits beside the
// forward's kernels on the side queue (a static 128 KB array needed an idle CU and started late)
__global__ __launch_bounds__(256) void hist_kernel(Keys K, int* __restrict__ H) {
  extern __shared__ int hist[];
  const int tid = threadIdx.x;
  const int V = (int)K.V;
  for (int v = tid; v < V; v += 256) hist[v] = 0;
  __syncthreads();
  const int64_t e0 = (int64_t)blockIdx.x * BE;
  uint32_t key[BE / 256];
#pragma unroll
  for (int i = 0; i < BE / 256; ++i) {
    const int64_t e = e0 + tid + i * 256;
    key[i] = e < K.n ? K.get(e) : 0xffffffffu;
  }
#pragma unroll
  for (int i = 0; i < BE / 256; ++i)
    if (key[i] != 0xffffffffu) atomicAdd(&hist[key[i]], 1);
  __syncthreads();
  int* h = H + (int64_t)blockIdx.x * V;
  for (int v = tid; v < V; v += 256) h[v] = hist[v];
}

// H[b][v] <- sum_{b' < b} H[b'][v];  total[v] = sum_b H[b][v].  Workgroup = 64 keys (lanes) x 4
// waves, wave w owning a contiguous quarter of the block range; quarters combined through LDS.
__global__ __launch_bounds__(256) void prefix_blocks_kernel(int* __restrict__ H, int64_t nb, int64_t V,
                                                            int* __restrict__ total, int* __restrict__ gsum) {
  __shared__ int part[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t v = (int64_t)blockIdx.x * 64 + lane;
  if (blockIdx.x == 0 && threadIdx.x == 0) total[V] = 0;
  const int64_t q = cdiv(nb, 4), b0 = w * q, b1 = min(nb, b0 + q);
  constexpr int U = 8;
  int h[U];
  int acc = 0;
  if (v < V) {
    for (int64_t b = b0; b < b1; b += U) {
#pragma unroll
      for (int u = 0; u < U; ++u) h[u] = b + u < b1 ? H[(b + u) * V + v] : 0;
#pragma unroll
      for (int u = 0; u < U; ++u) acc += h[u];
    }
  }
  part[w][lane] = acc;
  __syncthreads();
  int off = 0;
  for (int x = 0; x < w; ++x) off += part[x][lane];
  if (w == 3) {   // this group of 64 keys: per-key totals and their sum (the key scan's group sums)
    int t = v < V ? off + acc : 0;
    if (v < V) total[v] = t;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    if (lane == 0) gsum[blockIdx.x] = t;
  }
  if (v >= V) return;
  for (int64_t b = b0; b < b1; b += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) h[u] = b + u < b1 ? H[(b + u) * V + v] : 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (b + u < b1) H[(b + u) * V + v] = off;
      off += h[u];
    }
  }
}

// exclusive scan of the group sums in place (G groups of 64 keys; gsum[G] = the grand total): one workgroup,
// each thread a contiguous run of groups
__global__ __launch_bounds__(1024) void scan_groups_kernel(int* __restrict__ gsum, int64_t G) {
  __shared__ int ts[1024];
  const int tid = threadIdx.x;
  const int64_t per = cdiv(G, 1024), g0 = tid * per, g1 = min(G, g0 + per);
  int s = 0;
  for (int64_t g = g0; g < g1; ++g) s += gsum[g];
  ts[tid] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {     // inclusive Hillis-Steele scan of the thread sums
    const int x = tid >= o ? ts[tid - o] : 0;
    __syncthreads();
    ts[tid] += x;
    __syncthreads();
  }
  int off = ts[tid] - s;
  for (int64_t g = g0; g < g1; ++g) {
    const int x = gsum[g];
    gsum[g] = off;
    off += x;
  }
  if (tid == 1023) gsum[G] = ts[1023];
}

// start[v] = sum_{v' < v} total[v'] for v <= V: one wave per group of 64 keys, the group's offset plus an
// exclusive wave scan of its totals (total[V] = 0, so start[V] is the grand total)
__global__ __launch_bounds__(256) void start_kernel(const int* __restrict__ total, const int* __restrict__ gsum,
                                                    int64_t V, int* __restrict__ start) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), v = g * 64 + lane;
  if (g * 64 > V) return;
  const int t = v < V ? total[v] : 0;
  int x = t;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (v <= V) start[v] = gsum[g] + x - t;
}

// each block places its entries: the stable rank inside the block comes from a bitonic sort of the block's
// (key << IBITS | index) words (keys <= KBITS_MAX bits; unused slots sort last).  Thread t holds elements 2t, 2t+1:
// partners 1 apart swap in registers, 2..64 apart across lanes of one wave (shuffles), only the stages 128 and 256
// apart (3 of the 45) go through LDS with a barrier.
__device__ __forceinline__ void bsort_cas(uint32_t& x, uint32_t y, bool lower, bool asc) {
  // keep min when (this is the lower element) == (ascending), else max
  const uint32_t lo = x < y ? x : y, hi = x < y ? y : x;
  x = lower == asc ? lo : hi;
}
__global__ __launch_bounds__(256) void place_kernel(Keys K, const int* __restrict__ H, const int* __restrict__ start,
                                                    uint32_t* __restrict__ sk, uint32_t* __restrict__ sv) {
  __shared__ uint32_t w[BE];
  const int tid = threadIdx.x;
  const int64_t e0 = (int64_t)blockIdx.x * BE;
  const int cnt = (int)min((int64_t)BE, K.n - e0);
  uint32_t v[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int l = 2 * tid + i;
    v[i] = l < cnt ? (K.get(e0 + l) << IBITS | (uint32_t)l) : 0xffffffffu;
  }
  for (int k = 2; k <= BE; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j == 1) {
        const bool asc = ((2 * tid) & k) == 0;
        const uint32_t a = v[0], b = v[1];
        v[0] = asc ? (a < b ? a : b) : (a < b ? b : a);
        v[1] = asc ? (a < b ? b : a) : (a < b ? a : b);
      } else if (j <= 64) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int e = 2 * tid + i;
          const uint32_t y = (uint32_t)__shfl_xor((int)v[i], j >> 1, 64);
          bsort_cas(v[i], y, (e & j) == 0, (e & k) == 0);
        }
      } else {
        __syncthreads();   // the previous cross-wave stage's reads are done
        w[2 * tid] = v[0];
        w[2 * tid + 1] = v[1];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int e = 2 * tid + i;
          bsort_cas(v[i], w[e ^ j], (e & j) == 0, (e & k) == 0);
        }
      }
    }
  }
  __syncthreads();
  w[2 * tid] = v[0];
  w[2 * tid + 1] = v[1];
  __syncthreads();
  const int* h = H + (int64_t)blockIdx.x * K.V;
  for (int j = tid; j < cnt; j += 256) {
    const uint32_t x = w[j], k = x >> IBITS;
    int lo = 0, hi = j;                       // first position of key k in the sorted block
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if ((w[mid] >> IBITS) < k) lo = mid + 1;
      else hi = mid;
    }
    const int64_t pos = (int64_t)start[k] + h[k] + (j - lo);
    sk[pos] = k;
    sv[pos] = (uint32_t)(e0 + (x & (BE - 1)));
  }
}

// ---- hand-written LSD radix sort (tables past the counting sort's limits) ----------------------

// Stable rank of this lane's element among the elements of its wave with the same digit: the lanes below it
// holding that digit (peers from db ballots) plus the wave's running count row[dig] in LDS, which the highest
// such lane advances.  A wave's LDS accesses complete in order, so the read-then-write needs no fence; the
// calls must be made with every lane of the wave active.
__device__ __forceinline__ int wave_rank(uint32_t dig, bool valid, int db, int* row, int lane) {
  uint64_t m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < RB; ++b) {
    if (b < db) {
      const bool bit = (dig >> b) & 1u;
      const uint64_t x = __ballot(bit);
      m &= bit ? x : ~x;
    }
  }
  int r = 0;
  if (valid) {
    const int base = row[dig];
    r = base + __popcll(m & ((1ull << lane) - 1ull));
    if ((m >> lane) == 1ull) row[dig] = base + __popcll(m);
  }
  return r;
}

// digit width of an LSD sort over kb key bits: the fewest passes of <= RB bits, split evenly
__host__ __device__ inline int sort_passes(int kb) { return (kb + RB - 1) / RB; }
__host__ __device__ inline int sort_digit(int kb) { return (kb + sort_passes(kb) - 1) / sort_passes(kb); }

// Words key << 32 | entry; a pass reads its input in tiles of TB entries, wave w of a tile holding entries
// [w*ITB*64, (w+1)*ITB*64) lane-fastest, so (digit, tile, wave, iteration, lane) order is the input order within
// each digit: stable.  in == null: the first pass reads the keys.
__device__ __forceinline__ bool tile_load(const Keys& K, const uint64_t* in, int64_t tile, uint64_t (&word)[ITB]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t e0 = tile * TB + w * (ITB * 64) + lane;
  if (in) {
#pragma unroll
    for (int i = 0; i < ITB; ++i) word[i] = e0 + i * 64 < K.n ? in[e0 + i * 64] : 0ull;
  } else {
    int64_t raw[ITB];
#pragma unroll
    for (int i = 0; i < ITB; ++i) raw[i] = e0 + i * 64 < K.n ? *K.addr(e0 + i * 64) : 0;
#pragma unroll
    for (int i = 0; i < ITB; ++i) word[i] = (uint64_t)K.key_of(raw[i]) << 32 | (uint64_t)(e0 + i * 64);
  }
  return true;
}

// per-(digit, tile) counts of pass (shift, db): hist[d * tiles + tile]
__global__ __launch_bounds__(RT) void rsort_count_kernel(Keys K, const uint64_t* __restrict__ in, int shift, int db,
                                                         int* __restrict__ hist) {
  __shared__ int h[NBIN];
  const int tid = threadIdx.x;
  h[tid] = 0;
  uint64_t word[ITB];
  tile_load(K, in, blockIdx.x, word);
  __syncthreads();
  const int lane = tid & 63, w = tid >> 6;
  const uint32_t dmask = (1u << db) - 1u;
#pragma unroll
  for (int i = 0; i < ITB; ++i)
    if ((int64_t)blockIdx.x * TB + w * (ITB * 64) + i * 64 + lane < K.n)
      atomicAdd(&h[(uint32_t)(word[i] >> (32 + shift)) & dmask], 1);   // integer counts: order-free
  __syncthreads();
  if (tid < (1 << db)) hist[(int64_t)tid * gridDim.x + blockIdx.x] = h[tid];
}

// exclusive scan of hist[0..m) in place (tile counts past FUSED_SCAN_TILES), one workgroup
__global__ __launch_bounds__(RT) void rsort_scan_kernel(int* __restrict__ hist, int64_t m) {
  __shared__ int ts[RT];
  const int tid = threadIdx.x;
  const int64_t per = cdiv(m, RT), g0 = tid * per, g1 = min(m, g0 + per);
  int s = 0;
  for (int64_t g = g0; g < g1; ++g) s += hist[g];
  ts[tid] = s;
  __syncthreads();
  for (int o = 1; o < RT; o <<= 1) {
    const int x = tid >= o ? ts[tid - o] : 0;
    __syncthreads();
    ts[tid] += x;
    __syncthreads();
  }
  int off = ts[tid] - s;
  for (int64_t g = g0; g < g1; ++g) {
    const int x = hist[g];
    hist[g] = off;
    off += x;
  }
}

// one pass: rank the tile stably, place every word at (offset of its digit before this tile) + (waves before
// it) + rank.  scanned == 0: the workgroup forms its digits' offsets from the raw counts itself (thread d sums
// digit d over the tiles, then an exclusive scan over digits); else hist already holds them.  out == null:
// the last pass, writing the sorted keys / entries.
__global__ __launch_bounds__(RT) void rsort_scatter_kernel(Keys K, const uint64_t* __restrict__ in, int shift, int db,
                                                           const int* __restrict__ hist, int scanned,
                                                           uint64_t* __restrict__ out, uint32_t* __restrict__ sk,
                                                           uint32_t* __restrict__ sv) {
  __shared__ int cnt[RW * CPAD];
  __shared__ int wsum[RW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nb = 1 << db;
  const int64_t tiles = gridDim.x, tile = blockIdx.x;
  // this tile's global digit offsets (thread = digit), issued ahead of the ranking
  int tot = 0, before = 0;
  if (tid < nb) {
    if (scanned) {
      before = hist[(int64_t)tid * tiles + tile];
    } else {
      for (int64_t t = 0; t < tiles; ++t) {
        const int x = hist[(int64_t)tid * tiles + t];
        tot += x;
        before += t < tile ? x : 0;
      }
    }
  }
  uint64_t word[ITB];
  tile_load(K, in, tile, word);
  for (int j = tid; j < RW * CPAD; j += RT) cnt[j] = 0;
  __syncthreads();
  int* row = cnt + w * CPAD;
  const uint32_t dmask = (1u << db) - 1u;
  int rk[ITB];
#pragma unroll
  for (int i = 0; i < ITB; ++i) {
    const bool valid = tile * TB + w * (ITB * 64) + i * 64 + lane < K.n;
    rk[i] = wave_rank((uint32_t)(word[i] >> (32 + shift)) & dmask, valid, db, row, lane);
  }
  if (!scanned) {   // exclusive scan of the digit totals over digits (wave scan + wave sums)
    int x = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int off = x - tot;
    for (int k = 0; k < w; ++k) off += wsum[k];
    before += off;
  } else {
    __syncthreads();
  }
  if (tid < nb) {   // + the waves before, per digit
    int run = before;
#pragma unroll
    for (int ww = 0; ww < RW; ++ww) {
      const int t = cnt[ww * CPAD + tid];
      cnt[ww * CPAD + tid] = run;
      run += t;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < ITB; ++i) {
    const int64_t e = tile * TB + w * (ITB * 64) + i * 64 + lane;
    if (e >= K.n) continue;
    const int pos = row[(uint32_t)(word[i] >> (32 + shift)) & dmask] + rk[i];
    if (out) {
      out[pos] = word[i];
    } else {
      sk[pos] = (uint32_t)(word[i] >> 32);
      sv[pos] = (uint32_t)word[i];
    }
  }
}

// ---- gradient ---------------------------------------------------------------------------------
struct GradArgs {
  const uint32_t* sk;
  const uint32_t* sv;
  float* part;
  int64_t n, rows;
  const __bf16* dx;      // source 0 rows: scale * drop(m*d + c) * dx[m]
  float scale, drop_p;
  uint64_t salt;
  const uint64_t* seed_base;
  const __bf16* f;       // sources 1, 2 rows: w1[m] * f[m], w2[m] * f[m]
  const float* w1;
  const float* w2;
  float* dtable;
  const int* start;      // counting-sort path: start[v] = first sorted position of key v (v <= V); null on the radix path
  uint8_t* marks;        // nullable: marks[v] = the step's stamp for every key v (rs_item_grad_marked)
  uint8_t* epoch;        // ... and the stamp itself
};

// one workgroup per chunk of CH sorted entries.  Dependent global round trips: (keys, entries) ->
// (contribution rows, key bounds, the table rows of run heads) -> stores.
template <int D>
struct ChunkLds {
  float rowsum[CH][D + 4];   // +4: rows start on different banks
  uint32_t skey[CH + 1], sent[CH];
  uint32_t prevk, nextk;     // the sorted keys just before and just after the chunk (or a sentinel)
};

// chunk `chunk` of the sorted entries (one 256-thread workgroup), LDS at `L`
template <int D>
__device__ __forceinline__ void item_chunk(const GradArgs& a, int64_t chunk, ChunkLds<D>& L) {
  constexpr int TPE = D / 8, EPP = 256 / TPE, NPASS = CH / EPP;   // threads per entry row, rows per pass
  auto& rowsum = L.rowsum;
  auto& skey = L.skey;
  auto& sent = L.sent;
  const int tid = threadIdx.x;
  const int64_t base = chunk * CH;
  const int cnt = (int)min((int64_t)CH, a.n - base);
  const bool drop = a.drop_p > 0.f;
  const uint32_t s32 = drop ? seed32(eff_seed(a.salt, a.seed_base)) : 0u;
  const uint8_t stamp = a.marks && a.seed_base ? (uint8_t)*a.seed_base : 0;
  if (a.marks && tid < cnt) {
    const uint32_t k = a.sk[base + tid];
    if (k != 0) a.marks[k] = stamp;
  }
  if (a.marks && chunk == 0 && tid == 0) *a.epoch = stamp;
  if (tid < CH) {
    skey[tid + 1] = tid < cnt ? a.sk[base + tid] : 0xffffffffu;
    sent[tid] = tid < cnt ? a.sv[base + tid] : 0u;
  }
  if (tid == 0) skey[0] = 0xfffffffeu;   // sentinel: entry 0 always starts a run
  if (tid == CH) L.prevk = base > 0 ? a.sk[base - 1] : 0xfffffffeu;
  if (tid == CH + 1) L.nextk = base + cnt < a.n ? a.sk[base + cnt] : 0xfffffffeu;
  __syncthreads();
  // contribution rows + the current table rows of run heads (prefetched for the emit pass)
  float4 tab[NPASS][2];
#pragma unroll
  for (int ps = 0; ps < NPASS; ++ps) {
    const int j = ps * EPP + tid / TPE, c0 = (tid % TPE) * 8;
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = 0.f;
    tab[ps][0] = tab[ps][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    const uint32_t key = skey[j + 1];
    if (j < cnt && key != 0) {
      const uint32_t e = sent[j];
      const int src = (int)(e / (uint32_t)a.rows);
      const int64_t m = (int64_t)e - (int64_t)src * a.rows;
      if (src == 0) {
        load_chunk<__bf16>(v, a.dx + m * D + c0);
        float dm[8];
#pragma unroll
        for (int q = 0; q < 8; q += 2) {
          if (drop) drop_mul2(a.drop_p, s32, (uint64_t)(m * D + c0 + q), dm[q], dm[q + 1]);
          else dm[q] = dm[q + 1] = 1.f;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = v[q] * a.scale * dm[q];
      } else {
        const float w = src == 1 ? a.w1[m] : a.w2[m];
        load_chunk<__bf16>(v, a.f + m * D + c0);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] *= w;
      }
      if (skey[j] != key) {
        const float4* t = reinterpret_cast<const float4*>(a.dtable + (int64_t)key * D + c0);
        tab[ps][0] = t[0];
        tab[ps][1] = t[1];
      }
    }
    *reinterpret_cast<float4*>(&rowsum[j][c0]) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(&rowsum[j][c0 + 4]) = make_float4(v[4], v[5], v[6], v[7]);
  }
  __syncthreads();
  // per-column run sums in entry order, stored at the run's first row
  if (tid < D) {
    // the column's CH values into registers first (the run-total stores below alias rowsum, so
    // loads interleaved with them would be issued one at a time)
    const int c = tid;
    float col[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) col[j] = rowsum[j][c];
    float acc = 0.f;
    int rs = 0;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      if (j < cnt) {
        acc += col[j];
        if (j + 1 == cnt || skey[j + 2] != skey[j + 1]) {
          rowsum[rs][c] = acc;
          acc = 0.f;
          rs = j + 1;
        }
      }
    }
  }
  __syncthreads();
  // emit: whole key in this chunk -> table row (sole writer); else the chunk's partial
#pragma unroll
  for (int ps = 0; ps < NPASS; ++ps) {
    const int j = ps * EPP + tid / TPE, c0 = (tid % TPE) * 8;
    const uint32_t k = skey[j + 1];
    if (j >= cnt || skey[j] == k || k == 0) continue;
    const float4 r0 = *reinterpret_cast<const float4*>(&rowsum[j][c0]);
    const float4 r1 = *reinterpret_cast<const float4*>(&rowsum[j][c0 + 4]);
    // the key's run lies wholly in this chunk: it starts here (not continued from the entry before the chunk)
    // and ends here (the chunk's last key differs, or the entry after the chunk does)
    if ((j > 0 || L.prevk != k) && (skey[cnt] != k || L.nextk != k)) {
      float4* t = reinterpret_cast<float4*>(a.dtable + (int64_t)k * D + c0);
      float4 t0 = tab[ps][0], t1 = tab[ps][1];
      t0.x += r0.x; t0.y += r0.y; t0.z += r0.z; t0.w += r0.w;
      t1.x += r1.x; t1.y += r1.y; t1.z += r1.z; t1.w += r1.w;
      t[0] = t0;
      t[1] = t1;
    } else {
      float4* o = reinterpret_cast<float4*>(a.part + (chunk * 2 + (j == 0 ? 0 : 1)) * D + c0);
      o[0] = r0;
      o[1] = r1;
    }
  }
}

template <int D>
__global__ __launch_bounds__(256) void item_chunk_kernel(GradArgs a) {
  __shared__ __attribute__((aligned(16))) ChunkLds<D> L;
  item_chunk<D>(a, blockIdx.x, L);
}

// one wave per chunk: the chunk holding the first entry of a key that continues past the chunk
// sums that key's partials in chunk order and writes the table row
template <int D>
__device__ __forceinline__ void item_span(const GradArgs& a, int64_t nchunks, int64_t blk) {
  constexpr int CPL = D / 64 > 0 ? D / 64 : 1;    // columns per lane
  const int lane = threadIdx.x & 63;
  const int64_t ch = blk * 4 + (threadIdx.x >> 6);
  if (ch >= nchunks) return;
  const int64_t base = ch * CH;
  const int64_t last = min(a.n, base + CH) - 1;
  const uint32_t k = a.sk[last];
  if (k == 0) return;
  // the key continues past this chunk, and its run starts here (not in an earlier chunk)
  if (last + 1 >= a.n || a.sk[last + 1] != k) return;
  const bool head_here = a.sk[base] != k;
  if (!head_here && base > 0 && a.sk[base - 1] == k) return;
  const int own_slot = head_here ? 1 : 0;
  float acc[CPL];
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int c = lane + 64 * q;
    acc[q] = c < D ? a.part[(ch * 2 + own_slot) * D + c] : 0.f;
  }
  if (a.start) {
    // counting-sort path: the run's last chunk is known up front, so the trip count does not depend on loaded keys
    // and every chunk's partial load is in flight at once (the head scan below waits a round trip per 8 chunks:
    // cfg2 item_span 9.7 -> 15.7 us when it replaced this)
    const int64_t cl = ((int64_t)a.start[k + 1] - 1) / CH;
    int64_t cc = ch + 1;
    for (; cc + 7 <= cl; cc += 8) {
#pragma unroll
      for (int q = 0; q < CPL; ++q) {
        const int c = lane + 64 * q;
        if (c < D) {
          float u[8];
#pragma unroll
          for (int t = 0; t < 8; ++t) u[t] = a.part[((cc + t) * 2) * D + c];
#pragma unroll
          for (int t = 0; t < 8; ++t) acc[q] += u[t];
        }
      }
    }
    for (; cc <= cl; ++cc) {
#pragma unroll
      for (int q = 0; q < CPL; ++q) {
        const int c = lane + 64 * q;
        if (c < D) acc[q] += a.part[(cc * 2) * D + c];
      }
    }
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      const int c = lane + 64 * q;
      if (c < D) a.dtable[(int64_t)k * D + c] += acc[q];
    }
    return;
  }
  // later chunks whose first entry still has key k, in chunk order; eight chunks' heads and partials in flight
  const int64_t nch = cdiv(a.n, CH);
  bool more = true;
  for (int64_t cc = ch + 1; more && cc < nch; cc += 8) {
    uint32_t f[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) f[t] = cc + t < nch ? a.sk[(cc + t) * CH] : 0xfffffffeu;
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      const int c = lane + 64 * q;
      float u[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) u[t] = (c < D && cc + t < nch) ? a.part[((cc + t) * 2) * D + c] : 0.f;
      bool run = true;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        run = run && f[t] == k;
        if (run) acc[q] += u[t];
      }
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) more = more && f[t] == k;
  }
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int c = lane + 64 * q;
    if (c < D) a.dtable[(int64_t)k * D + c] += acc[q];
  }
}

template <int D>
__global__ __launch_bounds__(256) void item_span_kernel(GradArgs a, int64_t nchunks) {
  item_span<D>(a, nchunks, blockIdx.x);
}

}  // namespace ig

extern "C" {

int64_t rs_item_index_ws_bytes(int nsrc, int64_t rows, int64_t table_rows, int64_t d) {
  if (nsrc < 1 || nsrc > 3 || rows <= 0 || table_rows <= 0 || d <= 0) return -1;
  ig::Layout L;
  if (ig::layout(nsrc, rows, table_rows, d, L) != hipSuccess) return -1;
  return (int64_t)L.total_bytes;
}

int rs_item_index_layout(int nsrc, int64_t rows, int64_t table_rows, int64_t d, int64_t* out) {
  if (nsrc < 1 || nsrc > 3 || rows <= 0 || table_rows <= 0 || d <= 0 || !out) return RS_ERR_ARG;
  ig::Layout L;
  if (ig::layout(nsrc, rows, table_rows, d, L) != hipSuccess) return RS_ERR_ARG;
  out[0] = (int64_t)L.sk;
  out[1] = (int64_t)L.sv;
  out[2] = L.cs ? (int64_t)L.start : -1;
  out[3] = L.path;
  return 0;
}

int rs_item_index_build(int nsrc, const int64_t* keys0, const int64_t* keys1, const int64_t* keys2, int64_t rows,
                        int64_t table_rows, int64_t d, void* ws, int64_t ws_bytes, void* stream) {
  if (nsrc < 1 || nsrc > 3 || rows <= 0 || table_rows <= 0 || !ws || !keys0 || (nsrc > 1 && !keys1) ||
      (nsrc > 2 && !keys2) || nsrc * rows >= ((int64_t)1 << 31))
    return RS_ERR_ARG;
  ig::Layout L;
  hipError_t e = ig::layout(nsrc, rows, table_rows, d, L);
  if (e != hipSuccess) return (int)e;
  if ((int64_t)L.total_bytes > ws_bytes) return RS_ERR_ARG;
  char* w = (char*)ws;
  hipStream_t s = (hipStream_t)stream;
  const ig::Keys K = {{keys0, keys1, keys2}, rows, L.n, table_rows};
  uint32_t* sk = (uint32_t*)(w + L.sk);
  uint32_t* sv = (uint32_t*)(w + L.sv);
  int* start = (int*)(w + L.start);
  if (L.cs) {
    int* H = (int*)(w + L.H);
    int* total = (int*)(w + L.total);
    static const bool attr = [] {
      return hipFuncSetAttribute((const void*)ig::hist_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 ig::VMAX_LDS * (int)sizeof(int)) == hipSuccess;
    }();
    if (!attr) return RS_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(ig::hist_kernel, dim3((unsigned)L.nb), dim3(256), (size_t)L.V * sizeof(int), s, K, H);
    int* gsum = (int*)(w + L.temp);
    const int64_t G = cdiv(table_rows, 64);
    hipLaunchKernelGGL(ig::prefix_blocks_kernel, dim3((unsigned)G), dim3(256), 0, s, H, L.nb, table_rows, total, gsum);
    // start[v] = exclusive prefix of the per-key totals: group offsets, then a wave scan per group of 64 keys
    hipLaunchKernelGGL(ig::scan_groups_kernel, dim3(1), dim3(1024), 0, s, gsum, G);
    hipLaunchKernelGGL(ig::start_kernel, dim3((unsigned)cdiv(G + 1, 4)), dim3(256), 0, s, total, gsum, table_rows,
                       start);
    hipLaunchKernelGGL(ig::place_kernel, dim3((unsigned)L.nb), dim3(256), 0, s, K, H, start, sk, sv);
    return (int)hipGetLastError();
  }
  {
    uint64_t* ping = (uint64_t*)(w + L.ping);
    uint64_t* pong = (uint64_t*)(w + L.pong);
    int* hist = (int*)(w + L.hist);
    const int64_t tiles = cdiv(L.n, ig::TB);
    const int scanned = tiles > ig::FUSED_SCAN_TILES;
    const int passes = ig::sort_passes(L.kb), db0 = ig::sort_digit(L.kb);
    const uint64_t* in = nullptr;
    for (int p = 0; p < passes; ++p) {
      const int shift = p * db0, db = std::min(db0, L.kb - shift);
      uint64_t* out = p + 1 == passes ? nullptr : (p % 2 == 0 ? ping : pong);
      hipLaunchKernelGGL(ig::rsort_count_kernel, dim3((unsigned)tiles), dim3(ig::RT), 0, s, K, in, shift, db, hist);
      if (scanned)
        hipLaunchKernelGGL(ig::rsort_scan_kernel, dim3(1), dim3(ig::RT), 0, s, hist, (int64_t)(1 << db) * tiles);
      hipLaunchKernelGGL(ig::rsort_scatter_kernel, dim3((unsigned)tiles), dim3(ig::RT), 0, s, K, in, shift, db, hist,
                         scanned, out, sk, sv);
      in = out;
    }
  }
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  return (int)hipGetLastError();
}

}  // extern "C"

namespace ig {
// fp32 parity path, the bf16 path's chunk structure with fp32 rows and any width d: one workgroup per chunk of CH
// sorted entries sums each key run inside the chunk in entry order (the per-term arithmetic of the atomic kernels,
// embedding.hip); a run wholly inside the chunk goes to its table row (the row's only writer), a run crossing the
// chunk's edge leaves a partial in the chunk's slot (0: the run at its head, 1: the run at its tail), and
// item_span_f32_kernel adds a crossing run's partials in chunk order.  Deterministic -- the fp32 path's earlier
// float-atomic scatter made every fp32 training curve its own chaotic draw -- and parallel over chunks: the previous
// form (one workgroup per table row, its entries in one sequential chain) spent 0.7-1.6 ms of cfg2's fp32 step on
// the Zipf-hottest item's ~6,000 entries.
__device__ __forceinline__ float f32_term(const GradArgs& a, const float* __restrict__ dx, const float* __restrict__ f,
                                          int src, int64_t m, float w, float raw, int64_t d, int64_t c, uint64_t seed) {
  if (src == 0) {
    float t = raw * w;                      // dx * scale
    if (a.drop_p > 0.f) t *= drop_mul(a.drop_p, seed, (uint64_t)(m * d + c));
    return t;
  }
  return w * raw;                           // w1[m] * f or w2[m] * f
}

__global__ __launch_bounds__(256) void item_chunk_f32_kernel(GradArgs a, const float* __restrict__ dx,
                                                             const float* __restrict__ f, int64_t d) {
  __shared__ uint32_t skey[CH + 2];   // [0]: the key before the chunk, [1 .. cnt]: the chunk's, [cnt + 1]: the next
  __shared__ int sm_m[CH];
  __shared__ int sm_src[CH];
  __shared__ float sm_w[CH];
  const int tid = threadIdx.x;
  const int64_t chunk = blockIdx.x, base = chunk * CH;
  const int cnt = (int)min((int64_t)CH, a.n - base);
  if (tid < cnt) {
    skey[tid + 1] = a.sk[base + tid];
    const uint32_t ent = a.sv[base + tid];
    const int src = (int)(ent / (uint64_t)a.rows);
    const int64_t m = (int64_t)ent - (int64_t)src * a.rows;
    sm_m[tid] = (int)m;
    sm_src[tid] = src;
    sm_w[tid] = src == 0 ? a.scale : (src == 1 ? a.w1[m] : a.w2[m]);
  }
  if (tid == CH) skey[0] = base > 0 ? a.sk[base - 1] : 0xffffffffu;
  if (tid == CH + 1) skey[cnt + 1] = base + cnt < a.n ? a.sk[base + cnt] : 0xffffffffu;
  __syncthreads();
  const uint64_t seed = eff_seed(a.salt, a.seed_base);
  for (int64_t c = tid; c < d; c += blockDim.x) {
    float raw[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      raw[j] = 0.f;
      if (j < cnt) {
        const int64_t m = sm_m[j];
        raw[j] = sm_src[j] == 0 ? dx[m * d + c] : f[m * d + c];
      }
    }
    float acc = 0.f;
    int rs = 0;                               // the current run's first entry in the chunk
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      if (j < cnt) {
        acc += f32_term(a, dx, f, sm_src[j], sm_m[j], sm_w[j], raw[j], d, c, seed);
        const uint32_t k = skey[j + 1];
        if (j + 1 == cnt || skey[j + 2] != k) {        // the run ends at entry j of this chunk
          if (k != 0) {                                 // padding_idx 0: no gradient
            const bool from_before = rs == 0 && skey[0] == k;
            const bool past_end = j + 1 == cnt && skey[cnt + 1] == k;
            if (!from_before && !past_end) a.dtable[(int64_t)k * d + c] += acc;
            else a.part[(chunk * 2 + (rs == 0 ? 0 : 1)) * d + c] = acc;
          }
          acc = 0.f;
          rs = j + 1;
        }
      }
    }
  }
}

// one wave per chunk: the chunk holding the first entry of a run that continues past it sums the run's partials in
// chunk order and adds them to the table row
__global__ __launch_bounds__(256) void item_span_f32_kernel(GradArgs a, int64_t nchunks, int64_t d) {
  const int lane = threadIdx.x & 63;
  const int64_t ch = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (ch >= nchunks) return;
  const int64_t base = ch * CH, last = min(a.n, base + CH) - 1;
  const uint32_t k = a.sk[last];
  if (k == 0 || last + 1 >= a.n || a.sk[last + 1] != k) return;     // no run continues past this chunk
  const bool head_here = a.sk[base] != k;
  if (!head_here && base > 0 && a.sk[base - 1] == k) return;         // the run started in an earlier chunk
  int64_t e;                                                         // first entry past the run
  if (a.start) {
    e = a.start[k + 1];
  } else {
    int64_t lo = last + 1;
    e = a.n;
    while (lo < e) {
      const int64_t mid = (lo + e) >> 1;
      if (a.sk[mid] <= k) lo = mid + 1;
      else e = mid;
    }
  }
  const int64_t cl = (e - 1) / CH;                                   // the run's last chunk
  const int own = head_here ? 1 : 0;
  for (int64_t c = lane; c < d; c += 64) {
    float acc = a.part[(ch * 2 + own) * d + c];
    int64_t cc = ch + 1;
    for (; cc + 7 <= cl; cc += 8) {
      float u[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) u[t] = a.part[((cc + t) * 2) * d + c];
#pragma unroll
      for (int t = 0; t < 8; ++t) acc += u[t];
    }
    for (; cc <= cl; ++cc) acc += a.part[(cc * 2) * d + c];
    a.dtable[(int64_t)k * d + c] += acc;
  }
}
}  // namespace ig

static int item_grad_args(const void* ws, int nsrc, int64_t rows, int64_t table_rows, int64_t d, const void* dx,
                          float scale, float drop_p, uint64_t salt, const uint64_t* seed_base, const void* f,
                          const float* w1, const float* w2, float* dtable, ig::GradArgs& a, ig::Layout& L) {
  if (nsrc < 1 || nsrc > 3 || rows <= 0 || !ws || !dtable || !dx || (nsrc > 1 && (!f || !w1)) || (nsrc > 2 && !w2))
    return RS_ERR_ARG;
  hipError_t e = ig::layout(nsrc, rows, table_rows, d, L);
  if (e != hipSuccess) return (int)e;
  const char* w = (const char*)ws;
  a = {(const uint32_t*)(w + L.sk), (const uint32_t*)(w + L.sv), (float*)(w + L.part),
       L.n, rows, (const __bf16*)dx, scale, drop_p, salt, seed_base, (const __bf16*)f, w1, w2, dtable,
       L.cs ? (const int*)(w + L.start) : nullptr, nullptr, nullptr};
  return 0;
}

extern "C" {

int rs_item_grad(const void* ws, int nsrc, int64_t rows, int64_t table_rows, int64_t d, const void* dx, float scale,
                 float drop_p, uint64_t salt, const uint64_t* seed_base, const void* f, const float* w1,
                 const float* w2, float* dtable, void* stream) {
  return rs_item_grad_marked(ws, nsrc, rows, table_rows, d, dx, scale, drop_p, salt, seed_base, f, w1, w2, dtable,
                             nullptr, nullptr, stream);
}

int rs_item_grad_marked(const void* ws, int nsrc, int64_t rows, int64_t table_rows, int64_t d, const void* dx,
                        float scale, float drop_p, uint64_t salt, const uint64_t* seed_base, const void* f,
                        const float* w1, const float* w2, float* dtable, uint8_t* row_marks, uint8_t* epoch_out,
                        void* stream) {
  ig::GradArgs a;
  ig::Layout L;
  if (!row_marks != !epoch_out) return RS_ERR_ARG;
  if (int e = item_grad_args(ws, nsrc, rows, table_rows, d, dx, scale, drop_p, salt, seed_base, f, w1, w2, dtable,
                             a, L))
    return e;
  a.marks = row_marks;
  a.epoch = epoch_out;
  hipStream_t s = (hipStream_t)stream;
  const dim3 g1((unsigned)L.nchunks), g2((unsigned)cdiv(L.nchunks, 4));
  if (d == 64) {
    hipLaunchKernelGGL(ig::item_chunk_kernel<64>, g1, dim3(256), 0, s, a);
    hipLaunchKernelGGL(ig::item_span_kernel<64>, g2, dim3(256), 0, s, a, L.nchunks);
  } else if (d == 128) {
    hipLaunchKernelGGL(ig::item_chunk_kernel<128>, g1, dim3(256), 0, s, a);
    hipLaunchKernelGGL(ig::item_span_kernel<128>, g2, dim3(256), 0, s, a, L.nchunks);
  } else if (d == 256) {
    hipLaunchKernelGGL(ig::item_chunk_kernel<256>, g1, dim3(256), 0, s, a);
    hipLaunchKernelGGL(ig::item_span_kernel<256>, g2, dim3(256), 0, s, a, L.nchunks);
  } else {
    return RS_ERR_UNSUPPORTED;
  }
  return (int)hipGetLastError();
}

int rs_item_grad_f32(const void* ws, int nsrc, int64_t rows, int64_t table_rows, int64_t d, const float* dx, float scale,
                     float drop_p, uint64_t salt, const uint64_t* seed_base, const float* f, const float* w1,
                     const float* w2, float* dtable, void* stream) {
  ig::GradArgs a;
  ig::Layout L;
  if (int e = item_grad_args(ws, nsrc, rows, table_rows, d, dx, scale, drop_p, salt, seed_base, f, w1, w2, dtable,
                             a, L))
    return e;
  if (d <= 0 || table_rows < 2) return table_rows < 2 ? 0 : RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t nch = cdiv(L.n, ig::CH);
  hipLaunchKernelGGL(ig::item_chunk_f32_kernel, dim3((unsigned)nch), dim3(d > 128 ? 256 : (d > 64 ? 128 : 64)), 0, s,
                     a, dx, f, d);
  hipLaunchKernelGGL(ig::item_span_f32_kernel, dim3((unsigned)cdiv(nch, 4)), dim3(256), 0, s, a, nch, d);
  return (int)hipGetLastError();
}

}  // extern "C"
