// Top-n selection: util::select (reference util/select.h:28-55) and util::select_max_dot
// (reference util/select_max_dot.h:166-190), distributed as DistrArray::select /
// select_max_dot_broadcast do (reference DistrArray.cpp:170-276).
//
// Reference semantics: a min-heap of (v', i) keeps the n lexicographically LARGEST pairs, with
//   select:          v' = max ? (abs ? |x| : x) : (abs ? -|x| : -x),  returned value = max ? v' : -v'
//   select_max_dot:  v' = |x*y|,                                     returned value = v'
// so among equal v' the larger index wins; the result map is ordered by index.
//
// GPU: the order is that of the 128-bit composite (key, i) -- key the order-preserving 64-bit image
// of v', i the index, larger first -- which is exactly the reference's (v', i) order.
//  1. Radix threshold (shards longer than kRadixMin): histogram passes over 12-bit digits of the
//     composite, each restricted to the elements matching the digits fixed so far, until the
//     elements at or above the threshold T fit kRadixCap (typically 1-2 passes over the shard);
//     one compaction pass then collects them.
//  2. Each workgroup sorts a tile of up to 2048 candidates in LDS with a bitonic network
//     (descending) and keeps its best n; levels repeat until one tile remains.
//  1'. For n <= 16 (the solvers' selections: nroots, max_p) one pass instead: each thread keeps its
//     best K in registers, 4-way merge trees in LDS reduce a workgroup's lists to one, and the last
//     workgroup to arrive merges those and publishes the selected (index, value) pairs to the host
//     (k_select_local) -- one launch and no host round trip per digit.
// Ranks then all-gather their local best n and every rank merges the same candidate set with the
// same order on the host (deterministic, identical on all ranks).
#include <algorithm>
#include <cstring>
#include <optional>
#include <vector>

#include "ssp_internal.h"

namespace {

using ssp::kBlock;
constexpr int kTile = ssp::kSelectTile;
constexpr int kTileBlock = 1024;  // one compare-exchange per thread per bitonic stage

struct Cand {
  unsigned long long key;
  unsigned long long idx;
};

__host__ __device__ inline unsigned long long order_key(double v) {
  if (v == 0.0) v = 0.0;  // -0 and +0 compare equal in the reference's pair ordering
  unsigned long long b;
  memcpy(&b, &v, sizeof(b));
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__device__ __forceinline__ bool better(const Cand& a, const Cand& b) {
  return a.key > b.key || (a.key == b.key && a.idx > b.idx);
}

// mode 0: select (uses max/abs flags) on x; mode 1: |x*y|; mode 2: candidates from `in`.
struct SelectArgs {
  const double* x;
  const double* y;
  const Cand* in;
  size_t count;  // number of input elements (mode 0/1) or candidates (mode 2)
  size_t offset; // global index of x[0]
  int mode;
  int max;
  int ignore_sign;
  int keep;      // candidates kept per tile
  Cand* out;     // [gridDim.x][keep]
};

__global__ __launch_bounds__(kTileBlock) void k_select_tile(const SelectArgs a) {
  __shared__ Cand tile[kTile];
  const size_t t0 = size_t(blockIdx.x) * kTile;
  for (int s = threadIdx.x; s < kTile; s += kTileBlock) {
    const size_t g = t0 + s;
    Cand c{0ull, 0ull};  // padding sorts after every real candidate (key 0 is a NaN image)
    if (g < a.count) {
      if (a.mode == 2) {
        c = a.in[g];
      } else {
        double v;
        if (a.mode == 1) {
          v = fabs(a.x[g] * a.y[g]);
        } else {
          const double xv = a.x[g];
          v = a.max ? (a.ignore_sign ? fabs(xv) : xv) : (a.ignore_sign ? -fabs(xv) : -xv);
        }
        c.key = order_key(v);
        c.idx = a.offset + g;
      }
    }
    tile[s] = c;
  }
  __syncthreads();
  // Bitonic sort, descending by (key, idx).
  for (int k = 2; k <= kTile; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < kTile / 2; t += kTileBlock) {
        const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1));  // 2 j (t / j) + t % j, j a power of two
        const int l = i + j;
        const bool desc = ((i & k) == 0);
        Cand ci = tile[i], cl = tile[l];
        const bool swap = desc ? better(cl, ci) : better(ci, cl);
        if (swap) {
          tile[i] = cl;
          tile[l] = ci;
        }
      }
      __syncthreads();
    }
  }
  for (int s = threadIdx.x; s < a.keep; s += kTileBlock) a.out[size_t(blockIdx.x) * a.keep + s] = tile[s];
}

constexpr size_t kRadixMin = size_t(1) << 17;  // shorter shards go straight to the tile sort
constexpr size_t kRadixCap = size_t(1) << 16;  // candidates handed to the tile sort
constexpr int kDigitBits = 12;
constexpr int kBins = 1 << kDigitBits;

struct RadixArgs {
  const double* x;
  const double* y;
  size_t n;
  int neg;  // mode 0: v' = (abs ? |x| : x), negated when neg (select's max = false)
  int abs;
  // Digit extraction at the current composite position: the element matches the fixed prefix when
  // ((key ^ tkey) & pmask) == 0 (key phase) or key == tkey && ((i ^ tidx) & pmask) == 0 (index
  // phase); its digit is ((key or i) >> dshift) & dmask.
  unsigned long long pmask;
  int dshift;
  unsigned dmask;
  unsigned long long tkey, tidx;  // threshold composite (fixed bits, zeros below)
  unsigned* hist;                 // [kBins], zeroed before each pass
  Cand* cand;                     // compaction output
  unsigned long long* counter;
};

// Branch-free order_key of one element's v': mode 1 |x*y|; mode 0 the select transform (sign flips
// and absolute values as bit operations, so every input's bits map exactly as order_key maps them),
// -0 as +0, then the order-preserving image.
template <int MODE>
__device__ __forceinline__ unsigned long long elem_key(const RadixArgs& a, double xv, double yv) {
  double v = MODE == 1 ? fabs(xv * yv) : (a.abs ? fabs(xv) : xv);
  if (MODE == 0) v = a.neg ? -v : v;
  long long b = __double_as_longlong(v);
  b = (b << 1) != 0 ? b : 0;
  return (unsigned long long)(b ^ ((b >> 63) | (long long)0x8000000000000000ull));
}

template <bool IDX>
__device__ __forceinline__ int elem_digit(const RadixArgs& a, unsigned long long key, unsigned long long i) {
  const unsigned long long w = IDX ? i : key;
  const bool match = IDX ? (key == a.tkey && ((i ^ a.tidx) & a.pmask) == 0) : (((key ^ a.tkey) & a.pmask) == 0);
  return match ? int((w >> a.dshift) & a.dmask) : -1;
}

__device__ __forceinline__ void hist_add(unsigned* h, int d) {
  // Concentrated data sends whole waves to one bin: one atomic per wave then.
  const int d0 = __builtin_amdgcn_readfirstlane(d);
  const unsigned long long same = __ballot(d == d0);
  if (same == __ballot(1)) {
    if (d0 >= 0 && __lane_id() == 0) atomicAdd(&h[d0], unsigned(__popcll(same)));
  } else if (d >= 0) {
    atomicAdd(&h[d], 1u);
  }
}

// Streams the shard in iterations of kRadixU double2 slots per lane, unguarded while every slot is
// a whole pair, then one guarded tail; f(key, local index, valid) for each element, the same number
// of calls on every lane of a wave (the ballots in f need the whole wave).
constexpr int kRadixU = 4;
template <int MODE, typename F>
__device__ __forceinline__ void radix_stream(const RadixArgs& a, F&& f) {
  const size_t stride = size_t(gridDim.x) * kBlock, npair = a.n / 2, n2 = (a.n + 1) / 2;
  size_t p0 = size_t(blockIdx.x) * kBlock;
  for (; p0 + (kRadixU - 1) * stride + kBlock <= npair; p0 += kRadixU * stride) {
    double2 xv[kRadixU], yv[kRadixU];
#pragma unroll
    for (int u = 0; u < kRadixU; ++u) {
      const size_t i = 2 * (p0 + threadIdx.x + u * stride);
      xv[u] = ssp::ld2nt(a.x + i);
      if (MODE == 1) yv[u] = ssp::ld2nt(a.y + i);
    }
#pragma unroll
    for (int u = 0; u < kRadixU; ++u) {
      const unsigned long long i = 2 * (p0 + threadIdx.x + u * stride);
      f(elem_key<MODE>(a, xv[u].x, MODE == 1 ? yv[u].x : 0.0), i, true);
      f(elem_key<MODE>(a, xv[u].y, MODE == 1 ? yv[u].y : 0.0), i + 1, true);
    }
  }
  for (; p0 < n2; p0 += kRadixU * stride) {
#pragma unroll
    for (int u = 0; u < kRadixU; ++u) {
      const size_t i = 2 * (p0 + threadIdx.x + u * stride);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const bool ok = i + e < a.n;
        const double xe = ok ? a.x[i + e] : 0.0;
        const double ye = (MODE == 1 && ok) ? a.y[i + e] : 0.0;
        f(elem_key<MODE>(a, xe, ye), i + e, ok);
      }
    }
  }
}

template <int MODE, bool IDX>
__global__ __launch_bounds__(kBlock) void k_radix_hist(const RadixArgs a) {
  __shared__ unsigned h[kBins];
  for (int s = threadIdx.x; s < kBins; s += kBlock) h[s] = 0;
  __syncthreads();
  radix_stream<MODE>(a, [&](unsigned long long key, unsigned long long i, bool ok) {
    hist_add(h, ok ? elem_digit<IDX>(a, key, i) : -1);
  });
  __syncthreads();
  // Block histograms meet in one global histogram through integer atomics (order-free, so the
  // counts are exact and reproducible); only the bins this block touched are sent.  Replaces a
  // per-block table summed by a second kernel (131 us per pass at N = 1e8, latency-bound).
  for (int s = threadIdx.x; s < kBins; s += kBlock)
    if (h[s]) atomicAdd(&a.hist[s], h[s]);
}

// Every element whose composite is >= (tkey, tidx).  Slots are claimed once per wave (ballot, one
// atomic for the wave's survivors, lane prefix counts).  The slot order is arbitrary; the tile sort
// that follows orders the candidates completely, so the selection does not depend on it.
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_radix_compact(const RadixArgs a, size_t offset) {
  const unsigned long long lt = (1ull << __lane_id()) - 1ull;
  radix_stream<MODE>(a, [&](unsigned long long key, unsigned long long i, bool ok) {
    const bool take = ok && (key > a.tkey || (key == a.tkey && i >= a.tidx));
    const unsigned long long mask = __ballot(take);
    if (mask) {
      const int leader = __ffsll((long long)mask) - 1;
      unsigned long long base = 0;
      if (__lane_id() == leader) base = atomicAdd(a.counter, (unsigned long long)__popcll(mask));
      base = __shfl(base, leader, 64);
      const unsigned long long slot = base + __popcll(mask & lt);
      if (take && slot < kRadixCap) a.cand[slot] = Cand{key, offset + i};
    }
  });
}

// Single pass for a small n (nsel <= K <= 16; the solvers select nroots and max_p elements): every
// thread keeps its K best composites in registers, sorted, while it streams its elements (radix_stream's
// order).  The workgroup's 256 lists then meet in a 4-way merge tree in LDS (4 levels of K-step merges),
// and the last workgroup to arrive merges every workgroup's list the same way.  One read of the shard,
// one launch, no host round trip; the radix path needs a histogram pass and a host decision per digit,
// a compaction pass and the tile levels (k_select_tile) after it.  (Round 6 first merged the lists by
// lane-shuffle butterflies of bitonic merges: 0.08 / 0.15 ms per call for K = 8 / 16, mostly merging.)
constexpr size_t kLocalMaxK = 16;

// Field-wise selects: a select between two whole Cand values becomes a select between their
// addresses, which keeps the lists in scratch memory.
__device__ __forceinline__ Cand cand_pick(bool first, const Cand& x, const Cand& y) {
  return Cand{first ? x.key : y.key, first ? x.idx : y.idx};
}

template <int K>
__device__ __forceinline__ void cand_cswap(Cand& a, Cand& b) {  // a <- better, b <- worse
  const bool sw = better(b, a);
  const Cand x = a, y = b;
  a = cand_pick(sw, y, x);
  b = cand_pick(sw, x, y);
}

// c into the sorted list L (best first) when it beats the last entry.  The K comparisons with c are
// independent of one another (c's position is where they turn true), and every entry is then
// chosen from the old list -- its own value, c, or its predecessor -- so nothing waits on a chain of
// compare-and-swaps (a 15-deep chain of dependent 64-bit compares per insertion before).
template <int K>
__device__ __forceinline__ void cand_insert(Cand (&L)[K], Cand c) {
  if (!better(c, L[K - 1])) return;
  bool b[K];
#pragma unroll
  for (int j = 0; j < K; ++j) b[j] = better(c, L[j]);
  Cand N[K];
#pragma unroll
  for (int j = 0; j < K; ++j) N[j] = cand_pick(!b[j], L[j], j > 0 && b[j > 0 ? j - 1 : 0] ? L[j > 0 ? j - 1 : 0] : c);
#pragma unroll
  for (int j = 0; j < K; ++j) L[j] = N[j];
}

// L <- the K best of the sorted list L and the H-entry sorted list c (both best first; c stands for
// the K-list c followed by padding), sorted: the better of L[K-1-i] and c[i] (a bitonic sequence
// holding the K best), then a bitonic clean.  Counted loops with compile-time trip counts only: a
// shift-stepped loop was left rolled, and its uniform index sent L to scratch memory (2.3 ms per call
// at 12.5e6 elements).
template <int K, int H>
__device__ __forceinline__ void cand_merge_into(Cand (&L)[K], const Cand (&c)[H]) {
  constexpr int kLogK = K == 8 ? 3 : 4;
  static_assert((K == 8 || K == 16) && H <= K, "cand_merge_into: K is 8 or 16, H <= K");
#pragma unroll
  for (int i = 0; i < H; ++i) L[K - 1 - i] = cand_pick(better(L[K - 1 - i], c[i]), L[K - 1 - i], c[i]);
#pragma unroll
  for (int sh = 0; sh < kLogK; ++sh) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const int h = (K / 2) >> sh;
      if ((j & h) == 0) cand_cswap<K>(L[j], L[j + h]);
    }
  }
}

template <int K>
__device__ __forceinline__ void cand_merge(Cand (&L)[K], const Cand (&P)[K]) {
  cand_merge_into<K, K>(L, P);
}

// Sorts 8 candidates, best first (the 19-comparator network).
__device__ __forceinline__ void sort8(Cand (&c)[8]) {
  constexpr int kNet[19][2] = {{0, 2}, {1, 3}, {4, 6}, {5, 7}, {0, 4}, {1, 5}, {2, 6}, {3, 7}, {0, 1}, {2, 3},
                               {4, 5}, {6, 7}, {2, 4}, {3, 5}, {1, 4}, {3, 6}, {1, 2}, {3, 4}, {5, 6}};
#pragma unroll
  for (int s = 0; s < 19; ++s) cand_cswap<8>(c[kNet[s][0]], c[kNet[s][1]]);
}

// The largest head h (a lane's best key) that at least K heads of the wave reach (0 if none): K
// entries of the wave have a key >= it, so a key below it cannot be among the K best.  seg: the
// wave's 64 LDS slots; every lane of the wave takes part.
template <int K>
__device__ __forceinline__ unsigned long long wave_threshold(unsigned long long h, unsigned long long* seg) {
  __builtin_amdgcn_wave_barrier();
  seg[__lane_id()] = h;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  int cnt = 0;
#pragma unroll 16
  for (int j = 0; j < 64; ++j) cnt += seg[j] >= h;
  unsigned long long prop = cnt >= K ? h : 0ull;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const unsigned long long o = __shfl_xor(prop, off, 64);
    prop = o > prop ? o : prop;
  }
  return prop;
}

// k_select_local's pass over the shard (radix_stream's order and slots): each lane's 8 elements of an
// iteration that beat both its list's last entry and the wave threshold T are sorted by a network and
// merged into the list at once (one merge instead of up to 8 insertions, each a K-wide compare and
// select); T is refreshed after the first merge and after every later one that follows an element
// T turned away (a refresh when T filters nothing -- ascending data -- is wasted).  The guarded tail
// inserts one element at a time.
template <int MODE, int K>
__device__ __forceinline__ void select_stream(const RadixArgs& a, size_t offset, Cand (&L)[K], unsigned long long* seg) {
  static_assert(kRadixU == 4, "select_stream: 8 elements per lane and iteration");
  const size_t stride = size_t(gridDim.x) * kBlock, npair = a.n / 2, n2 = (a.n + 1) / 2;
  size_t p0 = size_t(blockIdx.x) * kBlock;
  unsigned long long T = 0;
  bool stale = true;  // wave-uniform: refresh T at the next merge (T has turned an element away since)
  for (; p0 + (kRadixU - 1) * stride + kBlock <= npair; p0 += kRadixU * stride) {
    double2 xv[kRadixU], yv[kRadixU];
#pragma unroll
    for (int u = 0; u < kRadixU; ++u) {
      const size_t i = 2 * (p0 + threadIdx.x + u * stride);
      xv[u] = ssp::ld2nt(a.x + i);
      if (MODE == 1) yv[u] = ssp::ld2nt(a.y + i);
    }
    Cand c[2 * kRadixU];
    bool any = false, rej = false;
#pragma unroll
    for (int u = 0; u < kRadixU; ++u) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const unsigned long long key =
            elem_key<MODE>(a, e ? xv[u].y : xv[u].x, MODE == 1 ? (e ? yv[u].y : yv[u].x) : 0.0);
        const Cand ce{key, offset + 2 * (p0 + threadIdx.x + u * stride) + e};
        const bool b = better(ce, L[K - 1]), keep = b && key >= T;
        c[2 * u + e] = cand_pick(keep, ce, Cand{0ull, 0ull});
        any |= keep;
        rej |= b && !keep;
      }
    }
    stale |= __ballot(rej) != 0;
    if (__ballot(any) == 0) continue;
    if (any) {
      sort8(c);
      cand_merge_into<K, 2 * kRadixU>(L, c);
    }
    if (stale) {  // skipped while T turns nothing away (e.g. every element better than the last)
      const unsigned long long t = wave_threshold<K>(L[0].key, seg);
      T = t > T ? t : T;
      stale = false;
    }
  }
  for (; p0 < n2; p0 += kRadixU * stride) {
#pragma unroll
    for (int u = 0; u < kRadixU; ++u) {
      const size_t i = 2 * (p0 + threadIdx.x + u * stride);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const bool ok = i + e < a.n;
        const double xe = ok ? a.x[i + e] : 0.0;
        const double ye = (MODE == 1 && ok) ? a.y[i + e] : 0.0;
        const unsigned long long key = elem_key<MODE>(a, xe, ye);
        if (ok && key >= T) cand_insert<K>(L, Cand{key, offset + i + e});
      }
    }
  }
}

// The K best of four sorted lists (best first) in LDS, into registers: K steps, each taking the better
// head of four (a tournament of three comparisons).  At step s the four read positions sum to s, so
// none passes K - 1.
template <int K>
__device__ __forceinline__ void merge4_lds(const Cand* l0, const Cand* l1, const Cand* l2, const Cand* l3,
                                           Cand (&out)[K]) {
  int i0 = 0, i1 = 0, i2 = 0, i3 = 0;
#pragma unroll
  for (int s = 0; s < K; ++s) {
    const Cand h0 = l0[i0], h1 = l1[i1], h2 = l2[i2], h3 = l3[i3];
    const bool a01 = !better(h1, h0), a23 = !better(h3, h2);  // ties: the earlier list
    const Cand w01 = cand_pick(a01, h0, h1), w23 = cand_pick(a23, h2, h3);
    const bool lo = !better(w23, w01);
    out[s] = cand_pick(lo, w01, w23);
    i0 += lo && a01;
    i1 += lo && !a01;
    i2 += !lo && a23;
    i3 += !lo && !a23;
  }
}

// Every thread's list (registers, sorted) merged into s_lists[0] by a 4-way tree in LDS
// (256 -> 64 -> 16 -> 4 -> 1 lists).
template <int K>
__device__ __forceinline__ void block_tree(const Cand (&L)[K], Cand (&s_lists)[kBlock][K]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int j = 0; j < K; ++j) s_lists[t][j] = L[j];
  __syncthreads();
#pragma unroll
  for (int q = kBlock / 4; q >= 1; q /= 4) {
    Cand o[K];
    if (t < q) merge4_lds<K>(s_lists[4 * t], s_lists[4 * t + 1], s_lists[4 * t + 2], s_lists[4 * t + 3], o);
    __syncthreads();
    if (t < q)
#pragma unroll
      for (int j = 0; j < K; ++j) s_lists[t][j] = o[j];
    __syncthreads();
  }
}

// LDS of the threshold-and-rank merges (block_rank, and the last workgroup's final merge).
struct RankLds {
  unsigned long long heads[2 * kBlock];
  Cand c[kBlock];  // the collected candidates
  unsigned long long t;
  unsigned m;      // their number
};

// Places the M collected candidates (R.c[0, M), M <= kBlock) by rank: each one's rank is the number
// of candidates better than it, plus equal composites at lower slots (only the empty-slot padding
// repeats), and ranks 0..K-1 go to s_lists[0].  8 candidates per step, their LDS reads issued
// together (one read at a time left every step waiting on LDS latency); R.c has kBlock slots and
// M <= kBlock, so j0 + 7 < kBlock, and slots at or past M are read and not counted.
template <int K>
__device__ __forceinline__ void rank_place(const RankLds& R, unsigned M, Cand (&s_lists)[kBlock][K]) {
  const unsigned t = threadIdx.x;
  if (t >= M) return;
  const Cand me = R.c[t];
  int r = 0;
  for (unsigned j0 = 0; j0 < M; j0 += 8) {
    Cand o[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) o[u] = R.c[j0 + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const unsigned j = j0 + u;
      r += j < M && (better(o[u], me) || (o[u].key == me.key && o[u].idx == me.idx && j < t));
    }
  }
  if (r < K) s_lists[0][r] = me;
}

// The block_tree result by a threshold and ranks, for lists whose best entries are few.  T is the
// largest head (L[0].key) that at least K heads of its wave reach: K entries of the workgroup have a
// key >= T, so an entry whose key is below T is beaten by K others and cannot be among the K best.
// The entries at or above T (M of them, at least K) are collected in LDS and placed by rank
// (rank_place).  No chain of dependent merge steps: a count over 64 heads and one over M
// candidates.  When more than kBlock entries pass (spread-out data, short shards with padded lists),
// the tree merges instead; the result is the same either way.
template <int K>
__device__ __forceinline__ void block_rank(const Cand (&L)[K], Cand (&s_lists)[kBlock][K], RankLds& R, bool rank) {
  if (!rank) return block_tree<K>(L, s_lists);
  const int t = threadIdx.x;
  const unsigned long long h = L[0].key;
  if (t == 0) {
    R.t = 0ull;
    R.m = 0u;
  }
  R.heads[t] = h;
  __syncthreads();
  const unsigned long long* wh = R.heads + (t & ~63);
  int cnt = 0;
#pragma unroll 16
  for (int j = 0; j < 64; ++j) cnt += wh[j] >= h;
  unsigned long long prop = cnt >= K ? h : 0ull;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const unsigned long long o = __shfl_xor(prop, off, 64);
    prop = o > prop ? o : prop;
  }
  if ((t & 63) == 0) atomicMax(&R.t, prop);
  __syncthreads();
  const unsigned long long T = R.t;
  int c = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) c += L[j].key >= T;
  unsigned pos = 0;
  if (c) pos = atomicAdd(&R.m, unsigned(c));
#pragma unroll
  for (int j = 0; j < K; ++j)
    if (j < c && pos + j < unsigned(kBlock)) R.c[pos + j] = L[j];
  __syncthreads();
  const unsigned M = R.m;
  if (M > unsigned(kBlock)) return block_tree<K>(L, s_lists);  // uniform: M is read after the barrier
  rank_place<K>(R, M, s_lists);
  __syncthreads();
}

// Where the last workgroup of k_select_local leaves the result: the K best composites in `out`
// (device), or -- host != nullptr -- the first `real` of them as (global index bits, returned value)
// pairs written through to coherent host memory, then `seq` in `flag` (k_publish's protocol, without
// the k_select_values and k_publish launches).
struct LocalOut {
  Cand* out;
  bool rank;  // block_rank's threshold-and-rank merge (else the LDS tree alone)
  // rank: the largest K-th best key over the workgroups (agent-scope atomic max; zero between
  // launches, reset by the last workgroup), the final merge's threshold
  unsigned long long* thresh;
  double* host;
  unsigned long long* flag;
  unsigned long long seq;
  int real;
};

// The value the reference returns for a selected element (select.h:52: max ? v' : -v', so the sign
// of a zero is the element's, not the key's); k_select_values computes the same.
template <int MODE>
__device__ __forceinline__ double returned_value(const RadixArgs& a, size_t li) {
  const double xv = a.x[li];
  if (MODE == 1) return fabs(xv * a.y[li]);
  const double v = a.neg ? (a.abs ? -fabs(xv) : -xv) : (a.abs ? fabs(xv) : xv);
  return a.neg ? -v : v;
}

#ifdef SSP_SELECT_CLOCKS
// Development probe (a build with -DSSP_SELECT_CLOCKS, never the shipped library): per-workgroup
// phase times of k_select_local (100 MHz wall clock), summarised by the last workgroup with printf.
__device__ unsigned long long g_sel_clk[4096][3];
#endif

template <int MODE, int K>
__global__ __launch_bounds__(kBlock) void k_select_local(const RadixArgs a, size_t offset, Cand* wg_lists,
                                                         const LocalOut lo, unsigned* counter) {
  static_assert(kBlock == 256, "block_tree: 4^4 lists");
  __shared__ Cand s_lists[kBlock][K];
  __shared__ unsigned s_last;
#ifdef SSP_SELECT_CLOCKS
  const unsigned long long c0 = wall_clock64();
#endif
  Cand L[K];
#pragma unroll
  for (int j = 0; j < K; ++j) L[j] = Cand{0ull, 0ull};  // sorts after every real candidate
  if (lo.rank) {
    __shared__ unsigned long long s_wave[kBlock];
    select_stream<MODE, K>(a, offset, L, s_wave + (threadIdx.x & ~63u));
  } else {
    radix_stream<MODE>(a, [&](unsigned long long key, unsigned long long i, bool ok) {
      if (ok) cand_insert<K>(L, Cand{key, offset + i});
    });
  }
#ifdef SSP_SELECT_CLOCKS
  __syncthreads();
  const unsigned long long c1 = wall_clock64();
#endif
  __shared__ RankLds s_rank;
  block_rank<K>(L, s_lists, s_rank, lo.rank);
#ifdef SSP_SELECT_CLOCKS
  if (threadIdx.x == 0) {
    const unsigned long long c2 = wall_clock64();
    __hip_atomic_store(&g_sel_clk[blockIdx.x & 4095][0], c0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&g_sel_clk[blockIdx.x & 4095][1], c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&g_sel_clk[blockIdx.x & 4095][2], c2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#endif
  // This workgroup's list, written through to the device scope (agent-scope atomic stores), then the
  // arrival; the last arriver reads every list with agent-scope loads (the fold_tail pattern).
  if (threadIdx.x < K) {
    Cand* o = wg_lists + size_t(blockIdx.x) * K + threadIdx.x;
    __hip_atomic_store(&o->key, s_lists[0][threadIdx.x].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&o->idx, s_lists[0][threadIdx.x].idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // This list's K-th best key: K entries of the launch reach it, so it is a threshold for all of them.
  if (lo.thresh && threadIdx.x == 0)
    (void)__hip_atomic_fetch_max(lo.thresh, s_lists[0][K - 1].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < 64) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // wave 0's list stores (and the max) have completed
    if (threadIdx.x == 0)
      s_last = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only: the loads are agent-scope
#ifdef SSP_SELECT_CLOCKS
  unsigned long long cc[3] = {(unsigned long long)wall_clock64(), 0, 0};
  int nchunk = 0;
#endif
  // The final merge by a threshold: only list entries at or above it are collected (a prefix of each
  // sorted list; most lists have none, and only their head is read), then placed by rank.  (Every
  // list in full through block_rank, two chunks of 256 lists at the C4 shard, took 15 / 38 us of the
  // 42 / 67 us K = 8 / 16 kernel.)  The threshold is the larger of two that K entries reach: the
  // launch's largest K-th best key (tight when the best elements sit together, e.g. a sorted
  // diagonal) and, per wave, the K-th best of its 2 x 64 workgroup heads (tight when they are spread
  // out).  More than kBlock entries at the threshold (ties): the chunked merge below.
  bool done = false;
  if (lo.thresh && gridDim.x <= 2 * kBlock) {
    const unsigned t = threadIdx.x;
    if (t == 0) {
      s_rank.t = __hip_atomic_load(lo.thresh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_rank.m = 0u;
    }
    unsigned long long hd[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const unsigned g = t + q * kBlock;
      hd[q] = g < gridDim.x
                  ? __hip_atomic_load(&wg_lists[size_t(g) * K].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                  : 0ull;
      s_rank.heads[(t & ~63u) * 2 + q * 64 + (t & 63u)] = hd[q];
    }
    __syncthreads();
    const unsigned long long* wh = s_rank.heads + (t & ~63u) * 2;
    int cnt[2] = {0, 0};
#pragma unroll 16
    for (int j = 0; j < 128; ++j) {
      const unsigned long long v = wh[j];
      cnt[0] += v >= hd[0];
      cnt[1] += v >= hd[1];
    }
    unsigned long long prop = cnt[0] >= K ? hd[0] : 0ull;
    prop = cnt[1] >= K && hd[1] > prop ? hd[1] : prop;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const unsigned long long o = __shfl_xor(prop, off, 64);
      prop = o > prop ? o : prop;
    }
    if ((t & 63u) == 0) atomicMax(&s_rank.t, prop);
    __syncthreads();
    const unsigned long long T = s_rank.t;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const unsigned g = t + q * kBlock;
      const Cand* wl = wg_lists + size_t(g) * K;
      if (g < gridDim.x && hd[q] >= T) {
        Cand P[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
          P[j].key = __hip_atomic_load(&wl[j].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          P[j].idx = __hip_atomic_load(&wl[j].idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        int c = 0;
#pragma unroll
        for (int j = 0; j < K; ++j) c += P[j].key >= T;
        const unsigned pos = atomicAdd(&s_rank.m, unsigned(c));
#pragma unroll
        for (int j = 0; j < K; ++j)
          if (j < c && pos + j < unsigned(kBlock)) s_rank.c[pos + j] = P[j];
      }
    }
    __syncthreads();
    const unsigned M = s_rank.m;
    if (M <= unsigned(kBlock)) {  // uniform: read after the barrier
      rank_place<K>(s_rank, M, s_lists);
      __syncthreads();
      done = true;
    }
  }
  // The workgroups' lists, kBlock at a time through block_rank; the running result rides along as
  // thread 0's input of the next chunk.
  Cand acc[K];
#pragma unroll
  for (int j = 0; j < K; ++j) acc[j] = Cand{0ull, 0ull};
  for (unsigned base = 0; !done && base < gridDim.x; base += kBlock) {
    const unsigned g = base + threadIdx.x;
    Cand P[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      P[j] = Cand{0ull, 0ull};
      if (g < gridDim.x) {
        P[j].key = __hip_atomic_load(&wg_lists[size_t(g) * K + j].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        P[j].idx = __hip_atomic_load(&wg_lists[size_t(g) * K + j].idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (threadIdx.x == 0 && base > 0) cand_merge<K>(P, acc);
    __syncthreads();  // s_lists is reused
    block_rank<K>(P, s_lists, s_rank, lo.rank);
#ifdef SSP_SELECT_CLOCKS
    if (nchunk < 2) cc[1 + nchunk++] = wall_clock64();
#endif
#pragma unroll
    for (int j = 0; j < K; ++j) acc[j] = s_lists[0][j];
  }
#ifdef SSP_SELECT_CLOCKS
  if (threadIdx.x == 0) {
    const unsigned long long c3 = wall_clock64();
    unsigned long long t0min = ~0ull, t0max = 0, t1max = 0, t2max = 0;
    double ss = 0, sm = 0;
    for (unsigned g = 0; g < gridDim.x && g < 4096; ++g) {
      const unsigned long long u0 = __hip_atomic_load(&g_sel_clk[g][0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long u1 = __hip_atomic_load(&g_sel_clk[g][1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long u2 = __hip_atomic_load(&g_sel_clk[g][2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t0min = u0 < t0min ? u0 : t0min;
      t0max = u0 > t0max ? u0 : t0max;
      t1max = u1 > t1max ? u1 : t1max;
      t2max = u2 > t2max ? u2 : t2max;
      ss += double(u1 - u0);
      sm += double(u2 - u1);
    }
    const double G = double(gridDim.x);
    printf("SELCLK K=%d G=%u n=%lu start_spread=%.2f stream_end=%.2f wg_merge_end=%.2f last_wg_done=%.2f "
           "mean_stream=%.2f mean_wg_merge=%.2f last: arrived=%.2f chunk0=%.2f chunk1=%.2f us\n", K, gridDim.x,
           (unsigned long)a.n, 0.01 * double(t0max - t0min), 0.01 * double(t1max - t0min), 0.01 * double(t2max - t0min),
           0.01 * double(c3 - t0min), 0.01 * ss / G, 0.01 * sm / G, 0.01 * double(cc[0] - t0min),
           0.01 * double(cc[1] - t0min), 0.01 * double(cc[2] - t0min));
  }
#endif
  // s_lists[0] = acc (read from LDS: no register indexing)
  if (!lo.host) {
    if (threadIdx.x < K) lo.out[threadIdx.x] = s_lists[0][threadIdx.x];
  } else if (threadIdx.x < unsigned(lo.real)) {
    const unsigned long long gi = s_lists[0][threadIdx.x].idx;
    __hip_atomic_store(lo.host + 2 * threadIdx.x, __longlong_as_double((long long)gi), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(lo.host + 2 * threadIdx.x + 1, returned_value<MODE>(a, size_t(gi - offset)),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x < 64) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // wave 0's result stores have completed (real <= 16)
    if (threadIdx.x == 0) {
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lo.thresh) __hip_atomic_store(lo.thresh, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lo.host) __hip_atomic_store(lo.flag, lo.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// Fixes digits of the composite threshold until at most kRadixCap elements lie at or above it,
// then compacts them into `cand`; returns their number in *count.
int radix_candidates(ssp_ctx* ctx, int mode, const double* x, const double* y, size_t n, size_t offset,
                     size_t nsel, int max, int ignore_sign, Cand* cand, unsigned* hist,
                     unsigned long long* counter, unsigned grid, size_t* count) {
  RadixArgs a{};
  a.x = x;
  a.y = y;
  a.n = n;
  a.neg = !max;
  a.abs = ignore_sign;
  a.hist = hist;
  int idx_bits = 1;
  while (idx_bits < 64 && ((n - 1) >> idx_bits) != 0) ++idx_bits;
  size_t need = nsel, above = 0;
  std::vector<unsigned> h(kBins);
  int bits = 0;  // composite bits fixed so far (0..128): key bits 63.., then local index bits 63..
  for (;;) {
    const int width = bits < 64 ? std::min(kDigitBits, 64 - bits) : std::min(kDigitBits, 128 - bits);
    const bool idx_phase = bits >= 64;
    const int fixed = idx_phase ? bits - 64 : bits;  // bits fixed within the current word
    a.pmask = fixed ? ~0ull << (64 - fixed) : 0ull;
    a.dshift = 64 - fixed - width;
    a.dmask = (1u << width) - 1u;
    SSP_TRY_HIP(hipMemsetAsync(hist, 0, sizeof(unsigned) * kBins, ctx->stream));
    if (mode == 1 && idx_phase)
      SSP_LAUNCH((k_radix_hist<1, true>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    else if (mode == 1)
      SSP_LAUNCH((k_radix_hist<1, false>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    else if (idx_phase)
      SSP_LAUNCH((k_radix_hist<0, true>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    else
      SSP_LAUNCH((k_radix_hist<0, false>), dim3(grid), dim3(kBlock), 0, ctx->stream, a);
    SSP_TRY_HIP(hipGetLastError());
    // hist is the context's result staging buffer: published to coherent host memory and polled
    // (ssp::fetch_result), not a D2H copy + stream synchronisation.
    SSP_TRY(ssp::fetch_result(ctx, reinterpret_cast<double*>(h.data()), kBins / 2));
    const int nb = 1 << width;
    size_t cum = 0;
    int b = nb - 1;
    for (; b > 0; --b) {
      if (cum + h[b] >= need) break;
      cum += h[b];
    }
    if (!idx_phase)
      a.tkey |= (unsigned long long)b << a.dshift;
    else
      a.tidx |= (unsigned long long)b << a.dshift;
    above += cum;
    need -= cum;
    bits += width;
    if (above + h[b] <= kRadixCap || bits >= 128) {
      *count = above + h[b];
      break;
    }
    if (bits == 64) bits = 128 - idx_bits;  // local indices have no bits above idx_bits
  }
  if (*count > kRadixCap) return ssp::set_error(SSP_ERR_UNSUPPORTED, "ssp_select: radix threshold did not converge");
  a.cand = cand;
  a.counter = counter;
  SSP_TRY_HIP(hipMemsetAsync(counter, 0, sizeof(unsigned long long), ctx->stream));
  if (mode == 1)
    SSP_LAUNCH(k_radix_compact<1>, dim3(grid), dim3(kBlock), 0, ctx->stream, a, offset);
  else
    SSP_LAUNCH(k_radix_compact<0>, dim3(grid), dim3(kBlock), 0, ctx->stream, a, offset);
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}

// Returned values recomputed from the selected elements as the reference returns them
// (select.h:52: max ? v' : -v', so the sign of a zero is the element's, not the key's), written
// beside their global indices (bit patterns) for one publication to the host.
__global__ void k_select_values(const Cand* best, int cnt, const double* x, const double* y, size_t offset, int mode,
                                int max, int ignore_sign, double* out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= cnt) return;
  const unsigned long long gi = best[e].idx;
  const size_t li = size_t(gi - offset);
  const double xv = x[li];
  double r;
  if (mode == 1) {
    r = fabs(xv * y[li]);
  } else {
    const double v = max ? (ignore_sign ? fabs(xv) : xv) : (ignore_sign ? -fabs(xv) : -xv);
    r = max ? v : -v;
  }
  out[2 * e] = __longlong_as_double((long long)gi);
  out[2 * e + 1] = r;
}

int select_impl(ssp_ctx* ctx, int mode, const double* x, const double* y, size_t n, size_t offset, size_t nsel,
                int max, int ignore_sign, size_t* idx_out, double* val_out, size_t* nout) {
  SSP_CHECK_CTX(ctx);
  if (!nout) return ssp::set_error(SSP_ERR_ARG, "ssp_select: null nout");
  *nout = 0;
  if (nsel > size_t(kTile / 2))
    return ssp::set_error(SSP_ERR_UNSUPPORTED, "ssp_select: n > 1024 not supported by the tile selection");
  if (n > 0 && (!x || (mode == 1 && !y))) return ssp::set_error(SSP_ERR_ARG, "ssp_select: null vector");
  const int keep = int(nsel);
  std::vector<size_t> sel_idx;  // this rank's best (global index, returned value)
  std::vector<double> sel_val;
  if (keep > 0 && n > 0) {
    // the op's ledger scope; the one-pass form closes it at its launch, so that the host's wait for the
    // published pairs is not counted as device time (the radix form's host decisions between its
    // passes are part of the op and stay inside)
    std::optional<ssp::LedgerScope> ls;
    ls.emplace(ctx, mode == 1 ? "select_max_dot" : "select", (mode == 1 ? 16.0 : 8.0) * n);
    // Level 0 reads the shard (short shards) or the radix candidates; later levels read the
    // previous level's survivors.
    const bool radix = n > kRadixMin;
    size_t count = radix ? kRadixCap : n;
    size_t tiles = (count + kTile - 1) / kTile;
    const size_t cap = tiles * size_t(keep);  // Cands per level buffer
    const unsigned grid = radix ? std::min<unsigned>(ssp::stream_grid(ctx, n, 4), unsigned(ctx->num_cus) * 4) : 0;
    // Workspace (doubles): two level buffers, radix candidates, the compaction counter; the
    // histogram lives in the result staging buffer (published to the host after each pass).
    const size_t w_lvl = 2 * cap * 2, w_cand = radix ? 2 * kRadixCap : 0;
    SSP_TRY(ssp::ensure_partial(ctx, w_lvl + w_cand + 2));
    SSP_TRY(ssp::ensure_result(ctx, kBins / 2));
    Cand* buf0 = reinterpret_cast<Cand*>(ctx->partial);
    Cand* buf1 = buf0 + cap;
    Cand* cand = buf1 + cap;
    unsigned* hist = reinterpret_cast<unsigned*>(ctx->result_dev);
    auto* counter = reinterpret_cast<unsigned long long*>(ctx->partial + w_lvl + w_cand);
    SelectArgs a{};
    a.keep = keep;
    a.out = buf0;
    bool local = false;      // k_select_local has left the K best in buf0
    bool published = false;  // ... or published the (index, value) pairs to the host itself
    if (radix && nsel <= kLocalMaxK) {
      // one pass, one launch: the K best (K = 8 or 16 >= nsel) of the shard into buf0, then the values
      // (k_select_local); two workgroups per CU (the K = 16 lists allow two waves per SIMD)
      RadixArgs r{};
      r.x = x;
      r.y = y;
      r.n = n;
      r.neg = !max;
      r.abs = ignore_sign;
      const unsigned lgrid = std::min<unsigned>(grid, unsigned(ctx->num_cus) * 2);
      const int K = nsel <= 8 ? 8 : 16;
      // The arrival counter is the reduction tails' top counter (zero between launches: every last
      // arriver resets it; one stream).  Unless results go by copy (SSP_PUBLISH=copy), the kernel
      // publishes the (index, value) pairs itself.
      unsigned* cnt = ctx->fold_counter + ssp::kFoldLine * ssp::kFoldShards;
      const size_t real = std::min(n, nsel);
      SSP_TRY(ssp::ensure_result(ctx, 2 * real));
      // the launch threshold: a 64-bit slot on the top counter's line (unused by the reduction tails)
      auto* thresh = reinterpret_cast<unsigned long long*>(cnt + 16);
      LocalOut lo{buf0, ctx->select_rank, ctx->select_rank ? thresh : nullptr, nullptr, nullptr, 0, int(real)};
      if (!ctx->publish_copy) {
        lo.host = ctx->result_host;
        lo.flag = ctx->pub_flag;
        lo.seq = ++ctx->pub_seq;
      }
      if (mode == 1 && K == 8) SSP_LAUNCH((k_select_local<1, 8>), dim3(lgrid), dim3(kBlock), 0, ctx->stream, r, offset, cand, lo, cnt);
      else if (mode == 1) SSP_LAUNCH((k_select_local<1, 16>), dim3(lgrid), dim3(kBlock), 0, ctx->stream, r, offset, cand, lo, cnt);
      else if (K == 8) SSP_LAUNCH((k_select_local<0, 8>), dim3(lgrid), dim3(kBlock), 0, ctx->stream, r, offset, cand, lo, cnt);
      else SSP_LAUNCH((k_select_local<0, 16>), dim3(lgrid), dim3(kBlock), 0, ctx->stream, r, offset, cand, lo, cnt);
      SSP_TRY_HIP(hipGetLastError());
      local = true;
      if (lo.host) {
        ls.reset();
        bool seen = true;
        SSP_TRY(ssp::wait_flag(ctx, lo.seq, &seen, "select"));
        for (size_t e = 0; e < real; ++e) {
          unsigned long long gi;
          std::memcpy(&gi, &ctx->result_host[2 * e], sizeof(gi));
          sel_idx.push_back(size_t(gi));
          sel_val.push_back(ctx->result_host[2 * e + 1]);
        }
        published = true;
      }
    } else if (radix) {
      SSP_TRY(radix_candidates(ctx, mode, x, y, n, offset, nsel, max, ignore_sign, cand, hist, counter, grid, &count));
      tiles = (count + kTile - 1) / kTile;
      a.in = cand;
      a.count = count;
      a.mode = 2;
    } else {
      a.x = x;
      a.y = y;
      a.count = count;
      a.offset = offset;
      a.mode = mode;
      a.max = max;
      a.ignore_sign = ignore_sign;
    }
    if (!local) {
      SSP_LAUNCH(k_select_tile, dim3(unsigned(tiles)), dim3(kTileBlock), 0, ctx->stream, a);
      SSP_TRY_HIP(hipGetLastError());
      count = tiles * size_t(keep);
    }
    Cand* cur = buf0;
    Cand* nxt = buf1;
    while (!local && tiles > 1) {
      tiles = (count + kTile - 1) / kTile;
      SelectArgs b{};
      b.in = cur;
      b.count = count;
      b.mode = 2;
      b.keep = keep;
      b.out = nxt;
      SSP_LAUNCH(k_select_tile, dim3(unsigned(tiles)), dim3(kTileBlock), 0, ctx->stream, b);
      SSP_TRY_HIP(hipGetLastError());
      count = tiles * size_t(keep);
      std::swap(cur, nxt);
    }
    // The best `real` candidates of this rank (padding sorts after them when n < nsel): indices and
    // returned values in one published block.
    if (!published) {
      const size_t real = std::min(n, nsel);
      SSP_TRY(ssp::ensure_result(ctx, 2 * real));
      SSP_LAUNCH(k_select_values, dim3(unsigned((real + 255) / 256)), dim3(256), 0, ctx->stream, cur, int(real), x,
                 y, offset, mode, max, ignore_sign, ctx->result_dev);
      SSP_TRY_HIP(hipGetLastError());
      std::vector<double> pub(2 * real);
      SSP_TRY(ssp::fetch_result(ctx, pub.data(), 2 * real));
      for (size_t e = 0; e < real; ++e) {
        unsigned long long gi;
        std::memcpy(&gi, &pub[2 * e], sizeof(gi));
        sel_idx.push_back(size_t(gi));
        sel_val.push_back(pub[2 * e + 1]);
      }
    }
  }
  // This rank's best n as (global index, returned value), then the fixed-size exchange: nsel
  // slots per rank plus the real count, and the same host merge on every rank.
  std::vector<size_t> lidx(nsel, 0);
  std::vector<double> lval(nsel, 0.0);
  std::copy(sel_idx.begin(), sel_idx.end(), lidx.begin());
  std::copy(sel_val.begin(), sel_val.end(), lval.begin());
  const int nr = ctx->nranks;
  std::vector<size_t> counts(nr), gidx(nsel * size_t(nr)), gval_bits(nsel * size_t(nr));
  const size_t my_count = sel_idx.size();
  SSP_TRY(ssp_allgather_host(ctx, &my_count, counts.data(), sizeof(size_t)));
  if (nsel) {
    SSP_TRY(ssp_allgather_host(ctx, lidx.data(), gidx.data(), sizeof(size_t) * nsel));
    SSP_TRY(ssp_allgather_host(ctx, lval.data(), gval_bits.data(), sizeof(double) * nsel));
  }
  const double* gval = reinterpret_cast<const double*>(gval_bits.data());
  return ssp_select_merge(nr, counts.data(), nsel, gidx.data(), gval, nsel, (mode == 1) ? 1 : max, idx_out, val_out,
                          nout);
}

}  // namespace

extern "C" {

int ssp_select_merge(int nranks, const size_t* counts, size_t stride, const size_t* idx, const double* val,
                     size_t nsel, int max, size_t* idx_out, double* val_out, size_t* nout) {
  if (!nout || nranks < 1 || (nranks > 0 && !counts)) return ssp::set_error(SSP_ERR_ARG, "ssp_select_merge: bad args");
  *nout = 0;
  struct Item {
    unsigned long long key;
    size_t idx;
    double val;
  };
  std::vector<Item> merged;
  for (int r = 0; r < nranks; ++r) {
    if (counts[r] > stride) return ssp::set_error(SSP_ERR_ARG, "ssp_select_merge: count exceeds stride");
    for (size_t e = 0; e < counts[r]; ++e) {
      const size_t s = size_t(r) * stride + e;
      merged.push_back({order_key(max ? val[s] : -val[s]), idx[s], val[s]});
    }
  }
  // The reference heap keeps the n largest (v', index) pairs: v' descending, larger index first.
  std::sort(merged.begin(), merged.end(),
            [](const Item& p, const Item& q) { return p.key > q.key || (p.key == q.key && p.idx > q.idx); });
  if (merged.size() > nsel) merged.resize(nsel);
  std::sort(merged.begin(), merged.end(), [](const Item& p, const Item& q) { return p.idx < q.idx; });
  for (size_t e = 0; e < merged.size(); ++e) {
    if (idx_out) idx_out[e] = merged[e].idx;
    if (val_out) val_out[e] = merged[e].val;
  }
  *nout = merged.size();
  return SSP_OK;
}

int ssp_select(ssp_ctx* ctx, const double* x, size_t n, size_t offset, size_t nsel, int max, int ignore_sign,
               size_t* idx_out, double* val_out, size_t* nout) {
  return select_impl(ctx, 0, x, nullptr, n, offset, nsel, max, ignore_sign, idx_out, val_out, nout);
}

int ssp_select_max_dot(ssp_ctx* ctx, const double* x, const double* y, size_t n, size_t offset, size_t nsel,
                       size_t* idx_out, double* val_out, size_t* nout) {
  return select_impl(ctx, 1, x, y, n, offset, nsel, 1, 0, idx_out, val_out, nout);
}

}  // extern "C"
