// Top-n selection: util::select (reference util/select.h:28-55) and util::select_max_dot
// (reference util/select_max_dot.h:166-190), distributed as DistrArray::select /
// select_max_dot_broadcast do (reference DistrArray.cpp:170-276).
//
// Reference semantics: a min-heap of (v', i) keeps the n lexicographically LARGEST pairs, with
//   select:          v' = max ? (abs ? |x| : x) : (abs ? -|x| : -x),  returned value = max ? v' : -v'
//   select_max_dot:  v' = |x*y|,                                     returned value = v'
// so among equal v' the larger index wins; the result map is ordered by index.
//
// GPU: each workgroup sorts a tile of up to 2048 (key, index) candidates in LDS with a bitonic
// network (descending) and keeps its best n; levels repeat until one tile remains.  key is the
// order-preserving 64-bit image of v', ties broken by index, so the order is exactly the
// reference's (v', i) order.  Ranks then all-gather their local best n and every rank merges the
// same candidate set with the same order on the host (deterministic, identical on all ranks).
#include <algorithm>
#include <cstring>
#include <vector>

#include "ssp_internal.h"

namespace {

using ssp::kBlock;
constexpr int kTile = ssp::kSelectTile;

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

inline double key_value(unsigned long long k) {
  unsigned long long b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  double v;
  std::memcpy(&v, &b, sizeof(v));
  return v;
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

__global__ __launch_bounds__(kBlock) void k_select_tile(const SelectArgs a) {
  __shared__ Cand tile[kTile];
  const size_t t0 = size_t(blockIdx.x) * kTile;
  for (int s = threadIdx.x; s < kTile; s += kBlock) {
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
      for (int t = threadIdx.x; t < kTile / 2; t += kBlock) {
        const int i = 2 * j * (t / j) + (t % j);
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
  for (int s = threadIdx.x; s < a.keep; s += kBlock) a.out[size_t(blockIdx.x) * a.keep + s] = tile[s];
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
  std::vector<Cand> local;
  if (keep > 0 && n > 0) {
    // Level 0 reads the shard; later levels read the previous level's survivors.
    size_t count = n;
    size_t tiles = (count + kTile - 1) / kTile;
    // Workspace: two candidate buffers sized for level 0's output.
    const size_t cap = tiles * size_t(keep);
    SSP_TRY(ssp::ensure_partial(ctx, 4 * cap + 4));
    Cand* buf0 = reinterpret_cast<Cand*>(ctx->partial);
    Cand* buf1 = buf0 + cap;
    SelectArgs a{};
    a.x = x;
    a.y = y;
    a.count = count;
    a.offset = offset;
    a.mode = mode;
    a.max = max;
    a.ignore_sign = ignore_sign;
    a.keep = keep;
    a.out = buf0;
    ssp::LedgerScope ls(ctx, mode == 1 ? "select_max_dot" : "select", (mode == 1 ? 16.0 : 8.0) * n);
    hipLaunchKernelGGL(k_select_tile, dim3(unsigned(tiles)), dim3(kBlock), 0, ctx->stream, a);
    SSP_TRY_HIP(hipGetLastError());
    count = tiles * size_t(keep);
    Cand* cur = buf0;
    Cand* nxt = buf1;
    while (tiles > 1) {
      tiles = (count + kTile - 1) / kTile;
      SelectArgs b{};
      b.in = cur;
      b.count = count;
      b.mode = 2;
      b.keep = keep;
      b.out = nxt;
      hipLaunchKernelGGL(k_select_tile, dim3(unsigned(tiles)), dim3(kBlock), 0, ctx->stream, b);
      SSP_TRY_HIP(hipGetLastError());
      count = tiles * size_t(keep);
      std::swap(cur, nxt);
    }
    local.resize(keep);
    SSP_TRY_HIP(hipMemcpyAsync(local.data(), cur, sizeof(Cand) * keep, hipMemcpyDeviceToHost, ctx->stream));
    SSP_TRY_HIP(hipStreamSynchronize(ctx->stream));
    const size_t real = std::min(n, nsel);
    local.resize(real);
  }
  // This rank's best n as (global index, returned value), then the fixed-size exchange: nsel
  // slots per rank plus the real count, and the same host merge on every rank.
  std::vector<size_t> lidx(nsel, 0);
  std::vector<double> lval(nsel, 0.0);
  for (size_t e = 0; e < local.size(); ++e) {
    const double v = key_value(local[e].key);
    lidx[e] = size_t(local[e].idx);
    lval[e] = (mode == 0 && !max) ? -v : v;
  }
  const int nr = ctx->nranks;
  std::vector<size_t> counts(nr), gidx(nsel * size_t(nr)), gval_bits(nsel * size_t(nr));
  const size_t my_count = local.size();
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
