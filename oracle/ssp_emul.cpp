// ORACLE / TEST INFRASTRUCTURE ONLY — never shipped, never loaded by the product libraries.
//
// A host-memory emulation of the libsubspace_hip.so C ABI (include/subspace_hip.h), so that the
// product's HOST code -- the restated solvers, the HBM handlers, the reverse-communication C API
// (iterative-solver_amd/host/*.cpp) -- can be linked against it (oracle/build/libitsolv_emul.so)
// and exercised on CPU-only machines, including several ranks over the host communicator
// (ssp_ctx_attach_host_comm + gloo or sockets).  Every "device" pointer is host memory; every
// operation is the reference's sequential loop (oracle_ops.c, ArrayHandlerIterable.h:46-102),
// reductions are summed locally and then over ranks through the callbacks, selection is the
// reference heap (util/select.h:28-55) per rank followed by the same merge rule ssp_select_merge
// documents.  GPU parity is proven by tests/test_*_gpu.py against the real library, not here.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <initializer_list>
#include <map>
#include <string>
#include <vector>

#include "oracle_ops.h"
#include "subspace_hip.h"

struct ssp_ctx {
  int rank = 0;
  int nranks = 1;
  ssp_host_allreduce_fn allreduce = nullptr;
  ssp_host_allgather_fn allgather = nullptr;
  void* user = nullptr;
  // Operation ledger (host clock here; HIP events in the real library), same names and bytes.
  struct Entry {
    std::string name;
    long long calls = 0;
    double ms = 0, bytes = 0;
  };
  bool ledger_on = false;
  std::vector<Entry> ledger;
  // ssp_gemm_inner_sparse_begin / _end: computed at _begin, delivered at _end
  bool sparse_pending = false;
  std::vector<double> sparse_result;
};

namespace {

// Arithmetic variants of the CPU path (checker knobs, never the product; ssp_emul_set_arith).  Both
// are valid builds of the reference's loops: 0/0 is the sequential, uncontracted arithmetic of an
// x86-64 build without FMA (the default, and what every parity fixture is generated with);
// sum order 1 = 8 interleaved partial sums folded pairwise (a vectorising build of
// std::inner_product), fma 1 = y + a*x contracted to fma(a, x, y) (-ffp-contract=fast on a CPU with
// FMA, as the GPU kernels do).  They measure which steps the reference algorithm itself decides by
// rounding (tests/fortran_cases.py).
int g_sum_order = 0;
int g_fma = 0;

inline double madd(double a, double x, double y) { return g_fma ? std::fma(a, x, y) : y + a * x; }

double dot_n(const double* x, const double* y, size_t n) {
  if (g_sum_order == 1) {
    double p[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    size_t i = 0;
    for (; i + 8 <= n; i += 8)
      for (int l = 0; l < 8; ++l) p[l] = madd(x[i + l], y[i + l], p[l]);
    for (int l = 0; i < n; ++i, ++l) p[l] = madd(x[i], y[i], p[l]);
    return ((p[0] + p[4]) + (p[2] + p[6])) + ((p[1] + p[5]) + (p[3] + p[7]));
  }
  double s = 0;
  for (size_t i = 0; i < n; ++i) s = madd(x[i], y[i], s);
  return s;
}

thread_local std::string g_err;

int fail(int code, const std::string& m) {
  g_err = m;
  return code;
}

int reduce(ssp_ctx* c, double* v, size_t n) {
  if (c->nranks <= 1 || n == 0) return SSP_OK;
  if (!c->allreduce || c->allreduce(v, n, c->user) != 0) return fail(SSP_ERR_COMM, "emul: allreduce failed");
  return SSP_OK;
}

// SSP_EMUL_TRACE=1: every device call on stderr as "op reads -> writes" with vector ids (allocation
// order), to see which vectors a solver's call sequence reads after which writes (a checker aid).
static bool trace_on() {
  static const bool on = std::getenv("SSP_EMUL_TRACE") != nullptr;
  return on;
}
static std::map<const void*, int>& trace_ids() {
  static std::map<const void*, int> ids;
  return ids;
}
static void trace(const char* op, std::initializer_list<const double*> rd, std::initializer_list<const double*> wr,
                  const double* const* rl = nullptr, int nr = 0, const double* const* wl = nullptr, int nw = 0) {
  if (!trace_on()) return;
  auto id = [](const double* p) {
    auto it = trace_ids().find(p);
    return it == trace_ids().end() ? -1 : it->second;
  };
  std::string line = op;
  for (auto p : rd) line += " " + std::to_string(id(p));
  for (int i = 0; i < nr; ++i) line += " " + std::to_string(id(rl[i]));
  line += " ->";
  for (auto p : wr) line += " " + std::to_string(id(p));
  for (int i = 0; i < nw; ++i) line += " " + std::to_string(id(wl[i]));
  std::fprintf(stderr, "%s\n", line.c_str());
}

struct Led {
  ssp_ctx* c;
  const char* name;
  double bytes;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  Led(ssp_ctx* ctx, const char* op, double b) : c(ctx), name(op), bytes(b) {}
  ~Led() {
    if (!c || !c->ledger_on) return;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (auto& e : c->ledger)
      if (e.name == name) {
        e.calls++, e.ms += ms, e.bytes += bytes;
        return;
      }
    c->ledger.push_back({name, 1, ms, bytes});
  }
};

uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
uint64_t stream_key(uint64_t seed, uint64_t stream) { return splitmix64(seed ^ (stream * 0xD1B54A32D192ED03ull)); }
double sign_of(uint64_t key, uint64_t g) { return (splitmix64(key ^ g) & 1) ? -1.0 : 1.0; }

void filter(const size_t* idx, const double* val, size_t nnz, size_t n, size_t off, std::vector<size_t>& li,
            std::vector<double>& lv) {
  for (size_t e = 0; e < nnz; ++e)
    if (idx[e] >= off && idx[e] < off + n) {
      li.push_back(idx[e] - off);
      lv.push_back(val[e]);
    }
}
}  // namespace

extern "C" {

const char* ssp_last_error(void) { return g_err.c_str(); }
const char* ssp_version(void) { return "ssp-emul (host emulation, test infrastructure)"; }
// The emulation's devices: SSP_EMUL_DEVICES of them (default 1), narrowed as the HIP runtime narrows
// them by HIP_VISIBLE_DEVICES (a comma-separated list), so the C API's device choice can be tested.
int ssp_device_count(void) {
  const char* e = std::getenv("SSP_EMUL_DEVICES");
  int n = (e && *e) ? std::atoi(e) : 1;
  if (const char* v = std::getenv("HIP_VISIBLE_DEVICES")) {
    int k = *v ? 1 : 0;
    for (const char* c = v; *c; ++c) k += *c == ',';
    n = std::min(n, k);
  }
  return n;
}
static int g_last_device = -1;
int ssp_ctx_create(int device, ssp_ctx** out) {
  g_last_device = device;
  *out = new ssp_ctx();
  return SSP_OK;
}
// test hook: the device of the last ssp_ctx_create
int ssp_emul_last_device(void) { return g_last_device; }
int ssp_ctx_destroy(ssp_ctx* c) {
  delete c;
  return SSP_OK;
}
void* ssp_ctx_stream(ssp_ctx*) { return nullptr; }
int ssp_synchronize(ssp_ctx*) { return SSP_OK; }
int ssp_alloc(ssp_ctx*, size_t n, double** out) {
  struct Reg {
    double** o;
    ~Reg() {
      if (trace_on() && *o) trace_ids()[*o] = int(trace_ids().size());
    }
  } reg{out};
  *out = static_cast<double*>(std::calloc(std::max<size_t>(n, 1), sizeof(double)));
  return *out ? SSP_OK : fail(SSP_ERR_NOMEM, "emul: calloc");
}
int ssp_free(ssp_ctx*, double* p) {
  std::free(p);
  return SSP_OK;
}
int ssp_release_cached(ssp_ctx*) { return SSP_OK; }
int ssp_memory_stats(ssp_ctx*, size_t* a, size_t* b) {
  *a = *b = 0;
  return SSP_OK;
}
int ssp_upload(ssp_ctx*, double* d, const double* h, size_t n) {
  if (n) std::memcpy(d, h, n * sizeof(double));
  return SSP_OK;
}
int ssp_download(ssp_ctx*, double* h, const double* d, size_t n) {
  if (n) std::memcpy(h, d, n * sizeof(double));
  return SSP_OK;
}
int ssp_comm_unique_id(char* id) {
  std::memset(id, 0, SSP_UNIQUE_ID_BYTES);
  return SSP_OK;
}
int ssp_ctx_attach_comm(ssp_ctx* c, int nranks, int rank, const char*) {
  if (nranks == 1) return SSP_OK;
  // SSP_EMUL_RCCL_JOIN=1 (the fallback rehearsal of tests/test_bench.py): the join "succeeds" with no
  // exchange behind it -- a caller must replace it (bench.py does, when another rank's join failed)
  const char* j = std::getenv("SSP_EMUL_RCCL_JOIN");
  if (j && *j == '1') {
    c->nranks = nranks;
    c->rank = rank;
    c->allreduce = nullptr;
    c->allgather = nullptr;
    return SSP_OK;
  }
  return fail(SSP_ERR_UNSUPPORTED, "emul: no RCCL; use ssp_ctx_attach_host_comm");
}
int ssp_ctx_attach_host_comm(ssp_ctx* c, int nranks, int rank, ssp_host_allreduce_fn ar, ssp_host_allgather_fn ag,
                             void* user) {
  c->nranks = nranks;
  c->rank = rank;
  c->allreduce = ar;
  c->allgather = ag;
  c->user = user;
  return SSP_OK;
}
int ssp_p2p_unique_id(char* id) {
  std::memset(id, 0, SSP_UNIQUE_ID_BYTES);
  std::memcpy(id, "/ssp_emul", 9);
  return SSP_OK;
}
int ssp_ctx_attach_p2p(ssp_ctx*, int nranks, int, const char*) {
  return nranks == 1 ? SSP_OK : fail(SSP_ERR_UNSUPPORTED, "emul: no device memory to share; use ssp_ctx_attach_host_comm");
}
int ssp_ctx_set_comm_timeout(ssp_ctx*, double seconds) {
  return seconds > 0 ? SSP_OK : fail(SSP_ERR_ARG, "ssp_ctx_set_comm_timeout: seconds must be > 0");
}
int sspx_debug_stall(ssp_ctx*, double) { return SSP_OK; }
int ssp_ctx_set_exact_max(ssp_ctx*, size_t) { return SSP_OK; }
int ssp_ctx_rank(ssp_ctx* c) { return c->rank; }
int ssp_ctx_nranks(ssp_ctx* c) { return c->nranks; }
int ssp_allreduce_sum(ssp_ctx* c, double* v, size_t n) { return reduce(c, v, n); }
int ssp_allgather_host(ssp_ctx* c, const void* s, void* r, size_t bytes) {
  if (c->nranks <= 1) {
    if (bytes) std::memcpy(r, s, bytes);
    return SSP_OK;
  }
  if (!c->allgather || c->allgather(s, r, bytes, c->user) != 0) return fail(SSP_ERR_COMM, "emul: allgather failed");
  return SSP_OK;
}
int ssp_shard_range(size_t n, int nranks, int rank, size_t* off, size_t* len) {
  const size_t p = size_t(nranks), r = size_t(rank), b = n / p, e = n % p;
  *off = r * b + std::min(r, e);
  *len = b + (r < e ? 1 : 0);
  return SSP_OK;
}
int ssp_ledger_enable(ssp_ctx* c, int on) {
  c->ledger_on = on != 0;
  return SSP_OK;
}
int ssp_ledger_reset(ssp_ctx* c) {
  c->ledger.clear();
  return SSP_OK;
}
int ssp_ledger_count(ssp_ctx* c) { return int(c->ledger.size()); }
int ssp_ledger_reserve(ssp_ctx*, int) { return SSP_OK; }
int ssp_ledger_entry(ssp_ctx* c, int i, const char** name, long long* calls, double* ms, double* bytes) {
  if (i < 0 || i >= int(c->ledger.size())) return fail(SSP_ERR_ARG, "ssp_ledger_entry: index out of range");
  const auto& e = c->ledger[size_t(i)];
  *name = e.name.c_str();
  *calls = e.calls;
  *ms = e.ms;
  *bytes = e.bytes;
  return SSP_OK;
}

int ssp_fill(ssp_ctx* c, double a, double* x, size_t n) {
  Led l(c, "fill", 8.0 * n);
  trace("fill", {}, {x});
  for (size_t i = 0; i < n; ++i) x[i] = a;
  return SSP_OK;
}
int ssp_scal(ssp_ctx* c, double a, double* x, size_t n) {
  Led l(c, "scal", 16.0 * n);
  trace("scal", {x}, {x});
  for (size_t i = 0; i < n; ++i) x[i] *= a;
  return SSP_OK;
}
int ssp_copy(ssp_ctx* c, double* x, const double* y, size_t n) {
  Led l(c, "copy", 16.0 * n);
  trace("copy", {y}, {x});
  if (n && x != y) std::memmove(x, y, n * sizeof(double));
  return SSP_OK;
}
int ssp_emul_set_arith(int sum_order, int fma) {
  if (sum_order < 0 || sum_order > 1 || fma < 0 || fma > 1) return SSP_ERR_ARG;
  g_sum_order = sum_order;
  g_fma = fma;
  return SSP_OK;
}
int ssp_axpy(ssp_ctx* c, double a, const double* x, double* y, size_t n) {
  Led l(c, "axpy", 24.0 * n);
  trace("axpy", {x, y}, {y});
  for (size_t i = 0; i < n; ++i) y[i] = madd(a, x[i], y[i]);
  return SSP_OK;
}
int ssp_dot(ssp_ctx* c, const double* x, const double* y, size_t n, double* out) {
  Led l(c, "dot", (x == y ? 8.0 : 16.0) * n);
  trace("dot", {x, y}, {});
  *out = dot_n(x, y, n);
  return reduce(c, out, 1);
}
int ssp_gemm_inner(ssp_ctx* c, const double* const* xx, int m, const double* const* yy, int k, size_t n, double* out) {
  std::vector<const double*> distinct(xx, xx + m);
  distinct.insert(distinct.end(), yy, yy + k);
  std::sort(distinct.begin(), distinct.end());
  Led l(c, "gemm_inner", 8.0 * n * double(std::unique(distinct.begin(), distinct.end()) - distinct.begin()));
  trace("gemm_inner", {}, {}, xx, m);
  trace("  with", {}, {}, yy, k);
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < k; ++j) out[size_t(i) * k + j] = dot_n(xx[i], yy[j], n);
  return reduce(c, out, size_t(m) * k);
}
int ssp_gemm_outer_sparse(ssp_ctx*, const double* alphas, const size_t* ptr, const size_t* idx, const double* val,
                          int k, double* const* yy, int m, size_t n, size_t offset);
int ssp_construct_solution(ssp_ctx* c, const double* palphas, const size_t* ptr, const size_t* idx,
                           const double* val, int kp, const double* alphas, const double* const* xx, int k,
                           double* const* yy, int m, size_t n, size_t offset) {
  trace("construct_solution", {}, {}, xx, k, yy, m);
  for (int j = 0; j < m; ++j)
    for (size_t e = 0; e < n; ++e) yy[j][e] = 0;
  if (kp > 0) ssp_gemm_outer_sparse(c, palphas, ptr, idx, val, kp, yy, m, n, offset);
  return ssp_gemm_outer(c, alphas, xx, k, yy, m, n);
}
static int gemm_outer_body(const double* al, const double* const* xx, int k, double* const* yy, int m, size_t n) {
  for (int j = 0; j < m; ++j)
    for (int i = 0; i < k; ++i) {
      const double a = al[size_t(i) * m + j];
      for (size_t e = 0; e < n; ++e) yy[j][e] = madd(a, xx[i][e], yy[j][e]);
    }
  return SSP_OK;
}
int ssp_gemm_outer_set(ssp_ctx* c, const double* al, const double* const* xx, int k, double* const* yy, int m,
                       size_t n) {
  Led l(c, "gemm_outer_set", 8.0 * n * (k + 1.0 * m));
  trace("gemm_outer_set", {}, {}, xx, k, yy, m);
  for (int j = 0; j < m; ++j)
    for (size_t e = 0; e < n; ++e) yy[j][e] = 0;
  return gemm_outer_body(al, xx, k, yy, m, n);
}
int ssp_gemm_outer(ssp_ctx* c, const double* al, const double* const* xx, int k, double* const* yy, int m, size_t n) {
  Led l(c, "gemm_outer", 8.0 * n * (k + 2.0 * m));
  trace("gemm_outer", {}, {}, xx, k, yy, m);
  return gemm_outer_body(al, xx, k, yy, m, n);
}
int ssp_axpy_inner(ssp_ctx* c, const double* cc, const double* x, double* const* yy, int m, const double* z, size_t n,
                   double* out) {
  trace("axpy_inner", {x, z}, {}, nullptr, 0, yy, m);
  for (int j = 0; j < m; ++j) {
    for (size_t e = 0; e < n; ++e) yy[j][e] = madd(cc[j], x[e], yy[j][e]);
    out[j] = dot_n(yy[j], z, n);
  }
  return reduce(c, out, size_t(m));
}
int ssp_scal_inner(ssp_ctx* c, double alpha, double* x, const double* const* yy, int m, size_t n, double* out) {
  trace("scal_inner", {x}, {x}, yy, m);
  for (size_t e = 0; e < n; ++e) x[e] *= alpha;
  for (int j = 0; j < m; ++j) out[j] = dot_n(x, yy[j], n);
  return reduce(c, out, size_t(m));
}
int ssp_axpy_norm(ssp_ctx* c, const double* cc, const double* x, double* const* yy, int m, size_t n, double* out) {
  trace("axpy_norm", {x}, {}, nullptr, 0, yy, m);
  for (int j = 0; j < m; ++j)
    for (size_t e = 0; e < n; ++e) yy[j][e] = madd(cc[j], x[e], yy[j][e]);
  *out = dot_n(yy[0], yy[0], n);
  return reduce(c, out, 1);
}
int ssp_axpy_gram(ssp_ctx* c, const double* cc, double* x, double xs, int store_x, double* const* yy, int m, size_t n,
                  double* out) {
  if (m < 1 || !cc || !out) return fail(SSP_ERR_ARG, "ssp_axpy_gram: bad arguments");
  const bool st = store_x && xs != 1.0;
  Led l(c, "axpy_gram", 8.0 * n * ((st ? 2.0 : 1.0) + 2.0 * m));
  if (st)
    trace("axpy_gram", {x}, {x}, nullptr, 0, yy, m);
  else
    trace("axpy_gram", {x}, {}, nullptr, 0, yy, m);
  std::vector<double> xv(n);
  for (size_t e = 0; e < n; ++e) xv[e] = x[e] * xs;
  if (st) std::copy(xv.begin(), xv.end(), x);
  for (int j = 0; j < m; ++j)
    for (size_t e = 0; e < n; ++e) yy[j][e] = madd(cc[j], xv[e], yy[j][e]);
  for (int j = 0; j < m; ++j) out[j] = dot_n(yy[0], yy[j], n);
  return reduce(c, out, size_t(m));
}
int ssp_transform_gram(ssp_ctx* c, const double* t, double* const* xx, const double* xs, int m, size_t n,
                       double* gram) {
  if (m < 1 || m > 8 || !t) return fail(SSP_ERR_ARG, "ssp_transform_gram: bad arguments");
  Led l(c, gram ? "transform_gram" : "transform", 16.0 * n * m);
  trace("transform", {}, {}, nullptr, 0, xx, m);
  // x_j <- sum_i t(i,j) (xs_i x_i), in order i = 0..m-1 (madd: the build's multiply-add), per element
  std::vector<double> in(static_cast<size_t>(m));
  for (size_t e = 0; e < n; ++e) {
    for (int i = 0; i < m; ++i) in[size_t(i)] = xx[i][e] * (xs ? xs[i] : 1.0);
    for (int j = 0; j < m; ++j) {
      double v = 0;
      for (int i = 0; i < m; ++i) v = madd(t[size_t(i) * m + j], in[size_t(i)], v);
      xx[j][e] = v;
    }
  }
  if (!gram) return SSP_OK;
  // one collective of the m (m + 1) / 2 pair dots (a <= b), the layout the device path reduces
  std::vector<double> pr;
  for (int i = 0; i < m; ++i)
    for (int j = i; j < m; ++j) pr.push_back(dot_n(xx[i], xx[j], n));
  const int rc = reduce(c, pr.data(), pr.size());
  if (rc != SSP_OK) return rc;
  for (int i = 0, q = 0; i < m; ++i)
    for (int j = i; j < m; ++j, ++q) gram[size_t(i) * m + j] = gram[size_t(j) * m + i] = pr[size_t(q)];
  return SSP_OK;
}
int ssp_transform_norms(ssp_ctx* c, const double* t, double* const* xx, const double* xs, int m, size_t n,
                        double* norms2) {
  if (!norms2) return fail(SSP_ERR_ARG, "ssp_transform_norms: null norms2");
  const int rc = ssp_transform_gram(c, t, xx, xs, m, n, nullptr);
  if (rc != SSP_OK) return rc;
  for (int j = 0; j < m; ++j) norms2[j] = dot_n(xx[j], xx[j], n);
  return reduce(c, norms2, size_t(m));
}
int ssp_axpy_pairs_norm(ssp_ctx* c, const double* cc, const double* const* xx, const double* xs, double* const* yy,
                        const double* ys, int m, size_t n, double* out) {
  if (m < 0 || (m > 0 && (!cc || !out))) return fail(SSP_ERR_ARG, "ssp_axpy_pairs_norm: bad arguments");
  Led l(c, "axpy_pairs_norm", 24.0 * n * m);
  trace("axpy_pairs_norm", {}, {}, xx, m, yy, m);
  for (int j = 0; j < m; ++j) {
    const double sx = xs ? xs[j] : 1.0, sy = ys ? ys[j] : 1.0;
    for (size_t e = 0; e < n; ++e) yy[j][e] = madd(cc[j], xx[j][e] * sx, yy[j][e] * sy);
    out[j] = dot_n(yy[j], yy[j], n);
  }
  return m ? reduce(c, out, size_t(m)) : SSP_OK;
}
int ssp_precondition(ssp_ctx*, double* const* a, int nvec, const double* d, const double* shift, size_t n) {
  trace("precondition", {d}, {}, nullptr, 0, a, nvec);
  for (int v = 0; v < nvec; ++v)
    for (size_t i = 0; i < n; ++i) a[v][i] = a[v][i] / ((d[i] - shift[v]) + 1e-15);
  return SSP_OK;
}

int ssp_precondition_norms(ssp_ctx* c, double* const* a, int nvec, const double* d, const double* shift, size_t n,
                           double* norms2) {
  if (nvec < 0 || nvec > 8 || (nvec > 0 && (!a || !shift || !norms2)))
    return fail(SSP_ERR_ARG, "ssp_precondition_norms: bad vectors (0 <= nvec <= 8)");
  if (nvec == 0) return SSP_OK;
  ssp_precondition(c, a, nvec, d, shift, n);
  for (int v = 0; v < nvec; ++v) norms2[v] = dot_n(a[v], a[v], n);
  return reduce(c, norms2, size_t(nvec));
}

int ssp_select_merge(int nranks, const size_t* counts, size_t stride, const size_t* idx, const double* val,
                     size_t nsel, int max, size_t* io, double* vo, size_t* nout) {
  struct It {
    double key;
    size_t idx;
    double val;
  };
  std::vector<It> all;
  for (int r = 0; r < nranks; ++r)
    for (size_t e = 0; e < counts[r]; ++e) {
      const size_t s = size_t(r) * stride + e;
      double k = max ? val[s] : -val[s];
      if (k == 0) k = 0;  // -0 and +0 compare equal in the heap's pair order
      all.push_back({k, idx[s], val[s]});
    }
  std::sort(all.begin(), all.end(),
            [](const It& a, const It& b) { return a.key > b.key || (a.key == b.key && a.idx > b.idx); });
  if (all.size() > nsel) all.resize(nsel);
  std::sort(all.begin(), all.end(), [](const It& a, const It& b) { return a.idx < b.idx; });
  for (size_t e = 0; e < all.size(); ++e) {
    if (io) io[e] = all[e].idx;
    if (vo) vo[e] = all[e].val;
  }
  *nout = all.size();
  return SSP_OK;
}

static int select_common(ssp_ctx* c, const std::vector<size_t>& li, const std::vector<double>& lv, size_t offset,
                         size_t nsel, int max, size_t* io, double* vo, size_t* nout) {
  const int nr = c->nranks;
  std::vector<size_t> sidx(nsel, 0), gidx(nsel * size_t(nr));
  std::vector<double> sval(nsel, 0.0), gval(nsel * size_t(nr));
  for (size_t e = 0; e < li.size(); ++e) {
    sidx[e] = li[e] + offset;
    sval[e] = lv[e];
  }
  size_t cnt = li.size();
  std::vector<size_t> counts(nr);
  if (int s = ssp_allgather_host(c, &cnt, counts.data(), sizeof(size_t))) return s;
  if (nsel) {
    if (int s = ssp_allgather_host(c, sidx.data(), gidx.data(), nsel * sizeof(size_t))) return s;
    if (int s = ssp_allgather_host(c, sval.data(), gval.data(), nsel * sizeof(double))) return s;
  }
  return ssp_select_merge(nr, counts.data(), nsel, gidx.data(), gval.data(), nsel, max, io, vo, nout);
}

int ssp_select(ssp_ctx* c, const double* x, size_t n, size_t offset, size_t nsel, int max, int ignore_sign,
               size_t* io, double* vo, size_t* nout) {
  const size_t k = std::min(n, nsel);
  std::vector<size_t> li(std::max<size_t>(k, 1));
  std::vector<double> lv(std::max<size_t>(k, 1));
  size_t got = 0;
  if (k) or_select(x, n, k, max, ignore_sign, li.data(), lv.data(), &got);
  li.resize(got);
  lv.resize(got);
  return select_common(c, li, lv, offset, nsel, max, io, vo, nout);
}
int ssp_select_max_dot(ssp_ctx* c, const double* x, const double* y, size_t n, size_t offset, size_t nsel, size_t* io,
                       double* vo, size_t* nout) {
  const size_t k = std::min(n, nsel);
  std::vector<size_t> li(std::max<size_t>(k, 1));
  std::vector<double> lv(std::max<size_t>(k, 1));
  size_t got = 0;
  if (k) or_select_max_dot(x, y, n, k, li.data(), lv.data(), &got);
  li.resize(got);
  lv.resize(got);
  return select_common(c, li, lv, offset, nsel, 1, io, vo, nout);
}

int ssp_sparse_copy(ssp_ctx*, double* x, size_t n, size_t off, const size_t* idx, const double* val, size_t nnz) {
  trace("sparse_copy", {}, {x});
  std::vector<size_t> li;
  std::vector<double> lv;
  filter(idx, val, nnz, n, off, li, lv);
  for (size_t i = 0; i < n; ++i) x[i] = 0;
  for (size_t e = 0; e < li.size(); ++e) x[li[e]] = lv[e];
  return SSP_OK;
}
int ssp_sparse_axpy(ssp_ctx*, double a, const size_t* idx, const double* val, size_t nnz, double* x, size_t n,
                    size_t off) {
  trace("sparse_axpy", {x}, {x});
  std::vector<size_t> li;
  std::vector<double> lv;
  filter(idx, val, nnz, n, off, li, lv);
  for (size_t e = 0; e < li.size(); ++e) x[li[e]] += a * lv[e];
  return SSP_OK;
}
int ssp_sparse_axpy_batch(ssp_ctx* c, int nvec, const size_t* ptr, const size_t* idx, const double* val,
                          double* const* xx, size_t n, size_t off) {
  for (int k = 0; k < nvec; ++k) ssp_sparse_axpy(c, 1.0, idx + ptr[k], val + ptr[k], ptr[k + 1] - ptr[k], xx[k], n, off);
  return SSP_OK;
}
int ssp_gemm_inner_sparse(ssp_ctx* c, const double* const* xx, int m, size_t n, size_t off, const size_t* ptr,
                          const size_t* idx, const double* val, int k, double* out) {
  trace("gemm_inner_sparse", {}, {}, xx, m);
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < k; ++j) {
      std::vector<size_t> li;
      std::vector<double> lv;
      filter(idx + ptr[j], val + ptr[j], ptr[j + 1] - ptr[j], n, off, li, lv);
      double s = 0;
      for (size_t e = 0; e < li.size(); ++e) s += xx[i][li[e]] * lv[e];
      out[size_t(i) * k + j] = s;
    }
  return reduce(c, out, size_t(m) * k);
}
int ssp_sparse_dot(ssp_ctx* c, const double* x, size_t n, size_t off, const size_t* idx, const double* val, size_t nnz,
                   double* out) {
  const size_t ptr[2] = {0, nnz};
  const double* xx[1] = {x};
  return ssp_gemm_inner_sparse(c, xx, 1, n, off, ptr, idx, val, 1, out);
}
int ssp_gemm_outer_sparse(ssp_ctx*, const double* al, const size_t* ptr, const size_t* idx, const double* val, int k,
                          double* const* yy, int m, size_t n, size_t off) {
  trace("gemm_outer_sparse", {}, {}, nullptr, 0, yy, m);
  for (int j = 0; j < m; ++j)
    for (int i = 0; i < k; ++i) {
      std::vector<size_t> li;
      std::vector<double> lv;
      filter(idx + ptr[i], val + ptr[i], ptr[i + 1] - ptr[i], n, off, li, lv);
      for (size_t e = 0; e < li.size(); ++e) yy[j][li[e]] += al[size_t(i) * m + j] * lv[e];
    }
  return SSP_OK;
}

// The diagonal families of itsolv_hbm/problems.h SyntheticSpec (same IEEE operations).
static double emul_frac_phi(size_t g, double phi) {
  const double f = double(g) * phi;
  return f - std::floor(f);
}
static double emul_d(const sspx_synth* s, size_t g) {
  return s->diag_kind == SSPX_DIAG_BOUNDED ? 1.0 + 2.0 * emul_frac_phi(g, 0x1.3c6ef372fe950p-1) : 1.0 + double(g);
}

int sspx_synth_action(ssp_ctx* c, const sspx_synth* sp, const double* const* xx, double* const* yy, int nvec,
                      size_t n, size_t off) {
  trace("synth_action", {}, {}, xx, nvec, yy, nvec);
  const int rank = sp->rank;
  std::vector<double> coef(size_t(nvec) * rank, 0.0);
  std::vector<uint64_t> key(rank);
  for (int l = 0; l < rank; ++l) key[l] = stream_key(sp->seed, 1000 + l);
  for (int v = 0; v < nvec; ++v)
    for (int l = 0; l < rank; ++l) {
      double s = 0;
      for (size_t i = 0; i < n; ++i) s += (l == 0 ? 1.0 : sign_of(key[l], off + i)) * xx[v][i];
      coef[size_t(v) * rank + l] = s;
    }
  if (int s = reduce(c, coef.data(), coef.size())) return s;
  for (int v = 0; v < nvec; ++v)
    for (size_t i = 0; i < n; ++i) {
      double t = 0;
      for (int l = 0; l < rank; ++l) t += (l == 0 ? 1.0 : sign_of(key[l], off + i)) * coef[size_t(v) * rank + l];
      yy[v][i] = emul_d(sp, off + i) * xx[v][i] + sp->rho * t;
    }
  return SSP_OK;
}
int sspx_synth_add_lowrank(ssp_ctx*, const sspx_synth* sp, double* const* yy, int nvec, size_t n, size_t off,
                           const double* w) {
  trace("synth_add_lowrank", {}, {}, yy, nvec, yy, nvec);
  for (int v = 0; v < nvec; ++v)
    for (size_t i = 0; i < n; ++i) {
      double t = 0;
      for (int l = 0; l < sp->rank; ++l)
        t += (l == 0 ? 1.0 : sign_of(stream_key(sp->seed, 1000 + l), off + i)) * w[size_t(v) * sp->rank + l];
      yy[v][i] += sp->rho * t;
    }
  return SSP_OK;
}
int sspx_synth_diagonal(ssp_ctx*, const sspx_synth* sp, double* d, size_t n, size_t off) {
  for (size_t i = 0; i < n; ++i) {
    if (sp->diag_kind == SSPX_DIAG_BOUNDED) {
      const double t = 2.0 * emul_frac_phi(off + i, 0x1.827f5352054c6p-1) - 1.0;
      const double s = sp->alpha * t;
      d[i] = emul_d(sp, off + i) * (1.0 + s);
    } else {
      d[i] = 1.0 + double(off + i) + sp->rank * sp->rho;
    }
  }
  return SSP_OK;
}
int sspx_synthetic_action(ssp_ctx* c, const double* const* xx, double* const* yy, int nvec, size_t n, size_t off,
                          double rho, int rank, unsigned long long seed) {
  const sspx_synth s{rho, rank, seed, SSPX_DIAG_LINEAR, 0.0, 1.0};
  return sspx_synth_action(c, &s, xx, yy, nvec, n, off);
}
int sspx_synthetic_add_lowrank(ssp_ctx* c, double* const* yy, int nvec, size_t n, size_t off, double rho, int rank,
                               unsigned long long seed, const double* w) {
  const sspx_synth s{rho, rank, seed, SSPX_DIAG_LINEAR, 0.0, 1.0};
  return sspx_synth_add_lowrank(c, &s, yy, nvec, n, off, w);
}
int sspx_synthetic_diagonal(ssp_ctx* c, double* d, size_t n, size_t off, double rho, int rank) {
  const sspx_synth s{rho, rank, 0, SSPX_DIAG_LINEAR, 0.0, 1.0};
  return sspx_synth_diagonal(c, &s, d, n, off);
}
int sspx_fill_random(ssp_ctx*, double* x, size_t n, size_t off, unsigned long long seed, unsigned long long vec) {
  const uint64_t key = stream_key(seed, vec);
  for (size_t i = 0; i < n; ++i) x[i] = double(splitmix64(key ^ (off + i)) >> 11) * (2.0 / 9007199254740992.0) - 1.0;
  return SSP_OK;
}
int sspx_dense_action(ssp_ctx*, const double* a, size_t ng, const double* const* xx, double* const* yy, int nvec,
                      size_t n, size_t off) {
  for (int v = 0; v < nvec; ++v)
    for (size_t r = 0; r < n; ++r) {
      double s = 0;
      for (size_t j = 0; j < ng; ++j) s += a[(off + r) * ng + j] * xx[v][j];
      yy[v][r] = s;
    }
  return SSP_OK;
}

// ---- deferred scal (include/subspace_hip.h): restated by definition -- each operand with a scale
// s != 1 is first stored scaled (the eager ssp_scal), then the unscaled call runs.
namespace {
struct Scaled {  // read operands: scaled temporaries where s != 1
  std::vector<std::vector<double>> tmp;
  std::vector<const double*> p;
  Scaled(const double* const* v, const double* s, int cnt, size_t n) {
    tmp.reserve(size_t(cnt));
    for (int i = 0; i < cnt; ++i) {
      if (s && s[i] != 1.0) {
        tmp.emplace_back(v[i], v[i] + n);
        for (auto& e : tmp.back()) e *= s[i];
        p.push_back(tmp.back().data());
      } else {
        p.push_back(v[i]);
      }
    }
  }
};
void scale_dest(double* const* y, const double* s, int cnt, size_t n) {
  for (int j = 0; s && j < cnt; ++j)
    if (s[j] != 1.0)
      for (size_t e = 0; e < n; ++e) y[j][e] *= s[j];
}
}  // namespace

int ssp_scal_copy(ssp_ctx* c, double a, double* x, const double* y, size_t n) {
  Led l(c, "scal_copy", 16.0 * n);
  trace("scal_copy", {y}, {x});
  for (size_t i = 0; i < n; ++i) x[i] = y[i] * a;
  return SSP_OK;
}
int ssp_axpy_scaled(ssp_ctx* c, double a, const double* x, double xs, double* y, double ys, size_t n) {
  Scaled sx(&x, &xs, 1, n);
  scale_dest(&y, &ys, 1, n);
  return ssp_axpy(c, a, sx.p[0], y, n);
}
int ssp_dot_scaled(ssp_ctx* c, const double* x, double xs, const double* y, double ys, size_t n, double* out) {
  if (x == y && xs == ys) {
    Scaled sx(&x, &xs, 1, n);
    return ssp_dot(c, sx.p[0], sx.p[0], n, out);
  }
  Scaled sx(&x, &xs, 1, n), sy(&y, &ys, 1, n);
  return ssp_dot(c, sx.p[0], sy.p[0], n, out);
}
int ssp_gemm_inner_scaled(ssp_ctx* c, const double* const* xx, const double* xs, int m, const double* const* yy,
                          const double* ys, int k, size_t n, double* out) {
  // the same vector on both sides stays one operand (the symmetric panel)
  std::map<std::pair<const double*, double>, std::vector<double>> cache;
  auto sc = [&](const double* const* v, const double* s, int cnt) {
    std::vector<const double*> p;
    for (int i = 0; i < cnt; ++i) {
      if (!s || s[i] == 1.0) {
        p.push_back(v[i]);
        continue;
      }
      auto& t = cache[{v[i], s[i]}];
      if (t.empty()) {
        t.assign(v[i], v[i] + n);
        for (auto& e : t) e *= s[i];
      }
      p.push_back(t.data());
    }
    return p;
  };
  auto px = sc(xx, xs, m), py = sc(yy, ys, k);
  return ssp_gemm_inner(c, px.data(), m, py.data(), k, n, out);
}
int ssp_gemm_outer_scaled(ssp_ctx* c, const double* al, const double* const* xx, const double* xs, int k,
                          double* const* yy, const double* ys, int m, size_t n) {
  Scaled sx(xx, xs, k, n);
  scale_dest(yy, ys, m, n);
  return ssp_gemm_outer(c, al, sx.p.data(), k, yy, m, n);
}
int ssp_gemm_outer_set_scaled(ssp_ctx* c, const double* al, const double* const* xx, const double* xs, int k,
                              double* const* yy, int m, size_t n) {
  Scaled sx(xx, xs, k, n);
  return ssp_gemm_outer_set(c, al, sx.p.data(), k, yy, m, n);
}
int ssp_gemm_inner_sparse_scaled(ssp_ctx* c, const double* const* xx, const double* xs, int m, size_t n, size_t off,
                                 const size_t* ptr, const size_t* idx, const double* val, int k, double* out) {
  Scaled sx(xx, xs, m, n);
  return ssp_gemm_inner_sparse(c, sx.p.data(), m, n, off, ptr, idx, val, k, out);
}
int ssp_gemm_inner_sparse_begin(ssp_ctx* c, const double* const* xx, const double* xs, int m, size_t n, size_t off,
                                const size_t* ptr, const size_t* idx, const double* val, int k) {
  c->sparse_pending = false;  // an uncollected result is discarded
  if (m < 0 || k < 0) return fail(SSP_ERR_ARG, "ssp_gemm_inner_sparse_begin: negative dimension");
  c->sparse_result.assign(size_t(m) * size_t(k), 0.0);
  if (m > 0 && k > 0)
    if (int st = ssp_gemm_inner_sparse_scaled(c, xx, xs, m, n, off, ptr, idx, val, k, c->sparse_result.data()))
      return st;
  c->sparse_pending = true;
  return SSP_OK;
}
int ssp_gemm_inner_sparse_end(ssp_ctx* c, double* out) {
  if (!c->sparse_pending) return fail(SSP_ERR_ARG, "ssp_gemm_inner_sparse_end: nothing pending");
  c->sparse_pending = false;
  if (!c->sparse_result.empty()) {
    if (!out) return fail(SSP_ERR_ARG, "ssp_gemm_inner_sparse_end: null argument");
    std::copy(c->sparse_result.begin(), c->sparse_result.end(), out);
  }
  return SSP_OK;
}
int ssp_construct_solution_scaled(ssp_ctx* c, const double* palphas, const size_t* ptr, const size_t* idx,
                                  const double* val, int kp, const double* alphas, const double* const* xx,
                                  const double* xs, int k, double* const* yy, int m, size_t n, size_t offset) {
  Scaled sx(xx, xs, k, n);
  return ssp_construct_solution(c, palphas, ptr, idx, val, kp, alphas, sx.p.data(), k, yy, m, n, offset);
}
int ssp_block_update(ssp_ctx* c, const double* palphas, const size_t* ptr, const size_t* idx, const double* val,
                     int kp, const double* alphas, const double* const* xx, const double* xs, int k, double* const* yy,
                     const double* ys, int m, size_t n, size_t offset) {
  trace("block_update", {}, {}, xx, k, yy, m);
  Scaled sx(xx, xs, k, n);
  scale_dest(yy, ys, m, n);
  if (kp > 0)
    if (int st = ssp_gemm_outer_sparse(c, palphas, ptr, idx, val, kp, yy, m, n, offset)) return st;
  return k > 0 ? ssp_gemm_outer(c, alphas, sx.p.data(), k, yy, m, n) : SSP_OK;
}
int sspx_synth_action_scaled(ssp_ctx* c, const sspx_synth* sp, const double* const* xx, const double* xs,
                             double* const* yy, int nvec, size_t n, size_t off) {
  Scaled sx(xx, xs, nvec, n);
  return sspx_synth_action(c, sp, sx.p.data(), yy, nvec, n, off);
}

}  // extern "C"
