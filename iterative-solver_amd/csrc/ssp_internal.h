// Internal declarations shared by the libsubspace_hip.so translation units.
// Public surface: include/subspace_hip.h.  Design: DESIGN.md.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstddef>
#include <cstdint>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "subspace_hip.h"

// Per-operation ledger: HIP events bracket each hot-path kernel on the context's stream, with the
// operation's algorithmic bytes, resolved lazily when read.
struct ssp_ledger_entry_t {
  std::string name;
  long long calls = 0;
  double ms = 0;
  double bytes = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
};

struct ssp_ctx {
  int device = 0;
  bool ledger_on = false;
  std::vector<ssp_ledger_entry_t> ledger;
  std::vector<hipEvent_t> event_pool;
  int num_cus = 256;
  hipStream_t stream = nullptr;

  // HBM arena: freed blocks are kept by rounded size and recycled (Q vectors are created and
  // destroyed every iteration with identical sizes).
  std::multimap<size_t, void*> free_blocks;
  std::unordered_map<void*, size_t> live_blocks;
  size_t bytes_in_use = 0;
  size_t bytes_cached = 0;

  // Device scratch for per-workgroup partial sums (deterministic two-pass reductions).
  double* partial = nullptr;
  size_t partial_cap = 0;  // doubles
  // Device + pinned host staging for small reduction results.  result_host and pub_flag are
  // coherent host memory: a publish kernel writes the result and then a sequence number, which the
  // host polls (fetch_result) instead of a D2H copy + stream synchronisation.
  double* result_dev = nullptr;
  double* result_host = nullptr;
  size_t result_cap = 0;  // doubles
  unsigned long long* pub_flag = nullptr;
  unsigned long long pub_seq = 0;

  // Upload ring: pinned host + device mirror for small per-call operand arrays (sparse index
  // lists).  Regions are reused only after a stream synchronisation at wrap-around.
  char* ring_host = nullptr;
  char* ring_dev = nullptr;
  size_t ring_cap = 0;
  size_t ring_head = 0;

  // Communicator (RCCL over xGMI, one process per GPU).
  ncclComm_t comm = nullptr;
  // Host-callback communicator (ssp_ctx_attach_host_comm), used instead of RCCL when set.
  ssp_host_allreduce_fn host_allreduce = nullptr;
  ssp_host_allgather_fn host_allgather = nullptr;
  void* host_user = nullptr;
  int nranks = 1;
  int rank = 0;
};

namespace ssp {

constexpr int kBlock = 256;        // 4 waves of 64 lanes
constexpr int kInnerRows = 16;     // one f64 MFMA tile of rows per gemm_inner launch
constexpr int kInnerCols = 64;     // up to 4 f64 MFMA tiles of columns per launch
constexpr int kOuterSrc = 64;      // sources per gemm_outer launch
constexpr int kOuterDst = 16;      // destinations per gemm_outer launch
constexpr int kOuterAlpha = 384;   // alphas carried in the kernel argument block
constexpr int kPrecVec = 16;       // vectors per precondition launch
constexpr int kSelectTile = 2048;  // candidates sorted per workgroup in select

int set_error(int code, const std::string& msg);
int hip_error(hipError_t e, const char* what);
int use_device(ssp_ctx* ctx);
int ensure_partial(ssp_ctx* ctx, size_t n_doubles);
int ensure_result(ssp_ctx* ctx, size_t n_doubles);
// Copies `bytes` from host into the upload ring and returns the device address.
int upload_small(ssp_ctx* ctx, const void* host, size_t bytes, void** dev);
// Sums the rank-local device results over ranks (no-op for one rank).
int allreduce_dev(ssp_ctx* ctx, double* buf, size_t n);
// Copies n doubles of ctx->result_dev to host `out` once every operation queued before it has
// completed (publish kernel + host poll of a sequence flag; see context.hip).
int fetch_result(ssp_ctx* ctx, double* out, size_t n);
// Grid size for streaming kernels: enough workgroups to fill 256 CUs, grid-stride beyond.
// Workgroups for a grid-stride streaming launch: enough for work_items / (kBlock * per_thread),
// at most blocks_per_cu per CU.
unsigned stream_grid(const ssp_ctx* ctx, size_t work_items, unsigned per_thread, unsigned blocks_per_cu = 8);

// Nontemporal 16-byte accesses for vectors streamed exactly once per kernel (measured on gfx950,
// tools/mb_stream.hip: +3-10 % on dot / axpy / gemm_outer against plain global loads/stores).
typedef double nt_double2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ld2nt(const double* p) {
  const nt_double2 v = __builtin_nontemporal_load(reinterpret_cast<const nt_double2*>(p));
  return make_double2(v.x, v.y);
}
__device__ __forceinline__ void st2nt(double* p, double2 v) {
  const nt_double2 w = {v.x, v.y};
  __builtin_nontemporal_store(w, reinterpret_cast<nt_double2*>(p));
}
bool aligned16(const void* p);

// Ledger scope: records a start event now and an end event at destruction (when enabled).
class LedgerScope {
 public:
  LedgerScope(ssp_ctx* ctx, const char* op, double bytes);
  ~LedgerScope();
  LedgerScope(const LedgerScope&) = delete;
  LedgerScope& operator=(const LedgerScope&) = delete;

 private:
  ssp_ctx* ctx_;
  int slot_ = -1;
  hipEvent_t start_ = nullptr;
};

// kernels_stream.hip
int launch_reduce_partials(ssp_ctx* ctx, const double* partial, int nblocks, int rows, int cols, double* out,
                           int ldo, int row0, int col0);

}  // namespace ssp

#define SSP_TRY_HIP(expr)                                   \
  do {                                                      \
    hipError_t _e = (expr);                                 \
    if (_e != hipSuccess) return ssp::hip_error(_e, #expr); \
  } while (0)

#define SSP_TRY(expr)              \
  do {                             \
    int _s = (expr);               \
    if (_s != SSP_OK) return _s;   \
  } while (0)

#define SSP_CHECK_CTX(ctx)                                              \
  do {                                                                  \
    if (!(ctx)) return ssp::set_error(SSP_ERR_ARG, "null ssp_ctx");     \
    SSP_TRY(ssp::use_device(ctx));                                      \
  } while (0)
