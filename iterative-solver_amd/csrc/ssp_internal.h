// Internal declarations shared by the libsubspace_hip.so translation units.
// Public surface: include/subspace_hip.h.  Design: DESIGN.md.
#pragma once
#include <hip/hip_ext.h>
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

namespace ssp {
struct P2PComm;  // comm_p2p.hip
}

struct ssp_ctx {
  int device = 0;
  bool ledger_on = false;
  std::vector<ssp_ledger_entry_t> ledger;
  std::vector<hipEvent_t> event_pool;
  int num_cus = 256;
  int inner_per_cu = 4;        // gemm_inner workgroups per CU (SSP_INNER_PER_CU: the A/B knob of tools/ab_inner.py)
  int outer_per_cu = 8;        // gemm_outer workgroups per CU (SSP_OUTER_WG_PER_CU: the A/B knob of tools/outer_cu_ab.py)
  int fused_per_cu = 8;        // workgroups per CU of the fused window passes (SSP_FUSED_PER_CU: tools/fused_cu_ab.py)
  bool select_rank = true;     // k_select_local's threshold-and-rank merge (SSP_SELECT_MERGE=tree: the LDS tree only)
  bool transform_wide = true;   // k_transform's doubled window for the self-dot instance, m > 4 (SSP_TRANSFORM_WIDE=0: off)
  bool synth_stride = false;  // SSP_SYNTH_SHAPE=stride: the synthetic apply kernel grid-strided (A/B)
  bool ledger_dispatch = false;  // SSP_LEDGER_TIMING=dispatch (LedgerScope)
  bool ledger_detail = false;    // SSP_LEDGER_DETAIL: per-instance ledger rows (LedgerScope::detail)
  bool synth_window = false;  // SSP_SYNTH_SHAPE=window: the synthetic apply kernel in the window shape (A/B)
  bool synth_merge = true;    // one launch for all full vector groups of a synthetic action (SSP_SYNTH_MERGE=0: one per group)
  // Shape of the 1 x 1 / 1 x 2 gemm_inner row kernel: window (default) or, with SSP_ROW_SHAPE=stride
  // in the environment at context creation, the round-2 grid-stride shape (A/B: tools/row_shape_ab.py).
  bool row_stride = false;
  // Hand-off of a device-resident reduction result (after k_reduce_partials / an allreduce) to the
  // host: the one-workgroup k_publish kernel (default), or with SSP_PUBLISH=copy a D2H copy of the
  // result followed by a stream write of the sequence flag (A/B: tools/latency_probe.py).
  bool publish_copy = false;
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
  // Arrival counter of the fused reduction tails (FoldTail); zero between launches.
  unsigned* fold_counter = nullptr;
  // One pending sparse inner product (ssp_gemm_inner_sparse_begin / _end): its own device staging,
  // coherent host results and sequence flag, so reductions issued before _end cannot overwrite them.
  double* async_dev = nullptr;
  double* async_host = nullptr;
  unsigned long long* async_flag = nullptr;
  unsigned long long async_seq = 0;
  bool async_pending = false;
  bool async_launched = false;  // false: computed synchronously into async_sync
  size_t async_n = 0;
  std::vector<double> async_sync;

  // Upload ring: pinned host + device mirror for small per-call operand arrays (sparse index
  // lists).  Regions are reused only after a stream synchronisation at wrap-around.  The arrays one
  // op stages are copied by ONE hipMemcpyAsync (flush_uploads, before the op's first launch that
  // reads them): [ring_pending, ring_head) is staged but not yet copied.
  char* ring_host = nullptr;
  char* ring_dev = nullptr;
  size_t ring_cap = 0;
  size_t ring_head = 0;
  size_t ring_pending = 0;
  // Rings replaced by a larger one: arrays staged in them may still be read by queued launches, so
  // they are freed with the context.
  std::vector<std::pair<char*, char*>> retired_rings;

  // Synthetic test problem (synthetic.hip): the per-element sign masks of u_1..u_{rank-1}, computed
  // once per (seed, rank, shard) and reused by every action of a solve.
  unsigned short* synth_mask = nullptr;
  size_t synth_mask_n = 0, synth_mask_offset = 0;
  unsigned long long synth_mask_seed = 0;
  int synth_mask_rank = 0;

  // Communicator (RCCL over xGMI, one process per GPU).
  ncclComm_t comm = nullptr;
  // Host-callback communicator (ssp_ctx_attach_host_comm), used instead of RCCL when set.
  ssp_host_allreduce_fn host_allreduce = nullptr;
  ssp_host_allgather_fn host_allgather = nullptr;
  void* host_user = nullptr;
  // Peer-memory communicator (ssp_ctx_attach_p2p, comm_p2p.hip), used instead of RCCL when set.
  ssp::P2PComm* p2p = nullptr;
  int nranks = 1;
  int rank = 0;
  // Fail-fast (comm_p2p.hip): every wait that depends on other ranks gives up after comm_timeout_s
  // (SSP_COMM_TIMEOUT_S, ssp_ctx_set_comm_timeout); the communicator is then aborted and every later
  // exchange on this context returns SSP_ERR_COMM with comm_fail_msg (the reference aborts the whole
  // job, DistrArray.cpp:16-23).
  double comm_timeout_s = 300.0;
  // Vectors of at most this many local elements take the reference's own arithmetic
  // (kernels_exact.hip: sequential sums, no fused multiply-adds); SSP_EXACT_MAX / ssp_ctx_set_exact_max.
  size_t exact_max = 2048;
  bool comm_failed = false;
  std::string comm_fail_msg;
  // Coherent host word a device-side exchange sets when it gave up (peer missing / mismatched).
  int* dev_err_host = nullptr;
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
// Stages `bytes` from host into the upload ring and returns the device address the data will have;
// the copy itself is issued by flush_uploads, which every launch that reads staged data is preceded by.
int upload_small(ssp_ctx* ctx, const void* host, size_t bytes, void** dev);
// One host-to-device copy of everything staged since the last flush (no-op when nothing is staged).
int flush_uploads(ssp_ctx* ctx);
// Sums the rank-local device results over ranks (no-op for one rank).
int allreduce_dev(ssp_ctx* ctx, double* buf, size_t n);
// After an attach: every rank takes the smallest exact_max of the communicator's ranks.
int agree_exact_max(ssp_ctx* ctx);
// The outcome of an RCCL call on the context's communicator (an error aborts it and returns
// SSP_ERR_COMM; ncclInProgress is waited out under the deadline).
int rccl_settle(ssp_ctx* ctx, ncclResult_t r, const char* what);
// Copies n doubles of ctx->result_dev to host `out` once every operation queued before it has
// completed (publish kernel + host poll of a sequence flag; see context.hip).
int fetch_result(ssp_ctx* ctx, double* out, size_t n);
// Sums ctx->result_dev[0, n) over ranks and delivers it to host `out` (allreduce_dev + fetch_result,
// or the peer-memory transport's fused exchange-and-publish).
int reduce_fetch(ssp_ctx* ctx, double* out, size_t n);
// Waits (host poll) until the publish flag carries seq; bounded when a communicator is attached.
int wait_flag(ssp_ctx* ctx, unsigned long long seq, bool* seen, const char* what = "reduction",
              const unsigned long long* flag = nullptr);
// Allocates the pending-sparse-inner buffers (kAsyncResults doubles) on first use.
constexpr size_t kAsyncResults = 64 * 32;
int ensure_async(ssp_ctx* ctx);
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
// Two timings (SSP_LEDGER_TIMING, read at context creation):
//   events   (default) an event recorded on the stream before the op's work and one after it: the op's
//            time includes any wait of an idle stream for the host to submit the op's first kernel;
//   dispatch the op's first kernel carries the start event and every kernel of the op the stop event
//            (hipExtLaunchKernel, through SSP_LAUNCH): first kernel start to last kernel end, the
//            interval a kernel trace shows for the op.
class LedgerScope {
 public:
  LedgerScope(ssp_ctx* ctx, const char* op, double bytes);
  ~LedgerScope();
  LedgerScope(const LedgerScope&) = delete;
  LedgerScope& operator=(const LedgerScope&) = delete;
  // SSP_LEDGER_DETAIL (read at context creation): the op's call and bytes move to the entry
  // "<op> [tag]" -- per-instance ledger rows (kernel shape) for the development tools
  void detail(const std::string& tag);
  // dispatch timing: the events for the next kernel launched on this thread inside an open scope, when
  // it is launched on that scope's context stream
  static bool dispatch_events(hipStream_t stream, hipEvent_t* start, hipEvent_t* stop);

 private:
  ssp_ctx* ctx_;
  int slot_ = -1;
  hipEvent_t start_ = nullptr;
  hipEvent_t stop_ = nullptr;  // dispatch timing
  bool launched_ = false;
  double last_bytes_ = 0;
  LedgerScope* prev_ = nullptr;
};

// Kernel launch on the context's stream: hipLaunchKernelGGL, or with dispatch-timed ledger events.
#define SSP_LAUNCH(K, G, B, SHM, ST, ...)                                                  \
  do {                                                                                    \
    hipEvent_t ssp_e0_ = nullptr, ssp_e1_ = nullptr;                                      \
    if (::ssp::LedgerScope::dispatch_events(ST, &ssp_e0_, &ssp_e1_))                      \
      hipExtLaunchKernelGGL(K, G, B, SHM, ST, ssp_e0_, ssp_e1_, 0u, __VA_ARGS__);         \
    else                                                                                  \
      hipLaunchKernelGGL(K, G, B, SHM, ST, __VA_ARGS__);                                  \
  } while (0)

// Window shape for streaming kernels (tools/mb_glds.hip mode a, profiles/r1/mb_stream_shapes.txt):
// a wave covers U x 64 consecutive double2 (U KiB) of each vector per visit.  Visits the whole
// windows of the n2 = n / 2 double2 positions (wave-granular grid stride), then the positions past
// the last whole window (thread-granular), then the odd last element when n is odd.  fw(p0) gets
// the lane's first position of a window (its others are p0 + 64 u), f(p) one position, fo(e) the
// odd element.
template <int U, typename FW, typename F, typename FO>
__device__ __forceinline__ void for_windows_in(size_t n, unsigned bid, unsigned nb, FW&& fw, F&& f, FO&& fo) {
  const int lane = threadIdx.x & 63;
  const size_t gw = size_t(bid) * (kBlock / 64) + (threadIdx.x >> 6);
  const size_t nw = size_t(nb) * (kBlock / 64);
  const size_t n2 = n >> 1, win = 64 * size_t(U), nwin = n2 / win;
  for (size_t c = gw; c < nwin; c += nw) fw(c * win + lane);
  for (size_t i = nwin * win + size_t(bid) * kBlock + threadIdx.x; i < n2; i += size_t(nb) * kBlock) f(i);
  if ((n & 1) && bid == 0 && threadIdx.x == 0) fo(n - 1);
}
// The same over the launch's own grid.
template <int U, typename FW, typename F, typename FO>
__device__ __forceinline__ void for_windows(size_t n, FW&& fw, F&& f, FO&& fo) {
  for_windows_in<U>(n, blockIdx.x, gridDim.x, static_cast<FW&&>(fw), static_cast<F&&>(f), static_cast<FO&&>(fo));
}

// Workgroups for a window-shaped launch over n doubles: one wave per window of u KiB, at most
// per_cu workgroups per CU (grid-stride beyond), at least one.
inline unsigned win_grid(const ssp_ctx* ctx, size_t n, int u, unsigned per_cu) {
  return stream_grid(ctx, ((n >> 1) / (64 * size_t(u)) + 1) * 64, 1, per_cu);
}

// Sum over the 256 threads of a workgroup; result valid in thread 0.  Fixed order.
__device__ inline double block_sum256(double v) {
  __shared__ double wsum[kBlock / 64];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) wsum[wave] = v;
  __syncthreads();
  double s = 0;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) s += wsum[w];
  }
  __syncthreads();  // wsum may be reused by the next call
  return s;
}

// block_sum256 of K values at once (each value's tree exactly block_sum256's); results in thread 0.
template <int K>
__device__ inline void block_sum256_multi(double (&v)[K]) {
  __shared__ double wsum[K][kBlock / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_down(v[k], off, 64);
    if (lane == 0) wsum[k][wave] = v[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      double s = 0;
#pragma unroll
      for (int w = 0; w < kBlock / 64; ++w) s += wsum[k][w];
      v[k] = s;
    }
  }
  __syncthreads();
}

// Reduction tail fused into the kernel that writes the per-workgroup partials (results of at most
// a few dozen doubles): the last workgroup to arrive folds partial[grid][nout] in exactly the order
// of the separate k_reduce_partials pass (per output: thread t sums workgroups t, t + 256, ...,
// then block_sum256), so results are bit-identical to the two-kernel form.  It then stores the
// results in device memory (`out`, for a following allreduce) or publishes them straight into
// coherent host memory followed by the sequence flag (one rank: no second kernel, no D2H copy).
//
// Hand-off: the write-through form of /opt/skills/guides/cdna_hip_programming.md §6 Guideline 16
// (R1; "equally valid" to release/acquire in the split-K recipe of §5): every partial is stored by
// wave 0 of its workgroup with an agent-scope relaxed atomic store, which is a write-through sc1
// store (store_partial); wave 0 drains it (s_waitcnt vmcnt(0)) before lane 0 adds to the arrival
// counters (agent-scope atomics, two levels); the last arriver reads EVERY partial with sc1 loads
// (agent-scope relaxed atomic loads), so its acquire reduces to fence(acquire, "wavefront"), which
// only keeps the compiler from hoisting those loads.  Guideline 16's conditions (1)-(4) for this form
// are checked in the emitted gfx950 assembly of every kernel with the tail by
// tests/test_fold_tail_isa.py.  The C++ memory-model form (release / acq_rel arrivals, agent-scope
// acquire fence; build with -DSSP_FOLD_RELACQ) was measured against it in one process on the same
// vectors (tools/ab_fold.py, profiles/r2/ab_fold_relacq.txt): bit-identical results, 5 % lower call
// latency at n = 1e3 (11.7 vs 12.3 us, within the host-timing noise), but dot at n = 1e8 28 % slower
// (320 vs 250 us: every one of the ~2000 workgroups writes back its L2 before arriving), so the
// write-through form stays.
constexpr unsigned kFoldShards = 8;  // arrival-counter shards (one per XCD's worth of workgroups)
constexpr unsigned kFoldLine = 32;   // unsigned per 128-B line
struct FoldTail {
  unsigned* counter;  // kFoldShards shard counters + the top counter, kFoldLine apart, all zero
  double* out;                // device results, or nullptr
  double* host;               // coherent host results, or nullptr
  unsigned long long* flag;   // with host: set to seq after the results
  unsigned long long seq;
  int nout;
};

// Stores one per-workgroup partial (callers: lanes of wave 0 only).
__device__ inline void store_partial(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int K = 1, int LK = 0>
__device__ inline void fold_tail(const double* partial, const FoldTail& t) {
  __shared__ unsigned s_last;
  if (threadIdx.x < 64) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // wave 0's partial stores have completed
    if (threadIdx.x == 0) {
      // Two-level arrival: workgroup b adds to shard b % 8 (each shard on a 128-B line of its own),
      // the last arriver of a shard resets it and adds to the top counter.  Eight shards keep ~2000
      // same-address atomics from serialising at the end of a launch (one counter: +15 us at 2048
      // workgroups, profiles/r1/latency_probe_fused.json).
      const unsigned G = gridDim.x, sh = blockIdx.x & (kFoldShards - 1);
      const unsigned nsh = G < kFoldShards ? G : kFoldShards, in_sh = (G - sh + kFoldShards - 1) / kFoldShards;
      unsigned last = 0;
      unsigned* c = t.counter + kFoldLine * sh;
#ifdef SSP_FOLD_RELACQ
      // A/B variant (tools/ab_fold.py): the C++ memory-model form -- release on the shard arrival,
      // acquire-release on the top arrival, agent-scope acquire fence in the last arriver.
      constexpr int kArrive = __ATOMIC_RELEASE, kTop = __ATOMIC_ACQ_REL;
#else
      constexpr int kArrive = __ATOMIC_RELAXED, kTop = __ATOMIC_RELAXED;
#endif
      if (__hip_atomic_fetch_add(c, 1u, kArrive, __HIP_MEMORY_SCOPE_AGENT) == in_sh - 1) {
        __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = __hip_atomic_fetch_add(t.counter + kFoldLine * kFoldShards, 1u, kTop, __HIP_MEMORY_SCOPE_AGENT) ==
               nsh - 1;
      }
      s_last = last;
    }
  }
  __syncthreads();
  if (!s_last) return;
#ifdef SSP_FOLD_RELACQ
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#else
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only: the loads are sc1
#endif
  const int G = int(gridDim.x);
  // K outputs at a time: their loads are issued together (K x L in flight per thread, L slots of
  // each output) and their workgroup sums share one LDS round.  Per output the order is that of the
  // separate pass whatever K is -- thread t adds workgroups t, t + 256, ... in that order, then
  // block_sum256's tree -- so every K gives the same bits; a kernel with many outputs (the fused Gram
  // of the block transform: 36) waits one cross-XCD load latency per K outputs instead of per output.
  // L: slots per output and trip (LK when given; by default at most 16 loads in flight, so the fold
  // adds few registers to a lean streaming kernel).  A launch of at most L * 256 workgroups folds each
  // group of K outputs in one trip.
  constexpr int L = LK > 0 ? LK : (K >= 2 ? (16 / K > 2 ? 16 / K : 2) : 8);
  for (int o0 = 0; o0 < t.nout; o0 += K) {
    double s[K];
#pragma unroll
    for (int k = 0; k < K; ++k) s[k] = 0;
    for (int b0 = threadIdx.x; b0 < G; b0 += L * kBlock) {
      double v[K][L];
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int u = 0; u < L; ++u) {
          const int b = b0 + u * kBlock;
          v[k][u] = b < G && o0 + k < t.nout
                        ? __hip_atomic_load(partial + size_t(b) * t.nout + o0 + k, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT)
                        : 0.0;
        }
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int u = 0; u < L; ++u)
          if (b0 + u * kBlock < G) s[k] += v[k][u];
    }
    block_sum256_multi<K>(s);
    if (threadIdx.x == 0) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if (o0 + k < t.nout) {
          if (t.host) __hip_atomic_store(t.host + o0 + k, s[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          else t.out[o0 + k] = s[k];
        }
      }
    }
  }
  if (threadIdx.x == 0) {
    __hip_atomic_store(t.counter + kFoldLine * kFoldShards, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t.host) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the results have reached host memory
      __hip_atomic_store(t.flag, t.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// Host side of FoldTail (context.hip): fold_begin fills the tail for nout results (host publication
// when no communicator is attached); fold_finish delivers the nout results to `out` (waiting on the
// flag, or allreduce + fetch_result).
int fold_begin(ssp_ctx* ctx, int nout, FoldTail* t);
int fold_finish(ssp_ctx* ctx, const FoldTail& t, double* out);

// comm_p2p.hip: transport-independent fail-fast helpers and the peer-memory transport.
// True when reductions/gathers go to other ranks (any transport, including a one-rank RCCL comm).
inline bool comm_attached(const ssp_ctx* ctx) {
  return ctx->comm_failed || ctx->comm || ctx->p2p || (ctx->host_allreduce && ctx->nranks > 1);
}
// SSP_ERR_COMM with the recorded failure, when the communicator has been aborted.
int comm_check(ssp_ctx* ctx);
// Records a communication failure on `what`, aborts the communicator (RCCL: ncclCommAbort; p2p: the
// shared abort word every rank polls) and returns SSP_ERR_COMM.
int comm_fail(ssp_ctx* ctx, const std::string& what);
// Polled once per few hundred spins by every host wait on a rank-dependent result: the deadline
// and RCCL's asynchronous error.  `t0` is the wait's start (steady clock, seconds).
int comm_poll(ssp_ctx* ctx, double t0, const char* what);
double now_s();
// hipStreamSynchronize, bounded by the deadline when a communicator is attached.
int sync_stream(ssp_ctx* ctx, const char* what);
// Peer-memory transport: in-place sum over ranks of n device doubles in fixed rank order (stream
// ordered), and the fused form that publishes the sum into the coherent host result buffer.
int p2p_allreduce_dev(ssp_ctx* ctx, double* buf, size_t n);
int p2p_allreduce_fetch(ssp_ctx* ctx, const double* src, double* out, size_t n);
int p2p_allgather_host(ssp_ctx* ctx, const void* send, void* recv, size_t bytes);
int p2p_detach(ssp_ctx* ctx);
// SSP_ERR_COMM (the communicator aborted) when a peer-memory exchange kernel gave up -- a peer missing
// past the deadline or a mismatched length -- as recorded in the coherent error word; else SSP_OK.
int device_exchange_error(ssp_ctx* ctx, const char* what);

// kernels_exact.hip: the reference's arithmetic for short vectors.  exact_inner forms the m x k (or,
// pairs, the m) dots for the tail of fold_begin (in result_dev for an exchange, or published to the
// host by the last workgroup; fold_finish delivers them); exact_outer updates (set: writes) the
// destinations.
bool exact_mode(const ssp_ctx* ctx, size_t n);
int exact_inner(ssp_ctx* ctx, const double* const* xx, const double* xs, int m, const double* const* yy,
                const double* ys, int k, size_t n, bool pairs, const FoldTail& tail);
int exact_outer(ssp_ctx* ctx, const double* alphas, const double* const* xx, const double* xs, int k,
                double* const* yy, const double* ys, int m, size_t n, bool set);

// kernels_stream.hip
// pub (one rank: fold_begin's tail with a host buffer): the sums go straight to the coherent host result
// buffer at the same offsets as in `out`, and the call's last pass (last = true) raises its flag;
// fold_finish delivers them.  Else into `out` (device), for reduce_fetch.
int launch_reduce_partials(ssp_ctx* ctx, const double* partial, int nblocks, int rows, int cols, double* out,
                           int ldo, int row0, int col0, const FoldTail* pub = nullptr, bool last = false);

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
