// Context, HBM arena, staging buffers and the RCCL communicator of libsubspace_hip.so.
//
// The reference keeps Q vectors on disk (DistrArrayFile, reference array/DistrArrayFile.cpp:164-200)
// or in MPI-3 windows and reduces with MPI_Allreduce (reference array/util/gemm.h:179-182).  Here
// every vector shard lives in HBM for the solver's lifetime and reductions are RCCL allreduces on
// the compute stream.
#include <immintrin.h>

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>

#include "ssp_internal.h"

namespace {
thread_local std::string g_last_error;

size_t round_block(size_t bytes) {
  // Small blocks to 256 B, large blocks to 2 MiB so that equal-length vectors share a bucket.
  if (bytes < (size_t(1) << 20)) return (bytes + 255) & ~size_t(255);
  const size_t g = size_t(2) << 20;
  return (bytes + g - 1) / g * g;
}
}  // namespace

namespace ssp {

int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int hip_error(hipError_t e, const char* what) {
  return set_error(SSP_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

int use_device(ssp_ctx* ctx) {
  int cur = -1;
  SSP_TRY_HIP(hipGetDevice(&cur));
  if (cur != ctx->device) SSP_TRY_HIP(hipSetDevice(ctx->device));
  return SSP_OK;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

unsigned stream_grid(const ssp_ctx* ctx, size_t work_items, unsigned per_thread, unsigned blocks_per_cu) {
  const size_t per_block = size_t(kBlock) * per_thread;
  size_t blocks = (work_items + per_block - 1) / per_block;
  const size_t cap = size_t(ctx->num_cus) * blocks_per_cu;  // grid-stride beyond
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  return unsigned(blocks);
}

int ensure_partial(ssp_ctx* ctx, size_t n) {
  if (n <= ctx->partial_cap) return SSP_OK;
  if (ctx->partial) {
    SSP_TRY(sync_stream(ctx, "reduction workspace growth"));
    SSP_TRY_HIP(hipFree(ctx->partial));
    ctx->partial = nullptr;
  }
  size_t cap = std::max(n, size_t(1) << 20);
  if (hipMalloc(&ctx->partial, cap * sizeof(double)) != hipSuccess)
    return set_error(SSP_ERR_NOMEM, "hipMalloc of reduction workspace failed");
  ctx->partial_cap = cap;
  return SSP_OK;
}

int ensure_result(ssp_ctx* ctx, size_t n) {
  if (n <= ctx->result_cap) return SSP_OK;
  SSP_TRY(sync_stream(ctx, "result staging growth"));
  if (ctx->result_dev) SSP_TRY_HIP(hipFree(ctx->result_dev));
  if (ctx->result_host) SSP_TRY_HIP(hipHostFree(ctx->result_host));
  ctx->result_dev = nullptr;
  ctx->result_host = nullptr;
  size_t cap = std::max(n, size_t(1) << 16);
  if (hipMalloc(&ctx->result_dev, cap * sizeof(double)) != hipSuccess)
    return set_error(SSP_ERR_NOMEM, "hipMalloc of result staging failed");
  if (hipHostMalloc(reinterpret_cast<void**>(&ctx->result_host), cap * sizeof(double), hipHostMallocCoherent) !=
      hipSuccess)
    return set_error(SSP_ERR_NOMEM, "hipHostMalloc of result staging failed");
  ctx->result_cap = cap;
  if (!ctx->pub_flag) {
    if (hipHostMalloc(reinterpret_cast<void**>(&ctx->pub_flag), 64, hipHostMallocCoherent) != hipSuccess)
      return set_error(SSP_ERR_NOMEM, "hipHostMalloc of the result flag failed");
    __atomic_store_n(ctx->pub_flag, ctx->pub_seq, __ATOMIC_RELEASE);
  }
  return SSP_OK;
}

int flush_uploads(ssp_ctx* ctx) {
  if (ctx->ring_head > ctx->ring_pending) {
    const size_t o = ctx->ring_pending;
    SSP_TRY_HIP(hipMemcpyAsync(ctx->ring_dev + o, ctx->ring_host + o, ctx->ring_head - o, hipMemcpyHostToDevice,
                               ctx->stream));
  }
  ctx->ring_pending = ctx->ring_head;
  return SSP_OK;
}

int upload_small(ssp_ctx* ctx, const void* host, size_t bytes, void** dev) {
  const size_t need = (bytes + 255) & ~size_t(255);
  if (need > ctx->ring_cap) {
    // arrays already staged in the old ring keep their addresses: it is retired, not freed
    SSP_TRY(flush_uploads(ctx));
    if (ctx->ring_dev || ctx->ring_host) ctx->retired_rings.emplace_back(ctx->ring_dev, ctx->ring_host);
    ctx->ring_dev = ctx->ring_host = nullptr;
    size_t cap = std::max(need * 2, size_t(4) << 20);
    if (hipMalloc(reinterpret_cast<void**>(&ctx->ring_dev), cap) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&ctx->ring_host), cap, hipHostMallocDefault) != hipSuccess)
      return set_error(SSP_ERR_NOMEM, "allocation of upload ring failed");
    ctx->ring_cap = cap;
    ctx->ring_head = ctx->ring_pending = 0;
  }
  if (ctx->ring_head + need > ctx->ring_cap) {
    // Wrap: copy what is staged, then every earlier copy out of the ring has completed once the
    // stream drains.  The staged regions keep their device addresses (the copy lands there).
    SSP_TRY(flush_uploads(ctx));
    SSP_TRY(sync_stream(ctx, "upload ring wrap"));
    ctx->ring_head = ctx->ring_pending = 0;
  }
  char* h = ctx->ring_host + ctx->ring_head;
  char* d = ctx->ring_dev + ctx->ring_head;
  ctx->ring_head += need;
  if (bytes) std::memcpy(h, host, bytes);
  *dev = d;
  return SSP_OK;
}

int allreduce_dev(ssp_ctx* ctx, double* buf, size_t n) {
  SSP_TRY(comm_check(ctx));
  if (n == 0) return SSP_OK;
  if (ctx->p2p) return p2p_allreduce_dev(ctx, buf, n);
  if (ctx->host_allreduce && ctx->nranks > 1) {
    // Host-callback communicator: stage through the host (test / fallback transport only).
    std::vector<double> h(n);
    SSP_TRY_HIP(hipMemcpyAsync(h.data(), buf, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    SSP_TRY(sync_stream(ctx, "host allreduce"));
    if (ctx->host_allreduce(h.data(), n, ctx->host_user) != 0)
      return comm_fail(ctx, "host allreduce callback failed (a peer closed or timed out)");
    SSP_TRY_HIP(hipMemcpyAsync(buf, h.data(), n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    SSP_TRY(sync_stream(ctx, "host allreduce"));
    return SSP_OK;
  }
  if (!ctx->comm) return SSP_OK;
  return rccl_settle(ctx, ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, ctx->comm, ctx->stream), "ncclAllReduce");
}

// Every rank of a new communicator takes the smallest exact_max among them (SSP_EXACT_MAX is read per
// process), so that equal shard lengths choose the same arithmetic on every rank.
int agree_exact_max(ssp_ctx* ctx) {
  if (ctx->nranks <= 1) return SSP_OK;
  const unsigned long long mine = ctx->exact_max;
  std::vector<unsigned long long> all(size_t(ctx->nranks));
  SSP_TRY(ssp_allgather_host(ctx, &mine, all.data(), sizeof(mine)));
  ctx->exact_max = size_t(*std::min_element(all.begin(), all.end()));
  return SSP_OK;
}

// The outcome of an RCCL call on the context's communicator: an error aborts it (every later exchange
// fails at once); ncclInProgress (a non-blocking communicator's answer) is waited out under the deadline.
int rccl_settle(ssp_ctx* ctx, ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return SSP_OK;
  if (r != ncclInProgress) return comm_fail(ctx, std::string(what) + ": " + ncclGetErrorString(r));
  const double t0 = now_s();
  ncclResult_t state = ncclInProgress;
  while (ncclCommGetAsyncError(ctx->comm, &state) == ncclSuccess && state == ncclInProgress) {
    if (now_s() - t0 > ctx->comm_timeout_s)
      return comm_fail(ctx, std::string(what) + ": still in progress after SSP_COMM_TIMEOUT_S");
    _mm_pause();
  }
  if (state != ncclSuccess) return comm_fail(ctx, std::string(what) + ": " + ncclGetErrorString(state));
  return SSP_OK;
}

// Publishes n doubles of the device result into coherent host memory (system-scope write-through
// stores), then, once every wave's stores have completed, the sequence number.  One workgroup: n is
// a reduction result (at most a few thousand doubles).
__global__ __launch_bounds__(256) void k_publish(const double* src, size_t n, double* dst,
                                                 unsigned long long* flag, unsigned long long seq) {
  for (size_t i = threadIdx.x; i < n; i += blockDim.x)
    __hip_atomic_store(dst + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Waits until the flag carries `seq`: the kernel that sets it is the last one queued, so every
// operation before it has completed too (stream order).  Polling the flag instead of a D2H copy +
// hipStreamSynchronize cuts the host-visible latency of a reduction (tools/sync_probe.hip,
// profiles/r1/sync_probe.txt).  The stream is queried every few hundred polls so that a failed
// kernel surfaces as an error instead of a hang.  *seen is false when the stream drained without the
// flag becoming visible (the writes of a finished kernel are visible all the same).  With a
// communicator attached the wait is bounded (comm_poll: SSP_COMM_TIMEOUT_S, RCCL's asynchronous
// error, the peer-memory transport's abort word), since the flag then depends on other ranks.
int wait_flag(ssp_ctx* ctx, unsigned long long seq, bool* seen, const char* what, const unsigned long long* flag) {
  if (!flag) flag = ctx->pub_flag;
  *seen = true;
  const bool ranks = comm_attached(ctx);
  const double t0 = ranks ? now_s() : 0.0;
  for (unsigned spin = 1;; ++spin) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) return SSP_OK;
    if ((spin & 255) == 0) {
      const hipError_t e = hipStreamQuery(ctx->stream);
      if (e == hipErrorNotReady) {
        if (ranks && (spin & 4095) == 0) SSP_TRY(comm_poll(ctx, t0, what));
        continue;
      }
      if (e != hipSuccess) return hip_error(e, what);
      *seen = __atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq;
      return SSP_OK;
    }
    _mm_pause();
  }
}

int ensure_async(ssp_ctx* ctx) {
  if (ctx->async_dev) return SSP_OK;
  if (hipMalloc(reinterpret_cast<void**>(&ctx->async_dev), kAsyncResults * sizeof(double)) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&ctx->async_host), kAsyncResults * sizeof(double),
                    hipHostMallocCoherent) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&ctx->async_flag), 64, hipHostMallocCoherent) != hipSuccess)
    return set_error(SSP_ERR_NOMEM, "allocation of the pending-result buffers failed");
  __atomic_store_n(ctx->async_flag, ctx->async_seq, __ATOMIC_RELEASE);
  return SSP_OK;
}

int fetch_result(ssp_ctx* ctx, double* out, size_t n) {
  if (n > ctx->result_cap) return set_error(SSP_ERR_ARG, "fetch_result: result larger than the staging buffer");
  const unsigned long long seq = ++ctx->pub_seq;
  if (ctx->publish_copy) {
    SSP_TRY_HIP(hipMemcpyAsync(ctx->result_host, ctx->result_dev, n * sizeof(double), hipMemcpyDeviceToHost,
                               ctx->stream));
    SSP_TRY_HIP(hipStreamWriteValue64(ctx->stream, ctx->pub_flag, seq, 0));
  } else {
    SSP_LAUNCH(k_publish, dim3(1), dim3(256), 0, ctx->stream, ctx->result_dev, n, ctx->result_host,
                       ctx->pub_flag, seq);
    SSP_TRY_HIP(hipGetLastError());
  }
  bool seen = true;
  SSP_TRY(wait_flag(ctx, seq, &seen));
  if (!seen)
    SSP_TRY_HIP(hipMemcpy(ctx->result_host, ctx->result_dev, n * sizeof(double), hipMemcpyDeviceToHost));
  std::memcpy(out, ctx->result_host, n * sizeof(double));
  return SSP_OK;
}

int reduce_fetch(ssp_ctx* ctx, double* out, size_t n) {
  if (ctx->p2p) return p2p_allreduce_fetch(ctx, ctx->result_dev, out, n);
  SSP_TRY(allreduce_dev(ctx, ctx->result_dev, n));
  return fetch_result(ctx, out, n);
}

int fold_begin(ssp_ctx* ctx, int nout, FoldTail* t) {
  SSP_TRY(comm_check(ctx));
  SSP_TRY(ensure_result(ctx, size_t(nout)));
  t->counter = ctx->fold_counter;
  t->nout = nout;
  t->flag = ctx->pub_flag;
  const bool ranks = comm_attached(ctx);
  if (ranks) {
    t->out = ctx->result_dev;
    t->host = nullptr;
    t->seq = 0;
  } else {
    t->out = nullptr;
    t->host = ctx->result_host;
    t->seq = ++ctx->pub_seq;
  }
  return SSP_OK;
}

int fold_finish(ssp_ctx* ctx, const FoldTail& t, double* out) {
  if (!t.host) return reduce_fetch(ctx, out, size_t(t.nout));
  bool seen = true;
  SSP_TRY(wait_flag(ctx, t.seq, &seen));
  std::memcpy(out, ctx->result_host, size_t(t.nout) * sizeof(double));
  return SSP_OK;
}

namespace {
hipEvent_t take_event(ssp_ctx* ctx) {
  if (!ctx->event_pool.empty()) {
    hipEvent_t e = ctx->event_pool.back();
    ctx->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

int ledger_slot(ssp_ctx* ctx, const char* op) {
  for (size_t i = 0; i < ctx->ledger.size(); ++i)
    if (ctx->ledger[i].name == op) return int(i);
  ctx->ledger.emplace_back();
  ctx->ledger.back().name = op;
  return int(ctx->ledger.size() - 1);
}

int ledger_resolve(ssp_ctx* ctx) {
  SSP_TRY_HIP(hipStreamSynchronize(ctx->stream));
  for (auto& e : ctx->ledger) {
    for (auto& pr : e.pending) {
      float ms = 0;
      SSP_TRY_HIP(hipEventElapsedTime(&ms, pr.first, pr.second));
      e.ms += ms;
      ctx->event_pool.push_back(pr.first);
      ctx->event_pool.push_back(pr.second);
    }
    e.pending.clear();
  }
  return SSP_OK;
}
}  // namespace

namespace {
thread_local LedgerScope* t_scope = nullptr;  // innermost open dispatch-timed scope
}

LedgerScope::LedgerScope(ssp_ctx* ctx, const char* op, double bytes) : ctx_(ctx) {
  if (!ctx->ledger_on) return;
  slot_ = ledger_slot(ctx, op);
  ctx->ledger[slot_].calls += 1;
  ctx->ledger[slot_].bytes += bytes;
  last_bytes_ = bytes;
  start_ = take_event(ctx);
  if (!start_) return;
  if (ctx->ledger_dispatch) {
    stop_ = take_event(ctx);
    if (!stop_) {
      ctx->event_pool.push_back(start_);
      start_ = nullptr;
      return;
    }
    prev_ = t_scope;
    t_scope = this;
    return;
  }
  (void)hipEventRecord(start_, ctx->stream);
}

bool LedgerScope::dispatch_events(hipStream_t stream, hipEvent_t* start, hipEvent_t* stop) {
  LedgerScope* s = t_scope;
  // only a launch on the open scope's own context stream carries its events (a kernel of another
  // context launched from this thread inside the scope keeps a plain launch)
  if (!s || stream != s->ctx_->stream) return false;
  *start = s->launched_ ? nullptr : s->start_;
  *stop = s->stop_;
  s->launched_ = true;
  return true;
}

void LedgerScope::detail(const std::string& tag) {
  if (slot_ < 0 || !ctx_->ledger_detail) return;
  const std::string name = ctx_->ledger[slot_].name + " [" + tag + "]";
  auto& from = ctx_->ledger[slot_];
  from.calls -= 1;
  const double b = last_bytes_;
  from.bytes -= b;
  const int to = ledger_slot(ctx_, name.c_str());
  ctx_->ledger[to].calls += 1;
  ctx_->ledger[to].bytes += b;
  slot_ = to;
}

LedgerScope::~LedgerScope() {
  if (slot_ < 0 || !start_) return;
  if (stop_) {  // dispatch timing
    t_scope = prev_;
    if (!launched_) {  // no kernel in this op (e.g. its work went to a nested op)
      ctx_->event_pool.push_back(start_);
      ctx_->event_pool.push_back(stop_);
      return;
    }
    ctx_->ledger[slot_].pending.emplace_back(start_, stop_);
  } else {
    hipEvent_t end = take_event(ctx_);
    if (!end) return;
    (void)hipEventRecord(end, ctx_->stream);
    ctx_->ledger[slot_].pending.emplace_back(start_, end);
  }
  if (ctx_->ledger[slot_].pending.size() > 4096) (void)ledger_resolve(ctx_);
}

}  // namespace ssp

extern "C" {

int ssp_ledger_enable(ssp_ctx* ctx, int enable) {
  SSP_CHECK_CTX(ctx);
  ctx->ledger_on = enable != 0;
  return SSP_OK;
}

int ssp_ledger_reset(ssp_ctx* ctx) {
  SSP_CHECK_CTX(ctx);
  SSP_TRY(ssp::ledger_resolve(ctx));
  ctx->ledger.clear();
  return SSP_OK;
}

int ssp_ledger_reserve(ssp_ctx* ctx, int n) {
  SSP_CHECK_CTX(ctx);
  SSP_TRY(ssp::use_device(ctx));
  while (int(ctx->event_pool.size()) < n) {
    hipEvent_t e = nullptr;
    SSP_TRY_HIP(hipEventCreate(&e));
    ctx->event_pool.push_back(e);
  }
  return SSP_OK;
}

int ssp_ledger_count(ssp_ctx* ctx) {
  if (!ctx) return -1;
  if (ssp::use_device(ctx) != SSP_OK || ssp::ledger_resolve(ctx) != SSP_OK) return -1;
  return int(ctx->ledger.size());
}

int ssp_ledger_entry(ssp_ctx* ctx, int i, const char** name, long long* calls, double* kernel_ms, double* bytes) {
  SSP_CHECK_CTX(ctx);
  SSP_TRY(ssp::ledger_resolve(ctx));
  if (i < 0 || size_t(i) >= ctx->ledger.size()) return ssp::set_error(SSP_ERR_ARG, "ssp_ledger_entry: bad index");
  const auto& e = ctx->ledger[i];
  if (name) *name = e.name.c_str();
  if (calls) *calls = e.calls;
  if (kernel_ms) *kernel_ms = e.ms;
  if (bytes) *bytes = e.bytes;
  return SSP_OK;
}

const char* ssp_last_error(void) { return g_last_error.c_str(); }

const char* ssp_version(void) { return "subspace_hip 0.1 (gfx950, fp64)"; }

int ssp_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int ssp_ctx_create(int device, ssp_ctx** out) {
  if (!out) return ssp::set_error(SSP_ERR_ARG, "ssp_ctx_create: null out");
  *out = nullptr;
  int ndev = 0;
  SSP_TRY_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev)
    return ssp::set_error(SSP_ERR_ARG, "ssp_ctx_create: device " + std::to_string(device) + " not present");
  SSP_TRY_HIP(hipSetDevice(device));
  auto* ctx = new ssp_ctx();
  ctx->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    ctx->num_cus = prop.multiProcessorCount;
  if (const char* rs = std::getenv("SSP_ROW_SHAPE")) ctx->row_stride = std::string(rs) == "stride";
  if (const char* pc = std::getenv("SSP_PUBLISH")) ctx->publish_copy = std::string(pc) == "copy";
  if (const char* ex = std::getenv("SSP_EXACT_MAX")) ctx->exact_max = size_t(std::strtoull(ex, nullptr, 10));
  if (const char* ip = std::getenv("SSP_INNER_PER_CU")) ctx->inner_per_cu = std::max(1, std::atoi(ip));
  if (const char* op = std::getenv("SSP_OUTER_WG_PER_CU")) ctx->outer_per_cu = std::max(1, std::atoi(op));
  if (const char* fp = std::getenv("SSP_FUSED_PER_CU")) ctx->fused_per_cu = std::max(1, std::atoi(fp));
  if (const char* tw = std::getenv("SSP_TRANSFORM_WIDE")) ctx->transform_wide = std::atoi(tw) != 0;
  if (const char* sm = std::getenv("SSP_SELECT_MERGE")) ctx->select_rank = std::string(sm) != "tree";
  if (const char* lt = std::getenv("SSP_LEDGER_TIMING")) ctx->ledger_dispatch = std::string(lt) == "dispatch";
  ctx->ledger_detail = std::getenv("SSP_LEDGER_DETAIL") != nullptr;
  if (const char* ss = std::getenv("SSP_SYNTH_SHAPE")) {
    ctx->synth_stride = std::string(ss) == "stride";
    ctx->synth_window = std::string(ss) == "window";
  }
  if (const char* sm = std::getenv("SSP_SYNTH_MERGE")) ctx->synth_merge = std::atoi(sm) != 0;
  if (const char* ct = std::getenv("SSP_COMM_TIMEOUT_S")) {
    const double v = std::atof(ct);
    if (v > 0) ctx->comm_timeout_s = v;
  }
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return ssp::set_error(SSP_ERR_HIP, "hipStreamCreate failed");
  }
  int s = ssp::ensure_partial(ctx, size_t(1) << 20);
  if (s == SSP_OK) s = ssp::ensure_result(ctx, size_t(1) << 16);
  if (s == SSP_OK) {
    const size_t bytes = sizeof(unsigned) * ssp::kFoldLine * (ssp::kFoldShards + 1);
    if (hipMalloc(reinterpret_cast<void**>(&ctx->fold_counter), bytes) != hipSuccess ||
        hipMemsetAsync(ctx->fold_counter, 0, bytes, ctx->stream) != hipSuccess)
      s = ssp::set_error(SSP_ERR_NOMEM, "allocation of the reduction counter failed");
  }
  if (s != SSP_OK) {
    ssp_ctx_destroy(ctx);
    return s;
  }
  *out = ctx;
  return SSP_OK;
}

int ssp_ctx_destroy(ssp_ctx* ctx) {
  if (!ctx) return SSP_OK;
  (void)hipSetDevice(ctx->device);
  (void)ssp::p2p_detach(ctx);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->comm) ncclCommDestroy(ctx->comm);
  if (ctx->dev_err_host) (void)hipHostFree(ctx->dev_err_host);
  for (auto& e : ctx->ledger)
    for (auto& pr : e.pending) {
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
  for (auto ev : ctx->event_pool) (void)hipEventDestroy(ev);
  for (auto& b : ctx->free_blocks) (void)hipFree(b.second);
  for (auto& b : ctx->live_blocks) (void)hipFree(b.first);
  if (ctx->partial) (void)hipFree(ctx->partial);
  if (ctx->result_dev) (void)hipFree(ctx->result_dev);
  if (ctx->result_host) (void)hipHostFree(ctx->result_host);
  if (ctx->pub_flag) (void)hipHostFree(ctx->pub_flag);
  if (ctx->fold_counter) (void)hipFree(ctx->fold_counter);
  if (ctx->async_dev) (void)hipFree(ctx->async_dev);
  if (ctx->async_host) (void)hipHostFree(ctx->async_host);
  if (ctx->async_flag) (void)hipHostFree(ctx->async_flag);
  if (ctx->synth_mask) (void)hipFree(ctx->synth_mask);
  if (ctx->ring_dev) (void)hipFree(ctx->ring_dev);
  if (ctx->ring_host) (void)hipHostFree(ctx->ring_host);
  for (auto& r : ctx->retired_rings) {
    if (r.first) (void)hipFree(r.first);
    if (r.second) (void)hipHostFree(r.second);
  }
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return SSP_OK;
}

void* ssp_ctx_stream(ssp_ctx* ctx) { return ctx ? reinterpret_cast<void*>(ctx->stream) : nullptr; }

int ssp_synchronize(ssp_ctx* ctx) {
  SSP_CHECK_CTX(ctx);
  return ssp::sync_stream(ctx, "synchronize");
}

int ssp_alloc(ssp_ctx* ctx, size_t n, double** out) {
  SSP_CHECK_CTX(ctx);
  if (!out) return ssp::set_error(SSP_ERR_ARG, "ssp_alloc: null out");
  const size_t bytes = round_block(std::max<size_t>(n, 1) * sizeof(double));
  auto it = ctx->free_blocks.find(bytes);
  void* p = nullptr;
  if (it != ctx->free_blocks.end()) {
    p = it->second;
    ctx->free_blocks.erase(it);
    ctx->bytes_cached -= bytes;
  } else {
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) {
      // Release the cache and retry once before reporting exhaustion.
      (void)hipGetLastError();
      (void)hipStreamSynchronize(ctx->stream);
      for (auto& b : ctx->free_blocks) (void)hipFree(b.second);
      ctx->free_blocks.clear();
      ctx->bytes_cached = 0;
      if (hipMalloc(&p, bytes) != hipSuccess) {
        (void)hipGetLastError();
        return ssp::set_error(SSP_ERR_NOMEM, "ssp_alloc: out of HBM for " + std::to_string(bytes) + " bytes");
      }
    }
  }
  ctx->live_blocks[p] = bytes;
  ctx->bytes_in_use += bytes;
  *out = static_cast<double*>(p);
  return SSP_OK;
}

int ssp_free(ssp_ctx* ctx, double* p) {
  if (!p) return SSP_OK;
  SSP_CHECK_CTX(ctx);
  auto it = ctx->live_blocks.find(p);
  if (it == ctx->live_blocks.end()) return ssp::set_error(SSP_ERR_ARG, "ssp_free: pointer not from ssp_alloc");
  // Stream-ordered reuse: a later ssp_alloc on the same stream can only be used by work queued
  // after every op that touched this block, so no synchronisation is needed here.
  ctx->free_blocks.emplace(it->second, p);
  ctx->bytes_cached += it->second;
  ctx->bytes_in_use -= it->second;
  ctx->live_blocks.erase(it);
  return SSP_OK;
}

int ssp_release_cached(ssp_ctx* ctx) {
  SSP_CHECK_CTX(ctx);
  SSP_TRY_HIP(hipStreamSynchronize(ctx->stream));
  for (auto& b : ctx->free_blocks) SSP_TRY_HIP(hipFree(b.second));
  ctx->free_blocks.clear();
  ctx->bytes_cached = 0;
  return SSP_OK;
}

int ssp_memory_stats(ssp_ctx* ctx, size_t* in_use, size_t* cached) {
  if (!ctx) return ssp::set_error(SSP_ERR_ARG, "null ssp_ctx");
  if (in_use) *in_use = ctx->bytes_in_use;
  if (cached) *cached = ctx->bytes_cached;
  return SSP_OK;
}

int ssp_upload(ssp_ctx* ctx, double* dst, const double* src, size_t n) {
  SSP_CHECK_CTX(ctx);
  if (n == 0) return SSP_OK;
  SSP_TRY_HIP(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  SSP_TRY_HIP(hipStreamSynchronize(ctx->stream));
  return SSP_OK;
}

int ssp_download(ssp_ctx* ctx, double* dst, const double* src, size_t n) {
  SSP_CHECK_CTX(ctx);
  if (n == 0) return SSP_OK;
  SSP_TRY_HIP(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  SSP_TRY_HIP(hipStreamSynchronize(ctx->stream));
  return SSP_OK;
}

int ssp_comm_unique_id(char* id_out) {
  if (!id_out) return ssp::set_error(SSP_ERR_ARG, "ssp_comm_unique_id: null buffer");
  static_assert(sizeof(ncclUniqueId) == SSP_UNIQUE_ID_BYTES, "unexpected ncclUniqueId size");
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return ssp::set_error(SSP_ERR_COMM, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  std::memcpy(id_out, &id, sizeof(id));
  return SSP_OK;
}

namespace {
// Set when a join is abandoned at its deadline: its helper thread stays blocked in RCCL's bootstrap
// (holding its socket and a device context), and a second bootstrap beside it in the same process is
// not something RCCL supports -- so no RCCL attach is attempted again in this process.
std::atomic<bool> g_rccl_join_abandoned{false};
}  // namespace

int ssp_ctx_attach_comm(ssp_ctx* ctx, int nranks, int rank, const char* id) {
  SSP_CHECK_CTX(ctx);
  if (nranks < 1 || rank < 0 || rank >= nranks || !id) return ssp::set_error(SSP_ERR_ARG, "ssp_ctx_attach_comm: bad rank");
  if (g_rccl_join_abandoned.load())
    return ssp::set_error(SSP_ERR_COMM_ABANDONED,
                          "ssp_ctx_attach_comm: an earlier RCCL join of this process was abandoned; end the process "
                          "(or attach the host-callback / peer-memory transport) -- do not retry RCCL");
  if (ctx->comm) {
    ncclCommDestroy(ctx->comm);
    ctx->comm = nullptr;
  }
  SSP_TRY(ssp::p2p_detach(ctx));
  ctx->host_allreduce = nullptr;
  ctx->host_allgather = nullptr;
  ctx->host_user = nullptr;
  ctx->nranks = nranks;
  ctx->rank = rank;
  ctx->comm_failed = false;
  ctx->comm_fail_msg.clear();
  // A one-rank communicator is created too: its collectives run through RCCL like any other, which
  // is how the RCCL calls are exercised on a one-GPU machine (tests/test_rccl_gpu.py).
  //
  // The join runs on a helper thread and this thread waits for it under the communication deadline
  // (ctx->comm_timeout_s, SSP_COMM_TIMEOUT_S): a rank that never arrives ends the join of the others
  // with SSP_ERR_COMM instead of a wait for ever (the reference aborts the job on a distributed error,
  // DistrArray.cpp:16-23).  RCCL's init blocks in its bootstrap until every rank has checked in, and
  // its non-blocking form (ncclConfig_t blocking = 0) does too (measured on the MI355X boxes:
  // tools/rccl_alone_probe.py, profiles/r5/rccl_alone_probe.txt), so the deadline cannot be polled from
  // inside RCCL.  The abandoned helper keeps the join's state alive on the heap; if the missing ranks
  // ever arrive it aborts the late communicator itself.  The process is then marked: every later RCCL
  // attach returns SSP_ERR_COMM_ABANDONED (bench.py falls back to the host hub on every rank).
  struct Join {
    std::mutex m;
    std::condition_variable cv;
    bool done = false, abandoned = false;
    ncclComm_t comm = nullptr;
    ncclResult_t r = ncclSuccess;
    ncclUniqueId uid;
    int nranks = 0, rank = 0, device = 0;
  };
  static const bool trace = std::getenv("SSP_COMM_TRACE") != nullptr;  // stage lines on stderr
  auto say = [&](const char* what) {
    if (trace) std::fprintf(stderr, "[ssp comm rank %d/%d %.3f] %s\n", rank, nranks, ssp::now_s(), what);
  };
  auto job = std::make_shared<Join>();
  std::memcpy(&job->uid, id, sizeof(job->uid));
  job->nranks = nranks;
  job->rank = rank;
  job->device = ctx->device;
  say("ncclCommInitRank (helper thread)");
  try {
    std::thread([job] {
      ncclComm_t c = nullptr;
      ncclResult_t r = hipSetDevice(job->device) == hipSuccess ? ncclCommInitRank(&c, job->nranks, job->uid, job->rank)
                                                                : ncclInvalidUsage;
      std::lock_guard<std::mutex> lk(job->m);
      job->comm = c;
      job->r = r;
      job->done = true;
      if (job->abandoned && c) ncclCommAbort(c);
      job->cv.notify_all();
    }).detach();
  } catch (const std::exception& e) {
    return ssp::set_error(SSP_ERR_COMM, std::string("ssp_ctx_attach_comm: no helper thread: ") + e.what());
  }
  std::unique_lock<std::mutex> lk(job->m);
  const auto limit = std::chrono::duration<double>(ctx->comm_timeout_s);
  if (!job->cv.wait_for(lk, limit, [&] { return job->done; })) {
    job->abandoned = true;
    g_rccl_join_abandoned.store(true);
    say("deadline: join abandoned");
    char t[64];
    std::snprintf(t, sizeof(t), "%g", ctx->comm_timeout_s);
    return ssp::set_error(SSP_ERR_COMM_ABANDONED,
                          std::string("ncclCommInitRank: rank ") + std::to_string(rank) + " of " + std::to_string(nranks) +
                              ": the communicator did not form within " + t +
                              " s (SSP_COMM_TIMEOUT_S): another rank is missing; the join is abandoned (no further "
                              "RCCL attach in this process)");
  }
  say("joined");
  if (job->r != ncclSuccess) {
    if (job->comm) ncclCommAbort(job->comm);
    return ssp::set_error(SSP_ERR_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(job->r));
  }
  ctx->comm = job->comm;
  return ssp::agree_exact_max(ctx);
}

int ssp_ctx_attach_host_comm(ssp_ctx* ctx, int nranks, int rank, ssp_host_allreduce_fn allreduce,
                             ssp_host_allgather_fn allgather, void* user) {
  SSP_CHECK_CTX(ctx);
  if (nranks < 1 || rank < 0 || rank >= nranks) return ssp::set_error(SSP_ERR_ARG, "ssp_ctx_attach_host_comm: bad rank");
  if (nranks > 1 && (!allreduce || !allgather))
    return ssp::set_error(SSP_ERR_ARG, "ssp_ctx_attach_host_comm: null callback");
  if (ctx->comm) {
    ncclCommDestroy(ctx->comm);
    ctx->comm = nullptr;
  }
  SSP_TRY(ssp::p2p_detach(ctx));
  ctx->comm_failed = false;
  ctx->comm_fail_msg.clear();
  ctx->nranks = nranks;
  ctx->rank = rank;
  ctx->host_allreduce = allreduce;
  ctx->host_allgather = allgather;
  ctx->host_user = user;
  return ssp::agree_exact_max(ctx);
}

int ssp_shard_range(size_t n, int nranks, int rank, size_t* offset, size_t* length) {
  if (nranks < 1 || rank < 0 || rank >= nranks || !offset || !length)
    return ssp::set_error(SSP_ERR_ARG, "ssp_shard_range: bad arguments");
  // make_distribution_spread_remainder (reference util/Distribution.h:99-109).
  const size_t p = size_t(nranks), r = size_t(rank);
  const size_t block = n / p, extra = n % p;
  *offset = r * block + std::min(r, extra);
  *length = block + (r < extra ? 1 : 0);
  return SSP_OK;
}

int ssp_ctx_rank(ssp_ctx* ctx) { return ctx ? ctx->rank : -1; }
int ssp_ctx_nranks(ssp_ctx* ctx) { return ctx ? ctx->nranks : 0; }

int ssp_allreduce_sum(ssp_ctx* ctx, double* buf, size_t n) {
  SSP_CHECK_CTX(ctx);
  SSP_TRY(ssp::allreduce_dev(ctx, buf, n));
  return ssp::sync_stream(ctx, "allreduce");
}

int ssp_allgather_host(ssp_ctx* ctx, const void* send, void* recv, size_t bytes) {
  SSP_CHECK_CTX(ctx);
  SSP_TRY(ssp::comm_check(ctx));
  if (ctx->p2p) return ssp::p2p_allgather_host(ctx, send, recv, bytes);
  if (ctx->host_allgather && ctx->nranks > 1) {
    if (ctx->host_allgather(send, recv, bytes, ctx->host_user) != 0)
      return ssp::comm_fail(ctx, "host allgather callback failed (a peer closed or timed out)");
    return SSP_OK;
  }
  if (!ctx->comm) {
    if (bytes) std::memcpy(recv, send, bytes);
    return SSP_OK;
  }
  const size_t total = bytes * size_t(ctx->nranks);
  const size_t dbl = (total + 7) / 8;
  SSP_TRY(ssp::ensure_result(ctx, dbl + (bytes + 7) / 8 + 1));
  char* dsend = reinterpret_cast<char*>(ctx->result_dev + dbl + 1);
  char* drecv = reinterpret_cast<char*>(ctx->result_dev);
  SSP_TRY_HIP(hipMemcpyAsync(dsend, send, bytes, hipMemcpyHostToDevice, ctx->stream));
  SSP_TRY(ssp::rccl_settle(ctx, ncclAllGather(dsend, drecv, bytes, ncclChar, ctx->comm, ctx->stream), "ncclAllGather"));
  SSP_TRY_HIP(hipMemcpyAsync(recv, drecv, total, hipMemcpyDeviceToHost, ctx->stream));
  return ssp::sync_stream(ctx, "allgather");
}

}  // extern "C"
