// Fail-fast waits for every transport, and the peer-memory transport (SSP_COMM=p2p).
//
// Fail fast.  The reference aborts the whole job on a distributed error (DistrArray.cpp:16-23,
// error() -> MPI_Abort).  Here every host wait whose completion depends on other ranks -- the
// reduction hand-off (wait_flag), a stream synchronisation with a communicator attached, the host
// all-gather and barrier -- is bounded by ctx->comm_timeout_s (SSP_COMM_TIMEOUT_S, default 300 s) and
// polls RCCL's asynchronous error.  On expiry the communicator is aborted (ncclCommAbort, or the
// shared abort word of the peer-memory transport) and the call returns SSP_ERR_COMM naming the
// operation; every later exchange on the context returns the same error at once.
//
// Peer-memory transport.  The ranks of one node exchange reduction partials through device memory
// they share by IPC (hipIpcGetMemHandle / hipIpcOpenMemHandle), with no RCCL: one workgroup per
// reduction pushes the rank's n partials into every rank's inbox with system-scope stores, raises a
// flag word in each, waits (bounded by a wall-clock deadline on the device) for every rank's flag in
// its own inbox, and sums the inbox in fixed rank order 0..R-1 -- so the result is bit-identical on
// every rank and independent of any library's algorithm choice (the reference's MPI_Allreduce,
// util/gemm.h:179-182, DistrArray.cpp:134-136).  Host data (select's all-gather, barriers) goes
// through a POSIX shared-memory segment.  Processes on ONE device may use it (RCCL refuses two
// ranks on one GPU), which is how the multi-rank device exchange runs on a one-GPU machine.
#include <fcntl.h>
#include <immintrin.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>

#include "ssp_internal.h"

namespace ssp {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int comm_check(ssp_ctx* ctx) {
  if (ctx->comm_failed) return set_error(SSP_ERR_COMM, ctx->comm_fail_msg);
  return SSP_OK;
}

namespace {
constexpr int kP2PMaxRanks = 16;
constexpr size_t kP2PSlot = 8192;              // doubles per (parity, source) inbox slot
constexpr size_t kP2PLine = 128;               // one flag word per source, a line of its own
constexpr size_t kP2PFlags = kP2PLine * kP2PMaxRanks;
constexpr size_t kP2PBytes = kP2PFlags + 2 * kP2PMaxRanks * kP2PSlot * sizeof(double);
constexpr size_t kP2PGather = size_t(64) << 10;  // host bytes per (parity, rank) of one gather round
constexpr unsigned kShmMagic = 0x53535032u;      // "SSP2"

// The shared host segment of one communicator (zero-filled by ftruncate on creation).
struct P2PShm {
  std::atomic<unsigned> attached[kP2PMaxRanks];
  std::atomic<int> abort_plus1;  // 0: running; q + 1: rank q gave up
  std::atomic<unsigned long long> host_seq[kP2PMaxRanks];
  std::atomic<int> vote[kP2PMaxRanks];  // attach self-test: 1 passed, 2 failed
  hipIpcMemHandle_t handle[kP2PMaxRanks];
  char gather[2][kP2PMaxRanks][kP2PGather];
};
static_assert(std::atomic<unsigned long long>::is_always_lock_free, "shared atomics must be lock-free");
}  // namespace

struct P2PComm {
  std::string name;
  P2PShm* shm = nullptr;
  char* buf = nullptr;                   // this rank's exchange buffer (flags + inbox slots)
  char* peer[kP2PMaxRanks] = {};         // every rank's buffer as mapped in this process
  unsigned seq = 0;                      // device exchanges so far
  unsigned long long host_seq = 0;       // host exchanges so far
  unsigned long long timeout_ticks = 0;  // device deadline in wall-clock ticks
};

namespace {
void p2p_mark_abort(ssp_ctx* ctx) {
  if (ctx->p2p && ctx->p2p->shm) {
    int expected = 0;
    ctx->p2p->shm->abort_plus1.compare_exchange_strong(expected, ctx->rank + 1);
  }
}

int p2p_aborted_by(const ssp_ctx* ctx) {
  if (!ctx->p2p || !ctx->p2p->shm) return -1;
  return ctx->p2p->shm->abort_plus1.load(std::memory_order_acquire) - 1;
}
}  // namespace

int comm_fail(ssp_ctx* ctx, const std::string& what) {
  if (!ctx->comm_failed) {
    ctx->comm_failed = true;
    ctx->comm_fail_msg = what + " [rank " + std::to_string(ctx->rank) + " of " + std::to_string(ctx->nranks) +
                         "; communicator aborted, every later exchange on this context fails]";
    if (ctx->comm) {
      ncclCommAbort(ctx->comm);
      ctx->comm = nullptr;
    }
    p2p_mark_abort(ctx);
  }
  return set_error(SSP_ERR_COMM, ctx->comm_fail_msg);
}

int comm_poll(ssp_ctx* ctx, double t0, const char* what) {
  if (ctx->comm) {
    ncclResult_t a = ncclSuccess;
    if (ncclCommGetAsyncError(ctx->comm, &a) == ncclSuccess && a != ncclSuccess && a != ncclInProgress)
      return comm_fail(ctx, std::string(what) + ": RCCL asynchronous error: " + ncclGetErrorString(a));
  }
  const int q = p2p_aborted_by(ctx);
  if (q >= 0 && q != ctx->rank)
    return comm_fail(ctx, std::string(what) + ": rank " + std::to_string(q) + " gave up on the exchange");
  // the peer-memory kernel gives up at the deadline itself and names the missing rank: the host
  // waits a little longer so that report arrives first
  if (now_s() - t0 > ctx->comm_timeout_s + (ctx->p2p ? std::min(5.0, ctx->comm_timeout_s) : 0.0)) {
    char t[64];
    std::snprintf(t, sizeof(t), "%g", ctx->comm_timeout_s);
    return comm_fail(ctx, std::string(what) + ": no completion within " + t +
                              " s (SSP_COMM_TIMEOUT_S): another rank is missing or behind");
  }
  return SSP_OK;
}

int sync_stream(ssp_ctx* ctx, const char* what) {
  if (!comm_attached(ctx)) {
    SSP_TRY_HIP(hipStreamSynchronize(ctx->stream));
    return SSP_OK;
  }
  SSP_TRY(comm_check(ctx));
  const hipError_t q = hipStreamQuery(ctx->stream);  // an idle stream: nothing to wait for
  if (q == hipSuccess) return ctx->p2p ? device_exchange_error(ctx, what) : SSP_OK;
  if (q != hipErrorNotReady) return hip_error(q, what);
  // A stream write of the next sequence number into the coherent host flag, then the bounded host
  // poll of wait_flag (which also queries the stream every few hundred polls): as fast as the
  // reduction hand-off, where a hipStreamQuery loop costs a runtime call per poll.
  const unsigned long long seq = ++ctx->pub_seq;
  SSP_TRY_HIP(hipStreamWriteValue64(ctx->stream, ctx->pub_flag, seq, 0));
  bool seen = true;  // a drained stream without the flag visible is synchronised all the same
  SSP_TRY(wait_flag(ctx, seq, &seen, what));
  // a peer-memory exchange queued before this point that gave up left NaN and its error word
  return ctx->p2p ? device_exchange_error(ctx, what) : SSP_OK;
}

// ---- peer-memory transport ------------------------------------------------------------------

__device__ __forceinline__ unsigned long long* p2p_flag(char* base, int src) {
  return reinterpret_cast<unsigned long long*>(base + kP2PLine * src);
}
__device__ __forceinline__ double* p2p_slot(char* base, unsigned parity, int src) {
  return reinterpret_cast<double*>(base + kP2PFlags) + (size_t(parity) * kP2PMaxRanks + src) * kP2PSlot;
}

struct P2PArgs {
  char* peer[kP2PMaxRanks];
  const double* src;                 // this rank's n partials (device)
  double* dst;                       // device destination (may be src), or null
  double* host_dst;                  // coherent host destination, or null
  unsigned long long* host_flag;     // with host_dst: set to host_seq after the results
  unsigned long long host_seq;
  int* err;                          // coherent host word: 1000 + q missing rank q, 2000 + q size mismatch
  int nranks, me;
  unsigned seq, n;
  unsigned long long timeout_ticks;
};

// One workgroup.  Hand-offs between processes (and, on a node, devices): every payload and flag word
// is a system-scope store, every read of them a system-scope load (the {sc0 sc1 stores and loads both
// sides} form of MI355X_MICROARCH.md §visibility), on uncached exchange memory; each storing wave
// drains its stores before the barrier that precedes the flags.  Inbox slots alternate by parity:
// rank q writes slot (s & 1, q) of this rank again only at exchange s + 2, which needs this rank's
// flag of exchange s + 1, raised after this kernel has read slot (s & 1, q).  A rank may already have
// raised its flag for s + 1 when this rank looks for s, hence the wrap-safe "at least s" test.
__global__ __launch_bounds__(256) void k_p2p_allreduce(const P2PArgs a) {
  __shared__ int s_err;
  const unsigned par = a.seq & 1;
  if (threadIdx.x == 0) s_err = 0;
  for (int q = 0; q < a.nranks; ++q) {
    double* d = p2p_slot(a.peer[q], par, a.me);
    for (unsigned i = threadIdx.x; i < a.n; i += blockDim.x)
      __hip_atomic_store(d + i, a.src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const unsigned long long word = (static_cast<unsigned long long>(a.seq) << 32) | a.n;
  if (threadIdx.x < unsigned(a.nranks))
    __hip_atomic_store(p2p_flag(a.peer[threadIdx.x], a.me), word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (threadIdx.x < 64) {  // wave 0: lane q waits for rank q's flag in this rank's inbox
    const int q = int(threadIdx.x);
    bool done = q >= a.nranks;
    const unsigned long long t0 = static_cast<unsigned long long>(wall_clock64());
    while (true) {
      if (!done) {
        const unsigned long long w =
            __hip_atomic_load(p2p_flag(a.peer[a.me], q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const unsigned ws = unsigned(w >> 32);
        if (int(ws - a.seq) >= 0) {
          done = true;
          if (ws == a.seq && unsigned(w & 0xffffffffu) != a.n) s_err = 2000 + q;
        }
      }
      if (__all(done)) break;
      if (static_cast<unsigned long long>(wall_clock64()) - t0 > a.timeout_ticks) {  // uniform: scalar clock
        if (!done) s_err = 1000 + q;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (s_err) {
    // No sum: the destination gets NaN, so that a consumer on the device cannot take this rank's
    // partials alone for the result; the host finds the error word at its next wait on the stream.
    const double nan = __builtin_nan("");
    for (unsigned i = threadIdx.x; i < a.n; i += blockDim.x) {
      if (a.host_dst)
        __hip_atomic_store(a.host_dst + i, nan, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      else
        a.dst[i] = nan;
    }
    if (threadIdx.x == 0) __hip_atomic_store(a.err, s_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
    for (unsigned i = threadIdx.x; i < a.n; i += blockDim.x) {
      double s = __hip_atomic_load(p2p_slot(a.peer[a.me], par, 0) + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      for (int q = 1; q < a.nranks; ++q)
        s += __hip_atomic_load(p2p_slot(a.peer[a.me], par, q) + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (a.host_dst)
        __hip_atomic_store(a.host_dst + i, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      else
        a.dst[i] = s;
    }
  }
  if (a.host_flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(a.host_flag, a.host_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

namespace {
int ensure_err_word(ssp_ctx* ctx) {
  if (ctx->dev_err_host) return SSP_OK;
  if (hipHostMalloc(reinterpret_cast<void**>(&ctx->dev_err_host), 64, hipHostMallocCoherent) != hipSuccess)
    return set_error(SSP_ERR_NOMEM, "hipHostMalloc of the exchange error word failed");
  __atomic_store_n(ctx->dev_err_host, 0, __ATOMIC_RELEASE);
  return SSP_OK;
}

P2PArgs p2p_args(ssp_ctx* ctx, const double* src, unsigned n) {
  P2PComm* p = ctx->p2p;
  P2PArgs a{};
  for (int q = 0; q < ctx->nranks; ++q) a.peer[q] = p->peer[q];
  a.src = src;
  a.err = ctx->dev_err_host;
  a.nranks = ctx->nranks;
  a.me = ctx->rank;
  a.seq = ++p->seq;
  a.n = n;
  a.timeout_ticks = p->timeout_ticks;
  return a;
}

}  // namespace

int device_exchange_error(ssp_ctx* ctx, const char* what) {
  if (!ctx->dev_err_host) return SSP_OK;
  const int e = __atomic_load_n(ctx->dev_err_host, __ATOMIC_ACQUIRE);
  if (!e) return SSP_OK;
  char t[64];
  std::snprintf(t, sizeof(t), "%g", ctx->comm_timeout_s);
  if (e >= 2000)
    return comm_fail(ctx, std::string(what) + ": rank " + std::to_string(e - 2000) +
                              " entered the same exchange with a different length (mismatched collective)");
  return comm_fail(ctx, std::string(what) + ": rank " + std::to_string(e - 1000) + " did not arrive within " + t +
                            " s (SSP_COMM_TIMEOUT_S)");
}

int p2p_allreduce_dev(ssp_ctx* ctx, double* buf, size_t n) {
  SSP_TRY(comm_check(ctx));
  for (size_t off = 0; off < n; off += kP2PSlot) {
    const unsigned c = unsigned(std::min(kP2PSlot, n - off));
    P2PArgs a = p2p_args(ctx, buf + off, c);
    a.dst = buf + off;
    SSP_LAUNCH(k_p2p_allreduce, dim3(1), dim3(256), 0, ctx->stream, a);
    SSP_TRY_HIP(hipGetLastError());
  }
  return SSP_OK;
}

int p2p_allreduce_fetch(ssp_ctx* ctx, const double* src, double* out, size_t n) {
  SSP_TRY(comm_check(ctx));
  if (n > ctx->result_cap) return set_error(SSP_ERR_ARG, "p2p_allreduce_fetch: result larger than the staging buffer");
  if (n > kP2PSlot) {  // large results: stream-ordered chunks into result_dev, then one hand-off
    if (src != ctx->result_dev)
      SSP_TRY_HIP(hipMemcpyAsync(ctx->result_dev, src, n * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
    SSP_TRY(p2p_allreduce_dev(ctx, ctx->result_dev, n));
    SSP_TRY(fetch_result(ctx, out, n));
    return device_exchange_error(ctx, "p2p allreduce");
  }
  P2PArgs a = p2p_args(ctx, src, unsigned(n));
  a.host_dst = ctx->result_host;
  a.host_flag = ctx->pub_flag;
  a.host_seq = ++ctx->pub_seq;
  SSP_LAUNCH(k_p2p_allreduce, dim3(1), dim3(256), 0, ctx->stream, a);
  SSP_TRY_HIP(hipGetLastError());
  bool seen = true;  // the kernel stores the sums into host memory itself: drained = visible
  SSP_TRY(wait_flag(ctx, a.host_seq, &seen));
  SSP_TRY(device_exchange_error(ctx, "p2p allreduce"));
  std::memcpy(out, ctx->result_host, n * sizeof(double));
  return SSP_OK;
}

// Host all-gather through the shared segment, kP2PGather bytes per round: rank q's chunk of round s
// sits in gather[s & 1][q]; it is rewritten at round s + 2 only after every rank has published s + 1,
// i.e. finished reading round s.  bytes = 0 is a barrier.
int p2p_allgather_host(ssp_ctx* ctx, const void* send, void* recv, size_t bytes) {
  SSP_TRY(comm_check(ctx));
  P2PComm* p = ctx->p2p;
  P2PShm* shm = p->shm;
  const int me = ctx->rank, R = ctx->nranks;
  for (size_t off = 0;; off += kP2PGather) {
    const size_t chunk = std::min(kP2PGather, bytes - std::min(bytes, off));
    const unsigned long long s = ++p->host_seq;
    const int par = int(s & 1);
    if (chunk) std::memcpy(shm->gather[par][me], static_cast<const char*>(send) + off, chunk);
    shm->host_seq[me].store(s, std::memory_order_release);
    const double t0 = now_s();
    for (int q = 0; q < R; ++q)
      for (unsigned spin = 1; shm->host_seq[q].load(std::memory_order_acquire) < s; ++spin) {
        if ((spin & 1023) == 0) SSP_TRY(comm_poll(ctx, t0, bytes ? "p2p allgather" : "p2p barrier"));
        _mm_pause();
      }
    if (chunk)
      for (int q = 0; q < R; ++q) std::memcpy(static_cast<char*>(recv) + size_t(q) * bytes + off, shm->gather[par][q], chunk);
    if (off + chunk >= bytes) break;
  }
  return SSP_OK;
}

int p2p_detach(ssp_ctx* ctx) {
  P2PComm* p = ctx->p2p;
  if (!p) return SSP_OK;
  if (p->shm && !ctx->comm_failed) {
    // Every rank leaves together, so no rank frees its inbox while another still writes into it; a
    // short deadline: a rank that never arrives has already failed.
    const double keep = ctx->comm_timeout_s;
    ctx->comm_timeout_s = std::min(keep, 30.0);
    (void)p2p_allgather_host(ctx, nullptr, nullptr, 0);
    ctx->comm_timeout_s = keep;
  }
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (int q = 0; q < kP2PMaxRanks; ++q)
    if (p->peer[q] && p->peer[q] != p->buf) (void)hipIpcCloseMemHandle(p->peer[q]);
  if (p->buf) (void)hipFree(p->buf);
  if (p->shm) munmap(p->shm, sizeof(P2PShm));
  delete p;
  ctx->p2p = nullptr;
  return SSP_OK;
}

}  // namespace ssp

extern "C" {

int ssp_ctx_set_comm_timeout(ssp_ctx* ctx, double seconds) {
  SSP_CHECK_CTX(ctx);
  if (!(seconds > 0)) return ssp::set_error(SSP_ERR_ARG, "ssp_ctx_set_comm_timeout: seconds must be > 0");
  ctx->comm_timeout_s = seconds;
  if (ctx->p2p) {
    int khz = 0;
    SSP_TRY_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device));
    ctx->p2p->timeout_ticks = static_cast<unsigned long long>(seconds * 1e3 * double(khz));
  }
  return SSP_OK;
}

// Test harness: one workgroup that spins on the device's wall clock for `ms` milliseconds (bounded:
// it always ends), so that a test can hold the stream busy past the communication deadline.
__global__ void k_debug_stall(unsigned long long ticks) {
  const unsigned long long t0 = static_cast<unsigned long long>(wall_clock64());
  while (static_cast<unsigned long long>(wall_clock64()) - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

int sspx_debug_stall(ssp_ctx* ctx, double ms) {
  SSP_CHECK_CTX(ctx);
  if (!(ms >= 0) || ms > 60e3) return ssp::set_error(SSP_ERR_ARG, "sspx_debug_stall: 0 <= ms <= 60000");
  int khz = 0;
  SSP_TRY_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device));
  SSP_LAUNCH(k_debug_stall, dim3(1), dim3(64), 0, ctx->stream,
                     static_cast<unsigned long long>(ms * double(khz)));
  SSP_TRY_HIP(hipGetLastError());
  return SSP_OK;
}

int ssp_p2p_unique_id(char* id_out) {
  if (!id_out) return ssp::set_error(SSP_ERR_ARG, "ssp_p2p_unique_id: null buffer");
  std::random_device rd;
  const unsigned long long r = (static_cast<unsigned long long>(rd()) << 32) ^ rd();
  std::memset(id_out, 0, SSP_UNIQUE_ID_BYTES);
  std::snprintf(id_out, SSP_UNIQUE_ID_BYTES, "/ssp_p2p_%d_%016llx", int(getpid()), r);
  return SSP_OK;
}

int ssp_ctx_attach_p2p(ssp_ctx* ctx, int nranks, int rank, const char* id) {
  using namespace ssp;
  SSP_CHECK_CTX(ctx);
  if (nranks < 1 || nranks > kP2PMaxRanks || rank < 0 || rank >= nranks || !id || id[0] != '/')
    return set_error(SSP_ERR_ARG, "ssp_ctx_attach_p2p: bad rank, rank count (<= 16) or id");
  if (ctx->comm) {
    ncclCommDestroy(ctx->comm);
    ctx->comm = nullptr;
  }
  SSP_TRY(p2p_detach(ctx));
  ctx->host_allreduce = nullptr;
  ctx->host_allgather = nullptr;
  ctx->host_user = nullptr;
  ctx->nranks = nranks;
  ctx->rank = rank;
  ctx->comm_failed = false;
  ctx->comm_fail_msg.clear();
  SSP_TRY(ensure_err_word(ctx));
  __atomic_store_n(ctx->dev_err_host, 0, __ATOMIC_RELEASE);
  auto* p = new P2PComm();
  p->name = std::string(id, strnlen(id, SSP_UNIQUE_ID_BYTES));
  ctx->p2p = p;
  auto fail = [&](int code, const std::string& msg) {
    const std::string m = "ssp_ctx_attach_p2p: " + msg;
    p2p_mark_abort(ctx);
    (void)shm_unlink(p->name.c_str());
    ctx->comm_failed = true;  // detach skips its closing barrier
    p2p_detach(ctx);
    ctx->comm_failed = false;
    ctx->nranks = 1;
    ctx->rank = 0;
    return set_error(code, m);
  };
  const int fd = shm_open(p->name.c_str(), O_CREAT | O_RDWR, 0600);
  if (fd < 0) return fail(SSP_ERR_COMM, "shm_open failed");
  if (ftruncate(fd, sizeof(P2PShm)) != 0) {
    close(fd);
    return fail(SSP_ERR_COMM, "ftruncate of the shared segment failed");
  }
  void* m = mmap(nullptr, sizeof(P2PShm), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (m == MAP_FAILED) return fail(SSP_ERR_COMM, "mmap of the shared segment failed");
  p->shm = static_cast<P2PShm*>(m);
  // Uncached device memory: the inbox is written by other processes (and, on a node, devices), so no
  // L2 may keep a copy of it.
  if (hipExtMallocWithFlags(reinterpret_cast<void**>(&p->buf), kP2PBytes, hipDeviceMallocUncached) != hipSuccess) {
    (void)hipGetLastError();
    p->buf = nullptr;
    return fail(SSP_ERR_NOMEM, "allocation of the exchange buffer failed");
  }
  if (hipMemset(p->buf, 0, kP2PBytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    return fail(SSP_ERR_HIP, "clearing the exchange buffer failed");
  if (hipIpcGetMemHandle(&p->shm->handle[rank], p->buf) != hipSuccess) {
    (void)hipGetLastError();
    return fail(SSP_ERR_HIP, "hipIpcGetMemHandle of the exchange buffer failed");
  }
  p->shm->attached[rank].store(kShmMagic, std::memory_order_release);
  const double t0 = now_s();
  for (int q = 0; q < nranks; ++q)
    while (p->shm->attached[q].load(std::memory_order_acquire) != kShmMagic) {
      if (p->shm->abort_plus1.load() != 0) return fail(SSP_ERR_COMM, "another rank failed to attach");
      if (now_s() - t0 > ctx->comm_timeout_s) return fail(SSP_ERR_COMM, "timed out waiting for the other ranks");
      usleep(100);
    }
  p->peer[rank] = p->buf;
  for (int q = 0; q < nranks; ++q) {
    if (q == rank) continue;
    void* ptr = nullptr;
    if (hipIpcOpenMemHandle(&ptr, p->shm->handle[q], hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      (void)hipGetLastError();
      return fail(SSP_ERR_HIP, "hipIpcOpenMemHandle of rank " + std::to_string(q) + "'s exchange buffer failed");
    }
    p->peer[q] = static_cast<char*>(ptr);
  }
  SSP_TRY(ssp_ctx_set_comm_timeout(ctx, ctx->comm_timeout_s));
  // Every rank has mapped the segment once all pass this barrier; the name is then no longer needed
  // (the mappings stay), so no segment outlives the job even if it is killed.
  const int s = p2p_allgather_host(ctx, nullptr, nullptr, 0);
  if (s != SSP_OK) return fail(s, ssp_last_error());
  if (rank == 0) (void)shm_unlink(p->name.c_str());
  // Self-test: one device exchange of known values (deadline at most 30 s), then a vote through the
  // shared segment -- which needs no device path -- so that every rank reaches the same verdict
  // and a caller can fall back to another transport consistently (bench.py --comm auto).
  const double keep = ctx->comm_timeout_s;
  SSP_TRY(ssp_ctx_set_comm_timeout(ctx, std::min(keep, 30.0)));
  constexpr int kTest = 5;
  double vals[kTest], got[kTest];
  for (int i = 0; i < kTest; ++i) vals[i] = double(rank + 1 + i);
  bool ok = hipMemcpy(ctx->result_dev, vals, sizeof(vals), hipMemcpyHostToDevice) == hipSuccess &&
            p2p_allreduce_fetch(ctx, ctx->result_dev, got, kTest) == SSP_OK;
  for (int i = 0; ok && i < kTest; ++i) ok = got[i] == double(nranks) * (nranks + 1) / 2 + double(nranks) * i;
  p->shm->vote[rank].store(ok ? 1 : 2, std::memory_order_release);
  bool all = true;
  const double tv = now_s();
  for (int q = 0; q < nranks; ++q) {
    int v;
    while ((v = p->shm->vote[q].load(std::memory_order_acquire)) == 0) {
      if (now_s() - tv > ctx->comm_timeout_s + 10) return fail(SSP_ERR_COMM, "self-test vote timed out");
      usleep(50);
    }
    all = all && v == 1;
  }
  if (!all) return fail(SSP_ERR_COMM, "self-test exchange failed on some rank (device path unusable)");
  SSP_TRY(ssp_ctx_set_comm_timeout(ctx, keep));
  return agree_exact_max(ctx);
}

}  // extern "C"
