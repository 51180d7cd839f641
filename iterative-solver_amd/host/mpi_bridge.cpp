// Run-time bridge to the caller's MPI library (see mpi_bridge.h).
#include "mpi_bridge.h"

#include <dlfcn.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

namespace molpro::linalg::hbm::mpi {
namespace {

void* sym(void* lib, const char* name) { return dlsym(lib ? lib : RTLD_DEFAULT, name); }

template <class F>
bool load(void* lib, const char* name, F& f) {
  f = reinterpret_cast<F>(sym(lib, name));
  return f != nullptr;
}

// One implementation over either handle type: H = int (MPICH ABI) or void* (Open MPI).
template <class H>
class Impl final : public Bridge {
 public:
  using Comm = H;
  using Dtype = H;
  using Op = H;
  using Info = H;

  // Resolves the entry points; false when one is missing.
  bool open(void* lib) {
    lib_ = lib;
    bool ok = load(lib, "MPI_Initialized", initialized_) && load(lib, "MPI_Finalized", finalized_) &&
              load(lib, "MPI_Init", init_) && load(lib, "MPI_Finalize", finalize_) &&
              load(lib, "MPI_Comm_size", comm_size_) && load(lib, "MPI_Comm_rank", comm_rank_) &&
              load(lib, "MPI_Allreduce", allreduce_) && load(lib, "MPI_Allgather", allgather_) &&
              load(lib, "MPI_Bcast", bcast_) && load(lib, "MPI_Comm_split_type", split_type_) &&
              load(lib, "MPI_Comm_free", comm_free_);
    if (!ok) return false;
    if constexpr (std::is_pointer_v<H>) {
      // Open MPI: handles are the addresses of predefined objects; f2c/c2f are functions
      // (MPI_IN_PLACE is (void*)1, MPI_COMM_TYPE_SHARED the first enumerator).
      ok = load(lib, "MPI_Comm_f2c", f2c_) && load(lib, "MPI_Comm_c2f", c2f_);
      world_ = static_cast<H>(sym(lib, "ompi_mpi_comm_world"));
      self_ = static_cast<H>(sym(lib, "ompi_mpi_comm_self"));
      null_ = static_cast<H>(sym(lib, "ompi_mpi_comm_null"));
      dbl_ = static_cast<H>(sym(lib, "ompi_mpi_double"));
      byte_ = static_cast<H>(sym(lib, "ompi_mpi_byte"));
      sum_ = static_cast<H>(sym(lib, "ompi_mpi_op_sum"));
      info_null_ = static_cast<H>(sym(lib, "ompi_mpi_info_null"));
      in_place_ = reinterpret_cast<void*>(1);
      shared_ = 0;
      return ok && world_ && self_ && null_ && dbl_ && byte_ && sum_ && info_null_;
    } else {
      // MPICH ABI (mpi.h of MPICH 3.x/4.x, Intel MPI, MVAPICH, Cray MPICH): fixed handle values, and
      // MPI_Comm_f2c is the identity macro.
      world_ = 0x44000000;
      self_ = 0x44000001;
      null_ = 0x04000000;
      dbl_ = 0x4c00080b;
      byte_ = 0x4c00010d;
      sum_ = 0x58000003;
      info_null_ = 0x1c000000;
      in_place_ = reinterpret_cast<void*>(-1);
      shared_ = 1;
      return true;
    }
  }

  bool active() override {
    int i = 0, f = 0;
    return initialized_(&i) == 0 && i && finalized_(&f) == 0 && !f;
  }

  bool valid(int64_t fcomm) override {
    if constexpr (std::is_pointer_v<H>) {
      if (fcomm < INT_MIN || fcomm > INT_MAX) return false;
      const Comm c = f2c_(int(fcomm));
      return c != nullptr && c != null_;
    } else {
      // An MPICH handle: kind in bits 30-31 (0 = invalid), object type in bits 26-29 (1 = communicator).
      if (fcomm < 0 || fcomm > 0xffffffffLL) return false;
      const uint32_t h = uint32_t(fcomm);
      return (h >> 30) != 0 && ((h >> 26) & 0xf) == 1;
    }
  }

  int size(int64_t fcomm) override {
    int s = 0;
    return comm_size_(comm(fcomm), &s) == 0 ? s : -1;
  }
  int rank(int64_t fcomm) override {
    int r = 0;
    return comm_rank_(comm(fcomm), &r) == 0 ? r : -1;
  }

  void node(int64_t fcomm, int* node_rank, int* node_size) override {
    Comm local{};
    const Comm c = comm(fcomm);
    int me = 0;
    comm_rank_(c, &me);
    if (split_type_(c, shared_, me, info_null_, &local) != 0) {
      *node_rank = me;
      *node_size = size(fcomm);
      return;
    }
    comm_rank_(local, node_rank);
    comm_size_(local, node_size);
    comm_free_(&local);
  }

  int allreduce_sum(int64_t fcomm, double* buf, size_t n) override {
    const Comm c = comm(fcomm);
    for (size_t off = 0; off < n; off += kMaxCount) {
      const int cnt = int(std::min(kMaxCount, n - off));
      if (allreduce_(in_place_, buf + off, cnt, dbl_, sum_, c) != 0) return 1;
    }
    return 0;
  }

  int allgather(int64_t fcomm, const void* send, void* recv, size_t bytes) override {
    const Comm c = comm(fcomm);
    const int nr = size(fcomm);
    if (nr < 1) return 1;
    if (bytes <= kMaxCount) return allgather_(send, int(bytes), byte_, recv, int(bytes), byte_, c) != 0;
    // Longer contributions go in pieces (MPI counts are int): gather a piece of every rank's
    // contribution, then place it at its offset in each rank's block.
    std::vector<char> piece;
    for (size_t off = 0; off < bytes; off += kMaxCount) {
      const size_t len = std::min(kMaxCount, bytes - off);
      piece.resize(len * size_t(nr));
      if (allgather_(static_cast<const char*>(send) + off, int(len), byte_, piece.data(), int(len), byte_, c) != 0)
        return 1;
      for (int r = 0; r < nr; ++r)
        std::memcpy(static_cast<char*>(recv) + size_t(r) * bytes + off, piece.data() + size_t(r) * len, len);
    }
    return 0;
  }

  int bcast(int64_t fcomm, void* buf, size_t bytes, int root) override {
    if (bytes > kMaxCount) return 1;
    return bcast_(buf, int(bytes), byte_, root, comm(fcomm)) != 0;
  }

  int64_t world() override { return c2f(world_); }
  int64_t self() override { return c2f(self_); }

  int init() override {
    int i = 0;
    if (initialized_(&i) != 0) return 1;
    if (i) return 0;
    if (init_(nullptr, nullptr) != 0) return 1;
    initialized_here_ = true;
    return 0;
  }
  int finalize() override {
    if (!initialized_here_) return 0;
    int f = 0;
    if (finalized_(&f) == 0 && f) return 0;
    initialized_here_ = false;
    return finalize_();
  }

  const char* abi() const override { return std::is_pointer_v<H> ? "Open MPI" : "MPICH"; }

 private:
  static constexpr size_t kMaxCount = size_t(1) << 30;

  Comm comm(int64_t fcomm) {
    if constexpr (std::is_pointer_v<H>)
      return f2c_(int(fcomm));
    else
      return Comm(uint32_t(fcomm));
  }
  int64_t c2f(Comm c) {
    if constexpr (std::is_pointer_v<H>)
      return int64_t(c2f_(c));
    else
      return int64_t(uint32_t(c));
  }

  void* lib_ = nullptr;
  bool initialized_here_ = false;
  int (*initialized_)(int*) = nullptr;
  int (*finalized_)(int*) = nullptr;
  int (*init_)(int*, char***) = nullptr;
  int (*finalize_)() = nullptr;
  int (*comm_size_)(Comm, int*) = nullptr;
  int (*comm_rank_)(Comm, int*) = nullptr;
  int (*allreduce_)(const void*, void*, int, Dtype, Op, Comm) = nullptr;
  int (*allgather_)(const void*, int, Dtype, void*, int, Dtype, Comm) = nullptr;
  int (*bcast_)(void*, int, Dtype, int, Comm) = nullptr;
  int (*split_type_)(Comm, int, int, Info, Comm*) = nullptr;
  int (*comm_free_)(Comm*) = nullptr;
  Comm (*f2c_)(int) = nullptr;
  int (*c2f_)(Comm) = nullptr;
  Comm world_{}, self_{}, null_{};
  Dtype dbl_{}, byte_{};
  Op sum_{};
  Info info_null_{};
  void* in_place_ = nullptr;
  int shared_ = 0;
};

std::unique_ptr<Bridge> make_bridge() {
  // The caller's library: its symbols in the global scope, or (loaded as a dependency of a module
  // opened RTLD_LOCAL, as Python extensions are) one of the usual sonames, already loaded -- never
  // loaded here (RTLD_NOLOAD): a process without MPI has no communicator to bridge.
  void* lib = nullptr;
  if (!sym(nullptr, "MPI_Initialized")) {
    std::vector<std::string> names;
    if (const char* e = std::getenv("ITSOLV_HBM_LIBMPI")) names.emplace_back(e);
    for (const char* n : {"libmpi.so.12", "libmpi.so.40", "libmpi.so", "libmpich.so.12", "libmpi_cray.so.12"})
      names.emplace_back(n);
    for (const auto& n : names)
      if ((lib = dlopen(n.c_str(), RTLD_NOW | RTLD_NOLOAD)) && sym(lib, "MPI_Initialized")) break;
    if (!lib) return nullptr;
  }
  const bool ompi = sym(lib, "ompi_mpi_comm_world") != nullptr;
  if (ompi) {
    auto b = std::make_unique<Impl<void*>>();
    if (b->open(lib)) return b;
  } else {
    auto b = std::make_unique<Impl<int>>();
    if (b->open(lib)) return b;
  }
  return nullptr;
}

// State of the "mpi" transport's host callbacks (ssp_ctx_attach_host_comm).
struct HostLink {
  Bridge* b;
  int64_t fcomm;
};
int link_allreduce(double* buf, size_t n, void* user) {
  auto* l = static_cast<HostLink*>(user);
  return l->b->allreduce_sum(l->fcomm, buf, n);
}
int link_allgather(const void* send, void* recv, size_t bytes, void* user) {
  auto* l = static_cast<HostLink*>(user);
  return l->b->allgather(l->fcomm, send, recv, bytes);
}

void need(int status, const std::string& what) {
  if (status != SSP_OK) throw std::runtime_error("MPI bridge: " + what + ": " + ssp_last_error());
}

}  // namespace

Bridge* bridge() {
  static std::unique_ptr<Bridge> b = make_bridge();
  return b.get();
}

int device_for(int64_t fcomm) {
  Bridge* b = bridge();
  int nr = 0, ns = 1;
  if (b) b->node(fcomm, &nr, &ns);
  const int nd = ssp_device_count();
  return nd > 0 ? nr % nd : 0;
}

namespace {
// One transport, attached collectively: every rank of fcomm takes the same outcome (an exception on
// every rank, with the first failing rank's reason, or success on every rank).
std::shared_ptr<void> attach_one(ssp_ctx* ctx, Bridge* b, int64_t fcomm, const std::string& t, int size, int rank) {
  if (t == "mpi") {
    auto link = std::make_shared<HostLink>(HostLink{b, fcomm});
    need(ssp_ctx_attach_host_comm(ctx, size, rank, link_allreduce, link_allgather, link.get()),
         "ssp_ctx_attach_host_comm");
    return link;
  }
  if (t != "p2p" && t != "rccl")
    throw std::runtime_error("MPI bridge: unknown transport '" + t + "' (ITSOLV_HBM_COMM: mpi, p2p or rccl)");
  int node_rank = 0, node_size = 1;
  b->node(fcomm, &node_rank, &node_size);
  // Every rank must agree on the outcome before the collective attach: a rank that cannot take part
  // would leave the others waiting.
  int reason = 0;
  if (t == "p2p" && node_size != size) reason = 1;                            // p2p is one node
  if (t == "rccl" && node_size > std::max(1, ssp_device_count())) reason = 2;  // RCCL: a device per rank
  double bad = reason ? 1.0 : 0.0;
  if (b->allreduce_sum(fcomm, &bad, 1) != 0) throw std::runtime_error("MPI bridge: MPI_Allreduce failed");
  if (bad > 0)
    throw std::runtime_error(reason == 1 || (reason == 0 && t == "p2p")
                                 ? "MPI bridge: transport p2p needs every rank of the communicator on one node"
                                 : "MPI bridge: transport rccl needs a device per rank on each node (use p2p or mpi)");
  char id[SSP_UNIQUE_ID_BYTES] = {};
  int s = SSP_OK;
  if (rank == 0) s = t == "p2p" ? ssp_p2p_unique_id(id) : ssp_comm_unique_id(id);
  double failed = s == SSP_OK ? 0.0 : 1.0;
  if (b->allreduce_sum(fcomm, &failed, 1) != 0) throw std::runtime_error("MPI bridge: MPI_Allreduce failed");
  if (failed > 0) throw std::runtime_error("MPI bridge: rank 0 could not create the " + t + " communicator id");
  if (b->bcast(fcomm, id, sizeof(id), 0) != 0) throw std::runtime_error("MPI bridge: MPI_Bcast failed");
  const int st = t == "p2p" ? ssp_ctx_attach_p2p(ctx, size, rank, id) : ssp_ctx_attach_comm(ctx, size, rank, id);
  const std::string why = st == SSP_OK ? std::string() : std::string(ssp_last_error());
  // the attach returns on every rank (joined, refused, or at the deadline): agree on its outcome
  double nfail = st == SSP_OK ? 0.0 : 1.0;
  if (b->allreduce_sum(fcomm, &nfail, 1) != 0) throw std::runtime_error("MPI bridge: MPI_Allreduce failed");
  if (nfail > 0)
    throw std::runtime_error("MPI bridge: " + std::string(t == "p2p" ? "ssp_ctx_attach_p2p" : "ssp_ctx_attach_comm") +
                             ": failed on " + std::to_string(int(nfail)) + " rank(s)" + (why.empty() ? "" : ": " + why));
  return nullptr;
}
}  // namespace

std::shared_ptr<void> attach(ssp_ctx* ctx, int64_t fcomm, const char* transport) {
  Bridge* b = bridge();
  if (!b || !b->active()) throw std::runtime_error("MPI bridge: no initialised MPI library in this process");
  if (!b->valid(fcomm)) throw std::runtime_error("MPI bridge: " + std::to_string(fcomm) + " is not a communicator");
  std::string t = transport && *transport ? transport : "";
  if (t.empty()) {
    const char* e = std::getenv("ITSOLV_HBM_COMM");
    t = e && *e ? e : "mpi";
  }
  const int size = b->size(fcomm), rank = b->rank(fcomm);
  if (size < 1 || rank < 0) throw std::runtime_error("MPI bridge: MPI_Comm_size / MPI_Comm_rank failed");
  // A comma-separated preference list ("rccl,mpi"): the first transport every rank could attach.  A
  // failed RCCL join leaves this process unable to try RCCL again (SSP_ERR_COMM_ABANDONED), but the
  // MPI and peer-memory transports attach in the same process.
  std::vector<std::string> prefs;
  for (size_t p0 = 0; p0 <= t.size();) {
    const size_t p1 = std::min(t.find(',', p0), t.size());
    if (p1 > p0) prefs.push_back(t.substr(p0, p1 - p0));
    p0 = p1 + 1;
  }
  if (prefs.empty()) prefs.push_back("mpi");
  for (size_t i = 0;; ++i) {
    try {
      return attach_one(ctx, b, fcomm, prefs[i], size, rank);
    } catch (const std::exception& e) {
      if (i + 1 == prefs.size()) throw;
      if (rank == 0)
        std::fprintf(stderr, "[itsolv_hbm] transport %s unavailable (%s); trying %s\n", prefs[i].c_str(), e.what(),
                     prefs[i + 1].c_str());
    }
  }
}

}  // namespace molpro::linalg::hbm::mpi
