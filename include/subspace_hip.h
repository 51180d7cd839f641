/*
 * subspace_hip.h — C ABI of libsubspace_hip.so, the MI355X (gfx950) implementation of the
 * subspace linear-algebra hot path of molpro::linalg::itsolv.
 *
 * Every entry point replaces one operation of the reference's ArrayHandler interface
 * (reference: src/molpro/linalg/array/ArrayHandler.h:184-222) acting on the LOCAL shard of
 * HBM-resident vectors, plus the MPI_Allreduce the reference's distributed handlers issue
 * after local reductions (src/molpro/linalg/array/util/gemm.h:179-182, DistrArray.cpp:134-136).
 *
 * Conventions:
 *  - All vector arguments are DEVICE pointers (double, FP64) of the calling rank's shard of
 *    length n; they must be 16-byte aligned (ssp_alloc guarantees 256 B).
 *  - Matrices are row-major, as subspace::Matrix is (reference itsolv/subspace/Matrix.h:23):
 *      gemm_inner: out[i*k + j] = <xx[i], yy[j]>            (reference util/gemm.h:267-279)
 *      gemm_outer: yy[j] += sum_i alphas[i*m + j] * xx[i]   (reference util/gemm.h:257-265)
 *  - Ops are ordered on the context's HIP stream.  Ops that return host values (dot,
 *    gemm_inner, select, sparse dot/gemm_inner) synchronise that stream before returning.
 *  - With a communicator attached (ssp_ctx_attach_comm), reductions are summed over ranks with
 *    RCCL allreduce on the same stream, so every rank receives bit-identical results.
 *  - No entry point throws.  Each returns an ssp_status; ssp_last_error() describes the last
 *    failure on the calling thread.  The C++ handler shim maps codes to the reference's
 *    exceptions (ArrayHandlerError, std::out_of_range, std::logic_error).
 */
#ifndef SUBSPACE_HIP_H
#define SUBSPACE_HIP_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  SSP_OK = 0,
  SSP_ERR_SIZE = 1,      /* incompatible vector sizes  -> util::ArrayHandlerError   */
  SSP_ERR_RANGE = 2,     /* matrix/vector count mismatch -> std::out_of_range       */
  SSP_ERR_ARG = 3,       /* invalid argument (null, misaligned, n too large)         */
  SSP_ERR_HIP = 4,       /* HIP runtime failure                                      */
  SSP_ERR_COMM = 5,      /* RCCL failure                                             */
  SSP_ERR_NOMEM = 6,     /* device or pinned allocation failed                      */
  SSP_ERR_UNSUPPORTED = 7, /* operation not defined for these operands -> logic_error */
  SSP_ERR_COMM_ABANDONED = 8 /* an RCCL join of this process was abandoned at its deadline: no further
                                RCCL attach in this process (end it); the host-callback and peer-memory
                                transports stay available */
} ssp_status;

typedef struct ssp_ctx ssp_ctx;

/* ---- context, memory, communicator ------------------------------------------------------ */
const char* ssp_last_error(void);
const char* ssp_version(void);
/* Number of visible HIP devices (0 when no GPU).  Does not create a context. */
int ssp_device_count(void);
int ssp_ctx_create(int device, ssp_ctx** out);
int ssp_ctx_destroy(ssp_ctx* ctx);
/* The hipStream_t all ops of this context run on (for event timing by callers). */
void* ssp_ctx_stream(ssp_ctx* ctx);
int ssp_synchronize(ssp_ctx* ctx);
/* Caching device allocator (HBM arena): Q vectors are created and destroyed every iteration
 * (reference itsolv/subspace/QSpace.h:80-84), so freed blocks are recycled by size. */
int ssp_alloc(ssp_ctx* ctx, size_t n, double** out);
int ssp_free(ssp_ctx* ctx, double* p);
int ssp_release_cached(ssp_ctx* ctx);
int ssp_memory_stats(ssp_ctx* ctx, size_t* bytes_in_use, size_t* bytes_cached);
int ssp_upload(ssp_ctx* ctx, double* dst_dev, const double* src_host, size_t n);
int ssp_download(ssp_ctx* ctx, double* dst_host, const double* src_dev, size_t n);

/* RCCL communicator over one process per GPU.  The id is SSP_UNIQUE_ID_BYTES opaque bytes made
 * by rank 0 with ssp_comm_unique_id and distributed by the caller (e.g. torch.distributed). */
#define SSP_UNIQUE_ID_BYTES 128
int ssp_comm_unique_id(char* id_out);
/* Collective: returns once every rank has joined, SSP_ERR_COMM when RCCL reports the join failed, or
 * SSP_ERR_COMM_ABANDONED when the communicator has not formed within the communication deadline
 * (ssp_ctx_set_comm_timeout; a rank is missing).  An abandoned join leaves its helper thread inside
 * RCCL's bootstrap, so every later ssp_ctx_attach_comm of the process returns SSP_ERR_COMM_ABANDONED at
 * once: do not retry -- end the process, or attach the host-callback / peer-memory transport. */
int ssp_ctx_attach_comm(ssp_ctx* ctx, int nranks, int rank, const char* id);
int ssp_ctx_rank(ssp_ctx* ctx);
int ssp_ctx_nranks(ssp_ctx* ctx);
/* In-place sum over ranks of n doubles in DEVICE memory (no-op without a communicator). */
int ssp_allreduce_sum(ssp_ctx* ctx, double* buf_dev, size_t n);
/* Gather `bytes` host bytes from every rank into recv (nranks*bytes), rank order. */
int ssp_allgather_host(ssp_ctx* ctx, const void* send, void* recv, size_t bytes);
/* Host-callback communicator in place of RCCL: reductions are staged through host memory and
 * handed to the callbacks (return 0 on success).  For transports without RCCL and for testing
 * the sharded path with several ranks on one device.  Replaces any attached RCCL communicator. */
typedef int (*ssp_host_allreduce_fn)(double* buf, size_t n, void* user);
typedef int (*ssp_host_allgather_fn)(const void* send, void* recv, size_t bytes, void* user);
int ssp_ctx_attach_host_comm(ssp_ctx* ctx, int nranks, int rank, ssp_host_allreduce_fn allreduce,
                             ssp_host_allgather_fn allgather, void* user);
/* Peer-memory communicator (no RCCL): the ranks of ONE node exchange reduction partials through
 * IPC-shared device memory (push into every rank's inbox, device-side flag wait, fixed rank-order
 * sum: bit-identical results on every rank) and host data through a POSIX shared-memory segment.
 * Several ranks may share one device.  `id` (SSP_UNIQUE_ID_BYTES, from ssp_p2p_unique_id on rank 0)
 * is distributed by the caller.  Collective: returns once every rank has attached.  At most 16 ranks.
 * Replaces any other communicator. */
int ssp_p2p_unique_id(char* id_out);
int ssp_ctx_attach_p2p(ssp_ctx* ctx, int nranks, int rank, const char* id);
/* Fail fast: every wait that depends on other ranks gives up after `seconds` (default 300, or
 * SSP_COMM_TIMEOUT_S at context creation), and RCCL's asynchronous errors are polled meanwhile; the
 * communicator is then aborted (ncclCommAbort / the peer-memory abort word) and the call, and every
 * later exchange on the context, returns SSP_ERR_COMM naming the operation -- the status-code form of
 * the reference's abort of the whole job on a distributed error (DistrArray.cpp:16-23). */
int ssp_ctx_set_comm_timeout(ssp_ctx* ctx, double seconds);
/* Vectors of at most n local elements (default 2048, or SSP_EXACT_MAX at context creation; 0 turns
 * it off; attaching a communicator gives every rank the smallest value among the ranks, and a later
 * call must pass the same n on every rank) are computed in the reference's own arithmetic: every dot a sequential sum in index order
 * (std::inner_product, ArrayHandlerIterable.h:76-82) and every y = alpha x + y rounded twice (no fused
 * multiply-add, ArrayHandlerIterable.h:65-74), gemm_inner / gemm_outer pairwise in the reference's loop
 * order (util/gemm.h:257-279), fused entry points as their documented unfused sequence.  Results on
 * such vectors are the reference CPU path's bit for bit; longer vectors use the bandwidth kernels.
 * Sharded, the choice is each rank's on its own shard length: when the global length puts the
 * longer shards (make_distribution_spread_remainder lengths differ by one) just above n and the
 * shorter ones at n, the ranks' partials come from both arithmetics -- in the same result layout,
 * summed as always, every rank receiving the same sums -- and the bit-for-bit claim is then void. */
int ssp_ctx_set_exact_max(ssp_ctx* ctx, size_t n);
/* Shard of a global length n owned by `rank` of `nranks` (host only, no context):
 * make_distribution_spread_remainder, reference util/Distribution.h:99-109. */
int ssp_shard_range(size_t n, int nranks, int rank, size_t* offset, size_t* length);

/* Operation ledger (measurement): when enabled, HIP events on the
 * context's stream bracket each hot-path kernel launch and the call's ALGORITHMIC bytes are
 * accumulated per operation name ("gemm_inner", "gemm_outer", "axpy", "dot", ...). */
int ssp_ledger_enable(ssp_ctx* ctx, int enable);
int ssp_ledger_reset(ssp_ctx* ctx);
int ssp_ledger_count(ssp_ctx* ctx);
/* Pre-create n ledger events (2 per recorded op), so that a ledger over a timed region creates none. */
int ssp_ledger_reserve(ssp_ctx* ctx, int n);
int ssp_ledger_entry(ssp_ctx* ctx, int i, const char** name, long long* calls, double* kernel_ms, double* bytes);

/* ---- dense (R x R, Q x Q, R x Q) operations: reference ArrayHandlerIterable.h:46-90,
 *      DistrArray.cpp:43-138 ------------------------------------------------------------- */
/* x[:] = alpha                         reference ArrayHandlerIterable.h:59-63 */
int ssp_fill(ssp_ctx* ctx, double alpha, double* x, size_t n);
/* x[:] *= alpha                        reference ArrayHandlerIterable.h:54-57 */
int ssp_scal(ssp_ctx* ctx, double alpha, double* x, size_t n);
/* x[:] = y[:]                          reference ArrayHandlerIterable.h:48-52 */
int ssp_copy(ssp_ctx* ctx, double* x, const double* y, size_t n);
/* y[:] += alpha * x[:]                 reference ArrayHandlerIterable.h:65-74 */
int ssp_axpy(ssp_ctx* ctx, double alpha, const double* x, double* y, size_t n);
/* *out = sum_ranks <x, y>              reference ArrayHandlerIterable.h:76-82, DistrArray.cpp:124-138 */
int ssp_dot(ssp_ctx* ctx, const double* x, const double* y, size_t n, double* out);
/* out (m x k, row-major) = <xx[i], yy[j]> summed over ranks.
 * reference util/gemm.h:157-184 (distributed) and :267-279 (pairwise default) */
int ssp_gemm_inner(ssp_ctx* ctx, const double* const* xx, int m, const double* const* yy, int k, size_t n,
                   double* out);
/* yy[j] += sum_i alphas[i*m + j] * xx[i], i in [0,k) sources, j in [0,m) destinations.
 * reference util/gemm.h:186-203 (distributed) and :257-265 (pairwise default) */
int ssp_gemm_outer(ssp_ctx* ctx, const double* alphas, const double* const* xx, int k, double* const* yy, int m,
                   size_t n);
/* yy[j] = sum_i alphas[i*m + j] * xx[i]: ssp_fill(0) on every destination followed by ssp_gemm_outer,
 * bit-identical, in one pass that does not read the destinations (construct_solution,
 * reference IterativeSolverTemplate.h:33-65).  k = 0 zero-fills. */
int ssp_gemm_outer_set(ssp_ctx* ctx, const double* alphas, const double* const* xx, int k, double* const* yy, int m,
                       size_t n);
/* Fused modified-Gram-Schmidt step: yy[j] += c[j] * x, then out[j] = <yy[j], z> summed over ranks.
 * Equals ssp_gemm_outer({x} -> yy) followed by ssp_gemm_inner(yy, {z}) with bit-identical yy; one
 * pass over yy (reference propose_rspace.h:430-443 issues them as separate handler calls). */
int ssp_axpy_inner(ssp_ctx* ctx, const double* c, const double* x, double* const* yy, int m, const double* z, size_t n,
                   double* out);
/* Steps of the sequential self-orthonormalisation of the new R vectors (reference
 * propose_rspace.h:450-465: scal(1/|r_i|, r_i); for j > i: r_j -= <r_i, r_j> r_i), fused so that
 * each step is two passes:
 *   ssp_scal_inner:  x *= alpha, then out[j] = <x, yy[j]> summed over ranks   (= ssp_scal then
 *                    ssp_gemm_inner({x}, yy), x bit-identical)                 bytes 8N(2 + m)
 *   ssp_axpy_norm:   yy[j] += c[j] * x, then *out = <yy[0], yy[0]> summed over ranks (= ssp_gemm_outer
 *                    then ssp_dot(yy[0], yy[0]), yy bit-identical)             bytes 8N(1 + 2m) */
int ssp_scal_inner(ssp_ctx* ctx, double alpha, double* x, const double* const* yy, int m, size_t n, double* out);
int ssp_axpy_norm(ssp_ctx* ctx, const double* c, const double* x, double* const* yy, int m, size_t n, double* out);
/* One pass per step of that loop (the HBM handlers' default since round 3):
 *   ssp_axpy_gram:   x_s = x * xs (stored into x when store_x and xs != 1: the scal's one rounding),
 *                    yy[j] += c[j] * x_s, then out[j] = <yy[0], yy[j]> for j < m summed over ranks --
 *                    the Gram row of the next vector to normalise, from which the caller takes its
 *                    norm (out[0]) and the next overlaps <r_{i+1}, r_j> = out[j - i - 1] / |r_{i+1}|
 *                    (= ssp_gemm_outer_scaled({x} -> yy) then ssp_gemm_inner({yy[0]}, yy), yy and x
 *                    bit-identical)                                           bytes 8N(1 + store + 2m) */
int ssp_axpy_gram(ssp_ctx* ctx, const double* c, double* x, double xs, int store_x, double* const* yy, int m,
                  size_t n, double* out);
/* Block transform of m vectors in place (the block self-orthonormalisation of the new R vectors,
 * itsolv_hbm/hbm_handlers.h): x_j <- sum_{i<m} t[i*m + j] (xs_i x_i) for j < m, the outputs of each
 * element formed from its loaded inputs before any is stored (the destinations are the sources), the
 * sum by fused multiply-adds in order i = 0..m-1 (on vectors of at most exact_max elements each
 * product rounded before its add).  With gram != NULL also gram[i*m + j] = <x_i', x_j'> of the new
 * vectors (m x m, symmetric), summed over ranks, in the same pass.  1 <= m <= 8; xs may be null (all 1).
 *                                                                          bytes 16 N m */
int ssp_transform_gram(ssp_ctx* ctx, const double* t, double* const* xx, const double* xs, int m, size_t n,
                       double* gram);
/* The same transform with only the self-dots of the new vectors, norms2[j] = <x_j', x_j'> summed over
 * ranks, formed in the same pass (the M accumulators of the plain kernel's window shape; short
 * vectors: the reference's sequential dots).                               bytes 16 N m */
int ssp_transform_norms(ssp_ctx* ctx, const double* t, double* const* xx, const double* xs, int m, size_t n,
                        double* norms2);
/* Residuals and their norms (construct_residual + update_errors, reference
 * LinearEigensystemDavidson.h:186-192, IterativeSolverTemplate.h:95-102) in one pass:
 *   yy[j] = ys[j] yy[j] + c[j] (xs[j] xx[j])  (= ssp_axpy_scaled per pair, yy bit-identical),
 *   out[j] = <yy[j], yy[j]> summed over ranks.  xs / ys may be null (all 1).   bytes 24N m */
int ssp_axpy_pairs_norm(ssp_ctx* ctx, const double* c, const double* const* xx, const double* xs, double* const* yy,
                        const double* ys, int m, size_t n, double* out);
/* a[v][i] /= (d[i] - shift[v] + 1e-15) for v in [0,nvec)   reference itsolv/IterativeSolver.h:34-55 */
int ssp_precondition(ssp_ctx* ctx, double* const* a, int nvec, const double* d, const double* shift, size_t n);
/* The same with the self-dots of the results, norms2[v] = <a_v', a_v'> summed over ranks, formed in the
 * same pass (short vectors: the reference's sequential dots, as ssp_gemm_inner).  0 <= nvec <= 8.
 *                                                                          bytes 8N (1 + 2 nvec) */
int ssp_precondition_norms(ssp_ctx* ctx, double* const* a, int nvec, const double* d, const double* shift, size_t n,
                           double* norms2);

/* ---- deferred scal (itsolv_hbm/hbm_vec.h, Vec::scale_by): an operand's value is s * (its stored
 *      contents); the kernel multiplies each element by s as it loads it -- the one rounding the
 *      reference's scal loop stores -- so every *_scaled call is bit-identical to ssp_scal(s, v) on
 *      each operand v with s != 1 followed by the unscaled call, without that pass over v (16 bytes
 *      per element).  Scale arrays may be null (all 1).  A read-modify-write destination's scale
 *      (ys) applies to the values read; what is stored is the plain result.  Replaces the separate
 *      scal pass of reference ArrayHandlerIterable.h:54-57 at the call sites of propose_rspace.h:17-28
 *      and :450-465 (normalisation of the new R vectors). ------------------------------------------ */
/* x[:] = alpha * y[:]  (the stored form of a scaled vector whose block is shared) */
int ssp_scal_copy(ssp_ctx* ctx, double alpha, double* x, const double* y, size_t n);
int ssp_axpy_scaled(ssp_ctx* ctx, double alpha, const double* x, double xs, double* y, double ys, size_t n);
int ssp_dot_scaled(ssp_ctx* ctx, const double* x, double xs, const double* y, double ys, size_t n, double* out);
int ssp_gemm_inner_scaled(ssp_ctx* ctx, const double* const* xx, const double* xs, int m, const double* const* yy,
                          const double* ys, int k, size_t n, double* out);
int ssp_gemm_outer_scaled(ssp_ctx* ctx, const double* alphas, const double* const* xx, const double* xs, int k,
                          double* const* yy, const double* ys, int m, size_t n);
int ssp_gemm_outer_set_scaled(ssp_ctx* ctx, const double* alphas, const double* const* xx, const double* xs, int k,
                              double* const* yy, int m, size_t n);
int ssp_gemm_inner_sparse_scaled(ssp_ctx* ctx, const double* const* xx, const double* xs, int m, size_t n,
                                 size_t offset, const size_t* ptr, const size_t* idx, const double* val, int k,
                                 double* out);
/* The same m x k sparse inner products split in two: _begin queues them and returns at once, _end
   delivers them to out (m*k doubles).  Other calls may come in between: the subspace update
   (subspace.h new_qspace_data) queues S(R,P)/H(P,R) ahead of the dense overlap rows, so the wait for
   those rows covers both and the sparse product needs no round trip of its own.  One product may be
   pending per context: _begin discards an uncollected one, _end with nothing pending is SSP_ERR_ARG.  With a
   communicator attached (a collective) or beyond the inline limits (m > 64, k > 32, > 64 local
   entries) _begin computes the result at once. */
int ssp_gemm_inner_sparse_begin(ssp_ctx* ctx, const double* const* xx, const double* xs, int m, size_t n,
                                size_t offset, const size_t* ptr, const size_t* idx, const double* val, int k);
int ssp_gemm_inner_sparse_end(ssp_ctx* ctx, double* out);
int ssp_construct_solution_scaled(ssp_ctx* ctx, const double* palphas, const size_t* ptr, const size_t* idx,
                                  const double* val, int kp, const double* alphas, const double* const* xx,
                                  const double* xs, int k, double* const* yy, int m, size_t n, size_t offset);
/* Block update of the block Gram-Schmidt step (itsolv_hbm/rspace.h block_gram_schmidt):
 *   yy[j] = ys[j] yy[j] + sum_i palphas[i*m + j] p_i + sum_s alphas[s*m + j] xs[s] xx[s]
 * bit-identical to ssp_scal(ys) + ssp_gemm_outer_sparse (P) + ssp_gemm_outer (dense sources), in one
 * pass over the destinations (the indices the P vectors touch are recomputed in that order). */
int ssp_block_update(ssp_ctx* ctx, const double* palphas, const size_t* ptr, const size_t* idx, const double* val,
                     int kp, const double* alphas, const double* const* xx, const double* xs, int k, double* const* yy,
                     const double* ys, int m, size_t n, size_t offset);

/* ---- selection: reference util/select.h:28-55, util/select_max_dot.h:166-190,
 *      DistrArray.cpp:170-276.  Local shard [offset, offset+n) of a global array.  Returns up
 *      to nsel (global index, value) pairs in ASCENDING INDEX order (std::map order), chosen
 *      over all ranks with the reference's tie rule (larger index wins a tie). ----------- */
int ssp_select(ssp_ctx* ctx, const double* x, size_t n, size_t offset, size_t nsel, int max, int ignore_sign,
               size_t* idx_out, double* val_out, size_t* nout);
/* Merge of per-rank selections (host only, no context): rank r's count[r] <= stride results are
 * idx/val[r*stride ...] as ssp_select returns them (val = x, |x| or |x*y|).  Keeps the nsel
 * largest (v', index) pairs, v' = max ? val : -val, ties to the larger index, and returns them
 * ordered by index -- the reference heap's result (util/select.h:28-55).  ssp_select and
 * ssp_select_max_dot (max = 1) merge their all-gathered candidates with this function. */
int ssp_select_merge(int nranks, const size_t* counts, size_t stride, const size_t* idx, const double* val,
                     size_t nsel, int max, size_t* idx_out, double* val_out, size_t* nout);
int ssp_select_max_dot(ssp_ctx* ctx, const double* x, const double* y, size_t n, size_t offset, size_t nsel,
                       size_t* idx_out, double* val_out, size_t* nout);

/* ---- dense x sparse (R x P): P = std::map<size_t,double>, passed as sorted global indices.
 *      reference ArrayHandlerIterableSparse.h:35-58, util/gemm.h:207-253,
 *      DistrArray.cpp:419-465.  Entries outside [offset, offset+n) are ignored. ---------- */
/* x = 0 then x[idx-offset] = val */
int ssp_sparse_copy(ssp_ctx* ctx, double* x, size_t n, size_t offset, const size_t* idx, const double* val,
                    size_t nnz);
/* x[idx-offset] += alpha * val */
int ssp_sparse_axpy(ssp_ctx* ctx, double alpha, const size_t* idx, const double* val, size_t nnz, double* x,
                    size_t n, size_t offset);
/* xx[k][idx-offset] += val over the entries [ptr[k], ptr[k+1]) of each of nvec sparse vectors (one
 * ssp_sparse_axpy(1.0) per vector, in one launch for up to 16 vectors and 256 local entries). */
int ssp_sparse_axpy_batch(ssp_ctx* ctx, int nvec, const size_t* ptr, const size_t* idx, const double* val,
                          double* const* xx, size_t n, size_t offset);
/* *out = sum_ranks sum_e x[idx_e-offset] * val_e */
int ssp_sparse_dot(ssp_ctx* ctx, const double* x, size_t n, size_t offset, const size_t* idx, const double* val,
                   size_t nnz, double* out);
/* out (m x k) = <xx[i], p_j>; p_j = entries [ptr[j], ptr[j+1]) of (idx, val). */
int ssp_gemm_inner_sparse(ssp_ctx* ctx, const double* const* xx, int m, size_t n, size_t offset, const size_t* ptr,
                          const size_t* idx, const double* val, int k, double* out);
/* yy[j] += sum_i alphas[i*m + j] * p_i; p_i = entries [ptr[i], ptr[i+1]). */
int ssp_gemm_outer_sparse(ssp_ctx* ctx, const double* alphas, const size_t* ptr, const size_t* idx,
                          const double* val, int k, double* const* yy, int m, size_t n, size_t offset);

/* construct_solution (reference IterativeSolverTemplate.h:33-65: fill(0), then gemm_outer over the
 * P, Q and D spaces) in one pass that does not read the destinations:
 *   yy[j] = sum_i palphas[i*m + j] p_i  +  sum_s alphas[s*m + j] xx[s]
 * with P = CSR (ptr, idx, val) of kp sparse vectors (global indices), bit-identical to
 * ssp_fill(0) + ssp_gemm_outer_sparse + ssp_gemm_outer (Q and D sources concatenated). */
int ssp_construct_solution(ssp_ctx* ctx, const double* palphas, const size_t* ptr, const size_t* idx,
                           const double* val, int kp, const double* alphas, const double* const* xx, int k,
                           double* const* yy, int m, size_t n, size_t offset);

/* ---- synthetic problem (harness only; not a reference operation) ----------------------------
 * H = diag(d) + rho * sum_{l<rank} u_l u_l^T, g = global index, u_0 = 1 and for l > 0
 * u_l(g) = +/-1 from a splitmix64 hash of (seed, l, g).  The rank-one (rank=1) case is the
 * matrix of reference test/itsolv/test_rayleigh_quotient.cpp:37-42.  yy[v] = H xx[v].
 * Diagonal families (itsolv_hbm/problems.h SyntheticSpec):
 *   SSPX_DIAG_LINEAR   d_g = 1 + g; sspx_synth_diagonal reports H_gg = 1 + g + rank*rho
 *   SSPX_DIAG_BOUNDED  d_g = 1 + 2 frac(g phi1); sspx_synth_diagonal reports the approximate
 *                      diagonal d_g (1 + alpha (2 frac(g phi2) - 1)) (C5's DIIS preconditioner) */
#define SSPX_DIAG_LINEAR 0
#define SSPX_DIAG_BOUNDED 1
typedef struct {
  double rho;
  int rank;                /* 1..16 */
  unsigned long long seed;
  int diag_kind;           /* SSPX_DIAG_* */
  double alpha;            /* SSPX_DIAG_BOUNDED: preconditioner mismatch */
  double target;           /* NonLinearEquations residual r = H (x - target 1); 0 is read as 1 (the
                              reference test's x = 1) */
} sspx_synth;
int sspx_synth_action(ssp_ctx* ctx, const sspx_synth* spec, const double* const* xx, double* const* yy, int nvec,
                      size_t n, size_t offset);
/* yy[v] = H (xs[v] xx[v]): the action on deferred-scaled parameters (xs may be null) */
int sspx_synth_action_scaled(ssp_ctx* ctx, const sspx_synth* spec, const double* const* xx, const double* xs,
                             double* const* yy, int nvec, size_t n, size_t offset);
/* yy[v] += rho * sum_l w[v*rank + l] u_l */
int sspx_synth_add_lowrank(ssp_ctx* ctx, const sspx_synth* spec, double* const* yy, int nvec, size_t n,
                           size_t offset, const double* w);
int sspx_synth_diagonal(ssp_ctx* ctx, const sspx_synth* spec, double* d, size_t n, size_t offset);
/* The SSPX_DIAG_LINEAR forms of the three calls above. */
int sspx_synthetic_action(ssp_ctx* ctx, const double* const* xx, double* const* yy, int nvec, size_t n,
                          size_t offset, double rho, int rank, unsigned long long seed);
/* yy[v] += rho * sum_l w[v*rank + l] u_l  (the low-rank part of H applied to P-space vectors) */
int sspx_synthetic_add_lowrank(ssp_ctx* ctx, double* const* yy, int nvec, size_t n, size_t offset, double rho,
                               int rank, unsigned long long seed, const double* w);
/* d[g] = H_gg = 1 + g + rank*rho */
int sspx_synthetic_diagonal(ssp_ctx* ctx, double* d, size_t n, size_t offset, double rho, int rank);
/* x[g] = uniform [-1,1) from splitmix64(seed, vec, g): G-independent benchmark data. */
int sspx_fill_random(ssp_ctx* ctx, double* x, size_t n, size_t offset, unsigned long long seed,
                     unsigned long long vec);
/* Test harness: occupies the context's stream for `ms` milliseconds (one workgroup spinning on the
 * device clock; always ends), to exercise the communication deadline. */
int sspx_debug_stall(ssp_ctx* ctx, double ms);
/* y = A x for a dense row-major n_global x n_global matrix A in device memory, local rows
 * [offset, offset+n) of y; x must be the full (gathered) vector.  Used for small fixtures. */
int sspx_dense_action(ssp_ctx* ctx, const double* a, size_t n_global, const double* const* xx, double* const* yy,
                      int nvec, size_t n, size_t offset);

#ifdef __cplusplus
}
#endif
#endif /* SUBSPACE_HIP_H */
