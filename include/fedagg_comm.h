/*
 * fedagg_comm.h -- the multi-GPU group -> global exchange of libfedagg.so (SURVEY.md §8(b) "the
 * multi-GPU entry takes an RCCL communicator handle", §8(e)).
 *
 * One process per GPU.  Rank r holds client group r and computes its ordered local partial (the
 * group step: any of fedagg.h's weighted-sum forms, described by fa_local_step); the partials are
 * then combined across the GPUs over RCCL / xGMI (the global step), pipelined in chunks so chunk
 * c's transfer runs beside chunk c+1's partial.  The whole step -- every chunk's local launch, the
 * RCCL point-to-point/collective calls and the owners' sums -- is issued by ONE call, with no
 * host round trip per chunk.
 *
 * Replaces (liuliuliu0605/FedML, python/fedml/):
 *   simulation/nccl/base_framework/common.py:196-210  fedml_nccl_reduce (reduce to rank 0)
 *   simulation/nccl/base_framework/common.py:212-228  fedml_nccl_broadcast (the global model out)
 *   simulation/nccl/base_framework/params.py:98-128   add_reduce_param / communicate (per tensor)
 *   simulation/nccl/base_framework/LocalAggregator.py:69-83  simulate_client (the local partial)
 *   simulation/mpi/fedavg_seq/FedAVGAggregator.py:201-236 + FedAvgClientManager.py:67-73 (the
 *     reference's own two-level reduce: worker partials, then an ORDERED sum on the server)
 *   simulation/mpi/hierarchical_fl/HierFedAvgCloudAggregator.py:140-157 (the cloud step over
 *     group models, pre-scaled per group by the local step's group_mode = MUL_N_DIV_N)
 *
 * Communicators: fa_comm_init creates an RCCL communicator (plus a second one split from it, so
 * the delivery of chunk c runs beside the owners' exchange of chunk c+1) from a unique id that the
 * binding distributes (MPI, a TCP store, ...); fa_comm_wrap borrows communicators the binding
 * already owns (e.g. torch ProcessGroupNCCL._comm_ptr()) and never destroys them.  Streams: the
 * local partials and the owners' sums run on the caller's hip_stream (e.g. a CU-masked stream,
 * fa_stream_create_cu_masked); the RCCL calls run on two internal streams of the fa_comm, ordered
 * against it with events; when the call returns, hip_stream is ordered after everything.  Calls
 * are asynchronous; the scratch buffer and the inputs must stay alive until hip_stream reaches
 * that point.  Every rank of the communicator must make the same sequence of calls with the same
 * n, chunks, align, collective and root.  Not thread-safe per fa_comm.
 *
 * Errors: 0 or a negative fa_status (FA_ERR_COMM for an RCCL failure, detail in fa_last_error());
 * the library never aborts.
 */
#ifndef FEDAGG_COMM_H
#define FEDAGG_COMM_H

#include <stdint.h>

#include "fedagg.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fa_comm fa_comm;

#define FA_COMM_ID_BYTES 128

/* The global step's exchange. */
enum fa_exchange {
    /* the full global model on `root`, summed IN RANK ORDER (bit-identical to the ordered sum of
     * the rank partials): chunk [a, b) is split into world-1 consecutive pieces, one per rank other
     * than root ("owners", ascending); every rank sends its partial of piece o to owner o
     * (point-to-point over every xGMI link), owner o sums the world partials in rank order
     * (SUM kernel) into d_out at the piece's place, then sends the piece to root (second
     * communicator).  Non-root ranks' d_out holds only the pieces they summed. */
    FA_XCHG_ORDERED = 0,
    /* the same, every owner's summed piece delivered to EVERY rank (reduce + broadcast) */
    FA_XCHG_ORDERED_ALL = 1,
    /* RCCL reduce (sum) to root, in place in d_out (RCCL's cross-rank order: ~1e-7, not bitwise) */
    FA_XCHG_REDUCE = 2,
    /* RCCL all-reduce (sum), in place in d_out on every rank */
    FA_XCHG_ALL_REDUCE = 3,
    /* RCCL reduce-scatter: rank r's d_out receives S = ceil(n / (world * align)) * align elements,
     * the global model's [r*S, min((r+1)*S, n)) (zero past n); no rank holds the whole model */
    FA_XCHG_REDUCE_SCATTER = 4
};

/* OR'ed into an ordered exchange (fa_group_reduce, fa_group_reduce_scratch_bytes): every rank, root
 * included, owns one of `world` pieces, and a rank's own partial piece goes through RCCL as a self
 * send / receive like everyone else's; each owner sums the received pieces in rank order into a
 * scratch area and the delivery sends them from there (to root, or to every rank, itself
 * included).  Same result bits as without it.  At world 1 it runs the whole exchange -- grouped
 * ncclSend/ncclRecv on both communicators, the event ordering, the owner's SUM, the second stream --
 * through RCCL on one GPU (what a one-GPU box can verify of the N > 1 path). */
#define FA_XCHG_LOOPBACK 0x100

/* The local (group) step whose result is exchanged. */
enum fa_local_kind {
    FA_LOCAL_FLAT = 0,           /* fa_weighted_sum over d_in[i] (n elements each)               */
    FA_LOCAL_TILED = 1,          /* fa_weighted_sum_tiled (tile_stride bytes between 4-KiB tiles)  */
    FA_LOCAL_GROUPED = 2,        /* fa_weighted_sum_grouped (several groups per rank + cloud term) */
    FA_LOCAL_GROUPED_TILED = 3,  /* fa_weighted_sum_grouped_tiled                                  */
    FA_LOCAL_PARTIAL = 4         /* the caller computed the partial already: d_partial (n elements) */
};

typedef struct fa_local_step {
    int32_t kind;                 /* enum fa_local_kind                                          */
    int32_t dtype;                /* input dtype (fa_dtype)                                      */
    int32_t mode;                 /* fa_mode of the client level                                 */
    int32_t k;                    /* clients on this rank (> 0 unless kind == FA_LOCAL_PARTIAL)   */
    const void *const *d_in;      /* k device pointers: client i's element 0                     */
    int64_t tile_stride;          /* TILED kinds: bytes between a client's consecutive tiles      */
    const double *coef;           /* k client coefficients (w_i or n_i), host                     */
    double divisor;               /* client-level divisor (MUL_N_DIV_N)                           */
    int32_t num_groups;           /* GROUPED kinds: groups on this rank                          */
    int32_t group_mode;           /* GROUPED kinds: fa_mode of the group level                   */
    const int32_t *group_ptr;     /* GROUPED kinds: num_groups + 1 client offsets                */
    const double *group_coef;     /* GROUPED kinds: per-group coefficient                        */
    const double *group_divisor;  /* GROUPED kinds: per-group divisor                            */
    const void *d_partial;        /* PARTIAL: this rank's partial, n elements of the partial type */
} fa_local_step;

/* A fresh RCCL unique id (rank 0 calls it and sends the FA_COMM_ID_BYTES bytes to every rank). */
int fa_comm_unique_id(void *id_out, int64_t id_bytes);
/* Create this rank's communicators over `world` ranks (collective: every rank calls it with the
 * same id) on HIP device hip_device. */
int fa_comm_init(int hip_device, int world, int rank, const void *id, fa_comm **out);
/* Borrow existing RCCL communicators (ncclComm_t): comm2 may be NULL (then the delivery shares
 * comm's stream and the pipeline has one RCCL stream).  Not destroyed by fa_comm_destroy. */
int fa_comm_wrap(int hip_device, void *nccl_comm, void *nccl_comm2, fa_comm **out);
/* Release the fa_comm (and the communicators it created); waits for its streams. */
int fa_comm_destroy(fa_comm *comm);
int fa_comm_size(const fa_comm *comm, int *world, int *rank);

/* Output element type of a local step (the partial's and d_out's dtype): int64 inputs under
 * MUL_W / MUL_N_DIV_N give F32, otherwise the input dtype. */
int fa_local_out_dtype(int dtype, int mode);

/*
 * The pipeline's plan, a pure function (the same on every rank): the chunks [chunk_lo[c],
 * chunk_hi[c]) cover [0, n), inner bounds multiples of `align` (>= 1), at most `chunks` of them;
 * for the ordered exchanges chunk c's piece of rank r is [piece_start[c*world + r],
 * + piece_size[c*world + r]) (size 0 for root), consecutive in rank order, inner bounds multiples
 * of `align`.  Arrays hold max_chunks (resp. max_chunks * world) entries; returns the number of
 * chunks (> 0) or a negative status.
 */
int fa_group_plan(int64_t n, int32_t chunks, int32_t align, int32_t world, int32_t root, int32_t max_chunks,
                  int64_t *chunk_lo, int64_t *chunk_hi, int64_t *piece_start, int64_t *piece_size);

/* Buffers of the ordered exchange's point-to-point operations (fa_group_ops). */
enum fa_xchg_buf { FA_XBUF_SEND = 0, FA_XBUF_RECV = 1, FA_XBUF_OUT = 2, FA_XBUF_SUM = 3 };

/* Flags of fa_group_plan_ex / fa_group_ops_ex. */
#define FA_XFLAG_DELIVER_ALL 1 /* FA_XCHG_ORDERED_ALL */
#define FA_XFLAG_LOOPBACK 2    /* FA_XCHG_LOOPBACK: every rank owns a piece, own pieces sent to self */

/*
 * The point-to-point operations rank `rank` issues for chunk `chunk` of the ordered exchanges
 * (phase 0: every rank's partial pieces to the owners, on the first communicator; phase 1: the
 * owners' summed pieces to the root, or to every rank with deliver_all), exactly as
 * fa_group_reduce issues them: op q goes to/from peer[q] (is_send[q]), count[q] elements at
 * offset[q] of buffer buf[q] (FA_XBUF_SEND: this rank's partial, FA_XBUF_RECV: the receive area,
 * rank-major per piece, FA_XBUF_OUT: d_out).  A pure function (no device): a binding or a test
 * can check that every rank's sends meet their peers' receives.  Returns the op count or < 0.
 */
int fa_group_ops(int64_t n, int32_t chunks, int32_t align, int32_t world, int32_t rank, int32_t root, int deliver_all,
                 int32_t phase, int32_t chunk, int32_t max_ops, int32_t *peer, int32_t *is_send, int32_t *buf,
                 int64_t *offset, int64_t *count);
/* The same two with FA_XFLAG_* flags (FA_XBUF_SUM: the owner's summed pieces of a LOOPBACK exchange,
 * this rank's pieces back to back in chunk order). */
int fa_group_plan_ex(int64_t n, int32_t chunks, int32_t align, int32_t world, int32_t root, int32_t flags,
                     int32_t max_chunks, int64_t *chunk_lo, int64_t *chunk_hi, int64_t *piece_start,
                     int64_t *piece_size);
int fa_group_ops_ex(int64_t n, int32_t chunks, int32_t align, int32_t world, int32_t rank, int32_t root,
                    int32_t flags, int32_t phase, int32_t chunk, int32_t max_ops, int32_t *peer, int32_t *is_send,
                    int32_t *buf, int64_t *offset, int64_t *count);

/* Bytes of device scratch fa_group_reduce needs for these arguments (on this rank). */
int fa_group_reduce_scratch_bytes(const fa_comm *comm, int exchange, const fa_local_step *local, int64_t n,
                                  int32_t chunks, int32_t align, int32_t root, int64_t *bytes);

/*
 * The group -> global step: this rank's local partial of elements [0, n) (chunked) and the
 * `exchange` across the communicator's ranks.  align: chunk (and piece) granularity in elements
 * (TILED kinds: a multiple of the input's tile elements, 4096 / sizeof(dtype)); d_out: n elements
 * of fa_local_out_dtype (FA_XCHG_REDUCE_SCATTER: S elements); d_scratch: scratch_bytes of device
 * memory (>= fa_group_reduce_scratch_bytes), not aliasing d_out or the inputs.
 */
int fa_group_reduce(fa_ctx *ctx, fa_comm *comm, int exchange, const fa_local_step *local, int64_t n,
                    int32_t chunks, int32_t align, int32_t root, void *d_out, void *d_scratch,
                    int64_t scratch_bytes, void *hip_stream);

/* Performance accounting (off by default): with timing on, every local-step launch on hip_stream
 * is bracketed by HIP events; fa_comm_local_time waits for them and returns their summed duration
 * (ms) and count since the last reset. */
int fa_comm_set_timing(fa_comm *comm, int enable);
int fa_comm_local_time(fa_comm *comm, int reset, double *ms, int64_t *launches);
/* Point-to-point operations this fa_comm has issued since it was created: counts[0..3] = sends and
 * receives on communicator 1, sends and receives on communicator 2. */
int fa_comm_op_counts(const fa_comm *comm, int64_t *counts);
/* The last exchange operation this fa_comm issued, as text (hang diagnostics); "" if none. */
int fa_comm_last_op(const fa_comm *comm, char *buf, int64_t buf_bytes);

#ifdef __cplusplus
}
#endif

#endif /* FEDAGG_COMM_H */
