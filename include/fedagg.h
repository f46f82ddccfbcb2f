/*
 * fedagg.h -- C ABI of the MI355X-native FedAvg-family aggregation engine (libfedagg.so).
 *
 * This is the drop-in boundary under the reference's server-side aggregation operator
 * (liuliuliu0605/FedML, python/fedml/; paths below are relative to that directory).  The
 * reference has no native code on this path: every entry point here replaces a Python loop of
 * PyTorch-CPU tensor ops.  Which loop each entry replaces:
 *
 *   fa_weighted_sum / fa_weighted_sum_multi
 *     FA_MODE_MUL_W        ml/aggregator/agg_operator.py:35-54   torch_aggregator, FedAvg/FedProx
 *                          ml/aggregator/agg_operator.py:100-133 SCAFFOLD / Mime (per dict)
 *                          simulation/sp/fedavg/fedavg_api.py:144-159 FedAvgAPI._aggregate
 *                          simulation/mpi/fedavg_seq/FedAvgClientManager.py:67-73 add_client_model
 *                          simulation/nccl/base_framework/LocalAggregator.py:69-83 + params.py:73-82
 *     FA_MODE_MUL_N_DIV_N  simulation/mpi/fedavg/FedAVGAggregator.py:99-116 _fedavg_aggregation_
 *                          simulation/mpi/hierarchical_fl/HierFedAvgCloudAggregator.py:140-172
 *     FA_MODE_SUM          ml/aggregator/agg_operator.py:55-63, 68-77 FedAvg_seq / FedDyn
 *                          simulation/mpi/fedavg_seq/FedAVGAggregator.py:201-236 aggregate
 *   fa_mix
 *                          HierFedAvgCloudAggregator.py:174-195 _pfedavg_mixing_ (dense CSR)
 *                          simulation/sp/decentralized/client_dsgd.py:104-122 (gossip step)
 *                          simulation/sp/decentralized/client_pushsum.py:127-156 (+ post_scale)
 *
 * Arithmetic contract (bit-exact to the reference on the same inputs; pinned by the golden
 * fixtures in tests/golden/): for every element e, clients i = 0..k-1 IN ORDER,
 *   MUL_W:       t_i = op(x_i[e] * c_i)
 *   MUL_N_DIV_N: t_i = op(op(x_i[e] * c_i) / divisor)
 *   SUM:         t_i = x_i[e]
 *   out[e] = t_0;  out[e] = op(out[e] + t_i) for i >= 1
 * op(.) computes in float (FA_DTYPE_F32/BF16/F16/I64-promoted) or double (F64), rounds once to
 * the storage type, and never fuses a multiply with an add.  Coefficients arrive as double
 * (w_i = n_i / N is a Python float) and are cast to the op type, as PyTorch casts a Python
 * scalar operand.  FA_DTYPE_I64 inputs: MUL_W -> float32 output (fp32(x) * fp32(w));
 * MUL_N_DIV_N -> float32 output (fp32((int64)(x * (int64)c)) / fp32(divisor)); SUM -> int64
 * output (two's-complement wrap).
 *
 * Memory: every data pointer is a DEVICE pointer on the context's HIP device, caller-owned
 * (e.g. torch tensors).  Outputs must not alias inputs.  Pointer tables, coefficients and
 * sizes are HOST arrays; the library stages them to the device itself.  Nothing in the hot call
 * allocates once the context's staging slots are warm.  Calls are asynchronous on `hip_stream`
 * (NULL = the null stream); host arrays may be reused as soon as a call returns.
 *
 * Errors: every entry returns FA_OK (0) or a negative fa_status; the library never aborts.
 * fa_strerror(code) names the code; fa_last_error() gives the detail of the calling thread's
 * last failure.  A context is not thread-safe: use one per thread or lock externally.
 */
#ifndef FEDAGG_H
#define FEDAGG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fa_ctx fa_ctx;

enum fa_dtype {
    FA_DTYPE_F32 = 0,
    FA_DTYPE_BF16 = 1,
    FA_DTYPE_F16 = 2,
    FA_DTYPE_F64 = 3,
    FA_DTYPE_I64 = 4
};

enum fa_mode {
    FA_MODE_MUL_W = 0,
    FA_MODE_MUL_N_DIV_N = 1,
    FA_MODE_SUM = 2
};

enum fa_status {
    FA_OK = 0,
    FA_ERR_INVALID = -1,  /* null pointer, k <= 0, n < 0, bad CSR, ...   */
    FA_ERR_DTYPE = -2,    /* dtype/mode combination not supported          */
    FA_ERR_HIP = -3,      /* a HIP runtime call failed (see fa_last_error) */
    FA_ERR_NOMEM = -4,    /* staging allocation failed                     */
    FA_ERR_COMM = -5      /* an RCCL call failed (fedagg_comm.h)           */
};

#define FA_ABI_VERSION 3

/* ABI version of the loaded library (== FA_ABI_VERSION of the header it was built with). */
int fa_abi_version(void);

/* Create a context bound to HIP device `hip_device` (owns pinned + device staging slots). */
int fa_ctx_create(int hip_device, fa_ctx **out);
/* Destroy a context; waits for the calls still using its staging slots. */
int fa_ctx_destroy(fa_ctx *ctx);

/*
 * One flat parameter vector per client:
 *   d_in[i] (i < k): device pointer to n elements of `dtype`; coef[i]: w_i (MUL_W) or n_i
 *   (MUL_N_DIV_N), ignored for SUM (may be NULL then); divisor: N (MUL_N_DIV_N only).
 *   d_out: n elements of the output type (see the contract above).
 * Replaces the per-key inner loop `for i in range(K)` of agg_operator.py:37-44 and its kin.
 */
int fa_weighted_sum(fa_ctx *ctx, int dtype, int mode, int64_t n, int32_t k,
                     const void *const *d_in, const double *coef, double divisor,
                     void *d_out, void *hip_stream);

/*
 * A whole state_dict in ONE launch: `num_segments` tensors (keys) of one dtype.
 *   seg_numel[s]            elements of key s;
 *   d_in[s * k + i]         client i's tensor for key s (device pointer);
 *   d_out[s]                output tensor for key s.
 * Same arithmetic per element as fa_weighted_sum; coef/divisor shared by all keys.
 * Replaces the outer `for k in avg_params.keys()` loop of agg_operator.py:37.
 */
int fa_weighted_sum_multi(fa_ctx *ctx, int dtype, int mode, int32_t num_segments,
                           const int64_t *seg_numel, int32_t k, const void *const *d_in,
                           const double *coef, double divisor, void *const *d_out,
                           void *hip_stream);

/*
 * Tile-interleaved inputs (the ClientArena "tiled" layout, fedml_amd/arena.py): each input is a
 * sequence of FA_TILE_BYTES slots placed `tile_stride` bytes apart, i.e. element e of client i is at
 *   d_in[i] + (e / E) * tile_stride + (e % E) * sizeof(dtype),   E = FA_TILE_BYTES / sizeof(dtype).
 * An arena of `capacity` clients stores tile t of client r at base + (t * capacity + r) * FA_TILE_BYTES,
 * so d_in[i] = base + r_i * FA_TILE_BYTES and tile_stride = capacity * FA_TILE_BYTES: the K slots one
 * workgroup reads are one contiguous run.  tile_stride == FA_TILE_BYTES is a flat input.  Inputs and
 * d_out 16-byte aligned; d_out is flat.  Same arithmetic per element as fa_weighted_sum.
 * Replaces the same loop (agg_operator.py:37-44); the layout is this engine's, not the reference's.
 */
#define FA_TILE_BYTES 4096
int fa_weighted_sum_tiled(fa_ctx *ctx, int dtype, int mode, int64_t n, int32_t k,
                          const void *const *d_in, int64_t tile_stride, const double *coef,
                          double divisor, void *d_out, void *hip_stream);
/* Several element ranges of one tiled arena in ONE launch (e.g. the per-rank slices of a
 * reduce-scatter chunk): segment s has seg_numel[s] elements, client i's input at d_in[s*k + i]
 * (= base + (t0_s * capacity + r_i) * FA_TILE_BYTES for a range starting at tile t0_s), output
 * d_out[s]; every segment shares tile_stride.  Same arithmetic as fa_weighted_sum_tiled. */
int fa_weighted_sum_tiled_multi(fa_ctx *ctx, int dtype, int mode, int32_t num_segments,
                                const int64_t *seg_numel, int32_t k, const void *const *d_in,
                                int64_t tile_stride, const double *coef, double divisor,
                                void *const *d_out, void *hip_stream);

/* A state_dict's float group (dtype F32, BF16, F16 or F64; n elements, inputs d_in[i]) and its
 * int64 group (n_i64 elements, inputs d_in_i64[i]: BatchNorm num_batches_tracked counters, which
 * the reference's `x * w` promotes to float32, agg_operator.py:37-44) reduced in ONE launch; both
 * share k, mode, coef and divisor.  tile_stride / tile_stride_i64: 0 = one flat row per client
 * (as fa_weighted_sum), else the tiled-arena stride (as fa_weighted_sum_tiled).  Outputs: d_out
 * (same dtype as the inputs) and d_out_i64 (float32 for MUL_W / MUL_N_DIV_N,
 * int64 for SUM).  Bit-identical to the two separate launches. */
int fa_weighted_sum_pair(fa_ctx *ctx, int dtype, int mode, int64_t n, int64_t n_i64, int32_t k,
                         const void *const *d_in, const void *const *d_in_i64, int64_t tile_stride,
                         int64_t tile_stride_i64, const double *coef, double divisor, void *d_out,
                         void *d_out_i64, void *hip_stream);
/* The same for a whole state_dict held as separate tensors (fa_weighted_sum_multi's tables, one
 * per group): num_segments float tensors (seg_numel[s], d_in[s*k + i], d_out[s]) and
 * num_segments_i64 int64 tensors (seg_numel_i64, d_in_i64, d_out_i64), one launch.  Replaces the
 * same per-key loop (agg_operator.py:37-44) over a model with BatchNorm counters. */
int fa_weighted_sum_pair_multi(fa_ctx *ctx, int dtype, int mode, int32_t num_segments,
                               const int64_t *seg_numel, int32_t num_segments_i64,
                               const int64_t *seg_numel_i64, int32_t k, const void *const *d_in,
                               const void *const *d_in_i64, const double *coef, double divisor,
                               void *const *d_out, void *const *d_out_i64, void *hip_stream);

/*
 * Two-level (grouped) reduction in one pass, one flat vector per client:
 *   clients [group_ptr[g], group_ptr[g+1]) form group g (group_ptr[0] = 0, group_ptr[G] = k,
 *   groups non-empty); G_g = the ordered `mode` reduction of the group's clients (coef[i],
 *   divisor as in fa_weighted_sum); t_g = G_g (group_mode SUM), op(G_g * group_coef[g]) (MUL_W)
 *   or op(op(G_g * group_coef[g]) / group_divisor[g]) (MUL_N_DIV_N); out = ordered sum of t_g.
 * Bit-identical to the separate launches of each level.  Replaces the reference's two-level
 * loops: hierarchical FL (sp/hierarchical_fl/group.py:60-62 + trainer.py:108-110; the MPI cloud
 * HierFedAvgCloudAggregator.py:140-157 over HierGroup.py:76 edge models) and FedAvg_seq
 * (fedavg_seq/FedAvgClientManager.py:67-73 + FedAVGAggregator.py:201-236).  dtype: F32, BF16,
 * F16, F64.
 */
int fa_weighted_sum_grouped(fa_ctx *ctx, int dtype, int mode, int64_t n, int32_t k,
                            const void *const *d_in, const double *coef, double divisor,
                            int32_t num_groups, const int32_t *group_ptr, int group_mode,
                            const double *group_coef, const double *group_divisor, void *d_out,
                            void *hip_stream);
/* fa_weighted_sum_grouped over tile-interleaved inputs (addressing as fa_weighted_sum_tiled). */
int fa_weighted_sum_grouped_tiled(fa_ctx *ctx, int dtype, int mode, int64_t n, int32_t k,
                                  const void *const *d_in, int64_t tile_stride, const double *coef,
                                  double divisor, int32_t num_groups, const int32_t *group_ptr,
                                  int group_mode, const double *group_coef,
                                  const double *group_divisor, void *d_out, void *hip_stream);

/*
 * FedOpt server step fused into the FedAvg pass (simulation/mpi/fedopt/FedOptAggregator.py:
 * 104-131 with server_optimizer = "sgd"): for every parameter tensor s (fp32) and element e,
 *   avg   = FedAvg of the clients (fa_weighted_sum MUL_W arithmetic, coef[i] = n_i / N)
 *   g     = param - avg                          (the reference's pseudo-gradient)
 *   g     = fma(param, weight_decay, g)          if weight_decay != 0
 *   m     = g (first_step) | fma(g, 1 - dampening, op(m * momentum))     if momentum != 0
 *   g     = nesterov ? fma(m, momentum, g) : m   if momentum != 0
 *   param = fma(g, -lr, param)
 * torch.optim.SGD semantics on CPU tensors (its add(alpha) is a fused multiply-add).  d_param[s]
 * and d_momentum[s] are updated IN PLACE; d_momentum may be NULL when momentum == 0.  Layout of
 * d_in as in fa_weighted_sum_multi.  Buffers that are not parameters (BatchNorm statistics) take
 * the plain average: aggregate them with fa_weighted_sum(_multi).
 */
int fa_fedavg_sgd(fa_ctx *ctx, int32_t num_segments, const int64_t *seg_numel, int32_t k,
                  const void *const *d_in, const double *coef, void *const *d_param,
                  void *const *d_momentum, double lr, double momentum, double dampening,
                  double weight_decay, int nesterov, int first_step, void *hip_stream);
/* fa_fedavg_sgd for ONE flat parameter over tile-interleaved inputs (addressing as
 * fa_weighted_sum_tiled); d_param / d_momentum are flat, 16-byte aligned. */
/*
 * FedOpt with server_optimizer = "rmsprop" (torch.optim.RMSprop, centered=False; the reference's
 * OptRepo passes lr and momentum, alpha = 0.99 and eps = 1e-8 are torch's defaults): per element
 *   g  = param - avg;  g = fma(param, weight_decay, g) if weight_decay != 0
 *   sq = fma((1 - alpha) * g, g, sq * alpha);  den = sqrt(sq) + eps
 *   momentum: m = m * momentum + g / den;  param = fma(m, -lr, param)
 *   else:     param = param + (-lr * g) / den
 * d_square_avg[s] (and d_momentum[s] when momentum != 0) updated in place; first_step treats them
 * as zero (torch's initial state).  The reference's CPU sqrt is MKL-VML (not correctly rounded),
 * so this is within 1e-6 relative of it, not bit-exact.
 */
int fa_fedavg_rmsprop(fa_ctx *ctx, int32_t num_segments, const int64_t *seg_numel, int32_t k,
                      const void *const *d_in, const double *coef, void *const *d_param,
                      void *const *d_square_avg, void *const *d_momentum, double lr, double alpha,
                      double eps, double weight_decay, double momentum, int first_step,
                      void *hip_stream);

int fa_fedavg_sgd_tiled(fa_ctx *ctx, int64_t n, int32_t k, const void *const *d_in,
                        int64_t tile_stride, const double *coef, void *d_param, void *d_momentum,
                        double lr, double momentum, double dampening, double weight_decay,
                        int nesterov, int first_step, void *hip_stream);

/*
 * Mixing / gossip: for every row r < rows, with CSR entries j in [row_ptr[r], row_ptr[r+1]):
 *   d_out[r][e] = ordered MUL_W reduction of d_in[cols[j]][e] * vals[j]   (entry order = CSR order)
 *   if post_scale: d_out2[r][e] = op(d_out[r][e] * post_scale[r])         (PushSum z = x / omega)
 * Dense rows (every column, zeros included, ascending) reproduce _pfedavg_mixing_ exactly, incl.
 * NaN from 0 * Inf; the DSGD row is [self, in-neighbours ascending].  dtype: F32, BF16 or F16.
 * num_in: number of input pointers (cols must be < num_in).  Outputs must not alias inputs.
 */
int fa_mix(fa_ctx *ctx, int dtype, int64_t n, int32_t rows, const int32_t *row_ptr,
           const int32_t *cols, const double *vals, int32_t num_in, const void *const *d_in,
           void *const *d_out, const double *post_scale, void *const *d_out2, void *hip_stream);

/* fa_mix over tile-interleaved inputs and outputs (addressing as fa_weighted_sum_tiled): input i's
 * FA_TILE_BYTES slots are in_tile_stride bytes apart, every output row's (and d_out2's)
 * out_tile_stride bytes apart -- a gossip round between two tiled ClientArenas.  Same arithmetic
 * per element as fa_mix; inputs and outputs 16-byte aligned. */
int fa_mix_tiled(fa_ctx *ctx, int dtype, int64_t n, int32_t rows, const int32_t *row_ptr,
                 const int32_t *cols, const double *vals, int32_t num_in, const void *const *d_in,
                 int64_t in_tile_stride, void *const *d_out, int64_t out_tile_stride,
                 const double *post_scale, void *const *d_out2, void *hip_stream);

/*
 * One PushSum gossip step with the weights on the DEVICE (simulation/sp/decentralized/
 * client_pushsum.py:127-156): fa_mix's rows for the models (x' = ordered CSR sum), the same rows
 * over the float32 weights d_omega_in[num_in] (omega' -> d_omega_out[rows], float32 per-op rounding,
 * the reference's numpy float32 chain), and z = x' * float32(1 / omega') into d_out2 -- the
 * post-scale computed on the device, no host round trip for omega.  Asynchronous on hip_stream.
 */
int fa_pushsum(fa_ctx *ctx, int dtype, int64_t n, int32_t rows, const int32_t *row_ptr, const int32_t *cols,
               const double *vals, int32_t num_in, const void *const *d_in, const float *d_omega_in,
               void *const *d_out, void *const *d_out2, float *d_omega_out, void *hip_stream);

/* Performance tuning only (results are identical for every variant): selects the weighted-sum
 * kernel's shape -- U clients per load group, S 16-byte vectors per lane, load cache policy,
 * double-buffered group prefetch.  0 = default; valid range [0, 9). */
int fa_ctx_set_variant(fa_ctx *ctx, int variant);
/* Performance tuning only: 0 disables the banded sliding-window mixing kernel (fa_mix then always
 * uses the general CSR kernel); default 1. */
int fa_ctx_set_mix_band(fa_ctx *ctx, int enable);

/*
 * A HIP stream restricted to `cu_count` of the device's CUs (spread evenly over the CU mask).
 * Launch the aggregation on it during multi-GPU rounds: the HBM stream saturates with about half
 * of the CUs, and the others stay free for the RCCL collective running beside it.  Destroy with
 * fa_stream_destroy.  Not part of the arithmetic contract.
 */
int fa_stream_create_cu_masked(int hip_device, int cu_count, void **out_stream);
int fa_stream_destroy(void *stream);

/*
 * fa_weighted_sum_multi for HOST-resident inputs and outputs (h_in: nseg*k host pointers,
 * key-major; h_out: nseg host pointers), SYNCHRONOUS: the inputs are packed into one mapped pinned
 * buffer owned by ctx, the kernel reads them and writes the results in place over PCIe (no
 * separate H2D/D2H copies), the call waits for it on hip_stream and copies the results out.
 * Rounds up to 1 MiB whose tables fit the kernel argument (3 KB) run on up to 64 workgroups that
 * end by storing a sequence number into the mapped buffer; the call spins on that word (a second
 * after the launch it falls back to a stream sync, which reports a fault) instead of an event
 * wait.  Replaces the reference loop (agg_operator.py:37-44) for small CPU-resident rounds, where
 * launch and copy latencies dominate (cfg1: LR-MNIST, K = 2, 63 KB per client).  Same
 * arithmetic and bits as fa_weighted_sum_multi.  Calls on one ctx must not overlap (as every
 * entry point: one thread per context at a time).
 */
int fa_weighted_sum_host(fa_ctx *ctx, int dtype, int mode, int32_t num_segments, const int64_t *seg_numel,
                         int32_t k, const void *const *h_in, const double *coef, double divisor,
                         void *const *h_out, void *hip_stream);

/*
 * Cross-dtype accumulation step of the reference's per-key client loop, for clients that disagree
 * on a key's dtype (python/fedml/ml/aggregator/agg_operator.py:37-44 and :55-63: `avg[k] += t` with
 * t = x_i[k] * w_i, or x_i[k], of another dtype than avg[k]):
 *   out[e] = A( C(acc[e]) + C(t[e]) ),  C = torch.promote_types(A, T), added in C's op-math
 *   (float for bf16/f16/f32, double for f64) and rounded to C, then cast to A.
 * Casts are c10's: int64 -> bf16/f16 and f64 -> bf16/f16 round through float32.  acc_dtype A is a
 * float type (F32/BF16/F16/F64); t_dtype T any FA_DTYPE.  out may alias acc.  Asynchronous on
 * hip_stream; 0 or a negative status.
 */
int fa_promote_add(fa_ctx *ctx, int acc_dtype, int t_dtype, int64_t n, const void *d_acc, const void *d_t,
                   void *d_out, void *hip_stream);

/*
 * Measurement only (no arithmetic contract, not an aggregation): streams `bytes` of d_buf (whole
 * FA_TILE_BYTES rows; a remainder is ignored) the way the weighted-sum kernel reads a tiled arena
 * group -- workgroup b reads rows [b R, (b + 1) R), R = rows_per_workgroup, each lane 16 bytes of every
 * row -- with no arithmetic and no output stream (d_word: one device word, written only with
 * vanishing probability).  Its duration gives the box's read ceiling for that pattern on those
 * pages (bench.py measured_read_ceiling).  Asynchronous on hip_stream; 0 or a negative status.
 */
int fa_read_probe(fa_ctx *ctx, const void *d_buf, int64_t bytes, int32_t rows_per_workgroup, void *d_word,
                  void *hip_stream);

/*
 * Arena storage (r06): `bytes` of physically contiguous device memory on ctx's device
 * (hipExtMallocWithFlags(hipDeviceMallocContiguous)), for the client arenas.  The weighted-sum
 * kernel's rate over a 64.5 GB arena depended on the allocation (9.28-10.0 ms per K = 128 x 125 M
 * step on one box, identical translation / L2 / request counters; profiles/r06n-r06q); contiguous
 * allocations ran at the fast end more often.  *d_out = NULL and FA_ERR_HIP when the device has no
 * contiguous range that large (the caller then allocates normally).  Synchronous.
 */
int fa_device_alloc_contiguous(fa_ctx *ctx, int64_t bytes, void **d_out);
/* Frees what fa_device_alloc_contiguous returned (synchronises the device, as hipFree does). */
int fa_device_free(fa_ctx *ctx, void *d_ptr);

/* Static name of a status code. */
const char *fa_strerror(int code);
/* Detail of the calling thread's last error ("" if none). */
const char *fa_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* FEDAGG_H */
