// comm.hip -- the multi-GPU group -> global exchange (include/fedagg_comm.h) over RCCL / xGMI.
//
// One call issues a whole step: per chunk the rank's local partial (fedagg.h's launchers on the
// caller's stream), the RCCL traffic (two internal streams, one per communicator) and, for the
// ordered exchanges, the owners' rank-ordered SUM -- all stream-ordered with events, so the host
// never waits inside the step and chunk c's transfer overlaps chunk c+1's partial.
//
// Why point-to-point for the ordered exchange: an 8 x MI355X node is a full xGMI mesh (one link
// per GPU pair).  A ring reduce moves the whole chunk over every ring link in sequence; here every
// rank sends each owner only that owner's 1/(G-1) piece, so all G-1 links of a GPU carry traffic
// at once and the busiest link carries L/(G-1) elements per chunk (DESIGN.md §6 cost model).
// Because every owner sums the G partials of its piece in RANK ORDER with the same SUM kernel as
// the single-GPU path, the result is bit-identical to the oracle's ordered two-level sum
// (reference: simulation/mpi/fedavg_seq/FedAVGAggregator.py:201-236).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "fa_internal.h"
#include "fedagg_comm.h"

using fa_detail::fail;

struct fa_comm {
  int device = 0, world = 1, rank = 0;
  ncclComm_t c1 = nullptr, c2 = nullptr;
  bool owns = false;
  hipStream_t sa = nullptr, sb = nullptr;  // RCCL streams of c1 / c2
  std::vector<hipEvent_t> pool;            // ordering events, reused call after call
  size_t next_ev = 0;
  bool timing = false;
  std::vector<hipEvent_t> tpool;           // timing events (pairs), reused after fa_comm_local_time
  size_t tnext = 0;
  double local_ms = 0.0;
  int64_t launches = 0;
  mutable std::mutex mu;                   // guards last_op (read by a watchdog thread)
  char last_op[192] = {0};
  int64_t nops[2][2] = {{0, 0}, {0, 0}};   // point-to-point ops issued: [communicator][send, recv]
};

namespace {

#define FA_NCCL(call)                                                                          \
  do {                                                                                         \
    ncclResult_t r_ = (call);                                                                  \
    if (r_ != ncclSuccess) return fail(FA_ERR_COMM, "%s: %s", #call, ncclGetErrorString(r_)); \
  } while (0)

int esize(int dtype) {
  switch (dtype) {
    case FA_DTYPE_F32: return 4;
    case FA_DTYPE_BF16: case FA_DTYPE_F16: return 2;
    case FA_DTYPE_F64: case FA_DTYPE_I64: return 8;
    default: return 0;
  }
}

bool nccl_type(int dtype, ncclDataType_t* t) {
  switch (dtype) {
    case FA_DTYPE_F32: *t = ncclFloat32; return true;
    case FA_DTYPE_BF16: *t = ncclBfloat16; return true;
    case FA_DTYPE_F16: *t = ncclFloat16; return true;
    case FA_DTYPE_F64: *t = ncclFloat64; return true;
    case FA_DTYPE_I64: *t = ncclInt64; return true;
    default: return false;
  }
}

void set_op(fa_comm* c, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
void set_op(fa_comm* c, const char* fmt, ...) {
  char buf[sizeof(c->last_op)];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  std::lock_guard<std::mutex> g(c->mu);
  memcpy(c->last_op, buf, sizeof(buf));
}

int event(fa_comm* c, hipEvent_t* out) {
  if (c->next_ev == c->pool.size()) {
    hipEvent_t e;
    FA_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->pool.push_back(e);
  }
  *out = c->pool[c->next_ev++];
  return FA_OK;
}

// `waiter` runs after everything queued on `src` so far.
int order(fa_comm* c, hipStream_t src, hipStream_t waiter) {
  hipEvent_t e;
  int rc = event(c, &e);
  if (rc) return rc;
  FA_HIP(hipEventRecord(e, src));
  FA_HIP(hipStreamWaitEvent(waiter, e, 0));
  return FA_OK;
}

// The same split as fedml_amd/distributed/group_reduce.py: chunk_bounds / split_bounds.
void bounds(int64_t n, int64_t parts, int64_t align, int64_t j, int64_t* lo, int64_t* hi) {
  const int64_t units = (n + align - 1) / align;
  *lo = std::min(n, units * j / parts * align);
  *hi = std::min(n, units * (j + 1) / parts * align);
}

int64_t num_chunks(int64_t n, int32_t chunks, int32_t align) {
  const int64_t units = (n + align - 1) / align;
  return units > 0 ? std::max<int64_t>(1, std::min<int64_t>(chunks, units)) : 1;
}

struct Plan {
  int64_t C = 0;
  std::vector<int64_t> lo, hi, pstart, psize;  // chunk bounds; per chunk x rank pieces
  std::vector<int64_t> roff;                    // per chunk: this rank's piece offset in its pieces
  int64_t mine = 0;                             // elements of all this rank's pieces
};

// loop (FA_XCHG_LOOPBACK): every rank, root included, owns one of `world` pieces.
void make_plan(int64_t n, int32_t chunks, int32_t align, int world, int root, int me, bool loop, Plan* p) {
  p->C = num_chunks(n, chunks, align);
  p->lo.resize(p->C); p->hi.resize(p->C);
  p->pstart.assign(p->C * world, 0); p->psize.assign(p->C * world, 0);
  p->roff.resize(p->C);
  p->mine = 0;
  for (int64_t c = 0; c < p->C; ++c) {
    bounds(n, p->C, align, c, &p->lo[c], &p->hi[c]);
    const int64_t a = p->lo[c], L = p->hi[c] - a;
    for (int r = 0; r < world; ++r) p->pstart[c * world + r] = a;
    int o = 0;
    for (int r = 0; r < world; ++r) {
      if (r == root && !loop) continue;
      int64_t plo, phi;
      bounds(L, loop ? world : world - 1, align, o++, &plo, &phi);
      p->pstart[c * world + r] = a + plo;
      p->psize[c * world + r] = phi - plo;
    }
    p->roff[c] = p->mine;
    p->mine += p->psize[c * world + me];
  }
}

// One point-to-point operation of the ordered exchange, as the executor issues it.
struct P2p {
  int peer;
  bool send;
  int buf;         // FA_XBUF_*: the send buffer (partials), the recv buffer, or d_out
  int64_t offset;  // elements into that buffer
  int64_t count;   // elements
};

// The ops of rank `me` in chunk ch: phase 0 = partials to the owners (communicator 1), phase 1 = the
// summed pieces to the root / to every rank (communicator 2).  A pure function of the plan: every
// rank derives its sends and its peers' matching receives from the same plan (fa_group_ops exports it
// for the CPU test that pairs them up and replays the data movement).  With `loop` a rank's own piece
// travels too (self send / receive in the same group) and the owner's sum lands in FA_XBUF_SUM, from
// where the delivery sends it -- to the root, or to every rank, itself included.
void xchg_ops(const Plan& p, int world, int me, int root, bool to_all, bool loop, int phase, int64_t ch,
              std::vector<P2p>& ops) {
  ops.clear();
  const int64_t L_me = p.psize[ch * world + me], s_me = p.pstart[ch * world + me];
  const int64_t r0 = world * p.roff[ch];
  for (int r = 0; r < world; ++r) {
    if (r == me && !loop) continue;
    const int64_t Lr = p.psize[ch * world + r], sr = p.pstart[ch * world + r];
    if (phase == 0) {
      if (Lr) ops.push_back(P2p{r, true, FA_XBUF_SEND, sr, Lr});
      if (L_me) ops.push_back(P2p{r, false, FA_XBUF_RECV, r0 + r * L_me, L_me});
    } else {
      if ((to_all || me == root) && Lr) ops.push_back(P2p{r, false, FA_XBUF_OUT, sr, Lr});
      if (L_me && (to_all || r == root))
        ops.push_back(loop ? P2p{r, true, FA_XBUF_SUM, p.roff[ch], L_me} : P2p{r, true, FA_XBUF_OUT, s_me, L_me});
    }
  }
}

int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

struct Scratch {
  int64_t send = 0, recv = 0, sum = 0, stage = 0, total = 0;  // byte offsets / total
};

int scratch_layout(int exchange, bool loop, const fa_local_step* L, int64_t n, int32_t chunks, int32_t align,
                   int world, int root, int me, int osz, Scratch* s) {
  s->send = s->recv = s->sum = s->stage = s->total = 0;
  if (exchange == FA_XCHG_ORDERED || exchange == FA_XCHG_ORDERED_ALL) {
    if (world <= 1 && !loop) return FA_OK;  // nothing to exchange
    Plan p;
    make_plan(n, chunks, align, world, root, me, loop, &p);
    const int64_t send_b = L->kind == FA_LOCAL_PARTIAL ? 0 : round_up(n * osz, 256);
    s->send = 0;
    s->recv = send_b;
    s->sum = send_b + round_up(world * p.mine * osz, 256);
    s->total = s->sum + (loop ? round_up(p.mine * osz, 256) : 0);
  } else if (exchange == FA_XCHG_REDUCE_SCATTER) {
    const int64_t S = (n + (int64_t)world * align - 1) / ((int64_t)world * align) * align;
    s->stage = 0;
    s->total = round_up(world * S * osz, 256);
  }
  return FA_OK;
}

int check_local(const fa_local_step* L) {
  if (!L) return fail(FA_ERR_INVALID, "fa_group_reduce: local step is NULL");
  if (L->kind < FA_LOCAL_FLAT || L->kind > FA_LOCAL_PARTIAL)
    return fail(FA_ERR_INVALID, "fa_group_reduce: unknown local kind %d", L->kind);
  if (!esize(L->dtype)) return fail(FA_ERR_DTYPE, "fa_group_reduce: dtype %d", L->dtype);
  if (L->kind == FA_LOCAL_PARTIAL) {
    if (!L->d_partial) return fail(FA_ERR_INVALID, "fa_group_reduce: d_partial is NULL");
    return FA_OK;
  }
  if (L->k <= 0 || !L->d_in) return fail(FA_ERR_INVALID, "fa_group_reduce: k must be > 0 with d_in set");
  if ((L->kind == FA_LOCAL_TILED || L->kind == FA_LOCAL_GROUPED_TILED) && L->tile_stride < FA_TILE_BYTES)
    return fail(FA_ERR_INVALID, "fa_group_reduce: tile_stride %lld < %d", (long long)L->tile_stride, FA_TILE_BYTES);
  if ((L->kind == FA_LOCAL_GROUPED || L->kind == FA_LOCAL_GROUPED_TILED) &&
      (L->num_groups <= 0 || !L->group_ptr))
    return fail(FA_ERR_INVALID, "fa_group_reduce: grouped local step without groups");
  return FA_OK;
}

// Elements [a, b) of the local partial into dst (device, b - a elements of the partial type), on st.
int run_local(fa_ctx* ctx, fa_comm* c, const fa_local_step* L, int64_t a, int64_t b, void* dst, hipStream_t st,
              std::vector<const void*>& ptrs) {
  if (b <= a) return FA_OK;
  const int es = esize(L->dtype);
  const bool tiled = L->kind == FA_LOCAL_TILED || L->kind == FA_LOCAL_GROUPED_TILED;
  const int64_t E = FA_TILE_BYTES / es;
  if (tiled && a % E) return fail(FA_ERR_INVALID, "fa_group_reduce: chunk start %lld is not tile-aligned", (long long)a);
  ptrs.resize(L->k);
  for (int i = 0; i < L->k; ++i)
    ptrs[i] = (const char*)L->d_in[i] + (tiled ? (a / E) * L->tile_stride : a * es);
  hipEvent_t t0 = nullptr, t1 = nullptr;
  if (c->timing) {
    while (c->tnext + 2 > c->tpool.size()) {
      hipEvent_t e;
      FA_HIP(hipEventCreate(&e));
      c->tpool.push_back(e);
    }
    t0 = c->tpool[c->tnext++];
    t1 = c->tpool[c->tnext++];
    FA_HIP(hipEventRecord(t0, st));
  }
  int rc;
  switch (L->kind) {
    case FA_LOCAL_FLAT:
      rc = fa_weighted_sum(ctx, L->dtype, L->mode, b - a, L->k, ptrs.data(), L->coef, L->divisor, dst, st);
      break;
    case FA_LOCAL_TILED:
      rc = fa_weighted_sum_tiled(ctx, L->dtype, L->mode, b - a, L->k, ptrs.data(), L->tile_stride, L->coef,
                                 L->divisor, dst, st);
      break;
    case FA_LOCAL_GROUPED:
      rc = fa_weighted_sum_grouped(ctx, L->dtype, L->mode, b - a, L->k, ptrs.data(), L->coef, L->divisor,
                                   L->num_groups, L->group_ptr, L->group_mode, L->group_coef, L->group_divisor,
                                   dst, st);
      break;
    default:  // FA_LOCAL_GROUPED_TILED
      rc = fa_weighted_sum_grouped_tiled(ctx, L->dtype, L->mode, b - a, L->k, ptrs.data(), L->tile_stride,
                                         L->coef, L->divisor, L->num_groups, L->group_ptr, L->group_mode,
                                         L->group_coef, L->group_divisor, dst, st);
      break;
  }
  if (rc) return rc;
  if (c->timing) {
    FA_HIP(hipEventRecord(t1, st));
    c->launches++;
  }
  return FA_OK;
}

int ordered(fa_ctx* ctx, fa_comm* c, bool to_all, bool loop, const fa_local_step* L, int64_t n, int32_t chunks,
            int32_t align, int root, char* out, char* scratch, hipStream_t st, int osz, ncclDataType_t nt) {
  const int world = c->world, me = c->rank;
  Plan p;
  make_plan(n, chunks, align, world, root, me, loop, &p);
  Scratch sl;
  scratch_layout(to_all ? FA_XCHG_ORDERED_ALL : FA_XCHG_ORDERED, loop, L, n, chunks, align, world, root, me, osz,
                 &sl);
  const bool partial = L->kind == FA_LOCAL_PARTIAL;
  const char* send = partial ? (const char*)L->d_partial : scratch + sl.send;
  char* recv = scratch + sl.recv;
  char* sums = scratch + sl.sum;  // loop: the owner's summed pieces, sent from here
  std::vector<const void*> ptrs, sum_in(world);
  std::vector<hipEvent_t> after_a2a(p.C);

  // the caller's stream has produced the inputs and owns `out`: both RCCL streams start after it
  int rc = order(c, st, c->sa);
  if (!rc) rc = order(c, st, c->sb);
  if (rc) return rc;

  std::vector<P2p> ops;
  char* bufs[4] = {(char*)send, recv, out, sums};
  auto issue = [&](const std::vector<P2p>& list, int which, const char* what) -> int {
    ncclComm_t comm = which ? c->c2 : c->c1;
    hipStream_t s = which ? c->sb : c->sa;
    ncclResult_t res = ncclGroupStart();
    for (size_t q = 0; q < list.size() && res == ncclSuccess; ++q) {
      const P2p& o = list[q];
      char* ptr = bufs[o.buf] + o.offset * osz;
      res = o.send ? ncclSend(ptr, (size_t)o.count, nt, o.peer, comm, s) : ncclRecv(ptr, (size_t)o.count, nt, o.peer, comm, s);
      if (res == ncclSuccess) c->nops[which][o.send ? 0 : 1]++;
    }
    const ncclResult_t end = ncclGroupEnd();  // closes the group whatever happened inside it
    if (res != ncclSuccess) return fail(FA_ERR_COMM, "%s send/recv: %s", what, ncclGetErrorString(res));
    if (end != ncclSuccess) return fail(FA_ERR_COMM, "%s ncclGroupEnd: %s", what, ncclGetErrorString(end));
    return FA_OK;
  };

  auto finish = [&](int64_t ch) -> int {  // owners' sum of chunk ch, then its delivery
    const int64_t L_me = p.psize[ch * world + me], s_me = p.pstart[ch * world + me];
    const int64_t r0 = world * p.roff[ch];
    if (L_me) {  // a rank with no piece (the root) neither waits for its sends nor orders its receives
      FA_HIP(hipStreamWaitEvent(st, after_a2a[ch], 0));  // behind the S(um)'s own stream, not the host
      for (int r = 0; r < world; ++r)  // loop: the own partial came through RCCL like the others
        sum_in[r] = r == me && !loop ? (const void*)(send + s_me * osz) : (const void*)(recv + (r0 + r * L_me) * osz);
      char* dst = loop ? sums + p.roff[ch] * osz : out + s_me * osz;
      int rc2 = fa_weighted_sum(ctx, fa_local_out_dtype(L->dtype, L->mode), FA_MODE_SUM, L_me, world, sum_in.data(),
                                nullptr, 1.0, dst, st);
      if (rc2) return rc2;
      rc2 = order(c, st, c->sb);
      if (rc2) return rc2;
    }
    set_op(c, "chunk %lld/%lld: delivery of the summed pieces %s", (long long)(ch + 1), (long long)p.C,
           to_all ? "to every rank" : "to the root");
    xchg_ops(p, world, me, root, to_all, loop, 1, ch, ops);
    return issue(ops, 1, "delivery");
  };

  for (int64_t ch = 0; ch < p.C; ++ch) {
    const int64_t a = p.lo[ch], b = p.hi[ch];
    if (!partial) {
      rc = run_local(ctx, c, L, a, b, (char*)send + a * osz, st, ptrs);
      if (rc) return rc;
    }
    rc = order(c, st, c->sa);
    if (rc) return rc;
    set_op(c, "chunk %lld/%lld: partials to the owners (point-to-point over every link)", (long long)(ch + 1),
           (long long)p.C);
    xchg_ops(p, world, me, root, to_all, loop, 0, ch, ops);
    rc = issue(ops, 0, "owner");
    if (rc) return rc;
    rc = event(c, &after_a2a[ch]);
    if (rc) return rc;
    FA_HIP(hipEventRecord(after_a2a[ch], c->sa));
    if (ch >= 1) {  // software pipeline: chunk ch-1's owner sum queues behind chunk ch's partial
      rc = finish(ch - 1);
      if (rc) return rc;
    }
  }
  rc = finish(p.C - 1);
  if (rc) return rc;
  rc = order(c, c->sb, st);  // the caller's stream continues after every delivery has landed
  if (!rc) rc = order(c, c->sa, st);
  return rc;
}

int reduce_like(fa_ctx* ctx, fa_comm* c, int exchange, const fa_local_step* L, int64_t n, int32_t chunks,
                int32_t align, int root, char* out, hipStream_t st, int osz, ncclDataType_t nt) {
  const int64_t C = num_chunks(n, chunks, align);
  std::vector<const void*> ptrs;
  const bool partial = L->kind == FA_LOCAL_PARTIAL;
  int rc = order(c, st, c->sa);
  if (rc) return rc;
  for (int64_t ch = 0; ch < C; ++ch) {
    int64_t a, b;
    bounds(n, C, align, ch, &a, &b);
    if (b <= a) continue;
    if (!partial) {
      rc = run_local(ctx, c, L, a, b, out + a * osz, st, ptrs);
      if (rc) return rc;
      rc = order(c, st, c->sa);
      if (rc) return rc;
    }
    const void* src = partial ? (const char*)L->d_partial + a * osz : out + a * osz;
    set_op(c, "chunk %lld/%lld: %s", (long long)(ch + 1), (long long)C,
           exchange == FA_XCHG_REDUCE ? "ncclReduce" : "ncclAllReduce");
    if (exchange == FA_XCHG_REDUCE)
      FA_NCCL(ncclReduce(src, out + a * osz, (size_t)(b - a), nt, ncclSum, root, c->c1, c->sa));
    else
      FA_NCCL(ncclAllReduce(src, out + a * osz, (size_t)(b - a), nt, ncclSum, c->c1, c->sa));
  }
  return order(c, c->sa, st);
}

int reduce_scatter(fa_ctx* ctx, fa_comm* c, const fa_local_step* L, int64_t n, int32_t chunks, int32_t align,
                   char* out, char* stage, hipStream_t st, int osz, ncclDataType_t nt) {
  const int world = c->world;
  const int64_t S = (n + (int64_t)world * align - 1) / ((int64_t)world * align) * align;
  const int64_t C = num_chunks(S, chunks, align);
  const bool partial = L->kind == FA_LOCAL_PARTIAL;
  std::vector<const void*> ptrs;
  int rc = order(c, st, c->sa);
  if (rc) return rc;
  for (int64_t ch = 0; ch < C; ++ch) {
    int64_t a, b;
    bounds(S, C, align, ch, &a, &b);
    const int64_t Lc = b - a, base = world * a;
    if (Lc <= 0) continue;
    for (int r = 0; r < world; ++r) {  // chunk-major staging: rank r's slice of the chunk at base + r*Lc
      const int64_t lo = r * S + a, hi = std::min(r * S + b, n);
      char* dst = stage + (base + r * Lc) * osz;
      if (hi > lo) {
        if (partial) {
          FA_HIP(hipMemcpyAsync(dst, (const char*)L->d_partial + lo * osz, (hi - lo) * osz, hipMemcpyDeviceToDevice, st));
        } else {
          rc = run_local(ctx, c, L, lo, hi, dst, st, ptrs);
          if (rc) return rc;
        }
      }
      const int64_t valid = std::max<int64_t>(hi - lo, 0);
      if (valid < Lc) FA_HIP(hipMemsetAsync(dst + valid * osz, 0, (Lc - valid) * osz, st));
    }
    rc = order(c, st, c->sa);
    if (rc) return rc;
    set_op(c, "chunk %lld/%lld: ncclReduceScatter", (long long)(ch + 1), (long long)C);
    FA_NCCL(ncclReduceScatter(stage + base * osz, out + a * osz, (size_t)Lc, nt, ncclSum, c->c1, c->sa));
  }
  return order(c, c->sa, st);
}

int create_streams(fa_comm* c) {
  fa_detail::DeviceGuard g(c->device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", c->device);
  FA_HIP(hipStreamCreateWithFlags(&c->sa, hipStreamNonBlocking));
  FA_HIP(hipStreamCreateWithFlags(&c->sb, hipStreamNonBlocking));
  return FA_OK;
}

}  // namespace

extern "C" {

int fa_local_out_dtype(int dtype, int mode) {
  return dtype == FA_DTYPE_I64 && mode != FA_MODE_SUM ? FA_DTYPE_F32 : dtype;
}

int fa_comm_unique_id(void* id_out, int64_t id_bytes) {
  if (!id_out || id_bytes < (int64_t)sizeof(ncclUniqueId))
    return fail(FA_ERR_INVALID, "fa_comm_unique_id: need %zu bytes", sizeof(ncclUniqueId));
  ncclUniqueId id;
  FA_NCCL(ncclGetUniqueId(&id));
  memcpy(id_out, &id, sizeof(id));
  return FA_OK;
}

int fa_comm_init(int hip_device, int world, int rank, const void* id, fa_comm** out) {
  if (!out || !id) return fail(FA_ERR_INVALID, "fa_comm_init: NULL argument");
  *out = nullptr;
  if (world < 1 || rank < 0 || rank >= world)
    return fail(FA_ERR_INVALID, "fa_comm_init: rank %d of world %d", rank, world);
  fa_detail::DeviceGuard g(hip_device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", hip_device);
  fa_comm* c = new (std::nothrow) fa_comm();
  if (!c) return fail(FA_ERR_NOMEM, "fa_comm_init: out of host memory");
  c->device = hip_device;
  c->world = world;
  c->rank = rank;
  c->owns = true;
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclResult_t r = ncclCommInitRank(&c->c1, world, uid, rank);
  if (r == ncclSuccess) r = ncclCommSplit(c->c1, 0, rank, &c->c2, nullptr);
  if (r != ncclSuccess) {
    fa_comm_destroy(c);
    return fail(FA_ERR_COMM, "fa_comm_init: %s", ncclGetErrorString(r));
  }
  int rc = create_streams(c);
  if (rc) {
    fa_comm_destroy(c);
    return rc;
  }
  *out = c;
  return FA_OK;
}

int fa_comm_wrap(int hip_device, void* nccl_comm, void* nccl_comm2, fa_comm** out) {
  if (!out || !nccl_comm) return fail(FA_ERR_INVALID, "fa_comm_wrap: NULL communicator");
  *out = nullptr;
  fa_comm* c = new (std::nothrow) fa_comm();
  if (!c) return fail(FA_ERR_NOMEM, "fa_comm_wrap: out of host memory");
  c->device = hip_device;
  c->c1 = (ncclComm_t)nccl_comm;
  c->c2 = nccl_comm2 ? (ncclComm_t)nccl_comm2 : c->c1;
  c->owns = false;
  int n = 0, r = 0;
  ncclResult_t e = ncclCommCount(c->c1, &n);
  if (e == ncclSuccess) e = ncclCommUserRank(c->c1, &r);
  if (e != ncclSuccess) {
    delete c;
    return fail(FA_ERR_COMM, "fa_comm_wrap: %s", ncclGetErrorString(e));
  }
  c->world = n;
  c->rank = r;
  int rc = create_streams(c);
  if (rc) {
    fa_comm_destroy(c);
    return rc;
  }
  if (c->c2 == c->c1) c->sb = c->sa;  // one communicator: one RCCL stream (its calls stay ordered)
  *out = c;
  return FA_OK;
}

int fa_comm_destroy(fa_comm* c) {
  if (!c) return FA_OK;
  fa_detail::DeviceGuard g(c->device);
  if (c->sa) (void)hipStreamSynchronize(c->sa);
  if (c->sb && c->sb != c->sa) (void)hipStreamSynchronize(c->sb);
  if (c->owns) {
    if (c->c2 && c->c2 != c->c1) (void)ncclCommDestroy(c->c2);
    if (c->c1) (void)ncclCommDestroy(c->c1);
  }
  for (hipEvent_t e : c->pool) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->tpool) (void)hipEventDestroy(e);
  if (c->sb && c->sb != c->sa) (void)hipStreamDestroy(c->sb);
  if (c->sa) (void)hipStreamDestroy(c->sa);
  delete c;
  return FA_OK;
}

int fa_comm_size(const fa_comm* c, int* world, int* rank) {
  if (!c) return fail(FA_ERR_INVALID, "fa_comm_size: comm is NULL");
  if (world) *world = c->world;
  if (rank) *rank = c->rank;
  return FA_OK;
}

int fa_group_plan_ex(int64_t n, int32_t chunks, int32_t align, int32_t world, int32_t root, int32_t flags,
                     int32_t max_chunks, int64_t* chunk_lo, int64_t* chunk_hi, int64_t* piece_start,
                     int64_t* piece_size) {
  if (n < 0 || chunks < 1 || align < 1 || world < 1 || root < 0 || root >= world || !chunk_lo || !chunk_hi ||
      (flags & ~(FA_XFLAG_DELIVER_ALL | FA_XFLAG_LOOPBACK)))
    return fail(FA_ERR_INVALID, "fa_group_plan: invalid arguments");
  Plan p;
  make_plan(n, chunks, align, world, root, 0, (flags & FA_XFLAG_LOOPBACK) != 0, &p);
  if (p.C > max_chunks) return fail(FA_ERR_INVALID, "fa_group_plan: %lld chunks > max_chunks %d", (long long)p.C, max_chunks);
  for (int64_t c = 0; c < p.C; ++c) {
    chunk_lo[c] = p.lo[c];
    chunk_hi[c] = p.hi[c];
    for (int r = 0; r < world; ++r) {
      if (piece_start) piece_start[c * world + r] = p.pstart[c * world + r];
      if (piece_size) piece_size[c * world + r] = p.psize[c * world + r];
    }
  }
  return (int)p.C;
}

int fa_group_plan(int64_t n, int32_t chunks, int32_t align, int32_t world, int32_t root, int32_t max_chunks,
                  int64_t* chunk_lo, int64_t* chunk_hi, int64_t* piece_start, int64_t* piece_size) {
  return fa_group_plan_ex(n, chunks, align, world, root, 0, max_chunks, chunk_lo, chunk_hi, piece_start, piece_size);
}

int fa_group_ops_ex(int64_t n, int32_t chunks, int32_t align, int32_t world, int32_t rank, int32_t root,
                    int32_t flags, int32_t phase, int32_t chunk, int32_t max_ops, int32_t* peer, int32_t* is_send,
                    int32_t* buf, int64_t* offset, int64_t* count) {
  if (n < 0 || chunks < 1 || align < 1 || world < 1 || rank < 0 || rank >= world || root < 0 || root >= world ||
      (phase != 0 && phase != 1) || chunk < 0 || (flags & ~(FA_XFLAG_DELIVER_ALL | FA_XFLAG_LOOPBACK)))
    return fail(FA_ERR_INVALID, "fa_group_ops: invalid arguments");
  const bool loop = (flags & FA_XFLAG_LOOPBACK) != 0;
  Plan p;
  make_plan(n, chunks, align, world, root, rank, loop, &p);
  if (chunk >= p.C) return fail(FA_ERR_INVALID, "fa_group_ops: chunk %d of %lld", chunk, (long long)p.C);
  std::vector<P2p> ops;
  if (world > 1 || loop) xchg_ops(p, world, rank, root, (flags & FA_XFLAG_DELIVER_ALL) != 0, loop, phase, chunk, ops);
  if ((int64_t)ops.size() > max_ops) return fail(FA_ERR_INVALID, "fa_group_ops: %zu ops > max_ops", ops.size());
  for (size_t q = 0; q < ops.size(); ++q) {
    if (peer) peer[q] = ops[q].peer;
    if (is_send) is_send[q] = ops[q].send;
    if (buf) buf[q] = ops[q].buf;
    if (offset) offset[q] = ops[q].offset;
    if (count) count[q] = ops[q].count;
  }
  return (int)ops.size();
}

int fa_group_ops(int64_t n, int32_t chunks, int32_t align, int32_t world, int32_t rank, int32_t root, int deliver_all,
                 int32_t phase, int32_t chunk, int32_t max_ops, int32_t* peer, int32_t* is_send, int32_t* buf,
                 int64_t* offset, int64_t* count) {
  return fa_group_ops_ex(n, chunks, align, world, rank, root, deliver_all ? FA_XFLAG_DELIVER_ALL : 0, phase, chunk,
                         max_ops, peer, is_send, buf, offset, count);
}

int fa_group_reduce_scratch_bytes(const fa_comm* c, int exchange, const fa_local_step* L, int64_t n,
                                  int32_t chunks, int32_t align, int32_t root, int64_t* bytes) {
  if (!c || !bytes) return fail(FA_ERR_INVALID, "fa_group_reduce_scratch_bytes: NULL argument");
  int rc = check_local(L);
  if (rc) return rc;
  const bool loop = (exchange & FA_XCHG_LOOPBACK) != 0;
  exchange &= ~FA_XCHG_LOOPBACK;
  // the same validity rules as fa_group_reduce: the two entry points accept the same exchanges
  if (exchange < FA_XCHG_ORDERED || exchange > FA_XCHG_REDUCE_SCATTER)
    return fail(FA_ERR_INVALID, "fa_group_reduce_scratch_bytes: unknown exchange %d", exchange);
  if (loop && exchange != FA_XCHG_ORDERED && exchange != FA_XCHG_ORDERED_ALL)
    return fail(FA_ERR_INVALID,
                "fa_group_reduce_scratch_bytes: FA_XCHG_LOOPBACK applies to the ordered exchanges only");
  if (n < 0 || chunks < 1 || align < 1 || root < 0 || root >= c->world)
    return fail(FA_ERR_INVALID, "fa_group_reduce_scratch_bytes: invalid n/chunks/align/root");
  Scratch s;
  scratch_layout(exchange, loop, L, n, chunks, align, c->world, root, c->rank,
                 esize(fa_local_out_dtype(L->dtype, L->mode)), &s);
  *bytes = s.total;
  return FA_OK;
}

int fa_group_reduce(fa_ctx* ctx, fa_comm* c, int exchange, const fa_local_step* L, int64_t n, int32_t chunks,
                    int32_t align, int32_t root, void* d_out, void* d_scratch, int64_t scratch_bytes,
                    void* hip_stream) {
  if (!ctx || !c) return fail(FA_ERR_INVALID, "fa_group_reduce: ctx/comm is NULL");
  int rc = check_local(L);
  if (rc) return rc;
  const bool loop = (exchange & FA_XCHG_LOOPBACK) != 0;
  exchange &= ~FA_XCHG_LOOPBACK;
  if (exchange < FA_XCHG_ORDERED || exchange > FA_XCHG_REDUCE_SCATTER)
    return fail(FA_ERR_INVALID, "fa_group_reduce: unknown exchange %d", exchange);
  if (loop && exchange != FA_XCHG_ORDERED && exchange != FA_XCHG_ORDERED_ALL)
    return fail(FA_ERR_INVALID, "fa_group_reduce: FA_XCHG_LOOPBACK applies to the ordered exchanges only");
  if (n < 0 || chunks < 1 || align < 1 || root < 0 || root >= c->world)
    return fail(FA_ERR_INVALID, "fa_group_reduce: invalid n/chunks/align/root");
  if (n > 0 && !d_out) return fail(FA_ERR_INVALID, "fa_group_reduce: d_out is NULL");
  const int od = fa_local_out_dtype(L->dtype, L->mode);
  const int osz = esize(od);
  ncclDataType_t nt;
  if (!nccl_type(od, &nt)) return fail(FA_ERR_DTYPE, "fa_group_reduce: dtype %d", od);
  if (L->kind == FA_LOCAL_TILED || L->kind == FA_LOCAL_GROUPED_TILED) {
    const int64_t E = FA_TILE_BYTES / esize(L->dtype);
    if (align % E) return fail(FA_ERR_INVALID, "fa_group_reduce: align %d is not a multiple of the tile (%lld)",
                               align, (long long)E);
  }
  Scratch s;
  scratch_layout(exchange, loop, L, n, chunks, align, c->world, root, c->rank, osz, &s);
  if (s.total > 0 && (!d_scratch || scratch_bytes < s.total))
    return fail(FA_ERR_INVALID, "fa_group_reduce: scratch of %lld bytes < %lld needed", (long long)scratch_bytes,
                (long long)s.total);
  if (n == 0) return FA_OK;
  fa_detail::DeviceGuard g(c->device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", c->device);
  hipStream_t st = (hipStream_t)hip_stream;
  c->next_ev = 0;
  char* out = (char*)d_out;
  std::vector<const void*> ptrs;
  if (c->world == 1 && !loop && (exchange == FA_XCHG_ORDERED || exchange == FA_XCHG_ORDERED_ALL)) {
    // no owners: the local step (or the partial) is the result; the RCCL exchanges still run their
    // collectives at world 1 (a copy), so one GPU exercises their stream ordering
    const int64_t C = num_chunks(n, chunks, align);
    for (int64_t ch = 0; ch < C; ++ch) {
      int64_t a, b;
      bounds(n, C, align, ch, &a, &b);
      if (L->kind == FA_LOCAL_PARTIAL) {
        if (b > a && (const void*)out != L->d_partial)
          FA_HIP(hipMemcpyAsync(out + a * osz, (const char*)L->d_partial + a * osz, (b - a) * osz,
                                hipMemcpyDeviceToDevice, st));
      } else if ((rc = run_local(ctx, c, L, a, b, out + a * osz, st, ptrs))) {
        return rc;
      }
    }
    return FA_OK;
  }
  char* scratch = (char*)d_scratch;
  switch (exchange) {
    case FA_XCHG_ORDERED:
    case FA_XCHG_ORDERED_ALL:
      return ordered(ctx, c, exchange == FA_XCHG_ORDERED_ALL, loop, L, n, chunks, align, root, out, scratch, st, osz,
                     nt);
    case FA_XCHG_REDUCE:
    case FA_XCHG_ALL_REDUCE:
      return reduce_like(ctx, c, exchange, L, n, chunks, align, root, out, st, osz, nt);
    default:
      return reduce_scatter(ctx, c, L, n, chunks, align, out, scratch + s.stage, st, osz, nt);
  }
}

int fa_comm_set_timing(fa_comm* c, int enable) {
  if (!c) return fail(FA_ERR_INVALID, "fa_comm_set_timing: comm is NULL");
  c->timing = enable != 0;
  return FA_OK;
}

int fa_comm_local_time(fa_comm* c, int reset, double* ms, int64_t* launches) {
  if (!c) return fail(FA_ERR_INVALID, "fa_comm_local_time: comm is NULL");
  for (size_t i = 0; i + 1 < c->tnext; i += 2) {
    FA_HIP(hipEventSynchronize(c->tpool[i + 1]));
    float dt = 0.f;
    FA_HIP(hipEventElapsedTime(&dt, c->tpool[i], c->tpool[i + 1]));
    c->local_ms += dt;
  }
  c->tnext = 0;
  if (ms) *ms = c->local_ms;
  if (launches) *launches = c->launches;
  if (reset) {
    c->local_ms = 0.0;
    c->launches = 0;
  }
  return FA_OK;
}

int fa_comm_op_counts(const fa_comm* c, int64_t* counts) {
  if (!c || !counts) return fail(FA_ERR_INVALID, "fa_comm_op_counts: NULL argument");
  for (int i = 0; i < 4; ++i) counts[i] = c->nops[i / 2][i % 2];
  return FA_OK;
}

int fa_comm_last_op(const fa_comm* c, char* buf, int64_t buf_bytes) {
  if (!c || !buf || buf_bytes <= 0) return fail(FA_ERR_INVALID, "fa_comm_last_op: invalid arguments");
  std::lock_guard<std::mutex> g(c->mu);
  snprintf(buf, (size_t)buf_bytes, "%s", c->last_op);
  return FA_OK;
}

}  // extern "C"
