"""The product's N > 1 path (GroupReducer with native=True -> NativeExchange -> fa_group_reduce) at
world 8 on the CPU.  On the GPUs, NativeExchange.run is ONE fa_group_reduce
call whose executor (fedml_amd/csrc/comm.hip, ``ordered``) issues, per chunk: the local partial, the
phase-0 point-to-point group on communicator 1 (fa_group_ops_ex phase 0), and -- one chunk behind,
the software pipeline -- the owners' rank-ordered SUM and the phase-1 delivery group on
communicator 2.  Here 8 real gloo processes run the SAME product objects (GroupReducer(native=True),
NativeExchange's local-step descriptors, its plan, its ``owned`` pieces) with only the executor
swapped for a Python mirror of comm.hip's ``ordered`` that issues the C library's own op lists
(fa_group_ops_ex, the exact sends / receives / buffers / offsets / counts RCCL gets) as gloo
batch_isend_irecv groups in the executor's order, on two process groups.  The local partials and
the owners' sums are the C oracle's (the product computes them with its HIP kernels: -m gpu tests).
A send without its receive, a wrong offset or a wrong pipeline order fails or hangs here, and the
global model on the root (ordered) or on every rank (ordered_all) is checked bit-for-bit against
the sequential rank-ordered sum; every ``owned`` piece as well.
"""
from __future__ import annotations

import ctypes
import os
import sys
import types

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_distributed_gloo import _spawn  # noqa: E402

SEND, RECV, OUT, SUM = 0, 1, 2, 3  # FA_XBUF_* (include/fedagg_comm.h)


def _np_view(addr, shape, strides, dtype=np.float32):
    """A numpy view of host memory at ``addr`` (a descriptor's client pointer)."""
    n_bytes = (np.array(shape) - 1) @ np.array(strides) + np.dtype(dtype).itemsize
    buf = (ctypes.c_char * int(n_bytes)).from_address(int(addr))
    return np.lib.stride_tricks.as_strided(np.frombuffer(buf, dtype=dtype), shape=shape, strides=strides)


def _local_partial(st, a, b):
    """The descriptor's local step over elements [a, b) with the C oracle (flat / tiled / grouped,
    the arithmetic fa_weighted_sum* run on the GPUs)."""
    from oracle import orc
    from fedml_amd import _native as N
    k = st.k
    E = N.TILE_BYTES // 4
    xs = []
    for i in range(k):
        if st.kind in (N.LOCAL_TILED, N.LOCAL_GROUPED_TILED):
            t0, t1 = a // E, -(-b // E)
            v = _np_view(st.d_in[i] + t0 * st.tile_stride, (t1 - t0, E), (st.tile_stride, 4)).reshape(-1)[:b - a]
        else:
            v = _np_view(st.d_in[i] + 4 * a, (b - a,), (4,))
        xs.append(torch.from_numpy(np.array(v)))
    coef = [st.coef[i] for i in range(k)] if st.mode != N.SUM else None
    if st.kind in (N.LOCAL_FLAT, N.LOCAL_TILED):
        return orc.weighted_sum(xs, st.mode, coef, st.divisor)
    terms = []  # grouped: per group G_g, then its epilogue, then the ordered sum over groups
    for g in range(st.num_groups):
        lo, hi = st.group_ptr[g], st.group_ptr[g + 1]
        G = orc.weighted_sum(xs[lo:hi], st.mode, None if coef is None else coef[lo:hi], st.divisor)
        if st.group_mode == N.MUL_W:
            G = orc.weighted_sum([G], N.MUL_W, [st.group_coef[g]])
        elif st.group_mode == N.MUL_N_DIV_N:
            G = orc.weighted_sum([G], N.MUL_N_DIV_N, [st.group_coef[g]], st.group_divisor[g])
        terms.append(G)
    return terms[0].clone() if len(terms) == 1 else orc.weighted_sum(terms, N.SUM)


def _ops(n, chunks, align, world, me, root, to_all, loop, phase, ch):
    from fedml_amd import _native as N
    cap = 4 * world
    peer, snd, buf = (ctypes.c_int32 * cap)(), (ctypes.c_int32 * cap)(), (ctypes.c_int32 * cap)()
    off, cnt = (ctypes.c_int64 * cap)(), (ctypes.c_int64 * cap)()
    flags = (N.XFLAG_DELIVER_ALL if to_all else 0) | (N.XFLAG_LOOPBACK if loop else 0)
    m = N.lib().fa_group_ops_ex(n, chunks, align, world, me, root, flags, phase, ch, cap, peer, snd, buf, off, cnt)
    assert m >= 0
    return [(peer[i], bool(snd[i]), buf[i], off[i], cnt[i]) for i in range(m)]


def _mirror_run(self, desc, n, align, out=None, stream=None):
    """comm.hip ``ordered`` (the fa_group_reduce executor of the ordered exchanges), issued over gloo:
    same plan, same op lists, same buffers, same pipeline order."""
    import torch.distributed as dist
    from fedml_amd import _native as N
    from fedml_amd.distributed.native_exchange import group_plan
    from oracle import orc
    st, keep, in_dt = desc
    assert self.collective in ("ordered", "ordered_all"), "the mirror runs the ordered exchanges"
    world, me, root, loop = self.comm.world, self.comm.rank, self.root, self.loopback
    to_all = self.collective == "ordered_all"
    plan = group_plan(n, self.chunks, align, world, root, loop)
    mine = sum(pc[me][1] for _, _, pc in plan)
    roff, o = [], 0
    for _, _, pc in plan:
        roff.append(o)
        o += pc[me][1]
    odt = torch.float32
    send = torch.full((n,), float("nan"), dtype=odt)
    recv = torch.full((world * mine,), float("nan"), dtype=odt)
    sums = torch.full((mine,), float("nan"), dtype=odt)
    if out is None:
        out = torch.full((n,), float("nan"), dtype=odt)
    bufs = {SEND: send, RECV: recv, OUT: out, SUM: sums}
    groups = (None, self.comm.group2)
    after = {}
    pend2 = []
    self.comm.issued = []

    def issue(ops, which):
        p2p, local = [], []
        for peer, is_send, b, off_, cnt in ops:
            view = bufs[b][off_:off_ + cnt]
            self.comm.issued.append((which, peer, is_send, b, off_, cnt))
            if peer == me:  # loopback self send / receive (RCCL pairs them; gloo has no self P2P)
                local.append((is_send, view))
                continue
            p2p.append(dist.P2POp(dist.isend if is_send else dist.irecv, view, peer, groups[which]))
        s_ = [v for s, v in local if s]
        r_ = [v for s, v in local if not s]
        assert len(s_) == len(r_) <= 1, "at most one self pair per group"
        for a_, b_ in zip(s_, r_):
            b_.copy_(a_)
        return dist.batch_isend_irecv(p2p) if p2p else []

    def finish(ch):
        a, b, pc = plan[ch]
        s_me, L_me = pc[me]
        r0 = world * roff[ch]
        if L_me:
            for w in after.pop(ch):  # (a gloo work is waited once: a second wait() waits for another message)
                w.wait()
            parts = [send[s_me:s_me + L_me] if (r == me and not loop) else recv[r0 + r * L_me:r0 + (r + 1) * L_me]
                     for r in range(world)]
            res = orc.weighted_sum([p.contiguous() for p in parts], N.SUM)
            (sums[roff[ch]:roff[ch] + L_me] if loop else out[s_me:s_me + L_me]).copy_(res)
        pend2.extend(issue(_ops(n, self.chunks, align, world, me, root, to_all, loop, 1, ch), 1))

    for ch, (a, b, _) in enumerate(plan):
        send[a:b] = _local_partial(st, a, b)
        after[ch] = issue(_ops(n, self.chunks, align, world, me, root, to_all, loop, 0, ch), 0)
        if ch >= 1:
            finish(ch - 1)
    finish(len(plan) - 1)
    for w in pend2:
        w.wait()
    for ws in after.values():
        for w in ws:
            w.wait()
    self._keep = keep
    return out


def _install_mirror():
    """GroupReducer(native=True) with the mirror executor: the fake fa_comm carries the world, the rank
    and a second process group (comm.hip's communicator 2)."""
    import torch.distributed as dist
    from fedml_amd.distributed import group_reduce, native_exchange

    comm = types.SimpleNamespace(world=dist.get_world_size(), rank=dist.get_rank(), device=0,
                                 group2=dist.new_group(list(range(dist.get_world_size()))),
                                 set_timing=lambda enable: None)
    group_reduce._native_comm = lambda group: comm
    native_exchange.NativeExchange.run = _mirror_run
    return comm


def _expected(parts):
    from oracle import orc
    return orc.weighted_sum(parts, 2)


def _bits(a, b):
    return torch.equal(a.reshape(-1).view(torch.int32), b.reshape(-1).view(torch.int32))


def _case_world(rank, world):
    from oracle import orc
    from fedml_amd.distributed.group_reduce import GroupReducer
    from fedml_amd.engine import MUL_N_DIV_N, MUL_W
    _install_mirror()
    K, P = 4 * world, 3 * 4096 + 1000 * world + 7
    g = torch.Generator().manual_seed(11)
    xs = [torch.randn(P, generator=g) for _ in range(K)]
    counts = [int(v) for v in torch.randint(50, 601, (K,), generator=g)]
    N_ = sum(counts)
    per = K // world
    ids = [list(range(r * per, (r + 1) * per)) for r in range(world)]
    parts = [orc.weighted_sum([xs[i] for i in ids[r]], MUL_W, [counts[i] / N_ for i in ids[r]]) for r in range(world)]
    exp = _expected(parts)
    for coll in ("ordered", "ordered_all"):
        for dst in sorted({0, world - 1}):
            for chunks in (1, 3, 8):
                for loop in (False, True):
                    red = GroupReducer(collective=coll, dst=dst, chunks=chunks, native=True, loopback=loop)
                    assert red.native is not None
                    got = red.fedavg([xs[i] for i in ids[rank]], [counts[i] / N_ for i in ids[rank]])
                    if rank == dst or coll == "ordered_all":
                        assert _bits(got, exp), (coll, dst, chunks, loop)
                    for lo, hi in red.owned or []:  # pieces this rank summed AND holds in its d_out
                        assert _bits(got[lo:hi], exp[lo:hi]), (coll, dst, chunks, loop, lo, hi)
    # the hierarchical formula (one group per rank; the grouped local step: group FedAvg, then the
    # cloud term (G * N_r) / N) and two groups per rank
    for gpr in (1, 2):
        gs = [ids[r][j * per // gpr:(j + 1) * per // gpr] for r in range(world) for j in range(gpr)]
        terms = []
        for grp in gs:
            Ng = sum(counts[i] for i in grp)
            G = orc.weighted_sum([xs[i] for i in grp], MUL_W, [counts[i] / Ng for i in grp])
            terms.append(orc.weighted_sum([G], MUL_N_DIV_N, [Ng], float(N_)))
        rparts = [orc.weighted_sum(terms[r * gpr:(r + 1) * gpr], 2) if gpr > 1 else terms[r] for r in range(world)]
        exp_h = _expected(rparts)
        red = GroupReducer(collective="ordered", chunks=4, native=True)
        mine = gs[rank * gpr:(rank + 1) * gpr]
        got = red.hierarchical_groups([xs[i] for grp in mine for i in grp], [[counts[i] for i in grp] for grp in mine],
                                      N_)
        if rank == 0:
            assert _bits(got, exp_h), gpr
    # the tiled arena local step (fa_weighted_sum_tiled's descriptor over a [tiles, capacity, E] group)
    E = 1024
    nt = -(-P // E)
    buf = torch.zeros(nt, per + 1, E)
    rows = list(range(1, per + 1))  # row 0 unused: the descriptor's row pointers are honoured
    for j, i in enumerate(ids[rank]):
        f = torch.zeros(nt * E)
        f[:P] = xs[i]
        buf[:, rows[j], :] = f.view(nt, E)
    red = GroupReducer(collective="ordered_all", chunks=3, native=True)
    got = red.fedavg_tiled(None, buf, rows, [counts[i] / N_ for i in ids[rank]], P)
    assert _bits(got, exp)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_native_exchange_mirror_gloo(world):
    _spawn(_case_world, world=world)


def test_mirror_issues_the_library_op_lists():
    """The mirror issues exactly fa_group_ops_ex's lists (not a re-derivation): a world-1 loopback run
    in this process records one self send + receive per phase and chunk, as comm.hip does."""
    import torch.distributed as dist
    from fedml_amd.distributed.group_reduce import GroupReducer
    from test_distributed_gloo import _free_port
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        comm = _install_mirror()
        xs = [torch.randn(9000) for _ in range(3)]
        red = GroupReducer(collective="ordered", chunks=3, native=True, loopback=True)
        got = red.fedavg(xs, [0.2, 0.3, 0.5])
        from oracle import orc
        assert _bits(got, orc.weighted_sum(xs, 0, [0.2, 0.3, 0.5]))
        per_phase = {}
        for which, peer, is_send, b, off, cnt in comm.issued:
            per_phase.setdefault(which, []).append((is_send, b))
        assert per_phase[0] == [(True, SEND), (False, RECV)] * 3
        assert per_phase[1] == [(False, OUT), (True, SUM)] * 3
    finally:
        from fedml_amd.distributed.group_reduce import release_groups
        release_groups()
        dist.destroy_process_group()
