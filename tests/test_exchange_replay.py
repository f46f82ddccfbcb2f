"""The ordered group -> global exchange of the C ABI (fa_group_reduce, include/fedagg_comm.h) replayed
on the CPU: every rank's point-to-point operations come from the library itself (fa_group_ops, the
list its executor issues to RCCL), are paired across ranks as RCCL pairs them (per phase and chunk,
one send per peer), and the data they move is replayed with numpy buffers -- every owner's
rank-ordered sum included -- so the whole-model result on the root (or on every rank) is checked
bit-for-bit against the sequential rank-ordered sum, for world sizes no single-GPU box can run.
A send without its matching receive (a hang on the GPUs) fails here."""
from __future__ import annotations

import ctypes
import itertools

import numpy as np
import pytest

from fedml_amd import _native as N

SEND, RECV, OUT, SUM = 0, 1, 2, 3


def ops(n, chunks, align, world, rank, root, to_all, phase, chunk, loop=False):
    L = N.lib()
    cap = 4 * world
    peer, snd, buf = (ctypes.c_int32 * cap)(), (ctypes.c_int32 * cap)(), (ctypes.c_int32 * cap)()
    off, cnt = (ctypes.c_int64 * cap)(), (ctypes.c_int64 * cap)()
    if not loop:  # the original entry point (flags = deliver_all only)
        m = L.fa_group_ops(n, chunks, align, world, rank, root, int(to_all), phase, chunk, cap, peer, snd, buf, off,
                           cnt)
    else:
        flags = (N.XFLAG_DELIVER_ALL if to_all else 0) | N.XFLAG_LOOPBACK
        m = L.fa_group_ops_ex(n, chunks, align, world, rank, root, flags, phase, chunk, cap, peer, snd, buf, off,
                              cnt)
    assert m >= 0, L.fa_last_error()
    return [(peer[i], bool(snd[i]), buf[i], off[i], cnt[i]) for i in range(m)]


def replay(n, chunks, align, world, root, to_all, seed=0, loop=False):
    from fedml_amd.distributed.native_exchange import group_plan
    rng = np.random.default_rng(seed)
    partial = [rng.standard_normal(n).astype(np.float32) for _ in range(world)]
    plan = group_plan(n, chunks, align, world, root, loopback=loop)
    # this rank's pieces, in chunk order, define its receive area (rank-major per piece) and, with
    # loop, its sum area (the pieces back to back)
    mine = [sum(pc[r][1] for _, _, pc in plan) for r in range(world)]
    recv = [np.full(world * mine[r], np.nan, np.float32) for r in range(world)]
    sums = [np.full(mine[r], np.nan, np.float32) for r in range(world)]
    out = [np.full(n, np.nan, np.float32) for _ in range(world)]
    bufs = [[partial[r], recv[r], out[r], sums[r]] for r in range(world)]
    roff = [0] * world
    for c, (a, b, pc) in enumerate(plan):
        if loop:
            assert all(pc[r][1] > 0 for r in range(world)) or b - a < world * align, "loop: every rank owns a piece"
        else:
            assert pc[root][1] == 0
        for phase in (0, 1):
            lists = {r: ops(n, chunks, align, world, r, root, to_all, phase, c, loop) for r in range(world)}
            sends = {(r, o[0]): o for r in range(world) for o in lists[r] if o[1]}
            recvs = {(o[0], r): o for r in range(world) for o in lists[r] if not o[1]}
            assert len(sends) == sum(o[1] for r in range(world) for o in lists[r]), "two sends to one peer"
            assert sends.keys() == recvs.keys(), f"unmatched ops in chunk {c} phase {phase}"
            for (src, dst), so in sends.items():
                ro = recvs[(src, dst)]
                assert so[4] == ro[4] > 0, "count mismatch"
                bufs[dst][ro[2]][ro[3]:ro[3] + ro[4]] = bufs[src][so[2]][so[3]:so[3] + so[4]]
            if phase == 0:  # owners' rank-ordered sum of their piece, into d_out at the piece's place
                for r in range(world):  # (loop: all from the receive area, into the sum area)
                    s_, L_ = pc[r]
                    if not L_:
                        continue
                    r0 = world * roff[r]
                    acc = None
                    for q in range(world):
                        own = q == r and not loop
                        x = partial[r][s_:s_ + L_] if own else recv[r][r0 + q * L_: r0 + (q + 1) * L_]
                        acc = x.copy() if acc is None else (acc + x).astype(np.float32)
                    if loop:
                        sums[r][roff[r]:roff[r] + L_] = acc
                    else:
                        out[r][s_:s_ + L_] = acc
                for r in range(world):
                    roff[r] += pc[r][1]
    exp = partial[0].copy()
    for q in range(1, world):
        exp = (exp + partial[q]).astype(np.float32)
    return out, exp


@pytest.mark.parametrize("world,root,to_all", [(w, r, t) for w in (2, 3, 4, 5, 8) for r in sorted({0, w - 1})
                                               for t in (False, True)])
@pytest.mark.parametrize("n,chunks,align", [(1000, 3, 1), (4096 * 5 + 17, 8, 1024), (64, 8, 256), (7, 4, 1)])
def test_ordered_exchange_replay(world, root, to_all, n, chunks, align):
    out, exp = replay(n, chunks, align, world, root, to_all, seed=world * 31 + n)
    targets = range(world) if to_all else [root]
    for r in targets:
        assert np.array_equal(out[r].view(np.int32), exp.view(np.int32)), f"rank {r}"


@pytest.mark.parametrize("world,root,to_all", [(w, r, t) for w in (1, 2, 3, 8) for r in sorted({0, w - 1})
                                               for t in (False, True)])
@pytest.mark.parametrize("n,chunks,align", [(1000, 3, 1), (4096 * 5 + 17, 8, 1024), (64, 8, 256)])
def test_loopback_exchange_replay(world, root, to_all, n, chunks, align):
    """FA_XCHG_LOOPBACK: every rank owns a piece and its own piece goes through a self send/receive;
    at world 1 that is the whole exchange the one-GPU box runs through RCCL."""
    out, exp = replay(n, chunks, align, world, root, to_all, seed=world * 17 + n, loop=True)
    targets = range(world) if to_all else [root]
    for r in targets:
        assert np.array_equal(out[r].view(np.int32), exp.view(np.int32)), f"rank {r}"


def test_loopback_ops_world1():
    """At world 1 every phase is a self send + receive of the whole chunk (nothing short-circuits)."""
    for phase in (0, 1):
        for to_all in (False, True):
            o = ops(10_000, 4, 256, 1, 0, 0, to_all, phase, 2, loop=True)
            assert sorted(x[1] for x in o) == [False, True] and all(x[0] == 0 for x in o)
            assert {x[2] for x in o} == ({SEND, RECV} if phase == 0 else {SUM, OUT})
    assert ops(10_000, 4, 256, 1, 0, 0, False, 0, 2) == []  # without the flag: no exchange at world 1


def test_ops_are_deterministic_and_pure():
    a = ops(125_000_000, 8, 1024, 8, 3, 0, False, 0, 5)
    b = ops(125_000_000, 8, 1024, 8, 3, 0, False, 0, 5)
    assert a == b and len(a) == 6 + 7  # its pieces to the 6 other owners; their 7 senders (root included) in
    root_ops = ops(125_000_000, 8, 1024, 8, 0, 0, False, 0, 5)
    assert all(o[1] for o in root_ops) and len(root_ops) == 7  # the root only sends in phase 0


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("loop", [False, True])
@pytest.mark.parametrize("to_all", [False, True])
def test_owned_pieces_are_in_d_out(world, loop, to_all):
    """NativeExchange.owned(rank) names only pieces that rank's d_out really holds after the exchange
    (replayed): under loopback + "ordered" a non-root owner sums into scratch, so it owns nothing
    there; without loopback the owner's sum lands in its d_out at the piece's place."""
    import types
    from fedml_amd.distributed.native_exchange import NativeExchange
    n, chunks, align, root = 1024 * 100 + 17, 4, 1024, 0
    out, exp = replay(n, chunks, align, world, root, to_all, seed=world * 7 + 3, loop=loop)
    for r in range(world):
        x = object.__new__(NativeExchange)
        x.collective, x.chunks, x.root, x.loopback = ("ordered_all" if to_all else "ordered"), chunks, root, loop
        x.comm = types.SimpleNamespace(world=world, rank=r)
        owned = x.owned(n, align)
        if loop and not to_all and r != root:
            assert owned == []
        elif not loop and r == root:
            assert owned == []  # the root owns no piece without loopback
        for lo, hi in owned:
            assert np.array_equal(out[r][lo:hi].view(np.int32), exp[lo:hi].view(np.int32)), (r, lo, hi)
