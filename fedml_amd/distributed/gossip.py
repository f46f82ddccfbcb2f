"""Multi-GPU decentralized gossip: n simulated nodes spread in contiguous blocks over the GPUs.

Reference step (per node, python/fedml/simulation/sp/decentralized/client_dsgd.py:92-122 and
client_pushsum.py:111-156): x_i <- x_i * W_ii + sum_{j in-neighbours, ascending} x_j * W_ji.

Placement: node i lives on rank owner(i) = i // ceil(n / world).  A step needs, on every rank,
the models of the in-neighbours of its nodes that live elsewhere (for a ring: one model from each
neighbouring rank -- a halo).  The step is:

  1. post the halo exchange (torch.distributed P2P = RCCL send/recv over xGMI, all at once);
  2. mix the INTERIOR rows (every input local) with the HIP mixing kernel while halos are in flight;
  3. wait, then mix the BOUNDARY rows.

Every output row is the same ordered per-element sum as on one GPU, so the result is bit-identical
to the single-GPU (and reference) step whatever the number of ranks.  The local mixing is
injectable (``local_mix``) so the exchange logic is testable with gloo on CPU.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ..core.distributed.topology.topology_manager import gossip_rows


def _engine_mix(xs, row_ptr, cols, vals, post_scale, outs, outs2):
    from ..engine import get_engine
    return get_engine(xs[0].device.index).mix(xs, row_ptr, cols, vals, post_scale, outs, outs2)


def _engine_pushsum(xs, row_ptr, cols, vals, omega_in, outs, outs2, omega_out):
    from ..engine import get_engine
    return get_engine(xs[0].device.index).pushsum(xs, row_ptr, cols, vals, omega_in, outs, outs2, omega_out)


class GossipPlan:
    """One rank's share of a distributed gossip step, as a pure function of (W, rank, world): the
    nodes it owns, the halo it receives and sends, its interior / boundary rows and the ring-ordered
    input list its mixing rows index.  DistributedGossip executes it; tests run every rank's local
    problem on one device through the same plan."""

    def __init__(self, W: np.ndarray, rank: int, world: int):
        self.W = np.asarray(W, dtype=np.float32)
        self.n = self.W.shape[0]
        self.rank, self.world = rank, world
        self.block = -(-self.n // world)
        self.mine = [i for i in range(self.n) if self.owner(i) == rank]
        row_ptr, cols, vals = gossip_rows(self.W, self.mine)
        self._rows = [(cols[row_ptr[r]:row_ptr[r + 1]], vals[row_ptr[r]:row_ptr[r + 1]]) for r in range(len(self.mine))]
        self.halo_in = sorted({c for cs, _ in self._rows for c in cs if self.owner(c) != rank})  # received
        # what this rank must send: for every other rank, its remote needs that live here
        self.halo_out: Dict[int, List[int]] = {}
        for r in range(world):
            if r == rank:
                continue
            theirs = [i for i in range(self.n) if self.owner(i) == r]
            _, cs, _ = gossip_rows(self.W, theirs)
            want = sorted({c for c in cs if self.owner(c) == rank})
            if want:
                self.halo_out[r] = want
        local_set = set(self.mine)
        self.interior = [r for r, (cs, _) in enumerate(self._rows) if all(c in local_set for c in cs)]
        self.boundary = [r for r in range(len(self.mine)) if r not in set(self.interior)]
        # inputs in ring order around this rank's block (left halo, own nodes, right halo): for a
        # banded W the mixing rows then read inputs (row + const + {-1, 0, 1}) and take the
        # sliding-window kernel
        half = self.n // 2
        self.inputs = sorted(list(self.mine) + list(self.halo_in), key=lambda v: (v - self.mine[0] + half) % self.n) \
            if self.mine else []
        self.index = {v: k for k, v in enumerate(self.inputs)}

    def owner(self, i: int) -> int:
        return min(i // self.block, self.world - 1)

    def csr(self, rows: Sequence[int]) -> Tuple[list, list, list]:
        """CSR of the given local rows over ``self.inputs`` positions."""
        row_ptr, cols, vals = [0], [], []
        for r in rows:
            cs, vs = self._rows[r]
            cols += [self.index[c] for c in cs]
            vals += vs
            row_ptr.append(len(cols))
        return row_ptr, cols, vals

    def mix_local(self, tensor_of: Dict[int, torch.Tensor], local_mix: Callable, rows: Sequence[int],
                  outs: List[torch.Tensor], outs2: Optional[List[torch.Tensor]] = None,
                  post_scale: Optional[Sequence[float]] = None):
        """Mix the given local rows (indices into ``mine``) from node models ``tensor_of``."""
        if not rows:
            return
        inputs = [tensor_of[v] for v in self.inputs]
        rp, cs, vs = self.csr(rows)
        ps = [post_scale[r] for r in rows] if post_scale is not None else None
        local_mix(inputs, rp, cs, vs, ps, [outs[r] for r in rows], [outs2[r] for r in rows] if outs2 is not None else None)

    def pushsum_local(self, tensor_of: Dict[int, torch.Tensor], omega_inputs: torch.Tensor, local_pushsum: Callable,
                      rows: Sequence[int], outs: List[torch.Tensor], outs2: List[torch.Tensor],
                      omega_out: torch.Tensor):
        """PushSum rows with the weights on the device: ``omega_inputs`` (float32, ``self.inputs``
        order) mixed by the same rows; omega' of local row r lands in omega_out[r]."""
        if not rows:
            return
        inputs = [tensor_of[v] for v in self.inputs]
        rp, cs, vs = self.csr(rows)
        om = torch.empty(len(rows), dtype=torch.float32, device=omega_out.device)
        local_pushsum(inputs, rp, cs, vs, omega_inputs, [outs[r] for r in rows], [outs2[r] for r in rows], om)
        omega_out.index_copy_(0, torch.tensor(list(rows), device=omega_out.device), om)


class DistributedGossip:
    def __init__(self, W: np.ndarray, group=None, local_mix: Optional[Callable] = None,
                 local_pushsum: Optional[Callable] = None):
        self.group = group
        self.local_pushsum = local_pushsum or _engine_pushsum
        self.plan = GossipPlan(W, dist.get_rank(group), dist.get_world_size(group))
        p = self.plan
        self.W, self.n, self.rank, self.world, self.block = p.W, p.n, p.rank, p.world, p.block
        self.mine, self.halo_in, self.halo_out = p.mine, p.halo_in, p.halo_out
        self.interior, self.boundary = p.interior, p.boundary
        self.local_mix = local_mix or _engine_mix

    def owner(self, i: int) -> int:
        return self.plan.owner(i)

    def step(self, local_models: Sequence[torch.Tensor], post_scale: Optional[Sequence[float]] = None,
             omega: Optional[torch.Tensor] = None):
        """local_models[k] = flat model of node self.mine[k]; returns (new_models, scaled or None).

        PushSum with the weights on the device: ``omega`` = float32 tensor of this rank's nodes'
        weights; the halo carries the neighbours' weights with their models, omega' is mixed by the
        same rows and 1/omega' applied on the device; returns (x', z', omega')."""
        assert len(local_models) == len(self.mine)
        proto = local_models[0]
        halo = {i: torch.empty_like(proto) for i in self.halo_in}
        ops = []
        for i in self.halo_in:
            ops.append(dist.P2POp(dist.irecv, halo[i], self.owner(i), self.group))
        for r, idxs in self.halo_out.items():
            for i in idxs:
                ops.append(dist.P2POp(dist.isend, local_models[self.mine.index(i)], r, self.group))
        if omega is not None:
            assert omega.dtype == torch.float32 and omega.numel() == len(self.mine)
            omega_halo = {i: torch.empty(1, dtype=torch.float32, device=omega.device) for i in self.halo_in}
            for i in self.halo_in:
                ops.append(dist.P2POp(dist.irecv, omega_halo[i], self.owner(i), self.group))
            for r, idxs in self.halo_out.items():
                for i in idxs:
                    k = self.mine.index(i)
                    ops.append(dist.P2POp(dist.isend, omega[k:k + 1], r, self.group))
        reqs = dist.batch_isend_irecv(ops) if ops else []
        if omega is not None:
            return self._pushsum_rest(local_models, halo, omega, omega_halo, reqs)
        tensor_of = {node: local_models[k] for k, node in enumerate(self.mine)}
        tensor_of.update(halo)
        outs = [torch.empty_like(proto) for _ in self.mine]
        outs2 = [torch.empty_like(proto) for _ in self.mine] if post_scale is not None else None
        # the interior rows read only local models: they overlap the halo exchange
        self.plan.mix_local(tensor_of, self.local_mix, self.interior, outs, outs2, post_scale)
        for q in reqs:
            q.wait()
        self.plan.mix_local(tensor_of, self.local_mix, self.boundary, outs, outs2, post_scale)
        return outs, outs2

    def _pushsum_rest(self, local_models, halo, omega, omega_halo, reqs):
        p = self.plan
        proto = local_models[0]
        tensor_of = {node: local_models[k] for k, node in enumerate(self.mine)}
        tensor_of.update(halo)
        outs = [torch.empty_like(proto) for _ in self.mine]
        outs2 = [torch.empty_like(proto) for _ in self.mine]
        omega_out = torch.empty(len(self.mine), dtype=torch.float32, device=omega.device)
        # weights in the plan's input order: own nodes now, the halo's once received
        om_in = torch.zeros(len(p.inputs), dtype=torch.float32, device=omega.device)
        own_pos = torch.tensor([p.index[v] for v in self.mine], device=omega.device)
        om_in.index_copy_(0, own_pos, omega)
        p.pushsum_local(tensor_of, om_in, self.local_pushsum, self.interior, outs, outs2, omega_out)
        for q in reqs:
            q.wait()
        if self.halo_in:
            halo_pos = torch.tensor([p.index[v] for v in self.halo_in], device=omega.device)
            om_in.index_copy_(0, halo_pos, torch.cat([omega_halo[i] for i in self.halo_in]))
        p.pushsum_local(tensor_of, om_in, self.local_pushsum, self.boundary, outs, outs2, omega_out)
        return outs, outs2, omega_out
