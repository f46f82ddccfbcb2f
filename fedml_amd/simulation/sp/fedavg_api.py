"""Single-process FedAvg round driver (reference: python/fedml/simulation/sp/fedavg/fedavg_api.py).

``FedAvgAPI._aggregate(w_locals)`` is the reference's inline FedAvg loop (fedavg_api.py:144-159,
bit-identical to FedMLAggOperator.agg's FedAvg branch), run on the MI355X engine.  ``train`` is a
compact version of the reference's round loop (:66-125): every round the clients are sampled as
the reference samples them (``_client_sampling``, :127-135, unless a ``sampler`` is injected),
each sampled client gets the global weights, trains with its ClientTrainer, and the updates are
averaged on the GPU.

The reference keeps each trained update as ``copy.deepcopy(w)`` (:101).  Here that copy is made
into a row of a ClientArena on the engine's device (ClientArena.adopt: one copy per dtype group,
the dict's entries rebound to the row's views), so ``_aggregate`` over the round's updates is
recognised as arena-resident and runs as one launch per dtype group over the rows instead of a
(key, client) pointer-table walk over separate allocations.
"""
from __future__ import annotations

import copy
import logging
from collections import OrderedDict
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ...arena import ClientArena
from ...ml.aggregator.state_dict_agg import fedavg


class FedAvgAPI:
    def __init__(self, args, device, model, client_trainers: Sequence = (), train_data: Sequence = (),
                 sample_nums: Sequence[int] = (), sampler: Optional[Callable[[int], List[int]]] = None):
        self.args = args
        self.device = device
        self.model = model
        self.client_trainers = list(client_trainers)
        self.train_data = list(train_data)
        self.sample_nums = list(sample_nums)
        self.sampler = sampler

    def _aggregate(self, w_locals: List[Tuple[int, "OrderedDict"]]):
        """Reference fedavg_api.py:144-159: avg[k] = sum_i x_i[k] * (n_i / N), client order."""
        return fedavg([params for _, params in w_locals], [n for n, _ in w_locals])

    def _arena_for(self, w, capacity):
        try:
            return ClientArena.for_model(w, capacity, device=self._engine_device())
        except TypeError:  # a dtype the arena does not hold: keep the reference's deep copies
            return None

    def _engine_device(self):
        dev = torch.device(self.device) if self.device is not None else None
        return dev if dev is not None and dev.type == "cuda" else None

    def _client_sampling(self, round_idx: int, client_num_in_total: int, client_num_per_round: int):
        """Reference fedavg_api.py:127-135: every client when all take part, else
        ``client_num_per_round`` of them drawn without replacement by numpy's global RNG reseeded
        with the round index (the same clients per round in every run)."""
        if client_num_in_total == client_num_per_round:
            return list(range(client_num_in_total))
        num_clients = min(client_num_per_round, client_num_in_total)
        np.random.seed(round_idx)
        return np.random.choice(range(client_num_in_total), num_clients, replace=False)

    def train(self, rounds: Optional[int] = None):
        rounds = rounds if rounds is not None else int(getattr(self.args, "comm_round", 1))
        w_global = self.model.state_dict()
        arena = None
        total = int(getattr(self.args, "client_num_in_total", len(self.client_trainers)))
        per_round = int(getattr(self.args, "client_num_per_round", total))
        for r in range(rounds):
            idx = self.sampler(r) if self.sampler else self._client_sampling(r, total, per_round)
            w_locals = []
            for j, i in enumerate(idx):
                i = int(i)
                trainer = self.client_trainers[i]
                trainer.set_model_params(copy.deepcopy(w_global))
                trainer.train(self.train_data[i], self.device, self.args)
                w = OrderedDict(trainer.get_model_params())
                if arena is None and self._engine_device() is not None:
                    # the server model lives on a HIP device: the updates' deep copies go to HBM rows;
                    # on a CPU model they stay CPU deep copies (the result then stays on the CPU too)
                    arena = self._arena_for(w, len(self.client_trainers))
                if arena is not None:
                    try:
                        arena.adopt(j, w)  # the reference's copy.deepcopy(w), into HBM row j
                    except (TypeError, KeyError):
                        w = copy.deepcopy(w)
                else:
                    w = copy.deepcopy(w)
                w_locals.append((self.sample_nums[i], w))
            w_global = self._aggregate(w_locals)
            self.model.load_state_dict(w_global)
            logging.info("round %d aggregated %d clients", r, len(w_locals))
        return w_global
