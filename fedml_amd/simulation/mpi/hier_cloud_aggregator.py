"""Cloud-side aggregator of MPI hierarchical FL with topology mixing (reference: python/fedml/
simulation/mpi/hierarchical_fl/HierFedAvgCloudAggregator.py:13-195 -- the fork's own code).

Each edge (group) server sends the list of models of its ``group_comm_round`` group rounds plus
their sample counts.  Results are bit-identical to the reference, including two of its quirks:

* ``aggregate`` averages every group round, then averages the LAST round's model list a second
  time, after the first pass overwrote edge 0's entry with that round's average (:73-96); the
  returned "global" model is therefore ``(avg*n_0)/N + sum_{e>=1} (x_e*n_e)/N``;
* ``mix`` returns the last round's mixed edge models except edge 0's, which the reference's
  ``_pfedavg_aggregation_`` replaced in place by the average of all mixed models (:123-138).

Formulas: ``_fedavg_aggregation_`` = (x*n)/N (MUL_N_DIV_N); ``_pfedavg_aggregation_`` =
(x*1)/K (MUL_N_DIV_N with n = 1); ``_pfedavg_mixing_`` = dense row of W, zeros included, ascending
(one fa_mix launch per key for ALL edges).
"""
from __future__ import annotations

import logging
import time
from typing import Dict, List, Tuple

import numpy as np

from ...core.distributed.topology.topology_manager import dense_rows
from ...ml.aggregator.state_dict_agg import MUL_N_DIV_N, aggregate, mix


class HierFedAVGCloudAggregator:
    def __init__(self, worker_num: int, server_aggregator=None, args=None):
        self.worker_num = worker_num
        self.aggregator = server_aggregator
        self.args = args
        self.model_dict: Dict[int, List[Tuple[int, dict]]] = {}
        self.sample_num_dict: Dict[int, List[int]] = {}
        self.flag_client_model_uploaded_dict = {i: False for i in range(worker_num)}

    def set_global_model_params(self, params):
        if self.aggregator:
            self.aggregator.set_model_params(params)

    def add_local_trained_result(self, index, model_list, sample_num_list):
        """model_list = [(global_round_idx, state_dict) per group round] (HierFedAvgCloudManager.py)."""
        self.model_dict[index] = model_list
        self.sample_num_dict[index] = sample_num_list
        self.flag_client_model_uploaded_dict[index] = True

    def check_whether_all_receive(self) -> bool:
        if not all(self.flag_client_model_uploaded_dict[i] for i in range(self.worker_num)):
            return False
        for i in range(self.worker_num):
            self.flag_client_model_uploaded_dict[i] = False
        return True

    def _round_list(self, r):
        return [(self.sample_num_dict[e][r], self.model_dict[e][r][1]) for e in range(self.worker_num)]

    def aggregate(self):
        t0 = time.time()
        rounds = len(self.sample_num_dict[0])
        model_list, averaged = None, None
        for r in range(rounds):
            model_list = self._round_list(r)
            averaged = self._fedavg_aggregation_(model_list)
            self.set_global_model_params(averaged)
        # the reference's second pass reads edge 0's entry, which its first pass overwrote
        model_list = [(model_list[0][0], averaged)] + model_list[1:]
        averaged = self._fedavg_aggregation_(model_list)
        self.set_global_model_params(averaged)
        logging.info("aggregate time cost: %.6f s", time.time() - t0)
        return averaged

    def mix(self, topology_manager):
        t0 = time.time()
        W = np.asarray(topology_manager.topology, dtype=np.float32)
        rounds = len(self.sample_num_dict[0])
        mixed, averaged = None, None
        for r in range(rounds):
            model_list = self._round_list(r)
            mixed, _ = mix([p for _, p in model_list], *dense_rows(W))
            averaged = self._pfedavg_aggregation_([(self.sample_num_dict[e][r], mixed[e])
                                                   for e in range(self.worker_num)])
            self.set_global_model_params(averaged)
        logging.info("mix time cost: %.6f s", time.time() - t0)
        return [averaged] + mixed[1:]

    @staticmethod
    def _fedavg_aggregation_(model_list):
        counts = [n for n, _ in model_list]
        return aggregate([p for _, p in model_list], MUL_N_DIV_N, counts, float(sum(counts)))

    @staticmethod
    def _pfedavg_aggregation_(model_list):
        K = len(model_list)
        return aggregate([p for _, p in model_list], MUL_N_DIV_N, [1] * K, float(K))

    @staticmethod
    def _pfedavg_mixing_(model_list, neighbor_topo_weight_list):
        w = np.asarray(neighbor_topo_weight_list, dtype=np.float32)
        K = len(model_list)
        rows, _ = mix([p for _, p in model_list], [0, K], list(range(K)), [float(v) for v in w])
        return rows[0]
