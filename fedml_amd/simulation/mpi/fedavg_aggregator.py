"""MPI-simulation FedAvg server aggregator (reference: python/fedml/simulation/mpi/fedavg/
FedAVGAggregator.py:15-116), transport-agnostic.

Collects one ``(sample_num, state_dict)`` per worker, then aggregates with the MPI simulator's
formula ``avg[k] += (x_i[k] * n_i) / N`` (FedAVGAggregator.py:99-116) -- a different rounding
than FedMLAggOperator.agg's ``x * (n/N)``, reproduced bit-for-bit by the engine's MUL_N_DIV_N mode.
"""
from __future__ import annotations

import logging
import time
from typing import Dict, List, Tuple

from ...ml.aggregator.ingest import ArrivalIngest
from ...ml.aggregator.state_dict_agg import fedavg_xn_div_n


class FedAVGAggregator:
    def __init__(self, worker_num: int, server_aggregator=None, args=None, device="cuda"):
        self.worker_num = worker_num
        # on-arrival ingest into HBM (the reference keeps the unpickled CPU dicts and loops over
        # them on the CPU after the last arrival): fedml_amd/ml/aggregator/ingest.py
        self.ingest = ArrivalIngest(worker_num, device) if ArrivalIngest.wants(device) else None
        self.aggregator = server_aggregator
        self.args = args
        self.model_dict: Dict[int, dict] = {}
        self.sample_num_dict: Dict[int, int] = {}
        self.flag_client_model_uploaded_dict = {i: False for i in range(worker_num)}

    def get_global_model_params(self):
        return self.aggregator.get_model_params() if self.aggregator else None

    def set_global_model_params(self, model_parameters):
        if self.aggregator:
            self.aggregator.set_model_params(model_parameters)

    def add_local_trained_result(self, index, model_params, sample_num):
        host = not any(getattr(v, "is_cuda", False) for v in model_params.values())
        if self.ingest is not None and type(model_params) is not dict and host:
            self.ingest.add(index, model_params)  # else: aggregated where it is (host path)
        self.model_dict[index] = model_params
        self.sample_num_dict[index] = sample_num
        self.flag_client_model_uploaded_dict[index] = True

    def check_whether_all_receive(self) -> bool:
        if not all(self.flag_client_model_uploaded_dict[i] for i in range(self.worker_num)):
            return False
        for i in range(self.worker_num):
            self.flag_client_model_uploaded_dict[i] = False
        return True

    def aggregate(self):
        t0 = time.time()
        model_list = [(self.sample_num_dict[i], self.model_dict[i]) for i in range(self.worker_num)]
        averaged = self._fedavg_aggregation_(model_list)
        if self.ingest is not None:
            # the reference's result stays on the host (CPU inputs): a pinned copy, which is also
            # what the MPI send of the global model pickles
            averaged = self.ingest.to_host(averaged)
            self.ingest.round_done()
        self.set_global_model_params(averaged)
        logging.info("aggregate time cost: %.6f s", time.time() - t0)
        return averaged

    @staticmethod
    def _fedavg_aggregation_(model_list: List[Tuple[int, dict]]):
        return fedavg_xn_div_n([p for _, p in model_list], [n for n, _ in model_list])
