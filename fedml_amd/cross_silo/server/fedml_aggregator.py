"""Cross-silo server round aggregator (reference: python/fedml/cross_silo/server/fedml_aggregator.py:
13-104) -- the production plugin path: collect K client updates, then
``on_before_aggregation -> aggregate -> on_after_aggregation`` on the user's ServerAggregator.

Client updates arrive as host state_dicts (the transports unpickle CPU tensors).  Where the
reference moves every tensor to the server device one by one on arrival
(``model_params_to_device``, ml/engine/ml_engine_adapter.py:234-254), this aggregator leaves them
where they are: the engine stages host tensors to the GPU inside ``aggregate`` (one launch per
dtype group for the whole round).
"""
from __future__ import annotations

import logging
import time
from typing import Dict


class FedMLAggregator:
    def __init__(self, client_num: int, device, args, server_aggregator):
        self.client_num = client_num
        self.device = device
        self.args = args
        if args is not None:
            args.device = device
        self.aggregator = server_aggregator
        self.model_dict: Dict[int, dict] = {}
        self.sample_num_dict: Dict[int, float] = {}
        self.flag_client_model_uploaded_dict = {i: False for i in range(client_num)}

    def get_global_model_params(self):
        return self.aggregator.get_model_params()

    def set_global_model_params(self, model_parameters):
        self.aggregator.set_model_params(model_parameters)

    def add_local_trained_result(self, index, model_params, sample_num):
        self.model_dict[index] = model_params
        self.sample_num_dict[index] = sample_num
        self.flag_client_model_uploaded_dict[index] = True

    def check_whether_all_receive(self) -> bool:
        if not all(self.flag_client_model_uploaded_dict[i] for i in range(self.client_num)):
            return False
        for i in range(self.client_num):
            self.flag_client_model_uploaded_dict[i] = False
        return True

    def aggregate(self):
        t0 = time.time()
        model_list = [(self.sample_num_dict[i], self.model_dict[i]) for i in range(self.client_num)]
        model_list, model_list_idxes = self.aggregator.on_before_aggregation(model_list)
        averaged = self.aggregator.aggregate(model_list)
        if isinstance(averaged, dict) and not _is_state_dict(averaged):
            # per-client results (the reference's {client_index: params} form, :86-94)
            count = len(averaged) - 1 if len(averaged) == self.client_num + 1 else len(averaged)
            for ci in range(count):
                averaged[ci] = self.aggregator.on_after_aggregation(averaged[ci])
        else:
            averaged = self.aggregator.on_after_aggregation(averaged)
        self.set_global_model_params(averaged)
        logging.info("aggregate time cost: %.6f s", time.time() - t0)
        return averaged, model_list, model_list_idxes


def _is_state_dict(d) -> bool:
    return all(isinstance(k, str) for k in d.keys())
