"""Cross-silo server round aggregator (reference: python/fedml/cross_silo/server/fedml_aggregator.py:
13-104) -- the production plugin path: collect K client updates, then
``on_before_aggregation -> aggregate -> on_after_aggregation`` on the user's ServerAggregator.

Client updates arrive as host state_dicts (the transports unpickle CPU tensors).  The reference
moves every non-``dict`` update to the server device on arrival, tensor by tensor and in place
(``model_params_to_device``, ml/engine/ml_engine_adapter.py:234-254, fedml_aggregator.py:57-66).
Here the arriving update is adopted into a row of a double-buffered ClientArena instead
(fedml_amd/ml/aggregator/ingest.py): pinned staging + one H2D per dtype group on a copy stream,
overlapped with waiting for the next client, the dict's entries rebound to the row's device views.
``aggregate`` then runs the user's ServerAggregator as the reference does; the default path
(FedMLAggOperator.agg) recognises the arena-resident updates and reduces the rows in one launch
per dtype group.  ``get_global_model_params_host`` hands the result to the broadcast as pinned
host tensors (fedml_server_manager.py:217-231 sends the global model).
"""
from __future__ import annotations

import logging
import time
from typing import Dict

from ...ml.aggregator.ingest import ArrivalIngest, move_to_device


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
        self.ingest = ArrivalIngest(client_num, device) if ArrivalIngest.wants(device) else None
        self._global_host = None

    def get_global_model_params(self):
        return self.aggregator.get_model_params()

    def set_global_model_params(self, model_parameters):
        self.aggregator.set_model_params(model_parameters)

    def add_local_trained_result(self, index, model_params, sample_num):
        # a plain ``dict`` stays where the user put it (reference :59-62); anything else is moved
        # to the server device on arrival -- here into this round's arena row
        if type(model_params) is not dict and self.ingest is not None:
            if not self.ingest.add(index, model_params):
                model_params = move_to_device(model_params, self.device)
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
        self._global_host = None
        if self.ingest is not None:
            if _is_state_dict(averaged):
                self._global_host = self.ingest.to_host(averaged)
            self.ingest.round_done()
        logging.info("aggregate time cost: %.6f s", time.time() - t0)
        return averaged, model_list, model_list_idxes

    def get_global_model_params_host(self):
        """The last aggregated global model in pinned host memory, ready for the broadcast
        (fedml_server_manager.py:217-231); falls back to the ServerAggregator's params."""
        return self._global_host if self._global_host is not None else self.get_global_model_params()


def _is_state_dict(d) -> bool:
    return all(isinstance(k, str) for k in d.keys())
