"""ServerAggregator plugin surface (reference: python/fedml/core/alg_frame/server_aggregator.py:13-124).

Same abstract methods and hook names/signatures as the reference, so a user's
``MyServerAggregator(ServerAggregator)`` (e.g. examples/cross_silo/mpi_customized_fedavg_mnist_lr_example/
my_server_aggregator.py:11-29 in the reference) runs unchanged; ``aggregate`` routes through the
MI355X engine (``FedMLAggOperator.agg``).

The reference's hooks also drive its DP / attack / defense / contribution subsystems
(core/dp, core/security, core/contribution).  Defenses that ARE alternative aggregations --
krum / multikrum, trimmed_mean, wise_median (coordinate-wise median) -- run here through
``FedMLDefender`` on the HIP engine, with the reference's hook order.  DP, attacks, contribution
assessment and the other defenses are outside this engine's scope: the hooks pass data through
untouched when they are off (the default), and raise NotImplementedError if a config turns one on.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from collections import OrderedDict
from typing import List, Tuple

from ...ml.aggregator.agg_operator import FedMLAggOperator
from ..security.fedml_defender import FedMLDefender

_OUT_OF_SCOPE_FLAGS = ("enable_dp", "enable_attack", "enable_contribution")


def _check_hooks_off(args):
    for flag in _OUT_OF_SCOPE_FLAGS:
        if getattr(args, flag, False):
            raise NotImplementedError(
                f"args.{flag}=True: the DP/attack/defense/contribution subsystems are not part of the "
                "MI355X aggregation engine")


class ServerAggregator(ABC):
    """Abstract server-side aggregator (reference server_aggregator.py:13)."""

    def __init__(self, model, args):
        self.model = model
        self.id = 0
        self.args = args
        self.eval_data = None
        self.final_contribution_assigment_dict = dict()
        _check_hooks_off(args)
        FedMLDefender.get_instance().init(args)

    def is_main_process(self):
        return True

    def set_id(self, aggregator_id):
        self.id = aggregator_id

    @abstractmethod
    def get_model_params(self):
        ...

    @abstractmethod
    def set_model_params(self, model_parameters):
        ...

    def on_before_aggregation(self, raw_client_model_or_grad_list: List[Tuple[float, OrderedDict]]):
        """Reference :42-65: before-aggregation defenses (krum, multikrum, trimmed_mean) select the
        clients; otherwise the identity."""
        client_idxs = [i for i in range(len(raw_client_model_or_grad_list))]
        d = FedMLDefender.get_instance()
        if d.is_defense_enabled():
            raw_client_model_or_grad_list = d.defend_before_aggregation(
                raw_client_grad_list=raw_client_model_or_grad_list, extra_auxiliary_info=self.get_model_params())
            client_idxs = d.get_benign_client_idxs(client_idxs=client_idxs)
        return raw_client_model_or_grad_list, client_idxs

    def aggregate(self, raw_client_model_or_grad_list: List[Tuple[float, OrderedDict]]):
        """Reference :67-76 -> the on-aggregation defense (wise_median) or FedMLAggOperator.agg."""
        d = FedMLDefender.get_instance()
        if d.is_defense_enabled():
            return d.defend_on_aggregation(raw_client_grad_list=raw_client_model_or_grad_list,
                                           base_aggregation_func=FedMLAggOperator.agg,
                                           extra_auxiliary_info=self.get_model_params())
        return FedMLAggOperator.agg(self.args, raw_client_model_or_grad_list)

    def on_after_aggregation(self, aggregated_model_or_grad: OrderedDict) -> OrderedDict:
        """Reference :78-86. With central DP off and the served defenses this is the identity."""
        d = FedMLDefender.get_instance()
        if d.is_defense_enabled():
            aggregated_model_or_grad = d.defend_after_aggregation(aggregated_model_or_grad)
        return aggregated_model_or_grad

    def assess_contribution(self):
        """Reference :88-117 (contribution assessment subsystem, off by default)."""
        return None

    @abstractmethod
    def test(self, test_data, device, args):
        ...

    def test_all(self, train_data_local_dict, test_data_local_dict, device, args) -> bool:
        return False
