"""ServerAggregator plugin surface (reference: python/fedml/core/alg_frame/server_aggregator.py:13-124).

Same abstract methods and hook names/signatures as the reference, so a user's
``MyServerAggregator(ServerAggregator)`` (e.g. examples/cross_silo/mpi_customized_fedavg_mnist_lr_example/
my_server_aggregator.py:11-29 in the reference) runs unchanged; ``aggregate`` routes through the
MI355X engine (``FedMLAggOperator.agg``).

The reference's hooks also drive its DP / attack / defense / contribution subsystems
(core/dp, core/security, core/contribution).  Those are outside this engine's scope: the hooks
pass data through untouched when they are off (the default), and raise NotImplementedError if a
config turns one on, instead of silently skipping it.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from collections import OrderedDict
from typing import List, Tuple

from ...ml.aggregator.agg_operator import FedMLAggOperator

_OUT_OF_SCOPE_FLAGS = ("enable_dp", "enable_attack", "enable_defense", "enable_contribution")


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
        """Reference :42-65. With DP clipping / attacks / defenses off this is the identity."""
        return raw_client_model_or_grad_list, list(range(len(raw_client_model_or_grad_list)))

    def aggregate(self, raw_client_model_or_grad_list: List[Tuple[float, OrderedDict]]):
        """Reference :67-76 -> FedMLAggOperator.agg(self.args, list)."""
        return FedMLAggOperator.agg(self.args, raw_client_model_or_grad_list)

    def on_after_aggregation(self, aggregated_model_or_grad: OrderedDict) -> OrderedDict:
        """Reference :78-86. With central DP / defenses off this is the identity."""
        return aggregated_model_or_grad

    def assess_contribution(self):
        """Reference :88-117 (contribution assessment subsystem, off by default)."""
        return None

    @abstractmethod
    def test(self, test_data, device, args):
        ...

    def test_all(self, train_data_local_dict, test_data_local_dict, device, args) -> bool:
        return False
