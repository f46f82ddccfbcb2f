"""FedMLDefender singleton (reference: python/fedml/core/security/fedml_defender.py:40-196) for the
robust aggregators of this engine: krum / multikrum, trimmed_mean and wise_median.  Same dispatch
(which defenses act before / on / after aggregation) and the same entry points; the per-element work
runs in the HIP kernels (fedml_amd/csrc/robust.hip).  Other defense types of the reference are
outside the aggregation path and raise NotImplementedError when configured.
"""
from __future__ import annotations

import logging
from collections import OrderedDict
from typing import Any, Callable, List, Tuple

from .constants import DEFENSE_KRUM, DEFENSE_MULTIKRUM, DEFENSE_TRIMMED_MEAN, DEFENSE_WISE_MEDIAN
from .defense.coordinate_wise_median_defense import CoordinateWiseMedianDefense
from .defense.coordinate_wise_trimmed_mean_defense import CoordinateWiseTrimmedMeanDefense
from .defense.krum_defense import KrumDefense


class FedMLDefender:
    _defender_instance = None

    @staticmethod
    def get_instance():
        if FedMLDefender._defender_instance is None:
            FedMLDefender._defender_instance = FedMLDefender()
        return FedMLDefender._defender_instance

    def __init__(self):
        self.is_enabled = False
        self.defense_type = None
        self.defender = None

    def init(self, args):
        if hasattr(args, "enable_defense") and args.enable_defense:
            self.args = args
            logging.info("------init defense..." + args.defense_type)
            self.is_enabled = True
            self.defense_type = args.defense_type.strip()
            if self.defense_type in (DEFENSE_KRUM, DEFENSE_MULTIKRUM):
                self.defender = KrumDefense(args)
            elif self.defense_type == DEFENSE_WISE_MEDIAN:
                self.defender = CoordinateWiseMedianDefense(args)
            elif self.defense_type == DEFENSE_TRIMMED_MEAN:
                self.defender = CoordinateWiseTrimmedMeanDefense(args)
            else:
                raise NotImplementedError(
                    f"defense_type {self.defense_type!r} is not served by the MI355X engine "
                    f"(supported: krum, multikrum, trimmed_mean, wise_median)")
        else:
            self.is_enabled = False
            self.defense_type = None
            self.defender = None

    def is_defense_enabled(self):
        return self.is_enabled

    def is_defense_on_aggregation(self):
        return self.is_defense_enabled() and self.defense_type in [DEFENSE_WISE_MEDIAN]

    def is_defense_before_aggregation(self):
        return self.is_defense_enabled() and self.defense_type in [DEFENSE_KRUM, DEFENSE_MULTIKRUM,
                                                                   DEFENSE_TRIMMED_MEAN]

    def is_defense_after_aggregation(self):
        return False

    def defend_before_aggregation(self, raw_client_grad_list: List[Tuple[float, OrderedDict]],
                                  extra_auxiliary_info: Any = None):
        if self.defender is None:
            raise Exception("defender is not initialized!")
        if self.is_defense_before_aggregation():
            return self.defender.defend_before_aggregation(raw_client_grad_list, extra_auxiliary_info)
        return raw_client_grad_list

    def defend_on_aggregation(self, raw_client_grad_list: List[Tuple[float, OrderedDict]],
                              base_aggregation_func: Callable = None, extra_auxiliary_info: Any = None):
        if self.defender is None:
            raise Exception("defender is not initialized!")
        if self.is_defense_on_aggregation():
            return self.defender.defend_on_aggregation(raw_client_grad_list, base_aggregation_func,
                                                       extra_auxiliary_info)
        return base_aggregation_func(args=self.args, raw_grad_list=raw_client_grad_list)

    def defend_after_aggregation(self, global_model):
        if self.defender is None:
            raise Exception("defender is not initialized!")
        return global_model

    def get_malicious_client_idxs(self):
        return self.defender.get_malicious_client_idxs() if hasattr(self.defender, "get_malicious_client_idxs") else []

    def get_benign_client_idxs(self, client_idxs):
        return [i for i in client_idxs if i not in self.get_malicious_client_idxs()]
