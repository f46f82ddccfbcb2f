"""Drop-in for python/fedml/core/security/defense/coordinate_wise_trimmed_mean_defense.py.

Despite its name the reference does not trim per coordinate: ``trimmed_mean`` (common/utils.py:
213-227) stably sorts the CLIENTS by their sample count and drops ``int(beta * K)`` from each end;
the server then averages the survivors with its base aggregation (FedAvg on the HIP engine).
That selection is host-side list logic and is reproduced exactly (tests/golden/g17_*).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Any, List, Tuple

from ..common.utils import trimmed_mean


class CoordinateWiseTrimmedMeanDefense(object):
    def __init__(self, config):
        self.beta = config.beta

    def defend_before_aggregation(self, raw_client_grad_list: List[Tuple[float, OrderedDict]],
                                  extra_auxiliary_info: Any = None):
        if self.beta > 1 / 2 or self.beta < 0:
            raise ValueError("the bound of beta is [0, 1/2)")
        return trimmed_mean(raw_client_grad_list, int(self.beta * len(raw_client_grad_list)))
