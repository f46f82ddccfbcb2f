"""Two-level (group -> global) FedAvg, single process (reference: python/fedml/simulation/sp/
hierarchical_fl/group.py:43-66 and trainer.py:78-122).

Group step: FedAvg over the group's clients, weights n_i / N_group (Group inherits FedAvgAPI's
_aggregate).  Global step: FedAvg over the group models, weights N_group / N_total
(trainer.py:100-110).  Both run on the MI355X engine.  The multi-GPU version (one group per GPU,
RCCL for the global step) is fedml_amd.distributed.group_reduce.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

from ...ml.aggregator.state_dict_agg import fedavg


def group_aggregate(w_locals: Sequence[Tuple[int, dict]]):
    """One group's FedAvg (group.py:60-62 -> FedAvgAPI._aggregate)."""
    return fedavg([p for _, p in w_locals], [n for n, _ in w_locals])


def hierarchical_round(groups: Dict[int, Sequence[Tuple[int, dict]]]):
    """groups[g] = [(n_i, state_dict_i) for the group's sampled clients] -> global state_dict.

    Groups are visited in sorted order (trainer.py:97); each group's weight is its summed sample
    count (group.py:37-41)."""
    w_groups: List[Tuple[int, dict]] = []
    for g in sorted(groups):
        members = groups[g]
        w_groups.append((sum(n for n, _ in members), group_aggregate(members)))
    return fedavg([p for _, p in w_groups], [n for n, _ in w_groups])
