"""FedAvg_seq two-level reduce (reference: python/fedml/simulation/mpi/fedavg_seq/
FedAvgClientManager.py:67-73 add_client_model, FedAVGAggregator.py:189-236).

Worker side: each worker simulates several clients and accumulates ``partial += x_i * w_i`` with
the server's weights ``w_i = n_i / N`` (get_average_weight).  Server side: plain ordered sum of the
worker partials.  Both on the MI355X engine:

* ``worker_partial`` folds a worker's whole client list in ONE launch per dtype group;
* ``add_client_model`` is the incremental form for clients that arrive one at a time: the
  reference's ``partial[k] += p * w`` equals the engine's ordered sum over [partial, p] with
  coefficients [1.0, w] (``partial * 1.0`` is exact for every float, incl. -0, NaN, subnormals).
"""
from __future__ import annotations

from typing import Dict, List, Sequence

from ...ml.aggregator.state_dict_agg import MUL_W, SUM, aggregate


def get_average_weight(sample_nums: Dict[int, int], client_indexes: Sequence[int]) -> Dict[int, float]:
    """fedavg_seq/FedAVGAggregator.py:189-199: Python float64 n_i / N over the sampled clients."""
    total = sum(sample_nums[c] for c in client_indexes)
    return {c: sample_nums[c] / total for c in client_indexes}


def worker_partial(client_params: Sequence[dict], weights: Sequence[float]):
    """The worker's accumulated partial over its clients, in order (one launch per dtype)."""
    return aggregate(list(client_params), MUL_W, list(weights))


def add_client_model(local_agg_model_params: dict, model_params: dict, weight: float = 1.0):
    """In-place-compatible incremental form of FedAvgClientManager.add_client_model (:67-73)."""
    if not local_agg_model_params:
        local_agg_model_params.update(aggregate([model_params], MUL_W, [weight]))
        return local_agg_model_params
    missing = [k for k in model_params if k not in local_agg_model_params]
    if missing:
        local_agg_model_params.update(aggregate([{k: model_params[k] for k in missing}], MUL_W, [weight]))
    present = {k: local_agg_model_params[k] for k in model_params if k not in missing}
    if present:
        # an integer buffer was promoted to float32 by the first `p * w`; `int * w` == fp32(int) * w
        incoming = {k: (model_params[k].to(present[k].dtype)
                        if present[k].is_floating_point() and not model_params[k].is_floating_point()
                        else model_params[k]) for k in present}
        upd = aggregate([present, incoming], MUL_W, [1.0, weight])
        local_agg_model_params.update(upd)
    return local_agg_model_params


def server_aggregate(worker_partials: List[dict]):
    """fedavg_seq/FedAVGAggregator.py:201-236: ordered plain sum of the non-empty partials."""
    return aggregate([p for p in worker_partials if len(p) > 0], SUM)
