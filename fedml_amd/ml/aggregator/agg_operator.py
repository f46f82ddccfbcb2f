"""Drop-in FedMLAggOperator on the MI355X engine.

Mirrors python/fedml/ml/aggregator/agg_operator.py of the reference (liuliuliu0605/FedML):
same class/function names, same arguments (``agg(args, raw_grad_list)``, positional or keyword),
same ``args.federated_optimizer`` switch, same outputs bit-for-bit (pinned by tests/golden/), and
the same exceptions for the same misuse.  What differs is where the arithmetic runs: every
branch is a handful of launches of the HIP kernels in fedml_amd/csrc/fedagg.hip instead of
2*K*#keys PyTorch-CPU ops.

Deliberate differences (no caller depends on them):
* the reference writes the result into client 0's dict (``avg_params = raw_grad_list[0][1]``,
  agg_operator.py:36) and, in the plain-sum branches, adds in place into client 0's tensors;
  this operator returns new tensors and leaves every input untouched;
* tf / jax / mxnet engines (agg_operator.py:137-220) operate on non-torch containers and are not
  part of the MI355X engine: selecting one raises NotImplementedError.
"""
from __future__ import annotations

import logging
from collections import OrderedDict
from typing import List, Tuple

from .state_dict_agg import MUL_W, SUM, aggregate

# args.ml_engine values (python/fedml/core/common/ml_engine_backend.py)
ML_ENGINE_FLAG = "ml_engine"
_TORCH = "torch"
_UNSUPPORTED_ENGINES = ("tf", "jax", "mxnet")


class FedMLAggOperator:
    @staticmethod
    def agg(args, raw_grad_list: List[Tuple[float, OrderedDict]]) -> OrderedDict:
        """Reference: agg_operator.py:9-30.  N = sum of the clients' sample counts."""
        opt = args.federated_optimizer
        if opt in ("SCAFFOLD", "Mime"):
            training_num = sum(n for n, _, _ in raw_grad_list)
        else:
            training_num = sum(n for n, _ in raw_grad_list)
        return model_aggregator(args, raw_grad_list, training_num)


def torch_aggregator(args, raw_grad_list, training_num):
    """Reference: agg_operator.py:33-134, one branch per federated optimizer."""
    opt = args.federated_optimizer
    if opt in ("FedAvg", "FedProx"):
        counts = [n for n, _ in raw_grad_list]
        return aggregate([p for _, p in raw_grad_list], MUL_W, [n / training_num for n in counts])
    if opt in ("FedAvg_seq", "FedDyn"):
        raw_grad_list[0]  # IndexError on an empty list, like the reference
        return aggregate([p for _, p in raw_grad_list], SUM)
    if opt in ("FedOpt", "FedNova"):
        # the reference's branch is `pass`, then `return avg_params` on an unbound local
        raise UnboundLocalError("local variable 'avg_params' referenced before assignment")
    if opt == "SCAFFOLD":
        # agg_operator.py:100-118: the loop's weighted sum is overwritten after the loop by the
        # LAST client's weights delta (for K = 1: client 0's x0 * w0) and the last client's
        # control-variate delta times 1 / client_num_in_total.  Only that result is computed.
        K = len(raw_grad_list)
        n0, w_last, c_last = raw_grad_list[-1]
        if K == 1:
            weights = aggregate([w_last], MUL_W, [n0 / training_num])
        else:
            weights = aggregate([w_last], SUM)
        c = aggregate([c_last], MUL_W, [1 / args.client_num_in_total])
        return weights, c
    if opt == "Mime":
        # agg_operator.py:120-133
        assert args.client_num_per_round == len(raw_grad_list)
        w = [n / training_num for n, _, _ in raw_grad_list]
        params = aggregate([p for _, p, _ in raw_grad_list], MUL_W, w)
        grads = aggregate([g for _, _, g in raw_grad_list], MUL_W, w)
        return params, grads
    # unknown optimizer string: the reference reaches `return avg_params` unbound
    raise UnboundLocalError("local variable 'avg_params' referenced before assignment")


def model_aggregator(args, raw_grad_list, training_num):
    """Reference: agg_operator.py:223-234 (engine dispatch on args.ml_engine)."""
    engine = getattr(args, ML_ENGINE_FLAG, _TORCH)
    if engine in _UNSUPPORTED_ENGINES:
        raise NotImplementedError(f"ml_engine={engine!r}: the MI355X aggregation engine aggregates torch tensors")
    return torch_aggregator(args, raw_grad_list, training_num)


logging.getLogger(__name__).addHandler(logging.NullHandler())
