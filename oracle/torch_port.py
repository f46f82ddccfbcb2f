"""Op-for-op PyTorch-CPU restatement of the reference aggregation loops -- TEST INFRASTRUCTURE ONLY.

Each function issues the same tensor ops, in the same order, as the reference function it cites
(paths relative to liuliuliu0605/FedML ``python/fedml/``), so it reproduces both the reference's
results (pinned bit-for-bit against tests/golden/) and its CPU cost (``bench.py`` times it as the
``cpu_baseline``; the reference's own files never travel to the GPU box).

Deliberate difference: the reference rebinds keys of client 0's dict (and, in the plain-sum
branches, adds in place into client 0's tensors).  The port works on a shallow copy of that dict
and clones where the reference would add into a caller tensor, so callers' inputs survive.
"""
from __future__ import annotations

import copy
from collections import OrderedDict


def torch_aggregator(optimizer, raw_grad_list, training_num, client_num_in_total=None,
                     client_num_per_round=None):
    """ml/aggregator/agg_operator.py:33-134 (torch_aggregator)."""
    if optimizer in ("FedAvg", "FedProx"):                     # :35-54
        avg = OrderedDict(raw_grad_list[0][1])
        for k in avg.keys():
            for i, (n_i, params) in enumerate(raw_grad_list):
                w = n_i / training_num
                if i == 0:
                    avg[k] = params[k] * w
                else:
                    avg[k] += params[k] * w
        return avg
    if optimizer in ("FedAvg_seq", "FedDyn"):                   # :55-63, :68-77
        avg = OrderedDict(raw_grad_list[0][1])
        for k in avg.keys():
            for i, (_, params) in enumerate(raw_grad_list):
                if i == 0:
                    avg[k] = params[k].clone()  # reference aliases client 0's tensor here
                else:
                    avg[k] += params[k]
        return avg
    if optimizer in ("FedOpt", "FedNova"):                      # :64-67 -> `return avg_params` unbound
        raise UnboundLocalError("local variable 'avg_params' referenced before assignment")
    if optimizer == "SCAFFOLD":                                 # :100-118
        _, tw0, tc0 = raw_grad_list[0]
        tw, tc = OrderedDict(tw0), OrderedDict(tc0)
        for k in tw.keys():
            for i, (n_i, wd, cd) in enumerate(raw_grad_list):
                w = n_i / training_num
                if i == 0:
                    tw[k] = wd[k] * w
                    tc[k] = cd[k].clone()
                else:
                    tw[k] += wd[k] * w
                    tc[k] += cd[k]
            w_c = 1 / client_num_in_total
            # defect kept: overwrite with the LAST client's entries (for K = 1 that is client 0's
            # already-rebound x0*w0 in the reference, i.e. tw[k] itself)
            tw[k] = tw[k] if len(raw_grad_list) == 1 else wd[k]
            tc[k] = cd[k] * w_c
        return tw, tc
    if optimizer == "Mime":                                     # :120-133
        _, p0, g0 = raw_grad_list[0]
        assert client_num_per_round == len(raw_grad_list)
        avg, avg_g = OrderedDict(p0), OrderedDict(g0)
        for k in avg.keys():
            for i, (n_i, params, grads) in enumerate(raw_grad_list):
                w = n_i / training_num
                if i == 0:
                    avg[k] = params[k] * w
                    avg_g[k] = grads[k] * w
                else:
                    avg[k] += params[k] * w
                    avg_g[k] += grads[k] * w
        return avg, avg_g
    return None  # unknown optimizer: the reference falls through and returns its unbound name


def agg(optimizer, raw_grad_list, client_num_in_total=None, client_num_per_round=None):
    """ml/aggregator/agg_operator.py:9-30 (FedMLAggOperator.agg)."""
    training_num = sum(t[0] for t in raw_grad_list)
    return torch_aggregator(optimizer, raw_grad_list, training_num, client_num_in_total,
                            client_num_per_round)


def sp_aggregate(w_locals):
    """simulation/sp/fedavg/fedavg_api.py:144-159 (FedAvgAPI._aggregate)."""
    return torch_aggregator("FedAvg", w_locals, sum(n for n, _ in w_locals))


def mpi_fedavg(model_list):
    """simulation/mpi/fedavg/FedAVGAggregator.py:99-116 ((x * n) / N)."""
    N = sum(n for n, _ in model_list)
    avg = OrderedDict(model_list[0][1])
    for k in avg.keys():
        for i, (n_i, params) in enumerate(model_list):
            if i == 0:
                avg[k] = params[k] * n_i / N
            else:
                avg[k] += params[k] * n_i / N
    return avg


def pfedavg_aggregation(model_list):
    """HierFedAvgCloudAggregator.py:159-172 ((x * 1) / K)."""
    K = len(model_list)
    avg = OrderedDict(model_list[0][1])
    for k in avg.keys():
        for i, (_, params) in enumerate(model_list):
            if i == 0:
                avg[k] = params[k] * 1 / K
            else:
                avg[k] += params[k] * 1 / K
    return avg


def pfedavg_mixing(model_list, weights):
    """HierFedAvgCloudAggregator.py:174-195 (dense row of W, zeros included, ascending j)."""
    avg = copy.deepcopy(model_list[0][1])  # the reference deep-copies client 0's dict
    for k in avg.keys():
        for i, (_, params) in enumerate(model_list):
            if i == 0:
                avg[k] = params[k] * weights[i]
            else:
                avg[k] += params[k] * weights[i]
    return avg


def cloud_aggregate(sample_num_dict, model_dict, worker_num):
    """HierFedAvgCloudAggregator.py:67-103 incl. the second application over the last round.

    model_dict[e][r] = (global_round_idx, state_dict).  The reference's first call rebinds the
    keys of edge 0's round-r dict to the round-r average; the second call then reads that dict.
    """
    R = len(sample_num_dict[0])
    model_list = None
    for r in range(R):
        model_list = [(sample_num_dict[e][r], model_dict[e][r][1]) for e in range(worker_num)]
        avg = mpi_fedavg(model_list)
    model_list = [(model_list[0][0], avg)] + model_list[1:]
    return mpi_fedavg(model_list)


def cloud_mix(sample_num_dict, model_dict, worker_num, W):
    """HierFedAvgCloudAggregator.py:105-138: per group round mix every edge, then average.

    Returned list = mixed models of the LAST group round, except entry 0, which the reference's
    _pfedavg_aggregation_ overwrote in place with the average.
    """
    R = len(sample_num_dict[0])
    edge = None
    for r in range(R):
        model_list = [(sample_num_dict[e][r], model_dict[e][r][1]) for e in range(worker_num)]
        edge = [(sample_num_dict[e][r], pfedavg_mixing(model_list, W[e])) for e in range(worker_num)]
        avg = pfedavg_aggregation(edge)
    return [avg] + [m for _, m in edge[1:]]


def fedavg_seq_worker(partial, params, weight):
    """simulation/mpi/fedavg_seq/FedAvgClientManager.py:67-73 (add_client_model)."""
    for name, p in params.items():
        if name not in partial:
            partial[name] = p * weight
        else:
            partial[name] += p * weight
    return partial


def fedavg_seq_weights(counts):
    """fedavg_seq/FedAVGAggregator.py:189-199 (get_average_weight): Python float64 n_i / N."""
    N = sum(counts)
    return [c / N for c in counts]


def fedavg_seq_server(partials):
    """fedavg_seq/FedAVGAggregator.py:201-236 (plain ordered sum of the worker partials)."""
    avg = OrderedDict(partials[0])
    for k in avg.keys():
        for i, p in enumerate(partials):
            if i == 0:
                avg[k] = p[k].clone()
            else:
                avg[k] += p[k]
    return avg


def dsgd_update(x_self, self_weight, neighbours):
    """sp/decentralized/client_dsgd.py:104-122: x <- x*W_ii; x += x_j * W_ji (receive order)."""
    x = [t.clone() for t in x_self]
    for t in x:
        t.mul_(self_weight)
    for params_j, w_j in neighbours:
        for t, t_j in zip(x, params_j):
            t.add_(t_j.mul(w_j))
    return x


def pushsum_update(x_self, self_weight, neighbours, omega, neighbour_omegas):
    """sp/decentralized/client_pushsum.py:127-156: DSGD step + omega push-sum, z = x * (1/omega)."""
    x = dsgd_update(x_self, self_weight, neighbours)
    omega = omega * self_weight
    for o in neighbour_omegas:
        omega += o
    z = [t.mul(1.0 / omega) for t in x]
    return x, z, omega
