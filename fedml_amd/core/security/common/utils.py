"""Helpers of the reference's python/fedml/core/security/common/utils.py that the robust
aggregators use (host-side list / key logic only; the per-element work runs in HIP kernels)."""
from __future__ import annotations


def is_weight_param(k):
    """utils.py:16-21: BatchNorm statistics are not weights."""
    return "running_mean" not in k and "running_var" not in k and "num_batches_tracked" not in k


def compute_a_score(local_sample_number):
    """utils.py:230-232 (the reference's placeholder score: the sample count)."""
    return local_sample_number


def trimmed_mean(model_list, trimmed_num):
    """utils.py:213-227: stable sort of the clients by score (sample count), drop `trimmed_num`
    from each end.  Returns the kept (sample_num, grad) tuples, same objects."""
    temp = [(n, grad, compute_a_score(n)) for n, grad in model_list]
    temp.sort(key=lambda t: t[2])
    temp = temp[trimmed_num: len(model_list) - trimmed_num]
    return [(t[0], t[1]) for t in temp]
