"""Host-side guards (CPU): the pinned-result recycling probe of the ingest path."""
from __future__ import annotations

import torch

from fedml_amd.ml.aggregator import ingest


def test_use_count_probe_holds_on_this_torch():
    assert ingest._USE_COUNT_OK  # torch 2.10: base count 2, +1 per derived view
    b = torch.empty(16)
    assert not ingest._storage_held([b, None])
    v = b.view(4, 4).T
    assert ingest._storage_held([b])
    del v
    assert not ingest._storage_held([b])


def test_use_count_probe_failure_means_always_held(monkeypatch):
    """If the private storage reference count ever stops behaving as probed at import, every pinned
    buffer counts as held: fresh buffers each round, a caller's result is never overwritten."""
    monkeypatch.setattr(ingest, "_USE_COUNT_OK", False)
    assert ingest._storage_held([torch.empty(4)])
    assert not ingest._storage_held([None])
