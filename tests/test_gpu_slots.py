"""Staged descriptor tables under several HIP streams (r05's slot protocol, fedagg.hip stage() /
release()): state_dict rounds whose pointer tables exceed the inline-argument size alternate between
two client sets (table copies) and repeat them (reuse hits, no per-call event), issued on two
streams and the default stream in a mixed order -- every result must equal the single-stream result
bit for bit (a copy overwriting a table that a kernel on another stream still reads would show)."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu


def _clients(K, sizes, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return [{f"p{j}": torch.randn(n, generator=g, device="cuda") for j, n in enumerate(sizes)} for _ in range(K)]


def test_staged_tables_across_streams():
    from fedml_amd.ml.aggregator.state_dict_agg import MUL_W, aggregate
    K = 8
    sizes = [1000 + 37 * j for j in range(64)]  # 64 keys: a table well past the 3 KB inline argument
    sets = [_clients(K, sizes, 11), _clients(K, sizes, 12)]
    w = [(i + 1) / sum(range(1, K + 1)) for i in range(K)]
    refs = [aggregate(d, MUL_W, w) for d in sets]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.current_stream()]
    outs = []
    for i in range(60):
        st = streams[(i * 7 // 3) % 3]
        which = (i // 2) % 2 if i < 30 else (i % 5 == 0)
        with torch.cuda.stream(st):
            outs.append((int(which), aggregate(sets[int(which)], MUL_W, w)))
    torch.cuda.synchronize()
    for which, out in outs:
        for key, ref in refs[which].items():
            assert torch.equal(out[key].view(torch.int32), ref.view(torch.int32)), key
