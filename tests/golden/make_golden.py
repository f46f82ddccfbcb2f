"""Generate the golden fixtures under tests/golden/ from the REFERENCE implementation.

Runs only in the build container, where the read-only reference is mounted at
/root/reference (it never travels to the GPU box; the fixtures it writes do).
Nothing from the reference is copied: this script imports the reference's own
functions, feeds them seeded synthetic client updates, and stores inputs and
outputs as plain arrays (see golden_io.py for the format).

Loading recipe:
  * ``fedml.ml.aggregator.agg_operator`` is imported behind stub parent packages
    (``import fedml`` itself needs torchvision, which is absent).
  * Methods that live in modules importing wandb / mpi4py / torchvision are
    extracted with ``ast`` (only the named FunctionDef) and executed with a stub
    ``self``.
  * The topology managers need ``nx.to_numpy_matrix`` (removed in networkx 3);
    ``nx.to_numpy_array`` yields the same values once cast to float32.

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import ast
import copy
import functools
import importlib
import json
import logging
import os
import random
import sys
import time
import types
from collections import OrderedDict

sys.dont_write_bytecode = True  # never write __pycache__ into the read-only reference

import networkx as nx
import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from golden_io import dtype_name, save_case, tensor_to_np  # noqa: E402

REF_PY = "/root/reference/python"
REF = REF_PY + "/fedml"


# ----------------------------------------------------------------------------- loading
def _stub_pkg(name: str, path: str) -> None:
    if name in sys.modules:
        return
    m = types.ModuleType(name)
    m.__path__ = [path]
    sys.modules[name] = m


def load_agg_operator():
    for name, sub in [
        ("fedml", ""),
        ("fedml.core", "/core"),
        ("fedml.core.common", "/core/common"),
        ("fedml.ml", "/ml"),
        ("fedml.ml.aggregator", "/ml/aggregator"),
    ]:
        _stub_pkg(name, REF + sub)
    return importlib.import_module("fedml.ml.aggregator.agg_operator")


def load_topology():
    if not hasattr(nx, "to_numpy_matrix"):
        nx.to_numpy_matrix = nx.to_numpy_array
    for name, sub in [
        ("fedml", ""),
        ("fedml.core", "/core"),
        ("fedml.core.distributed", "/core/distributed"),
        ("fedml.core.distributed.topology", "/core/distributed/topology"),
    ]:
        _stub_pkg(name, REF + sub)
    stm = importlib.import_module("fedml.core.distributed.topology.symmetric_topology_manager")
    tu = importlib.import_module("fedml.core.distributed.topology.topo_utils")
    return stm, tu


def extract_method(relpath: str, class_name: str, func_name: str, extra_globals=None):
    """Compile ONLY `class_name.func_name` from a reference file and return it as a function."""
    path = os.path.join(REF, relpath)
    with open(path) as f:
        tree = ast.parse(f.read(), filename=path)
    for node in tree.body:
        if isinstance(node, ast.ClassDef) and node.name == class_name:
            for item in node.body:
                if isinstance(item, ast.FunctionDef) and item.name == func_name:
                    mod = ast.Module(body=[item], type_ignores=[])
                    g = {"copy": copy, "torch": torch, "np": np, "logging": logging, "time": time}
                    if extra_globals:
                        g.update(extra_globals)
                    exec(compile(mod, path, "exec"), g)
                    return g[func_name]
    raise KeyError(f"{relpath}:{class_name}.{func_name}")


class _Off:
    """Stub for FedMLAttacker / FedMLDefender singletons: every feature disabled."""

    @classmethod
    def get_instance(cls):
        return cls()

    def is_model_attack(self):
        return False

    def is_defense_enabled(self):
        return False


# ----------------------------------------------------------------------------- data
def gen_clients(seed, K, layout, kind="normal"):
    """K client state_dicts with the given [(key, shape, dtype)] layout."""
    g = torch.Generator().manual_seed(seed)
    clients = []
    for i in range(K):
        d = OrderedDict()
        for key, shape, dt in layout:
            if dt in (torch.int64, torch.int32):
                d[key] = torch.randint(0, 50, shape, generator=g, dtype=dt)
            else:
                if kind == "normal":
                    v = torch.randn(shape, generator=g, dtype=torch.float64)
                elif kind == "cancel":
                    # near-cancelling values: large common magnitude, alternating sign per client
                    base = torch.randn(shape, generator=g, dtype=torch.float64) * 1e3
                    v = base * (1 if i % 2 == 0 else -1) + torch.randn(shape, generator=g, dtype=torch.float64) * 1e-3
                elif kind == "wide":
                    v = torch.randn(shape, generator=g, dtype=torch.float64) * torch.exp2(
                        torch.randint(-30, 30, shape, generator=g).double())
                else:
                    raise ValueError(kind)
                d[key] = v.to(dt)
        clients.append(d)
    return clients


def gen_counts(seed, K, lo=50, hi=600):
    rng = np.random.RandomState(seed)
    return [int(v) for v in rng.randint(lo, hi + 1, size=K)]


def pack(clients, outputs, meta):
    arrays = {}
    keys = list(clients[0].keys())
    for i, c in enumerate(clients):
        for k in keys:
            arrays[f"x{i}__{k}"] = tensor_to_np(c[k])
    for j, o in enumerate(outputs):
        for k in keys:
            arrays[f"y{j}__{k}"] = tensor_to_np(o[k])
    meta = dict(meta)
    meta.update(
        num_clients=len(clients),
        num_outputs=len(outputs),
        keys=keys,
        in_dtypes=[dtype_name(clients[0][k]) for k in keys],
        out_dtypes=[dtype_name(outputs[0][k]) for k in keys],
        shapes=[list(clients[0][k].shape) for k in keys],
    )
    return meta, arrays


WRITTEN = []


def write(name, clients, outputs, meta, extra=None):
    meta, arrays = pack(clients, outputs, meta)
    meta["name"] = name
    if extra:
        arrays.update(extra)
    path = os.path.join(HERE, name + ".npz")
    save_case(path, meta, arrays)
    WRITTEN.append((name, os.path.getsize(path)))


def dc(x):
    return copy.deepcopy(x)


class Args(types.SimpleNamespace):
    pass


LR_LAYOUT = [("linear.weight", (10, 784), torch.float32), ("linear.bias", (10,), torch.float32)]


# ----------------------------------------------------------------------------- cases
def cases_agg_operator(ao):
    """G1/G2/G3/G5/G9 through FedMLAggOperator.agg (agg_operator.py:9-134)."""
    agg = ao.FedMLAggOperator.agg
    seed = 100
    # G1: fp32 FedAvg, flat parameter vectors
    for K in (1, 2, 3, 7, 32):
        for P in (1, 3, 1000, 4099):
            seed += 1
            clients = gen_clients(seed, K, [("w", (P,), torch.float32)])
            n = gen_counts(seed, K)
            out = agg(Args(federated_optimizer="FedAvg"), list(zip(n, dc(clients))))
            write(f"g1_fedavg_f32_K{K}_P{P}", clients, [out],
                  dict(kind="agg", optimizer="FedAvg", n=n, ref="agg_operator.py:35-44"))
    # G1: FedProx branch (agg_operator.py:45-54), LR layout (config 1 shape)
    clients = gen_clients(7, 2, LR_LAYOUT)
    n = gen_counts(7, 2)
    for opt in ("FedAvg", "FedProx"):
        out = agg(Args(federated_optimizer=opt), list(zip(n, dc(clients))))
        write(f"g1_{opt.lower()}_lr_K2", clients, [out],
              dict(kind="agg", optimizer=opt, n=n, ref="agg_operator.py:35-54"))
    # G1: cancellation-heavy and wide-exponent values
    for kind in ("cancel", "wide"):
        clients = gen_clients(11, 16, [("w", (2053,), torch.float32)], kind=kind)
        n = gen_counts(11, 16)
        out = agg(Args(federated_optimizer="FedAvg"), list(zip(n, dc(clients))))
        write(f"g1_fedavg_f32_{kind}_K16", clients, [out],
              dict(kind="agg", optimizer="FedAvg", n=n, ref="agg_operator.py:35-44"))
    # G2: bf16 FedAvg (per-op bf16 rounding, fp32 weight)
    for K, P in ((7, 4099), (32, 1000), (3, 5)):
        clients = gen_clients(200 + K, K, [("w", (P,), torch.bfloat16), ("b", (17,), torch.bfloat16)])
        n = gen_counts(200 + K, K)
        out = agg(Args(federated_optimizer="FedAvg"), list(zip(n, dc(clients))))
        write(f"g2_fedavg_bf16_K{K}_P{P}", clients, [out],
              dict(kind="agg", optimizer="FedAvg", n=n, ref="agg_operator.py:35-44"))
    # fp16 and fp64 FedAvg (same operator, other storage types)
    for dt, tag in ((torch.float16, "f16"), (torch.float64, "f64")):
        clients = gen_clients(300, 5, [("w", (999,), dt)])
        n = gen_counts(300, 5)
        out = agg(Args(federated_optimizer="FedAvg"), list(zip(n, dc(clients))))
        write(f"g2_fedavg_{tag}_K5", clients, [out],
              dict(kind="agg", optimizer="FedAvg", n=n, ref="agg_operator.py:35-44"))
    # G3: mixed-dtype state_dict (fp32 params + int64 num_batches_tracked-style scalars)
    layout = [
        ("conv1.weight", (8, 3, 3, 3), torch.float32),
        ("bn1.weight", (8,), torch.float32),
        ("bn1.bias", (8,), torch.float32),
        ("bn1.num_batches_tracked", (), torch.int64),
        ("fc.weight", (10, 72), torch.float32),
        ("fc.bias", (10,), torch.float32),
        ("layer.num_batches_tracked", (), torch.int64),
    ]
    for K in (2, 5):
        clients = gen_clients(400 + K, K, layout)
        n = gen_counts(400 + K, K)
        out = agg(Args(federated_optimizer="FedAvg"), list(zip(n, dc(clients))))
        write(f"g3_fedavg_mixed_K{K}", clients, [out],
              dict(kind="agg", optimizer="FedAvg", n=n, ref="agg_operator.py:35-44"))
    # G5: plain sum branches FedAvg_seq / FedDyn (agg_operator.py:55-63, 68-77), incl. int64 sums
    layout = [("w", (1001,), torch.float32), ("steps", (), torch.int64), ("h", (33,), torch.bfloat16)]
    for opt in ("FedAvg_seq", "FedDyn"):
        clients = gen_clients(500, 6, layout)
        n = gen_counts(500, 6)
        out = agg(Args(federated_optimizer=opt), list(zip(n, dc(clients))))
        write(f"g5_{opt.lower()}_sum_K6", clients, [out],
              dict(kind="agg", optimizer=opt, n=n, ref="agg_operator.py:55-77"))
    # G9: edge values -- +-0, subnormals, inf/nan, huge counts
    K = 4
    vals = torch.tensor([0.0, -0.0, 1e-45, -1e-45, 1.17e-38, 3.4e38, -3.4e38, float("inf"),
                         float("-inf"), float("nan"), 1.0, -1.0, 1e-30, 7.0, 0.1, -0.0],
                        dtype=torch.float32)
    clients = []
    for i in range(K):
        g = torch.Generator().manual_seed(900 + i)
        perm = torch.randperm(vals.numel(), generator=g)
        clients.append(OrderedDict(w=vals[perm].clone()))
    for name, n in (("g9_edge_values_K4", [3, 5, 7, 11]),
                    ("g9_edge_bigcounts_K4", [2 ** 24 + 1, 3, 2 ** 30 + 7, 99991])):
        out = agg(Args(federated_optimizer="FedAvg"), list(zip(n, dc(clients))))
        write(name, clients, [out], dict(kind="agg", optimizer="FedAvg", n=n, ref="agg_operator.py:35-44"))
    # G9: inexact n_i/N (N = 3 * 7 * 13), normal data
    clients = gen_clients(950, 3, [("w", (4099,), torch.float32)])
    n = [7, 13, 273 - 20]
    out = agg(Args(federated_optimizer="FedAvg"), list(zip(n, dc(clients))))
    write("g9_inexact_weights_K3", clients, [out], dict(kind="agg", optimizer="FedAvg", n=n,
                                                        ref="agg_operator.py:35-44"))
    # SCAFFOLD / Mime (agg_operator.py:100-133) -- two-dict outputs, with SCAFFOLD's overwrite defect
    K = 4
    lay = [("w", (257,), torch.float32), ("b", (9,), torch.float32)]
    xs = gen_clients(960, K, lay)
    cs = gen_clients(961, K, lay)
    n = gen_counts(960, K)
    out = agg(Args(federated_optimizer="SCAFFOLD", client_num_in_total=10),
              [(n[i], dc(xs[i]), dc(cs[i])) for i in range(K)])
    extra = {}
    for i in range(K):
        for k in ("w", "b"):
            extra[f"c{i}__{k}"] = tensor_to_np(cs[i][k])
    write("g5_scaffold_K4", xs, [out[0], out[1]],
          dict(kind="agg", optimizer="SCAFFOLD", n=n, client_num_in_total=10,
               ref="agg_operator.py:100-118"), extra)
    out = agg(Args(federated_optimizer="Mime", client_num_per_round=K),
              [(n[i], dc(xs[i]), dc(cs[i])) for i in range(K)])
    write("g5_mime_K4", xs, [out[0], out[1]],
          dict(kind="agg", optimizer="Mime", n=n, client_num_per_round=K,
               ref="agg_operator.py:120-133"), extra)


def cases_call_sites():
    """a6 / a7 / a8 / a12: the inline re-implementations of the same loop."""
    sp_aggregate = extract_method("simulation/sp/fedavg/fedavg_api.py", "FedAvgAPI", "_aggregate")
    mpi_agg = extract_method("simulation/mpi/fedavg/FedAVGAggregator.py", "FedAVGAggregator",
                             "_fedavg_aggregation_")
    stub = types.SimpleNamespace()
    # a6: SP FedAvgAPI._aggregate (fedavg_api.py:144-159)
    clients = gen_clients(600, 9, [("w", (3001,), torch.float32), ("b", (10,), torch.float32)])
    n = gen_counts(600, 9)
    out = sp_aggregate(stub, list(zip(n, dc(clients))))
    write("g1_sp_aggregate_K9", clients, [out], dict(kind="sp_aggregate", n=n, ref="fedavg_api.py:144-159"))
    # a7: MPI (x*n)/N (FedAVGAggregator.py:99-116) -- G4, incl. config-1 LR layout, K=2
    for K, lay, tag in ((3, [("w", (4099,), torch.float32)], "K3"),
                        (32, [("w", (1000,), torch.float32)], "K32"),
                        (2, LR_LAYOUT, "lr_K2")):
        clients = gen_clients(610 + K, K, lay)
        n = gen_counts(610 + K, K)
        out = mpi_agg(stub, list(zip(n, dc(clients))))
        write(f"g4_mpi_xn_div_N_{tag}", clients, [out],
              dict(kind="mpi_fedavg", n=n, ref="simulation/mpi/fedavg/FedAVGAggregator.py:99-116"))
    # a7 with bf16 and with counts >= 2^24
    clients = gen_clients(620, 4, [("w", (777,), torch.bfloat16)])
    n = gen_counts(620, 4)
    out = mpi_agg(stub, list(zip(n, dc(clients))))
    write("g4_mpi_xn_div_N_bf16_K4", clients, [out], dict(kind="mpi_fedavg", n=n,
                                                          ref="FedAVGAggregator.py:99-116"))
    clients = gen_clients(621, 3, [("w", (501,), torch.float32)])
    n = [2 ** 24 + 3, 2 ** 25 + 1, 5]
    out = mpi_agg(stub, list(zip(n, dc(clients))))
    write("g4_mpi_xn_div_N_bigcounts_K3", clients, [out], dict(kind="mpi_fedavg", n=n,
                                                               ref="FedAVGAggregator.py:99-116"))
    # a7 with int64 buffers: (x * n) is an int64 op, then true_divide -> float32
    lay = [("w", (301,), torch.float32), ("bn.num_batches_tracked", (), torch.int64),
           ("cnt", (7,), torch.int64)]
    clients = gen_clients(622, 5, lay)
    clients[2]["cnt"][3] = 2 ** 40 + 12345
    n = gen_counts(622, 5)
    out = mpi_agg(stub, list(zip(n, dc(clients))))
    write("g4_mpi_xn_div_N_int64_K5", clients, [out], dict(kind="mpi_fedavg", n=n,
                                                           ref="FedAVGAggregator.py:99-116"))

    # a12: fedavg_seq two-level reduce (FedAvgClientManager.py:67-73 + FedAVGAggregator.py:189-236)
    add_client_model = extract_method("simulation/mpi/fedavg_seq/FedAvgClientManager.py",
                                      "FedAVGClientManager", "add_client_model")
    get_average_weight = extract_method("simulation/mpi/fedavg_seq/FedAVGAggregator.py",
                                        "FedAVGAggregator", "get_average_weight")
    seq_aggregate = extract_method("simulation/mpi/fedavg_seq/FedAVGAggregator.py",
                                   "FedAVGAggregator", "aggregate")
    K = 10
    clients = gen_clients(630, K, [("w", (2049,), torch.float32), ("b", (10,), torch.float32)])
    n = gen_counts(630, K)
    server = types.SimpleNamespace(train_data_local_num_dict={i: n[i] for i in range(K)})
    wdict = get_average_weight(server, list(range(K)))
    schedule = [[0, 1, 2, 3], [4, 5, 6], [7, 8, 9]]
    partials = []
    for wk in schedule:
        acc = {}
        for ci in wk:
            add_client_model(None, acc, dc(clients[ci]), weight=wdict[ci])
        partials.append(acc)
    seq_server = types.SimpleNamespace(
        worker_num=len(schedule), model_dict={i: partials[i] for i in range(len(schedule))},
        set_global_model_params=lambda p: None)
    out = seq_aggregate(seq_server)
    write("g6_fedavg_seq_two_level_K10", clients, [out],
          dict(kind="fedavg_seq", n=n, schedule=schedule,
               ref="fedavg_seq/FedAvgClientManager.py:67-73; fedavg_seq/FedAVGAggregator.py:189-236"))

    # a6 hierarchical SP: group _aggregate then global _aggregate weighted by group sample counts
    K = 12
    groups = [[0, 1, 2, 3, 4], [5, 6], [7, 8, 9, 10, 11]]
    clients = gen_clients(640, K, [("w", (1537,), torch.float32), ("b", (10,), torch.float32)])
    n = gen_counts(640, K)
    w_groups = []
    for grp in groups:
        gw = sp_aggregate(stub, [(n[i], dc(clients[i])) for i in grp])
        w_groups.append((sum(n[i] for i in grp), gw))
    out = sp_aggregate(stub, w_groups)
    write("g7_hier_sp_K12_G3", clients, [out],
          dict(kind="hier_sp", n=n, groups=groups,
               ref="sp/hierarchical_fl/group.py:43-66; trainer.py:100-110; fedavg_api.py:144-159"))

    # a8 MPI cloud aggregate() with its double application (HierFedAvgCloudAggregator.py:67-103)
    cloud_fedavg = extract_method("simulation/mpi/hierarchical_fl/HierFedAvgCloudAggregator.py",
                                  "HierFedAVGCloudAggregator", "_fedavg_aggregation_")
    cloud_aggregate = extract_method("simulation/mpi/hierarchical_fl/HierFedAvgCloudAggregator.py",
                                     "HierFedAVGCloudAggregator", "aggregate",
                                     {"FedMLAttacker": _Off, "FedMLDefender": _Off})
    E, R = 3, 2  # edges (workers) x group_comm_round
    edge_models = gen_clients(650, E * R, [("w", (1025,), torch.float32), ("b", (10,), torch.float32)])
    ne = [gen_counts(650 + e, R) for e in range(E)]
    cloud = types.SimpleNamespace(
        worker_num=E,
        sample_num_dict={e: list(ne[e]) for e in range(E)},
        model_dict={e: [(r, dc(edge_models[e * R + r])) for r in range(R)] for e in range(E)},
    )
    cloud._fedavg_aggregation_ = functools.partial(cloud_fedavg, cloud)
    cloud.set_global_model_params = lambda p: None
    cloud.test_on_cloud_for_all_clients = lambda r: None
    cloud.get_global_model_params = lambda: None
    out = cloud_aggregate(cloud)
    write("g7_hier_cloud_aggregate_E3_R2", edge_models, [out],
          dict(kind="hier_cloud", edges=E, group_comm_round=R, edge_counts=ne,
               note="client index = e*R + r",
               ref="mpi/hierarchical_fl/HierFedAvgCloudAggregator.py:67-103,140-157"))
    return cloud_fedavg


def cases_topology_and_mixing(stm, tu):
    """a9 / a10 / a11: mixing matrices, _pfedavg_mixing_, mix(), DSGD / PushSum gossip steps."""
    # a10: topologies
    extra = {}
    meta_topos = []
    for n in (8, 256):
        m = stm.SymmetricTopologyManager(n, 2)
        m.generate_custom_topology(Args(topo_name="ring"))
        extra[f"W_ring_{n}"] = np.asarray(m.topology, dtype=np.float32)
        meta_topos.append(f"W_ring_{n}")
    for name, fn in (("complete", tu.get_complete_overlay), ("star", tu.get_star_overlay),
                     ("isolated", tu.get_isolated_overlay)):
        for n in (8, 9):
            extra[f"W_{name}_{n}"] = np.asarray(fn(n), dtype=np.float32)
            meta_topos.append(f"W_{name}_{n}")
    for n in (9, 16):
        extra[f"W_2d_torus_{n}"] = np.asarray(tu.get_2d_torus_overlay(n), dtype=np.float32)
        meta_topos.append(f"W_2d_torus_{n}")
    for n in (7, 8):
        extra[f"W_balanced_tree_{n}"] = np.asarray(tu.get_balanced_tree_overlay(n, 2), dtype=np.float32)
        meta_topos.append(f"W_balanced_tree_{n}")
    m = stm.SymmetricTopologyManager(10, 4)
    m.generate_topology()
    extra["W_symmetric_10_4"] = np.asarray(m.topology, dtype=np.float32)
    meta_topos.append("W_symmetric_10_4")
    for n, p, s in ((8, 0.5, 3), (12, 0.3, 4)):
        random.seed(s)
        extra[f"W_random_{n}_seed{s}"] = np.asarray(tu.get_random_overlay(n, p), dtype=np.float32)
        meta_topos.append(f"W_random_{n}_seed{s}")
    blob = np.frombuffer(json.dumps({"name": "topologies", "matrices": meta_topos,
                                     "ref": "symmetric_topology_manager.py:22-78; topo_utils.py:6-94",
                                     "random_seed_note": "python `random.seed(s)` before get_random_overlay"}
                                    ).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "topologies.npz"), meta=blob, **extra)
    WRITTEN.append(("topologies", os.path.getsize(os.path.join(HERE, "topologies.npz"))))

    # a9: _pfedavg_mixing_ rows + mix() (return value incl. edge-0 overwrite) + _pfedavg_aggregation_
    mixing = extract_method("simulation/mpi/hierarchical_fl/HierFedAvgCloudAggregator.py",
                            "HierFedAVGCloudAggregator", "_pfedavg_mixing_")
    pagg = extract_method("simulation/mpi/hierarchical_fl/HierFedAvgCloudAggregator.py",
                          "HierFedAVGCloudAggregator", "_pfedavg_aggregation_")

    def consensus_speed(W, r, args):  # wandb-free stand-in for utils.cal_mixing_consensus_speed
        A = np.array(W) - 1 / np.shape(W)[0]
        return 1 - np.linalg.norm(A, ord=2) ** 2

    mix = extract_method("simulation/mpi/hierarchical_fl/HierFedAvgCloudAggregator.py",
                         "HierFedAVGCloudAggregator", "mix",
                         {"cal_mixing_consensus_speed": consensus_speed})
    for topo in ("ring", "complete"):
        E = 8
        W = extra[f"W_{topo}_{E}"]
        edges = gen_clients(700, E, [("w", (1531,), torch.float32), ("b", (10,), torch.float32)])
        ne = gen_counts(700, E)
        stub = types.SimpleNamespace()
        rows = [mixing(stub, [(ne[j], dc(edges[j])) for j in range(E)], W[i]) for i in range(E)]
        write(f"g8_pfedavg_mixing_{topo}_E{E}", edges, rows,
              dict(kind="mix_rows", n=ne, topology=f"W_{topo}_{E}",
                   ref="HierFedAvgCloudAggregator.py:174-195"), {"W": W})
    # mix() with group_comm_round = 2 (the returned list has edge 0 replaced by the average)
    E, R = 8, 2
    W = extra["W_ring_8"]
    edge_models = gen_clients(710, E * R, [("w", (515,), torch.float32), ("b", (10,), torch.float32)])
    ne = [gen_counts(710 + e, R) for e in range(E)]
    cloud = types.SimpleNamespace(
        worker_num=E, args=Args(enable_wandb=False),
        sample_num_dict={e: list(ne[e]) for e in range(E)},
        model_dict={e: [(r, dc(edge_models[e * R + r])) for r in range(R)] for e in range(E)},
    )
    cloud._pfedavg_mixing_ = functools.partial(mixing, cloud)
    cloud._pfedavg_aggregation_ = functools.partial(pagg, cloud)
    cloud.set_global_model_params = lambda p: None
    cloud.test_on_cloud_for_all_clients = lambda r: None
    topo_mgr = types.SimpleNamespace(topology=W, get_in_neighbor_weights=lambda i: W[i])
    outs = mix(cloud, topo_mgr)
    write("g8_cloud_mix_ring_E8_R2", edge_models, outs,
          dict(kind="hier_mix", edges=E, group_comm_round=R, edge_counts=ne, topology="W_ring_8",
               note="client index = e*R + r",
               ref="HierFedAvgCloudAggregator.py:105-138,159-195"), {"W": W})
    # mixing with Inf / NaN in a zero-weight neighbour (0*inf = nan propagates in the dense loop)
    edges = gen_clients(720, 8, [("w", (64,), torch.float32)])
    edges[4]["w"][3] = float("inf")
    edges[5]["w"][7] = float("nan")
    edges[6]["w"][9] = -0.0
    W = extra["W_ring_8"]
    rows = [mixing(types.SimpleNamespace(), [(1, dc(edges[j])) for j in range(8)], W[i]) for i in range(8)]
    write("g9_mixing_nonfinite_ring_E8", edges, rows,
          dict(kind="mix_rows", n=[1] * 8, topology="W_ring_8", ref="HierFedAvgCloudAggregator.py:174-195"),
          {"W": W})

    # a11: DSGD / PushSum update_local_parameters at the function level (distinct model objects)
    dsgd = extract_method("simulation/sp/decentralized/client_dsgd.py", "ClientDSGD", "update_local_parameters")
    pushsum = extract_method("simulation/sp/decentralized/client_pushsum.py", "ClientPushsum",
                             "update_local_parameters")

    class _M:
        def __init__(self, tensors):
            self.ps = [torch.nn.Parameter(t.clone(), requires_grad=False) for t in tensors]

        def parameters(self):
            return iter(self.ps)

    n_nodes = 8
    W = extra["W_ring_8"]
    lay = [("w", (10, 97), torch.float32), ("b", (10,), torch.float32)]
    xs = gen_clients(730, n_nodes, lay)
    outs, outs_ps = [], []
    omegas = [1.0 + 0.125 * i for i in range(n_nodes)]
    omega_out = []
    for i in range(n_nodes):
        for fn, sink in ((dsgd, outs), (pushsum, outs_ps)):
            me = types.SimpleNamespace(
                id=i, topology=W[i], model_x=_M(list(xs[i].values())), model=_M(list(xs[i].values())),
                neighbors_weight_dict=OrderedDict(), neighbors_topo_weight_dict=OrderedDict(),
                neighbors_omega_dict=OrderedDict(), omega=omegas[i])
            # receive order = ascending sender id (decentralized_fl_api.py:115-120)
            for j in range(n_nodes):
                if W[j][i] != 0 and j != i:
                    me.neighbors_weight_dict[j] = _M(list(xs[j].values()))
                    me.neighbors_topo_weight_dict[j] = W[j][i]
                    me.neighbors_omega_dict[j] = omegas[j] * W[j][i]
            fn(me)
            sink.append(OrderedDict((k, p.data.clone()) for k, p in zip(xs[i].keys(), me.model.ps)))
            if fn is pushsum:
                omega_out.append(float(me.omega))
    write("g8_dsgd_ring_N8", xs, outs,
          dict(kind="dsgd", topology="W_ring_8", ref="sp/decentralized/client_dsgd.py:92-122"), {"W": W})
    write("g8_pushsum_ring_N8", xs, outs_ps,
          dict(kind="pushsum", topology="W_ring_8", omegas_in=omegas, omegas_out=omega_out,
               ref="sp/decentralized/client_pushsum.py:111-156"), {"W": W})


def cases_fedopt():
    """§8(f) next #2: FedOpt server step (simulation/mpi/fedopt/FedOptAggregator.py:48-131): FedAvg,
    pseudo-gradient g = w_global - avg, torch optimizer step on the global parameters; buffers
    take the average (cast into the buffer's dtype by load_state_dict).  Three rounds so the
    momentum buffer's first and later updates are both recorded."""
    for name, sub in [("fedml.simulation", "/simulation"), ("fedml.simulation.mpi", "/simulation/mpi"),
                      ("fedml.simulation.mpi.fedopt", "/simulation/mpi/fedopt")]:
        _stub_pkg(name, REF + sub)
    optrepo = importlib.import_module("fedml.simulation.mpi.fedopt.optrepo")
    g = {"OptRepo": optrepo.OptRepo}
    rel = "simulation/mpi/fedopt/FedOptAggregator.py"
    meth = {m: extract_method(rel, "FedOptAggregator", m, g) for m in
            ("_instantiate_opt", "get_model_params", "get_global_model_params", "set_global_model_params",
             "add_local_trained_result", "check_whether_all_receive", "aggregate", "set_model_global_grads")}

    for opt_name, lr, mom in (("sgd", 0.7, 0.9), ("sgd", 1.0, 0.0), ("rmsprop", 0.01, 0.9), ("rmsprop", 0.05, 0.0)):
        torch.manual_seed(5)
        model = torch.nn.Sequential(torch.nn.Linear(33, 17), torch.nn.BatchNorm1d(17), torch.nn.Linear(17, 5))
        with torch.no_grad():
            model[1].running_mean.normal_()
            model[1].running_var.uniform_(0.5, 2.0)
        init = OrderedDict((k, v.clone()) for k, v in model.state_dict().items())

        class Agg:  # the server_aggregator the FedOpt aggregator wraps (default_aggregator.py:17-23)
            def __init__(self, m):
                self.model = m

            def get_model_params(self):
                return self.model.state_dict()

            def set_model_params(self, p):
                self.model.load_state_dict(p)

        W = 4
        self_ = types.SimpleNamespace(aggregator=Agg(model), worker_num=W, model_dict={}, sample_num_dict={},
                                      flag_client_model_uploaded_dict={i: False for i in range(W)},
                                      args=Args(server_optimizer=opt_name, server_lr=lr, server_momentum=mom))
        for m, f in meth.items():
            setattr(self_, m, functools.partial(f, self_))
        self_.opt = self_._instantiate_opt()
        arrays, rounds = {}, []
        for k, v in init.items():
            arrays[f"init__{k}"] = tensor_to_np(v)
        for r in range(3):
            clients = gen_clients(800 + 10 * r + int(mom * 10), W,
                                  [(k, tuple(v.shape), v.dtype) for k, v in init.items()])
            n = gen_counts(800 + r, W)
            for i in range(W):
                self_.add_local_trained_result(i, dc(clients[i]), n[i])
                for k in init:
                    arrays[f"r{r}_x{i}__{k}"] = tensor_to_np(clients[i][k])
            assert self_.check_whether_all_receive()
            out = self_.aggregate()
            for k, v in out.items():
                arrays[f"r{r}_y__{k}"] = tensor_to_np(v)
            rounds.append({"n": n})
        meta = {"name": f"g10_fedopt_{opt_name}_lr{lr}_m{mom}", "kind": "fedopt", "server_optimizer": opt_name,
                "server_lr": lr, "server_momentum": mom, "rounds": rounds, "keys": list(init.keys()),
                "dtypes": [dtype_name(v) for v in init.values()],
                "params": [k for k, _ in model.named_parameters()],
                "ref": "simulation/mpi/fedopt/FedOptAggregator.py:48-131"}
        path = os.path.join(HERE, meta["name"] + ".npz")
        save_case(path, meta, arrays)
        WRITTEN.append((meta["name"], os.path.getsize(path)))


def load_mpc():
    for name, sub in [("fedml", ""), ("fedml.core", "/core"), ("fedml.core.mpc", "/core/mpc")]:
        _stub_pkg(name, REF + sub)
    return (importlib.import_module("fedml.core.mpc.lightsecagg"),
            importlib.import_module("fedml.core.mpc.secagg"))


def _np_dict_to_torch(d):
    return OrderedDict((k, torch.from_numpy(np.array(v, dtype=np.int64, copy=True))) for k, v in d.items())


def _adversarial_i64(rng, shape, p):
    """int64 values in and far outside [0, p): negatives, multiples of p, near the int64 ends."""
    n = int(np.prod(shape))
    v = rng.randint(0, p, size=n).astype(np.int64)
    sel = rng.randint(0, 6, size=n)
    big = rng.randint(-2 ** 62, 2 ** 62, size=n, dtype=np.int64) * 2 + rng.randint(0, 2, size=n)
    v = np.where(sel == 1, -v, v)
    v = np.where(sel == 2, v + p * rng.randint(1, 9, size=n), v)
    v = np.where(sel == 3, big, v)
    v = np.where(sel == 4, np.int64(2 ** 63 - 1) - rng.randint(0, 3, size=n), v)
    return v.reshape(shape)


def _real_values(rng, shape, q):
    """float64 values that stress my_q: ties at the 2^-q grid, both signs, large and tiny."""
    n = int(np.prod(shape))
    sel = rng.randint(0, 6, size=n)
    v = rng.standard_normal(n)
    v = np.where(sel == 1, (rng.randint(-2000, 2000, size=n) + 0.5) / 2.0 ** q, v)  # exact ties
    v = np.where(sel == 2, rng.standard_normal(n) * 2.0 ** rng.randint(0, 40, size=n), v)  # large
    v = np.where(sel == 3, rng.standard_normal(n) * 2.0 ** -rng.randint(q, q + 30, size=n), v)  # tiny
    return v.reshape(shape)


def cases_secagg():
    """§8(f) next #4: finite-field secure aggregation (core/mpc/lightsecagg.py, core/mpc/secagg.py,
    cross_silo/lightsecagg/lsa_fedml_aggregator.py:101-175, cross_silo/secagg/sa_fedml_aggregator.py:
    138-184), generated by running the reference's functions on seeded inputs."""
    import warnings
    lsa, sa = load_mpc()
    np.random.seed(1234)  # mask_encoding draws its noise from the global numpy RNG
    rng = np.random.RandomState(77)
    layout = [("fc.weight", (5, 7)), ("fc.bias", (5,)), ("bn.num_batches_tracked", ()), ("v", (13,))]

    # S1: aggregate_models_in_finite (lightsecagg.py:134-145 == secagg.py:148-159)
    for p, K in ((2 ** 15 - 19, 5), (2 ** 61 - 1, 4), (2 ** 15 - 19, 1)):
        clients = [OrderedDict((k, _adversarial_i64(rng, s, p)) for k, s in layout) for _ in range(K)]
        out = lsa.aggregate_models_in_finite(dc(clients), p)
        assert out2_equal(out, sa.aggregate_models_in_finite(dc(clients), p))
        write(f"g11_finite_sum_p{p}_K{K}", [_np_dict_to_torch(c) for c in clients], [_np_dict_to_torch(out)],
              dict(kind="finite_sum", p=p, ref="core/mpc/lightsecagg.py:134-145"))

    # S2: my_q / transform_tensor_to_finite (+ model_masking) on float32 / float64 / int64 tensors
    for p, q in ((2 ** 15 - 19, 8), (2 ** 31 - 1, 16), (2 ** 61 - 1, 20)):
        d = OrderedDict()
        d["w32"] = torch.from_numpy(_real_values(rng, (67,), q).astype(np.float32))
        sp = torch.tensor([0.0, -0.0, float("nan"), float("inf"), -float("inf"), 3e38, -3e38, 2.0 ** 62,
                           -2.0 ** 63, 2.0 ** 63, 0.5 / 2 ** q, -0.5 / 2 ** q, 1.5 / 2 ** q, -2.5 / 2 ** q],
                          dtype=torch.float32)
        d["special32"] = sp
        d["w64"] = torch.from_numpy(_real_values(rng, (3, 11), q))
        d["special64"] = sp.double()
        d["n64"] = torch.from_numpy(rng.randint(-10 ** 6, 10 ** 6, size=(9,)).astype(np.int64))
        d["n64_big"] = torch.tensor([2 ** 62, -2 ** 62, 2 ** 63 - 1, -2 ** 63, 7, -7, 0], dtype=torch.int64)
        d["scalar"] = torch.tensor(5, dtype=torch.int64)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            fin = lsa.transform_tensor_to_finite(OrderedDict((k, v.clone()) for k, v in d.items()), p, q)
            fin_copy = {k: np.array(v, copy=True) for k, v in fin.items()}
            dims = [int(np.prod(v.shape)) for v in d.values()]
            mask = rng.randint(p, size=(sum(dims), 1))
            masked = lsa.model_masking(fin, dims, mask, p)
        outs = [_np_dict_to_torch(fin_copy), _np_dict_to_torch(masked)]
        meta, arrays = pack([d], outs, dict(kind="finite_quantize", p=p, q_bits=q,
                                            ref="core/mpc/lightsecagg.py:83-95,150-154,187-192"))
        arrays["mask"] = mask.astype(np.int64)
        name = f"g12_my_q_p{p}_q{q}"
        meta["name"] = name
        save_case(os.path.join(HERE, name + ".npz"), meta, arrays)
        WRITTEN.append((name, os.path.getsize(os.path.join(HERE, name + ".npz"))))

    # S3: my_q_inv / transform_finite_to_tensor (lightsecagg.py:157-185), incl. 0-d -> shape [1]
    for p, q in ((2 ** 15 - 19, 8), (2 ** 61 - 1, 20), (2 ** 15 - 18, 4)):
        fin = OrderedDict((k, _adversarial_i64(rng, s, p)) for k, s in layout)
        fin["in_range"] = rng.randint(0, p, size=(41,)).astype(np.int64)
        fin["edge"] = np.array([0, 1, (p - 1) // 2, (p - 1) // 2 + 1, p // 2, p - 1, p, -1], dtype=np.int64)
        src = _np_dict_to_torch(fin)
        out = lsa.transform_finite_to_tensor(OrderedDict((k, np.array(v, copy=True)) for k, v in fin.items()), p, q)
        write(f"g13_my_q_inv_p{p}_q{q}", [src], [OrderedDict((k, v.clone()) for k, v in out.items())],
              dict(kind="finite_dequantize", p=p, q_bits=q, ref="core/mpc/lightsecagg.py:157-185"))

    # S4: LightSecAgg end to end (client masking + encoded-mask exchange, server LCC decoding and
    # reconstruction), lsa_fedml_aggregator.py:101-175
    g = {"LCC_decoding_with_points": lsa.LCC_decoding_with_points,
         "transform_finite_to_tensor": lsa.transform_finite_to_tensor}
    rel = "cross_silo/lightsecagg/lsa_fedml_aggregator.py"
    mrec = extract_method(rel, "LightSecAggAggregator", "aggregate_mask_reconstruction", g)
    arec = extract_method(rel, "LightSecAggAggregator", "aggregate_model_reconstruction", g)
    for N, p, q in ((5, 2 ** 15 - 19, 8), (8, 2 ** 31 - 1, 16), (3, 2 ** 15 - 19, 10)):
        U, T = N, N // 2
        model = [("fc.weight", (6, 11)), ("fc.bias", (6,)), ("bn.running_mean", (6,)),
                 ("bn.num_batches_tracked", ()), ("head", (37,))]
        weights = []
        for i in range(N):
            w = OrderedDict()
            for k, s in model:
                if k.endswith("num_batches_tracked"):
                    w[k] = torch.tensor(3 + i, dtype=torch.int64)
                else:
                    w[k] = torch.from_numpy((rng.standard_normal(s) * 0.5).astype(np.float32))
            weights.append(w)
        dims = [int(np.prod(s)) for _, s in model]
        total = sum(dims)
        d = int(np.ceil(float(total) / (U - T))) * (U - T)
        local_masks = [np.random.randint(p, size=(d, 1)) for _ in range(N)]
        enc = [lsa.mask_encoding(d, N, U, T, p, local_masks[j]) for j in range(N)]
        masked = []
        for i in range(N):
            fin = lsa.transform_tensor_to_finite(OrderedDict((k, v.clone()) for k, v in weights[i].items()), p, q)
            masked.append(lsa.model_masking(fin, dims, local_masks[i], p))
        active = list(range(N))
        agg_enc = {i: lsa.compute_aggregate_encoded_mask({j: enc[j][i] for j in range(N)}, p, active)
                   for i in range(N)}
        self_ = types.SimpleNamespace(
            total_dimension=total, client_num=N, targeted_number_active_clients=U, privacy_guarantee=T,
            prime_number=p, precision_parameter=q, dimensions=dims,
            aggregate_encoded_mask_dict={i: np.array(v) for i, v in agg_enc.items()},
            model_dict={i: {k: np.array(v, copy=True) for k, v in masked[i].items()} for i in range(N)},
            set_global_model_params=lambda params: None)
        self_.aggregate_mask_reconstruction = functools.partial(mrec, self_)
        inputs = [_np_dict_to_torch(m) for m in masked]
        amask = self_.aggregate_mask_reconstruction(active)
        out = arec(self_, active, active)
        F = np.zeros((U, d // (U - T)), dtype=np.int64)
        for i in active:
            F[i, :] = agg_enc[i]
        meta, arrays = pack(inputs, [OrderedDict((k, v.clone()) for k, v in out.items())],
                            dict(kind="lsa_reconstruct", p=p, q_bits=q, N=N, U=U, T=T, dims=dims, d=d,
                                 ref="cross_silo/lightsecagg/lsa_fedml_aggregator.py:101-175"))
        arrays["F"] = F
        arrays["aggregate_mask"] = np.asarray(amask, dtype=np.int64).reshape(-1)
        name = f"g14_lsa_reconstruct_N{N}_p{p}"
        meta["name"] = name
        save_case(os.path.join(HERE, name + ".npz"), meta, arrays)
        WRITTEN.append((name, os.path.getsize(os.path.join(HERE, name + ".npz"))))
        # the true aggregate is recovered: sum of the local masks == the decoded mask (mod p)
        ok = np.array_equal(np.mod(sum(m[:total, 0] for m in local_masks), p), arrays["aggregate_mask"][:total])
        print(f"lsa N={N} p={p}: decoded mask == sum of local masks: {ok}")

    # S5: SecAgg model reconstruction (sa_fedml_aggregator.py:138-184) with a given aggregate mask:
    # flags all set (every client summed, mod after each add) and the real server flow, where
    # check_whether_all_receive (:84-90) has already cleared every flag (only client 0's model is kept)
    arec_sa = extract_method("cross_silo/secagg/sa_fedml_aggregator.py", "SecAggAggregator",
                             "aggregate_model_reconstruction",
                             {"transform_finite_to_tensor": sa.transform_finite_to_tensor})
    for N, p, q, flags in ((4, 2 ** 15 - 19, 8, "all"), (4, 2 ** 15 - 19, 8, "none"),
                           (5, 2 ** 61 - 1, 12, "some")):
        model = [("w", (9, 4)), ("b", (9,)), ("nbt", ())]
        dims = [int(np.prod(s)) for _, s in model]
        total = sum(dims)
        clients = [OrderedDict((k, _adversarial_i64(rng, s, p)) for k, s in model) for _ in range(N)]
        amask = rng.randint(0, p, size=total).astype(np.int64)
        fl = {i: {"all": True, "none": False, "some": i % 2 == 1}[flags] for i in range(N)}
        self_ = types.SimpleNamespace(
            prime_number=p, precision_parameter=q, dimensions=dims,
            model_dict={i: {k: np.array(v, copy=True) for k, v in clients[i].items()} for i in range(N)},
            flag_client_model_uploaded_dict=dict(fl),
            aggregate_mask_reconstruction=lambda *a: amask)
        active = list(range(N))
        out = arec_sa(self_, active, active, None, None)
        meta, arrays = pack([_np_dict_to_torch(c) for c in clients], [OrderedDict((k, v.clone()) for k, v in out.items())],
                            dict(kind="sa_reconstruct", p=p, q_bits=q, flags=[fl[i] for i in range(N)], dims=dims,
                                 ref="cross_silo/secagg/sa_fedml_aggregator.py:138-184"))
        arrays["aggregate_mask"] = amask
        name = f"g15_sa_reconstruct_{flags}_p{p}"
        meta["name"] = name
        save_case(os.path.join(HERE, name + ".npz"), meta, arrays)
        WRITTEN.append((name, os.path.getsize(os.path.join(HERE, name + ".npz"))))


def cases_sa_mask():
    """SecAgg's mask re-expansion (cross_silo/secagg/sa_fedml_aggregator.py:92-136), run from the
    reference itself: BGW decoding of the shares, then numpy's legacy MT19937 streams
    (np.random.seed + randint) per surviving client (flag set) or per pair of a dropped client --
    all / none / some flagged, a rejection-heavy prime (40961: 37.5% of draws rejected), d > 624."""
    _, sa = load_mpc()
    amr = extract_method("cross_silo/secagg/sa_fedml_aggregator.py", "SecAggAggregator",
                         "aggregate_mask_reconstruction", {"BGW_decoding": sa.BGW_decoding})
    rng = np.random.RandomState(4242)
    for N, p, d, flags in ((4, 2 ** 15 - 19, 3001, "all"), (5, 40961, 2500, "none"), (6, 2 ** 31 - 1, 1500, "some"),
                           (3, 40961, 700, "some")):
        T = int(np.floor(N / 2))
        SS_rx = rng.randint(0, p, size=(N, N)).astype(np.int64)
        public_key_list = rng.randint(0, p, size=(2, N)).astype(np.int64)
        active = [int(v) for v in rng.permutation(N)]
        fl = {i: {"all": True, "none": False, "some": i % 2 == 0}[flags] for i in range(N)}
        self_ = types.SimpleNamespace(total_dimension=d, privacy_guarantee=T, prime_number=p,
                                      targeted_number_active_clients=N, flag_client_model_uploaded_dict=dict(fl))
        mask = amr(self_, active, SS_rx, public_key_list)
        name = f"g21_sa_mask_{flags}_N{N}_p{p}"
        np.savez(os.path.join(HERE, name + ".npz"), SS_rx=SS_rx, public_key_list=public_key_list,
                 active=np.array(active, dtype=np.int64), flags=np.array([fl[i] for i in range(N)]),
                 mask=np.asarray(mask, dtype=np.int64), meta=np.array(json.dumps(dict(
                     kind="sa_mask", N=N, T=T, p=p, d=d, ref="cross_silo/secagg/sa_fedml_aggregator.py:92-136"))))
        WRITTEN.append((name, os.path.getsize(os.path.join(HERE, name + ".npz"))))


def load_defenses():
    for name, sub in [("fedml", ""), ("fedml.core", "/core"), ("fedml.core.security", "/core/security"),
                      ("fedml.core.security.common", "/core/security/common"),
                      ("fedml.core.security.defense", "/core/security/defense")]:
        _stub_pkg(name, REF + sub)
    med = importlib.import_module("fedml.core.security.defense.coordinate_wise_median_defense")
    tm = importlib.import_module("fedml.core.security.defense.coordinate_wise_trimmed_mean_defense")
    kr = importlib.import_module("fedml.core.security.defense.krum_defense")
    return med.CoordinateWiseMedianDefense, tm.CoordinateWiseTrimmedMeanDefense, kr.KrumDefense


def _robust_clients(seed, K, layout, special=True, levels=None):
    g = torch.Generator().manual_seed(seed)
    clients = []
    for i in range(K):
        d = OrderedDict()
        for key, shape, dt in layout:
            if dt in (torch.int64,):
                d[key] = torch.randint(0, 9, shape, generator=g, dtype=dt)
                continue
            v = torch.randn(shape, generator=g, dtype=torch.float64)
            if levels:  # few distinct values -> many ties
                v = torch.round(v * levels) / levels
            if special:
                u = torch.rand(shape, generator=g)
                v = torch.where(u < 0.03, torch.zeros_like(v), v)
                v = torch.where((u >= 0.03) & (u < 0.06), -torch.zeros_like(v), v)
                v = torch.where((u >= 0.06) & (u < 0.07), torch.full_like(v, float("inf")), v)
                v = torch.where((u >= 0.07) & (u < 0.08), torch.full_like(v, -float("inf")), v)
                v = torch.where((u >= 0.08) & (u < 0.085), torch.full_like(v, float("nan")), v)
            d[key] = v.to(dt)
        clients.append(d)
    return clients


def cases_robust():
    """§8(f) next #3: robust aggregation (core/security/defense/coordinate_wise_median_defense.py,
    coordinate_wise_trimmed_mean_defense.py + common/utils.py:213-232, krum_defense.py)."""
    Median, Trimmed, Krum = load_defenses()
    flat = [("fc.weight", (10, 50), torch.float32), ("fc.bias", (10,), torch.float32)]
    bn = [("conv.weight", (4, 3, 3, 3), torch.float32), ("bn.weight", (4,), torch.float32),
          ("bn.bias", (4,), torch.float32), ("bn.running_mean", (4,), torch.float32),
          ("bn.running_var", (4,), torch.float32), ("bn.num_batches_tracked", (), torch.int64),
          ("fc.weight", (3, 4), torch.float32), ("fc.bias", (3,), torch.float32)]
    # R1: coordinate-wise median (torch.median over the client axis = lower median, NaN first)
    seed = 900
    for K in (1, 2, 3, 4, 5, 8, 13, 32, 64, 100):
        for levels in (None, 4):
            seed += 1
            clients = _robust_clients(seed, K, flat, levels=levels)
            n = gen_counts(seed, K)
            out = Median(Args()).defend_on_aggregation(list(zip(n, dc(clients))))
            write(f"g16_median_f32_K{K}" + ("_ties" if levels else ""), clients, [out],
                  dict(kind="median", n=n, ref="core/security/defense/coordinate_wise_median_defense.py:18-44"))
    for dt, tag, K in ((torch.bfloat16, "bf16", 7), (torch.float16, "f16", 6), (torch.float64, "f64", 9)):
        lay = [(k, s, dt) for k, s, _ in flat]
        clients = _robust_clients(950 + K, K, lay, levels=8)
        n = gen_counts(950 + K, K)
        out = Median(Args()).defend_on_aggregation(list(zip(n, dc(clients))))
        write(f"g16_median_{tag}_K{K}", clients, [out], dict(kind="median", n=n,
              ref="core/security/defense/coordinate_wise_median_defense.py:18-44"))
    # a non-BN int64 key: torch.cat promotes to float32, the key comes back float32
    lay = flat + [("step", (3,), torch.int64)]
    clients = _robust_clients(960, 5, lay)
    n = gen_counts(960, 5)
    out = Median(Args()).defend_on_aggregation(list(zip(n, dc(clients))))
    write("g16_median_mixed_int_K5", clients, [out], dict(kind="median", n=n,
          ref="core/security/defense/coordinate_wise_median_defense.py:18-44"))
    # BatchNorm statistics: vectorize_weight skips them but the write-back walk does not -> error
    clients = _robust_clients(961, 5, bn, special=False)
    n = gen_counts(961, 5)
    try:
        Median(Args()).defend_on_aggregation(list(zip(n, dc(clients))))
        err = None
    except Exception as e:  # noqa: BLE001
        err = [type(e).__name__, str(e)]
    assert err is not None
    write("g16_median_bn_error_K5", clients, [clients[0]], dict(kind="median", n=n, error=err,
          ref="core/security/defense/coordinate_wise_median_defense.py:35-43"))

    # R2: "trimmed mean": sorts clients by sample count (compute_a_score) and drops beta*K per end
    for K, beta, counts in ((10, 0.1, None), (10, 0.25, None), (7, 0.49, None), (6, 0.0, None),
                            (9, 0.2, [5, 3, 5, 1, 3, 5, 2, 2, 9])):
        n = counts or gen_counts(970 + K, K)
        clients = _robust_clients(970 + K, K, flat, special=False)
        raw = list(zip(n, clients))
        sel = Trimmed(Args(beta=beta)).defend_before_aggregation(raw)
        idx = [next(i for i, (_, c) in enumerate(raw) if c is sc) for _, sc in sel]
        write(f"g17_trimmed_K{K}_b{beta}", clients, [clients[0]],
              dict(kind="trimmed", n=n, beta=beta, selected=idx,
                   ref="core/security/defense/coordinate_wise_trimmed_mean_defense.py:20-28, common/utils.py:213-232"))

    # R3: Krum / multi-Krum selection and scores
    for K, f, m, lay in ((10, 2, 1, flat), (16, 3, 4, flat), (12, 2, 3, bn), (8, 1, 1, flat)):
        clients = _robust_clients(980 + K, K, lay, special=False)
        g = torch.Generator().manual_seed(K)
        for b in range(f):  # byzantine clients: scaled noise
            for k2, v in clients[b * 3 % K].items():
                if v.is_floating_point():
                    clients[b * 3 % K][k2] = v + 5.0 * torch.randn(v.shape, generator=g).to(v.dtype)
        n = gen_counts(980 + K, K)
        raw = list(zip(n, clients))
        d = Krum(Args(byzantine_client_num=f, krum_param_m=m))
        sel = d.defend_before_aggregation(raw)
        idx = [next(i for i, (_, c) in enumerate(raw) if c is sc) for _, sc in sel]
        import fedml.core.security.common.utils as su
        scores = d._compute_krum_score([su.vectorize_weight(c) for c in clients])
        write(f"g18_krum_K{K}_f{f}_m{m}", clients, [clients[0]],
              dict(kind="krum", n=n, byzantine_client_num=f, krum_param_m=m, selected=idx, scores=scores,
                   ref="core/security/defense/krum_defense.py:27-66"))
    try:
        Krum(Args(byzantine_client_num=4, krum_param_m=1)).defend_before_aggregation(
            list(zip([1] * 9, _robust_clients(1, 9, flat, special=False))))
        err = None
    except ValueError as e:
        err = ["ValueError", str(e)]
    assert err is not None
    with open(os.path.join(HERE, "g18_krum_errors.json"), "w") as fh:
        json.dump({"K9_f4_m1": err}, fh)


def cases_krum_half():
    """Krum over bfloat16 / float16 models (krum_defense.py:27-66): vectorize_weight keeps the model
    dtype, so `(v_i - v_j)` and `.norm()` run in it.  Records the reference's selection, scores and
    every pair's `compute_euclidean_distance(v_i, v_j).item() ** 2` (utils.py:24-27); the f16
    overflow case has a client far enough out that its distances' float16 norm overflows to inf."""
    _, _, Krum = load_defenses()
    import fedml.core.security.common.utils as su
    flat = [("fc.weight", (10, 50), None), ("fc.bias", (10,), None)]
    for dt, tag, K, f, m, scale in ((torch.bfloat16, "bf16", 10, 2, 1, 5.0), (torch.bfloat16, "bf16", 12, 2, 3, 5.0),
                                    (torch.float16, "f16", 10, 2, 2, 5.0), (torch.float16, "f16ovf", 8, 1, 1, 6000.0)):
        lay = [(k, sh, dt) for k, sh, _ in flat]
        clients = _robust_clients(1990 + K + len(tag), K, lay, special=False)
        g = torch.Generator().manual_seed(K + 7)
        for b in range(f):  # byzantine clients: scaled noise, in the model dtype
            for k2, v in clients[b * 3 % K].items():
                clients[b * 3 % K][k2] = v + (scale * torch.randn(v.shape, generator=g)).to(v.dtype)
        n = gen_counts(1990 + K, K)
        raw = list(zip(n, clients))
        d = Krum(Args(byzantine_client_num=f, krum_param_m=m))
        sel = d.defend_before_aggregation(raw)
        idx = [next(i for i, (_, c) in enumerate(raw) if c is sc) for _, sc in sel]
        vec = [su.vectorize_weight(c) for c in clients]
        assert vec[0].dtype == dt
        scores = d._compute_krum_score(vec)
        dists = [[su.compute_euclidean_distance(vec[i], vec[j]).item() ** 2 if i != j else 0.0 for j in range(K)]
                 for i in range(K)]
        write(f"g18_krum_{tag}_K{K}_f{f}_m{m}", clients, [clients[0]],
              dict(kind="krum", n=n, byzantine_client_num=f, krum_param_m=m, selected=idx, scores=scores,
                   dists=dists, vector_dtype=str(dt).replace("torch.", ""),
                   ref="core/security/defense/krum_defense.py:27-66, common/utils.py:8-27"))


def cases_sp_sampling():
    """The SP round driver's client sampling (simulation/sp/fedavg/fedavg_api.py:127-135), run from the
    reference itself: the client indexes per round for several (in_total, per_round) settings."""
    fn = extract_method("simulation/sp/fedavg/fedavg_api.py", "FedAvgAPI", "_client_sampling")
    cases = {}
    for total, per in ((10, 10), (10, 4), (7, 3), (100, 10), (1000, 64), (5, 9)):
        cases[f"{total}_{per}"] = [[int(v) for v in fn(None, r, total, per)] for r in range(6)]
    with open(os.path.join(HERE, "g20_sp_sampling.json"), "w") as fh:
        json.dump({"ref": "simulation/sp/fedavg/fedavg_api.py:127-135", "rounds": 6, "cases": cases}, fh)


def cases_krum_f64():
    """Krum over float64 models (krum_defense.py:27-66): vectorize_weight keeps float64, so every
    `(v_i - v_j).norm()` runs in float64.  `near_tie`: the honest clients are one base vector plus
    offsets of ~1e-10, below float32's resolution of the values -- in float32 every honest distance
    would round to 0 and the selection would fall to the lowest index, while the reference's float64
    distances (and its float32 scores, which still resolve ~1e-20) pick another client."""
    _, _, Krum = load_defenses()
    import fedml.core.security.common.utils as su
    lay = [("fc.weight", (10, 50), torch.float64), ("fc.bias", (10,), torch.float64),
           ("bn.running_mean", (10,), torch.float64)]
    for tag, K, f, m in (("spread", 10, 2, 1), ("spread", 12, 2, 3), ("near_tie", 10, 2, 1), ("near_tie", 11, 2, 2)):
        g = torch.Generator().manual_seed(2024 + K + len(tag))
        if tag == "spread":
            clients = _robust_clients(3030 + K, K, lay, special=False)
            for b in range(f):
                for k2, v in clients[b * 3 % K].items():
                    clients[b * 3 % K][k2] = v + 5.0 * torch.randn(v.shape, generator=g, dtype=torch.float64)
        else:
            base = _robust_clients(3030 + K, 1, lay, special=False)[0]
            clients = []
            for i in range(K):
                scale = 1e-10 * (1.0 + 0.37 * ((i + 5) % K))  # the tightest client is not client 0
                clients.append(OrderedDict((k2, v + scale * torch.randn(v.shape, generator=g, dtype=torch.float64))
                                           for k2, v in base.items()))
            for b in range(f):
                for k2, v in clients[(b * 3 + 1) % K].items():
                    clients[(b * 3 + 1) % K][k2] = v + 5.0 * torch.randn(v.shape, generator=g, dtype=torch.float64)
        n = gen_counts(3030 + K, K)
        raw = list(zip(n, clients))
        d = Krum(Args(byzantine_client_num=f, krum_param_m=m))
        sel = d.defend_before_aggregation(raw)
        idx = [next(i for i, (_, c) in enumerate(raw) if c is sc) for _, sc in sel]
        vec = [su.vectorize_weight(c) for c in clients]
        assert vec[0].dtype == torch.float64
        scores = d._compute_krum_score(vec)
        dists = [[su.compute_euclidean_distance(vec[i], vec[j]).item() ** 2 if i != j else 0.0 for j in range(K)]
                 for i in range(K)]
        if tag == "near_tie":  # the float32 measurement would not reproduce this selection
            v32 = [v.float() for v in vec]
            s32 = d._compute_krum_score(v32)
            idx32 = torch.argsort(torch.Tensor(s32)).tolist()[:m]
            assert idx32 != idx, (idx32, idx)
        write(f"g18_krum_f64_{tag}_K{K}_f{f}_m{m}", clients, [clients[0]],
              dict(kind="krum", n=n, byzantine_client_num=f, krum_param_m=m, selected=idx, scores=scores,
                   dists=dists, vector_dtype="float64",
                   ref="core/security/defense/krum_defense.py:27-66, common/utils.py:8-27"))


def _band_kappa_max(vec):
    """max over pairs of kappa_ij = (A_i + A_j) / D_ij, A_i = |x_i - c|^2 with c the per-coordinate
    median of clients 0..4 (the Gram form's centre, fedml_amd/csrc/robust.hip), exact in float64."""
    X = torch.stack([v.double() for v in vec])
    K = X.shape[0]
    c = torch.stack(vec[:5]).median(0).values.double() if K >= 5 else X[0]
    A = ((X - c) ** 2).sum(1)
    best = 0.0
    for i in range(K):
        for j in range(i + 1, K):
            D = float(((X[i] - X[j]) ** 2).sum())
            best = max(best, float(A[i] + A[j]) / D)
    return best


def cases_krum_band():
    """r06: Krum over float32 models whose pairs sit in the Gram form's cancellation band (kappa_max
    2..16), so that the selection there is pinned by the REFERENCE: `offset` --
    clients 0..2 (three of the five that define the Gram form's centre) shifted by delta, every honest
    pair at kappa ~ (delta^2 + s^2) / s^2; `pair` -- the last client a near copy of the one before it.
    Records the reference's selection, scores and every `compute_euclidean_distance(v_i, v_j).item()
    ** 2` (krum_defense.py:27-66, common/utils.py:8-27) and the realised kappa_max."""
    _, _, Krum = load_defenses()
    import fedml.core.security.common.utils as su
    lr = [("linear.weight", (10, 784), torch.float32), ("linear.bias", (10,), torch.float32)]
    sm = [("fc.weight", (10, 196), torch.float32), ("fc.bias", (10,), torch.float32)]  # P = 1,970
    for tag, lay, K, f, m, kind, kappa in (("lr_offset16", lr, 6, 1, 1, "offset", 15.9),
                                           ("p1970_offset8", sm, 12, 2, 1, "offset", 8.0),
                                           ("p1970_offset16m3", sm, 12, 2, 3, "offset", 15.9),
                                           ("p1970_pair12", sm, 10, 2, 2, "pair", 12.0)):
        g = torch.Generator().manual_seed(4040 + K + int(kappa * 10) + len(tag))
        sgm = 1e-2
        base = OrderedDict((k, 0.05 * torch.randn(sh, generator=g)) for k, sh, _ in lay)
        clients = [OrderedDict((k, (v + sgm * torch.randn(v.shape, generator=g)).float()) for k, v in base.items())
                   for _ in range(K)]
        if kind == "offset":  # delta by bisection until the realised kappa_max is within 2 % of the target
            honest = clients[:3]
            lo, hi = 0.0, 20 * sgm
            for _ in range(40):
                delta = 0.5 * (lo + hi)
                clients[:3] = [OrderedDict((k, (v + delta).float()) for k, v in c.items()) for c in honest]
                km = _band_kappa_max([su.vectorize_weight(c) for c in clients])
                if abs(km - kappa) <= 0.02 * kappa:
                    break
                lo, hi = (delta, hi) if km < kappa else (lo, delta)
        else:
            eps = sgm * (2 * 1.29 / kappa) ** 0.5
            clients[K - 1] = OrderedDict((k, (v + eps * torch.randn(v.shape, generator=g)).float())
                                         for k, v in clients[K - 2].items())
        n = gen_counts(4040 + K, K)
        raw = list(zip(n, clients))
        d = Krum(Args(byzantine_client_num=f, krum_param_m=m))
        sel = d.defend_before_aggregation(raw)
        idx = [next(i for i, (_, c) in enumerate(raw) if c is sc) for _, sc in sel]
        vec = [su.vectorize_weight(c) for c in clients]
        assert vec[0].dtype == torch.float32
        scores = d._compute_krum_score(vec)
        dists = [[su.compute_euclidean_distance(vec[i], vec[j]).item() ** 2 if i != j else 0.0 for j in range(K)]
                 for i in range(K)]
        km = _band_kappa_max(vec)
        assert abs(km - kappa) <= 0.02 * kappa or kind == "pair", (tag, km)
        write(f"g18_krum_band_{tag}_K{K}_f{f}_m{m}", clients, [clients[0]],
              dict(kind="krum", n=n, byzantine_client_num=f, krum_param_m=m, selected=idx, scores=scores,
                   dists=dists, vector_dtype="float32", kappa_max=km, construction=kind,
                   ref="core/security/defense/krum_defense.py:27-66, common/utils.py:8-27"))


def out2_equal(a, b):
    return all(np.array_equal(np.asarray(a[k]), np.asarray(b[k])) for k in a)


def layouts(ao):
    """Model layouts used by the configs: names/shapes/dtypes only (no weights)."""
    for name, sub in [("fedml.model", "/model"), ("fedml.model.cv", "/model/cv")]:
        _stub_pkg(name, REF + sub)
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        rn = importlib.import_module("fedml.model.cv.resnet_gn").resnet18()
    sd = rn.state_dict()
    out = {"resnet18_gn": [[k, list(v.shape), dtype_name(v)] for k, v in sd.items()]}
    # ViT-B/16 (synthetic: the reference has no ViT) in torchvision's state_dict order
    D, L, M, C = 768, 12, 3072, 1000
    vit = [["class_token", [1, 1, D], "bfloat16"], ["conv_proj.weight", [D, 3, 16, 16], "bfloat16"],
           ["conv_proj.bias", [D], "bfloat16"], ["encoder.pos_embedding", [1, 197, D], "bfloat16"]]
    for i in range(L):
        p = f"encoder.layers.encoder_layer_{i}."
        vit += [[p + "ln_1.weight", [D], "bfloat16"], [p + "ln_1.bias", [D], "bfloat16"],
                [p + "self_attention.in_proj_weight", [3 * D, D], "bfloat16"],
                [p + "self_attention.in_proj_bias", [3 * D], "bfloat16"],
                [p + "self_attention.out_proj.weight", [D, D], "bfloat16"],
                [p + "self_attention.out_proj.bias", [D], "bfloat16"],
                [p + "ln_2.weight", [D], "bfloat16"], [p + "ln_2.bias", [D], "bfloat16"],
                [p + "mlp.0.weight", [M, D], "bfloat16"], [p + "mlp.0.bias", [M], "bfloat16"],
                [p + "mlp.3.weight", [D, M], "bfloat16"], [p + "mlp.3.bias", [D], "bfloat16"]]
    vit += [["encoder.ln.weight", [D], "bfloat16"], ["encoder.ln.bias", [D], "bfloat16"],
            ["heads.head.weight", [C, D], "bfloat16"], ["heads.head.bias", [C], "bfloat16"]]
    out["vit_b16_bf16"] = vit
    out["lr_mnist"] = [["linear.weight", [10, 784], "float32"], ["linear.bias", [10], "float32"]]
    with open(os.path.join(HERE, "layouts.json"), "w") as f:
        json.dump(out, f, indent=0)
    for k, v in out.items():
        numel = sum(int(np.prod(s)) for _, s, _ in v)
        print(f"layout {k}: {len(v)} tensors, {numel} elements")


def cases_promotion():
    """G19: clients that DISAGREE on a key's dtype, through the reference's FedMLAggOperator.agg:
    every ``avg[k] += x_i[k] * w_i`` (and the plain-sum branch's ``avg[k] += x_i[k]``) is an
    in-place add across dtypes -- computed in the promoted type of (avg, term), rounded to avg's
    dtype (agg_operator.py:37-44, 55-63)."""
    ao = load_agg_operator()
    agg = ao.FedMLAggOperator.agg
    f32, f64, bf, f16, i64, i32, i16 = (torch.float32, torch.float64, torch.bfloat16, torch.float16, torch.int64,
                                       torch.int32, torch.int16)

    def clients_of(seed, spec):
        """spec: [(key, shape, [dtype per client])]: wide-magnitude values so roundings matter."""
        g = torch.Generator().manual_seed(seed)
        K = len(spec[0][2])
        out = [OrderedDict() for _ in range(K)]
        for key, shape, dts in spec:
            for i, dt in enumerate(dts):
                if dt in (i64, i32, i16):
                    lim = {i64: 2 ** 40, i32: 2 ** 30, i16: 2 ** 14}[dt]
                    out[i][key] = torch.randint(-lim, lim, shape, generator=g, dtype=dt)
                else:
                    v = torch.randn(shape, generator=g, dtype=f64) * torch.exp2(
                        torch.randint(-12, 12, shape, generator=g).double())
                    out[i][key] = v.to(dt)
        return out

    cases = [
        ("g19_promote_fedavg_K5", "FedAvg", [("w", (1000,), [f32, f64, bf, i64, f16]),
                                             ("v", (7, 3), [bf, f32, f16, f64, i64]),
                                             ("s", (), [i64, f32, f64, i64, bf])]),
        ("g19_promote_fedavg_K3", "FedAvg", [("a", (513,), [f64, f32, f32]),
                                             ("b", (257,), [f16, bf, f32]),
                                             ("c", (129,), [bf, i64, i64]),
                                             ("d", (65,), [f16, i64, f64])]),
        ("g19_promote_sum_K4", "FedAvg_seq", [("w", (1000,), [f32, f64, bf, f16]),
                                              ("n", (33,), [i64, i32, i64, i16]),
                                              ("h", (17,), [bf, f32, i64, f16]),
                                              ("q", (9,), [f16, i64, bf, f32])]),
    ]
    for name, opt, spec in cases:
        clients = clients_of(len(WRITTEN) + 1900, spec)
        n = gen_counts(19, len(clients))
        out = agg(Args(federated_optimizer=opt), list(zip(n, dc(clients))))
        meta = dict(kind="agg", optimizer=opt, n=n, ref="agg_operator.py:35-63 (in-place add across dtypes)",
                    client_in_dtypes=[[dtype_name(c[k]) for k in c] for c in clients])
        write(name, clients, [out], meta)


def main():
    if len(sys.argv) > 1:  # regenerate only the named families, e.g. `make_golden.py secagg`
        for part in sys.argv[1:]:
            globals()["cases_" + part]()
        for name, s in WRITTEN:
            print(f"{name:45s} {s:9d} B")
        return
    ao = load_agg_operator()
    stm, tu = load_topology()
    cases_agg_operator(ao)
    cases_call_sites()
    cases_topology_and_mixing(stm, tu)
    cases_fedopt()
    cases_secagg()
    cases_promotion()
    layouts(ao)
    total = sum(s for _, s in WRITTEN)
    for name, s in WRITTEN:
        print(f"{name:45s} {s:9d} B")
    print(f"total {total / 1e6:.2f} MB in {len(WRITTEN)} files")


if __name__ == "__main__":
    main()
