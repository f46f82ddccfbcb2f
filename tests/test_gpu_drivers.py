"""The round drivers (callers of the engine) reproduce the reference functions they mirror,
bit-for-bit, on the golden fixtures generated from those very functions."""
from __future__ import annotations

import os
import types
from collections import OrderedDict

import numpy as np
import pytest
import torch

from golden_io import GOLDEN_DIR, client_dicts, expected_dicts, load_case
from refcases import assert_dict_bits

pytestmark = pytest.mark.gpu


def case(name):
    return load_case(os.path.join(GOLDEN_DIR, name + ".npz"))


def on_gpu(d):
    return OrderedDict((k, v.cuda()) for k, v in d.items())


def cpu(d):
    return OrderedDict((k, v.cpu()) for k, v in d.items())


@pytest.mark.parametrize("where", ["cpu", "cuda"])
def test_sp_fedavg_aggregate(where):
    from fedml_amd.simulation.sp.fedavg_api import FedAvgAPI
    meta, arr = case("g1_sp_aggregate_K9")
    cl = client_dicts(meta, arr)
    if where == "cuda":
        cl = [on_gpu(c) for c in cl]
    api = FedAvgAPI(types.SimpleNamespace(), "cuda:0", None)
    got = api._aggregate(list(zip(meta["n"], cl)))
    assert_dict_bits(cpu(got), expected_dicts(meta, arr)[0], "sp")


@pytest.mark.parametrize("name", ["g4_mpi_xn_div_N_K3", "g4_mpi_xn_div_N_K32", "g4_mpi_xn_div_N_lr_K2",
                                  "g4_mpi_xn_div_N_bf16_K4", "g4_mpi_xn_div_N_bigcounts_K3",
                                  "g4_mpi_xn_div_N_int64_K5"])
def test_mpi_fedavg_aggregator(name):
    from fedml_amd.simulation.mpi.fedavg_aggregator import FedAVGAggregator
    meta, arr = case(name)
    cl = client_dicts(meta, arr)
    agg = FedAVGAggregator(worker_num=len(cl))
    for i in reversed(range(len(cl))):  # arrival order must not matter
        assert not agg.check_whether_all_receive()
        agg.add_local_trained_result(i, cl[i], meta["n"][i])
    assert agg.check_whether_all_receive()
    got = agg.aggregate()
    assert_dict_bits(cpu(got), expected_dicts(meta, arr)[0], name)


def test_fedavg_seq_two_level():
    from fedml_amd.simulation.mpi import fedavg_seq as fs
    meta, arr = case("g6_fedavg_seq_two_level_K10")
    cl = [on_gpu(c) for c in client_dicts(meta, arr)]
    n = meta["n"]
    w = fs.get_average_weight({i: n[i] for i in range(len(n))}, list(range(len(n))))
    # batched worker partials
    partials = [fs.worker_partial([cl[i] for i in wk], [w[i] for i in wk]) for wk in meta["schedule"]]
    got = fs.server_aggregate(partials)
    exp = expected_dicts(meta, arr)[0]
    assert_dict_bits(cpu(got), exp, "fedavg_seq batched")
    # incremental add_client_model, clients arriving one by one
    partials = []
    for wk in meta["schedule"]:
        acc = {}
        for i in wk:
            fs.add_client_model(acc, cl[i], w[i])
        partials.append(acc)
    assert_dict_bits(cpu(fs.server_aggregate(partials)), exp, "fedavg_seq incremental")


def test_add_client_model_int_buffers():
    """int64 buffers are promoted by the first p*w and keep the reference's arithmetic after."""
    from fedml_amd.simulation.mpi import fedavg_seq as fs
    from oracle import torch_port
    g = torch.Generator().manual_seed(3)
    cl = [OrderedDict(w=torch.randn(1000, generator=g), steps=torch.randint(0, 99, (), generator=g))
          for _ in range(4)]
    ws = [0.1, 0.2, 0.3, 0.4]
    exp, acc = {}, {}
    for c, w in zip(cl, ws):
        torch_port.fedavg_seq_worker(exp, c, w)
        fs.add_client_model(acc, on_gpu(c), w)
    assert_dict_bits(cpu(acc), OrderedDict(exp), "int buffers")


def test_hierarchical_sp():
    from fedml_amd.simulation.sp.hierarchical import hierarchical_round
    meta, arr = case("g7_hier_sp_K12_G3")
    cl = [on_gpu(c) for c in client_dicts(meta, arr)]
    n = meta["n"]
    groups = {g: [(n[i], cl[i]) for i in members] for g, members in enumerate(meta["groups"])}
    assert_dict_bits(cpu(hierarchical_round(groups)), expected_dicts(meta, arr)[0], "hier sp")


def _cloud(meta, cl):
    from fedml_amd.simulation.mpi.hier_cloud_aggregator import HierFedAVGCloudAggregator
    E, R = meta["edges"], meta["group_comm_round"]
    agg = HierFedAVGCloudAggregator(worker_num=E)
    for e in range(E):
        agg.add_local_trained_result(e, [(r, on_gpu(cl[e * R + r])) for r in range(R)], meta["edge_counts"][e])
    assert agg.check_whether_all_receive()
    return agg


def test_hier_cloud_aggregate_with_reference_double_pass():
    meta, arr = case("g7_hier_cloud_aggregate_E3_R2")
    agg = _cloud(meta, client_dicts(meta, arr))
    assert_dict_bits(cpu(agg.aggregate()), expected_dicts(meta, arr)[0], "cloud aggregate")


def test_hier_cloud_mix():
    meta, arr = case("g8_cloud_mix_ring_E8_R2")
    agg = _cloud(meta, client_dicts(meta, arr))
    topo = types.SimpleNamespace(topology=arr["W"])
    got = agg.mix(topo)
    exp = expected_dicts(meta, arr)
    assert len(got) == len(exp)
    for j, (g, e) in enumerate(zip(got, exp)):
        assert_dict_bits(cpu(g), e, f"mix[{j}]")


@pytest.mark.parametrize("name", ["g8_pfedavg_mixing_ring_E8", "g8_pfedavg_mixing_complete_E8",
                                  "g9_mixing_nonfinite_ring_E8"])
def test_pfedavg_mixing_rows(name):
    from fedml_amd.simulation.mpi.hier_cloud_aggregator import HierFedAVGCloudAggregator
    meta, arr = case(name)
    cl = [on_gpu(c) for c in client_dicts(meta, arr)]
    W = arr["W"]
    exp = expected_dicts(meta, arr)
    for i in range(W.shape[0]):
        got = HierFedAVGCloudAggregator._pfedavg_mixing_([(meta["n"][j], cl[j]) for j in range(len(cl))], W[i])
        assert_dict_bits(cpu(got), exp[i], f"{name} row {i}")


def test_dsgd_and_pushsum_steps():
    from fedml_amd.simulation.sp.decentralized import dsgd_step, pushsum_step
    meta, arr = case("g8_dsgd_ring_N8")
    cl = [on_gpu(c) for c in client_dicts(meta, arr)]
    for g, e in zip(dsgd_step(cl, arr["W"]), expected_dicts(meta, arr)):
        assert_dict_bits(cpu(g), e, "dsgd")
    meta, arr = case("g8_pushsum_ring_N8")
    cl = [on_gpu(c) for c in client_dicts(meta, arr)]
    _, z, om = pushsum_step(cl, arr["W"], meta["omegas_in"])
    assert om == meta["omegas_out"]
    for g, e in zip(z, expected_dicts(meta, arr)):
        assert_dict_bits(cpu(g), e, "pushsum")


def test_cross_silo_round_with_user_server_aggregator():
    """A user-defined ServerAggregator subclass drives a full cross-silo aggregation round."""
    from fedml_amd.core.alg_frame.server_aggregator import ServerAggregator
    from fedml_amd.cross_silo.server.fedml_aggregator import FedMLAggregator

    class MyServerAggregator(ServerAggregator):
        def get_model_params(self):
            return self.model.state_dict()

        def set_model_params(self, p):
            self.model.load_state_dict(p)

        def test(self, test_data, device, args):
            return None

    meta, arr = case("g1_fedavg_lr_K2")
    cl = client_dicts(meta, arr)
    model = torch.nn.Module()
    model.linear = torch.nn.Linear(784, 10)
    args = types.SimpleNamespace(federated_optimizer="FedAvg")
    srv = FedMLAggregator(client_num=2, device="cuda:0", args=args, server_aggregator=MyServerAggregator(model, args))
    srv.add_local_trained_result(1, cl[1], meta["n"][1])
    assert not srv.check_whether_all_receive()
    srv.add_local_trained_result(0, cl[0], meta["n"][0])
    assert srv.check_whether_all_receive()
    avg, _, idx = srv.aggregate()
    exp = expected_dicts(meta, arr)[0]
    assert_dict_bits(cpu(avg), exp, "cross-silo")
    assert idx == [0, 1]
    assert torch.equal(model.linear.weight.detach().cpu(), exp["linear.weight"])


def test_default_server_aggregator_round():
    from fedml_amd.ml.aggregator.default_aggregator import create_server_aggregator
    model = torch.nn.Sequential(torch.nn.Linear(8, 4))
    args = types.SimpleNamespace(federated_optimizer="FedAvg", dataset="synthetic")
    agg = create_server_aggregator(model, args)
    g = torch.Generator().manual_seed(0)
    ups = [(10 * (i + 1), OrderedDict((k, torch.randn(v.shape, generator=g)) for k, v in model.state_dict().items()))
           for i in range(3)]
    avg = agg.aggregate(agg.on_before_aggregation(ups)[0])
    agg.set_model_params(agg.on_after_aggregation(avg))
    data = [(torch.randn(16, 8, generator=g), torch.randint(0, 4, (16,), generator=g))]
    acc, loss, _, _ = agg.test(data, "cuda:0", args)
    assert 0.0 <= acc <= 1.0 and loss > 0


@pytest.mark.parametrize("name", ["g3_fedavg_mixed_K5", "g2_fedavg_bf16_K7_P4099", "g1_fedavg_lr_K2",
                                  "g2_fedavg_f64_K5", "g9_edge_values_K4"])
@pytest.mark.parametrize("src", ["cpu", "cuda"])
def test_client_arena_fedavg(name, src):
    """Updates ingested into a ClientArena (host via pinned staging, or device) aggregate to the
    reference's FedAvg result."""
    from fedml_amd.arena import ClientArena
    meta, arr = case(name)
    cl = client_dicts(meta, arr)
    arena = ClientArena.for_model(cl[0], capacity=len(cl) + 1, device="cuda:0")
    for i, c in enumerate(cl):
        arena.write(i, on_gpu(c) if src == "cuda" else c)
    got = arena.fedavg(meta["n"], clients=list(range(len(cl))))
    assert_dict_bits(cpu(got), expected_dicts(meta, arr)[0], f"arena:{name}")


def test_client_arena_rejects_wrong_dtype():
    from fedml_amd.arena import ClientArena
    tmpl = OrderedDict(w=torch.zeros(10), b=torch.zeros(3, dtype=torch.bfloat16))
    arena = ClientArena.for_model(tmpl, capacity=2, device="cuda:0")
    with pytest.raises(TypeError):
        arena.write(0, OrderedDict(w=torch.zeros(10, dtype=torch.float64), b=torch.zeros(3, dtype=torch.bfloat16)))
    with pytest.raises(KeyError):
        arena.write(0, OrderedDict(w=torch.zeros(10)))


def test_arena_fused_hierarchical_sp_golden():
    """SP hierarchical round (group FedAvg then global FedAvg over groups) in ONE kernel pass."""
    from fedml_amd.arena import ClientArena
    meta, arr = case("g7_hier_sp_K12_G3")
    cl = client_dicts(meta, arr)
    arena = ClientArena.for_model(cl[0], capacity=len(cl), device="cuda:0")
    for i, c in enumerate(cl):
        arena.write(i, c)
    got = arena.hierarchical(meta["groups"], meta["n"], formula="sp")
    assert_dict_bits(cpu(got), expected_dicts(meta, arr)[0], "fused hier sp")


def test_arena_fused_fedavg_seq_golden():
    """fedavg_seq two-level reduce (worker partials with global weights, then the plain sum), fused."""
    from fedml_amd.arena import ClientArena
    from fedml_amd.engine import MUL_W, SUM
    meta, arr = case("g6_fedavg_seq_two_level_K10")
    cl = client_dicts(meta, arr)
    arena = ClientArena.for_model(cl[0], capacity=len(cl), device="cuda:0")
    for i, c in enumerate(cl):
        arena.write(i, c)
    n = meta["n"]
    sched = meta["schedule"]
    w = [n[i] / sum(n) for wk in sched for i in wk]
    got = arena.aggregate_grouped(sched, MUL_W, w, 1.0, SUM)
    assert_dict_bits(cpu(got), expected_dicts(meta, arr)[0], "fused fedavg_seq")


@pytest.mark.parametrize("name", ["g10_fedopt_sgd_lr0.7_m0.9", "g10_fedopt_sgd_lr1.0_m0.0",
                                  "g10_fedopt_rmsprop_lr0.01_m0.9", "g10_fedopt_rmsprop_lr0.05_m0.0"])
@pytest.mark.parametrize("where", ["cuda", "cpu"])
def test_fedopt_fused_server_step_golden(name, where):
    """FedOptAggregator (fused FedAvg + optimizer step) == the reference's FedOptAggregator, 3 rounds:
    bit-exact for SGD; for RMSprop within 1e-6 relative (normwise per tensor) -- the reference's
    CPU sqrt is MKL-VML, not correctly rounded -- and the buffers (plain averages) bit-exact."""
    from golden_io import np_to_tensor
    from refcases import fedopt_expected
    from fedml_amd.simulation.mpi.fedopt_aggregator import FedOptAggregator
    meta, arr = case(name)
    model = torch.nn.Sequential(torch.nn.Linear(33, 17), torch.nn.BatchNorm1d(17), torch.nn.Linear(17, 5))
    model.load_state_dict(OrderedDict((k, np_to_tensor(arr[f"init__{k}"], dt))
                                      for k, dt in zip(meta["keys"], meta["dtypes"])))
    model = model.to("cuda:0" if where == "cuda" else "cpu")

    class Agg:
        def __init__(self, m):
            self.model = m

        def get_model_params(self):
            return self.model.state_dict()

        def set_model_params(self, p):
            self.model.load_state_dict(p)

    args = types.SimpleNamespace(server_optimizer=meta["server_optimizer"], server_lr=meta["server_lr"],
                                 server_momentum=meta["server_momentum"])
    fo = FedOptAggregator(worker_num=4, server_aggregator=Agg(model), args=args)
    for r, (rd, exp) in enumerate(zip(meta["rounds"], fedopt_expected(meta, arr))):
        for i in range(4):
            fo.add_local_trained_result(i, OrderedDict((k, np_to_tensor(arr[f"r{r}_x{i}__{k}"], dt))
                                                       for k, dt in zip(meta["keys"], meta["dtypes"])), rd["n"][i])
        assert fo.check_whether_all_receive()
        got = cpu(fo.aggregate())
        if meta["server_optimizer"] == "sgd":
            assert_dict_bits(got, exp, f"{name} round {r}")
            continue
        params = set(meta["params"])
        for k in exp:
            if k in params:
                rel = float((got[k].double() - exp[k].double()).norm() / exp[k].double().norm())
                assert rel <= 1e-6, (name, r, k, rel)
            else:
                assert_dict_bits(OrderedDict([(k, got[k])]), OrderedDict([(k, exp[k])]), f"{name} round {r}")


def _rmsprop_cr(p, avg, sq, buf, lr, alpha, eps, wd, momentum):
    """torch.optim.RMSprop's CPU op sequence (rmsprop.py _single_tensor_rmsprop, ATen's contracted
    addcmul / addcdiv) with a CORRECTLY ROUNDED sqrt, float32 via exact float64 emulation."""
    f, d = (lambda x: x.float()), (lambda x: x.double())
    g = p - avg
    if wd:
        g = f(d(p) * wd32(wd) + d(g))
    s1 = torch.tensor(1 - alpha, dtype=torch.float32)
    sq = f(d(s1 * g) * d(g) + d(sq * torch.tensor(alpha, dtype=torch.float32)))
    den = f(d(sq).sqrt()) + torch.tensor(eps, dtype=torch.float32)
    nlr = torch.tensor(-lr, dtype=torch.float32)
    if momentum:
        buf = buf * torch.tensor(momentum, dtype=torch.float32) + g / den
        p = f(d(buf) * d(nlr) + d(p))
    else:
        p = p + (nlr * g) / den
    return p, sq, buf


def wd32(wd):
    return float(torch.tensor(wd, dtype=torch.float32))


@pytest.mark.parametrize("momentum,wd", [(0.0, 0.0), (0.9, 0.0), (0.5, 1e-3)])
def test_fedavg_rmsprop_vs_torch_optimizer(momentum, wd):
    """fa_fedavg_rmsprop over 4 rounds, 1 M parameters: bit-exact to torch.optim.RMSprop's op
    sequence with a correctly rounded sqrt, and within 1e-6 relative (normwise) of
    torch.optim.RMSprop itself on this host's CPU (whose sqrt is MKL-VML, not correctly rounded)."""
    from oracle import orc
    from fedml_amd.engine import get_engine
    eng = get_engine(0)
    g = torch.Generator().manual_seed(11)
    n, K, lr, alpha, eps = 1 << 20, 6, 0.01, 0.99, 1e-8
    p_cpu = torch.nn.Parameter(torch.randn(n, generator=g))
    opt = torch.optim.RMSprop([p_cpu], lr=lr, momentum=momentum, weight_decay=wd)
    p_dev = p_cpu.detach().clone().cuda()
    p_cr, sq_cr, buf_cr = p_cpu.detach().clone(), torch.zeros(n), torch.zeros(n)
    sq = torch.empty(n, device="cuda:0")
    buf = torch.empty(n, device="cuda:0")
    for r in range(4):
        xs = [p_cr + 0.1 * torch.randn(n, generator=g) for _ in range(K)]
        w = [(i + 1) / (K * (K + 1) / 2) for i in range(K)]
        avg = orc.weighted_sum(xs, 0, w)
        opt.zero_grad()
        p_cpu.grad = p_cpu.detach() - avg
        opt.step()
        p_cr, sq_cr, buf_cr = _rmsprop_cr(p_cr, avg, sq_cr, buf_cr, lr, alpha, eps, wd, momentum)
        eng.fedavg_rmsprop([[x.cuda() for x in xs]], w, [p_dev], [sq], [buf] if momentum else None, lr,
                           weight_decay=wd, momentum=momentum, first_step=(r == 0))
        got = p_dev.cpu()
        assert torch.equal(got.view(torch.int32), p_cr.view(torch.int32)), r
        exp = p_cpu.detach()
        rel = float((got.double() - exp.double()).norm() / exp.double().norm())
        assert rel <= 1e-6, (r, rel)


def test_pushsum_step_device_omega():
    """PushSum with the weights on the device (fa_pushsum): omega' mixed by the same rows in float32,
    1/omega' and z on the GPU -- the reference's outputs (g8 fixture) bit for bit, then 3 more steps
    on a 37-node ring equal to the host bookkeeping path."""
    from fedml_amd.core.distributed.topology.topology_manager import SymmetricTopologyManager
    from fedml_amd.simulation.sp.decentralized import pushsum_step
    meta, arr = case("g8_pushsum_ring_N8")
    cl = [on_gpu(c) for c in client_dicts(meta, arr)]
    x, z, om = pushsum_step(cl, arr["W"], torch.tensor(meta["omegas_in"], dtype=torch.float32, device="cuda:0"))
    assert om.is_cuda and om.cpu().tolist() == meta["omegas_out"]
    for g, e in zip(z, expected_dicts(meta, arr)):
        assert_dict_bits(cpu(g), e, "pushsum device omega")
    m = SymmetricTopologyManager(37, 4)
    m.generate_topology()
    g = torch.Generator().manual_seed(4)
    nodes = [OrderedDict(w=torch.randn(3001, generator=g).cuda(), b=torch.randn(7, generator=g).cuda()) for _ in range(37)]
    om_host = [np.float32(1.0 + i / 37) for i in range(37)]
    om_dev = torch.tensor([float(o) for o in om_host], dtype=torch.float32, device="cuda:0")
    xa, xb = nodes, nodes
    for step in range(3):
        xa, za, om_host = pushsum_step(xa, m.topology, om_host)
        xb, zb, om_dev = pushsum_step(xb, m.topology, om_dev)
        assert [float(o) for o in om_host] == om_dev.cpu().tolist(), step
        for a, b in zip(za, zb):
            assert_dict_bits(cpu(a), cpu(b), f"step {step}")
