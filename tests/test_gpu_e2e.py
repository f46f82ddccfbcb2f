"""End-to-end FL rounds with the engine as the drop-in aggregator (BASELINE configs[0]: the
reference's quick_start -- FedAvg, logistic regression on MNIST-shaped data, 2 clients).

Each round: every client loads the global model, trains locally (ClientTrainer), and the server
averages the updates.  The same loop is run twice, once aggregating with fedml_amd and once with
the reference's op sequence (oracle/torch_port.py); local training is deterministic and identical
in both, so the global models after R rounds must be bit-identical -- by induction, every round's
aggregation was.  MNIST itself is not downloadable here: the data are synthetic
784-feature, 10-class samples of the reference's shapes (fedml/model/linear/lr.py:4-12)."""
from __future__ import annotations

import copy
import types
from collections import OrderedDict

import pytest
import torch

from refcases import assert_dict_bits

pytestmark = pytest.mark.gpu


class LogisticRegression(torch.nn.Module):
    """fedml/model/linear/lr.py: Linear(784, 10) + sigmoid."""

    def __init__(self, d_in=784, d_out=10):
        super().__init__()
        self.linear = torch.nn.Linear(d_in, d_out)

    def forward(self, x):
        return torch.sigmoid(self.linear(x))


def make_trainer_cls():
    from fedml_amd.core.alg_frame.client_trainer import ClientTrainer

    class LRTrainer(ClientTrainer):
        """ml/trainer/my_model_trainer_classification.py: SGD, CrossEntropy, `epochs` local epochs."""

        def get_model_params(self):
            return OrderedDict((k, v.detach().clone()) for k, v in self.model.state_dict().items())

        def set_model_params(self, model_parameters):
            self.model.load_state_dict(model_parameters)

        def train(self, train_data, device, args):
            model = self.model.to(device)
            model.train()
            opt = torch.optim.SGD(model.parameters(), lr=args.learning_rate)
            loss_fn = torch.nn.CrossEntropyLoss()
            for _ in range(args.epochs):
                for x, y in train_data:
                    opt.zero_grad()
                    loss_fn(model(x.to(device)), y.to(device)).backward()
                    opt.step()
    return LRTrainer


def client_data(n_clients, seed=0, batch=32):
    g = torch.Generator().manual_seed(seed)
    data, nums = [], []
    for c in range(n_clients):
        n = 64 + 37 * c  # unequal sample counts -> non-trivial FedAvg weights
        x = torch.rand(n, 784, generator=g)
        y = torch.randint(0, 10, (n,), generator=g)
        data.append([(x[i:i + batch], y[i:i + batch]) for i in range(0, n, batch)])
        nums.append(n)
    return data, nums


def run_rounds(aggregate, device, n_clients=2, rounds=3, epochs=2):
    torch.manual_seed(0)
    args = types.SimpleNamespace(learning_rate=0.05, epochs=epochs, comm_round=rounds)
    global_model = LogisticRegression().to(device)
    trainers = [make_trainer_cls()(LogisticRegression().to(device), args) for _ in range(n_clients)]
    data, nums = client_data(n_clients)
    w_global = OrderedDict((k, v.clone()) for k, v in global_model.state_dict().items())
    for _ in range(rounds):
        w_locals = []
        for i, t in enumerate(trainers):
            t.set_model_params(copy.deepcopy(w_global))
            t.train(data[i], device, args)
            w_locals.append((nums[i], t.get_model_params()))
        w_global = aggregate(w_locals)
    return w_global


def _ref_aggregate(w_locals):
    """The reference's op sequence on CPU copies (agg_operator.py:35-44 / fedavg_api.py:144-159)."""
    import oracle.torch_port as tp
    dev = next(iter(w_locals[0][1].values())).device
    cpu = [(n, OrderedDict((k, v.detach().cpu().clone()) for k, v in d.items())) for n, d in w_locals]
    out = tp.sp_aggregate(cpu)
    return OrderedDict((k, v.to(dev)) for k, v in out.items())


@pytest.mark.parametrize("n_clients", [2, 5])
@pytest.mark.parametrize("where", ["cuda:0", "cpu"])
def test_fedavg_rounds_dropin_operator(n_clients, where):
    """configs[0] through FedMLAggOperator.agg (the server's plugin call), GPU- or CPU-resident
    training (CPU: the host-ingest path packs the CPU state_dicts for the device)."""
    from fedml_amd.ml.aggregator.agg_operator import FedMLAggOperator
    args = types.SimpleNamespace(federated_optimizer="FedAvg")
    got = run_rounds(lambda wl: FedMLAggOperator.agg(args, wl), where, n_clients)
    exp = run_rounds(_ref_aggregate, where, n_clients)
    for k in exp:
        assert got[k].device.type == exp[k].device.type, k
    assert_dict_bits(OrderedDict((k, v.cpu()) for k, v in got.items()),
                     OrderedDict((k, v.cpu()) for k, v in exp.items()), "global model after 3 rounds")


def test_fedavg_api_train_loop():
    """fedml_amd.simulation.sp.fedavg_api.FedAvgAPI.train (the reference's SP round loop)."""
    from fedml_amd.simulation.sp.fedavg_api import FedAvgAPI
    torch.manual_seed(0)
    args = types.SimpleNamespace(learning_rate=0.05, epochs=2, comm_round=3)
    model = LogisticRegression().to("cuda:0")
    trainers = [make_trainer_cls()(LogisticRegression().to("cuda:0"), args) for _ in range(3)]
    data, nums = client_data(3)
    api = FedAvgAPI(args, "cuda:0", model, trainers, data, nums)
    got = api.train()
    exp = run_rounds(_ref_aggregate, "cuda:0", n_clients=3)
    assert_dict_bits(OrderedDict((k, v.cpu()) for k, v in got.items()),
                     OrderedDict((k, v.cpu()) for k, v in exp.items()), "FedAvgAPI.train")


def run_rounds_sampled(aggregate, device, total, per_round, rounds=3, epochs=1, keep=None):
    """The reference's SP loop with its client sampling (fedavg_api.py:80-84, 127-135: np.random.seed
    (round_idx) + np.random.choice without replacement) and its aggregation on CPU copies."""
    import numpy as np
    torch.manual_seed(0)
    args = types.SimpleNamespace(learning_rate=0.05, epochs=epochs, comm_round=rounds)
    global_model = LogisticRegression().to(device)
    trainers = [make_trainer_cls()(LogisticRegression().to(device), args) for _ in range(total)]
    data, nums = client_data(total)
    w_global = OrderedDict((k, v.clone()) for k, v in global_model.state_dict().items())
    for r in range(rounds):
        if total == per_round:
            idx = list(range(total))
        else:
            np.random.seed(r)
            idx = np.random.choice(range(total), min(per_round, total), replace=False)
        w_locals = []
        for i in idx:
            t = trainers[int(i)]
            t.set_model_params(copy.deepcopy(w_global))
            t.train(data[int(i)], device, args)
            w_locals.append((nums[int(i)], t.get_model_params()))
        w_global = aggregate(w_locals)
        if keep is not None:
            keep.append(OrderedDict((k, v.detach().cpu().clone()) for k, v in w_global.items()))
    return w_global


@pytest.mark.parametrize("where", ["cuda:0", "cpu"])
def test_fedavg_api_train_samples_like_the_reference(where):
    """FedAvgAPI.train with client_num_per_round < client_num_in_total and no injected sampler: the
    reference's _client_sampling picks the clients, and the global model after 3 rounds is
    bit-identical to the reference loop's; on a CPU model the result stays on the CPU."""
    from fedml_amd.simulation.sp.fedavg_api import FedAvgAPI
    torch.manual_seed(0)
    total, per_round = 7, 3
    args = types.SimpleNamespace(learning_rate=0.05, epochs=1, comm_round=3, client_num_in_total=total,
                                 client_num_per_round=per_round)
    model = LogisticRegression().to(where)
    trainers = [make_trainer_cls()(LogisticRegression().to(where), args) for _ in range(total)]
    data, nums = client_data(total)
    api = FedAvgAPI(args, where, model, trainers, data, nums)
    got = api.train()
    exp = run_rounds_sampled(_ref_aggregate, where, total, per_round)
    assert all(v.device.type == torch.device(where).type for v in got.values())
    assert_dict_bits(OrderedDict((k, v.cpu()) for k, v in got.items()),
                     OrderedDict((k, v.cpu()) for k, v in exp.items()), "FedAvgAPI.train sampled")
