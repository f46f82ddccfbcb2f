"""FedOpt server aggregator (reference: python/fedml/simulation/mpi/fedopt/FedOptAggregator.py:
14-131) with the server optimizer step fused into the aggregation pass.

Reference semantics, reproduced bit-for-bit (fixtures g10_*):
* FedAvg of the clients' state_dicts (weights n_i / N, client order);
* parameters: pseudo-gradient ``grad = w_global - avg`` (set_model_global_grads :118-131), then a
  ``torch.optim`` step of the global parameters; the optimizer is re-created every round with its
  state carried over (:104-112), so momentum persists across rounds;
* everything that is not a parameter (BatchNorm running statistics, ``num_batches_tracked``) takes
  the average, cast into the buffer's dtype by ``load_state_dict`` (an int64 buffer truncates).

The MI355X path runs the average, the pseudo-gradient and the SGD update of every parameter in ONE
kernel pass (``fa_fedavg_sgd``: reads the K client tensors, the parameter and its momentum buffer,
writes the parameter and the buffer in place), instead of FedAvg + state_dict copies + a separate
optimizer pass.  Server optimizers: ``sgd`` (momentum, dampening, nesterov, weight decay as
torch.optim.SGD; bit-exact) and ``rmsprop`` (torch.optim.RMSprop defaults alpha = 0.99, eps = 1e-8,
centered = False; within 1e-6 relative -- the reference's CPU sqrt is MKL-VML, not correctly
rounded).  The reference instantiates its optimizer with ``lr=`` and ``momentum=`` for any name
(FedOptAggregator.py:49-54), so those two are the only ones it can construct (Adam, Adagrad, ...
raise TypeError there); others raise NotImplementedError here.
"""
from __future__ import annotations

import logging
import time
from typing import Dict, List

import torch

from ...engine import get_engine
from ...ml.aggregator.state_dict_agg import MUL_W, aggregate


class FedOptAggregator:
    def __init__(self, worker_num: int, server_aggregator, args):
        self.worker_num = worker_num
        self.aggregator = server_aggregator
        self.args = args
        name = str(getattr(args, "server_optimizer", "sgd")).lower()
        if name not in ("sgd", "rmsprop"):
            raise NotImplementedError(f"server_optimizer={name!r}: the fused FedOpt step implements 'sgd' and "
                                      "'rmsprop' (the optimizers the reference can construct with momentum=)")
        self.opt_name = name
        self.lr = float(args.server_lr)
        self.momentum = float(getattr(args, "server_momentum", 0.0) or 0.0)
        self.dampening = float(getattr(args, "server_dampening", 0.0) or 0.0)
        self.weight_decay = float(getattr(args, "server_weight_decay", 0.0) or 0.0)
        self.nesterov = bool(getattr(args, "server_nesterov", False))
        self.model_dict: Dict[int, dict] = {}
        self.sample_num_dict: Dict[int, int] = {}
        self.flag_client_model_uploaded_dict = {i: False for i in range(worker_num)}
        self.momentum_buffer: Dict[str, torch.Tensor] = {}
        self.square_avg: Dict[str, torch.Tensor] = {}  # rmsprop state

    def get_global_model_params(self):
        return self.aggregator.get_model_params()

    def set_global_model_params(self, model_parameters):
        self.aggregator.set_model_params(model_parameters)

    def add_local_trained_result(self, index, model_params, sample_num):
        self.model_dict[index] = model_params
        self.sample_num_dict[index] = sample_num
        self.flag_client_model_uploaded_dict[index] = True

    def check_whether_all_receive(self) -> bool:
        if not all(self.flag_client_model_uploaded_dict[i] for i in range(self.worker_num)):
            return False
        for i in range(self.worker_num):
            self.flag_client_model_uploaded_dict[i] = False
        return True

    def aggregate(self):
        t0 = time.time()
        counts = [self.sample_num_dict[i] for i in range(self.worker_num)]
        dicts = [self.model_dict[i] for i in range(self.worker_num)]
        N = sum(counts)
        w = [c / N for c in counts]
        model = self.aggregator.model
        named = [(k, p) for k, p in model.named_parameters() if p.requires_grad]
        stepped = {k for k, _ in named}
        all_params = {k for k, _ in model.named_parameters()}
        dev = next(model.parameters()).device
        eng = get_engine(dev.index if dev.type == "cuda" else None)
        on_gpu = dev.type == "cuda"
        # global parameters: fused FedAvg + pseudo-gradient + SGD step, in place
        gparams = [p.data if on_gpu else p.data.to(eng.device) for _, p in named]
        segs = [[d[k].to(eng.device).contiguous() for d in dicts] for k, _ in named]
        first = [k not in (self.square_avg if self.opt_name == "rmsprop" else self.momentum_buffer) for k, _ in named]
        rms = self.opt_name == "rmsprop"
        for (k, p), g in zip(named, gparams):
            if self.momentum != 0.0 and k not in self.momentum_buffer:
                self.momentum_buffer[k] = torch.empty_like(g)
            if rms and k not in self.square_avg:
                self.square_avg[k] = torch.empty_like(g)
        for flag in (True, False):
            idx = [j for j, f in enumerate(first) if f == flag]
            if not idx:
                continue
            mbufs = [self.momentum_buffer[named[j][0]] for j in idx] if self.momentum != 0.0 else None
            if rms:
                eng.fedavg_rmsprop([segs[j] for j in idx], w, [gparams[j] for j in idx],
                                   [self.square_avg[named[j][0]] for j in idx], mbufs, self.lr,
                                   weight_decay=self.weight_decay, momentum=self.momentum, first_step=flag)
            else:
                eng.fedavg_sgd([segs[j] for j in idx], w, [gparams[j] for j in idx], mbufs,
                               self.lr, self.momentum, self.dampening, self.weight_decay, self.nesterov,
                               first_step=flag)
        if not on_gpu:
            with torch.no_grad():
                for (_, p), g in zip(named, gparams):
                    p.data.copy_(g.cpu())
        # buffers (and frozen parameters, which the reference leaves at their old value)
        sd = model.state_dict()
        rest = [k for k in dicts[0].keys() if k not in all_params]
        if rest:
            avg = aggregate([{k: d[k] for k in rest} for d in dicts], MUL_W, w)
            with torch.no_grad():
                for k in rest:
                    sd[k].copy_(avg[k])  # load_state_dict semantics: cast into the buffer dtype
        logging.info("aggregate time cost: %.6f s", time.time() - t0)
        return self.get_global_model_params()
