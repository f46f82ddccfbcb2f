"""DefaultServerAggregator (reference: python/fedml/ml/aggregator/default_aggregator.py:12-106) and
create_server_aggregator (aggregator_creator.py:6-13).

get/set of the global model are state_dict moves; ``aggregate`` is inherited from
ServerAggregator and runs on the MI355X engine.  ``test`` evaluates accuracy / loss of the global
model (classification: cross-entropy; stackoverflow_lr: multi-label BCE), returning the
reference's ``(test_acc, test_loss, None, None)`` tuple; the reference's wandb/mlops logging is
not part of this engine.
"""
from __future__ import annotations

import logging

import torch
from torch import nn

from ...core.alg_frame.server_aggregator import ServerAggregator


class DefaultServerAggregator(ServerAggregator):
    def __init__(self, model, args):
        super().__init__(model, args)
        self.cpu_transfer = bool(getattr(self.args, "cpu_transfer", False))

    def get_model_params(self):
        if self.cpu_transfer:
            return self.model.cpu().state_dict()
        return self.model.state_dict()

    def set_model_params(self, model_parameters):
        self.model.load_state_dict(model_parameters)

    def _test(self, test_data, device, args):
        model = self.model.to(device)
        model.eval()
        multilabel = getattr(args, "dataset", None) == "stackoverflow_lr"
        criterion = (nn.BCELoss(reduction="sum") if multilabel else nn.CrossEntropyLoss()).to(device)
        correct = total = 0
        loss_sum = 0.0
        with torch.no_grad():
            for x, target in test_data:
                x, target = x.to(device), target.to(device)
                pred = model(x)
                loss = criterion(pred, target)
                if multilabel:
                    hit = (pred > 0.5).int().eq(target).sum(axis=-1).eq(target.size(1)).sum()
                else:
                    hit = pred.argmax(1).eq(target).sum()
                correct += int(hit.item())
                loss_sum += float(loss.item()) * target.size(0)
                total += target.numel() if target.dim() == 2 and not multilabel else target.size(0)
        return {"test_correct": correct, "test_loss": loss_sum, "test_total": total}

    def test(self, test_data, device, args):
        m = self._test(test_data, device, args)
        acc = m["test_correct"] / max(1, m["test_total"])
        loss = m["test_loss"] / max(1, m["test_total"])
        logging.info({"test_acc": acc, "test_loss": loss})
        return acc, loss, None, None


def create_server_aggregator(model, args):
    """Reference aggregator_creator.py:6-13 (dataset-specific subclasses share the default path)."""
    return DefaultServerAggregator(model, args)
