from .sa_fedml_aggregator import SecAggAggregator

__all__ = ["SecAggAggregator"]
