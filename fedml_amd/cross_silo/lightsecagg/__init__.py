from .lsa_fedml_aggregator import LightSecAggAggregator

__all__ = ["LightSecAggAggregator"]
