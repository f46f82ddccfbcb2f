"""fedml_amd -- MI355X-native server-side aggregation engine for FedML-style federated learning.

Drop-in for the FedAvg-family aggregation path of liuliuliu0605/FedML (python/fedml): the same
operator / plugin surface (``FedMLAggOperator.agg``, ``ServerAggregator``), bit-identical results,
arithmetic in hand-written HIP kernels for gfx950 (``fedml_amd/csrc/fedagg.hip``) behind a C ABI
(``include/fedagg.h``).
"""
__version__ = "0.1.0"
