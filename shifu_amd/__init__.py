"""shifu_amd - an MI355X-native tabular ML pipeline with the capabilities of Shifu.

Layers: cli (L7) -> steps (L6 processors) -> models/formats (L5) ->
algos + ops HIP kernels (L4) -> parallel runtime over RCCL/xGMI (L3) -> config (L2) ->
data IO (L1).
"""
__version__ = "0.1.0"
