"""spwgnn_amd — MI355X-native (gfx950) engine for the SPWGNN tower-stability propagation network.

Hot path (src/Networks.py + src/Blocks.py of irmakguzey/SPWGNN) as hand-written HIP kernels in
libspwgnn_hip.so behind a C ABI (include/spwgnn.h); this package is the host-side mirror of the
reference's interface (PropagationNetwork.getModel → fit / predict).
"""
from .batch import TowerBatch
from .engine import RunConfig
from .network import GraphNetwork
from .keras_api import PropagationNetwork, KerasModel

__all__ = ["TowerBatch", "RunConfig", "GraphNetwork", "PropagationNetwork", "KerasModel"]
