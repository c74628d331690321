"""realtime-st-gcn_amd — MI355X-native (gfx950 HIP) ST-GCN hot path behind the reference's nn.Module API.

Loaded by path (the directory name has dashes): see ``__graft_entry__.load_package()``.
Public surface mirrors maximyudayev/Realtime-ST-GCN: ``MODELS`` (models/__init__.py:11-20),
``Graph``, ``StgcnLayer``, ``ConvTemporalGraphical``, ``LayerNorm``, ``BatchNorm1d``.
"""
from . import _lib, data, loss, metrics, native, optim, parallel, routing, segment, syncbn  # noqa: F401
from .syncbn import convert_sync_batchnorm, revert_sync_batchnorm  # noqa: F401
from .graph import Graph, PKU_MMD  # noqa: F401
from .modules import BatchNorm1d, ConvTemporalGraphical, LayerNorm, StgcnLayer, set_compute_dtype  # noqa: F401
from .stgcn import Model as Stgcn  # noqa: F401

MODELS = {
    "st-gcn": Stgcn,
}

try:  # optional families, registered when present
    from .rtstgcn import Model as RtStgcn  # noqa: F401
    MODELS["rt-st-gcn"] = RtStgcn
except ImportError:  # pragma: no cover
    pass
try:
    from .aagcn import Model as AaGcn  # noqa: F401
    MODELS["aa-gcn"] = AaGcn
except ImportError:  # pragma: no cover
    pass
