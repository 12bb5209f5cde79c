"""Model registry -- drop-in for the reference's ``model/__init__.py:11-14``.

``get_model(model_type, **model_opts)`` looks ``model_type`` up and calls the
class with ``model_opts[model_type]`` (the yaml ``model.dstdgcn`` section);
unknown names raise KeyError exactly like the reference's dict lookup.
"""
from .dstdgcn import DSTDGC, DSTDGCB, DSTDGCN, BatchNorm, Conv2d, ConvTemporalGraphical, ST_GCNN_layer  # noqa: F401

_REGISTRY = {"dstdgcn": DSTDGCN}


def get_model(model_type, **model_opts):
    return _REGISTRY[model_type](**model_opts[model_type])
