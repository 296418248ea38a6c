"""MI355X-native GraphSAGE sample-and-aggregate path (drop-in for the
reference's src/models.py GraphSage / SageLayer / Classification)."""
from . import _lib  # noqa: F401
from .graph import CSRGraph, rmat_pairs  # noqa: F401
from .sampler import RNG, DeviceSampler, Sample, pyset_union_of_lists, sample  # noqa: F401

__version__ = "0.1.0"
