"""gsgpu — MI355X-native streaming Connected Components for Gelly Streaming.

Python mirror of the reference's operator surface over libgsgpu.so (C ABI: include/gsgpu.h).
"""
from ._abi import GsError, GsgpuUnavailable, available, lib, EXPORTED_SYMBOLS  # noqa: F401
from .summary import DisjointSet, UpdateCC, CombineCC, combine_cc  # noqa: F401
from .aggregation import (SimpleEdgeStream, SummaryBulkAggregation, ConnectedComponents,  # noqa: F401
                          SummaryTreeReduce, ConnectedComponentsTree)
from .bipartite import Candidates, BipartitenessCheck  # noqa: F401
from .comm import Comm  # noqa: F401

__all__ = ["DisjointSet", "UpdateCC", "CombineCC", "combine_cc", "SimpleEdgeStream",
           "SummaryBulkAggregation", "ConnectedComponents", "SummaryTreeReduce", "ConnectedComponentsTree",
           "Candidates", "BipartitenessCheck", "GsError", "GsgpuUnavailable",
           "available", "lib"]
