"""HIP-graph capture with Python's cyclic garbage collector held off.

A collection that runs while a stream is capturing can free an unreachable
``torch.cuda.CUDAGraph`` (e.g. one held by a collector or policy that is no longer referenced);
its destructor then calls a HIP API that a capturing stream forbids
(``hipErrorStreamCaptureUnsupported``) and the process aborts.  Every capture in this package
goes through :func:`graph_capture`: dead cycles are collected first, then the collector is
disabled until the capture ends."""
import contextlib
import gc

import torch


@contextlib.contextmanager
def graph_capture(graph: "torch.cuda.CUDAGraph"):
    gc.collect()
    was_enabled = gc.isenabled()
    gc.disable()
    try:
        with torch.cuda.graph(graph):
            yield
    finally:
        if was_enabled:
            gc.enable()
