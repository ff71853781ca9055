"""neural_amd -- MI355X-native weight-only-quantized matmul core with Neural Speed's BesTLA operator surface.

The product is libneural_amd.so (C-ABI: include/neural_amd.h).  This package is its Python host mirror:
  neural_amd.bestla            quantize / qpack / unpack / split, DeviceWeight (load + forward), fused QKV / FFN
  neural_amd.parallel_context  tensor-parallel communicator (RCCL over xGMI through torch.distributed)
  neural_amd.tp                TP weight sharding rules (model_split_type) and row/column-parallel linears
"""
from ._lib import LIB_PATH, NativeLibraryMissing, lib  # noqa: F401

__all__ = ["LIB_PATH", "NativeLibraryMissing", "lib"]
