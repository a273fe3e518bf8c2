"""decds_amd — MI355X-native (gfx950) RLNC chunkset codec behind decds-lib's chunkset API.

The hot path (RLNC 10->16 encode and >=10->10 repair of 10 MiB chunksets, decds-lib
chunkset.rs / blob.rs) runs in hand-written HIP kernels in libdecds_rlnc.so, reached through the
C-ABI in include/decds_rlnc.h. This package is the Python-side binding used by tests and bench.py.
"""
from ._capi import (CHUNKSET_BYTES, CODED_PIECE_BYTES, K, N, NO_CANDIDATE, PIECE_BYTES, REPAIR_PLAN_BYTES,
                    STATUS, STATUS_NAMES, DecdsError)
from .blob import Blob, HostBuffer, RepairingBlob
from .chunkset import Chunk, ChunkSet, Context, RepairingChunkSet
from .wire import BlobHeader

__all__ = ["Context", "Chunk", "ChunkSet", "RepairingChunkSet", "Blob", "RepairingBlob", "BlobHeader", "HostBuffer",
           "DecdsError", "K", "N", "CHUNKSET_BYTES", "PIECE_BYTES", "CODED_PIECE_BYTES", "REPAIR_PLAN_BYTES",
           "NO_CANDIDATE", "STATUS", "STATUS_NAMES"]
