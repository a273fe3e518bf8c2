"""ctypes binding of libdecds_rlnc.so (include/decds_rlnc.h).

This is the same binding a Rust maintainer writes as an `extern "C"` block.
Loading fails loudly when the library is missing: there is no pure-Python or CPU fallback for the
codec; every compute call runs the gfx950 kernels.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libdecds_rlnc.so")
# tuning runs load an alternative build of the same sources (tools/kbench.py); default: in-tree lib
LIB_PATH = os.environ.get("DECDS_LIB", LIB_PATH)

K = 10                  # ChunkSet::NUM_ORIGINAL_CHUNKS (chunkset.rs:19)
N = 16                  # ChunkSet::NUM_ERASURE_CODED_CHUNKS (chunkset.rs:21)
CHUNKSET_BYTES = 10 * (1 << 20)                     # ChunkSet::BYTE_LENGTH (chunkset.rs:20)
PIECE_BYTES = (CHUNKSET_BYTES + 1 + K - 1) // K     # PADDED_CHUNK_BYTE_LEN (chunkset.rs:117)
CODED_PIECE_BYTES = PIECE_BYTES + K                 # coding vector || payload
REPAIR_PLAN_BYTES = 128
CODED_PITCH_ALIGNED = 1048704       # recommended device layout (include/decds_rlnc.h): 128-B-aligned payloads
CODED_ROW_OFFSET_ALIGNED = 118
NO_CANDIDATE = 0xFF

# status codes, 1:1 with decds-lib/src/errors.rs (see include/decds_rlnc.h)
OK = 0
STATUS_NAMES = {
    0: "Ok",
    1: "InvalidChunksetSize",
    2: "InvalidChunkMetadata",
    3: "ChunksetReadyToRepair",
    4: "ChunkDecodingFailed",
    5: "ChunksetNotYetReadyToRepair",
    6: "ChunksetRepairingFailed",
    7: "InvalidErasureCodedShareId",
    8: "EmptyDataForBlob",
    9: "InvalidChunksetId",
    10: "ChunksetAlreadyRepaired",
    11: "InvalidProofInChunk",
    12: "BlobHeaderSerializationFailed",
    13: "BlobHeaderDeserializationFailed",
    14: "ProofCarryingChunkSerializationFailed",
    15: "ProofCarryingChunkDeserializationFailed",
    16: "InvalidStartBound",
    17: "InvalidEndBound",
    -1: "HipError",
    -2: "InvalidArgument",
    -3: "NoDevice",
    -4: "OutOfDeviceMemory",
}
STATUS = {v: k for k, v in STATUS_NAMES.items()}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                "decds_amd: %s is missing — build it with `python -m decds_amd.build` "
                "(hipcc --offload-arch=gfx950); there is no fallback implementation" % LIB_PATH)
        try:
            # torch ships its own libamdhip64: load it first so the library binds to the same HIP
            # runtime instead of a second copy from /opt/rocm (two runtimes in one process break
            # torch's device init and pointer sharing)
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        _declare(L)
        _lib = L
    return _lib


def _declare(L):
    c = ctypes
    P, U8P, I8P, I32P, SZ, VP = c.c_void_p, c.POINTER(c.c_uint8), c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p
    sig = {
        "decds_ctx_create": (c.c_int, [c.c_int, c.POINTER(c.c_void_p)]),
        "decds_ctx_destroy": (c.c_int, [P]),
        "decds_ctx_set_field": (c.c_int, [P, c.c_uint32, c.c_uint8]),
        "decds_ctx_get_field": (c.c_int, [P, c.POINTER(c.c_uint32), c.POINTER(c.c_uint8)]),
        "decds_status_string": (c.c_char_p, [c.c_int]),
        "decds_last_error": (c.c_char_p, []),
        "decds_device_count": (c.c_int, []),
        "decds_encode_batch": (c.c_int, [P, VP, SZ, VP, VP, SZ, VP]),
        "decds_repair_plan_batch": (c.c_int, [P, VP, SZ, SZ, VP, VP, I8P, I32P, VP]),
        "decds_decode_batch": (c.c_int, [P, VP, SZ, SZ, VP, VP, I32P, VP, VP]),
        "decds_repair_batch": (c.c_int, [P, VP, SZ, SZ, VP, VP, I8P, VP, I32P, VP, VP]),
        "decds_fill_random_device": (c.c_int, [P, c.c_uint64, c.c_uint64, VP, SZ, VP]),
        "decds_fill_random_host": (None, [c.c_uint64, c.c_uint64, VP, SZ]),
        "decds_rank_push": (c.c_int, [VP, VP, c.POINTER(c.c_uint32), VP, c.c_uint32]),
        "decds_chunkset_new": (c.c_int, [P, SZ, VP, SZ, VP, c.POINTER(c.c_void_p)]),
        "decds_chunkset_get_chunk": (c.c_int, [P, SZ, VP, SZ, c.POINTER(SZ)]),
        "decds_chunkset_id": (SZ, [P]),
        "decds_chunkset_free": (None, [P]),
        "decds_chunkset_get_root_commitment": (c.c_int, [P, VP]),
        "decds_chunkset_get_chunk_proof": (c.c_int, [P, SZ, VP, SZ, c.POINTER(SZ)]),
        "decds_chunkset_append_blob_inclusion_proof": (c.c_int, [P, VP, SZ]),
        "decds_repairing_chunkset_new": (c.c_int, [P, SZ, VP, c.POINTER(c.c_void_p)]),
        "decds_repairing_chunkset_add_chunk": (c.c_int, [P, SZ, SZ, VP, SZ, VP, SZ]),
        "decds_repairing_chunkset_add_chunk_unvalidated": (c.c_int, [P, SZ, VP, SZ]),
        "decds_repairing_chunkset_is_ready_to_repair": (c.c_int, [P]),
        "decds_repairing_chunkset_repair": (c.c_int, [P, VP, SZ, c.POINTER(SZ)]),
        "decds_repairing_chunkset_free": (None, [P]),
        "decds_blob_encode_host": (c.c_int, [P, VP, SZ, VP, VP, SZ]),
        "decds_blob_repair_host": (c.c_int, [P, VP, SZ, VP, SZ, VP, VP, SZ]),
        "decds_host_register": (c.c_int, [VP, SZ]),
        "decds_commit_batch": (c.c_int, [P, VP, SZ, SZ, c.c_uint64, VP, VP, VP, VP]),
        "decds_blake3": (None, [VP, SZ, VP]),
        "decds_chunk_digest": (None, [c.c_uint64, c.c_uint64, VP, SZ, VP]),
        "decds_validate_batch": (c.c_int, [P, VP, SZ, SZ, VP, VP, SZ, VP, SZ, VP, VP, VP, VP]),
        "decds_blake3_parallel": (None, [VP, SZ, VP, c.c_int]),
        "decds_pcc_encoded_len": (SZ, [c.c_uint64, c.c_uint64, SZ, SZ]),
        "decds_pcc_to_bytes": (c.c_int, [c.c_uint64, c.c_uint64, VP, SZ, VP, SZ, VP, SZ, c.POINTER(SZ)]),
        "decds_pcc_from_bytes": (c.c_int, [VP, SZ, c.POINTER(c.c_uint64), c.POINTER(c.c_uint64),
                                           c.POINTER(c.c_void_p), c.POINTER(SZ), c.POINTER(c.c_void_p),
                                           c.POINTER(SZ), c.POINTER(SZ)]),
        "decds_blob_header_encoded_len": (SZ, [c.c_uint64, c.c_uint64, SZ]),
        "decds_blob_header_to_bytes": (c.c_int, [c.c_uint64, c.c_uint64, VP, VP, VP, SZ, VP, SZ, c.POINTER(SZ)]),
        "decds_blob_header_from_bytes": (c.c_int, [VP, SZ, c.POINTER(c.c_uint64), c.POINTER(c.c_uint64), VP, VP,
                                                   c.POINTER(c.c_void_p), c.POINTER(SZ), c.POINTER(SZ)]),
        "decds_merkle_tree": (c.c_int, [VP, SZ, VP, VP]),
        "decds_merkle_verify": (c.c_int, [SZ, VP, VP, SZ, VP]),
        "decds_host_unregister": (c.c_int, [VP]),
        "decds_host_alloc": (c.c_int, [SZ, c.POINTER(c.c_void_p)]),
        "decds_host_free": (c.c_int, [VP]),
        "decds_host_cache_trim": (SZ, []),
        "decds_blake3_stream_new": (c.c_void_p, []),
        "decds_blake3_stream_update": (None, [VP, VP, SZ, c.c_int]),
        "decds_blake3_stream_finalize": (None, [VP, VP]),
        "decds_blake3_stream_free": (None, [VP]),
        "decds_host_is_registered": (c.c_int, [VP, SZ]),
        "decds_device_status": (c.c_int, [P]),
        "decds_blob_encode_host_multi": (c.c_int, [VP, SZ, VP, SZ, VP, VP, SZ]),
        "decds_blob_repair_host_multi": (c.c_int, [VP, SZ, VP, SZ, VP, SZ, VP, VP, SZ]),
        "decds_blob_new": (c.c_int, [VP, SZ, VP, SZ, VP, c.POINTER(c.c_void_p)]),
        "decds_blob_get_header": (c.c_int, [P, c.POINTER(c.c_uint64), c.POINTER(c.c_uint64), VP, VP,
                                            c.POINTER(c.c_void_p)]),
        "decds_blob_proof_len": (SZ, [P]),
        "decds_blob_get_chunk": (c.c_int, [P, SZ, SZ, c.POINTER(c.c_void_p), VP, SZ]),
        "decds_blob_get_share": (c.c_int, [P, SZ, VP, SZ, VP, SZ]),
        "decds_blob_free": (None, [P]),
        "decds_repairing_blob_new": (c.c_int, [P, c.c_uint64, c.c_uint64, VP, VP, c.POINTER(c.c_void_p)]),
        "decds_repairing_blob_new_multi": (c.c_int, [VP, SZ, c.c_uint64, c.c_uint64, VP, VP, c.POINTER(c.c_void_p)]),
        "decds_repairing_blob_set_device_budget": (c.c_int, [P, c.c_uint64]),
        "decds_repairing_blob_memory": (c.c_int, [P, c.POINTER(c.c_uint64), SZ]),
        "decds_repairing_blob_add_chunk": (c.c_int, [P, c.c_uint64, c.c_uint64, VP, SZ, VP, SZ]),
        "decds_repairing_blob_add_chunks": (c.c_int, [P, SZ, VP, VP, VP, SZ, VP]),
        "decds_repairing_blob_is_chunkset_ready_to_repair": (c.c_int, [P, SZ, c.POINTER(c.c_int)]),
        "decds_repairing_blob_is_chunkset_already_repaired": (c.c_int, [P, SZ, c.POINTER(c.c_int)]),
        "decds_repairing_blob_get_repaired_chunkset": (c.c_int, [P, SZ, VP, SZ, c.POINTER(SZ)]),
        "decds_repairing_blob_free": (None, [P]),
        "decds_encode_commit_workspace_bytes": (SZ, [SZ]),
        "decds_encode_kernel_name": (c.c_char_p, [SZ]),
        "decds_decode_kernel_name": (c.c_char_p, [SZ]),
        "decds_repair_kernel_name": (c.c_char_p, [SZ]),
        "decds_tuning": (c.c_uint64, [c.c_char_p, c.c_uint64, c.c_int]),
        "decds_encode_commit_batch": (c.c_int, [P, VP, SZ, VP, VP, SZ, c.c_uint64, VP, VP, VP, VP, VP]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args


EXPORTED = [
    "decds_ctx_create", "decds_ctx_destroy", "decds_ctx_set_field", "decds_ctx_get_field",
    "decds_status_string", "decds_last_error", "decds_device_count", "decds_encode_batch",
    "decds_repair_plan_batch", "decds_decode_batch", "decds_repair_batch",
    "decds_fill_random_device", "decds_fill_random_host", "decds_rank_push", "decds_chunkset_new",
    "decds_chunkset_get_chunk", "decds_chunkset_id", "decds_chunkset_free",
    "decds_repairing_chunkset_new", "decds_repairing_chunkset_add_chunk_unvalidated",
    "decds_repairing_chunkset_is_ready_to_repair", "decds_repairing_chunkset_repair",
    "decds_repairing_chunkset_free", "decds_blob_encode_host", "decds_blob_repair_host",
    "decds_host_register", "decds_host_unregister", "decds_commit_batch", "decds_blake3",
    "decds_merkle_tree", "decds_merkle_verify", "decds_chunk_digest", "decds_validate_batch",
    "decds_chunkset_get_root_commitment", "decds_chunkset_get_chunk_proof",
    "decds_chunkset_append_blob_inclusion_proof", "decds_repairing_chunkset_add_chunk",
    "decds_blake3_parallel", "decds_pcc_encoded_len", "decds_pcc_to_bytes", "decds_pcc_from_bytes",
    "decds_blob_header_encoded_len", "decds_blob_header_to_bytes", "decds_blob_header_from_bytes",
    "decds_host_alloc", "decds_host_free", "decds_host_is_registered", "decds_device_status",
    "decds_blob_encode_host_multi", "decds_blob_repair_host_multi", "decds_blob_new", "decds_blob_get_header",
    "decds_blob_proof_len", "decds_blob_get_chunk", "decds_blob_get_share", "decds_blob_free",
    "decds_repairing_blob_new", "decds_repairing_blob_add_chunk", "decds_repairing_blob_add_chunks",
    "decds_repairing_blob_is_chunkset_ready_to_repair", "decds_repairing_blob_is_chunkset_already_repaired",
    "decds_repairing_blob_get_repaired_chunkset", "decds_repairing_blob_free", "decds_repairing_blob_new_multi",
    "decds_repairing_blob_set_device_budget", "decds_repairing_blob_memory",
    "decds_encode_commit_workspace_bytes", "decds_encode_commit_batch", "decds_encode_kernel_name",
    "decds_decode_kernel_name", "decds_repair_kernel_name", "decds_host_cache_trim", "decds_blake3_stream_new", "decds_blake3_stream_update",
    "decds_blake3_stream_finalize", "decds_blake3_stream_free", "decds_tuning",
]


class DecdsError(Exception):
    """Mirror of decds-lib's DecdsError (errors.rs:3-48): `kind` is the variant name."""

    def __init__(self, status, message=""):
        self.status = status
        self.kind = STATUS_NAMES.get(status, "Unknown(%d)" % status)
        super().__init__("%s: %s" % (self.kind, message))

    def __eq__(self, other):
        return isinstance(other, DecdsError) and other.status == self.status

    __hash__ = Exception.__hash__


def check(status):
    if status != OK:
        raise DecdsError(status, lib().decds_last_error().decode(errors="replace"))
    return status
