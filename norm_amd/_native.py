"""ctypes binding of libnfec.so (include/nfec.h).

The library is built in-tree (norm_amd/_lib/libnfec.so, see norm_amd/Makefile and
__graft_entry__.build()).  There is no fallback: if the library is missing or a call
fails, an exception is raised.
"""
import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# NFEC_LIBRARY selects another build of the same ABI: the diagnostic library with the A/B
# variants and probes of the kernels (make -C norm_amd diag -> _lib/libnfec_diag.so)
PRODUCT_LIB_PATH = os.path.join(_HERE, "_lib", "libnfec.so")
LIB_PATH = os.environ.get("NFEC_LIBRARY") or PRODUCT_LIB_PATH
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "nfec.h")

NFEC_RS8, NFEC_RS16, NFEC_MDP = 1, 2, 3
NFEC_OK, NFEC_EINVAL, NFEC_ENOMEM, NFEC_EDEVICE, NFEC_ERANGE, NFEC_ENOTSUP = 0, -1, -2, -3, -4, -5
NFEC_ACCUMULATE = 1
NFEC_FEATURE_RS16_TOEPLITZ, NFEC_FEATURE_RS16_TOEPLITZ2 = 1, 2
NFEC_OPT_RS16_SHARED_TABLES, NFEC_OPT_RS16_TOEPLITZ_OFF, NFEC_OPT_RS16_TOEPLITZ_ON, NFEC_OPT_HOST_ONLY = 1, 2, 4, 8
NFEC_OPT_RS16_TOEPLITZ_ONE_LEVEL = 16
# encode paths (nfec_codec_encode_paths)
NFEC_PATH_FIXED, NFEC_PATH_RUNTIME, NFEC_PATH_RS16_SPLIT, NFEC_PATH_RS16_PRODUCT, NFEC_PATH_GENERIC = 0, 1, 2, 3, 4
NFEC_PATH_COUNT = 5
PATH_NAMES = ("fixed", "runtime", "rs16_split", "rs16_product", "generic")
NFEC_DPATH_COUNT = 4
DPATH_NAMES = ("fixed", "runtime", "rs16_tower", "generic")
NFEC_HOST_GF_SCALAR, NFEC_HOST_GF_AVX2, NFEC_HOST_GF_GFNI = 0, 1, 2


class NfecError(RuntimeError):
    def __init__(self, code, what):
        super().__init__(f"{what} failed with {code}: {last_error()}")
        self.code = code


class BlockBatch(ctypes.Structure):
    _fields_ = [
        ("blocks", ctypes.c_void_p),
        ("block_stride", ctypes.c_uint64),
        ("seg_stride", ctypes.c_uint32),
        ("nblocks", ctypes.c_uint32),
        ("num_data", ctypes.c_void_p),
        ("flags", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
    ]


class CodecInfo(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("num_data", ctypes.c_uint32),
        ("num_parity", ctypes.c_uint32),
        ("vector_size", ctypes.c_uint32),
        ("symbol_bytes", ctypes.c_uint32),
    ]


class CodecConfig(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("num_data", ctypes.c_uint32),
        ("num_parity", ctypes.c_uint32),
        ("vector_size", ctypes.c_uint32),
        ("devices", ctypes.POINTER(ctypes.c_int32)),
        ("num_devices", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
    ]


class Fti(ctypes.Structure):
    _fields_ = [
        ("fec_id", ctypes.c_uint8),
        ("fec_m", ctypes.c_uint8),
        ("fec_group_size", ctypes.c_uint8),
        ("reserved", ctypes.c_uint8),
        ("instance_id", ctypes.c_uint16),
        ("segment_size", ctypes.c_uint16),
        ("num_data", ctypes.c_uint16),
        ("num_parity", ctypes.c_uint16),
        ("object_size", ctypes.c_uint64),
    ]


class NpcParams(ctypes.Structure):
    _fields_ = [
        ("segment_size", ctypes.c_uint32),
        ("num_data", ctypes.c_uint32),
        ("num_parity", ctypes.c_uint32),
        ("parity_fraction", ctypes.c_double),
        ("b_max", ctypes.c_uint64),
        ("i_max", ctypes.c_uint64),
    ]


class NpcLayout(ctypes.Structure):
    _fields_ = [
        ("num_segments", ctypes.c_uint64),
        ("input_segments", ctypes.c_uint64),
        ("num_blocks", ctypes.c_uint64),
        ("num_data", ctypes.c_uint32),
        ("num_parity", ctypes.c_uint32),
        ("last_block_data", ctypes.c_uint32),
        ("segment_size", ctypes.c_uint32),
        ("last_segment_bytes", ctypes.c_uint32),
        ("kind", ctypes.c_int32),
        ("il_width", ctypes.c_uint64),
        ("il_height", ctypes.c_uint64),
        ("il_size", ctypes.c_uint64),
        ("i_max", ctypes.c_uint64),
    ]


_P = ctypes.c_void_p
_U8 = ctypes.c_uint8
_U16 = ctypes.c_uint16
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_I = ctypes.c_int
_SIGS = {
    "nfec_abi_version": (_I, []),
    "nfec_build_id": (ctypes.c_char_p, []),
    "nfec_device_count": (_I, []),
    "nfec_last_error": (ctypes.c_char_p, []),
    "nfec_build_generator": (_I, [_I, _U32, _U32, _P, ctypes.c_size_t]),
    "nfec_codec_create": (_I, [_I, _I, _U32, _U32, _U32, ctypes.POINTER(_P)]),
    "nfec_codec_create_ex": (_I, [ctypes.POINTER(CodecConfig), ctypes.POINTER(_P)]),
    "nfec_codec_num_devices": (_I, [_P, ctypes.POINTER(ctypes.c_int32), _U32]),
    "nfec_codec_destroy": (None, [_P]),
    "nfec_codec_get_info": (_I, [_P, ctypes.POINTER(CodecInfo)]),
    "nfec_codec_features": (_I, [_P]),
    "nfec_codec_encode_paths": (_I, [_P, ctypes.POINTER(_U64), _U32]),
    "nfec_codec_decode_paths": (_I, [_P, ctypes.POINTER(_U64), _U32]),
    "nfec_codec_get_generator": (_I, [_P, _P, ctypes.c_size_t]),
    "nfec_encode": (_I, [_P, ctypes.POINTER(BlockBatch), _P]),
    "nfec_decode": (_I, [_P, ctypes.POINTER(BlockBatch), _P, _U32, _P, _P, _P]),
    "nfec_encode_host": (_I, [_P, ctypes.POINTER(BlockBatch)]),
    "nfec_decode_host": (_I, [_P, ctypes.POINTER(BlockBatch), _P, _U32, _P, _P]),
    "nfec_encode_host_vectors": (_I, [_P, _P, _U32, _P, _U32]),
    "nfec_decode_host_vectors": (_I, [_P, _P, _U32, _P, _P, _U32, _P, _P, _U32]),
    "nfec_encode_host_vectors_async": (_I, [_P, _P, _U32, _P, _U32, _P]),
    "nfec_decode_host_vectors_async": (_I, [_P, _P, _U32, _P, _P, _U32, _P, _P, _U32, _P]),
    "nfec_request_test": (_I, [_P]),
    "nfec_request_wait": (_I, [_P]),
    "nfec_encode_segment": (_I, [_P, _U32, _P, _P]),
    "nfec_encode_segment_host": (_I, [_P, _U32, _P, _P]),
    "nfec_gf8_addmul_host": (_I, [_P, _P, _U8, ctypes.c_size_t, _I]),
    "nfec_gf16_addmul_host": (_I, [_P, _P, ctypes.c_uint16, ctypes.c_size_t, _I]),
    "nfec_gf_dot_host": (_I, [_I, _P, _P, _P, ctypes.c_uint32, ctypes.c_size_t, _I, _I]),
    "nfec_decode_vectors_host": (_I, [_P, _P, _U32, _U32, _P]),
    "nfec_decode_host_preferred": (_I, [_P, _U32, _U32]),
    "nfec_decode_vectors": (_I, [_P, _P, _U32, _U32, _P]),
    "nfec_dropin_sizeof": (ctypes.c_size_t, [_I, _I]),
    "nfec_util_fill": (_I, [ctypes.POINTER(BlockBatch), _U32, _U32, _U64, _U64, _P]),
    "nfec_util_erasures": (_I, [_P, _U32, _P, _U32, _U32, _U32, _U64, _U64, _P]),
    "nfec_util_zero_slots": (_I, [ctypes.POINTER(BlockBatch), _P, _U32, _P, _U32, _P]),
    "nfec_util_stream_copy": (_I, [_P, _P, _U64, _P]),
    "nfec_host_threads": (_I, [ctypes.POINTER(_U32), ctypes.POINTER(_U32), ctypes.POINTER(_U32)]),
    "nfec_util_pool_check": (_I, [_U32, _I]),
    "nfec_util_gather_probe": (_I, [_P, _U32, _U32, _U32, _U32, _U32, ctypes.POINTER(ctypes.c_double),
                                    ctypes.POINTER(_U32)]),
    "nfec_fti_write": (_I, [ctypes.POINTER(Fti), _P, ctypes.c_size_t]),
    "nfec_fti_read": (_I, [_U8, _P, ctypes.c_size_t, ctypes.POINTER(Fti)]),
    "nfec_payload_id_length": (_I, [_U8]),
    "nfec_payload_id_write": (_I, [_U8, _U8, _U32, _U16, _U16, _P]),
    "nfec_payload_id_read": (_I, [_U8, _U8, _P, ctypes.POINTER(_U32), ctypes.POINTER(_U16), ctypes.POINTER(_U16)]),
    "nfec_sender_codec": (_I, [_U16, _U16, _U8, _I, ctypes.POINTER(_I), ctypes.POINTER(_U8), ctypes.POINTER(_U8)]),
    "nfec_receiver_codec": (_I, [_U8, _U8, _U16, _I, ctypes.POINTER(_I)]),
    "nfec_vector_size": (_U32, [_U16]),
    "nfec_npc_default_params": (None, [ctypes.POINTER(NpcParams)]),
    "nfec_npc_layout_for": (_I, [ctypes.POINTER(NpcParams), _U64, _I, ctypes.POINTER(NpcLayout)]),
    "nfec_npc_positions": (_I, [ctypes.POINTER(NpcLayout), _U64, _U64, _P]),
    "nfec_npc_encode_file": (_I, [_I, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(NpcParams)]),
    "nfec_npc_decode_file": (_I, [_I, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(NpcParams),
                                  ctypes.POINTER(_U64), ctypes.c_char_p, ctypes.c_size_t]),
    "nfec_npc_encode_file_multi": (_I, [_P, _I, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(NpcParams)]),
    "nfec_npc_decode_file_multi": (_I, [_P, _I, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(NpcParams),
                                        ctypes.POINTER(_U64), ctypes.c_char_p, ctypes.c_size_t]),
    "nfec_crc32_slots": (_I, [ctypes.POINTER(BlockBatch), _U32, _U32, _P, _P]),
}

_lib = None


def lib():
    """Load libnfec.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libnfec.so not built ({LIB_PATH}); run __graft_entry__.build() or make -C norm_amd")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def last_error():
    if _lib is None:
        return ""
    msg = _lib.nfec_last_error()
    return msg.decode() if msg else ""


def check(rc, what):
    if rc < 0:
        raise NfecError(rc, what)
    return rc


def source_build_id(root=None):
    """SHA-256 of the library's sources in this tree, computed as norm_amd/Makefile computes
    nfec_build_id(): csrc/*.{cpp,hip,hpp,h} then include/*.h and include/norm_fec/*.h, each sorted by path."""
    import glob
    import hashlib

    root = root or os.path.dirname(_HERE)
    csrc = sorted(p for ext in ("cpp", "hip", "hpp", "h")
                  for p in glob.glob(os.path.join(root, "norm_amd", "csrc", "*." + ext)))
    inc = sorted(glob.glob(os.path.join(root, "include", "*.h")) + glob.glob(os.path.join(root, "include", "norm_fec", "*.h")))
    h = hashlib.sha256()
    for path in csrc + inc:
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def declared_symbols():
    """Function names declared in include/nfec.h (used by the ABI export test)."""
    text = open(HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nfec_[a-z0-9_]+)\s*\(", text)))
