"""NORM wire-format pieces on the FEC path, over the C ABI (include/nfec.h, csrc/wire.cpp).

The FEC Object Transmission Information extension (normMessage.h:785-1029) carries what a
receiver needs to build its decoder; the FEC payload ID (normMessage.h:396-567) names the
block and symbol of every NORM_DATA.  make_encoder()/make_decoder() apply the sender and
receiver codec choices (normSession.cpp:764-883, normNode.cpp:290-356), returning an
Init()ed drop-in codec with vector size = segment size + the 8-byte stream payload header.
"""
import ctypes
from dataclasses import dataclass

from . import _native as N


@dataclass
class FecObjectInfo:
    fec_id: int
    segment_size: int
    num_data: int
    num_parity: int
    object_size: int = 0
    fec_m: int = 8
    fec_group_size: int = 1
    instance_id: int = 0

    def _c(self):
        return N.Fti(self.fec_id, self.fec_m, self.fec_group_size, 0, self.instance_id, self.segment_size,
                     self.num_data, self.num_parity, self.object_size)


def write_fti(info: FecObjectInfo) -> bytes:
    """The FTI header extension bytes (16; 12 for fec_id 5)."""
    buf = (ctypes.c_uint8 * 16)()
    n = N.check(N.lib().nfec_fti_write(ctypes.byref(info._c()), buf, 16), "nfec_fti_write")
    return bytes(buf[:n])


def read_fti(fec_id: int, ext: bytes) -> FecObjectInfo:
    f = N.Fti()
    src = (ctypes.c_uint8 * len(ext)).from_buffer_copy(ext) if ext else (ctypes.c_uint8 * 1)()
    N.check(N.lib().nfec_fti_read(fec_id, src, len(ext), ctypes.byref(f)), "nfec_fti_read")
    return FecObjectInfo(f.fec_id, f.segment_size, f.num_data, f.num_parity, f.object_size, f.fec_m,
                         f.fec_group_size, f.instance_id)


def payload_id_length(fec_id: int) -> int:
    return N.lib().nfec_payload_id_length(fec_id)


def write_payload_id(fec_id: int, fec_m: int, block_id: int, symbol_id: int, block_len: int = 0) -> bytes:
    buf = (ctypes.c_uint8 * 8)()
    n = N.check(N.lib().nfec_payload_id_write(fec_id, fec_m, block_id, symbol_id, block_len, buf),
                "nfec_payload_id_write")
    return bytes(buf[:n])


def read_payload_id(fec_id: int, fec_m: int, data: bytes):
    """-> (block_id, symbol_id, block_len); block_len is 0 except for fec_id 129."""
    need = payload_id_length(fec_id)
    if need == 0 or len(data) < need:
        raise N.NfecError(N.NFEC_EINVAL, "read_payload_id")
    src = (ctypes.c_uint8 * len(data)).from_buffer_copy(data)
    b, s, bl = ctypes.c_uint32(), ctypes.c_uint16(), ctypes.c_uint16()
    N.check(N.lib().nfec_payload_id_read(fec_id, fec_m, src, ctypes.byref(b), ctypes.byref(s), ctypes.byref(bl)),
            "nfec_payload_id_read")
    return b.value, s.value, bl.value


def sender_codec(num_data: int, num_parity: int, fec_id: int = 0, assume_mdp: bool = False):
    """-> (kind, fec_id, fec_m) as NormSession::StartSender picks them."""
    k, f, m = ctypes.c_int(), ctypes.c_uint8(), ctypes.c_uint8()
    N.check(N.lib().nfec_sender_codec(num_data, num_parity, fec_id, int(assume_mdp), ctypes.byref(k), ctypes.byref(f),
                                      ctypes.byref(m)), "nfec_sender_codec")
    return k.value, f.value, m.value


def receiver_codec(fec_id: int, fec_m: int, instance_id: int = 0, assume_mdp: bool = False) -> int:
    k = ctypes.c_int()
    N.check(N.lib().nfec_receiver_codec(fec_id, fec_m, instance_id, int(assume_mdp), ctypes.byref(k)),
            "nfec_receiver_codec")
    return k.value


def vector_size(segment_size: int) -> int:
    return N.lib().nfec_vector_size(segment_size)


def _classes():
    from . import codec as C

    return {N.NFEC_RS8: (C.NormEncoderRS8, C.NormDecoderRS8), N.NFEC_RS16: (C.NormEncoderRS16, C.NormDecoderRS16),
            N.NFEC_MDP: (C.NormEncoderMDP, C.NormDecoderMDP)}


def make_encoder(num_data: int, num_parity: int, segment_size: int, fec_id: int = 0, assume_mdp: bool = False,
                 object_size: int = 0):
    """Sender side: -> (Init()ed encoder, the FecObjectInfo to advertise)."""
    kind, fid, fm = sender_codec(num_data, num_parity, fec_id, assume_mdp)
    if kind == 0:  # numParity 0: the reference sends without an encoder (normSession.cpp:890-898)
        raise N.NfecError(N.NFEC_EINVAL, "numParity 0: NORM creates no encoder")
    enc = _classes()[kind][0]()
    if not enc.Init(num_data, num_parity, vector_size(segment_size)):
        raise N.NfecError(N.NFEC_ERANGE, "encoder Init")
    return enc, FecObjectInfo(fid, segment_size, num_data, num_parity, object_size, fm)


def make_decoder(info: FecObjectInfo, assume_mdp: bool = False):
    """Receiver side, from a parsed FTI: -> Init()ed decoder."""
    kind = receiver_codec(info.fec_id, info.fec_m, info.instance_id, assume_mdp)
    dec = _classes()[kind][1]()
    if not dec.Init(info.num_data, info.num_parity, vector_size(info.segment_size)):
        raise N.NfecError(N.NFEC_ERANGE, "decoder Init")
    return dec
