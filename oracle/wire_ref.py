"""TEST INFRASTRUCTURE ONLY: a struct-module restatement of NORM's FEC wire fields, the
checker for norm_amd/csrc/wire.cpp.  Only tests/ import this.

Parity unpinned: the reference's accessors (include/normMessage.h) need protolib's
protokit.h, an un-vendored submodule that is empty under /root/reference, so they cannot be
compiled here, and the reference holds no packet captures or wire fixtures.  The layouts
below are read off the header's offset enums and setters, cited per function.
"""
import struct

FTI_TYPE = 64  # NormHeaderExtension::FTI, normMessage.h:330


def fti(fec_id, segment_size, num_data, num_parity, object_size=0, fec_m=8, group=1, instance=0):
    msb, lsb = object_size >> 32, object_size & 0xFFFFFFFF
    if fec_id == 2:  # NormFtiExtension2, normMessage.h:785-839 (length 4 words)
        return struct.pack(">BBHIBBHHH", FTI_TYPE, 4, msb, lsb, fec_m, group, segment_size, num_data, num_parity)
    if fec_id == 5:  # NormFtiExtension5, normMessage.h:898-942 (length 3 words, u8 block sizes)
        return struct.pack(">BBHIHBB", FTI_TYPE, 3, msb, lsb, segment_size, num_data, num_parity)
    if fec_id == 129:  # NormFtiExtension129, normMessage.h:977-1029 (length 4 words)
        return struct.pack(">BBHIHHHH", FTI_TYPE, 4, msb, lsb, instance, segment_size, num_data, num_parity)
    raise ValueError(fec_id)


def payload_id(fec_id, fec_m, block, symbol, block_len=0):
    """NormPayloadId setters, normMessage.h:396-567."""
    if fec_id == 5 or (fec_id == 2 and fec_m == 8):
        return struct.pack(">I", ((block << 8) | (symbol & 0xFF)) & 0xFFFFFFFF)
    if fec_id == 2 and fec_m == 16:
        return struct.pack(">HH", block & 0xFFFF, symbol)
    if fec_id == 129:
        return struct.pack(">IHH", block, block_len, symbol)
    raise ValueError((fec_id, fec_m))


def sender_codec(num_data, num_parity, fec_id=0, assume_mdp=False):
    """NormSession::StartSender codec choice, normSession.cpp:834-873 -> (kind, fec_id, m)
    with kind 1 RS8, 2 RS16, 3 MDP, 0 no codec (numParity 0, normSession.cpp:890-898)."""
    if num_parity == 0:
        return (0, fec_id or 5, 8)
    if num_data + num_parity <= 255:
        return (3, 129, 8) if assume_mdp else (1, fec_id or 5, 8)
    return (2, 2, 16)


def receiver_codec(fec_id, fec_m, instance=0, assume_mdp=False):
    """NormSenderNode::AllocateBuffers decoder choice, normNode.cpp:290-356 (None = refused)."""
    if fec_id == 2:
        return {8: 1, 16: 2}.get(fec_m)
    if fec_id == 5:
        return 1
    if fec_id == 129:
        return 3 if assume_mdp else (1 if instance == 0 else None)
    return None
