"""NORM wire format on the FEC path (include/nfec.h nfec_fti_* / nfec_payload_id_* / codec
choice), host only.  Checked against oracle/wire_ref.py (struct restatement of
normMessage.h) and against hand-written byte strings taken from the header's offset enums;
parity unpinned (no reference wire fixtures exist, see oracle/wire_ref.py)."""
import numpy as np
import pytest

from norm_amd import _native as N
from norm_amd import wire as W
from oracle import wire_ref as R


def test_fti_known_bytes():
    # fec 5, 1400-byte segments, 64+32, object 0x0123_456789AB
    info = W.FecObjectInfo(5, 1400, 64, 32, 0x0123456789AB)
    assert W.write_fti(info) == bytes.fromhex("4003 0123 456789ab 0578 40 20")
    # fec 2 m 16, G 1, 1000+200
    info = W.FecObjectInfo(2, 1024, 1000, 200, 7, fec_m=16)
    assert W.write_fti(info) == bytes.fromhex("4004 0000 00000007 10 01 0400 03e8 00c8")
    # fec 129 instance 0
    info = W.FecObjectInfo(129, 512, 200, 55, 1 << 40, instance_id=0)
    assert W.write_fti(info) == bytes.fromhex("4004 0100 00000000 0000 0200 00c8 0037")


@pytest.mark.parametrize("fec_id", [2, 5, 129])
def test_fti_round_trip_matches_restatement(fec_id):
    rng = np.random.default_rng(fec_id)
    for _ in range(200):
        top = 255 if fec_id == 5 else 65535
        nd, npar = int(rng.integers(1, top + 1)), int(rng.integers(0, top + 1))
        seg, size = int(rng.integers(1, 65536)), int(rng.integers(0, 1 << 48))
        fm = int(rng.choice([8, 16])) if fec_id == 2 else 8
        inst = int(rng.integers(0, 65536)) if fec_id == 129 else 0
        info = W.FecObjectInfo(fec_id, seg, nd, npar, size, fec_m=fm, instance_id=inst)
        raw = W.write_fti(info)
        assert raw == R.fti(fec_id, seg, nd, npar, size, fm, 1, inst)
        back = W.read_fti(fec_id, raw + b"\xee" * 4)  # trailing bytes (next extension) ignored
        assert back == info


def test_fti_rejects():
    with pytest.raises(N.NfecError):
        W.write_fti(W.FecObjectInfo(5, 1400, 256, 32))  # u8 field on the wire
    with pytest.raises(N.NfecError):
        W.write_fti(W.FecObjectInfo(7, 1400, 64, 32))
    with pytest.raises(N.NfecError):
        W.write_fti(W.FecObjectInfo(2, 1400, 64, 32, 1 << 48))
    good = W.write_fti(W.FecObjectInfo(129, 1400, 64, 32))
    with pytest.raises(N.NfecError):
        W.read_fti(129, good[:15])
    with pytest.raises(N.NfecError):
        W.read_fti(129, b"\x03" + good[1:])  # not an FTI extension
    with pytest.raises(N.NfecError):
        W.read_fti(2, good[:1] + b"\x03" + good[2:])  # length field too small for fec 2


PID = [(2, 8), (2, 16), (5, 8), (129, 8)]


@pytest.mark.parametrize("fec_id,fec_m", PID)
def test_payload_id_round_trip_matches_restatement(fec_id, fec_m):
    rng = np.random.default_rng(fec_id * 100 + fec_m)
    bmax = {8: 1 << 24, 16: 1 << 16}[fec_m] if fec_id != 129 else 1 << 32
    smax = 256 if (fec_id == 5 or fec_m == 8) and fec_id != 129 else 65536
    for _ in range(300):
        b, s, bl = int(rng.integers(0, bmax)), int(rng.integers(0, smax)), int(rng.integers(0, 65536))
        bl = bl if fec_id == 129 else 0
        raw = W.write_payload_id(fec_id, fec_m, b, s, bl)
        assert raw == R.payload_id(fec_id, fec_m, b, s, bl)
        assert len(raw) == W.payload_id_length(fec_id)
        assert W.read_payload_id(fec_id, fec_m, raw) == (b, s, bl)


def test_payload_id_known_bytes():
    assert W.write_payload_id(5, 8, 0x123456, 0x9A) == bytes.fromhex("1234569a")
    assert W.write_payload_id(2, 16, 0xBEEF, 0x0102) == bytes.fromhex("beef0102")
    assert W.write_payload_id(129, 8, 0xDEADBEEF, 7, 64) == bytes.fromhex("deadbeef 0040 0007")
    assert W.payload_id_length(3) == 0
    with pytest.raises(N.NfecError):
        W.write_payload_id(2, 12, 1, 1)


@pytest.mark.parametrize("nd,npar,fid,mdp", [(64, 32, 0, False), (200, 55, 2, False), (200, 56, 0, False),
                                             (1000, 200, 5, False), (64, 32, 0, True), (255, 1, 0, True),
                                             (64, 0, 0, False), (300, 0, 0, False), (64, 0, 0, True),
                                             (300, 0, 2, True)])
def test_sender_codec_choice(nd, npar, fid, mdp):
    assert W.sender_codec(nd, npar, fid, mdp) == R.sender_codec(nd, npar, fid, mdp)


def test_sender_without_parity_advertises_rs8_fec_id():
    # normSession.cpp:890-898: no parity -> no encoder, fec_id = fecId or 5, m = 8, whatever
    # the block size or ASSUME_MDP_FEC
    assert W.sender_codec(300, 0) == (0, 5, 8)
    assert W.sender_codec(64, 0, 0, True) == (0, 5, 8)
    assert W.sender_codec(64, 0, 2) == (0, 2, 8)
    with pytest.raises(N.NfecError):
        W.make_encoder(64, 0, 1392)


@pytest.mark.parametrize("fid", [0, 1, 2, 5, 129, 200])
@pytest.mark.parametrize("fm", [8, 16, 12])
@pytest.mark.parametrize("inst", [0, 3])
@pytest.mark.parametrize("mdp", [False, True])
def test_receiver_codec_choice(fid, fm, inst, mdp):
    want = R.receiver_codec(fid, fm, inst, mdp)
    if want is None:
        with pytest.raises(N.NfecError):
            W.receiver_codec(fid, fm, inst, mdp)
    else:
        assert W.receiver_codec(fid, fm, inst, mdp) == want


def test_vector_size_adds_stream_header():
    assert W.vector_size(1392) == 1400  # the headline workload's vector
    assert W.vector_size(65535) == 65543


@pytest.mark.gpu
@pytest.mark.parametrize("nd,npar,mdp", [(64, 32, False), (400, 100, False), (64, 32, True)])
def test_fti_sender_to_receiver_repair(nd, npar, mdp):
    """A sender picks its codec and advertises the FTI; the receiver parses the extension,
    builds its decoder from it, files symbols by payload ID and repairs the block."""
    seg = 1392 if nd + npar <= 255 else 1390
    enc, info = W.make_encoder(nd, npar, seg, assume_mdp=mdp, object_size=nd * seg)
    raw = W.write_fti(info)
    rx_info = W.read_fti(info.fec_id, raw)
    dec = W.make_decoder(rx_info, assume_mdp=mdp)
    vec = W.vector_size(seg)
    assert dec.GetVectorSize() == vec and type(dec).__name__.endswith(type(enc).__name__[len("NormEncoder"):])
    rng = np.random.default_rng(nd)
    src = [rng.integers(0, 256, vec, dtype=np.uint8) for _ in range(nd)]
    par = [np.zeros(vec, np.uint8) for _ in range(npar)]
    for s in range(nd):
        enc.Encode(s, src[s], par)
    packets = [(W.write_payload_id(info.fec_id, info.fec_m, 9, s, nd), v) for s, v in enumerate(src + par)]
    lost = set(rng.choice(nd, min(npar, nd) // 2, replace=False).tolist())
    block = [np.zeros(vec, np.uint8) for _ in range(nd + npar)]
    for pid, payload in packets:
        b, s, _ = W.read_payload_id(rx_info.fec_id, rx_info.fec_m, pid)
        assert b == 9
        if s not in lost:
            block[s][:] = payload
    locs = sorted(lost)
    assert dec.Decode(block, nd, len(locs), locs) == len(locs)
    for s in range(nd):
        assert np.array_equal(block[s], src[s]), s
