"""npc, the reference's offline file precoder (src/common/normPrecode.cpp), on the GPU path.

CPU: the CRC table against the reference's printed constants, block sizing, file layout and
the interleaver map against oracle/npc_ref.py.  GPU: whole files encoded by
nfec_npc_encode_file are byte-identical to the restated reference loop, and decoded files
(clean, with repairable damage, with too much damage) match it too.  Format parity is
unpinned beyond the CRC (see oracle/npc_ref.py)."""
import ctypes
import os
import zlib

import numpy as np
import pytest

from norm_amd import _native as N
from norm_amd import npc
from oracle import npc_ref as R


def test_crc_table_matches_reference_constants():
    t = R.crc32_table()
    # CRC32_TABLE entries as printed in normPrecode.cpp:1238-1301
    known = {0: 0x00000000, 1: 0x77073096, 2: 0xEE0E612C, 3: 0x990951BA, 8: 0x0EDB8832, 128: 0xEDB88320,
             129: 0x9ABFB3B6, 200: 0x95BF4A82, 254: 0x5A05DF1B, 255: 0x2D02EF8D}
    for i, v in known.items():
        assert t[i] == v, i
    rng = np.random.default_rng(1)
    for n in (0, 1, 7, 1020, 1396):
        buf = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert R.crc32_bytewise(buf) == zlib.crc32(buf) & 0xFFFFFFFF


def _params(**kw):
    return npc.make_params(**kw)


SIZES = [0, 1, 1019, 1020, 1021, 50_000, 1_000_000, 123_456_789]


@pytest.mark.parametrize("fs", SIZES)
@pytest.mark.parametrize("kw", [dict(block=64, parity=8), dict(auto=10), dict(), dict(auto=50, bmax=100),
                                dict(segment=517, block=300, parity=20, imax=0)])
def test_layout_matches_restatement(fs, kw):
    p = _params(**kw)
    for encode in (True, False):
        size = fs if encode else (fs // p.segment_size) * p.segment_size
        want = R.resolve(size, encode, p.segment_size, p.num_data, p.num_parity, p.parity_fraction, p.b_max)
        if want is None or 0 in want:
            with pytest.raises(N.NfecError):
                npc.layout(p, size, encode)
            continue
        try:
            lay = npc.layout(p, size, encode)
        except N.NfecError:
            assert not encode  # decode of a size whose last block holds no data (tested below)
            continue
        assert (lay.num_data, lay.num_parity) == want
        assert lay.kind == (N.NFEC_RS16 if sum(want) > 256 else N.NFEC_RS8)
        assert (lay.il_width, lay.il_height, lay.il_size) == R.init_interleaver(lay.num_segments, p.i_max)
        if encode:
            k, m, ds = lay.num_data, lay.num_parity, p.segment_size - 4
            nin = 1 + -(-size // ds) if size else 1
            assert lay.input_segments == nin
            nb = -(-nin // k)
            assert lay.num_blocks == nb and lay.last_block_data == nin - (nb - 1) * k
            assert lay.num_segments == (nb - 1) * (k + m) + lay.last_block_data + m


def test_layout_rejects():
    with pytest.raises(N.NfecError):
        npc.layout(_params(segment=11, block=10, parity=2), 1000)   # meta segment would overflow
    with pytest.raises(N.NfecError):
        npc.layout(_params(block=10, parity=0), 1000)
    with pytest.raises(N.NfecError):
        npc.layout(_params(block=60000, parity=6000), 1000)
    with pytest.raises(N.NfecError):
        npc.layout(_params(block=10, parity=4), 1024 * 4, encode=False)  # 4 segments: last block has no data
    with pytest.raises(N.NfecError):
        npc.layout(_params(block=10, parity=4), 1000, encode=False)      # not whole segments


@pytest.mark.parametrize("imax", [0, 1000, 7, 13, 30])
def test_interleaver_positions_match_restatement(imax):
    rng = np.random.default_rng(imax)
    ns = sorted(set(list(range(1, 200)) + rng.integers(200, 5000, 40).tolist()))
    p = _params(block=4, parity=1, imax=imax)
    for n in ns:
        lay = N.NpcLayout()
        lay.num_segments = n
        lay.i_max = imax
        lay.il_width, lay.il_height, lay.il_size = R.init_interleaver(n, imax)
        got = npc.positions(lay)
        want = [R.interleaver_offset(s, n, R.init_interleaver(n, imax), imax) for s in range(n)]
        assert got.tolist() == want, n
        assert sorted(want) == list(range(n)), n  # a permutation of the file's slots
    del p


def test_command_prefixes():
    assert npc._command_type("enc") == ("encode", False)
    assert npc._command_type("in") == ("input", True)
    assert npc._command_type("seg") == ("segment", True)
    assert npc._command_type("de") == (None, None)  # debug / decode: ambiguous, as in the reference
    assert npc._command_type("i") == (None, None)
    assert npc.default_output_name("/x/y/data.tar.gz") == "data.tar_gz.npc"
    assert npc.default_output_name("plain") == "plain.npc"


# ---------------- GPU: whole files ----------------

CASES = [  # name, file size, params
    ("small", 5000, dict(block=8, parity=2)),             # rotation (b*m) % k != 0 from block 1 on
    ("exact", 1020 * 40, dict(block=16, parity=4)),       # file ends on a segment boundary
    ("empty", 0, dict(block=8, parity=2)),
    ("multi_il", 300_000, dict(block=20, parity=5, imax=7)),   # many interleaver blocks
    ("auto10", 200_000, dict(auto=10)),                   # one RS8 block, reference auto sizing
    ("rs16", 400_000, dict(segment=516, block=300, parity=20)),
    ("rs16_odd", 100_000, dict(segment=517, block=250, parity=10)),
    ("seg1400", 700_001, dict(segment=1404, block=64, parity=32)),
]


def _write(tmp_path, name, size, seed=0):
    data = np.random.default_rng(seed).integers(0, 256, size, dtype=np.uint8).tobytes()
    path = tmp_path / name
    path.write_bytes(data)
    return path, data


@pytest.mark.gpu
@pytest.mark.parametrize("name,size,kw", CASES)
def test_encode_file_matches_reference_loop(tmp_path, name, size, kw):
    src, data = _write(tmp_path, f"{name}.bin", size)
    p = _params(**kw)
    lay = npc.layout(p, size)
    out = tmp_path / "out.npc"
    npc.encode_file(str(src), str(out), p)
    want = R.encode(data, src.name, p.segment_size, lay.num_data, lay.num_parity, p.i_max)
    got = out.read_bytes()
    assert len(got) == len(want)
    assert got == want


def _corrupt(buf, ss, lay, per_block, rng, p):
    """flip a byte in `per_block` random segments of each FEC block (file slots via the map)"""
    b = bytearray(buf)
    pos = npc.positions(lay)
    k, m = lay.num_data, lay.num_parity
    for blk in range(lay.num_blocks):
        nd = lay.last_block_data if blk + 1 == lay.num_blocks else k
        for t in rng.choice(nd + m, min(per_block, nd + m), replace=False):
            slot = int(pos[blk * (k + m) + t])
            b[slot * ss + int(rng.integers(0, ss))] ^= 0x5A
    return bytes(b)


@pytest.mark.gpu
@pytest.mark.parametrize("name,size,kw,damage", [
    ("one_block", 150_000, dict(auto=20), 20),            # single block: repairs are exact
    ("m_mult_k", 200_000, dict(block=16, parity=16), 16),  # (b*m) % k == 0: every block exact
    ("rotated", 100_000, dict(block=20, parity=6), 3),    # the reference's rotation: mis-repairs
    ("rs16", 150_000, dict(segment=516, block=300, parity=20), 20),  # one (shortened) block
    ("default_auto", 20_000, dict(), 15),  # the reference's defaults: RS16 k=21, m=2100
])
def test_decode_file_matches_reference_loop(tmp_path, name, size, kw, damage):
    src, data = _write(tmp_path, f"{name}.dat", size, seed=3)
    p = _params(**kw)
    enc = tmp_path / "x.npc"
    npc.encode_file(str(src), str(enc), p)
    clean = enc.read_bytes()
    # clean decode, output named from the meta segment
    cwd = os.getcwd()
    (tmp_path / "dec").mkdir()
    os.chdir(tmp_path / "dec")
    try:
        path, nbytes = npc.decode_file(str(enc), None, p)
        assert path == src.name and nbytes == size
        assert open(path, "rb").read() == data
        os.unlink(path)
    finally:
        os.chdir(cwd)
    lay = npc.layout(p, len(clean), encode=False)
    bad = _corrupt(clean, p.segment_size, lay, damage, np.random.default_rng(4), p)
    enc.write_bytes(bad)
    out = tmp_path / "y.out"
    _, nbytes = npc.decode_file(str(enc), str(out), p)
    want_name, want = R.decode(bad, p.segment_size, lay.num_data, lay.num_parity, p.i_max)
    got = out.read_bytes()
    assert want_name == src.name and got == want
    if name != "rotated":
        assert got == data


@pytest.mark.gpu
def test_decode_too_many_errors(tmp_path):
    src, data = _write(tmp_path, "t.bin", 30_000)
    p = _params(block=10, parity=3)
    enc = tmp_path / "t.npc"
    npc.encode_file(str(src), str(enc), p)
    lay = npc.layout(p, enc.stat().st_size, encode=False)
    bad = _corrupt(enc.read_bytes(), p.segment_size, lay, 4, np.random.default_rng(5), p)
    enc.write_bytes(bad)
    with pytest.raises(R.TooManyErrors):
        R.decode(bad, p.segment_size, 10, 3, p.i_max)
    with pytest.raises(N.NfecError):
        npc.decode_file(str(enc), str(tmp_path / "t.out"), p)


@pytest.mark.gpu
def test_cli_round_trip(tmp_path):
    src, data = _write(tmp_path, "cli.input.bin", 77_777, seed=9)
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        assert npc.main(["encode", "input", str(src), "seg", "1000", "block", "30", "parity", "6"]) == 0
        assert (tmp_path / "cli.input_bin.npc").exists()
        src.rename(tmp_path / "orig.bin")
        assert npc.main(["decode", "input", "cli.input_bin.npc", "seg", "1000", "block", "30", "parity", "6"]) == 0
        assert (tmp_path / "cli.input.bin").read_bytes() == data
        assert npc.main(["de", "input", "cli.input_bin.npc"]) == 1  # ambiguous command
    finally:
        os.chdir(cwd)


# ---------------- several devices (contiguous block ranges, one pipeline each) ----------------

def test_device_list_validation_without_gpu(tmp_path):
    """an empty device list fails before any file or GPU is touched"""
    p = _params(block=8, parity=2)
    src, _ = _write(tmp_path, "v.bin", 1000)
    rc = N.lib().nfec_npc_encode_file_multi(None, 0, os.fsencode(str(src)), os.fsencode(str(tmp_path / "v.npc")),
                                            ctypes.byref(p))
    assert rc == N.NFEC_EINVAL
    assert not (tmp_path / "v.npc").exists()


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
@pytest.mark.parametrize("name,size,kw", [CASES[3], CASES[5], CASES[7]])
def test_multi_device_files_identical(tmp_path, devices, name, size, kw):
    """the same pass over a device list ({0, 0}: two pipelines on one GPU) writes the same bytes,
    encode and damaged decode, as the reference loop"""
    src, data = _write(tmp_path, f"{name}.bin", size, seed=11)
    p = _params(**kw)
    enc = tmp_path / "m.npc"
    npc.encode_file(str(src), str(enc), p, devices=devices)
    lay = npc.layout(p, size)
    want = R.encode(data, src.name, p.segment_size, lay.num_data, lay.num_parity, p.i_max)
    assert enc.read_bytes() == want
    dl = npc.layout(p, len(want), encode=False)
    bad = _corrupt(want, p.segment_size, dl, max(1, dl.num_parity // 2), np.random.default_rng(12), p)
    enc.write_bytes(bad)
    out = tmp_path / "m.out"
    _, nbytes = npc.decode_file(str(enc), str(out), p, devices=devices)
    want_name, want_out = R.decode(bad, p.segment_size, dl.num_data, dl.num_parity, p.i_max)
    assert out.read_bytes() == want_out and nbytes == len(want_out)


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["first", "last"])
def test_multi_device_too_many_errors(tmp_path, where):
    """an undecodable block in the first range (whose worker opens the output) or the last one
    fails the whole pass with the reference's fatal error, and no worker is left waiting"""
    src, _ = _write(tmp_path, "e.bin", 60_000)
    p = _params(block=10, parity=3)
    enc = tmp_path / "e.npc"
    npc.encode_file(str(src), str(enc), p, devices=[0, 0, 0])
    lay = npc.layout(p, enc.stat().st_size, encode=False)
    b = bytearray(enc.read_bytes())
    pos = npc.positions(lay)
    blk = 0 if where == "first" else lay.num_blocks - 1
    for t in range(4):  # 4 bad segments > 3 parity
        b[int(pos[blk * 13 + t]) * p.segment_size + 5] ^= 1
    enc.write_bytes(bytes(b))
    with pytest.raises(N.NfecError):
        npc.decode_file(str(enc), str(tmp_path / "e.out"), p, devices=[0, 0, 0])


@pytest.mark.gpu
def test_cli_device_list(tmp_path):
    src, data = _write(tmp_path, "d.bin", 90_000, seed=2)
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        assert npc.main(["encode", "input", str(src), "block", "16", "parity", "4", "device", "0,0"]) == 0
        src.rename(tmp_path / "orig.bin")
        assert npc.main(["decode", "input", "d_bin.npc", "block", "16", "parity", "4", "device", "0,0"]) == 0
        assert (tmp_path / "d.bin").read_bytes() == data
    finally:
        os.chdir(cwd)
