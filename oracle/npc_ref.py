"""TEST INFRASTRUCTURE ONLY: a literal restatement of the reference's npc encode/decode
loops (src/common/normPrecode.cpp), the checker for norm_amd/csrc/npc.cpp.  Only tests/
import this.  The FEC arithmetic goes through the C oracle's per-segment Encode/Decode
restatements (oracle/norm_fec_oracle.c), called exactly as npc calls NormEncoder/NormDecoder.

Pinning: npc needs protolib (ProtoApp, ProtoFile), an un-vendored submodule, so the tool
cannot be built here and the reference ships no .npc files: the file format is unpinned
except for the CRC, whose table is checked against CRC32_TABLE's printed constants
(normPrecode.cpp:1238-1301) in tests/test_npc.py.
"""
import ctypes
import math
import zlib

import numpy as np

from . import pyoracle as orc

SEGMENT_MAX = 8192


def crc32_table():
    """CRC32_TABLE (normPrecode.cpp:1238-1301): reflected 0x04C11DB7."""
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ (0xEDB88320 if c & 1 else 0)
        t.append(c)
    return t


_TAB = crc32_table()


def crc32_bytewise(buf):
    """ComputeCRC32 (normPrecode.cpp:1303-1313), byte at a time."""
    r = 0xFFFFFFFF
    for b in bytes(buf):
        r = _TAB[(r ^ b) & 0xFF] ^ (r >> 8)
    return r ^ 0xFFFFFFFF


def crc32(buf):
    # the same function as crc32_bytewise (checked in tests/test_npc.py); zlib is faster
    return zlib.crc32(bytes(buf)) & 0xFFFFFFFF


def resolve(file_size, encode, segment=1024, block=196, parity=4, pf=100.0, bmax=65536):
    """OnStartup's auto sizing (normPrecode.cpp:383-434) -> (numData, numParity) or None."""
    nd, np_ = block, parity
    if pf >= 0.0:
        if encode:
            bs = (file_size // (segment - 4)) & 0xFFFFFFFF
            if file_size % (segment - 4):
                bs += 1
            bs += 1
        else:
            ns = file_size // segment
            bs = int((ns / (1.0 + pf)) + 0.5)
        if bs > bmax:
            bs = bmax
        par = int((pf * bs) + 0.5)
        if bs + par > 65536:
            scale = 65536.0 / float(bs + par)
            bs = int(scale * bs)
            par = int(scale * par)
        nd, np_ = bs, par
    if nd + np_ > 65536:
        return None
    return nd, np_


def init_interleaver(n, imax):
    """InitInterleaver (normPrecode.cpp:450-462) -> (width, height, size)."""
    w = int(math.sqrt(float(n)))
    h = n // w
    if n % h:
        h += 1
    if imax > 0 and (w > imax or h > imax):
        h = w = imax
    return w, h, w * h


def interleaver_offset(seg, n, geom, imax):
    """ComputeInterleaverOffset (normPrecode.cpp:465-556), in segments."""
    W, H, S = geom
    w, h = W, H
    if imax > 0:
        blk, seg = seg // S, seg % S
    else:
        blk = 0
    last = n - 1
    if blk == last // S and n % S:
        lbs = n % S
        w = int(math.sqrt(float(lbs)))
        h = lbs // w
        if lbs % h:
            h += 1
    col, row = seg // h, seg % h
    iid = row * w + col
    if blk:
        iid += blk * S
    if iid >= n:
        last = n - 1
        if blk:
            iid, last = iid % S, last % S
        max_row, max_col = last // w, last % w
        empty = h - max_row - 1
        delta = 1 + empty * col
        if col > max_col:
            delta += row - max_row
            delta += col - max_col - 1
        else:
            delta += row - max_row - 1
        last_col, last_row = last // h, last % h
        last_row += delta
        if last_col == max_col and last_row > max_row:
            last_col += 1
            last_row -= max_row + 1
        col = last_col + last_row // max_row
        row = last_row % max_row
        iid = row * w + col
        if blk:
            iid += blk * S
    return iid


class _Codec:
    def __init__(self, k, m, vec):
        self.k, self.m, self.vec = k, m, vec
        self.rs16 = k + m > 256  # normPrecode.cpp:624-628, :911-915
        self.gen = orc.generator(orc.RS16 if self.rs16 else orc.RS8, k, m)
        assert self.gen is not None, "encoder Init fails (numData + numParity too large)"

    def encode(self, seg_id, data, parity):
        arr = (ctypes.c_void_p * self.m)(*[p.ctypes.data for p in parity])
        f = orc.lib().orc_rs16_encode if self.rs16 else orc.lib().orc_rs8_encode
        f(self.gen.ctypes.data, self.k, self.m, self.vec, seg_id, data.ctypes.data, arr)

    def decode(self, vecs, nd, locs):
        arr = (ctypes.c_void_p * len(vecs))(*[v.ctypes.data for v in vecs])
        el = (ctypes.c_uint * len(locs))(*locs)
        f = orc.lib().orc_rs16_decode if self.rs16 else orc.lib().orc_rs8_decode
        return f(self.gen.ctypes.data, self.k, self.m, self.vec, arr, nd, len(locs), el)


def encode(data, name, segment, k, m, imax=1000):
    """NormPrecodeApp::Encode (normPrecode.cpp:588-826) -> the .npc bytes."""
    ss, ds = segment, segment - 4
    fs = len(data)
    nin = 1 + fs // ds
    last_seg = fs % ds
    if last_seg:
        nin += 1
    else:
        last_seg = ds
    nb = nin // k
    lbs = nin % k
    if lbs:
        nb += 1
    else:
        lbs = k
    nout = (nb - 1) * (k + m) + lbs + m
    geom = init_interleaver(nout, imax)
    codec = _Codec(k, m, ds)
    out = bytearray(nout * ss)
    parity = [np.zeros(ss, np.uint8) for _ in range(m)]
    meta = np.zeros(SEGMENT_MAX, np.uint8)
    meta[:8] = np.frombuffer(fs.to_bytes(8, "big"), np.uint8)
    nm = name.encode()[:ss - 12]
    meta[8:8 + len(nm)] = np.frombuffer(nm, np.uint8)
    block_id, parity_count, parity_ready = 0, 0, False
    in_id, out_id, rd = 0, 0, 0
    while out_id < nout:
        pos = interleaver_offset(out_id, nout, geom, imax)
        seg = np.zeros(ss, np.uint8)
        if parity_ready:
            seg[:ds] = parity[m - parity_count][:ds]
            parity_count -= 1
            if parity_count == 0:
                for p in parity:
                    p[:] = 0
                parity_ready = False
                block_id += 1
        else:
            in_id += 1
            if in_id == 1:
                seg[:ds] = meta[:ds]
            else:
                n = ds if in_id != nin else last_seg
                seg[:n] = np.frombuffer(data[rd:rd + n], np.uint8)
                rd += n
            codec.encode(out_id % k, seg, parity)  # the reference's segment id (:746)
            nd = k if block_id != nb - 1 else lbs
            parity_count += 1
            if nd == parity_count:
                parity_count = m
                parity_ready = True
        seg[ds:ds + 4] = np.frombuffer(crc32(seg[:ds]).to_bytes(4, "big"), np.uint8)
        out[pos * ss:(pos + 1) * ss] = seg.tobytes()
        out_id += 1
    return bytes(out)


class TooManyErrors(Exception):
    pass


def decode(npc, segment, k, m, imax=1000):
    """NormPrecodeApp::Decode (normPrecode.cpp:828-1227) -> (meta file name, output bytes)."""
    ss, ds = segment, segment - 4
    nin = len(npc) // ss
    assert len(npc) % ss == 0
    nb = nin // (k + m)
    lbs = nin % (k + m)
    if lbs:
        lbs -= m
        nb += 1
    else:
        lbs = k
    geom = init_interleaver(nin, imax)
    codec = _Codec(k, m, ds)
    out = bytearray()
    out_size, name = 0, ""
    in_id = 0
    for b in range(nb):
        nd = k if b != nb - 1 else lbs
        vecs, locs = [], []
        for i in range(nd + m):
            pos = interleaver_offset(in_id, nin, geom, imax)
            in_id += 1
            seg = np.frombuffer(npc[pos * ss:(pos + 1) * ss], np.uint8).copy()
            if crc32(seg[:ds]).to_bytes(4, "big") != seg[ds:ds + 4].tobytes():
                locs.append(i)
                if len(locs) > m:
                    raise TooManyErrors(b)
                seg[:ds] = 0
            vecs.append(seg)
        if locs:
            codec.decode(vecs, nd, locs)
        for i in range(nd):
            if b == 0 and i == 0:
                out_size = int.from_bytes(vecs[0][:8].tobytes(), "big")
                raw = vecs[0][8:8 + min(4096, ss - 12)].tobytes()
                name = raw.split(b"\0", 1)[0].decode(errors="surrogateescape")
                continue
            n = ds
            if b == nb - 1 and i == nd - 1:
                n = out_size % ds or ds
            out += vecs[i][:n].tobytes()
    return name, bytes(out)
