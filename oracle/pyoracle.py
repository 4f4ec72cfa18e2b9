"""ctypes wrapper of oracle/_build/liboracle.so -- the CPU restatement of NORM's FEC codecs.

TEST INFRASTRUCTURE ONLY (checker and CPU baseline).  The product (norm_amd) never
imports this module.  See norm_fec_oracle.h for what is pinned against the reference.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
RS8, RS16, MDP = 1, 2, 3
SEED = 0x4E4F524D  # "NORM"

_P, _U, _I = ctypes.c_void_p, ctypes.c_uint, ctypes.c_int
_SIGS = {
    "orc_gf8_tables": (None, [_P, _P, _P]),
    "orc_gf8_mul_table": (None, [_P]),
    "orc_gf16_tables": (None, [_P, _P, _P]),
    "orc_galois_tables": (None, [_P, _P, _P]),
    "orc_rs8_generator": (_I, [_U, _U, _P]),
    "orc_rs16_generator": (_I, [_U, _U, _P]),
    "orc_rs8_encode": (None, [_P, _U, _U, _U, _U, _P, _P]),
    "orc_rs16_encode": (None, [_P, _U, _U, _U, _U, _P, _P]),
    "orc_rs8_decode": (_I, [_P, _U, _U, _U, _P, _U, _U, _P]),
    "orc_rs16_decode": (_I, [_P, _U, _U, _U, _P, _U, _U, _P]),
    "orc_mdp_generator_poly": (_I, [_U, _P]),
    "orc_mdp_encode": (None, [_P, _U, _U, _P, _P, _P]),
    "orc_mdp_decode": (_I, [_U, _U, _P, _U, _U, _P]),
    "orc_encode_blocks": (_I, [_I, _U, _U, _U, _P, ctypes.c_uint64, _U, _P, _U]),
    "orc_decode_blocks": (_I, [_I, _U, _U, _U, _P, ctypes.c_uint64, _U, _P, _P, _U, _P, _P, _U]),
    "orc_splitmix64_mix": (ctypes.c_uint64, [ctypes.c_uint64]),
    "orc_fill_segment": (None, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, _P, _U]),
    "orc_erasure_pattern": (_U, [ctypes.c_uint64, ctypes.c_uint64, _U, _U, _P]),
    "orc_bench_rs8": (_I, [_U, _U, _U, _U, _U, _U, ctypes.c_uint64, _P, _P, _P]),
}
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.run(["make", "-C", HERE], check=True, capture_output=True)
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _lib = L
    return _lib


def gf8_tables():
    e = np.zeros(510, np.uint8); lg = np.zeros(256, np.int32); inv = np.zeros(256, np.uint8)
    lib().orc_gf8_tables(e.ctypes.data, lg.ctypes.data, inv.ctypes.data)
    return e, lg, inv


def gf8_mul_table():
    t = np.zeros((256, 256), np.uint8)
    lib().orc_gf8_mul_table(t.ctypes.data)
    return t


def gf16_tables():
    e = np.zeros(2 * 65535, np.uint16); lg = np.zeros(65536, np.int32); inv = np.zeros(65536, np.uint16)
    lib().orc_gf16_tables(e.ctypes.data, lg.ctypes.data, inv.ctypes.data)
    return e, lg, inv


def galois_tables():
    ginv = np.zeros(256, np.uint8); gexp = np.zeros(512, np.uint8); gm = np.zeros((256, 256), np.uint8)
    lib().orc_galois_tables(ginv.ctypes.data, gexp.ctypes.data, gm.ctypes.data)
    return ginv, gexp, gm


def generator(kind, k, m):
    """Full n x k systematic generator (RS8/RS16) as the reference builds it, or None."""
    if kind == RS8:
        g = np.zeros((k + m, k), np.uint8)
        rc = lib().orc_rs8_generator(k, m, g.ctypes.data)
    else:
        g = np.zeros((k + m, k), np.uint16)
        rc = lib().orc_rs16_generator(k, m, g.ctypes.data)
    return g if rc == 0 else None


def mdp_generator_poly(m):
    g = np.zeros(m + 1, np.uint8)
    assert lib().orc_mdp_generator_poly(m, g.ctypes.data) == 0
    return g


def fill_segment(block, seg, nbytes, seed=SEED):
    out = np.zeros(nbytes, np.uint8)
    lib().orc_fill_segment(seed, block, seg, out.ctypes.data, nbytes)
    return out


def erasure_pattern(block, range_, count, seed=SEED):
    out = np.zeros(max(count, 1), np.uint16)
    n = lib().orc_erasure_pattern(seed, block, range_, count, out.ctypes.data)
    return out[:n]


def make_blocks(k, m, vec, nblocks, seg_stride=None, num_data=None, seed=SEED, first_block=0):
    """Host batch [nblocks, k+m, seg_stride] with the synthetic source in slots [0, nd)."""
    stride = seg_stride or ((vec + 7) // 8 * 8)
    blocks = np.zeros((nblocks, k + m, stride), np.uint8)
    for b in range(nblocks):
        nd = k if num_data is None else int(num_data[b])
        for s in range(nd):
            lib().orc_fill_segment(seed, first_block + b, s, blocks[b, s].ctypes.data, vec)
    return blocks


def encode_blocks(kind, k, m, vec, blocks, num_data=None):
    """Reference call pattern: zero parity, then Encode() once per source segment."""
    nd = None if num_data is None else np.ascontiguousarray(num_data, np.uint16)
    rc = lib().orc_encode_blocks(kind, k, m, vec, blocks.ctypes.data, blocks.strides[0], blocks.strides[1],
                                 nd.ctypes.data if nd is not None else None, blocks.shape[0])
    assert rc == 0
    return blocks


def encode_block_with_generator(kind, enc_full, k, m, vec, src):
    """Reference call pattern for one block (zeroed parity, one Encode() per source segment,
    normEncoderRS8.cpp:473-483 / normEncoderRS16.cpp:472-482) with a given full (k+m) x k
    generator -- for codes whose generator the oracle would take too long to rebuild per call
    (C4: RS16 k=4096, ~30 s).  src: uint8 [k, >= vec].  Returns parity uint8 [m, vec]."""
    enc_full = np.ascontiguousarray(enc_full, np.uint16 if kind == RS16 else np.uint8)
    assert enc_full.shape == (k + m, k)
    par = np.zeros((m, vec), np.uint8)
    ptrs = (ctypes.c_void_p * m)(*[par[i].ctypes.data for i in range(m)])
    fn = lib().orc_rs16_encode if kind == RS16 else lib().orc_rs8_encode
    src = np.ascontiguousarray(src)
    for j in range(k):
        fn(enc_full.ctypes.data, k, m, vec, j, src[j].ctypes.data, ptrs)
    return par


def decode_blocks(kind, k, m, vec, blocks, locs, counts, num_data=None):
    """Reference Decode() per block (MDP: missing parity passed as NULL).  Returns status."""
    nd = None if num_data is None else np.ascontiguousarray(num_data, np.uint16)
    locs = np.ascontiguousarray(locs, np.uint16)
    counts = np.ascontiguousarray(counts, np.uint16)
    status = np.zeros(blocks.shape[0], np.int32)
    rc = lib().orc_decode_blocks(kind, k, m, vec, blocks.ctypes.data, blocks.strides[0], blocks.strides[1],
                                 nd.ctypes.data if nd is not None else None, locs.ctypes.data, locs.shape[1],
                                 counts.ctypes.data, status.ctypes.data, blocks.shape[0])
    assert rc == 0
    return status


def bench_rs8(k=64, m=32, vec=1400, nblocks=1000, erasures=16, threads=1, seed=SEED):
    te, td, bad = ctypes.c_double(), ctypes.c_double(), ctypes.c_uint64()
    rc = lib().orc_bench_rs8(k, m, vec, nblocks, erasures, threads, seed, ctypes.byref(te), ctypes.byref(td),
                             ctypes.byref(bad))
    assert rc == 0
    return te.value, td.value, bad.value
