"""The C-ABI boundary: libnfec.so loads, exports every symbol include/nfec.h declares, and its
host-side generator construction (Init's math; Lagrange closed form) equals the oracle's
restatement of the reference's Vandermonde-invert-multiply construction."""
import ctypes

import numpy as np
import pytest

from norm_amd import _native as N


def test_library_loads_and_exports_header_symbols():
    L = N.lib()
    declared = N.declared_symbols()
    assert len(declared) >= 17
    for name in declared:
        assert hasattr(L, name), f"{name} declared in include/nfec.h but not exported"
    assert L.nfec_abi_version() == 1


def test_library_built_from_this_tree():
    """The prebuilt libnfec.so (it travels to the GPU box, git keeps sources only) embeds the
    SHA-256 of the sources it was built from; it must be this tree's."""
    built = N.lib().nfec_build_id().decode()
    assert len(built) == 64
    assert built == N.source_build_id(), "libnfec.so is stale: rebuild with make -C norm_amd"


def test_drop_in_classes_exported():
    import subprocess

    out = subprocess.run(["nm", "-DC", N.LIB_PATH], capture_output=True, text=True).stdout
    for cls in ("NormEncoderRS8", "NormDecoderRS8", "NormEncoderRS16", "NormDecoderRS16", "NormEncoderMDP",
                "NormDecoderMDP"):
        assert f"{cls}::Init(unsigned int, unsigned int, unsigned short)" in out
    assert "NormEncoderRS8::Encode(unsigned int, char const*, char**)" in out
    assert "NormDecoderRS8::Decode(char**, unsigned int, unsigned int, unsigned int*)" in out


def test_no_gpu_fails_loudly():
    L = N.lib()
    if L.nfec_device_count() > 0:
        pytest.skip("a GPU is present")
    h = ctypes.c_void_p()
    rc = L.nfec_codec_create(0, N.NFEC_RS8, 64, 32, 1400, ctypes.byref(h))
    assert rc == N.NFEC_EDEVICE and not h


RS8_SHAPES = [(1, 1), (1, 254), (254, 1), (16, 4), (64, 16), (64, 32), (200, 55), (128, 127), (100, 3)]


@pytest.mark.parametrize("k,m", RS8_SHAPES)
def test_host_generator_rs8_matches_oracle(orc, k, m):
    from norm_amd.codec import build_generator

    ref = orc.generator(orc.RS8, k, m)
    assert np.array_equal(build_generator(N.NFEC_RS8, k, m), ref[k:])


@pytest.mark.parametrize("k,m", [(1, 1), (40, 10), (400, 100), (300, 256)])
def test_host_generator_rs16_matches_oracle(orc, k, m):
    from norm_amd.codec import build_generator

    ref = orc.generator(orc.RS16, k, m)
    assert np.array_equal(build_generator(N.NFEC_RS16, k, m), ref[k:])


@pytest.mark.parametrize("k,m", [(64, 32), (10, 5), (1, 1), (200, 55)])
def test_host_mdp_block_map_matches_oracle_lfsr(orc, k, m):
    """MDP parity is linear in the data: the block map column j is the LFSR's response to a
    unit impulse at step j (normEncoderMDP.cpp:178-211), computed here by the oracle."""
    from norm_amd.codec import build_generator

    G = build_generator(N.NFEC_MDP, k, m)
    g = orc.mdp_generator_poly(m)
    for j in range(k):
        par = [np.zeros(1, np.uint8) for _ in range(m)]
        arr = (ctypes.c_void_p * m)(*[p.ctypes.data for p in par])
        scratch = np.zeros(1, np.uint8)
        for s in range(k):
            d = np.array([1 if s == j else 0], np.uint8)
            orc.lib().orc_mdp_encode(g.ctypes.data, m, 1, d.ctypes.data, arr, scratch.ctypes.data)
        assert np.array_equal(G[:, j], np.array([p[0] for p in par], np.uint8))


def test_generator_limits():
    L = N.lib()
    buf = np.zeros(1 << 20, np.uint8)
    assert L.nfec_build_generator(N.NFEC_RS8, 200, 56, buf.ctypes.data, buf.nbytes) == N.NFEC_ERANGE
    assert L.nfec_build_generator(N.NFEC_MDP, 250, 6, buf.ctypes.data, buf.nbytes) == N.NFEC_ERANGE
    assert L.nfec_build_generator(N.NFEC_RS8, 200, 55, buf.ctypes.data, buf.nbytes) == N.NFEC_OK
    assert L.nfec_build_generator(N.NFEC_RS8, 64, 32, buf.ctypes.data, 10) == N.NFEC_EINVAL


def test_codec_config_validation_without_gpu():
    """nfec_codec_create_ex checks its arguments before it needs a device"""
    cfg = N.CodecConfig()
    cfg.kind, cfg.num_data, cfg.num_parity, cfg.vector_size = N.NFEC_RS16, 400, 100, 1400
    h = ctypes.c_void_p()
    cfg.flags = 1 << 7
    assert N.lib().nfec_codec_create_ex(ctypes.byref(cfg), ctypes.byref(h)) == N.NFEC_EINVAL
    cfg.flags = N.NFEC_OPT_RS16_TOEPLITZ_OFF | N.NFEC_OPT_RS16_TOEPLITZ_ON
    assert N.lib().nfec_codec_create_ex(ctypes.byref(cfg), ctypes.byref(h)) == N.NFEC_EINVAL
    cfg.flags = 0
    cfg.num_devices = 2  # a device count with no list
    assert N.lib().nfec_codec_create_ex(ctypes.byref(cfg), ctypes.byref(h)) == N.NFEC_EINVAL
    if N.lib().nfec_device_count() == 0:
        devs = (ctypes.c_int32 * 2)(0, 0)
        cfg.devices = ctypes.cast(devs, ctypes.POINTER(ctypes.c_int32))
        assert N.lib().nfec_codec_create_ex(ctypes.byref(cfg), ctypes.byref(h)) == N.NFEC_EDEVICE
    assert not h
