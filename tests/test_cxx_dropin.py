"""The C++ drop-in surface (include/norm_fec/normEncoder*.h) exercised the way NORM uses it.

tests/native/nfec_fectest is the reference's fecTest (src/common/fecTest.cpp:23-135) restated
against the GPU classes: Init, per-segment Encode and whole-block Decode called through
NormEncoder* / NormDecoder* base pointers, Destroy + re-Init, delete through the base class.
It is built with plain g++ against libnfec.so (no HIP headers), as a NORM tree would link it.
Its encoded block, Decode() return value and repaired block are compared byte for byte with
the oracle's reference call pattern on the same input.
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "_build", "nfec_fectest")


def test_fectest_links_against_libnfec_only():
    """Every symbol resolves at load (LD_BIND_NOW) and the usage path runs without a GPU."""
    assert os.path.exists(EXE), "build() builds tests/native"
    r = subprocess.run([EXE], env=dict(os.environ, LD_BIND_NOW="1"), capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage" in r.stderr
    ldd = subprocess.run(["ldd", EXE], capture_output=True, text=True).stdout
    assert "libnfec.so" in ldd and "not found" not in ldd


NATIVE = os.path.join(ROOT, "tests", "native")
SRC = os.path.join(NATIVE, "nfec_fectest.cpp")


def _syntax(*incs):
    return subprocess.run(["g++", "-std=c++11", "-fsyntax-only"] + [f"-I{i}" for i in incs] + [SRC],
                          capture_output=True, text=True, timeout=120)


def test_reference_named_headers_shadow_the_reference():
    """NORM's call sites include normEncoderMDP.h / normEncoderRS8.h / normEncoderRS16.h by name
    (normSession.cpp:3-5).  With include/norm_fec ahead of the tree's include/ (INTEGRATION.md
    section 1) the engine's headers win; poison/ holds #error stand-ins under the reference
    names, so the order is what makes the unit compile."""
    good = _syntax(os.path.join(ROOT, "include", "norm_fec"), os.path.join(NATIVE, "poison"))
    assert good.returncode == 0, good.stderr
    bad = _syntax(os.path.join(NATIVE, "poison"), os.path.join(ROOT, "include", "norm_fec"))
    assert bad.returncode != 0 and "was picked up instead of include/norm_fec" in bad.stderr


def test_reference_include_guards():
    """Same guards as the reference headers, so a stray second include of either is a no-op."""
    want = {"normEncoder.h": "_NORM_ENCODER", "normEncoderRS8.h": "_NORM_ENCODER_RS8",
            "normEncoderRS16.h": "_NORM_ENCODER_RS16", "normEncoderMDP.h": "_NORM_ENCODER_MDP"}
    for name, guard in want.items():
        text = open(os.path.join(ROOT, "include", "norm_fec", name)).read()
        assert f"#ifndef {guard}\n#define {guard}\n" in text, name


@pytest.mark.skipif(not os.path.isdir("/root/reference/include"), reason="reference tree absent (GPU box)")
def test_headers_shadow_the_real_reference_include_dir():
    r = _syntax(os.path.join(ROOT, "include", "norm_fec"), "/root/reference/include")
    assert r.returncode == 0, r.stderr


def test_dropin_layout_matches_library():
    """sizeof() of the six classes as a NORM unit sees them equals the library's (no GPU)."""
    r = subprocess.run([EXE, "layout"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "errors 0" in r.stdout, r.stdout + r.stderr


KINDS = {"rs8": 1, "rs16": 2, "mdp": 3}
CASES = [
    # kind, k, m, vec, numData, erasures (sorted), null parity, input ("-": fecTest's printable data)
    ("rs16", 400, 100, 64, 400, [17, 433], False, "-"),          # fecTest.cpp:13-16 shape, 2 of n erased
    ("rs16", 400, 100, 1400, 400, list(range(0, 400, 8)), True, "rand"),  # 50 source erasures, vec 1400
    ("rs16", 40, 10, 65, 40, [3, 39, 41], True, "rand"),        # odd vector: last byte never written
    ("rs8", 64, 32, 1400, 64, list(range(3, 64, 4)), True, "rand"),        # the headline shape, 16 lost
    ("rs8", 64, 32, 1400, 64, [0, 5, 63, 64, 70, 95], True, "rand"),      # source + parity lost
    ("rs8", 64, 16, 1408, 40, [1, 2, 39, 40, 55], True, "rand"),          # shortened block, vec = 1400 + 8
    ("rs8", 16, 4, 64, 16, [0, 1, 2, 3, 4], False, "rand"),               # more erasures than parity -> 0
    ("mdp", 64, 32, 1400, 64, list(range(5, 64, 6)) + [70], True, "rand"),
    ("mdp", 16, 4, 33, 12, [2, 7, 13], True, "rand"),
]


def _no_gpu():
    from norm_amd import _native as N

    return N.lib().nfec_device_count() == 0


@pytest.mark.parametrize("kind,k,m,vec,nd,locs,nullpar,src", CASES)
def test_fectest_host_only_matches_oracle(orc, tmp_path, kind, k, m, vec, nd, locs, nullpar, src):
    """No GPU (this container): Init builds host-only codecs (NFEC_OPT_HOST_ONLY) and the
    drop-in's per-call Encode / Decode run on the CPU -- the same bytes as the oracle."""
    if not _no_gpu():
        pytest.skip("a gfx950 is visible: the GPU variants below cover this box")
    err = _run_fectest(orc, tmp_path, kind, k, m, vec, nd, locs, nullpar, src, {"NFEC_FECTEST_GPU": "0"})
    assert "host_only=1/1" in err, err


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["host_calls", "gpu_calls", "gpu_calls_2dev"])
@pytest.mark.parametrize("kind,k,m,vec,nd,locs,nullpar,src", CASES)
def test_fectest_matches_oracle(orc, tmp_path, kind, k, m, vec, nd, locs, nullpar, src, mode):
    """host_calls: the drop-in's host per-call defaults on a GPU codec; gpu_calls: the per-call
    GPU round trips (NFEC_FECTEST_GPU=1); gpu_calls_2dev: the same on a codec striped over the
    device list {0, 0} (NfecCodecBase::SetDevices, NFEC_FECTEST_DEVICES)"""
    env = {"NFEC_FECTEST_GPU": "0" if mode == "host_calls" else "1"}
    if mode == "gpu_calls_2dev":
        env["NFEC_FECTEST_DEVICES"] = "0,0"
    err = _run_fectest(orc, tmp_path, kind, k, m, vec, nd, locs, nullpar, src, env)
    assert "host_only=0/0" in err, err
    assert ("devices=2/2" if mode == "gpu_calls_2dev" else "devices=1/1") in err, err


def _run_fectest(orc, tmp_path, kind, k, m, vec, nd, locs, nullpar, src, env_extra):
    n = nd + m
    if src == "-":
        data = np.zeros((nd, vec), np.uint8)
        for i in range(nd):
            data[i, : vec - 1] = ord("a") + i % 26
        inp = "-"
    else:
        data = np.random.default_rng(nd * 131 + m).integers(0, 256, (nd, vec), dtype=np.uint8)
        inp = str(tmp_path / "in.bin")
        data.tofile(inp)
    out = tmp_path / "out.bin"
    env = dict(os.environ, **env_extra)
    r = subprocess.run([EXE, kind, str(k), str(m), str(vec), str(nd), inp, str(out), str(int(nullpar))]
                       + [str(x) for x in locs], capture_output=True, text=True, timeout=120, env=env)
    dump = np.fromfile(out, np.uint8)
    assert dump.size == 2 * n * vec + 4, r.stderr
    assert "layout_errors=0" in r.stderr, r.stderr  # inline accessors and sizeof agree with the library
    tx = dump[: n * vec].reshape(n, vec)
    status = int(dump[n * vec: n * vec + 4].view(np.int32)[0])
    rx = dump[n * vec + 4:].reshape(n, vec)

    # oracle: the same block through the reference call pattern
    blocks = np.zeros((1, k + m, vec), np.uint8)
    blocks[0, :nd] = data
    nda = np.array([nd], np.uint16)
    kid = KINDS[kind]
    ref = orc.encode_blocks(kid, k, m, vec, blocks.copy(), nda)
    assert np.array_equal(tx, ref[0, :n]), "parity differs from the oracle's Encode"
    want = ref.copy()
    for s in locs:
        want[0, s] = 0
    el = np.zeros((1, m + len(locs)), np.uint16)
    el[0, : len(locs)] = locs
    st_ref = orc.decode_blocks(kid, k, m, vec, want, el, np.array([len(locs)], np.uint16), nda)
    assert status == int(st_ref[0])
    # source slots: repaired (or left as received); parity slots are never written by Decode
    assert np.array_equal(rx[:nd], want[0, :nd])
    got_par = rx[nd:]
    exp_par = ref[0, nd:n].copy()
    for s in locs:
        if s >= nd:
            exp_par[s - nd] = 0
    assert np.array_equal(got_par, exp_par)
    if status:
        assert r.returncode == 0, r.stderr
        nbytes = vec & ~1 if kind == "rs16" else vec  # RS16 never repairs an odd last byte
        assert np.array_equal(rx[:nd, :nbytes], data[:, :nbytes])
    return r.stderr


def test_fectest_explicit_device_list_is_not_a_host_fallback(tmp_path):
    """The host-only fallback is for a process with no usable gfx950 and no device chosen: a
    device list given through NfecCodecBase::SetDevices that cannot be opened makes Init fail
    (the reference's Init-returns-false path), here (no GPU) and on a box with a bad ordinal."""
    if not _no_gpu():
        pytest.skip("needs a process without a usable gfx950")
    inp = tmp_path / "in.bin"
    np.zeros((16, 64), np.uint8).tofile(inp)
    env = dict(os.environ, NFEC_FECTEST_GPU="0", NFEC_FECTEST_DEVICES="0,0")
    r = subprocess.run([EXE, "rs8", "16", "4", "64", "16", str(inp), str(tmp_path / "out.bin"), "0", "1"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "Init(16, 4, 64) failed" in r.stderr, r.stderr
    # and the default (no device chosen) still falls back, with its notice
    env.pop("NFEC_FECTEST_DEVICES")
    r = subprocess.run([EXE, "rs8", "16", "4", "64", "16", str(inp), str(tmp_path / "out.bin"), "0", "1"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and "built a host-only codec" in r.stderr, r.stderr
