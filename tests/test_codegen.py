"""The generated kernel sources under norm_amd/csrc/gen_*.hip are committed (the GPU box builds
nothing), so they must be exactly what tools/codegen/*.py produce: a hand edit or a stale
generator would otherwise ship unnoticed.  Each generator is rerun into a temp dir and the
output byte-compared with the committed file."""
import filecmp
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# product kernels; gen_rs8_asm.py (the round-1 2-role encode) feeds the diagnostic library only
GENERATORS = ["rs8_bitsliced", "rs8_q4", "fdec_asm", "solve_asm", "gf16_t3", "gf16_tw", "rs8_rt"]


@pytest.mark.parametrize("name", GENERATORS)
def test_generated_kernel_is_reproducible(name, tmp_path):
    out = tmp_path / f"gen_{name}.hip"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "codegen", f"gen_{name}.py"), str(out)],
                   check=True, cwd=ROOT)
    committed = os.path.join(ROOT, "norm_amd", "csrc", f"gen_{name}.hip")
    assert filecmp.cmp(str(out), committed, shallow=False), \
        f"norm_amd/csrc/gen_{name}.hip differs from tools/codegen/gen_{name}.py's output: regenerate it"


def test_every_generated_source_has_a_generator():
    gen = sorted(f[4:-4] for f in os.listdir(os.path.join(ROOT, "norm_amd", "csrc"))
                 if f.startswith("gen_") and f.endswith(".hip"))
    assert gen == sorted(GENERATORS)


def test_product_library_has_no_probe_or_variant_kernels():
    """The A/B variants and timing probes (some compute wrong parity on purpose) are built into
    the diagnostic library only (make -C norm_amd diag); the product library holds the default
    kernels and reads no NFEC_*_VARIANT switch."""
    import re

    data = open(os.path.join(ROOT, "norm_amd", "_lib", "libnfec.so"), "rb").read()
    assert b"_probe_" not in data
    assert not re.search(rb"_v[0-9]+_k[0-9]+_m[0-9]+", data)
    assert not re.search(rb"NFEC_[A-Z0-9]*VARIANT", data)
    assert b"rs8_asm_enc" not in data
    for name in GENERATORS:
        src = open(os.path.join(ROOT, "norm_amd", "csrc", f"gen_{name}.hip")).read()
        assert "getenv" not in src and "_probe_" not in src, name
