"""Generate tests/golden/rs16_c4_generator.json: the BASELINE C4 generator (RS16, k=4096,
m=256) as the oracle builds it by the reference's own construction -- Vandermonde fill,
invert_vdm, matmul, identity top (NormEncoderRS16::Init, src/common/normEncoderRS16.cpp:399-461,
restated in oracle/norm_fec_oracle.c build_generator).  That is O((n-k)k^2), ~30 s of CPU, so it
runs once here and the result is committed: SHA-256 of the 256 x 4096 parity rows (little-endian
uint16, row-major) plus four rows in full.  The codec's own generator (a closed form,
norm_amd/csrc/gf_host.cpp) is checked against this in tests/test_c4_c5.py.

Test infrastructure: the oracle builds the fixture, the product is what it checks."""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

K, M = 4096, 256
SAMPLE_ROWS = [0, 1, 100, 255]


def main():
    import numpy as np

    from oracle import pyoracle as orc

    t0 = time.time()
    g = orc.generator(orc.RS16, K, M)
    assert g is not None
    assert np.array_equal(g[:K], np.eye(K, dtype=np.uint16)), "systematic top"
    par = np.ascontiguousarray(g[K:]).astype("<u2")
    out = {
        "_source": "oracle restatement of NormEncoderRS16::Init (src/common/normEncoderRS16.cpp:399-461)",
        "k": K, "m": M,
        "parity_rows_sha256": hashlib.sha256(par.tobytes()).hexdigest(),
        "rows": {str(r): par[r].tobytes().hex() for r in SAMPLE_ROWS},
        "oracle_seconds": round(time.time() - t0, 1),
    }
    with open(os.path.join(HERE, "rs16_c4_generator.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main()
