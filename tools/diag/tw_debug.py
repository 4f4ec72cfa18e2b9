"""Tower kernel debug: encode a few RS16 shapes, report which parity rows / columns of bytes
differ from the oracle (diagnostic only)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from norm_amd import NFEC_RS16, NormEncoderRS16  # noqa: E402
import oracle.pyoracle as orc  # noqa: E402

for k, m, vec, nb, pattern in [(4, 4, 64, 1, "one"), (4, 4, 64, 1, "rand"), (8, 4, 64, 1, "rand"),
                               (5, 20, 64, 1, "rand"), (100, 20, 1400, 3, "rand"), (64, 11, 64, 2, "rand")]:
    enc = NormEncoderRS16()
    assert enc.Init(k, m, vec)
    host = orc.make_blocks(k, m, vec, nb)
    if pattern == "one":
        host[:, :k, :] = 0
        host[:, 0, 0] = 1
    ref = orc.encode_blocks(NFEC_RS16, k, m, vec, host.copy())
    dev = torch.from_numpy(host).cuda()
    enc.encode_blocks(dev)
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    bad = got != ref
    print(f"k={k} m={m} vec={vec} nb={nb} {pattern}: {int(bad.sum())} bad bytes")
    if bad.any():
        rows = np.nonzero(bad.any(axis=(0, 2)))[0]
        cols = np.nonzero(bad.any(axis=(0, 1)))[0]
        print("  bad slots", rows.tolist()[:40], "bad byte cols", cols.tolist()[:20], "...", len(cols))
        b, r, c = np.argwhere(bad)[0]
        print("  first", b, r, c, "got", got[b, r, c:c + 8].tolist(), "want", ref[b, r, c:c + 8].tolist())
        zero = (got[:, k:, :] == host[:, k:, :]).all(axis=2) if False else None
