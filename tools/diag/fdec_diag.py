"""Diagnostic: fused decode vs oracle on a small batch; prints mismatching blocks/slots."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

import norm_amd as na
from oracle import pyoracle as orc

k, m, vec = 64, 32, 1400
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 23
es = int(sys.argv[2]) if len(sys.argv) > 2 else 16
enc, dec = na.NormEncoderRS8(), na.NormDecoderRS8()
assert enc.Init(k, m, vec) and dec.Init(k, m, vec)
host = orc.encode_blocks(orc.RS8, k, m, vec, orc.make_blocks(k, m, vec, nb))
clean = host.copy()
locs = np.zeros((nb, m), np.uint16)
counts = np.zeros(nb, np.uint16)
for b in range(nb):
    src = orc.erasure_pattern(b, k, es)
    locs[b, :len(src)] = src
    counts[b] = len(src)
    for s in src:
        host[b, s] = 0
dev = torch.from_numpy(host).cuda()
st = dec.decode_blocks(dev, torch.from_numpy(locs.astype(np.int16)).cuda(), torch.from_numpy(counts.astype(np.int16)).cuda())
torch.cuda.synchronize()
out = dev.cpu().numpy()
print("status", st.cpu().numpy()[:8])
bad = 0
for b in range(nb):
    d = np.nonzero((out[b] != clean[b]).any(axis=1))[0]
    if len(d):
        bad += 1
        if bad <= 4:
            s = d[0]
            nbytes = int((out[b, s] != clean[b, s]).sum())
            first = int(np.nonzero(out[b, s] != clean[b, s])[0][0])
            print(f"block {b}: bad slots {d.tolist()} erased {locs[b, :counts[b]].tolist()}; slot {s}: {nbytes} bad bytes, first at {first}; out {out[b, s, first:first+8].tolist()} ref {clean[b, s, first:first+8].tolist()}")
print("bad blocks", bad, "of", nb)
