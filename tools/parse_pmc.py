"""Summarise rocprofv3 PMC passes (tools/pmc.sh) per kernel: average counter value per dispatch.

HBM traffic per launch follows MI355X_MICROARCH.md (HBM section): FETCH_SIZE reads exactly half
of the bytes of a wide coalesced streaming read on gfx950, so read bytes = 2 * FETCH_SIZE KiB;
WRITE_SIZE is exact for 16-byte-per-lane streaming stores (our stores are 8-byte; reported as is).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(root):
    root = root.rstrip('/')
    # counter rows can come per XCD/SE instance: sum the rows of one dispatch, then average
    # over dispatches (per-launch totals)
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        tag = os.path.relpath(f, root).split(os.sep)[0]  # pass directory: dispatch ids restart per pass
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            cname = r.get("Counter_Name", "")
            try:
                val = float(r.get("Counter_Value", "nan"))
            except ValueError:
                continue
            per[name][cname][(tag, r.get("Dispatch_Id", ""))] += val
    out = {}
    for name, ctrs in per.items():
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        d = {c: sum(v.values()) / len(v) for c, v in ctrs.items()}
        d["dispatches"] = max(len(v) for v in ctrs.values())
        if "FETCH_SIZE" in d:
            d["hbm_read_bytes_corrected"] = 2 * d["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in d:
            d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
        out[short] = d
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()
    # traffic summary for bench.py (encode kernel, bench workload)
    # the encode kernel of the bench workload (the 4-role q4 kernel by default, then the 2-role
    # assembly kernel, then the compiler-built one)
    names = sorted((k_ for k_, v in out.items() if "enc" in k_ and "k64_m32" in k_ and "FETCH_SIZE" in v),
                   key=lambda n: ("q4" not in n, "asm" not in n))
    enc = [out[n] for n in names]
    if enc and len(sys.argv) > 2:
        e = enc[0]
        traffic = {
            "blocks": 65536, "k": 64, "m": 32, "vec": 1400,
            "kernel": [k_ for k_, v in out.items() if v is e][0],
            "encode_hbm_bytes_per_launch": round(e["hbm_read_bytes_corrected"] + e["hbm_write_bytes"]),
            "read_bytes_corrected": round(e["hbm_read_bytes_corrected"]),
            "write_bytes": round(e["hbm_write_bytes"]),
            "valu_insts_per_launch": round(e["SQ_INSTS_VALU"]) if "SQ_INSTS_VALU" in e else None,
            "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; read = 2 x FETCH_SIZE KiB "
                      "(gfx950 correction, MI355X_MICROARCH.md HBM), write = WRITE_SIZE KiB",
        }
        # the repair kernel of the same workload (the fused per-block repair, 16 source erasures)
        dec = [n for n, v in out.items() if "fdec" in n and "k64_m32" in n and "FETCH_SIZE" in v]
        if dec:
            d = out[dec[0]]
            traffic.update({
                "decode_kernel": dec[0],
                "decode_hbm_bytes_per_launch": round(d["hbm_read_bytes_corrected"] + d["hbm_write_bytes"]),
                "decode_read_bytes_corrected": round(d["hbm_read_bytes_corrected"]),
                "decode_write_bytes": round(d["hbm_write_bytes"]),
                "decode_valu_insts_per_launch": round(d["SQ_INSTS_VALU"]) if "SQ_INSTS_VALU" in d else None,
                "decode_salu_insts_per_launch": round(d["SQ_INSTS_SALU"]) if "SQ_INSTS_SALU" in d else None,
            })
        traffic["source"] = os.path.relpath(root) if not os.path.isabs(root) else root
        with open(sys.argv[2], "w") as f:
            json.dump(traffic, f, indent=1)
            f.write("\n")


if __name__ == "__main__":
    main(sys.argv[1])
