"""Generate tests/golden/galois_tables.json from the REFERENCE's own galois.cpp.

Runs only where /root/reference exists (the build container).  It compiles
src/common/galois.cpp in place (oracle/ref/Makefile -> oracle/_ref/dump_galois) and
stores the three constant tables (GINV, GEXP, GMULT) as hex strings.  The fixture is
data: the reference's own table contents, used to pin the oracle's GF(2^8) arithmetic.
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def main():
    ref = os.environ.get("NORM_REF", "/root/reference")
    if not os.path.isdir(ref):
        sys.exit("reference tree not present; fixture is committed, nothing to do")
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref", f"REF={ref}"], check=True)
    out = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "dump_galois")], check=True,
                         capture_output=True, text=True).stdout
    tables = json.loads(out)
    tables["_source"] = "USNavalResearchLaboratory/norm src/common/galois.cpp (GINV :37, GEXP :58, GMULT :95)"
    with open(os.path.join(HERE, "galois_tables.json"), "w") as f:
        json.dump(tables, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main()
