"""Regenerate INTEGRATION.md section 1's per-call table from tools/percall's JSON lines
(profiles/r04/percall.jsonl by default):  python tools/percall_table.py [file] [--write]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def fmt(v):
    if v < 0:
        return "—"
    if v < 1:
        return f"{v:.2f}"
    if v < 100:
        return f"{v:.1f}"
    if v < 1000:
        return f"{v:.0f}"
    return f"{v:,.0f}"


def table(rows):
    def get(kind, k, m, vec, e):
        for r in rows:
            if (r["kind"], r["k"], r["m"], r["vec"], r["erasures"]) == (kind, k, m, vec, e):
                return r
        raise KeyError((kind, k, m, vec, e))

    def enc(r):
        return fmt(r["encode_us_per_call"]), fmt(r["encode_gpu_us_per_call"]), fmt(r["oracle_encode_us_per_call"])

    def dec(r):
        return fmt(r["decode_host_us_per_call"]), fmt(r["decode_gpu_us_per_call"]), fmt(r["oracle_decode_us_per_call"])

    out = ["| Call | Drop-in (host), µs | GPU round trip, µs | CPU reference restatement, µs |", "|---|---|---|---|"]
    for label, key in [("RS8(64,16) `Encode` (one segment)", ("rs8", 64, 16, 1408, 8)),
                       ("RS8(64,32) `Encode` (one segment)", ("rs8", 64, 32, 1408, 16)),
                       ("RS8(16,4) `Encode` (one segment)", ("rs8", 16, 4, 1408, 4))]:
        h, g, o = enc(get(*key))
        out.append(f"| {label} | **{h}** | {g} | {o} |")
    for label, key in [("RS8(16,4) `Decode` (one block, 4 erasures)", ("rs8", 16, 4, 1408, 4)),
                       ("RS8(64,16) `Decode` (8 erasures)", ("rs8", 64, 16, 1408, 8)),
                       ("RS8(64,32) `Decode` (16 erasures)", ("rs8", 64, 32, 1408, 16)),
                       ("RS8(64,32) × 1400 B `Decode` (16 erasures)", ("rs8", 64, 32, 1400, 16)),
                       ("RS8(200,55) `Decode` (55 erasures)", ("rs8", 200, 55, 1408, 55)),
                       ("RS8(128,127) `Decode` (100 erasures)", ("rs8", 128, 127, 1408, 100)),
                       ("RS8(128,127) × 8192 B `Decode` (100 erasures, 8 threads)", ("rs8", 128, 127, 8192, 100))]:
        h, g, o = dec(get(*key))
        out.append(f"| {label} | **{h}** | {g} | {o} |")
    for label, key in [("MDP(64,32) `Encode` / `Decode` (16 erasures)", ("mdp", 64, 32, 1408, 16)),
                       ("RS16(400,20) × 1400 B `Encode` / `Decode` (10 erasures)", ("rs16", 400, 20, 1400, 10)),
                       ("RS16(400,100) × 1400 B `Encode` / `Decode` (50 erasures, 8 threads)", ("rs16", 400, 100, 1400, 50))]:
        r = get(*key)
        (he, ge, oe), (hd, gd, od) = enc(r), dec(r)
        ref = "—" if oe == "—" else f"{oe} / {od}"
        out.append(f"| {label} | **{he}** / **{hd}** | {ge} / {gd} | {ref} |")
    for label, key in [("MDP(128,127) `Decode` (100 erasures)", ("mdp", 128, 127, 1408, 100)),
                       ("MDP(128,127) × 8192 B `Decode` (100 erasures, 8 threads)", ("mdp", 128, 127, 8192, 100))]:
        h, g, o = dec(get(*key))
        out.append(f"| {label} | **{h}** | {g} | {o} |")
    return "\n".join(out) + "\n"


def main():
    args = [a for a in sys.argv[1:] if a != "--write"]
    path = args[0] if args else os.path.join(ROOT, "profiles", "r04", "percall.jsonl")
    rows = [json.loads(line) for line in open(path) if line.strip()]
    t = table(rows)
    if "--write" not in sys.argv:
        sys.stdout.write(t)
        return
    p = os.path.join(ROOT, "INTEGRATION.md")
    s = open(p).read()
    a = s.index("| Call | Drop-in (host), µs |")
    b = s.index("\n\n", a)
    open(p, "w").write(s[:a] + t.rstrip("\n") + s[b:])


if __name__ == "__main__":
    main()
