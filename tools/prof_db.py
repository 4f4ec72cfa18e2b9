"""Summaries from a rocprofv3 results.db (the default output format): per-kernel stats
(calls, total, average, min, max in us) or, with --seq, the dispatch sequence with grid sizes."""
import argparse
import sqlite3


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--seq", action="store_true")
    p.add_argument("--min-us", type=float, default=0.0)
    p.add_argument("--match", default="")
    a = p.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, duration, grid_x, workgroup_x from kernels order by start").fetchall()
    rows = [(n, d / 1000.0, g, w) for n, d, g, w in rows if a.match in n and d / 1000.0 >= a.min_us]
    if a.seq:
        for n, d, g, w in rows:
            print(f"{d:10.1f} {g // max(w, 1):8d} {n[:110]}")
        return
    st = {}
    for n, d, _, _ in rows:
        s = st.setdefault(n, [0, 0.0, 1e30, 0.0])
        s[0] += 1
        s[1] += d
        s[2] = min(s[2], d)
        s[3] = max(s[3], d)
    print(f"{'calls':>6} {'total_us':>12} {'avg_us':>10} {'min_us':>10} {'max_us':>10}  kernel")
    for n, (k, t, lo, hi) in sorted(st.items(), key=lambda x: -x[1][1]):
        print(f"{k:6d} {t:12.1f} {t / k:10.1f} {lo:10.1f} {hi:10.1f}  {n[:100]}")


if __name__ == "__main__":
    main()
