#!/usr/bin/env python3
"""Summarise a rocprofv3 results .db (kernel trace) → per-kernel count / total / avg / min / max (µs).
usage: tools/prof_summary.py <results.db> [--csv out.csv]"""
import sqlite3
import sys


def summarize(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
                     "max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), max(lds_size), max(scratch_size) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    out = []
    tot = sum(r[2] for r in rows)
    for name, n, s, a, mn, mx, vg, ag, sg, lds, scr in rows:
        out.append(dict(kernel=name, calls=n, total_us=s / 1e3, avg_us=a / 1e3, min_us=mn / 1e3, max_us=mx / 1e3,
                        pct=100.0 * s / tot, vgpr=vg, agpr=ag, sgpr=sg, lds=lds, scratch=scr))
    return out


if __name__ == "__main__":
    res = summarize(sys.argv[1])
    hdr = f"{'kernel':70s} {'calls':>6s} {'total_us':>12s} {'avg_us':>11s} {'min_us':>10s} {'max_us':>10s} {'pct':>6s} vgpr agpr lds"
    lines = [hdr]
    for r in res:
        k = r["kernel"][:70]
        lines.append(f"{k:70s} {r['calls']:6d} {r['total_us']:12.1f} {r['avg_us']:11.2f} {r['min_us']:10.2f} "
                     f"{r['max_us']:10.2f} {r['pct']:6.2f} {r['vgpr']} {r['agpr']} {r['lds']}")
    txt = "\n".join(lines)
    print(txt)
    if "--out" in sys.argv:
        open(sys.argv[sys.argv.index("--out") + 1], "w").write(txt + "\n")
