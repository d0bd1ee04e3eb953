#!/usr/bin/env python3
"""The last kernels of a rocprofv3 kernel trace (results .db) in launch order: start offset and duration (µs), the
workgroup count and the kernel name — one call's sequence of launches (pilots, first pass, merge, later passes).
usage: tools/prof_timeline.py <results.db> [n_last=16] [skip_last=0]"""
import sqlite3
import sys


def timeline(db, n, skip=0):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, grid_x, workgroup_x from kernels order by start").fetchall()
    rows = rows[:len(rows) - skip] if skip else rows
    rows = rows[-n:]
    t0 = rows[0][1] if rows else 0
    return [((s - t0) / 1e3, (e - s) / 1e3, g // max(w, 1), name) for name, s, e, g, w in rows]


if __name__ == "__main__":
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    for t, d, wgs, name in timeline(sys.argv[1], n, skip):
        print(f"{t:10.1f} {d:9.1f} wgs={wgs:<6d} {name[:96]}")
