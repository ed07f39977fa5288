"""Summarise a rocprofv3 --kernel-trace SQLite output (not collected by pytest)."""
import sqlite3
import sys

import numpy as np


def summary(db, top=30):
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration, start, end from kernels order by start").fetchall()
    tot = sum(r[1] for r in rows)
    agg = {}
    for n, d, _, _ in rows:
        a = agg.setdefault(n, [0, 0.0])
        a[0] += 1
        a[1] += d
    out = [f"{'kernel':<90} {'calls':>6} {'total_us':>10} {'avg_us':>8} {'pct':>6}"]
    for n, (k, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
        out.append(f"{n[:90]:<90} {k:>6} {d / 1e3:>10.1f} {d / k / 1e3:>8.2f} {100 * d / tot:>6.2f}")
    s = np.array([r[2] for r in rows], float)
    e = np.array([r[3] for r in rows], float)
    out.append(f"kernels {len(rows)}, busy {tot / 1e3:.1f} us, span {(e.max() - s.min()) / 1e3:.1f} us")
    return "\n".join(out)


if __name__ == "__main__":
    print(summary(sys.argv[1]))
