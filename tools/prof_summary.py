"""Summarise a rocprofv3 ``--kernel-trace`` database (``<dir>/*_results.db``): kernel time by
name (calls, total, average, share) plus dispatch count and the busy span, for ``profiles/``."""
import glob
import sqlite3
import sys


def summary(path, top=40, width=90):
    db = path if path.endswith(".db") else glob.glob(f"{path}/*results.db")[0]
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), min(start), max(end) from kernels "
                     "group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows)
    n = sum(r[1] for r in rows)
    span = max(r[4] for r in rows) - min(r[3] for r in rows)
    out = [f"{n} dispatches, {tot / 1e6:.3f} ms kernel time, {span / 1e6:.3f} ms span",
           f"{'kernel':<{width}} {'calls':>6} {'total_us':>10} {'avg_us':>9} {'%':>6}"]
    for name, cnt, d, _, _ in rows[:top]:
        nm = name if len(name) <= width else name[:width - 3] + "..."
        out.append(f"{nm:<{width}} {cnt:>6} {d / 1e3:>10.1f} {d / 1e3 / cnt:>9.2f} {100 * d / tot:>6.1f}")
    return "\n".join(out)


if __name__ == "__main__":
    print(summary(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40))
