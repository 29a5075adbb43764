"""Summarise a rocprofv3 ``*_results.db`` (rocpd sqlite): per-kernel totals, and optionally the
busy/idle split of the last N dispatches (to see launch gaps inside hipGraph replays).

  python tools/rocpd_stats.py gpurun_out/prof/run_results.db [--top 30] [--tail 2000] [--csv out.csv]
"""
import argparse
import sqlite3


def load(db):
    c = sqlite3.connect(db)
    q = """select k.kernel_name, d.start, d.end, d.grid_size_x, d.grid_size_y, d.grid_size_z,
                  d.workgroup_size_x from rocpd_kernel_dispatch d
           join rocpd_info_kernel_symbol k on d.kernel_id = k.id order by d.start"""
    return c.execute(q).fetchall()


def short(name, n=90):
    name = name.split("(")[0] if "(" in name and not name.startswith("void") else name
    return name if len(name) <= n else name[:n - 3] + "..."


def summarize(rows, top):
    agg = {}
    for name, s, e, *_ in rows:
        t, cnt = agg.get(name, (0, 0))
        agg[name] = (t + (e - s), cnt + 1)
    tot = sum(t for t, _ in agg.values())
    out = []
    for name, (t, cnt) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        out.append((short(name), cnt, t / 1e3, t / cnt / 1e3, 100.0 * t / tot))
    return tot, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--tail", type=int, default=0, help="also analyse the last N dispatches")
    ap.add_argument("--csv", default=None)
    ap.add_argument("--seq", type=int, default=0,
                    help="print the last N dispatches in order (name, grid, duration, gap)")
    a = ap.parse_args()
    rows = load(a.db)
    tot, out = summarize(rows, a.top)
    print(f"{len(rows)} dispatches, {tot / 1e6:.3f} ms kernel time")
    print(f"{'kernel':90s} {'calls':>7s} {'total_us':>10s} {'avg_us':>9s} {'%':>6s}")
    for r in out:
        print(f"{r[0]:90s} {r[1]:7d} {r[2]:10.1f} {r[3]:9.2f} {r[4]:6.1f}")
    if a.csv:
        with open(a.csv, "w") as f:
            f.write("kernel,calls,total_us,avg_us,pct\n")
            for r in out:
                f.write(f"\"{r[0]}\",{r[1]},{r[2]:.1f},{r[3]:.3f},{r[4]:.2f}\n")
    if a.tail:
        sub = rows[-a.tail:]
        span = sub[-1][2] - sub[0][1]
        busy = sum(e - s for _, s, e, *_ in sub)
        print(f"\nlast {len(sub)} dispatches: span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us "
              f"({100.0 * busy / span:.1f}%), mean gap {(span - busy) / max(len(sub) - 1, 1) / 1e3:.2f} us")
        t2, out2 = summarize(sub, a.top)
        for r in out2:
            print(f"{r[0]:90s} {r[1]:7d} {r[2]:10.1f} {r[3]:9.2f} {r[4]:6.1f}")
    if a.seq:
        sub = rows[-a.seq:]
        prev = None
        print(f"\n{'#':>5s} {'dur_us':>9s} {'gap_us':>8s} {'grid':>18s}  kernel")
        for i, (name, s, e, gx, gy, gz, wx) in enumerate(sub):
            gap = (s - prev) / 1e3 if prev is not None else 0.0
            prev = e
            print(f"{i:5d} {(e - s) / 1e3:9.1f} {gap:8.1f} {f'{gx}x{gy}x{gz}/{wx}':>18s}  {short(name, 110)}")


if __name__ == "__main__":
    main()
