"""Per-kernel summary of a rocprofv3 ``--kernel-trace`` SQLite output (``*_results.db``).

ROCm 7 writes the rocpd database by default; this prints (and optionally writes as CSV) the
kernels sorted by total time, with the grid, VGPR count and the share of all kernel time.
``--per-step N`` divides totals by N (the number of profiled training steps).

    python scripts/rocpd_stats.py gpurun_out/prof/run_results.db --per-step 13 --csv profiles/x.csv
"""
import argparse
import csv
import sqlite3
import sys


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--per-step", type=float, default=0.0)
    ap.add_argument("--csv", default=None)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--short", type=int, default=90, help="truncate kernel names to this many chars")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), max(grid_x*grid_y*grid_z/"
        "(workgroup_x*workgroup_y*workgroup_z)), max(vgpr_count), max(accum_vgpr_count), max(scratch_size) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    div = a.per_step if a.per_step > 0 else 1.0
    hdr = ["kernel", "calls", "total_us" if div == 1 else "us_per_step", "avg_us", "pct", "workgroups", "vgpr",
           "agpr", "scratch"]
    out = []
    for name, n, tot, avg, wg, vg, ag, sc in rows:
        out.append([name[:a.short], n, round(tot / 1e3 / div, 2), round(avg / 1e3, 2), round(100 * tot / total, 2),
                    wg, vg, ag, sc])
    w = csv.writer(sys.stdout)
    w.writerow(hdr)
    for r in out[:a.top]:
        w.writerow(r)
    print(f"# total kernel time {total / 1e6:.3f} ms ({total / 1e6 / div:.3f} ms per step), {len(rows)} kernels")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            cw = csv.writer(f)
            cw.writerow(hdr)
            cw.writerows(out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
