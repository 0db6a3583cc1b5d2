"""Kernel statistics (total / calls / mean / share) from a rocprofv3 rocpd SQLite database (--kernel-trace with the
default output format), for the profiles/ summaries: python scripts/rocpd_stats.py <run_results.db> [top]."""
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rows = db.execute("select name, count(*), sum(end - start) from kernels group by name").fetchall()
    tot = sum(r[2] for r in rows)
    n = sum(r[1] for r in rows)
    print(f"total kernel time {tot / 1e6:.1f} ms over {n} launches")
    for name, calls, t in sorted(rows, key=lambda r: -r[2])[:top]:
        print(f"{t / 1e6:9.1f} ms {calls:7d} {t / calls / 1e3:9.1f} us {100 * t / tot:5.1f}%  {name[:150]}")


if __name__ == "__main__":
    main()
