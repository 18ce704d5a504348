"""Per-kernel summary of a rocprofv3 --kernel-trace SQLite output (rocpd):
calls, average / total microseconds; optional name filter."""
import glob
import sqlite3
import sys


def main(path, pat=None, per=None):
    dbs = glob.glob(path + "/**/*.db", recursive=True) if not path.endswith(".db") else [path]
    c = sqlite3.connect(dbs[0])
    q = "select name, count(*), avg(end-start)/1000.0, sum(end-start)/1000.0 from kernels"
    if pat:
        q += f" where name like '%{pat}%'"
    q += " group by name order by sum(end-start) desc"
    rows = c.execute(q).fetchall()
    for name, n, avg, tot in rows[:40]:
        extra = f"  {tot / per:9.2f} us/step" if per else ""
        print(f"{n:6d} {avg:10.2f} us avg {tot:12.1f} us total{extra}  {name[:100]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] != "-" else None,
         float(sys.argv[3]) if len(sys.argv) > 3 else None)
