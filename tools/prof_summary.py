"""Summarise a rocprofv3 ``--kernel-trace`` database (rocpd SQLite) into a
markdown table + CSV for ``profiles/``.

  python tools/prof_summary.py gpurun_out/prof_c1/run_results.db profiles/NAME "title" [steps]
"""
import csv
import sqlite3
import sys


def main():
    db, out, title = sys.argv[1], sys.argv[2], sys.argv[3]
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else None
    c = sqlite3.connect(db)
    rows = list(c.execute("SELECT name, total_calls, total_duration, average, percentage FROM top_kernels "
                          "ORDER BY total_duration DESC"))
    total_us = sum(r[2] for r in rows)
    with open(out + ".csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
        for r in rows:
            w.writerow([r[0], r[1], f"{r[2]:.3f}", f"{r[3]:.3f}", f"{r[4]:.2f}"])
    with open(out + ".md", "w") as f:
        f.write(f"# {title}\n\n")
        f.write(f"Total GPU kernel time: {total_us / 1e3:.3f} ms")
        if steps:
            f.write(f" over {steps} steps = {total_us / 1e3 / steps:.3f} ms/step")
        f.write("\n\n| kernel | calls | avg ms | per-step ms | % |\n|---|---|---|---|---|\n")
        for name, calls, tot, avg, pct in rows:
            per = f"{tot / 1e3 / steps:.3f}" if steps else ""
            f.write(f"| `{name[:100]}` | {calls} | {avg / 1e3:.3f} | {per} | {pct:.1f} |\n")
    print(open(out + ".md").read())


if __name__ == "__main__":
    main()
