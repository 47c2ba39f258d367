"""Print a per-step kernel timeline (start offset, duration, queue) from a rocprofv3
--kernel-trace database: shows what is on the critical path and what overlaps.

  python tools/timeline.py gpurun_out/prof_x/run_results.db [first_kernel_substring] [n_steps]
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "upsample"
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    qcol = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else None)
    rows = list(c.execute(f"select name, start, end, {qcol or 0} from kernels order by start"))
    starts = [i for i, r in enumerate(rows) if anchor in r[0]]
    if len(starts) < nsteps + 1:
        print("not enough steps found")
        return
    i0, i1 = starts[-nsteps - 1], starts[-1]
    t0 = rows[i0][1]
    busy_end = t0
    for name, s, e, q in rows[i0:i1]:
        gap = max(0, s - busy_end)
        busy_end = max(busy_end, e)
        print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap / 1e3:6.1f}  q{q}  {name[:70]}")
    print(f"steps: {nsteps}, wall {(rows[i1][1] - t0) / 1e6 / nsteps:.3f} ms/step")


if __name__ == "__main__":
    main()
