"""Summarise a rocprofv3 ``--kernel-trace --stats --output-format csv`` run into
``profiles/NAME.md`` (per-kernel table + one steady-state step's timeline) and
``profiles/NAME.csv``.

  python tools/prof_csv_summary.py gpurun_out/prof_val/runc/538_ profiles/NAME "title" STEPS
"""
import csv
import sys


def main():
    base, out, title, steps = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    stats = list(csv.DictReader(open(base + "kernel_stats.csv")))
    stats.sort(key=lambda r: -int(r["TotalDurationNs"]))
    total = sum(int(r["TotalDurationNs"]) for r in stats)
    with open(out + ".csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
        for r in stats:
            w.writerow([r["Name"], r["Calls"], f"{int(r['TotalDurationNs']) / 1e3:.3f}",
                        f"{float(r['AverageNs']) / 1e3:.3f}", f"{float(r['Percentage']):.2f}"])
    trace = list(csv.DictReader(open(base + "kernel_trace.csv")))
    trace.sort(key=lambda r: int(r["Start_Timestamp"]))
    anchors = [i for i, r in enumerate(trace) if "upsample" in r["Kernel_Name"] or "ups_moments" in r["Kernel_Name"]]
    with open(out + ".md", "w") as f:
        f.write(f"# {title}\n\nTotal GPU kernel time: {total / 1e6:.3f} ms over {steps} timed + warmup steps "
                f"(per-kernel calls include warmup)\n\n")
        f.write("| kernel | calls | avg ms | % |\n|---|---|---|---|\n")
        for r in stats:
            f.write(f"| `{r['Name'][:100]}` | {r['Calls']} | {float(r['AverageNs']) / 1e6:.3f} | "
                    f"{float(r['Percentage']):.1f} |\n")
        if len(anchors) >= 2:
            i0, i1 = anchors[-2], anchors[-1]
            t0 = int(trace[i0]["Start_Timestamp"])
            f.write(f"\n## One steady-state step (last full step): "
                    f"{(int(trace[i1]['Start_Timestamp']) - t0) / 1e3:.1f} us\n\n")
            f.write("| start us | dur us | stream | kernel |\n|---|---|---|---|\n")
            for r in trace[i0:i1]:
                s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                f.write(f"| {(s - t0) / 1e3:.1f} | {(e - s) / 1e3:.1f} | {r.get('Stream_Id', '')} | "
                        f"`{r['Kernel_Name'][:70]}` |\n")
    print(open(out + ".md").read()[:3000])


if __name__ == "__main__":
    main()
