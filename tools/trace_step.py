"""One step of a rocprofv3 kernel trace as a markdown table (start / duration / stream / kernel),
steps delimited by a marker kernel (default: the input op, ups_moments_u8).
Usage: python tools/trace_step.py TRACE.csv STEP [MARKER] >> profiles/X.md"""
import csv
import sys


def main():
    path, k = sys.argv[1], int(sys.argv[2])
    marker = sys.argv[3] if len(sys.argv) > 3 else "ups_moments"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ups = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    seg = rows[ups[k]:ups[k + 1]]
    t0 = int(seg[0]["Start_Timestamp"])
    period = (int(rows[ups[k + 1]]["Start_Timestamp"]) - t0) / 1e3
    print(f"## Step {k} of the trace: {period:.1f} us (next step's first kernel at that offset)\n")
    print("| start us | dur us | stream | kernel |\n|---|---|---|---|")
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"| {(s - t0) / 1e3:.1f} | {(e - s) / 1e3:.1f} | {r['Stream_Id']} | `{r['Kernel_Name'][:70]}` |")


if __name__ == "__main__":
    main()
