"""Summarise rocprofv3 ``--pmc ... --output-format csv`` passes into one markdown table.

  python tools/pmc_summary.py OUT.md "title" DURATIONS.csv PASS_DIR [PASS_DIR ...]

Each PASS_DIR is a ``-d`` directory of one counter pass; every ``*counter_collection.csv``
below it is read. Values are averaged per dispatch of each kernel. DURATIONS.csv is a
``tools/prof_csv_summary.py`` per-kernel CSV (kernel, calls, total_us, avg_us, percent);
it supplies the average kernel time, so FETCH_SIZE / WRITE_SIZE (KB) become GB/s of
L2<->HBM traffic.
"""
import collections
import csv
import glob
import os
import sys


def _pass_key(d):
    """A pass is named by its full (normalised) path: two passes may share a leaf name."""
    return os.path.normpath(os.path.abspath(d))


def read_pass(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    spans = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
            # dispatch ids restart per process / agent: key by (file, agent, dispatch)
            key = (path, r.get("Agent_Id", ""), r["Dispatch_Id"])
            spans[key] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    # profiled (serialised) kernel time of this pass, us per dispatch
    per_k = collections.defaultdict(list)
    for k, ns in spans.values():
        per_k[k].append(ns / 1e3)
    for k, v in per_k.items():
        vals[k]["_time_us:" + _pass_key(d)] = v
    return vals


def main():
    out, title, dur_csv, dirs = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4:]
    dur = {r["kernel"]: float(r["avg_us"]) for r in csv.DictReader(open(dur_csv))}
    merged = collections.defaultdict(dict)
    read_cache = {d: read_pass(d) for d in dirs}
    for d in dirs:
        for k, cs in read_cache[d].items():
            for c, v in cs.items():
                merged[k][c] = sum(v) / len(v)
    kernels = sorted(merged, key=lambda k: -dur.get(k, 0.0))
    with open(out, "w") as f:
        f.write(f"# {title}\n\nrocprofv3 --pmc, one pass per counter group ({len(dirs)} passes), "
                "values averaged per dispatch. Kernel time from the kernel-trace run "
                f"(`{dur_csv}`).\n\n")
        for k in kernels:
            if dur.get(k, 0.0) < 20.0:  # skip tiny kernels (< 20 us)
                continue
            cs = merged[k]
            t_us = dur[k]
            f.write(f"## `{k[:110]}`\n\navg time {t_us:.1f} us unprofiled\n\n| counter | value |\n|---|---|\n")
            for c in sorted(cs):
                if not c.startswith("_"):
                    f.write(f"| {c} | {cs[c]:.4g} |\n")
                else:
                    f.write(f"| profiled time us ({c.split(':', 1)[1]}) | {cs[c]:.1f} |\n")
            pt = {c.split(":", 1)[1]: v for c, v in cs.items() if c.startswith("_time_us:")}
            derived = []
            def pass_time(counter):
                for d in dirs:
                    name = _pass_key(d)
                    if name in pt and counter in read_cache[d].get(k, {}):
                        return pt[name]
                return t_us
            if "FETCH_SIZE" in cs:
                derived.append(("HBM read GB/s (FETCH_SIZE KB / profiled time)",
                                cs["FETCH_SIZE"] * 1024 / (pass_time("FETCH_SIZE") * 1e3)))
            if "WRITE_SIZE" in cs:
                derived.append(("HBM write GB/s (WRITE_SIZE KB / profiled time)",
                                cs["WRITE_SIZE"] * 1024 / (pass_time("WRITE_SIZE") * 1e3)))
            if "SQ_VALU_MFMA_BUSY_CYCLES" in cs:
                # summed over the SIMDs (ASSUMED 1024 = 256 CUs x 4), priced at a FIXED 2.4 GHz (the
                # MI355X peak engine clock: an upper bound on the cycles available, so the fraction
                # is a lower bound).  GRBM_GUI_ACTIVE / 8 / time is shown beside it only as a
                # diagnostic: for kernels of a few hundred us it reads 3.0-3.5 GHz (counter skew
                # across the 8 XCDs around short dispatches), which is not a physical clock
                tm = pass_time("SQ_VALU_MFMA_BUSY_CYCLES")
                derived.append(("MFMA busy fraction (MFMA_BUSY / 1024 SIMDs / (profiled time x 2.4 GHz))",
                                cs["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (tm * 1e-6 * 2.4e9)))
                if cs.get("GRBM_GUI_ACTIVE", 0) > 0:
                    ghz = cs["GRBM_GUI_ACTIVE"] / 8 / (pass_time("GRBM_GUI_ACTIVE") * 1e3)
                    derived.append(("diagnostic only: GRBM_GUI_ACTIVE / 8 XCDs / profiled time, GHz", ghz))
            if "SQ_LDS_BANK_CONFLICT" in cs and cs.get("SQ_LDS_IDX_ACTIVE", 0) > 0:
                derived.append(("LDS bank-conflict cycles / LDS active", cs["SQ_LDS_BANK_CONFLICT"] / cs["SQ_LDS_IDX_ACTIVE"]))
            for name, v in derived:
                f.write(f"| *{name}* | {v:.3g} |\n")
            f.write("\n")


if __name__ == "__main__":
    main()
