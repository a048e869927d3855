"""Summarises profiles/tools/collect_skew.sh output for the c3skew line's dominant class: the
replay kernel's average duration (kernel trace) and HBM bytes per step from the PMC passes
(2 x FETCH_SIZE + WRITE_SIZE, KB = 1024 B; gfx950 FETCH_SIZE counts 64 B per 128-byte read,
profiles/r4/fetch_calibration.json), summed over the class's replay dispatches of the timed
step (the generation's own dispatches are k_generate*, excluded).

    python profiles/tools/summarize_skew.py gpurun_out/prof_skew_<tag> profiles/r6/<name>.json
"""
import csv
import glob
import json
import os
import sys


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    bench = json.load(open(os.path.join(src, "bench.json")))
    cls = bench["per_class"][0]
    stats = {r["Name"]: dict(calls=int(r["Calls"]), avg_ms=float(r["AverageNs"]) / 1e6, pct=float(r["Percentage"]))
             for r in rows(os.path.join(src, "trace", "**", "*kernel_stats.csv"))}
    tot = {}
    for r in rows(os.path.join(src, "pmc*", "**", "*counter_collection.csv")):
        if not r["Kernel_Name"].startswith("void k_replay"):
            continue
        tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    fetch, write = tot.get("FETCH_SIZE"), tot.get("WRITE_SIZE")
    out = {"class": cls["max_ops"], "docs": cls["docs"], "ops": cls["ops"], "kernel_ms_line": cls["kernel_ms"],
           "kernel_stats": stats, "alg_bytes_per_launch": cls["alg_bytes"],
           "hbm_bytes_per_launch": None if fetch is None else (2 * fetch + write) * 1024.0,
           "hbm_bytes_per_launch_raw": None if fetch is None else (fetch + write) * 1024.0}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "kernel_stats"}))


if __name__ == "__main__":
    main()
