"""Summarises profiles/tools/collect.sh output: per-kernel average duration from the kernel
trace, SQ counters per replayed op, and HBM bytes per launch from FETCH_SIZE/WRITE_SIZE
(gfx950: FETCH_SIZE doubled, MI355X_MICROARCH.md 'HBM'; both reported in KB = 1024 B).

    python profiles/tools/summarize.py gpurun_out/prof_<tag> profiles/<round>/<name>.json
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
    ops = bench["config"]["ops_per_step"]
    stats = {r["Name"]: dict(calls=int(r["Calls"]), avg_ms=float(r["AverageNs"]) / 1e6,
                              pct=float(r["Percentage"]))
             for r in rows(os.path.join(src, "trace", "**", "*kernel_stats.csv"))}
    counters, steps = {}, {}
    for r in rows(os.path.join(src, "pmc*", "**", "*counter_collection.csv")):
        # one step = the LDS-tier launch + (paged / HBM tier) hand-over launch; all replay
        # kernels are summed and divided by the number of LDS-tier dispatches
        if not r["Kernel_Name"].startswith("void k_replay"):
            continue
        counters[r["Counter_Name"]] = counters.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        if "k_replay<TierLdsT" in r["Kernel_Name"]:
            steps.setdefault(r["Counter_Name"], set()).add(r["Dispatch_Id"])
    counters = {k: v / max(len(steps.get(k, ())), 1) for k, v in counters.items()}
    per_op = {k: v / ops for k, v in counters.items() if k.startswith("SQ_INSTS") or k.startswith("SQ_WAIT")
              or k in ("SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_LDS_BANK_CONFLICT",
                       "SQ_LDS_IDX_ACTIVE", "SQ_ACTIVE_INST_VALU")}
    hbm = None
    if "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
        hbm = 2 * counters["FETCH_SIZE"] * 1024 + counters["WRITE_SIZE"] * 1024
    out = dict(bench=bench, kernels=stats, replay_counters_per_step=counters, replay_per_op=per_op,
               hbm_bytes_per_step=hbm,
               note="counters of every k_replay* dispatch summed per step (LDS-tier launch + hand-over launch);"
                    " FETCH_SIZE doubled per the gfx950 correction; KB = 1024 B")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(dict(kernels=stats, per_op=per_op, hbm=hbm), indent=1))


if __name__ == "__main__":
    main()
