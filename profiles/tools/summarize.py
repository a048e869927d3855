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
    hbm = raw = req = None
    if "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
        # FETCH_SIZE doubled: on gfx950 it tallies TCC_EA0_RDREQ x 64 B while the requests are
        # 128 B (MI355X_MICROARCH.md 'HBM'); profiles/tools/fetch_probe.hip measured the same 1/2
        # on this kernel's own page-window read pattern (profiles/r4/fetch_calibration.json)
        hbm = 2 * counters["FETCH_SIZE"] * 1024 + counters["WRITE_SIZE"] * 1024
        raw = counters["FETCH_SIZE"] * 1024 + counters["WRITE_SIZE"] * 1024
    if "TCC_EA0_RDREQ_sum" in counters:
        # cross-check from the request counts: 128 B per read request (32 B ones counted apart),
        # 64 B per 64-byte write request, 32 B per other write request
        rd = counters["TCC_EA0_RDREQ_sum"]
        rd32 = counters.get("TCC_EA0_RDREQ_32B_sum", 0.0)
        wr = counters.get("TCC_EA0_WRREQ_sum", 0.0)
        wr64 = counters.get("TCC_EA0_WRREQ_64B_sum", 0.0)
        req = (rd - rd32) * 128 + rd32 * 32 + wr64 * 64 + (wr - wr64) * 32
    out = dict(bench=bench, kernels=stats, replay_counters_per_step=counters, replay_per_op=per_op,
               hbm_bytes_per_step=hbm, hbm_bytes_per_step_raw=raw, hbm_bytes_per_step_from_requests=req,
               note="counters of every k_replay* dispatch summed per step (LDS-tier launch + hand-over launch);"
                    " hbm_bytes_per_step = 2 x FETCH_SIZE + WRITE_SIZE (gfx950 correction, measured on the"
                    " kernel's read pattern: profiles/r4/fetch_calibration.json); _raw = FETCH_SIZE + WRITE_SIZE;"
                    " _from_requests = TCC_EA0 read / write request counts x their sizes; KB = 1024 B")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(dict(kernels=stats, per_op=per_op, hbm=hbm, hbm_raw=raw, hbm_req=req), indent=1))


if __name__ == "__main__":
    main()
