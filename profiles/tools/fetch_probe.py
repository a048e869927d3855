"""Puts fetch_probe's known byte counts next to the PMC counters it ran under (fetch.sh):
per probe kernel, FETCH_SIZE (KB = 1024 B) and TCC_EA0_RDREQ against the bytes the lanes
requested and the bytes of the distinct 64 B / 128 B lines they touched.

    python3 profiles/tools/fetch_probe.py gpurun_out/fp > profiles/r4/fetch_calibration.json
"""
import csv
import glob
import json
import os
import sys


def counters(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            out.setdefault(k, {})
            out[k][r["Counter_Name"]] = out[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def main():
    d = sys.argv[1]
    exp = [json.loads(x) for x in open(os.path.join(d, "expected.jsonl"))]
    c = counters(os.path.join(d, "p1"))
    c2 = counters(os.path.join(d, "p2"))
    rows = []
    for e in exp:
        k = e["kernel"]
        f = c.get(k, {}).get("FETCH_SIZE", 0.0) * 1024
        rq = c2.get(k, {}).get("TCC_EA0_RDREQ_sum", 0.0)
        rows.append(dict(kernel=k, requested_bytes=e["requested"], lines64_bytes=e["lines64"],
                         lines128_bytes=e["lines128"], fetch_size_bytes=f, rdreq=rq,
                         fetch_over_lines128=round(f / e["lines128"], 4) if e["lines128"] else None,
                         rdreq_x128_over_lines128=round(rq * 128 / e["lines128"], 4) if e["lines128"] else None))
    print(json.dumps(dict(
        rows=rows,
        note="FETCH_SIZE = TCC_EA0_RDREQ x 64 B while each read request moves a 128-byte line: the "
             "reported bytes are 1/2 of the lines fetched, for the wide stream and for the paged "
             "window's 22-slot page reads alike (k_pages) -- the x2 correction applies to this "
             "kernel's page traffic; short scattered reads (k_probe16, k_text8) are fetched as whole "
             "lines too (see rdreq)"), indent=1))


if __name__ == "__main__":
    main()
