"""bench.py --config c3skew: the C3 job (10^9 messages over 100k documents) with Zipf-skewed
document lengths (fluidframework_amd/skew.py; SURVEY.md section 7 hard part 5, 8e).

Documents are sharded by message count (skew.shard_range_ops), grouped into size classes on
every rank, and each class is replayed by its own handle -- capacities sized for its longest
document, its own HIP stream -- with the class of the longest documents launched first; inside
each batch the library dispatches documents longest first (mt_batch order).  The step is the
whole rank's job: every class reset + applied, then every class synchronised.  Inputs are
generated on the GPU (untimed, mt_generate_docs) and stay resident in HBM.
"""
import os
import sys
import time

import numpy as np


def class_caps(bench, cfg, max_ops):
    """Capacities of the handle of a size class, sized for its longest document from the C3
    high-water marks (183 pages, ~3.5k live segments, ~11k live text units at 10k messages:
    pages and segments grow with the length, the unsettled table and the heap with the
    collaboration window).  Classes up to 10k messages keep the C3 bench's tight tier (its LDS
    capacities fixed at compile time; the HBM pages must hold its 192); longer ones run the
    full-capacity paged tier at their own capacities."""
    caps = bench.capacities(dict(cfg, ops=10000))
    text = 4096
    while text < 2.5 * max_ops:
        text *= 2
    uid = 1 << 15
    while uid < 4 * max_ops:
        uid *= 2
    # pages: the measured peaks are 0.0154-0.0161 per message above 10k (c3skew: 3080 at 200k,
    # 1496 at 100k, 629 at 40k, 323 at 20k); 200k -> 3200 pages (a document that still outgrows
    # it moves to the growth step's region by itself)
    pages = max(192, int(max_ops * 0.0155) + 100)
    caps.update(page_capacity=pages, text_capacity=text,
                props_capacity=int(0.3 * max_ops) + 512, uid_capacity=min(uid, 1 << 20))
    if max_ops > 10000:
        for k in ("lds_page_capacity", "lds_unsettled_capacity", "lds_page_heap_capacity", "lds_narrow_overlap"):
            caps.pop(k, None)
        # unsettled table / heap at the measured peaks plus a margin (c3skew classes above 10k
        # messages: <= 194 / 181; the growth step takes a document past them -- none on the
        # bench's streams, profiles/r5/bench_c3skew_r5t.json): with the page metadata in HBM
        # (>= 512 pages, mt_replay.hip use_hm) a 200k-message document takes 21.7 KB of LDS,
        # 7 per CU, a 100k one 16.3 KB, 10 per CU (profiles/tools/lds_footprint.py 1650 216 200 8 1)
        caps.update(unsettled_capacity=216, page_heap_capacity=200)
    return caps


def _calibration_for(bench, max_ops):
    """(case name, port-over-reference ratio without a callback) of the calibration case whose
    document length matches a size class (oracle/calibrate.py; the reference cannot travel)."""
    import json
    try:
        cal = json.load(open(bench.CALIBRATION))
    except (OSError, ValueError):
        return None
    best = None
    for name, c in cal.items():
        if not (isinstance(c, dict) and name.startswith("c3")):
            continue
        d = abs(np.log(c["ops_per_doc"] / max_ops))
        if best is None or d < best[0]:
            best = (d, name, c["ratio_port_over_reference_nocb"])
    return None if best is None else (best[1], best[2])


def run_skew(args, cfg, rank, world, local_rank, dist, bench):
    from fluidframework_amd import MergeTreeBatch
    from fluidframework_amd.skew import shard_range_ops, size_classes, zipf_lengths
    total_docs = cfg["docs"]
    lens_all = zipf_lengths(total_docs, total_docs * cfg["ops"], cfg["zipf_s"], cfg["max_ops"], cfg["lens_seed"])
    lo, hi = shard_range_ops(lens_all, world, rank)
    ids = np.arange(lo, hi, dtype=np.int32)
    lens = lens_all[lo:hi]
    classes = size_classes(lens, cfg["classes"])
    if args.skew_classes:
        keep = {int(x) for x in args.skew_classes.split(",")}
        classes = [(b, i) for b, i in classes if b in keep]
    t_gen = time.time()
    runs = []
    for max_ops, idx in classes:        # longest class first
        mt = MergeTreeBatch(len(idx), device=local_rank, **class_caps(bench, cfg, max_ops))
        prio = getattr(args, "skew_priority", 0)
        if prio and not runs:
            mt.set_stream_priority(1)       # the longest class: its waiting documents go first
        elif prio >= 2 and max_ops <= 10000:
            mt.set_stream_priority(-1)
        ccfg = dict(cfg, ops=int(max_ops))
        batch = mt.generate(ccfg, ops_per_doc=lens[idx], doc_ids=ids[idx])
        gsum = mt.checksums()
        so, sd = mt.generated_seeds(ccfg, doc_ids=ids[idx])
        mt.load_initial_text(so, sd)
        runs.append(dict(max_ops=max_ops, idx=idx, mt=mt, batch=batch, gen=gsum, ops=int(lens[idx].sum()),
                         cfg=ccfg))
        print(f"c3skew: class <= {max_ops}: {len(idx)} documents, {runs[-1]['ops']} messages generated "
              f"({time.time() - t_gen:.1f} s)", file=sys.stderr, flush=True)
    t_gen = time.time() - t_gen

    def step():
        for r in runs:
            r["mt"].reset()
            r["batch"].apply_async()
            if args.skew_serial:
                r["mt"].sync()
        for r in runs:
            r["mt"].sync()

    for _ in range(args.warmup):
        step()

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step()
        print(f"c3skew: step {k + 1}: {time.perf_counter() - t0:.2f} s", file=sys.stderr, flush=True)
    barrier()
    elapsed = time.perf_counter() - t0
    n_ops = int(sum(r["ops"] for r in runs))
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        t = torch.tensor([n_ops], dtype=torch.int64, device="cuda")
        dist.all_reduce(t)
        total_ops = int(t.item())
    else:
        total_ops = n_ops
    ok = True
    per_class = []
    for r in runs:
        st = r["mt"].status()
        sums = r["mt"].checksums()
        same = bool(np.array_equal(sums, r["gen"])) and int((st != 0).sum()) == 0
        ok = ok and same
        # algorithmic bytes of the class's replay (SURVEY 8d B_op, as bench.run_replay): op
        # records + result records + inserted UTF-16 units (a generated batch's text arena holds
        # exactly the insert payloads) + the final state write-back
        n, t, p = r["batch"].sizes()
        alg = (n * (bench.OP_BYTES + bench.RESULT_BYTES) + 2 * t +
               int(sums["n_segments"].astype(np.int64).sum()) * bench.SEG_BYTES +
               2 * int(sums["length"].astype(np.int64).sum()))
        per_class.append(dict(max_ops=r["max_ops"], docs=int(len(r["idx"])), ops=r["ops"],
                              kernel_ms=round(float(r["mt"].last_kernel_ms()), 1), alg_bytes=alg,
                              replay_equals_generation=same, grown=r["mt"].last_grown(),
                              peaks=r["mt"].last_paged_peaks()))
    # the dominant class -- the most messages (the longest documents: the 200k class carries a
    # third of the job) -- its roofline.  (Not the longest kernel time: the classes share the
    # GPU, and a short class's launch can end last while it waited for CUs.)
    dom = max(per_class, key=lambda c: c["ops"])
    achieved = dom["alg_bytes"] / (dom["kernel_ms"] / 1000.0) if dom["kernel_ms"] > 0 else 0.0
    # measured HBM traffic of the dominant class's replay (profiles/tools/collect_skew.sh: rocprofv3
    # FETCH_SIZE / WRITE_SIZE passes over that class alone, 2 x FETCH_SIZE + WRITE_SIZE per step)
    traffic = traffic_raw = None
    try:
        import json
        pm = json.load(open(bench.PROFILE_PMC)).get("c3skew", {})
        if pm.get("class") == dom["max_ops"] and pm.get("docs") == dom["docs"] and pm.get("ops") == dom["ops"]:
            traffic, traffic_raw = pm.get("hbm_bytes_per_launch"), pm.get("hbm_bytes_per_launch_raw")
    except (OSError, ValueError):
        pass
    roofline = {"bound": "hbm", "achieved": round(achieved / 1e9, 3), "peak": bench.HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": achieved / bench.HBM_PEAK, "traffic": traffic, "traffic_raw": traffic_raw,
                "kernel": f"k_replay_paged (class <= {dom['max_ops']} messages, its own stream)",
                "kernel_ms": dom["kernel_ms"], "alg_bytes_per_launch": dom["alg_bytes"]}
    # oracle sample and CPU baseline (rank 0): per size class, a sample of >= 16 x threads
    # documents spread over the class's length distribution (its longest included), generated
    # by the CPU restatement on parallel host threads (its generator replays them: their
    # checksums are the check against the GPU's), then replayed again from their op records,
    # timed class by class with every thread busy (documents taken longest first as threads
    # free up).  The job's CPU time is each class's messages at its own rate, summed.
    mism, sampled, cpu = 0, 0, None
    if rank == 0 and not args.no_cpu:
        from concurrent.futures import ThreadPoolExecutor
        sys.path.insert(0, os.path.join(bench.REPO, "oracle"))
        import pyoracle
        threads = args.cpu_threads or bench.host_cores()
        per = max(16 * threads, 32)
        picks = []   # (class, position in the class, document)
        for ri, r in enumerate(runs):
            srt = np.argsort(lens[r["idx"]], kind="stable")
            m = min(len(srt), per)
            sel = sorted({int(srt[q]) for q in np.linspace(0, len(srt) - 1, m).round().astype(int)})
            picks += [(ri, j, int(r["idx"][j])) for j in sel]
        t_o = time.time()

        def gen(pk):
            _, _, d = pk
            g = pyoracle.generate(dict(cfg, ops=int(lens[d])), int(ids[d]), keep=True)
            g["sum"] = g.pop("doc").outputs()["checksum"]
            return g

        order = sorted(range(len(picks)), key=lambda k: -int(lens[picks[k][2]]))   # longest first
        with ThreadPoolExecutor(max(1, threads)) as ex:
            gens = dict(zip(order, ex.map(gen, [picks[k] for k in order])))
        print(f"c3skew: oracle generated {len(picks)} sample documents ({time.time() - t_o:.1f} s)",
              file=sys.stderr, flush=True)
        for k, (ri, j, d) in enumerate(picks):
            got = runs[ri]["mt"].checksums()[j]
            osum = gens[k]["sum"]
            sampled += 1
            mism += int(any(got[f] != osum[f] for f in ("length", "text_hash", "props_hash", "delta_hash")))
        classes_cpu = []
        t_job = 0.0
        for ri, r in enumerate(runs):
            ks = sorted((k for k in range(len(picks)) if picks[k][0] == ri), key=lambda k: -int(lens[picks[k][2]]))
            ops, text, props, seed, doc_off, seed_off = [], [], [], [], [0], [0]
            tb = pb = 0
            for k in ks:
                g = gens[k]
                o = g["ops"].copy()
                ins = o["kind"] == 0
                o["payload"][ins] += tb
                hp = o["props"] != 0xFFFFFFFF
                o["props"][hp] += pb
                ops.append(o)
                text.append(g["text"])
                props.append(g["props"])
                seed.append(g["seed"])
                tb += len(g["text"])
                pb += len(g["props"])
                doc_off.append(doc_off[-1] + len(o))
                seed_off.append(seed_off[-1] + len(g["seed"]))
            arrays = dict(ops=np.concatenate(ops), text=np.concatenate(text), props=np.concatenate(props),
                          seed=np.concatenate(seed), doc_off=np.asarray(doc_off, dtype=np.int64),
                          seed_off=np.asarray(seed_off, dtype=np.int64))
            t_c = time.perf_counter()
            osums, ost = pyoracle.replay_batch(arrays, threads=threads)
            t_c = time.perf_counter() - t_c
            mism += int(sum(osums[q] != gens[k]["sum"] for q, k in enumerate(ks)) + (ost != 0).sum())
            n_c = int(doc_off[-1])
            rate = n_c / t_c
            t_job += r["ops"] / rate
            cal = _calibration_for(bench, r["max_ops"])
            classes_cpu.append(dict(max_ops=r["max_ops"], docs=len(ks), messages=n_c, seconds=round(t_c, 3),
                                    ops_per_s=round(rate, 1),
                                    reference_estimate=(round(rate / cal[1], 1) if cal else None),
                                    calibration=(cal[0] if cal else None)))
            print(f"c3skew: CPU class <= {r['max_ops']}: {len(ks)} documents, {n_c} messages, {t_c:.2f} s "
                  f"({rate / 1e6:.2f} M ops/s)", file=sys.stderr, flush=True)
        total_job = int(sum(r["ops"] for r in runs))
        value_cpu = total_job / t_job
        t_ref = sum(r["ops"] / c["reference_estimate"] for r, c in zip(runs, classes_cpu) if c["reference_estimate"])
        ref_ok = all(c["reference_estimate"] for c in classes_cpu)
        cpu = dict(value=round(value_cpu, 1), unit="ops/s", cores=threads, kind="port", host_cpus=os.cpu_count(),
                   sample=f"oracle/mt_oracle.c replay, class by class, of {sampled} documents (>= {per} per class "
                          f"or the whole class, spread over its lengths, longest included) on {threads} host "
                          f"threads; the job's CPU time = each class's messages at its measured rate",
                   per_class=classes_cpu,
                   reference_estimate=(dict(value=round(total_job / t_ref, 1), unit="ops/s", cores=threads,
                                            how="each class's port rate / the port-over-reference ratio measured "
                                                "at its length (profiles/r6/cpu_calibration.json: transpiled "
                                                "reference MergeTree, observer without a delta callback, under "
                                                "Node, one thread each), combined like the port's")
                                       if ref_ok else None))
    if dist is not None:
        import torch
        t = torch.tensor([1 if ok else 0], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        ok = bool(t.item())
    if rank != 0:
        return None
    value = total_ops * args.steps / elapsed
    line = {"metric": "sequenced merge-tree ops applied/sec (node) at 100k docs; bit-exact text+props", "value": round(value, 1), "unit": "ops/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1000.0 / args.steps, 3), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "int32", "data": "synthetic (device generator, Zipf lengths)",
            "config": {"workload": "c3skew", "docs_total": total_docs, "ops_total": int(lens_all.sum()),
                       "zipf_s": cfg["zipf_s"], "max_ops": cfg["max_ops"], "classes": cfg["classes"],
                       "median_ops": int(np.median(lens_all)), "docs_at_max": int((lens_all == cfg["max_ops"]).sum()),
                       "parallelism": f"dp{world} (op-balanced shards)"},
            "roofline": roofline, "cpu_baseline": cpu,
            "parity": {"replay_equals_generation": ok, "oracle_docs": sampled, "oracle_mismatches": mism},
            "per_class": per_class, "gen_s": round(t_gen, 1)}
    return line
