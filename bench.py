#!/usr/bin/env python3
"""Benchmark: sequenced merge-tree ops applied per second on MI355X (BASELINE.json metric).

One *step* = replaying one batch of synthetic sequenced messages through the observer
replicas of every document on the GPU (Client.applyMsg semantics, bit-exact with the
reference), starting from the documents' initial contents.  The default workload is the
one the metric is quoted on, BASELINE.json configs[2] (C3: 100k documents x 10k ops,
8 writers, refSeq lag <= 64, insert 0.5 / remove 0.3 / annotate 0.2 with property sets):
the fixed 100k-document job is sharded over the ranks (contiguous shards,
fluidframework_amd.shard.shard_range), so N=1 replays all 100k documents on one GPU and
N=8 gives every GPU a 12.5k-document shard (strong scaling; documents are independent, so
there is no data-path collective).  The only collective is an RCCL all-gather of
per-document checksums after the timed region.  `--docs D` instead gives every rank D
documents (weak scaling), `--shard r` replays shard r of the 8-way split on one GPU, and
`--config c2` runs configs[1] (10k documents x 2k insert/remove ops per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3] [--docs D] [--ops O]

Inputs are generated on the GPU (untimed) and stay resident in HBM; the timed region is
reset + replay kernels only.  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK = 8.0e12          # MI355X_MICROARCH.md: HBM3E 8 TB/s
SEG_BYTES = 40             # segA 16 + segO 8 + segB 16
OP_BYTES = 32              # mt_op_rec
RESULT_BYTES = 16          # per-op result record (position, length) in B_op
PROFILE_PMC = os.path.join(REPO, "profiles", "pmc_summary.json")
CALIBRATION = os.path.join(REPO, "profiles", "r6", "cpu_calibration.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--docs", type=int, default=0,
                    help="documents per GPU (weak scaling; default: the config's whole job sharded over the ranks)")
    ap.add_argument("--ops", type=int, default=0, help="ops per document (default: config)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0 = every core this process may use)")
    ap.add_argument("--cpu-sample-docs", type=int, default=0, help="0 = all docs of rank 0")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-ingest", action="store_true", help="skip the encode / H2D upload rates")
    ap.add_argument("--lds-cap", type=int, default=0, help="segments per document in the LDS tier (0 = default)")
    ap.add_argument("--seg-cap", type=int, default=0, help="flat HBM segments per document (0 = default; sweeps)")
    ap.add_argument("--skew-classes", default="",
                    help="c3skew: replay only these size classes (comma-separated bounds; diagnostics)")
    ap.add_argument("--skew-priority", type=int, default=0,
                    help="c3skew: the longest class's stream at the device's highest priority (1), the "
                         "shortest classes' at its lowest (2: both), 0 none")
    ap.add_argument("--skew-serial", action="store_true",
                    help="c3skew: run the size classes one after another instead of concurrently")
    ap.add_argument("--heap-cap", type=int, default=0, help="zamboni heap entries per document (0 = default)")
    ap.add_argument("--shard", type=int, default=-1,
                    help="replay shard r of the 8-way split of the config's job on this one GPU")
    ap.add_argument("--page-caps", default="", help="paged layout LDS capacities 'pages,unsettled,heap' (sweeps)")
    ap.add_argument("--paged-slices", type=int, default=0,
                    help="mt_options.paged_slices for paged configs (0 = off; see include/mt_replay.h)")
    ap.add_argument("--verify-per-rank", type=int, default=4,
                    help="N > 1: documents of every rank's shard re-derived by the CPU oracle on rank 0")
    return ap.parse_args()


def progress(rank, msg):
    """A progress line on stderr (rank 0): long runs write something every few seconds."""
    if rank == 0:
        print(f"bench: {msg}", file=sys.stderr, flush=True)


def host_cores():
    """CPUs this process may run on: the affinity mask, capped by a cgroup CPU quota (a GPU
    box shows the whole machine in os.cpu_count() but grants a share of it)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def launch(args):
    """`--gpus N` without a torch.distributed launcher: start N ranks (one process per GPU)
    through torch.distributed.run as a child process -- before this process touches the GPU
    -- and exit with its status.  Rank 0 prints the JSON line."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def oracle_checksums(cfg, global_docs, threads):
    """mt_checksum of each generated document re-derived on the CPU by the oracle (the
    checker: oracle/mt_oracle.c generates the same stream and replays it)."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    from fluidframework_amd.wire import CHECKSUM_DTYPE

    def one(d):
        g = pyoracle.generate(cfg, int(d), keep=True)
        return g["doc"].outputs()["checksum"]

    out = np.zeros(len(global_docs), dtype=CHECKSUM_DTYPE)
    with ThreadPoolExecutor(max(1, threads)) as ex:
        for i, cs in enumerate(ex.map(one, global_docs)):
            out[i] = cs
    return out


def verify_shards(dist, rank, world, n_total, cfg, local, gen_sums, device, per_rank, threads):
    """The multi-GPU exchange step and its check.  Rank r owns the global documents
    shard_range(n_total, world, r).  Every rank's replay checksums (`local`: a uint8 tensor
    filled on the device, or a CHECKSUM_DTYPE array) and generation checksums are
    all-gathered (RCCL over xGMI with backend nccl); rank 0 then checks that the timed
    replay reproduced the generation for every document of every shard, and that
    `per_rank` documents of every shard equal the CPU oracle's replay of the same global
    documents.  Returns the report on rank 0, None elsewhere."""
    from fluidframework_amd.shard import digest, gather_checksums, shard_range
    got = gather_checksums(local, dist, device=device, n_total=n_total)
    gen = gather_checksums(gen_sums, dist, device=device, n_total=n_total)
    if rank != 0:
        return None
    gdocs = []
    for r in range(world):
        lo, hi = shard_range(n_total, world, r)
        if hi > lo:
            gdocs += sorted({lo + int(x) for x in np.linspace(0, hi - lo - 1, num=max(1, min(per_rank, hi - lo)))})
    orc = oracle_checksums(cfg, gdocs, threads) if per_rank > 0 else None
    mism = int(sum(got[g] != orc[j] for j, g in enumerate(gdocs))) if orc is not None else None
    return dict(docs_gathered=int(len(got)), replay_equals_generation=bool(np.array_equal(got, gen)),
                oracle_docs=len(gdocs) if orc is not None else 0, oracle_mismatches=mism,
                digest=digest(got))


def shard_plan(args, cfg, world, rank):
    """(documents on this rank, first global document, documents in the whole job,
    scaling).  Default: the config's whole job split over the ranks (strong scaling; C2 is
    a single-GPU configuration, so it stays per GPU); `--docs D`: D per rank (weak);
    `--shard r`: shard r of the job's 8-way split, on one GPU."""
    from fluidframework_amd.shard import shard_range
    if args.docs:
        return args.docs, rank * args.docs, args.docs * world, "weak"
    if args.config == "c2":
        return cfg["docs"], rank * cfg["docs"], cfg["docs"] * world, "weak"
    total = cfg["docs"] if args.config == "c3" else min(cfg["docs"], 16384)
    if args.shard >= 0:
        lo, hi = shard_range(total, 8, args.shard)
        return hi - lo, lo, hi - lo, "weak"
    lo, hi = shard_range(total, world, rank)
    return hi - lo, lo, total, "strong"


def capacities(cfg, tight=True):
    """Per-document capacities sized for the workload (DESIGN.md 'HBM layout').  The paged
    capacities (page / unsettled / page heap) size the HBM arrays and the full-capacity paged
    tier; with `tight`, smaller LDS capacities run first (lds_*: more documents per CU) and
    the library hands any document that could outgrow them to the full tier by itself."""
    if cfg["writers"] > 8 or cfg["lag"] > 64 or cfg["p_insert_props"] > 0 or cfg["ops"] > 4000:
        # annotate keeps segments apart (property sets differ): ~0.4 live segments per op.
        # Documents outgrow the LDS tier early and continue in the paged layout; the flat
        # HBM arrays only hold what the LDS tier spills.
        segs = max(1024, int(cfg["ops"] * 0.5) + 512)
        deep = cfg["lag"] > 64
        caps = dict(seg_capacity=256, text_capacity=1 << 16, heap_capacity=512, props_capacity=segs + 256,
                    # high-water marks (mt_last_paged_peaks) at 10k ops: C3 183 pages, 208
                    # table entries, 173 heap entries (all 100k documents); C4 (minSeq ~1k ops
                    # behind) far more
                    page_capacity=max(64, segs // 20 if not deep else segs // 14),
                    page_heap_capacity=2560 if deep else 512,
                    unsettled_capacity=2560 if deep else 320,
                    uid_capacity=1 << 16)
        if tight and deep and cfg["ops"] <= 10000 and cfg["writers"] <= 64:
            # C4 peaks over 4096 documents: 208 pages, 1810 table entries, 841 heap entries;
            # 99 KB per document at the full capacities (1 per CU); the tight tier packs its
            # table (12-byte entries: every client id fits 8 bits): 52.8 KB here, 3 per CU
            caps.update(lds_page_capacity=224, lds_unsettled_capacity=1900, lds_page_heap_capacity=900)
        if tight and not deep and cfg["ops"] <= 10000:
            # the paged layout's LDS footprint sets documents per CU: 27 KB at the full
            # capacities (6 per CU), 13.1 KB here (12 per CU; the tight tier is compiled for 3
            # waves/SIMD, the run-time-capacity tiers for 2: mt_kernels.h paged_waves)
            caps.update(lds_page_capacity=192, lds_unsettled_capacity=220, lds_page_heap_capacity=192,
                        lds_narrow_overlap=1 if cfg["writers"] <= 32 else 0)
        return caps
    # C2: documents stay in the LDS tier (<= ~100 live segments): a flat-only handle
    return dict(seg_capacity=512, text_capacity=1 << 15, heap_capacity=1024, props_capacity=512 + 128,
                page_capacity=-1)


def _decode_slice(chunk_list):
    """Worker: SnapshotLoader's host half for a slice of summaries -- JSON chunks parsed and
    specToSegment'ed into mt_seg_rec records (snapshot.decode_chunks + SnapshotBatch)."""
    from fluidframework_amd.snapshot import SnapshotBatch, decode_chunks
    from fluidframework_amd.wire import Interner
    sb = SnapshotBatch(Interner(synthetic=True))
    for ch in chunk_list:
        sb.add_doc(decode_chunks(ch))
    a = sb.arrays()
    return len(chunk_list), int(len(a["segs"]))


def c5_decode_rate(counts, recs, text, props, mn, cu, chunk, n_sample, threads):
    """Summary decode as its own line: the sample's summaries are emitted as SnapshotV1 JSON
    chunks (untimed), then decoded back to device records on the host cores (timed).  The
    device load (mt_snapshots_load_async) starts from records; this is the step before it."""
    from concurrent.futures import ProcessPoolExecutor
    from fluidframework_amd.snapshot import encode_chunks, record_specs
    from fluidframework_amd.wire import Interner
    it = Interner(synthetic=True)
    c = np.asarray(counts, dtype=np.int64)
    r0 = np.concatenate([[0], np.cumsum(c[:, 0])])
    t0 = np.concatenate([[0], np.cumsum(c[:, 1])])
    p0 = np.concatenate([[0], np.cumsum(c[:, 2])])
    names = {i: f"client-{i}" for i in range(-2, 4096)}
    docs = []
    for d in range(n_sample):
        rs = recs[r0[d]:r0[d + 1]]
        specs, lengths = record_specs(rs, text[t0[d]:t0[d + 1]], props[p0[d]:p0[d + 1]], it, names)
        docs.append(encode_chunks(specs, lengths, int(mn[d]), int(cu[d]), chunk))
    nbytes = sum(len(v) for ch in docs for v in ch.values())
    per = -(-len(docs) // threads)
    parts = [docs[i:i + per] for i in range(0, len(docs), per)]
    with ProcessPoolExecutor(len(parts)) as ex:
        list(ex.map(_decode_slice, parts[:1]))          # warm the workers' imports
        t = time.perf_counter()
        done = list(ex.map(_decode_slice, parts))
        t = time.perf_counter() - t
    n = sum(x[0] for x in done)
    py = dict(value=round(n / t, 1), unit="docs/s", cores=len(parts), kind="port",
              sample=f"{n} summaries ({nbytes / 1e6:.1f} MB of chunk JSON, {sum(x[1] for x in done)} segment specs) "
                     f"decoded by fluidframework_amd/snapshot.py on {len(parts)} host processes, {t:.2f} s")
    # the native decoder (include/mt_snapshot.h) on the same blobs: bytes in, mt_seg_rec out
    from fluidframework_amd.snapdec import SummaryDecoder
    dec = SummaryDecoder(Interner(synthetic=True), threads=threads)
    packed = dec.pack(docs)
    dec.decode_packed(*packed)                          # warm (page in, allocator)
    reps = 3
    t = time.perf_counter()
    for _ in range(reps):
        out, _ = dec.decode_packed(*packed)
    t = (time.perf_counter() - t) / reps
    return dict(value=round(len(docs) / t, 1), unit="docs/s", cores=threads, kind="native",
                mb_per_s=round(nbytes / t / 1e6, 1),
                sample=f"{len(docs)} summaries ({nbytes / 1e6:.1f} MB of chunk JSON, {len(out['segs'])} segment specs) "
                       f"decoded by libmtsnapdec.so on {threads} host threads, {t * 1e3:.1f} ms (mean of {reps})",
                python_restatement=py)


def c5_end_to_end(mt, counts, recs, text, props, mn, cu, chunk, tail_arr, tail, sums, status, n_emit, threads,
                  slice_docs=16384):
    """Cold catch-up end to end, from summary JSON bytes to replayed tails, for every document
    of the handle: MergeTreeBatch.catch_up (native decode of slice k + 1 on the host while
    slice k uploads and loads on the GPU) followed by the tails.  n_emit distinct summaries
    are emitted as SnapshotV1 JSON chunks (untimed) and document d takes summary d % n_emit
    and its tail, so document d must end as the device-only step left document d % n_emit."""
    from fluidframework_amd.snapdec import SummaryDecoder
    from fluidframework_amd.snapshot import encode_chunks, record_specs
    from fluidframework_amd.wire import Interner
    it = Interner(synthetic=True)
    c = np.asarray(counts, dtype=np.int64)
    r0 = np.concatenate([[0], np.cumsum(c[:, 0])])
    t0 = np.concatenate([[0], np.cumsum(c[:, 1])])
    p0 = np.concatenate([[0], np.cumsum(c[:, 2])])
    names = {i: f"client-{i}" for i in range(-2, 4096)}
    emitted = []
    for d in range(n_emit):
        specs, lengths = record_specs(recs[r0[d]:r0[d + 1]], text[t0[d]:t0[d + 1]], props[p0[d]:p0[d + 1]], it, names)
        emitted.append(SummaryDecoder.pack([encode_chunks(specs, lengths, int(mn[d]), int(cu[d]), chunk)]))
    # the tails continue with the short ids the summaries' loads assign (getOrAddShortClientId
    # in first-seen order, as a reference client loading the summary would): decoded once here
    remap = np.zeros((n_emit, 4097), dtype=np.uint16)   # writer ids 0..4096 (others unchanged)
    _, _, cl = SummaryDecoder(Interner(synthetic=True), threads=threads).decode_packed_full(
        [p for e in emitted for p in e[0]], [b for e in emitted for b in e[1]],
        list(np.cumsum([0] + [len(e[0]) for e in emitted])))
    for d in range(n_emit):
        remap[d] = np.arange(4097, dtype=np.uint16)
        for name, short in cl[d].items():
            k = int(name[len("client-"):])
            if 0 <= k <= 4096:
                remap[d, k] = short
    n = mt.n_docs
    paths, blobs, off = [], [], [0]
    for d in range(n):
        ep, eb, _ = emitted[d % n_emit]
        paths += ep
        blobs += eb
        off.append(len(paths))
    nbytes = sum(len(b) for b in blobs)
    src = np.arange(n) % n_emit
    # a tail writer the summary does not name gets the next short id (first seen in the tail)
    t_emit = tail_arr["ops"].reshape(-1, tail)[:n_emit]
    for d in range(n_emit):
        nxt = len(cl[d]) + 1
        named = {int(k[len("client-"):]) for k in cl[d]}
        for k in t_emit[d]["client"].tolist():
            if k <= 4096 and k not in named:
                named.add(k)
                remap[d, k] = nxt
                nxt += 1
    ops = tail_arr["ops"].reshape(-1, tail)[src].copy()
    c = ops["client"].astype(np.int64)
    ops["client"] = np.where(c <= 4096, remap[src[:, None], np.minimum(c, 4096)], c)
    ops = ops.ravel()
    tb = mt.upload(dict(tail_arr, ops=ops, doc_off=np.arange(n + 1, dtype=np.int64) * tail))
    best = None
    for dec_threads in sorted({threads, max(1, threads - 1)}):   # all cores, or one left to the uploads
        times = []
        for rep in range(3):   # the first run warms the decoder's buffers and the workers
            mt.sync()
            t = time.perf_counter()
            mt.catch_up(None, Interner(synthetic=True), threads=dec_threads, slice_docs=slice_docs,
                        packed=(paths, blobs, off))
            tb.apply_async()
            mt.sync()
            times.append(time.perf_counter() - t)
        if best is None or min(times[1:]) < best[0]:
            best = (min(times[1:]), dec_threads)
    el, threads = best
    tb.free()
    ok = bool(np.array_equal(mt.checksums(), sums[src]) and np.array_equal(mt.status(), status[src]))
    return dict(value=round(n / el, 1), unit="docs/s", cores=threads, json_mb_per_s=round(nbytes / el / 1e6, 1),
                slice_docs=slice_docs, equals_device_only_step=ok,
                sample=f"{n} documents ({nbytes / 1e6:.0f} MB of summary JSON, {n_emit} distinct summaries) "
                       f"decoded on {threads} host threads (+ the upload thread), uploaded, loaded and their {tail}-op tails replayed: "
                       f"{el:.3f} s (best of 2 after a warm-up run)")


def c5_roofline(load, counts, tail_arr, sums, n_tail, load_ms, tail_ms):
    """Roofline of C5's dominant kernel: the summary load (k_load_header:
    reads every 32-byte mt_seg_rec, its text and property words; writes the segment rows and
    the text) or the tail replay (the C3 accounting: op records, results, payload, final state)."""
    import numpy as np
    n_segs = int(len(load["segs"]))
    text_units = int(counts[:, 1].sum())
    props_words = int(counts[:, 2].sum())
    load_bytes = n_segs * (32 + SEG_BYTES) + 4 * text_units + 4 * props_words
    ops = tail_arr["ops"]
    ins = ops["kind"] == 0
    final_bytes = int(sums["n_segments"].astype(np.int64).sum()) * SEG_BYTES + 2 * int(sums["length"].astype(np.int64).sum())
    tail_bytes = n_tail * (OP_BYTES + RESULT_BYTES) + 2 * int(ops["pos2"][ins].sum()) + final_bytes
    load_dom = load_ms >= tail_ms
    ms, alg = (load_ms, load_bytes) if load_dom else (tail_ms, tail_bytes)
    achieved = alg / (ms / 1000.0) / 1e9 if ms > 0 else 0.0
    return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": achieved / (HBM_PEAK / 1e9), "traffic": None,
            "kernel": "k_load_header (summary load)" if load_dom else "k_replay (64-op tails)",
            "kernel_ms": round(ms, 3), "alg_bytes_per_launch": alg,
            "other_kernel_ms": round(tail_ms if load_dom else load_ms, 3)}


def run_c5(args, cfg, rank, world, local_rank, dist):
    """Config C5 (cold catch-up): every document's SnapshotV1 summary is loaded
    (mt_snapshots_load_async: reloadFromSegments + loadBody) and its tail of `tail` sequenced
    messages replayed.  Inputs (decoded summaries as mt_seg_rec records, tail batch) are
    resident in HBM; the summaries are SnapshotV1.extractSync of the observer after `ops`
    generated messages (mt_extract_snapshots, untimed), the tail is messages ops+1..ops+tail
    of the same generated streams."""
    import numpy as np
    from fluidframework_amd import MergeTreeBatch
    from fluidframework_amd.snapshot import load_arrays_from_extract
    docs = args.docs or cfg["docs"] // 8          # the 1M summaries shard over 8 GPUs
    K, tail = cfg["ops"], cfg["tail"]
    caps = dict(seg_capacity=1024, text_capacity=1 << 14, heap_capacity=1024, props_capacity=1024,
                lds_seg_capacity=args.lds_cap or 256, page_capacity=-1)
    mt = MergeTreeBatch(docs, device=local_rank, **caps)
    base = rank * docs
    t_prep = time.time()
    g1 = mt.generate(dict(cfg, ops=K), base)
    counts, recs, text, props, mn, cu = mt.extract_snapshots_raw()
    g1.free()
    load = load_arrays_from_extract(counts, recs, text, props, mn, cu, cfg["chunk"])
    g2 = mt.generate(dict(cfg, ops=K + tail), base)
    host = g2.download()
    g2.free()
    idx = (np.arange(docs)[:, None] * (K + tail) + K + np.arange(tail)[None, :]).ravel()
    tail_arr = dict(ops=host["ops"][idx], doc_off=np.arange(docs + 1, dtype=np.int64) * tail,
                    text=host["text"], props=host["props"])
    snaps = mt.upload_snapshots(load)
    tb = mt.upload(tail_arr)
    t_prep = time.time() - t_prep

    def step():
        snaps.load_async()
        tb.apply_async()

    for _ in range(args.warmup):
        step()
        mt.sync()
    if dist is not None:
        dist.barrier()
    mt.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    mt.sync()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    load_ms, tail_ms = mt.last_load_ms(), mt.last_kernel_ms()   # (the last step's, HIP events)
    status = mt.status()
    sums = mt.checksums()
    if rank != 0:
        return
    n_tail = int(len(idx))
    roofline = c5_roofline(load, counts, tail_arr, sums, n_tail, load_ms, tail_ms)
    cpu = parity = decode = e2e = None
    if not args.no_cpu:
        threads = args.cpu_threads or host_cores()
        decode = c5_decode_rate(counts, recs, text, props, mn, cu, cfg["chunk"], min(docs, 4000), threads)
        e2e = c5_end_to_end(mt, counts, recs, text, props, mn, cu, cfg["chunk"], tail_arr, tail, sums, status,
                            min(docs, 4000), threads)
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import pyoracle                            # the checker, timed as the CPU baseline
        n_sample = args.cpu_sample_docs or min(docs, 20000)
        lo = {k: v for k, v in load.items()}
        lo["doc_off"] = load["doc_off"][: n_sample + 1]
        sa = dict(tail_arr, doc_off=tail_arr["doc_off"][: n_sample + 1])
        threads = args.cpu_threads or host_cores()
        t_c = time.perf_counter()
        osums, ost = pyoracle.load_replay_batch(lo, sa, threads=threads)
        t_c = time.perf_counter() - t_c
        cpu = dict(value=round(n_sample / t_c, 1), unit="docs/s", cores=threads, kind="port",
                   sample=f"oracle/mt_oracle.c orc_load + tail replay of docs [0,{n_sample}) on {threads} host threads, "
                          f"{t_c:.2f} s ({n_sample * tail / t_c:.0f} tail ops/s)")
        parity = dict(docs_checked=n_sample, mismatches=int((osums != sums[:n_sample]).sum() + (ost != status[:n_sample]).sum()))
    docs_total = docs * world
    print(json.dumps({
        "metric": "cold catch-up: SnapshotV1 summaries loaded + tail ops replayed per second (config C5)",
        "value": round(docs_total * args.steps / elapsed, 1), "unit": "docs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1000 / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int32", "data": "synthetic",
        "tail_ops_per_s": round(n_tail * world * args.steps / elapsed, 1),
        "config": {"workload": f"c5: {docs} summaries/GPU (doc {cfg['seed_len']} units + {K} generated ops, "
                               f"chunkSize {cfg['chunk']}), {tail}-op tails, {cfg['writers']} writers",
                   "docs_total": docs_total, "summary_segments": int(len(load["segs"])),
                   "summary_text_units": int(counts[:, 1].sum()), "body_docs": int((load["n_header"] <
                                                                                     np.diff(load["doc_off"])).sum()),
                   "parallelism": f"doc-shard x{world}"},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "summary_decode": decode,
        "end_to_end": e2e,
        "parity": {"status_nonzero": int((status != 0).sum()), "oracle_sample": parity},
        "prep_s": round(t_prep, 2),
    }))


def run_live(args, rank, world, local_rank, dist):
    """Live-client path: participant replicas applying their own
    local ops, the acks of them and remote writers' ops, on a live_client handle.  The event
    streams are the reference's own (tests/golden/ref_live_bench.json.gz: 8 participant
    streams of 4000 steps, made by oracle/ref_harness.mjs live), each replicated over the
    documents; one step = reset + one batch of every document's whole stream, resident in
    HBM.  CPU baseline: the C restatement as the same participant (oracle/mt_oracle.c, pinned
    to these streams by tests/test_oracle.py) replaying rank 0's documents on the host's
    cores; its checksums are compared with the GPU's document by document."""
    import gzip
    import numpy as np
    from fluidframework_amd import MergeTreeBatch
    from fluidframework_amd.wire import Batch, Interner
    fx = json.load(gzip.open(os.path.join(REPO, "tests", "golden", "ref_live_bench.json.gz"), "rt"))
    streams = fx["docs"]
    docs = args.docs or 4096
    # encode each stream once; the replicas share its records and arenas (offsets into them)
    b = Batch(Interner(synthetic=True))
    for st in streams:
        ent = []
        for ev in st["events"]:
            if ev[0] == "L":
                ent.append(("local", ev[1]))
            else:
                _, cid, seq, ref, msn, op = ev
                m = dict(clientId=cid, sequenceNumber=seq, referenceSequenceNumber=ref, minimumSequenceNumber=msn,
                         type="op", contents=op)
                ent.append(("ack" if cid == "local-0" else "msg", m))
        b.add_live_doc(st["seed_text"], ent, {"local-0": 0})
    e = b.arrays()
    sid = (rank * docs + np.arange(docs)) % len(streams)
    lens = np.diff(e["doc_off"])[sid]
    idx = np.concatenate([np.arange(e["doc_off"][k], e["doc_off"][k + 1]) for k in sid])
    slen = np.diff(e["seed_off"])[sid]
    sidx = np.concatenate([np.arange(e["seed_off"][k], e["seed_off"][k + 1]) for k in sid])
    a = dict(ops=e["ops"][idx], doc_off=np.concatenate([[0], np.cumsum(lens)]).astype(np.int64),
             text=e["text"], props=e["props"], seed=e["seed"][sidx] if len(sidx) else e["seed"][:1],
             seed_off=np.concatenate([[0], np.cumsum(slen)]).astype(np.int64))
    n_events = int(lens.sum())
    threads = args.cpu_threads or host_cores()
    mt = MergeTreeBatch(docs, device=local_rank, seg_capacity=4096, text_capacity=1 << 15, props_capacity=4096,
                        heap_capacity=4096, lds_seg_capacity=args.lds_cap if args.lds_cap > 0 else -1, live_client=1)
    mt.load_initial_text(a["seed_off"], a["seed"])
    batch = mt.upload(a)

    def step():
        mt.reset()
        batch.apply_async()

    for _ in range(args.warmup):
        step()
        mt.sync()
    if dist is not None:
        dist.barrier()
    mt.sync()
    t0 = time.perf_counter()
    kms = 0.0
    for _ in range(args.steps):
        step()
        mt.sync()
        kms += mt.last_kernel_ms()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    status = mt.status()
    # parity: every replica ends with the reference participant's text, localSeq and queue
    sample = list(range(min(docs, 32)))
    bad = 0
    counts = mt.pending_counts()
    for d in sample:
        st = streams[(rank * docs + d) % len(streams)]
        bad += int(mt.get_text(d) != st["out"]["text"] or
                   tuple(counts[d]) != (st["out"]["localSeq"], st["out"]["pending"]))
    if rank != 0:
        return
    cpu = oracle_sample = None
    if not args.no_cpu:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import pyoracle                            # the checker, timed as the CPU baseline
        # bounded sample: at most ~24M events of CPU work (all of rank 0's 4096 documents)
        n_sample = args.cpu_sample_docs or min(docs, max(1, 24_000_000 // max(int(lens.max()), 1)))
        sel_end = int(a["doc_off"][n_sample])
        sub = dict(a, ops=a["ops"][:sel_end], doc_off=a["doc_off"][: n_sample + 1],
                   seed_off=a["seed_off"][: n_sample + 1])
        t_c = time.perf_counter()
        osums, ost = pyoracle.replay_batch(sub, threads=threads)
        t_c = time.perf_counter() - t_c
        cpu = dict(value=round(sel_end / t_c, 1), unit="events/s", cores=threads, kind="port",
                   host_cpus=os.cpu_count(),
                   sample=f"oracle/mt_oracle.c participant replay of rank-0 docs [0,{n_sample}) of the same "
                          f"batch ({sel_end} events) on {threads} host threads, {t_c:.2f} s")
        cal = _live_calibration()
        if cal and cal.get("ratio_port_over_reference"):
            r = cal["ratio_port_over_reference"]
            cpu["reference_estimate"] = dict(
                value=round(cpu["value"] / r, 1), unit="events/s", cores=threads,
                how=f"port value / {r} (port vs the transpiled reference participant on the same streams, one "
                    f"thread each, in the build container; {cal['sample']})")
        sums = mt.checksums()
        oracle_sample = dict(docs_checked=n_sample,
                             mismatches=int((osums != sums[:n_sample]).sum() + (ost != status[:n_sample]).sum()))
    print(json.dumps({
        "metric": "live-client merge-tree events applied/sec (local ops + acks + remote ops)",
        "value": round(n_events * world * args.steps / elapsed, 1), "unit": "events/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1000 / args.steps, 3),
        "kernel_ms_per_step": round(kms / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int32",
        "data": "the reference's participant streams (ref_live_bench), replicated",
        "config": {"workload": f"live: {docs} participant documents/GPU x {n_events // docs} events "
                               f"(local ops 0.3, acks, remote ops from 8 writers, lag 48)",
                   "docs_total": docs * world, "events_per_step": n_events * world,
                   "parallelism": f"doc-shard x{world}"},
        "cpu_baseline": cpu,
        "reference_calibration": _live_calibration(),
        "parity": {"status_nonzero": int((status != 0).sum()), "docs_checked": len(sample), "mismatches": bad,
                   "oracle_sample": oracle_sample},
    }))


def _live_calibration():
    """The reference participant's own speed on the same streams (one thread, measured in the
    build container: the reference cannot travel to the GPU box)."""
    p = os.path.join(REPO, "profiles", "r3", "live_calibration.json")
    if not os.path.exists(p):
        return None
    c = json.load(open(p))
    return dict(value=round(c["events_per_s"], 1), unit="events/s", cores=1, kind="reference",
                sample=f"{c['events']} events, {os.path.relpath(p, REPO)}",
                ratio_port_over_reference=c.get("ratio_port_over_reference"))


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but {world} rank(s) were launched")
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    configs = json.load(open(os.path.join(REPO, "bench", "configs.json")))
    runner = dispatch(args)
    if args.config == "live":
        runner(args, rank, world, local_rank, dist)
    else:
        runner(args, dict(configs[args.config]), rank, world, local_rank, dist)
    if dist is not None:
        dist.destroy_process_group()


def dispatch(args):
    """The runner of `--config`: c5 (cold catch-up), live (participant replicas), c3skew
    (skewed lengths, bench_skew.py) or the uniform replay (c2 / c3 / c4)."""
    if args.config == "live":
        return run_live
    if args.config == "c5":
        return run_c5
    if args.config == "c3skew":
        import bench_skew
        mod = sys.modules[__name__]

        def skew(args, cfg, rank, world, local_rank, dist):
            line = bench_skew.run_skew(args, cfg, rank, world, local_rank, dist, mod)
            if line is not None:
                print(json.dumps(line), flush=True)
        return skew
    if args.config in ("c2", "c3", "c4"):
        return run_replay
    raise SystemExit(f"bench.py: unknown --config {args.config}")


def c3_logs():
    """The reference's own C3 message logs (tests/golden/ref_c3_full): (fixture, JSON blobs)."""
    import gzip
    from fluidframework_amd.opdec import MessageDecoder
    from fluidframework_amd.wire import compact_msgs_to_dicts
    fx = json.load(gzip.open(os.path.join(REPO, "tests", "golden", "ref_c3_full.json.gz"), "rt"))
    return fx, MessageDecoder.pack([compact_msgs_to_dicts(d["msgs"]) for d in fx["docs"]])


def ingest_rates(mt, host, step_s, caps, device, pipeline=None):
    """What the timed region leaves out, reported beside it: the host encode of
    sequenced messages into op records (the reference's own C3 message logs, ref_c3_full,
    through wire.Batch -- the encoder encode.js mirrors) and the H2D upload of this step's op
    records and arenas from pageable host memory (mt_batch_upload), so that a log ingested
    from the host would replay at value_with_upload."""
    import gzip
    from fluidframework_amd.wire import Batch, Interner, compact_msgs_to_dicts
    fx = json.load(gzip.open(os.path.join(REPO, "tests", "golden", "ref_c3_full.json.gz"), "rt"))
    msgs = [compact_msgs_to_dicts(d["msgs"]) for d in fx["docs"]]
    t = time.perf_counter()
    b = Batch(Interner(synthetic=True))
    for d, m in zip(fx["docs"], msgs):
        b.add_doc(d["seed_text"], m)
    b.arrays()
    t_enc = time.perf_counter() - t
    n_msgs = sum(len(m) for m in msgs)
    nbytes = host["ops"].nbytes + host["text"].nbytes + host["props"].nbytes + host["doc_off"].nbytes
    mt.sync()
    t = time.perf_counter()
    up = mt.upload(host)
    mt.sync()
    t_up = time.perf_counter() - t
    up.free()
    n_ops = len(host["ops"])
    # the native encoder (mt_opdec, libmtsnapdec.so) on the same logs as JSON text, each
    # document's log repeated to 512 documents, on the host's cores
    from fluidframework_amd.opdec import MessageDecoder
    blobs = MessageDecoder.pack(msgs)
    reps = max(1, 512 // len(blobs))
    many = blobs * reps
    threads = host_cores()
    dec = MessageDecoder(Interner(synthetic=True), threads=threads)
    dec.decode_packed(many[:len(blobs)])   # (warm: thread pool buffers)
    t = time.perf_counter()
    dec.decode_packed(many)
    t_nat = time.perf_counter() - t
    del dec
    nat_msgs, nat_mb = n_msgs * reps, sum(len(x) for x in many) / 1e6
    nat_rate = nat_msgs / t_nat
    return {"encode": {"value": round(n_msgs / t_enc, 1), "unit": "messages/s", "cores": 1,
                       "sample": f"{n_msgs} messages of tests/golden/ref_c3_full (JSON message objects -> op records "
                                 f"+ arenas, fluidframework_amd/wire.py Batch), {t_enc:.2f} s"},
            "encode_native": {"value": round(nat_rate, 1), "unit": "messages/s", "cores": threads,
                              "MB_per_s": round(nat_mb / t_nat, 1),
                              "sample": f"{nat_msgs} messages ({nat_mb:.0f} MB of JSON: the ref_c3_full logs x {reps}) "
                                        f"-> op records + arenas by mt_opdec_decode + fetch (libmtsnapdec.so, equal to "
                                        f"wire.Batch: tests/test_snapdec.py), {t_nat:.2f} s"},
            "value_with_native_encode_and_upload_serial": round(n_ops / (step_s + t_up + n_ops / nat_rate), 1),
            "pipeline": pipeline or ingest_pipeline(caps, device, fx, blobs, threads),
            "h2d_upload": {"bytes": int(nbytes), "s": round(t_up, 3), "GB_per_s": round(nbytes / t_up / 1e9, 2),
                           "how": "mt_batch_upload of this step's op records, text and property arenas from pageable "
                                  "host memory (validation + hipMemcpy)"},
            "value_with_upload": round(n_ops / (step_s + t_up), 1)}


def ingest_pipeline(caps, device, fx, blobs, threads, slice_docs=3072, n_slices=8):
    """The C3 job from JSON message logs, overlapped (MergeTreeBatch.ingest_logs): the native
    encoder turns slice k + 1's logs into op records on the host's cores while slice k is
    uploaded and slice k - 1 replays on the GPU.  Slices of `slice_docs` C3 documents (the
    reference's own 10k-message logs, tests/golden/ref_c3_full, repeated), `n_slices` of them
    on a fresh handle at the bench's capacities.  Each stage is also timed alone on one slice;
    the overlapped rate is compared with the slowest stage's.  Checked: every copy of a log
    replays to the same checksums, and those equal the C restatement's."""
    from fluidframework_amd import Interner, MergeTreeBatch
    from fluidframework_amd.opdec import MessageDecoder
    nd = len(blobs)
    n_docs = slice_docs * n_slices
    mt = MergeTreeBatch(n_docs, device=device, **caps)
    seeds = [np.frombuffer(d["seed_text"].encode("utf-16-le"), dtype="<u2") for d in fx["docs"]]
    seed_off = np.concatenate([[0], np.cumsum([len(seeds[d % nd]) for d in range(n_docs)])]).astype(np.int64)
    seed = np.concatenate([seeds[d % nd] for d in range(n_docs)]).astype(np.uint16)

    def slices():
        for k in range(n_slices):
            d0 = k * slice_docs
            yield d0, [blobs[d % nd] for d in range(d0, d0 + slice_docs)]

    # the stages alone, on one slice (warm buffers: the decoder's, a second pass)
    dec = MessageDecoder(Interner(synthetic=True), threads=threads)
    one = [blobs[d % nd] for d in range(slice_docs)]
    dec.decode_packed(one)
    t = time.perf_counter()
    out = dec.decode_packed(one)
    t_enc = time.perf_counter() - t
    n_slice = len(out["ops"])
    full = dict(out, doc_off=np.concatenate([out["doc_off"], np.full(n_docs - slice_docs, out["doc_off"][-1])]))
    mt.load_initial_text(seed_off, seed)
    mt.sync()
    t = time.perf_counter()
    b = mt.upload(full)
    t_up = time.perf_counter() - t
    t = time.perf_counter()
    b.apply_async()
    mt.sync()
    t_rep = time.perf_counter() - t
    b.free()
    del out, full, dec
    # the pipeline: an untimed pass over two slices first warms the handle's encoder and its
    # two arena sets (a running ingest service keeps them: fresh pages fault under 16 threads)
    mt.reset()
    mt.load_initial_text(seed_off, seed)
    mt.ingest_logs(((k * slice_docs, [blobs[d % nd] for d in range(k * slice_docs, (k + 1) * slice_docs)])
                    for k in range(2)), threads=threads)
    mt.reset()
    mt.load_initial_text(seed_off, seed)
    mt.sync()
    busy = mt.ingest_logs(slices(), threads=threads)
    n_all = n_slice * n_slices
    sums = mt.checksums()
    same = all(np.array_equal(sums[d], sums[d % nd]) for d in range(n_docs))
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    ref, _ = MessageDecoder(Interner(synthetic=True), threads=threads).decode(blobs[:nd],
                                                                               [d["seed_text"] for d in fx["docs"]])
    osums, ost = pyoracle.replay_batch(ref, threads=min(threads, nd))
    same = same and bool(np.array_equal(sums[:nd], osums)) and int((ost != 0).sum()) == 0
    del mt
    rates = {"encode": n_slice / t_enc, "upload": n_slice / t_up, "replay": n_slice / t_rep}
    slowest = min(rates, key=rates.get)
    overlapped = n_all / busy["wall"]
    serial = n_all / (n_slices * (t_enc + t_up + t_rep))
    return {"value": round(overlapped, 1), "unit": "messages/s",
            "messages": n_all, "slices": n_slices, "docs_per_slice": slice_docs, "wall_s": round(busy["wall"], 3),
            "stage_rates": {k: round(v, 1) for k, v in rates.items()}, "slowest_stage": slowest,
            "fraction_of_slowest": round(overlapped / rates[slowest], 3),
            "serial_value": round(serial, 1),
            "busy_s": {k: round(v, 3) for k, v in busy.items() if k not in ("wall", "encode_slices")},
            "encode_slices_s": [round(v, 3) for v in busy["encode_slices"]],
            "checksums_equal_oracle": same,
            "how": f"JSON message logs (tests/golden/ref_c3_full's 4 reference-made 10k-message C3 logs, repeated) "
                   f"-> MergeTreeBatch.ingest_logs: native encode (libmtsnapdec mt_opdec, {threads} host threads) "
                   f"of slice k+1 || upload (mt_batch_upload) of slice k || replay of slice k-1 on the GPU; "
                   f"stage rates timed alone on one slice ({slice_docs} documents; the replay of one slice "
                   f"does not fill the GPU as the 100k-document job does)"}


def run_replay(args, cfg, rank, world, local_rank, dist):
    """Uniform replay (c2 / c3 / c4): the default line, BASELINE configs[2]."""
    from fluidframework_amd import MergeTreeBatch
    docs, doc_base, docs_total, scaling = shard_plan(args, cfg, world, rank)
    if args.ops:
        cfg["ops"] = args.ops

    caps = capacities(cfg)
    if args.lds_cap:
        caps["lds_seg_capacity"] = args.lds_cap
    if args.seg_cap:
        caps["seg_capacity"] = args.seg_cap
    if args.heap_cap:
        caps["heap_capacity"] = args.heap_cap
    if args.page_caps:
        pp, ut, ph = (int(x) for x in args.page_caps.split(","))
        caps.update(lds_page_capacity=pp, lds_unsettled_capacity=ut, lds_page_heap_capacity=ph)
    if args.paged_slices and caps.get("page_capacity", 0) > 0:
        caps["paged_slices"] = args.paged_slices
    # the overlapped ingest first, while the process holds nothing else: after the step it ran
    # 7-10 % slower in its host encode (the line vs tools/ingest_probe.py, profiles/r6); rank 0
    # only, like the CPU baseline (the host's cores are shared by the ranks)
    pipeline = None
    with_ingest = not args.no_ingest and rank == 0
    if with_ingest:
        fx, blobs = c3_logs()
        pipeline = ingest_pipeline(caps, local_rank, fx, blobs, host_cores())
        del fx, blobs
    t_gen = time.time()
    mt = MergeTreeBatch(docs, device=local_rank, **caps)
    batch = mt.generate(cfg, doc_base)          # untimed: inputs resident in HBM
    gen_peaks = mt.last_paged_peaks() if caps.get("page_capacity", 0) > 0 else None
    gen_sums = mt.checksums()
    t_gen = time.time() - t_gen
    seed_off, seed = mt.generated_seeds(cfg, doc_base)
    mt.load_initial_text(seed_off, seed)
    n_ops = batch.n_ops
    progress(rank, f"generated {docs} documents, {n_ops} messages ({t_gen:.1f} s)")

    def step():
        mt.reset()
        batch.apply_async()

    for k in range(args.warmup):
        step()
        mt.sync()
        progress(rank, f"warmup step {k + 1}/{args.warmup}")

    def barrier():
        if dist is not None:
            dist.barrier()

    kernel_ms = []
    barrier()
    mt.sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step()
        mt.sync()                     # per-step sync to read this step's kernel events
        kernel_ms.append(mt.last_kernel_ms())
        progress(rank, f"step {k + 1}/{args.steps}: {kernel_ms[-1]:.0f} ms")   # (stderr, after the sync)
    mt.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        t = torch.tensor([n_ops], dtype=torch.int64, device="cuda")
        dist.all_reduce(t)                # shards may differ by one document
        total_ops = int(t.item())
    else:
        total_ops = n_ops

    hbm_docs = mt.last_hbm_docs()
    peaks = mt.last_paged_peaks() if caps.get("page_capacity", 0) > 0 else None
    status = mt.status()
    sums = mt.checksums()
    replay_consistent = bool(np.array_equal(sums, gen_sums)) and int((status != 0).sum()) == 0

    threads = args.cpu_threads or host_cores()
    # the only collective: all-gather of per-document checksums over RCCL/xGMI, verified
    shards = None
    if dist is not None:
        import torch
        local = torch.empty(docs * 32, dtype=torch.uint8, device="cuda")
        mt.checksums_device(local.data_ptr())
        shards = verify_shards(dist, rank, world, docs_total, cfg, local, gen_sums, torch.device("cuda", local_rank),
                               args.verify_per_rank, threads)
        ok = torch.tensor([1 if replay_consistent else 0], device="cuda")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        replay_consistent = bool(ok.item())
        if rank == 0 and not (shards["replay_equals_generation"] and shards["oracle_mismatches"] in (0, None)):
            replay_consistent = False

    if rank != 0:
        return

    ms_per_step = elapsed * 1000.0 / args.steps
    value = total_ops * args.steps / elapsed

    # roofline: algorithmic bytes per launch (DESIGN.md "Roofline accounting")
    host = batch.download()
    ins = host["ops"]["kind"] == 0
    payload_chars = int(host["ops"]["pos2"][ins].sum())
    final_bytes = int(sums["n_segments"].astype(np.int64).sum()) * SEG_BYTES + 2 * int(sums["length"].astype(np.int64).sum())
    alg_bytes = n_ops * (OP_BYTES + RESULT_BYTES) + 2 * payload_chars + final_bytes
    k_ms = float(np.mean(kernel_ms))
    achieved = alg_bytes / (k_ms / 1000.0)
    ingest = None if not with_ingest else ingest_rates(mt, host, ms_per_step / 1000.0, caps, local_rank,
                                                             pipeline)
    traffic = traffic_raw = None
    if os.path.exists(PROFILE_PMC):
        try:
            pm = json.load(open(PROFILE_PMC)).get(args.config, {})
            if pm.get("docs") == docs and pm.get("ops") == cfg["ops"] and pm.get("seed_base", 0) == doc_base:
                traffic = pm.get("hbm_bytes_per_launch")
                traffic_raw = pm.get("hbm_bytes_per_launch_raw")
        except Exception:
            traffic = None

    cpu = None
    parity = None
    if not args.no_cpu and rank == 0:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import pyoracle                            # the checker, timed as the CPU baseline
        # bounded sample: about 100M ops of CPU work, ~10 s on 16 host threads (all of C2's
        # rank-0 documents); rank 0 only (the host's cores are shared by the ranks), reported
        # as the CPU baseline at N = 1 only
        n_sample = args.cpu_sample_docs or min(docs, max(1, 100_000_000 // max(cfg["ops"], 1)))
        off = host["doc_off"]
        sel_end = int(off[n_sample])
        arrays = dict(ops=host["ops"][:sel_end], doc_off=off[: n_sample + 1], text=host["text"],
                      props=host["props"], seed_off=seed_off[: n_sample + 1], seed=seed)
        t_c = time.perf_counter()
        osums, ost = pyoracle.replay_batch(arrays, threads=threads)
        t_c = time.perf_counter() - t_c
        cpu = dict(value=round(sel_end / t_c, 1), unit="ops/s", cores=threads, kind="port",
                   host_cpus=os.cpu_count(),
                   sample=f"oracle/mt_oracle.c replay of rank-0 docs [0,{n_sample}) of the same "
                          f"{args.config} batch ({sel_end} ops) on {threads} host threads, {t_c:.2f} s")
        parity = dict(docs_checked=n_sample,
                      mismatches=int((osums != sums[:n_sample]).sum() + (ost != 0).sum()))
        if world > 1:
            cpu = None
        # the reference itself cannot travel: its single-thread speed relative to the port on
        # the same streams is measured in the build container (oracle/calibrate.py)
        try:
            cal = json.load(open(CALIBRATION)).get(args.config)
        except (OSError, ValueError):
            cal = None
        if cal and cpu is not None:
            # the no-callback ratio: the reference's fastest replay, so the estimate is an upper bound
            r = cal["ratio_port_over_reference_nocb"]
            cpu["reference_estimate"] = dict(
                value=round(cpu["value"] / r, 1), unit="ops/s", cores=threads,
                how=f"port value / {r} (port vs transpiled reference MergeTree, observer without a delta "
                    f"callback, under {cal['reference_runtime']}, one thread each, {cal['docs']} docs / "
                    f"{cal['ops']} {args.config} ops; {os.path.relpath(CALIBRATION, REPO)}); with the "
                    f"position-recording callback the ratio is {cal['ratio_port_over_reference']}")

    assert world == args.gpus
    out = {
        "metric": "sequenced merge-tree ops applied/sec (node) at 100k docs; bit-exact text+props",
        "value": round(value, 1),
        "unit": "ops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {
            "workload": f"{args.config}: {docs} docs/GPU x {cfg['ops']} sequenced ops, {cfg['writers']} writers, "
                        f"refSeq lag <= {cfg['lag']}, insert {cfg['p_insert']} / remove {cfg['p_remove']}"
                        f"{' / annotate ' + str(round(1 - cfg['p_insert'] - cfg['p_remove'], 3)) if cfg['p_insert'] + cfg['p_remove'] < 1 else ''}",
            "docs_total": docs_total, "docs_per_gpu": docs, "ops_per_doc": cfg["ops"], "ops_per_step": total_ops,
            "parallelism": f"doc-shard x{world}",
        },
        "roofline": {
            "bound": "hbm", "achieved": round(achieved / 1e9, 3), "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": achieved / HBM_PEAK, "traffic": traffic,
            "traffic_raw": traffic_raw,
            "traffic_correction": ("2 x FETCH_SIZE + WRITE_SIZE: on gfx950 FETCH_SIZE counts 64 B per 128-byte read "
                                   "request; measured 1/2 on this kernel's page-window, uid-map and text read "
                                   "patterns (profiles/r4/fetch_calibration.json) and cross-checked by the L2 "
                                   "request counts (profiles/pmc_summary.json)") if traffic is not None else None,
            "kernel": ("k_replay<TierLdsT<false>> (first ops) + k_replay_paged<TierPagedT<false>> (rest)"
                       if caps.get("page_capacity", 0) > 0 else
                       "k_replay<TierLdsT<false>> + k_replay<TierGlbT<false>> (HBM-tier hand-over)"),
            "kernel_ms": round(k_ms, 3), "alg_bytes_per_launch": alg_bytes,
            "docs_replayed_from_hbm": hbm_docs,
            "paged_peaks": peaks,
            "paged_caps": {"lds": [caps.get("lds_page_capacity"), caps.get("lds_unsettled_capacity"),
                                   caps.get("lds_page_heap_capacity")],
                           "hbm": [caps.get("page_capacity"), caps.get("unsettled_capacity"),
                                   caps.get("page_heap_capacity")]},
        },
        "cpu_baseline": cpu,
        "ingest": ingest,
        "parity": {"replay_equals_generation": replay_consistent, "oracle_sample": parity,
                   "shards": shards},
        "gen_s": round(t_gen, 2),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
