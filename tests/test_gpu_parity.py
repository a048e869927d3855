"""HIP path vs the reference (golden fixtures made by the reference itself) and vs the CPU
oracle, through the C ABI.  Bit-exact on every output: text, length, leaf-block partition,
segment table, property sets, every delta-callback record, checksums."""
import numpy as np
import pytest

import golden_util as gu

pytestmark = pytest.mark.gpu


def _gpu_batch(n_docs, **kw):
    """A handle for one storage tier: without paged capacities, a flat-only one (page_capacity
    -1: the library's default handle is paged, see test_gpu_default_handle_is_unbounded)."""
    from fluidframework_amd import MergeTreeBatch
    kw.setdefault("delta_log_capacity", 1 << 18)
    kw.setdefault("seg_capacity", 8192)       # flat tiers: the 10k-op fixtures hold ~4.5k segments
    kw.setdefault("text_capacity", 1 << 17)
    kw.setdefault("page_capacity", -1)
    return MergeTreeBatch(n_docs, **kw)


def _gpu_outputs(mt, doc):
    rows, leaves = mt.get_segments(doc)
    return dict(text=mt.get_text(doc), length=mt.get_length(doc), leaves=leaves, segs=rows,
                seg_props=mt.get_all_segment_props(doc),
                deltas=mt.get_delta_log(doc), status=int(mt.status()[doc]))


# Storage tiers: "lds" = default LDS tier (large documents continue in the flat HBM tier),
# "hbm" = flat HBM tier only, "tiny" = 16-segment LDS tier (most documents overflow
# mid-batch), "paged" = every document in the paged layout from the start, "tiny_paged" =
# documents overflowing a 16-segment LDS tier continue in the paged layout.
TIERS = {
    "lds": dict(lds_seg_capacity=0),
    "hbm": dict(lds_seg_capacity=-1),
    "tiny": dict(lds_seg_capacity=16),
    "paged": dict(lds_seg_capacity=-1, page_capacity=256, unsettled_capacity=2048, page_heap_capacity=2048),
    "tiny_paged": dict(lds_seg_capacity=16, page_capacity=256, unsettled_capacity=2048, page_heap_capacity=2048),
    # a tight paged tier far below the documents' needs: documents are handed to the
    # full-capacity paged launch mid-batch (and at load), generators regenerate there
    "tight": dict(lds_seg_capacity=16, page_capacity=256, unsettled_capacity=2048, page_heap_capacity=2048,
                  lds_page_capacity=24, lds_unsettled_capacity=40, lds_page_heap_capacity=40),
    # a narrow tight tier (32-bit overlap masks): documents whose clients above 32 remove
    # overlapping ranges (C4: 64 writers) move to the full tier
    "narrow": dict(lds_seg_capacity=16, page_capacity=256, unsettled_capacity=2048, page_heap_capacity=2048,
                   lds_page_capacity=200, lds_unsettled_capacity=600, lds_page_heap_capacity=600,
                   lds_narrow_overlap=1),
    # HBM paged capacities far below the documents' needs: the growth step moves documents
    # to larger regions, round after round, mid-batch (mt_last_grown)
    "grow": dict(lds_seg_capacity=16, page_capacity=12, unsettled_capacity=16, page_heap_capacity=16),
}


@pytest.mark.parametrize("tier", list(TIERS))
@pytest.mark.parametrize("name", gu.ALL_FIXTURES)
def test_gpu_matches_reference(name, tier):
    fx = gu.load(name)
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    mt = _gpu_batch(len(fx["docs"]), **TIERS[tier])
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    bad = []
    for i, doc in enumerate(fx["docs"]):
        errs = gu.compare_oracle(_gpu_outputs(mt, i), gu.expected(doc, interner))
        if errs:
            bad.append((doc["doc"], errs))
    assert not bad, f"{name}: {bad[:4]}"
    paged = [mt.is_paged(i) for i in range(len(fx["docs"]))]
    if tier == "paged":
        assert all(paged)
    elif "paged" not in tier and tier not in ("tight", "narrow", "grow"):
        assert not any(paged)


@pytest.mark.parametrize("tier", ["lds", "paged", "tight", "grow"])
def test_gpu_skewed_batch_longest_first(tier):
    """A batch whose documents differ in length (60 to 10k messages, interleaved) is
    dispatched longest first (mt_batch.order, DevState.order): every tier's launches serve
    their documents through the permutation, and each document equals the reference."""
    small, c3, full = gu.load("ref_small"), gu.load("ref_c3"), gu.load("ref_c3_full")
    interner = gu.interner_for(small)
    docs = []
    for k in range(4):
        docs += small["docs"][3 * k:3 * k + 3] + [c3["docs"][k], full["docs"][k]]
    a = gu.encode_docs(small, interner, docs)
    lens = np.diff(a["doc_off"])
    assert len(set(lens.tolist())) >= 3
    mt = _gpu_batch(len(docs), delta_log_capacity=1 << 20, **TIERS[tier])
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    assert (mt.status() == 0).all(), mt.status()
    bad = []
    for i, doc in enumerate(docs):
        errs = gu.compare_oracle(_gpu_outputs(mt, i), gu.expected(doc, interner))
        if errs:
            bad.append((i, errs))
    assert not bad, bad[:4]


def test_gpu_generator_per_document_lengths(oracle_lib):
    """mt_generate_docs: document d's stream is the first ops_per_doc[d] messages of the
    mt_generate stream of its global index doc_ids[d] (the C restatement's generator at that
    length and index), and the skewed batch replays, longest first, to the generated state."""
    import json
    import os
    cfg = dict(json.load(open(os.path.join(gu.GOLDEN, "..", "..", "bench", "configs.json")))["c3"], ops=3000)
    lens = np.array([40, 3000, 700, 1, 0, 2200, 150, 1200], dtype=np.int32)
    ids = np.array([9, 3, 40, 7, 1, 12, 2, 100], dtype=np.int32)   # global indices (the draws)
    mt = _gpu_batch(len(lens), **TIERS["tight"])
    b = mt.generate(cfg, ops_per_doc=lens, doc_ids=ids)
    got = b.download()
    assert np.array_equal(np.diff(got["doc_off"]), lens)
    gsums = mt.checksums()
    for d, n in enumerate(lens):
        g = oracle_lib.generate(dict(cfg, ops=int(n)), int(ids[d]), keep=True)
        lo, hi = got["doc_off"][d], got["doc_off"][d + 1]
        f = ["seq", "ref_seq", "min_seq", "pos1", "pos2", "client", "kind"]
        assert np.array_equal(got["ops"][lo:hi][f], g["ops"][f]), d
        osum = g["doc"].outputs()["checksum"]
        for k in ("length", "text_hash", "props_hash", "delta_hash"):
            assert gsums[d][k] == osum[k], (d, k)
    seed_off, seed = mt.generated_seeds(cfg, doc_ids=ids)
    mt.load_initial_text(seed_off, seed)
    b.apply_async()
    mt.sync()
    assert np.array_equal(mt.checksums(), gsums)


# the growth step also raises the text / property arenas and the uid -> page map
GROW_EXTRA = {"pages": {}, "text": dict(text_capacity=1024), "props": dict(props_capacity=96),
              "uids": dict(uid_capacity=256)}


@pytest.mark.parametrize("name,extra", [(n, "pages") for n in ("ref_c3_full", "ref_c4_full", "ref_c3_long")] +
                         [(n, e) for n in ("ref_c3_full", "ref_c4_full") for e in ("text", "props", "uids")])
def test_gpu_growth_past_the_handle_sizing(name, extra):
    """Documents far larger than the handle's paged capacities (12 pages, 16 table / heap
    entries; the 10k-op C3 / C4 documents need ~200 pages, ~200-1800 entries) -- and, per
    case, its text arena, property records or uid map -- are moved to larger HBM regions by
    the growth step, several times, mid-batch; they end equal to the reference -- text, tree,
    segments, properties, every delta record -- and so does a second batch on the same
    handle."""
    fx = gu.load(name)
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    mt = _gpu_batch(len(fx["docs"]), delta_log_capacity=1 << 20, **TIERS["grow"], **GROW_EXTRA[extra])
    mt.load_initial_text(a["seed_off"], a["seed"])
    half = np.asarray([lo + (hi - lo) // 2 for lo, hi in zip(a["doc_off"][:-1], a["doc_off"][1:])])
    sel1 = np.concatenate([np.arange(lo, m) for lo, m in zip(a["doc_off"][:-1], half)])
    sel2 = np.concatenate([np.arange(m, hi) for m, hi in zip(half, a["doc_off"][1:])])
    off1 = np.concatenate([[0], np.cumsum(half - a["doc_off"][:-1])]).astype(np.int64)
    off2 = np.concatenate([[0], np.cumsum(a["doc_off"][1:] - half)]).astype(np.int64)
    mt.apply_arrays(dict(a, ops=a["ops"][sel1], doc_off=off1))
    g1 = mt.last_grown()
    assert g1["grown"] >= len(fx["docs"]) and g1["rounds"] >= 2, g1
    mt.apply_arrays(dict(a, ops=a["ops"][sel2], doc_off=off2))
    g2 = mt.last_grown()
    assert g2["in_big_region"] == len(fx["docs"]), g2
    assert (mt.status() == 0).all()
    bad = []
    for i, doc in enumerate(fx["docs"]):
        errs = gu.compare_oracle(_gpu_outputs(mt, i), gu.expected(doc, interner))
        if errs:
            bad.append((doc["doc"], errs))
    assert not bad, f"{name}: {bad[:4]}"


@pytest.mark.parametrize("tier", ["lds", "paged"])
@pytest.mark.parametrize("name", ["ref_c3", "ref_ext", "ref_ext_long"])
def test_gpu_checksums_match_oracle(oracle_lib, name, tier):
    fx = gu.load(name)
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    mt = _gpu_batch(len(fx["docs"]), **TIERS[tier])
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    sums = mt.checksums()
    osums, ost = oracle_lib.replay_batch(a, threads=2)
    assert (ost == 0).all()
    for f in ("length", "text_hash", "props_hash", "delta_hash", "n_segments"):
        assert np.array_equal(sums[f], osums[f]), f


@pytest.mark.parametrize("tier", ["lds", "tiny_paged"])
def test_gpu_split_batches_equal_single_batch(oracle_lib, tier):
    """Applying a document's messages in several calls equals one call (state persists)."""
    fx = gu.load("ref_c2")
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    mt1 = _gpu_batch(len(fx["docs"]))
    mt1.load_initial_text(a["seed_off"], a["seed"])
    mt1.apply_arrays(a)
    mt2 = _gpu_batch(len(fx["docs"]), **TIERS[tier])
    mt2.load_initial_text(a["seed_off"], a["seed"])
    off = a["doc_off"]
    for lo_frac, hi_frac in ((0.0, 0.3), (0.3, 0.31), (0.31, 1.0)):
        sel, noff = [], [0]
        for d in range(len(off) - 1):
            n = off[d + 1] - off[d]
            lo, hi = off[d] + int(n * lo_frac), off[d] + int(n * hi_frac)
            sel.append(np.arange(lo, hi))
            noff.append(noff[-1] + hi - lo)
        idx = np.concatenate(sel)
        mt2.apply_arrays(dict(a, ops=a["ops"][idx], doc_off=np.asarray(noff, dtype=np.int64)))
    s1, s2 = mt1.checksums(), mt2.checksums()
    assert np.array_equal(s1, s2)
    if tier == "tiny_paged":
        assert any(mt2.is_paged(i) for i in range(len(fx["docs"])))


@pytest.mark.parametrize("tier", list(TIERS))
@pytest.mark.parametrize("name", gu.MAINT_FIXTURES)
def test_gpu_maintenance_events_match_reference(name, tier):
    """mergeTreeMaintenanceCallback SPLIT / APPEND / UNLINK counts per document equal the
    reference's own callback (tests/golden/ref_maint.json) on every storage tier."""
    fx = gu.load(name)
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    mt = _gpu_batch(len(fx["docs"]), **TIERS[tier])
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    assert (mt.status() == 0).all()
    got = mt.maintenance_counts().tolist()
    assert got == gu.maint_counts(name), name


@pytest.mark.parametrize("tier", ["lds", "hbm", "paged", "tiny_paged", "tight", "narrow"])
@pytest.mark.parametrize("cfgname,ops,docs", [("c2", 400, 16), ("c3", 400, 16), ("c4", 500, 6), ("c3", 3000, 4),
                                              ("c4w", 1500, 4), ("c4x", 3000, 2)])
def test_gpu_generator_matches_oracle(oracle_lib, cfgname, ops, docs, tier):
    import json
    import os
    if ops > 1000 and tier in ("hbm", "lds"):
        pytest.skip("long streams: paged tiers only")
    configs = json.load(open(os.path.join(gu.GOLDEN, "..", "..", "bench", "configs.json")))
    # c4w: 200 writers -- overlapping removes by short ids far above 64 (reused overlap slots);
    # c4x: lag 400 -- more clients overlapping at once than the 63 slots (overflow sets)
    cfg = {"c4w": dict(configs["c4"], writers=200, lag=100),
           "c4x": dict(configs["c4"], writers=200, lag=400)}.get(cfgname) or configs[cfgname]
    cfg = dict(cfg, ops=ops)
    caps = dict(TIERS[tier])
    if cfgname == "c4x":   # (the generator has no growth step: ~3.2k unsettled segments at lag 400)
        caps.update(unsettled_capacity=4096, page_heap_capacity=2048)
    mt = _gpu_batch(docs, **caps)
    b = mt.generate(cfg)
    got = b.download()
    gsums = mt.checksums()
    omaint = []
    # the arenas are packed document after document (u32 offsets address the whole batch):
    # every insert's payload follows the previous one, and nothing is left between them
    ops_all = got["ops"]
    ins = ops_all["kind"] == 0
    assert np.array_equal(ops_all["payload"][ins][1:], (ops_all["payload"][ins] + ops_all["pos2"][ins])[:-1])
    assert len(got["text"]) == int(ops_all["pos2"][ins].sum())
    withp = ops_all["props"] != 0xFFFFFFFF
    assert np.all(np.diff(ops_all["props"][withp].astype(np.int64)) > 0)
    for d in range(docs):
        g = oracle_lib.generate(cfg, d, keep=True)
        lo, hi = got["doc_off"][d], got["doc_off"][d + 1]
        ops_d = got["ops"][lo:hi].copy()
        assert np.array_equal(ops_d[["seq", "ref_seq", "min_seq", "pos1", "pos2", "client", "kind"]],
                              g["ops"][["seq", "ref_seq", "min_seq", "pos1", "pos2", "client", "kind"]]), d
        gi = ops_d["kind"] == 0
        for op, oop in zip(ops_d[gi][:50], g["ops"][gi][:50]):   # the payload text equals the oracle's
            assert np.array_equal(got["text"][op["payload"]:op["payload"] + op["pos2"]],
                                  g["text"][oop["payload"]:oop["payload"] + oop["pos2"]]), d
        osum = g["doc"].outputs()["checksum"]
        for f in ("length", "text_hash", "props_hash", "delta_hash"):
            assert gsums[d][f] == osum[f], (d, f)
        omaint.append(g["doc"].maintenance())
    # replaying the generated batch from the seeds reproduces the same final state
    seed_off, seed = mt.generated_seeds(cfg)
    mt.load_initial_text(seed_off, seed)
    b.apply_async()
    mt.sync()
    assert np.array_equal(mt.checksums(), gsums)
    # the generator kernels keep no event counts; the (delta-logging) replay does
    assert mt.maintenance_counts().tolist() == omaint


# summary headers larger than the flat capacities (48 segments) on a paged handle: staged by
# k_load_header and paged by k_load_convert at load
SNAP_TIERS = dict(TIERS, paged_load=dict(seg_capacity=48, lds_seg_capacity=16, props_capacity=4096,
                                         page_capacity=256, unsettled_capacity=2048, page_heap_capacity=2048))


@pytest.mark.parametrize("tier", ["lds", "hbm", "paged", "tiny_paged", "paged_load"])
@pytest.mark.parametrize("name", gu.SNAP_FIXTURES)
def test_gpu_snapshot_load_matches_reference(name, tier):
    """Config C5 (cold catch-up) through mt_load_snapshots: after the load the device tree
    equals the reference's (reloadFromSegments shape, body appends, segments, properties);
    after the tail the outputs and every delta callback equal the reference's; summaries the
    reference fails to load fail with the same status."""
    fx = gu.load(name)
    docs = fx["docs"]   # every reference-made document (snap_status models each one)
    interner = gu.Interner()
    la, oa = gu.encode_snap_docs(fx, interner, docs)
    mt = _gpu_batch(len(docs), **SNAP_TIERS[tier])
    mt.load_snapshots(la)
    st = mt.status()
    if tier == "paged_load":   # the large headers were paged at load
        big = [i for i in range(len(docs)) if la["n_header"][i] > 48 and st[i] == 0]
        assert big and all(mt.is_paged(i) for i in big)
    bad = []
    for i, doc in enumerate(docs):
        want = gu.snap_status(doc)
        if want:
            if st[i] != want:
                bad.append((doc["doc"], "load status", int(st[i])))
            continue
        errs = gu.compare_oracle(_gpu_outputs(mt, i), gu.expected_snap(doc, interner, "load_out"))
        if errs:
            bad.append((doc["doc"], "after load", errs))
    assert not bad, f"{name}: {bad[:4]}"
    mt.apply_arrays(oa)
    for i, doc in enumerate(docs):
        if gu.snap_status(doc):
            continue
        errs = gu.compare_oracle(_gpu_outputs(mt, i), gu.expected_snap(doc, interner))
        if errs:
            bad.append((doc["doc"], errs))
    assert not bad, f"{name}: {bad[:4]}"


@pytest.mark.parametrize("tier", ["lds", "paged"])
@pytest.mark.parametrize("name", gu.SNAP_FIXTURES)
def test_gpu_summaries_native_decoder_match_reference(name, tier):
    """MergeTreeBatch.load_summaries: the reference-written blobs decoded by the native
    decoder (libmtsnapdec.so) and loaded; catch-up + tail ops continue its client maps.  The
    tree after the tail equals the reference's."""
    from fluidframework_amd.wire import Batch
    fx = gu.load(name)
    docs = [d for d in fx["docs"] if gu.snap_status(d) == 0]
    interner = gu.Interner()
    mt = _gpu_batch(len(docs), **SNAP_TIERS[tier])
    catchup, clients = mt.load_summaries([d["chunks"] for d in docs], interner, threads=4)
    assert (mt.status() == 0).all()
    b = Batch(interner)
    for d, cu, cl in zip(docs, catchup, clients):
        b.add_doc("", list(cu) + gu.compact_msgs_to_dicts(d.get("tail", [])), clients=cl)
    mt.apply_arrays(b.arrays())
    bad = []
    for i, doc in enumerate(docs):
        errs = gu.compare_oracle(_gpu_outputs(mt, i), gu.expected_snap(doc, interner))
        if errs:
            bad.append((doc["doc"], errs))
    assert not bad, f"{name}: {bad[:4]}"


@pytest.mark.parametrize("slice_docs", [1, 7])
@pytest.mark.parametrize("tier", ["lds", "paged", "paged_load"])
def test_gpu_catch_up_in_slices_matches_reference(tier, slice_docs):
    """MergeTreeBatch.catch_up: the reference-written summaries decoded slice by slice on a
    host thread while earlier slices load into their document ranges on the GPU
    (mt_snapshots_upload_range); every document, whatever its status (Q6 failures,
    MT_DOC_ALIASED), ends as load_summaries leaves it, and after the tails as the reference."""
    from fluidframework_amd.wire import Batch
    fx = gu.load("ref_snap_body")
    docs = fx["docs"]
    ref_i, got_i = gu.Interner(), gu.Interner()
    ref = _gpu_batch(len(docs), **SNAP_TIERS[tier])
    got = _gpu_batch(len(docs), **SNAP_TIERS[tier])
    cu_r, cl_r = ref.load_summaries([d["chunks"] for d in docs], ref_i, threads=4)
    cu_g, cl_g = got.catch_up([d["chunks"] for d in docs], got_i, threads=3, slice_docs=slice_docs)
    assert cu_r == cu_g and cl_r == cl_g
    assert np.array_equal(ref.status(), got.status())
    assert np.array_equal(ref.checksums(), got.checksums())
    assert got.last_load_ms() > 0   # (HIP events around the last slice's load kernels)
    ok = [i for i, d in enumerate(docs) if gu.snap_status(d) == 0]
    b = Batch(got_i)
    for i, d in enumerate(docs):
        b.add_doc("", (list(cu_g[i]) + gu.compact_msgs_to_dicts(d.get("tail", []))) if i in ok else [],
                  clients=cl_g[i])
    got.apply_arrays(b.arrays())
    bad = []
    for i in ok:
        errs = gu.compare_oracle(_gpu_outputs(got, i), gu.expected_snap(docs[i], got_i))
        if errs:
            bad.append((docs[i]["doc"], errs))
    assert not bad, bad[:4]


@pytest.mark.parametrize("tier", ["lds", "paged"])
@pytest.mark.parametrize("name", ["ref_snap", "ref_snap_body"])
def test_gpu_snapshot_emission_matches_reference(name, tier):
    """SnapshotV1 emission from device state (mt_extract_snapshots = extractSync, then
    snapshot.encode_chunks = emit): the summary of the replayed observer equals, byte for
    byte, the one the reference wrote for the same op stream."""
    from fluidframework_amd.snapshot import encode_chunks, record_specs
    from fluidframework_amd.wire import Batch, compact_msgs_to_dicts
    fx = gu.load(name)
    interner = gu.Interner()
    b = Batch(interner)
    for doc in fx["docs"]:
        b.add_doc(doc["seed_text"], compact_msgs_to_dicts(doc["msgs"]))
    a = b.arrays()
    mt = _gpu_batch(len(fx["docs"]), **TIERS[tier])
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    assert (mt.status() == 0).all()
    snaps = mt.extract_snapshots()
    for i, doc in enumerate(fx["docs"]):
        names = {v: k for k, v in b.clients[i].items()}
        s = snaps[i]
        specs, lengths = record_specs(s["segs"], s["text"], s["props"], interner, names)
        got = encode_chunks(specs, lengths, s["min_seq"], s["cur_seq"], fx["config"]["chunk"])
        assert got == doc["chunks"], (name, doc["doc"])


@pytest.mark.parametrize("tier", ["lds", "hbm", "paged"])
def test_gpu_start_collaboration_window(tier):
    """startOrUpdateCollaboration(id, minSeq, currentSeq): a stream whose sequence numbers are
    all shifted by K, replayed from window (K, K), ends in the same text, properties and
    segments as the unshifted one from (0, 0); a message at or below the window's
    currentSeq / minSeq fails as the reference's asserts (client.ts:824-826,
    mergeTree.ts:1752-1755)."""
    fx = gu.load("ref_c3")
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    n = len(fx["docs"])
    K = 1000
    base = _gpu_batch(n, **TIERS[tier])
    base.load_initial_text(a["seed_off"], a["seed"])
    base.apply_arrays(a)
    sh = dict(a, ops=a["ops"].copy())
    for f in ("seq", "ref_seq", "min_seq"):
        sh["ops"][f] += K
    mt = _gpu_batch(n, **TIERS[tier])
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.start_collaboration(np.full(n, K, np.int32), np.full(n, K, np.int32))
    mt.apply_arrays(sh)
    assert (mt.status() == 0).all()
    s0, s1 = base.checksums(), mt.checksums()
    for f in ("length", "text_hash", "props_hash", "n_segments"):
        assert np.array_equal(s0[f], s1[f]), f
    for d in range(n):
        assert mt.get_text(d) == base.get_text(d)
    # the unshifted stream against window (K, K): its first message is not above currentSeq
    bad = _gpu_batch(n, **TIERS[tier])
    bad.load_initial_text(a["seed_off"], a["seed"])
    bad.start_collaboration(np.full(n, K, np.int32), np.full(n, K, np.int32))
    bad.apply_arrays(a)
    assert (bad.status() == 2).all()   # MT_DOC_SEQ_ORDER, client.ts:462-463
    # a stream above the window's currentSeq whose minSeq is below the window's minSeq
    low = dict(sh, ops=sh["ops"].copy())
    low["ops"]["seq"] += K
    mt2 = _gpu_batch(n, **TIERS[tier])
    mt2.load_initial_text(a["seed_off"], a["seed"])
    mt2.start_collaboration(np.full(n, 2 * K, np.int32), np.full(n, 2 * K, np.int32))
    mt2.apply_arrays(low)
    assert (mt2.status() == 3).all()   # MT_DOC_MINSEQ_ORDER, client.ts:464-465
    with pytest.raises(RuntimeError):
        mt2.start_collaboration(np.full(n, 5, np.int32), np.full(n, 4, np.int32))


OVF_TIERS = dict({t: TIERS[t] for t in ("paged", "tiny_paged", "tight", "narrow", "grow")},
                 # a 64-unit overflow arena: handed to the growth step (cause 11) again and again
                 grow_arena64=dict(TIERS["grow"], overlap_arena_capacity=64),
                 tight_arena64=dict(TIERS["tight"], overlap_arena_capacity=64))


@pytest.mark.parametrize("tier", list(OVF_TIERS))
def test_gpu_overlap_beyond_the_slots_matches_reference(tier):
    """More clients whose overlapping removes are unsettled at once than the 63 overlap slots
    (200 writers, lag 400: ~80; removedClientOverlap is an unbounded list, MT/mergeTree.ts:
    2577-2585): paged documents keep the segments' whole lists in overflow sets, and the
    documents equal the reference's (tests/golden/ref_wide400) -- every tier that meets them,
    the growth step included (its overflow arena grows with the document)."""
    fx = gu.load("ref_wide400")
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    mt = _gpu_batch(len(fx["docs"]), **OVF_TIERS[tier])
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    assert (mt.status() == 0).all(), mt.status()
    if tier.endswith("arena64"):
        assert mt.last_grown()["in_big_region"] == len(fx["docs"])
    bad = []
    for i, doc in enumerate(fx["docs"]):
        errs = gu.compare_oracle(_gpu_outputs(mt, i), gu.expected(doc, interner))
        if errs:
            bad.append((doc["doc"], errs))
    assert not bad, bad[:4]


@pytest.mark.parametrize("tier", ["paged", "tight", "grow"])
def test_gpu_overflow_sets_are_reclaimed(oracle_lib, tier):
    """removedClientOverlap lists leave with their segments (zamboni unlinks or merges them,
    MT/mergeTree.ts:1322-1398).  Over a 60k-message document with 200 writers at lag 400
    (tests/golden/ref_wide_long, made by the reference) overflow sets are made all along, few
    live at once: the arena's halves are compacted (pg_ovf_compact), so from a 512-unit start
    the most units the half in use ever holds stays within twice the peak of the reference's
    live lists (the C restatement's count of every removedClientOverlap list in the tree after
    each message, as [n, ids...] units), the arena within four times it -- far below the units
    made over the document's life -- and the document equals the reference's."""
    fx = gu.load("ref_wide_long")
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    od = oracle_lib.OracleDoc.new(a["seed"][: a["seed_off"][1]])
    od.apply_all(a["ops"], a["text"], a["props"])
    peak_live = od.overlap_units()[1]
    mt = _gpu_batch(len(fx["docs"]), delta_log_capacity=1 << 21, overlap_arena_capacity=512,
                    **OVF_TIERS[tier])
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    assert (mt.status() == 0).all(), mt.status()
    for i, doc in enumerate(fx["docs"]):
        assert not gu.compare_oracle(_gpu_outputs(mt, i), gu.expected(doc, interner)), doc["doc"]
        ar = mt.get_overlap_arena(i)
        print(tier, ar, mt.last_grown())
        assert ar["largest_set"] >= 2                 # sets were made (clients beyond the 63 slots)
        assert ar["made"] > 2 * ar["capacity"], ar    # far more than the arena ever held: reclaimed
        assert ar["live_units"] <= ar["fill"]
        assert ar["peak_fill"] <= 2 * peak_live, (ar, peak_live)
        assert ar["capacity"] <= max(512, 4 * peak_live), (ar, peak_live)


# ---------------------------------------------------------------- error model
@pytest.mark.parametrize("tier", list(TIERS))
def test_gpu_error_model_matches_reference(tier):
    """Faulted streams (tests/golden/ref_errors, made by the reference): each document stops
    with the status of the reference's throw -- completeAndLogOp (MT/client.ts:462-465),
    updateSeqNumbers (:824-826), setMinSeq (MT/mergeTree.ts:1755) -- and its state at that
    point (the op applied, zamboni run, every delta record) equals the reference's at the
    throw; the other documents of the batch are unaffected."""
    fx = gu.load("ref_errors")
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    mt = _gpu_batch(len(fx["docs"]), **TIERS[tier])
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    bad = []
    for i, doc in enumerate(fx["docs"]):
        errs = gu.compare_oracle(_gpu_outputs(mt, i), gu.expected(doc, interner), status=gu.error_status(doc))
        if errs:
            bad.append((doc["doc"], doc["fault"], errs))
    assert not bad, bad[:4]


def test_gpu_text_arena_grows_with_the_document():
    """Documents whose text outgrows the handle's arena (~2.9k-unit documents, 1024 units per
    half; TextSegment.append is unbounded, MT/textSegment.ts:74-85) are handed to the growth
    step between messages and continue with a doubled arena in the big region; every document
    of the batch equals the reference."""
    small, big = gu.load("ref_small"), gu.load("ref_c3")
    interner = gu.interner_for(small)
    docs = small["docs"][:6] + big["docs"][:2]
    a = gu.encode_docs(small, interner, docs)
    mt = _gpu_batch(len(docs), lds_seg_capacity=-1, page_capacity=16, unsettled_capacity=1024, text_capacity=1024)
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    assert (mt.status() == 0).all(), mt.status()
    assert mt.last_grown()["in_big_region"] >= 2
    for i, doc in enumerate(docs):
        assert not gu.compare_oracle(_gpu_outputs(mt, i), gu.expected(doc, interner)), i


# ---------------------------------------------------------------- full-length streams
def _bench_caps(fx):
    import bench
    cfg = dict(fx["config"])
    return bench.capacities(cfg)


@pytest.mark.parametrize("name", gu.FULL_FIXTURES)
def test_gpu_full_streams_fast_path(oracle_lib, name):
    """The replay fast path the bench times -- no delta log, the bench's own capacities (C3:
    the tight tier with its capacities fixed at compile time) -- on the reference's full
    10k-message streams: text, segments, leaf partition and properties equal the reference's,
    and every checksum (delta hash included) equals the C restatement's."""
    fx = gu.load(name)
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    mt = _gpu_batch(len(fx["docs"]), delta_log_capacity=0, **_bench_caps(fx))
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    assert (mt.status() == 0).all()
    osums, ost = oracle_lib.replay_batch(a, threads=2)
    assert (ost == 0).all() and np.array_equal(mt.checksums(), osums)
    for i, doc in enumerate(fx["docs"]):
        exp = dict(gu.expected(doc, interner), deltas=None)   # no delta log: its hash is checked above
        rows, leaves = mt.get_segments(i)
        got = dict(text=mt.get_text(i), length=mt.get_length(i), leaves=leaves, segs=rows,
                   seg_props=mt.get_all_segment_props(i), deltas=None,
                   status=int(mt.status()[i]))
        assert not gu.compare_oracle(got, exp), i


@pytest.mark.parametrize("name", gu.ALL_FIXTURES + ["ref_c3_long", "ref_c3_60k", "ref_wide400"])
def test_gpu_c3_tight_tier_matches_reference(oracle_lib, name):
    """The bench's C3 tight tier (mt_replay.hip launch_paged: P_C3, capacities fixed at compile
    time, 32-bit overlap masks) behind a 16-segment LDS tier, so every document of every
    fixture passes through it -- converted from the flat tier, handed over when it outgrows 192
    pages / 220 entries or its clients above 32 overlap -- with no delta log: text, segments,
    leaf partition and property sets equal the reference's and every checksum (delta hash
    included) the C restatement's."""
    import json
    import os
    import bench
    fx = gu.load(name)
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    cfg = dict(json.load(open(os.path.join(bench.REPO, "bench", "configs.json")))["c3"], ops=10000)
    caps = dict(bench.capacities(cfg), lds_seg_capacity=16)
    assert (caps["lds_page_capacity"], caps["lds_unsettled_capacity"], caps["lds_page_heap_capacity"]) == (192, 220, 192)
    mt = _gpu_batch(len(fx["docs"]), delta_log_capacity=0, **caps)
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    osums, ost = oracle_lib.replay_batch(a, threads=2)
    assert np.array_equal(mt.status(), ost)
    assert np.array_equal(mt.checksums(), osums)
    bad = []
    for i, doc in enumerate(fx["docs"]):
        exp = dict(gu.expected(doc, interner), deltas=None)
        got = dict(_gpu_outputs_nolog(mt, i), deltas=None)
        errs = gu.compare_oracle(got, exp, status=int(ost[i]))
        if errs:
            bad.append((doc["doc"], errs))
    assert not bad, bad[:4]


@pytest.mark.parametrize("name", gu.FULL_FIXTURES)
def test_gpu_full_streams_at_bench_capacities(name):
    """The configs' full stream lengths (10k messages per document, made by the reference)
    replayed with exactly the capacities bench.py runs (C3: paged LDS capacities 192/220/192,
    C4: 256/2048/1024): every output and every delta record equals the reference's."""
    fx = gu.load(name)
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    caps = _bench_caps(fx)
    mt = _gpu_batch(len(fx["docs"]), delta_log_capacity=1 << 19, **caps)
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    bad = []
    for i, doc in enumerate(fx["docs"]):
        errs = gu.compare_oracle(_gpu_outputs(mt, i), gu.expected(doc, interner))
        if errs:
            bad.append((doc["doc"], errs))
    assert not bad, f"{name} at {caps}: {bad}"
    assert all(mt.is_paged(i) for i in range(len(fx["docs"])))
    assert mt.maintenance_counts().tolist() == gu.maint_counts(name)


# ---------------------------------------------------------------- delta log bounds
def test_gpu_delta_log_overflow_keeps_whole_records():
    """A delta log smaller than the stream: the kept records are whole and equal the
    reference's first records; the read reports the overflow (MT_E_OVERFLOW) instead of
    handing out a header without its entries; a reset empties it."""
    from fluidframework_amd import DeltaLogOverflow
    fx = gu.load("ref_ext")
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    mt = _gpu_batch(len(fx["docs"]), delta_log_capacity=301)
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    for i, doc in enumerate(fx["docs"]):
        want = gu.expected(doc, interner)["deltas"]
        with pytest.raises(DeltaLogOverflow) as ei:
            mt.get_delta_log(i)
        kept = ei.value.records
        assert 0 < len(kept) <= 301 and kept == want[: len(kept)]
        # the kept words end exactly at a record boundary
        j = 0
        while j < len(kept):
            seq, kind, n = kept[j: j + 3]
            j += 3
            for _ in range(n):
                j += 2
                if kind == 2:
                    j += 1 + 2 * kept[j]
        assert j == len(kept)
    assert (mt.status() == 0).all()
    mt.delta_log_reset()
    mt.sync()
    assert mt.get_delta_log(0) == []


# ---------------------------------------------------------------- C-ABI input validation
def test_gpu_abi_rejects_out_of_bounds_batches():
    """Malformed batches fail with MT_E_INVALID on the host instead of faulting the device:
    non-monotonic or oversized offsets, payloads / props records outside their arenas."""
    fx = gu.load("ref_small")
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    mt = _gpu_batch(len(fx["docs"]))
    mt.load_initial_text(a["seed_off"], a["seed"])
    ins = np.nonzero(a["ops"]["kind"] == 0)[0][0]
    cases = []
    off = a["doc_off"].copy()
    off[3], off[4] = off[4], off[3]
    cases.append(dict(a, doc_off=off))
    off = a["doc_off"].copy()
    off[-1] += 5
    cases.append(dict(a, doc_off=off))
    ops = a["ops"].copy()
    ops[ins]["payload"] = len(a["text"])
    cases.append(dict(a, ops=ops))
    ops = a["ops"].copy()
    ops[ins]["props"] = len(a["props"]) + 7
    cases.append(dict(a, ops=ops))
    ops = a["ops"].copy()
    ops[ins]["kind"] = 9
    cases.append(dict(a, ops=ops))
    for c in cases:
        with pytest.raises(RuntimeError, match=r"\(-1\)"):
            mt.apply_arrays(c)
    mt.apply_arrays(a)   # the handle is still usable
    assert (mt.status() == 0).all()
    for i, doc in enumerate(fx["docs"]):
        assert not gu.compare_oracle(_gpu_outputs(mt, i), gu.expected(doc, interner)), i


# ---------------------------------------------------------------- drop-in ceilings
def test_gpu_tight_tier_hands_documents_over():
    """LDS capacities of the tight paged tier far below the documents' peaks: the library
    moves each document to the full-capacity launch before the message that could outgrow
    them (no generation fallback in the caller); every output equals the reference's."""
    fx = gu.load("ref_c3_full")
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    caps = dict(_bench_caps(fx), lds_page_capacity=40, lds_unsettled_capacity=64, lds_page_heap_capacity=64)
    mt = _gpu_batch(len(fx["docs"]), delta_log_capacity=1 << 19, **caps)
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    assert mt.last_paged_peaks()["tight_handovers"] == len(fx["docs"])
    for i, doc in enumerate(fx["docs"]):
        assert not gu.compare_oracle(_gpu_outputs(mt, i), gu.expected(doc, interner)), i


@pytest.mark.parametrize("lds_tier", [True, False])
def test_gpu_sliced_paged_schedule_matches_reference(lds_tier):
    """mt_options.paged_slices: more documents than one tight paged launch holds at once
    (4 reference documents x 800 replicas = 3200 > 3072 resident), so the paged replay runs
    as slices that each leave a window of documents out, then a last unlimited launch.  Every
    replica's checksum equals the unsliced replay's, and sampled replicas equal the
    reference's outputs.  Without the LDS tier (lds_seg_capacity -1) nothing has set the
    documents' resume points before the first slice: every slice after it must still resume,
    not restart."""
    fx = gu.load("ref_c3_full")
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    k = 800
    nd = len(fx["docs"]) * k
    lens = np.diff(a["doc_off"])
    rep = dict(a)
    rep["ops"] = np.tile(a["ops"], k)
    rep["doc_off"] = np.concatenate([[0], np.cumsum(np.tile(lens, k))]).astype(np.int64)
    slen = np.diff(a["seed_off"])
    seed_off = np.concatenate([[0], np.cumsum(np.tile(slen, k))]).astype(np.int64)
    seed = np.tile(a["seed"], k)
    caps = dict(_bench_caps(fx))
    if not lds_tier:
        caps["lds_seg_capacity"] = -1
    sums = {}
    for slices in (0, 8):
        mt = _gpu_batch(nd, delta_log_capacity=0, paged_slices=slices, **caps)
        mt.load_initial_text(seed_off, seed)
        mt.apply_arrays(rep)
        assert (mt.status() == 0).all()
        sums[slices] = mt.checksums()
        if slices:
            for i in (0, 1, nd - 130, nd - 1):   # first / last windows and the tail
                out = _gpu_outputs(mt, i)
                out["deltas"] = gu.expected(fx["docs"][i % 4], interner)["deltas"]   # no log on this handle
                assert not gu.compare_oracle(out, gu.expected(fx["docs"][i % 4], interner)), i
        del mt
    assert sums[0].tobytes() == sums[8].tobytes()
    assert all(sums[8][i].tobytes() == sums[8][i % 4].tobytes() for i in range(nd))


@pytest.mark.parametrize("uid_capacity,text_capacity", [(65536, 1 << 17), (16384, 1 << 17), (16384, 4096)])
def test_gpu_long_documents_match_reference(uid_capacity, text_capacity):
    """30k-message documents (~45k segment ids created, ~10.5k live segments at the end):
    segment ids are renumbered when the uid -> page map runs out (uid_capacity 16384 forces
    it several times), and every output still equals the reference's.  With a 4096-unit text
    arena the renumbering's scratch (the arena's idle half, 2 x pages int32) and the text
    itself both come from the growth step raising the arena (cause 4) as the document grows."""
    import bench
    fx = gu.load("ref_c3_long")
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    caps = dict(bench.capacities(dict(fx["config"])), uid_capacity=uid_capacity, text_capacity=text_capacity)
    mt = _gpu_batch(len(fx["docs"]), delta_log_capacity=1 << 20, **caps)
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    for i, doc in enumerate(fx["docs"]):
        assert not gu.compare_oracle(_gpu_outputs(mt, i), gu.expected(doc, interner)), i


# ---------------------------------------------------------------- rich callback stream
# (+ "hm": >= 512 pages, so the delta log runs on the kHM tier, P_HM_LOG)
RICH_TIERS = dict(TIERS, hm=dict(TIERS["paged"], page_capacity=600))


@pytest.mark.parametrize("tier", list(RICH_TIERS))
def test_gpu_rich_callback_stream_matches_reference(tier):
    """delta_log_mode 1: every mergeTreeDeltaCallback with its segments' state (text or marker,
    properties after the op) and every mergeTreeMaintenanceCallback (SPLIT / APPEND / UNLINK
    with the segments as the reference passes them, MT/mergeTree.ts:1343-1373, 2264-2269), in
    the reference's order -- compared with the reference's own callbacks (tests/golden/ref_rich)."""
    fx = gu.load("ref_rich")
    interner = gu.Interner()
    a = gu.encode_docs(fx, interner)
    mt = _gpu_batch(len(fx["docs"]), delta_log_mode=1, delta_log_capacity=1 << 20, **RICH_TIERS[tier])
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    assert (mt.status() == 0).all()
    for i, doc in enumerate(fx["docs"]):
        got, want = gu.parse_rich_log(mt.get_delta_log(i)), gu.expected_rich(doc, interner)
        bad = next((j for j, (x, y) in enumerate(zip(got, want)) if x != y), None)
        assert bad is None and len(got) == len(want), (doc["doc"], bad, len(got), len(want),
                                                       got[bad] if bad is not None else None,
                                                       want[bad] if bad is not None else None)
    # the maintenance records are not part of the delta hash
    plain = _gpu_batch(len(fx["docs"]), **RICH_TIERS[tier])
    plain.load_initial_text(a["seed_off"], a["seed"])
    plain.apply_arrays(a)
    assert np.array_equal(plain.checksums(), mt.checksums())


@pytest.mark.parametrize("name", ["ref_c3_full", "ref_c4_full", "ref_wide400", "ref_c3_long"])
def test_gpu_default_handle_is_unbounded(name):
    """A handle built with no capacity options (the drop-in default) takes documents of any
    size: the reference's MergeTree has no per-document ceiling (removedClientOverlap and
    TextSegment.append are unbounded, MT/mergeTree.ts:2577-2585, MT/textSegment.ts:74-85).  The
    10k-message C3 / C4 documents (~4k live segments), the 200-writer lag-400 streams (~80
    concurrent overlapping removers) and the 30k-message documents replay equal to the
    reference, the growth step raising whatever the small default starting capacities lack."""
    from fluidframework_amd import MergeTreeBatch
    fx = gu.load(name)
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    mt = MergeTreeBatch(len(fx["docs"]), delta_log_capacity=1 << 21)
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    assert (mt.status() == 0).all(), mt.status()
    bad = []
    for i, doc in enumerate(fx["docs"]):
        errs = gu.compare_oracle(_gpu_outputs(mt, i), gu.expected(doc, interner))
        if errs:
            bad.append((doc["doc"], errs))
    assert not bad, bad[:4]
    assert all(mt.is_paged(i) for i in range(len(fx["docs"])))


# (each capacity set once per fixture length: the 100k document at the 200k class's
# capacities and through growth from 12 pages, the 60k one at the uniform C3 and 100k class's)
XL_CASES = [("ref_c3_xl", "class_200k"), ("ref_c3_xl", "grow"), ("ref_c3_60k", "c3_bench"),
            ("ref_c3_60k", "class_100k"), ("ref_c3_200k", "class_200k")]


@pytest.mark.parametrize("name,caps", XL_CASES)
def test_gpu_xl_documents_match_reference(name, caps):
    """The skewed bench's long classes (c3skew: 40k-200k messages per document) pinned to the
    reference: a 60k- and a 100k-message C3 document (tests/golden/ref_c3_60k / ref_c3_xl, made
    by the reference) replayed at the capacities of the bench's 100k and 200k classes
    (bench_skew.class_caps: 1.6k / 3.2k pages, the two-level page search), at the uniform C3
    bench's (the tight tier hands them to the full tier, which hands them to the growth step
    as they pass 275 pages) and at the grow tier's (12 pages: growth round after round) --
    text, leaf partition, segment table, property sets and every delta record equal.  (At the
    class capacities, >= 512 pages, the delta log runs on the kHM tier: P_HM_LOG, and
    P_BIG_HM_LOG once growth passes 512 pages.)"""
    import json
    import os
    import bench
    import bench_skew
    fx = gu.load(name)
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    cfg = json.load(open(os.path.join(bench.REPO, "bench", "configs.json")))["c3skew"]
    kw = {"c3_bench": bench.capacities(dict(fx["config"], ops=10000)),
          "class_100k": bench_skew.class_caps(bench, cfg, 100000),
          "class_200k": bench_skew.class_caps(bench, cfg, 200000),
          "grow": TIERS["grow"]}[caps]
    mt = _gpu_batch(len(fx["docs"]), **dict(kw, delta_log_capacity=1 << 22))
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    assert (mt.status() == 0).all(), mt.status()
    bad = []
    for i, doc in enumerate(fx["docs"]):
        errs = gu.compare_oracle(_gpu_outputs(mt, i), gu.expected(doc, interner))
        if errs:
            bad.append((doc["doc"], errs))
    assert not bad, bad
    if caps in ("c3_bench", "grow"):
        assert mt.last_grown()["grown"] >= 1


# ---------------------------------------------------------------- HBM page metadata (kHM)
HM_CASES = {
    # the skewed bench's long classes: 1.6k / 3.2k pages from the start
    "class_100k": ("ref_c3_60k", lambda b, bs, cfg: bs.class_caps(b, cfg, 100000)),
    "class_200k": ("ref_c3_xl", lambda b, bs, cfg: bs.class_caps(b, cfg, 200000)),
    # the c3skew cap itself: a 200k-message document (~3k pages) at its class's capacities, and
    # grown from 12 pages round after round
    "class_200k_cap": ("ref_c3_200k", lambda b, bs, cfg: bs.class_caps(b, cfg, 200000)),
    "grow_200k": ("ref_c3_200k", lambda b, bs, cfg: TIERS["grow"]),
    # 12 pages at first: growth rounds until the big region passes 512 pages (P_BIG_HM)
    "grow_60k": ("ref_c3_60k", lambda b, bs, cfg: TIERS["grow"]),
    # more concurrent overlapping removers than the 63 slots: overflow sets on the kHM tier
    "wide_long": ("ref_wide_long", lambda b, bs, cfg: dict(TIERS["paged"], page_capacity=600)),
    "wide400": ("ref_wide400", lambda b, bs, cfg: dict(TIERS["paged"], page_capacity=512)),
}


@pytest.mark.parametrize("case", list(HM_CASES))
def test_gpu_hbm_page_metadata_matches_reference(case):
    """Documents of >= 512 pages without a delta log replay on the kHM tiers (mt_replay.hip
    use_hm: P_HM, P_BIG_HM), whose page metadata stays in HBM (LDS keeps one byte per page):
    text, leaf partition, segment table and property sets equal the reference's.  (With a
    delta log: test_gpu_xl_documents_match_reference, P_HM_LOG.)"""
    import json
    import os
    import bench
    import bench_skew
    name, kw_of = HM_CASES[case]
    fx = gu.load(name)
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    cfg = json.load(open(os.path.join(bench.REPO, "bench", "configs.json")))["c3skew"]
    kw = dict(kw_of(bench, bench_skew, cfg))
    kw["delta_log_capacity"] = 0
    mt = _gpu_batch(len(fx["docs"]), **kw)
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    assert (mt.status() == 0).all(), mt.status()
    bad = []
    for i, doc in enumerate(fx["docs"]):
        o = _gpu_outputs_nolog(mt, i)
        exp = dict(gu.expected(doc, interner))
        o["deltas"] = exp["deltas"]
        errs = gu.compare_oracle(o, exp)
        if errs:
            bad.append((doc["doc"], errs))
    assert not bad, bad
    if case in ("grow_60k", "grow_200k"):
        assert mt.last_grown()["grown"] >= 1


def _gpu_outputs_nolog(mt, doc):
    rows, leaves = mt.get_segments(doc)
    return dict(text=mt.get_text(doc), length=mt.get_length(doc), leaves=leaves, segs=rows,
                seg_props=mt.get_all_segment_props(doc), status=int(mt.status()[doc]))
