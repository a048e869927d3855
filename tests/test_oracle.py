"""Pins the CPU restatement oracle (oracle/mt_oracle.c) to the reference itself: every
golden fixture under tests/golden/ was produced by the reference's own MergeTree/Client
(transpiled by oracle/build_ref.py, driven by oracle/ref_harness.mjs)."""
import numpy as np
import pytest

import golden_util as gu


@pytest.mark.parametrize("name", gu.ALL_FIXTURES + gu.LONG_FIXTURES + gu.WIDE_FIXTURES + gu.XL_FIXTURES)
def test_oracle_matches_reference(oracle_lib, name):
    fx = gu.load(name)
    interner = gu.interner_for(fx)
    for doc in fx["docs"]:
        a = gu.encode_docs(fx, interner, [doc])
        od = oracle_lib.OracleDoc.new(a["seed"][: a["seed_off"][1]])
        od.apply_all(a["ops"], a["text"], a["props"])
        errs = gu.compare_oracle(od.outputs(), gu.expected(doc, interner))
        assert not errs, f"{name} doc {doc['doc']}: {errs}"


def test_oracle_error_model_matches_reference(oracle_lib):
    """Faulted streams (tests/golden/ref_errors): the oracle stops with the status of the
    reference's throw (completeAndLogOp / updateSeqNumbers / setMinSeq asserts) and its state
    at that point -- op applied, zamboni run -- equals the reference's state at the throw."""
    fx = gu.load("ref_errors")
    interner = gu.interner_for(fx)
    seen = set()
    for doc in fx["docs"]:
        a = gu.encode_docs(fx, interner, [doc])
        od = oracle_lib.OracleDoc.new(a["seed"][: a["seed_off"][1]])
        od.apply_all(a["ops"], a["text"], a["props"])
        want = gu.error_status(doc)
        seen.add(want)
        errs = gu.compare_oracle(od.outputs(), gu.expected(doc, interner), status=want)
        assert not errs, f"doc {doc['doc']} ({doc['fault']}): {errs}"
    assert seen == {2, 3, 7, 8, 9}


@pytest.mark.parametrize("name", gu.MAINT_FIXTURES)
def test_oracle_maintenance_events_match_reference(oracle_lib, name):
    """mergeTreeMaintenanceCallback SPLIT/APPEND/UNLINK counts (MT/mergeTree.ts:2264-2269,
    :1343-1373) equal the reference's own callback on every document."""
    fx = gu.load(name)
    interner = gu.interner_for(fx)
    want = gu.maint_counts(name)
    assert want is not None and len(want) == len(fx["docs"])
    for i, doc in enumerate(fx["docs"]):
        a = gu.encode_docs(fx, interner, [doc])
        od = oracle_lib.OracleDoc.new(a["seed"][: a["seed_off"][1]])
        assert od.apply_all(a["ops"], a["text"], a["props"]) == 0
        assert od.maintenance() == want[i], f"{name} doc {doc['doc']}"


@pytest.mark.parametrize("name", ["ref_small", "ref_c2", "ref_c3", "ref_c4", "ref_c3_full", "ref_c4_full"])
def test_oracle_generator_reproduces_reference_streams(oracle_lib, name):
    """The generator (shared spec) draws identical op streams whether the view
    lengths come from the reference or from the oracle."""
    fx = gu.load(name)
    interner = gu.interner_for(fx)
    for doc in fx["docs"]:
        a = gu.encode_docs(fx, interner, [doc])
        g = oracle_lib.generate(fx["config"], doc["doc"])
        assert np.array_equal(g["ops"], a["ops"]), f"doc {doc['doc']} ops differ"
        assert np.array_equal(g["text"][: len(a["text"])], a["text"])
        assert np.array_equal(g["seed"], a["seed"][: a["seed_off"][1]])


def test_batch_replay_checksums_consistent(oracle_lib):
    fx = gu.load("ref_c3")
    interner = gu.interner_for(fx)
    a = gu.encode_docs(fx, interner)
    s1, st1 = oracle_lib.replay_batch(a, threads=1)
    s4, st4 = oracle_lib.replay_batch(a, threads=4)
    assert (st1 == 0).all() and np.array_equal(s1, s4)
    for i, doc in enumerate(fx["docs"]):
        assert s1[i]["length"] == doc["out"]["length"]


@pytest.mark.parametrize("name", gu.SNAP_FIXTURES)
def test_oracle_snapshot_load_matches_reference(oracle_lib, name):
    """Config C5: the restated SnapshotLoader (orc_load) rebuilds the reference's tree
    (reloadFromSegments 7-per-block shape, loadBody appends) and the tail replays identically;
    the reference's load failure on unsettled summaries with a body is reproduced."""
    fx = gu.load(name)
    checked = 0
    for doc in fx["docs"]:
        want = gu.snap_status(doc)
        interner = gu.Interner()
        la, oa = gu.encode_snap_docs(fx, interner, [doc])
        od = oracle_lib.OracleDoc.load(la["segs"], la["n_header"][0], la["text"], la["props"],
                                       la["min_seq"][0], la["cur_seq"][0])
        if want:
            assert od.outputs()["status"] == want, doc["doc"]
            continue
        errs = gu.compare_oracle(od.outputs(), gu.expected_snap(doc, interner, "load_out"))
        assert not errs, f"{name} doc {doc['doc']} after load: {errs}"
        od.apply_all(oa["ops"], oa["text"], oa["props"])
        errs = gu.compare_oracle(od.outputs(), gu.expected_snap(doc, interner))
        assert not errs, f"{name} doc {doc['doc']}: {errs}"
        checked += 1
    assert checked >= 4


def test_snapshot_decoder_totals():
    """Decoded summaries agree with their own header metadata (MT/snapshotLoader.ts:162-193
    shipAsserts): total segment count and total length."""
    import json as _json
    from fluidframework_amd.snapshot import decode_chunks, to_latest_version
    for name in gu.SNAP_FIXTURES:
        for doc in gu.load(name)["docs"]:
            snap = decode_chunks(doc["chunks"])
            meta = to_latest_version("header", _json.loads(doc["chunks"]["header"]))["headerMetadata"]
            assert len(snap.header_specs) + len(snap.body_specs) == meta["totalSegmentCount"]


@pytest.mark.parametrize("name", ["ref_snap", "ref_snap_body"])
def test_snapshot_encoder_round_trip(name):
    """encode_chunks(decode(summary)) reproduces the reference's SnapshotV1.emit output
    byte for byte (the summaries in the fixtures were written by the reference)."""
    from fluidframework_amd.snapshot import SnapshotBatch, decode_chunks, encode_chunks, record_specs
    fx = gu.load(name)
    cs = fx["config"]["chunk"]
    for doc in fx["docs"]:
        interner = gu.Interner()
        sb = SnapshotBatch(interner)
        snap = decode_chunks(doc["chunks"])
        short = sb.add_doc(snap)
        a = sb.arrays()
        names = {v: k for k, v in short.items()}
        specs, lengths = record_specs(a["segs"], a["text"], a["props"], interner, names)
        assert encode_chunks(specs, lengths, snap.min_seq, snap.cur_seq, cs) == doc["chunks"], doc["doc"]


def _live_docs():
    """Live-participant fixture documents without reconnects (the oracle does not model
    regeneratePendingOp): all 8 ref_live_bench streams (4000 steps each) and the others'."""
    out = []
    for name in ["ref_live_bench", "ref_live", "ref_live_long", "ref_live_markers", "ref_live_deep"]:
        out += [(name, d) for d in gu.load(name)["docs"] if not any(e[0] == "R" for e in d["events"])]
    return out


def test_oracle_live_participant_matches_reference(oracle_lib):
    """The restatement as a participant (MT_F_LOCAL ops, MT_F_ACK echoes, remote ops around
    unacked segments) equals the reference Client on its own streams: text, length, leaf
    partition, segment table, property sets, every delta record, localSeq and pending groups;
    then, after the fixture's drain acks every pending op, the drained replica."""
    from fluidframework_amd.wire import Batch, Interner
    docs = _live_docs()
    assert len(docs) >= 9
    for name, doc in docs:
        it = Interner(synthetic=True)
        b = Batch(it)
        b.add_live_doc(doc["seed_text"], gu.live_entries(doc), {"local-0": 0})
        n_run = len(b.recs)
        b = Batch(it)   # the same stream + the drain (same interner: the same records first)
        b.add_live_doc(doc["seed_text"], gu.live_entries(doc) + gu.live_entries(dict(events=doc["drain"])),
                       {"local-0": 0})
        a = b.arrays()
        d = oracle_lib.OracleDoc.new(a["seed"][:a["seed_off"][1]])
        assert d.apply_all(a["ops"][:n_run], a["text"], a["props"]) == 0
        errs = gu.compare_oracle(d.outputs(), gu.expected_live(doc, it))
        assert d.pending_counts() == (doc["out"]["localSeq"], doc["out"]["pending"]), (name, doc["doc"])
        assert not errs, (name, doc["doc"], errs)
        assert d.apply_all(a["ops"][n_run:], a["text"], a["props"]) == 0
        o = d.outputs()
        exp = gu.expected(dict(doc, out=dict(doc["drained"], deltas=[])), it)
        assert d.pending_counts()[1] == doc["drained"]["pending"] == 0
        assert (o["text"], o["leaves"], o["segs"].tolist(), o["seg_props"]) == \
            (exp["text"], exp["leaves"], exp["segs"], exp["seg_props"]), (name, doc["doc"])


def _replay_live_with_reconnects(oracle_lib, doc, interner):
    """Replay one live fixture document on the restatement event by event, reconnects
    included: at each "R" every pending op is regenerated (orc_regenerate) and compared with
    the reference's regeneratePendingOp output.  Returns (doc, errors)."""
    from fluidframework_amd.live import OP_GROUP, regen_op
    from fluidframework_amd.wire import F_ACK, F_LOCAL, Batch, DocEncoder
    ids = {"local-0": 0}
    ids.update({e[1]: 0 for e in doc["events"] if e[0] == "R"})
    b = Batch(interner)
    enc = DocEncoder(b, ids)
    steps = []
    me = "local-0"
    for ev in doc["events"] + doc["drain"]:
        lo = len(b.recs)
        if ev[0] == "L":
            b._msg(enc, dict(clientId="local-0", sequenceNumber=-1, referenceSequenceNumber=0,
                             minimumSequenceNumber=0, contents=ev[1]), F_LOCAL)
            steps.append(("L", lo, len(b.recs), ev[1]))
        elif ev[0] == "M":
            _, cid, seq, ref, msn, op = ev
            b._msg(enc, dict(clientId=cid, sequenceNumber=seq, referenceSequenceNumber=ref,
                             minimumSequenceNumber=msn, type="op", contents=op), F_ACK if cid == me else 0)
            steps.append(("M", lo, len(b.recs), cid == me))
        else:
            me = ev[1]
            steps.append(("R", ev[2]))
    b.doc_off.append(len(b.recs))
    steps.insert(len(doc["events"]), ("X",))   # the end of the stream: the fixture's "out" state
    a = b.arrays()
    d = oracle_lib.OracleDoc.new(np.frombuffer(doc["seed_text"].encode("utf-16-le"), dtype="<u2"))
    unseq, errs = [], []
    for i, st in enumerate(steps):
        if st[0] == "X":
            yield d, errs
        elif st[0] in ("L", "M"):
            if d.apply_all(a["ops"][st[1]:st[2]], a["text"], a["props"]):
                errs.append(f"status {d.outputs()['status']} at event {i}")
                break
            if st[0] == "L":
                unseq.append(st[3])
            elif st[3]:
                unseq.pop(0)
        else:
            got = []
            for op in unseq:
                members = op["ops"] if op["type"] == OP_GROUP else [op]
                out = []
                for m in members:
                    r = d.regenerate(m["type"])
                    assert r is not None, "no pending group to regenerate"
                    recs, text, props = r
                    out += [regen_op(interner, m, rec, text, props) for rec in recs]
                got.append(out[0] if len(out) == 1 else {"ops": out, "type": OP_GROUP})
            if got != st[1]:
                errs.append(f"regenerated ops differ at event {i}")
            unseq = list(st[1])
        if errs:
            break
    yield d, errs


@pytest.mark.parametrize("name", ["ref_live", "ref_live_long", "ref_live_markers", "ref_live_deep", "ref_live_xl",
                                  "ref_live_60k"])
def test_oracle_live_reconnects_match_reference(oracle_lib, name):
    """Every live fixture document, reconnects included: each regenerated op list equals the
    reference's, and the final state (text, length, leaves, segment table, property sets,
    delta records, localSeq, pending groups) and the drained replica equal the reference's."""
    from fluidframework_amd.wire import Interner
    for doc in gu.load(name)["docs"]:
        it = Interner(synthetic=True)
        run = _replay_live_with_reconnects(oracle_lib, doc, it)
        d, errs = next(run)
        assert not errs, (name, doc["doc"], errs)
        errs = gu.compare_oracle(d.outputs(), gu.expected_live(doc, it))
        assert d.pending_counts() == (doc["out"]["localSeq"], doc["out"]["pending"]), (name, doc["doc"])
        assert not errs, (name, doc["doc"], errs)
        d, errs = next(run)
        assert not errs, (name, doc["doc"], errs)
        o = d.outputs()
        exp = gu.expected(dict(doc, out=dict(doc["drained"], deltas=[])), it)
        assert d.pending_counts()[1] == doc["drained"]["pending"] == 0
        assert (o["text"], o["leaves"], o["segs"].tolist(), o["seg_props"]) == \
            (exp["text"], exp["leaves"], exp["segs"], exp["seg_props"]), (name, doc["doc"])


@pytest.mark.parametrize("name", ["ref_readouts", "ref_readouts_wide", "ref_readouts_xl"])
def test_oracle_readouts_match_reference_in_every_view(oracle_lib, name):
    """MergeTree.getLength(refSeq, clientId), getContainingSegment and getPosition in every
    writer view of the collab window -- including the views below the writer's latest refSeq,
    which the reference answers from partial lengths (MT/partialLengths.ts:455-486) rather than
    from its leaves' nodeLength -- equal the reference's (the oracle restates the partial
    lengths as each leaf's +len at its insert and -len at its removal, oracle/mt_oracle.c
    seg_partial)."""
    fx = gu.load(name)
    interner = gu.interner_for(fx)
    n_stale = n_stale_cont = 0
    for doc in fx["docs"]:
        a = gu.encode_docs(fx, interner, [doc])
        od = oracle_lib.OracleDoc.new(a["seed"][: a["seed_off"][1]])
        assert od.apply_all(a["ops"], a["text"], a["props"]) == 0
        rows = od.outputs()["segs"]
        for ref, cli, want, stale, _ in doc["lengths"]:
            assert od.view_length(ref, cli) == want, (doc["doc"], ref, cli, stale)
            n_stale += stale
        for pos, ref, cli, exp, stale in doc["containing"]:
            got = od.containing(pos, ref, cli)
            where = (doc["doc"], pos, ref, cli, stale)
            n_stale_cont += stale
            if exp is None:
                assert got is None, where
                continue
            offset, vpos, lpos, clen = exp[:4]
            assert got is not None and got[1:] == (offset, vpos, lpos), (where, got, exp)
            assert rows[got[0]][0] == clen, where
    assert n_stale > 200000 and n_stale_cont > 1000


@pytest.mark.parametrize("name", gu.WIDE_FIXTURES)
def test_oracle_overlap_unit_count(oracle_lib, name):
    """The restatement's running count of removedClientOverlap units (the bound the device's
    overflow arena is tested against) equals a recount of the final tree's lists."""
    fx = gu.load(name)
    interner = gu.interner_for(fx)
    for doc in fx["docs"]:
        a = gu.encode_docs(fx, interner, [doc])
        od = oracle_lib.OracleDoc.new(a["seed"][: a["seed_off"][1]])
        od.apply_all(a["ops"], a["text"], a["props"])
        segs = od.outputs()["segs"]
        novl = segs[:, 5]
        now, peak = od.overlap_units()
        assert now == int((novl[novl > 0] + 1).sum()) and peak >= now > 0
