"""Live-client path: a participant Client's own unsequenced ops, their acks,
remote ops resolved around unacked segments and reconnect regeneration, on the GPU
(live_client handles) against streams the reference itself produced
(tests/golden/ref_live*.json.gz, oracle/ref_harness.mjs "live"), and on reconnect-free
streams against the C restatement's participant replay (oracle/mt_oracle.c, itself pinned to
the same fixtures by tests/test_oracle.py).  Checked per document: every local op the facade returns, every op
regeneratePendingOp rebuilds, the final text / length / leaf partition / segment table (unacked
seq and removedSeq = -1) / property sets, every delta-callback record, localSeq and the
pending segment groups."""
import numpy as np
import pytest

import golden_util as gu
from fluidframework_amd.wire import F_ACK, F_LOCAL, Batch, Interner

LIVE_FIXTURES = ["ref_live", "ref_live_long", "ref_live_markers", "ref_live_deep", "ref_live_xl"]


def _msg(ev):
    _, cid, seq, ref, msn, op = ev
    return dict(clientId=cid, sequenceNumber=seq, referenceSequenceNumber=ref, minimumSequenceNumber=msn,
                type="op", contents=op)


# ---------------------------------------------------------------- CPU: encoding
def test_live_encoding_flags():
    """Local ops -> MT_F_LOCAL records of client 0; the echo of one (the local client's long id,
    GROUPs member by member) -> MT_F_ACK; an empty GROUP -> a seq/msn-only record."""
    b = Batch(Interner(synthetic=True))
    ack = dict(clientId="me", sequenceNumber=5, referenceSequenceNumber=3, minimumSequenceNumber=1, type="op",
               contents={"type": 3, "ops": [{"pos1": 0, "pos2": 1, "type": 1},
                                             {"pos1": 0, "seg": "x", "type": 0}]})
    empty = dict(clientId="other", sequenceNumber=6, referenceSequenceNumber=3, minimumSequenceNumber=1,
                 type="op", contents={"type": 3, "ops": []})
    b.add_live_doc("", [("local", {"pos1": 0, "seg": "ab", "type": 0}), ("ack", ack), ("msg", empty)],
                   {"me": 0})
    ops = b.arrays()["ops"]
    assert ops["flags"].tolist() == [F_LOCAL, F_ACK | 1, F_ACK, 0]
    assert ops["client"].tolist() == [0, 0, 0, 1]
    assert ops["kind"].tolist() == [0, 1, 0, 3]


def test_live_fixtures_are_reference_made():
    # ref_live_deep: segments sit in up to 13 pending groups, documents hold up to 478 of them
    deep = gu.load("ref_live_deep")
    assert max(d["out"]["maxGroupDepth"] for d in deep["docs"]) > 8
    assert max(d["out"]["pending"] for d in deep["docs"]) > 255
    for name in LIVE_FIXTURES:
        fx = gu.load(name)
        assert fx["config"]["steps"] > 0 and len(fx["docs"]) >= 3
        kinds = set()
        for d in fx["docs"]:
            kinds |= {e[0] for e in d["events"]}
        assert kinds == {"L", "M", "R"}, (name, kinds)


# ---------------------------------------------------------------- GPU
def _run_doc(doc, log=True, lds=-1, caps=None):
    from fluidframework_amd.live import LiveClient
    interner = Interner(synthetic=True)
    caps = caps or dict(seg_capacity=16384, text_capacity=1 << 17)
    lc = LiveClient(doc["seed_text"], delta_log_capacity=(1 << 20) if log else 0, interner=interner,
                    lds_seg_capacity=lds, **caps)
    lc.startOrUpdateCollaboration("local-0")
    unseq = []
    errs = []
    for ev in doc["events"]:
        if ev[0] == "L":
            op = ev[1]
            if op["type"] == 0:
                got = lc.insertSegmentLocal(op["pos1"], op["seg"])
            elif op["type"] == 1:
                got = lc.removeRangeLocal(op["pos1"], op["pos2"])
            else:
                got = lc.annotateRangeLocal(op["pos1"], op["pos2"], op["props"], op.get("combiningOp"))
            if got != op:
                errs.append(f"local op {got} != {op}")
            unseq.append(op)
        elif ev[0] == "M":
            if ev[1] == lc.long_client_id:
                unseq.pop(0)
            lc.applyMsg(_msg(ev))
        else:
            _, new_id, regen = ev
            lc.startOrUpdateCollaboration(new_id)
            got = [lc.regeneratePendingOp(o) for o in unseq]
            if got != regen:
                errs.append(f"regenerated ops differ at reconnect {new_id}")
            unseq = regen
        if len(errs) > 3:
            break
    lc.flush()
    return lc, interner, errs


# grow: starting capacities far below the documents' (64 segments, 1024 text units, 16 segment
# groups): the live growth step doubles them, round after round, mid-stream
GROW_CAPS = dict(seg_capacity=64, text_capacity=1024, live_group_capacity=16)


@pytest.mark.gpu
@pytest.mark.parametrize("lds", [-1, 64, 192, "grow"], ids=["hbm", "lds64", "lds192", "grow"])
@pytest.mark.parametrize("name", LIVE_FIXTURES + ["ref_live_60k"])
def test_live_client_matches_reference(name, lds):
    """hbm: the flat HBM tier only; lds64 / lds192: each flush staged in LDS (TierLiveLdsT)
    while the document fits 64 / 192 segments, continuing in the HBM tier beyond; grow: the HBM
    tier from capacities far below the documents' (the live growth step raises them: equal to
    the reference all the same, every delta record included)."""
    fx = gu.load(name)
    bad = []
    for doc in fx["docs"]:
        lc, interner, errs = _run_doc(doc, lds=-1 if lds == "grow" else lds, caps=GROW_CAPS if lds == "grow" else None)
        mt = lc.mt
        rows, leaves = mt.get_segments(0)
        o = dict(text=mt.get_text(0), length=mt.get_length(0), leaves=leaves, segs=rows,
                 seg_props=mt.get_all_segment_props(0),
                 deltas=mt.get_delta_log(0), status=int(mt.status()[0]))
        errs += gu.compare_oracle(o, gu.expected_live(doc, interner))
        ls, ng = lc.pendingCounts()
        if (ls, ng) != (doc["out"]["localSeq"], doc["out"]["pending"]):
            errs.append(f"localSeq/pending {(ls, ng)} != {(doc['out']['localSeq'], doc['out']['pending'])}")
        if errs:
            bad.append((doc["doc"], errs[:4]))
        lc.close()
    assert not bad, bad


@pytest.mark.gpu
def test_live_client_drained_matches_reference_and_observer():
    """The server then sequences every op still pending (the reference's drain in the
    fixture): the acked replica equals the reference's (text, segment table, leaf partition,
    property sets) and an observer replaying the whole sequenced stream holds the same text.
    (Property sets need not match the observer's: a participant skips remote updates of keys
    it has pending, SegmentPropertiesManager.shouldModifyKey, and the reference's own
    replicas differ there.)"""
    from fluidframework_amd import MergeTreeBatch
    fx = gu.load("ref_live")
    for doc in fx["docs"][:3]:
        lc, interner, errs = _run_doc(doc, log=False)
        assert not errs, errs
        for ev in doc["drain"]:
            lc.applyMsg(_msg(ev))
        assert lc.pendingCounts()[1] == doc["drained"]["pending"] == 0
        rows, leaves = lc.mt.get_segments(0)
        exp = gu.expected(dict(doc, out=dict(doc["drained"], deltas=[])), interner)
        assert lc.getText() == exp["text"]
        assert list(leaves) == exp["leaves"]
        assert rows.tolist() == exp["segs"]
        assert lc.mt.get_all_segment_props(0) == exp["seg_props"]
        obs = MergeTreeBatch(1, seg_capacity=16384, text_capacity=1 << 17, lds_seg_capacity=-1)
        b = Batch(Interner(synthetic=True))
        b.add_doc(doc["seed_text"], [_msg(e) for e in doc["events"] + doc["drain"] if e[0] == "M"])
        a = b.arrays()
        obs.load_initial_text(a["seed_off"], a["seed"])
        obs.apply_arrays(a)
        assert int(obs.status()[0]) == 0
        assert obs.get_text(0) == lc.getText()
        lc.close()
        obs.close()


@pytest.mark.gpu
def test_live_flags_rejected_on_observer_handles():
    from fluidframework_amd import MergeTreeBatch
    mt = MergeTreeBatch(1, seg_capacity=256)
    b = Batch(Interner(synthetic=True))
    b.add_live_doc("", [("local", {"pos1": 0, "seg": "ab", "type": 0})], {"me": 0})
    with pytest.raises(RuntimeError, match="live_client"):
        mt.apply_arrays(b.arrays())
    mt.close()


@pytest.mark.gpu
def test_live_local_ops_and_invalid_ranges():
    """getValidOpRange (MT/client.ts:486-548): out-of-range local ops return None and change
    nothing; valid ones apply at once in the local view."""
    from fluidframework_amd.live import LiveClient
    lc = LiveClient("hello")
    lc.startOrUpdateCollaboration("me")
    assert lc.insertSegmentLocal(6, "x") is None
    assert lc.removeRangeLocal(5, 6) is None
    assert lc.removeRangeLocal(2, 2) is None
    assert lc.insertSegmentLocal(5, " world") == {"pos1": 5, "seg": " world", "type": 0}
    assert lc.removeRangeLocal(0, 1) == {"pos1": 0, "pos2": 1, "type": 1}
    assert lc.getText() == "ello world"
    assert lc.pendingCounts() == (2, 2)
    lc.applyMsg(dict(clientId="me", sequenceNumber=1, referenceSequenceNumber=0, minimumSequenceNumber=0,
                     type="op", contents={"pos1": 5, "seg": " world", "type": 0}))
    assert lc.pendingCounts() == (2, 1)
    # a local transaction (GROUP) is acked member by member by its echo
    grp = {"ops": [{"pos1": 0, "seg": "ab", "type": 0}, {"pos1": 2, "pos2": 4, "type": 1}], "type": 3}
    lc.localTransaction(grp)
    assert lc.getText() == "ablo world" and lc.pendingCounts() == (4, 3)
    lc.applyMsg(dict(clientId="me", sequenceNumber=2, referenceSequenceNumber=1, minimumSequenceNumber=0,
                     type="op", contents={"pos1": 0, "pos2": 1, "type": 1}))
    lc.applyMsg(dict(clientId="me", sequenceNumber=3, referenceSequenceNumber=2, minimumSequenceNumber=1,
                     type="op", contents=grp))
    assert lc.pendingCounts() == (4, 0) and lc.getText() == "ablo world"
    lc.close()


@pytest.mark.gpu
def test_regenerate_with_small_buffers_leaves_the_document():
    """mt_regenerate_pending with output buffers too small for the oldest group fails with
    MT_E_OVERFLOW before touching anything: the group is still pending and a second call with
    room regenerates it."""
    from fluidframework_amd import MergeTreeBatch
    mt = MergeTreeBatch(1, seg_capacity=256, lds_seg_capacity=-1, live_client=1)
    b = Batch(Interner(synthetic=True))
    b.add_live_doc("abc", [("local", {"pos1": 1, "seg": "xyz", "type": 0})], {"me": 0})
    a = b.arrays()
    mt.load_initial_text(a["seed_off"], a["seed"])
    mt.apply_arrays(a)
    before = mt.pending_counts().tolist()
    with pytest.raises(RuntimeError, match="too small"):
        mt.regenerate_pending(0, cap=4, text_cap=2, props_cap=16)
    assert mt.pending_counts().tolist() == before and int(mt.status()[0]) == 0
    recs, text, _ = mt.regenerate_pending(0)
    assert len(recs) == 1 and int(recs[0]["pos1"]) == 1 and text[:3].tobytes().decode("utf-16-le") == "xyz"
    mt.close()


@pytest.mark.gpu
def test_live_checksums_match_oracle_participant():
    """Device checksums of live documents (text, property runs, every delta callback) equal
    the C restatement's participant replay (oracle/mt_oracle.c, pinned to the reference by
    tests/test_oracle.py) on the reference's participant streams without reconnects."""
    import os
    import sys
    from fluidframework_amd import MergeTreeBatch
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import pyoracle
    docs = [d for name in ["ref_live_bench", "ref_live_deep"] for d in gu.load(name)["docs"]
            if not any(e[0] == "R" for e in d["events"])]
    b = Batch(Interner(synthetic=True))
    for d in docs:
        b.add_live_doc(d["seed_text"], gu.live_entries(d), {"local-0": 0})
    a = b.arrays()
    osums, ost = pyoracle.replay_batch(a)
    assert ost.tolist() == [0] * len(docs)
    for lds in (-1, 192):   # the HBM tier; LDS-staged (TierLiveLdsT) with hand-over
        mt = MergeTreeBatch(len(docs), seg_capacity=16384, text_capacity=1 << 17, props_capacity=1 << 16,
                            heap_capacity=4096, lds_seg_capacity=lds, live_client=1)
        mt.load_initial_text(a["seed_off"], a["seed"])
        mt.apply_arrays(a)
        assert mt.status().tolist() == [0] * len(docs)
        sums = mt.checksums()
        for f in sums.dtype.names:
            assert sums[f].tolist() == osums[f].tolist(), (lds, f)
        mt.close()
