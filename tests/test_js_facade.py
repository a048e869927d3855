"""The Node facade (fluidframework_amd/js: N-API addon + encoder + Client-shaped views):
the addon builds and loads, its encoder produces exactly the Python encoder's wire bytes
for the reference-generated fixtures, and (GPU) a fixture replayed through
Client.applyMsg-shaped calls matches the reference's text, length and properties."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import golden_util as gu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JS = os.path.join(REPO, "fluidframework_amd", "js")
TOOL = os.path.join(REPO, "tests", "js", "fixture_tool.js")
pytestmark = pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")


def _node(*args, timeout=300):
    out = subprocess.run(["node", TOOL, *args], capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout)


def _addon():
    from fluidframework_amd import build
    build.build()
    build.build_snapdec()
    build.build_node_addon()   # rebuilds when binding.cc or the libraries are newer
    if not os.path.exists(os.path.join(JS, "mtreplay.node")):
        subprocess.check_call(["sh", os.path.join(JS, "build.sh")])


def test_addon_loads_and_fails_loudly_without_gpu():
    _addon()
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = subprocess.run(["node", "-e", "const m=require(process.argv[1]); new m.GpuMergeTreeBatch(2, {});", JS],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "no CPU fallback" in r.stderr


@pytest.mark.parametrize("name", ["ref_ext", "ref_ext_long", "ref_small", "ref_combine"])
def test_js_encoder_matches_python_encoder(name):
    fx = gu.load(name)
    got = _node("encode", os.path.join(gu.GOLDEN, name + ".json.gz"))
    interner = gu.Interner()   # real (non-synthetic) interning, as the JS encoder does
    a = gu.encode_docs(fx, interner)
    assert got["docOff"] == a["doc_off"].tolist()
    assert bytes.fromhex(got["ops"]) == a["ops"].tobytes()
    n_text = len(bytes.fromhex(got["text"])) // 2
    assert bytes.fromhex(got["text"]) == a["text"][:n_text].tobytes()
    n_props = len(bytes.fromhex(got["props"])) // 4
    assert bytes.fromhex(got["props"]) == a["props"][:n_props].tobytes()
    assert got["keys"] == interner.keys


@pytest.mark.gpu
@pytest.mark.parametrize("name,mode", [("ref_ext", "replay"), ("ref_c3", "replay"), ("ref_combine", "replay"),
                                       ("ref_c3_full", "replaydefault"), ("ref_wide400", "replaydefault")])
def test_js_facade_replays_fixture_like_reference(name, mode):
    """Client.applyMsg through the Node facade, then getText / getLength /
    getPropertiesAtPosition equal the reference's.  replaydefault: `new GpuMergeTreeBatch(n)`
    with no options -- the drop-in default takes the 10k-message C3 documents (~4k live
    segments) and the 200-writer streams (~80 concurrent overlapping removers) unbounded."""
    _addon()
    fx = gu.load(name)
    got = _node(mode, os.path.join(gu.GOLDEN, name + ".json.gz"), timeout=600)
    for d, g in zip(fx["docs"], got["docs"]):
        assert "error" not in g, g
        assert g["text"] == d["out"]["text"]
        assert g["length"] == d["out"]["length"]
        # properties at probed positions == the reference's segment properties there
        runs = []
        pos = 0
        for s in d["out"]["segs"]:
            if s["rseq"] is None:
                runs.append((pos, s["len"], s["props"]))
                pos += s["len"]
        for p, props in g["props"]:
            exp = next((r[2] for r in runs if r[0] <= p < r[0] + r[1]), None)
            assert props == exp, (p, props, exp)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ref_ext", "ref_c3"])
def test_js_facade_maintenance_counts_match_reference(name):
    _addon()
    got = _node("maint", os.path.join(gu.GOLDEN, name + ".json.gz"))
    assert got["docs"] == gu.maint_counts(name)


@pytest.mark.parametrize("name", gu.SNAP_FIXTURES)
def test_js_snapshot_decoder_matches_python(name):
    """The Node facade's summary decoder (js/snapshot.js) writes exactly the mt_seg_rec records
    and arenas of fluidframework_amd/snapshot.py for the reference-written summaries."""
    fx = gu.load(name)
    got = _node("snapenc", os.path.join(gu.GOLDEN, name + ".json.gz"))
    from fluidframework_amd.snapshot import SnapshotBatch, decode_chunks
    sb = SnapshotBatch(gu.Interner())
    for d in fx["docs"]:
        sb.add_doc(decode_chunks(d["chunks"]))
    a = sb.arrays()
    assert bytes.fromhex(got["segs"]) == a["segs"].tobytes()
    assert got["docSegOff"] == a["doc_off"].tolist() and got["nHeader"] == a["n_header"].tolist()
    assert got["minSeq"] == a["min_seq"].tolist() and got["curSeq"] == a["cur_seq"].tolist()
    n_text = len(bytes.fromhex(got["text"])) // 2
    assert bytes.fromhex(got["text"]) == a["text"][:n_text].tobytes()
    n_props = len(bytes.fromhex(got["props"])) // 4
    assert bytes.fromhex(got["props"]) == a["props"][:n_props].tobytes()


@pytest.mark.parametrize("name", gu.SNAP_FIXTURES)
def test_js_native_summary_decoder_matches_python(name):
    """decodeSummaries (the native decoder, include/mt_snapshot.h, through the addon; what
    GpuMergeTreeBatch.loadSnapshots uses) gives the records, arenas, client maps and catch-up
    messages of fluidframework_amd/snapshot.py.  Host-only: no device call."""
    _addon()
    fx = gu.load(name)
    got = _node("snapnative", os.path.join(gu.GOLDEN, name + ".json.gz"))
    from fluidframework_amd.snapshot import SnapshotBatch, decode_chunks
    sb = SnapshotBatch(gu.Interner())
    clients, catchup = [], []
    for d in fx["docs"]:
        snap = decode_chunks(d["chunks"])
        clients.append(sb.add_doc(snap))
        catchup.append(snap.catchup)
    a = sb.arrays()
    assert bytes.fromhex(got["segs"]) == a["segs"].tobytes()
    assert got["docSegOff"] == a["doc_off"].tolist() and got["nHeader"] == a["n_header"].tolist()
    assert got["minSeq"] == a["min_seq"].tolist() and got["curSeq"] == a["cur_seq"].tolist()
    assert bytes.fromhex(got["text"]) == a["text"].tobytes()
    assert bytes.fromhex(got["props"]) == a["props"].tobytes()
    assert [dict(c) for c in got["clients"]] == clients
    assert got["catchup"] == catchup


@pytest.mark.gpu
@pytest.mark.parametrize("name", gu.SNAP_FIXTURES)
def test_js_facade_loads_snapshots_like_reference(name):
    """GpuMergeTreeBatch.loadSnapshots (Client.load for every document) + GpuClient.applyMsg of
    the tails: text, length and properties equal the reference's; the reference's load
    failures throw "MergeTree insert failed", and a body that loadBody
    re-inserts (MT_DOC_ALIASED) throws the facade's own error -- every document compared."""
    _addon()
    fx = gu.load(name)
    got = {g["doc"]: g for g in _node("loadsnap", os.path.join(gu.GOLDEN, name + ".json.gz"))["docs"]}
    assert len(got) == len(fx["docs"])
    for d in fx["docs"]:
        want = gu.snap_status(d)
        g = got[d["doc"]]
        if want == 10:
            assert "insert segments twice" in g.get("error", ""), g
            continue
        if want:
            assert g.get("error", "").startswith("MergeTree insert failed"), g
            continue
        assert "error" not in g, g
        assert g["text"] == d["out"]["text"] and g["length"] == d["out"]["length"]
        runs, pos = [], 0
        for s in d["out"]["segs"]:
            if s["rseq"] is None:
                runs.append((pos, s["len"], s["props"]))
                pos += s["len"]
        for p, props in g["props"]:
            exp = next((r[2] for r in runs if r[0] <= p < r[0] + r[1]), None)
            assert props == exp, (p, props, exp)


@pytest.mark.gpu
def test_js_facade_throws_the_reference_errors():
    """Faulted streams (tests/golden/ref_errors): the facade throws the reference's
    AssertionError with the reference's message (completeAndLogOp MT/client.ts:462-465,
    updateSeqNumbers :824-826, setMinSeq MT/mergeTree.ts:1755)."""
    _addon()
    fx = gu.load("ref_errors")
    got = _node("replay", os.path.join(gu.GOLDEN, "ref_errors.json.gz"))
    for d, g in zip(fx["docs"], got["docs"]):
        assert g.get("type") == d["error"]["name"] == "AssertionError", (d["fault"], g)
        assert g["error"] == d["error"]["message"], (d["fault"], g)


def _ref_calls(doc):
    return [[seq, kind, [list(x) for x in segs]] for seq, kind, n, segs in doc["out"]["deltas"]]


@pytest.mark.gpu
@pytest.mark.parametrize("name,cap,every", [("ref_ext", 2048, 37), ("ref_c3", 4096, 100), ("ref_c4_full", 1 << 16, 1000)])
def test_js_facade_delta_callbacks_match_reference_across_flushes(name, cap, every):
    """mergeTreeDeltaCallback(opArgs, {operation, deltaSegments}) as the facade fires it equals
    the reference's raw callback stream (MT/mergeTree.ts:2014-2021, 2625-2632, 2738-2745):
    same records, positions, lengths and propertyDeltas -- with a device log far smaller than
    the whole stream, drained and reset at every flush."""
    _addon()
    fx = gu.load(name)
    got = _node("deltas", os.path.join(gu.GOLDEN, name + ".json.gz"), str(cap), str(every), timeout=600)
    assert got["error"] is None, got["error"]
    total = 0
    for d, calls in zip(fx["docs"], got["calls"]):
        want = _ref_calls(d)
        assert calls == want, (name, d["doc"], next(i for i, (a, b) in enumerate(zip(calls, want)) if a != b))
        total += sum(3 + sum(2 + (1 + 2 * len(s[2]) if len(s) > 2 else 0) for s in c[2]) for c in want)
    assert total > cap * len(fx["docs"])   # the stream is longer than the log: it was drained


@pytest.mark.gpu
def test_js_facade_delta_log_overflow_throws():
    """A single flush larger than the device log fails loudly instead of dropping callbacks."""
    _addon()
    got = _node("deltas", os.path.join(gu.GOLDEN, "ref_c3.json.gz"), "512", "100000")
    assert got["error"] and "overflowed its delta log" in got["error"]


@pytest.mark.gpu
def test_js_facade_rich_callbacks_match_reference():
    """The facade's mergeTreeDeltaCallback / mergeTreeMaintenanceCallback stream -- opArgs.op,
    segments carrying text / refType and properties at the event, SPLIT / APPEND / UNLINK as
    event objects -- equals the reference's own callbacks (tests/golden/ref_rich), across
    flushes that drain and reset the device log."""
    _addon()
    fx = gu.load("ref_rich")
    got = _node("rich", os.path.join(gu.GOLDEN, "ref_rich.json.gz"), "97", timeout=600)
    assert got["error"] is None, got["error"]
    for d, ev in zip(fx["docs"], got["events"]):
        assert all(e[0] == "M" or e[4] in (0, 1, 2) for e in ev)       # opArgs.op is the member op
        mine = [e[:4] if e[0] == "D" else e for e in ev]
        bad = next((j for j, (x, y) in enumerate(zip(mine, d["events"])) if x != y), None)
        assert bad is None and len(mine) == len(d["events"]), (d["doc"], bad, mine[bad] if bad is not None else None,
                                                               d["events"][bad] if bad is not None else None)


_WINDOW_JS = r"""
const m = require(process.argv[1]);
const b = new m.GpuMergeTreeBatch(2, {});
b.loadInitialText(["abc", "abc"]);
const c0 = b.client(0), c1 = b.client(1);
c0.startOrUpdateCollaboration("obs");
c1.startOrUpdateCollaboration("obs", 10, 10);
const op = (seq, ref, msn, pos, text) => ({clientId: "w1", sequenceNumber: seq,
    referenceSequenceNumber: ref, minimumSequenceNumber: msn, clientSequenceNumber: seq,
    type: "op", contents: {type: 0, pos1: pos, seg: text}});
c0.applyMsg(op(1, 0, 0, 0, "x")); c0.applyMsg(op(2, 1, 1, 4, "y"));
c1.applyMsg(op(11, 10, 10, 0, "x")); c1.applyMsg(op(12, 11, 11, 4, "y"));
const out = {t0: c0.getText(), t1: c1.getText(), s1: c1.getCurrentSeq()};
c1.startOrUpdateCollaboration("renamed", 50, 50);   // already collaborating: rename only
c1.applyMsg(op(13, 12, 12, 0, "z"));
out.t2 = c1.getText();
const b2 = new m.GpuMergeTreeBatch(1, {});
b2.loadInitialText(["abc"]);
const d = b2.client(0);
d.startOrUpdateCollaboration("obs", 10, 10);
d.applyMsg(op(5, 0, 0, 0, "q"));
try { d.getText(); out.err = null; } catch (e) { out.err = e.message; }
console.log(JSON.stringify(out));
"""


@pytest.mark.gpu
def test_js_facade_start_collaboration_window():
    """startOrUpdateCollaboration(id, minSeq, currentSeq) starts the document's collab window
    there (MT/client.ts:1053-1073, MT/mergeTree.ts:1287-1294): a stream numbered from it
    replays like the same stream numbered from 0; a later call only renames the client; a
    message at or below the window fails with the reference's assertion."""
    _addon()
    r = subprocess.run(["node", "-e", _WINDOW_JS, JS], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout)
    assert out["t0"] == out["t1"] == "xabcy" and out["s1"] == 12
    assert out["t2"] == "zxabcy"
    assert out["err"] == "Incoming remote op sequence# <= local collabWindow's currentSequence#"


@pytest.mark.gpu
def test_js_facade_live_client_matches_reference():
    """GpuClient on a liveClient batch (the reference language's drop-in for a participant
    Client): local ops, acks and regeneratePendingOp over the reference's live streams give
    the reference's text, length and regenerated ops."""
    _addon()
    fx = gu.load("ref_live")
    got = _node("live", os.path.join(gu.GOLDEN, "ref_live.json.gz"))
    for d, g in zip(fx["docs"], got["docs"]):
        assert g["errs"] == [], g["errs"][:3]
        assert g["text"] == d["out"]["text"]
        assert g["length"] == d["out"]["length"]
        # mergeTreeDeltaCallback stream: local ops (seq -1, no sequencedMessage), remote ops,
        # propertyDeltas undefined where an outstanding local rewrite blocked a remote annotate
        assert g["deltas"] == d["out"]["deltas"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ref_live_xl", "ref_live_60k"])
def test_js_facade_default_live_batch_is_unbounded(name):
    """`new GpuMergeTreeBatch(n, {liveClient: 1})` with no capacity options (2048 segments,
    32k text units, 1024 segment groups to start) replays participant streams far beyond them
    -- 20k- and 60k-event live documents made by the reference, thousands of live segments and
    pending groups -- equal to the reference: every local op, every regenerated op, the final
    text and length.  The live growth step doubles what a document would outgrow, for the whole
    batch, before the message that would (segmentGroups and the pending queue are unbounded in
    the reference, MT/mergeTree.ts:1955-1962)."""
    _addon()
    fx = gu.load(name)
    got = _node("live", os.path.join(gu.GOLDEN, name + ".json.gz"), "default", timeout=900)
    for d, g in zip(fx["docs"], got["docs"]):
        assert g["errs"] == [], g["errs"][:3]
        assert g["text"] == d["out"]["text"]
        assert g["length"] == d["out"]["length"]


# ---------------------------------------------------------------- SharedSegmentSequence events
def test_js_sequence_event_restatement_matches_reference_events():
    """tests/js/sequence_event.js (SequenceEvent.ranges over SortedSegmentSet, restated for the
    GPU box) reproduces every reference event's ranges from its segments' ordinals and
    positions (CPU)."""
    got = _node("evpin", os.path.join(gu.GOLDEN, "ref_events.json.gz"))
    assert got["events"] > 50000 and got["mismatches"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("name,every,layout", [("ref_events", 100000, "flat"), ("ref_events", 37, "flat"),
                                               ("ref_events_full", 100000, "paged"), ("ref_events", 37, "paged")])
def test_js_facade_sequence_events_match_reference(name, every, layout):
    """A listener builds SharedSegmentSequence's event objects over GpuClient callbacks
    (getPosition + segment ordinals, SEQ/sequence.ts:139-149): every event's positions,
    ordinals and ranges equal those of the reference's own SequenceDeltaEvent /
    SequenceMaintenanceEvent (tests/golden/ref_events), in one flush or in flushes of 37
    messages (segment objects keep their identity across flushes), on flat documents and on
    a paged batch (ref_events_full: the configs' 10k-message C3 / C4 documents)."""
    _addon()
    fx = gu.load(name)
    got = _node("events", os.path.join(gu.GOLDEN, name + ".json.gz"), str(every), layout, timeout=600)["events"]
    for d, evs in zip(fx["docs"], got):
        assert len(evs) == len(d["events"]), d["doc"]
        for k, (g, w) in enumerate(zip(evs, d["events"])):
            assert g == w, (d["doc"], k, g, w)


@pytest.mark.gpu
def test_js_facade_readouts_match_reference():
    """GpuClient.getPosition / getContainingSegment and client.mergeTree.getLength /
    getContainingSegment / getPosition in the observer's and writers' views equal the
    reference's (tests/golden/ref_readouts), in every view of the collab window: the views
    below a writer's latest refSeq included (partial lengths, as the reference)."""
    _addon()
    fx = gu.load("ref_readouts")
    got = _node("readouts", os.path.join(gu.GOLDEN, "ref_readouts.json.gz"), timeout=600)["docs"]
    for d, g in zip(fx["docs"], got):
        want = [[r, c, n] for r, c, n, st, _ in d["lengths"][::g["stride"]]]
        assert g["lengths"] == want, d["doc"]
        for q, (x, y) in enumerate(zip(g["containing"], d["containing"])):
            assert x == y[:4], (d["doc"], q, x, y)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ref_snap", "ref_snap_body"])
def test_js_facade_snapshot_matches_reference(name):
    """Client.snapshot through the Node facade (new format: SnapshotV1 extracted on the GPU,
    emitted by js/snapshot.js): every blob equals, byte for byte, the summary the reference
    wrote for the same replica (SEQ/sequence.ts:576, MT/snapshotV1.ts:87-252)."""
    _addon()
    fx = gu.load(name)
    got = _node("snapemit", os.path.join(gu.GOLDEN, name + ".json.gz"), timeout=600)
    for d in fx["docs"]:
        assert got[d["doc"] if isinstance(d["doc"], str) else str(d["doc"])] == d["chunks"], (name, d["doc"])


@pytest.mark.gpu
def test_js_facade_flush_async_equals_flush():
    """flushAsync (napi_async_work: the GPU batch runs off the Node thread) gives the same
    documents as flush, and the batch refuses other calls while it is in flight."""
    _addon()
    got = _node("async", os.path.join(gu.GOLDEN, "ref_c3.json.gz"), "250", timeout=600)
    assert got["equal"] and got["texts"] and got["sawBusy"]
