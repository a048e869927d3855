"""Helpers turning reference-generated golden fixtures (tests/golden/*.json.gz, made by
tests/golden/make_golden.py from the reference itself) into wire-format inputs and
id-space expected outputs, and comparing implementation outputs against them."""
import gzip
import json
import os

import numpy as np

from fluidframework_amd.snapshot import SnapshotBatch, decode_chunks
from fluidframework_amd.wire import Batch, Interner, compact_msgs_to_dicts, from_fixture

MAINT_FIXTURES = ["ref_small", "ref_c2", "ref_c3", "ref_c4", "ref_ext", "ref_ext_long", "ref_farm", "ref_c3_full",
                  "ref_c4_full"]
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
INT_MIN = -2 ** 31
ALL_FIXTURES = ["ref_small", "ref_c2", "ref_c3", "ref_c4", "ref_ext", "ref_ext_long", "ref_farm", "ref_c3_full",
                "ref_c4_full", "ref_combine", "ref_wide"]
# the configs' full stream lengths (10k messages per document)
FULL_FIXTURES = ["ref_c3_full", "ref_c4_full"]
# long-lived documents (30k messages)
LONG_FIXTURES = ["ref_c3_long"]
# the skewed bench's long classes: one 60k-, one 100k- and one 200k-message C3 document (the
# c3skew cap; 1k-3k pages)
XL_FIXTURES = ["ref_c3_60k", "ref_c3_xl", "ref_c3_200k"]
# more clients' overlapping removes unsettled at once than the 63 overlap slots (paged tiers:
# overflow sets)
WIDE_FIXTURES = ["ref_wide400", "ref_wide_long"]
SNAP_FIXTURES = ["ref_snap", "ref_snap_body", "ref_snap_files"]
# error model (tests/golden/make_golden.py --errors): the reference's throw -> mt_doc_status
ERROR_STATUS = {
    "Incoming remote op sequence# <= local collabWindow's currentSequence#": 2,   # MT/client.ts:462-463
    "Incoming remote op minSequence# < local collabWindow's minSequence#": 3,      # MT/client.ts:464-465
    "Incoming op sequence# < local collabWindow's currentSequence#": 7,            # MT/client.ts:824
    "Incoming op sequence# < minSequence#": 8,                                     # MT/client.ts:826
    "false == true": 9,                                                            # MT/mergeTree.ts:1755
}


def error_status(doc):
    return ERROR_STATUS[doc["error"]["message"]]


def load(name):
    with gzip.open(os.path.join(GOLDEN, name + ".json.gz"), "rt") as fh:
        return json.load(fh)


def maint_counts(name):
    """Reference [SPLIT, APPEND, UNLINK] maintenance-event counts per document of a replay
    fixture (tests/golden/make_maint.py), or None when the fixture has none."""
    with open(os.path.join(GOLDEN, "ref_maint.json")) as f:
        return json.load(f).get(name)


def interner_for(fixture):
    return Interner(synthetic=not fixture["config"].get("ext", False))


def encode_docs(fixture, interner, docs=None):
    b = Batch(interner)
    for d in (fixture["docs"] if docs is None else docs):
        # a farm's observer (client 0) has its own long id: short id 0, as in the reference
        own = {f"client-{d['observer_name']}": 0} if "observer_name" in d else None
        b.add_doc(d["seed_text"], compact_msgs_to_dicts(d["msgs"]), clients=own)
    return b.arrays()


def _sid(v):
    """value id as int32 (the oracle reports signed ints)."""
    return v - 2 ** 32 if v >= 2 ** 31 else v


def expected(doc, interner):
    out = doc["out"]
    segs = []
    seg_props = []
    for r in out["segs"]:
        segs.append([r["len"], r["seq"], r["cli"], INT_MIN if r["rseq"] is None else r["rseq"],
                     INT_MIN if r["rcli"] is None else r["rcli"], len(r["ovl"]),
                     -1 if r["marker"] is None else r["marker"], 0 if r["props"] is None else 1])
        seg_props.append(None if r["props"] is None else
                         [(interner.key(k), interner.val(from_fixture(v))) for k, v in r["props"].items()])
    flat = []
    for seq, kind, n, dsegs in out["deltas"]:
        flat += [seq, kind, n]
        for s in dsegs:
            flat += [s[0], s[1]]
            if kind == 2:
                pd = s[2]
                flat.append(len(pd))
                for k, v in pd.items():
                    flat += [interner.key(k), _sid(interner.val(from_fixture(v)))]
    return dict(text=out["text"], length=out["length"], leaves=out["leaves"], segs=segs,
                seg_props=seg_props, deltas=flat)


def expected_live(doc, interner):
    """expected() of a live-participant fixture (ref_live*): propertyDeltas undefined -> -1."""
    exp = expected(dict(doc, out=dict(doc["out"], deltas=[])), interner)
    flat = []
    for seq, kind, n, dsegs in doc["out"]["deltas"]:
        flat += [seq, kind, n]
        for s in dsegs:
            flat += [s[0], s[1]]
            if kind == 2:
                if len(s) < 3:          # propertyDeltas undefined: an outstanding local rewrite
                    flat.append(-1)
                    continue
                flat.append(len(s[2]))
                for k, v in s[2].items():
                    flat += [interner.key(k), _sid(interner.val(v))]
    exp["deltas"] = flat
    return exp


def live_entries(doc, local="local-0"):
    """A live fixture document without reconnects -> Batch.add_live_doc entries."""
    ent = []
    for ev in doc["events"]:
        if ev[0] == "L":
            ent.append(("local", ev[1]))
        else:
            _, cid, seq, ref, msn, op = ev
            m = dict(clientId=cid, sequenceNumber=seq, referenceSequenceNumber=ref, minimumSequenceNumber=msn,
                     type="op", contents=op)
            ent.append(("ack" if cid == local else "msg", m))
    return ent


def compare_oracle(o, exp, status=0):
    errs = []
    if o["status"] != status:
        errs.append(f"status {o['status']} != {status}")
    if o["text"] != exp["text"]:
        errs.append("text")
    if o["length"] != exp["length"]:
        errs.append(f"length {o['length']} != {exp['length']}")
    if o["leaves"] != exp["leaves"]:
        errs.append("leaves")
    if o["segs"].tolist() != exp["segs"]:
        errs.append("segs")
    if o["seg_props"] != exp["seg_props"]:
        errs.append("seg_props")
    if o["deltas"] != exp["deltas"]:
        errs.append("deltas")
    return errs


# ---------------------------------------------------------------- summaries (config C5)
def encode_snap_docs(fixture, interner, docs=None):
    """(load arrays for mt_load_snapshots / orc_load, op arrays of the catch-up + tail
    messages) for snapshot fixtures (tests/golden/make_golden.py SNAP_*)."""
    sb, b = SnapshotBatch(interner), Batch(interner)
    for d in (fixture["docs"] if docs is None else docs):
        snap = decode_chunks(d["chunks"])
        clients = sb.add_doc(snap)
        b.add_doc("", list(snap.catchup) + compact_msgs_to_dicts(d.get("tail", [])), clients=clients)
    return sb.arrays(), b.arrays()


def snap_status(doc):
    """Expected document status: MT_DOC_ALIASED (10) when the reference's loadBody re-inserted
    segments of its never-emptied batch (observed on the reference during the load; the
    engine stops there, whatever the reference did next -- its setOrdinal asserts come from
    that tree), MT_DOC_INSERT_FAILED for the reference's load failure, 0
    otherwise.  Every reference-made document has one."""
    if doc.get("aliased"):
        return 10
    err = doc.get("error")
    if err is None:
        return 0
    if err.startswith("MergeTree insert failed"):
        return 1
    raise AssertionError(f"unmodelled reference error in {doc.get('doc')}: {err}")


def expected_snap(doc, interner, key="out"):
    """expected() for a loaded replica: the reference numbers the loading client after the
    header's writers (specToSegment runs before startOrUpdateCollaboration); the engine
    numbers it 0 and keeps first-seen order for the others."""
    obs = doc["observer"]

    def remap(r):
        if r is None or r < 0:
            return r
        return 0 if r == obs else (r + 1 if r < obs else r)

    out = json.loads(json.dumps(doc[key]))
    for r in out["segs"]:
        r["cli"] = remap(r["cli"])
        r["rcli"] = remap(r["rcli"])
    return expected(dict(out=out), interner)


# ---------------------------------------------------------------- rich callback streams
def _state_ids(st, interner):
    kind = ("m", st["m"]) if "m" in st else ("t", st["t"])
    props = None if st["p"] is None else tuple((interner.key(k), interner.val(from_fixture(v)))
                                                for k, v in st["p"].items())
    return kind + (props,)


def expected_rich(doc, interner):
    """The reference's callback stream (tests/golden/ref_rich: harness "rich") in id space."""
    out = []
    for ev in doc["events"]:
        if ev[0] == "D":
            _, seq, kind, segs = ev
            out.append(("D", seq, kind, tuple(
                (pos, ln, None if pd is None else tuple((interner.key(k), _sid(interner.val(from_fixture(v))))
                                                        for k, v in pd.items()), _state_ids(st, interner))
                for pos, ln, pd, st in segs)))
        else:
            _, kind, segs = ev
            out.append(("M", kind, tuple((ln, _state_ids(st, interner)) for ln, st in segs)))
    return out


def parse_rich_log(log, ext=None):
    """A rich device delta log (mt_options.delta_log_mode 1) -> expected_rich's form.  On a
    segment_ordinals handle every entry also carries [uid, position, ordinal]: with a list
    `ext`, one (events index, [(uid, position, ordinal tuple | None) per segment]) item per
    event is appended to it."""
    out, i = [], 0
    cur = []

    def state(ln):
        nonlocal i
        flags = log[i]
        i += 1
        if flags & 1:
            kind = ("m", log[i])
            i += 1
        else:
            words = (ln + 1) // 2
            units = []
            for w in log[i:i + words]:
                units += [w & 0xFFFF, (w >> 16) & 0xFFFF]
            i += words
            kind = ("t", bytes(b for u in units[:ln] for b in (u & 0xFF, u >> 8)).decode("utf-16-le",
                                                                                         errors="surrogatepass"))
        np_ = log[i]
        i += 1
        props = None
        if np_ >= 0:
            props = tuple((log[i + 2 * q], log[i + 2 * q + 1] & 0xFFFFFFFF) for q in range(np_))
            i += 2 * np_
        if flags & 4:   # uid, position at the event, ordinal length (-1: none), characters
            uid, pos, olen = log[i] & 0xFFFFFFFF, log[i + 1], log[i + 2]
            cur.append((uid, pos, tuple(log[i + 3:i + 3 + olen]) if olen >= 0 else None))
            i += 3 + max(olen, 0)
        return kind + (props,)

    while i < len(log):
        seq, kind, n = log[i:i + 3]
        i += 3
        cur = []
        if kind >= 0:
            segs = []
            for _ in range(n):
                pos, ln = log[i:i + 2]
                i += 2
                pd = None
                if kind == 2:
                    npd = log[i]
                    pd = tuple((log[i + 1 + 2 * q], log[i + 2 + 2 * q]) for q in range(npd))
                    i += 1 + 2 * npd
                segs.append((pos, ln, pd, state(ln)))
            out.append(("D", seq, kind, tuple(segs)))
        else:
            segs = []
            for _ in range(n):
                ln = log[i]
                i += 1
                segs.append((ln, state(ln)))
            out.append(("M", kind, tuple(segs)))
        if ext is not None:
            ext.append(cur)
    return out


def sorted_segment_ranges(items):
    """SequenceEvent.ranges (SEQ/sequenceDeltaEvent.ts:40-53): the event's segments added in
    order to a SortedSegmentSet (MT/sortedSegmentSet.ts:29-84) -- kept sorted by ordinal
    (JS string order: UTF-16 code units), one whose ordinal is already present dropped (Q8;
    an undefined ordinal compares false both ways, so it is found "equal" to whatever the
    binary search probes).  items: [(ordinal tuple | None, payload)]; returns the payloads
    in the set's order.  (A restatement for the tests, pinned on the reference's own events:
    tests/test_events.py.)"""
    out = []

    def lt(a, b):   # a < b as JS compares strings (undefined: never)
        return a is not None and b is not None and a < b

    for o, payload in items:
        if not out:
            out.append((o, payload))
            continue
        lo, hi = 0, len(out) - 1
        while True:
            mid = lo + (hi - lo) // 2
            m = out[mid][0]
            if lt(o, m):             # item at mid > ordinal
                if lo == mid:
                    out.insert(mid, (o, payload))
                    break
                hi = mid - 1
            elif lt(m, o):           # item at mid < ordinal
                if mid == hi:
                    out.insert(mid + 1, (o, payload))
                    break
                lo = mid + 1
            else:
                break                # exists: not added
    return [p for _, p in out]
