#!/usr/bin/env python3
"""Regenerates the golden fixtures in tests/golden/ from the reference itself.

Runs only in the build container (needs /root/reference and node): builds the transpiled
reference with oracle/build_ref.py, then drives it with oracle/ref_harness.mjs.  Each
fixture holds, per document, the input op log (compact messages) and the reference's
outputs (text, length, property runs, leaf-block partition, segment table, every delta
callback).  The fixtures are data, not reference source.

    python3 tests/golden/make_golden.py [--snapshots | --farm | --errors | --rich | --events | --live |
                                         --readouts-xl | --only name,name]
"""
import gzip
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

FIXTURES = {
    # name: (base config from bench/configs.json or inline, overrides, docs)
    "ref_c2": ("c2", {"ops": 2000}, 4),
    "ref_c3": ("c3", {"ops": 2500}, 4),
    "ref_c4": ("c4", {"ops": 3000}, 3),
    # the configs' full stream lengths (C3 / C4 at 10k messages): thousands of live segments,
    # deep paged layouts, page splits and repacks late in the stream
    "ref_c3_full": ("c3", {"ops": 10000}, 4),
    "ref_c4_full": ("c4", {"ops": 10000}, 2),
    # non-rewrite combining ops: incr / consensus / unknown names leave NaN,
    # undefined and {value: undefined, seq} in property sets
    "ref_combine": (None, {"ext": True, "seed": 4242, "ops": 700, "writers": 5, "lag": 40, "seed_len": 40,
                           "p_insert": 0.4, "p_remove": 0.2, "text_max": 12, "p_newline": 0.05,
                           "p_len_continue": 0.8, "p_insert_props": 0.3, "n_keys": 4,
                           "max_keys_per_op": 3, "p_marker": 0.05, "p_rewrite": 0.2, "p_combine": 0.4,
                           "p_group": 0.05, "p_noop": 0.02, "p_empty": 0.02, "p_oob": 0.02}, 8),
    # 200 writers, lag 100: overlapping removes by short ids far above 64 (removedClientOverlap
    # is an unbounded list; the device masks index reusable overlap slots)
    "ref_wide": ("c4", {"ops": 4000, "writers": 200, "lag": 100, "seed": 7171}, 2),
    # 200 writers, lag 400: ~80 clients' overlapping removes unsettled at once -- more than the
    # 63 overlap slots, so the device keeps overflow sets (MT_OVF_BIT)
    "ref_wide400": ("c4", {"ops": 3000, "writers": 200, "lag": 400, "seed": 7272}, 2),
    # 200 writers, lag 400, removes 0.5, over 60k messages: overflow sets made all along the
    # document's life, few live at once (the arena is compacted, not grown without bound)
    "ref_wide_long": ("c4", {"ops": 60000, "writers": 200, "lag": 400, "seed": 7373, "p_insert": 0.4,
                             "p_remove": 0.5}, 1),
    # a long-lived document: 30k messages (~45k segment ids created, ~12k live segments)
    "ref_c3_long": ("c3", {"ops": 30000}, 2),
    # the long classes of the skewed bench (c3skew: 40k-200k messages; 1.5k-3.2k pages): one
    # C3-mix document of 60k and one of 100k messages
    "ref_c3_60k": ("c3", {"ops": 60000, "seed": 6060}, 1),
    "ref_c3_xl": ("c3", {"ops": 100000, "seed": 10100}, 1),
    # the c3skew cap: one C3-mix document of 200k messages (~3 000 pages at its peak)
    "ref_c3_200k": ("c3", {"ops": 200000, "seed": 20200}, 1),
    "ref_small": ("c2", {"ops": 60, "seed_len": 5, "writers": 3, "lag": 6}, 24),
    "ref_ext": (None, {"ext": True, "seed": 77, "ops": 700, "writers": 5, "lag": 40, "seed_len": 40,
                       "p_insert": 0.5, "p_remove": 0.3, "text_max": 12, "p_newline": 0.08,
                       "p_len_continue": 0.8, "p_insert_props": 0.3, "n_keys": 5,
                       "max_keys_per_op": 3, "p_marker": 0.1, "p_rewrite": 0.3, "p_group": 0.1,
                       "p_noop": 0.05, "p_empty": 0.05, "p_oob": 0.05}, 8),
    "ref_ext_long": (None, {"ext": True, "seed": 91, "ops": 1500, "writers": 12, "lag": 300,
                            "seed_len": 600, "p_insert": 0.45, "p_remove": 0.35, "text_max": 300,
                            "p_newline": 0.002, "p_len_continue": 0.97, "p_insert_props": 0.2,
                            "n_keys": 4, "max_keys_per_op": 2, "p_marker": 0.02, "p_rewrite": 0.2,
                            "p_group": 0.05, "p_noop": 0.02, "p_empty": 0.01, "p_oob": 0.02}, 3),
}

# Cold catch-up (config C5): observer after `ops` messages -> SnapshotV1 summary
# (chunkSize `chunk`) -> fresh Client.load -> `tail` generated messages (harness "snap").
# settle: every writer caught up before the summary (no merge info); "alternate" = even docs.
SNAP_BASE = {"seed": 5150, "writers": 4, "lag": 32, "seed_len": 64, "p_insert": 0.5, "p_remove": 0.3,
             "text_max": 8, "p_newline": 0.02, "p_len_continue": 0.75, "p_insert_props": 0.2, "n_keys": 8,
             "n_values": 16, "p_null": 0.1, "max_keys_per_op": 2}
SNAP_FIXTURES = {
    # header-only summaries (2-8 KB documents fit one 10000-unit chunk), 64-op tails as in C5
    "ref_snap": (dict(SNAP_BASE, ops=500, tail=64, chunk=10000, settle="alternate"), 16),
    # header + body chunks: settled documents load; unsettled ones hit SURVEY Q6 (the body
    # append resolves root.cachedLength in view (NonCollabClient, 0): "insert failed")
    # 64 documents: unsettled bodies that survive the Q6 failure hit loadBody's re-insertion
    # (MT_DOC_ALIASED; docs 33 and 53)
    "ref_snap_body": (dict(SNAP_BASE, seed=5151, writers=3, ops=300, tail=64, chunk=150, settle="alternate"), 64),
}
# The reference's own summary fixtures (SEQ/test/snapshots, data files of its tests),
# loaded and followed by a generated tail (harness "loadfile").
SNAP_FILES = ["v1/headerOnly", "v1/headerAndBody", "v1/largeBody", "v1/withMarkers", "v1/withAnnotations",
              "legacy/headerOnly", "legacy/withAnnotations", "legacyWithCatchUp/headerAndBody"]
SNAP_FILE_CFG = dict(SNAP_BASE, seed=5152, tail=40)
SNAP_DIR = "/root/reference/packages/dds/sequence/src/test/snapshots"


def _dump(name, data):
    with gzip.open(os.path.join(HERE, name + ".json.gz"), "wt") as fh:
        json.dump(data, fh, separators=(",", ":"))


def make_snapshot_fixtures():
    for name, (cfg, ndocs) in SNAP_FIXTURES.items():
        with tempfile.TemporaryDirectory() as td:
            cp, op = os.path.join(td, "cfg.json"), os.path.join(td, "out.json")
            json.dump(cfg, open(cp, "w"))
            subprocess.check_call(["node", os.path.join(REPO, "oracle", "ref_harness.mjs"), "snap", cp, "0",
                                   str(ndocs), op])
            data = json.load(open(op))
        for d in data["docs"]:
            for k in ("out", "load_out"):
                if k in d:
                    d[k].pop("tree", None)
        _dump(name, data)
        print(name, ndocs, "docs", sum("error" in d for d in data["docs"]), "reference errors")
    with tempfile.TemporaryDirectory() as td:
        cp, op = os.path.join(td, "cfg.json"), os.path.join(td, "out.json")
        json.dump(SNAP_FILE_CFG, open(cp, "w"))
        files = [os.path.join(SNAP_DIR, f + ".json") for f in SNAP_FILES]
        subprocess.check_call(["node", os.path.join(REPO, "oracle", "ref_harness.mjs"), "loadfile", cp, op] + files)
        data = json.load(open(op))
    for d in data["docs"]:
        for k in ("out", "load_out"):
            d[k].pop("tree", None)
    _dump("ref_snap_files", data)
    print("ref_snap_files", len(data["docs"]), "docs")


# Config C1: the reference's conflict farm (MTT/client.conflictFarm.spec.ts defaultOptions,
# its seeds) run unchanged; the fixture is client 0's (the observer's) message stream.
FARM_MIN_LENGTHS = [1, 16, 512]
FARM_MAX_CLIENTS = 8


def make_farm_fixture():
    with tempfile.TemporaryDirectory() as td:
        op = os.path.join(td, "out.json")
        subprocess.check_call(["node", os.path.join(REPO, "oracle", "ref_harness.mjs"), "farm", op,
                               str(FARM_MAX_CLIENTS)] + [str(m) for m in FARM_MIN_LENGTHS])
        data = json.load(open(op))
    data["config"]["ext"] = True          # real (non-synthetic) property interning
    for d in data["docs"]:
        d["out"].pop("tree", None)
    _dump("ref_farm", data)
    print("ref_farm", len(data["docs"]), "docs", sum(len(d["msgs"]) for d in data["docs"]), "messages")


# Error model: generated streams with one fault injected per document, replayed by the
# reference until its first throw (harness "replayerr"); the fixture holds the error and the
# observer's state at the throw.  Faults trigger completeAndLogOp (MT/client.ts:462-465),
# updateSeqNumbers (:824-826) and setMinSeq (MT/mergeTree.ts:1755).
ERR_CFG = {"ops": 80, "seed_len": 12, "writers": 3, "lag": 6}
ERR_KINDS = ["seq_dup_op", "msn_back_op", "seq_back_noop", "msn_above_seq", "msn_back_noop", "group_seq_dup"]


def _inject(msgs, kind, t0):
    """msgs: compact [k, seq, ref, msn, op(, type)]; returns the faulted stream (cut after the
    fault: the reference stops there)."""
    msgs = [list(m) for m in msgs]
    k, seq, ref, msn, op = msgs[t0][:5]
    pseq, pmsn = msgs[t0 - 1][1], msgs[t0 - 1][3]
    if kind == "seq_dup_op":
        msgs[t0][1] = pseq
    elif kind == "msn_back_op":
        msgs[t0][3] = pmsn - 1
    elif kind == "seq_back_noop":
        msgs[t0] = [k, pseq - 1, ref, pmsn, None, "noop"]
    elif kind == "msn_above_seq":
        msgs[t0][3] = seq + 1
    elif kind == "msn_back_noop":
        msgs[t0] = [k, seq, ref, pmsn - 1, None, "noop"]
    elif kind == "group_seq_dup":
        msgs[t0][1] = pseq
        msgs[t0][4] = {"type": 3, "ops": [op, {"pos1": 0, "seg": "zz", "type": 0}]}
    return msgs[: t0 + 1]


def make_error_fixture():
    configs = json.load(open(os.path.join(REPO, "bench", "configs.json")))
    cfg = dict(configs["c3"], **ERR_CFG)
    ndocs = 3 * len(ERR_KINDS)
    with tempfile.TemporaryDirectory() as td:
        cp, gp, lp, op = (os.path.join(td, f) for f in ("cfg.json", "gen.json", "logs.json", "out.json"))
        json.dump(cfg, open(cp, "w"))
        subprocess.check_call(["node", os.path.join(REPO, "oracle", "ref_harness.mjs"), "gen", cp, "0", str(ndocs), gp])
        gen = json.load(open(gp))
        docs = []
        for d in gen["docs"]:
            i = d["doc"]
            kind = ERR_KINDS[i % len(ERR_KINDS)]
            t0 = 30 + 7 * (i // len(ERR_KINDS))
            docs.append(dict(doc=i, fault=kind, seed_text=d["seed_text"], msgs=_inject(d["msgs"], kind, t0)))
        json.dump({"docs": docs}, open(lp, "w"))
        subprocess.check_call(["node", os.path.join(REPO, "oracle", "ref_harness.mjs"), "replayerr", lp, op])
        outs = json.load(open(op))["docs"]
    for d, o in zip(docs, outs):
        d["out"], d["error"] = o["out"], o["error"]
        assert d["error"] is not None, d["fault"]
    _dump("ref_errors", dict(config=cfg, docs=docs))
    print("ref_errors", len(docs), "docs", sorted({d["error"]["message"][:40] for d in docs}))


# Callback streams with the segments' state (harness "rich"): every mergeTreeDeltaCallback and
# mergeTreeMaintenanceCallback of replays of existing fixtures' streams (first documents).
RICH_FROM = [("ref_ext", 4), ("ref_c3", 2), ("ref_combine", 2)]


def make_rich_fixture():
    out = []
    with tempfile.TemporaryDirectory() as td:
        for name, n in RICH_FROM:
            with gzip.open(os.path.join(HERE, name + ".json.gz"), "rt") as fh:
                fx = json.load(fh)
            docs = [dict(doc=f"{name}/{d['doc']}", seed_text=d["seed_text"], msgs=d["msgs"]) for d in fx["docs"][:n]]
            lp, op = os.path.join(td, "logs.json"), os.path.join(td, "out.json")
            json.dump({"docs": docs}, open(lp, "w"))
            subprocess.check_call(["node", os.path.join(REPO, "oracle", "ref_harness.mjs"), "rich", lp, op])
            ev = json.load(open(op))["docs"]
            for d, e in zip(docs, ev):
                d["events"] = e["events"]
                d["source"] = name
                out.append(d)
    _dump("ref_rich", dict(config={"ext": True, "sources": RICH_FROM}, docs=out))
    print("ref_rich", len(out), "docs", sum(len(d["events"]) for d in out), "events")


# SharedSegmentSequence's event objects (harness "events"): the reference's own
# SequenceDeltaEvent / SequenceMaintenanceEvent built in every callback -- positions and
# ordinals of the callback segments, and the ranges the events keep (ordinal order, equal
# ordinals dropped).  Streams: the rich fixture's sources plus deeper trees.
EVENTS_FROM = RICH_FROM + [("ref_c4", 1), ("ref_wide", 1), ("ref_ext_long", 1)]


# The configs' full-length streams (C3 / C4 at 10k messages, paged-size documents: thousands of
# live segments, page splits and repacks) for the paged layout's ordinals.
EVENTS_FULL_FROM = [("ref_c3_full", 1), ("ref_c4_full", 1)]
# more clients overlapping at once than the 63 overlap slots: the paged layout's overflow sets
EVENTS_WIDE_FROM = [("ref_wide400", 2)]


def make_events_fixture(name="ref_events", sources=EVENTS_FROM):
    out = []
    with tempfile.TemporaryDirectory() as td:
        for name_src, n in sources:
            with gzip.open(os.path.join(HERE, name_src + ".json.gz"), "rt") as fh:
                fx = json.load(fh)
            docs = [dict(doc=f"{name_src}/{d['doc']}", seed_text=d["seed_text"], msgs=d["msgs"]) for d in fx["docs"][:n]]
            lp, op = os.path.join(td, "logs.json"), os.path.join(td, "out.json")
            json.dump({"docs": docs}, open(lp, "w"))
            subprocess.check_call(["node", os.path.join(REPO, "oracle", "ref_harness.mjs"), "events", lp, op])
            ev = json.load(open(op))["docs"]
            for d, e in zip(docs, ev):
                d["events"] = e["events"]
                d["source"] = name_src
                out.append(d)
    _dump(name, dict(config={"ext": True, "sources": sources}, docs=out))
    print(name, len(out), "docs", sum(len(d["events"]) for d in out), "events")


# long documents grown through page splits and repacks (>= 1k pages): read-outs on the paged
# and HBM-page-metadata (kHM) tiers
READOUTS_XL_FROM = [("ref_c3_60k", 1), ("ref_wide_long", 1)]


# Read-outs of the final replicas (harness "readouts"): MergeTree.getLength(refSeq, clientId),
# getContainingSegment(pos, refSeq, clientId) and getPosition in the observer's and the
# writers' views, on the events fixture's streams.
def make_readouts_fixture(out_name="ref_readouts", sources=EVENTS_FROM):
    out = []
    with tempfile.TemporaryDirectory() as td:
        for name, n in sources:
            with gzip.open(os.path.join(HERE, name + ".json.gz"), "rt") as fh:
                fx = json.load(fh)
            docs = [dict(doc=f"{name}/{d['doc']}", seed_text=d["seed_text"], msgs=d["msgs"]) for d in fx["docs"][:n]]
            lp, op = os.path.join(td, "logs.json"), os.path.join(td, "out.json")
            json.dump({"docs": docs}, open(lp, "w"))
            subprocess.check_call(["node", os.path.join(REPO, "oracle", "ref_harness.mjs"), "readouts", lp, op])
            for d, r in zip(docs, json.load(open(op))["docs"]):
                d.update(r)
                d["source"] = name
                out.append(d)
    _dump(out_name, dict(config={"ext": True, "sources": sources}, docs=out))
    print(out_name, len(out), "docs", sum(len(d["containing"]) for d in out), "queries")


# Live-client path (harness "live"): a participant client's own unsequenced
# ops, their acks, remote writers' ops resolved around unacked segments, and reconnects with
# regeneratePendingOp.  Few keys / values: remote annotates collide with pending local ones.
LIVE_BASE = {"writers": 4, "lag": 16, "seed_len": 24, "text_max": 6, "p_insert": 0.5, "p_remove": 0.25,
             "p_newline": 0.02, "p_len_continue": 0.6, "p_insert_props": 0.2, "n_keys": 4, "n_values": 4,
             "max_keys_per_op": 2, "p_null": 0.1, "p_rewrite": 0.3}
LIVE_FIXTURES = {
    "ref_live": (dict(LIVE_BASE, seed=4242, steps=600, p_local=0.35, p_reconnect=0.01, p_ack=0.45), 6),
    # long runs: thousands of segments, many zamboni passes around pending segments
    "ref_live_long": (dict(LIVE_BASE, seed=4343, steps=4000, writers=8, lag=48, p_local=0.3, p_reconnect=0.004,
                           p_ack=0.6, n_keys=8, n_values=16), 3),
    # a long-lived participant: 20k events, thousands of live segments, reconnects
    "ref_live_xl": (dict(LIVE_BASE, seed=4747, steps=20000, writers=8, lag=48, p_local=0.3, p_reconnect=0.001,
                         p_ack=0.6, n_keys=8, n_values=16), 3),
    # a participant over 60k events (~18k live segments, thousands of pending groups over its
    # life): the default live handle grows its capacities round after round (live growth step)
    "ref_live_60k": (dict(LIVE_BASE, seed=4848, steps=60000, writers=8, lag=48, p_local=0.3, p_reconnect=0.0005,
                          p_ack=0.6, n_keys=8, n_values=16), 1),
    # bench.py --config live: long streams without reconnects, replicated across documents
    "ref_live_bench": (dict(LIVE_BASE, seed=4545, steps=4000, writers=8, lag=48, p_local=0.3, p_reconnect=0.0,
                            p_ack=0.6, n_keys=8, n_values=16), 8),
    # deep segment-group queues: short text, mostly local annotates, few acks -- segments sit in
    # up to 8 pending groups at once (the device FIFO's depth)
    "ref_live_deep": (dict(LIVE_BASE, seed=4646, steps=500, seed_len=8, text_max=3, p_local=0.55, p_reconnect=0.005,
                           p_ack=0.2, p_insert=0.25, p_remove=0.05, track_depth=1), 6),
    # markers (local and remote) among the text: regenerated marker inserts
    "ref_live_markers": (dict(LIVE_BASE, seed=4444, steps=800, p_local=0.4, p_reconnect=0.015, p_ack=0.4,
                              p_marker=0.15), 4),
}


def make_live_fixtures(only=None):
    for name, (cfg, ndocs) in LIVE_FIXTURES.items():
        if only and name not in only:
            continue
        with tempfile.TemporaryDirectory() as td:
            cp, op = os.path.join(td, "cfg.json"), os.path.join(td, "out.json")
            json.dump(cfg, open(cp, "w"))
            subprocess.check_call(["node", os.path.join(REPO, "oracle", "ref_harness.mjs"), "live", cp, "0",
                                   str(ndocs), op])
            data = json.load(open(op))
        for d in data["docs"]:
            d["out"].pop("tree", None)
        _dump(name, data)
        print(name, ndocs, "docs", sum(len(d["events"]) for d in data["docs"]), "events")


def main():
    subprocess.check_call([sys.executable, os.path.join(REPO, "oracle", "build_ref.py")])
    if "--live" in sys.argv[1:]:
        only = sys.argv[sys.argv.index("--live") + 1].split(",") if len(sys.argv) > sys.argv.index("--live") + 1 else None
        make_live_fixtures(only)
        return
    if "--snapshots" in sys.argv[1:]:
        make_snapshot_fixtures()
        return
    if "--farm" in sys.argv[1:]:
        make_farm_fixture()
        return
    if "--errors" in sys.argv[1:]:
        make_error_fixture()
        return
    if "--rich" in sys.argv[1:]:
        make_rich_fixture()
        return
    if "--events" in sys.argv[1:]:
        make_events_fixture()
        make_events_fixture("ref_events_full", EVENTS_FULL_FROM)
        make_events_fixture("ref_events_wide", EVENTS_WIDE_FROM)
        make_readouts_fixture()
        make_readouts_fixture("ref_readouts_wide", EVENTS_WIDE_FROM)
        return
    if "--readouts-xl" in sys.argv[1:]:
        make_readouts_fixture("ref_readouts_xl", READOUTS_XL_FROM)
        return
    if "--wide" in sys.argv[1:]:   # (only the overflow-set fixtures)
        make_events_fixture("ref_events_wide", EVENTS_WIDE_FROM)
        make_readouts_fixture("ref_readouts_wide", EVENTS_WIDE_FROM)
        return
    only = None
    if "--only" in sys.argv[1:]:
        only = set(sys.argv[sys.argv.index("--only") + 1].split(","))
    configs = json.load(open(os.path.join(REPO, "bench", "configs.json")))
    for name, (base, over, ndocs) in FIXTURES.items():
        if only is not None and name not in only:
            continue
        cfg = dict(configs[base]) if base else {}
        cfg.update(over)
        with tempfile.TemporaryDirectory() as td:
            cp = os.path.join(td, "cfg.json")
            op = os.path.join(td, "out.json")
            json.dump(cfg, open(cp, "w"))
            subprocess.check_call(["node", os.path.join(REPO, "oracle", "ref_harness.mjs"), "gen", cp,
                                   "0", str(ndocs), op])
            data = json.load(open(op))
        for d in data["docs"]:
            d["out"].pop("tree", None)
            d.pop("ref_ns", None)
        with gzip.open(os.path.join(HERE, name + ".json.gz"), "wt") as fh:
            json.dump(data, fh, separators=(",", ":"))
        print(name, ndocs, "docs")
    if only is not None:
        return
    make_snapshot_fixtures()
    make_farm_fixture()
    make_error_fixture()
    make_rich_fixture()
    make_events_fixture()
    make_events_fixture("ref_events_full", EVENTS_FULL_FROM)
    make_events_fixture("ref_events_wide", EVENTS_WIDE_FROM)
    make_readouts_fixture()
    make_readouts_fixture("ref_readouts_wide", EVENTS_WIDE_FROM)
    make_readouts_fixture("ref_readouts_xl", READOUTS_XL_FROM)
    make_live_fixtures()


if __name__ == "__main__":
    main()
