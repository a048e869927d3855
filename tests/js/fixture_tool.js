"use strict";
// Test driver for the Node facade (fluidframework_amd/js).  Usage:
//   node tests/js/fixture_tool.js encode <fixture.json.gz>   -> JSON {ops,text,props,docOff} (hex)
//   node tests/js/fixture_tool.js replay <fixture.json.gz>   -> JSON per doc {text,length,status,props}
//   node tests/js/fixture_tool.js loadsnap <snapshot fixture> -> the same after loadSnapshots + tail
// The fixtures were produced by the reference itself (tests/golden/make_golden.py).
const fs = require("fs");
const zlib = require("zlib");
const path = require("path");
const repo = path.join(__dirname, "..", "..");
const { BatchEncoder, Interner } = require(path.join(repo, "fluidframework_amd", "js", "encode.js"));

function load(file) {
    return JSON.parse(zlib.gunzipSync(fs.readFileSync(file)).toString("utf8"));
}
function msgs(doc) {
    return doc.msgs.map((rec) => ({
        clientId: `client-${rec[0]}`, sequenceNumber: rec[1], referenceSequenceNumber: rec[2],
        minimumSequenceNumber: rec[3], contents: rec[4], type: rec.length > 5 ? rec[5] : "op",
    }));
}
const hex = (a) => Buffer.from(a.buffer, a.byteOffset, a.byteLength).toString("hex");
// NaN / undefined property values (combining ops, SURVEY Q4) as the fixtures write them
const jsReplacer = (key, v) => ((typeof v === "number" && Number.isNaN(v)) ? { $nan: 1 }
    : (v === undefined && key !== "" ? { $undef: 1 } : v));

// key-order-independent form (the reference's op objects put combiningOp first)
function canonJson(v) {
    if (Array.isArray(v)) { return v.map(canonJson); }
    if (v !== null && typeof v === "object") {
        const o = {};
        for (const k of Object.keys(v).sort()) { o[k] = canonJson(v[k]); }
        return o;
    }
    return v;
}
const [mode, file, ...extra] = process.argv.slice(2);
const fx = load(file);
if (mode === "encode") {
    const enc = new BatchEncoder(new Interner());
    for (const d of fx.docs) { enc.addDoc(msgs(d), new Map()); }
    const a = enc.arrays();
    process.stdout.write(JSON.stringify({
        ops: hex(a.ops), text: hex(a.text), props: hex(a.props), docOff: Array.from(a.docOff, Number),
        keys: enc.interner.keys, vals: enc.interner.vals,
    }));
} else if (mode === "replay" || mode === "replaydefault") {
    // replaydefault: a batch built with no options at all (the drop-in default: paged, unbounded)
    const { GpuMergeTreeBatch } = require(path.join(repo, "fluidframework_amd", "js"));
    const batch = mode === "replaydefault" ? new GpuMergeTreeBatch(fx.docs.length)
        : new GpuMergeTreeBatch(fx.docs.length, { segCapacity: 4096, textCapacity: 1 << 17 });
    batch.loadInitialText(fx.docs.map((d) => d.seed_text));
    const views = fx.docs.map((d, i) => {
        const c = batch.client(i);
        c.startOrUpdateCollaboration("observer");
        for (const m of msgs(d)) { c.applyMsg(m); }
        return c;
    });
    const out = views.map((c, i) => {
        try {
            const len = c.getLength();
            const probe = [];
            for (let p = 0; p < len; p += Math.max(1, Math.floor(len / 7))) { probe.push([p, c.getPropertiesAtPosition(p) || null]); }
            return { text: c.getText(), length: len, props: probe };
        } catch (e) {
            return { error: e.message, type: e.constructor.name };
        }
    });
    process.stdout.write(JSON.stringify({ docs: out, ms: batch.lastKernelMs() }, jsReplacer));
} else if (mode === "live") {
    // live-client streams (ref_live*): one liveClient batch, one GpuClient per document; local
    // ops through insertSegmentLocal / removeRangeLocal / annotateRangeLocal, sequenced messages
    // (acks included) through applyMsg, reconnects through regeneratePendingOp
    // (extra[0] "default": the drop-in default -- no capacity options; the live growth step
    // raises whatever the documents outgrow; no delta log)
    const { GpuMergeTreeBatch } = require(path.join(repo, "fluidframework_amd", "js", "index.js"));
    const dflt = extra[0] === "default";
    const b = new GpuMergeTreeBatch(fx.docs.length, dflt ? { liveClient: 1 }
        : { segCapacity: 16384, textCapacity: 1 << 17, liveClient: 1, deltaLogCapacity: 1 << 16 });
    b.loadInitialText(fx.docs.map((d) => d.seed_text));
    const docs = [];
    const deltas = fx.docs.map(() => []);
    const cs = fx.docs.map((d, i) => {
        const c = b.client(i);
        c.startOrUpdateCollaboration("local-0");
        // the reference harness's record: [seq or -1, operation, n, [[position, length(, propertyDeltas)]...]]
        if (!dflt) c.mergeTreeDeltaCallback = (opArgs, dargs) => {
            deltas[i].push([opArgs.sequencedMessage ? opArgs.sequencedMessage.sequenceNumber : -1, dargs.operation,
                dargs.deltaSegments.length, dargs.deltaSegments.map((x) => (x.propertyDeltas !== undefined
                    ? [x.position, x.segment.cachedLength, x.propertyDeltas] : [x.position, x.segment.cachedLength]))]);
        };
        return c;
    });
    fx.docs.forEach((d, i) => {
        const c = cs[i];
        let unseq = [];
        const errs = [];
        for (const ev of d.events) {
            if (ev[0] === "L") {
                const op = ev[1];
                let got;
                if (op.type === 0) { got = c.insertSegmentLocal(op.pos1, op.seg); }
                else if (op.type === 1) { got = c.removeRangeLocal(op.pos1, op.pos2); }
                else { got = c.annotateRangeLocal(op.pos1, op.pos2, op.props, op.combiningOp); }
                if (JSON.stringify(canonJson(got)) !== JSON.stringify(canonJson(op))) { errs.push(`local ${JSON.stringify(got)}`); }
                unseq.push(op);
            } else if (ev[0] === "M") {
                const [, cid, seq, ref, msn, op] = ev;
                if (cid === c.longClientId) { unseq.shift(); }
                c.applyMsg({ clientId: cid, sequenceNumber: seq, referenceSequenceNumber: ref,
                    minimumSequenceNumber: msn, type: "op", contents: op });
            } else {
                c.startOrUpdateCollaboration(ev[1]);
                const got = unseq.map((o) => c.regeneratePendingOp(o));
                if (JSON.stringify(canonJson(got)) !== JSON.stringify(canonJson(ev[2]))) { errs.push(`regen at ${ev[1]}`); }
                unseq = ev[2];
            }
        }
        docs.push({ doc: d.doc, text: c.getText(), length: c.getLength(), errs });
    });
    b.flush();
    docs.forEach((x, i) => { x.deltas = deltas[i]; });
    process.stdout.write(JSON.stringify({ docs }));
} else if (mode === "deltas") {
    // deltas <fixture> <deltaLogCapacity> <flushEvery>: every mergeTreeDeltaCallback the
    // facade fires while the messages are applied in flushes of <flushEvery> messages per
    // document (the device log is drained and reset at every flush)
    const { GpuMergeTreeBatch } = require(path.join(repo, "fluidframework_amd", "js"));
    const cap = parseInt(extra[0], 10), every = parseInt(extra[1], 10);
    const batch = new GpuMergeTreeBatch(fx.docs.length,
        { segCapacity: 8192, textCapacity: 1 << 17, deltaLogCapacity: cap, deltaLogMode: 0 });
    batch.loadInitialText(fx.docs.map((d) => d.seed_text));
    const calls = fx.docs.map(() => []);
    const views = fx.docs.map((d, i) => {
        const c = batch.client(i);
        c.startOrUpdateCollaboration("observer");
        c.mergeTreeDeltaCallback = (opArgs, args) => {
            calls[i].push([opArgs.sequencedMessage.sequenceNumber, args.operation,
                args.deltaSegments.map((s) => (s.propertyDeltas !== undefined ? [s.position, s.segment.cachedLength, s.propertyDeltas]
                    : [s.position, s.segment.cachedLength]))]);
        };
        return c;
    });
    const all = fx.docs.map((d) => msgs(d));
    let error = null;
    try {
        const longest = Math.max(...all.map((m) => m.length));
        for (let t = 0; t < longest; t += every) {
            all.forEach((m, i) => { for (const x of m.slice(t, t + every)) { views[i].applyMsg(x); } });
            batch.flush();
        }
    } catch (e) {
        error = e.message;
    }
    process.stdout.write(JSON.stringify({ calls, error }));
} else if (mode === "rich") {
    // rich <ref_rich fixture> <flushEvery>: every delta and maintenance callback the facade
    // fires, in the reference harness's format (segments' state at the event)
    const { GpuMergeTreeBatch } = require(path.join(repo, "fluidframework_amd", "js"));
    const every = parseInt(extra[0], 10);
    const batch = new GpuMergeTreeBatch(fx.docs.length,
        { segCapacity: 8192, textCapacity: 1 << 17, deltaLogCapacity: 1 << 20 });
    batch.loadInitialText(fx.docs.map((d) => d.seed_text));
    const events = fx.docs.map(() => []);
    const st = (seg) => Object.assign(seg.type === "Marker" ? { m: seg.refType } : { t: seg.text },
        { p: seg.properties === undefined ? null : seg.properties });
    const views = fx.docs.map((d, i) => {
        const c = batch.client(i);
        c.startOrUpdateCollaboration("observer");
        c.mergeTreeDeltaCallback = (opArgs, args) => {
            events[i].push(["D", opArgs.sequencedMessage.sequenceNumber, args.operation,
                args.deltaSegments.map((x) => [x.position, x.segment.cachedLength,
                    x.propertyDeltas === undefined ? null : x.propertyDeltas, st(x.segment)]),
                opArgs.op === undefined ? null : opArgs.op.type]);
        };
        c.mergeTreeMaintenanceCallback = (args) => {
            events[i].push(["M", args.operation, args.deltaSegments.map((x) => [x.segment.cachedLength, st(x.segment)])]);
        };
        return c;
    });
    const all = fx.docs.map((d) => msgs(d));
    let error = null;
    try {
        const longest = Math.max(...all.map((m) => m.length));
        for (let t = 0; t < longest; t += every) {
            all.forEach((m, i) => { for (const x of m.slice(t, t + every)) { views[i].applyMsg(x); } });
            batch.flush();
        }
    } catch (e) {
        error = e.message;
    }
    process.stdout.write(JSON.stringify({ events, error }, jsReplacer));
} else if (mode === "events") {
    // events <ref_events fixture> <flushEvery>: a listener's view of every event, built the
    // way SharedSegmentSequence does (sequence_event.js restates SequenceEvent.ranges) over
    // the facade's callbacks -> per event [segs: [getPosition, ordinal codes, cachedLength],
    // ranges: [[index into deltaSegments, position]]], the harness's format; "paged": the
    // documents live in the paged layout (a 16-segment LDS tier, then pages)
    const { GpuMergeTreeBatch } = require(path.join(repo, "fluidframework_amd", "js"));
    const { sequenceEventRanges } = require(path.join(__dirname, "sequence_event.js"));
    const every = parseInt(extra[0], 10);
    const paged = extra[1] === "paged" ? { ldsSegCapacity: 16, pageCapacity: 256, unsettledCapacity: 2048,
        pageHeapCapacity: 2048 } : {};
    const batch = new GpuMergeTreeBatch(fx.docs.length,
        Object.assign({ segCapacity: 8192, textCapacity: 1 << 18, deltaLogCapacity: 1 << 23 }, paged));
    batch.loadInitialText(fx.docs.map((d) => d.seed_text));
    const events = fx.docs.map(() => []);
    const codes = (seg) => (seg.ordinal === undefined ? null : Array.from(seg.ordinal, (ch) => ch.charCodeAt(0)));
    const rec = (c, args) => {
        const segs = args.deltaSegments.map((d) => [c.getPosition(d.segment), codes(d.segment), d.segment.cachedLength]);
        const ranges = sequenceEventRanges(args, c).map((r) => [args.deltaSegments.findIndex((d) => d.segment === r.segment),
            r.position]);
        return [segs, ranges];
    };
    const views = fx.docs.map((d, i) => {
        const c = batch.client(i);
        c.startOrUpdateCollaboration("observer");
        c.mergeTreeDeltaCallback = (opArgs, args) => {
            events[i].push(["D", opArgs.sequencedMessage ? opArgs.sequencedMessage.sequenceNumber : -1, args.operation,
                opArgs.sequencedMessage === undefined, ...rec(c, args)]);
        };
        c.mergeTreeMaintenanceCallback = (args) => { events[i].push(["M", args.operation, ...rec(c, args)]); };
        return c;
    });
    const all = fx.docs.map((d) => msgs(d));
    const longest = Math.max(...all.map((m) => m.length));
    for (let t = 0; t < longest; t += every) {
        all.forEach((m, i) => { for (const x of m.slice(t, t + every)) { views[i].applyMsg(x); } });
        batch.flush();
    }
    process.stdout.write(JSON.stringify({ events }));
} else if (mode === "evpin") {
    // evpin <ref_events fixture>: sequence_event.js on the fixture's own ordinals and positions
    // (CPU: pins the restatement on the reference's events)
    const { sequenceEventRanges } = require(path.join(__dirname, "sequence_event.js"));
    let bad = 0, n = 0;
    for (const d of fx.docs) {
        for (const ev of d.events) {
            const [segs, ranges] = ev[0] === "D" ? [ev[4], ev[5]] : [ev[2], ev[3]];
            const objs = segs.map(([pos, ord]) => ({ pos, ordinal: ord === null ? undefined : String.fromCharCode(...ord) }));
            const args = { operation: ev[0] === "D" ? ev[2] : ev[1], deltaSegments: objs.map((o) => ({ segment: o })) };
            const got = sequenceEventRanges(args, { getPosition: (seg) => seg.pos })
                .map((r) => [objs.indexOf(r.segment), r.position]);
            n++;
            if (JSON.stringify(got) !== JSON.stringify(ranges)) { bad++; }
        }
    }
    process.stdout.write(JSON.stringify({ events: n, mismatches: bad }));
} else if (mode === "readouts") {
    // readouts <ref_readouts fixture>: Client / MergeTree read-outs through the facade
    const { GpuMergeTreeBatch } = require(path.join(repo, "fluidframework_amd", "js"));
    const batch = new GpuMergeTreeBatch(fx.docs.length,
        { segCapacity: 8192, textCapacity: 1 << 17, deltaLogCapacity: 1 << 22 });
    batch.loadInitialText(fx.docs.map((d) => d.seed_text));
    const views = fx.docs.map((d, i) => {
        const c = batch.client(i);
        c.startOrUpdateCollaboration("observer");
        for (const m of msgs(d)) { c.applyMsg(m); }
        return c;
    });
    // every view is answered (stale ones too: partial lengths, as the reference)
    const refused = (f) => f();
    const out = fx.docs.map((d, i) => {
        const c = views[i];
        const mt = c.mergeTree;
        // lengths: every view of a document with few, every 97th of the others (fetches are per call)
        const stride = d.lengths.length > 2000 ? 97 : 1;
        const lengths = d.lengths.filter((x, k) => k % stride === 0).map(([ref, cli]) =>
            [ref, cli, cli === 0 ? c.getLength() : refused(() => mt.getLength(ref, cli))]);
        const containing = d.containing.map(([pos, ref, cli]) => refused(() => {
            const { segment, offset } = cli === 0 ? c.getContainingSegment(pos) : mt.getContainingSegment(pos, ref, cli);
            if (segment === undefined) { return [pos, ref, cli, null]; }
            const st = Object.assign(segment.type === "Marker" ? { m: segment.refType } : { t: segment.text },
                { p: segment.properties === undefined ? null : segment.properties });
            return [pos, ref, cli, [offset, mt.getPosition(segment, ref, cli), c.getPosition(segment), segment.cachedLength,
                segment.ordinal === undefined ? null : Array.from(segment.ordinal, (ch) => ch.charCodeAt(0)), st]];
        }));
        return { lengths, containing, stride };
    });
    process.stdout.write(JSON.stringify({ docs: out }, jsReplacer));
} else if (mode === "snapemit") {
    // snapemit <snapshot fixture>: each document's op stream replayed through the facade, then
    // Client.snapshot (new format) -> {doc: {path: contents}}; the reference summarised the
    // same replica into doc.chunks
    const { GpuMergeTreeBatch } = require(path.join(repo, "fluidframework_amd", "js"));
    const batch = new GpuMergeTreeBatch(fx.docs.length, { segCapacity: 4096, textCapacity: 1 << 17,
        mergeTreeSnapshotChunkSize: fx.config.chunk });
    batch.loadInitialText(fx.docs.map((d) => d.seed_text));
    const out = {};
    fx.docs.forEach((d, i) => {
        const c = batch.client(i);
        c.startOrUpdateCollaboration("observer");
        for (const m of msgs(d)) { c.applyMsg(m); }
    });
    fx.docs.forEach((d, i) => {
        const last = d.msgs[d.msgs.length - 1];
        const tree = batch.client(i).snapshot({ deltaManager: { minimumSequenceNumber: last[3], lastSequenceNumber: last[1] } },
            undefined, []);
        out[d.doc] = Object.fromEntries(tree.entries.map((e) => [e.path, e.value.contents]));
    });
    process.stdout.write(JSON.stringify(out));
} else if (mode === "async") {
    // async <fixture> <flushEvery>: flushAsync() vs flush() on two batches -> equal checksums
    const { GpuMergeTreeBatch } = require(path.join(repo, "fluidframework_amd", "js"));
    const every = parseInt(extra[0], 10);
    const mk = () => {
        const b = new GpuMergeTreeBatch(fx.docs.length, { segCapacity: 8192, textCapacity: 1 << 17 });
        b.loadInitialText(fx.docs.map((d) => d.seed_text));
        return [b, fx.docs.map((d, i) => { const c = b.client(i); c.startOrUpdateCollaboration("observer"); return c; })];
    };
    const [b1, v1] = mk(), [b2, v2] = mk();
    const all = fx.docs.map((d) => msgs(d));
    const longest = Math.max(...all.map((m) => m.length));
    (async () => {
        let sawBusy = false;
        for (let t = 0; t < longest; t += every) {
            all.forEach((m, i) => { for (const x of m.slice(t, t + every)) { v1[i].applyMsg(x); v2[i].applyMsg(x); } });
            b1.flush();
            const p = b2.flushAsync();
            try { b2.status(); } catch (e) { sawBusy = sawBusy || /in flight/.test(e.message); }
            await p;
        }
        const s = (b) => b.checksums().map((x) => [x.length, x.textHash.toString(), x.propsHash.toString(),
            x.deltaHash.toString()]);
        process.stdout.write(JSON.stringify({ equal: JSON.stringify(s(b1)) === JSON.stringify(s(b2)), sawBusy,
            texts: v2.map((c) => c.getText()).every((t, i) => t === v1[i].getText()) }));
    })().catch((e) => { console.error(e); process.exit(1); });
} else if (mode === "maint") {
    // maint <fixture.json.gz> -> [[split, append, unlink] per doc] through the facade
    const { GpuMergeTreeBatch } = require(path.join(repo, "fluidframework_amd", "js"));
    const batch = new GpuMergeTreeBatch(fx.docs.length,
        { segCapacity: 4096, textCapacity: 1 << 17, deltaLogCapacity: 1 << 18 });
    batch.loadInitialText(fx.docs.map((d) => d.seed_text));
    const views = fx.docs.map((d, i) => {
        const c = batch.client(i);
        c.startOrUpdateCollaboration("observer");
        for (const m of msgs(d)) { c.applyMsg(m); }
        return c;
    });
    const out = views.map((c) => { const m = c.getMaintenanceCounts(); return [m.split, m.append, m.unlink]; });
    process.stdout.write(JSON.stringify({ docs: out }));
} else if (mode === "snapenc") {
    const { SnapshotEncoder, decodeChunks } = require(path.join(repo, "fluidframework_amd", "js", "snapshot.js"));
    const { Grow } = require(path.join(repo, "fluidframework_amd", "js", "encode.js"));
    const enc = new SnapshotEncoder(new Interner(), Grow);
    for (const d of fx.docs) { enc.addDoc(decodeChunks(d.chunks), new Map()); }
    const a = enc.arrays();
    process.stdout.write(JSON.stringify({
        segs: hex(a.segs.subarray(0, a.nSegs * 32)), text: hex(a.text), props: hex(a.props),
        docSegOff: Array.from(a.docSegOff, Number), nHeader: Array.from(a.nHeader),
        minSeq: Array.from(a.minSeq), curSeq: Array.from(a.curSeq),
    }));
} else if (mode === "snapnative") {
    // the same arrays from the native decoder (include/mt_snapshot.h through the addon)
    const { decodeSummaries } = require(path.join(repo, "fluidframework_amd", "js"));
    const a = decodeSummaries(fx.docs.map((d) => d.chunks), new Interner(), 4);
    process.stdout.write(JSON.stringify({
        segs: hex(a.segs), text: hex(a.text), props: hex(a.props),
        docSegOff: Array.from(a.docSegOff, Number), nHeader: Array.from(a.nHeader),
        minSeq: Array.from(a.minSeq), curSeq: Array.from(a.curSeq),
        clients: a.clients.map((m) => Array.from(m.entries())), catchup: a.catchup,
    }));
} else if (mode === "loadsnap") {
    // summaries (snapshot fixtures: reference-written chunks) loaded through
    // GpuMergeTreeBatch.loadSnapshots, then the tail messages through GpuClient.applyMsg
    const { GpuMergeTreeBatch } = require(path.join(repo, "fluidframework_amd", "js"));
    const docs = fx.docs;   // every reference-made document (load failures throw on the first call)
    const batch = new GpuMergeTreeBatch(docs.length, { segCapacity: 4096, textCapacity: 1 << 17 });
    batch.loadSnapshots(docs.map((d) => d.chunks));
    const out = docs.map((d, i) => {
        const c = batch.client(i);
        c.startOrUpdateCollaboration("loader");
        try {
            for (const m of msgs({ msgs: d.tail || [] })) { c.applyMsg(m); }
            const len = c.getLength();
            const probe = [];
            for (let p = 0; p < len; p += Math.max(1, Math.floor(len / 7))) { probe.push([p, c.getPropertiesAtPosition(p) || null]); }
            return { doc: d.doc, text: c.getText(), length: len, props: probe };
        } catch (e) {
            return { doc: d.doc, error: e.message, type: e.constructor.name };
        }
    });
    process.stdout.write(JSON.stringify({ docs: out }));
}
