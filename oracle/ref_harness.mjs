// TEST INFRASTRUCTURE ONLY: drives the *transpiled reference* (oracle/_ref, built by
// oracle/build_ref.py from /root/reference) as the observer replica of SURVEY.md App. A:
//   observer = new Client(segmentFromSpec, logger)            MT/client.ts:75-84
//   seed text inserted before collaboration (seq 0, client -1) MT/client.ts:202, 394-442
//   observer.startOrUpdateCollaboration("observer")            MT/client.ts:1053-1073
//   observer.applyMsg(msg) for every sequenced message         MT/client.ts:797-819
// and records what the product must reproduce bit-exactly: final text, length, property
// runs, every mergeTreeDeltaCallback (op kind, observer position, length, propertyDeltas),
// plus the leaf segment table / B-tree shape for debugging.
//
// Modes:
//   gen   : synthesise op streams with the shared generator (DESIGN.md "Synthetic op
//           streams"); the writer's view length comes from the reference itself
//           (MergeTree.getLength(refSeq, clientId), MT/mergeTree.ts:1610).
//   replay: replay op logs given as JSON.
// Usage:
//   node oracle/ref_harness.mjs gen  <config.json> <doc_begin> <doc_end> <out.json>
//   node oracle/ref_harness.mjs replay <logs.json> <out.json>
//   node oracle/ref_harness.mjs replayerr <logs.json> <out.json>
//   node oracle/ref_harness.mjs snap <config.json> <doc_begin> <doc_end> <out.json>
//   node oracle/ref_harness.mjs loadfile <config.json> <out.json> <snapshot.json>...
//   node oracle/ref_harness.mjs farm <out.json> <maxClients> <minLength>...
//   node oracle/ref_harness.mjs live <config.json> <doc_begin> <doc_end> <out.json>
import fs from "fs";
import * as MT from "./_ref/mt/index.mjs";
import { SnapshotV1 } from "./_ref/mt/snapshotV1.mjs";
import { MockStorage } from "./_ref/shims/test-runtime-utils.mjs";
import random from "./_ref/shims/random-js.mjs";
import { annotateRange, insertAtRefPos, removeRange, runMergeTreeOperationRunner, generateClientNames }
    from "./_ref/mt/test/mergeTreeOperationRunner.mjs";
import { TestClient } from "./_ref/mt/test/testClient.mjs";
import { SequenceDeltaEvent, SequenceMaintenanceEvent } from "./_ref/seq/sequenceDeltaEvent.mjs";

const { Client, TextSegment, Marker } = MT;

function segmentFromSpec(spec) {           // SEQ/sequenceFactory.ts:31-37
    const t = TextSegment.fromJSONObject(spec);
    if (t) { return t; }
    const m = Marker.fromJSONObject(spec);
    if (m) { return m; }
    throw new Error("bad spec");
}
const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };

// ---------------------------------------------------------------- shared generator PRNG
// xoshiro128** seeded through splitmix32 (identical in oracle/mt_oracle.c and the HIP
// generator kernel).
function splitmix32(state) {
    state.x = (state.x + 0x9E3779B9) | 0;
    let z = state.x;
    z = Math.imul(z ^ (z >>> 16), 0x85EBCA6B);
    z = Math.imul(z ^ (z >>> 13), 0xC2B2AE35);
    return (z ^ (z >>> 16)) >>> 0;
}
class Rng {
    constructor(seed, doc) {
        const st = { x: (seed ^ Math.imul(doc + 1, 0x9E3779B9)) | 0 };
        this.s = [splitmix32(st), splitmix32(st), splitmix32(st), splitmix32(st)];
    }
    next() {
        const s = this.s;
        const rotl = (x, k) => ((x << k) | (x >>> (32 - k))) >>> 0;
        const result = Math.imul(rotl(Math.imul(s[1], 5) >>> 0, 7), 9) >>> 0;
        const t = (s[1] << 9) >>> 0;
        s[2] = (s[2] ^ s[0]) >>> 0;
        s[3] = (s[3] ^ s[1]) >>> 0;
        s[1] = (s[1] ^ s[2]) >>> 0;
        s[0] = (s[0] ^ s[3]) >>> 0;
        s[2] = (s[2] ^ t) >>> 0;
        s[3] = rotl(s[3], 11);
        return result;
    }
    uniform(n) { return Math.floor(this.next() * n / 4294967296); }
}
const frac = (p) => Math.floor(p * 4294967296);

function genText(rng, n, pNl) {
    let s = "";
    for (let i = 0; i < n; i++) {
        const v = rng.next();
        s += (v < pNl) ? "\n" : String.fromCharCode(97 + rng.uniform(26));
    }
    return s;
}
function genProps(rng, cfg) {
    const nk = 1 + rng.uniform(cfg.max_keys_per_op);
    const props = {};
    const seen = new Set();
    for (let j = 0; j < nk; j++) {
        const key = rng.uniform(cfg.n_keys);
        const isNull = rng.next() < frac(cfg.p_null);
        const val = rng.uniform(cfg.n_values);
        if (seen.has(key)) { continue; }
        seen.add(key);
        props[`k${key}`] = isNull ? null : val;
    }
    return props;
}

// ---------------------------------------------------------------- observer replica
function makeObserver(seedText) {
    const c = new Client(segmentFromSpec, logger);
    if (seedText.length > 0) {
        c.insertSegmentLocal(0, TextSegment.make(seedText));
    }
    c.startOrUpdateCollaboration("observer");
    const deltas = [];
    c.mergeTreeDeltaCallback = (opArgs, dargs) => {
        const mt = c.mergeTree;
        const cw = mt.getCollabWindow();
        const rec = [opArgs.sequencedMessage ? opArgs.sequencedMessage.sequenceNumber : -1,
            dargs.operation, dargs.deltaSegments.length];
        const segs = [];
        for (const d of dargs.deltaSegments) {
            const seg = d.segment;
            const pos = seg.parent ? mt.getPosition(seg, cw.currentSeq, cw.clientId) : -1;
            segs.push(d.propertyDeltas !== undefined ? [pos, seg.cachedLength, jsClone(d.propertyDeltas)]
                : [pos, seg.cachedLength]);
        }
        rec.push(segs);
        deltas.push(rec);
    };
    return { c, deltas };
}

function makeMsg(k, seq, ref, msn, cseq, contents) {
    return {
        clientId: `client-${k}`, sequenceNumber: seq, referenceSequenceNumber: ref,
        minimumSequenceNumber: msn, clientSequenceNumber: cseq, type: "op", contents,
        timestamp: 0, term: 1, traces: [],
    };
}

// Property values as the reference holds them, JS-only values included: non-rewrite
// combining ops leave NaN (incr), undefined and {value: undefined, seq} (consensus) in
// property sets (SURVEY Q4).  jsClone copies without JSON's loss; jsReplacer writes them as
// {"$nan": 1} / {"$undef": 1} in fixtures.
function jsClone(v) {
    if (Array.isArray(v)) { return v.map(jsClone); }
    if (v !== null && typeof v === "object") {
        const o = {};
        for (const k of Object.keys(v)) { o[k] = jsClone(v[k]); }
        return o;
    }
    return v;
}
function jsReplacer(key, v) {
    if (typeof v === "number" && Number.isNaN(v)) { return { $nan: 1 }; }
    if (v === undefined && key !== "") { return { $undef: 1 }; }
    return v;
}

function collectOutputs(c, deltas) {
    const mt = c.mergeTree;
    const cw = mt.getCollabWindow();
    const text = c.createTextHelper().getText(cw.currentSeq, cw.clientId);
    const segs = [];
    const runs = [];
    const leaves = [];
    const shape = (block) => {
        const out = [];
        for (let i = 0; i < block.childCount; i++) {
            const ch = block.children[i];
            if (ch.isLeaf()) {
                out.push(null);
            } else {
                out.push(shape(ch));
            }
        }
        return out;
    };
    mt.walkAllSegments(mt.root, (seg) => {
        const rec = {
            len: seg.cachedLength, seq: seg.seq, cli: seg.clientId,
            rseq: seg.removedSeq === undefined ? null : seg.removedSeq,
            rcli: seg.removedClientId === undefined ? null : seg.removedClientId,
            ovl: seg.removedClientOverlap ? [...seg.removedClientOverlap] : [],
            marker: Marker.is(seg) ? seg.refType : null,
            // copied now: a later annotate mutates the live object (outputs taken mid-run)
            props: seg.properties === undefined ? null : jsClone(seg.properties),
        };
        segs.push(rec);
        if (seg.removedSeq === undefined) {
            const p = seg.properties === undefined ? null : JSON.stringify(seg.properties);
            if (runs.length && runs[runs.length - 1][1] === p) {
                runs[runs.length - 1][0] += seg.cachedLength;
            } else {
                runs.push([seg.cachedLength, p]);
            }
        }
        return true;
    });
    // leaf-block partition: childCount of every block whose children are segments
    const walk = (block) => {
        if (block.childCount === 0 || block.children[0].isLeaf()) {
            leaves.push(block.childCount);
            return;
        }
        for (let i = 0; i < block.childCount; i++) { walk(block.children[i]); }
    };
    walk(mt.root);
    return {
        text, length: c.getLength(), currentSeq: cw.currentSeq, minSeq: cw.minSeq,
        runs: runs.map(([l, p]) => [l, p === null ? null : JSON.parse(p)]),
        segs, leaves, tree: shape(mt.root), deltas,
    };
}

function genDoc(cfg, doc) {
    const rng = new Rng(cfg.seed >>> 0, doc);
    const seedText = genText(rng, cfg.seed_len, 0);
    const { c, deltas } = makeObserver(seedText);
    const W = cfg.writers;
    const lastRef = new Array(W + 1).fill(0);
    const cseq = new Array(W + 1).fill(0);
    const msgs = [];
    const t0 = process.hrtime.bigint();
    for (let t = 1; t <= cfg.ops; t++) {
        const k = 1 + rng.uniform(W);
        let lo = Math.max(lastRef[k], t - 1 - cfg.lag);
        if (lo < 0) { lo = 0; }
        const r = lo + rng.uniform(t - 1 - lo + 1);
        lastRef[k] = r;
        let msn = Infinity;
        for (let j = 1; j <= W; j++) { msn = Math.min(msn, lastRef[j]); }
        const shortId = c.getOrAddShortClientId(`client-${k}`);
        const len = c.mergeTree.getLength(r, shortId);
        const u = rng.next();
        let op;
        if (len === 0 || u < frac(cfg.p_insert)) {
            const pos = rng.uniform(len + 1);
            const tl = 1 + rng.uniform(cfg.text_max);
            const text = genText(rng, tl, frac(cfg.p_newline));
            let seg = text;
            if (cfg.p_insert_props > 0 && rng.next() < frac(cfg.p_insert_props)) {
                seg = { text, props: genProps(rng, cfg) };
            }
            op = { pos1: pos, seg, type: 0 };
        } else {
            const p1 = rng.uniform(len);
            let n = 1;
            while (n < 64 && rng.next() < frac(cfg.p_len_continue)) { n++; }
            const p2 = Math.min(p1 + n, len);
            if (u < frac(cfg.p_insert + cfg.p_remove)) {
                op = { pos1: p1, pos2: p2, type: 1 };
            } else {
                op = { pos1: p1, pos2: p2, props: genProps(rng, cfg), type: 2 };
            }
        }
        const msg = makeMsg(k, t, r, msn, ++cseq[k], op);
        msgs.push([k, t, r, msn, op]);
        c.applyMsg(JSON.parse(JSON.stringify(msg)));
    }
    const ns = Number(process.hrtime.bigint() - t0);
    const out = collectOutputs(c, deltas);
    return { doc, seed_text: seedText, msgs, out, ref_ns: ns };
}

// Edge-case streams (fixtures only; replayed by the oracle and the HIP path, never
// re-generated by them): markers, rewrite annotates, GROUP messages, noop messages, empty
// inserts, ranges past the view end, and non-numeric / falsy property values.
const EXT_VALUES = [0, 1, "", "x", false, true, { a: 1, b: [1, 2] }, { b: [1, 2], a: 1 }, [0], "0", 2.5, null];
function genPropsExt(rng, cfg) {
    const nk = 1 + rng.uniform(cfg.max_keys_per_op);
    const props = {};
    for (let j = 0; j < nk; j++) {
        const key = `k${rng.uniform(cfg.n_keys)}`;
        const v = EXT_VALUES[rng.uniform(EXT_VALUES.length)];
        if (key in props) { continue; }
        props[key] = v;
    }
    return props;
}
function genOpExt(rng, cfg, len) {
    const u = rng.next();
    if (len === 0 || u < frac(cfg.p_insert)) {
        const pos = rng.uniform(len + 1);
        if (rng.next() < frac(cfg.p_marker)) {
            const seg = { marker: { refType: 1 + rng.uniform(2) } };
            if (rng.next() < frac(0.5)) { seg.props = genPropsExt(rng, cfg); }
            return { pos1: pos, seg, type: 0 };
        }
        const empty = rng.next() < frac(cfg.p_empty);
        const text = empty ? "" : genText(rng, 1 + rng.uniform(cfg.text_max), frac(cfg.p_newline));
        let seg = text;
        if (rng.next() < frac(cfg.p_insert_props)) { seg = { text, props: genPropsExt(rng, cfg) }; }
        return { pos1: pos, seg, type: 0 };
    }
    const p1 = rng.uniform(len);
    let n = 1;
    while (n < 300 && rng.next() < frac(cfg.p_len_continue)) { n++; }
    let p2 = Math.min(p1 + n, len);
    if (rng.next() < frac(cfg.p_oob)) { p2 = len + 1 + rng.uniform(5); }
    if (u < frac(cfg.p_insert + cfg.p_remove)) { return { pos1: p1, pos2: p2, type: 1 }; }
    const op = { pos1: p1, pos2: p2, props: genPropsExt(rng, cfg), type: 2 };
    if (cfg.p_combine && rng.next() < frac(cfg.p_combine)) {
        // non-rewrite combining ops (MT/properties.ts:26-59 via
        // MT/segmentPropertiesManager.ts:93-107): incr (with and without default/min),
        // consensus, and a name combine() does not know
        const COMBINE = [{ name: "incr" }, { name: "incr", defaultValue: 1, minValue: 0 }, { name: "consensus" },
            { name: "consensus", defaultValue: 5 }, { name: "max" }, { name: "max", defaultValue: "d" }];
        op.combiningOp = COMBINE[rng.uniform(COMBINE.length)];
    } else if (rng.next() < frac(cfg.p_rewrite)) { op.combiningOp = { name: "rewrite" }; }
    return op;
}
function genDocExt(cfg, doc) {
    const rng = new Rng(cfg.seed >>> 0, doc);
    const seedText = genText(rng, cfg.seed_len, frac(cfg.p_newline));
    const { c, deltas } = makeObserver(seedText);
    const W = cfg.writers;
    const lastRef = new Array(W + 1).fill(0);
    const cseq = new Array(W + 1).fill(0);
    const msgs = [];
    for (let t = 1; t <= cfg.ops; t++) {
        const k = 1 + rng.uniform(W);
        let lo = Math.max(lastRef[k], t - 1 - cfg.lag);
        if (lo < 0) { lo = 0; }
        const r = lo + rng.uniform(t - 1 - lo + 1);
        lastRef[k] = r;
        let msn = Infinity;
        for (let j = 1; j <= W; j++) { msn = Math.min(msn, lastRef[j]); }
        const shortId = c.getOrAddShortClientId(`client-${k}`);
        let len = c.mergeTree.getLength(r, shortId);
        let contents;
        let type = "op";
        const g = rng.next();
        if (g < frac(cfg.p_noop)) {
            type = "noop";
            contents = null;
        } else if (g < frac(cfg.p_noop + cfg.p_group)) {
            const members = [];
            const m = 2 + rng.uniform(2);
            let removed = 0;
            for (let j = 0; j < m; j++) {
                const op = genOpExt(rng, cfg, Math.max(0, len - removed));
                if (op.type === 1) { removed += Math.max(0, Math.min(op.pos2, len) - op.pos1); }
                if (op.type === 0 && typeof op.seg === "string") { len += op.seg.length; }
                members.push(op);
            }
            contents = { type: 3, ops: members };
        } else {
            contents = genOpExt(rng, cfg, len);
        }
        const msg = makeMsg(k, t, r, msn, ++cseq[k], contents);
        msg.type = type;
        msgs.push([k, t, r, msn, contents, type]);
        c.applyMsg(JSON.parse(JSON.stringify(msg)));
    }
    const out = collectOutputs(c, deltas);
    return { doc, seed_text: seedText, msgs, out, ref_ns: 0 };
}

function replayDoc(log) {
    const { c, deltas } = makeObserver(log.seed_text);
    const cseq = {};
    for (const [k, t, r, msn, op, type] of log.msgs) {
        cseq[k] = (cseq[k] || 0) + 1;
        const msg = makeMsg(k, t, r, msn, cseq[k], op);
        if (type) { msg.type = type; }
        c.applyMsg(msg);
    }
    return collectOutputs(c, deltas);
}

// replayDoc that stops at the first exception (the reference's asserts / throws, e.g.
// completeAndLogOp MT/client.ts:462-465, updateSeqNumbers :824-826, setMinSeq
// MT/mergeTree.ts:1752-1755): records the error and the observer's state at the throw.
function replayErrDoc(log) {
    const { c, deltas } = makeObserver(log.seed_text);
    const cseq = {};
    let error = null;
    for (let i = 0; i < log.msgs.length; i++) {
        const [k, t, r, msn, op, type] = log.msgs[i];
        cseq[k] = (cseq[k] || 0) + 1;
        const msg = makeMsg(k, t, r, msn, cseq[k], op);
        if (type) { msg.type = type; }
        try {
            c.applyMsg(msg);
        } catch (e) {
            error = { name: e.name, message: e.message, at: i };
            break;
        }
    }
    const out = collectOutputs(c, deltas);
    delete out.tree;
    return { out, error };
}

// Every callback the observer fires, in order, with the segments' state at the event:
// mergeTreeDeltaCallback -> ["D", seq, operation, [[position, cachedLength, propertyDeltas |
// null, state] ...]] and mergeTreeMaintenanceCallback (SPLIT/APPEND/UNLINK, MT/mergeTree.ts:
// 1343-1373, 2264-2269) -> ["M", operation, [[cachedLength, state] ...]]; state = {t: text |
// m: refType, p: properties | null}.
function segState(seg) {
    const st = Marker.is(seg) ? { m: seg.refType } : { t: seg.text };
    st.p = seg.properties === undefined ? null : jsClone(seg.properties);
    return st;
}
function replayRichDoc(log) {
    const { c } = makeObserver(log.seed_text);
    const events = [];
    c.mergeTreeDeltaCallback = (opArgs, dargs) => {
        const mt = c.mergeTree;
        const cw = mt.getCollabWindow();
        events.push(["D", opArgs.sequencedMessage ? opArgs.sequencedMessage.sequenceNumber : -1, dargs.operation,
            dargs.deltaSegments.map((d) => [d.segment.parent ? mt.getPosition(d.segment, cw.currentSeq, cw.clientId) : -1,
                d.segment.cachedLength, d.propertyDeltas === undefined ? null : jsClone(d.propertyDeltas),
                segState(d.segment)])]);
    };
    c.mergeTree.mergeTreeMaintenanceCallback = (args) => {
        events.push(["M", args.operation, args.deltaSegments.map((d) => [d.segment.cachedLength, segState(d.segment)])]);
    };
    const cseq = {};
    for (const [k, t, r, msn, op, type] of log.msgs) {
        cseq[k] = (cseq[k] || 0) + 1;
        const msg = makeMsg(k, t, r, msn, cseq[k], op);
        if (type) { msg.type = type; }
        c.applyMsg(msg);
    }
    return { doc: log.doc, events };
}

// SharedSegmentSequence's event objects over the observer (SEQ/sequence.ts:139-149): every
// callback builds the reference's own SequenceDeltaEvent / SequenceMaintenanceEvent and reads
// it as a synchronous listener does (its ranges are lazy: positions and ordinals at callback
// time).  Per event: ["D", seq, operation, isLocal, segs, ranges] / ["M", operation, segs,
// ranges] with segs[i] = [Client.getPosition(segment), segment.ordinal as char codes (null:
// none), cachedLength] for deltaSegments[i], and ranges = [[index into deltaSegments,
// position]] in the event's order (SortedSegmentSet: by ordinal, equal ordinals dropped, Q8).
function ordCodes(seg) {
    return seg.ordinal === undefined ? null : Array.from(seg.ordinal, (ch) => ch.charCodeAt(0));
}
function eventRecord(c, args, ev) {
    const segs = args.deltaSegments.map((d) => [c.getPosition(d.segment), ordCodes(d.segment), d.segment.cachedLength]);
    const ranges = ev.ranges.map((r) => [args.deltaSegments.findIndex((d) => d.segment === r.segment), r.position]);
    return [segs, ranges];
}
function replayEventsDoc(log) {
    const { c } = makeObserver(log.seed_text);
    const events = [];
    c.mergeTreeDeltaCallback = (opArgs, dargs) => {
        const ev = new SequenceDeltaEvent(opArgs, dargs, c);
        events.push(["D", opArgs.sequencedMessage ? opArgs.sequencedMessage.sequenceNumber : -1, dargs.operation,
            ev.isLocal, ...eventRecord(c, dargs, ev)]);
    };
    c.mergeTree.mergeTreeMaintenanceCallback = (args) => {
        const ev = new SequenceMaintenanceEvent(args, c);
        events.push(["M", args.operation, ...eventRecord(c, args, ev)]);
    };
    const cseq = {};
    for (const [k, t, r, msn, op, type] of log.msgs) {
        cseq[k] = (cseq[k] || 0) + 1;
        const msg = makeMsg(k, t, r, msn, cseq[k], op);
        if (type) { msg.type = type; }
        c.applyMsg(msg);
    }
    return { doc: log.doc, events };
}

// Read-outs of the final replica (MT/mergeTree.ts:1610-1667): MergeTree.getLength(refSeq,
// clientId) and getContainingSegment(pos, refSeq, clientId) in the observer's view and in every
// writer's view the collab window holds (refSeq in [minSeq, currentSeq], every writer), and
// getPosition of the found segment in that view.  A writer's view below the refSeq of its
// latest message is one the client can no longer hold ("stale", flag 1): there the reference
// answers from partial lengths that need not add up to its own leaves' nodeLength (each length
// entry also records that sum), and the replay backend refuses the query.  Segments are
// identified by their observer position and contents.
function readoutsDoc(log) {
    const { c } = makeObserver(log.seed_text);
    c.mergeTreeDeltaCallback = undefined;
    const cseq = {};
    const lastRef = {};
    for (const [k, t, r, msn, op, type] of log.msgs) {
        cseq[k] = (cseq[k] || 0) + 1;
        const msg = makeMsg(k, t, r, msn, cseq[k], op);
        if (type) { msg.type = type; }
        c.applyMsg(msg);
        const cli = c.getShortClientId(msg.clientId);
        lastRef[cli] = Math.max(lastRef[cli] === undefined ? r : lastRef[cli], r);
    }
    const mt = c.mergeTree;
    const cw = mt.getCollabWindow();
    const rng = new Rng(777, log.doc.length);
    const leafSum = (ref, cli) => {
        let s = 0;
        const walk = (b) => {
            for (let i = 0; i < b.childCount; i++) {
                const x = b.children[i];
                if (x.isLeaf()) { s += mt.nodeLength(x, ref, cli) || 0; } else { walk(x); }
            }
        };
        walk(mt.root);
        return s;
    };
    const views = [[cw.currentSeq, cw.clientId, 0]];
    for (let cli = 1; c.getLongClientId(cli) !== undefined; cli++) {
        if (lastRef[cli] === undefined) { continue; }
        for (let ref = cw.minSeq; ref <= cw.currentSeq; ref++) { views.push([ref, cli, ref < lastRef[cli] ? 1 : 0]); }
    }
    const lengths = views.map(([ref, cli, stale]) => [ref, cli, mt.getLength(ref, cli), stale, leafSum(ref, cli)]);
    // getContainingSegment / getPosition on a sample of the views: the observer's, and per
    // writer its oldest and latest views, the one at its latest refSeq, the one just below it
    // (stale) and two more drawn from the window
    const sample = [views[0]];
    const byCli = {};
    for (const v of views.slice(1)) { (byCli[v[1]] = byCli[v[1]] || []).push(v); }
    for (const cli of Object.keys(byCli)) {
        const vs = byCli[cli];
        const at = vs.findIndex((v) => v[2] === 0);
        const pick = new Set([0, vs.length - 1, rng.uniform(vs.length), rng.uniform(vs.length)]);
        if (at >= 0) { pick.add(at); }
        if (at > 0) { pick.add(at - 1); }
        for (const i of [...pick].sort((x, y) => x - y)) { sample.push(vs[i]); }
    }
    const containing = [];
    for (const [ref, cli, stale] of sample) {
        const len = mt.getLength(ref, cli);
        for (let q = 0; q < 2; q++) {
            const pos = q === 1 ? len : rng.uniform(len + 1);
            const { segment, offset } = mt.getContainingSegment(pos, ref, cli);
            if (segment === undefined) {
                containing.push([pos, ref, cli, null, stale]);
                continue;
            }
            containing.push([pos, ref, cli, [offset, mt.getPosition(segment, ref, cli),
                c.getPosition(segment), segment.cachedLength, ordCodes(segment), segState(segment)], stale]);
        }
    }
    return { doc: log.doc, minSeq: cw.minSeq, currentSeq: cw.currentSeq, lengths, containing };
}

// The ordinal invariant the GPU engine's representation rests on (mt_engine.h "segment
// ordinals"): between messages every node's ordinal is its parent's ordinal plus one
// character.  Replays each stream and checks the whole tree after every message; returns
// the number of messages checked and the first violation (null: none).
function ordProbeDoc(log) {
    const { c } = makeObserver(log.seed_text);
    c.mergeTreeDeltaCallback = undefined;
    const bad = (mt) => {
        const walk = (b) => {
            for (let i = 0; i < b.childCount; i++) {
                const x = b.children[i];
                if (x.ordinal.length !== b.ordinal.length + 1 || x.ordinal.slice(0, -1) !== b.ordinal) { return true; }
                if (!x.isLeaf() && walk(x)) { return true; }
            }
            return false;
        };
        return walk(mt.root);
    };
    const cseq = {};
    let n = 0;
    for (const [k, t, r, msn, op, type] of log.msgs) {
        cseq[k] = (cseq[k] || 0) + 1;
        const msg = makeMsg(k, t, r, msn, cseq[k], op);
        if (type) { msg.type = type; }
        c.applyMsg(msg);
        n++;
        if (bad(c.mergeTree)) { return { doc: log.doc, messages: n, violation: t }; }
    }
    return { doc: log.doc, messages: n, violation: null };
}

// Maintenance events (mergeTreeMaintenanceCallback, MT/mergeTree.ts:1343-1373 scourNode
// UNLINK/APPEND, :2264-2269 splitLeafSegment SPLIT) counted per document over the same
// observer replay as replayDoc: [SPLIT, APPEND, UNLINK].
function maintDoc(log) {
    const { c } = makeObserver(log.seed_text);
    const counts = [0, 0, 0];
    c.mergeTreeMaintenanceCallback = (args) => {
        const i = args.operation === -2 ? 0 : args.operation === -1 ? 1 : args.operation === -3 ? 2 : -1;
        if (i >= 0) { counts[i]++; }
    };
    const cseq = {};
    for (const [k, t, r, msn, op, type] of log.msgs) {
        cseq[k] = (cseq[k] || 0) + 1;
        const msg = makeMsg(k, t, r, msn, cseq[k], op);
        if (type) { msg.type = type; }
        c.applyMsg(msg);
    }
    return counts;
}

// ---------------------------------------------------------------- snapshots (config C5)
// Cold catch-up = SnapshotV1 summary + tail ops (SURVEY.md S4): the observer after K ops is
// summarised with the reference's own SnapshotV1.extractSync/emit (MT/snapshotV1.ts:87-252),
// a fresh Client loads it through Client.load -> SnapshotLoader (MT/snapshotLoader.ts:36-228),
// then the tail ops are generated against (and applied to) the loaded replica.
const loaderLogger = { ...logger, shipAssert() {}, debugAssert() {} };

function treeChunks(tree) {
    // path -> contents of the merge-tree blobs (a SharedString snapshot nests them under
    // "content"; SnapshotV1.emit puts them at the top)
    const out = {};
    const walk = (t) => {
        for (const e of t.entries) {
            if (e.type === "Blob") { out[e.path] = e.value.contents; }
        }
    };
    const content = tree.entries.find((e) => e.type === "Tree" && e.path === "content");
    walk(content ? content.value : tree);
    return out;
}

// `aliased`: loadBody inserted a segment that was already in the tree (its batch of plain
// segments is never emptied, MT/snapshotLoader.ts:207-227) -- observed on the reference's
// own insertSegments during the load (MT_DOC_ALIASED)
async function loadClient(tree, options, probe) {
    const c = new Client(segmentFromSpec, logger, options || {});
    const runtime = { logger: loaderLogger, clientId: "loader", options: {} };
    const content = tree.entries.find((e) => e.type === "Tree" && e.path === "content");
    const storage = new MockStorage(content ? content.value : tree);
    const mt = c.mergeTree;
    const insert = mt.insertSegments;
    if (probe) {
        mt.insertSegments = function (pos, segments, ...rest) {
            if (!probe.aliased && segments.some((sg) => sg.parent !== undefined && sg.cachedLength > 0)) {
                probe.aliased = true;
            }
            return insert.call(this, pos, segments, ...rest);
        };
    }
    try {
        const { catchupOpsP } = await c.load(runtime, storage);
        const catchup = await catchupOpsP;
        return { c, catchup };
    } finally {
        if (probe) { delete mt.insertSegments; }
    }
}

function attachDeltas(c) {
    const deltas = [];
    c.mergeTreeDeltaCallback = (opArgs, dargs) => {
        const mt = c.mergeTree;
        const cw = mt.getCollabWindow();
        const rec = [opArgs.sequencedMessage ? opArgs.sequencedMessage.sequenceNumber : -1,
            dargs.operation, dargs.deltaSegments.length];
        const segs = [];
        for (const d of dargs.deltaSegments) {
            const seg = d.segment;
            const pos = seg.parent ? mt.getPosition(seg, cw.currentSeq, cw.clientId) : -1;
            segs.push(d.propertyDeltas !== undefined ? [pos, seg.cachedLength, d.propertyDeltas]
                : [pos, seg.cachedLength]);
        }
        rec.push(segs);
        deltas.push(rec);
    };
    return deltas;
}

// One generated message (the generator of genDoc) against replica c at seq t.
function genStep(rng, cfg, c, t, lastRef, cseq) {
    const W = cfg.writers;
    const k = 1 + rng.uniform(W);
    let lo = Math.max(lastRef[k], t - 1 - cfg.lag);
    if (lo < 0) { lo = 0; }
    const r = lo + rng.uniform(t - 1 - lo + 1);
    lastRef[k] = r;
    let msn = Infinity;
    for (let j = 1; j <= W; j++) { msn = Math.min(msn, lastRef[j]); }
    const shortId = c.getOrAddShortClientId(`client-${k}`);
    const len = c.mergeTree.getLength(r, shortId);
    const u = rng.next();
    let op;
    if (len === 0 || u < frac(cfg.p_insert)) {
        const pos = rng.uniform(len + 1);
        const tl = 1 + rng.uniform(cfg.text_max);
        const text = genText(rng, tl, frac(cfg.p_newline));
        let seg = text;
        if (cfg.p_insert_props > 0 && rng.next() < frac(cfg.p_insert_props)) {
            seg = { text, props: genProps(rng, cfg) };
        }
        op = { pos1: pos, seg, type: 0 };
    } else {
        const p1 = rng.uniform(len);
        let n = 1;
        while (n < 64 && rng.next() < frac(cfg.p_len_continue)) { n++; }
        const p2 = Math.min(p1 + n, len);
        if (u < frac(cfg.p_insert + cfg.p_remove)) {
            op = { pos1: p1, pos2: p2, type: 1 };
        } else {
            op = { pos1: p1, pos2: p2, props: genProps(rng, cfg), type: 2 };
        }
    }
    return [k, t, r, msn, op, ++cseq[k]];
}

async function snapDoc(cfg, doc) {
    const rng = new Rng(cfg.seed >>> 0, doc);
    const seedText = genText(rng, cfg.seed_len, 0);
    const opts = { mergeTreeSnapshotChunkSize: cfg.chunk };
    const c = new Client(segmentFromSpec, logger, opts);
    if (seedText.length > 0) { c.insertSegmentLocal(0, TextSegment.make(seedText)); }
    c.startOrUpdateCollaboration("observer");
    const W = cfg.writers;
    const lastRef = new Array(W + 1).fill(0);
    const cseq = new Array(W + 1).fill(0);
    const msgs = [];
    for (let t = 1; t <= cfg.ops; t++) {
        const [k, tt, r, msn, op, cs] = genStep(rng, cfg, c, t, lastRef, cseq);
        msgs.push([k, tt, r, msn, op]);
        c.applyMsg(JSON.parse(JSON.stringify(makeMsg(k, tt, r, msn, cs, op))));
    }
    let t0 = cfg.ops;
    if (cfg.settle === true || (cfg.settle === "alternate" && doc % 2 === 0)) {
        // every writer caught up: a non-op message moves minSeq to the current seq, so the
        // summary holds no merge info (MT/snapshotV1.ts:196-215)
        t0 += 1;
        for (let j = 1; j <= W; j++) { lastRef[j] = t0; }
        const m = makeMsg(1, t0, t0 - 1, t0, ++cseq[1], null);
        m.type = "noop";
        msgs.push([1, t0, t0 - 1, t0, null, "noop"]);
        c.applyMsg(m);
    }
    const snap = new SnapshotV1(c.mergeTree, logger);
    snap.extractSync();
    const tree = snap.emit();
    const chunks = treeChunks(tree);
    const rec = { doc, seed_text: seedText, msgs, chunks };
    let loaded;
    const probe = { aliased: false };
    try {
        loaded = await loadClient(tree, {}, probe);
    } catch (e) {
        rec.error = String(e.message || e).split(":")[0];
        if (probe.aliased) { rec.aliased = true; }
        return rec;
    }
    if (probe.aliased) { rec.aliased = true; }
    const c2 = loaded.c;
    rec.observer = c2.getShortClientId("loader");
    rec.load_out = collectOutputs(c2, []);
    const deltas = attachDeltas(c2);
    const tail = [];
    for (let t = t0 + 1; t <= t0 + cfg.tail; t++) {
        const [k, tt, r, msn, op, cs] = genStep(rng, cfg, c2, t, lastRef, cseq);
        tail.push([k, tt, r, msn, op]);
        try {
            c2.applyMsg(JSON.parse(JSON.stringify(makeMsg(k, tt, r, msn, cs, op))));
        } catch (e) {
            rec.tail = tail;
            rec.error = String(e.message || e).split(":")[0];
            if (process.env.SNAP_DEBUG) { console.error(e.stack); }
            return rec;
        }
    }
    rec.tail = tail;
    rec.out = collectOutputs(c2, deltas);
    return rec;
}

// A snapshot file of the reference's own tests (SEQ/test/snapshots/*/*.json: an ITree of a
// SharedString) loaded the same way, then a generated tail.
async function loadFileDoc(path, cfg, doc) {
    const tree = JSON.parse(fs.readFileSync(path, "utf8"));
    const chunks = treeChunks(tree);
    const rec = { doc, file: path.split("/").slice(-2).join("/"), chunks };
    const probe = { aliased: false };
    const { c, catchup } = await loadClient(tree, {}, probe);
    if (probe.aliased) { rec.aliased = true; }
    rec.catchup = catchup.length;
    rec.observer = c.getShortClientId("loader");
    rec.load_out = collectOutputs(c, []);
    const deltas = attachDeltas(c);
    const rng = new Rng(cfg.seed >>> 0, doc);
    const base = c.getCurrentSeq();
    const W = cfg.writers;
    const lastRef = new Array(W + 1).fill(base);
    const cseq = new Array(W + 1).fill(0);
    const tail = [];
    for (let t = base + 1; t <= base + cfg.tail; t++) {
        const [k, tt, r, msn, op, cs] = genStep(rng, cfg, c, t, lastRef, cseq);
        tail.push([k, tt, r, msn, op]);
        c.applyMsg(JSON.parse(JSON.stringify(makeMsg(k, tt, r, msn, cs, op))));
    }
    rec.tail = tail;
    rec.out = collectOutputs(c, deltas);
    return rec;
}

// ---------------------------------------------------------------- conflict farm (config C1)
// The reference's own randomized convergence farm (MTT/client.conflictFarm.spec.ts with its
// defaultOptions and seeds), run unchanged; client 0 only applies remote ops (the observer
// baseline, MTT/mergeTreeOperationRunner.ts:107-109).  Every message it receives -- and its
// direct updateMinSeq(seq) calls between runner passes, recorded as non-op messages -- is
// the op log; its final state is the expected output.
async function farmDoc(minLength, maxClients, doc) {
    const opts = {
        minLength: { min: minLength, max: minLength }, clients: { min: 1, max: maxClients },
        opsPerRoundRange: { min: 1, max: 128 }, rounds: 8,
        operations: [removeRange, annotateRange, insertAtRefPos], growthFunc: (x) => x * 2,
    };
    const clientNames = generateClientNames();
    const mt = random.engines.mt19937();
    mt.seedWithArray([0xDEADBEEF, 0xFEEDBED, minLength]);
    const clients = [new TestClient({ blockUpdateMarkers: true })];
    clients.forEach((c, i) => c.startOrUpdateCollaboration(clientNames[i]));
    const obs = clients[0];
    const msgs = [];
    const apply = obs.applyMsg.bind(obs);
    obs.applyMsg = (m) => {
        msgs.push([m.clientId, m.sequenceNumber, m.referenceSequenceNumber, m.minimumSequenceNumber,
            JSON.parse(JSON.stringify(m.contents)), m.type]);
        return apply(m);
    };
    const deltas = attachDeltas(obs);
    let seq = 0;
    while (clients.length < opts.clients.max) {
        clients.forEach((c) => c.updateMinSeq(seq));
        msgs.push(["A", seq, seq, seq, null, "noop"]);
        const target = Math.max(opts.clients.min, opts.growthFunc(clients.length));
        for (let cc = clients.length; cc < target; cc++) {
            clients.push(await TestClient.createFromClientSnapshot(clients[0], clientNames[cc]));
        }
        seq = runMergeTreeOperationRunner(mt, seq, clients, minLength, opts);
    }
    return { doc, minLength, seed_text: "", msgs, observer_name: clientNames[0], out: collectOutputs(obs, deltas) };
}

// ---------------------------------------------------------------- live client (SURVEY §8f #4)
// A participant Client ("local", short id 0) with its own unsequenced ops, W remote writers
// and a sequencer: every step either applies a local op (insertSegmentLocal /
// removeRangeLocal / annotateRangeLocal, MT/client.ts:164-211), sequences the oldest
// submitted local op (its echo acks it: applyMsg -> ackPendingSegment, :589-626, 810-812),
// sequences a remote writer's op (generated in its view (refSeq, client) of this replica,
// as genStep), or reconnects: the unsequenced ops are dropped, the client takes a new long id
// (startOrUpdateCollaboration, :1065-1071) and regeneratePendingOp (:855-893) rebuilds each
// pending op, in order, for resubmission.  Events: ["L", op] | ["M", clientId, seq, refSeq,
// msn, op] | ["R", newClientId, [regenerated op per pending op]].  msn = the minimum of
// the writers' last refSeqs and the refSeqs of the local client's unsequenced ops (or the
// refSeq of its last sequenced op).
function pendingGroups(c) {
    const all = [];
    c.mergeTree.pendingSegments.walk((g) => all.push(g));
    return all;
}
function genLocalOp(rng, cfg, len) {
    const u = rng.next();
    if (len === 0 || u < frac(cfg.p_insert)) {
        const pos = rng.uniform(len + 1);
        const text = genText(rng, 1 + rng.uniform(cfg.text_max), frac(cfg.p_newline));
        const props = (cfg.p_insert_props > 0 && rng.next() < frac(cfg.p_insert_props)) ? genProps(rng, cfg) : undefined;
        const marker = cfg.p_marker > 0 && rng.next() < frac(cfg.p_marker) ? 1 + rng.uniform(3) : 0;
        return { kind: 0, pos, text, props, marker };
    }
    const p1 = rng.uniform(len);
    let n = 1;
    while (n < 64 && rng.next() < frac(cfg.p_len_continue)) { n++; }
    const p2 = Math.min(p1 + n, len);
    if (u < frac(cfg.p_insert + cfg.p_remove)) { return { kind: 1, p1, p2 }; }
    const props = genProps(rng, cfg);
    const rw = cfg.p_rewrite > 0 && rng.next() < frac(cfg.p_rewrite);
    return { kind: 2, p1, p2, props, comb: rw ? { name: "rewrite" } : undefined };
}
function liveDoc(cfg, doc) {
    const rng = new Rng(cfg.seed >>> 0, doc);
    const seedText = genText(rng, cfg.seed_len, 0);
    const c = new Client(segmentFromSpec, logger);
    if (seedText.length > 0) { c.insertSegmentLocal(0, TextSegment.make(seedText)); }
    let localId = "local-0";
    c.startOrUpdateCollaboration(localId);
    const deltas = attachDeltas(c);
    const W = cfg.writers;
    const lastRef = new Array(W + 1).fill(0);
    const cseq = new Array(W + 1).fill(0);
    let lcseq = 0;
    let localRef = 0;          // refSeq of the local client's last sequenced op
    let t = 0;
    let prevMsn = 0;
    const unseq = [];          // [{op, ref, sgs}]
    const events = [];
    const nextMsn = () => {
        let m = localRef;
        for (const u of unseq) { m = Math.min(m, u.ref); }
        for (let j = 1; j <= W; j++) { m = Math.min(m, lastRef[j]); }
        prevMsn = Math.max(prevMsn, m);
        return prevMsn;
    };
    const submit = (op, before) => {
        const sgs = pendingGroups(c).slice(before);
        unseq.push({ op, ref: c.getCurrentSeq(), sgs });
    };
    const trace = [];          // cfg.trace (debugging): the local text after every event
    let maxDepth = 0;          // deepest segment-group queue of any segment (cfg.track_depth)
    for (let step = 0; step < cfg.steps; step++) {
        if (cfg.track_depth) {
            c.mergeTree.walkAllSegments(c.mergeTree.root, (sg) => {
                maxDepth = Math.max(maxDepth, sg.segmentGroups.size);
                return true;
            });
        }
        if (cfg.trace && trace.length < events.length) {
            const t = c.createTextHelper().getText(c.getCurrentSeq(), 0);
            if (cfg.trace === 2) {       // + the leaf table: [len, seq, removedSeq, #groups] per segment, leaf blocks
                const segs = [];
                c.mergeTree.walkAllSegments(c.mergeTree.root, (sg) => {
                    segs.push(sg.cachedLength, sg.seq, sg.removedSeq === undefined ? null : sg.removedSeq,
                        sg.segmentGroups.size);
                    return true;
                });
                const leaves = [];
                const walk = (b) => {
                    if (b.childCount === 0 || b.children[0].isLeaf()) { leaves.push(b.childCount); return; }
                    for (let i = 0; i < b.childCount; i++) { walk(b.children[i]); }
                };
                walk(c.mergeTree.root);
                // zamboni heap (array order): [maxSeq, leaf index of the segment or -1]; needsScour per leaf block
                const idx = new Map();
                let n = 0;
                c.mergeTree.walkAllSegments(c.mergeTree.root, (sg) => { idx.set(sg, n++); return true; });
                const heap = c.mergeTree.segmentsToScour.L.slice(1).map((e) =>
                    [e.maxSeq, e.segment.parent && idx.has(e.segment) ? idx.get(e.segment) : -1]);
                const flags = [];
                const walkf = (b) => {
                    if (b.childCount === 0 || b.children[0].isLeaf()) {
                        flags.push(b.needsScour === undefined ? -1 : (b.needsScour ? 1 : 0));
                        return;
                    }
                    for (let i = 0; i < b.childCount; i++) { walkf(b.children[i]); }
                };
                walkf(c.mergeTree.root);
                trace.push([t, segs, leaves, heap, flags]);
            } else {
                trace.push(t);
            }
        }
        const u = rng.next();
        if (u < frac(cfg.p_local)) {
            const len = c.getLength();
            const g = genLocalOp(rng, cfg, len);
            const before = pendingGroups(c).length;
            let op;
            if (g.kind === 0) {
                const seg = g.marker ? Marker.make(g.marker, g.props) : TextSegment.make(g.text, g.props);
                op = c.insertSegmentLocal(g.pos, seg);
            } else if (g.kind === 1) {
                op = c.removeRangeLocal(g.p1, g.p2);
            } else {
                op = c.annotateRangeLocal(g.p1, g.p2, g.props, g.comb);
            }
            if (!op) { continue; }
            op = JSON.parse(JSON.stringify(op));
            events.push(["L", op]);
            submit(op, before);
        } else if (u < frac(cfg.p_local + cfg.p_reconnect)) {
            if (unseq.length === 0) { continue; }
            localId = `local-${events.length}`;
            c.startOrUpdateCollaboration(localId);
            const old = unseq.splice(0, unseq.length);
            const regen = [];
            for (const e of old) {
                const before = pendingGroups(c).length;
                const sg = e.op.type === 3 ? e.sgs : e.sgs[0];
                const nop = JSON.parse(JSON.stringify(c.regeneratePendingOp(e.op, sg)));
                regen.push(nop);
                submit(nop, before - (e.op.type === 3 ? e.op.ops.length : 1));
            }
            events.push(["R", localId, regen]);
        } else if (unseq.length > 0 && rng.next() < frac(cfg.p_ack)) {
            const e = unseq.shift();
            t++;
            localRef = e.ref;
            const msg = makeMsg(0, t, e.ref, nextMsn(), ++lcseq, e.op);
            msg.clientId = localId;
            events.push(["M", localId, t, e.ref, msg.minimumSequenceNumber, e.op]);
            c.applyMsg(JSON.parse(JSON.stringify(msg)));
        } else {
            t++;
            const k = 1 + rng.uniform(W);
            let lo = Math.max(lastRef[k], t - 1 - cfg.lag, prevMsn);
            const r = lo + rng.uniform(t - 1 - lo + 1);
            lastRef[k] = r;
            const msn = nextMsn();
            const shortId = c.getOrAddShortClientId(`client-${k}`);
            const len = c.mergeTree.getLength(r, shortId);
            const g = genLocalOp(rng, cfg, len);
            let op;
            if (g.kind === 0 && g.marker) {
                op = { pos1: g.pos, seg: g.props ? { marker: { refType: g.marker }, props: g.props }
                    : { marker: { refType: g.marker } }, type: 0 };
            } else if (g.kind === 0) {
                op = { pos1: g.pos, seg: g.props ? { text: g.text, props: g.props } : g.text, type: 0 };
            } else if (g.kind === 1) {
                op = { pos1: g.p1, pos2: g.p2, type: 1 };
            } else {
                op = { pos1: g.p1, pos2: g.p2, props: g.props, type: 2 };
                if (g.comb) { op.combiningOp = g.comb; }
            }
            const msg = makeMsg(k, t, r, msn, ++cseq[k], op);
            events.push(["M", `client-${k}`, t, r, msn, op]);
            c.applyMsg(JSON.parse(JSON.stringify(msg)));
        }
    }
    const out = collectOutputs(c, deltas);
    if (cfg.trace) { out.trace = trace; }
    out.pending = pendingGroups(c).length;
    out.localSeq = c.mergeTree.getCollabWindow().localSeq;
    if (cfg.track_depth) { out.maxGroupDepth = maxDepth; }
    // drain: the server sequences every op still unsequenced (their echoes ack them)
    const drain = [];
    while (unseq.length > 0) {
        const e = unseq.shift();
        t++;
        localRef = e.ref;
        const msg = makeMsg(0, t, e.ref, nextMsn(), ++lcseq, e.op);
        msg.clientId = localId;
        drain.push(["M", localId, t, e.ref, msg.minimumSequenceNumber, e.op]);
        c.applyMsg(JSON.parse(JSON.stringify(msg)));
    }
    const drained = collectOutputs(c, []);
    drained.pending = pendingGroups(c).length;
    delete drained.deltas;
    delete drained.tree;
    return { doc, seed_text: seedText, events, out, drain, drained };
}

const [mode, ...rest] = process.argv.slice(2);
async function main() {
    if (mode === "gen") {
        const cfg = JSON.parse(fs.readFileSync(rest[0], "utf8"));
        const d0 = parseInt(rest[1], 10), d1 = parseInt(rest[2], 10);
        const docs = [];
        for (let d = d0; d < d1; d++) { docs.push(cfg.ext ? genDocExt(cfg, d) : genDoc(cfg, d)); }
        fs.writeFileSync(rest[3], JSON.stringify({ config: cfg, docs }, cfg.p_combine ? jsReplacer : undefined));
    } else if (mode === "live") {
        // live <config.json> <doc_begin> <doc_end> <out.json>
        const cfg = JSON.parse(fs.readFileSync(rest[0], "utf8"));
        const d0 = parseInt(rest[1], 10), d1 = parseInt(rest[2], 10);
        const docs = [];
        for (let d = d0; d < d1; d++) { docs.push(liveDoc(cfg, d)); }
        fs.writeFileSync(rest[3], JSON.stringify({ config: cfg, docs }));
    } else if (mode === "livetime") {
        // livetime <live.json(.gz)> <out.json>: the reference participant Client replaying the
        // live streams' local ops and sequenced messages (no reconnects), one thread, timed
        const raw = fs.readFileSync(rest[0]);
        const fx = JSON.parse((rest[0].endsWith(".gz") ? (await import("zlib")).gunzipSync(raw) : raw).toString());
        let ns = 0n, events = 0;
        for (const d of fx.docs) {
            const c = new Client(segmentFromSpec, logger);
            if (d.seed_text.length > 0) { c.insertSegmentLocal(0, TextSegment.make(d.seed_text)); }
            c.startOrUpdateCollaboration("local-0");
            const evs = d.events.map((ev) => (ev[0] === "L" ? ev : ["M", makeMsg(0, ev[2], ev[3], ev[4], 0, ev[5])]));
            evs.forEach((ev, i) => { if (ev[0] === "M") { ev[1].clientId = d.events[i][1]; } });
            const t0 = process.hrtime.bigint();
            for (const ev of evs) {
                if (ev[0] === "L") {
                    const op = ev[1];
                    if (op.type === 0) { c.insertSegmentLocal(op.pos1, segmentFromSpec(op.seg)); }
                    else if (op.type === 1) { c.removeRangeLocal(op.pos1, op.pos2); }
                    else { c.annotateRangeLocal(op.pos1, op.pos2, op.props, op.combiningOp); }
                } else {
                    c.applyMsg(ev[1]);
                }
            }
            ns += process.hrtime.bigint() - t0;
            events += evs.length;
            const text = c.createTextHelper().getText(c.getCurrentSeq(), c.getClientId());
            if (text !== d.out.text) { throw new Error(`doc ${d.doc}: replay differs from the fixture`); }
        }
        const sec = Number(ns) / 1e9;
        fs.writeFileSync(rest[1], JSON.stringify({ events, seconds: sec, events_per_s: events / sec, node: process.version }));
    } else if (mode === "replay") {
        const logs = JSON.parse(fs.readFileSync(rest[0], "utf8"));
        const outs = logs.docs.map((d) => ({ doc: d.doc, out: replayDoc(d) }));
        fs.writeFileSync(rest[1], JSON.stringify({ docs: outs }));
    } else if (mode === "rich") {
        const logs = JSON.parse(fs.readFileSync(rest[0], "utf8"));
        fs.writeFileSync(rest[1], JSON.stringify({ docs: logs.docs.map((d) => replayRichDoc(d)) }, jsReplacer));
    } else if (mode === "events") {
        const logs = JSON.parse(fs.readFileSync(rest[0], "utf8"));
        fs.writeFileSync(rest[1], JSON.stringify({ docs: logs.docs.map((d) => replayEventsDoc(d)) }, jsReplacer));
    } else if (mode === "ordprobe") {
        const logs = JSON.parse(fs.readFileSync(rest[0], "utf8"));
        fs.writeFileSync(rest[1], JSON.stringify({ docs: logs.docs.map((d) => ordProbeDoc(d)) }));
    } else if (mode === "readouts") {
        const logs = JSON.parse(fs.readFileSync(rest[0], "utf8"));
        fs.writeFileSync(rest[1], JSON.stringify({ docs: logs.docs.map((d) => readoutsDoc(d)) }, jsReplacer));
    } else if (mode === "replayerr") {
        const logs = JSON.parse(fs.readFileSync(rest[0], "utf8"));
        fs.writeFileSync(rest[1], JSON.stringify({ docs: logs.docs.map((d) => replayErrDoc(d)) }));
    } else if (mode === "maint") {
        const logs = JSON.parse(fs.readFileSync(rest[0], "utf8"));
        fs.writeFileSync(rest[1], JSON.stringify(logs.docs.map((d) => maintDoc(d))));
    } else if (mode === "time") {
        // time <gen.json> <out.json> [repeats] [nocb]: the reference's Client.applyMsg replay
        // of every document's stream (messages pre-built, observer with the delta callback
        // that records positions, as replayDoc -- or with no callback at all when "nocb"),
        // one thread; the CPU-baseline calibration
        const logs = JSON.parse(fs.readFileSync(rest[0], "utf8"));
        const reps = rest[2] ? parseInt(rest[2], 10) : 1;
        const nocb = rest[3] === "nocb";
        let ns = 0n, ops = 0;
        for (let rep = 0; rep < reps; rep++) {
            for (const d of logs.docs) {
                const { c } = makeObserver(d.seed_text);
                if (nocb) { c.mergeTreeDeltaCallback = undefined; }
                const cseq = {};
                const msgs = d.msgs.map(([k, t, r, msn, op, type]) => {
                    cseq[k] = (cseq[k] || 0) + 1;
                    const m = makeMsg(k, t, r, msn, cseq[k], op);
                    if (type) { m.type = type; }
                    return m;
                });
                const t0 = process.hrtime.bigint();
                for (const m of msgs) { c.applyMsg(m); }
                ns += process.hrtime.bigint() - t0;
                ops += msgs.length;
            }
        }
        const s = Number(ns) / 1e9;
        fs.writeFileSync(rest[1], JSON.stringify({ ops, seconds: s, ops_per_s: ops / s, node: process.version, nocb }));
    } else if (mode === "snap") {
        const cfg = JSON.parse(fs.readFileSync(rest[0], "utf8"));
        const d0 = parseInt(rest[1], 10), d1 = parseInt(rest[2], 10);
        const docs = [];
        for (let d = d0; d < d1; d++) { docs.push(await snapDoc(cfg, d)); }
        fs.writeFileSync(rest[3], JSON.stringify({ config: cfg, docs }));
    } else if (mode === "farm") {
        // farm <out.json> <maxClients> <minLength>...
        const docs = [];
        const maxClients = parseInt(rest[1], 10);
        for (let i = 2; i < rest.length; i++) { docs.push(await farmDoc(parseInt(rest[i], 10), maxClients, i - 2)); }
        fs.writeFileSync(rest[0], JSON.stringify({ config: { farm: true, clients: maxClients }, docs }));
    } else if (mode === "loadfile") {
        const cfg = JSON.parse(fs.readFileSync(rest[0], "utf8"));
        const docs = [];
        for (let i = 2; i < rest.length; i++) { docs.push(await loadFileDoc(rest[i], cfg, i - 2)); }
        fs.writeFileSync(rest[1], JSON.stringify({ config: cfg, docs }));
    } else {
        console.error("usage: ref_harness.mjs gen|replay|snap|loadfile ...");
        process.exit(2);
    }
}
main().catch((e) => { console.error(e); process.exit(1); });
