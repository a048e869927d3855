"use strict";
/**
 * index.js -- Node facade of the MI355X merge-tree replay backend.
 *
 * GpuMergeTreeBatch owns N observer replicas resident on one GPU (one handle of the C ABI,
 * include/mt_replay.h, through the N-API addon js/binding.cc).  batch.client(doc) returns a
 * Client-shaped view of one document with the surface SharedSegmentSequence uses on the
 * reference Client (merge-tree/src/client.ts:43; sequence/src/sequence.ts:131-142,
 * 473-600): applyMsg, startOrUpdateCollaboration, getLength, getText (as
 * createTextHelper().getText), getPropertiesAtPosition, getCurrentSeq and the
 * mergeTreeDeltaCallback property.
 *
 * applyMsg only queues the message (the GPU applies whole batches); any read, or an
 * explicit batch.flush(), applies everything queued for every document in one launch.
 * Per-document failures are raised from the next call on that document with the
 * reference's messages and error types (client.ts:462-465, 824-826; mergeTree.ts:2244).
 * There is no CPU fallback: without the addon or a GPU the constructor throws.
 */
const assert = require("assert");
const path = require("path");
const { BatchEncoder, Interner, VAL_NULL } = require("./encode");
const { treeChunks } = require("./snapshot");

const native = require(path.join(__dirname, "mtreplay.node"));

const DOC_STATUS = {
    1: () => new Error("MergeTree insert failed"),
    2: () => new assert.AssertionError({ message: "Incoming remote op sequence# <= local collabWindow's currentSequence#" }),
    3: () => new assert.AssertionError({ message: "Incoming remote op minSequence# < local collabWindow's minSequence#" }),
    4: () => new Error("merge-tree replay: a per-document capacity was exceeded"),
    5: () => new Error("merge-tree replay: combiningOp result not modelled"),
    6: () => new Error("merge-tree replay: internal error"),
    // updateSeqNumbers (client.ts:824-826) and setMinSeq (mergeTree.ts:1755, no message)
    7: () => new assert.AssertionError({ message: "Incoming op sequence# < local collabWindow's currentSequence#" }),
    8: () => new assert.AssertionError({ message: "Incoming op sequence# < minSequence#" }),
    // (Node's message for a bare assert(): what the reference throws on this runtime)
    9: () => new assert.AssertionError({ message: "false == true" }),
};

/** JS own-key order: integer-like keys ascending first, then insertion order. */
function jsKeyOrder(pairs) {
    const isIndex = (k) => /^(0|[1-9][0-9]*)$/.test(k) && Number(k) < 4294967295;
    const ints = pairs.filter(([k]) => isIndex(k)).sort((a, b) => Number(a[0]) - Number(b[0]));
    return ints.concat(pairs.filter(([k]) => !isIndex(k)));
}

/**
 * SnapshotLoader's host half for many summaries (snapshotLoader.ts:36-228) in native code
 * (include/mt_snapshot.h through the addon): the mt_load_snapshots arrays with property ids
 * mapped into `interner` (first-seen order), the short client maps and the catch-up
 * messages per document.  snapshot.js (decodeChunks + SnapshotEncoder) is the same in JS.
 */
function decodeSummaries(summaries, interner, threads = 8) {
    const paths = [], blobs = [], off = [0];
    for (const s of summaries) {
        const ch = s.entries ? treeChunks(s) : s;
        for (const k of Object.keys(ch)) { paths.push(k); blobs.push(ch[k]); }
        off.push(paths.length);
    }
    const a = native.decodeSummaries(paths, blobs, off, threads);
    const km = a.keys.map((k) => interner.key(k));
    const vm = a.vals.map((v) => (interner.val(JSON.parse(v)) & 0x3FFFFFFF) >>> 0);
    for (const v of vm) { interner.noteUnkeyed(v); }   // held by some key of a loaded summary
    const dv = new DataView(a.segs.buffer, a.segs.byteOffset, a.segs.byteLength);
    const p = a.props;
    for (let r = 0; r < a.segs.byteLength; r += 32) {
        const o = dv.getUint32(r + 16, true);
        if (o === 0xFFFFFFFF) { continue; }
        for (let j = 0, n = p[o]; j < n; j++) {
            const k = o + 1 + 2 * j;
            p[k] = km[p[k]];
            const v = p[k + 1];
            if (v !== VAL_NULL) { p[k + 1] = (vm[(v & 0x3FFFFFFF) >>> 0] | (v & 0x80000000)) >>> 0; }
        }
    }
    a.clients = a.clients.map((c) => new Map(JSON.parse(c).map((id, i) => [id, i + 1])));
    a.catchup = Array.from(a.catchup, (b) => (b < 0n ? [] : JSON.parse(blobs[Number(b)])));
    return a;
}

class GpuMergeTreeBatch {
    /**
     * @param {number} nDocs  documents (observer replicas) on this GPU
     * @param {object} options  mt_options: device, segCapacity, textCapacity, deltaLogCapacity, ...
     */
    constructor(nDocs, options = {}) {
        // the facade reads the rich delta log: callback segments carry their state, and the
        // maintenance events are records of their own (mt_options.delta_log_mode 1)
        if (options.deltaLogCapacity && options.deltaLogMode === undefined) {
            options = Object.assign({}, options, { deltaLogMode: 1 });
        }
        this.rich = !!options.deltaLogCapacity && options.deltaLogMode === 1;
        // live-client batches (liveClient: 1) back participant Clients: local ops, acks and
        // reconnect regeneration (SURVEY §8f #4); they replay from HBM (ldsSegCapacity -1)
        this.live = !!options.liveClient;
        if (this.live) { options = Object.assign({ ldsSegCapacity: -1 }, options); }
        this.h = native.create(nDocs, options);
        this.nDocs = nDocs;
        this.interner = new Interner();
        this.clients = Array.from({ length: nDocs }, () => new Map());
        this.pending = Array.from({ length: nDocs }, () => []);
        this.queued = 0;
        this.failed = new Int32Array(nDocs);
        this.views = new Map();
        this.logPos = new Int32Array(nDocs);
        this.wantsDeltas = !!options.deltaLogCapacity;
    }

    /** Initial contents of every document (Client.insertSegmentLocal before collaboration). */
    loadInitialText(texts) {
        assert(texts.length === this.nDocs);
        let total = 0;
        for (const t of texts) { total += t.length; }
        const seed = new Uint16Array(Math.max(total, 1));
        const off = new BigInt64Array(this.nDocs + 1);
        let k = 0;
        texts.forEach((t, d) => {
            off[d] = BigInt(k);
            for (let i = 0; i < t.length; i++) { seed[k++] = t.charCodeAt(i); }
        });
        off[this.nDocs] = BigInt(k);
        native.loadInitialText(this.h, off, seed);
        this.logPos.fill(0);
    }

    /**
     * Client.load for every document (client.ts:938-946 -> SnapshotLoader.initialize,
     * snapshotLoader.ts:36-228): summaries[d] is a summary ITree (a SharedString's, or
     * SnapshotV1.emit's) or its {path: contents} blobs.  Replaces every document's state;
     * legacy catch-up messages are queued like SharedSegmentSequence.loadCore applies them.
     * A summary the reference cannot load fails that document the same way.
     */
    loadSnapshots(summaries, threads = 8) {
        assert(summaries.length === this.nDocs);
        this.flush();
        const a = decodeSummaries(summaries, this.interner, threads);
        native.loadSnapshots(this.h, a.docSegOff, a.nHeader, a.segs, a.text, a.props, a.minSeq, a.curSeq);
        this.failed.fill(0);
        this.logPos.fill(0);
        const st = native.status(this.h);
        for (let d = 0; d < this.nDocs; d++) {
            this.clients[d] = a.clients[d];
            if (st[d] !== 0) { this.failed[d] = st[d]; }
            const v = this.views.get(d);
            if (v) { v.currentSeq = a.curSeq[d]; }
            for (const m of a.catchup[d]) { this.pending[d].push(m); this.queued++; }
        }
    }

    client(doc) {
        let v = this.views.get(doc);
        if (!v) {
            v = new GpuClient(this, doc);
            this.views.set(doc, v);
        }
        return v;
    }

    /** Applies every queued message of every document (one mt_apply_ops). */
    flush() {
        if (this.queued === 0) { return; }
        const enc = new BatchEncoder(this.interner);
        this.applied = this.pending;   // the messages of this flush, for the callbacks' opArgs
        for (let d = 0; d < this.nDocs; d++) {
            enc.addDoc(this.pending[d], this.clients[d]);
        }
        this.pending = Array.from({ length: this.nDocs }, () => []);
        this.queued = 0;
        const a = enc.arrays();
        native.applyOps(this.h, a.docOff, a.ops, a.text, a.props);
        const st = native.status(this.h);
        for (let d = 0; d < this.nDocs; d++) {
            if (st[d] !== 0 && this.failed[d] === 0) { this.failed[d] = st[d]; }
        }
        if (this.wantsDeltas) {
            // every view drains its records, then the device logs restart empty: a long-lived
            // batch never runs out of log capacity (a single flush that overflows it throws)
            try {
                for (const v of this.views.values()) { v._emitDeltas(); }
            } finally {
                native.deltaLogReset(this.h);
                this.logPos.fill(0);
            }
        }
    }

    status() { this.flush(); return native.status(this.h); }

    /** mt_checksum per document: {length, nSegments, textHash, propsHash, deltaHash}. */
    checksums() {
        this.flush();
        const ab = native.checksums(this.h);
        const dv = new DataView(ab);
        const out = [];
        for (let d = 0; d < this.nDocs; d++) {
            const o = d * 32;
            out.push({
                length: dv.getUint32(o, true), nSegments: dv.getUint32(o + 4, true),
                textHash: dv.getBigUint64(o + 8, true), propsHash: dv.getBigUint64(o + 16, true),
                deltaHash: dv.getBigUint64(o + 24, true),
            });
        }
        return out;
    }

    lastKernelMs() { return native.lastKernelMs(this.h); }

    dispose() { native.destroy(this.h); }
}

/** Client-shaped view of one document (the observer replica). */
class GpuClient {
    constructor(batch, doc) {
        this.batch = batch;
        this.doc = doc;
        this.longClientId = undefined;
        this.currentSeq = 0;
        this.mergeTreeDeltaCallback = undefined;
        this.mergeTreeMaintenanceCallback = undefined;
    }

    _check() {
        const code = this.batch.failed[this.doc];
        if (code) { throw DOC_STATUS[code] ? DOC_STATUS[code]() : new Error(`document status ${code}`); }
    }

    _sync() {
        this.batch.flush();
        this._check();
    }

    /**
     * Client.startOrUpdateCollaboration (client.ts:1053-1073): the observer is short id 0.
     * The first call with an id starts the collab window at (minSeq, currentSeq)
     * (MergeTree.startCollaboration, mergeTree.ts:1287-1294); later calls only rename it.
     */
    startOrUpdateCollaboration(longClientId, minSeq = 0, currentSeq = 0) {
        if (longClientId === undefined) { return; }
        if (this.batch.live) {
            // the local client is short id 0 under every long id it has had (client.ts:1065-1071)
            this.batch.clients[this.doc].set(longClientId, 0);
        }
        if (this.longClientId === undefined) {
            this.longClientId = longClientId;
            if (minSeq !== 0 || currentSeq !== 0) {
                this.batch.flush();
                const ms = new Int32Array(this.batch.nDocs).fill(-1);
                const cs = new Int32Array(this.batch.nDocs);
                ms[this.doc] = minSeq;
                cs[this.doc] = currentSeq;
                native.startCollaboration(this.batch.h, ms, cs);
                this.currentSeq = currentSeq;
            }
        } else {
            this.longClientId = longClientId;
        }
    }

    /** Client.applyMsg (client.ts:797-819); applied on the GPU at the next flush. */
    applyMsg(msg) {
        this._check();
        if (msg.clientId === this.longClientId && msg.clientId !== undefined) {
            if (!this.batch.live) {
                throw new Error("merge-tree replay: the observer replica has no local ops to acknowledge");
            }
            // the echo of one of our own ops: ackPendingSegment (client.ts:589-626, 810-812)
            this.batch.pending[this.doc].push({ __ack: msg });
        } else {
            this.batch.pending[this.doc].push(msg);
        }
        this.batch.queued++;
        this.currentSeq = msg.sequenceNumber;
    }

    // ------------------------------------------------------------ live client (liveClient: 1)
    /** getValidOpRange for a local op (client.ts:486-548). */
    _validRange(start, end, insert) {
        const length = this.getLength();
        if (start === undefined || start < 0 || start > length || (start === length && !insert)) { return false; }
        if (!insert || end !== undefined) {
            if (end === undefined || end <= start) { return false; }
        }
        return true;
    }

    _local(op) {
        if (!this.batch.live) { throw new Error("merge-tree replay: local ops need a batch created with liveClient: 1"); }
        this.batch.pending[this.doc].push({ __local: op });
        this.batch.queued++;
        return op;
    }

    /** Client.insertSegmentLocal (client.ts:202-211); segment: an ISegment or its JSON. */
    insertSegmentLocal(pos, segment) {
        const spec = segment && typeof segment.toJSONObject === "function" ? segment.toJSONObject() : segment;
        const len = typeof spec === "string" ? spec.length : (spec && spec.text !== undefined ? spec.text.length : 1);
        if (len <= 0 || !this._validRange(pos, undefined, true)) { return undefined; }
        return this._local({ pos1: pos, seg: spec, type: 0 });
    }

    /** Client.removeRangeLocal (client.ts:189-196). */
    removeRangeLocal(start, end) {
        if (!this._validRange(start, end, false)) { return undefined; }
        return this._local({ pos1: start, pos2: end, type: 1 });
    }

    /** Client.annotateRangeLocal (client.ts:164-179). */
    annotateRangeLocal(start, end, props, combiningOp) {
        if (!this._validRange(start, end, false)) { return undefined; }
        const op = { pos1: start, pos2: end, props, type: 2 };
        if (combiningOp !== undefined) { op.combiningOp = combiningOp; }
        return this._local(op);
    }

    /** Client.localTransaction (client.ts:961-981): every member applied as its own local op. */
    localTransaction(groupOp) {
        for (const op of groupOp.ops) {
            if (op.type === 0) { this.insertSegmentLocal(op.pos1, op.seg); }
            else if (op.type === 1) { this.removeRangeLocal(op.pos1, op.pos2); }
            else if (op.type === 2) { this.annotateRangeLocal(op.pos1, op.pos2, op.props, op.combiningOp); }
        }
    }

    /**
     * Client.regeneratePendingOp (client.ts:855-893) for the oldest pending op(s): resetOp is
     * the op as it was submitted (a GROUP is rebuilt member by member); segmentGroup is not
     * needed (the device holds the groups).  Positions come from findReconnectionPostition
     * (:675-707) on the GPU (mt_regenerate_pending).
     */
    regeneratePendingOp(resetOp) {
        this._sync();
        const members = resetOp.type === 3 ? resetOp.ops : [resetOp];
        const out = [];
        for (const m of members) {
            const r = native.regeneratePending(this.batch.h, this.doc);
            if (r === null) { throw new Error("regeneratePendingOp: no pending segment group"); }
            for (let i = 0; i < r.recs.length; i += 8) {
                const kind = r.recs[i], pos1 = r.recs[i + 1], pos2 = r.recs[i + 2];
                if (kind === 0) {
                    const toff = r.recs[i + 4] >>> 0, tlen = r.recs[i + 5] >>> 0, poff = r.recs[i + 6] >>> 0;
                    const flags = r.recs[i + 7];
                    let props;
                    if (poff !== 0xFFFFFFFF) {
                        const pairs = [];
                        for (let j = 0; j < r.props[poff]; j++) {
                            pairs.push([this.batch.interner.keyName(r.props[poff + 1 + 2 * j]),
                                this.batch.interner.value(r.props[poff + 2 + 2 * j])]);
                        }
                        props = {};
                        for (const [k, v] of jsKeyOrder(pairs)) { props[k] = v; }
                    }
                    let seg;
                    if (flags & 2) {
                        seg = { marker: { refType: toff } };
                        if (props) { seg.props = props; }
                    } else {
                        const text = String.fromCharCode.apply(null, Array.from(r.text.subarray(toff, toff + tlen)));
                        seg = props ? { text, props } : text;
                    }
                    out.push({ pos1, seg, type: 0 });
                } else if (kind === 1) {
                    out.push({ pos1, pos2, type: 1 });
                } else {
                    const op = { pos1, pos2, props: m.props, type: 2 };
                    if (m.combiningOp !== undefined) { op.combiningOp = m.combiningOp; }
                    out.push(op);
                }
            }
        }
        return out.length === 1 ? out[0] : { ops: out, type: 3 };
    }

    getCurrentSeq() { return this.currentSeq; }

    getLength() { this._sync(); return native.getLength(this.batch.h, this.doc); }

    getText() { this._sync(); return native.getText(this.batch.h, this.doc); }

    createTextHelper() { return { getText: () => this.getText() }; }

    /** Client.getPropertiesAtPosition (client.ts:1011-1025). */
    getPropertiesAtPosition(pos) {
        this._sync();
        const { runs, records } = native.getPropRuns(this.batch.h, this.doc);
        for (let i = 0; i < runs.length; i += 3) {
            const start = runs[i], len = runs[i + 1], rec = runs[i + 2];
            if (pos >= start && pos < start + len) {
                if (rec === 0xFFFFFFFF) { return undefined; }
                const n = records[rec];
                const pairs = [];
                for (let j = 0; j < n; j++) {
                    pairs.push([this.batch.interner.keyName(records[rec + 1 + 2 * j]),
                        this.batch.interner.value(records[rec + 2 + 2 * j])]);
                }
                const props = {};
                for (const [k, v] of jsKeyOrder(pairs)) { props[k] = v; }
                return props;
            }
        }
        return undefined;
    }

    /**
     * mergeTreeMaintenanceCallback events of this document so far (MergeTreeMaintenanceType
     * SPLIT / APPEND / UNLINK, mergeTreeDeltaCallback.ts:15-35), as counts; needs a batch
     * created with deltaLogCapacity > 0.
     */
    getMaintenanceCounts() {
        this._sync();
        const m = native.maintenanceCounts(this.batch.h);
        return { split: m[3 * this.doc], append: m[3 * this.doc + 1], unlink: m[3 * this.doc + 2] };
    }

    /** A segment's state at an event (rich log), as the ISegment fields listeners read. */
    _segment(log, i, len) {
        const flags = log[i++];
        let seg;
        if (flags & 1) {
            seg = { type: "Marker", refType: log[i++], cachedLength: len };
        } else {
            const words = (len + 1) >> 1;
            const units = new Array(len);
            for (let u = 0; u < len; u++) { const w = log[i + (u >> 1)]; units[u] = (u & 1) ? (w >>> 16) : (w & 0xFFFF); }
            i += words;
            seg = { type: "TextSegment", text: String.fromCharCode(...units), cachedLength: len };
        }
        const np = log[i++];
        if (np >= 0) {
            const pairs = [];
            for (let j = 0; j < np; j++) {
                pairs.push([this.batch.interner.keyName(log[i]), this.batch.interner.value(log[i + 1] >>> 0)]);
                i += 2;
            }
            seg.properties = {};
            for (const [k, v] of jsKeyOrder(pairs)) { seg.properties[k] = v; }
        }
        return [seg, i];
    }

    /**
     * Replays the device delta log of the last flush into the reference's callbacks:
     * mergeTreeDeltaCallback(opArgs, {operation, deltaSegments}) (mergeTreeDeltaCallback.ts:
     * 33-59; call sites mergeTree.ts:2014-2021, 2625-2632, 2738-2745) with opArgs {op,
     * sequencedMessage, groupOp} and deltaSegments [{segment, propertyDeltas}] -- segment =
     * the segment's state at the event (cachedLength, text or refType, properties) plus its
     * observer `position` at callback time (what SequenceDeltaEvent.ranges reads) -- and
     * mergeTreeMaintenanceCallback({operation: SPLIT -2 | APPEND -1 | UNLINK -3,
     * deltaSegments}) (mergeTree.ts:1343-1373, 2264-2269), in the reference's order.
     */
    _emitDeltas() {
        const cb = this.mergeTreeDeltaCallback, mcb = this.mergeTreeMaintenanceCallback;
        const rich = this.batch.rich;
        const log = native.getDeltaLog(this.batch.h, this.doc);
        const msgs = (this.batch.applied && this.batch.applied[this.doc]) || [];
        let mi = 0, member = 0, lastSeq = null;
        let i = this.batch.logPos[this.doc];
        while (i + 3 <= log.length) {
            const seq = log[i], kind = log[i + 1], n = log[i + 2];
            i += 3;
            const deltaSegments = [];
            for (let s = 0; s < n; s++) {
                const pos = kind >= 0 ? log[i++] : -1;
                const len = log[i++];
                let delta;
                if (kind === 2) {
                    const npd = log[i++];
                    const pd = [];
                    for (let j = 0; j < npd; j++) {
                        pd.push([this.batch.interner.keyName(log[i]), this.batch.interner.value(log[i + 1] >>> 0)]);
                        i += 2;
                    }
                    if (npd < 0) {
                        // live client: an outstanding local rewrite blocked the remote annotate
                        // (segmentPropertiesManager.ts:48-51): propertyDeltas undefined
                        delta = {};
                    } else {
                        delta = { propertyDeltas: {} };
                        // (a rewrite-deleted key set to undefined reports undefined, as the reference)
                        for (const [k, v] of pd) { delta.propertyDeltas[k] = v; }
                    }
                } else {
                    delta = {};
                }
                let segment = { cachedLength: len };
                if (rich) { [segment, i] = this._segment(log, i, len); }
                delta.segment = segment;
                if (kind >= 0) {
                    // a zero-length insert's segment is never linked (blockInsert skips it,
                    // mergeTree.ts:2229) but is still in the callback: position -1
                    delta.position = pos;
                }
                deltaSegments.push(delta);
            }
            if (kind < 0) {
                if (mcb) { mcb({ operation: kind, deltaSegments }); }
                continue;
            }
            if (seq === -1) {
                // live client: the local client's own op (no sequencedMessage), in queue order
                while (mi < msgs.length && msgs[mi].__local === undefined) { mi++; }
                const op = mi < msgs.length ? msgs[mi++].__local : undefined;
                lastSeq = null;
                if (cb) { cb({ op }, { operation: kind, deltaSegments }); }
                continue;
            }
            // opArgs: the message with this sequence number; a GROUP's members in order
            if (seq !== lastSeq) { member = 0; lastSeq = seq; } else { member++; }
            while (mi < msgs.length && (msgs[mi].__local !== undefined || msgs[mi].__ack !== undefined ||
                msgs[mi].sequenceNumber !== seq)) { mi++; }
            const msg = mi < msgs.length ? msgs[mi] : { sequenceNumber: seq };
            const contents = msg.contents;
            const isGroup = contents && contents.type === 3;
            const opArgs = { op: isGroup ? contents.ops[member] : contents, sequencedMessage: msg };
            if (isGroup) { opArgs.groupOp = contents; }
            if (cb) { cb(opArgs, { operation: kind, deltaSegments }); }
        }
        this.batch.logPos[this.doc] = i;
    }

    /**
     * SequenceDeltaEvent (sequence/src/sequenceDeltaEvent.ts:26-118) for a callback's
     * arguments: ranges in document order with the positions the callback carries.  (The
     * reference sorts by segment ordinal and drops ranges whose ordinals collide, SURVEY Q8;
     * the positions here are exact.)
     */
    static sequenceDeltaEvent(opArgs, deltaArgs, clientId) {
        const ranges = deltaArgs.deltaSegments.filter((d) => d.position >= 0)
            .map((d) => ({ operation: deltaArgs.operation, position: d.position, propertyDeltas: d.propertyDeltas,
                segment: d.segment }))
            .sort((a, b) => a.position - b.position);
        return {
            opArgs, deltaArgs, isLocal: opArgs.sequencedMessage === undefined, isEmpty: deltaArgs.deltaSegments.length === 0,
            deltaOperation: deltaArgs.operation, ranges, first: ranges[0], last: ranges[ranges.length - 1], clientId,
        };
    }
}

module.exports = { GpuMergeTreeBatch, GpuClient, decodeSummaries, native, VAL_NULL };
