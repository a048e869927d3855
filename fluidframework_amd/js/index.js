"use strict";
/**
 * index.js -- Node facade of the MI355X merge-tree replay backend.
 *
 * GpuMergeTreeBatch owns N observer replicas resident on one GPU (one handle of the C ABI,
 * include/mt_replay.h, through the N-API addon js/binding.cc).  batch.client(doc) returns a
 * Client-shaped view of one document with the surface SharedSegmentSequence uses on the
 * reference Client (merge-tree/src/client.ts:43; sequence/src/sequence.ts:131-142,
 * 240-251, 473-600): applyMsg, startOrUpdateCollaboration, getLength, getText (as
 * createTextHelper().getText), getPropertiesAtPosition, getPosition, getContainingSegment,
 * getCurrentSeq, getShortClientId / getLongClientId, snapshot, the mergeTreeDeltaCallback /
 * mergeTreeMaintenanceCallback properties and a `mergeTree` view (getLength(refSeq,
 * clientId), getPosition, getContainingSegment).  Callback segments are objects kept per
 * segment id (a segment is the same object in every event, as in the reference) with the
 * state, cachedLength and ordinal they had at the event, so SharedSegmentSequence's own
 * SequenceDeltaEvent (sequence/src/sequenceDeltaEvent.ts) runs unchanged on a GpuClient.
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
const { treeChunks, recordSpecs, emitTree } = require("./snapshot");

// segment object -> its device id (mt_seg_info.uid) for getPosition outside a callback
const segUid = new WeakMap();

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
    // SnapshotLoader.loadBody re-inserted segments of its never-emptied batch (mt_types.h)
    10: () => new Error("merge-tree replay: the summary body makes SnapshotLoader insert segments twice " +
        "(snapshotLoader.ts:207-227); the document is not replayed past that point"),
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
        // event handles keep segment ordinals (SequenceDeltaEvent orders ranges by them), in
        // the flat tiers and the paged layout alike
        if (this.rich && options.segmentOrdinals === undefined) {
            options = Object.assign({}, options, { segmentOrdinals: 1 });
        }
        this.ordinals = !!options.segmentOrdinals;
        this.chunkSize = options.mergeTreeSnapshotChunkSize || 10000;   // SnapshotV1.chunkSize
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
        this.segObjs = Array.from({ length: nDocs }, () => new Map());   // per document: id -> segment
        this.inflight = null;
    }

    _idle() {
        if (this.inflight) { throw new Error("merge-tree replay: a flushAsync() is in flight on this batch"); }
    }

    /** Initial contents of every document (Client.insertSegmentLocal before collaboration). */
    loadInitialText(texts) {
        this._idle();
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
        this.segObjs = Array.from({ length: this.nDocs }, () => new Map());
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
        this.segObjs = Array.from({ length: this.nDocs }, () => new Map());
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

    _encodePending() {
        const enc = new BatchEncoder(this.interner);
        this.applied = this.pending;   // the messages of this flush, for the callbacks' opArgs
        for (let d = 0; d < this.nDocs; d++) {
            enc.addDoc(this.pending[d], this.clients[d]);
        }
        this.pending = Array.from({ length: this.nDocs }, () => []);
        this.queued = 0;
        return enc.arrays();
    }

    /** Applies every queued message of every document (one mt_apply_ops). */
    flush() {
        this._idle();
        if (this.queued === 0) { return; }
        const a = this._encodePending();
        native.applyOps(this.h, a.docOff, a.ops, a.text, a.props);
        this._afterApply();
    }

    /**
     * flush() with the GPU work on a worker thread (napi_async_work): resolves once the batch
     * is applied and its callbacks have fired.  Messages queued meanwhile wait for the next
     * flush; any other call on the batch throws until it resolves (a handle is single-writer).
     */
    async flushAsync() {
        while (this.inflight) { await this.inflight.catch(() => undefined); }
        if (this.queued === 0) { return; }
        const a = this._encodePending();
        this.inflight = native.applyOpsAsync(this.h, a.docOff, a.ops, a.text, a.props);
        try {
            await this.inflight;
        } finally {
            this.inflight = null;
        }
        this._afterApply();
    }

    _afterApply() {
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

    /**
     * Client.snapshot for every document (client.ts:901-937, new summary format): each
     * document's SnapshotV1 ITree (snapshotV1.ts:87-252), extracted on the GPU
     * (mt_extract_snapshots) and emitted as the reference's JSON blobs.
     */
    snapshots() {
        this.flush();
        const ex = native.extractSnapshots(this.h);
        const out = [];
        let r0 = 0, t0 = 0, p0 = 0;
        for (let d = 0; d < this.nDocs; d++) {
            const nr = Number(ex.counts[3 * d]), nt = Number(ex.counts[3 * d + 1]), np = Number(ex.counts[3 * d + 2]);
            const segs = ex.segs.subarray(32 * r0, 32 * (r0 + nr));
            const names = this._clientNames(d);
            const { specs, lengths } = recordSpecs(segs, ex.text.subarray(t0, t0 + nt), ex.props.subarray(p0, p0 + np),
                this.interner, names);
            out.push(emitTree(specs, lengths, ex.minSeq[d], ex.curSeq[d], this.chunkSize));
            r0 += nr;
            t0 += nt;
            p0 += np;
        }
        return { trees: out, minSeq: ex.minSeq, curSeq: ex.curSeq };
    }

    // short client id -> long id of document d (0: the replica's own id)
    _clientNames(d) {
        const inv = new Map();
        for (const [k, v] of this.clients[d]) { if (!inv.has(v)) { inv.set(v, k); } }
        const v = this.views.get(d);
        return (id) => (id === 0 && v && v.longClientId !== undefined ? v.longClientId : inv.get(id));
    }

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

    /**
     * A segment's state at an event (rich log), as the ISegment fields listeners read.  On an
     * ordinals handle the entry also names the segment (its id: the same object is reused for
     * it in every event, as the reference passes one ISegment) and carries the position
     * Client.getPosition reads at the event and the segment's ordinal.  Returns [seg, i, pos].
     */
    _segment(log, i, len) {
        const flags = log[i++];
        const st = { cachedLength: len };
        if (flags & 1) {
            st.type = "Marker";
            st.refType = log[i++];
        } else {
            const words = (len + 1) >> 1;
            let text = "";
            for (let u = 0; u < len; u += 2048) {
                const units = [];
                for (let k = u; k < Math.min(len, u + 2048); k++) {
                    const w = log[i + (k >> 1)];
                    units.push((k & 1) ? (w >>> 16) : (w & 0xFFFF));
                }
                text += String.fromCharCode(...units);
            }
            i += words;
            st.type = "TextSegment";
            st.text = text;
        }
        const np = log[i++];
        if (np >= 0) {
            const pairs = [];
            for (let j = 0; j < np; j++) {
                pairs.push([this.batch.interner.keyName(log[i]), this.batch.interner.value(log[i + 1] >>> 0)]);
                i += 2;
            }
            st.properties = {};
            for (const [k, v] of jsKeyOrder(pairs)) { st.properties[k] = v; }
        }
        let seg = st, pos;
        if (flags & 4) {   // [uid, position at the event, ordinal length (-1: none), characters]
            const uid = log[i] >>> 0, olen = log[i + 2];
            pos = log[i + 1];
            st.ordinal = olen >= 0 ? String.fromCharCode(...log.subarray(i + 3, i + 3 + olen)) : undefined;
            i += 3 + Math.max(olen, 0);
            seg = this._segObject(uid, st);
        }
        return [seg, i, pos];
    }

    // the document's object for segment `uid` (0: never linked -- a fresh object), updated to `st`
    _segObject(uid, st) {
        const objs = this.batch.segObjs[this.doc];
        let seg = uid ? objs.get(uid) : undefined;
        if (seg === undefined) {
            seg = {};
            if (uid) {
                objs.set(uid, seg);
                segUid.set(seg, uid);
            }
        }
        for (const k of ["text", "refType", "properties"]) { if (!(k in st)) { delete seg[k]; } }
        Object.assign(seg, st);
        return seg;
    }

    // a read-out (native getContainingSegment / getSegmentByUid) as the segment's object
    _segFromInfo(r) {
        const st = { cachedLength: r.length, seq: r.seq, clientId: r.clientId };
        if (r.markerRefType >= 0) {
            st.type = "Marker";
            st.refType = r.markerRefType;
        } else {
            st.type = "TextSegment";
            st.text = r.text;
        }
        if (r.removedSeq !== -2147483648) {
            st.removedSeq = r.removedSeq;
            st.removedClientId = r.removedClientId;
        }
        if (r.propPairs) {
            const pairs = [];
            for (let j = 0; j < r.propPairs.length; j += 2) {
                pairs.push([this.batch.interner.keyName(r.propPairs[j]), this.batch.interner.value(r.propPairs[j + 1])]);
            }
            st.properties = {};
            for (const [k, v] of jsKeyOrder(pairs)) { st.properties[k] = v; }
        }
        if (r.ordinal !== undefined) { st.ordinal = r.ordinal; }
        return this._segObject(r.uid, st);
    }

    /**
     * Client.getPosition(segment) (client.ts:291-293, mergeTree.ts:1619-1636).  Inside a
     * callback, a segment of that event reads the position it had when the reference fired it
     * (what SequenceDeltaEvent.ranges computes); otherwise the segment's position after the
     * last flush -- 0 once it left the tree (the reference walks no parent then).
     */
    getPosition(segment) {
        if (this._evPos !== undefined && this._evPos.has(segment)) { return this._evPos.get(segment); }
        return this.mergeTree.getPosition(segment, this.currentSeq, 0);
    }

    /** Client.getContainingSegment(pos) (client.ts:1006-1009, mergeTree.ts:1656-1667). */
    getContainingSegment(pos) {
        return this.mergeTree.getContainingSegment(pos, this.currentSeq, 0);
    }

    /** Client.getShortClientId / getLongClientId (client.ts:637-661): the observer is 0. */
    getShortClientId(longClientId) {
        if (longClientId === this.longClientId) { return 0; }
        return this.batch.clients[this.doc].get(longClientId);
    }

    getLongClientId(shortClientId) { return this.batch._clientNames(this.doc)(shortClientId); }

    getClientId() { return 0; }

    /**
     * The MergeTree methods SharedSegmentSequence and its users reach through client.mergeTree
     * (mergeTree.ts:1610-1667): views (refSeq, clientId) with short client ids; a remote view
     * must be one the client can still hold (include/mt_replay.h "segment read-outs").
     */
    get mergeTree() {
        if (this._mt === undefined) {
            const self = this;
            const h = () => self.batch.h;
            this._mt = {
                get length() { return self.getLength(); },
                getLength(refSeq, clientId) {
                    self._sync();
                    return native.getViewLengths(h(), Uint32Array.of(self.doc), Int32Array.of(refSeq),
                        Int32Array.of(clientId))[0];
                },
                getPosition(segment, refSeq, clientId) {
                    const uid = segUid.get(segment);
                    if (uid === undefined) { return 0; }
                    self._sync();
                    const r = native.getSegmentByUid(h(), self.doc, uid, refSeq, clientId);
                    return r === null ? 0 : r.position;
                },
                getContainingSegment(pos, refSeq, clientId) {
                    self._sync();
                    const r = native.getContainingSegment(h(), self.doc, pos, refSeq, clientId);
                    return r === null ? { segment: undefined, offset: undefined }
                        : { segment: self._segFromInfo(r), offset: r.offset };
                },
                get mergeTreeDeltaCallback() { return self.mergeTreeDeltaCallback; },
                set mergeTreeDeltaCallback(f) { self.mergeTreeDeltaCallback = f; },
                get mergeTreeMaintenanceCallback() { return self.mergeTreeMaintenanceCallback; },
                set mergeTreeMaintenanceCallback(f) { self.mergeTreeMaintenanceCallback = f; },
            };
        }
        return this._mt;
    }

    /**
     * Client.snapshot(runtime, handle, catchUpMsgs) (client.ts:901-937) in the new summary
     * format (mergeTree options newMergeTreeSnapshotFormat): updateSeqNumbers(the runtime's
     * minimumSequenceNumber, lastSequenceNumber), then SnapshotV1.extractSync + emit
     * (snapshotV1.ts:87-252) -> the ITree, blobs byte-equal with the reference's.
     */
    snapshot(runtime, handle, catchUpMsgs) {
        assert(catchUpMsgs === undefined || catchUpMsgs.length === 0, "New format should not emit catchup ops");
        const dm = runtime.deltaManager;
        this._check();
        this.batch.pending[this.doc].push({ __update: { seq: dm.lastSequenceNumber, msn: dm.minimumSequenceNumber } });
        this.batch.queued++;
        this.currentSeq = Math.max(this.currentSeq, dm.lastSequenceNumber);
        this._sync();
        const s = this.batch.snapshots();
        assert.strictEqual(s.minSeq[this.doc], dm.minimumSequenceNumber);
        return s.trees[this.doc];
    }

    /**
     * Replays the device delta log of the last flush into the reference's callbacks:
     * mergeTreeDeltaCallback(opArgs, {operation, deltaSegments}) (mergeTreeDeltaCallback.ts:
     * 33-59; call sites mergeTree.ts:2014-2021, 2625-2632, 2738-2745) with opArgs {op,
     * sequencedMessage, groupOp} and deltaSegments [{segment, propertyDeltas}] -- segment =
     * the segment's state at the event (cachedLength, text or refType, properties, ordinal)
     * plus our `position` field (its observer position at callback time) -- and
     * mergeTreeMaintenanceCallback({operation: SPLIT -2 | APPEND -1 | UNLINK -3,
     * deltaSegments}) (mergeTree.ts:1343-1373, 2264-2269), in the reference's order.
     */
    _emitDeltas() {
        const cb = this.mergeTreeDeltaCallback, mcb = this.mergeTreeMaintenanceCallback;
        const rich = this.batch.rich;
        const log = native.getDeltaLog(this.batch.h, this.doc);
        const msgs = (this.batch.applied && this.batch.applied[this.doc]) || [];
        const objs = this.batch.segObjs[this.doc];
        let mi = 0, member = 0, lastSeq = null;
        let i = this.batch.logPos[this.doc];
        while (i + 3 <= log.length) {
            const seq = log[i], kind = log[i + 1], n = log[i + 2];
            i += 3;
            const deltaSegments = [];
            const evPos = new Map();
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
                let segment = { cachedLength: len }, epos;
                if (rich) { [segment, i, epos] = this._segment(log, i, len); }
                if (epos !== undefined) { evPos.set(segment, epos); }
                delta.segment = segment;
                if (kind >= 0) {
                    // a zero-length insert's segment is never linked (blockInsert skips it,
                    // mergeTree.ts:2229) but is still in the callback: position -1
                    delta.position = pos;
                }
                deltaSegments.push(delta);
            }
            this._evPos = evPos;
            try {
                if (kind < 0) {
                    if (mcb) { mcb({ operation: kind, deltaSegments }); }
                    // the segment an UNLINK drops / an APPEND absorbs leaves the tree
                    const gone = kind === -3 ? deltaSegments[0] : (kind === -1 ? deltaSegments[1] : undefined);
                    if (gone !== undefined && segUid.has(gone.segment)) { objs.delete(segUid.get(gone.segment)); }
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
                    msgs[mi].__update !== undefined || msgs[mi].sequenceNumber !== seq)) { mi++; }
                const msg = mi < msgs.length ? msgs[mi] : { sequenceNumber: seq };
                const contents = msg.contents;
                const isGroup = contents && contents.type === 3;
                const opArgs = { op: isGroup ? contents.ops[member] : contents, sequencedMessage: msg };
                if (isGroup) { opArgs.groupOp = contents; }
                if (cb) { cb(opArgs, { operation: kind, deltaSegments }); }
            } finally {
                this._evPos = undefined;
            }
        }
        this.batch.logPos[this.doc] = i;
    }
}

module.exports = { GpuMergeTreeBatch, GpuClient, decodeSummaries, native, VAL_NULL };
