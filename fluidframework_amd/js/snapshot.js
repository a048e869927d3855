"use strict";
/**
 * snapshot.js -- SnapshotV1 summaries for the Node facade: decodes summary chunks the way
 * the reference loader does (SnapshotLoader.initialize/loadHeader/loadBody/specToSegment,
 * merge-tree/src/snapshotLoader.ts:36-228; SnapshotV1.processChunk snapshotV1.ts:266-277;
 * toLatestVersion snapshotChunks.ts:136-188) into the fixed 32-byte mt_seg_rec records of
 * mt_load_snapshots (include/mt_types.h).  Mirror of fluidframework_amd/snapshot.py.
 */
const HEADER = "header";
const BODY = "body";
const NON_COLLAB = -2;            // NonCollabClient            constants.ts:15
const RSEQ_NONE = -2147483648;    // removedSeq === undefined
const NO_PROPS = 0xFFFFFFFF;
const F_MARKER = 2;
const SEG_MERGE_INFO = 0x10;
const SEG_HAS_SEQ = 0x20;
const SEG_BYTES = 32;

function legacyHeaderMetadata(path, chunk) {   // buildHeaderMetadataForLegecyChunk :169-188
    if (path !== HEADER) { return undefined; }
    if (chunk.headerMetadata !== undefined) { return chunk.headerMetadata; }
    const ids = [{ id: HEADER }];
    if (chunk.chunkLengthChars < chunk.totalLengthChars) { ids.push({ id: BODY }); }
    return {
        orderedChunkMetadata: ids, minSequenceNumber: chunk.chunkMinSequenceNumber,
        sequenceNumber: chunk.chunkSequenceNumber, totalLength: chunk.totalLengthChars,
        totalSegmentCount: chunk.totalSegmentCount,
    };
}

function toLatestVersion(path, chunk) {       // toLatestVersion :136-167
    if (chunk.version === "1") { return chunk; }
    if (chunk.version === undefined) {
        return {
            version: "1", length: chunk.chunkLengthChars, segmentCount: chunk.chunkSegmentCount,
            headerMetadata: legacyHeaderMetadata(path, chunk), segments: chunk.segmentTexts,
            startIndex: chunk.chunkStartSegmentIndex,
        };
    }
    throw new Error(`Unsupported chunk path: ${path} version: ${chunk.version}`);
}

/** Blob path -> contents of a summary ITree (merge-tree blobs under "content" for a SharedString). */
function treeChunks(tree) {
    const content = tree.entries.find((e) => e.type === "Tree" && e.path === "content");
    const t = content ? content.value : tree;
    const out = {};
    for (const e of t.entries) { if (e.type === "Blob") { out[e.path] = e.value.contents; } }
    return out;
}

/** SnapshotLoader.initialize over blob contents: {headerSpecs, bodySpecs, minSeq, curSeq, catchup}. */
function decodeChunks(chunks) {
    if (chunks[HEADER] === undefined) { throw new Error("header blob missing"); }
    const header = toLatestVersion(HEADER, JSON.parse(chunks[HEADER]));
    const meta = header.headerMetadata;
    if (meta === undefined) { throw new Error("header metadata not available"); }
    const curSeq = meta.sequenceNumber;
    const minSeq = meta.minSequenceNumber !== undefined && meta.minSequenceNumber !== null ? meta.minSequenceNumber : curSeq;
    let body = [];
    const ordered = meta.orderedChunkMetadata;
    if (header.segmentCount !== meta.totalSegmentCount) {          // loadBody :170-172
        for (const md of ordered.slice(1)) {
            body = body.concat(toLatestVersion(md.id, JSON.parse(chunks[md.id])).segments);
        }
    }
    let catchup = [];
    const blobs = Object.keys(chunks);
    if (blobs.length === ordered.length + 1) {                     // :72-79
        const ids = new Set(ordered.map((m) => m.id));
        const rest = blobs.filter((b) => !ids.has(b));
        if (rest.length !== 1) { throw new Error(`There should be only one blob with catch up ops: ${rest.length}`); }
        catchup = JSON.parse(chunks[rest[0]]);
    } else if (blobs.length !== ordered.length) {
        throw new Error("Unexpected blobs in snapshot");
    }
    return { headerSpecs: header.segments, bodySpecs: body, minSeq, curSeq, catchup };
}

/** Records of many summaries for mt_load_snapshots (one per document, in handle order). */
class SnapshotEncoder {
    constructor(interner, Grow) {
        this.interner = interner;
        this.segs = new Grow(Uint8Array, 32 * 1024);
        this.nSegs = 0;
        this.text = new Grow(Uint16Array, 16 * 1024);
        this.props = new Grow(Uint32Array, 4 * 1024);
        this.docOff = [0];
        this.nHeader = [];
        this.minSeq = [];
        this.curSeq = [];
    }

    _props(p) {
        const off = this.props.n;
        const keys = Object.keys(p);
        this.props.push(keys.length >>> 0);
        for (const k of keys) {
            const kid = this.interner.key(k), vid = this.interner.val(p[k]);
            this.interner.note(kid, vid);
            this.props.push(kid);
            this.props.push(vid);
        }
        return off;
    }

    /** specToSegment :86-118 (+ SharedStringFactory.segmentFromSpec, sequenceFactory.ts:31-37). */
    _rec(spec, short) {
        const merge = !!spec && typeof spec === "object" && "json" in spec;   // hasMergeInfo
        const js = merge ? spec.json : spec;
        let len = 0, payload = 0, props = NO_PROPS, flags = 0, seq = 0, client = NON_COLLAB;
        let rseq = RSEQ_NONE, rcli = 0;
        let pr;
        if (typeof js === "string") {
            payload = this.text.n;
            this.text.reserve(js.length);
            for (let i = 0; i < js.length; i++) { this.text.a[this.text.n++] = js.charCodeAt(i); }
            len = js.length;
        } else if (js && typeof js === "object" && "text" in js) {
            payload = this.text.n;
            this.text.reserve(js.text.length);
            for (let i = 0; i < js.text.length; i++) { this.text.a[this.text.n++] = js.text.charCodeAt(i); }
            len = js.text.length;
            pr = js.props;
        } else if (js && typeof js === "object" && "marker" in js) {
            flags = F_MARKER;
            payload = js.marker.refType | 0;
            len = 1;
            pr = js.props;
        } else {
            throw new Error(`unsupported segment spec ${JSON.stringify(js)}`);
        }
        if (pr) { props = this._props(pr); }          // TextSegment.make / Marker.make: `if (props)`
        if (merge) {
            flags |= SEG_MERGE_INFO | (spec.seq !== undefined ? SEG_HAS_SEQ : 0);
            if (spec.client !== undefined) { client = short(spec.client); }
            if (spec.seq !== undefined) { seq = spec.seq; }
            if (spec.removedSeq !== undefined) { rseq = spec.removedSeq; }
            if (spec.removedClient !== undefined) { rcli = short(spec.removedClient); }
        }
        this.segs.reserve(SEG_BYTES);
        const dv = new DataView(this.segs.a.buffer, this.segs.a.byteOffset + this.segs.n, SEG_BYTES);
        dv.setInt32(0, len, true);
        dv.setInt32(4, seq, true);
        dv.setInt32(8, rseq, true);
        dv.setUint32(12, payload >>> 0, true);
        dv.setUint32(16, props >>> 0, true);
        dv.setInt16(20, client, true);
        dv.setInt16(22, rcli, true);
        dv.setUint8(24, flags);
        for (let i = 25; i < SEG_BYTES; i++) { dv.setUint8(i, 0); }
        this.segs.n += SEG_BYTES;
        this.nSegs++;
    }

    /** Adds one decoded summary; `clients` (Map long -> short, observer 0) receives its writers. */
    addDoc(snap, clients) {
        const short = (id) => {
            let s = clients.get(id);
            if (s === undefined) {
                s = clients.size + 1;
                clients.set(id, s);
            }
            return s;
        };
        for (const spec of snap.headerSpecs) { this._rec(spec, short); }
        this.nHeader.push(snap.headerSpecs.length);
        for (const spec of snap.bodySpecs) { this._rec(spec, short); }
        this.docOff.push(this.nSegs);
        this.minSeq.push(snap.minSeq);
        this.curSeq.push(snap.curSeq);
    }

    arrays() {
        return {
            docSegOff: BigInt64Array.from(this.docOff.map(BigInt)), nHeader: Int32Array.from(this.nHeader),
            segs: this.segs.a.subarray(0, Math.max(this.segs.n, SEG_BYTES)), nSegs: this.nSegs,
            text: this.text.view(), props: this.props.view(),
            minSeq: Int32Array.from(this.minSeq), curSeq: Int32Array.from(this.curSeq),
        };
    }
}

/**
 * Summary emission from mt_extract_snapshots records (one document): ISegment.toJSONObject
 * (textSegment.ts:48-54, mergeTree.ts:478-482, 690-694) with extractSync's merge-info wrapper
 * (snapshotV1.ts:222-241) -> {specs, lengths}.  `names[short id]` = the long client id.
 */
function recordSpecs(segs, text, props, interner, names) {
    const dv = new DataView(segs.buffer, segs.byteOffset, segs.byteLength);
    const specs = [], lengths = [];
    for (let r = 0; r + SEG_BYTES <= segs.byteLength; r += SEG_BYTES) {
        const len = dv.getInt32(r, true), seq = dv.getInt32(r + 4, true), rseq = dv.getInt32(r + 8, true);
        const payload = dv.getUint32(r + 12, true), pr = dv.getUint32(r + 16, true);
        const client = dv.getInt16(r + 20, true), rcli = dv.getInt16(r + 22, true), flags = dv.getUint8(r + 24);
        let propsObj;
        if (pr !== NO_PROPS) {
            propsObj = {};   // V8 orders integer-like keys first, as the reference's objects
            for (let j = 0; j < props[pr]; j++) {
                propsObj[interner.keyName(props[pr + 1 + 2 * j])] = interner.value(props[pr + 2 + 2 * j] >>> 0);
            }
        }
        let js;
        if (flags & F_MARKER) {
            js = { marker: { refType: payload } };
            if (propsObj !== undefined) { js.props = propsObj; }
        } else {
            let t = "";
            for (let i = 0; i < len; i += 4096) {
                t += String.fromCharCode.apply(null, Array.from(text.subarray(payload + i, payload + Math.min(len, i + 4096))));
            }
            js = propsObj === undefined ? t : { text: t, props: propsObj };
        }
        if (flags & SEG_MERGE_INFO) {
            const raw = { json: js };
            if (flags & SEG_HAS_SEQ) {
                raw.seq = seq;
                raw.client = names(client);
            }
            if (rseq !== RSEQ_NONE) {
                raw.removedSeq = rseq;
                raw.removedClient = names(rcli);
            }
            js = raw;
        }
        specs.push(js);
        lengths.push(len);
    }
    return { specs, lengths };
}

/**
 * SnapshotV1.emit (snapshotV1.ts:87-154): chunks of >= chunkSize units (getSeqLengthSegs
 * :59-81), the first is the header with the metadata; every blob is JSON.stringify of its
 * MergeTreeChunkV1 (serializeAsMaxSupportedVersion, snapshotChunks.ts:124-134).  Returns the
 * ITree a summarizer uploads.
 */
function emitTree(specs, lengths, minSeq, curSeq, chunkSize = 10000) {
    const header = { minSequenceNumber: minSeq, sequenceNumber: curSeq, orderedChunkMetadata: [],
        totalLength: 0, totalSegmentCount: 0 };
    const chunks = [];
    do {
        const start = header.totalSegmentCount;
        const segments = [];
        let length = 0, count = 0;
        while (length < chunkSize && start + count < specs.length) {
            segments.push(specs[start + count]);
            length += lengths[start + count];
            count++;
        }
        chunks.push({ version: "1", segmentCount: count, length, segments, startIndex: start });
        header.totalSegmentCount += count;
        header.totalLength += length;
    } while (header.totalSegmentCount < specs.length);
    const head = chunks.shift();
    head.headerMetadata = header;
    header.orderedChunkMetadata = [{ id: "header" }];
    const blob = (path, chunk) => ({ mode: "100644", path, type: "Blob",
        value: { contents: JSON.stringify(chunk), encoding: "utf-8" } });
    const entries = chunks.map((ch, i) => {
        const id = `body_${i}`;
        header.orderedChunkMetadata.push({ id });
        return blob(id, ch);
    });
    return { entries: [blob("header", head), ...entries], id: null };
}

module.exports = { SnapshotEncoder, decodeChunks, treeChunks, toLatestVersion, recordSpecs, emitTree };
