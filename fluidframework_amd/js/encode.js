"use strict";
/**
 * encode.js -- turns ISequencedDocumentMessage objects carrying merge-tree ops
 * (protocol-definitions/src/protocol.ts:132-172, merge-tree/src/ops.ts:63-110) into the
 * binary wire format of include/mt_types.h: one 32-byte mt_op_rec per op, a UTF-16 text
 * arena and a u32 property arena.  Mirrors fluidframework_amd/wire.py (the Python encoder
 * the tests use) field for field.
 *
 * Client ids are interned per document in first-seen order with the observer at 0, like
 * Client.getOrAddShortClientId (merge-tree/src/client.ts:637-661); only equality of short
 * ids matters to the replay.  Property keys and values are interned per batch; value ids
 * carry MT_VAL_FALSY_BIT when the JS value is falsy (the `rewrite` rule tests
 * `!newProps[key]`, merge-tree/src/segmentPropertiesManager.ts:72).
 */

const OP_INSERT = 0;
const OP_REMOVE = 1;
const OP_ANNOTATE = 2;
const OP_NOOP = 3;
const OP_GROUP = 3;          // MergeTreeDeltaType.GROUP in the op JSON (ops.ts:33)
const F_GROUP_MORE = 1;
const F_LOCAL = 8;           // live handles: the local client's own unsequenced op (mt_types.h)
const F_ACK = 16;            // live handles: the sequenced echo of one of them
const F_MARKER = 2;
const NO_PROPS = 0xFFFFFFFF;
const VAL_NULL = 0xFFFFFFFF;
const VAL_UNDEF = 0xFFFFFFFE;       // a key set to the JS value undefined
const VAL_FALSY_BIT = 0x80000000;
const VAL_NOMATCH_BIT = 0x40000000; // matchProperties never finds the value equal
const COMBINE_NONE = 0;
const COMBINE_REWRITE = 1;
const COMBINE_OTHER = 2;
const COMBINE_TABLE = 3;
const OP_BYTES = 32;

/**
 * Canonical JSON (sorted keys): matchProperties compares nested values structurally.  NaN and
 * undefined -- left in property sets by non-rewrite combining ops (SURVEY Q4) -- get tokens
 * of their own.
 */
function canonical(v) {
    if (v === undefined) { return "undefined"; }
    if (typeof v === "number" && Number.isNaN(v)) { return "NaN"; }
    if (v === null || typeof v !== "object") { return JSON.stringify(v); }
    if (Array.isArray(v)) { return `[${v.map(canonical).join(",")}]`; }
    return `{${Object.keys(v).sort().map((k) => `${JSON.stringify(k)}:${canonical(v[k])}`).join(",")}}`;
}

/** matchProperties(a, a) is false for a set holding v (NaN, or undefined at any depth). */
function noMatch(v) {
    if (v === undefined || (typeof v === "number" && Number.isNaN(v))) { return true; }
    if (v !== null && typeof v === "object") { return Object.keys(v).some((k) => noMatch(v[k])); }
    return false;
}

class Unsupported extends Error {}

/**
 * Properties.combine(op, currentValue, undefined, seq) (merge-tree/src/properties.ts:26-59) as
 * SegmentPropertiesManager.addProperties calls it for a non-rewrite combining op
 * (segmentPropertiesManager.ts:93-107: the new value is never passed in; SURVEY Q4).
 */
function jsCombine(op, cur, seq) {
    if (cur === undefined) { cur = op.defaultValue; }
    if (op.name === "incr") {
        if (op.minValue && typeof op.minValue !== "number") { throw new Unsupported("incr with a non-numeric minValue"); }
        return cur + undefined;   // NaN, or a string; never below a numeric minValue
    }
    if (op.name === "consensus") {
        if (cur === undefined) { return { value: undefined, seq }; }
        if (cur === null) { throw new Unsupported("consensus over null"); }
        if (typeof cur === "object" && cur.seq === -1) { throw new Unsupported("consensus over a shared {seq: -1}"); }
        return cur;
    }
    return cur;
}

class Interner {
    constructor() {
        this.keys = [];
        this.keyIds = new Map();
        this.vals = [];
        this.valIds = new Map();
        // the values each key can hold (ids without flag bits), for combining-op tables
        // (wire.py Interner.note / held_values)
        this.keyVals = new Map();
        this.unkeyed = new Set();
    }
    note(kid, vid) {
        if (vid === VAL_NULL || vid === VAL_UNDEF) { return; }
        let s = this.keyVals.get(kid);
        if (s === undefined) { s = new Set(); this.keyVals.set(kid, s); }
        s.add((vid & 0x3FFFFFFF) >>> 0);
    }
    noteUnkeyed(vid) {
        if (vid === VAL_NULL || vid === VAL_UNDEF) { return; }
        this.unkeyed.add((vid & 0x3FFFFFFF) >>> 0);
    }
    heldValues(kids) {
        const out = new Set(this.unkeyed);
        for (const k of kids) {
            const s = this.keyVals.get(k);
            if (s !== undefined) { for (const v of s) { out.add(v); } }
        }
        return Array.from(out).sort((a, b) => a - b);
    }
    key(k) {
        let i = this.keyIds.get(k);
        if (i === undefined) {
            i = this.keys.length;
            this.keyIds.set(k, i);
            this.keys.push(k);
        }
        return i;
    }
    val(v) {
        if (v === null) { return VAL_NULL; }
        if (v === undefined) { return VAL_UNDEF; }
        const c = canonical(v);
        let i = this.valIds.get(c);
        if (i === undefined) {
            i = this.vals.length;
            this.valIds.set(c, i);
            this.vals.push(v);
        }
        return (i | (v ? 0 : VAL_FALSY_BIT) | (noMatch(v) ? VAL_NOMATCH_BIT : 0)) >>> 0;
    }
    keyName(id) { return this.keys[id]; }
    value(id) {
        if (id === VAL_NULL) { return null; }
        if (id === VAL_UNDEF) { return undefined; }
        return this.vals[(id & ~(VAL_FALSY_BIT | VAL_NOMATCH_BIT)) >>> 0];
    }
}

/** Growable typed-array builder. */
class Grow {
    constructor(Ctor, cap = 1024) {
        this.Ctor = Ctor;
        this.a = new Ctor(cap);
        this.n = 0;
    }
    reserve(k) {
        if (this.n + k <= this.a.length) { return; }
        let cap = this.a.length * 2;
        while (cap < this.n + k) { cap *= 2; }
        const b = new this.Ctor(cap);
        b.set(this.a.subarray(0, this.n));
        this.a = b;
    }
    push(x) { this.reserve(1); this.a[this.n++] = x; }
    view() { return this.a.subarray(0, Math.max(this.n, 1)); }
}

/**
 * Accumulates the messages of N documents (CSR by document) ready for mt_apply_ops.
 * Documents are added in handle order; each document's messages in sequence order.
 */
class BatchEncoder {
    constructor(interner = new Interner()) {
        this.interner = interner;
        this.ops = new Grow(Uint8Array, 32 * 1024);
        this.nOps = 0;
        this.text = new Grow(Uint16Array, 16 * 1024);
        this.props = new Grow(Uint32Array, 4 * 1024);
        this.docOff = [0];
    }

    _text(s) {
        const off = this.text.n;
        this.text.reserve(s.length);
        for (let i = 0; i < s.length; i++) { this.text.a[this.text.n++] = s.charCodeAt(i); }
        return [off, s.length];
    }

    _props(p, combine = COMBINE_NONE) {
        const off = this.props.n;
        const keys = Object.keys(p);
        this.props.push((keys.length | (combine << 16)) >>> 0);
        for (const k of keys) {
            const kid = this.interner.key(k), vid = this.interner.val(p[k]);
            this.interner.note(kid, vid);
            this.props.push(kid);
            this.props.push(vid);
        }
        return off;
    }

    /**
     * A non-rewrite combining op's record (SURVEY Q4): the keys, then combine(op, old,
     * undefined, seq) for every value one of its keys can hold now (Interner.heldValues) -- [n, new value of an absent key,
     * (old, new) x n]; VAL_NULL deletes.  Mirrors wire.py Batch._combine_rec.
     */
    _combineProps(p, comb, seq) {
        const it = this.interner;
        const kids = Object.keys(p).map((k) => it.key(k));
        let absent;
        const pairs = [];
        try {
            absent = it.val(jsCombine(comb, undefined, seq));
            for (const i of it.heldValues(kids)) {
                const v = it.vals[i];
                pairs.push([it.val(v), it.val(jsCombine(comb, v, seq))]);
            }
        } catch (e) {
            if (!(e instanceof Unsupported)) { throw e; }
            return this._props(p, COMBINE_OTHER);
        }
        const off = this._props(p, COMBINE_TABLE);
        for (const kid of kids) {
            it.note(kid, absent);
            for (const [, n] of pairs) { it.note(kid, n); }
        }
        this.props.push(pairs.length);
        this.props.push(absent);
        for (const [o, n] of pairs) { this.props.push(o); this.props.push(n); }
        return off;
    }

    _rec(r) {
        this.ops.reserve(OP_BYTES);
        const dv = new DataView(this.ops.a.buffer, this.ops.a.byteOffset + this.ops.n, OP_BYTES);
        dv.setInt32(0, r.seq, true);
        dv.setInt32(4, r.refSeq, true);
        dv.setInt32(8, r.minSeq, true);
        dv.setInt32(12, r.pos1, true);
        dv.setInt32(16, r.pos2, true);
        dv.setUint32(20, r.payload >>> 0, true);
        dv.setUint32(24, r.props >>> 0, true);
        dv.setUint16(28, r.client, true);
        dv.setUint8(30, r.kind);
        dv.setUint8(31, r.flags);
        this.ops.n += OP_BYTES;
        this.nOps++;
    }

    _op(msg, client, op, more) {
        const r = {
            seq: msg.sequenceNumber, refSeq: msg.referenceSequenceNumber, minSeq: msg.minimumSequenceNumber,
            client, flags: more ? F_GROUP_MORE : 0, props: NO_PROPS, pos1: 0, pos2: 0, payload: 0, kind: OP_NOOP,
        };
        if (op.type === OP_INSERT) {
            const seg = op.seg;
            r.kind = OP_INSERT;
            r.pos1 = op.pos1;
            if (!seg) {
                // `if (op.seg)` is falsy: applyInsertOp returns without touching the tree
                // (client.ts:402-426) -> only the seq/msn update
                r.kind = OP_NOOP;
            } else if (typeof seg === "string") {
                [r.payload, r.pos2] = this._text(seg);
            } else if (seg.text !== undefined) {
                [r.payload, r.pos2] = this._text(seg.text);
                if (seg.props !== undefined && seg.props !== null) { r.props = this._props(seg.props); }
            } else if (seg.marker !== undefined) {
                r.flags |= F_MARKER;
                r.payload = seg.marker.refType | 0;
                r.pos2 = 1;
                if (seg.props !== undefined && seg.props !== null) { r.props = this._props(seg.props); }
            } else {
                throw new Error(`unsupported insert segment ${JSON.stringify(seg)}`);
            }
        } else if (op.type === OP_REMOVE || op.type === OP_ANNOTATE) {
            if (op.relativePos1 !== undefined || op.relativePos2 !== undefined || op.register !== undefined) {
                throw new Error("relative-position and register ops are not supported by the replay backend");
            }
            r.kind = op.type;
            r.pos1 = op.pos1;
            r.pos2 = op.pos2;
            if (op.type === OP_ANNOTATE) {
                const c = op.combiningOp;
                if (c && c.name !== "rewrite") {
                    r.props = this._combineProps(op.props, c, msg.sequenceNumber);
                } else {
                    r.props = this._props(op.props, c ? COMBINE_REWRITE : COMBINE_NONE);
                }
            }
        } else {
            throw new Error(`unsupported op type ${op.type}`);
        }
        this._rec(r);
    }

    /**
     * Appends one document's messages.  `clients` is the document's persistent long->short
     * id map (observer = 0), shared across batches so ids stay stable.
     */
    addDoc(msgs, clients) {
        const short = (id) => {
            let s = clients.get(id);
            if (s === undefined) {
                s = 1;
                for (const v of clients.values()) { s = Math.max(s, v + 1); }
                clients.set(id, s);
            }
            return s;
        };
        const members = (msg, c, flags) => {
            const op = msg.contents;
            if (op.type === OP_GROUP && op.ops.length === 0) {
                // an empty GROUP applies nothing; applyMsg still updates seq/msn (client.ts:818)
                this._rec({
                    seq: msg.sequenceNumber, refSeq: msg.referenceSequenceNumber, minSeq: msg.minimumSequenceNumber,
                    client: c, kind: OP_NOOP, flags: 0, props: NO_PROPS, pos1: 0, pos2: 0, payload: 0,
                });
                return;
            }
            const ops = op.type === OP_GROUP ? op.ops : [op];
            ops.forEach((m, i) => {
                this._op(msg, c, m, i + 1 < ops.length);
                const at = this.ops.n - 1;          // the flags byte of the record just written
                this.ops.a[at] |= flags;
            });
        };
        for (const msg of msgs) {
            if (msg.__local !== undefined) {        // live handles: a local op (client 0)
                members({ sequenceNumber: -1, referenceSequenceNumber: 0, minimumSequenceNumber: 0,
                    contents: msg.__local }, 0, F_LOCAL);
                continue;
            }
            if (msg.__ack !== undefined) {          // live handles: the echo of a local op
                members(msg.__ack, 0, F_ACK);
                continue;
            }
            if (msg.__update !== undefined) {       // Client.updateSeqNumbers(msn, seq) (client.ts:821-828)
                this._rec({
                    seq: msg.__update.seq, refSeq: msg.__update.seq, minSeq: msg.__update.msn, client: 0,
                    kind: OP_NOOP, flags: 0, props: NO_PROPS, pos1: 0, pos2: 0, payload: 0,
                });
                continue;
            }
            const c = short(msg.clientId);
            if (msg.type !== undefined && msg.type !== "op") {
                this._rec({
                    seq: msg.sequenceNumber, refSeq: msg.referenceSequenceNumber, minSeq: msg.minimumSequenceNumber,
                    client: c, kind: OP_NOOP, flags: 0, props: NO_PROPS, pos1: 0, pos2: 0, payload: 0,
                });
                continue;
            }
            members(msg, c, 0);
        }
        this.docOff.push(this.nOps);
    }

    arrays() {
        return {
            docOff: BigInt64Array.from(this.docOff.map(BigInt)),
            ops: this.ops.a.subarray(0, this.ops.n),
            text: this.text.view(),
            props: this.props.view(),
        };
    }
}

module.exports = {
    BatchEncoder, Interner, Grow, canonical,
    OP_INSERT, OP_REMOVE, OP_ANNOTATE, OP_NOOP, F_GROUP_MORE, F_MARKER, F_LOCAL, F_ACK, NO_PROPS, VAL_NULL, VAL_UNDEF,
    VAL_FALSY_BIT, VAL_NOMATCH_BIT, jsCombine,
};
