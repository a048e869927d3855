"""Host-side encoding of sequenced merge-tree messages into the binary wire format of
include/mt_types.h (one 32-byte ``mt_op_rec`` per op, a UTF-16 text arena and a u32
props arena).

This is the Python mirror of the JS facade's encoder (fluidframework_amd/js/encode.js):
it accepts ``ISequencedDocumentMessage``-shaped dicts (PD/protocol.ts:132-172) carrying
IMergeTree ops (MT/ops.ts:63-110) and interns client ids (first-seen order per document,
like Client.getOrAddShortClientId MT/client.ts:637-661), property keys and property values.
"""
import json
import numpy as np

OP_INSERT, OP_REMOVE, OP_ANNOTATE, OP_NOOP = 0, 1, 2, 3
F_GROUP_MORE, F_MARKER = 1, 2
NO_PROPS = 0xFFFFFFFF
VAL_NULL = 0xFFFFFFFF
VAL_FALSY_BIT = 0x80000000
COMBINE_NONE, COMBINE_REWRITE, COMBINE_OTHER = 0, 1, 2

OP_DTYPE = np.dtype([
    ("seq", "<i4"), ("ref_seq", "<i4"), ("min_seq", "<i4"), ("pos1", "<i4"), ("pos2", "<i4"),
    ("payload", "<u4"), ("props", "<u4"), ("client", "<u2"), ("kind", "u1"), ("flags", "u1"),
])
assert OP_DTYPE.itemsize == 32

CHECKSUM_DTYPE = np.dtype([
    ("length", "<u4"), ("n_segments", "<u4"), ("text_hash", "<u8"), ("props_hash", "<u8"),
    ("delta_hash", "<u8"),
])
assert CHECKSUM_DTYPE.itemsize == 32


def canonical_json(v):
    """Canonical form used to intern property values: matchProperties
    (MT/properties.ts:61-92) compares nested objects structurally, ignoring key order."""
    return json.dumps(v, sort_keys=True, separators=(",", ":"), ensure_ascii=False)


def js_falsy(v):
    return v is None or v is False or v == "" or (isinstance(v, (int, float)) and not isinstance(v, bool) and v == 0)


class Interner:
    """Property key / value interning shared by every document of a batch."""

    def __init__(self, synthetic=False):
        self.keys, self.key_ids = [], {}
        self.vals, self.val_ids = [], {}
        self.synthetic = synthetic

    def key(self, k):
        if self.synthetic:
            return int(k[1:])
        i = self.key_ids.get(k)
        if i is None:
            i = self.key_ids[k] = len(self.keys)
            self.keys.append(k)
        return i

    def val(self, v):
        if v is None:
            return VAL_NULL
        if self.synthetic:
            return int(v) | (VAL_FALSY_BIT if int(v) == 0 else 0)
        c = canonical_json(v)
        i = self.val_ids.get(c)
        if i is None:
            i = len(self.vals)
            self.val_ids[c] = i
            self.vals.append(v)
        return i | (VAL_FALSY_BIT if js_falsy(v) else 0)

    def key_name(self, kid):
        return f"k{kid}" if self.synthetic else self.keys[kid]

    def val_value(self, vid):
        if vid == VAL_NULL:
            return None
        if self.synthetic:
            return vid & ~VAL_FALSY_BIT
        return self.vals[vid & ~VAL_FALSY_BIT]


class DocEncoder:
    """Encodes one document's messages; arenas are shared by a Batch."""

    def __init__(self, batch, short=None):
        self.batch = batch
        self.short = dict(short) if short else {}
        self.next = 1 + max(self.short.values(), default=0)   # the observer is 0

    def client(self, long_id):
        s = self.short.get(long_id)
        if s is None:
            s = self.short[long_id] = self.next
            self.next += 1
        return s


class Batch:
    """Accumulates encoded documents into CSR arrays ready for the C ABI."""

    def __init__(self, interner=None):
        self.interner = interner or Interner()
        self.recs = []
        self.text = []
        self.props = []
        self.doc_off = [0]
        self.seed_off = [0]
        self.seed = []
        self.clients = []          # per document: long client id -> short id

    def _props_rec(self, props, combine=COMBINE_NONE):
        off = len(self.props)
        items = list(props.items())
        self.props.append(len(items) | (combine << 16))
        for k, v in items:
            self.props.append(self.interner.key(k))
            self.props.append(self.interner.val(v))
        return off

    def _text(self, s):
        off = len(self.text)
        b = s.encode("utf-16-le")
        self.text.extend(np.frombuffer(b, dtype="<u2").tolist())
        return off, len(b) // 2

    def _op(self, enc, msg, op, more):
        c = enc.client(msg["clientId"])
        base = dict(seq=msg["sequenceNumber"], ref_seq=msg["referenceSequenceNumber"],
                    min_seq=msg["minimumSequenceNumber"], client=c,
                    flags=F_GROUP_MORE if more else 0, props=NO_PROPS, pos1=0, pos2=0, payload=0)
        t = op["type"]
        if t == OP_INSERT:
            seg = op.get("seg")
            base["kind"] = OP_INSERT
            base["pos1"] = op["pos1"]
            if not seg and not isinstance(seg, dict):
                # `if (op.seg)` is falsy (e.g. ""): applyInsertOp returns false without
                # touching the tree (MT/client.ts:402-426) -> only the seq/msn update.
                base["kind"] = OP_NOOP
            elif isinstance(seg, str):
                base["payload"], base["pos2"] = self._text(seg)
            elif isinstance(seg, dict) and "text" in seg:
                base["payload"], base["pos2"] = self._text(seg["text"])
                if seg.get("props") is not None:
                    base["props"] = self._props_rec(seg["props"])
            elif isinstance(seg, dict) and "marker" in seg:
                base["flags"] |= F_MARKER
                base["payload"] = int(seg["marker"].get("refType", 0))
                base["pos2"] = 1
                if seg.get("props") is not None:
                    base["props"] = self._props_rec(seg["props"])
            else:
                raise ValueError(f"unsupported insert segment {seg!r}")
        elif t in (OP_REMOVE, OP_ANNOTATE):
            base["kind"] = t
            base["pos1"], base["pos2"] = op["pos1"], op["pos2"]
            if t == OP_ANNOTATE:
                comb = op.get("combiningOp")
                code = COMBINE_NONE if not comb else (
                    COMBINE_REWRITE if comb.get("name") == "rewrite" else COMBINE_OTHER)
                base["props"] = self._props_rec(op["props"], code)
        else:
            raise ValueError(f"unsupported op type {t}")
        self.recs.append(base)

    def add_doc(self, seed_text, msgs, clients=None):
        """clients: long id -> short id already known for this document (a loaded summary's
        writers, snapshot.SnapshotBatch.clients); new ids continue after them."""
        enc = DocEncoder(self, clients)
        self.clients.append(enc.short)
        s = seed_text.encode("utf-16-le")
        self.seed.extend(np.frombuffer(s, dtype="<u2").tolist())
        self.seed_off.append(len(self.seed))
        for msg in msgs:
            if msg.get("type", "op") != "op":
                enc.client(msg["clientId"])
                self.recs.append(dict(seq=msg["sequenceNumber"], ref_seq=msg["referenceSequenceNumber"],
                                      min_seq=msg["minimumSequenceNumber"], client=enc.client(msg["clientId"]),
                                      kind=OP_NOOP, flags=0, props=NO_PROPS, pos1=0, pos2=0, payload=0))
                continue
            op = msg["contents"]
            if op["type"] == 3:        # GROUP
                members = op["ops"]
                for i, m in enumerate(members):
                    self._op(enc, msg, m, i + 1 < len(members))
            else:
                self._op(enc, msg, op, False)
        self.doc_off.append(len(self.recs))

    def arrays(self):
        ops = np.zeros(len(self.recs), dtype=OP_DTYPE)
        for i, r in enumerate(self.recs):
            for k, v in r.items():
                ops[i][k] = v
        return dict(ops=ops,
                    doc_off=np.asarray(self.doc_off, dtype=np.int64),
                    text=np.asarray(self.text if self.text else [0], dtype=np.uint16),
                    props=np.asarray(self.props if self.props else [0], dtype=np.uint32),
                    seed_off=np.asarray(self.seed_off, dtype=np.int64),
                    seed=np.asarray(self.seed if self.seed else [0], dtype=np.uint16))


def compact_msgs_to_dicts(msgs):
    """Reference-harness compact log [[k, seq, ref, msn, op], ...] -> message dicts."""
    out = []
    for rec in msgs:
        k, t, r, m, op = rec[:5]
        typ = rec[5] if len(rec) > 5 else "op"
        out.append(dict(clientId=f"client-{k}", sequenceNumber=t, referenceSequenceNumber=r,
                        minimumSequenceNumber=m, type=typ, contents=op))
    return out


def gen_thresholds(cfg):
    frac = lambda p: int(p * 4294967296.0)   # noqa: E731  (floor for p >= 0, as Math.floor)
    return dict(p_insert=frac(cfg["p_insert"]), p_insert_remove=frac(cfg["p_insert"] + cfg["p_remove"]),
                p_newline=frac(cfg["p_newline"]), p_len_continue=frac(cfg["p_len_continue"]),
                p_insert_props=frac(cfg["p_insert_props"]), p_null=frac(cfg["p_null"]))
