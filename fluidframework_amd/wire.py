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
F_GROUP_MORE, F_MARKER, F_LOCAL, F_ACK = 1, 2, 8, 16
NO_PROPS = 0xFFFFFFFF
VAL_NULL = 0xFFFFFFFF
VAL_UNDEF = 0xFFFFFFFE          # a key set to the JS value undefined
VAL_FALSY_BIT = 0x80000000
VAL_NOMATCH_BIT = 0x40000000    # matchProperties never finds the value equal (NaN, undefined inside)
VAL_ID_MASK = 0x3FFFFFFF
COMBINE_NONE, COMBINE_REWRITE, COMBINE_OTHER, COMBINE_TABLE = 0, 1, 2, 3

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


class _JsValue:
    """The JS values JSON cannot hold that non-rewrite combining ops leave in property sets
    (SURVEY Q4): NaN (`incr`) and undefined (`consensus`' {value: undefined, seq}, unknown
    combining-op names on an absent key)."""

    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return self.name


NAN = _JsValue("NaN")
UNDEF = _JsValue("undefined")


def from_fixture(v):
    """Fixture encoding of JS-only values ({"$nan": 1}, {"$undef": 1}; oracle/ref_harness.mjs
    jsReplacer) -> NAN / UNDEF."""
    if isinstance(v, dict):
        if len(v) == 1 and "$nan" in v:
            return NAN
        if len(v) == 1 and "$undef" in v:
            return UNDEF
        return {k: from_fixture(x) for k, x in v.items()}
    if isinstance(v, list):
        return [from_fixture(x) for x in v]
    return v


def _has_js_value(v):
    if v is NAN or v is UNDEF:
        return True
    if isinstance(v, dict):
        return any(_has_js_value(x) for x in v.values())
    if isinstance(v, list):
        return any(_has_js_value(x) for x in v)
    return False


def _js_number(x):
    """A number as a JS Number (one double type: 1, 1.0 and 1e0 are the same value)."""
    try:
        f = float(x)
    except OverflowError:          # an integer lexeme beyond the double range: +-Infinity
        f = float("inf") if x > 0 else float("-inf")
    if f.is_integer() and abs(f) < 1e21:
        return str(int(f))
    return repr(f)


def canonical_json(v):
    """Canonical form used to intern property values: matchProperties
    (MT/properties.ts:61-92) compares with === (numbers as JS Numbers) and nested objects
    structurally, ignoring key order."""
    if v is None or isinstance(v, (bool, str)):
        return json.dumps(v, ensure_ascii=False)
    if isinstance(v, int):
        return str(v) if -2 ** 53 < v < 2 ** 53 else _js_number(v)
    if isinstance(v, float):
        return _js_number(v)
    if v is NAN or v is UNDEF:
        return v.name
    if isinstance(v, list):
        return "[" + ",".join(canonical_json(x) for x in v) + "]"
    return "{" + ",".join(json.dumps(k, ensure_ascii=False) + ":" + canonical_json(v[k]) for k in sorted(v)) + "}"


def js_falsy(v):
    return (v is None or v is False or v == "" or v is NAN or v is UNDEF or
            (isinstance(v, (int, float)) and not isinstance(v, bool) and v == 0))


def js_nomatch(v):
    """matchProperties(a, a) is false for a property set holding v: NaN !== NaN, and an
    undefined member fails `b[key] === undefined` (also inside nested objects)."""
    return _has_js_value(v)


def _js_num_str(x):
    if isinstance(x, bool):
        return "true" if x else "false"
    if isinstance(x, float) and x.is_integer() and abs(x) < 1e21:
        return str(int(x))
    return str(x)


def _js_to_string(v):
    """String(v) for the values JSON can carry (ToPrimitive of objects / arrays)."""
    if v is None or v is UNDEF:
        return ""
    if v is NAN:
        return "NaN"
    if isinstance(v, str):
        return v
    if isinstance(v, (bool, int, float)):
        return _js_num_str(v)
    if isinstance(v, list):
        return ",".join("" if x is None or x is UNDEF else _js_to_string(x) for x in v)
    return "[object Object]"


class Unsupported(ValueError):
    pass


def js_combine(op, cur, seq):
    """Properties.combine(op, currentValue, undefined, seq) (MT/properties.ts:26-59) as
    SegmentPropertiesManager.addProperties calls it for a non-rewrite combining op
    (MT/segmentPropertiesManager.ts:93-107: the new value is never passed in)."""
    if cur is UNDEF:
        cur = op.get("defaultValue", UNDEF)
    name = op.get("name")
    if name == "incr":
        if cur is UNDEF or cur is None or cur is NAN or isinstance(cur, (bool, int, float)):
            r = NAN                                     # x + undefined
        else:
            r = _js_to_string(cur) + "undefined"
        mv = op.get("minValue")
        if mv and not (isinstance(mv, (int, float)) and not isinstance(mv, bool)):
            raise Unsupported("incr with a non-numeric minValue")
        return r                                        # NaN / "...undefined" < n is false
    if name == "consensus":
        if cur is UNDEF:
            return {"value": UNDEF, "seq": seq}
        if cur is None:
            raise Unsupported("consensus over null (the reference throws a TypeError)")
        if isinstance(cur, dict) and cur.get("seq") == -1:
            raise Unsupported("consensus over a shared {seq: -1} value (mutated in place)")
        return cur
    return cur


class Interner:
    """Property key / value interning shared by every document of a batch."""

    def __init__(self, synthetic=False):
        self.keys, self.key_ids = [], {}
        self.vals, self.val_ids = [], {}
        self.synthetic = synthetic
        # the values each key can hold (ids without flag bits), for combining-op tables:
        # every (key, value) written by a record, plus values of unknown key (decoded summaries)
        self.key_vals, self.unkeyed = {}, set()

    def note(self, kid, vid):
        if not self.synthetic and vid not in (VAL_NULL, VAL_UNDEF):
            self.key_vals.setdefault(kid, set()).add(vid & VAL_ID_MASK)

    def note_unkeyed(self, vid):
        if not self.synthetic and vid not in (VAL_NULL, VAL_UNDEF):
            self.unkeyed.add(vid & VAL_ID_MASK)

    def held_values(self, kids):
        """Ids of every value one of the keys `kids` can hold, ascending."""
        out = set(self.unkeyed)
        for k in kids:
            out |= self.key_vals.get(k, set())
        return sorted(out)

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
        if v is UNDEF:
            return VAL_UNDEF
        if self.synthetic:
            return int(v) | (VAL_FALSY_BIT if int(v) == 0 else 0)
        c = canonical_json(v)
        i = self.val_ids.get(c)
        if i is None:
            i = len(self.vals)
            self.val_ids[c] = i
            self.vals.append(v)
        return i | (VAL_FALSY_BIT if js_falsy(v) else 0) | (VAL_NOMATCH_BIT if js_nomatch(v) else 0)

    def key_name(self, kid):
        return f"k{kid}" if self.synthetic else self.keys[kid]

    def val_value(self, vid):
        if vid == VAL_NULL:
            return None
        if vid == VAL_UNDEF:
            return UNDEF
        if self.synthetic:
            return vid & ~VAL_FALSY_BIT
        return self.vals[vid & ~(VAL_FALSY_BIT | VAL_NOMATCH_BIT)]


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
            kid, vid = self.interner.key(k), self.interner.val(v)
            self.interner.note(kid, vid)
            self.props.append(kid)
            self.props.append(vid)
        return off

    def _combine_rec(self, props, comb, seq):
        """A non-rewrite combining op's record: the keys, then the transform of
        every value one of the op's keys can hold at this point (Interner.held_values: the
        values written under those keys so far, plus decoded summaries' values) --
        [n, new value of an absent key, (old, new) x n] -- as combine(op, old, undefined, seq)
        yields it; new = VAL_NULL deletes the key.  The results become values those keys can
        hold.  Unsupported results (the reference throws, or mutates a shared value) keep
        COMBINE_OTHER: the document fails with MT_DOC_UNSUPPORTED."""
        it = self.interner
        if it.synthetic:
            return self._props_rec(props, COMBINE_OTHER)
        kids = [it.key(k) for k in props]
        try:
            absent = it.val(js_combine(comb, UNDEF, seq))
            pairs = []
            for i in it.held_values(kids):
                v = it.vals[i]
                pairs.append((it.val(v), it.val(js_combine(comb, v, seq))))
        except Unsupported:
            return self._props_rec(props, COMBINE_OTHER)
        off = self._props_rec(props, COMBINE_TABLE)
        for kid in kids:
            it.note(kid, absent)
            for _, n in pairs:
                it.note(kid, n)
        self.props.append(len(pairs))
        self.props.append(absent)
        for o, n in pairs:
            self.props.append(o)
            self.props.append(n)
        return off

    def _text(self, s):
        off = len(self.text)
        b = s.encode("utf-16-le", errors="surrogatepass")   # (JS strings may hold lone surrogates)
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
                if comb and comb.get("name") != "rewrite":
                    base["props"] = self._combine_rec(op["props"], comb, msg["sequenceNumber"])
                else:
                    base["props"] = self._props_rec(op["props"], COMBINE_REWRITE if comb else COMBINE_NONE)
        else:
            raise ValueError(f"unsupported op type {t}")
        self.recs.append(base)

    def add_doc(self, seed_text, msgs, clients=None):
        """clients: long id -> short id already known for this document (a loaded summary's
        writers, snapshot.SnapshotBatch.clients); new ids continue after them."""
        enc = DocEncoder(self, clients)
        self.clients.append(enc.short)
        s = seed_text.encode("utf-16-le", errors="surrogatepass")
        self.seed.extend(np.frombuffer(s, dtype="<u2").tolist())
        self.seed_off.append(len(self.seed))
        for msg in msgs:
            if msg.get("type", "op") != "op":
                enc.client(msg["clientId"])
                self.recs.append(dict(seq=msg["sequenceNumber"], ref_seq=msg["referenceSequenceNumber"],
                                      min_seq=msg["minimumSequenceNumber"], client=enc.client(msg["clientId"]),
                                      kind=OP_NOOP, flags=0, props=NO_PROPS, pos1=0, pos2=0, payload=0))
                continue
            self._msg(enc, msg)
        self.doc_off.append(len(self.recs))

    def _msg(self, enc, msg, flags=0):
        op = msg["contents"]
        if op["type"] == 3 and not op["ops"]:
            # an empty GROUP applies nothing; applyMsg still updates seq/msn (MT/client.ts:818)
            self.recs.append(dict(seq=msg["sequenceNumber"], ref_seq=msg["referenceSequenceNumber"],
                                  min_seq=msg["minimumSequenceNumber"], client=enc.client(msg["clientId"]),
                                  kind=OP_NOOP, flags=0, props=NO_PROPS, pos1=0, pos2=0, payload=0))
            return
        members = op["ops"] if op["type"] == 3 else [op]      # GROUP
        for i, m in enumerate(members):
            self._op(enc, msg, m, i + 1 < len(members))
            self.recs[-1]["flags"] |= flags

    def add_live_doc(self, seed_text, entries, clients):
        """One document of a live-client handle (mt_options.live_client).  entries, in order:
        ("local", op) -- the local client's own op as insertSegmentLocal / removeRangeLocal /
        annotateRangeLocal return it (MT_F_LOCAL); ("ack", msg) -- the sequenced echo of one
        (MT_F_ACK, one record per GROUP member); ("msg", msg) -- any other sequenced message.
        clients maps long ids to short ids, the local client's ids to 0."""
        enc = DocEncoder(self, clients)
        self.clients.append(enc.short)
        s = seed_text.encode("utf-16-le", errors="surrogatepass")
        self.seed.extend(np.frombuffer(s, dtype="<u2").tolist())
        self.seed_off.append(len(self.seed))
        local_key = next((k for k, v in enc.short.items() if v == 0), None)
        for what, x in entries:
            if what == "local":
                m = dict(clientId=local_key, sequenceNumber=-1, referenceSequenceNumber=0,
                         minimumSequenceNumber=0, contents=x)
                self._msg(enc, m, F_LOCAL)
            elif what == "ack":
                self._msg(enc, x, F_ACK)
            elif x.get("type", "op") != "op":
                self.recs.append(dict(seq=x["sequenceNumber"], ref_seq=x["referenceSequenceNumber"],
                                      min_seq=x["minimumSequenceNumber"], client=enc.client(x["clientId"]),
                                      kind=OP_NOOP, flags=0, props=NO_PROPS, pos1=0, pos2=0, payload=0))
            else:
                self._msg(enc, x)
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
