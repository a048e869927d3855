"""SnapshotV1 summaries (cold catch-up, config C5) on the host side of the C ABI.

Decoding mirrors the reference loader: ``SnapshotLoader.initialize/loadHeader/loadBody/
specToSegment`` (MT/snapshotLoader.ts:36-228), ``SnapshotV1.processChunk`` (MT/snapshotV1.ts:
266-277) and ``toLatestVersion`` / ``buildHeaderMetadataForLegecyChunk``
(MT/snapshotChunks.ts:136-188).  Chunk text is parsed here (``JSON.parse`` in the
reference); the tree is rebuilt on the GPU from fixed-width segment records
(``mt_seg_rec``, include/mt_types.h) by ``mt_load_snapshots``.

Encoding (``encode_chunks``) mirrors ``SnapshotV1.emit/getSeqLengthSegs``
(MT/snapshotV1.ts:59-154) for segment records extracted on the GPU
(``mt_extract_snapshots`` = ``SnapshotV1.extractSync`` :156-252).

MT/ = packages/dds/merge-tree/src/ in the reference.
"""
import json

import numpy as np

from .wire import Interner

SEG_DTYPE = np.dtype([
    ("len", "<i4"), ("seq", "<i4"), ("removed_seq", "<i4"), ("payload", "<u4"), ("props", "<u4"),
    ("client", "<i2"), ("removed_client", "<i2"), ("flags", "u1"), ("_pad", "u1", (7,)),
])
assert SEG_DTYPE.itemsize == 32

NON_COLLAB = -2              # NonCollabClient            MT/constants.ts:15
UNIVERSAL_SEQ = 0            # UniversalSequenceNumber    MT/constants.ts:11
RSEQ_NONE = -2 ** 31         # removedSeq === undefined
NO_PROPS = 0xFFFFFFFF
F_MARKER = 2
SEG_MERGE_INFO = 0x10        # mt_types.h MT_SEG_MERGE_INFO
SEG_HAS_SEQ = 0x20           # mt_types.h MT_SEG_HAS_SEQ
HEADER = "header"            # SnapshotLegacy.header      MT/snapshotlegacy.ts
BODY = "body"                # SnapshotLegacy.body
CHUNK_SIZE = 10000           # SnapshotV1.chunkSize       MT/snapshotV1.ts:42


class SnapshotError(ValueError):
    pass


def _legacy_header_metadata(path, chunk):
    """buildHeaderMetadataForLegecyChunk MT/snapshotChunks.ts:169-188."""
    if path != HEADER:
        return None
    if chunk.get("headerMetadata") is not None:
        return chunk["headerMetadata"]
    ids = [{"id": HEADER}]
    if chunk["chunkLengthChars"] < chunk["totalLengthChars"]:
        ids.append({"id": BODY})
    return dict(orderedChunkMetadata=ids, minSequenceNumber=chunk.get("chunkMinSequenceNumber"),
                sequenceNumber=chunk.get("chunkSequenceNumber"), totalLength=chunk["totalLengthChars"],
                totalSegmentCount=chunk["totalSegmentCount"])


def to_latest_version(path, chunk):
    """toLatestVersion MT/snapshotChunks.ts:136-167."""
    v = chunk.get("version")
    if v == "1":
        return chunk
    if v is None:
        return dict(version="1", length=chunk["chunkLengthChars"], segmentCount=chunk["chunkSegmentCount"],
                    headerMetadata=_legacy_header_metadata(path, chunk), segments=chunk["segmentTexts"],
                    startIndex=chunk["chunkStartSegmentIndex"])
    raise SnapshotError(f"Unsupported chunk path: {path} version: {v}")


def tree_chunks(tree):
    """Blob path -> contents of a summary ITree.  A SharedString summary nests the
    merge-tree blobs under "content" (sequence.ts snapshot); SnapshotV1.emit puts them at
    the top.  (MockStorage reads blobs the same way, test-runtime-utils/src/mockStorage.ts.)"""
    content = next((e for e in tree["entries"] if e["type"] == "Tree" and e["path"] == "content"), None)
    t = content["value"] if content else tree
    return {e["path"]: e["value"]["contents"] for e in t["entries"] if e["type"] == "Blob"}


def has_merge_info(spec):
    """hasMergeInfo MT/snapshotChunks.ts:72-74."""
    return isinstance(spec, dict) and "json" in spec


class SnapshotDoc:
    """One decoded summary: the header and body segment specs in order, the collaboration
    window from the header metadata, and the legacy catch-up messages (if any)."""

    def __init__(self, header_specs, body_specs, min_seq, cur_seq, catchup=()):
        self.header_specs = header_specs
        self.body_specs = body_specs
        self.min_seq = min_seq
        self.cur_seq = cur_seq
        self.catchup = list(catchup)


def _blob_text(v):
    """A blob's bytes as the JS string the reference parses: fromBase64ToUtf8 is
    Buffer.toString("utf8"), which replaces every maximal ill-formed subsequence by U+FFFD --
    the same rule as Python's "replace" handler."""
    return v.decode("utf-8", errors="replace") if isinstance(v, (bytes, bytearray)) else v


def decode_chunks(chunks):
    """SnapshotLoader.initialize (MT/snapshotLoader.ts:36-84, 120-228) over blob contents
    (JSON text; the reference base64-decodes first, MT/snapshotV1.ts:274)."""
    if HEADER not in chunks:
        raise SnapshotError("header blob missing")
    header = to_latest_version(HEADER, json.loads(_blob_text(chunks[HEADER])))
    meta = header.get("headerMetadata")
    if meta is None:
        raise SnapshotError("header metadata not available")
    seq = meta["sequenceNumber"]
    msn = meta["minSequenceNumber"] if meta.get("minSequenceNumber") is not None else seq
    body = []
    ordered = meta["orderedChunkMetadata"]
    if header["segmentCount"] != meta["totalSegmentCount"]:        # loadBody :170-172
        for md in ordered[1:]:
            ch = to_latest_version(md["id"], json.loads(_blob_text(chunks[md["id"]])))
            body += ch["segments"]
    catchup = []
    blobs = list(chunks)
    if len(blobs) == len(ordered) + 1:                               # :72-79
        rest = [b for b in blobs if b not in {m["id"] for m in ordered}]
        if len(rest) != 1:
            raise SnapshotError(f"There should be only one blob with catch up ops: {len(rest)}")
        catchup = json.loads(_blob_text(chunks[rest[0]]))
    elif len(blobs) != len(ordered):
        raise SnapshotError("Unexpected blobs in snapshot")
    return SnapshotDoc(header["segments"], body, msn, seq, catchup)


class SnapshotBatch:
    """Segment records of many summaries for mt_load_snapshots.

    Short client ids follow Client.getOrAddShortClientId's first-seen order over
    specToSegment (header specs, then body specs; MT/snapshotLoader.ts:86-118), with the
    loading observer as id 0 (the engine's ids only need to be injective; ids 1..64 index
    the overlap masks).  ``clients[d]`` is the map to continue with for the catch-up ops
    (wire.Batch.add_doc(..., clients=...))."""

    def __init__(self, interner=None):
        self.interner = interner or Interner()
        self.segs = []
        self.text = []
        self.props = []
        self.doc_off = [0]
        self.n_header = []
        self.min_seq = []
        self.cur_seq = []
        self.clients = []

    def _short(self, short, long_id):
        s = short.get(long_id)
        if s is None:
            s = short[long_id] = len(short) + 1
        return s

    def _props(self, props):
        off = len(self.props)
        items = list(props.items())
        self.props.append(len(items))
        for k, v in items:
            kid, vid = self.interner.key(k), self.interner.val(v)
            self.interner.note(kid, vid)
            self.props.append(kid)
            self.props.append(vid)
        return off

    def _rec(self, spec, short):
        """specToSegment MT/snapshotLoader.ts:86-118 (+ SharedStringFactory.segmentFromSpec,
        SEQ/sequenceFactory.ts:31-37)."""
        r = dict(len=0, seq=UNIVERSAL_SEQ, removed_seq=RSEQ_NONE, payload=0, props=NO_PROPS,
                 client=NON_COLLAB, removed_client=0, flags=0)
        js = spec["json"] if has_merge_info(spec) else spec
        if isinstance(js, str):
            text, props = js, None
        elif isinstance(js, dict) and "text" in js:
            text, props = js["text"], js.get("props")
        elif isinstance(js, dict) and "marker" in js:
            text, props = None, js.get("props")
            r["flags"] = F_MARKER
            r["payload"] = int(js["marker"].get("refType", 0))
            r["len"] = 1
        else:
            raise SnapshotError(f"unsupported segment spec {js!r}")
        if text is not None:
            b = text.encode("utf-16-le", errors="surrogatepass")
            r["payload"] = len(self.text)
            self.text.extend(np.frombuffer(b, dtype="<u2").tolist())
            r["len"] = len(b) // 2
        if isinstance(props, dict):    # TextSegment.make / Marker.make `if (props)`: {} too (Q5)
            r["props"] = self._props(props)
        if has_merge_info(spec):
            r["flags"] |= SEG_MERGE_INFO | (SEG_HAS_SEQ if spec.get("seq") is not None else 0)
            if spec.get("client") is not None:
                r["client"] = self._short(short, spec["client"])
            if spec.get("seq") is not None:
                r["seq"] = spec["seq"]
            if spec.get("removedSeq") is not None:
                r["removed_seq"] = spec["removedSeq"]
            if spec.get("removedClient") is not None:
                r["removed_client"] = self._short(short, spec["removedClient"])
        return r

    def add_doc(self, snap):
        short = {}
        for spec in snap.header_specs:
            self.segs.append(self._rec(spec, short))
        self.n_header.append(len(snap.header_specs))
        for spec in snap.body_specs:
            self.segs.append(self._rec(spec, short))
        self.doc_off.append(len(self.segs))
        self.min_seq.append(snap.min_seq)
        self.cur_seq.append(snap.cur_seq)
        self.clients.append(short)
        return short

    def arrays(self):
        segs = np.zeros(len(self.segs), dtype=SEG_DTYPE)
        for i, r in enumerate(self.segs):
            for k, v in r.items():
                segs[i][k] = v
        return dict(segs=segs, doc_off=np.asarray(self.doc_off, dtype=np.int64),
                    n_header=np.asarray(self.n_header, dtype=np.int32),
                    text=np.asarray(self.text if self.text else [0], dtype=np.uint16),
                    props=np.asarray(self.props if self.props else [0], dtype=np.uint32),
                    min_seq=np.asarray(self.min_seq, dtype=np.int32),
                    cur_seq=np.asarray(self.cur_seq, dtype=np.int32))


# ---------------------------------------------------------------- emission
def js_key_order(items):
    """V8 own-key order of an object built by insertion: integer-like keys ascending first."""
    def is_index(k):
        return k.isdigit() and (k == "0" or not k.startswith("0")) and int(k) < 4294967295
    ints = sorted((kv for kv in items if is_index(kv[0])), key=lambda kv: int(kv[0]))
    return ints + [kv for kv in items if not is_index(kv[0])]


def js_stringify(v):
    """JSON.stringify for the values a summary holds (key order as given)."""
    return json.dumps(v, separators=(",", ":"), ensure_ascii=False)


def record_specs(recs, text, props, interner, client_names):
    """ISegment.toJSONObject (MT/textSegment.ts:48-54, MT/mergeTree.ts:478-482, 690-694) and
    the merge-info wrapper of extractSync (MT/snapshotV1.ts:222-241) for extracted records.
    Returns (specs, lengths)."""
    specs, lengths = [], []
    for r in recs:
        props_obj = None
        if int(r["props"]) != NO_PROPS:
            o = int(r["props"])
            n = int(props[o])
            items = [(interner.key_name(int(props[o + 1 + 2 * j])), interner.val_value(int(props[o + 2 + 2 * j])))
                     for j in range(n)]
            props_obj = dict(js_key_order(items))
        if r["flags"] & F_MARKER:
            js = {"marker": {"refType": int(r["payload"])}}
            if props_obj is not None:
                js["props"] = props_obj
        else:
            p0, ln = int(r["payload"]), int(r["len"])
            t = np.asarray(text[p0:p0 + ln], dtype="<u2").tobytes().decode("utf-16-le", errors="surrogatepass")
            js = t if props_obj is None else {"text": t, "props": props_obj}
        if r["flags"] & SEG_MERGE_INFO:
            raw = {"json": js}
            if r["flags"] & SEG_HAS_SEQ:
                raw["seq"] = int(r["seq"])
                raw["client"] = client_names[int(r["client"])]
            if int(r["removed_seq"]) != RSEQ_NONE:
                raw["removedSeq"] = int(r["removed_seq"])
                raw["removedClient"] = client_names[int(r["removed_client"])]
            js = raw
        specs.append(js)
        lengths.append(int(r["len"]))
    return specs, lengths


def encode_chunks(specs, lengths, min_seq, cur_seq, chunk_size=CHUNK_SIZE):
    """SnapshotV1.emit (MT/snapshotV1.ts:59-154): chunks of >= chunk_size units
    (getSeqLengthSegs), the first is the header with the metadata; {path: JSON text} as
    serializeAsMaxSupportedVersion writes it (JSON.stringify of the v1 chunk)."""
    chunks = []
    total_n = total_len = 0
    while True:
        seg, length, count = [], 0, 0
        while length < chunk_size and total_n + count < len(specs):
            seg.append(specs[total_n + count])
            length += lengths[total_n + count]
            count += 1
        chunks.append(dict(version="1", segmentCount=count, length=length, segments=seg, startIndex=total_n))
        total_n += count
        total_len += length
        if not total_n < len(specs):
            break
    head = chunks[0]
    ids = [{"id": HEADER}] + [{"id": f"{BODY}_{i}"} for i in range(len(chunks) - 1)]
    head["headerMetadata"] = dict(minSequenceNumber=min_seq, sequenceNumber=cur_seq, orderedChunkMetadata=ids,
                                  totalLength=total_len, totalSegmentCount=total_n)
    out = {HEADER: js_stringify(head)}
    for i, ch in enumerate(chunks[1:]):
        out[f"{BODY}_{i}"] = js_stringify(ch)
    return out


def load_arrays_from_extract(counts, recs, text, props, min_seq, cur_seq, chunk_size=CHUNK_SIZE):
    """mt_extract_snapshots output -> mt_load_snapshots input without a JSON round trip:
    offsets rebased to the concatenated arenas, and the header/body split emit() would make
    (a record is in the header chunk iff the lengths before it sum to < chunk_size,
    getSeqLengthSegs MT/snapshotV1.ts:59-81)."""
    counts = np.asarray(counts, dtype=np.int64)
    n_docs = len(counts)
    doc_off = np.zeros(n_docs + 1, dtype=np.int64)
    doc_off[1:] = np.cumsum(counts[:, 0])
    t_off = np.concatenate([[0], np.cumsum(counts[:, 1])[:-1]]).astype(np.int64)
    p_off = np.concatenate([[0], np.cumsum(counts[:, 2])[:-1]]).astype(np.int64)
    segs = np.array(recs, copy=True)
    doc_of = np.repeat(np.arange(n_docs), counts[:, 0])
    text_rec = (segs["flags"] & F_MARKER) == 0
    segs["payload"][text_rec] += t_off[doc_of[text_rec]].astype(np.uint32)
    has_p = segs["props"] != NO_PROPS
    segs["props"][has_p] += p_off[doc_of[has_p]].astype(np.uint32)
    lens = segs["len"].astype(np.int64)
    cinc = np.cumsum(lens)
    start = np.zeros(n_docs, dtype=np.int64)                      # lengths before each document
    if len(cinc):
        nz = doc_off[:-1] > 0
        start[nz] = cinc[doc_off[:-1][nz] - 1]
    before = (cinc - lens) - start[doc_of]                       # within the document
    in_header = before < chunk_size
    n_header = np.zeros(n_docs, dtype=np.int32)
    np.add.at(n_header, doc_of, in_header.astype(np.int32))
    return dict(segs=segs, doc_off=doc_off, n_header=n_header, text=text, props=props,
                min_seq=np.asarray(min_seq, dtype=np.int32), cur_seq=np.asarray(cur_seq, dtype=np.int32))
