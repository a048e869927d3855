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


def decode_chunks(chunks):
    """SnapshotLoader.initialize (MT/snapshotLoader.ts:36-84, 120-228) over blob contents
    (JSON text; the reference base64-decodes first, MT/snapshotV1.ts:274)."""
    if HEADER not in chunks:
        raise SnapshotError("header blob missing")
    header = to_latest_version(HEADER, json.loads(chunks[HEADER]))
    meta = header.get("headerMetadata")
    if meta is None:
        raise SnapshotError("header metadata not available")
    seq = meta["sequenceNumber"]
    msn = meta["minSequenceNumber"] if meta.get("minSequenceNumber") is not None else seq
    body = []
    ordered = meta["orderedChunkMetadata"]
    if header["segmentCount"] != meta["totalSegmentCount"]:        # loadBody :170-172
        for md in ordered[1:]:
            ch = to_latest_version(md["id"], json.loads(chunks[md["id"]]))
            body += ch["segments"]
    catchup = []
    blobs = list(chunks)
    if len(blobs) == len(ordered) + 1:                               # :72-79
        rest = [b for b in blobs if b not in {m["id"] for m in ordered}]
        if len(rest) != 1:
            raise SnapshotError(f"There should be only one blob with catch up ops: {len(rest)}")
        catchup = json.loads(chunks[rest[0]])
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
            self.props.append(self.interner.key(k))
            self.props.append(self.interner.val(v))
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
