"""Native host encode of sequenced messages (include/mt_snapshot.h ``mt_opdec_*``, in
libmtsnapdec.so): ISequencedDocumentMessage JSON (PD/protocol.ts:132-172) carrying IMergeTree
ops (MT/ops.ts:63-110) -> the op records, text and property arenas ``mt_batch_upload`` takes.

The output equals ``wire.Batch.add_doc`` (the Python encoder, mirrored by the JS facade's
js/encode.js) on the same messages, property keys / values numbered in the caller's
``wire.Interner`` in first-seen document order (tests/test_snapdec.py compares the two on the
reference's fixtures).  JSON is parsed and encoded on ``threads`` host threads in C++.  Not
covered natively -- the caller encodes with ``wire.Batch``: non-rewrite combining ops (their
transform tables need every value the keys held before, ``Batch._combine_rec``) and documents
that continue a known short-id map (``Batch.add_doc(clients=...)``).
"""
import ctypes
import json

import numpy as np

from . import snapdec
from .snapdec import _p, _text
from .wire import OP_DTYPE, VAL_FALSY_BIT, VAL_NULL, Interner

NO_PROPS = 0xFFFFFFFF


class EncodeError(ValueError):
    pass


class MessageDecoder:
    """decode(docs) -> (arrays, clients): ``arrays`` as ``wire.Batch.arrays()`` (ops, doc_off,
    text, props; seed_off / seed from ``seeds``), ``clients[d]`` the document's {long id:
    short id} map.  ``docs[d]`` is one document's messages: a JSON array text (str / bytes)
    or a list of message dicts (serialised here)."""

    def __init__(self, interner=None, threads=8):
        self.interner = interner or Interner()
        self.threads = threads
        self.lib = snapdec.load()
        self.h = self.lib.mt_snapdec_create(1 if self.interner.synthetic else 0)
        self._kmap, self._vmap = [], []   # the decoder's ids -> the interner's

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.mt_snapdec_destroy(self.h)
            self.h = None

    @staticmethod
    def pack(docs):
        out = []
        for m in docs:
            if isinstance(m, (bytes, bytearray)):
                out.append(bytes(m))
            elif isinstance(m, str):
                out.append(m.encode("utf-8", errors="surrogatepass"))
            else:
                # (escaped non-ASCII: a lone surrogate is a \u escape, as JSON.stringify writes it)
                out.append(json.dumps(m, separators=(",", ":")).encode("ascii"))   # (as JSON.stringify)
        return out

    def decode_packed(self, blobs, alloc=None, doc_off_out=None):
        """mt_opdec_decode + fetch over already serialised documents: the arrays with the
        decoder's own property ids (remap() numbers them in the interner).  alloc(n, dtype):
        where the op / text / property arrays go (reused buffers: no page faults on fresh
        memory); doc_off_out: the (n + 1) offsets' array."""
        n = len(blobs)
        jp = (ctypes.c_char_p * max(n, 1))(*blobs)
        jl = np.asarray([len(x) for x in blobs] or [0], dtype=np.uint64)
        if self.lib.mt_opdec_decode(self.h, n, jp, _p(jl), self.threads) != 0:
            raise EncodeError(self.lib.mt_snapdec_error(self.h).decode())
        no, nt, npr = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self.lib.mt_opdec_sizes(self.h, ctypes.byref(no), ctypes.byref(nt), ctypes.byref(npr))
        alloc = alloc or (lambda m, dt: np.empty(m, dtype=dt))
        out = dict(ops=alloc(no.value, OP_DTYPE),
                   doc_off=doc_off_out if doc_off_out is not None else np.zeros(n + 1, dtype=np.int64),
                   text=alloc(nt.value, np.uint16) if nt.value else np.zeros(1, dtype=np.uint16),
                   props=alloc(npr.value, np.uint32) if npr.value else np.zeros(1, dtype=np.uint32))
        self.lib.mt_opdec_fetch(self.h, _p(out["doc_off"]), _p(out["ops"]), _p(out["text"]), _p(out["props"]))
        return out

    def remap(self, out):
        """The decoder's key / value ids -> the interner's (first-seen order kept), with
        Interner.note for every (key, value) a record writes, as Batch._props_rec does."""
        it, lib = self.interner, self.lib
        if it.synthetic:
            return
        for i in range(len(self._kmap), lib.mt_snapdec_num_keys(self.h)):
            self._kmap.append(it.key(_text(lib.mt_snapdec_key, self.h, i)))
        for i in range(len(self._vmap), lib.mt_snapdec_num_values(self.h)):
            self._vmap.append(it.val(json.loads(_text(lib.mt_snapdec_value, self.h, i))) & (VAL_FALSY_BIT - 1))
        starts = out["ops"]["props"][out["ops"]["props"] != NO_PROPS].astype(np.int64)
        if not len(starts):
            return
        p = out["props"]
        cnt = (p[starts] & 0xFFFF).astype(np.int64)
        tot = int(cnt.sum())
        if not tot:
            return
        km, vm = np.asarray(self._kmap, dtype=np.uint32), np.asarray(self._vmap, dtype=np.uint32)
        first = np.repeat(np.cumsum(cnt) - cnt, cnt)
        kpos = np.repeat(starts + 1, cnt) + 2 * (np.arange(tot) - first)
        p[kpos] = km[p[kpos]]
        v = p[kpos + 1]
        live = v != VAL_NULL
        falsy = np.uint32(VAL_FALSY_BIT)
        v[live] = vm[v[live] & ~falsy] | (v[live] & falsy)
        p[kpos + 1] = v
        for kid, vid in np.unique(np.stack([p[kpos], p[kpos + 1]], axis=1), axis=0).tolist():
            it.note(int(kid), int(vid))

    def clients(self, n):
        out = []
        for d in range(n):
            ids = json.loads(_text(self.lib.mt_opdec_doc_clients, self.h, d))
            out.append({c: k + 1 for k, c in enumerate(ids)})
        return out

    def decode(self, docs, seeds=None):
        blobs = self.pack(docs)
        out = self.decode_packed(blobs)
        self.remap(out)
        seed = [np.frombuffer(s.encode("utf-16-le", errors="surrogatepass"), dtype="<u2")
                for s in (seeds or [""] * len(blobs))]
        out["seed_off"] = np.concatenate([[0], np.cumsum([len(x) for x in seed])]).astype(np.int64)
        out["seed"] = np.concatenate(seed).astype(np.uint16) if out["seed_off"][-1] else np.zeros(1, dtype=np.uint16)
        return out, self.clients(len(blobs))
