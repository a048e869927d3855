"""ctypes binding of the native summary decoder (include/mt_snapshot.h, libmtsnapdec.so).

Same output as ``snapshot.decode_chunks`` + ``SnapshotBatch`` (the Python restatement of
SnapshotLoader.initialize / loadHeader / loadBody / specToSegment, MT/snapshotLoader.ts:
36-228): mt_seg_rec records and arenas for ``mt_load_snapshots``, property keys / values
numbered in the caller's ``wire.Interner`` (first-seen, document order) and the short client
maps.  Blob JSON is parsed on ``threads`` host threads in C++ (the reference's JSON.parse
step).
"""
import ctypes
import json
import os
from collections.abc import Sequence

import numpy as np

from .snapshot import NO_PROPS, SEG_DTYPE, SnapshotError
from .wire import VAL_FALSY_BIT, VAL_NULL, Interner

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmtsnapdec.so")

_P, _I, _U32, _I64, _U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_int64, ctypes.c_uint64
SIGNATURES = [
    ("mt_snapdec_create", _P, [_I]),
    ("mt_snapdec_destroy", None, [_P]),
    ("mt_snapdec_error", ctypes.c_char_p, [_P]),
    ("mt_snapdec_decode", _I, [_P, _U32, _P, _P, _P, _P, _P, _I]),
    ("mt_snapdec_sizes", _I, [_P, _P, _P, _P]),
    ("mt_snapdec_fetch", _I, [_P, _P, _P, _P, _P, _P, _P, _P, _P]),
    ("mt_snapdec_key", _I64, [_P, _U32, _P, _U64]),
    ("mt_snapdec_value", _I64, [_P, _U32, _P, _U64]),
    ("mt_snapdec_num_keys", _U32, [_P]),
    ("mt_snapdec_num_values", _U32, [_P]),
    ("mt_snapdec_doc_clients", _I64, [_P, _U32, _P, _U64]),
    ("mt_snapdec_all_clients", _I64, [_P, _P, _U64]),
    ("mt_opdec_decode", _I, [_P, _U32, _P, _P, _I]),
    ("mt_opdec_sizes", _I, [_P, _P, _P, _P]),
    ("mt_opdec_fetch", _I, [_P, _P, _P, _P, _P]),
    ("mt_opdec_doc_clients", _I64, [_P, _U32, _P, _U64]),
]
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"summary decoder library missing: {LIB_PATH} (run __graft_entry__.build())")
        lib = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def _text(fn, h, i):
    n = fn(h, i, None, 0)
    buf = ctypes.create_string_buffer(max(n, 1))
    fn(h, i, buf, n)
    return buf.raw[:n].decode("utf-8", errors="surrogatepass")


class ClientMaps(Sequence):
    """Per document the short client id map to continue with ({long id: short id}), parsed
    on access from the decoder's one-call dump (mt_snapdec_all_clients)."""

    def __init__(self, lines):
        self._lines = lines

    def __len__(self):
        return len(self._lines)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        return {c: k + 1 for k, c in enumerate(json.loads(self._lines[i]))}

    def __add__(self, other):
        return ClientMaps(self._lines + list(other._lines))

    def __eq__(self, other):
        return list(self) == list(other)


class SummaryDecoder:
    """decode(summaries) -> (arrays, catchup, clients): ``arrays`` as SnapshotBatch.arrays(),
    ``catchup[d]`` the legacy catch-up blob's text (None: none), ``clients[d]`` the short id
    map to continue with (wire.Batch.add_doc(..., clients=...)).  Property keys / values are
    numbered in ``interner`` (shared with the caller's op batches) in the decoder's first-seen
    order; a synthetic interner maps k<n> / integers directly."""

    def __init__(self, interner=None, threads=8):
        self.interner = interner or Interner()
        self.threads = threads
        self.lib = load()
        self.h = self.lib.mt_snapdec_create(1 if self.interner.synthetic else 0)
        self._kmap, self._vmap = [], []   # the decoder's ids -> the interner's

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.mt_snapdec_destroy(self.h)
            self.h = None

    @staticmethod
    def pack(summaries):
        """Blob tables for mt_snapdec_decode: per document the blobs in insertion order."""
        paths, blobs, off = [], [], [0]
        for chunks in summaries:
            for k, v in chunks.items():
                paths.append(k.encode("utf-8"))
                blobs.append(v.encode("utf-8", errors="surrogatepass") if isinstance(v, str) else bytes(v))
            off.append(len(paths))
        return paths, blobs, off

    def decode_packed(self, paths, blobs, off, alloc=None):
        """mt_snapdec_decode + fetch: the arrays with the decoder's own property ids.  alloc(n,
        dtype) -> array supplies the three arenas (segs, text, props), e.g. page-locked memory
        for a fast upload; numpy's allocator otherwise."""
        n = len(off) - 1
        nb = len(paths)
        offa = np.asarray(off, dtype=np.int64)
        pp = (ctypes.c_char_p * max(nb, 1))(*paths)
        pl = np.asarray([len(x) for x in paths] or [0], dtype=np.uint32)
        jp = (ctypes.c_char_p * max(nb, 1))(*blobs)
        jl = np.asarray([len(x) for x in blobs] or [0], dtype=np.uint64)
        rc = self.lib.mt_snapdec_decode(self.h, n, _p(offa), pp, _p(pl), jp, _p(jl), self.threads)
        if rc != 0:
            raise SnapshotError(self.lib.mt_snapdec_error(self.h).decode())
        ns, nt, npr = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self.lib.mt_snapdec_sizes(self.h, ctypes.byref(ns), ctypes.byref(nt), ctypes.byref(npr))
        def arena(m, dt):   # filled whole by fetch; an empty arena is one zero
            if alloc is not None:
                a = alloc(max(m, 1), dt)
                if not m:
                    a[:] = 0
                return a
            return np.empty(m, dtype=dt) if m else np.zeros(1, dtype=dt)
        out = dict(segs=arena(ns.value, SEG_DTYPE)[:ns.value], doc_off=np.zeros(n + 1, dtype=np.int64),
                   n_header=np.zeros(n, dtype=np.int32), text=arena(nt.value, np.uint16),
                   props=arena(npr.value, np.uint32), min_seq=np.zeros(n, dtype=np.int32),
                   cur_seq=np.zeros(n, dtype=np.int32))
        cu = np.zeros(n, dtype=np.int64)
        self.lib.mt_snapdec_fetch(self.h, _p(out["doc_off"]), _p(out["n_header"]), _p(out["segs"]), _p(out["text"]),
                                  _p(out["props"]), _p(out["min_seq"]), _p(out["cur_seq"]), _p(cu))
        return out, cu

    def _remap(self, out):
        """The decoder's key / value ids -> the interner's (first-seen order kept)."""
        it, lib = self.interner, self.lib
        for i in range(len(self._kmap), lib.mt_snapdec_num_keys(self.h)):
            self._kmap.append(it.key(_text(lib.mt_snapdec_key, self.h, i)))
        for i in range(len(self._vmap), lib.mt_snapdec_num_values(self.h)):
            self._vmap.append(it.val(json.loads(_text(lib.mt_snapdec_value, self.h, i))) & (VAL_FALSY_BIT - 1))
            it.note_unkeyed(self._vmap[-1])   # held by some key of a loaded summary
        km, vm = np.asarray(self._kmap, dtype=np.uint32), np.asarray(self._vmap, dtype=np.uint32)
        if np.array_equal(km, np.arange(len(km))) and np.array_equal(vm, np.arange(len(vm))):
            return
        starts = out["segs"]["props"][out["segs"]["props"] != NO_PROPS].astype(np.int64)
        p = out["props"]
        cnt = p[starts].astype(np.int64)
        tot = int(cnt.sum())
        if not tot:
            return
        first = np.repeat(np.cumsum(cnt) - cnt, cnt)
        kpos = np.repeat(starts + 1, cnt) + 2 * (np.arange(tot) - first)
        p[kpos] = km[p[kpos]]
        v = p[kpos + 1]
        live = v != VAL_NULL
        falsy = np.uint32(VAL_FALSY_BIT)
        v[live] = vm[v[live] & ~falsy] | (v[live] & falsy)
        p[kpos + 1] = v

    def decode(self, summaries):
        return self.decode_packed_full(*self.pack(summaries))

    def decode_packed_full(self, paths, blobs, off, alloc=None):
        """decode() of already packed blob tables (pack())."""
        out, cu = self.decode_packed(paths, blobs, off, alloc)
        if not self.interner.synthetic:
            self._remap(out)
        catchup = [None] * len(cu)
        for d in np.flatnonzero(cu >= 0).tolist():   # legacy summaries only
            catchup[d] = blobs[cu[d]].decode("utf-8", errors="surrogatepass")
        size = self.lib.mt_snapdec_all_clients(self.h, None, 0)
        buf = ctypes.create_string_buffer(max(size, 1))
        self.lib.mt_snapdec_all_clients(self.h, buf, size)
        lines = buf.raw[:size].decode("utf-8", errors="surrogatepass").split("\n")[:-1] if size else []
        return out, catchup, ClientMaps(lines)
