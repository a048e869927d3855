"""fluidframework_amd -- MI355X replay / catch-up backend for Fluid Framework's merge-tree.

The hot path (Client.applyMsg over thousands of independent SharedString documents) runs in
hand-written HIP kernels (csrc/) behind the C ABI in include/mt_replay.h.  This Python
module is host plumbing mirroring the reference `Client` surface for tests and the bench;
the Node/N-API facade in js/ is the reference-language binding."""
import ctypes

import numpy as np

from . import _native
from .wire import CHECKSUM_DTYPE, OP_DTYPE, Batch, Interner  # noqa: F401

__all__ = ["MergeTreeBatch", "DeviceBatch", "Batch", "Interner", "DeltaLogOverflow"]


class DeltaLogOverflow(RuntimeError):
    """A document's delta log dropped records (mt_get_delta_log -> MT_E_OVERFLOW); `records`
    holds the whole records that were kept."""

    def __init__(self, msg, records):
        super().__init__(msg)
        self.records = records


class PinnedArray:
    """A page-locked host buffer (mt_host_alloc) and its numpy view (`a`); the buffer is freed
    with this object, so keep it alive while the view is in use."""

    def __init__(self, lib, n, dtype):
        dt = np.dtype(dtype)
        nbytes = max(int(n), 1) * dt.itemsize
        self.lib = lib
        self.p = lib.mt_host_alloc(nbytes)
        if not self.p:
            raise MemoryError(f"mt_host_alloc({nbytes}) failed")
        self.a = np.frombuffer((ctypes.c_uint8 * nbytes).from_address(self.p), dtype=dt)

    def __del__(self):
        p, self.p = getattr(self, "p", None), None
        if p:
            try:
                self.lib.mt_host_free(p)
            except Exception:
                pass


class MergeTreeBatch:
    """N observer replicas (one per document) resident on one GPU.

    Mirrors, per document, `new Client(...)` + `startOrUpdateCollaboration` (MT/client.ts:
    75-84, 1053-1073), `applyMsg` (:797-819), `getLength` (:1051), `getText` via
    MergeTreeTextHelper (MT/textSegment.ts:154-172) and `getPropertiesAtPosition` (:1011-1025).
    """

    def __init__(self, n_docs, device=0, seg_capacity=0, block_capacity=0, heap_capacity=0,
                 text_capacity=0, props_capacity=0, delta_log_capacity=0, lds_seg_capacity=0,
                 page_capacity=0, page_heap_capacity=0, unsettled_capacity=0, uid_capacity=0,
                 lds_page_capacity=0, lds_unsettled_capacity=0, lds_page_heap_capacity=0, lds_narrow_overlap=0,
                 delta_log_mode=0, live_client=0, live_group_capacity=0, paged_slices=0, segment_ordinals=0,
                 overlap_arena_capacity=0):
        self.lib = _native.load()
        opt = _native.MtOptions(device, seg_capacity, block_capacity, heap_capacity,
                                text_capacity, props_capacity, delta_log_capacity,
                                lds_seg_capacity, page_capacity, page_heap_capacity,
                                unsettled_capacity, uid_capacity, lds_page_capacity,
                                lds_unsettled_capacity, lds_page_heap_capacity, lds_narrow_overlap,
                                delta_log_mode, live_client, live_group_capacity, paged_slices,
                                segment_ordinals, overlap_arena_capacity)
        self.h = self.lib.mt_create(n_docs, ctypes.byref(opt))
        if not self.h:
            raise RuntimeError("mt_create failed (no HIP device visible, or out of device memory)")
        self.n_docs = n_docs

    def close(self):
        if self.h:
            self.lib.mt_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            msg = f"{what} failed ({rc}): {self.lib.mt_last_error(self.h).decode()}"
            raise RuntimeError(msg)

    # -------------------------------------------------------------- input
    def load_initial_text(self, seed_off, seed):
        seed_off = np.ascontiguousarray(seed_off, dtype=np.int64)
        seed = np.ascontiguousarray(seed, dtype=np.uint16)
        self._check(self.lib.mt_load_initial_text(self.h, _native.ptr(seed_off), _native.ptr(seed)),
                    "mt_load_initial_text")

    def start_collaboration(self, min_seq, cur_seq):
        """Client.startOrUpdateCollaboration(id, minSeq, currentSeq) for every document with
        min_seq[d] >= 0 (before its first message)."""
        ms = np.ascontiguousarray(min_seq, dtype=np.int32)
        cs = np.ascontiguousarray(cur_seq, dtype=np.int32)
        if ms.shape != (self.n_docs,) or cs.shape != (self.n_docs,):
            raise ValueError("start_collaboration: one minSeq and one currentSeq per document")
        self._check(self.lib.mt_start_collaboration(self.h, _native.ptr(ms), _native.ptr(cs)),
                    "mt_start_collaboration")

    def reset(self):
        """Asynchronously re-initialise every document from the loaded initial contents."""
        self._check(self.lib.mt_reset(self.h), "mt_reset")

    def apply_arrays(self, a):
        ops = np.ascontiguousarray(a["ops"], dtype=OP_DTYPE)
        off = np.ascontiguousarray(a["doc_off"], dtype=np.int64)
        text = np.ascontiguousarray(a["text"], dtype=np.uint16)
        props = np.ascontiguousarray(a["props"], dtype=np.uint32)
        self._check(self.lib.mt_apply_ops(self.h, _native.ptr(off), _native.ptr(ops), len(ops),
                                          _native.ptr(text), len(text), _native.ptr(props), len(props)),
                    "mt_apply_ops")

    @staticmethod
    def _snap_args(la):
        from .snapshot import SEG_DTYPE
        return [np.ascontiguousarray(la["doc_off"], dtype=np.int64), np.ascontiguousarray(la["n_header"], dtype=np.int32),
                np.ascontiguousarray(la["segs"], dtype=SEG_DTYPE), np.ascontiguousarray(la["text"], dtype=np.uint16),
                np.ascontiguousarray(la["props"], dtype=np.uint32), np.ascontiguousarray(la["min_seq"], dtype=np.int32),
                np.ascontiguousarray(la["cur_seq"], dtype=np.int32)]

    def load_snapshots(self, la):
        """Client.load of a decoded SnapshotV1 summary into every document
        (snapshot.SnapshotBatch.arrays(); MT/snapshotLoader.ts:36-228)."""
        off, nh, segs, text, props, mn, cu = self._snap_args(la)
        if len(off) != self.n_docs + 1:
            raise ValueError("one summary per document")
        self._check(self.lib.mt_load_snapshots(self.h, _native.ptr(off), _native.ptr(nh), _native.ptr(segs), len(segs),
                                               _native.ptr(text), len(text), _native.ptr(props), len(props),
                                               _native.ptr(mn), _native.ptr(cu)), "mt_load_snapshots")

    def load_summaries(self, summaries, interner, threads=8):
        """Client.load of every document from its summary blobs ({path: JSON text}, one dict
        per document): decoded on the host by the native decoder (snapdec, include/
        mt_snapshot.h; MT/snapshotLoader.ts:36-228), then loaded as load_snapshots does.
        Returns (catchup, clients): per document the legacy catch-up messages and the short
        client map its ops continue with (wire.Batch.add_doc(..., clients=...))."""
        import json as _json
        from .snapdec import SummaryDecoder
        la, catchup, clients = SummaryDecoder(interner, threads).decode(summaries)
        self.load_snapshots(la)
        return [_json.loads(c) if c is not None else [] for c in catchup], clients

    def upload_snapshots(self, la, doc_lo=0):
        """Device-resident summaries (mt_snapshots_upload); .load_async() enqueues a load.  With
        fewer summaries than documents, summary d is for document doc_lo + d
        (mt_snapshots_upload_range)."""
        off, nh, segs, text, props, mn, cu = self._snap_args(la)
        n = len(off) - 1
        s = self.lib.mt_snapshots_upload_range(self.h, doc_lo, n, _native.ptr(off), _native.ptr(nh), _native.ptr(segs),
                                               len(segs), _native.ptr(text), len(text), _native.ptr(props), len(props),
                                               _native.ptr(mn), _native.ptr(cu))
        if not s:
            raise RuntimeError(f"mt_snapshots_upload failed: {self.lib.mt_last_error(self.h).decode()}")
        return DeviceSnapshots(self, s)

    def catch_up(self, summaries, interner, threads=8, slice_docs=8192, packed=None):
        """Cold catch-up of every document from its summary blobs ({path: JSON text} per
        document; or `packed` = snapdec.SummaryDecoder.pack(summaries)), as load_summaries,
        in slices of `slice_docs` documents: the native decoder parses slice k + 1 on the
        host (a worker thread; the decoder's own threads inside) while slice k is uploaded
        and its load runs on the GPU (mt_snapshots_upload_range + mt_snapshots_load_async).
        Returns (catchup, clients) as load_summaries; the loads are enqueued on the handle's
        stream (sync() waits)."""
        import json as _json
        import queue
        import threading
        from .snapdec import SummaryDecoder
        paths, blobs, off = packed if packed is not None else SummaryDecoder.pack(summaries)
        if len(off) != self.n_docs + 1:
            raise ValueError("one summary per document")
        dec = SummaryDecoder(interner, threads)
        q = queue.Queue(maxsize=2)   # decoded slices waiting for their upload
        # arenas the decoder writes straight into, reused from slice to slice (and call to
        # call: no page faults once warm): three sets circulate -- one uploading, two decoded
        # or decoding.  (Page-locked arenas were measured slower: pinning costs more than the
        # ~17 GB/s pageable upload loses.)
        free_sets = queue.Queue()
        pool = getattr(self, "_catchup_arenas", None) or [{}, {}, {}]
        self._catchup_arenas = pool
        for ps in pool:
            free_sets.put(ps)

        stop = threading.Event()   # the consumer failed: the producer stops at its next slice

        def produce():
            try:
                for d0 in range(0, self.n_docs, slice_docs):
                    if stop.is_set():
                        return
                    d1 = min(self.n_docs, d0 + slice_docs)
                    b0, b1 = off[d0], off[d1]
                    sub = (paths[b0:b1], blobs[b0:b1], [o - b0 for o in off[d0:d1 + 1]])
                    pset = free_sets.get()

                    def alloc(m, dt, pset=pset):
                        key = np.dtype(dt).str
                        a = pset.get(key)
                        if a is None or len(a) < m:
                            a = np.empty(int(m * 1.25) + 64, dtype=dt)
                            pset[key] = a
                        return a[:m]
                    out, catchup, clients = dec.decode_packed_full(*sub, alloc=alloc)
                    q.put((d0, out, catchup, clients, pset))
                q.put(None)
            except BaseException as e:   # surfaces in the consumer
                q.put(e)

        t = threading.Thread(target=produce, daemon=True)
        t.start()
        from .snapdec import ClientMaps
        catchup_all, clients_all, held = [], ClientMaps([]), []
        try:
            while True:
                item = q.get()
                if item is None:
                    break
                if isinstance(item, BaseException):
                    raise item
                d0, out, catchup, clients, pset = item
                snaps = self.upload_snapshots(out, doc_lo=d0)   # synchronous copies: the set is free again
                free_sets.put(pset)
                snaps.load_async()
                held.append(snaps)   # device copies stay alive until the loads have run
                cu_msgs = [[] for _ in catchup]
                for i, c in enumerate(catchup):
                    if c is not None:
                        cu_msgs[i] = _json.loads(c)
                catchup_all += cu_msgs
                clients_all = clients_all + clients
        finally:
            # on any exit: unblock and join the producer (it may wait for a free arena set or
            # on the queue), finish the enqueued loads, free every uploaded snapshot set
            stop.set()
            while t.is_alive():
                try:
                    item = q.get(timeout=0.05)
                    if isinstance(item, tuple):
                        free_sets.put(item[4])
                except queue.Empty:
                    pass
                free_sets.put({})
            t.join()
            try:
                self.sync()
            finally:
                for s_ in held:
                    s_.free()
        return catchup_all, clients_all

    def ingest_logs(self, slices, interner=None, threads=8, pinned=True):
        """Sequenced message logs in, replayed documents out, as a pipeline (SEQ/sequence.ts:579-616
        feeds SharedSegmentSequence JSON messages): ``slices`` yields (d0, blobs) -- the JSON
        message arrays of documents [d0, d0 + len(blobs)), in document order.  A host thread
        encodes slice k + 1 (the native encoder, mt_opdec, its own threads inside) while this
        thread uploads slice k (mt_batch_upload) and enqueues its replay on the handle's
        stream, behind slice k - 1's (mt_batch_apply_async).  Arenas are reused from slice to
        slice, and so is the encoder (its buffers stay warm from call to call for the same
        interner and thread count); with `pinned` the arenas are page-locked (mt_host_alloc),
        so the upload is a DMA that takes no host core from the encoder.  Returns the seconds each stage was busy: {"encode",
        "upload", "apply_wait", "wall"} (apply_wait: time the caller's thread waited for the
        previous slice's replay) and "encode_slices", each slice's encode seconds."""
        import queue
        import threading
        import time as _time
        from .opdec import MessageDecoder
        interner = interner or getattr(self, "_ingest_interner", None) or Interner(synthetic=True)
        self._ingest_interner = interner
        dec = getattr(self, "_ingest_dec", None)
        if dec is None or dec.interner is not interner or dec.threads != threads:
            dec = self._ingest_dec = MessageDecoder(interner, threads=threads)
        q = queue.Queue(maxsize=1)                     # one encoded slice waiting for its upload
        free_sets = queue.Queue()
        for ps in getattr(self, "_ingest_arenas", None) or [{}, {}]:
            free_sets.put(ps)
        stop = threading.Event()
        busy = {"encode": 0.0, "upload": 0.0, "apply_wait": 0.0, "encode_slices": []}

        def produce():
            try:
                for d0, blobs in slices:
                    if stop.is_set():
                        return
                    pset = free_sets.get()
                    if stop.is_set():
                        return

                    def alloc(m, dt, pset=pset):
                        key = np.dtype(dt).str
                        a = pset.get(key)
                        if a is None or len(a) < m:
                            n = int(m * 1.25) + 64
                            if pinned:
                                pset["pin" + key] = PinnedArray(self.lib, n, dt)
                                a = pset["pin" + key].a
                            else:
                                a = np.empty(n, dtype=dt)
                            pset[key] = a
                        return a[:m]
                    t = _time.perf_counter()
                    off = pset.setdefault("off", np.zeros(self.n_docs + 1, dtype=np.int64))
                    n = len(blobs)
                    sub = np.zeros(n + 1, dtype=np.int64)
                    out = dec.decode_packed(blobs, alloc=alloc, doc_off_out=sub)
                    dec.remap(out)
                    off[: d0 + 1] = 0
                    off[d0 + 1: d0 + n + 1] = sub[1:]
                    off[d0 + n + 1:] = sub[-1]
                    out["doc_off"] = off
                    busy["encode_slices"].append(_time.perf_counter() - t)
                    busy["encode"] += busy["encode_slices"][-1]
                    q.put((out, pset))
                q.put(None)
            except BaseException as e:   # surfaces in the consumer
                q.put(e)

        t_wall = _time.perf_counter()
        th = threading.Thread(target=produce, daemon=True)
        th.start()
        prev = None
        try:
            while True:
                item = q.get()
                if item is None:
                    break
                if isinstance(item, BaseException):
                    raise item
                out, pset = item
                t = _time.perf_counter()
                b = self.upload(out)   # (validation + copies: the arena set is free again after)
                busy["upload"] += _time.perf_counter() - t
                free_sets.put(pset)
                if prev is not None:
                    # before this slice's replay is queued: hipFree waits for the device to go
                    # idle, and slice k - 1's replay has ended while slice k was encoded, so
                    # nothing waits here (after the enqueue it would wait -- spinning a host
                    # core the encoder needs -- for slice k's whole replay)
                    t = _time.perf_counter()
                    prev.free()
                    busy["apply_wait"] += _time.perf_counter() - t
                t = _time.perf_counter()
                b.apply_async()        # (waits for the previous slice's replay and growth step)
                busy["apply_wait"] += _time.perf_counter() - t
                prev = b
            self.sync()
        finally:
            stop.set()
            while th.is_alive():
                try:
                    item = q.get(timeout=0.05)
                    if isinstance(item, tuple):
                        free_sets.put(item[1])
                except queue.Empty:
                    pass
                free_sets.put({})
            th.join()
            if prev is not None:
                self.sync()
                prev.free()
            self._ingest_arenas = []
            while not free_sets.empty():
                ps = free_sets.get()
                if ps:
                    self._ingest_arenas.append(ps)
        busy["wall"] = _time.perf_counter() - t_wall
        return busy

    def extract_snapshots_raw(self):
        """mt_extract_snapshots as concatenated arrays: (counts[n_docs, 3], records, text,
        props, min_seq, cur_seq); record offsets are relative to their document's arenas."""
        from .snapshot import SEG_DTYPE
        io = np.zeros(3 * self.n_docs, dtype=np.int64)
        self._check(self.lib.mt_extract_snapshots(self.h, _native.ptr(io), None, None, None, None, None),
                    "mt_extract_snapshots")
        tot = io.reshape(-1, 3).sum(axis=0)
        recs = np.zeros(max(int(tot[0]), 1), dtype=SEG_DTYPE)
        text = np.zeros(max(int(tot[1]), 1), dtype=np.uint16)
        props = np.zeros(max(int(tot[2]), 1), dtype=np.uint32)
        mn = np.zeros(self.n_docs, dtype=np.int32)
        cu = np.zeros(self.n_docs, dtype=np.int32)
        self._check(self.lib.mt_extract_snapshots(self.h, _native.ptr(io), _native.ptr(recs), _native.ptr(text),
                                                  _native.ptr(props), _native.ptr(mn), _native.ptr(cu)),
                    "mt_extract_snapshots")
        return io.reshape(-1, 3), recs[: int(tot[0])], text, props, mn, cu

    def extract_snapshots(self):
        """SnapshotV1.extractSync of every document (mt_extract_snapshots): per document
        (records, text, props, min_seq, cur_seq); records index that document's arenas."""
        from .snapshot import SEG_DTYPE
        io = np.zeros(3 * self.n_docs, dtype=np.int64)
        self._check(self.lib.mt_extract_snapshots(self.h, _native.ptr(io), None, None, None, None, None),
                    "mt_extract_snapshots")
        tot = io.reshape(-1, 3).sum(axis=0)
        recs = np.zeros(max(int(tot[0]), 1), dtype=SEG_DTYPE)
        text = np.zeros(max(int(tot[1]), 1), dtype=np.uint16)
        props = np.zeros(max(int(tot[2]), 1), dtype=np.uint32)
        mn = np.zeros(self.n_docs, dtype=np.int32)
        cu = np.zeros(self.n_docs, dtype=np.int32)
        self._check(self.lib.mt_extract_snapshots(self.h, _native.ptr(io), _native.ptr(recs), _native.ptr(text),
                                                  _native.ptr(props), _native.ptr(mn), _native.ptr(cu)),
                    "mt_extract_snapshots")
        out = []
        c = io.reshape(-1, 3)
        r0 = t0 = p0 = 0
        for d in range(self.n_docs):
            nr, nt, np_ = (int(x) for x in c[d])
            out.append(dict(segs=recs[r0:r0 + nr], text=text[t0:t0 + nt], props=props[p0:p0 + np_],
                            min_seq=int(mn[d]), cur_seq=int(cu[d])))
            r0, t0, p0 = r0 + nr, t0 + nt, p0 + np_
        return out

    def upload(self, a):
        return DeviceBatch(self, a)

    def generate(self, cfg, doc_base=0, trace=None, ops_per_doc=None, doc_ids=None):
        """Device-generated batch (mt_generate); ops_per_doc: a length per document, doc_ids:
        their global indices (mt_generate_docs), else cfg["ops"] each and doc_base + d."""
        c = _native.gen_cfg(cfg)
        if ops_per_doc is not None or doc_ids is not None:
            lens = None if ops_per_doc is None else np.ascontiguousarray(ops_per_doc, dtype=np.int32)
            ids = None if doc_ids is None else np.ascontiguousarray(doc_ids, dtype=np.int32)
            for x in (lens, ids):
                if x is not None and x.shape != (self.n_docs,):
                    raise ValueError("ops_per_doc / doc_ids: one per document")
            b = self.lib.mt_generate_docs(self.h, ctypes.byref(c), doc_base, _native.ptr(lens), _native.ptr(ids),
                                          _native.ptr(trace))
        else:
            b = self.lib.mt_generate(self.h, ctypes.byref(c), doc_base, _native.ptr(trace))
        if not b:
            raise RuntimeError(f"mt_generate failed: {self.lib.mt_last_error(self.h).decode()}")
        return DeviceBatch(self, None, handle=b)

    def generated_seeds(self, cfg, doc_base=0, doc_ids=None):
        c = _native.gen_cfg(cfg)
        ids = None if doc_ids is None else np.ascontiguousarray(doc_ids, dtype=np.int32)
        off = np.zeros(self.n_docs + 1, dtype=np.int64)
        self._check(self.lib.mt_generated_seeds_docs(self.h, ctypes.byref(c), doc_base, _native.ptr(ids),
                                                     _native.ptr(off), None), "mt_generated_seeds")
        seed = np.zeros(max(int(off[-1]), 1), dtype=np.uint16)
        self._check(self.lib.mt_generated_seeds_docs(self.h, ctypes.byref(c), doc_base, _native.ptr(ids),
                                                     _native.ptr(off), _native.ptr(seed)), "mt_generated_seeds")
        return off, seed

    def sync(self):
        self._check(self.lib.mt_sync(self.h), "mt_sync")

    def last_hbm_docs(self):
        """Documents of the last batch replayed from HBM (outgrew the LDS tier)."""
        out = np.zeros(8, dtype=np.uint32)
        self._check(self.lib.mt_last_hbm_docs(self.h, _native.ptr(out)), "mt_last_hbm_docs")
        return dict(total=int(out[0]), spilled=int(out[1]), segments=int(out[2]), blocks=int(out[3]), heap=int(out[4]),
                    text=int(out[5]), props=int(out[6]), at_load=int(out[7]))

    def last_paged_peaks(self):
        """High-water marks of the paged documents of the last batch / generation."""
        out = np.zeros(5, dtype=np.uint32)
        self._check(self.lib.mt_last_paged_peaks(self.h, _native.ptr(out)), "mt_last_paged_peaks")
        return dict(pages=int(out[0]), unsettled=int(out[1]), heap=int(out[2]), segments=int(out[3]),
                    tight_handovers=int(out[4]))

    def last_grown(self):
        """The last batch's growth step (mt_last_grown): documents moved to larger paged
        capacities, rounds, documents in the big region and its capacities."""
        out = np.zeros(6, dtype=np.uint32)
        self._check(self.lib.mt_last_grown(self.h, _native.ptr(out)), "mt_last_grown")
        return dict(zip(["grown", "rounds", "in_big_region", "pages", "unsettled", "heap"], (int(x) for x in out)))

    def last_kernel_ms(self):
        return float(self.lib.mt_last_kernel_ms(self.h))

    def set_stream_priority(self, priority):
        """mt_set_stream_priority: > 0 the device's highest stream priority, < 0 its lowest."""
        self._check(self.lib.mt_set_stream_priority(self.h, int(priority)), "mt_set_stream_priority")

    def last_load_ms(self):
        """Device time of the most recent snapshot load's kernels (mt_last_load_ms)."""
        return float(self.lib.mt_last_load_ms(self.h))

    # -------------------------------------------------------------- read-out
    def status(self):
        out = np.zeros(self.n_docs, dtype=np.int32)
        self._check(self.lib.mt_get_status(self.h, _native.ptr(out)), "mt_get_status")
        return out

    def get_length(self, doc):
        out = ctypes.c_uint32()
        self._check(self.lib.mt_get_length(self.h, doc, ctypes.byref(out)), "mt_get_length")
        return out.value

    def get_text(self, doc):
        n = ctypes.c_uint32()
        self._check(self.lib.mt_get_text(self.h, doc, None, 0, ctypes.byref(n)), "mt_get_text")
        buf = np.zeros(max(n.value, 1), dtype=np.uint16)
        self._check(self.lib.mt_get_text(self.h, doc, _native.ptr(buf), n.value, ctypes.byref(n)),
                    "mt_get_text")
        return buf[: n.value].tobytes().decode("utf-16-le", errors="surrogatepass")

    def get_segments(self, doc):
        nr, nl = ctypes.c_uint32(), ctypes.c_uint32()
        self._check(self.lib.mt_get_segments(self.h, doc, None, 0, ctypes.byref(nr), None, 0,
                                             ctypes.byref(nl)), "mt_get_segments")
        rows = np.zeros((max(nr.value, 1), 8), dtype=np.int32)
        leaves = np.zeros(max(nl.value, 1), dtype=np.int32)
        self._check(self.lib.mt_get_segments(self.h, doc, _native.ptr(rows), nr.value, ctypes.byref(nr),
                                             _native.ptr(leaves), nl.value, ctypes.byref(nl)),
                    "mt_get_segments")
        return rows[: nr.value], leaves[: nl.value].tolist()

    def get_overlap_arena(self, doc):
        """A paged document's overflow overlap arena (mt_get_overlap_arena)."""
        out = np.zeros(7, dtype=np.int32)
        self._check(self.lib.mt_get_overlap_arena(self.h, doc, _native.ptr(out)), "mt_get_overlap_arena")
        return dict(zip(["capacity", "fill", "half", "largest_set", "live_units", "made", "peak_fill"],
                        (int(x) for x in out)))

    def get_segment_props(self, doc, i):
        pairs = np.zeros(64, dtype=np.uint32)
        n = ctypes.c_int32()
        self._check(self.lib.mt_get_segment_props(self.h, doc, i, _native.ptr(pairs), 32, ctypes.byref(n)),
                    "mt_get_segment_props")
        if n.value < 0:
            return None
        return [(int(pairs[2 * j]), int(pairs[2 * j + 1])) for j in range(n.value)]

    def get_all_segment_props(self, doc):
        """get_segment_props of every segment, from one copy of the document."""
        n = ctypes.c_uint64()
        self._check(self.lib.mt_get_all_segment_props(self.h, doc, None, 0, ctypes.byref(n)), "mt_get_all_segment_props")
        buf = np.zeros(max(n.value, 1), dtype=np.int32)
        self._check(self.lib.mt_get_all_segment_props(self.h, doc, _native.ptr(buf), n.value, ctypes.byref(n)),
                    "mt_get_all_segment_props")
        out, w, b = [], 0, buf.tolist()
        while w < n.value:
            k = b[w]
            w += 1
            if k < 0:
                out.append(None)
                continue
            out.append([(b[w + 2 * j] & 0xFFFFFFFF, b[w + 2 * j + 1] & 0xFFFFFFFF) for j in range(k)])
            w += 2 * k
        return out

    # -------------------------------------------------------------- segment read-outs
    @staticmethod
    def _seg_info(info, text):
        if info.row < 0:
            return None
        out = dict(row=info.row, uid=info.uid, position=info.position, offset=info.offset, length=info.length,
                   seq=info.seq, client=info.client, removed_seq=info.removed_seq,
                   removed_client=info.removed_client, marker_ref_type=info.marker_ref_type,
                   ordinal=list(info.ordinal[:info.ordinal_len]) if info.ordinal_len >= 0 else None)
        if info.marker_ref_type < 0:
            out["text"] = text[:info.text_len].tobytes().decode("utf-16-le", errors="surrogatepass")
        return out

    def get_containing_segment(self, doc, pos, ref_seq=0, client=0, text_cap=1 << 16):
        """MergeTree.getContainingSegment(pos, refSeq, clientId) (MT/mergeTree.ts:1656-1667):
        the segment's read-out (dict) with `offset` = pos - its position, or None."""
        info = _native.MtSegInfo()
        text = np.zeros(text_cap, dtype=np.uint16)
        self._check(self.lib.mt_get_containing_segment(self.h, doc, pos, ref_seq, client, ctypes.byref(info),
                                                       _native.ptr(text), text_cap), "mt_get_containing_segment")
        return self._seg_info(info, text)

    def get_segment_by_uid(self, doc, uid, ref_seq=0, client=0, text_cap=1 << 16):
        """MergeTree.getPosition(segment, refSeq, clientId) (:1619-1636) of segment `uid` as
        the read-out's `position`; None once it left the tree."""
        info = _native.MtSegInfo()
        text = np.zeros(text_cap, dtype=np.uint16)
        self._check(self.lib.mt_get_segment_by_uid(self.h, doc, uid, ref_seq, client, ctypes.byref(info),
                                                   _native.ptr(text), text_cap), "mt_get_segment_by_uid")
        return self._seg_info(info, text)

    def get_view_lengths(self, docs, ref_seq, client):
        """MergeTree.getLength(refSeq, clientId) (:1610-1612) for each (doc, refSeq, client):
        the root's partial length in a remote view (every refSeq of the collab window,
        MT/partialLengths.ts:455-486), the local length for client 0."""
        docs = np.ascontiguousarray(docs, dtype=np.uint32)
        ref = np.ascontiguousarray(ref_seq, dtype=np.int32)
        cli = np.ascontiguousarray(client, dtype=np.int32)
        out = np.zeros(len(docs), dtype=np.int32)
        self._check(self.lib.mt_get_view_lengths(self.h, len(docs), _native.ptr(docs), _native.ptr(ref),
                                                 _native.ptr(cli), _native.ptr(out)), "mt_get_view_lengths")
        return out

    def get_prop_runs(self, doc):
        nr, nw = ctypes.c_uint32(), ctypes.c_uint32()
        self._check(self.lib.mt_get_prop_runs(self.h, doc, None, 0, ctypes.byref(nr), None, 0,
                                              ctypes.byref(nw)), "mt_get_prop_runs")
        runs = np.zeros((max(nr.value, 1), 3), dtype=np.uint32)
        recs = np.zeros(max(nw.value, 1), dtype=np.uint32)
        self._check(self.lib.mt_get_prop_runs(self.h, doc, _native.ptr(runs), nr.value, ctypes.byref(nr),
                                              _native.ptr(recs), nw.value, ctypes.byref(nw)),
                    "mt_get_prop_runs")
        out = []
        for s, l, r in runs[: nr.value].tolist():
            if r == 0xFFFFFFFF:
                out.append((s, l, None))
            else:
                n = int(recs[r])
                out.append((s, l, [(int(recs[r + 1 + 2 * j]), int(recs[r + 2 + 2 * j])) for j in range(n)]))
        return out

    def get_properties_at_position(self, doc, pos):
        for s, l, p in self.get_prop_runs(doc):
            if s <= pos < s + l:
                return p
        return None

    def debug_raw(self, doc):
        """Raw segment records (n x 8 u32: segA, segB) and the 32-word document header."""
        n = ctypes.c_uint32()
        hdr = np.zeros(32, dtype=np.int32)
        self._check(self.lib.mt_debug_raw(self.h, doc, None, 0, ctypes.byref(n), _native.ptr(hdr)), "mt_debug_raw")
        rows = np.zeros((max(n.value, 1), 8), dtype=np.uint32)
        self._check(self.lib.mt_debug_raw(self.h, doc, _native.ptr(rows), n.value, ctypes.byref(n), None),
                    "mt_debug_raw")
        return rows[:n.value], hdr

    def is_paged(self, doc):
        """True when the document lives in the paged layout (DESIGN.md 'Paged documents')."""
        return bool(self.debug_raw(doc)[1][24])

    def get_delta_log(self, doc):
        """The document's delta-log records since the last reset (oracle layout); raises
        DeltaLogOverflow when records were dropped (delta_log_capacity too small)."""
        n = ctypes.c_uint32()
        buf = np.zeros(1, dtype=np.int32)
        rc = self.lib.mt_get_delta_log(self.h, doc, None, 0, ctypes.byref(n))
        if rc not in (0, _native.MT_E_OVERFLOW):
            self._check(rc, "mt_get_delta_log")
        buf = np.zeros(max(n.value, 1), dtype=np.int32)
        rc = self.lib.mt_get_delta_log(self.h, doc, _native.ptr(buf), n.value, ctypes.byref(n))
        if rc == _native.MT_E_OVERFLOW:
            raise DeltaLogOverflow(self.lib.mt_last_error(self.h).decode(), buf[: n.value].tolist())
        self._check(rc, "mt_get_delta_log")
        return buf[: n.value].tolist()

    def delta_log_reset(self):
        """Empties every document's delta log (after its records were consumed)."""
        self._check(self.lib.mt_delta_log_reset(self.h), "mt_delta_log_reset")

    def maintenance_counts(self):
        """[n_docs, 3] SPLIT / APPEND / UNLINK mergeTreeMaintenanceCallback event counts
        (needs delta_log_capacity > 0)."""
        out = np.zeros((self.n_docs, 3), dtype=np.uint32)
        self._check(self.lib.mt_maintenance_counts(self.h, _native.ptr(out)), "mt_maintenance_counts")
        return out

    # -------------------------------------------------------------- live-client handles
    def regenerate_pending(self, doc, cap=1 << 16, text_cap=1 << 20, props_cap=1 << 20):
        """mt_regenerate_pending: the ops rebuilt from the oldest pending segment group
        (records, text, props), or None when nothing is pending."""
        out = np.zeros(cap, dtype=_native.REGEN_DTYPE)
        text = np.zeros(text_cap, dtype=np.uint16)
        props = np.zeros(props_cap, dtype=np.uint32)
        n = ctypes.c_int32(0)
        self._check(self.lib.mt_regenerate_pending(self.h, doc, _native.ptr(out), cap, ctypes.byref(n),
                                                   _native.ptr(text), text_cap, _native.ptr(props), props_cap),
                    "mt_regenerate_pending")
        if n.value < 0:
            return None
        return out[:n.value], text, props

    def pending_counts(self):
        """[n_docs, 2]: collabWindow.localSeq and the pending segment groups per document."""
        out = np.zeros((self.n_docs, 2), dtype=np.int32)
        self._check(self.lib.mt_pending_counts(self.h, _native.ptr(out)), "mt_pending_counts")
        return out

    def checksums(self):
        out = np.zeros(self.n_docs, dtype=CHECKSUM_DTYPE)
        self._check(self.lib.mt_checksums(self.h, _native.ptr(out)), "mt_checksums")
        return out

    def checksums_device(self, device_ptr):
        self._check(self.lib.mt_checksums_device(self.h, ctypes.c_void_p(device_ptr)), "mt_checksums_device")


class DeviceBatch:
    """A batch of encoded messages resident in HBM (mt_batch)."""

    def __init__(self, owner, a, handle=None):
        self.owner = owner
        lib = owner.lib
        if handle is None:
            ops = np.ascontiguousarray(a["ops"], dtype=OP_DTYPE)
            off = np.ascontiguousarray(a["doc_off"], dtype=np.int64)
            text = np.ascontiguousarray(a["text"], dtype=np.uint16)
            props = np.ascontiguousarray(a["props"], dtype=np.uint32)
            handle = lib.mt_batch_upload(owner.h, _native.ptr(off), _native.ptr(ops), len(ops),
                                         _native.ptr(text), len(text), _native.ptr(props), len(props))
            if not handle:
                raise RuntimeError(f"mt_batch_upload failed: {lib.mt_last_error(owner.h).decode()}")
        self.b = handle
        self.n_ops = int(lib.mt_batch_num_ops(self.b))

    def apply_async(self):
        self.owner._check(self.owner.lib.mt_batch_apply_async(self.owner.h, self.b), "mt_batch_apply_async")

    def sizes(self):
        """(op records, text units, property words) of the batch."""
        n, t, p = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self.owner.lib.mt_batch_sizes(self.b, ctypes.byref(n), ctypes.byref(t), ctypes.byref(p))
        return int(n.value), int(t.value), int(p.value)

    def download(self):
        lib = self.owner.lib
        n, t, p = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        lib.mt_batch_sizes(self.b, ctypes.byref(n), ctypes.byref(t), ctypes.byref(p))
        off = np.zeros(self.owner.n_docs + 1, dtype=np.int64)
        ops = np.zeros(n.value, dtype=OP_DTYPE)
        text = np.zeros(max(t.value, 1), dtype=np.uint16)
        props = np.zeros(max(p.value, 1), dtype=np.uint32)
        rc = lib.mt_batch_download(self.b, _native.ptr(off), _native.ptr(ops), _native.ptr(text),
                                   _native.ptr(props))
        if rc:
            raise RuntimeError("mt_batch_download failed")
        return dict(doc_off=off, ops=ops, text=text, props=props)

    def free(self):
        if self.b:
            self.owner.lib.mt_batch_free(self.b)
            self.b = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DeviceSnapshots:
    """Decoded summaries resident in HBM (mt_snapshots)."""

    def __init__(self, owner, handle):
        self.owner, self.s = owner, handle

    def load_async(self):
        self.owner._check(self.owner.lib.mt_snapshots_load_async(self.owner.h, self.s), "mt_snapshots_load_async")

    def free(self):
        if self.s:
            self.owner.lib.mt_snapshots_free(self.s)
            self.s = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
