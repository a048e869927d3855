"""TEST INFRASTRUCTURE ONLY -- ctypes binding of the CPU restatement oracle
(oracle/liboracle.so, built from oracle/mt_oracle.c).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker."""
import ctypes
import os
import subprocess

import numpy as np

from fluidframework_amd.wire import CHECKSUM_DTYPE, OP_DTYPE, gen_thresholds

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
_lib = None


class GenCfg(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint32), ("ops", ctypes.c_int32), ("writers", ctypes.c_int32),
                ("lag", ctypes.c_int32), ("seed_len", ctypes.c_int32), ("text_max", ctypes.c_int32),
                ("n_keys", ctypes.c_int32), ("n_values", ctypes.c_int32),
                ("max_keys_per_op", ctypes.c_int32), ("_pad", ctypes.c_int32),
                ("p_insert", ctypes.c_uint64), ("p_insert_remove", ctypes.c_uint64),
                ("p_newline", ctypes.c_uint64), ("p_len_continue", ctypes.c_uint64),
                ("p_insert_props", ctypes.c_uint64), ("p_null", ctypes.c_uint64)]


def build():
    subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        i32, u64 = ctypes.c_int32, ctypes.c_uint64
        L.orc_new.restype = P
        L.orc_new.argtypes = [P, i32]
        L.orc_free.argtypes = [P]
        L.orc_apply.argtypes = [P, P, P, P]
        L.orc_apply.restype = i32
        L.orc_status.argtypes = [P]
        L.orc_status.restype = i32
        L.orc_pending_counts.argtypes = [P, P]
        L.orc_regenerate.argtypes = [P, i32, P, i32, P, i32, P, i32]
        L.orc_regenerate.restype = i32
        L.orc_view_length.argtypes = [P, i32, i32]
        L.orc_view_length.restype = i32
        L.orc_containing.argtypes = [P, i32, i32, i32, P]
        L.orc_containing.restype = None
        L.orc_position.argtypes = [P, i32, i32, i32]
        L.orc_position.restype = i32
        L.orc_length.argtypes = [P]
        L.orc_length.restype = i32
        L.orc_text.argtypes = [P, P, i32]
        L.orc_text.restype = i32
        L.orc_segments.argtypes = [P, P, i32]
        L.orc_segments.restype = i32
        L.orc_segment_props.argtypes = [P, i32, P, i32]
        L.orc_segment_props.restype = i32
        L.orc_leaves.argtypes = [P, P, i32]
        L.orc_leaves.restype = i32
        L.orc_checksum.argtypes = [P, P]
        L.orc_maintenance.argtypes = [P, P]
        L.orc_overlap_units.argtypes = [P, P]
        L.orc_deltas.argtypes = [P, P, i32]
        L.orc_deltas.restype = i32
        L.orc_set_record_deltas.argtypes = [P, i32]
        L.orc_generate.argtypes = [P, i32, P, i32, P, i32, P, P, i32, P, P, P, P]
        L.orc_generate.restype = i32
        L.orc_replay_batch.argtypes = [i32, P, P, P, P, P, P, P, P, i32]
        L.orc_replay_batch.restype = i32
        L.orc_load_replay_batch.argtypes = [i32, P, P, P, P, P, P, P, P, P, P, P, P, P, i32]
        L.orc_load_replay_batch.restype = i32
        L.orc_load.restype = P
        L.orc_load.argtypes = [P, i32, i32, P, P, i32, i32]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def make_cfg(cfg):
    th = gen_thresholds(cfg)
    return GenCfg(seed=cfg["seed"], ops=cfg["ops"], writers=cfg["writers"], lag=cfg["lag"],
                  seed_len=cfg["seed_len"], text_max=cfg["text_max"], n_keys=cfg["n_keys"],
                  n_values=cfg["n_values"], max_keys_per_op=cfg["max_keys_per_op"], **th)


class OracleDoc:
    def __init__(self, handle):
        self.h = handle

    def __del__(self):
        if self.h:
            lib().orc_free(self.h)
            self.h = None

    @classmethod
    def new(cls, seed):
        seed = np.ascontiguousarray(seed, dtype=np.uint16)
        d = cls(lib().orc_new(_p(seed), len(seed)))
        lib().orc_set_record_deltas(d.h, 1)
        return d

    @classmethod
    def load(cls, segs, n_header, text, props, min_seq, cur_seq):
        """A replica loaded from a decoded summary (orc_load = Client.load, MT/snapshotLoader.ts)."""
        segs = np.ascontiguousarray(segs)
        text = np.ascontiguousarray(text, dtype=np.uint16)
        props = np.ascontiguousarray(props, dtype=np.uint32)
        d = cls(lib().orc_load(_p(segs), int(n_header), len(segs), _p(text), _p(props), int(min_seq), int(cur_seq)))
        lib().orc_set_record_deltas(d.h, 1)
        return d

    def apply_all(self, ops, text, props):
        ops = np.ascontiguousarray(ops, dtype=OP_DTYPE)
        text = np.ascontiguousarray(text, dtype=np.uint16)
        props = np.ascontiguousarray(props, dtype=np.uint32)
        L = lib()
        base = ops.ctypes.data
        for i in range(len(ops)):
            st = L.orc_apply(self.h, ctypes.c_void_p(base + 32 * i), _p(text), _p(props))
            if st:
                return st
        return 0

    def pending_counts(self):
        """(collabWindow.localSeq, pending segment groups) of a live participant."""
        o = np.zeros(2, dtype=np.int32)
        lib().orc_pending_counts(self.h, _p(o))
        return int(o[0]), int(o[1])

    def regenerate(self, kind, cap=4096):
        """orc_regenerate: (records as REGEN_DTYPE, text, props) or None without a group."""
        from fluidframework_amd._native import REGEN_DTYPE
        recs = np.zeros(cap, dtype=REGEN_DTYPE)
        text = np.zeros(1 << 16, dtype=np.uint16)
        props = np.zeros(1 << 16, dtype=np.uint32)
        n = lib().orc_regenerate(self.h, int(kind), _p(recs), cap, _p(text), len(text), _p(props), len(props))
        if n == -1:
            return None
        if n < 0:
            raise RuntimeError(f"orc_regenerate failed ({n})")
        return recs[:n], text, props

    def maintenance(self):
        """[SPLIT, APPEND, UNLINK] mergeTreeMaintenanceCallback counts (orc_maintenance)."""
        m = np.zeros(3, dtype=np.uint32)
        lib().orc_maintenance(self.h, _p(m))
        return m.tolist()

    def overlap_units(self):
        """removedClientOverlap lists as overflow-set units: (now, peak after any message)."""
        m = np.zeros(2, dtype=np.int64)
        lib().orc_overlap_units(self.h, _p(m))
        return int(m[0]), int(m[1])

    def view_length(self, ref_seq, client):
        """MergeTree.getLength(refSeq, clientId) (partial lengths: stale views included)."""
        return int(lib().orc_view_length(self.h, int(ref_seq), int(client)))

    def containing(self, pos, ref_seq, client):
        """getContainingSegment in a view: (segment index, offset, position in the view,
        observer position), or None when the reference finds no segment."""
        o = np.zeros(4, dtype=np.int32)
        lib().orc_containing(self.h, int(pos), int(ref_seq), int(client), _p(o))
        return None if o[0] < 0 else tuple(int(x) for x in o)

    def outputs(self):
        L = lib()
        n = L.orc_text(self.h, None, 0)
        buf = np.zeros(max(n, 1), dtype=np.uint16)
        L.orc_text(self.h, _p(buf), n)
        text = buf[:n].tobytes().decode("utf-16-le", errors="surrogatepass")
        ns = L.orc_segments(self.h, None, 0)
        segs = np.zeros((max(ns, 1), 8), dtype=np.int32)
        L.orc_segments(self.h, _p(segs), ns)
        nl = L.orc_leaves(self.h, None, 0)
        leaves = np.zeros(max(nl, 1), dtype=np.int32)
        L.orc_leaves(self.h, _p(leaves), nl)
        nd = L.orc_deltas(self.h, None, 0)
        dl = np.zeros(max(nd, 1), dtype=np.int32)
        L.orc_deltas(self.h, _p(dl), nd)
        cs = np.zeros(1, dtype=CHECKSUM_DTYPE)
        L.orc_checksum(self.h, _p(cs))
        props = []
        pbuf = np.zeros(256, dtype=np.uint32)
        for i in range(ns):
            k = L.orc_segment_props(self.h, i, _p(pbuf), 128)
            props.append(None if k < 0 else [(int(pbuf[2 * j]), int(pbuf[2 * j + 1])) for j in range(k)])
        return dict(text=text, length=L.orc_length(self.h), segs=segs[:ns], leaves=leaves[:nl].tolist(),
                    deltas=dl[:nd].tolist(), checksum=cs[0], status=L.orc_status(self.h), seg_props=props)


def generate(cfg, doc, keep=False):
    """Generate one document's op stream (the oracle supplies the writers' view lengths)."""
    n = cfg["ops"]
    ops = np.zeros(n, dtype=OP_DTYPE)
    text = np.zeros(n * cfg["text_max"] + 16, dtype=np.uint16)
    props = np.zeros(n * (1 + 2 * cfg["max_keys_per_op"]) + 16, dtype=np.uint32)
    seed = np.zeros(max(cfg["seed_len"], 1), dtype=np.uint16)
    tu, pu, sl = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    keepp = ctypes.c_void_p()
    c = make_cfg(cfg)
    got = lib().orc_generate(ctypes.byref(c), doc, _p(ops), n, _p(text), len(text), ctypes.byref(tu),
                             _p(props), len(props), ctypes.byref(pu), _p(seed), ctypes.byref(sl),
                             ctypes.byref(keepp) if keep else None)
    if got < 0:
        raise RuntimeError(f"oracle generation failed for doc {doc}")
    out = dict(ops=ops[:got], text=text[:max(tu.value, 1)], props=props[:max(pu.value, 1)],
               seed=seed[:sl.value])
    if keep:
        d = OracleDoc(keepp.value)
        out["doc"] = d
    return out


def replay_batch(arrays, threads=1):
    n_docs = len(arrays["doc_off"]) - 1
    sums = np.zeros(n_docs, dtype=CHECKSUM_DTYPE)
    status = np.zeros(n_docs, dtype=np.int32)
    a = {k: np.ascontiguousarray(v) for k, v in arrays.items()}
    lib().orc_replay_batch(n_docs, _p(a["doc_off"]), _p(a["ops"]), _p(a["text"]), _p(a["props"]),
                           _p(a["seed_off"]), _p(a["seed"]), _p(sums), _p(status), threads)
    return sums, status


def load_replay_batch(load, arrays, threads=1):
    """Config C5 on the CPU: every document's summary loaded (orc_load), then its ops."""
    n_docs = len(arrays["doc_off"]) - 1
    sums = np.zeros(n_docs, dtype=CHECKSUM_DTYPE)
    status = np.zeros(n_docs, dtype=np.int32)
    la = {k: np.ascontiguousarray(v) for k, v in load.items()}
    a = {k: np.ascontiguousarray(v) for k, v in arrays.items()}
    lib().orc_load_replay_batch(n_docs, _p(la["doc_off"]), _p(la["n_header"]), _p(la["segs"]), _p(la["text"]),
                                _p(la["props"]), _p(la["min_seq"]), _p(la["cur_seq"]), _p(a["doc_off"]),
                                _p(a["ops"]), _p(a["text"]), _p(a["props"]), _p(sums), _p(status), threads)
    return sums, status
