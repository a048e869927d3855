"""Live-client path: a participant `Client` -- one that submits its own ops
-- backed by a document on the GPU.

`LiveClient` mirrors the reference `Client`'s local surface (MT/client.ts):
`startOrUpdateCollaboration` (:1053-1073), `insertSegmentLocal` / `removeRangeLocal` /
`annotateRangeLocal` (:164-211, with `getValidOpRange`'s validation :486-548), `applyMsg`
(:797-819: the echo of one of its own ops acks it, `ackPendingSegment` :589-626),
`regeneratePendingOp` (:855-893) after a reconnect, and the read-outs (`getText`,
`getLength`, `getPropertiesAtPosition`, `getCurrentSeq`).  The merge-tree work -- the local
ops' UnassignedSequenceNumber segments, segment groups, acks, remote ops resolved around
unacked segments, reconnect positions -- runs in the HIP engine (TierLiveT in
csrc/mt_engine.h, k_regen in csrc/mt_replay.hip).  Calls are queued and applied as one
batch on the next read or `flush()`; there is no CPU fallback.
"""
import numpy as np

from . import MergeTreeBatch
from .wire import NO_PROPS as MT_NO_PROPS_U32, Batch, Interner

OP_INSERT, OP_REMOVE, OP_ANNOTATE, OP_GROUP = 0, 1, 2, 3
F_MARKER = 2


def regen_op(interner, reset, rec, text, props):
    """One mt_regen_rec (include/mt_replay.h) -> the op regeneratePendingOp returns
    (OpBuilder.createInsertSegmentOp / createRemoveRangeOp / createAnnotateRangeOp)."""
    kind = int(rec["kind"])
    if kind == OP_INSERT:
        pset = None
        if int(rec["props_off"]) != MT_NO_PROPS_U32:
            o = int(rec["props_off"])
            n = int(props[o])
            pset = {interner.key_name(int(props[o + 1 + 2 * j])):
                    interner.val_value(int(props[o + 2 + 2 * j])) for j in range(n)}
        if int(rec["flags"]) & F_MARKER:
            seg = {"marker": {"refType": int(rec["text_off"])}}
        else:
            t0, tl = int(rec["text_off"]), int(rec["text_len"])
            s = text[t0:t0 + tl].tobytes().decode("utf-16-le")
            seg = {"text": s} if pset is not None else s
        if pset is not None:
            seg["props"] = pset
        return {"pos1": int(rec["pos1"]), "seg": seg, "type": OP_INSERT}
    if kind == OP_REMOVE:
        return {"pos1": int(rec["pos1"]), "pos2": int(rec["pos2"]), "type": OP_REMOVE}
    op = {"pos1": int(rec["pos1"]), "pos2": int(rec["pos2"]), "props": reset["props"], "type": OP_ANNOTATE}
    if reset.get("combiningOp") is not None:
        op["combiningOp"] = reset["combiningOp"]
    return op


class LiveClient:
    """One GPU document replica owned by a participant client (short id 0)."""

    def __init__(self, seed_text="", device=0, seg_capacity=4096, text_capacity=1 << 16, delta_log_capacity=0,
                 interner=None, lds_seg_capacity=-1, live_group_capacity=0):
        # lds_seg_capacity > 0: each flush stages the document in LDS (TierLiveLdsT) while it
        # fits, continuing in the HBM tier when it outgrows it.  The capacities are where the
        # document starts: the live growth step raises what it outgrows (mt_replay.hip)
        self.mt = MergeTreeBatch(1, device=device, seg_capacity=seg_capacity, text_capacity=text_capacity,
                                 lds_seg_capacity=lds_seg_capacity, delta_log_capacity=delta_log_capacity,
                                 live_client=1, live_group_capacity=live_group_capacity)
        units = np.frombuffer(seed_text.encode("utf-16-le"), dtype="<u2")
        self.mt.load_initial_text(np.array([0, len(units)], dtype=np.int64),
                                  units if len(units) else np.zeros(1, dtype=np.uint16))
        self.interner = interner or Interner()
        self.short = {}              # long client id -> short id (the local client's ids -> 0)
        self.long_client_id = None
        self.queue = []              # ("local" | "ack" | "msg", op / message) not yet applied
        self.log = []                # delta-log words drained so far (delta_log_capacity > 0)

    # -------------------------------------------------------------- collaboration
    def startOrUpdateCollaboration(self, long_client_id, min_seq=0, current_seq=0):
        """MT/client.ts:1053-1073: the first id starts collaboration (short id 0); a later one
        (reconnect) renames the local client -- its old ids keep mapping to short id 0."""
        if long_client_id is None:
            return
        if self.long_client_id is None:
            self.short[long_client_id] = 0
            self.mt.start_collaboration(np.array([min_seq], np.int32), np.array([current_seq], np.int32))
        else:
            self.short[long_client_id] = 0
        self.long_client_id = long_client_id

    # -------------------------------------------------------------- local ops
    def _valid_range(self, start, end, insert):
        """getValidOpRange for a local op (MT/client.ts:505-545)."""
        length = self.getLength()
        if start is None or start < 0 or start > length or (start == length and not insert):
            return False
        if not insert or end is not None:
            if end is None or end <= start:
                return False
        return True

    def insertSegmentLocal(self, pos, seg):
        """seg: the segment's JSON (a string, {"text", "props"} or {"marker", "props"}); returns
        the op to submit, or None (MT/client.ts:202-211)."""
        if isinstance(seg, str) and len(seg) == 0:
            return None
        if not self._valid_range(pos, None, True):
            return None
        op = {"pos1": pos, "seg": seg, "type": OP_INSERT}
        self.queue.append(("local", op))
        return op

    def removeRangeLocal(self, start, end):
        if not self._valid_range(start, end, False):
            return None
        op = {"pos1": start, "pos2": end, "type": OP_REMOVE}
        self.queue.append(("local", op))
        return op

    def annotateRangeLocal(self, start, end, props, combining_op=None):
        if not self._valid_range(start, end, False):
            return None
        op = {"pos1": start, "pos2": end, "props": props, "type": OP_ANNOTATE}
        if combining_op is not None:
            op["combiningOp"] = combining_op
        self.queue.append(("local", op))
        return op

    def localTransaction(self, group_op):
        """MT/client.ts:961-981: every member of a local GROUP op applied as its own local op
        (each with its own segment group; the GROUP's echo acks them member by member)."""
        for op in group_op["ops"]:
            if op["type"] == OP_INSERT:
                self.insertSegmentLocal(op["pos1"], op["seg"])
            elif op["type"] == OP_REMOVE:
                self.removeRangeLocal(op["pos1"], op["pos2"])
            elif op["type"] == OP_ANNOTATE:
                self.annotateRangeLocal(op["pos1"], op["pos2"], op["props"], op.get("combiningOp"))

    # -------------------------------------------------------------- sequenced messages
    def applyMsg(self, msg):
        self.queue.append(("ack" if msg["clientId"] == self.long_client_id else "msg", msg))

    def flush(self):
        if not self.queue:
            return
        b = Batch(self.interner)
        b.add_live_doc("", self.queue, self.short)
        self.short = b.clients[-1]
        self.queue = []
        a = b.arrays()
        self.mt.apply_arrays(a)
        st = int(self.mt.status()[0])
        if st:
            hdr = np.zeros(32, np.int32)
            self.mt.lib.mt_debug_raw(self.mt.h, 0, None, 0, None, hdr.ctypes.data)
            raise RuntimeError(f"live document failed: mt_doc_status {st} (diagnostic {int(hdr[27])})")

    # -------------------------------------------------------------- reconnect
    def regeneratePendingOp(self, reset_op):
        """MT/client.ts:855-893: rebuild a pending op (the oldest one: the caller resubmits its
        pending ops in order) for resubmission.  A GROUP is rebuilt member by member."""
        self.flush()
        members = reset_op["ops"] if reset_op["type"] == OP_GROUP else [reset_op]
        ops = []
        for m in members:
            r = self.mt.regenerate_pending(0)
            if r is None:
                raise RuntimeError("regeneratePendingOp: no pending segment group")
            recs, text, props = r
            for rec in recs:
                ops.append(self._regen_op(m, rec, text, props))
        return ops[0] if len(ops) == 1 else {"ops": ops, "type": OP_GROUP}

    def _regen_op(self, reset, rec, text, props):
        return regen_op(self.interner, reset, rec, text, props)

    # -------------------------------------------------------------- read-outs (local view)
    def getLength(self):
        self.flush()
        return self.mt.get_length(0)

    def getText(self):
        self.flush()
        return self.mt.get_text(0)

    def getPropertiesAtPosition(self, pos):
        self.flush()
        return self.mt.get_properties_at_position(0, pos)

    def pendingCounts(self):
        """(collabWindow.localSeq, pending segment groups)."""
        self.flush()
        ls, ng = self.mt.pending_counts()[0]
        return int(ls), int(ng)

    def close(self):
        self.mt.close()
