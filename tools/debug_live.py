"""Debug tool (GPU box): replays live-client streams event by event (tools/_live_trace.json,
made by oracle/ref_harness.mjs live with "trace": 1) and reports the first event after which
the GPU's local text differs from the reference's, or the document fails."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from fluidframework_amd.live import LiveClient  # noqa: E402
from fluidframework_amd.wire import Interner  # noqa: E402


def main(path, batch=False, log=False):
    fx = json.load(open(path))
    print(f"--- batch={batch} log={log}")
    for doc in fx["docs"]:
        lc = LiveClient(doc["seed_text"], seg_capacity=16384, text_capacity=1 << 17, interner=Interner(synthetic=True),
                        delta_log_capacity=(1 << 20) if log else 0)
        lc.startOrUpdateCollaboration("local-0")
        unseq = []
        trace = doc["out"]["trace"] + [doc["out"]["text"]]
        INT_MIN = -2 ** 31
        for i, ev in enumerate(doc["events"]):
            try:
                if ev[0] == "L":
                    op = ev[1]
                    if op["type"] == 0:
                        lc.insertSegmentLocal(op["pos1"], op["seg"])
                    elif op["type"] == 1:
                        lc.removeRangeLocal(op["pos1"], op["pos2"])
                    else:
                        lc.annotateRangeLocal(op["pos1"], op["pos2"], op["props"], op.get("combiningOp"))
                    unseq.append(op)
                elif ev[0] == "M":
                    if ev[1] == lc.long_client_id:
                        unseq.pop(0)
                    _, cid, seq, ref, msn, op = ev
                    lc.applyMsg(dict(clientId=cid, sequenceNumber=seq, referenceSequenceNumber=ref,
                                     minimumSequenceNumber=msn, type="op", contents=op))
                else:
                    lc.startOrUpdateCollaboration(ev[1])
                    got = [lc.regeneratePendingOp(o) for o in unseq]
                    if got != ev[2]:
                        print(f"doc {doc['doc']} event {i}: regenerated ops differ")
                        for g, e in zip(got, ev[2]):
                            if g != e:
                                print("   got", g, "\n   exp", e)
                        break
                    unseq = ev[2]
                if batch and i + 1 < len(doc["events"]):
                    continue
                t = lc.getText()
            except RuntimeError as e:
                hdr = np.zeros(32, np.int32)
                lc.mt.lib.mt_debug_raw(lc.mt.h, 0, None, 0, None, hdr.ctypes.data)
                print(f"doc {doc['doc']} event {i} {ev}: {e}; diag {hdr[27]}")
                print("  previous events:", doc["events"][max(0, i - 3):i])
                break
            tr = trace[i]
            if isinstance(tr, list) and batch:
                tr = tr[0]
            if isinstance(tr, list):
                tr, rsegs, rleaves, rheap, rflags = tr
                rows, leaves = lc.mt.get_segments(0)
                hp = np.zeros(2 * 4096, np.int32)
                fl = np.zeros(4096, np.int32)
                nh = ctypes.c_uint32(0)
                nf = ctypes.c_uint32(0)
                lc.mt.lib.mt_debug_heap(lc.mt.h, 0, hp.ctypes.data, 4096, ctypes.byref(nh), fl.ctypes.data, 4096,
                                        ctypes.byref(nf))
                gheap = hp[:2 * nh.value].reshape(-1, 2).tolist()
                gflags = fl[:nf.value].tolist()
                if gheap != rheap or gflags != rflags:
                    print(f"doc {doc['doc']} event {i} {ev}: heap or flags differ")
                    print("  previous events:", doc["events"][max(0, i - 3):i])
                    print("  got heap", gheap)
                    print("  exp heap", rheap)
                    print("  got flags", gflags)
                    print("  exp flags", rflags)
                    break
                g = [[int(r[0]), int(r[1]), None if r[3] == INT_MIN else int(r[3])] for r in rows]
                e = [rsegs[4 * j:4 * j + 3] for j in range(len(rsegs) // 4)]
                if g != e or list(leaves) != rleaves:
                    k = next((j for j in range(min(len(g), len(e))) if g[j] != e[j]), min(len(g), len(e)))
                    print(f"doc {doc['doc']} event {i} {ev}: segment table differs at {k} (leaves equal: {list(leaves) == rleaves})")
                    print("  previous events:", doc["events"][max(0, i - 3):i])
                    print("  got", g[max(0, k - 4):k + 6])
                    print("  exp", [rsegs[4 * j:4 * j + 4] for j in range(max(0, k - 4), min(len(e), k + 6))])
                    print("  got leaves", list(leaves)[:40])
                    print("  exp leaves", rleaves[:40])
                    break
            if t != tr:
                k = next((j for j in range(min(len(t), len(tr))) if t[j] != tr[j]), min(len(t), len(tr)))
                print(f"doc {doc['doc']} event {i} {ev}: text differs at {k}: got {t[max(0,k-10):k+20]!r} exp {tr[max(0,k-10):k+20]!r}")
                print("  previous events:", doc["events"][max(0, i - 3):i])
                rows, leaves = lc.mt.get_segments(0)
                print("  segs:", rows.tolist()[:60])
                break
        else:
            print(f"doc {doc['doc']}: all {len(doc['events'])} events match")
        lc.close()


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    path = args[0] if args else os.path.join(os.path.dirname(os.path.abspath(__file__)), "_live_trace.json")
    main(path, batch="--batch" in sys.argv, log="--log" in sys.argv)
