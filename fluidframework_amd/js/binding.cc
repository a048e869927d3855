// binding.cc -- thin N-API addon over the C ABI of include/mt_replay.h (libmtreplay.so) and
// the summary decoder of include/mt_snapshot.h (libmtsnapdec.so).
//
// The reference's host language is TypeScript on Node; its merge-tree boundary is the
// class Client (packages/dds/merge-tree/src/client.ts:43) fed by
// SharedSegmentSequence.processMergeTreeMsg -> client.applyMsg
// (packages/dds/sequence/src/sequence.ts:579-600).  This addon exposes the batched
// replacement to JS; js/index.js builds the Client-shaped facade on top of it and
// js/encode.js turns ISequencedDocumentMessage objects into the binary wire format.
//
// Ownership: JS owns the message buffers (typed arrays); mt_apply_ops copies them to the
// device.  The handle (device state) is owned by a JS external whose finalizer calls
// mt_destroy.  Errors: negative MT_E_* codes become thrown JS Errors carrying
// mt_last_error(); per-document failures are reported through status().
//
// Build (node-gyp is not available offline): fluidframework_amd/js/build.sh.
#include <node_api.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mt_replay.h"
#include "../../include/mt_snapshot.h"

namespace {

#define NAPI_CALL(env, call)                                                \
    do {                                                                    \
        if ((call) != napi_ok) {                                            \
            napi_throw_error((env), nullptr, "N-API call failed: " #call); \
            return nullptr;                                                 \
        }                                                                   \
    } while (0)

struct Handle {
    mt_handle *h = nullptr;
};

void finalize_handle(napi_env, void *data, void *) {
    auto *hd = static_cast<Handle *>(data);
    if (hd->h) mt_destroy(hd->h);
    delete hd;
}

napi_value throw_rc(napi_env env, const Handle *hd, int rc, const char *what) {
    std::string msg = std::string(what) + " failed (" + std::to_string(rc) + "): " +
                      (hd && hd->h ? mt_last_error(hd->h) : "");
    napi_throw_error(env, nullptr, msg.c_str());
    return nullptr;
}

bool get_args(napi_env env, napi_callback_info info, size_t n, napi_value *argv) {
    size_t argc = n;
    if (napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr) != napi_ok || argc < n) {
        napi_throw_type_error(env, nullptr, "wrong number of arguments");
        return false;
    }
    return true;
}

Handle *get_handle(napi_env env, napi_value v) {
    void *p = nullptr;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p || !static_cast<Handle *>(p)->h) {
        napi_throw_type_error(env, nullptr, "invalid or destroyed handle");
        return nullptr;
    }
    return static_cast<Handle *>(p);
}

// data pointer + element count of any TypedArray
bool typed(napi_env env, napi_value v, void **data, size_t *len) {
    napi_typedarray_type t;
    napi_value ab;
    size_t off;
    if (napi_get_typedarray_info(env, v, &t, len, data, &ab, &off) != napi_ok) {
        napi_throw_type_error(env, nullptr, "expected a TypedArray");
        return false;
    }
    return true;
}

int32_t get_i32(napi_env env, napi_value v) {
    int32_t x = 0;
    napi_get_value_int32(env, v, &x);
    return x;
}

napi_value make_u32(napi_env env, uint32_t x) {
    napi_value r;
    napi_create_uint32(env, x, &r);
    return r;
}

// create(nDocs, {device, segCapacity, ...}) -> external handle  (mt_create)
napi_value Create(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    uint32_t n = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[0], &n));
    mt_options o;
    memset(&o, 0, sizeof(o));
    const char *names[] = {"device", "segCapacity", "blockCapacity", "heapCapacity", "textCapacity",
                           "propsCapacity", "deltaLogCapacity", "ldsSegCapacity", "pageCapacity",
                           "pageHeapCapacity", "unsettledCapacity", "uidCapacity", "ldsPageCapacity",
                           "ldsUnsettledCapacity", "ldsPageHeapCapacity", "ldsNarrowOverlap", "deltaLogMode",
                           "liveClient", "liveGroupCapacity", "pagedSlices", "segmentOrdinals",
                           "overlapArenaCapacity"};
    int32_t *fields[] = {&o.device, &o.seg_capacity, &o.block_capacity, &o.heap_capacity, &o.text_capacity,
                         &o.props_capacity, &o.delta_log_capacity, &o.lds_seg_capacity, &o.page_capacity,
                         &o.page_heap_capacity, &o.unsettled_capacity, &o.uid_capacity, &o.lds_page_capacity,
                         &o.lds_unsettled_capacity, &o.lds_page_heap_capacity, &o.lds_narrow_overlap,
                         &o.delta_log_mode, &o.live_client, &o.live_group_capacity, &o.paged_slices,
                         &o.segment_ordinals, &o.overlap_arena_capacity};
    for (int i = 0; i < 22; i++) {
        bool has = false;
        napi_has_named_property(env, argv[1], names[i], &has);
        if (has) {
            napi_value v;
            napi_get_named_property(env, argv[1], names[i], &v);
            *fields[i] = get_i32(env, v);
        }
    }
    auto *hd = new Handle();
    hd->h = mt_create(n, &o);
    if (!hd->h) {
        delete hd;
        napi_throw_error(env, nullptr,
                         "mt_create failed: no HIP device visible or out of device memory "
                         "(the replay backend has no CPU fallback)");
        return nullptr;
    }
    napi_value ext;
    NAPI_CALL(env, napi_create_external(env, hd, finalize_handle, nullptr, &ext));
    return ext;
}

napi_value Destroy(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    void *p = nullptr;
    NAPI_CALL(env, napi_get_value_external(env, argv[0], &p));
    auto *hd = static_cast<Handle *>(p);
    if (hd && hd->h) {
        mt_destroy(hd->h);
        hd->h = nullptr;
    }
    return nullptr;
}

// loadInitialText(h, seedOff: BigInt64Array, seed: Uint16Array)
napi_value LoadInitialText(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    void *off, *txt;
    size_t noff, ntxt;
    if (!typed(env, argv[1], &off, &noff) || !typed(env, argv[2], &txt, &ntxt)) return nullptr;
    if (noff != mt_num_docs(hd->h) + 1) {
        napi_throw_range_error(env, nullptr, "seedOff must hold nDocs + 1 offsets");
        return nullptr;
    }
    const int64_t *so = (const int64_t *)off;
    if (so[0] != 0 || so[noff - 1] < 0 || (uint64_t)so[noff - 1] > ntxt) {
        napi_throw_range_error(env, nullptr, "seedOff exceeds the seed text");
        return nullptr;
    }
    const int rc = mt_load_initial_text(hd->h, (const int64_t *)off, (const uint16_t *)txt);
    if (rc) return throw_rc(env, hd, rc, "mt_load_initial_text");
    return nullptr;
}

// startCollaboration(h, minSeq: Int32Array, currentSeq: Int32Array) -- per document, -1 = leave
napi_value StartCollaboration(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    void *ms, *cs;
    size_t nms, ncs;
    if (!typed(env, argv[1], &ms, &nms) || !typed(env, argv[2], &cs, &ncs)) return nullptr;
    if (nms != mt_num_docs(hd->h) || ncs != nms) {
        napi_throw_range_error(env, nullptr, "minSeq / currentSeq must hold one entry per document");
        return nullptr;
    }
    const int rc = mt_start_collaboration(hd->h, (const int32_t *)ms, (const int32_t *)cs);
    if (rc) return throw_rc(env, hd, rc, "mt_start_collaboration");
    return nullptr;
}

// applyOps(h, docOff: BigInt64Array, ops: Uint8Array (32-byte records), text: Uint16Array,
//          props: Uint32Array) -- Client.applyMsg for every message (mt_apply_ops)
napi_value ApplyOps(napi_env env, napi_callback_info info) {
    napi_value argv[5];
    if (!get_args(env, info, 5, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    void *off, *ops, *txt, *props;
    size_t noff, nops, ntxt, nprops;
    if (!typed(env, argv[1], &off, &noff) || !typed(env, argv[2], &ops, &nops) ||
        !typed(env, argv[3], &txt, &ntxt) || !typed(env, argv[4], &props, &nprops))
        return nullptr;
    if (noff != mt_num_docs(hd->h) + 1 || nops % sizeof(mt_op_rec) != 0) {
        napi_throw_range_error(env, nullptr, "docOff must hold nDocs + 1 offsets; ops whole 32-byte records");
        return nullptr;
    }
    const int rc = mt_apply_ops(hd->h, (const int64_t *)off, (const mt_op_rec *)ops, nops / sizeof(mt_op_rec),
                                (const uint16_t *)txt, ntxt, (const uint32_t *)props, nprops);
    if (rc) return throw_rc(env, hd, rc, "mt_apply_ops");
    return nullptr;
}

// applyOpsAsync(h, docOff, ops, text, props) -> Promise: mt_apply_ops on a worker thread
// (napi_async_work) so the Node thread keeps running while the GPU applies the batch.  The
// typed arrays are pinned by references until the work completes; the facade issues no other
// call on the handle meanwhile (a handle is single-writer).
struct ApplyWork {
    napi_async_work work = nullptr;
    napi_deferred deferred = nullptr;
    napi_ref refs[4] = {nullptr, nullptr, nullptr, nullptr};
    napi_ref href = nullptr;
    Handle *hd = nullptr;
    const int64_t *off = nullptr;
    const mt_op_rec *ops = nullptr;
    uint64_t n_ops = 0;
    const uint16_t *text = nullptr;
    uint64_t n_text = 0;
    const uint32_t *props = nullptr;
    uint64_t n_props = 0;
    int rc = 0;
    std::string err;
};
void apply_execute(napi_env, void *data) {
    auto *w = static_cast<ApplyWork *>(data);
    w->rc = mt_apply_ops(w->hd->h, w->off, w->ops, w->n_ops, w->text, w->n_text, w->props, w->n_props);
    if (w->rc) w->err = std::string("mt_apply_ops failed (") + std::to_string(w->rc) + "): " + mt_last_error(w->hd->h);
}
void apply_complete(napi_env env, napi_status, void *data) {
    auto *w = static_cast<ApplyWork *>(data);
    if (w->rc == 0) {
        napi_value u;
        napi_get_undefined(env, &u);
        napi_resolve_deferred(env, w->deferred, u);
    } else {
        napi_value msg, e;
        napi_create_string_utf8(env, w->err.c_str(), NAPI_AUTO_LENGTH, &msg);
        napi_create_error(env, nullptr, msg, &e);
        napi_reject_deferred(env, w->deferred, e);
    }
    for (napi_ref r : w->refs)
        if (r) napi_delete_reference(env, r);
    if (w->href) napi_delete_reference(env, w->href);
    napi_delete_async_work(env, w->work);
    delete w;
}
napi_value ApplyOpsAsync(napi_env env, napi_callback_info info) {
    napi_value argv[5];
    if (!get_args(env, info, 5, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    void *off, *ops, *txt, *props;
    size_t noff, nops, ntxt, nprops;
    if (!typed(env, argv[1], &off, &noff) || !typed(env, argv[2], &ops, &nops) ||
        !typed(env, argv[3], &txt, &ntxt) || !typed(env, argv[4], &props, &nprops))
        return nullptr;
    if (noff != mt_num_docs(hd->h) + 1 || nops % sizeof(mt_op_rec) != 0) {
        napi_throw_range_error(env, nullptr, "docOff must hold nDocs + 1 offsets; ops whole 32-byte records");
        return nullptr;
    }
    auto *w = new ApplyWork();
    w->hd = hd;
    w->off = (const int64_t *)off;
    w->ops = (const mt_op_rec *)ops;
    w->n_ops = nops / sizeof(mt_op_rec);
    w->text = (const uint16_t *)txt;
    w->n_text = ntxt;
    w->props = (const uint32_t *)props;
    w->n_props = nprops;
    for (int i = 0; i < 4; i++) NAPI_CALL(env, napi_create_reference(env, argv[1 + i], 1, &w->refs[i]));
    NAPI_CALL(env, napi_create_reference(env, argv[0], 1, &w->href));
    napi_value promise, name;
    NAPI_CALL(env, napi_create_promise(env, &w->deferred, &promise));
    NAPI_CALL(env, napi_create_string_utf8(env, "mt_apply_ops", NAPI_AUTO_LENGTH, &name));
    NAPI_CALL(env, napi_create_async_work(env, nullptr, name, apply_execute, apply_complete, w, &w->work));
    NAPI_CALL(env, napi_queue_async_work(env, w->work));
    return promise;
}

// a segment read-out (mt_seg_info) as a JS object, or null
napi_value seg_info_object(napi_env env, const mt_seg_info &s, const uint16_t *text) {
    napi_value o, v;
    if (s.row < 0) {
        napi_get_null(env, &o);
        return o;
    }
    napi_create_object(env, &o);
    const struct {
        const char *k;
        int64_t v;
    } fs[] = {{"row", s.row}, {"uid", (int64_t)s.uid}, {"position", s.position}, {"offset", s.offset},
              {"length", s.length}, {"seq", s.seq}, {"clientId", s.client}, {"removedSeq", s.removed_seq},
              {"removedClientId", s.removed_client}, {"markerRefType", s.marker_ref_type}};
    for (const auto &f : fs) {
        napi_create_int64(env, f.v, &v);
        napi_set_named_property(env, o, f.k, v);
    }
    if (s.marker_ref_type < 0) {
        napi_create_string_utf16(env, (const char16_t *)text, (size_t)s.text_len, &v);
        napi_set_named_property(env, o, "text", v);
    }
    if (s.ordinal_len >= 0) {
        napi_create_string_utf16(env, (const char16_t *)s.ordinal, (size_t)s.ordinal_len, &v);
        napi_set_named_property(env, o, "ordinal", v);
    }
    return o;
}
// getContainingSegment(h, doc, pos, refSeq, clientId) / getSegmentByUid(h, doc, uid, refSeq,
// clientId) -> {row, uid, position, offset, length, seq, clientId, removedSeq, removedClientId,
// markerRefType, text?, ordinal?} | null
napi_value SegmentQuery(napi_env env, napi_callback_info info, bool by_uid) {
    napi_value argv[5];
    if (!get_args(env, info, 5, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    uint32_t doc = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    double key = 0;
    NAPI_CALL(env, napi_get_value_double(env, argv[2], &key));
    const int32_t ref = get_i32(env, argv[3]), cli = get_i32(env, argv[4]);
    if (doc >= mt_num_docs(hd->h) || !(key >= 0 && key <= 4294967295.0)) {
        napi_throw_range_error(env, nullptr, "document index or position out of range");
        return nullptr;
    }
    std::vector<uint16_t> text(1 << 16);
    mt_seg_info s;
    const int rc = by_uid ? mt_get_segment_by_uid(hd->h, doc, (uint32_t)key, ref, cli, &s, text.data(), (uint32_t)text.size())
                          : mt_get_containing_segment(hd->h, doc, (int32_t)key, ref, cli, &s, text.data(),
                                                      (uint32_t)text.size());
    if (rc) return throw_rc(env, hd, rc, by_uid ? "mt_get_segment_by_uid" : "mt_get_containing_segment");
    napi_value o = seg_info_object(env, s, text.data());
    if (s.row >= 0) {   // its property set: propPairs = [key id, value id]* (null: none)
        std::vector<uint32_t> pairs(2 * 64);
        int32_t np = 0;
        const int rc2 = mt_get_segment_props(hd->h, doc, (uint32_t)s.row, pairs.data(), 64, &np);
        if (rc2) return throw_rc(env, hd, rc2, "mt_get_segment_props");
        napi_value v;
        if (np < 0) {
            napi_get_null(env, &v);
        } else {
            void *pd = nullptr;
            napi_value ab;
            NAPI_CALL(env, napi_create_arraybuffer(env, std::max<size_t>(2 * np, 1) * 4, &pd, &ab));
            memcpy(pd, pairs.data(), 2 * (size_t)np * 4);
            NAPI_CALL(env, napi_create_typedarray(env, napi_uint32_array, 2 * (size_t)np, ab, 0, &v));
        }
        napi_set_named_property(env, o, "propPairs", v);
    }
    return o;
}
napi_value GetContainingSegment(napi_env env, napi_callback_info info) { return SegmentQuery(env, info, false); }
napi_value GetSegmentByUid(napi_env env, napi_callback_info info) { return SegmentQuery(env, info, true); }

// getViewLengths(h, docs: Uint32Array, refSeq: Int32Array, clientId: Int32Array) -> Int32Array
napi_value GetViewLengths(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (!get_args(env, info, 4, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    void *docs, *ref, *cli;
    size_t nd, nr, nc;
    if (!typed(env, argv[1], &docs, &nd) || !typed(env, argv[2], &ref, &nr) || !typed(env, argv[3], &cli, &nc)) return nullptr;
    if (nr != nd || nc != nd) {
        napi_throw_range_error(env, nullptr, "one refSeq and clientId per query");
        return nullptr;
    }
    for (size_t q = 0; q < nd; q++)
        if (((const uint32_t *)docs)[q] >= mt_num_docs(hd->h)) {
            napi_throw_range_error(env, nullptr, "document index out of range");
            return nullptr;
        }
    napi_value ab, out;
    void *pd = nullptr;
    NAPI_CALL(env, napi_create_arraybuffer(env, std::max<size_t>(nd, 1) * 4, &pd, &ab));
    const int rc = mt_get_view_lengths(hd->h, (uint32_t)nd, (const uint32_t *)docs, (const int32_t *)ref,
                                       (const int32_t *)cli, (int32_t *)pd);
    if (rc) return throw_rc(env, hd, rc, "mt_get_view_lengths");
    NAPI_CALL(env, napi_create_typedarray(env, napi_int32_array, nd, ab, 0, &out));
    return out;
}

// extractSnapshots(h) -> {counts: BigInt64Array[3 nDocs], segs: Uint8Array (32-byte mt_seg_rec),
// text: Uint16Array, props: Uint32Array, minSeq: Int32Array, curSeq: Int32Array} --
// SnapshotV1.extractSync of every document (mt_extract_snapshots; snapshotV1.ts:156-252)
napi_value ExtractSnapshots(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    const uint32_t nd = mt_num_docs(hd->h);
    std::vector<int64_t> io(3 * (size_t)nd);
    int rc = mt_extract_snapshots(hd->h, io.data(), nullptr, nullptr, nullptr, nullptr, nullptr);
    if (rc) return throw_rc(env, hd, rc, "mt_extract_snapshots");
    uint64_t tr = 0, tt = 0, tp = 0;
    for (uint32_t d = 0; d < nd; d++) {
        tr += io[3 * d];
        tt += io[3 * d + 1];
        tp += io[3 * d + 2];
    }
    struct Arr {
        const char *name;
        napi_typedarray_type t;
        size_t n, esz;
    } arrs[] = {{"counts", napi_bigint64_array, 3 * (size_t)nd, 8}, {"segs", napi_uint8_array, tr * sizeof(mt_seg_rec), 1},
                {"text", napi_uint16_array, tt, 2},      {"props", napi_uint32_array, tp, 4},
                {"minSeq", napi_int32_array, nd, 4},     {"curSeq", napi_int32_array, nd, 4}};
    napi_value out;
    NAPI_CALL(env, napi_create_object(env, &out));
    void *pd[6] = {};
    for (int i = 0; i < 6; i++) {
        napi_value ab, a;
        NAPI_CALL(env, napi_create_arraybuffer(env, std::max<size_t>(arrs[i].n, 1) * arrs[i].esz, &pd[i], &ab));
        NAPI_CALL(env, napi_create_typedarray(env, arrs[i].t, arrs[i].n, ab, 0, &a));
        NAPI_CALL(env, napi_set_named_property(env, out, arrs[i].name, a));
    }
    memcpy(pd[0], io.data(), io.size() * 8);
    rc = mt_extract_snapshots(hd->h, (int64_t *)pd[0], (mt_seg_rec *)pd[1], (uint16_t *)pd[2], (uint32_t *)pd[3],
                              (int32_t *)pd[4], (int32_t *)pd[5]);
    if (rc) return throw_rc(env, hd, rc, "mt_extract_snapshots");
    return out;
}

// loadSnapshots(h, docSegOff: BigInt64Array, nHeader: Int32Array, segs: Uint8Array (32-byte
//               mt_seg_rec), text: Uint16Array, props: Uint32Array, minSeq: Int32Array,
//               curSeq: Int32Array) -- Client.load of a decoded summary into every document
//               (mt_load_snapshots; snapshotLoader.ts:36-228)
napi_value LoadSnapshots(napi_env env, napi_callback_info info) {
    napi_value argv[8];
    if (!get_args(env, info, 8, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    void *off, *nh, *segs, *txt, *props, *mn, *cu;
    size_t noff, nnh, nsegs, ntxt, nprops, nmn, ncu;
    if (!typed(env, argv[1], &off, &noff) || !typed(env, argv[2], &nh, &nnh) || !typed(env, argv[3], &segs, &nsegs) ||
        !typed(env, argv[4], &txt, &ntxt) || !typed(env, argv[5], &props, &nprops) || !typed(env, argv[6], &mn, &nmn) ||
        !typed(env, argv[7], &cu, &ncu))
        return nullptr;
    const uint32_t nd = mt_num_docs(hd->h);
    if (noff != nd + 1 || nnh != nd || nmn != nd || ncu != nd || nsegs % sizeof(mt_seg_rec) != 0) {
        napi_throw_range_error(env, nullptr, "one summary per document; segs whole 32-byte records");
        return nullptr;
    }
    const uint64_t n_recs = (uint64_t)((const int64_t *)off)[nd];
    if (n_recs * sizeof(mt_seg_rec) > nsegs) {
        napi_throw_range_error(env, nullptr, "docSegOff exceeds segs");
        return nullptr;
    }
    const int rc = mt_load_snapshots(hd->h, (const int64_t *)off, (const int32_t *)nh, (const mt_seg_rec *)segs, n_recs,
                                     (const uint16_t *)txt, ntxt, (const uint32_t *)props, nprops,
                                     (const int32_t *)mn, (const int32_t *)cu);
    if (rc) return throw_rc(env, hd, rc, "mt_load_snapshots");
    return nullptr;
}

// status(h) -> Int32Array[nDocs]   (enum mt_doc_status)
napi_value Status(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    const uint32_t n = mt_num_docs(hd->h);
    void *data;
    napi_value ab, arr;
    NAPI_CALL(env, napi_create_arraybuffer(env, (size_t)n * 4, &data, &ab));
    const int rc = mt_get_status(hd->h, (int32_t *)data);
    if (rc) return throw_rc(env, hd, rc, "mt_get_status");
    NAPI_CALL(env, napi_create_typedarray(env, napi_int32_array, n, ab, 0, &arr));
    return arr;
}

// getLength(h, doc) -> number   (Client.getLength, client.ts:1051)
napi_value GetLength(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    uint32_t len = 0;
    const int rc = mt_get_length(hd->h, (uint32_t)get_i32(env, argv[1]), &len);
    if (rc) return throw_rc(env, hd, rc, "mt_get_length");
    return make_u32(env, len);
}

// getText(h, doc) -> string   (MergeTreeTextHelper.getText, textSegment.ts:154-172)
napi_value GetText(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    const uint32_t doc = (uint32_t)get_i32(env, argv[1]);
    uint32_t n = 0;
    int rc = mt_get_text(hd->h, doc, nullptr, 0, &n);
    if (rc) return throw_rc(env, hd, rc, "mt_get_text");
    std::vector<uint16_t> buf(n ? n : 1);
    rc = mt_get_text(hd->h, doc, buf.data(), n, &n);
    if (rc) return throw_rc(env, hd, rc, "mt_get_text");
    napi_value s;
    NAPI_CALL(env, napi_create_string_utf16(env, (const char16_t *)buf.data(), n, &s));
    return s;
}

// getPropRuns(h, doc) -> {runs: Uint32Array (start, length, record) x n, records: Uint32Array}
napi_value GetPropRuns(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    const uint32_t doc = (uint32_t)get_i32(env, argv[1]);
    uint32_t nr = 0, nw = 0;
    int rc = mt_get_prop_runs(hd->h, doc, nullptr, 0, &nr, nullptr, 0, &nw);
    if (rc) return throw_rc(env, hd, rc, "mt_get_prop_runs");
    void *rd, *wd;
    napi_value rab, wab, ra, wa, obj;
    NAPI_CALL(env, napi_create_arraybuffer(env, (size_t)3 * nr * 4, &rd, &rab));
    NAPI_CALL(env, napi_create_arraybuffer(env, (size_t)nw * 4, &wd, &wab));
    rc = mt_get_prop_runs(hd->h, doc, (uint32_t *)rd, nr, &nr, (uint32_t *)wd, nw, &nw);
    if (rc) return throw_rc(env, hd, rc, "mt_get_prop_runs");
    NAPI_CALL(env, napi_create_typedarray(env, napi_uint32_array, (size_t)3 * nr, rab, 0, &ra));
    NAPI_CALL(env, napi_create_typedarray(env, napi_uint32_array, nw, wab, 0, &wa));
    NAPI_CALL(env, napi_create_object(env, &obj));
    NAPI_CALL(env, napi_set_named_property(env, obj, "runs", ra));
    NAPI_CALL(env, napi_set_named_property(env, obj, "records", wa));
    return obj;
}

// getDeltaLog(h, doc) -> Int32Array (only with deltaLogCapacity > 0; oracle layout)
napi_value GetDeltaLog(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    const uint32_t doc = (uint32_t)get_i32(env, argv[1]);
    uint32_t n = 0;
    int rc = mt_get_delta_log(hd->h, doc, nullptr, 0, &n);
    if (rc) return throw_rc(env, hd, rc, "mt_get_delta_log");   // incl. MT_E_OVERFLOW: fail loudly
    void *d;
    napi_value ab, arr;
    NAPI_CALL(env, napi_create_arraybuffer(env, (size_t)n * 4, &d, &ab));
    rc = mt_get_delta_log(hd->h, doc, (int32_t *)d, n, &n);
    if (rc) return throw_rc(env, hd, rc, "mt_get_delta_log");
    NAPI_CALL(env, napi_create_typedarray(env, napi_int32_array, n, ab, 0, &arr));
    return arr;
}

// deltaLogReset(h) -- empties every document's delta log (mt_delta_log_reset)
napi_value DeltaLogReset(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    const int rc = mt_delta_log_reset(hd->h);
    if (rc) return throw_rc(env, hd, rc, "mt_delta_log_reset");
    return nullptr;
}

// maintenanceCounts(h) -> Uint32Array [nDocs * 3]: SPLIT, APPEND, UNLINK per document
// (mergeTreeMaintenanceCallback events; only with deltaLogCapacity > 0)
napi_value MaintenanceCounts(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    const uint32_t n = 3u * mt_num_docs(hd->h);
    void *d;
    napi_value ab, arr;
    NAPI_CALL(env, napi_create_arraybuffer(env, (size_t)n * 4, &d, &ab));
    const int rc = mt_maintenance_counts(hd->h, (uint32_t *)d);
    if (rc) return throw_rc(env, hd, rc, "mt_maintenance_counts");
    NAPI_CALL(env, napi_create_typedarray(env, napi_uint32_array, n, ab, 0, &arr));
    return arr;
}

// checksums(h) -> ArrayBuffer of mt_checksum[nDocs] (32 B each)
napi_value Checksums(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    void *d;
    napi_value ab;
    NAPI_CALL(env, napi_create_arraybuffer(env, (size_t)mt_num_docs(hd->h) * sizeof(mt_checksum), &d, &ab));
    const int rc = mt_checksums(hd->h, (mt_checksum *)d);
    if (rc) return throw_rc(env, hd, rc, "mt_checksums");
    return ab;
}

napi_value LastKernelMs(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    napi_value r;
    NAPI_CALL(env, napi_create_double(env, mt_last_kernel_ms(hd->h), &r));
    return r;
}

napi_value NumDocs(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    return make_u32(env, mt_num_docs(hd->h));
}

// regeneratePending(h, doc) -> {recs: Int32Array (8 words per mt_regen_rec), text: Uint16Array,
// props: Uint32Array} or null when no segment group is pending  (mt_regenerate_pending)
napi_value RegeneratePending(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    Handle *hd = get_handle(env, argv[0]);
    if (!hd) return nullptr;
    uint32_t doc = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    const uint32_t cap = 1u << 16, tcap = 1u << 20, pcap = 1u << 20;   // a group holds <= one record per segment
    std::vector<mt_regen_rec> recs(cap);
    std::vector<uint16_t> text(tcap);
    std::vector<uint32_t> props(pcap);
    int32_t n = 0;
    if (mt_regenerate_pending(hd->h, doc, recs.data(), cap, &n, text.data(), tcap, props.data(), pcap) != 0) {
        napi_throw_error(env, nullptr, mt_last_error(hd->h));
        return nullptr;
    }
    napi_value out;
    if (n < 0) {
        NAPI_CALL(env, napi_get_null(env, &out));
        return out;
    }
    uint32_t tu = 0, pw = 0;
    for (int i = 0; i < n; i++) {
        if (recs[i].kind == MT_OP_INSERT && !(recs[i].flags & MT_F_MARKER)) tu = std::max(tu, recs[i].text_off + recs[i].text_len);
        if (recs[i].props_off != MT_NO_PROPS) pw = std::max(pw, recs[i].props_off + 1 + 2 * props[recs[i].props_off]);
    }
    NAPI_CALL(env, napi_create_object(env, &out));
    napi_value a;
    void *data = nullptr;
    napi_value ab;
    NAPI_CALL(env, napi_create_arraybuffer(env, (size_t)n * sizeof(mt_regen_rec), &data, &ab));
    if (n) memcpy(data, recs.data(), (size_t)n * sizeof(mt_regen_rec));
    NAPI_CALL(env, napi_create_typedarray(env, napi_int32_array, (size_t)n * 8, ab, 0, &a));
    NAPI_CALL(env, napi_set_named_property(env, out, "recs", a));
    NAPI_CALL(env, napi_create_arraybuffer(env, std::max<size_t>(tu, 1) * 2, &data, &ab));
    if (tu) memcpy(data, text.data(), (size_t)tu * 2);
    NAPI_CALL(env, napi_create_typedarray(env, napi_uint16_array, tu, ab, 0, &a));
    NAPI_CALL(env, napi_set_named_property(env, out, "text", a));
    NAPI_CALL(env, napi_create_arraybuffer(env, std::max<size_t>(pw, 1) * 4, &data, &ab));
    if (pw) memcpy(data, props.data(), (size_t)pw * 4);
    NAPI_CALL(env, napi_create_typedarray(env, napi_uint32_array, pw, ab, 0, &a));
    NAPI_CALL(env, napi_set_named_property(env, out, "props", a));
    return out;
}

// decodeSummaries(paths: string[], blobs: string[], docBlobOff: number[], threads) ->
// {docSegOff, nHeader, segs, text, props, minSeq, curSeq, catchup, keys, vals, clients}:
// SnapshotLoader's host half (include/mt_snapshot.h) over every document's blobs.  Property
// ids in props are the decoder's (keys[i] / JSON.parse(vals[i])); the facade maps them into
// its interner.  catchup[d] = index of the document's legacy catch-up blob or -1.
napi_value DecodeSummaries(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (!get_args(env, info, 4, argv)) return nullptr;
    uint32_t nb = 0, nd1 = 0;
    NAPI_CALL(env, napi_get_array_length(env, argv[0], &nb));
    NAPI_CALL(env, napi_get_array_length(env, argv[2], &nd1));
    if (nd1 == 0) {
        napi_throw_error(env, nullptr, "decodeSummaries: empty document offsets");
        return nullptr;
    }
    std::vector<std::string> paths(nb), blobs(nb);
    std::vector<const char *> pp(nb), jp(nb);
    std::vector<uint32_t> pl(nb);
    std::vector<uint64_t> jl(nb);
    auto str = [&](napi_value arr, uint32_t i, std::string &out) -> bool {
        napi_value v;
        size_t n = 0;
        if (napi_get_element(env, arr, i, &v) != napi_ok) return false;
        if (napi_get_value_string_utf8(env, v, nullptr, 0, &n) != napi_ok) return false;
        out.resize(n + 1);
        if (napi_get_value_string_utf8(env, v, &out[0], n + 1, &n) != napi_ok) return false;
        out.resize(n);
        return true;
    };
    for (uint32_t i = 0; i < nb; i++) {
        if (!str(argv[0], i, paths[i]) || !str(argv[1], i, blobs[i])) {
            napi_throw_type_error(env, nullptr, "decodeSummaries: paths and blobs must be strings");
            return nullptr;
        }
        pp[i] = paths[i].data();
        pl[i] = (uint32_t)paths[i].size();
        jp[i] = blobs[i].data();
        jl[i] = blobs[i].size();
    }
    std::vector<int64_t> off(nd1);
    for (uint32_t i = 0; i < nd1; i++) {
        napi_value v;
        double x = 0;
        NAPI_CALL(env, napi_get_element(env, argv[2], i, &v));
        NAPI_CALL(env, napi_get_value_double(env, v, &x));
        // integers in [0, blobs.length] only (a NaN or out-of-range double is UB to cast)
        if (!(x >= 0 && x <= (double)nb) || x != (double)(int64_t)x) {
            napi_throw_range_error(env, nullptr, "decodeSummaries: docBlobOff entries must be integers in [0, blobs.length]");
            return nullptr;
        }
        off[i] = (int64_t)x;
        if (i > 0 && off[i] < off[i - 1]) {
            napi_throw_range_error(env, nullptr, "decodeSummaries: docBlobOff must be non-decreasing");
            return nullptr;
        }
    }
    const uint32_t nd = nd1 - 1;
    if (off[0] != 0 || off[nd] != (int64_t)nb) {
        napi_throw_range_error(env, nullptr, "decodeSummaries: docBlobOff must run from 0 to blobs.length");
        return nullptr;
    }
    const int threads = get_i32(env, argv[3]);
    mt_snapdec *dec = mt_snapdec_create(0);
    if (mt_snapdec_decode(dec, nd, off.data(), pp.data(), pl.data(), jp.data(), jl.data(), threads) != 0) {
        napi_throw_error(env, nullptr, mt_snapdec_error(dec));
        mt_snapdec_destroy(dec);
        return nullptr;
    }
    uint64_t ns = 0, nt = 0, npr = 0;
    mt_snapdec_sizes(dec, &ns, &nt, &npr);
    napi_value out, a, ab;
    void *pd[9] = {};
    NAPI_CALL(env, napi_create_object(env, &out));
    struct Arr {
        const char *name;
        napi_typedarray_type t;
        size_t n, esz;
    } arrs[] = {{"docSegOff", napi_bigint64_array, nd + 1u, 8}, {"nHeader", napi_int32_array, nd, 4},
                {"segs", napi_uint8_array, ns * sizeof(mt_seg_rec), 1}, {"text", napi_uint16_array, nt, 2},
                {"props", napi_uint32_array, npr, 4},     {"minSeq", napi_int32_array, nd, 4},
                {"curSeq", napi_int32_array, nd, 4},      {"catchup", napi_bigint64_array, nd, 8}};
    for (int i = 0; i < 8; i++) {
        NAPI_CALL(env, napi_create_arraybuffer(env, std::max<size_t>(arrs[i].n * arrs[i].esz, 8), &pd[i], &ab));
        memset(pd[i], 0, std::max<size_t>(arrs[i].n * arrs[i].esz, 8));
        NAPI_CALL(env, napi_create_typedarray(env, arrs[i].t, arrs[i].n, ab, 0, &a));
        NAPI_CALL(env, napi_set_named_property(env, out, arrs[i].name, a));
    }
    mt_snapdec_fetch(dec, (int64_t *)pd[0], (int32_t *)pd[1], (mt_seg_rec *)pd[2], (uint16_t *)pd[3], (uint32_t *)pd[4],
                     (int32_t *)pd[5], (int32_t *)pd[6], (int64_t *)pd[7]);
    auto strings = [&](const char *name, uint32_t n, int64_t (*get)(const mt_snapdec *, uint32_t, char *, uint64_t)) -> bool {
        napi_value arr, v;
        if (napi_create_array_with_length(env, n, &arr) != napi_ok) return false;
        std::string buf;
        for (uint32_t i = 0; i < n; i++) {
            const int64_t len = get(dec, i, nullptr, 0);
            buf.resize((size_t)std::max<int64_t>(len, 0));
            get(dec, i, &buf[0], buf.size());
            if (napi_create_string_utf8(env, buf.data(), buf.size(), &v) != napi_ok) return false;
            if (napi_set_element(env, arr, i, v) != napi_ok) return false;
        }
        return napi_set_named_property(env, out, name, arr) == napi_ok;
    };
    const bool ok = strings("keys", mt_snapdec_num_keys(dec), mt_snapdec_key) &&
                    strings("vals", mt_snapdec_num_values(dec), mt_snapdec_value) &&
                    strings("clients", nd, mt_snapdec_doc_clients);
    mt_snapdec_destroy(dec);
    if (!ok) {
        napi_throw_error(env, nullptr, "decodeSummaries: N-API string conversion failed");
        return nullptr;
    }
    return out;
}

napi_value Init(napi_env env, napi_value exports) {
    struct {
        const char *name;
        napi_callback fn;
    } fns[] = {{"create", Create},         {"destroy", Destroy},           {"loadInitialText", LoadInitialText},
                 {"startCollaboration", StartCollaboration},
               {"applyOps", ApplyOps},     {"loadSnapshots", LoadSnapshots},     {"status", Status},             {"getLength", GetLength},
               {"getText", GetText},       {"getPropRuns", GetPropRuns},   {"getDeltaLog", GetDeltaLog},
               {"deltaLogReset", DeltaLogReset},
               {"maintenanceCounts", MaintenanceCounts},
               {"checksums", Checksums},   {"lastKernelMs", LastKernelMs}, {"numDocs", NumDocs},
               {"regeneratePending", RegeneratePending}, {"decodeSummaries", DecodeSummaries},
               {"applyOpsAsync", ApplyOpsAsync},         {"getContainingSegment", GetContainingSegment},
               {"getSegmentByUid", GetSegmentByUid},     {"getViewLengths", GetViewLengths},
               {"extractSnapshots", ExtractSnapshots}};
    for (auto &f : fns) {
        napi_value v;
        NAPI_CALL(env, napi_create_function(env, f.name, NAPI_AUTO_LENGTH, f.fn, nullptr, &v));
        NAPI_CALL(env, napi_set_named_property(env, exports, f.name, v));
    }
    return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
