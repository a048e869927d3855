/*
 * TEST INFRASTRUCTURE ONLY -- CPU restatement ("oracle") of the reference merge-tree's
 * observer replay path.  Used by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the checker; never linked into the product.
 */
#ifndef MT_ORACLE_H
#define MT_ORACLE_H
#include <stdint.h>
#include "../include/mt_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_doc orc_doc;

/* Synthetic op-stream generator parameters (DESIGN.md "Synthetic op streams"). */
/* probabilities are thresholds floor(p * 2^32) compared against a u32 draw */
typedef struct orc_gen_cfg {
    uint32_t seed;
    int32_t ops, writers, lag, seed_len, text_max, n_keys, n_values, max_keys_per_op;
    int32_t _pad;
    uint64_t p_insert, p_insert_remove, p_newline, p_len_continue, p_insert_props, p_null;
} orc_gen_cfg;

orc_doc *orc_new(const uint16_t *seed_text, int32_t seed_len);
void orc_free(orc_doc *d);
/* Load a decoded SnapshotV1 summary (header records first, then body records). */
orc_doc *orc_load(const mt_seg_rec *recs, int32_t n_header, int32_t n_total, const uint16_t *text_arena,
                  const uint32_t *props_arena, int32_t min_seq, int32_t cur_seq);
/* Apply one record; returns mt_doc_status.  Once a doc has failed it stays failed. */
int32_t orc_apply(orc_doc *d, const mt_op_rec *op, const uint16_t *text_arena,
                  const uint32_t *props_arena);
int32_t orc_status(const orc_doc *d);
/* live participant: out[0] = collabWindow.localSeq, out[1] = pending segment groups */
void orc_pending_counts(const orc_doc *d, int32_t *out);
/* one regenerated op; the layout of mt_regen_rec (include/mt_replay.h) */
typedef struct orc_regen_rec {
    int32_t kind, pos1, pos2, local_seq;
    uint32_t text_off, text_len, props_off, flags;
} orc_regen_rec;
/* regeneratePendingOp of the oldest pending group (one non-GROUP op of kind `kind`); records; returns their count, -1: no pending group, -2: a
   buffer too small, -3: an internal inconsistency */
int32_t orc_regenerate(orc_doc *d, int32_t kind, orc_regen_rec *out, int32_t cap, uint16_t *text,
                       int32_t text_cap, uint32_t *props, int32_t props_cap);
int32_t orc_view_length(orc_doc *d, int32_t ref_seq, int32_t client);
/* MergeTree.getContainingSegment / getPosition in a remote view (partial lengths at interior
   nodes): out = {segment index (-1: undefined), offset, position in the view, observer position} */
void orc_containing(orc_doc *d, int32_t pos, int32_t ref_seq, int32_t client, int32_t *out);
int32_t orc_position(orc_doc *d, int32_t seg_index, int32_t ref_seq, int32_t client);
int32_t orc_length(orc_doc *d);
int32_t orc_text(orc_doc *d, uint16_t *out, int32_t cap);
/* segment rows of 8 int32: len, seq, client, rseq(INT32_MIN=none), rclient, n_overlap,
   marker(-1 none else refType), props_handle_present */
int32_t orc_segments(orc_doc *d, int32_t *out, int32_t cap_rows);
int32_t orc_leaves(orc_doc *d, int32_t *out, int32_t cap);
/* props of live segment i (in walk order, including removed): returns count or -1 if the
   segment has no property object; writes (key, value) pairs */
int32_t orc_segment_props(orc_doc *d, int32_t seg_index, uint32_t *out, int32_t cap_pairs);
void orc_checksum(orc_doc *d, mt_checksum *out);
/* mergeTreeMaintenanceCallback event counts since creation: [SPLIT, APPEND, UNLINK]
   (MT/mergeTree.ts:2264-2269, :1368-1373, :1343-1348) */
void orc_maintenance(orc_doc *d, uint32_t *out);
/* removedClientOverlap lists of the segments in the tree (MT/mergeTree.ts:2577-2585), counted
   as [n, ids...] (n + 1 u16 units each, the device's overflow-set form): {now, maximum after
   any message so far} -- the bound the device's overflow arena is tested against */
void orc_overlap_units(const orc_doc *d, int64_t *out);
uint64_t orc_text_hash(const uint16_t *t, int32_t n);
/* delta log: flattened records  [seq, kind, nsegs, (pos, len, ndeltas, (key, oldval)*)*]* */
int32_t orc_deltas(orc_doc *d, int32_t *out, int32_t cap);
void orc_set_record_deltas(orc_doc *d, int32_t on);

/* Generate one document's op stream with the oracle as the view-length source.
   Returns number of records, or -1 on capacity/failed doc. */
int32_t orc_generate(const orc_gen_cfg *cfg, int32_t doc, mt_op_rec *ops, int32_t ops_cap,
                     uint16_t *text, int32_t text_cap, int32_t *text_used,
                     uint32_t *props, int32_t props_cap, int32_t *props_used,
                     uint16_t *seed_out, int32_t *seed_len_out, orc_doc **keep);

void orc_set_gen_trace(int32_t *trace);   /* per-op writer view lengths (diagnostic) */

/* Replay a CSR batch of documents on `threads` host threads; fills checksum/status. */
int32_t orc_replay_batch(int32_t n_docs, const int64_t *doc_op_off, const mt_op_rec *ops,
                         const uint16_t *text_arena, const uint32_t *props_arena,
                         const int64_t *seed_off, const uint16_t *seed_arena,
                         mt_checksum *out_sum, int32_t *out_status, int32_t threads);

/* Config C5 on `threads` host threads: load each document's summary, replay its ops. */
int32_t orc_load_replay_batch(int32_t n_docs, const int64_t *seg_off, const int32_t *n_header,
                              const mt_seg_rec *segs, const uint16_t *seg_text, const uint32_t *seg_props,
                              const int32_t *min_seq, const int32_t *cur_seq, const int64_t *doc_op_off,
                              const mt_op_rec *ops, const uint16_t *text_arena, const uint32_t *props_arena,
                              mt_checksum *out_sum, int32_t *out_status, int32_t threads);

#ifdef __cplusplus
}
#endif
#endif
