/*
 * mt_replay.h -- C-ABI drop-in boundary of the MI355X merge-tree replay backend.
 *
 * The reference has no FFI: its boundary is the TypeScript class `Client`
 * (packages/dds/merge-tree/src/client.ts:43), constructed once per SharedString by
 * SharedSegmentSequence (packages/dds/sequence/src/sequence.ts:131-134) and fed one
 * sequenced message at a time through Client.applyMsg (client.ts:797-819).  This library
 * replaces N such observer Clients with one handle that owns N documents resident in HBM
 * and applies whole batches of sequenced messages per document in HIP kernels.  The
 * binding a maintainer adds on the reference side is the N-API addon in
 * fluidframework_amd/js/ (INTEGRATION.md shows it); ctypes (Python) binds the same symbols.
 *
 * Conventions: every function returns 0 on success or a negative MT_E_* code; the text of
 * the last error is available from mt_last_error().  Per-document failures (the
 * reference's throws / asserts, enum mt_doc_status in mt_types.h) do not fail the call:
 * the document is marked and skipped by later batches, other documents continue.
 * A handle is single-writer; calls are synchronous unless named *_async.
 */
#ifndef MT_REPLAY_H
#define MT_REPLAY_H
#include <stddef.h>
#include <stdint.h>

#include "mt_types.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MT_E_INVALID (-1)    /* bad argument */
#define MT_E_HIP (-2)        /* HIP runtime error */
#define MT_E_NOMEM (-3)      /* device allocation failed */
#define MT_E_NODEVICE (-4)   /* no HIP device visible: the product has no CPU fallback */
#define MT_E_OVERFLOW (-5)   /* a document's delta log overflowed (mt_get_delta_log) */
#define MT_E_STALE_VIEW (-6) /* reserved (round 4 refused remote views below a client's latest refSeq;
                                 they are answered since round 5) */

typedef struct mt_handle mt_handle;
typedef struct mt_batch mt_batch;

/* Per-document capacities (0 = default).  By default (page_capacity 0) a handle has the
   paged layout and no capacity is a limit: the paged ones (page / unsettled / page heap), the
   text / property arenas, the uid map and the overflow overlap arena are starting points that
   the growth step raises per document (mt_last_grown), as the reference's documents grow
   without bound (MT/mergeTree.ts:2577-2585, MT/textSegment.ts:74-85).  page_capacity < 0
   opts into a flat-only handle, whose capacities are hard (MT_DOC_CAPACITY beyond them) --
   except on a live_client handle, where the live growth step (run by mt_sync) doubles the
   flat capacities a document would outgrow (segments, blocks, heap, text, property records,
   live_group_capacity) for the whole handle before that message. */
typedef struct mt_options {
    int32_t device;          /* HIP device ordinal (one process per GPU) */
    int32_t seg_capacity;    /* leaf segments per document in the flat tiers (default 2048;
                                512 on a paged handle, where it only receives what the LDS
                                tier hands to the paged layout) */
    int32_t block_capacity;  /* blocks per tree level per document  (default seg/2) */
    int32_t heap_capacity;   /* zamboni LRU heap entries            (default 2*seg) */
    int32_t text_capacity;   /* UTF-16 units per document text arena half (default 32768) */
    int32_t props_capacity;  /* property-set records per document   (default seg) */
    int32_t delta_log_capacity; /* int32 words of per-document delta log; 0 = hash only */
    int32_t lds_seg_capacity;   /* segments a document may hold while staged in LDS
                                   (default 192; -1 = always replay from HBM).  A document
                                   that outgrows it is replayed from HBM transparently.
                                   Live handles: staged only for a value > 0 (default: HBM). */
    int32_t page_capacity;      /* paged layout for documents that outgrow the LDS tier:
                                   pages (level-1 B-tree nodes, <= 64 segments each) per
                                   document to start with (default 64; the growth step raises
                                   it); < 0 = a flat-only handle (such documents replay from
                                   the flat HBM tier, O(segments) per op, within its hard
                                   capacities).  Live handles are flat-only. */
    int32_t page_heap_capacity; /* zamboni heap entries of a paged document (default 1024;
                                   256 with the default page_capacity) */
    int32_t unsettled_capacity; /* segments of a paged document inserted or removed above
                                   minSeq (default 256) */
    int32_t uid_capacity;       /* entries of a paged document's segment-id -> page map
                                   (default 65536; 8192 with the default page_capacity): ids
                                   are renumbered when they run out, and the growth step
                                   raises it when live segments fill it.  (The renumbering
                                   borrows the idle half of the text arena as 2 x pages int32
                                   scratch: a text_capacity below twice the page count is
                                   raised by the growth step first, cause 4.) */
    /* Tight paged tier (0 = off): LDS capacities below the three above.  Documents are
       replayed at these first (a smaller LDS footprint: more documents per CU); one that
       does not fit, or whose next message could outgrow them, continues -- from that
       message -- in a second launch at the full capacities. */
    int32_t lds_page_capacity;
    int32_t lds_unsettled_capacity;
    int32_t lds_page_heap_capacity;
    /* 1: the tight tier keeps removedClientOverlap masks of short ids 1..32 only (4 bytes
       per LDS segment instead of 8); a document one of whose clients above 32 removes an
       already-removed segment continues in the full tier.  For documents with few writers. */
    int32_t lds_narrow_overlap;
    /* Delta log layout (with delta_log_capacity > 0): 0 = the callback records of
       mt_get_delta_log; 1 = rich: every logged segment also carries its state at the event
       (text or marker refType, property set), and mergeTreeMaintenanceCallback events
       (SPLIT / APPEND / UNLINK, MT/mergeTree.ts:1343-1373, 2264-2269) are records too --
       what the Node facade turns into callback objects.  Removed segments keep their text
       until they are unlinked. */
    int32_t delta_log_mode;
    /* 1: live-client handle -- every document backs a participant Client whose short id 0 is
       the local client (startOrUpdateCollaboration's own id, MT/client.ts:1053-1064):
       records flagged MT_F_LOCAL are its own unsequenced ops, MT_F_ACK records the sequenced
       echoes of them (ackPendingSegment), and mt_regenerate_pending rebuilds the oldest
       pending op after a reconnect.  Live handles replay from HBM, or staged in LDS while
       they fit lds_seg_capacity > 0 (no paged tier); a segment can be in 16 pending segment
       groups at once (MT_DOC_CAPACITY beyond). */
    int32_t live_client;
    /* live handles: segment groups (unacked ops, one per regenerated segment after a
       reconnect) a document may have outstanding (default 1024, at most 65535) */
    int32_t live_group_capacity;
    /* paged documents, when the batch's documents are not a whole number of resident rounds
       (n = R x resident + r, 0 < r): replay them in `paged_slices` slices of their ops,
       each launch leaving out a different window of r documents, so that every launch is R
       full rounds and the r left-over documents' work is spread over all of them instead of
       running as a last, nearly empty round (0 = off).  Results are identical. */
    int32_t paged_slices;
    /* 1 (with delta_log_mode 1): keep every segment's ordinal (MergeBlock.setOrdinal /
       nodeUpdateOrdinals, MT/mergeTree.ts:347-372, 2553-2575) -- the strings
       SortedSegmentSet and SequenceDeltaEvent order and dedup ranges by (Q8).  Each rich log
       entry then also carries the segment's id, its position as Client.getPosition reads it
       inside the callback, and its ordinal; mt_get_segment_info reads the current ones.  Every
       tier keeps them, the paged layout included; the replay fast path and the synthetic
       generator keep none. */
    int32_t segment_ordinals;
    /* u16 units of a paged document's overflow overlap arena: the removedClientOverlap lists of
       segments whose overlapping removers outnumber the 63 mask slots (default 8192; the
       growth step doubles it for a document that fills half of it) */
    int32_t overlap_arena_capacity;
} mt_options;

/* Synthetic op-stream generator parameters (DESIGN.md "Synthetic op streams"); the
   probabilities are thresholds floor(p * 2^32) compared against a u32 draw. */
typedef struct mt_gen_cfg {
    uint32_t seed;
    int32_t ops, writers, lag, seed_len, text_max, n_keys, n_values, max_keys_per_op;
    int32_t _pad;
    uint64_t p_insert, p_insert_remove, p_newline, p_len_continue, p_insert_props, p_null;
} mt_gen_cfg;

/* Creates n_docs observer replicas (`new Client(...)` + startOrUpdateCollaboration,
   client.ts:75-84, 1053-1073) on opt->device. */
mt_handle *mt_create(uint32_t n_docs, const mt_options *opt);
void mt_destroy(mt_handle *h);
const char *mt_last_error(const mt_handle *h);
uint32_t mt_num_docs(const mt_handle *h);

/* Initial document contents, inserted before collaboration starts (seq 0, client
   LocalClientId -- Client.insertSegmentLocal client.ts:202-215).  seed_off[n_docs+1]
   indexes seed_text (UTF-16).  Resets every document. */
int mt_load_initial_text(mt_handle *h, const int64_t *seed_off, const uint16_t *seed_text);
/* Re-initialises every document from the contents last given to mt_load_initial_text
   (kept in HBM); asynchronous on the handle's stream. */
int mt_reset(mt_handle *h);
/* Client.startOrUpdateCollaboration(longClientId, minSeq, currentSeq) -> MergeTree.
   startCollaboration (client.ts:1053-1073, mergeTree.ts:1287-1294): sets every listed
   document's collab window (minSeq, currentSeq) before its first message; the zamboni heap
   starts empty.  min_seq[d] < 0 leaves document d as it is; otherwise 0 <= min_seq[d] <=
   cur_seq[d] (MT_E_INVALID).  Host arrays [n_docs]; mt_reset / mt_load_initial_text
   return documents to (0, 0). */
int mt_start_collaboration(mt_handle *h, const int32_t *min_seq, const int32_t *cur_seq);

/* Client.applyMsg for every message of a batch (client.ts:797-819).  Records are grouped
   per document in sequence order: doc_op_off[n_docs+1] indexes ops.  Host buffers; the
   call uploads, applies and synchronises. */
int mt_apply_ops(mt_handle *h, const int64_t *doc_op_off, const mt_op_rec *ops, uint64_t n_ops,
                 const uint16_t *text, uint64_t text_len, const uint32_t *props,
                 uint64_t props_len);

/* Cold catch-up (config C5): replaces every document's state with a decoded SnapshotV1
   summary -- Client.load -> SnapshotLoader.initialize (packages/dds/merge-tree/src/
   snapshotLoader.ts:36-228): loadHeader = reloadFromSegments (mergeTree.ts:1229-1284) +
   startOrUpdateCollaboration(min_seq, cur_seq) (client.ts:1053-1073), then loadBody's
   appends (snapshotLoader.ts:195-227).  Document d's records are
   segs[doc_seg_off[d] .. doc_seg_off[d+1]), the first n_header[d] from the header chunk;
   payload / props index the text (UTF-16) and props arenas.  A document whose load fails
   like the reference's ("MergeTree insert failed") gets that status.  Catch-up
   and tail messages then go through mt_apply_ops as usual.  On a handle with a paged
   layout (page_capacity > 0) a header larger than seg_capacity is staged and built
   straight into pages (its text / property records still need text_capacity /
   props_capacity); otherwise it fails with MT_DOC_CAPACITY.  Synchronous. */
int mt_load_snapshots(mt_handle *h, const int64_t *doc_seg_off, const int32_t *n_header, const mt_seg_rec *segs,
                      uint64_t n_segs, const uint16_t *text, uint64_t text_len, const uint32_t *props,
                      uint64_t props_len, const int32_t *min_seq, const int32_t *cur_seq);
/* The same in two steps: a device-resident set of decoded summaries (uploaded once), then
   loads enqueued on the handle's stream (mt_sync waits). */
typedef struct mt_snapshots mt_snapshots;
mt_snapshots *mt_snapshots_upload(mt_handle *h, const int64_t *doc_seg_off, const int32_t *n_header,
                                  const mt_seg_rec *segs, uint64_t n_segs, const uint16_t *text, uint64_t text_len,
                                  const uint32_t *props, uint64_t props_len, const int32_t *min_seq,
                                  const int32_t *cur_seq);
/* ... for documents [doc_lo, doc_lo + n_docs) of the handle only (summary d -> document
   doc_lo + d; the arrays are sized n_docs): a cold catch-up that decodes and loads the
   handle's documents in slices, each slice's load overlapping the host decode of the next
   (fluidframework_amd.MergeTreeBatch.catch_up).  mt_snapshots_load_async leaves the other
   documents untouched. */
mt_snapshots *mt_snapshots_upload_range(mt_handle *h, uint32_t doc_lo, uint32_t n_docs, const int64_t *doc_seg_off,
                                        const int32_t *n_header, const mt_seg_rec *segs, uint64_t n_segs,
                                        const uint16_t *text, uint64_t text_len, const uint32_t *props,
                                        uint64_t props_len, const int32_t *min_seq, const int32_t *cur_seq);
int mt_snapshots_load_async(mt_handle *h, const mt_snapshots *s);
void mt_snapshots_free(mt_snapshots *s);
/* Device time of the most recent snapshot load's kernels (k_load_header and, for documents
   that load straight into pages, the conversion; HIP events on the handle's stream; waits
   for them).  0 before any load. */
float mt_last_load_ms(mt_handle *h);

/* Summary emission: SnapshotV1.extractSync (snapshotV1.ts:156-252) of every document's
   current state as mt_seg_rec records in summary order (runs below minSeq coalesced, merge
   info above it; flags MT_SEG_*), text and props arenas as for mt_load_snapshots (client
   ids are the documents' short ids).  Two calls: with recs == NULL, io[3*n_docs] receives
   per document {records, text units, props words}; then, io unchanged, the arrays sized by
   their sums are filled (documents back to back).  min_seq/cur_seq (nullable) receive the
   collaboration window -- the header metadata. */
int mt_extract_snapshots(mt_handle *h, int64_t *io, mt_seg_rec *recs, uint16_t *text, uint32_t *props,
                         int32_t *min_seq, int32_t *cur_seq);

/* Device-resident batches (bench / pipelined path). */
mt_batch *mt_batch_upload(mt_handle *h, const int64_t *doc_op_off, const mt_op_rec *ops,
                          uint64_t n_ops, const uint16_t *text, uint64_t text_len,
                          const uint32_t *props, uint64_t props_len);
int mt_batch_apply_async(mt_handle *h, const mt_batch *b);   /* enqueue on the handle's stream */
uint64_t mt_batch_num_ops(const mt_batch *b);
void mt_batch_free(mt_batch *b);
/* Page-locked host memory (hipHostMalloc) for the arenas a host encoder writes and
   mt_batch_upload copies from: the copy is then a DMA, with no host-side staging copy on the
   cores the encoder runs on.  NULL on failure; mt_host_free(NULL) is a no-op. */
void *mt_host_alloc(uint64_t bytes);
void mt_host_free(void *p);
int mt_sync(mt_handle *h);
/* Device time of the most recent replay kernel (HIP events on the handle's stream). */
float mt_last_kernel_ms(const mt_handle *h);
/* Recreates the handle's stream (after a sync) at a scheduling priority: > 0 the device's
   highest, < 0 its lowest, 0 the default.  For handles that share one GPU (bench_skew.py's size
   classes): the high-priority stream's waiting workgroups dispatch first as CUs free up. */
int mt_set_stream_priority(mt_handle *h, int priority);
/* Documents of the most recent batch that outgrew the LDS tier and were replayed from HBM:
   out[8] = {total, spilled before a message, segments, blocks, heap, text, property
   records, at load} (the causes count LDS capacities hit inside a message). */
int mt_last_hbm_docs(mt_handle *h, uint32_t *out);
/* High-water marks of the paged documents of the most recent batch (or generation):
   out[5] = {pages, unsettled-table entries, zamboni heap entries, segments, documents handed
   from the tight to the full-capacity paged tier}; sizing aid for the paged capacities. */
int mt_last_paged_peaks(mt_handle *h, uint32_t *out);

/* Growth step of the most recent batch (mt_sync runs it; see mt_options: the paged
   capacities are where documents start, not a limit): out[6] = {documents handed to it,
   rounds, documents now in the big region, its page / unsettled-table / heap capacities
   (0 if none)}.  A document whose next message could outgrow the last paged tier moves, with
   its state, into a region with those capacities doubled (up to the 160 KiB of LDS one paged
   launch may stage) and continues there; only beyond that does it fail with
   MT_DOC_CAPACITY.  A batch applied with mt_batch_apply_async must stay allocated until
   mt_sync (mt_batch_free of a pending batch finishes the step first). */
int mt_last_grown(mt_handle *h, uint32_t *out);

/* Generates ops_per_doc synthetic messages per document on the device, applying them as
   it goes (the generator reads each writer's view length from the live replica), and
   returns them as a device-resident batch.  Documents end in the generated final state;
   call mt_load_initial_text again to replay the batch from scratch. */
mt_batch *mt_generate(mt_handle *h, const mt_gen_cfg *cfg, uint32_t doc_index_base,
                      int32_t *view_len_trace /* nullable host [n_docs*ops*4] diagnostic:
                                                 per op {view length, n_seg, refSeq,
                                                 client} */);
/* mt_generate with a length per document: ops_per_doc[n_docs] messages (nullable: cfg->ops
   each), and global document indices doc_ids[n_docs] (nullable: doc_index_base + d).
   Document d's stream is the first ops_per_doc[d] messages of the stream mt_generate draws
   for its global index (the draws do not depend on the length), so skewed batches (bench
   c3skew) reuse the oracle's generator for parity. */
mt_batch *mt_generate_docs(mt_handle *h, const mt_gen_cfg *cfg, uint32_t doc_index_base,
                           const int32_t *ops_per_doc, const int32_t *doc_ids, int32_t *view_len_trace);
/* Initial seed texts as the generator draws them (seed_off[n_docs+1], seed_text); _docs:
   for the global indices doc_ids[n_docs] (nullable: doc_index_base + d). */
int mt_generated_seeds_docs(mt_handle *h, const mt_gen_cfg *cfg, uint32_t doc_index_base, const int32_t *doc_ids,
                            int64_t *seed_off, uint16_t *seed_text);
int mt_generated_seeds(mt_handle *h, const mt_gen_cfg *cfg, uint32_t doc_index_base,
                       int64_t *seed_off, uint16_t *seed_text);
/* Copies a batch back to the host (arrays sized by mt_batch_sizes). */
int mt_batch_sizes(const mt_batch *b, uint64_t *n_ops, uint64_t *text_len, uint64_t *props_len);
int mt_batch_download(const mt_batch *b, int64_t *doc_op_off, mt_op_rec *ops, uint16_t *text,
                      uint32_t *props);

/* ---- read-out (MergeTree.length client.ts:1051; getText textSegment.ts:154-172;
        getPropertiesAtPosition client.ts:1011-1025) ---- */
int mt_get_status(mt_handle *h, int32_t *out_status);                 /* [n_docs] */
int mt_get_length(mt_handle *h, uint32_t doc, uint32_t *out);
int mt_get_text(mt_handle *h, uint32_t doc, uint16_t *out, uint32_t cap, uint32_t *out_len);
/* Observer-visible property runs: rows of (start, length, props_record_index) plus the
   records [count, (key, value)*].  Returns counts through the out pointers. */
int mt_get_prop_runs(mt_handle *h, uint32_t doc, uint32_t *runs, uint32_t cap_runs,
                     uint32_t *n_runs, uint32_t *records, uint32_t cap_words,
                     uint32_t *n_words);
/* Diagnostic: segment rows of 8 int32 (len, seq, client, rseq, rclient, n_overlap,
   marker refType or -1, has_props) in document order, and the leaf-block partition. */
int mt_get_segments(mt_handle *h, uint32_t doc, int32_t *rows, uint32_t cap_rows,
                    uint32_t *n_rows, int32_t *leaves, uint32_t cap_leaves, uint32_t *n_leaves);
/* Diagnostic: a paged document's overflow overlap arena (MT_OVF_BIT sets) as
   {capacity in u16 units, fill of the current half, current half, largest set made,
   units the live sets take (the sets segment rows name, each counted once), units of every
   set made, the most units the half in use ever held}; zeros for a document without one.  Compaction keeps the fill bounded by the live
   sets, not by every set ever made (MT/mergeTree.ts:1322-1398 drops a list with its segment). */
int mt_get_overlap_arena(mt_handle *h, uint32_t doc, int32_t *out /* [7] */);
/* Every segment's property set in document order, from one copy of the document: per segment
   [n, (key, value) x n] (n = -1: properties undefined); *n_words = the words written or, with
   out = NULL / a short buffer, needed.  (mt_get_segment_props one segment at a time copies the
   document each call.) */
int mt_get_all_segment_props(mt_handle *h, uint32_t doc, int32_t *out, uint64_t cap_words, uint64_t *n_words);
int mt_get_segment_props(mt_handle *h, uint32_t doc, uint32_t seg_index, uint32_t *pairs,
                         uint32_t cap_pairs, int32_t *n_pairs);
/* ---- segment read-outs of the Client / MergeTree surface SharedSegmentSequence calls
        (SEQ/sequence.ts:240, 251; MT/mergeTree.ts:1610-1667; MT/client.ts getPosition /
        getContainingSegment).  A view is (ref_seq, client): client is a short client id as
        the encoder numbered it, 0 = this replica (its view is the observer view whatever the
        ref_seq, MT/mergeTree.ts:1692-1698).  A remote view takes any ref_seq of the collab
        window [minSeq, currentSeq] (MT_E_INVALID outside it).  Interior nodes answer a remote
        view from their partial lengths (nodeLength / blockLength, MT/partialLengths.ts:455-486),
        leaves by visibility: every segment adds its length when the view holds its insert and
        subtracts it when the view holds its removal, so in a view below the client's latest
        refSeq a node can count a segment the client removed but had not seen inserted as
        negative, as the reference does (pinned on every view of tests/golden/ref_readouts*). ---- */
typedef struct mt_seg_info {
    int32_t row;             /* index in document order (-1: no such segment) */
    uint32_t uid;            /* segment id: stable for the segment's life (a split's left half
                                keeps it, the right half gets a new one) */
    int32_t position;        /* getPosition in the queried view: lengths of the segments before it */
    int32_t offset;          /* mt_get_containing_segment: pos - position; else 0 */
    int32_t length;          /* cachedLength */
    int32_t seq, client;     /* -1 = UnassignedSequenceNumber (live handles) */
    int32_t removed_seq;     /* MT_RSEQ_NONE when not removed */
    int32_t removed_client;
    int32_t marker_ref_type; /* -1: a TextSegment */
    int32_t text_len;        /* UTF-16 units of its text written to the caller's buffer */
    int32_t ordinal_len;     /* -1: no ordinals on this handle (mt_options.segment_ordinals) */
    uint16_t ordinal[16];    /* MergeNode.ordinal's characters (MT/mergeTree.ts:347-372) */
} mt_seg_info;
/* MergeTree.getContainingSegment(pos, refSeq, clientId) (MT/mergeTree.ts:1656-1667):
   searchBlock's descent (:1830-1862) -- at every level the first child whose length in the
   view (partial lengths for interior nodes) exceeds pos; row -1 when it finds no segment
   (past the end, or, in a view below the client's latest refSeq, a block whose leaves do not
   hold the position: the reference does not backtrack). */
int mt_get_containing_segment(mt_handle *h, uint32_t doc, int32_t pos, int32_t ref_seq, int32_t client,
                              mt_seg_info *out, uint16_t *text, uint32_t text_cap);
/* MergeTree.getPosition(segment, refSeq, clientId) (MT/mergeTree.ts:1619-1636) of the segment
   with id uid (from a delta-log entry or an earlier read-out); row -1 once it left the tree
   (unlinked, or appended to its neighbour: the reference's getPosition of such a segment
   walks no parent and returns 0). */
int mt_get_segment_by_uid(mt_handle *h, uint32_t doc, uint32_t uid, int32_t ref_seq, int32_t client,
                          mt_seg_info *out, uint16_t *text, uint32_t text_cap);
/* MergeTree.getLength(refSeq, clientId) (MT/mergeTree.ts:1610-1612) for n (doc, ref_seq,
   client) queries: the root's partial length in each view. */
int mt_get_view_lengths(mt_handle *h, uint32_t n, const uint32_t *docs, const int32_t *ref_seq,
                        const int32_t *client, int32_t *out);
/* Debug: raw segment records (8 u32 per segment: segA then segB) and the 32-word header. */
int mt_debug_raw(mt_handle *h, uint32_t doc, uint32_t *rows, uint32_t cap_rows, uint32_t *n_rows,
                 int32_t *hdr_words);
/* Debug: section timers of a build with -DMT_PROF (MT_E_INVALID otherwise). */
int mt_debug_prof(mt_handle *h, uint64_t *out /* [128] */, int reset);
/* Debug (flat documents): the zamboni heap in array order ({maxSeq, leaf index of its segment
   or -1} pairs) and every leaf block's needsScour flag (-1 undefined, 0, 1). */
int mt_debug_heap(mt_handle *h, uint32_t doc, int32_t *heap, uint32_t cap, uint32_t *n_heap, int32_t *flags,
                  uint32_t cap_flags, uint32_t *n_flags);
/* Delta log (only with delta_log_capacity > 0), oracle layout: one record per
   mergeTreeDeltaCallback (MT/mergeTreeDeltaCallback.ts:33-41; call sites MT/mergeTree.ts:
   2014-2021, 2625-2632, 2738-2745) = [seq, kind, n, (position, cachedLength
   [, npd, (key, old value) x npd]) x n].  Records are whole: when a record does not fit
   the remaining capacity it is dropped, the document's log stops and this call returns
   MT_E_OVERFLOW (after filling out / n with the records that were kept). */
int mt_get_delta_log(mt_handle *h, uint32_t doc, int32_t *out, uint32_t cap, uint32_t *n);
/* Empties every document's delta log and clears its overflow flag (asynchronous, on the
   handle's stream): a reader that has consumed the records calls it before the next batch. */
int mt_delta_log_reset(mt_handle *h);

/* mergeTreeMaintenanceCallback events per document since its creation (only with
   delta_log_capacity > 0, MT_E_INVALID otherwise): out[3*doc + {0,1,2}] = SPLIT
   (splitLeafSegment, MT/mergeTree.ts:2260-2272), APPEND and UNLINK (scourNode,
   MT/mergeTree.ts:1322-1398).  (The events themselves, with the segments' state, are
   records of the rich delta log, delta_log_mode 1.) */
int mt_maintenance_counts(mt_handle *h, uint32_t *out);

/* Per-document checksums (mt_types.h), to host memory or straight into device memory
   on the handle's device (e.g. a torch tensor's data_ptr() before an RCCL all-gather). */
int mt_checksums(mt_handle *h, mt_checksum *out);

/* Live-client handles: regeneratePendingOp for the oldest pending segment group of one
   document (MT/client.ts:709-766 resetPendingDeltaToOps + findReconnectionPostition
   :675-707).  The group is dequeued; every member segment, in document order, yields one op
   at its position relative to the group's localSeq and joins a new group with the same
   localSeq at the tail of the queue (a remove whose segment a remote remove has replaced
   yields none).  Insert ops carry the segment's text (out_text) and property set (out_props:
   [n, (key, value) x n] or MT_NO_PROPS when it has none); annotate ops carry positions only
   (their props / combiningOp are the pending op's own).  *n_out = -1: no pending group.
   Output buffers too small for the group: MT_E_OVERFLOW with *n_out = -2 and the document
   unchanged (mt_last_error names the sizes needed); retry with larger buffers. */
typedef struct mt_regen_rec {
    int32_t kind;        /* MT_OP_INSERT / MT_OP_REMOVE / MT_OP_ANNOTATE */
    int32_t pos1, pos2;  /* remove / annotate: [pos1, pos2); insert: pos1 */
    int32_t local_seq;   /* the group's localSeq */
    uint32_t text_off;   /* insert: offset of the text in out_text (marker: refType) */
    uint32_t text_len;   /* insert: UTF-16 units (marker: 1) */
    uint32_t props_off;  /* insert: offset of the property set in out_props, or MT_NO_PROPS */
    uint32_t flags;      /* MT_F_MARKER */
} mt_regen_rec;
int mt_regenerate_pending(mt_handle *h, uint32_t doc, mt_regen_rec *out, uint32_t cap, int32_t *n_out,
                          uint16_t *out_text, uint32_t text_cap, uint32_t *out_props, uint32_t props_cap);
/* Live-client handles: {collabWindow.localSeq, pending segment groups} of every document
   ([n_docs][2]). */
int mt_pending_counts(mt_handle *h, int32_t *out);
int mt_checksums_device(mt_handle *h, void *device_out);

#ifdef __cplusplus
}
#endif
#endif
