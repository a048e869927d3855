/*
 * mt_types.h -- binary wire format shared by the C-ABI boundary (include/mt_replay.h),
 * the HIP kernels and the CPU oracle.
 *
 * One sequenced merge-tree message (ISequencedDocumentMessage carrying an
 * IMergeTreeInsert/Remove/Annotate op; PD/protocol.ts:132-172, MT/ops.ts:63-110) is encoded
 * as one 32-byte mt_op_rec.  A GROUP op (MT/ops.ts:104-107) becomes one record per member
 * with MT_F_GROUP_MORE set on all but the last (members share seq/refSeq/client and the
 * seq/msn update happens once, after the last member: MT/client.ts:768-819).  A non-"op"
 * message only advances seq/msn (MT/client.ts:805,818) and is encoded as MT_OP_NOOP.
 *
 * Text payloads are UTF-16 code units (JS string semantics, MT/textSegment.ts:45,105) in a
 * separate arena.  Property sets are interned to 32-bit key/value ids by the host; values
 * carry MT_VAL_FALSY_BIT when the JS value is falsy (needed by the `rewrite` rule
 * `!newProps[key]`, MT/segmentPropertiesManager.ts:72).
 */
#ifndef MT_TYPES_H
#define MT_TYPES_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum mt_op_kind {
    MT_OP_INSERT = 0,     /* MergeTreeDeltaType.INSERT   MT/ops.ts:30 */
    MT_OP_REMOVE = 1,     /* MergeTreeDeltaType.REMOVE   MT/ops.ts:31 */
    MT_OP_ANNOTATE = 2,   /* MergeTreeDeltaType.ANNOTATE MT/ops.ts:32 */
    MT_OP_NOOP = 3,       /* non-"op" message: seq/msn update only */
    MT_OP_LOAD_REMOVED = 4, /* internal (summary load): removal info of the segment the
                              preceding MT_F_LOAD insert appended */
    MT_OP_LOAD_ALIASED = 5 /* internal (summary load): loadBody re-inserts segments that are
                              already in the tree (MT_DOC_ALIASED) */
};

enum mt_op_flags {
    MT_F_GROUP_MORE = 1,  /* another member of the same GROUP message follows */
    MT_F_MARKER = 2,      /* insert of a Marker (length 1); payload = refType */
    MT_F_LOAD = 4,        /* internal (summary load): a body segment appended by
                             SnapshotLoader.loadBody (MT/snapshotLoader.ts:195-227) --
                             insertSegments with opArgs undefined: no delta callback, no
                             seq/msn update */
    MT_F_LOCAL = 8,       /* live handles: the local client's own unsequenced op
                             (insertSegmentLocal / removeRangeLocal / annotateRangeLocal,
                             MT/client.ts:164-211): applied at refSeq = currentSeq with
                             UnassignedSequenceNumber; seq / ref_seq / min_seq are ignored */
    MT_F_ACK = 16         /* live handles: the sequenced echo of one of the local client's
                             ops (applyMsg with msg.clientId == longClientId ->
                             ackPendingSegment, MT/client.ts:589-626, 810-812); kind = the
                             member op's type, positions ignored */
};

#define MT_NO_PROPS 0xFFFFFFFFu      /* props field: no property set */
#define MT_VAL_NULL 0xFFFFFFFFu      /* value id of JSON null (delete) */
#define MT_VAL_UNDEF 0xFFFFFFFEu     /* value id of JS undefined (a key set to undefined) */
#define MT_VAL_FALSY_BIT 0x80000000u /* value id flag: JS value is falsy */
#define MT_VAL_NOMATCH_BIT 0x40000000u /* value id flag: matchProperties never finds it equal
                                          (NaN, undefined, objects holding them) */
#define MT_COMBINE_NONE 0u
#define MT_COMBINE_REWRITE 1u        /* ICombiningOp { name: "rewrite" } */
#define MT_COMBINE_OTHER 2u          /* a combining op whose result is not modelled (the
                                        reference throws or mutates a shared value) */
#define MT_COMBINE_TABLE 3u          /* any other combining op: the record
                                        carries combine(op, old, undefined, seq) for every
                                        value -- [n, new value of an absent key,
                                        (old, new) x n] after the (key, value) pairs */

typedef struct mt_op_rec {
    int32_t seq;        /* sequenceNumber */
    int32_t ref_seq;    /* referenceSequenceNumber */
    int32_t min_seq;    /* minimumSequenceNumber */
    int32_t pos1;       /* op.pos1 */
    int32_t pos2;       /* remove/annotate: op.pos2; insert: payload length (UTF-16 units) */
    uint32_t payload;   /* insert: offset into the text arena (UTF-16 units);
                           marker insert: refType */
    uint32_t props;     /* offset (u32 words) of a props-op record in the props arena, or
                           MT_NO_PROPS.  record = [count | combine<<16, (key, value) x count
                           (, transform table: MT_COMBINE_TABLE)] */
    uint16_t client;    /* short client id of the writer (first-seen order, observer = 0) */
    uint8_t kind;       /* enum mt_op_kind */
    uint8_t flags;      /* enum mt_op_flags */
} mt_op_rec;

/* One segment of a decoded SnapshotV1 summary (SnapshotLoader.specToSegment,
   MT/snapshotLoader.ts:86-118): header segments first, then body segments, per document.
   A spec without merge info has seq 0 (UniversalSequenceNumber) and client -2
   (NonCollabClient). */
typedef struct mt_seg_rec {
    int32_t len;            /* UTF-16 units (Marker: 1) */
    int32_t seq;            /* spec.seq, default 0 */
    int32_t removed_seq;    /* spec.removedSeq, INT32_MIN when undefined */
    uint32_t payload;       /* text arena offset (UTF-16 units); Marker: refType */
    uint32_t props;         /* props record [count, (key, value) x count] or MT_NO_PROPS */
    int16_t client;         /* short id of spec.client, or -2 */
    int16_t removed_client; /* short id of spec.removedClient (when removed_seq is set) */
    uint8_t flags;          /* MT_F_MARKER | MT_SEG_MERGE_INFO | MT_SEG_HAS_SEQ */
    uint8_t pad[7];
} mt_seg_rec;
/* mt_seg_rec.flags written by mt_extract_snapshots (SnapshotV1.extractSync): the spec carries
   merge info {json, seq?, client?, removedSeq?, removedClient?} (MT/snapshotChunks.ts:61-67);
   HAS_SEQ: seq/client present (inserted above minSeq) */
#define MT_SEG_MERGE_INFO 0x10
#define MT_SEG_HAS_SEQ 0x20

/* Per-document verification checksum: all-gathered across ranks. */
typedef struct mt_checksum {
    uint32_t length;     /* observer length, MergeTree.length MT/mergeTree.ts:1617 */
    uint32_t n_segments; /* live leaf segments (diagnostic, tree-shape dependent) */
    uint64_t text_hash;  /* chunked FNV-1a 64 of the getText() string (MT/textSegment.ts:154) */
    uint64_t props_hash; /* FNV-1a 64 over the observer-visible property runs */
    uint64_t delta_hash; /* FNV-1a 64 over every mergeTreeDeltaCallback record */
    /* exact definitions: DESIGN.md "Checksums"; restated in oracle/mt_oracle.c */
} mt_checksum;

/* Per-document status codes (mt_doc_status). */
enum mt_doc_status {
    MT_DOC_OK = 0,
    MT_DOC_INSERT_FAILED = 1,   /* "MergeTree insert failed" MT/mergeTree.ts:2243-2249 */
    MT_DOC_SEQ_ORDER = 2,       /* assert currentSeq < seq     MT/client.ts:462-463 (completeAndLogOp) */
    MT_DOC_MINSEQ_ORDER = 3,    /* assert minSeq <= msn        MT/client.ts:464-465 (completeAndLogOp) */
    MT_DOC_CAPACITY = 4,        /* a per-document capacity was exceeded */
    MT_DOC_UNSUPPORTED = 5,     /* a combining op whose result the engine does not model */
    MT_DOC_INTERNAL = 6,        /* engine invariant violated (bug) */
    MT_DOC_SEQ_BACKWARDS = 7,   /* assert currentSeq <= seq    MT/client.ts:824 (updateSeqNumbers) */
    MT_DOC_MSN_ABOVE_SEQ = 8,   /* assert min <= seq           MT/client.ts:826 (updateSeqNumbers) */
    MT_DOC_MSN_BACKWARDS = 9,   /* assert minSeq <= msn        MT/mergeTree.ts:1755 (setMinSeq) */
    /* Summary load: SnapshotLoader.loadBody never empties its batch of plain segments
       (MT/snapshotLoader.ts:207-227), so a flush after the first one appends segments that
       are already in the tree -- one ISegment object at two places.  The reference carries
       on with that tree (its later setOrdinal asserts, MT/mergeTree.ts:366-368, come from
       it); the engine stops the document at the re-insertion. */
    MT_DOC_ALIASED = 10
};

#ifdef __cplusplus
}
#endif
#endif
