/*
 * mt_snapshot.h -- native host decoder of SnapshotV1 summaries (config C5's host half).
 *
 * SnapshotLoader.initialize / loadHeader / loadBody / specToSegment (MT/snapshotLoader.ts:
 * 36-228), SnapshotV1.processChunk (MT/snapshotV1.ts:266-277) and toLatestVersion /
 * buildHeaderMetadataForLegecyChunk (MT/snapshotChunks.ts:136-188) over the summaries' blob
 * texts (JSON), straight into the mt_seg_rec records + text / props arenas that
 * mt_load_snapshots / mt_snapshots_upload (include/mt_replay.h) take.  Blobs are parsed on
 * `threads` host threads; records are built in document order so that property keys and
 * values are interned in the same first-seen order as fluidframework_amd.wire.Interner.
 * Host-only (libmtsnapdec.so, built with g++); the GPU path is unchanged.
 */
#ifndef MT_SNAPSHOT_H
#define MT_SNAPSHOT_H
#include <stdint.h>

#include "mt_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mt_snapdec mt_snapdec;

/* synthetic: keys "k<n>" -> n and integer values -> themselves (wire.Interner(synthetic=True));
   otherwise keys and values are interned (values by canonical JSON, sorted object keys). */
mt_snapdec *mt_snapdec_create(int synthetic);
void mt_snapdec_destroy(mt_snapdec *s);
const char *mt_snapdec_error(const mt_snapdec *s);

/* Decodes n_docs summaries.  Document d owns blobs [blob_off[d], blob_off[d + 1]); blob b is
   its path (paths[b], path_len[b] bytes) and its contents (json[b], json_len[b] bytes of
   UTF-8 JSON text).  Returns 0, or -1 with the first failing document's message in
   mt_snapdec_error (the reference throws there).  The result replaces the previous one. */
int mt_snapdec_decode(mt_snapdec *s, uint32_t n_docs, const int64_t *blob_off, const char *const *paths,
                      const uint32_t *path_len, const char *const *json, const uint64_t *json_len, int threads);

/* sizes of the last result: segment records, text units, props words */
int mt_snapdec_sizes(const mt_snapdec *s, uint64_t *n_segs, uint64_t *text_len, uint64_t *props_len);

/* the last result: doc_seg_off[n_docs + 1], n_header[n_docs], segs[n_segs], text, props,
   min_seq[n_docs], cur_seq[n_docs] (the mt_load_snapshots arguments), and per document the
   index of its legacy catch-up blob (-1: none; the caller parses those messages).  The
   documents are copied into the caller's arrays in parallel, on the decode's threads; any
   pointer may be null (that output is skipped). */
int mt_snapdec_fetch(const mt_snapdec *s, int64_t *doc_seg_off, int32_t *n_header, mt_seg_rec *segs, uint16_t *text,
                     uint32_t *props, int32_t *min_seq, int32_t *cur_seq, int64_t *catchup_blob);

/* interned names (non-synthetic): key / value id i as UTF-8 (values: canonical JSON); the
   length is returned, the text copied when out is non-null (cap bytes) */
int64_t mt_snapdec_key(const mt_snapdec *s, uint32_t i, char *out, uint64_t cap);
int64_t mt_snapdec_value(const mt_snapdec *s, uint32_t i, char *out, uint64_t cap);
uint32_t mt_snapdec_num_keys(const mt_snapdec *s);
/* document d's writers as a JSON array of long client ids, short id 1..n in order
   (specToSegment's getOrAddShortClientId first-seen order; the catch-up ops continue it) */
int64_t mt_snapdec_doc_clients(const mt_snapdec *s, uint32_t d, char *out, uint64_t cap);
/* every document's array, in order, each followed by '\n' (one call for a whole batch) */
int64_t mt_snapdec_all_clients(const mt_snapdec *s, char *out, uint64_t cap);
uint32_t mt_snapdec_num_values(const mt_snapdec *s);

/* Sequenced messages -> op records: the host encode in front of mt_batch_upload, native.
   Document d's messages are one JSON array of ISequencedDocumentMessage objects
   (PD/protocol.ts:132-172; clientId, sequenceNumber, referenceSequenceNumber,
   minimumSequenceNumber, type, contents = an IMergeTree op, MT/ops.ts:63-110) in json[d]
   (json_len[d] bytes).  Records as fluidframework_amd/wire.py Batch.add_doc makes them (the
   encoder the JS facade mirrors, js/encode.js): one mt_op_rec per op (GROUP members with
   MT_F_GROUP_MORE, an empty GROUP or a non-"op" message a MT_OP_NOOP record), short client
   ids first-seen per document from 1, property keys / values interned on this decoder in
   first-seen document order (mt_snapdec_key / mt_snapdec_value, shared with summary
   decoding).  A non-rewrite combining op fails the decode (its transform table needs every
   value its keys have held: wire.Batch builds it), as do malformed messages; the error names
   the first failing document.  `threads` workers take documents dynamically. */
int mt_opdec_decode(mt_snapdec *s, uint32_t n_docs, const char *const *json, const uint64_t *json_len, int threads);
int mt_opdec_sizes(const mt_snapdec *s, uint64_t *n_ops, uint64_t *text_len, uint64_t *props_len);
/* doc_op_off[n_docs + 1], ops[n_ops], text[text_len], props[props_len] (each nullable) */
int mt_opdec_fetch(const mt_snapdec *s, int64_t *doc_op_off, mt_op_rec *ops, uint16_t *text, uint32_t *props);
/* document d's long client ids in short-id order (id 1 first) as a JSON array; null for a
   message without a clientId */
int64_t mt_opdec_doc_clients(const mt_snapdec *s, uint32_t d, char *out, uint64_t cap);

#ifdef __cplusplus
}
#endif
#endif
