/*
 * psx.h — C ABI of the MI355X row-update apply path (Bosen / petuum_ps server apply).
 *
 * This is the drop-in boundary for ONE hot path of the reference: the server-side
 * apply of serialized worker increments (ClientSendOpLogMsg payloads) into dense and
 * sparse parameter-table rows, plus serve-back of row bytes.  Every entry point is a
 * plain C function over plain pointers and sizes; no torch or HIP C++ types appear in
 * the signatures (a `void*` HIP stream handle is the only device-runtime object).
 *
 * Reference seams each entry point replaces (paths relative to the reference repo):
 *   psx_ctx_create          Server::Init                 src/petuum_ps/server/server.cpp:18-31
 *   psx_register_sender     bg_version_map_[bg] = -1     src/petuum_ps/server/server.cpp:21-24
 *   psx_table_create        Server::CreateTable /        src/petuum_ps/server/server.cpp:33-44
 *                           ServerTable::ServerTable     src/petuum_ps/server/server_table.cpp:19-93
 *   psx_apply_stream        Server::ApplyOpLogUpdateVersion
 *                                                        src/petuum_ps/server/server.hpp:46-48,
 *                                                        src/petuum_ps/server/server.cpp:120-179
 *   psx_apply_streams_device  the same, for K device-resident messages applied in order
 *   psx_apply_indexed       the same with producer record offsets: replaces
 *                           SerializedOpLogReader::Next's size chain
 *                                                        src/petuum_ps/server/serialized_oplog_reader.hpp:57-84
 *   psx_apply_indexed_rows  the same with producer record-row lists: dense records placed
 *                           without reading their row ids from the stream (checked in the apply)
 *   psx_ctx_set_pipeline    (new) overlap a call's index stage with the previous call's apply
 *   psx_table_load_rows     AbstractRow::ResetRowData    src/petuum_ps_common/storage/numeric_store_row.hpp:142-145
 *   psx_table_read_rows     VectorStore::CopyToMem       src/petuum_ps_common/storage/vector_store.hpp:115-118
 *   psx_serialize_rows      ServerRow::Serialize         src/petuum_ps/server/server_row.hpp:65-71
 *   psx_serialize_dirty     Server::CreateSendServerPushRowMsgs  src/petuum_ps/server/server.cpp:189-309
 *   psx_row_flags           ServerRow::IsDirty / FindRow src/petuum_ps/server/server_row.hpp:90-96,
 *                                                        src/petuum_ps/server/server_table.cpp:136-141
 *   psx_pack_stream(_indexed) CreateOpLogMsgs + OpLogSerializer + RowOpLogSerializer (client pack)
 *                                                        src/petuum_ps/thread/abstract_bg_worker.cpp:590-649,
 *                                                        src/petuum_ps/client/oplog_serializer.hpp:12-37,
 *                                                        src/petuum_ps/thread/row_oplog_serializer.hpp:139-166,
 *                                                        src/petuum_ps_common/oplog/dense_row_oplog.hpp:112-136
 *   psx_row_importance      ServerRow::get_importance    src/petuum_ps/server/server_row.hpp:120-130
 *   psx_row_versions        VersionServerRow::get_version src/petuum_ps/server/version_server_row.hpp:66
 *   psx_table_set_adarevision  AdaRevisionServerTableLogic::Init (server_table_logic = AdaRevision)
 *                                                        src/petuum_ps/server/adarevision_server_table_logic.cpp:19-36,
 *                                                        src/petuum_ps/server/server_table.cpp:83-93
 *   psx_row_sent            Server::RowSent -> ServerRowSent  src/petuum_ps/server/server.cpp:436-441,
 *                                                        src/petuum_ps/server/server_thread.cpp:221
 *   psx_adarevision_state   AdaRevisionRow               src/petuum_ps/server/adarevision_server_table_logic.hpp:11-22
 *   psx_serialize_partial   Server::CreateSendServerPushRowMsgsPartial
 *                                                        src/petuum_ps/server/server.cpp:311-420,
 *                           ServerTable::GetPartialTableToSendRegular / AppendRowsToBuffsPartial
 *                                                        src/petuum_ps/server/server_table.cpp:301-346,381-420
 *   psx_encode/decode_oplog_header  ClientSendOpLogMsg  src/petuum_ps/thread/ps_msgs.hpp:1003-1055,
 *                                                        src/petuum_ps_common/thread/msg_base.hpp:81-188
 *   psx_encode/decode_push_header   ServerPushRowMsg    src/petuum_ps/thread/ps_msgs.hpp:1057-1103
 *   psx_handle_oplog_msg    ServerThread::HandleOpLogMsg (apply + ClockUntil)
 *                                                        src/petuum_ps/server/server_thread.cpp:224-266
 *   psx_ctx_set_compat      SerializedOpLogReader's int32 offset_
 *                                                        src/petuum_ps/server/serialized_oplog_reader.hpp:137
 *   psx_clock_until         Server::ClockUntil -> VectorClock::TickUntil
 *                                                        src/petuum_ps/server/server.cpp:62-79,
 *                                                        src/petuum_ps_common/util/vector_clock.cpp:28-79
 *   psx_min_clock           Server::GetMinClock          src/petuum_ps/server/server.cpp:181-184
 *   psx_row_subscribe       Server::FindCreateRow + SSPPushServerThread::RowSubscribe
 *                                                        src/petuum_ps/server/server.cpp:46-60,
 *                                                        src/petuum_ps/server/ssp_push_server_thread.cpp:51-54,
 *                                                        src/petuum_ps/server/callback_subs.hpp:21-28
 *   psx_apply_push_body     SSPPushBgWorker::ApplyServerPushedRow -> SerializedRowReader -> ResetRowData
 *                                                        src/petuum_ps/thread/ssp_push_bg_worker.cpp:70-122,
 *                                                        src/petuum_ps/client/serialized_row_reader.hpp:30-100,
 *                                                        src/petuum_ps_common/storage/numeric_store_row.hpp:142-145
 *   psx_serialize_push      Server::CreateSendServerPushRowMsgs with subscriptions (one body per client)
 *                                                        src/petuum_ps/server/server.cpp:189-309,
 *                                                        src/petuum_ps/server/server_table.cpp:197-261,
 *                                                        src/petuum_ps/server/callback_subs.hpp:39-59
 *
 * Error behaviour: the reference aborts via glog CHECK on a version gap
 * (server.cpp:124-126) or an unknown table id (serialized_oplog_reader.hpp:112-120).
 * Here every call returns a psx_status instead; a failed call applies nothing: every
 * check of an apply call (framing, tables, row range, columns, the sorted/map capacity
 * dry run, AdaRevision snapshots, duplicate rows) runs on the device before any table is
 * touched.  The one stated exception is a producer record-row list that disagrees with
 * its stream (psx_apply_indexed_rows): that is found inside the apply, so only the rows
 * concerned are left unchanged.  Errors discovered by device kernels are reported by the next psx_sync() —
 * or by the next call that reads or serves rows, which first settles the calls in
 * flight (so it sees every accepted message, as the reference server thread does).
 * Versions of a rejected call: a call the device rejects gives each of its senders'
 * versions back when the error is settled, unless a later call from that sender was
 * accepted in between (then the version stays consumed, as an empty message would consume
 * it); the error text names each rejected (bg_id, version) and which of the two happened.
 * So a sender that settles before its next message (PSX_SEAM_SYNC, or psx_sync) can send
 * the corrected message again with the same version.
 *
 * Threading: one host thread per context (one context = one server shard = one
 * reference ServerThread, server_thread.hpp:90).  Buffers are borrowed for the call
 * (host buffers) or until the next psx_sync() (device buffers).
 */
#ifndef PSX_H_
#define PSX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSX_ABI_VERSION 9

/* Maximum number of messages fused into one psx_apply_streams_device call. */
#define PSX_MAX_FUSED_STREAMS 16
/* Maximum number of tables per context. */
#define PSX_MAX_TABLES 64
/* Clients of the per-client push: PETUUM_MAX_NUM_CLIENTS as the reference builds it
 * (defns.mk: -DPETUUM_MAX_NUM_CLIENTS=64; CallBackSubs' bitset, callback_subs.hpp:96). */
#define PSX_MAX_CLIENTS 64

typedef enum psx_status {
  PSX_OK = 0,
  PSX_ERR_INVALID_ARG = 1,    /* null pointer, bad config, misaligned device stream */
  PSX_ERR_VERSION = 2,        /* CHECK_EQ(bg_version+1, version) server.cpp:124 */
  PSX_ERR_UNKNOWN_TABLE = 3,  /* CHECK(table_iter != end) serialized_oplog_reader.hpp:112 */
  PSX_ERR_MALFORMED = 4,      /* stream shorter than its headers say, negative counts */
  PSX_ERR_ROW_RANGE = 5,      /* row id not owned by this shard's row range */
  PSX_ERR_CAPACITY = 6,       /* a sorted/map row would exceed max_entries, a column >= row_capacity
                                 of a dense row, or no AdaRevision snapshot slot; nothing applied
                                 or sent */
  PSX_ERR_DEVICE = 7,         /* HIP runtime error */
  PSX_ERR_OOM = 8,            /* device allocation failed */
  PSX_ERR_BUFFER_TOO_SMALL = 9,
  PSX_ERR_UNSUPPORTED = 10,   /* e.g. the same table twice inside one message */
  PSX_ERR_SENDER = 11,        /* bg id never registered (Server::Init bg_ids) */
  PSX_ERR_NO_DEVICE = 12,     /* no HIP device visible */
  PSX_ERR_STATE = 13          /* server-logic state missing: an AdaRevision record names a
                                 (row, version) with no accum_gradients_ snapshot (CHECK,
                                 adarevision_server_table_logic.cpp:114-116); nothing applied */
} psx_status;

/* Row storage kinds (TableInfo.row_type -> registered AbstractRow). */
typedef enum psx_row_kind {
  PSX_ROW_DENSE = 0,      /* DenseRow<V>          = NumericStoreRow<VectorStore,V>   dense_row.hpp:9-41 */
  PSX_ROW_SORTED_MAP = 1, /* SortedVectorMapRow<V>= NumericStoreRow<SortedVectorMapStore,V> */
  PSX_ROW_MAP = 2         /* SparseRow<V>         = NumericStoreRow<MapStore,V>      sparse_row.hpp */
} psx_row_kind;

typedef enum psx_dtype {
  PSX_F32 = 0,
  PSX_F64 = 1,
  PSX_I32 = 2,
  PSX_I64 = 3
} psx_dtype;

/* Mirrors the fields of TableInfo (configs.hpp:170-210) the apply path reads, plus
 * the shard geometry that replaces ServerTable's boost::unordered_map<row_id,row>:
 * row r is owned iff (r - row_offset) % row_stride == 0 and its slot
 * (r - row_offset) / row_stride < max_rows.  row_stride = 1 gives a row-range shard;
 * row_stride = num_comm_channels * num_clients reproduces the reference's modulo
 * placement (context.hpp:291-304). */
typedef struct psx_table_config {
  int32_t table_id;
  int32_t row_kind;                 /* psx_row_kind */
  int32_t dtype;                    /* psx_dtype */
  int32_t oplog_dense_serialized;   /* TableInfo.oplog_dense_serialized */
  int64_t row_capacity;             /* TableInfo.row_capacity (dense width) */
  int64_t dense_row_oplog_capacity; /* TableInfo.dense_row_oplog_capacity (dense record width) */
  int64_t row_offset;
  int64_t row_stride;
  int64_t max_rows;
  int64_t max_entries;              /* sorted/map rows: device slots per row */
  /* ABI 2: */
  int32_t accum_importance;         /* 1: rows accumulate importance on apply, as ServerTable
                                       selects under SSPAggr + RelativeMagnitude/FIFO_N_ReMag
                                       (server_table.cpp:26-47; NSSumImpCalc,
                                       ns_sum_imp_calc.hpp:57-98) */
  int32_t version_maintain;         /* ABI 3 (was reserved0): TableInfo.version_maintain (configs.hpp:207).
                                       Dense records carry VersionDenseRowOpLog's trailer
                                       {uint64 version; bool end_of_version} (version_dense_row_oplog.hpp:161-180,
                                       parsed and not otherwise used without a server logic); rows are
                                       VersionServerRow: version_ = 1 at creation, +1 per applied record,
                                       appended to every serialized row (version_server_row.hpp:11-71).
                                       Dense rows with dense-serialized kDenseRowOpLog records only. */
  int64_t server_push_row_upper_bound; /* TableInfo.server_push_row_upper_bound (configs.hpp:181):
                                       rows per table per partial push; 0 -> 100 (table_gflags.cpp:21) */
  /* ABI 3: */
  int32_t row_oplog_type;           /* TableInfo.row_oplog_type (configs.hpp:35-40): 0 kDenseRowOpLog;
                                       3 kDenseRowOpLogFloat16 = dense records uint16[cap] binary16,
                                       decompressed to f32 before the add (dense_row_oplog_float16.hpp:144-157;
                                       f32 tables only).  1/2 select sparse row oplogs, which change nothing on
                                       the server for sparse-serialized tables (abstract_row_oplog.hpp:64-78). */
  /* ABI 8 (was reserved1): */
  int32_t row_bytes_f16;            /* 1: DenseRowFloat16<float> rows (dense_row_float16.hpp:13; the row type
                                       apps/matrixfact's matrixfact_split16 registers, :47,560): stored and
                                       updated in f32, serialized (row reads, pushes) as binary16 uint16[cap]
                                       through Float16Compressor::compress (vector_store_float16.hpp:91-99;
                                       the third-party header is unpinned: parity unpinned).  Dense f32 rows
                                       only.  A client context caching such rows takes pushed bodies through
                                       psx_apply_push_body only when row_capacity is even (4-byte records). */
} psx_table_config;

/* One device-resident ClientSendOpLogMsg payload (ps_msgs.hpp:1003-1055 after its
 * 41-byte header): `data` points at the serialized stream, 4-byte aligned. */
typedef struct psx_stream {
  const void *data;
  size_t size;        /* get_avai_size() */
  int32_t bg_id;      /* sender bg thread id */
  uint32_t version;   /* ClientSendOpLogMsg::get_version() */
} psx_stream;

typedef struct psx_ctx psx_ctx;

/* ---- lifecycle ---------------------------------------------------------- */
int32_t psx_abi_version(void);
/* Visible HIP devices (hipGetDeviceCount); PSX_ERR_NO_DEVICE with *n = 0 when none. */
psx_status psx_device_count(int32_t *n);
psx_status psx_ctx_create(int32_t device, int32_t server_id, psx_ctx **out);
psx_status psx_ctx_destroy(psx_ctx *ctx);
/* Use an external hipStream_t (e.g. the caller's compute stream); NULL restores the
 * context's own stream. */
psx_status psx_ctx_set_stream(psx_ctx *ctx, void *hip_stream);
void *psx_ctx_get_stream(psx_ctx *ctx);
psx_status psx_register_sender(psx_ctx *ctx, int32_t bg_id);
/* Version last applied for a sender (-1 before its first message). */
psx_status psx_sender_version(psx_ctx *ctx, int32_t bg_id, int64_t *version);

/* ---- tables -------------------------------------------------------------- */
psx_status psx_table_create(psx_ctx *ctx, const psx_table_config *cfg);
/* Overwrite num_rows dense rows starting at row id first_row (row ids step by
 * row_stride) with src (num_rows * row_capacity values); marks the rows present.
 * src_on_device != 0 means src is device memory. */
psx_status psx_table_load_rows(psx_ctx *ctx, int32_t table_id, int64_t first_row,
                               int64_t num_rows, const void *src, int32_t src_on_device);
/* Copy num_rows dense rows (same addressing) into dst; absent rows read as zero. */
psx_status psx_table_read_rows(psx_ctx *ctx, int32_t table_id, int64_t first_row,
                               int64_t num_rows, void *dst, int32_t dst_on_device);
/* Per-row flags for num_rows rows: bit0 = row exists (created on first touch,
 * server.cpp:163-166), bit1 = dirty since last psx_clear_dirty. */
psx_status psx_row_flags(psx_ctx *ctx, int32_t table_id, int64_t first_row,
                         int64_t num_rows, uint8_t *dst);
psx_status psx_clear_dirty(psx_ctx *ctx, int32_t table_id);
/* Accumulated importance of num_rows rows (same addressing as psx_row_flags): the
 * f64 sum, since the row was last sent, of each applied record's NSSumImpCalc value —
 * dense record: sum_i |u_i / v_i| (|u_i| where v_i == 0), v_i the value before the add;
 * sparse record: sum_i |u_i|.  Zero for tables without accum_importance and for rows
 * never applied (the reference leaves importance_ uninitialized, server_row.hpp:16-19). */
psx_status psx_row_importance(psx_ctx *ctx, int32_t table_id, int64_t first_row,
                              int64_t num_rows, double *dst);

/* VersionServerRow::get_version (version_server_row.hpp:66) of num_rows rows (same
 * addressing as psx_row_flags): 1 + records applied since creation for version tables;
 * 0 for rows that do not exist and for tables without version_maintain
 * (abstract_server_row.hpp:71). */
psx_status psx_row_versions(psx_ctx *ctx, int32_t table_id, int64_t first_row,
                            int64_t num_rows, uint64_t *dst);

/* ---- apply (the hot path) -------------------------------------------------- */
/* Server::ApplyOpLogUpdateVersion (server.cpp:120-179): host bytes, borrowed only for the
 * call (serialized_oplog_reader.hpp:22: the reader does not take ownership; the server
 * thread frees the message after the call, server_thread.cpp:457-458).
 * Default (PSX_SEAM_ASYNC): the bytes are copied into one of two HBM staging slots on the
 * context's copy stream and the call returns as soon as the copy has read them (page-locked
 * caller memory copies at the PCIe DMA rate); the apply is enqueued behind the copy, so
 * message k's apply runs beside message k+1's copy.  Version and sender errors return at
 * once; what only the device sees (framing, unknown tables, row range, capacity) fails the
 * call with nothing applied and is reported by the next call that settles (psx_sync, a
 * push, a row read), as for psx_apply_streams_device.  PSX_SEAM_SYNC (psx_ctx_set_seam):
 * every call also settles before it returns, so its own device errors come back from it. */
psx_status psx_apply_stream(psx_ctx *ctx, const void *oplog, size_t oplog_size,
                            int32_t bg_id, uint32_t version);
#define PSX_SEAM_ASYNC 0
#define PSX_SEAM_SYNC 1
psx_status psx_ctx_set_seam(psx_ctx *ctx, int32_t mode);
/* n device-resident messages, applied as if by n ApplyOpLogUpdateVersion calls in
 * array order (per-row update order preserved => bit-exact float sums).  Asynchronous
 * on the context stream; device buffers must stay valid until psx_sync(). */
psx_status psx_apply_streams_device(psx_ctx *ctx, const psx_stream *streams, int32_t n);
/* psx_apply_streams_device with producer-supplied record indexes (SURVEY §8(b)
 * psx_apply_indexed): record_offsets[i] (device, 8-byte aligned; NULL = none) holds, for
 * every record of message i, all tables in stream order, the byte offset of its row id —
 * exactly psx_pack_stream's record_offsets.  Sparse tables then skip the sequential
 * record walk (SerializedOpLogReader::Next's size chain, serialized_oplog_reader.hpp:
 * 57-84): the offsets are copied and the chain checked in parallel; a sparse table's
 * entries that do not describe its records are PSX_ERR_MALFORMED at psx_sync, nothing
 * applied.  Dense tables' entries are counted but not read (fixed stride). */
psx_status psx_apply_indexed(psx_ctx *ctx, const psx_stream *streams, const uint64_t *const *record_offsets,
                             int32_t n);
/* psx_apply_indexed plus producer record-row lists: record_rows[i] (device, 4-byte aligned;
 * NULL = none) holds, for every record of message i, all tables in stream order, the row
 * id the producer packed into it — psx_pack_stream_indexed's record_rows, i.e. the pack
 * tables' row_ids in record order.  record_offsets may be NULL (no sparse index).  Dense
 * tables on the fast path then place records from the lists instead of reading every
 * record's row id from the stream (a 4-byte read that costs one 128-byte DRAM line per
 * record), and the apply kernel checks each record's row id against its slot as it loads
 * the record (same cache line as the payload).  Contract difference, stated: a list that
 * disagrees with its stream is found during the apply, so the call is PSX_ERR_MALFORMED
 * at psx_sync with the rows whose records disagree left unchanged (not created, not
 * dirtied) and every other row of the call applied.  A list entry naming a row twice or
 * outside the shard leaves its message's claim count short, which is caught before any
 * apply: the call is replayed from the stream on the ordered path, exactly as for a
 * duplicate row (exact result; the stream's own row ids decide).  A stream row id that
 * differs from its list entry — outside the shard or not — is a disagreement like any
 * other.  Tables whose apply kernel does not check rows (importance, AdaRevision,
 * partial-coverage and >= 4 GiB calls) ignore the lists. */
psx_status psx_apply_indexed_rows(psx_ctx *ctx, const psx_stream *streams, const uint64_t *const *record_offsets,
                                  const int32_t *const *record_rows, int32_t n);
/* Wait for all queued work and report any device-detected error. */
psx_status psx_sync(psx_ctx *ctx);

/* ---- serve-back -------------------------------------------------------------- */
/* Serialize rows exactly as ServerRow::Serialize (dense: V[capacity]; sorted map:
 * Entry{int32,V}[n] in store order; map: {int32,V}[n]; version tables append
 * uint64 version, VersionServerRow::Serialize) framed as RecordBuff records
 * {int32 row_id; size_t size; bytes} (record_buff.hpp:41-53).  Absent rows are
 * skipped.  *used receives the bytes written. */
psx_status psx_serialize_rows(psx_ctx *ctx, int32_t table_id, const int32_t *row_ids,
                              int32_t n, void *out, size_t cap, size_t *used);

/* Server push body for every dirty row of every table (Server::CreateSendServerPushRowMsgs,
 * server.cpp:189-309): per table (creation order) int32 table_id, the dirty rows as
 * RecordBuff records in ascending row id, then int32 -1 between tables / -2 at the end
 * (context.hpp:123-129).  clear_dirty resets the rows' dirty bit and importance (server_table.cpp:234-235).
 * On PSX_ERR_BUFFER_TOO_SMALL *used holds the bytes needed and nothing is cleared.
 * out_on_device != 0: out is a 4-byte-aligned device buffer. */
psx_status psx_serialize_dirty(psx_ctx *ctx, void *out, size_t cap, size_t *used,
                               int32_t out_on_device, int32_t clear_dirty);

/* Partial push body (Server::CreateSendServerPushRowMsgsPartial, server.cpp:311-420): the
 * same framing as psx_serialize_dirty, but per table only the first
 * server_push_row_upper_bound candidate rows, in send order.  Candidates are all dirty
 * rows (the reference samples candidates with probability
 * min(1, upper_bound*row_candidate_factor/rows) from a time-seeded generator,
 * server_table.cpp:301-335; with that probability at 1 the sets coincide).  Importance
 * tables send rows by importance, largest first, ties by ascending row id
 * (SortCandidateVectorImportance, server_table.cpp:272-287); other tables in ascending
 * row id (the reference shuffles them randomly, :263-270).  Sent rows have dirty and
 * importance reset when clear_dirty != 0 (AppendRowsToBuffsPartial :398-399).  When no
 * table has a row to send nothing is written and *used = 0 (server.cpp:348).
 * On PSX_ERR_BUFFER_TOO_SMALL *used holds the bytes needed and nothing is cleared. */
psx_status psx_serialize_partial(psx_ctx *ctx, void *out, size_t cap, size_t *used,
                                 int32_t out_on_device, int32_t clear_dirty);

/* ---- message headers --------------------------------------------------------------- */
/* MsgType values (msg_base.hpp:14-40) of the two messages on the path. */
#define PSX_MSG_CLIENT_SEND_OPLOG 12
#define PSX_MSG_SERVER_PUSH_ROW 18
/* ClientSendOpLogMsg (ps_msgs.hpp:1003-1055): the ArbitrarySizedMsg prefix MsgType(4)
 * seq(8) ack(8) avai_size(8) (msg_base.hpp:81-188), then is_clock(1) client_id(4)
 * version(4) bg_clock(4): 41 bytes, packed, little endian; the oplog stream follows. */
#define PSX_OPLOG_MSG_HEADER_BYTES 41
typedef struct psx_oplog_msg_header {
  uint64_t seq_num;     /* NumberedMsg::get_seq_num (flow control, msg_tracker.cpp) */
  uint64_t ack_num;
  uint64_t avai_size;   /* payload bytes */
  int32_t is_clock;     /* bool */
  int32_t client_id;
  uint32_t version;     /* the sender's message version (server.cpp:124-126) */
  int32_t bg_clock;     /* the sender's clock when is_clock (server_thread.cpp:262-263) */
} psx_oplog_msg_header;
/* ServerPushRowMsg (ps_msgs.hpp:1057-1103): the same prefix, then clock(4) version(4)
 * is_clock(1): 37 bytes; the push body follows. */
#define PSX_PUSH_MSG_HEADER_BYTES 37
typedef struct psx_push_msg_header {
  uint64_t seq_num;
  uint64_t ack_num;
  uint64_t avai_size;
  int32_t clock;        /* the server's min clock (ssp_push_server_thread.cpp:28-31) */
  uint32_t version;     /* the receiver's last applied message version */
  int32_t is_clock;
} psx_push_msg_header;
/* out: PSX_OPLOG_MSG_HEADER_BYTES / PSX_PUSH_MSG_HEADER_BYTES bytes.  Decode checks the
 * message type and that avai_size payload bytes follow within msg_size. */
psx_status psx_encode_oplog_header(const psx_oplog_msg_header *h, void *out);
psx_status psx_decode_oplog_header(const void *msg, size_t msg_size, psx_oplog_msg_header *h);
psx_status psx_encode_push_header(const psx_push_msg_header *h, void *out);
psx_status psx_decode_push_header(const void *msg, size_t msg_size, psx_push_msg_header *h);

/* Reference-compatibility mode.  PSX_COMPAT_INT32_STREAM_OFFSETS: reject (PSX_ERR_UNSUPPORTED,
 * nothing applied) any message of 2 GiB or more — the reference's SerializedOpLogReader
 * keeps its cursor in an int32 offset_ (serialized_oplog_reader.hpp:137); producers split
 * larger batches (wire.split_stream).  Default 0: 64-bit offsets, any size. */
#define PSX_COMPAT_INT32_STREAM_OFFSETS 1
psx_status psx_ctx_set_compat(psx_ctx *ctx, int32_t flags);

/* Overlap each apply call's index stage (decode, dense index, claim counts) with the
 * previous call's apply kernels: the stage runs on the context's side stream once call
 * k-2 has finished, so it may start BEFORE work the caller enqueued on the context stream
 * after the previous apply call has finished.  Opt-in contract: the messages (and record
 * lists) of a call are complete when the call is made (e.g. produced before the previous
 * apply call, or synchronized by the caller).  Modes: 0 off (default); PSX_PIPELINE_LISTED
 * for calls whose fast dense tables all place records from record-row lists
 * (psx_apply_indexed_rows with a list for every message: a light index stage); and
 * PSX_PIPELINE_ALL for every call. */
#define PSX_PIPELINE_LISTED 1
#define PSX_PIPELINE_ALL 2
psx_status psx_ctx_set_pipeline(psx_ctx *ctx, int32_t mode);

/* ServerThread::HandleOpLogMsg's server part (server_thread.cpp:224-266) on a whole
 * ClientSendOpLogMsg in host memory: decode the header, apply the payload
 * (psx_apply_stream) and, for a clock message, psx_clock_until(sender, bg_clock);
 * *clock_changed receives the new min clock if it advanced, else 0 (then the caller pushes,
 * psx_serialize_push, and acks). */
psx_status psx_handle_oplog_msg(psx_ctx *ctx, const void *msg, size_t msg_size, int32_t sender,
                                int32_t *clock_changed);

/* ---- clocks (SSP) ------------------------------------------------------------------- */
/* bg_clock_: every registered sender starts at clock 0 (Server::Init, server.cpp:21-24).
 * psx_clock_until advances bg_id's clock to `clock` one tick at a time
 * (VectorClock::TickUntil); *new_min_clock receives the new minimum clock over all
 * senders if it advanced, 0 otherwise — ClockUntil's "clock changed", after which the
 * reference server fulfils waiting row requests and pushes (server_thread.cpp:262-288). */
psx_status psx_clock_until(psx_ctx *ctx, int32_t bg_id, int32_t clock, int32_t *new_min_clock);
psx_status psx_min_clock(psx_ctx *ctx, int32_t *min_clock);
psx_status psx_sender_clock(psx_ctx *ctx, int32_t bg_id, int32_t *clock);

/* ---- subscriptions and the per-client push (SSPPush) --------------------------------- */
/* GlobalContext::get_num_clients(): the clients psx_serialize_push writes bodies for
 * (1..PSX_MAX_CLIENTS, default 1). */
psx_status psx_set_num_clients(psx_ctx *ctx, int32_t num_clients);
/* Row request path (ServerThread::HandleRowRequest, server_thread.cpp:185-200): create each
 * listed row if it does not exist (ServerTable::CreateRow; an AdaRevision table draws its
 * ServerRowCreated initial values, in list order) and subscribe client_id to it. */
psx_status psx_row_subscribe(psx_ctx *ctx, int32_t table_id, const int32_t *row_ids, int32_t n,
                             int32_t client_id);
/* CallBackSubs bitsets of num_rows rows (psx_row_flags addressing), bit c = client c. */
psx_status psx_row_subscriptions(psx_ctx *ctx, int32_t table_id, int64_t first_row, int64_t num_rows,
                                 uint64_t *dst);
/* Server::CreateSendServerPushRowMsgs as SSPPush runs it: one body per client c in
 * [0, num_clients), written to out[c] (cap[c] bytes; used[c] receives its size): per
 * table (creation order) int32 table_id, the dirty rows client c subscribes to as
 * RecordBuff records in ascending row id, int32 -1 between tables, -2 at the end.  Every
 * client gets a body, even one without rows.  With clear_dirty, a dirty row some client
 * subscribes to has dirty and importance reset and ServerRowSent(its subscriber count)
 * runs; a dirty row nobody subscribes to stays dirty (server_table.cpp:222-225).
 * PSX_ERR_BUFFER_TOO_SMALL (out == NULL or some cap too small): used[] holds the sizes,
 * nothing is cleared.  psx_serialize_dirty is the single-body form in which one client
 * subscribes to every row.  out_on_device: out[c] are 4-byte-aligned device buffers. */
psx_status psx_serialize_push(psx_ctx *ctx, void *const *out, const size_t *cap, size_t *used,
                              int32_t out_on_device, int32_t clear_dirty);

/* ---- client side of serve-back ------------------------------------------------------ */
/* A push body (or row-request reply) applied to this context used as a client process
 * cache: SSPPushBgWorker::ApplyServerPushedRow (ssp_push_bg_worker.cpp:70-122) walks it
 * with SerializedRowReader (serialized_row_reader.hpp:30-100) and, for every record of a
 * row the cache holds (flags bit0; with insert_missing also rows it does not hold —
 * InsertNonexistentRow, abstract_bg_worker.cpp:853-870), replaces the row with the bytes:
 * ResetRowData (numeric_store_row.hpp:142-145) — dense rows are overwritten
 * (VectorStore::ResetData), sorted/map rows are rebuilt from the entries (Deserialize).
 * Version tables take the trailing uint64 as the row's version (ExtractRowVersion,
 * abstract_bg_worker.cpp:1032-1040).  A row twice in one body ends with its last record.
 * Oplog replay onto the reset row (no_oplog_replay = false) is the caller's.  Records of
 * rows outside the context's shard are skipped; an unknown table, a malformed body or a
 * sorted/map row over max_entries fails the call with nothing applied.  body_on_device: a
 * 4-byte-aligned device buffer (walked on the device); otherwise host bytes, borrowed for
 * the call.  Synchronous. */
psx_status psx_apply_push_body(psx_ctx *ctx, const void *body, size_t size, int32_t body_on_device,
                               int32_t insert_missing);

/* ---- AdaRevision server-table logic ------------------------------------------------ */
/* AdaRevisionServerTableLogic (src/petuum_ps/server/adarevision_server_table_logic.cpp),
 * the server-table logic apps register as TableInfo.server_table_logic
 * (apps/matrixfact/src/matrixfact_adarevision.cpp:633-635; its run script sets
 * server_table_logic=1 and version_maintain=true).  Per record, per element, in f32:
 * g_bck = accum - accum_at(record's row version, 0 if none); eta_old = step/sqrt(z_max);
 * z += u*(u + 2*g_bck); z_max = max(z, z_max); eta = step/sqrt(z_max);
 * delta = -(eta*u) + (eta_old - eta)*g_bck; accum += u; then the row gets += delta through
 * the table's ordinary apply (dirty, importance, version).  A push (psx_serialize_dirty /
 * _partial with clear_dirty) and psx_row_sent snapshot accum under (row, row version) for
 * num_clients clients; a record with end_of_version releases one client. */
typedef struct psx_adarevision_config {
  float init_step_size;            /* FLAGS_init_step_size (:8; reference default 0.1) */
  int32_t gaussian_init;           /* FLAGS_random_init == "guassian" (:10,30-34,43-49; the default):
                                      a row created by an apply first gets row_capacity N(0, 0.1)
                                      draws of one mt19937(12345), in creation order */
  uint64_t old_grad_upper_bound;   /* FLAGS_old_grad_upper_bound (:9; default 10000): the partial push
                                      sends nothing from the table while that many snapshots are live
                                      (AllowSend, :192-197; server_table.cpp:293-295) */
  int32_t push_clients;            /* num_clients of ServerRowSent for the push paths = clients subscribed
                                      to the pushed rows (server_table.cpp:253-254,413-414); 0 -> 1 */
  int32_t max_snapshots_per_row;   /* HBM slots per row for live snapshots, 1..8; 0 -> 4.  Exceeding it is
                                      PSX_ERR_CAPACITY (the reference's map is unbounded) */
} psx_adarevision_config;

/* Attach the logic to a table before its first apply: f32 dense rows, dense-serialized
 * kDenseRowOpLog records of row_capacity values (:65-68).  A context with an AdaRevision
 * table takes dense-serialized tables only and rejects a row twice in one message
 * (PSX_ERR_UNSUPPORTED at psx_sync): there is no ordered replay for the logic. */
psx_status psx_table_set_adarevision(psx_ctx *ctx, int32_t table_id, const psx_adarevision_config *cfg);
/* Server::RowSent after a row request reply (server_thread.cpp:221, server.cpp:436-441):
 * ServerRowSent for the listed rows; a no-op for tables without a logic. */
psx_status psx_row_sent(psx_ctx *ctx, int32_t table_id, const int32_t *row_ids, int32_t n,
                        int32_t num_clients);
/* AdaRevisionRow state of num_rows rows (accum_gradients_, z_, z_max_; [num_rows][row_capacity]
 * each, any may be NULL) and the number of live snapshots (old_accum_gradients_.size()). */
psx_status psx_adarevision_state(psx_ctx *ctx, int32_t table_id, int64_t first_row, int64_t num_rows,
                                 float *accum, float *z, float *z_max, uint64_t *live_snapshots);

/* ---- client-side pack ------------------------------------------------------------ */
/* One table's oplog rows for psx_pack_stream: row i's oplog is the `capacity` values at
 * oplogs + i*capacity (a DenseRowOpLog's oplogs_, dense_row_oplog.hpp). Device memory. */
typedef struct psx_pack_table {
  int32_t table_id;
  int32_t dtype;              /* psx_dtype */
  int32_t dense_serialized;   /* TableInfo.oplog_dense_serialized: 1 SerializeDense, 0 SerializeSparse */
  int32_t reserved0;          /* must be 0 */
  int64_t capacity;           /* dense_row_oplog_capacity (values per row oplog) */
  int64_t num_rows;
  const int32_t *row_ids;     /* device, num_rows */
  const void *oplogs;         /* device, num_rows * capacity values */
} psx_pack_table;

/* Pack n tables into one message payload (Appendix A) on the device, byte-identical to
 * the reference client's CreateOpLogMsgs + OpLogSerializer + RowOpLogSerializer:
 * tables in ascending id, tables with no rows omitted, records in the given row order;
 * dense records V[capacity]; sparse records the non-zero (`!= 0`) columns ascending.
 * No table with rows -> *used = 0 (an empty message, abstract_bg_worker.cpp:670-682).
 * out: 4-byte-aligned device buffer of cap bytes (NULL to size: returns
 * PSX_ERR_BUFFER_TOO_SMALL with *used).  record_offsets (optional, device): receives
 * for every record, in message order, the byte offset of its row id — a producer-side
 * record index.  Synchronous on the context stream. */
psx_status psx_pack_stream(psx_ctx *ctx, const psx_pack_table *tables, int32_t n, void *out,
                           size_t cap, size_t *used, uint64_t *record_offsets);
/* psx_pack_stream that also writes record_rows (optional, device int32): the row id of
 * every record in message order, for psx_apply_indexed_rows. */
psx_status psx_pack_stream_indexed(psx_ctx *ctx, const psx_pack_table *tables, int32_t n, void *out,
                                   size_t cap, size_t *used, uint64_t *record_offsets, int32_t *record_rows);

/* ---- multi-GPU: the per-server split and the exchange ------------------------------ */
/* The client's per-server split (AbstractBgWorker::CreateOpLogMsgs, abstract_bg_worker.cpp:
 * 590-649, routing each row by GetPartitionServerID, row_oplog_serializer.hpp:100-124) of
 * one packed message resident on this context's GPU: owner o (0 <= o < nowners) owns rows
 * [row_begin[o], row_begin[o + 1]) (row-range shards; row_begin has nowners + 1 entries).
 * out receives the owners' sub-streams back to back in owner order (device, 4-byte
 * aligned), each a complete Appendix-A message: its tables in the message's order, tables
 * without records for the owner omitted, records in message order; out_sizes[o] (host)
 * its bytes — 0 (an empty message, abstract_bg_worker.cpp:670-682) for an owner with no
 * records.  The tables are this context's (record formats); record_offsets as in
 * psx_apply_indexed (NULL: sparse tables are walked).  A row outside every owner's range
 * is PSX_ERR_ROW_RANGE.  out == NULL or out_cap too small: PSX_ERR_BUFFER_TOO_SMALL with
 * out_sizes filled; size + nowners * (4 + 16 * tables in the message) always suffices.
 * Synchronous on the context stream. */
#define PSX_MAX_SPLIT_OWNERS 64
psx_status psx_split_stream(psx_ctx *ctx, const void *stream, size_t size, const uint64_t *record_offsets,
                            int32_t nowners, const int64_t *row_begin, void *out, size_t out_cap,
                            uint64_t *out_sizes);
/* ABI 7: psx_split_stream with the record formats given by the caller instead of the
 * context's tables — the client side of the split needs only each table's record format
 * (TableInfo's dtype, row kind, oplog_dense_serialized, dense_row_oplog_capacity,
 * version_maintain, row_oplog_type; the reference client's sample row oplog,
 * server_table.cpp:56-67), not a server table.  formats[i] is checked as psx_table_create
 * checks those fields; the shard geometry (row_offset, row_stride, max_rows) is ignored and
 * nothing is allocated for rows.  ctx supplies the device, the stream and the split's
 * scratch.  A message whose tables are all dense-serialized needs no record-offset buffer. */
psx_status psx_split_stream_formats(psx_ctx *ctx, const psx_table_config *formats, int32_t nformats,
                                    const void *stream, size_t size, const uint64_t *record_offsets,
                                    int32_t nowners, const int64_t *row_begin, void *out, size_t out_cap,
                                    uint64_t *out_sizes);

/* The exchange (RCCL over xGMI, one process per GPU): replaces the reference's ZeroMQ
 * transport of per-server messages (SendOpLogMsgs, abstract_bg_worker.cpp:651-689 ->
 * ServerThread receive, server_thread.cpp:419-426) for batches already on the GPUs.
 * psx_comm_unique_id on one rank; every rank passes the same id to psx_comm_create.
 * psx_exchange_sizes then psx_exchange_streams are collectives: send holds nranks
 * sub-streams back to back in owner order (send_sizes[p] bytes for rank p, multiples of
 * 4); recv receives the sub-streams addressed to this rank back to back in source-rank
 * order (recv_sizes[p] from rank p, as psx_exchange_sizes returned them) — the order
 * psx_apply_streams_device then applies them in.  hip_stream: the stream both run on
 * (NULL: the null stream); psx_exchange_sizes synchronizes it, psx_exchange_streams does
 * not. */
#define PSX_COMM_ID_BYTES 128
typedef struct psx_comm psx_comm;
psx_status psx_comm_unique_id(void *id);
psx_status psx_comm_create(const void *id, int32_t nranks, int32_t rank, int32_t device, psx_comm **out);
psx_status psx_comm_destroy(psx_comm *comm);
const char *psx_comm_last_error(psx_comm *comm);
psx_status psx_exchange_sizes(psx_comm *comm, const uint64_t *send_sizes, uint64_t *recv_sizes, void *hip_stream);
psx_status psx_exchange_streams(psx_comm *comm, const void *send, const uint64_t *send_sizes, void *recv,
                                const uint64_t *recv_sizes, void *hip_stream);
/* ABI 7: psx_exchange_streams with explicit byte displacements (MPI alltoallv's): peer p's
 * send_sizes[p] bytes start at send + send_displs[p], and p's recv_sizes[p] bytes land at
 * recv + recv_displs[p].  A zero size skips the peer — e.g. a rank's own sub-stream, which
 * its owner can apply straight from the send buffer instead of copying it to itself. */
psx_status psx_exchange_streams_v(psx_comm *comm, const void *send, const uint64_t *send_sizes,
                                  const uint64_t *send_displs, void *recv, const uint64_t *recv_sizes,
                                  const uint64_t *recv_displs, void *hip_stream);
/* ABI 7: psx_exchange_sizes without the synchronization, so that a pipelined caller can
 * enqueue chunk k+1's sizes behind chunk k's bytes: send_sizes is copied before the call
 * returns; recv_sizes (page-locked host memory, else PSX_ERR_INVALID_ARG) is written by
 * hip_stream and valid once the stream has passed this call (an event recorded after it,
 * or hipStreamSynchronize).  Same collective as psx_exchange_sizes (every rank calls it in
 * the same order). */
psx_status psx_exchange_sizes_async(psx_comm *comm, const uint64_t *send_sizes, uint64_t *recv_sizes,
                                    void *hip_stream);
/* ABI 9: what RCCL itself reports for this communicator, so that a multi-GPU run can show
 * how many ranks the exchange really spanned (not the launcher's world size):
 * nranks = ncclCommCount, rank = ncclCommUserRank, device = ncclCommCuDevice, version =
 * ncclGetVersion (e.g. 22603 for 2.26.3), path = the librccl shared object this process
 * loaded (dl_iterate_phdr), NUL-terminated and cut to path_cap bytes.  Any out pointer may
 * be NULL.  The reference's equivalent fact is the server list a client sends to
 * (GetPartitionServerID, context.hpp:291-304). */
psx_status psx_comm_info(psx_comm *comm, int32_t *nranks, int32_t *rank, int32_t *device, int32_t *version,
                         char *path, size_t path_cap);
/* ABI 9: bytes this rank has enqueued for each peer (sent[p]) and from each peer (recv[p])
 * through psx_exchange_streams(_v) since psx_comm_create or the last reset (reset != 0
 * zeroes the counters after reading them); each array holds nranks entries (NULL skips
 * it).  The per-server byte counts the reference's bg worker accumulates per send
 * (abstract_bg_worker.cpp:651-689). */
psx_status psx_comm_peer_bytes(psx_comm *comm, uint64_t *sent, uint64_t *recv, int32_t reset);

/* ---- server statistics ------------------------------------------------------------ */
/* ABI 7: what the reference server thread accumulates around each apply with
 * STATS_SERVER_ACCUM_APPLY_OPLOG_BEGIN/END (server_thread.cpp:240-244 ->
 * server_accum_apply_oplog_sec / server_accum_oplog_recv_mb, stats.cpp:1153-1162), per
 * context, since its creation or the last reset.  Always on, at one event pair per psx_sync
 * interval (not per call: an event costs the queue a few microseconds). */
typedef struct psx_apply_stats {
  uint64_t calls;          /* apply calls accepted (psx_apply_stream and the device forms) */
  uint64_t messages;       /* ClientSendOpLogMsg payloads in them */
  uint64_t oplog_bytes;    /* their payload bytes (server_accum_oplog_recv_mb = oplog_bytes / 2^20) */
  double apply_sec;        /* server_accum_apply_oplog_sec: per psx_sync interval, the device time from
                              its first call's first stage to its last call's finish, summed (idle
                              time between the calls of an interval included; a duplicate-row
                              replay, run inside psx_sync, is not in it) */
  uint64_t settled_calls;  /* calls whose time is in apply_sec (those settled by a psx_sync) */
} psx_apply_stats;
/* Copy the statistics into *out (may be NULL); reset != 0 zeroes them afterwards. */
psx_status psx_ctx_stats(psx_ctx *ctx, psx_apply_stats *out, int32_t reset);

/* ---- diagnostics ---------------------------------------------------------------- */
const char *psx_last_error(psx_ctx *ctx);
const char *psx_status_string(psx_status s);
/* Per-kernel HIP-event timing on the context stream (off by default).  on: 0 off,
 * 1 every pipeline kernel, 2 only the apply kernels (dense_apply / ada_apply /
 * ordered_apply: one event pair per launch, the least perturbation of a timed loop). */
psx_status psx_timing_enable(psx_ctx *ctx, int32_t on);
psx_status psx_timing_read(psx_ctx *ctx, const char *kernel, double *total_ms,
                           int64_t *launches);
psx_status psx_timing_reset(psx_ctx *ctx);

#ifdef __cplusplus
}
#endif

#endif /* PSX_H_ */
