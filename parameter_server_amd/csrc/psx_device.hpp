// psx_device.hpp — definitions shared by the host runtime and the CDNA4 kernels.
//
// Device layout (one context = one server shard, see DESIGN.md "Data layout in HBM"):
//   dense table   : V rows[max_rows][row_capacity]            (slot-major, row_capacity*sizeof(V) B/row)
//   row flags     : uint8 flags[max_rows]  bit0 exists, bit1 dirty  (ServerRow::dirty_, server_row.hpp:133)
//   inverse index : int32 inv[B][max_rows]  record number of slot s in message b, -1 = absent.
//                   All -1 between calls: the apply kernel restores every entry it reads.
//   segments      : Seg segs[kMaxFused][kMaxTables]  (stream b, table t) decoded by decode_streams
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace psx {

constexpr int kMaxFused = 16;   // == PSX_MAX_FUSED_STREAMS
constexpr int kNsStride = 32;   // OrdArgs::nsplit: uint32 words between two counters
constexpr int kMaxTables = 64;  // == PSX_MAX_TABLES
constexpr int kWave = 64;

// Status bits (device-written).  Per-call word = status[0] (reset by decode at the
// start of each call), sticky word = status[1] (OR of all calls since psx_sync).
enum : uint32_t {
  kStMalformed = 1u << 0,
  kStUnknownTable = 1u << 1,
  kStRowRange = 1u << 2,
  kStCapacity = 1u << 3,
  kStUnsupported = 1u << 4,
  kStDuplicateRow = 1u << 5,   // a row appears twice in one message: replay on the ordered path
  kStState = 1u << 6,          // AdaRevision: a record names a (row, version) with no snapshot
  kStRowsMismatch = 1u << 7,   // a producer record-row list disagrees with its stream (found by the
                               // apply; not fatal to the rest of the call: see psx_apply_indexed_rows)
  kStWalkLost = 1u << 8,       // window-parallel decode: a predecessor window's state never arrived
  kStWalkBound = 1u << 9,      // window-parallel decode: a walker state outside its message's
                               // record-offset range (internal error; nothing applied)
};
constexpr uint32_t kStFatal = kStMalformed | kStUnknownTable | kStRowRange | kStCapacity |
                              kStUnsupported | kStState | kStWalkLost | kStWalkBound;
constexpr int kAdaMaxS = 8;     // AdaRevision snapshot slots per row (psx_adarevision_config)

// Table directory passed by value to the decoder.
struct TableDir {
  int32_t n;
  int32_t table_id[kMaxTables];
  int32_t vsize[kMaxTables];
  int32_t dense_serialized[kMaxTables];
  int64_t dense_body[kMaxTables];   // bytes of a dense record after its row id (dense_body_bytes)
};

// Device-resident messages of one fused call, passed by value.
struct StreamSet {
  const uint8_t *data[kMaxFused];
  uint64_t size[kMaxFused];
  uint64_t recoff_base[kMaxFused];   // sparse record-offset workspace start per stream
  int32_t n;
};

// One (stream, table) segment.
struct Seg {
  int64_t rec0;       // byte offset of the first record's row_id, -1 = table absent
  int32_t num_rows;
  int32_t sparse;     // 1: record offsets live in recoff[recoff_base[b] + k]
  int64_t ord0;       // records of the message before this table (index into a record-row list)
};

// Inverse-index addressing: entry (slot s, message b) lives at inv[s*ss + b*sb]; the
// runtime uses the batch-major layout.
// Batch-major ([b][s]: ss = 1, sb = max_rows) keeps one message's scattered writes
// inside a max_rows*4-byte window so the XCD L2s can merge them.
struct InvLayout {
  int64_t ss;
  int64_t sb;
};

// Arguments of dense_apply (passed by value).
struct DenseArgs {
  StreamSet ss;
  const Seg *segs;
  int t;
  int B;
  int64_t stride;     // record stride in bytes = 4 + cap*sizeof(V)
  int64_t cap;        // dense_row_oplog_capacity (elements applied per record)
  int64_t row_cap;    // row_capacity (elements per table row)
  int64_t max_rows;
  void *table;
  uint8_t *flags;
  int32_t *inv;
  int64_t inv_ss;
  int64_t inv_sb;
  const uint32_t *counters;
  uint32_t *sticky;
  uint32_t *call_status;
  const uint8_t *zero_chunk;   // >= 2 KiB of zeros, stands in for absent messages
  double *imp;                 // non-null: accumulate NSSumImpCalc importance per slot
  uint64_t *ver;               // non-null: VersionServerRow::version_ per slot (+1 per record)
  uint32_t rows_mask;          // bit b: message b was placed from the producer's record rows, so
                               // every record's row id is checked against its slot in the apply
  int64_t row_offset, row_stride;   // shard geometry (expected row id of a slot)
  int32_t store_nt;                 // table-row policy (PSX_VARIANT_DENSE_STORE): bit0 nt store, bit1 nt load
};

// AdaRevision server-table logic on one f32 dense table (psx_ada.hip).
struct AdaArgs {
  StreamSet ss;
  const Seg *segs;
  int t;
  int B;
  int64_t stride;              // dense record stride in bytes
  int64_t cap;                 // row_capacity == dense_row_oplog_capacity
  int64_t max_rows;
  float *table;
  uint8_t *flags;
  int32_t *inv;
  int64_t inv_ss, inv_sb;
  const uint32_t *counters;
  const uint32_t *sticky;
  uint32_t *call_status;
  double *imp;                 // importance tables (SSPAggr)
  uint64_t *ver;               // version tables
  float *acc, *z, *zmax;       // AdaRevisionRow per slot [max_rows][cap]
  int version_records;         // records carry {uint64 version; bool end_of_version}
  float step;                  // init_step_size_
  int S;                       // snapshot slots per row (<= kAdaMaxS)
  uint64_t *snap_ver, *snap_cnt;   // [max_rows][S]; count 0 = free
  float *snap_acc;             // [max_rows][S][cap]
  uint32_t *words;             // [0] live snapshots, [1] rows created this call, [2] error bits
  uint64_t *new_keys;          // rows created this call: (message << 32 | record), slot
  int32_t *new_slots;
};

// Producer-supplied record indexes of one call (psx_apply_indexed): for message b, the
// byte offset of every record's row id, all tables in stream order (psx_pack_stream's
// record_offsets); nullptr: walk that message.  rows[b] (psx_apply_indexed_rows): the row
// id of every record, all tables in stream order (the rows the producer packed).
struct IdxSet {
  const uint64_t *p[kMaxFused];
  const int32_t *rows[kMaxFused];
};

// Fast-path dense tables of one call (for the duplicate-row gate).
struct TableMask {
  int32_t n;
  int32_t t[kMaxTables];
};

// Arguments of the ordered path (psx_ordered.hip).
struct OrdArgs {
  StreamSet ss;
  const Seg *segs;
  int t;
  int B;
  int kind;               // psx_row_kind
  int dense_records;      // 1: records are dense V[cap] (duplicate-row replay)
  int64_t stride;         // dense record stride
  int64_t cap;            // dense_row_oplog_capacity
  int64_t row_cap;        // row_capacity (dense width; bound on sparse columns)
  int64_t row_offset, row_stride, max_rows;
  const uint64_t *recoff;
  int32_t *cnt;
  int32_t *off;
  int32_t *tsum;
  uint64_t *list;         // records grouped by slot: (message << 56) | byte offset of the row id
  uint64_t *list_tmp;     // the list's mirror region: scratch of the long-list sort (> 64 records)
  int32_t *touched;       // slots with >= 1 record this call (unordered)
  uint32_t *ntouched;     // its length (zeroed by decode_streams)
  void *dense;
  int32_t *nent;
  uint8_t *entries;
  int64_t max_entries;
  uint8_t *flags;
  uint32_t *call_status;
  const uint32_t *sticky;
  int force;              // replay: ignore the sticky duplicate flag
  double *imp;            // non-null: accumulate NSSumImpCalc importance per slot
  uint64_t *ver;          // non-null: VersionServerRow::version_ per slot (+1 per record)
  int rec_f16;            // dense records are binary16 (kDenseRowOpLogFloat16)
  uint32_t *keyflag;      // sorted/map tables: set once a key outside [0, max_entries) is seen
                          // (from then on every call runs the capacity dry run)
  int32_t *grow;          // split tables (256 < max_entries <= 1024): entries the call's records
                          // can add per slot (zero between calls); null otherwise
  int32_t *split;         // [2][max_rows] row descriptors {slot, list begin, list end, image
                          // size} (int4): touched slots whose image fits 256 entries, the rest
  uint32_t *nsplit;       // the lists' lengths: 256-entry, 1,024-entry, heavy, capacity dry run, light
                          // (counter k at nsplit[k * kNsStride]: one 128-B line each, so the
                          // blocks' atomics on different counters do not queue on one line)
  int32_t desc;           // 1: `touched` holds split-list row descriptors (the apply launches)
  int32_t spill;          // split tables, spill mode: ordered_offsets sends only rows already
                          // near 256 entries to the 1,024-entry list; the 256-entry launch
                          // hands a row that outgrows its image to that list (spill_list,
                          // nspill) untouched, and the 1,024-entry launch runs after it
  int32_t *spill_list;
  uint32_t *nspill;
  const int32_t *heavy_end;  // heavy-first (spill bit 1): heavy row descriptors end here (the
  const uint32_t *nheavy;    // 256-entry list's region), listed backwards; the 256-entry
                             // launch takes them first
  int32_t lite;              // split tables: ordered_offsets lists light rows apart (starts_lite)
  int32_t probe;             // PSX_DEBUG_ORD_PROBE (timing only, results wrong): 1 the register
                             // apply does each row's setup and write-back but no record
  const int32_t *light;      // the 256-entry launch: light row descriptors, taken four to a wave
  const uint32_t *nlight;    // (lite_quad), after the heavy rows and before the others
  int32_t counted;           // split tables: 1 the walk already counted this call's records
                             // (WalkCount): ordered_count is not launched; 2: it also placed
                             // each record in its slot's list (WalkCount.wfill); 3: ordered_count
                             // counts and places them.  Placed (>= 2): ordered_offsets zeroes
                             // the counts and ordered_fill needs no atomics
  // finish_call folded into this apply launch (the call's last): fin_ring >= 0 is the call's
  // status ring slot, so call_status = status + 1 + fin_ring and the sticky word, the call's
  // log entry and the block counter follow from call_status (kCallRing layout); the last
  // block does finish_call's work (psx_ordered.hip finish_tail).  -1: no fold.
  int32_t fin_ring;
  // The capacity dry run doing ordered_classify's work first (pipelined split tables,
  // psx_ordered.hip launch_ordered_prep_rows): plist/nplist are the call slot's compact
  // touched list and its length (ordered_place); null otherwise.
  const int4 *plist;
  const uint32_t *nplist;
  // Bucket lists (split tables, ranked counts): a slot's records sit at list[slot * bucket_m
  // + place], written by the count (the walk's or ordered_count's) — no prefix over the
  // counts, no ordered_fill.  0: prefix lists.
  int32_t bucket_m;
  int32_t classify_slots;   // the dry run's prologue classifies its 256 slots (bucket lists)
};
// The context's status words (psx_runtime.cpp d_status): [0] sticky, [1 + k] the call ring,
// [1 + kCallRing + k] the call log, [1 + 2 kCallRing] the folded finish's block counter.
constexpr int kCallRing = 64;

// ordered_count's work for one split sorted/map table (grow set), done by the window-parallel
// walk as it writes each record's offset (psx_walk.hip): per record cnt[slot] += 1 and
// grow[slot] += its pairs (prefix lists; with bucket lists the record's list entry instead,
// and the prep sums the pairs, psx_ordered.hip o_grow), kStRowRange for a row outside the
// shard; walk_head zeroes
// ordered_offsets' counters.  The pointers are the call slot's count state (a pipelined walk
// runs beside the previous call's ordered work, which uses the other slot's).
struct WalkCount {
  int64_t row_offset, row_stride, max_rows;
  int32_t *cnt;
  int32_t *grow;
  uint32_t *nsplit;   // ordered_offsets' list counters [0..4]
  int32_t *tsum;      // its record-range base [0]
  int32_t on;
  int32_t pad;
  int2 *wfill;        // non-null: per record (its recoff index) {slot, its place in the slot's record
                      // list} from the count's returned value, for ordered_fill (-1: no slot)
  uint64_t *bucket;   // non-null (bucket lists): the record's list entry goes straight to
  int32_t bucket_m;   // bucket[slot * bucket_m + place]; place >= bucket_m sets kStDuplicateRow
  int32_t pad2;       // (the call is then replayed with prefix lists)
};

// A side stream and two events for launches that run beside the context stream.
struct Fork {
  hipStream_t aux;
  hipEvent_t fork, join;
};

// Arguments of the serve-back kernels (psx_serve.hip).
struct ServeArgs {
  const uint8_t *flags;
  const int32_t *nent;
  const uint8_t *dense;      // dense rows
  const uint8_t *entries;    // sorted/map entries
  int kind;
  int vsize;
  int64_t row_cap;
  int64_t max_entries;
  int64_t row_offset, row_stride, max_rows;
  int64_t *sizes;
  int64_t *offs;
  uint8_t *out;              // record region base (4-byte aligned)
  uint8_t *flags_rw;         // non-null: clear bit1 (dirty) of every emitted row
  double *imp_rw;            // non-null (with flags_rw): reset importance of every emitted row
  const uint64_t *ver;       // non-null: version table, append uint64 version to every row body
  const uint64_t *subs;      // non-null: only rows with (subs[s] & cmask) != 0 (per-client push)
  uint64_t cmask;
  // partial push (psx_serialize_partial)
  const double *imp;         // importance per slot (null: no importance ordering)
  double *keys;              // sort keys per slot: importance (or 0) if dirty, -1 otherwise
  int32_t *vals;             // slot ids (sort payload)
  uint32_t *ndirty;          // dirty-row count
  const int32_t *sel;        // emit list: slots in send order
  int64_t nsel;
  int64_t *lsizes;           // record bytes per list entry
  int64_t *loffs;            // exclusive prefix of lsizes + scan tile sums
  int f16;                   // DenseRowFloat16 rows: row bytes are binary16 (row_cap * 2, records 2-aligned)
};

// One table of a device-side pack (psx_pack.hip).
struct PackTab {
  const int32_t *row_ids;
  const uint8_t *oplogs;   // [nrows][cap] values
  int64_t nrows;
  int64_t cap;
  int32_t vsize;
  int32_t sparse;          // 1: SerializeSparse records
  int32_t src16;           // 1: every oplog row starts 16-byte aligned (dense copies use 16-B loads)
  int64_t rec0;            // byte offset of the table's first record in the message
  int64_t rec_base;        // index of the table's first record in the record-offset index
  int64_t *sizes;          // sparse: record bytes per row
  int64_t *offs;           // sparse: exclusive prefix of sizes (+ scan tile sums)
};

// Message header words of a pack: num_tables and each table header.
struct PackHdr {
  int32_t n;
  int64_t pos[kMaxTables + 1];
  int32_t len[kMaxTables + 1];
  uint32_t w[kMaxTables + 1][4];
};

// Importance term of one dense element (ns_sum_imp_calc.hpp:87-90), before the add:
// |double(u) / double(v)|, |double(u)| when v == 0.
template <typename V>
__device__ __forceinline__ double imp_term(V old, V u) {
  const double dv = (double)old, du = (double)u;
  return __builtin_fabs(dv == 0.0 ? du : du / dv);
}

// f32 values: the IEEE f64 division is ~12 dependent f64 ops and makes the apply
// ALU-bound, so the quotient is built from an f32 reciprocal estimate q0 = u * rcp(v)
// plus one exact f64 remainder step: rem = u - q0*v is exact in f64 (24x24-bit product),
// and q = q0 + rem * rcp(v) has relative error < 2^-45 (vs 2^-53 for the division) —
// inside the importance tolerance (rel 1e-12; importance is an f64 sum of |terms|).
// Non-normal estimates (v or u/v outside the f32 normal range, inf, NaN) take the
// exact division.
template <>
__device__ __forceinline__ double imp_term<float>(float old, float u) {
  if (old == 0.0f) return __builtin_fabs((double)u);
  if (u == 0.0f) return 0.0;
  const float r0 = __builtin_amdgcn_rcpf(old);
  const float q0 = u * r0;
  const float ar = __builtin_fabsf(r0), aq = __builtin_fabsf(q0);
  if (ar >= 1.17549435e-38f && ar <= 3.40282347e38f && aq >= 1.17549435e-38f && aq <= 3.40282347e38f) {
    const double dq0 = (double)q0;
    const double rem = __builtin_fma(-dq0, (double)old, (double)u);
    return __builtin_fabs(__builtin_fma(rem, (double)r0, dq0));
  }
  return __builtin_fabs((double)u / (double)old);
}

// Float16Compressor::decompress (dense_row_oplog_float16.hpp:144-157; third-party header,
// unpinned): binary16 -> binary32 bits, exact for every finite value and infinity (the
// hardware conversion); NaNs keep their payload shifted into the mantissa, unquieted, as
// the oracle's restatement does.
__device__ __forceinline__ uint32_t half_to_f32_bits(uint32_t h) {
  const uint32_t hw = __builtin_bit_cast(uint32_t, (float)__builtin_bit_cast(_Float16, (uint16_t)h));
  const bool nan = (h & 0x7fffu) > 0x7c00u;
  return nan ? (((h & 0x8000u) << 16) | 0x7f800000u | ((h & 0x3ffu) << 13)) : hw;
}

// Float16Compressor::compress (vector_store_float16.hpp:94-96; unpinned third-party header,
// restated from its published algorithm):
// the mantissa truncated, below the smallest normal through float x 2^37 -> int, above
// 65504 -> infinity, NaN payloads kept (the smallest half NaN when their top bits are 0).
__device__ __forceinline__ uint32_t f32_to_half_fc(float value) {
  constexpr int32_t infN = 0x7F800000, maxN = 0x477FE000, minN = 0x38800000;
  constexpr int32_t infC = infN >> 13, nanN = (infC + 1) << 13, maxC = maxN >> 13, minC = minN >> 13;
  constexpr int32_t subC = 0x003FF, maxD = infC - maxC - 1, minD = minC - subC - 1;
  uint32_t u = __builtin_bit_cast(uint32_t, value);
  uint32_t sign = u & 0x80000000u;
  int32_t v = (int32_t)(u ^ sign);
  sign >>= 16;
  const float mag = __builtin_bit_cast(float, v);
  const int32_t sub = minN > v ? (int32_t)(__builtin_bit_cast(float, 0x52000000) * mag) : 0;
  v ^= (sub ^ v) & -(int32_t)(minN > v);
  v ^= (infN ^ v) & -(int32_t)((infN > v) & (v > maxN));
  v ^= (nanN ^ v) & -(int32_t)((nanN > v) & (v > infN));
  v = (int32_t)((uint32_t)v >> 13);
  v ^= ((v - maxD) ^ v) & -(int32_t)(v > maxC);
  v ^= ((v - minD) ^ v) & -(int32_t)(v > subC);
  return ((uint32_t)v | sign) & 0xffffu;
}

__device__ __forceinline__ uint32_t half_to_f32_bits_hw(uint32_t h) {
  return __builtin_bit_cast(uint32_t, (float)__builtin_bit_cast(_Float16, (uint16_t)h));
}

// Butterfly sum over the 64 lanes of a wave; every lane receives the total.
__device__ __forceinline__ double wave_sum_f64(double x) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
  return x;
}

// One record of a push body (psx_client.hip): its table, row, and payload bytes.
struct PushEntry {
  int32_t table_id;
  int32_t row_id;
  uint64_t offset;   // byte offset of the row bytes in the body
  uint64_t size;     // size_t size of the record (row bytes + version trailer)
};

// A client-cache table as the push apply sees it (device array, one per table).
struct ClientTable {
  int32_t table_id;
  int32_t kind;      // psx_row_kind
  int32_t vsize;
  int32_t es;        // sizeof(Entry<V>)
  int64_t row_cap;
  int64_t max_entries;
  int64_t row_offset, row_stride, max_rows;
  uint8_t *flags;
  uint8_t *dense;
  uint8_t *entries;
  int32_t *nent;
  uint64_t *ver;     // version tables: the pushed row version
  int32_t *claim;    // per slot, zero between calls
  int32_t f16;       // DenseRowFloat16 rows: pushed row bytes are binary16, decompressed on reset
};

// psx_split_stream (psx_split.hip): one table of the message being split, stream order.
struct SplitTab {
  int64_t k0;        // flattened index of its first record
  int64_t rec0;      // dense: byte offset of record 0; sparse: index into recoff
  int64_t stride;    // dense record stride
  int32_t sparse;
  int32_t vsize;     // sparse value size
};

constexpr int kMaxSplitOwners = 64;   // == PSX_MAX_SPLIT_OWNERS

struct SplitArgs {
  const uint8_t *msg;
  const uint64_t *recoff;
  const SplitTab *tabs;
  int32_t ntab;
  int32_t nowners;
  int64_t nrec, ntiles;                     // records; tiles of 64 records
  int64_t row_begin[kMaxSplitOwners + 1];   // owner o: rows [row_begin[o], row_begin[o+1])
  uint64_t *src_off, *meta;                 // per record: byte offset; owner << 48 | table << 40 | size
  int64_t *tile_bytes, *tile_pre, *scan_tmp;   // [nowners][ntiles] bytes, its exclusive scan (+1)
  int64_t *ot_count, *ot_bytes;             // [nowners][ntab]
  const int64_t *owner_base, *hdr_shift;    // [nowners], [nowners][ntab]
  uint8_t *out;
  uint32_t *status;
};

// Write a few 4-byte words (table ids and separators) into the body.
struct Words {
  int32_t n;
  int64_t pos[2 * kMaxTables + 1];
  int32_t val[2 * kMaxTables + 1];
};

}  // namespace psx
