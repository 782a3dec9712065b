/*
 * psx_oracle.c — CPU restatement of the Bosen (petuum_ps) row-update apply path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP path in
 * parameter_server_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product path never links or calls it.
 *
 * Pinning: the reference cannot be compiled in this image (its row/store headers
 * include glog/logging.h and boost headers, neither installed, and stand-in headers are
 * not allowed), so this restatement is pinned by the reference's own known-answer
 * tests, transcribed as fixtures in tests/golden/reference_kats.json:
 *   tests/petuum_ps/storage/store_test.cpp:42-49   (VectorInc)
 *   tests/petuum_ps/storage/store_test.cpp:80-92   (SIncGet)
 *   tests/petuum_ps/storage/store_test.cpp:94-116  (SShrink)
 *   apps/lda/src/row_test.cpp:11-46                (SortedVectorMapRow inc + serialize)
 * The wire-format walk (SerializedOpLogReader) is restated from the code and has no
 * reference test of its own: "parity unpinned" for the stream framing itself.
 *
 * Every function cites the reference file:line it restates (paths relative to the
 * reference repo root).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

#define ORC_OK 0
#define ORC_ERR_INVALID_ARG 1
#define ORC_ERR_VERSION 2
#define ORC_ERR_UNKNOWN_TABLE 3
#define ORC_ERR_MALFORMED 4
#define ORC_ERR_CAPACITY 6
#define ORC_ERR_UNSUPPORTED 10
#define ORC_ERR_SENDER 11
#define ORC_ERR_STATE 13

enum { KIND_DENSE = 0, KIND_SORTED_MAP = 1, KIND_MAP = 2 };
enum { DT_F32 = 0, DT_F64 = 1, DT_I32 = 2, DT_I64 = 3 };

static size_t dt_size(int dt) { return (dt == DT_F32 || dt == DT_I32) ? 4 : 8; }

/* ------------------------------------------------------------------------ */
/* Scalar helpers: V += d and V == 0 for the four value types.  Integer adds wrap
 * (two's complement), which is what the reference's int32/int64 += does on every
 * platform it builds for. */
typedef union { float f; double d; int32_t i; int64_t l; uint64_t raw; } val_t;

static val_t v_load(const void *p, int dt) {
  val_t v; v.raw = 0;
  memcpy(&v, p, dt_size(dt));
  return v;
}
static void v_store(void *p, val_t v, int dt) { memcpy(p, &v, dt_size(dt)); }
static val_t v_add(val_t a, val_t b, int dt) {
  val_t r; r.raw = 0;
  switch (dt) {
    case DT_F32: r.f = a.f + b.f; break;
    case DT_F64: r.d = a.d + b.d; break;
    case DT_I32: r.i = (int32_t)((uint32_t)a.i + (uint32_t)b.i); break;
    default: r.l = (int64_t)((uint64_t)a.l + (uint64_t)b.l); break;
  }
  return r;
}
static int v_is_zero(val_t a, int dt) {
  switch (dt) {
    case DT_F32: return a.f == 0.0f;
    case DT_F64: return a.d == 0.0;
    case DT_I32: return a.i == 0;
    default: return a.l == 0;
  }
}
/* a < b and a > b as in SortedVectorMapStore::LinearSearchAndMove
 * (sorted_vector_map_store.hpp:241-286). */
static int v_lt(val_t a, val_t b, int dt) {
  switch (dt) {
    case DT_F32: return a.f < b.f;
    case DT_F64: return a.d < b.d;
    case DT_I32: return a.i < b.i;
    default: return a.l < b.l;
  }
}

/* ------------------------------------------------------------------------ */
/* Open-addressing int32 -> int64 map; stands in for boost::unordered_map<int32,
 * ServerRow*> (server_table.hpp:158) and std::unordered_map<int32,V> (map_store.hpp:45). */
typedef struct {
  int32_t *keys;
  int64_t *vals;
  uint8_t *used;   /* 0 empty, 1 used, 2 tombstone */
  int64_t cap;
  int64_t count;
  int64_t tombs;
} imap_t;

static uint64_t hash32(int32_t k) {
  uint64_t x = (uint32_t)k;
  x ^= x >> 16; x *= 0x7feb352dULL; x ^= x >> 15; x *= 0x846ca68bULL; x ^= x >> 16;
  return x;
}
static int imap_init(imap_t *m, int64_t cap) {
  int64_t c = 16;
  while (c < cap * 2) c <<= 1;
  m->keys = (int32_t *)calloc((size_t)c, sizeof(int32_t));
  m->vals = (int64_t *)calloc((size_t)c, sizeof(int64_t));
  m->used = (uint8_t *)calloc((size_t)c, 1);
  m->cap = c; m->count = 0; m->tombs = 0;
  return (m->keys && m->vals && m->used) ? 0 : -1;
}
static void imap_free(imap_t *m) { free(m->keys); free(m->vals); free(m->used); memset(m, 0, sizeof(*m)); }
static int64_t imap_find(const imap_t *m, int32_t k) {
  if (m->cap == 0) return -1;
  uint64_t i = hash32(k) & (uint64_t)(m->cap - 1);
  for (;;) {
    if (m->used[i] == 0) return -1;
    if (m->used[i] == 1 && m->keys[i] == k) return (int64_t)i;
    i = (i + 1) & (uint64_t)(m->cap - 1);
  }
}
static int imap_grow(imap_t *m);
static int64_t imap_insert(imap_t *m, int32_t k, int64_t v) {
  int64_t f = imap_find(m, k);
  if (f >= 0) { m->vals[f] = v; return f; }
  if ((m->count + m->tombs + 1) * 2 > m->cap) { if (imap_grow(m)) return -1; }
  uint64_t i = hash32(k) & (uint64_t)(m->cap - 1);
  while (m->used[i] == 1) i = (i + 1) & (uint64_t)(m->cap - 1);
  if (m->used[i] == 2) m->tombs--;
  m->used[i] = 1; m->keys[i] = k; m->vals[i] = v; m->count++;
  return (int64_t)i;
}
static int imap_grow(imap_t *m) {
  imap_t n;
  if (imap_init(&n, (m->count + 1) * 2)) return -1;
  for (int64_t i = 0; i < m->cap; ++i)
    if (m->used[i] == 1) imap_insert(&n, m->keys[i], m->vals[i]);
  imap_free(m);
  *m = n;
  return 0;
}
static void imap_erase_at(imap_t *m, int64_t slot) { m->used[slot] = 2; m->count--; m->tombs++; }

/* ------------------------------------------------------------------------ */
/* std::mt19937 ([rand.eng.mers], C++11) and libstdc++'s normal_distribution<float>
 * (bits/random.tcc: Marsaglia's polar method on generate_canonical<float, 24> draws, the
 * second value of each pair cached): AdaRevisionServerTableLogic draws every row it creates
 * from one mt19937(12345) through normal_distribution<float>(0, 0.1)
 * (adarevision_server_table_logic.cpp:30-34,43-46).  Restated here (the product uses
 * <random> itself); pinned to libstdc++ by tests/golden/make_rng_golden.cpp. */
typedef struct { uint32_t mt[624]; int idx; int saved_ok; float saved; } orc_rng;

static void rng_seed(orc_rng *g, uint32_t s) {
  g->mt[0] = s;
  for (int i = 1; i < 624; ++i) g->mt[i] = 1812433253u * (g->mt[i - 1] ^ (g->mt[i - 1] >> 30)) + (uint32_t)i;
  g->idx = 624;
  g->saved_ok = 0;
  g->saved = 0.0f;
}
static uint32_t rng_u32(orc_rng *g) {
  if (g->idx >= 624) {
    for (int i = 0; i < 624; ++i) {
      uint32_t y = (g->mt[i] & 0x80000000u) | (g->mt[(i + 1) % 624] & 0x7fffffffu);
      g->mt[i] = g->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    g->idx = 0;
  }
  uint32_t y = g->mt[g->idx++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}
/* generate_canonical<float, 24>: one 32-bit draw, (float)x / 2^32, kept below 1 */
static float rng_canonical(orc_rng *g) {
  float r = (float)rng_u32(g) / 4294967296.0f;
  return r >= 1.0f ? nextafterf(1.0f, 0.0f) : r;
}
static float rng_normal(orc_rng *g, float mean, float stddev) {
  float ret;
  if (g->saved_ok) {
    g->saved_ok = 0;
    ret = g->saved;
  } else {
    float x, y, r2;
    do {
      x = (float)(2.0f * rng_canonical(g) - 1.0);   /* result_type(2.0) * u - 1.0: a double subtraction */
      y = (float)(2.0f * rng_canonical(g) - 1.0);
      r2 = x * x + y * y;
    } while (r2 > 1.0 || r2 == 0.0);
    const float mult = sqrtf(-2 * logf(r2) / r2);
    g->saved = x * mult;
    g->saved_ok = 1;
    ret = y * mult;
  }
  return ret * stddev + mean;
}

/* Test hook: the first n draws of normal_distribution<float>(mean, stddev) on mt19937(seed). */
void orc_rng_normals(uint32_t seed, float mean, float stddev, int64_t n, float *out) {
  orc_rng g;
  rng_seed(&g, seed);
  for (int64_t i = 0; i < n; ++i) out[i] = rng_normal(&g, mean, stddev);
}

/* old_accum_gradients_ entry: (row, version) -> (accum_gradients_, clients left)
 * (adarevision_server_table_logic.hpp:64-67) */
typedef struct { int32_t row; uint64_t version; float *acc; size_t count; } orc_snap;

/* ------------------------------------------------------------------------ */
/* Rows. */
typedef struct {
  /* dense: VectorStore<V> (vector_store.hpp:64-102), zeroed at Init */
  uint8_t *dense;
  /* sorted map: SortedVectorMapStore<V> (sorted_vector_map_store.hpp) */
  uint8_t *entries;      /* Entry<V>{int32 first; V second} packed per the C++ layout */
  int64_t num_entries;
  int64_t capacity;
  /* map: MapStore<V> (map_store.hpp:45) col -> index into vals */
  imap_t map;
  int dirty;             /* ServerRow::dirty_ (server_row.hpp:133) */
  double importance;     /* ServerRow::importance_ (server_row.hpp:143); the reference leaves it
                            uninitialized (:16-19), this restatement starts it at 0 */
  uint64_t version;      /* VersionServerRow::version_ (version_server_row.hpp:13-19,69): 1 at
                            creation, +1 per applied record; read only for version tables */
  float *ada_acc, *ada_z, *ada_zmax;   /* AdaRevisionRow (adarevision_server_table_logic.hpp:11-22) */
  uint64_t subs;         /* CallBackSubs::subscriptions_ (callback_subs.hpp:96), client c = bit c */
} orc_row;

typedef struct {
  int32_t table_id;
  int kind, dt;
  int dense_serialized;
  int64_t row_capacity;
  int64_t oplog_capacity;
  int importance;        /* ApplyRow*AccumImportance selected (server_table.cpp:26-47) */
  int version_maintain;  /* TableInfo.version_maintain (configs.hpp:207) */
  int f16_records;       /* row_oplog_type kDenseRowOpLogFloat16 (configs.hpp:39) */
  int f16_rows;          /* DenseRowFloat16 rows: served as binary16 (vector_store_float16.hpp:91-99) */
  int ada;               /* AdaRevisionServerTableLogic attached (server_table.cpp:83-93) */
  float ada_step;        /* FLAGS_init_step_size (adarevision_server_table_logic.cpp:8,22) */
  uint64_t ada_upper;    /* FLAGS_old_grad_upper_bound (:9,192-197) */
  int ada_gauss;         /* FLAGS_random_init == "guassian" (:10,30-34) */
  size_t ada_clients;    /* clients a pushed row goes to (ServerRowSent's num_clients) */
  orc_rng ada_rng;
  orc_snap *snaps;       /* old_accum_gradients_ */
  int64_t nsnaps, snaps_cap;
  imap_t index;          /* row_id -> row number */
  orc_row **rows;
  int64_t nrows, rows_cap;
} orc_table;

typedef struct {
  orc_table *tables[64];
  int ntables;
  int32_t bg_ids[1024];
  int64_t bg_versions[1024];
  int32_t bg_clocks[1024];   /* bg_clock_ (server.hpp; VectorClock, vector_clock.cpp) */
  int32_t min_clock;         /* VectorClock::min_clock_: -1 until the first AddClock */
  int nbg;
} orc_server;

/* sizeof(Entry<V>) with natural alignment: {int32, int32} = 8, {int32, 8B} = 16. */
static size_t entry_size(int dt) { return dt_size(dt) == 4 ? 8 : 16; }
static size_t entry_val_off(int dt) { return dt_size(dt) == 4 ? 4 : 8; }

orc_server *orc_server_create(void) {
  orc_server *s = (orc_server *)calloc(1, sizeof(orc_server));
  if (s) s->min_clock = -1;   /* VectorClock() : min_clock_(-1) (vector_clock.cpp:5-6) */
  return s;
}

static void row_free(orc_table *t, orc_row *r) {
  free(r->dense); free(r->entries);
  free(r->ada_acc); free(r->ada_z); free(r->ada_zmax);
  if (t->kind == KIND_MAP) imap_free(&r->map);
  free(r);
}

void orc_server_destroy(orc_server *s) {
  if (!s) return;
  for (int i = 0; i < s->ntables; ++i) {
    orc_table *t = s->tables[i];
    for (int64_t r = 0; r < t->nrows; ++r) row_free(t, t->rows[r]);
    for (int64_t k = 0; k < t->nsnaps; ++k) free(t->snaps[k].acc);
    free(t->snaps);
    free(t->rows); imap_free(&t->index); free(t);
  }
  free(s);
}

/* Server::Init: bg_version_map_[bg] = -1 (server.cpp:21-24). */
/* Server::Init (server.cpp:18-31): bg_clock_.AddClock(bg, 0), bg_version_map_[bg] = -1.
 * AddClock (vector_clock.cpp:19-26) lowers min_clock_ to the new clock, or sets it when
 * it is still -1. */
int orc_register_sender(orc_server *s, int32_t bg) {
  for (int i = 0; i < s->nbg; ++i) if (s->bg_ids[i] == bg) return ORC_OK;
  if (s->nbg >= 1024) return ORC_ERR_INVALID_ARG;
  s->bg_ids[s->nbg] = bg; s->bg_versions[s->nbg] = -1; s->bg_clocks[s->nbg] = 0; s->nbg++;
  if (s->min_clock == -1 || 0 < s->min_clock) s->min_clock = 0;
  return ORC_OK;
}

/* VectorClock::IsUniqueMin (vector_clock.cpp:66-79) */
static int clock_is_unique_min(const orc_server *s, int i) {
  if (s->bg_clocks[i] != s->min_clock) return 0;
  int n = 0;
  for (int k = 0; k < s->nbg; ++k)
    if (s->bg_clocks[k] == s->min_clock && ++n > 1) return 0;
  return 1;
}

/* Server::ClockUntil -> VectorClock::TickUntil (server.cpp:62-79, vector_clock.cpp:38-51):
 * tick the sender's clock up to `clock`, one Tick (:28-36) at a time; returns the new
 * min clock if it advanced, 0 otherwise; -1 for an unknown sender.  (No snapshots: the
 * snapshot_clock branch is out of scope.) */
int32_t orc_clock_until(orc_server *s, int32_t bg, int32_t clock) {
  int i = 0;
  while (i < s->nbg && s->bg_ids[i] != bg) ++i;
  if (i == s->nbg) return -1;
  int32_t changed = 0;
  for (int32_t n = clock - s->bg_clocks[i]; n > 0; --n) {
    if (clock_is_unique_min(s, i)) {
      ++s->bg_clocks[i];
      changed = ++s->min_clock;
    } else {
      ++s->bg_clocks[i];
    }
  }
  return changed;
}

int32_t orc_min_clock(orc_server *s) { return s->min_clock; }   /* Server::GetMinClock (:181-184) */

static orc_table *find_table(orc_server *s, int32_t table_id) {
  for (int i = 0; i < s->ntables; ++i) if (s->tables[i]->table_id == table_id) return s->tables[i];
  return NULL;
}

/* Server::CreateTable / ServerTable::ServerTable (server.cpp:33-44,
 * server_table.cpp:19-93). */
int orc_table_create(orc_server *s, int32_t table_id, int kind, int dt, int dense_serialized,
                     int64_t row_capacity, int64_t oplog_capacity) {
  if (s->ntables >= 64 || find_table(s, table_id)) return ORC_ERR_INVALID_ARG;
  if (kind < 0 || kind > 2 || dt < 0 || dt > 3) return ORC_ERR_INVALID_ARG;
  if (dense_serialized && (oplog_capacity <= 0)) return ORC_ERR_INVALID_ARG;
  if (kind == KIND_DENSE && dense_serialized && oplog_capacity > row_capacity) return ORC_ERR_INVALID_ARG;
  orc_table *t = (orc_table *)calloc(1, sizeof(orc_table));
  t->table_id = table_id; t->kind = kind; t->dt = dt; t->dense_serialized = dense_serialized;
  t->row_capacity = row_capacity; t->oplog_capacity = oplog_capacity;
  imap_init(&t->index, 1024);
  s->tables[s->ntables++] = t;
  return ORC_OK;
}

/* ServerTable::CreateRow -> AbstractRow::Init(row_capacity) (server_table.cpp:143-162). */
static orc_row *create_row(orc_table *t, int32_t row_id) {
  orc_row *r = (orc_row *)calloc(1, sizeof(orc_row));
  r->version = 1;   /* VersionServerRow(row_data): version_(1) (version_server_row.hpp:17-19) */
  if (t->ada) {     /* AdaRevisionRow(row_size): accum 0, z 1, z_max 1 (adarevision_server_table_logic.hpp:12-16) */
    size_t n = (size_t)(t->row_capacity ? t->row_capacity : 1);
    r->ada_acc = (float *)calloc(n, sizeof(float));
    r->ada_z = (float *)malloc(n * sizeof(float));
    r->ada_zmax = (float *)malloc(n * sizeof(float));
    for (size_t i = 0; i < n; ++i) { r->ada_z[i] = 1.0f; r->ada_zmax[i] = 1.0f; }
  }
  if (t->kind == KIND_DENSE) {
    r->dense = (uint8_t *)calloc((size_t)(t->row_capacity ? t->row_capacity : 1), dt_size(t->dt));
  } else if (t->kind == KIND_SORTED_MAP) {
    /* SortedVectorMapStore::Init(capacity) (sorted_vector_map_store.hpp:131-135) */
    r->capacity = t->row_capacity;
    r->entries = (uint8_t *)malloc((size_t)(r->capacity ? r->capacity : 1) * entry_size(t->dt));
  } else {
    imap_init(&r->map, 16);
  }
  if (t->nrows == t->rows_cap) {
    t->rows_cap = t->rows_cap ? t->rows_cap * 2 : 1024;
    t->rows = (orc_row **)realloc(t->rows, (size_t)t->rows_cap * sizeof(orc_row *));
  }
  t->rows[t->nrows] = r;
  imap_insert(&t->index, row_id, t->nrows);
  t->nrows++;
  return r;
}

static orc_row *find_row(orc_table *t, int32_t row_id) {
  int64_t slot = imap_find(&t->index, row_id);
  return slot < 0 ? NULL : t->rows[t->index.vals[slot]];
}

/* ---- SortedVectorMapStore<V> (sorted_vector_map_store.hpp) --------------- */
#define ENT_KEY(r, i, es) (*(int32_t *)((r)->entries + (size_t)(i) * (es)))
#define ENT_VALP(r, i, es, vo) ((r)->entries + (size_t)(i) * (es) + (vo))

/* FindIndex (:230-238) */
static int64_t svm_find(const orc_row *r, int32_t key, size_t es) {
  for (int64_t i = 0; i < r->num_entries; ++i) if (ENT_KEY(r, i, es) == key) return i;
  return -1;
}

/* LinearSearchAndMove(vector_idx, forward=false) (:264-285): bubble backward while
 * the new value is strictly greater than its predecessor. */
static void svm_move_backward(orc_row *r, int64_t idx, int dt) {
  size_t es = entry_size(dt), vo = entry_val_off(dt);
  val_t val = v_load(ENT_VALP(r, idx, es, vo), dt);
  int64_t new_idx = idx;
  for (int64_t i = idx - 1; i >= 0; --i) {
    if (v_lt(v_load(ENT_VALP(r, i, es, vo), dt), val, dt)) new_idx = i;
    else break;
  }
  if (new_idx < idx) {
    uint8_t tmp[16];
    memcpy(tmp, r->entries + (size_t)idx * es, es);
    memmove(r->entries + (size_t)(new_idx + 1) * es, r->entries + (size_t)new_idx * es,
            (size_t)(idx - new_idx) * es);
    memcpy(r->entries + (size_t)new_idx * es, tmp, es);
  }
}

/* Inc(key, delta) (:175-197) over the private Inc (:305-337).  Capacity growth
 * (+kBlockSize=64) and compaction (:288-301) only change allocation, never the
 * observable entry order, so they are restated as plain reallocation. */
static void svm_inc(orc_row *r, int32_t key, val_t delta, int dt) {
  size_t es = entry_size(dt), vo = entry_val_off(dt);
  if (v_is_zero(delta, dt)) return;                      /* :306 */
  int64_t idx = svm_find(r, key, es);
  if (idx == -1) {                                       /* :309-322 insert */
    if (r->num_entries == r->capacity) {
      r->capacity += 64;
      r->entries = (uint8_t *)realloc(r->entries, (size_t)r->capacity * es);
    }
    idx = r->num_entries++;
    memset(r->entries + (size_t)idx * es, 0, es);
    ENT_KEY(r, idx, es) = key;
    v_store(ENT_VALP(r, idx, es, vo), delta, dt);
    svm_move_backward(r, idx, dt);
    return;
  }
  /* :325-334 found: add in place (NO re-sort), remove on reaching zero */
  val_t nv = v_add(v_load(ENT_VALP(r, idx, es, vo), dt), delta, dt);
  v_store(ENT_VALP(r, idx, es, vo), nv, dt);
  if (v_is_zero(nv, dt)) {
    memmove(r->entries + (size_t)idx * es, r->entries + (size_t)(idx + 1) * es,
            (size_t)(r->num_entries - idx - 1) * es);      /* RemoveOneEntryAndCompact :288-291 */
    r->num_entries--;
  }
}

/* ---- MapStore<V>::Inc (map_store.hpp:60-65) -------------------------------- */
static void map_inc(orc_row *r, int32_t col, val_t delta, int dt) {
  int64_t slot = imap_find(&r->map, col);
  if (slot < 0) slot = imap_insert(&r->map, col, 0);   /* data_[col_id] default-inserts 0 */
  val_t cur; cur.raw = (uint64_t)r->map.vals[slot];    /* value bits live in the map slot */
  val_t nv = v_add(cur, delta, dt);
  if (dt_size(dt) == 4) nv.raw &= 0xffffffffULL;
  r->map.vals[slot] = (int64_t)nv.raw;
  if (v_is_zero(nv, dt)) imap_erase_at(&r->map, slot);
}

/* NumericStoreRow::ApplyBatchIncUnsafe (numeric_store_row.hpp:166-175) for one sparse
 * record, dispatched on the store type. */
static double v_to_double(val_t v, int dt) {
  switch (dt) {
    case DT_F32: return (double)v.f;
    case DT_F64: return v.d;
    case DT_I32: return (double)v.i;
    default: return (double)v.l;
  }
}

static void apply_sparse_record(orc_table *t, orc_row *r, const int32_t *cols,
                                const uint8_t *vals, int32_t n) {
  size_t vs = dt_size(t->dt);
  if (t->importance) {
    /* NSSumImpCalc::ApplyBatchIncGetImportance (ns_sum_imp_calc.hpp:57-77): the sum of
     * |u_i| in record order, accumulated into importance_ (server_row.hpp:43-49,124-126) */
    double acc = 0;
    for (int32_t i = 0; i < n; ++i) acc += fabs(v_to_double(v_load(vals + (size_t)i * vs, t->dt), t->dt));
    r->importance += acc;
  }
  for (int32_t i = 0; i < n; ++i) {
    val_t d = v_load(vals + (size_t)i * vs, t->dt);
    if (t->kind == KIND_DENSE) {
      /* VectorStore::Inc (vector_store.hpp:100-102) */
      uint8_t *p = r->dense + (size_t)cols[i] * vs;
      v_store(p, v_add(v_load(p, t->dt), d, t->dt), t->dt);
    } else if (t->kind == KIND_SORTED_MAP) {
      svm_inc(r, cols[i], d, t->dt);
    } else {
      map_inc(r, cols[i], d, t->dt);
    }
  }
}

/* NumericStoreRow::ApplyDenseBatchIncUnsafe (numeric_store_row.hpp:177-185):
 * val[i] += upd[i] for i < num_updates (= dense_row_oplog_capacity). For non-dense
 * stores the reference's GetPtr does not exist; a dense record is applied element
 * by element through Inc (the per-column meaning of a dense oplog). */
#define ORC_DENSE_LOOP(T, ADD)                                   \
  do {                                                           \
    T *val = (T *)r->dense;                                      \
    for (int64_t i = 0; i < n; ++i) {                            \
      T u;                                                       \
      memcpy(&u, upd + (size_t)i * sizeof(T), sizeof(T));        \
      val[i] = ADD(val[i], u);                                   \
    }                                                            \
  } while (0)
#define ORC_FADD(a, b) ((a) + (b))
#define ORC_I32ADD(a, b) ((int32_t)((uint32_t)(a) + (uint32_t)(b)))
#define ORC_I64ADD(a, b) ((int64_t)((uint64_t)(a) + (uint64_t)(b)))

/* NSSumImpCalc::ApplyDenseBatchIncGetImportance (ns_sum_imp_calc.hpp:79-98): per element,
 * importance = (double(val) == 0) ? double(u) : double(u) / double(val) with val the value
 * before the add, summed as |importance| in element order; then val += u. */
#define ORC_DENSE_IMP_LOOP(T, ADD)                               \
  do {                                                           \
    T *val = (T *)r->dense;                                      \
    double acc = 0;                                              \
    for (int64_t i = 0; i < n; ++i) {                            \
      T u;                                                       \
      memcpy(&u, upd + (size_t)i * sizeof(T), sizeof(T));        \
      double dv = (double)val[i], du = (double)u;                \
      acc += fabs(dv == 0 ? du : du / dv);                       \
      val[i] = ADD(val[i], u);                                   \
    }                                                            \
    r->importance += acc;                                        \
  } while (0)

static void apply_dense_record(orc_table *t, orc_row *r, const uint8_t *upd, int64_t n) {
  if (t->kind == KIND_DENSE && t->importance) {
    switch (t->dt) {
      case DT_F32: ORC_DENSE_IMP_LOOP(float, ORC_FADD); break;
      case DT_F64: ORC_DENSE_IMP_LOOP(double, ORC_FADD); break;
      case DT_I32: ORC_DENSE_IMP_LOOP(int32_t, ORC_I32ADD); break;
      default: ORC_DENSE_IMP_LOOP(int64_t, ORC_I64ADD); break;
    }
  } else if (t->kind == KIND_DENSE) {
    /* the typed `val[i] += upd[i]` loop of numeric_store_row.hpp:181-184 */
    switch (t->dt) {
      case DT_F32: ORC_DENSE_LOOP(float, ORC_FADD); break;
      case DT_F64: ORC_DENSE_LOOP(double, ORC_FADD); break;
      case DT_I32: ORC_DENSE_LOOP(int32_t, ORC_I32ADD); break;
      default: ORC_DENSE_LOOP(int64_t, ORC_I64ADD); break;
    }
  } else {
    for (int64_t i = 0; i < n; ++i) {
      val_t d = v_load(upd + (size_t)i * dt_size(t->dt), t->dt);
      if (t->kind == KIND_SORTED_MAP) svm_inc(r, (int32_t)i, d, t->dt);
      else map_inc(r, (int32_t)i, d, t->dt);
    }
  }
}

/* ---- AdaRevision server-table logic (adarevision_server_table_logic.cpp) ---------- */
/* Init (:19-36): attached to a table as TableInfo.server_table_logic selects it
 * (server_table.cpp:83-93).  AdaRevision treats updates as a dense float row of
 * row_capacity values (:65-68). */
int orc_table_set_adarevision(orc_server *s, int32_t table_id, float init_step, int gaussian,
                              uint64_t upper_bound, int32_t push_clients) {
  orc_table *t = find_table(s, table_id);
  if (!t || push_clients <= 0) return ORC_ERR_INVALID_ARG;
  if (t->kind != KIND_DENSE || t->dt != DT_F32 || !t->dense_serialized || t->f16_records ||
      t->oplog_capacity != t->row_capacity || t->nrows)
    return ORC_ERR_UNSUPPORTED;
  t->ada = 1;
  t->ada_step = init_step;
  t->ada_gauss = gaussian ? 1 : 0;
  t->ada_upper = upper_bound;
  t->ada_clients = (size_t)push_clients;
  rng_seed(&t->ada_rng, 12345);   /* gen_ = new std::mt19937(12345) (:32) */
  return ORC_OK;
}

static void apply_dense_record(orc_table *t, orc_row *r, const uint8_t *upd, int64_t n);

/* ServerRowCreated (:38-50) for a row CreateRow makes on first touch (server.cpp:163-166):
 * with random_init "guassian", row_capacity N(0, 0.1) draws go through RowBatchInc_. */
static void ada_row_created(orc_table *t, orc_row *r) {
  if (!t->ada_gauss) return;
  int64_t n = t->row_capacity;
  float *d = (float *)malloc((size_t)n * sizeof(float));
  for (int64_t i = 0; i < n; ++i) d[i] = rng_normal(&t->ada_rng, 0.0f, 0.1f);
  apply_dense_record(t, r, (const uint8_t *)d, n);
  r->dirty = 1;
  r->version++;
  free(d);
}

static orc_snap *ada_find(orc_table *t, int32_t row, uint64_t version) {
  for (int64_t k = 0; k < t->nsnaps; ++k)
    if (t->snaps[k].row == row && t->snaps[k].version == version) return &t->snaps[k];
  return NULL;
}

/* ApplyRowOpLog (:52-175): per element, in float, the AdaRevision step against the
 * accumulated gradient as of the record's row version (0: none), then RowBatchInc_ of the
 * deltas (:173-174).  A version without a snapshot is the reference's CHECK (:116). */
static int ada_apply(orc_table *t, orc_row *r, int32_t row_id, const uint8_t *upd, uint64_t rv, int eov) {
  int64_t n = t->row_capacity;
  orc_snap *sn = NULL;
  if (rv != 0) {
    sn = ada_find(t, row_id, rv);
    if (!sn) return ORC_ERR_STATE;
  }
  float *d = (float *)malloc((size_t)n * sizeof(float));
  const float step = t->ada_step;
  for (int64_t i = 0; i < n; ++i) {
    float u;
    memcpy(&u, upd + (size_t)i * 4, 4);
    float g_bck = r->ada_acc[i] - (sn ? sn->acc[i] : 0.0f);
    float eta_old = step / sqrtf(r->ada_zmax[i]);
    r->ada_z[i] += u * (u + 2 * g_bck);
    r->ada_zmax[i] = (r->ada_z[i] < r->ada_zmax[i]) ? r->ada_zmax[i] : r->ada_z[i];   /* std::max */
    float eta = step / sqrtf(r->ada_zmax[i]);
    d[i] = -(eta * u) + (eta_old - eta) * g_bck;
    r->ada_acc[i] += u;
  }
  if (sn && eov && --sn->count == 0) {   /* :165-170 */
    free(sn->acc);
    *sn = t->snaps[--t->nsnaps];
  }
  apply_dense_record(t, r, (const uint8_t *)d, n);
  free(d);
  return ORC_OK;
}

/* ServerRowSent (:177-190): old_accum_gradients_.insert({(row, get_version()),
 * (accum_gradients_, num_clients)}); an existing key is kept (std::map::insert). */
static void ada_row_sent(orc_table *t, int32_t row_id, orc_row *r, size_t num_clients) {
  uint64_t v = t->version_maintain ? r->version : 0;
  if (ada_find(t, row_id, v)) return;
  if (t->nsnaps == t->snaps_cap) {
    t->snaps_cap = t->snaps_cap ? 2 * t->snaps_cap : 64;
    t->snaps = (orc_snap *)realloc(t->snaps, (size_t)t->snaps_cap * sizeof(orc_snap));
  }
  orc_snap *sn = &t->snaps[t->nsnaps++];
  sn->row = row_id;
  sn->version = v;
  sn->count = num_clients;
  sn->acc = (float *)malloc((size_t)t->row_capacity * sizeof(float));
  memcpy(sn->acc, r->ada_acc, (size_t)t->row_capacity * sizeof(float));
}

/* Server::RowSent (server.cpp:436-441) -> ServerTable::RowSent (server_table.cpp:191-195):
 * what ServerThread::ReplyRowRequest does after serving a row (server_thread.cpp:221). */
int orc_row_sent(orc_server *s, int32_t table_id, int32_t row_id, int32_t num_clients) {
  orc_table *t = find_table(s, table_id);
  orc_row *r = t ? find_row(t, row_id) : NULL;
  if (!r || num_clients <= 0) return ORC_ERR_INVALID_ARG;
  if (t->ada) ada_row_sent(t, row_id, r, (size_t)num_clients);
  return ORC_OK;
}

/* AdaRevisionRow state of a row and the number of live old_accum_gradients_ entries. */
int orc_ada_state(orc_server *s, int32_t table_id, int32_t row_id, float *acc, float *z, float *zmax) {
  orc_table *t = find_table(s, table_id);
  orc_row *r = t ? find_row(t, row_id) : NULL;
  if (!r || !t->ada) return ORC_ERR_INVALID_ARG;
  size_t nb = (size_t)t->row_capacity * sizeof(float);
  memcpy(acc, r->ada_acc, nb);
  memcpy(z, r->ada_z, nb);
  memcpy(zmax, r->ada_zmax, nb);
  return ORC_OK;
}
int64_t orc_ada_num_snapshots(orc_server *s, int32_t table_id) {
  orc_table *t = find_table(s, table_id);
  return t ? t->nsnaps : -1;
}

static int32_t rd32(const uint8_t *p) { int32_t v; memcpy(&v, p, 4); return v; }
static uint64_t rd64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }

/* Float16Compressor::decompress, called by DenseRowOpLogFloat16::ParseDenseSerializedOpLog
 * (dense_row_oplog_float16.hpp:144-157).  float16_compressor.hpp is fetched by
 * third_party/third_party.mk:281-290 with no pinned version and is absent here, so this
 * restates IEEE-754 binary16 -> binary32, which is exact (a unique result) for every
 * finite value and infinity; NaNs keep their payload shifted into the binary32 mantissa
 * (no quieting).  Parity for the fp16 record format is "unpinned". */
static float half_to_float(uint16_t h) {
  uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu, bits;
  if (e == 0x1f) {
    bits = sign | 0x7f800000u | (m << 13);
  } else if (e != 0) {
    bits = sign | ((e + 112u) << 23) | (m << 13);
  } else if (m == 0) {
    bits = sign;
  } else {                       /* subnormal half: normalise */
    uint32_t k = 0;
    while (!(m & 0x400u)) { m <<= 1; ++k; }
    bits = sign | ((113u - k) << 23) | ((m & 0x3ffu) << 13);
  }
  float f;
  memcpy(&f, &bits, 4);
  return f;
}
float orc_half_to_float(uint16_t h) { return half_to_float(h); }

/* Bytes of one dense record body after its row id: DenseRowOpLog V[cap]
 * (dense_row_oplog.hpp:138-144), VersionDenseRowOpLog V[cap] + uint64 version + bool
 * end_of_version (version_dense_row_oplog.hpp:173-180), DenseRowOpLogFloat16
 * uint16[cap] (dense_row_oplog_float16.hpp:144-157). */
static size_t dense_body_bytes(const orc_table *t) {
  if (t->f16_records) return (size_t)t->oplog_capacity * 2;
  return (size_t)t->oplog_capacity * dt_size(t->dt) + (t->version_maintain ? 9 : 0);
}

/* Walk the stream exactly as SerializedOpLogReader::Restart/Next/StartNewTable
 * (serialized_oplog_reader.hpp:30-133) with AbstractRowOpLog::ParseSparseSerializedOpLog
 * (abstract_row_oplog.hpp:64-78) / DenseRowOpLog::ParseDenseSerializedOpLog
 * (dense_row_oplog.hpp:138-144).  mode 0 only validates; 1 applies each record through
 * ServerTable::ApplyRowOpLog (server_table.cpp:164-189), creating missing rows first
 * (server.cpp:163-166); 2 is the reference's own loop shape, one pass that checks each
 * record as it reaches it and applies it (server.cpp:154-178) — a malformed stream is
 * then found part-way, after the records before it were applied (the reference CHECK-
 * aborts there), so mode 2 is for timing only (bench.py's cpu_baseline legs). */
static int walk_stream(orc_server *s, const uint8_t *b, size_t size, int mode) {
  const int apply = mode != 0;
  if (size < 4) return ORC_ERR_MALFORMED;
  int32_t num_tables = rd32(b);
  size_t off = 4;
  if (num_tables < 0) return ORC_ERR_MALFORMED;
  int32_t seen[64]; int nseen = 0;
  for (int32_t tt = 0; tt < num_tables; ++tt) {
    if (off + 16 > size) return ORC_ERR_MALFORMED;
    int32_t table_id = rd32(b + off);
    uint64_t update_size = rd64(b + off + 4);
    int32_t num_rows = rd32(b + off + 12);
    off += 16;
    orc_table *t = find_table(s, table_id);
    if (!t) return ORC_ERR_UNKNOWN_TABLE;
    if (update_size != dt_size(t->dt) || num_rows < 0) return ORC_ERR_MALFORMED;
    for (int i = 0; i < nseen; ++i) if (seen[i] == table_id) return ORC_ERR_UNSUPPORTED;
    if (nseen < 64) seen[nseen++] = table_id;
    size_t vs = dt_size(t->dt);
    for (int32_t k = 0; k < num_rows; ++k) {
      if (off + 4 > size) return ORC_ERR_MALFORMED;
      int32_t row_id = rd32(b + off);
      off += 4;
      if (t->dense_serialized) {
        size_t rs = dense_body_bytes(t);
        if (off + rs > size) return ORC_ERR_MALFORMED;
        if (apply) {
          orc_row *r = find_row(t, row_id);
          if (!r) {
            r = create_row(t, row_id);
            if (t->ada) ada_row_created(t, r);
          }
          if (t->ada) {
            uint64_t rv = 0;
            int eov = 0;
            if (t->version_maintain) {   /* ExtractOpLogVersion (server_table.cpp:527-535) */
              size_t vo = (size_t)t->oplog_capacity * dt_size(t->dt);
              rv = rd64(b + off + vo);
              eov = b[off + vo + 8] != 0;
            }
            int st = ada_apply(t, r, row_id, b + off, rv, eov);
            if (st) return st;
          } else if (t->f16_records) {
            /* ParseDenseSerializedOpLog decompresses into the sample oplog's f32 buffer,
             * which is then applied as a dense float record */
            float *tmp = (float *)malloc((size_t)t->oplog_capacity * sizeof(float));
            for (int64_t i = 0; i < t->oplog_capacity; ++i) {
              uint16_t h; memcpy(&h, b + off + (size_t)i * 2, 2);
              tmp[i] = half_to_float(h);
            }
            apply_dense_record(t, r, (const uint8_t *)tmp, t->oplog_capacity);
            free(tmp);
          } else {
            apply_dense_record(t, r, b + off, t->oplog_capacity);
          }
          r->dirty = 1;
          r->version++;   /* VersionServerRow::ApplyDenseBatchInc* (version_server_row.hpp:44-53) */
        }
        off += rs;
      } else {
        if (off + 4 > size) return ORC_ERR_MALFORMED;
        int32_t n = rd32(b + off);
        if (n < 0) return ORC_ERR_MALFORMED;
        size_t rs = 4 + (size_t)n * (4 + vs);
        if (off + rs > size) return ORC_ERR_MALFORMED;
        const int32_t *cols = (const int32_t *)(b + off + 4);
        if (mode != 1 && t->kind == KIND_DENSE) {
          for (int32_t i = 0; i < n; ++i) {
            int32_t c; memcpy(&c, b + off + 4 + (size_t)i * 4, 4);
            if (c < 0 || c >= t->row_capacity) return ORC_ERR_CAPACITY;
          }
        }
        if (apply) {
          orc_row *r = find_row(t, row_id);
          if (!r) r = create_row(t, row_id);
          /* cols may be unaligned in a host buffer: copy out (on the stack when short) */
          int32_t stack_cols[256];
          int32_t *cc = n <= 256 ? stack_cols : (int32_t *)malloc((size_t)n * 4);
          memcpy(cc, cols, (size_t)n * 4);
          apply_sparse_record(t, r, cc, b + off + 4 + (size_t)n * 4, n);
          if (cc != stack_cols) free(cc);
          r->dirty = 1;
          r->version++;   /* VersionServerRow::ApplyBatchInc* (version_server_row.hpp:28-42) */
        }
        off += rs;
      }
    }
  }
  return ORC_OK;
}

/* Server::ApplyOpLogUpdateVersion (server.cpp:120-179). */
int orc_apply_stream(orc_server *s, const void *oplog, size_t size, int32_t bg, uint32_t version) {
  int bi = -1;
  for (int i = 0; i < s->nbg; ++i) if (s->bg_ids[i] == bg) bi = i;
  if (bi < 0) return ORC_ERR_SENDER;
  if (s->bg_versions[bi] + 1 != (int64_t)version) return ORC_ERR_VERSION;   /* :124-126 */
  if (size == 0) { s->bg_versions[bi] = version; return ORC_OK; }          /* :128 */
  const uint8_t *b = (const uint8_t *)oplog;
  if (size >= 4 && rd32(b) == 0) { s->bg_versions[bi] = version; return ORC_OK; } /* Restart() false */
  int st = walk_stream(s, b, size, 0);
  if (st != ORC_OK) return st;
  s->bg_versions[bi] = version;
  return walk_stream(s, b, size, 1);
}

/* The reference's loop shape for the timed CPU baseline: one walk that validates each
 * record as it reaches it and applies it (server.cpp:154-178), instead of
 * orc_apply_stream's validate-then-apply pair of walks (which the checker needs so that a
 * failed message applies nothing).  Results are identical on well-formed streams. */
int orc_apply_stream_once(orc_server *s, const void *oplog, size_t size, int32_t bg, uint32_t version) {
  int bi = -1;
  for (int i = 0; i < s->nbg; ++i) if (s->bg_ids[i] == bg) bi = i;
  if (bi < 0) return ORC_ERR_SENDER;
  if (s->bg_versions[bi] + 1 != (int64_t)version) return ORC_ERR_VERSION;   /* :124-126 */
  s->bg_versions[bi] = version;
  if (size == 0) return ORC_OK;                                              /* :128 */
  const uint8_t *b = (const uint8_t *)oplog;
  if (size >= 4 && rd32(b) == 0) return ORC_OK;
  return walk_stream(s, b, size, 2);
}

int64_t orc_sender_version(orc_server *s, int32_t bg) {
  for (int i = 0; i < s->nbg; ++i) if (s->bg_ids[i] == bg) return s->bg_versions[i];
  return -2;
}

/* ---- row access ------------------------------------------------------------ */
int orc_row_exists(orc_server *s, int32_t table_id, int32_t row_id) {
  orc_table *t = find_table(s, table_id);
  return (t && find_row(t, row_id)) ? 1 : 0;
}
int orc_row_dirty(orc_server *s, int32_t table_id, int32_t row_id) {
  orc_table *t = find_table(s, table_id);
  orc_row *r = t ? find_row(t, row_id) : NULL;
  return r ? r->dirty : 0;
}
int64_t orc_num_rows(orc_server *s, int32_t table_id) {
  orc_table *t = find_table(s, table_id);
  return t ? t->nrows : -1;
}

/* ServerTable ctor's importance selection (server_table.cpp:26-47): under SSPAggr with a
 * RelativeMagnitude / FIFO_N_ReMag update-sort policy the table applies through
 * ApplyRow{Dense,}BatchIncAccumImportance and sorts push candidates by importance. */
int orc_table_set_importance(orc_server *s, int32_t table_id, int on) {
  orc_table *t = find_table(s, table_id);
  if (!t) return ORC_ERR_INVALID_ARG;
  t->importance = on ? 1 : 0;
  return ORC_OK;
}

/* TableInfo.version_maintain (configs.hpp:207): records are VersionDenseRowOpLog
 * (server_table.cpp:56-61) and rows VersionServerRow (server_table.cpp:149-153).  Only
 * dense-serialized DenseRowOpLog tables: the reference writes a sparse version record's
 * trailer at the wrong offset (version_dense_row_oplog.hpp:133-159) and parses sparse
 * records without it (abstract_row_oplog.hpp:64-78), and the version sample oplog exists
 * only for row_oplog_type kDenseRowOpLog (server_table.cpp:56-67). */
int orc_table_set_version_maintain(orc_server *s, int32_t table_id, int on) {
  orc_table *t = find_table(s, table_id);
  if (!t) return ORC_ERR_INVALID_ARG;
  if (on && (!t->dense_serialized || t->f16_records)) return ORC_ERR_UNSUPPORTED;
  t->version_maintain = on ? 1 : 0;
  return ORC_OK;
}

/* row_oplog_type kDenseRowOpLogFloat16 (server_table.cpp:68-72): dense records are
 * uint16[cap]; float tables only (CHECK(update_size == sizeof(float)),
 * dense_row_oplog_float16.hpp:28). */
int orc_table_set_f16_records(orc_server *s, int32_t table_id, int on) {
  orc_table *t = find_table(s, table_id);
  if (!t) return ORC_ERR_INVALID_ARG;
  if (on && (t->dt != DT_F32 || t->version_maintain)) return ORC_ERR_UNSUPPORTED;
  t->f16_records = on ? 1 : 0;
  return ORC_OK;
}

/* DenseRowFloat16<float> rows (dense_row_float16.hpp:13, registered by matrixfact_split16.cpp:47,560):
 * stored as float, Inc adds in float (vector_store_float16.hpp:131-134), serialized as
 * binary16 through Float16Compressor::compress (:91-99). */
int orc_table_set_f16_rows(orc_server *s, int32_t table_id, int on) {
  orc_table *t = find_table(s, table_id);
  if (!t) return ORC_ERR_INVALID_ARG;
  if (on && (t->kind != KIND_DENSE || t->dt != DT_F32)) return ORC_ERR_UNSUPPORTED;
  t->f16_rows = on ? 1 : 0;
  return ORC_OK;
}

/* Float16Compressor::compress, the float -> binary16 direction VectorStoreFloat16::Serialize
 * calls (vector_store_float16.hpp:94-96).  float16_compressor.hpp is fetched unpinned by
 * third_party/third_party.mk:281-290 and absent here; this restates the published
 * algorithm of that class (branch-free, bit-level): the magnitude's mantissa is truncated
 * (round toward zero), values below the smallest normal half become subnormals through a
 * float multiply by 2^37 converted to int (truncation), values above 65504 become infinity,
 * NaNs keep the top 10 payload bits (the smallest half NaN when those are zero).  Parity
 * unpinned: no reference test or fixture holds a compressed value. */
uint16_t orc_float_to_half(float value) {
  union { float f; int32_t si; uint32_t ui; } v, sc;
  const int32_t infN = 0x7F800000, maxN = 0x477FE000, minN = 0x38800000;
  const int32_t infC = infN >> 13, nanN = (infC + 1) << 13, maxC = maxN >> 13, minC = minN >> 13;
  const int32_t subC = 0x003FF, maxD = infC - maxC - 1, minD = minC - subC - 1;
  v.f = value;
  uint32_t sign = v.ui & 0x80000000u;
  v.ui ^= sign;
  sign >>= 16;
  sc.si = 0x52000000;                                    /* 2^37 */
  const int32_t sub = minN > v.si ? (int32_t)(sc.f * v.f) : 0;
  v.si ^= (sub ^ v.si) & -(int32_t)(minN > v.si);
  v.si ^= (infN ^ v.si) & -(int32_t)((infN > v.si) & (v.si > maxN));
  v.si ^= (nanN ^ v.si) & -(int32_t)((nanN > v.si) & (v.si > infN));
  v.ui >>= 13;
  v.si ^= ((v.si - maxD) ^ v.si) & -(int32_t)(v.si > maxC);
  v.si ^= ((v.si - minD) ^ v.si) & -(int32_t)(v.si > subC);
  return (uint16_t)(v.ui | sign);
}

/* orc_float_to_half over an array (raw bits in and out: no float conversion on the way) */
void orc_floats_to_halves(const float *in, uint16_t *out, size_t n) {
  for (size_t i = 0; i < n; ++i) out[i] = orc_float_to_half(in[i]);
}

/* VersionServerRow::get_version (version_server_row.hpp:66); 0 for a plain ServerRow
 * (abstract_server_row.hpp:71) and for absent rows. */
int orc_row_version(orc_server *s, int32_t table_id, int32_t row_id, uint64_t *out) {
  orc_table *t = find_table(s, table_id);
  if (!t) return ORC_ERR_INVALID_ARG;
  orc_row *r = find_row(t, row_id);
  *out = (r && t->version_maintain) ? r->version : 0;
  return ORC_OK;
}

/* ServerRow::get_importance (server_row.hpp:120-122); absent rows read 0. */
int orc_row_importance(orc_server *s, int32_t table_id, int32_t row_id, double *out) {
  orc_table *t = find_table(s, table_id);
  if (!t) return ORC_ERR_INVALID_ARG;
  orc_row *r = find_row(t, row_id);
  *out = r ? r->importance : 0.0;
  return ORC_OK;
}

/* AbstractRow::ResetRowData (numeric_store_row.hpp:142-145 -> VectorStore::ResetData
 * vector_store.hpp:89-92) for a dense row, creating it if absent. */
int orc_load_dense_row(orc_server *s, int32_t table_id, int32_t row_id, const void *src) {
  orc_table *t = find_table(s, table_id);
  if (!t || t->kind != KIND_DENSE) return ORC_ERR_INVALID_ARG;
  orc_row *r = find_row(t, row_id);
  if (!r) r = create_row(t, row_id);
  memcpy(r->dense, src, (size_t)t->row_capacity * dt_size(t->dt));
  return ORC_OK;
}

/* Bulk variant: rows first_row, first_row+stride, ... */
int orc_load_dense_rows(orc_server *s, int32_t table_id, int64_t first_row, int64_t stride,
                        int64_t n, const void *src) {
  orc_table *t = find_table(s, table_id);
  if (!t || t->kind != KIND_DENSE) return ORC_ERR_INVALID_ARG;
  size_t rb = (size_t)t->row_capacity * dt_size(t->dt);
  for (int64_t i = 0; i < n; ++i) {
    int st = orc_load_dense_row(s, table_id, (int32_t)(first_row + i * stride),
                                (const uint8_t *)src + (size_t)i * rb);
    if (st) return st;
  }
  return ORC_OK;
}

/* VectorStore::CopyToMem (vector_store.hpp:115-118); absent rows read as zero. */
int orc_read_dense_rows(orc_server *s, int32_t table_id, int64_t first_row, int64_t stride,
                        int64_t n, void *dst) {
  orc_table *t = find_table(s, table_id);
  if (!t || t->kind != KIND_DENSE) return ORC_ERR_INVALID_ARG;
  size_t rb = (size_t)t->row_capacity * dt_size(t->dt);
  for (int64_t i = 0; i < n; ++i) {
    orc_row *r = find_row(t, (int32_t)(first_row + i * stride));
    uint8_t *d = (uint8_t *)dst + (size_t)i * rb;
    if (r) memcpy(d, r->dense, rb); else memset(d, 0, rb);
  }
  return ORC_OK;
}

/* ServerRow::Serialize -> store Serialize: VectorStore (vector_store.hpp:75-80),
 * SortedVectorMapStore (:148-152, entries in store order), MapStore (map_store.hpp:89-100;
 * the reference emits unordered_map order, this oracle emits ascending column order —
 * parity for MapStore rows is defined on the {col -> value} map).
 * Version tables append VersionServerRow's uint64 version_ (version_server_row.hpp:55-64).
 * Returns the byte count, or -1 if the row is absent, or -2 if cap is too small. */
static int64_t serialize_row_body(orc_table *t, orc_row *r, void *out, size_t cap);
int64_t orc_serialize_row(orc_server *s, int32_t table_id, int32_t row_id, void *out, size_t cap) {
  orc_table *t = find_table(s, table_id);
  orc_row *r = t ? find_row(t, row_id) : NULL;
  if (!r) return -1;
  int64_t nb = serialize_row_body(t, r, out, cap);
  if (nb < 0 || !t->version_maintain) return nb;
  if ((size_t)nb + 8 > cap) return -2;
  memcpy((uint8_t *)out + nb, &r->version, 8);
  return nb + 8;
}

static int64_t serialize_row_body(orc_table *t, orc_row *r, void *out, size_t cap) {
  size_t vs = dt_size(t->dt);
  if (t->kind == KIND_DENSE && t->f16_rows) {   /* VectorStoreFloat16::Serialize */
    size_t nb = (size_t)t->row_capacity * 2;
    if (nb > cap) return -2;
    for (int64_t i = 0; i < t->row_capacity; ++i) {
      float x;
      memcpy(&x, r->dense + (size_t)i * 4, 4);
      const uint16_t h = orc_float_to_half(x);
      memcpy((uint8_t *)out + (size_t)i * 2, &h, 2);
    }
    return (int64_t)nb;
  }
  if (t->kind == KIND_DENSE) {
    size_t nb = (size_t)t->row_capacity * vs;
    if (nb > cap) return -2;
    memcpy(out, r->dense, nb);
    return (int64_t)nb;
  }
  if (t->kind == KIND_SORTED_MAP) {
    size_t es = entry_size(t->dt);
    size_t nb = (size_t)r->num_entries * es;
    if (nb > cap) return -2;
    memcpy(out, r->entries, nb);
    return (int64_t)nb;
  }
  size_t rec = 4 + vs;
  size_t nb = (size_t)r->map.count * rec;
  if (nb > cap) return -2;
  /* collect and sort by column */
  int64_t n = 0;
  int32_t *cols = (int32_t *)malloc((size_t)(r->map.count + 1) * 4);
  uint64_t *vals = (uint64_t *)malloc((size_t)(r->map.count + 1) * 8);
  for (int64_t i = 0; i < r->map.cap; ++i)
    if (r->map.used[i] == 1) { cols[n] = r->map.keys[i]; vals[n] = (uint64_t)r->map.vals[i]; n++; }
  for (int64_t i = 1; i < n; ++i) {          /* insertion sort: rows are small */
    int32_t c = cols[i]; uint64_t v = vals[i]; int64_t j = i - 1;
    while (j >= 0 && cols[j] > c) { cols[j + 1] = cols[j]; vals[j + 1] = vals[j]; --j; }
    cols[j + 1] = c; vals[j + 1] = v;
  }
  uint8_t *o = (uint8_t *)out;
  for (int64_t i = 0; i < n; ++i) {
    memcpy(o, &cols[i], 4);
    memcpy(o + 4, &vals[i], vs);
    o += rec;
  }
  free(cols); free(vals);
  return (int64_t)nb;
}

/* Value lookup for any row type: Get(col) (vector_store.hpp:94-98,
 * sorted_vector_map_store.hpp:160-165, map_store.hpp:51-58). Writes raw bytes. */
int orc_get(orc_server *s, int32_t table_id, int32_t row_id, int32_t col, void *out) {
  orc_table *t = find_table(s, table_id);
  if (!t) return ORC_ERR_INVALID_ARG;
  size_t vs = dt_size(t->dt);
  memset(out, 0, vs);
  orc_row *r = find_row(t, row_id);
  if (!r) return ORC_OK;
  if (t->kind == KIND_DENSE) {
    if (col >= 0 && col < t->row_capacity) memcpy(out, r->dense + (size_t)col * vs, vs);
  } else if (t->kind == KIND_SORTED_MAP) {
    size_t es = entry_size(t->dt);
    int64_t i = svm_find(r, col, es);
    if (i >= 0) memcpy(out, ENT_VALP(r, i, es, entry_val_off(t->dt)), vs);
  } else {
    int64_t slot = imap_find(&r->map, col);
    if (slot >= 0) { uint64_t v = (uint64_t)r->map.vals[slot]; memcpy(out, &v, vs); }
  }
  return ORC_OK;
}

/* Direct store-level entry point used by the known-answer tests: apply one
 * Inc(col, delta) to a row (creating it), i.e. AbstractRow::ApplyIncUnsafe
 * (numeric_store_row.hpp:160-164). */
int orc_row_inc(orc_server *s, int32_t table_id, int32_t row_id, int32_t col, const void *delta) {
  orc_table *t = find_table(s, table_id);
  if (!t) return ORC_ERR_INVALID_ARG;
  orc_row *r = find_row(t, row_id);
  if (!r) r = create_row(t, row_id);
  apply_sparse_record(t, r, &col, (const uint8_t *)delta, 1);
  return ORC_OK;
}

/* ---- pack (client side) ------------------------------------------------------ */
/* Size of one row record for a DenseRowOpLog holding `vals` (capacity values):
 * SerializedOpLogBuffer::AppendRowOpLog (row_oplog_serializer.hpp:41-56) with
 * GetDenseSerializedSize (dense_row_oplog.hpp:107-109) or, after
 * ClearZerosAndGetNoneZeroSize (:91-101), GetSparseSerializedSize (:103-106). */
static size_t count_nonzero(const uint8_t *vals, int64_t cap, int dt) {
  size_t nz = 0, vs = dt_size(dt);
  for (int64_t c = 0; c < cap; ++c) if (!v_is_zero(v_load(vals + (size_t)c * vs, dt), dt)) nz++;
  return nz;
}

/* Build one Appendix-A stream (the payload of one ClientSendOpLogMsg) from per-table
 * dense oplog matrices, as CreateOpLogMsgs + OpLogSerializer + RowOpLogSerializer do
 * (abstract_bg_worker.cpp:590-649, oplog_serializer.hpp:12-37,
 * row_oplog_serializer.hpp:139-166):
 *   int32 num_tables; per table (ascending table_id, std::map order):
 *   int32 table_id; size_t update_size; int32 num_rows; records...
 * Dense records: SerializeDense (dense_row_oplog.hpp:133-136) = V[capacity];
 * sparse: SerializeSparse (:112-131) = int32 n; int32 cols[n] ascending non-zero; V vals[n].
 * Tables with no rows are omitted (FinalizeOpLogMsgStats erases them,
 * abstract_bg_worker.cpp:568-588).  Returns bytes written, or 0 if cap too small,
 * or (size_t)-1 on bad input.  Pass out=NULL to size. */
size_t orc_pack_stream(int ntables, const int32_t *table_ids, const int32_t *dtypes,
                       const int32_t *dense_serialized, const int64_t *capacities,
                       const int64_t *nrows, const int32_t *const *row_ids,
                       const void *const *oplogs, void *out, size_t cap) {
  int order[64];
  if (ntables < 0 || ntables > 64) return (size_t)-1;
  int n_nonempty = 0;
  for (int i = 0; i < ntables; ++i) if (nrows[i] > 0) order[n_nonempty++] = i;
  for (int i = 1; i < n_nonempty; ++i) {            /* ascending table id */
    int x = order[i], j = i - 1;
    while (j >= 0 && table_ids[order[j]] > table_ids[x]) { order[j + 1] = order[j]; --j; }
    order[j + 1] = x;
  }
  size_t total = 4;
  for (int k = 0; k < n_nonempty; ++k) {
    int i = order[k];
    size_t vs = dt_size(dtypes[i]);
    total += 16;
    for (int64_t r = 0; r < nrows[i]; ++r) {
      const uint8_t *v = (const uint8_t *)oplogs[i] + (size_t)r * (size_t)capacities[i] * vs;
      if (dense_serialized[i]) total += 4 + (size_t)capacities[i] * vs;
      else total += 8 + count_nonzero(v, capacities[i], dtypes[i]) * (4 + vs);
    }
  }
  if (n_nonempty == 0) total = 0;   /* empty message: avai_size 0 (abstract_bg_worker.cpp:670-682) */
  if (!out) return total;
  if (total > cap) return 0;
  if (total == 0) return 0;
  uint8_t *o = (uint8_t *)out;
  int32_t nt = n_nonempty;
  memcpy(o, &nt, 4); o += 4;
  for (int k = 0; k < n_nonempty; ++k) {
    int i = order[k];
    int dt = dtypes[i];
    uint64_t us = dt_size(dt);
    int32_t nr = (int32_t)nrows[i];
    memcpy(o, &table_ids[i], 4); memcpy(o + 4, &us, 8); memcpy(o + 12, &nr, 4); o += 16;
    for (int64_t r = 0; r < nrows[i]; ++r) {
      const uint8_t *v = (const uint8_t *)oplogs[i] + (size_t)r * (size_t)capacities[i] * us;
      memcpy(o, &row_ids[i][r], 4); o += 4;
      if (dense_serialized[i]) {
        memcpy(o, v, (size_t)capacities[i] * us); o += (size_t)capacities[i] * us;
      } else {
        int32_t nz = (int32_t)count_nonzero(v, capacities[i], dt);
        memcpy(o, &nz, 4);
        uint8_t *ci = o + 4, *vi = o + 4 + (size_t)nz * 4;
        for (int64_t c = 0; c < capacities[i]; ++c) {
          const uint8_t *p = v + (size_t)c * us;
          if (v_is_zero(v_load(p, dt), dt)) continue;
          int32_t cc = (int32_t)c;
          memcpy(ci, &cc, 4); ci += 4;
          memcpy(vi, p, us); vi += us;
        }
        o = vi;
      }
    }
  }
  return total;
}

/* GlobalContext::GetPartitionServerID (context.hpp:291-304):
 * client = (row / C) % num_clients; channel = row % C;
 * server thread id = client*1000 + 1 + channel (context.hpp:100-104,410-414). */
int32_t orc_partition_server(int32_t row_id, int32_t num_channels, int32_t num_clients,
                             int32_t channel) {
  int32_t client = (row_id / num_channels) % num_clients;
  return client * 1000 + 1 + channel;
}

/* ---- serve-back framing ------------------------------------------------------- */
/* RecordBuff::Append (record_buff.hpp:41-53): {int32 id; size_t size; bytes}.
 * Serialize a list of rows of one table into consecutive records, skipping absent
 * rows.  Returns bytes written, or -2 when cap is too small. */
int64_t orc_serialize_records(orc_server *s, int32_t table_id, const int32_t *row_ids, int32_t n,
                              void *out, size_t cap) {
  uint8_t *o = (uint8_t *)out;
  size_t used = 0;
  uint8_t *tmp = NULL; size_t tmp_cap = 0;
  for (int32_t i = 0; i < n; ++i) {
    orc_table *t = find_table(s, table_id);
    orc_row *r = t ? find_row(t, row_ids[i]) : NULL;
    if (!r) continue;
    size_t need = (size_t)t->row_capacity * 16 + (size_t)r->num_entries * 16 +
                  (size_t)(t->kind == KIND_MAP ? r->map.count : 0) * 16 + 24;
    if (need > tmp_cap) { free(tmp); tmp_cap = need; tmp = (uint8_t *)malloc(tmp_cap); }
    int64_t nb = orc_serialize_row(s, table_id, row_ids[i], tmp, tmp_cap);
    if (nb < 0) { free(tmp); return -3; }
    if (used + 12 + (size_t)nb > cap) { free(tmp); return -2; }
    uint64_t sz = (uint64_t)nb;
    memcpy(o + used, &row_ids[i], 4); memcpy(o + used + 4, &sz, 8);
    memcpy(o + used + 12, tmp, (size_t)nb);
    used += 12 + (size_t)nb;
  }
  free(tmp);
  return (int64_t)used;
}

/* ---- serve-back push body (server.cpp:189-309) --------------------------------- */
/* Server::CreateSendServerPushRowMsgs for one client that subscribes to every row:
 * per table (in the given order) int32 table_id, then ServerTable::AppendTableToBuffs
 * (server_table.cpp:197-261) = every dirty row as a RecordBuff record
 * {int32 row_id; size_t size; ServerRow::Serialize bytes}, resetting dirty_ (:229);
 * tables are separated by int32 -1 and the body ends with int32 -2
 * (context.hpp:123-129).  The reference walks storage_ (a boost::unordered_map) in
 * hash order; this restatement emits rows in ascending row id, the order the device
 * path uses.  Returns bytes written, -2 if cap is too small. */
static int cmp_i32(const void *a, const void *b) {
  int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
  return (x > y) - (x < y);
}

int64_t orc_serialize_dirty(orc_server *s, const int32_t *table_ids, int ntables, void *out, size_t cap,
                            int clear) {
  uint8_t *o = (uint8_t *)out;
  size_t used = 0;
  for (int ti = 0; ti < ntables; ++ti) {
    orc_table *t = find_table(s, table_ids[ti]);
    if (!t) return -3;
    if (used + 4 > cap) return -2;
    memcpy(o + used, &table_ids[ti], 4);
    used += 4;
    int32_t *ids = (int32_t *)malloc((size_t)(t->nrows + 1) * 4);
    int64_t nd = 0;
    for (int64_t i = 0; i < t->index.cap; ++i)
      if (t->index.used[i] == 1 && t->rows[t->index.vals[i]]->dirty) ids[nd++] = t->index.keys[i];
    qsort(ids, (size_t)nd, 4, cmp_i32);
    int64_t w = orc_serialize_records(s, table_ids[ti], ids, (int32_t)nd, o + used, cap - used);
    if (w < 0) { free(ids); return w; }
    used += (size_t)w;
    if (clear)   /* ResetDirty + ResetImportance_ (server_table.cpp:234-235), ServerRowSent (:252-255) */
      for (int64_t k = 0; k < nd; ++k) {
        orc_row *r = find_row(t, ids[k]);
        r->dirty = 0; r->importance = 0;
        if (t->ada) ada_row_sent(t, ids[k], r, t->ada_clients);
      }
    free(ids);
    if (used + 4 > cap) return -2;
    int32_t sep = ti + 1 < ntables ? -1 : -2;
    memcpy(o + used, &sep, 4);
    used += 4;
  }
  return (int64_t)used;
}

/* ---- partial push (SSPAggr) ------------------------------------------------------ */
/* Server::CreateSendServerPushRowMsgsPartial (server.cpp:311-420) for one client that
 * subscribes to every row.  Per table: candidates = dirty rows
 * (GetPartialTableToSendRegular, server_table.cpp:301-346, with select_prob = 1: the
 * reference samples with a time-seeded generator, so only the all-candidates case is
 * deterministic); importance tables order them by importance descending, ties by
 * ascending row id (SortCandidateVectorImportance :272-287); other tables by ascending
 * row id (the reference shuffles, :263-270); the first upper_bounds[ti] rows are sent
 * through AppendRowsToBuffsPartial (:381-420): ResetDirty, ResetImportance, record.
 * Body: per table int32 table_id, records, int32 -1 | -2.  Returns 0 when no table has
 * a row to send (server.cpp:348), -2 if cap is too small. */
static orc_table *g_sort_table;
static int cmp_importance(const void *a, const void *b) {
  int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
  double ix = find_row(g_sort_table, x)->importance, iy = find_row(g_sort_table, y)->importance;
  if (ix == iy) return (x > y) - (x < y);
  return ix > iy ? -1 : 1;
}

int64_t orc_serialize_partial(orc_server *s, const int32_t *table_ids, int ntables,
                              const int64_t *upper_bounds, void *out, size_t cap, int clear) {
  int32_t *sel[64];
  int64_t nsel[64];
  int any = 0;
  if (ntables > 64) return -3;
  for (int ti = 0; ti < ntables; ++ti) {
    orc_table *t = find_table(s, table_ids[ti]);
    if (!t) { for (int k = 0; k < ti; ++k) free(sel[k]); return -3; }
    int32_t *ids = (int32_t *)malloc((size_t)(t->nrows + 1) * 4);
    int64_t nd = 0;
    for (int64_t i = 0; i < t->index.cap; ++i)
      if (t->index.used[i] == 1 && t->rows[t->index.vals[i]]->dirty) ids[nd++] = t->index.keys[i];
    qsort(ids, (size_t)nd, 4, cmp_i32);
    if (t->importance) { g_sort_table = t; qsort(ids, (size_t)nd, 4, cmp_importance); }
    if (nd > upper_bounds[ti]) nd = upper_bounds[ti];
    if (t->ada && (uint64_t)t->nsnaps >= t->ada_upper) nd = 0;   /* !AllowSend() (server_table.cpp:293-295) */
    sel[ti] = ids; nsel[ti] = nd;
    if (nd) any = 1;
  }
  int64_t ret = 0;
  if (any) {
    uint8_t *o = (uint8_t *)out;
    size_t used = 0;
    for (int ti = 0; ti < ntables && ret >= 0; ++ti) {
      if (used + 4 > cap) { ret = -2; break; }
      memcpy(o + used, &table_ids[ti], 4);
      used += 4;
      int64_t w = orc_serialize_records(s, table_ids[ti], sel[ti], (int32_t)nsel[ti], o + used, cap - used);
      if (w < 0) { ret = w; break; }
      used += (size_t)w;
      if (used + 4 > cap) { ret = -2; break; }
      int32_t sep = ti + 1 < ntables ? -1 : -2;
      memcpy(o + used, &sep, 4);
      used += 4;
    }
    if (ret == 0) {
      ret = (int64_t)used;
      if (clear)
        for (int ti = 0; ti < ntables; ++ti) {
          orc_table *t = find_table(s, table_ids[ti]);
          for (int64_t k = 0; k < nsel[ti]; ++k) {   /* AppendRowsToBuffsPartial (server_table.cpp:398-416) */
            orc_row *r = find_row(t, sel[ti][k]);
            r->dirty = 0; r->importance = 0;
            if (t->ada) ada_row_sent(t, sel[ti][k], r, t->ada_clients);
          }
        }
    }
  }
  for (int ti = 0; ti < ntables; ++ti) free(sel[ti]);
  return ret;
}

/* ---- subscriptions and the per-client push (SSPPush) ----------------------------- */
/* ServerThread::HandleRowRequest -> Server::FindCreateRow + SSPPushServerThread::RowSubscribe
 * (server_thread.cpp:185-200, server.cpp:46-60, ssp_push_server_thread.cpp:51-54,
 * CallBackSubs::Subscribe callback_subs.hpp:21-28): create the row if missing (its
 * AdaRevision ServerRowCreated included), then set the client's bit. */
int orc_subscribe(orc_server *s, int32_t table_id, int32_t row_id, int32_t client_id) {
  orc_table *t = find_table(s, table_id);
  if (!t) return ORC_ERR_UNKNOWN_TABLE;
  if (client_id < 0 || client_id >= 64) return ORC_ERR_INVALID_ARG;
  orc_row *r = find_row(t, row_id);
  if (!r) {
    r = create_row(t, row_id);
    if (t->ada) ada_row_created(t, r);
  }
  r->subs |= (uint64_t)1 << client_id;
  return ORC_OK;
}

uint64_t orc_row_subs(orc_server *s, int32_t table_id, int32_t row_id) {
  orc_table *t = find_table(s, table_id);
  orc_row *r = t ? find_row(t, row_id) : NULL;
  return r ? r->subs : 0;
}

/* Server::CreateSendServerPushRowMsgs (server.cpp:189-309) for num_clients clients, one
 * unsplit message body each: per table (in the order given) int32 table_id, then
 * ServerTable::AppendTableToBuffs (server_table.cpp:197-261): a row no client subscribes
 * to is skipped and stays dirty (:222-225); a clean row is skipped; a dirty subscribed row
 * has dirty_ and importance_ reset (:233-235), is serialized once and appended to every
 * subscribed client's buffer (CallBackSubs::AppendRowToBuffs, callback_subs.hpp:39-59),
 * then ServerRowSent(row, version, subscriber count) (:250-255); tables are separated by
 * int32 -1 and every body ends with -2.  Rows go in ascending row id (the reference
 * iterates a boost::unordered_map, whose order is unspecified).  outs[c]/caps[c]: client
 * c's buffer; used[c] receives its size.  Returns 0, -2 if a buffer is too small (nothing
 * is cleared then), -3 for an unknown table. */
int64_t orc_serialize_push(orc_server *s, const int32_t *table_ids, int ntables, int nclients, void **outs,
                           const size_t *caps, int64_t *used, int clear) {
  if (nclients <= 0 || nclients > 64) return -3;
  for (int c = 0; c < nclients; ++c) used[c] = 0;
  /* size pass: one RecordBuff record per (row, subscribed client) */
  size_t scap = 1 << 16;
  uint8_t *scratch = (uint8_t *)malloc(scap);
  for (int ti = 0; ti < ntables; ++ti) {
    orc_table *t = find_table(s, table_ids[ti]);
    if (!t) { free(scratch); return -3; }
    for (int c = 0; c < nclients; ++c) used[c] += 8;   /* table id + separator */
    for (int64_t i = 0; i < t->index.cap; ++i) {
      if (t->index.used[i] != 1) continue;
      orc_row *r = t->rows[t->index.vals[i]];
      if (!r->subs || !r->dirty) continue;
      int64_t w;
      while ((w = orc_serialize_records(s, t->table_id, &t->index.keys[i], 1, scratch, scap)) == -2) {
        scap *= 4;
        free(scratch);
        scratch = (uint8_t *)malloc(scap);
      }
      for (int c = 0; c < nclients; ++c)
        if ((r->subs >> c) & 1) used[c] += w;
    }
  }
  free(scratch);
  for (int c = 0; c < nclients; ++c)
    if ((size_t)used[c] > caps[c]) return -2;
  int64_t pos[64];
  for (int c = 0; c < nclients; ++c) pos[c] = 0;
  for (int ti = 0; ti < ntables; ++ti) {
    orc_table *t = find_table(s, table_ids[ti]);
    for (int c = 0; c < nclients; ++c) {
      memcpy((uint8_t *)outs[c] + pos[c], &table_ids[ti], 4);
      pos[c] += 4;
    }
    int32_t *ids = (int32_t *)malloc((size_t)(t->nrows + 1) * 4);
    int64_t nd = 0;
    for (int64_t i = 0; i < t->index.cap; ++i)
      if (t->index.used[i] == 1) {
        orc_row *r = t->rows[t->index.vals[i]];
        if (r->subs && r->dirty) ids[nd++] = t->index.keys[i];
      }
    qsort(ids, (size_t)nd, 4, cmp_i32);
    for (int64_t k = 0; k < nd; ++k) {
      orc_row *r = find_row(t, ids[k]);
      size_t nc = 0;
      for (int c = 0; c < nclients; ++c) {
        if (!((r->subs >> c) & 1)) continue;
        int64_t w = orc_serialize_records(s, t->table_id, &ids[k], 1, (uint8_t *)outs[c] + pos[c], caps[c] - pos[c]);
        if (w < 0) { free(ids); return w; }
        pos[c] += w;
        ++nc;
      }
      if (clear) {
        r->dirty = 0;
        r->importance = 0;
        if (t->ada) ada_row_sent(t, ids[k], r, nc);
      }
    }
    free(ids);
    for (int c = 0; c < nclients; ++c) {
      int32_t sep = ti + 1 < ntables ? -1 : -2;
      memcpy((uint8_t *)outs[c] + pos[c], &sep, 4);
      pos[c] += 4;
    }
  }
  return 0;
}
