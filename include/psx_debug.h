/*
 * psx_debug.h — kernel selectors of libpsx (not part of the reference boundary).
 * The defaults are the measured winners; the alternatives are the kernels the product
 * itself falls back to (v2 for >= 4 GiB streams, v4 for partially covered calls),
 * selectable so the parity suite covers every kernel and A/B runs stay interleaved in one
 * process (cdna_hip_programming.md §5.4 rule 24).  Variants that lost their A/B are
 * removed (their logs stay under profiles/).
 */
#ifndef PSX_DEBUG_H_
#define PSX_DEBUG_H_
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

enum {
  PSX_VARIANT_DENSE_APPLY = 1,  /* 0: auto (default), 1: force v2, 2: force v4 compact */
  PSX_VARIANT_ORD_SPLIT = 6     /* rows of sorted/map tables with 256 < max_entries <= 1024:
                                   3 (default): spill mode with rows of >= 4 records taken first;
                                   2: spill mode (rows start on the 256-entry launch unless already
                                   7/8 full; a row that outgrows it is redone, untouched, by a
                                   1,024-entry launch that follows); 1: classified by entries + Incs
                                   into a 256- and a 1,024-entry launch that run concurrently;
                                   0: one 1,024-entry launch */,
  PSX_VARIANT_DECODE = 7        /* 1: walked messages with sparse tables decode window-parallel
                                   (psx_walk.hip, where eligible; the default), 0: one workgroup
                                   per message (decode_streams) */,
  PSX_STAT_WALK_CALLS = 8       /* read: calls decoded window-parallel since load (set: reset) */,
  PSX_VARIANT_DENSE_STORE = 9,  /* dense table rows: bit0 non-temporal store, bit1 non-temporal load
                                   (0 plain/plain, 1 plain load + nt store, 3 nt/nt) */
  PSX_DEBUG_WALK_TRACE = 11,    /* 1: walked calls record per-window timestamps (psx_debug_walk_trace) */
  PSX_VARIANT_WALK_CUS = 12,    /* the walk's persistent grid: 0 half the CUs, 1 every CU (default),
                                   n >= 2 (at most 8): n blocks per CU */
  PSX_VARIANT_WALK_COUNT = 13   /* 1 (default): on walked calls the walk counts the records of split
                                   sorted/map tables into the call slot's count state (no
                                   ordered_count launch); 0: ordered_count counts them */,
  PSX_VARIANT_FOLD_FINISH = 14  /* 1 (default): a call whose last launch is an ordered apply on the
                                   context stream does finish_call's work in that launch's last
                                   block (no finish_call launch); 0: finish_call launched */,
  PSX_VARIANT_WALK_LEVELS = 15  /* the walk's composed exit-map levels: window j's exit state follows
                                   from the state 2^levels windows back (default 4; 0: window by
                                   window) */,
  PSX_VARIANT_WALK_SHAPE = 16   /* the walk's block x window (x entry candidates, = threads unless
                                   named): 0 1,024 threads x 96 KiB, 1 1,024 x 32 KiB, 2 512 x 24 KiB,
                                   3 256 x 16 KiB, 4 512 x 48 KiB (default), 5 512 x 48 KiB x 256,
                                   6 512 x 48 KiB x 128 */,
  PSX_VARIANT_CALL_EVENTS = 17  /* events enqueued per call: bit 0 an event pair per call for
                                   psx_ctx_stats (default 0: one pair per psx_sync interval), bit 1
                                   the slot-free event on every call (default 0: only while the
                                   context pipelines) */,
  PSX_VARIANT_OFFSETS_GRID = 18, /* ordered_offsets' grid cap (blocks of 256 slots; default 1,024) */
  PSX_VARIANT_DRY_GRID = 19,    /* the capacity dry run's grid cap (default 128) */
  PSX_VARIANT_WALK_RANK = 20    /* 1 (default): split sorted/map tables get each record's place in
                                   its slot's list from the count (the walk's or ordered_count's),
                                   so ordered_fill needs no atomics; 0: ordered_fill takes the
                                   places back from the counts */,
  PSX_VARIANT_ORD_LITE = 22,    /* 1: split sorted/map tables (256 < max_entries <= 1024) give rows of
                                   <= 3 records whose image stays within 64 entries to a launch of
                                   their own, four to a wave, 16 lanes each; 0 (default): one row per
                                   wave */
  PSX_DEBUG_ORD_PROBE = 23,     /* debug build only (libpsx_debug.so; -1 in libpsx.so); timing only (results wrong), bits: 1 the register apply of split
                                   tables does each row's setup (record references, headers, first
                                   record's pairs, image, key map) but applies no record; 2 it
                                   writes no row back; 4 it loads no record reference, header
                                   or pair (a row is its image, key map and write-back) */
  PSX_VARIANT_PREP_HALVES = 25, /* 1 (default): a pipelined call's split sorted/map tables do the
                                   records' half of the ordered prep (ordered_place, ordered_fill)
                                   on the prep stream beside the previous call's apply and the rows'
                                   half (ordered_classify, dry run) on the context stream; 0: all of
                                   it (ordered_offsets, ordered_fill, dry run) on the context stream */
  PSX_VARIANT_CLASSIFY_GRID = 26, /* ordered_classify's grid cap (blocks of 256 touched rows;
                                   default 256) */
  PSX_VARIANT_CLASSIFY_DRY = 27, /* 1 (default): with the prep in halves, ordered_classify runs as the
                                   capacity dry run's prologue (one launch: each block files its 256
                                   touched rows and dry-runs the ones that may overflow); 0: two launches */
  PSX_VARIANT_WALK_CUS_PIPELINED = 28, /* PSX_VARIANT_WALK_CUS for pipelined calls (default 0: half
                                   the CUs, the rest left to the previous call's apply) */
  PSX_VARIANT_STREAM_PRIORITY = 29, /* read at psx_ctx_create: 0 (default) every stream at the normal
                                   priority; 1 the prep stream at the lowest; 2 also the context's own
                                   stream at the highest */
  PSX_VARIANT_ORD_BUCKET = 30,  /* 1 (default): a split sorted/map table's record lists are buckets of 16
                                   places per row, written by the count itself (no prefix over the
                                   counts, no ordered_fill; unpipelined calls classify the slots in the
                                   dry run's prologue: one launch after the count); a row with more
                                   records in one call makes the call replay with prefix lists.
                                   0: prefix lists */
  PSX_VARIANT_PIPE_SLOTS = 31,  /* pipelined calls with bucket lists: 1 no ordered_place on the prep
                                   stream, the dry run's prologue classifies the slots themselves on
                                   the context stream; 0 (default): ordered_place's compact list */
  PSX_VARIANT_SIDE_CU_MASK = 32, /* read at psx_ctx_create: 0 (default) no CU masks; k >= 2 the prep
                                   stream on one 32-bit word of the CU mask in k (a pipelined call's
                                   walk then takes max(PSX_VARIANT_WALK_CUS_PIPELINED, 1)
                                   blocks per CU of it); -k also the context's own
                                   stream on the other words */
  PSX_VARIANT_EVENT_SCOPE = 33, /* read at psx_ctx_create: the release scope of the events that order
                                   one of the context's streams after another (pipelined call slots,
                                   concurrent apply launches): 0 system (HIP's default), 1 device
                                   (hipEventReleaseToDevice), 2 (default) no system fence
                                   (hipEventDisableSystemFence) */
  PSX_STAT_DENSE_LAST = 24,     /* read: the dense apply kernel the last call launched (2 v2, 3 v3,
                                   4 v4; 0 none since load) */
  PSX_DEBUG_WALK_SKEW = 21      /* tests only: 1 skews every exit state the walk publishes early from
                                   its composed maps by one record; the cross-check after the
                                   window's resolve must fail the call (PSX_ERR_DEVICE, nothing
                                   applied) */
};

/* Returns the previous variant, or -1 for an unknown selector. */
int32_t psx_debug_set_variant(int32_t which, int32_t variant);
int32_t psx_debug_get_variant(int32_t which);

/* The last walked call's per-window timestamps (PSX_DEBUG_WALK_TRACE on): 10 uint64 per
   (window, message) item in ticket order (item = window * B + message) — ticket taken,
   window in LDS, exit map done, predecessor's state seen, own state published, records
   expanded — in s_memrealtime ticks (100 MHz), then the composed exit's outcome (low bits:
   tried, predecessor state ok, in a table, entry in range, map found, records left; high 32
   bits: the map entry), then the speculative phase's steps: every word's count, the jump
   table, the candidates' exits.  Copies min(items, max_items) items and
   returns the call's item count, 0 when no call walked, -1 on error. */
int64_t psx_debug_walk_trace(struct psx_ctx *ctx, uint64_t *out, int64_t max_items);

/* The box's HBM read rate: GB/s of a read-only sweep (16-B non-temporal loads) over the
   device buffer [buf, buf + bytes), mean of reps launches after one warm-up, timed with HIP
   events on a stream of its own.  buf 16-B aligned, bytes >= 16 KiB (the tail past the
   last 16 KiB tile is not read).  Returns -1 on bad arguments or a HIP error. */
double psx_debug_read_sweep(const void *buf, int64_t bytes, int32_t reps);

#ifdef __cplusplus
}
#endif
#endif
