/*
 * kme.h -- C ABI of the MI355X-native matching core (drop-in for the KProcessor matching path).
 *
 * The reference runs one `MatchingEngine implements Processor<String, Order>` per stream task
 * (/root/reference/src/main/java/KProcessor.java:52, 63-445; "KP" below) that handles ONE record
 * per process() call against five RocksDB stores.  This ABI is what that processor's JNI / Panama
 * FFM binding calls instead: the Java side buffers records into an epoch and hands
 * the epoch over as structure-of-arrays; the engine returns, per input, exactly what the reference
 * would have forwarded ("IN" echo, maker/taker fills, "OUT" echo: KP:97, 124, 272-273).
 *
 * Plain C: integers, pointers and sizes only.  All functions return a kme_status (0 = OK).
 * One submitting thread per handle (the reference's process() is never concurrent either).
 */
#ifndef KME_H
#define KME_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KME_ABI_VERSION 7

/* Order.action codes (KP:65-75). */
enum kme_action {
    KME_ADD_SYMBOL = 0, KME_REMOVE_SYMBOL = 1, KME_BUY = 2, KME_SELL = 3, KME_CANCEL = 4,
    KME_BOUGHT = 5, KME_SOLD = 6, KME_REJECT = 7,
    KME_CREATE_BALANCE = 100, KME_TRANSFER = 101, KME_PAYOUT = 200
};

typedef enum kme_status {
    KME_OK = 0,
    KME_E_INVALID = 1,      /* bad argument / handle */
    KME_E_CAPACITY = 2,     /* epoch, order pool, oid table, trade buffer or symbol capacity exceeded */
    KME_E_DOMAIN = 3,       /* input where the reference throws (NPE) or never terminates, or that
                               falls outside the documented parity domain (detail: kme_domain) */
    KME_E_UNFUNDED = 4,     /* FUNDED mode: acceptance of some order is not provably
                               independent of the ledger (see kme_mode).  NOT fatal: the records
                               before kme_epoch_status.n_effective took effect, nothing after them
                               did (an order epoch whose proof fails: none of it), and the engine
                               accepts further epochs -- e.g. after TRANSFER records that top the
                               accounts up, the refused records can be resubmitted. */
    KME_E_UNSUPPORTED = 5,  /* operation not available in this mode (PAYOUT of an absent symbol in
                               FUNDED mode needs the positions ledger) */
    KME_E_HIP = 6,          /* HIP runtime error */
    KME_E_FAILED = 7        /* engine already failed; like the reference's dead stream thread,
                               it accepts nothing further */
} kme_status;

/* Detail for KME_E_DOMAIN / KME_E_CAPACITY (kme_epoch_status.detail). */
enum kme_domain {
    KME_D_NONE = 0,
    KME_D_NPE_POSITION = 1,  /* position null with adj != 0 (KP:179-180, 332): negative sizes */
    KME_D_NPE_BUCKET = 2,    /* log10 bit scan points at an empty level (KP:234-235, 252-253; H5) */
    KME_D_NPE_ORDER = 3,     /* missing order node (KP:236-237, 257) */
    KME_D_NPE_BALANCE = 4,   /* balance null (KP:157, 286, 331) */
    KME_D_HANG = 5,          /* removeAllOrders on a non-empty book never returns (KP:341-353) */
    KME_D_NPE_BOOK = 6,      /* book missing for a resting order (KP:294) */
    KME_D_PRICE = 7,         /* a resting price outside 0..126 aliases buckets across symbols (KP:379-416) */
    KME_D_DUP_OID = 8,       /* BUY/SELL reuses the oid of a live order (KP:221 would corrupt lists) */
    KME_D_FUNDED_RANGE = 9,  /* FUNDED mode without KME_FLAG_SERIAL_FALLBACK: BUY/SELL price outside
                                0..100 or size < 0 (with the flag such an epoch runs serially) */
    KME_D_SENTINEL_OID = 10, /* reserved (no longer raised) */
    KME_D_CAP_POOL = 11, KME_D_CAP_OIDTAB = 12, KME_D_CAP_TRADES = 13, KME_D_CAP_SYMBOL = 14,
    KME_D_CAP_ACCOUNT = 15, KME_D_CAP_LEDGER = 16, KME_D_CAP_EPOCH = 17,
    KME_D_UNPROVEN = 18,     /* KME_E_UNFUNDED of the epoch as a whole: the funded proof failed, so
                                none of its records took effect (error_index -1, n_effective 0),
                                whatever other fault the epoch holds further on -- except a fault of
                                record 0 itself, which is reported instead (the reference throws
                                there whatever the ledger holds; nothing takes effect either way) */
    KME_D_SID_RANGE = 19,    /* ADD_SYMBOL of sid = Long.MIN_VALUE or |sid| >= 2^55: the bucket pointer
                                (sid << 8) | price (KP:379-381) then aliases other books' buckets */
    KME_D_GUARD_OTPOS = 20,  /* internal consistency check (k_match_lanes): an oid-table position
                                outside the table; never expected (a bug report, not an input fault) */
    KME_D_GUARD_SLOT = 21,   /* internal consistency check (k_match_lanes): a node slot outside the
                                pool; never expected */
    KME_D_GUARD_LOOKBACK = 22  /* internal check (KME_E_HIP): a small sort's or scan's look-back found
                                an earlier tile's word missing for ~1 s; never expected */
};

/* Engine modes.
 * EXACT : every store of the reference (Books, Buckets, Orders, Balances, Positions, KP:30-49) is
 *         kept bit-exactly on the device, including the value-keyed position writes (KP:434-436).
 *         One wavefront applies the epoch in arrival order (the ledger couples all symbols).
 * FUNDED: symbol groups are matched in parallel, one wavefront per group.  Legal only while every
 *         BUY/SELL provably passes checkBalance (KP:167-182) -- the engine verifies this per epoch
 *         with a conservative per-account reservation bound and fails with KME_E_UNFUNDED
 *         otherwise.  Tape and book state are bit-exact; the ledger keeps account existence and
 *         the reservation bound only (exact balances/positions: EXACT mode). */
enum kme_mode { KME_MODE_EXACT = 0, KME_MODE_FUNDED = 1 };

/* kme_config.flags
 * KME_FLAG_EXACT_LEDGER (FUNDED, SURVEY §8 row f next-2): after the parallel matching of each
 *   epoch its ledger effects -- createBalance / transfer (KP:131-146), checkBalance's reservation
 *   and position adjustment (KP:167-182), both fillOrder calls per trade (KP:276-287) and
 *   postRemoveAdjustments (KP:325-333), with the value-keyed position writes of KP:434-436 -- are
 *   applied to device Balances / Positions tables exactly as the reference's arrival order would,
 *   so the final ledger stores are bit-exact too (kme_snapshot_ledger).  Balances are per-account
 *   sums and positions per (account, symbol) chains, applied in parallel; chains a value-keyed write
 *   couples are replayed together in arrival order; an epoch with too many such couplings takes the
 *   serial replay (kme_epoch_status.ledger_serial).  env KME_LEDGER_SERIAL=1: always serial. */
#define KME_FLAG_EXACT_LEDGER 1u
/* KME_FLAG_SERIAL_FALLBACK (FUNDED, requires KME_FLAG_EXACT_LEDGER; SURVEY §8 row f next-2, the
 *   validate-and-replay relaxation): an epoch whose funded proof fails -- some checkBalance
 *   (KP:177) or transfer debit (KP:142) might reject -- is not refused with KME_E_UNFUNDED but
 *   matched by the serial EXACT engine on the exact ledger (every reject as in the reference), after
 *   which the funded bounds restart from the exact balances.  kme_epoch_status.serial_fallback
 *   tells which epochs took that path. */
#define KME_FLAG_SERIAL_FALLBACK 2u
/* With KME_FLAG_SERIAL_FALLBACK the FUNDED engine takes every record the reference takes: besides an
 *   unprovable epoch, an epoch runs serially when it holds a BUY/SELL priced outside 0..100 or of
 *   negative size, a record of an account id outside [0, max_accounts), a record on a sparse symbol
 *   (|sid| >= max_symbols, kme_config.max_sparse_symbols) or on a symbol whose book holds such an order
 *   (a level above 100, a negative size) -- the parallel matchers keep prices 0..100 and sizes >= 0.
 * KME_FLAG_REFUSE_SERIAL (FUNDED, without SERIAL_FALLBACK; kme_multi sets it on its shards when it can
 *   consolidate): such an epoch is refused as unproven (KME_E_UNFUNDED / KME_D_UNPROVEN, nothing of it
 *   takes effect) instead of faulting, so that the caller can hand it to an engine that takes it. */
#define KME_FLAG_REFUSE_SERIAL 4u

typedef struct kme_config {
    uint32_t abi_version;      /* KME_ABI_VERSION */
    uint32_t mode;             /* kme_mode */
    uint32_t max_symbols;      /* symbol groups: |sid| < max_symbols (books +sid and -sid, KP:184-191) */
    uint32_t max_accounts;     /* FUNDED: account ids 0 <= aid < max_accounts */
    uint32_t max_epoch;        /* max records per submitted epoch */
    uint32_t max_trades;       /* max trades per epoch (each trade = 2 fill records) */
    uint64_t max_resting;      /* resting orders the Orders store holds (FUNDED adds 64 node slots per
                                  symbol for the per-group allocation chunks; total < 2^31; FUNDED:
                                  max_resting + 64 (max_symbols + 1) + max_epoch <= 2^29) */
    uint64_t ledger_capacity;  /* exact ledger: entries Balances and Positions take before their first
                                  growth (kme_ledger_stats; the tables grow between epochs) */
    int32_t device;            /* HIP device ordinal */
    uint32_t credit_shards;    /* FUNDED: number of symbol shards an account's credit is split over
                                  (0 or 1 = one engine).  Each shard proves its own orders against
                                  floor(credit / n) and ceil(debit / n), so the shards' reservations
                                  together never exceed the account's cash. */
    uint32_t flags;            /* KME_FLAG_* */
    int32_t light_max;         /* FUNDED: a symbol group with at most this many records in an epoch is
                                  matched by one lane of a wavefront shared with 31 other groups
                                  (k_match_lanes), a busier one by a whole wavefront (k_match); both
                                  run concurrently.  0 = engine default (128), < 0 = wavefronts only.
                                  Results are identical either way. */
    uint32_t max_sparse_symbols; /* symbols with |sid| >= max_symbols the stores hold (KP:184-191 takes any
                                  long): 0 = the default, 4,096 for EXACT mode and FUNDED with
                                  KME_FLAG_SERIAL_FALLBACK, none otherwise; KME_SPARSE_NONE = none.
                                  Only the serial engine handles them (max_symbols + sparse <= 2^24). */
    uint32_t _reserved;
} kme_config;
#define KME_SPARSE_NONE 0xFFFFFFFFu

/* One epoch of input records, structure-of-arrays (Order fields KP:451-456).  The reference's
 * optional next/prev input fields must be null and are not carried. */
typedef struct kme_orders {
    const int32_t* action;
    const int64_t* oid;
    const int64_t* aid;
    const int64_t* sid;
    const int32_t* price;
    const int32_t* size;
} kme_orders;

/* One trade = the reference's two fill records (executeTrade, KP:265-274):
 *   maker fill  {taker BUY ? SOLD : BOUGHT, maker_oid, maker_aid, maker_sid, price 0, size}
 *   taker fill  {taker BUY ? BOUGHT : SOLD, taker oid, aid, sid, taker.price - maker_price, size} */
typedef struct kme_trade {
    int64_t maker_oid, maker_aid, maker_sid;
    int32_t maker_price, size;
} kme_trade; /* 32 bytes */

/* Per-epoch results.  For input i the reference forwards, in order:
 *   IN  = input i unchanged;
 *   for t in [trade_off[i], trade_off[i+1]): maker fill, taker fill of trades[t];
 *   OUT = input i with action = out_action[i], size = out_size[i],
 *         prev = (out_flags[i] & KME_OUT_HAS_PREV) ? out_prev[i] : null, next = null. */
#define KME_OUT_HAS_PREV 1u
typedef struct kme_epoch_result {
    int32_t* out_action;   /* [n] */
    int32_t* out_size;     /* [n] */
    int64_t* out_prev;     /* [n] */
    uint8_t* out_flags;    /* [n] */
    uint32_t* trade_off;   /* [n + 1] exclusive prefix sum of per-input trade counts */
    kme_trade* trades;     /* [trades_cap] */
    uint32_t trades_cap;
} kme_epoch_result;

/* On an error the records [0, n_effective) of the submission took effect exactly as the reference
 * would have processed them, and their results are valid (out_* [0, n_effective),
 * trade_off[0 .. n_effective], trades[0 .. trade_off[n_effective])): the reference forwards and
 * commits every record before the one that throws (KP:97, 124-125).  Nothing from the faulting
 * record on is answered.  Every error except KME_E_UNFUNDED leaves the engine failed. */
typedef struct kme_epoch_status {
    int32_t status;        /* kme_status of the epoch */
    int32_t detail;        /* kme_domain */
    int64_t error_index;   /* input index of the first fault, or -1 (a fault of the epoch as a whole) */
    uint32_t n_inputs;
    uint32_t n_trades;
    uint64_t n_orders;     /* BUY/SELL/CANCEL records (headline metric unit) */
    uint64_t n_rests, n_maker_visits, n_cancel_ok;
    uint32_t serial_fallback;   /* epochs (device sub-epochs of kme_submit_epoch) that ran serially
                                   under KME_FLAG_SERIAL_FALLBACK */
    uint32_t n_effective;       /* records of the submission that took effect (= n_inputs when OK) */
    uint32_t ledger_repaired;   /* KME_FLAG_EXACT_LEDGER: position chains the parallel ledger pass replayed
                                   in arrival order because a value-keyed write (KP:434-436) reached them */
    uint32_t ledger_serial;     /* KME_FLAG_EXACT_LEDGER: epochs whose ledger the serial replay applied
                                   (too many such couplings, or the parallel pass is off) */
} kme_epoch_status;

typedef struct kme_engine kme_engine;

/* Creates the stores (KP:30-49) in HBM and binds them (MatchingEngine.init, KP:86-93). */
kme_status kme_create(const kme_config* cfg, kme_engine** out);
/* MatchingEngine.close (KP:129): frees device memory. */
kme_status kme_destroy(kme_engine* e);

/* Use this HIP stream (hipStream_t) for all device work; NULL = the engine's own stream.  The own
 * stream is non-blocking: nothing orders it after work the caller queued on another stream (torch's
 * fill of an output tensor, say), so a device buffer handed to an entry below must be ready when
 * the call is made -- synchronize first, or pass the caller's stream here. */
kme_status kme_set_stream(kme_engine* e, void* hip_stream);

/* MatchingEngine.process (KP:96-126) for n records, HOST buffers, synchronous.  In FUNDED mode the
 * epoch is split at account records (CREATE_BALANCE / TRANSFER) so that the reservation bound is
 * checked per run; the result arrays are filled as one epoch. */
kme_status kme_submit_epoch(kme_engine* e, const kme_orders* in, uint32_t n,
                            kme_epoch_result* out, kme_epoch_status* st);

/* Same for DEVICE-resident inputs and outputs (pointers into HBM), asynchronous on the engine
 * stream; completes at kme_wait.  `out` may be NULL to keep results in engine-owned buffers
 * (see kme_device_results).  No splitting: a FUNDED epoch must not mix account records with
 * orders of a just-created account (kme_submit_epoch does that split for host callers). */
kme_status kme_submit_epoch_device(kme_engine* e, const kme_orders* in_dev, uint32_t n,
                                   const kme_epoch_result* out_dev);
/* Completes the OLDEST device epoch in flight.  Up to two device epochs may be in flight: a second
 * kme_submit_epoch_device before kme_wait queues the next epoch behind the first on the stream (the
 * GPU does not idle on the caller's turnaround; give each its own `out_dev`, the engine-owned
 * buffers hold only the newest epoch's results).  A third submit, kme_submit_epoch, checkpoint and
 * restore return KME_E_INVALID while epochs are in flight.  An epoch refused with KME_E_UNFUNDED
 * while a later one is in flight fails the engine (that one ran without the refused records). */
kme_status kme_wait(kme_engine* e, kme_epoch_status* st);
/* Engine-owned device result buffers of the last device epoch. */
kme_status kme_device_results(kme_engine* e, kme_epoch_result* out_dev);

/* ---- Host epochs at device rate: the Java processor's path ----
 * kme_submit_epoch above copies pageable arrays and waits; a JVM feeding the engine at rate keeps two
 * epochs of records in caller-owned host memory that the engine's copy engines reach directly (JVM
 * direct ByteBuffers), and overlaps the PCIe transfers of one epoch with the kernels of the other.
 *
 * kme_host_register: make `bytes` of caller host memory at `host` DMA-able and device-mapped
 * (hipHostRegister); kme_host_unregister undoes it (no epoch using it may be in flight). */
kme_status kme_host_register(kme_engine* e, void* host, size_t bytes);
kme_status kme_host_unregister(kme_engine* e, void* host);
/* MatchingEngine.process (KP:96-126) for n records whose inputs and results live in host memory
 * registered with kme_host_register.  Asynchronous: the H2D of the six input columns (copy stream),
 * the epoch's kernels (engine stream) and the D2H of the results -- out_action / out_size / out_prev /
 * out_flags [n], trade_off [n + 1] and trades [0, trade_off[n]) (copy stream; the trades by a copy
 * kernel that reads their count on the device) -- are queued and the call returns.  kme_poll tells
 * when the oldest epoch is done, kme_wait completes it; the results are valid after kme_wait.  Up to
 * two epochs in flight (as kme_submit_epoch_device): the inputs of epoch k + 1 cross PCIe while
 * epoch k's kernels run.  As on the device path the epoch is not split at account records. */
kme_status kme_submit_epoch_host(kme_engine* e, const kme_orders* in_host, uint32_t n,
                                 const kme_epoch_result* out_host);
/* Non-blocking: *done = 1 when the oldest epoch in flight has completed (kme_wait will not block) or
 * none is in flight, 0 while it runs.  The processor's wall-clock punctuator polls with it, so the
 * stream thread never blocks on the GPU (the reference's process() never waits either, KP:96). */
kme_status kme_poll(kme_engine* e, int* done);

/* One MatchOut record as the processor forwards it (KP:97, 124, 272-273): key "IN" (kind 0) or "OUT"
 * (kind 1 = a maker / taker fill, kind 2 = the OUT echo), value = an Order (KP:449-458). */
typedef struct kme_row {
    int64_t oid, aid, sid;
    int64_t prev;          /* Order.prev when has_prev (the OUT echo of an append, KP:217), else null */
    int32_t action, price, size;
    uint8_t kind, has_prev;
    uint8_t _pad[2];
} kme_row; /* 48 bytes */
/* Expands the results of records [0, n) of an epoch into its MatchOut rows, in order: IN, the maker
 * and taker fill of each trade (executeTrade, KP:265-274), OUT.  *n_rows = rows needed; nothing is
 * written past cap (KME_E_CAPACITY when they do not fit).  Host buffers; the JNI glue and the host-path
 * harness both use it. */
kme_status kme_expand_rows(const kme_orders* in, uint32_t n, const kme_epoch_result* res, kme_row* rows,
                           size_t cap, size_t* n_rows);
/* The same rows, written by n_threads host threads (records split into contiguous ranges; each
 * range's first row follows from trade_off alone), for callers that hand whole epochs to one
 * consumer (the JNI glue).  n_threads 0 = the machine's hardware threads, at most 16; at most 64. */
kme_status kme_expand_rows_mt(const kme_orders* in, uint32_t n, const kme_epoch_result* res, kme_row* rows,
                              size_t cap, size_t* n_rows, uint32_t n_threads);

/* Identifies the sources libkme was built from (a hash of csrc/ and include/): the test session
 * rebuilds the library when it differs from the tree's. */
const char* kme_build_id(void);

/* Persistence (SURVEY §8 row f next-3; the reference keeps its state in RocksDB stores with
 * changelogs, KP:30-49, and commits after every record, KP:125).  kme_checkpoint writes the
 * engine's device state -- books, buckets, resting orders, the FUNDED reservation ledger or the
 * EXACT Balances/Positions, and the input sequence number -- to a file, between
 * epochs (call it after the epoch whose input offsets are being committed).  kme_restore loads
 * such a file into a freshly created engine of the same configuration; processing then resumes with
 * the records after the committed offset and produces exactly the tape an uninterrupted engine
 * would.  KME_E_INVALID on a config / format mismatch, KME_E_FAILED if the engine has failed. */
kme_status kme_checkpoint(kme_engine* e, const char* path);
kme_status kme_restore(kme_engine* e, const char* path);
/* The same with an application record stored beside the state in the one file: what the caller needs
 * to resume exactly at that point -- the Java processor keeps the last input offset the state covers
 * and the MatchOut rows of completed epochs it has not forwarded yet.  The file is
 * written to `path`.tmp, flushed to disk and renamed over `path`, so a crash leaves the previous
 * checkpoint whole.  kme_restore_app: *app_bytes = the record's size; when it exceeds app_cap (app
 * may be NULL with app_cap 0) the call returns KME_E_CAPACITY and changes nothing (call again with a
 * large enough buffer).  Format-3 files (ABI 6) restore too. */
kme_status kme_checkpoint_app(kme_engine* e, const char* path, const void* app, size_t app_bytes);
kme_status kme_restore_app(kme_engine* e, const char* path, void* app, size_t app_cap, size_t* app_bytes);
/* What the file holds is the stores' live content (format 3): group states, the price levels whose
 * bit is set, the used node pool, the FUNDED reservation ledger, the live Balances / Positions entries;
 * the oid table is rebuilt from the resting orders on restore, the ledger tables at the size their
 * entries need.  Every checkpoint file (and kme_multi manifest) ends with a trailer: the application
 * record's size and a 64-bit digest of all bytes before it.  A restore recomputes the digest over
 * what it reads and refuses a file that does not match (KME_E_INVALID, engine untouched).
 * kme_checkpoint_inspect reads the trailer only: a commit point records (bytes, digest) of the
 * checkpoint it wrote in a changelogged store, and a restart checks the file it finds against that
 * record before trusting it. */
typedef struct kme_checkpoint_info {
    uint64_t file_bytes;   /* the whole file */
    uint64_t app_bytes;    /* the application record */
    uint64_t digest;       /* of every byte before the trailer */
} kme_checkpoint_info;
kme_status kme_checkpoint_inspect(const char* path, kme_checkpoint_info* out);
/* The state changelog: the file at `path` cut into chunks of chunk_bytes (>= 4096;
 * the last one shorter), hashes[k] = a 64-bit content hash of chunk k (host threads).  *n_chunks = the
 * count; KME_E_CAPACITY when it exceeds cap.  Format 4 keeps unchanged stores at unchanged offsets, so
 * the chunks whose hash changed since the last commit are what changed. */
kme_status kme_checkpoint_chunks(const char* path, uint32_t chunk_bytes, uint64_t* hashes, size_t cap, size_t* n_chunks);

/* The exact ledger's tables (EXACT mode, FUNDED + KME_FLAG_EXACT_LEDGER; else KME_E_UNSUPPORTED).
 * Balances and Positions grow without bound in the reference (RocksDB, KP:30-37; H2 keeps stale
 * value-keyed positions forever, KP:283-284, 434-436).  Here they are hash tables in HBM that the
 * engine rehashes into larger ones between epochs, before the entries in use plus the most that the
 * epochs in flight and the next one could add (one Balances entry per record, one Positions entry per
 * ledger effect: a record's check or refund, two fills per trade) could pass half load; ledger_capacity
 * only sets the initial size.  KME_D_CAP_LEDGER then means the device is out of memory. */
typedef struct kme_ledger_info {
    uint64_t bal_slots, pos_slots;   /* table sizes */
    uint64_t bal_used, pos_used;     /* slots in use (live entries and tombstones) */
    uint32_t grows;                  /* rehashes so far */
    uint32_t _pad;
} kme_ledger_info;
kme_status kme_ledger_stats(kme_engine* e, kme_ledger_info* out);

/* Canonical text snapshots (sorted), identical in format to the reference stores' contents:
 *   books : "B <key> <msb> <lsb>" (Books), "K <bucketPtr> <firstOid> <lastOid>" (Buckets),
 *           "O <oid> <action> <aid> <sid> <price> <size> <next|null> <prev|null>" (Orders)
 *   ledger: "A <aid> <balance>" (Balances), "P <keyMsb> <keyLsb> <amount> <available>" (Positions);
 *           EXACT mode, or FUNDED with KME_FLAG_EXACT_LEDGER (otherwise KME_E_UNSUPPORTED).
 * *text is malloc'd; free with kme_free. */
kme_status kme_snapshot_books(kme_engine* e, char** text, size_t* len);
kme_status kme_snapshot_ledger(kme_engine* e, char** text, size_t* len);
void kme_free(void* p);

/* Top-of-book market data per symbol group g (device buffer of max_symbols entries, async; the sparse
 * symbols of kme_config.max_sparse_symbols are not part of it):
 * {best bid price, best ask price, bid qty, ask qty} as int32 (-1 / 0 when a side is empty).
 * Bid = highest price in book +g, ask = lowest price in book -g (book 0 is shared). */
typedef struct kme_tob { int32_t bid_px, ask_px, bid_qty, ask_qty; } kme_tob;
kme_status kme_top_of_book(kme_engine* e, kme_tob* dev_out);
/* The same for a list of groups (device array of n group ids, e.g. the symbols of this engine's
 * partition): dev_out[k] = top of book of dev_groups[k] (-1 / 0 for an id >= max_symbols).  With
 * symbols keyed over N engines this is the engine's share of the market-data snapshot that
 * bench.py all-gathers over RCCL. */
kme_status kme_top_of_book_groups(kme_engine* e, const uint32_t* dev_groups, uint32_t n, kme_tob* dev_out);

/* ---- Multi-GPU: one engine per GPU, symbols keyed over them (kme_shard_of) ----
 * An RCCL communicator over the node's engines.  kme_comm_unique_id (on one rank) fills 128 bytes
 * that the caller hands to every rank over any channel (torch.distributed, a Kafka control topic);
 * kme_comm_init joins rank `rank` of `n_ranks` on the engine's device (blocks until all joined).
 * RCCL is loaded at the first call (env KME_RCCL_LIB, default librccl.so.1): libkme itself does not
 * depend on it. */
typedef struct kme_comm kme_comm;
/* Loads the RCCL the kme_comm_* calls use, once per process: `path` (NULL = env KME_RCCL_LIB, else
 * librccl.so.1).  A process that already runs an RCCL (torch's) passes that library's path, so one
 * RCCL serves both.  KME_E_INVALID when another copy was loaded already (a kme_comm_* call without
 * kme_rccl_load loads the default), KME_E_UNSUPPORTED when it cannot be loaded. */
kme_status kme_rccl_load(const char* path);
/* The last RCCL failure of this process as text (ncclGetErrorString of the result and
 * ncclGetLastError; "" when none): every kme_comm_* call that returns KME_E_HIP for an RCCL result
 * records it here (and prints it to stderr). */
const char* kme_rccl_last_error(void);
kme_status kme_comm_unique_id(void* id128);
kme_status kme_comm_init(kme_engine* e, uint32_t n_ranks, uint32_t rank, const void* id128, kme_comm** out);
kme_status kme_comm_destroy(kme_comm* c);
/* Per-epoch market data, the only collective of the data path: this engine's top of book for its
 * n_groups symbol groups (as kme_top_of_book_groups) into its own block of dev_all (rows_per_rank
 * rows per rank, rank-major; rows past n_groups are -1 / 0), then an in-place ncclAllGather over
 * xGMI on the engine stream, so every rank holds the node's snapshot (16 B per symbol). */
kme_status kme_market_data_allgather(kme_engine* e, kme_comm* c, const uint32_t* dev_groups, uint32_t n_groups,
                                     uint32_t rows_per_rank, kme_tob* dev_all);
/* Credit between symbol shards (credit_shards = N > 1; between epochs, none in flight).  Each shard
 * proves its orders against its own share of an account's cash and the funded bound only falls, so a
 * share can run dry while the others hold cash.  kme_credit_state: this engine's
 * funded bound and demand so far per account, two int64 device arrays of max_accounts
 * (dev_out[0, A) and dev_out[A, 2A)); an account this engine does not hold reports bound 0 and
 * demand -1.  kme_credit_adjust: the re-split of the pooled bound from every shard's pair (dev_all =
 * N such blocks, shard-major) over the shards that hold the account: every engine computes the same
 * split and the shares sum to the pooled bound, so the account's cash still covers all of them.
 * kme_credit_rebalance: state, all-gather over RCCL, adjust -- a collective every rank calls and
 * every rank completes: a rank that cannot re-split (an epoch in flight: KME_E_INVALID, a failed
 * engine: KME_E_FAILED) still takes part with a status word, and then no rank adjusts; that rank
 * returns its own status, the others KME_E_INVALID.  All three have completed on the device when they
 * return (dev_out may be read on any stream). */
kme_status kme_credit_state(kme_engine* e, int64_t* dev_out);
kme_status kme_credit_adjust(kme_engine* e, const int64_t* dev_all, uint32_t n_shards, uint32_t my_shard);
kme_status kme_credit_rebalance(kme_engine* e, kme_comm* c);

/* ---- Multi-GPU drop-in: one MatchIn stream over N engines ----
 * The reference's processor takes its one-partition MatchIn whole (topic.js:17-18, KP:51-52).  A
 * kme_multi is N FUNDED engines (devices[k]; a device may repeat) behind the host-epoch calls of one
 * engine: each epoch is split by symbol (kme_router_split: Kafka's keyed partitioner over |sid|,
 * cancels to their order's partition, account records to every engine with 1/N of the credit), the
 * parts run as host epochs on their engines concurrently, and kme_multi_wait merges the results
 * into input order -- the caller's kme_epoch_result is exactly one engine's over the whole stream.
 * Before every epoch the engines' funded credit is pooled and split again (kme_credit_state /
 * kme_credit_adjust), queued on the engine streams behind the epochs in flight (env
 * KME_MULTI_REBALANCE_EVERY = epochs between re-splits, 0 = never).  cfg: FUNDED, credit_shards is
 * set to N; flags 0, or EXACT_LEDGER | SERIAL_FALLBACK (the shards themselves run with flags 0: the
 * exact ledger couples every symbol).  The trades of one merged epoch must fit max_trades.  A fault of
 * a shard fails the whole (the other shards went past it): the records before the first fault in
 * input order are answered (n_effective), as one engine answers them, then it accepts nothing further
 * -- except, with EXACT_LEDGER | SERIAL_FALLBACK, a refusal of the funded proof (KME_E_UNFUNDED): the
 * shards are retired and one engine of those flags on devices[0] takes the stream (SURVEY §8e:
 * outside the funded domain only one engine is exact), built by replaying the input history kept
 * since the start (env KME_MULTI_HISTORY records at most, default 2^25; past it the refusal stays
 * fatal, kme_multi_info says so and stderr says it once); it answers the rest of that epoch and every
 * later one, synchronously at submit.  Its checkpoints are the one engine's (the manifest says so).
 * The history survives restarts: each checkpoint appends the records since the previous one to
 * `path`.hist (fsync'd before the manifest naming its length and digest is committed), and a restore
 * reads it back. */
typedef struct kme_multi kme_multi;
kme_status kme_multi_create(const kme_config* cfg, uint32_t n, const int32_t* devices, kme_multi** out);
kme_status kme_multi_destroy(kme_multi* m);
/* as kme_submit_epoch_host / kme_poll / kme_wait (two epochs in flight; out->trades_cap >= max_trades) */
kme_status kme_multi_submit_epoch_host(kme_multi* m, const kme_orders* in_host, uint32_t n, const kme_epoch_result* out_host);
kme_status kme_multi_poll(kme_multi* m, int* done);
kme_status kme_multi_wait(kme_multi* m, kme_epoch_status* st);
/* as kme_checkpoint_app / kme_restore_app: every engine to `path`.g<generation>.<k>, the input history
 * onto `path`.hist, then a manifest at `path` (written and renamed last: the commit of the set); a
 * restore also rebuilds the router's oid directory from the engines' resting orders and reads the
 * history back (a missing or damaged `path`.hist does not fail the restore: consolidation is off) */
kme_status kme_multi_checkpoint_app(kme_multi* m, const char* path, const void* app, size_t app_bytes);
kme_status kme_multi_restore_app(kme_multi* m, const char* path, void* app, size_t app_cap, size_t* app_bytes);
/* engine k (snapshots, diagnostics) */
kme_status kme_multi_engine(kme_multi* m, uint32_t k, kme_engine** out);
/* Whether an epoch the shards cannot prove is survivable now (can_consolidate: the flags allow it, the
 * shards still run and the input history since the start is complete), the history's size and cap, the
 * records of it the last checkpoint made durable, and the checkpoint generation. */
typedef struct kme_multi_status {
    uint32_t n_engines, consolidated, can_consolidate, failed;
    uint64_t history_records, history_cap, history_saved, generation;
} kme_multi_status;
kme_status kme_multi_info(kme_multi* m, kme_multi_status* out);

/* Wall-clock (HIP event) duration in ms of each kernel phase of the last epoch; index by name
 * (kme_phase_names).  Used by bench.py for the roofline of the dominant kernel. */
#define KME_MAX_PHASES 16
kme_status kme_phase_times(kme_engine* e, float* ms, int* n_phases);
const char* kme_phase_name(int i);
/* 0 = off, KME_TIMING_ALL (1) = every phase, KME_TIMING_MATCH = the matching phase only (timing
 * events serialise the stream around them, ~10 us each) */
#define KME_TIMING_ALL 1
#define KME_TIMING_MATCH 2
kme_status kme_enable_timing(kme_engine* e, int enable);

/* Serialises a processed epoch exactly as consumer.js prints MatchOut (consumer.js:19):
 * "IN <json>\nOUT <json>\n..." with Jackson's Order layout (KP:488-494).  Host buffers.
 * Writes at most cap bytes; *len receives the full length (call again with a bigger buffer
 * if *len > cap). */
kme_status kme_tape_json(const kme_orders* in, uint32_t n, const kme_epoch_result* res,
                         char* buf, size_t cap, size_t* len);

/* The same text produced on the GPU (SURVEY §8 row f next-1): `in_dev` = the epoch's device
 * inputs, `res_dev` = its device results (NULL: the engine-owned results of the last
 * kme_submit_epoch_device), `out_dev` = a device buffer of `cap` bytes.  Stream-ordered on the
 * engine stream and synchronous; *len = the full length.  Nothing is written when *len > cap
 * (call again with a bigger buffer); KME_E_CAPACITY when one epoch's text would exceed 4 GiB. */
kme_status kme_tape_json_device(kme_engine* e, const kme_orders* in_dev, uint32_t n, const kme_epoch_result* res_dev,
                                void* out_dev, size_t cap, size_t* len);

/* Jackson JsonDeserializer<Order> (KP:513-520) for one record: numbers or numeric strings,
 * unknown properties rejected, next/prev must be absent or null. */
kme_status kme_order_from_json(const char* json, size_t len, int32_t* action, int64_t* oid,
                               int64_t* aid, int64_t* sid, int32_t* price, int32_t* size);

/* Kafka's default keyed partitioner over decimal(|sid|) (murmur2, toPositive, % n). */
uint32_t kme_shard_of(int64_t sid, uint32_t n_shards);

/* Partition router (replaces kme/sharding.py PartitionRouter on the product
 * path).  One MatchIn stream over n engines, each input answered by exactly one of them:
 * BUY/SELL/ADD_SYMBOL/REMOVE_SYMBOL/PAYOUT -> kme_shard_of(sid, n); CANCEL (no symbol,
 * exchange_test.js:101) -> the partition of the last BUY/SELL with its oid (a directory kept by the
 * router; an unknown oid -> 0, which rejects it, KP:290); CREATE_BALANCE/TRANSFER -> every
 * partition (KME_ROUTE_ALL; echoed by partition 0 only); anything else -> 0.  Not thread-safe. */
typedef struct kme_router kme_router;
#define KME_ROUTE_ALL (-1)
typedef struct kme_orders_buf {   /* writable kme_orders */
    int32_t* action;
    int64_t* oid;
    int64_t* aid;
    int64_t* sid;
    int32_t* price;
    int32_t* size;
} kme_orders_buf;
kme_status kme_router_create(uint32_t n_partitions, uint64_t directory_capacity, kme_router** out);
kme_status kme_router_destroy(kme_router* r);
/* dest[i] = partition of input i (or KME_ROUTE_ALL); updates the oid directory. */
kme_status kme_router_route(kme_router* r, const kme_orders* in, uint32_t n, int32_t* dest);
/* Routes and splits: partition k's records, in arrival order, into parts[k] (arrays of capacity
 * n), counts[k] of them; optional echo[k][j] = 1 if partition k answers its j-th record (0 for the
 * copies of account records on partitions > 0) and index[k][j] = its input index. */
kme_status kme_router_split(kme_router* r, const kme_orders* in, uint32_t n, const kme_orders_buf* parts,
                            uint32_t* counts, uint8_t* const* echo, uint32_t* const* index);
uint64_t kme_router_directory_size(const kme_router* r);

/* Diagnostics: per-symbol-group words written by a -DKME_STAMPS build of the match kernel
 * (in-kernel s_memtime stamps; zero in the product build).  Copies min(n, max_symbols * 32). */
#define KME_DBG_WORDS 48
kme_status kme_debug_counters(kme_engine* e, uint64_t* out, size_t n);

const char* kme_strerror(int status);
const char* kme_domain_str(int detail);

#ifdef __cplusplus
}
#endif
#endif
