/*
 * kme_oracle.h -- CPU restatement of the reference matching path.  TEST INFRASTRUCTURE ONLY.
 *
 * This is the checker, never the product: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  It restates, line by line, the Kafka Streams processor
 * `KProcessor.MatchingEngine` (reference src/main/java/KProcessor.java:63-445, "KP" below) with
 * the five key-value stores (KP:30-49) as hash maps, Java int/long wrap arithmetic, and the
 * double-precision log10 bit scans (KP:371-377) replaced by the exact integer threshold table
 * they imply under a correctly rounded log10 (tools/gen_log10_table.py).
 *
 * PARITY UNPINNED: the reference ships no tests, fixtures or golden vectors
 * and it cannot run in this image (no JDK / kafka-streams jars).  Golden vectors under
 * tests/golden/ are produced by this restatement; see DESIGN.md "Oracle".
 */
#ifndef KME_ORACLE_H
#define KME_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One output record as the reference forwards it: key "IN"/"OUT" (KP:97,124,272-273) and the
 * Order value (KP:449-458).  next/prev are Java `Long` (nullable). */
typedef struct ko_rec {
    int32_t key;      /* 0 = "IN", 1 = "OUT" */
    int32_t action;
    int64_t oid, aid, sid;
    int32_t price, size;
    int64_t next, prev;
    int32_t has_next, has_prev;
} ko_rec; /* 64 bytes */

/* Domain errors: places where the reference throws (killing the stream thread) or never
 * terminates.  State after one of these is undefined, as in the reference. */
enum {
    KO_OK = 0,
    KO_E_NPE_POSITION = 1,   /* checkBalance/postRemoveAdjustments: position null, adj != 0 (KP:179-180, 332) */
    KO_E_NPE_BUCKET = 2,     /* tryMatch: bit scan points at an empty bucket (KP:234-235, 252-253) */
    KO_E_NPE_ORDER = 3,      /* tryMatch/removeOrder: missing order node (KP:236-237, 257) */
    KO_E_NPE_BALANCE = 4,    /* fillOrder/postRemoveAdjustments/payout: balance null (KP:157, 286, 331) */
    KO_E_HANG = 5,           /* removeAllOrders on a non-empty book never terminates (KP:341-353) */
    KO_E_NPE_BOOK = 6        /* removeOrder: book missing for a resting order (KP:294, 301) */
};

typedef struct ko_engine ko_engine;

ko_engine* ko_create(void);
void ko_destroy(ko_engine* e);

/* MatchingEngine.process (KP:96-126) over n records given as SoA.  Appends the forwarded
 * records to the engine's tape.  has_next/has_prev may be NULL (all null links).
 * Returns KO_OK, or the first domain error (then *n_done is the index of the faulting record). */
int ko_process_batch(ko_engine* e, size_t n, const int32_t* action, const int64_t* oid,
                     const int64_t* aid, const int64_t* sid, const int32_t* price,
                     const int32_t* size, size_t* n_done);

/* Tape access: records forwarded since the last ko_tape_clear. */
size_t ko_tape_len(const ko_engine* e);
const ko_rec* ko_tape(const ko_engine* e);
void ko_tape_clear(ko_engine* e);
/* When disabled the engine still runs every store operation but does not keep the tape
 * (used to time the path without the tape buffer growing). */
void ko_set_keep_tape(ko_engine* e, int keep);
uint64_t ko_records_forwarded(const ko_engine* e);

/* Jackson-format JSON of one Order value (KP:488-494): {"action":..,..,"next":..,"prev":..}.
 * Returns the length written (buf must hold >= 256 bytes). */
size_t ko_order_json(const ko_rec* r, char* buf);
/* Whole tape as consumer.js prints it ("IN {...}\n" / "OUT {...}\n", consumer.js:19). Caller
 * frees with ko_free. */
char* ko_tape_text(const ko_engine* e, size_t* len);

/* Canonical, sorted text dump of the book stores (Books, Buckets, Orders: KP:38-49) and of the
 * ledger stores (Balances, Positions: KP:30-37).  Caller frees with ko_free. */
char* ko_dump_books(const ko_engine* e, size_t* len);
char* ko_dump_ledger(const ko_engine* e, size_t* len);
void ko_free(void* p);

/* The log10-derived bit scans (KP:371-377) -- exported for the table test. */
int32_t ko_first_set_bit_pos(int64_t n);
int32_t ko_last_set_bit_pos(int64_t n);

#ifdef __cplusplus
}
#endif
#endif
