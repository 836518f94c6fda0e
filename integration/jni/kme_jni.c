/* kme_jni.c -- JNI glue for GpuMatchingEngine.java, the processor that replaces the reference's
 * MatchingEngine at its topology (KProcessor.java:52, `.addProcessor("MatchingEngine", ...)`).
 *
 * The product path at rate (include/kme.h, "Host epochs at device rate"): this file allocates two
 * slots of page-aligned host memory -- the six Order columns of an epoch (structure of arrays, native
 * byte order) and the MatchOut rows that come back -- registers them with the engine once, and hands
 * them to Java as direct ByteBuffers (NewDirectByteBuffer), so an epoch crosses PCIe straight from and
 * to the buffers Java reads and writes: no array pinning, no copies through the JNI boundary, no two
 * registrations sharing a page, and the garbage collector is never blocked on the GPU.
 *
 *   create(...)               the engine (or nDevices symbol-shard engines, kme_multi), its slots and
 *                             their result buffers
 *   buffer(h, slot, column)   the slot's column 0..5 (action, oid, aid, sid, price, size) or 6 (rows)
 *   submit(h, slot, n)        kme_submit_epoch_host: H2D, kernels, D2H queued; returns at once
 *   poll(h)                   kme_poll: 1 when the oldest epoch in flight is done (punctuator)
 *   complete(h, slot, st)     kme_wait + kme_expand_rows_mt into the slot's row buffer, in the
 *                             reference's order: IN (KP:97), maker / taker fill per trade
 *                             (executeTrade, KP:265-274), OUT (KP:124); st[0..3] = status, domain
 *                             detail, error index, records that took effect (kme_epoch_status).  The
 *                             rows stay "ready" (not yet forwarded) until forwarded(h, slot).
 *   forwarded(h, slot)        Java has forwarded the slot's rows
 *   checkpoint(h, path, off, gen, info)
 *                             the commit point: kme_checkpoint_app of the engine
 *                             state with an application record = the commit's generation, the last
 *                             input offset the state covers and the rows of every ready slot, oldest
 *                             first; info = the file's size and digest (kme_checkpoint_inspect), which
 *                             the processor logs to its changelogged commit store
 *   restore(h, path, out)     kme_restore_app: the state, the offset (out[0]) and the ready rows back
 *                             in their slots (out[1] = how many, then (slot, rows) pairs, oldest first);
 *                             out[6..8] = the file's generation, size and digest (checked by the
 *                             processor against the commit store's record)
 *   shardStatus(h, out)       nDevices > 1: whether an epoch no shard can prove is survivable now
 *                             (kme_multi_info: the input history since the start is complete), the
 *                             history's size, cap and durable part; a single engine: status INVALID
 *   stateChunks(h, path, chunkBytes, changed)
 *                             the checkpoint file as fixed-size chunks: which ones changed since the
 *                             last call (a content hash per chunk); the processor puts those into its
 *                             changelogged commit store, so the state follows the task to any
 *                             instance
 *
 * On an error the rows of the records that took effect ([0, n_effective)) are still produced: the
 * reference forwards and commits every record before the one that throws (KP:97, 124-125).
 *
 * Build (JDK present): integration/jni/build.sh.  This container has no JDK; the CPU test suite
 * compiles this file with -fsyntax-only against tests/jni_stub/jni.h (a declaration subset) and the GPU
 * suite drives it through a JNIEnv made with ctypes (tests/test_jni_glue.py).
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "kme.h"

#define NCOL 7                     /* six Order columns + the row buffer */

typedef struct jslot {
    void* col[NCOL];               /* page-aligned, registered; Java sees them as direct ByteBuffers */
    size_t bytes[NCOL];
    kme_orders in;
    kme_row* rows;
    size_t rows_cap;
    kme_epoch_result res;          /* native host results, registered */
    uint32_t n;                    /* records of the epoch in flight (0 = none) */
    int64_t ready_rows;            /* rows completed and not yet forwarded (-1 = none) */
    uint64_t ready_seq;            /* completion order of the ready rows */
} jslot;

typedef struct jkme {
    kme_engine* e;                 /* one engine, or */
    kme_multi* m;                  /* nDevices > 1: symbol shards on devices device .. device + nDevices - 1 */
    uint32_t max_epoch, max_trades;
    uint64_t completions;
    jslot slot[2];
    uint64_t* chash;               /* stateChunks: the content hash of each chunk the last call saw */
    size_t nchash;
    int32_t chunk_bytes;
} jkme;

/* the application record of a checkpoint (kme_checkpoint_app) */
#define JREC_MAGIC 0x324a4d4bu   /* "KMJ2" */
typedef struct jrec_head { uint32_t magic, n_ready; int64_t offset; int64_t generation; } jrec_head;
typedef struct jrec_slot { uint32_t slot, _pad; uint64_t rows; } jrec_slot;

static void throw_state(JNIEnv* env, const char* msg) {
    jclass c = (*env)->FindClass(env, "java/lang/IllegalStateException");
    if (c) (*env)->ThrowNew(env, c, msg);
}

static void* aligned(size_t bytes) {
    void* p = NULL;
    if (posix_memalign(&p, 4096, bytes ? (bytes + 4095) & ~(size_t)4095 : 4096) != 0) return NULL;
    memset(p, 0, bytes ? bytes : 1);
    return p;
}

/* the single-engine and the multi-engine calls behind one handle */
static kme_status h_submit(jkme* h, const kme_orders* in, uint32_t n, const kme_epoch_result* r) {
    return h->m ? kme_multi_submit_epoch_host(h->m, in, n, r) : kme_submit_epoch_host(h->e, in, n, r);
}
static kme_status h_poll(jkme* h, int* done) { return h->m ? kme_multi_poll(h->m, done) : kme_poll(h->e, done); }
static kme_status h_wait(jkme* h, kme_epoch_status* st) { return h->m ? kme_multi_wait(h->m, st) : kme_wait(h->e, st); }
static kme_status h_checkpoint(jkme* h, const char* p, const void* app, size_t bytes) {
    return h->m ? kme_multi_checkpoint_app(h->m, p, app, bytes) : kme_checkpoint_app(h->e, p, app, bytes);
}
static kme_status h_restore(jkme* h, const char* p, void* app, size_t cap, size_t* bytes) {
    return h->m ? kme_multi_restore_app(h->m, p, app, cap, bytes) : kme_restore_app(h->e, p, app, cap, bytes);
}

static void free_handle(jkme* h) {
    if (!h) return;
    if (h->e || h->m) {   /* epochs still in flight (a processor torn down mid-stream): their copies land first */
        kme_epoch_status st;
        for (int k = 0; k < 2; ++k)
            if (h->slot[k].n) {
                (void)h_wait(h, &st);
                h->slot[k].n = 0;
            }
    }
    for (int s = 0; s < 2; ++s) {
        jslot* sl = &h->slot[s];
        void* res[6] = {sl->res.out_action, sl->res.out_size, sl->res.out_prev, sl->res.out_flags, sl->res.trade_off,
                        sl->res.trades};
        for (int k = 0; k < NCOL; ++k) {
            if (sl->col[k] && h->e) kme_host_unregister(h->e, sl->col[k]);
            free(sl->col[k]);
        }
        for (int k = 0; k < 6; ++k) {
            if (res[k] && h->e) kme_host_unregister(h->e, res[k]);
            free(res[k]);
        }
    }
    if (h->e) kme_destroy(h->e);
    if (h->m) kme_multi_destroy(h->m);
    free(h->chash);
    free(h);
}

/* page-aligned host memory; registered with the engine (one engine: the epochs' PCIe copies go
   straight from and to it).  A kme_multi reads and writes the slots on the host (split, merge). */
static int alloc_registered(jkme* h, void** p, size_t bytes) {
    *p = aligned(bytes);
    return *p && (!h->e || kme_host_register(h->e, *p, bytes) == KME_OK);
}

/* static native long create(int mode, int maxSymbols, int maxEpoch, long maxResting, int maxTrades,
 *                           int maxAccounts, int flags, int device, int nDevices, long ledgerCapacity)
 * nDevices > 1: symbol shards on devices device .. device + nDevices - 1 (kme_multi: FUNDED, flags 0, or
 * the default EXACT_LEDGER | SERIAL_FALLBACK -- then an unprovable epoch consolidates onto one engine);
 * nDevices < 0: -nDevices shards all on `device` (tests on a one-GPU box). */
JNIEXPORT jlong JNICALL Java_GpuMatchingEngine_create(JNIEnv* env, jclass cls, jint mode, jint maxSymbols,
                                                        jint maxEpoch, jlong maxResting, jint maxTrades,
                                                        jint maxAccounts, jint flags, jint device, jint nDevices,
                                                        jlong ledgerCapacity) {
    (void)cls;
    if (maxEpoch <= 0 || maxTrades <= 0) { throw_state(env, "kme: maxEpoch and maxTrades must be positive"); return 0; }
    if (nDevices == 0 || nDevices > 1024 || nDevices < -1024) { throw_state(env, "kme: nDevices out of range"); return 0; }
    if (ledgerCapacity < 0) { throw_state(env, "kme: ledgerCapacity must not be negative"); return 0; }
    kme_config cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.abi_version = KME_ABI_VERSION;
    cfg.mode = (uint32_t)mode;
    cfg.max_symbols = (uint32_t)maxSymbols;
    cfg.max_accounts = (uint32_t)maxAccounts;
    cfg.max_epoch = (uint32_t)maxEpoch;
    cfg.max_trades = (uint32_t)maxTrades;
    cfg.max_resting = (uint64_t)maxResting;
    /* EXACT Balances / Positions (EXACT mode, or FUNDED with the exact ledger): a Positions entry per
       (account, symbol) ever filled -- fillOrder never removes the entry it reads (KP:283, H2) */
    cfg.ledger_capacity = (uint64_t)ledgerCapacity;
    cfg.device = device;
    cfg.flags = (uint32_t)flags;   /* KME_FLAG_EXACT_LEDGER | KME_FLAG_SERIAL_FALLBACK: the reference's
                                      semantics for any stream, parallel where the funded proof holds */
    jkme* h = (jkme*)calloc(1, sizeof *h);
    if (!h) { throw_state(env, "kme: out of host memory"); return 0; }
    h->max_epoch = (uint32_t)maxEpoch;
    h->max_trades = (uint32_t)maxTrades;
    kme_status s;
    if (nDevices == 1) {
        s = kme_create(&cfg, &h->e);
    } else {
        const int nd = nDevices > 0 ? nDevices : -nDevices;
        int32_t devs[1024];
        for (int k = 0; k < nd; ++k) devs[k] = nDevices > 0 ? device + k : device;
        s = kme_multi_create(&cfg, (uint32_t)nd, devs, &h->m);
    }
    if (s != KME_OK) {
        h->e = NULL;
        h->m = NULL;
        free_handle(h);
        throw_state(env, kme_strerror(s));
        return 0;
    }
    const size_t E = (size_t)maxEpoch, T = (size_t)maxTrades;
    for (int k = 0; k < 2; ++k) {
        jslot* sl = &h->slot[k];
        const size_t cb[NCOL] = {4 * E, 8 * E, 8 * E, 8 * E, 4 * E, 4 * E, sizeof(kme_row) * (2 * E + 2 * T)};
        int ok = 1;
        for (int c = 0; c < NCOL && ok; ++c) {
            sl->bytes[c] = cb[c];
            ok = alloc_registered(h, &sl->col[c], cb[c]);
        }
        kme_epoch_result* r = &sl->res;
        ok = ok && alloc_registered(h, (void**)&r->out_action, 4 * E) && alloc_registered(h, (void**)&r->out_size, 4 * E) &&
             alloc_registered(h, (void**)&r->out_prev, 8 * E) && alloc_registered(h, (void**)&r->out_flags, E) &&
             alloc_registered(h, (void**)&r->trade_off, 4 * (E + 1)) &&
             alloc_registered(h, (void**)&r->trades, sizeof(kme_trade) * T);
        if (!ok) {
            free_handle(h);
            throw_state(env, "kme: cannot allocate or register the slot buffers");
            return 0;
        }
        r->trades_cap = (uint32_t)maxTrades;
        sl->in.action = (const int32_t*)sl->col[0];
        sl->in.oid = (const int64_t*)sl->col[1];
        sl->in.aid = (const int64_t*)sl->col[2];
        sl->in.sid = (const int64_t*)sl->col[3];
        sl->in.price = (const int32_t*)sl->col[4];
        sl->in.size = (const int32_t*)sl->col[5];
        sl->rows = (kme_row*)sl->col[6];
        sl->rows_cap = cb[6] / sizeof(kme_row);
        sl->ready_rows = -1;
    }
    return (jlong)(intptr_t)h;
}

/* static native void destroy(long h) */
JNIEXPORT void JNICALL Java_GpuMatchingEngine_destroy(JNIEnv* env, jclass cls, jlong handle) {
    (void)env; (void)cls;
    free_handle((jkme*)(intptr_t)handle);
}

/* static native ByteBuffer buffer(long h, int slot, int column): the slot's column 0..5 (action, oid,
 * aid, sid, price, size: maxEpoch elements each) or 6 (the MatchOut rows: 2 maxEpoch + 2 maxTrades of
 * 48 bytes), as a direct ByteBuffer over the registered native memory (valid until destroy). */
JNIEXPORT jobject JNICALL Java_GpuMatchingEngine_buffer(JNIEnv* env, jclass cls, jlong handle, jint slot, jint column) {
    (void)cls;
    jkme* h = (jkme*)(intptr_t)handle;
    if (!h || slot < 0 || slot > 1 || column < 0 || column >= NCOL) { throw_state(env, "kme: no such buffer"); return NULL; }
    return (*env)->NewDirectByteBuffer(env, h->slot[slot].col[column], (jlong)h->slot[slot].bytes[column]);
}

/* static native int submit(long h, int slot, int n): the slot's n buffered records as one epoch,
 * asynchronously (at most two epochs in flight); returns a kme_status. */
JNIEXPORT jint JNICALL Java_GpuMatchingEngine_submit(JNIEnv* env, jclass cls, jlong handle, jint slot, jint n) {
    (void)env; (void)cls;
    jkme* h = (jkme*)(intptr_t)handle;
    if (!h || slot < 0 || slot > 1 || n <= 0 || (uint32_t)n > h->max_epoch) return KME_E_INVALID;
    jslot* sl = &h->slot[slot];
    if (sl->n || sl->ready_rows >= 0) return KME_E_INVALID;   /* in flight, or its rows not forwarded yet */
    const kme_status s = h_submit(h, &sl->in, (uint32_t)n, &sl->res);
    if (s == KME_OK) sl->n = (uint32_t)n;
    return s;
}

/* static native int poll(long h): 1 when the oldest epoch in flight is done (complete() will not
 * block) or none is in flight, 0 while it runs, -status on an error. */
JNIEXPORT jint JNICALL Java_GpuMatchingEngine_poll(JNIEnv* env, jclass cls, jlong handle) {
    (void)env; (void)cls;
    jkme* h = (jkme*)(intptr_t)handle;
    if (!h) return -KME_E_INVALID;
    int done = 0;
    const kme_status s = h_poll(h, &done);
    return s == KME_OK ? (jint)done : -(jint)s;
}

/* static native int complete(long h, int slot, long[] status): waits for the slot's epoch (the oldest
 * in flight) and writes the MatchOut rows of the records that took effect into the slot's row buffer.
 * Returns the row count; status[0..3] = kme_status, domain detail, error index, records that took
 * effect.  The rows are ready until forwarded(h, slot). */
JNIEXPORT jint JNICALL Java_GpuMatchingEngine_complete(JNIEnv* env, jclass cls, jlong handle, jint slot,
                                                         jlongArray status) {
    (void)cls;
    jkme* h = (jkme*)(intptr_t)handle;
    if (!h || slot < 0 || slot > 1 || !h->slot[slot].n) { throw_state(env, "kme: no epoch in flight on this slot"); return -1; }
    if (!status || (*env)->GetArrayLength(env, status) < 4) { throw_state(env, "kme: status needs 4 entries"); return -1; }
    jslot* sl = &h->slot[slot];
    kme_epoch_status st;
    memset(&st, 0, sizeof st);
    const kme_status s = h_wait(h, &st);
    const uint32_t n = sl->n;
    sl->n = 0;
    const uint32_t ne = s == KME_OK ? n : (st.n_effective < n ? st.n_effective : n);
    size_t rows = 0;
    const kme_status x = ne ? kme_expand_rows_mt(&sl->in, ne, &sl->res, sl->rows, sl->rows_cap, &rows, 0) : KME_OK;
    jlong stv[4];
    stv[0] = (jlong)(s != KME_OK ? s : x);
    stv[1] = (jlong)(s != KME_OK ? st.detail : (x != KME_OK ? KME_D_CAP_TRADES : 0));
    stv[2] = (jlong)(s != KME_OK ? st.error_index : -1);
    stv[3] = (jlong)(x == KME_OK ? ne : 0);
    (*env)->SetLongArrayRegion(env, status, 0, 4, stv);
    if (x != KME_OK) rows = 0;   /* (cannot happen: the row buffer holds 2 maxEpoch + 2 maxTrades rows) */
    sl->ready_rows = (int64_t)rows;
    sl->ready_seq = ++h->completions;
    return (jint)rows;
}

/* static native void forwarded(long h, int slot): the slot's ready rows have been forwarded. */
JNIEXPORT void JNICALL Java_GpuMatchingEngine_forwarded(JNIEnv* env, jclass cls, jlong handle, jint slot) {
    (void)env; (void)cls;
    jkme* h = (jkme*)(intptr_t)handle;
    if (h && slot >= 0 && slot <= 1) h->slot[slot].ready_rows = -1;
}

/* static native String statusText(int status) */
JNIEXPORT jstring JNICALL Java_GpuMatchingEngine_statusText(JNIEnv* env, jclass cls, jint s) {
    (void)cls;
    return (*env)->NewStringUTF(env, kme_strerror(s));
}

/* the ready slots, oldest completion first */
static int ready_order(const jkme* h, int order[2]) {
    int n = 0;
    for (int s = 0; s < 2; ++s)
        if (h->slot[s].ready_rows >= 0) order[n++] = s;
    if (n == 2 && h->slot[order[0]].ready_seq > h->slot[order[1]].ready_seq) { order[0] = 1; order[1] = 0; }
    return n;
}

/* static native int checkpoint(long h, String path, long offset, long generation, long[] info): the
 * commit point (called from the commit hook's StateStore.flush(), before Kafka Streams commits the
 * consumed offsets): nothing may be in flight.  The file holds the engine state after
 * every record up to `offset` and the MatchOut rows of the ready slots, so a restart loses no output of
 * a committed record; info[0..1] = the file's size and digest. */
JNIEXPORT jint JNICALL Java_GpuMatchingEngine_checkpoint(JNIEnv* env, jclass cls, jlong handle, jstring path,
                                                           jlong offset, jlong generation, jlongArray info) {
    (void)cls;
    jkme* h = (jkme*)(intptr_t)handle;
    if (!h || !path || h->slot[0].n || h->slot[1].n) return KME_E_INVALID;
    if (!info || (*env)->GetArrayLength(env, info) < 2) return KME_E_INVALID;
    int order[2];
    const int nr = ready_order(h, order);
    size_t bytes = sizeof(jrec_head);
    for (int k = 0; k < nr; ++k) bytes += sizeof(jrec_slot) + sizeof(kme_row) * (size_t)h->slot[order[k]].ready_rows;
    char* rec = (char*)malloc(bytes);
    if (!rec) return KME_E_CAPACITY;
    jrec_head hd = {JREC_MAGIC, (uint32_t)nr, (int64_t)offset, (int64_t)generation};
    memcpy(rec, &hd, sizeof hd);
    size_t at = sizeof hd;
    for (int k = 0; k < nr; ++k) {
        const jslot* sl = &h->slot[order[k]];
        jrec_slot rs = {(uint32_t)order[k], 0, (uint64_t)sl->ready_rows};
        memcpy(rec + at, &rs, sizeof rs);
        at += sizeof rs;
        memcpy(rec + at, sl->rows, sizeof(kme_row) * (size_t)sl->ready_rows);
        at += sizeof(kme_row) * (size_t)sl->ready_rows;
    }
    const char* p = (*env)->GetStringUTFChars(env, path, NULL);
    kme_status s = KME_E_INVALID;
    kme_checkpoint_info ci;
    memset(&ci, 0, sizeof ci);
    if (p) {
        s = h_checkpoint(h, p, rec, bytes);
        if (s == KME_OK) s = kme_checkpoint_inspect(p, &ci);
        (*env)->ReleaseStringUTFChars(env, path, p);
    }
    free(rec);
    jlong iv[2] = {(jlong)ci.file_bytes, (jlong)ci.digest};
    (*env)->SetLongArrayRegion(env, info, 0, 2, iv);
    return (jint)s;
}

/* static native int restore(long h, String path, long[] out): a fresh engine takes the state of the
 * checkpoint; out[0] = the last input offset it covers, out[1] = ready slots (rows to forward before
 * anything else), then (slot, rows) per ready slot, oldest first -- their rows are back in the
 * slots' row buffers; out[6..8] = the checkpoint's generation, file size and digest.  A file without
 * the processor's record is refused before the engine is touched.  Returns a kme_status. */
JNIEXPORT jint JNICALL Java_GpuMatchingEngine_restore(JNIEnv* env, jclass cls, jlong handle, jstring path,
                                                        jlongArray out) {
    (void)cls;
    jkme* h = (jkme*)(intptr_t)handle;
    if (!h || !path || !out || (*env)->GetArrayLength(env, out) < 9) return KME_E_INVALID;
    if (h->slot[0].n || h->slot[1].n) return KME_E_INVALID;
    const char* p = (*env)->GetStringUTFChars(env, path, NULL);
    if (!p) return KME_E_INVALID;
    kme_checkpoint_info ci;
    memset(&ci, 0, sizeof ci);
    kme_status s = kme_checkpoint_inspect(p, &ci);
    /* a checkpoint without the processor's record is not this processor's: refused untouched */
    if (s == KME_OK && ci.app_bytes < sizeof(jrec_head)) s = KME_E_INVALID;
    char* rec = NULL;
    size_t bytes = 0;
    if (s == KME_OK) {
        rec = (char*)malloc((size_t)ci.app_bytes);
        s = rec ? h_restore(h, p, rec, (size_t)ci.app_bytes, &bytes) : KME_E_CAPACITY;
    }
    (*env)->ReleaseStringUTFChars(env, path, p);
    jlong o[9] = {-1, 0, 0, 0, 0, 0, 0, 0, 0};
    if (s == KME_OK) {
        jrec_head hd;
        if (bytes < sizeof hd || (memcpy(&hd, rec, sizeof hd), hd.magic != JREC_MAGIC) || hd.n_ready > 2) {
            s = KME_E_INVALID;   /* (the state is restored already: the processor fails on this status) */
        } else {
            o[0] = hd.offset;
            o[6] = hd.generation;
            o[7] = (jlong)ci.file_bytes;
            o[8] = (jlong)ci.digest;
            size_t at = sizeof hd;
            for (uint32_t k = 0; k < hd.n_ready && s == KME_OK; ++k) {
                jrec_slot rs;
                if (at + sizeof rs > bytes) { s = KME_E_INVALID; break; }
                memcpy(&rs, rec + at, sizeof rs);
                at += sizeof rs;
                if (rs.slot > 1 || rs.rows > h->slot[rs.slot].rows_cap || at + sizeof(kme_row) * rs.rows > bytes) {
                    s = KME_E_INVALID;
                    break;
                }
                jslot* sl = &h->slot[rs.slot];
                memcpy(sl->rows, rec + at, sizeof(kme_row) * rs.rows);
                at += sizeof(kme_row) * rs.rows;
                sl->ready_rows = (int64_t)rs.rows;
                sl->ready_seq = ++h->completions;
                o[2 + 2 * k] = rs.slot;
                o[3 + 2 * k] = (jlong)rs.rows;
                o[1] = k + 1;
            }
        }
    }
    free(rec);
    (*env)->SetLongArrayRegion(env, out, 0, 9, o);
    return (jint)s;
}

/* ---- the state changelog: the committed checkpoint file, cut into fixed-size
 * chunks, goes to the processor's changelogged commit store -- only the chunks whose content changed
 * since the last commit (format 4 keeps unchanged stores at unchanged offsets: group states, accounts
 * and the pool prefix first) -- so the state follows the task to any instance, as the reference's
 * changelogged stores do (KP:30-49). */
/* static native int stateChunks(long h, String path, int chunkBytes, long[] hashes, long[] changed): the
 * file at `path` cut into chunks of chunkBytes (the last one shorter): hashes[k] = chunk k's content
 * hash, changed[0..] = the indices of the chunks whose hash differs from what the last call saw (every
 * chunk after create, or when chunkBytes changes), ascending.  Returns the number of chunks n
 * (hashes[0, n)) and writes how many changed into changed[0] ahead of them (changed[1..]); -kme_status
 * on an error (an array too short: -KME_E_CAPACITY, nothing recorded). */
JNIEXPORT jint JNICALL Java_GpuMatchingEngine_stateChunks(JNIEnv* env, jclass cls, jlong handle, jstring path,
                                                            jint chunkBytes, jlongArray hashes, jlongArray changed) {
    (void)cls;
    jkme* h = (jkme*)(intptr_t)handle;
    if (!h || !path || !hashes || !changed || chunkBytes < 4096) return -KME_E_INVALID;
    const jint cap = (*env)->GetArrayLength(env, hashes);
    if ((*env)->GetArrayLength(env, changed) < cap + 1) return -KME_E_CAPACITY;
    const char* p = (*env)->GetStringUTFChars(env, path, NULL);
    if (!p) return -KME_E_INVALID;
    uint64_t* hs = (uint64_t*)malloc((size_t)(cap > 0 ? cap : 1) * sizeof(uint64_t));
    size_t n = 0;
    kme_status s = hs ? kme_checkpoint_chunks(p, (uint32_t)chunkBytes, hs, (size_t)cap, &n) : KME_E_CAPACITY;
    (*env)->ReleaseStringUTFChars(env, path, p);
    jlong* out = s == KME_OK ? (jlong*)malloc((1 + n) * sizeof(jlong)) : NULL;
    if (s == KME_OK && !out) s = KME_E_CAPACITY;
    if (s != KME_OK) { free(hs); return -(jint)s; }
    const int same_cut = h->chash && h->chunk_bytes == chunkBytes;
    jlong nc = 0;
    for (size_t k = 0; k < n; ++k)
        if (!(same_cut && k < h->nchash && h->chash[k] == hs[k])) out[1 + nc++] = (jlong)k;
    out[0] = nc;
    (*env)->SetLongArrayRegion(env, changed, 0, (jsize)(1 + nc), out);
    if (n) (*env)->SetLongArrayRegion(env, hashes, 0, (jsize)n, (const jlong*)hs);
    free(out);
    free(h->chash);
    h->chash = hs;
    h->nchash = n;
    h->chunk_bytes = chunkBytes;
    return (jint)n;
}

/* static native int inspect(String path, long[] out): kme_checkpoint_inspect -- out[0..2] = the file's
 * size, its application record's size and its digest (the trailer only). */
JNIEXPORT jint JNICALL Java_GpuMatchingEngine_inspect(JNIEnv* env, jclass cls, jstring path, jlongArray out) {
    (void)cls;
    if (!path || !out || (*env)->GetArrayLength(env, out) < 3) return KME_E_INVALID;
    const char* p = (*env)->GetStringUTFChars(env, path, NULL);
    if (!p) return KME_E_INVALID;
    kme_checkpoint_info ci;
    memset(&ci, 0, sizeof ci);
    const kme_status s = kme_checkpoint_inspect(p, &ci);
    (*env)->ReleaseStringUTFChars(env, path, p);
    const jlong o[3] = {(jlong)ci.file_bytes, (jlong)ci.app_bytes, (jlong)ci.digest};
    (*env)->SetLongArrayRegion(env, out, 0, 3, o);
    return (jint)s;
}

JNIEXPORT jint JNICALL Java_GpuMatchingEngine_shardStatus(JNIEnv* env, jclass cls, jlong handle, jlongArray out) {
    (void)cls;
    jkme* h = (jkme*)(intptr_t)handle;
    if (!h || !h->m || !out || (*env)->GetArrayLength(env, out) < 8) return KME_E_INVALID;
    kme_multi_status ms;
    memset(&ms, 0, sizeof ms);
    const kme_status s = kme_multi_info(h->m, &ms);
    const jlong o[8] = {(jlong)ms.n_engines, (jlong)ms.consolidated, (jlong)ms.can_consolidate, (jlong)ms.failed,
                        (jlong)ms.history_records, (jlong)ms.history_cap, (jlong)ms.history_saved, (jlong)ms.generation};
    (*env)->SetLongArrayRegion(env, out, 0, 8, o);
    return (jint)s;
}
