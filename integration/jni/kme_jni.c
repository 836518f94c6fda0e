/* kme_jni.c -- JNI glue for GpuMatchingEngine.java, the processor that replaces the reference's
 * MatchingEngine at its topology (KProcessor.java:52, `.addProcessor("MatchingEngine", ...)`).
 *
 * The product path at rate (include/kme.h, "Host epochs at device rate"): the Java side owns two
 * slots of JVM direct ByteBuffers -- the six Order columns of an epoch (structure of arrays, native
 * byte order) and the MatchOut rows that come back -- and this file registers them with the engine
 * once (kme_host_register), so an epoch crosses PCIe straight from and to them: no array pinning, no
 * copies through the JNI boundary, and the garbage collector is never blocked on the GPU.
 *
 *   bind(h, slot, action, oid, aid, sid, price, size, rows)   the slot's buffers (checked, registered)
 *   submit(h, slot, n)        kme_submit_epoch_host: H2D, kernels, D2H queued; returns at once
 *   poll(h)                   kme_poll: 1 when the oldest epoch in flight is done (punctuator)
 *   complete(h, slot, st)     kme_wait + kme_expand_rows_mt into the slot's row buffer, in the
 *                             reference's order: IN (KP:97), maker / taker fill per trade
 *                             (executeTrade, KP:265-274), OUT (KP:124); st[0..3] = status, domain
 *                             detail, error index, records that took effect (kme_epoch_status)
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
#include <stdlib.h>
#include <string.h>

#include "kme.h"

typedef struct jslot {
    kme_orders in;                 /* the slot's direct ByteBuffers (Java writes the records) */
    kme_row* rows;                 /* direct ByteBuffer of MatchOut rows (Java reads them) */
    size_t rows_cap;
    void* regs[7];                 /* what bind() registered */
    kme_epoch_result res;          /* native host results, registered at create() */
    uint32_t n;                    /* records of the epoch in flight (0 = none) */
} jslot;

typedef struct jkme {
    kme_engine* e;
    uint32_t max_epoch, max_trades;
    jslot slot[2];
} jkme;

static void throw_state(JNIEnv* env, const char* msg) {
    jclass c = (*env)->FindClass(env, "java/lang/IllegalStateException");
    if (c) (*env)->ThrowNew(env, c, msg);
}

static void* aligned(size_t bytes) {
    void* p = NULL;
    return posix_memalign(&p, 4096, bytes ? bytes : 1) == 0 ? p : NULL;
}

static void free_handle(jkme* h) {
    if (!h) return;
    for (int s = 0; s < 2; ++s) {
        jslot* sl = &h->slot[s];
        for (int k = 0; k < 7; ++k)
            if (sl->regs[k] && h->e) kme_host_unregister(h->e, sl->regs[k]);
        void* res[6] = {sl->res.out_action, sl->res.out_size, sl->res.out_prev, sl->res.out_flags, sl->res.trade_off,
                        sl->res.trades};
        for (int k = 0; k < 6; ++k) {
            if (res[k] && h->e) kme_host_unregister(h->e, res[k]);
            free(res[k]);
        }
    }
    if (h->e) kme_destroy(h->e);
    free(h);
}

/* static native long create(int mode, int maxSymbols, int maxEpoch, long maxResting, int maxTrades,
 *                           int maxAccounts, int flags, int device) */
JNIEXPORT jlong JNICALL Java_GpuMatchingEngine_create(JNIEnv* env, jclass cls, jint mode, jint maxSymbols,
                                                        jint maxEpoch, jlong maxResting, jint maxTrades,
                                                        jint maxAccounts, jint flags, jint device) {
    (void)cls;
    if (maxEpoch <= 0 || maxTrades <= 0) { throw_state(env, "kme: maxEpoch and maxTrades must be positive"); return 0; }
    kme_config cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.abi_version = KME_ABI_VERSION;
    cfg.mode = (uint32_t)mode;
    cfg.max_symbols = (uint32_t)maxSymbols;
    cfg.max_accounts = (uint32_t)maxAccounts;
    cfg.max_epoch = (uint32_t)maxEpoch;
    cfg.max_trades = (uint32_t)maxTrades;
    cfg.max_resting = (uint64_t)maxResting;
    cfg.ledger_capacity = 1u << 20;
    cfg.device = device;
    cfg.flags = (uint32_t)flags;   /* KME_FLAG_EXACT_LEDGER | KME_FLAG_SERIAL_FALLBACK: the reference's
                                      semantics for any stream, parallel where the funded proof holds */
    jkme* h = (jkme*)calloc(1, sizeof *h);
    if (!h) { throw_state(env, "kme: out of host memory"); return 0; }
    h->max_epoch = (uint32_t)maxEpoch;
    h->max_trades = (uint32_t)maxTrades;
    const kme_status s = kme_create(&cfg, &h->e);
    if (s != KME_OK) {
        h->e = NULL;
        free_handle(h);
        throw_state(env, kme_strerror(s));
        return 0;
    }
    const size_t E = (size_t)maxEpoch;
    for (int k = 0; k < 2; ++k) {
        kme_epoch_result* r = &h->slot[k].res;
        r->out_action = (int32_t*)aligned(sizeof(int32_t) * E);
        r->out_size = (int32_t*)aligned(sizeof(int32_t) * E);
        r->out_prev = (int64_t*)aligned(sizeof(int64_t) * E);
        r->out_flags = (uint8_t*)aligned(E);
        r->trade_off = (uint32_t*)aligned(sizeof(uint32_t) * (E + 1));
        r->trades = (kme_trade*)aligned(sizeof(kme_trade) * (size_t)maxTrades);
        r->trades_cap = (uint32_t)maxTrades;
        const size_t bytes[6] = {4 * E, 4 * E, 8 * E, E, 4 * (E + 1), sizeof(kme_trade) * (size_t)maxTrades};
        void* p[6] = {r->out_action, r->out_size, r->out_prev, r->out_flags, r->trade_off, r->trades};
        for (int q = 0; q < 6; ++q) {
            if (!p[q] || kme_host_register(h->e, p[q], bytes[q]) != KME_OK) {
                free_handle(h);
                throw_state(env, "kme: cannot allocate or register the result buffers");
                return 0;
            }
        }
    }
    return (jlong)(intptr_t)h;
}

/* static native void destroy(long h) */
JNIEXPORT void JNICALL Java_GpuMatchingEngine_destroy(JNIEnv* env, jclass cls, jlong handle) {
    (void)env; (void)cls;
    free_handle((jkme*)(intptr_t)handle);
}

/* static native int bind(long h, int slot, ByteBuffer action, ByteBuffer oid, ByteBuffer aid,
 *                        ByteBuffer sid, ByteBuffer price, ByteBuffer size, ByteBuffer rows)
 * Direct buffers of at least maxEpoch elements each (int / long columns) and rows for
 * 2 maxEpoch + 2 maxTrades MatchOut rows of 48 bytes; returns a kme_status. */
JNIEXPORT jint JNICALL Java_GpuMatchingEngine_bind(JNIEnv* env, jclass cls, jlong handle, jint slot, jobject action,
                                                     jobject oid, jobject aid, jobject sid, jobject price, jobject size,
                                                     jobject rows) {
    (void)cls;
    jkme* h = (jkme*)(intptr_t)handle;
    if (!h || slot < 0 || slot > 1 || h->slot[slot].n) return KME_E_INVALID;
    jslot* sl = &h->slot[slot];
    const size_t E = h->max_epoch;
    jobject bufs[7] = {action, oid, aid, sid, price, size, rows};
    const size_t need[7] = {4 * E, 8 * E, 8 * E, 8 * E, 4 * E, 4 * E,
                            sizeof(kme_row) * (2 * E + 2 * (size_t)h->max_trades)};
    void* addr[7];
    for (int k = 0; k < 7; ++k) {
        if (!bufs[k]) return KME_E_INVALID;
        addr[k] = (*env)->GetDirectBufferAddress(env, bufs[k]);
        const jlong cap = (*env)->GetDirectBufferCapacity(env, bufs[k]);
        if (!addr[k] || cap < 0 || (size_t)cap < need[k] || ((uintptr_t)addr[k] & 7u)) return KME_E_INVALID;
    }
    for (int k = 0; k < 7; ++k) {
        if (sl->regs[k]) { kme_host_unregister(h->e, sl->regs[k]); sl->regs[k] = NULL; }
        const kme_status s = kme_host_register(h->e, addr[k], need[k]);
        if (s != KME_OK) return s;
        sl->regs[k] = addr[k];
    }
    sl->in.action = (const int32_t*)addr[0];
    sl->in.oid = (const int64_t*)addr[1];
    sl->in.aid = (const int64_t*)addr[2];
    sl->in.sid = (const int64_t*)addr[3];
    sl->in.price = (const int32_t*)addr[4];
    sl->in.size = (const int32_t*)addr[5];
    sl->rows = (kme_row*)addr[6];
    sl->rows_cap = need[6] / sizeof(kme_row);
    return KME_OK;
}

/* static native int submit(long h, int slot, int n): the slot's n buffered records as one epoch,
 * asynchronously (at most two epochs in flight); returns a kme_status. */
JNIEXPORT jint JNICALL Java_GpuMatchingEngine_submit(JNIEnv* env, jclass cls, jlong handle, jint slot, jint n) {
    (void)env; (void)cls;
    jkme* h = (jkme*)(intptr_t)handle;
    if (!h || slot < 0 || slot > 1 || n <= 0 || (uint32_t)n > h->max_epoch) return KME_E_INVALID;
    jslot* sl = &h->slot[slot];
    if (sl->n || !sl->rows) return KME_E_INVALID;   /* in flight already, or never bound */
    const kme_status s = kme_submit_epoch_host(h->e, &sl->in, (uint32_t)n, &sl->res);
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
    const kme_status s = kme_poll(h->e, &done);
    return s == KME_OK ? (jint)done : -(jint)s;
}

/* static native int complete(long h, int slot, long[] status): waits for the slot's epoch (the oldest
 * in flight) and writes the MatchOut rows of the records that took effect into the slot's row buffer.
 * Returns the row count; status[0..3] = kme_status, domain detail, error index, records that took
 * effect. */
JNIEXPORT jint JNICALL Java_GpuMatchingEngine_complete(JNIEnv* env, jclass cls, jlong handle, jint slot,
                                                         jlongArray status) {
    (void)cls;
    jkme* h = (jkme*)(intptr_t)handle;
    if (!h || slot < 0 || slot > 1 || !h->slot[slot].n) { throw_state(env, "kme: no epoch in flight on this slot"); return -1; }
    if (!status || (*env)->GetArrayLength(env, status) < 4) { throw_state(env, "kme: status needs 4 entries"); return -1; }
    jslot* sl = &h->slot[slot];
    kme_epoch_status st;
    memset(&st, 0, sizeof st);
    const kme_status s = kme_wait(h->e, &st);
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
    if (x != KME_OK) return 0;   /* (cannot happen: the row buffer holds 2 maxEpoch + 2 maxTrades rows) */
    return (jint)rows;
}

/* static native String statusText(int status) */
JNIEXPORT jstring JNICALL Java_GpuMatchingEngine_statusText(JNIEnv* env, jclass cls, jint s) {
    (void)cls;
    return (*env)->NewStringUTF(env, kme_strerror(s));
}

/* static native int checkpoint(long h, String path) / restore(long h, String path): persistence
 * in place of the RocksDB changelogs (KP:30-49); between epochs (nothing in flight), before commit. */
static jint ckpt(JNIEnv* env, jlong handle, jstring path, int restore) {
    jkme* h = (jkme*)(intptr_t)handle;
    if (!h || !path) return KME_E_INVALID;
    const char* p = (*env)->GetStringUTFChars(env, path, NULL);
    if (!p) return KME_E_INVALID;
    const kme_status s = restore ? kme_restore(h->e, p) : kme_checkpoint(h->e, p);
    (*env)->ReleaseStringUTFChars(env, path, p);
    return (jint)s;
}
JNIEXPORT jint JNICALL Java_GpuMatchingEngine_checkpoint(JNIEnv* env, jclass cls, jlong h, jstring path) {
    (void)cls;
    return ckpt(env, h, path, 0);
}
JNIEXPORT jint JNICALL Java_GpuMatchingEngine_restore(JNIEnv* env, jclass cls, jlong h, jstring path) {
    (void)cls;
    return ckpt(env, h, path, 1);
}
