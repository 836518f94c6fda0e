/* kme_jni.c -- JNI glue for GpuMatchingEngine.java, the processor that replaces the reference's
 * MatchingEngine at its topology (KProcessor.java:52, `.addProcessor("MatchingEngine", ...)`).
 *
 * The Java side buffers input Orders into an epoch (structure of arrays), calls submit(), and
 * forwards the rows this file expands from the epoch result, in the reference's order: for input i
 * the IN echo (KP:97), then the maker fill and the taker fill of each trade (executeTrade,
 * KP:265-274), then the OUT echo (KP:124).  On an error the rows of the records that took effect
 * ([0, n_effective), kme.h kme_epoch_status) are still produced: the reference forwards and commits
 * every record before the one that throws (KP:97, 124-125).
 *
 * Build (JDK present): integration/jni/build.sh.  This container has no JDK; the CPU test suite
 * compiles this file with -fsyntax-only against tests/jni_stub/jni.h (a declaration subset) so that
 * it stays in step with include/kme.h.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "kme.h"

/* Fill record actions (KP:265-274). */
enum { JKME_BOUGHT = 5, JKME_SOLD = 6, JKME_BUY = 2 };

typedef struct jkme {
    kme_engine* e;
    uint32_t max_epoch, max_trades;
    kme_epoch_result res;          /* host result buffers, reused by every submit */
} jkme;

static void throw_state(JNIEnv* env, const char* msg) {
    jclass c = (*env)->FindClass(env, "java/lang/IllegalStateException");
    if (c) (*env)->ThrowNew(env, c, msg);
}

static void free_handle(jkme* h) {
    if (!h) return;
    if (h->e) kme_destroy(h->e);
    free(h->res.out_action);
    free(h->res.out_size);
    free(h->res.out_prev);
    free(h->res.out_flags);
    free(h->res.trade_off);
    free(h->res.trades);
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
    h->res.out_action = (int32_t*)malloc(sizeof(int32_t) * (size_t)maxEpoch);
    h->res.out_size = (int32_t*)malloc(sizeof(int32_t) * (size_t)maxEpoch);
    h->res.out_prev = (int64_t*)malloc(sizeof(int64_t) * (size_t)maxEpoch);
    h->res.out_flags = (uint8_t*)malloc((size_t)maxEpoch);
    h->res.trade_off = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)maxEpoch + 1));
    h->res.trades = (kme_trade*)malloc(sizeof(kme_trade) * (size_t)maxTrades);
    h->res.trades_cap = (uint32_t)maxTrades;
    if (!h->res.out_action || !h->res.out_size || !h->res.out_prev || !h->res.out_flags || !h->res.trade_off ||
        !h->res.trades) {
        free_handle(h);
        throw_state(env, "kme: out of host memory");
        return 0;
    }
    const kme_status s = kme_create(&cfg, &h->e);
    if (s != KME_OK) {
        h->e = NULL;
        free_handle(h);
        throw_state(env, kme_strerror(s));
        return 0;
    }
    return (jlong)(intptr_t)h;
}

/* static native void destroy(long h) */
JNIEXPORT void JNICALL Java_GpuMatchingEngine_destroy(JNIEnv* env, jclass cls, jlong handle) {
    (void)env; (void)cls;
    free_handle((jkme*)(intptr_t)handle);
}

/* static native int submit(long h, int n, int[] action, long[] oid, long[] aid, long[] sid,
 *                          int[] price, int[] size,
 *                          byte[] kind, int[] oAction, long[] oOid, long[] oAid, long[] oSid,
 *                          int[] oPrice, int[] oSize, long[] oPrev, byte[] oHasPrev, long[] status)
 * Runs the n buffered records as one epoch and writes the MatchOut rows (kind 0 = "IN", 1 = fill,
 * 2 = "OUT") of the records that took effect.  Returns the row count; status[0..2] = kme_status,
 * domain detail, error index.  The output arrays need 2 n + 2 maxTrades rows. */
JNIEXPORT jint JNICALL Java_GpuMatchingEngine_submit(JNIEnv* env, jclass cls, jlong handle, jint n,
        jintArray action, jlongArray oid, jlongArray aid, jlongArray sid, jintArray price, jintArray size,
        jbyteArray kind, jintArray oAction, jlongArray oOid, jlongArray oAid, jlongArray oSid,
        jintArray oPrice, jintArray oSize, jlongArray oPrev, jbyteArray oHasPrev, jlongArray status) {
    (void)cls;
    jkme* h = (jkme*)(intptr_t)handle;
    if (!h || n < 0 || (uint32_t)n > h->max_epoch) { throw_state(env, "kme: bad handle or epoch size"); return -1; }
    const jsize rows_cap = (*env)->GetArrayLength(env, kind);
    if ((int64_t)rows_cap < 2 * (int64_t)n) { throw_state(env, "kme: output arrays too small"); return -1; }

    /* inputs: pinned for the duration of the (synchronous) submission */
    kme_orders in;
    int32_t* a = (int32_t*)(*env)->GetPrimitiveArrayCritical(env, action, NULL);
    int64_t* o = (int64_t*)(*env)->GetPrimitiveArrayCritical(env, oid, NULL);
    int64_t* ac = (int64_t*)(*env)->GetPrimitiveArrayCritical(env, aid, NULL);
    int64_t* sd = (int64_t*)(*env)->GetPrimitiveArrayCritical(env, sid, NULL);
    int32_t* pr = (int32_t*)(*env)->GetPrimitiveArrayCritical(env, price, NULL);
    int32_t* sz = (int32_t*)(*env)->GetPrimitiveArrayCritical(env, size, NULL);
    in.action = a; in.oid = o; in.aid = ac; in.sid = sd; in.price = pr; in.size = sz;
    kme_epoch_status st;
    memset(&st, 0, sizeof st);
    const kme_status s = kme_submit_epoch(h->e, &in, (uint32_t)n, &h->res, &st);

    /* rows of the records that took effect */
    const uint32_t ne = s == KME_OK ? (uint32_t)n : st.n_effective;
    jint rows = 0;
    jbyte* k = (jbyte*)(*env)->GetPrimitiveArrayCritical(env, kind, NULL);
    int32_t* ra = (int32_t*)(*env)->GetPrimitiveArrayCritical(env, oAction, NULL);
    int64_t* ro = (int64_t*)(*env)->GetPrimitiveArrayCritical(env, oOid, NULL);
    int64_t* rc = (int64_t*)(*env)->GetPrimitiveArrayCritical(env, oAid, NULL);
    int64_t* rs = (int64_t*)(*env)->GetPrimitiveArrayCritical(env, oSid, NULL);
    int32_t* rp = (int32_t*)(*env)->GetPrimitiveArrayCritical(env, oPrice, NULL);
    int32_t* rz = (int32_t*)(*env)->GetPrimitiveArrayCritical(env, oSize, NULL);
    int64_t* rv = (int64_t*)(*env)->GetPrimitiveArrayCritical(env, oPrev, NULL);
    jbyte* rh = (jbyte*)(*env)->GetPrimitiveArrayCritical(env, oHasPrev, NULL);
    int overflow = 0;
    for (uint32_t i = 0; i < ne && !overflow; ++i) {
        const uint32_t t0 = h->res.trade_off[i], t1 = h->res.trade_off[i + 1];
        if ((int64_t)rows + 2 + 2 * (int64_t)(t1 - t0) > (int64_t)rows_cap) { overflow = 1; break; }
        /* IN: the input unchanged (KP:97) */
        k[rows] = 0; ra[rows] = a[i]; ro[rows] = o[i]; rc[rows] = ac[i]; rs[rows] = sd[i];
        rp[rows] = pr[i]; rz[rows] = sz[i]; rv[rows] = 0; rh[rows] = 0; ++rows;
        const int taker_buy = a[i] == JKME_BUY;
        for (uint32_t t = t0; t < t1; ++t) {
            const kme_trade* tr = &h->res.trades[t];
            /* maker fill: {SOLD|BOUGHT, maker oid/aid/sid, 0, size} */
            k[rows] = 1; ra[rows] = taker_buy ? JKME_SOLD : JKME_BOUGHT; ro[rows] = tr->maker_oid;
            rc[rows] = tr->maker_aid; rs[rows] = tr->maker_sid; rp[rows] = 0; rz[rows] = tr->size;
            rv[rows] = 0; rh[rows] = 0; ++rows;
            /* taker fill: {BOUGHT|SOLD, taker oid/aid/sid, taker.price - maker.price, size} */
            k[rows] = 1; ra[rows] = taker_buy ? JKME_BOUGHT : JKME_SOLD; ro[rows] = o[i]; rc[rows] = ac[i];
            rs[rows] = sd[i]; rp[rows] = (int32_t)((uint32_t)pr[i] - (uint32_t)tr->maker_price);
            rz[rows] = tr->size; rv[rows] = 0; rh[rows] = 0; ++rows;
        }
        /* OUT: the mutated order (KP:124; prev set by addOrder, KP:218) */
        k[rows] = 2; ra[rows] = h->res.out_action[i]; ro[rows] = o[i]; rc[rows] = ac[i]; rs[rows] = sd[i];
        rp[rows] = pr[i]; rz[rows] = h->res.out_size[i];
        rh[rows] = (h->res.out_flags[i] & KME_OUT_HAS_PREV) ? 1 : 0;
        rv[rows] = rh[rows] ? h->res.out_prev[i] : 0;
        ++rows;
    }
    (*env)->ReleasePrimitiveArrayCritical(env, oHasPrev, rh, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, oPrev, rv, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, oSize, rz, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, oPrice, rp, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, oSid, rs, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, oAid, rc, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, oOid, ro, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, oAction, ra, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, kind, k, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, size, sz, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, price, pr, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, sid, sd, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, aid, ac, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, oid, o, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, action, a, JNI_ABORT);

    jlong stv[3];
    stv[0] = (jlong)s;
    stv[1] = (jlong)st.detail;
    stv[2] = (jlong)st.error_index;
    (*env)->SetLongArrayRegion(env, status, 0, 3, stv);
    if (overflow) { throw_state(env, "kme: output arrays too small for the epoch's trades"); return -1; }
    return rows;
}

/* static native String statusText(int status) */
JNIEXPORT jstring JNICALL Java_GpuMatchingEngine_statusText(JNIEnv* env, jclass cls, jint s) {
    (void)cls;
    return (*env)->NewStringUTF(env, kme_strerror(s));
}

/* static native int checkpoint(long h, String path) / restore(long h, String path): persistence
 * in place of the RocksDB changelogs (KP:30-49); call checkpoint after a flush, before commit. */
static jint ckpt(JNIEnv* env, jlong handle, jstring path, int restore) {
    jkme* h = (jkme*)(intptr_t)handle;
    if (!h) return KME_E_INVALID;
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
