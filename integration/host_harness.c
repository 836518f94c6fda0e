/* host_harness.c -- the Java processor's path at rate, timed in C (bench.py `host_path`).
 *
 * GpuMatchingEngine.java + kme_jni.c per epoch, mirrored here without a JVM:
 *   fill     the epoch's records go into the slot's registered input columns (Java's absolute
 *            ByteBuffer puts, one per field and record);
 *   submit   kme_submit_epoch_host: H2D, kernels, D2H queued, returns at once;
 *   complete kme_wait + kme_expand_rows_mt into the slot's registered row buffer (exactly what
 *            Java_GpuMatchingEngine_complete does: up to 16 native threads), then one pass over the
 *            rows on the calling thread (Java's stream thread builds an Order per row from them).
 * Two slots and at most two epochs in flight: the schedule of GpuMatchingEngine.process / flush /
 * completeOldest.  The clock runs from the first fill to the last completed epoch, so the figure is
 * PCIe- and host-inclusive; it is reported beside the device-resident value, never as it.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "kme.h"

typedef struct hslot {
    int32_t *action, *price, *size;
    int64_t *oid, *aid, *sid;
    kme_row* rows;
    size_t rows_cap;
    kme_epoch_result res;
    uint32_t n;
} hslot;

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void* page_alloc(size_t bytes) {
    void* p = NULL;
    return posix_memalign(&p, 4096, bytes ? bytes : 1) == 0 ? p : NULL;
}

/* Stats out: [0] seconds, [1] rows forwarded, [2] fill seconds, [3] complete (wait) seconds,
 * [4] expand + row-read seconds, [5] trades, [6] checksum of the rows read, [7] expand seconds. */
int kme_host_path_run(kme_engine* e, const kme_orders* stream, uint32_t epoch, uint32_t n_epochs, uint32_t max_trades,
                      double* stats) {
    if (!e || !stream || !epoch || !stats) return KME_E_INVALID;
    hslot sl[2];
    memset(sl, 0, sizeof sl);
    int rc = KME_OK;
    const size_t E = epoch;
    for (int s = 0; s < 2 && rc == KME_OK; ++s) {
        hslot* h = &sl[s];
        h->action = (int32_t*)page_alloc(4 * E); h->price = (int32_t*)page_alloc(4 * E); h->size = (int32_t*)page_alloc(4 * E);
        h->oid = (int64_t*)page_alloc(8 * E); h->aid = (int64_t*)page_alloc(8 * E); h->sid = (int64_t*)page_alloc(8 * E);
        h->rows_cap = 2 * E + 2 * (size_t)max_trades;
        h->rows = (kme_row*)page_alloc(sizeof(kme_row) * h->rows_cap);
        h->res.out_action = (int32_t*)page_alloc(4 * E); h->res.out_size = (int32_t*)page_alloc(4 * E);
        h->res.out_prev = (int64_t*)page_alloc(8 * E); h->res.out_flags = (uint8_t*)page_alloc(E);
        h->res.trade_off = (uint32_t*)page_alloc(4 * (E + 1));
        h->res.trades = (kme_trade*)page_alloc(sizeof(kme_trade) * (size_t)max_trades);
        h->res.trades_cap = max_trades;
        void* p[13] = {h->action, h->price, h->size, h->oid, h->aid, h->sid, h->rows, h->res.out_action, h->res.out_size,
                       h->res.out_prev, h->res.out_flags, h->res.trade_off, h->res.trades};
        const size_t b[13] = {4 * E, 4 * E, 4 * E, 8 * E, 8 * E, 8 * E, sizeof(kme_row) * h->rows_cap, 4 * E, 4 * E, 8 * E,
                              E, 4 * (E + 1), sizeof(kme_trade) * (size_t)max_trades};
        for (int k = 0; k < 13 && rc == KME_OK; ++k) {
            if (!p[k]) rc = KME_E_INVALID;
            else {
                memset(p[k], 0, b[k]);   /* first touch outside the clock */
                rc = kme_host_register(e, p[k], b[k]);
            }
        }
    }
    double t_fill = 0, t_wait = 0, t_rows = 0, t_expand = 0, trades = 0;
    uint64_t rows_total = 0, check = 0;
    int inflight = 0, oldest = 0;
    const double t0 = now_s();
    for (uint32_t k = 0; k <= n_epochs && rc == KME_OK; ++k) {
        /* completeOldest: before a slot is refilled (two in flight), and for the tail */
        while (rc == KME_OK && inflight > 0 && (inflight == 2 || k == n_epochs)) {
            hslot* h = &sl[oldest];
            const double a = now_s();
            kme_epoch_status st;
            rc = kme_wait(e, &st);
            const double b = now_s();
            t_wait += b - a;
            if (rc != KME_OK) break;
            const kme_orders in = {h->action, h->oid, h->aid, h->sid, h->price, h->size};
            size_t nr = 0;
            rc = kme_expand_rows_mt(&in, h->n, &h->res, h->rows, h->rows_cap, &nr, 0);
            if (rc != KME_OK) break;
            t_expand += now_s() - b;
            for (size_t q = 0; q < nr; ++q)   /* the JVM reads every row (one Order each) */
                check += (uint64_t)h->rows[q].oid + (uint64_t)h->rows[q].size + h->rows[q].kind;
            t_rows += now_s() - b;
            rows_total += nr;
            trades += st.n_trades;
            h->n = 0;
            oldest ^= 1;
            --inflight;
        }
        if (rc != KME_OK || k == n_epochs) break;
        /* process(): the epoch's records into the free slot's columns, then flush() */
        hslot* h = &sl[k & 1];
        const double a = now_s();
        const size_t base = (size_t)k * E;
        memcpy(h->action, stream->action + base, 4 * E);
        memcpy(h->oid, stream->oid + base, 8 * E);
        memcpy(h->aid, stream->aid + base, 8 * E);
        memcpy(h->sid, stream->sid + base, 8 * E);
        memcpy(h->price, stream->price + base, 4 * E);
        memcpy(h->size, stream->size + base, 4 * E);
        t_fill += now_s() - a;
        const kme_orders in = {h->action, h->oid, h->aid, h->sid, h->price, h->size};
        rc = kme_submit_epoch_host(e, &in, epoch, &h->res);
        if (rc != KME_OK) break;
        h->n = epoch;
        if (inflight == 0) oldest = (int)(k & 1);
        ++inflight;
    }
    const double t1 = now_s();
    while (inflight-- > 0) { kme_epoch_status st; kme_wait(e, &st); }
    for (int s = 0; s < 2; ++s) {
        hslot* h = &sl[s];
        void* p[13] = {h->action, h->price, h->size, h->oid, h->aid, h->sid, h->rows, h->res.out_action, h->res.out_size,
                       h->res.out_prev, h->res.out_flags, h->res.trade_off, h->res.trades};
        for (int k = 0; k < 13; ++k) {
            if (p[k]) kme_host_unregister(e, p[k]);
            free(p[k]);
        }
    }
    stats[0] = t1 - t0;
    stats[1] = (double)rows_total;
    stats[2] = t_fill;
    stats[3] = t_wait;
    stats[4] = t_rows;
    stats[5] = trades;
    stats[6] = (double)(check & ((1ull << 52) - 1));
    stats[7] = t_expand;
    return rc;
}

/* The partition router at rate (kme_router.cpp, the front of kme_multi / GpuMatchingEngine with
 * nDevices > 1), timed here in C: n_epochs epochs of `epoch` records of `stream` into `parts`
 * partitions through one router (the oid directory carries over), alternately kme_router_route and
 * kme_router_split into buffers made and touched before the clock.  Host-only work.
 * Stats out: [0] route records/s (best epoch), [1] split records/s (best epoch), [2] directory size. */
int kme_router_rate_run(const kme_orders* stream, uint32_t epoch, uint32_t n_epochs, uint32_t parts, double* stats) {
    if (!stream || !epoch || !parts || parts > 64 || !stats) return KME_E_INVALID;
    kme_router* r = NULL;
    int rc = kme_router_create(parts, (uint64_t)epoch * n_epochs, &r);
    if (rc != KME_OK) return rc;
    const size_t E = epoch;
    int32_t* dest = (int32_t*)page_alloc(4 * E);
    kme_orders_buf bufs[64];
    uint8_t* echo[64];
    uint32_t* index[64];
    uint32_t counts[64];
    memset(bufs, 0, sizeof bufs);
    memset(echo, 0, sizeof echo);
    memset(index, 0, sizeof index);
    int ok = dest != NULL;
    for (uint32_t k = 0; k < parts && ok; ++k) {
        bufs[k].action = (int32_t*)page_alloc(4 * E); bufs[k].price = (int32_t*)page_alloc(4 * E);
        bufs[k].size = (int32_t*)page_alloc(4 * E);
        bufs[k].oid = (int64_t*)page_alloc(8 * E); bufs[k].aid = (int64_t*)page_alloc(8 * E);
        bufs[k].sid = (int64_t*)page_alloc(8 * E);
        echo[k] = (uint8_t*)page_alloc(E); index[k] = (uint32_t*)page_alloc(4 * E);
        ok = bufs[k].action && bufs[k].price && bufs[k].size && bufs[k].oid && bufs[k].aid && bufs[k].sid && echo[k] && index[k];
        if (ok) {   /* first touch outside the clock */
            memset(bufs[k].action, 0, 4 * E); memset(bufs[k].price, 0, 4 * E); memset(bufs[k].size, 0, 4 * E);
            memset(bufs[k].oid, 0, 8 * E); memset(bufs[k].aid, 0, 8 * E); memset(bufs[k].sid, 0, 8 * E);
            memset(echo[k], 0, E); memset(index[k], 0, 4 * E);
        }
    }
    if (ok) memset(dest, 0, 4 * E);
    double best_route = 0, best_split = 0;
    for (uint32_t ep = 0; ep < n_epochs && ok && rc == KME_OK; ++ep) {
        const size_t b = (size_t)ep * E;
        const kme_orders in = {stream->action + b, stream->oid + b, stream->aid + b, stream->sid + b, stream->price + b,
                               stream->size + b};
        const double t0 = now_s();
        if (ep % 2 == 0) rc = kme_router_route(r, &in, epoch, dest);
        else rc = kme_router_split(r, &in, epoch, bufs, counts, echo, index);
        const double rate = (double)E / (now_s() - t0);
        if (ep % 2 == 0) { if (rate > best_route) best_route = rate; }
        else if (rate > best_split) best_split = rate;
    }
    stats[0] = best_route;
    stats[1] = best_split;
    stats[2] = (double)kme_router_directory_size(r);
    for (uint32_t k = 0; k < parts; ++k) {
        free(bufs[k].action); free(bufs[k].price); free(bufs[k].size);
        free(bufs[k].oid); free(bufs[k].aid); free(bufs[k].sid); free(echo[k]); free(index[k]);
    }
    free(dest);
    kme_router_destroy(r);
    return ok ? rc : KME_E_INVALID;
}
