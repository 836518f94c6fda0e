// kme_multi.cpp -- one MatchIn stream over N engines (symbol shards), behind the same host-epoch
// calls as one engine: the drop-in's multi-GPU path (include/kme.h "Multi-GPU drop-in").
//
// The reference runs one processor over a one-partition MatchIn (topic.js:17-18,
// exchange_test.js:14-16; KP:51-52).  Books of different symbols never interact, so an epoch is split
// by the C router (kme_router_split: Kafka's keyed partitioner over |sid|, cancels to their order's
// partition, account records to every partition with 1/N of the credit each), each part goes to its
// engine as a host epoch (device k of the list, credit_shards = N), and the results come back merged
// into input order through the router's index -- the caller sees one epoch's kme_epoch_result,
// exactly what one engine over the whole stream returns.  Between epochs the engines' funded credit
// is pooled and split again (kme_credit_state / kme_credit_adjust), queued on the
// engine streams behind the epochs in flight, the blocks moved between devices by peer copies.
//
// Outside the funded domain the symbols cannot be split exactly (the ledger couples every symbol,
// KP:167-182, 276-287; SURVEY §8e: "replicas only").  With cfg.flags = EXACT_LEDGER | SERIAL_FALLBACK
// (the drop-in's default) the first epoch some shard cannot prove is not fatal: the shards are
// retired and ONE engine of those flags (the consolidated engine, on devices[0]) takes the stream --
// built by replaying the input history kept since the start into it, then answering the records the
// shards did not, and every epoch after (consolidate()).  The history survives restarts: every
// checkpoint appends the records since the last one to `path`.hist (fsync'd before the manifest that
// names its length and digest is committed), and a restore reads it back (kme_multi_info reports
// whether consolidation is still possible, and a loss of the history is logged once on stderr).
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "kme.h"
#include "kme_internal.h"

namespace {

void* page_alloc(size_t bytes) {
    void* p = nullptr;
    if (posix_memalign(&p, 4096, std::max<size_t>((bytes + 4095) & ~(size_t)4095, 4096)) != 0) return nullptr;
    std::memset(p, 0, std::max<size_t>(bytes, 1));
    return p;
}

// One shard's part of one epoch slot: its records (router output), which of them it answers and
// their input indices, and its results.
struct Part {
    kme_orders_buf in{};
    uint8_t* echo = nullptr;
    uint32_t* index = nullptr;
    kme_epoch_result res{};
    uint32_t count = 0;
    std::vector<void*> mem;
};

enum : int { kSlotIdle = 0, kSlotQueued, kSlotCollected, kSlotDone };

constexpr char kMultiMagic2[8] = {'K', 'M', 'E', 'M', 'U', 'L', 'T', '2'};
constexpr char kMultiMagic[8] = {'K', 'M', 'E', 'M', 'U', 'L', 'T', '3'};
// the manifest: this header, n shard records (the digest and size of each shard's file: the
// manifest's own digest covers them), the application record, the trailer (kme_internal.h).
// Format 3 adds the input history's length and digest (`path`.hist: HistRec records, appended at
// each checkpoint; 0 records: no history, consolidation is off); format-2 manifests restore as 0.
struct MultiHeader2 {
    char magic[8];
    uint32_t n, _pad;
    uint64_t generation;
    uint64_t app_bytes;
};
struct MultiHeader {
    char magic[8];
    uint32_t n, _pad;
    uint64_t generation;
    uint64_t app_bytes;
    uint64_t hist_records, hist_digest;
};
// one record of `path`.hist (the Order fields of one input record, in input order)
struct HistRec {
    int64_t oid, aid, sid;
    int32_t action, price, size, _pad;
};
static_assert(sizeof(HistRec) == 40, "history record");
struct MultiShard {
    uint64_t file_bytes, digest;
};

}  // namespace

struct kme_multi {
    kme_config cfg{};                      // per engine (credit_shards = n)
    uint32_t n = 0;
    std::vector<kme_engine*> eng;
    std::vector<int> dev;
    kme_router* router = nullptr;
    std::vector<Part> part[2];             // per slot, per shard
    uint32_t slot_n[2] = {};
    kme_epoch_result slot_out[2] = {};
    int slot_mode[2] = {};                 // kSlot*: the slot's epoch is queued on the shards, collected, or done
    std::vector<kme_epoch_status> sst[2];  // per slot: the shards' statuses once collected
    kme_epoch_status done[2] = {};         // per slot: the merged status of an epoch that ran at submit
    int inflight = 0;
    uint32_t sub_count = 0;
    int failed = 0;
    // credit re-splitting: per engine n blocks of (bound, demand) on its device
    std::vector<int64_t*> d_credit;
    std::vector<hipEvent_t> ev_state, ev_copied;
    bool credit_used = false;
    uint32_t rebalance_every = 1, since_rebalance = 0;
    uint64_t generation = 0;               // checkpoint generation (shard files path.g<gen>.<k>)
    // consolidation (cfg.flags EXACT_LEDGER | SERIAL_FALLBACK at n > 1)
    bool can_consolidate = false;
    kme_config cons_cfg{};                 // the consolidated engine's configuration
    kme_engine* cons = nullptr;            // set once the shards are retired
    std::vector<int32_t> h_action, h_price, h_size;   // every record submitted since the start (SoA)
    std::vector<int64_t> h_oid, h_aid, h_sid;
    bool hist_valid = false;               // the history starts at the stream's start and is complete
    uint64_t hist_cap = 0;                 // records it may hold (env KME_MULTI_HISTORY)
    uint64_t hist_start[2] = {};           // per slot: the history position of its epoch's first record
    std::string hist_file;                 // the file the history was last appended to ("": none yet)
    uint64_t hist_saved = 0;               // records of the history in hist_file (fsync'd)
    kme::Digest hist_dg;                   // over those records' bytes
    bool hist_lost_logged = false;
    kme_epoch_result scratch{};            // host results of one consolidated run
    std::vector<char> scratch_mem;
};

static void free_parts(kme_multi* m) {
    for (auto& slot : m->part)
        for (size_t k = 0; k < slot.size(); ++k) {
            for (void* p : slot[k].mem) {
                if (k < m->eng.size() && m->eng[k]) (void)kme_host_unregister(m->eng[k], p);
                std::free(p);
            }
            slot[k].mem.clear();
        }
}

extern "C" {

kme_status kme_multi_destroy(kme_multi* m) {
    if (!m) return KME_E_INVALID;
    for (uint32_t k = 0; k < m->eng.size(); ++k) {   // queued epochs land before their buffers go
        if (!m->eng[k]) continue;
        kme_epoch_status st;
        for (int q = 0; q < m->inflight; ++q) (void)kme_wait(m->eng[k], &st);
    }
    free_parts(m);
    for (size_t k = 0; k < m->d_credit.size(); ++k) {
        (void)hipSetDevice(m->dev[k]);
        if (m->d_credit[k]) (void)hipFree(m->d_credit[k]);
        if (m->ev_state[k]) (void)hipEventDestroy(m->ev_state[k]);
        if (m->ev_copied[k]) (void)hipEventDestroy(m->ev_copied[k]);
    }
    for (kme_engine* e : m->eng)
        if (e) kme_destroy(e);
    if (m->cons) kme_destroy(m->cons);
    if (m->router) kme_router_destroy(m->router);
    delete m;
    return KME_OK;
}

kme_status kme_multi_create(const kme_config* cfg, uint32_t n, const int32_t* devices, kme_multi** out) {
    if (!cfg || !out || n == 0 || n > 1024 || !devices) return KME_E_INVALID;
    // shards prove their orders against their share of each account's credit: FUNDED, no exact ledger
    // (it couples every symbol, kme_create refuses it with credit_shards > 1)
    // flags 0, or (n > 1) EXACT_LEDGER | SERIAL_FALLBACK: the shards prove their epochs as with flags 0,
    // and an epoch they cannot prove consolidates the stream onto one engine of those flags
    const uint32_t both = KME_FLAG_EXACT_LEDGER | KME_FLAG_SERIAL_FALLBACK;
    if (cfg->mode != KME_MODE_FUNDED || (n > 1 && cfg->flags != 0 && cfg->flags != both)) return KME_E_INVALID;
    kme_multi* m = new kme_multi();
    m->cfg = *cfg;
    m->cfg.credit_shards = n;
    m->n = n;
    if (n > 1 && cfg->flags == both) {
        m->can_consolidate = true;
        // the shards refuse what only a serial engine takes (a record outside the funded domain, a sparse
        // symbol) as unproven, so that it consolidates too instead of faulting
        m->cfg.flags = KME_FLAG_REFUSE_SERIAL;
        m->cons_cfg = *cfg;
        m->cons_cfg.credit_shards = 1;
        m->cons_cfg.device = devices[0];
        m->hist_valid = true;
        m->hist_cap = 1ull << 25;
        if (const char* v = std::getenv("KME_MULTI_HISTORY")) m->hist_cap = (uint64_t)std::strtoull(v, nullptr, 10);
    }
    if (const char* v = std::getenv("KME_MULTI_REBALANCE_EVERY")) m->rebalance_every = (uint32_t)std::max(0, std::atoi(v));
    kme_status s = kme_router_create(n, (uint64_t)cfg->max_resting + cfg->max_epoch, &m->router);
    for (uint32_t k = 0; k < n && s == KME_OK; ++k) {
        kme_config c = m->cfg;
        c.device = devices[k];
        kme_engine* e = nullptr;
        s = kme_create(&c, &e);
        m->eng.push_back(e);
        m->dev.push_back(devices[k]);
    }
    const size_t E = cfg->max_epoch, T = cfg->max_trades;
    for (int slot = 0; slot < 2 && s == KME_OK; ++slot) {
        m->part[slot].resize(n);
        m->sst[slot].resize(n);
        for (uint32_t k = 0; k < n && s == KME_OK; ++k) {
            Part& p = m->part[slot][k];
            auto get = [&](size_t bytes) -> void* {
                void* q = page_alloc(bytes);
                if (!q) { s = KME_E_CAPACITY; return nullptr; }
                p.mem.push_back(q);
                if (kme_host_register(m->eng[k], q, bytes) != KME_OK) s = KME_E_HIP;
                return q;
            };
            p.in.action = (int32_t*)get(4 * E); p.in.oid = (int64_t*)get(8 * E); p.in.aid = (int64_t*)get(8 * E);
            p.in.sid = (int64_t*)get(8 * E); p.in.price = (int32_t*)get(4 * E); p.in.size = (int32_t*)get(4 * E);
            p.echo = (uint8_t*)get(E);
            p.index = (uint32_t*)get(4 * E);
            p.res.out_action = (int32_t*)get(4 * E); p.res.out_size = (int32_t*)get(4 * E);
            p.res.out_prev = (int64_t*)get(8 * E); p.res.out_flags = (uint8_t*)get(E);
            p.res.trade_off = (uint32_t*)get(4 * (E + 1));
            p.res.trades = (kme_trade*)get(sizeof(kme_trade) * T);
            p.res.trades_cap = (uint32_t)T;
        }
    }
    if (s == KME_OK && n > 1) {
        const size_t A = cfg->max_accounts;
        for (uint32_t k = 0; k < n && s == KME_OK; ++k) {
            int64_t* d = nullptr;
            hipEvent_t a = nullptr, b = nullptr;
            if (hipSetDevice(m->dev[k]) != hipSuccess || hipMalloc((void**)&d, (size_t)n * 2 * A * sizeof(int64_t)) != hipSuccess ||
                hipEventCreateWithFlags(&a, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&b, hipEventDisableTiming) != hipSuccess)
                s = KME_E_HIP;
            m->d_credit.push_back(d);
            m->ev_state.push_back(a);
            m->ev_copied.push_back(b);
        }
    }
    if (s != KME_OK) {
        kme_multi_destroy(m);
        return s;
    }
    *out = m;
    return KME_OK;
}

}  // extern "C"

// The pooled credit split again over the shards, queued behind every engine's epochs in flight and
// before the next epoch: each engine's (bound, demand) block after its last epoch, copied to every
// other engine's device, then each engine's adjust (every engine computes the same split).
static kme_status rebalance_enqueue(kme_multi* m) {
    const uint32_t n = m->n;
    const size_t A = m->cfg.max_accounts, blk = 2 * A;
    for (uint32_t k = 0; k < n; ++k) {
        hipStream_t st = kme::engine_stream(m->eng[k]);
        if (hipSetDevice(m->dev[k]) != hipSuccess) return KME_E_HIP;
        if (m->credit_used)   // the last round's copies out of this block have been made
            for (uint32_t j = 0; j < n; ++j)
                if (j != k && hipStreamWaitEvent(st, m->ev_copied[j], 0) != hipSuccess) return KME_E_HIP;
        if (kme_status s = kme::credit_state_enqueue(m->eng[k], m->d_credit[k] + k * blk)) return s;
        if (hipEventRecord(m->ev_state[k], st) != hipSuccess) return KME_E_HIP;
    }
    for (uint32_t j = 0; j < n; ++j) {
        hipStream_t st = kme::engine_stream(m->eng[j]);
        if (hipSetDevice(m->dev[j]) != hipSuccess) return KME_E_HIP;
        for (uint32_t k = 0; k < n; ++k) {
            if (k == j) continue;
            if (hipStreamWaitEvent(st, m->ev_state[k], 0) != hipSuccess ||
                hipMemcpyPeerAsync(m->d_credit[j] + k * blk, m->dev[j], m->d_credit[k] + k * blk, m->dev[k],
                                   blk * sizeof(int64_t), st) != hipSuccess)
                return KME_E_HIP;
        }
        if (kme_status s = kme::credit_adjust_enqueue(m->eng[j], m->d_credit[j], n, j, blk)) return s;
        if (hipEventRecord(m->ev_copied[j], st) != hipSuccess) return KME_E_HIP;
    }
    m->credit_used = true;
    return KME_OK;
}

// Routes records [a, a + n) of the caller's epoch to the shards (slot's part buffers) and queues
// every shard's part as a host epoch.
static kme_status split_submit(kme_multi* m, int slot, const kme_orders* in, uint32_t a, uint32_t n) {
    std::vector<Part>& parts = m->part[slot];
    std::vector<kme_orders_buf> bufs(m->n);
    std::vector<uint32_t> counts(m->n);
    std::vector<uint8_t*> echo(m->n);
    std::vector<uint32_t*> index(m->n);
    for (uint32_t k = 0; k < m->n; ++k) {
        bufs[k] = parts[k].in;
        echo[k] = parts[k].echo;
        index[k] = parts[k].index;
    }
    const kme_orders sub{in->action + a, in->oid + a, in->aid + a, in->sid + a, in->price + a, in->size + a};
    kme_status s = kme_router_split(m->router, &sub, n, bufs.data(), counts.data(), echo.data(), index.data());
    if (s != KME_OK) return s;
    // (a part is a subset of the epoch: it fits max_epoch)
    for (uint32_t k = 0; k < m->n; ++k) {
        Part& p = parts[k];
        p.count = counts[k];
        const kme_orders pin{p.in.action, p.in.oid, p.in.aid, p.in.sid, p.in.price, p.in.size};
        s = kme_submit_epoch_host(m->eng[k], &pin, p.count, &p.res);
        if (s != KME_OK) {   // the shards before k hold a part of this epoch: nothing consistent remains
            m->failed = 1;
            // their parts land before anything can free the slot's buffers (kme_multi_destroy waits only
            // for the epochs counted in flight)
            kme_epoch_status st;
            for (uint32_t j = 0; j < k; ++j) (void)kme_wait(m->eng[j], &st);
            return s;
        }
    }
    return KME_OK;
}

// Every shard's part of the slot's epoch completed (kme_wait, oldest first on each engine).
static void collect(kme_multi* m, int slot) {
    for (uint32_t k = 0; k < m->n; ++k) (void)kme_wait(m->eng[k], &m->sst[slot][k]);
    m->slot_mode[slot] = kSlotCollected;
}

// The shards' results of records [a, a + n) merged into the caller's arrays at record a and trade
// `tbase` (out->trade_off[a] == tbase already); the status is relative to record a.
static kme_epoch_status merge(kme_multi* m, int slot, uint32_t n, const kme_epoch_result& out, uint32_t a, uint32_t tbase) {
    std::vector<Part>& parts = m->part[slot];
    const std::vector<kme_epoch_status>& sst = m->sst[slot];
    kme_epoch_status tot{};
    tot.error_index = -1;
    // the first record (input order) a shard did not answer: its fault, or everything after a refusal
    uint32_t limit = n;
    int32_t lim_status = KME_OK, lim_detail = 0;
    int64_t lim_index = -1;
    for (uint32_t k = 0; k < m->n; ++k) {
        const kme_epoch_status& s = sst[k];
        tot.serial_fallback += s.serial_fallback;
        if (s.status == KME_OK) continue;
        const uint32_t ne = std::min(s.n_effective, parts[k].count);
        const uint32_t at = ne < parts[k].count ? parts[k].index[ne] : n;
        if (at < limit || (at == limit && lim_status == KME_OK)) {
            limit = at;
            lim_status = s.status;
            lim_detail = s.detail;
            lim_index = s.error_index >= 0 && (uint64_t)s.error_index < parts[k].count ? (int64_t)parts[k].index[s.error_index] : -1;
        }
    }
    // OUT echoes and per-record trade counts (trade_off[a + i + 1] for now), each shard on its own thread
    auto scatter = [&](uint32_t k) {
        const Part& p = parts[k];
        const uint32_t* to = p.res.trade_off;
        for (uint32_t j = 0; j < p.count; ++j) {
            if (!p.echo[j]) continue;
            const uint32_t i = p.index[j];
            if (i >= limit) break;
            out.out_action[a + i] = p.res.out_action[j];
            out.out_size[a + i] = p.res.out_size[j];
            out.out_prev[a + i] = p.res.out_prev[j];
            out.out_flags[a + i] = p.res.out_flags[j];
            out.trade_off[a + i + 1] = to[j + 1] - to[j];
        }
    };
    std::vector<std::thread> th;
    for (uint32_t k = 1; k < m->n; ++k) th.emplace_back(scatter, k);
    scatter(0);
    for (auto& t : th) t.join();
    th.clear();
    uint64_t acc = 0;
    for (uint32_t i = 0; i < limit; ++i) {
        acc += out.trade_off[a + i + 1];
        if (tbase + acc > out.trades_cap) {   // the merged epoch's trades do not fit: its prefix that does
            limit = i;
            lim_status = KME_E_CAPACITY;
            lim_detail = KME_D_CAP_TRADES;
            lim_index = i;
            acc -= out.trade_off[a + i + 1];
            break;
        }
        out.trade_off[a + i + 1] = (uint32_t)(tbase + acc);
    }
    auto gather = [&](uint32_t k) {
        const Part& p = parts[k];
        const uint32_t* to = p.res.trade_off;
        for (uint32_t j = 0; j < p.count; ++j) {
            if (!p.echo[j]) continue;
            const uint32_t i = p.index[j];
            if (i >= limit) break;
            const uint32_t c = to[j + 1] - to[j];
            if (c) std::memcpy(out.trades + out.trade_off[a + i], p.res.trades + to[j], (size_t)c * sizeof(kme_trade));
        }
    };
    for (uint32_t k = 1; k < m->n; ++k) th.emplace_back(gather, k);
    gather(0);
    for (auto& t : th) t.join();
    for (uint32_t k = 0; k < m->n; ++k) {
        const Part& p = parts[k];
        for (uint32_t j = 0; j < p.count; ++j) {   // counted once: partition 0 answers account records
            if (!p.echo[j] || p.index[j] >= limit) continue;
            const int32_t act = p.in.action[j];
            tot.n_orders += (act == KME_BUY || act == KME_SELL || act == KME_CANCEL) ? 1 : 0;
        }
        if (sst[k].status == KME_OK) {
            tot.n_rests += sst[k].n_rests;
            tot.n_cancel_ok += sst[k].n_cancel_ok;
        }
    }
    tot.n_inputs = n;
    tot.n_trades = (uint32_t)acc;
    tot.n_maker_visits = acc;
    tot.n_effective = limit;
    tot.status = lim_status;
    tot.detail = lim_detail;
    tot.error_index = lim_status == KME_OK ? -1 : lim_index;
    return tot;
}

// ------------------------------------------------------------------ consolidation
static void hist_clear(kme_multi* m) {
    m->hist_valid = false;
    std::vector<int32_t>().swap(m->h_action); std::vector<int32_t>().swap(m->h_price); std::vector<int32_t>().swap(m->h_size);
    std::vector<int64_t>().swap(m->h_oid); std::vector<int64_t>().swap(m->h_aid); std::vector<int64_t>().swap(m->h_sid);
}
// the history is gone while the shards still run: an unprovable epoch is fatal from here on (once on stderr)
static void hist_lost(kme_multi* m, const char* why) {
    hist_clear(m);
    if (m->can_consolidate && !m->cons && !m->hist_lost_logged) {
        std::fprintf(stderr, "kme_multi: input history %s: an epoch the shards cannot prove is fatal from here on "
                             "(KME_E_UNFUNDED)\n", why);
        m->hist_lost_logged = true;
    }
}
static void hist_append(kme_multi* m, const kme_orders* in, uint32_t n) {
    if (!m->hist_valid) return;
    if (m->h_action.size() + n > m->hist_cap) {   // too long to replay: consolidation is off from here on
        hist_lost(m, "past KME_MULTI_HISTORY records");
        return;
    }
    try {   // (up to KME_MULTI_HISTORY records of 40 B on the host: no exception may leave the C ABI)
        m->h_action.insert(m->h_action.end(), in->action, in->action + n);
        m->h_oid.insert(m->h_oid.end(), in->oid, in->oid + n);
        m->h_aid.insert(m->h_aid.end(), in->aid, in->aid + n);
        m->h_sid.insert(m->h_sid.end(), in->sid, in->sid + n);
        m->h_price.insert(m->h_price.end(), in->price, in->price + n);
        m->h_size.insert(m->h_size.end(), in->size, in->size + n);
    } catch (const std::bad_alloc&) {
        hist_lost(m, "out of host memory");
    }
}
static kme_orders hist_at(const kme_multi* m, uint64_t a) {
    return kme_orders{m->h_action.data() + a, m->h_oid.data() + a, m->h_aid.data() + a, m->h_sid.data() + a,
                      m->h_price.data() + a, m->h_size.data() + a};
}

// Records in[0, n) on the consolidated engine (kme_submit_epoch: synchronous, split at max_epoch and
// at account records), their results into `out` from record a and trade out->trade_off[a] on (out may
// be null: a replay, results dropped).  *st: totals; status of the first fault (records before it
// answered, n_effective relative to in).
static kme_status cons_run(kme_multi* m, const kme_orders& in, uint32_t n, const kme_epoch_result* out, uint32_t a,
                           kme_epoch_status* st) {
    kme_epoch_status tot{};
    tot.error_index = -1;
    tot.n_inputs = n;
    uint32_t tbase = out ? out->trade_off[a] : 0;
    const uint32_t E = m->cons_cfg.max_epoch;
    const kme_epoch_result& r = m->scratch;
    for (uint32_t b = 0; b < n || (n == 0 && b == 0); b += E) {
        const uint32_t k = std::min(E, n - b);
        const kme_orders part{in.action + b, in.oid + b, in.aid + b, in.sid + b, in.price + b, in.size + b};
        kme_epoch_status es{};
        const kme_status rc = kme_submit_epoch(m->cons, &part, k, const_cast<kme_epoch_result*>(&r), &es);
        const uint32_t ne = rc == KME_OK ? k : es.n_effective;
        const uint32_t nt = r.trade_off[ne];
        if (out) {
            if (tbase + (uint64_t)nt > out->trades_cap) {   // the merged epoch's trades must fit one engine's buffer
                tot.status = KME_E_CAPACITY; tot.detail = KME_D_CAP_TRADES; tot.error_index = b;
                tot.n_effective = b;
                break;
            }
            std::memcpy(out->out_action + a + b, r.out_action, ne * sizeof(int32_t));
            std::memcpy(out->out_size + a + b, r.out_size, ne * sizeof(int32_t));
            std::memcpy(out->out_prev + a + b, r.out_prev, ne * sizeof(int64_t));
            std::memcpy(out->out_flags + a + b, r.out_flags, ne);
            for (uint32_t q = 1; q <= ne; ++q) out->trade_off[a + b + q] = tbase + r.trade_off[q];
            if (nt) std::memcpy(out->trades + tbase, r.trades, (size_t)nt * sizeof(kme_trade));
        }
        tbase += nt;
        tot.n_trades += nt;
        tot.n_maker_visits += nt;
        tot.n_orders += es.n_orders; tot.n_rests += es.n_rests; tot.n_cancel_ok += es.n_cancel_ok;
        tot.serial_fallback += es.serial_fallback; tot.ledger_repaired += es.ledger_repaired; tot.ledger_serial += es.ledger_serial;
        if (rc != KME_OK) {
            tot.status = es.status; tot.detail = es.detail;
            tot.error_index = es.error_index >= 0 ? b + es.error_index : -1;
            tot.n_effective = b + ne;
            break;
        }
        tot.n_effective = b + k;
        if (n == 0) break;
    }
    if (st) *st = tot;
    return (kme_status)tot.status;
}

// The shards are retired: one engine of cons_cfg (exact ledger + serial fallback) takes the stream
// from history record `upto` on, after replaying [0, upto) into it -- the state the reference holds
// after those records, whatever the shards' funded bounds could prove.  Every shard epoch must have
// landed (nothing in flight on them).
// the host results of one consolidated run (one max_epoch sub-epoch of kme_submit_epoch)
static void alloc_scratch(kme_multi* m) {
    if (!m->scratch_mem.empty()) return;
    const size_t E = m->cons_cfg.max_epoch, T = m->cons_cfg.max_trades;
    m->scratch_mem.assign(E * (4 + 4 + 8 + 1) + 4 * (E + 1) + T * sizeof(kme_trade) + 64, 0);
    char* q = m->scratch_mem.data();
    auto take = [&](size_t bytes) { char* r = q; q += (bytes + 7) & ~(size_t)7; return r; };
    m->scratch.out_action = (int32_t*)take(4 * E);
    m->scratch.out_size = (int32_t*)take(4 * E);
    m->scratch.out_prev = (int64_t*)take(8 * E);
    m->scratch.out_flags = (uint8_t*)take(E);
    m->scratch.trade_off = (uint32_t*)take(4 * (E + 1));
    m->scratch.trades = (kme_trade*)take(T * sizeof(kme_trade));
    m->scratch.trades_cap = (uint32_t)T;
}

static kme_status consolidate(kme_multi* m, uint64_t upto) {
    alloc_scratch(m);
    // the shards go first (their memory, and their registrations of the part buffers)
    free_parts(m);
    for (kme_engine*& e : m->eng) {
        if (e) kme_destroy(e);
        e = nullptr;
    }
    if (kme_status s = kme_create(&m->cons_cfg, &m->cons)) { m->cons = nullptr; return s; }
    kme_epoch_status st{};
    const kme_status rc = cons_run(m, hist_at(m, 0), (uint32_t)upto, nullptr, 0, &st);
    if (rc != KME_OK) return rc;   // (the history took effect once already: it cannot fault now)
    hist_clear(m);                 // not needed any more
    return KME_OK;
}

// A refused epoch (`tot`, records [0, tot.n_effective) of slot s's epoch answered in its out): when
// the history allows it, consolidate and answer the rest of that epoch, and re-run the newer epoch
// (slot s ^ 1) if it was queued on the shards (their results of it are dropped).  Returns false when
// consolidation is not possible (the refusal stands).
static bool consolidate_at(kme_multi* m, int s, kme_epoch_status& tot) {
    if (!m->can_consolidate || m->cons || !m->hist_valid || tot.status != KME_E_UNFUNDED) return false;
    const int s2 = s ^ 1;
    const bool newer = m->slot_mode[s2] == kSlotQueued || m->slot_mode[s2] == kSlotCollected;
    if (m->slot_mode[s2] == kSlotQueued) collect(m, s2);   // (the shards drain; the results are dropped)
    const uint32_t n = m->slot_n[s], ne = tot.n_effective;
    const kme_orders h2 = hist_at(m, m->hist_start[s2]);
    const uint32_t n2 = m->slot_n[s2];
    // the newer epoch's records live in the history too; consolidate() clears it, so keep a copy
    std::vector<int32_t> c_act, c_pr, c_sz;
    std::vector<int64_t> c_oid, c_aid, c_sid;
    if (newer) {
        c_act.assign(h2.action, h2.action + n2); c_pr.assign(h2.price, h2.price + n2); c_sz.assign(h2.size, h2.size + n2);
        c_oid.assign(h2.oid, h2.oid + n2); c_aid.assign(h2.aid, h2.aid + n2); c_sid.assign(h2.sid, h2.sid + n2);
    }
    std::vector<int32_t> r_act, r_pr, r_sz;
    std::vector<int64_t> r_oid, r_aid, r_sid;
    {
        const kme_orders h = hist_at(m, m->hist_start[s] + ne);
        const uint32_t k = n - ne;
        r_act.assign(h.action, h.action + k); r_pr.assign(h.price, h.price + k); r_sz.assign(h.size, h.size + k);
        r_oid.assign(h.oid, h.oid + k); r_aid.assign(h.aid, h.aid + k); r_sid.assign(h.sid, h.sid + k);
    }
    if (consolidate(m, m->hist_start[s] + ne) != KME_OK) {
        m->failed = 1;
        tot.status = KME_E_FAILED;
        return true;
    }
    kme_epoch_status rest{};
    const kme_orders rin{r_act.data(), r_oid.data(), r_aid.data(), r_sid.data(), r_pr.data(), r_sz.data()};
    (void)cons_run(m, rin, n - ne, &m->slot_out[s], ne, &rest);
    tot.n_orders += rest.n_orders; tot.n_rests += rest.n_rests; tot.n_cancel_ok += rest.n_cancel_ok;
    tot.n_trades += rest.n_trades; tot.n_maker_visits += rest.n_trades;
    tot.serial_fallback += rest.serial_fallback; tot.ledger_repaired += rest.ledger_repaired;
    tot.ledger_serial += rest.ledger_serial;
    tot.status = rest.status; tot.detail = rest.detail;
    tot.error_index = rest.status == KME_OK ? -1 : (rest.error_index >= 0 ? ne + rest.error_index : -1);
    tot.n_effective = ne + rest.n_effective;
    if (rest.status != KME_OK) m->failed = 1;
    if (newer) {
        kme_epoch_status st2{};
        const kme_orders in2{c_act.data(), c_oid.data(), c_aid.data(), c_sid.data(), c_pr.data(), c_sz.data()};
        if (rest.status == KME_OK) {
            m->slot_out[s2].trade_off[0] = 0;
            (void)cons_run(m, in2, n2, &m->slot_out[s2], 0, &st2);
        } else {
            st2.status = KME_E_FAILED; st2.error_index = -1; st2.n_inputs = n2;
        }
        if (st2.status != KME_OK) m->failed = 1;
        m->done[s2] = st2;
        m->slot_mode[s2] = kSlotDone;
    }
    return true;
}

extern "C" {

// An epoch of orders only is split and queued (asynchronous, as kme_submit_epoch_host).  An epoch
// with account records runs now, in runs split at them (as kme_submit_epoch splits host epochs): the
// funded proof books a transfer's credit from the next epoch on, so orders of an account funded in
// the same epoch would not be provable; the epoch in flight before it is collected first.
kme_status kme_multi_submit_epoch_host(kme_multi* m, const kme_orders* in, uint32_t n, const kme_epoch_result* out) {
    if (!m || !in || !out || !out->out_action || !out->out_size || !out->out_prev || !out->out_flags || !out->trade_off ||
        !out->trades)
        return KME_E_INVALID;
    if (m->failed) return KME_E_FAILED;
    if (n > m->cfg.max_epoch) return KME_E_CAPACITY;
    if (m->inflight == 2) return KME_E_INVALID;
    if (out->trades_cap < m->cfg.max_trades) return KME_E_INVALID;
    auto is_acct = [&](uint32_t i) { return in->action[i] == KME_CREATE_BALANCE || in->action[i] == KME_TRANSFER; };
    bool mixed = false;
    for (uint32_t i = 0; i < n && !mixed; ++i) mixed = is_acct(i);
    const int slot = (int)(m->sub_count & 1);
    auto finish = [&]() {
        m->slot_n[slot] = n;
        m->slot_out[slot] = *out;
        ++m->sub_count;
        ++m->inflight;
        return KME_OK;
    };
    auto run_consolidated = [&]() {   // one engine takes the stream: synchronously, at submit
        out->trade_off[0] = 0;
        kme_epoch_status st{};
        (void)cons_run(m, *in, n, out, 0, &st);
        if (st.status != KME_OK) m->failed = 1;
        m->done[slot] = st;
        m->slot_mode[slot] = kSlotDone;
        return finish();
    };
    if (m->cons) return run_consolidated();
    m->hist_start[slot] = m->h_action.size();
    hist_append(m, in, n);
    auto rebalance = [&]() -> kme_status {
        if (m->n > 1 && m->rebalance_every && m->sub_count > 0 && ++m->since_rebalance >= m->rebalance_every) {
            m->since_rebalance = 0;
            if (kme_status s = rebalance_enqueue(m)) { m->failed = 1; return s; }
        }
        return KME_OK;
    };
    if (!mixed) {
        if (kme_status s = rebalance()) return s;
        if (kme_status s = split_submit(m, slot, in, 0, n)) return s;
        m->slot_mode[slot] = kSlotQueued;
    } else {
        if (m->inflight) {   // the older epoch completes first (its answered prefix decides a consolidation)
            const int other = slot ^ 1;
            if (m->slot_mode[other] == kSlotQueued) collect(m, other);
            if (m->slot_mode[other] == kSlotCollected) {
                m->slot_out[other].trade_off[0] = 0;
                kme_epoch_status t = merge(m, other, m->slot_n[other], m->slot_out[other], 0, 0);
                if (t.status != KME_OK) (void)consolidate_at(m, other, t);
                if (t.status != KME_OK) m->failed = 1;
                m->done[other] = t;
                m->slot_mode[other] = kSlotDone;
            }
            if (m->failed) return KME_E_FAILED;
            if (m->cons) return run_consolidated();
        }
        kme_epoch_status tot{};
        tot.error_index = -1;
        tot.n_inputs = n;
        out->trade_off[0] = 0;
        uint32_t a = 0, tbase = 0;
        while (a < n) {
            const bool kind = is_acct(a);
            uint32_t b = a;
            while (b < n && is_acct(b) == kind) ++b;
            if (!kind)
                if (kme_status s = rebalance()) return s;
            if (kme_status s = split_submit(m, slot, in, a, b - a)) return s;
            collect(m, slot);
            const kme_epoch_status r = merge(m, slot, b - a, *out, a, tbase);
            tot.n_orders += r.n_orders; tot.n_rests += r.n_rests; tot.n_cancel_ok += r.n_cancel_ok;
            tot.serial_fallback += r.serial_fallback;
            tbase += r.n_trades;
            if (r.status != KME_OK) {
                tot.status = r.status;
                tot.detail = r.detail;
                tot.error_index = r.error_index >= 0 ? a + r.error_index : -1;
                tot.n_effective = a + r.n_effective;
                tot.n_trades = tbase;
                tot.n_maker_visits = tbase;
                m->slot_n[slot] = n;
                m->slot_out[slot] = *out;
                if (consolidate_at(m, slot, tot)) tbase = tot.n_trades;   // the rest of the epoch answered
                break;
            }
            a = b;
            tot.n_effective = a;
        }
        tot.n_trades = tbase;
        tot.n_maker_visits = tbase;
        if (tot.status != KME_OK) m->failed = 1;
        m->done[slot] = tot;
        m->slot_mode[slot] = kSlotDone;
    }
    return finish();
}

kme_status kme_multi_poll(kme_multi* m, int* done) {
    if (!m || !done) return KME_E_INVALID;
    *done = 1;
    if (m->inflight == 0) return KME_OK;
    const int slot = (int)((m->sub_count - (uint32_t)m->inflight) & 1);
    if (m->slot_mode[slot] != kSlotQueued) return KME_OK;
    for (kme_engine* e : m->eng) {   // (an engine's oldest epoch in flight is this slot's part)
        int d = 0;
        if (kme_status s = kme_poll(e, &d)) return s;
        if (!d) { *done = 0; return KME_OK; }
    }
    return KME_OK;
}

// Completes the oldest epoch: every shard's part, merged into input order.
kme_status kme_multi_wait(kme_multi* m, kme_epoch_status* st) {
    if (!m) return KME_E_INVALID;
    if (m->inflight == 0) {
        kme_epoch_status tot{};
        tot.error_index = -1;
        tot.status = m->failed ? KME_E_FAILED : KME_OK;
        if (st) *st = tot;
        return (kme_status)tot.status;
    }
    const int slot = (int)((m->sub_count - (uint32_t)m->inflight) & 1);
    --m->inflight;
    kme_epoch_status tot;
    if (m->slot_mode[slot] == kSlotDone) {
        tot = m->done[slot];
    } else {
        if (m->slot_mode[slot] == kSlotQueued) collect(m, slot);
        m->slot_out[slot].trade_off[0] = 0;
        tot = merge(m, slot, m->slot_n[slot], m->slot_out[slot], 0, 0);
        // a refusal of the funded proof consolidates the stream onto one exact engine when the
        // configuration allows it; any other fault leaves the shards out of step with one another (the
        // others went past it): like the reference's dead stream thread, nothing further is accepted
        if (tot.status != KME_OK) (void)consolidate_at(m, slot, tot);
        if (tot.status != KME_OK) m->failed = 1;
    }
    m->slot_mode[slot] = kSlotIdle;
    if (st) *st = tot;
    return (kme_status)tot.status;
}

kme_status kme_multi_info(kme_multi* m, kme_multi_status* out) {
    if (!m || !out) return KME_E_INVALID;
    *out = kme_multi_status{};
    out->n_engines = m->n;
    out->consolidated = m->cons ? 1u : 0u;
    out->can_consolidate = m->can_consolidate && !m->cons && m->hist_valid ? 1u : 0u;
    out->failed = m->failed ? 1u : 0u;
    out->history_records = m->hist_valid ? (uint64_t)m->h_action.size() : 0;
    out->history_cap = m->can_consolidate ? m->hist_cap : 0;
    out->history_saved = m->hist_valid ? m->hist_saved : 0;
    out->generation = m->generation;
    return KME_OK;
}

kme_status kme_multi_engine(kme_multi* m, uint32_t k, kme_engine** out) {
    if (!m || !out || k >= m->n) return KME_E_INVALID;
    *out = m->cons ? m->cons : m->eng[k];   // (consolidated: the one engine)
    return KME_OK;
}

// pwrite of all n bytes (a regular file takes them whole unless the disk is full)
static bool pwrite_all(int fd, const void* p, size_t n, uint64_t off) {
    const char* c = static_cast<const char*>(p);
    while (n) {
        const ssize_t w = pwrite(fd, c, n, (off_t)off);
        if (w <= 0) return false;
        c += w; n -= (size_t)w; off += (uint64_t)w;
    }
    return true;
}

// The history's records since the last checkpoint appended to `base`.hist and fsync'd (the whole
// history when the last append went to another file; a tail a failed checkpoint left past the saved
// records is cut first).  *records / *digest: what the manifest names (0: no history to keep).
static kme_status hist_save(kme_multi* m, const std::string& base, uint64_t* records, uint64_t* digest) {
    *records = 0;
    *digest = 0;
    if (!m->can_consolidate || m->cons || !m->hist_valid) return KME_OK;
    const std::string f = base + ".hist";
    if (m->hist_file != f) { m->hist_file = f; m->hist_saved = 0; m->hist_dg = kme::Digest(); }
    const uint64_t n = m->h_action.size();
    const int fd = open(f.c_str(), O_WRONLY | O_CREAT, 0644);
    if (fd < 0) return KME_E_INVALID;
    bool ok = ftruncate(fd, (off_t)(m->hist_saved * sizeof(HistRec))) == 0;
    std::vector<HistRec> buf((size_t)std::min<uint64_t>(n - m->hist_saved, 1u << 16));
    kme::Digest dg = m->hist_dg;
    for (uint64_t a = m->hist_saved; ok && a < n;) {
        const size_t k = (size_t)std::min<uint64_t>(buf.size(), n - a);
        for (size_t i = 0; i < k; ++i)
            buf[i] = HistRec{m->h_oid[a + i], m->h_aid[a + i], m->h_sid[a + i], m->h_action[a + i], m->h_price[a + i], m->h_size[a + i], 0};
        ok = pwrite_all(fd, buf.data(), k * sizeof(HistRec), a * sizeof(HistRec));
        dg.update(buf.data(), k * sizeof(HistRec));
        a += k;
    }
    ok = ok && fsync(fd) == 0;
    ok = close(fd) == 0 && ok;
    ok = ok && (m->hist_saved > 0 || kme::sync_dir_of(f));   // (a new file: its directory entry too)
    if (!ok) return KME_E_INVALID;
    m->hist_saved = n;
    m->hist_dg = dg;
    *records = n;
    *digest = dg.final();
    return KME_OK;
}

// The history the manifest names read back from `base`.hist: false when the file is missing, short,
// or its first `records` records are not the ones the manifest's digest covers.
static bool hist_load(kme_multi* m, const std::string& base, uint64_t records, uint64_t digest) {
    if (records > m->hist_cap) return false;
    const std::string f = base + ".hist";
    FILE* fp = std::fopen(f.c_str(), "rb");
    if (!fp) return false;
    const size_t n = (size_t)records;
    try {
        m->h_action.resize(n); m->h_price.resize(n); m->h_size.resize(n);
        m->h_oid.resize(n); m->h_aid.resize(n); m->h_sid.resize(n);
    } catch (const std::bad_alloc&) {
        std::fclose(fp);
        hist_clear(m);
        return false;
    }
    std::vector<HistRec> buf(std::min<size_t>(n, 1u << 16));
    kme::Digest dg;
    bool ok = true;
    for (size_t a = 0; ok && a < n;) {
        const size_t k = std::min(buf.size(), n - a);
        ok = std::fread(buf.data(), sizeof(HistRec), k, fp) == k;
        dg.update(buf.data(), k * sizeof(HistRec));
        for (size_t i = 0; ok && i < k; ++i) {
            const HistRec& r = buf[i];
            m->h_oid[a + i] = r.oid; m->h_aid[a + i] = r.aid; m->h_sid[a + i] = r.sid;
            m->h_action[a + i] = r.action; m->h_price[a + i] = r.price; m->h_size[a + i] = r.size;
        }
        a += k;
    }
    std::fclose(fp);
    if (!ok || dg.final() != digest) { hist_clear(m); return false; }
    m->hist_valid = true;
    m->hist_file = f;
    m->hist_saved = records;
    m->hist_dg = dg;
    m->hist_lost_logged = false;
    return true;
}

// Checkpoint: every engine into path.g<generation>.<k>, the input history's new records onto
// path.hist, then the manifest at `path` (CkptWriter: written to path.tmp, fsync'd, renamed, the
// directory fsync'd -- the commit of the set), and only then are the previous generation's files
// removed: a crash at any point leaves a manifest whose shard files all exist and whose history is a
// prefix of path.hist.
kme_status kme_multi_checkpoint_app(kme_multi* m, const char* path, const void* app, size_t app_bytes) {
    if (!m || !path || (app_bytes && !app)) return KME_E_INVALID;
    if (m->failed) return KME_E_FAILED;
    if (m->inflight) return KME_E_INVALID;
    const uint64_t gen = m->generation + 1;
    const std::string base(path);
    // consolidated: the one engine's file (.0), the manifest says so
    const uint32_t nf = m->cons ? 1 : m->n;
    std::vector<MultiShard> shards(nf);
    for (uint32_t k = 0; k < nf; ++k) {
        const std::string f = base + ".g" + std::to_string(gen) + "." + std::to_string(k);
        if (kme_status s = kme_checkpoint_app(m->cons ? m->cons : m->eng[k], f.c_str(), nullptr, 0)) return s;
        kme_checkpoint_info ci{};
        if (kme_status s = kme_checkpoint_inspect(f.c_str(), &ci)) return s;
        shards[k] = {ci.file_bytes, ci.digest};
    }
    MultiHeader h{};
    std::memcpy(h.magic, kMultiMagic, sizeof h.magic);
    h.n = m->n;
    h._pad = m->cons ? 1u : 0u;            // 1: consolidated (one engine's file)
    h.generation = gen;
    h.app_bytes = app_bytes;
    if (kme_status s = hist_save(m, base, &h.hist_records, &h.hist_digest)) return s;
    {
        kme::CkptWriter w(path);
        bool ok = w.write(&h, sizeof h) && w.write(shards.data(), shards.size() * sizeof(MultiShard)) && w.write(app, app_bytes) &&
                  w.commit(app_bytes, nullptr);
        if (!ok) return KME_E_INVALID;
    }
    for (uint32_t k = 0; k < m->n && m->generation; ++k)   // (the older generation may have had n files)
        std::remove((base + ".g" + std::to_string(m->generation) + "." + std::to_string(k)).c_str());
    if (h.hist_records == 0) {   // no history kept (consolidated, or lost): no file either
        std::remove((base + ".hist").c_str());
        if (m->hist_file == base + ".hist") { m->hist_file.clear(); m->hist_saved = 0; }
    }
    m->generation = gen;
    return KME_OK;
}

kme_status kme_multi_restore_app(kme_multi* m, const char* path, void* app, size_t app_cap, size_t* app_bytes) {
    if (!m || !path) return KME_E_INVALID;
    if (m->failed) return KME_E_FAILED;
    if (m->inflight) return KME_E_INVALID;
    if (app_bytes) *app_bytes = 0;
    kme::CkptReader r(path);
    MultiHeader h{};
    bool ok = r.read(h.magic, sizeof h.magic);
    if (ok && std::memcmp(h.magic, kMultiMagic2, sizeof h.magic) == 0) {   // format 2: no history
        MultiHeader2 h2{};
        ok = r.read(reinterpret_cast<char*>(&h2) + sizeof h2.magic, sizeof h2 - sizeof h2.magic);
        h.n = h2.n; h._pad = h2._pad; h.generation = h2.generation; h.app_bytes = h2.app_bytes;
    } else {
        ok = ok && std::memcmp(h.magic, kMultiMagic, sizeof h.magic) == 0 &&
             r.read(reinterpret_cast<char*>(&h) + sizeof h.magic, sizeof h - sizeof h.magic);
    }
    ok = ok && h.n == m->n && h.app_bytes < (1ull << 40) && h._pad <= 1 && (h._pad == 0 || m->can_consolidate) &&
         (h._pad == 1 || !m->cons);
    const uint32_t nf = h._pad ? 1 : m->n;
    std::vector<MultiShard> shards(ok ? nf : 0);
    std::vector<char> rec;
    ok = ok && r.read(shards.data(), shards.size() * sizeof(MultiShard));
    if (ok) {
        rec.resize(h.app_bytes);
        ok = r.read(rec.data(), rec.size());
    }
    kme::CkptTrailer t{};
    ok = ok && r.verify(&t);
    if (!ok) return KME_E_INVALID;
    if (app_bytes) *app_bytes = rec.size();
    if (rec.size() > app_cap || (rec.size() && !app)) return KME_E_CAPACITY;
    // every shard's file is the one the manifest committed (before any engine is touched)
    const std::string base(path);
    auto shard_path = [&](uint32_t k) { return base + ".g" + std::to_string(h.generation) + "." + std::to_string(k); };
    for (uint32_t k = 0; k < nf; ++k) {
        kme_checkpoint_info ci{};
        if (kme_checkpoint_inspect(shard_path(k).c_str(), &ci) != KME_OK || ci.file_bytes != shards[k].file_bytes ||
            ci.digest != shards[k].digest)
            return KME_E_INVALID;
    }
    hist_clear(m);           // (the history of the checkpoint's stream is read back below)
    if (h._pad) {            // a consolidated stream: the one engine
        if (!m->cons) {
            free_parts(m);
            for (kme_engine*& e : m->eng) {
                if (e) kme_destroy(e);
                e = nullptr;
            }
            if (kme_status s = kme_create(&m->cons_cfg, &m->cons)) { m->cons = nullptr; m->failed = 1; return s; }
        }
        if (kme_status s = kme_restore(m->cons, shard_path(0).c_str())) { m->failed = 1; return s; }
        alloc_scratch(m);
        m->generation = h.generation;
        if (rec.size()) std::memcpy(app, rec.data(), rec.size());
        return KME_OK;
    }
    for (uint32_t k = 0; k < m->n; ++k) {
        if (kme_status s = kme_restore(m->eng[k], shard_path(k).c_str())) {
            if (k > 0) m->failed = 1;   // some shards restored, others not
            return s;
        }
    }
    // the router's oid directory: every resting order's partition (a cancel of an order resting
    // nowhere is rejected by whichever engine gets it, KP:290-291, so no other entry matters)
    for (uint32_t k = 0; k < m->n; ++k) {
        std::vector<int64_t> oids;
        if (kme_status s = kme::resting_oids(m->eng[k], oids)) { m->failed = 1; return s; }
        kme::router_seed(m->router, oids.data(), oids.size(), k);
    }
    // the input history up to the checkpoint: consolidation stays possible after the restart
    if (m->can_consolidate) {
        if (h.hist_records == 0) hist_lost(m, "not in the checkpoint (lost before it, or a format-2 manifest)");
        else if (!hist_load(m, base, h.hist_records, h.hist_digest)) hist_lost(m, "unreadable (path.hist missing, short or not the manifest's)");
    }
    m->generation = h.generation;
    if (rec.size()) std::memcpy(app, rec.data(), rec.size());
    return KME_OK;
}

}  // extern "C"
