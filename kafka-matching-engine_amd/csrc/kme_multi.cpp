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
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

constexpr char kMultiMagic[8] = {'K', 'M', 'E', 'M', 'U', 'L', 'T', '2'};
// the manifest: this header, n shard records (the digest and size of each shard's file: the
// manifest's own digest covers them), the application record, the trailer (kme_internal.h)
struct MultiHeader {
    char magic[8];
    uint32_t n, _pad;
    uint64_t generation;
    uint64_t app_bytes;
};
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
    if (m->router) kme_router_destroy(m->router);
    delete m;
    return KME_OK;
}

kme_status kme_multi_create(const kme_config* cfg, uint32_t n, const int32_t* devices, kme_multi** out) {
    if (!cfg || !out || n == 0 || n > 1024 || !devices) return KME_E_INVALID;
    // shards prove their orders against their share of each account's credit: FUNDED, no exact ledger
    // (it couples every symbol, kme_create refuses it with credit_shards > 1)
    if (cfg->mode != KME_MODE_FUNDED || (n > 1 && cfg->flags != 0)) return KME_E_INVALID;
    kme_multi* m = new kme_multi();
    m->cfg = *cfg;
    m->cfg.credit_shards = n;
    m->n = n;
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
        if (m->inflight) {
            const int other = slot ^ 1;
            if (m->slot_mode[other] == kSlotQueued) collect(m, other);
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
    m->slot_n[slot] = n;
    m->slot_out[slot] = *out;
    ++m->sub_count;
    ++m->inflight;
    return KME_OK;
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
        // any fault leaves the shards out of step with one another (the others went past it): like
        // the reference's dead stream thread, nothing further is accepted
        if (tot.status != KME_OK) m->failed = 1;
    }
    m->slot_mode[slot] = kSlotIdle;
    if (st) *st = tot;
    return (kme_status)tot.status;
}

kme_status kme_multi_engine(kme_multi* m, uint32_t k, kme_engine** out) {
    if (!m || !out || k >= m->n) return KME_E_INVALID;
    *out = m->eng[k];
    return KME_OK;
}

// Checkpoint: every engine into path.g<generation>.<k>, then the manifest at `path` (CkptWriter:
// written to path.tmp, fsync'd, renamed, the directory fsync'd -- the commit of the set), and only then
// are the previous generation's files removed: a crash at any point leaves a manifest whose shard
// files all exist.
kme_status kme_multi_checkpoint_app(kme_multi* m, const char* path, const void* app, size_t app_bytes) {
    if (!m || !path || (app_bytes && !app)) return KME_E_INVALID;
    if (m->failed) return KME_E_FAILED;
    if (m->inflight) return KME_E_INVALID;
    const uint64_t gen = m->generation + 1;
    const std::string base(path);
    std::vector<MultiShard> shards(m->n);
    for (uint32_t k = 0; k < m->n; ++k) {
        const std::string f = base + ".g" + std::to_string(gen) + "." + std::to_string(k);
        if (kme_status s = kme_checkpoint_app(m->eng[k], f.c_str(), nullptr, 0)) return s;
        kme_checkpoint_info ci{};
        if (kme_status s = kme_checkpoint_inspect(f.c_str(), &ci)) return s;
        shards[k] = {ci.file_bytes, ci.digest};
    }
    MultiHeader h{};
    std::memcpy(h.magic, kMultiMagic, sizeof h.magic);
    h.n = m->n;
    h.generation = gen;
    h.app_bytes = app_bytes;
    {
        kme::CkptWriter w(path);
        bool ok = w.write(&h, sizeof h) && w.write(shards.data(), shards.size() * sizeof(MultiShard)) && w.write(app, app_bytes) &&
                  w.commit(app_bytes, nullptr);
        if (!ok) return KME_E_INVALID;
    }
    for (uint32_t k = 0; k < m->n && m->generation; ++k)
        std::remove((base + ".g" + std::to_string(m->generation) + "." + std::to_string(k)).c_str());
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
    bool ok = r.read(&h, sizeof h) && std::memcmp(h.magic, kMultiMagic, sizeof h.magic) == 0 && h.n == m->n &&
              h.app_bytes < (1ull << 40);
    std::vector<MultiShard> shards(ok ? m->n : 0);
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
    for (uint32_t k = 0; k < m->n; ++k) {
        kme_checkpoint_info ci{};
        if (kme_checkpoint_inspect(shard_path(k).c_str(), &ci) != KME_OK || ci.file_bytes != shards[k].file_bytes ||
            ci.digest != shards[k].digest)
            return KME_E_INVALID;
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
    m->generation = h.generation;
    if (rec.size()) std::memcpy(app, rec.data(), rec.size());
    return KME_OK;
}

}  // extern "C"
