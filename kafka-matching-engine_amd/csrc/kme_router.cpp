// kme_router.cpp -- the host side of symbol sharding: one MatchIn
// stream split over N engines by symbol, each input answered by exactly one engine.
//
// The reference produces every record to partition 0 of MatchIn (exchange_test.js:14-16,
// topic.js:17-18) and one processor matches them all (KP:51-52).  Books of different symbols never
// interact, so the stream partitions by |sid| -- Kafka's default keyed partitioner (murmur2 of the
// decimal key, kme_shard_of), as a producer keyed by symbol would place the records.  A CANCEL
// carries no symbol (exchange_test.js:101): it goes to the partition that received the last
// BUY/SELL carrying its oid, found in an oid -> partition directory kept here (an oid never seen
// goes to partition 0, which rejects it as the reference does, KP:290).  Account records go to every
// partition (each engine proves its orders against 1/n of the credit, kme_config.credit_shards) and
// are echoed by partition 0 only.  Any other action goes to partition 0.  Same rules as
// kme/sharding.py PartitionRouter, which tests/test_router.py holds this file to.
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <new>
#include <thread>
#include <vector>

#include "kme.h"
#include "kme_internal.h"

namespace {

enum : int32_t { A_ADD_SYMBOL = 0, A_REMOVE_SYMBOL = 1, A_BUY = 2, A_SELL = 3, A_CANCEL = 4, A_PAYOUT = 200,
                 A_CREATE_BALANCE = 100, A_TRANSFER = 101 };

inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// oid -> partition, open addressing (linear probing), never deleted: the last BUY/SELL with an
// oid decides, as in PartitionRouter.  Slots hold oid + 1 (0 = empty); oid -1, whose key would be
// 0, is kept in a side slot.
struct Directory {
    std::vector<uint64_t> key;
    std::vector<uint16_t> val;
    uint64_t used = 0;
    bool has_m1 = false;
    uint16_t m1_val = 0;

    explicit Directory(uint64_t cap) {
        uint64_t c = 1024;
        while (c < 2 * cap) c <<= 1;
        key.assign(c, 0);
        val.assign(c, 0);
    }
    void grow() {
        std::vector<uint64_t> k2(key.size() * 2, 0);
        std::vector<uint16_t> v2(key.size() * 2, 0);
        const uint64_t m = k2.size() - 1;
        for (size_t s = 0; s < key.size(); ++s) {
            if (!key[s]) continue;
            uint64_t h = mix64(key[s] - 1) & m;
            while (k2[h]) h = (h + 1) & m;
            k2[h] = key[s];
            v2[h] = val[s];
        }
        key.swap(k2);
        val.swap(v2);
    }
    void put(int64_t oid, uint16_t p) {
        if (oid == -1) { has_m1 = true; m1_val = p; return; }
        if (2 * (used + 1) > key.size()) grow();
        const uint64_t k = (uint64_t)oid + 1, m = key.size() - 1;
        uint64_t h = mix64((uint64_t)oid) & m;
        while (key[h] && key[h] != k) h = (h + 1) & m;
        if (!key[h]) { key[h] = k; ++used; }
        val[h] = p;
    }
    void prefetch(int64_t oid) const {
        const uint64_t h = mix64((uint64_t)oid) & (key.size() - 1);
        __builtin_prefetch(&key[h]);
        __builtin_prefetch(&val[h]);
    }
    int32_t get(int64_t oid) const {
        if (oid == -1) return has_m1 ? m1_val : -1;
        const uint64_t k = (uint64_t)oid + 1, m = key.size() - 1;
        uint64_t h = mix64((uint64_t)oid) & m;
        while (key[h]) {
            if (key[h] == k) return val[h];
            h = (h + 1) & m;
        }
        return -1;
    }
};

}  // namespace

// The directory is split by oid hash into `ndir` sub-directories, each owned by one thread of a
// route call: a thread scans the whole batch but only looks up / updates the oids of its own
// sub-directory, so every oid's BUY/SELL/CANCEL sequence is still applied in arrival order.
struct kme_router {
    uint32_t n;
    uint32_t ndir;
    std::vector<Directory> dir;
    std::vector<int32_t> sym_part;   // |sid| -> partition cache (-1 = not computed), for |sid| < 2^24
    kme_router(uint32_t parts, uint64_t cap, uint32_t threads) : n(parts), ndir(threads), sym_part((size_t)1 << 16, -1) {
        dir.reserve(threads);
        for (uint32_t t = 0; t < threads; ++t) dir.emplace_back(cap / threads + 1);
    }
    uint32_t part_of_sid(int64_t sid) {
        const uint64_t u = sid < 0 ? 0ull - (uint64_t)sid : (uint64_t)sid;
        if (u >= ((uint64_t)1 << 24)) return kme_shard_of(sid, n);
        if (u >= sym_part.size()) sym_part.resize((size_t)1 << 24, -1);
        int32_t& c = sym_part[u];
        if (c < 0) c = (int32_t)kme_shard_of(sid, n);
        return (uint32_t)c;
    }
    uint32_t owner(int64_t oid) const { return (uint32_t)((mix64((uint64_t)oid ^ 0x5bd1e995ull) >> 40) % ndir); }
};

namespace kme {
void router_seed(kme_router* r, const int64_t* oids, size_t n, uint32_t partition) {
    for (size_t i = 0; i < n; ++i) r->dir[r->owner(oids[i])].put(oids[i], (uint16_t)partition);
}
}  // namespace kme

extern "C" {

kme_status kme_router_create(uint32_t n_partitions, uint64_t directory_capacity, kme_router** out) {
    if (!out || n_partitions == 0 || n_partitions > 65535) return KME_E_INVALID;
    uint32_t threads = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (const char* v = std::getenv("KME_ROUTER_THREADS")) threads = (uint32_t)std::max(1, std::min(64, std::atoi(v)));
    *out = new (std::nothrow) kme_router(n_partitions, directory_capacity, threads);
    return *out ? KME_OK : KME_E_CAPACITY;
}

kme_status kme_router_destroy(kme_router* r) {
    delete r;
    return KME_OK;
}

kme_status kme_router_route(kme_router* r, const kme_orders* in, uint32_t n, int32_t* dest) {
    if (!r || !in || (n && !dest)) return KME_E_INVALID;
    // symbol records first (a pure function of the sid; fills the cache single-threaded)
    for (uint32_t i = 0; i < n; ++i) {
        const int32_t a = in->action[i];
        switch (a) {
        case A_BUY: case A_SELL: case A_ADD_SYMBOL: case A_REMOVE_SYMBOL: case A_PAYOUT:
            dest[i] = (int32_t)r->part_of_sid(in->sid[i]);
            break;
        case A_CREATE_BALANCE: case A_TRANSFER:
            dest[i] = KME_ROUTE_ALL;
            break;
        default:                                             // CANCEL: below; others: partition 0
            dest[i] = 0;
            break;
        }
    }
    // the oid directory: BUY/SELL record their partition, CANCEL takes it (unknown oid: 0).  A
    // thread keeps its cancels' answers locally (no shared cache lines while the threads run) and
    // prefetches the probe slots of the records a few ahead (the directory is much larger than
    // the caches: one miss per probe otherwise)
    std::vector<std::vector<std::pair<uint32_t, int32_t>>> found(r->ndir);
    auto work = [&](uint32_t t) {
        Directory& d = r->dir[t];
        auto& res = found[t];
        constexpr uint32_t AHEAD = 16;
        for (uint32_t i = 0; i < n; ++i) {
            if (i + AHEAD < n) {
                const int32_t a2 = in->action[i + AHEAD];
                const int64_t o2 = in->oid[i + AHEAD];
                if ((a2 == A_BUY || a2 == A_SELL || a2 == A_CANCEL) && r->owner(o2) == t) d.prefetch(o2);
            }
            const int32_t a = in->action[i];
            if (a != A_BUY && a != A_SELL && a != A_CANCEL) continue;
            const int64_t oid = in->oid[i];
            if (r->owner(oid) != t) continue;
            if (a == A_CANCEL) {
                const int32_t p = d.get(oid);
                res.emplace_back(i, p < 0 ? 0 : p);
            } else {
                d.put(oid, (uint16_t)dest[i]);
            }
        }
    };
    if (r->ndir == 1 || n < (1u << 14)) {
        for (uint32_t t = 0; t < r->ndir; ++t) work(t);
    } else {
        std::vector<std::thread> th;
        for (uint32_t t = 1; t < r->ndir; ++t) th.emplace_back(work, t);
        work(0);
        for (auto& x : th) x.join();
    }
    for (const auto& v : found)
        for (const auto& f : v) dest[f.first] = f.second;
    return KME_OK;
}

kme_status kme_router_split(kme_router* r, const kme_orders* in, uint32_t n, const kme_orders_buf* parts,
                            uint32_t* counts, uint8_t* const* echo, uint32_t* const* index) {
    if (!r || !in || !parts || !counts) return KME_E_INVALID;
    std::vector<int32_t> dest(n);
    const kme_status s = kme_router_route(r, in, n, dest.data());
    if (s != KME_OK) return s;
    for (uint32_t k = 0; k < r->n; ++k) counts[k] = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const int32_t d = dest[i];
        const uint32_t k0 = d == KME_ROUTE_ALL ? 0 : (uint32_t)d, k1 = d == KME_ROUTE_ALL ? r->n : (uint32_t)d + 1;
        for (uint32_t k = k0; k < k1; ++k) {
            const uint32_t j = counts[k]++;
            const kme_orders_buf& p = parts[k];
            p.action[j] = in->action[i]; p.oid[j] = in->oid[i]; p.aid[j] = in->aid[i];
            p.sid[j] = in->sid[i]; p.price[j] = in->price[i]; p.size[j] = in->size[i];
            if (echo && echo[k]) echo[k][j] = (uint8_t)(d != KME_ROUTE_ALL || k == 0);
            if (index && index[k]) index[k][j] = i;
        }
    }
    return KME_OK;
}

uint64_t kme_router_directory_size(const kme_router* r) {
    if (!r) return 0;
    uint64_t s = 0;
    for (const Directory& d : r->dir) s += d.used + (d.has_m1 ? 1 : 0);
    return s;
}

}  // extern "C"
