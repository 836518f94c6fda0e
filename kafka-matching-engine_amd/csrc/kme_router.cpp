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
//
// Work is O(records) in three parallel passes over a thread pool of the caller's call: (1) each
// thread takes a contiguous range -- a symbol record's partition from a per-sid cache, and which
// directory shard owns each BUY/SELL/CANCEL oid (a hash); (2) the records of each directory shard
// are bucketed in arrival order as 16-byte items (oid, input index, partition or cancel; a counting
// sort over (range, shard)); (3) each thread owns one directory shard and streams its items -- a
// BUY/SELL records its partition, a CANCEL takes it -- with the probe slots a few items ahead
// prefetched.  The directory slots
// are 16 bytes (oid + 1, partition: one cache line per probe) in 2 MiB-aligned memory advised for
// huge pages (the directory outgrows every cache: each probe is a DRAM access, and with 4 KiB pages a
// TLB miss too).  kme_router_split then counts and scatters each range's records per partition.
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "kme.h"
#include "kme_internal.h"

namespace {

enum : int32_t { A_ADD_SYMBOL = 0, A_REMOVE_SYMBOL = 1, A_BUY = 2, A_SELL = 3, A_CANCEL = 4, A_PAYOUT = 200,
                 A_CREATE_BALANCE = 100, A_TRANSFER = 101 };

// action -> what the router does with the record: C_SYM = routed by |sid|, C_DIR = goes through the
// oid directory (BUY/SELL record, CANCEL looks up), C_ALL = to every partition; 0 = partition 0
enum : uint8_t { C_SYM = 1, C_DIR = 2, C_ALL = 4 };
constexpr uint64_t kSymMask = ((uint64_t)1 << 24) - 1;   // the per-sid partition cache covers |sid| <= kSymMask
constexpr uint8_t action_class(int a) {
    return a == A_BUY || a == A_SELL ? C_SYM | C_DIR
         : a == A_CANCEL ? C_DIR
         : a == A_ADD_SYMBOL || a == A_REMOVE_SYMBOL || a == A_PAYOUT ? C_SYM
         : a == A_CREATE_BALANCE || a == A_TRANSFER ? C_ALL : 0;
}
struct ClassTable {
    uint8_t v[256];
    constexpr ClassTable() : v() { for (int a = 0; a < 256; ++a) v[a] = action_class(a); }
};
constexpr ClassTable kClassTable;
constexpr const uint8_t* kClass = kClassTable.v;

inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// one BUY/SELL/CANCEL for its directory shard: all pass (3) reads, so that its pass streams
struct Item {
    int64_t oid;
    uint32_t i;        // input index
    int32_t p;         // BUY/SELL: its partition; CANCEL: -1
};

struct Slot {
    uint64_t key;      // oid + 1 (0 = empty)
    uint32_t val;      // partition
    uint32_t _pad;
};

void* huge_alloc(size_t bytes) {
    void* p = nullptr;
    const size_t align = (size_t)2 << 20;
    bytes = (bytes + align - 1) & ~(align - 1);
    if (posix_memalign(&p, align, bytes) != 0) return nullptr;
    (void)madvise(p, bytes, MADV_HUGEPAGE);
    std::memset(p, 0, bytes);
    return p;
}

// oid -> partition, open addressing (linear probing), never deleted: the last BUY/SELL with an oid
// decides, as in PartitionRouter.  oid -1, whose key would be 0, is kept in a side slot.
struct Directory {
    Slot* s = nullptr;
    uint64_t mask = 0, used = 0;
    bool has_m1 = false;
    uint32_t m1_val = 0;

    explicit Directory(uint64_t cap) {
        uint64_t c = 1024;
        while (c < 2 * cap) c <<= 1;
        s = (Slot*)huge_alloc(c * sizeof(Slot));
        mask = s ? c - 1 : 0;
    }
    ~Directory() { std::free(s); }
    Directory(const Directory&) = delete;
    Directory& operator=(const Directory&) = delete;
    Directory(Directory&& o) noexcept : s(o.s), mask(o.mask), used(o.used), has_m1(o.has_m1), m1_val(o.m1_val) { o.s = nullptr; }

    bool grow() {
        const uint64_t c = 2 * (mask + 1);
        Slot* t = (Slot*)huge_alloc(c * sizeof(Slot));
        if (!t) return false;
        for (uint64_t k = 0; k <= mask; ++k) {
            if (!s[k].key) continue;
            uint64_t h = mix64(s[k].key - 1) & (c - 1);
            while (t[h].key) h = (h + 1) & (c - 1);
            t[h] = s[k];
        }
        std::free(s);
        s = t;
        mask = c - 1;
        return true;
    }
    // the slot holding oid, or the empty slot ending its probe sequence (oid != -1)
    Slot& probe(int64_t oid) {
        const uint64_t k = (uint64_t)oid + 1;
        uint64_t h = mix64((uint64_t)oid) & mask;
        while (s[h].key && s[h].key != k) h = (h + 1) & mask;
        return s[h];
    }
    bool put(int64_t oid, uint32_t p) {
        if (oid == -1) { has_m1 = true; m1_val = p; return true; }
        if (2 * (used + 1) > mask + 1 && !grow()) return false;
        Slot& sl = probe(oid);
        used += !sl.key;
        sl.key = (uint64_t)oid + 1;
        sl.val = p;
        return true;
    }
    void prefetch(int64_t oid) const { __builtin_prefetch(&s[mix64((uint64_t)oid) & mask]); }
};

// f(t) for t in [0, nt) on nt threads (the calling thread takes t = 0)
template <class F>
void parallel(uint32_t nt, F&& f) {
    if (nt <= 1) { f(0u); return; }
    std::vector<std::thread> th;
    th.reserve(nt - 1);
    for (uint32_t t = 1; t < nt; ++t) th.emplace_back(f, t);
    f(0u);
    for (auto& x : th) x.join();
}

}  // namespace

struct kme_router {
    uint32_t n;
    uint32_t nthr;
    std::vector<Directory> dir;                  // directory shard t: the oids with owner(oid) == t
    int32_t* sym_part;                           // |sid| -> partition + 1 (0 = not computed), |sid| < 2^24
    // per call scratch
    std::vector<uint8_t> own;
    std::vector<Item> items;
    std::vector<int32_t> dest;
    bool oom = false;

    kme_router(uint32_t parts, uint64_t cap, uint32_t threads)
        : n(parts), nthr(threads), sym_part((int32_t*)std::calloc((size_t)1 << 24, sizeof(int32_t))) {
        if (!sym_part) oom = true;
        dir.reserve(threads);
        for (uint32_t t = 0; t < threads; ++t) {
            dir.emplace_back(cap / threads + 1);
            if (!dir.back().s) oom = true;
        }
    }
    uint32_t part_of_sid(int64_t sid) {
        const uint64_t u = sid < 0 ? 0ull - (uint64_t)sid : (uint64_t)sid;
        if (u > kSymMask) return kme_shard_of(sid, n);
        int32_t c = __atomic_load_n(&sym_part[u], __ATOMIC_RELAXED);
        if (c == 0) {                                // (threads racing here store the same value)
            c = (int32_t)kme_shard_of(sid, n) + 1;
            __atomic_store_n(&sym_part[u], c, __ATOMIC_RELAXED);
        }
        return (uint32_t)(c - 1);
    }
    ~kme_router() { std::free(sym_part); }
    kme_router(const kme_router&) = delete;
    kme_router& operator=(const kme_router&) = delete;
    uint32_t owner(int64_t oid) const { return (uint32_t)(((mix64((uint64_t)oid ^ 0x5bd1e995ull) >> 32) * nthr) >> 32); }
};

namespace kme {
void router_seed(kme_router* r, const int64_t* oids, size_t n, uint32_t partition) {
    for (size_t i = 0; i < n; ++i) r->dir[r->owner(oids[i])].put(oids[i], partition);
}
}  // namespace kme

static kme_status route(kme_router* r, const kme_orders* in, uint32_t n, int32_t* dest) {
    const uint32_t T = n < (1u << 14) ? 1u : r->nthr;   // small batches: no thread start-up
    const uint32_t D = r->nthr;                          // directory shards
    if (D > 255) return KME_E_INVALID;
    r->own.resize(n);
    uint8_t* own = r->own.data();
    std::vector<uint32_t> cnt((size_t)T * D, 0);
    auto range = [&](uint32_t t, uint32_t& a, uint32_t& b) {
        a = (uint32_t)((uint64_t)n * t / T);
        b = (uint32_t)((uint64_t)n * (t + 1) / T);
    };
    // (1) partitions of the symbol records; directory shard of every BUY/SELL/CANCEL.  Branch-free
    // over the action (random in a live stream: a branch per record would mispredict half the time);
    // counts in thread-local memory (no cache line shared while the threads run)
    parallel(T, [&](uint32_t t) {
        uint32_t a, b;
        range(t, a, b);
        std::vector<uint32_t> c(D + 1, 0);                   // c[D]: records with no directory work
        for (uint32_t i = a; i < b; ++i) {
            const int32_t act = in->action[i];
            const uint8_t k = (uint32_t)act < 256 ? kClass[act] : 0;
            const int64_t sid = in->sid[i];
            const uint64_t u = sid < 0 ? 0ull - (uint64_t)sid : (uint64_t)sid;
            int32_t p = __atomic_load_n(&r->sym_part[u & kSymMask], __ATOMIC_RELAXED) - 1;
            if (__builtin_expect((k & C_SYM) && (u > kSymMask || p < 0), 0)) p = (int32_t)r->part_of_sid(sid);
            dest[i] = (k & C_SYM) ? p : k == C_ALL ? KME_ROUTE_ALL : 0;
            const uint32_t o = (k & C_DIR) ? r->owner(in->oid[i]) : D;
            own[i] = (uint8_t)o;
            ++c[o];
        }
        std::copy(c.begin(), c.begin() + D, &cnt[(size_t)t * D]);
    });
    // (2) each directory shard's records in arrival order: offsets shard-major, then range
    std::vector<uint32_t> off((size_t)T * D), start(D + 1, 0);
    uint64_t acc = 0;
    for (uint32_t d = 0; d < D; ++d) {
        start[d] = (uint32_t)acc;
        for (uint32_t t = 0; t < T; ++t) {
            off[(size_t)t * D + d] = (uint32_t)acc;
            acc += cnt[(size_t)t * D + d];
        }
    }
    start[D] = (uint32_t)acc;
    r->items.resize(acc);
    Item* items = r->items.data();
    parallel(T, [&](uint32_t t) {
        uint32_t a, b;
        range(t, a, b);
        std::vector<uint32_t> o(&off[(size_t)t * D], &off[(size_t)t * D] + D);
        for (uint32_t i = a; i < b; ++i) {
            const uint32_t w = own[i];
            if (w < D) items[o[w]++] = Item{in->oid[i], i, in->action[i] == A_CANCEL ? -1 : dest[i]};
        }
    });
    // (3) each directory shard applies its records in arrival order (a BUY/SELL records its
    // partition, a CANCEL takes it; unknown oid: 0), prefetching the probe slots a few ahead
    std::atomic<bool> oom{false};
    auto apply = [&](uint32_t d) {
        Directory& dir = r->dir[d];
        constexpr uint32_t AHEAD = 16;
        const uint32_t a = start[d], b = start[d + 1];
        for (uint32_t k = a; k < b; ++k) {
            if (k + AHEAD < b) dir.prefetch(items[k + AHEAD].oid);
            const Item it = items[k];
            if (__builtin_expect(it.oid == -1, 0)) {
                if (it.p < 0) dest[it.i] = dir.has_m1 ? (int32_t)dir.m1_val : 0;
                else { dir.has_m1 = true; dir.m1_val = (uint32_t)it.p; }
                continue;
            }
            if (__builtin_expect(2 * (dir.used + 1) > dir.mask + 1, 0) && !dir.grow()) {
                oom.store(true, std::memory_order_relaxed);
                return;
            }
            Slot& sl = dir.probe(it.oid);
            const uint64_t key = (uint64_t)it.oid + 1;
            const bool found = sl.key == key;
            if (it.p < 0) {
                dest[it.i] = found ? (int32_t)sl.val : 0;
            } else {
                dir.used += !found;
                sl.key = key;
                sl.val = (uint32_t)it.p;
            }
        }
    };
    // a small batch (kme_multi splits an epoch at its account-record runs: many small calls) applies
    // the shards inline, with no thread start-up, as passes 1 and 2 do
    if (T == 1) {
        for (uint32_t d = 0; d < D; ++d) apply(d);
    } else {
        parallel(D, apply);
    }
    return oom.load() ? KME_E_CAPACITY : KME_OK;
}

extern "C" {

kme_status kme_router_create(uint32_t n_partitions, uint64_t directory_capacity, kme_router** out) {
    if (!out || n_partitions == 0 || n_partitions > 65535) return KME_E_INVALID;
    uint32_t threads = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (const char* v = std::getenv("KME_ROUTER_THREADS")) threads = (uint32_t)std::max(1, std::min(64, std::atoi(v)));
    kme_router* r = new (std::nothrow) kme_router(n_partitions, directory_capacity, threads);
    if (r && r->oom) { delete r; r = nullptr; }
    *out = r;
    return r ? KME_OK : KME_E_CAPACITY;
}

kme_status kme_router_destroy(kme_router* r) {
    delete r;
    return KME_OK;
}

kme_status kme_router_route(kme_router* r, const kme_orders* in, uint32_t n, int32_t* dest) {
    if (!r || !in || (n && !dest)) return KME_E_INVALID;
    return route(r, in, n, dest);
}

kme_status kme_router_split(kme_router* r, const kme_orders* in, uint32_t n, const kme_orders_buf* parts,
                            uint32_t* counts, uint8_t* const* echo, uint32_t* const* index) {
    if (!r || !in || !parts || !counts) return KME_E_INVALID;
    r->dest.resize(n);
    int32_t* dest = r->dest.data();
    const kme_status s = route(r, in, n, dest);
    if (s != KME_OK) return s;
    const uint32_t P = r->n;
    const uint32_t T = n < (1u << 14) ? 1u : r->nthr;
    std::vector<uint32_t> cnt((size_t)T * P, 0);
    auto range = [&](uint32_t t, uint32_t& a, uint32_t& b) {
        a = (uint32_t)((uint64_t)n * t / T);
        b = (uint32_t)((uint64_t)n * (t + 1) / T);
    };
    // (per-thread counters and write positions in thread-local memory: no shared cache line)
    parallel(T, [&](uint32_t t) {
        uint32_t a, b;
        range(t, a, b);
        std::vector<uint32_t> c(P, 0);
        uint32_t all = 0;
        for (uint32_t i = a; i < b; ++i) {
            const int32_t d = dest[i];
            if (d == KME_ROUTE_ALL) ++all;
            else ++c[d];
        }
        for (uint32_t k = 0; k < P; ++k) cnt[(size_t)t * P + k] = c[k] + all;
    });
    for (uint32_t k = 0; k < P; ++k) {   // each range's first slot in partition k
        uint32_t acc = 0;
        for (uint32_t t = 0; t < T; ++t) {
            const uint32_t c = cnt[(size_t)t * P + k];
            cnt[(size_t)t * P + k] = acc;
            acc += c;
        }
        counts[k] = acc;
    }
    parallel(T, [&](uint32_t t) {
        uint32_t a, b;
        range(t, a, b);
        std::vector<uint32_t> o(&cnt[(size_t)t * P], &cnt[(size_t)t * P] + P);
        for (uint32_t i = a; i < b; ++i) {
            const int32_t d = dest[i];
            const uint32_t k0 = d == KME_ROUTE_ALL ? 0 : (uint32_t)d, k1 = d == KME_ROUTE_ALL ? P : (uint32_t)d + 1;
            for (uint32_t k = k0; k < k1; ++k) {
                const uint32_t j = o[k]++;
                const kme_orders_buf& p = parts[k];
                p.action[j] = in->action[i]; p.oid[j] = in->oid[i]; p.aid[j] = in->aid[i];
                p.sid[j] = in->sid[i]; p.price[j] = in->price[i]; p.size[j] = in->size[i];
                if (echo && echo[k]) echo[k][j] = (uint8_t)(d != KME_ROUTE_ALL || k == 0);
                if (index && index[k]) index[k][j] = i;
            }
        }
    });
    return KME_OK;
}

uint64_t kme_router_directory_size(const kme_router* r) {
    if (!r) return 0;
    uint64_t s = 0;
    for (const Directory& d : r->dir) s += d.used + (d.has_m1 ? 1 : 0);
    return s;
}

}  // extern "C"
