// kme_internal.h -- what kme_multi.cpp (the N-engine drop-in) needs of an engine beyond kme.h: its
// stream and device, and stream-ordered credit re-splitting that queues behind epochs in flight
// (kme_credit_state / kme_credit_adjust refuse them; these are ordered by the engine stream instead).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>
#include <vector>

#include "kme.h"

namespace kme {

hipStream_t engine_stream(kme_engine* e);
int engine_device(kme_engine* e);
const kme_config& engine_config(kme_engine* e);
// (bound, demand) per account into dev_out[0, 2A), after everything queued on the engine stream
kme_status credit_state_enqueue(kme_engine* e, int64_t* dev_out);
// the re-split from n blocks of `stride` words (shard-major), before anything queued later
kme_status credit_adjust_enqueue(kme_engine* e, const int64_t* dev_all, uint32_t n, uint32_t me, size_t stride);
// the oids of the resting orders (nothing in flight): a router's directory rebuilt after a restore
kme_status resting_oids(kme_engine* e, std::vector<int64_t>& out);
// a router's oid directory entries: each oid's last BUY/SELL went to `partition` (kme_router.cpp)
void router_seed(kme_router* r, const int64_t* oids, size_t n, uint32_t partition);

// ------------------------------------------------------------------ checkpoint files
// Every checkpoint file (an engine's, a kme_multi manifest) ends with a trailer: the application
// record's size and a 64-bit digest of every byte before the trailer, computed while writing
// (kme_checkpoint_inspect reads it without the rest; a restore recomputes it over what it read).
// Trailer "KMEDGST2" (round 6): a tree digest -- every kDigestBlock bytes of the file hashed on their
// own, then the block digests and the length -- so that writer and reader hash blocks on many host
// threads; "KMEDGST1" files (one Digest over the whole stream) are still read.
struct CkptTrailer {
    uint64_t app_bytes;
    uint64_t digest;
    char magic[8];
};
constexpr char kTrailerMagic[8] = {'K', 'M', 'E', 'D', 'G', 'S', 'T', '1'};
constexpr char kTrailerMagic2[8] = {'K', 'M', 'E', 'D', 'G', 'S', 'T', '2'};
constexpr uint64_t kDigestBlock = 1ull << 20;

// Four independent multiply-rotate lanes over 8-byte words (a dependency chain per lane, so the
// host hashes at several GB/s); the tail bytes of a stream are zero-padded into a last word.
struct Digest {
    uint64_t h[4] = {0x243f6a8885a308d3ull, 0x13198a2e03707344ull, 0xa4093822299f31d0ull, 0x082efa98ec4e6c89ull};
    uint64_t n = 0;            // bytes consumed
    uint8_t tail[32];
    uint32_t nt = 0;           // bytes waiting in tail
    static uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
    void block(const uint8_t* p) {
        for (int l = 0; l < 4; ++l) {
            uint64_t w;
            __builtin_memcpy(&w, p + 8 * l, 8);
            h[l] = rotl(h[l] ^ (w * 0x9e3779b97f4a7c15ull), 29) * 0xbf58476d1ce4e5b9ull;
        }
    }
    void update(const void* data, size_t len) {
        const uint8_t* p = static_cast<const uint8_t*>(data);
        n += len;
        if (nt) {
            const size_t take = len < 32 - nt ? len : 32 - nt;
            __builtin_memcpy(tail + nt, p, take);
            nt += (uint32_t)take; p += take; len -= take;
            if (nt < 32) return;
            block(tail);
            nt = 0;
        }
        for (; len >= 32; p += 32, len -= 32) block(p);
        if (len) { __builtin_memcpy(tail, p, len); nt = (uint32_t)len; }
    }
    uint64_t final() const {
        Digest d = *this;
        if (d.nt) { __builtin_memset(d.tail + d.nt, 0, 32 - d.nt); d.block(d.tail); }
        uint64_t x = d.n * 0x94d049bb133111ebull;
        for (int l = 0; l < 4; ++l) x = rotl(x ^ d.h[l], 31) * 0x9e3779b97f4a7c15ull;
        return x ^ (x >> 29);
    }
};

// the tree digest's root: the block digests in file order, then the length
uint64_t tree_digest(const uint64_t* blocks, size_t n_blocks, uint64_t bytes);

// Pinned host slots for a writer's device reads (an engine keeps one, made at its first checkpoint):
// kRingSlots slots of kRingSlot bytes, each with an event marking its copies done.
constexpr int kRingSlots = 8;
constexpr size_t kRingSlot = 8ull << 20;   // (a multiple of kDigestBlock)
struct PinnedRing {
    char* slot[kRingSlots] = {};
    hipEvent_t ev[kRingSlots] = {};
    int device = 0;
    bool ready = false;
    bool init(int dev);      // allocates on first use
    void release();
};

// Writes `path`.tmp, then (commit) the trailer, fsync of the file, rename over `path` and fsync of
// the directory: after commit() returns true the new file is the durable one.  The file is assembled
// in slots of kRingSlot bytes, each one file range: host bytes are copied in (write), device bytes
// land by stream-ordered copies (write_dev, a PinnedRing's slots); a full slot goes to a pool of host
// threads that wait for its copies, hash its digest blocks and pwrite it at its offset, while the
// next slot fills.  Without a ring the slots are heap memory and each is written as it fills.
struct CkptWriter {
    struct Impl;
    Impl* im = nullptr;
    bool ok = false;
    explicit CkptWriter(const char* p, PinnedRing* ring = nullptr, hipStream_t stream = nullptr);
    ~CkptWriter();
    bool write(const void* data, size_t len);
    bool write_dev(const void* dev, size_t len);   // (a writer made with a ring)
    bool commit(uint64_t app_bytes, uint64_t* digest_out);
    const char* error() const;                      // what failed, when something did
};
// Reads a checkpoint file; verify() checks the trailer's digest (KMEDGST2: every block hashed again on
// host threads from the file; KMEDGST1: the stream hashed as it was read).
struct CkptReader {
    FILE* f = nullptr;
    Digest dg;
    std::string path;
    uint64_t size = 0;         // the file's size (trailer included)
    uint64_t pos = 0;          // bytes read
    bool tree = false;         // the trailer is KMEDGST2
    bool ok = false;
    explicit CkptReader(const char* p);
    ~CkptReader();
    bool read(void* data, size_t len);
    bool at_trailer() const;   // everything before the trailer consumed
    bool verify(CkptTrailer* t);
};
// fsync of the directory that holds `path` (a rename is durable only then)
bool sync_dir_of(const std::string& path);

// tests only (kme_runtime.cpp): env KME_TEST_FAIL == what
bool test_hook_fail(const char* what);

}  // namespace kme
