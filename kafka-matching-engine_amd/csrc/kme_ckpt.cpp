// kme_ckpt.cpp -- the checkpoint files' writer and reader (kme_internal.h): a file assembled in
// fixed slots that host threads hash and write while the next slot fills, a tree digest in the
// trailer, and its verification on host threads.
//
// The commit point of the drop-in writes the whole device state (the reference's
// changelogged stores, KP:30-49, committed after every record, KP:125).  At the C3 shape that is ~1 GB,
// and one Digest over the stream runs at ~4 GB/s on one host core -- most of a commit's time.  Here
// every kDigestBlock bytes are hashed on their own (in parallel, by the thread that writes their
// slot), and the trailer holds the digest of the block digests: the file's bytes still decide it, and
// a reader checks it block-parallel again.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>

#include "kme_internal.h"

namespace kme {

uint64_t tree_digest(const uint64_t* blocks, size_t n_blocks, uint64_t bytes) {
    Digest d;
    d.update(blocks, n_blocks * sizeof(uint64_t));
    d.update(&bytes, sizeof bytes);
    return d.final();
}

static bool pwrite_full(int fd, const char* p, size_t n, uint64_t off) {
    while (n) {
        const ssize_t w = ::pwrite(fd, p, n, (off_t)off);
        if (w <= 0) return false;
        p += w; n -= (size_t)w; off += (uint64_t)w;
    }
    return true;
}
static bool pread_full(int fd, char* p, size_t n, uint64_t off) {
    while (n) {
        const ssize_t r = ::pread(fd, p, n, (off_t)off);
        if (r <= 0) return false;
        p += r; n -= (size_t)r; off += (uint64_t)r;
    }
    return true;
}
static void block_digests(const char* p, size_t len, std::vector<uint64_t>& out) {
    for (size_t b = 0; b < len; b += kDigestBlock) {
        Digest d;
        d.update(p + b, std::min<size_t>(kDigestBlock, len - b));
        out.push_back(d.final());
    }
}
static unsigned host_threads(unsigned cap) {
    return std::max(1u, std::min(cap, std::thread::hardware_concurrency()));
}

bool PinnedRing::init(int dev) {
    if (ready) return true;
    device = dev;
    for (int k = 0; k < kRingSlots; ++k) {
        if (hipHostMalloc((void**)&slot[k], kRingSlot, hipHostMallocDefault) != hipSuccess ||
            hipEventCreateWithFlags(&ev[k], hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            release();
            return false;
        }
    }
    ready = true;
    return true;
}
void PinnedRing::release() {
    for (int k = 0; k < kRingSlots; ++k) {
        if (slot[k]) (void)hipHostFree(slot[k]);
        if (ev[k]) (void)hipEventDestroy(ev[k]);
        slot[k] = nullptr;
        ev[k] = nullptr;
    }
    ready = false;
}

// ------------------------------------------------------------------ writer
struct CkptWriter::Impl {
    std::string path, tmp;
    int fd = -1;
    PinnedRing* ring = nullptr;
    hipStream_t stream = nullptr;
    std::vector<char> heap;                  // the one slot of a writer without a ring
    int nslots = 1;
    int cur = 0;                             // the slot being filled
    size_t fill = 0;                         // its bytes
    bool cur_dev = false;                    // it has device copies in flight
    uint64_t base = 0;                       // its file offset
    struct Job {
        int slot;
        uint64_t off;
        size_t len;
        bool dev;
        std::vector<uint64_t> dg;            // its blocks' digests
    };
    std::deque<Job> jobs;                    // every slot submitted, in file order
    std::mutex mu;
    std::condition_variable cv;
    bool busy[kRingSlots] = {};
    std::deque<size_t> queue;                // jobs to run
    size_t running = 0;
    std::vector<std::thread> th;
    bool stop = false;
    std::atomic<bool> fail{false};
    std::string err;

    char* slot_ptr(int s) { return ring ? ring->slot[s] : heap.data(); }
    void set_err(const char* what) {
        std::lock_guard<std::mutex> g(mu);
        if (err.empty()) err = what;
        fail = true;
    }
    bool run(Job& j) {
        if (j.dev && hipEventSynchronize(ring->ev[j.slot]) != hipSuccess) { set_err("device read"); return false; }
        const char* p = slot_ptr(j.slot);
        block_digests(p, j.len, j.dg);
        if (!pwrite_full(fd, p, j.len, j.off)) { set_err("file write"); return false; }
        // start the slot's write-back now, so that commit()'s fsync finds most of the file on disk
        // (the disk works while later slots are copied and hashed)
        (void)::sync_file_range(fd, (off64_t)j.off, (off64_t)j.len, SYNC_FILE_RANGE_WRITE);
        return true;
    }
    void worker() {
        if (ring) (void)hipSetDevice(ring->device);
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return stop || !queue.empty(); });
            if (queue.empty()) return;
            const size_t k = queue.front();
            queue.pop_front();
            ++running;
            Job& j = jobs[k];                // (a deque keeps its elements where they are)
            lk.unlock();
            if (!fail) (void)run(j);
            lk.lock();
            --running;
            busy[j.slot] = false;
            cv.notify_all();
        }
    }
    // the current slot is free to fill
    void acquire() {
        if (!ring) return;
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return !busy[cur]; });
    }
    void submit() {
        if (fill == 0) return;
        if (cur_dev && hipEventRecord(ring->ev[cur], stream) != hipSuccess) set_err("device read");
        if (!ring) {
            jobs.push_back(Job{cur, base, fill, cur_dev, {}});
            if (!fail) (void)run(jobs.back());
        } else {
            if (th.empty()) {
                const unsigned T = host_threads(12);
                for (unsigned t = 0; t < T; ++t) th.emplace_back([this] { worker(); });
            }
            // (under the lock: a worker indexes `jobs` under it, and push_back may move the deque's
            // block map -- the elements themselves stay where they are)
            std::lock_guard<std::mutex> g(mu);
            jobs.push_back(Job{cur, base, fill, cur_dev, {}});
            busy[cur] = true;
            queue.push_back(jobs.size() - 1);
            cv.notify_all();
        }
        base += fill;
        fill = 0;
        cur_dev = false;
        cur = (cur + 1) % nslots;
    }
    void drain() {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return queue.empty() && running == 0; });
            stop = true;
        }
        cv.notify_all();
        for (auto& t : th) t.join();
        th.clear();
    }
};

CkptWriter::CkptWriter(const char* p, PinnedRing* ring, hipStream_t stream) : im(new Impl) {
    im->path = p;
    im->tmp = std::string(p) + ".tmp";
    im->ring = ring && ring->ready ? ring : nullptr;
    im->stream = stream;
    im->nslots = im->ring ? kRingSlots : 1;
    if (!im->ring) im->heap.resize(kRingSlot);
    im->fd = ::open(im->tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    ok = im->fd >= 0;
    if (!ok) im->err = "file open";
}
CkptWriter::~CkptWriter() {
    if (!im) return;
    // (a writer that failed may leave device copies into a slot it never submitted: drained, so that
    // the next writer's host bytes in that slot cannot be overwritten by them)
    if (im->ring && hipStreamSynchronize(im->stream) != hipSuccess) (void)hipGetLastError();
    im->drain();                             // (nothing may still read a slot or write the file)
    if (im->fd >= 0) {
        ::close(im->fd);
        std::remove(im->tmp.c_str());
    }
    delete im;
}
bool CkptWriter::write(const void* data, size_t len) {
    const char* p = static_cast<const char*>(data);
    while (ok && len) {
        im->acquire();
        const size_t c = std::min(len, kRingSlot - im->fill);
        std::memcpy(im->slot_ptr(im->cur) + im->fill, p, c);
        im->fill += c;
        p += c;
        len -= c;
        if (im->fill == kRingSlot) im->submit();
        ok = !im->fail;
    }
    return ok;
}
bool CkptWriter::write_dev(const void* dev, size_t len) {
    if (!im->ring) { ok = false; im->err = "device read without a ring"; return false; }
    const char* p = static_cast<const char*>(dev);
    while (ok && len) {
        im->acquire();
        const size_t c = std::min(len, kRingSlot - im->fill);
        if (hipMemcpyAsync(im->slot_ptr(im->cur) + im->fill, p, c, hipMemcpyDeviceToHost, im->stream) != hipSuccess) {
            (void)hipGetLastError();
            im->set_err("device read");
            ok = false;
            return false;
        }
        im->cur_dev = true;
        im->fill += c;
        p += c;
        len -= c;
        if (im->fill == kRingSlot) im->submit();
        ok = !im->fail;
    }
    return ok;
}
bool CkptWriter::commit(uint64_t app_bytes, uint64_t* digest_out) {
    if (!ok) return false;
    im->submit();
    im->drain();
    if (im->fail) { ok = false; return false; }
    std::vector<uint64_t> blocks;
    for (const Impl::Job& j : im->jobs) blocks.insert(blocks.end(), j.dg.begin(), j.dg.end());
    CkptTrailer t{};
    t.app_bytes = app_bytes;
    t.digest = tree_digest(blocks.data(), blocks.size(), im->base);
    std::memcpy(t.magic, kTrailerMagic2, sizeof t.magic);
    ok = pwrite_full(im->fd, reinterpret_cast<const char*>(&t), sizeof t, im->base);
    ok = ::fsync(im->fd) == 0 && ok;
    ok = ::close(im->fd) == 0 && ok;
    im->fd = -1;
    ok = ok && std::rename(im->tmp.c_str(), im->path.c_str()) == 0;
    if (!ok) {
        std::remove(im->tmp.c_str());
        if (im->err.empty()) im->err = "file commit";
        return false;
    }
    ok = sync_dir_of(im->path);
    if (digest_out) *digest_out = t.digest;
    return ok;
}
const char* CkptWriter::error() const { return im->err.empty() ? "" : im->err.c_str(); }

// ------------------------------------------------------------------ reader
CkptReader::CkptReader(const char* p) : path(p) {
    f = std::fopen(p, "rb");
    if (!f) return;
    ok = std::fseek(f, 0, SEEK_END) == 0;
    const long sz = ok ? std::ftell(f) : -1;
    ok = ok && sz >= (long)sizeof(CkptTrailer);
    size = sz > 0 ? (uint64_t)sz : 0;
    CkptTrailer t{};
    ok = ok && std::fseek(f, sz - (long)sizeof t, SEEK_SET) == 0 && std::fread(&t, sizeof t, 1, f) == 1;
    tree = ok && std::memcmp(t.magic, kTrailerMagic2, sizeof t.magic) == 0;
    ok = ok && std::fseek(f, 0, SEEK_SET) == 0;
}
CkptReader::~CkptReader() {
    if (f) std::fclose(f);
}
bool CkptReader::read(void* data, size_t len) {
    if (!ok) return false;
    if (pos + len + sizeof(CkptTrailer) > size) { ok = false; return false; }   // (never into the trailer)
    if (tree && len >= (32u << 20)) {   // a large store: pread on host threads (the digest is checked after)
        const int fd = ::fileno(f);
        const unsigned T = host_threads(8);
        const size_t part = (len / T + 4095) & ~(size_t)4095;
        std::vector<int> good(T, 1);
        std::vector<std::thread> th;
        for (unsigned w = 0; w < T; ++w)
            th.emplace_back([&, w] {
                const size_t a = std::min(len, (size_t)w * part), b = std::min(len, a + part);
                if (b > a && !pread_full(fd, static_cast<char*>(data) + a, b - a, pos + a)) good[w] = 0;
            });
        for (auto& x : th) x.join();
        for (int g : good) ok = ok && g;
        ok = ok && std::fseek(f, (long)(pos + len), SEEK_SET) == 0;
        if (ok) pos += len;
        return ok;
    }
    ok = len == 0 || std::fread(data, 1, len, f) == len;
    if (ok && !tree) dg.update(data, len);
    if (ok) pos += len;
    return ok;
}
bool CkptReader::at_trailer() const { return ok && pos + sizeof(CkptTrailer) == size; }
bool CkptReader::verify(CkptTrailer* t) {
    if (!at_trailer()) return false;
    ok = std::fread(t, sizeof *t, 1, f) == 1;
    if (!ok) return false;
    if (!tree) {
        ok = std::memcmp(t->magic, kTrailerMagic, sizeof t->magic) == 0 && t->digest == dg.final();
        return ok;
    }
    // every block hashed again from the file, on host threads (the bytes read are in the page cache)
    const uint64_t n = pos;
    const size_t nb = (size_t)((n + kDigestBlock - 1) / kDigestBlock);
    std::vector<uint64_t> blocks(nb);
    const int fd = ::fileno(f);                       // (the inode read so far, whatever `path` names now)
    const unsigned T = (unsigned)std::min<size_t>(std::max<size_t>(nb, 1), host_threads(16));
    std::vector<int> good(T, 1);
    std::vector<std::thread> th;
    for (unsigned w = 0; w < T; ++w)
        th.emplace_back([&, w] {
            std::vector<char> buf(kDigestBlock);
            for (size_t k = w; k < nb; k += T) {
                const uint64_t at = (uint64_t)k * kDigestBlock;
                const size_t len = (size_t)std::min<uint64_t>(kDigestBlock, n - at);
                if (!pread_full(fd, buf.data(), len, at)) { good[w] = 0; return; }
                Digest d;
                d.update(buf.data(), len);
                blocks[k] = d.final();
            }
        });
    for (auto& x : th) x.join();
    for (int g : good) ok = ok && g;
    ok = ok && t->digest == tree_digest(blocks.data(), nb, n);
    return ok;
}

}  // namespace kme
