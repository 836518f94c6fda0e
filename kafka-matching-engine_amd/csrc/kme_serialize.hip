// kme_serialize.hip -- device serializer of a processed epoch (SURVEY.md §8 row f "next-1").
//
// The records the reference forwards for input i (KP:97 "IN", KP:272-273 maker / taker fills,
// KP:124 "OUT"), each serialised by JsonSerializer<Order> (KP:477-495: Jackson, creator
// properties in declaration order, null links) and printed as consumer.js prints MatchOut
// (consumer.js:19): "<key> <json>\n".  Byte-identical to the host kme_tape_json (kme_host.cpp).
//
// Two passes over the epoch, one thread per input record: k_ser_len computes each input's byte
// count, an exclusive scan (the DPP scan of kme_kernels.hip) turns the counts into offsets, and
// k_ser_write prints every input's lines at its offset.  Adjacent threads write adjacent byte
// ranges; a thread packs its bytes into aligned dwords and uses byte stores only for the partial
// words at the ends of its range.
#include <hip/hip_runtime.h>

#include "kme.h"
#include "kme_device.h"
#include "kme_launch.h"

namespace kme {

#define KDEV __device__ __forceinline__

// {"action":A,"oid":O,"aid":A,"sid":S,"price":P,"size":Z,"next":null,"prev":V}: the literal part
constexpr uint32_t ORDER_FIXED = 10 + 7 + 7 + 7 + 9 + 8 + 20 + 1;

KDEV uint32_t ndig(uint64_t u) {
    uint32_t n = 1;
    uint64_t p = 10;
    while (n < 20 && u >= p) { ++n; p *= 10; }
    return n;
}
KDEV uint32_t len_i64(int64_t v) { return (v < 0 ? 1u : 0u) + ndig(v < 0 ? 0ull - (uint64_t)v : (uint64_t)v); }
KDEV uint32_t order_len(int32_t action, int64_t oid, int64_t aid, int64_t sid, int32_t price, int32_t size,
                        bool has_prev, int64_t prev) {
    return ORDER_FIXED + len_i64(action) + len_i64(oid) + len_i64(aid) + len_i64(sid) + len_i64(price) +
           len_i64(size) + (has_prev ? len_i64(prev) : 4u);
}

struct SerIn {
    const int32_t* action;
    const int64_t *oid, *aid, *sid;
    const int32_t *price, *size;
};
struct SerRes {
    const int32_t* out_action;
    const int32_t* out_size;
    const int64_t* out_prev;
    const uint8_t* out_flags;
    const uint32_t* trade_off;
    const TradeRec* trades;
};

// Bytes of input i's lines: "IN " order "\n", per trade 2 x ("OUT " order "\n"), "OUT " order "\n".
KDEV uint64_t input_bytes(const SerIn& in, const SerRes& r, uint32_t i) {
    const int32_t a = in.action[i];
    const int64_t oid = in.oid[i], aid = in.aid[i], sid = in.sid[i];
    const int32_t price = in.price[i];
    uint64_t b = 3 + order_len(a, oid, aid, sid, price, in.size[i], false, 0) + 1;
    const bool taker_buy = a == BUY;
    for (uint32_t t = r.trade_off[i]; t < r.trade_off[i + 1]; ++t) {
        const TradeRec tr = r.trades[t];
        b += 4 + order_len(taker_buy ? SOLD : BOUGHT, tr.moid, tr.maid, tr.msid, 0, tr.size, false, 0) + 1;
        const int32_t dp = (int32_t)((uint32_t)price - (uint32_t)tr.mprice);
        b += 4 + order_len(taker_buy ? BOUGHT : SOLD, oid, aid, sid, dp, tr.size, false, 0) + 1;
    }
    b += 4 + order_len(r.out_action[i], oid, aid, sid, price, r.out_size[i], (r.out_flags[i] & KME_OUT_HAS_PREV) != 0,
                       r.out_prev[i]) + 1;
    return b;
}
// Per-input byte counts (u32, for the offset scan) and their exact u64 total (one atomic per block).
__global__ void __launch_bounds__(256) k_ser_len(SerIn in, SerRes r, uint32_t n, uint32_t* len,
                                                 unsigned long long* total) {
    __shared__ unsigned long long red[256];
    unsigned long long sum = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t b = input_bytes(in, r, i);
        len[i] = b > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)b;
        sum += b;
    }
    red[threadIdx.x] = sum;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0 && red[0]) atomicAdd(total, red[0]);
}

// Byte sink over [start, end) of the output: aligned dwords, byte stores at the ragged ends.
struct Sink {
    uint8_t* out;
    uint64_t start, pos;
    uint32_t acc;
    KDEV void put(uint8_t c) {
        const uint32_t k = (uint32_t)(pos & 3);
        acc = k == 0 ? (uint32_t)c : (acc | ((uint32_t)c << (8 * k)));
        if (k == 3) {
            const uint64_t w = pos - 3;
            if (w >= start) {
                *reinterpret_cast<uint32_t*>(out + w) = acc;
            } else {
                for (uint64_t q = start; q <= pos; ++q) out[q] = (uint8_t)(acc >> (8 * (q - w)));
            }
        }
        ++pos;
    }
    KDEV void flush() {
        const uint32_t k = (uint32_t)(pos & 3);
        if (k == 0) return;
        const uint64_t w = pos - k;
        for (uint64_t q = w > start ? w : start; q < pos; ++q) out[q] = (uint8_t)(acc >> (8 * (q - w)));
    }
    KDEV void lit(const char* s) {
#pragma nounroll
        while (*s) put((uint8_t)*s++);
    }
    // decimal digits of u < 10^9, most significant first (width w, zero padded when pad)
    KDEV void dig9(uint32_t u, bool pad) {
        uint32_t p = 100000000u;
        if (!pad) while (p > 1 && u < p) p /= 10;
#pragma nounroll
        for (; p; p /= 10) { put((uint8_t)('0' + u / p)); u %= p; }
    }
    // an int64 as decimal: at most three 9-digit chunks, each printed with 32-bit arithmetic
    KDEV void num(int64_t v) {
        uint64_t u = v < 0 ? 0ull - (uint64_t)v : (uint64_t)v;
        if (v < 0) put('-');
        const uint32_t c0 = (uint32_t)(u % 1000000000ull);
        u /= 1000000000ull;
        const uint32_t c1 = (uint32_t)(u % 1000000000ull);
        const uint32_t c2 = (uint32_t)(u / 1000000000ull);
        if (c2) { dig9(c2, false); dig9(c1, true); dig9(c0, true); }
        else if (c1) { dig9(c1, false); dig9(c0, true); }
        else dig9(c0, false);
    }
    KDEV void order(const char* key, int32_t action, int64_t oid, int64_t aid, int64_t sid, int32_t price, int32_t size,
                    bool has_prev, int64_t prev) {
        lit(key);
        lit("{\"action\":"); num(action);
        lit(",\"oid\":"); num(oid);
        lit(",\"aid\":"); num(aid);
        lit(",\"sid\":"); num(sid);
        lit(",\"price\":"); num(price);
        lit(",\"size\":"); num(size);
        lit(",\"next\":null,\"prev\":");
        if (has_prev) num(prev); else lit("null");
        lit("}\n");
    }
};

__global__ void __launch_bounds__(256) k_ser_write(SerIn in, SerRes r, uint32_t n, const uint32_t* off, uint8_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Sink s{out, off[i], off[i], 0};
    const int32_t a = in.action[i];
    const int64_t oid = in.oid[i], aid = in.aid[i], sid = in.sid[i];
    const int32_t price = in.price[i];
    s.order("IN ", a, oid, aid, sid, price, in.size[i], false, 0);
    const bool taker_buy = a == BUY;
    for (uint32_t t = r.trade_off[i]; t < r.trade_off[i + 1]; ++t) {
        const TradeRec tr = r.trades[t];
        s.order("OUT ", taker_buy ? SOLD : BOUGHT, tr.moid, tr.maid, tr.msid, 0, tr.size, false, 0);
        s.order("OUT ", taker_buy ? BOUGHT : SOLD, oid, aid, sid, (int32_t)((uint32_t)price - (uint32_t)tr.mprice),
                tr.size, false, 0);
    }
    s.order("OUT ", r.out_action[i], oid, aid, sid, price, r.out_size[i], (r.out_flags[i] & KME_OUT_HAS_PREV) != 0,
            r.out_prev[i]);
    s.flush();
}

static inline uint32_t cdiv_u(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

void launch_ser_len(const kme_orders& in, const kme_epoch_result& r, uint32_t n, uint32_t* len, unsigned long long* total,
                    hipStream_t st) {
    (void)hipMemsetAsync(total, 0, sizeof(unsigned long long), st);
    if (n == 0) return;
    SerIn si{in.action, in.oid, in.aid, in.sid, in.price, in.size};
    SerRes sr{r.out_action, r.out_size, r.out_prev, r.out_flags, r.trade_off, reinterpret_cast<const TradeRec*>(r.trades)};
    const uint32_t nb = cdiv_u(n, 256) < 2048 ? cdiv_u(n, 256) : 2048;
    hipLaunchKernelGGL(k_ser_len, dim3(nb), dim3(256), 0, st, si, sr, n, len, total);
}
void launch_ser_write(const kme_orders& in, const kme_epoch_result& r, uint32_t n, const uint32_t* off, void* out,
                      hipStream_t st) {
    if (n == 0) return;
    SerIn si{in.action, in.oid, in.aid, in.sid, in.price, in.size};
    SerRes sr{r.out_action, r.out_size, r.out_prev, r.out_flags, r.trade_off, reinterpret_cast<const TradeRec*>(r.trades)};
    hipLaunchKernelGGL(k_ser_write, dim3(cdiv_u(n, 256)), dim3(256), 0, st, si, sr, n, off, (uint8_t*)out);
}

}  // namespace kme
