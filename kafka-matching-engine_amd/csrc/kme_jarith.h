// kme_jarith.h -- device helpers shared by the kernel translation units (kme_kernels.hip,
// kme_ledger.hip): Java int / long arithmetic (two's-complement wrap-around, as the reference's
// `int` and `long` fields compute, KP:172-176, 286, 331), the 64-bit mixer of the hash tables, and
// the epoch's error word (kme.h kme_epoch_status).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kme.h"
#include "kme_device.h"

namespace kme {

#define KDEV __device__ __forceinline__
#define KC __attribute__((address_space(4)))   // constant address space: scalar loads

// ------------------------------------------------------------------ Java arithmetic (wraps)
KDEV int32_t jiadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
KDEV int32_t jisub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
KDEV int32_t jimul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
KDEV int32_t jineg(int32_t a) { return (int32_t)(0u - (uint32_t)a); }
KDEV int64_t jladd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
KDEV int64_t jlsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
KDEV int64_t jlmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }
KDEV int64_t jlneg(int64_t a) { return (int64_t)(0ull - (uint64_t)a); }
KDEV int64_t lmax(int64_t a, int64_t b) { return a >= b ? a : b; }
KDEV int64_t lmin(int64_t a, int64_t b) { return a <= b ? a : b; }
KDEV int32_t imin(int32_t a, int32_t b) { return a <= b ? a : b; }

KDEV int lane_id() { return (int)(threadIdx.x & 63); }

KDEV uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// ------------------------------------------------------------------ the epoch's error word
// (index << 16) | (detail << 8) | status; UINT64_MAX = none.  atomicMin keeps the earliest fault.
KDEV uint64_t err_code(int status, int detail, int64_t idx) {
    uint64_t ix = idx < 0 ? 0xFFFFFFFFFFFFull : (uint64_t)idx;
    return (ix << 16) | ((uint64_t)(detail & 0xFF) << 8) | (uint64_t)(status & 0xFF);
}
KDEV void raise_thread(unsigned long long* ctr, int status, int detail, int64_t idx) {
    atomicMin(&ctr[ci(C_ERR)], (unsigned long long)err_code(status, detail, idx));
}
KDEV void raise_wave(unsigned long long* ctr, int status, int detail, int64_t idx) {
    // every lane issues the (idempotent) atomicMin: a lane-0 branch here, inside the matching
    // loops, makes the compiler treat their exits as divergent (uniform state moves to VGPRs)
    atomicMin(&ctr[ci(C_ERR)], (unsigned long long)err_code(status, detail, idx));
}
KDEV bool failed(const unsigned long long* ctr) {
    return __hip_atomic_load(&ctr[ci(C_ERR)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ~0ull;
}
// The records of the epoch that still take effect: every record before the first fault raised so
// far (the reference forwards and commits each record before the one that throws, KP:97, 124-125);
// none after a fault of the epoch as a whole (no index: the funded proof, trade capacity).
KDEV uint32_t err_limit(const unsigned long long* ctr, uint32_t n) {
    const unsigned long long c = __hip_atomic_load(&ctr[ci(C_ERR)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (c == ~0ull) return n;
    const unsigned long long ix = c >> 16;
    if (ix == 0xFFFFFFFFFFFFull) return 0;
    return ix < n ? (uint32_t)ix : n;
}

}  // namespace kme
