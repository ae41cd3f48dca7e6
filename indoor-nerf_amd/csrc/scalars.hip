// Per-step scalars of a captured training step (graphs.StepScalars): the graph's first launch copies
// this replay's slot of a host ring into the device slots the other launches read. The host fills
// slot (replay index mod n_slots) before the replay; a device counter advanced by this launch picks
// the same slot, so nothing is queued between two replays (the pinned host->device copy and the event
// guarding its slot that this replaces cost 8 us per step, profiles/r04zf_ab_upload.jsonl).
#include "common.h"

namespace nerf {

// ctl[0]: replays so far; ctl[1]: words of range A (at word 0); ctl[2]: first word of range B;
// ctl[3]: words of range B. One block: every thread reads ctl[0] before thread 0 advances it, and
// publishes the new count to the host (done, in the mapped ring) once every slot word is read (each
// load's value was stored before the barrier): the host reuses a slot only after the fetch that read
// it, with no event between replays. A relaxed store: a release at system scope compiles to a
// write-back of the whole L2 (the previous step's dirty lines) before it.
// With `done`, the last 8 bytes of a slot carry the index of the replay the host wrote it for: a slot
// whose tag is not this fetch's count (a replay without its upload: the slot still holds an earlier
// replay's scalars) sets the sticky error word behind `done` to count + 1, which the host checks at
// its next upload — the step would otherwise run on another step's seeds and coefficients.
__global__ void __launch_bounds__(256) scalars_fetch_kernel(const uint32_t* ring, int64_t slot_words, int n_slots,
                                                           int64_t* ctl, uint32_t* dst, int64_t* done) {
    const int64_t c = ctl[0];
    const int64_t na = ctl[1], b0 = ctl[2], nb = ctl[3];
    const uint32_t* src = ring + (c % n_slots) * slot_words;
    if (done && threadIdx.x == 0) {
        // both host words in one round trip (the error word is read whether or not the tag matches)
        const int64_t tag = __hip_atomic_load(reinterpret_cast<const int64_t*>(src + slot_words - 2), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_SYSTEM);
        const int64_t err = __hip_atomic_load(done + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (tag != c && err == 0) __hip_atomic_store(done + 1, c + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    for (int64_t i = threadIdx.x; i < na + nb; i += blockDim.x) {
        const int64_t w = i < na ? i : b0 + (i - na);
        // system scope: the host wrote the slot after this ring was last read; no cached copy is used
        dst[w] = __hip_atomic_load(src + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        ctl[0] = c + 1;
        if (done) __hip_atomic_store(done, c + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace nerf

using namespace nerf;

extern "C" int nerf_host_ring_alloc(int64_t n_bytes, void** host) {
    NERF_REQUIRE(n_bytes > 0 && host, "host_ring_alloc: %lld bytes", (long long)n_bytes);
    *host = nullptr;
    const hipError_t e = hipHostMalloc(host, (size_t)n_bytes, hipHostMallocMapped | hipHostMallocCoherent);
    NERF_REQUIRE(e == hipSuccess, "host_ring_alloc: hipHostMalloc(%lld): %s", (long long)n_bytes,
                 hipGetErrorString(e));
    return NERF_OK;
}

extern "C" int nerf_host_ring_free(void* host) {
    if (!host) return NERF_OK;
    const hipError_t e = hipHostFree(host);
    NERF_REQUIRE(e == hipSuccess, "host_ring_free: %s", hipGetErrorString(e));
    return NERF_OK;
}

extern "C" int nerf_scalars_fetch(const void* host_ring, int64_t slot_bytes, int n_slots, int64_t done_offset,
                                  int64_t* d_ctl, void* d_dst, void* stream) {
    NERF_REQUIRE(host_ring && d_ctl && d_dst && n_slots >= 1 && slot_bytes > 0 && slot_bytes % 4 == 0,
                 "scalars_fetch: ring %p ctl %p dst %p slots %d slot_bytes %lld", host_ring, (void*)d_ctl, d_dst,
                 n_slots, (long long)slot_bytes);
    NERF_REQUIRE(done_offset < 0 || (done_offset >= n_slots * slot_bytes && done_offset % 8 == 0 && slot_bytes % 8 == 0),
                 "scalars_fetch: done_offset %lld overlaps the slots or is unaligned (slot_bytes %lld)",
                 (long long)done_offset, (long long)slot_bytes);
    void* dev_ring = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&dev_ring, const_cast<void*>(host_ring), 0);
    NERF_REQUIRE(e == hipSuccess, "scalars_fetch: ring is not mapped host memory (%s)", hipGetErrorString(e));
    hipLaunchKernelGGL(scalars_fetch_kernel, dim3(1), dim3(256), 0, as_stream(stream),
                       static_cast<const uint32_t*>(dev_ring), slot_bytes / 4, n_slots, d_ctl,
                       static_cast<uint32_t*>(d_dst),
                       done_offset < 0 ? nullptr
                                       : reinterpret_cast<int64_t*>(static_cast<char*>(dev_ring) + done_offset));
    NERF_CHECK_LAUNCH("scalars_fetch");
    return NERF_OK;
}
