// capi.cpp — the extern "C" boundary declared in include/decds_rlnc.h: context management,
// argument checking, status mapping onto DecdsError (decds-lib/src/errors.rs) and the batch
// launchers. Every compute entry point runs the gfx950 kernels; there is no host fallback.
#include <hip/hip_runtime.h>

#include <atomic>

#include <cstdlib>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/decds_rlnc.h"
#include "capi_internal.h"
#include "rlnc_kernels.h"
#include "rlnc_layout.h"

using namespace decds;

static thread_local std::string g_last_error;
static std::atomic<int> g_live_ctx{0};  // contexts created and not yet destroyed
// hip_status.h: set when the error being reported was found pending before a launch (an earlier
// call's, not the launch's); decds_hip_error names it as such
static thread_local std::string g_pending_before;

namespace decds {
void hip_tolerate(hipError_t e, const char *what) {
    (void)what;  // the call site names the tolerated failure; nothing is reported
    if (e != hipSuccess) (void)hipGetLastError();  // consumed here, never a later launch's
}

hipError_t hip_launch_begin(const char *kernel) {
    const hipError_t p = hipPeekAtLastError();
    if (p == hipSuccess) return hipSuccess;
    (void)hipGetLastError();
    // the library consumes every failure it reports (decds_hip_error) or tolerates (hip_tolerate), so
    // an error pending here was left by a HIP call outside the library on this thread
    g_pending_before = std::string("left pending before launching ") + kernel +
                       " by an earlier HIP call on this thread, outside the library (not this launch's)";
    return p;
}
}  // namespace decds

int decds_set_error(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

int decds_hip_error(hipError_t e, const char *what) {
    (void)hipGetLastError();  // reported here: the thread's error slot is left clean for later launches
    if (!g_pending_before.empty()) {  // not this call's failure (hip_launch_begin)
        std::string note;
        note.swap(g_pending_before);
        return decds_set_error(DECDS_ERR_HIP, "%s: %s (%d) %s", what, hipGetErrorString(e), (int)e, note.c_str());
    }
    return decds_set_error(DECDS_ERR_HIP, "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
}

int decds_ctx_bind(const decds_ctx *ctx) {
    if (!ctx) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null context");
    hipError_t e = hipSetDevice(ctx->device);
    return e == hipSuccess ? DECDS_OK : decds_hip_error(e, "hipSetDevice");
}

hipError_t decds_ctx_scratch(decds_ctx *ctx, size_t bytes, uint8_t **out) {
    if (ctx->host_scratch_cap < bytes) {
        if (ctx->host_scratch) hip_tolerate(hipFree(ctx->host_scratch), "hipFree");
        ctx->host_scratch = nullptr;
        ctx->host_scratch_cap = 0;
        hipError_t e = hipMalloc(reinterpret_cast<void **>(&ctx->host_scratch), bytes);
        if (e) return e;
        ctx->host_scratch_cap = bytes;
    }
    *out = ctx->host_scratch;
    return hipSuccess;
}

hipError_t decds_ctx_host_small(decds_ctx *ctx, size_t bytes, uint8_t **out) {
    if (ctx->host_small_cap < bytes) {
        if (ctx->host_small) hip_tolerate(hipHostFree(ctx->host_small), "hipHostFree");
        ctx->host_small = nullptr;
        ctx->host_small_cap = 0;
        hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&ctx->host_small), bytes, DECDS_HOST_MALLOC_FLAGS);
        if (e) {
            (void)hipGetLastError();  // this call's own error, returned
            return e;
        }
        ctx->host_small_cap = bytes;
    }
    *out = ctx->host_small;
    return hipSuccess;
}

extern "C" {

const char *decds_last_error(void) { return g_last_error.c_str(); }

const char *decds_status_string(int s) {
    switch (s) {
        case DECDS_OK: return "ok";
        case DECDS_ERR_INVALID_CHUNKSET_SIZE: return "invalid chunkset size";
        case DECDS_ERR_INVALID_CHUNK_METADATA: return "invalid chunk metadata";
        case DECDS_ERR_CHUNKSET_READY_TO_REPAIR: return "chunkset ready to repair";
        case DECDS_ERR_CHUNK_DECODING_FAILED: return "chunk decoding failed";
        case DECDS_ERR_CHUNKSET_NOT_YET_READY: return "chunkset not yet ready to repair";
        case DECDS_ERR_CHUNKSET_REPAIRING_FAILED: return "chunkset repairing failed";
        case DECDS_ERR_INVALID_SHARE_ID: return "invalid erasure coded share id";
        case DECDS_ERR_EMPTY_DATA_FOR_BLOB: return "empty data for blob";
        case DECDS_ERR_INVALID_CHUNKSET_ID: return "invalid chunkset id";
        case DECDS_ERR_CHUNKSET_ALREADY_REPAIRED: return "chunkset already repaired";
        case DECDS_ERR_INVALID_PROOF_IN_CHUNK: return "invalid proof in chunk";
        case DECDS_ERR_BLOB_HEADER_SERIALIZATION_FAILED: return "failed to serialize blob header";
        case DECDS_ERR_BLOB_HEADER_DESERIALIZATION_FAILED: return "failed to deserialize blob header";
        case DECDS_ERR_PCC_SERIALIZATION_FAILED: return "failed to serialize proof carrying chunk";
        case DECDS_ERR_PCC_DESERIALIZATION_FAILED: return "failed to deserialize proof carrying chunk";
        case DECDS_ERR_INVALID_START_BOUND: return "invalid start bound";
        case DECDS_ERR_INVALID_END_BOUND: return "invalid end bound";
        case DECDS_ERR_HIP: return "HIP runtime error";
        case DECDS_ERR_INVALID_ARGUMENT: return "invalid argument";
        case DECDS_ERR_NO_DEVICE: return "no gfx950 device";
        case DECDS_ERR_OUT_OF_DEVICE_MEMORY: return "out of device memory";
        default: return "unknown status";
    }
}

int decds_device_count(void) {
    int n = 0;
    const hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        hip_tolerate(e, "hipGetDeviceCount");  // no device: 0, and the thread's error slot left clean
        return 0;
    }
    return n;
}

int decds_ctx_create(int device, decds_ctx **out) {
    if (!out) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null out pointer");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    hip_tolerate(e, "hipGetDeviceCount");  // reported as DECDS_ERR_NO_DEVICE below, not left pending
    if (e != hipSuccess || n == 0)
        return decds_set_error(DECDS_ERR_NO_DEVICE, "no HIP device visible (%s)",
                               e == hipSuccess ? "count 0" : hipGetErrorString(e));
    if (device < 0 || device >= n)
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "device %d out of range [0,%d)", device, n);
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) return decds_hip_error(e, "hipGetDeviceProperties");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return decds_set_error(DECDS_ERR_NO_DEVICE, "device %d is %s; these kernels are built for gfx950 only",
                               device, prop.gcnArchName);
    if ((e = hipSetDevice(device)) != hipSuccess) return decds_hip_error(e, "hipSetDevice");
    if ((e = configure_kernels()) != hipSuccess) return decds_hip_error(e, "hipFuncSetAttribute");
    decds_ctx *c = new decds_ctx;
    c->device = device;
    c->poly = POLY_DEFAULT;
    c->marker = (uint8_t)MARKER_DEFAULT;
    c->gen = host_gf_generator(POLY_DEFAULT);
    c->geom.num_cus = prop.multiProcessorCount;
    configure_geom(c->geom);
    if ((e = hipMalloc(reinterpret_cast<void **>(&c->geom.counters),
                       LaunchGeom::N_COUNTERS * LaunchGeom::COUNTER_STRIDE * sizeof(uint32_t))) != hipSuccess) {
        delete c;
        return decds_hip_error(e, "hipMalloc (tile counters)");
    }
    if ((e = hipMemset(c->geom.counters, 0, LaunchGeom::N_COUNTERS * LaunchGeom::COUNTER_STRIDE * sizeof(uint32_t))) !=
        hipSuccess) {
        hip_tolerate(hipFree(c->geom.counters), "hipFree");
        delete c;
        return decds_hip_error(e, "hipMemset (tile counters)");
    }
    g_live_ctx.fetch_add(1);
    *out = c;
    return DECDS_OK;
}

int decds_ctx_destroy(decds_ctx *ctx) {
    if (!ctx) return DECDS_OK;
    hip_tolerate(hipSetDevice(ctx->device), "hipSetDevice");
    decds_lanes_destroy(ctx);
    if (ctx->pipe) decds::pipe_destroy(ctx->pipe);  // drains its streams first
    if (ctx->host_scratch) hip_tolerate(hipFree(ctx->host_scratch), "hipFree");
    if (ctx->host_small) hip_tolerate(hipHostFree(ctx->host_small), "hipHostFree");
    // the last context out returns the cached page-locked blocks (no idle pinned memory)
    if (g_live_ctx.fetch_sub(1) == 1) (void)host_cache_trim();
    if (ctx->geom.counters) {
        hip_tolerate(hipDeviceSynchronize(), "hipDeviceSynchronize");  // no launch may still count on them
        hip_tolerate(hipFree(ctx->geom.counters), "hipFree");
    }
    delete ctx;
    return DECDS_OK;
}

int decds_device_status(const decds_ctx *ctx) {
    int s = decds_ctx_bind(ctx);
    if (s) return s;
    // a sticky device fault surfaces here; report it rather than whichever call runs next
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return decds_hip_error(e, "device status");
    e = hipGetLastError();
    return e == hipSuccess ? DECDS_OK : decds_hip_error(e, "device status (last error)");
}

int decds_ctx_set_field(decds_ctx *ctx, uint32_t poly, uint8_t marker) {
    if (!ctx) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null context");
    if (poly < 0x100 || poly > 0x1FF) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "poly must be degree 8");
    if (marker == 0) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "marker must be non-zero");
    const uint32_t gen = host_gf_generator(poly);
    if (gen == 0) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "poly 0x%X is reducible: no GF(2^8)", poly);
    ctx->gen = gen;
    ctx->poly = poly;
    ctx->marker = marker;
    return DECDS_OK;
}

int decds_ctx_get_field(const decds_ctx *ctx, uint32_t *poly, uint8_t *marker) {
    if (!ctx) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null context");
    if (poly) *poly = ctx->poly;
    if (marker) *marker = ctx->marker;
    return DECDS_OK;
}

static int check_pitch(size_t pitch) {
    if (pitch < F)
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "coded pitch %zu < %llu", pitch, (unsigned long long)F);
    if ((N - 1) * (uint64_t)pitch + F >= (1ull << 31))  // row offsets stay inside a 2 GiB buffer descriptor
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "coded pitch %zu too large", pitch);
    return DECDS_OK;
}

static int check_n(size_t n) {
    if (n == 0 || n > (1u << 24))
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "chunkset count %zu outside [1, 2^24]", n);
    return DECDS_OK;
}

int decds_encode_batch(decds_ctx *ctx, const uint8_t *src, size_t n, const uint8_t *coeffs,
                       uint8_t *dst, size_t dst_pitch, void *stream) {
    int s;
    if ((s = decds_ctx_bind(ctx)) || (s = check_n(n)) || (s = check_pitch(dst_pitch))) return s;
    if (!src || !coeffs || !dst) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null buffer");
    hipError_t e = launch_encode(ctx->geom, src, n, coeffs, dst, dst_pitch, ctx->poly, ctx->marker,
                                 (hipStream_t)stream);
    return e == hipSuccess ? DECDS_OK : decds_hip_error(e, "rlnc_encode_kernel launch");
}

const char *decds_encode_kernel_name(size_t n_chunksets) { return encode_kernel_name(n_chunksets); }
const char *decds_decode_kernel_name(size_t n_chunksets) { return decode_kernel_name(n_chunksets); }
uint64_t decds_tuning(const char *name, uint64_t value, int set) {
    return name ? set_tuning(name, value, set != 0) : UINT64_MAX;
}

int decds_repair_plan_batch(decds_ctx *ctx, const uint8_t *coded, size_t coded_pitch, size_t n,
                            const uint8_t *cand, uint8_t *plan, int8_t *verdicts, int32_t *status,
                            void *stream) {
    int s;
    if ((s = decds_ctx_bind(ctx)) || (s = check_n(n)) || (s = check_pitch(coded_pitch))) return s;
    if (!coded || !cand || !plan || !verdicts || !status)
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null buffer");
    hipError_t e = launch_repair_plan(coded, coded_pitch, n, cand, plan, verdicts, status, ctx->poly,
                                      ctx->gen, (hipStream_t)stream);
    return e == hipSuccess ? DECDS_OK : decds_hip_error(e, "rlnc_plan_kernel launch");
}

int decds_decode_batch(decds_ctx *ctx, const uint8_t *coded, size_t coded_pitch, size_t n,
                       const uint8_t *plan, uint8_t *dst, int32_t *status, decds_repair_info *info,
                       void *stream) {
    int s;
    if ((s = decds_ctx_bind(ctx)) || (s = check_n(n)) || (s = check_pitch(coded_pitch))) return s;
    if (!coded || !plan || !dst || !status) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null buffer");
    if (reinterpret_cast<uintptr_t>(info) & 3u) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "info not 4-byte aligned");
    hipError_t e = launch_decode(ctx->geom, coded, coded_pitch, n, plan, dst, status, nullptr, nullptr, ctx->poly,
                                 ctx->marker, reinterpret_cast<uint8_t *>(info), (hipStream_t)stream);
    return e == hipSuccess ? DECDS_OK : decds_hip_error(e, "rlnc_decode_kernel launch");
}

int decds_repair_batch(decds_ctx *ctx, const uint8_t *coded, size_t coded_pitch, size_t n,
                       const uint8_t *cand, uint8_t *plan, int8_t *verdicts, uint8_t *dst,
                       int32_t *status, decds_repair_info *info, void *stream) {
    int s;
    if ((s = decds_ctx_bind(ctx)) || (s = check_n(n)) || (s = check_pitch(coded_pitch))) return s;
    if (!coded || !cand || !plan || !verdicts || !dst || !status)
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null buffer");
    if (reinterpret_cast<uintptr_t>(info) & 3u) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "info not 4-byte aligned");
    hipError_t e = launch_repair(ctx->geom, coded, coded_pitch, n, cand, plan, verdicts, dst, status, ctx->poly, ctx->gen,
                                 ctx->marker, reinterpret_cast<uint8_t *>(info), (hipStream_t)stream);
    return e == hipSuccess ? DECDS_OK : decds_hip_error(e, "repair launch");
}

const char *decds_repair_kernel_name(size_t n_chunksets) { return repair_kernel_name(n_chunksets); }

int decds_fill_random_device(decds_ctx *ctx, uint64_t seed, uint64_t byte_offset, uint8_t *dst,
                             size_t nbytes, void *stream) {
    int s;
    if ((s = decds_ctx_bind(ctx))) return s;
    if (!dst && nbytes) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null buffer");
    hipError_t e = launch_fill_random(seed, byte_offset, dst, nbytes, (hipStream_t)stream);
    return e == hipSuccess ? DECDS_OK : decds_hip_error(e, "fill_random launch");
}

}  // extern "C"
