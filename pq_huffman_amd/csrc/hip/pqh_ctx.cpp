// pqh_ctx.cpp -- context, error and scratch management for the pqh C ABI (pqh.h).
#include <cstdlib>
#include <cstring>

#include <algorithm>
#include <vector>
#include <cmath>

#include "pqh_internal.h"

int pqh_set_error(pqh_ctx* ctx, int code, const char* fmt, ...) {
    if (ctx) {
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(ctx->err, sizeof(ctx->err), fmt, ap);
        va_end(ap);
    }
    return code;
}

// fixed-point exponent of the k-means sums: s = 61 - ceil(log2(max|x| * n)), clamped, so
// that n values of magnitude <= max|x| scaled by 2^s stay below 2^61 (pqh_kmeans.hip)
int pqh_kmeans_fixed_shift(float max_abs, long long n) {
    if (!(max_abs > 0.0f) || n <= 0) return 40;
    if (std::isinf(max_abs)) return -126;
    const double b = (double)max_abs * (double)n;
    int s = 61 - (int)std::ceil(std::log2(b));
    return std::max(-126, std::min(100, s));
}

bool pqh_debug_sync() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("PQH_DEBUG_SYNC");
        v = (e && *e && *e != '0') ? 1 : 0;
    }
    return v == 1;
}

int pqh_use_device(pqh_ctx* ctx) {
    PQH_HIP(ctx, hipSetDevice(ctx->device));
    return PQH_OK;
}

int pqh_ensure_ws(pqh_ctx* ctx, size_t bytes) {
    if (bytes <= ctx->ws_bytes) return PQH_OK;
    if (ctx->ws) {
        PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
        ctx->ws_bytes = 0;
        PQH_HIP(ctx, hipFree(ctx->ws));
        ctx->ws = nullptr;
    }
    // 25% slack so that slowly growing requests do not reallocate every call; the exact
    // size when the slack does not fit
    for (size_t want : {bytes + bytes / 4 + 4096, bytes}) {
        if (hipMalloc(&ctx->ws, want) == hipSuccess) {
            ctx->ws_bytes = want;
            return PQH_OK;
        }
        ctx->ws = nullptr;
        (void)hipGetLastError();
    }
    return pqh_set_error(ctx, PQH_ERR_NOMEM, "workspace: cannot allocate %zu bytes", bytes);
}

int pqh_ensure_enc_scratch(pqh_ctx* ctx, size_t bytes) {
    if (bytes <= ctx->enc_scr_bytes) return PQH_OK;
    if (ctx->enc_scr) {
        PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
        ctx->enc_scr_bytes = 0;
        PQH_HIP(ctx, hipFree(ctx->enc_scr));
        ctx->enc_scr = nullptr;
    }
    if (hipMalloc(&ctx->enc_scr, bytes) != hipSuccess) {
        ctx->enc_scr = nullptr;
        (void)hipGetLastError();
        return pqh_set_error(ctx, PQH_ERR_NOMEM, "encode scratch: cannot allocate %zu bytes", bytes);
    }
    ctx->enc_scr_bytes = bytes;
    return PQH_OK;
}

extern "C" {

int pqh_device_count(int* count) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return n > 0 ? PQH_OK : PQH_ERR_NO_DEVICE;
}

int pqh_ctx_create(pqh_ctx_t** out, int device) {
    if (!out) return PQH_ERR_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return PQH_ERR_NO_DEVICE;
    if (device < 0 || device >= n) return PQH_ERR_ARG;
    pqh_ctx* ctx = new pqh_ctx();
    ctx->device = device;
    if (hipSetDevice(device) != hipSuccess) {
        delete ctx;
        return PQH_ERR_HIP;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        ctx->num_cus = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return PQH_ERR_HIP;
    }
    ctx->own_stream = true;
    if (hipMalloc(&ctx->d_diag, 8 * sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(ctx->d_diag, 0, 8 * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&ctx->d_sched, (size_t)2 * kSchedSet * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(ctx->d_sched, 0, (size_t)2 * kSchedSet * sizeof(uint32_t)) != hipSuccess) {
        if (ctx->d_diag) (void)hipFree(ctx->d_diag);
        if (ctx->d_sched) (void)hipFree(ctx->d_sched);
        (void)hipStreamDestroy(ctx->stream);
        delete ctx;
        return PQH_ERR_HIP;
    }
    *out = ctx;
    return PQH_OK;
}

int pqh_ctx_create_cu_split(pqh_ctx_t** out, int device, int cus, int complement) {
    int rc = pqh_ctx_create(out, device);
    if (rc) return rc;
    pqh_ctx* ctx = *out;
    if (cus == 0 || cus >= ctx->num_cus) return PQH_OK;
    // every (num_cus / cus)-th compute unit, so the subset spans all XCDs / shader engines;
    // complement: every other compute unit (a disjoint partner stream).  cus < 0: every
    // compute unit, as a CU-masked stream -- HIP gives such a stream a hardware queue of its
    // own instead of one shared from its pool of GPU_MAX_HW_QUEUES
    if (cus < 0) {
        cus = ctx->num_cus;
        complement = 0;
    }
    std::vector<uint32_t> mask((ctx->num_cus + 31) / 32, 0u);
    const int stride = std::max(1, ctx->num_cus / cus);
    std::vector<char> pick(ctx->num_cus, 0);
    int used = 0;
    for (int cu = 0; cu < ctx->num_cus && used < cus; cu += stride, ++used) pick[cu] = 1;
    for (int cu = 0; cu < ctx->num_cus; ++cu)
        if ((pick[cu] != 0) != (complement != 0)) mask[cu / 32] |= 1u << (cu % 32);
    hipStream_t s = nullptr;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
        pqh_ctx_destroy(ctx);
        *out = nullptr;
        return PQH_ERR_HIP;
    }
    (void)hipStreamDestroy(ctx->stream);
    ctx->stream = s;
    ctx->own_stream = true;
    int n_on = 0;   // persistent grids are sized to the CUs this stream can use
    for (uint32_t w : mask) n_on += __builtin_popcount(w);
    ctx->num_cus = std::max(1, n_on);
    return PQH_OK;
}

int pqh_ctx_create_cu_limited(pqh_ctx_t** out, int device, int cus) {
    return pqh_ctx_create_cu_split(out, device, cus, 0);
}

void* pqh_ctx_stream(const pqh_ctx_t* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int pqh_ctx_destroy(pqh_ctx_t* ctx) {
    if (!ctx) return PQH_OK;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->ws) (void)hipFree(ctx->ws);
    if (ctx->d_diag) (void)hipFree(ctx->d_diag);
    if (ctx->lb_state) (void)hipFree(ctx->lb_state);
    if (ctx->enc_scr) (void)hipFree(ctx->enc_scr);
    if (ctx->sort_state) (void)hipFree(ctx->sort_state);
    if (ctx->d_sched) (void)hipFree(ctx->d_sched);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return PQH_OK;
}

int pqh_ctx_release_scratch(pqh_ctx_t* ctx) {
    if (!ctx) return PQH_ERR_ARG;
    PQH_HIP(ctx, hipSetDevice(ctx->device));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));   // no launch may still use them
    if (ctx->ws) (void)hipFree(ctx->ws);
    if (ctx->enc_scr) (void)hipFree(ctx->enc_scr);
    if (ctx->lb_state) (void)hipFree(ctx->lb_state);
    if (ctx->sort_state) (void)hipFree(ctx->sort_state);
    ctx->ws = ctx->enc_scr = nullptr;
    ctx->ws_bytes = ctx->enc_scr_bytes = 0;
    ctx->lb_state = nullptr;
    ctx->lb_cap = 0;
    ctx->sort_state = nullptr;
    ctx->sort_cap = 0;
    return PQH_OK;
}

int pqh_ctx_set_stream(pqh_ctx_t* ctx, void* hip_stream) {
    if (!ctx) return PQH_ERR_ARG;
    if (ctx->own_stream) {
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipStreamDestroy(ctx->stream);
        ctx->own_stream = false;
    }
    ctx->stream = (hipStream_t)hip_stream;
    return PQH_OK;
}

int pqh_ctx_set_tuning(pqh_ctx_t* ctx, int key, double value) {
    if (!ctx || value < 0.0) return PQH_ERR_ARG;
    switch (key) {
        case PQH_TUNE_ASSIGN_WGS_PER_CU:
            ctx->tune_wgs_per_cu = value;
            return PQH_OK;
        case PQH_TUNE_HIST_SPLIT: {
            const int v = (int)value;
            if (v != 0 && v != 1 && v != 2 && v != 4 && v != 8) return PQH_ERR_ARG;
            ctx->tune_hist_split = v;
            return PQH_OK;
        }
        case PQH_TUNE_HIST_BLOCK: {
            const int v = (int)value;
            if (v != 0 && v != 256 && v != 1024) return PQH_ERR_ARG;
            ctx->tune_hist_block = v;
            return PQH_OK;
        }
        case PQH_TUNE_ENC_IMPL: {
            const int v = (int)value;
            if (v != 0 && v != 1 && v != 2) return PQH_ERR_ARG;
            ctx->tune_enc_impl = v;
            return PQH_OK;
        }
        default:
            return PQH_ERR_ARG;
    }
}

int pqh_ctx_sync(pqh_ctx_t* ctx) {
    if (!ctx) return PQH_ERR_ARG;
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return PQH_OK;
}

const char* pqh_ctx_last_error(const pqh_ctx_t* ctx) { return ctx ? ctx->err : "no context"; }

const char* pqh_status_string(int s) {
    switch (s) {
        case PQH_OK: return "ok";
        case PQH_ERR_ARG: return "invalid argument";
        case PQH_ERR_NO_DEVICE: return "no HIP device";
        case PQH_ERR_HIP: return "HIP runtime error";
        case PQH_ERR_UNSUPPORTED: return "unsupported configuration";
        case PQH_ERR_CODE_TOO_LONG: return "Huffman code longer than 56 bits";
        case PQH_ERR_CORRUPT: return "corrupt stream";
        case PQH_ERR_NOMEM: return "out of memory";
        case PQH_ERR_CAPACITY: return "output buffer too small";
        case PQH_ERR_REMOTE: return "another rank's part of the sharded call failed";
        case PQH_ERR_COMM: return "a collective hook failed";
        default: return "unknown status";
    }
}

}  // extern "C"

int pqh_prio(const char* name, int def) {
    char key[64];
    std::snprintf(key, sizeof key, "PQH_PRIO_%s", name);
    const char* e = std::getenv(key);
    if (!e || e[0] < '0' || e[0] > '3') return def;
    return e[0] - '0';
}
